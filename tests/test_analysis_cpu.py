"""CPU side of the analysis helpers (no GPU): the oracle restatements of
utils.oracle_ranking / rank_of_src_in_df pinned to the reference's outputs
(tests/golden/oracle.npz, sweepq.npz), the sweep_q / find_opt_oracle control
flow of the facade driven by the reference's recorded capacities, and the
argument validation of rq_oracle_dp / rq_rank_table / rq_u_int."""
import ctypes as C

import numpy as np
import pandas as pd
import pytest

from oracle import oracle as O
from redqueen_amd import _lib as L
from redqueen_amd import utils as U
from redqueen_amd.opt_model import SimOpts

COLS = ["event_id", "time_delta", "src_id", "t", "sink_id"]


def df_of(g, key):
    return pd.DataFrame({c: g[key + "_" + c] for c in COLS})


def oracle_cases(g):
    for c in g["cases"]:
        c = str(c)
        df = df_of(g, c)
        om = g[c + "_omit"]
        if om.size:
            df = df[~df.src_id.isin(om)]
        et, w = U._oracle_w(df, float(g[c + "_end"][0]))
        for i, q in enumerate(g[c + "_q"]):
            yield c, i, df, et, w, float(q), float(g[c + "_s"][0])


def test_oracle_dp_restatement_matches_reference(golden):
    g = golden("oracle.npz")
    n_checked = 0
    for c, i, df, et, w, q, s in oracle_cases(g):
        cost, ev, rk = O.oracle_dp(w, q, s)
        key = "%s_%d" % (c, i)
        assert cost == g[key + "_cost"][0], key
        assert np.array_equal(ev, g[key + "_events"]), key
        assert np.array_equal(rk, g[key + "_ranks"]), key
        assert np.array_equal(np.concatenate([[0.0], et.values]), g[key + "_t"]), key
        assert np.array_equal(w[1:], g[key + "_tdelta"]), key
        n_checked += 1
    assert n_checked == 16


def test_oracle_dp_edge_cases():
    # n = 0: J is 1 x 2, nothing to decide (utils.py:211-221)
    cost, ev, rk = O.oracle_dp(np.asarray([0.0, 3.0]), 1.0, 1.0)
    assert cost == 0.0 and list(ev) == [0] and list(rk) == [0]
    # q -> 0: post after every event; q -> inf: never post
    w = np.diff(np.concatenate([[0.0, 0.0], np.arange(1, 11) * 0.1, [2.0]]))
    _, ev, rk = O.oracle_dp(w, 1e-12, 1.0)
    assert ev[:-1].all() and not rk.any()
    _, ev, rk = O.oracle_dp(w, 1e12, 1.0)
    assert not ev.any() and list(rk) == list(range(11))


def test_rank_table_restatement_matches_reference(golden):
    g = golden("sweepq.npz")
    df = df_of(g, "rt_readme")
    for src in (1, 2, -1):
        for fill, key in ((True, "rt_readme_%d" % (src + 1)), (False, "rt_readme_%d_nofill" % (src + 1))):
            tab, idx, sinks = O.rank_table(df.t.values, df.src_id.values, df.sink_id.values, src, fill)
            assert np.array_equal(tab, g[key], equal_nan=True), key
            assert np.array_equal(idx, g["rt_readme_index"])
            assert np.array_equal(sinks, g["rt_readme_cols"])
    d5 = df_of(g, "rt_k5")
    tab, _, _ = O.rank_table(d5.t.values, d5.src_id.values, d5.sink_id.values, 1)
    assert np.array_equal(tab, g["rt_k5_tab"], equal_nan=True)


def test_sweep_q_control_flow_matches_reference(golden, monkeypatch):
    """The facade's sweep_q, fed the capacities the reference measured, retraces the
    reference's q sequence and returns its q bit for bit (utils.py:521-607)."""
    g = golden("sweepq.npz")
    trace_q, trace_cap = list(g["sq_trace_q"]), list(g["sq_trace_cap"])
    seen = []

    def fake_cap(sim_opts, q, seeds=None, **kw):
        i = len(seen)
        assert q == trace_q[i], (i, q, trace_q[i])
        seen.append(q)
        return trace_cap[i]
    monkeypatch.setattr(U, "calc_q_capacity_iter", fake_cap)
    monkeypatch.setattr(U, "_wall_df", lambda so: None)
    last_mean = float(g["sq_rlast_mean"][0])
    monkeypatch.setattr(U, "rank_of_src_in_df",
                        lambda df, src: pd.DataFrame([[last_mean]]))
    so = SimOpts.std_poisson(world_seed=1, world_rate=100.0)
    assert U.sweep_q(so, capacity_cap=50.0, parallel=False) == g["sq_q"][0]
    q2 = U.sweep_q(so, capacity_cap=20.0, parallel=False, tol=1e-3, only_tol=True, max_iters=6)
    assert q2 == g["sq_q2"][0]
    assert len(seen) == len(trace_q)
    # the notebook's own q_init (opt_broadcast.ipynb:2813) from that wall mean
    q_init = (4 * last_mean ** 2 * 1.0 ** 2) / (np.pi * np.pi * (50.0 + 1) ** 4)
    assert q_init == 0.0005753494376300199


def test_find_opt_oracle_control_flow(golden, monkeypatch):
    """find_opt_oracle's search, with the oracle DP restated on the CPU standing in
    for rq_oracle_dp, reaches the reference's (q, cost, #events)."""
    g = golden("oracle.npz")
    wall = df_of(g, "p100")
    monkeypatch.setattr(U, "_wall_df", lambda so: wall)

    def cpu_batch(ws, qs, ss):
        return [O.oracle_dp(w, q, s) for w, q, s in zip(ws, qs, ss)]
    monkeypatch.setattr(U, "oracle_dp_batch", cpu_batch)
    so = SimOpts.std_poisson(world_seed=1, world_rate=100.0).update({"end_time": 10.0})
    res = U.find_opt_oracle(50, so)
    assert res["q"] == g["fo_q"][0] and res["cost"] == g["fo_cost"][0]
    assert res["df"].events.sum() == g["fo_events"][0]
    with pytest.raises(AssertionError):
        U.oracle_ranking(pd.concat([wall, wall.assign(sink_id=7)]), so)


def test_analysis_abi_validation():
    lib = L.lib()
    b = C.c_size_t()
    assert lib.rq_oracle_workspace_size(-1, 10, C.byref(b)) == L.RQ_EINVAL
    assert lib.rq_oracle_workspace_size(2, 2_000_000, C.byref(b)) == L.RQ_EINVAL
    assert lib.rq_oracle_workspace_size(2, 100, C.byref(b)) == 0 and b.value >= 2 * 101 * 2 * 8
    assert lib.rq_oracle_dp(None, None, None, None, 0, 10, None, None, None, None, None, 0, None) == 0
    assert lib.rq_oracle_dp(None, None, None, None, 1, 10, None, None, None, None, None, 0,
                            None) == L.RQ_EINVAL
    assert lib.rq_rank_table(None, None, None, 10, 2, 1, 1, 5, None, None, None, None) == L.RQ_EINVAL
    assert lib.rq_u_int(None, None, 10, 2, None, None, 1, 1.0, None, None, 0, None) == L.RQ_EINVAL
