"""rq_oracle_dp / rq_rank_table / rq_u_int on the GPU against the reference's own
outputs (tests/golden/oracle.npz, sweepq.npz, kat_runs.npz) and the CPU oracle.

Bit-exact: oracle cost / events / ranks, rank tables, find_opt_oracle's (q, cost),
worker_oracle's metrics on the reference's df.  u_int_opt: the reference's BLAS
dgemv may associate the follower dot differently -> rel 1e-12.
"""
import numpy as np
import pandas as pd
import pytest

from tests.test_analysis_cpu import COLS, df_of, oracle_cases

pytestmark = pytest.mark.gpu


def _ctx():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle import oracle as O
    from redqueen_amd import utils as U
    return O, U


def test_oracle_ranking_bit_exact(golden):
    O, U = _ctx()
    from redqueen_amd.opt_model import SimOpts
    g = golden("oracle.npz")
    n = 0
    for c, i, df, et, w, q, s in oracle_cases(g):
        key = "%s_%d" % (c, i)
        so = SimOpts.std_poisson(world_seed=0, world_rate=1.0).update(
            {"q": q, "s": s, "end_time": float(g[c + "_end"][0])})
        om = g[c + "_omit"]
        odf, cost = U.oracle_ranking(df_of(g, c), so, omit_src_ids=list(om) if om.size else None)
        assert cost == g[key + "_cost"][0], key
        assert np.array_equal(odf.events.values, g[key + "_events"]), key
        assert np.array_equal(odf.ranks.values, g[key + "_ranks"]), key
        assert np.array_equal(odf.t.values, g[key + "_t"]), key
        assert np.array_equal(odf.t_delta.values, g[key + "_tdelta"]), key
        n += 1
    assert n == 16


def test_oracle_dp_batched_equals_single_and_cpu(golden):
    """All golden walls x q in ONE launch, plus random walls at sizes that take the
    LDS (n <= 8190) and the global-column path (n > 8190), vs the CPU restatement."""
    O, U = _ctx()
    g = golden("oracle.npz")
    ws, qs, ss, exp = [], [], [], []
    for c, i, df, et, w, q, s in oracle_cases(g):
        ws.append(w), qs.append(q), ss.append(s)
        key = "%s_%d" % (c, i)
        exp.append((g[key + "_cost"][0], g[key + "_events"], g[key + "_ranks"]))
    rs = np.random.RandomState(5)
    for n, q, s in ((1, 0.3, 2.0), (63, 1.0, 1.0), (64, 0.01, 3.0), (65, 5.0, 0.5),
                    (3000, 2.0, 1.0), (8300, 40.0, 1.0)):
        t = np.cumsum(rs.exponential(0.01, n))
        w = np.diff(np.concatenate([[0.0, 0.0], t, [t[-1] + 0.5]]))
        ws.append(w), qs.append(q), ss.append(s)
        exp.append(O.oracle_dp(w, q, s))
    got = U.oracle_dp_batch(ws, qs, ss)
    for k, ((c, e, r), (c2, e2, r2)) in enumerate(zip(got, exp)):
        assert c == c2 and np.array_equal(e, e2) and np.array_equal(r, r2), k
    # the big one alone (global columns, 1024 threads) gives the same answer
    (c, e, r), = U.oracle_dp_batch([ws[-1]], [qs[-1]], [ss[-1]])
    assert c == exp[-1][0] and np.array_equal(e, exp[-1][1])


def test_find_opt_oracle_and_worker_oracle(golden, monkeypatch):
    O, U = _ctx()
    from redqueen_amd import opt_runs as R
    from redqueen_amd.opt_model import SimOpts
    g = golden("oracle.npz")
    wall = df_of(g, "p100")
    monkeypatch.setattr(U, "_wall_df", lambda so: wall)
    so = SimOpts.std_poisson(world_seed=1, world_rate=100.0).update({"end_time": 10.0})
    res = U.find_opt_oracle(50, so)
    assert res["q"] == g["fo_q"][0] and res["cost"] == g["fo_cost"][0]
    assert res["df"].events.sum() == g["fo_events"][0]
    # worker_oracle's scoring of the reference's oracle df (RealData posts + world)
    wdf = df_of(g, "wo_df")
    op = {}
    R.add_perf(op, wdf, so)
    for k in ["top_1", "avg_rank", "r_2", "world_events", "num_events"]:
        assert float(op[k]) == g["wo_" + k][0], k
    assert int(np.sum(res["df"].events == 1)) == g["wo_r0_num_events"][0]


def test_worker_oracle_end_to_end():
    """worker_oracle on a GPU-simulated world: the oracle hits the target capacity and
    its RealData replay posts exactly those times (plus oracle_eps)."""
    O, U = _ctx()
    from redqueen_amd import opt_runs as R
    from redqueen_amd.opt_model import SimOpts
    so = SimOpts.std_poisson(world_seed=1, world_rate=100.0).update({"end_time": 10.0})
    op = R.worker_oracle((1, 50, None, so, None))
    assert abs(op["r0_num_events"] - 50) <= 1
    assert op["num_events"] == op["r0_num_events"]
    assert 0.0 < op["top_1"] < 10.0 and op["world_events"] > 800


def test_rank_table_and_u_int(golden):
    O, U = _ctx()
    from redqueen_amd.opt_model import SimOpts
    g = golden("sweepq.npz")
    df = df_of(g, "rt_readme")
    for src in (1, 2, -1):
        tab = U.rank_of_src_in_df(df, src)
        assert np.array_equal(tab.values, g["rt_readme_%d" % (src + 1)], equal_nan=True)
        assert np.array_equal(tab.index.values, g["rt_readme_index"])
        assert np.array_equal(tab.columns.values, g["rt_readme_cols"])
        nf = U.rank_of_src_in_df(df, src, fill=False)
        assert np.array_equal(nf.values, g["rt_readme_%d_nofill" % (src + 1)], equal_nan=True)
    # pivot on event_id instead of t
    by_eid = U.rank_of_src_in_df(df, 1, with_time=False)
    assert by_eid.shape[1] == 3 and by_eid.index.name == "event_id"
    rd = SimOpts(src_id=1, end_time=100.0, s=np.asarray([1.0, 1.0]), q=1.0, sink_ids=[1, 2, 3],
                 other_sources=[], edge_list=[(1, 1)])
    u = U.u_int_opt(df, sim_opts=rd, follower_ids=[1, 3])
    assert u == pytest.approx(g["rt_readme_uint"][0], rel=1e-12)
    d5 = df_of(g, "rt_k5")
    so5 = SimOpts(src_id=1, end_time=100.0, s=np.asarray([0.5, 1.5]), q=1.0,
                  sink_ids=[5001, 5002], other_sources=[], edge_list=[(1, 5001)])
    assert np.array_equal(U.rank_of_src_in_df(d5, 1).values, g["rt_k5_tab"], equal_nan=True)
    assert U.u_int_opt(d5, sim_opts=so5) == pytest.approx(g["rt_k5_uint"][0], rel=1e-12)


def test_u_int_kat_k1(golden):
    """Notebook KAT K1 (opt_broadcast.ipynb:88): u_int_opt = 24.2522515977514."""
    O, U = _ctx()
    from redqueen_amd.opt_model import SimOpts
    k = golden("kat_runs.npz")
    so = SimOpts.std_poisson(world_seed=42, world_rate=1000.0)
    n = k["k1_t"].size
    df = pd.DataFrame({"event_id": np.arange(100, 100 + n), "time_delta": k["k1_dt"],
                       "src_id": k["k1_src"], "t": k["k1_t"], "sink_id": np.full(n, 1001)})
    assert U.u_int_opt(df, sim_opts=so) == pytest.approx(k["k1_uint"][0], rel=1e-12)
    assert k["k1_uint"][0] == pytest.approx(24.2522515977514, rel=1e-12)


def test_sweep_q_gpu_matches_engine_oracle():
    """sweep_q on the GPU: every capacity estimate is a GPU batch over seeds
    100..119; the same control flow on the CPU engine oracle's capacities gives the
    same q bit for bit, and q lands near the reference's (different RNG)."""
    O, U = _ctx()
    from redqueen_amd.opt_model import SimOpts
    so = SimOpts.std_poisson(world_seed=1, world_rate=100.0)
    q_gpu = U.sweep_q(so, capacity_cap=50.0)
    caps = {}

    def cpu_cap(sim_opts, q, seeds=None, **kw):
        sc = O.Scenario(sim_opts.update({"q": q}).get_dict(), ("opt", 0))
        _, cnt, _ = O.engine_batch(sc, 20, 100, False)
        caps[q] = cnt[:, 0].astype(np.float64)
        return caps[q]
    orig = U.calc_q_capacity_iter
    try:
        U.calc_q_capacity_iter = cpu_cap
        q_cpu = U.sweep_q(so, capacity_cap=50.0)
    finally:
        U.calc_q_capacity_iter = orig
    assert q_gpu == q_cpu
    for q, c in caps.items():
        assert np.array_equal(U.calc_q_capacity_iter(so, q), c)
    assert 0.25 < q_gpu / 0.00021575603911125744 < 4.0


def test_u_int_scalar_s_like_reference(golden):
    """u_int_opt with a scalar s computes the reference's numpy expression (utils.py:
    78-81): for one follower the [n_t, n_t] broadcast sum, the reference's value bit
    for bit; for two followers the reference's ValueError (errors.npz)."""
    O, U = _ctx()
    g = golden("errors.npz")
    df = df_of(g, "ui")
    v = U.u_int_opt(df, src_id=1, end_time=100.0, s=1.0, q=2.0, follower_ids=[1])
    assert v == g["ui_scalar_f1"][0]
    assert str(g["ui_scalar_f2_err"][0]) == "ValueError"
    with pytest.raises(ValueError):
        U.u_int_opt(df, src_id=1, end_time=100.0, s=1.0, q=2.0, follower_ids=[1, 3])
