"""The batched replay on RAW sink ids (rq_metrics_replay / rq_metrics_replay_batch,
SURVEY.md 8(b)) through the C ABI.

Expected values: the reference's own returned metrics (golden fixtures made by
tests/golden/gen_golden.py from /root/reference), the C oracle's restatement of
utils.py Appendix B (oracle/rq_oracle.c, pinned to those fixtures by
tests/test_oracle.py) where a case has no fixture, and -- at full C3 size -- the
engine's own fused metrics, which must equal a replay of the dataframe it exports.
"""
import ctypes as C

import numpy as np
import pandas as pd
import pytest

from redqueen_amd import graphs

pytestmark = pytest.mark.gpu
KS = [1, 2, 5, 10]
I64_MIN, I64_MAX = np.iinfo(np.int64).min, np.iinfo(np.int64).max


def _ctx():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle import oracle as O
    from redqueen_amd import _lib as L
    from redqueen_amd import utils as U
    return torch, O, L, U


def _dev(torch, a, dt):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).cuda()


def _abi_replay(torch, L, t, src, sink, eid, src_id, end, Ks, large=False):
    """rq_metrics_replay called through the C ABI exactly as a foreign binding would."""
    lib = L.lib()
    Kc = np.ascontiguousarray(Ks, dtype=np.int32)
    nb = C.c_size_t()
    assert lib.rq_replay_workspace_size(len(t), 1, len(Ks), L.REPLAY_LARGE if large else 0,
                                        C.byref(nb)) == 0
    ws = torch.empty(nb.value, dtype=torch.uint8, device="cuda")
    tt, ts, tk = _dev(torch, t, np.float64), _dev(torch, src, np.int64), _dev(torch, sink, np.int64)
    te = _dev(torch, eid, np.int64) if eid is not None else None
    out = torch.empty(len(Ks) + 2, dtype=torch.float64, device="cuda")
    cnt = torch.empty(4, dtype=torch.int64, device="cuda")
    rc = lib.rq_metrics_replay(tt.data_ptr(), ts.data_ptr(), tk.data_ptr(),
                               te.data_ptr() if te is not None else None, len(t), int(src_id),
                               float(end), Kc.ctypes.data_as(L._pi32), len(Ks), out.data_ptr(),
                               cnt.data_ptr(), ws.data_ptr(), ws.numel(),
                               torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    return out.cpu().numpy(), cnt.cpu().numpy()


def _readme_df(O, d, name, so):
    sc = O.Scenario(so, ("opt", 0))
    return pd.DataFrame(sc.expand(d["t_" + name], d["dt_" + name], d["src_" + name]))


def test_abi_raw_sink_ids(golden):
    """Raw int64 sink ids of any magnitude (incl. INT64_MIN / INT64_MAX) give the
    reference's values: the pivot columns are the device's business."""
    torch, O, L, U = _ctx()
    d = golden("readme_runs.npz")
    so = graphs.readme()
    for name in ("101", "3", "wall", "pois"):
        df = _readme_df(O, d, name, so)
        exp = d["met_" + name]
        sink = df.sink_id.values
        for remap in ({1: 1, 2: 2, 3: 3}, {1: I64_MIN, 2: -5, 3: I64_MAX},
                      {1: 10 ** 17 + 3, 2: 7, 3: -(10 ** 18)}):
            raw = np.vectorize(remap.get, otypes=[np.int64])(sink)
            for large in (False, True):
                got, cnt = _abi_replay(torch, L, df.t.values, df.src_id.values, raw,
                                       df.event_id.values, so["src_id"], so["end_time"], KS, large)
                assert np.array_equal(got, exp), (name, remap, large, got - exp)
                assert cnt[0] == d["cnt_" + name][0] and cnt[1] == d["cnt_" + name][1]
                assert cnt[3] == 3


def test_batch_equals_reference_values(golden):
    """Every README run and the notebook KATs as ONE batch each: bit-exact."""
    torch, O, L, U = _ctx()
    d = golden("readme_runs.npz")
    so = graphs.readme()
    names = ["%d" % s for s in d["seeds"]] + ["wall", "pois", "max"]
    dfs = [_readme_df(O, d, n, so) for n in names]
    res = U.replay_frames(dfs, so["src_id"], so["end_time"], KS)
    for i, n in enumerate(names):
        got = np.asarray([res["top_%d" % k][i] for k in KS] + [res.avg_rank[i], res.r_2[i]])
        assert np.array_equal(got, d["met_" + n]), n
        assert res.num_events[i] == d["cnt_" + n][0] and res.world_events[i] == d["cnt_" + n][1]
    k = golden("kat_runs.npz")
    so2 = graphs.kat_two_walls()
    kdfs = [pd.DataFrame(O.Scenario(so2, ("opt", 0)).expand(k[n + "_t"], k[n + "_dt"], k[n + "_src"]))
            for n in ("k3", "k4", "k5", "k6")]
    res = U.replay_frames(kdfs, 1, 100.0, KS)
    for i, n in enumerate(("k3", "k4", "k5", "k6")):
        got = np.asarray([res["top_%d" % kk][i] for kk in KS] + [res.avg_rank[i], res.r_2[i]])
        assert np.array_equal(got, k[n + "_met"]), n


def _oracle_met(O, df, src_id, end):
    top, avg, r2, cnt = O.metrics_df(df.t.values, df.src_id.values, df.sink_id.values,
                                     df.event_id.values, src_id, end, KS)
    return np.asarray(top + [avg, r2]), cnt


def test_batch_adversarial_and_fractional(golden):
    """Tie-heavy and fractional-cell dataframes (the sequential fallback) mixed with
    plain ones in one batch; a common end_time, so the oracle restatement is the
    expectation (it equals the reference on each of these at its own end_time:
    tests/test_oracle.py)."""
    torch, O, L, U = _ctx()
    dfs = []
    for fname, cols in (("adversarial.npz", ("_eid", "_src", "_t", "_sink")),
                        ("frac.npz", ("_event_id", "_src_id", "_t", "_sink_id"))):
        g = golden(fname)
        for c in g["cases"]:
            dfs.append(pd.DataFrame({"event_id": g[c + cols[0]], "src_id": g[c + cols[1]],
                                     "t": g[c + cols[2]], "sink_id": g[c + cols[3]]}))
    d = golden("readme_runs.npz")
    dfs.insert(3, _readme_df(O, d, "101", graphs.readme()))
    end = max(float(x.t.max()) for x in dfs) + 1.0
    res = U.replay_frames(dfs, 1, end, KS)
    for i, df in enumerate(dfs):
        exp, cnt = _oracle_met(O, df, 1, end)
        got = np.asarray([res["top_%d" % k][i] for k in KS] + [res.avg_rank[i], res.r_2[i]])
        assert np.array_equal(got, exp), (i, got - exp)
        assert res.sinks[i] == df.sink_id.nunique()


def _random_df(rs, n_events, sinks, dup_p=0.0, tie_p=0.0, own_p=0.2):
    rows, t = [], 0.0
    for e in range(n_events):
        if rs.rand() >= tie_p:
            t += float(rs.exponential(0.1))
        src = 1 if rs.rand() < own_p else int(rs.randint(2, 9))
        ss = list(rs.choice(sinks, rs.randint(1, 40), replace=False))
        if rs.rand() < dup_p:
            ss.append(ss[0])
        rows += [(100 + e, src, t, int(y)) for y in ss]
    return pd.DataFrame.from_records(rows, columns=["event_id", "src_id", "t", "sink_id"])


@pytest.mark.parametrize("dup_p,tie_p", [(0.0, 0.0), (0.05, 0.3)])
def test_wide_dataframes_global_tables(dup_p, tie_p):
    """> 3071 unique sinks: the LDS table gives up, the df is rerun with the large
    workspace (global hash tables; the fallback's per-sink state in HBM)."""
    torch, O, L, U = _ctx()
    rs = np.random.RandomState(5 + int(dup_p * 100))
    sinks = np.unique(rs.randint(-5 * 10 ** 11, 5 * 10 ** 11, 6100, dtype=np.int64))[:6000]
    rs.shuffle(sinks)
    df = _random_df(rs, 1500, sinks, dup_p, tie_p)
    end = float(df.t.max()) + 0.25
    exp, cnt = _oracle_met(O, df, 1, end)
    assert df.sink_id.nunique() > 3071
    got, c = _abi_replay(torch, L, df.t.values, df.src_id.values, df.sink_id.values,
                         df.event_id.values, 1, end, KS, large=False)
    assert c[2] == L.RQ_EOVERFLOW and np.isnan(got).all()   # needs the large workspace
    got, c = _abi_replay(torch, L, df.t.values, df.src_id.values, df.sink_id.values,
                         df.event_id.values, 1, end, KS, large=True)
    assert np.array_equal(got, exp), got - exp
    assert c[3] == df.sink_id.nunique() and c[0] == cnt[0] and c[1] == cnt[1]
    m = U.replay_metrics(df, 1, end, KS)   # the facade retries with the large workspace itself
    assert np.array_equal(np.asarray(m["top_k"] + [m["avg_rank"], m["r_2"]]), exp)


def test_batch_errors_are_per_dataframe():
    """An unsorted and an empty dataframe are rejected without touching their neighbours."""
    torch, O, L, U = _ctx()
    rs = np.random.RandomState(3)
    sinks = np.arange(50, 90, dtype=np.int64)
    good = [_random_df(rs, 200, sinks) for _ in range(3)]
    bad = good[1].iloc[::-1].reset_index(drop=True)
    empty = good[0].iloc[:0]
    dfs = [good[0], bad, empty, good[2], good[1]]
    end = max(float(x.t.max()) for x in good) + 1.0
    res = U.replay_frames(dfs, 1, end, KS)
    assert res.pivot_rows[1] == L.RQ_EUNSORTED and np.isnan(res.avg_rank[1])
    assert res.pivot_rows[2] == 0 and np.isnan(res.avg_rank[2])
    for i in (0, 3, 4):
        exp, _ = _oracle_met(O, dfs[i], 1, end)
        got = np.asarray([res["top_%d" % k][i] for k in KS] + [res.avg_rank[i], res.r_2[i]])
        assert np.array_equal(got, exp)
    # without event ids the counts are unknown (-1), the metrics are unchanged
    no_eid = [d.drop(columns=["event_id"]) for d in good]
    r2 = U.replay_frames(no_eid, 1, end, KS)
    assert (r2.num_events == -1).all()
    assert np.array_equal(r2.avg_rank.values, U.replay_frames(good, 1, end, KS).avg_rank.values)


def test_c3_exported_frames_replay_to_engine_metrics():
    """Full C3 size: 64 replicas' dataframes (~7e5 rows each), exported by
    rq_log_expand and replayed as one batch, give exactly the metrics the fused
    sweep computed for the same replicas (two independent GPU paths to the
    reference's arithmetic)."""
    torch, O, L, U = _ctx()
    from redqueen_amd import engine
    so = graphs.c3()
    g = engine.Graph(so["src_id"], so["other_sources"], so["sink_ids"], so["edge_list"],
                     so["end_time"])
    R = 64
    res = g.run("opt", q=so["q"], s=so["s"], n_rep=R, ctrl_seed=901, world_seed=901,
                randomize=True, event_log=True, Ks=(1, 2))
    assert int(res.status.max().item()) == 0
    ro, cols = res.log_columns()
    off = torch.from_numpy(ro).cuda()
    assert int(ro[-1]) > 100000 * R
    m, c = U.replay_columns(cols["t"], cols["src_id"], cols["sink_id"], cols["event_id"], off,
                            so["src_id"], so["end_time"], (1, 2))
    assert torch.equal(m, res.metrics)
    assert torch.equal(c[:, 0], res.counts[:, 0]) and torch.equal(c[:, 1], res.counts[:, 1])
    assert torch.equal(c[:, 2], res.counts[:, 3])   # pivot rows = the sweep's row count


def test_malformed_df_offsets_rejected(golden):
    """A df_off range that is negative, decreasing or past n_rows touches no workspace
    and reports RQ_EINVAL in counts[d][2]; the well-formed dataframes of the same call
    keep the reference's values."""
    torch, O, L, U = _ctx()
    d = golden("readme_runs.npz")
    so = graphs.readme()
    df = _readme_df(O, d, "101", so)
    n = len(df)
    exp = d["met_101"]
    cat = lambda c, k: np.concatenate([df[c].values] * k)  # noqa: E731
    t = _dev(torch, cat("t", 2), np.float64)
    src = _dev(torch, cat("src_id", 2), np.int64)
    sink = _dev(torch, cat("sink_id", 2), np.int64)
    eid = _dev(torch, cat("event_id", 2), np.int64)
    for bad in ([0, n, n - 5, 2 * n], [0, n, 2 * n + 7, 2 * n], [0, n, -3, 2 * n]):
        off = _dev(torch, bad, np.int64)
        o, c = U.replay_columns(t, src, sink, eid, off, so["src_id"], so["end_time"], KS)
        o, c = o.cpu().numpy(), c.cpu().numpy()
        assert np.array_equal(o[0], exp) and c[0, 2] > 0, bad
        assert c[1, 2] == L.RQ_EINVAL and np.isnan(o[1]).all(), (bad, c[1])
