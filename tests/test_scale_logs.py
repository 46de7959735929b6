"""Reference runs at the headline scale (VERDICT r05 "next" 1): 8 whole C3 runs (1000
followers, ~7e5 df rows each) and 2 runs of graphs.c5_mid (500 bursty Hawkes sources,
T = 1000), made by tests/golden/gen_golden.py --scale-logs from /root/reference.

Each dataframe is rebuilt from the reference's event log with the reference's row
layout (State.get_dataframe, opt_model.py:85-97) and checked against the recorded
shape and crc32 of every column; then the reference's own time_in_top_k (K = 1, 2, 5,
10), average_rank and int_r_2 (utils.py:84-121) and counts (opt_runs.py:41-48) must
come back bit for bit -- from the C oracle here (CPU) and, under -m gpu, from
rq_metrics_replay, rq_metrics_replay_batch and the C ABI entry itself.
"""
import zlib

import numpy as np
import pandas as pd
import pytest

from redqueen_amd import graphs

KS = [1, 2, 5, 10]


def _graph(run):
    return graphs.c3() if run.startswith("c3_") else graphs.c5_mid()


def _rebuild(O, d, run):
    so = _graph(run)
    df = O.Scenario(so, ("opt", 0)).expand(d[run + "_t"], np.zeros_like(d[run + "_t"]), d[run + "_src"])
    return so, df


def _check_layout(d, run, df):
    shape, crc = d[run + "_shape"], d[run + "_crc"]
    assert len(df["t"]) == shape[0]
    for k, c in enumerate(("t", "src_id", "sink_id", "event_id")):
        assert zlib.crc32(np.ascontiguousarray(df[c]).tobytes()) == crc[k], (run, c)
    assert np.unique(df["sink_id"]).size == shape[4]


def _runs(d):
    return [str(r) for r in d["runs"]]


def test_fixture_covers_headline_scale(golden):
    d = golden("scale_logs.npz")
    runs = _runs(d)
    assert sum(r.startswith("c3_") for r in runs) >= 8
    assert sum(r.startswith("c5m_") for r in runs) >= 2
    for r in runs:
        assert d[r + "_shape"][0] > (6 * 10 ** 5 if r.startswith("c3_") else 3 * 10 ** 5)
    # c5_mid: C5's source side (500 Hawkes broadcasters before the trim)
    assert all(k == "Hawkes" for k, _ in graphs.c5_mid()["other_sources"])
    assert len(graphs.c5_mid()["other_sources"]) > 300


def test_c3_runs_are_dist_c3_replicas(golden):
    """The C3 runs are replicas 0..7 of the 10k-replica reference ensemble dist_c3.npz
    (same seeds): posts, world events, events, top-1 and average rank agree."""
    d = golden("scale_logs.npz")
    e = golden("dist_c3.npz")["data"]
    for r in _runs(d):
        if not r.startswith("c3_"):
            continue
        i = int(r.split("_")[1])
        sh, met = d[r + "_shape"], d[r + "_met"]
        assert np.array_equal(e[i], [sh[1], sh[2], sh[3], met[0], met[4]]), r


def test_oracle_metrics_equal_reference_at_scale(golden):
    """The C oracle's Appendix-B restatement on the rebuilt dataframes == the values
    utils.py returned on the reference's own dataframes (CPU)."""
    from oracle import oracle as O
    d = golden("scale_logs.npz")
    for r in _runs(d):
        so, df = _rebuild(O, d, r)
        _check_layout(d, r, df)
        top, avg, r2, cnt = O.metrics_df(df["t"], df["src_id"], df["sink_id"], df["event_id"],
                                         so["src_id"], so["end_time"], KS)
        assert np.array_equal(np.asarray(top + [avg, r2]), d[r + "_met"]), r
        assert cnt[0] == d[r + "_shape"][1] and cnt[1] == d[r + "_shape"][2], r


@pytest.mark.gpu
def test_gpu_replay_equals_reference_at_scale(golden):
    """rq_metrics_replay (one df over the chip), rq_metrics_replay_batch (all ten dfs in
    one launch) and the raw C ABI call: the reference's values bit for bit."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle import oracle as O
    from redqueen_amd import utils as U
    from test_gpu_replay_batch import _abi_replay
    from redqueen_amd import _lib as L
    d = golden("scale_logs.npz")
    runs = _runs(d)
    dfs, sos = [], []
    for r in runs:
        so, cols = _rebuild(O, d, r)
        _check_layout(d, r, cols)
        df = pd.DataFrame(cols)
        exp = d[r + "_met"]
        m = U.replay_metrics(df, so["src_id"], so["end_time"], KS)
        got = np.asarray(m["top_k"] + [m["avg_rank"], m["r_2"]])
        assert np.array_equal(got, exp), (r, got - exp)
        assert m["num_own"] == d[r + "_shape"][1] and m["num_world"] == d[r + "_shape"][2]
        got, cnt = _abi_replay(torch, L, df.t.values, df.src_id.values, df.sink_id.values,
                               df.event_id.values, so["src_id"], so["end_time"], KS)
        assert np.array_equal(got, exp), (r, "abi")
        assert cnt[0] == d[r + "_shape"][1] and cnt[3] == d[r + "_shape"][4]
        dfs.append(df)
        sos.append(so)
    # one batch per end time (the batch takes one end_time): C3 (T = 100), c5_mid (1000)
    for end in sorted({so["end_time"] for so in sos}):
        idx = [i for i, so in enumerate(sos) if so["end_time"] == end]
        res = U.replay_frames([dfs[i] for i in idx], 1, end, KS)
        for j, i in enumerate(idx):
            got = np.asarray([res["top_%d" % k][j] for k in KS] + [res.avg_rank[j], res.r_2[j]])
            assert np.array_equal(got, d[runs[i] + "_met"]), runs[i]
            assert res.num_events[j] == d[runs[i] + "_shape"][1]
            assert res.world_events[j] == d[runs[i] + "_shape"][2]
