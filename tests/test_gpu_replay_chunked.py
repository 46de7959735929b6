"""The chunked replay: ONE dataframe spread over many workgroups (chunks of 4096 rows,
per-sink carries composed across chunks; rq_replay.hip rq_rc_*).

Expected values: the reference's own returned metrics on its dataframes (golden
fixtures, gen_golden.py), the C oracle's Appendix-B restatement (pinned to those
fixtures by tests/test_oracle.py) on long random dataframes with ties, duplicate
(t, sink) rows and own posts across chunk boundaries, and -- at full C3 size -- the
fused sweep's own metrics; the chunked path must also equal the one-workgroup path
bit for bit.  RQ_RP_CHUNK=1 forces the chunked path whatever the df's size.
"""
import os

import numpy as np
import pandas as pd
import pytest

from redqueen_amd import graphs
from tests.test_gpu_replay_batch import KS, _ctx, _readme_df

pytestmark = pytest.mark.gpu


def _replay(torch, U, df, src_id, end, chunked, Ks=KS):
    dev = "cuda"
    t = torch.from_numpy(np.ascontiguousarray(df.t.values, dtype=np.float64)).to(dev)
    s = torch.from_numpy(np.ascontiguousarray(df.src_id.values, dtype=np.int64)).to(dev)
    k = torch.from_numpy(np.ascontiguousarray(df.sink_id.values, dtype=np.int64)).to(dev)
    e = torch.from_numpy(np.ascontiguousarray(df.event_id.values, dtype=np.int64)).to(dev) \
        if "event_id" in df.columns else None
    old = os.environ.get("RQ_RP_CHUNK")
    os.environ["RQ_RP_CHUNK"] = "1" if chunked else "0"
    try:
        m, c = U.replay_columns(t, s, k, e, None, src_id, end, Ks, chunked=chunked)
    finally:
        if old is None:
            del os.environ["RQ_RP_CHUNK"]
        else:
            os.environ["RQ_RP_CHUNK"] = old
    return m[0].cpu().numpy(), c[0].cpu().numpy()


def _random_df(rs, n_events, sinks, dup_p=0.0, tie_p=0.0, own_p=0.2):
    """Events of 1..min(40, #sinks) distinct sinks (+ a duplicated sink row with
    probability dup_p), equal times with probability tie_p, own posts own_p."""
    rows, t = [], 0.0
    hi = min(40, len(sinks)) + 1
    for e in range(n_events):
        if rs.rand() >= tie_p:
            t += float(rs.exponential(0.1))
        src = 1 if rs.rand() < own_p else int(rs.randint(2, 9))
        ss = list(rs.choice(sinks, rs.randint(1, hi), replace=False))
        if rs.rand() < dup_p:
            ss.append(ss[0])
        rows += [(100 + e, src, t, int(y)) for y in ss]
    return pd.DataFrame.from_records(rows, columns=["event_id", "src_id", "t", "sink_id"])


def _oracle(O, df, src_id, end, Ks=KS):
    top, avg, r2, cnt = O.metrics_df(df.t.values, df.src_id.values, df.sink_id.values,
                                     df.event_id.values, src_id, end, Ks)
    return np.asarray(list(top) + [avg, r2]), cnt


def test_reference_dataframes(golden):
    """The reference's own dataframes and returned values, through the chunked path."""
    torch, O, L, U = _ctx()
    d = golden("readme_runs.npz")
    so = graphs.readme()
    for name in ("101", "1", "2", "3", "5", "7", "11", "13", "wall", "pois", "long", "max"):
        df = _readme_df(O, d, name, so)
        end = 400.0 if name == "long" else so["end_time"]   # gen_golden's long horizon
        got, cnt = _replay(torch, U, df, so["src_id"], end, True)
        assert np.array_equal(got, d["met_" + name]), (name, got - d["met_" + name])
        assert cnt[0] == d["cnt_" + name][0] and cnt[1] == d["cnt_" + name][1]


@pytest.mark.parametrize("n_events,n_sinks,dup_p,tie_p,own_p", [
    (6000, 5, 0.0, 0.0, 0.2),      # few sinks: long per-sink runs across chunks
    (3000, 300, 0.0, 0.3, 0.05),   # equal-time groups spanning chunk boundaries
    (3000, 1500, 0.0, 0.0, 0.5),   # many sinks, many own posts
    (2500, 40, 0.03, 0.3, 0.2),    # duplicate (t, sink) rows: the pivot-mean fallback
    (2500, 4000, 0.0, 0.1, 0.2),   # near the chunked path's sink limit
    (1500, 6000, 0.0, 0.1, 0.2),   # > 4096 sinks: handed to the one-workgroup path
])
def test_long_random_dataframes(n_events, n_sinks, dup_p, tie_p, own_p):
    torch, O, L, U = _ctx()
    rs = np.random.RandomState(n_events + n_sinks)
    sinks = np.unique(rs.randint(-10 ** 12, 10 ** 12, n_sinks + 50, dtype=np.int64))[:n_sinks]
    df = _random_df(rs, n_events, sinks, dup_p, tie_p, own_p)
    assert len(df) > 2 * 4096
    end = float(df.t.max()) + 0.5
    exp, cnt = _oracle(O, df, 1, end)
    got_c, c_c = _replay(torch, U, df, 1, end, True)
    got_o, c_o = _replay(torch, U, df, 1, end, False)
    assert np.array_equal(got_o, exp), got_o - exp
    assert np.array_equal(got_c, exp), got_c - exp
    assert np.array_equal(c_c, c_o), (c_c, c_o)
    assert c_c[0] == cnt[0] and c_c[1] == cnt[1]


def test_single_and_tiny_dataframes():
    torch, O, L, U = _ctx()
    one = pd.DataFrame({"event_id": [100], "src_id": [2], "t": [1.5], "sink_id": [7]})
    got, c = _replay(torch, U, one, 1, 3.0, True)
    exp, _ = _oracle(O, one, 1, 3.0)
    assert np.array_equal(got, exp) and c[2] == 1
    rs = np.random.RandomState(9)
    df = _random_df(rs, 700, np.arange(20, dtype=np.int64), 0.0, 0.2)   # < one chunk
    got, c = _replay(torch, U, df, 1, float(df.t.max()) + 1, True)
    exp, _ = _oracle(O, df, 1, float(df.t.max()) + 1)
    assert np.array_equal(got, exp)


def test_unsorted_long_dataframe_rejected():
    torch, O, L, U = _ctx()
    rs = np.random.RandomState(4)
    df = _random_df(rs, 3000, np.arange(30, dtype=np.int64))
    df.loc[len(df) // 2 + 4097, "t"] = -1.0   # in a later chunk
    got, c = _replay(torch, U, df, 1, 1e9, True)
    assert c[2] == L.RQ_EUNSORTED and np.isnan(got).all()


def test_c3_replica_dataframe_one_call():
    """One exported C3 replica (~7e5 rows) through the facade's single-df entry: the
    chunked path, equal to the fused sweep's metrics for that replica and to the
    one-workgroup replay."""
    torch, O, L, U = _ctx()
    from redqueen_amd import engine
    so = graphs.c3()
    g = engine.Graph(so["src_id"], so["other_sources"], so["sink_ids"], so["edge_list"], so["end_time"])
    res = g.run("opt", q=so["q"], s=so["s"], n_rep=2, ctrl_seed=77, world_seed=77, randomize=True,
                event_log=True, Ks=(1, 2))
    for i in range(2):
        df = res.dataframe(i)
        assert len(df) > 500000
        got_c, c_c = _replay(torch, U, df, so["src_id"], so["end_time"], True, (1, 2))
        got_o, c_o = _replay(torch, U, df, so["src_id"], so["end_time"], False, (1, 2))
        assert np.array_equal(got_c, res.metrics[i].cpu().numpy())
        assert np.array_equal(got_c, got_o) and np.array_equal(c_c, c_o)
        assert c_c[2] == int(res.counts[i, 3])
        m = U.replay_metrics(df, so["src_id"], so["end_time"], (1, 2))   # facade: chunked by size
        assert m["top_k"] == list(got_c[:2]) and m["avg_rank"] == got_c[2]
