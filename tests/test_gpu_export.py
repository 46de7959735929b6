"""GPU expansion of event logs into the reference's dataframe rows (rq_log_rows /
rq_log_expand, State.get_dataframe opt_model.py:85-97) vs the oracle's row-by-row
restatement (Scenario.expand), and the columnar export round trip."""
import numpy as np
import pandas as pd
import pytest

from tests.test_gpu_engine import _ctx, _graph, _world_with_seeds

pytestmark = pytest.mark.gpu
COLS = ["event_id", "time_delta", "src_id", "t", "sink_id"]


def _check(res, O, so, i):
    t, s = res.events(i)
    dt = O.state_time_deltas(t)
    sc = O.Scenario(so, ("opt", 0))
    ref = sc.expand(t, dt, s)
    df = res.dataframe(i)
    assert list(df.columns) == COLS
    for c in COLS:
        assert np.array_equal(df[c].values, ref[c]), c
    return len(df)


def test_readme_batch_rows():
    torch, engine, graphs, O = _ctx()
    so = graphs.readme()
    g = _graph(engine, so)
    res = g.run("opt", q=so["q"], s=so["s"], n_rep=12, ctrl_seed=7, world_seed=7, randomize=True,
                event_log=True)
    n = sum(_check(res, O, so, i) for i in range(12))
    full = res.dataframe()
    assert len(full) == n and list(full.columns) == ["replica"] + COLS
    assert np.array_equal(np.unique(full.replica.values), np.arange(12))


def test_c3_and_duplicate_edges():
    torch, engine, graphs, O = _ctx()
    so = graphs.c3()
    g = _graph(engine, so)
    res = g.run("opt", q=so["q"], s=so["s"], n_rep=3, ctrl_seed=11, world_seed=11, randomize=True,
                event_log=True)
    for i in range(3):
        assert _check(res, O, so, i) > 100000
    # unsorted edge lists, a source with no edges, a sink nobody posts to
    so2 = dict(graphs.readme())
    so2["edge_list"] = [(3, 3), (1, 3), (2, 3), (2, 1), (1, 1), (2, 2)]
    so2["sink_ids"] = [1, 2, 3, 9]
    so2["other_sources"] = list(so2["other_sources"]) + [("Poisson", {"src_id": 4, "seed": 3,
                                                                     "rate": 2.0})]
    g2 = _graph(engine, so2)
    res2 = g2.run("opt", q=1.0, s=1.0, n_rep=2, ctrl_seed=3, event_log=True)
    assert (res2.status.cpu().numpy() == 0).all()
    for i in range(2):
        _check(res2, O, so2, i)


def test_manager_dataframe_and_export(tmp_path):
    torch, engine, graphs, O = _ctx()
    from redqueen_amd import export
    from redqueen_amd.opt_model import SimOpts
    so = SimOpts(**graphs.readme())
    m = so.create_manager_with_opt(101)
    m.run_dynamic()
    df = m.state.get_dataframe()
    t, s = m.state._t, m.state._src
    ref = O.Scenario(graphs.readme(), ("opt", 101)).expand(t, O.state_time_deltas(t), s)
    for c in COLS:
        assert np.array_equal(df[c].values, ref[c]), c
    g = _graph(engine, graphs.readme())
    res = g.run("opt", q=1.0, s=graphs.readme()["s"], n_rep=5, ctrl_seed=1, event_log=True)
    n = export.write_npz(res, tmp_path / "a.npz")
    back = export.read_npz(tmp_path / "a.npz")
    assert len(back) == n
    pd.testing.assert_frame_equal(export.read_npz(tmp_path / "a.npz", 3), res.dataframe(3))
    try:
        import pyarrow.parquet as pq
    except ImportError:
        return
    assert export.write_parquet(res, tmp_path / "a.parquet") == n
    tab = pq.read_table(str(tmp_path / "a.parquet")).to_pandas()
    pd.testing.assert_frame_equal(tab, back)
    assert export.write_ipc(res, tmp_path / "a.arrow") == n
