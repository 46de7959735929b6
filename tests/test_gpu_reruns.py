"""Fast-path coverage of run_dynamic's edge cases (VERDICT r05 "next" 2 and 4).

* max_events (opt_model.py:241, :271 `while num_events < max_events`) on the fast tiled
  sweeps: the tile keeps the events numbered below it (truncate_tile) -- bit-identical
  to the exact sequential sweep, events included, on the fused (<= 64 sources) and the
  general (> 64) sweep.
* Reruns of the flagged replicas only (rq_batch_desc.rep_idx, ABI v6): an overflowed
  replica at doubled capacities, a tie-flagged one (equal event times on a fast sweep)
  on the exact sequential sweep; the batch equals the all-rerun result bit for bit and
  Graph.reruns counts exactly the flagged replicas.
"""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))


def _ctx():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from redqueen_amd import _lib as L
    from redqueen_amd import engine, graphs
    return torch, L, engine, graphs


def _graph(engine, so, **kw):
    return engine.Graph(so["src_id"], so["other_sources"], so["sink_ids"], so["edge_list"],
                        so["end_time"], **kw)


def _same(torch, a, b, events=False):
    assert torch.equal(a.metrics.isnan(), b.metrics.isnan())
    assert torch.equal(a.metrics.nan_to_num(), b.metrics.nan_to_num())
    assert torch.equal(a.counts, b.counts)
    if events:
        n = a.counts[:, 2]
        for i in range(a.counts.shape[0]):
            k = int(n[i].item())
            assert torch.equal(a.ev_t[i, :k], b.ev_t[i, :k]) and torch.equal(a.ev_src[i, :k], b.ev_src[i, :k]), i


@pytest.mark.parametrize("wl", ["c3", "g120"])
def test_max_events_on_the_fast_sweep(wl):
    """max_events no longer forces the sequential sweep: the fast sweep's tile cut gives
    the sequential sweep's results bit for bit (metrics, counts, the event log), for cuts
    inside a tile, at tile edges, before the first event and past the last."""
    torch, L, engine, graphs = _ctx()
    so = getattr(graphs, wl)()
    g = _graph(engine, so)
    R = 256
    kw = dict(q=so["q"], s=so["s"], n_rep=R, ctrl_seed=31, world_seed=31, randomize=True,
              Ks=(1, 2), event_log=True)
    full = g.run("opt", **kw)
    mean_ev = float(full.counts[:, 2].double().mean().item())
    for me in (0, 1, 63, 64, 65, 129, int(mean_ev * 0.7), int(mean_ev), 10 ** 7):
        v = g.run("opt", max_events=me, plan_only=True, **{k: x for k, x in kw.items() if k != "event_log"})
        assert v["variant"] % 10 not in (1, 4), (me, v)   # a fast variant
        fast = g.run("opt", max_events=me, **kw)
        seq = g.run("opt", max_events=me, sweep_mode=2, **kw)
        _same(torch, fast, seq, events=True)
        assert int(fast.counts[:, 2].max().item()) <= me
    # the cut at max_events = the first max_events events of the unbounded run
    me = int(mean_ev * 0.5)
    cut = g.run("opt", max_events=me, **kw)
    for i in range(0, R, 37):
        assert torch.equal(cut.ev_t[i, :me], full.ev_t[i, :me]) and torch.equal(cut.ev_src[i, :me], full.ev_src[i, :me])


def test_only_flagged_replicas_rerun(monkeypatch):
    """10k C3 replicas with capacities squeezed (RQ_CAP_SQUEEZE) until only a few
    replicas overflow: Graph.run reruns exactly those (Graph.reruns), and the batch equals
    the unsqueezed run bit for bit."""
    torch, L, engine, graphs = _ctx()
    so = graphs.c3()
    g = _graph(engine, so)
    R = 10000
    kw = dict(q=so["q"], s=so["s"], n_rep=R, ctrl_seed=5, world_seed=5, randomize=True, Ks=(1,))
    ref = g.run("opt", **kw)
    assert g.reruns == 0
    ovf = L.ST_ROWS_OVERFLOW | L.ST_STREAM_OVERFLOW
    lo, hi, pick = 0.2, 1.0, None
    for _ in range(24):   # the squeeze at which 1..40 of the 10k replicas overflow
        mid = 0.5 * (lo + hi)
        monkeypatch.setenv("RQ_CAP_SQUEEZE", "%.6f" % mid)
        raw = g.run("opt", check=False, **kw)
        n = int(((raw.status & ovf) != 0).sum().item())
        if 1 <= n <= 40:
            pick = mid
            break
        lo, hi = (mid, hi) if n > 40 else (lo, mid)
    assert pick is not None
    flagged = int(((raw.status & ovf) != 0).sum().item())
    g.reset_capacity_memo()
    got = g.run("opt", **kw)
    assert g.reruns == flagged
    assert int(got.status.max().item()) == 0
    _same(torch, got, ref)
    # the memo of a rare overflow stays empty (a few replicas rerun cheaply)
    assert g._cap_scale == {}


def test_tie_flagged_replicas_rerun_on_the_exact_sweep():
    """C3 plus a registered static plugin whose posts are rounded to 1e-3 (Bursty): some
    replicas meet equal event times, the fast sweep flags them RQ_ST_TIE and only they
    rerun on the exact sequential sweep; the batch equals the all-sequential run bit for
    bit."""
    torch, L, engine, graphs = _ctx()
    from realdata_worlds import BurstyMixin
    from redqueen_amd.opt_model import Broadcaster

    class Bursty(BurstyMixin, Broadcaster):
        pass
    so = graphs.c3()
    fol = sorted({b for a, b in so["edge_list"] if a != so["src_id"]})[:40]
    so = dict(so, other_sources=so["other_sources"] + [(Bursty, {"src_id": 9000, "seed": 1,
                                                                 "rate": 0.02, "size": 6})],
              edge_list=so["edge_list"] + [(9000, f) for f in fol])
    g = _graph(engine, so)
    R = 512
    kw = dict(q=so["q"], s=so["s"], n_rep=R, ctrl_seed=3, world_seed=3, randomize=True, Ks=(1, 2))
    raw = g.run("opt", check=False, **kw)
    tied = int(((raw.status & L.ST_TIE) != 0).sum().item())
    assert 0 < tied < R // 2
    got = g.run("opt", **kw)
    assert g.reruns == tied
    seq = g.run("opt", sweep_mode=2, **kw)
    _same(torch, got, seq)


def test_device_realdata_streams_on_the_fast_sweep():
    """Per-replica RealData times handed over as device arrays (Graph.run(rd_streams=...),
    rq_batch_desc.rd_*): the fast sweep plays them (no graph-level repeats), and replica
    k equals a one-replica run whose graph carries replica k's times as its own RealData
    source (same seeds), and the engine oracle."""
    torch, L, engine, graphs = _ctx()
    from oracle import oracle as O
    so = graphs.c3()
    fol = sorted({b for a_, b in so["edge_list"] if a_ != so["src_id"]})[::25]
    base = dict(so, edge_list=so["edge_list"] + [(9000, f) for f in fol])
    world = dict(base, other_sources=so["other_sources"] + [("RealData", {"src_id": 9000, "times": []})])
    g = _graph(engine, world)
    R, n = 6, 40
    rs = np.random.RandomState(11)
    host = [np.sort(rs.uniform(0, so["end_time"], n)) for _ in range(R)]
    t = torch.from_numpy(np.concatenate(host)).cuda()
    off = torch.arange(0, R * n + 1, n, dtype=torch.int64, device="cuda")
    kw = dict(q=so["q"], s=so["s"], ctrl_seed=40, world_seed=40, randomize=True, Ks=(1, 2))
    plan = g.run("opt", n_rep=R, plan_only=True, **kw)
    assert plan["variant"] % 10 not in (1, 4), plan
    res = g.run("opt", n_rep=R, event_log=True, rd_streams=([9000], t, off, [n]), **kw)
    assert int(res.status.max().item()) == 0
    for k in (0, 3, R - 1):
        wk = dict(base, other_sources=so["other_sources"] + [("RealData", {"src_id": 9000, "times": host[k]})])
        gk = _graph(engine, wk)
        one = gk.run("opt", n_rep=1, q=so["q"], s=so["s"], ctrl_seed=40 + k, world_seed=40 + k,
                     randomize=True, Ks=(1, 2), event_log=True)
        assert torch.equal(one.metrics[0], res.metrics[k]) and torch.equal(one.counts[0], res.counts[k])
        # the engine oracle of replica k's world (randomize_other_sources(40 + k))
        sc_so = dict(wk, other_sources=[(nm, dict(x, seed=40 + k + 99 * j) if "seed" in x else x)
                                        for j, (nm, x) in enumerate(wk["other_sources"])])
        t_o, _dt, s_o = O.engine_run(O.Scenario(sc_so, ("opt", 40 + k)))
        te, se = res.events(k)
        assert np.array_equal(te, t_o) and np.array_equal(se, s_o)


def test_more_caller_streams_than_side_pipes():
    """Batches issued round-robin on six caller streams -- more than the library's four
    side-stream pipes per thread (rq_api.cpp SidePipes: keyed by device and caller stream,
    least recently used re-homed) -- give the same rows as one stream."""
    torch, L, engine, graphs = _ctx()
    so = graphs.c3()
    g = _graph(engine, so)
    kw = dict(q=so["q"], s=so["s"], n_rep=2000, randomize=True, Ks=(1,), check=False)
    ref = [g.run("opt", ctrl_seed=k, world_seed=k, **kw) for k in range(12)]
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream() for _ in range(6)]
    got = []
    for k in range(12):
        with torch.cuda.stream(streams[k % 6]):
            got.append(g.run("opt", ctrl_seed=k, world_seed=k, **kw))
    torch.cuda.synchronize()
    for a, b in zip(ref, got):
        assert torch.equal(a.metrics, b.metrics) and torch.equal(a.counts, b.counts)
