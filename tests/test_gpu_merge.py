"""The general fast sweep on merged streams (rq_merge_streams, the default for > 64
sources) against the same sweep merging the per-source streams itself (sweep_mode 6)
and against the engine oracle.

The merge must reproduce the play order of Manager.run_dynamic (opt_model.py:241-314)
as the engine defines it: time order, equal times in stream order, a source's equal
times in stream order.  Bar: bit-exact event logs, counts, status and metrics.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _ctx():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from redqueen_amd import engine, graphs
    from oracle import oracle as O
    return torch, engine, graphs, O


def _graph(engine, so):
    return engine.Graph(so["src_id"], so["other_sources"], so["sink_ids"], so["edge_list"],
                        so["end_time"])


def _same(torch, a, b, events=True):
    assert torch.equal(a.status, b.status)
    assert torch.equal(a.counts, b.counts)
    assert torch.equal(a.metrics.isnan(), b.metrics.isnan())
    assert torch.equal(a.metrics.nan_to_num(), b.metrics.nan_to_num())
    if events and a.ev_t is not None:
        for i in range(a.counts.shape[0]):
            ta, sa = a.events(i)
            tb, sb = b.events(i)
            assert np.array_equal(ta, tb) and np.array_equal(sa, sb), i


def _bursty(graphs, n_src=200, n_fol=300, seed=5):
    """A > 64-source world: Poisson2 + bursty Hawkes walls, degree 4."""
    return graphs.followers_graph(num_followers=n_fol, num_sources=n_src, degree=4, end_time=40.0,
                                  kinds=("Poisson2", "Hawkes"), world_rate=0.7, alpha=1.5,
                                  beta=2.5, seed=seed, network_seed=seed + 1)


@pytest.mark.parametrize("Ks", [(1,), (1, 2, 5)])
@pytest.mark.parametrize("world", ["g120", "bursty"])
def test_merged_equals_windowed(world, Ks):
    torch, engine, graphs, O = _ctx()
    so = graphs.g120() if world == "g120" else _bursty(graphs)
    g = _graph(engine, so)
    kw = dict(q=so["q"], s=so["s"], n_rep=300, ctrl_seed=77, world_seed=77, randomize=True, Ks=Ks)
    plan = g.run("opt", plan_only=True, **kw)
    assert plan["sources_per_lane"] == 0, plan          # merged streams
    assert g.run("opt", plan_only=True, sweep_mode=6, **kw)["sources_per_lane"] >= 2
    a = g.run("opt", **kw)
    b = g.run("opt", sweep_mode=6, **kw)
    _same(torch, a, b)
    # event logs of the fast sweep: merged == windowed, and == the engine oracle
    a = g.run("opt", event_log=True, **kw)
    b = g.run("opt", event_log=True, sweep_mode=6, **kw)
    _same(torch, a, b)
    for r in (0, 151, 299):
        u = 77 + r
        w = dict(so)
        w["other_sources"] = [(n, dict(x, seed=(u + 99 * i) & 0xFFFFFFFF)) if "seed" in x else (n, x)
                              for i, (n, x) in enumerate(so["other_sources"])]
        met, (t_o, _, s_o) = O.engine_metrics(O.Scenario(w, ("opt", u)), Ks)
        t, s = a.events(r)
        assert np.array_equal(t, t_o) and np.array_equal(s, s_o), r
        top, avg, r2, _ = met
        assert np.array_equal(a.metrics[r].cpu().numpy(), np.asarray(list(top) + [avg, r2])), r


def test_merged_poisson_controlled_many_sources():
    """A Poisson2-controlled run (the controlled stream is one of the merged streams)."""
    torch, engine, graphs, O = _ctx()
    so = _bursty(graphs, n_src=150, n_fol=120, seed=9)
    g = _graph(engine, so)
    rates = torch.linspace(0.0, 6.0, 64, dtype=torch.float64)
    kw = dict(n_rep=64, ctrl_seed=3, world_seed=3, randomize=True, ctrl_rate=rates, Ks=(1, 3))
    _same(torch, g.run("poisson", **kw), g.run("poisson", sweep_mode=6, **kw))
    _same(torch, g.run("poisson", event_log=True, **kw),
          g.run("poisson", event_log=True, sweep_mode=6, **kw))


@pytest.mark.parametrize("world", ["readme", "eight"])
def test_small_merge_equals_bucket_merge(world, monkeypatch):
    """<= 8 streams: one thread merges a replica (rq_merge_small) -- the same merged
    sequence as the bucket rounds of rq_merge_streams (RQ_MERGE_SMALL=0), event for
    event, and the engine oracle."""
    torch, engine, graphs, O = _ctx()
    so = graphs.readme() if world == "readme" else \
        graphs.followers_graph(num_followers=40, num_sources=7, degree=3, end_time=30.0,
                               kinds=("Poisson2", "Hawkes"), world_rate=1.5, alpha=1.5, beta=2.5,
                               seed=8, network_seed=9)
    g = _graph(engine, so)
    kw = dict(q=so["q"], s=so["s"], n_rep=700, ctrl_seed=21, world_seed=21, randomize=True,
              Ks=(1, 2), event_log=True)
    assert g.run("opt", plan_only=True, **kw)["sources_per_lane"] == 0   # merged streams
    a = g.run("opt", **kw)
    monkeypatch.setenv("RQ_MERGE_SMALL", "0")
    b = g.run("opt", **kw)
    monkeypatch.delenv("RQ_MERGE_SMALL")
    _same(torch, a, b)
    assert int(a.status.max().item()) == 0
    from tests.test_gpu_engine import _cmp_replica, _oracle, _world_with_seeds
    for r in (0, 699):
        met_o, t_o, s_o = _oracle(O, _world_with_seeds(so, 21 + r), ("opt", 21 + r), (1, 2))
        _cmp_replica(a, r, met_o, t_o, s_o, (1, 2))


def _tie_world(n_at5):
    T = np.sort(np.concatenate([np.full(n_at5, 5.0), np.full(700, 7.25), np.linspace(0.5, 19.5, 301)]))
    return dict(src_id=1, end_time=20.0, s=np.asarray([1.0, 2.0, 0.5]), q=0.7, sink_ids=[10, 11, 12, 13],
                other_sources=[("RealData", {"src_id": 2, "times": T.tolist()}),
                               ("Poisson", {"src_id": 3, "seed": 5, "rate": 30.0}),
                               ("Hawkes", {"src_id": 4, "seed": 9, "l_0": 5.0, "alpha": 2.0, "beta": 5.0}),
                               ("RealData", {"src_id": 5, "times": [5.0] * 9 + [7.25, 9.0]})],
                edge_list=[(1, 10), (1, 11), (1, 13), (2, 10), (2, 12), (3, 11), (4, 12), (4, 13),
                           (5, 13), (5, 10)])


@pytest.mark.parametrize("small", ["0", "1"])
def test_merged_equal_time_groups(small, monkeypatch):
    """Equal-time groups larger than a merge round's buffer share (1500 arrivals at one
    time, 700 at another) on the fast sweeps forced by sweep_mode 5 (legacy kernels:
    merged) and 6 with sweep_mode-1-like RealData handling: the merged order equals the
    windowed one.  The bucket merge (RQ_MERGE_SMALL=0) flags TIE; the per-thread merge
    of a few streams (the default at <= 8) has no equal-time cap."""
    torch, engine, graphs, O = _ctx()
    monkeypatch.setenv("RQ_MERGE_SMALL", small)
    so = _tie_world(1500)
    g = _graph(engine, so)
    for seed in (1, 2):
        a = g.run("opt", q=so["q"], s=so["s"], n_rep=4, ctrl_seed=seed, Ks=(1, 3), sweep_mode=5,
                  event_log=True, check=False)
        b = g.run("opt", q=so["q"], s=so["s"], n_rep=4, ctrl_seed=seed, Ks=(1, 3), sweep_mode=1,
                  event_log=True, check=False)
        if small == "0":   # (the sweep flags equal times too: no assertion the other way)
            assert int(a.status[0].item()) & 4
        # the fused sweep (mode 1) and the merged general sweep (mode 5) play the same events
        for i in range(4):
            ta, sa = a.events(i)
            tb, sb = b.events(i)
            assert np.array_equal(ta, tb) and np.array_equal(sa, sb)
        assert torch.equal(a.counts, b.counts) and torch.equal(a.metrics, b.metrics)


@pytest.mark.parametrize("small", ["0", "1"])
def test_merged_tie_group_beyond_round_capacity(small, monkeypatch):
    """3000 arrivals at one time: more than one merge round holds.  The bucket merge
    (RQ_MERGE_SMALL=0) emits them in rounds and flags RQ_ST_TIE; with check=True the
    engine reruns the batch on the exact sequential sweep, so the result equals
    sweep_mode 2 and the oracle.  The per-thread merge of a few streams orders them
    exactly."""
    torch, engine, graphs, O = _ctx()
    monkeypatch.setenv("RQ_MERGE_SMALL", small)
    so = _tie_world(3000)
    g = _graph(engine, so)
    a = g.run("opt", q=so["q"], s=so["s"], n_rep=2, ctrl_seed=4, Ks=(1, 2), sweep_mode=5, check=False)
    if small == "0":
        assert int(a.status[0].item()) & 4
    assert int(a.counts[0, 2].item()) > 0
    b = g.run("opt", q=so["q"], s=so["s"], n_rep=2, ctrl_seed=4, Ks=(1, 2), sweep_mode=5)
    c = g.run("opt", q=so["q"], s=so["s"], n_rep=2, ctrl_seed=4, Ks=(1, 2), sweep_mode=2)
    _same(torch, b, c, events=False)
    met, (t_o, _, s_o) = O.engine_metrics(O.Scenario(so, ("opt", 4)), (1, 2))
    top, avg, r2, _ = met
    assert np.array_equal(b.metrics[0].cpu().numpy(), np.asarray(list(top) + [avg, r2]))


@pytest.mark.parametrize("wl", ["c3", "g120"])
def test_pipelined_chunks_and_longest_first_order(wl, monkeypatch):
    """rq_run_batch's chunk plans change no result bit: one chunk larger than the resident
    sweep slots in index order and in the longest-first order of rq_order_replicas
    (RQ_ORDER=1: the work queue hands the replicas out by length), the default two
    pipelined chunks, and many small chunks on two streams (fork / join events) give
    identical per-replica outputs."""
    torch, engine, graphs, O = _ctx()
    so = getattr(graphs, wl)()
    g = _graph(engine, so)
    R = 9000 if wl == "c3" else 12000
    kw = dict(q=so["q"], s=so["s"], n_rep=R, ctrl_seed=77, world_seed=77, randomize=True, Ks=(1,))
    idx = g.run("opt", chunk=R, **kw)
    monkeypatch.setenv("RQ_ORDER", "1")
    one = g.run("opt", chunk=R, **kw)
    monkeypatch.delenv("RQ_ORDER")
    _same(torch, one, idx)
    assert g.run("opt", chunk=R, plan_only=True, **kw)["chunk"] == R
    dflt = g.run("opt", **kw)
    small = g.run("opt", chunk=700, **kw)
    assert int(one.status.max().item()) == 0
    _same(torch, one, dflt)
    _same(torch, one, small)
