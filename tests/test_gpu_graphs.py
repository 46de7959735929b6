"""Every graph the reference accepts (Manager.__init__, opt_model.py:158-175), on the
GPU, bit for bit against the engine-semantics oracle (oracle/rq_oracle.c):

* multigraphs -- duplicate (source, sink) edges: each event repeats the sink's rows
  (opt_model.py:306-307), RedQueen's tracked rank grows by the multiplicity
  (:74-76) and the pivot cells average the repeated rows' ranks; the all-RealData
  multigraph worlds equal the REFERENCE's own df (tests/test_gpu_realdata.py,
  realdata.npz rdmg*);
* more than 512 sources (the two-level merge feeding the fast sweep, up to 262144; the
  sequential sweep at 16 and 32 sources per lane up to 2048, on the merged sequence
  above);
* the repeat-stream skip of the per-wave sink-bit sweep (a stream's second event
  before the next reset walks no sinks): on and off, bit for bit;
* 50k sinks (per-wave sink bits for K = 1, int16 ranks for K > 1, and the
  sequential sweep with its per-sink state in global memory).

A duplicated CONTROLLED edge with a RedQueen controller is refused (RQ_EINVAL /
ValueError): the reference's sqrt_s_by_q (one entry per edge) no longer matches
its ranks (one per distinct follower) and its first non-own event raises.
"""
import numpy as np
import pytest

from tests.test_gpu_engine import _cmp_replica, _ctx, _graph, _oracle, _world_with_seeds

pytestmark = pytest.mark.gpu


def _multigraph(rs, n_src=12, n_sinks=40, deg=6, n_fol=10, ctrl_dup=False):
    """A C3-like world whose wall sources repeat some of their edges 1-3 times."""
    sinks = list(range(1, n_sinks + 1))
    fol = sorted(int(x) for x in rs.choice(sinks, n_fol, replace=False))
    edges = [(1, f) for f in fol]
    if ctrl_dup:
        edges += [(1, fol[0]), (1, fol[3])]
    others = []
    for k in range(n_src):
        sid = 100 + k
        for y in rs.choice(sinks, deg, replace=False):
            for _ in range(1 + (rs.randint(0, 4) if rs.rand() < 0.4 else 0)):
                edges.append((sid, int(y)))
        if k % 2:
            others.append(("Hawkes", {"src_id": sid, "seed": 7 + k, "l_0": 0.6, "alpha": 1.0, "beta": 5.0}))
        else:
            others.append(("Poisson2", {"src_id": sid, "seed": 7 + k, "rate": 0.8}))
    order = rs.permutation(len(edges))
    edges = [edges[i] for i in order]   # duplicates anywhere in the list
    return dict(src_id=1, end_time=40.0, q=2.0, s=1.0, sink_ids=sinks, other_sources=others,
                edge_list=edges)


@pytest.mark.parametrize("event_log", [False, True])
def test_multigraph_redqueen_randomized(event_log):
    torch, engine, graphs, O = _ctx()
    so = _multigraph(np.random.RandomState(3))
    g = _graph(engine, so)
    Ks = (1, 2, 5)
    R = 24
    res = g.run("opt", q=so["q"], s=so["s"], n_rep=R, ctrl_seed=40, world_seed=40, randomize=True,
                Ks=Ks, event_log=event_log)
    assert int(res.status.max().item()) == 0
    for r in range(0, R, 5):
        u = 40 + r
        met_o, t_o, s_o = _oracle(O, _world_with_seeds(so, u), ("opt", u), Ks)
        _cmp_replica(res, r, met_o, t_o, s_o, Ks)
    if event_log:   # the exported df repeats the duplicated sinks' rows
        df = res.dataframe(0)
        sc = O.Scenario(_world_with_seeds(so, 40), ("opt", 40))
        t, dt, s = O.engine_run(sc)
        cols = sc.expand(t, dt, s)
        for c in ("event_id", "src_id", "t", "sink_id"):
            assert np.array_equal(df[c].values, cols[c]), c


def test_multigraph_duplicated_controlled_edges():
    """A Poisson2 controlled source with duplicated follower edges posts the
    duplicated rows too; RedQueen with them is refused like the reference raises."""
    torch, engine, graphs, O = _ctx()
    from redqueen_amd import _lib as L
    from redqueen_amd.opt_model import SimOpts
    so = _multigraph(np.random.RandomState(5), ctrl_dup=True)
    g = _graph(engine, so)
    res = g.run("poisson", ctrl_seed=9, ctrl_rate=[2.5], n_rep=1, Ks=(1, 2), event_log=True)
    met_o, t_o, s_o = _oracle(O, so, ("poisson", 9, 2.5), (1, 2))
    _cmp_replica(res, 0, met_o, t_o, s_o, (1, 2))
    with pytest.raises(L.RQError) as e:
        g.run("opt", q=1.0, s=1.0, n_rep=1, ctrl_seed=1)
    assert e.value.code == L.RQ_EINVAL
    m = SimOpts(**so).create_manager_with_opt(3)
    with pytest.raises(ValueError):
        m.run_dynamic()


def _many_sources(n_src, n_sinks=120, deg=3, T=6.0, seed=11):
    rs = np.random.RandomState(seed)
    sinks = list(range(1, n_sinks + 1))
    fol = sorted(int(x) for x in rs.choice(sinks, 30, replace=False))
    edges = [(0, f) for f in fol]
    others = []
    for k in range(n_src):
        sid = 1000 + k
        edges += [(sid, int(y)) for y in rs.choice(sinks, deg, replace=False)]
        if k % 3 == 0:
            others.append(("Hawkes", {"src_id": sid, "seed": k, "l_0": 0.3, "alpha": 1.0, "beta": 4.0}))
        else:
            others.append(("Poisson2", {"src_id": sid, "seed": k, "rate": 0.4}))
    return dict(src_id=0, end_time=T, q=1.0, s=1.0, sink_ids=sinks, other_sources=others,
                edge_list=edges)


@pytest.mark.parametrize("n_src,seq", [(600, False), (1500, False), (3000, False), (6000, False),
                                       (12000, False), (40000, False), (600, True), (1500, True),
                                       (3000, True), (6000, True), (12000, True)])
def test_more_than_512_sources(n_src, seq):
    """> 512 sources: the fast general sweep plays the two-level merged sequence
    (rq_merge_streams over groups of 512 streams, then over the groups' sequences; any
    number of sources up to 65535); the exact sequential sweep (sweep_mode 2) owns 16 / 32
    sources per lane up to 2048 and plays the same merged sequence above that.  Past the
    per-stream tables LDS takes (~8k streams) both read them from global memory (the GT
    instances).  Event logs and metrics == the engine oracle."""
    torch, engine, graphs, O = _ctx()
    so = _many_sources(n_src)
    g = _graph(engine, so)
    kw = dict(sweep_mode=2) if seq else {}
    plan = g.run("opt", q=1.0, s=1.0, n_rep=4, plan_only=True, **kw)
    if seq:
        assert plan["variant"] in (1, 4), plan
        assert plan["sources_per_lane"] == (16 if n_src <= 1024 else 32 if n_src <= 2048 else 0), plan
    else:
        assert plan["variant"] not in (1, 4) and plan["sources_per_lane"] == 0, plan
    Ks = (1, 2)
    res = g.run("opt", q=1.0, s=1.0, n_rep=4, ctrl_seed=2, world_seed=2, randomize=True, Ks=Ks,
                event_log=True, **kw)
    assert int(res.status.max().item()) == 0
    for r in (0, 3):
        met_o, t_o, s_o = _oracle(O, _world_with_seeds(so, 2 + r), ("opt", 2 + r), Ks)
        _cmp_replica(res, r, met_o, t_o, s_o, Ks)
    if not seq:   # and without the event log, K = 1 (the per-wave sink-bit instance)
        r1 = g.run("opt", q=1.0, s=1.0, n_rep=4, ctrl_seed=2, world_seed=2, randomize=True, Ks=(1,))
        met_o, t_o, s_o = _oracle(O, _world_with_seeds(so, 2 + 3), ("opt", 2 + 3), (1,))
        _cmp_replica(r1, 3, met_o, t_o, s_o, (1,))


def test_65000_sources_fast_equals_sequential():
    """The largest graph the u16 stream ids take: the fast and the sequential sweep on
    merged streams with global per-stream tables agree bit for bit (and the plan says so)."""
    torch, engine, graphs, O = _ctx()
    so = _many_sources(65000, T=2.0)
    g = _graph(engine, so)
    assert g.run("opt", q=1.0, s=1.0, n_rep=4, plan_only=True)["sources_per_lane"] == 0
    a = g.run("opt", q=1.0, s=1.0, n_rep=4, ctrl_seed=3, world_seed=3, randomize=True, Ks=(1, 2),
              event_log=True)
    b = g.run("opt", q=1.0, s=1.0, n_rep=4, ctrl_seed=3, world_seed=3, randomize=True, Ks=(1, 2),
              event_log=True, sweep_mode=2)
    assert int(a.status.max().item()) == 0 and int((b.status & 3).max().item()) == 0
    assert torch.equal(a.metrics, b.metrics) and torch.equal(a.counts, b.counts)
    for r in range(4):
        ta, sa = a.events(r)
        tb, sb = b.events(r)
        assert np.array_equal(ta, tb) and np.array_equal(sa, sb)


@pytest.mark.parametrize("n_src", [70000, 140000])
def test_more_than_65535_sources(n_src):
    """Past the u16 stream ids (round 6): the two-level merge carries group-local ids at
    its first level and global ones at the second, with each entry's bits 16-23 in a side
    array the sweeps read (rq_batch_desc limit: 512 groups of 512 = 262144 sources).  The
    fast and the sequential sweep agree bit for bit, events included, and replica 0 ==
    the engine oracle."""
    torch, engine, graphs, O = _ctx()
    so = _many_sources(n_src, T=0.5)
    g = _graph(engine, so)
    assert g.n_streams == n_src + 1
    kw = dict(q=1.0, s=1.0, n_rep=2, ctrl_seed=4, world_seed=4, randomize=True, Ks=(1, 2),
              event_log=True)
    a = g.run("opt", **kw)
    b = g.run("opt", sweep_mode=2, **kw)
    assert int(a.status.max().item()) == 0 and int((b.status & 3).max().item()) == 0
    assert torch.equal(a.metrics, b.metrics) and torch.equal(a.counts, b.counts)
    for r in range(2):
        ta, sa = a.events(r)
        tb, sb = b.events(r)
        assert np.array_equal(ta, tb) and np.array_equal(sa, sb)
    assert int(sa.max()) > 1000 + 65535   # streams past the u16 range did play
    met_o, t_o, s_o = _oracle(O, _world_with_seeds(so, 4), ("opt", 4), (1, 2))
    _cmp_replica(a, 0, met_o, t_o, s_o, (1, 2))


def test_more_than_2048_sources_what_needs_the_sequential_sweep():
    """Past 2048 sources the runs that need the exact sequential sweep run on the merged
    sequence (round 4: RQ_EUNSUPPORTED): a RealData source with repeated times among 3000
    and a multigraph -- == the engine oracle; max_events among 3000 sources runs the fast
    general sweep since round 6 (truncate_tile) -- == the engine oracle too; and a
    3000-source fast run == its sequential twin on a continuous world."""
    torch, engine, graphs, O = _ctx()
    so = _many_sources(3000)
    # a RealData broadcaster (recorded times, with repeats) and a duplicated edge
    rd = np.round(np.sort(np.random.RandomState(4).uniform(0, so["end_time"], 25)), 1)
    so_rd = dict(so, other_sources=so["other_sources"] + [("RealData", {"src_id": 9000, "times": rd})],
                 edge_list=so["edge_list"] + [(9000, 3), (9000, 7), (1000, so["edge_list"][30][1])])
    Ks = (1, 3)
    for world, kw, seq in ((so_rd, {}, True), (so, dict(max_events=400), False)):
        g = _graph(engine, world)
        plan = g.run("opt", q=1.0, s=1.0, n_rep=3, plan_only=True, **kw)
        assert (plan["variant"] in (1, 4)) == seq and plan["sources_per_lane"] == 0, plan
        res = g.run("opt", q=1.0, s=1.0, n_rep=3, ctrl_seed=5, world_seed=5, randomize=True, Ks=Ks,
                    event_log=True, **kw)
        assert int((res.status & 3).max().item()) == 0
        for r in (0, 2):
            met_o, t_o, s_o = _oracle(O, _world_with_seeds(world, 5 + r), ("opt", 5 + r), Ks,
                                      max_events=kw.get("max_events"))
            _cmp_replica(res, r, met_o, t_o, s_o, Ks)
    g = _graph(engine, so)
    a = g.run("opt", q=1.0, s=1.0, n_rep=64, ctrl_seed=1, world_seed=1, randomize=True, Ks=Ks)
    b = g.run("opt", q=1.0, s=1.0, n_rep=64, ctrl_seed=1, world_seed=1, randomize=True, Ks=Ks,
              sweep_mode=2)
    assert torch.equal(a.metrics, b.metrics) and torch.equal(a.counts, b.counts)


def _bursty(n_src=200, n_sinks=3000, deg=40, n_fol=900, T=6.0, seed=17):
    """Per-wave sink bits on merged streams (K = 1, too many streams x sink words for
    the BITS tables): bursty Hawkes streams, so a stream often plays again before the
    controller's next post."""
    rs = np.random.RandomState(seed)
    sinks = list(range(1, n_sinks + 1))
    fol = sorted(int(x) for x in rs.choice(sinks, n_fol, replace=False))
    edges = [(0, f) for f in fol]
    others = []
    for k in range(n_src):
        sid = 10 + k
        d = 0 if k % 37 == 5 else (150 if k % 29 == 3 else deg)   # no sinks / > 128 sinks
        edges += [(sid, int(y)) for y in rs.choice(sinks, d, replace=False)]
        if k % 2:
            others.append(("Hawkes", {"src_id": sid, "seed": k, "l_0": 0.4, "alpha": 1.0, "beta": 1.6}))
        else:
            others.append(("Poisson2", {"src_id": sid, "seed": k, "rate": 0.7}))
    return dict(src_id=0, end_time=T, q=0.05, s=1.0, sink_ids=sinks, other_sources=others,
                edge_list=edges)


@pytest.mark.parametrize("ctrl", ["opt", "poisson"])
def test_repeat_stream_skip(ctrl, monkeypatch):
    """The per-wave sink-bit sweep skips the sink walk of an event whose stream already
    played since the last reset (a post, or -- Poisson control -- an own-stream
    arrival): every sink of its row is out of the top-1 set and valid.  Skip on
    (default) == skip off (RQ_SKIP=0) bit for bit, and both == the engine oracle."""
    torch, engine, graphs, O = _ctx()
    so = _bursty()
    g = _graph(engine, so)
    R, Ks = 12, (1,)
    kw = dict(n_rep=R, ctrl_seed=30, world_seed=30, randomize=True, Ks=Ks)
    if ctrl == "opt":
        args, kw = ("opt",), dict(kw, q=so["q"], s=so["s"])
    else:
        args, kw = ("poisson",), dict(kw, ctrl_rate=[3.0])
    plan = g.run(*args, plan_only=True, **kw)
    assert plan["variant"] == 3 and plan["sources_per_lane"] == 0, plan
    res = g.run(*args, **kw)
    monkeypatch.setenv("RQ_SKIP", "0")
    res0 = g.run(*args, **kw)
    monkeypatch.delenv("RQ_SKIP")
    assert int(res.status.max().item()) == 0
    assert torch.equal(res.metrics, res0.metrics)
    assert torch.equal(res.counts, res0.counts)
    for r in (0, 5, R - 1):
        c = ("opt", 30 + r) if ctrl == "opt" else ("poisson", 30 + r, 3.0)
        met_o, t_o, s_o = _oracle(O, _world_with_seeds(so, 30 + r), c, Ks)
        _cmp_replica(res, r, met_o, t_o, s_o, Ks)


def _wide(n_sinks=50000, n_src=40, deg=60, T=4.0):
    rs = np.random.RandomState(21)
    sinks = list(range(10, 10 + n_sinks))
    fol = sorted(int(x) for x in rs.choice(sinks, 400, replace=False))
    edges = [(1, f) for f in fol]
    others = []
    for k in range(n_src):
        sid = 2 + k
        ys = [int(y) for y in rs.choice(sinks, deg, replace=False)]
        ys += [int(y) for y in rs.choice(fol, 6, replace=False) if int(y) not in ys][:3]
        edges += [(sid, y) for y in ys]   # a simple graph (no duplicated edge)
        others.append(("Poisson2", {"src_id": sid, "seed": 3 + k, "rate": 1.5}))
    return dict(src_id=1, end_time=T, q=0.5, s=1.0, sink_ids=sinks, other_sources=others,
                edge_list=edges)


@pytest.mark.parametrize("Ks,kw,variant", [
    ((1,), {}, 3),                                  # K = 1: per-wave LDS sink bits
    ((1, 2), {}, 0),                                # int16 ranks, one wave per block (fused or not)
    ((1, 2), dict(sweep_mode=2, event_log=True), 4),   # sequential, per-sink state in HBM
])
def test_50k_sinks(Ks, kw, variant):
    torch, engine, graphs, O = _ctx()
    so = _wide()
    g = _graph(engine, so)
    plan = g.run("opt", q=so["q"], s=so["s"], n_rep=6, Ks=Ks, plan_only=True, **kw)
    assert plan["variant"] % 10 == variant, plan
    res = g.run("opt", q=so["q"], s=so["s"], n_rep=6, ctrl_seed=70, world_seed=70, randomize=True,
                Ks=Ks, **kw)
    assert int(res.status.max().item()) == 0
    for r in (0, 5):
        met_o, t_o, s_o = _oracle(O, _world_with_seeds(so, 70 + r), ("opt", 70 + r), Ks)
        _cmp_replica(res, r, met_o, t_o, s_o, Ks)
