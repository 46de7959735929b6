"""GPU parity of the simulation engine against the CPU oracle (engine semantics).

The oracle (oracle/rq_oracle.c, rqo_engine_run) is an independent sequential
restatement of the engine semantics; the metrics it reports come from the
Appendix-B restatement of utils.py applied to the *expanded dataframe*
(rqo_metrics_df), i.e. a different algorithm than the kernels' incremental
row aggregates.  The bar is bit-exact equality of every event time, every
source id and every metric double.
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


def _world_with_seeds(so, u):
    """randomize_other_sources(u): other-source idx gets seed u + 99*idx (opt_model.py:795-804)."""
    so = dict(so)
    so["other_sources"] = [(n, dict(kw, seed=(u + 99 * i) & 0xFFFFFFFF)) if "seed" in kw else (n, kw)
                           for i, (n, kw) in enumerate(so["other_sources"])]
    return so


def _graph(engine, so):
    ctrl_a = ctrl_b = None
    return engine.Graph(so["src_id"], so["other_sources"], so["sink_ids"], so["edge_list"],
                        so["end_time"], ctrl_a=ctrl_a, ctrl_b=ctrl_b)


def _oracle(O, so, ctrl, Ks, max_events=None):
    sc = O.Scenario(so, ctrl, max_events=max_events)
    met, (t, dt, s) = O.engine_metrics(sc, Ks)
    return met, t, s


MODES = ["fast", "scatter", "log", "legacy", "fastlog", "legacylog", "window", "windowlog", "gen", "genlog"]


def _mode_kw(mode):
    """fast: the fused windowed sweep (K=1 runs on sink bitsets); scatter: the same
    with per-sink LDS ranks (sweep_mode=3); log: the sequential event-log variant
    (sweep_mode=2), events compared too; legacy: pre-generated streams + serial
    wave-min merge (sweep_mode=4); fastlog: the fused sweep writing the event log
    itself (event_log=True, auto mode), events compared too; legacylog: the general
    (pre-generated streams) fast sweep writing the event log (sweep_mode=4).
    legacy / legacylog play the streams merged by rq_merge_streams; window /
    windowlog (sweep_mode=6) the same general sweep merging the streams itself
    (per-source register windows).  fast / fastlog / scatter run the fused sweep on
    merged streams (the default); gen / genlog (sweep_mode=7) the fused sweep generating
    its arrivals in-kernel."""
    if mode == "windowlog":
        return dict(event_log=True, sweep_mode=6)
    if mode == "genlog":
        return dict(event_log=True, sweep_mode=7)
    if mode == "log":
        return dict(event_log=True, sweep_mode=2)
    if mode == "fastlog":
        return dict(event_log=True, sweep_mode=0)
    if mode == "legacylog":
        return dict(event_log=True, sweep_mode=4)
    return dict(event_log=False, sweep_mode={"scatter": 3, "legacy": 4, "window": 6, "gen": 7}.get(mode, 0))


def _cmp_replica(res, i, met_o, t_o, s_o, Ks):
    if res.ev_t is not None:
        t, s = res.events(i)
        assert t.shape == t_o.shape, (t.shape, t_o.shape)
        assert np.array_equal(s, s_o)
        assert np.array_equal(t, t_o), np.max(np.abs(t - t_o))
    m = res.metrics[i].cpu().numpy()
    top, avg, r2, cnt = met_o
    exp = np.asarray(list(top) + [avg, r2])
    assert np.array_equal(m, exp), (m, exp)
    c = res.counts[i].cpu().numpy()
    assert c[0] == cnt[0] and c[1] == cnt[1] and c[3] == cnt[2], (c, cnt)
    assert c[2] == len(t_o)


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("seed", [101, 5, 7])
def test_readme_single(seed, mode):
    torch, engine, graphs, O = _ctx()
    so = graphs.readme()
    g = _graph(engine, so)
    Ks = (1, 2, 5)
    res = g.run("opt", q=so["q"], s=so["s"], n_rep=1, ctrl_seed=seed, Ks=Ks, **_mode_kw(mode))
    met_o, t_o, s_o = _oracle(O, so, ("opt", seed), Ks)
    _cmp_replica(res, 0, met_o, t_o, s_o, Ks)
    assert int(res.status[0].item()) == 0


@pytest.mark.parametrize("mode", MODES)
def test_readme_batch_randomized(mode):
    torch, engine, graphs, O = _ctx()
    so = graphs.readme()
    g = _graph(engine, so)
    R = 48
    res = g.run("opt", q=so["q"], s=so["s"], n_rep=R, ctrl_seed=1000, world_seed=1000,
                randomize=True, Ks=(1,), **_mode_kw(mode))
    for r in range(0, R, 7):
        u = 1000 + r
        met_o, t_o, s_o = _oracle(O, _world_with_seeds(so, u), ("opt", u), (1,))
        _cmp_replica(res, r, met_o, t_o, s_o, (1,))


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("seed", [3, 4, 17])
def test_mixed_kinds(seed, mode):
    torch, engine, graphs, O = _ctx()
    so = graphs.mixed()
    g = _graph(engine, so)
    Ks = (1, 2, 5, 10)
    res = g.run("opt", q=so["q"], s=so["s"], n_rep=1, ctrl_seed=seed, Ks=Ks, **_mode_kw(mode))
    met_o, t_o, s_o = _oracle(O, so, ("opt", seed), Ks)
    _cmp_replica(res, 0, met_o, t_o, s_o, Ks)


@pytest.mark.parametrize("mode", MODES)
def test_kat_weights_and_grid(mode):
    torch, engine, graphs, O = _ctx()
    so = graphs.kat_two_walls((0.5, 1.5))
    g = _graph(engine, so)
    qs = np.asarray([0.01, 1.0, 30.0])
    s = np.asarray([[0.5, 1.5], [1.0, 1.0], [1.5, 0.25]])
    res = g.run("opt", q=qs, s=s, n_rep=3, ctrl_seed=11, seed_mod=3, Ks=(1, 2), **_mode_kw(mode))
    for gi in range(3):
        for r in range(3):
            sog = dict(so, q=float(qs[gi]), s=s[gi])
            met_o, t_o, s_o = _oracle(O, sog, ("opt", 11 + r), (1, 2))
            _cmp_replica(res, gi * 3 + r, met_o, t_o, s_o, (1, 2))


@pytest.mark.parametrize("mode", MODES)
def test_poisson_controlled_and_wall(mode):
    torch, engine, graphs, O = _ctx()
    so = graphs.readme()
    g = _graph(engine, so)
    rates = torch.tensor([4.0, 0.0, 9.5, 1.25], dtype=torch.float64)
    res = g.run("poisson", n_rep=4, ctrl_seed=7, ctrl_rate=rates, Ks=(1,), **_mode_kw(mode))
    for r in range(4):
        met_o, t_o, s_o = _oracle(O, so, ("poisson", 7 + r, float(rates[r])), (1,))
        _cmp_replica(res, r, met_o, t_o, s_o, (1,))
    res = g.run("wall", n_rep=1, Ks=(1, 3), **_mode_kw(mode))
    met_o, t_o, s_o = _oracle(O, so, ("wall",), (1, 3))
    _cmp_replica(res, 0, met_o, t_o, s_o, (1, 3))


@pytest.mark.parametrize("mode", MODES)
def test_max_events(mode):
    torch, engine, graphs, O = _ctx()
    so = graphs.readme()
    g = _graph(engine, so)
    res = g.run("opt", q=1.0, s=so["s"], n_rep=1, ctrl_seed=101, max_events=500, Ks=(1,),
                **_mode_kw(mode))
    met_o, t_o, s_o = _oracle(O, so, ("opt", 101), (1,), max_events=500)
    assert len(t_o) == 500
    _cmp_replica(res, 0, met_o, t_o, s_o, (1,))


@pytest.mark.parametrize("mode", MODES)
def test_c3_replicas(mode):
    torch, engine, graphs, O = _ctx()
    so = graphs.c3()
    g = _graph(engine, so)
    R = 6
    res = g.run("opt", q=so["q"], s=so["s"], n_rep=R, ctrl_seed=500, world_seed=500,
                randomize=True, Ks=(1, 10), **_mode_kw(mode))
    assert int(res.status.abs().sum().item()) == 0
    for r in range(0, R, 2):
        u = 500 + r
        met_o, t_o, s_o = _oracle(O, _world_with_seeds(so, u), ("opt", u), (1, 10))
        _cmp_replica(res, r, met_o, t_o, s_o, (1, 10))


def test_large_batch_no_overflow_and_determinism():
    torch, engine, graphs, O = _ctx()
    so = graphs.c3()
    g = _graph(engine, so)
    a = g.run("opt", q=so["q"], s=so["s"], n_rep=2048, ctrl_seed=0, world_seed=0,
              randomize=True, Ks=(1,))
    b = g.run("opt", q=so["q"], s=so["s"], n_rep=2048, ctrl_seed=0, world_seed=0,
              randomize=True, Ks=(1,), chunk=300)
    c = g.run("opt", q=so["q"], s=so["s"], n_rep=2048, ctrl_seed=0, world_seed=0,
              randomize=True, Ks=(1,), sweep_mode=2)
    d = g.run("opt", q=so["q"], s=so["s"], n_rep=2048, ctrl_seed=0, world_seed=0,
              randomize=True, Ks=(1,), sweep_mode=3)
    e = g.run("opt", q=so["q"], s=so["s"], n_rep=2048, ctrl_seed=0, world_seed=0,
              randomize=True, Ks=(1,), sweep_mode=4)
    f = g.run("opt", q=so["q"], s=so["s"], n_rep=2048, ctrl_seed=0, world_seed=0,
              randomize=True, Ks=(1,), sweep_mode=7)
    assert g.run("opt", q=so["q"], s=so["s"], n_rep=2048, Ks=(1,), plan_only=True)["variant"] == 22
    assert g.run("opt", q=so["q"], s=so["s"], n_rep=2048, Ks=(1,), sweep_mode=7, plan_only=True)["variant"] == 12
    assert torch.equal(a.metrics, f.metrics) and torch.equal(a.counts, f.counts)
    assert torch.equal(a.metrics, b.metrics) and torch.equal(a.counts, b.counts)
    # the fused bitset sweep, the sequential event-log variant, the rank-scatter sweep
    # and the legacy pre-generated-stream sweep are the same machine
    assert torch.equal(a.metrics, c.metrics) and torch.equal(a.counts, c.counts)
    assert torch.equal(a.metrics, d.metrics) and torch.equal(a.counts, d.counts)
    assert torch.equal(a.metrics, e.metrics) and torch.equal(a.counts, e.counts)
    assert torch.equal(a.status, e.status)
    assert int(a.status.sum().item()) == 0
    ev = a.n_events.double().mean().item()
    assert 4800 < ev < 6200, ev


def _tie_world():
    """Two RealData walls on the same quarter-grid times (duplicates inside each
    and across both) plus a Poisson wall: equal-time pivot rows everywhere,
    including across the sweep's 64-event tile boundaries."""
    rng = np.random.RandomState(77)
    T = np.sort(np.round(rng.uniform(0.0, 50.0, 150) * 4.0) / 4.0)
    so = dict(src_id=1, end_time=50.0, s=np.asarray([1.0, 2.0]), q=1.5, sink_ids=[10, 11, 12],
              other_sources=[("RealData", {"src_id": 2, "times": T.tolist()}),
                             ("RealData", {"src_id": 3, "times": T.tolist()}),
                             ("Poisson", {"src_id": 4, "seed": 5, "rate": 2.0})],
              edge_list=[(1, 10), (1, 11), (2, 10), (2, 11), (3, 11), (3, 12), (4, 12), (4, 10)])
    return so, T


@pytest.mark.parametrize("mode", MODES)
def test_equal_time_rows(mode):
    torch, engine, graphs, O = _ctx()
    so, T = _tie_world()
    ctimes = T[::3].copy()
    g = engine.Graph(so["src_id"], so["other_sources"], so["sink_ids"], so["edge_list"],
                     so["end_time"], ctrl_a=ctimes)
    Ks = (1, 2)
    res = g.run("times", n_rep=1, Ks=Ks, **_mode_kw(mode))
    met_o, t_o, s_o = _oracle(O, so, ("times", ctimes), Ks)
    _cmp_replica(res, 0, met_o, t_o, s_o, Ks)
    g2 = _graph(engine, so)
    for seed in (1, 2, 3):
        res = g2.run("opt", q=so["q"], s=so["s"], n_rep=1, ctrl_seed=seed, Ks=Ks, **_mode_kw(mode))
        met_o, t_o, s_o = _oracle(O, so, ("opt", seed), Ks)
        _cmp_replica(res, 0, met_o, t_o, s_o, Ks)


def test_tie_fallback_many_sources_event_log():
    """More than 64 sources with an event log runs the fast general sweep first.  Two
    Poisson2 walls with the same seed and rate post at identical times into a shared
    sink, so equal-time rows set RQ_ST_TIE and Graph.run(check=True) reruns the batch
    on the sequential sweep: the result equals sweep_mode=2 and the engine oracle."""
    torch, engine, graphs, O = _ctx()
    extra = [("Poisson", {"src_id": 100 + k, "seed": 7 + k, "rate": 0.3}) for k in range(66)]
    so = dict(src_id=1, end_time=50.0, s=np.asarray([1.0, 2.0]), q=1.5, sink_ids=[10, 11, 12],
              other_sources=[("Poisson2", {"src_id": 2, "seed": 5, "rate": 3.0}),
                             ("Poisson2", {"src_id": 3, "seed": 5, "rate": 3.0})] + extra,
              edge_list=[(1, 10), (1, 11), (2, 10), (2, 11), (3, 11), (3, 12)] +
                        [(100 + k, 10 + k % 3) for k in range(66)])
    g = _graph(engine, so)
    Ks = (1,)   # K = 1: the fast sink-bit general sweep writes event logs itself
    kw = dict(q=so["q"], s=so["s"], n_rep=2, ctrl_seed=3, Ks=Ks)
    assert g.n_streams > 64
    assert g.run("opt", event_log=True, plan_only=True, **kw)["variant"] % 10 != 1   # fast first
    fast = g.run("opt", event_log=True, check=False, **kw)
    assert int(fast.status[0].item()) & 4   # the ties were seen
    a = g.run("opt", event_log=True, **kw)
    b = g.run("opt", event_log=True, sweep_mode=2, **kw)
    assert torch.equal(a.metrics, b.metrics) and torch.equal(a.counts, b.counts)
    met_o, t_o, s_o = _oracle(O, so, ("opt", 3), Ks)
    _cmp_replica(a, 0, met_o, t_o, s_o, Ks)


def test_fast_sweep_equal_times_disjoint_sinks():
    """The tiled sweep's vectorised row placement on equal-time rows (forced with
    sweep_mode=1): two RealData walls on the same (distinct) times feeding
    disjoint sinks -- every sink is touched at most once per time, so keeping
    the last row is the reference's pivot exactly; rows tie inside and across
    64-event tiles."""
    torch, engine, graphs, O = _ctx()
    so, T = _tie_world()
    T = np.unique(T)
    so = dict(so, other_sources=[("RealData", {"src_id": 2, "times": T.tolist()}),
                                 ("RealData", {"src_id": 3, "times": T.tolist()}),
                                 ("Poisson", {"src_id": 4, "seed": 5, "rate": 2.0})],
              edge_list=[(1, 10), (1, 11), (2, 10), (3, 12), (4, 11)])
    g = _graph(engine, so)
    for seed, Ks in [(1, (1, 2)), (2, (1, 2)), (3, (1,)), (4, (1,))]:   # (1,): bitset variant
        res = g.run("opt", q=so["q"], s=so["s"], n_rep=1, ctrl_seed=seed, Ks=Ks, sweep_mode=1)
        assert int(res.status[0].item()) & 4   # the ties were seen
        met_o, t_o, s_o = _oracle(O, so, ("opt", seed), Ks)
        _cmp_replica(res, 0, met_o, t_o, s_o, Ks)


@pytest.mark.parametrize("Ks", [(1,), (1, 3)])
def test_fused_window_equal_time_blocks(Ks):
    """Tile formation when many arrivals share one time: a RealData wall with 300
    arrivals at t=5 (more than a ring, a window and a tile hold), runs of 40 at
    other times, and Poisson / Hawkes walls around them.  The fused windowed
    sweep (sweep_mode=1) must play exactly the events, rows and TIE flags of the
    legacy serial-merge sweep (sweep_mode=4) -- both keep the last of equal-time
    rows, so both differ from the reference's averaged pivot cells here.
    (sweep_mode 5 = mode 1 on the legacy kernels.)"""
    torch, engine, graphs, O = _ctx()
    T = np.sort(np.concatenate([np.full(300, 5.0), np.full(40, 7.25), np.full(40, 2.0),
                                np.linspace(0.5, 19.5, 77)]))
    so = dict(src_id=1, end_time=20.0, s=np.asarray([1.0, 2.0, 0.5]), q=0.7, sink_ids=[10, 11, 12, 13],
              other_sources=[("RealData", {"src_id": 2, "times": T.tolist()}),
                             ("Poisson", {"src_id": 3, "seed": 5, "rate": 30.0}),
                             ("Hawkes", {"src_id": 4, "seed": 9, "l_0": 5.0, "alpha": 2.0, "beta": 5.0}),
                             ("RealData", {"src_id": 5, "times": [5.0] * 9 + [7.25, 9.0]})],
              edge_list=[(1, 10), (1, 11), (1, 13), (2, 10), (2, 12), (3, 11), (4, 12), (4, 13),
                         (5, 13), (5, 10)])
    g = _graph(engine, so)
    for seed in (1, 2, 3):
        a = g.run("opt", q=so["q"], s=so["s"], n_rep=4, ctrl_seed=seed, Ks=Ks, sweep_mode=1)
        b = g.run("opt", q=so["q"], s=so["s"], n_rep=4, ctrl_seed=seed, Ks=Ks, sweep_mode=5)
        assert torch.equal(a.counts, b.counts)
        assert torch.equal(a.metrics, b.metrics)
        assert torch.equal(a.status, b.status)
        assert int(a.status[0].item()) & 4


@pytest.mark.parametrize("mode", ["fast", "legacy"])
def test_work_queue_replicas(mode):
    """Replicas past the resident wave slots come from the sweep's work queue (persistent
    grid, SweepArgs.wq): they must equal the oracle bit for bit and equal a chunked run
    whose launches all fit the resident slots (static replica per wave)."""
    torch, engine, graphs, O = _ctx()
    so = graphs.readme()
    g = _graph(engine, so)
    R = 20000
    kw = _mode_kw(mode)
    a = g.run("opt", q=so["q"], s=so["s"], n_rep=R, ctrl_seed=3000, world_seed=3000,
              randomize=True, Ks=(1, 2), **kw)
    b = g.run("opt", q=so["q"], s=so["s"], n_rep=R, ctrl_seed=3000, world_seed=3000,
              randomize=True, Ks=(1, 2), chunk=1000, **kw)
    assert int(a.status.abs().sum().item()) == 0
    assert torch.equal(a.metrics, b.metrics) and torch.equal(a.counts, b.counts)
    for r in (0, 4095, 4096, 8191, 8192, 12345, R - 1):
        u = 3000 + r
        met_o, t_o, s_o = _oracle(O, _world_with_seeds(so, u), ("opt", u), (1, 2))
        _cmp_replica(a, r, met_o, t_o, s_o, (1, 2))


def test_work_queue_c3():
    """The bench network (C3) at 1.5 launches' worth of wave slots: queue == chunked."""
    torch, engine, graphs, O = _ctx()
    so = graphs.c3()
    g = _graph(engine, so)
    R = 6000
    a = g.run("opt", q=so["q"], s=so["s"], n_rep=R, ctrl_seed=77, world_seed=77, randomize=True, Ks=(1,))
    b = g.run("opt", q=so["q"], s=so["s"], n_rep=R, ctrl_seed=77, world_seed=77, randomize=True, Ks=(1,),
              chunk=500)
    assert int(a.status.abs().sum().item()) == 0
    assert torch.equal(a.metrics, b.metrics) and torch.equal(a.counts, b.counts)
    for r in (4500, R - 1):
        u = 77 + r
        met_o, t_o, s_o = _oracle(O, _world_with_seeds(so, u), ("opt", u), (1,))
        _cmp_replica(a, r, met_o, t_o, s_o, (1,))


@pytest.mark.parametrize("wl", ["c3", "g120"])
def test_capacity_overflow_rerun(wl, monkeypatch):
    """The merged sequence and the pivot rows are sized from the SUM of a replica's wall
    events (mean + 8 sigma); a replica past them is flagged (RQ_ST_STREAM_OVERFLOW /
    RQ_ST_ROWS_OVERFLOW) and Graph.run(check=True) reruns the batch with doubled
    capacities.  Forced here by undersized capacities (RQ_CAP_SQUEEZE): the flagged first
    pass leaves no trace -- the result equals the normal run bit for bit, and the oracle."""
    torch, engine, graphs, O = _ctx()
    from redqueen_amd import _lib as L
    so = getattr(graphs, wl)()
    g = _graph(engine, so)
    kw = dict(q=so["q"], s=so["s"], n_rep=64, ctrl_seed=9, world_seed=9, randomize=True, Ks=(1,))
    ref = g.run("opt", **kw)
    monkeypatch.setenv("RQ_CAP_SQUEEZE", "0.45")
    raw = g.run("opt", check=False, **kw)
    assert int(((raw.status & (L.ST_ROWS_OVERFLOW | L.ST_STREAM_OVERFLOW)) != 0).sum().item()) > 0
    got = g.run("opt", **kw)
    assert int(got.status.max().item()) == 0
    assert torch.equal(got.metrics, ref.metrics) and torch.equal(got.counts, ref.counts)
    met_o, t_o, s_o = _oracle(O, _world_with_seeds(so, 9 + 5), ("opt", 9 + 5), (1,))
    _cmp_replica(got, 5, met_o, t_o, s_o, (1,))
