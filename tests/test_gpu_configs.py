"""The BASELINE configs beyond the bench line, as GPU parity cases.

C5 (10k followers, 500 bursty Hawkes sources): bit-exact vs the engine oracle on
a shortened horizon (T=100, ~5e4 events per replica: the oracle finishes in
seconds) and, at the full T=1000 (~5e5 events per replica), two replicas bit-exact
against the C oracle's batch path plus size-independent checks: no overflow,
batch == sharded sub-batches, event counts at the Hawkes mean.  C4 (README graph x 64 q x 4 s): the full grid at 64 replicas per point,
sharded as 8 ranks would run it, equal to the unsharded grid; grid means move with
q as RedQueen's budget law says (posts fall as q grows)."""
import numpy as np
import pytest

from tests.test_gpu_engine import _cmp_replica, _ctx, _graph, _world_with_seeds

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("Ks", [(1, 5), (1,)])
def test_c5_short_horizon_bit_exact(Ks):
    """Ks=(1,) runs the K=1 per-wave LDS sink-bit sweep (plan variant 3), (1, 5) the
    per-sink int16 ranks."""
    torch, engine, graphs, O = _ctx()
    so = dict(graphs.c5(), end_time=100.0)
    g = _graph(engine, so)
    R = 8
    kw = dict(q=so["q"], s=so["s"], n_rep=R, ctrl_seed=40, world_seed=40, randomize=True, Ks=Ks)
    assert g.run("opt", plan_only=True, **kw)["variant"] == (3 if Ks == (1,) else 0)
    # the fast sweep writes the event log itself: events compared too
    res = g.run("opt", event_log=True, **kw)
    assert g.run("opt", event_log=True, plan_only=True, **kw)["variant"] != 1
    assert int(res.status.max().item()) == 0
    for r in (0, 5):
        u = 40 + r
        sc = O.Scenario(_world_with_seeds(so, u), ("opt", u))
        met, (t, dt, s) = O.engine_metrics(sc, Ks)
        _cmp_replica(res, r, met, t, s, Ks)


def test_sink_bits_sweep_many_posts():
    """The K=1 sink-bit sweep (> 64 sources, > 2048 sinks) on a post-heavy graph
    (q = 1e3: the post path ORs the follower set into the bits every few events):
    equal to the per-sink-rank sweep (sweep_mode 3) on every replica and bit-exact
    against the engine oracle."""
    torch, engine, graphs, O = _ctx()
    so = graphs.followers_graph(num_followers=3000, num_sources=96, degree=3, end_time=20.0)
    so["q"] = 1e3
    g = _graph(engine, so)
    kw = dict(q=so["q"], s=so["s"], n_rep=24, ctrl_seed=3, world_seed=3, randomize=True, Ks=(1,))
    assert g.run("opt", plan_only=True, **kw)["variant"] == 3
    res = g.run("opt", event_log=True, **kw)
    ref = g.run("opt", sweep_mode=3, **kw)
    assert int(res.status.max().item()) == 0
    assert torch.equal(res.metrics, ref.metrics) and torch.equal(res.counts, ref.counts)
    assert float(res.counts[:, 0].double().mean().item()) > 50   # posts: the OR path ran
    for r in (0, 11):
        u = 3 + r
        sc = O.Scenario(_world_with_seeds(so, u), ("opt", u))
        met, (t, dt, s) = O.engine_metrics(sc, (1,))
        _cmp_replica(res, r, met, t, s, (1,))


def test_c5_full_horizon_properties():
    torch, engine, graphs, O = _ctx()
    from redqueen_amd import dist
    so = graphs.c5()
    g = _graph(engine, so)
    R = 96
    kw = dict(q=so["q"], s=so["s"], ctrl_seed=9, world_seed=9, randomize=True, Ks=(1,))
    full = g.run("opt", n_rep=R, **kw)
    assert int(full.status.max().item()) == 0
    parts = []
    for rank in range(4):
        a, b = dist.shard(R, 4, rank)
        parts.append(g.run("opt", n_rep=R, replica0=a, n_local=b - a, **kw).metrics)
    assert torch.equal(torch.cat(parts), full.metrics)
    ev = full.counts[:, 1].double().mean().item()   # world events: 500 x l0 T / (1 - a/b)
    assert abs(ev - 500 * 0.5 * 1000 / 0.5) < 0.02 * 500000, ev
    top = full.metrics[:, 0].cpu().numpy()
    assert np.all((top >= 0) & (top <= 1000.0))


def test_c5_full_horizon_replicas_bit_exact():
    """Full C5 (T=1000, ~5e5 events and ~5e7 sink updates per replica) through the
    bench's own kernel (plan variant 3, K=1 sink bits): replicas 0 and 3 equal the
    C oracle bit for bit -- metrics and counts from rqo_engine_batch, and the whole
    event sequence (t, stream) from rqo_engine_run against the event-log run."""
    torch, engine, graphs, O = _ctx()
    so = graphs.c5()
    g = _graph(engine, so)
    kw = dict(q=so["q"], s=so["s"], n_rep=4, ctrl_seed=11, world_seed=11, randomize=True, Ks=(1,))
    assert g.run("opt", plan_only=True, **kw)["variant"] == 3
    plain = g.run("opt", **kw)
    logd = g.run("opt", event_log=True, **kw)
    assert int(plain.status.max().item()) == 0 and int(logd.status.max().item()) == 0
    assert torch.equal(plain.metrics, logd.metrics) and torch.equal(plain.counts, logd.counts)
    for r in (0, 3):
        u = 11 + r
        out, cnt, _ = O.engine_batch(O.Scenario(so, ("opt", 0)), 1, u, True, (1,), 1)
        m = plain.metrics[r].cpu().numpy()
        assert np.array_equal(m, out[0]), (r, m, out[0])
        c = plain.counts[r].cpu().numpy()
        assert (c[0], c[1], c[2]) == tuple(int(x) for x in cnt[0]), (r, c, cnt[0])
        assert c[2] > 400000
        t_o, _, s_o = O.engine_run(O.Scenario(_world_with_seeds(so, u), ("opt", u)))
        t, s = logd.events(r)
        assert np.array_equal(s, s_o) and np.array_equal(t, t_o), r


def test_c4_full_config():
    """C4 at its full size: 64 q x 4 s grid points x 1000 replicas (256k replicas, chunked
    by the engine), run whole and as the 8 grid-balanced shards 8 GPUs would run; every
    per-replica row and the fixed-order grid means agree; one replica per s column
    equals the oracle."""
    torch, engine, graphs, O = _ctx()
    from redqueen_amd import dist
    so = graphs.readme()
    g = _graph(engine, so)
    grid = graphs.c4_grid()
    qs = np.asarray([q for q, _ in grid])
    sm = np.asarray([[s1, s2] for _, (s1, s2) in grid])
    n_rep = 1000
    kw = dict(q=qs, s=sm, ctrl_seed=0, world_seed=0, randomize=True, Ks=(1,), seed_mod=n_rep)
    full = g.run("opt", n_rep=n_rep, **kw)
    assert full.metrics.shape[0] == len(grid) * n_rep == 256000
    assert int(full.status.max().item()) == 0
    # the 8 shards dist.run_sharded gives 8 GPUs: the same replica window of every grid
    # point (rq_batch_desc.rep_lo / rep_cnt), reassembled in global order
    parts, ev = [], []
    for rank in range(8):
        lo, hi = dist.grid_shard(n_rep, 8, rank)
        r = g.run("opt", n_rep=n_rep, rep_lo=lo, rep_cnt=hi - lo, **kw)
        assert torch.equal(r.metrics.reshape(len(grid), hi - lo, -1),
                           full.metrics.reshape(len(grid), n_rep, -1)[:, lo:hi])
        assert np.array_equal(r.global_ids, (np.arange(len(grid))[:, None] * n_rep +
                                             np.arange(lo, hi)[None, :]).ravel())
        parts.append(r.metrics.reshape(len(grid), hi - lo, -1))
        ev.append(int(r.counts[:, 2].sum().item()))
    allm = torch.cat(parts, 1).reshape(len(grid) * n_rep, -1)
    assert torch.equal(allm, full.metrics)
    # balanced by grid point: every shard sees every q (contiguous cuts of the flattened
    # space gave max/mean 1.16 in events)
    assert max(ev) / (sum(ev) / 8) <= 1.02, ev
    assert torch.equal(dist.grid_means(allm, len(grid), n_rep), dist.grid_means(full.metrics, len(grid), n_rep))
    posts = full.counts[:, 0].double().reshape(len(grid), n_rep).mean(1).cpu().numpy()
    for si in range(4):
        p = posts[si * 64:(si + 1) * 64]
        assert p[0] > p[-1] and np.all(np.diff(p) <= 0.02 * p[0] + 2.0)
    for gi, r in ((5, 999), (64 + 40, 123), (128 + 63, 0), (192 + 17, 500)):
        dd = dict(so, q=float(qs[gi]), s=sm[gi])
        (top, avg, r2, cnt), _ = O.engine_metrics(O.Scenario(_world_with_seeds(dd, r), ("opt", r)), (1,))
        row = full.metrics[gi * n_rep + r].cpu().numpy()
        assert row[0] == top[0] and row[1] == avg and row[2] == r2


def test_c4_grid_sharded():
    torch, engine, graphs, O = _ctx()
    from redqueen_amd import dist
    so = graphs.readme()
    g = _graph(engine, so)
    grid = graphs.c4_grid()
    qs = np.asarray([q for q, _ in grid])
    sm = np.asarray([[s1, s2] for _, (s1, s2) in grid])
    n_rep = 64
    kw = dict(q=qs, s=sm, ctrl_seed=0, world_seed=0, randomize=True, Ks=(1,), seed_mod=n_rep)
    full = g.run("opt", n_rep=n_rep, **kw)
    assert int(full.status.max().item()) == 0
    m8 = []
    for rank in range(8):
        a, b = dist.shard(len(grid) * n_rep, 8, rank)
        m8.append(g.run("opt", n_rep=n_rep, replica0=a, n_local=b - a, **kw).metrics)
    assert torch.equal(torch.cat(m8), full.metrics)
    posts = full.counts[:, 0].double().reshape(len(grid), n_rep).mean(1).cpu().numpy()
    for si in range(4):
        p = posts[si * 64:(si + 1) * 64]
        assert p[0] > p[-1] and np.all(np.diff(p) <= 0.05 * p[0] + 5.0)
    # a replica of the grid == the oracle at its (q, s, seed)
    for gi in (0, 64 * 1 + 17, 64 * 3 + 63):
        u = 0   # seed_mod = n_rep: replica 0 of every grid point runs seed 0
        dd = dict(so, q=float(qs[gi]), s=sm[gi])
        (top, avg, r2, cnt), _ = O.engine_metrics(O.Scenario(_world_with_seeds(dd, u), ("opt", u)), (1,))
        row = full.metrics[gi * n_rep].cpu().numpy()
        assert row[0] == top[0] and row[1] == avg and row[2] == r2


def test_c5_workspace_within_free_memory():
    """The workspace is planned against the device memory this process can get
    (rq_batch_desc.ws_budget = 0.9 x (free + torch's cached blocks + the graph's own
    workspace)), not a fixed 200 GiB: with all but 6 GiB of the device held
    through torch, a C5 batch runs in smaller pipelined chunks inside what is left and
    gives the unconstrained batch's bits."""
    torch, engine, graphs, O = _ctx()
    so = graphs.c5()
    g = _graph(engine, so)
    kw = dict(q=so["q"], s=so["s"], n_rep=1024, ctrl_seed=21, world_seed=21, randomize=True,
              Ks=(1,))
    free_plan = g.run("opt", plan_only=True, **kw)
    ref = g.run("opt", **kw)
    assert int(ref.status.max().item()) == 0
    ref_m, ref_c = ref.metrics.clone(), ref.counts.clone()
    big = g.workspace_bytes()
    assert big > 12 * 2 ** 30, big   # ~20 MB per replica in flight
    del ref
    g.release_workspaces()
    torch.cuda.empty_cache()
    free, _ = torch.cuda.mem_get_info()
    hog = torch.empty(free - 6 * 2 ** 30, dtype=torch.uint8, device="cuda")
    try:
        plan = g.run("opt", plan_only=True, **kw)
        assert plan["chunk"] < free_plan["chunk"], (plan, free_plan)
        res = g.run("opt", **kw)
        assert g.workspace_bytes() <= 6 * 2 ** 30
        assert torch.equal(res.metrics, ref_m) and torch.equal(res.counts, ref_c)
    finally:
        del hog
        g.release_workspaces()
        torch.cuda.empty_cache()
