"""The reference's plugin point for broadcasters: SimOpts.registerSource
(opt_model.py:768-771) with a STATIC class implementing initialize() /
get_all_times() (:336-338, :391-394).  The host runs the plugin's own code (once
per run, or once per replica with the seeds randomize_other_sources gives it,
:795-804) and the engine plays the times as RealData streams -- per-replica ones
through rq_batch_desc.rd_* (ABI v3).  Expected values: tests/golden/plugin.npz,
written by gen_golden.py with the same class over the reference's Broadcaster.
A DYNAMIC plugin's own times come from its get_next_event_time on the host: a
self-driven one (its schedule moves only on its own events) from its own schedule,
verified against the run's event sequence; a reactive one (its schedule moves on other
sources' events) from the run's other events, rerun until the run reproduces them
(opt_model.reactive_plugin_times, Graph._run_reactive).  Expected values:
tests/golden/dynplugin.npz, dist_knock.npz."""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
KS = [1, 2, 5, 10]
COLS = ["event_id", "time_delta", "src_id", "t", "sink_id"]
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))


def _setup():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from realdata_worlds import BurstyMixin, plugin_world
    from redqueen_amd import engine
    from redqueen_amd.opt_model import Broadcaster, SimOpts

    class Bursty(BurstyMixin, Broadcaster):
        pass
    SimOpts.registerSource("Bursty", Bursty)
    return engine, SimOpts, Bursty, plugin_world()


def test_registered_static_broadcaster_single_run(golden):
    engine, SimOpts, Bursty, (w, ctrl, us) = _setup()
    from redqueen_amd import utils as U
    d = golden("plugin.npz")
    so = SimOpts(**w)
    m = so.create_manager_with_times(np.asarray(ctrl))
    m.run_dynamic()
    df = m.state.get_dataframe()
    for c in COLS:
        assert np.array_equal(df[c].values, d["base_" + c]), c
    got = U.replay_metrics(df, so.src_id, so.end_time, KS)
    assert np.array_equal(np.asarray(got["top_k"] + [got["avg_rank"], got["r_2"]]), d["base_met"])


def test_registered_static_broadcaster_randomized_batch(golden):
    """16 replicas in ONE batch, each with its own plugin times (per-replica RealData
    streams): every replica's metrics equal the reference's run of
    randomize_other_sources(u)."""
    engine, SimOpts, Bursty, (w, ctrl, us) = _setup()
    d = golden("plugin.npz")
    g = engine.Graph(w["src_id"], w["other_sources"], w["sink_ids"], w["edge_list"],
                     w["end_time"], ctrl_a=ctrl)
    assert [p[3] for p in g.plugins] == [2, 6]
    res = g.run("times", n_rep=len(us), world_seed=0, randomize=True, Ks=KS)
    m = res.metrics.cpu().numpy()
    c = res.counts.cpu().numpy()
    assert np.array_equal(m, d["rand_met"]), m - d["rand_met"]
    assert np.array_equal(c[:, 0], d["rand_cnt"][:, 0]) and np.array_equal(c[:, 1], d["rand_cnt"][:, 1])
    assert np.array_equal(c[:, 2], d["rand_cnt"][:, 2])
    # a shard of the same batch (replicas 5..11) sees the same per-replica times
    r2 = g.run("times", n_rep=len(us), world_seed=0, randomize=True, Ks=KS, replica0=5, n_local=7)
    assert np.array_equal(r2.metrics.cpu().numpy(), d["rand_met"][5:12])


def _dyn_setup():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from realdata_worlds import BurstyMixin, KnockedOffMixin, RenewalMixin, dyn_plugin_world
    from redqueen_amd import engine
    from redqueen_amd.opt_model import Broadcaster, SimOpts

    class Bursty(BurstyMixin, Broadcaster):
        pass

    class Renewal(RenewalMixin, Broadcaster):
        pass

    class KnockedOff(KnockedOffMixin, Broadcaster):
        pass
    SimOpts.registerSource("Bursty", Bursty)
    SimOpts.registerSource("Renewal", Renewal)
    SimOpts.registerSource("KnockedOff", KnockedOff)
    return engine, SimOpts, dyn_plugin_world()


def test_self_driven_dynamic_plugin_single_run(golden):
    """A registered DYNAMIC broadcaster whose schedule moves only on its own events
    (Renewal: gamma gaps through its own RandomState, None on the others'): the host
    plays its own events through get_next_event_time, the GPU plays the times, and the
    run's whole event sequence is fed back to a fresh copy of it to verify it is
    self-driven.  The df equals the reference's run_dynamic df bit for bit."""
    engine, SimOpts, (w, ctrl, us) = _dyn_setup()
    from redqueen_amd import utils as U
    d = golden("dynplugin.npz")
    so = SimOpts(**w)
    m = so.create_manager_with_times(np.asarray(ctrl))
    m.run_dynamic()
    df = m.state.get_dataframe()
    for c in COLS:
        assert np.array_equal(df[c].values, d["base_" + c]), c
    got = U.replay_metrics(df, so.src_id, so.end_time, KS)
    assert np.array_equal(np.asarray(got["top_k"] + [got["avg_rank"], got["r_2"]]), d["base_met"])


def test_self_driven_dynamic_plugin_randomized_batch(golden):
    """16 replicas in one batch with randomize_other_sources seeds: every replica's
    metrics and counts equal the reference's run (the batch's first replica is checked
    to be self-driven through its own event log)."""
    engine, SimOpts, (w, ctrl, us) = _dyn_setup()
    d = golden("dynplugin.npz")
    g = engine.Graph(w["src_id"], w["other_sources"], w["sink_ids"], w["edge_list"],
                     w["end_time"], ctrl_a=ctrl)
    assert [(p[3], p[4]) for p in g.plugins] == [(2, True), (6, False)]
    res = g.run("times", n_rep=len(us), world_seed=0, randomize=True, Ks=KS)
    m = res.metrics.cpu().numpy()
    c = res.counts.cpu().numpy()
    assert np.array_equal(m, d["rand_met"]), m - d["rand_met"]
    assert np.array_equal(c[:, :3], d["rand_cnt"])


def _knock_world(w):
    return dict(w, other_sources=[("KnockedOff", {"src_id": 2, "seed": 21, "rate": 1.0})] +
                w["other_sources"][1:])


def test_reactive_dynamic_plugin_single_run(golden):
    """A dynamic plugin whose schedule reacts to other sources' events (KnockedOff, the
    reference's SmartPoisson idea): the manager's run_dynamic plays it to the fixed point
    and its df equals the reference's run_dynamic df bit for bit."""
    engine, SimOpts, (w, ctrl, us) = _dyn_setup()
    from redqueen_amd import utils as U
    d = golden("dynplugin.npz")
    so = SimOpts(**_knock_world(w))
    m = so.create_manager_with_times(np.asarray(ctrl))
    m.run_dynamic()
    df = m.state.get_dataframe()
    for c in COLS:
        assert np.array_equal(df[c].values, d["knock_" + c]), c
    got = U.replay_metrics(df, so.src_id, so.end_time, KS)
    assert np.array_equal(np.asarray(got["top_k"] + [got["avg_rank"], got["r_2"]]), d["knock_met"])


def test_reactive_dynamic_plugin_randomized_batch(golden):
    """16 replicas in one batch with randomize_other_sources seeds: the probe finds the
    plugin reactive, the batch is replayed to the fixed point, and every replica's
    metrics and counts equal the reference's run."""
    engine, SimOpts, (w, ctrl, us) = _dyn_setup()
    d = golden("dynplugin.npz")
    w2 = _knock_world(w)
    g = engine.Graph(w2["src_id"], w2["other_sources"], w2["sink_ids"], w2["edge_list"],
                     w2["end_time"], ctrl_a=ctrl)
    res = g.run("times", n_rep=len(us), world_seed=0, randomize=True, Ks=KS)
    assert g.reactive_reruns >= 1
    m = res.metrics.cpu().numpy()
    c = res.counts.cpu().numpy()
    assert np.array_equal(m, d["knock_rand_met"]), m - d["knock_rand_met"]
    assert np.array_equal(c[:, :3], d["knock_rand_cnt"])


def _fixed_point(g, res, w, cls, kws, me=None, n=None):
    """Every replica's (the first n) plugin times reproduce themselves from its run's
    other events."""
    from redqueen_amd.opt_model import reactive_plugin_times
    for k in range(len(res.global_ids) if n is None else n):
        t, src = res.events(k)
        got = reactive_plugin_times(cls(**kws(int(res.global_ids[k]))), 0.0, w["sink_ids"],
                                    w["edge_list"], w["end_time"], t, src, max_events=me)
        assert np.array_equal(got, t[src == 2]), k


def test_reactive_plugin_beside_redqueen(golden):
    """KnockedOff beside the RedQueen broadcaster, whose posts react to the plugin's
    events in turn: the batch reaches the fixed point (every replica's plugin times come
    back unchanged from its own run), and the ensemble matches the reference's own
    ensemble of the same world (dist_knock.npz) in mean, spread and shape."""
    import torch
    import ensemble as E
    engine, SimOpts, (w, ctrl, us) = _dyn_setup()
    from realdata_worlds import KnockedOffMixin
    from redqueen_amd.opt_model import Broadcaster

    class KnockedOff(KnockedOffMixin, Broadcaster):
        pass
    d = golden("dist_knock.npz")
    assert d["data"].shape[0] >= 10000
    w2 = _knock_world(w)
    g = engine.Graph(w2["src_id"], w2["other_sources"], w2["sink_ids"], w2["edge_list"],
                     w2["end_time"])
    stride = int(d["seed_stride"][0])
    R = 4000
    u = torch.arange(R, dtype=torch.int64) * stride + 7
    res = g.run("opt", q=w2["q"], s=w2["s"], n_rep=R, ctrl_seed=u, world_seed=u, randomize=True,
                Ks=KS, event_log=True)
    assert g.reactive_reruns >= 1
    print("reruns to the fixed point:", g.reactive_reruns)
    assert int((res.status & 3).max().item()) == 0
    _fixed_point(g, res, w2, KnockedOff,
                 lambda i: {"src_id": 2, "seed": (i * stride + 7) & 0xFFFFFFFF, "rate": 1.0}, n=256)
    cols = [str(c) for c in d["cols"]]
    ref = {c: d["data"][:, i] for i, c in enumerate(cols)}
    c = res.counts.double().cpu().numpy()
    m = res.metrics.cpu().numpy()
    eng = {"posts": c[:, 0], "world": c[:, 1], "events": c[:, 2], "avg": m[:, len(KS)],
           "r2": m[:, len(KS) + 1]}
    for i, k in enumerate(KS):
        eng["top%d" % k] = m[:, i]
    E.compare("gpu_knock_opt", eng, ref, z_bound=2.576)


def _rarely_reactive():
    """Renewal (self-driven) except in the replicas whose seed is listed: there, like
    KnockedOff, another source's event moves its schedule."""
    from realdata_worlds import RenewalMixin
    from redqueen_amd.opt_model import Broadcaster

    class RarelyReactive(RenewalMixin, Broadcaster):
        REACT = set()

        def __init__(self, src_id, seed, scale=0.6):
            super().__init__(src_id, seed, scale)
            self._react = seed in self.REACT

        def get_next_interval(self, event):
            if self._react and event is not None and event.src_id != self.src_id:
                return self.get_current_time(event) - self.last_self_event_time + 0.01
            return super().get_next_interval(event)
    return RarelyReactive


@pytest.mark.parametrize("n_rep,react", [(16, {5}), (640, set(range(7, 640, 10)))])
def test_dynamic_plugin_verified_beyond_replica_zero(n_rep, react):
    """A dynamic plugin that reacts to other sources only in a few replicas, none of them
    replica 0: every replica of a batch of <= 64 is verified, a seeded
    sample of 64 above that, so the batch is found reactive and replayed to the fixed
    point instead of returning those replicas played as if self-driven: every replica's
    plugin times come back unchanged from its own event log, and the self-driven
    replicas equal a shard of them run alone."""
    engine, SimOpts, (w, ctrl, us) = _dyn_setup()
    RR = _rarely_reactive()
    RR.REACT = set(react)
    SimOpts.registerSource("RarelyReactive", RR)
    w2 = dict(w, other_sources=[("RarelyReactive", {"src_id": 2, "seed": 21, "scale": 0.6})] +
              w["other_sources"][1:])
    g = engine.Graph(w2["src_id"], w2["other_sources"], w2["sink_ids"], w2["edge_list"],
                     w2["end_time"], ctrl_a=ctrl)
    assert 0 not in react
    res = g.run("times", n_rep=n_rep, world_seed=0, randomize=True, Ks=KS, event_log=True)
    assert g.reactive_reruns >= 1
    assert int((res.status & 3).max().item()) == 0   # no overflow (ties are exact here: RealData)
    _fixed_point(g, res, w2, RR, lambda i: {"src_id": 2, "seed": i, "scale": 0.6})
    # replicas 0..4 (seeds 0..4: randomize_other_sources gives source idx 0 seed u) are
    # self-driven: that shard runs without the reactive path and equals the batch's rows
    g2 = engine.Graph(w2["src_id"], w2["other_sources"], w2["sink_ids"], w2["edge_list"],
                      w2["end_time"], ctrl_a=ctrl)
    r5 = g2.run("times", n_rep=n_rep, world_seed=0, randomize=True, Ks=KS, replica0=0, n_local=5)
    assert not hasattr(g2, "reactive_reruns")
    assert np.array_equal(r5.metrics.cpu().numpy(), res.metrics.cpu().numpy()[:5])


def _grid_setup():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from realdata_worlds import GridBurstyMixin, GridKnockMixin, grid_tie_world
    from redqueen_amd import engine
    from redqueen_amd.opt_model import Broadcaster, SimOpts

    class GridBursty(GridBurstyMixin, Broadcaster):
        pass

    class GridKnock(GridKnockMixin, Broadcaster):
        pass
    SimOpts.registerSource("GridBursty", GridBursty)
    SimOpts.registerSource("GridKnock", GridKnock)
    return engine, SimOpts, grid_tie_world()


def test_reactive_plugin_equal_time_order(golden):
    """a reactive dynamic plugin whose posts land EXACTLY on static sources'
    times (every source on a binary grid; tests/golden/gridtie.npz, 2-12 such ties per
    world).  run_dynamic plays a static time only when it is strictly earlier than the
    dynamic sources' next event (opt_model.py:289-290), so at an equal time the plugin
    (src 7, the largest id) plays BEFORE the RealData controlled source (4) and the static
    plugin (6): the host fixed point (reactive_plugin_times, static_ids), the stream
    order of the graph (dynamic sources first, RQ_SRCF_DYNAMIC) and the controller flags
    all follow it.  The manager's df and the 32-replica randomized batch equal the
    reference's bit for bit."""
    engine, SimOpts, (w, ctrl, us) = _grid_setup()
    from redqueen_amd import utils as U
    d = golden("gridtie.npz")
    assert (d["rand_ties"] > 0).all()
    so = SimOpts(**w)
    m = so.create_manager_with_times(np.asarray(ctrl))
    m.run_dynamic()
    df = m.state.get_dataframe()
    for c in COLS:
        assert np.array_equal(df[c].values, d["base_" + c]), c
    got = U.replay_metrics(df, so.src_id, so.end_time, KS)
    assert np.array_equal(np.asarray(got["top_k"] + [got["avg_rank"], got["r_2"]]), d["base_met"])
    g = engine.Graph(w["src_id"], w["other_sources"], w["sink_ids"], w["edge_list"],
                     w["end_time"], ctrl_a=ctrl)
    assert g.static_src_ids == {6}
    # the stream order: the dynamic plugin's stream before every static one
    assert list(g.stream_src_ids) == [7, 4, 6]
    res = g.run("times", n_rep=len(us), world_seed=0, randomize=True, Ks=KS)
    mm = res.metrics.cpu().numpy()
    c = res.counts.cpu().numpy()
    assert np.array_equal(mm, d["rand_met"]), mm - d["rand_met"]
    assert np.array_equal(c[:, :3], d["rand_cnt"])
