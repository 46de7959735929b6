"""OptPWSignificance on the GPU (controller of every sweep variant) against the CPU
engine oracle bit for bit, the facade's create_manager_with_significance, the
batched grid, and the reference's 8k-replica ensemble (99% CI)."""
import numpy as np
import pytest

import ensemble as E
from tests.test_gpu_engine import MODES, _cmp_replica, _ctx, _graph, _mode_kw, _world_with_seeds
from tests.test_significance_cpu import KAT_BASE, KS

pytestmark = pytest.mark.gpu


def _sig(S=24, F=2):
    k = np.arange(S)
    return np.stack([0.2 + np.sin(np.pi * k / S + f) ** 2 for f in range(F)])


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("seed", [1, 41])
def test_kat_graph_bit_exact(seed, mode):
    torch, engine, graphs, O = _ctx()
    so = dict(KAT_BASE, s=[1.0, 1.0])
    g = _graph(engine, so)
    sig = _sig()
    Ks = (1, 2, 5)
    res = g.run("sig", q=1.0, s_pw=sig, period=10.0, n_rep=1, ctrl_seed=seed, Ks=Ks,
                **_mode_kw(mode))
    sc = O.Scenario(so, ("sig", seed, sig, 10.0))
    met, (t, dt, s) = O.engine_metrics(sc, Ks)
    _cmp_replica(res, 0, met, t, s, Ks)


@pytest.mark.parametrize("mode", MODES)
def test_c3_world_randomized_bit_exact(mode):
    """1000-follower network: per-(stream, segment) intensity tables, 50 sources."""
    torch, engine, graphs, O = _ctx()
    so = graphs.c3()
    g = _graph(engine, so)
    S = 7
    rs = np.random.RandomState(3)
    sig = rs.uniform(0.0, 2.0, (g.n_followers, S)) * (rs.uniform(size=(g.n_followers, 1)) < 0.8)
    R = 16
    res = g.run("sig", q=so["q"], s_pw=sig, period=13.0, n_rep=R, ctrl_seed=500, world_seed=500,
                randomize=True, Ks=(1,), **_mode_kw(mode))
    for r in range(0, R, 5):
        u = 500 + r
        sc = O.Scenario(_world_with_seeds(so, u), ("sig", u, sig, 13.0))
        met, (t, dt, s) = O.engine_metrics(sc, (1,))
        _cmp_replica(res, r, met, t, s, (1,))


def test_facade_manager_and_grid():
    torch, engine, graphs, O = _ctx()
    from redqueen_amd import batch
    from redqueen_amd import utils as U
    from redqueen_amd.opt_model import SimOpts
    so = SimOpts(s=np.asarray([1.0, 1.0]), **KAT_BASE)
    m = so.create_manager_with_significance(1, time_period=10.0, num_segments=24)
    m.run_dynamic()
    df = m.state.get_dataframe()
    sc = O.Scenario(so.get_dict(), ("sig", 1, np.ones((2, 24)), 10.0))
    met, (t, dt, s) = O.engine_metrics(sc, (1,))
    assert U.num_tweets_of(df, sim_opts=so) == np.sum(s == 1)
    assert U.time_in_top_k(df, K=1, sim_opts=so) == met[0][0]
    with pytest.raises(AssertionError):
        so.create_manager_with_significance(1, time_period=10.0, significance=np.ones((3, 4)))
    # the grid: seeds x q in one launch == the oracle replica by replica
    sig = _sig()
    out = batch.run_significance(so, sig, 10.0, seeds=range(20), qs=[0.5, 2.0], Ks=(1,))
    assert len(out) == 40 and (out.status == 0).all()
    for i in (0, 7, 25, 39):
        u, q = int(out.seed[i]), float(out.q[i])
        sc = O.Scenario(_world_with_seeds(so.update({"q": q}).get_dict(), u), ("sig", u, sig, 10.0))
        (top, avg, r2, cnt), _ = O.engine_metrics(sc, (1,))
        assert out.top_1[i] == top[0] and out.avg_rank[i] == avg and out.num_events[i] == cnt[0]
    # capacity iteration: one batch over seeds 1000..1024 == the oracle
    so2 = so.update({"s": sig})
    caps = U.calc_significance_capacity_iter(so2, 0.7, 10.0)
    sc = O.Scenario(so2.update({"q": 0.7}).get_dict(), ("sig", 0, sig, 10.0))
    _, cnt, _ = O.engine_batch(sc, 25, 1000, False, (1,), 4)
    assert np.array_equal(caps, cnt[:, 0].astype(float))


def test_ensemble_vs_reference(golden):
    torch, engine, graphs, O = _ctx()
    from redqueen_amd import batch
    from redqueen_amd.opt_model import SimOpts
    d = golden("dist_sig.npz")
    cols = [str(c) for c in d["cols"]]
    ref = {c: d["data"][:, i] for i, c in enumerate(cols)}
    n = d["data"].shape[0]
    so = SimOpts(s=np.asarray([1.0, 1.0]), **KAT_BASE)
    out = batch.run_significance(so, d["sig"], 10.0, seeds=range(n), Ks=KS)
    assert (out.status == 0).all()
    eng = {"posts": out.num_events.values, "world": out.world_events.values,
           "events": out.events.values, "avg": out.avg_rank.values, "r2": out.r_2.values}
    for k in KS:
        eng["top%d" % k] = out["top_%d" % k].values
    # replica r: world randomize_other_sources(r), seeds r and r + 99 (clusters r mod 99)
    ind = E.independent_rows(n, 2)
    E.compare("gpu_sig", eng, ref, clusters=99, indep_eng=ind, indep_ref=ind, z_bound=2.576)


def _err_worlds():
    """The worlds of tests/golden/errors.npz (gen_golden.gen_errors), as plain data."""
    base = dict(src_id=1, end_time=20.0, q=1.0, s=np.asarray([1.0, 1.0]), sink_ids=[5001, 5002],
                other_sources=[("Poisson2", {"src_id": 1000, "seed": 42, "rate": 10.0}),
                               ("Poisson2", {"src_id": 1001, "seed": 43, "rate": 10.0})])
    full = [(1, 5001), (1, 5002), (1000, 5001), (1001, 5002)]
    return {"edgeless": (dict(base, edge_list=full[:3]), None),
            "zerosig": (dict(base, edge_list=full), np.asarray([[1.0, 2.0, 1.0, 0.5], [0.0, 0.0, 0.0, 0.0]])),
            "ok": (dict(base, edge_list=full), np.asarray([[1.0, 2.0, 1.0, 0.5], [0.0, 1.0, 0.0, 0.0]]))}


def test_unreached_event_raises_like_reference(golden):
    """An event whose source reaches no follower with positive significance: the
    reference raises (take_one_sample's int(nan), opt_model.py:557-566) -- so does the
    facade, for a manager and for a batch; a world without one runs."""
    torch, engine, graphs, O = _ctx()
    from redqueen_amd import batch
    from redqueen_amd.opt_model import SimOpts
    g = golden("errors.npz")
    for name, (w, sig) in _err_worlds().items():
        ref = str(g["sig_%s_err" % name][0])
        so = SimOpts(**w)
        m = so.create_manager_with_significance(3, time_period=10.0, significance=sig,
                                                num_segments=None if sig is not None else 4)
        sig_b = sig if sig is not None else np.ones((2, 4))
        if ref == "none":
            m.run_dynamic()
            assert m.state.get_num_events() > 0
            batch.run_significance(so, sig_b, 10.0, seeds=range(4))
        else:
            assert ref == "ValueError"
            with pytest.raises(ValueError):
                m.run_dynamic()
            with pytest.raises(ValueError):
                batch.run_significance(so, sig_b, 10.0, seeds=range(4))


def test_silent_unreached_source_does_not_raise():
    """A source that reaches no follower with positive significance but never posts
    (rate 0 here) raises nothing in the reference -- take_one_sample only runs for an
    event that is played -- so the batch raises nothing either; the same world with
    that source posting raises (test_unreached_event_raises_like_reference)."""
    torch, engine, graphs, O = _ctx()
    from redqueen_amd import batch
    from redqueen_amd.opt_model import SimOpts
    w, sig = _err_worlds()["zerosig"]
    w = dict(w, other_sources=[("Poisson2", {"src_id": 1000, "seed": 42, "rate": 10.0}),
                               ("Poisson2", {"src_id": 1001, "seed": 43, "rate": 0.0})])
    so = SimOpts(**w)
    out = batch.run_significance(so, sig, 10.0, seeds=range(4))
    assert len(out) == 4 and (out.status == 0).all()
    m = so.create_manager_with_significance(3, time_period=10.0, significance=sig)
    m.run_dynamic()
    assert m.state.get_num_events() > 0


def test_capped_last_event_like_reference(golden):
    """Under a max_events cap run_dynamic stops before it hands its last event to the
    controller (opt_model.py:271-281): the reference does not raise when the capped
    run's LAST event is the first one of a source that reaches no follower with
    positive significance, and raises one event later (errors.npz sig_cap_*: k = the
    index of that event in the reference's run).  The facade and the batch agree, at
    the k of the engine's own run."""
    torch, engine, graphs, O = _ctx()
    from redqueen_amd import batch
    from redqueen_amd.opt_model import SimOpts
    g = golden("errors.npz")
    assert str(g["sig_cap_1_err"][0]) == "none" and str(g["sig_cap_2_err"][0]) == "ValueError"
    w, sig = _err_worlds()["zerosig"]
    so = SimOpts(**w)
    first_raise = None
    for cap in range(1, 200):
        m = so.create_manager_with_significance(3, time_period=10.0, significance=sig)
        try:
            m.run_dynamic(max_events=cap)
        except ValueError:
            first_raise = cap
            break
        df = m.state.get_dataframe()
        assert 1001 not in set(df.src_id[df.event_id < df.event_id.max()])
    assert first_raise is not None and first_raise >= 2
    k = first_raise - 2   # cap k + 1 ran, cap k + 2 raised
    m = so.create_manager_with_significance(3, time_period=10.0, significance=sig)
    m.run_dynamic(max_events=k + 1)
    ev = m.state.get_dataframe().groupby("event_id").src_id.first().values
    assert len(ev) == k + 1 and ev[k] == 1001
    # the batch on the same run (controller seed 3, the world's own seeds)
    batch.run_significance(so, sig, 10.0, seeds=[3], randomize=False, max_events=k + 1)
    with pytest.raises(ValueError):
        batch.run_significance(so, sig, 10.0, seeds=[3], randomize=False, max_events=k + 2)
