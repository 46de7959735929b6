"""Host-side logic of the drop-in surface (no GPU): SimOpts / Manager API parity
with the reference (opt_model.py:755-1013), the df row layout, the graph
generators against the reference's networks."""
import numpy as np
import pytest

from oracle import oracle as O
from redqueen_amd import graphs
from redqueen_amd.opt_model import (Hawkes, Manager, Opt, PiecewiseConst, Poisson, Poisson2,
                                    RealData, SimOpts, State)


def test_simopts_roundtrip_and_registry():
    """The reference's own self-test, test_simOpts (opt_model.py:970-1013)."""
    init_opts = {'src_id': 1, 'end_time': 100.0, 's': np.array([1, 2]), 'q': 1.0,
                 'other_sources': [(Poisson, {'src_id': 2, 'seed': 1}),
                                   (Poisson, {'src_id': 3, 'seed': 1})],
                 'sink_ids': [1001, 1000],
                 'edge_list': [(1, 1001), (1, 1000), (2, 1000), (3, 1001)]}
    s = SimOpts(**init_opts)
    assert s.get_dict() == init_opts
    assert s.update({'src_id': 2}).src_id == 2
    assert s.create_other_sources()[0].src_id == 2
    init2 = dict(init_opts, other_sources=[
        ('Poisson', {'src_id': 2, 'seed': 1, 'rate': 1000.0}),
        ('Poisson2', {'src_id': 3, 'seed': 1, 'rate': 1000.0}),
        ('Hawkes', {'src_id': 4, 'seed': 1, 'l_0': 1.0, 'alpha': 1.0, 'beta': 10.0}),
        ('PiecewiseConst', {'src_id': 5, 'seed': 1, 'rates': [0.0, 0.5, 1.0],
                            'change_times': [0, 50, 75]}),
        ('Opt', {'src_id': 6, 'seed': 1, 's': np.array([1.0]), 'q': 1.0}),
        ('RealData', {'src_id': 7, 'times': [0, 50, 75]})])
    s = SimOpts(**init2)
    kinds = [type(x) for x in s.create_other_sources()]
    assert kinds == [Poisson, Poisson2, Hawkes, PiecewiseConst, Opt, RealData]
    with pytest.raises(KeyError):
        SimOpts(src_id=1)
    with pytest.raises(ValueError):
        SimOpts(**dict(init_opts, other_sources=[('Nope', {})])).create_other_sources()


def test_factories_and_validation():
    so = SimOpts(**graphs.readme())
    with pytest.raises(ValueError):
        so.create_manager_with_poisson(seed=1)
    with pytest.raises(ValueError):
        so.create_manager_with_poisson(seed=1, rate=1.0, capacity=3)
    m = so.create_manager_with_poisson(seed=1, capacity=250)
    assert isinstance(m.sources[0], Poisson2) and m.sources[0].rate == 2.5
    w = so.create_manager_for_wall()
    assert all(e[0] != so.src_id for e in w.edge_list) and w.sink_ids == so.sink_ids
    r = so.randomize_other_sources(7)
    assert [kw["seed"] for _, kw in r.other_sources] == [7, 106]
    with pytest.raises(AssertionError):
        Manager([Opt(1, 0), Opt(1, 1)], sink_ids=[1], end_time=1.0, edge_list=[])
    with pytest.raises(AssertionError):
        Manager([Opt(1, 0)], sink_ids=[1, 1], end_time=1.0, edge_list=[])
    with pytest.raises(AssertionError):
        Manager([Opt(1, 0)], sink_ids=[1], end_time=1.0, edge_list=[(2, 1)])
    with pytest.raises(AssertionError):
        Manager([Opt(1, 0)], sink_ids=[1], end_time=1.0, edge_list=[(1, 5)])
    with pytest.raises(AssertionError):
        PiecewiseConst(2, 0, change_times=[0, 5, 3], rates=[1, 2, 3])
    m = Manager([Opt(1, 0), Poisson(2, 0)], sink_ids=[1, 2], end_time=1.0)
    assert m.edge_list == [(1, 1), (1, 2), (2, 1), (2, 2)]
    with pytest.raises(IndexError):   # scalar s: the reference indexes s.shape[0] too
        so.create_manager_with_significance(1, 10.0)
    m = so.update({"s": np.asarray([1.0, 2.0, 3.0])}).create_manager_with_significance(
        1, 10.0, num_segments=4)
    assert m.sources[0].s_pw.shape == (3, 4) and m.sources[0].time_period == 10.0


def test_state_log_without_a_run():
    """The event list of a State (the df rows are expanded on the GPU: test_gpu_export)."""
    so = graphs.readme()
    sc = O.Scenario(so, ("opt", 101))
    t, dt, s = O.engine_run(sc)
    st = State(0.0, so["sink_ids"])
    assert len(st.get_dataframe()) == 0
    st._set_log(t, s, so["edge_list"])
    assert st.get_num_events() == len(t)
    ev = st.events[3]
    assert ev.event_id == 103 and ev.src_id == s[3] and ev.cur_time == t[3]
    assert ev.time_delta == dt[3]   # accumulated State.time (opt_model.py:68)
    assert np.array_equal([e.time_delta for e in st.events], O.state_time_deltas(t))


def test_graph_generators_reproduce_reference_networks(golden):
    g = golden("graphs.npz")
    assert np.array_equal(np.asarray(graphs.make_edge_list(1000, 50, 5, 1024, 1000, 5000)), g["c3"])
    assert np.array_equal(np.asarray(graphs.make_edge_list(20, 7, 3, 5, 1000, 5000)), g["small"])
    so = graphs.followers_graph(num_followers=50, num_sources=20, degree=1, kinds=("Hawkes",),
                                world_rate=100.0, max_num_followers=80)
    assert np.array_equal(np.asarray(so["edge_list"]), g["mf_edges"])
    assert np.array_equal(np.asarray(so["sink_ids"]), g["mf_sinks"])
    assert so["q"] == g["mf_q"][0]
    c3 = graphs.c3()
    assert len(c3["sink_ids"]) == 1000 and len(c3["other_sources"]) == 50
    assert len(c3["edge_list"]) == 6000


def test_inference_queue_helpers():
    """run_inference_queue's batching rule (host logic): worlds batch when they share a
    network and carry randomize_other_sources seeds; extract_perf_fields keeps the
    reference's performance fields."""
    from redqueen_amd import opt_runs as R
    from redqueen_amd.opt_model import SimOpts
    a = SimOpts.std_poisson(world_rate=4.0, world_seed=45)
    b = SimOpts.std_poisson(world_rate=4.0, world_seed=46)
    assert R._world_key(a) == R._world_key(b) and R._randomize_seed(a) == 45
    c = a.randomize_other_sources(7)
    assert R._randomize_seed(c) == 7
    two = SimOpts(src_id=1, end_time=5.0, q=1.0, s=1.0, sink_ids=[1],
                  other_sources=[("Poisson2", {"src_id": 2, "seed": 3, "rate": 1.0}),
                                 ("Poisson2", {"src_id": 3, "seed": 4, "rate": 1.0})],
                  edge_list=[(1, 1), (2, 1), (3, 1)])
    assert R._randomize_seed(two) is None and R._randomize_seed(two.randomize_other_sources(9)) == 9
    op = {"seed": 1, "q": 2.0, "type": "Opt", "top_1": 0.5, "avg_rank": 1.0, "r_2": 2.0,
          "num_events": 3, "world_events": 4, "capacity": 3.0}
    assert list(R.extract_perf_fields(op)) == R.perf_opts.performance_fields


def test_opt_runs_multiple_follower_names_are_drop_in(golden):
    """redqueen_amd.opt_runs exports the reference's multiple-follower helpers with its
    signatures (opt_runs.py:651-795) -- called exactly as tests/golden/gen_golden.py called
    the reference's, they give its networks, sources and rates bit for bit."""
    from redqueen_amd import opt_runs as R
    g = golden("graphs.npz")
    for name, (nf, nb, deg, seed) in {"c3": (1000, 50, 5, 1024), "small": (20, 7, 3, 5)}.items():
        e = R.make_edge_list(num_followers=nf, num_broadcasters=nb, degree=deg, seed=seed,
                             follower_id_offset=1000, broadcaster_id_offset=5000,
                             opts=R.mk_edge_list_opts)
        assert np.array_equal(np.asarray(e, dtype=np.int64), g[name]), name
    so = R.prepare_multiple_followers_sim_opts(num_followers=50, opts=R.multiple_follower_opts.set_new(
        kind="Hawkes", num_other_broadcasters=20, max_num_followers=80))
    assert np.array_equal(np.asarray(so.edge_list), g["mf_edges"])
    assert np.array_equal(np.asarray(so.sink_ids), g["mf_sinks"]) and so.q == g["mf_q"][0]
    assert np.array_equal([x[1]["src_id"] for x in so.other_sources], g["mf_src"])
    for kind in ("PiecewiseConst", "Poisson2"):
        so = R.prepare_multiple_followers_sim_opts(num_followers=10, opts=R.multiple_follower_opts.set_new(
            kind=kind, num_other_broadcasters=6, max_num_followers=20, follower_other_degree=2))
        k = "mf_" + kind.lower()
        assert np.array_equal(np.asarray(so.edge_list), g[k + "_edges"]), kind
        assert np.array_equal([x[1]["src_id"] for x in so.other_sources], g[k + "_src"])
        assert np.array_equal([x[1]["seed"] for x in so.other_sources], g[k + "_seed"])
        if kind == "PiecewiseConst":
            assert np.array_equal(np.asarray([x[1]["rates"] for x in so.other_sources]), g[k + "_rates"])
            assert np.array_equal(np.asarray([x[1]["change_times"] for x in so.other_sources]),
                                  g[k + "_times"])
        else:
            assert np.array_equal([x[1]["rate"] for x in so.other_sources], g[k + "_rates"])
    assert R.make_piecewise_const(24) == list(g["pwc24"])
    src = R.create_phased_pwconst_broadcaster(7, 3, [1.0, 2.0, 3.0], 2.0, 30.0, 4)
    assert src[0] == "PiecewiseConst" and list(src[1]["change_times"]) == [0.0, 10.0, 20.0]
    assert np.allclose(src[1]["rates"], np.asarray([2.0, 3.0, 1.0]) * 6.0 / 6.0)
    t = R.trim_sim_opts(so)
    assert t.q == so.q and list(t.sink_ids) == list(so.sink_ids)
    assert callable(R.run_inference) and callable(R.run_inference_queue)
