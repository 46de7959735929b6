"""The reference's plugin point for broadcasters: SimOpts.registerSource
(opt_model.py:768-771) with a STATIC class implementing initialize() /
get_all_times() (:336-338, :391-394).  The host runs the plugin's own code (once
per run, or once per replica with the seeds randomize_other_sources gives it,
:795-804) and the engine plays the times as RealData streams -- per-replica ones
through rq_batch_desc.rd_* (ABI v3).  Expected values: tests/golden/plugin.npz,
written by gen_golden.py with the same class over the reference's Broadcaster.
A dynamic plugin has no kernel and raises NotImplementedError (RQ_EUNSUPPORTED)."""
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


def test_dynamic_plugin_is_unsupported():
    engine, SimOpts, Bursty, (w, ctrl, us) = _setup()
    from redqueen_amd.opt_model import Broadcaster

    class Chatty(Broadcaster):
        def __init__(self, src_id, seed):
            super().__init__(src_id, seed)

        def get_next_interval(self, event):
            return 1.0
    SimOpts.registerSource("Chatty", Chatty)
    w2 = dict(w, other_sources=[("Chatty", {"src_id": 2, "seed": 1})],
              edge_list=[e for e in w["edge_list"] if e[0] != 6])
    so = SimOpts(**w2)
    with pytest.raises(NotImplementedError):
        so.create_manager_with_times(np.asarray(ctrl)).run_dynamic()
    with pytest.raises(NotImplementedError):
        engine.Graph(w2["src_id"], w2["other_sources"], w2["sink_ids"], w2["edge_list"],
                     w2["end_time"])
