"""Host side of the reactive dynamic plugins (opt_model.reactive_plugin_times): given
the OTHER sources' events of a reference run, run_dynamic's loop (opt_model.py:271-311)
with the plugin beside them reproduces the plugin's own event times of that run bit for
bit -- for the reactive KnockedOff (the reference's SmartPoisson idea, :436-455) and for
the self-driven Renewal.  Expected values: tests/golden/dynplugin.npz (the reference's
run_dynamic dfs)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))


def _events(d, key):
    """(t, src_id) per event of a fixture df, in event order."""
    eid = d[key + "_event_id"]
    _, first = np.unique(eid, return_index=True)
    return d[key + "_t"][first], d[key + "_src_id"][first].astype(np.int64)


def _plugins():
    from realdata_worlds import KnockedOffMixin, RenewalMixin, dyn_plugin_world
    from redqueen_amd.opt_model import Broadcaster

    class Renewal(RenewalMixin, Broadcaster):
        pass

    class KnockedOff(KnockedOffMixin, Broadcaster):
        pass
    return Renewal, KnockedOff, dyn_plugin_world()


def test_reactive_plugin_times_reproduce_the_reference(golden):
    from redqueen_amd.opt_model import reactive_plugin_times
    d = golden("dynplugin.npz")
    Renewal, KnockedOff, (w, ctrl, us) = _plugins()
    for key, inst in (("knock", KnockedOff(src_id=2, seed=21, rate=1.0)),
                      ("base", Renewal(src_id=2, seed=21, scale=0.6))):
        t, src = _events(d, key)
        own = t[src == 2]
        assert own.size > 3
        got = reactive_plugin_times(inst, 0.0, w["sink_ids"], w["edge_list"], w["end_time"], t, src)
        assert np.array_equal(got, own), (key, got, own)


def test_reactive_plugin_times_ignore_the_plugins_own_log_entries(golden):
    """The plugin's own entries of the log it is handed are dropped: a log with the
    plugin's events moved (a previous iteration's guess) gives the same times."""
    from redqueen_amd.opt_model import reactive_plugin_times
    d = golden("dynplugin.npz")
    _R, KnockedOff, (w, ctrl, us) = _plugins()
    t, src = _events(d, "knock")
    own = t[src == 2]
    others = src != 2
    guess_t = np.concatenate([t[others], [1.5, 2.5]])
    guess_s = np.concatenate([src[others], [2, 2]])
    o = np.argsort(guess_t, kind="stable")
    got = reactive_plugin_times(KnockedOff(src_id=2, seed=21, rate=1.0), 0.0, w["sink_ids"],
                                w["edge_list"], w["end_time"], guess_t[o], guess_s[o])
    assert np.array_equal(got, own)


def test_reactive_plugin_times_max_events(golden):
    """run_dynamic stops after max_events events: the plugin's times stop there too."""
    from redqueen_amd.opt_model import reactive_plugin_times
    d = golden("dynplugin.npz")
    _R, KnockedOff, (w, ctrl, us) = _plugins()
    t, src = _events(d, "knock")
    n = 12
    got = reactive_plugin_times(KnockedOff(src_id=2, seed=21, rate=1.0), 0.0, w["sink_ids"],
                                w["edge_list"], w["end_time"], t, src, max_events=n)
    assert np.array_equal(got, t[:n][src[:n] == 2])
