"""rq_metrics_replay on the GPU vs the reference's own metric values (bit-exact).

The dataframes are rebuilt from the golden event logs (reference runs) with
the reference's row layout; the expected numbers are what utils.time_in_top_k /
average_rank / int_r_2 returned on those very dataframes.
"""
import numpy as np
import pandas as pd
import pytest

from redqueen_amd import graphs

pytestmark = pytest.mark.gpu
KS = [1, 2, 5, 10]


def _ctx():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle import oracle as O
    from redqueen_amd import utils as U
    return O, U


def _df(O, so, ctrl, t, dt, s):
    d = O.Scenario(so, ctrl).expand(t, dt, s)
    return pd.DataFrame(d)


def _replay(U, df, src, end):
    m = U.replay_metrics(df, src, end, KS)
    return np.asarray(m["top_k"] + [m["avg_rank"], m["r_2"]]), m


def test_readme_runs(golden):
    O, U = _ctx()
    d = golden("readme_runs.npz")
    so = graphs.readme()
    names = ["%d" % s for s in d["seeds"]] + ["wall", "pois", "long", "max"]
    for name in names:
        so_ = dict(so, end_time=400.0) if name == "long" else so
        df = _df(O, so_, ("wall",) if name == "wall" else ("opt", 0),
                 d["t_" + name], d["dt_" + name], d["src_" + name])
        got, m = _replay(U, df, so["src_id"], so_["end_time"])
        assert np.array_equal(got, d["met_" + name]), (name, got - d["met_" + name])
        assert m["num_own"] == d["cnt_" + name][0] and m["num_world"] == d["cnt_" + name][1]


def test_notebook_kats(golden):
    O, U = _ctx()
    d = golden("kat_runs.npz")
    so = graphs.kat_two_walls()
    for name in ("k3", "k4", "k5", "k6"):
        df = _df(O, so, ("opt", 0), d[name + "_t"], d[name + "_dt"], d[name + "_src"])
        assert df.shape == (d[name + "_cnt"][2], 5)
        got, m = _replay(U, df, 1, 100.0)
        assert np.array_equal(got, d[name + "_met"]), name
        assert m["num_own"] == d[name + "_cnt"][0]
    assert d["k3_met"][0] == 30.650573346374472
    # K2: time_in_top_k(df, src_id=x, K=10) on the std_poisson run
    so1 = dict(src_id=1, other_sources=[("Poisson2", {"src_id": 2, "seed": 42, "rate": 1000.0})],
               end_time=1.0, sink_ids=[1001], s=np.asarray([1.0]), q=1.0,
               edge_list=[(1, 1001), (2, 1001)])
    df = _df(O, so1, ("opt", 0), d["k1_t"], np.zeros_like(d["k1_t"]), d["k1_src"])
    for x, exp in zip((1, 2), d["k2_top10"]):
        assert U.time_in_top_k(df, K=10, src_id=x, end_time=1.0) == exp


@pytest.mark.parametrize("fname,cols", [("adversarial.npz", ("_eid", "_src", "_t", "_sink")),
                                        ("frac.npz", ("_event_id", "_src_id", "_t", "_sink_id"))])
def test_adversarial_and_fractional(golden, fname, cols):
    O, U = _ctx()
    d = golden(fname)
    for c in d["cases"]:
        df = pd.DataFrame({"event_id": d[c + cols[0]], "src_id": d[c + cols[1]],
                           "t": d[c + cols[2]], "sink_id": d[c + cols[3]]})
        got, _ = _replay(U, df, 1, d[c + "_end"][0])
        assert np.array_equal(got, d[c + "_met"]), (c, got - d[c + "_met"])


def test_public_functions_and_errors(golden):
    O, U = _ctx()
    from redqueen_amd.opt_model import SimOpts
    d = golden("readme_runs.npz")
    so = SimOpts(**graphs.readme())
    df = _df(O, graphs.readme(), ("opt", 0), d["t_101"], d["dt_101"], d["src_101"])
    assert U.time_in_top_k(df=df, K=1, sim_opts=so) == 19.0135536585858
    assert U.average_rank(df, sim_opts=so) == 16947.525806415997
    assert U.int_r_2(df, so) == d["met_101"][5]
    assert U.num_tweets_of(df, sim_opts=so) == 402.0
    op = U.add_perf({}, df, so)
    assert op["num_events"] == 402 and op["world_events"] == d["cnt_101"][1]
    bad = df.iloc[::-1].reset_index(drop=True)
    with pytest.raises(Exception):
        U.time_in_top_k(bad, K=1, sim_opts=so)
