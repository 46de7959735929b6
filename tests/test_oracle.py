"""The CPU oracle pinned against the reference's own outputs (tests/golden/).

Every fixture was produced by importing MPI-SWS/RedQueen in the build
container (tests/golden/gen_golden.py); these tests only read the data.
"""
import math

import numpy as np
import pytest

import ensemble as E
from oracle import oracle as O
from redqueen_amd import graphs

KS = [1, 2, 5, 10]


def npsum_input(n):   # same generator as gen_golden.npsum_input
    rs = np.random.RandomState(1000003 + n)
    return rs.standard_normal(n) * np.exp(rs.uniform(-30, 30, n))


def test_npsum_matches_numpy(golden):
    d = golden("npsum.npz")
    for n, s in zip(d["sizes"], d["sums"]):
        assert O.npsum(npsum_input(int(n))) == s, n


def test_mt19937_legacy_draws(golden):
    d = golden("mt_draws.npz")
    n_checked = 0
    for key in d.files:
        kind, seed = key.split("_")[0], int(key.split("_")[1])
        if kind == "rs":
            got = O.mt_draws(seed, 0, n=256)
        elif kind == "exp":
            got = O.mt_draws(seed, 1, 0.37, n=256)
        elif kind == "uni":
            got = O.mt_draws(seed, 3, 3.0, 100.0, n=256)
        else:
            lam = float(key.split("_")[2])
            got = O.mt_draws(seed, 2, lam, n=64)
        assert np.array_equal(got, d[key]), key
        n_checked += 1
    assert n_checked > 50


def test_philox_random123_kat():
    assert O.philox([0, 0, 0, 0], [0, 0]) == [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]
    assert O.philox([0xffffffff] * 4, [0xffffffff] * 2) == \
        [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]
    assert O.philox([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344],
                    [0xa4093822, 0x299f31d0]) == [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]


def _ulps(a, b):
    if a == b:
        return 0.0
    return abs(a - b) / (math.ulp(abs(b)) if b != 0 else math.ulp(0.0))


def test_spec_log_exp_within_one_ulp():
    rs = np.random.RandomState(7)
    L = O.lib()
    xs = np.concatenate([rs.uniform(0, 1, 20000), rs.uniform(1 - 1e-6, 1, 5000),
                         np.exp(rs.uniform(-700, 0, 5000)), [2.0 ** -53, 0.5, 1.0]])
    worst = max(_ulps(L.rqo_spec_log(float(x)), math.log(x)) for x in xs if x > 0)
    assert worst <= 1.0
    ys = np.concatenate([-rs.uniform(0, 50, 20000), -rs.uniform(0, 700, 5000), [0.0, -1e-12]])
    worst = max(_ulps(L.rqo_spec_exp(float(y)), math.exp(y)) for y in ys)
    assert worst <= 1.0
    assert L.rqo_spec_exp(-800.0) == 0.0


def _ref_events(sc):
    return O.ref_run(sc, numpy_exp=True, dot_fma=1)


def _check_events(t, dt, s, ft, fdt, fs):
    assert len(t) == len(ft)
    assert np.array_equal(s, fs)
    assert np.array_equal(t, ft)
    assert np.array_equal(dt, fdt)


def _metrics_of(sc, t, dt, s, end=None, src=None):
    df = sc.expand(t, dt, s)
    top, avg, r2, cnt = O.metrics_df(df["t"], df["src_id"], df["sink_id"], df["event_id"],
                                     sc.src_id if src is None else src,
                                     sc.end_time if end is None else end, KS)
    return np.asarray(top + [avg, r2]), cnt


def test_reference_run_readme_bit_exact(golden):
    d = golden("readme_runs.npz")
    so = graphs.readme()
    for seed in d["seeds"]:
        sc = O.Scenario(so, ("opt", int(seed)))
        t, dt, s = _ref_events(sc)
        _check_events(t, dt, s, d["t_%d" % seed], d["dt_%d" % seed], d["src_%d" % seed])
        met, cnt = _metrics_of(sc, t, dt, s)
        assert np.array_equal(met, d["met_%d" % seed])
        assert cnt[0] == d["cnt_%d" % seed][0] and cnt[1] == d["cnt_%d" % seed][1]


def test_reference_run_variants_bit_exact(golden):
    d = golden("readme_runs.npz")
    so = graphs.readme()
    cases = {"wall": (so, ("wall",), None), "pois": (so, ("poisson", 7, 400 / 100.0), None),
             "long": (dict(so, end_time=400.0), ("opt", 3), None),
             "max": (so, ("opt", 101), 500)}
    for name, (so_, ctrl, maxev) in cases.items():
        sc = O.Scenario(so_, ctrl, max_events=maxev)
        t, dt, s = _ref_events(sc)
        _check_events(t, dt, s, d["t_" + name], d["dt_" + name], d["src_" + name])
        met, cnt = _metrics_of(sc, t, dt, s, src=so["src_id"])
        assert np.array_equal(met, d["met_" + name]), name
    # the long run has more than 8192 pivot rows: chunked np.sum exercised
    assert len(d["t_long"]) > 8192


def test_reference_run_all_kinds_bit_exact(golden):
    d = golden("mixed_runs.npz")
    so = graphs.mixed()
    for seed in (3, 4):
        sc = O.Scenario(so, ("opt", seed))
        t, dt, s = _ref_events(sc)
        _check_events(t, dt, s, d["t_%d" % seed], d["dt_%d" % seed], d["src_%d" % seed])
        met, _ = _metrics_of(sc, t, dt, s)
        assert np.array_equal(met, d["met_%d" % seed])


def test_notebook_kats(golden):
    d = golden("kat_runs.npz")
    # K3..K6: opt_broadcast.ipynb:5443-5615 (values in SURVEY.md Appendix C)
    so1 = graphs.kat_two_walls((1.0, 1.0))
    so5 = graphs.kat_two_walls((0.5, 1.5))
    for name, so, ctrl in [("k3", so1, ("opt", 1)), ("k4", so1, ("poisson", 45, 324 / 100.0)),
                           ("k5", so5, ("opt", 1)), ("k6", so5, ("poisson", 4, 325 / 100.0))]:
        sc = O.Scenario(so, ctrl)
        t, dt, s = _ref_events(sc)
        _check_events(t, dt, s, d[name + "_t"], d[name + "_dt"], d[name + "_src"])
        met, cnt = _metrics_of(sc, t, dt, s)
        assert np.array_equal(met, d[name + "_met"]), name
    assert d["k3_met"][0] == 30.650573346374472 and d["k3_met"][4] == 172.61428368229843
    assert d["k5_met"][0] == 30.612478277225335 and d["k6_met"][4] == 299.4093214809409
    # K1/K2: std_poisson(42, 1000), Opt seed 1, T=1
    so = dict(src_id=1, other_sources=[("Poisson2", {"src_id": 2, "seed": 42, "rate": 1000.0})],
              end_time=1.0, sink_ids=[1001], s=np.asarray([1.0]), q=1.0,
              edge_list=[(1, 1001), (2, 1001)])
    sc = O.Scenario(so, ("opt", 1))
    t, dt, s = _ref_events(sc)
    assert np.array_equal(t, d["k1_t"]) and np.array_equal(s, d["k1_src"])
    df = sc.expand(t, dt, s)
    for src, exp in zip((1, 2), d["k2_top10"]):
        top, _, _, _ = O.metrics_df(df["t"], df["src_id"], df["sink_id"], df["event_id"], src,
                                    1.0, [10])
        assert top[0] == exp


def test_metrics_on_adversarial_dfs(golden):
    for fname, cols in (("adversarial.npz", ("_t", "_src", "_sink", "_eid")),
                        ("frac.npz", ("_t", "_src_id", "_sink_id", "_event_id"))):
        d = golden(fname)
        for c in d["cases"]:
            top, avg, r2, _ = O.metrics_df(d[c + cols[0]], d[c + cols[1]], d[c + cols[2]],
                                           d[c + cols[3]], 1, d[c + "_end"][0], KS)
            assert np.array_equal(np.asarray(top + [avg, r2]), d[c + "_met"]), (fname, c)


def test_engine_semantics_match_reference_distribution(golden):
    """Engine semantics (Philox streams, clean times, O(1) u increments) vs the
    reference over 10k C2 replicas: every mean inside the 99% CI (|z| < 2.576)."""
    d = golden("dist_c2.npz")
    cols = [str(c) for c in d["cols"]]
    ref = {c: d["data"][:, i] for i, c in enumerate(cols)}
    so = graphs.readme()
    n = d["data"].shape[0]
    out, cnt, _ = O.engine_batch(O.Scenario(so, ("opt", 0)), n, 0, True, KS, 8)
    eng = {"opt_posts": cnt[:, 0], "opt_world": cnt[:, 1], "opt_events": cnt[:, 2]}
    for i, k in enumerate(KS):
        eng["opt_top%d" % k] = out[:, i]
    eng["opt_avg"], eng["opt_r2"] = out[:, len(KS)], out[:, len(KS) + 1]
    # Poisson comparator: capacity = the RedQueen replica's posts (opt_runs.worker_poisson)
    rates = cnt[:, 0] / so["end_time"]
    off = int(d["poisson_seed_offset"][0])
    out2, cnt2, _ = O.engine_batch(O.Scenario(so, ("poisson", 0, 1.0)), n, 0, True, KS, 8,
                                   ctrl_rates=rates, ctrl_seed_offset=off)
    eng["poi_posts"], eng["poi_world"] = cnt2[:, 0], cnt2[:, 1]
    for i, k in enumerate(KS):
        eng["poi_top%d" % k] = out2[:, i]
    eng["poi_avg"], eng["poi_r2"] = out2[:, len(KS)], out2[:, len(KS) + 1]
    # replica r: world randomize_other_sources(r) -> seeds r, r + 99 (clusters r mod 99)
    ind = E.independent_rows(n, 2)
    E.compare("oracle_c2", eng, ref, clusters=99, indep_eng=ind, indep_ref=ind, z_bound=2.576)


def test_engine_world_distributions(golden):
    d = golden("dist_world.npz")
    worlds = {
        "hawkes": dict(src_id=1, end_time=50.0, s=1.0, q=1.0, sink_ids=[1, 2],
                       other_sources=[("Hawkes", {"src_id": 2, "seed": 0, "l_0": 2.0,
                                                  "alpha": 1.0, "beta": 2.0}),
                                      ("Hawkes", {"src_id": 3, "seed": 0, "l_0": 5.0,
                                                  "alpha": 2.0, "beta": 10.0})],
                       edge_list=[(2, 1), (3, 1), (3, 2)]),
        "pwconst": dict(src_id=1, end_time=60.0, s=1.0, q=1.0, sink_ids=[1, 2],
                        other_sources=[("PiecewiseConst", {"src_id": 2, "seed": 0,
                                                           "change_times": [0.0, 20.0, 45.0],
                                                           "rates": [3.0, 0.5, 6.0]}),
                                       ("Poisson", {"src_id": 3, "seed": 0, "rate": 4.0}),
                                       ("Poisson2", {"src_id": 4, "seed": 0, "rate": 2.5})],
                        edge_list=[(2, 1), (3, 2), (4, 1), (4, 2)]),
    }
    # randomize_other_sources(u) gives source k seed u + 99 k, so replicas r and r + 99
    # share streams: the means use the cluster-robust variance (clusters r mod 99), the
    # spread / shape tests the rows that share no stream (E.independent_rows)
    for name, so in worlds.items():
        ref = d[name].astype(np.float64)
        ns = len(so["other_sources"])
        out, cnt, _ = O.engine_batch(O.Scenario(so, ("wall",)), 40000, 0, True, KS, 8)
        eng = {"world": cnt[:, 1]}
        rr = {"world": ref[:, :ns].sum(1)}
        for i in range(len(KS) + 2):
            eng["m%d" % i], rr["m%d" % i] = out[:, i], ref[:, ns + i]
        E.compare("oracle_world_" + name, eng, rr, clusters=99,
                  indep_eng=E.independent_rows(len(out), ns),
                  indep_ref=E.independent_rows(len(ref), ns), z_bound=2.576)


def test_discarded_hawkes_draw_under_cluster_variance(golden):
    """Round 1 replaced the reference's 10k-replica Hawkes world draw at seed0 0 by a 30k
    draw at seed0 3e6 after its top-5 mean sat ~3 naive sd off the engine's.  That draw
    (regenerated: dist_hawkes0.npz) shares streams between replicas r and r + 99; under
    the cluster-robust variance of the mean its worst z is -2.53, inside the 99 % band
    per statistic, and every spread / shape test passes family-wise.  The two reference
    draws differ from EACH OTHER by up to |z| 2.65 on the same statistics."""
    d = golden("dist_hawkes0.npz")
    ref = d["hawkes"].astype(np.float64)
    w = golden("dist_world.npz")["hawkes"].astype(np.float64)
    so = dict(src_id=1, end_time=50.0, s=1.0, q=1.0, sink_ids=[1, 2],
              other_sources=[("Hawkes", {"src_id": 2, "seed": 0, "l_0": 2.0, "alpha": 1.0,
                                         "beta": 2.0}),
                             ("Hawkes", {"src_id": 3, "seed": 0, "l_0": 5.0, "alpha": 2.0,
                                         "beta": 10.0})],
              edge_list=[(2, 1), (3, 1), (3, 2)])
    out, cnt, _ = O.engine_batch(O.Scenario(so, ("wall",)), 40000, 0, True, KS, 8)
    eng, rr, ww = {"world": cnt[:, 1]}, {"world": ref[:, :2].sum(1)}, {"world": w[:, :2].sum(1)}
    for i in range(len(KS) + 2):
        eng["m%d" % i], rr["m%d" % i], ww["m%d" % i] = out[:, i], ref[:, 2 + i], w[:, 2 + i]
    rec = E.compare("oracle_world_hawkes_seed0", eng, rr, clusters=99, z_bound=2.576,
                    indep_eng=E.independent_rows(len(out), 2),
                    indep_ref=E.independent_rows(len(ref), 2))
    assert 2.4 < rec["max_abs_z"] < 2.576
    # reference vs reference: the same statistics, the same cluster-robust z
    rr_ = E.compare("reference_hawkes_seed0_vs_3e6", rr, ww, clusters=99,
                    indep_eng=E.independent_rows(len(ref), 2),
                    indep_ref=E.independent_rows(len(w), 2))
    assert rr_["max_abs_z"] > 2.0


def test_engine_is_deterministic_and_seed_sensitive():
    so = graphs.readme()
    a = O.engine_run(O.Scenario(so, ("opt", 5)))
    b = O.engine_run(O.Scenario(so, ("opt", 5)))
    c = O.engine_run(O.Scenario(so, ("opt", 6)))
    assert all(np.array_equal(x, y) for x, y in zip(a, b))
    assert not np.array_equal(a[0], c[0])
    # every event time is within [0, T] and non-decreasing
    assert np.all(np.diff(a[0]) >= 0) and a[0][0] >= 0 and a[0][-1] <= 100.0


def test_engine_c3_matches_reference_distribution(golden):
    """Engine semantics on the C3 bench network vs the reference's 10k replicas of it."""
    d = golden("dist_c3.npz")
    assert d["data"].shape[0] >= 10000
    cols = [str(c) for c in d["cols"]]
    ref = {c: d["data"][:, i] for i, c in enumerate(cols)}
    so = graphs.c3()
    out, cnt, _ = O.engine_batch(O.Scenario(so, ("opt", 0)), 1024, 500000, True, (1,), 8,
                                 seed_stride=int(d["seed_stride"][0]))
    eng = {"posts": cnt[:, 0], "world": cnt[:, 1], "events": cnt[:, 2], "top1": out[:, 0],
           "avg": out[:, 1]}
    E.compare("oracle_c3", eng, ref, z_bound=2.576)


def test_engine_g120_matches_reference_distribution(golden):
    """Engine semantics on a > 64-source world (graphs.g120: the general sweep's
    instances) vs the reference's replicas of it (dist_g120.npz)."""
    d = golden("dist_g120.npz")
    cols = [str(c) for c in d["cols"]]
    ref = {c: d["data"][:, i] for i, c in enumerate(cols)}
    so = graphs.g120()
    out, cnt, _ = O.engine_batch(O.Scenario(so, ("opt", 0)), 4096, 900000, True, KS, 8,
                                 seed_stride=int(d["seed_stride"][0]))
    eng = {"posts": cnt[:, 0], "world": cnt[:, 1], "events": cnt[:, 2], "avg": out[:, len(KS)],
           "r2": out[:, len(KS) + 1]}
    for i, k in enumerate(KS):
        eng["top%d" % k] = out[:, i]
    E.compare("oracle_g120", eng, ref, z_bound=2.576)


def test_realdata_worlds_both_restatements_exact(golden):
    """All-RealData worlds (create_manager_with_times): the reference restatement
    AND the engine-semantics restatement reproduce the reference's whole df -- event
    order under equal times, accumulated time_delta -- and its metrics (realdata.npz)."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from realdata_worlds import realdata_worlds
    d = golden("realdata.npz")
    for name, w, ctrl, maxev in realdata_worlds():
        sc = O.Scenario(w, ("times", np.asarray(ctrl, dtype=np.float64)), max_events=maxev)
        for run in (O.ref_run, O.engine_run):
            t, dt, s = run(sc)
            cols = sc.expand(t, dt, s)
            for c in ("event_id", "time_delta", "src_id", "t", "sink_id"):
                assert np.array_equal(cols[c], d[name + "_" + c]), (name, run.__name__, c)
            top, avg, r2, cnt = O.metrics_df(cols["t"], cols["src_id"], cols["sink_id"],
                                             cols["event_id"], w["src_id"], w["end_time"], KS)
            assert np.array_equal(np.asarray(top + [avg, r2]), d[name + "_met"]), name
            assert np.array_equal(O.state_time_deltas(t), dt)


def test_engine_c5_mid_matches_reference_distribution(golden):
    """Engine semantics on C5's source side (graphs.c5_mid: 500 bursty Hawkes broadcasters
    at T = 1000, ~3.2 x 10^5 events per replica) vs the reference's own replicas of it
    (dist_c5m.npz)."""
    d = golden("dist_c5m.npz")
    cols = [str(c) for c in d["cols"]]
    ref = {c: d["data"][:, i] for i, c in enumerate(cols)}
    so = graphs.c5_mid()
    out, cnt, _ = O.engine_batch(O.Scenario(so, ("opt", 0)), 96, 700000, True, KS, 8,
                                 seed_stride=int(d["seed_stride"][0]))
    eng = {"posts": cnt[:, 0], "world": cnt[:, 1], "events": cnt[:, 2], "avg": out[:, len(KS)],
           "r2": out[:, len(KS) + 1]}
    for i, k in enumerate(KS):
        eng["top%d" % k] = out[:, i]
    E.compare("oracle_c5m", eng, ref, z_bound=2.576)
