"""OptPWSignificance (opt_model.py:547-623) on the CPU oracle: the reference
restatement (MT19937) reproduces the reference's runs bit for bit, including the
notebook's "Testing out significance" cells (opt_broadcast.ipynb:5469, :5569:
325 / 323 posts, top-1 29.6750640797 / 30.2860675318); the engine semantics
(Philox draws, thinning at the per-event bound) match the reference's 8k-replica
ensemble within 99% CIs."""
import numpy as np
import pytest

import ensemble as E
from oracle import oracle as O

KS = [1, 2, 5, 10]
KAT_BASE = dict(src_id=1, end_time=100.0, q=1.0, sink_ids=[5001, 5002],
                other_sources=[("Poisson2", {"src_id": 1000, "seed": 42, "rate": 10.0}),
                               ("Poisson2", {"src_id": 1001, "seed": 43, "rate": 10.0})],
                edge_list=[(1000, 5001), (1001, 5002), (1, 5001), (1, 5002)])
SO_SIG = dict(src_id=1, s=1.0, q=1.0, end_time=20.0,
              other_sources=[("Poisson2", {"src_id": 1000, "seed": 42, "rate": 50.0})],
              sink_ids=[5001], edge_list=[(1, 5001), (1000, 5001)])


def scenario(key, g):
    so = dict(SO_SIG) if key == "sig" else dict(KAT_BASE, s=[1.0, 1.0])
    seed, period, q = g[key + "_par"]
    return so, O.Scenario(so, ("sig", int(seed), g[key + "_sig"], period))


@pytest.mark.parametrize("key", ["s1", "s41", "s7", "sig"])
def test_reference_restatement_bit_exact(golden, key):
    g = golden("sig_runs.npz")
    so, sc = scenario(key, g)
    t, dt, src = O.ref_run(sc)
    assert np.array_equal(t, g[key + "_t"]) and np.array_equal(src, g[key + "_src"])
    assert np.array_equal(dt, g[key + "_dt"])
    d = sc.expand(t, dt, src)
    top, avg, r2, cnt = O.metrics_df(d["t"], d["src_id"], d["sink_id"], d["event_id"], 1,
                                     so["end_time"], Ks=KS)
    assert np.array_equal(np.asarray(top + [avg, r2]), g[key + "_met"])
    assert cnt[0] == g[key + "_cnt"][0] and cnt[1] == g[key + "_cnt"][1]


def test_notebook_values(golden):
    g = golden("sig_runs.npz")
    assert g["s1_cnt"][0] == 325 and g["s1_cnt"][2] == 2594
    assert round(g["s1_met"][0], 10) == 29.6750640797
    assert round(g["s1_met"][4], 9) == 171.548425075
    assert g["s41_cnt"][0] == 323 and g["s41_cnt"][2] == 2590
    assert round(g["s41_met"][0], 10) == 30.2860675318


def test_engine_matches_reference_distribution(golden):
    d = golden("dist_sig.npz")
    cols = [str(c) for c in d["cols"]]
    ref = {c: d["data"][:, i] for i, c in enumerate(cols)}
    n = d["data"].shape[0]
    sc = O.Scenario(dict(KAT_BASE, s=[1.0, 1.0]), ("sig", 0, d["sig"], 10.0))
    out, cnt, _ = O.engine_batch(sc, n, 0, True, KS, 8)
    eng = {"posts": cnt[:, 0], "world": cnt[:, 1], "events": cnt[:, 2],
           "avg": out[:, len(KS)], "r2": out[:, len(KS) + 1]}
    for i, k in enumerate(KS):
        eng["top%d" % k] = out[:, i]
    # replica r: world randomize_other_sources(r), seeds r and r + 99 (clusters r mod 99)
    ind = E.independent_rows(n, 2)
    E.compare("oracle_sig", eng, ref, clusters=99, indep_eng=ind, indep_ref=ind, z_bound=2.576)
