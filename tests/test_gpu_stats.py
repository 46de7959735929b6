"""GPU ensembles vs the reference's 10k-replica C2 ensemble (99% CI per mean)."""
import math

import numpy as np
import pytest

from redqueen_amd import graphs

pytestmark = pytest.mark.gpu
KS = [1, 2, 5, 10]


def test_c2_redqueen_vs_poisson_distribution(golden):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from redqueen_amd import batch
    from redqueen_amd.opt_model import SimOpts
    d = golden("dist_c2.npz")
    cols = [str(c) for c in d["cols"]]
    ref = {c: d["data"][:, i] for i, c in enumerate(cols)}
    n = d["data"].shape[0]
    off = int(d["poisson_seed_offset"][0]) if "poisson_seed_offset" in d.files else 0
    df = batch.run_opt_vs_poisson(SimOpts(**graphs.readme()), seeds=range(n), Ks=KS,
                                  poisson_seed_offset=off)
    assert (df.status == 0).all()
    for typ, pre in (("Opt", "opt_"), ("Poisson", "poi_")):
        sub = df[df.type == typ]
        eng = {pre + "posts": sub.num_events.values, pre + "world": sub.world_events.values,
               pre + "avg": sub.avg_rank.values, pre + "r2": sub.r_2.values}
        for k in KS:
            eng[pre + "top%d" % k] = sub["top_%d" % k].values
        for k, v in eng.items():
            r = ref[k]
            z = (v.mean() - r.mean()) / math.sqrt(v.var() / len(v) + r.var() / len(r))
            assert abs(z) < 2.576, (k, r.mean(), v.mean(), z)
