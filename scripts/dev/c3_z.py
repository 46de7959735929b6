"""z-values of the C3 ensemble test (tests/test_gpu_stats.py) for a given fixture file."""
import math
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from redqueen_amd import engine, graphs  # noqa: E402

d = np.load(sys.argv[1])
cols = [str(c) for c in d["cols"]]
ref = {c: d["data"][:, i] for i, c in enumerate(cols)}
so = graphs.c3()
g = engine.Graph(so["src_id"], so["other_sources"], so["sink_ids"], so["edge_list"], so["end_time"])
stride = int(d["seed_stride"][0])
u = torch.arange(10000, dtype=torch.int64) * stride + 7
res = g.run("opt", q=so["q"], s=so["s"], n_rep=10000, ctrl_seed=u, world_seed=u, randomize=True, Ks=(1,))
eng = {"posts": res.counts[:, 0].double().cpu().numpy(), "world": res.counts[:, 1].double().cpu().numpy(),
       "events": res.counts[:, 2].double().cpu().numpy(),
       "top1": res.metrics[:, 0].cpu().numpy(), "avg": res.metrics[:, 1].cpu().numpy()}
print("reference rows", d["data"].shape[0])
for k, v in eng.items():
    r = ref[k]
    z = (v.mean() - r.mean()) / math.sqrt(v.var() / len(v) + r.var() / len(r))
    print(k, "ref %.6g gpu %.6g z %.3f" % (r.mean(), v.mean(), z))
