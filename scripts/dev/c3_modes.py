"""C3 (10k replicas) kernel times per sweep mode: 0 the fused sweep, 4 pre-generated
streams + rq_merge_streams + the merged-stream sweep, 6 pre-generated streams + the
windowed sweep.  HIP-event times from the library (rq_timing)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from redqueen_amd import _lib as L, engine, graphs  # noqa: E402

so = graphs.c3()
g = engine.Graph(so["src_id"], so["other_sources"], so["sink_ids"], so["edge_list"], so["end_time"])
R = 10000
for mode in (0, 4, 6, 0, 4):
    kw = dict(q=so["q"], s=so["s"], n_rep=R, ctrl_seed=0, world_seed=0, randomize=True, Ks=(1,),
              sweep_mode=mode, check=False)
    ref = g.run("opt", **kw)
    torch.cuda.synchronize()
    ms = np.zeros(5)
    nl = np.zeros(5, dtype=np.int64)
    L.lib().rq_timing(1)
    for _ in range(5):
        r = g.run("opt", **kw)
    torch.cuda.synchronize()
    L.lib().rq_timing_read(ms.ctypes.data_as(L._pd), nl.ctypes.data_as(L._pi64))
    L.lib().rq_timing(0)
    names = ["gen", "sweep", "scan", "replay", "merge"]
    print(json.dumps({"mode": mode, "plan": g.run("opt", plan_only=True, **kw),
                      "ms": {n: round(ms[k] / 5, 4) for k, n in enumerate(names)},
                      "equal_to_first": bool(torch.equal(r.metrics, ref.metrics))}), flush=True)
