"""C5 sweep phase split: per-launch sweep time with RQ_SWEEP_DBG = 0 (full), 1 (skip
phase C, the per-sink updates and aggregates), 2 (skip the wall sink updates), 3 (skip
the controller).  Profiling only -- the skipped runs compute nothing meaningful.
usage: RQ_SWEEP_DBG=k python scripts/c5_phase.py [replicas]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from redqueen_amd import _lib as L  # noqa: E402
from redqueen_amd import engine, graphs  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 else 2560
so = graphs.c5()
g = engine.Graph(so["src_id"], so["other_sources"], so["sink_ids"], so["edge_list"], so["end_time"])
g.run("opt", q=so["q"], s=so["s"], n_rep=R, ctrl_seed=7, world_seed=7, randomize=True, check=False)
torch.cuda.synchronize()
L.lib().rq_timing(1)
res = g.run("opt", q=so["q"], s=so["s"], n_rep=R, ctrl_seed=0, world_seed=0, randomize=True, check=False)
torch.cuda.synchronize()
ms = np.zeros(5)
nl = np.zeros(5, dtype=np.int64)
L.lib().rq_timing_read(ms.ctypes.data_as(L._pd), nl.ctypes.data_as(L._pi64))
ev = int(res.counts[:, 2].sum())
print("dbg=%s R=%d gen %.1f ms sweep %.1f ms scan %.2f ms events %d (%.3g ev/s in the sweep)" %
      (os.environ.get("RQ_SWEEP_DBG", "0"), R, ms[0], ms[1], ms[2], ev, ev / (ms[1] * 1e-3)), flush=True)
