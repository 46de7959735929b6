"""A/B of the replay kernels (RQ_SO_PATH selects the build): 256 C3 dfs as one batch
and one C3 df, kernel time from the library's HIP events."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from redqueen_amd import _lib as L  # noqa: E402
from redqueen_amd import engine, graphs, utils  # noqa: E402


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    ms = np.zeros(5)
    nl = np.zeros(5, dtype=np.int64)
    L.lib().rq_timing(1)
    for _ in range(reps):
        out = fn()
    torch.cuda.synchronize()
    L.lib().rq_timing_read(ms.ctypes.data_as(L._pd), nl.ctypes.data_as(L._pi64))
    L.lib().rq_timing(0)
    return out, ms / reps


so = graphs.c3()
g = engine.Graph(so["src_id"], so["other_sources"], so["sink_ids"], so["edge_list"], so["end_time"])
NDF = int(os.environ.get("RQ_AB_NDF", "256"))   # dataframes in the batch
r2 = g.run("opt", q=so["q"], s=so["s"], n_rep=NDF, ctrl_seed=0, world_seed=0, randomize=True, event_log=True)
ro, cols = r2.log_columns()
off = torch.from_numpy(ro).cuda()
nrow = int(ro[-1])
res = {"so": os.environ.get("RQ_SO_PATH", "librq.so")}
for tag, ck in (("batch", False),) + ((("batch_chunked", True),) if NDF <= 256 else ()):
    if ck:
        os.environ["RQ_RP_CHUNK"] = "1"
    (m, c), ms = timed(lambda: utils.replay_columns(cols["t"], cols["src_id"], cols["sink_id"], cols["event_id"],
                                                     off, so["src_id"], so["end_time"], (1,), chunked=ck), 5)
    os.environ.pop("RQ_RP_CHUNK", None)
    res[tag] = {"ms_replay": ms[3], "ms_scan": ms[2], "TBps_32B": 32 * nrow / (ms[3] + ms[2]) / 1e9,
                "equal": bool(torch.equal(m, r2.metrics))}
a0, a1 = int(ro[0]), int(ro[1])
one = {k: v[a0:a1].contiguous() for k, v in cols.items()}
(m, c), ms = timed(lambda: utils.replay_columns(one["t"], one["src_id"], one["sink_id"], one["event_id"], None,
                                                 so["src_id"], so["end_time"], (1,)), 5)
res["one_df"] = {"ms_replay": ms[3], "ms_scan": ms[2], "equal": bool(torch.equal(m[0], r2.metrics[0]))}
print(json.dumps(res), flush=True)
