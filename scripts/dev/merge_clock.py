"""Phase split of rq_merge_streams on C5 (diagnostic -DRQ_PHASE_CLOCK build loaded
through RQ_SO_PATH): per-round s_memtime sums of one thread per block."""
import ctypes as C
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: F401
from redqueen_amd import _lib as L, engine, graphs
WL = os.environ.get("RQ_WL", "c5")
so = graphs.c5() if WL == "c5" else graphs.c3()
g = engine.Graph(so["src_id"], so["other_sources"], so["sink_ids"], so["edge_list"], so["end_time"])
lib = L.lib()
lib.rq_phase_clock.argtypes = [C.POINTER(C.c_ulonglong)]
os.environ["RQ_CLK_MERGE"] = "1"
R = 1024 if WL == "c5" else 10000
for k in range(2):
    g.run("opt", q=so["q"], s=so["s"], n_rep=R, ctrl_seed=0, world_seed=0, randomize=True, check=False)
    torch.cuda.synchronize()
    out = (C.c_ulonglong * 8)()
    rc = lib.rq_phase_clock(out)
    names = {0: "walk", 1: "barrier after walk", 2: "bucket scan", 3: "scatter", 6: "rank + write"}
    tot = sum(out[q] for q in names)
    print(rc, {n: round(out[q] / max(tot, 1), 3) for q, n in names.items()},
          "rounds/replica %.1f retries/replica %.2f ticks/round %.0f" % (out[4] / R, out[5] / R, tot / max(out[4], 1)),
          flush=True)
