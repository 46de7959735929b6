"""Per-phase s_memtime split of the fused sweep (diagnostic build with -DRQ_PHASE_CLOCK,
loaded through RQ_SO_PATH).  Prints the fraction of wave time in each phase."""
import ctypes as C
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from redqueen_amd import _lib as L, engine, graphs
so = graphs.c3()
g = engine.Graph(so["src_id"], so["other_sources"], so["sink_ids"], so["edge_list"], so["end_time"])
lib = L.lib()
lib.rq_phase_clock.argtypes = [C.POINTER(C.c_ulonglong)]
for k in range(2):
    g.run("opt", q=so["q"], s=so["s"], n_rep=10000, ctrl_seed=0, world_seed=0, randomize=True, check=False)
    out = (C.c_ulonglong * 8)()
    rc = lib.rq_phase_clock(out)
    tot = sum(out[:6])
    names = ["A1 generation", "window + cut", "stage + rank sort", "B controller", "C aggregates", "rows"]
    print(rc, {n: round(out[q] / tot, 3) for q, n in enumerate(names)}, "per replica Mticks", tot / 1e4 / 1e6)
    print("refill iterations per replica %.1f, lanes stepping per iteration %.2f" % (out[6] / 1e4, out[7] / max(out[6], 1)))
