"""Per-phase s_memtime split of rq_rp_fast's batch loop on the 256 exported C3
dataframes (diagnostic build with -DRQ_PHASE_CLOCK via RQ_SO_PATH, RQ_CLK_REPLAY=1)."""
import ctypes as C
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ["RQ_CLK_REPLAY"] = "1"
import torch
from redqueen_amd import _lib as L, engine, graphs, utils
so = graphs.c3()
g = engine.Graph(so["src_id"], so["other_sources"], so["sink_ids"], so["edge_list"], so["end_time"])
r2 = g.run("opt", q=so["q"], s=so["s"], n_rep=256, ctrl_seed=0, world_seed=0, randomize=True, event_log=True)
ro, cols = r2.log_columns()
off = torch.from_numpy(ro).cuda()
lib = L.lib()
lib.rq_phase_clock.argtypes = [C.POINTER(C.c_ulonglong)]
names = ["top+load issue+barrier1", "C1 list walk", "A tickets+scan", "barriers 2-4, B, lists",
         "D1 scans", "C2 ranks", "prep next (hash)", "D2 barrier5+totals+stores"]
nb = (int(ro[-1]) + 2047) // 2048
for k in range(3):
    out = (C.c_ulonglong * 8)()
    lib.rq_phase_clock(out)   # clear
    m, c = utils.replay_columns(cols["t"], cols["src_id"], cols["sink_id"], None, off, so["src_id"],
                                so["end_time"], (1,))
    torch.cuda.synchronize()
    rc = lib.rq_phase_clock(out)
    tot = sum(out)
    # per wave per batch (16 waves per workgroup)
    print(rc, {n: round(out[q] / tot, 3) for q, n in enumerate(names)},
          "ticks per wave-batch %.0f" % (tot / (16.0 * nb)))
