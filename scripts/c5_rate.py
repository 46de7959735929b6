"""C5 (10k followers, 500 Hawkes, T=1000) sweep throughput at 1 and 2 rounds of wave slots
(A/B of the replica work queue: RQ_FW_STATIC=1 restores one replica per wave)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from redqueen_amd import engine, graphs
so = graphs.c5()
g = engine.Graph(so["src_id"], so["other_sources"], so["sink_ids"], so["edge_list"], so["end_time"])
print("plan", g.run("opt", q=so["q"], s=so["s"], n_rep=2560, randomize=True, plan_only=True), flush=True)
for R in (2560, 5120):
    g.run("opt", q=so["q"], s=so["s"], n_rep=R, ctrl_seed=7, world_seed=7, randomize=True)
    torch.cuda.synchronize(); t0 = time.perf_counter()
    res = g.run("opt", q=so["q"], s=so["s"], n_rep=R, ctrl_seed=0, world_seed=0, randomize=True, check=False)
    torch.cuda.synchronize(); el = time.perf_counter() - t0
    ev = int(res.counts[:, 2].sum())
    print("R=%d: %.3f s, %.1f replicas/s, %.3g events/s, status %d" % (R, el, R / el, ev / el, int(res.status.max())),
          flush=True)
    del res
    torch.cuda.empty_cache()
