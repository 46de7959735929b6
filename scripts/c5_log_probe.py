"""C5 with the event log (the fast general sweep writes it): sweep time and log bytes."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from redqueen_amd import engine, graphs
so = graphs.c5()
g = engine.Graph(so["src_id"], so["other_sources"], so["sink_ids"], so["edge_list"], so["end_time"])
R = int(sys.argv[1]) if len(sys.argv) > 1 else 1280
kw = dict(q=so["q"], s=so["s"], n_rep=R, ctrl_seed=0, world_seed=0, randomize=True, Ks=(1,))
print("plan", g.run("opt", event_log=True, plan_only=True, **kw), flush=True)
for ev in (False, True, True):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    res = g.run("opt", event_log=ev, **kw)
    torch.cuda.synchronize(); el = time.perf_counter() - t0
    n = int(res.counts[:, 2].sum())
    print("event_log=%s: %.3f s, %.1f replicas/s, %.3g events/s, log %.2f GB, status %d" %
          (ev, el, R / el, n / el, 12 * n / 1e9 if ev else 0.0, int(res.status.max())), flush=True)
