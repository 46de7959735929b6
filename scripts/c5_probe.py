"""C5 (10k followers, 500 Hawkes sources, T=1000): GPU vs oracle on two replicas + timing."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from redqueen_amd import engine, graphs
from oracle import oracle as O
so = graphs.c5()
g = engine.Graph(so["src_id"], so["other_sources"], so["sink_ids"], so["edge_list"], so["end_time"])
print("plan", g.run("opt", q=so["q"], s=so["s"], n_rep=256, randomize=True, plan_only=True), flush=True)
for R in (256, 1024):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    res = g.run("opt", q=so["q"], s=so["s"], n_rep=R, ctrl_seed=0, world_seed=0, randomize=True)
    torch.cuda.synchronize(); el = time.perf_counter() - t0
    ev = int(res.counts[:, 2].sum())
    print("R=%d: %.3f s, %.1f replicas/s, %.3g events/s, events/replica %.0f, status %d" %
          (R, el, R / el, ev / el, ev / R, int(res.status.max())), flush=True)
for u in (0, 1):
    sc = O.Scenario(dict(so, other_sources=[(n, dict(kw, seed=u + 99 * i)) for i, (n, kw) in
                                             enumerate(so["other_sources"])]), ("opt", u))
    t0 = time.perf_counter()
    (top, avg, r2, cnt), (t, dt, s) = O.engine_metrics(sc, (1,))
    m = res.metrics[u].cpu().numpy()
    print("oracle %.1fs" % (time.perf_counter() - t0), "match", bool(np.array_equal(m, np.asarray(list(top) + [avg, r2]))),
          int(res.counts[u, 2]), len(t), flush=True)
