"""Per-step host/GPU timing of the bench step (diagnostic; not part of the bench)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from redqueen_amd import engine, graphs
from redqueen_amd import _lib as L
so = graphs.c3()
g = engine.Graph(so["src_id"], so["other_sources"], so["sink_ids"], so["edge_list"], so["end_time"])
R = 10000
for k in range(12):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = g.run("opt", q=so["q"], s=so["s"], n_rep=R, ctrl_seed=k * R, world_seed=k * R,
                randomize=True, Ks=(1,), check=False)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("step %d: enqueue %.2f ms, total %.2f ms" % (k, (t1 - t0) * 1e3, (t2 - t0) * 1e3), flush=True)
t0 = time.perf_counter()
for k in range(10):
    res = g.run("opt", q=so["q"], s=so["s"], n_rep=R, ctrl_seed=k * R, world_seed=k * R,
                randomize=True, Ks=(1,), check=False)
torch.cuda.synchronize()
print("10 back-to-back: %.2f ms/step" % ((time.perf_counter() - t0) * 1e2))
L.lib().rq_timing(1)
t0 = time.perf_counter()
for k in range(10):
    res = g.run("opt", q=so["q"], s=so["s"], n_rep=R, ctrl_seed=k * R, world_seed=k * R,
                randomize=True, Ks=(1,), check=False)
torch.cuda.synchronize()
print("10 back-to-back, kernel timing on: %.2f ms/step" % ((time.perf_counter() - t0) * 1e2))
L.lib().rq_timing(0)
t0 = time.perf_counter()
tot = torch.zeros((), dtype=torch.int64, device="cuda")
for k in range(10):
    res = g.run("opt", q=so["q"], s=so["s"], n_rep=R, ctrl_seed=k * R, world_seed=k * R,
                randomize=True, Ks=(1,), check=False)
    m = res.metrics.mean(0)
    tot += res.counts[:, 2].sum()
torch.cuda.synchronize()
print("10 back-to-back + torch reductions: %.2f ms/step" % ((time.perf_counter() - t0) * 1e2))
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tot = torch.zeros((), dtype=torch.int64, device="cuda")
    for k in range(10):
        res = g.run("opt", q=so["q"], s=so["s"], n_rep=R, ctrl_seed=k * R, world_seed=k * R,
                    randomize=True, Ks=(1,), check=False)
        m = res.metrics.mean(0)
        tot += res.counts[:, 2].sum()
    torch.cuda.synchronize()
    print("explicit stream + torch reductions: %.2f ms/step" % ((time.perf_counter() - t0) * 1e2))
t0 = time.perf_counter()
for k in range(10):
    res = g.run("opt", q=so["q"], s=so["s"], n_rep=R, ctrl_seed=k * R, world_seed=k * R,
                randomize=True, Ks=(1,), check=False)
    torch.cuda.synchronize()
    m = res.metrics.mean(0)
    tot += res.counts[:, 2].sum()
torch.cuda.synchronize()
print("sync then reductions: %.2f ms/step" % ((time.perf_counter() - t0) * 1e2))
