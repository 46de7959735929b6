"""C4 shard balance on one GPU: the 8 shards an 8-GPU run would take, timed one
after another with the library's HIP-event kernel timers (rq_timing), for the
round-2 contiguous cut of the flattened (grid point, replica) space and for the
grid-balanced replica windows dist.run_sharded now uses.

    python scripts/c4_shard_balance.py [--reps 3] > shard_balance.json
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--n-rep", type=int, default=1000)
    ap.add_argument("--world", type=int, default=8)
    a = ap.parse_args()
    from redqueen_amd import _lib as L
    from redqueen_amd import dist, engine, graphs
    so = graphs.readme()
    g = engine.Graph(so["src_id"], so["other_sources"], so["sink_ids"], so["edge_list"], so["end_time"])
    grid = graphs.c4_grid()
    qs = np.asarray([q for q, _ in grid])
    sm = np.asarray([[s1, s2] for _, (s1, s2) in grid])
    n_rep, W = a.n_rep, a.world
    kw = dict(q=qs, s=sm, ctrl_seed=0, world_seed=0, randomize=True, Ks=(1,), seed_mod=n_rep,
              check=False)
    lib = L.lib()

    def shard_kw(mode, k):
        if mode == "contiguous":
            lo, hi = dist.shard(len(grid) * n_rep, W, k)
            return dict(replica0=lo, n_local=hi - lo)
        lo, hi = dist.grid_shard(n_rep, W, k)
        return dict(rep_lo=lo, rep_cnt=hi - lo)

    out = {"workload": "C4: README graph, 64 q x 4 s x %d replicas, %d shards" % (n_rep, W)}
    for mode in ("contiguous", "grid"):
        for k in range(W):   # warm every shape once (code objects, workspace)
            g.run("opt", n_rep=n_rep, **shard_kw(mode, k), **kw)
        torch.cuda.synchronize()
        sweep, scan, events = [], [], []
        for k in range(W):
            lib.rq_timing(1)
            ev = 0
            for _ in range(a.reps):
                r = g.run("opt", n_rep=n_rep, **shard_kw(mode, k), **kw)
                ev = int(r.counts[:, 2].sum().item())
            torch.cuda.synchronize()
            ms = np.zeros(5)
            nl = np.zeros(5, dtype=np.int64)
            lib.rq_timing_read(ms.ctypes.data_as(L._pd), nl.ctypes.data_as(L._pi64))
            lib.rq_timing(0)
            sweep.append(ms[1] / a.reps)
            scan.append(ms[2] / a.reps)
            events.append(ev)
        tot = [s + c for s, c in zip(sweep, scan)]
        out[mode] = {"sweep_ms": sweep, "scan_ms": scan, "events": events,
                     "max_over_mean_ms": max(tot) / (sum(tot) / W),
                     "max_over_mean_events": max(events) / (sum(events) / W)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
