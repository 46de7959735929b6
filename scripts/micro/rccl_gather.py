"""Cost of the bench step's exchange at world size 1 (RCCL group, in-process store):
all_gather_into_tensor alone, dist.gather_rows, and with the step's grid_means, timed
over 200 calls each with HIP events and wall clock."""
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from redqueen_amd import dist as D  # noqa: E402

dev = torch.device("cuda", 0)
dist.init_process_group("nccl", device_id=dev, store=dist.HashStore(), rank=0, world_size=1)
x = torch.rand(10000, 3, dtype=torch.float64, device=dev)
out = torch.empty_like(x)


def timed(name, fn, n=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    print("%-28s %8.1f us/call (events) %8.1f us/call (wall)" %
          (name, e0.elapsed_time(e1) * 1e3 / n, (time.perf_counter() - t0) * 1e6 / n), flush=True)


timed("all_gather_into_tensor", lambda: dist.all_gather_into_tensor(out, x))
timed("all_reduce 24 B", lambda: dist.all_reduce(x[0]))
timed("gather_rows(force)", lambda: D.gather_rows(x, 10000, force=True))
timed("gather_rows + grid_means", lambda: D.grid_means(D.gather_rows(x, 10000, force=True), 1, 10000))
timed("grid_means only", lambda: D.grid_means(x, 1, 10000))

# does the collective block the host until the GPU work queued before it is done?
for name, fn in (("all_gather_into_tensor", lambda: dist.all_gather_into_tensor(out, x)),
                 ("gather_rows(force)", lambda: D.gather_rows(x, 10000, force=True)),
                 ("async all_gather", lambda: dist.all_gather_into_tensor(out, x, async_op=True))):
    torch.cuda.synchronize()
    torch.cuda._sleep(200_000_000)     # ~0.1 s of GPU time queued ahead
    t0 = time.perf_counter()
    fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("%-28s host call %8.1f us, then sync %8.1f us" % (name, (t1 - t0) * 1e6, (t2 - t1) * 1e6),
          flush=True)
dist.destroy_process_group()
