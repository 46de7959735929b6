"""Multi-GPU replica sharding.

One process per GPU.  The flattened (grid point, replica) index space
i = g * n_rep + r is cut into contiguous shards, one per rank; every rank runs
its shard through the engine (seeds and grid point follow the GLOBAL index,
so a replica's outputs do not depend on the number of GPUs).  The only
exchange is one all-gather of the per-replica metric rows at the end (RCCL
over xGMI with the nccl backend, gloo on CPU), after which every rank reduces
per grid point in fixed replica order -- bit-identical for 1, 2, 4, 8 GPUs.

The reference's counterpart is the mp.Pool / mp.Queue fan-out of
utils.calc_q_capacity_iter (utils.py:463-468) and opt_runs.run_inference_queue
(opt_runs.py:560-646).
"""
import torch
import torch.distributed as dist


def shard(n_total, world, rank):
    """Contiguous [start, end) of replica ids owned by `rank`."""
    return n_total * rank // world, n_total * (rank + 1) // world


def gather_rows(local, n_total, world=None, rank=None, group=None):
    """All-gather per-replica rows [n_local, C] of every rank into [n_total, C]
    in global replica order (ranks own contiguous, possibly unequal, shards)."""
    if world is None:
        world = dist.get_world_size(group) if dist.is_initialized() else 1
    if world == 1:
        return local
    rank = dist.get_rank(group) if rank is None else rank
    sizes = [shard(n_total, world, r)[1] - shard(n_total, world, r)[0] for r in range(world)]
    m = max(sizes)
    # gloo exchanges host tensors (a CPU-only or test group); nccl = RCCL over xGMI
    dev = torch.device("cpu") if dist.get_backend(group) == "gloo" else local.device
    pad = torch.zeros((m,) + tuple(local.shape[1:]), dtype=local.dtype, device=dev)
    pad[:local.shape[0]] = local.to(dev)
    out = torch.empty((world * m,) + tuple(local.shape[1:]), dtype=local.dtype, device=dev)
    dist.all_gather_into_tensor(out, pad, group=group)
    return torch.cat([out[r * m:r * m + sizes[r]] for r in range(world)], 0).to(local.device)


def grid_means(rows, n_grid, n_rep):
    """Per-grid-point means of gathered rows [n_grid*n_rep, C].  One reduction
    launch: torch's sum over a dimension uses no atomics and a reduction order fixed
    by the shape and device, so the result depends only on the gathered rows --
    bit-identical on every rank and however the replicas were sharded."""
    x = rows.reshape(n_grid, n_rep, -1).to(torch.float64)
    return x.sum(1) / n_rep


def run_sharded(graph, n_grid, n_rep, world=None, rank=None, group=None, **run_kw):
    """Run this rank's shard of an (n_grid x n_rep) batch and return the gathered
    per-replica metrics [n_grid*n_rep, nK+2] and counts [n_grid*n_rep, 4]."""
    if world is None:
        world = dist.get_world_size(group) if dist.is_initialized() else 1
        rank = dist.get_rank(group) if dist.is_initialized() else 0
    R = n_grid * n_rep
    a, b = shard(R, world, rank)
    if b > a:
        res = graph.run(n_rep=n_rep, replica0=a, n_local=b - a, **run_kw)
        lm, lc = res.metrics, res.counts
    else:   # more ranks than replicas: this rank only takes part in the exchange
        res = None
        nk = len(run_kw.get("Ks", (1,)))
        dev = torch.device("cuda", torch.cuda.current_device())
        lm = torch.empty((0, nk + 2), dtype=torch.float64, device=dev)
        lc = torch.empty((0, 4), dtype=torch.int64, device=dev)
    m = gather_rows(lm, R, world, rank, group)
    c = gather_rows(lc, R, world, rank, group)
    return m, c, res
