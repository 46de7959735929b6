"""Multi-GPU replica sharding.

One process per GPU.  A batch is an (n_grid x n_rep) grid of replicas with
global ids i = g * n_rep + r.  Rank k owns the replica window
[n_rep * k / world, n_rep * (k + 1) / world) of EVERY grid point (the engine's
rq_batch_desc.rep_lo / rep_cnt), so each rank sees the whole q range: the work
per replica varies strongly with q (C4: ~3.9k events per replica at the smallest
q against ~2.1k at the largest), and a cut of the flattened (g, r) space into
contiguous blocks would hand one rank all the expensive grid points.  Seeds and
grid point follow the GLOBAL id, so a replica's outputs do not depend on the
number of GPUs.  The only exchange is one all-gather of the per-replica metric
rows at the end (RCCL over xGMI with the nccl backend, gloo on CPU), after which
every rank reduces per grid point in fixed replica order -- bit-identical for
1, 2, 4, 8 GPUs.

The reference's counterpart is the mp.Pool / mp.Queue fan-out of
utils.calc_q_capacity_iter (utils.py:463-468) and opt_runs.run_inference_queue
(opt_runs.py:560-646).
"""
import torch
import torch.distributed as dist


def shard(n_total, world, rank):
    """Contiguous [start, end) of `n_total` items owned by `rank`."""
    return n_total * rank // world, n_total * (rank + 1) // world


def grid_shard(n_rep, world, rank):
    """The replica window [lo, hi) of every grid point that `rank` owns."""
    return shard(n_rep, world, rank)


def _world_rank(world, rank, group):
    if world is None:
        world = dist.get_world_size(group) if dist.is_initialized() else 1
    if rank is None:
        rank = dist.get_rank(group) if dist.is_initialized() and world > 1 else 0
    return world, rank


def _all_gather_padded(local, m, world, group):
    # gloo exchanges host tensors (a CPU-only or test group); nccl = RCCL over xGMI
    dev = torch.device("cpu") if dist.get_backend(group) == "gloo" else local.device
    pad = torch.zeros((m,) + tuple(local.shape[1:]), dtype=local.dtype, device=dev)
    pad[:local.shape[0]] = local.to(dev)
    out = torch.empty((world * m,) + tuple(local.shape[1:]), dtype=local.dtype, device=dev)
    dist.all_gather_into_tensor(out, pad, group=group)
    return out


def gather_rows(local, n_total, world=None, rank=None, group=None, force=False):
    """All-gather per-replica rows [n_local, C] of every rank into [n_total, C]
    in global replica order (ranks own contiguous, possibly unequal, shards).
    ``force``: run the collective even for a world of one (bench.py --dist, the
    world-size-1 RCCL test) instead of returning ``local``."""
    world, rank = _world_rank(world, rank, group)
    if world == 1 and not force:
        return local
    sizes = [shard(n_total, world, r)[1] - shard(n_total, world, r)[0] for r in range(world)]
    m = max(sizes)
    out = _all_gather_padded(local, m, world, group)
    return torch.cat([out[r * m:r * m + sizes[r]] for r in range(world)], 0).to(local.device)


def gather_grid_rows(local, n_grid, n_rep, world=None, rank=None, group=None, force=False):
    """All-gather per-replica rows of grid_shard()s: rank k holds [n_grid * cnt_k, C]
    (grid point major, its replica window minor); returns [n_grid * n_rep, C] in
    global replica order i = g * n_rep + r.  ``force`` as in gather_rows."""
    world, rank = _world_rank(world, rank, group)
    if world == 1 and not force:
        return local
    wins = [grid_shard(n_rep, world, r) for r in range(world)]
    m = n_grid * max(hi - lo for lo, hi in wins)
    out = _all_gather_padded(local, m, world, group)
    tail = tuple(local.shape[1:])
    parts = [out[r * m:r * m + n_grid * (hi - lo)].reshape((n_grid, hi - lo) + tail)
             for r, (lo, hi) in enumerate(wins)]
    # windows are consecutive in r: concatenating along the replica axis is global order
    return torch.cat(parts, 1).reshape((n_grid * n_rep,) + tail).to(local.device)


def grid_means(rows, n_grid, n_rep):
    """Per-grid-point means of gathered rows [n_grid*n_rep, C].  One reduction
    launch: torch's sum over a dimension uses no atomics and a reduction order fixed
    by the shape and device, so the result depends only on the gathered rows --
    bit-identical on every rank and however the replicas were sharded."""
    x = rows.reshape(n_grid, n_rep, -1).to(torch.float64)
    # divide by a tensor: torch's tensor / python-scalar multiplies by the reciprocal
    return x.sum(1) / torch.full((), float(n_rep), dtype=torch.float64, device=x.device)


def run_sharded(graph, n_grid, n_rep, world=None, rank=None, group=None, force=False, **run_kw):
    """Run this rank's shard of an (n_grid x n_rep) batch -- the same replica window
    of every grid point -- and return the gathered per-replica metrics
    [n_grid*n_rep, nK+2] and counts [n_grid*n_rep, 4] (and this rank's BatchResult).
    ``force``: exchange through the collective even for a world of one."""
    world, rank = _world_rank(world, rank, group)
    from . import _lib as L
    L.warn_hw_queues(dist.is_initialized() and dist.get_backend(group) != "gloo")
    lo, hi = grid_shard(n_rep, world, rank)
    if hi > lo:
        res = graph.run(n_rep=n_rep, rep_lo=lo, rep_cnt=hi - lo, **run_kw)
        lm, lc = res.metrics, res.counts
    else:   # more ranks than replicas per grid point: this rank only takes part in the exchange
        res = None
        nk = len(run_kw.get("Ks", (1,)))
        dev = torch.device("cuda", torch.cuda.current_device())
        lm = torch.empty((0, nk + 2), dtype=torch.float64, device=dev)
        lc = torch.empty((0, 4), dtype=torch.int64, device=dev)
    m = gather_grid_rows(lm, n_grid, n_rep, world, rank, group, force)
    c = gather_grid_rows(lc, n_grid, n_rep, world, rank, group, force)
    return m, c, res
