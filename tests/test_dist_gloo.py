"""Replica sharding + all-gather + ordered per-grid reduction over gloo, world 2/3."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from redqueen_amd import dist as D

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rows(a, b, C=5):
    i = torch.arange(a, b, dtype=torch.float64)[:, None]
    return torch.sin(i * 1.37 + torch.arange(C, dtype=torch.float64)) * (i + 1)


def _grid_rows(n_grid, n_rep, lo, hi):
    """Rows of the replica window [lo, hi) of every grid point, grid point major."""
    ids = [g * n_rep + r for g in range(n_grid) for r in range(lo, hi)]
    return torch.cat([_rows(i, i + 1) for i in ids], 0) if ids else _rows(0, 0)


def _worker(rank, world, port, n_grid, n_rep, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    R = n_grid * n_rep
    a, b = D.shard(R, world, rank)
    rows = D.gather_rows(_rows(a, b), R)
    means = D.grid_means(rows, n_grid, n_rep)
    lo, hi = D.grid_shard(n_rep, world, rank)
    grows = D.gather_grid_rows(_grid_rows(n_grid, n_rep, lo, hi), n_grid, n_rep)
    assert (grows == rows).all()
    q.put((rank, rows.numpy(), means.numpy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n_grid,n_rep", [(2, 3, 5), (3, 2, 7), (2, 1, 1), (3, 4, 2)])
def test_sharded_gather_is_rank_count_independent(world, n_grid, n_rep):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_grid, n_rep, q))
             for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    R = n_grid * n_rep
    full = _rows(0, R).numpy()
    ref_means = D.grid_means(torch.from_numpy(full), n_grid, n_rep).numpy()
    for _, rows, means in out:
        assert (rows == full).all()
        assert (means == ref_means).all()


def test_shards_cover_exactly():
    for R in (1, 7, 64, 1001):
        for w in (1, 2, 3, 8):
            cov = []
            for r in range(w):
                a, b = D.shard(R, w, r)
                cov += list(range(a, b))
            assert cov == list(range(R))


def test_grid_shards_see_every_grid_point():
    """grid_shard: every rank owns the same replica window of every grid point, the
    windows tile [0, n_rep), and per-rank replica counts differ by at most n_grid."""
    for n_grid, n_rep in ((1, 10), (64, 1000), (6, 7), (3, 2)):
        for w in (1, 2, 3, 8):
            wins = [D.grid_shard(n_rep, w, r) for r in range(w)]
            assert wins[0][0] == 0 and wins[-1][1] == n_rep
            assert all(wins[k][1] == wins[k + 1][0] for k in range(w - 1))
            sizes = [n_grid * (hi - lo) for lo, hi in wins]
            assert max(sizes) - min(sizes) <= n_grid


def test_hw_queue_requirement_without_the_callers_help():
    """the engine's two pipeline streams need >= 8 HIP hardware
    queues beside an RCCL group.  Importing the package raises GPU_MAX_HW_QUEUES to 8
    when the caller left it unset (HIP not up yet); a caller who set fewer is warned once
    by dist.run_sharded under a live nccl group (gloo groups exchange host tensors)."""
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k != "GPU_MAX_HW_QUEUES"}
    out = subprocess.run([sys.executable, "-c",
                          "import os, redqueen_amd._lib as L; "
                          "print(os.environ['GPU_MAX_HW_QUEUES'], L.HW_QUEUES, L.HW_QUEUES_SET_BY_PACKAGE)"],
                         env=env, capture_output=True, text=True, cwd=ROOT, timeout=300)
    assert out.returncode == 0, out.stderr
    assert out.stdout.split() == ["8", "8", "True"]
    env["GPU_MAX_HW_QUEUES"] = "4"   # the caller's own choice is kept, and reported
    out = subprocess.run([sys.executable, "-c",
                          "import os, redqueen_amd._lib as L; "
                          "print(os.environ['GPU_MAX_HW_QUEUES'], L.HW_QUEUES_SET_BY_PACKAGE, "
                          "L.hw_queue_advice(True) is not None, L.hw_queue_advice(False))"],
                         env=env, capture_output=True, text=True, cwd=ROOT, timeout=300)
    assert out.stdout.split() == ["4", "False", "True", "None"], out.stdout + out.stderr
    from redqueen_amd import _lib as L
    assert L.hw_queue_advice(True, 8) is None and L.hw_queue_advice(True, 32) is None
    assert "GPU_MAX_HW_QUEUES=8" in L.hw_queue_advice(True, 4)
    assert "unset" in L.hw_queue_advice(True, None)
