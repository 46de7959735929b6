"""The real multi-process path through the engine: world-size-2
run_sharded with BOTH ranks on the one GPU of the test box and gloo for the
exchange (the driver's 8-GPU runs use nccl = RCCL over xGMI; only the transport
differs).  Each rank runs its replica window of every grid point of a q x s x
seeds grid and its half of a C3 batch; the gathered per-replica rows and the
fixed-order grid means must equal the unsharded single-process batch bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cases():
    from redqueen_amd import graphs
    c1 = graphs.readme()
    qs = np.logspace(-4, 7, 6)
    ss = [(1.0, 1.0), (0.5, 1.5)]
    grid_q = np.repeat(qs[None, :], len(ss), 0).ravel()
    grid_s = np.repeat(np.asarray(ss, dtype=np.float64), len(qs), 0)
    return [("c4", c1, dict(ctrl="opt", q=grid_q, s=grid_s, ctrl_seed=17, world_seed=17,
                            randomize=True, seed_mod=50, Ks=(1, 2)), len(grid_q), 50),
            ("c3", graphs.c3(), dict(ctrl="opt", q=graphs.c3()["q"], s=graphs.c3()["s"],
                                     ctrl_seed=3, world_seed=3, randomize=True, Ks=(1,)), 1, 96)]


def _graph(so):
    from redqueen_amd import engine
    return engine.Graph(so["src_id"], so["other_sources"], so["sink_ids"], so["edge_list"],
                        so["end_time"])


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from redqueen_amd import dist as D
    out = {}
    for name, so, kw, n_grid, n_rep in _cases():
        g = _graph(so)
        m, c, _ = D.run_sharded(g, n_grid, n_rep, **kw)
        out[name] = (m.cpu().numpy(), c.cpu().numpy(),
                     D.grid_means(m, n_grid, n_rep).cpu().numpy())
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def test_run_sharded_two_ranks_equals_unsharded():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from redqueen_amd import dist as D
    ctx = mp.get_context("spawn")
    qu = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, qu)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(qu.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for name, so, kw, n_grid, n_rep in _cases():
        res = _graph(so).run(n_rep=n_rep, **kw)
        m, c = res.metrics, res.counts
        gm = D.grid_means(m, n_grid, n_rep).cpu().numpy()
        for r in (0, 1):
            rm, rc, rg = got[r][name]
            assert np.array_equal(rm, m.cpu().numpy()), (name, r)
            assert np.array_equal(rc, c.cpu().numpy()), (name, r)
            assert np.array_equal(rg, gm), (name, r)


def _bench_worker(rank, world, port, q):
    """bench.py's own step function (make_step) on this rank, gloo for the exchange."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    import torch.distributed as dist
    import bench
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = {}
    for wl, R in (("c4", 6), ("c3", 48)):
        so, _ = bench.workload(wl)
        step, n, _ = bench.make_step(wl, _graph(so), so, R, world, rank, torch.device("cuda", 0), (1,))
        _, means = step(1)
        out[wl] = (n, means.cpu().numpy())
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def test_bench_step_two_ranks_equals_one():
    """bench.py's step at world size 2 (C4: each rank the replica window of every grid
    point; C3: each rank its own replicas) gathers the same rows and so computes the
    same ensemble / per-grid-point means, bit for bit, as one rank running the whole
    step (the driver's N-GPU bench runs exactly this step over RCCL)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import bench
    ctx = mp.get_context("spawn")
    qu = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_bench_worker, args=(r, 2, port, qu)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(qu.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for wl, R in (("c4", 6), ("c3", 48)):
        so, _ = bench.workload(wl)
        step, n, _ = bench.make_step(wl, _graph(so), so, 2 * R, 1, 0, torch.device("cuda", 0), (1,))
        _, means = step(1)
        for r in (0, 1):
            assert got[r][wl][0] == n
            assert np.array_equal(got[r][wl][1], means.cpu().numpy()), (wl, r)
