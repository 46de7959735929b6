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


def _rccl_worker(q):
    """A fresh process: a world-size-1 nccl (= RCCL) group bound to the device before
    any other GPU work, then every exchange of redqueen_amd.dist on device tensors
    through it (force=True skips the world == 1 shortcut)."""
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    import torch.distributed as dist
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", device_id=dev, store=dist.HashStore(), rank=0,
                            world_size=1)
    assert dist.get_backend() == "nccl"
    from redqueen_amd import dist as D
    import bench
    out = {}
    x = torch.arange(7 * 3, dtype=torch.float64, device=dev).reshape(7, 3) / 3.0
    out["x"] = x.cpu().numpy()
    pad = D._all_gather_padded(x, 9, 1, None)
    assert pad.is_cuda
    out["padded"] = pad.cpu().numpy()
    rows = D.gather_rows(x, 7, force=True)
    assert rows.is_cuda
    out["rows"] = rows.cpu().numpy()
    gr = D.gather_grid_rows(x[:6], 2, 3, force=True)
    assert gr.is_cuda
    out["grid_rows"] = gr.cpu().numpy()
    for name, so, kw, n_grid, n_rep in _cases():
        m, c, _ = D.run_sharded(_graph(so), n_grid, n_rep, force=True, **kw)
        out[name] = (m.cpu().numpy(), c.cpu().numpy())
    for wl, R in (("c4", 6), ("c3", 48)):
        so, _ = bench.workload(wl)
        step, n, _ = bench.make_step(wl, _graph(so), so, R, 1, 0, dev, (1,), force=True)
        _, means = step(1)
        out["bench_" + wl] = means.cpu().numpy()
    torch.cuda.synchronize()
    dist.destroy_process_group()
    q.put(out)


def test_rccl_world_one_exchanges_on_device():
    """RCCL executes: a child process with a world-size-1 nccl group drives
    _all_gather_padded, gather_rows, gather_grid_rows, run_sharded and bench's own step
    through the collective on device tensors; every result equals its input (the
    exchange of one rank is the identity) and the engine's direct run, bit for bit."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import bench
    ctx = mp.get_context("spawn")
    qu = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(qu,))
    p.start()
    got = qu.get(timeout=300)
    p.join(timeout=120)
    assert p.exitcode == 0
    x = got["x"]
    assert np.array_equal(got["padded"][:7], x) and not got["padded"][7:].any()
    assert np.array_equal(got["rows"], x)
    assert np.array_equal(got["grid_rows"], x[:6])
    for name, so, kw, n_grid, n_rep in _cases():
        res = _graph(so).run(n_rep=n_rep, **kw)
        assert np.array_equal(got[name][0], res.metrics.cpu().numpy()), name
        assert np.array_equal(got[name][1], res.counts.cpu().numpy()), name
    dev = torch.device("cuda", 0)
    for wl, R in (("c4", 6), ("c3", 48)):
        so, _ = bench.workload(wl)
        step, n, _ = bench.make_step(wl, _graph(so), so, R, 1, 0, dev, (1,))
        _, means = step(1)
        assert np.array_equal(got["bench_" + wl], means.cpu().numpy()), wl
