#!/usr/bin/env python
"""bench.py -- RedQueen Monte-Carlo throughput on MI355X.

Metric (BASELINE.json): RedQueen replicas/s (+ simulated events/s) per node on
the 1000-sink synthetic graph, 1/2/4/8 GPUs.  Workload = config C3 ("syn1k",
SURVEY.md 8(d)): 1000 followers, 50 other sources (25 Poisson2 rate 1 + 25
Hawkes l_0=1 alpha=1 beta=10), degree 5, T=100, q=1e6, s_i=1; every replica
has its own world (randomize_other_sources) and RedQueen seed.

One step = one batch of --replicas replicas PER GPU (weak scaling) through the
whole hot path: arrival-stream generation, RedQueen sweep, metric scan
(time_in_top_k K=1, average_rank, int_r_2, num_events, world_events), then for
N>1 the RCCL all-gather of the per-replica metric rows and the ensemble means.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import json
import os
import sys
import time

# The engine pipelines a batch's chunks on two HIP streams (rq_run_batch) and an RCCL
# group adds its own; with HIP's default of 4 hardware queues per process the engine's two
# streams then share one queue and the pipeline serialises (C3: 2.93 -> 3.42 ms per step
# with a world-size-1 group, 2.97 ms with 8 queues; profiles/r05_dist_queues.txt).  Set
# before HIP initialises; gpurun allows up to 32.
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md); 6.29 TB/s measured copy
N_CU = 256              # MI355X: 8 XCDs x 32 CUs
# algorithmic bytes per unit (DESIGN.md "Roofline accounting")
SWEEP_B_PER_WALL_EVENT = 8      # read one arrival time (the windowed general sweep)
MRG_SWEEP_B_PER_WALL_EVENT = 10  # read one merged (t f64, stream u16) entry
MERGE_B_PER_WALL_EVENT = 18     # rq_merge_streams: read the arrival (8), write the entry (10)
SWEEP_B_PER_ROW = 24            # write t f64 + sumR f64 + nvalid u32 + cnt[K=1] u32
SCAN_B_PER_ROW = 24             # read the same row back
GEN_B_PER_WALL_EVENT = 8        # write one arrival time


def e2e_gbs(events_per_s):
    return SWEEP_B_PER_ROW * events_per_s / 1e9


def workload(name):
    from redqueen_amd import graphs
    if name == "c4":
        return graphs.readme(), ("C4: README graph (3 sources, 3 sinks), T=100, RedQueen x 64 q "
                                 "(logspace(-4, 7)) x 4 s ((1,1), (0.5,1.5), (1.5,0.5), (1,0.25)), "
                                 "grid-window sharded, per-grid-point means")
    if name == "c3":
        return graphs.c3(), ("C3 syn1k: 1000 followers, 50 sources (25 Poisson2 rate 1 + 25 Hawkes "
                             "l0=1 a=1 b=10), degree 5, T=100, q=1e6, s=1, RedQueen, "
                             "randomized worlds")
    if name == "c2":
        return graphs.readme(), "C2: README graph (3 sources, 3 sinks), T=100, RedQueen"
    if name == "c5":
        return graphs.c5(), ("C5: 10k followers, 500 Hawkes (l0=0.5 a=1 b=2), degree 5, T=1000, "
                             "q=1e8, RedQueen, randomized worlds")
    raise SystemExit("unknown workload " + name)


def cpu_baseline(so, n_threads, sample, Ks=(1,), grid=None):
    """Oracle (C port of the reference algorithm + Appendix-B metrics) on host cores.
    grid: [(q, s)] -- the sample is spread evenly over these grid points (C4)."""
    from oracle import oracle as O
    pts = [dict(so)] if not grid else [dict(so, q=float(q), s=np.asarray(s, dtype=float))
                                        for q, s in grid]
    per = max(1, sample // len(pts))
    t0 = time.perf_counter()
    tot = 0
    for k, d in enumerate(pts):
        out, cnt, t = O.engine_batch(O.Scenario(d, ("opt", 0)), per, k * per, True, Ks, n_threads)
        tot += t
    el = time.perf_counter() - t0
    return per * len(pts) / el, tot / el, el


def pmc_summary_paths(workload):
    """Committed PMC summaries of this workload, newest round first."""
    import glob
    return sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_%s_pmc_summary.json" % workload)),
                  reverse=True)


def ref_cpu_baseline(workload):
    """The reference itself (pure Python, multiprocessing over replicas) timed in the
    build container by scripts/ref_cpu_baseline.py -- /root/reference does not exist on
    the GPU box, so the measured line is read from the committed profile."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_ref_cpu_baseline.jsonl")),
                       reverse=True):
        for ln in open(path):
            try:
                d = json.loads(ln)
            except ValueError:
                continue
            if d.get("config") == workload:
                return {"value": d["replicas_per_s"], "unit": "replicas/s", "cores": d["procs"],
                        "kind": "reference",
                        "sample": "%d %s replicas of the reference's Manager.run_dynamic + "
                                  "time_in_top_k/average_rank, multiprocessing.Pool(%d), %.0f s "
                                  "(measured in the build container, %s)" %
                                  (d["replicas"], workload.upper(), d["procs"], d["wall_s"],
                                   os.path.relpath(path, ROOT))}
    return None


def pmc_traffic(workload, R, plan):
    """HBM bytes per sweep launch from the committed rocprofv3 PMC summary of this
    same command (scripts/gpu_pmc.sh -> scripts/pmc_summary.py: FETCH_SIZE x2 per
    the gfx950 correction + WRITE_SIZE), when workload, replicas and plan match AND
    its build stamp is the loaded library's (librq.so + sources sha256)."""
    from redqueen_amd import _lib as L
    stamp = L.build_stamp()
    for path in pmc_summary_paths(workload):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        meta = d.get("_meta", {})
        if meta.get("workload") != workload or meta.get("replicas") != R or \
                meta.get("variant") != plan["variant"]:
            continue
        if any(meta.get(k) != v for k, v in stamp.items()):
            continue
        for k, v in d.items():
            if k.startswith("rq_sweep") and "hbm_write_bytes" in v and "hbm_read_bytes" in v:
                issue = {q: v[q] for q in ("frac_active_inst", "frac_wait_any", "frac_wait_inst",
                                           "wave_slot_occupancy") if q in v}
                c = v.get("counters", {})
                # VALU issue ceiling: one wave64 VALU instruction per 2 cycles per SIMD
                # (MI355X_MICROARCH.md), 4 SIMDs per CU, over the launch's cycles on one
                # XCD (GRBM_GUI_ACTIVE is summed over the 8 XCDs)
                if c.get("SQ_INSTS_VALU") and c.get("GRBM_GUI_ACTIVE"):
                    cyc = c["GRBM_GUI_ACTIVE"] / 8.0
                    issue["valu_insts"] = c["SQ_INSTS_VALU"]
                    issue["issue_frac"] = c["SQ_INSTS_VALU"] / (N_CU * 4 * cyc / 2.0)
                if v.get("serial_avg_ns"):
                    issue["serial_avg_ms"] = v["serial_avg_ns"] * 1e-6
                return v["hbm_read_bytes"] + v["hbm_write_bytes"], os.path.relpath(path, ROOT), issue
    return None, None, None


def serial_probe(L, g, pkw, chunk, steps):
    """Per-launch kernel times with every kernel alone on the chip, measured live: the
    timed step's batch (same replicas per launch: the plan's chunk) with the library's
    pipeline off (RQ_PIPE=1: every chunk's generation, merge, sweep and scan in order
    on the caller's one stream) and nothing else queued, HIP events around each launch.
    In the timed region two caller streams' kernels share the chip and stretch each
    launch's HIP-event time; these are the durations the kernel itself needs (the same
    figure as a rocprofv3 kernel trace under AMD_SERIALIZE_KERNEL=3).
    Returns (ms per launch [gen, sweep, scan, -, merge], launches)."""
    pkw = {k: v for k, v in pkw.items() if k != "chunk"}
    old = os.environ.get("RQ_PIPE")
    os.environ["RQ_PIPE"] = "1"
    try:
        g.run("opt", ctrl_seed=7_000_000, world_seed=7_000_000, check=False, chunk=chunk, **pkw)
        torch.cuda.synchronize()
        L.lib().rq_timing(1)
        for k in range(steps):
            g.run("opt", ctrl_seed=7_000_001 + k, world_seed=7_000_001 + k, check=False,
                  chunk=chunk, **pkw)
        torch.cuda.synchronize()
        ms = np.zeros(5)
        nl = np.zeros(5, dtype=np.int64)
        L.lib().rq_timing_read(ms.ctypes.data_as(L._pd), nl.ctypes.data_as(L._pi64))
        L.lib().rq_timing(0)
    finally:
        if old is None:
            os.environ.pop("RQ_PIPE", None)
        else:
            os.environ["RQ_PIPE"] = old
    return ms / np.maximum(nl, 1), nl


def make_step(wl, g, so, R, world, rank, dev, Ks, group=None, force=False, chunk=0):
    """The bench step of a workload, on this rank: (step(k) -> (this rank's BatchResult,
    ensemble means), replicas per step over all ranks, plan kwargs).
    c2 / c3 / c5: R replicas per GPU with their own seeds, one all-gather of the
    per-replica metric rows (RCCL over xGMI), the ensemble means.
    c4: the 64 q x 4 s grid with R replicas per grid point per GPU -- rank k runs the
    k-th replica window of EVERY grid point (dist.run_sharded), one all-gather, then
    per-grid-point means in fixed replica order (dist.grid_means).
    force: the all-gather runs through the process group even for one rank (--dist).
    chunk: replicas per pipelined chunk inside one call (0: the library's plan)."""
    from redqueen_amd import dist as D
    if wl == "c4":
        from redqueen_amd import graphs
        grid = graphs.c4_grid()
        qs = np.asarray([q for q, _ in grid])
        sm = np.asarray([list(s) for _, s in grid])
        n_rep = R * world
        lo, hi = D.grid_shard(n_rep, world, rank)
        kw = dict(q=qs, s=sm, randomize=True, Ks=Ks, seed_mod=n_rep, chunk=chunk)

        def step(k):
            base = k * n_rep
            m, c, res = D.run_sharded(g, len(grid), n_rep, world, rank, group, force,
                                      ctrl="opt", ctrl_seed=base, world_seed=base, check=False,
                                      **kw)
            return res, D.grid_means(m, len(grid), n_rep)
        return step, len(grid) * n_rep, dict(kw, n_rep=n_rep, rep_lo=lo, rep_cnt=hi - lo)

    def step(k):
        base = (k * world + rank) * R
        res = g.run("opt", q=so["q"], s=so["s"], n_rep=R, ctrl_seed=base, world_seed=base,
                    randomize=True, Ks=Ks, check=False, chunk=chunk)
        m = res.metrics
        if world > 1 or force:
            # RCCL over xGMI: the only exchange
            m = D.gather_rows(m, world * R, world, rank, group, force=force)
        # ensemble means (redqueen_amd.dist.grid_means): identical on every rank
        return res, D.grid_means(m, 1, m.shape[0])[0]
    return step, R * world, dict(q=so["q"], s=so["s"], n_rep=R, randomize=True, Ks=Ks, chunk=chunk)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=3)
    # C5 default: two rounds of the 2048 waves the general sweep keeps resident
    ap.add_argument("--replicas", type=int, default=0,
                    help="replicas per GPU per step (default: C3/C2 10000, C5 4096)")
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=0)
    ap.add_argument("--streams", type=int, default=0,
                    help="caller streams the steps alternate over (the engine keeps a "
                         "workspace and side stream per caller stream, so step k's tail "
                         "overlaps step k+1's generation and merge); 1 = one stream; "
                         "0 = 2, except C5, whose 164 GB step workspace does not fit twice "
                         "in HBM (the second stream would plan smaller chunks: same mean "
                         "rate, mixed launch sizes; gpurun_out/r05m)")
    ap.add_argument("--probe-steps", type=int, default=0,
                    help="steps of the serialised probe after the timed region (per-launch "
                         "kernel times with each kernel alone on the chip; default 3, C5 1)")
    ap.add_argument("--chunk", type=int, default=-1,
                    help="replicas per pipelined chunk inside one call: -1 = the whole call "
                         "when the steps alternate over >= 2 caller streams (the steps then "
                         "overlap each other, and the library's two-chunk split inside a call "
                         "only adds launches: C3 2.71 -> 2.58 ms per step, C4 25.1 -> 24.7, "
                         "gpurun_out/chunkab, chunkc4), else the library's plan; 0 = the "
                         "library's plan")
    ap.add_argument("--dist", action="store_true",
                    help="at N = 1 too: a world-size-1 RCCL group, the step's all-gather "
                         "runs through it")
    a = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=dev)
    elif a.dist:   # one rank, no rendezvous: an in-process store
        dist.init_process_group("nccl", device_id=dev, store=dist.HashStore(), rank=0,
                                world_size=1)
    grouped = dist.is_initialized()

    from redqueen_amd import engine
    from redqueen_amd import _lib as L
    from redqueen_amd import dist as D
    so, desc = workload(a.workload)
    g = engine.Graph(so["src_id"], so["other_sources"], so["sink_ids"], so["edge_list"],
                     so["end_time"])
    # replicas per GPU per step (c4: per grid point per GPU)
    # C5: 8192 = two pipelined chunks of 4096 (the general sweep's resident waves): 16.0k
    # replicas/s against 15.8k at 4096 (profiles/r04_c5_ab.txt)
    R = a.replicas or {"c5": 8192, "c4": 1000}.get(a.workload, 10000)
    Ks = (1,)
    n_streams = a.streams or (1 if a.workload == "c5" else 2)
    chunk = a.chunk if a.chunk >= 0 else (1 << 30 if n_streams >= 2 else 0)   # clamped to the call
    step, rep_step, pkw = make_step(a.workload, g, so, R, world, rank, dev, Ks,
                                    force=grouped, chunk=chunk)
    plan = g.run("opt", plan_only=True, **pkw)

    # capacity check once at full size (overflow -> the engine reruns with doubled
    # capacities; every launch of the run has the timed launches' shape, so a rocprofv3
    # average over the whole command matches the per-launch HIP-event time), then
    # warmup so the timed region starts with every buffer allocated
    ok = g.run("opt", ctrl_seed=0, world_seed=0, check=True, **pkw)
    del ok
    mask = L.ST_ROWS_OVERFLOW | L.ST_STREAM_OVERFLOW

    def accumulate(res, acc):
        # per step: one reduction of the count columns, one of the overflow bits, one
        # count of the replicas the fast sweep flagged RQ_ST_TIE (equal event times:
        # check=True would rerun them on the exact sequential sweep; never taken by
        # the continuous-time bench worlds, and reported so that it shows if it is)
        if res is None:   # a rank without replicas (more ranks than replicas per point)
            return
        acc[0] += res.counts.sum(0)
        torch.maximum(acc[1], (res.status & mask).max(), out=acc[1])
        acc[2] += ((res.status & L.ST_TIE) != 0).sum()

    def new_acc():
        return [torch.zeros(4, dtype=torch.int64, device=dev),
                torch.zeros((), dtype=torch.int32, device=dev),
                torch.zeros((), dtype=torch.int64, device=dev)]

    # steps alternate over caller streams: step k's batch, exchange, means and tallies are
    # ordered on stream k % S, so the next step's generation and merge (another stream,
    # its own workspace and side stream) fill the wave slots this step's sweep tail and
    # scan leave; every step still runs all of its work inside the timed region, which
    # ends with a device-wide synchronize
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream(device=dev)
                                                for _ in range(n_streams - 1)]

    def run_steps(ks):
        accs = []
        for st in streams:
            with torch.cuda.stream(st):
                accs.append(new_acc())
        for k in ks:
            with torch.cuda.stream(streams[k % len(streams)]):
                res, means = step(k)
                accumulate(res, accs[k % len(streams)])
        return accs

    # the warmup runs the exact timed body (every stream, its workspace and side stream):
    # HIP loads a kernel's code object on its first launch (tens of ms for torch's), which
    # must not land in the timed region
    L.lib().rq_timing(1)
    run_steps([k + 10_000 for k in range(max(len(streams), a.warmup))])
    torch.cuda.synchronize()

    L.lib().rq_timing(1)
    if grouped:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    accs = run_steps(range(a.steps))
    torch.cuda.synchronize()
    if grouped:
        dist.barrier()
    el = time.perf_counter() - t0
    csum = sum(x[0] for x in accs)
    status = torch.stack([x[1] for x in accs]).max()
    ties = sum(x[2] for x in accs)
    ms = np.zeros(5)
    nl = np.zeros(5, dtype=np.int64)
    L.lib().rq_timing_read(ms.ctypes.data_as(L._pd), nl.ctypes.data_as(L._pi64))
    L.lib().rq_timing(0)
    t = torch.tensor([el], dtype=torch.float64, device=dev)
    if grouped:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t.item())

    rows_l, posts_l = int(csum[3].item()), int(csum[0].item())   # this rank
    tot = csum.clone()
    if grouped:   # reporting only, after the timed region
        dist.all_reduce(tot)
    local_ev = int(tot[2].item())   # events of all ranks
    replicas = rep_step * a.steps
    value = replicas / el
    ev_rate = local_ev / el

    # the kernels alone (outside the timed region): the roofline's launch duration
    sms, snl = serial_probe(L, g, pkw, plan["chunk"],
                            a.probe_steps or (1 if a.workload == "c5" else 3))

    # roofline of the dominant kernel (the sweep), per launch, this rank
    n_sweep = max(1, int(nl[1]))
    sweep_ms = ms[1] / n_sweep
    sweep_ms_serial = float(sms[1]) if snl[1] else None
    # per LAUNCH: a step runs one launch of each kernel per replica chunk (the engine's
    # pipelined chunks, rq_run_batch), so the step's bytes are split over its launches
    lps = n_sweep / a.steps
    ev_rank = local_ev / world / a.steps / lps
    rows_step = rows_l / a.steps / lps
    posts_step = posts_l / a.steps / lps
    # the fused sweep (variant >= 10) generates its arrivals in LDS: no arrival reads
    fused = 10 <= plan["variant"] < 20   # 20+: the fused sweep on merged streams (reads them)
    merged = not fused and plan["sources_per_lane"] == 0   # rq_merge_streams feeds the sweep
    b_wall = MRG_SWEEP_B_PER_WALL_EVENT if merged else SWEEP_B_PER_WALL_EVENT
    sweep_bytes = (0 if fused else b_wall * (ev_rank - posts_step)) + \
        SWEEP_B_PER_ROW * rows_step
    achieved_live = sweep_bytes / (sweep_ms * 1e-3) / 1e9
    # the headline fraction: the kernel's own launch duration (serialised probe); the
    # overlapped HIP-event time of the timed region is kept as frac_live
    achieved = sweep_bytes / (sweep_ms_serial * 1e-3) / 1e9 if sweep_ms_serial else achieved_live
    scan_ms = ms[2] / max(1, int(nl[2]))
    gen_ms = ms[0] / max(1, int(nl[0]))
    scan_gbs = SCAN_B_PER_ROW * rows_step / (scan_ms * 1e-3) / 1e9 if scan_ms > 0 else None
    gen_gbs = GEN_B_PER_WALL_EVENT * (ev_rank - posts_step) / (gen_ms * 1e-3) / 1e9 \
        if gen_ms > 0 else None
    merge_ms = ms[4] / max(1, int(nl[4]))
    merge_gbs = MERGE_B_PER_WALL_EVENT * (ev_rank - posts_step) / (merge_ms * 1e-3) / 1e9 \
        if merge_ms > 0 else None

    traffic, traffic_src, issue = pmc_traffic(a.workload, R, plan)
    if issue and "issue_frac" in issue:
        # the same ceiling over this run's own HIP-event launch time at the PMC run's clock
        issue["issue_frac_2400mhz_probe_time"] = issue["valu_insts"] / (
            N_CU * 4 * 2.4e9 / 2.0 * (sweep_ms_serial or sweep_ms) * 1e-3)

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu:
        nt = min(16, os.cpu_count() or 1)
        sample = a.cpu_sample or {"c5": 2, "c4": 512}.get(a.workload, 128) * nt
        cgrid = None
        if a.workload == "c4":   # 16 grid points spread over the q x s grid
            from redqueen_amd import graphs
            cgrid = graphs.c4_grid()[::16]
        crate, cev, cel = cpu_baseline(so, nt, sample, Ks, cgrid)
        cpu = {"value": crate, "unit": "replicas/s", "cores": nt, "kind": "port",
               "sample": "%d %s replicas through the C oracle (engine semantics + Appendix-B "
                         "metrics), %d pthreads, %.1f s, %.0f events/s" %
                         (sample, a.workload.upper(), nt, cel, cev)}

    if rank == 0:
        line = {
            "metric": "redqueen_replicas_per_sec",
            "value": value,
            "unit": "replicas/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": el / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (Philox-seeded arrival streams on the reference's %s network)" %
                    a.workload.upper(),
            "config": {"workload": desc, "replicas_per_gpu": rep_step // world, "global_batch": rep_step,
                       "parallelism": ("grid-window sharded dp%d (each rank: every grid point's "
                                       "replica window)" if a.workload == "c4" else
                                       "replica-sharded dp%d") % world, "Ks": list(Ks),
                       "replicas_per_chunk": int(plan["chunk"])},
            "events_per_sec": ev_rate,
            "events_per_replica": local_ev / replicas,
            "overflow": int(status.item()),
            "tie_replicas": int(ties.item()),
            # HIP-event time per launch inside the timed region (two caller streams' kernels
            # share the chip: each launch's time is stretched by the overlap)
            "kernels_ms_per_launch": {"gen_streams": gen_ms, "merge_streams": merge_ms, "sweep": sweep_ms,
                                      "scan": scan_ms},
            # the same launches alone on the chip (serial_probe: pipeline off, one stream)
            "kernels_ms_per_launch_serial": {"gen_streams": float(sms[0]), "merge_streams": float(sms[4]),
                                             "sweep": sweep_ms_serial, "scan": float(sms[2]),
                                             "launches": [int(x) for x in snl]},
            "launches_per_step": lps,
            "caller_streams": len(streams),
            "sweep_plan": plan,
            "roofline": {"bound": "hbm", "kernel": "rq_sweep", "achieved": achieved,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "duration_ms": sweep_ms_serial or sweep_ms,
                         "duration_source": "serial_probe: the launch alone on the chip, HIP events"
                                            if sweep_ms_serial else "timed region, HIP events",
                         "bytes_per_launch": sweep_bytes,
                         "achieved_live": achieved_live, "frac_live": achieved_live / HBM_PEAK_GBS,
                         "traffic": traffic,
                         "traffic_source": traffic_src,
                         # what does bound it: SQ issue / wait shares of the wave cycles and
                         # issue_frac = VALU instructions / the VALU issue ceiling (same PMC run)
                         "issue": issue,
                         "issue_frac": issue.get("issue_frac") if issue else None,
                         "wave_slot_occupancy": issue.get("wave_slot_occupancy") if issue else None,
                         # the same algorithmic bytes over the launch's duration with every
                         # kernel serialised (stamped PMC summary, AMD_SERIALIZE_KERNEL=3
                         # trace): in the timed run the two streams' kernels share the chip,
                         # which stretches each launch's HIP-event time
                         "frac_serialized": (sweep_bytes / (issue["serial_avg_ms"] * 1e-3) / 1e9 /
                                             HBM_PEAK_GBS) if issue and issue.get("serial_avg_ms") else None,
                         "note": "sweep is latency/issue-bound (serial event chain per replica); "
                                 "algorithmic bytes = 24 B/pivot row written%s" %
                                 ("" if fused else " + %d B/wall event read" % b_wall)},
            "scan_gbs": scan_gbs,
            "gen_gbs": gen_gbs,
            "merge_gbs": merge_gbs,
            # SURVEY 8(d)'s end-to-end figure: 24 B per simulated event (one pivot row
            # written and read back) at the whole job's event rate
            "roofline_e2e": {"bytes_per_event": SWEEP_B_PER_ROW, "achieved": e2e_gbs(ev_rate),
                             "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": e2e_gbs(ev_rate) / HBM_PEAK_GBS / world},
            "exchange": ("RCCL all-gather (process group of %d)" % world) if grouped else None,
            "cpu_baseline": cpu,
            "cpu_baseline_reference": ref_cpu_baseline(a.workload),
        }
        print(json.dumps(line), flush=True)
    if grouped:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
