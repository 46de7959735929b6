#!/usr/bin/env python
"""Time the REFERENCE (MPI-SWS/RedQueen, pure Python) on its own CPU path, here in
the build container -- a measured baseline, never a target.

    MPLBACKEND=Agg python scripts/ref_cpu_baseline.py [--c2 256] [--c3 64] [--procs 8]

Pattern: utils.calc_q_capacity_iter's multiprocessing.Pool over replicas
(utils.py:463-468); per replica the opt_runs.worker_opt work (opt_runs.py:51-106):
create_manager_with_opt + run_dynamic + get_dataframe + add_perf's metrics
(time_in_top_k K=1, average_rank, int_r_2, event counts).  C2 = README graph
(randomize_other_sources(r), Opt seed r); C3 = the 1000-follower bench graph
(redqueen_amd.graphs.c3).  Imports /root/reference with the decorated_options
stand-in of tests/golden/_shim (the reference never travels to the GPU box).
Prints one JSON line per config: replicas, wall seconds, replicas/s, events/s, procs.
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import time
import warnings

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden", "_shim"))
sys.path.insert(0, "/root/reference")
sys.path.insert(0, ROOT)
warnings.filterwarnings("ignore")
os.environ.setdefault("MPLBACKEND", "Agg")


def _worker(args):
    name, r = args
    warnings.filterwarnings("ignore")
    from redqueen.opt_model import SimOpts
    import redqueen.utils as U
    from redqueen_amd import graphs as G
    so = SimOpts(**(G.readme() if name == "c2" else G.c3()))
    u = r if name == "c2" else 5000 * r
    m = so.randomize_other_sources(u).create_manager_with_opt(seed=u)
    m.run_dynamic()
    df = m.state.get_dataframe()
    U.time_in_top_k(df=df, K=1, sim_opts=so)
    U.average_rank(df, sim_opts=so)
    U.int_r_2(df, so)
    len(df.event_id[df.src_id == so.src_id].unique())
    len(df.event_id[df.src_id != so.src_id].unique())
    return m.state.get_num_events()


def run(name, n, procs):
    t0 = time.time()
    with mp.Pool(procs) as pool:
        ev = pool.map(_worker, [(name, r) for r in range(n)], chunksize=1)
    dt = time.time() - t0
    return {"config": name, "replicas": n, "procs": procs, "wall_s": dt,
            "replicas_per_s": n / dt, "events_per_s": sum(ev) / dt,
            "mean_events": sum(ev) / n, "cpu": os.cpu_count()}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--c2", type=int, default=256)
    ap.add_argument("--c3", type=int, default=64)
    ap.add_argument("--procs", type=int, default=8)
    a = ap.parse_args()
    for name, n in (("c2", a.c2), ("c3", a.c3)):
        if n:
            print(json.dumps(run(name, n, a.procs)), flush=True)
