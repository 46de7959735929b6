#!/usr/bin/env python
"""Wall time of opt_runs.run_inference_queue on the reference's own inference
configurations (opt_runs.py:284-331: 10 q x N = 10 seeds, T = 100, Poisson / Hawkes /
PiecewiseConst worlds), with the Oracle legs' q searches batched (one rq_oracle_dp
launch per search round over all 100 replicas, utils.find_opt_oracle_batch) and,
for comparison, searched replica by replica (the round-3 path).  The reference's
notebook ran three such worlds in 14 min 50 s (opt_broadcast.ipynb:609-610).

    python scripts/bench_inference.py [--out profiles/r04_inference.json]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    ap.add_argument("--worlds", default="poisson,hawkes,piecewise")
    a = ap.parse_args()
    import logging
    logging.disable(logging.ERROR)   # the per-replica 'kdd' exception records
    import torch
    from redqueen_amd import opt_runs as R
    from redqueen_amd import utils as U
    cfg = {"poisson": R.poisson_inf_opts, "hawkes": R.hawkes_inf_opts,
           "piecewise": R.piecewise_inf_opts}
    # warm the code objects / torch allocator outside the timed runs
    R.run_inference_queue(N=1, opts=cfg["poisson"])
    torch.cuda.synchronize()
    rows = []
    batch_fn = U.find_opt_oracle_batch
    for name in a.worlds.split(","):
        for mode in ("batched", "per_replica"):
            if mode == "per_replica":
                def one_by_one(targets, sos, max_events=None, walls=None, **kw):
                    # each replica's search on its own: one DP launch per search step
                    return [batch_fn([t], [so], [me], walls=[w], **kw)[0]
                            for t, so, me, w in zip(targets, sos, max_events, walls)]
                U.find_opt_oracle_batch = one_by_one
            t0 = time.perf_counter()
            out = R.run_inference_queue(opts=cfg[name])
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            U.find_opt_oracle_batch = batch_fn
            n = {k: int((out.df.type == k).sum()) for k in ("Opt", "Poisson", "Oracle")}
            rows.append({"world": name, "oracle_search": mode, "wall_s": el, "rows": n,
                         "N": 10, "q_points": 10})
            print(json.dumps(rows[-1]), flush=True)
    if a.out:
        with open(a.out, "w") as fh:
            json.dump({"command": "python scripts/bench_inference.py", "runs": rows,
                       "reference_notebook": "3 worlds x (10 q x 10 seeds + Poisson/Oracle/kdd "
                                             "follow-ups): 14 min 50 s (opt_broadcast.ipynb:609-610)"},
                      fh, indent=1)


if __name__ == "__main__":
    main()
