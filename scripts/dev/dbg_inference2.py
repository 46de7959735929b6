import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from oracle import oracle as O  # noqa: E402
from redqueen_amd import opt_runs as R  # noqa: E402
from redqueen_amd.opt_model import SimOpts  # noqa: E402


def gen(seed):
    return SimOpts.std_poisson(world_rate=4.0, world_seed=seed + 42).update({"end_time": 20.0})


out = R.run_inference_queue(N=3, T=20.0, num_segments=4, sim_opts_gen=gen, log_q_high=3, log_q_low=-1)
opt = [r for r in out.raw_results if r["type"] == "Opt"]
poi = [r for r in out.raw_results if r["type"] == "Poisson"]
bad = 0
for r, p in zip(opt, poi):
    so = gen(r["seed"]).update({"q": r["q"]})
    rate = r["capacity"] / 20.0
    (top, avg, r2, cnt), (t_o, _, s_o) = O.engine_metrics(O.Scenario(so.get_dict(), ("poisson", r["seed"], rate)), (1,))
    ok = (p["top_1"], p["avg_rank"], p["r_2"], p["num_events"]) == (top[0], avg, r2, cnt[0])
    if not ok:
        bad += 1
        print("q", r["q"], "seed", r["seed"], "cap", r["capacity"], repr(rate), "gpu", p["top_1"], p["avg_rank"],
              p["num_events"], p["world_events"], "orc", top[0], avg, cnt)
        # the same replica alone on the GPU
        m = so.create_manager_with_poisson(seed=r["seed"], capacity=r["capacity"])
        m.run_dynamic()
        t, s = m.state._t, m.state._src
        print("   single run events == oracle:", np.array_equal(t, t_o) and np.array_equal(s, s_o),
              "metrics", m.result.metrics[0].cpu().numpy())
print("bad", bad, "of", len(poi))
