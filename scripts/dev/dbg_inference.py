"""Debug: Poisson leg of run_inference_queue vs the engine oracle, per replica."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from oracle import oracle as O  # noqa: E402
from redqueen_amd.batch import compiled_graph  # noqa: E402
from redqueen_amd.opt_model import SimOpts  # noqa: E402

N = 3
qs = np.logspace(-1, 3, num=10)
T = 20.0
worlds = [SimOpts.std_poisson(world_rate=4.0, world_seed=s + 42).update({"end_time": T}) for s in range(N)]
g = compiled_graph(worlds[0])
sd = np.arange(N)
us = sd + 42
seed_t = torch.as_tensor(np.tile(sd, len(qs)))
u_t = torch.as_tensor(np.tile(us, len(qs)))
ro = g.run("opt", q=qs, s=g.s_matrix(1.0, len(qs)), n_rep=N, ctrl_seed=seed_t, world_seed=u_t, randomize=True, Ks=(1,))
posts = ro.num_events.double()
rate = posts / T
for mode, el in ((0, False), (3, False), (4, False), (0, True)):
    rp = g.run("poisson", n_rep=len(qs) * N, ctrl_seed=seed_t, world_seed=u_t, randomize=True,
               ctrl_rate=rate, Ks=(1,), sweep_mode=mode, event_log=el)
    print("plan", g.run("poisson", n_rep=len(qs) * N, ctrl_seed=seed_t, world_seed=u_t, randomize=True,
               ctrl_rate=rate, Ks=(1,), sweep_mode=mode, event_log=el, plan_only=True))
    m = rp.metrics.cpu().numpy()
    bad = 0
    for i in range(len(qs) * N):
        seed = int(sd[i % N])
        r = float(rate[i].item())
        so = worlds[i % N]
        (top, avg, r2, cnt), (t_o, _, s_o) = O.engine_metrics(O.Scenario(so.get_dict(), ("poisson", seed, r)), (1,))
        if el:
            t, s = rp.events(i)
        else:
            t, s = t_o, s_o
        same_ev = np.array_equal(t, t_o) and np.array_equal(s, s_o)
        if not (m[i, 0] == top[0] and m[i, 1] == avg and m[i, 2] == r2) or not same_ev:
            bad += 1
            if bad < 4:
                print("mode", mode, "rep", i, "seed", seed, "rate", r, "ev_same", same_ev, len(t), len(t_o),
                      "gpu", m[i], "orc", top[0], avg, r2, "status", int(rp.status[i]))
                if len(t) == len(t_o):
                    k = np.nonzero((t != t_o) | (s != s_o))[0]
                    print("   first diff", k[:3], t[k[:3]] if len(k) else None, t_o[k[:3]] if len(k) else None)
    print("mode", mode, "bad", bad, "of", len(qs) * N, flush=True)
