"""Debug: fast vs log sweep vs oracle on tie-heavy worlds (GPU)."""
import sys, numpy as np, torch
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
from test_gpu_engine import _tie_world, _oracle
from redqueen_amd import engine
from oracle import oracle as O

so, T = _tie_world()
variants = {
    "full": so,
    "one_rd": dict(so, other_sources=[so["other_sources"][0], so["other_sources"][2]],
                   edge_list=[e for e in so["edge_list"] if e[0] != 3]),
    "two_rd": dict(so, other_sources=so["other_sources"][:2],
                   edge_list=[e for e in so["edge_list"] if e[0] != 4]),
}
for name, w in variants.items():
    for ctrl in ("times", "wall", "opt"):
        ct = T[::3].copy()
        g = engine.Graph(w["src_id"], w["other_sources"], w["sink_ids"], w["edge_list"], w["end_time"],
                         ctrl_a=ct if ctrl == "times" else None)
        kw = dict(n_rep=1, Ks=(1, 2))
        if ctrl == "opt":
            kw.update(q=w["q"], s=w["s"], ctrl_seed=1)
        a = g.run(ctrl, **kw)
        b = g.run(ctrl, event_log=True, sweep_mode=2, **kw)
        oc = ("times", ct) if ctrl == "times" else (("opt", 1) if ctrl == "opt" else ("wall",))
        met_o, t_o, s_o = _oracle(O, w, oc, (1, 2))
        print(name, ctrl, "fast", a.metrics[0].cpu().numpy(), a.counts[0].cpu().numpy(), int(a.status[0]))
        print(name, ctrl, "log ", b.metrics[0].cpu().numpy(), b.counts[0].cpu().numpy(), int(b.status[0]))
        print(name, ctrl, "orac", list(met_o[0]) + [met_o[1], met_o[2]], met_o[3], len(t_o))
