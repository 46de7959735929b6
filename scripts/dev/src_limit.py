"""Plan (and a 2-replica run) for worlds of many sources: where the planner stops."""
import sys
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from test_gpu_graphs import _many_sources  # noqa: E402
from redqueen_amd import engine  # noqa: E402
for n in [int(x) for x in sys.argv[1:]]:
    so = _many_sources(n, T=2.0)
    g = engine.Graph(so["src_id"], so["other_sources"], so["sink_ids"], so["edge_list"], so["end_time"])
    for kw in ({}, dict(sweep_mode=2)):
        try:
            p = g.run("opt", q=1.0, s=1.0, n_rep=2, plan_only=True, **kw)
            r = g.run("opt", q=1.0, s=1.0, n_rep=2, ctrl_seed=1, world_seed=1, randomize=True, **kw)
            print(n, kw, p["variant"], p["lds_bytes_per_block"], "ok", r.counts[:, 2].tolist(), flush=True)
        except Exception as e:
            print(n, kw, "ERR", e, flush=True)
