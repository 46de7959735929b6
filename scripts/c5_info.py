import sys, os
sys.path.insert(0, "/root/repo")
from redqueen_amd import engine, graphs
so = graphs.c5()
g = engine.Graph(so["src_id"], so["other_sources"], so["sink_ids"], so["edge_list"], so["end_time"])
print(g.run("opt", q=so["q"], s=so["s"], n_rep=4096, plan_only=True))
