"""Scenario builders: the reference's synthetic-graph generators and the
benchmark configurations C1-C5 of SURVEY.md section 8(d).

Host-side only (numpy), they produce SimOpts keyword dicts
(opt_model.py:773-780).  ``make_edge_list`` and ``trim`` follow
opt_runs.make_edge_list (opt_runs.py:662-685) and opt_runs.trim_sim_opts
(:705-718) draw for draw, so a given seed yields the reference's network.
"""
import numpy as np


def make_edge_list(num_followers, num_broadcasters, degree, seed, follower_id_offset=0,
                   broadcaster_id_offset=0, preferential_attachment=False):
    """Each follower follows `degree` distinct broadcasters (opt_runs.py:662-685)."""
    rs = np.random.RandomState(seed)
    weight = np.ones(num_broadcasters)
    p = weight / weight.sum()
    edges = []
    for sink in range(follower_id_offset, follower_id_offset + num_followers):
        if preferential_attachment:
            p = weight / weight.sum()
        for b in rs.choice(num_broadcasters, degree, replace=False, p=p):
            if preferential_attachment:
                weight[b] += 1
            edges.append((int(b) + broadcaster_id_offset, sink))
    return edges


def trim(so):
    """Keep only the controlled source's followers and the broadcasters that reach
    them; q = (#followers)^2 (opt_runs.trim_sim_opts, opt_runs.py:705-718)."""
    fol = {t for s, t in so["edge_list"] if s == so["src_id"]}
    edges = [(s, t) for s, t in so["edge_list"] if t in fol]
    reach = {s for s, _ in edges}
    out = dict(so)
    out.update(sink_ids=sorted(fol), edge_list=edges,
               other_sources=[x for x in so["other_sources"] if x[1]["src_id"] in reach],
               q=1.0 * len(fol) ** 2)
    return out


def readme():
    """C1: the README network (README.md:60-81)."""
    return dict(src_id=1, end_time=100.0, s={1: 1.0, 3: 1.0}, q=1.0, sink_ids=[1, 2, 3],
                other_sources=[("Poisson2", {"src_id": 2, "seed": 42, "rate": 10}),
                               ("Hawkes", {"src_id": 3, "seed": 43, "l_0": 10, "alpha": 1.0,
                                           "beta": 10.0})],
                edge_list=[(1, 1), (1, 3), (2, 1), (2, 2), (2, 3), (3, 3)])


def kat_two_walls(s=(1.0, 1.0)):
    """Notebook KAT network (opt_broadcast.ipynb:5443-5450)."""
    return dict(src_id=1, end_time=100.0, q=1.0, s=np.asarray(s, dtype=float),
                sink_ids=[5001, 5002],
                other_sources=[("Poisson2", {"src_id": 1000, "seed": 42, "rate": 10.0}),
                               ("Poisson2", {"src_id": 1001, "seed": 43, "rate": 10.0})],
                edge_list=[(1000, 5001), (1001, 5002), (1, 5001), (1, 5002)])


def mixed():
    """All source kinds in one small world (used by the parity tests)."""
    return dict(src_id=1, end_time=50.0, s=np.asarray([1.0, 2.0, 0.5]), q=2.0,
                sink_ids=[10, 11, 12, 13],
                other_sources=[("PiecewiseConst", {"src_id": 4, "seed": 9,
                                                   "change_times": [0.0, 10.0, 30.0],
                                                   "rates": [2.0, 8.0, 1.0]}),
                               ("Poisson", {"src_id": 5, "seed": 10, "rate": 3.0}),
                               ("RealData", {"src_id": 6,
                                             "times": [0.5, 7.25, 7.5, 33.0, 49.0, 60.0]}),
                               ("Hawkes", {"src_id": 7, "seed": 11, "l_0": 1.5, "alpha": 0.5,
                                           "beta": 2.0})],
                edge_list=[(1, 10), (1, 11), (1, 12), (4, 10), (4, 13), (5, 11), (5, 12),
                           (6, 10), (6, 11), (6, 12), (6, 13), (7, 12), (7, 13)])


def followers_graph(num_followers=1000, num_sources=50, degree=5, end_time=100.0,
                    kinds=("Poisson2", "Hawkes"), world_rate=1.0, alpha=1.0, beta=10.0,
                    seed=42, network_seed=1024, max_num_followers=None):
    """C3 ("syn1k") and C5: the construction of
    opt_runs.prepare_multiple_followers_sim_opts (opt_runs.py:726-795) with the
    broadcaster kinds interleaved in contiguous blocks (first half kinds[0], ...).
    Followers 1000.., broadcasters 5000.., the controlled source 1 follows all."""
    rs = np.random.RandomState(seed)
    nmax = num_followers if max_num_followers is None else max_num_followers
    fol_ids = 1000 + np.arange(nmax)
    b_ids = 5000 + np.arange(num_sources)
    edges = make_edge_list(nmax, num_sources, degree, network_seed,
                           follower_id_offset=1000, broadcaster_id_offset=5000)
    others = []
    per = int(np.ceil(num_sources / len(kinds)))
    for k, x in enumerate(b_ids):
        kind = kinds[min(k // per, len(kinds) - 1)]
        kw = {"src_id": int(x), "seed": int(seed + x)}
        if kind in ("Poisson", "Poisson2"):
            kw["rate"] = world_rate
        elif kind == "Hawkes":
            kw.update(l_0=world_rate, alpha=alpha, beta=beta)
        else:
            raise ValueError(kind)
        others.append((kind, kw))
    edges = edges + [(1, int(x)) for x in rs.choice(fol_ids, num_followers, replace=False)]
    so = dict(src_id=1, end_time=end_time, s=np.ones(num_followers), sink_ids=list(fol_ids),
              other_sources=others, edge_list=edges, q=1.0 * num_followers ** 2)
    return trim(so)


def c3():
    """1000 followers, 25 Poisson2 (rate 1) + 25 Hawkes (l_0=1, alpha=1, beta=10), T=100."""
    return followers_graph()


def c5():
    """10k followers, 500 bursty Hawkes (l_0=0.5, alpha=1, beta=2), T=1000, q=1e8."""
    return followers_graph(num_followers=10000, num_sources=500, degree=5, end_time=1000.0,
                           kinds=("Hawkes",), world_rate=0.5, alpha=1.0, beta=2.0)


def c5_small():
    """C5's bursty regime at C5's own horizon, small enough for the reference to run
    10k replicas (~2 s each): 4 followers, 4 Hawkes broadcasters (l_0 = 0.5, alpha = 1,
    beta = 2: stationary rate 1, branching ratio 0.5), degree 2, T = 1000, q = 16."""
    return followers_graph(num_followers=4, num_sources=4, degree=2, end_time=1000.0,
                           kinds=("Hawkes",), world_rate=0.5, alpha=1.0, beta=2.0)


def c5_mid():
    """C5's source side at C5's horizon, small enough for a handful of reference runs
    (minutes each): 500 bursty Hawkes broadcasters (l_0 = 0.5, alpha = 1, beta = 2), 100
    followers of degree 5, T = 1000, q = 1e4 (the trim keeps the ~316 broadcasters that
    reach a follower).  The reference-run replay fixture `scale_logs.npz` uses it."""
    return followers_graph(num_followers=100, num_sources=500, degree=5, end_time=1000.0,
                           kinds=("Hawkes",), world_rate=0.5, alpha=1.0, beta=2.0)


def g120():
    """A > 64-source world (the general sweep's instances, like C5) small enough for the
    reference to run thousands of replicas: 60 followers, 120 broadcasters (Poisson2
    rate 0.5 / Hawkes l_0 0.5, alpha 1, beta 4), degree 4, T = 20 (the trim keeps the
    broadcasters that reach a follower)."""
    return followers_graph(num_followers=60, num_sources=120, degree=4, end_time=20.0,
                           world_rate=0.5, alpha=1.0, beta=4.0)


C4_S = [(1.0, 1.0), (0.5, 1.5), (1.5, 0.5), (1.0, 0.25)]


def c4_grid(n_q=64):
    """C4: README graph x q = logspace(-4, 7, 64) (opt_runs.py:289-291) x the four s."""
    qs = np.logspace(-4, 7, n_q)
    return [(q, s) for s in C4_S for q in qs]
