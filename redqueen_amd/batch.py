"""Batched replica grids: the multiprocessing drivers of the reference as GPU batches.

The reference runs one (seed, q, s) replica per process through mp.Pool /
mp.Queue (utils.calc_q_capacity_iter :447-470, opt_runs.worker_opt /
worker_poisson :51-126, opt_runs.run_inference_queue :560-646) and collects
``perf_opts.performance_fields`` (opt_runs.py:33-38) via add_perf (:41-48).
Here a whole grid is one launch sequence of the engine; the result is a
DataFrame with the same fields (seed, q, type, top_K..., avg_rank, r_2,
num_events, world_events, capacity).
"""
import collections
import hashlib

import numpy as np
import pandas as pd
import torch

from .engine import Graph

_CACHE = collections.OrderedDict()


def _val_key(v):
    # arrays (RealData times, PiecewiseConst tables) by dtype, shape and a content
    # hash: numpy's repr elides the middle of arrays longer than 1000 elements
    if isinstance(v, (np.ndarray, list, tuple)):
        a = np.ascontiguousarray(np.asarray(v))
        if a.dtype != object:
            return (str(a.dtype), a.shape, hashlib.sha1(a.tobytes()).hexdigest())
    return repr(v)


def _key(so):
    return (so.src_id, float(so.end_time), tuple(map(tuple, so.edge_list)),
            tuple(so.sink_ids), repr([(n if isinstance(n, str) else n.__name__,
                                       sorted((k, _val_key(v)) for k, v in kw.items()))
                                      for n, kw in so.other_sources]))


def compiled_graph(sim_opts):
    """Device-resident graph for a SimOpts (cached on its contents)."""
    k = _key(sim_opts)
    g = _CACHE.get(k)
    if g is None:
        g = Graph(sim_opts.src_id, sim_opts.other_sources, sim_opts.sink_ids, sim_opts.edge_list,
                  sim_opts.end_time)
        _CACHE[k] = g
        while len(_CACHE) > 8:
            _CACHE.popitem(last=False)
    return g


def _frame(res, seeds, qs, kind, Ks):
    m = res.metrics.cpu().numpy()
    c = res.counts.cpu().numpy()
    st = res.status.cpu().numpy()
    d = {"seed": seeds, "q": qs, "type": kind}
    for i, k in enumerate(Ks):
        d["top_" + str(k)] = m[:, i]
    d["avg_rank"] = m[:, len(Ks)]
    d["r_2"] = m[:, len(Ks) + 1]
    d["num_events"] = c[:, 0]
    d["world_events"] = c[:, 1]
    d["capacity"] = c[:, 0].astype(np.float64)
    d["events"] = c[:, 2]
    d["status"] = st
    return pd.DataFrame(d)


def run_grid(sim_opts, qs=None, ss=None, seeds=range(10), randomize=True, Ks=(1,),
             max_events=None, chunk=0):
    """RedQueen over the grid qs x ss x seeds.

    qs: iterable of q (default [sim_opts.q]); ss: iterable of s (scalar, vector over
    the sorted followers or dict), default [sim_opts.s]; seeds: replica seeds u --
    the RedQueen seed is u and, with randomize, the world is
    sim_opts.randomize_other_sources(u) (the C2 protocol); every grid point sees
    the same seeds (common random numbers, as calc_q_capacity_iter does)."""
    g = compiled_graph(sim_opts)
    qs = [sim_opts.q] if qs is None else list(qs)
    ss = [sim_opts.s] if ss is None else list(ss)
    seeds = np.asarray(list(seeds), dtype=np.int64)
    grid_q, grid_s = [], []
    for s in ss:
        for q in qs:
            grid_q.append(float(q))
            grid_s.append(g.s_matrix(s, 1)[0])
    qv = np.asarray(grid_q)
    sm = np.ascontiguousarray(np.stack(grid_s)) if grid_s and g.n_followers else \
        np.zeros((len(grid_q), g.n_followers))
    R = len(seeds)
    seed_t = torch.as_tensor(np.tile(seeds, len(grid_q)))
    res = g.run("opt", q=qv, s=sm, n_rep=R, ctrl_seed=seed_t, world_seed=seed_t,
                randomize=randomize, Ks=Ks, max_events=max_events, chunk=chunk)
    df = _frame(res, np.tile(seeds, len(grid_q)), np.repeat(qv, R), "Opt", Ks)
    df["s_idx"] = np.repeat(np.arange(len(grid_q)) // max(1, len(qs)), R)
    return df


def run_opt_vs_poisson(sim_opts, seeds=range(10), randomize=True, Ks=(1,), max_events=None,
                       poisson_seed_offset=0):
    """worker_opt then worker_poisson (opt_runs.py:51-126) for every seed: the
    Poisson broadcaster gets the RedQueen replica's capacity (posts) as
    rate = capacity / end_time on the same world; its seed is seed +
    poisson_seed_offset (0 = the reference's worker_poisson)."""
    g = compiled_graph(sim_opts)
    seeds = np.asarray(list(seeds), dtype=np.int64)
    st = torch.as_tensor(seeds)
    ro = g.run("opt", q=float(sim_opts.q), s=sim_opts.s, n_rep=len(seeds), ctrl_seed=st,
               world_seed=st, randomize=randomize, Ks=Ks, max_events=max_events)
    # capacity / end_time with IEEE division on the host (create_manager_with_poisson,
    # opt_model.py:829): torch's tensor / scalar multiplies by the reciprocal, which is
    # an ulp off for most capacities -- and every Poisson time with it
    rate = torch.as_tensor(ro.num_events.cpu().numpy().astype(np.float64) / float(sim_opts.end_time))
    rp = g.run("poisson", n_rep=len(seeds), ctrl_seed=st + int(poisson_seed_offset),
               world_seed=st, randomize=randomize, ctrl_rate=rate, Ks=Ks, max_events=max_events)
    a = _frame(ro, seeds, np.full(len(seeds), float(sim_opts.q)), "Opt", Ks)
    b = _frame(rp, seeds, np.full(len(seeds), float(sim_opts.q)), "Poisson", Ks)
    b["capacity"] = a["capacity"].values
    return pd.concat([a, b], ignore_index=True)


def run_significance(sim_opts, significance, time_period, seeds=range(10), randomize=True,
                     Ks=(1,), max_events=None, qs=None):
    """OptPWSignificance (create_manager_with_significance, opt_model.py:850-884) for
    every seed (x every q in qs): significance [sinks x segments] (or one row of
    segments for all followers); seed u runs world randomize_other_sources(u)."""
    from .opt_model import OptPWSignificance
    g = compiled_graph(sim_opts)
    qs = [sim_opts.q] if qs is None else list(qs)
    seeds = np.asarray(list(seeds), dtype=np.int64)
    spw = OptPWSignificance(sim_opts.src_id, 0, significance, time_period)._s_pw_for(g.n_followers)
    qv = np.asarray(qs, dtype=np.float64)
    # the reference raises (take_one_sample's int(nan)) in a run in which a source that
    # reaches no follower with positive significance actually posts: when such sources
    # exist, the batch keeps its event logs and every replica's log is checked
    from .opt_model import _sig_bad_sources, _sig_reach_check
    bad = set()
    for q in qv:
        bad |= _sig_bad_sources(g, sim_opts.edge_list, spw, float(q))
    R = len(seeds)
    seed_t = torch.as_tensor(np.tile(seeds, len(qv)))
    res = g.run("sig", q=qv, s_pw=spw, period=float(time_period), n_rep=R, ctrl_seed=seed_t,
                world_seed=seed_t, randomize=randomize, Ks=Ks, max_events=max_events,
                event_log=bool(bad))
    if bad:
        n = res.counts[:, 2].cpu().numpy()
        src = res.ev_src.cpu().numpy()
        ids = g.stream_src_ids
        for i in range(src.shape[0]):
            _sig_reach_check(g, sim_opts.edge_list, spw, 1.0, ids[src[i, :n[i]]], bad=bad,
                             max_events=max_events)
    return _frame(res, np.tile(seeds, len(qv)), np.repeat(qv, R), "OptPW", Ks)
