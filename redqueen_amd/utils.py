"""Drop-in surface of the reference's ``redqueen/utils.py`` metric functions.

``time_in_top_k`` / ``average_rank`` / ``int_r_2`` / ``num_tweets_of``
(utils.py:84-121, :170-176) take a dataframe in the reference's row layout
and return numpy float64 scalars, computed by ``rq_metrics_replay`` on the GPU
with the reference's exact arithmetic (rank scan, pivot mean, ffill, numpy
pairwise sums).  The only host work is handing the
columns over: the df's sink ids are factorised into pivot-column indices
(np.unique) and the columns are copied to device memory.
``calc_q_capacity_iter`` (utils.py:447-470) runs its seeds as one GPU batch.
"""
import ctypes as C
import datetime as D
import sys

import numpy as np


def mb(val, default):
    return val if val is not None else default


def logTime(chkpoint):
    print('*** \x1b[31m{}\x1b[0m Checkpoint: {}'.format(D.datetime.now(), chkpoint))
    sys.stdout.flush()


def def_s_vec(num_followers):
    return np.ones(num_followers, dtype=float) / (num_followers ** 2)


def is_sorted(x, ascending=True):
    return np.all((np.diff(x) * (1.0 if ascending else -1.0) >= 0))


# ------------------------------------------------------------------ GPU replay
_WS = {}


def replay_metrics(df, src_id, end_time, Ks=(1,)):
    """All metrics of one df in one GPU pass.  Returns dict with top_k (list),
    avg_rank, r_2, num_own, num_world, rows, cols."""
    import torch
    from . import _lib as L
    if len(df) == 0:
        raise KeyError("empty dataframe")   # the reference fails on an empty df too
    dev = torch.device("cuda", torch.cuda.current_device())
    t = np.ascontiguousarray(df["t"].values, dtype=np.float64)
    src = np.ascontiguousarray(df["src_id"].values, dtype=np.int64)
    sinks, col = np.unique(df["sink_id"].values, return_inverse=True)
    col = np.ascontiguousarray(col, dtype=np.int32)
    eid = np.ascontiguousarray(df["event_id"].values, dtype=np.int64) \
        if "event_id" in df.columns else None
    n, S = t.size, int(sinks.size)
    Ks = np.ascontiguousarray(Ks, dtype=np.int32)
    nbytes = C.c_size_t()
    L.check("rq_replay_workspace_size", L.lib().rq_replay_workspace_size(n, S, C.byref(nbytes)))
    ws = _WS.get(dev.index)
    if ws is None or ws.numel() < nbytes.value:
        ws = torch.empty(nbytes.value, dtype=torch.uint8, device=dev)
        _WS[dev.index] = ws
    tt = torch.from_numpy(t).to(dev)
    ts = torch.from_numpy(src).to(dev)
    tc = torch.from_numpy(col).to(dev)
    te = torch.from_numpy(eid).to(dev) if eid is not None else None
    out = torch.empty(Ks.size + 2, dtype=torch.float64, device=dev)
    cnt = torch.empty(4, dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    L.check("rq_metrics_replay", L.lib().rq_metrics_replay(
        tt.data_ptr(), ts.data_ptr(), tc.data_ptr(), te.data_ptr() if te is not None else None,
        n, S, int(src_id), float(end_time), Ks.ctypes.data_as(L._pi32), Ks.size,
        out.data_ptr(), cnt.data_ptr(), ws.data_ptr(), ws.numel(), st))
    o = out.cpu().numpy()
    c = cnt.cpu().numpy()
    if c[2] < 0:
        raise L.RQError("rq_metrics_replay (df 't' column must be non-decreasing)",
                        L.RQ_EUNSORTED)
    return {"top_k": [np.float64(v) for v in o[:Ks.size]], "avg_rank": np.float64(o[Ks.size]),
            "r_2": np.float64(o[Ks.size + 1]), "num_own": int(c[0]), "num_world": int(c[1]),
            "rows": int(c[2]), "cols": int(c[3])}


def time_in_top_k(df, K, src_id=None, end_time=None, sim_opts=None):
    """Calculate int I(r(t) <= k) dt for the given src_id (utils.py:84-98)."""
    if sim_opts is not None:
        src_id = mb(src_id, sim_opts.src_id)
        end_time = mb(end_time, sim_opts.end_time)
    return replay_metrics(df, src_id, end_time, (K,))["top_k"][0]


def average_rank(df, src_id=None, end_time=None, sim_opts=None, **kwargs):
    """Calculate int r(t) dt for the given src_id (utils.py:101-114)."""
    if sim_opts is not None:
        src_id = mb(src_id, sim_opts.src_id)
        end_time = mb(end_time, sim_opts.end_time)
    return replay_metrics(df, src_id, end_time, (1,))["avg_rank"]


def int_r_2(df, sim_opts):
    """Returns int avg-rank^2(t) dt (utils.py:117-121)."""
    return replay_metrics(df, sim_opts.src_id, sim_opts.end_time, (1,))["r_2"]


def num_tweets_of(df, broadcaster_id=None, sim_opts=None):
    """Number of distinct events of the broadcaster in the df (utils.py:170-176)."""
    if sim_opts is not None:
        broadcaster_id = mb(broadcaster_id, sim_opts.src_id)
    assert broadcaster_id is not None, "Must either provide either broadcaster_id or sim_opts."
    end = float(df["t"].max()) if len(df) else 0.0
    return 1.0 * replay_metrics(df, broadcaster_id, end, (1,))["num_own"]


def add_perf(op, df, sim_opts, Ks=(1,)):
    """opt_runs.add_perf (opt_runs.py:41-48) in one GPU pass."""
    m = replay_metrics(df, sim_opts.src_id, sim_opts.end_time, tuple(Ks))
    for k, v in zip(Ks, m["top_k"]):
        op['top_' + str(k)] = v
    op['avg_rank'] = m["avg_rank"]
    op['r_2'] = m["r_2"]
    op['world_events'] = m["num_world"]
    op['num_events'] = m["num_own"]
    return op


# ------------------------------------------------------------ q sweeps (batched)
def calc_q_capacity_iter(sim_opts, q, seeds=None, parallel=True, dynamic=True, max_events=None):
    """Posts of RedQueen per seed at this q (utils.py:447-470), all seeds as one
    GPU batch; ``parallel``/``dynamic`` are accepted for signature parity."""
    from .batch import compiled_graph
    if seeds is None:
        seeds = range(100, 120)
    seeds = np.asarray(list(seeds), dtype=np.int64)
    import torch
    g = compiled_graph(sim_opts)
    res = g.run("opt", q=float(q), s=sim_opts.s, n_rep=len(seeds),
                ctrl_seed=torch.as_tensor(seeds), max_events=max_events)
    return res.num_events.double().cpu().numpy()
