"""Drop-in surface of the reference's ``redqueen/utils.py`` metric functions.

``time_in_top_k`` / ``average_rank`` / ``int_r_2`` / ``num_tweets_of``
(utils.py:84-121, :170-176) take a dataframe in the reference's row layout
and return numpy float64 scalars, computed by ``rq_metrics_replay`` on the GPU
with the reference's exact arithmetic (rank scan, pivot mean, ffill, numpy
pairwise sums).  The only host work is handing the
columns over to device memory: sink ids go over raw and the pivot columns are
built on the device.  ``replay_frames`` / ``replay_columns`` replay many
dataframes in one batched call (rq_metrics_replay_batch).
``calc_q_capacity_iter`` (utils.py:447-470) runs its seeds as one GPU batch.

Analysis helpers on the same footing: ``rank_of_src_in_df`` (utils.py:38-56)
and ``u_int_opt`` (:59-81) run ``rq_rank_table`` / ``rq_u_int``;
``oracle_ranking`` (:181-245) runs the oracle's O(n^2) dynamic program as
``rq_oracle_dp`` (one workgroup per wall, batched over walls / q values), and
``get_oracle_df`` / ``find_opt_oracle`` (:248-340) and ``sweep_q`` (:521-607)
keep the reference's control flow around GPU batches.
"""
import ctypes as C
import datetime as D
import logging
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


def _replay_ws(dev, nbytes):
    ws = _WS.get(dev.index)
    if ws is None or ws.numel() < nbytes:
        _WS[dev.index] = None
        ws = torch_empty_u8(nbytes, dev)
        _WS[dev.index] = ws
    return ws


def torch_empty_u8(n, dev):
    import torch
    return torch.empty(max(256, int(n)), dtype=torch.uint8, device=dev)


def replay_columns(t, src, sink, eid=None, df_off=None, src_id=0, end_time=0.0, Ks=(1,), chunked=None):
    """rq_metrics_replay(_batch) on device columns (torch tensors: t f64, src / sink /
    event_id i64, df_off i64 [n_df + 1] or None for one dataframe).  Sink ids are raw:
    the pivot columns are built on the device.  Returns (metrics [n_df, nK + 2],
    counts [n_df, 4]) device tensors; counts[:, 2] < 0 flags a rejected dataframe
    (RQ_EUNSORTED).  Dataframes wider than the LDS tables are rerun with the large
    workspace, as the engine reruns overflowing replicas.  ``chunked``: None = give
    few long dataframes the chunked (many-workgroup) replay's workspace; True / False
    = always / never (A/B; the library then picks the path, env RQ_RP_CHUNK forces it)."""
    import torch
    from . import _lib as L
    dev = t.device
    n = int(t.numel())
    n_df = 1 if df_off is None else int(df_off.numel()) - 1
    Ks = np.ascontiguousarray(Ks, dtype=np.int32)
    out = torch.empty((n_df, Ks.size + 2), dtype=torch.float64, device=dev)
    cnt = torch.empty((n_df, 4), dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    lib = L.lib()
    # few long dataframes: room for the chunked (many-workgroup) replay
    if chunked is None:
        chunked = n_df <= 64 and n >= 2 * L.REPLAY_CHUNK_ROWS * n_df
    f0 = L.REPLAY_CHUNKED if chunked else 0
    for flags in (f0, f0 | L.REPLAY_LARGE):
        nbytes = C.c_size_t()
        L.check("rq_replay_workspace_size",
                lib.rq_replay_workspace_size(n, n_df, Ks.size, flags, C.byref(nbytes)))
        ws = _replay_ws(dev, nbytes.value)
        ptr = lambda x: x.data_ptr() if x is not None and x.numel() else None  # noqa: E731
        args = (ptr(t), ptr(src), ptr(sink), ptr(eid))
        tail = (int(src_id), float(end_time), Ks.ctypes.data_as(L._pi32), Ks.size,
                out.data_ptr(), cnt.data_ptr(), ws.data_ptr(), ws.numel(), st)
        if df_off is None:
            L.check("rq_metrics_replay", lib.rq_metrics_replay(*args, n, *tail))
        else:
            L.check("rq_metrics_replay_batch",
                    lib.rq_metrics_replay_batch(*args, df_off.data_ptr(), n_df, n, *tail))
        if (flags & L.REPLAY_LARGE) or not bool((cnt[:, 2] == L.RQ_EOVERFLOW).any().item()):
            break
    return out, cnt


def replay_metrics(df, src_id, end_time, Ks=(1,)):
    """All metrics of one df in one GPU pass.  Returns dict with top_k (list),
    avg_rank, r_2, num_own, num_world, rows, cols."""
    import torch
    from . import _lib as L
    if len(df) == 0:
        raise KeyError("empty dataframe")   # the reference fails on an empty df too
    dev = torch.device("cuda", torch.cuda.current_device())

    def col(name):
        return torch.from_numpy(np.ascontiguousarray(df[name].values, dtype=np.int64)).to(dev)
    tt = torch.from_numpy(np.ascontiguousarray(df["t"].values, dtype=np.float64)).to(dev)
    te = col("event_id") if "event_id" in df.columns else None
    o, c = replay_columns(tt, col("src_id"), col("sink_id"), te, None, src_id, end_time, Ks)
    o = o[0].cpu().numpy()
    c = c[0].cpu().numpy()
    nK = len(Ks)
    if c[2] == L.RQ_EUNSORTED:
        raise L.RQError("rq_metrics_replay (df 't' column must be non-decreasing)",
                        L.RQ_EUNSORTED)
    if c[2] < 0:
        raise L.RQError("rq_metrics_replay", int(c[2]))
    return {"top_k": [np.float64(v) for v in o[:nK]], "avg_rank": np.float64(o[nK]),
            "r_2": np.float64(o[nK + 1]), "num_own": int(c[0]), "num_world": int(c[1]),
            "rows": int(c[2]), "cols": int(c[3])}


def replay_frames(dfs, src_id, end_time, Ks=(1,)):
    """Metrics of many dataframes (the reference's per-replica utils calls) in one
    batched replay: a pandas DataFrame with top_K..., avg_rank, r_2, num_events,
    world_events per input df."""
    import pandas as pd
    import torch
    cols = ["top_" + str(k) for k in Ks] + ["avg_rank", "r_2", "num_events", "world_events",
                                            "pivot_rows", "sinks"]
    dfs = list(dfs)
    if not dfs:
        return pd.DataFrame({c: [] for c in cols})
    has_eid = ["event_id" in d.columns for d in dfs]
    if any(has_eid) and not all(has_eid):
        # world_events needs every dataframe's event ids (num_tweets_of / add_perf count
        # distinct event_id values): refuse rather than drop them for all dataframes
        raise ValueError("replay_frames: %d of %d dataframes lack an 'event_id' column" %
                         (has_eid.count(False), len(dfs)))
    dev = torch.device("cuda", torch.cuda.current_device())
    lens = np.asarray([len(d) for d in dfs], dtype=np.int64)
    off = torch.from_numpy(np.concatenate([[0], np.cumsum(lens)])).to(dev)

    def cat(name, dt):
        return torch.from_numpy(np.ascontiguousarray(
            np.concatenate([d[name].values for d in dfs]) if len(dfs) else np.zeros(0), dtype=dt)).to(dev)
    eid = cat("event_id", np.int64) if all(has_eid) else None
    o, c = replay_columns(cat("t", np.float64), cat("src_id", np.int64), cat("sink_id", np.int64),
                          eid, off, src_id, end_time, Ks)
    o, c = o.cpu().numpy(), c.cpu().numpy()
    res = {("top_" + str(k)): o[:, i] for i, k in enumerate(Ks)}
    res.update(avg_rank=o[:, len(Ks)], r_2=o[:, len(Ks) + 1], num_events=c[:, 0],
               world_events=c[:, 1], pivot_rows=c[:, 2], sinks=c[:, 3])
    return pd.DataFrame(res)


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


# ------------------------------------------------------------- rank table / u_int
def _dev():
    import torch
    return torch.device("cuda", torch.cuda.current_device())


def _put(a, dtype):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a, dtype=dtype)).to(_dev())


def _rank_table_dev(df, src_id, fill=True, with_time=True):
    """rq_rank_table on the df columns; returns (table, index) device tensors + sink ids."""
    import torch
    from . import _lib as L
    if len(df) == 0:
        raise ValueError("No objects to concatenate")   # pandas' pivot of an empty df
    key = df["t"].values if with_time else df["event_id"].values
    t = np.ascontiguousarray(key, dtype=np.float64)
    sinks, col = np.unique(df["sink_id"].values, return_inverse=True)
    n_t = int(np.unique(t).size)
    S = int(sinks.size)
    dev = _dev()
    tab = torch.empty((n_t, S), dtype=torch.float64, device=dev)
    idx = torch.empty(n_t, dtype=torch.float64, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    tt, ts, tc = _put(t, np.float64), _put(df["src_id"].values, np.int64), _put(col, np.int32)
    st = torch.cuda.current_stream().cuda_stream
    L.check("rq_rank_table", L.lib().rq_rank_table(
        tt.data_ptr(), ts.data_ptr(), tc.data_ptr(), t.size, S, int(src_id), int(bool(fill)), n_t,
        tab.data_ptr(), idx.data_ptr(), err.data_ptr(), st))
    if int(err.item()) & 1:
        raise L.RQError("rq_rank_table (df must be sorted by its pivot index)", L.RQ_EUNSORTED)
    return tab, idx, sinks


def rank_of_src_in_df(df, src_id, fill=True, with_time=True):
    """Calculates the rank of the src_id at each time instant in the list of events
    (utils.py:38-56): a DataFrame indexed by the unique t (or event_id), one column
    per sink_id, computed by rq_rank_table."""
    import pandas as pd
    tab, idx, sinks = _rank_table_dev(df, src_id, fill, with_time)
    index = idx.cpu().numpy()
    if not with_time:
        index = index.astype(np.int64)
    return pd.DataFrame(tab.cpu().numpy(), index=pd.Index(index, name="t" if with_time else "event_id"),
                        columns=pd.Index(sinks, name="sink_id"))


def u_int_opt(df, src_id=None, end_time=None, s=None, q=None, follower_ids=None, sim_opts=None):
    """Calculate the integral of u(t) for the given src_id assuming that the
    broadcaster was following the optimal strategy (utils.py:59-81):
    sum_k (r_k[followers] . sqrt(s/q)) * dt_k on the GPU rank table.  The row dot
    runs in follower order (the reference's BLAS dgemv may associate differently:
    equal to ~1e-15 relative, not bit for bit)."""
    import torch
    from . import _lib as L
    if sim_opts is not None:
        src_id = mb(src_id, sim_opts.src_id)
        end_time = mb(end_time, sim_opts.end_time)
        s = mb(s, sim_opts.s)
        q = mb(q, sim_opts.q)
        follower_ids = mb(follower_ids, sim_opts.sink_ids)
    if follower_ids is None:
        follower_ids = sorted(df.sink_id[df.src_id == src_id].unique())
    tab, idx, sinks = _rank_table_dev(df, src_id)
    pos = {int(x): i for i, x in enumerate(sinks)}
    missing = [f for f in follower_ids if int(f) not in pos]
    if missing:
        raise KeyError("{} not in index".format(missing))
    fcol = np.asarray([pos[int(f)] for f in follower_ids], dtype=np.int32)
    if np.ndim(s) == 0:
        # a scalar s: the reference's `r_t[follower_ids].values.dot(np.sqrt(s / q))`
        # scales the [n_t, F] rank block instead of reducing it, and `u_values * u_dt`
        # then broadcasts ([n_t, n_t] for one follower, a ValueError for most F) --
        # the same numpy expression on the GPU-built rank table, errors included
        r = tab.cpu().numpy()[:, fcol]
        u_values = r.dot(np.sqrt(s / q))
        u_dt = np.diff(np.concatenate([idx.cpu().numpy(), [end_time]]))
        return np.sum(u_values * u_dt)
    wts = np.sqrt(np.asarray(s, dtype=np.float64) / q) * np.ones(len(fcol))
    n_t = tab.shape[0]
    ws = torch.empty(max(1, n_t), dtype=torch.float64, device=_dev())
    out = torch.empty(1, dtype=torch.float64, device=_dev())
    tf, tw = _put(fcol, np.int32), _put(wts, np.float64)
    st = torch.cuda.current_stream().cuda_stream
    L.check("rq_u_int", L.lib().rq_u_int(tab.data_ptr(), idx.data_ptr(), n_t, tab.shape[1],
                                         tf.data_ptr(), tw.data_ptr(), len(fcol), float(end_time),
                                         out.data_ptr(), ws.data_ptr(), ws.numel() * 8, st))
    return np.float64(out.item())


# -------------------------------------------------------------------- the oracle
def _oracle_w(df, end_time):
    """event_times = df.groupby('event_id').t.mean(); w = np.diff([0, 0, times, end])
    (utils.py:200-207)."""
    event_times = df.groupby('event_id').t.mean()
    w = np.diff(np.concatenate([[0.0], [0.0], event_times.values, [end_time]]))
    return event_times, w


def oracle_dp_batch(ws, qs, ss):
    """rq_oracle_dp over several walls at once: ws[i] = w of wall i (len n_i + 2),
    qs[i], ss[i] its q and s.  Returns [(cost, events, ranks)] (numpy)."""
    import torch
    from . import _lib as L
    n = np.asarray([len(w) - 2 for w in ws], dtype=np.int64)
    if np.any(n < 0):
        raise ValueError("w needs n + 2 >= 2 entries")
    if len(ws) == 0:
        return []
    w_off = np.concatenate([[0], np.cumsum(n + 2)]).astype(np.int64)
    o_off = np.concatenate([[0], np.cumsum(n + 1)]).astype(np.int64)
    n_max = int(n.max())
    nbytes = C.c_size_t()
    L.check("rq_oracle_workspace_size", L.lib().rq_oracle_workspace_size(len(ws), n_max, C.byref(nbytes)))
    dev = _dev()
    wsp = torch.empty(nbytes.value, dtype=torch.uint8, device=dev)
    tw = _put(np.concatenate([np.asarray(w, dtype=np.float64) for w in ws]), np.float64)
    twoff, tooff = _put(w_off, np.int64), _put(o_off, np.int64)
    tq, tsv = _put(qs, np.float64), _put(ss, np.float64)
    cost = torch.empty(len(ws), dtype=torch.float64, device=dev)
    ev = torch.empty(int(o_off[-1]), dtype=torch.int32, device=dev)
    rk = torch.empty(int(o_off[-1]), dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    L.check("rq_oracle_dp", L.lib().rq_oracle_dp(
        tw.data_ptr(), twoff.data_ptr(), tq.data_ptr(), tsv.data_ptr(), len(ws), n_max,
        cost.data_ptr(), ev.data_ptr(), rk.data_ptr(), tooff.data_ptr(), wsp.data_ptr(),
        wsp.numel(), st))
    c, e, r = cost.cpu().numpy(), ev.cpu().numpy(), rk.cpu().numpy()
    return [(np.float64(c[i]), e[o_off[i]:o_off[i + 1]].astype(np.int64),
             r[o_off[i]:o_off[i + 1]].astype(np.int64)) for i in range(len(ws))]


def _scalar_s(s):
    if isinstance(s, dict):
        raise TypeError("unsupported operand type(s) for *: 'float' and 'dict'")
    a = np.asarray(s, dtype=np.float64).ravel()
    if a.size != 1:
        raise ValueError("oracle_ranking is implemented for one follower (s must be a scalar)")
    return float(a[0])


def oracle_ranking(df, sim_opts, omit_src_ids=None, follower_ids=None):
    """Returns the best places the oracle would have put events (utils.py:181-245).
    Optionally, it can remove sources, use a custom weight vector and have a
    custom list of followers.  The DP runs on the GPU (rq_oracle_dp)."""
    import pandas as pd
    if omit_src_ids is not None:
        df = df[~df.src_id.isin(omit_src_ids)]

    if follower_ids is not None:
        df = sorted(df[df.sink_id.isin(follower_ids)])   # sic (utils.py:190)
    else:
        follower_ids = sorted(df.sink_id.unique())

    assert len(follower_ids) == 1, "Oracle has been implemented only for 1 follower."

    q = sim_opts.q
    s = sim_opts.s
    event_times, w = _oracle_w(df, sim_opts.end_time)
    n = event_times.shape[0]
    if n > 1e6:
        logging.error('Not running for n > 1e6 events')
        return []
    (cost, u_star, oracle_ranks), = oracle_dp_batch([w], [float(q)], [_scalar_s(s)])
    oracle_df = pd.DataFrame.from_dict({
        'ranks': oracle_ranks,
        'events': u_star,
        'at': np.concatenate([[0.0], event_times.values]),
        't': np.concatenate([[0.0], event_times.values]),
        't_delta': w[1:]
    })
    return oracle_df, cost


def _wall_df(sim_opts):
    wall_mgr = sim_opts.create_manager_for_wall()
    wall_mgr.run_dynamic()
    return wall_mgr.state.get_dataframe()


def get_oracle_df(sim_opts, with_cost=False):
    """utils.py:248-257: oracle on the wall of sim_opts' other sources."""
    oracle_df, cost = oracle_ranking(df=_wall_df(sim_opts), sim_opts=sim_opts)
    if with_cost:
        return oracle_df, cost
    else:
        return oracle_df


def _oracle_search(target_events, max_events=None, tol=1e-2, verbose=False):
    """find_opt_oracle's q search (utils.py:260-340) as a coroutine: yields the next q
    to try, receives (event count, cost) of the oracle there, and returns (q, key) -- key is
    the reference's result key ('oracle_df' when q = 1 already meets the target,
    utils.py:277, else 'df').  The exponential search and the bisection are the
    reference's step for step; only the DP evaluations are batched by the driver."""
    q_hi, q_init, q_lo = 1.0 * 2, 1.0, 1.0 / 2

    def terminate_cond(opt_events):
        return np.abs(opt_events - target_events) / (target_events * 1.0) < tol or \
            (opt_events == np.ceil(target_events)) or \
            (opt_events == np.floor(target_events))

    num_events, _ = yield q_init
    if terminate_cond(num_events):
        return q_init, 'oracle_df'   # sic: key (utils.py:277)

    if num_events > target_events:
        while True:
            q_lo = q_init
            q_init *= 2
            q_hi = q_init
            num_events, _ = yield q_init
            if verbose:
                logTime('q_lo = {}, q_hi = {}, num_events = {} '.format(q_lo, q_hi, num_events))
            if terminate_cond(num_events):
                return q_init, 'df'
            if num_events <= target_events:
                break
    elif num_events < target_events:
        while True:
            q_hi = q_init
            q_init /= 2
            q_lo = q_init
            num_events, _ = yield q_init
            if verbose:
                logTime('q_lo = {}, q_hi = {}, num_events = {} '.format(q_lo, q_hi, num_events))
            if terminate_cond(num_events):
                return q_init, 'df'
            if num_events >= target_events or num_events == max_events:
                break

    if verbose:
        logTime('q_lo = {}, q_hi = {}'.format(q_lo, q_hi))

    while True:
        q_try = (q_lo + q_hi) / 2.0
        opt_events, cost = yield q_try
        if verbose:
            logTime('q_try = {}, events = {}, cost = {}'.format(q_try, opt_events, cost))
        if terminate_cond(opt_events):
            return q_try, 'df'
        elif opt_events < target_events:
            q_hi = q_try
        else:
            q_lo = q_try


def find_opt_oracle_batch(targets, sim_opts_list, max_events=None, walls=None, tol=1e-2,
                          verbose=False):
    """find_opt_oracle for many (target, sim_opts) at once: every search advances in
    lockstep and each round of q evaluations is ONE rq_oracle_dp launch over all the
    searches still running (one workgroup per wall).  ``walls``: the wall dataframes
    (default: each sim_opts' wall, simulated once).  Returns the reference's result
    dicts, in order."""
    import pandas as pd
    n = len(targets)
    max_events = [None] * n if max_events is None else list(max_events)
    if walls is None:
        walls = [_wall_df(so) for so in sim_opts_list]
    prep = []
    for k in range(n):
        wdf = walls[k]
        follower_ids = sorted(wdf.sink_id.unique())
        assert len(follower_ids) == 1, "Oracle has been implemented only for 1 follower."
        event_times, w = _oracle_w(wdf, sim_opts_list[k].end_time)
        if event_times.shape[0] > 1e6:   # oracle_ranking returns [] (utils.py:205-207)
            logging.error('Not running for n > 1e6 events')
            raise ValueError("not enough values to unpack (expected 2, got 0)")
        prep.append((event_times, w, _scalar_s(sim_opts_list[k].s)))
    gens = [_oracle_search(targets[k], max_events[k], tol, verbose) for k in range(n)]
    q_next = [g.send(None) for g in gens]
    last = [None] * n
    out = [None] * n
    active = list(range(n))
    while active:
        res = oracle_dp_batch([prep[k][1] for k in active], [float(q_next[k]) for k in active],
                              [prep[k][2] for k in active])
        still = []
        for k, (cost, ev, rk) in zip(active, res):
            last[k] = (q_next[k], cost, ev, rk)
            try:
                q_next[k] = gens[k].send((int(ev.sum()), cost))
                still.append(k)
            except StopIteration as stop:
                q, key = stop.value
                event_times, w, _ = prep[k]
                oracle_df = pd.DataFrame.from_dict({
                    'ranks': rk, 'events': ev,
                    'at': np.concatenate([[0.0], event_times.values]),
                    't': np.concatenate([[0.0], event_times.values]),
                    't_delta': w[1:]})
                out[k] = {'q': q, 'cost': cost, key: oracle_df}
        active = still
    return out


def find_opt_oracle(target_events, sim_opts, max_events=None, tol=1e-2, verbose=False):
    """Sweep q and get the best run of the oracle (utils.py:260-340): the
    reference's exponential search + bisection, each step one GPU DP on the
    (deterministic) wall, which is simulated once."""
    return find_opt_oracle_batch([target_events], [sim_opts], [max_events], tol=tol,
                                 verbose=verbose)[0]


def find_opt_oracle_q(target_events, sim_opts, tol=1e-1, verbose=False):
    res = find_opt_oracle(target_events, sim_opts, tol, verbose)   # sic: tol -> max_events
    return res['q']


def find_opt_oracle_time_top_k(target_events, K, sim_opts, tol=1e-1, verbose=False):
    logTime('This method is incorrect.')
    res = find_opt_oracle(target_events, sim_opts, tol, verbose)
    df = res['df']
    return np.sum(df.t_delta[df.ranks <= K - 1])


# --------------------------------------------------------------------- sweep_q
def q_int_worker(params):
    sim_opts, seed, dynamic, max_events = params
    return calc_q_capacity_iter(sim_opts, sim_opts.q, seeds=[seed], max_events=max_events)[0]


def sweep_q(sim_opts, capacity_cap, tol=1e-2, verbose=False, q_init=None, parallel=True,
            dynamic=True, max_events=None, max_iters=float('inf'), only_tol=False):
    """Find q whose mean RedQueen capacity over seeds 100..119 meets capacity_cap
    (utils.py:521-607): the reference's exponential bracket + bisection; every
    capacity estimate is one GPU batch (calc_q_capacity_iter)."""
    # We know that on average, the integral of u(t) decreases with increasing 'q'

    def terminate_cond(new_capacity):
        return abs(new_capacity - capacity_cap) / capacity_cap < tol or \
            (not only_tol and np.ceil(capacity_cap - 1) <= new_capacity <= np.ceil(capacity_cap + 1))

    def cap_at(q):
        return calc_q_capacity_iter(sim_opts, q, dynamic=dynamic, parallel=parallel,
                                    max_events=max_events).mean()

    if q_init is None:
        r_t = rank_of_src_in_df(_wall_df(sim_opts), -1)
        q_init = (4 * (r_t.iloc[-1].mean() ** 2) * (sim_opts.end_time) ** 2) / \
            (np.pi * np.pi * (capacity_cap + 1) ** 4)
        if verbose:
            logTime('q_init = {}'.format(q_init))

    # Step 1: Find the upper/lower bound by exponential increase/decrease
    init_cap = cap_at(q_init)
    if terminate_cond(init_cap):
        return q_init
    if verbose:
        logTime('Initial capacity = {}, target capacity = {}, q_init = {}'
                .format(init_cap, capacity_cap, q_init))

    q = q_init
    if init_cap < capacity_cap:
        iters = 0
        while True:
            iters += 1
            q_hi = q
            q /= 2.0
            q_lo = q
            capacity = cap_at(q)
            if verbose:
                logTime('q = {}, capacity = {}'.format(q, capacity))
            if terminate_cond(capacity):
                return q
            if capacity >= capacity_cap:
                break
            if iters > max_iters:
                if verbose:
                    logTime('Breaking because of max-iters: {}.'.format(max_iters))
                return q
    else:
        iters = 0
        while True:
            iters += 1
            q_lo = q
            q *= 2.0
            q_hi = q
            capacity = cap_at(q)
            if verbose:
                logTime('q = {}, capacity = {}'.format(q, capacity))
            if terminate_cond(capacity):
                return q
            if capacity <= capacity_cap:
                break
            if iters > max_iters:
                if verbose:
                    logTime('Breaking because of max-iters: {}.'.format(max_iters))
                return q

    if verbose:
        logTime('q_hi = {}, q_lo = {}'.format(q_hi, q_lo))

    # Step 2: Keep bisecting on 's' until we arrive at a close enough solution.
    while True:
        q = (q_hi + q_lo) / 2.0
        new_capacity = cap_at(q)
        if verbose:
            logTime('new_capacity = {}, q = {}'.format(new_capacity, q))
        if terminate_cond(new_capacity):
            break
        elif new_capacity > capacity_cap:
            q_lo = q
        else:
            q_hi = q

    # Step 3: Return
    return q


# ------------------------------------------------------------ significance sweeps
def significance_q_int_worker(params):
    sim_opts, seed, time_period = params
    m = sim_opts.create_manager_with_significance(seed, significance=sim_opts.s,
                                                  time_period=time_period)
    m.run_dynamic()
    return num_tweets_of(m.state.get_dataframe(), sim_opts=sim_opts)


def calc_significance_capacity_iter(sim_opts, q, time_period, seeds=None, parallel=True,
                                    max_events=None):
    """OptPWSignificance capacities per seed at this q (utils.py:496-518), with
    sim_opts.s as the [sinks x segments] significance.  parallel=True (the
    reference's pool path: posts per replica) is one GPU batch over the seeds;
    parallel=False keeps the reference's sequential path, which scores u_int_opt."""
    from .batch import compiled_graph
    import torch
    if seeds is None:
        seeds = range(1000, 1025)
    sim_opts = sim_opts.update({'q': q})
    seeds = np.asarray(list(seeds), dtype=np.int64)
    if not parallel:
        capacities = np.zeros(len(seeds), dtype=float)
        for idx, seed in enumerate(seeds):
            m = sim_opts.create_manager_with_significance(seed=int(seed), significance=sim_opts.s,
                                                          time_period=time_period)
            m.run_dynamic()
            capacities[idx] = u_int_opt(m.state.get_dataframe(), sim_opts=sim_opts)
        return capacities
    from .opt_model import OptPWSignificance
    g = compiled_graph(sim_opts)
    sig = np.asarray(sim_opts.s, dtype=float)
    assert sig.ndim == 2 and sig.shape[0] == len(sim_opts.sink_ids), \
        "Number of sink_ids is not the same as size of significance."
    spw = OptPWSignificance(sim_opts.src_id, 0, sig, time_period, q)._s_pw_for(g.n_followers)
    res = g.run("sig", q=float(q), s_pw=spw, period=float(time_period), n_rep=len(seeds),
                ctrl_seed=torch.as_tensor(seeds), max_events=max_events)
    return res.num_events.double().cpu().numpy()


def sweep_q_with_significance(sim_opts, capacity_cap, time_period, tol=1e-2, parallel=True,
                              verbose=False, q_init=None):
    """utils.py:610-700: sweep_q for the OptPWSignificance broadcaster; every
    capacity estimate is one GPU batch (calc_significance_capacity_iter)."""

    def terminate_cond(new_capacity):
        return abs(new_capacity - capacity_cap) / capacity_cap < tol or \
            np.ceil(capacity_cap - 1) <= new_capacity <= np.ceil(capacity_cap + 1)

    def cap_at(q):
        return calc_significance_capacity_iter(sim_opts=sim_opts, q=q, time_period=time_period,
                                               parallel=parallel).mean()

    if q_init is None:
        r_t = rank_of_src_in_df(_wall_df(sim_opts), -1)
        q_init = (4 * (r_t.iloc[-1].mean() ** 2) * (sim_opts.end_time) ** 2) / \
            (np.pi * np.pi * (capacity_cap + 1) ** 4)
        if verbose:
            logTime('q_init = {}'.format(q_init))

    init_cap = cap_at(q_init)
    if terminate_cond(init_cap):
        logTime('q_init meets the conditions.')
        return q_init
    if verbose:
        logTime('Initial capacity = {}, target capacity = {}, q_init = {}'
                .format(init_cap, capacity_cap, q_init))

    q = q_init
    if init_cap < capacity_cap:
        while True:
            q_hi = q
            q /= 2.0
            q_lo = q
            capacity = cap_at(q)
            if verbose:
                logTime('q = {}, capacity = {}'.format(q, capacity))
            if terminate_cond(capacity):
                return q
            if capacity >= capacity_cap:
                break
    else:
        while True:
            q_lo = q
            q *= 2.0
            q_hi = q
            capacity = cap_at(q)
            if verbose:
                logTime('q = {}, capacity = {}'.format(q, capacity))
            if terminate_cond(capacity):
                return q
            if capacity <= capacity_cap:
                break

    if verbose:
        logTime('q_hi = {}, q_lo = {}'.format(q_hi, q_lo))

    while True:
        q = (q_hi + q_lo) / 2.0
        new_capacity = cap_at(q)
        if verbose:
            logTime('new_capacity = {}, q = {}'.format(new_capacity, q))
        if terminate_cond(new_capacity):
            break
        elif new_capacity > capacity_cap:
            q_lo = q
        else:
            q_hi = q
    return q
