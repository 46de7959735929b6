"""Drop-in surface of the reference's ``redqueen/opt_runs.py`` workers.

``add_perf`` (opt_runs.py:41-48), ``worker_opt`` (:51-106), ``worker_poisson``
(:109-126) and ``worker_oracle`` (:129-155) keep their parameter tuples and
result dicts; each simulation is one GPU run (librq.so) and every metric one
``rq_metrics_replay`` pass.  For many seeds at once use ``redqueen_amd.batch``
(one launch for the whole grid) instead of a process pool.
"""
import logging

import numpy as np

from .utils import add_perf as _add_perf_ks
from .utils import find_opt_oracle


class _Options:
    """The fields of decorated_options.Options that opt_runs reads."""

    def __init__(self, **kw):
        self.__dict__.update(kw)

    def _get_dict(self):
        return dict(self.__dict__)

    def set_new(self, **kw):
        d = self._get_dict()
        d.update(kw)
        return _Options(**d)


Ks = [1]
perf_opts = _Options(oracle_eps=1e-10,  # This is how much after the event that the Oracle tweets.
                     Ks=Ks,
                     performance_fields=['seed', 'q', 'type'] +
                                        ['top_' + str(k) for k in Ks] +
                                        ['avg_rank', 'r_2', 'num_events', 'world_events'])


def add_perf(op, df, sim_opts):
    """opt_runs.add_perf: top_K for perf_opts.Ks, avg_rank, r_2, world_events,
    num_events -- one GPU replay of the df."""
    return _add_perf_ks(op, df, sim_opts, Ks=tuple(perf_opts.Ks))


def _wall_intensities(df, sim_opts, num_segments):
    """Posts per (sink, segment) / segment length, rows in sim_opts.sink_ids order
    (opt_runs.py:69-84; the reference's .ix lookup is .loc here: pandas >= 1.0)."""
    wall = df[df.src_id != sim_opts.src_id]
    T = sim_opts.end_time
    seg = (wall.t.values / T * num_segments).astype(int)
    sinks = list(sim_opts.sink_ids)
    pos = {s: i for i, s in enumerate(sinks)}
    segs = np.unique(seg)
    out = np.full((len(sinks), segs.size), np.nan)
    if segs.size:
        si = np.searchsorted(segs, seg)
        cnt = np.zeros_like(out)
        np.add.at(cnt, (np.asarray([pos[s] for s in wall.sink_id.values], dtype=int), si), 1.0)
        seen = cnt > 0
        out[seen] = cnt[seen] / (T / num_segments)
    return out


def worker_opt(params):
    try:
        seed, sim_opts, num_segments, queue = params
    except ValueError:
        logging.warning('Setting num_segments=10 for world-rate in worker_opt.')
        seed, sim_opts, queue = params
        num_segments = 10
    sim_mgr = sim_opts.create_manager_with_opt(seed=seed)
    sim_mgr.run_dynamic()
    df = sim_mgr.state.get_dataframe()
    num_events = len(df.event_id[df.src_id == sim_opts.src_id].unique())
    op = {
        'type': 'Opt',
        'seed': seed,
        'capacity': num_events * 1.0,
        'sim_opts': sim_opts,
        'q': sim_opts.q,
        'wall_intensities': _wall_intensities(df, sim_opts, num_segments),
    }
    add_perf(op, df, sim_opts)
    if queue is not None:
        queue.put(op)
    return op


def worker_poisson(params):
    seed, capacity, sim_opts, queue = params
    sim_mgr = sim_opts.create_manager_with_poisson(seed=seed, capacity=capacity)
    sim_mgr.run_dynamic()
    df = sim_mgr.state.get_dataframe()
    op = {'type': 'Poisson', 'seed': seed, 'sim_opts': sim_opts, 'q': sim_opts.q}
    add_perf(op, df, sim_opts)
    if queue is not None:
        queue.put(op)
    return op


def worker_oracle(params):
    """Oracle at the given capacity (find_opt_oracle on the GPU DP), replayed as a
    RealData broadcaster on the same world (opt_runs.py:129-155)."""
    seed, capacity, max_events, sim_opts, queue = params
    opt_oracle = find_opt_oracle(capacity, sim_opts, max_events=max_events)
    oracle_df = opt_oracle['df']   # sic: KeyError when q = 1 already meets the target
    opt_oracle_mgr = sim_opts.create_manager_with_times(oracle_df.t[oracle_df.events == 1] +
                                                        perf_opts.oracle_eps)
    opt_oracle_mgr.run_dynamic()
    df = opt_oracle_mgr.state.get_dataframe()
    op = {
        'type': 'Oracle',
        'seed': seed,
        'sim_opts': sim_opts,
        'q': sim_opts.q,
        'r0_num_events': np.sum(oracle_df.events == 1),
        'num_events': np.sum(df.src_id == sim_opts.src_id)
    }
    add_perf(op, df, sim_opts)
    if queue is not None:
        queue.put(op)
    return op
