"""Drop-in surface of the reference's ``redqueen/opt_runs.py`` workers.

``add_perf`` (opt_runs.py:41-48), ``worker_opt`` (:51-106), ``worker_poisson``
(:109-126) and ``worker_oracle`` (:129-155) keep their parameter tuples and
result dicts; each simulation is one GPU run (librq.so) and every metric one
``rq_metrics_replay`` pass.  For many seeds at once use ``redqueen_amd.batch``
(one launch for the whole grid) instead of a process pool.  ``run_inference`` /
``run_inference_queue`` (:350-440, :560-646) batch the q x seed grid on the GPU; the
multiple-follower helpers (``make_edge_list``, ``create_phased_pwconst_broadcaster``,
``trim_sim_opts``, ``prepare_multiple_followers_sim_opts``, :651-795) are host-side
network builders with the reference's draw order.
"""
import logging

import numpy as np

from .utils import add_perf as _add_perf_ks
from .utils import find_opt_oracle
from . import utils


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


def _optioned(fn):
    """decorated_options' @optioned('opts'): arguments not passed explicitly are taken
    from the ``opts`` bundle's fields."""
    import functools
    import inspect
    sig = inspect.signature(fn)

    @functools.wraps(fn)
    def wrapper(*args, **kwargs):
        opts = kwargs.pop("opts", None)
        if opts is not None:
            bound = sig.bind_partial(*args, **kwargs)
            for name in sig.parameters:
                if name not in bound.arguments and hasattr(opts, name):
                    kwargs[name] = getattr(opts, name)
        return fn(*args, **kwargs)
    return wrapper


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
    return _oracle_op(seed, sim_opts, opt_oracle, queue)


def _oracle_op(seed, sim_opts, opt_oracle, queue=None):
    """worker_oracle after its search (opt_runs.py:135-155)."""
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


def extract_perf_fields(return_obj, exclude_fields=None, include_fields=None):
    """opt_runs.extract_perf_fields (opt_runs.py:345-354), fields in
    perf_opts.performance_fields order (the reference iterates a set)."""
    include_fields = include_fields if include_fields is not None else set()
    exclude_fields = exclude_fields if exclude_fields is not None else set()
    fields = [f for f in perf_opts.performance_fields if f not in exclude_fields]
    fields += sorted(set(include_fields) - set(fields) - set(exclude_fields))
    return {f: return_obj[f] for f in fields}


def _world_key(so):
    """The world of a SimOpts without its sources' seeds (batchable replicas share it):
    the network, the sources' parameters and the followers' significance s (one batch
    runs every replica with one s per grid point)."""
    from .batch import _val_key
    s = so.s
    s_key = repr(sorted((int(k), float(v)) for k, v in s.items())) if isinstance(s, dict) \
        else _val_key(np.ravel(np.asarray(s, dtype=np.float64)))
    return (so.src_id, float(so.end_time), tuple(map(tuple, so.edge_list)), tuple(so.sink_ids),
            s_key,
            repr([(n if isinstance(n, str) else n.__name__,
                   sorted((k, _val_key(v)) for k, v in kw.items() if k != "seed"))
                  for n, kw in so.other_sources]))


def _randomize_seed(so):
    """u such that so's other sources carry the randomize_other_sources(u) seeds
    (u + 99 idx, opt_model.py:795-804), or None."""
    idx_seeds = [(i, kw["seed"]) for i, (_, kw) in enumerate(so.other_sources) if "seed" in kw]
    if len(idx_seeds) != len(so.other_sources):
        return None
    if not idx_seeds:
        return 0
    u = (int(idx_seeds[0][1]) - 99 * idx_seeds[0][0]) & 0xFFFFFFFF
    ok = all((int(s) & 0xFFFFFFFF) == ((u + 99 * i) & 0xFFFFFFFF) for i, s in idx_seeds)
    return u if ok else None


def _opt_poisson_batches(worlds, qs, seeds, num_segments):
    """worker_opt then worker_poisson for every (q, seed) as two GPU batches over the
    q x seed grid; worlds[k] = sim_opts_gen(seeds[k]) (one shared network whose
    sources carry randomize_other_sources(u_k) seeds).  Returns the op dicts in
    (q, seed) order: [(opt_op, poisson_op)]."""
    import torch
    from .batch import compiled_graph
    base = worlds[0]
    g = compiled_graph(base)
    N = len(seeds)
    us = np.asarray([_randomize_seed(w) for w in worlds], dtype=np.int64)
    sd = np.asarray(seeds, dtype=np.int64)
    Ks = tuple(perf_opts.Ks)
    qv = np.asarray(qs, dtype=np.float64)
    seed_t = torch.as_tensor(np.tile(sd, len(qv)))
    u_t = torch.as_tensor(np.tile(us, len(qv)))
    ro = g.run("opt", q=qv, s=g.s_matrix(base.s, len(qv)), n_rep=N, ctrl_seed=seed_t,
               world_seed=u_t, randomize=True, Ks=Ks, event_log=True)
    # capacity / end_time as create_manager_with_poisson divides (host IEEE division;
    # torch's tensor / scalar multiplies by the reciprocal)
    rate = ro.num_events.cpu().numpy().astype(np.float64) / float(base.end_time)
    rp = g.run("poisson", n_rep=len(qv) * N, ctrl_seed=seed_t, world_seed=u_t, randomize=True,
               ctrl_rate=torch.as_tensor(rate), Ks=Ks)
    ro_m, ro_c = ro.metrics.cpu().numpy(), ro.counts.cpu().numpy()
    rp_m, rp_c = rp.metrics.cpu().numpy(), rp.counts.cpu().numpy()
    row_off, cols = ro.log_columns()
    host = {k: v.cpu().numpy() for k, v in cols.items()}
    import pandas as pd
    out = []
    for gi, q in enumerate(qv):
        for k, seed in enumerate(sd):
            i = gi * N + k
            so = worlds[k].update({"q": float(q)})
            a, b = int(row_off[i]), int(row_off[i + 1])
            df = pd.DataFrame({c: host[c][a:b] for c in ("event_id", "time_delta", "src_id", "t", "sink_id")})
            op = {"type": "Opt", "seed": int(seed), "capacity": float(ro_c[i, 0]), "sim_opts": so,
                  "q": so.q, "wall_intensities": _wall_intensities(df, so, num_segments)}
            pp = {"type": "Poisson", "seed": int(seed), "sim_opts": so, "q": so.q}
            for dst, m, c in ((op, ro_m[i], ro_c[i]), (pp, rp_m[i], rp_c[i])):
                for j, kk in enumerate(Ks):
                    dst["top_" + str(kk)] = np.float64(m[j])
                dst["avg_rank"] = np.float64(m[len(Ks)])
                dst["r_2"] = np.float64(m[len(Ks) + 1])
                dst["world_events"] = int(c[1])
                dst["num_events"] = int(c[0])
            out.append((op, pp))
    return out


def run_inference(N=None, T=None, num_segments=None, sim_opts_gen=None, log_q_high=None,
                  log_q_low=None, opts=None):
    """opt_runs.run_inference (opt_runs.py:350-440): the q x seed sweep with, after every
    RedQueen replica, Poisson and the Oracle at its capacity -- run_inference_queue's
    legs (the q x seed grid as GPU batches) without its Karimi follow-up, which
    run_inference has commented out.  Returns Options(df, raw_results, capacities)."""
    return _run_inference(N, T, num_segments, sim_opts_gen, log_q_high, log_q_low, opts,
                          kdd=False)


def run_inference_queue(N=None, T=None, num_segments=None, sim_opts_gen=None, log_q_high=None,
                        log_q_low=None, num_procs=None, opts=None):
    """opt_runs.run_inference_queue (opt_runs.py:560-646): for every q in
    logspace(log_q_low, log_q_high, 10) and seed in range(N), RedQueen on
    sim_opts_gen(seed).update({'q': q}) (worker_opt), then the follow-ups the
    reference queues after each Opt result: Poisson at the Opt replica's capacity
    (worker_poisson) and the Oracle at that capacity (worker_oracle).

    The Opt and Poisson legs run as two GPU batches over the whole q x seed grid
    when the generated worlds share one network and their sources carry
    randomize_other_sources seeds (every sim_opts_gen of opt_runs.py:290-331 does),
    else one GPU run per replica; the Oracle leg is one GPU DP search per replica.
    ``num_procs`` is accepted for signature parity (no process pool).

    The reference's 'kdd' follow-up (Karimi et al., broadcast.opt.optimizer) is not
    vendored: there it raises in its worker and is logged as an exception record,
    which never enters the results -- here it is logged the same way.  An Oracle
    task that raises (worker_oracle's KeyError when q = 1 already meets the
    capacity, utils.py:271-276) is logged and dropped as the reference's queue does.
    Returns Options(df, raw_results, capacities) with the same fields."""
    return _run_inference(N, T, num_segments, sim_opts_gen, log_q_high, log_q_low, opts,
                          kdd=True)


def _run_inference(N, T, num_segments, sim_opts_gen, log_q_high, log_q_low, opts, kdd):
    import pandas as pd
    if opts is not None:   # @optioned(option_arg='opts'): explicit arguments win
        d = opts._get_dict() if hasattr(opts, "_get_dict") else dict(opts)
        N = d.get("N", N) if N is None else N
        T = d.get("T", T) if T is None else T
        num_segments = d.get("num_segments", num_segments) if num_segments is None else num_segments
        sim_opts_gen = d.get("sim_opts_gen", sim_opts_gen) if sim_opts_gen is None else sim_opts_gen
        log_q_high = d.get("log_q_high", log_q_high) if log_q_high is None else log_q_high
        log_q_low = d.get("log_q_low", log_q_low) if log_q_low is None else log_q_low
    qs = np.logspace(log_q_low, log_q_high, num=10)
    seeds = list(range(N))
    worlds = [sim_opts_gen(seed) for seed in seeds]
    results, raw_results = [], []
    capacities = {q: [] for q in qs}
    batchable = N > 0 and len({_world_key(w) for w in worlds}) == 1 and \
        all(_randomize_seed(w) is not None for w in worlds)
    if batchable:
        pairs = _opt_poisson_batches(worlds, qs, seeds, num_segments)
    else:
        pairs = []
        for q in qs:
            for seed, w in zip(seeds, worlds):
                op = worker_opt((seed, w.update({"q": q}), num_segments, None))
                pp = worker_poisson((seed, op["capacity"], op["sim_opts"], None))
                pairs.append((op, pp))
    # the Oracle legs: every replica's q search in lockstep, one rq_oracle_dp launch per
    # search round over all of them (utils.find_opt_oracle_batch); the wall of a seed is
    # the same at every q, so it is simulated once per seed
    walls = {}
    for op, _ in pairs:
        if op["seed"] not in walls:
            walls[op["seed"]] = utils._wall_df(op["sim_opts"])
    try:
        searches = utils.find_opt_oracle_batch(
            [op["capacity"] for op, _ in pairs], [op["sim_opts"] for op, _ in pairs],
            [op["world_events"] for op, _ in pairs], walls=[walls[op["seed"]] for op, _ in pairs])
    except Exception:   # a search raised: every replica's own search below, as the reference
        searches = [None] * len(pairs)
    for (op, pp), srch in zip(pairs, searches):
        raw_results.append(op)
        results.append(extract_perf_fields(op))
        capacities[op["q"]].append((op["seed"], op["capacity"]))
        raw_results.append(pp)
        results.append(extract_perf_fields(pp))
        try:
            if srch is None:
                orc = worker_oracle((op["seed"], op["capacity"], op["world_events"], op["sim_opts"], None))
            else:
                orc = _oracle_op(op["seed"], op["sim_opts"], srch)
        except Exception as e:   # the reference's worker_combined: an 'Exception' record
            logging.error("Exception while handling: %r", {"type": "Exception", "error": e,
                                                           "broadcaster_type": "Oracle"})
        else:
            raw_results.append(orc)
            results.append(extract_perf_fields(orc))
        if kdd:
            logging.error("Exception while handling: %r", {
                "type": "Exception", "broadcaster_type": "kdd",
                "error": NameError("broadcast.opt.optimizer (Karimi et al.) is not vendored")})
    return _Options(df=pd.DataFrame.from_records(results), raw_results=raw_results,
                    capacities=capacities)


# The reference's inference configurations (opt_runs.py:284-331), for
# run_inference_queue(opts=...).
dilation = 100.0
simulation_opts = _Options(world_rate=1000.0 / dilation, world_alpha=1.0, world_beta=10.0,
                           N=10, T=1.0 * dilation, num_segments=10,
                           log_q_low=-6 + np.log10(dilation), log_q_high=5 + np.log10(dilation))


def piecewise_sim_opt_factory(N=None, T=None, num_segments=None, world_rate=None, opts=None):
    """opt_runs.piecewise_sim_opt_factory (opt_runs.py:294-306)."""
    from .opt_model import SimOpts
    d = opts._get_dict() if opts is not None else {}
    N = d.get("N") if N is None else N
    T = d.get("T") if T is None else T
    num_segments = d.get("num_segments") if num_segments is None else num_segments
    world_rate = d.get("world_rate") if world_rate is None else world_rate
    random_state = np.random.RandomState(42)
    world_changing_rates = random_state.uniform(low=world_rate / 2.0, high=world_rate, size=num_segments)
    world_change_times = np.arange(num_segments) * T / num_segments

    def sim_opts_gen(seed):
        return SimOpts.std_piecewise_const(world_rates=world_changing_rates,
                                           world_change_times=world_change_times,
                                           world_seed=seed + 42).update({'end_time': T})

    return (opts or _Options()).set_new(N=N, T=T, num_segments=num_segments, sim_opts_gen=sim_opts_gen)


def _std_poisson_gen(seed):
    from .opt_model import SimOpts
    return SimOpts.std_poisson(world_rate=simulation_opts.world_rate,
                               world_seed=seed + 42).update({'end_time': simulation_opts.T})


def _std_hawkes_gen(seed):
    from .opt_model import SimOpts
    return SimOpts.std_hawkes(world_seed=seed, world_lambda_0=simulation_opts.world_rate,
                              world_alpha=simulation_opts.world_alpha,
                              world_beta=simulation_opts.world_beta).update({'end_time': simulation_opts.T})


poisson_inf_opts = simulation_opts.set_new(sim_opts_gen=_std_poisson_gen)
piecewise_inf_opts = piecewise_sim_opt_factory(opts=simulation_opts)
hawkes_inf_opts = simulation_opts.set_new(sim_opts_gen=_std_hawkes_gen)


# ---------------------------------------------------------------- multiple followers
# opt_runs.py:651-795: the networks of the multiple-follower experiments (C3 / C5's
# construction, graphs.followers_graph), built on the host with the reference's draws.

def make_piecewise_const(num_segments):
    """A piecewise-constant semi-sinusoid of num_segments segments (opt_runs.py:653-657)."""
    import pandas as pd
    true_values = np.sin(np.arange(0, np.pi, step=0.001))
    seg_idx = np.arange(true_values.shape[0]) // (true_values.shape[0] / num_segments)
    return pd.Series(true_values).groupby(seg_idx).mean().tolist()


mk_edge_list_opts = _Options(num_followers=100, num_broadcasters=100, degree=5, seed=42,
                             follower_id_offset=1000, broadcaster_id_offset=5000)


@_optioned
def make_edge_list(num_followers, num_broadcasters, degree, seed, follower_id_offset=0,
                   broadcaster_id_offset=0, preferential_attachment=False):
    """Each follower follows ``degree`` distinct broadcasters drawn by RandomState(seed)
    (opt_runs.py:663-686; graphs.make_edge_list, pinned by tests/golden/graphs.npz)."""
    from .graphs import make_edge_list as _mk
    return _mk(num_followers, num_broadcasters, degree, seed, follower_id_offset,
               broadcaster_id_offset, preferential_attachment)


def create_phased_pwconst_broadcaster(src_id, seed, rel_rates, avg_rate, end_time, phase_shift):
    """A PiecewiseConst source over num_segments equal segments of [0, end_time), its
    relative rates rotated by ``phase_shift`` and scaled to average ``avg_rate``
    (opt_runs.py:689-702)."""
    num_segments = len(rel_rates)
    assert int(phase_shift) == phase_shift, "The phase shift cannot be fractional."
    phase_shift %= num_segments
    change_times = np.arange(num_segments) * (end_time / num_segments)
    shifted_rates = np.asarray(rel_rates[phase_shift:] + rel_rates[:phase_shift])
    actual_rates = shifted_rates * (avg_rate * num_segments) / np.sum(shifted_rates)
    return ('PiecewiseConst', {'src_id': src_id, 'seed': seed, 'change_times': change_times,
                               'rates': actual_rates})


def trim_sim_opts(sim_opts):
    """Only the controlled source's followers and the broadcasters reaching them stay;
    q = (#followers)^2 (opt_runs.py:705-718)."""
    intended = set(t for s_, t in sim_opts.edge_list if s_ == sim_opts.src_id)
    new_edges = [(s_, t) for s_, t in sim_opts.edge_list if t in intended]
    reach = set(s_ for s_, _ in new_edges)
    return sim_opts.update({
        'sink_ids': sorted(intended),
        'edge_list': new_edges,
        'other_sources': [x for x in sim_opts.other_sources if x[1]['src_id'] in reach],
        'q': 1.0 * (len(intended) ** 2),
    })


multiple_follower_opts = _Options(seed=42, world_alpha=1.0, world_beta=10.0, world_rate=100.0,
                                  kind='PiecewiseConst', num_other_broadcasters=1000,
                                  max_num_followers=500, follower_other_degree=1)


@_optioned
def prepare_multiple_followers_sim_opts(num_followers, num_other_broadcasters, max_num_followers,
                                        seed, world_rate, world_alpha, world_beta,
                                        follower_other_degree, kind):
    """The multiple-follower world (opt_runs.py:725-795): a fixed network over
    max_num_followers (seed 1024), num_other_broadcasters of one kind (seed + src_id
    each), the controlled source 1 following num_followers of them drawn by
    RandomState(seed), trimmed to those followers (trim_sim_opts).  T = 100."""
    from .opt_model import SimOpts
    assert num_other_broadcasters >= follower_other_degree, (
        "There should be more other broadcasters than followers per node.")
    end_time = 100.0
    rs = np.random.RandomState(seed)
    follower_ids = 1000 + np.arange(max_num_followers)
    b_ids = 5000 + np.arange(num_other_broadcasters)
    network = make_edge_list(num_followers=max_num_followers, num_broadcasters=num_other_broadcasters,
                             degree=follower_other_degree, seed=1024, follower_id_offset=1000,
                             broadcaster_id_offset=5000, opts=mk_edge_list_opts)
    if kind == 'PiecewiseConst':
        pcw = make_piecewise_const(24)
        others = [create_phased_pwconst_broadcaster(src_id=x, seed=seed + x, rel_rates=pcw,
                                                    avg_rate=world_rate, end_time=end_time,
                                                    phase_shift=x) for x in b_ids]
    elif kind == 'Hawkes':
        others = [('Hawkes', {'src_id': x, 'seed': seed + x, 'l_0': world_rate,
                              'alpha': world_alpha, 'beta': world_beta}) for x in b_ids]
    elif kind == 'Poisson2':
        logging.warning('The rates are being randomised for Poisson2')
        others = [('Poisson2', {'src_id': x, 'seed': seed + x,
                                'rate': world_rate * np.abs(rs.randn() + 1.0)}) for x in b_ids]
    else:
        raise ValueError('Cannot create broadcasters of kind "{}"'.format(kind))
    network.extend([(1, x) for x in rs.choice(follower_ids, num_followers, replace=False)])
    so = SimOpts(src_id=1, end_time=end_time, s=np.asarray([1.0] * num_followers),
                 sink_ids=follower_ids, other_sources=others, edge_list=network,
                 q=1.0 * (num_followers ** 2))
    return trim_sim_opts(so)
