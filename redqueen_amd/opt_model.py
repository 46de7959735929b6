"""Drop-in surface of the reference's ``redqueen/opt_model.py``.

Same class names, constructor arguments, factories, validation and errors as
the reference (file:line below); the simulation itself runs in librq.so on
the GPU.  Broadcaster objects here are parameter holders: their arrival
processes are implemented by the gfx950 kernels (engine semantics),
so ``get_next_interval`` is not called from Python.

    SimOpts            opt_model.py:755-967
    Manager            opt_model.py:144-314
    State / Event      opt_model.py:20-141
    Poisson, Poisson2, Hawkes, PiecewiseConst, RealData, Opt   :381-750
"""
import logging
import warnings

import numpy as np
import pandas as pd

from . import _lib as L
from .utils import is_sorted, mb


class Event:
    def __init__(self, event_id, time_delta, cur_time, src_id, sink_ids, metadata=None):
        self.event_id = event_id
        self.time_delta = time_delta
        self.cur_time = cur_time
        self.src_id = src_id
        self.sink_ids = sink_ids
        self.metadata = metadata

    def __repr__(self):
        return ('[ Event_id: {}, time_delta: {}, cur_time: {}, src_id: {} ]'
                .format(self.event_id, self.time_delta, self.cur_time, self.src_id))


class State:
    """Event log of one run (opt_model.py:35-141), filled from the engine's SoA log."""

    def __init__(self, cur_time, sink_ids):
        self.num_sinks = len(sink_ids)
        self.time = cur_time
        self.sink_ids = list(sink_ids)
        self._start = cur_time
        self._t = np.zeros(0)
        self._src = np.zeros(0, dtype=np.int64)
        self._edges = []
        self._events = None
        self._result = None

    def _set_log(self, t, src, edge_list, result=None):
        self._result = result
        self._t = np.asarray(t, dtype=np.float64)
        self._src = np.asarray(src, dtype=np.int64)
        self._edges = list(edge_list)
        self._events = None
        if self._t.size:
            self.time = self._accumulate()[1]

    def _time_delta(self):
        return self._accumulate()[0]

    def _accumulate(self):
        """Event.time_delta as the reference accumulates it: time_delta_k = t_k - time,
        time += time_delta_k (opt_model.py:68, :304); returns (time_delta, final time).
        time == t_k except after a rounded subtraction; the chain is redone from those
        events until it heals."""
        t = self._t
        if not t.size:
            return t, self._start
        prev = np.concatenate([[self._start], t[:-1]])
        td = t - prev
        dirty = np.flatnonzero(prev + td != t)
        k, n = 0, t.size
        final = prev[-1] + td[-1]
        for k0 in dirty:
            if k0 < k:
                continue
            s = prev[k0] + td[k0]
            k = k0 + 1
            while k < n and s != t[k - 1]:
                td[k] = t[k] - s
                s = s + td[k]
                k += 1
            if k == n:
                final = s
        return td, float(final)

    @property
    def events(self):
        if self._events is None:
            sinks = {}
            for s, d in self._edges:
                sinks.setdefault(s, []).append(d)
            td = self._time_delta()
            self._events = [Event(100 + k, float(td[k]), float(self._t[k]), int(self._src[k]),
                                  list(sinks.get(int(self._src[k]), [])))
                            for k in range(self._t.size)]
        return self._events

    def get_num_events(self):
        return int(self._t.size)

    def get_dataframe(self):
        """One row per (event, sink) in event order then edge-list order, columns
        event_id, time_delta, src_id, t, sink_id (State.get_dataframe, :85-97); the
        rows are expanded on the GPU from the run's event log (rq_log_expand)."""
        if self._result is None or self._t.size == 0:
            return pd.DataFrame.from_records([])
        df = self._result.dataframe(0)
        if len(df) == 0:
            return pd.DataFrame.from_records([])
        return df


# ----------------------------------------------------------------- broadcasters
class Broadcaster:
    """Base of every broadcaster (opt_model.py:323-378).

    The built-in kinds are parameter holders: their arrival processes are the
    engine's kernels.  A class a user registers with ``SimOpts.registerSource``
    keeps the reference's plugin contract: ``__init__(src_id, seed, ...)`` gets
    ``self.random_state = RandomState(seed)``; a STATIC one (``is_dynamic =
    False``) implements ``initialize()`` and ``get_all_times()`` after
    ``init_state(start_time, all_sink_ids, follower_sink_ids, end_time)``.  The host
    calls them (once per run, or once per replica of a randomized batch) and the
    times play as RealData-kind streams on the GPU.  A DYNAMIC plugin
    (``get_next_interval`` queried on every event, opt_model.py:351-369) runs when it
    is SELF-DRIVEN -- its schedule moves only on its own events, as Poisson's and
    Hawkes' do: the host plays its own events through ``get_next_event_time`` to get
    its times (dynamic_plugin_times), the GPU plays them, and every run then feeds a
    fresh copy of the plugin the run's whole event sequence, in play order, as
    run_dynamic would (verify_dynamic_plugin): a plugin whose schedule reacts to
    another source's event (the reference's SmartPoisson, say) raises
    NotImplementedError (RQ_EUNSUPPORTED) instead of returning a different run."""
    _rq_kind = None

    def __init__(self, src_id, seed):
        self.src_id = src_id
        self.seed = seed
        self.random_state = np.random.RandomState(seed)
        self.t_delta = None
        self.end_time = None
        self.last_self_event_time = None
        self.used = False
        self.is_dynamic = True

    def is_fresh(self):
        return not self.used

    def init_state(self, start_time, all_sink_ids, follower_sink_ids, end_time):
        self.sink_ids = sorted(follower_sink_ids)
        self.state = State(start_time, all_sink_ids)
        self.start_time = start_time
        self.end_time = end_time

    def get_all_times(self):
        assert not self.is_dynamic
        raise NotImplementedError()

    def get_next_event_time(self, event):
        """opt_model.py:351-369: the delay to this source's next event after `event`
        (None: the start); the host calls it only for dynamic plugins."""
        cur_time = self.get_current_time(event)
        self.used = True
        if event is None or event.src_id == self.src_id:
            self.last_self_event_time = cur_time
        t_delta = self.get_next_interval(event)
        if t_delta is not None:
            self.t_delta = t_delta
        ret_t_delta = self.last_self_event_time + self.t_delta - cur_time
        if ret_t_delta < 0:
            logging.warning('src_id: {}, event_id: {}, returned t_delta = {} < 0, set to 0 instead.'
                            .format(self.src_id, event.event_id, ret_t_delta))
            ret_t_delta = 0.0
        return ret_t_delta

    def get_current_time(self, event):
        return event.cur_time if event is not None else self.start_time

    def get_next_interval(self, event):  # pragma: no cover - engine-side
        raise NotImplementedError("arrival processes run in librq.so (gfx950)")

    def _kwargs(self):
        return {"src_id": self.src_id, "seed": self.seed}


def _schedule(obj):
    """The absolute time of a dynamic source's next event: last_self_event_time +
    t_delta (Broadcaster.get_next_event_time, opt_model.py:351-369)."""
    if obj.t_delta is None:
        raise TypeError("unsupported operand type(s) for +: 'float' and 'NoneType' "
                        "(broadcaster %s returned no first interval)" % type(obj).__name__)
    return obj.last_self_event_time + obj.t_delta


DYNAMIC_PLUGIN_MAX_EVENTS = 10 ** 7


def dynamic_plugin_times(obj, start_time, sink_ids, edge_list, end_time):
    """Own event times of a SELF-DRIVEN dynamic plugin instance (see Broadcaster): the
    first call get_next_event_time(None) at start_time, then one call per own event,
    as run_dynamic makes them (opt_model.py:251-311); an event's time is the schedule
    last_self_event_time + t_delta (the engine plays every source's own times).  The
    events handed over carry the plugin's own src_id, cur_time and sink list; their
    event_id and time_delta are unknown here (-1, NaN) -- a plugin that reads them is
    not self-driven and fails the run's verification."""
    followers = [e[1] for e in edge_list if e[0] == obj.src_id]
    obj.init_state(start_time, list(sink_ids), followers, end_time)
    obj.get_next_event_time(None)
    t = []
    nxt = _schedule(obj)
    while nxt <= end_time:
        if nxt < (t[-1] if t else start_time):
            # run_dynamic clamps a negative delay to 0 relative to the LAST event of any
            # source (opt_model.py:364-367): that depends on the other sources
            raise NotImplementedError("broadcaster %s (src_id %r) scheduled an event before its "
                                      "previous one: not supported by the GPU engine"
                                      % (type(obj).__name__, obj.src_id))
        if len(t) >= DYNAMIC_PLUGIN_MAX_EVENTS:
            raise ValueError("broadcaster %s (src_id %r) posted more than %d events"
                             % (type(obj).__name__, obj.src_id, DYNAMIC_PLUGIN_MAX_EVENTS))
        t.append(nxt)
        obj.get_next_event_time(Event(-1, float("nan"), nxt, obj.src_id, followers))
        nxt = _schedule(obj)
    return np.asarray(t, dtype=np.float64)


class PluginReacts(NotImplementedError):
    """A dynamic plugin's schedule moved on another source's event (verify_dynamic_plugin):
    Graph.run then plays the batch through the reactive fixed point (Graph._run_reactive)."""


def verify_dynamic_plugin(fresh, start_time, sink_ids, edge_list, end_time, ev_t, ev_src,
                          times, max_events=None):
    """Feed a fresh copy of a dynamic plugin every event of a run in play order
    (ev_t / ev_src: the engine's event log), as run_dynamic does (opt_model.py:271-311:
    get_next_event_time(last_event) for every event, event ids from 100, time_delta on
    the accumulated State.time); its schedule must put each of its own events where the
    engine played them (`times`).  Raises PluginReacts otherwise: the plugin's schedule
    depends on other sources' events, and the batch is replayed to the reactive fixed
    point (engine.Graph._run_reactive)."""
    sinks = {}
    for a_, b_ in edge_list:
        sinks.setdefault(a_, []).append(b_)
    fresh.init_state(start_time, list(sink_ids), sinks.get(fresh.src_id, []), end_time)
    fresh.get_next_event_time(None)
    own = iter(np.asarray(times, dtype=np.float64))
    state_time = start_time
    n = len(ev_t)
    bad = None
    for k in range(n):
        t, src = float(ev_t[k]), int(ev_src[k])
        if src == fresh.src_id:
            want = next(own, None)
            sched = _schedule(fresh)
            if want is None or sched != want or t != want:
                bad = (k, t, sched)
                break
        ev = Event(100 + k, t - state_time, t, src, list(sinks.get(src, [])))
        state_time += ev.time_delta
        if max_events is not None and k + 1 >= max_events:
            break   # run_dynamic stops before it hands the last event over
        fresh.get_next_event_time(ev)
    else:
        if max_events is None or n < max_events:
            sched = _schedule(fresh)
            if next(own, None) is not None or sched <= end_time:
                bad = (n, None, sched)
    if bad is not None:
        raise PluginReacts(
            "dynamic broadcaster %s (src_id %r) is not self-driven: its schedule reacts to "
            "other sources' events (at event %d: played %r, its schedule %r)"
            % (type(fresh).__name__, fresh.src_id, bad[0], bad[1], bad[2]))


REACTIVE_MAX_ITERATIONS = 1000


def reactive_plugin_times(fresh, start_time, sink_ids, edge_list, end_time, ev_t, ev_src,
                          max_events=None, static_ids=()):
    """Own event times of a dynamic plugin whose schedule may react to other sources'
    events, given the OTHER sources' events of a run (ev_t / ev_src in play order; the
    plugin's own entries in the log are dropped): run_dynamic's loop (opt_model.py:271-311)
    with this plugin beside that fixed sequence.  After every event -- its own and the
    others', event ids from 100, time_delta on the accumulated State.time -- the plugin's
    get_next_event_time(event) gives its delay r, and its next event comes at
    State.time + r unless another event comes first.  Equal times: the plugin is dynamic,
    so it plays before a STATIC source's event (run_dynamic plays a static time only when
    it is strictly earlier, opt_model.py:289-290; ``static_ids``: the src_ids of the
    Poisson2 / PiecewiseConst / RealData / static-plugin sources of the run) and, against a
    dynamic source (Poisson, Hawkes, RedQueen, another dynamic plugin), in src_id order
    (the sorted (t_delta, src_id) of the dynamic sources, :279-281).
    Exact when the other events do not depend on the plugin's; Graph.run / Manager.run_dynamic
    rerun with these times until the run reproduces them (the fixed point)."""
    sinks = {}
    for a_, b_ in edge_list:
        sinks.setdefault(a_, []).append(b_)
    me = fresh.src_id
    fresh.init_state(start_time, list(sink_ids), sinks.get(me, []), end_time)
    r = fresh.get_next_event_time(None)
    ev_t = np.asarray(ev_t, dtype=np.float64)
    ev_src = np.asarray(ev_src)
    keep = ev_src != me
    ot, osrc = ev_t[keep], ev_src[keep]
    static_ids = {int(x) for x in static_ids}
    out = []
    state_time = float(start_time)
    j, k, n_o = 0, 0, len(ot)
    while max_events is None or k < max_events:
        cand = state_time + r
        if j < n_o and (float(ot[j]) < cand or (float(ot[j]) == cand and int(osrc[j]) < me and
                                                int(osrc[j]) not in static_ids)):
            t, src = float(ot[j]), int(osrc[j])
            j += 1
        else:
            if not cand <= end_time:
                break   # every other event played (they are <= end_time)
            if len(out) >= DYNAMIC_PLUGIN_MAX_EVENTS:
                raise ValueError("broadcaster %s (src_id %r) posted more than %d events"
                                 % (type(fresh).__name__, me, DYNAMIC_PLUGIN_MAX_EVENTS))
            t, src = cand, me
            out.append(cand)
        ev = Event(100 + k, t - state_time, t, src, list(sinks.get(src, [])))
        state_time += ev.time_delta
        k += 1
        if max_events is not None and k >= max_events:
            break   # run_dynamic stops before it hands the last event over
        r = fresh.get_next_event_time(ev)
    return np.asarray(out, dtype=np.float64)


def source_times(obj, start_time, sink_ids, edge_list, end_time):
    """Times of a registered plugin instance: static (plugin_times) or self-driven
    dynamic (dynamic_plugin_times)."""
    if getattr(obj, "is_dynamic", True):
        return dynamic_plugin_times(obj, start_time, sink_ids, edge_list, end_time)
    return plugin_times(obj, start_time, sink_ids, edge_list, end_time)


def plugin_times(obj, start_time, sink_ids, edge_list, end_time):
    """Times of a registered static broadcaster instance, as run_dynamic collects
    them (init_state + initialize + get_all_times, opt_model.py:256-264), sorted and
    clipped at end_time (events past end_time never play); a time before start_time
    raises ValueError (the reference would play it with a negative time_delta)."""
    if getattr(obj, "is_dynamic", True):
        raise NotImplementedError(
            "broadcaster %s is dynamic (get_next_interval per event): use source_times "
            "(self-driven dynamic plugins)" % type(obj).__name__)
    followers = [e[1] for e in edge_list if e[0] == obj.src_id]
    obj.init_state(start_time, list(sink_ids), followers, end_time)
    obj.initialize()
    t = np.sort(np.asarray(obj.get_all_times(), dtype=np.float64).ravel())
    if t.size and t[0] < start_time:
        # run_dynamic would play it first with a negative time_delta (the built-in
        # RealData drops such times itself, opt_model.py:727); the engine's streams
        # start at start_time, so refuse instead of dropping it silently
        raise ValueError("broadcaster %s (src_id %r) returned a time %r before start_time %r: "
                         "not supported by the GPU engine" %
                         (type(obj).__name__, obj.src_id, float(t[0]), start_time))
    return t[t <= end_time]


class Poisson(Broadcaster):
    _rq_kind = L.SRC_POISSON

    def __init__(self, src_id, seed, rate=1.0):
        super().__init__(src_id, seed)
        self.rate = rate

    def _kwargs(self):
        return dict(super()._kwargs(), rate=self.rate)


class Poisson2(Broadcaster):
    _rq_kind = L.SRC_POISSON2

    def __init__(self, src_id, seed, rate=1.0):
        super().__init__(src_id, seed)
        self.rate = rate
        self.is_dynamic = False

    def _kwargs(self):
        return dict(super()._kwargs(), rate=self.rate)


class SmartPoisson(Broadcaster):
    """Present for name parity (opt_model.py:436-455); not registered, no kernel."""

    def __init__(self, src_id, seed, rate=1.0):
        super().__init__(src_id, seed)
        self.rate = rate


class Hawkes(Broadcaster):
    _rq_kind = L.SRC_HAWKES

    def __init__(self, src_id, seed, l_0=1.0, alpha=1.0, beta=10.0):
        super().__init__(src_id, seed)
        self.l_0, self.alpha, self.beta = l_0, alpha, beta

    def _kwargs(self):
        return dict(super()._kwargs(), l_0=self.l_0, alpha=self.alpha, beta=self.beta)


class PiecewiseConst(Broadcaster):
    _rq_kind = L.SRC_PWCONST

    def __init__(self, src_id, seed, change_times, rates):
        super().__init__(src_id, seed)
        assert is_sorted(change_times)
        self.change_times = change_times
        self.rates = rates
        self.is_dynamic = False

    def _kwargs(self):
        return dict(super()._kwargs(), change_times=self.change_times, rates=self.rates)


class RealData(Broadcaster):
    _rq_kind = L.SRC_REALDATA

    def __init__(self, src_id, times):
        super().__init__(src_id, 0)
        self.times = np.asarray(times)
        self.is_dynamic = False

    def get_num_events(self):
        return len(self.times)

    def _kwargs(self):
        return {"src_id": self.src_id, "times": self.times}


class Opt(Broadcaster):
    """RedQueen (opt_model.py:493-544)."""
    _rq_kind = L.SRC_OPT

    def __init__(self, src_id, seed, q=1.0, s=1.0):
        super().__init__(src_id, seed)
        self.q = q
        self.s = s


class OptPWSignificance(Broadcaster):
    """RedQueen with a piecewise-constant periodic significance (opt_model.py:547-623):
    s_vec is [followers x segments] (or one row of segments spread to every follower,
    :590-604) over time_period; run by the sweep kernels' OptPWSignificance controller."""
    _rq_kind = L.SRC_OPTPW

    def __init__(self, src_id, seed, s_vec, time_period, q=1.0):
        super().__init__(src_id, seed)
        self.s_pw = np.asarray(s_vec)
        self.q = q
        self.old_ranks = 0
        self.time_period = time_period
        self.init = False

    def _s_pw_for(self, n_followers):
        s_pw = np.asarray(self.s_pw, dtype=np.float64)
        if s_pw.ndim == 1:
            # Spread the same s_pw to all the followers (opt_model.py:590-602)
            s_pw = s_pw.repeat(n_followers).reshape((n_followers, -1), order='F')
        if s_pw.ndim != 2 or s_pw.shape[0] != n_followers:
            raise ValueError("operands could not be broadcast together: significance rows {} vs "
                             "{} followers".format(s_pw.shape[0] if s_pw.ndim else 0, n_followers))
        return s_pw


def _sig_bad_sources(g, edge_list, s_pw, q):
    """Stream src_ids whose events reach no follower with positive significance: for
    them take_one_sample sees an all-zero piecewise intensity, s_max = 0 and int(nan)
    (opt_model.py:557-566, :610-614).  The engine draws nothing for such an event."""
    fol = {int(f): i for i, f in enumerate(g.followers)}
    pw = {}
    for a, b in edge_list:   # rank_diff counts edge multiplicity
        if int(a) != g.src_id and int(b) in fol:
            pw[int(a)] = pw.get(int(a), 0.0) + np.sqrt(np.asarray(s_pw[fol[int(b)]]) / q)
    return {int(j) for j in g.stream_src_ids
            if int(j) != g.src_id and not (int(j) in pw and np.max(pw[int(j)]) > 0.0)}


def _sig_reach_check(g, edge_list, s_pw, q, ev_src, bad=None, max_events=None):
    """OptPWSignificance raises where the reference does: in a run in which an event
    of a source from _sig_bad_sources is actually played (ev_src = the run's event
    sources) AND handed to the controller's get_next_interval.  run_dynamic hands
    every played event to the dynamic sources at the start of the next loop step
    (opt_model.py:271-281), which a max_events cap ends first: the run's last event
    when it reached the cap is never seen by the controller."""
    if bad is None:
        bad = _sig_bad_sources(g, edge_list, s_pw, q)
    if max_events is not None and len(ev_src) >= max_events:
        ev_src = ev_src[:max(0, int(max_events) - 1)]
    hit = [int(j) for j in np.unique(ev_src) if int(j) in bad]
    if hit:
        raise ValueError("cannot convert float NaN to integer (OptPWSignificance.take_one_sample: "
                         "an event of source {} reaches no follower with positive significance)"
                         .format(hit[0]))


# ----------------------------------------------------------------------- Manager
class Manager:
    def __init__(self, sources, sink_ids=None, end_time=None, edge_list=None, sim_opts=None,
                 start_time=0):
        if sim_opts is not None:
            edge_list = mb(edge_list, sim_opts.edge_list)
            sink_ids = mb(sink_ids, sim_opts.sink_ids)
            end_time = mb(end_time, sim_opts.end_time)
        assert len(sources) > 0, "No sources."
        assert len(sink_ids) > 0, "No sinks."
        assert len(set(x.src_id for x in sources)) == len(sources), "Duplicates in sources."
        assert len(set(sink_ids)) == len(sink_ids), "Duplicates in sink_ids."
        if edge_list is None:
            edge_list = [(src.src_id, dst) for src in sources for dst in sink_ids]
        else:
            known = set(src.src_id for src in sources)
            assert set(x[0] for x in edge_list).issubset(known), "Unknown sources in edge_list."
            assert set(x[1] for x in edge_list).issubset(set(sink_ids)), \
                "Unknown sinks in edge_list."
        self.end_time = end_time
        self.edge_list = edge_list
        self.sink_ids = sink_ids
        self.state = State(start_time, sink_ids)
        self.sources = sources
        self.sim_opts = sim_opts
        self.start_time = start_time

    def get_state(self):
        return self.state

    def run(self):
        warnings.warn('Consider using `run_dynamic` instead of `run`.')
        return self.run_till()

    def run_till(self, end_time=None):
        if end_time is not None:
            logging.warning('Warning: deprecation warning: end_time should not be set.')
            self.end_time = end_time
        return self.run_dynamic()

    def _controlled(self):
        ctrl = None
        if self.sim_opts is not None:
            for s in self.sources:
                if s.src_id == self.sim_opts.src_id and isinstance(s, (Opt, OptPWSignificance, Poisson2,
                                                                       PiecewiseConst, RealData)):
                    ctrl = s
        if ctrl is None:
            opts = [s for s in self.sources if isinstance(s, (Opt, OptPWSignificance))]
            if len(opts) > 1:
                raise NotImplementedError("more than one Opt broadcaster in one run")
            ctrl = opts[0] if opts else None
        return ctrl

    def run_dynamic(self, max_events=float('inf')):
        from .engine import Graph
        if max_events is None:
            max_events = float('inf')
        for src in self.sources:
            if not src.is_fresh():
                raise ValueError('Source with id: {} is not fresh.'.format(src.src_id))
        ctrl = self._controlled()
        others = [s for s in self.sources if s is not ctrl]
        for s in others:
            if s._rq_kind in (L.SRC_OPT, L.SRC_OPTPW):
                raise NotImplementedError("broadcaster %s has no engine kernel" %
                                          type(s).__name__)
        if ctrl is None:
            ids = [s.src_id for s in self.sources] + [e[0] for e in self.edge_list]
            ctrl_id = min(ids) - 1
        else:
            ctrl_id = ctrl.src_id
        # registered plugin broadcasters: their own initialize() / get_all_times(), or a
        # dynamic plugin's own schedule (self-driven: reproduced by the run at once;
        # reactive: recomputed from the run's other events until the run reproduces it)
        import copy
        probes = []
        other_desc = []
        for s in others:
            if s._rq_kind is not None:
                other_desc.append((type(s).__name__, s._kwargs()))
                continue
            fresh = copy.deepcopy(s) if getattr(s, "is_dynamic", True) else None
            t = source_times(s, self.start_time, self.sink_ids, self.edge_list, self.end_time)
            kw = {"src_id": s.src_id, "times": t}
            if fresh is not None:
                kw["dynamic"] = True   # ties: played as the dynamic source it is (RQ_SRCF_DYNAMIC)
            other_desc.append(("RealData", kw))
            if fresh is not None:
                probes.append((fresh, t, len(other_desc) - 1))
        if isinstance(ctrl, (Opt, OptPWSignificance)):
            fl = [e[1] for e in self.edge_list if e[0] == ctrl.src_id]
            if len(set(fl)) != len(fl):
                # the reference's per-edge follower vectors (sqrt_s_by_q / old_ranks,
                # opt_model.py:510-517, :582) against one rank per distinct follower:
                # its first non-own event raises
                raise ValueError("shapes (%d,) and (%d,) not aligned: duplicated edges of the "
                                 "controlled source %r" % (len(fl), len(set(fl)), ctrl.src_id))
        ctrl_a = ctrl_b = None
        if isinstance(ctrl, PiecewiseConst):
            ctrl_a, ctrl_b = ctrl.change_times, ctrl.rates
        elif isinstance(ctrl, RealData):
            ctrl_a = ctrl.times
        maxev = None if max_events == float('inf') else int(max_events)
        seed = 0 if ctrl is None else int(ctrl.seed) & 0xFFFFFFFF

        def play(desc):
            g = Graph(ctrl_id, desc, self.sink_ids, self.edge_list, self.end_time,
                      start_time=self.start_time, ctrl_a=ctrl_a, ctrl_b=ctrl_b)
            if isinstance(ctrl, Opt):
                if isinstance(ctrl.s, dict):
                    s = ctrl.s
                else:
                    s = np.ones(g.n_followers) * np.asarray(ctrl.s, dtype=float)
                return g.run("opt", q=ctrl.q, s=s, ctrl_seed=seed, max_events=maxev, event_log=True)
            if isinstance(ctrl, OptPWSignificance):
                s_pw = ctrl._s_pw_for(g.n_followers)
                res = g.run("sig", q=ctrl.q, s_pw=s_pw, period=float(ctrl.time_period),
                            ctrl_seed=seed, max_events=maxev, event_log=True)
                _sig_reach_check(g, self.edge_list, s_pw, ctrl.q, res.events(0)[1], max_events=maxev)
                return res
            if isinstance(ctrl, Poisson2):
                return g.run("poisson", ctrl_seed=seed, ctrl_rate=[float(ctrl.rate)],
                             max_events=maxev, event_log=True)
            if isinstance(ctrl, PiecewiseConst):
                return g.run("pwconst", ctrl_seed=seed, max_events=maxev, event_log=True)
            if isinstance(ctrl, RealData):
                return g.run("times", max_events=maxev, event_log=True)
            return g.run("wall", max_events=maxev, event_log=True)

        res = play(other_desc)
        t, src = res.events(0)
        # the run's static sources (their equal-time events play after a dynamic plugin's)
        static_ids = {s.src_id for s in self.sources
                      if not getattr(s, "is_dynamic", True) and s is not ctrl}
        if isinstance(ctrl, (Poisson2, PiecewiseConst, RealData)):
            static_ids.add(ctrl.src_id)
        for it in range(REACTIVE_MAX_ITERATIONS + 1):
            new = [reactive_plugin_times(copy.deepcopy(fresh), self.start_time, self.sink_ids,
                                         self.edge_list, self.end_time, t, src, max_events=maxev,
                                         static_ids=static_ids)
                   for fresh, _times, _pos in probes]
            if all(np.array_equal(a, times) for a, (_f, times, _p) in zip(new, probes)):
                break
            if it == REACTIVE_MAX_ITERATIONS:
                raise NotImplementedError(
                    "reactive dynamic broadcasters did not reach a fixed point in %d reruns"
                    % REACTIVE_MAX_ITERATIONS)
            probes = [(fresh, nt, pos) for (fresh, _t, pos), nt in zip(probes, new)]
            for _f, nt, pos in probes:
                other_desc[pos] = ("RealData", {"src_id": other_desc[pos][1]["src_id"], "times": nt,
                                                "dynamic": True})
            res = play(other_desc)
            t, src = res.events(0)
        for s in self.sources:
            s.used = True
        self.state._set_log(t, src, self.edge_list, res)
        self.result = res
        return self


# ----------------------------------------------------------------------- SimOpts
class SimOpts:
    """Holds the options; its methods return managers (opt_model.py:755-967)."""

    broadcasters = {
        'Hawkes': Hawkes,
        'RealData': RealData,
        'Opt': Opt,
        'PiecewiseConst': PiecewiseConst,
        'Poisson': Poisson,
        'Poisson2': Poisson2,
        'OptPWSignificance': OptPWSignificance,
    }

    @classmethod
    def registerSource(cls, sourceName, sourceConstructor):
        cls.broadcasters[sourceName] = sourceConstructor

    def __init__(self, **kwargs):
        self.src_id = kwargs['src_id']
        self.s = kwargs['s']
        self.q = kwargs['q']
        self.other_sources = kwargs['other_sources']
        self.sink_ids = kwargs['sink_ids']
        self.edge_list = kwargs['edge_list']
        self.end_time = kwargs['end_time']

    def create_other_sources(self):
        others = []
        for x in self.other_sources:
            if callable(x[0]):
                others.append(x[0](**x[1]))
            elif x[0] in self.broadcasters:
                others.append(self.broadcasters[x[0]](**x[1]))
            else:
                raise ValueError('Unknown type of broadcaster: {}'.format(x[0]))
        return others

    def randomize_other_sources(self, using_seed):
        other_sources = []
        for idx, (x, y) in enumerate(self.other_sources):
            assert 'seed' in y, 'Do not know how to randomize {}.'.format(x)
            y_new = y.copy()
            y_new['seed'] = using_seed + 99 * idx
            other_sources.append((x, y_new))
        return self.update({'other_sources': other_sources})

    def create_manager_with_opt(self, seed):
        opt = Opt(src_id=self.src_id, seed=seed, s=self.s, q=self.q)
        return Manager(sim_opts=self, sources=[opt] + self.create_other_sources())

    def create_manager_with_broadcaster(self, broadcaster):
        assert broadcaster.src_id == self.src_id, \
            "Broadcaster has src_id = {}; expected = {}".format(broadcaster.src_id, self.src_id)
        return Manager(sim_opts=self, sources=[broadcaster] + self.create_other_sources())

    def create_manager_with_poisson(self, seed, rate=None, capacity=None):
        if rate is None and capacity is None:
            raise ValueError('One of rate or capacity must be specified.')
        elif rate is None:
            rate = capacity / self.end_time
        elif capacity is None:
            pass
        else:
            raise ValueError('Only one of rate or capacity must be specified.')
        poisson = Poisson2(src_id=self.src_id, seed=seed, rate=rate)
        return Manager(sim_opts=self, sources=[poisson] + self.create_other_sources())

    def create_manager_with_piecewise_const(self, seed, change_times, rates):
        assert len(change_times) == len(rates)
        piecewise = PiecewiseConst(src_id=self.src_id, seed=seed, change_times=change_times,
                                   rates=rates)
        return Manager(sim_opts=self, sources=[piecewise] + self.create_other_sources())

    def create_manager_with_significance(self, seed, time_period, significance=None,
                                         num_segments=None):
        """Manager with an OptPWSignificance broadcaster (opt_model.py:850-884): the
        significance, or s extended to num_segments per follower."""
        num_followers = len(self.sink_ids)
        if significance is not None:
            significance = np.asarray(significance).astype(float)
        else:
            s_vec = np.asarray(self.s)
            if s_vec.shape[0] == 1 and num_segments is not None:
                s_vec = np.ones((num_followers, num_segments), dtype=float) * s_vec[:, None]
            if num_segments is not None:
                s_vec = np.ones((num_followers, num_segments)) * s_vec[:, None]
            significance = s_vec
        assert len(significance.shape) == 2, "Significance must be 2 dimensional."
        assert significance.shape[1] == num_segments or num_segments is None, \
            "Number of segments in significance do not match"
        assert significance.shape[0] == len(self.sink_ids), \
            "Number of sink_ids is not the same as size of significance."
        opt_pw = OptPWSignificance(src_id=self.src_id, seed=seed, s_vec=significance,
                                   time_period=time_period, q=self.q)
        return Manager(sim_opts=self, sources=[opt_pw] + self.create_other_sources())

    def create_manager_for_wall(self):
        edge_list = [x for x in self.edge_list if x[0] != self.src_id]
        return Manager(sim_opts=self.update({'edge_list': edge_list}),
                       sources=self.create_other_sources())

    def create_manager_with_times(self, event_times):
        deterministic = RealData(self.src_id, event_times)
        return Manager(sim_opts=self, sources=[deterministic] + self.create_other_sources())

    def get_dict(self):
        return {'src_id': self.src_id, 'q': self.q, 's': self.s,
                'other_sources': self.other_sources, 'sink_ids': self.sink_ids,
                'edge_list': self.edge_list, 'end_time': self.end_time}

    def copy(self):
        return self.update({})

    def update(self, changes):
        new_opts = self.get_dict()
        new_opts.update(changes)
        return SimOpts(**new_opts)

    @staticmethod
    def std_poisson(world_seed, world_rate):
        return SimOpts(src_id=1,
                       other_sources=[('Poisson2', {'src_id': 2, 'seed': world_seed,
                                                    'rate': world_rate})],
                       end_time=1.0, sink_ids=[1001], s=np.asarray([1.0]), q=1.0,
                       edge_list=[(1, 1001), (2, 1001)])

    @staticmethod
    def std_hawkes(world_seed, world_lambda_0, world_alpha, world_beta):
        assert world_alpha / world_beta <= 1.0, "The Hawkes wall will explode."
        return SimOpts(src_id=1,
                       other_sources=[('Hawkes', {'src_id': 2, 'seed': world_seed,
                                                  'l_0': world_lambda_0, 'alpha': world_alpha,
                                                  'beta': world_beta})],
                       end_time=1.0, sink_ids=[1001], s=np.asarray([1.0]), q=1.0,
                       edge_list=[(1, 1001), (2, 1001)])

    @staticmethod
    def std_piecewise_const(world_seed, world_change_times, world_rates):
        return SimOpts(src_id=1,
                       other_sources=[('PiecewiseConst', {'src_id': 2, 'seed': world_seed,
                                                          'change_times': world_change_times,
                                                          'rates': world_rates})],
                       end_time=1.0, sink_ids=[1001], s=np.asarray([1.0]), q=1.0,
                       edge_list=[(1, 1001), (2, 1001)])
