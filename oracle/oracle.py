"""ctypes front-end of the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg
import this module; the product package ``redqueen_amd`` never does.

Scenarios are described with the reference's own vocabulary: a SimOpts-like
dict (``src_id, s, q, other_sources, sink_ids, edge_list, end_time`` --
opt_model.py:773-780) plus the controlled broadcaster, as in
``create_manager_with_opt`` (:806), ``create_manager_with_poisson`` (:821),
``create_manager_for_wall`` (:886), ``create_manager_with_times`` (:893) and
``create_manager_with_piecewise_const`` (:839).
"""
import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# env RQO_SO_PATH: an alternative build of the same sources (the sanitizer build,
# scripts/asan_cpu.sh)
_LIB = os.environ.get("RQO_SO_PATH") or os.path.join(_HERE, "librq_oracle.so")

POISSON, POISSON2, HAWKES, PWCONST, REALDATA, OPT, OPTPW = 1, 2, 3, 4, 5, 6, 7
KIND = {"Poisson": POISSON, "Poisson2": POISSON2, "Hawkes": HAWKES,
        "PiecewiseConst": PWCONST, "RealData": REALDATA, "Opt": OPT}


class _Source(C.Structure):
    _fields_ = [("kind", C.c_int32), ("n_arr", C.c_int32), ("src_id", C.c_int64),
                ("seed", C.c_uint32), ("flags", C.c_uint32), ("p0", C.c_double), ("p1", C.c_double),
                ("p2", C.c_double), ("a", C.POINTER(C.c_double)), ("b", C.POINTER(C.c_double))]


class _Scenario(C.Structure):
    _fields_ = [("n_sources", C.c_int32), ("sources", C.POINTER(_Source)),
                ("n_sinks", C.c_int32), ("sink_ids", C.POINTER(C.c_int64)),
                ("n_edges", C.c_int64), ("edge_src", C.POINTER(C.c_int64)),
                ("edge_sink", C.POINTER(C.c_int64)), ("start_time", C.c_double),
                ("end_time", C.c_double), ("max_events", C.c_int64)]


class _Events(C.Structure):
    _fields_ = [("cap", C.c_int64), ("n", C.c_int64), ("t", C.POINTER(C.c_double)),
                ("time_delta", C.POINTER(C.c_double)), ("src_id", C.POINTER(C.c_int64))]


VEXP = C.CFUNCTYPE(None, C.POINTER(C.c_double), C.c_int64, C.POINTER(C.c_double))

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        L = C.CDLL(_LIB)
        d, i64, i32 = C.POINTER(C.c_double), C.POINTER(C.c_int64), C.POINTER(C.c_int32)
        L.rqo_npsum.restype = C.c_double
        L.rqo_npsum.argtypes = [d, C.c_int64]
        L.rqo_metrics_df.restype = C.c_int
        L.rqo_metrics_df.argtypes = [d, i64, i64, i64, C.c_int64, C.c_int64, C.c_double,
                                     i32, C.c_int32, C.c_int32, d, i64]
        L.rqo_mt_draws.argtypes = [C.c_uint32, C.c_int32, C.c_double, C.c_double, C.c_int64, d]
        L.rqo_philox4x32_10.argtypes = [C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                        C.POINTER(C.c_uint32)]
        L.rqo_philox_uniform.restype = C.c_double
        L.rqo_philox_uniform.argtypes = [C.c_uint32, C.c_uint32, C.c_uint64]
        L.rqo_kind_salt.restype = C.c_uint32
        L.rqo_kind_salt.argtypes = [C.c_int32]
        L.rqo_ref_run.restype = C.c_int
        L.rqo_ref_run.argtypes = [C.POINTER(_Scenario), VEXP, C.c_int32, C.POINTER(_Events)]
        L.rqo_engine_run.restype = C.c_int
        L.rqo_engine_run.argtypes = [C.POINTER(_Scenario), C.POINTER(_Events)]
        L.rqo_engine_batch.restype = C.c_int64
        L.rqo_engine_batch.argtypes = [C.POINTER(_Scenario), C.c_int64, C.c_uint32, C.c_int32,
                                       i32, C.c_int32, C.c_int32, d, C.c_uint32, C.c_uint32, d, i64]
        L.rqo_oracle_dp.restype = C.c_int
        L.rqo_oracle_dp.argtypes = [d, C.c_int64, C.c_double, C.c_double, d, i64, i64]
        L.rqo_rank_table.restype = C.c_int
        L.rqo_rank_table.argtypes = [d, i64, i32, C.c_int64, C.c_int32, C.c_int64, C.c_int32,
                                     C.c_int64, d, d]
        L.rqo_spec_log.restype = C.c_double
        L.rqo_spec_log.argtypes = [C.c_double]
        L.rqo_spec_exp.restype = C.c_double
        L.rqo_spec_exp.argtypes = [C.c_double]
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(C.POINTER(t))


def npsum(x):
    x = np.ascontiguousarray(x, dtype=np.float64)
    return lib().rqo_npsum(_p(x, C.c_double), x.size)


def metrics_df(t, src, sink, event_id, src_id, end_time, Ks=(1,), row_mode=0):
    """Appendix-B metrics. Returns (top_k list, avg_rank, r_2, counts[4])."""
    t = np.ascontiguousarray(t, dtype=np.float64)
    src = np.ascontiguousarray(src, dtype=np.int64)
    sink = np.ascontiguousarray(sink, dtype=np.int64)
    eid = np.ascontiguousarray(event_id, dtype=np.int64)
    Ks = np.ascontiguousarray(Ks, dtype=np.int32)
    out = np.zeros(len(Ks) + 2)
    cnt = np.zeros(4, dtype=np.int64)
    rc = lib().rqo_metrics_df(_p(t, C.c_double), _p(src, C.c_int64), _p(sink, C.c_int64),
                              _p(eid, C.c_int64), t.size, int(src_id), float(end_time),
                              _p(Ks, C.c_int32), len(Ks), row_mode, _p(out, C.c_double),
                              _p(cnt, C.c_int64))
    if rc:
        raise ValueError("rqo_metrics_df failed: %d" % rc)
    return list(out[:len(Ks)]), out[len(Ks)], out[len(Ks) + 1], cnt


def oracle_dp(w, q, s):
    """utils.oracle_ranking's DP on w = np.diff([0, 0, times..., end]) (n = len(w) - 2).
    Returns (cost, events[n+1], ranks[n+1])."""
    w = np.ascontiguousarray(w, dtype=np.float64)
    n = w.size - 2
    ev = np.zeros(n + 1, dtype=np.int64)
    rk = np.zeros(n + 1, dtype=np.int64)
    cost = C.c_double()
    rc = lib().rqo_oracle_dp(_p(w, C.c_double), n, float(q), float(s), C.byref(cost),
                             _p(ev, C.c_int64), _p(rk, C.c_int64))
    if rc:
        raise ValueError("rqo_oracle_dp failed: %d" % rc)
    return cost.value, ev, rk


def rank_table(t, src, sink, src_id, fill=True):
    """utils.rank_of_src_in_df -> (table [n_t][S], index [n_t], sorted sink ids)."""
    t = np.ascontiguousarray(t, dtype=np.float64)
    src = np.ascontiguousarray(src, dtype=np.int64)
    sinks, col = np.unique(np.asarray(sink), return_inverse=True)
    col = np.ascontiguousarray(col, dtype=np.int32)
    n_t = int(np.unique(t).size)
    tab = np.zeros((n_t, sinks.size))
    idx = np.zeros(n_t)
    rc = lib().rqo_rank_table(_p(t, C.c_double), _p(src, C.c_int64), _p(col, C.c_int32), t.size,
                              sinks.size, int(src_id), int(bool(fill)), n_t, _p(tab, C.c_double),
                              _p(idx, C.c_double))
    if rc:
        raise ValueError("rqo_rank_table failed: %d" % rc)
    return tab, idx, sinks


def mt_draws(seed, kind, p=0.0, q=0.0, n=16):
    out = np.zeros(n)
    lib().rqo_mt_draws(seed, kind, p, q, n, _p(out, C.c_double))
    return out


def philox(ctr, key):
    c = (C.c_uint32 * 4)(*ctr)
    k = (C.c_uint32 * 2)(*key)
    o = (C.c_uint32 * 4)()
    lib().rqo_philox4x32_10(c, k, o)
    return list(o)


class Scenario:
    """Flattened scenario: sources[0] is the controlled broadcaster."""

    def __init__(self, sim_opts, ctrl, max_events=None, start_time=0.0):
        so = sim_opts
        src_id = so["src_id"]
        edges = list(so["edge_list"])
        kind = ctrl[0]
        if kind == "wall":
            edges = [e for e in edges if e[0] != src_id]
        self._keep = []
        srcs = []
        if kind == "opt":
            fol = sorted(e[1] for e in edges if e[0] == src_id)
            s = so["s"]
            if isinstance(s, dict):
                svec = np.asarray([s[x] for x in fol], dtype=float)
            else:
                svec = np.ones(len(fol)) * np.asarray(s, dtype=float)
            srcs.append(self._src(OPT, src_id, ctrl[1], q=so["q"], a=svec))
        elif kind == "poisson":
            srcs.append(self._src(POISSON2, src_id, ctrl[1], rate=ctrl[2]))
        elif kind == "pwconst":
            srcs.append(self._src(PWCONST, src_id, ctrl[1], a=ctrl[2], b=ctrl[3]))
        elif kind == "times":
            srcs.append(self._src(REALDATA, src_id, 0, a=ctrl[1]))
        elif kind == "sig":
            # ("sig", seed, s_pw [sorted followers][S], time_period): OptPWSignificance
            spw = np.atleast_2d(np.asarray(ctrl[2], dtype=np.float64))
            src = self._src(OPTPW, src_id, ctrl[1], q=so["q"], a=spw.ravel())
            src.n_arr = spw.shape[1]
            src.p1 = float(ctrl[3])
            srcs.append(src)
        elif kind == "wall":
            srcs.append(self._src(0, src_id, 0))
        else:
            raise ValueError(kind)
        for name, kw in so["other_sources"]:
            k = KIND[name]
            if k == HAWKES:
                srcs.append(self._src(k, kw["src_id"], kw["seed"], l0=kw.get("l_0", 1.0),
                                      alpha=kw.get("alpha", 1.0), beta=kw.get("beta", 10.0)))
            elif k in (POISSON, POISSON2):
                srcs.append(self._src(k, kw["src_id"], kw["seed"], rate=kw.get("rate", 1.0)))
            elif k == PWCONST:
                srcs.append(self._src(k, kw["src_id"], kw["seed"], a=kw["change_times"],
                                      b=kw["rates"]))
            elif k == REALDATA:
                srcs.append(self._src(k, kw["src_id"], 0, a=kw["times"]))
                srcs[-1].flags = 1 if kw.get("dynamic") else 0
            else:
                raise ValueError(name)
        self.sources = srcs
        self.src_id = src_id
        self.end_time = float(so["end_time"])
        self.edges = edges
        self.sink_ids = np.asarray(so["sink_ids"], dtype=np.int64)
        self.edge_src = np.asarray([e[0] for e in edges], dtype=np.int64)
        self.edge_sink = np.asarray([e[1] for e in edges], dtype=np.int64)
        arr = (_Source * len(srcs))(*srcs)
        self._arr = arr
        self.c = _Scenario(len(srcs), arr, len(self.sink_ids), _p(self.sink_ids, C.c_int64),
                           len(edges), _p(self.edge_src, C.c_int64), _p(self.edge_sink, C.c_int64),
                           float(start_time), self.end_time,
                           -1 if max_events is None else int(max_events))

    def _src(self, kind, sid, seed, rate=0.0, l0=0.0, alpha=0.0, beta=0.0, q=1.0, a=None, b=None):
        s = _Source()
        s.kind, s.src_id, s.seed = kind, int(sid), int(seed) & 0xFFFFFFFF
        if kind in (POISSON, POISSON2):
            s.p0 = float(rate)
        elif kind == HAWKES:
            s.p0, s.p1, s.p2 = float(l0), float(alpha), float(beta)
        elif kind in (OPT, OPTPW):
            s.p0 = float(q)
        if a is not None:
            a = np.ascontiguousarray(a, dtype=np.float64)
            self._keep.append(a)
            s.a = _p(a, C.c_double)
            s.n_arr = a.size
        if b is not None:
            b = np.ascontiguousarray(b, dtype=np.float64)
            self._keep.append(b)
            s.b = _p(b, C.c_double)
        return s

    def sinks_of(self, sid):
        return [e[1] for e in self.edges if e[0] == sid]

    def expand(self, ev_t, ev_dt, ev_src):
        """Events -> reference df columns (State.get_dataframe, opt_model.py:85-97)."""
        # one row per (event, sink): events in play order, each event's sinks in
        # edge_list order (duplicates kept) -- vectorised as a CSR gather
        ev_src = np.asarray(ev_src, dtype=np.int64)
        if self.edge_src.size == 0:
            ev_src = ev_src[:0]
        order = np.argsort(self.edge_src, kind="stable")          # edge-list order per source
        srcs, first, deg = np.unique(self.edge_src[order], return_index=True, return_counts=True)
        col = self.edge_sink[order]
        k = np.searchsorted(srcs, ev_src)
        known = (k < len(srcs)) & (srcs[np.minimum(k, len(srcs) - 1)] == ev_src)
        d = np.where(known, deg[np.minimum(k, len(srcs) - 1)], 0)
        beg = np.where(known, first[np.minimum(k, len(srcs) - 1)], 0)
        ev = np.repeat(np.arange(len(ev_src)), d)
        within = np.arange(ev.size) - np.repeat(np.cumsum(d) - d, d)
        return dict(event_id=(100 + ev).astype(np.int64),
                    time_delta=np.asarray(ev_dt, dtype=np.float64)[ev],
                    src_id=ev_src[ev], t=np.asarray(ev_t, dtype=np.float64)[ev],
                    sink_id=col[np.repeat(beg, d) + within].astype(np.int64))


def state_time_deltas(t, start=0.0):
    """Event.time_delta of the reference for event times t: time_delta_k = t_k - time,
    time += time_delta_k, time starting at start (opt_model.py:68, :304)."""
    out = np.empty(len(t))
    s = float(start)
    for k, tk in enumerate(np.asarray(t, dtype=np.float64)):
        out[k] = tk - s
        s = s + out[k]
    return out


def _events(cap):
    t = np.zeros(cap); dt = np.zeros(cap); s = np.zeros(cap, dtype=np.int64)
    ev = _Events(cap, 0, _p(t, C.c_double), _p(dt, C.c_double), _p(s, C.c_int64))
    return ev, t, dt, s


def _numpy_vexp(x, n, out):
    if n:
        xa = np.ctypeslib.as_array(x, shape=(n,))
        oa = np.ctypeslib.as_array(out, shape=(n,))
        oa[:] = np.exp(xa)


_VEXP_NUMPY = VEXP(_numpy_vexp)


def ref_run(sc, numpy_exp=True, dot_fma=1, cap=1 << 20):
    """Reference-exact run_dynamic (MT19937).  Returns (t, time_delta, src_id)."""
    ev, t, dt, s = _events(cap)
    fn = _VEXP_NUMPY if numpy_exp else C.cast(None, VEXP)
    rc = lib().rqo_ref_run(C.byref(sc.c), fn, dot_fma, C.byref(ev))
    if rc:
        raise RuntimeError("rqo_ref_run failed: %d" % rc)
    return t[:ev.n].copy(), dt[:ev.n].copy(), s[:ev.n].copy()


def engine_run(sc, cap=1 << 22):
    """Engine-semantics run (Philox).  Returns (t, time_delta, src_id)."""
    ev, t, dt, s = _events(cap)
    rc = lib().rqo_engine_run(C.byref(sc.c), C.byref(ev))
    if rc:
        raise RuntimeError("rqo_engine_run failed: %d" % rc)
    return t[:ev.n].copy(), dt[:ev.n].copy(), s[:ev.n].copy()


def engine_metrics(sc, Ks=(1,)):
    """Engine run + Appendix-B metrics on its expanded df."""
    t, dt, s = engine_run(sc)
    df = sc.expand(t, dt, s)
    if df["t"].size == 0:
        return None, (t, dt, s)
    return metrics_df(df["t"], df["src_id"], df["sink_id"], df["event_id"], sc.src_id,
                      sc.end_time, Ks), (t, dt, s)


def engine_batch(sc, n_rep, seed0=0, randomize=True, Ks=(1,), n_threads=1, ctrl_rates=None,
                 ctrl_seed_offset=0, seed_stride=1):
    """n_rep replicas: replica r uses seed u + ctrl_seed_offset (u = seed0 + r) for the
    controlled source and,
    with randomize, u + 99*idx for other source idx.  Returns (metrics [n_rep, nK+2],
    counts [n_rep, 3] = posts, world, events, total events)."""
    Ks = np.ascontiguousarray(Ks, dtype=np.int32)
    out = np.zeros((n_rep, len(Ks) + 2))
    cnt = np.zeros((n_rep, 3), dtype=np.int64)
    rp = None
    if ctrl_rates is not None:
        rates = np.ascontiguousarray(ctrl_rates, dtype=np.float64)
        rp = _p(rates, C.c_double)
    tot = lib().rqo_engine_batch(C.byref(sc.c), n_rep, seed0, int(randomize),
                                 _p(Ks, C.c_int32), len(Ks), n_threads, rp, ctrl_seed_offset,
                                 seed_stride, _p(out, C.c_double), _p(cnt, C.c_int64))
    if tot < 0:
        raise RuntimeError("rqo_engine_batch failed: %d" % tot)
    return out, cnt, tot
