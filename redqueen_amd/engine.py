"""Engine front-end: a device-resident graph + batched runs through librq.so.

``Graph`` is the compiled form of a SimOpts (opt_model.py:755-967): other
sources, sinks and edge list are validated like ``Manager.__init__``
(opt_model.py:145-181) and uploaded once.  ``Graph.run`` enqueues one batch
(seeds x grid points) on the current torch stream and returns torch tensors;
torch is only the device-memory / stream plumbing.
"""
import ctypes as C
import math

import numpy as np
import torch

from . import _lib as L

KIND_BY_NAME = {"Poisson": L.SRC_POISSON, "Poisson2": L.SRC_POISSON2, "Hawkes": L.SRC_HAWKES,
                "PiecewiseConst": L.SRC_PWCONST, "RealData": L.SRC_REALDATA, "Opt": L.SRC_OPT}
CTRL_BY_NAME = {"opt": L.SRC_OPT, "poisson": L.SRC_POISSON2, "pwconst": L.SRC_PWCONST,
                "times": L.SRC_REALDATA, "wall": L.SRC_NONE, "sig": L.SRC_OPTPW}


def _arr(x, dt):
    return np.ascontiguousarray(np.asarray(x, dtype=dt))


def _source_class(name):
    """The class behind an other_sources entry: a built-in name, a name registered
    with SimOpts.registerSource (opt_model.py:768-771), or a callable."""
    if isinstance(name, str):
        if name in KIND_BY_NAME:
            return None
        from .opt_model import SimOpts
        cls = SimOpts.broadcasters.get(name)
        if cls is None:
            raise ValueError("Unknown type of broadcaster: {}".format(name))
        return cls
    return name


def _source_kind(name):
    if isinstance(name, str) and name in KIND_BY_NAME:
        return KIND_BY_NAME[name]
    cls = _source_class(name)
    kind = getattr(cls, "_rq_kind", None)
    return L.SRC_REALDATA if kind is None else kind   # a plugin: its times as RealData


class Graph:
    """Compiled network.  ``other_sources``: list of (name-or-class, kwargs)."""

    def __init__(self, src_id, other_sources, sink_ids, edge_list, end_time, start_time=0.0,
                 ctrl_a=None, ctrl_b=None):
        self._keep = []
        srcs = []
        self.has_realdata = False
        # registered static plugin broadcasters: (position in other_sources, class, kwargs)
        self.plugins = []
        # src_ids of the static wall sources (run_dynamic plays their times only when
        # strictly earlier than the dynamic sources' next event, opt_model.py:289-290)
        self.static_src_ids = set()
        for idx, (name, kw) in enumerate(other_sources):
            kind = _source_kind(name)
            cls = _source_class(name)
            dyn_plugin = False
            if cls is not None and getattr(cls, "_rq_kind", None) is None:
                # graph-level times: the instance its own kwargs make (the seed as given);
                # randomized batches replace them per replica (run(randomize=True)).  A
                # dynamic plugin must be self-driven: every run checks it (_verify_dynamic)
                from .opt_model import source_times
                inst = cls(**kw)
                dyn = bool(getattr(inst, "is_dynamic", True))
                self.plugins.append((idx, cls, dict(kw), int(kw["src_id"]), dyn))
                dyn_plugin = dyn
                kw = {"src_id": kw["src_id"],
                      "times": source_times(inst, float(start_time), sink_ids, edge_list,
                                            float(end_time))}
            self.has_realdata = self.has_realdata or kind == L.SRC_REALDATA
            # a dynamic broadcaster replayed from its times (a dynamic plugin, or RealData
            # kwargs dynamic=True): equal times order it as a dynamic source
            dyn_rd = kind == L.SRC_REALDATA and (bool(kw.get("dynamic")) or dyn_plugin)
            if kind in (L.SRC_POISSON2, L.SRC_PWCONST) or (kind == L.SRC_REALDATA and not dyn_rd):
                self.static_src_ids.add(int(kw["src_id"]))
            if kind == L.SRC_OPT:
                raise NotImplementedError("an Opt broadcaster among the other sources")
            d = L.SourceDesc()
            d.kind = kind
            d.src_id = int(kw["src_id"])
            d.seed = int(kw.get("seed", 0)) & 0xFFFFFFFF
            d.flags = L.SRCF_DYNAMIC if dyn_rd else 0
            if kind in (L.SRC_POISSON, L.SRC_POISSON2):
                d.p0 = float(kw.get("rate", 1.0))
            elif kind == L.SRC_HAWKES:
                d.p0 = float(kw.get("l_0", 1.0))
                d.p1 = float(kw.get("alpha", 1.0))
                d.p2 = float(kw.get("beta", 10.0))
            elif kind == L.SRC_PWCONST:
                a = _arr(kw["change_times"], np.float64)
                b = _arr(kw["rates"], np.float64)
                if a.size != b.size:
                    raise ValueError("change_times and rates differ in length")
                self._keep += [a, b]
                d.n_arr = a.size
                d.a = a.ctypes.data_as(L._pd)
                d.b = b.ctypes.data_as(L._pd)
            elif kind == L.SRC_REALDATA:
                a = _arr(kw["times"], np.float64)
                self._keep.append(a)
                d.n_arr = a.size
                d.a = a.ctypes.data_as(L._pd)
            srcs.append(d)
        self.src_id = int(src_id)
        self.end_time = float(end_time)
        self.start_time = float(start_time)
        self.sink_ids = _arr(sink_ids, np.int64)
        edges = list(edge_list)
        self._edges = edges
        self.edge_src = _arr([e[0] for e in edges], np.int64)
        self.edge_sink = _arr([e[1] for e in edges], np.int64)
        arr = (L.SourceDesc * max(1, len(srcs)))(*srcs)
        gd = L.GraphDesc()
        gd.n_sources = len(srcs)
        gd.sources = arr
        gd.n_sinks = self.sink_ids.size
        gd.sink_ids = self.sink_ids.ctypes.data_as(L._pi64)
        gd.n_edges = len(edges)
        gd.edge_src = self.edge_src.ctypes.data_as(L._pi64)
        gd.edge_sink = self.edge_sink.ctypes.data_as(L._pi64)
        gd.ctrl_src_id = self.src_id
        gd.start_time = self.start_time
        gd.end_time = self.end_time
        if ctrl_a is not None:
            ca = _arr(ctrl_a, np.float64)
            self._keep.append(ca)
            gd.ctrl_n_arr = ca.size
            gd.ctrl_a = ca.ctypes.data_as(L._pd)
            if ctrl_b is not None:
                cb = _arr(ctrl_b, np.float64)
                self._keep.append(cb)
                gd.ctrl_b = cb.ctypes.data_as(L._pd)
        h = C.c_void_p()
        L.check("rq_graph_build", L.lib().rq_graph_build(C.byref(gd), C.byref(h)))
        self._h = h
        info = np.zeros(8, dtype=np.int64)
        L.lib().rq_graph_info(h, info.ctypes.data_as(L._pi64))
        self.n_streams, self.n_sinks, self.n_followers, self.n_edges, self.ctrl_idx = (
            int(v) for v in info[:5])
        self.stream_src_ids = np.zeros(self.n_streams, dtype=np.int64)
        L.lib().rq_graph_source_ids(h, self.stream_src_ids.ctypes.data_as(L._pi64))
        self.followers = np.zeros(max(1, self.n_followers), dtype=np.int64)[:self.n_followers]
        if self.n_followers:
            L.lib().rq_graph_followers(h, self.followers.ctypes.data_as(L._pi64))
        # one workspace per caller stream: batches enqueued on different streams may run
        # at the same time and must not share buffers
        self._wss = {}
        self._cap_scale = {}   # _cap_key(...) -> cap_scale an overflow rerun needed (reset_capacity_memo)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                L.lib().rq_graph_free(h)
            except Exception:
                pass

    def workspace_bytes(self, stream=None):
        """Bytes of the workspace held for ``stream`` (default: the current stream)."""
        use = stream or torch.cuda.current_stream()
        ws = self._wss.get(use.cuda_stream)
        return 0 if ws is None else ws.numel()

    def release_workspaces(self):
        """Drop every stream's workspace (the caching allocator keeps the blocks)."""
        self._wss.clear()

    # ------------------------------------------------------------------
    def s_matrix(self, s, n_grid=1):
        """s as in SimOpts (scalar, vector over sorted followers, or dict sink->s)."""
        F = self.n_followers
        if isinstance(s, dict):
            row = np.asarray([s[int(x)] for x in self.followers], dtype=np.float64)
        else:
            row = np.ones(F, dtype=np.float64) * np.asarray(s, dtype=np.float64)
        return np.ascontiguousarray(np.tile(row, (n_grid, 1)))

    def run(self, *args, stream=None, **kw):
        """Enqueue one batch on ``stream`` (default: the current torch stream).  Every
        tensor the batch reads or writes is allocated with that stream current, so
        the caching allocator, the library and the status check all agree on it.
        With a dynamic plugin among the sources, the batch's replicas (all of a batch of
        <= 64, else a seeded sample of 64) are checked to be self-driven (_verify_dynamic);
        when one reacts to other sources' events the whole batch is replayed to the
        reactive fixed point (_run_reactive) before the result is returned."""
        from .opt_model import PluginReacts
        use = stream or torch.cuda.current_stream()
        with torch.cuda.stream(use):
            res = self._run(*args, stream=use, **kw)
            if any(p[4] for p in self.plugins) and not kw.get("plan_only"):
                try:
                    self._verify_dynamic(args, dict(kw, stream=use), res)
                except PluginReacts:
                    res = self._run_reactive(args, dict(kw, stream=use), res)
            return res

    def _run(self, ctrl="opt", q=1.0, s=None, n_rep=1, ctrl_seed=0, world_seed=0,
            randomize=False, seed_mod=0, ctrl_rate=None, Ks=(1,), max_events=None,
            event_log=False, cap_scale=1.0, chunk=0, stream=None, check=True, sweep_mode=0, replica0=0, n_local=0,
            plan_only=False, s_pw=None, period=None, rep_lo=0, rep_cnt=0, rd_override=None,
            rd_streams=None, rep_idx=None):
        """Enqueue one batch.  ``q``: scalar or [n_grid]; ``s``: per grid point
        row(s) over the sorted followers ([n_grid, F]) or anything ``s_matrix``
        takes.  Seeds: int base (seed + replica id) or a device uint32 tensor.
        ``ctrl="sig"`` (OptPWSignificance): ``s_pw`` [F, S] or [n_grid, F, S] over the
        sorted followers and ``period`` T.
        ``rep_lo`` / ``rep_cnt``: run only replicas [rep_lo, rep_lo + rep_cnt) of every grid
        point (a balanced multi-GPU shard, rq_batch_desc.rep_lo); ``replica0`` / ``n_local``
        then index that n_grid x rep_cnt space, and so do the outputs.
        ``rd_streams = (src_ids, times, off, caps)``: per-replica times of the graph's
        RealData sources ``src_ids`` (declared with no times) already on the device --
        replica i (global id) plays times[off[i * n + k] .. off[i * n + k + 1]) for source
        k, sorted, within [start_time, end_time]; ``caps[k]`` >= any replica's count
        (rq_batch_desc.rd_*, read in place: no host pass per replica).
        ``rep_idx``: run exactly these global replica ids (rq_batch_desc.rep_idx; replica0,
        n_local and the rep_lo / rep_cnt window are then ignored); output k = rep_idx[k]."""
        dev = torch.device("cuda", torch.cuda.current_device())
        ck = CTRL_BY_NAME[ctrl] if isinstance(ctrl, str) else int(ctrl)
        qv = _arr(np.atleast_1d(q), np.float64)
        n_grid = qv.size
        if ck == L.SRC_OPT:
            if s is None:
                raise ValueError("s required for the RedQueen broadcaster")
            sm = np.asarray(s, dtype=np.float64) if (isinstance(s, np.ndarray) and s.ndim == 2) \
                else self.s_matrix(s, n_grid)
            sm = np.ascontiguousarray(sm, dtype=np.float64)
            if sm.shape != (n_grid, self.n_followers):
                raise ValueError("s must be [n_grid, n_followers]")
        else:
            sm = np.zeros((n_grid, max(1, self.n_followers)))
        spw = None
        if ck == L.SRC_OPTPW:
            if s_pw is None or period is None:
                raise ValueError("s_pw and period required for OptPWSignificance")
            spw = np.asarray(s_pw, dtype=np.float64)
            if spw.ndim == 2:
                spw = np.broadcast_to(spw, (n_grid,) + spw.shape)
            spw = np.ascontiguousarray(spw)
            if spw.ndim != 3 or spw.shape[:2] != (n_grid, self.n_followers) or spw.shape[2] < 1:
                raise ValueError("s_pw must be [n_grid, n_followers, n_segments]")
        R_all = n_grid * int(n_rep)
        cnt = int(rep_cnt) if rep_cnt else int(n_rep)
        lo = int(rep_lo) if rep_cnt else 0
        R = int(n_local) if n_local else n_grid * cnt - int(replica0)
        # global replica ids of this call's outputs (rq_global_replica)
        sp = np.arange(int(replica0), int(replica0) + R, dtype=np.int64)
        gids = sp if cnt == int(n_rep) else (sp // cnt) * int(n_rep) + lo + sp % cnt
        if rep_idx is not None:
            gids = _arr(rep_idx, np.int64)
            R, replica0, n_local, lo, rep_cnt = gids.size, 0, gids.size, 0, 0
            if R < 1 or gids.min() < 0 or gids.max() >= R_all:
                raise ValueError("rep_idx: global ids in [0, n_grid * n_rep) expected")
        Ks = _arr(Ks, np.int32)
        if not 1 <= Ks.size <= L.MAX_K:
            raise ValueError("1..%d K values per run" % L.MAX_K)
        b = L.BatchDesc()
        b.ctrl_kind = ck
        b.n_grid = n_grid
        b.q = qv.ctypes.data_as(L._pd)
        b.s = sm.ctypes.data_as(L._pd)
        b.n_rep = int(n_rep)
        keep = []
        if torch.is_tensor(ctrl_seed):
            cs = ctrl_seed.to(device=dev, dtype=torch.int32).contiguous()
            keep.append(cs)
            b.ctrl_seed = cs.data_ptr()
        else:
            b.ctrl_seed0 = int(ctrl_seed) & 0xFFFFFFFF
        b.randomize_world = int(bool(randomize))
        if torch.is_tensor(world_seed):
            ws_ = world_seed.to(device=dev, dtype=torch.int32).contiguous()
            keep.append(ws_)
            b.world_seed = ws_.data_ptr()
        else:
            b.world_seed0 = int(world_seed) & 0xFFFFFFFF
        b.seed_mod = int(seed_mod)
        if rd_streams is not None:
            if self.plugins:
                raise ValueError("rd_streams and registered plugin broadcasters are exclusive")
            sids, td, to, caps = rd_streams
            sid = _arr(sids, np.int64)
            cap = _arr(caps, np.int64)
            if not (torch.is_tensor(td) and torch.is_tensor(to) and td.dtype == torch.float64 and
                    to.dtype == torch.int64 and td.is_cuda and to.is_cuda and to.is_contiguous()
                    and td.is_contiguous() and to.numel() == R_all * sid.size + 1
                    and cap.size == sid.size and 1 <= sid.size <= L.MAX_RD):
                raise ValueError("rd_streams: (src_ids[n], device f64 times, device i64 "
                                 "off[n_grid * n_rep * n + 1], caps[n]) expected")
            keep += [sid, cap, td, to]
            b.n_rd = sid.size
            b.rd_src_id = sid.ctypes.data_as(L._pi64)
            b.rd_cap = cap.ctypes.data_as(L._pi64)
            b.rd_times = td.data_ptr()
            b.rd_off = to.data_ptr()
        elif self.plugins and (randomize or rd_override is not None):
            self._plugin_streams(b, keep, dev, R_all, gids, world_seed, int(seed_mod), rd_override)
        if ck == L.SRC_POISSON2:
            if ctrl_rate is None:
                raise ValueError("ctrl_rate required for a Poisson controlled source")
            cr = torch.as_tensor(ctrl_rate, dtype=torch.float64, device=dev).reshape(-1)
            if cr.numel() == 1:
                cr = cr.expand(R_all)
            cr = cr.contiguous()
            keep.append(cr)
            b.ctrl_rate = cr.data_ptr()
            b.ctrl_rate_max = float(cr.max().item()) if cr.numel() else 0.0
        b.Ks = Ks.ctypes.data_as(L._pi32)
        b.nK = Ks.size
        b.max_events = -1 if max_events is None or max_events == float("inf") else int(max_events)
        b.flags = L.RUN_EVENT_LOG if event_log else 0
        b.cap_scale = float(cap_scale)
        b.chunk = int(chunk)
        b.sweep_mode = int(sweep_mode)
        b.replica0 = int(replica0)
        b.n_local = int(n_local)
        b.rep_lo = lo
        b.rep_cnt = int(rep_cnt)
        if rep_idx is not None:
            keep.append(gids)
            b.rep_idx = gids.ctypes.data_as(L._pi64)
        if spw is not None:
            b.n_seg = spw.shape[2]
            b.period = float(period)
            b.s_pw = spw.ctypes.data_as(L._pd)
        lib = L.lib()
        if plan_only:
            b.ws_budget = self._ws_budget(dev)
            info = (C.c_int64 * 8)()
            L.check("rq_plan_info", lib.rq_plan_info(self._h, C.byref(b), info))
            keys = ("variant", "sources_per_lane", "ring_depth", "waves_per_block",
                    "blocks_per_cu", "columns_in_lds", "lds_bytes_per_block", "chunk")
            return dict(zip(keys, (int(v) for v in info)))
        return self._run_loop(lib, b, keep, dev, R, Ks, n_grid, n_rep, ck, event_log,
                              gids, check, stream)

    def _launch(self, lib, b, dev, R, Ks, n_grid, n_rep, event_log, use):
        """One rq_run_batch of R output replicas on stream ``use``.  The outputs (and the
        event log) are allocated first, so the workspace budget is what is left after them."""
        sk = use.cuda_stream
        metrics = torch.empty((R, Ks.size + 2), dtype=torch.float64, device=dev)
        counts = torch.empty((R, 4), dtype=torch.int64, device=dev)
        status = torch.empty(R, dtype=torch.int32, device=dev)
        out = L.Outputs()
        out.metrics, out.counts, out.status = metrics.data_ptr(), counts.data_ptr(), status.data_ptr()
        ev_t = ev_src = None
        if event_log:
            cap = C.c_int64()
            L.check("rq_event_capacity", lib.rq_event_capacity(self._h, C.byref(b), C.byref(cap)))
            ev_t = torch.empty((R, cap.value), dtype=torch.float64, device=dev)
            ev_src = torch.empty((R, cap.value), dtype=torch.int32, device=dev)
            out.ev_t, out.ev_src, out.ev_cap = ev_t.data_ptr(), ev_src.data_ptr(), cap.value
        nbytes = C.c_size_t()
        b.ws_budget = self._ws_budget(dev, sk)
        L.check("rq_workspace_size", lib.rq_workspace_size(self._h, C.byref(b), C.byref(nbytes)))
        ws = self._wss.get(sk)
        if ws is None or ws.numel() < nbytes.value:
            self._wss[sk] = ws = None
            ws = self._wss[sk] = torch.empty(max(256, nbytes.value), dtype=torch.uint8, device=dev)
        L.check("rq_run_batch", lib.rq_run_batch(self._h, C.byref(b), C.byref(out),
                                                 ws.data_ptr(), ws.numel(), sk))
        return BatchResult(self, metrics, counts, status, ev_t, ev_src, Ks, n_grid, int(n_rep))

    # an overflow memo is kept only when at least this share of a batch overflowed (a
    # few flagged replicas rerun alone, cheaply; a batch mostly over capacity would pay a
    # second pass every call)
    CAP_MEMO_SHARE = 1.0 / 16

    def _cap_key(self, b, ck):
        """Capacity-relevant inputs of a run: controller kind, max_events set, sweep
        mode, and the octave of the controller's rate parameter (RedQueen: the q range;
        Poisson: the largest rate) -- an overflow at one q says nothing about another."""
        qk = None
        if ck in (L.SRC_OPT, L.SRC_OPTPW) and b.n_grid > 0:
            qs = np.ctypeslib.as_array(b.q, shape=(b.n_grid,))
            qk = (int(np.floor(np.log2(max(qs.min(), 1e-300)))), int(np.floor(np.log2(max(qs.max(), 1e-300)))))
        elif ck == L.SRC_POISSON2:
            qk = int(np.floor(np.log2(max(b.ctrl_rate_max, 1e-300))))
        return (ck, b.max_events >= 0, int(b.sweep_mode), qk)

    def reset_capacity_memo(self):
        """Forget the capacity scales earlier overflow reruns of this graph remembered."""
        self._cap_scale.clear()

    def _run_loop(self, lib, b, keep, dev, R, Ks, n_grid, n_rep, ck, event_log, gids,
                  check, use):
        """The batch, then -- with ``check`` -- only its flagged replicas again
        (rq_batch_desc.rep_idx: the same global ids, so the same seeds and inputs): an
        overflowed one (RQ_ST_*_OVERFLOW) at doubled capacities, a tie-flagged one of a
        fast sweep (RQ_ST_TIE: equal event times) on the exact sequential sweep; their
        rows replace the flagged rows.  ``self.reruns`` counts the replicas rerun."""
        key = self._cap_key(b, ck)
        b.cap_scale = max(b.cap_scale, self._cap_scale.get(key, 1.0))
        res = self._launch(lib, b, dev, R, Ks, n_grid, n_rep, event_log, use)
        res.replica0 = int(gids[0]) if len(gids) else 0
        res.global_ids = gids
        self.reruns = 0
        if not check:
            return res
        gids = np.asarray(gids, dtype=np.int64)
        # per output replica: the sweep mode it last ran with, and whether that run was the
        # exact sequential sweep (from the library's own plan: rq_plan_info variant 1 / 4)
        mode = np.full(R, int(b.sweep_mode), dtype=np.int64)
        seq = np.full(R, b.sweep_mode == 2 or self._plan_variant(lib, b) % 10 in (1, 4))
        scale = np.full(R, float(b.cap_scale))
        while True:
            use.synchronize()
            st = res.status.cpu().numpy()
            if (st & L.ST_UNORDERED).any():
                raise NotImplementedError(
                    "more than 2048 arrivals at one time in a sequential run over > 2048 sources "
                    "(RQ_ST_UNORDERED): their play order is not the reference's")
            ovf = (st & (L.ST_ROWS_OVERFLOW | L.ST_STREAM_OVERFLOW)) != 0
            tie = ((st & L.ST_TIE) != 0) & ~seq & ~ovf
            if not ovf.any() and not tie.any():
                return res
            if ovf.any():
                if scale[ovf].max() > 64:
                    raise L.RQError("rq_run_batch", L.RQ_EOVERFLOW)
                scale[ovf] *= 2.0
                if ovf.sum() >= self.CAP_MEMO_SHARE * R:
                    self._cap_scale[key] = max(self._cap_scale.get(key, 1.0), float(scale[ovf].max()))
            # equal event times in a fast tiled sweep: those replicas on the exact sequential sweep
            mode[tie] = 2
            seq[tie] = True
            # one rerun per (sweep mode, capacity scale) group of flagged replicas
            flagged = np.flatnonzero(ovf | tie)
            for m_, s_ in sorted({(int(mode[k]), float(scale[k])) for k in flagged}):
                pick = flagged[(mode[flagged] == m_) & (scale[flagged] == s_)]
                self._rerun_into(lib, b, dev, res, pick, gids[pick], s_, m_, Ks, n_grid, n_rep,
                                 event_log, use)
                self.reruns += int(pick.size)

    def _rerun_into(self, lib, b, dev, res, pick, ids, scale, mode, Ks, n_grid, n_rep, event_log, use):
        """Rerun global replicas ``ids`` (outputs ``pick`` of ``res``) and scatter them in."""
        sub = L.BatchDesc.from_buffer_copy(b)
        idx = np.ascontiguousarray(ids, dtype=np.int64)
        sub.rep_idx = idx.ctypes.data_as(L._pi64)
        sub.replica0, sub.n_local, sub.rep_lo, sub.rep_cnt = 0, int(idx.size), 0, 0
        sub.cap_scale = float(scale)
        sub.sweep_mode = int(mode)
        sub.chunk = 0
        r = self._launch(lib, sub, dev, int(idx.size), Ks, n_grid, n_rep, event_log, use)
        _scatter(res, pick, r, dev, event_log)

    def _ws_budget(self, dev, sk=None):
        """The workspace's device-memory budget (rq_batch_desc.ws_budget): 0.9 x what this
        process can get -- the device's free memory, torch's cached (reserved, unallocated)
        blocks and the stream's own workspace, which the next one replaces."""
        if not torch.cuda.is_available():
            return 0   # plan queries without a device: the library's default
        free, _total = torch.cuda.mem_get_info(dev)
        cached = torch.cuda.memory_reserved(dev) - torch.cuda.memory_allocated(dev)
        ws = self._wss.get(sk if sk is not None else torch.cuda.current_stream().cuda_stream)
        held = ws.numel() if ws is not None else 0
        return int(0.9 * (free + cached + held))

    def _plugin_streams(self, b, keep, dev, R_all, gids, world_seed, seed_mod, override=None):
        """Per-replica times of the registered plugin broadcasters of a randomized
        batch: replica i's instance gets seed u_i + 99 idx (randomize_other_sources,
        opt_model.py:795-804) and the host runs its initialize() / get_all_times() (or a
        self-driven dynamic plugin's schedule); ``override``: {global id: [times per
        plugin]} instead (the reactive fixed point).  The times reach the kernels as
        per-replica RealData streams (rq_batch_desc.rd_*)."""
        wseed = world_seed.to(torch.int64).cpu().numpy() if torch.is_tensor(world_seed) else None
        nrd = len(self.plugins)
        if nrd > L.MAX_RD:
            raise NotImplementedError("more than %d plugin broadcasters" % L.MAX_RD)
        counts = np.zeros((R_all, nrd), dtype=np.int64)
        chunks = []
        for i in gids:   # increasing: rd_off is a prefix over the global ids
            i = int(i)
            ts = override[i] if override is not None else \
                [self._plugin_source_times(inst)
                 for inst in self._plugin_instances(i, wseed, world_seed, seed_mod)]
            for c, t in enumerate(ts):
                t = np.asarray(t, dtype=np.float64)
                counts[i, c] = t.size
                chunks.append(t)
        off = np.concatenate([[0], np.cumsum(counts.ravel())]).astype(np.int64)
        times = np.concatenate(chunks) if chunks else np.zeros(0)
        td = torch.from_numpy(np.ascontiguousarray(np.concatenate([times, [0.0]]))).to(dev)
        to = torch.from_numpy(off).to(dev)
        sid = _arr([p[3] for p in self.plugins], np.int64)
        cap = _arr(counts.max(0) if R_all else np.zeros(nrd), np.int64)
        keep += [td, to, sid, cap]
        b.n_rd = nrd
        b.rd_src_id = sid.ctypes.data_as(L._pi64)
        b.rd_cap = cap.ctypes.data_as(L._pi64)
        b.rd_times = td.data_ptr()
        b.rd_off = to.data_ptr()

    def _plugin_instances(self, i, wseed, world_seed, seed_mod):
        """Fresh instances of the registered plugins for global replica i of a
        randomized batch: seed u_i + 99 idx (randomize_other_sources, opt_model.py:795-804)."""
        k = i % seed_mod if seed_mod > 0 else i
        u = int(wseed[i]) if wseed is not None else int(world_seed) + k
        return [cls(**dict(kw, seed=(u + 99 * idx) & 0xFFFFFFFF))
                for idx, cls, kw, _sid, _dyn in self.plugins]

    def _plugin_source_times(self, inst):
        from .opt_model import source_times
        return source_times(inst, self.start_time, self.sink_ids, self._edges, self.end_time)

    VERIFY_ALL = 64   # dynamic-plugin check: every replica of a batch this small, else a sample

    def _verify_dynamic(self, args, kw, res):
        """A dynamic plugin is played from its own schedule: check that it is self-driven
        -- rerun replicas with their event log and feed a fresh copy of each dynamic plugin
        the whole event sequence in play order (opt_model.verify_dynamic_plugin), which
        raises when its schedule reacts to another source's event.  Every replica of a
        batch of <= 64 (one probe batch), else 64 replicas drawn with a seed fixed by the
        batch (one probe run each): a plugin that reacts only in some replicas is caught
        whenever one of them is probed.  Cost: one event-logged run of the probed replicas
        plus a host replay of their events through the plugin (~10-50 ms per replica)."""
        from .opt_model import verify_dynamic_plugin
        gids = np.asarray(res.global_ids, dtype=np.int64)
        R = len(gids)
        if not R:
            return
        base = dict(kw)
        r0 = int(base.get("replica0", 0))
        base.update(event_log=True, check=True)
        if R <= self.VERIFY_ALL:
            probes = [(np.arange(R), self._run(*args, **dict(base, replica0=r0, n_local=R)))]
        else:
            rng = np.random.default_rng([0x52510000, R, int(gids[0])])
            pick = np.sort(rng.choice(R, self.VERIFY_ALL, replace=False))
            probes = [(np.asarray([j]), self._run(*args, **dict(base, replica0=r0 + int(j), n_local=1)))
                      for j in pick]
        ws = kw.get("world_seed", 0)
        wseed = ws.to(torch.int64).cpu().numpy() if torch.is_tensor(ws) else None
        me = kw.get("max_events")
        me = None if me is None or me == float("inf") else int(me)
        for idx, probe in probes:
            for k, j in enumerate(idx):
                t_ev, s_ev = probe.events(k)
                i = int(gids[j])
                if kw.get("randomize"):
                    make = lambda: self._plugin_instances(i, wseed, ws, int(kw.get("seed_mod", 0)))  # noqa: E731
                else:
                    make = lambda: [cls(**kw_) for _idx, cls, kw_, _sid, _dyn in self.plugins]  # noqa: E731
                for fresh, gen, p in zip(make(), make(), self.plugins):
                    if not p[4]:
                        continue
                    times = self._plugin_source_times(gen)
                    verify_dynamic_plugin(fresh, self.start_time, self.sink_ids, self._edges,
                                          self.end_time, t_ev, s_ev, times, max_events=me)

    def _run_reactive(self, args, kw, res):
        """A batch whose dynamic plugins react to other sources' events, played to the
        fixed point of run_dynamic's loop: every replica's plugin times are recomputed
        from its run's other events (opt_model.reactive_plugin_times, a fresh plugin
        instance per replica) and ONLY the replicas whose times moved are replayed with
        them (per-replica RealData streams, a replica list: rq_batch_desc.rep_idx), until
        no replica's times move; events before a plugin event whose time changed never
        change (every source sees only earlier events), so each rerun fixes at least one
        more plugin event of every replica still moving.  Each replica's result is the
        probe in which its times reproduced themselves (no extra final run).  At most
        max(REACTIVE_MAX_ITERATIONS, 2 x the most plugin events of a replica + 16) reruns,
        else NotImplementedError.  Cost per rerun: one event-logged run of the moving
        replicas and a host pass over their events."""
        from .opt_model import REACTIVE_MAX_ITERATIONS, reactive_plugin_times
        gids = np.asarray(res.global_ids, dtype=np.int64)
        ws = kw.get("world_seed", 0)
        wseed = ws.to(torch.int64).cpu().numpy() if torch.is_tensor(ws) else None
        rand = bool(kw.get("randomize"))
        sm = int(kw.get("seed_mod", 0))
        me = kw.get("max_events")
        me = None if me is None or me == float("inf") else int(me)
        ctrl = args[0] if args else kw.get("ctrl", "opt")
        static_ids = set(self.static_src_ids)
        if ctrl in ("poisson", "pwconst", "times"):
            static_ids.add(self.src_id)   # a static controlled source (Poisson2 / PWConst / RealData)

        def make(i):
            if rand:
                return self._plugin_instances(i, wseed, ws, sm)
            return [cls(**kw_) for _idx, cls, kw_, _sid, _dyn in self.plugins]
        times = {int(i): [self._plugin_source_times(inst) for inst in make(int(i))] for i in gids}
        probe_kw = dict(kw, event_log=True, check=True)
        dev = torch.device("cuda", torch.cuda.current_device())
        out = None
        moving = np.arange(len(gids))
        n_max = max((len(t) for ts in times.values() for t in ts), default=0)
        cap_it = max(REACTIVE_MAX_ITERATIONS, 2 * n_max + 16)
        self.reactive_replayed = 0
        for it in range(cap_it + 1):
            pk = dict(probe_kw, rd_override=times)
            if out is not None:   # only the replicas still moving
                pk["rep_idx"] = gids[moving]
            probe = self._run(*args, **pk)
            if out is None:
                out = probe
            else:
                _scatter(out, moving, probe, dev, True)
            self.reactive_replayed += len(moving)
            nxt = []
            for kl, k in enumerate(moving):
                i = int(gids[k])
                t_ev, s_ev = probe.events(kl)
                insts, cur = make(i), times[i]
                new = list(cur)
                for c, p in enumerate(self.plugins):
                    if p[4]:
                        new[c] = reactive_plugin_times(insts[c], self.start_time, self.sink_ids,
                                                       self._edges, self.end_time, t_ev, s_ev,
                                                       max_events=me, static_ids=static_ids)
                if any(not np.array_equal(a_, b_) for a_, b_ in zip(new, cur)):
                    times[i] = new
                    nxt.append(k)
            if not nxt:
                break
            if it == cap_it:
                raise NotImplementedError("reactive dynamic broadcasters: no fixed point after %d "
                                          "reruns" % cap_it)
            moving = np.asarray(nxt, dtype=np.int64)
        self.reactive_reruns = it
        if not kw.get("event_log"):
            out.ev_t = out.ev_src = None
        out.global_ids = gids
        out.replica0 = int(gids[0]) if len(gids) else 0
        return out

    def _plan_variant(self, lib, b):
        info = (C.c_int64 * 8)()
        L.check("rq_plan_info", lib.rq_plan_info(self._h, C.byref(b), info))
        return int(info[0])


class BatchResult:
    """Per-replica outputs (torch tensors on the device), replica i = g * n_rep + r."""

    def __init__(self, graph, metrics, counts, status, ev_t, ev_src, Ks, n_grid, n_rep):
        self.graph = graph
        self.metrics, self.counts, self.status = metrics, counts, status
        self.ev_t, self.ev_src = ev_t, ev_src
        self.Ks = list(int(k) for k in Ks)
        self.n_grid, self.n_rep = n_grid, n_rep

    def top_k(self, k):
        return self.metrics[:, self.Ks.index(k)]

    @property
    def avg_rank(self):
        return self.metrics[:, len(self.Ks)]

    @property
    def r_2(self):
        return self.metrics[:, len(self.Ks) + 1]

    @property
    def num_events(self):
        return self.counts[:, 0]

    @property
    def world_events(self):
        return self.counts[:, 1]

    @property
    def n_events(self):
        return self.counts[:, 2]

    def log_columns(self, stream=None):
        """The reference dataframe rows of every replica's event log, expanded on the
        GPU (rq_log_rows + rq_log_expand; State.get_dataframe, opt_model.py:85-97).
        Returns (row_off [R+1] host int64, {event_id, time_delta, src_id, t, sink_id}
        device tensors); replica i owns rows [row_off[i], row_off[i+1])."""
        if self.ev_t is None:
            raise ValueError("run with event_log=True to export the event log")
        use = stream or torch.cuda.current_stream()
        with torch.cuda.stream(use):
            return self._log_columns(use)

    def _log_columns(self, use):
        dev = self.ev_t.device
        R, cap = self.ev_t.shape
        st = use.cuda_stream
        row_off = torch.empty(R + 1, dtype=torch.int64, device=dev)
        lib = L.lib()
        L.check("rq_log_rows", lib.rq_log_rows(self.graph._h, self.ev_src.data_ptr(),
                                               self.counts.data_ptr(), R, cap,
                                               row_off.data_ptr(), st))
        ro = row_off.cpu().numpy()
        n = int(ro[-1])
        cols = {"event_id": torch.empty(n, dtype=torch.int64, device=dev),
                "time_delta": torch.empty(n, dtype=torch.float64, device=dev),
                "src_id": torch.empty(n, dtype=torch.int64, device=dev),
                "t": torch.empty(n, dtype=torch.float64, device=dev),
                "sink_id": torch.empty(n, dtype=torch.int64, device=dev)}
        if n:
            L.check("rq_log_expand", lib.rq_log_expand(
                self.graph._h, self.ev_t.data_ptr(), self.ev_src.data_ptr(),
                self.counts.data_ptr(), R, cap, row_off.data_ptr(),
                *(cols[k].data_ptr() for k in ("event_id", "time_delta", "src_id", "t", "sink_id")),
                st))
        return ro, cols

    def dataframe(self, i=None):
        """State.get_dataframe() of replica i, or of all replicas with a leading
        'replica' column (i=None); rows expanded on the GPU."""
        import pandas as pd
        ro, cols = self.log_columns()
        host = {k: v.cpu().numpy() for k, v in cols.items()}
        if i is not None:
            a, b = int(ro[i]), int(ro[i + 1])
            return pd.DataFrame({k: host[k][a:b] for k in
                                 ("event_id", "time_delta", "src_id", "t", "sink_id")})
        gids = getattr(self, "global_ids", None)
        if gids is None:
            gids = np.arange(len(ro) - 1, dtype=np.int64) + getattr(self, "replica0", 0)
        rep = np.repeat(np.asarray(gids, dtype=np.int64), np.diff(ro))
        return pd.DataFrame(dict(replica=rep, **host))

    def events(self, i):
        """(t, src_id) numpy arrays of replica i (needs event_log=True)."""
        n = int(self.counts[i, 2].item())
        t = self.ev_t[i, :n].cpu().numpy()
        s = self.graph.stream_src_ids[self.ev_src[i, :n].cpu().numpy()]
        return t, s


def expected_events(graph_kw):
    """Rough expected event count of a world (for sizing benchmarks)."""
    span = graph_kw["end_time"] - graph_kw.get("start_time", 0.0)
    tot = 0.0
    for name, kw in graph_kw["other_sources"]:
        if name in ("Poisson", "Poisson2"):
            tot += kw.get("rate", 1.0) * span
        elif name == "Hawkes":
            br = kw.get("alpha", 1.0) / kw.get("beta", 10.0)
            tot += kw.get("l_0", 1.0) * span / max(1e-9, 1 - br)
    return tot if math.isfinite(tot) else 0.0


def _scatter(res, pick, r, dev, event_log):
    """Rows of BatchResult ``r`` into outputs ``pick`` of ``res`` (event logs widened to
    the larger capacity when ``event_log``)."""
    at = torch.from_numpy(np.asarray(pick, dtype=np.int64)).to(dev)
    res.metrics.index_copy_(0, at, r.metrics)
    res.counts.index_copy_(0, at, r.counts)
    res.status.index_copy_(0, at, r.status)
    if event_log:
        cap, cap2 = res.ev_t.shape[1], r.ev_t.shape[1]
        if cap2 > cap:   # a larger event capacity: widen every replica's log row
            t2 = torch.empty((res.ev_t.shape[0], cap2), dtype=res.ev_t.dtype, device=dev)
            s2 = torch.empty((res.ev_src.shape[0], cap2), dtype=res.ev_src.dtype, device=dev)
            t2[:, :cap] = res.ev_t
            s2[:, :cap] = res.ev_src
            res.ev_t, res.ev_src = t2, s2
        res.ev_t[at, :cap2] = r.ev_t
        res.ev_src[at, :cap2] = r.ev_src
