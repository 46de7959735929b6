"""ctypes binding of librq.so (include/rq.h).

The product path has exactly one implementation: the gfx950 kernels in
librq.so.  If the shared object is missing this module raises at import --
there is no CPU fallback.
"""
import ctypes as C
import os
import warnings

import torch  # noqa: F401  -- load torch's HIP runtime first so librq.so binds to it

# HIP hardware queues per process.  rq_run_batch pipelines a batch's chunks on two
# streams and an RCCL group adds its own; at HIP's default of 4 queues the engine's two
# streams then share one queue and the pipeline serialises (C3: 2.93 -> 3.42 ms per step
# with a world-size-1 group, profiles/r05_dist_queues.txt).  HIP reads the count when it
# initialises, so the package raises it to HW_QUEUES_MIN at import when the caller has
# not set it and HIP is not up yet; otherwise dist.run_sharded warns once (hw_queue_advice).
HW_QUEUES_MIN = 8
HW_QUEUES_SET_BY_PACKAGE = False
if "GPU_MAX_HW_QUEUES" not in os.environ and not torch.cuda.is_initialized():
    os.environ["GPU_MAX_HW_QUEUES"] = str(HW_QUEUES_MIN)
    HW_QUEUES_SET_BY_PACKAGE = True
# the count this process's HIP runtime uses: None = unknown (HIP was up before the import
# and the variable unset, i.e. HIP's default of 4)
HW_QUEUES = int(os.environ["GPU_MAX_HW_QUEUES"]) if "GPU_MAX_HW_QUEUES" in os.environ else None


def hw_queue_advice(group_live, queues=-1):
    """The warning an engine run under a live process group deserves when its HIP
    runtime has fewer than HW_QUEUES_MIN hardware queues (None: no warning).  queues:
    the count to judge (None: unset, HIP's default); -1: this process's (HW_QUEUES)."""
    q = HW_QUEUES if queues == -1 else queues
    if not group_live or (q is not None and q >= HW_QUEUES_MIN):
        return None
    return ("redqueen_amd: GPU_MAX_HW_QUEUES=%s with a process group open: the RCCL streams and "
            "the engine's two pipeline streams share HIP's hardware queues and the pipeline "
            "serialises (C3: ~17%% slower per step).  Set GPU_MAX_HW_QUEUES=%d before HIP "
            "initialises (before the first torch.cuda call)."
            % ("unset (4)" if q is None else q, HW_QUEUES_MIN))


_warned_queues = False


def warn_hw_queues(group_live):
    global _warned_queues
    msg = hw_queue_advice(group_live)
    if msg and not _warned_queues:
        _warned_queues = True
        warnings.warn(msg, RuntimeWarning, stacklevel=3)
    return msg

_HERE = os.path.dirname(os.path.abspath(__file__))
SO_PATH = os.environ.get("RQ_SO_PATH") or os.path.join(_HERE, "librq.so")   # env: A/B builds only

RQ_OK, RQ_EINVAL, RQ_EOVERFLOW, RQ_EHIP, RQ_ENOMEM, RQ_EUNSORTED, RQ_EUNSUPPORTED = (
    0, -1, -2, -3, -4, -5, -6)
SRC_NONE, SRC_POISSON, SRC_POISSON2, SRC_HAWKES, SRC_PWCONST, SRC_REALDATA, SRC_OPT, SRC_OPTPW = range(8)
ST_ROWS_OVERFLOW, ST_STREAM_OVERFLOW, ST_TIE, ST_EMPTY, ST_UNORDERED = 1, 2, 4, 8, 16
RUN_EVENT_LOG = 1
ABI_VERSION = 6
SRCF_DYNAMIC = 1   # rq_source_desc.flags: a RealData source that is a dynamic broadcaster's times
REPLAY_LARGE = 1
REPLAY_CHUNKED = 2
REPLAY_CHUNK_ROWS = 4096   # RC_L: rows per workgroup of the chunked replay
MAX_K = 4
MAX_RD = 64

_P = C.c_void_p
_pd = C.POINTER(C.c_double)
_pi64 = C.POINTER(C.c_int64)
_pi32 = C.POINTER(C.c_int32)
_pu32 = C.POINTER(C.c_uint32)


class SourceDesc(C.Structure):
    _fields_ = [("kind", C.c_int32), ("n_arr", C.c_int32), ("src_id", C.c_int64),
                ("seed", C.c_uint32), ("flags", C.c_uint32), ("p0", C.c_double),
                ("p1", C.c_double), ("p2", C.c_double), ("a", _pd), ("b", _pd)]


class GraphDesc(C.Structure):
    _fields_ = [("n_sources", C.c_int32), ("sources", C.POINTER(SourceDesc)),
                ("n_sinks", C.c_int32), ("sink_ids", _pi64), ("n_edges", C.c_int64),
                ("edge_src", _pi64), ("edge_sink", _pi64), ("ctrl_src_id", C.c_int64),
                ("start_time", C.c_double), ("end_time", C.c_double), ("ctrl_n_arr", C.c_int32),
                ("ctrl_a", _pd), ("ctrl_b", _pd)]


class BatchDesc(C.Structure):
    _fields_ = [("ctrl_kind", C.c_int32), ("n_grid", C.c_int32), ("q", _pd), ("s", _pd),
                ("n_rep", C.c_int64), ("ctrl_seed", _P), ("ctrl_seed0", C.c_uint32),
                ("randomize_world", C.c_int32), ("world_seed", _P), ("world_seed0", C.c_uint32),
                ("seed_mod", C.c_int64), ("ctrl_rate", _P), ("ctrl_rate_max", C.c_double),
                ("Ks", _pi32), ("nK", C.c_int32), ("max_events", C.c_int64),
                ("flags", C.c_int32), ("cap_scale", C.c_double), ("chunk", C.c_int64),
                ("replica0", C.c_int64), ("n_local", C.c_int64), ("sweep_mode", C.c_int32),
                ("n_seg", C.c_int32), ("period", C.c_double), ("s_pw", _pd),
                ("n_rd", C.c_int32), ("rd_src_id", _pi64), ("rd_cap", _pi64), ("rd_times", _P),
                ("rd_off", _P), ("rep_lo", C.c_int64), ("rep_cnt", C.c_int64),
                ("ws_budget", C.c_int64), ("rep_idx", _pi64)]


class Outputs(C.Structure):
    _fields_ = [("metrics", _P), ("counts", _P), ("status", _P), ("ev_t", _P),
                ("ev_src", _P), ("ev_cap", C.c_int64)]


class RQError(RuntimeError):
    def __init__(self, fn, code):
        self.code = code
        super().__init__("%s failed: %s (%d)" % (fn, strerror(code), code))


_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(SO_PATH):
        raise ImportError("redqueen_amd: %s is missing -- build it with "
                          "`python -c 'import __graft_entry__ as g; g.build()'` "
                          "(there is no CPU fallback)" % SO_PATH)
    L = C.CDLL(SO_PATH)
    L.rq_abi_version.restype = C.c_int
    L.rq_strerror.restype = C.c_char_p
    L.rq_strerror.argtypes = [C.c_int]
    L.rq_graph_build.argtypes = [C.POINTER(GraphDesc), C.POINTER(_P)]
    L.rq_graph_free.argtypes = [_P]
    L.rq_graph_info.argtypes = [_P, _pi64]
    L.rq_graph_source_ids.argtypes = [_P, _pi64]
    L.rq_graph_followers.argtypes = [_P, _pi64]
    L.rq_workspace_size.argtypes = [_P, C.POINTER(BatchDesc), C.POINTER(C.c_size_t)]
    L.rq_event_capacity.argtypes = [_P, C.POINTER(BatchDesc), _pi64]
    L.rq_plan_info.argtypes = [_P, C.POINTER(BatchDesc), _pi64]
    L.rq_run_batch.argtypes = [_P, C.POINTER(BatchDesc), C.POINTER(Outputs), _P, C.c_size_t, _P]
    L.rq_replay_workspace_size.argtypes = [C.c_int64, C.c_int64, C.c_int32, C.c_int32,
                                           C.POINTER(C.c_size_t)]
    L.rq_metrics_replay.argtypes = [_P, _P, _P, _P, C.c_int64, C.c_int64, C.c_double,
                                    _pi32, C.c_int32, _P, _P, _P, C.c_size_t, _P]
    L.rq_metrics_replay_batch.argtypes = [_P, _P, _P, _P, _P, C.c_int64, C.c_int64, C.c_int64,
                                          C.c_double, _pi32, C.c_int32, _P, _P, _P, C.c_size_t, _P]
    L.rq_oracle_workspace_size.argtypes = [C.c_int32, C.c_int64, C.POINTER(C.c_size_t)]
    L.rq_oracle_dp.argtypes = [_P, _P, _P, _P, C.c_int32, C.c_int64, _P, _P, _P, _P, _P,
                               C.c_size_t, _P]
    L.rq_rank_table.argtypes = [_P, _P, _P, C.c_int64, C.c_int32, C.c_int64, C.c_int32,
                                C.c_int64, _P, _P, _P, _P]
    L.rq_u_int.argtypes = [_P, _P, C.c_int64, C.c_int32, _P, _P, C.c_int32, C.c_double, _P, _P,
                           C.c_size_t, _P]
    L.rq_log_rows.argtypes = [_P, _P, _P, C.c_int64, C.c_int64, _P, _P]
    L.rq_log_expand.argtypes = [_P, _P, _P, _P, C.c_int64, C.c_int64, _P, _P, _P, _P, _P, _P, _P]
    L.rq_timing.argtypes = [C.c_int]
    L.rq_timing_read.argtypes = [_pd, _pi64]
    for fn in ("rq_timing", "rq_timing_read", "rq_graph_build", "rq_graph_free", "rq_graph_info", "rq_graph_source_ids",
               "rq_graph_followers", "rq_workspace_size", "rq_event_capacity", "rq_run_batch",
               "rq_replay_workspace_size", "rq_metrics_replay", "rq_metrics_replay_batch",
               "rq_oracle_workspace_size",
               "rq_oracle_dp", "rq_rank_table", "rq_u_int", "rq_log_rows", "rq_log_expand"):
        getattr(L, fn).restype = C.c_int
    if L.rq_abi_version() != ABI_VERSION:
        raise ImportError("librq.so ABI version mismatch")
    _lib = L
    return L


def build_stamp():
    """Identity of the loaded engine build: sha256 of librq.so and of its sources
    (csrc/ + include/rq.h).  Profiling summaries carry it, so a number measured on
    another build is recognised as such (bench.py drops it)."""
    import glob
    import hashlib
    h = hashlib.sha256()
    with open(SO_PATH, "rb") as f:
        h.update(f.read())
    src = hashlib.sha256()
    root = os.path.dirname(_HERE)
    # the files librq.so is built from (csrc/asan.mk, the host-sanitizer build, is not
    # one of them and does not travel to the GPU box)
    for fn in sorted(glob.glob(os.path.join(_HERE, "csrc", "*")) +
                     [os.path.join(root, "include", "rq.h")]):
        if os.path.isfile(fn) and (fn.endswith((".hip", ".h", ".cpp")) or
                                   os.path.basename(fn) == "Makefile"):
            with open(fn, "rb") as f:
                src.update(os.path.basename(fn).encode() + b"\0" + f.read())
    return {"librq_sha256": h.hexdigest()[:16], "csrc_sha256": src.hexdigest()[:16]}


def strerror(code):
    try:
        return lib().rq_strerror(code).decode()
    except Exception:  # pragma: no cover
        return "error"


def check(fn, code):
    if code != RQ_OK:
        raise RQError(fn, code)


EXPORTED = ["rq_abi_version", "rq_strerror", "rq_graph_build", "rq_graph_free", "rq_graph_info",
            "rq_graph_source_ids", "rq_graph_followers", "rq_workspace_size",
            "rq_event_capacity", "rq_plan_info", "rq_run_batch", "rq_replay_workspace_size",
            "rq_metrics_replay", "rq_metrics_replay_batch", "rq_oracle_workspace_size", "rq_oracle_dp", "rq_rank_table",
            "rq_u_int", "rq_log_rows", "rq_log_expand", "rq_timing", "rq_timing_read"]
