"""librq.so loads here (no GPU) and exports every symbol include/rq.h declares;
argument validation happens before any HIP call (so it is testable on CPU)."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from redqueen_amd import _lib as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "rq.h")).read()
    return sorted(set(re.findall(r"^(?:int|const char\*)\s+(rq_\w+)\(", src, re.M)))


def test_exports_every_declared_symbol():
    names = header_functions()
    assert len(names) >= 14
    lib = L.lib()
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(L.EXPORTED)


def test_status_bits_match_the_header():
    """The RQ_ST_* status bits the Python side tests equal include/rq.h's."""
    src = open(os.path.join(ROOT, "include", "rq.h")).read()
    bits = {m.group(1): int(m.group(2)) for m in re.finditer(r"#define RQ_ST_(\w+)\s+(\d+)", src)}
    assert bits == {"ROWS_OVERFLOW": L.ST_ROWS_OVERFLOW, "STREAM_OVERFLOW": L.ST_STREAM_OVERFLOW,
                    "TIE": L.ST_TIE, "EMPTY": L.ST_EMPTY, "UNORDERED": L.ST_UNORDERED}, bits


def test_version_and_errors():
    lib = L.lib()
    assert lib.rq_abi_version() == L.ABI_VERSION == 6
    assert lib.rq_strerror(L.RQ_EINVAL) == b"invalid argument"
    assert lib.rq_strerror(-99) == b"unknown error"


def _desc(sink_ids, edges, sources, ctrl=1, end=10.0):
    keep = []
    arr = (L.SourceDesc * max(1, len(sources)))()
    for i, (kind, sid, extra) in enumerate(sources):
        arr[i].kind, arr[i].src_id, arr[i].p0 = kind, sid, 1.0
        if extra is not None:
            a = np.ascontiguousarray(extra[0], dtype=np.float64)
            b = np.ascontiguousarray(extra[1], dtype=np.float64)
            keep += [a, b]
            arr[i].n_arr = a.size
            arr[i].a, arr[i].b = a.ctypes.data_as(L._pd), b.ctypes.data_as(L._pd)
    sk = np.ascontiguousarray(sink_ids, dtype=np.int64)
    es = np.ascontiguousarray([e[0] for e in edges], dtype=np.int64)
    ed = np.ascontiguousarray([e[1] for e in edges], dtype=np.int64)
    keep += [sk, es, ed, arr]
    d = L.GraphDesc()
    d.n_sources, d.sources = len(sources), arr
    d.n_sinks, d.sink_ids = sk.size, sk.ctypes.data_as(L._pi64)
    d.n_edges = len(edges)
    d.edge_src, d.edge_sink = es.ctypes.data_as(L._pi64), ed.ctypes.data_as(L._pi64)
    d.ctrl_src_id, d.start_time, d.end_time = ctrl, 0.0, end
    return d, keep


def _build(*a, **k):
    d, keep = _desc(*a, **k)
    h = C.c_void_p()
    return L.lib().rq_graph_build(C.byref(d), C.byref(h))


P2 = L.SRC_POISSON2


@pytest.mark.parametrize("case,expect", [
    (([1, 1], [(2, 1)], [(P2, 2, None)]), L.RQ_EINVAL),                 # Duplicates in sink_ids.
    (([1, 2], [(3, 1)], [(P2, 2, None)]), L.RQ_EINVAL),                 # Unknown sources in edge_list.
    (([1, 2], [(2, 9)], [(P2, 2, None)]), L.RQ_EINVAL),                 # Unknown sinks in edge_list.
    (([1, 2], [(2, 1)], [(P2, 2, None), (P2, 2, None)]), L.RQ_EINVAL),  # Duplicates in sources.
    (([1, 2], [(2, 1)], [(P2, 1, None)]), L.RQ_EINVAL),                 # clashes with src_id
    (([], [], [(P2, 2, None)]), L.RQ_EINVAL),                           # No sinks.
    (([1, 2], [(2, 1)], [(L.SRC_PWCONST, 2, ([0.0, 5.0, 2.0], [1, 2, 3]))]), L.RQ_EINVAL),
    (([1, 2], [(2, 1)], [(L.SRC_PWCONST, 2, ([1.0, 5.0], [1, 2]))]), L.RQ_EINVAL),
    (([1, 2], [(2, 1), (2, 1)], [(P2, 2, None)]), "accepted"),          # duplicate edge (a multigraph)
    (([1, 2], [(1, 1), (1, 1), (2, 1)], [(P2, 2, None)]), "accepted"),  # duplicate controlled edge
    ((list(range(1, 50001)), [(2, 1), (2, 50000)], [(P2, 2, None)]), "accepted"),   # 50k sinks
    (([1, 2], [(s, 1) for s in range(2, 602)], [(P2, s, None) for s in range(2, 602)]), "accepted"),
    (([1, 2], [(2, 1)], [(L.SRC_OPT, 2, None)]), L.RQ_EUNSUPPORTED),    # Opt as a wall source
])
def test_graph_build_validation(case, expect):
    """The reference's Manager.__init__ rules (opt_model.py:158-175); every graph it
    accepts passes validation -- duplicate edges, any sink or source count.  Without a
    GPU an accepted graph stops at its device upload (RQ_ENOMEM / RQ_EHIP)."""
    rc = _build(*case)
    if expect == "accepted":
        assert rc not in (L.RQ_EINVAL, L.RQ_EUNSUPPORTED), rc
    else:
        assert rc == expect


def test_source_flags_validation():
    """rq_source_desc.flags (ABI v6): RQ_SRCF_DYNAMIC only on a RealData source (a dynamic
    broadcaster's replayed times); any other bit is refused."""
    def build(kind, flags):
        d, keep = _desc([1, 2], [(2, 1)], [(kind, 2, None)])
        d.sources[0].flags = flags
        if kind == L.SRC_REALDATA:
            t = np.asarray([0.5, 1.5])
            keep.append(t)
            d.sources[0].n_arr, d.sources[0].a = 2, t.ctypes.data_as(L._pd)
        h = C.c_void_p()
        return L.lib().rq_graph_build(C.byref(d), C.byref(h))
    assert build(L.SRC_POISSON2, L.SRCF_DYNAMIC) == L.RQ_EINVAL
    assert build(L.SRC_HAWKES, L.SRCF_DYNAMIC) == L.RQ_EINVAL
    assert build(L.SRC_REALDATA, 2) == L.RQ_EINVAL
    assert build(L.SRC_REALDATA, L.SRCF_DYNAMIC) not in (L.RQ_EINVAL, L.RQ_EUNSUPPORTED)
    src = open(os.path.join(ROOT, "include", "rq.h")).read()
    assert re.search(r"#define RQ_SRCF_DYNAMIC\s+%d\b" % L.SRCF_DYNAMIC, src)
    assert "const int64_t* rep_idx;" in src   # the replica list closes rq_batch_desc
    assert [f[0] for f in L.BatchDesc._fields_][-1] == "rep_idx"


def test_workspace_queries_validate():
    lib = L.lib()
    n = C.c_size_t()
    assert lib.rq_workspace_size(None, None, C.byref(n)) == L.RQ_EINVAL
    assert lib.rq_replay_workspace_size(100, 1, 1, 0, C.byref(n)) == 0 and n.value >= 100 * 32
    small = n.value
    assert lib.rq_replay_workspace_size(100, 1, 1, L.REPLAY_LARGE, C.byref(n)) == 0
    assert n.value >= small + 100 * 96
    assert lib.rq_replay_workspace_size(-1, 1, 1, 0, C.byref(n)) == L.RQ_EINVAL
    assert lib.rq_replay_workspace_size(10, 0, 1, 0, C.byref(n)) == L.RQ_EINVAL
    assert lib.rq_replay_workspace_size(10, 1, 5, 0, C.byref(n)) == L.RQ_EINVAL
    k = np.asarray([1], dtype=np.int32)
    # argument validation happens before any HIP call
    assert lib.rq_metrics_replay(None, None, None, None, 10, 1, 1.0, k.ctypes.data_as(L._pi32),
                                 1, None, None, None, 0, None) == L.RQ_EINVAL
    assert lib.rq_metrics_replay_batch(None, None, None, None, None, 2, 10, 1, 1.0,
                                       k.ctypes.data_as(L._pi32), 1, None, None, None, 0,
                                       None) == L.RQ_EINVAL
    k0 = np.asarray([0], dtype=np.int32)   # K >= 1 (time_in_top_k compares r <= K - 1)
    buf = (C.c_char * 4096)()
    assert lib.rq_metrics_replay(None, None, None, None, 0, 1, 1.0, k0.ctypes.data_as(L._pi32),
                                 1, buf, buf, buf, 4096, None) == L.RQ_EINVAL
