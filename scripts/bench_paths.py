"""Secondary measurements (not the bench line): the HBM-facing kernels of the path.

  * sweep with the event log on (RQ_RUN_EVENT_LOG, the fast merged sweep since round 6;
    10k replicas): writes 12 B per event (t f64 + source i32) + 24 B per pivot row and
    reads 10 B per merged wall entry
  * rq_log_rows + rq_log_expand: State.get_dataframe rows for a whole batch,
    12 B read per event + 40 B written per (event, sink) row
  * rq_scan: 24 B read per pivot row (timed inside the plain C3 run)
  * rq_metrics_replay_batch on the 256 exported C3 dataframes (24 B read per df row,
    32 B with event ids) and rq_metrics_replay on one df through the pandas facade
  * rq_oracle_dp: n = 8000 walls, 64 instances
  * the exact sequential sweep (the fallback for multigraphs and repeated RealData
    times): the C3 network with duplicated edges, a 600-source world, C3 with a
    max_events cap forced onto it (seq_max_events_c3) -- replicas/s and events/s
  * the fast paths round 6 opened: C3 with max_events = 4000 (fast_max_events_c3: the
    tile cut), C3 with a per-replica RealData stream handed over as device arrays
    (fast_realdata_c3: rq_batch_desc.rd_*)
Per-kernel times come from the library's HIP events (rq_timing) on the launch stream.
--only a,b runs just those sections, so a rocprofv3 PMC pass can hold ONE workload
(scripts/gpu_paths_pmc.sh).
usage: python scripts/bench_paths.py [--reps N] [--only SECTIONS]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from redqueen_amd import _lib as L  # noqa: E402
from redqueen_amd import engine, graphs, utils  # noqa: E402

PEAK = 8000.0
SECTIONS = ["sweep_event_log", "log_expand", "scan", "replay_batch", "replay_batch_eid", "replay_batch_1024",
            "replay_batch_eid_chunked", "replay_one_df", "replay_one_df_one_workgroup",
            "replay_one_df_facade", "oracle_dp", "seq_multigraph_c3", "seq_600_sources",
            "seq_max_events_c3", "fast_max_events_c3", "fast_realdata_c3", "fast_600_sources",
            "fast_3000_sources"]
REPLAY = {"log_expand", "replay_batch", "replay_batch_eid", "replay_batch_1024", "replay_batch_eid_chunked",
          "replay_one_df", "replay_one_df_one_workgroup", "replay_one_df_facade"}


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    ms = np.zeros(5)
    nl = np.zeros(5, dtype=np.int64)
    L.lib().rq_timing(1)
    t0 = time.perf_counter()
    for _ in range(reps):
        out = fn()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / reps
    L.lib().rq_timing_read(ms.ctypes.data_as(L._pd), nl.ctypes.data_as(L._pi64))
    L.lib().rq_timing(0)
    return out, ms / reps, wall


def graph_of(so):
    return engine.Graph(so["src_id"], so["other_sources"], so["sink_ids"], so["edge_list"],
                        so["end_time"])


def sweep_event_log(g, so, a, res):
    R = 10000
    run = lambda: g.run("opt", q=so["q"], s=so["s"], n_rep=R, ctrl_seed=0, world_seed=0,  # noqa: E731
                        randomize=True, event_log=True, check=False)
    r, ms, wall = timed(run, a.reps)
    ev = int(r.counts[:, 2].sum())
    rows = int(r.counts[:, 3].sum())
    walls = int(r.counts[:, 2].sum() - r.counts[:, 0].sum())
    b = 12 * ev + 24 * rows + 10 * walls
    plan = g.run("opt", q=so["q"], s=so["s"], n_rep=R, event_log=True, randomize=True, plan_only=True)
    res["sweep_event_log"] = {"replicas": R, "events": ev, "rows": rows, "ms": ms[1],
                              "launches_per_run": 2, "bytes": b,
                              "bytes_note": "12 B/event logged + 24 B/pivot row + 10 B/merged wall entry read",
                              "GBps": b / ms[1] / 1e6, "frac": b / ms[1] / 1e6 / PEAK, "plan": plan}


def scan(g, so, a, res):
    # one stream, one chunk: the scan's HIP-event time is its own (pipelined chunks
    # overlap other kernels and their launch times with them)
    os.environ["RQ_PIPE"] = "1"
    R3 = 10000
    run3 = lambda: g.run("opt", q=so["q"], s=so["s"], n_rep=R3, ctrl_seed=0, world_seed=0,  # noqa: E731
                         randomize=True, check=False)
    r3, ms, wall = timed(run3, a.reps)
    rows3 = int(r3.counts[:, 3].sum())
    del os.environ["RQ_PIPE"]
    res["scan"] = {"replicas": R3, "rows": rows3, "ms": ms[2], "bytes": 24 * rows3,
                   "GBps": 24 * rows3 / ms[2] / 1e6, "frac": 24 * rows3 / ms[2] / 1e6 / PEAK}


def replay(g, so, a, res, want):
    # batch dataframe expansion: 256 replicas (one block each, enough to fill the
    # 256 CUs; ~7 GB of columns)
    R2 = 256
    r2 = g.run("opt", q=so["q"], s=so["s"], n_rep=R2, ctrl_seed=0, world_seed=0, randomize=True,
               event_log=True)
    if want("log_expand"):
        (ro, cols), ms, wall = timed(lambda: r2.log_columns(), a.reps)
    else:
        ro, cols = r2.log_columns()
    nrow = int(ro[-1])
    ev2 = int(r2.counts[:, 2].sum())
    if want("log_expand"):
        b = 40 * nrow + 12 * ev2 * 2   # rows written; events read by both passes
        res["log_expand"] = {"replicas": R2, "rows": nrow, "ms": ms[3], "bytes": b,
                             "GBps": b / ms[3] / 1e6, "frac": b / ms[3] / 1e6 / PEAK}
    # rq_metrics_replay_batch (raw sink ids): the 256 exported C3 dataframes as one batch
    # (24 B read per df row: t, src_id, sink_id; +8 B with event ids)
    off = torch.from_numpy(ro).cuda()
    for tag, eid in (("replay_batch", None), ("replay_batch_eid", cols["event_id"])):
        if not want(tag):
            continue
        (m4, c4), ms, wall = timed(lambda: utils.replay_columns(
            cols["t"], cols["src_id"], cols["sink_id"], eid, off, so["src_id"], so["end_time"],
            (1,)), a.reps)
        per_row = 24 + (8 if eid is not None else 0)
        res[tag] = {"dataframes": R2, "rows": nrow, "ms_fast": ms[3], "ms_scan": ms[2],
                    "wall_ms": wall * 1e3, "bytes": per_row * nrow,
                    "GBps": per_row * nrow / (ms[3] + ms[2]) / 1e6,
                    "frac": per_row * nrow / (ms[3] + ms[2]) / 1e6 / PEAK,
                    "equal_to_sweep": bool(torch.equal(m4, r2.metrics))}
    if want("replay_batch_1024"):   # 1024 dataframes: four per CU
        r3 = g.run("opt", q=so["q"], s=so["s"], n_rep=1024, ctrl_seed=0, world_seed=0,
                   randomize=True, event_log=True)
        ro3, cols3 = r3.log_columns()
        off3 = torch.from_numpy(ro3).cuda()
        n3 = int(ro3[-1])
        (m6, c6), ms, wall = timed(lambda: utils.replay_columns(
            cols3["t"], cols3["src_id"], cols3["sink_id"], None, off3, so["src_id"], so["end_time"],
            (1,)), a.reps)
        res["replay_batch_1024"] = {"dataframes": 1024, "rows": n3, "ms_fast": ms[3], "ms_scan": ms[2],
                                    "wall_ms": wall * 1e3, "bytes": 24 * n3,
                                    "GBps": 24 * n3 / (ms[3] + ms[2]) / 1e6,
                                    "frac": 24 * n3 / (ms[3] + ms[2]) / 1e6 / PEAK,
                                    "equal_to_sweep": bool(torch.equal(m6, r3.metrics))}
        del r3, cols3, off3
    if want("replay_batch_eid_chunked"):   # the same batch through the chunked path, forced (A/B)
        os.environ["RQ_RP_CHUNK"] = "1"
        (m4, c4), ms, wall = timed(lambda: utils.replay_columns(
            cols["t"], cols["src_id"], cols["sink_id"], cols["event_id"], off, so["src_id"],
            so["end_time"], (1,), chunked=True), a.reps)
        del os.environ["RQ_RP_CHUNK"]
        res["replay_batch_eid_chunked"] = {"dataframes": R2, "rows": nrow, "ms_replay": ms[3],
                                           "ms_scan": ms[2], "GBps": 32 * nrow / (ms[3] + ms[2]) / 1e6,
                                           "equal_to_sweep": bool(torch.equal(m4, r2.metrics))}
    # ONE dataframe (device columns): the chunked path (default for a long df) and the
    # one-workgroup path; and through the pandas facade (host -> device copies included)
    a0, a1 = int(ro[0]), int(ro[1])
    one = {k: v[a0:a1].contiguous() for k, v in cols.items()}
    for tag, ck in (("replay_one_df", None), ("replay_one_df_one_workgroup", False)):
        if not want(tag):
            continue
        if ck is False:
            os.environ["RQ_RP_CHUNK"] = "0"
        (m5, c5), ms, wall = timed(lambda: utils.replay_columns(
            one["t"], one["src_id"], one["sink_id"], one["event_id"], None, so["src_id"],
            so["end_time"], (1,), chunked=ck), a.reps)
        os.environ.pop("RQ_RP_CHUNK", None)
        res[tag] = {"rows": a1 - a0, "ms_replay": ms[3], "ms_scan": ms[2], "ms": ms[3] + ms[2],
                    "wall_ms": wall * 1e3, "GBps": 32 * (a1 - a0) / (ms[3] + ms[2]) / 1e6,
                    "equal_to_sweep": bool(torch.equal(m5[0], r2.metrics[0]))}
    if want("replay_one_df_facade"):
        df = r2.dataframe(0)
        _, ms, wall = timed(lambda: utils.replay_metrics(df, so["src_id"], so["end_time"], (1,)), a.reps)
        res["replay_one_df_facade"] = {"rows": len(df), "ms": ms[3] + ms[2], "wall_ms": wall * 1e3,
                                       "GBps": 32 * len(df) / (ms[3] + ms[2]) / 1e6}


def oracle(a, res):
    rs = np.random.RandomState(0)
    n = 8000
    ws = []
    for i in range(64):
        t = np.cumsum(rs.exponential(0.01, n))
        ws.append(np.diff(np.concatenate([[0.0, 0.0], t, [t[-1] + 1.0]])))
    qs, ss = list(rs.uniform(1, 100, 64)), [1.0] * 64
    _, ms, wall = timed(lambda: utils.oracle_dp_batch(ws, qs, ss), a.reps)
    cells = 64 * n * n / 2
    res["oracle_dp"] = {"instances": 64, "n": n, "ms": ms[3], "wall_ms": wall * 1e3,
                        "Gcells_per_s": cells / ms[3] / 1e6}


def seq_world(name):
    """The worlds the fast sweeps hand to the exact sequential sweep."""
    if name == "seq_multigraph_c3":
        # C3 with every 10th wall edge listed twice: duplicate (source, sink) rows make
        # pandas-mean pivot cells (opt_model.py:306-307, utils.py:54-55)
        so = graphs.c3()
        extra = [e for k, e in enumerate(so["edge_list"]) if e[0] != so["src_id"] and k % 10 == 0]
        return dict(so, edge_list=list(so["edge_list"]) + extra), None
    if name in ("seq_600_sources", "fast_600_sources"):
        # 600 broadcasters: the fast general sweep on the two-level merged sequence, or
        # (seq_: sweep_mode 2) the sequential sweep with 16 sources per lane
        return graphs.followers_graph(num_followers=1000, num_sources=600, degree=5,
                                      end_time=20.0, world_rate=1.0, alpha=1.0, beta=10.0), None
    if name == "fast_3000_sources":
        return graphs.followers_graph(num_followers=3000, num_sources=3000, degree=5,
                                      end_time=4.0, world_rate=1.0, alpha=1.0, beta=10.0), None
    if name in ("seq_max_events_c3", "fast_max_events_c3"):
        return graphs.c3(), 4000
    if name == "fast_realdata_c3":
        # C3 + one RealData broadcaster (src 9000, declared without times) into 40
        # followers; each replica plays its own ~100 times (rate 1 over T = 100)
        so = graphs.c3()
        fol = sorted({b for a_, b in so["edge_list"] if a_ != so["src_id"]})[::25]
        return dict(so, other_sources=so["other_sources"] + [("RealData", {"src_id": 9000, "times": []})],
                    edge_list=so["edge_list"] + [(9000, f) for f in fol]), None
    raise KeyError(name)


def seq(name, a, res, R=4096):
    so, max_ev = seq_world(name)
    g = graph_of(so)
    kw = dict(q=so["q"], s=so["s"], n_rep=R, ctrl_seed=0, world_seed=0, randomize=True,
              max_events=max_ev, Ks=(1,),
              sweep_mode=2 if name in ("seq_600_sources", "seq_max_events_c3") else 0)
    if name == "fast_realdata_c3":
        n = 100
        gen = torch.Generator(device="cuda").manual_seed(9)
        t = torch.sort(torch.rand((R, n), generator=gen, device="cuda", dtype=torch.float64) *
                       so["end_time"], dim=1).values.contiguous().reshape(-1)
        off = torch.arange(0, R * n + 1, n, dtype=torch.int64, device="cuda")
        kw["rd_streams"] = ([9000], t, off, [n])
    plan = g.run("opt", plan_only=True, **{k: v for k, v in kw.items() if k != "rd_streams"})
    r, ms, wall = timed(lambda: g.run("opt", check=False, **kw), a.reps)
    ev = int(r.counts[:, 2].sum())
    res[name] = {"replicas": R, "sources": len(so["other_sources"]), "sinks": len(so["sink_ids"]),
                 "edges": len(so["edge_list"]), "max_events": max_ev, "events": ev,
                 "events_per_replica": ev / R, "sweep_ms": ms[1], "step_ms": wall * 1e3,
                 "replicas_per_s": R / wall, "events_per_s": ev / wall,
                 "status_max": int(r.status.max().item()),
                 "tie_replicas": int(((r.status & L.ST_TIE) != 0).sum().item()), "plan": plan}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--only", default="", help="comma-separated sections: " + ",".join(SECTIONS))
    a = ap.parse_args()
    only = set(a.only.split(",")) if a.only else set(SECTIONS)
    bad = only - set(SECTIONS)
    if bad:
        raise SystemExit("unknown sections: %s" % sorted(bad))
    want = lambda k: k in only  # noqa: E731
    torch.cuda.set_device(0)
    so = graphs.c3()
    g = graph_of(so)
    res = {}
    if want("sweep_event_log"):
        sweep_event_log(g, so, a, res)
    if only & REPLAY:
        replay(g, so, a, res, want)
    if want("scan"):
        scan(g, so, a, res)
    if want("oracle_dp"):
        oracle(a, res)
    for k in ("seq_multigraph_c3", "seq_600_sources", "seq_max_events_c3", "fast_max_events_c3",
              "fast_realdata_c3", "fast_600_sources", "fast_3000_sources"):
        if want(k):
            seq(k, a, res)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
