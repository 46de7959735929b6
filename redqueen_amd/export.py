"""Columnar export of batched event logs.

The reference materialises one pandas frame per replica through
``State.get_dataframe`` (opt_model.py:85-97) -- 40 bytes per (event, sink) row
built by Python loops.  Here a whole ``RQ_RUN_EVENT_LOG`` batch is expanded on
the GPU (``rq_log_rows`` / ``rq_log_expand``) into the same five columns plus a
``replica`` column, then written once as Arrow IPC / Parquet (pyarrow) or npz,
so reference-style pandas analysis runs on GPU outputs without per-row Python.

    res = graph.run("opt", ..., n_rep=R, event_log=True)
    write_parquet(res, "logs.parquet")       # or write_ipc / write_npz
    df = read_npz("logs.npz")                # replica, event_id, ..., sink_id
"""
import numpy as np

COLUMNS = ("event_id", "time_delta", "src_id", "t", "sink_id")


def host_columns(res):
    """(row_off, {replica, event_id, time_delta, src_id, t, sink_id} numpy) of a batch."""
    ro, cols = res.log_columns()
    gids = getattr(res, "global_ids", None)
    if gids is None:
        gids = np.arange(len(ro) - 1, dtype=np.int64) + getattr(res, "replica0", 0)
    out = {"replica": np.repeat(np.asarray(gids, dtype=np.int64), np.diff(ro))}
    for k in COLUMNS:
        out[k] = cols[k].cpu().numpy()
    return ro, out


def to_arrow(res):
    import pyarrow as pa
    _, cols = host_columns(res)
    return pa.table({k: pa.array(v) for k, v in cols.items()})


def write_ipc(res, path):
    import pyarrow as pa
    tab = to_arrow(res)
    with pa.OSFile(str(path), "wb") as f, pa.ipc.new_file(f, tab.schema) as w:
        w.write_table(tab)
    return tab.num_rows


def write_parquet(res, path):
    import pyarrow.parquet as pq
    tab = to_arrow(res)
    pq.write_table(tab, str(path))
    return tab.num_rows


def write_npz(res, path):
    ro, cols = host_columns(res)
    np.savez(str(path), row_off=ro, **cols)
    return int(ro[-1])


def read_npz(path, replica=None):
    """DataFrame of an npz export (all replicas, or one in the reference layout)."""
    import pandas as pd
    z = np.load(str(path), allow_pickle=False)
    if replica is None:
        return pd.DataFrame({k: z[k] for k in ("replica",) + COLUMNS})
    ro = z["row_off"]
    a, b = int(ro[replica]), int(ro[replica + 1])
    return pd.DataFrame({k: z[k][a:b] for k in COLUMNS})
