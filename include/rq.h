/*
 * rq.h -- C ABI of librq.so, the MI355X (gfx950) RedQueen Monte-Carlo engine.
 *
 * The reference (MPI-SWS/RedQueen) is pure Python with no FFI; these entry
 * points replace the following in-process Python calls (file:line into the
 * reference):
 *
 *   rq_graph_build      SimOpts(**kw)                      opt_model.py:773-780
 *                       + Manager.__init__ validation       opt_model.py:145-181
 *                       + Broadcaster.init_state sink lists opt_model.py:340-344
 *   rq_run_batch        SimOpts.create_manager_with_opt     opt_model.py:806-811
 *                       / _with_poisson :821-837 / _for_wall :886-891
 *                       / _with_times :893-898 / _with_piecewise_const :839-848
 *                       -> Manager.run_dynamic              opt_model.py:241-314
 *                       -> State.get_dataframe              opt_model.py:85-97
 *                       -> utils.time_in_top_k / average_rank / int_r_2 /
 *                          num_tweets_of                    utils.py:84-121,170-176
 *                       over a seeds x q x s grid, i.e. the loops of
 *                       utils.calc_q_capacity_iter          utils.py:447-470 and
 *                       opt_runs.worker_opt/worker_poisson  opt_runs.py:51-126
 *                       with opt_runs.add_perf's fields     opt_runs.py:41-48
 *   rq_metrics_replay   utils.time_in_top_k(df, K, ...)     utils.py:84-98
 *   (_batch: many dfs)  utils.average_rank(df, ...)         utils.py:101-114
 *                       utils.int_r_2(df, ...)              utils.py:117-121
 *                       utils.num_tweets_of(df, ...)        utils.py:170-176
 *                       on dataframes in the reference's row layout (raw sink ids).
 *   rq_oracle_dp        utils.oracle_ranking(df, sim_opts)  utils.py:181-245
 *                       (batched over walls / q values: the loops of
 *                       find_opt_oracle :260-340 and opt_runs.worker_oracle
 *                       opt_runs.py:129-155)
 *   rq_rank_table       utils.rank_of_src_in_df(df, src)    utils.py:38-56
 *   rq_u_int            utils.u_int_opt(df, ...)            utils.py:59-81
 *   rq_log_rows /       State.get_dataframe()               opt_model.py:85-97
 *   rq_log_expand       for every replica of an RQ_RUN_EVENT_LOG batch at once
 *
 * Conventions
 *   - every function returns 0 (RQ_OK) or a negative rq_status; no C++
 *     exception crosses the ABI; rq_strerror() names a code.
 *   - rq_graph_t handles are immutable after build and may be shared by threads.
 *   - rq_run_batch / rq_metrics_replay are stream-ordered and asynchronous:
 *     they enqueue work on `hip_stream` (a hipStream_t, NULL = default stream)
 *     and never touch caller memory on the host side.  The caller owns every
 *     device buffer (workspace and outputs) and must keep them alive until the
 *     stream has passed the work.  rq_run_batch stages its per-run parameter
 *     tables through a ring of 4 pinned host buffers owned by the graph handle:
 *     the ring is allocated (hipHostMalloc) on the first call and when a larger
 *     table is needed, and a call waits (hipEventSynchronize) for the copy
 *     issued by the call 4 earlier on the same graph before reusing its slot --
 *     so a warm-up call keeps allocation out of timed regions, and a caller
 *     issuing many batches back to back runs at most 4 copies ahead.
 *     rq_metrics_replay never allocates or waits.  One device per process; the
 *     caller selects it.
 *   - "device pointer" = memory allocated on the current HIP device
 *     (e.g. torch.empty(..., device="cuda").data_ptr()).
 */
#ifndef RQ_H
#define RQ_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RQ_ABI_VERSION 6
#define RQ_MAX_K 4 /* at most 4 K values (perf_opts.Ks, opt_runs.py:31-38) per run */

typedef enum {
    RQ_OK = 0,
    RQ_EINVAL = -1,       /* bad argument / reference would raise (assert, ValueError, KeyError) */
    RQ_EOVERFLOW = -2,    /* a capacity was too small (see per-replica status bits)    */
    RQ_EHIP = -3,         /* a HIP runtime call failed                                   */
    RQ_ENOMEM = -4,       /* host or device allocation failed                            */
    RQ_EUNSORTED = -5,    /* replay: df 't' column is not non-decreasing                 */
    RQ_EUNSUPPORTED = -6  /* valid for the reference, not supported by this engine       */
} rq_status;

/* broadcaster kinds (SimOpts.broadcasters, opt_model.py:758-766) */
typedef enum {
    RQ_SRC_NONE = 0,      /* controlled slot only: create_manager_for_wall          */
    RQ_SRC_POISSON = 1,   /* Poisson        opt_model.py:424-433 (dynamic)          */
    RQ_SRC_POISSON2 = 2,  /* Poisson2       opt_model.py:381-421 (static)           */
    RQ_SRC_HAWKES = 3,    /* Hawkes         opt_model.py:458-490                    */
    RQ_SRC_PWCONST = 4,   /* PiecewiseConst opt_model.py:626-689                    */
    RQ_SRC_REALDATA = 5,  /* RealData       opt_model.py:711-750                    */
    RQ_SRC_OPT = 6,       /* Opt = RedQueen opt_model.py:493-544 (controlled only)  */
    RQ_SRC_OPTPW = 7      /* OptPWSignificance opt_model.py:547-623 (controlled only) */
} rq_src_kind;

typedef struct rq_source_desc {
    int32_t kind;        /* rq_src_kind                                                   */
    int32_t n_arr;       /* PWCONST: #segments; REALDATA: #times                           */
    int64_t src_id;
    uint32_t seed;       /* kwargs['seed'] (RandomState seed, opt_model.py:329)            */
    uint32_t flags;      /* RQ_SRCF_* (ABI v6; was reserved, 0)                            */
    double p0, p1, p2;   /* POISSON/POISSON2: rate; HAWKES: l_0, alpha, beta               */
    const double* a;     /* host: PWCONST change_times[n_arr]; REALDATA times[n_arr]       */
    const double* b;     /* host: PWCONST rates[n_arr]                                     */
} rq_source_desc;
/* rq_source_desc.flags: RQ_SRCF_DYNAMIC on an RQ_SRC_REALDATA source = its times are a
   DYNAMIC broadcaster's (a registered plugin with is_dynamic, opt_model.py:259-260,
   replayed from its times): at an equal time it plays before every static source and
   among the dynamic ones (the controller included) in src_id order
   (opt_model.py:279-281, :289-290), like the built-in Poisson / Hawkes. */
#define RQ_SRCF_DYNAMIC 1

typedef struct rq_graph_desc {
    int32_t n_sources;                /* SimOpts.other_sources, in list order          */
    const rq_source_desc* sources;    /* host                                           */
    int32_t n_sinks;
    const int64_t* sink_ids;          /* host, SimOpts.sink_ids                          */
    int64_t n_edges;
    const int64_t* edge_src;          /* host, SimOpts.edge_list in list order           */
    const int64_t* edge_sink;
    int64_t ctrl_src_id;              /* SimOpts.src_id                                  */
    double start_time;                /* Manager start_time (0 in every reference call)  */
    double end_time;                  /* SimOpts.end_time                                */
    /* controlled broadcaster parameters used by RQ_SRC_PWCONST / RQ_SRC_REALDATA runs */
    int32_t ctrl_n_arr;
    const double* ctrl_a;             /* host: change_times or event_times               */
    const double* ctrl_b;             /* host: rates                                     */
} rq_graph_desc;

typedef struct rq_graph* rq_graph_t;

/* status bits written per replica into rq_outputs.status */
#define RQ_ST_ROWS_OVERFLOW 1    /* metric-row / event-log capacity exceeded: rerun with larger cap_scale */
#define RQ_ST_STREAM_OVERFLOW 2  /* a source's arrival stream exceeded its capacity: rerun      */
/* A replica flagged with either overflow bit ran TRUNCATED: its metrics and counts cover
   only the events that fit and are not the reference's.  Every other replica of the batch
   is exact.  The library never reruns by itself: the Python Graph.run(check=True) reruns
   the batch with doubled cap_scale (and remembers the scale for the graph's later runs);
   check=False hands the flagged rows back as they are, for the caller to mask or rerun. */
#define RQ_ST_TIE 4              /* events at equal times shared a pivot row.  Exact (pivot cells
                                    averaged like pandas) in the sequential sweep -- sweep_mode 2,
                                    a multigraph, repeated graph-level RealData times; the fast
                                    tiled sweep keeps the last row, so for a replica flagged
                                    here avg-rank / r^2 may differ: rerun it with sweep_mode 2
                                    (alone: rep_idx; Graph.run(check=True) does) */
#define RQ_ST_EMPTY 8            /* no event reached any sink: the reference's df is empty      */
#define RQ_ST_UNORDERED 16       /* a sequential run over > 2048 sources (merged streams) met more
                                    than 2048 arrivals at ONE time (replayed data only): their
                                    order is not the reference's, the replica is not played    */

#define RQ_RUN_EVENT_LOG 1       /* also write the (t, source) event log (for get_dataframe)    */

typedef struct rq_batch_desc {
    int32_t ctrl_kind;           /* RQ_SRC_OPT / OPTPW / POISSON2 / PWCONST / REALDATA / NONE   */
    int32_t n_grid;              /* grid points                                                  */
    const double* q;             /* host [n_grid] (OPT)                                          */
    const double* s;             /* host [n_grid * n_followers], sorted-follower order (OPT)     */
    int64_t n_rep;               /* replicas per grid point; replica id i = g * n_rep + r        */
    const uint32_t* ctrl_seed;   /* device [n_grid*n_rep] or NULL: ctrl_seed0 + k(i)             */
    uint32_t ctrl_seed0;
    int32_t randomize_world;     /* 1: world seeds = u_i + 99*idx (randomize_other_sources,      */
                                 /*    opt_model.py:795-804); 0: the graph's fixed seeds         */
    const uint32_t* world_seed;  /* device [n_grid*n_rep] u_i, or NULL: world_seed0 + k(i)       */
    uint32_t world_seed0;
    int64_t seed_mod;            /* k(i) = i % seed_mod if > 0 else i; seed_mod = n_rep gives    */
                                 /* every grid point the same seeds (calc_q_capacity_iter)       */
    const double* ctrl_rate;     /* device [n_grid*n_rep] Poisson2 rate (RQ_SRC_POISSON2)        */
    double ctrl_rate_max;        /* host: max of ctrl_rate, sizes the stream capacity            */
    const int32_t* Ks;           /* host [nK], nK <= RQ_MAX_K                                     */
    int32_t nK;
    int64_t max_events;          /* run_dynamic(max_events); < 0 = unbounded                     */
    int32_t flags;               /* RQ_RUN_EVENT_LOG                                              */
    double cap_scale;            /* >= 1: multiplies every auto-sized capacity                   */
    int64_t chunk;               /* replicas per launch (0 = library default: the batch in an   */
                                 /* even number of chunks of <= 131072, pipelined on two streams */
                                 /* within the workspace budget, ws_budget below)               */
    int64_t replica0;            /* this call runs global replicas [replica0, replica0+n_local):  */
    int64_t n_local;             /* a shard of the grid (0 = all n_grid*n_rep); outputs are      */
                                 /* indexed locally, seeds and grid point use the global id     */
    int32_t sweep_mode;          /* 0 auto: a fast tiled sweep unless the run needs the exact
                                    sequential one (a multigraph; the graph's own RealData
                                    times repeat a time); max_events cuts the fast sweeps'
                                    tiles, per-replica RealData streams play on them (a replica
                                    meeting equal times is flagged RQ_ST_TIE); the fast sweeps
                                    write the event log themselves.
                                    The fast sweeps play MERGED streams: rq_gen_streams writes
                                    every source's arrivals, rq_merge_streams merges them into
                                    one (t, stream) sequence per replica, and the sweep plays it
                                    in tiles of 64 entries (the fused sweep for <= 64 sources,
                                    the general sweep above);
                                    1 fast whenever max_events allows; 2 force the sequential
                                    sweep; 3 as 0 but never a K=1 sink-bit variant (per-sink
                                    ranks); 4 / 5 as 0 / 1 on the general sweep instead of the
                                    fused one; 6 as 4 with the general sweep merging the
                                    per-source streams itself (register windows, the round-2
                                    kernel); 7 as 0 with the fused sweep generating its arrivals
                                    in-kernel (LDS rings, the round-2 kernel).  Every variant
                                    gives the same bits; 6 and 7 are kept for A/B checks      */
    /* RQ_SRC_OPTPW (create_manager_with_significance, opt_model.py:850-884): the follower
       significance s_pw[g][f][k] over n_seg equal segments of time_period, rows in the
       order of rq_graph_followers (sorted follower ids), q from q[g] */
    int32_t n_seg;
    double period;
    const double* s_pw;          /* host [n_grid][n_followers][n_seg]                            */
    /* Per-replica times of RealData sources -- the static broadcasters a user registers
       with SimOpts.registerSource (opt_model.py:768-771): the host runs their
       initialize() / get_all_times() (:336-338, :391-394) once per replica (seeded as
       randomize_other_sources gives them) and hands the times over here.  Source k is the
       graph's RealData source rd_src_id[k] (declared with no times); replica i (global id)
       plays rd_times[rd_off[i * n_rd + k] .. rd_off[i * n_rd + k + 1]), sorted and within
       [start_time, end_time].  n_rd = 0: every RealData source plays its graph times. */
    int32_t n_rd;                /* <= RQ_MAX_RD                                                 */
    const int64_t* rd_src_id;    /* host [n_rd]                                                  */
    const int64_t* rd_cap;       /* host [n_rd]: the most times any replica gives source k       */
    const double* rd_times;      /* device                                                       */
    const int64_t* rd_off;       /* device [n_grid * n_rep * n_rd + 1]                           */
    /* Per-grid-point replica window (ABI v4): this call's replica space is the
       n_grid x rep_cnt grid of global ids i = g * n_rep + rep_lo + rr, rr < rep_cnt,
       flattened as g * rep_cnt + rr; replica0 / n_local then select a contiguous part
       of THAT space and outputs are indexed by it.  A multi-GPU shard that takes the
       same replica window of every grid point sees every grid point (every q), so
       shards cost the same however the work per replica varies with q.
       rep_cnt = 0: the whole grid (rep_lo = 0, rep_cnt = n_rep). */
    int64_t rep_lo;
    int64_t rep_cnt;
    /* Device-memory budget of the workspace (ABI v5), bytes.  With the library's chunking
       (chunk = 0) the plan takes smaller chunks (an even count when pipelined) until the
       buffer sets in flight fit it; RQ_ENOMEM when one replica does not.  0: the library's
       default -- rq_workspace_size / rq_plan_info / rq_event_capacity take 0.9 x the
       device's free memory (hipMemGetInfo), rq_run_batch the workspace_bytes it is handed
       (so a workspace sized by rq_workspace_size always fits; the chunking, never the
       results, may differ).  A caller that frees or reuses memory of its own (a caching
       allocator) passes its reclaimable total here so both calls plan alike.  The
       environment variable RQ_WS_BUDGET_GB caps either. */
    int64_t ws_budget;
    /* Replica list (ABI v6): host [n_local] global ids (i = g * n_rep + r, each in
       [0, n_grid * n_rep)); the call runs exactly these replicas, output k = replica
       rep_idx[k] -- seeds, grid point and per-replica inputs (ctrl_seed, world_seed,
       ctrl_rate, rd_*) come from the global id as in the full batch, so a replica gives
       the same bits alone as inside its batch.  Requires replica0 = 0, rep_cnt = 0 and
       n_local > 0.  The caller reruns only a batch's flagged replicas with it (an
       RQ_ST_*_OVERFLOW replica at a larger cap_scale, an RQ_ST_TIE one on the exact
       sequential sweep, sweep_mode 2).  NULL: the replica space above. */
    const int64_t* rep_idx;
} rq_batch_desc;
#define RQ_MAX_RD 64

typedef struct rq_outputs {
    double* metrics;   /* device [R][nK + 2]: top_K..., avg_rank, r_2  (R = n_local or n_grid*rep_cnt) */
    int64_t* counts;   /* device [R][4]: num_events (own posts that reached a sink = the   */
                       /* reference 'capacity'), world_events, n_events (all), pivot rows   */
    int32_t* status;   /* device [R]: RQ_ST_* bits                                            */
    double* ev_t;      /* device [R][ev_cap] event times   (RQ_RUN_EVENT_LOG)                */
    int32_t* ev_src;   /* device [R][ev_cap] source index  (rq_graph_source_ids order)       */
    int64_t ev_cap;
} rq_outputs;

int rq_abi_version(void);
const char* rq_strerror(int code);

int rq_graph_build(const rq_graph_desc* desc, rq_graph_t* out);
int rq_graph_free(rq_graph_t g);
/* info[0] n_streams, [1] n_sinks, [2] n_followers, [3] n_edges, [4] ctrl stream index or -1 */
int rq_graph_info(rq_graph_t g, int64_t* info);
/* src_id of every stream index (the ev_src values); ids[n_streams], host */
int rq_graph_source_ids(rq_graph_t g, int64_t* ids);
/* sink ids in follower order (the order of rq_batch_desc.s), host */
int rq_graph_followers(rq_graph_t g, int64_t* ids);

/* bytes of device workspace rq_run_batch needs for this graph/batch */
int rq_workspace_size(rq_graph_t g, const rq_batch_desc* b, size_t* bytes);
/* suggested per-replica event-log capacity for RQ_RUN_EVENT_LOG */
int rq_event_capacity(rq_graph_t g, const rq_batch_desc* b, int64_t* cap);
/* how rq_run_batch will run this batch (diagnostics / occupancy reporting):
 * info[0] sweep variant (0 fast tiled, 1 sequential exact, 2 fast tiled on K=1 sink
 * bitsets, 3 fast tiled on K=1 per-wave LDS sink bits, 4 sequential exact with the
 * per-sink state in global memory; +10 fused), [1] sources per lane,
 * [2] arrival-ring depth W, [3] waves per block, [4] blocks per CU (runtime occupancy,
 * 0 without a device), [5] sink columns in LDS (1) or global (0), [6] dynamic LDS
 * bytes per block, [7] replicas per chunk */
int rq_plan_info(rq_graph_t g, const rq_batch_desc* b, int64_t* info);

int rq_run_batch(rq_graph_t g, const rq_batch_desc* b, const rq_outputs* out,
                 void* workspace, size_t workspace_bytes, void* hip_stream);

/* Metrics of dataframes in the reference's row layout (State.get_dataframe,
 * opt_model.py:85-97): one row per (event, sink) in df order, 't' non-decreasing
 * within a dataframe, sink ids RAW (any int64; the pivot columns -- the sorted
 * unique sink ids of each dataframe -- are built on the device).  Replaces
 *   utils.time_in_top_k(df, K, src_id, end_time)      utils.py:84-98
 *   utils.average_rank(df, src_id, end_time)           utils.py:101-114
 *   utils.int_r_2(df, sim_opts)                        utils.py:117-121
 *   utils.num_tweets_of(df, src_id) (+ world events)   utils.py:170-176, opt_runs.py:41-48
 * with the reference's arithmetic bit for bit (rank_of_src_in_df utils.py:38-56:
 * per-sink rank scan, pivot mean of duplicate (t, sink) rows, ffill; numpy's
 * pairwise sums).
 *   t, src, sink, event_id : device [n_rows] (event_id may be NULL)
 *   out                    : device [n_df][nK + 2]  top_K..., avg_rank, r_2 (NaN on error)
 *   counts                 : device [n_df][4]       num_tweets_of(src_id), world events
 *                            (-1 without event ids or if event_id decreases), pivot rows
 *                            (0: empty df; RQ_EUNSORTED: 't' decreases; RQ_EOVERFLOW: the df
 *                            needs the RQ_REPLAY_LARGE workspace; RQ_EINVAL: its df_off range
 *                            is malformed -- negative, decreasing, past n_rows or >= 2^31 rows),
 *                            unique sinks
 * Workspace: rq_replay_workspace_size; the small one serves dataframes with <= 3071
 * unique sinks (the per-sink state lives in LDS), RQ_REPLAY_LARGE any width.
 * RQ_REPLAY_CHUNKED adds room (~32 B per row + 192 KB per dataframe) for spreading ONE
 * long dataframe over many workgroups (chunks of 4096 rows; <= 4096 unique sinks), which
 * the call uses for up to 64 dataframes averaging >= 8192 rows (a batch of many
 * dataframes runs one workgroup per dataframe).
 * Per dataframe: < 2^31 rows. */
#define RQ_REPLAY_LARGE 1
#define RQ_REPLAY_CHUNKED 2
int rq_replay_workspace_size(int64_t n_rows, int64_t n_df, int32_t nK, int32_t flags, size_t* bytes);
int rq_metrics_replay(const double* t, const int64_t* src, const int64_t* sink,
                      const int64_t* event_id, int64_t n_rows, int64_t src_id, double end_time,
                      const int32_t* Ks, int32_t nK, double* out, int64_t* counts,
                      void* workspace, size_t workspace_bytes, void* hip_stream);
/* Many dataframes at once (the replicas of a batch, the reference's loop of
 * utils calls over opt_runs worker outputs): dataframe d owns rows
 * [df_off[d], df_off[d + 1]) of the concatenated columns; df_off device [n_df + 1],
 * n_rows = df_off[n_df]. */
int rq_metrics_replay_batch(const double* t, const int64_t* src, const int64_t* sink,
                            const int64_t* event_id, const int64_t* df_off, int64_t n_df,
                            int64_t n_rows, int64_t src_id, double end_time, const int32_t* Ks,
                            int32_t nK, double* out, int64_t* counts, void* workspace,
                            size_t workspace_bytes, void* hip_stream);

/* Offline oracle (utils.oracle_ranking) for n_inst single-follower walls at once.
 * Instance i: n_i wall events, w_i[0..n_i+2) = np.diff([0, 0, event_times..., end_time])
 * (utils.py:207), q_i, s_i.  Device arrays: w (instances concatenated), w_off[n_inst+1]
 * (prefix of n_i + 2), q[n_inst], s[n_inst], out_off[n_inst+1] (prefix of n_i + 1).
 * Outputs (device): cost[i] = J[0, 0]; events / ranks [out_off[i] .. + n_i + 1) = the
 * oracle_df 'events' and 'ranks' columns.  n_max >= every n_i (<= 1e6, the reference's
 * own limit); workspace: rq_oracle_workspace_size (n_inst (n_max+1)^2 / 8 bytes of
 * decision bits). */
int rq_oracle_workspace_size(int32_t n_inst, int64_t n_max, size_t* bytes);
int rq_oracle_dp(const double* w, const int64_t* w_off, const double* q, const double* s,
                 int32_t n_inst, int64_t n_max, double* cost, int32_t* events, int32_t* ranks,
                 const int64_t* out_off, void* workspace, size_t workspace_bytes, void* hip_stream);

/* rank_of_src_in_df: table[n_t][n_cols] (device) of the rank of src_id in every sink's
 * feed at every unique t (index[n_t], device); cells = mean of the (t, sink) ranks, then
 * forward-filled per column when fill != 0 (NaN before a sink's first row / without fill).
 * Rows in df order, t non-decreasing; n_t = number of unique t.  err (device int32[1]):
 * 0 ok, bit 0 t not sorted, bit 1 n_t wrong. */
int rq_rank_table(const double* t, const int64_t* src, const int32_t* sink_col, int64_t n_rows,
                  int32_t n_cols, int64_t src_id, int32_t fill, int64_t n_t, double* table,
                  double* index, int32_t* err, void* hip_stream);

/* u_int_opt from a filled rank table: sum_k (sum_f table[k, fcol[f]] * wts[f]) * dt_k with
 * dt_k = index[k+1] - index[k] (end_time - index[n_t-1] last), numpy pairwise sum.
 * wts = sqrt(s / q) per follower (device), fcol their table columns (device).
 * out: device double[1]; workspace >= n_t * 8 bytes. */
int rq_u_int(const double* table, const double* index, int64_t n_t, int32_t n_cols,
             const int32_t* fcol, const double* wts, int32_t n_f, double end_time, double* out,
             void* workspace, size_t workspace_bytes, void* hip_stream);

/* Dataframe rows of a batch's event logs (State.get_dataframe, opt_model.py:85-97):
 * one row per (event, sink of an edge of the event's source), event order then
 * edge-list order.  ev_t / ev_src / counts are rq_run_batch's outputs (RQ_RUN_EVENT_LOG,
 * counts[i][2] = events of replica i), ev_cap their row stride.
 * rq_log_rows writes row_off[n_rep + 1] (device): replica i owns rows
 * [row_off[i], row_off[i+1]).  rq_log_expand then fills the five reference columns
 * (device, row_off[n_rep] rows each): event_id (100 + event index), time_delta, src_id,
 * t, sink_id.  time_delta follows the reference's accumulated State.time
 * (opt_model.py:68, :304): time_delta_k = t_k - time_{k-1}, time_k = time_{k-1} +
 * time_delta_k, time_{-1} = start_time -- which differs from t_k - t_{k-1} in the last
 * bit wherever the running sum has rounded. */
int rq_log_rows(rq_graph_t g, const int32_t* ev_src, const int64_t* counts, int64_t n_rep,
                int64_t ev_cap, int64_t* row_off, void* hip_stream);
int rq_log_expand(rq_graph_t g, const double* ev_t, const int32_t* ev_src, const int64_t* counts,
                  int64_t n_rep, int64_t ev_cap, const int64_t* row_off, int64_t* event_id,
                  double* time_delta, int64_t* src_id, double* t, int64_t* sink_id,
                  void* hip_stream);

/* Per-kernel timing for benchmarks: rq_timing(1) starts recording HIP events
 * around every kernel this library launches (on the caller's stream);
 * rq_timing_read() waits for them and returns, per kernel class
 * [0 stream generation, 1 sweep, 2 scan, 3 replay, 4 merge], the summed milliseconds
 * and the number of launches, then clears the record.  rq_timing(0) stops. */
int rq_timing(int enable);
int rq_timing_read(double* ms, int64_t* launches);

#ifdef __cplusplus
}
#endif
#endif /* RQ_H */
