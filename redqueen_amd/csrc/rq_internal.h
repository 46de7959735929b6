// rq_internal.h -- kernel argument blocks shared by rq_kernels.hip and rq_api.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <map>
#include <mutex>
#include <tuple>

#include "../../include/rq.h"

// global replica id of position s of a call's replica space (rq_batch_desc.rep_lo /
// rep_cnt): the n_grid x rep_cnt window of every grid point's n_rep replicas
__host__ __device__ __forceinline__ int64_t rq_global_replica(int64_t s, int64_t n_rep, int64_t rep_lo,
                                                               int64_t rep_cnt)
{
    return rep_cnt == n_rep ? s : (s / rep_cnt) * n_rep + rep_lo + s % rep_cnt;
}

struct GenArgs {
    int64_t n_chunk, chunk0, rep0;   // local replica = chunk0 + rl, space position = rep0 + local
    int64_t n_rep, rep_lo, rep_cnt;  // global id = rq_global_replica(rep0 + local, ...)
    const int64_t* rep_idx;          // rq_batch_desc.rep_idx (device copy): global id = rep_idx[local]
    int n_str, ctrl_idx, ctrl_stream_kind, randomize;
    int64_t seed_mod;
    const uint32_t* ctrl_seed;
    uint32_t ctrl_seed0;
    const uint32_t* world_seed;
    uint32_t world_seed0;
    const double* ctrl_rate;
    const int* kind;
    const int* orig_idx;
    const uint32_t* seed;
    const double *p0, *p1, *p2;
    const int *arr_off, *arr_n;
    const double *arr_a, *arr_b;
    const int64_t* st_off;
    const int* cap;
    int64_t capsum;
    double start, end;
    double* streams;
    int* slen;                       // [n_str][slen_stride]: lane-coalesced stores
    int64_t slen_stride;             // >= n_chunk (the chunk buffers' replica capacity)
    int32_t* status;
    // per-replica RealData times (rq_batch_desc.rd_*): stream j -> source k or -1
    const int* rd_k;
    int n_rd;
    const double* rd_times;
    const int64_t* rd_off;
};

// global id of a call's local replica: the replica list (rq_batch_desc.rep_idx) or the
// replica space position rep0 + local
__host__ __device__ __forceinline__ int64_t rq_replica_of(const GenArgs& a, int64_t local)
{
    return a.rep_idx ? a.rep_idx[local] : rq_global_replica(a.rep0 + local, a.n_rep, a.rep_lo, a.rep_cnt);
}

#define RQ_MAX_STREAMS 2048   // 512 per fast instance (8 per lane); LOG instances 16 / 32 per lane

struct SweepArgs {
    int64_t n_chunk, chunk0, n_rep, rep0;
    int wpb, n_str, n_sinks, n_sinks_pad, ctrl_idx, ctrl_kind, n_fol;
    int Ks[RQ_MAX_K];
    int64_t ctrl_src_id;
    int64_t seed_mod;
    const uint32_t* ctrl_seed;
    uint32_t ctrl_seed0;
    const int64_t* src_id;     // [n_str]
    const double* inv_c;       // [n_grid][n_str]
    const double* pw_c;        // OptPWSignificance: [n_grid][n_str][n_seg] (else null)
    const double* pw_max;      // [n_grid][n_str]
    int n_seg;
    double period;
    const int* csr_ptr;        // [n_str + 1]
    const int* csr_col;        // sink columns, edge-list order per source
    const int* outdeg_f;       // [n_str] edges into the controlled source's followers
    const int* cbf_g;          // [n_str] the controller posts first at an equal time (GT instances)
    const int* fol;            // [n_fol] follower columns
    const int64_t* st_off;
    int64_t capsum;
    const double* streams;
    const int* slen;           // [n_str][slen_stride]
    int64_t slen_stride;
    double start, end;
    int64_t max_events;
    int64_t cap_rows;
    double* rows_t;
    double* rows_sum;
    uint32_t* rows_valid;
    uint32_t* rows_cnt;
    int* sall;
    int64_t* counts;
    int32_t* status;
    double* ev_t;
    int32_t* ev_src;
    int64_t ev_cap;
    int n_csr;
    const uint32_t* masks;   // [n_str][nw] sink bitsets (BITS variant)
    int nw, mstride;         // words per bitset; LDS row stride in words (odd: bank spread)
    const uint32_t* fbits;   // follower set as a sink bitset [nwl] (BL variant)
    int nwl;                 // BL: words per per-wave T / V bitset = ceil(n_sinks / 32)
    size_t lds_fbits;        // BL: the follower bitset's place in the block's shared LDS
    size_t lds_skip;         // BL + MRG: per-wave stream stamps / first-lane table (0: no skipping)
    size_t lds_etab;         // fused sweep: rq_exp's table (64 x u64) in the block's shared LDS
    int dbg;                 // profiling: 1 skip phase C, 2 skip sink updates, 3 skip phase B
    unsigned long long* clk; // RQ_PHASE_CLOCK builds only: per-phase s_memtime sums [8]
    double tile_target;      // fused sweep: arrivals a tile aims at (the cut adapts to it)
    int fw_hmin;             // fused sweep: a ring showing fewer arrivals forces refill passes (1..H)
    size_t lds_invc;         // general sweep, one grid point: 1/c_j [n_str] in the block's shared LDS
    int invc_shared;         //   (else each wave loads its replica's grid point at the start of its wave region)
    int fw_thr;              // fused sweep: opportunistic refill passes while >= fw_thr rings are below W
    int fw_hfill;            // fused sweep: a forced refill run ends once every ring shows >= fw_hfill
    int* wq;                 // fused sweep: replica work queue (zeroed per launch; null = one replica per wave)
    int col_in_lds, win;     // general sweep: CSR copied to LDS; arrival-ring depth
    size_t lds_col, lds_ptr, lds_odf, lds_cbf, lds_wave, lds_wave_stride, lds_rank_off, lds_win_off, lds_x_off, lds_mask,
        lds_total, lds_stage_off;
    GenArgs gen;             // fused sweep: arrival generation parameters
    // duplicate edges: stream j's CSR row is layers of distinct sinks, ending at
    // lay_end[lay_ptr[j] .. lay_ptr[j+1]) (null: one layer per row, a simple graph)
    const int* lay_ptr;
    const int* lay_end;
    // LOG sweep with the per-sink state in global memory (more sinks than LDS holds):
    // gs_slots wave slots of gs_stride bytes (rank int + gtag/gcnt/gsum per sink)
    char* gs;
    int64_t gs_stride;
    int gs_slots;
    // general fast sweep on merged streams (rq_merge_streams): replica rl's arrivals of
    // every source in play order, mrg_t / mrg_j [rl * mrg_stride + k], k < mrg_len[rl]
    const double* mrg_t;
    const uint16_t* mrg_j;
    const uint8_t* mrg_jh;     // > 65535 streams: bits 16-23 of each entry's stream (else null)
    const int* mrg_len;
    int64_t mrg_stride;        // entries per replica of mrg_t / mrg_j
    // longest-first play order of the chunk's replicas (rq_order_replicas over mrg_len):
    // the wave slots and the work queue take chunk replica order[q] for queue position q
    // (null: q itself).  Outputs stay indexed by replica, so no result bit depends on it.
    const int* order;
};

// rq_merge_streams: one block per replica merges its pre-generated per-source streams
// into the (t, stream) sequence the sweep plays -- time order, equal times in stream
// order, a source's equal times in stream order (the windowed sweep's stage rank)
struct MergeArgs {
    int64_t n_chunk, chunk0;
    int n_str;
    int64_t capsum;
    const int64_t* st_off;
    const double* streams;
    const int* slen;        // [n_str][slen_stride]
    int64_t slen_stride;
    double end;
    double* out_t;          // [C][mrg_stride]
    uint16_t* out_j;        // [C][mrg_stride] the stream (a group-local one at a two-level merge's first level)
    uint8_t* out_jh;        // > 65535 streams: bits 16-23 of the stream (else null)
    int* out_len;           // [C]
    int64_t mrg_stride;     // capacity per replica: past it the replica is flagged RQ_ST_STREAM_OVERFLOW
    int32_t* status;        // RQ_ST_TIE (strict_ties: RQ_ST_UNORDERED) when > RQ_MG_CAP arrivals share one time
    int strict_ties;        // the sequential sweep plays this sequence: no exact rerun behind it
    // two-level merge (> RQ_MG_B sources): the first level merges group g's streams
    // [g RQ_MG_B, (g + 1) RQ_MG_B) of replica rl (grid y = group) into out_* at
    // [(rl n_grp + g) mrg_stride]; the second level (sub-merge) takes those n_grp
    // sequences -- sub_t / sub_j / sub_len, sub_stride entries each -- as its streams
    const double* sub_t;
    const uint16_t* sub_j;
    const int* sub_len;
    int n_grp;
    int64_t sub_stride;
    // streams per first-level group: RQ_MG_B, or 64 (one-wave blocks) up to 64 groups of
    // them -- the second level then has more streams walking (a lane per group) per round
    int grp_sz;
    unsigned long long* clk;   // RQ_PHASE_CLOCK builds only: per-phase s_memtime sums [8]
};
#define RQ_NPSUM1_LDS 516   // doubles of wave_npsum<1> scratch (== rq::npsum_lds_doubles<1>())
// threads per block of the merged-stream sweep instances (1024: <= 128 VGPRs)
#ifndef RQ_MRG_LB
#define RQ_MRG_LB 1024
#endif
// wall events per branch-free batch of the merged-stream K = 1 sink-bit sweep: C5 sweep
// per 4096 replicas on one stream (same box, round 5) 4: 139.0, 5: 136.1, 6: 135.0 ms;
// the pipelined 8192-replica step 382.6 / 372.0 / 374.5 ms (gpurun_out/abc5)
// merged-stream sweeps: a tile's rows are stored at the top of the next tile, ahead of
// its prefetch loads (RowStage::flush_pend); 0 = at the end of their own tile (A/B)
#ifndef RQ_MRG_DEFER
#define RQ_MRG_DEFER 1
#endif
#ifndef RQ_MRG_BLB
#define RQ_MRG_BLB 5
#endif
#define RQ_MG_B 512         // merge block: one source per thread (the fast general sweep: <= 512)

struct ScanArgs {
    int64_t n_chunk, chunk0;
    const int64_t* nrows;   // number of pivot rows of replica rl at nrows[(chunk0+rl)*nrows_stride]
    int64_t nrows_stride;
    const int* sall;        // sink columns S of replica rl (chunk-relative)
    int64_t row_stride;
    const double* rows_t;
    const double* rows_sum;
    const uint32_t* rows_valid;
    const uint32_t* rows_cnt;
    double end;
    double* metrics;
    int* wq;                // replica work queue (zeroed before the launch; null = one replica per wave)
};

hipError_t rq_launch_gen(const GenArgs& a, hipStream_t s);
// log: 0 fast tiled sweep, 1 sequential (LOG) sweep, 2 LOG with the per-sink state in
// global memory (SweepArgs.gs)
hipError_t rq_launch_sweep(const SweepArgs& a, int spl, int nK, int col16, int log, int bits, hipStream_t s);
hipError_t rq_launch_scan(const ScanArgs& a, int nK, hipStream_t s);
int rq_sweep_blocks_per_cu(int spl, int nK, int col16, int W, int log, int bits, int wpb, size_t lds);
// spl = 0 in rq_launch_sweep / rq_sweep_blocks_per_cu: the fast sweep reading merged streams
hipError_t rq_launch_merge(const MergeArgs& a, hipStream_t s);
// > RQ_MG_B sources: level 1 over n_grp groups (a.n_str streams, grid C x n_grp), then
// the second level over the groups' sequences (a.sub_*, a.n_grp "streams")
hipError_t rq_launch_merge_groups(const MergeArgs& a, hipStream_t s);
hipError_t rq_launch_merge_sub(const MergeArgs& a, hipStream_t s);
// merged entries carry the stream as u16 (+ a u8 of its high bits past 65535 streams);
// the two-level merge takes up to RQ_MG_B groups of RQ_MG_B streams
#define RQ_MAX_STREAMS_MRG (RQ_MG_B * RQ_MG_B)
// longest-first order of n <= 65536 replicas by len (descending; ties in any order)
hipError_t rq_launch_order(const int* len, int64_t n, int* order, hipStream_t s);
hipError_t rq_launch_sweep_fw(const SweepArgs& a, int nK, int col16, int W, int bits, hipStream_t s);
int rq_fw_blocks_per_cu(int nK, int col16, int W, int bits, int wpb, size_t lds, int pw);
int rq_cu_count();   // CUs of the current device (256 on MI355X when the query fails)

// Blocks per CU a kernel reaches at `threads` threads and `lds` bytes of dynamic LDS
// (the runtime's occupancy: VGPR, SGPR and LDS limits), cached per (kernel, threads,
// lds).  rq_run_batch may be called from several threads at once (rq.h), so the cache
// is mutex-guarded; 0 when the query fails (no device).
template <class K>
int rq_occupancy(K kernel, int threads, size_t lds)
{
    static std::mutex mu;
    static std::map<std::tuple<const void*, int, size_t>, int> cache;
    const auto key = std::make_tuple(reinterpret_cast<const void*>(kernel), threads, lds);
    std::lock_guard<std::mutex> lock(mu);
    const auto it = cache.find(key);
    if (it != cache.end()) return it->second;
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kernel, threads, lds) != hipSuccess) nb = 0;
    cache.emplace(key, nb);
    return nb;
}

// ---- dataframe replay (rq_replay.hip) ----
// per-dataframe status, in the workspace
struct RpInfo {
    int64_t n_piv;            // pivot rows (unique t)
    int64_t n_own, n_world;   // distinct event ids of the source / of the others
    int32_t S;                // unique sink ids (pivot columns)
    int32_t flags;            // RP_*
};
#define RP_FALLBACK 1    // a duplicate (t, sink) pivot cell: the sequential replay owns the df
#define RP_UNSORTED 2    // 't' decreases
#define RP_GLOBAL 4      // more unique sinks than the LDS table: needs the global-table pass
#define RP_EIDBAD 8      // event_id decreases: the event counts are unknown
#define RP_BIG 16        // needs the large workspace (or exceeds it)
#define RP_EMPTYDF 32    // no rows
#define RP_BADOFF 64     // df_off[d] .. df_off[d + 1] is not a valid row range (< 2^31 rows)
#define RP_MID 256       // more unique sinks than the small LDS table: the full-table pass takes it
#define RP_CSKIP 128     // chunked mode: the df is not chunkable (> RC_S sinks, the INT64_MIN id):
                         // the one-workgroup path (rq_rp_fast) takes it
enum { RP_PHASE_FAST = 0, RP_PHASE_GLOBAL = 1, RP_PHASE_KEYS = 2, RP_PHASE_SEQ = 3, RP_PHASE_SCAN = 4,
       RP_PHASE_CHUNK = 5, RP_PHASE_SMALL = 6 };
// chunked replay (one dataframe over many workgroups): rows per chunk, most unique sinks
// per dataframe, hash slots per dataframe
#define RC_L 4096
#define RC_S 4096
#define RC_HT 8192
struct RcCarry {     // one chunk's effect on one sink (rq_rc_sum)
    int n;           // rows of the sink in the chunk
    int after;       // rows after its last own row in the chunk (-1: no own row)
    double last_t;   // t of its last row in the chunk
};
struct RcState {     // a sink's state entering a chunk (rq_rc_scan)
    int r;           // rank of its last row (-1: no row yet, a NaN cell)
    int pad;
    double last_t;   // t of its last row
};

struct RpArgs {
    const double* t;
    const int64_t* src;
    const int64_t* sink;
    const int64_t* eid;       // may be null
    const int64_t* df_off;    // device [n_df + 1], or null: one dataframe of n_rows rows
    int64_t n_df, n_rows;
    int64_t src_id;
    double end;
    int Ks[RQ_MAX_K];
    int nK;
    RpInfo* info;             // [n_df]
    // pivot rows of dataframe d at rows [df_off[d], ...): dt, cell sum, #valid, #<=K-1
    double* rows_dt;
    double* rows_sum;
    uint32_t* rows_valid;
    uint32_t* rows_cnt;       // [row][nK]
    int64_t* keys;            // [n_rows]: sorted unique sink ids of fallback dataframes
    // large workspace only (null otherwise): per-df hash tables, slots [4 r0, 4 r1)
    uint64_t* gkeys;          // [4 n_rows]
    void* gstate;             // [4 n_rows] x 16 B
    double* metrics;          // [n_df][nK + 2]
    int64_t* counts;          // [n_df][4]
    // chunked mode (RP_PHASE_CHUNK; null otherwise): per df chunk prefix [n_df + 1], hash
    // tables [n_df][RC_HT], per chunk the group base, carries / entering states [chunk][RC_S]
    int chunked;
    int first_tier;         // 0: the small-table pass runs first (RP_PHASE_SMALL), 1: the full-table pass
    int64_t max_chunks;
    int64_t* cbase;
    uint64_t* ht_keys;
    int* ht_dense;
    int* gstart;              // [chunk] t-group starts in the chunk
    int64_t* gbase;           // [chunk] t-groups started before the chunk (within its df)
    RcCarry* carry;
    RcState* state;
    unsigned long long* clk;  // RQ_PHASE_CLOCK builds only: rq_rp_fast per-phase s_memtime sums [8]
};
hipError_t rq_launch_rp(const RpArgs& a, int phase, hipStream_t s);

// ---- analysis kernels (rq_analysis.hip) ----
struct OracleArgs {
    const double* w;          // device, concatenated per instance: w[n_i + 2]
    const int64_t* w_off;     // device [n_inst + 1]
    const double* q;          // device [n_inst]
    const double* s;          // device [n_inst]
    int n_inst;
    int64_t n_max;
    double* cost;             // device [n_inst]
    int32_t* events;          // device, concatenated [n_i + 1]
    int32_t* ranks;           // device, concatenated [n_i + 1]
    const int64_t* out_off;   // device [n_inst + 1]
    uint64_t* bits;           // workspace [n_inst][bits_stride]
    int64_t bits_stride;
    double* gcol;             // workspace [n_inst][2][n_max + 2] (global-column mode)
};
hipError_t rq_launch_oracle_dp(const OracleArgs& a, bool lds, hipStream_t s);

struct RankTableArgs {
    const double* t;
    const int64_t* src;
    const int32_t* col;
    int64_t n_rows;
    int n_cols;
    int64_t src_id;
    int fill;
    int64_t n_t;
    double* table;            // [n_t][n_cols]
    double* index;            // [n_t]
    int32_t* err;             // [1]: 1 unsorted t, 2 n_t mismatch
};
hipError_t rq_launch_rank_table(const RankTableArgs& a, hipStream_t s);

struct UIntArgs {
    const double* table;
    const double* index;
    int64_t n_t;
    int n_cols;
    const int32_t* fcol;
    const double* wts;
    int n_f;
    double end;
    double* x;                // workspace [n_t]
    double* out;              // [1]
};
hipError_t rq_launch_u_int(const UIntArgs& a, hipStream_t s);

struct LogArgs {
    const double* ev_t;       // [n_rep][ev_cap]
    const int32_t* ev_src;    // [n_rep][ev_cap] stream indices
    const int64_t* counts;    // [n_rep][4], [2] = events
    int64_t n_rep, ev_cap;
    const int* csr_ptr;       // [n_str + 1]
    const int* csr_col;       // sink columns, edge-list order per stream
    int n_str;
    const int64_t* src_ids;   // [n_str]
    const int64_t* sink_ids;  // [n_sinks] sorted
    double start;
    int64_t* row_off;         // [n_rep + 1]
    int64_t* event_id;
    double* time_delta;
    int64_t* src_id;
    double* t;
    int64_t* sink_id;
};
hipError_t rq_launch_log_rows(const LogArgs& a, hipStream_t s);
hipError_t rq_launch_log_expand(const LogArgs& a, hipStream_t s);
