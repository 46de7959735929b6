// rq_replay.hip -- metrics of dataframes in the reference's row layout, on the
// raw (t, src_id, sink_id[, event_id]) columns, many dataframes per call.
//
// Reference: utils.rank_of_src_in_df (utils.py:38-56) -> time_in_top_k /
// average_rank / int_r_2 (utils.py:84-121) and num_tweets_of (:170-176), on the
// df State.get_dataframe builds (opt_model.py:85-97).  SURVEY.md Appendix B is
// the exact arithmetic (rank scan per sink, pivot on unique t x sorted sink ids
// with the mean of duplicate (t, sink) cells, ffill, numpy pairwise sums).
//
// Kernels (one launch each, every dataframe of the batch in the same launch):
//
//   rq_rp_fast<NK, GLOBAL>   one 1024-thread workgroup per dataframe, rows in
//       batches of 1024 (the next batch's loads are in flight during the current
//       one and staged through LDS at its end).  Sink ids get a dense slot from a
//       hash table (LDS, <= 3071 unique sinks; the GLOBAL instance keeps it in HBM
//       for wider dataframes), so no host-side factorisation is needed.
//       Per batch: every row takes a ticket in its sink's bucket (an LDS atomic on
//       the sink's slot); a sink with several rows in the batch gets a list of them
//       (one allocator atomic for the bucket), and each row scans its sink's list for
//       the rows before it, its predecessor and the latest own rows at / before it,
//       so rank = pos - lastown (utils.py:43-46) for every row at once, with the
//       carried per-sink state (count, last own row, last t-group) from earlier
//       batches.  Each row then contributes the change of its pivot cell
//       (rank - previous rank of that sink; NaN -> value for the first row) to a
//       block scan in row order; at the last row of every t-group the running
//       totals ARE the pivot row (sum of the forward-filled cells, #non-NaN cells,
//       #cells <= K-1).  All of it is integer arithmetic, so it is exact; a pivot
//       row of integral cells sums exactly in any order, which is what numpy's
//       pairwise row sum returns.  A dataframe with two rows of one sink at one t
//       (a pandas pivot MEAN, possibly fractional) is handed to rq_rp_seq.
//   rq_rp_keys       sorted unique sink ids of those dataframes (bitonic sort).
//   rq_rp_seq<NK>    the exact sequential replay (one wavefront per dataframe,
//       pivot-cell means and numpy-pairwise row sums while fractional cells are
//       live) for the dataframes rq_rp_fast handed over.
//   rq_rp_scan<NK>   numpy-order integrals over each dataframe's pivot rows
//       (wave_npsum, rq_device.h) + the per-dataframe counts.
//
// HBM: 24 B per df row read (t f64, src i64, sink i64) + 8 B with event ids;
// pivot rows written once (dt f64, sum f64, #valid u32, #<=K-1 u32 per K) and
// read once by the scan.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "rq_device.h"
#include "rq_internal.h"

#pragma clang fp contract(off)

using namespace rq;

namespace {

#ifndef RQ_RP_B
#define RQ_RP_B 1024
#endif
constexpr int RP_B = RQ_RP_B;           // rows per batch = threads per workgroup
constexpr int RP_W = RP_B / 64;         // waves per workgroup
constexpr int RP_H = 4 * RP_B;          // LDS hash slots
constexpr int RP_LOG_H = RP_B == 1024 ? 12 : RP_B == 512 ? 11 : 10;
constexpr int RP_HMAX = RP_H - RP_B - 1;   // unique sinks the LDS table takes: a batch can
                                           // insert RP_B more and still leave an empty slot
// the small tier: a half-size LDS table (<= RP_B - 1 unique sinks) and <= 64 VGPRs, so two
// workgroups share a CU and one's barriers overlap the other's work; wider dataframes
// (or nK > RP_SMALL_NK) go on to the full table, then the global one
constexpr int RP_HS = 2 * RP_B;
constexpr int RP_LOG_HS = RP_LOG_H - 1;
constexpr int RP_HMAX_S = RP_HS - RP_B - 1;
constexpr int RP_SMALL_NK = 1;
// rq_rp_fast rows per thread: where a workgroup has its CU to itself (no more dataframes
// than CUs: RQ_RP_RFEW with the small table, 2 with the full one, whose LDS never shares
// its CU), else 1 (two small-table workgroups per CU).  256 C3 dataframes: 4.35 ms at 1
// row per thread, 3.76 at 2, 3.62 at 3 (scripts/bench_paths.py replay_batch); since the
// per-wave list allocator (round 5) 2.79 ms at 3, 2.645 at 2
#ifndef RQ_RP_RFEW
#define RQ_RP_RFEW 2
#endif
// the list walk reads two entries of each list per wait up to this many rows per thread
// (256 C3 dataframes at 2 rows per thread: 2.645 -> 2.62 ms)
#ifndef RQ_RP_KU2_MAXR
#define RQ_RP_KU2_MAXR 2
#endif
constexpr int RP_RFEW = RQ_RP_RFEW;   // the small table's rows per thread, one workgroup per CU
// the bucket word of a sink: rows of it in this batch (low RP_BB bits), list offset (next)
constexpr int RP_BB = RP_RFEW * RP_B < 4096 ? 12 : 13;
constexpr int RP_BM = (1 << RP_BB) - 1;
static_assert(RP_RFEW * RP_B < (1 << RP_BB) && RP_B * 2 < (1 << RP_BB) && 2 * RP_BB <= 30,
              "bucket fields");
constexpr uint64_t RP_EMPTY_KEY = 0x8000000000000000ull;   // INT64_MIN: gets its own slot

struct alignas(16) RpSlot {
    int cnt;        // rows of this sink so far (pos of its last row; 0: none yet, cell NaN)
    int lastown;    // pos of its latest own row (0: none); its last row's rank = cnt - lastown
    int lastgroup;  // t-group of its last row (-1: none)
    int bucket;     // this batch: rows of the sink (bits 0-11), list offset (bits 12-23)
};

__device__ __forceinline__ uint32_t rp_hash(uint64_t k, int bits)
{
    return (uint32_t)((k * 0x9E3779B97F4A7C15ull) >> (64 - bits));
}

// open addressing, linear probing; returns the slot of key k (inserting it).  A full
// table (only possible once more sinks than the tier takes arrive in one batch) sets
// *full and returns the sentinel slot mask + 1: the caller's tier gives the dataframe up.
__device__ __forceinline__ uint32_t rp_insert(unsigned long long* keys, uint32_t mask, int bits,
                                              uint64_t k, int* count, int* full)
{
    uint32_t h = rp_hash(k, bits);
    for (uint32_t p = 0; p <= mask; ++p) {
        const unsigned long long cur = keys[h];
        if (cur == k) return h;
        if (cur == RP_EMPTY_KEY) {
            const unsigned long long old = atomicCAS(&keys[h], (unsigned long long)RP_EMPTY_KEY,
                                                     (unsigned long long)k);
            if (old == RP_EMPTY_KEY) {
                atomicAdd(count, 1);
                return h;
            }
            if (old == k) return h;
        }
        h = (h + 1) & mask;
    }
    *full = 1;
    return mask + 1;
}

__device__ __forceinline__ int64_t df_begin(const RpArgs& a, int64_t d) { return a.df_off ? a.df_off[d] : 0; }
__device__ __forceinline__ int64_t df_end(const RpArgs& a, int64_t d) { return a.df_off ? a.df_off[d + 1] : a.n_rows; }

// global-table capacity of a dataframe of n rows: a power of two >= 2n, <= 2^24
// (its region in the large workspace is slots [4 r0, 4 r1), so it never overlaps)
__device__ __forceinline__ int rp_gbits(int64_t n)
{
    int b = 1;
    while (b < 24 && ((int64_t)1 << b) < 2 * n) ++b;
    return b;
}

// ---- wave scans on DPP (VALU latency; ds_bpermute shuffles cost ~100 cycles a step
// and these chains are the batch's critical path) ----
// inclusive 64-lane sum of 32-bit values (two's complement wrap, so int works too)
__device__ __forceinline__ int scan_add_i32(int v) { return (int)wave_scan_add((uint32_t)v); }
// inclusive 64-lane sum of int32 values as int64 (16-bit halves scanned apart: exact)
__device__ __forceinline__ int64_t scan_add_i64_of_i32(int v)
{
    const int hi = scan_add_i32(v >> 16);
    const int lo = scan_add_i32(v & 0xFFFF);
    return (int64_t)hi * 65536 + (int64_t)lo;
}
// inclusive 64-lane sum of int64 values of magnitude < 2^47 (16-bit low halves and
// the high parts scanned apart: exact)
__device__ __forceinline__ int64_t scan_add_i64_small(int64_t v)
{
    const int hi = scan_add_i32((int)(v >> 16));
    const int lo = scan_add_i32((int)(v & 0xFFFF));
    return (int64_t)hi * 65536 + (int64_t)lo;
}
// 16-lane (row 0) inclusive scans of the wave totals
__device__ __forceinline__ int row_scan_add(int v)
{
    uint32_t x = (uint32_t)v;
    x += dpp0<0x111, 0xF>(x);
    x += dpp0<0x112, 0xF>(x);
    x += dpp0<0x114, 0xF>(x);
    x += dpp0<0x118, 0xF>(x);
    return (int)x;
}
__device__ __forceinline__ int64_t row_scan_add(int64_t v)
{
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t lo = (uint32_t)v, hi = (uint32_t)((uint64_t)v >> 32);
        uint32_t plo, phi;
        switch (k) {
        case 0: plo = dpp0<0x111, 0xF>(lo); phi = dpp0<0x111, 0xF>(hi); break;
        case 1: plo = dpp0<0x112, 0xF>(lo); phi = dpp0<0x112, 0xF>(hi); break;
        case 2: plo = dpp0<0x114, 0xF>(lo); phi = dpp0<0x114, 0xF>(hi); break;
        default: plo = dpp0<0x118, 0xF>(lo); phi = dpp0<0x118, 0xF>(hi); break;
        }
        v += (int64_t)(((uint64_t)phi << 32) | plo);
    }
    return v;
}

__device__ __forceinline__ int lane_bcast(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ int64_t lane_bcast(int64_t v, int l) { return bcast_i64(v, l); }

// the 16 wave totals t[0..16) (LDS) of a block scan -> this wave's exclusive
// prefix and the block total (w: this wave, uniform)
template <class T>
__device__ __forceinline__ void totals_add(const T* t, int w, T& pre, T& tot)
{
    T x = lane_id() < RP_W ? t[lane_id()] : (T)0;
    x = row_scan_add(x);
    tot = lane_bcast(x, RP_W - 1);
    pre = w > 0 ? lane_bcast(x, w - 1) : (T)0;
}
template <int NK>
struct RpAcc {
    int64_t s;      // sum of the (integral) forward-filled pivot cells
    int v;          // non-NaN cells
    int c[NK];      // cells <= K-1
};

}  // namespace

// ============================================================================
// rq_rp_fast: one workgroup per dataframe
// ============================================================================
// TIER 0: small LDS table (first pass), 1: full LDS table (the dataframes tier 0 gave up:
// RP_MID), 2: global table (those tier 1 gave up: RP_GLOBAL).  A batch is R * RP_B rows:
// thread tid owns rows tid * R .. tid * R + R - 1 (row order within the thread, so every
// block scan runs over per-thread partial sums: one barrier set per R * RP_B rows).
template <int NK, int TIER, int R>
__device__ __forceinline__ void rp_fast_body(RpArgs a)
{
    constexpr bool GLOBAL = TIER == 2;
    constexpr int BR = R * RP_B;
    const int64_t d = blockIdx.x;
    const int tid = threadIdx.x;
    const int lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
    RpInfo* inf = a.info + d;
    if (GLOBAL && !(inf->flags & RP_GLOBAL)) return;   // only the dataframes the LDS pass gave up
    if (TIER == 1 && a.first_tier == 0 && !(inf->flags & RP_MID)) return;   // ... the small pass gave up
    if (TIER == a.first_tier && a.chunked && !(inf->flags & RP_CSKIP)) return;   // the chunked pass took it
    const int64_t r0 = df_begin(a, d), r1 = df_end(a, d);
    const int64_t nd = r1 - r0;
    // a malformed caller range (decreasing / negative offsets, past n_rows, >= 2^31 rows:
    // the row positions below are int) touches no workspace; rq_rp_scan reports RQ_EINVAL
    if (r0 < 0 || r1 < r0 || r1 > a.n_rows || nd >= ((int64_t)1 << 31)) {
        if (TIER == a.first_tier && tid == 0) {
            inf->flags = RP_BADOFF;
            inf->n_piv = 0;
            inf->n_own = 0;
            inf->n_world = 0;
            inf->S = 0;
        }
        return;
    }

    extern __shared__ __align__(16) unsigned char rp_smem[];
    unsigned char* sp = rp_smem;
    auto carve = [&](size_t bytes) {
        unsigned char* p = sp;
        sp += (bytes + 15) & ~(size_t)15;
        return p;
    };
    double* tb = reinterpret_cast<double*>(carve(8 * (BR + 2)));         // [0] prev, [1+i], [BR+1] next
    int64_t* eb = reinterpret_cast<int64_t*>(carve(8 * (BR + 1)));       // [0] prev eid, [1+i]
    int* gb = reinterpret_cast<int*>(carve(4 * BR));                      // t-group of row i
    int* lst = reinterpret_cast<int*>(carve(4 * BR));                     // sink buckets: 2 row + own
    int64_t* wsum = reinterpret_cast<int64_t*>(carve(8 * 16));            // wave totals (int64)
    int* ws32 = reinterpret_cast<int*>(carve(4 * 16 * (NK + 6)));         // wave totals (int)
    int* misc = reinterpret_cast<int*>(carve(4 * 16));                    // flags, counters
    unsigned long long* tkeys;
    RpSlot* tst;
    uint32_t tmask;
    int tbits;
    int64_t tcap;
    if constexpr (GLOBAL) {
        tbits = rp_gbits(nd);
        tcap = (int64_t)1 << tbits;
        tkeys = reinterpret_cast<unsigned long long*>(a.gkeys) + 4 * r0;
        tst = reinterpret_cast<RpSlot*>(a.gstate) + 4 * r0;
    } else {
        constexpr int H = TIER == 0 ? RP_HS : RP_H;
        tbits = TIER == 0 ? RP_LOG_HS : RP_LOG_H;
        tcap = H;
        tkeys = reinterpret_cast<unsigned long long*>(carve(8 * (H + 1)));
        tst = reinterpret_cast<RpSlot*>(carve(sizeof(RpSlot) * (H + 1)));
    }
    tmask = (uint32_t)(tcap - 1);
    // misc: [0] unique sinks, [1] sentinel-key seen, [2] dup, [3] unsorted, [4] eid bad,
    //       [5] own events, [6] world events, [7] key dump cursor, [8] bucket allocator,
    //       [9] table full (a batch's new sinks found no empty slot: this tier gives up)
    if (tid < 16) misc[tid] = 0;
    if (TIER == a.first_tier && tid == 0) inf->flags = 0;   // this call's status (the first pass)
    for (int64_t h = tid; h <= tcap; h += RP_B) {
        tkeys[h] = RP_EMPTY_KEY;
        tst[h] = RpSlot{0, 0, -1, 0};
    }
    if (GLOBAL && 2 * nd > tcap) {   // > 2^23 unique sinks possible: not supported
        if (tid == 0) atomicOr(&inf->flags, RP_BIG);
        return;
    }
    if (GLOBAL) __threadfence();   // the table's reset reaches L2 before the atomics below
    __syncthreads();

    // the bucket word of a sink: LDS atomics, or (global table) atomics at L2 for every
    // access -- the CU's L1 may hold a stale copy of a line an atomic changed
    auto bk_add = [&](RpSlot* p) { return atomicAdd(&p->bucket, 1); };
    auto bk_read = [&](RpSlot* p) { return GLOBAL ? atomicOr(&p->bucket, 0) : p->bucket; };
    auto bk_write = [&](RpSlot* p, int v) {
        if (GLOBAL) atomicExch(&p->bucket, v); else p->bucket = v;
    };

    int km1[NK];
#pragma unroll
    for (int q = 0; q < NK; ++q) km1[q] = a.Ks[q] - 1;
    const bool has_eid = a.eid != nullptr;

#ifdef RQ_PHASE_CLOCK
    // diagnostic builds: per-wave s_memtime per phase of the batch loop (RQ_CLK_REPLAY)
    unsigned long long ck[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long tk = __builtin_amdgcn_s_memtime();
#define RP_CLK(q)                                                   \
    do {                                                            \
        const unsigned long long t2 = __builtin_amdgcn_s_memtime(); \
        ck[q] += t2 - tk;                                           \
        tk = t2;                                                    \
    } while (0)
#else
#define RP_CLK(q) \
    do {          \
    } while (0)
#endif
    // carries across batches
    int64_t Gc = 0;        // t-groups started so far
    RpAcc<NK> carry;
    carry.s = 0;
    carry.v = 0;
#pragma unroll
    for (int q = 0; q < NK; ++q) carry.c[q] = 0;
    bool aborted = false;

    // A batch's rows reach the workgroup through LDS: the loads for batch b + 1 are
    // issued at the top of batch b and consumed only at its end (prep), so they are
    // in flight across its barriers and nothing loaded is carried over the loop's
    // back edge (the waitcnt pass would otherwise wait for them early).
    //   tb[0] = t of the previous batch's last row, tb[1 + i] = row i, tb[BR + 1] =
    //   t of the first row of the following batch; eb likewise for event ids.
    bool own_c[R];       // this thread's rows of the current batch: own posts?
    uint32_t slot_c[R];  // ... their sinks' slots
    auto load = [&](int64_t nb0, double (&t_)[R], int64_t (&s_)[R], int64_t (&k_)[R],
                    int64_t (&e_)[R]) __attribute__((always_inline)) {
        // unconditional loads at a clamped row (prep masks the rows past r1): no
        // exec-masked zeroing of the destinations, whose write-after-write wait on the
        // previous batch's loads stalled the loop top
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int64_t ii = nb0 + tid * R + r;
            const int64_t ic = ii < r1 ? ii : r1 - 1;   // nd > 0 (the caller checks)
            t_[r] = a.t[ic];
            s_[r] = a.src[ic];
            k_[r] = a.sink[ic];
            e_[r] = has_eid ? a.eid[ic] : 0;
        }
    };
    auto prep = [&](int64_t nb0, const double (&t_)[R], const int64_t (&s_)[R], const int64_t (&k_)[R],
                    const int64_t (&e_)[R], double t_after, double t_before,
                    int64_t e_before) __attribute__((always_inline)) {
        if (tid == 0) {
            tb[0] = t_before;
            eb[0] = e_before;
            tb[BR + 1] = t_after;
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int row = tid * R + r;
            const bool v = nb0 + row < r1;
            tb[1 + row] = v ? t_[r] : 0.0;
            if (has_eid) eb[1 + row] = e_[r];
            own_c[r] = v && s_[r] == a.src_id;
            slot_c[r] = 0;
            if (v) {
                if ((uint64_t)k_[r] == RP_EMPTY_KEY) {
                    slot_c[r] = (uint32_t)tcap;   // the sentinel id's own slot
                    if (misc[1] == 0 && atomicExch(&misc[1], 1) == 0) atomicAdd(&misc[0], 1);
                } else {
                    slot_c[r] = rp_insert(tkeys, tmask, tbits, (uint64_t)k_[r], &misc[0], &misc[9]);
                }
            }
        }
    };
    // the next batch's rows: loaded in the middle of the batch before (after its prep,
    // before its pivot-row stores, so the loop top issues no loads behind fresh stores --
    // vmcnt retires in issue order), consumed by this batch's prep
    double tn[R];
    int64_t sn[R], kn[R], en[R];
    double tnn = 0.0;   // the t right after the next batch
    if (nd > 0) {
        double t0[R];
        int64_t s0[R], k0[R], e0[R];
        load(r0, t0, s0, k0, e0);
        double ta = 0.0;
        if (tid == 0 && r0 + BR < r1) ta = a.t[r0 + BR];
        prep(r0, t0, s0, k0, e0, ta, 0.0, 0);
        load(r0 + BR, tn, sn, kn, en);
        if (tid == 0 && r0 + 2 * BR < r1) tnn = a.t[r0 + 2 * BR];
    }

    for (int64_t b0 = r0; b0 < r1; b0 += BR) {

        // ---- A: neighbours of every row; its ticket in its sink's bucket ----
        __syncthreads();
        RP_CLK(0);   // loop top, barrier 1
        const int last = (int)((r1 - b0) < BR ? (r1 - b0) : BR);
        const double t_last = tb[last];
        const int64_t e_last = has_eid ? eb[last] : 0;
        bool valid[R], start[R], endg[R];
        double ti[R], tnx[R];
        int ticket[R];
        int st_loc = 0, evo = 0, evw = 0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int row = tid * R + r;
            const int64_t i = b0 + row;
            valid[r] = i < r1;
            ti[r] = tb[1 + row];
            const double t_prev = tb[row];
            tnx[r] = tb[row + 2];
            const bool first_row = i == r0;
            start[r] = valid[r] && (first_row || ti[r] != t_prev);
            endg[r] = valid[r] && (i == r1 - 1 || tnx[r] != ti[r]);
            ticket[r] = valid[r] ? bk_add(tst + slot_c[r]) : 0;   // rows of this sink before me: unordered
            if (valid[r] && !first_row && ti[r] < t_prev) misc[3] = 1;
            if (has_eid && valid[r]) {
                const int64_t ei = eb[1 + row], e_prev = eb[row];
                const bool fe = first_row || ei != e_prev;
                if (!first_row && ei < e_prev) misc[4] = 1;
                evo += fe && own_c[r];
                evw += fe && !own_c[r];
            }
            st_loc += start[r];
        }
        if (!GLOBAL && (misc[0] > (TIER == 0 ? RP_HMAX_S : RP_HMAX) || misc[9]))
            aborted = true;   // uniform: read after the barrier

        // ---- B: t-group of every row (block scan of group starts) + event counts;
        //      buckets of more than one row get list space ----
        const int st_incl = scan_add_i32(st_loc);
        int nbo = 0, nbw = 0;
        if (has_eid) {
            nbo = scan_add_i32(evo);
            nbw = scan_add_i32(evw);
        }
        if (lane == 63) {
            ws32[w] = st_incl;
            ws32[16 + w] = nbo;
            ws32[32 + w] = nbw;
        }
        RP_CLK(2);   // A: neighbours, tickets, group-start scan
        __syncthreads();
        if (aborted) break;
        int st_pre, st_tot, n_ev_own, n_ev_world, dummy;
        totals_add(ws32, w, st_pre, st_tot);
        totals_add(ws32 + 16, w, dummy, n_ev_own);
        totals_add(ws32 + 32, w, dummy, n_ev_world);
        int64_t G[R];   // each row's t-group (pivot row index)
        {
            int64_t g = Gc + (int64_t)(st_pre + st_incl - st_loc) - 1;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                g += start[r];
                G[r] = g;
                gb[tid * R + r] = (int)g;
            }
        }
        RpSlot st0[R];   // state before this batch
        int m[R];        // rows of the row's sink in this batch
        int need = 0;    // list space of this thread's ticket-0 rows of sinks with > 1 row
#pragma unroll
        for (int r = 0; r < R; ++r) {
            RpSlot* sl = tst + slot_c[r];
            st0[r] = valid[r] ? *sl : RpSlot{0, 0, -1, 0};
            // (low bits: the ticket-0 row may already have added the list offset)
            m[r] = valid[r] ? ((GLOBAL ? bk_read(sl) : st0[r].bucket) & RP_BM) : 0;
            need += (valid[r] && m[r] > 1 && ticket[r] == 0) ? m[r] : 0;
        }
        {   // one allocator atomic per wave (a wave-wide scan places the lists)
            const int incl = scan_add_i32(need);
            int wb = 0;
            if (lane == 63 && incl > 0) wb = atomicAdd(&misc[8], incl);
            int off = __builtin_amdgcn_readlane(wb, 63) + incl - need;
#pragma unroll
            for (int r = 0; r < R; ++r)
                if (valid[r] && m[r] > 1 && ticket[r] == 0) {
                    bk_write(tst + slot_c[r], (off << RP_BB) | m[r]);
                    off += m[r];
                }
        }
        RP_CLK(3);   // barrier 2, B: totals, groups, states, list space
        __syncthreads();

        // ---- C: each row's place among its sink's rows in this batch ----
        int boff[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            boff[r] = 0;
            if (valid[r] && m[r] > 1) {
                boff[r] = bk_read(tst + slot_c[r]) >> RP_BB;
                lst[boff[r] + ticket[r]] = 2 * (tid * R + r) + (own_c[r] ? 1 : 0);   // row, own flag
            }
        }
        __syncthreads();
        RP_CLK(3);   // barrier 3, list placement, barrier 4
        int xs[R], xv[R], xc[R][NK];
        // j: my sink's rows before me; pred: the last of them; own_le / own_lt: its latest
        // own row at or before / before me (rows in batch order).  The R rows' lists are
        // walked side by side, so each step has R independent LDS reads in flight.
        int jj[R], pred_[R], ole[R], olt[R], mm[R];
        int mmax = 0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            jj[r] = 0;
            pred_[r] = -1;
            ole[r] = own_c[r] ? tid * R + r : -1;
            olt[r] = -1;
            mm[r] = valid[r] && m[r] > 1 ? m[r] : 0;
            mmax = mmax > mm[r] ? mmax : mm[r];
        }
        auto visit = [&](int r, int v) __attribute__((always_inline)) {
            const int y = v >> 1;
            if (y < tid * R + r) {
                ++jj[r];
                pred_[r] = pred_[r] > y ? pred_[r] : y;
                if (v & 1) {
                    olt[r] = olt[r] > y ? olt[r] : y;
                    ole[r] = ole[r] > y ? ole[r] : y;
                }
            }
        };
        // one or two rows per thread: two entries of each list per LDS wait (1024 C3
        // dataframes 8.82 -> 8.35 ms); three rows: their three reads share each wait
        constexpr int KU = R <= RQ_RP_KU2_MAXR ? 2 : 1;
        for (int k = 0; k < mmax; k += KU) {
            int v[KU][R];
#pragma unroll
            for (int u = 0; u < KU; ++u)
#pragma unroll
                for (int r = 0; r < R; ++r) v[u][r] = k + u < mm[r] ? lst[boff[r] + k + u] : 0x7FFFFFFF;
#pragma unroll
            for (int u = 0; u < KU; ++u)
#pragma unroll
                for (int r = 0; r < R; ++r) visit(r, v[u][r]);
        }
        RP_CLK(1);   // C1: the list walk
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int j = jj[r], pred = pred_[r], own_le = ole[r], own_lt = olt[r];
            int j_le = 0, j_lt = 0;   // positions of own_le / own_lt among the bucket
            if (mm[r] > 0 && (own_le >= 0 || own_lt >= 0)) {
                for (int k = 0; k < mm[r]; ++k) {
                    const int y = lst[boff[r] + k] >> 1;
                    j_le += y < own_le;
                    j_lt += y < own_lt;
                }
            } else if (own_le >= 0) {
                j_le = j;   // own_le == row
            }
            xs[r] = 0;
            xv[r] = 0;
#pragma unroll
            for (int q = 0; q < NK; ++q) xc[r][q] = 0;
            if (valid[r]) {
                const RpSlot s0 = st0[r];
                const int pos = s0.cnt + j + 1;
                const int lastown = own_le >= 0 ? s0.cnt + j_le + 1 : s0.lastown;
                const int rank = pos - lastown;
                int prevrank, prevg;
                if (j > 0) {
                    prevrank = (pos - 1) - (own_lt >= 0 ? s0.cnt + j_lt + 1 : s0.lastown);
                    prevg = gb[pred];
                } else {
                    prevrank = s0.cnt > 0 ? s0.cnt - s0.lastown : -1;
                    prevg = s0.lastgroup;
                }
                if (prevg == (int)G[r]) misc[2] = 1;   // two rows of one sink at one t: a pivot mean
                const bool pnan = prevrank < 0;
                xs[r] = rank - (pnan ? 0 : prevrank);
                xv[r] = pnan ? 1 : 0;
#pragma unroll
                for (int q = 0; q < NK; ++q)
                    xc[r][q] = (rank <= km1[q] ? 1 : 0) - ((!pnan && prevrank <= km1[q]) ? 1 : 0);
                if (j == m[r] - 1) {   // my sink's last row of this batch carries its state on
                    RpSlot* sl = tst + slot_c[r];
                    sl->cnt = pos;
                    sl->lastown = lastown;
                    sl->lastgroup = (int)G[r];
                    bk_write(sl, 0);
                }
            }
        }

        // the next batch's rows (their loads have landed by now) into LDS, sinks hashed
        // (tb / eb were last read in A, two barriers ago)
        RP_CLK(5);   // C2: own-row positions, ranks, carried states
        // (unconditional: after the last batch it only writes LDS nobody reads; a skipped
        // prep left the loads' registers pending on the back edge, and the loop top
        // waited on them -- vmcnt(0) between each row's loads)
        prep(b0 + BR, tn, sn, kn, en, tnn, t_last, e_last);
        // the batch after next (in flight across the next batch's barriers)
        load(b0 + 2 * BR, tn, sn, kn, en);
        tnn = 0.0;
        if (tid == 0 && b0 + 3 * BR < r1) tnn = a.t[b0 + 3 * BR];
        RP_CLK(6);   // next batch into LDS + its hash inserts, the one after issued

        // ---- D: running totals in row order; the last row of a t-group emits its pivot row ----
        // this thread's rows: inclusive prefixes in registers; the threads' totals are
        // block-scanned (|a row's change| < 2^31, so R rows' sum < 2^47: two 32-bit scans)
        int64_t ls = 0;
        int lv = 0, lc[NK];
#pragma unroll
        for (int q = 0; q < NK; ++q) lc[q] = 0;
        int64_t ps[R];
        int pv[R], pc[R][NK];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            ls += xs[r];
            lv += xv[r];
            ps[r] = ls;
            pv[r] = lv;
#pragma unroll
            for (int q = 0; q < NK; ++q) {
                lc[q] += xc[r][q];
                pc[r][q] = lc[q];
            }
        }
        RpAcc<NK> x;   // inclusive over the wave's threads
        x.s = scan_add_i64_small(ls);
        x.v = scan_add_i32(lv);
#pragma unroll
        for (int q = 0; q < NK; ++q) x.c[q] = scan_add_i32(lc[q]);
        if (lane == 63) {
            wsum[w] = x.s;
            ws32[80 + w] = x.v;
#pragma unroll
            for (int q = 0; q < NK; ++q) ws32[96 + 16 * q + w] = x.c[q];
        }
        RP_CLK(4);   // D1: running-total scans
        __syncthreads();
        RpAcc<NK> pre, tot;
        totals_add(wsum, w, pre.s, tot.s);
        totals_add(ws32 + 80, w, pre.v, tot.v);
#pragma unroll
        for (int q = 0; q < NK; ++q) totals_add(ws32 + 96 + 16 * q, w, pre.c[q], tot.c[q]);
        // this thread's exclusive base: carry + earlier waves + earlier lanes
        const int64_t bs = carry.s + pre.s + (x.s - ls);
        const int bv = carry.v + pre.v + (x.v - lv);
        int bc[NK];
#pragma unroll
        for (int q = 0; q < NK; ++q) bc[q] = carry.c[q] + pre.c[q] + (x.c[q] - lc[q]);
#pragma unroll
        for (int r = 0; r < R; ++r) {
#ifdef RQ_RP_NOSTORE   // diagnostic only: the stores stay in the code but never run
            if (endg[r] && a.n_df < 0) {
#else
            if (endg[r]) {
#endif
                const int64_t i = b0 + tid * R + r;
                const int64_t row = r0 + G[r];
                a.rows_dt[row] = (i == r1 - 1 ? a.end : tnx[r]) - ti[r];
                a.rows_sum[row] = (double)(bs + ps[r]);
                a.rows_valid[row] = (uint32_t)(bv + pv[r]);
#pragma unroll
                for (int q = 0; q < NK; ++q) a.rows_cnt[row * NK + q] = (uint32_t)(bc[q] + pc[r][q]);
            }
        }
        carry.s += tot.s;
        carry.v += tot.v;
#pragma unroll
        for (int q = 0; q < NK; ++q) carry.c[q] += tot.c[q];
        Gc += st_tot;
        if (tid == 0) {
            misc[5] += n_ev_own;
            misc[6] += n_ev_world;
            misc[8] = 0;   // bucket allocator (read in B, two barriers ago)
        }
        RP_CLK(7);   // D2: barrier 5, block totals, pivot-row stores
        if (misc[3]) break;   // unsorted (set in A, read after barriers): the df is rejected
    }
#ifdef RQ_PHASE_CLOCK
    if (lane == 0 && a.clk)
        for (int q = 0; q < 8; ++q) atomicAdd(&a.clk[q], ck[q]);
#endif
#undef RP_CLK

    __syncthreads();
    if (aborted) {
        if (tid == 0) atomicOr(&inf->flags, TIER == 0 ? RP_MID : RP_GLOBAL);
        return;
    }
    const int S = misc[0];
    const bool dup = misc[2] != 0;
    if (tid == 0) {
        inf->n_piv = Gc;
        inf->S = S;
        inf->n_own = misc[5];
        inf->n_world = misc[6];
        int fl = 0;
        if (dup) fl |= RP_FALLBACK;
        if (misc[3]) fl |= RP_UNSORTED;
        if (misc[4]) fl |= RP_EIDBAD;
        if (nd == 0) fl |= RP_EMPTYDF;
        inf->flags = fl;   // clears RP_GLOBAL after the global pass
    }
    // the sequential replay needs this dataframe's sorted unique sink ids: dump them
    if (dup && !misc[3]) {
        if (tid == 0) misc[7] = 0;
        __syncthreads();
        for (int64_t h = tid; h <= tcap; h += RP_B) {
            const unsigned long long k = tkeys[h];
            const bool occ = h < tcap ? k != RP_EMPTY_KEY : misc[1] != 0;
            if (occ) {
                const int at = atomicAdd(&misc[7], 1);
                a.keys[r0 + at] = h < tcap ? (int64_t)k : (int64_t)RP_EMPTY_KEY;
            }
        }
    }
}

template <int NK, bool GLOBAL, int R>
__global__ __launch_bounds__(RP_B) void rq_rp_fast(RpArgs a)
{
    rp_fast_body<NK, GLOBAL ? 2 : 1, R>(a);
}
// R == 1: <= 64 VGPRs so two workgroups (half-size tables) share a CU
template <int NK, int R>
__global__ __launch_bounds__(RP_B) __attribute__((amdgpu_waves_per_eu(R == 1 ? 8 : 4, R == 1 ? 8 : 4))) void rq_rp_fast_s(RpArgs a)
{
    rp_fast_body<NK, 0, R>(a);
}

// ============================================================================
// rq_rp_keys: sort the unique sink ids of every fallback dataframe (ascending,
// the pivot_table column order).  Bitonic over the next power of two, in LDS up
// to 8192 keys, else in the large workspace's table region.
// ============================================================================
constexpr int RP_KEYS_LDS = 8192;

__global__ __launch_bounds__(RP_B) void rq_rp_keys(RpArgs a)
{
    const int64_t d = blockIdx.x;
    RpInfo* inf = a.info + d;
    const int fl = inf->flags;
    if (!(fl & RP_FALLBACK) || (fl & (RP_UNSORTED | RP_GLOBAL | RP_BIG))) return;
    const int64_t r0 = df_begin(a, d);
    const int S = inf->S;
    int64_t* keys = a.keys + r0;
    int n2 = 1;
    while (n2 < S) n2 <<= 1;
    __shared__ int64_t lds[RP_KEYS_LDS];
    int64_t* buf = lds;
    if (n2 > RP_KEYS_LDS) {
        if (!a.gkeys) {
            if (threadIdx.x == 0) atomicOr(&inf->flags, RP_BIG);
            return;
        }
        buf = reinterpret_cast<int64_t*>(a.gkeys) + 4 * r0;   // this df's table region (>= 2 S)
    }
    for (int k = threadIdx.x; k < n2; k += RP_B) buf[k] = k < S ? keys[k] : INT64_MAX;
    __syncthreads();
    for (int k = 2; k <= n2; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int x = threadIdx.x; x < n2; x += RP_B) {
                const int y = x ^ j;
                if (y > x) {
                    const int64_t u = buf[x], v = buf[y];
                    const bool up = (x & k) == 0;
                    if ((u > v) == up) {
                        buf[x] = v;
                        buf[y] = u;
                    }
                }
            }
            __syncthreads();
        }
    }
    for (int k = threadIdx.x; k < S; k += RP_B) keys[k] = buf[k];
}

// ============================================================================
// rq_rp_seq: the exact sequential replay of one dataframe per wavefront, for
// the dataframes with pivot means (duplicate (t, sink) rows).  Per-sink state in
// LDS when it fits (40 B per sink), else in the large workspace.
// ============================================================================
constexpr size_t RP_SEQ_LDS = 120 * 1024;

template <int NK>
__global__ __launch_bounds__(64) void rq_rp_seq(RpArgs a)
{
    const int64_t d = blockIdx.x;
    RpInfo* inf = a.info + d;
    const int fl = inf->flags;
    if (!(fl & RP_FALLBACK) || (fl & (RP_UNSORTED | RP_GLOBAL | RP_BIG))) return;
    extern __shared__ double lds_rp[];
    const int lane = lane_id();
    const int64_t r0 = df_begin(a, d), r1 = df_end(a, d);
    const int64_t n_rows = r1 - r0;
    const int S = inf->S;
    const int64_t* keys = a.keys + r0;
    const double* T = a.t + r0;
    const int64_t* SRC = a.src + r0;
    const int64_t* SNK = a.sink + r0;

    // per-sink state
    char* base;
    if ((size_t)S * 40 <= RP_SEQ_LDS) {
        base = reinterpret_cast<char*>(lds_rp + npsum_lds_doubles<1>());
    } else {
        if (!a.gstate) {
            if (lane == 0) atomicOr(&inf->flags, RP_BIG);
            return;
        }
        base = reinterpret_cast<char*>(a.gstate) + (size_t)64 * r0;   // the df's state region (64 B/row)
    }
    double* cell = reinterpret_cast<double*>(base);
    double* gsum = cell + S;
    int* pos = reinterpret_cast<int*>(gsum + S);
    int* last = pos + S;
    int* gtag = pos + 2 * S;
    int* gcnt = pos + 3 * S;
    int* ctag = pos + 4 * S;
    int* touched = pos + 5 * S;
    for (int c = lane; c < S; c += 64) {
        pos[c] = 0;
        last[c] = 0;
        gtag[c] = -1;
        gcnt[c] = 0;
        ctag[c] = 0x7fffffff;
        cell[c] = __builtin_nan("");
        gsum[c] = 0.0;
    }
    __threadfence_block();
    __builtin_amdgcn_wave_barrier();

    int km1[NK];
#pragma unroll
    for (int q = 0; q < NK; ++q) km1[q] = a.Ks[q] - 1;
    int64_t sum_int = 0;       // sum of the integral live cells
    int nfrac = 0;             // live cells with a fractional value
    int nvalid = 0;
    int cnt[NK];
#pragma unroll
    for (int q = 0; q < NK; ++q) cnt[q] = 0;
    int ntouch = 0;            // touched sinks of the open t-group
    int group = 0;
    double gt = 0.0;           // t of the open group
    bool open = false;

    // pivot rows: t staged per lane, stored 64 at a time; converted to dt at the end
    double r_t = 0.0, r_sum = 0.0;
    int r_valid = 0, r_cnt[NK];
#pragma unroll
    for (int q = 0; q < NK; ++q) r_cnt[q] = 0;
    int64_t nrow = 0;
    double* lds = lds_rp;   // wave_npsum scratch
    double* R_t = a.rows_dt + r0;
    double* R_s = a.rows_sum + r0;
    uint32_t* R_v = a.rows_valid + r0;
    uint32_t* R_c = a.rows_cnt + r0 * NK;

    auto store_row = [&](int64_t rr) {
        R_t[rr] = r_t;
        R_s[rr] = r_sum;
        R_v[rr] = (uint32_t)r_valid;
#pragma unroll
        for (int q = 0; q < NK; ++q) R_c[rr * NK + q] = (uint32_t)r_cnt[q];
    };

    // close the open t-group: new cells = mean of the group's ranks per sink
    auto finalize = [&]() {
        int64_t dsum = 0;
        int dfrac = 0, dvalid = 0;
        int dle[NK];
#pragma unroll
        for (int q = 0; q < NK; ++q) dle[q] = 0;
        for (int b = 0; b < ntouch; b += 64) {
            const int k = b + lane;
            const bool act = k < ntouch;
            double nw = 0.0, od = 0.0;
            if (act) {
                const int c = touched[k];
                nw = gsum[c] / (double)gcnt[c];
                od = cell[c];
                cell[c] = nw;
                gsum[c] = 0.0;
                gcnt[c] = 0;
            }
            const bool onan = act && od != od;
            const bool ofr = act && !onan && od != __builtin_floor(od);
            const bool nfr = act && nw != __builtin_floor(nw);
            dvalid += popc(__ballot(onan));
            dfrac += popc(__ballot(nfr)) - popc(__ballot(ofr));
            int64_t dv = 0;
            if (act && !nfr) dv += (int64_t)nw;
            if (act && !onan && !ofr) dv -= (int64_t)od;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) dv += __shfl_xor(dv, o, 64);
            dsum += dv;
#pragma unroll
            for (int q = 0; q < NK; ++q) {
                const double th = (double)km1[q];
                dle[q] += popc(__ballot(act && nw <= th)) - popc(__ballot(act && !onan && od <= th));
            }
        }
        sum_int += dsum;
        nfrac += dfrac;
        nvalid += dvalid;
#pragma unroll
        for (int q = 0; q < NK; ++q) cnt[q] += dle[q];
        ntouch = 0;
        double rowsum;
        if (nfrac == 0) {
            rowsum = (double)sum_int;
        } else {
            // fractional cells are live: numpy's pairwise sum over the row, NaN -> 0
            auto val = [&](int64_t c, double* v) {
                const double x = cell[c];
                v[0] = x != x ? 0.0 : x;
            };
            double r1v[1];
            wave_npsum<1>((int64_t)S, val, lds, r1v);
            rowsum = r1v[0];
        }
        const int slot = (int)(nrow & 63);
        if (lane == slot) {
            r_t = gt;
            r_sum = rowsum;
            r_valid = nvalid;
#pragma unroll
            for (int q = 0; q < NK; ++q) r_cnt[q] = cnt[q];
        }
        if (slot == 63) store_row(nrow - 63 + lane);
        ++nrow;
        ++group;
    };

    double tprev = -RQ_INF;
    for (int64_t i0 = 0; i0 < n_rows; i0 += 64) {
        const int64_t i = i0 + lane;
        const bool valid = i < n_rows;
        const double ti = valid ? T[i] : RQ_INF;
        const int64_t si = valid ? SRC[i] : 0;
        int ci = 0;
        if (valid) {   // column = rank of the sink id among the sorted unique ids
            const int64_t k = SNK[i];
            int lo = 0, hi = S;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (keys[mid] < k) lo = mid + 1; else hi = mid;
            }
            ci = lo;
        }
        double tp = __shfl_up(ti, 1, 64);
        if (lane == 0) tp = tprev;
        const uint64_t starts = __ballot(valid && (ti != tp || (i0 == 0 && lane == 0)));
        tprev = __shfl(ti, 63, 64);
        const int nv = (int)((n_rows - i0) < 64 ? (n_rows - i0) : 64);
        int lo = 0;
        while (lo < nv) {
            // sub-range [lo, hi): same t
            const uint64_t later = starts & ~((2ull << lo) - 1ull);   // starts strictly after lo
            const int hi = later ? (__ffsll((unsigned long long)later) - 1) : nv;
            const bool isstart = (starts >> lo) & 1ull;
            if (isstart && open) finalize();
            if (isstart) {
                gt = bcast_d(ti, lo);
                open = true;
            }
            // ranks of rows [lo, hi) in df order, same-sink rows in successive rounds
            bool pend = lane >= lo && lane < hi;
            while (__ballot(pend)) {
                if (pend) atomicMin(&ctag[ci], lane);
                __threadfence_block();
                __builtin_amdgcn_wave_barrier();
                const bool lead = pend && ctag[ci] == lane;
                if (lead) {
                    const int p = pos[ci] + 1;
                    pos[ci] = p;
                    if (si == a.src_id) last[ci] = p;
                    const int r = p - last[ci];
                    if (gtag[ci] != group) {
                        gtag[ci] = group;
                        gsum[ci] = 0.0;
                        gcnt[ci] = 0;
                    }
                    gsum[ci] += (double)r;
                    gcnt[ci] += 1;
                }
                // new touched sinks of this group: the lead rows whose sink had gcnt == 1
                const bool fresh = lead && gcnt[ci] == 1;
                const uint64_t fm = __ballot(fresh);
                if (fresh) {
                    const int k = ntouch + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(fm >> 32),
                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)fm, 0u));
                    touched[k] = ci;
                }
                ntouch += popc(fm);
                __threadfence_block();
                __builtin_amdgcn_wave_barrier();
                if (lead) ctag[ci] = 0x7fffffff;
                pend = pend && !lead;
                __threadfence_block();
                __builtin_amdgcn_wave_barrier();
            }
            lo = hi;
        }
    }
    if (open) finalize();
    {   // flush the staged rows
        const int rem = (int)(nrow & 63);
        if (lane < rem) store_row(nrow - rem + lane);
    }
    __threadfence_block();
    __builtin_amdgcn_wave_barrier();
    // pivot-row t -> dt in place, left to right (a chunk reads t[k + 64] before the
    // next chunk overwrites it)
    for (int64_t k0 = 0; k0 < nrow; k0 += 64) {
        const int64_t k = k0 + lane;
        double dt = 0.0;
        if (k < nrow) dt = (k + 1 < nrow ? R_t[k + 1] : a.end) - R_t[k];
        __threadfence_block();
        __builtin_amdgcn_wave_barrier();
        if (k < nrow) R_t[k] = dt;
        __threadfence_block();
        __builtin_amdgcn_wave_barrier();
    }
    if (lane == 0) inf->n_piv = nrow;
}

// ============================================================================
// Chunked replay: ONE dataframe over many workgroups (RP_PHASE_CHUNK).
//
// rank = (rows of the sink so far) - (position of its latest own row), so a chunk's
// effect on a sink is a function of the sink's entering rank r alone: after an own
// row of the sink inside the chunk, r_out = rows after it (a constant); without one,
// r_out = max(r, 0) + n (NaN stays NaN if n = 0).  These compose associatively, so:
//   rq_rc_plan   chunk counts per dataframe (prefix), per-df status reset
//   rq_rc_clear  per-df sink hash tables emptied
//   rq_rc_hash   every chunk inserts its sink ids (global atomics): S per dataframe
//   rq_rc_dense  dense sink ids in table order
//   rq_rc_sum    per chunk and sink: rows, rows after the last own row, last t; per chunk:
//                t-group starts, first-of-event counts, unsorted / event-id checks
//   rq_rc_scan   per sink, a wave scans the chunk functions: the state every chunk
//                enters with; per dataframe the t-group base of every chunk
//   rq_rc_apply  every chunk replays its rows exactly as rq_rp_fast does, starting from
//                those states and from the pivot row they sum to
//   rq_rc_keys   unique sink ids of dataframes with a pivot mean, for rq_rp_seq
// A dataframe with more than RC_S unique sinks (or the INT64_MIN id) is flagged
// RP_CSKIP and left to rq_rp_fast.
// ============================================================================
__device__ __forceinline__ int64_t rc_df_of_chunk(const RpArgs& a, int64_t c)
{
    int64_t lo = 0, hi = a.n_df;   // the last d with cbase[d] <= c (empty dfs share a base)
    while (hi - lo > 1) {
        const int64_t mid = (lo + hi) >> 1;
        if (a.cbase[mid] <= c) lo = mid; else hi = mid;
    }
    return lo;
}
constexpr int RC_HBITS = 13;   // log2(RC_HT)
static_assert((1 << RC_HBITS) == RC_HT, "RC_HT");
static_assert(RC_L % RP_B == 0, "chunks hold whole batches");
constexpr int RC_SKIP = RP_BADOFF | RP_EMPTYDF | RP_CSKIP;

__device__ __forceinline__ int rc_dense(const uint64_t* hk, const int* hd, uint64_t k)
{
    uint32_t h = rp_hash(k, RC_HBITS);
    for (int p = 0; p < RC_HT; ++p) {   // rq_rc_hash inserted every key (bounded all the same)
        if (hk[h] == k) return hd[h];
        h = (h + 1) & (RC_HT - 1);
    }
    return 0;
}

__global__ __launch_bounds__(1024) void rq_rc_plan(RpArgs a)
{
    __shared__ int wtot[16];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    int64_t run = 0;
    for (int64_t d0 = 0; d0 < a.n_df; d0 += 1024) {
        const int64_t d = d0 + tid;
        int nc = 0;
        if (d < a.n_df) {
            const int64_t r0 = df_begin(a, d), r1 = df_end(a, d), nd = r1 - r0;
            RpInfo* inf = a.info + d;
            int fl = 0;
            if (r0 < 0 || r1 < r0 || r1 > a.n_rows || nd >= ((int64_t)1 << 31)) fl = RP_BADOFF;
            else if (nd == 0) fl = RP_EMPTYDF;
            else nc = (int)((nd + RC_L - 1) / RC_L);
            inf->n_piv = 0;
            inf->n_own = 0;
            inf->n_world = 0;
            inf->S = 0;
            inf->flags = fl;
        }
        const int inc = (int)wave_scan_add((uint32_t)nc);
        if (lane == 63) wtot[w] = inc;
        __syncthreads();
        int64_t pre = 0, tot = 0;
        for (int k = 0; k < 16; ++k) {
            pre += k < w ? wtot[k] : 0;
            tot += wtot[k];
        }
        if (d < a.n_df) a.cbase[d] = run + pre + inc - nc;
        run += tot;
        __syncthreads();
    }
    if (tid == 0) a.cbase[a.n_df] = run;
}

__global__ __launch_bounds__(256) void rq_rc_clear(RpArgs a)
{
    const int64_t n = a.n_df * RC_HT;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
        a.ht_keys[i] = RP_EMPTY_KEY;
}

// the chunk of this block: df d, rows [c0, c1); false if the block has none
__device__ __forceinline__ bool rc_chunk(const RpArgs& a, int64_t& d, int64_t& r0, int64_t& r1, int64_t& c0,
                                         int64_t& c1)
{
    const int64_t c = blockIdx.x;
    if (c >= a.cbase[a.n_df]) return false;
    d = rc_df_of_chunk(a, c);
    r0 = df_begin(a, d);
    r1 = df_end(a, d);
    c0 = r0 + (c - a.cbase[d]) * RC_L;
    c1 = c0 + RC_L < r1 ? c0 + RC_L : r1;
    return true;
}

__global__ __launch_bounds__(1024) void rq_rc_hash(RpArgs a)
{
    int64_t d, r0, r1, c0, c1;
    if (!rc_chunk(a, d, r0, r1, c0, c1)) return;
    RpInfo* inf = a.info + d;
    if (inf->flags & RC_SKIP) return;
    unsigned long long* keys = reinterpret_cast<unsigned long long*>(a.ht_keys + d * RC_HT);
    for (int64_t i = c0 + threadIdx.x; i < c1; i += 1024) {
        const uint64_t k = (uint64_t)a.sink[i];
        if (k == RP_EMPTY_KEY) {
            atomicOr(&inf->flags, RP_CSKIP);
            continue;
        }
        uint32_t h = rp_hash(k, RC_HBITS);
        bool done = false;
        for (int p = 0; p < RC_HT && !done; ++p) {
            const unsigned long long cur = keys[h];   // a stale EMPTY is settled by the CAS
            if (cur == k) {
                done = true;
            } else if (cur == RP_EMPTY_KEY) {
                const unsigned long long old = atomicCAS(&keys[h], (unsigned long long)RP_EMPTY_KEY,
                                                         (unsigned long long)k);
                if (old == RP_EMPTY_KEY) atomicAdd(&inf->S, 1);
                done = old == RP_EMPTY_KEY || old == k;
            }
            if (!done) h = (h + 1) & (RC_HT - 1);
        }
        if (!done) atomicOr(&inf->flags, RP_CSKIP);   // table full: > RC_HT unique sinks
    }
}

__global__ __launch_bounds__(1024) void rq_rc_dense(RpArgs a)
{
    __shared__ int wtot[16];
    const int64_t d = blockIdx.x;
    RpInfo* inf = a.info + d;
    if (inf->flags & RC_SKIP) return;
    if (inf->S > RC_S) {
        if (threadIdx.x == 0) atomicOr(&inf->flags, RP_CSKIP);
        return;
    }
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint64_t* keys = a.ht_keys + d * RC_HT;
    int* dense = a.ht_dense + d * RC_HT;
    constexpr int PER = RC_HT / 1024;
    int occ[PER], m = 0;
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        occ[u] = keys[tid * PER + u] != RP_EMPTY_KEY;
        m += occ[u];
    }
    const int inc = (int)wave_scan_add((uint32_t)m);
    if (lane == 63) wtot[w] = inc;
    __syncthreads();
    int pre = 0;
    for (int k = 0; k < w; ++k) pre += wtot[k];
    int at = pre + inc - m;
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        dense[tid * PER + u] = occ[u] ? at : -1;
        at += occ[u];
    }
}

constexpr int RC_PER = RC_L / 1024;   // rows per thread in rq_rc_sum

__global__ __launch_bounds__(1024) void rq_rc_sum(RpArgs a)
{
    extern __shared__ int rc_sum_smem[];   // 4 x RC_S ints
    int* n_ = rc_sum_smem;
    int* lown = n_ + RC_S;
    int* lrow = lown + RC_S;
    int* aft = lrow + RC_S;
    __shared__ int red[4][16];
    int64_t d, r0, r1, c0, c1;
    if (!rc_chunk(a, d, r0, r1, c0, c1)) return;
    RpInfo* inf = a.info + d;
    if (inf->flags & RC_SKIP) return;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int S = inf->S;
    const uint64_t* hk = a.ht_keys + d * RC_HT;
    const int* hd = a.ht_dense + d * RC_HT;
    for (int s = tid; s < S; s += 1024) {
        n_[s] = 0;
        lown[s] = -1;
        lrow[s] = -1;
        aft[s] = 0;
    }
    __syncthreads();
    int slot[RC_PER], li[RC_PER];
    int starts = 0, ev_own = 0, ev_world = 0, unsorted = 0, eidbad = 0;
    const bool has_eid = a.eid != nullptr;
#pragma unroll
    for (int u = 0; u < RC_PER; ++u) {
        li[u] = u * 1024 + tid;
        const int64_t i = c0 + li[u];
        slot[u] = -1;
        if (i < c1) {
            const double t = a.t[i];
            const bool own = a.src[i] == a.src_id;
            slot[u] = rc_dense(hk, hd, (uint64_t)a.sink[i]);
            atomicAdd(&n_[slot[u]], 1);
            atomicMax(&lrow[slot[u]], li[u]);
            if (own) atomicMax(&lown[slot[u]], li[u]);
            if (i == r0) {
                starts += 1;
            } else {
                const double tp = a.t[i - 1];
                starts += t != tp;
                unsorted |= t < tp;
            }
            if (has_eid) {
                const int64_t e = a.eid[i];
                bool fe = true;
                if (i > r0) {
                    const int64_t ep = a.eid[i - 1];
                    fe = e != ep;
                    eidbad |= e < ep;
                }
                ev_own += fe && own;
                ev_world += fe && !own;
            }
        }
    }
    // chunk totals (one atomic per quantity and block)
    const uint32_t s0 = wave_sum_u32((uint32_t)starts), s1 = wave_sum_u32((uint32_t)ev_own),
                   s2 = wave_sum_u32((uint32_t)ev_world);
    const uint64_t fu = __ballot(unsorted), fe = __ballot(eidbad);
    if (lane == 0) {
        red[0][w] = (int)s0;
        red[1][w] = (int)s1;
        red[2][w] = (int)s2;
        red[3][w] = (fu ? 1 : 0) | (fe ? 2 : 0);
    }
    __syncthreads();
    if (tid == 0) {
        int t0 = 0, t1 = 0, t2 = 0, f = 0;
        for (int k = 0; k < 16; ++k) {
            t0 += red[0][k];
            t1 += red[1][k];
            t2 += red[2][k];
            f |= red[3][k];
        }
        a.gstart[blockIdx.x] = t0;
        if (t1) atomicAdd(reinterpret_cast<unsigned long long*>(&inf->n_own), (unsigned long long)t1);
        if (t2) atomicAdd(reinterpret_cast<unsigned long long*>(&inf->n_world), (unsigned long long)t2);
        if (f & 1) atomicOr(&inf->flags, RP_UNSORTED);
        if (f & 2) atomicOr(&inf->flags, RP_EIDBAD);
    }
    // rows after each sink's last own row
#pragma unroll
    for (int u = 0; u < RC_PER; ++u)
        if (slot[u] >= 0 && lown[slot[u]] >= 0 && li[u] > lown[slot[u]]) atomicAdd(&aft[slot[u]], 1);
    __syncthreads();
    RcCarry* out = a.carry + (int64_t)blockIdx.x * RC_S;
    for (int s = tid; s < S; s += 1024) {
        RcCarry cr;
        cr.n = n_[s];
        cr.after = lown[s] >= 0 ? aft[s] : -1;
        cr.last_t = cr.n > 0 ? a.t[c0 + lrow[s]] : 0.0;
        out[s] = cr;
    }
}

// a chunk's function on a sink's rank: CONST (an own row: r -> val) or SHIFT (r -> max(r, 0)
// + val for val > 0, identity for val = 0); has: the chunk has rows of the sink (last t lt)
struct RcFn {
    int isconst, val, has;
    double lt;
};
__device__ __forceinline__ RcFn rc_compose(const RcFn& later, const RcFn& earlier)
{
    RcFn o;
    if (later.isconst) return later;
    o.isconst = earlier.isconst;
    o.val = earlier.val + later.val;
    o.has = earlier.has | later.has;
    o.lt = later.has ? later.lt : earlier.lt;
    return o;
}
__device__ __forceinline__ RcFn rc_shfl_up(const RcFn& f, int off)
{
    RcFn g;
    g.isconst = __shfl_up(f.isconst, off, 64);
    g.val = __shfl_up(f.val, off, 64);
    g.has = __shfl_up(f.has, off, 64);
    g.lt = __shfl_up(f.lt, off, 64);
    return g;
}
__device__ __forceinline__ RcFn rc_shfl(const RcFn& f, int l)
{
    RcFn g;
    g.isconst = __shfl(f.isconst, l, 64);
    g.val = __shfl(f.val, l, 64);
    g.has = __shfl(f.has, l, 64);
    g.lt = __shfl(f.lt, l, 64);
    return g;
}

// grid (n_df, RC_S / 16) x 1024: wave w of block (d, y) scans sink 16 y + w of df d
__global__ __launch_bounds__(1024) void rq_rc_scan(RpArgs a)
{
    const int64_t d = blockIdx.x;
    RpInfo* inf = a.info + d;
    if (inf->flags & RC_SKIP) return;
    const int lane = lane_id(), w = threadIdx.x >> 6;
    const int64_t cb = a.cbase[d], nch = a.cbase[d + 1] - cb;
    if (blockIdx.y == 0 && w == 0) {   // the t-group base of every chunk
        int64_t run = 0;
        for (int64_t k0 = 0; k0 < nch; k0 += 64) {
            const int64_t k = k0 + lane;
            const int g = k < nch ? a.gstart[cb + k] : 0;
            const int inc = (int)wave_scan_add((uint32_t)g);
            if (k < nch) a.gbase[cb + k] = run + inc - g;
            run += (int64_t)__shfl(inc, 63, 64);
        }
        if (lane == 0) inf->n_piv = run;
    }
    const int s = (int)blockIdx.y * 16 + w;
    if (s >= inf->S) return;
    RcFn P{0, 0, 0, 0.0};   // the chunks before this group, composed
    for (int64_t k0 = 0; k0 < nch; k0 += 64) {
        const int64_t k = k0 + lane;
        RcFn f{0, 0, 0, 0.0};
        if (k < nch) {
            const RcCarry cr = a.carry[(cb + k) * RC_S + s];
            f.isconst = cr.after >= 0;
            f.val = f.isconst ? cr.after : cr.n;
            f.has = cr.n > 0;
            f.lt = cr.last_t;
        }
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const RcFn g = rc_shfl_up(f, off);
            if (lane >= off) f = rc_compose(f, g);
        }
        RcFn ex = rc_shfl_up(f, 1);
        if (lane == 0) ex = RcFn{0, 0, 0, 0.0};
        const RcFn e = rc_compose(ex, P);
        if (k < nch) {
            RcState st;
            st.r = e.isconst ? e.val : (e.val > 0 ? e.val : -1);
            st.pad = 0;
            st.last_t = e.lt;
            a.state[(cb + k) * RC_S + s] = st;
        }
        P = rc_compose(rc_shfl(f, 63), P);
    }
}

template <int NK>
__global__ __launch_bounds__(RP_B) void rq_rc_apply(RpArgs a)
{
    int64_t d, r0, r1, c0, c1;
    if (!rc_chunk(a, d, r0, r1, c0, c1)) return;
    RpInfo* inf = a.info + d;
    if (inf->flags & (RC_SKIP | RP_UNSORTED)) return;
    const int64_t c = blockIdx.x;
    const int tid = threadIdx.x;
    const int lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int S = inf->S;
    const uint64_t* hk = a.ht_keys + d * RC_HT;
    const int* hd = a.ht_dense + d * RC_HT;

    extern __shared__ __align__(16) unsigned char rc_smem[];
    unsigned char* sp = rc_smem;
    auto carve = [&](size_t bytes) {
        unsigned char* p = sp;
        sp += (bytes + 15) & ~(size_t)15;
        return p;
    };
    double* tb = reinterpret_cast<double*>(carve(8 * (RP_B + 2)));       // [0] prev, [1+i], [RP_B+1] next
    int* gb = reinterpret_cast<int*>(carve(4 * RP_B));                    // t-group of row i
    int* lst = reinterpret_cast<int*>(carve(4 * RP_B));                   // sink buckets: rows
    int64_t* wsum = reinterpret_cast<int64_t*>(carve(8 * 16));            // wave totals (int64)
    int* ws32 = reinterpret_cast<int*>(carve(4 * 16 * (NK + 6)));         // wave totals (int)
    int* misc = reinterpret_cast<int*>(carve(4 * 16));                    // [2] dup, [8] bucket allocator
    RpSlot* tst = reinterpret_cast<RpSlot*>(carve(sizeof(RpSlot) * RC_S));

    int km1[NK];
#pragma unroll
    for (int q = 0; q < NK; ++q) km1[q] = a.Ks[q] - 1;

    // every sink's state entering the chunk, and the pivot row it sums to
    const RcState* stin = a.state + c * RC_S;
    const double t_bnd = c0 > r0 ? a.t[c0 - 1] : 0.0;
    const bool spans = c0 > r0 && a.t[c0] == t_bnd;   // the chunk continues the previous t-group
    const int64_t G0 = a.gbase[c];
    int64_t ps = 0;
    int pv = 0, pc[NK];
#pragma unroll
    for (int q = 0; q < NK; ++q) pc[q] = 0;
    for (int s = tid; s < S; s += RP_B) {
        const RcState e = stin[s];
        if (e.r >= 0) {
            // cnt = r + 1, lastown = 1: the next row's rank is r + 1; a cell in the
            // spanning t-group keeps its group (a second row there is a pivot mean)
            tst[s] = RpSlot{e.r + 1, 1, (spans && e.last_t == t_bnd) ? (int)(G0 - 1) : -1, 0};
            ps += e.r;
            pv += 1;
#pragma unroll
            for (int q = 0; q < NK; ++q) pc[q] += e.r <= km1[q] ? 1 : 0;
        } else {
            tst[s] = RpSlot{0, 0, -1, 0};
        }
    }
    if (tid < 16) misc[tid] = 0;
    {
        int64_t s64 = ps;   // this wave's sum (int64 butterfly)
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) s64 += __shfl_xor(s64, o, 64);
        const int sv = scan_add_i32(pv);
        if (lane == 63) {
            wsum[w] = s64;
            ws32[80 + w] = sv;
        }
#pragma unroll
        for (int q = 0; q < NK; ++q) {
            const int sq = scan_add_i32(pc[q]);
            if (lane == 63) ws32[96 + 16 * q + w] = sq;
        }
    }
    __syncthreads();
    RpAcc<NK> carry;
    {
        int64_t pre64;
        int pre;
        totals_add(wsum, w, pre64, carry.s);
        totals_add(ws32 + 80, w, pre, carry.v);
#pragma unroll
        for (int q = 0; q < NK; ++q) totals_add(ws32 + 96 + 16 * q, w, pre, carry.c[q]);
    }
    int64_t Gc = G0;
    __syncthreads();   // totals read before the batch loop reuses them

    bool own_c = false;
    int slot_c = 0;
    auto prep = [&](int64_t nb0, double t_, int64_t s_, int64_t k_, double t_after, double t_before) {
        const bool v = nb0 + tid < c1;
        tb[1 + tid] = v ? t_ : 0.0;
        if (tid == 0) {
            tb[0] = t_before;
            tb[RP_B + 1] = t_after;
        }
        own_c = v && s_ == a.src_id;
        slot_c = v ? rc_dense(hk, hd, (uint64_t)k_) : 0;
    };
    {
        const int64_t i0 = c0 + tid;
        double t0 = 0.0, ta = 0.0;
        int64_t s0 = 0, k0 = 0;
        if (i0 < c1) {
            t0 = a.t[i0];
            s0 = a.src[i0];
            k0 = a.sink[i0];
        }
        if (tid == 0 && c0 + RP_B < r1) ta = a.t[c0 + RP_B];
        prep(c0, t0, s0, k0, ta, t_bnd);
    }
    // the next batch's row: loaded in the middle of the batch before, after its prep and
    // before its pivot-row stores (rp_fast_body), at a clamped index (prep masks past c1)
    double tn, tnn = 0.0;
    int64_t sn, kn;
    auto load_next = [&](int64_t nb0) __attribute__((always_inline)) {
        const int64_t in = nb0 + tid;
        const int64_t ic = in < c1 ? in : c1 - 1;   // c1 > c0: the loop runs
        tn = a.t[ic];
        sn = a.src[ic];
        kn = a.sink[ic];
        tnn = 0.0;
        if (tid == 0 && nb0 + RP_B < r1) tnn = a.t[nb0 + RP_B];
    };
    if (c1 > c0) load_next(c0 + RP_B);

    for (int64_t b0 = c0; b0 < c1; b0 += RP_B) {
        const int64_t i = b0 + tid;
        const bool valid = i < c1;

        // ---- A: neighbours of every row; its ticket in its sink's bucket ----
        __syncthreads();
        const int last = (int)((c1 - b0) < RP_B ? (c1 - b0) : RP_B);
        const double ti = tb[1 + tid];
        const double t_prev = tb[tid], t_next = tb[tid + 2];
        const double t_last = tb[last];
        const bool first_row = i == r0;
        const bool start = valid && (first_row || ti != t_prev);
        const bool endg = valid && (i == r1 - 1 || t_next != ti);
        const bool own = own_c;
        RpSlot* sl = tst + slot_c;
        const int ticket = valid ? atomicAdd(&sl->bucket, 1) : 0;

        // ---- B: t-group of every row (block scan of group starts); list space ----
        const int st_incl = scan_add_i32((int)start);
        if (lane == 63) ws32[w] = st_incl;
        __syncthreads();
        int st_pre, st_tot;
        totals_add(ws32, w, st_pre, st_tot);
        const int64_t G = Gc + (int64_t)(st_pre + st_incl) - 1;
        gb[tid] = (int)G;
        const RpSlot st0 = valid ? *sl : RpSlot{0, 0, -1, 0};
        const int m = valid ? (st0.bucket & 0xFFF) : 0;
        {   // list space: one allocator atomic per wave (rp_fast_body)
            const int need = valid && m > 1 && ticket == 0 ? m : 0;
            const int incl = scan_add_i32(need);
            int wb = 0;
            if (lane == 63 && incl > 0) wb = atomicAdd(&misc[8], incl);
            if (need) sl->bucket = ((__builtin_amdgcn_readlane(wb, 63) + incl - need) << 12) | m;
        }
        __syncthreads();

        // ---- C: my place among my sink's rows in this batch ----
        int boff = 0;
        if (valid && m > 1) {
            boff = sl->bucket >> 12;
            lst[boff + ticket] = 2 * tid + (own ? 1 : 0);   // row, own flag
        }
        __syncthreads();
        int j = 0, pred = -1, own_le = own ? tid : -1, own_lt = -1;
        auto visit = [&](int v) __attribute__((always_inline)) {
            const int y = v >> 1;
            if (y < tid) {
                ++j;
                pred = pred > y ? pred : y;
                if (v & 1) {
                    own_lt = own_lt > y ? own_lt : y;
                    own_le = own_le > y ? own_le : y;
                }
            }
        };
        if (valid && m > 1) {
            for (int k = 0; k < m; k += 2) {   // two entries per LDS wait
                const int v0 = lst[boff + k];
                const int v1 = k + 1 < m ? lst[boff + k + 1] : 0x7FFFFFFF;
                visit(v0);
                visit(v1);
            }
        }
        int j_le = 0, j_lt = 0;
        if (valid && m > 1 && (own_le >= 0 || own_lt >= 0)) {
            for (int k = 0; k < m; ++k) {
                const int y = lst[boff + k] >> 1;
                j_le += y < own_le;
                j_lt += y < own_lt;
            }
        } else if (own_le >= 0) {
            j_le = j;
        }
        RpAcc<NK> x;
        x.s = 0;
        x.v = 0;
#pragma unroll
        for (int q = 0; q < NK; ++q) x.c[q] = 0;
        if (valid) {
            const int pos = st0.cnt + j + 1;
            const int lastown = own_le >= 0 ? st0.cnt + j_le + 1 : st0.lastown;
            const int rank = pos - lastown;
            int prevrank, prevg;
            if (j > 0) {
                prevrank = (pos - 1) - (own_lt >= 0 ? st0.cnt + j_lt + 1 : st0.lastown);
                prevg = gb[pred];
            } else {
                prevrank = st0.cnt > 0 ? st0.cnt - st0.lastown : -1;
                prevg = st0.lastgroup;
            }
            if (prevg == (int)G) misc[2] = 1;   // two rows of one sink at one t: a pivot mean
            const bool pnan = prevrank < 0;
            x.s = rank - (pnan ? 0 : prevrank);
            x.v = pnan ? 1 : 0;
#pragma unroll
            for (int q = 0; q < NK; ++q)
                x.c[q] = (rank <= km1[q] ? 1 : 0) - ((!pnan && prevrank <= km1[q]) ? 1 : 0);
            if (j == m - 1) {
                sl->cnt = pos;
                sl->lastown = lastown;
                sl->lastgroup = (int)G;
                sl->bucket = 0;
            }
        }
        prep(b0 + RP_B, tn, sn, kn, tnn, t_last);
        load_next(b0 + 2 * RP_B);

        // ---- D: running totals in row order; the last row of a t-group emits its pivot row ----
        x.s = scan_add_i64_of_i32((int)x.s);
        x.v = scan_add_i32(x.v);
#pragma unroll
        for (int q = 0; q < NK; ++q) x.c[q] = scan_add_i32(x.c[q]);
        if (lane == 63) {
            wsum[w] = x.s;
            ws32[80 + w] = x.v;
#pragma unroll
            for (int q = 0; q < NK; ++q) ws32[96 + 16 * q + w] = x.c[q];
        }
        __syncthreads();
        RpAcc<NK> pre, tot;
        totals_add(wsum, w, pre.s, tot.s);
        totals_add(ws32 + 80, w, pre.v, tot.v);
#pragma unroll
        for (int q = 0; q < NK; ++q) totals_add(ws32 + 96 + 16 * q, w, pre.c[q], tot.c[q]);
        if (endg) {
            const int64_t row = r0 + G;
            a.rows_dt[row] = (i == r1 - 1 ? a.end : t_next) - ti;
            a.rows_sum[row] = (double)(carry.s + pre.s + x.s);
            a.rows_valid[row] = (uint32_t)(carry.v + pre.v + x.v);
#pragma unroll
            for (int q = 0; q < NK; ++q) a.rows_cnt[row * NK + q] = (uint32_t)(carry.c[q] + pre.c[q] + x.c[q]);
        }
        carry.s += tot.s;
        carry.v += tot.v;
#pragma unroll
        for (int q = 0; q < NK; ++q) carry.c[q] += tot.c[q];
        Gc += st_tot;
        if (tid == 0) misc[8] = 0;   // bucket allocator (read in B, two barriers ago)
    }
    __syncthreads();
    if (tid == 0 && misc[2]) atomicOr(&inf->flags, RP_FALLBACK);
}

// unique sink ids of the chunked dataframes with a pivot mean (rq_rp_keys sorts them)
__global__ __launch_bounds__(1024) void rq_rc_keys(RpArgs a)
{
    const int64_t d = blockIdx.x;
    const RpInfo* inf = a.info + d;
    const int fl = inf->flags;
    if (!(fl & RP_FALLBACK) || (fl & (RC_SKIP | RP_UNSORTED))) return;
    const int64_t r0 = df_begin(a, d);
    const uint64_t* hk = a.ht_keys + d * RC_HT;
    const int* hd = a.ht_dense + d * RC_HT;
    for (int h = threadIdx.x; h < RC_HT; h += 1024)
        if (hk[h] != RP_EMPTY_KEY) a.keys[r0 + hd[h]] = (int64_t)hk[h];
}

// ============================================================================
// rq_rp_scan: numpy-order integrals over each dataframe's pivot rows
// (one wavefront per dataframe) and the per-dataframe outputs
// ============================================================================
template <int NK>
__global__ __launch_bounds__(256) void rq_rp_scan(RpArgs a)
{
    constexpr int NV = NK + 2;
    extern __shared__ double lds_rs[];
    const int w = threadIdx.x >> 6;
    const int lane = lane_id();
    const int64_t d = (int64_t)blockIdx.x * 4 + w;
    if (d >= a.n_df) return;
    double* lds = lds_rs + (size_t)w * npsum_lds_doubles<NV>();
    const RpInfo inf = a.info[d];
    const int64_t r0 = df_begin(a, d);
    double* out = a.metrics + d * NV;
    int64_t* cnt = a.counts + d * 4;
    const bool eid_ok = a.eid && !(inf.flags & RP_EIDBAD);
    const int bad = inf.flags & (RP_UNSORTED | RP_GLOBAL | RP_BIG | RP_EMPTYDF | RP_BADOFF);
    if (lane == 0) {
        cnt[0] = eid_ok ? inf.n_own : -1;
        cnt[1] = eid_ok ? inf.n_world : -1;
        cnt[2] = (inf.flags & RP_BADOFF) ? RQ_EINVAL
                 : (inf.flags & RP_UNSORTED) ? RQ_EUNSORTED
                 : (inf.flags & (RP_GLOBAL | RP_BIG)) ? RQ_EOVERFLOW
                 : (inf.flags & RP_EMPTYDF) ? 0 : inf.n_piv;
        cnt[3] = inf.S;
    }
    if (bad || inf.n_piv <= 0) {
        if (lane < NV) out[lane] = __builtin_nan("");
        return;
    }
    const int64_t n = inf.n_piv;
    const double S = (double)inf.S;
    const double* Rd = a.rows_dt + r0;
    const double* Rs = a.rows_sum + r0;
    const uint32_t* Rv = a.rows_valid + r0;
    const uint32_t* Rc = a.rows_cnt + r0 * NK;
    struct Row {
        double dt, s;
        uint32_t v, c[NK];
    };
    auto ld = [&](uint32_t kk) {
        Row r;
        r.dt = Rd[kk];
        r.s = Rs[kk];
        r.v = Rv[kk];
#pragma unroll
        for (int q = 0; q < NK; ++q) r.c[q] = Rc[kk * NK + q];
        return r;
    };
    auto tld = [&](uint32_t) { return 0.0; };
    auto vf = [&](const Row& r, double, double* v) {
        const double m = r.s / (double)r.v;
#pragma unroll
        for (int q = 0; q < NK; ++q) v[q] = ((double)r.c[q] / S) * r.dt;
        v[NK] = m * r.dt;
        v[NK + 1] = (m * m) * r.dt;
    };
    double res[NV];
    // one wave per df (<= 4 per CU for batches of a few hundred): a whole leaf per trip
    // (16 rows per lane) halves the chain of load latencies a long df's scan waits on
    wave_npsum_rows<NV, false, Row, 16>(n, 0.0, ld, tld, vf, lds, res);
    if (lane == 0) {
#pragma unroll
        for (int s = 0; s < NV; ++s) out[s] = res[s];
    }
}

// ============================================================================
// launch wrappers
// ============================================================================
namespace {
template <int TIER>
size_t rp_fast_lds(int nK, int R)
{
    auto al = [](size_t b) { return (b + 15) & ~(size_t)15; };
    const size_t br = (size_t)R * RP_B;
    size_t s = al(8 * (br + 2)) + al(8 * (br + 1)) + al(4 * br) + al(4 * br) + al(8 * 16) +
               al(4 * 16 * (nK + 6)) + al(4 * 16);
    const size_t h = TIER == 0 ? RP_HS : RP_H;
    if (TIER < 2) s += al(8 * (h + 1)) + al(sizeof(RpSlot) * (h + 1));
    return s;
}

size_t rc_apply_lds(int nK)
{
    auto al = [](size_t b) { return (b + 15) & ~(size_t)15; };
    return al(8 * (RP_B + 2)) + al(4 * RP_B) + al(4 * RP_B) + al(8 * 16) + al(4 * 16 * (nK + 6)) +
           al(4 * 16) + al(sizeof(RpSlot) * RC_S);
}

int rp_num_cus()
{
    static thread_local int dev = -1, cus = 0;
    int d = 0;
    if (hipGetDevice(&d) != hipSuccess) return 256;
    if (d != dev) {
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess || cus <= 0)
            cus = 256;
        dev = d;
    }
    return cus;
}

template <int NK>
hipError_t rp_launch_t(const RpArgs& a, int phase, hipStream_t s)
{
    const unsigned nd = (unsigned)a.n_df;
    // no more dataframes than CUs: every workgroup has a CU to itself (2 rows per thread)
    const bool few = nd <= (unsigned)rp_num_cus();
    switch (phase) {
    case RP_PHASE_SMALL:
        if constexpr (NK <= RP_SMALL_NK) {
            if (few) hipLaunchKernelGGL((rq_rp_fast_s<NK, RP_RFEW>), dim3(nd), dim3(RP_B), rp_fast_lds<0>(NK, RP_RFEW), s, a);
            else hipLaunchKernelGGL((rq_rp_fast_s<NK, 1>), dim3(nd), dim3(RP_B), rp_fast_lds<0>(NK, 1), s, a);
        }
        break;
    case RP_PHASE_FAST:   // the full table's LDS keeps one workgroup per CU anyway
        hipLaunchKernelGGL((rq_rp_fast<NK, false, 2>), dim3(nd), dim3(RP_B), rp_fast_lds<1>(NK, 2), s, a);
        break;
    case RP_PHASE_GLOBAL:
        if (few) hipLaunchKernelGGL((rq_rp_fast<NK, true, 2>), dim3(nd), dim3(RP_B), rp_fast_lds<2>(NK, 2), s, a);
        else hipLaunchKernelGGL((rq_rp_fast<NK, true, 1>), dim3(nd), dim3(RP_B), rp_fast_lds<2>(NK, 1), s, a);
        break;
    case RP_PHASE_KEYS:
        hipLaunchKernelGGL(rq_rp_keys, dim3(nd), dim3(RP_B), 0, s, a);
        break;
    case RP_PHASE_SEQ: {
        const size_t lds = npsum_lds_doubles<1>() * sizeof(double) + RP_SEQ_LDS;
        hipLaunchKernelGGL((rq_rp_seq<NK>), dim3(nd), dim3(64), lds, s, a);
        break;
    }
    case RP_PHASE_CHUNK: {
        const unsigned mc = (unsigned)a.max_chunks;
        hipLaunchKernelGGL(rq_rc_plan, dim3(1), dim3(1024), 0, s, a);
        const unsigned cl = (unsigned)std::min<int64_t>(1024, (a.n_df * RC_HT + 255) / 256);
        hipLaunchKernelGGL(rq_rc_clear, dim3(cl), dim3(256), 0, s, a);
        hipLaunchKernelGGL(rq_rc_hash, dim3(mc), dim3(1024), 0, s, a);
        hipLaunchKernelGGL(rq_rc_dense, dim3(nd), dim3(1024), 0, s, a);
        hipLaunchKernelGGL(rq_rc_sum, dim3(mc), dim3(1024), 4 * RC_S * sizeof(int), s, a);
        hipLaunchKernelGGL(rq_rc_scan, dim3(nd, RC_S / 16), dim3(1024), 0, s, a);
        const size_t lds = rc_apply_lds(NK);
        hipLaunchKernelGGL((rq_rc_apply<NK>), dim3(mc), dim3(RP_B), lds, s, a);
        hipLaunchKernelGGL(rq_rc_keys, dim3(nd), dim3(1024), 0, s, a);
        break;
    }
    default: {
        const size_t lds = 4 * npsum_lds_doubles<NK + 2>() * sizeof(double);
        hipLaunchKernelGGL((rq_rp_scan<NK>), dim3((nd + 3) / 4), dim3(256), lds, s, a);
        break;
    }
    }
    return hipGetLastError();
}
}  // namespace

hipError_t rq_launch_rp(const RpArgs& a, int phase, hipStream_t s)
{
    if (a.n_df <= 0) return hipSuccess;
    switch (a.nK) {
    case 1: return rp_launch_t<1>(a, phase, s);
    case 2: return rp_launch_t<2>(a, phase, s);
    case 3: return rp_launch_t<3>(a, phase, s);
    default: return rp_launch_t<4>(a, phase, s);
    }
}
