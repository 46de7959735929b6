// rq_merge.hip -- the general fast sweep's arrival merge as its own kernel.
//
// Manager.run_dynamic (opt_model.py:241-314) plays the other sources' events in
// (time, source) order; with > 64 sources the arrivals are pre-generated per source
// (rq_gen_streams), and a sweep wave that merges 500 streams itself touches each
// source's stream 8 bytes at a time -- the lines are evicted between touches (round 2:
// ~10x the algorithmic read bytes).  Here one block per replica merges them once:
//
//   thread j owns source j (<= RQ_MG_B sources; a one-wave block for <= 64) and reads
//   its stream in aligned
//   64-byte chunks (two in registers, the next load issued between rounds), so every
//   line is read once;
//   rounds: every arrival before a cut tau (tau adapts so a round holds ~MG_TARGET)
//   goes to an LDS buffer with its time sub-bucket (M equal slices of [t_lo, tau),
//   a monotone map of t) and its slot in that bucket (LDS atomics), a block scan of the
//   bucket counts places the buckets, and each arrival's rank inside its bucket --
//   (t, source, buffer index) order, a bucket holds ~1 arrival -- gives its place;
//   the round is written out contiguously: mrg_t f64 / mrg_j u16 [replica][capsum].
//
// A source's arrivals enter the buffer in stream order (a lane's buffer indices grow),
// so equal times keep stream order within a source and source order across sources:
// the order the windowed sweep's stage rank gives (rq_device.h stage_rank).
// More than MG_CAP arrivals at ONE time (only replayed data can do that) cannot be
// ordered in a round: the block emits them MG_CAP at a time and flags RQ_ST_TIE, which
// sends the batch to the exact sequential sweep (engine.Graph.run(check=True)).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstdlib>
#include <type_traits>

#include "rq_device.h"
#include "rq_internal.h"

#pragma clang fp contract(off)

using namespace rq;

namespace {

// block sizes: RQ_MG_B (512) threads for 65-512 sources, one wave for <= 64 (the fused
// sweep's worlds); per block size B: rounds of <= 4B arrivals over 4B sub-buckets
constexpr int MG_SB = 11;           // bits of a slot / buffer index (< MG_CAP)
template <int B>
struct MgCfg {
    static constexpr int W = B / 64;
    static constexpr int CAP = 4 * B;       // arrivals per round (LDS buffer)
    static constexpr int M = 4 * B;         // time sub-buckets per round (4 per thread in the scan)
    static constexpr int TARGET = 3 * B;    // arrivals a round aims at
    static_assert(CAP <= (1 << MG_SB) && M <= (1 << MG_SB), "packed fields");
};

// eight consecutive arrivals of one stream (a 64-byte aligned chunk)
struct Chunk {
    double4 a, b;
};

__device__ __forceinline__ double sel8(Chunk c, int k)
{
    const double a0 = (k & 1) ? c.a.y : c.a.x, a1 = (k & 1) ? c.a.w : c.a.z;
    const double a2 = (k & 1) ? c.b.y : c.b.x, a3 = (k & 1) ? c.b.w : c.b.z;
    const double b0 = (k & 2) ? a1 : a0, b1 = (k & 2) ? a3 : a2;
    return (k & 4) ? b1 : b0;
}

__device__ __forceinline__ Chunk load_chunk(const double* p)
{
    const double4* q = reinterpret_cast<const double4*>(p);
    return Chunk{q[0], q[1]};
}

// the second half of a 128-byte line, whose first half was read before: nothing reads
// the line again, so it is loaded non-temporally (the L2 may drop it first and keep the
// lines whose second half is still to come)
typedef double rq_v4d __attribute__((ext_vector_type(4)));
__device__ __forceinline__ Chunk load_chunk_last(const double* p)
{
    const rq_v4d* q = reinterpret_cast<const rq_v4d*>(p);
    const rq_v4d x = __builtin_nontemporal_load(q), y = __builtin_nontemporal_load(q + 1);
    return Chunk{make_double4(x.x, x.y, x.z, x.w), make_double4(y.x, y.y, y.z, y.w)};
}

// arrival k (0..15) of the two chunks; both halves selected as values (a select of the
// chunks themselves would put them in scratch memory)
__device__ __forceinline__ double sel16(Chunk c, Chunk nx, int k)
{
    const double x0 = sel8(c, k & 7), x1 = sel8(nx, k & 7);
    return (k & 8) ? x1 : x0;
}

// sub-bucket of t in [t_lo, tau): non-decreasing in t (a NaN scale -- tau one ulp
// above t_lo = 0 -- sends every arrival of the round to the last bucket)
template <int M>
__device__ __forceinline__ int sub_of(double t, double t_lo, double scale)
{
    const double x = (t - t_lo) * scale;
    return x < (double)(M - 1) ? (int)x : M - 1;
}

}  // namespace

// the u16 stream of arrival k (0..15) of two 8-entry chunks of a sub-merge input
__device__ __forceinline__ uint32_t selj16(uint4 c, uint4 nx, int k)
{
    const uint4 v = (k & 8) ? nx : c;
    const uint32_t w0 = (k & 2) ? v.y : v.x, w1 = (k & 2) ? v.w : v.z;
    const uint32_t w = (k & 4) ? w1 : w0;
    return (k & 1) ? (w >> 16) : (w & 0xFFFFu);
}

// SUB: the second level of a two-level merge (> RQ_MG_B sources): thread g owns the
// merged sequence of stream group g (its entries carry their own stream ids)
// WIDE: more than 65535 streams (the second level writes bits 16-23 to out_jh)
template <int MG_B, bool SUB, bool WIDE = false>
__global__ __launch_bounds__(MG_B) void rq_merge_streams(MergeArgs a)
{
    constexpr int MG_W = MgCfg<MG_B>::W, MG_CAP = MgCfg<MG_B>::CAP, MG_M = MgCfg<MG_B>::M;
    constexpr int MG_TARGET = MgCfg<MG_B>::TARGET;
    // the one-wave instance (<= 64 streams, rounds of <= 256) keeps its slot / sub-bucket
    // pair, stream and bucket bases in 16 bits: 7.7 instead of 9.2 KB per block, so 20
    // blocks share a CU (its VGPR bound) instead of 17
    constexpr bool NARROW = MG_B <= 64 && !SUB;
    constexpr int BS_SH = NARROW ? 8 : MG_SB;   // bs = (sub-bucket << BS_SH) | slot
    static_assert(!NARROW || (MG_CAP <= 256 && MG_M <= 256), "16-bit fields");
    using BS_T = typename std::conditional<NARROW, uint16_t, uint32_t>::type;
    using BJ_T = typename std::conditional<WIDE, uint32_t, uint16_t>::type;   // global ids > 65535
    __shared__ double bt[MG_CAP];          // round buffer (arrival order)
    __shared__ BS_T bs[MG_CAP];            // (sub-bucket << BS_SH) | slot
    __shared__ BJ_T bj[MG_CAP];            // the arrival's stream
    __shared__ double st[MG_CAP];          // bucket order
    __shared__ uint32_t sk[MG_CAP];        // (stream << MG_SB) | buffer index (streams < 2^21)
    __shared__ uint32_t cnt[MG_M];
    __shared__ BS_T bbase[MG_M + 1];
    __shared__ double wmin[MG_W];
    __shared__ uint32_t wsum[MG_W];
    __shared__ uint32_t nb;

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int64_t rl = blockIdx.x;
    // the first level of a two-level merge: block (rl, group) merges streams
    // [group MG_B, group MG_B + MG_B); one level: gridDim.y == 1
    const int grp = SUB ? 0 : (int)blockIdx.y, ngrp = SUB ? 1 : (int)gridDim.y;
    const int j = (SUB ? 0 : grp * MG_B) + tid;
    // the stream id an entry carries out: group-local at a two-level merge's first level
    // (< RQ_MG_B: u16 whatever the source count), global otherwise; the second level
    // (SUB) turns its group g's local ids back into global ones, g RQ_MG_B + local
    const uint32_t jout = SUB ? (uint32_t)tid * (uint32_t)a.grp_sz : (uint32_t)(j - grp * MG_B);
    int L = 0;
    const double* src = a.streams;
    const uint16_t* srcj = nullptr;   // SUB: the entries' own stream ids
    if constexpr (SUB) {
        srcj = a.sub_j;
        src = a.sub_t;
        if (tid < a.n_grp) {
            const int64_t q = rl * a.n_grp + tid;
            L = a.sub_len[q];
            src = a.sub_t + q * a.sub_stride;
            srcj = a.sub_j + q * a.sub_stride;
        }
    } else if (j < a.n_str) {
        L = a.slen[(int64_t)j * a.slen_stride + rl];
        src = a.streams + rl * a.capsum + a.st_off[j];
    }
    // the stream's aligned chunks [p8, p8 + 8) in c and [p8 + 8, p8 + 16) in nx, with
    // p8 <= p < p8 + 16: a round's walk reads registers only; after the walk a lane that
    // moved into nx shifts it down and issues the load of the next chunk, which has the
    // rest of the round to arrive (a lane that runs through both chunks inside one walk
    // -- a burst -- loads synchronously)
    // (loads are unconditional, clamped to the stream's last chunk -- or to the buffer's
    // start for an empty stream -- so they land straight in c / nx and are waited for
    // only where the values are used)
    Chunk c, nx;
    uint4 cj = make_uint4(0, 0, 0, 0), nxj = make_uint4(0, 0, 0, 0);   // SUB: the chunks' stream ids
    int p = 0, p8 = 0;
    const int lastc = L > 0 ? (L - 1) & ~7 : 0;
#define RQ_MG_CHUNK(q) load_chunk(src + ((q) < lastc ? (q) : lastc))
#define RQ_MG_JCHUNK(q) (*reinterpret_cast<const uint4*>(srcj + ((q) < lastc ? (q) : lastc)))
#define RQ_MG_RELOAD(p0)                 \
    do {                                 \
        p8 = (p0) & ~7;                  \
        c = RQ_MG_CHUNK(p8);             \
        nx = RQ_MG_CHUNK(p8 + 8);        \
        if (SUB) {                       \
            cj = RQ_MG_JCHUNK(p8);       \
            nxj = RQ_MG_JCHUNK(p8 + 8);  \
        }                                \
    } while (0)
#define RQ_MG_HEAD() (p < L ? sel16(c, nx, p - p8) : RQ_INF)
    RQ_MG_RELOAD(0);
    double head = L > 0 ? c.a.x : RQ_INF;

    for (int k = tid; k < MG_M; k += MG_B) cnt[k] = 0;
    if (tid == 0) nb = 0;
    {
        const double m = wave_min_f64(head);
        const uint32_t s = wave_sum_u32((uint32_t)L);
        if (lane == 0) {
            wmin[w] = m;
            wsum[w] = s;
        }
    }
    __syncthreads();
    double t_lo = wmin[0];
    uint32_t total = 0;
#pragma unroll
    for (int k = 0; k < MG_W; ++k) {
        t_lo = wmin[k] < t_lo ? wmin[k] : t_lo;
        total += wsum[k];
    }
    double span = (a.end - t_lo) * ((double)MG_TARGET / (double)(total > 1 ? total : 1));
    int64_t outpos = 0;
    double* out_t = a.out_t + (rl * ngrp + grp) * a.mrg_stride;
    uint16_t* out_j = a.out_j + (rl * ngrp + grp) * a.mrg_stride;
    int status = 0;
    __syncthreads();   // wmin / wsum read before the first round rewrites them
#ifdef RQ_PHASE_CLOCK
    // diagnostic builds: block-0-thread view of where a round's time goes
    unsigned long long ck[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tc0 = 0, tc1 = 0;
#define RQ_MG_TICK(k)                                                    \
    do {                                                                 \
        tc1 = __builtin_amdgcn_s_memtime();                              \
        ck[k] += tc1 - tc0;                                              \
        tc0 = tc1;                                                       \
    } while (0)
#else
#define RQ_MG_TICK(k) do { } while (0)
#endif

    while (t_lo <= a.end) {
#ifdef RQ_PHASE_CLOCK
        tc0 = __builtin_amdgcn_s_memtime();
        ck[4] += 1;
#endif
        double tau = t_lo + span;
        if (!(tau > t_lo)) tau = next_up(t_lo);
        const double scale = (double)MG_M / (tau - t_lo);
        const int p0 = p, p8_0 = p8;
        // ---- every arrival before tau into the buffer (a lane stops at a full buffer) ----
        bool more = true;
        uint32_t nb1 = 0;   // one-wave blocks: the buffer cursor
#ifndef RQ_MG_VEC
#define RQ_MG_VEC 1
#endif
        if (RQ_MG_VEC) {
            // the cached ones, every lane at once: a lane's arrivals before tau are the run
            // [k0, k0 + cl) of its 16 cached (the stream is sorted), one wave prefix sum
            // places them, and the 16 register slots are unrolled (static indices)
            const double cv[16] = {c.a.x, c.a.y, c.a.z, c.a.w, c.b.x, c.b.y, c.b.z, c.b.w,
                                   nx.a.x, nx.a.y, nx.a.z, nx.a.w, nx.b.x, nx.b.y, nx.b.z, nx.b.w};
            const int k0 = p - p8;
            int cl = 0;
#pragma unroll
            for (int k = 0; k < 16; ++k) cl += (k >= k0 && p8 + k < L && cv[k] < tau) ? 1 : 0;
            const uint32_t incl = wave_scan_add((uint32_t)cl);
            const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
            uint32_t b0;
            if constexpr (MG_W == 1) {
                b0 = nb1;
                nb1 += tot;
            } else {
                b0 = 0;
                if (lane == 0 && tot) b0 = atomicAdd(&nb, tot);
                b0 = (uint32_t)__builtin_amdgcn_readlane((int)b0, 0);
            }
            const int base = (int)(b0 + incl) - cl;
            const int room = MG_CAP - base;
            const int take = cl < room ? cl : (room > 0 ? room : 0);
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const int e = k - k0;
                if (e >= 0 && e < take) {
                    const int idx = base + e;
                    const int sb = sub_of<MG_M>(cv[k], t_lo, scale);
                    const uint32_t slot = atomicAdd(&cnt[sb], 1u);
                    bt[idx] = cv[k];
                    bj[idx] = SUB ? jout + selj16(cj, nxj, k) : jout;
                    bs[idx] = (BS_T)(((uint32_t)sb << BS_SH) | slot);
                }
            }
            p += take;
            if (take < cl) more = false;   // the buffer is full
            if (p - p8 == 16 && p < L) RQ_MG_RELOAD(p);   // a burst: both chunks consumed
            head = RQ_MG_HEAD();
        }
        // the rest of a burst (a lane ran through both chunks), one arrival per step
        for (;;) {
            const bool act = more && head < tau;
            const uint64_t m = __ballot(act);
            if (!m) break;
            uint32_t b0;
            if constexpr (MG_W == 1) {   // one wave: the buffer cursor is a register
                b0 = nb1;
                nb1 += (uint32_t)__popcll(m);
            } else {
                const int fl = __ffsll((unsigned long long)m) - 1;
                b0 = 0;
                if (lane == fl) b0 = atomicAdd(&nb, (uint32_t)__popcll(m));
                b0 = (uint32_t)__builtin_amdgcn_readlane((int)b0, fl);
            }
            if (act) {
                const uint32_t idx = b0 + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
                if (idx < (uint32_t)MG_CAP) {
                    const int sb = sub_of<MG_M>(head, t_lo, scale);
                    const uint32_t slot = atomicAdd(&cnt[sb], 1u);
                    bt[idx] = head;
                    bj[idx] = SUB ? jout + selj16(cj, nxj, p - p8) : jout;
                    bs[idx] = (BS_T)(((uint32_t)sb << BS_SH) | slot);
                    ++p;
                    if (p - p8 == 16 && p < L) RQ_MG_RELOAD(p);   // a burst: both chunks consumed
                    head = RQ_MG_HEAD();
                } else {
                    more = false;
                }
            }
        }
        {
            const double m = wave_min_f64(head);
            if (lane == 0) wmin[w] = m;
        }
        if (p - p8 >= 8) {   // into nx: its successor's load overlaps the rest of the round
            c = nx;
            p8 += 8;
#ifndef RQ_MG_NTL
#define RQ_MG_NTL 1
#endif
            if (RQ_MG_NTL && ((p8 + 8) & 8))   // the second half of its line: the line's last use
                nx = load_chunk_last(src + ((p8 + 8) < lastc ? (p8 + 8) : lastc));
            else
                nx = RQ_MG_CHUNK(p8 + 8);
            if (SUB) {
                cj = nxj;
                nxj = RQ_MG_JCHUNK(p8 + 8);
            }
        }
        if constexpr (MG_W == 1) {
            if (lane == 0) nb = nb1;
        }
        RQ_MG_TICK(0);
        __syncthreads();
        RQ_MG_TICK(1);
        const uint32_t nr_all = nb;
        uint32_t nr = nr_all;
        if (nr_all > (uint32_t)MG_CAP) {
            if (tau != next_up(t_lo)) {
                // too many for one round: undo it and halve the cut
                p = p0;   // the chunks in registers still hold p0 unless a burst or the shift moved them
                if (p8 != p8_0) RQ_MG_RELOAD(p0);
                head = RQ_MG_HEAD();
                for (int k = tid; k < MG_M; k += MG_B) cnt[k] = 0;
                __syncthreads();
                if (tid == 0) nb = 0;
                span = (tau - t_lo) * 0.5;
                __syncthreads();
#ifdef RQ_PHASE_CLOCK
                ck[5] += 1;
#endif
                continue;
            }
            // more than MG_CAP arrivals at t_lo itself: take the first MG_CAP (any subset
            // of equal times is a time prefix) and flag the replica
            nr = MG_CAP;
            status |= a.strict_ties ? RQ_ST_UNORDERED : RQ_ST_TIE;
        }
        if (outpos + (int64_t)nr > a.mrg_stride) {   // past the merged capacity (uniform)
            status |= RQ_ST_STREAM_OVERFLOW;
            break;
        }
        double t_next = wmin[0];
#pragma unroll
        for (int k = 1; k < MG_W; ++k) t_next = wmin[k] < t_next ? wmin[k] : t_next;
        // ---- bucket bases: exclusive scan of cnt (4 buckets per thread) ----
        uint32_t v0 = cnt[4 * tid], v1 = cnt[4 * tid + 1], v2 = cnt[4 * tid + 2], v3 = cnt[4 * tid + 3];
        const uint32_t tsum = v0 + v1 + v2 + v3;
        const uint32_t incl = wave_scan_add(tsum);
        if (lane == 63) wsum[w] = incl;
        __syncthreads();
        if (tid == 0) nb = 0;   // every thread read nb before this barrier
        uint32_t wo = 0;
#pragma unroll
        for (int k = 0; k < MG_W; ++k) wo += k < w ? wsum[k] : 0u;
        {
            const uint32_t b = wo + incl - tsum;
            bbase[4 * tid] = (BS_T)b;
            bbase[4 * tid + 1] = (BS_T)(b + v0);
            bbase[4 * tid + 2] = (BS_T)(b + v0 + v1);
            bbase[4 * tid + 3] = (BS_T)(b + v0 + v1 + v2);
            cnt[4 * tid] = cnt[4 * tid + 1] = cnt[4 * tid + 2] = cnt[4 * tid + 3] = 0;
            if (tid == 0) bbase[MG_M] = (BS_T)nr;
        }
        __syncthreads();
        RQ_MG_TICK(2);
        // ---- into bucket order ----
        for (int i = tid; i < (int)nr; i += MG_B) {
            const uint32_t x = bs[i];
            const uint32_t pos = (uint32_t)bbase[x >> BS_SH] + (x & ((1u << BS_SH) - 1u));
            st[pos] = bt[i];
            sk[pos] = ((uint32_t)bj[i] << MG_SB) | (uint32_t)i;
        }
        __syncthreads();
        RQ_MG_TICK(3);
        // ---- rank inside the bucket, written out in play order ----
        for (int i = tid; i < (int)nr; i += MG_B) {
            const double x = st[i];
            const uint32_t kx = sk[i];
            const int sb = sub_of<MG_M>(x, t_lo, scale);
            const int g0 = (int)bbase[sb], g1 = (int)bbase[sb + 1];
            int r = 0;
            for (int k = g0; k < g1; ++k) {
                const double y = st[k];
                r += (y < x || (y == x && sk[k] < kx)) ? 1 : 0;
            }
#ifndef RQ_MG_NT
#define RQ_MG_NT 1
#endif
            // streaming stores: the output must not evict the input lines (C3 merge reads
            // 1.71 -> 1.37 x its 8 B per arrival, profiles/r04_merge_traffic.txt)
            if (RQ_MG_NT) {
                __builtin_nontemporal_store(x, &out_t[outpos + g0 + r]);
                __builtin_nontemporal_store((uint16_t)(kx >> MG_SB), &out_j[outpos + g0 + r]);
            } else {
                out_t[outpos + g0 + r] = x;
                out_j[outpos + g0 + r] = (uint16_t)(kx >> MG_SB);
            }
            if (WIDE) a.out_jh[(rl * ngrp + grp) * a.mrg_stride + outpos + g0 + r] = (uint8_t)(kx >> (MG_SB + 16));
        }
        RQ_MG_TICK(6);
        outpos += nr;
        // next cut: aim at MG_TARGET arrivals, grow at most 4x per round
        const double wdt = tau - t_lo;
        const double f = (double)MG_TARGET / (double)(nr > 64 ? nr : 64);
        span = wdt * (f < 4.0 ? f : 4.0);
        t_lo = t_next;   // the heads after the walk (an equal-time round: t_lo again)
    }
#ifdef RQ_PHASE_CLOCK
    // phases: 0 walk, 1 barrier after the walk, 2 bucket scan, 3 scatter, 6 rank + write;
    // 4 rounds, 5 retried rounds
    if (a.clk && w == 0 && lane == 0)
        for (int k = 0; k < 8; ++k) atomicAdd(&a.clk[k], ck[k]);
#endif
#undef RQ_MG_TICK
#undef RQ_MG_HEAD
#undef RQ_MG_RELOAD
#undef RQ_MG_CHUNK
    if (tid == 0) {
        a.out_len[rl * ngrp + grp] = (int)outpos;
        if (status) atomicOr(&a.status[a.chunk0 + rl], status);
    }
}

// A handful of streams (C4 / C2: the README graph's three, ~2100 arrivals per replica):
// the bucket rounds ran a 64-lane block with 3 lanes walking, so here the merge is a
// RANKING instead.  A block stages its replica's streams in LDS (coalesced), then every
// arrival finds its place in the play order at once: its index in its own stream plus,
// per other stream j', the arrivals of j' that play before it -- those at an earlier
// time, or at the same time when j' < j (equal times in stream order, as the bucket
// rounds emit them) -- by binary search in LDS, and is written there.  No equal-time
// cap; the same (t, stream) sequence.
template <int NS>
__global__ __launch_bounds__(256) void rq_merge_rank(MergeArgs a)
{
    extern __shared__ double mr_sh[];
    const int64_t rl = blockIdx.x;
    const int tid = threadIdx.x;
    const double* base = a.streams + rl * a.capsum;
    int len[NS], off[NS];
    int64_t total = 0;
#pragma unroll
    for (int j = 0; j < NS; ++j) {
        len[j] = j < a.n_str ? a.slen[(int64_t)j * a.slen_stride + rl] : 0;
        off[j] = j < a.n_str ? (int)a.st_off[j] : 0;
        total += len[j];
    }
#pragma unroll
    for (int j = 0; j < NS; ++j)
        for (int i = tid; i < len[j]; i += blockDim.x) mr_sh[off[j] + i] = base[off[j] + i];
    __syncthreads();
    double* ot = a.out_t + rl * a.mrg_stride;
    uint16_t* oj = a.out_j + rl * a.mrg_stride;
#pragma unroll
    for (int j = 0; j < NS; ++j) {
        for (int i = tid; i < len[j]; i += blockDim.x) {
            const double t = mr_sh[off[j] + i];
            int64_t r = i;
#pragma unroll
            for (int q = 0; q < NS; ++q) {
                if (q == j || len[q] == 0) continue;
                // arrivals of stream q before t: t' < t, or t' <= t for q < j
                const double* v = mr_sh + off[q];
                int lo = 0, hi = len[q];
                while (lo < hi) {
                    const int mid = (lo + hi) >> 1;
                    const double x = v[mid];
                    if (x < t || (q < j && x == t)) lo = mid + 1;
                    else hi = mid;
                }
                r += lo;
            }
            // plain stores: the inputs are in LDS (nothing to protect in L2), and the
            // scattered 8-B / 2-B entries of a line merge in L2 before the write-back
            // (nontemporal stores wrote 2.0 x the 10 B per entry; C4 27.7 -> 25.9 ms)
            if (r < a.mrg_stride) {
                ot[r] = t;
                oj[r] = (uint16_t)j;
            }
        }
    }
    if (tid == 0) {
        a.out_len[rl] = (int)(total < a.mrg_stride ? total : a.mrg_stride);
        if (total > a.mrg_stride) atomicOr(&a.status[a.chunk0 + rl], RQ_ST_STREAM_OVERFLOW);
    }
}

hipError_t rq_launch_merge(const MergeArgs& a, hipStream_t s)
{
    if (a.n_chunk <= 0) return hipSuccess;
    if (a.n_str > RQ_MG_B) return hipErrorInvalidValue;
    const char* e = getenv("RQ_MERGE_SMALL");   // A/B and the bucket merge's own tests only
    const bool small_on = !e || atoi(e) != 0;
    // <= 8 streams whose buffers fit a block's LDS: the ranking merge
    const size_t lds = (size_t)a.capsum * sizeof(double);
    if (small_on && a.n_str <= 8 && lds <= 64 * 1024) {
        if (a.n_str <= 4)
            hipLaunchKernelGGL((rq_merge_rank<4>), dim3((unsigned)a.n_chunk), dim3(256), lds, s, a);
        else
            hipLaunchKernelGGL((rq_merge_rank<8>), dim3((unsigned)a.n_chunk), dim3(256), lds, s, a);
        return hipGetLastError();
    }
    if (a.n_str <= 64)
        hipLaunchKernelGGL((rq_merge_streams<64, false>), dim3((unsigned)a.n_chunk), dim3(64), 0, s, a);
    else
        hipLaunchKernelGGL((rq_merge_streams<RQ_MG_B, false>), dim3((unsigned)a.n_chunk), dim3(RQ_MG_B), 0, s, a);
    return hipGetLastError();
}

hipError_t rq_launch_merge_groups(const MergeArgs& a, hipStream_t s)
{
    if (a.n_chunk <= 0) return hipSuccess;
    if (a.grp_sz != 64 && a.grp_sz != RQ_MG_B) return hipErrorInvalidValue;
    const int ng = (a.n_str + a.grp_sz - 1) / a.grp_sz;
    if (ng < 2 || ng > RQ_MG_B || a.n_str > RQ_MAX_STREAMS_MRG) return hipErrorInvalidValue;
    if (a.grp_sz == 64)
        hipLaunchKernelGGL((rq_merge_streams<64, false>), dim3((unsigned)a.n_chunk, (unsigned)ng), dim3(64), 0, s, a);
    else
        hipLaunchKernelGGL((rq_merge_streams<RQ_MG_B, false>), dim3((unsigned)a.n_chunk, (unsigned)ng), dim3(RQ_MG_B), 0,
                           s, a);
    return hipGetLastError();
}

hipError_t rq_launch_merge_sub(const MergeArgs& a, hipStream_t s)
{
    if (a.n_chunk <= 0) return hipSuccess;
    if (a.n_grp < 1 || a.n_grp > RQ_MG_B || !a.sub_t || !a.sub_j || !a.sub_len) return hipErrorInvalidValue;
    // <= 64 groups are <= 32768 streams: 16-bit ids; past 65535 streams the WIDE instance
    if (a.n_grp <= 64) {
        hipLaunchKernelGGL((rq_merge_streams<64, true>), dim3((unsigned)a.n_chunk), dim3(64), 0, s, a);
    } else if (a.out_jh) {
        hipLaunchKernelGGL((rq_merge_streams<RQ_MG_B, true, true>), dim3((unsigned)a.n_chunk), dim3(RQ_MG_B), 0, s, a);
    } else {
        hipLaunchKernelGGL((rq_merge_streams<RQ_MG_B, true>), dim3((unsigned)a.n_chunk), dim3(RQ_MG_B), 0, s, a);
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Longest-first replica order for the sweeps' work queues (LPT): the sweep of a
// replica costs about its merged length, and the waves take replicas in queue order,
// so the longest go first and the launch ends on short ones.  One wave (it must find a
// slot while another stream's sweep holds the chip): a counting sort of the lengths
// into OB buckets of (max - len) (descending length; replicas of one bucket in any
// order -- outputs are indexed by replica, so the order changes no result bit, only
// which wave plays which replica when).
// ---------------------------------------------------------------------------
namespace {
constexpr int OB = 1024;   // buckets (16 per lane)
}

__global__ __launch_bounds__(64) void rq_order_replicas(const int* __restrict__ len, int n, int* __restrict__ order)
{
    __shared__ uint32_t hist[OB];
    const int lane = threadIdx.x;
    int mn = 0x7fffffff, mx = 0;
    for (int i = lane; i < n; i += 64) {
        const int v = len[i];
        mn = v < mn ? v : mn;
        mx = v > mx ? v : mx;
    }
    for (int k = lane; k < OB; k += 64) hist[k] = 0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const int a = __shfl_xor(mn, o), b = __shfl_xor(mx, o);
        mn = a < mn ? a : mn;
        mx = b > mx ? b : mx;
    }
    const int64_t span = (int64_t)mx - mn + 1;
    auto bucket = [&](int v) -> int { return (int)(((int64_t)(mx - v) * OB) / span); };
    wave_lds_sync();
    for (int i = lane; i < n; i += 64) atomicAdd(&hist[bucket(len[i])], 1u);
    wave_lds_sync();
    // exclusive scan: lane l owns buckets [16 l, 16 l + 16)
    uint32_t h[OB / 64], sum = 0;
#pragma unroll
    for (int k = 0; k < OB / 64; ++k) {
        h[k] = hist[lane * (OB / 64) + k];
        sum += h[k];
    }
    uint32_t base = wave_scan_add(sum) - sum;
#pragma unroll
    for (int k = 0; k < OB / 64; ++k) {
        hist[lane * (OB / 64) + k] = base;
        base += h[k];
    }
    wave_lds_sync();
    for (int i = lane; i < n; i += 64) order[atomicAdd(&hist[bucket(len[i])], 1u)] = i;
}

hipError_t rq_launch_order(const int* len, int64_t n, int* order, hipStream_t s)
{
    if (n <= 0) return hipSuccess;
    if (n > 65536) return hipErrorInvalidValue;
    hipLaunchKernelGGL(rq_order_replicas, dim3(1), dim3(64), 0, s, len, (int)n, order);
    return hipGetLastError();
}
