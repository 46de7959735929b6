// rq_device.h -- gfx950 device helpers shared by the engine kernels.
//
//   * Philox4x32-10 (Salmon et al. SC'11) -- the engine's counter-based RNG:
//     stream (seed, salt), draw d -> call d>>1, uniform from words (0,1) or
//     (2,3).  The CPU oracle has its own implementation pinned by Random123's
//     known-answer vectors; GPU == oracle is checked by the parity tests.
//   * wave64 helpers (min / ballot / broadcast).
//   * wave_npsum: numpy's float64 np.sum order (8192-element chunks, pairwise
//     tree with 8-accumulator leaves <= 128) evaluated by one wavefront: the
//     leaves run 8 lanes x 8 leaves at a time, the tree above them is walked
//     by the (uniform) wave with an LDS stack.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rq_spec.h"

#pragma clang fp contract(off)

#define RQ_INF __builtin_huge_val()

namespace rq {

// rq_exp's table (rq_tables.h) in constant memory; the fused sweep stages a copy in LDS
static __constant__ uint64_t rq_exp_tab_c[RQ_EXP_TAB_N] = RQ_EXP_TAB_INIT;

__device__ __forceinline__ void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1)
{
    // each round's two 32x32 -> 64-bit products as ONE v_mad_u64_u32 apiece (measured
    // 262 vs 363 SIMD cycles per wave64 call against separate mul_hi / mul_lo:
    // scripts/micro/philox_rate.hip); the bits are the same
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
        const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
        c[0] = n0;
        c[1] = (uint32_t)p1;
        c[2] = n2;
        c[3] = (uint32_t)p0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}

__host__ __device__ __forceinline__ uint32_t kind_salt(int kind, bool ctrl)
{
    return 0x52510000u | (uint32_t)kind | (ctrl ? 0x100u : 0u);
}

// Sequential reader of one Philox stream (one lane, one source).
struct PhiloxStream {
    uint32_t key0, key1;
    uint64_t d;        // next draw index
    uint32_t w2, w3;   // second half of the last call
    __device__ __forceinline__ PhiloxStream(uint32_t seed, uint32_t salt)
        : key0(seed), key1(salt), d(0), w2(0), w3(0) {}
    __device__ __forceinline__ double next()
    {
        double u;
        if ((d & 1) == 0) {
            const uint64_t call = d >> 1;
            uint32_t c[4] = {(uint32_t)call, (uint32_t)(call >> 32), 0u, 0u};
            philox4x32_10(c, key0, key1);
            w2 = c[2];
            w3 = c[3];
            u = rq_uniform53(c[0], c[1]);
        } else {
            u = rq_uniform53(w2, w3);
        }
        ++d;
        return u;
    }
};

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }

// set bits of a 64-bit wave mask in the lanes below this one (v_mbcnt_lo / _hi): no
// per-lane 64-bit "below" constant that the compiler hoists out of a loop and spills
__device__ __forceinline__ int mbcnt64(uint64_t m)
{
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
// ... at or below this lane
__device__ __forceinline__ int mbcnt64_incl(uint64_t m)
{
    return mbcnt64(m) + (int)((m >> lane_id()) & 1ull);
}

__device__ __forceinline__ double wave_min(double v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, 64));
    return v;
}

__device__ __forceinline__ double bcast_d(double v, int src_lane)
{
    const uint64_t b = rq_dbl_bits(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, src_lane);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), src_lane);
    return rq_bits_dbl(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ int bcast_i(int v, int src_lane)
{
    return __builtin_amdgcn_readlane(v, src_lane);
}

// a wave-uniform 64-bit value (a ballot, a mask built from ballots) pinned to SGPRs, so
// the code derived from it stays on the scalar unit
__device__ __forceinline__ uint64_t sgpr_u64(uint64_t v)
{
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ int64_t bcast_i64(int64_t v, int src_lane)
{
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, src_lane);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), src_lane);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

// order this wave's LDS stores before its later LDS loads of other lanes' data
__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// the same for per-wave state in GLOBAL memory that lanes of one wave hand to each
// other (a lane reads what another lane stored): workgroup-scope release / acquire,
// i.e. the wave's stores complete before any lane's next load
__device__ __forceinline__ void wave_mem_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

__device__ __forceinline__ int popc(uint64_t m) { return __popcll(m); }

// ---- DPP wave reductions (result in lane 63, returned through v_readlane) ----
template <int CTRL, int ROWMASK>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)v, CTRL, ROWMASK, 0xF, false);
}
__device__ __forceinline__ uint32_t umin32(uint32_t a, uint32_t b) { return a < b ? a : b; }

// min over the 64 lanes: quad swaps, half-row / row mirrors, then row broadcasts 15, 31
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v)
{
    v = umin32(v, dpp_u32<0xB1, 0xF>(v));    // quad_perm [1,0,3,2]
    v = umin32(v, dpp_u32<0x4E, 0xF>(v));    // quad_perm [2,3,0,1]
    v = umin32(v, dpp_u32<0x141, 0xF>(v));   // row_half_mirror
    v = umin32(v, dpp_u32<0x140, 0xF>(v));   // row_mirror
    v = umin32(v, dpp_u32<0x142, 0xA>(v));   // row_bcast:15 -> rows 1, 3
    v = umin32(v, dpp_u32<0x143, 0xC>(v));   // row_bcast:31 -> rows 2, 3
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// sum over the 64 lanes (same DPP pattern, adds; disabled rows add 0), via lane 63
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v)
{
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// N independent 64-lane sums interleaved stage by stage (so the DPP read-after-
// write hazards of one chain are covered by the others); totals end in lane 63
template <int N>
__device__ __forceinline__ void wave_sum_u32_n(uint32_t (&v)[N])
{
#define RQ_SUM_STAGE(CTRL, RM)                                                                   \
    _Pragma("unroll") for (int k = 0; k < N; ++k) v[k] +=                                       \
        (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v[k], CTRL, RM, 0xF, false);
    RQ_SUM_STAGE(0xB1, 0xF)
    RQ_SUM_STAGE(0x4E, 0xF)
    RQ_SUM_STAGE(0x141, 0xF)
    RQ_SUM_STAGE(0x140, 0xF)
    RQ_SUM_STAGE(0x142, 0xA)
    RQ_SUM_STAGE(0x143, 0xC)
#undef RQ_SUM_STAGE
}

// v into lane l (v, l uniform): v_cmp + v_cndmask
__device__ __forceinline__ int writelane(int old, int v, int l) { return lane_id() == l ? v : old; }
// the same with v_writelane_b32: v and l must be wave-uniform
// (the LLVM intrinsic, which this clang has no builtin for; the backend moves the
// lane select to m0 when both operands are SGPRs)
__device__ int rq_llvm_writelane(int v, int l, int old) __asm("llvm.amdgcn.writelane");
__device__ __forceinline__ int wlane(int old, int v, int l) { return rq_llvm_writelane(v, l, old); }

// ---- DPP prefix scans (inclusive): row shifts 1, 2, 4, 8 then row broadcasts 15, 31.
// A lane whose DPP source is out of its row (or whose row is masked off) reads 0,
// the identity of both OR and ADD.
template <int CTRL, int RM>
__device__ __forceinline__ uint32_t dpp0(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, RM, 0xF, false);
}
// full row mask + bound_ctrl: every lane is written (its source or 0)
template <int CTRL>
__device__ __forceinline__ uint32_t dppz(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t wave_scan_add(uint32_t v)
{
    v += dpp0<0x111, 0xF>(v);
    v += dpp0<0x112, 0xF>(v);
    v += dpp0<0x114, 0xF>(v);
    v += dpp0<0x118, 0xF>(v);
    v += dpp0<0x142, 0xA>(v);
    v += dpp0<0x143, 0xC>(v);
    return v;
}
__device__ __forceinline__ uint32_t wave_scan_or(uint32_t v)
{
    v |= dpp0<0x111, 0xF>(v);
    v |= dpp0<0x112, 0xF>(v);
    v |= dpp0<0x114, 0xF>(v);
    v |= dpp0<0x118, 0xF>(v);
    v |= dpp0<0x142, 0xA>(v);
    v |= dpp0<0x143, 0xC>(v);
    return v;
}
// Segmented scans: a segment starts at every lane whose flag is set.  c[s] = ~0
// unless a segment starts inside this lane's window before step s (Hillis-Steele
// with head flags); the flags do not depend on the scanned words, so they are
// built once per tile.  The combine is an AND with c[s], never a select: a select
// may be lowered to an EXEC-masked DPP op, and DPP reads 0 from lanes EXEC disables.
struct SegFlags {
    uint32_t c0, c1, c2, c3, c4, c5;
    __device__ __forceinline__ void init(bool head)
    {
        uint32_t f = head ? 1u : 0u;
        c0 = f - 1u;  f |= dpp0<0x111, 0xF>(f);
        c1 = f - 1u;  f |= dpp0<0x112, 0xF>(f);
        c2 = f - 1u;  f |= dpp0<0x114, 0xF>(f);
        c3 = f - 1u;  f |= dpp0<0x118, 0xF>(f);
        c4 = f - 1u;  f |= dpp0<0x142, 0xA>(f);
        c5 = f - 1u;
        // opaque masks: keeps `x & c` a single v_and_or_b32 instead of a lane-mask select
        __asm__("" : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(c4), "+v"(c5));
    }
    __device__ __forceinline__ uint32_t scan_or(uint32_t v) const
    {
        v |= dpp0<0x111, 0xF>(v) & c0;
        v |= dpp0<0x112, 0xF>(v) & c1;
        v |= dpp0<0x114, 0xF>(v) & c2;
        v |= dpp0<0x118, 0xF>(v) & c3;
        v |= dpp0<0x142, 0xA>(v) & c4;
        v |= dpp0<0x143, 0xC>(v) & c5;
        return v;
    }
    // the same scan with bound_ctrl on the row shifts (an out-of-row source reads 0
    // either way), so each of those steps folds into one v_and_b32_dpp + v_or_b32
    // The row-broadcast steps take the previous step's shifted word t as the DPP
    // `old` of the rows they leave unwritten, so no zeroing move is needed: a window
    // that holds no segment head at step k held none at step k-1 (c_k != 0 implies
    // c_{k-1} != 0), so t & c_k is already contained in v and OR-ing it is a no-op.
    __device__ __forceinline__ uint32_t scan_or_z(uint32_t m) const
    {
        uint32_t t = dppz<0x111>(m);
        uint32_t v = m | (t & c0);
        t = dppz<0x112>(v);
        v |= t & c1;
        t = dppz<0x114>(v);
        v |= t & c2;
        t = dppz<0x118>(v);
        v |= t & c3;
        t = (uint32_t)__builtin_amdgcn_update_dpp((int)t, (int)v, 0x142, 0xA, 0xF, false);
        v |= t & c4;
        t = (uint32_t)__builtin_amdgcn_update_dpp((int)t, (int)v, 0x143, 0xC, 0xF, false);
        v |= t & c5;
        return v;
    }
    __device__ __forceinline__ uint32_t scan_add(uint32_t v) const
    {
        v += dpp0<0x111, 0xF>(v) & c0;
        v += dpp0<0x112, 0xF>(v) & c1;
        v += dpp0<0x114, 0xF>(v) & c2;
        v += dpp0<0x118, 0xF>(v) & c3;
        v += dpp0<0x142, 0xA>(v) & c4;
        v += dpp0<0x143, 0xC>(v) & c5;
        return v;
    }
};

// rank of this lane's staged arrival (ti at slot `lane`) among the tile's staged
// times st_t[0..n) in (t, slot) order.  st_t[n..64) must hold +INF (never below a
// finite ti).  First #{t < ti} alone (one compare and one carry-add per slot, reads
// broadcast from LDS, 8 slots per wait); those ranks are a permutation of 0..n-1,
// i.e. sum to n(n-1)/2, exactly when no two staged times are equal -- otherwise the
// count is redone with the slot tie-break.
__device__ __forceinline__ int stage_rank(const double* st_t, int n, double ti, int lane)
{
    int rnk = 0;
    for (int q = 0; q < n; q += 8) {
        double2 x[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) x[u] = *reinterpret_cast<const double2*>(st_t + q + 2 * u);
#pragma unroll
        for (int u = 0; u < 4; ++u) rnk += (x[u].x < ti ? 1 : 0) + (x[u].y < ti ? 1 : 0);
    }
    const uint32_t sum = wave_sum_u32(lane < n ? (uint32_t)rnk : 0u);
    if (sum == (uint32_t)(n * (n - 1) / 2)) return rnk;
    rnk = 0;
    for (int q = 0; q < n; q += 2) {
        const double2 x = *reinterpret_cast<const double2*>(st_t + q);
        rnk += (x.x < ti || (x.x == ti && q < lane)) ? 1 : 0;
        rnk += (x.y < ti || (x.y == ti && q + 1 < lane)) ? 1 : 0;
    }
    return rnk;
}

// min of a double over the 64 lanes (every lane gets it)
// v_min_f64 without the compiler's sNaN canonicalisation of both inputs (operands
// here are times or +INF, never NaN).  The trailing s_nop covers the two wait
// states a following DPP read of the result needs (the hazard recognizer does not
// look into inline asm).
__device__ __forceinline__ double min_raw(double a, double b)
{
    double r;
    __asm__("v_min_f64 %0, %1, %2\n\ts_nop 1" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

__device__ __forceinline__ double wave_min_f64(double x)
{
#define RQ_MIN_STAGE(CTRL, RM)                                                                     \
    {                                                                                              \
        const uint64_t b = rq_dbl_bits(x);                                                         \
        const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)b, CTRL, RM,   \
                                                                  0xF, false);                     \
        const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0x7FF00000, (int)(uint32_t)(b >> 32), \
                                                                  CTRL, RM, 0xF, false);           \
        x = min_raw(x, rq_bits_dbl(((uint64_t)hi << 32) | lo));                                    \
    }
    RQ_MIN_STAGE(0xB1, 0xF)
    RQ_MIN_STAGE(0x4E, 0xF)
    RQ_MIN_STAGE(0x141, 0xF)
    RQ_MIN_STAGE(0x140, 0xF)
    RQ_MIN_STAGE(0x142, 0xA)
    RQ_MIN_STAGE(0x143, 0xC)
#undef RQ_MIN_STAGE
    return bcast_d(x, 63);
}

// the next double above finite x
// inclusive prefix min over the 64 lanes (times / +INF): row shifts 1, 2, 4, 8 then
// row broadcasts 15, 31.  A lane a step does not write keeps the DPP `old`, here
// the previous step's shifted value t, which is >= the lane's running min already,
// so min(v, t) leaves it unchanged (step 1 takes v itself).
__device__ __forceinline__ double wave_scan_min_f64(double v)
{
    uint64_t b = rq_dbl_bits(v);
    uint32_t tlo = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)b, (int)(uint32_t)b, 0x111, 0xF, 0xF, false);
    uint32_t thi = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)(b >> 32), (int)(uint32_t)(b >> 32), 0x111,
                                                          0xF, 0xF, false);
    v = min_raw(v, rq_bits_dbl(((uint64_t)thi << 32) | tlo));
#define RQ_SCANMIN_STAGE(CTRL, RM)                                                                      \
    {                                                                                                   \
        b = rq_dbl_bits(v);                                                                             \
        tlo = (uint32_t)__builtin_amdgcn_update_dpp((int)tlo, (int)(uint32_t)b, CTRL, RM, 0xF, false);  \
        thi = (uint32_t)__builtin_amdgcn_update_dpp((int)thi, (int)(uint32_t)(b >> 32), CTRL, RM, 0xF, \
                                                    false);                                             \
        v = min_raw(v, rq_bits_dbl(((uint64_t)thi << 32) | tlo));                                       \
    }
    RQ_SCANMIN_STAGE(0x112, 0xF)
    RQ_SCANMIN_STAGE(0x114, 0xF)
    RQ_SCANMIN_STAGE(0x118, 0xF)
    RQ_SCANMIN_STAGE(0x142, 0xA)
    RQ_SCANMIN_STAGE(0x143, 0xC)
#undef RQ_SCANMIN_STAGE
    return v;
}
// the value of lane l - 1 (+INF at lane 0): DPP wave_shr:1
__device__ __forceinline__ double wave_shr1_inf_f64(double v)
{
    const uint64_t b = rq_dbl_bits(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)b, 0x138, 0xF, 0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0x7FF00000, (int)(uint32_t)(b >> 32), 0x138, 0xF, 0xF,
                                                              false);
    return rq_bits_dbl(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ double next_up(double x)
{
    if (x == 0.0) return rq_bits_dbl(1ull);
    const uint64_t b = rq_dbl_bits(x);
    return rq_bits_dbl(x > 0.0 ? b + 1 : b - 1);
}

// order-preserving map of a double onto uint64 (negative values reversed)
__device__ __forceinline__ uint64_t order_key(double t)
{
    const uint64_t b = rq_dbl_bits(t);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

// ---------------------------------------------------------------------------
// numpy-order float64 sum of NV sequences of length n, by ONE wavefront.
// VAL(k, v) fills v[0..NV) with element k of each sequence.
// lds: >= rq_npsum_lds_doubles<NV>() doubles, private to this wave.
// ---------------------------------------------------------------------------
template <int NV>
__host__ __device__ constexpr int npsum_lds_doubles()
{
    // leaf values [NV][128] + leaf (off,len) [128][2 ints = 1 double] + the tree's levels
    // [8][128] uint16 + their node counts [8] ints
    return NV * 128 + 128 + 256 + 4;
}

// numpy's pairwise tree over m <= 8192 elements (pairwise_sum: a node of len > 128
// elements splits at n2 = len / 2 rounded down to a multiple of 8), planned by one wave
// level by level -- no serial walk.  With len = 8k + r (r < 8), n2 = 8 floor(k/2): the
// children are 8 floor(k/2) and 8 ceil(k/2) + r elements, so only the LAST node of a
// level carries the remainder r = m % 8 and a level is its nodes' unit counts k (two
// nodes per lane: j = lane, lane + 64).  A leaf passes through to the next level
// unchanged, so the last level is the leaves left to right.  Leaves hold >= 64 elements
// unless m <= 128, hence <= 65 leaves and depth <= 7 (8192 = 1024 units, 6 halvings to
// 16 units, one more for the remainder).
// leaf[2L] / leaf[2L+1]: leaf L's offset / length; lev[d * 128 + j]: node j of level d's
// first child index at level d + 1 | (split << 8); cnt[d]: nodes at level d; tmp: 128
// ints of scratch.  Returns the leaf count; depth = the last level's index.
__device__ __forceinline__ int npsum_plan(int m, int* leaf, uint16_t* lev, int* cnt, int* tmp, int& depth)
{
    const int lane = lane_id();
    const int r = m & 7;
    const uint64_t lt = (1ull << lane) - 1;
    int n = 1, d = 0;
    int kA = lane == 0 ? (m >> 3) : 0, kB = 0;
    for (;;) {
        const bool vA = lane < n, vB = lane + 64 < n;
        const int lenA = 8 * kA + (lane == n - 1 ? r : 0);
        const int lenB = 8 * kB + (lane + 64 == n - 1 ? r : 0);
        const bool sA = vA && lenA > 128, sB = vB && lenB > 128;
        const uint64_t bA = __ballot(sA), bB = __ballot(sB);
        if ((bA | bB) == 0 || d == 7) {
            // leaves: exclusive prefix sum of the lengths (lane order, then lane + 64)
            const uint32_t iA = wave_scan_add(vA ? (uint32_t)lenA : 0u);
            const uint32_t iB = wave_scan_add(vB ? (uint32_t)lenB : 0u);
            const int totA = __builtin_amdgcn_readlane((int)iA, 63);
            if (vA) {
                leaf[2 * lane] = (int)iA - lenA;
                leaf[2 * lane + 1] = lenA;
            }
            if (vB) {
                leaf[2 * (lane + 64)] = totA + (int)iB - lenB;
                leaf[2 * (lane + 64) + 1] = lenB;
            }
            wave_lds_sync();
            depth = d;
            return n;
        }
        const int pA = popc(bA);
        const int cA = lane + popc(bA & lt);
        const int cB = lane + 64 + pA + popc(bB & lt);
        if (vA) {
            lev[d * 128 + lane] = (uint16_t)(cA | (sA ? 256 : 0));
            tmp[cA] = sA ? (kA >> 1) : kA;
            if (sA) tmp[cA + 1] = (kA + 1) >> 1;
        }
        if (vB) {
            lev[d * 128 + lane + 64] = (uint16_t)(cB | (sB ? 256 : 0));
            tmp[cB] = sB ? (kB >> 1) : kB;
            if (sB) tmp[cB + 1] = (kB + 1) >> 1;
        }
        if (lane == 0) cnt[d] = n;
        n += pA + popc(bB);
        ++d;
        wave_lds_sync();
        kA = lane < n ? tmp[lane] : 0;
        kB = lane + 64 < n ? tmp[lane + 64] : 0;
        wave_lds_sync();   // every lane's reads of tmp before the next level's writes
    }
}

// fold the leaf values leafv[s * 128 + L] up the planned tree in place, level by level
// (node j's children sit at indices >= j, and every read of a level precedes its
// writes): a split node is left + right in numpy's order, a pass-through node keeps its
// child's value bit for bit (-0.0 included).  The root's values end in cv (every lane).
template <int NV>
__device__ __forceinline__ void npsum_fold(int depth, const uint16_t* lev, const int* cnt, double* leafv,
                                           double cv[NV])
{
    const int lane = lane_id();
    for (int d = depth - 1; d >= 0; --d) {
        const int n = cnt[d];
        double vA[NV], vB[NV];
        const bool okA = lane < n, okB = lane + 64 < n;
        const int eA = okA ? lev[d * 128 + lane] : 0;
        const int eB = okB ? lev[d * 128 + lane + 64] : 0;
        const int cA = eA & 255, cB = eB & 255;
#pragma unroll
        for (int s = 0; s < NV; ++s) {
            vA[s] = leafv[s * 128 + cA];
            vB[s] = leafv[s * 128 + cB];
            if (eA & 256) vA[s] = vA[s] + leafv[s * 128 + cA + 1];
            if (eB & 256) vB[s] = vB[s] + leafv[s * 128 + cB + 1];
        }
        wave_lds_sync();
#pragma unroll
        for (int s = 0; s < NV; ++s) {
            if (okA) leafv[s * 128 + lane] = vA[s];
            if (okB) leafv[s * 128 + lane + 64] = vB[s];
        }
        wave_lds_sync();
    }
#pragma unroll
    for (int s = 0; s < NV; ++s) cv[s] = leafv[s * 128];
    wave_lds_sync();   // before the next chunk's plan reuses leafv as scratch
}

template <int NV, class VAL>
__device__ void wave_npsum(int64_t n, VAL&& val, double* lds, double out[NV])
{
    const int lane = lane_id();
    const int grp = lane >> 3, jj = lane & 7;
    double* leafv = lds;                                   // [NV][128]
    int* leaf = reinterpret_cast<int*>(lds + NV * 128);    // [128][2]
    uint16_t* levt = reinterpret_cast<uint16_t*>(lds + NV * 128 + 128);   // [8][128]
    int* lcnt = reinterpret_cast<int*>(lds + NV * 128 + 128 + 256);         // [8]

    double res[NV];
#pragma unroll
    for (int s = 0; s < NV; ++s) res[s] = 0.0;

    for (int64_t c0 = 0; c0 < n; c0 += 8192) {
        const int m = (int)((n - c0) < 8192 ? (n - c0) : 8192);
        // ---- the leaves of pairwise(m), left to right, and the tree above them ----
        int depth = 0;
        const int nleaf = npsum_plan(m, leaf, levt, lcnt, reinterpret_cast<int*>(leafv), depth);
        // ---- leaf values: 8 leaves per round, lane jj = accumulator jj ----
        for (int L0 = 0; L0 < nleaf; L0 += 8) {
            const int L = L0 + grp;
            const bool act = L < nleaf;
            const int off = act ? leaf[2 * L] : 0;
            const int len = act ? leaf[2 * L + 1] : 0;
            double r[NV];
#pragma unroll
            for (int s = 0; s < NV; ++s) r[s] = 0.0;
            const int lim = len - (len % 8);
            if (len >= 8) {
                val(c0 + off + jj, r);
                for (int i = 8; i < lim; i += 8) {
                    double v[NV];
                    val(c0 + off + i + jj, v);
#pragma unroll
                    for (int s = 0; s < NV; ++s) r[s] += v[s];
                }
            }
#pragma unroll
            for (int s = 0; s < NV; ++s) {
                double x = r[s];
                x = x + __shfl_xor(x, 1, 64);   // (r0+r1), (r2+r3), ...
                x = x + __shfl_xor(x, 2, 64);   // ((r0+r1)+(r2+r3)), ...
                x = x + __shfl_xor(x, 4, 64);   // (...)+((r4+r5)+(r6+r7))
                r[s] = x;
            }
            if (act && jj == 0) {
                double v[NV];
                if (len < 8) {
#pragma unroll
                    for (int s = 0; s < NV; ++s) r[s] = -0.0;
                }
                for (int i = (len >= 8 ? lim : 0); i < len; ++i) {
                    val(c0 + off + i, v);
#pragma unroll
                    for (int s = 0; s < NV; ++s) r[s] += v[s];
                }
#pragma unroll
                for (int s = 0; s < NV; ++s) leafv[s * 128 + L] = r[s];
            }
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // ---- the tree above the leaves, level by level ----
        double cv[NV];
        npsum_fold<NV>(depth, levt, lcnt, leafv, cv);
#pragma unroll
        for (int s = 0; s < NV; ++s) res[s] = res[s] + cv[s];
        __builtin_amdgcn_wave_barrier();
    }
#pragma unroll
    for (int s = 0; s < NV; ++s) out[s] = res[s];
}

// ---------------------------------------------------------------------------
// wave_npsum over a row log (the sweep's / replay's pivot rows): the same numpy
// order as wave_npsum, but a leaf's 8 accumulator lanes take 32 consecutive rows
// per trip (4 per lane, in the accumulators' order), so each load instruction of a
// trip covers whole 128 B lines of every column and no line is needed again by a
// later trip -- with ~6 waves per SIMD interleaving 8 leaves each, lines fetched
// for the next trip were evicted from L2 before use (1.5x the algorithmic bytes).
// TNEXT: the value of row k needs t[k + 1] (end past the last row), taken from the
// next lane on DPP (row_shl:1; lane 7 of a group from lane 0 by row_shr:7).
// LD(uint32_t k) -> Row (32-bit row offsets: saddr + voffset loads); VF(const Row&,
// double t_next, double* v).  n < 2^32.
// ---------------------------------------------------------------------------
__device__ __forceinline__ double dpp_shl1_f64(double x)
{
    const uint64_t b = rq_dbl_bits(x);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)b, 0x101, 0xF, 0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(b >> 32), 0x101, 0xF, 0xF, false);
    return rq_bits_dbl(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ double dpp_shr7_f64(double x)
{
    const uint64_t b = rq_dbl_bits(x);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)b, 0x117, 0xF, 0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(b >> 32), 0x117, 0xF, 0xF, false);
    return rq_bits_dbl(((uint64_t)hi << 32) | lo);
}

template <int NV, bool TNEXT, class Row, int TU = 8, class LD, class TLD, class VF>
__device__ void wave_npsum_rows(int64_t n, double end, LD&& ld, TLD&& tld, VF&& vf, double* lds,
                                double out[NV])
{
    const int lane = lane_id();
    const int grp = lane >> 3, jj = lane & 7;
    double* leafv = lds;
    int* leaf = reinterpret_cast<int*>(lds + NV * 128);
    uint16_t* levt = reinterpret_cast<uint16_t*>(lds + NV * 128 + 128);   // [8][128]
    int* lcnt = reinterpret_cast<int*>(lds + NV * 128 + 128 + 256);         // [8]
    double res[NV];
#pragma unroll
    for (int s = 0; s < NV; ++s) res[s] = 0.0;

    for (int64_t c0 = 0; c0 < n; c0 += 8192) {
        const int m = (int)((n - c0) < 8192 ? (n - c0) : 8192);
        int depth = 0;
        const int nleaf = npsum_plan(m, leaf, levt, lcnt, reinterpret_cast<int*>(leafv), depth);
        for (int L0 = 0; L0 < nleaf; L0 += 8) {
            const int L = L0 + grp;
            const bool act = L < nleaf;
            const int off = act ? leaf[2 * L] : 0;
            const int len = act ? leaf[2 * L + 1] : 0;
            double r[NV];
#pragma unroll
            for (int s = 0; s < NV; ++s) r[s] = 0.0;
            const int lim = len - (len % 8);
            // a trip: up to TU rows per lane (8 TU per group), all loads in flight at once
            for (int i = 0; i < lim; i += 8 * TU) {
                const int nu = (lim - i) >> 3 < TU ? (lim - i) >> 3 : TU;   // group-uniform
                const int64_t e0 = c0 + off + i + jj;
                Row R[TU];
#pragma unroll
                for (int u = 0; u < TU; ++u)
                    if (u < nu) R[u] = ld((uint32_t)(e0 + 8 * u));
                double tx = end;
                if constexpr (TNEXT) if (jj == 7) {
                    const int64_t ka = c0 + off + i + 8 * nu;   // the row after lane 7's last
                    if (ka < n) tx = tld((uint32_t)ka);
                }
#pragma unroll
                for (int u = 0; u < TU; ++u) {
                    if (u < nu) {
                        double tn = 0.0;
                        if constexpr (TNEXT) {
                            const double nb = dpp_shl1_f64(R[u].t);
                            const double w7 = u + 1 < nu ? dpp_shr7_f64(R[u + 1 < TU ? u + 1 : TU - 1].t) : tx;
                            tn = jj == 7 ? w7 : nb;
                        }
                        double v[NV];
                        vf(R[u], tn, v);
#pragma unroll
                        for (int s = 0; s < NV; ++s) r[s] = (u == 0 && i == 0) ? v[s] : r[s] + v[s];
                    }
                }
            }
#pragma unroll
            for (int s = 0; s < NV; ++s) {
                double x = r[s];
                x = x + __shfl_xor(x, 1, 64);
                x = x + __shfl_xor(x, 2, 64);
                x = x + __shfl_xor(x, 4, 64);
                r[s] = x;
            }
            if (act && jj == 0) {
                double v[NV];
                if (len < 8) {
#pragma unroll
                    for (int s = 0; s < NV; ++s) r[s] = -0.0;
                }
                for (int k = (len >= 8 ? lim : 0); k < len; ++k) {
                    const int64_t e = c0 + off + k;
                    const Row Rk = ld((uint32_t)e);
                    double tn = 0.0;
                    if constexpr (TNEXT) tn = e + 1 < n ? tld((uint32_t)(e + 1)) : end;
                    vf(Rk, tn, v);
#pragma unroll
                    for (int s = 0; s < NV; ++s) r[s] += v[s];
                }
#pragma unroll
                for (int s = 0; s < NV; ++s) leafv[s * 128 + L] = r[s];
            }
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        double cv[NV];
        npsum_fold<NV>(depth, levt, lcnt, leafv, cv);
#pragma unroll
        for (int s = 0; s < NV; ++s) res[s] = res[s] + cv[s];
        __builtin_amdgcn_wave_barrier();
    }
#pragma unroll
    for (int s = 0; s < NV; ++s) out[s] = res[s];
}

}  // namespace rq
