// rq_sweep_core.h -- per-event state machine shared by the two sweep kernels.
//
// Pivot-row aggregates (utils.py:38-56 / :84-121): for
// the pivot row at time t we need  sumR  = sum of the ranks of all sinks that
// already have a row (NaN cells skipped by pandas' mean), nvalid = their
// count, and cnt[K] = #sinks with rank <= K-1.  They change incrementally:
//   other event j : each edge (j,i) raises rank_i by one (NaN -> 1), so
//                   sumR += outdeg(j); sumF (the followers' part) += outdeg_F(j)
//   own post      : every follower's rank -> 0, so sumR -= sumF, sumF = 0
// Only the counts need per-sink state (rank_i in LDS) and wave ballots.
#pragma once
#include "rq_device.h"
#include "rq_internal.h"

namespace rq {

template <int NK>
struct Agg {
    int64_t sumR, sumF;
    int nvalid;
    int cnt[NK];
    int km1[NK];
    __device__ __forceinline__ void init(const int* Ks)
    {
        sumR = 0;
        sumF = 0;
        nvalid = 0;
#pragma unroll
        for (int q = 0; q < NK; ++q) {
            cnt[q] = 0;
            km1[q] = Ks[q] - 1;
        }
    }
    // other source's event: sinks col[e0..e1) in edge-list order (distinct)
    template <class COL>
    __device__ __forceinline__ void wall(int* rank, const COL* col, int e0, int e1, int odf, int lane)
    {
        int dvalid = 0;
        int dle[NK];
#pragma unroll
        for (int q = 0; q < NK; ++q) dle[q] = 0;
        for (int e = e0; e < e1; e += 64) {
            const int ee = e + lane;
            const bool act = ee < e1;
            int r = 0, c = 0;
            if (act) {
                c = (int)col[ee];
                r = rank[c];
                rank[c] = r < 0 ? 1 : r + 1;
            }
            const bool inv = act && r < 0;
            dvalid += popc(__ballot(inv));
#pragma unroll
            for (int q = 0; q < NK; ++q) {
                dle[q] += popc(__ballot(inv && 1 <= km1[q]));
                dle[q] -= popc(__ballot(act && r >= 0 && r == km1[q]));
            }
        }
        nvalid += dvalid;
#pragma unroll
        for (int q = 0; q < NK; ++q) cnt[q] += dle[q];
        sumR += e1 - e0;
        sumF += odf;
    }
    // own post: every follower's rank -> 0 (State.apply_event, opt_model.py:71-72)
    template <class COL>
    __device__ __forceinline__ void own(int* rank, const COL* fol, int F, int lane)
    {
        int dvalid = 0;
        int dle[NK];
#pragma unroll
        for (int q = 0; q < NK; ++q) dle[q] = 0;
        for (int f0 = 0; f0 < F; f0 += 64) {
            const int f = f0 + lane;
            const bool act = f < F;
            int r = 0, c = 0;
            if (act) {
                c = (int)fol[f];
                r = rank[c];
            }
            dvalid += popc(__ballot(act && r < 0));
#pragma unroll
            for (int q = 0; q < NK; ++q) dle[q] -= popc(__ballot(act && r >= 0 && r <= km1[q]));
            if (act) rank[c] = 0;
        }
#pragma unroll
        for (int q = 0; q < NK; ++q) cnt[q] += dle[q] + (0 <= km1[q] ? F : 0);
        nvalid += dvalid;
        sumR -= sumF;
        sumF = 0;
    }
};

// One pivot row per distinct event time; lane (row & 63) stages a row until
// its 64-row tile is written with one coalesced store per field.
template <int NK>
struct RowStage {
    double r_t, r_sum;
    int r_valid;
    int r_cnt[NK];
    int64_t nrow, cap;
    double last_t;
    double* Rt;
    double* Rs;
    uint32_t* Rv;
    uint32_t* Rc;
    __device__ __forceinline__ void init(double* t, double* s, uint32_t* v, uint32_t* c, int64_t cap_)
    {
        r_t = 0.0;
        r_sum = 0.0;
        r_valid = 0;
#pragma unroll
        for (int q = 0; q < NK; ++q) r_cnt[q] = 0;
        nrow = 0;
        cap = cap_;
        last_t = -RQ_INF;
        Rt = t;
        Rs = s;
        Rv = v;
        Rc = c;
    }
    // returns false when the capacity is exhausted
    __device__ __forceinline__ bool emit(double t, const Agg<NK>& g, int lane, int& status)
    {
        if (nrow > 0 && t == last_t) {
            // same timestamp as the previous row: pivot_table merges them
            status |= RQ_ST_TIE;
            const int64_t rr = nrow - 1;
            if ((nrow & 63) != 0) {
                if (lane == (int)(rr & 63)) {
                    r_sum = (double)g.sumR;
                    r_valid = g.nvalid;
#pragma unroll
                    for (int q = 0; q < NK; ++q) r_cnt[q] = g.cnt[q];
                }
            } else if (lane == 0) {
                Rs[rr] = (double)g.sumR;
                Rv[rr] = (uint32_t)g.nvalid;
#pragma unroll
                for (int q = 0; q < NK; ++q) Rc[rr * NK + q] = (uint32_t)g.cnt[q];
            }
            return true;
        }
        if (nrow >= cap) {
            status |= RQ_ST_ROWS_OVERFLOW;
            return false;
        }
        const int slot = (int)(nrow & 63);
        if (lane == slot) {
            r_t = t;
            r_sum = (double)g.sumR;
            r_valid = g.nvalid;
#pragma unroll
            for (int q = 0; q < NK; ++q) r_cnt[q] = g.cnt[q];
        }
        ++nrow;
        last_t = t;
        if (slot == 63) store(nrow - 64 + lane);
        return true;
    }
    __device__ __forceinline__ void store(int64_t rr)
    {
        Rt[rr] = r_t;
        Rs[rr] = r_sum;
        Rv[rr] = (uint32_t)r_valid;
#pragma unroll
        for (int q = 0; q < NK; ++q) Rc[rr * NK + q] = (uint32_t)r_cnt[q];
    }
    __device__ __forceinline__ void flush(int lane)
    {
        const int rem = (int)(nrow & 63);
        if (lane < rem) store(nrow - rem + lane);
    }
};

// optional (t, source index) event log, staged the same way
struct EvStage {
    double e_t;
    int e_src;
    int64_t n, cap;
    double* Et;
    int32_t* Es;
    __device__ __forceinline__ void init(double* t, int32_t* s, int64_t cap_)
    {
        e_t = 0.0;
        e_src = 0;
        n = 0;
        cap = cap_;
        Et = t;
        Es = s;
    }
    __device__ __forceinline__ void push(double t, int src, int lane, int& status)
    {
        if (n < cap) {
            const int slot = (int)(n & 63);
            if (lane == slot) {
                e_t = t;
                e_src = src;
            }
            if (slot == 63) {
                Et[n - 63 + lane] = e_t;
                Es[n - 63 + lane] = e_src;
            }
        } else {
            status |= RQ_ST_ROWS_OVERFLOW;
        }
        ++n;
    }
    __device__ __forceinline__ void flush(int lane)
    {
        if (n <= cap) {
            const int rem = (int)(n & 63);
            if (lane < rem) {
                Et[n - rem + lane] = e_t;
                Es[n - rem + lane] = e_src;
            }
        }
    }
};

// The RedQueen controller's exponentials: one Philox call per lane yields 128
// standard exponentials per batch; draw k of the batch lives in lane k>>1.
struct OptDraws {
    uint32_t seed, salt;
    uint64_t batch;
    int k;
    double x0, x1;
    __device__ __forceinline__ void init(uint32_t seed_)
    {
        seed = seed_;
        salt = kind_salt(RQ_SRC_OPT, true);
        batch = 0;
        k = 128;
        x0 = 0.0;
        x1 = 0.0;
    }
    __device__ __forceinline__ double next(int lane)
    {
        if (k == 128) {
            const uint64_t call = batch * 64 + lane;
            uint32_t c[4] = {(uint32_t)call, (uint32_t)(call >> 32), 0u, 0u};
            philox4x32_10(c, seed, salt);
            x0 = rq_std_exponential(rq_uniform53(c[0], c[1]));
            x1 = rq_std_exponential(rq_uniform53(c[2], c[3]));
            ++batch;
            k = 0;
        }
        const double x = bcast_d((k & 1) ? x1 : x0, k >> 1);
        ++k;
        return x;
    }
};

}  // namespace rq
