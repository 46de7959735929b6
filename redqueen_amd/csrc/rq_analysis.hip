// rq_analysis.hip -- gfx950 kernels for the analysis side of the hot path:
//
//   rq_oracle_dp    utils.oracle_ranking (utils.py:181-245): the offline
//                   oracle's backward dynamic program over a single-follower
//                   wall, J[r,k] = min(q/2 + J[0,k+1], s/2 w[k+1] (r+1)^2 +
//                   J[r+1,k+1]), then its forward policy walk.
//   rq_rank_table   utils.rank_of_src_in_df (utils.py:38-56): per-sink rank
//                   scan, pivot on unique t with the mean of duplicate
//                   (t, sink) cells, optional per-column forward fill.
//   rq_u_int        utils.u_int_opt (utils.py:59-81): rows of the rank table
//                   dotted with sqrt(s/q) over the followers, times dt,
//                   summed in numpy's pairwise order.
//   rq_log_rows /   State.get_dataframe (opt_model.py:85-97) for a whole batch
//   rq_log_expand   of event logs: one row per (event, sink of an edge of the
//                   event's source) in event order then edge-list order.
//
// None of these is a dense contraction (no MFMA); they are latency / HBM bound
// and laid out so that every global access of a wavefront is contiguous.
#include <hip/hip_runtime.h>

#include "rq_device.h"
#include "rq_internal.h"

#pragma clang fp contract(off)

using namespace rq;

// ============================================================================
// 1. oracle DP.  One workgroup per instance (a wall of n events, its own q, s).
//    Column k of J depends only on column k+1, so the columns run from k = n
//    down to 0 with one barrier each; rows r < min(k+1, n) are spread over the
//    threads.  Two column buffers (LDS when they fit, else global) alternate.
//    The decision lhs < rhs of every (r, k) is kept as one bit (ballot of a
//    wavefront's 64 consecutive rows), so the forward walk
//    (utils.py:230-238) needs no second pass over J:  n^2/8 bytes per instance.
//    Exactness: the reference evaluates 0.5*q + J[0,k+1] and
//    ((0.5*s)*w[k+1])*float((r+1)**2) + J[r+1,k+1] and keeps the first
//    argument of min() unless the second is strictly smaller -- restated
//    literally (no FMA: contract(off)).
//    Quirk kept: J is zero-initialised and row n of column n is never written,
//    so column n-1 reads J[n, n] = 0 (not n^2/2).
// ============================================================================
template <bool LDS>
__global__ __launch_bounds__(1024) void rq_oracle_dp_k(OracleArgs a)
{
    extern __shared__ double lds_od[];
    const int inst = blockIdx.x;
    const int64_t w0 = a.w_off[inst];
    const int64_t n = a.w_off[inst + 1] - w0 - 2;
    const double* w = a.w + w0;
    const double q = a.q[inst];
    const double s = a.s[inst];
    const int tid = threadIdx.x, nt = blockDim.x;
    const int64_t wpc = (n + 1 + 63) / 64;                    // 64-bit words per column
    uint64_t* bits = a.bits + (size_t)inst * a.bits_stride;   // [n+1 columns][wpc]
    double* c0 = LDS ? lds_od : a.gcol + (size_t)inst * 2 * (a.n_max + 2);
    double* c1 = c0 + (n + 2);
    if (n < 0) return;

    // column n+1: J[r, n+1] = r**2 / 2 (np.arange(n + 1) ** 2 / 2)
    for (int64_t r = tid; r <= n; r += nt) c0[r] = (double)(r * r) / 2.0;
    __syncthreads();
    double* cur = c0;   // column k+1
    double* nxt = c1;   // column k
    const double hq = 0.5 * q;
    const double hs = 0.5 * s;
    for (int64_t k = n; k >= 0; --k) {
        const int64_t m = (k + 1 < n) ? k + 1 : n;   // rows written in column k
        const double lhs = hq + cur[0];
        const double ck = hs * w[k + 1];
        // rows are swept by whole wavefronts so each ballot covers 64 consecutive rows
        for (int64_t rb = (int64_t)(tid & ~63); rb < m; rb += nt) {
            const int64_t r = rb + (tid & 63);
            bool post = false;
            if (r < m) {
                const double r1 = (double)((r + 1) * (r + 1));
                const double rhs = ck * r1 + cur[r + 1];
                post = lhs < rhs;
                nxt[r] = (rhs < lhs) ? rhs : lhs;     // Python min(lhs, rhs)
            }
            const uint64_t b = __ballot(post);
            if ((tid & 63) == 0) bits[k * wpc + (rb >> 6)] = b;
        }
        // row n of column n: J[n, n] = 0, never written by the reference (column n-1
        // reads it); the other rows >= m of a column are never read again
        if (tid == 0 && k == n) nxt[n] = 0.0;
        __syncthreads();
        double* tmp = cur;
        cur = nxt;
        nxt = tmp;
    }
    // forward policy walk (utils.py:230-238): one lane, decisions from the bits
    if (tid == 0) {
        const int64_t o = a.out_off[inst];
        a.cost[inst] = cur[0];   // J[0, 0]
        int64_t rk = 0;
        a.ranks[o] = 0;
        for (int64_t k = 0; k < n; ++k) {
            const uint64_t word = bits[k * wpc + (rk >> 6)];
            const bool post = (word >> (rk & 63)) & 1ull;
            a.events[o + k] = post ? 1 : 0;
            rk = post ? 0 : rk + 1;
            a.ranks[o + k + 1] = (int32_t)rk;
        }
        a.events[o + n] = 0;
    }
}

hipError_t rq_launch_oracle_dp(const OracleArgs& a, bool lds, hipStream_t s)
{
    if (a.n_inst <= 0) return hipSuccess;
    const int nt = a.n_max + 1 >= 4096 ? 1024 : 256;
    if (lds) {
        const size_t bytes = 2 * (size_t)(a.n_max + 2) * sizeof(double);
        hipLaunchKernelGGL(rq_oracle_dp_k<true>, dim3(a.n_inst), dim3(nt), bytes, s, a);
    } else {
        hipLaunchKernelGGL(rq_oracle_dp_k<false>, dim3(a.n_inst), dim3(nt), 0, s, a);
    }
    return hipGetLastError();
}

// ============================================================================
// 2. rank table.  One wavefront per 64 sink columns; lane c owns column
//    blockIdx*64 + c.  The rows (df order, t non-decreasing) are read 64 at a
//    time, coalesced, and walked in order with register broadcasts: the owning
//    lane advances its column's position / last-own-post counters
//    (steps_to, utils.py:43-46) and accumulates the (t, sink) cell; when t
//    changes every lane emits its cell for the finished t -- the mean of the
//    cell's ranks, else (fill) the column's previous value, else NaN -- so a
//    table row is one 8*64-byte contiguous store per wavefront.
// ============================================================================
__global__ __launch_bounds__(64) void rq_rank_table_k(RankTableArgs a)
{
    const int lane = lane_id();
    const int64_t c = (int64_t)blockIdx.x * 64 + lane;
    const bool own_col = c < a.n_cols;
    const double NaN = __builtin_nan("");
    int64_t pos = 0, last = 0;
    double csum = 0.0;
    int ccnt = 0;
    double prev = NaN;           // the column's last value (ffill)
    int64_t row = -1;            // table row of the current t
    double cur_t = 0.0;
    int err = 0;
    auto emit = [&]() {
        double v;
        if (ccnt > 0) {
            v = csum / (double)ccnt;
            prev = v;
        } else {
            v = a.fill ? prev : NaN;
        }
        if (own_col && row < a.n_t) a.table[row * a.n_cols + c] = v;
        if (lane == 0 && row < a.n_t && blockIdx.x == 0) a.index[row] = cur_t;
        csum = 0.0;
        ccnt = 0;
    };
    for (int64_t i0 = 0; i0 < a.n_rows; i0 += 64) {
        const int64_t i = i0 + lane;
        double ti = 0.0;
        int key = -1;   // col * 2 + (src == src_id)
        if (i < a.n_rows) {
            ti = a.t[i];
            key = a.col[i] * 2 + (a.src[i] == a.src_id ? 1 : 0);
        }
        const int cnt = (int)((a.n_rows - i0) < 64 ? (a.n_rows - i0) : 64);
        for (int j = 0; j < cnt; ++j) {
            const double tj = __shfl(ti, j, 64);
            const int kj = __shfl(key, j, 64);
            if (row < 0 || tj != cur_t) {
                if (row >= 0) {
                    if (tj < cur_t) err = 1;   // df not sorted by t
                    emit();
                }
                ++row;
                cur_t = tj;
            }
            if ((int64_t)(kj >> 1) == c) {
                ++pos;
                if (kj & 1) last = pos;
                csum += (double)(pos - last);
                ++ccnt;
            }
        }
    }
    if (row >= 0) emit();
    if (lane == 0 && blockIdx.x == 0) {
        if (row + 1 != a.n_t) err |= 2;
        a.err[0] = err;
    }
}

hipError_t rq_launch_rank_table(const RankTableArgs& a, hipStream_t s)
{
    const unsigned blocks = (unsigned)((a.n_cols + 63) / 64);
    hipLaunchKernelGGL(rq_rank_table_k, dim3(blocks), dim3(64), 0, s, a);
    return hipGetLastError();
}

// ============================================================================
// 3. u_int_opt.  Row k of the rank table: u_k = sum_f table[k, col_f] * w_f
//    (follower order), x_k = u_k * dt_k with dt_k = t_{k+1} - t_k and the last
//    one end_time - t_last (np.diff(concatenate([index, [end_time]]))); the
//    result is numpy's pairwise np.sum of x (one wavefront, wave_npsum).
//    NaN ranks (a follower with no row yet) propagate exactly as in numpy.
// ============================================================================
__global__ __launch_bounds__(256) void rq_u_int_rows_k(UIntArgs a)
{
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= a.n_t) return;
    double u = 0.0;
    for (int f = 0; f < a.n_f; ++f) u = u + a.table[k * a.n_cols + a.fcol[f]] * a.wts[f];
    const double dt = (k + 1 < a.n_t ? a.index[k + 1] : a.end) - a.index[k];
    a.x[k] = u * dt;
}

__global__ __launch_bounds__(64) void rq_u_int_sum_k(UIntArgs a)
{
    extern __shared__ double lds_ui[];
    double out[1];
    const double* x = a.x;
    wave_npsum<1>(a.n_t, [&](int64_t k, double v[1]) { v[0] = x[k]; }, lds_ui, out);
    if (lane_id() == 0) a.out[0] = out[0];
}

hipError_t rq_launch_u_int(const UIntArgs& a, hipStream_t s)
{
    if (a.n_t > 0) {
        hipLaunchKernelGGL(rq_u_int_rows_k, dim3((unsigned)((a.n_t + 255) / 256)), dim3(256), 0, s, a);
        if (hipGetLastError() != hipSuccess) return hipErrorLaunchFailure;
    }
    hipLaunchKernelGGL(rq_u_int_sum_k, dim3(1), dim3(64), npsum_lds_doubles<1>() * sizeof(double), s, a);
    return hipGetLastError();
}

// ============================================================================
// 4. event-log expansion.  rows: one wavefront per replica sums the out-degrees
//    of its events; a single block turns the per-replica counts into offsets.
//    expand: one block per replica walks its events in chunks of 1024: a block
//    scan of the out-degrees gives each event's first row, then every thread
//    takes consecutive ROWS (binary search of its event in the chunk's offsets in
//    LDS), so the 40 bytes per row go out as coalesced column stores.
// ============================================================================
__global__ __launch_bounds__(256) void rq_log_rows_k(LogArgs a)
{
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= a.n_rep) return;
    const int lane = lane_id();
    const int64_t n = a.counts[r * 4 + 2];
    const int32_t* src = a.ev_src + r * a.ev_cap;
    int64_t sum = 0;
    for (int64_t k = lane; k < n; k += 64) {
        const int j = src[k];
        sum += a.csr_ptr[j + 1] - a.csr_ptr[j];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
    if (lane == 0) a.row_off[r + 1] = sum;
}

__global__ __launch_bounds__(1024) void rq_log_scan_k(LogArgs a)
{
    __shared__ int64_t wsum[16];
    __shared__ int64_t carry;
    const int tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
    if (tid == 0) {
        carry = 0;
        a.row_off[0] = 0;
    }
    __syncthreads();
    for (int64_t b = 0; b < a.n_rep; b += 1024) {
        const int64_t i = b + tid;
        int64_t v = i < a.n_rep ? a.row_off[i + 1] : 0;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int64_t u = __shfl_up(v, o, 64);
            if (lane >= o) v += u;
        }
        if (lane == 63) wsum[w] = v;
        __syncthreads();
        int64_t pre = carry;
        for (int q = 0; q < w; ++q) pre += wsum[q];
        if (i < a.n_rep) a.row_off[i + 1] = pre + v;   // inclusive prefix of counts
        __syncthreads();
        if (tid == 1023) carry = pre + v;
        __syncthreads();
    }
}

__global__ __launch_bounds__(1024) void rq_log_expand_k(LogArgs a)
{
    constexpr int NT = 1024, CH = 1024, NW = NT / 64;   // one event per thread per chunk
    __shared__ int64_t off[CH + 1];
    __shared__ int32_t sj[CH];
    __shared__ double stt[CH];
    __shared__ double std_[CH];
    __shared__ int64_t wsum[NW];
    __shared__ double state_time;   // State.time after the previous chunk (accumulated)
    __shared__ int any_dirty;
    const int64_t r = blockIdx.x;
    const int tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
    const int64_t n = a.counts[r * 4 + 2];
    const double* T = a.ev_t + r * a.ev_cap;
    const int32_t* J = a.ev_src + r * a.ev_cap;
    int64_t row0 = a.row_off[r];
    if (tid == 0) state_time = a.start;
    for (int64_t c0 = 0; c0 < n; c0 += CH) {
        const int m = (int)((n - c0) < CH ? (n - c0) : CH);
        if (tid == 0) any_dirty = 0;
        __syncthreads();
        // this thread's event: degree + a block exclusive scan.  time_delta follows the
        // reference's State: time_delta_k = t_k - time_{k-1}, time_k = time_{k-1} +
        // time_delta_k (opt_model.py:68, :304).  time_k == t_k unless the subtraction
        // rounded (t_k > 2 time_{k-1}: early events, long gaps), and the next exact
        // subtraction heals it; so every event assumes time_{k-1} == t_{k-1} and one
        // thread redoes the chain from each event where that fails ("dirty").
        const int e = tid;
        int64_t d = 0;
        bool dirty = false;
        if (e < m) {
            const int j = J[c0 + e];
            const double tk = T[c0 + e];
            d = a.csr_ptr[j + 1] - a.csr_ptr[j];
            sj[e] = j;
            stt[e] = tk;
            const double sp = e > 0 ? T[c0 + e - 1] : state_time;
            const double td = tk - sp;
            std_[e] = td;
            dirty = sp + td != tk;
        }
        if (dirty) any_dirty = 1;
        int64_t v = d;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int64_t u = __shfl_up(v, o, 64);
            if (lane >= o) v += u;
        }
        if (lane == 63) wsum[w] = v;
        __syncthreads();
        int64_t pre = 0, chunk_rows = 0;
        for (int q = 0; q < NW; ++q) {
            pre += q < w ? wsum[q] : 0;
            chunk_rows += wsum[q];
        }
        if (e < m) off[e] = pre + v - d;
        if (tid == 0) off[m] = chunk_rows;
        __syncthreads();
        if (tid == 0) {
            // the accumulated chain, sequentially, in a chunk where some event's
            // time != t (rare: the chunk's speculative values are kept otherwise)
            double s = state_time;
            if (any_dirty)
                for (int k = 0; k < m; ++k) {
                    const double td = stt[k] - s;
                    std_[k] = td;
                    s = s + td;
                }
            state_time = any_dirty ? s : stt[m - 1];
        }
        __syncthreads();
        // rows of this chunk, one per thread, coalesced column stores
        for (int64_t x = tid; x < chunk_rows; x += NT) {
            int lo = 0, hi = m;   // last e with off[e] <= x
            while (hi - lo > 1) {
                const int mid = (lo + hi) >> 1;
                if (off[mid] <= x) lo = mid;
                else hi = mid;
            }
            const int ev = lo;
            const int j = sj[ev];
            const int64_t rr = row0 + x;
            a.event_id[rr] = 100 + c0 + ev;
            a.time_delta[rr] = std_[ev];
            a.src_id[rr] = a.src_ids[j];
            a.t[rr] = stt[ev];
            a.sink_id[rr] = a.sink_ids[a.csr_col[a.csr_ptr[j] + (x - off[ev])]];
        }
        row0 += chunk_rows;
        __syncthreads();
    }
}

hipError_t rq_launch_log_rows(const LogArgs& a, hipStream_t s)
{
    hipLaunchKernelGGL(rq_log_rows_k, dim3((unsigned)((a.n_rep + 3) / 4)), dim3(256), 0, s, a);
    if (hipGetLastError() != hipSuccess) return hipErrorLaunchFailure;
    hipLaunchKernelGGL(rq_log_scan_k, dim3(1), dim3(1024), 0, s, a);
    return hipGetLastError();
}

hipError_t rq_launch_log_expand(const LogArgs& a, hipStream_t s)
{
    hipLaunchKernelGGL(rq_log_expand_k, dim3((unsigned)a.n_rep), dim3(1024), 0, s, a);
    return hipGetLastError();
}
