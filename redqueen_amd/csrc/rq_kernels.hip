// rq_kernels.hip -- the gfx950 engine: stream generation, RedQueen sweep,
// metric scan, df replay.  Launch wrappers at the bottom are called by the
// C ABI in rq_api.cpp.
//
// Data layout in HBM (one chunk of C replicas in flight):
//   streams  f64  [C][capsum]          per-source clean arrival times, source j
//                                      at [st_off[j], st_off[j] + cap[j])
//   slen     i32  [C][n_str]           stream lengths
//   rows     SoA  [C][cap_rows] x {t f64, sumR f64, nvalid u32, cnt u32[nK]}
//                                      one record per pivot row (unique event time)
//   sall     i32  [C]                  sink columns S_all seen by the replica
//
// Kernel roles (reference file:line they replace):
//   rq_gen_streams  Poisson :424-433, Poisson2 :396-405, Hawkes :466-490,
//                   PiecewiseConst :642-663, RealData :722-750 -- one lane per
//                   (replica, source), 256 replicas of ONE source per block so a
//                   block never diverges on the source kind.
//   rq_sweep        Manager.run_dynamic :241-314 + Opt.get_next_interval
//                   :502-544 + State.apply_event :61-83 + the per-row part of
//                   rank_of_src_in_df utils.py:38-56 -- one wavefront per
//                   replica; lanes own sources (arrival heads) and sinks
//                   (feed ranks in LDS); u(t) enters as the O(1) increment c_j.
//   rq_scan         time_in_top_k :84-98, average_rank :101-114, int_r_2
//                   :117-121 -- one wavefront per replica, numpy sum order.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rq_device.h"
#include "rq_internal.h"

#pragma clang fp contract(off)

using namespace rq;

// ============================================================================
// 1. arrival streams
// ============================================================================
__global__ __launch_bounds__(256) void rq_gen_streams(GenArgs a)
{
    const int64_t rl = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int j = blockIdx.y;
    if (rl >= a.n_chunk) return;
    const int64_t i = a.chunk0 + rl;
    const bool is_ctrl = j == a.ctrl_idx;
    const int kind = is_ctrl ? a.ctrl_stream_kind : a.kind[j];

    const int64_t k = a.seed_mod > 0 ? i % a.seed_mod : i;
    uint32_t seed;
    if (is_ctrl) {
        seed = a.ctrl_seed ? a.ctrl_seed[i] : a.ctrl_seed0 + (uint32_t)k;
    } else if (a.randomize) {
        const uint32_t u = a.world_seed ? a.world_seed[i] : a.world_seed0 + (uint32_t)k;
        seed = u + 99u * (uint32_t)a.orig_idx[j];
    } else {
        seed = a.seed[j];
    }
    PhiloxStream ps(seed, kind_salt(kind, is_ctrl));

    double* out = a.streams + rl * a.capsum + a.st_off[j];
    const int cap = a.cap[j];
    const double start = a.start, end = a.end;
    int n = 0;
    bool ovf = false;
#define RQ_EMIT(tv)                      \
    do {                                 \
        if (n < cap) {                   \
            out[n++] = (tv);             \
        } else {                         \
            ovf = true;                  \
        }                                \
    } while (0)

    if (kind == RQ_SRC_POISSON || kind == RQ_SRC_POISSON2) {
        const double rate = is_ctrl ? a.ctrl_rate[i] : a.p0[j];
        if (rate > 0.0) {
            const double inv = 1.0 / rate;
            double t = start;
            for (;;) {
                t = t + rq_std_exponential(ps.next()) * inv;
                if (!(t <= end)) break;
                RQ_EMIT(t);
                if (ovf) break;
            }
        }
    } else if (kind == RQ_SRC_HAWKES) {
        const double l0 = a.p0[j], alpha = a.p1[j], nbeta = -a.p2[j];
        double tau = start, eta = 0.0;
        bool done = false;
        while (!done && !ovf) {
            const double B = l0 + eta;
            if (!(B > 0.0)) break;
            const double inv = 1.0 / B;
            double t = tau;
            for (;;) {
                const double x = rq_std_exponential(ps.next());
                const double v = ps.next();
                const double tc = t + x * inv;
                if (!(tc <= end)) {
                    done = true;
                    break;
                }
                const double decay = rq_exp(nbeta * (tc - tau));
                const double rate = l0 + eta * decay;
                if (v < rate / B) {
                    eta = eta * decay + alpha;
                    tau = tc;
                    RQ_EMIT(tc);
                    break;
                }
                t = tc;
            }
        }
    } else if (kind == RQ_SRC_PWCONST) {
        const int off = a.arr_off[j], na = a.arr_n[j];
        const double* ct = a.arr_a + off;
        const double* rt = a.arr_b + off;
        double mx = rt[0];
        for (int q = 1; q < na; ++q) mx = rt[q] > mx ? rt[q] : mx;
        if (mx > 0.0) {
            const double inv = 1.0 / mx;
            double t = start;
            for (;;) {
                t = t + rq_std_exponential(ps.next()) * inv;
                if (!(t <= end)) break;
                const double v = ps.next();
                int lo = 0, hi = na;   // bisect_right(change_times, t)
                while (lo < hi) {
                    const int mid = (lo + hi) >> 1;
                    if (t < ct[mid]) hi = mid;
                    else lo = mid + 1;
                }
                int idx = lo - 1;
                if (idx < 0) idx += na;
                if (v < rt[idx] / mx) {
                    RQ_EMIT(t);
                    if (ovf) break;
                }
            }
        }
    } else if (kind == RQ_SRC_REALDATA) {
        // host pre-sorted, filtered to [start, end]
        const int off = a.arr_off[j], na = a.arr_n[j];
        for (int q = 0; q < na && !ovf; ++q) RQ_EMIT(a.arr_a[off + q]);
    }
#undef RQ_EMIT
    a.slen[rl * a.n_str + j] = n;
    if (ovf) atomicOr(&a.status[i], RQ_ST_STREAM_OVERFLOW);
}

// ============================================================================
// 2. sweep: one wavefront per replica
// ============================================================================
template <int SPL, int NK>
__global__ __launch_bounds__(256) void rq_sweep(SweepArgs a)
{
    extern __shared__ int lds_rank[];
    const int lane = lane_id();
    const int w = threadIdx.x >> 6;
    const int64_t rl = (int64_t)blockIdx.x * a.wpb + w;
    if (rl >= a.n_chunk) return;
    const int64_t i = a.chunk0 + rl;
    const int g = (int)(i / a.n_rep);

    int* rank = lds_rank + (size_t)w * a.n_sinks_pad;
    for (int c = lane; c < a.n_sinks; c += 64) rank[c] = -1;   // NaN: no row yet

    // ---- arrival heads: lane owns sources [lane*SPL, lane*SPL+SPL) ----
    const double* st = a.streams + rl * a.capsum;
    const int* slen = a.slen + rl * a.n_str;
    double head[SPL];
    int pos[SPL], len[SPL], off[SPL];
#pragma unroll
    for (int q = 0; q < SPL; ++q) {
        const int j = lane * SPL + q;
        if (j < a.n_str) {
            off[q] = a.st_off[j];
            len[q] = slen[j];
            pos[q] = 0;
            head[q] = len[q] > 0 ? st[off[q]] : RQ_INF;
        } else {
            off[q] = 0;
            len[q] = 0;
            pos[q] = 0;
            head[q] = RQ_INF;
        }
    }
    double lmin = RQ_INF;
    int larg = 0;
#pragma unroll
    for (int q = 0; q < SPL; ++q)
        if (head[q] < lmin) {
            lmin = head[q];
            larg = q;
        }

    // ---- controlled broadcaster ----
    const bool opt = a.ctrl_kind == RQ_SRC_OPT;
    double opt_next = opt ? a.start : RQ_INF;
    const int64_t k = a.seed_mod > 0 ? i % a.seed_mod : i;
    const uint32_t oseed = a.ctrl_seed ? a.ctrl_seed[i] : a.ctrl_seed0 + (uint32_t)k;
    const uint32_t osalt = kind_salt(RQ_SRC_OPT, true);
    uint64_t obatch = 0;
    int okk = 128;          // index inside the current batch of 128 exponentials
    double ox0 = 0.0, ox1 = 0.0;
    const double* invc = a.inv_c + (int64_t)g * a.n_str;

    // ---- pivot-row aggregates (Appendix B of SURVEY.md) ----
    int64_t sumR = 0, sumF = 0;
    int nvalid = 0;
    int cnt[NK];
    int Km1[NK];
#pragma unroll
    for (int q = 0; q < NK; ++q) {
        cnt[q] = 0;
        Km1[q] = a.Ks[q] - 1;
    }

    // row staging: lane (row & 63) holds a row until its tile is flushed
    double r_t = 0.0, r_sum = 0.0;
    int r_valid = 0;
    int r_cnt[NK];
#pragma unroll
    for (int q = 0; q < NK; ++q) r_cnt[q] = 0;
    const int64_t rbase = rl * a.cap_rows;
    double* Rt = a.rows_t + rbase;
    double* Rs = a.rows_sum + rbase;
    uint32_t* Rv = a.rows_valid + rbase;
    uint32_t* Rc = a.rows_cnt + rbase * NK;   // [row][NK]
    int64_t nrow = 0;
    double last_t = -RQ_INF;

    // event log staging
    const bool evlog = a.ev_t != nullptr;
    double e_t = 0.0;
    int e_src = 0;
    double* Et = evlog ? a.ev_t + i * a.ev_cap : nullptr;
    int32_t* Es = evlog ? a.ev_src + i * a.ev_cap : nullptr;

    int64_t n_events = 0, posts = 0, world = 0;
    int status = 0;
    const int64_t maxev = a.max_events;

    for (;;) {
        if (maxev >= 0 && n_events >= maxev) break;
        // -------- next event: min over lanes, ties -> lowest lane/source --------
        const double tw = wave_min(lmin);
        const uint64_t cand = __ballot(lmin == tw);
        const int wl = cand ? (__ffsll((unsigned long long)cand) - 1) : 0;
        const int wq = bcast_i(larg, wl);
        const int jw = wl * SPL + wq;
        bool own;
        double tev;
        if (opt) {
            own = opt_next < tw || (opt_next == tw && (tw == RQ_INF || a.ctrl_src_id < a.src_id[jw]));
            tev = own ? opt_next : tw;
        } else {
            own = jw == a.ctrl_idx;
            tev = tw;
        }
        if (!(tev <= a.end)) break;

        // event log
        if (evlog) {
            if (n_events < a.ev_cap) {
                const int slot = (int)(n_events & 63);
                if (lane == slot) {
                    e_t = tev;
                    e_src = own ? a.ctrl_idx : jw;
                }
                if (slot == 63) {
                    Et[n_events - 63 + lane] = e_t;
                    Es[n_events - 63 + lane] = e_src;
                }
            } else {
                status |= RQ_ST_ROWS_OVERFLOW;
            }
        }
        ++n_events;

        int nsinks;
        if (own) {
            // -------- own post: every follower's rank -> 0 (opt_model.py:71-72) --------
            const int F = a.n_fol;
            nsinks = F;
            int dvalid = 0;
            int dle[NK];
#pragma unroll
            for (int q = 0; q < NK; ++q) dle[q] = 0;
            for (int f0 = 0; f0 < F; f0 += 64) {
                const int f = f0 + lane;
                const bool act = f < F;
                int r = 0;
                int c = 0;
                if (act) {
                    c = a.fol[f];
                    r = rank[c];
                }
                const bool inv = act && r < 0;
                dvalid += popc(__ballot(inv));
#pragma unroll
                for (int q = 0; q < NK; ++q) dle[q] -= popc(__ballot(act && r >= 0 && r <= Km1[q]));
                if (act) rank[c] = 0;
            }
#pragma unroll
            for (int q = 0; q < NK; ++q) cnt[q] += dle[q] + (0 <= Km1[q] ? F : 0);
            nvalid += dvalid;
            sumR -= sumF;
            sumF = 0;
            if (opt) {
                opt_next = RQ_INF;
            } else {
                // controlled stream (Poisson2 / PiecewiseConst / RealData): advance its head
#pragma unroll
                for (int q = 0; q < SPL; ++q)
                    if (lane == wl && q == wq) {
                        ++pos[q];
                        head[q] = pos[q] < len[q] ? st[off[q] + pos[q]] : RQ_INF;
                    }
            }
            if (F > 0) ++posts;
        } else {
            // -------- other source jw --------
#pragma unroll
            for (int q = 0; q < SPL; ++q)
                if (lane == wl && q == wq) {
                    ++pos[q];
                    head[q] = pos[q] < len[q] ? st[off[q] + pos[q]] : RQ_INF;
                }
            if (opt) {
                // one Exp(c_j) draw per non-own event (opt_model.py:536-544)
                if (okk == 128) {
                    const uint64_t call = obatch * 64 + lane;
                    uint32_t c[4] = {(uint32_t)call, (uint32_t)(call >> 32), 0u, 0u};
                    philox4x32_10(c, oseed, osalt);
                    ox0 = rq_std_exponential(rq_uniform53(c[0], c[1]));
                    ox1 = rq_std_exponential(rq_uniform53(c[2], c[3]));
                    ++obatch;
                    okk = 0;
                }
                const double x = bcast_d((okk & 1) ? ox1 : ox0, okk >> 1);
                ++okk;
                const double ic = invc[jw];
                const double e = ic > 0.0 ? x * ic : RQ_INF;
                const double c2 = tev + e;
                if (c2 < opt_next) opt_next = c2;
            }
            const int e0 = a.csr_ptr[jw], e1 = a.csr_ptr[jw + 1];
            nsinks = e1 - e0;
            int dvalid = 0;
            int dle[NK];
#pragma unroll
            for (int q = 0; q < NK; ++q) dle[q] = 0;
            for (int e = e0; e < e1; e += 64) {
                const int ee = e + lane;
                const bool act = ee < e1;
                int r = 0, c = 0;
                if (act) {
                    c = a.csr_col[ee];
                    r = rank[c];
                    rank[c] = r < 0 ? 1 : r + 1;
                }
                const bool inv = act && r < 0;
                dvalid += popc(__ballot(inv));
#pragma unroll
                for (int q = 0; q < NK; ++q) {
                    dle[q] += popc(__ballot(inv && 1 <= Km1[q]));
                    dle[q] -= popc(__ballot(act && r >= 0 && r == Km1[q]));
                }
            }
            nvalid += dvalid;
#pragma unroll
            for (int q = 0; q < NK; ++q) cnt[q] += dle[q];
            sumR += nsinks;
            sumF += a.outdeg_f[jw];
            if (nsinks > 0) ++world;
        }

        // lane-local min refresh for the lane whose head moved
        if (lane == wl) {
            lmin = RQ_INF;
            larg = 0;
#pragma unroll
            for (int q = 0; q < SPL; ++q)
                if (head[q] < lmin) {
                    lmin = head[q];
                    larg = q;
                }
        }

        // -------- pivot row --------
        if (nsinks > 0) {
            if (nrow > 0 && tev == last_t) {
                // same timestamp as the previous row: pivot_table merges them
                status |= RQ_ST_TIE;
                const int64_t rr = nrow - 1;
                if ((nrow & 63) != 0) {
                    if (lane == (int)(rr & 63)) {
                        r_sum = (double)sumR;
                        r_valid = nvalid;
#pragma unroll
                        for (int q = 0; q < NK; ++q) r_cnt[q] = cnt[q];
                    }
                } else if (lane == 0 && rr < a.cap_rows) {
                    Rs[rr] = (double)sumR;
                    Rv[rr] = (uint32_t)nvalid;
#pragma unroll
                    for (int q = 0; q < NK; ++q) Rc[rr * NK + q] = (uint32_t)cnt[q];
                }
            } else {
                if (nrow >= a.cap_rows) {
                    status |= RQ_ST_ROWS_OVERFLOW;
                    break;
                }
                const int slot = (int)(nrow & 63);
                if (lane == slot) {
                    r_t = tev;
                    r_sum = (double)sumR;
                    r_valid = nvalid;
#pragma unroll
                    for (int q = 0; q < NK; ++q) r_cnt[q] = cnt[q];
                }
                ++nrow;
                last_t = tev;
                if (slot == 63) {
                    const int64_t rr = nrow - 64 + lane;
                    Rt[rr] = r_t;
                    Rs[rr] = r_sum;
                    Rv[rr] = (uint32_t)r_valid;
#pragma unroll
                    for (int q = 0; q < NK; ++q) Rc[rr * NK + q] = (uint32_t)r_cnt[q];
                }
            }
        }
    }

    // flush the partial tiles
    {
        const int rem = (int)(nrow & 63);
        if (lane < rem) {
            const int64_t rr = nrow - rem + lane;
            Rt[rr] = r_t;
            Rs[rr] = r_sum;
            Rv[rr] = (uint32_t)r_valid;
#pragma unroll
            for (int q = 0; q < NK; ++q) Rc[rr * NK + q] = (uint32_t)r_cnt[q];
        }
        if (evlog && n_events <= a.ev_cap) {
            const int erem = (int)(n_events & 63);
            if (lane < erem) {
                Et[n_events - erem + lane] = e_t;
                Es[n_events - erem + lane] = e_src;
            }
        }
    }
    if (lane == 0) {
        int64_t* cnto = a.counts + i * 4;
        cnto[0] = posts;
        cnto[1] = world;
        cnto[2] = n_events;
        cnto[3] = nrow;
        a.sall[rl] = nvalid;
        if (nrow == 0) status |= RQ_ST_EMPTY;
        if (status) atomicOr(&a.status[i], status);
    }
}

// ============================================================================
// 3. scan: numpy-order integrals over the pivot rows, one wavefront per replica
// ============================================================================
template <int NK>
__global__ __launch_bounds__(256) void rq_scan(ScanArgs a)
{
    constexpr int NV = NK + 2;
    extern __shared__ double lds_scan[];
    const int w = threadIdx.x >> 6;
    const int64_t rl = (int64_t)blockIdx.x * 4 + w;
    if (rl >= a.n_chunk) return;
    const int64_t i = a.chunk0 + rl;
    double* lds = lds_scan + (size_t)w * npsum_lds_doubles<NV>();

    const int64_t n = a.nrows_from_counts ? a.counts[i * 4 + 3] : a.nrows;
    const double S = (double)(a.sall ? a.sall[rl] : a.ncols);
    const int64_t rbase = a.row_stride * rl;
    const double* Rt = a.rows_t + rbase;
    const double* Rs = a.rows_sum + rbase;
    const uint32_t* Rv = a.rows_valid + rbase;
    const uint32_t* Rc = a.rows_cnt + rbase * NK;
    const double end = a.end;
    double* out = a.metrics + i * NV;

    if (n <= 0) {
        if (lane_id() < NV) out[lane_id()] = __builtin_nan("");
        return;
    }
    auto val = [&](int64_t kk, double* v) {
        const double t0 = Rt[kk];
        const double t1 = kk + 1 < n ? Rt[kk + 1] : end;
        const double dt = t1 - t0;
        const double m = Rs[kk] / (double)Rv[kk];
#pragma unroll
        for (int q = 0; q < NK; ++q) v[q] = ((double)Rc[kk * NK + q] / S) * dt;
        v[NK] = m * dt;
        v[NK + 1] = (m * m) * dt;
    };
    double res[NV];
    wave_npsum<NV>(n, val, lds, res);
    if (lane_id() == 0) {
#pragma unroll
        for (int s = 0; s < NV; ++s) out[s] = res[s];
    }
}

// ============================================================================
// launch wrappers
// ============================================================================
template <int SPL, int NK>
static hipError_t launch_sweep_t(const SweepArgs& a, hipStream_t s)
{
    const unsigned blocks = (unsigned)((a.n_chunk + a.wpb - 1) / a.wpb);
    const size_t lds = (size_t)a.wpb * a.n_sinks_pad * sizeof(int);
    hipLaunchKernelGGL((rq_sweep<SPL, NK>), dim3(blocks), dim3(64 * a.wpb), lds, s, a);
    return hipGetLastError();
}

template <int SPL>
static hipError_t launch_sweep_k(const SweepArgs& a, int nK, hipStream_t s)
{
    switch (nK) {
    case 1: return launch_sweep_t<SPL, 1>(a, s);
    case 2: return launch_sweep_t<SPL, 2>(a, s);
    case 3: return launch_sweep_t<SPL, 3>(a, s);
    default: return launch_sweep_t<SPL, 4>(a, s);
    }
}

hipError_t rq_launch_gen(const GenArgs& a, hipStream_t s)
{
    if (a.n_chunk <= 0 || a.n_str <= 0) return hipSuccess;
    dim3 grid((unsigned)((a.n_chunk + 255) / 256), (unsigned)a.n_str);
    hipLaunchKernelGGL(rq_gen_streams, grid, dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t rq_launch_sweep(const SweepArgs& a, int spl, int nK, hipStream_t s)
{
    if (a.n_chunk <= 0) return hipSuccess;
    switch (spl) {
    case 1: return launch_sweep_k<1>(a, nK, s);
    case 2: return launch_sweep_k<2>(a, nK, s);
    case 4: return launch_sweep_k<4>(a, nK, s);
    default: return launch_sweep_k<8>(a, nK, s);
    }
}

template <int NK>
static hipError_t launch_scan_t(const ScanArgs& a, hipStream_t s)
{
    const unsigned blocks = (unsigned)((a.n_chunk + 3) / 4);
    const size_t lds = 4 * npsum_lds_doubles<NK + 2>() * sizeof(double);
    hipLaunchKernelGGL((rq_scan<NK>), dim3(blocks), dim3(256), lds, s, a);
    return hipGetLastError();
}

hipError_t rq_launch_scan(const ScanArgs& a, int nK, hipStream_t s)
{
    if (a.n_chunk <= 0) return hipSuccess;
    switch (nK) {
    case 1: return launch_scan_t<1>(a, s);
    case 2: return launch_scan_t<2>(a, s);
    case 3: return launch_scan_t<3>(a, s);
    default: return launch_scan_t<4>(a, s);
    }
}
