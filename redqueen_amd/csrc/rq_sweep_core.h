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
static_assert(npsum_lds_doubles<1>() == RQ_NPSUM1_LDS, "wave_npsum<1> scratch size (rq_api.cpp plans it)");

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
    // other source's event: sinks colat(e0..e1) in edge-list order (distinct).
    // Two 64-sink tiles per round so their LDS latencies overlap.
    template <class RT, class CF>
    __device__ __forceinline__ void wall(RT* rank, CF&& colat, int e0, int e1, int odf, int lane)
    {
        const int pa = e0 + lane < e1 ? colat(e0 + lane) : 0;
        const int pb = e0 + 64 + lane < e1 ? colat(e0 + 64 + lane) : 0;
        wall_pf(rank, colat, pa, pb, e0, e1, odf, lane);
    }
    // the same with the first 128 sinks' columns already loaded (pa / pb = sink of
    // edge e0 + lane / e0 + 64 + lane): the caller issues the next event's column
    // loads before this event's LDS work, so global column reads overlap it
    template <class RT, class CF>
    __device__ __forceinline__ void wall_pf(RT* rank, CF&& colat, int pa, int pb, int e0, int e1, int odf,
                                            int lane)
    {
        int dvalid = 0;
        int dle[NK];
#pragma unroll
        for (int q = 0; q < NK; ++q) dle[q] = 0;
        for (int e = e0; e < e1; e += 128) {
            const int ea = e + lane, eb = e + 64 + lane;
            const bool acta = ea < e1, actb = eb < e1;
            const int ca = e == e0 ? pa : (acta ? colat(ea) : 0);
            const int cb = e == e0 ? pb : (actb ? colat(eb) : 0);
            const int ra = acta ? (int)rank[ca] : 0;
            const int rb = actb ? (int)rank[cb] : 0;
            constexpr int kSat = sizeof(RT) == 2 ? 32767 : 0x7FFFFFFF;   // saturating (K <= 32767)
            if (acta) rank[ca] = (RT)(ra < 0 ? 1 : (ra < kSat ? ra + 1 : ra));
            if (actb) rank[cb] = (RT)(rb < 0 ? 1 : (rb < kSat ? rb + 1 : rb));
            const bool inva = acta && ra < 0, invb = actb && rb < 0;
            dvalid += popc(__ballot(inva)) + popc(__ballot(invb));
#pragma unroll
            for (int q = 0; q < NK; ++q) {
                if (1 <= km1[q]) dle[q] += popc(__ballot(inva)) + popc(__ballot(invb));
                dle[q] -= popc(__ballot(acta && ra == km1[q])) + popc(__ballot(actb && rb == km1[q]));
            }
        }
        nvalid += dvalid;
#pragma unroll
        for (int q = 0; q < NK; ++q) cnt[q] += dle[q];
        sumR += e1 - e0;
        sumF += odf;
    }
    // own post: every follower's rank -> 0 (State.apply_event, opt_model.py:71-72)
    template <class RT, class CF>
    __device__ __forceinline__ void own(RT* rank, CF&& folat, int F, int lane)
    {
        int dvalid = 0;
        int dle[NK];
#pragma unroll
        for (int q = 0; q < NK; ++q) dle[q] = 0;
        // 4 x 64 followers per round: their (distinct) sink ids are loaded together
        for (int f0 = 0; f0 < F; f0 += 256) {
            int c[4], r[4];
            bool act[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int f = f0 + 64 * u + lane;
                act[u] = f < F;
                c[u] = act[u] ? folat(f) : 0;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) r[u] = act[u] ? (int)rank[c[u]] : 0;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                dvalid += popc(__ballot(act[u] && r[u] < 0));
#pragma unroll
                for (int q = 0; q < NK; ++q) dle[q] -= popc(__ballot(act[u] && r[u] >= 0 && r[u] <= km1[q]));
                if (act[u]) rank[c[u]] = (RT)0;
            }
        }
#pragma unroll
        for (int q = 0; q < NK; ++q) cnt[q] += dle[q] + (0 <= km1[q] ? F : 0);
        nvalid += dvalid;
        sumR -= sumF;
        sumF = 0;
    }
};

// K = 1 aggregates on sink bitsets (n_sinks <= 2048): lane w holds word w of
//   T = valid sinks with rank 0 (the top-1 set) and V = sinks with a row.
// A wall event of source j with follower word m: V |= m, T &= ~m (NaN -> 1 and
// 0 -> 1 both leave / stay out of the top); a post: T |= F, V |= F.  Counts
// come from one DPP wave sum of popc(T) | popc(V) << 16; sumR/sumF as in Agg.
struct AggB {
    int64_t sumR, sumF;
    int nvalid;
    int cnt[1];
    uint32_t T, V, F;
    const uint32_t* M;   // LDS [n_str][stride], words [0, nw) used
    int nw, stride;
    __device__ __forceinline__ void init(const uint32_t* M_, int nw_, int stride_, int ctrl_idx, int lane)
    {
        sumR = 0;
        sumF = 0;
        nvalid = 0;
        cnt[0] = 0;
        T = 0u;
        V = 0u;
        M = M_;
        nw = nw_;
        stride = stride_;
        F = lane < nw ? M[ctrl_idx * stride + lane] : 0u;
    }
    __device__ __forceinline__ void wall(int j, int deg, int odf, int lane)
    {
        const uint32_t m = lane < nw ? M[j * stride + lane] : 0u;
        V |= m;
        T &= ~m;
        sumR += deg;
        sumF += odf;
    }
    // wall event with this lane's follower word already loaded
    __device__ __forceinline__ void wall_m(uint32_t m, int deg, int odf)
    {
        V |= m;
        T &= ~m;
        sumR += deg;
        sumF += odf;
    }
    __device__ __forceinline__ uint32_t packed() const
    {
        return (uint32_t)__popc(T) | ((uint32_t)__popc(V) << 16);
    }
    __device__ __forceinline__ void own()
    {
        T |= F;
        V |= F;
        sumR -= sumF;
        sumF = 0;
    }
    __device__ __forceinline__ void sync()
    {
        const uint32_t tot = wave_sum_u32((uint32_t)__popc(T) | ((uint32_t)__popc(V) << 16));
        cnt[0] = (int)(tot & 0xFFFFu);
        nvalid = (int)(tot >> 16);
    }
};

// K = 1 aggregates for any number of sinks (the general sweep's BL instances):
// per-wave LDS bitsets T (valid sinks at rank 0) and V (sinks with a row), one bit
// per sink instead of an int16 rank -- 1/8 of the LDS, so more waves per CU.
//   wall event : its sinks (distinct; lanes may share a word) clear T and set V with
//                ds_and/or_rtn, the returned old bits give the count changes;
//   post       : T |= F, V |= F word-parallel with the follower set F (shared LDS).
// Updates the Agg<NK> it is given (NK = 1: cnt[0] = #sinks at rank 0).
struct AggL {
    uint32_t* T;
    uint32_t* V;
    const uint32_t* F;
    int nw, nsink;
    __device__ __forceinline__ void init(uint32_t* T_, uint32_t* V_, const uint32_t* F_, int nw_, int lane,
                                         int nsink_ = 0x7fffffff)
    {
        T = T_;
        V = V_;
        F = F_;
        nw = nw_;
        nsink = nsink_;
        for (int k = lane; k < nw; k += 64) {
            T[k] = 0u;
            V[k] = 0u;
        }
    }
    template <int NK, class CF>
    __device__ __forceinline__ void wall_pf(Agg<NK>& g, CF&& colat, int pa, int pb, int e0, int e1, int odf,
                                            int lane)
    {
        int dvalid = 0, dtop = 0;
        const bool vfull = g.nvalid >= nsink;   // every sink seen: V is all ones, leave it
        for (int e = e0; e < e1; e += 128) {
            const int ea = e + lane, eb = e + 64 + lane;
            const bool acta = ea < e1, actb = eb < e1;
            const int ca = e == e0 ? pa : (acta ? colat(ea) : 0);
            const int cb = e == e0 ? pb : (actb ? colat(eb) : 0);
            uint32_t ta = 0u, va = 1u, tb = 0u, vb = 1u;
            if (acta) {
                const uint32_t bit = 1u << (ca & 31);
                ta = atomicAnd(&T[ca >> 5], ~bit) & bit;
                if (!vfull) va = atomicOr(&V[ca >> 5], bit) & bit;
            }
            if (actb) {
                const uint32_t bit = 1u << (cb & 31);
                tb = atomicAnd(&T[cb >> 5], ~bit) & bit;
                if (!vfull) vb = atomicOr(&V[cb >> 5], bit) & bit;
            }
            dvalid += popc(__ballot(va == 0u)) + popc(__ballot(vb == 0u));
            dtop += popc(__ballot(ta != 0u)) + popc(__ballot(tb != 0u));
        }
        g.nvalid += dvalid;
        g.cnt[0] -= dtop;
        g.sumR += e1 - e0;
        g.sumF += odf;
    }
    template <int NK>
    __device__ __forceinline__ void own(Agg<NK>& g, int lane)
    {
        uint32_t dc = 0u, dv = 0u;
        for (int k = lane; k < nw; k += 64) {
            const uint32_t f = F[k], t = T[k], v = V[k];
            dc += (uint32_t)__popc(f & ~t);
            dv += (uint32_t)__popc(f & ~v);
            T[k] = t | f;
            V[k] = v | f;
        }
        g.cnt[0] += (int)wave_sum_u32(dc);
        g.nvalid += (int)wave_sum_u32(dv);
        g.sumR -= g.sumF;
        g.sumF = 0;
    }
};

// Exact aggregates for the sequential (LOG) sweep, equal event times included.
// pivot_table(index='t', columns='sink_id', values='rank') averages the ranks
// of all rows sharing (t, sink): a sink touched m > 1 times by events at one
// time shows the mean of its m ranks in that row -- and, through ffill, in
// every later row until it is touched again.  Per sink: rank (true rank,
// drives increments), gtag/gcnt/gsum (group id, touches and rank sum of its
// last equal-time group); its pivot cell is gsum/gcnt.  Row sums are exact
// int64 while every cell is integral, else a numpy-order pass over the sinks
// (pandas' DataFrame.mean(1) sums each row pairwise).
template <int NK>
struct AggX {
    int64_t sumI;          // sum of the integral cells of valid sinks
    int nvalid, nfrac, gid;
    int cnt[NK], km1[NK];
    int* rank;
    int* gtag;
    int* gcnt;
    int* gsum;
    __device__ __forceinline__ void init(const int* Ks, int* rank_, int* x, int stride, int n_sinks,
                                         int lane)
    {
        sumI = 0;
        nvalid = 0;
        nfrac = 0;
        gid = 0;
#pragma unroll
        for (int q = 0; q < NK; ++q) {
            cnt[q] = 0;
            km1[q] = Ks[q] - 1;
        }
        rank = rank_;
        gtag = x;
        gcnt = x + stride;
        gsum = x + 2 * stride;
        for (int c = lane; c < n_sinks; c += 64) {
            gtag[c] = -1;
            gcnt[c] = 0;
            gsum[c] = 0;
        }
    }
    // one event's rows: sinks colat(e0..e1) (distinct), new rank 0 (own) or +1 (wall)
    template <class CF>
    __device__ __forceinline__ void touch(CF&& colat, int e0, int e1, bool own, int lane)
    {
        for (int e = e0; e < e1; e += 64) {
            const int ee = e + lane;
            const bool act = ee < e1;
            bool nv = false, fup = false, fdn = false;
            int dsum = 0;
            bool up[NK], dn[NK];
#pragma unroll
            for (int q = 0; q < NK; ++q) up[q] = dn[q] = false;
            if (act) {
                const int c = colat(ee);
                const int r = rank[c], tg = gtag[c], k = gcnt[c], sm = gsum[c];
                const bool ov = tg >= 0;
                const int rn = own ? 0 : (r < 0 ? 1 : r + 1);
                const int nk = tg == gid ? k + 1 : 1;
                const int ns = tg == gid ? sm + rn : rn;
                rank[c] = rn;
                gtag[c] = gid;
                gcnt[c] = nk;
                gsum[c] = ns;
                const int kk = k > 0 ? k : 1;
                const bool oint = ov && sm % kk == 0;
                const bool nint = ns % nk == 0;
                nv = !ov;
                fup = !nint && !(ov && !oint);
                fdn = nint && ov && !oint;
                dsum = (nint ? ns / nk : 0) - (oint ? sm / kk : 0);
#pragma unroll
                for (int q = 0; q < NK; ++q) {
                    const bool a1 = ns <= km1[q] * nk;
                    const bool a0 = ov && sm <= km1[q] * kk;
                    up[q] = a1 && !a0;
                    dn[q] = a0 && !a1;
                }
            }
            nvalid += popc(__ballot(nv));
            nfrac += popc(__ballot(fup)) - popc(__ballot(fdn));
#pragma unroll
            for (int q = 0; q < NK; ++q) cnt[q] += popc(__ballot(up[q])) - popc(__ballot(dn[q]));
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) dsum += __shfl_xor(dsum, o, 64);
            sumI += dsum;
        }
    }
    // the current pivot row's sum over the sinks (NaN cells count 0)
    __device__ __forceinline__ double row_sum(int n_sinks, double* lds)
    {
        if (nfrac == 0) return (double)sumI;
        double out[1];
        wave_npsum<1>((int64_t)n_sinks,
                      [&](int64_t kk, double* v) {
                          const int c = (int)kk;
                          v[0] = gtag[c] >= 0 ? (double)gsum[c] / (double)gcnt[c] : 0.0;
                      },
                      lds, out);
        return out[0];
    }
};

// Pivot rows.  LOG sweep: lane (row - s0) stages a row until 64 are staged,
// then one coalesced store per field.  The fast sweep stores whole tiles
// itself and only keeps nrow / last_t here (s0 == nrow).
template <int NK>
struct RowStage {
    double r_t, r_sum;
    int r_valid;
    int r_cnt[NK];
    int64_t nrow, s0, cap;
    double last_t;
    // the replica's rows start at row rb of the kernel's row arrays (wave-uniform bases);
    // a row's address is rebuilt at each store from rb, which an empty asm makes opaque,
    // so the compiler cannot hoist four per-lane 64-bit row pointers out of the tile
    // loop and spill them (they were reloaded from scratch every tile)
    double* Rt0;
    double* Rs0;
    uint32_t* Rv0;
    uint32_t* Rc0;
    int64_t rb;
    // merged-stream sweep (place_rows<NK, true>): this lane's rows of the last tile, kept
    // in registers and stored by flush_pend() at the top of the next tile, ahead of that
    // tile's prefetch loads.  vmcnt retires in issue order, so rows stored at the end of
    // a tile made the loop-latch wait on the prefetched tile wait on the fresh stores too.
    uint32_t p_o, p_w;   // the rows' indices in the replica (~0u: none)
    double p_ot, p_os, p_wt, p_ws;
    int p_ov, p_wv;
    int p_oc[NK], p_wc[NK];
    __device__ __forceinline__ void init(double* t, double* s, uint32_t* v, uint32_t* c, int64_t rb_,
                                         int64_t cap_)
    {
        p_o = p_w = ~0u;
        r_t = 0.0;
        r_sum = 0.0;
        r_valid = 0;
#pragma unroll
        for (int q = 0; q < NK; ++q) r_cnt[q] = 0;
        nrow = 0;
        s0 = 0;
        cap = cap_;
        last_t = -RQ_INF;
        Rt0 = t;
        Rs0 = s;
        Rv0 = v;
        Rc0 = c;
        rb = rb_;
    }
    // row rr of this replica <- (t, sum, valid, cnt)
    __device__ __forceinline__ void write(int64_t rr, double t, double sum, int valid, const int* cnt)
    {
        int64_t b = rb;
        __asm__ volatile("" : "+v"(b));
        const int64_t r = b + rr;
        Rt0[r] = t;
        Rs0[r] = sum;
        Rv0[r] = (uint32_t)valid;
#pragma unroll
        for (int q = 0; q < NK; ++q) Rc0[r * NK + q] = (uint32_t)cnt[q];
    }
    // one whole row (no tie merge: the caller closes equal-time groups itself)
    __device__ __forceinline__ bool put(double t, double sum, int valid, const int* cnt, int lane,
                                       int& status)
    {
        if (nrow >= cap) {
            status |= RQ_ST_ROWS_OVERFLOW;
            return false;
        }
        const int slot = (int)(nrow - s0);
        if (lane == slot) {
            r_t = t;
            r_sum = sum;
            r_valid = valid;
#pragma unroll
            for (int q = 0; q < NK; ++q) r_cnt[q] = cnt[q];
        }
        ++nrow;
        last_t = t;
        if (slot == 63) {
            store(s0 + lane);
            s0 = nrow;
        }
        return true;
    }
    __device__ __forceinline__ void store(int64_t rr) { write(rr, r_t, r_sum, r_valid, r_cnt); }
    __device__ __forceinline__ void flush_pend()
    {
        if (p_o != ~0u) write(p_o, p_ot, p_os, p_ov, p_oc);
        if (p_w != ~0u) write(p_w, p_wt, p_ws, p_wv, p_wc);
        p_o = p_w = ~0u;
    }
    __device__ __forceinline__ void flush(int lane)
    {
        const int rem = (int)(nrow - s0);
        if (lane < rem) store(s0 + lane);
        s0 = nrow;
    }
};

// ---- B: RedQueen controller over a tile (opt_model.py:502-544) ----
//  Lane q < n holds wall event q (time tt, stream tj).  Candidate after wall event
//  q: c_q = t_q + Exp(1)/c_{j_q} (draw ndraw + q of the controller's stream); the
//  post fires before wall event q when the running min beats t_q (ties: lower
//  src_id first, cbf); a post resets the min.  One prefix-min per post.
//  Out: ownm bit q = a post right before wall event q, at time ot (lane q).
//  OptPWSignificance (pwc != null, opt_model.py:547-623): the candidate is the first
//  point after t_q of a Poisson process whose intensity is the event's increment
//  pw_j[k] over the periodic significance segments k of T, drawn by thinning at
//  the bound max_k pw_j[k] from the phase t_q mod T (take_one_sample, :558-573);
//  event q's draws are Philox calls (event index, iteration) -- any count per lane.
__device__ __forceinline__ double optpw_sample(double tt, const double* row, double smax, int S,
                                               double T, uint64_t e, uint32_t oseed)
{
    if (!(smax > 0.0)) return RQ_INF;
    const double inv = 1.0 / smax;
    const double ph = fmod(tt, T);
    double ns = 0.0;
    for (uint32_t it = 1; it < (1u << 20); ++it) {
        uint32_t w4[4] = {(uint32_t)e, (uint32_t)(e >> 32), it, 0u};
        philox4x32_10(w4, oseed, kind_salt(RQ_SRC_OPTPW, true));
        ns = ns + rq_std_exponential(rq_uniform53(w4[0], w4[1])) * inv;
        int idx = (int)(((double)S * fmod(ns + ph, T)) / T);
        idx = idx < S ? idx : S - 1;
        if (rq_uniform53(w4[2], w4[3]) * smax < row[idx]) return tt + ns;
    }
    return RQ_INF;
}

template <bool PW>
__device__ __forceinline__ void controller_tile(int n, bool act, double tt, int tj, const double* invc,
                                                const int* cbf, uint32_t oseed, uint64_t& ndraw,
                                                double& opt_next, uint64_t& ownm, double& ot,
                                                const double* pwc = nullptr,
                                                const double* pwmax = nullptr, int S = 0,
                                                double T = 0.0)
{
    const int lane = lane_id();
    double c = RQ_INF;
    bool cb = false;
    if (PW && act && pwc) {
        c = optpw_sample(tt, pwc + (size_t)tj * S, pwmax[tj], S, T, ndraw + (uint64_t)lane, oseed);
        cb = cbf[tj] != 0;
    } else if (act) {
        const uint64_t d = ndraw + (uint64_t)lane;   // draw d: Philox call d>>1, half d&1
        const uint64_t call = d >> 1;
        uint32_t w4[4] = {(uint32_t)call, (uint32_t)(call >> 32), 0u, 0u};
        philox4x32_10(w4, oseed, kind_salt(RQ_SRC_OPT, true));
        const double x = rq_std_exponential((d & 1) ? rq_uniform53(w4[2], w4[3])
                                                    : rq_uniform53(w4[0], w4[1]));
        const double ic = invc[tj];
        const double e = ic > 0.0 ? x * ic : RQ_INF;
        c = tt + e;
        cb = cbf[tj] != 0;
    }
    ndraw += (uint64_t)n;
    int s0 = 0;
    double cur = opt_next;
    for (;;) {
        // prefix min of the candidates from lane s0 on (DPP), then shifted one lane
        const double inc = wave_scan_min_f64((lane >= s0 && act) ? c : RQ_INF);
        const double m = min_raw(cur, wave_shr1_inf_f64(inc));
        const uint64_t b = __ballot(lane >= s0 && act && (m < tt || (m == tt && cb)));
        if (b == 0) {
            if (n > 0) cur = fmin(cur, bcast_d(inc, n - 1));
            break;
        }
        const int is = __ffsll((unsigned long long)b) - 1;
        ownm |= 1ull << is;
        if (lane == is) ot = m;
        cur = RQ_INF;
        s0 = is;
    }
    opt_next = cur;
}

// ---- max_events inside a fast tile (run_dynamic's `while num_events < max_events`,
//  opt_model.py:271).  After phase B, lane q's post (ownm bit q) is event number
//  n_events + q + #posts before q, its wall event the next one.  Keeps the events
//  numbered < M: the wall events of lanes < nk (a prefix: the numbers grow with the lane)
//  with their posts; a post right before wall event nk that still fits becomes the
//  replica's final post (opt_next, played by the post-loop path), else opt_next = INF.
//  The tile shrinks to nk lanes; true = the replica ends with this tile.
__device__ __forceinline__ bool truncate_tile(int64_t M, int64_t n_events, int& n, bool& act, double& tt,
                                              int& tj, uint64_t& ownm, double ot, double& opt_next)
{
    if (M < 0) return false;
    const int lane = lane_id();
    const int64_t pp = n_events + lane + mbcnt64(ownm);
    const int64_t pw = pp + (int64_t)((ownm >> lane) & 1ull);
    const int nk = __popcll(__ballot(act && pw < M));
    if (nk >= n) return false;
    const bool lone = ((ownm >> nk) & 1ull) != 0ull && bcast_i64(pp, nk) < M;
    opt_next = lone ? bcast_d(ot, nk) : RQ_INF;
    ownm &= nk > 0 ? (~0ull >> (64 - nk)) : 0ull;
    n = nk;
    act = lane < nk;
    if (!act) {
        tt = RQ_INF;
        tj = 0;
    }
    return true;
}

// ---- pivot rows of a tile: lane q may hold a post row (before its wall event,
//  aggregates o*) and a wall row (w*).  pivot_table keeps one row per distinct t
//  (the last): a row is dropped when the next row has the same time; a first row
//  equal to the previous tile's last row overwrites it.  ma = ballot(has_o|has_w),
//  nonzero.  Returns true when the row capacity overflowed (stop the replica).
//  DEFER: the rows go to rs's pending slots (empty on entry: flush_pend() ran since the
//  last call); rows per replica stay below 2^32 (rows <= 2 x merged entries + 1, int).
template <int NK, bool DEFER = false>
__device__ __forceinline__ bool place_rows(RowStage<NK>& rs, uint64_t ma, bool has_o, bool has_w, double ot,
                                           double tt, int64_t osum, int oval, const int* ocnt,
                                           int64_t wsum, int wval, const int* wcnt, int& status)
{
    const int lane = lane_id();
    const uint64_t mo = __ballot(has_o), mw = __ballot(has_w);
    // the next row-holding lane above this one (per-lane shifts, no hoisted lane masks)
    const uint64_t above = lane < 63 ? ma >> (lane + 1) : 0ull;
    const bool nxt = above != 0;
    const double ft = has_o ? ot : tt;
    const double nft = __shfl(ft, nxt ? lane + __ffsll((unsigned long long)above) : lane, 64);
    const bool keep_o = has_o && !(has_w ? ot == tt : (nxt && ot == nft));
    const bool keep_w = has_w && !(nxt && tt == nft);
    const bool tie0 = rs.nrow > 0 && bcast_d(ft, __ffsll((unsigned long long)ma) - 1) == rs.last_t;
    const uint64_t ko = __ballot(keep_o), kw = __ballot(keep_w);
    if (tie0 || ko != mo || kw != mw) status |= RQ_ST_TIE;
    const int64_t r0 = rs.nrow - (tie0 ? 1 : 0);
    const int64_t po = r0 + mbcnt64(ko) + mbcnt64(kw);
    const int64_t pw = po + (keep_o ? 1 : 0);
    if constexpr (DEFER) {
        rs.p_o = keep_o && po < rs.cap ? (uint32_t)po : ~0u;
        rs.p_w = keep_w && pw < rs.cap ? (uint32_t)pw : ~0u;
        rs.p_ot = ot;
        rs.p_os = (double)osum;
        rs.p_ov = oval;
        rs.p_wt = tt;
        rs.p_ws = (double)wsum;
        rs.p_wv = wval;
#pragma unroll
        for (int q = 0; q < NK; ++q) {
            rs.p_oc[q] = ocnt[q];
            rs.p_wc[q] = wcnt[q];
        }
    } else {
        if (keep_o && po < rs.cap) rs.write(po, ot, (double)osum, oval, ocnt);
        if (keep_w && pw < rs.cap) rs.write(pw, tt, (double)wsum, wval, wcnt);
    }
    rs.last_t = bcast_d(has_w ? tt : ot, 63 - __builtin_clzll(ma));   // always kept
    rs.nrow = r0 + __popcll(ko) + __popcll(kw);
    rs.s0 = rs.nrow;
    if (rs.nrow > rs.cap) {
        rs.nrow = rs.cap;
        rs.s0 = rs.cap;
        status |= RQ_ST_ROWS_OVERFLOW;
        return true;
    }
    return false;
}

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

}  // namespace rq
