// rq_kernels.hip -- the gfx950 engine: stream generation, RedQueen sweep,
// metric scan (the dataframe replay is rq_replay.hip).  Launch wrappers at the bottom are called by the
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
#include "rq_sweep_core.h"
#include "rq_gen.h"
#include <type_traits>
#include <algorithm>
#include <cstdlib>

#pragma clang fp contract(off)

using namespace rq;

// ============================================================================
// 1. arrival streams
// ============================================================================
__global__ __launch_bounds__(256) void rq_gen_streams(GenArgs a)
{
    // rq_exp's table in LDS: a Hawkes candidate's exp looks up two per-lane words in its
    // dependent chain (from __constant__ memory these were vector loads at L1/L2 latency)
    __shared__ uint64_t etab[RQ_EXP_TAB_N];
    for (int e = threadIdx.x; e < RQ_EXP_TAB_N; e += blockDim.x) etab[e] = rq_exp_tab_c[e];
    __syncthreads();
    const int64_t rl = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int j = (int)(blockIdx.z * gridDim.y + blockIdx.y);   // > 32768 streams fold into z
    if (rl >= a.n_chunk || j >= a.n_str) return;
    const int64_t o = a.chunk0 + rl;      // local output index
    const int64_t i = rq_replica_of(a, o);   // global id (seeds)
    SrcGen gen;
    gen.init(a, j, i, etab);

    double* out = a.streams + rl * a.capsum + a.st_off[j];   // 128-byte aligned (host pads)
    const int cap = a.cap[j];                                   // multiple of 16
    int n = 0;
    bool ovf = false;
    // arrivals are staged RQ_GEN_W at a time in registers (compile-time shift, no
    // scratch) and written as one lane-contiguous chunk: 16 = a whole 128-byte line per
    // lane, so no line is written in halves at different times (C3: written bytes 1.22 ->
    // 1.04 x the 8 B per arrival; 8: gen 5 % faster at 90 instead of 106 VGPRs)
#ifndef RQ_GEN_W
#define RQ_GEN_W 16
#endif
    constexpr int GW = RQ_GEN_W;
    static_assert(GW == 8 || GW == 16, "staging width");
    double sb[GW];
#pragma unroll
    for (int k = 0; k < GW; ++k) sb[k] = 0.0;
    while (!gen.done && !ovf) {
        double tv;
        if (gen.step(&tv, a.end)) {
            if (n < cap) {
#pragma unroll
                for (int k = 0; k + 1 < GW; ++k) sb[k] = sb[k + 1];
                sb[GW - 1] = tv;
                ++n;
                if ((n & (GW - 1)) == 0) {
                    double4* d = reinterpret_cast<double4*>(out + n - GW);
#pragma unroll
                    for (int k = 0; k < GW / 4; ++k) d[k] = make_double4(sb[4 * k], sb[4 * k + 1], sb[4 * k + 2], sb[4 * k + 3]);
                }
            } else {
                ovf = true;
            }
        }
    }
    {   // the last partial chunk: values sit in sb[GW-r .. GW-1]; written as one whole
        // chunk (slots past n hold stale values nobody reads: readers stop at slen)
        const int r = n & (GW - 1);
        if (r > 0) {
            // shift the staged values left by GW - r (log-steps of static shifts: no scratch)
            const int sh = GW - r;
#pragma unroll
            for (int st = 1; st < GW; st <<= 1) {
                const bool on = (sh & st) != 0;
#pragma unroll
                for (int k = 0; k < GW; ++k) sb[k] = on ? sb[k + st < GW ? k + st : GW - 1] : sb[k];
            }
            // whole 64-byte halves, only those holding arrivals
            double4* d = reinterpret_cast<double4*>(out + (n - r));
#pragma unroll
            for (int k = 0; k < GW / 4; ++k)
                if (k < 2 || r > 8) d[k] = make_double4(sb[4 * k], sb[4 * k + 1], sb[4 * k + 2], sb[4 * k + 3]);
        }
    }
    a.slen[(int64_t)j * a.slen_stride + rl] = n;   // consecutive lanes, consecutive ints
    if (ovf) atomicOr(&a.status[o], RQ_ST_STREAM_OVERFLOW);
}

// ============================================================================
// 2. sweep: one wavefront per replica, 64-arrival tiles in three phases.
//    A  merge: lanes own sources; each step is a DPP wave-min over order-
//       preserving time keys (high word, low word only on a tie).  Every
//       source keeps a ring of its next W arrivals in LDS, refilled for all
//       sources at once when one runs dry.  Arrival #k of the tile -> lane k.
//    B  controller: the world is exogenous, so the RedQueen candidates of the
//       whole tile are drawn in parallel and the posts found by prefix-mins.
//    C  apply: the only sequential part -- the per-sink rank updates in LDS;
//       each event's aggregates are parked in its lane and the pivot rows
//       (equal-time rows merged) are placed and stored by all lanes at once.
//    LOG = the event log / max_events variant: phase C goes event by event.
//    GS  = LOG with the per-sink state (rank, pivot-cell group) in global memory, one
//          slot per resident wave (SweepArgs.gs): any number of sinks.
// ============================================================================
//    MRG = the fast sweep on merged streams (rq_merge_streams): a tile is the next 64
//          entries of the replica's (t, stream) sequence, loaded one tile ahead.
//    GT  = (merged streams only) the per-stream tables -- CSR row starts, follower
//          out-degrees, controller tie flags, 1/c_j -- read from global memory instead of
//          LDS: graphs of more streams than those tables fit in LDS (up to 65535).
template <int SPL, int NK, class COL, int W, bool LOG, bool BITS, bool BL, bool GS = false, bool MRG = false,
          bool GT = false>
__global__ __launch_bounds__(LOG ? 256 : (MRG ? RQ_MRG_LB : (SPL >= 4 ? 512 : 1024))) void rq_sweep(SweepArgs a)
{
    extern __shared__ double lds_g[];
    char* base = reinterpret_cast<char*>(lds_g);
    const int lane = lane_id();
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));   // wave-uniform: SGPR addressing
    int* cptr = reinterpret_cast<int*>(base + a.lds_ptr);
    int* odf = reinterpret_cast<int*>(base + a.lds_odf);
    int* cbf = reinterpret_cast<int*>(base + a.lds_cbf);
    // sink columns: COL = uint16_t -> LDS copy, COL = int -> global (compile-time,
    // so LDS reads never wait on outstanding global traffic)
    constexpr bool col_lds = sizeof(COL) == 2;
    COL* col_l = reinterpret_cast<COL*>(base + a.lds_col);
    const int* col_g = a.csr_col;
    if (col_lds && !BITS)
        for (int e = threadIdx.x; e < a.n_csr; e += blockDim.x) col_l[e] = (COL)a.csr_col[e];
    // BITS: per-stream sink bitsets instead of the columns
    uint32_t* msk = reinterpret_cast<uint32_t*>(base + a.lds_mask);
    if (BITS)
        for (int e = threadIdx.x; e < a.n_str * a.mstride; e += blockDim.x) {
            const int jj = e / a.mstride, ww = e - jj * a.mstride;
            msk[e] = ww < a.nw ? a.masks[jj * a.nw + ww] : 0u;
        }
    for (int j = threadIdx.x; j <= a.n_str && !GT; j += blockDim.x) cptr[j] = a.csr_ptr[j];
    for (int j = threadIdx.x; j < a.n_str && !GT; j += blockDim.x) {
        odf[j] = a.outdeg_f[j];
        // the controller (a dynamic source) posts before a wall event at the same time
        // when that source is static (run_dynamic plays a static time only if it is
        // strictly earlier, opt_model.py:289-290) or has a larger src_id (the sorted
        // (t_delta, src_id) of the dynamic sources, :279-281)
        cbf[j] = a.cbf_g[j];   // the graph's table (static sources, RQ_SRCF_DYNAMIC)
    }
    // BL: the follower set as a sink bitset, shared by the block's waves
    uint32_t* fbl = reinterpret_cast<uint32_t*>(base + a.lds_fbits);
    if (BL)
        for (int k = threadIdx.x; k < a.nwl; k += blockDim.x) fbl[k] = a.fbits[k];
    // one grid point: the controller's 1/c_j table is the same for every replica, so the
    // block holds one copy (its LDS goes to the sink columns instead of 8 per-wave copies)
    double* invc_sh = reinterpret_cast<double*>(base + a.lds_invc);
    if (a.invc_shared && !GT)
        for (int j = threadIdx.x; j < a.n_str; j += blockDim.x) invc_sh[j] = a.inv_c[j];
    // the tables the sweep reads: LDS, or (GT) global
    const int* cptr_r = GT ? a.csr_ptr : cptr;
    const int* odf_r = GT ? a.outdeg_f : odf;
    const int* cbf_r = GT ? a.cbf_g : cbf;
    __syncthreads();   // block-shared tables ready; no block barrier below this line
    char* wb = base + a.lds_wave + (size_t)w * a.lds_wave_stride;
    double* invc = a.invc_shared ? invc_sh : reinterpret_cast<double*>(wb);
    // ranks: exact int for the LOG variant (pivot cells average them); the fast
    // sweep only compares them with K-1, so int16 saturating at 32767 is exact
    using RT = typename std::conditional<LOG, int, int16_t>::type;
    // GS: this wave's slot of the global per-sink state (the grid never exceeds the slots)
    char* gsb = GS ? a.gs + (size_t)(blockIdx.x * a.wpb + w) * (size_t)a.gs_stride : nullptr;
    RT* rank = GS ? reinterpret_cast<RT*>(gsb) : reinterpret_cast<RT*>(wb + a.lds_rank_off);
    double* win = reinterpret_cast<double*>(wb + a.lds_win_off);
    // first replica: the wave's static slot; with a work queue (a.wq) the wave then
    // takes replicas nslot, nslot + 1, ... until the chunk is exhausted
    const int64_t nslot = (int64_t)gridDim.x * a.wpb;
    for (int64_t qi = (int64_t)blockIdx.x * a.wpb + w; qi < a.n_chunk;) {
    const int64_t rl = a.order ? (int64_t)a.order[qi] : qi;   // longest first (rq_order_replicas)
    const int64_t o = a.chunk0 + rl;
    const int64_t i = rq_replica_of(a.gen, o);
    const int g = (int)(i / a.n_rep);
    AggL agl;
    if (BL) {
        uint32_t* tb = reinterpret_cast<uint32_t*>(wb + a.lds_rank_off);
        agl.init(tb, tb + a.nwl, fbl, a.nwl, lane, a.n_sinks);
    }
    if (!a.invc_shared && !GT)
        for (int j = lane; j < a.n_str; j += 64) invc[j] = a.inv_c[(int64_t)g * a.n_str + j];
    const double* invc_r = GT ? a.inv_c + (int64_t)g * a.n_str : invc;
    if (!BITS && !BL)
        for (int c = lane; c < a.n_sinks; c += 64) rank[c] = -1;   // NaN: no row yet
    // BL + MRG: stream stamps (the reset epoch the stream last played in) and the
    // first-lane table of a tile segment
    int* sk_stamp = (BL && MRG && a.lds_skip) ? reinterpret_cast<int*>(wb + a.lds_skip) : nullptr;
    int* sk_first = sk_stamp ? sk_stamp + a.n_str : nullptr;
    int sk_ep = 0;   // resets (posts / own-stream arrivals) so far
    if (BL && MRG && sk_stamp)
        for (int j = lane; j < a.n_str; j += 64) {
            sk_stamp[j] = -1;
            sk_first[j] = 64;
        }
    wave_lds_sync();
    if (GS) wave_mem_sync();

    // ---- arrivals: lane owns sources [lane*SPL, lane*SPL+SPL) ----
    const double* st = a.streams + rl * a.capsum;
    double head[SPL];
    int pos[SPL], fil[SPL], len[SPL], off[SPL];
    // fast sweep: a register window of each source's next W arrivals (INF past its
    // end), reloaded from the stream buffer only for the sources a tile advanced
    constexpr int HW = LOG ? 1 : W;
    double wv[SPL][HW];
    auto load_win = [&](int q) __attribute__((always_inline)) {
#pragma unroll
        for (int h = 0; h < HW; ++h) wv[q][h] = pos[q] + h < len[q] ? st[off[q] + pos[q] + h] : RQ_INF;
    };
#pragma unroll
    for (int q = 0; q < SPL; ++q) {
        const int j = lane * SPL + q;
        off[q] = j < a.n_str && !MRG ? (int)a.st_off[j] : 0;
        len[q] = j < a.n_str && !MRG ? a.slen[(int64_t)j * a.slen_stride + rl] : 0;
        pos[q] = 0;
        fil[q] = 0;
    }
    // refill every ring that is at most half full (and not exhausted)
    auto refill = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int q = 0; q < SPL; ++q) {
            const int j = lane * SPL + q;
            const bool need = fil[q] < len[q] && fil[q] - pos[q] <= W / 2;
            const int nf = need ? ((pos[q] + W) < len[q] ? pos[q] + W : len[q]) : fil[q];
            // two half-ring chunks: all loads of a chunk in flight before its LDS stores
#pragma unroll
            for (int h = 0; h < W; h += W / 2) {
                double v[W / 2];
#pragma unroll
                for (int k = 0; k < W / 2; ++k)
                    v[k] = fil[q] + h + k < nf ? st[off[q] + fil[q] + h + k] : 0.0;
#pragma unroll
                for (int k = 0; k < W / 2; ++k)
                    if (fil[q] + h + k < nf) win[j * W + ((fil[q] + h + k) & (W - 1))] = v[k];
            }
            fil[q] = nf;
        }
    };
    double lmin = RQ_INF;
    int larg = 0;
    if constexpr (LOG) {
        refill();
#pragma unroll
        for (int q = 0; q < SPL; ++q) {
            head[q] = len[q] > 0 ? win[(lane * SPL + q) * W] : RQ_INF;
            if (head[q] < lmin) {
                lmin = head[q];
                larg = q;
            }
        }
    } else if constexpr (!MRG) {
#pragma unroll
        for (int q = 0; q < SPL; ++q) load_win(q);
    }
    // MRG: the replica's merged sequence; lane l holds entry mpos + l of the next tile
    // (entry index of the replica's first entry; opaque at each tile's loads, so no
    // per-lane 64-bit sequence pointers are hoisted out of the tile loop and spilled)
    const int64_t mb = MRG ? rl * a.mrg_stride : 0;
    auto mload = [&](int64_t e, double& t_, int& j_) __attribute__((always_inline)) {
        int64_t x = mb;
        __asm__ volatile("" : "+v"(x));
        t_ = a.mrg_t[x + e];
        j_ = a.mrg_j[x + e];
        if (GT && a.mrg_jh) j_ |= (int)a.mrg_jh[x + e] << 16;   // > 65535 streams: always the GT instances
    };
    const int mlen = MRG ? a.mrg_len[rl] : 0;
    int mpos = 0;
    double nxt_t = RQ_INF;
    int nxt_j = 0;
    if (MRG && lane < mlen) mload(lane, nxt_t, nxt_j);
    double span = -1.0;   // fast sweep: adaptive tile width in time (< 0: not estimated yet)
    double* st_t = reinterpret_cast<double*>(win);   // fast sweep: tile staging (64 t + 64 j)
    int* st_j = reinterpret_cast<int*>(st_t + 64);

    const bool opt = a.ctrl_kind == RQ_SRC_OPT || a.ctrl_kind == RQ_SRC_OPTPW;
    const double* pwc = a.pw_c ? a.pw_c + (size_t)g * a.n_str * a.n_seg : nullptr;
    const double* pwm = a.pw_c ? a.pw_max + (size_t)g * a.n_str : nullptr;
    double opt_next = opt ? a.start : RQ_INF;
    const int64_t k = a.seed_mod > 0 ? i % a.seed_mod : i;
    const uint32_t oseed = a.ctrl_seed ? a.ctrl_seed[i] : a.ctrl_seed0 + (uint32_t)k;
    uint64_t ndraw = 0;   // wall events seen so far = the controller's draw index
    auto colat = [&](int e) -> int { return col_lds ? (int)col_l[e] : col_g[e]; };
    const int fol0 = cptr_r[a.ctrl_idx];
    auto folat = [&](int f) -> int { return colat(fol0 + f); };

    Agg<NK> ag;
    ag.init(a.Ks);
    AggB agb;
    if (BITS) agb.init(msk, a.nw, a.mstride, a.ctrl_idx, lane);
    RowStage<NK> rs;
    const int64_t rbase = rl * a.cap_rows;
    rs.init(a.rows_t, a.rows_sum, a.rows_valid, a.rows_cnt, rbase, a.cap_rows);
    EvStage es;
    if (LOG && a.ev_t) es.init(a.ev_t + o * a.ev_cap, a.ev_src + o * a.ev_cap, a.ev_cap);

    int64_t n_events = 0, posts = 0, world = 0;
    int status = 0;
    // LOG: exact per-sink pivot cells; rows are closed per distinct event time
    AggX<NK> ax;
    double* xlds = nullptr;
    bool pend = false;      // an equal-time group is open
    double pend_t = 0.0;
    if (LOG) {
        int* xs = GS ? reinterpret_cast<int*>(gsb + 4 * (size_t)a.n_sinks_pad)
                     : reinterpret_cast<int*>(wb + a.lds_x_off);
        xlds = reinterpret_cast<double*>(wb + a.lds_x_off + (GS ? 0 : 12 * (size_t)a.n_sinks_pad));
        ax.init(a.Ks, reinterpret_cast<int*>(rank), xs, a.n_sinks_pad, a.n_sinks, lane);
        if (GS) wave_mem_sync();
    }
    // one event's rows: every layer of stream j's CSR row (a layer's sinks are distinct;
    // duplicate edges put a sink's k-th occurrence in layer k-1, opt_model.py:306-307);
    // the controlled row's first layer is the follower list (folat)
    auto touch_row = [&](int j, bool own, int e0, int e1) __attribute__((always_inline)) {
        int l0 = 0, l1 = 0;
        if (a.lay_ptr) {
            l0 = a.lay_ptr[j];
            l1 = a.lay_ptr[j + 1];
            e1 = a.lay_end[l0];
        }
        if (own) ax.touch(folat, 0, a.n_fol, true, lane);
        else ax.touch(colat, e0, e1, false, lane);
        if (GS) wave_mem_sync();
        for (int l = l0 + 1; l < l1; ++l) {
            const int e2 = a.lay_end[l];
            ax.touch(colat, e1, e2, own, lane);
            if (GS) wave_mem_sync();
            e1 = e2;
        }
    };
    auto close_row = [&]() __attribute__((always_inline)) -> bool {
        pend = false;
        return rs.put(pend_t, ax.row_sum(a.n_sinks, xlds), ax.nvalid, ax.cnt, lane, status);
    };
    // LOG: one event of the log (State.apply_event); false = stop the replica
    auto event = [&](double tev, bool own, int jw, int e0, int e1) __attribute__((always_inline)) -> bool {
        if (a.max_events >= 0 && n_events >= a.max_events) return false;
        if (a.ev_t) es.push(tev, own ? a.ctrl_idx : jw, lane, status);
        ++n_events;
        const int nsinks = own ? a.n_fol : e1 - e0;
        if (nsinks > 0) {
            if (pend && tev == pend_t) {
                status |= RQ_ST_TIE;
            } else {
                if (pend && !close_row()) return false;
                ++ax.gid;
                pend = true;
                pend_t = tev;
            }
            if (own) {
                touch_row(a.ctrl_idx, true, 0, 0);
                ++posts;
            } else {
                touch_row(jw, false, e0, e1);
                ++world;
            }
        }
        return true;
    };

    bool stop = false;
    for (;;) {
        // ---- A: the next <= 64 arrivals (t <= end) in (t, source) order; lane n holds #n ----
        double tt = RQ_INF;
        int tj = 0, n = 0;
        bool fin_w = false;
        if constexpr (MRG) {
            if (mpos >= mlen) break;   // every arrival played
            n = mlen - mpos < 64 ? mlen - mpos : 64;
            tt = lane < n ? nxt_t : RQ_INF;
            tj = lane < n ? nxt_j : 0;
            mpos += n;
            fin_w = mpos >= mlen;
            // the next tile's loads stay in flight through phases B and C
            nxt_t = RQ_INF;
            nxt_j = 0;
            if (mpos + lane < mlen) mload(mpos + lane, nxt_t, nxt_j);
        } else if constexpr (!LOG) {
            // windowed: every arrival before a cut tau, tau < the W-th pending arrival of
            // every source that has more (so the tile is complete) and tuned so the tile
            // holds <= 64; staged in source order, rank-sorted into (t, source) order --
            // the reference's (time, src_id) order (opt_model.py:279-281)
            double lb = RQ_INF;
            lmin = RQ_INF;
#pragma unroll
            for (int q = 0; q < SPL; ++q) {
                lmin = wv[q][0] < lmin ? wv[q][0] : lmin;
                if (pos[q] + W < len[q] && wv[q][W - 1] < lb) lb = wv[q][W - 1];
            }
            const double tfirst = wave_min_f64(lmin);
            if (!(tfirst <= a.end)) break;   // every source consumed
            const double tmax = wave_min_f64(lb);
            int cq[SPL];
            int c = 0;
            bool trunc = !(tmax > tfirst);
            if (!trunc) {
                double cut = tmax;
                if (span > 0.0 && tfirst + span < cut) cut = tfirst + span;
                if (!(cut > tfirst)) cut = next_up(tfirst);
                for (;;) {
                    c = 0;
#pragma unroll
                    for (int q = 0; q < SPL; ++q) {
                        cq[q] = 0;
#pragma unroll
                        for (int h = 0; h < W; ++h) cq[q] += wv[q][h] < cut ? 1 : 0;
                        c += cq[q];
                    }
                    n = (int)wave_sum_u32((uint32_t)c);
                    if (n <= 64) break;
                    const double nc = tfirst + (cut - tfirst) * 0.5;
                    const double lo = next_up(tfirst);
                    if (nc > tfirst && nc < cut) {
                        cut = nc < lo ? lo : nc;
                    } else if (cut != lo) {
                        cut = lo;
                    } else {
                        trunc = true;   // > 64 arrivals share tfirst
                        break;
                    }
                }
                if (!trunc) span = (cut - tfirst) * (a.tile_target / (double)(n > 8 ? n : 8));
            }
            int off_l;
            if (trunc) {
                // the arrivals equal to tfirst, in source order, up to the first source
                // whose window may continue at tfirst, at most 64
                int qb = SPL;   // this lane's first such source
#pragma unroll
                for (int q = SPL - 1; q >= 0; --q)
                    if (pos[q] + W < len[q] && wv[q][W - 1] == tfirst) qb = q;
                const uint64_t bl = __ballot(qb < SPL);
                const int lbn = bl ? __ffsll((unsigned long long)bl) - 1 : 64;
                c = 0;
#pragma unroll
                for (int q = 0; q < SPL; ++q) {
                    cq[q] = 0;
#pragma unroll
                    for (int h = 0; h < W; ++h) cq[q] += wv[q][h] == tfirst ? 1 : 0;
                    if (lane > lbn || (lane == lbn && q > qb)) cq[q] = 0;
                    c += cq[q];
                }
                off_l = (int)wave_scan_add((uint32_t)c) - c;
                int room = 64 - off_l;
                c = 0;
#pragma unroll
                for (int q = 0; q < SPL; ++q) {
                    room = room > 0 ? room : 0;
                    cq[q] = cq[q] < room ? cq[q] : room;
                    room -= cq[q];
                    c += cq[q];
                }
                n = (int)wave_sum_u32((uint32_t)c);
            } else {
                off_l = (int)wave_scan_add((uint32_t)c) - c;
            }
            // stage in source order; rank = #staged arrivals before this one in (t, source)
            // order, the staged times read back two at a time (broadcast ds_read_b128)
            {
                int k = off_l;
#pragma unroll
                for (int q = 0; q < SPL; ++q)
#pragma unroll
                    for (int h = 0; h < W; ++h)
                        if (h < cq[q]) {
                            st_t[k] = wv[q][h];
                            st_j[k] = lane * SPL + q;
                            ++k;
                        }
                if (lane >= n) st_t[lane] = RQ_INF;   // the rank loop reads whole blocks of 8
            }
            wave_lds_sync();
            const bool actw = lane < n;
            const double ti = actw ? st_t[lane] : RQ_INF;
            const int ji = actw ? st_j[lane] : 0;
            const int rnk = stage_rank(st_t, n, ti, lane);
            wave_lds_sync();
            if (actw) {
                st_t[rnk] = ti;
                st_j[rnk] = ji;
            }
            wave_lds_sync();
            tt = actw ? st_t[lane] : RQ_INF;
            tj = actw ? st_j[lane] : 0;
            wave_lds_sync();   // the staging area is rewritten by the next tile
            // consume: a source the tile advanced by c shifts its window by c in
            // registers and loads only the c arrivals that enter it (each arrival is
            // read from the stream buffer once)
            bool left = false;
#pragma unroll
            for (int q = 0; q < SPL; ++q) {
                const int c = cq[q];
                if (c > 0) {
                    pos[q] += c;
                    double nw[HW];
#pragma unroll
                    for (int h = 0; h < HW; ++h) {
                        double x = RQ_INF;
#pragma unroll
                        for (int s = h + 1; s < HW; ++s)
                            if (c == s - h) x = wv[q][s];
                        nw[h] = x;
                    }
#pragma unroll
                    for (int h = 0; h < HW; ++h)
                        if (h + c >= HW && pos[q] + h < len[q]) nw[h] = st[off[q] + pos[q] + h];
#pragma unroll
                    for (int h = 0; h < HW; ++h) wv[q][h] = nw[h];
                }
                left = left || pos[q] < len[q];
            }
            fin_w = !__ballot(left);
        }
        while (LOG && n < 64) {
            const uint64_t key = order_key(lmin);
            const uint32_t khi = (uint32_t)(key >> 32), klo = (uint32_t)key;
            const uint32_t mhi = wave_min_u32(khi);
            uint64_t cand = __ballot(khi == mhi);
            if (__popcll(cand) > 1) {
                const uint32_t mlo = wave_min_u32(khi == mhi ? klo : 0xFFFFFFFFu);
                cand = __ballot(khi == mhi && klo == mlo);
            }
            const int wl = __ffsll((unsigned long long)cand) - 1;
            const double tw = bcast_d(lmin, wl);
            if (!(tw <= a.end)) break;
            const int wq = SPL == 1 ? 0 : bcast_i(larg, wl);
            if (lane == n) {
                tt = tw;
                tj = wl * SPL + wq;
            }
            ++n;
            // advance the winning source; refill the rings if it ran dry
            bool dry = false;
#pragma unroll
            for (int q = 0; q < SPL; ++q)
                if (lane == wl && q == wq) {
                    ++pos[q];
                    dry = pos[q] < len[q] && pos[q] == fil[q];
                }
            if (__ballot(dry)) refill();
            if (lane == wl) {
                lmin = RQ_INF;
                larg = 0;
#pragma unroll
                for (int q = 0; q < SPL; ++q) {
                    if (q == wq)
                        head[q] = pos[q] < len[q] ? win[(lane * SPL + q) * W + (pos[q] & (W - 1))]
                                                  : RQ_INF;
                    if (head[q] < lmin) {
                        lmin = head[q];
                        larg = q;
                    }
                }
            }
        }
        const bool fin = LOG && !MRG ? n < 64 : fin_w;
        bool act = lane < n;
        int e0 = 0, e1 = 0, od = 0;
        if (act) {
            e0 = cptr_r[tj];
            e1 = cptr_r[tj + 1];
            od = odf_r[tj];
        }
        // ---- B: RedQueen controller over the tile (opt_model.py:536-556) ----
        //  candidate after wall event i: c_i = t_i + Exp(1)/c_{j_i}; the post fires
        //  before wall event i when the running min beats t_i (ties: lower src_id
        //  first); a post resets the min.  One prefix-min per post.
        uint64_t ownm = 0;
        double ot = RQ_INF;
        if (opt && a.dbg != 3)
            controller_tile<true>(n, act, tt, tj, invc_r, cbf_r, oseed, ndraw, opt_next, ownm, ot, pwc, pwm, a.n_seg,
                            a.period);
        // max_events on the fast sweeps: the tile keeps the events numbered below it and
        // the replica ends with it (the LOG sweep's event() counts them one by one)
        bool cut = false;
        if (!LOG && a.max_events >= 0)
            cut = truncate_tile(a.max_events, n_events, n, act, tt, tj, ownm, ot, opt_next);
        ownm = sgpr_u64(ownm);   // wave-uniform: phase C's bookkeeping stays scalar
        // ---- C: apply the tile's events in order ----
        if (LOG) {
            for (int q = 0; q < n; ++q) {
                if ((ownm >> q) & 1ull) {
                    if (!event(bcast_d(ot, q), true, 0, 0, 0)) {
                        stop = true;
                        break;
                    }
                }
                const int jw = bcast_i(tj, q);
                if (!event(bcast_d(tt, q), !opt && jw == a.ctrl_idx, jw, bcast_i(e0, q),
                           bcast_i(e1, q))) {
                    stop = true;
                    break;
                }
            }
        } else if (a.dbg == 1) {
            n_events += n;
        } else {
            const bool own_b = act && ((ownm >> lane) & 1ull);     // controller post before #lane
            if (a.ev_t) {
                // event log (t, stream): lane q's post (if any) then its arrival, in tile order
                const int64_t pp = n_events + lane + mbcnt64(ownm);
                const int64_t pw = pp + (own_b ? 1 : 0);
                double* Et = a.ev_t + o * a.ev_cap;
                int32_t* Es = a.ev_src + o * a.ev_cap;
                if (own_b && pp < a.ev_cap) {
                    Et[pp] = ot;
                    Es[pp] = a.ctrl_idx;
                }
                if (act && pw < a.ev_cap) {
                    Et[pw] = tt;
                    Es[pw] = tj;
                }
                if (n_events + n + __popcll(ownm) > a.ev_cap) status |= RQ_ST_ROWS_OVERFLOW;
            }
            const bool strm_own = act && !opt && tj == a.ctrl_idx;  // controlled stream's arrival
            const bool has_o = own_b && a.n_fol > 0;
            const bool has_w = act && e1 > e0;
            // the walk only updates the per-sink ranks; lane q keeps the aggregates
            // after its controller post (o*) and after its own event (w*)
            int64_t osum = 0, wsum = 0;
            int oval = 0, wval = 0;
            int ocnt[NK], wcnt[NK];
#pragma unroll
            for (int kq = 0; kq < NK; ++kq) ocnt[kq] = wcnt[kq] = 0;
            if (BITS) {
                // batches of 8 events: follower words loaded up front, the 8 wave
                // sums interleaved; aggregates land in lane q via v_writelane
                const int deg = e1 - e0;
                int wsl = 0, wsh = 0, osl = 0, osh = 0, oc0 = 0, wc0 = 0;
                for (int q0 = 0; q0 < n; q0 += 8) {
                    uint32_t m[8], pk[8];
                    int jk[8];
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        jk[k] = bcast_i(tj, q0 + k < n ? q0 + k : n - 1);
                        m[k] = lane < agb.nw ? agb.M[jk[k] * agb.stride + lane] : 0u;
                    }
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        const int q = q0 + k;
                        pk[k] = 0u;
                        if (q < n) {
                            if ((ownm >> q) & 1ull) {
                                agb.own();
                                agb.sync();
                                osl = wlane(osl, (int)(uint32_t)agb.sumR, q);
                                osh = wlane(osh, (int)(agb.sumR >> 32), q);
                                oval = wlane(oval, agb.nvalid, q);
                                oc0 = wlane(oc0, agb.cnt[0], q);
                            }
                            if (!opt && jk[k] == a.ctrl_idx)
                                agb.own();
                            else
                                agb.wall_m(m[k], bcast_i(deg, q), bcast_i(od, q));
                            pk[k] = agb.packed();
                            wsl = wlane(wsl, (int)(uint32_t)agb.sumR, q);
                            wsh = wlane(wsh, (int)(agb.sumR >> 32), q);
                        }
                    }
                    wave_sum_u32_n<8>(pk);
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        if (q0 + k < n) {
                            const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)pk[k], 63);
                            wval = wlane(wval, (int)(tot >> 16), q0 + k);
                            wc0 = wlane(wc0, (int)(tot & 0xFFFFu), q0 + k);
                        }
                    }
                }
                wsum = (int64_t)(((uint64_t)(uint32_t)wsh << 32) | (uint32_t)wsl);
                osum = (int64_t)(((uint64_t)(uint32_t)osh << 32) | (uint32_t)osl);
                wcnt[0] = wc0;
                ocnt[0] = oc0;
            } else {
              if constexpr (BL) {
                // batches of up to 8 wall events (no post inside, <= 128 sinks each): the
                // batch's columns are loaded together, then every LDS atomic of the batch
                // is issued back to back -- a wave's LDS operations complete in order, so
                // each returns the T / V bits as of its own event's turn -- and counted
                // after; one latency chain per batch instead of one per event
                int wsl = 0, wsh = 0, osl = 0, osh = 0;
                // MRG (delta mode): per event only its kills / new valid sinks go to its lane;
                // own posts and own-stream arrivals leave the absolute counts after them
                // (anchors); sumR / sumF come from segmented scans after the tile
                constexpr bool DM = MRG;
                int dcnt = 0, dval = 0, acnt = 0, aval = 0;
                const int cnt0 = ag.cnt[0], val0 = ag.nvalid;
                const int64_t S0 = ag.sumR, F0 = ag.sumF;
                // per tile: events that cannot join a batch -- an own-stream arrival, no
                // sinks or more than 128 -- and the batch breaks (those, an own post
                // before the event, the end of the tile)
                const int degl = e1 - e0;
                const uint64_t specm =
                    __ballot(act && ((!opt && tj == a.ctrl_idx) || degl == 0 || degl > 128 || a.dbg == 2));
                const uint64_t brk = sgpr_u64(specm | ownm | (n >= 64 ? 0ull : ~0ull << n));
                // the word a lane with no sink in a batch slot touches with a no-op atomic
                // (its own word: no same-address serialisation)
                const int nopw = lane < agl.nw ? lane : 0;
                constexpr int BLB = MRG ? RQ_MRG_BLB : 8;
                // MRG: an event whose stream already played since the last reset (a post, or
                // an own-stream arrival) finds every sink of its row out of the top-1 set and
                // valid -- its deltas are 0 and it needs no walk (~43 % of C5's events)
                uint64_t needm = ~0ull;
                if (MRG && sk_stamp) {
                    const uint64_t sownm = __ballot(strm_own);
                    const int seg = mbcnt64_incl(ownm) + mbcnt64(sownm);
                    const int nres = __popcll(ownm) + __popcll(sownm);
                    const bool wl = act && !strm_own && degl > 0;
                    bool rep = false;
                    for (int sg = 0; sg <= nres; ++sg) {
                        const bool mine = wl && seg == sg;
                        if (!__ballot(mine)) continue;
                        // the segment's first lane of each stream; then the stamps move on
                        if (mine) atomicMin(&sk_first[tj], lane);
                        wave_lds_sync();
                        if (mine) rep = sk_first[tj] != lane || sk_stamp[tj] == sk_ep + sg;
                        wave_lds_sync();
                        if (mine) {
                            sk_stamp[tj] = sk_ep + sg;
                            sk_first[tj] = 64;
                        }
                        wave_lds_sync();
                    }
                    sk_ep += nres;
                    needm = sgpr_u64(__ballot(!rep));
                }
                // the lanes left to visit: posts, events played alone, batched events (all
                // wave-uniform: kept in SGPRs, the batch bookkeeping on the scalar unit)
                uint64_t pend = sgpr_u64((ownm | specm | needm) & (n >= 64 ? ~0ull : ((1ull << n) - 1)));
                while (pend) {
                    const int q = __builtin_amdgcn_readfirstlane(__builtin_ctzll(pend));
                    if ((ownm >> q) & 1ull) {
                        agl.own(ag, lane);
                        if (DM) {
                            acnt = wlane(acnt, ag.cnt[0], q);
                            aval = wlane(aval, ag.nvalid, q);
                        } else {
                            osl = wlane(osl, (int)(uint32_t)ag.sumR, q);
                            osh = wlane(osh, (int)(ag.sumR >> 32), q);
                            oval = wlane(oval, ag.nvalid, q);
                            ocnt[0] = wlane(ocnt[0], ag.cnt[0], q);
                        }
                    }
                    if ((specm >> q) & 1ull) {
                        // an own-stream arrival, or no / more than 128 sinks: one event alone
                        const int c_b = ag.cnt[0], v_b = ag.nvalid;
                        const bool sown = !opt && bcast_i(tj, q) == a.ctrl_idx;
                        if (sown) {
                            agl.own(ag, lane);
                        } else if (a.dbg != 2) {
                            const int f0 = bcast_i(e0, q), f1 = bcast_i(e1, q);
                            const int ca = f0 + lane < f1 ? colat(f0 + lane) : 0;
                            const int cb = f0 + 64 + lane < f1 ? colat(f0 + 64 + lane) : 0;
                            agl.wall_pf(ag, colat, ca, cb, f0, f1, bcast_i(od, q), lane);
                        }
                        if (DM) {
                            if (sown) {
                                acnt = wlane(acnt, ag.cnt[0], q);
                                aval = wlane(aval, ag.nvalid, q);
                            } else {
                                dcnt = wlane(dcnt, c_b - ag.cnt[0], q);
                                dval = wlane(dval, ag.nvalid - v_b, q);
                            }
                        } else {
                            wsl = wlane(wsl, (int)(uint32_t)ag.sumR, q);
                            wsh = wlane(wsh, (int)(ag.sumR >> 32), q);
                            wval = wlane(wval, ag.nvalid, q);
                            wcnt[0] = wlane(wcnt[0], ag.cnt[0], q);
                        }
                        pend &= pend - 1;
                        continue;
                    }
                    if (!((needm >> q) & 1ull)) {   // a post before a skipped event
                        pend &= pend - 1;
                        continue;
                    }
                    // the next <= BLB needed events from q, all before the next break (8; the
                    // merged-stream instances RQ_MRG_BLB (5) so the batch fits their 128
                    // VGPRs); without skipping, events q .. q+m-1
                    const uint64_t nb = q < 63 ? brk & (~0ull << (q + 1)) : 0ull;
                    uint64_t cand = needm & (nb ? (nb & (0ull - nb)) - 1 : ~0ull) & (~0ull << q);
                    int evk[BLB];
                    int m = 0, lastq = q;
#pragma unroll
                    for (int k = 0; k < BLB; ++k) {
                        evk[k] = 63;
                        if (cand) {
                            evk[k] = __builtin_ctzll(cand);
                            lastq = evk[k];
                            ++m;
                            cand &= cand - 1;
                        }
                    }
                    pend = lastq >= 63 ? 0ull : pend & (~0ull << (lastq + 1));
                    // straight-line batch: every slot loads and issues its atomics (slots
                    // past m and lanes past the event's sinks: index 0, no-op masks), so the
                    // compiler keeps the 16 loads and then the atomics in flight together
                    auto batch = [&](auto vf) __attribute__((always_inline)) {
                        constexpr bool VF = decltype(vf)::value;   // V all ones: leave it
                        int ca[BLB], cb[BLB];
                        bool aa[BLB], ab[BLB];
#pragma unroll
                        for (int k = 0; k < BLB; ++k) {
                            const int f0 = bcast_i(e0, evk[k]);
                            const int f1 = k < m ? bcast_i(e1, evk[k]) : f0;
                            aa[k] = f0 + lane < f1;
                            ab[k] = f0 + 64 + lane < f1;
                            ca[k] = colat(aa[k] ? f0 + lane : 0);
                            cb[k] = colat(ab[k] ? f0 + 64 + lane : 0);
                        }
                        uint32_t ta[BLB], tb[BLB], va[BLB], vb[BLB];
#pragma unroll
                        for (int k = 0; k < BLB; ++k) {
                            const uint32_t ba = aa[k] ? 1u << (ca[k] & 31) : 0u;
                            const uint32_t bb = ab[k] ? 1u << (cb[k] & 31) : 0u;
                            const int wa = aa[k] ? ca[k] >> 5 : nopw;
                            const int wb = ab[k] ? cb[k] >> 5 : nopw;
                            ta[k] = atomicAnd(&agl.T[wa], ~ba) & ba;
                            tb[k] = atomicAnd(&agl.T[wb], ~bb) & bb;
                            if (!VF) {
                                va[k] = ba & ~atomicOr(&agl.V[wa], ba);
                                vb[k] = bb & ~atomicOr(&agl.V[wb], bb);
                            }
                        }
#pragma unroll
                        for (int k = 0; k < BLB; ++k) {
                            if (k < m) {
                                const int qk = evk[k];
                                const int dk = popc(__ballot(ta[k] != 0u)) + popc(__ballot(tb[k] != 0u));
                                const int dv = VF ? 0 : popc(__ballot(va[k] != 0u)) + popc(__ballot(vb[k] != 0u));
                                ag.cnt[0] -= dk;
                                ag.nvalid += dv;
                                if (DM) {
                                    dcnt = wlane(dcnt, dk, qk);
                                    if (!VF) dval = wlane(dval, dv, qk);
                                } else {
                                    ag.sumR += bcast_i(degl, qk);
                                    ag.sumF += bcast_i(od, qk);
                                    wsl = wlane(wsl, (int)(uint32_t)ag.sumR, qk);
                                    wsh = wlane(wsh, (int)(ag.sumR >> 32), qk);
                                    wval = wlane(wval, ag.nvalid, qk);
                                    wcnt[0] = wlane(wcnt[0], ag.cnt[0], qk);
                                }
                            }
                        }
                    };
                    if (ag.nvalid >= a.n_sinks)
                        batch(std::true_type{});
                    else
                        batch(std::false_type{});
                }
                if constexpr (DM) {
                    // rank sums: a wall event adds its degree (sumR) and its follower edges
                    // (sumF); a post or own-stream arrival drops sumF from sumR (AggL)
                    const bool rst = own_b || strm_own;
                    const uint64_t rm = __ballot(rst);
                    const bool hasr = mbcnt64_incl(rm) != 0;   // reset at or before #lane
                    const bool wl = act && !strm_own;
                    const int deg = wl ? e1 - e0 : 0;
                    const int odv = wl ? od : 0;
                    SegFlags sf;
                    sf.init(rst);
                    const int pdeg = (int)wave_scan_add((uint32_t)deg);
                    const int64_t sfq = (int64_t)(int)sf.scan_add((uint32_t)odv) + (hasr ? 0 : F0);
                    int64_t dec = 0;
                    // counts: the last anchor at or before #lane, minus / plus the deltas since
                    const uint32_t P = wave_scan_add((uint32_t)dcnt), PV = wave_scan_add((uint32_t)dval);
                    int bc = cnt0, bv = val0;
                    uint32_t oc = 0u, ov = 0u;
                    for (uint64_t bm = rm; bm; bm &= bm - 1) {
                        const int r = __ffsll((unsigned long long)bm) - 1;
                        const int64_t D = r == 0 ? F0 : bcast_i64(sfq, r - 1);
                        if (lane >= r) {
                            dec += D;
                            bc = bcast_i(acnt, r);
                            bv = bcast_i(aval, r);
                            oc = (uint32_t)bcast_i((int)P, r) - (uint32_t)bcast_i(dcnt, r);
                            ov = (uint32_t)bcast_i((int)PV, r) - (uint32_t)bcast_i(dval, r);
                        }
                    }
                    wsum = S0 + pdeg - dec;
                    osum = S0 + (pdeg - deg) - dec;
                    wcnt[0] = bc - (int)(P - oc);
                    wval = bv + (int)(PV - ov);
                    ocnt[0] = acnt;
                    oval = aval;
                    if (n > 0) {
                        ag.sumR = bcast_i64(wsum, n - 1);
                        ag.sumF = bcast_i64(sfq, n - 1);
                    }
                } else {
                    wsum = (int64_t)(((uint64_t)(uint32_t)wsh << 32) | (uint32_t)wsl);
                    osum = (int64_t)(((uint64_t)(uint32_t)osh << 32) | (uint32_t)osl);
                }
              } else {
                // the first 128 sink columns of events q + 1 .. q + PF are in flight while
              // event q runs (global columns: an L2 round trip outlasts one event's work)
              constexpr int PF = col_lds ? 1 : 4;
              int pa[PF], pb[PF];
              auto fetch = [&](int q, int& ra, int& rb) __attribute__((always_inline)) {
                  ra = rb = 0;
                  if (q < n) {
                      const int f0 = bcast_i(e0, q), f1 = bcast_i(e1, q);
                      ra = f0 + lane < f1 ? colat(f0 + lane) : 0;
                      rb = f0 + 64 + lane < f1 ? colat(f0 + 64 + lane) : 0;
                  }
              };
#pragma unroll
              for (int d = 0; d < PF; ++d) fetch(d, pa[d], pb[d]);
              for (int q = 0; q < n; ++q) {
                const int ca = pa[0], cb = pb[0];
                const int qe0 = bcast_i(e0, q), qe1 = bcast_i(e1, q);
#pragma unroll
                for (int d = 0; d + 1 < PF; ++d) {
                    pa[d] = pa[d + 1];
                    pb[d] = pb[d + 1];
                }
                fetch(q + PF, pa[PF - 1], pb[PF - 1]);
                if ((ownm >> q) & 1ull) {
                    if (BL) agl.own(ag, lane);
                    else ag.own(rank, folat, a.n_fol, lane);
                    if (lane == q) {
                        osum = ag.sumR;
                        oval = ag.nvalid;
#pragma unroll
                        for (int kq = 0; kq < NK; ++kq) ocnt[kq] = ag.cnt[kq];
                    }
                }
                const int jw = bcast_i(tj, q);
                if (!opt && jw == a.ctrl_idx) {
                    if (BL) agl.own(ag, lane);
                    else ag.own(rank, folat, a.n_fol, lane);
                } else if (a.dbg != 2) {
                    if (BL) agl.wall_pf(ag, colat, ca, cb, qe0, qe1, bcast_i(od, q), lane);
                    else ag.wall_pf(rank, colat, ca, cb, qe0, qe1, bcast_i(od, q), lane);
                }
                if (lane == q) {
                    wsum = ag.sumR;
                    wval = ag.nvalid;
#pragma unroll
                    for (int kq = 0; kq < NK; ++kq) wcnt[kq] = ag.cnt[kq];
                }
              }
              }
            }
            const uint64_t mo = __ballot(has_o), ma = mo | __ballot(has_w);
            n_events += n + __popcll(ownm);
            posts += __popcll(mo) + __popcll(__ballot(has_w && strm_own));
            world += __popcll(__ballot(has_w && !strm_own));
            if (ma && place_rows<NK>(rs, ma, has_o, has_w, ot, tt, osum, oval, ocnt, wsum, wval, wcnt, status))
                stop = true;
        }
        if (stop || fin || cut) break;
    }
    // the controller's last post after the final arrival (or the tile max_events cut)
    if (!stop && opt && opt_next <= a.end && (LOG || a.max_events < 0 || n_events < a.max_events)) {
        if (LOG) {
            event(opt_next, true, 0, 0, 0);
        } else {
            if (a.ev_t && lane == 0) {
                if (n_events < a.ev_cap) {
                    a.ev_t[o * a.ev_cap + n_events] = opt_next;
                    a.ev_src[o * a.ev_cap + n_events] = a.ctrl_idx;
                } else {
                    status |= RQ_ST_ROWS_OVERFLOW;
                }
            }
            ++n_events;
            if (BITS) {
                agb.own();
                agb.sync();
                ag.sumR = agb.sumR;
                ag.nvalid = agb.nvalid;
                ag.cnt[0] = agb.cnt[0];
            } else if (BL) {
                agl.own(ag, lane);
            } else {
                ag.own(rank, folat, a.n_fol, lane);
            }
            if (a.n_fol > 0) {
                ++posts;
                int64_t rr = rs.nrow;
                if (rs.nrow > 0 && opt_next == rs.last_t) {
                    status |= RQ_ST_TIE;
                    rr = rs.nrow - 1;
                } else if (rs.nrow >= rs.cap) {
                    status |= RQ_ST_ROWS_OVERFLOW;
                    rr = -1;
                } else {
                    ++rs.nrow;
                    rs.s0 = rs.nrow;
                    rs.last_t = opt_next;
                }
                if (rr >= 0 && lane == 0) {
                    rs.write(rr, opt_next, (double)ag.sumR, ag.nvalid, ag.cnt);
                }
            }
        }
    }
    if (LOG && pend) close_row();
    if (BITS) {
        agb.sync();
        ag.nvalid = agb.nvalid;
    }
    rs.flush(lane);
    if (LOG && a.ev_t) es.flush(lane);
    if (lane == 0) {
        int64_t* cnto = a.counts + o * 4;
        cnto[0] = posts;
        cnto[1] = world;
        cnto[2] = n_events;
        cnto[3] = rs.nrow;
        a.sall[rl] = LOG ? ax.nvalid : ag.nvalid;   // BITS: synced below
        if (rs.nrow == 0) status |= RQ_ST_EMPTY;
        if (status) atomicOr(&a.status[o], status);
    }
    if (!a.wq) break;
    int nx = 0;
    if (lane == 0) nx = atomicAdd(a.wq, 1);
    qi = nslot + __builtin_amdgcn_readfirstlane(nx);
    }   // replica loop
}

// ============================================================================
// 3. scan: numpy-order integrals over the pivot rows, one wavefront per replica
// ============================================================================
template <int NK, int WPE>
__global__ __launch_bounds__(256, WPE) void rq_scan(ScanArgs a)
{
    constexpr int NV = NK + 2;
    extern __shared__ double lds_scan[];
    const int w = threadIdx.x >> 6;
    double* lds = lds_scan + (size_t)w * npsum_lds_doubles<NV>();
    // persistent: a wave's first replica is its slot, the next ones come from the
    // queue (10k one-wave replicas over ~4k resident waves otherwise leave a tail)
    const int64_t nslot = (int64_t)gridDim.x * 4;
    int64_t rl = (int64_t)blockIdx.x * 4 + w;
    while (rl < a.n_chunk) {
        const int64_t i = a.chunk0 + rl;
        const int64_t n = a.nrows[i * a.nrows_stride];
        const double S = (double)a.sall[rl];
        const int64_t rbase = a.row_stride * rl;
        const double* Rt = a.rows_t + rbase;
        const double* Rs = a.rows_sum + rbase;
        const uint32_t* Rv = a.rows_valid + rbase;
        const uint32_t* Rc = a.rows_cnt + rbase * NK;
        const double end = a.end;
        double* out = a.metrics + i * NV;
        if (n <= 0) {
            if (lane_id() < NV) out[lane_id()] = __builtin_nan("");
        } else {
            struct Row {
                double t, s;
                uint32_t v, c[NK];
            };
            auto ld = [&](uint32_t kk) {
                Row r;
                r.t = Rt[kk];
                r.s = Rs[kk];
                r.v = Rv[kk];
#pragma unroll
                for (int q = 0; q < NK; ++q) r.c[q] = Rc[kk * NK + q];
                return r;
            };
            auto tld = [&](uint32_t kk) { return Rt[kk]; };
            auto vf = [&](const Row& r, double t1, double* v) {
                const double dt = t1 - r.t;
                const double m = r.s / (double)r.v;
#pragma unroll
                for (int q = 0; q < NK; ++q) v[q] = ((double)r.c[q] / S) * dt;
                v[NK] = m * dt;
                v[NK + 1] = (m * m) * dt;
            };
            double res[NV];
            // fewer waves / SIMD: the registers for a whole leaf (<= 16 rows per lane) in
            // one trip (2), or for the 10-11 rows of C3's 80-88-row leaves (3)
            wave_npsum_rows<NV, true, Row, (WPE <= 2 ? 16 : WPE == 3 ? 12 : 8)>(n, end, ld, tld, vf, lds, res);
            if (lane_id() == 0) {
#pragma unroll
                for (int s = 0; s < NV; ++s) out[s] = res[s];
            }
        }
        if (!a.wq) break;
        int nx = 0;
        if (lane_id() == 0) nx = atomicAdd(a.wq, 1);
        rl = nslot + __builtin_amdgcn_readfirstlane(nx);
    }
}

// ============================================================================
// launch wrappers
// ============================================================================
int rq_cu_count()
{
    // thread-safe one-time query (function-local static initialisation)
    static const int n = [] {
        int dev = 0, c = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0)
            c = 256;
        return c;
    }();
    return n;
}
template <int SPL, int NK, class COL, int W, bool LOG, bool BITS = false, bool BL = false, bool GS = false,
          bool MRG = false, bool GT = false>
static int occ_t(int wpb, size_t lds);
template <int SPL, int NK, class COL, int W, bool LOG, bool BITS = false, bool BL = false, bool GS = false,
          bool MRG = false, bool GT = false>
static hipError_t launch_sweep_t(const SweepArgs& a, hipStream_t s)
{
    unsigned blocks = (unsigned)((a.n_chunk + a.wpb - 1) / a.wpb);
    if (a.wq) {
        // persistent grid: every resident wave slot once, the rest from the queue
        const int nb_c = occ_t<SPL, NK, COL, W, LOG, BITS, BL, GS, MRG, GT>(a.wpb, a.lds_total);
        const unsigned cap = (unsigned)(nb_c > 0 ? nb_c : 1) * (unsigned)rq_cu_count();
        if (cap < blocks) blocks = cap;
    }
    if (GS) {   // one global per-sink state slot per wave of the grid
        const unsigned cap = (unsigned)(a.gs_slots / a.wpb);
        if (!a.wq || cap < 1) return hipErrorInvalidValue;
        if (cap < blocks) blocks = cap;
    }
    hipLaunchKernelGGL((rq_sweep<SPL, NK, COL, W, LOG, BITS, BL, GS, MRG, GT>), dim3(blocks), dim3(64 * a.wpb), a.lds_total,
                       s, a);
    return hipGetLastError();
}

template <int SPL, class COL, int W, bool LOG, bool GS = false>
static hipError_t launch_sweep_k(const SweepArgs& a, int nK, hipStream_t s)
{
    switch (nK) {
    case 1: return launch_sweep_t<SPL, 1, COL, W, LOG, false, false, GS>(a, s);
    case 2: return launch_sweep_t<SPL, 2, COL, W, LOG, false, false, GS>(a, s);
    case 3: return launch_sweep_t<SPL, 3, COL, W, LOG, false, false, GS>(a, s);
    default: return launch_sweep_t<SPL, 4, COL, W, LOG, false, false, GS>(a, s);
    }
}

// the fast general sweep: a register window of W = 4 arrivals per source
constexpr int kGW = 4;
template <int SPL>
static hipError_t launch_sweep_c(const SweepArgs& a, int nK, int col16, int bits, hipStream_t s)
{
    if constexpr (SPL >= 2)
        if (bits == 2)   // K = 1 on per-wave LDS sink bits (> 64 sources)
            return col16 ? launch_sweep_t<SPL, 1, uint16_t, kGW, false, false, true>(a, s)
                         : launch_sweep_t<SPL, 1, int, kGW, false, false, true>(a, s);
    if (bits)   // K = 1 on sink bitsets
        return launch_sweep_t<SPL, 1, uint16_t, kGW, false, true>(a, s);
    return col16 ? launch_sweep_k<SPL, uint16_t, kGW, false>(a, nK, s)
                 : launch_sweep_k<SPL, int, kGW, false>(a, nK, s);
}

// the sequential sweep on merged streams (> RQ_MAX_STREAMS sources): one instance per K
// variant and per-sink state placement (GS); per-stream tables in global memory (GT)
template <bool GS>
static hipError_t launch_sweep_lm(const SweepArgs& a, int nK, hipStream_t s)
{
    switch (nK) {
    case 1: return launch_sweep_t<1, 1, int, 4, true, false, false, GS, true, true>(a, s);
    case 2: return launch_sweep_t<1, 2, int, 4, true, false, false, GS, true, true>(a, s);
    case 3: return launch_sweep_t<1, 3, int, 4, true, false, false, GS, true, true>(a, s);
    default: return launch_sweep_t<1, 4, int, 4, true, false, false, GS, true, true>(a, s);
    }
}

// the fast sweep on merged streams: one instance per (K variant, column type)
template <int NK, class COL>
static hipError_t launch_sweep_mk(const SweepArgs& a, hipStream_t s)
{
    return launch_sweep_t<1, NK, COL, kGW, false, false, false, false, true>(a, s);
}
// the same with the per-stream tables in global memory (GT: more streams than the LDS
// tables take; global columns, no sink bitsets)
static hipError_t launch_sweep_mg(const SweepArgs& a, int nK, int bits, hipStream_t s)
{
    if (bits == 2) return launch_sweep_t<1, 1, int, kGW, false, false, true, false, true, true>(a, s);
    if (bits) return hipErrorInvalidValue;
    switch (nK) {
    case 1: return launch_sweep_t<1, 1, int, kGW, false, false, false, false, true, true>(a, s);
    case 2: return launch_sweep_t<1, 2, int, kGW, false, false, false, false, true, true>(a, s);
    case 3: return launch_sweep_t<1, 3, int, kGW, false, false, false, false, true, true>(a, s);
    default: return launch_sweep_t<1, 4, int, kGW, false, false, false, false, true, true>(a, s);
    }
}
template <class COL>
static hipError_t launch_sweep_m(const SweepArgs& a, int nK, int bits, hipStream_t s)
{
    if (bits == 2) return launch_sweep_t<1, 1, COL, kGW, false, false, true, false, true>(a, s);
    if (bits) return launch_sweep_t<1, 1, uint16_t, kGW, false, true, false, false, true>(a, s);
    switch (nK) {
    case 1: return launch_sweep_mk<1, COL>(a, s);
    case 2: return launch_sweep_mk<2, COL>(a, s);
    case 3: return launch_sweep_mk<3, COL>(a, s);
    default: return launch_sweep_mk<4, COL>(a, s);
    }
}
template <class COL>
static int occ_m(int nK, int bits, int wpb, size_t lds)
{
    if (bits == 2) return occ_t<1, 1, COL, kGW, false, false, true, false, true>(wpb, lds);
    if (bits) return occ_t<1, 1, uint16_t, kGW, false, true, false, false, true>(wpb, lds);
    switch (nK) {
    case 1: return occ_t<1, 1, COL, kGW, false, false, false, false, true>(wpb, lds);
    case 2: return occ_t<1, 2, COL, kGW, false, false, false, false, true>(wpb, lds);
    case 3: return occ_t<1, 3, COL, kGW, false, false, false, false, true>(wpb, lds);
    default: return occ_t<1, 4, COL, kGW, false, false, false, false, true>(wpb, lds);
    }
}

hipError_t rq_launch_gen(const GenArgs& a, hipStream_t s)
{
    if (a.n_chunk <= 0 || a.n_str <= 0) return hipSuccess;
    const unsigned gy = (unsigned)std::min(a.n_str, 32768);
    dim3 grid((unsigned)((a.n_chunk + 255) / 256), gy, (unsigned)((a.n_str + gy - 1) / gy));
    hipLaunchKernelGGL(rq_gen_streams, grid, dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t rq_launch_sweep(const SweepArgs& a, int spl, int nK, int col16, int log, int bits, hipStream_t s)
{
    if (a.n_chunk <= 0) return hipSuccess;
    // event log / max_events / duplicate edges / > 512 sources: the sequential variant,
    // W = 8; one source per lane when they fit (the per-lane ring state of eight sources
    // costs ~200 VGPRs and spills; 16 / 32 per lane spill more -- correctness instances
    // for 513..2048 sources, global columns only)
    // > 2048 sources: the sequential sweep on merged streams (global columns, 4-deep
    // rings the instance never fills)
    if (log && spl <= 0) return log == 2 ? launch_sweep_lm<true>(a, nK, s) : launch_sweep_lm<false>(a, nK, s);
    if (spl < 0) return launch_sweep_mg(a, nK, bits, s);   // merged streams, global tables
    if (log == 2)
        switch (spl) {
        case 1: return col16 ? launch_sweep_k<1, uint16_t, 8, true, true>(a, nK, s)
                             : launch_sweep_k<1, int, 8, true, true>(a, nK, s);
        case 8: return col16 ? launch_sweep_k<8, uint16_t, 8, true, true>(a, nK, s)
                             : launch_sweep_k<8, int, 8, true, true>(a, nK, s);
        case 16: return launch_sweep_k<16, int, 8, true, true>(a, nK, s);
        default: return launch_sweep_k<32, int, 4, true, true>(a, nK, s);   // 4-deep rings: LDS
        }
    if (log)
        switch (spl) {
        case 1: return col16 ? launch_sweep_k<1, uint16_t, 8, true>(a, nK, s)
                             : launch_sweep_k<1, int, 8, true>(a, nK, s);
        case 8: return col16 ? launch_sweep_k<8, uint16_t, 8, true>(a, nK, s)
                             : launch_sweep_k<8, int, 8, true>(a, nK, s);
        case 16: return launch_sweep_k<16, int, 8, true>(a, nK, s);
        default: return launch_sweep_k<32, int, 4, true>(a, nK, s);
        }
    if (spl == 0)   // merged streams
        return col16 ? launch_sweep_m<uint16_t>(a, nK, bits, s) : launch_sweep_m<int>(a, nK, bits, s);
    switch (spl) {
    case 1: return launch_sweep_c<1>(a, nK, col16, bits, s);
    case 2: return launch_sweep_c<2>(a, nK, col16, bits, s);
    case 4: return launch_sweep_c<4>(a, nK, col16, bits, s);
    default: return launch_sweep_c<8>(a, nK, col16, bits, s);
    }
}

// blocks of 64*wpb threads per CU the chosen sweep instance reaches with `lds`
// bytes of dynamic LDS (VGPR, SGPR and LDS limits all applied by the runtime)
template <int SPL, int NK, class COL, int W, bool LOG, bool BITS, bool BL, bool GS, bool MRG, bool GT>
static int occ_t(int wpb, size_t lds)
{
    return rq_occupancy(rq_sweep<SPL, NK, COL, W, LOG, BITS, BL, GS, MRG, GT>, 64 * wpb, lds);
}
template <int SPL, class COL, int W, bool LOG, bool GS = false>
static int occ_k(int nK, int wpb, size_t lds)
{
    switch (nK) {
    case 1: return occ_t<SPL, 1, COL, W, LOG, false, false, GS>(wpb, lds);
    case 2: return occ_t<SPL, 2, COL, W, LOG, false, false, GS>(wpb, lds);
    case 3: return occ_t<SPL, 3, COL, W, LOG, false, false, GS>(wpb, lds);
    default: return occ_t<SPL, 4, COL, W, LOG, false, false, GS>(wpb, lds);
    }
}
template <int SPL>
static int occ_c(int nK, int col16, int W, int bits, int wpb, size_t lds)
{
    (void)W;
    if constexpr (SPL >= 2)
        if (bits == 2)
            return col16 ? occ_t<SPL, 1, uint16_t, kGW, false, false, true>(wpb, lds)
                         : occ_t<SPL, 1, int, kGW, false, false, true>(wpb, lds);
    if (bits) return occ_t<SPL, 1, uint16_t, kGW, false, true>(wpb, lds);
    return col16 ? occ_k<SPL, uint16_t, kGW, false>(nK, wpb, lds) : occ_k<SPL, int, kGW, false>(nK, wpb, lds);
}
int rq_sweep_blocks_per_cu(int spl, int nK, int col16, int W, int log, int bits, int wpb, size_t lds)
{
    if (spl < 0 && !log) {   // merged streams, global tables (launch_sweep_mg)
        if (bits == 2) return occ_t<1, 1, int, kGW, false, false, true, false, true, true>(wpb, lds);
        if (bits) return 0;
        switch (nK) {
        case 1: return occ_t<1, 1, int, kGW, false, false, false, false, true, true>(wpb, lds);
        case 2: return occ_t<1, 2, int, kGW, false, false, false, false, true, true>(wpb, lds);
        case 3: return occ_t<1, 3, int, kGW, false, false, false, false, true, true>(wpb, lds);
        default: return occ_t<1, 4, int, kGW, false, false, false, false, true, true>(wpb, lds);
        }
    }
    if (log && spl <= 0) {   // the sequential sweep on merged streams (launch_sweep_lm)
        const bool gs = log == 2;
        switch (nK) {
        case 1: return gs ? occ_t<1, 1, int, 4, true, false, false, true, true, true>(wpb, lds)
                          : occ_t<1, 1, int, 4, true, false, false, false, true, true>(wpb, lds);
        case 2: return gs ? occ_t<1, 2, int, 4, true, false, false, true, true, true>(wpb, lds)
                          : occ_t<1, 2, int, 4, true, false, false, false, true, true>(wpb, lds);
        case 3: return gs ? occ_t<1, 3, int, 4, true, false, false, true, true, true>(wpb, lds)
                          : occ_t<1, 3, int, 4, true, false, false, false, true, true>(wpb, lds);
        default: return gs ? occ_t<1, 4, int, 4, true, false, false, true, true, true>(wpb, lds)
                           : occ_t<1, 4, int, 4, true, false, false, false, true, true>(wpb, lds);
        }
    }
    if (log == 2)
        switch (spl) {
        case 1: return col16 ? occ_k<1, uint16_t, 8, true, true>(nK, wpb, lds) : occ_k<1, int, 8, true, true>(nK, wpb, lds);
        case 8: return col16 ? occ_k<8, uint16_t, 8, true, true>(nK, wpb, lds) : occ_k<8, int, 8, true, true>(nK, wpb, lds);
        case 16: return occ_k<16, int, 8, true, true>(nK, wpb, lds);
        default: return occ_k<32, int, 4, true, true>(nK, wpb, lds);
        }
    if (log)
        switch (spl) {
        case 1: return col16 ? occ_k<1, uint16_t, 8, true>(nK, wpb, lds) : occ_k<1, int, 8, true>(nK, wpb, lds);
        case 8: return col16 ? occ_k<8, uint16_t, 8, true>(nK, wpb, lds) : occ_k<8, int, 8, true>(nK, wpb, lds);
        case 16: return occ_k<16, int, 8, true>(nK, wpb, lds);
        default: return occ_k<32, int, 4, true>(nK, wpb, lds);
        }
    if (spl == 0) return col16 ? occ_m<uint16_t>(nK, bits, wpb, lds) : occ_m<int>(nK, bits, wpb, lds);
    switch (spl) {
    case 1: return occ_c<1>(nK, col16, W, bits, wpb, lds);
    case 2: return occ_c<2>(nK, col16, W, bits, wpb, lds);
    case 4: return occ_c<4>(nK, col16, W, bits, wpb, lds);
    default: return occ_c<8>(nK, col16, W, bits, wpb, lds);
    }
}

template <int NK, int WPE>
static unsigned scan_blocks(const ScanArgs& a, size_t lds)
{
    unsigned blocks = (unsigned)((a.n_chunk + 3) / 4);
    if (a.wq) {   // persistent grid: every resident block once
        const int nb = rq_occupancy(rq_scan<NK, WPE>, 256, lds);
        const unsigned cap = (unsigned)(nb > 0 ? nb : 1) * (unsigned)rq_cu_count();
        if (cap < blocks) blocks = cap;
    }
    return blocks;
}
template <int NK>
static hipError_t launch_scan_t(const ScanArgs& a, hipStream_t s)
{
    const size_t lds = 4 * npsum_lds_doubles<NK + 2>() * sizeof(double);
    // waves per SIMD the build targets (VGPR budget): A/B knob RQ_SCAN_WPE.  2 (a whole
    // leaf per trip, 176 VGPRs at K = 1) measured 0.296 ms on the C3 step's scan against
    // 0.313 / 0.332 / 0.645 / 0.805 ms at 3 / 4 / 6 / 8 (same box, profiles/r03_scan_ab.txt)
    static const int wpe = getenv("RQ_SCAN_WPE") ? atoi(getenv("RQ_SCAN_WPE")) : 2;
    if (wpe >= 8)
        hipLaunchKernelGGL((rq_scan<NK, 8>), dim3(scan_blocks<NK, 8>(a, lds)), dim3(256), lds, s, a);
    else if (wpe >= 6)
        hipLaunchKernelGGL((rq_scan<NK, 6>), dim3(scan_blocks<NK, 6>(a, lds)), dim3(256), lds, s, a);
    else if (wpe >= 4)
        hipLaunchKernelGGL((rq_scan<NK, 4>), dim3(scan_blocks<NK, 4>(a, lds)), dim3(256), lds, s, a);
    else if (wpe == 3)
        hipLaunchKernelGGL((rq_scan<NK, 3>), dim3(scan_blocks<NK, 3>(a, lds)), dim3(256), lds, s, a);
    else
        hipLaunchKernelGGL((rq_scan<NK, 2>), dim3(scan_blocks<NK, 2>(a, lds)), dim3(256), lds, s, a);
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
