// rq_sweep_fw.hip -- the fused windowed sweep (<= 64 sources: arrivals generated
// in-kernel) and its launch wrappers, called by the C ABI in rq_api.cpp.  The
// general sweep, the stream generator and the scan are in rq_kernels.hip.
//
// Kernel role (reference file:line it replaces): Manager.run_dynamic
// opt_model.py:241-314 with every broadcaster's get_next_interval (Poisson :424-433,
// Poisson2 :396-405, Hawkes :466-490, PiecewiseConst :642-663, RealData :722-750,
// Opt :502-544, OptPWSignificance :547-623) + State.apply_event :61-83 + the per-row
// part of rank_of_src_in_df utils.py:38-56.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rq_device.h"
#include "rq_internal.h"
#include "rq_sweep_core.h"
#include "rq_gen.h"
#include <type_traits>
#include <cstdlib>

#pragma clang fp contract(off)

using namespace rq;

// ============================================================================
// fused windowed sweep (n_str <= 64).  Lane j owns stream j and GENERATES its
//     arrivals (SrcGen) into an LDS ring -- no stream buffer, no generator
//     kernel.  A tile is every pending arrival earlier than a cut tau, found from
//     the next H arrivals of each ring held in registers (a ring's unseen
//     arrivals are >= its H-th, so tau <= min over rings of the H-th keeps the
//     tile complete); tau adapts so a tile holds <= 64 arrivals.  The tile is
//     staged in source order and rank-sorted into (t, stream) order -- the
//     reference's (time, src_id) order (opt_model.py:279-281).  Phase B is the
//     same controller; phase C for K = 1 runs lane-parallel over the tile's
//     events: per sink-bitset word, segmented prefix ORs (segments start at the
//     posts) give each event's top-1 set, plain prefix ORs its valid set.
// ============================================================================
// MRG: the arrivals come pre-generated (rq_gen_streams) and merged into the replica's
// (t, stream) sequence (rq_merge_streams): a tile is its next 64 entries, loaded one tile
// ahead, and phase A (refill passes, window cut, rank sort) disappears
template <int NK, class COL, int W, int H, bool BITS, bool PW, bool MRG>
__device__ __forceinline__ void sweep_fw_body(SweepArgs a)
{
    static_assert((W & (W - 1)) == 0 && H <= W, "ring");
    extern __shared__ double lds_g[];
    char* base = reinterpret_cast<char*>(lds_g);
    const int lane = lane_id();
    const int w = threadIdx.x >> 6;
    int* cptr = reinterpret_cast<int*>(base + a.lds_ptr);
    int* odf = reinterpret_cast<int*>(base + a.lds_odf);
    int* cbf = reinterpret_cast<int*>(base + a.lds_cbf);
    constexpr bool col_lds = sizeof(COL) == 2;
    COL* col_l = reinterpret_cast<COL*>(base + a.lds_col);
    const int* col_g = a.csr_col;
    if (col_lds && !BITS)
        for (int e = threadIdx.x; e < a.n_csr; e += blockDim.x) col_l[e] = (COL)a.csr_col[e];
    uint32_t* msk = reinterpret_cast<uint32_t*>(base + a.lds_mask);
    const int ms = a.mstride;
    if (BITS)   // row n_str stays zero: the mask row of a lane without a wall event
        for (int e = threadIdx.x; e < (a.n_str + 1) * ms; e += blockDim.x) {
            const int jj = e / ms, ww = e - jj * ms;
            msk[e] = (jj < a.n_str && ww < a.nw) ? a.masks[jj * a.nw + ww] : 0u;
        }
    uint64_t* etab = reinterpret_cast<uint64_t*>(base + a.lds_etab);
    for (int e = threadIdx.x; e < RQ_EXP_TAB_N; e += blockDim.x) etab[e] = rq_exp_tab_c[e];
    for (int j = threadIdx.x; j <= a.n_str; j += blockDim.x) cptr[j] = a.csr_ptr[j];
    for (int j = threadIdx.x; j < a.n_str; j += blockDim.x) {
        odf[j] = a.outdeg_f[j];
        // the controller (a dynamic source) posts before a wall event at the same time
        // when that source is static (run_dynamic plays a static time only if it is
        // strictly earlier, opt_model.py:289-290) or has a larger src_id (the sorted
        // (t_delta, src_id) of the dynamic sources, :279-281)
        cbf[j] = a.cbf_g[j];   // the graph's table (static sources, RQ_SRCF_DYNAMIC)
    }
    __syncthreads();   // block-shared tables ready; no block barrier below this line
    char* wb = base + a.lds_wave + (size_t)w * a.lds_wave_stride;
    double* invc = reinterpret_cast<double*>(wb);
    int16_t* rank = reinterpret_cast<int16_t*>(wb + a.lds_rank_off);   // saturating, exact vs K-1
    // BITS: word w of the follower set F (.x) and of the top-1 set T (.y), read by
    // broadcast LDS loads in phase C (T is written back by the tile's last lane)
    uint2* ft = reinterpret_cast<uint2*>(wb + a.lds_rank_off);
    double* ring = reinterpret_cast<double*>(wb + a.lds_win_off) + lane * (W + 1);   // odd stride
    double* st_t = reinterpret_cast<double*>(wb + a.lds_stage_off);
    int* st_j = reinterpret_cast<int*>(st_t + 64);
    // first replica: the wave's static slot; with a work queue (a.wq) the wave then takes
    // replicas nslot, nslot + 1, ... in queue order until the chunk is exhausted (every
    // wave leaves once the counter passes n_chunk)
    const int64_t nslot = (int64_t)gridDim.x * a.wpb;
    for (int64_t qi = (int64_t)blockIdx.x * a.wpb + w; qi < a.n_chunk;) {
    const int64_t rl = a.order ? (int64_t)a.order[qi] : qi;   // longest first (rq_order_replicas)
    const int64_t o = a.chunk0 + rl;
    const int64_t i = rq_replica_of(a.gen, o);
    const int g = (int)(i / a.n_rep);
    for (int j = lane; j < a.n_str; j += 64) invc[j] = a.inv_c[(int64_t)g * a.n_str + j];
    if (!BITS)
        for (int c = lane; c < a.n_sinks; c += 64) rank[c] = -1;   // NaN: no row yet
    wave_lds_sync();

#ifdef RQ_PHASE_CLOCK
    unsigned long long ck[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long tk = __builtin_amdgcn_s_memtime();
#define RQ_CLK(q)                                                   \
    do {                                                            \
        const unsigned long long t2 = __builtin_amdgcn_s_memtime(); \
        ck[q] += t2 - tk;                                           \
        tk = t2;                                                    \
    } while (0)
#else
#define RQ_CLK(q) \
    do {          \
    } while (0)
#endif
    constexpr bool DEFER = MRG && RQ_MRG_DEFER;   // rows stored one tile late (RowStage::flush_pend)
    SrcGen gen;
    if (lane < a.n_str && !MRG) gen.init(a.gen, lane, i, etab);
    else gen.none();
    int pos = 0, fil = 0;   // arrivals consumed / generated by this lane's source
    // MRG: the replica's merged sequence; lane l holds entry mpos + l of the next tile
    // (entry index of the replica's first entry; opaque at each tile's loads, so no
    // per-lane 64-bit sequence pointers are hoisted out of the tile loop and spilled)
    const int64_t mb = MRG ? rl * a.mrg_stride : 0;
    auto mload = [&](int64_t e, double& t_, int& j_) __attribute__((always_inline)) {
        int64_t x = mb;
        __asm__ volatile("" : "+v"(x));
        t_ = a.mrg_t[x + e];
        j_ = a.mrg_j[x + e];
    };
    const int mlen = MRG ? a.mrg_len[rl] : 0;
    int mpos = 0;
    double nxt_t = RQ_INF;
    int nxt_j = 0;
    if (MRG && lane < mlen) mload(lane, nxt_t, nxt_j);

    const bool opt = a.ctrl_kind == RQ_SRC_OPT || a.ctrl_kind == RQ_SRC_OPTPW;
    // OptPWSignificance only in the PW instances: the thinning loop's registers stay out
    // of the RedQueen controller's allocation
    const double* pwc = PW ? a.pw_c + (size_t)g * a.n_str * a.n_seg : nullptr;
    const double* pwm = PW ? a.pw_max + (size_t)g * a.n_str : nullptr;
    double opt_next = opt ? a.start : RQ_INF;
    const int64_t k = a.seed_mod > 0 ? i % a.seed_mod : i;
    const uint32_t oseed = a.ctrl_seed ? a.ctrl_seed[i] : a.ctrl_seed0 + (uint32_t)k;
    uint64_t ndraw = 0;   // wall events seen so far = the controller's draw index
    auto colat = [&](int e) -> int { return col_lds ? (int)col_l[e] : col_g[e]; };
    const int fol0 = cptr[a.ctrl_idx];
    auto folat = [&](int f) -> int { return colat(fol0 + f); };

    Agg<NK> ag;
    ag.init(a.Ks);
    AggB agb;
    if (BITS) {
        agb.init(msk, a.nw, ms, a.ctrl_idx, lane);
        if (lane < ((a.nw + 1) & ~1)) ft[lane] = make_uint2(agb.F, 0u);   // agb.F = 0 past nw
    }
    RowStage<NK> rs;
    const int64_t rbase = rl * a.cap_rows;
    rs.init(a.rows_t, a.rows_sum, a.rows_valid, a.rows_cnt, rbase, a.cap_rows);

    int64_t n_events = 0, posts = 0, world = 0;
    int status = 0;
    double span = -1.0;   // adaptive tile width in time (< 0: not estimated yet)
    bool stop = false;
    // A refill pass steps every ring below W once and costs the same however few lanes
    // step; passes taken only while >= thr rings are below W keep the lanes busy, and a
    // ring is forced full only when it shows fewer than fw_hmin arrivals (the cut below
    // is bounded by each ring's last visible arrival, so a short ring only narrows it).
    const int thr = a.fw_thr;
    auto refill_pass = [&]() __attribute__((always_inline)) {
#ifdef RQ_PHASE_CLOCK
        ck[6] += 1;   // refill passes
        ck[7] += __popcll(__ballot(!gen.done && fil - pos < W));   // lanes stepping
#endif
        if (!gen.done && fil - pos < W) {
            double tv;
            if (gen.step(&tv, a.end)) {
                ring[fil & (W - 1)] = tv;
                ++fil;
            }
        }
    };
    for (;;) {
        int n = 0;
        bool act, fin;
        double tt;
        int tj;
        if constexpr (MRG) {
            if (mpos >= mlen) break;   // every arrival played
            n = mlen - mpos < 64 ? mlen - mpos : 64;
            act = lane < n;
            tt = act ? nxt_t : RQ_INF;
            tj = act ? nxt_j : 0;
            mpos += n;
            fin = mpos >= mlen;
            if constexpr (DEFER) rs.flush_pend();   // the last tile's rows, ahead of the loads
            // the next tile's loads stay in flight through phases B and C
            nxt_t = RQ_INF;
            nxt_j = 0;
            if (mpos + lane < mlen) mload(mpos + lane, nxt_t, nxt_j);
            RQ_CLK(2);
        } else {
        // ---- A1: opportunistic passes while >= thr rings are below W; if some unfinished
        //      ring shows < hmin arrivals, passes until every ring shows >= hfill ----
        {
            bool hard = __ballot(!gen.done && fil - pos < a.fw_hmin) != 0;
            for (;;) {
                const uint64_t need = __ballot(!gen.done && fil - pos < W);
                if (!need || (!hard && __popcll(need) < thr)) break;
                refill_pass();
                // a forced run lasts until every ring shows >= fw_hfill arrivals
                if (hard) hard = __ballot(!gen.done && fil - pos < a.fw_hfill) != 0;
            }
        }
        RQ_CLK(0);   // A1: ring refills (arrival generation)
        const int avail = fil - pos;
        double v[H];
#pragma unroll
        for (int q = 0; q < H; ++q) v[q] = q < avail ? ring[(pos + q) & (W - 1)] : RQ_INF;
        const bool more = !gen.done || avail > H;        // arrivals past the window exist
        // the last arrival the window shows (avail >= hmin >= 1 for an unfinished ring):
        // this ring's unseen arrivals are >= it, so it bounds the cut
        double vb = v[0];
#pragma unroll
        for (int q = 1; q < H; ++q) vb = q < avail ? v[q] : vb;
        const double tfirst = wave_min_f64(v[0]);
        if (!(tfirst < RQ_INF)) break;                   // everything consumed
        const double tmax = wave_min_f64(more ? vb : RQ_INF);

        // ---- A2: the cut (exclusive): complete below tmax, <= 64 arrivals ----
        int c = 0;
        bool trunc = !(tmax > tfirst);   // a ring's window is all at tfirst: equal-time prefix
        if (!trunc) {
            double cut = tmax;
            if (span > 0.0 && tfirst + span < cut) cut = tfirst + span;
            if (!(cut > tfirst)) cut = next_up(tfirst);
            for (;;) {
                c = 0;
#pragma unroll
                for (int q = 0; q < H; ++q) c += v[q] < cut ? 1 : 0;
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
        if (trunc) {
            // the arrivals equal to tfirst, in stream order, up to the first ring whose
            // window may continue at tfirst, at most 64
            c = 0;
#pragma unroll
            for (int q = 0; q < H; ++q) c += v[q] == tfirst ? 1 : 0;
            const uint64_t bl = __ballot(more && vb == tfirst);
            const int lb = bl ? __ffsll((unsigned long long)bl) - 1 : 64;
            if (lane > lb) c = 0;
        }
        const int off = (int)wave_scan_add((uint32_t)c) - c;
        if (trunc) {
            c = off >= 64 ? 0 : (c < 64 - off ? c : 64 - off);
            n = (int)wave_sum_u32((uint32_t)c);
        }

        RQ_CLK(1);   // window + A2 cut
        // ---- A3: stage in stream order, rank-sort into (t, stream) order ----
#pragma unroll
        for (int q = 0; q < H; ++q)
            if (q < c) {
                st_t[off + q] = v[q];
                st_j[off + q] = lane;
            }
        if (lane >= n) st_t[lane] = RQ_INF;   // the rank loop reads whole blocks of 8
        wave_lds_sync();
        act = lane < n;
        const double ti = act ? st_t[lane] : RQ_INF;
        const int ji = act ? st_j[lane] : 0;
        // rank = #staged arrivals before this one in (t, stream) order (stage_rank:
        // broadcast LDS reads, 8 slots per wait); profiling only: dbg 4 skips it
        const int rnk = a.dbg != 4 ? stage_rank(st_t, n, ti, lane) : lane;
        wave_lds_sync();
        if (act) {
            st_t[rnk] = ti;
            st_j[rnk] = ji;
        }
        wave_lds_sync();
        tt = act ? st_t[lane] : RQ_INF;
        tj = act ? st_j[lane] : 0;
        pos += c;
        fin = !__ballot(!gen.done || pos < fil);
        RQ_CLK(2);   // A3 stage + rank sort
        }   // !MRG

        int e0 = 0, e1 = 0, od = 0;
        if (act) {
            e0 = cptr[tj];
            e1 = cptr[tj + 1];
            od = odf[tj];
        }
        // ---- B: RedQueen controller over the tile ----
        uint64_t ownm = 0;
        double ot = RQ_INF;
        if (opt && a.dbg != 3) controller_tile<PW>(n, act, tt, tj, invc, cbf, oseed, ndraw, opt_next, ownm, ot, pwc, pwm, a.n_seg,
                            a.period);

        RQ_CLK(3);   // B controller
        // max_events: the tile keeps the events numbered below it, the replica ends here
        if (a.max_events >= 0 && truncate_tile(a.max_events, n_events, n, act, tt, tj, ownm, ot, opt_next))
            fin = true;
        // ---- C: aggregates after each event ----
        const bool own_b = act && ((ownm >> lane) & 1ull);       // controller post before #lane
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
        const bool strm_own = act && !opt && tj == a.ctrl_idx;   // controlled stream's arrival
        const bool has_o = own_b && a.n_fol > 0;
        const bool has_w = act && e1 > e0;
        int64_t osum = 0, wsum = 0;
        int oval = 0, wval = 0;
        int ocnt[NK], wcnt[NK];
#pragma unroll
        for (int kq = 0; kq < NK; ++kq) ocnt[kq] = wcnt[kq] = 0;
        if (a.dbg == 1) {
            // profiling only: skip phase C
        } else if (BITS) {
            // segments of the tile start at its own events (posts / own-stream arrivals)
            const bool rst = own_b || strm_own;
            const uint64_t rm = __ballot(rst);
            const bool hasr = mbcnt64_incl(rm) != 0;   // own event at or before #lane
            const bool wl = act && !strm_own;                        // a wall event
            const int deg = wl ? e1 - e0 : 0;
            const int odv = wl ? od : 0;
            SegFlags sf;
            sf.init(rst);
            // sumR / sumF: wall adds deg / odf, an own event drops sumF from sumR
            const int pdeg = (int)wave_scan_add((uint32_t)deg);
            const int64_t sfq = (int64_t)(int)sf.scan_add((uint32_t)odv) + (hasr ? 0 : agb.sumF);
            int64_t dec = 0;
            for (uint64_t b = rm; b; b &= b - 1) {
                const int r = __ffsll((unsigned long long)b) - 1;
                const int64_t D = r == 0 ? agb.sumF : bcast_i64(sfq, r - 1);
                if (lane >= r) dec += D;
            }
            wsum = agb.sumR + pdeg - dec;
            osum = agb.sumR + (pdeg - deg) - dec;
            // sink bitsets, one word at a time, every event of the tile at once; F and T
            // words come from LDS broadcasts, the mask row of a non-wall lane is the zero
            // row n_str, and the tile's last lane stores the new T word
            const bool vfull = agb.nvalid == a.n_sinks;
            const int last = n - 1;
            const uint32_t* mr = msk + (wl ? tj : a.n_str) * ms;
            const bool wlast = lane == last;
            int cw = 0, vw = 0, vo = 0;
            uint32_t nV = agb.V;
            if (vfull) {
                // two words per trip (ft holds an even number of words, the pad word's F
                // and T are zero), their DPP chains interleaved
                for (int ww = 0; ww < a.nw; ww += 2) {
                    const uint2 f0 = ft[ww], f1 = ft[ww + 1];
                    const uint32_t u0 = sf.scan_or_z(mr[ww]);          // wall union since the segment start
                    const uint32_t u1 = sf.scan_or_z(mr[ww + 1]);
                    const uint32_t t0 = (hasr ? f0.x : f0.y) & ~u0;    // top-1 set after #lane
                    const uint32_t t1 = (hasr ? f1.x : f1.y) & ~u1;
                    cw += __popc(t0) + __popc(t1);
                    if (wlast) {
                        ft[ww].y = t0;
                        ft[ww + 1].y = t1;
                    }
                }
            } else {
                for (int ww = 0; ww < a.nw; ++ww) {
                    const uint2 fw2 = ft[ww];
                    const uint32_t m = mr[ww];
                    const uint32_t u = sf.scan_or_z(m);
                    const uint32_t tq = (hasr ? fw2.x : fw2.y) & ~u;
                    cw += __popc(tq);
                    if (wlast) ft[ww].y = tq;
                    const uint32_t Vw = (uint32_t)__builtin_amdgcn_readlane((int)agb.V, ww);
                    const uint32_t x = wave_scan_or(m);
                    const uint32_t vq = Vw | x | (hasr ? fw2.x : 0u);  // valid set after #lane
                    vw += __popc(vq);
                    const uint32_t xe = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x138, 0xF, 0xF, false);
                    vo += __popc(Vw | xe | fw2.x);                     // after the post before #lane
                    nV = (uint32_t)wlane((int)nV, __builtin_amdgcn_readlane((int)vq, last), ww);
                }
            }
            wcnt[0] = cw;
            ocnt[0] = a.n_fol;   // a post puts every follower at rank 0
            wval = vfull ? a.n_sinks : vw;
            oval = vfull ? a.n_sinks : vo;
            if (n > 0) {
                if (!vfull) {
                    agb.V = nV;
                    agb.nvalid = bcast_i(vw, last);
                }
                agb.sumR = bcast_i64(wsum, last);
                agb.sumF = bcast_i64(sfq, last);
            }
        } else {
            for (int q = 0; q < n; ++q) {
                if ((ownm >> q) & 1ull) {
                    ag.own(rank, folat, a.n_fol, lane);
                    if (lane == q) {
                        osum = ag.sumR;
                        oval = ag.nvalid;
#pragma unroll
                        for (int kq = 0; kq < NK; ++kq) ocnt[kq] = ag.cnt[kq];
                    }
                }
                const int jw = bcast_i(tj, q);
                if (!opt && jw == a.ctrl_idx)
                    ag.own(rank, folat, a.n_fol, lane);
                else
                    ag.wall(rank, colat, bcast_i(e0, q), bcast_i(e1, q), bcast_i(od, q), lane);
                if (lane == q) {
                    wsum = ag.sumR;
                    wval = ag.nvalid;
#pragma unroll
                    for (int kq = 0; kq < NK; ++kq) wcnt[kq] = ag.cnt[kq];
                }
            }
        }
        RQ_CLK(4);   // C aggregates
        const uint64_t mo = __ballot(has_o), ma = mo | __ballot(has_w);
        n_events += n + __popcll(ownm);
        posts += __popcll(mo) + __popcll(__ballot(has_w && strm_own));
        world += __popcll(__ballot(has_w && !strm_own));
        if (ma && place_rows<NK, DEFER>(rs, ma, has_o, has_w, ot, tt, osum, oval, ocnt, wsum, wval, wcnt, status))
            stop = true;
        RQ_CLK(5);   // rows
        if (stop || fin) break;
    }
    if constexpr (DEFER) rs.flush_pend();
#ifdef RQ_PHASE_CLOCK
    if (lane == 0 && a.clk)
        for (int q = 0; q < 8; ++q) atomicAdd(&a.clk[q], ck[q]);
#endif
    if (BITS) agb.T = lane < a.nw ? ft[lane].y : 0u;   // the top-1 set back in its lane words
    // the controller's last post after the final arrival (or the tile max_events cut)
    if (!stop && opt && opt_next <= a.end && (a.max_events < 0 || n_events < a.max_events)) {
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
    if (BITS) {
        agb.sync();
        ag.nvalid = agb.nvalid;
    }
    if (lane == 0) {
        int64_t* cnto = a.counts + o * 4;
        cnto[0] = posts;
        cnto[1] = world;
        cnto[2] = n_events;
        cnto[3] = rs.nrow;
        a.sall[rl] = ag.nvalid;
        if (rs.nrow == 0) status |= RQ_ST_EMPTY;
        if (status) atomicOr(&a.status[o], status);
    }
    if (!a.wq) break;
    int nx = 0;
    if (lane == 0) nx = atomicAdd(a.wq, 1);
    qi = nslot + __builtin_amdgcn_readfirstlane(nx);
    }   // replica loop
}

template <int NK, class COL, int W, int H, bool BITS, bool PW = false, bool MRG = false>
__global__ __launch_bounds__(1024) void rq_sweep_fw(SweepArgs a)
{
    sweep_fw_body<NK, COL, W, H, BITS, PW, MRG>(a);
}
// the merged-stream instances: no generator state, so a tighter VGPR budget buys waves
// (RQ_FWM_WPE waves per SIMD; the planner picks the block size that fills them)
#ifndef RQ_FWM_WPE
#define RQ_FWM_WPE 4
#endif
template <int NK, class COL, bool BITS>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(RQ_FWM_WPE))) void rq_sweep_fwm(SweepArgs a)
{
    sweep_fw_body<NK, COL, 16, 8, BITS, false, true>(a);
}

// ============================================================================
// launch wrappers
// ============================================================================
// fused windowed sweep: (W, H) in {(16, 8), (8, 4)}; OptPWSignificance (PW) instances
// exist for uint16 columns and W = 16 only (make_plan keeps other PW runs off this path)
template <int NK, class COL, int W, bool BITS, bool PW = false, bool MRG = false>
static int occ_fw_t(int wpb, size_t lds);
template <int NK, class COL, int W, bool BITS, bool PW = false, bool MRG = false>
static hipError_t launch_fw_t(const SweepArgs& a, hipStream_t s)
{
    unsigned blocks = (unsigned)((a.n_chunk + a.wpb - 1) / a.wpb);
    if (a.wq) {
        // persistent grid: every resident wave slot once, the rest from the queue
        const int nb = occ_fw_t<NK, COL, W, BITS, PW, MRG>(a.wpb, a.lds_total);
        const unsigned cap = (unsigned)(nb > 0 ? nb : 1) * (unsigned)rq_cu_count();
        if (cap < blocks) blocks = cap;
    }
    if constexpr (MRG)
        hipLaunchKernelGGL((rq_sweep_fwm<NK, COL, BITS>), dim3(blocks), dim3(64 * a.wpb), a.lds_total, s, a);
    else
        hipLaunchKernelGGL((rq_sweep_fw<NK, COL, W, (W > 16 ? 8 : W / 2), BITS, PW, MRG>), dim3(blocks), dim3(64 * a.wpb),
                           a.lds_total, s, a);
    return hipGetLastError();
}
template <class COL, int W, bool PW = false, bool MRG = false>
static hipError_t launch_fw_k(const SweepArgs& a, int nK, hipStream_t s)
{
    switch (nK) {
    case 1: return launch_fw_t<1, COL, W, false, PW, MRG>(a, s);
    case 2: return launch_fw_t<2, COL, W, false, PW, MRG>(a, s);
    case 3: return launch_fw_t<3, COL, W, false, PW, MRG>(a, s);
    default: return launch_fw_t<4, COL, W, false, PW, MRG>(a, s);
    }
}
hipError_t rq_launch_sweep_fw(const SweepArgs& a, int nK, int col16, int W, int bits, hipStream_t s)
{
    if (a.n_chunk <= 0) return hipSuccess;
    if (W == 0) {   // merged streams (RedQueen / Poisson / replayed controllers)
        if (a.pw_c) return hipErrorInvalidValue;
        if (bits) return launch_fw_t<1, uint16_t, 16, true, false, true>(a, s);
        return col16 ? launch_fw_k<uint16_t, 16, false, true>(a, nK, s) : launch_fw_k<int, 16, false, true>(a, nK, s);
    }
    if (a.pw_c) {
        if (!col16 || W != 16) return hipErrorInvalidValue;
        return bits ? launch_fw_t<1, uint16_t, 16, true, true>(a, s) : launch_fw_k<uint16_t, 16, true>(a, nK, s);
    }
    if (bits)
        return W == 32 ? launch_fw_t<1, uint16_t, 32, true>(a, s)
             : W == 16 ? launch_fw_t<1, uint16_t, 16, true>(a, s) : launch_fw_t<1, uint16_t, 8, true>(a, s);
    if (W == 16) return col16 ? launch_fw_k<uint16_t, 16>(a, nK, s) : launch_fw_k<int, 16>(a, nK, s);
    return col16 ? launch_fw_k<uint16_t, 8>(a, nK, s) : launch_fw_k<int, 8>(a, nK, s);
}
template <int NK, class COL, int W, bool BITS, bool PW, bool MRG>
static int occ_fw_t(int wpb, size_t lds)
{
    if constexpr (MRG) return rq_occupancy(rq_sweep_fwm<NK, COL, BITS>, 64 * wpb, lds);
    else return rq_occupancy(rq_sweep_fw<NK, COL, W, (W > 16 ? 8 : W / 2), BITS, PW, MRG>, 64 * wpb, lds);
}
template <class COL, int W, bool PW = false, bool MRG = false>
static int occ_fw_k(int nK, int wpb, size_t lds)
{
    switch (nK) {
    case 1: return occ_fw_t<1, COL, W, false, PW, MRG>(wpb, lds);
    case 2: return occ_fw_t<2, COL, W, false, PW, MRG>(wpb, lds);
    case 3: return occ_fw_t<3, COL, W, false, PW, MRG>(wpb, lds);
    default: return occ_fw_t<4, COL, W, false, PW, MRG>(wpb, lds);
    }
}
// W = 0: the merged-stream instances
int rq_fw_blocks_per_cu(int nK, int col16, int W, int bits, int wpb, size_t lds, int pw)
{
    if (W == 0) {
        if (pw) return -1;
        if (bits) return occ_fw_t<1, uint16_t, 16, true, false, true>(wpb, lds);
        return col16 ? occ_fw_k<uint16_t, 16, false, true>(nK, wpb, lds) : occ_fw_k<int, 16, false, true>(nK, wpb, lds);
    }
    if (pw) {
        if (!col16 || W != 16) return -1;
        return bits ? occ_fw_t<1, uint16_t, 16, true, true>(wpb, lds) : occ_fw_k<uint16_t, 16, true>(nK, wpb, lds);
    }
    if (bits)
        return W == 32 ? occ_fw_t<1, uint16_t, 32, true>(wpb, lds)
             : W == 16 ? occ_fw_t<1, uint16_t, 16, true>(wpb, lds) : occ_fw_t<1, uint16_t, 8, true>(wpb, lds);
    if (W == 16) return col16 ? occ_fw_k<uint16_t, 16>(nK, wpb, lds) : occ_fw_k<int, 16>(nK, wpb, lds);
    return col16 ? occ_fw_k<uint16_t, 8>(nK, wpb, lds) : occ_fw_k<int, 8>(nK, wpb, lds);
}
