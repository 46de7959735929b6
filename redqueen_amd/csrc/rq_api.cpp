#include <cstdlib>
// rq_api.cpp -- host side of the C ABI declared in include/rq.h.
//
// rq_graph_build does what SimOpts + Manager.__init__ + Broadcaster.init_state
// do in the reference (opt_model.py:145-181, :340-344, :773-780): validate the
// network, give every sink a dense column (sorted sink id order, the
// pivot_table column order of utils.py:54-55), build the per-source sink lists
// in edge_list order (the Event.sink_ids of opt_model.py:306-307) as CSR, and
// upload everything once.  rq_run_batch only enqueues kernels.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <numeric>
#include <unordered_map>
#include <vector>

#include "../../include/rq.h"
#include "rq_internal.h"
#include "rq_tables.h"

namespace {

template <class T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    ~DevBuf() { if (p) (void)hipFree(p); }
    int upload(const std::vector<T>& v)
    {
        n = v.size();
        if (hipMalloc(&p, std::max<size_t>(1, n) * sizeof(T)) != hipSuccess) return RQ_ENOMEM;
        if (n && hipMemcpy(p, v.data(), n * sizeof(T), hipMemcpyHostToDevice) != hipSuccess)
            return RQ_EHIP;
        return RQ_OK;
    }
};

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Optional per-kernel timing (rq_timing): HIP events recorded on the launch
// stream around every kernel, summed by rq_timing_read.  Off by default.
enum { K_GEN = 0, K_SWEEP = 1, K_SCAN = 2, K_REPLAY = 3, K_MERGE = 4, K_N = 5 };
bool g_timing = false;
unsigned long long* g_clk = nullptr;   // RQ_PHASE_CLOCK builds: the sweep's / merge's phase clocks
#ifdef RQ_PHASE_CLOCK
unsigned long long* phase_clk()
{
    if (!g_clk && hipMalloc(&g_clk, 8 * sizeof(unsigned long long)) == hipSuccess)
        (void)hipMemset(g_clk, 0, 8 * sizeof(unsigned long long));
    return g_clk;
}
#endif

std::vector<std::pair<hipEvent_t, hipEvent_t>> g_ev[K_N];

struct TimedLaunch {
    int k;
    hipStream_t s;
    hipEvent_t a = nullptr, b = nullptr;
    TimedLaunch(int k_, hipStream_t s_) : k(k_), s(s_)
    {
        if (g_timing && hipEventCreate(&a) == hipSuccess && hipEventCreate(&b) == hipSuccess)
            (void)hipEventRecord(a, s);
    }
    ~TimedLaunch()
    {
        if (a && b) {
            (void)hipEventRecord(b, s);
            g_ev[k].push_back({a, b});
        }
    }
};

// Side streams of the pipelined chunk loop (rq_run_batch): per host thread AND per
// caller stream, created on first use on the caller's current device, with the fork /
// join events.  Work on them is always bracketed by a wait on the caller's stream (fork)
// and a wait of the caller's stream on them (join), so the call stays stream-ordered for
// the caller; batches issued on different caller streams get different side streams and
// so overlap (a caller alternating two streams overlaps one batch's tail with the next
// batch's generation and merge).
struct SidePipe {
    int dev = -1;
    hipStream_t caller = nullptr;
    uint64_t used = 0;   // last use (SidePipes' LRU clock)
    hipStream_t s[2] = {nullptr, nullptr};
    hipEvent_t fork = nullptr, join[2] = {nullptr, nullptr};
    // drop the streams and events (made on device `dev`) once their work is done
    void release()
    {
        if (dev < 0) return;
        int cur = -1;
        (void)hipGetDevice(&cur);
        if (cur != dev) (void)hipSetDevice(dev);
        for (int k = 0; k < 2; ++k) {
            if (s[k]) {
                (void)hipStreamSynchronize(s[k]);
                (void)hipStreamDestroy(s[k]);
            }
            if (join[k]) (void)hipEventDestroy(join[k]);
            s[k] = nullptr;
            join[k] = nullptr;
        }
        if (fork) (void)hipEventDestroy(fork);
        fork = nullptr;
        if (cur >= 0 && cur != dev) (void)hipSetDevice(cur);
        dev = -1;
    }
    int get(int n, hipStream_t* out)
    {
        int d = 0;
        if (hipGetDevice(&d) != hipSuccess) return RQ_EHIP;
        if (dev != d) {   // first use (or another device's pipe re-homed): fresh streams and events
            release();
            dev = d;
        }
        if (!fork && hipEventCreateWithFlags(&fork, hipEventDisableTiming) != hipSuccess) return RQ_EHIP;
        for (int k = 0; k < n && k < 2; ++k) {
            if (!s[k] && hipStreamCreateWithFlags(&s[k], hipStreamNonBlocking) != hipSuccess) return RQ_EHIP;
            if (!join[k] && hipEventCreateWithFlags(&join[k], hipEventDisableTiming) != hipSuccess) return RQ_EHIP;
            out[k] = s[k];
        }
        return RQ_OK;
    }
};
// a few (device, caller stream) pairs per thread (the engine's users run on one or two
// streams); the null stream has the same handle on every device, hence the device in the
// key.  Past kPipes the least recently used entry is re-homed: on the same device its
// streams and events are kept (only the owner changes), on another they are destroyed
// once idle and made afresh.
constexpr int kPipes = 4;
struct SidePipes {
    SidePipe p[kPipes];
    uint64_t clock = 0;
    SidePipe& of(hipStream_t caller)
    {
        int d = -1;
        (void)hipGetDevice(&d);
        SidePipe* lru = &p[0];
        for (SidePipe& x : p) {
            if (x.used && x.caller == caller && (x.dev == d || x.dev < 0)) {
                x.used = ++clock;
                return x;
            }
            if (x.used < lru->used) lru = &x;
        }
        if (lru->dev >= 0 && lru->dev != d) lru->release();
        lru->caller = caller;
        lru->used = ++clock;
        return *lru;
    }
    // no destructor: a thread's pipes live until the process ends (HIP may already be
    // torn down when thread_local destructors run at exit)
};
thread_local SidePipes t_pipes;

}  // namespace

namespace {
constexpr int kStages = 4;
struct Stage {
    void* buf = nullptr;
    size_t bytes = 0;
    hipEvent_t done = nullptr;
};
}  // namespace

struct rq_graph {
    // pinned staging ring for the per-run parameter tables
    std::mutex stage_mu;
    Stage stage[kStages];
    int stage_next = 0;
    ~rq_graph()
    {
        for (Stage& st : stage) {
            if (st.done) {
                (void)hipEventSynchronize(st.done);
                (void)hipEventDestroy(st.done);
            }
            if (st.buf) (void)hipHostFree(st.buf);
        }
    }
    int n_str = 0, ctrl_idx = -1, n_sinks = 0, n_fol = 0;
    int64_t n_edges = 0, ctrl_src_id = 0;
    double start = 0.0, end = 0.0;
    // per stream (dynamic sources by src_id, then static ones by src_id); the controlled
    // slot has kind RQ_SRC_NONE
    std::vector<int64_t> src_id;
    std::vector<int> kind, orig_idx, arr_off, arr_n;
    std::vector<int> is_static;   // 1: a static source (equal times play after the dynamic ones)
    std::vector<uint32_t> seed;
    std::vector<double> p0, p1, p2, arr_a, arr_b;
    std::vector<int> csr_ptr, csr_col, outdeg_f, fol;
    std::vector<int64_t> fol_ids;
    std::vector<int64_t> sink_ids;   // sorted: the sink column -> sink id map
    DevBuf<int64_t> d_sink_ids;
    std::vector<int> csr_col_el;     // sink columns in edge-list order for every stream
    DevBuf<int> d_csr_col_el;
    std::vector<int> col_to_fol;     // sink column -> follower position or -1
    // duplicate (source, sink) edges (a multigraph, opt_model.py:169-175 accepts them): the
    // sweep's CSR row of a source holds its distinct sinks first (layer 0), then the 2nd
    // occurrences (layer 1), ...; every layer has distinct sinks.  lay_end[lay_ptr[j] ..
    // lay_ptr[j+1]) are the CSR ends of stream j's layers.  multi: some row has > 1 layer.
    bool multi = false, ctrl_dup = false;
    // two of the graph's own RealData times are equal -- among the wall sources
    // (rd_ties), or with the controlled slot's replayed times too (rd_ties_ctrl, runs with
    // an RQ_SRC_REALDATA controller): every replica meets that tie, so such runs go to the
    // exact sequential sweep directly
    bool rd_ties = false, rd_ties_ctrl = false;
    std::vector<int> lay_ptr, lay_end;
    DevBuf<int> d_lay_ptr, d_lay_end;
    // per-stream sink bitsets (32 sinks per word) for the K=1 bitset sweep, n_sinks <= 2048
    int nw = 0;
    std::vector<uint32_t> masks;
    DevBuf<uint32_t> d_mask;
    std::vector<uint32_t> fbits;   // follower set as a sink bitset (BL sweep)
    DevBuf<uint32_t> d_fbits;
    // controlled-slot arrays (PiecewiseConst / RealData controlled runs)
    int ctrl_arr_off = 0, ctrl_arr_n = 0;
    DevBuf<int64_t> d_src_id;
    DevBuf<int> d_kind, d_orig, d_arr_off, d_arr_n, d_csr_ptr, d_csr_col, d_outdeg_f, d_fol, d_cbf;
    DevBuf<uint32_t> d_seed;
    DevBuf<double> d_p0, d_p1, d_p2, d_arr_a, d_arr_b;
};

namespace {

struct Plan {
    int nK = 1, spl = 1, wpb = 4, n_sinks_pad = 0;
    int64_t R = 0, chunk = 0, capsum = 0, cap_rows = 0;
    int64_t rep_lo = 0, rep_cnt = 0;   // per-grid-point replica window (rq_batch_desc.rep_lo/rep_cnt)
    std::vector<int> cap;
    std::vector<int64_t> st_off;
    std::vector<int> rd_k;   // stream -> per-replica RealData source k (rq_batch_desc.rd_*) or -1
    // sequential (event log / max_events) sweep variant; K=1 sink-bitset variant
    bool log = false, bits = false;
    // K=1 on per-wave LDS sink bits for graphs past the bitset variant (> 64 sources)
    bool bl = false;
    size_t g_fb = 0, g_etab = 0, g_inv = 0, g_skip = 0;
    bool g_inv_sh = false;   // general sweep: 1/c_j in the block's shared LDS (one grid point)
    bool gs = false;         // LOG sweep: per-sink state in global memory, gs_slots wave slots
    int64_t gs_slots = 0, gs_stride = 0;
    // fused windowed sweep (n_str <= 64): arrivals generated in-kernel, window depth fw_h
    bool fw = false;
    int fw_h = 8, mstride = 1;
    // general fast sweep on merged streams (rq_merge_streams; sweep_mode 6: the windowed
    // per-source merge inside the sweep instead)
    bool mrg = false;
    // the sequential sweep over > RQ_MAX_STREAMS sources: it plays the merged sequence
    // too (its own per-lane rings hold <= 32 sources per lane)
    bool lmrg = false;
    // merged streams with the per-stream tables (CSR starts, follower out-degrees, tie
    // flags, 1/c_j) in global memory: graphs whose tables do not fit LDS (the GT instances;
    // the sequential ones on merged streams always)
    bool gt = false;
    size_t off_mt = 0, off_mj = 0, off_mjh = 0, off_mlen = 0;
    int64_t mrg_stride = 0;   // merged entries per replica (capacity)
    int n_grp = 1;            // > RQ_MG_B sources: groups of the two-level merge
    int grp_sz = RQ_MG_B;     //   streams per group (64 up to 64 groups: MergeArgs.grp_sz)
    int64_t sub_stride = 0;   //   entries per (replica, group) of the first level
    size_t off_sub_t = 0, off_sub_j = 0, off_sub_len = 0;
    // the fused sweep's phases B / C on merged streams (rq_gen_streams + rq_merge_streams
    // instead of in-kernel generation; sweep_mode 7: the in-kernel generating sweep)
    bool fwm = false;
    // general sweep LDS layout
    int gwpb = 4, gwin = 16, gcol_lds = 1, gcol16 = 0;
    size_t g_col = 0, g_ptr = 0, g_odf = 0, g_cbf = 0, g_wave = 0, g_wave_stride = 0, g_rank_off = 0,
           g_win_off = 0, g_x_off = 0, g_total = 0, g_stage_off = 0;
    size_t tables_bytes = 0;
    // resident sweep waves per CU of the chosen instance (the persistent grid's slots)
    int wpc = 0;
    // pipelined chunks (merged-stream sweeps): nbuf buffer sets, chunk k on stream k % nbuf
    // with set k % nbuf, so chunk k+1's generation / merge and chunk k-1's scan fill the
    // wave slots chunk k's sweep tail leaves (rq_run_batch); off_set0 + set * set_stride
    // is a set's base, the per-chunk offsets below are relative to it
    int nbuf = 1;
    bool order = false;   // longest-first replica order for the sweep (rq_order_replicas)
    size_t off_set0 = 0, set_stride = 0, off_ord = 0;
    size_t off_pwc = 0, off_pwmax = 0;
    size_t off_invc = 0, off_streams = 0, off_slen = 0, off_rt = 0, off_rs = 0, off_rv = 0,
           off_rc = 0, off_sall = 0, off_wq = 0, off_stoff = 0, off_cap = 0, off_rdk = 0, off_repidx = 0, off_gs = 0,
           total = 0;
};

constexpr size_t kLdsMax = 160 * 1024;
constexpr int kBitsMaxSinks = 2048;   // bitset sweep: one 32-sink word per lane

double stream_mean_var(const rq_graph* g, int j, int kind, const rq_batch_desc* b, double* var)
{
    const double span = g->end - g->start;
    double m = 0.0;
    *var = 0.0;
    switch (kind) {
    case RQ_SRC_POISSON:
    case RQ_SRC_POISSON2: {
        const double rate = j == g->ctrl_idx ? b->ctrl_rate_max : g->p0[j];
        m = std::max(0.0, rate) * span;
        *var = m;
        break;
    }
    case RQ_SRC_HAWKES: {
        const double l0 = g->p0[j], al = g->p1[j], be = g->p2[j];
        const double br = be > 0.0 ? al / be : 1.0;
        if (br < 0.95) {
            m = l0 * span / (1.0 - br);
            *var = l0 * span / ((1.0 - br) * (1.0 - br) * (1.0 - br));
        } else {
            m = l0 * span * 40.0 + 1000.0;
            *var = m * m;
        }
        break;
    }
    case RQ_SRC_PWCONST: {
        const int off = g->arr_off[j], n = g->arr_n[j];
        for (int k = 0; k < n; ++k) {
            const double lo = std::max(g->arr_a[off + k], g->start);
            const double hi = std::min(k + 1 < n ? g->arr_a[off + k + 1] : g->end, g->end);
            if (hi > lo) m += std::max(0.0, g->arr_b[off + k]) * (hi - lo);
        }
        *var = m;
        break;
    }
    case RQ_SRC_REALDATA:
        m = g->arr_n[j];
        *var = 0.0;
        break;
    default:
        break;
    }
    return m;
}

// the buffer layout of one chunk plan (p->chunk, p->nbuf): offsets and p->total
void plan_layout(const rq_graph* g, const rq_batch_desc* b, Plan* p);

// device-memory budget of a plan's workspace: the caller's (rq_batch_desc.ws_budget),
// else `fallback` (rq_run_batch: the workspace it was handed) or, with none, 0.9 x the
// device's free memory; RQ_WS_BUDGET_GB caps it
double ws_budget(const rq_batch_desc* b, double fallback)
{
    double bud = b && b->ws_budget > 0 ? (double)b->ws_budget : fallback;
    if (!(bud > 0.0)) {
        size_t fr = 0, tot = 0;
        bud = hipMemGetInfo(&fr, &tot) == hipSuccess ? 0.9 * (double)fr : 200.0 * (1 << 30);
    }
    if (const char* e = getenv("RQ_WS_BUDGET_GB")) bud = std::min(bud, atof(e) * (1 << 30));
    return bud;
}

int make_plan(const rq_graph* g, const rq_batch_desc* b, Plan* p, double budget)
{
    if (!g || !b) return RQ_EINVAL;
    if (b->nK < 1 || b->nK > RQ_MAX_K || !b->Ks) return RQ_EINVAL;
    if (b->n_grid < 1 || b->n_rep < 1) return RQ_EINVAL;
    const int ck = b->ctrl_kind;
    if (ck != RQ_SRC_OPT && ck != RQ_SRC_OPTPW && ck != RQ_SRC_POISSON2 && ck != RQ_SRC_PWCONST &&
        ck != RQ_SRC_REALDATA && ck != RQ_SRC_NONE)
        return RQ_EINVAL;
    if (ck == RQ_SRC_OPT && (!b->q || (g->n_fol > 0 && !b->s))) return RQ_EINVAL;
    if (ck == RQ_SRC_OPTPW &&
        (!b->q || b->n_seg < 1 || b->n_seg > 4096 || !(b->period > 0.0) || (g->n_fol > 0 && !b->s_pw)))
        return RQ_EINVAL;
    if (ck == RQ_SRC_POISSON2 && !b->ctrl_rate) return RQ_EINVAL;
    if ((ck == RQ_SRC_PWCONST) && g->ctrl_arr_n < 1) return RQ_EINVAL;
    const double scale = b->cap_scale >= 1.0 ? b->cap_scale : 1.0;
    p->nK = b->nK;
    // the call's replica space: the [rep_lo, rep_lo + rep_cnt) window of every grid point
    if (b->rep_cnt < 0 || (b->rep_cnt > 0 && (b->rep_lo < 0 || b->rep_lo + b->rep_cnt > b->n_rep)))
        return RQ_EINVAL;
    p->rep_lo = b->rep_cnt > 0 ? b->rep_lo : 0;
    p->rep_cnt = b->rep_cnt > 0 ? b->rep_cnt : b->n_rep;
    const int64_t Rall = (int64_t)b->n_grid * p->rep_cnt;
    if (b->replica0 < 0 || b->n_local < 0 || b->replica0 + b->n_local > Rall) return RQ_EINVAL;
    p->R = b->n_local > 0 ? b->n_local : Rall - b->replica0;
    if (p->R < 1) return RQ_EINVAL;
    // a replica list (ABI v6): n_local global ids of the whole n_grid x n_rep grid
    if (b->rep_idx) {
        if (b->replica0 != 0 || b->rep_cnt != 0 || b->n_local < 1) return RQ_EINVAL;
        const int64_t nall = (int64_t)b->n_grid * b->n_rep;
        for (int64_t k = 0; k < b->n_local; ++k)
            if (b->rep_idx[k] < 0 || b->rep_idx[k] >= nall) return RQ_EINVAL;
    }
    p->chunk = b->chunk > 0 ? std::min<int64_t>(b->chunk, p->R) : std::min<int64_t>(p->R, 16384);
    p->cap.assign(g->n_str, 0);
    p->st_off.assign(g->n_str, 0);
    p->rd_k.assign(g->n_str, -1);
    if (b->n_rd < 0 || b->n_rd > RQ_MAX_RD) return RQ_EINVAL;
    if (b->n_rd > 0) {
        if (!b->rd_src_id || !b->rd_cap || !b->rd_times || !b->rd_off) return RQ_EINVAL;
        for (int k = 0; k < b->n_rd; ++k) {
            int jk = -1;
            for (int j = 0; j < g->n_str; ++j)
                if (g->src_id[j] == b->rd_src_id[k]) jk = j;
            // a RealData wall source of the graph, named once
            if (jk < 0 || jk == g->ctrl_idx || g->kind[jk] != RQ_SRC_REALDATA || p->rd_k[jk] >= 0 ||
                b->rd_cap[k] < 0 || b->rd_cap[k] > ((int64_t)1 << 30))
                return RQ_EINVAL;
            p->rd_k[jk] = k;
        }
    }
    double wall_caps = 0.0, wall_mean = 0.0, wall_var = 0.0;
    int64_t ctrl_cap = 0;
    for (int j = 0; j < g->n_str; ++j) {
        int kind = g->kind[j];
        if (j == g->ctrl_idx)
            kind = (ck == RQ_SRC_OPT || ck == RQ_SRC_OPTPW || ck == RQ_SRC_NONE) ? RQ_SRC_NONE : ck;
        double var;
        const double m = stream_mean_var(g, j, kind, b, &var);
        int64_t c = 0;
        if (kind != RQ_SRC_NONE)
            c = kind == RQ_SRC_REALDATA ? (p->rd_k[j] >= 0 ? b->rd_cap[p->rd_k[j]] : (int64_t)m)
                                        : (int64_t)std::ceil((m + 8.0 * std::sqrt(var) + 32.0) * scale);
        if (c > (int64_t)1 << 30) return RQ_EINVAL;
        c = (c + 15) & ~(int64_t)15;   // whole 128-byte lines: the merge's loads, the generator's stores
        p->cap[j] = (int)c;
        p->st_off[j] = p->capsum;
        p->capsum += c;
        if (j == g->ctrl_idx) {
            ctrl_cap = c;
        } else {
            wall_caps += (double)c;
            if (kind != RQ_SRC_NONE) {
                wall_mean += kind == RQ_SRC_REALDATA ? (double)c : m;
                wall_var += var;
            }
        }
    }
    // the wall events of a replica together: mean + 8 sigma of their SUM (the streams'
    // own 8-sigma capacities add up to far more: C5 769k against 511k); a replica past it
    // is flagged (RQ_ST_STREAM_OVERFLOW / RQ_ST_ROWS_OVERFLOW) and Graph.run(check=True)
    // reruns the batch with doubled capacities
    double squeeze = 1.0;   // tests only: undersized capacities exercise the overflow reruns
    if (const char* e = getenv("RQ_CAP_SQUEEZE")) squeeze = std::max(0.01, std::min(1.0, atof(e)));
    const double walls_agg = std::ceil((wall_mean + 8.0 * std::sqrt(wall_var) + 32.0) * scale * squeeze);
    const bool opt_ctrl = ck == RQ_SRC_OPT || ck == RQ_SRC_OPTPW;
    // merged sequence per replica: every arrival of every stream (the controlled one too)
    p->mrg_stride = std::min<int64_t>(p->capsum, ((int64_t)walls_agg + ctrl_cap + 64 + 15) & ~(int64_t)15);
    // pivot rows <= events: walls + posts; RedQueen posts at most once per wall event (+1),
    // so the old bound was 2 x the walls; posts are sized max(4096, walls / 4) now (C3: ~180
    // per replica, C5: ~1400; the C4 grid's q = 1e-4 corner: 1816 on 2075 walls)
    double rows = wall_caps + (opt_ctrl ? wall_caps + 1.0 : (double)ctrl_cap) + 8.0;
    rows = std::min(rows, walls_agg + (opt_ctrl ? std::max(4096.0, std::ceil(walls_agg / 4.0)) + 1.0
                                                : (double)ctrl_cap) + 8.0);
    if (b->max_events >= 0) rows = std::min(rows, (double)b->max_events + 1.0);
    // a multiple of 32 rows: replica row bases stay aligned to the scan's 32-row trips
    p->cap_rows = (std::max<int64_t>(64, (int64_t)rows) + 31) & ~(int64_t)31;
    // Opt / OptPWSignificance with a duplicated controlled edge: the reference's follower
    // vectors (sqrt_s_by_q, old_ranks: one entry per edge) no longer match the ranks (one
    // per distinct follower) and its first non-own event raises ValueError
    if (g->ctrl_dup && (ck == RQ_SRC_OPT || ck == RQ_SRC_OPTPW)) return RQ_EINVAL;
    if (g->n_str > RQ_MAX_STREAMS_MRG) return RQ_EUNSUPPORTED;
    p->spl = g->n_str <= 64 ? 1 : g->n_str <= 128 ? 2 : g->n_str <= 256 ? 4 : 8;
    p->n_sinks_pad = (g->n_sinks + 1) | 1;   // odd stride: spreads replicas over LDS banks
    const size_t per_wave = (size_t)p->n_sinks_pad * 4;
    p->wpb = per_wave * 4 <= 64 * 1024 ? 4 : per_wave * 2 <= 80 * 1024 ? 2 : 1;

    // the sequential exact variant when equal event times are certain: the graph's own
    // RealData times (every replica plays them) repeat a time; otherwise RealData and
    // the per-replica plugin streams play on the fast sweeps, which flag RQ_ST_TIE on any
    // equal-time pair, and the caller reruns the flagged replicas on the exact sequential
    // sweep (rq_batch_desc.rep_idx).  max_events cuts the fast sweeps' tiles
    // (truncate_tile); the fast sweeps write the event log themselves.
    const bool rd_ties = ck == RQ_SRC_REALDATA ? g->rd_ties_ctrl : g->rd_ties;
    p->log = b->sweep_mode == 2 || (rd_ties && b->sweep_mode != 1 && b->sweep_mode != 5);
    for (int q = 0; q < b->nK; ++q) p->log = p->log || b->Ks[q] > 32767;   // int16 ranks
    // a multigraph (duplicate edges make fractional pivot cells, the exact sequential
    // sweep's business); > 512 sources: the fast general sweep plays the two-level merged
    // sequence (rq_merge_streams per group of 512, then over the groups), the windowed
    // sweep (mode 6) owns <= 8 sources per lane
    p->log = p->log || g->multi || (g->n_str > 512 && b->sweep_mode == 6);
    const int nwl = (g->n_sinks + 31) / 32;

  replan:
    // the sequential sweep owns <= 32 sources per lane; past that it plays the merged
    // (t, stream) sequence of rq_merge_streams like the fast general sweep
    p->lmrg = p->log && g->n_str > RQ_MAX_STREAMS;
    if (p->log) p->spl = g->n_str <= 64 ? 1 : g->n_str <= 512 ? 8 : g->n_str <= 1024 ? 16 : 32;
    p->mstride = g->nw | 1;   // odd row stride: one LDS bank per stream for a given word
    p->bits = !p->log && p->nK == 1 && b->Ks[0] == 1 && g->nw > 0 && b->sweep_mode != 3 &&
              (size_t)g->n_str * p->mstride * 4 <= 64 * 1024;
    if (p->bits) p->spl = g->n_str <= 64 ? 1 : g->n_str <= 128 ? 2 : g->n_str <= 256 ? 4 : 8;
    p->bl = !p->log && !p->bits && p->nK == 1 && b->Ks[0] == 1 && p->spl >= 2 && b->sweep_mode != 3;
    // K = 1 with too many sinks for int16 ranks in LDS (> 24k): per-wave sink BITS, which
    // exist for 2+ sources per lane (lanes past the sources idle)
    if (!p->log && !p->bits && !p->bl && p->nK == 1 && b->Ks[0] == 1 && b->sweep_mode != 3 &&
        2 * (size_t)p->n_sinks_pad > 48 * 1024) {
        p->spl = std::max(p->spl, 2);
        p->bl = true;
    }
    p->gs = false;
    // the fast general sweep plays the merged (t, stream) sequence: the merge kernel reads
    // every stream line once (one source per thread, <= RQ_MG_B sources)
    p->mrg = (!p->log && b->sweep_mode != 6) || p->lmrg;
    // > RQ_MG_B sources: two levels; groups of 64 streams (one-wave first-level blocks) while
    // <= 64 of them cover the graph, so the second level walks up to 64 sequences a round
    // instead of 2-8 (600 sources: 2 groups of <= 512 -> 10 of <= 64)
    p->grp_sz = g->n_str <= 64 * 64 ? 64 : RQ_MG_B;
    if (const char* e = getenv("RQ_MG_GRP"))   // A/B only
        p->grp_sz = atoi(e) == 64 && g->n_str <= 64 * 64 ? 64 : RQ_MG_B;
    p->n_grp = g->n_str > RQ_MG_B ? (g->n_str + p->grp_sz - 1) / p->grp_sz : 1;
    if (const char* e = getenv("RQ_MRG")) p->mrg = p->lmrg || (p->mrg && atoi(e) != 0);   // A/B only
    // without the merged streams the windowed sweep owns <= 8 sources per lane
    if (!p->mrg && !p->log && g->n_str > 512) {
        p->log = true;
        goto replan;
    }

    // general sweep: pick (ring depth W, waves per block) for the most waves per CU
    {
        int best = -1;
        // sink columns live in LDS as uint16 when they fit, else they are read from
        // global memory as int (the kernel's COL type selects the path at compile time)
        // both placements are scored: LDS columns only win at equal waves per CU
        // LOG: the per-sink state in LDS, or (gs) in global memory for more sinks than fit
        // GT (merged streams only): the per-stream tables in global memory -- tried when no
        // layout with them in LDS fits, always for the sequential sweep on merged streams
        for (int gt = p->lmrg ? 1 : 0; gt <= (p->mrg ? 1 : 0) && best < 0; ++gt)
        for (int gs = 0; gs <= (p->log ? 1 : 0); ++gs)
        for (int col_lds = g->n_sinks <= 65535 && !(p->log && p->spl >= 16) && !gt ? 1 : 0; col_lds >= 0; --col_lds) {
            if (gt && p->bits) continue;   // the sink-bitset instances keep their tables in LDS
            if (const char* e = getenv("RQ_G_COLLDS"))   // tuning only: force the column placement
                if (atoi(e) != col_lds) continue;
            const int c16 = col_lds;
            // BITS: sink bitsets [n_str][nw] replace the columns (and the per-wave ranks)
            const size_t colb = p->bits ? 4 * (size_t)g->n_str * p->mstride
                                        : (col_lds ? 2 * g->csr_col.size() : 0);
            size_t sh = 0;
            const size_t o_col = sh;  sh = align_up(sh + colb, 16);
            const size_t tabn = gt ? 0 : (size_t)g->n_str;
            const size_t o_ptr = sh;  sh = align_up(sh + 4 * (tabn + (gt ? 0 : 1)), 16);
            const size_t o_odf = sh;  sh = align_up(sh + 4 * tabn, 16);
            const size_t o_cbf = sh;  sh = align_up(sh + 4 * tabn, 16);
            const size_t o_fb = sh;   if (p->bl) sh = align_up(sh + 4 * (size_t)nwl, 16);
            // one grid point: the 1/c_j table once per block instead of once per wave
            const bool inv_sh = b->n_grid == 1 && !gt;
            const size_t o_inv = sh;  if (inv_sh) sh = align_up(sh + 8 * (size_t)g->n_str, 16);
            const int spl = p->spl;
            int only_w = 0;
            if (const char* e = getenv("RQ_G_W")) only_w = atoi(e);   // tuning only
            // LOG: LDS rings of W = 8 per source (4 at 32 sources per lane); the fast sweep:
            // a register window of 4
            for (int W : {8, 4}) {
                if ((p->log ? (spl >= 32 ? 4 : 8) : 4) != W) continue;
                if (only_w && W != only_w) continue;
                const size_t r_off = inv_sh || gt ? 0 : align_up(8 * (size_t)g->n_str, 16);
                const size_t rank_b = p->log ? (gs ? 0 : 4) : (p->bits ? 0 : 2);   // fast: int16 saturating
            const int spl_i = p->mrg ? (gt ? -1 : 0) : spl;   // the instance: 0 = merged streams, -1 with GT
                // BL: two bits per sink (T, V words) in place of the int16 ranks
                const size_t w_off = p->bl ? align_up(r_off + 8 * (size_t)nwl, 16)
                                           : align_up(r_off + rank_b * (size_t)p->n_sinks_pad, 16);
                // LOG: rings of W arrivals for each real source; fast: the tile's staging
                size_t stride = p->log && !p->lmrg ? align_up(w_off + 8 * (size_t)g->n_str * W, 16)
                                                   : align_up(w_off + 64 * 12, 16);
                // LOG: per-sink gtag/gcnt/gsum (gs: in global memory) + a wave_npsum<1>
                // scratch (RQ_NPSUM1_LDS doubles)
                const size_t x_off = stride;
                if (p->log) stride = align_up(x_off + (gs ? 0 : 12 * (size_t)p->n_sinks_pad) + 8 * (size_t)RQ_NPSUM1_LDS, 16);
                for (int wpb : {16, 12, 10, 8, 6, 5, 4, 3, 2, 1}) {
                    if (p->log && wpb > 4) continue;   // LOG instances: 256-thread blocks
                    if (!p->log && !p->mrg && spl >= 4 && wpb > 8) continue;   // 512-thread instances
                    if (p->mrg && 64 * wpb > RQ_MRG_LB) continue;
                    const size_t tot = sh + wpb * stride;
                    if (tot > kLdsMax) continue;
                    // resident waves per CU: the runtime's occupancy for this instance
                    // (VGPR/SGPR/LDS); without a device, the LDS bound capped at 16
                    int blocks = rq_sweep_blocks_per_cu(spl_i, p->nK, c16, W, p->log ? 1 + gs : 0,
                                                        p->bl ? 2 : p->bits, wpb, tot);
                    if (blocks <= 0) blocks = (int)std::min<size_t>(kLdsMax / tot, 16 / wpb);
                    const int waves = blocks * wpb;
                    // LDS columns skip the global latency; LDS sink state wherever it fits
                    const int score = waves * 8 + col_lds * 2 + (gs ? 0 : 100000);
                    if (score > best) {
                        best = score;
                        p->wpc = waves;
                        p->gs = gs;
                        p->gs_slots = std::min<int64_t>((int64_t)align_up((size_t)p->chunk, (size_t)wpb),
                                                        (int64_t)blocks * wpb * rq_cu_count());
                        p->gwin = W; p->gwpb = wpb; p->gcol_lds = col_lds; p->gcol16 = c16;
                        p->g_col = o_col; p->g_ptr = o_ptr; p->g_odf = o_odf; p->g_cbf = o_cbf;
                        p->g_wave = sh; p->g_wave_stride = stride; p->g_rank_off = r_off;
                        p->g_win_off = w_off; p->g_x_off = x_off; p->g_total = tot; p->g_fb = o_fb;
                        p->g_inv = o_inv; p->g_inv_sh = inv_sh; p->gt = gt;
                    }
                }
            }
        }
        if (best < 0) {
            if (p->log) return RQ_EUNSUPPORTED;
            p->log = true;   // no fast instance fits this graph: the exact sequential sweep
            goto replan;
        }
        // stream ids past 16 bits are read (mrg_jh) by the GT instances only; such graphs'
        // tables never fit LDS, so they always get one
        if (p->mrg && g->n_str > 65535 && !p->gt) return RQ_EUNSUPPORTED;
        // BL on merged streams: a per-wave stamp (the reset epoch a stream last played in)
        // and first-lane table per stream let a tile skip the events whose stream already
        // played since the last post -- their sinks are out of the top-1 set and valid.
        // Only where it costs no resident waves.
        p->g_skip = 0;
        if (p->bl && p->mrg && !p->gs) {
            const size_t st2 = align_up(p->g_wave_stride + 8 * (size_t)g->n_str, 16);
            const size_t tot2 = p->g_wave + p->gwpb * st2;
            int blocks = tot2 <= kLdsMax ? rq_sweep_blocks_per_cu(p->gt ? -1 : 0, p->nK, p->gcol16, p->gwin, 0, 2, p->gwpb, tot2) : 0;
            if (tot2 <= kLdsMax && blocks <= 0) blocks = (int)std::min<size_t>(kLdsMax / tot2, 16 / p->gwpb);
            bool on = blocks * p->gwpb >= p->wpc;
            if (const char* e = getenv("RQ_SKIP")) on = on && atoi(e) != 0;   // A/B only
            if (on) {
                p->g_skip = p->g_wave_stride;
                p->g_wave_stride = st2;
                p->g_total = tot2;
            }
        }
    }

    // fused windowed sweep: one stream per lane, rings of W arrivals generated in LDS,
    // a window of H per ring in registers; (W, H, waves per block) for the most waves per CU
    const bool pw = b->ctrl_kind == RQ_SRC_OPTPW;
    p->fw = !p->log && !p->bl && g->n_str <= 64 && b->sweep_mode != 4 && b->sweep_mode != 5 &&
            b->sweep_mode != 6;
    p->fwm = p->fw && !pw && b->sweep_mode != 7;
    if (const char* e = getenv("RQ_FWM")) p->fwm = p->fwm && atoi(e) != 0;   // A/B only
    if (p->fw) {
        int best = -1;
        const int c16 = p->bits ? 1 : (g->n_sinks <= 65535 ? 1 : 0);
        if (pw && !c16) p->fw = false;   // OptPWSignificance fused instances: uint16 columns
        // BITS: sink bitsets [n_str + 1][mstride] (row n_str all zero: the mask of a
        // lane without a wall event) replace the columns
        const size_t colb = p->bits ? 4 * (size_t)(g->n_str + 1) * p->mstride
                                    : (c16 ? 2 * g->csr_col.size() : 0);
        size_t sh = 0;
        const size_t o_col = sh;  sh = align_up(sh + colb, 16);
        const size_t o_ptr = sh;  sh = align_up(sh + 4 * (g->n_str + 1), 16);
        const size_t o_odf = sh;  sh = align_up(sh + 4 * g->n_str, 16);
        const size_t o_cbf = sh;  sh = align_up(sh + 4 * g->n_str, 16);
        const size_t o_etab = sh; sh = align_up(sh + RQ_EXP_TAB_N * 8, 16);   // rq_exp's table
        int only_w = 0;
        if (const char* e = getenv("RQ_FW_W")) only_w = atoi(e);   // tuning only
        for (int W : {32, 16, 8}) {
            if (!p->fw) break;
            if (only_w && W != only_w) continue;
            if (pw && W != 16) continue;
            if (W == 32 && !p->bits) continue;   // 32-deep rings: K = 1 bitset instance only
            const int H = W > 16 ? 8 : W / 2;    // register window
            const size_t r_off = align_up(8 * (size_t)g->n_str, 16);
            // per wave: BITS -> (F, T) word pairs [nw]; else int16 sink ranks
            const size_t w_off = align_up(r_off + (p->bits ? 8 * (size_t)((g->nw + 1) & ~1) : 2 * (size_t)p->n_sinks_pad), 16);
            // merged streams: no arrival rings
            const size_t s_off = align_up(w_off + (p->fwm ? 0 : 8 * (size_t)g->n_str * (W + 1)), 16);
            const size_t stride = align_up(s_off + 64 * 12, 16);
            for (int wpb : {16, 12, 10, 8, 6, 5, 4, 3, 2, 1}) {
                const size_t tot = sh + wpb * stride;
                if (tot > kLdsMax) continue;
                int blocks = rq_fw_blocks_per_cu(p->nK, c16, p->fwm ? 0 : W, p->bits, wpb, tot, pw);
                if (blocks <= 0) blocks = (int)std::min<size_t>(kLdsMax / tot, 16 / wpb);
                const int waves = blocks * wpb;
                const int score = waves * 4 + (W == 16 ? 2 : W == 32 ? 1 : 0);
                if (score > best) {
                    best = score;
                    p->wpc = waves;
                    p->gwin = W; p->fw_h = H; p->gwpb = wpb; p->gcol_lds = c16; p->gcol16 = c16;
                    p->g_col = o_col; p->g_ptr = o_ptr; p->g_odf = o_odf; p->g_cbf = o_cbf;
                    p->g_wave = sh; p->g_wave_stride = stride; p->g_rank_off = r_off;
                    p->g_win_off = w_off; p->g_stage_off = s_off; p->g_x_off = 0; p->g_total = tot;
                    p->g_etab = o_etab;
                }
            }
        }
        if (best < 0) p->fw = false;
    }
    if (!p->fw) p->fwm = false;
    if (p->fw) p->mrg = p->fwm;   // the merge kernel feeds the fused sweep too

    // pipelined chunks for the merged-stream sweeps (not the sequential LOG sweep, whose
    // global per-sink slots are sized for one grid): the batch in an even number of
    // chunks of <= 131072 replicas on two streams, so the two streams' generation, merge,
    // sweep and scan run side by side and one chunk's sweep tail is the other's work.
    // C3, 10k replicas (profiles/r04_pipe_ab.txt): one stream 3.02 ms per step; two
    // streams x 2 chunks of 5000 2.82 ms; 3 x 3334 3.36; 5 x 2000 4.15; 10 x 1000 5.98
    // (the sweep is latency-bound per replica: a chunk much below the resident wave
    // slots leaves them empty)
    p->nbuf = 1;
    p->order = false;
    if (p->mrg && !p->log) {
        int nb = 2;
        if (const char* e = getenv("RQ_PIPE")) nb = std::max(1, std::min(3, atoi(e)));   // A/B only
        if (b->chunk <= 0) {
            // two chunks (one per stream) up to 2^17 replicas each: C4's 256k replicas of
            // the README graph 16 x 16000 -> 2 x 128000: 7.1 -> 9.2 M replicas/s (a
            // generator launch of 16000 x 3 streams is ~0.7 waves per SIMD)
            int64_t nch = (p->R + 131071) / 131072;
            if (nb > 1) nch = std::max<int64_t>(2, (nch + 1) & ~(int64_t)1);   // even: both streams busy
            if (const char* e = getenv("RQ_PIPE_CHUNK"))   // A/B only
                nch = (p->R + std::max<int64_t>(64, atoll(e)) - 1) / std::max<int64_t>(64, atoll(e));
            nch = std::max<int64_t>(1, std::min(nch, p->R));
            p->chunk = (p->R + nch - 1) / nch;
        }
        const int64_t nch = (p->R + p->chunk - 1) / p->chunk;
        p->nbuf = (int)std::min<int64_t>(nb, nch);
    }

    // the workspace within the device-memory budget (C5: ~20 MB per replica in flight):
    // with the library's chunking, smaller chunks (an even count when pipelined) until the
    // nbuf buffer sets in flight fit; a caller-fixed chunk is the caller's business
    plan_layout(g, b, p);
    if (b->chunk <= 0 && budget > 0.0) {
        while ((double)p->total > budget) {
            if (p->chunk <= 1) return RQ_ENOMEM;
            int64_t c = (int64_t)((double)p->chunk * budget / (double)p->total * 0.97);
            c = std::max<int64_t>(1, std::min<int64_t>(c, p->chunk - 1));
            int64_t nch = (p->R + c - 1) / c;
            if (p->nbuf > 1) nch = (nch + 1) & ~(int64_t)1;
            p->chunk = (p->R + nch - 1) / nch;
            plan_layout(g, b, p);
        }
    }

    // longest-first order (rq_order_replicas) of the replicas the sweep's work queue hands
    // out (a chunk larger than the resident wave slots): measured neutral on C3 (3.01 vs
    // 3.02 ms per step) and slower on C5 (8192 replicas in one chunk: sweep 424 ms against
    // 400 ms in index order, profiles/r04_c5_ab.txt) -- off unless RQ_ORDER=1 (A/B)
    if (const char* e = getenv("RQ_ORDER")) {
        p->order = atoi(e) != 0 && p->mrg && !p->log && p->chunk > (int64_t)std::max(1, p->wpc) * rq_cu_count() &&
                   p->chunk <= 65536;   // rq_order_replicas sorts <= 65536 replicas per launch
        if (p->order) plan_layout(g, b, p);
    }
    return RQ_OK;
}

void plan_layout(const rq_graph* g, const rq_batch_desc* b, Plan* p)
{
    // the sequential sweep's global per-sink slots: no more than the chunk's replicas
    if (p->gs) p->gs_slots = std::min<int64_t>(p->gs_slots, (int64_t)align_up((size_t)p->chunk, (size_t)p->gwpb));
    const size_t A = 256;
    const int64_t C = p->chunk;
    size_t o = 0;
    p->off_invc = o;    o = o + sizeof(double) * (size_t)b->n_grid * g->n_str;
    p->off_stoff = o;   o = o + sizeof(int64_t) * g->n_str;
    p->off_cap = o;     o = o + sizeof(int) * g->n_str;
    p->off_rdk = o;     o = o + sizeof(int) * g->n_str;
    o = align_up(o, 8);
    p->off_repidx = o;  o = o + sizeof(int64_t) * (b->rep_idx ? (size_t)p->R : 0);
    const size_t nseg = b->ctrl_kind == RQ_SRC_OPTPW ? (size_t)b->n_seg : 0;
    o = align_up(o, 8);
    p->off_pwc = o;     o = o + sizeof(double) * (size_t)b->n_grid * g->n_str * nseg;
    p->off_pwmax = o;   o = o + sizeof(double) * (nseg ? (size_t)b->n_grid * g->n_str : 0);
    p->tables_bytes = o;
    o = align_up(o, A);
    // one buffer set per pipelined stream; offsets relative to the set's base
    p->off_set0 = o;
    const size_t o_set = o;
    o = 0;
    const int64_t strm = p->fw && !p->fwm ? 0 : C;   // the generating fused sweep keeps its arrivals in LDS
    const size_t strm_bytes = sizeof(double) * (size_t)strm * p->capsum;
    p->off_slen = o;    o = align_up(o + sizeof(int) * (size_t)strm * g->n_str, A);
    // two-level merge: per (replica, group) the first level's sequences
    p->sub_stride = 0;
    if (p->mrg && p->n_grp > 1)
        for (int gq = 0; gq < p->n_grp; ++gq) {
            int64_t c = 0;
            for (int j = gq * p->grp_sz; j < std::min(g->n_str, (gq + 1) * p->grp_sz); ++j) c += p->cap[j];
            p->sub_stride = std::max(p->sub_stride, (c + 15) & ~(int64_t)15);
        }
    const int64_t subc = p->sub_stride > 0 ? C * p->n_grp : 0;
    p->off_sub_t = o;   o = align_up(o + sizeof(double) * (size_t)subc * p->sub_stride, A);
    p->off_sub_j = o;   o = align_up(o + sizeof(uint16_t) * (size_t)subc * p->sub_stride, A);
    p->off_sub_len = o; o = align_up(o + sizeof(int) * (size_t)subc, A);
    const int64_t mrgc = p->mrg ? C : 0;   // merged sequences: t f64, stream u16, length
    p->off_mt = o;      o = align_up(o + sizeof(double) * (size_t)mrgc * p->mrg_stride, A);
    p->off_mj = o;      o = align_up(o + sizeof(uint16_t) * (size_t)mrgc * p->mrg_stride, A);
    // > 65535 streams: each entry's stream bits 16-23
    p->off_mjh = o;     o = align_up(o + (g->n_str > 65535 ? (size_t)mrgc * p->mrg_stride : 0), A);
    p->off_mlen = o;    o = align_up(o + sizeof(int) * (size_t)mrgc, A);
    p->off_ord = o;     o = align_up(o + sizeof(int) * (size_t)(p->order ? C : 0), A);
    const size_t o_rows = o;
    p->off_rt = o;      o = align_up(o + sizeof(double) * (size_t)C * p->cap_rows, A);
    p->off_rs = o;      o = align_up(o + sizeof(double) * (size_t)C * p->cap_rows, A);
    p->off_rv = o;      o = align_up(o + sizeof(uint32_t) * (size_t)C * p->cap_rows, A);
    p->off_rc = o;      o = align_up(o + sizeof(uint32_t) * (size_t)C * p->cap_rows * p->nK, A);
    // the per-source streams are dead once merged (rq_merge_streams runs before the sweep
    // writes its first row, in the same stream's order): they share the pivot rows' bytes
    if (p->mrg && strm_bytes <= o - o_rows) {
        p->off_streams = o_rows;
    } else {
        p->off_streams = o;
        o = align_up(o + strm_bytes, A);
    }
    p->off_sall = o;    o = align_up(o + sizeof(int) * (size_t)C, A);
    p->off_wq = o;      o = align_up(o + 2 * sizeof(int), A);   // [0] sweep, [1] scan queue
    p->set_stride = o;
    o = o_set + (size_t)p->nbuf * p->set_stride;
    // LOG + gs: per resident wave, rank int + gtag/gcnt/gsum int per sink
    p->gs_stride = p->gs ? (int64_t)align_up(16 * (size_t)p->n_sinks_pad, A) : 0;
    p->off_gs = o;      o = align_up(o + (size_t)(p->gs ? p->gs_slots : 0) * p->gs_stride, A);
    p->total = o;
}

}  // namespace

extern "C" {

int rq_abi_version(void) { return RQ_ABI_VERSION; }

const char* rq_strerror(int code)
{
    switch (code) {
    case RQ_OK: return "ok";
    case RQ_EINVAL: return "invalid argument";
    case RQ_EOVERFLOW: return "capacity overflow";
    case RQ_EHIP: return "HIP runtime error";
    case RQ_ENOMEM: return "out of memory";
    case RQ_EUNSORTED: return "dataframe t column is not sorted";
    case RQ_EUNSUPPORTED: return "unsupported by this engine";
    default: return "unknown error";
    }
}

int rq_graph_build(const rq_graph_desc* d, rq_graph_t* out)
{
    if (!d || !out) return RQ_EINVAL;
    *out = nullptr;
    if (d->n_sinks < 1 || !d->sink_ids) return RQ_EINVAL;              // "No sinks."
    if (d->n_sources < 0 || (d->n_sources > 0 && !d->sources)) return RQ_EINVAL;
    if (d->n_edges < 0 || (d->n_edges > 0 && (!d->edge_src || !d->edge_sink))) return RQ_EINVAL;
    if (!(d->end_time >= d->start_time)) return RQ_EINVAL;
    rq_graph* g = new (std::nothrow) rq_graph();
    if (!g) return RQ_ENOMEM;
    std::unique_ptr<rq_graph> guard(g);
    g->start = d->start_time;
    g->end = d->end_time;
    g->ctrl_src_id = d->ctrl_src_id;

    // sinks: dense columns in sorted id order; "Duplicates in sink_ids."
    std::vector<int64_t> sinks(d->sink_ids, d->sink_ids + d->n_sinks);
    std::sort(sinks.begin(), sinks.end());
    if (std::adjacent_find(sinks.begin(), sinks.end()) != sinks.end()) return RQ_EINVAL;
    g->n_sinks = d->n_sinks;
    g->sink_ids = sinks;
    std::unordered_map<int64_t, int> col;
    for (int c = 0; c < g->n_sinks; ++c) col[sinks[c]] = c;

    // sources: other sources + the controlled slot, in the order run_dynamic plays equal
    // times (opt_model.py:279-290): the dynamic sources (Poisson, Hawkes, a dynamic
    // broadcaster's replayed times) by src_id, then the static ones (Poisson2,
    // PiecewiseConst, RealData; the controlled slot -- a RedQueen controller's ties are
    // the sweep's cbf flags, the other controlled kinds are static) by src_id.  The merge
    // and the sequential sweep play equal times in stream order.
    struct S { int64_t id; int orig; int cls; };
    std::vector<S> order;
    for (int k = 0; k < d->n_sources; ++k) {
        const rq_source_desc& s = d->sources[k];
        if (s.kind < RQ_SRC_POISSON || s.kind > RQ_SRC_REALDATA) return RQ_EUNSUPPORTED;
        if ((s.flags & ~(uint32_t)RQ_SRCF_DYNAMIC) || ((s.flags & RQ_SRCF_DYNAMIC) && s.kind != RQ_SRC_REALDATA))
            return RQ_EINVAL;
        if (s.kind == RQ_SRC_PWCONST || s.kind == RQ_SRC_REALDATA) {
            if (s.n_arr < (s.kind == RQ_SRC_PWCONST ? 1 : 0) || (s.n_arr > 0 && !s.a)) return RQ_EINVAL;
            if (s.kind == RQ_SRC_PWCONST && !s.b) return RQ_EINVAL;
        }
        const bool stat = s.kind == RQ_SRC_POISSON2 || s.kind == RQ_SRC_PWCONST ||
                          (s.kind == RQ_SRC_REALDATA && !(s.flags & RQ_SRCF_DYNAMIC));
        order.push_back({s.src_id, k, stat ? 1 : 0});
    }
    order.push_back({d->ctrl_src_id, -1, 1});
    {
        std::vector<int64_t> ids;
        for (const S& o : order) ids.push_back(o.id);
        std::sort(ids.begin(), ids.end());
        if (std::adjacent_find(ids.begin(), ids.end()) != ids.end()) return RQ_EINVAL;   // "Duplicates in sources."
    }
    std::sort(order.begin(), order.end(),
              [](const S& x, const S& y) { return x.cls != y.cls ? x.cls < y.cls : x.id < y.id; });
    g->n_str = (int)order.size();
    std::unordered_map<int64_t, int> sidx;
    for (int j = 0; j < g->n_str; ++j) {
        const S& o = order[j];
        sidx[o.id] = j;
        g->src_id.push_back(o.id);
        g->orig_idx.push_back(o.orig);
        g->is_static.push_back(o.cls);
        g->arr_off.push_back((int)g->arr_a.size());
        if (o.orig < 0) {
            g->ctrl_idx = j;
            g->kind.push_back(RQ_SRC_NONE);
            g->seed.push_back(0);
            g->p0.push_back(0); g->p1.push_back(0); g->p2.push_back(0);
            g->ctrl_arr_off = (int)g->arr_a.size();
            int n = 0;
            if (d->ctrl_n_arr > 0 && d->ctrl_a) {
                std::vector<double> a(d->ctrl_a, d->ctrl_a + d->ctrl_n_arr);
                if (d->ctrl_b) {   // piecewise: keep order (asserted sorted)
                    if (!std::is_sorted(a.begin(), a.end())) return RQ_EINVAL;
                    for (int q = 0; q < d->ctrl_n_arr; ++q) {
                        g->arr_a.push_back(a[q]);
                        g->arr_b.push_back(d->ctrl_b[q]);
                    }
                    n = d->ctrl_n_arr;
                } else {           // real data: times in [start, end], sorted
                    std::vector<double> keep;
                    for (double t : a) if (t >= g->start && t <= g->end) keep.push_back(t);
                    std::sort(keep.begin(), keep.end());
                    for (double t : keep) { g->arr_a.push_back(t); g->arr_b.push_back(0.0); }
                    n = (int)keep.size();
                }
            }
            g->ctrl_arr_n = n;
            g->arr_n.push_back(n);
            continue;
        }
        const rq_source_desc& s = d->sources[o.orig];
        g->kind.push_back(s.kind);
        g->seed.push_back(s.seed);
        g->p0.push_back(s.p0); g->p1.push_back(s.p1); g->p2.push_back(s.p2);
        int n = 0;
        if (s.kind == RQ_SRC_PWCONST) {
            // PiecewiseConst asserts (opt_model.py:631, :644-645)
            if (!std::is_sorted(s.a, s.a + s.n_arr)) return RQ_EINVAL;
            if (s.a[0] != g->start || g->end < s.a[s.n_arr - 1]) return RQ_EINVAL;
            for (int q = 0; q < s.n_arr; ++q) { g->arr_a.push_back(s.a[q]); g->arr_b.push_back(s.b[q]); }
            n = s.n_arr;
        } else if (s.kind == RQ_SRC_REALDATA) {
            std::vector<double> keep;
            for (int q = 0; q < s.n_arr; ++q)
                if (s.a[q] >= g->start && s.a[q] <= g->end) keep.push_back(s.a[q]);
            std::sort(keep.begin(), keep.end());
            for (double t : keep) { g->arr_a.push_back(t); g->arr_b.push_back(0.0); }
            n = (int)keep.size();
        } else if (s.kind == RQ_SRC_HAWKES) {
            if (!(s.p0 >= 0.0) || !(s.p1 >= 0.0) || !(s.p2 >= 0.0)) return RQ_EINVAL;
        }
        g->arr_n.push_back(n);
    }

    {
        std::vector<double> tw, tc;
        for (int j = 0; j < g->n_str; ++j)
            if (g->kind[j] == RQ_SRC_REALDATA)
                tw.insert(tw.end(), g->arr_a.begin() + g->arr_off[j], g->arr_a.begin() + g->arr_off[j] + g->arr_n[j]);
        if (!d->ctrl_b)   // replayed controller times (change times of a piecewise one are not events)
            tc.assign(g->arr_a.begin() + g->ctrl_arr_off, g->arr_a.begin() + g->ctrl_arr_off + g->ctrl_arr_n);
        std::sort(tw.begin(), tw.end());
        g->rd_ties = std::adjacent_find(tw.begin(), tw.end()) != tw.end();
        tc.insert(tc.end(), tw.begin(), tw.end());
        std::sort(tc.begin(), tc.end());
        g->rd_ties_ctrl = std::adjacent_find(tc.begin(), tc.end()) != tc.end();
    }

    // edges: "Unknown sources/sinks in edge_list." ; CSR in edge-list order
    std::vector<std::vector<int>> rows(g->n_str);
    for (int64_t e = 0; e < d->n_edges; ++e) {
        auto si = sidx.find(d->edge_src[e]);
        auto ci = col.find(d->edge_sink[e]);
        if (si == sidx.end() || ci == col.end()) return RQ_EINVAL;
        rows[si->second].push_back(ci->second);
    }
    g->n_edges = d->n_edges;
    // followers of the controlled source: sorted distinct sink order (Opt.sink_ids,
    // opt_model.py:341, as the State's follower ranks key them)
    std::vector<int> fcols = rows[g->ctrl_idx];
    std::sort(fcols.begin(), fcols.end());
    g->ctrl_dup = std::adjacent_find(fcols.begin(), fcols.end()) != fcols.end();
    fcols.erase(std::unique(fcols.begin(), fcols.end()), fcols.end());
    g->n_fol = (int)fcols.size();
    g->col_to_fol.assign(g->n_sinks, -1);
    for (int f = 0; f < g->n_fol; ++f) {
        g->col_to_fol[fcols[f]] = f;
        g->fol_ids.push_back(sinks[fcols[f]]);
    }
    g->fol = fcols;
    g->csr_ptr.push_back(0);
    g->lay_ptr.push_back(0);
    std::vector<int> seen(g->n_sinks, 0);
    for (int j = 0; j < g->n_str; ++j) {
        // layer k holds the (k+1)-th occurrence of each sink, in edge-list order; the
        // controlled row's layer 0 is the sorted follower list the sweep indexes by
        // follower position
        std::vector<std::vector<int>> layers;
        for (int c : rows[j]) {
            const int k = seen[c]++;
            if ((int)layers.size() <= k) layers.emplace_back();
            layers[k].push_back(c);
        }
        for (int c : rows[j]) seen[c] = 0;
        if (j == g->ctrl_idx && !layers.empty()) layers[0] = fcols;
        g->multi = g->multi || layers.size() > 1;
        int of = 0;
        for (const std::vector<int>& l : layers) {
            for (int c : l) {
                g->csr_col.push_back(c);
                of += g->col_to_fol[c] >= 0;
            }
            g->lay_end.push_back((int)g->csr_col.size());
        }
        if (layers.empty()) g->lay_end.push_back((int)g->csr_col.size());
        g->lay_ptr.push_back((int)g->lay_end.size());
        g->outdeg_f.push_back(of);
        g->csr_ptr.push_back((int)g->csr_col.size());
        // dataframe export: every stream's sinks in edge-list order (duplicates included:
        // Event.sink_ids, opt_model.py:306-307)
        for (int c : rows[j]) g->csr_col_el.push_back(c);
    }

    if (g->n_sinks <= kBitsMaxSinks) {
        g->nw = (g->n_sinks + 31) / 32;
        g->masks.assign((size_t)g->n_str * g->nw, 0u);
        for (int j = 0; j < g->n_str; ++j)
            for (int e = g->csr_ptr[j]; e < g->csr_ptr[j + 1]; ++e) {
                const int c = g->csr_col[e];
                g->masks[(size_t)j * g->nw + c / 32] |= 1u << (c % 32);
            }
    }

    g->fbits.assign((g->n_sinks + 31) / 32, 0u);
    for (int c : g->fol) g->fbits[c / 32] |= 1u << (c % 32);
    // the controller posts before a wall event at the same time when that source is static
    // or has a larger src_id (opt_model.py:279-281, :289-290): the sweeps' per-stream flag,
    // in global memory for the GT instances (the others build it in LDS)
    std::vector<int> cbf(g->n_str);
    for (int j = 0; j < g->n_str; ++j) cbf[j] = g->is_static[j] || g->ctrl_src_id < g->src_id[j];

    int rc;
    if (g->nw > 0 && (rc = g->d_mask.upload(g->masks))) return rc;
    if ((rc = g->d_fbits.upload(g->fbits))) return rc;
    if ((rc = g->d_src_id.upload(g->src_id)) || (rc = g->d_kind.upload(g->kind)) ||
        (rc = g->d_orig.upload(g->orig_idx)) || (rc = g->d_arr_off.upload(g->arr_off)) ||
        (rc = g->d_arr_n.upload(g->arr_n)) || (rc = g->d_csr_ptr.upload(g->csr_ptr)) ||
        (rc = g->d_csr_col.upload(g->csr_col)) || (rc = g->d_outdeg_f.upload(g->outdeg_f)) ||
        (rc = g->d_fol.upload(g->fol)) || (rc = g->d_seed.upload(g->seed)) ||
        (rc = g->d_p0.upload(g->p0)) || (rc = g->d_p1.upload(g->p1)) ||
        (rc = g->d_p2.upload(g->p2)) || (rc = g->d_arr_a.upload(g->arr_a)) ||
        (rc = g->d_arr_b.upload(g->arr_b)) || (rc = g->d_sink_ids.upload(g->sink_ids)) ||
        (rc = g->d_csr_col_el.upload(g->csr_col_el)) || (rc = g->d_cbf.upload(cbf)))
        return rc;
    if (g->multi && ((rc = g->d_lay_ptr.upload(g->lay_ptr)) || (rc = g->d_lay_end.upload(g->lay_end))))
        return rc;
    *out = guard.release();
    return RQ_OK;
}

int rq_graph_free(rq_graph_t g)
{
    delete g;
    return RQ_OK;
}

int rq_graph_info(rq_graph_t g, int64_t* info)
{
    if (!g || !info) return RQ_EINVAL;
    info[0] = g->n_str;
    info[1] = g->n_sinks;
    info[2] = g->n_fol;
    info[3] = g->n_edges;
    info[4] = g->ctrl_idx;
    return RQ_OK;
}

int rq_graph_source_ids(rq_graph_t g, int64_t* ids)
{
    if (!g || !ids) return RQ_EINVAL;
    std::copy(g->src_id.begin(), g->src_id.end(), ids);
    return RQ_OK;
}

int rq_graph_followers(rq_graph_t g, int64_t* ids)
{
    if (!g || !ids) return RQ_EINVAL;
    std::copy(g->fol_ids.begin(), g->fol_ids.end(), ids);
    return RQ_OK;
}

int rq_workspace_size(rq_graph_t g, const rq_batch_desc* b, size_t* bytes)
{
    if (!bytes) return RQ_EINVAL;
    Plan p;
    const int rc = make_plan(g, b, &p, ws_budget(b, 0.0));
    if (rc) return rc;
    *bytes = p.total;
    return RQ_OK;
}

int rq_plan_info(rq_graph_t g, const rq_batch_desc* b, int64_t* info)
{
    if (!info) return RQ_EINVAL;
    Plan p;
    const int rc = make_plan(g, b, &p, ws_budget(b, 0.0));
    if (rc) return rc;
    info[0] = (p.log ? (p.gs ? 4 : 1) : (p.bits ? 2 : (p.bl ? 3 : 0))) + (p.fwm ? 20 : p.fw ? 10 : 0);
    info[1] = p.mrg ? 0 : p.spl;   // 0: merged streams (lanes own no sources)
    info[2] = p.gwin;
    info[3] = p.gwpb;
    info[4] = p.fw ? rq_fw_blocks_per_cu(p.nK, p.gcol16, p.fwm ? 0 : p.gwin, p.bits, p.gwpb, p.g_total,
                                          b->ctrl_kind == RQ_SRC_OPTPW)
                   : rq_sweep_blocks_per_cu(p.mrg ? (p.gt ? -1 : 0) : p.spl, p.nK, p.gcol16, p.gwin, p.log ? 1 + p.gs : 0,
                                            p.bl ? 2 : p.bits, p.gwpb, p.g_total);
    info[5] = p.gcol_lds;
    info[6] = (int64_t)p.g_total;
    info[7] = p.chunk;
    return RQ_OK;
}

int rq_event_capacity(rq_graph_t g, const rq_batch_desc* b, int64_t* cap)
{
    if (!cap) return RQ_EINVAL;
    Plan p;
    const int rc = make_plan(g, b, &p, ws_budget(b, 0.0));
    if (rc) return rc;
    *cap = p.cap_rows;
    return RQ_OK;
}

int rq_run_batch(rq_graph_t g, const rq_batch_desc* b, const rq_outputs* out, void* workspace,
                 size_t workspace_bytes, void* hip_stream)
{
    Plan p;
    // the same plan as rq_workspace_size gave when the caller fixes the budget; else the
    // chunks that fit the workspace handed over
    int rc = make_plan(g, b, &p, ws_budget(b, (double)workspace_bytes));
    if (rc) return rc;
    if (!out || !out->metrics || !out->counts || !out->status || !workspace) return RQ_EINVAL;
    if (workspace_bytes < p.total) return RQ_EINVAL;
    if ((b->flags & RQ_RUN_EVENT_LOG) && (!out->ev_t || !out->ev_src || out->ev_cap < 1))
        return RQ_EINVAL;
    hipStream_t s = (hipStream_t)hip_stream;
    char* ws = (char*)workspace;

    // c_j = sum over edges (j, i), i a follower, of sqrt(s_i / q)  (opt_model.py:515, :536)
    std::vector<double> invc((size_t)b->n_grid * g->n_str, 0.0);
    if (b->ctrl_kind == RQ_SRC_OPT) {
        std::vector<double> w(g->n_fol);
        for (int gi = 0; gi < b->n_grid; ++gi) {
            for (int f = 0; f < g->n_fol; ++f) w[f] = std::sqrt(b->s[(size_t)gi * g->n_fol + f] / b->q[gi]);
            for (int j = 0; j < g->n_str; ++j) {
                if (j == g->ctrl_idx) continue;
                double c = 0.0;
                // edge-list order (duplicate edges count once each), as the oracle sums
                for (int e = g->csr_ptr[j]; e < g->csr_ptr[j + 1]; ++e) {
                    const int f = g->col_to_fol[g->csr_col_el[e]];
                    if (f >= 0) c = c + w[f];
                }
                invc[(size_t)gi * g->n_str + j] = c > 0.0 ? 1.0 / c : 0.0;
            }
        }
    }
    // OptPWSignificance: per (grid point, stream) the intensity increment of one event
    // of stream j per significance segment, pw[k] = sum over edges (j, i), i a follower,
    // of sqrt(s_pw[i, k] / q) (opt_model.py:613-614 with rank_diff_i = edge multiplicity),
    // edge-list order; and its max over k (the thinning bound, :563)
    std::vector<double> pwc, pwmax;
    if (b->ctrl_kind == RQ_SRC_OPTPW) {
        const int S = b->n_seg;
        pwc.assign((size_t)b->n_grid * g->n_str * S, 0.0);
        pwmax.assign((size_t)b->n_grid * g->n_str, 0.0);
        for (int gi = 0; gi < b->n_grid; ++gi)
            for (int j = 0; j < g->n_str; ++j) {
                if (j == g->ctrl_idx) continue;
                double* row = &pwc[((size_t)gi * g->n_str + j) * S];
                for (int e = g->csr_ptr[j]; e < g->csr_ptr[j + 1]; ++e) {
                    const int f = g->col_to_fol[g->csr_col_el[e]];
                    if (f < 0) continue;
                    const double* sp = b->s_pw + ((size_t)gi * g->n_fol + f) * S;
                    for (int k = 0; k < S; ++k) row[k] = row[k] + std::sqrt(sp[k] / b->q[gi]);
                }
                double m = 0.0;
                for (int k = 0; k < S; ++k) m = row[k] > m ? row[k] : m;
                pwmax[(size_t)gi * g->n_str + j] = m;
            }
    }
    // parameter tables [inv_c | st_off | cap | rd_k | pw_c | pw_max]: staged in one of the graph's pinned host
    // buffers so the copy is truly asynchronous (a pageable copy would stall the host)
    {
        std::lock_guard<std::mutex> lk(g->stage_mu);
        Stage& st = g->stage[g->stage_next];
        g->stage_next = (g->stage_next + 1) % kStages;
        if (st.bytes < p.tables_bytes) {
            // grow the whole ring at once (pinned allocation is slow: never leave a stage
            // to be allocated by a later, possibly timed, call); round up to 64 KiB
            const size_t want = align_up(p.tables_bytes, (size_t)65536);
            for (Stage& x : g->stage) {
                if (x.done && hipEventSynchronize(x.done) != hipSuccess) return RQ_EHIP;
                if (x.bytes >= want) continue;
                if (x.buf) (void)hipHostFree(x.buf);
                x.buf = nullptr;
                x.bytes = 0;
                if (hipHostMalloc(&x.buf, want, hipHostMallocDefault) != hipSuccess) return RQ_ENOMEM;
                x.bytes = want;
                if (!x.done && hipEventCreateWithFlags(&x.done, hipEventDisableTiming) != hipSuccess)
                    return RQ_EHIP;
            }
        }
        if (st.done && hipEventSynchronize(st.done) != hipSuccess) return RQ_EHIP;
        char* tab = (char*)st.buf;
        std::memcpy(tab + p.off_invc, invc.data(), invc.size() * sizeof(double));
        std::memcpy(tab + p.off_stoff, p.st_off.data(), p.st_off.size() * sizeof(int64_t));
        std::memcpy(tab + p.off_cap, p.cap.data(), p.cap.size() * sizeof(int));
        std::memcpy(tab + p.off_rdk, p.rd_k.data(), p.rd_k.size() * sizeof(int));
        if (b->rep_idx) std::memcpy(tab + p.off_repidx, b->rep_idx, sizeof(int64_t) * (size_t)p.R);
        if (!pwc.empty()) {
            std::memcpy(tab + p.off_pwc, pwc.data(), pwc.size() * sizeof(double));
            std::memcpy(tab + p.off_pwmax, pwmax.data(), pwmax.size() * sizeof(double));
        }
        if (hipMemcpyAsync(ws, tab, p.tables_bytes, hipMemcpyHostToDevice, s) != hipSuccess ||
            hipEventRecord(st.done, s) != hipSuccess)
            return RQ_EHIP;
    }
    if (hipMemsetAsync(out->status, 0, sizeof(int32_t) * p.R, s) != hipSuccess) return RQ_EHIP;

    const int ctrl_stream_kind =
        (b->ctrl_kind == RQ_SRC_OPT || b->ctrl_kind == RQ_SRC_OPTPW || b->ctrl_kind == RQ_SRC_NONE)
            ? RQ_SRC_NONE : b->ctrl_kind;
    // pipelined chunks: chunk k runs on stream k % nbuf (the caller's stream and up to two
    // side streams, forked after the tables / status above and joined before returning)
    // with buffer set k % nbuf, so a set is reused only in its own stream's order
    hipStream_t pst[3] = {s, nullptr, nullptr};
    SidePipe& t_pipe = t_pipes.of(s);
    // the join of the side streams on EVERY exit: an error return inside the chunk loop
    // must not leave work queued on a side stream that writes the caller's buffers after
    // the caller's stream has moved on (the caller frees them when the call fails)
    struct Join {
        hipStream_t* pst;
        SidePipe& sp;
        int n = 1;
        int done()
        {
            int rc = RQ_OK;
            for (int k = 1; k < n; ++k)
                if (hipEventRecord(sp.join[k - 1], pst[k]) != hipSuccess ||
                    hipStreamWaitEvent(pst[0], sp.join[k - 1], 0) != hipSuccess)
                    rc = RQ_EHIP;
            n = 1;
            return rc;
        }
        ~Join() { (void)done(); }
    } join{pst, t_pipe};
    if (p.nbuf > 1) {
        if ((rc = t_pipe.get(p.nbuf - 1, pst + 1)) != RQ_OK) return rc;
        if (hipEventRecord(t_pipe.fork, s) != hipSuccess) return RQ_EHIP;
        for (int k = 1; k < p.nbuf; ++k) {
            if (hipStreamWaitEvent(pst[k], t_pipe.fork, 0) != hipSuccess) return RQ_EHIP;
            join.n = k + 1;
        }
    }
    int64_t ci = 0;
    for (int64_t c0 = 0; c0 < p.R; c0 += p.chunk, ++ci) {
        const int64_t C = std::min(p.chunk, p.R - c0);
        hipStream_t s = pst[ci % p.nbuf];
        char* wsb = ws + p.off_set0 + (size_t)(ci % p.nbuf) * p.set_stride;   // this chunk's buffer set
        GenArgs ga{};
        ga.n_chunk = C;
        ga.chunk0 = c0;
        ga.rep0 = b->replica0;
        ga.n_rep = b->n_rep;
        ga.rep_lo = p.rep_lo;
        ga.rep_cnt = p.rep_cnt;
        ga.rep_idx = b->rep_idx ? (const int64_t*)(ws + p.off_repidx) : nullptr;
        ga.n_str = g->n_str;
        ga.ctrl_idx = g->ctrl_idx;
        ga.ctrl_stream_kind = ctrl_stream_kind;
        ga.randomize = b->randomize_world;
        ga.seed_mod = b->seed_mod;
        ga.ctrl_seed = b->ctrl_seed;
        ga.ctrl_seed0 = b->ctrl_seed0;
        ga.world_seed = b->world_seed;
        ga.world_seed0 = b->world_seed0;
        ga.ctrl_rate = b->ctrl_rate;
        ga.kind = g->d_kind.p;
        ga.orig_idx = g->d_orig.p;
        ga.seed = g->d_seed.p;
        ga.p0 = g->d_p0.p;
        ga.p1 = g->d_p1.p;
        ga.p2 = g->d_p2.p;
        ga.arr_off = g->d_arr_off.p;
        ga.arr_n = g->d_arr_n.p;
        ga.arr_a = g->d_arr_a.p;
        ga.arr_b = g->d_arr_b.p;
        ga.st_off = (const int64_t*)(ws + p.off_stoff);
        ga.cap = (const int*)(ws + p.off_cap);
        ga.capsum = p.capsum;
        ga.start = g->start;
        ga.end = g->end;
        ga.streams = (double*)(wsb + p.off_streams);
        ga.slen = (int*)(wsb + p.off_slen);
        ga.slen_stride = p.chunk;
        ga.status = out->status;
        if (b->n_rd > 0) {
            ga.rd_k = (const int*)(ws + p.off_rdk);
            ga.n_rd = b->n_rd;
            ga.rd_times = b->rd_times;
            ga.rd_off = b->rd_off;
        }
        if (!p.fw || p.fwm) {
            TimedLaunch tl(K_GEN, s);
            if (rq_launch_gen(ga, s) != hipSuccess) return RQ_EHIP;
        }
        if (p.mrg) {
            MergeArgs ma{};
            ma.n_chunk = C;
            ma.chunk0 = c0;
            ma.n_str = g->n_str;
            ma.capsum = p.capsum;
            ma.st_off = ga.st_off;
            ma.streams = ga.streams;
            ma.slen = ga.slen;
            ma.slen_stride = ga.slen_stride;
            ma.end = g->end;
            ma.out_t = (double*)(wsb + p.off_mt);
            ma.out_j = (uint16_t*)(wsb + p.off_mj);
            ma.out_jh = g->n_str > 65535 ? (uint8_t*)(wsb + p.off_mjh) : nullptr;
            ma.out_len = (int*)(wsb + p.off_mlen);
            ma.mrg_stride = p.mrg_stride;
            ma.status = out->status;
            ma.strict_ties = p.lmrg ? 1 : 0;
#ifdef RQ_PHASE_CLOCK
            if (getenv("RQ_CLK_MERGE")) ma.clk = phase_clk();   // else the sweep's phases only
#endif
            TimedLaunch tl(K_MERGE, s);
            if (p.n_grp > 1) {
                // level 1: each group of grp_sz streams into its own sequence
                ma.grp_sz = p.grp_sz;
                MergeArgs m1 = ma;
                m1.out_t = (double*)(wsb + p.off_sub_t);
                m1.out_j = (uint16_t*)(wsb + p.off_sub_j);   // group-local streams: u16 always
                m1.out_jh = nullptr;
                m1.out_len = (int*)(wsb + p.off_sub_len);
                m1.mrg_stride = p.sub_stride;
                if (rq_launch_merge_groups(m1, s) != hipSuccess) return RQ_EHIP;
                // level 2: the groups' sequences into the replica's play order
                ma.sub_t = m1.out_t;
                ma.sub_j = m1.out_j;
                ma.sub_len = m1.out_len;
                ma.n_grp = p.n_grp;
                ma.sub_stride = p.sub_stride;
                if (rq_launch_merge_sub(ma, s) != hipSuccess) return RQ_EHIP;
            } else if (rq_launch_merge(ma, s) != hipSuccess) {
                return RQ_EHIP;
            }
        }

        SweepArgs sa{};
        sa.n_chunk = C;
        sa.chunk0 = c0;
        sa.n_rep = b->n_rep;
        sa.rep0 = b->replica0;
        sa.wpb = p.wpb;
        sa.n_str = g->n_str;
        sa.n_sinks = g->n_sinks;
        sa.n_sinks_pad = p.n_sinks_pad;
        sa.ctrl_idx = g->ctrl_idx;
        sa.ctrl_kind = b->ctrl_kind;
        sa.n_fol = b->ctrl_kind == RQ_SRC_NONE ? 0 : g->n_fol;
        for (int q = 0; q < RQ_MAX_K; ++q) sa.Ks[q] = q < b->nK ? b->Ks[q] : 1;
        sa.ctrl_src_id = g->ctrl_src_id;
        sa.seed_mod = b->seed_mod;
        sa.ctrl_seed = b->ctrl_seed;
        sa.ctrl_seed0 = b->ctrl_seed0;
        sa.src_id = g->d_src_id.p;
        sa.inv_c = (const double*)(ws + p.off_invc);
        if (b->ctrl_kind == RQ_SRC_OPTPW) {
            sa.pw_c = (const double*)(ws + p.off_pwc);
            sa.pw_max = (const double*)(ws + p.off_pwmax);
            sa.n_seg = b->n_seg;
            sa.period = b->period;
        }
        sa.csr_ptr = g->d_csr_ptr.p;
        sa.csr_col = g->d_csr_col.p;
        sa.outdeg_f = g->d_outdeg_f.p;
        sa.cbf_g = g->d_cbf.p;
        sa.fol = g->d_fol.p;
        sa.st_off = (const int64_t*)(ws + p.off_stoff);
        sa.capsum = p.capsum;
        sa.streams = (const double*)(wsb + p.off_streams);
        sa.slen = (const int*)(wsb + p.off_slen);
        sa.slen_stride = p.chunk;
        if (p.mrg) {
            sa.mrg_t = (const double*)(wsb + p.off_mt);
            sa.mrg_j = (const uint16_t*)(wsb + p.off_mj);
            sa.mrg_jh = g->n_str > 65535 ? (const uint8_t*)(wsb + p.off_mjh) : nullptr;
            sa.mrg_len = (const int*)(wsb + p.off_mlen);
            sa.mrg_stride = p.mrg_stride;
            if (p.order) {
                int* ord = (int*)(wsb + p.off_ord);
                if (rq_launch_order(sa.mrg_len, C, ord, s) != hipSuccess) return RQ_EHIP;
                sa.order = ord;
            }
        }
        sa.start = g->start;
        sa.end = g->end;
        sa.max_events = b->max_events;
        sa.cap_rows = p.cap_rows;
        sa.rows_t = (double*)(wsb + p.off_rt);
        sa.rows_sum = (double*)(wsb + p.off_rs);
        sa.rows_valid = (uint32_t*)(wsb + p.off_rv);
        sa.rows_cnt = (uint32_t*)(wsb + p.off_rc);
        sa.sall = (int*)(wsb + p.off_sall);
        sa.counts = out->counts;
        sa.status = out->status;
        if (b->flags & RQ_RUN_EVENT_LOG) {
            sa.ev_t = out->ev_t;
            sa.ev_src = out->ev_src;
            sa.ev_cap = out->ev_cap;
        }
        {
            sa.n_csr = (int)g->csr_col.size();
            sa.wpb = p.gwpb;
            sa.win = p.gwin;
            sa.col_in_lds = p.gcol_lds;
            sa.lds_col = p.g_col;
            sa.lds_ptr = p.g_ptr;
            sa.lds_odf = p.g_odf;
            sa.lds_cbf = p.g_cbf;
            sa.lds_wave = p.g_wave;
            sa.lds_wave_stride = p.g_wave_stride;
            sa.lds_rank_off = p.g_rank_off;
            sa.lds_win_off = p.g_win_off;
            sa.lds_x_off = p.g_x_off;
            sa.lay_ptr = g->multi ? g->d_lay_ptr.p : nullptr;
            sa.lay_end = g->multi ? g->d_lay_end.p : nullptr;
            if (p.gs) {
                sa.gs = ws + p.off_gs;
                sa.gs_stride = p.gs_stride;
                sa.gs_slots = (int)p.gs_slots;
            }
            sa.lds_mask = p.g_col;   // BITS: the bitsets take the columns' place
            sa.masks = g->d_mask.p;
            sa.nw = g->nw;
            sa.mstride = p.mstride;
            sa.fbits = g->d_fbits.p;
            sa.nwl = (g->n_sinks + 31) / 32;
            sa.lds_fbits = p.g_fb;
            sa.lds_skip = p.g_skip;
            sa.lds_etab = p.g_etab;
            sa.lds_invc = p.g_inv;
            sa.invc_shared = !p.fw && p.g_inv_sh;
            if (const char* d = getenv("RQ_SWEEP_DBG")) sa.dbg = atoi(d);   // profiling only
            sa.tile_target = 58.0;   // measured on C3: 40 -> 895k, 48 -> 943k, 58 -> 964k, 62 -> 956k replicas/s
            if (const char* e = getenv("RQ_FW_TILE")) sa.tile_target = atof(e);   // tuning only
            // refill policy (C3, sweep ms): forced passes only when a ring shows < 2 arrivals
            // (the cut is bounded by each ring's last visible arrival), opportunistic passes
            // while >= n_str / 2 rings are below W -- (H, n/3) 4.12, (2, n/3) 3.86,
            // (2, n/2) 3.79, (2, 0.64 n) 3.89, (1, n/2) 3.84-3.88
            sa.fw_hmin = std::min(2, p.fw_h);
            if (const char* e = getenv("RQ_FW_HMIN")) sa.fw_hmin = std::max(1, std::min(p.fw_h, atoi(e)));   // tuning only
            sa.fw_thr = g->n_str >= 6 ? (g->n_str + 1) / 2 : 2;
            if (const char* e = getenv("RQ_FW_THR")) sa.fw_thr = std::max(1, atoi(e));   // tuning only
            // a forced run (some ring < fw_hmin) ends once every ring shows H arrivals, not W:
            // (C3 sweep ms) fill to 16 3.85, 12 3.78, 8 3.69-3.71, 6 3.69, 4 3.71
            sa.fw_hfill = p.fw_h;
            if (const char* e = getenv("RQ_FW_HFILL")) sa.fw_hfill = std::max(1, std::min(p.gwin, atoi(e)));   // tuning only
#ifdef RQ_PHASE_CLOCK
            sa.clk = phase_clk();
#endif
            sa.lds_total = p.g_total;
            sa.lds_stage_off = p.g_stage_off;
            sa.gen = ga;
            // fused sweep: waves past their first replica take the next one from a queue,
            // so the launch tail is spread over every CU instead of whole 16-wave blocks
            static const int wq_off = getenv("RQ_FW_STATIC") ? atoi(getenv("RQ_FW_STATIC")) : 0;   // A/B only
            // both queues of this chunk (sweep, scan) zeroed by one memset
            if (hipMemsetAsync(wsb + p.off_wq, 0, 2 * sizeof(int), s) != hipSuccess) return RQ_EHIP;
            if (!wq_off || p.gs) {   // both sweep kinds take replicas past the first from the queue (GS needs it)
                sa.wq = (int*)(wsb + p.off_wq);
            }
            TimedLaunch tl(K_SWEEP, s);
            const hipError_t e = p.fw ? rq_launch_sweep_fw(sa, p.nK, p.gcol16, p.fwm ? 0 : p.gwin, p.bits, s)
                                      : rq_launch_sweep(sa, p.mrg ? (p.gt ? -1 : 0) : p.spl, p.nK, p.gcol16, p.log ? 1 + p.gs : 0,
                                                        p.bl ? 2 : p.bits, s);
            if (e != hipSuccess) return RQ_EHIP;
        }

        ScanArgs sc{};
        sc.n_chunk = C;
        sc.chunk0 = c0;
        sc.nrows = out->counts + 3;
        sc.nrows_stride = 4;
        sc.sall = (const int*)(wsb + p.off_sall);
        sc.row_stride = p.cap_rows;
        sc.rows_t = sa.rows_t;
        sc.rows_sum = sa.rows_sum;
        sc.rows_valid = sa.rows_valid;
        sc.rows_cnt = sa.rows_cnt;
        sc.end = g->end;
        sc.metrics = out->metrics;
        sc.wq = (int*)(wsb + p.off_wq) + 1;
        {
            TimedLaunch tl(K_SCAN, s);
            if (rq_launch_scan(sc, p.nK, s) != hipSuccess) return RQ_EHIP;
        }
    }
    return join.done();   // the caller's stream waits for every side stream
}

int rq_timing(int enable)
{
    for (int k = 0; k < K_N; ++k) {
        for (auto& e : g_ev[k]) {
            (void)hipEventDestroy(e.first);
            (void)hipEventDestroy(e.second);
        }
        g_ev[k].clear();
    }
    g_timing = enable != 0;
    return RQ_OK;
}

int rq_timing_read(double* ms, int64_t* launches)
{
    if (!ms || !launches) return RQ_EINVAL;
    for (int k = 0; k < K_N; ++k) {
        double tot = 0.0;
        for (auto& e : g_ev[k]) {
            float f = 0.0f;
            if (hipEventSynchronize(e.second) != hipSuccess) return RQ_EHIP;
            if (hipEventElapsedTime(&f, e.first, e.second) != hipSuccess) return RQ_EHIP;
            tot += f;
        }
        ms[k] = tot;
        launches[k] = (int64_t)g_ev[k].size();
    }
    return rq_timing(g_timing ? 1 : 0);
}

namespace {
// replay workspace: per-df status, pivot rows, fallback sink keys; the large
// layout adds per-df hash tables / sequential-replay state (slots [4 r0, 4 r1))
struct RpPlan {
    size_t off_info, off_dt, off_sum, off_valid, off_cnt, off_keys, off_gkeys, off_gstate, small, large;
    // chunked replay area (RQ_REPLAY_CHUNKED), after the large area when both are asked for
    int64_t max_chunks;
    size_t c_cbase, c_hkeys, c_hdense, c_gstart, c_gbase, c_carry, c_state, chunk;
};
RpPlan rp_plan(int64_t n_rows, int64_t n_df, int32_t nK)
{
    RpPlan p{};
    const size_t A = 256, n = (size_t)std::max<int64_t>(n_rows, 1);
    size_t o = 0;
    p.off_info = o;  o = align_up(o + sizeof(RpInfo) * (size_t)std::max<int64_t>(n_df, 1), A);
    p.off_dt = o;    o = align_up(o + 8 * n, A);
    p.off_sum = o;   o = align_up(o + 8 * n, A);
    p.off_valid = o; o = align_up(o + 4 * n, A);
    p.off_cnt = o;   o = align_up(o + 4 * n * (size_t)nK, A);
    p.off_keys = o;  o = align_up(o + 8 * n, A);
    p.small = o;
    p.off_gkeys = o; o = align_up(o + 8 * 4 * n, A);
    p.off_gstate = o; o = align_up(o + 16 * 4 * n, A);
    p.large = o;
    // chunk area, offsets relative to its start: per df the chunk prefix and a sink hash
    // table; per chunk (<= n_rows / RC_L + n_df) its t-group counts and RC_S carries / states
    const size_t nd = (size_t)std::max<int64_t>(n_df, 1);
    p.max_chunks = std::max<int64_t>(n_rows, 0) / RC_L + std::max<int64_t>(n_df, 1);
    const size_t mc = (size_t)p.max_chunks;
    size_t c = 0;
    p.c_cbase = c;  c = align_up(c + 8 * (nd + 1), A);
    p.c_hkeys = c;  c = align_up(c + 8 * nd * RC_HT, A);
    p.c_hdense = c; c = align_up(c + 4 * nd * RC_HT, A);
    p.c_gstart = c; c = align_up(c + 4 * mc, A);
    p.c_gbase = c;  c = align_up(c + 8 * mc, A);
    p.c_carry = c;  c = align_up(c + sizeof(RcCarry) * mc * RC_S, A);
    p.c_state = c;  c = align_up(c + sizeof(RcState) * mc * RC_S, A);
    p.chunk = c;
    return p;
}

int rp_run(const double* t, const int64_t* src, const int64_t* sink, const int64_t* event_id,
           const int64_t* df_off, int64_t n_df, int64_t n_rows, int64_t src_id, double end_time,
           const int32_t* Ks, int32_t nK, double* out, int64_t* counts, void* workspace,
           size_t workspace_bytes, void* hip_stream)
{
    if (!out || !counts || !workspace || !Ks || n_df < 1 || n_rows < 0) return RQ_EINVAL;
    if (n_rows > 0 && (!t || !src || !sink)) return RQ_EINVAL;
    if (nK < 1 || nK > RQ_MAX_K) return RQ_EINVAL;
    for (int q = 0; q < nK; ++q)
        if (Ks[q] < 1) return RQ_EINVAL;
    const RpPlan p = rp_plan(n_rows, n_df, nK);
    if (workspace_bytes < p.small) return RQ_EINVAL;
    // workspace tiers (rq_replay_workspace_size): small [+ large] [+ chunk]
    const bool both = workspace_bytes >= p.large + p.chunk;
    const bool large = workspace_bytes >= p.large;
    const bool has_chunk = both || (!large && workspace_bytes >= p.small + p.chunk);
    char* ws = (char*)workspace;
    char* cw = ws + (both ? p.large : p.small);
    // one dataframe over many workgroups: few, long dataframes (a batch of many fills the
    // chip with one workgroup each)
    bool chunked = has_chunk && n_df <= 64 && n_rows >= 2 * (int64_t)RC_L * n_df;
    if (const char* e = getenv("RQ_RP_CHUNK")) chunked = has_chunk && atoi(e) != 0;   // A/B only
    RpArgs a{};
    a.t = t;
    a.src = src;
    a.sink = sink;
    a.eid = event_id;
    a.df_off = df_off;
    a.n_df = n_df;
    a.n_rows = n_rows;
    a.src_id = src_id;
    a.end = end_time;
    a.nK = nK;
    for (int q = 0; q < RQ_MAX_K; ++q) a.Ks[q] = q < nK ? Ks[q] : 1;
#ifdef RQ_PHASE_CLOCK
    if (getenv("RQ_CLK_REPLAY")) a.clk = phase_clk();
#endif
    a.info = (RpInfo*)(ws + p.off_info);
    a.rows_dt = (double*)(ws + p.off_dt);
    a.rows_sum = (double*)(ws + p.off_sum);
    a.rows_valid = (uint32_t*)(ws + p.off_valid);
    a.rows_cnt = (uint32_t*)(ws + p.off_cnt);
    a.keys = (int64_t*)(ws + p.off_keys);
    a.gkeys = large ? (uint64_t*)(ws + p.off_gkeys) : nullptr;
    a.gstate = large ? (void*)(ws + p.off_gstate) : nullptr;
    a.metrics = out;
    a.counts = counts;
    // the small-table tier (two workgroups per CU) first, for one K; A/B knob RQ_RP_SMALL
    a.first_tier = nK == 1 ? 0 : 1;
    if (const char* e = getenv("RQ_RP_SMALL")) a.first_tier = (nK == 1 && atoi(e) != 0) ? 0 : 1;   // A/B only
    if (chunked) {
        a.chunked = 1;
        a.max_chunks = p.max_chunks;
        a.cbase = (int64_t*)(cw + p.c_cbase);
        a.ht_keys = (uint64_t*)(cw + p.c_hkeys);
        a.ht_dense = (int*)(cw + p.c_hdense);
        a.gstart = (int*)(cw + p.c_gstart);
        a.gbase = (int64_t*)(cw + p.c_gbase);
        a.carry = (RcCarry*)(cw + p.c_carry);
        a.state = (RcState*)(cw + p.c_state);
    }
    hipStream_t s = (hipStream_t)hip_stream;
    {
        TimedLaunch tl(K_REPLAY, s);
        if (chunked && rq_launch_rp(a, RP_PHASE_CHUNK, s) != hipSuccess) return RQ_EHIP;
        if (a.first_tier == 0 && rq_launch_rp(a, RP_PHASE_SMALL, s) != hipSuccess) return RQ_EHIP;
        if (rq_launch_rp(a, RP_PHASE_FAST, s) != hipSuccess) return RQ_EHIP;
        if (large && rq_launch_rp(a, RP_PHASE_GLOBAL, s) != hipSuccess) return RQ_EHIP;
        if (rq_launch_rp(a, RP_PHASE_KEYS, s) != hipSuccess) return RQ_EHIP;
        if (rq_launch_rp(a, RP_PHASE_SEQ, s) != hipSuccess) return RQ_EHIP;
    }
    TimedLaunch tl(K_SCAN, s);
    return rq_launch_rp(a, RP_PHASE_SCAN, s) == hipSuccess ? RQ_OK : RQ_EHIP;
}
}  // namespace

int rq_replay_workspace_size(int64_t n_rows, int64_t n_df, int32_t nK, int32_t flags, size_t* bytes)
{
    if (!bytes || n_rows < 0 || n_df < 1 || nK < 1 || nK > RQ_MAX_K) return RQ_EINVAL;
    const RpPlan p = rp_plan(n_rows, n_df, nK);
    *bytes = ((flags & RQ_REPLAY_LARGE) ? p.large : p.small) + ((flags & RQ_REPLAY_CHUNKED) ? p.chunk : 0);
    return RQ_OK;
}

int rq_metrics_replay(const double* t, const int64_t* src, const int64_t* sink,
                      const int64_t* event_id, int64_t n_rows, int64_t src_id, double end_time,
                      const int32_t* Ks, int32_t nK, double* out, int64_t* counts, void* workspace,
                      size_t workspace_bytes, void* hip_stream)
{
    return rp_run(t, src, sink, event_id, nullptr, 1, n_rows, src_id, end_time, Ks, nK, out,
                  counts, workspace, workspace_bytes, hip_stream);
}

int rq_metrics_replay_batch(const double* t, const int64_t* src, const int64_t* sink,
                            const int64_t* event_id, const int64_t* df_off, int64_t n_df,
                            int64_t n_rows, int64_t src_id, double end_time, const int32_t* Ks,
                            int32_t nK, double* out, int64_t* counts, void* workspace,
                            size_t workspace_bytes, void* hip_stream)
{
    if (!df_off) return RQ_EINVAL;
    return rp_run(t, src, sink, event_id, df_off, n_df, n_rows, src_id, end_time, Ks, nK, out,
                  counts, workspace, workspace_bytes, hip_stream);
}

}  // extern "C"

// ============================================================================
// analysis entry points (rq_analysis.hip)
// ============================================================================
namespace {
constexpr size_t kOracleLdsMax = 128 * 1024;
size_t oracle_bits_stride(int64_t n_max) { return (size_t)(n_max + 1) * (size_t)((n_max + 1 + 63) / 64); }
bool oracle_lds(int64_t n_max) { return 2 * (size_t)(n_max + 2) * sizeof(double) <= kOracleLdsMax; }
}  // namespace

extern "C" {

int rq_oracle_workspace_size(int32_t n_inst, int64_t n_max, size_t* bytes)
{
    if (!bytes || n_inst < 0 || n_max < 0 || n_max > 1000000) return RQ_EINVAL;
    size_t b = align_up((size_t)n_inst * oracle_bits_stride(n_max) * sizeof(uint64_t), 256);
    if (!oracle_lds(n_max)) b += (size_t)n_inst * 2 * (size_t)(n_max + 2) * sizeof(double);
    *bytes = std::max<size_t>(b, 256);
    return RQ_OK;
}

int rq_oracle_dp(const double* w, const int64_t* w_off, const double* q, const double* s,
                 int32_t n_inst, int64_t n_max, double* cost, int32_t* events, int32_t* ranks,
                 const int64_t* out_off, void* workspace, size_t workspace_bytes, void* hip_stream)
{
    if (n_inst < 0) return RQ_EINVAL;
    if (n_inst == 0) return RQ_OK;
    if (!w || !w_off || !q || !s || !cost || !events || !ranks || !out_off || !workspace) return RQ_EINVAL;
    size_t need = 0;
    const int rc = rq_oracle_workspace_size(n_inst, n_max, &need);
    if (rc != RQ_OK) return rc;
    if (workspace_bytes < need) return RQ_EINVAL;
    OracleArgs a{};
    a.w = w;
    a.w_off = w_off;
    a.q = q;
    a.s = s;
    a.n_inst = n_inst;
    a.n_max = n_max;
    a.cost = cost;
    a.events = events;
    a.ranks = ranks;
    a.out_off = out_off;
    a.bits = (uint64_t*)workspace;
    a.bits_stride = (int64_t)oracle_bits_stride(n_max);
    a.gcol = (double*)((char*)workspace +
                       align_up((size_t)n_inst * oracle_bits_stride(n_max) * sizeof(uint64_t), 256));
    hipStream_t st = (hipStream_t)hip_stream;
    TimedLaunch tl(K_REPLAY, st);
    return rq_launch_oracle_dp(a, oracle_lds(n_max), st) == hipSuccess ? RQ_OK : RQ_EHIP;
}

int rq_rank_table(const double* t, const int64_t* src, const int32_t* sink_col, int64_t n_rows,
                  int32_t n_cols, int64_t src_id, int32_t fill, int64_t n_t, double* table,
                  double* index, int32_t* err, void* hip_stream)
{
    if (!t || !src || !sink_col || !table || !index || !err) return RQ_EINVAL;
    if (n_rows < 1 || n_cols < 1 || n_t < 1 || n_t > n_rows) return RQ_EINVAL;
    RankTableArgs a{};
    a.t = t;
    a.src = src;
    a.col = sink_col;
    a.n_rows = n_rows;
    a.n_cols = n_cols;
    a.src_id = src_id;
    a.fill = fill ? 1 : 0;
    a.n_t = n_t;
    a.table = table;
    a.index = index;
    a.err = err;
    hipStream_t st = (hipStream_t)hip_stream;
    TimedLaunch tl(K_REPLAY, st);
    return rq_launch_rank_table(a, st) == hipSuccess ? RQ_OK : RQ_EHIP;
}

int rq_u_int(const double* table, const double* index, int64_t n_t, int32_t n_cols,
             const int32_t* fcol, const double* wts, int32_t n_f, double end_time, double* out,
             void* workspace, size_t workspace_bytes, void* hip_stream)
{
    if (!table || !index || !out || !workspace || n_t < 1 || n_cols < 1 || n_f < 0) return RQ_EINVAL;
    if (n_f > 0 && (!fcol || !wts)) return RQ_EINVAL;
    if (workspace_bytes < (size_t)n_t * sizeof(double)) return RQ_EINVAL;
    UIntArgs a{};
    a.table = table;
    a.index = index;
    a.n_t = n_t;
    a.n_cols = n_cols;
    a.fcol = fcol;
    a.wts = wts;
    a.n_f = n_f;
    a.end = end_time;
    a.x = (double*)workspace;
    a.out = out;
    hipStream_t st = (hipStream_t)hip_stream;
    TimedLaunch tl(K_SCAN, st);
    return rq_launch_u_int(a, st) == hipSuccess ? RQ_OK : RQ_EHIP;
}

}  // extern "C"

// ============================================================================
// event-log export (State.get_dataframe at batch scale)
// ============================================================================
extern "C" {

int rq_log_rows(rq_graph_t g, const int32_t* ev_src, const int64_t* counts, int64_t n_rep,
                int64_t ev_cap, int64_t* row_off, void* hip_stream)
{
    if (!g || !ev_src || !counts || !row_off || n_rep < 1 || ev_cap < 1) return RQ_EINVAL;
    LogArgs a{};
    a.ev_src = ev_src;
    a.counts = counts;
    a.n_rep = n_rep;
    a.ev_cap = ev_cap;
    a.csr_ptr = g->d_csr_ptr.p;
    a.n_str = g->n_str;
    a.row_off = row_off;
    hipStream_t st = (hipStream_t)hip_stream;
    TimedLaunch tl(K_REPLAY, st);
    return rq_launch_log_rows(a, st) == hipSuccess ? RQ_OK : RQ_EHIP;
}

int rq_log_expand(rq_graph_t g, const double* ev_t, const int32_t* ev_src, const int64_t* counts,
                  int64_t n_rep, int64_t ev_cap, const int64_t* row_off, int64_t* event_id,
                  double* time_delta, int64_t* src_id, double* t, int64_t* sink_id,
                  void* hip_stream)
{
    if (!g || !ev_t || !ev_src || !counts || !row_off || n_rep < 1 || ev_cap < 1) return RQ_EINVAL;
    if (!event_id || !time_delta || !src_id || !t || !sink_id) return RQ_EINVAL;
    LogArgs a{};
    a.ev_t = ev_t;
    a.ev_src = ev_src;
    a.counts = counts;
    a.n_rep = n_rep;
    a.ev_cap = ev_cap;
    a.csr_ptr = g->d_csr_ptr.p;
    a.csr_col = g->d_csr_col_el.p;
    a.n_str = g->n_str;
    a.src_ids = g->d_src_id.p;
    a.sink_ids = g->d_sink_ids.p;
    a.start = g->start;
    a.row_off = const_cast<int64_t*>(row_off);
    a.event_id = event_id;
    a.time_delta = time_delta;
    a.src_id = src_id;
    a.t = t;
    a.sink_id = sink_id;
    hipStream_t st = (hipStream_t)hip_stream;
    TimedLaunch tl(K_REPLAY, st);
    return rq_launch_log_expand(a, st) == hipSuccess ? RQ_OK : RQ_EHIP;
}

}  // extern "C"

extern "C" int rq_phase_clock(unsigned long long* host8)
{
    // RQ_PHASE_CLOCK diagnostic builds only: copy out and clear the per-phase
    // s_memtime sums of every rq_sweep_fw wave since the last call
    if (!host8) return RQ_EINVAL;
    for (int q = 0; q < 8; ++q) host8[q] = 0;
    if (!g_clk) return RQ_EUNSUPPORTED;
    if (hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(host8, g_clk, 8 * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemset(g_clk, 0, 8 * sizeof(unsigned long long)) != hipSuccess)
        return RQ_EHIP;
    return RQ_OK;
}
