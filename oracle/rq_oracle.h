/*
 * rq_oracle.h -- CPU oracle for the RedQueen broadcasting hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in redqueen_amd/ links, loads or calls
 * this code; only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg use it, and only as the checker / the timed CPU baseline.
 *
 * What it restates (file:line into the reference, MPI-SWS/RedQueen):
 *   rqo_npsum           numpy's pairwise add.reduce (8192-element chunks)
 *                       used by np.sum in utils.py:98, :114, :121
 *   rqo_metrics_df      utils.rank_of_src_in_df :38-56 + time_in_top_k :84-98
 *                       + average_rank :101-114 + int_r_2 :117-121 +
 *                       num_tweets_of :170-176 / opt_runs.add_perf :41-48
 *   rqo_mt_*            numpy legacy RandomState (MT19937, random_sample,
 *                       exponential, uniform, poisson) behind
 *                       opt_model.py:329, :399-402, :433, :481-484, :540, :651-658
 *   rqo_philox4x32_10   Philox4x32-10 (Random123), the engine's RNG
 *   rqo_ref_run         Manager.run_dynamic opt_model.py:241-314 with the
 *                       broadcasters Poisson :424-433, Poisson2 :381-421,
 *                       Hawkes :458-490, Opt :493-544, PiecewiseConst
 *                       :626-689, RealData :711-750, Broadcaster
 *                       get_next_event_time :351-369, State.apply_event
 *                       :61-83 -- every quirk kept (accumulated state.time,
 *                       static-vs-dynamic tie rule, O(n) Hawkes rate).
 *   rqo_engine_run      the SAME model under the engine's documented
 *                       semantics (DESIGN.md "engine semantics"): Philox
 *                       streams, clean per-source times, O(1) RedQueen
 *                       increments c_j.  The gfx950 kernels must reproduce
 *                       this bit for bit.
 */
#ifndef RQ_ORACLE_H
#define RQ_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    RQO_POISSON = 1,   /* dynamic Poisson      opt_model.py:424 */
    RQO_POISSON2 = 2,  /* static Poisson2      opt_model.py:381 */
    RQO_HAWKES = 3,    /* dynamic Hawkes       opt_model.py:458 */
    RQO_PWCONST = 4,   /* static piecewise     opt_model.py:626 */
    RQO_REALDATA = 5,  /* static fixed times   opt_model.py:711 */
    RQO_OPT = 6,       /* RedQueen controller  opt_model.py:493 */
    RQO_OPTPW = 7      /* OptPWSignificance    opt_model.py:547 */
};

typedef struct {
    int32_t kind;
    int32_t n_arr;      /* PWCONST: #segments; REALDATA: #times; OPT: #followers;
                           OPTPW: #significance segments S */
    int64_t src_id;
    uint32_t seed;
    uint32_t flags;     /* 1: a REALDATA source that replays a DYNAMIC broadcaster's times
                           (rq.h RQ_SRCF_DYNAMIC): ties order it as a dynamic source */
    double p0, p1, p2;  /* POISSON*: rate; HAWKES: l_0, alpha, beta; OPT: q; OPTPW: q, period */
    const double* a;    /* PWCONST change_times; REALDATA times; OPT s (sorted followers);
                           OPTPW s_pw [sorted followers][S] */
    const double* b;    /* PWCONST rates */
} rqo_source;

typedef struct {
    int32_t n_sources;
    const rqo_source* sources;   /* manager order: [controlled] + other_sources */
    int32_t n_sinks;
    const int64_t* sink_ids;
    int64_t n_edges;
    const int64_t* edge_src;
    const int64_t* edge_sink;
    double start_time, end_time;
    int64_t max_events;          /* < 0: unbounded */
} rqo_scenario;

typedef struct {
    int64_t cap;
    int64_t n;            /* out */
    double* t;            /* event.cur_time                     */
    double* time_delta;   /* event.time_delta                   */
    int64_t* src_id;      /* event.src_id                       */
} rqo_events;

/* vector exp hook: out[i] = exp(x[i]) for i < n (NULL -> libm exp loop) */
typedef void (*rqo_vexp_fn)(const double* x, int64_t n, double* out);

double rqo_npsum(const double* x, int64_t n);
double rqo_pairwise(const double* x, int64_t n);

/* Metrics on a reference-layout event dataframe (rows in df order).
 * out[0..nK) top_k, out[nK] avg_rank, out[nK+1] r_2 ; counts[0] = num own
 * events (distinct event_id, src == src_id), counts[1] = world events,
 * counts[2] = number of pivot rows, counts[3] = number of sink columns.
 * row_mode: 0 = pairwise over columns, 1 = sequential over columns. */
int rqo_metrics_df(const double* t, const int64_t* src, const int64_t* sink,
                   const int64_t* event_id, int64_t n_rows, int64_t src_id,
                   double end_time, const int32_t* Ks, int32_t nK, int32_t row_mode,
                   double* out, int64_t* counts);

/* numpy legacy RandomState */
typedef struct { uint32_t mt[624]; int32_t pos; } rqo_mt;
void rqo_mt_seed(rqo_mt* s, uint32_t seed);
uint32_t rqo_mt_next32(rqo_mt* s);
double rqo_mt_double(rqo_mt* s);
double rqo_mt_exponential(rqo_mt* s, double scale);
int64_t rqo_mt_poisson(rqo_mt* s, double lam);
/* draw-KAT helper: kind 0 double, 1 exponential(p), 2 poisson(p), 3 uniform(p, q) */
void rqo_mt_draws(uint32_t seed, int32_t kind, double p, double q, int64_t n, double* out);

void rqo_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
double rqo_philox_uniform(uint32_t seed, uint32_t salt, uint64_t draw);

/* dot flavour for the RedQueen rate (numpy .dot -> BLAS ddot): 0 mul+add, 1 fma */
int rqo_ref_run(const rqo_scenario* sc, rqo_vexp_fn vexp, int32_t dot_fma, rqo_events* ev);
int rqo_engine_run(const rqo_scenario* sc, rqo_events* ev);

/* kind salt used as Philox key[1] for a source of the given kind */
uint32_t rqo_kind_salt(int32_t kind);

/* Batched CPU baseline: n_rep replicas of the engine model, replica r uses
 * world seeds (u_r + 99*idx) and controlled seed u_r where u_r = seed0 + stride * r
 * (seed_stride 0 = 1),
 * metrics with Appendix-B semantics.  out: [n_rep][nK+2], counts [n_rep][3]
 * (posts, world, events).  n_threads pthreads.  ctrl_rates (may be NULL):
 * per-replica rate of a Poisson2 controlled source (sources[0] must be
 * POISSON2).  Returns total events. */
int64_t rqo_engine_batch(const rqo_scenario* sc, int64_t n_rep, uint32_t seed0,
                         int32_t randomize, const int32_t* Ks, int32_t nK,
                         int32_t n_threads, const double* ctrl_rates, uint32_t ctrl_seed_offset, uint32_t seed_stride,
                         double* out, int64_t* counts);

/* rq_oracle_analysis.c: utils.oracle_ranking (utils.py:181-245) on w[0..n+2)
 * = np.diff([0, 0, event_times..., end_time]); events/ranks [n+1]. */
int rqo_oracle_dp(const double* w, int64_t n, double q, double s, double* cost,
                  int64_t* events, int64_t* ranks);
/* utils.rank_of_src_in_df (utils.py:38-56): table [n_t][n_cols], index [n_t] */
int rqo_rank_table(const double* t, const int64_t* src, const int32_t* col, int64_t n_rows,
                   int32_t n_cols, int64_t src_id, int32_t fill, int64_t n_t, double* table,
                   double* index);

/* the engine's arithmetic spec (redqueen_amd/csrc/rq_spec.h), exported for tests */
double rqo_spec_log(double x);
double rqo_spec_exp(double x);

#ifdef __cplusplus
}
#endif
#endif
