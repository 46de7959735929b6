/*
 * rq_oracle.c -- CPU oracle (TEST INFRASTRUCTURE ONLY, see rq_oracle.h).
 *
 * Compiled with -ffp-contract=off so every product below is rounded before
 * it is added, exactly as numpy evaluates `I_values * I_dt` and then sums.
 */
#include "rq_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "../redqueen_amd/csrc/rq_spec.h"

/* ------------------------------------------------------------------------ */
/* numpy pairwise summation (numpy/_core/src/umath/loops_utils.h.src) and the */
/* 8192-element buffered outer reduction used by np.sum on float64.          */
/* ------------------------------------------------------------------------ */
double rqo_pairwise(const double* a, int64_t n)
{
    if (n < 8) {
        double res = -0.0;
        for (int64_t i = 0; i < n; i++) res += a[i];
        return res;
    }
    if (n <= 128) {
        double r[8];
        int64_t i;
        for (int j = 0; j < 8; j++) r[j] = a[j];
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; j++) r[j] += a[i + j];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; i++) res += a[i];
        return res;
    }
    int64_t n2 = n / 2;
    n2 -= n2 % 8;
    return rqo_pairwise(a, n2) + rqo_pairwise(a + n2, n - n2);
}

double rqo_npsum(const double* a, int64_t n)
{
    double res = 0.0;
    for (int64_t off = 0; off < n; off += 8192) {
        int64_t m = n - off < 8192 ? n - off : 8192;
        res = res + rqo_pairwise(a + off, m);
    }
    return res;
}

/* ------------------------------------------------------------------------ */
/* Appendix-B metrics on a df (utils.py:38-56, :84-121, :170-176)            */
/* ------------------------------------------------------------------------ */
static int cmp_i64(const void* a, const void* b)
{
    int64_t x = *(const int64_t*)a, y = *(const int64_t*)b;
    return (x > y) - (x < y);
}

static const double* g_sort_t;
static int cmp_row_by_t(const void* a, const void* b)
{
    int64_t i = *(const int64_t*)a, j = *(const int64_t*)b;
    double x = g_sort_t[i], y = g_sort_t[j];
    if (x < y) return -1;
    if (x > y) return 1;
    return (i > j) - (i < j);
}

static int64_t count_distinct(int64_t* v, int64_t n)
{
    if (n == 0) return 0;
    qsort(v, (size_t)n, sizeof(int64_t), cmp_i64);
    int64_t c = 1;
    for (int64_t i = 1; i < n; i++) c += v[i] != v[i - 1];
    return c;
}

static int64_t find_col(const int64_t* cols, int64_t S, int64_t key)
{
    int64_t lo = 0, hi = S - 1;
    while (lo <= hi) {
        int64_t mid = (lo + hi) >> 1;
        if (cols[mid] < key) lo = mid + 1;
        else if (cols[mid] > key) hi = mid - 1;
        else return mid;
    }
    return -1;
}

int rqo_metrics_df(const double* t, const int64_t* src, const int64_t* sink,
                   const int64_t* event_id, int64_t n_rows, int64_t src_id,
                   double end_time, const int32_t* Ks, int32_t nK, int32_t row_mode,
                   double* out, int64_t* counts)
{
    if (n_rows <= 0) return -1;
    int rc = -4;
    int64_t* cols = NULL; int64_t* colidx = NULL; double* rank = NULL;
    int64_t* pos = NULL; int64_t* last = NULL; int64_t* order = NULL;
    double* cell = NULL; double* gsum = NULL; int64_t* gcnt = NULL; int64_t* touched = NULL;
    double* rowbuf = NULL; double* tk = NULL; double* mk = NULL; double* ik = NULL;
    double* xs = NULL; int64_t* ids = NULL;

    cols = malloc(sizeof(int64_t) * n_rows);
    colidx = malloc(sizeof(int64_t) * n_rows);
    rank = malloc(sizeof(double) * n_rows);
    order = malloc(sizeof(int64_t) * n_rows);
    if (!cols || !colidx || !rank || !order) goto done;

    /* columns = sorted unique sink ids (pivot_table column order) */
    memcpy(cols, sink, sizeof(int64_t) * n_rows);
    int64_t S = count_distinct(cols, n_rows);
    {
        int64_t w = 1;
        for (int64_t i = 1; i < n_rows; i++)
            if (cols[i] != cols[w - 1]) cols[w++] = cols[i];
    }
    pos = calloc((size_t)S, sizeof(int64_t));
    last = calloc((size_t)S, sizeof(int64_t));
    if (!pos || !last) goto done;

    /* rank per row: groupby(sink).transform(steps_to) -- pos - cummax(own pos) */
    for (int64_t i = 0; i < n_rows; i++) {
        int64_t c = find_col(cols, S, sink[i]);
        colidx[i] = c;
        pos[c] += 1;
        if (src[i] == src_id) last[c] = pos[c];
        rank[i] = (double)(pos[c] - last[c]);
    }

    /* pivot rows = sorted unique t; group rows by t (stable) */
    int sorted = 1;
    for (int64_t i = 0; i < n_rows; i++) order[i] = i;
    for (int64_t i = 1; i < n_rows; i++)
        if (t[i] < t[i - 1]) { sorted = 0; break; }
    if (!sorted) {
        g_sort_t = t;
        qsort(order, (size_t)n_rows, sizeof(int64_t), cmp_row_by_t);
    }

    cell = malloc(sizeof(double) * S);
    gsum = calloc((size_t)S, sizeof(double));
    gcnt = calloc((size_t)S, sizeof(int64_t));
    touched = malloc(sizeof(int64_t) * S);
    rowbuf = malloc(sizeof(double) * S);
    tk = malloc(sizeof(double) * n_rows);
    mk = malloc(sizeof(double) * n_rows);
    ik = malloc(sizeof(double) * n_rows * (nK > 0 ? nK : 1));
    xs = malloc(sizeof(double) * n_rows);
    if (!cell || !gsum || !gcnt || !touched || !rowbuf || !tk || !mk || !ik || !xs) goto done;
    for (int64_t c = 0; c < S; c++) cell[c] = NAN;

    int64_t nt = 0;
    for (int64_t a = 0; a < n_rows;) {
        double tv = t[order[a]];
        int64_t b = a, ntouch = 0;
        while (b < n_rows && t[order[b]] == tv) {
            int64_t r = order[b], c = colidx[r];
            if (gcnt[c] == 0) touched[ntouch++] = c;
            gsum[c] += rank[r];
            gcnt[c] += 1;
            b++;
        }
        for (int64_t q = 0; q < ntouch; q++) {
            int64_t c = touched[q];
            cell[c] = gsum[c] / (double)gcnt[c];  /* pivot_table mean of duplicates */
            gsum[c] = 0.0;
            gcnt[c] = 0;
        }
        /* ffill is implicit: cell[] keeps the last value per column */
        int64_t valid = 0;
        for (int64_t c = 0; c < S; c++) {
            int nan = cell[c] != cell[c];
            rowbuf[c] = nan ? 0.0 : cell[c];
            valid += !nan;
        }
        double rs;
        if (row_mode == 0) rs = rqo_npsum(rowbuf, S);
        else { rs = 0.0; for (int64_t c = 0; c < S; c++) rs += rowbuf[c]; }
        mk[nt] = rs / (double)valid;
        for (int32_t k = 0; k < nK; k++) {
            double thr = (double)(Ks[k] - 1);
            int64_t le = 0;
            for (int64_t c = 0; c < S; c++) le += (cell[c] <= thr);
            ik[(int64_t)k * n_rows + nt] = (double)le / (double)S;
        }
        tk[nt] = tv;
        nt++;
        a = b;
    }

    /* dt = diff(concat(index, [end_time])) and the np.sum's */
    for (int32_t k = 0; k < nK; k++) {
        for (int64_t r = 0; r < nt; r++) {
            double dt = (r + 1 < nt ? tk[r + 1] : end_time) - tk[r];
            xs[r] = ik[(int64_t)k * n_rows + r] * dt;
        }
        out[k] = rqo_npsum(xs, nt);
    }
    for (int64_t r = 0; r < nt; r++) {
        double dt = (r + 1 < nt ? tk[r + 1] : end_time) - tk[r];
        xs[r] = mk[r] * dt;
    }
    out[nK] = rqo_npsum(xs, nt);
    for (int64_t r = 0; r < nt; r++) {
        double dt = (r + 1 < nt ? tk[r + 1] : end_time) - tk[r];
        xs[r] = (mk[r] * mk[r]) * dt;
    }
    out[nK + 1] = rqo_npsum(xs, nt);

    if (counts) {
        int64_t n_own = 0, n_world = 0;
        if (event_id) {
            ids = malloc(sizeof(int64_t) * n_rows);
            if (!ids) goto done;
            for (int64_t i = 0; i < n_rows; i++) if (src[i] == src_id) ids[n_own++] = event_id[i];
            n_own = count_distinct(ids, n_own);
            for (int64_t i = 0; i < n_rows; i++) if (src[i] != src_id) ids[n_world++] = event_id[i];
            n_world = count_distinct(ids, n_world);
        }
        counts[0] = n_own;
        counts[1] = n_world;
        counts[2] = nt;
        counts[3] = S;
    }
    rc = 0;
done:
    free(cols); free(colidx); free(rank); free(pos); free(last); free(order);
    free(cell); free(gsum); free(gcnt); free(touched); free(rowbuf);
    free(tk); free(mk); free(ik); free(xs); free(ids);
    return rc;
}

/* ------------------------------------------------------------------------ */
/* numpy legacy RandomState: MT19937 init_genrand seeding + random_sample     */
/* ------------------------------------------------------------------------ */
void rqo_mt_seed(rqo_mt* s, uint32_t seed)
{
    s->mt[0] = seed;
    for (int i = 1; i < 624; i++)
        s->mt[i] = 1812433253u * (s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) + (uint32_t)i;
    s->pos = 624;
}

static void mt_twist(rqo_mt* s)
{
    for (int i = 0; i < 624; i++) {
        uint32_t y = (s->mt[i] & 0x80000000u) | (s->mt[(i + 1) % 624] & 0x7fffffffu);
        uint32_t v = s->mt[(i + 397) % 624] ^ (y >> 1);
        if (y & 1u) v ^= 0x9908b0dfu;
        s->mt[i] = v;
    }
    s->pos = 0;
}

uint32_t rqo_mt_next32(rqo_mt* s)
{
    if (s->pos >= 624) mt_twist(s);
    uint32_t y = s->mt[s->pos++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

double rqo_mt_double(rqo_mt* s)
{
    uint32_t a = rqo_mt_next32(s);
    uint32_t b = rqo_mt_next32(s);
    return rq_uniform53(a, b);
}

double rqo_mt_exponential(rqo_mt* s, double scale)
{
    return scale * -log(1.0 - rqo_mt_double(s));
}

static double loggam(double x)
{
    static const double a[10] = {
        8.333333333333333e-02, -2.777777777777778e-03, 7.936507936507937e-04,
        -5.952380952380952e-04, 8.417508417508418e-04, -1.917526917526918e-03,
        6.410256410256410e-03, -2.955065359477124e-02, 1.796443723688307e-01,
        -1.39243221690590e+00};
    if (x == 1.0 || x == 2.0) return 0.0;
    int64_t n = x < 7.0 ? (int64_t)(7 - x) : 0;
    double x0 = x + (double)n;
    double x2 = (1.0 / x0) * (1.0 / x0);
    double lg2pi = 1.8378770664093453e+00;
    double gl0 = a[9];
    for (int k = 8; k >= 0; k--) {
        gl0 *= x2;
        gl0 += a[k];
    }
    double gl = gl0 / x0 + 0.5 * lg2pi + (x0 - 0.5) * log(x0) - x0;
    if (x < 7.0) {
        for (int64_t k = 1; k <= n; k++) {
            gl -= log(x0 - 1.0);
            x0 -= 1.0;
        }
    }
    return gl;
}

int64_t rqo_mt_poisson(rqo_mt* s, double lam)
{
    if (lam >= 10) {  /* PTRS, Hormann 1993 */
        double slam = sqrt(lam), loglam = log(lam);
        double b = 0.931 + 2.53 * slam;
        double a = -0.059 + 0.02483 * b;
        double invalpha = 1.1239 + 1.1328 / (b - 3.4);
        double vr = 0.9277 - 3.6224 / (b - 2);
        for (;;) {
            double U = rqo_mt_double(s) - 0.5;
            double V = rqo_mt_double(s);
            double us = 0.5 - fabs(U);
            int64_t k = (int64_t)floor((2 * a / us + b) * U + lam + 0.43);
            if ((us >= 0.07) && (V <= vr)) return k;
            if ((k < 0) || ((us < 0.013) && (V > us))) continue;
            if ((log(V) + log(invalpha) - log(a / (us * us) + b)) <=
                (-lam + (double)k * loglam - loggam((double)k + 1)))
                return k;
        }
    }
    if (lam == 0) return 0;
    double enlam = exp(-lam), prod = 1.0;
    int64_t X = 0;
    for (;;) {
        prod *= rqo_mt_double(s);
        if (prod > enlam) X += 1;
        else return X;
    }
}

void rqo_mt_draws(uint32_t seed, int32_t kind, double p, double q, int64_t n, double* out)
{
    rqo_mt s;
    rqo_mt_seed(&s, seed);
    for (int64_t i = 0; i < n; i++) {
        if (kind == 0) out[i] = rqo_mt_double(&s);
        else if (kind == 1) out[i] = rqo_mt_exponential(&s, p);
        else if (kind == 2) out[i] = (double)rqo_mt_poisson(&s, p);
        else out[i] = p + (q - p) * rqo_mt_double(&s);
    }
}

/* ------------------------------------------------------------------------ */
/* Philox4x32-10 (Salmon et al., SC'11; Random123 constants)                */
/* ------------------------------------------------------------------------ */
void rqo_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4])
{
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
    uint32_t k0 = key[0], k1 = key[1];
    for (int r = 0; r < 10; r++) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        uint32_t n1 = (uint32_t)p1;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        uint32_t n3 = (uint32_t)p0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

uint32_t rqo_kind_salt(int32_t kind) { return 0x52510000u | (uint32_t)kind; }

/* the engine's d-th uniform of stream (seed, salt) */
double rqo_philox_uniform(uint32_t seed, uint32_t salt, uint64_t d)
{
    uint64_t call = d >> 1;
    uint32_t ctr[4] = {(uint32_t)call, (uint32_t)(call >> 32), 0u, 0u};
    uint32_t key[2] = {seed, salt};
    uint32_t w[4];
    rqo_philox4x32_10(ctr, key, w);
    return (d & 1) ? rq_uniform53(w[2], w[3]) : rq_uniform53(w[0], w[1]);
}

/* ------------------------------------------------------------------------ */
/* growable arrays                                                           */
/* ------------------------------------------------------------------------ */
typedef struct { double* v; int64_t n, cap; } dvec;
static int dvec_push(dvec* a, double x)
{
    if (a->n == a->cap) {
        int64_t nc = a->cap ? a->cap * 2 : 64;
        double* nv = realloc(a->v, sizeof(double) * nc);
        if (!nv) return -1;
        a->v = nv;
        a->cap = nc;
    }
    a->v[a->n++] = x;
    return 0;
}

static int sinks_of(const rqo_scenario* sc, int64_t sid, int64_t* outv)
{
    int n = 0;
    for (int64_t e = 0; e < sc->n_edges; e++)
        if (sc->edge_src[e] == sid) outv[n++] = sc->edge_sink[e];
    return n;
}

static int cmp_dbl(const void* a, const void* b)
{
    double x = *(const double*)a, y = *(const double*)b;
    return (x > y) - (x < y);
}

static int64_t bisect_right(const double* a, int64_t n, double x)
{
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        int64_t mid = (lo + hi) >> 1;
        if (x < a[mid]) hi = mid;
        else lo = mid + 1;
    }
    return lo;
}

/* ------------------------------------------------------------------------ */
/* Reference-exact Manager.run_dynamic (MT19937 streams)                      */
/* ------------------------------------------------------------------------ */
typedef struct {
    const rqo_source* s;
    int dynamic;
    rqo_mt rs;
    double last_self, t_delta, start_time, end_time;
    int64_t* sinks; int n_sinks;         /* edge-list sinks of this source   */
    dvec times;                          /* static: get_all_times()          */
    dvec prev;                           /* Hawkes prev_excitations          */
    /* Opt */
    int opt_init; int64_t n_fol; int64_t* fol; int64_t* trk; double* w; double old_rate;
    /* OptPWSignificance: old_ranks, sqrt(s_pw / q) [n_fol][S], pw_intensity [S] */
    int64_t* old; double* sq; double* pw; int err;
} refsrc;

static void vexp_libm(const double* x, int64_t n, double* out)
{
    for (int64_t i = 0; i < n; i++) out[i] = exp(x[i]);
}

static double hawkes_rate(refsrc* b, double t, rqo_vexp_fn vexp, dvec* tmp, dvec* tmp2)
{
    tmp->n = 0;
    for (int64_t i = 0; i < b->prev.n; i++) {
        double s = b->prev.v[i];
        if (s <= t) dvec_push(tmp, b->s->p2 * -1.0 * (t - s));
    }
    while (tmp2->cap < tmp->n + 1) dvec_push(tmp2, 0.0);
    vexp(tmp->v, tmp->n, tmp2->v);
    double sum = 0.0;
    for (int64_t i = 0; i < tmp->n; i++) sum = sum + tmp2->v[i];
    return b->s->p0 + b->s->p1 * sum;
}

typedef struct { double cur_time; int64_t src_id; const int64_t* sinks; int n_sinks; } refevent;

/* returns 1 and sets *out if the interval changed, 0 for None */
static int ref_next_interval(refsrc* b, const refevent* ev, rqo_vexp_fn vexp, int dot_fma,
                             dvec* tmp, dvec* tmp2, double* out)
{
    const rqo_source* s = b->s;
    double cur = ev ? ev->cur_time : b->start_time;
    int own = ev == NULL || ev->src_id == s->src_id;
    switch (s->kind) {
    case RQO_POISSON:
        if (own) { *out = rqo_mt_exponential(&b->rs, 1.0 / s->p0); return 1; }
        return 0;
    case RQO_HAWKES:
        if (own) {
            double t = cur;
            double bound = hawkes_rate(b, t, vexp, tmp, tmp2);
            double td;
            for (;;) {
                td = rqo_mt_exponential(&b->rs, 1.0 / bound);
                double u = rqo_mt_double(&b->rs);
                if (u < hawkes_rate(b, t + td, vexp, tmp, tmp2) / bound) break;
                t += td;
            }
            dvec_push(&b->prev, t + td);
            *out = t + td - cur;
            return 1;
        }
        return 0;
    case RQO_OPT: {
        if (!b->opt_init) {
            b->opt_init = 1;
            for (int64_t i = 0; i < b->n_fol; i++) b->trk[i] = 0;
            for (int64_t i = 0; i < b->n_fol; i++) b->w[i] = sqrt(s->a[i] / s->p0);
        }
        /* state.apply_event(event): tracked ranks (opt_model.py:70-76) */
        if (ev) {
            if (ev->src_id == s->src_id) {
                for (int64_t i = 0; i < b->n_fol; i++) b->trk[i] = 0;
            } else {
                for (int k = 0; k < ev->n_sinks; k++)
                    for (int64_t i = 0; i < b->n_fol; i++)
                        if (b->fol[i] == ev->sinks[k]) { b->trk[i] += 1; break; }
            }
        }
        if (ev == NULL) { b->old_rate = 0.0; *out = 0.0; return 1; }
        if (ev->src_id == s->src_id) { b->old_rate = 0.0; *out = INFINITY; return 1; }
        double nr = 0.0;
        for (int64_t i = 0; i < b->n_fol; i++) {
            double r = (double)b->trk[i];
            nr = dot_fma ? fma(b->w[i], r, nr) : nr + b->w[i] * r;
        }
        double diff = nr - b->old_rate;
        b->old_rate = nr;
        double td_new = rqo_mt_exponential(&b->rs, 1.0 / diff);
        if (b->last_self + b->t_delta > ev->cur_time + td_new) {
            *out = ev->cur_time + td_new - b->last_self;
            return 1;
        }
        return 0;
    }
    case RQO_OPTPW: {
        /* OptPWSignificance.get_next_interval, opt_model.py:580-623 */
        const int64_t S = s->n_arr;
        const double T = s->p1;
        if (!b->opt_init) {
            b->opt_init = 1;
            for (int64_t i = 0; i < b->n_fol; i++) b->trk[i] = 0;
            for (int64_t i = 0; i < b->n_fol * S; i++) b->sq[i] = sqrt(s->a[i] / s->p0);
        }
        if (ev) {   /* state.apply_event (tracked ranks, :70-76) */
            if (ev->src_id == s->src_id) {
                for (int64_t i = 0; i < b->n_fol; i++) b->trk[i] = 0;
            } else {
                for (int k = 0; k < ev->n_sinks; k++)
                    for (int64_t i = 0; i < b->n_fol; i++)
                        if (b->fol[i] == ev->sinks[k]) { b->trk[i] += 1; break; }
            }
        }
        if (ev == NULL || ev->src_id == s->src_id) {   /* :597-605 */
            for (int64_t i = 0; i < b->n_fol; i++) b->old[i] = 0;
            *out = ev == NULL ? 0.0 : INFINITY;
            return 1;
        }
        /* pw_intensity = (sqrt(s_pw / q) * rank_diff[:, None]).sum(0)   :613-614 */
        for (int64_t k = 0; k < S; k++) {
            double acc = 0.0;
            for (int64_t i = 0; i < b->n_fol; i++) {
                const double x = b->sq[i * S + k] * (double)(b->trk[i] - b->old[i]);
                acc = i == 0 ? x : acc + x;
            }
            b->pw[k] = acc;
        }
        /* take_one_sample (:560-573) */
        double smax = b->pw[0];
        for (int64_t k = 1; k < S; k++) if (b->pw[k] > smax) smax = b->pw[k];
        if (!(smax > 0.0)) { b->err = 1; return 0; }   /* reference: int(nan) ValueError */
        const double phase = fmod(ev->cur_time, T);
        double ns = 0.0;
        for (;;) {
            ns += rqo_mt_exponential(&b->rs, 1.0 / smax);
            const int64_t idx = (int64_t)(((double)S * fmod(ns + phase, T)) / T);
            if (idx < 0 || idx >= S) { b->err = 1; return 0; }   /* IndexError */
            if (rqo_mt_double(&b->rs) < b->pw[idx] / smax) break;
        }
        for (int64_t i = 0; i < b->n_fol; i++) b->old[i] = b->trk[i];
        if (b->last_self + b->t_delta > ev->cur_time + ns) {
            *out = ev->cur_time + ns - b->last_self;
            return 1;
        }
        return 0;
    }
    default:
        return 0;
    }
}

static double ref_next_event_time(refsrc* b, const refevent* ev, rqo_vexp_fn vexp, int dot_fma,
                                  dvec* tmp, dvec* tmp2)
{
    double cur = ev ? ev->cur_time : b->start_time;
    if (ev == NULL || ev->src_id == b->s->src_id) b->last_self = cur;
    double td;
    if (ref_next_interval(b, ev, vexp, dot_fma, tmp, tmp2, &td)) b->t_delta = td;
    double ret = b->last_self + b->t_delta - cur;
    if (ret < 0) ret = 0.0;
    return ret;
}

typedef struct { double t; int64_t src; } tsrc;
static int cmp_tsrc(const void* a, const void* b)
{
    const tsrc* x = a; const tsrc* y = b;
    if (x->t < y->t) return -1;
    if (x->t > y->t) return 1;
    return (x->src > y->src) - (x->src < y->src);
}

static int ref_initialize_static(refsrc* b)
{
    const rqo_source* s = b->s;
    double duration = b->end_time - b->start_time;
    if (s->kind == RQO_POISSON2) {
        int64_t n = rqo_mt_poisson(&b->rs, s->p0 * duration);
        double* u = malloc(sizeof(double) * (n + 1));
        if (!u) return -1;
        for (int64_t i = 0; i < n; i++)
            u[i] = b->start_time + (b->end_time - b->start_time) * rqo_mt_double(&b->rs);
        qsort(u, (size_t)n, sizeof(double), cmp_dbl);
        for (int64_t i = 0; i < n; i++) dvec_push(&b->times, u[i]);
        free(u);
    } else if (s->kind == RQO_PWCONST) {
        double mx = s->b[0];
        for (int i = 1; i < s->n_arr; i++) if (s->b[i] > mx) mx = s->b[i];
        int64_t n = rqo_mt_poisson(&b->rs, mx * duration);
        double* u = malloc(sizeof(double) * (n + 1));
        if (!u) return -1;
        for (int64_t i = 0; i < n; i++)
            u[i] = b->start_time + (b->end_time - b->start_time) * rqo_mt_double(&b->rs);
        qsort(u, (size_t)n, sizeof(double), cmp_dbl);
        for (int64_t i = 0; i < n; i++) {
            int64_t idx = bisect_right(s->a, s->n_arr, u[i]) - 1;
            if (idx < 0) idx += s->n_arr;
            if (rqo_mt_double(&b->rs) < s->b[idx] / mx) dvec_push(&b->times, u[i]);
        }
        free(u);
    } else if (s->kind == RQO_REALDATA) {
        for (int i = 0; i < s->n_arr; i++)
            if (s->a[i] >= b->start_time) dvec_push(&b->times, s->a[i]);
    }
    return 0;
}

int rqo_ref_run(const rqo_scenario* sc, rqo_vexp_fn vexp, int32_t dot_fma, rqo_events* ev)
{
    if (!vexp) vexp = vexp_libm;
    int rc = -4;
    int ns = sc->n_sources;
    refsrc* B = calloc((size_t)ns, sizeof(refsrc));
    int64_t* all_sinks = malloc(sizeof(int64_t) * (sc->n_edges + 1) * (ns + 1));
    dvec tmp = {0}, tmp2 = {0};
    tsrc* st = NULL;
    int64_t nst = 0;
    if (!B || !all_sinks) goto done;

    for (int i = 0; i < ns; i++) {
        refsrc* b = &B[i];
        b->s = &sc->sources[i];
        b->dynamic = b->s->kind == RQO_POISSON || b->s->kind == RQO_HAWKES ||
                     b->s->kind == RQO_OPT || b->s->kind == RQO_OPTPW;
        rqo_mt_seed(&b->rs, b->s->seed);
        b->start_time = sc->start_time;
        b->end_time = sc->end_time;
        b->sinks = all_sinks + (int64_t)i * (sc->n_edges + 1);
        b->n_sinks = sinks_of(sc, b->s->src_id, b->sinks);
        if (b->s->kind == RQO_OPT || b->s->kind == RQO_OPTPW) {
            /* followers: sorted(follower_sink_ids), opt_model.py:341 */
            b->n_fol = b->n_sinks;
            b->fol = malloc(sizeof(int64_t) * (b->n_fol + 1));
            b->trk = malloc(sizeof(int64_t) * (b->n_fol + 1));
            b->w = malloc(sizeof(double) * (b->n_fol + 1));
            if (!b->fol || !b->trk || !b->w) goto done;
            memcpy(b->fol, b->sinks, sizeof(int64_t) * b->n_fol);
            qsort(b->fol, (size_t)b->n_fol, sizeof(int64_t), cmp_i64);
            if (b->s->kind == RQO_OPTPW) {
                const int64_t S = b->s->n_arr;
                b->old = malloc(sizeof(int64_t) * (b->n_fol + 1));
                b->sq = malloc(sizeof(double) * (b->n_fol * S + 1));
                b->pw = malloc(sizeof(double) * (S + 1));
                if (!b->old || !b->sq || !b->pw || S < 1) goto done;
            }
        }
        if (!b->dynamic) {
            if (ref_initialize_static(b)) goto done;
            nst += b->times.n;
        }
    }
    st = malloc(sizeof(tsrc) * (nst + 1));
    if (!st) goto done;
    {
        int64_t w = 0;
        for (int i = 0; i < ns; i++)
            if (!B[i].dynamic)
                for (int64_t k = 0; k < B[i].times.n; k++) {
                    st[w].t = B[i].times.v[k];
                    st[w].src = B[i].s->src_id;
                    w++;
                }
        qsort(st, (size_t)nst, sizeof(tsrc), cmp_tsrc);
    }

    {
        double state_time = sc->start_time;
        refevent last, *lastp = NULL;
        int64_t sidx = 0;
        ev->n = 0;
        for (;;) {
            if (sc->max_events >= 0 && ev->n >= sc->max_events) break;
            double td = INFINITY;
            int64_t nsrc = -1;
            int have = 0;
            for (int i = 0; i < ns; i++) {
                if (!B[i].dynamic) continue;
                double r = ref_next_event_time(&B[i], lastp, vexp, dot_fma, &tmp, &tmp2);
                if (B[i].err) { rc = -7; goto done; }
                int64_t id = B[i].s->src_id;
                if (!have || r < td || (r == td && id < nsrc)) { td = r; nsrc = id; have = 1; }
            }
            double cur = state_time, et;
            int64_t esrc;
            if (sidx < nst && cur + td > st[sidx].t) {
                et = st[sidx].t;
                esrc = st[sidx].src;
                sidx++;
            } else {
                et = cur + td;
                esrc = nsrc;
            }
            if (et > sc->end_time) break;
            if (ev->n >= ev->cap) { rc = -2; goto done; }
            ev->t[ev->n] = et;
            ev->time_delta[ev->n] = et - cur;
            ev->src_id[ev->n] = esrc;
            ev->n++;
            state_time += et - cur;
            last.cur_time = et;
            last.src_id = esrc;
            last.sinks = NULL;
            last.n_sinks = 0;
            for (int i = 0; i < ns; i++)
                if (B[i].s->src_id == esrc) { last.sinks = B[i].sinks; last.n_sinks = B[i].n_sinks; }
            if (!last.sinks) last.n_sinks = 0;
            lastp = &last;
        }
    }
    rc = 0;
done:
    if (B) {
        for (int i = 0; i < ns; i++) {
            free(B[i].times.v); free(B[i].prev.v);
            free(B[i].fol); free(B[i].trk); free(B[i].w);
            free(B[i].old); free(B[i].sq); free(B[i].pw);
        }
    }
    free(B); free(all_sinks); free(tmp.v); free(tmp2.v); free(st);
    return rc;
}

/* ------------------------------------------------------------------------ */
/* Engine semantics (the spec the gfx950 kernels follow bit for bit)          */
/* ------------------------------------------------------------------------ */
typedef struct { uint32_t seed, salt; uint64_t d; } pstream;
static double pnext(pstream* p) { return rqo_philox_uniform(p->seed, p->salt, p->d++); }

/* generate the full clean stream of one non-controlled (or Poisson2-controlled) source */
static int engine_stream(const rqo_source* s, uint32_t salt, double start, double end, dvec* out)
{
    pstream p = {s->seed, salt, 0};
    out->n = 0;
    switch (s->kind) {
    case RQO_POISSON:
    case RQO_POISSON2: {
        if (!(s->p0 > 0.0)) return 0;
        double inv = 1.0 / s->p0, t = start;
        for (;;) {
            t = t + rq_std_exponential(pnext(&p)) * inv;
            if (!(t <= end)) return 0;
            if (dvec_push(out, t)) return -1;
        }
    }
    case RQO_HAWKES: {
        double l0 = s->p0, alpha = s->p1, nbeta = -s->p2;
        double tau = start, eta = 0.0;
        for (;;) {
            double B = l0 + eta;
            if (!(B > 0.0)) return 0;
            double inv = 1.0 / B, t = tau;
            for (;;) {
                double x = rq_std_exponential(pnext(&p));
                double v = pnext(&p);
                double tc = t + x * inv;
                if (!(tc <= end)) return 0;
                double decay = rq_exp_t(nbeta * (tc - tau), rq_exp_tab);
                double rate = l0 + eta * decay;
                if (v * B < rate) {   /* engine: division-free thinning test */
                    eta = eta * decay + alpha;
                    tau = tc;
                    if (dvec_push(out, tc)) return -1;
                    break;
                }
                /* engine: refreshed bound after a rejection (lambda only decays) */
                t = tc;
                B = rate;
                inv = 1.0 / rate;
            }
        }
    }
    case RQO_PWCONST: {
        double mx = s->b[0];
        for (int i = 1; i < s->n_arr; i++) if (s->b[i] > mx) mx = s->b[i];
        if (!(mx > 0.0)) return 0;
        double inv = 1.0 / mx, t = start;
        for (;;) {
            t = t + rq_std_exponential(pnext(&p)) * inv;
            if (!(t <= end)) return 0;
            double v = pnext(&p);
            int64_t idx = bisect_right(s->a, s->n_arr, t) - 1;
            if (idx < 0) idx += s->n_arr;
            if (v * mx < s->b[idx])
                if (dvec_push(out, t)) return -1;
        }
    }
    case RQO_REALDATA: {
        for (int i = 0; i < s->n_arr; i++)
            if (s->a[i] >= start && s->a[i] <= end)
                if (dvec_push(out, s->a[i])) return -1;
        if (out->n > 1) qsort(out->v, (size_t)out->n, sizeof(double), cmp_dbl);   /* v may be NULL */
        return 0;
    }
    default:
        return 0;
    }
}

/* engine OptPWSignificance draw for wall event number e (rq_sweep_core.h optpw_sample):
   thinning at smax from the phase t mod T, Philox call (e, iteration) per candidate */
static double optpw_sample(double tt, const double* row, double smax, int64_t S, double T,
                           uint64_t e, uint32_t seed)
{
    if (!(smax > 0.0)) return INFINITY;
    const double inv = 1.0 / smax;
    const double ph = fmod(tt, T);
    double ns = 0.0;
    const uint32_t key[2] = {seed, rqo_kind_salt(RQO_OPTPW) | 0x100u};
    for (uint32_t it = 1; it < (1u << 20); ++it) {
        const uint32_t ctr[4] = {(uint32_t)e, (uint32_t)(e >> 32), it, 0u};
        uint32_t w4[4];
        rqo_philox4x32_10(ctr, key, w4);
        ns = ns + rq_std_exponential(rq_uniform53(w4[0], w4[1])) * inv;
        int64_t idx = (int64_t)(((double)S * fmod(ns + ph, T)) / T);
        idx = idx < S ? idx : S - 1;
        if (rq_uniform53(w4[2], w4[3]) * smax < row[idx]) return tt + ns;
    }
    return INFINITY;
}

/* 1: source j plays its equal-time events after the dynamic sources' (a static source,
   opt_model.py:289-290); source 0 with a RedQueen / OptPWSignificance controller is dynamic */
static int engine_static(const rqo_scenario* sc, int j, int opt)
{
    const rqo_source* s = &sc->sources[j];
    if (j == 0 && opt) return 0;
    return s->kind == RQO_POISSON2 || s->kind == RQO_PWCONST || (s->kind == RQO_REALDATA && !(s->flags & 1u));
}

int rqo_engine_run(const rqo_scenario* sc, rqo_events* ev)
{
    int rc = -4;
    double* pwc = NULL;
    double* pwmax = NULL;
    int ns = sc->n_sources;
    dvec* st = calloc((size_t)ns, sizeof(dvec));
    int64_t* head = calloc((size_t)ns, sizeof(int64_t));
    double* invc = calloc((size_t)ns, sizeof(double));
    int64_t* fol = malloc(sizeof(int64_t) * (sc->n_edges + 1));
    double* w = malloc(sizeof(double) * (sc->n_edges + 1));
    if (!st || !head || !invc || !fol || !w) goto done;

    const rqo_source* ctrl = &sc->sources[0];
    const int optpw = ctrl->kind == RQO_OPTPW;
    int opt = ctrl->kind == RQO_OPT || optpw;   /* a controller that reacts to the wall */
    int64_t nf = 0;
    const int64_t S = optpw ? ctrl->n_arr : 0;
    uint64_t nwall = 0;
    if (optpw) {
        /* engine semantics of OptPWSignificance: pw_j[k] = sum over edges (j, i), i a
           follower, of sqrt(s_pw[i][k] / q), edge-list order; bound max_k pw_j[k] */
        nf = sinks_of(sc, ctrl->src_id, fol);
        qsort(fol, (size_t)nf, sizeof(int64_t), cmp_i64);
        pwc = calloc((size_t)(ns * S + 1), sizeof(double));
        pwmax = calloc((size_t)ns + 1, sizeof(double));
        if (!pwc || !pwmax || S < 1) goto done;
        for (int j = 1; j < ns; j++) {
            double* row = pwc + (int64_t)j * S;
            for (int64_t e = 0; e < sc->n_edges; e++) {
                if (sc->edge_src[e] != sc->sources[j].src_id) continue;
                for (int64_t i = 0; i < nf; i++)
                    if (fol[i] == sc->edge_sink[e]) {
                        for (int64_t k = 0; k < S; k++) row[k] = row[k] + sqrt(ctrl->a[i * S + k] / ctrl->p0);
                        break;
                    }
            }
            double m = 0.0;
            for (int64_t k = 0; k < S; k++) m = row[k] > m ? row[k] : m;
            pwmax[j] = m;
        }
    } else if (opt) {
        nf = sinks_of(sc, ctrl->src_id, fol);
        qsort(fol, (size_t)nf, sizeof(int64_t), cmp_i64);
        for (int64_t i = 0; i < nf; i++) w[i] = sqrt(ctrl->a[i] / ctrl->p0);
        /* c_j = sum over edges (j, i), i a follower, in edge-list order */
        for (int j = 1; j < ns; j++) {
            double c = 0.0;
            for (int64_t e = 0; e < sc->n_edges; e++) {
                if (sc->edge_src[e] != sc->sources[j].src_id) continue;
                for (int64_t i = 0; i < nf; i++)
                    if (fol[i] == sc->edge_sink[e]) { c = c + w[i]; break; }
            }
            invc[j] = c > 0.0 ? 1.0 / c : 0.0;
        }
    }
    for (int j = 0; j < ns; j++) {
        if (j == 0 && opt) continue;
        uint32_t salt = rqo_kind_salt(sc->sources[j].kind) | (j == 0 ? 0x100u : 0u);
        if (engine_stream(&sc->sources[j], salt, sc->start_time, sc->end_time, &st[j])) goto done;
    }

    {
        pstream po = {ctrl->seed, rqo_kind_salt(RQO_OPT) | 0x100u, 0};
        double opt_next = opt ? sc->start_time : INFINITY;
        double state_time = sc->start_time;   /* State.time, accumulated (opt_model.py:68) */
        ev->n = 0;
        for (;;) {
            if (sc->max_events >= 0 && ev->n >= sc->max_events) break;
            int bj = -1;
            double bt = INFINITY;
            int64_t bid = 0;
            for (int j = 0; j < ns; j++) {
                double tj;
                if (j == 0 && opt) tj = opt_next;
                else tj = head[j] < st[j].n ? st[j].v[head[j]] : INFINITY;
                int64_t id = sc->sources[j].src_id;
                /* ties (opt_model.py:279-281, :289-290): every dynamic source -- the
                   RedQueen controller, Poisson, Hawkes, a dynamic broadcaster's replayed
                   times -- before every static one, src_id order within each class */
                const int cj = engine_static(sc, j, opt), cb = bj >= 0 ? engine_static(sc, bj, opt) : 0;
                const int beats = cj != cb ? cj < cb : id < bid;
                if (tj < bt || (tj == bt && bj >= 0 && beats)) { bt = tj; bj = j; bid = id; }
            }
            if (bj < 0 || !(bt <= sc->end_time)) break;
            if (ev->n >= ev->cap) { rc = -2; goto done; }
            ev->t[ev->n] = bt;
            ev->time_delta[ev->n] = bt - state_time;
            state_time = state_time + ev->time_delta[ev->n];
            ev->src_id[ev->n] = bid;
            ev->n++;
            if (bj == 0 && opt) {
                opt_next = INFINITY;
            } else {
                head[bj]++;
                if (optpw && bj != 0) {
                    double cand = optpw_sample(bt, pwc + (int64_t)bj * S, pwmax[bj], S, ctrl->p1,
                                               nwall++, ctrl->seed);
                    if (cand < opt_next) opt_next = cand;
                } else if (opt && bj != 0) {
                    double x = rq_std_exponential(pnext(&po));
                    double e = invc[bj] > 0.0 ? x * invc[bj] : INFINITY;
                    double cand = bt + e;
                    if (cand < opt_next) opt_next = cand;
                }
            }
        }
    }
    rc = 0;
done:
    if (st) for (int j = 0; j < ns; j++) free(st[j].v);
    free(st); free(head); free(invc); free(fol); free(w); free(pwc); free(pwmax);
    return rc;
}

/* ------------------------------------------------------------------------ */
/* Batched CPU baseline (engine model + Appendix-B metrics, pthreads)         */
/* ------------------------------------------------------------------------ */
double rqo_spec_log(double x) { return rq_log(x); }
double rqo_spec_exp(double x) { return rq_exp_t(x, rq_exp_tab); }

typedef struct {
    const rqo_scenario* sc; int64_t r0, r1; uint32_t seed0; int randomize; const double* rates;
    uint32_t ctrl_off, stride;
    const int32_t* Ks; int32_t nK; double* out; int64_t* counts; int64_t events; int rc;
} batch_job;

static void* batch_worker(void* arg)
{
    batch_job* j = arg;
    const rqo_scenario* sc = j->sc;
    int ns = sc->n_sources;
    rqo_source* srcs = malloc(sizeof(rqo_source) * ns);
    int64_t cap = 1 << 16;
    rqo_events ev = {cap, 0, malloc(sizeof(double) * cap), malloc(sizeof(double) * cap),
                     malloc(sizeof(int64_t) * cap)};
    int64_t* sinkmap_n = calloc((size_t)ns, sizeof(int64_t));
    int64_t** sinkmap = calloc((size_t)ns, sizeof(int64_t*));
    int64_t rcap = 0;
    double* rt = NULL; int64_t* rsrc = NULL; int64_t* rsink = NULL; int64_t* reid = NULL;
    j->rc = -4;
    if (!srcs || !ev.t || !ev.time_delta || !ev.src_id || !sinkmap_n || !sinkmap) goto out;
    for (int i = 0; i < ns; i++) {
        sinkmap[i] = malloc(sizeof(int64_t) * (sc->n_edges + 1));
        if (!sinkmap[i]) goto out;
        sinkmap_n[i] = sinks_of(sc, sc->sources[i].src_id, sinkmap[i]);
    }
    for (int64_t r = j->r0; r < j->r1; r++) {
        uint32_t u = j->seed0 + j->stride * (uint32_t)r;
        memcpy(srcs, sc->sources, sizeof(rqo_source) * ns);
        srcs[0].seed = u + j->ctrl_off;
        if (j->rates) srcs[0].p0 = j->rates[r];
        if (j->randomize)
            for (int i = 1; i < ns; i++) srcs[i].seed = u + 99u * (uint32_t)(i - 1);
        rqo_scenario s2 = *sc;
        s2.sources = srcs;
        for (;;) {
            int e = rqo_engine_run(&s2, &ev);
            if (e == 0) break;
            if (e != -2) goto out;
            cap *= 2;
            free(ev.t); free(ev.time_delta); free(ev.src_id);
            ev.cap = cap;
            ev.t = malloc(sizeof(double) * cap);
            ev.time_delta = malloc(sizeof(double) * cap);
            ev.src_id = malloc(sizeof(int64_t) * cap);
            if (!ev.t || !ev.time_delta || !ev.src_id) goto out;
        }
        int64_t nrow = 0;
        for (int64_t e = 0; e < ev.n; e++)
            for (int i = 0; i < ns; i++)
                if (sc->sources[i].src_id == ev.src_id[e]) { nrow += sinkmap_n[i]; break; }
        if (nrow > rcap) {
            rcap = nrow * 2;
            free(rt); free(rsrc); free(rsink); free(reid);
            rt = malloc(sizeof(double) * rcap); rsrc = malloc(sizeof(int64_t) * rcap);
            rsink = malloc(sizeof(int64_t) * rcap); reid = malloc(sizeof(int64_t) * rcap);
            if (!rt || !rsrc || !rsink || !reid) goto out;
        }
        int64_t w = 0, nposts = 0, nworld = 0;
        for (int64_t e = 0; e < ev.n; e++)
            for (int i = 0; i < ns; i++)
                if (sc->sources[i].src_id == ev.src_id[e]) {
                    for (int64_t k = 0; k < sinkmap_n[i]; k++) {
                        rt[w] = ev.t[e]; rsrc[w] = ev.src_id[e]; rsink[w] = sinkmap[i][k];
                        reid[w] = 100 + e; w++;
                    }
                    break;
                }
        double* o = j->out + r * (j->nK + 2);
        int64_t cnt[4] = {0, 0, 0, 0};
        if (nrow > 0) {
            if (rqo_metrics_df(rt, rsrc, rsink, reid, nrow, sc->sources[0].src_id, sc->end_time,
                               j->Ks, j->nK, 0, o, cnt)) goto out;
        } else {
            for (int k = 0; k < j->nK + 2; k++) o[k] = NAN;
        }
        nposts = cnt[0]; nworld = cnt[1];
        j->counts[r * 3 + 0] = nposts;
        j->counts[r * 3 + 1] = nworld;
        j->counts[r * 3 + 2] = ev.n;
        j->events += ev.n;
    }
    j->rc = 0;
out:
    if (sinkmap) for (int i = 0; i < ns; i++) free(sinkmap[i]);
    free(sinkmap); free(sinkmap_n); free(srcs);
    free(ev.t); free(ev.time_delta); free(ev.src_id);
    free(rt); free(rsrc); free(rsink); free(reid);
    return NULL;
}

int64_t rqo_engine_batch(const rqo_scenario* sc, int64_t n_rep, uint32_t seed0,
                         int32_t randomize, const int32_t* Ks, int32_t nK,
                         int32_t n_threads, const double* ctrl_rates, uint32_t ctrl_seed_offset, uint32_t seed_stride,
                         double* out, int64_t* counts)
{
    if (n_threads < 1) n_threads = 1;
    pthread_t* th = malloc(sizeof(pthread_t) * n_threads);
    batch_job* jobs = calloc((size_t)n_threads, sizeof(batch_job));
    if (!th || !jobs) { free(th); free(jobs); return -4; }
    for (int i = 0; i < n_threads; i++) {
        jobs[i].sc = sc; jobs[i].seed0 = seed0; jobs[i].randomize = randomize;
        jobs[i].Ks = Ks; jobs[i].nK = nK; jobs[i].out = out; jobs[i].counts = counts;
        jobs[i].rates = ctrl_rates;
        jobs[i].ctrl_off = ctrl_seed_offset;
        jobs[i].stride = seed_stride ? seed_stride : 1u;
        jobs[i].r0 = n_rep * i / n_threads;
        jobs[i].r1 = n_rep * (i + 1) / n_threads;
        pthread_create(&th[i], NULL, batch_worker, &jobs[i]);
    }
    int64_t total = 0;
    int rc = 0;
    for (int i = 0; i < n_threads; i++) {
        pthread_join(th[i], NULL);
        total += jobs[i].events;
        if (jobs[i].rc) rc = jobs[i].rc;
    }
    free(th); free(jobs);
    return rc ? rc : total;
}
