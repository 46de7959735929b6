/*
 * rq_oracle_analysis.c -- CPU restatement of the reference's analysis helpers.
 *
 * TEST INFRASTRUCTURE ONLY (see rq_oracle.h): the checker for rq_oracle_dp,
 * rq_rank_table and rq_u_int of librq.so, pinned itself against the
 * reference's outputs in tests/golden/oracle.npz and sweepq.npz.
 *
 *   rqo_oracle_dp    utils.oracle_ranking, utils.py:181-245, literally: the
 *                    full (n+1) x (n+2) J matrix, zero-initialised, last
 *                    column r**2/2 (:213), the backward loop (:215-220), the
 *                    forward policy (:225-234).
 *   rqo_rank_table   utils.rank_of_src_in_df, utils.py:38-56 (steps_to, pivot
 *                    mean, ffill).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "rq_oracle.h"

int rqo_oracle_dp(const double* w, int64_t n, double q, double s, double* cost,
                  int64_t* events, int64_t* ranks)
{
    if (n < 0) return -1;
    const int64_t C = n + 2;
    double* J = (double*)calloc((size_t)(n + 1) * (size_t)C, sizeof(double));
    if (!J) return -4;
    /* J[:, n + 1] = (np.arange(n + 1) ** 2) / 2                       :213 */
    for (int64_t r = 0; r <= n; ++r) J[r * C + n + 1] = (double)(r * r) / 2.0;
    /* for k in range(n, -1, -1): for r in range(min(k + 1, n)):         :215-220 */
    for (int64_t k = n; k >= 0; --k) {
        const int64_t m = k + 1 < n ? k + 1 : n;
        for (int64_t r = 0; r < m; ++r) {
            const double a = 0.5 * q + J[0 * C + k + 1];
            const double b = 0.5 * s * w[k + 1] * (double)((r + 1) * (r + 1)) + J[(r + 1) * C + k + 1];
            J[r * C + k] = b < a ? b : a;   /* Python min(a, b) */
        }
    }
    /* forward pass                                                      :225-234 */
    ranks[0] = 0;
    for (int64_t k = 0; k < n; ++k) {
        const double lhs = 0.5 * q + J[0 * C + k + 1];
        const double rhs = 0.5 * s * w[k + 1] * (double)((ranks[k] + 1) * (ranks[k] + 1)) +
                           J[(ranks[k] + 1) * C + k + 1];
        if (lhs < rhs) {
            events[k] = 1;
            ranks[k + 1] = 0;
        } else {
            events[k] = 0;
            ranks[k + 1] = ranks[k] + 1;
        }
    }
    events[n] = 0;
    *cost = J[0];
    free(J);
    return 0;
}

int rqo_rank_table(const double* t, const int64_t* src, const int32_t* col, int64_t n_rows,
                   int32_t n_cols, int64_t src_id, int32_t fill, int64_t n_t, double* table,
                   double* index)
{
    int64_t* pos = (int64_t*)calloc((size_t)n_cols, sizeof(int64_t));
    int64_t* last = (int64_t*)calloc((size_t)n_cols, sizeof(int64_t));
    double* sum = (double*)calloc((size_t)n_cols, sizeof(double));
    int64_t* cnt = (int64_t*)calloc((size_t)n_cols, sizeof(int64_t));
    double* prev = (double*)malloc((size_t)n_cols * sizeof(double));
    if (!pos || !last || !sum || !cnt || !prev) return -4;
    for (int32_t c = 0; c < n_cols; ++c) prev[c] = NAN;
    int64_t row = -1;
    int rc = 0;
    for (int64_t i = 0; i <= n_rows; ++i) {
        if (i == n_rows || row < 0 || t[i] != t[i - 1]) {
            if (row >= 0) {
                if (row >= n_t) { rc = -2; break; }
                index[row] = t[i - 1];
                for (int32_t c = 0; c < n_cols; ++c) {
                    double v;
                    if (cnt[c]) { v = sum[c] / (double)cnt[c]; prev[c] = v; }
                    else v = fill ? prev[c] : NAN;
                    table[row * n_cols + c] = v;
                    sum[c] = 0.0;
                    cnt[c] = 0;
                }
            }
            if (i == n_rows) break;
            if (row >= 0 && t[i] < t[i - 1]) { rc = -5; break; }
            ++row;
        }
        /* steps_to: pos - cummax(pos where src == src_id)               :43-46 */
        const int32_t c = col[i];
        pos[c] += 1;
        if (src[i] == src_id) last[c] = pos[c];
        sum[c] += (double)(pos[c] - last[c]);
        cnt[c] += 1;
    }
    if (rc == 0 && row + 1 != n_t) rc = -2;
    free(pos); free(last); free(sum); free(cnt); free(prev);
    return rc;
}
