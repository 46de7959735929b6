/*
 * rq_spec.h -- arithmetic that DEFINES the engine's simulation semantics.
 *
 * Everything in here is evaluated bit-identically by the gfx950 kernels
 * (hipcc) and by the CPU oracle (gcc): only IEEE-754 double +, -, *, /, fused
 * multiply-add (fma(): one rounding on both sides) and integer/bit operations, no
 * other libm function, constant tables from rq_tables.h, and the translation units that include it
 * are compiled with -ffp-contract=off (the pragma below repeats that for
 * clang).  This is what makes "GPU event log == oracle event log, bit for bit"
 * a testable statement even though the GPU has no correctly rounded log/exp.
 *
 *  - rq_uniform53(): the 53-bit [0,1) double built from two 32-bit words, the
 *    same construction numpy's legacy RandomState uses for random_sample()
 *    (reference draws: opt_model.py:329 RandomState(seed); used at :433,
 *    :481, :484, :540).
 *  - rq_log(): argument reduction + minimax polynomial in the classic fdlibm
 *    style (x = 2^k (1+f), Remez series in s = f/(2+f)); rq_exp_t(): table-driven
 *    (2^(j/32) from rq_tables.h, degree-6 Taylor polynomial, no division).  Both
 *    are within 1 ulp of the correctly rounded result over the ranges the engine
 *    uses; the oracle tests pin that against glibc.
 *  - rq_std_exponential(u) = -log(1-u): numpy legacy_standard_exponential.
 *
 * This header is plain C99 so the oracle (C) can include it; the HIP build
 * sees RQ_HD = __host__ __device__.
 */
#ifndef RQ_SPEC_H
#define RQ_SPEC_H

#include <stdint.h>
#include <math.h>
#include "rq_tables.h"

#if defined(__HIPCC__)
#define RQ_HD __host__ __device__ __forceinline__
#define RQ_HD_COLD static __host__ __device__ __attribute__((noinline))
#pragma clang fp contract(off)
#else
#define RQ_HD static inline
#define RQ_HD_COLD static
#endif

RQ_HD uint64_t rq_dbl_bits(double x)
{
    union { double d; uint64_t u; } c;
    c.d = x;
    return c.u;
}

RQ_HD double rq_bits_dbl(uint64_t u)
{
    union { double d; uint64_t u; } c;
    c.u = u;
    return c.d;
}

/* numpy legacy random_sample(): ((a >> 5) * 2^26 + (b >> 6)) / 2^53 */
RQ_HD double rq_uniform53(uint32_t a, uint32_t b)
{
    return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) / 9007199254740992.0;
}

/* Natural log for finite x > 0 (subnormals handled; x <= 0 -> -inf/NaN). */
RQ_HD double rq_log(double x)
{
    const double ln2_hi = 6.93147180369123816490e-01;
    const double ln2_lo = 1.90821492927058770002e-10;
    const double Lg1 = 6.666666666666735130e-01;
    const double Lg2 = 3.999999999940941908e-01;
    const double Lg3 = 2.857142874366239149e-01;
    const double Lg4 = 2.222219843214978396e-01;
    const double Lg5 = 1.818357216161805012e-01;
    const double Lg6 = 1.531383769920937332e-01;
    const double Lg7 = 1.479819860511658591e-01;

    uint64_t ux = rq_dbl_bits(x);
    if (!(x > 0.0)) {
        if (x == 0.0) return rq_bits_dbl(0xfff0000000000000ull);  /* -inf */
        return rq_bits_dbl(0x7ff8000000000000ull);  /* NaN */
    }
    if ((ux >> 52) >= 0x7ffu) return x + x;      /* +inf / NaN */

    int32_t k = 0;
    if ((ux >> 52) == 0) {                       /* subnormal: scale by 2^54 */
        x = x * 18014398509481984.0;
        ux = rq_dbl_bits(x);
        k = -54;
    }
    int32_t hx = (int32_t)(ux >> 32);
    k += (hx >> 20) - 1023;
    hx &= 0x000fffff;
    /* normalise m into [sqrt(2)/2, sqrt(2)) */
    int32_t i = (hx + 0x95f64) & 0x100000;
    uint64_t um = ((uint64_t)(uint32_t)(hx | (i ^ 0x3ff00000)) << 32) | (ux & 0xffffffffu);
    k += (i >> 20);
    double f = rq_bits_dbl(um) - 1.0;
    double dk = (double)k;

    double s = f / (2.0 + f);
    double z = s * s;
    double w = z * z;
    double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
    double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
    double R = t2 + t1;
    double hfsq = 0.5 * f * f;
    if (f == 0.0) return dk * ln2_hi + dk * ln2_lo;
    return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
}

/* e^x, table-driven (no division): x = k ln2/32 + r with k = round(32 x / ln2) from the
 * 1.5 * 2^52 shift, |r| <= ln2/64; e^x = 2^(k>>5) * s_j * (1 + tail_j) * e^r with
 * s_j = 2^(j/32) (j = k & 31, rq_tables.h) and e^r - 1 = r + r^2 (1/2 + r/6 + r^2/24 +
 * r^3/120 + r^4/720) (truncation < 2^-58).  Products go through fma (one rounding,
 * identical on gfx950 and in C's fma()).  `adj` is added to the scale's bits (the
 * out-of-range path pre-scales by 2^+-1000).  `tab` is RQ_EXP_TAB_INIT (kernels pass
 * an LDS or __constant__ copy; its words 64..67 are the polynomial's coefficients). */
RQ_HD double rq_exp_core(double x, const uint64_t* tab, uint64_t adj)
{
    const double kd0 = x * RQ_EXP_INVLN2N + 0x1.8p52;
    const uint64_t ki = rq_dbl_bits(kd0);
    const double kd = kd0 - 0x1.8p52;
    double r = fma(kd, -RQ_EXP_LN2HI, x);
    r = fma(kd, -RQ_EXP_LN2LO, r);
    const uint32_t j = (uint32_t)ki & 31u;
    const double tail = rq_bits_dbl(tab[2 * j]);
    const double sc = rq_bits_dbl(tab[2 * j + 1] + (ki << 47) + adj);
    const double r2 = r * r;
    const double c6 = rq_bits_dbl(tab[64]), c24 = rq_bits_dbl(tab[65]);     /* 1/6, 1/24 */
    const double c120 = rq_bits_dbl(tab[66]), c720 = rq_bits_dbl(tab[67]);  /* 1/120, 1/720 */
    const double p = fma(r, fma(r, fma(r, fma(r, c720, c120), c24), c6), 0.5);
    const double tmp = fma(r2, p, r) + tail;
    return fma(sc, tmp, sc);
}

/* NaN -> NaN, x > 709.78 -> +inf, x < -745.14 -> 0; otherwise outside [-708, 709]
 * the scale 2^(k>>5) is applied in two steps (2^+-1000 first) */
RQ_HD_COLD double rq_exp_special(double x, const uint64_t* tab)
{
    if (x != x) return x + x;
    if (x > 709.782712893383973096) return rq_bits_dbl(0x7ff0000000000000ull);
    if (x < -745.13321910194110842) return 0.0;
    if (x < 0.0) return rq_exp_core(x, tab, 1000ull << 52) * rq_bits_dbl((uint64_t)(1023 - 1000) << 52);
    return rq_exp_core(x, tab, (uint64_t)0 - (1000ull << 52)) * rq_bits_dbl((uint64_t)(1023 + 1000) << 52);
}

RQ_HD double rq_exp_t(double x, const uint64_t* tab)
{
    if (!(x >= -708.0 && x <= 709.0)) return rq_exp_special(x, tab);
    return rq_exp_core(x, tab, 0);
}

#if !defined(__HIPCC__)
static const uint64_t rq_exp_tab[RQ_EXP_TAB_N] = RQ_EXP_TAB_INIT;
#endif

/* numpy legacy_standard_exponential: -log(1 - U) */
RQ_HD double rq_std_exponential(double u)
{
    return -rq_log(1.0 - u);
}

#endif /* RQ_SPEC_H */
