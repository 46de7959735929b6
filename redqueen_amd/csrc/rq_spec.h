/*
 * rq_spec.h -- arithmetic that DEFINES the engine's simulation semantics.
 *
 * Everything in here is evaluated bit-identically by the gfx950 kernels
 * (hipcc) and by the CPU oracle (gcc): only IEEE-754 double +, -, *, / and
 * integer/bit operations, no libm, and the translation units that include it
 * are compiled with -ffp-contract=off (the pragma below repeats that for
 * clang).  This is what makes "GPU event log == oracle event log, bit for bit"
 * a testable statement even though the GPU has no correctly rounded log/exp.
 *
 *  - rq_uniform53(): the 53-bit [0,1) double built from two 32-bit words, the
 *    same construction numpy's legacy RandomState uses for random_sample()
 *    (reference draws: opt_model.py:329 RandomState(seed); used at :433,
 *    :481, :484, :540).
 *  - rq_log()/rq_exp(): argument reduction + minimax polynomials in the
 *    classic fdlibm style (log: x = 2^k (1+f), Remez series in s = f/(2+f);
 *    exp: x = k ln2 + r, rational Remez form).  Both are within 1 ulp of the
 *    correctly rounded result over the ranges the engine uses; the oracle
 *    tests pin that against glibc.
 *  - rq_std_exponential(u) = -log(1-u): numpy legacy_standard_exponential.
 *
 * This header is plain C99 so the oracle (C) can include it; the HIP build
 * sees RQ_HD = __host__ __device__.
 */
#ifndef RQ_SPEC_H
#define RQ_SPEC_H

#include <stdint.h>

#if defined(__HIPCC__)
#define RQ_HD __host__ __device__ __forceinline__
#pragma clang fp contract(off)
#else
#define RQ_HD static inline
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

/* e^x for finite x; large negative -> 0, large positive -> +inf. */
RQ_HD double rq_exp(double x)
{
    const double ln2HI = 6.93147180369123816490e-01;
    const double ln2LO = 1.90821492927058770002e-10;
    const double invln2 = 1.44269504088896338700e+00;
    const double P1 = 1.66666666666666019037e-01;
    const double P2 = -2.77777777770155933842e-03;
    const double P3 = 6.61375632143793436117e-05;
    const double P4 = -1.65339022054652515390e-06;
    const double P5 = 4.13813679705723846039e-08;

    if (x != x) return x + x;
    if (x > 709.782712893383973096) return rq_bits_dbl(0x7ff0000000000000ull);
    if (x < -745.13321910194110842) return 0.0;         /* underflow */
    if (x > -3.7252902984e-09 && x < 3.7252902984e-09) return 1.0 + x;

    /* k = round(x / ln2) */
    double kd = x * invln2;
    int32_t k = (int32_t)(kd < 0.0 ? kd - 0.5 : kd + 0.5);
    double hi = x - (double)k * ln2HI;
    double lo = (double)k * ln2LO;
    double r = hi - lo;
    double t = r * r;
    double c = r - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
    double y = 1.0 - ((lo - (r * c) / (2.0 - c)) - hi);

    /* y * 2^k, with a two-step scale so k in [-1074, 1024] stays exact */
    if (k >= -1021) {
        if (k == 1024) return y * 2.0 * rq_bits_dbl((uint64_t)(1023 + 1023) << 52);
        return y * rq_bits_dbl((uint64_t)(k + 1023) << 52);
    }
    return y * rq_bits_dbl((uint64_t)(k + 1000 + 1023) << 52) *
           rq_bits_dbl((uint64_t)(-1000 + 1023) << 52);
}

/* numpy legacy_standard_exponential: -log(1 - U) */
RQ_HD double rq_std_exponential(double u)
{
    return -rq_log(1.0 - u);
}

#endif /* RQ_SPEC_H */
