// Microbenchmark: SIMD cycles per wave64 call of the arrival generator's pieces on
// gfx950 (Philox4x32-10, rq_uniform53, rq_log, rq_exp, an f64 division) -- where a
// refill pass of the fused sweep spends its VALU time.  Independent chains per lane
// (8 in flight) so the number is issue cost, not latency.
// build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -I../../redqueen_amd/csrc gen_cost.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "rq_spec.h"
#include "rq_device.h"

using namespace rq;

static __constant__ uint64_t etab_c[RQ_EXP_TAB_N] = RQ_EXP_TAB_INIT;

/* fdlibm exp (the round-1/2 engine's rq_exp), for comparison */
RQ_HD double rq_exp_fdlibm(double x)
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


template <int V>
__global__ __launch_bounds__(256) void k(double* out, int iters)
{
    constexpr int C = 8;
    __shared__ uint64_t etab_l[RQ_EXP_TAB_N];
    if (threadIdx.x < RQ_EXP_TAB_N) etab_l[threadIdx.x] = etab_c[threadIdx.x];
    __syncthreads();
    double x[C], acc = 0.0;
    uint32_t s[C];
#pragma unroll
    for (int q = 0; q < C; ++q) {
        x[q] = 0.25 + 1e-7 * (threadIdx.x + 64 * q);
        s[q] = threadIdx.x * 8 + q;
    }
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int q = 0; q < C; ++q) {
            if (V == 0) {   // Philox4x32-10 + two 53-bit uniforms
                uint32_t c[4] = {s[q], (uint32_t)i, 0u, 0u};
                philox4x32_10(c, 0x1234u, 0x5678u);
                x[q] += rq_uniform53(c[0], c[1]) + rq_uniform53(c[2], c[3]);
                s[q] = c[3];
            } else if (V == 7) {   // Philox4x32-10 with a per-lane key (the generator's (seed, salt))
                uint32_t c[4] = {(uint32_t)i, 0u, 0u, 0u};
                philox4x32_10(c, s[q], 0x52510000u | (threadIdx.x & 7));
                x[q] += rq_uniform53(c[0], c[1]) + rq_uniform53(c[2], c[3]);
                s[q] = c[3];
            } else if (V == 1) {   // -log(1 - u)
                x[q] = rq_std_exponential(x[q] * 0.5);
            } else if (V == 2) {   // exp of a negative argument (fdlibm)
                x[q] = rq_exp_fdlibm(-x[q] - 0.5);
            } else if (V == 5) {   // table exp, __constant__ table
                x[q] = rq_exp_t(-x[q] - 0.5, etab_c);
            } else if (V == 6) {   // table exp, LDS table
                x[q] = rq_exp_t(-x[q] - 0.5, etab_l);
            } else if (V == 3) {   // f64 division
                x[q] = 1.0 / (x[q] + 1.5);
            } else {               // an f64 multiply-add (reference op)
                x[q] = x[q] * 0.999 + 0.001;
            }
        }
    }
#pragma unroll
    for (int q = 0; q < C; ++q) acc += x[q];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main()
{
    int dev = 0, cus = 0, clk = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);   // kHz
    const int blocks = cus * 4, threads = 256, iters = 400;   // 4 waves per SIMD
    double* out;
    hipMalloc(&out, sizeof(double) * blocks * threads);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const char* names[] = {"philox4x32-10 + 2 uniform53", "rq_std_exponential (rq_log)", "rq_exp (fdlibm)",
                           "f64 division", "f64 mul+add", "rq_exp_t (__constant__ table)", "rq_exp_t (LDS table)",
                           "philox4x32-10, per-lane key"};
    for (int v = 0; v < 8; ++v) {
        float best = 1e30f;
        for (int rep = 0; rep < 3; ++rep) {
            hipEventRecord(a);
            switch (v) {
            case 0: hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(threads), 0, 0, out, iters); break;
            case 1: hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(threads), 0, 0, out, iters); break;
            case 2: hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(threads), 0, 0, out, iters); break;
            case 3: hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(threads), 0, 0, out, iters); break;
            case 4: hipLaunchKernelGGL(k<4>, dim3(blocks), dim3(threads), 0, 0, out, iters); break;
            case 5: hipLaunchKernelGGL(k<5>, dim3(blocks), dim3(threads), 0, 0, out, iters); break;
            case 6: hipLaunchKernelGGL(k<6>, dim3(blocks), dim3(threads), 0, 0, out, iters); break;
            default: hipLaunchKernelGGL(k<7>, dim3(blocks), dim3(threads), 0, 0, out, iters); break;
            }
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms = 0.f;
            hipEventElapsedTime(&ms, a, b);
            if (ms < best) best = ms;
        }
        // wave-calls per SIMD = waves per SIMD * iters * 8 chains
        const double calls = (double)blocks * threads / 64 / (cus * 4) * iters * 8;
        const double cyc = best * 1e-3 * clk * 1e3 / calls;
        printf("%-32s %8.3f ms  %7.1f SIMD cycles per wave64 call (clock %d MHz)\n", names[v], best, cyc,
               clk / 1000);
    }
    return 0;
}
