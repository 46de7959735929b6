// Microbenchmark: Philox4x32-10 formulations on gfx950 (mul_hi + mul_lo vs one 32x32->64 mad).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ void philox_a(uint32_t c[4], uint32_t k0, uint32_t k1)
{
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t lo0 = 0xD2511F53u * c[0];
        const uint32_t hi0 = __umulhi(0xD2511F53u, c[0]);
        const uint32_t lo1 = 0xCD9E8D57u * c[2];
        const uint32_t hi1 = __umulhi(0xCD9E8D57u, c[2]);
        const uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
        c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
}
__device__ __forceinline__ void philox_b(uint32_t c[4], uint32_t k0, uint32_t k1)
{
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
        c[0] = n0; c[1] = (uint32_t)p1; c[2] = n2; c[3] = (uint32_t)p0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
}
template <int V>
__global__ void k(uint32_t* out, int iters)
{
    uint32_t c[4] = {threadIdx.x, blockIdx.x, 0u, 0u}, acc = 0;
    for (int i = 0; i < iters; ++i) {
        c[2] = i;
        if (V == 0) philox_a(c, 7u, 9u); else philox_b(c, 7u, 9u);
        acc ^= c[0] ^ c[1] ^ c[2] ^ c[3];
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}
__global__ void f64log(double* out, int iters)
{
    double x = 1.0 + threadIdx.x * 1e-6, acc = 0.0;
    for (int i = 0; i < iters; ++i) { acc += x / (2.0 + x); x = x * 1.0000001; }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}
int main()
{
    const int blocks = 256 * 8, threads = 256, iters = 2000;
    uint32_t* out; double* dout;
    hipMalloc(&out, sizeof(uint32_t) * blocks * threads);
    hipMalloc(&dout, sizeof(double) * blocks * threads);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    for (int v = 0; v < 3; ++v) {
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(a);
            if (v == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(threads), 0, 0, out, iters);
            else if (v == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(threads), 0, 0, out, iters);
            else hipLaunchKernelGGL(f64log, dim3(blocks), dim3(threads), 0, 0, dout, iters);
            hipEventRecord(b); hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b);
            const double calls = (double)blocks * threads * iters;
            // per wave-call cycles at 2.4 GHz over 1024 SIMDs
            printf("variant %d: %.3f ms, %.2f Gcalls/s, %.1f SIMD-cycles per wave64 call\n", v, ms,
                   calls / ms / 1e6, (ms * 1e-3 * 2.4e9 * 1024) / (calls / 64));
        }
    }
    return 0;
}
