// Microbenchmark: read bandwidth of the scan's access pattern on gfx950.  10k
// "replicas" of 5460 rows in SoA arrays (t f64, s f64, v u32, c u32: 24 B / row, 1.31
// GB), one wave per replica, persistent grid of 4 waves/SIMD, every row read once:
//   P = 8: 8 lane groups x 8 lanes, a load instruction covers 8 rows (64 B of a
//          f64 column) in each of 8 leaves 128 rows apart -- the rq_scan trip;
//   P = 16: 4 groups x 16 lanes, an instruction covers 16 rows (one 128-B line);
//   P = 64: the whole wave on 64 consecutive rows (4 lines of a f64 column).
// Each lane sums what it loads (so nothing is dead) and writes one double.
// build: hipcc -O3 --offload-arch=gfx950 scan_pattern.hip -o scan_pattern
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

template <int P>
__global__ __launch_bounds__(256, 4) void rd(const double* __restrict__ t, const double* __restrict__ s,
                                             const uint32_t* __restrict__ v, const uint32_t* __restrict__ c,
                                             int n, int stride, int reps, int* wq, double* out)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int g = lane / P, j = lane % P;
    constexpr int G = 64 / P;             // groups (leaves) per wave
    const int nslot = gridDim.x * 4;
    double acc = 0.0;
    for (int r = blockIdx.x * 4 + w; r < reps;) {
        const int64_t base = (int64_t)r * stride;
        // leaf rounds: G leaves of 128 rows; a trip = 8 loads per lane per column
        constexpr int LEAF = 8 * P > 128 ? 8 * P : 128;
        for (int L0 = 0; L0 < n; L0 += LEAF * G) {
            const int off = L0 + g * LEAF;
            for (int i = 0; i < LEAF; i += 8 * P) {
                double a0[8], a1[8];
                uint32_t b0[8], b1[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    int k = off + i + u * P + j;
                    k = k < n ? k : n - 1;
                    a0[u] = t[base + k];
                    a1[u] = s[base + k];
                    b0[u] = v[base + k];
                    b1[u] = c[base + k];
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) acc += a0[u] * (double)b0[u] + a1[u] / (double)(b1[u] | 1u);
            }
        }
        int nx = 0;
        if (lane == 0) nx = atomicAdd(wq, 1);
        r = nslot + __builtin_amdgcn_readfirstlane(nx);
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main()
{
    const int n = 5460, stride = 5472, reps = 10000;
    const size_t rows = (size_t)stride * reps;
    double *t, *s, *out;
    uint32_t *v, *c;
    int* wq;
    hipMalloc(&t, rows * 8);
    hipMalloc(&s, rows * 8);
    hipMalloc(&v, rows * 4);
    hipMalloc(&c, rows * 4);
    hipMemset(t, 0, rows * 8);
    hipMemset(s, 0, rows * 8);
    hipMemset(v, 1, rows * 4);
    hipMemset(c, 1, rows * 4);
    int dev = 0, cus = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    int nb = 0;
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, rd<8>, 256, 0);
    const int blocks_max = cus * (nb > 0 ? nb : 4);
    hipMalloc(&out, (size_t)blocks_max * 256 * 8);
    hipMalloc(&wq, 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const double bytes = 24.0 * n * reps;
    for (int occ : {0, 4}) {   // 0: as many waves as fit; 4: 4 waves per SIMD like rq_scan<1, 4>
    const int blocks = occ ? cus * occ : blocks_max;
    for (int p : {8, 16, 64}) {
        float best = 1e30f;
        for (int rep = 0; rep < 5; ++rep) {
            hipMemset(wq, 0, 4);
            hipEventRecord(e0);
            if (p == 8) hipLaunchKernelGGL(rd<8>, dim3(blocks), dim3(256), 0, 0, t, s, v, c, n, stride, reps, wq, out);
            else if (p == 16) hipLaunchKernelGGL(rd<16>, dim3(blocks), dim3(256), 0, 0, t, s, v, c, n, stride, reps, wq, out);
            else hipLaunchKernelGGL(rd<64>, dim3(blocks), dim3(256), 0, 0, t, s, v, c, n, stride, reps, wq, out);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0.f;
            hipEventElapsedTime(&ms, e0, e1);
            if (ms < best) best = ms;
        }
        printf("P=%2d lanes per group: %.3f ms  %.0f GB/s (blocks %d)\n", p, best, bytes / (best * 1e-3) / 1e9, blocks);
    }
    }
    return 0;
}
