// FETCH_SIZE calibration for the access widths the engine uses (rocprofv3's HBM
// read counter is calibrated only for 16 B/lane streaming reads on gfx950,
// MI355X_MICROARCH.md "HBM"): each kernel streams a 1 GiB buffer (past the 256 MiB
// Infinity Cache) once with 4, 8 or 16 B per lane, coalesced, and one kernel reads
// it the way rq_scan's leaf groups do (8-lane groups, 64 B each, groups 1 KiB apart,
// walking their 1 KiB block).  Compare FETCH_SIZE x 1024 with the byte count.
// build: hipcc -O3 --offload-arch=gfx950 fetch_calib.hip -o fetch_calib
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <class T>
__global__ __launch_bounds__(256) void stream_read(const T* p, size_t n, unsigned long long* out)
{
    unsigned long long acc = 0;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const T v = p[i];
        acc += (unsigned long long)v;
    }
    if (acc == 0x12345) out[0] = acc;
}
struct V4 { uint32_t x, y, z, w; };
__global__ __launch_bounds__(256) void stream_read16(const V4* p, size_t n, unsigned long long* out)
{
    unsigned long long acc = 0;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const V4 v = p[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 0x12345) out[0] = acc;
}
// rq_scan's pattern: a wave owns 8 KiB (1024 doubles = 8 leaves of 128); group g of
// 8 lanes reads leaf g's 16 rows per step (two 64 B loads), 8 steps per leaf.
__global__ __launch_bounds__(256) void leaf_read(const double* p, size_t n, unsigned long long* out)
{
    const int lane = threadIdx.x & 63, grp = lane >> 3, jj = lane & 7;
    const size_t w = (blockIdx.x * 256 + threadIdx.x) >> 6, nw = (size_t)gridDim.x * 4;
    double acc = 0.0;
    for (size_t base = w * 1024; base < n; base += nw * 1024) {
        const double* q = p + base + grp * 128;
        for (int i = 0; i < 128; i += 16) acc += q[i + jj] + q[i + 8 + jj];
    }
    if (acc == 1.2345) out[0] = 1;
}

int main()
{
    const size_t bytes = (size_t)1 << 30;
    void* buf;
    unsigned long long* out;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 8) != hipSuccess) return 1;
    (void)hipMemset(buf, 1, bytes);
    const int grid = 4096;
    hipLaunchKernelGGL(stream_read<uint32_t>, dim3(grid), dim3(256), 0, 0, (const uint32_t*)buf, bytes / 4, out);
    hipLaunchKernelGGL(stream_read<uint64_t>, dim3(grid), dim3(256), 0, 0, (const uint64_t*)buf, bytes / 8, out);
    hipLaunchKernelGGL(stream_read16, dim3(grid), dim3(256), 0, 0, (const V4*)buf, bytes / 16, out);
    hipLaunchKernelGGL(leaf_read, dim3(grid), dim3(256), 0, 0, (const double*)buf, bytes / 8, out);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    std::printf("bytes per kernel %zu (%.1f KiB)\n", bytes, bytes / 1024.0);
    return 0;
}
