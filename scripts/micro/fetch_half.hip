// FETCH_SIZE / WRITE_SIZE calibration for the per-lane 64-byte accesses of the
// arrival streams (rq_gen_streams stores 64-B chunks; rq_merge_streams loads them):
// is a 64-B (half-line) request tallied as 64 B, and does a line whose halves are
// requested at different times cost two fetches?  Each kernel touches a 1 GiB buffer
// (past the 256 MiB Infinity Cache), one 128-B line per lane:
//   rd_full    4 x 32-B loads per lane: the whole line in one go          (1 GiB)
//   rd_pair    2 x 32-B loads (first half), then 2 (second half)          (1 GiB)
//   rd_half0   first halves only                                          (0.5 GiB)
//   rd_half1   second halves only (a separate launch: far apart in time)  (0.5 GiB)
//   wr_full / wr_half0 / wr_half1: the same for stores
// Compare FETCH_SIZE / WRITE_SIZE (KiB) x 1024 with these byte counts.
// build: hipcc -O3 --offload-arch=gfx950 fetch_half.hip -o fetch_half
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(256) void rd_full(const double4* p, size_t nl, double* out)
{
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= nl) return;
    const double4 a = p[4 * i], b = p[4 * i + 1], c = p[4 * i + 2], d = p[4 * i + 3];
    const double s = a.x + b.y + c.z + d.w;
    if (s == 1.2345) out[0] = s;
}
__global__ __launch_bounds__(256) void rd_pair(const double4* p, size_t nl, double* out)
{
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= nl) return;
    const double4 a = p[4 * i], b = p[4 * i + 1];
    double s = a.x + b.y;
    __builtin_amdgcn_s_waitcnt(0);
    const double4 c = p[4 * i + 2], d = p[4 * i + 3];
    s += c.z + d.w;
    if (s == 1.2345) out[0] = s;
}
template <int H>
__global__ __launch_bounds__(256) void rd_half(const double4* p, size_t nl, double* out)
{
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= nl) return;
    const double4 a = p[4 * i + 2 * H], b = p[4 * i + 2 * H + 1];
    const double s = a.x + b.y;
    if (s == 1.2345) out[0] = s;
}
__global__ __launch_bounds__(256) void wr_full(double4* p, size_t nl)
{
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= nl) return;
    const double v = (double)i;
    for (int k = 0; k < 4; ++k) p[4 * i + k] = make_double4(v, v, v, v);
}
template <int H>
__global__ __launch_bounds__(256) void wr_half(double4* p, size_t nl)
{
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= nl) return;
    const double v = (double)i;
    p[4 * i + 2 * H] = make_double4(v, v, v, v);
    p[4 * i + 2 * H + 1] = make_double4(v, v, v, v);
}

int main()
{
    const size_t bytes = (size_t)1 << 30, nl = bytes / 128;
    double4* buf;
    double* out;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 8) != hipSuccess) return 1;
    (void)hipMemset(buf, 1, bytes);
    const unsigned grid = (unsigned)((nl + 255) / 256);
    hipLaunchKernelGGL(rd_full, dim3(grid), dim3(256), 0, 0, buf, nl, out);
    hipLaunchKernelGGL(rd_pair, dim3(grid), dim3(256), 0, 0, buf, nl, out);
    hipLaunchKernelGGL(rd_half<0>, dim3(grid), dim3(256), 0, 0, buf, nl, out);
    hipLaunchKernelGGL(rd_half<1>, dim3(grid), dim3(256), 0, 0, buf, nl, out);
    hipLaunchKernelGGL(wr_full, dim3(grid), dim3(256), 0, 0, buf, nl);
    hipLaunchKernelGGL(wr_half<0>, dim3(grid), dim3(256), 0, 0, buf, nl);
    hipLaunchKernelGGL(wr_half<1>, dim3(grid), dim3(256), 0, 0, buf, nl);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    std::printf("bytes per full kernel %zu (%.1f KiB), half kernels half that\n", bytes, bytes / 1024.0);
    return 0;
}
