// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE for the access widths the hot path uses
// (MI355X_MICROARCH.md, HBM section: "FETCH_SIZE reports exactly 1/2 of the bytes of a wide
// coalesced streaming read (16 B/lane) ... Other access widths are uncalibrated: calibrate on a
// known byte count in your own access pattern").
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/fetch_calib.hip -o tools/fetch_calib
//   rocprofv3 --pmc FETCH_SIZE -d <dir> -o run --output-format csv -- tools/fetch_calib
//   rocprofv3 --pmc WRITE_SIZE -d <dir> -o run --output-format csv -- tools/fetch_calib
//   python tools/fetch_calib.py --fetch <dir> --write <dir> --out profiles/<round>/fetch_calib.json
//
// Each kernel moves a known number of bytes over a 96 MiB buffer (three times the 32 MiB of
// aggregate L2, so every line leaves L2 once per launch), one kernel per pattern:
//   rd_f32_soa   5 float streams, 4 B per lane per stream (k_linearize / k_edge corner staging)
//   rd_f64       8 B per lane, coalesced (records, Y', W, per-edge sums)
//   rd_f64_sc1   8 B per lane, sc1 (the fused step's hand-off loads)
//   rd_f128      16 B per lane (the guide's calibrated width: FETCH_SIZE = 1/2 of the bytes)
//   wr_f64       8 B per lane plain stores
//   wr_f64_sc1   8 B per lane sc1 stores (contributions, group sums)
//   wr_f32       4 B per lane plain stores
//   wr_f128      16 B per lane plain stores
// The host prints each kernel's byte count; tools/fetch_calib.py divides the counters by it.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef __attribute__((address_space(1))) unsigned long long gu64;

__global__ __launch_bounds__(256) void rd_f32_soa(const float* a, size_t n, float* sink) {   // 5 streams of n floats
    float s = 0.f;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        s += a[i] + a[n + i] + a[2 * n + i] + a[3 * n + i] + a[4 * n + i];
    if (s == 1234.5f) sink[0] = s;
}
__global__ __launch_bounds__(256) void rd_f64(const double* a, size_t n, double* sink) {
    double s = 0.0;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) s += a[i];
    if (s == 1234.5) sink[0] = s;
}
__global__ __launch_bounds__(256) void rd_f64_sc1(const double* a, size_t n, double* sink) {
    double s = 0.0;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        s += __longlong_as_double((long long)__hip_atomic_load((gu64*)(a + i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    if (s == 1234.5) sink[0] = s;
}
__global__ __launch_bounds__(256) void rd_f128(const double2* a, size_t n, double* sink) {
    double s = 0.0;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const double2 v = a[i];
        s += v.x + v.y;
    }
    if (s == 1234.5) sink[0] = s;
}
__global__ __launch_bounds__(256) void wr_f64(double* a, size_t n) {
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) a[i] = (double)i;
}
__global__ __launch_bounds__(256) void wr_f64_sc1(double* a, size_t n) {
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        __hip_atomic_store((gu64*)(a + i), (unsigned long long)__double_as_longlong((double)i), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}
__global__ __launch_bounds__(256) void wr_f32(float* a, size_t n) {
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) a[i] = (float)i;
}
__global__ __launch_bounds__(256) void wr_f128(double2* a, size_t n) {
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) a[i] = double2{(double)i, 1.0};
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s failed: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
    const size_t bytes = 96ull << 20;
    void* buf;
    double* sink;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(buf, 0, bytes));
    const dim3 grid(2048), block(256);
    const size_t n32 = bytes / 4, n64 = bytes / 8, n128 = bytes / 16;
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(rd_f32_soa, grid, block, 0, 0, (const float*)buf, n32 / 5, (float*)sink);
        hipLaunchKernelGGL(rd_f64, grid, block, 0, 0, (const double*)buf, n64, sink);
        hipLaunchKernelGGL(rd_f64_sc1, grid, block, 0, 0, (const double*)buf, n64, sink);
        hipLaunchKernelGGL(rd_f128, grid, block, 0, 0, (const double2*)buf, n128, sink);
        hipLaunchKernelGGL(wr_f64, grid, block, 0, 0, (double*)buf, n64);
        hipLaunchKernelGGL(wr_f64_sc1, grid, block, 0, 0, (double*)buf, n64);
        hipLaunchKernelGGL(wr_f32, grid, block, 0, 0, (float*)buf, n32);
        hipLaunchKernelGGL(wr_f128, grid, block, 0, 0, (double2*)buf, n128);
        CK(hipDeviceSynchronize());
    }
    std::printf("{\"rd_f32_soa\": %zu, \"rd_f64\": %zu, \"rd_f64_sc1\": %zu, \"rd_f128\": %zu, "
                "\"wr_f64\": %zu, \"wr_f64_sc1\": %zu, \"wr_f32\": %zu, \"wr_f128\": %zu}\n",
                (n32 / 5) * 5 * 4, n64 * 8, n64 * 8, n128 * 16, n64 * 8, n64 * 8, n32 * 4, n128 * 16);
    CK(hipFree(buf));
    CK(hipFree(sink));
    return 0;
}
