// Micro-benchmark of the large-m reduced-system elimination (gj_blocked, m > 30) in isolation.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/solve_bench.hip -o tools/solve_bench -lrccl && tools/solve_bench [m] [threads]
// One 256-thread workgroup solves a random SPD packed system REPS times; prints the median
// s_memtime ticks per solve and the max relative error against a host Cholesky solve.
#ifndef MCC_GJB_STAMPS
#define MCC_GJB_STAMPS
#endif
#include "../multi_camera_calibration_amd/csrc/mcc_kernels.hip"

#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

constexpr int REPS = 16;

__global__ __launch_bounds__(1024) void k_solve_bench(const double* packed, int m, double* xout, long long* ticks, int* err) {
    extern __shared__ double smb[];
    const int M = 16 * ((m + 15) / 16);
    double* x = smb;
    double* A = smb + M;
    double* PV = A + M * (M + 1);
    for (int rep = 0; rep < REPS; ++rep) {
        __syncthreads();
        long long t0 = 0;
        if (threadIdx.x == 0) t0 = (long long)__builtin_amdgcn_s_memtime();
        if (threadIdx.x == 0) mcc::g_gjb_stamps[63] = t0;
        mcc::gj_blocked(packed, x, A, PV, m, err);
        __syncthreads();
        if (threadIdx.x == 0) ticks[rep] = (long long)__builtin_amdgcn_s_memtime() - t0;
    }
    for (int t = threadIdx.x; t < m; t += blockDim.x) xout[t] = x[t];
}

int main(int argc, char** argv) {
    const int m = argc > 1 ? std::atoi(argv[1]) : 90;
    const int nt = argc > 2 ? std::atoi(argv[2]) : 256;   // workgroup size
    std::mt19937_64 rng(11);
    std::normal_distribution<double> nd;
    std::vector<double> B(m * m), S(m * m, 0.0), r(m);
    for (auto& v : B) v = nd(rng);
    for (int i = 0; i < m; ++i)
        for (int j = 0; j < m; ++j) {
            double s = i == j ? 0.5 * m : 0.0;
            for (int k = 0; k < m; ++k) s += B[i * m + k] * B[j * m + k];
            S[i * m + j] = s;
        }
    for (auto& v : r) v = nd(rng);
    const int ntri = m * (m + 1) / 2;
    std::vector<double> packed(ntri + 2 * m + 2, 0.0);
    for (int i = 0, t = 0; i < m; ++i)
        for (int j = i; j < m; ++j) packed[t++] = S[i * m + j];
    for (int i = 0; i < m; ++i) packed[ntri + i] = r[i];
    // host Cholesky reference
    std::vector<double> L(S), y(r);
    for (int j = 0; j < m; ++j) {
        double d = L[j * m + j];
        for (int k = 0; k < j; ++k) d -= L[j * m + k] * L[j * m + k];
        d = std::sqrt(d);
        L[j * m + j] = d;
        for (int i = j + 1; i < m; ++i) {
            double v = L[i * m + j];
            for (int k = 0; k < j; ++k) v -= L[i * m + k] * L[j * m + k];
            L[i * m + j] = v / d;
        }
    }
    for (int i = 0; i < m; ++i) { for (int k = 0; k < i; ++k) y[i] -= L[i * m + k] * y[k]; y[i] /= L[i * m + i]; }
    for (int i = m - 1; i >= 0; --i) { for (int k = i + 1; k < m; ++k) y[i] -= L[k * m + i] * y[k]; y[i] /= L[i * m + i]; }
    double *dp, *dx;
    long long* dt;
    int* de;
    (void)hipMalloc(&dp, sizeof(double) * packed.size());
    (void)hipMalloc(&dx, sizeof(double) * m);
    (void)hipMalloc(&dt, sizeof(long long) * REPS);
    (void)hipMalloc(&de, sizeof(int));
    (void)hipMemcpy(dp, packed.data(), sizeof(double) * packed.size(), hipMemcpyHostToDevice);
    (void)hipMemset(de, 0, sizeof(int));
    const int M = 16 * ((m + 15) / 16);
    const size_t shm = sizeof(double) * (M + M * (M + 1) + 2 * 16 * mcc::kBlkLd);
    (void)hipFuncSetAttribute((const void*)k_solve_bench, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(k_solve_bench, dim3(1), dim3(nt), shm, 0, dp, m, dx, dt, de);   // warm-up
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL(k_solve_bench, dim3(1), dim3(nt), shm, 0, dp, m, dx, dt, de);
    (void)hipEventRecord(e1, 0);
    hipError_t e = hipDeviceSynchronize();
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    std::vector<double> x(m);
    std::vector<long long> t(REPS);
    int err = 0;
    (void)hipMemcpy(x.data(), dx, sizeof(double) * m, hipMemcpyDeviceToHost);
    (void)hipMemcpy(t.data(), dt, sizeof(long long) * REPS, hipMemcpyDeviceToHost);
    (void)hipMemcpy(&err, de, sizeof(int), hipMemcpyDeviceToHost);
    double emax = 0, xmax = 0;
    for (int i = 0; i < m; ++i) { emax = std::max(emax, std::fabs(x[i] - y[i])); xmax = std::max(xmax, std::fabs(y[i])); }
    std::sort(t.begin(), t.end());
#ifdef MCC_GJB_STAMPS
    long long st[64];
    (void)hipMemcpyFromSymbol(st, HIP_SYMBOL(mcc::g_gjb_stamps), sizeof(st));
    const int nb = (m + 15) / 16;
    std::printf("  load %lld  first pivot %lld\n", st[0] - st[63], st[1] - st[0]);
    for (int kb = 0; kb < nb; ++kb)
        std::printf("  kb %d: scale-row %lld  eliminate(+next pivot) %lld\n", kb, st[2 + 3 * kb] - st[1 + 3 * kb],
                    st[3 + 3 * kb] - st[2 + 3 * kb]);
#endif
    std::printf("m=%d %s err=%d median_ticks=%lld min=%lld rel_err=%.3e  kernel %.1f us for %d solves (%.2f us each)\n", m,
                hipGetErrorString(e), err, t[REPS / 2], t[0], emax / xmax, ms * 1e3, REPS, ms * 1e3 / REPS);
    return 0;
}
