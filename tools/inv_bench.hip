// Micro-benchmark of the helper's in-place inverse (gj_inverse_blocked, m > 30) in isolation.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DMCC_PART=5 -Iinclude tools/inv_bench.hip -o tools/inv_bench.bin
//   tools/inv_bench.bin [m] [0|1|2]
// One workgroup of kSolveThreads inverts a random SPD system REPS times (S reloaded into LDS each
// time); prints the median s_memrealtime time per inversion (us), max |S S^-1 - I| and a hash of
// the inverse's bits (bitwise A/B of variants).  Second argument: 0 round 5's schedule, 1 the same with
// its phases timed, 2 the look-ahead (gj_inverse_blocked<true>), 3 the look-ahead with its first pivot
// block as a separate prologue (19.1 vs 22.7 us at m = 90: faster alone, but inlined into the helper
// it spilled, and with the helper's refinement indices made opaque to stop that, the shard lost 0.7 us).  (Row strides M + 2, + 3, + 5 instead
// of M + 1 measured the same, 19.4-19.7 us at m = 90.)
#include "../multi_camera_calibration_amd/csrc/mcc_kernels.hip"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

constexpr int REPS = 16;

// gj_inverse_blocked with its phases timed (thread 0, s_memrealtime, summed over the pivot blocks):
// [0] the pivot block's inverse, [1] the pivot block row, [2] the other blocks, [3] the pivot column
__device__ bool inv_phased(double* A, double* PV, int M, long long* ph) {
    using namespace mcc;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
    const int nb = M / 16, ld = M + 1;
    __shared__ int bad_s;
    if (tid == 0) bad_s = 0;
    long long t = (long long)__builtin_amdgcn_s_memrealtime();
    auto lap = [&](int k) {
        const long long u = (long long)__builtin_amdgcn_s_memrealtime();
        if (tid == 0) ph[k] += u - t;
        t = u;
    };
    for (int kb = 0; kb < nb; ++kb) {
        if (wave == 0 && !gjb_inverse16(A + 16 * kb * ld + 16 * kb, ld, PV, lane) && lane == 0) bad_s = 1;
        __syncthreads();
        lap(0);
        for (int it = wave; it < nb - 1; it += nw) {
            const int jb = it < kb ? it : it + 1;
            double* C = A + 16 * kb * ld + 16 * jb;
            blk_mfma(C, ld, PV, kBlkLd, C, ld, false, true);
        }
        __syncthreads();
        lap(1);
        for (int it = wave; it < (nb - 1) * (nb - 1); it += nw) {
            const int r = it / (nb - 1), c = it % (nb - 1);
            const int ib = r < kb ? r : r + 1, jb = c < kb ? c : c + 1;
            blk_mfma(A + 16 * ib * ld + 16 * jb, ld, A + 16 * ib * ld + 16 * kb, ld, A + 16 * kb * ld + 16 * jb, ld,
                     true, false);
        }
        __syncthreads();
        lap(2);
        for (int it = wave; it < nb; it += nw) {
            double* C = A + 16 * it * ld + 16 * kb;
            if (it != kb) {
                blk_mfma(C, ld, C, ld, PV, kBlkLd, true, true);
            } else {
                const int i = lane & 15, g = lane >> 4;
#pragma unroll
                for (int c = 0; c < 4; ++c) C[i * ld + 4 * g + c] = PV[i * kBlkLd + 4 * g + c];
            }
        }
        __syncthreads();
        lap(3);
    }
    return bad_s == 0;
}

// (A/B) the look-ahead with its kb = -1 step as a separate prologue
__device__ bool inv_lookahead_prologue(double* A, double* PV, int M) {
    using namespace mcc;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
    const int nb = M / 16, ld = M + 1, n1 = nb - 1;
    __shared__ int bad_s;
    if (tid == 0) bad_s = 0;
    auto blk = [&](int ib, int jb) { return A + 16 * ib * ld + 16 * jb; };
    auto pvb = [&](int kb) { return PV + (kb & 1) * 16 * kBlkLd; };
    if (wave == 0 && !gjb_inverse16(blk(0, 0), ld, pvb(0), lane) && lane == 0) bad_s = 1;
    __syncthreads();
    for (int it = wave; it < nb - 1; it += nw) {
        double* C = blk(0, it + 1);
        blk_mfma(C, ld, pvb(0), kBlkLd, C, ld, false, true);
    }
    __syncthreads();
    for (int kb = 0; kb < nb; ++kb) {
        if (kb + 1 < nb) {
            if (wave == 0) {
                blk_mfma(blk(kb + 1, kb + 1), ld, blk(kb + 1, kb), ld, blk(kb, kb + 1), ld, true, false);
                if (!gjb_inverse16(blk(kb + 1, kb + 1), ld, pvb(kb + 1), lane) && lane == 0) bad_s = 1;
            } else {
                for (int it = wave - 1; it < n1 * n1 - 1; it += nw - 1) {
                    const int t = it < kb * n1 + kb ? it : it + 1;
                    const int r = t / n1, c = t % n1;
                    const int ib = r < kb ? r : r + 1, jb = c < kb ? c : c + 1;
                    blk_mfma(blk(ib, jb), ld, blk(ib, kb), ld, blk(kb, jb), ld, true, false);
                }
            }
        } else {
            for (int it = wave; it < n1 * n1; it += nw) {
                const int r = it / n1, c = it % n1;
                const int ib = r < kb ? r : r + 1, jb = c < kb ? c : c + 1;
                blk_mfma(blk(ib, jb), ld, blk(ib, kb), ld, blk(kb, jb), ld, true, false);
            }
        }
        __syncthreads();
        const bool next = kb + 1 < nb;
        const int nrow = next ? nb - 2 : 0;
        for (int it0 = wave; it0 < nb + nrow; it0 += nw) {
            const int it = next && it0 <= kb + 1 ? (it0 == 0 ? kb + 1 : it0 - 1) : it0;
            if (it < nb) {
                double* C = blk(it, kb);
                if (it != kb) {
                    blk_mfma(C, ld, C, ld, pvb(kb), kBlkLd, true, true);
                    if (it == kb + 1) blk_mfma(C, ld, pvb(kb + 1), kBlkLd, C, ld, false, true);
                } else {
                    const int i = lane & 15, g = lane >> 4;
                    const double* P = pvb(kb);
#pragma unroll
                    for (int c = 0; c < 4; ++c) C[i * ld + 4 * g + c] = P[i * kBlkLd + 4 * g + c];
                }
            } else {
                const int q = it - nb;
                const int jb = q < kb ? q : q + 2;
                double* C = blk(kb + 1, jb);
                blk_mfma(C, ld, pvb(kb + 1), kBlkLd, C, ld, false, true);
            }
        }
        __syncthreads();
    }
    return bad_s == 0;
}

__global__ __launch_bounds__(mcc::kSolveThreads) void k_inv_bench(const double* Sg, int m, double* out, long long* ticks, int* ok, long long* ph, int phased) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    const int tid = threadIdx.x, M = 16 * ((m + 15) / 16);
    const int ld = M + 1;
    double* A = sm;
    double* PV = sm + M * ld;
    bool good = true;
    for (int rep = 0; rep < REPS; ++rep) {
        for (int t = tid; t < M * M; t += blockDim.x) {
            const int i = t / M, j = t % M;
            A[i * ld + j] = i < m && j < m ? Sg[i * m + j] : (i == j ? 1.0 : 0.0);
        }
        __syncthreads();
        long long t0 = 0, c0 = 0;
        if (tid == 0) { t0 = (long long)__builtin_amdgcn_s_memrealtime(); c0 = (long long)__builtin_amdgcn_s_memtime(); }
        good &= phased == 1 ? inv_phased(A, PV, M, ph) : phased == 2 ? mcc::gj_inverse_blocked<true>(A, PV, PV + 16 * mcc::kBlkLd, M) : phased == 3 ? inv_lookahead_prologue(A, PV, M) : mcc::gj_inverse_blocked<false>(A, PV, PV + 16 * mcc::kBlkLd, M);
        __syncthreads();
        if (tid == 0) {
            ticks[rep] = (long long)__builtin_amdgcn_s_memrealtime() - t0;
            ticks[REPS + rep] = (long long)__builtin_amdgcn_s_memtime() - c0;
        }
        __syncthreads();
    }
    for (int t = tid; t < m * m; t += blockDim.x) out[t] = A[(t / m) * ld + t % m];
    if (tid == 0) *ok = good;
}

int main(int argc, char** argv) {
    const int m = argc > 1 ? std::atoi(argv[1]) : 90;
    const int M = 16 * ((m + 15) / 16);
    std::mt19937_64 rng(7);
    std::normal_distribution<double> nd;
    std::vector<double> B(m * m), S(m * m, 0.0);
    for (auto& v : B) v = nd(rng);
    auto dsc = [](int i) { return std::sqrt(1.0 + 1e3 * (i % 6 < 3)); };   // the rotation / translation scales
    for (int i = 0; i < m; ++i)
        for (int j = 0; j < m; ++j) {
            double s = (i == j) ? m : 0.0;
            for (int k = 0; k < m; ++k) s += B[i * m + k] * B[j * m + k];
            S[i * m + j] = s * dsc(i) * dsc(j);
        }
    double *dS, *dout;
    long long* dt;
    int* dok;
    hipMalloc(&dS, sizeof(double) * m * m); hipMalloc(&dout, sizeof(double) * m * m);
    hipMalloc(&dt, sizeof(long long) * 2 * REPS); hipMalloc(&dok, sizeof(int));
    long long* dph;
    hipMalloc(&dph, sizeof(long long) * 8);
    hipMemset(dph, 0, sizeof(long long) * 8);
    const int phased = argc > 2 ? std::atoi(argv[2]) : 0;
    hipMemcpy(dS, S.data(), sizeof(double) * m * m, hipMemcpyHostToDevice);
    const size_t shm = (M * (M + 1) + 2 * 16 * mcc::kBlkLd) * sizeof(double);
    hipFuncSetAttribute((const void*)&k_inv_bench, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    for (int w = 0; w < 200; ++w)   // (the clock ramp: a lone workgroup on an idle chip runs slow at first)
        hipLaunchKernelGGL(k_inv_bench, dim3(1), dim3(mcc::kSolveThreads), shm, 0, dS, m, dout, dt, dok, dph, phased);
    hipMemset(dph, 0, sizeof(long long) * 8);
    hipLaunchKernelGGL(k_inv_bench, dim3(1), dim3(mcc::kSolveThreads), shm, 0, dS, m, dout, dt, dok, dph, phased);
    if (hipDeviceSynchronize() != hipSuccess) { std::printf("kernel failed\n"); return 1; }
    std::vector<long long> t(2 * REPS);
    std::vector<double> I(m * m);
    int ok = 0;
    hipMemcpy(t.data(), dt, sizeof(long long) * 2 * REPS, hipMemcpyDeviceToHost);
    const double ghz = 0.1 * (double)t[REPS + REPS / 2] / (double)t[REPS / 2];
    hipMemcpy(I.data(), dout, sizeof(double) * m * m, hipMemcpyDeviceToHost);
    hipMemcpy(&ok, dok, sizeof(int), hipMemcpyDeviceToHost);
    std::sort(t.begin() + 1, t.begin() + REPS);
    double err = 0;
    for (int i = 0; i < m; ++i)
        for (int j = 0; j < m; ++j) {
            double s = 0;
            for (int k = 0; k < m; ++k) s += S[i * m + k] * I[k * m + j];
            err = std::max(err, std::fabs(s - (i == j ? 1.0 : 0.0)));
        }
    unsigned long long h = 1469598103934665603ull;
    for (double v : I) { unsigned long long b; std::memcpy(&b, &v, 8); h = (h ^ b) * 1099511628211ull; }
    std::printf("m=%d inverse median %.2f us (min %.2f, first %.2f) |S S^-1 - I| %.3e ok %d bits %016llx (s_memtime at %.2f GHz)\n", m,
                t[REPS / 2] * 0.01, t[1] * 0.01, t[0] * 0.01, err, ok, h, ghz);
    if (phased == 1) {
        long long ph[8];
        hipMemcpy(ph, dph, sizeof(ph), hipMemcpyDeviceToHost);
        std::printf("  phases (us per inversion): pivot inverse %.2f, pivot row %.2f, other blocks %.2f, pivot column %.2f\n",
                    ph[0] * 0.01 / REPS, ph[1] * 0.01 / REPS, ph[2] * 0.01 / REPS, ph[3] * 0.01 / REPS);
    }
    return 0;
}
#if defined(MCC_PART) && MCC_PART != 0
size_t mcc_solve_shmem(int) { return 0; }   // (part 5 alone: the attribute helpers' reference)
#endif
