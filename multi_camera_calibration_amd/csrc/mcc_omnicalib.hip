// mcc_omnicalib.hip -- CDNA4 kernels of the omnidir intrinsic calibration (cv::omnidir::calibrate,
// src/omnidir.cpp:1067-1211).
//
// One loop step of calibrate = one launch of k_oc_step, one 256-thread workgroup per view:
//   phase 0  wave 0 applies the previous step's pending pose update of this view
//            (x_v += alpha2 ((U^-1 rp - coef U^-1 1) - Y_v yc)) and its |G|^2, |x|^2 partials;
//   phase A  every thread projects its corners with the Mei model and writes the 2 x 16 rows of
//            [d/d(om, T) | d/d(fx, fy, s, cx, cy, xi, k1, k2, p1, p2)] (JacobianRow order,
//            src/omnidir.cpp:65-73) and E = img - proj into LDS;
//   phase B  the 16 x 16 Gram J^T J of the view's 2N x 16 strip on the matrix cores: every wave
//            takes every 4th block of 4 rows and issues v_mfma_f64_16x16x4_f64 with the same
//            register as A (J^T, 16 x 4) and B (J, 4 x 16); J^T E rides along as one VALU FMA;
//            the four waves' partial tiles are summed in LDS in wave order, and the rows / columns
//            of fixed intrinsics (flags2idx) masked to 0 (subMatrix);
//   phase C  wave 0 inverts the view's 6 x 6 pose block U (register Gauss-Jordan), and the
//            workgroup forms the block-arrow Schur contribution S_v = V_v - W_v^T U^-1 W_v (55),
//            the reduced right-hand sides of JTE and of the ones vector, and the scalars of the
//            Sherman-Morrison correction; written write-through (sc1), then a two-level
//            fixed-order last-arriver reduction (groups of ~sqrt(n) views, then the groups);
//   final    the last arriver runs calibrate's stop test on |G| / |x| of the update applied in
//            phase 0, solves the 10 x 10 reduced system for both right-hand sides, applies the
//            rank-one correction of JTJ + epsilon (epsilon added to EVERY entry, :925) and the
//            alpha_smooth2 factor, updates the intrinsics, and leaves the pose update pending.
// FP64 throughout, like the reference (calibrate converts its inputs to CV_64F, :1083-1094).
#include <hip/hip_runtime.h>

#include "mcc_device.hpp"
#include "mcc_omnicalib_internal.h"

namespace mcc {

typedef double oc_v4d __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) unsigned long long oc_gu64;
typedef __attribute__((address_space(1))) int oc_gi32;

__device__ __forceinline__ void oc_st(double* p, double v) {
    __hip_atomic_store((oc_gu64*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double oc_ld(const double* p) {
    return __longlong_as_double((long long)__hip_atomic_load((oc_gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
// write-through hand-off (MI355X_MICROARCH.md "visibility", Valid forms row 1): every handed-off
// double is an 8-B sc1 store, storing waves drain vmcnt(0) before the barrier, one lane takes the
// ticket, the last arriver reads with sc1 loads.  Resets the counter for the next launch.
__device__ __forceinline__ bool oc_arrive(int* counter, int expected) {
    __shared__ int last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const int t = __hip_atomic_fetch_add((oc_gi32*)counter, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = (t == expected - 1);
        if (last) __hip_atomic_store((oc_gi32*)counter, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    return last;
}
__device__ __forceinline__ double oc_readlane(double v, int l) {
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)u, l);
    const unsigned hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), l);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// sum_{q < n} p[q * kOcLc] in q order; the sc1 loads are issued 16 at a time so a group costs one
// or two memory round trips instead of n dependent ones
__device__ __forceinline__ double oc_sum(const double* p, int n) {
    constexpr int B = 16;
    double v = 0.0;
    for (int q0 = 0; q0 < n; q0 += B) {
        double b[B];
#pragma unroll
        for (int u = 0; u < B; ++u) b[u] = oc_ld(p + (size_t)min(q0 + u, n - 1) * kOcLc);
#pragma unroll
        for (int u = 0; u < B; ++u) v += q0 + u < n ? b[u] : 0.0;
    }
    return v;
}

// packed upper-triangle index of (i, j), i <= j, of a 10 x 10 matrix (row i holds 10 - i entries)
__device__ __forceinline__ int oc_up(int i, int j) { return i * 10 - (i * (i - 1)) / 2 + (j - i); }

struct OcIntr {
    double fx, fy, s, cx, cy, xi, k1, k2, p1, p2;
};

// cv::omnidir::projectPoints for one corner (src/omnidir.cpp:141-244): pixel (pu, pv) and, with
// JAC, the two 16-entry Jacobian rows.  R / T: the view pose; Jl: the left SO(3) Jacobian of om
// (dXc/dom = -[R X]x Jl(om), the same derivative as OpenCV's dXcdR * dRdom^T).
template <bool JAC>
__device__ __forceinline__ void oc_corner(const double* R, const double* Jl, const double* T, const OcIntr& q,
                                          double X, double Y, double Z, double& pu, double& pv, double* ju,
                                          double* jv) {
    const double RX0 = R[0] * X + R[1] * Y + R[2] * Z;
    const double RX1 = R[3] * X + R[4] * Y + R[5] * Z;
    const double RX2 = R[6] * X + R[7] * Y + R[8] * Z;
    const double Xc0 = RX0 + T[0], Xc1 = RX1 + T[1], Xc2 = RX2 + T[2];
    const double nrm = sqrt(Xc0 * Xc0 + Xc1 * Xc1 + Xc2 * Xc2);
    const double r_1 = 1.0 / nrm;
    const double Xs0 = Xc0 * r_1, Xs1 = Xc1 * r_1, Xs2 = Xc2 * r_1;
    const double iden = 1.0 / (Xs2 + q.xi);
    const double xu0 = Xs0 * iden, xu1 = Xs1 * iden;
    const double r2 = xu0 * xu0 + xu1 * xu1, r4 = r2 * r2;
    const double cd = 1.0 + q.k1 * r2 + q.k2 * r4;
    const double xd0 = xu0 * cd + 2.0 * q.p1 * xu0 * xu1 + q.p2 * (r2 + 2.0 * xu0 * xu0);
    const double xd1 = xu1 * cd + q.p1 * (r2 + 2.0 * xu1 * xu1) + 2.0 * q.p2 * xu0 * xu1;
    pu = q.fx * xd0 + q.s * xd1 + q.cx;
    pv = q.fy * xd1 + q.cy;
    if (!JAC) return;
    // dxp/dXc = F * dxd/dxu * dxu/dXs * dXs/dXc
    const double r_3 = r_1 * r_1 * r_1;
    const double S00 = r_1 - Xc0 * Xc0 * r_3, S11 = r_1 - Xc1 * Xc1 * r_3, S22 = r_1 - Xc2 * Xc2 * r_3;
    const double S01 = -(Xc0 * Xc1) * r_3, S02 = -(Xc0 * Xc2) * r_3, S12 = -(Xc1 * Xc2) * r_3;
    // dxu/dXc (2 x 3) = [[iden, 0, -xu0 iden], [0, iden, -xu1 iden]] * dXs/dXc
    const double a0 = iden, a2 = -xu0 * iden, b1 = iden, b2 = -xu1 * iden;
    const double U0 = a0 * S00 + a2 * S02, U1 = a0 * S01 + a2 * S12, U2 = a0 * S02 + a2 * S22;
    const double V0 = b1 * S01 + b2 * S02, V1 = b1 * S11 + b2 * S12, V2 = b1 * S12 + b2 * S22;
    const double temp1 = 2.0 * q.k1 * xu0 + 4.0 * q.k2 * xu0 * r2;
    const double temp2 = 2.0 * q.k1 * xu1 + 4.0 * q.k2 * xu1 * r2;
    const double A00 = q.k2 * r4 + 6.0 * q.p2 * xu0 + 2.0 * q.p1 * xu1 + xu0 * temp1 + q.k1 * r2 + 1.0;
    const double A01 = 2.0 * q.p1 * xu0 + 2.0 * q.p2 * xu1 + xu0 * temp2;
    const double A10 = 2.0 * q.p1 * xu0 + 2.0 * q.p2 * xu1 + xu1 * temp1;
    const double A11 = q.k2 * r4 + 2.0 * q.p2 * xu0 + 6.0 * q.p1 * xu1 + xu1 * temp2 + q.k1 * r2 + 1.0;
    // FA = [[fx, s], [0, fy]] * A
    const double F00 = q.fx * A00 + q.s * A10, F01 = q.fx * A01 + q.s * A11;
    const double F10 = q.fy * A10, F11 = q.fy * A11;
    const double du0 = F00 * U0 + F01 * V0, du1 = F00 * U1 + F01 * V1, du2 = F00 * U2 + F01 * V2;
    const double dv0 = F10 * U0 + F11 * V0, dv1 = F10 * U1 + F11 * V1, dv2 = F10 * U2 + F11 * V2;
    // d/dom = d * dXc/dom with dXc/dom = -[RX]x Jl, -[RX]x = [[0, RX2, -RX1], [-RX2, 0, RX0], [RX1, -RX0, 0]]
    const double mu0 = du1 * (-RX2) + du2 * RX1;
    const double mu1 = du0 * RX2 + du2 * (-RX0);
    const double mu2 = du0 * (-RX1) + du1 * RX0;
    const double mv0 = dv1 * (-RX2) + dv2 * RX1;
    const double mv1 = dv0 * RX2 + dv2 * (-RX0);
    const double mv2 = dv0 * (-RX1) + dv1 * RX0;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        ju[j] = mu0 * Jl[j] + mu1 * Jl[3 + j] + mu2 * Jl[6 + j];
        jv[j] = mv0 * Jl[j] + mv1 * Jl[3 + j] + mv2 * Jl[6 + j];
    }
    ju[3] = du0; ju[4] = du1; ju[5] = du2;
    jv[3] = dv0; jv[4] = dv1; jv[5] = dv2;
    ju[6] = xd0; ju[7] = 0.0; jv[6] = 0.0; jv[7] = xd1;   // df
    ju[8] = xd1; jv[8] = 0.0;                              // ds
    ju[9] = 1.0; ju[10] = 0.0; jv[9] = 0.0; jv[10] = 1.0;  // dc
    const double dx0 = -xu0 * iden, dx1 = -xu1 * iden;     // dxu/dxi
    ju[11] = F00 * dx0 + F01 * dx1;                        // dxi
    jv[11] = F10 * dx0 + F11 * dx1;
    const double K0 = xu0 * r2, K1 = xu0 * r4, K2 = 2.0 * xu0 * xu1, K3 = r2 + 2.0 * xu0 * xu0;   // dxd0/dkp
    const double L0 = xu1 * r2, L1 = xu1 * r4, L2 = r2 + 2.0 * xu1 * xu1, L3 = 2.0 * xu0 * xu1;  // dxd1/dkp
    ju[12] = q.fx * K0 + q.s * L0; ju[13] = q.fx * K1 + q.s * L1;
    ju[14] = q.fx * K2 + q.s * L2; ju[15] = q.fx * K3 + q.s * L3;
    jv[12] = q.fy * L0; jv[13] = q.fy * L1; jv[14] = q.fy * L2; jv[15] = q.fy * L3;
}

__device__ __forceinline__ void oc_pose(const double* pose, double* R, double* Jl) {
    const double w[3] = {pose[0], pose[1], pose[2]};
    Rot r;
    rodrigues_v2m(w, r);
#pragma unroll
    for (int k = 0; k < 9; ++k) R[k] = r.R[k];
    so3_jac(w, r, +1.0, Jl);
}

__global__ __launch_bounds__(256) void k_oc_step(OcArgs a) {
    OcState* st = a.st;
    if (st->done) return;
    const int v = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int n = a.n;
    const int c0 = a.view_off[v], np = a.view_off[v + 1] - c0;
    const int rows = 2 * np, rows4 = (rows + 3) & ~3, r4max = (2 * a.max_np + 3) & ~3;
    extern __shared__ double sm[];
    double* Jl = sm;                  // [r4max][16]
    double* el = Jl + 16 * r4max;     // [r4max]
    double* Cp = el + r4max;          // [4][256] per-wave Gram tiles
    double* jp = Cp + 1024;           // [4][64]  per-wave J^T E partials
    __shared__ double pose[6], intr[10], msk[10], nrm[2][6];
    __shared__ double C[256], je[16], je_raw[16], Ui[36], zbl[6], zul[6], Yl[60], tot[kOcLc];

    // ---- phase 0: the pending pose update of the previous step (fillFixed never touches poses)
    const int pending = st->pending;
    if (tid < 6) {
        const double xo = a.x[6 * (size_t)v + tid];
        double g = 0.0, xn = xo;
        if (pending) {
            const double al = st->alpha2, cf = st->coef;
            double s = 0.0;
#pragma unroll
            for (int j = 0; j < 10; ++j) s += a.Yv[60 * (size_t)v + tid * 10 + j] * a.yc[j];
            g = al * ((a.zb[6 * (size_t)v + tid] - cf * a.zu[6 * (size_t)v + tid]) - s);
            xn = xo + g;
            a.x[6 * (size_t)v + tid] = xn;
            a.G[6 * (size_t)v + tid] = g;
        }
        pose[tid] = xn;
        nrm[0][tid] = g * g;
        nrm[1][tid] = xo * xo;
    } else if (tid >= 64 && tid < 74) {
        intr[tid - 64] = a.x[6 * (size_t)n + tid - 64];
        msk[tid - 64] = a.mask[tid - 64];
    }
    __syncthreads();

    // ---- phase A: projection + 2 x 16 Jacobian rows into LDS
    {
        double R[9], Jr[9];
        oc_pose(pose, R, Jr);
        const double T[3] = {pose[3], pose[4], pose[5]};
        const OcIntr q{intr[0], intr[1], intr[2], intr[3], intr[4], intr[5], intr[6], intr[7], intr[8], intr[9]};
        for (int c = tid; c < np; c += 256) {
            const size_t g = (size_t)c0 + c;
            double ju[16], jv[16], pu, pv;
            oc_corner<true>(R, Jr, T, q, a.ox[g], a.oy[g], a.oz[g], pu, pv, ju, jv);
            double* du = Jl + 32 * (size_t)c;
#pragma unroll
            for (int j = 0; j < 16; ++j) { du[j] = ju[j]; du[16 + j] = jv[j]; }
            el[2 * c] = a.iu[g] - pu;
            el[2 * c + 1] = a.iv[g] - pv;
        }
        for (int r = rows + tid; r < rows4; r += 256) {
#pragma unroll
            for (int j = 0; j < 16; ++j) Jl[16 * r + j] = 0.0;
            el[r] = 0.0;
        }
    }
    __syncthreads();

    // ---- phase B: Gram of the 2N x 16 strip on the matrix cores, J^T E on the VALU
    {
        oc_v4d acc = {0.0, 0.0, 0.0, 0.0};
        double jacc = 0.0;
        const int rr = lane >> 4, cc = lane & 15, nblk = rows4 >> 2;
        for (int b = wave; b < nblk; b += 4) {
            const int r = 4 * b + rr;
            const double av = Jl[16 * r + cc];   // A[cc][rr] = J[r][cc] = B[rr][cc]
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, av, acc, 0, 0, 0);
            jacc += av * el[r];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) Cp[wave * 256 + (rr + 4 * i) * 16 + cc] = acc[i];
        jp[wave * 64 + lane] = jacc;
    }
    __syncthreads();
    {   // fixed intrinsics (flags2idx) drop out of the normal equations: subMatrix as a 0/1 mask
        const int i = tid >> 4, j = tid & 15;
        const double mi = i < 6 ? 1.0 : msk[i - 6], mj = j < 6 ? 1.0 : msk[j - 6];
        C[tid] = (((Cp[tid] + Cp[256 + tid]) + Cp[512 + tid]) + Cp[768 + tid]) * (mi * mj);
    }
    if (tid < 16) {
        double s = 0.0;
#pragma unroll
        for (int w = 0; w < 4; ++w)
#pragma unroll
            for (int q = 0; q < 4; ++q) s += jp[w * 64 + q * 16 + tid];
        je_raw[tid] = s;   // J^T E before the reduction (computeJacobian's JTE)
        je[tid] = tid < 6 ? s : s * msk[tid - 6];
    }
    __syncthreads();

    // ---- phase C: U^-1 (wave 0 register Gauss-Jordan; U = JEx^T JEx is SPD), Schur pieces
    if (wave == 0) {
        const int li = lane < 6 ? lane : 0;
        double row[12];
#pragma unroll
        for (int j = 0; j < 6; ++j) { row[j] = C[li * 16 + j]; row[6 + j] = li == j ? 1.0 : 0.0; }
        double dii = 1.0;
        bool bad = false;
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            const double piv = oc_readlane(row[k], k);
            bad |= !(piv > 0.0);
            const double pv = piv > 0.0 ? piv : 1.0;
            const double ip = 1.0 / pv;
            if (lane == k) dii = pv;
            const double f = lane == k ? 0.0 : row[k] * ip;
            double pr[12];
#pragma unroll
            for (int j = k + 1; j < 12; ++j) pr[j] = oc_readlane(row[j], k);
#pragma unroll
            for (int j = k + 1; j < 12; ++j) row[j] -= f * pr[j];
        }
        if (lane < 6) {
            const double id = 1.0 / dii;
            double zb = 0.0, zu = 0.0;
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                const double h = row[6 + j] * id;
                Ui[lane * 6 + j] = h;
                zb += h * je[j];
                zu += h;
            }
            zbl[lane] = zb;
            zul[lane] = zu;
        }
        if (bad && lane == 0) atomicOr(&st->error, 1);
    }
    __syncthreads();
    if (tid < 60) {   // Y = U^-1 W (6 x 10), W = C[0:6, 6:16]
        const int i = tid / 10, j = tid % 10;
        double y = 0.0;
#pragma unroll
        for (int k = 0; k < 6; ++k) y += Ui[i * 6 + k] * C[k * 16 + 6 + j];
        Yl[tid] = y;
        a.Yv[60 * (size_t)v + tid] = y;
    } else if (tid >= 64 && tid < 70) {
        a.zb[6 * (size_t)v + tid - 64] = zbl[tid - 64];
    } else if (tid >= 70 && tid < 76) {
        a.zu[6 * (size_t)v + tid - 70] = zul[tid - 70];
    } else if (tid >= 80 && tid < 86) {
        a.jte[6 * (size_t)v + tid - 80] = je[tid - 80];
    }
    __syncthreads();
    double* out = a.contrib + (size_t)v * kOcLc;
    if (tid < 55) {
        int i = 0, rem = tid;
        while (rem >= 10 - i) { rem -= 10 - i; ++i; }
        const int j = i + rem;
        double s = C[(6 + i) * 16 + 6 + j];
#pragma unroll
        for (int k = 0; k < 6; ++k) s -= C[k * 16 + 6 + i] * Yl[k * 10 + j];
        oc_st(out + kOcS + tid, s);
    } else if (tid < 65) {
        const int j = tid - 55;
        double s = je[6 + j];
#pragma unroll
        for (int k = 0; k < 6; ++k) s -= C[k * 16 + 6 + j] * zbl[k];
        oc_st(out + kOcRb + j, s);
    } else if (tid < 75) {
        const int j = tid - 65;
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < 6; ++k) s += C[k * 16 + 6 + j] * zul[k];
        oc_st(out + kOcWu + j, s);
    } else if (tid < 85) {
        oc_st(out + kOcJc + tid - 75, je_raw[6 + tid - 75]);
    } else if (tid < 89) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < 6; ++k)
            s += tid == kOcAb ? zbl[k] : tid == kOcAu ? zul[k] : tid == kOcNg ? nrm[0][k] : nrm[1][k];
        oc_st(out + tid, s);
    }

    // ---- two-level fixed-order reduction of the contributions
    const int grp = v / a.group_size, g0 = grp * a.group_size, gn = min(a.group_size, n - g0);
    if (!oc_arrive(&a.cnt[grp], gn)) return;
    if (tid < kOcLc) oc_st(a.gsum + (size_t)grp * kOcLc + tid, oc_sum(a.contrib + (size_t)g0 * kOcLc + tid, gn));
    if (!oc_arrive(&a.cnt[a.n_groups], a.n_groups)) return;
    if (tid < kOcLc) tot[tid] = oc_sum(a.gsum + tid, a.n_groups);
    __syncthreads();
    if (wave != 0) return;

    // ---- final: stop test, reduced solve, Sherman-Morrison, intrinsic update (wave 0)
    const int k = st->iter;
    double change = st->change;
    if (pending) change = sqrt(tot[kOcNg] + st->normG2_c) / sqrt(tot[kOcNx] + st->normX2_c);
    const int ct = st->crit_type;
    const bool stop = (ct == 1 && k >= st->max_count) || (ct == 2 && change <= st->eps) ||
                      (ct == 3 && (change <= st->eps || k >= st->max_count));
    if (lane == 0) st->change = change;
    if (stop) {
        if (lane == 0) { st->done = 1; st->pending = 0; }
        return;
    }
    const double alpha2 = 1.0 - pow(1.0 - 0.01, (double)k + 1.0);   // alpha_smooth2 (:1133)
    const double epsilon = 0.01 * pow(0.9, (double)k / 10);          // (:1135)
    const int li = lane < 10 ? lane : 0;
    const bool free_i = msk[li] != 0.0;
    double row[12];
#pragma unroll
    for (int j = 0; j < 10; ++j) {
        const double sv = tot[kOcS + (li <= j ? oc_up(li, j) : oc_up(j, li))];
        row[j] = free_i ? sv : (j == li ? 1.0 : 0.0);
    }
    row[10] = free_i ? tot[kOcRb + li] : 0.0;
    row[11] = free_i ? 1.0 - tot[kOcWu + li] : 0.0;
    // Gauss-Jordan, lane l keeps row l.  S is symmetric but can turn numerically indefinite (the
    // f / xi coupling of the Mei model makes it near-singular, as is the reference's dense JTJ): a
    // non-positive diagonal pivot falls back to the unused row of largest |entry|; an exactly singular
    // system gives G = 0 for the whole step, as the reference's Mat::inv() (DECOMP_LU) returns a
    // zero matrix then
    bool used = lane >= 10, singular = false;
    int pcol = -1;
    double dii = 1.0;
#pragma unroll
    for (int kk = 0; kk < 10; ++kk) {
        // the diagonal in natural order while it is positive: the elimination order of the
        // reference's dense LU on this (near-SPD) block, whose rounding the step reproduces
        int pl = kk;
        if (!(oc_readlane(row[kk], kk) > 0.0) || __builtin_amdgcn_readlane((int)used, kk) != 0) {
            pl = -1;
            double best = 0.0;
#pragma unroll
            for (int l = 0; l < 10; ++l) {
                const double c = fabs(oc_readlane(row[kk], l));
                const bool u = __builtin_amdgcn_readlane((int)used, l) != 0;
                if (!u && c > best) { best = c; pl = l; }
            }
            if (pl < 0) { singular = true; break; }
        }
        const double piv = oc_readlane(row[kk], pl);
        const double ip = 1.0 / piv;
        if (lane == pl) { dii = piv; used = true; pcol = kk; }
        const double f = lane == pl ? 0.0 : row[kk] * ip;
        double pr[12];
#pragma unroll
        for (int j = kk + 1; j < 12; ++j) pr[j] = oc_readlane(row[j], pl);
#pragma unroll
        for (int j = kk + 1; j < 12; ++j) row[j] -= f * pr[j];
    }
    // lane j takes the solution of column j from the lane that pivoted it
    const double sb = lane < 10 && !singular ? row[10] / dii : 0.0;
    const double su = lane < 10 && !singular ? row[11] / dii : 0.0;
    double yb = 0.0, yu = 0.0;
#pragma unroll
    for (int j = 0; j < 10; ++j) {
        const unsigned long long own = __ballot(pcol == j);
        const int src = own ? (int)__builtin_ctzll(own) : 0;
        const double vb = oc_readlane(sb, src), vu = oc_readlane(su, src);
        if (lane == j) { yb = vb; yu = vu; }
    }
    // 1^T A^-1 b = sum_v 1^T U^-1 rp_v - (sum_v W_v^T U^-1 1)^T yb + 1_free^T yb (and for u)
    const double wm = lane < 10 ? msk[lane] - tot[kOcWu + lane] : 0.0;
    double s1 = tot[kOcAb], s2 = tot[kOcAu];
#pragma unroll
    for (int l = 0; l < 10; ++l) {
        s1 += oc_readlane(wm * yb, l);
        s2 += oc_readlane(wm * yu, l);
    }
    double coef = epsilon * s1 / (1.0 + epsilon * s2);
    // A + epsilon 1 1^T singular (Sherman-Morrison denominator 0) or A singular: G = 0 for the step
    const bool skip = singular || !isfinite(coef);
    if (skip) coef = 0.0;
    const double yc = skip ? 0.0 : yb - coef * yu;
    const double a2 = skip ? 0.0 : alpha2;
    const double gc = a2 * yc;
    double ng = 0.0, nx = 0.0;
    double xo = 0.0;
    if (lane < 10) {
        xo = a.x[6 * (size_t)n + lane];
        a.x[6 * (size_t)n + lane] = xo + gc;
        a.yc[lane] = yc;
        a.G[6 * (size_t)n + lane] = gc;
        a.jte[6 * (size_t)n + lane] = tot[kOcJc + lane];
    }
#pragma unroll
    for (int l = 0; l < 10; ++l) {
        ng += oc_readlane(gc * gc, l);
        nx += oc_readlane(xo * xo, l);
    }
    if (lane == 0) {
        st->normG2_c = ng;
        st->normX2_c = nx;
        st->alpha2 = a2;   // 0: the poses' pending G is 0 too
        st->coef = coef;
        st->pending = 1;
        st->iter = k + 1;
    }
}

// estimateUncertainties' squared reprojection errors, per view (src/omnidir.cpp:1766-1803)
__global__ __launch_bounds__(64) void k_oc_err(OcErrArgs a) {
    const int v = blockIdx.x, lane = threadIdx.x;
    const int c0 = a.view_off[v], np = a.view_off[v + 1] - c0;
    const double* pose = a.x + 6 * (size_t)v;
    double R[9], Jr[9];
    oc_pose(pose, R, Jr);
    const double T[3] = {pose[3], pose[4], pose[5]};
    const double* qi = a.x + 6 * (size_t)a.n;
    const OcIntr q{qi[0], qi[1], qi[2], qi[3], qi[4], qi[5], qi[6], qi[7], qi[8], qi[9]};
    double s = 0.0;
    for (int c = lane; c < np; c += 64) {
        const size_t g = (size_t)c0 + c;
        double pu, pv;
        oc_corner<false>(R, Jr, T, q, a.ox[g], a.oy[g], a.oz[g], pu, pv, nullptr, nullptr);
        const double ex = a.iu[g] - pu, ey = a.iv[g] - pv;
        s += ex * ex + ey * ey;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
    if (lane == 0) a.view_sq[v] = s;
}

}  // namespace mcc

size_t mcc_oc_shmem(int max_np) {
    const size_t r4 = (size_t)((2 * max_np + 3) & ~3);
    return sizeof(double) * (17 * r4 + 1024 + 256);
}

hipError_t mcc_oc_set_attrs(int max_np) {
    return hipFuncSetAttribute((const void*)mcc::k_oc_step, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)mcc_oc_shmem(max_np));
}

hipError_t mcc_launch_oc_step(const mcc::OcArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(mcc::k_oc_step, dim3(a.n), dim3(256), mcc_oc_shmem(a.max_np), s, a);
    return hipGetLastError();
}

hipError_t mcc_launch_oc_err(const mcc::OcErrArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(mcc::k_oc_err, dim3(a.n), dim3(64), 0, s, a);
    return hipGetLastError();
}
