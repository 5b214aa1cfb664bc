// mcc_kernels.hip -- CDNA4 (gfx950) kernels of one Gauss-Newton step of the reference's
// multi-camera extrinsic BA (MultiCameraCalibration::optimizeExtrinsics, src/multicalib.cpp:462-514).
//
// Step dataflow:
//   k_linearize   one workgroup per photo vertex, one wavefront per edge (camera observing it):
//                 [pending photo update of the previous step, fused here], edge prologue
//                 (compose_motion + fl32 pose), corner sweep (lanes over corners, FP64 projection
//                 + 2x6 Jacobian strips, float32 residual), VALU butterfly reduce-scatter of the
//                 27 normal-equation sums, chain rule to the photo / global blocks, 6x6 photo
//                 inverse (register Gauss-Jordan), Schur factors Y'_e.
//                 m <= 30 (single GPU): the WHOLE step is this one kernel -- per-photo packed
//                 contributions, a two-level write-through last-arriver reduction, and the final
//                 arriver's stop test + reduced solve + camera update (multi-GPU: with the
//                 in-kernel peer exchange of the packed system first).
//   k_schur       m > 30 (or RCCL): camera-pair-block work items of S = sum H_gg - sum Y' H_gp^T
//                 and r, plus norm chunks; two-level write-through hand-off into the packed system.
//   k_solve       m > 30 / RCCL: [peer exchange], stop test, blocked Gauss-Jordan (16 x 16 blocks,
//                 MFMA f64 block products, look-ahead pivot inverses), camera update.
//   k_backsub     standalone photo back-substitution (flush of a pending update / deltaX output).
//   k_project_error  computeProjectError's per-edge float32 sums.
// The per-corner and per-edge blocks are at most 6x6: FP64 VALU, latency
// bound; MFMA appears only in the large-m reduced solve.  All reductions are fixed-order, so a run
// is bitwise reproducible.
#include <array>
#include <map>
#include <mutex>
#include <hip/hip_runtime.h>

#include <algorithm>

#include "mcc_device.hpp"
#include "mcc_internal.h"

// The library is built from this file compiled once per part (-DMCC_PART=0..5, in parallel: one
// translation unit took ~5 minutes).  Each part holds the non-template kernels and the launch
// wrappers (and so the template instantiations) of one family; without MCC_PART it is all of them.
//   0 host helpers, peers, backsub, project_error   1 k_linearize   2 k_group L = 16
//   3 k_group L = 32   4 the split step's k_prep / k_prep4 / k_edge / k_photo   5 k_schur, k_solve
#ifdef MCC_PART
#define MCC_IN(n) (MCC_PART == (n))
#else
#define MCC_IN(n) 1
#endif
// per-part kernel attributes (mcc_set_kernel_attrs, part 0, calls them)
hipError_t mcc_attrs_linearize(size_t shmem);
hipError_t mcc_attrs_group16(size_t shmem);
hipError_t mcc_attrs_group32(size_t shmem);
hipError_t mcc_attrs_photo(size_t shmem);
hipError_t mcc_attrs_solve(size_t shmem);

namespace mcc {

// ---------------------------------------------------------------- diagnostic stamps
// Diagnostic builds (-DMCC_DIAG, libmcc_diag.so only) stamp s_memtime at phase boundaries
// (-DMCC_DIAG_RT: the chip-wide 100 MHz s_memrealtime instead, for timelines across XCDs).
#ifdef MCC_DIAG_RT
#define MCC_DIAG_CLOCK() __builtin_amdgcn_s_memrealtime()
#else
#define MCC_DIAG_CLOCK() __builtin_amdgcn_s_memtime()
#endif
#ifdef MCC_DIAG
#define STAMPP(ptr, stride, k)                                                                     \
    do {                                                                                           \
        if (threadIdx.x == 0 && (ptr)) {                                                           \
            __builtin_amdgcn_sched_barrier(0);                                                     \
            (ptr)[(stride) * (size_t)blockIdx.x + (k)] = (long long)MCC_DIAG_CLOCK();              \
            __builtin_amdgcn_sched_barrier(0);                                                     \
        }                                                                                          \
    } while (0)
#else
#define STAMPP(ptr, stride, k) do { } while (0)
#endif
#define STAMP(k) STAMPP(a.stamps, kStampStride, k)
// stamp into an explicit slot row (ptr already points at this workgroup's row), by thread `who`
#ifdef MCC_DIAG
#define SSTAMP(ptr, k, who)                                                                        \
    do {                                                                                           \
        if (threadIdx.x == (who) && (ptr)) {                                                       \
            __builtin_amdgcn_sched_barrier(0);                                                     \
            (ptr)[k] = (long long)MCC_DIAG_CLOCK();                                                \
            __builtin_amdgcn_sched_barrier(0);                                                     \
        }                                                                                          \
    } while (0)
#else
#define SSTAMP(ptr, k, who) do { } while (0)
#endif
// chip-wide 100 MHz clock (s_memtime is per XCD): cross-workgroup timelines
#ifdef MCC_DIAG
#define RSTAMP(k)                                                                                  \
    do {                                                                                           \
        if (threadIdx.x == 0 && a.stamps)                                                          \
            a.stamps[kStampStride * (size_t)blockIdx.x + (k)] = (long long)__builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define RSTAMP(k) do { } while (0)
#endif

// ---------------------------------------------------------------- wave reduction
// Reduce-scatter butterfly of 32 per-lane doubles across the 64 lanes: 32 shuffles of 64-bit
// values instead of 6*27.  Afterwards lane l (and l^1) holds the full sum of value index
// idx(l) = 16*b5 + 8*b4 + 4*b3 + 2*b2 + b1.
template <int W>
__device__ __forceinline__ void bfly_step(double* v, int lane) {
    const bool hi = (lane & (2 * W)) != 0;
#pragma unroll
    for (int j = 0; j < W; ++j) {
        const double send = hi ? v[j] : v[j + W];
        const double keep = hi ? v[j + W] : v[j];
        v[j] = keep + __shfl_xor(send, 2 * W);
    }
}
// Cross-lane exchanges in VALU (no LDS crossbar): v_permlane32_swap / v_permlane16_swap
// (gfx950) move whole half-waves / rows, DPP row_ror / quad_perm the rest.
__device__ __forceinline__ double ull_f64(unsigned lo, unsigned hi) {
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
// vdst = a, src = b: lanes 32-63 of a <-> lanes 0-31 of b
__device__ __forceinline__ void pl32_swap(double& a, double& b) {
    const unsigned long long A = __double_as_longlong(a), B = __double_as_longlong(b);
    const auto l = __builtin_amdgcn_permlane32_swap((unsigned)A, (unsigned)B, false, false);
    const auto h = __builtin_amdgcn_permlane32_swap((unsigned)(A >> 32), (unsigned)(B >> 32), false, false);
    a = ull_f64(l[0], h[0]);
    b = ull_f64(l[1], h[1]);
}
// odd rows (16 lanes) of a <-> even rows of b
__device__ __forceinline__ void pl16_swap(double& a, double& b) {
    const unsigned long long A = __double_as_longlong(a), B = __double_as_longlong(b);
    const auto l = __builtin_amdgcn_permlane16_swap((unsigned)A, (unsigned)B, false, false);
    const auto h = __builtin_amdgcn_permlane16_swap((unsigned)(A >> 32), (unsigned)(B >> 32), false, false);
    a = ull_f64(l[0], h[0]);
    b = ull_f64(l[1], h[1]);
}
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
    const unsigned long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)b, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(b >> 32), CTRL, 0xF, 0xF, false);
    return ull_f64((unsigned)lo, (unsigned)hi);
}
constexpr int kDppRor4 = 0x124, kDppRor8 = 0x128, kDppRor12 = 0x12C;   // row_ror:n, dst[i] = src[(i - n) & 15]
constexpr int kDppXor2 = 0x4E, kDppXor1 = 0xB1;                         // quad_perm [2,3,0,1] / [1,0,3,2]

// fixed-order full wave sum: xor 32, 16 by permlane swaps of v with itself, 8, 4, 2, 1 by DPP
__device__ __forceinline__ double wave_sum(double v) {
    {
        double a = v, b = v;
        pl32_swap(a, b);
        v = a + b;
    }
    {
        double a = v, b = v;
        pl16_swap(a, b);
        v = a + b;
    }
    v += dpp_f64<kDppRor8>(v);
    {
        const bool hi = (threadIdx.x & 4) != 0;
        const double p4 = dpp_f64<kDppRor4>(v), p12 = dpp_f64<kDppRor12>(v);
        v += hi ? p4 : p12;
    }
    v += dpp_f64<kDppXor2>(v);
    v += dpp_f64<kDppXor1>(v);
    return v;
}

// Same butterfly as bfly_step<16..1> + final xor 1 (lanes with the partner bit set keep the
// upper half), with every exchange in VALU.
__device__ __forceinline__ double wave_reduce_scatter32(double* v, int lane) {
#pragma unroll
    for (int j = 0; j < 16; ++j) { double a = v[j], b = v[j + 16]; pl32_swap(a, b); v[j] = a + b; }   // xor 32
#pragma unroll
    for (int j = 0; j < 8; ++j) { double a = v[j], b = v[j + 8]; pl16_swap(a, b); v[j] = a + b; }      // xor 16
    {
        const bool hi = (lane & 8) != 0;   // xor 8: rotate a row by 8
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const double send = hi ? v[j] : v[j + 4], keep = hi ? v[j + 4] : v[j];
            v[j] = keep + dpp_f64<kDppRor8>(send);
        }
    }
    {
        const bool hi = (lane & 4) != 0;   // xor 4: i - 4 for the upper, i + 4 = i - 12 for the lower
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const double send = hi ? v[j] : v[j + 2], keep = hi ? v[j + 2] : v[j];
            const double p4 = dpp_f64<kDppRor4>(send), p12 = dpp_f64<kDppRor12>(send);
            v[j] = keep + (hi ? p4 : p12);
        }
    }
    {
        const bool hi = (lane & 2) != 0;   // xor 2
        const double send = hi ? v[0] : v[1], keep = hi ? v[1] : v[0];
        v[0] = keep + dpp_f64<kDppXor2>(send);
    }
    return v[0] + dpp_f64<kDppXor1>(v[0]);   // xor 1
}
__device__ __forceinline__ int bfly_index(int lane) {
    return ((lane >> 5) & 1) * 16 + ((lane >> 4) & 1) * 8 + ((lane >> 3) & 1) * 4 +
           ((lane >> 2) & 1) * 2 + ((lane >> 1) & 1);
}
__device__ __forceinline__ double readlane_f64(double v, int l) {
    const unsigned long long b = __double_as_longlong(v);
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)b, l);
    const unsigned hi = __builtin_amdgcn_readlane((unsigned)(b >> 32), l);
    return __longlong_as_double(((unsigned long long)hi << 32) | lo);
}


constexpr int kCamStride = 24;  // LDS camera table row: R (9), Jl (9), T (3), pad
constexpr int kIntrStride = 20; // LDS intrinsics row: fx, fy, cx, cy, skew, xi, k[12], pad

// ---------------------------------------------------------------- per-edge LDS record
struct EdgeLds {
    double R[9];      // Rodrigues(fl32(om)) used by the projection
    double T[3];      // fl32(T)
    double Gp[36];    // photo chain: J_photo = J' Gp (J' = [-D[Y]x | D], 2x6 per corner)
    double Gg[36];    // global-block chain
    double A[36];     // reduced A' (full 6x6)
    double b[6];      // reduced b'
    double Hpp[36];   // Gp^T A' Gp
    double Hgg[36];   // Gg^T A' Gg
    double Hgp[36];   // Gg^T A' Gp
    double gp[6], gg[6];
    double Xp[36], Xg[36];  // scratch A' Gp, A' Gg
    int cam, side, off, n;
    int has_global, edge, pad0, pad1;
};
static_assert(sizeof(EdgeLds) % 16 == 0, "EdgeLds alignment");

// G (6x6) = [[Grr, 0], [Gtr, Gtt]]; Gtt == nullptr means identity.
__device__ __forceinline__ void store_G(double* G, const double* Grr, const double* Gtr, const double* Gtt) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            G[i * 6 + j] = Grr ? Grr[i * 3 + j] : 0.0;
            G[i * 6 + 3 + j] = 0.0;
            G[(3 + i) * 6 + j] = Gtr ? Gtr[i * 3 + j] : 0.0;
            G[(3 + i) * 6 + 3 + j] = Gtt ? Gtt[i * 3 + j] : (i == j ? 1.0 : 0.0);
        }
}

// ---------------------------------------------------------------- edge prologue (one lane)
// compose_motion(photo, camera) [+ compose_motion(ds, photofront) for BACK edges], float32
// composed pose, Rodrigues of it for the projection, and the chain maps G = blockdiag(Jl, I) M.
// src/mymulticalib.cpp:468-614 (pinhole), src/multicalib.cpp:717-824 (omni),
// src/doubleSide.cpp:288-430 (double side).  Rodrigues matrices and Jacobians of the photo, the
// cameras and the double-side transform come from the workgroup's LDS tables (phase 0).
struct PhotoLds {
    double xp[6];        // photo parameters (double of the float32 state)
    double xo[6];        // photo parameters before the pending update (float32 values)
    double R1[9], Jr1[9];
    double Rds[9], Jrds[9], dst[3], pad0;
    double Hs[36], gs[6], Lm[36], z[6], il[6];
    double dgl[128];     // global-block delta of the previous solve (pending update)
    double nrm[2];       // ||G||^2, ||x||^2 of this photo's last applied update (fused step)
    double cn[2];        // state snapshot: camera-block ||G||^2, ||x||^2 of the last update
    int iter0, pad1[3];  // state snapshot: completed updates
    int bn[8];           // per camera block: number of the photo's edges in it (fused step)
    unsigned char bl[5][64];   // per camera block: those edges in edge order
    // followed by the camera table [C][kCamStride], the intrinsics [C][kIntrStride] and the
    // photo's corners [5][max_cpp] (float)
};
static_assert(sizeof(PhotoLds) % 16 == 0, "PhotoLds alignment");

// the tail of cvRodrigues2 vector -> matrix given theta, sin, cos (OpenCV order, no contraction)
__device__ __forceinline__ void rodrigues_formula(const double* r, double th, double sn, double c, double* R) {
#pragma clang fp contract(off)
    const double c1 = 1. - c;
    const double itheta = 1. / th;
    const double rx = r[0] * itheta, ry = r[1] * itheta, rz = r[2] * itheta;
    const double rrt[9] = {rx * rx, rx * ry, rx * rz, rx * ry, ry * ry, ry * rz, rx * rz, ry * rz, rz * rz};
    const double r_x[9] = {0, -rz, ry, rz, 0, -rx, -ry, rx, 0};
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        const double I = (k == 0 || k == 4 || k == 8) ? 1.0 : 0.0;
        R[k] = c * I + c1 * rrt[k] + sn * r_x[k];
    }
}
// Rodrigues of rf given the trig (th0, s0, c0) of a nearby angle th0 (the log of the FP64
// composed rotation): cos/sin(|rf|) by a 3rd-order shift from th0 (|rf| - th0 ~ 1e-7), which
// agrees with libm cos/sin to a few ulp; falls back to sincos if the angles are not close.
__device__ __forceinline__ void rodrigues_near(const double r[3], double th0, double s0, double c0, Rot& o) {
    double th;
    {
#pragma clang fp contract(off)
        th = sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
    }
    const double d = th - th0;
    if (!(fabs(d) < 1e-6) || th < 1e-3) {
        rodrigues_v2m(r, o);
        return;
    }
    const double d2 = d * d;
    const double c = c0 - s0 * d - c0 * d2 * 0.5 + s0 * d2 * d * (1.0 / 6.0);
    const double sn = s0 + c0 * d - s0 * d2 * 0.5 - c0 * d2 * d * (1.0 / 6.0);
    o.th = th; o.s = sn; o.c = c;
    rodrigues_formula(r, th, sn, c, o.R);
}



// float32 composed pose -> L.T, L.R (projection) and Jl(fl32 om)
__device__ __forceinline__ void finish_pose(const double* om, const double* T, double th, double sn, double cs,
                                            EdgeLds& L, double* Jl) {
    // Rvectran1 / Tvectran1 -> float32 (src/mymulticalib.cpp:546-553)
    double rf[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) { rf[k] = (double)(float)om[k]; L.T[k] = (double)(float)T[k]; }
    Rot rp;
    rodrigues_near(rf, th, sn, cs, rp);
#pragma unroll
    for (int k = 0; k < 9; ++k) L.R[k] = rp.R[k];
    so3_jac(rf, rp, +1.0, Jl);
}

template <int MODEL>
__device__ void edge_prologue(const PhotoLds& P, const double* ctab, EdgeLds& L) {
    const int cam = L.cam, side = L.side;
    const double T1[3] = {P.xp[3], P.xp[4], P.xp[5]};
    const double* R2 = ctab + kCamStride * cam;
    const double* Jl2 = R2 + 9;
    const double* T2 = R2 + 18;
    Motion f;
    double th3, s3, c3;
    compose(P.R1, P.Jr1, T1, R2, Jl2, T2, f, th3, s3, c3);
    double Jl[9], t9[9], u9[9];
    if (side == MCC_BACK) {
        // compose_motion(ds, photofront), src/mymulticalib.cpp:503-506.  R(om_front) is the FP64
        // composed rotation itself (equal to Rodrigues(om_front) to rounding).
        Rot rf0;
        rf0.th = th3; rf0.s = s3; rf0.c = c3;
        double Jlf[9];
        so3_jac(f.om, rf0, +1.0, Jlf);
        Motion b;
        double th, sn, cs;
        compose(P.Rds, P.Jrds, P.dst, f.R, Jlf, f.T, b, th, sn, cs);
        finish_pose(b.om, b.T, th, sn, cs, L, Jl);
        // photo: E2 * D1 = [[A2b A1, 0], [B2b A1, R2]]   (src/mymulticalib.cpp:509-512)
        mat3_mul(b.A2, f.A1, t9);
        mat3_mul(Jl, t9, u9);
        mat3_mul(b.B2, f.A1, t9);
        store_G(L.Gp, u9, t9, R2);
        if (MODEL == MCC_MODEL_DOUBLESIDE) {
            // ds block: [[A1b, 0], [0, R_front]]  (src/doubleSide.cpp:398-399)
            mat3_mul(Jl, b.A1, u9);
            store_G(L.Gg, u9, nullptr, f.R);
            L.has_global = 1;
        } else {
            // camera block as the reference chains it (src/mymulticalib.cpp:514-517), which
            // omits dTt/dTf * dTf/dRc at :516 (hazard A12): [[A2b A2, 0], [B2b A2, I]]
            mat3_mul(b.A2, f.A2, t9);
            mat3_mul(Jl, t9, u9);
            mat3_mul(b.B2, f.A2, t9);
            store_G(L.Gg, u9, t9, nullptr);
            L.has_global = cam != 0;
        }
    } else {
        finish_pose(f.om, f.T, th3, s3, c3, L, Jl);
        mat3_mul(Jl, f.A1, u9);
        store_G(L.Gp, u9, nullptr, R2);
        if (MODEL == MCC_MODEL_DOUBLESIDE) {
            for (int k = 0; k < 36; ++k) L.Gg[k] = 0.0;   // zero ds jacobian on the front (doubleSide.cpp:335-336)
            L.has_global = 0;
        } else {
            mat3_mul(Jl, f.A2, u9);
            store_G(L.Gg, u9, f.B2, nullptr);
            L.has_global = cam != 0;
        }
    }
}


// ---------------------------------------------------------------- wave-cooperative edge prologue
// The same chain as edge_prologue (src/mymulticalib.cpp:468-614, src/multicalib.cpp:717-824,
// src/doubleSide.cpp:288-430) computed by the wave that sweeps the edge: lanes own matrix
// entries (3-term dot products instead of one lane doing every 3x3 product), while the rotation
// logs / Rodrigues / Jacobian coefficients every entry needs are evaluated by all lanes.  Value
// paths keep OpenCV's operation order with contraction off.
__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ double dot3_nc(double a0, double b0, double a1, double b1, double a2, double b2) {
#pragma clang fp contract(off)
    return a0 * b0 + a1 * b1 + a2 * b2;
}
__device__ __forceinline__ double add_nc(double a, double b) {
#pragma clang fp contract(off)
    return a + b;
}
// row i (runtime) of I + s1 [w]x + s2 [w]x^2
__device__ __forceinline__ void so3_poly_row(const double* w, double s1, double s2, int i, double* row) {
    double M[9];
    so3_poly(w, s1, s2, M);
    row[0] = i == 0 ? M[0] : (i == 1 ? M[3] : M[6]);
    row[1] = i == 0 ? M[1] : (i == 1 ? M[4] : M[7]);
    row[2] = i == 0 ? M[2] : (i == 1 ? M[5] : M[8]);
}
// column j (runtime) of I + s1 [w]x + s2 [w]x^2
__device__ __forceinline__ void so3_poly_col(const double* w, double s1, double s2, int j, double* col) {
    double M[9];
    so3_poly(w, s1, s2, M);
    col[0] = j == 0 ? M[0] : (j == 1 ? M[1] : M[2]);
    col[1] = j == 0 ? M[3] : (j == 1 ? M[4] : M[5]);
    col[2] = j == 0 ? M[6] : (j == 1 ? M[7] : M[8]);
}
// so3_jac's coefficients: J = I + sign*a [w]x + b [w]x^2
__device__ __forceinline__ void jac_coef(double th, double s, double c, double& a, double& b) {
    const double t2 = th * th;
    if (th < 1e-2) {
        a = 0.5 - t2 * (1.0 / 24.0) + t2 * t2 * (1.0 / 720.0);
        b = 1.0 / 6.0 - t2 * (1.0 / 120.0) + t2 * t2 * (1.0 / 5040.0);
    } else {
        a = (1.0 - c) / t2;
        b = (th - s) / (t2 * th);
    }
}
// so3_jac_inv's coefficient: J^-1 = I - sign*0.5 [w]x + ci [w]x^2
__device__ __forceinline__ double jinv_coef(double th, double s, double c) {
    const double t2 = th * th;
    if (th < 1e-2) return 1.0 / 12.0 + t2 * (1.0 / 720.0) + t2 * t2 * (1.0 / 30240.0);
    return 1.0 / t2 - (1.0 + c) / (2.0 * th * s);
}
// row i of -[q]x
__device__ __forceinline__ void negskew_row(const double* q, int i, double* row) {
    row[0] = i == 0 ? 0.0 : (i == 1 ? -q[2] : q[1]);
    row[1] = i == 0 ? q[2] : (i == 1 ? 0.0 : -q[0]);
    row[2] = i == 0 ? -q[1] : (i == 1 ? q[0] : 0.0);
}

template <int MODEL>
__device__ __forceinline__ void edge_prologue_wave(const PhotoLds& P, const double* ctab, EdgeLds& L, int lane) {
    const int cam = L.cam, side = L.side;
    const double* R2 = ctab + kCamStride * cam;
    const double* Jl2 = R2 + 9;
    const double* T2 = R2 + 18;
    double* X = L.Xp;    // R3 [0..8], T3 [9..11], q [12..14]; back: Rb [18..26], Tb [27..29], qb [30..32]
    double* W = L.Xg;    // A1 [0..8], A2 [9..17], B2 [18..26]; back: A1b [27..35]
    double* Wb = L.Hgp;  // back: A2b [0..8], B2b [9..17]
    // ---- compose_motion(photo, camera) values: R3 = R2 R1, q = R2 T1, T3 = q + T2
    if (lane < 9) {
        const int i = lane / 3, j = lane % 3;
        X[lane] = dot3_nc(R2[i * 3], P.R1[j], R2[i * 3 + 1], P.R1[3 + j], R2[i * 3 + 2], P.R1[6 + j]);
    } else if (lane < 12) {
        const int i = lane - 9;
        const double q = dot3_nc(R2[i * 3], P.xp[3], R2[i * 3 + 1], P.xp[4], R2[i * 3 + 2], P.xp[5]);
        X[12 + i] = q;
        X[9 + i] = add_nc(q, T2[i]);
    }
    wave_sync_lds();
    double om[3], th, sn, cs;
    {
        double R3[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) R3[k] = X[k];
        rodrigues_m2v(R3, om, th, sn, cs);
    }
    // ---- A1 = Jr^-1(om3) Jr(om1), A2 = Jl^-1(om3) Jl(om2), B2 = -[q]x Jl(om2)
    if (lane < 27) {
        const int blk = lane / 9, e = lane % 9, i = e / 3, j = e % 3;
        double row[3];
        if (blk < 2) {
            so3_poly_row(om, blk == 0 ? 0.5 : -0.5, jinv_coef(th, sn, cs), i, row);
        } else {
            const double q[3] = {X[12], X[13], X[14]};
            negskew_row(q, i, row);
        }
        const double* B = blk == 0 ? P.Jr1 : Jl2;
        W[lane] = blk < 2 && rot_jzero(sn, cs) ? 0.0 : row[0] * B[j] + row[1] * B[3 + j] + row[2] * B[6 + j];
    }
    if (side != MCC_BACK) {
        wave_sync_lds();
        // float32 composed pose (src/mymulticalib.cpp:546-553), its Rodrigues and Jl
        double rf[3], Tf[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) { rf[k] = (double)(float)om[k]; Tf[k] = (double)(float)X[9 + k]; }
        Rot rp;
        rodrigues_near(rf, th, sn, cs, rp);
        double ja, jb;
        jac_coef(rp.th, rp.s, rp.c, ja, jb);
        if (lane == 0) {
#pragma unroll
            for (int k = 0; k < 9; ++k) L.R[k] = rp.R[k];
#pragma unroll
            for (int k = 0; k < 3; ++k) L.T[k] = Tf[k];
            L.has_global = MODEL == MCC_MODEL_DOUBLESIDE ? 0 : (cam != 0);
        }
        // Gp = [[Jl A1, 0], [0, R2]];  Gg = [[Jl A2, 0], [B2, I]]  (DoubleSide front: 0,
        // src/doubleSide.cpp:335-336)
        for (int e = lane; e < 72; e += 64) {
            const int w = e / 36, r = (e % 36) / 6, c = e % 6;
            double v;
            if (r < 3 && c < 3) {
                double row[3];
                so3_poly_row(rf, ja, jb, r, row);
                const double* M = w == 0 ? W : W + 9;
                v = row[0] * M[c] + row[1] * M[3 + c] + row[2] * M[6 + c];
                if (w == 1 && MODEL == MCC_MODEL_DOUBLESIDE) v = 0.0;
            } else if (r < 3) {
                v = 0.0;
            } else if (c < 3) {
                v = (w == 1 && MODEL != MCC_MODEL_DOUBLESIDE) ? W[18 + (r - 3) * 3 + c] : 0.0;
            } else {
                v = w == 0 ? R2[(r - 3) * 3 + c - 3]
                           : (MODEL == MCC_MODEL_DOUBLESIDE ? 0.0 : (r == c ? 1.0 : 0.0));
            }
            (w == 0 ? L.Gp : L.Gg)[r * 6 + c] = v;
        }
        return;
    }
    // ---- BACK: compose_motion(ds, photofront), src/mymulticalib.cpp:503-518,
    // src/doubleSide.cpp:320-328; R(om_front) is the FP64 composed rotation R3
    double fa, fb;
    jac_coef(th, sn, cs, fa, fb);   // Jlf = Jl(om_front)
    if (lane < 9) {
        const int i = lane / 3, j = lane % 3;
        X[18 + lane] = dot3_nc(X[i * 3], P.Rds[j], X[i * 3 + 1], P.Rds[3 + j], X[i * 3 + 2], P.Rds[6 + j]);
    } else if (lane < 12) {
        const int i = lane - 9;
        const double q = dot3_nc(X[i * 3], P.dst[0], X[i * 3 + 1], P.dst[1], X[i * 3 + 2], P.dst[2]);
        X[30 + i] = q;
        X[27 + i] = add_nc(q, X[9 + i]);
    }
    wave_sync_lds();
    double omb[3], thb, snb, csb;
    {
        double Rb[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) Rb[k] = X[18 + k];
        rodrigues_m2v(Rb, omb, thb, snb, csb);
    }
    // A1b = Jr^-1(omb) Jr(ds), A2b = Jl^-1(omb) Jlf, B2b = -[qb]x Jlf
    if (lane < 27) {
        const int blk = lane / 9, e = lane % 9, i = e / 3, j = e % 3;
        double row[3], col[3];
        if (blk < 2) {
            so3_poly_row(omb, blk == 0 ? 0.5 : -0.5, jinv_coef(thb, snb, csb), i, row);
        } else {
            const double q[3] = {X[30], X[31], X[32]};
            negskew_row(q, i, row);
        }
        if (blk == 0) {
            col[0] = P.Jrds[j]; col[1] = P.Jrds[3 + j]; col[2] = P.Jrds[6 + j];
        } else {
            so3_poly_col(om, fa, fb, j, col);
        }
        const double v = blk < 2 && rot_jzero(snb, csb) ? 0.0 : row[0] * col[0] + row[1] * col[1] + row[2] * col[2];
        if (blk == 0) W[27 + e] = v;
        else Wb[(blk - 1) * 9 + e] = v;
    }
    wave_sync_lds();
    double rf[3], Tf[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) { rf[k] = (double)(float)omb[k]; Tf[k] = (double)(float)X[27 + k]; }
    Rot rp;
    rodrigues_near(rf, thb, snb, csb, rp);
    double ja, jb;
    jac_coef(rp.th, rp.s, rp.c, ja, jb);
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < 9; ++k) L.R[k] = rp.R[k];
#pragma unroll
        for (int k = 0; k < 3; ++k) L.T[k] = Tf[k];
        L.has_global = MODEL == MCC_MODEL_DOUBLESIDE ? 1 : (cam != 0);
    }
    // Gp = [[Jl A2b A1, 0], [B2b A1, R2]];  Gg (MyMulti, hazard A12) = [[Jl A2b A2, 0], [B2b A2, I]];
    // Gg (DoubleSide ds block) = [[Jl A1b, 0], [0, R_front]]
    for (int e = lane; e < 72; e += 64) {
        const int w = e / 36, r = (e % 36) / 6, c = e % 6;
        const bool ds = w == 1 && MODEL == MCC_MODEL_DOUBLESIDE;
        const double* M = w == 0 ? W : W + 9;   // A1 (photo) / A2 (camera)
        double v;
        if (r < 3 && c < 3) {
            double row[3];
            so3_poly_row(rf, ja, jb, r, row);
            if (ds) {
                v = row[0] * W[27 + c] + row[1] * W[30 + c] + row[2] * W[33 + c];
            } else {
                v = 0.0;
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    const double am = Wb[k * 3] * M[c] + Wb[k * 3 + 1] * M[3 + c] + Wb[k * 3 + 2] * M[6 + c];
                    v += row[k] * am;
                }
            }
        } else if (r < 3) {
            v = 0.0;
        } else if (c < 3) {
            const int i = r - 3;
            v = ds ? 0.0 : Wb[9 + i * 3] * M[c] + Wb[9 + i * 3 + 1] * M[3 + c] + Wb[9 + i * 3 + 2] * M[6 + c];
        } else {
            v = w == 0 ? R2[(r - 3) * 3 + c - 3] : (ds ? X[(r - 3) * 3 + c - 3] : (r == c ? 1.0 : 0.0));
        }
        (w == 0 ? L.Gp : L.Gg)[r * 6 + c] = v;
    }
}

// ---------------------------------------------------------------- per-corner models
// Pinhole (cvProjectPoints2Internal order).  Float32 pixel and D = d(u,v)/dXc (2x3).
// PRISM: 0 k1..k6 (RATIONAL: k4..k6), 1 + thin prism s1..s4, 2 + the tilted sensor (tau_x, tau_y):
// tm = matTilt (3 x 3, row-major; computeTiltProjectionMatrix, formed on the host in FP64 --
// mcc_create), vecTilt = matTilt (xd0, yd0, 1), (xd, yd) = vecTilt(0..1) / vecTilt(2), and the 2 x 2
// dMatTilt = (matTilt(r, c) vecTilt(2) - matTilt(2, c) vecTilt(r)) / vecTilt(2)^2 in the chain
template <bool RATIONAL, int PRISM>
__device__ __forceinline__ void pinhole_corner(const double* R, const double* T, const double* k,
                                               double fx, double fy, double cx, double cy,
                                               double X, double Y, double Z, double* Yr,
                                               float& u, float& v, double* D, const double* tm = nullptr) {
    double x, y, z, r2, r4, r6, cdist, icdist2;
    double t0 = 0.0, t1 = 0.0, t2 = 1.0, ip = 1.0;   // vecTilt, invProj (PRISM == 2)
    {
#pragma clang fp contract(off)
        Yr[0] = R[0] * X + R[1] * Y + R[2] * Z;
        Yr[1] = R[3] * X + R[4] * Y + R[5] * Z;
        Yr[2] = R[6] * X + R[7] * Y + R[8] * Z;
        x = Yr[0] + T[0];
        y = Yr[1] + T[1];
        z = Yr[2] + T[2];
        z = z ? 1. / z : 1;
        x *= z;
        y *= z;
        r2 = x * x + y * y;
        r4 = r2 * r2;
        r6 = r4 * r2;
        const double a1 = 2 * x * y, a2 = r2 + 2 * x * x, a3 = r2 + 2 * y * y;
        cdist = 1 + k[0] * r2 + k[1] * r4 + k[4] * r6;
        icdist2 = RATIONAL ? 1. / (1 + k[5] * r2 + k[6] * r4 + k[7] * r6) : 1.0;
        double xd = (RATIONAL ? x * cdist * icdist2 : x * cdist) + k[2] * a1 + k[3] * a2;
        double yd = (RATIONAL ? y * cdist * icdist2 : y * cdist) + k[2] * a3 + k[3] * a1;
        if (PRISM) {
            xd = xd + k[8] * r2 + k[9] * r4;
            yd = yd + k[10] * r2 + k[11] * r4;
        }
        if (PRISM == 2) {   // matTilt * Vec3d(xd0, yd0, 1): Matx's row sums, left to right
            t0 = tm[0] * xd + tm[1] * yd + tm[2];
            t1 = tm[3] * xd + tm[4] * yd + tm[5];
            t2 = tm[6] * xd + tm[7] * yd + tm[8];
            ip = t2 ? 1. / t2 : 1;
            xd = ip * t0;
            yd = ip * t1;
        }
        u = (float)(xd * fx + cx);
        v = (float)(yd * fy + cy);
    }
    // derivative of the distortion map w.r.t. the normalised point (x, y)
    const double cc = cdist * icdist2;
    const double dc = k[0] + 2 * k[1] * r2 + 3 * k[4] * r4;
    double g = dc * icdist2;
    if (RATIONAL) g -= cdist * icdist2 * icdist2 * (k[5] + 2 * k[6] * r2 + 3 * k[7] * r4);
    double P1 = 0.0, P2 = 0.0;
    if (PRISM) { P1 = k[8] + 2 * r2 * k[9]; P2 = k[10] + 2 * r2 * k[11]; }
    const double xy2g = 2 * x * y * g;
    double m00 = cc + 2 * x * x * g + 2 * k[2] * y + 6 * k[3] * x + 2 * x * P1;
    double m01 = xy2g + 2 * k[2] * x + 2 * k[3] * y + 2 * y * P1;
    double m10 = xy2g + 2 * k[2] * x + 2 * k[3] * y + 2 * x * P2;
    double m11 = cc + 2 * y * y * g + 6 * k[2] * y + 2 * k[3] * x + 2 * y * P2;
    if (PRISM == 2) {   // the tilt's 2 x 2 Jacobian (dMatTilt) after the distortion map
        const double ip2 = ip * ip;
        const double d00 = (tm[0] * t2 - tm[6] * t0) * ip2, d01 = (tm[1] * t2 - tm[7] * t0) * ip2;
        const double d10 = (tm[3] * t2 - tm[6] * t1) * ip2, d11 = (tm[4] * t2 - tm[7] * t1) * ip2;
        const double n00 = d00 * m00 + d01 * m10, n01 = d00 * m01 + d01 * m11;
        const double n10 = d10 * m00 + d11 * m10, n11 = d10 * m01 + d11 * m11;
        m00 = n00; m01 = n01; m10 = n10; m11 = n11;
    }
    const double fzx = fx * z, fzy = fy * z;
    D[0] = fzx * m00;
    D[1] = fzx * m01;
    D[2] = -fzx * (m00 * x + m01 * y);
    D[3] = fzy * m10;
    D[4] = fzy * m11;
    D[5] = -fzy * (m10 * x + m11 * y);
}

// Mei omnidirectional model (src/omnidir.cpp:141-208 order).
__device__ __forceinline__ void omni_corner(const double* R, const double* T, const double* k,
                                            double f0, double f1, double c0, double c1, double s,
                                            double xi, double X, double Y, double Z, double* Yr,
                                            float& u, float& v, double* D) {
    double Xc[3], nrm, Xs[3], xu0, xu1, r2, r4;
    {
#pragma clang fp contract(off)
        Yr[0] = R[0] * X + R[1] * Y + R[2] * Z;
        Yr[1] = R[3] * X + R[4] * Y + R[5] * Z;
        Yr[2] = R[6] * X + R[7] * Y + R[8] * Z;
        Xc[0] = Yr[0] + T[0];
        Xc[1] = Yr[1] + T[1];
        Xc[2] = Yr[2] + T[2];
        nrm = sqrt(Xc[0] * Xc[0] + Xc[1] * Xc[1] + Xc[2] * Xc[2]);
        const double inrm = 1. / nrm;
        Xs[0] = Xc[0] * inrm;
        Xs[1] = Xc[1] * inrm;
        Xs[2] = Xc[2] * inrm;
        xu0 = Xs[0] / (Xs[2] + xi);
        xu1 = Xs[1] / (Xs[2] + xi);
        r2 = xu0 * xu0 + xu1 * xu1;
        r4 = r2 * r2;
        const double k1 = k[0], k2 = k[1], p1 = k[2], p2 = k[3];
        const double xd0 = xu0 * (1 + k1 * r2 + k2 * r4) + 2 * p1 * xu0 * xu1 + p2 * (r2 + 2 * xu0 * xu0);
        const double xd1 = xu1 * (1 + k1 * r2 + k2 * r4) + p1 * (r2 + 2 * xu1 * xu1) + 2 * p2 * xu0 * xu1;
        u = (float)(f0 * xd0 + s * xd1 + c0);
        v = (float)(f1 * xd1 + c1);
    }
    const double k1 = k[0], k2 = k[1], p1 = k[2], p2 = k[3];
    const double r_1 = 1.0 / nrm, r_3 = r_1 * r_1 * r_1;
    const double den = 1.0 / (Xs[2] + xi);
    const double a00 = den, a02 = -Xs[0] * den * den, a11 = den, a12 = -Xs[1] * den * den;
    const double t1 = 2 * k1 * xu0 + 4 * k2 * xu0 * r2;
    const double t2 = 2 * k1 * xu1 + 4 * k2 * xu1 * r2;
    const double b00 = k2 * r4 + 6 * p2 * xu0 + 2 * p1 * xu1 + xu0 * t1 + k1 * r2 + 1;
    const double b01 = 2 * p1 * xu0 + 2 * p2 * xu1 + xu0 * t2;
    const double b10 = 2 * p1 * xu0 + 2 * p2 * xu1 + xu1 * t1;
    const double b11 = k2 * r4 + 2 * p2 * xu0 + 6 * p1 * xu1 + xu1 * t2 + k1 * r2 + 1;
    const double q00 = f0 * b00 + s * b10, q01 = f0 * b01 + s * b11;
    const double q10 = f1 * b10, q11 = f1 * b11;
    const double w00 = q00 * a00, w01 = q01 * a11, w02 = q00 * a02 + q01 * a12;
    const double w10 = q10 * a00, w11 = q11 * a11, w12 = q10 * a02 + q11 * a12;
    const double d0 = w00 * Xc[0] + w01 * Xc[1] + w02 * Xc[2];
    const double d1 = w10 * Xc[0] + w11 * Xc[1] + w12 * Xc[2];
    D[0] = w00 * r_1 - d0 * r_3 * Xc[0];
    D[1] = w01 * r_1 - d0 * r_3 * Xc[1];
    D[2] = w02 * r_1 - d0 * r_3 * Xc[2];
    D[3] = w10 * r_1 - d1 * r_3 * Xc[0];
    D[4] = w11 * r_1 - d1 * r_3 * Xc[1];
    D[5] = w12 * r_1 - d1 * r_3 * Xc[2];
}

// ---------------------------------------------------------------- photo back-substitution
// dp = z - sum_e Y_e^T dg_e (z = Hpp^-1 gp, Y_e = Hgp_e Hpp^-1) for one photo (one thread);
// used by k_backsub.
__device__ __forceinline__ void photo_delta(const int* photo_ptr, const int* gblock, const double* Y,
                                           const double* zp, const double* dg, int p, double t[6]) {
    const double* z = zp + 6 * (size_t)p;
#pragma unroll
    for (int k = 0; k < 6; ++k) t[k] = z[k];
    for (int e = photo_ptr[p]; e < photo_ptr[p + 1]; ++e) {
        const int g = gblock[e];
        if (g < 0) continue;
        const double* Ye = Y + 36 * (size_t)e;
        const double* d = dg + 6 * g;
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            double s = 0.0;
#pragma unroll
            for (int i = 0; i < 6; ++i) s += Ye[i * 6 + k] * d[i];
            t[k] -= s;
        }
    }
}

// fused path: dp = z - W dg with the photo's 6 x m pending-update matrix (k_linearize phase E)
__device__ __forceinline__ void photo_delta_w(const double* W, int m, const double* zp, const double* dg, int p,
                                             double t[6]) {
    const double* z = zp + 6 * (size_t)p;
    const double* Wp = W + (size_t)p * 6 * m;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        double s = 0.0;
        for (int c = 0; c < m; ++c) s += Wp[k * m + c] * dg[c];
        t[k] = z[k] - s;
    }
}

// ---------------------------------------------------------------- cross-workgroup hand-off
// Publish this workgroup's global stores and take a ticket; returns true (uniformly) in the
// last of `expected` arrivals, which then sees every other arrival's stores.  Agent-scope
// release/acquire as in /opt/skills/guides/cdna_hip_programming.md section 6 (G16); the last
// arriver resets the counter for the next launch.
__device__ __forceinline__ bool arrive_last(int* counter, int expected) {
    __shared__ int last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int t = __hip_atomic_fetch_add(counter, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = (t == expected - 1);
        if (last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(counter, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    __syncthreads();
    return last;
}

// Write-through (sc1) hand-off without release/acquire fences, MI355X_MICROARCH.md section
// "visibility", Valid forms table row 1: every handed-off double is stored with an 8-B agent-scope
// relaxed atomic store (global_store sc1), every storing wave drains vmcnt(0) before the
// workgroup barrier, ONE lane adds to the counter, the workgroup whose add came last loads every
// handed-off double with sc1 loads after a barrier.  (A release fence here writes back the XCD
// L2's freshly dirtied lines of the whole linearisation: ~6 us per workgroup.)
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) int gi32;
__device__ __forceinline__ void st_sc1(double* p, double v) {
    __hip_atomic_store((gu64*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// two doubles (16-B aligned) in one 16-B write-through store: MI355X_MICROARCH.md prices 8-B
// `sc1` stores at 2.7x the per-byte time of 16-B ones (one fabric write per lane each)
typedef double f64x2_t __attribute__((ext_vector_type(2)));
// The s_nop covers the VMEM store-data hazard the compiler does not see through inline asm: a store of
// more than 64 bits whose data VGPRs the next VALU instruction overwrites needs a wait state (k_group's
// slot stores, round 5: the compiler reused the first store's data registers for the next address at
// once, and the slots held addresses)
__device__ __forceinline__ void st_sc1_x2(double* p, double a, double b) {
    f64x2_t v;
    v.x = a;
    v.y = b;
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ double ld_sc1(const double* p) {
    return __longlong_as_double((long long)__hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ bool arrive_last_sc1(int* counter, int expected, long long* stamp = nullptr) {
    __shared__ int last_sc1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave
    __syncthreads();
    SSTAMP(stamp, 0, 0);
    if (threadIdx.x == 0) {
        const int t = __hip_atomic_fetch_add((gi32*)counter, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last_sc1 = (t == expected - 1);
        if (last_sc1) __hip_atomic_store((gi32*)counter, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    return last_sc1;
}

// packed upper-triangle index t -> (i, j), row i holding m - i entries
__device__ __forceinline__ void packed_ij(int t, int m, int& i, int& j) {
    int rem = t, row = 0;
    while (rem >= m - row) { rem -= m - row; ++row; }
    i = row;
    j = row + rem;
}
// the same in closed form (no loop: row i starts at i m - i (i - 1) / 2; a float root, then at most
// one step either way), for m <= 128
__device__ __forceinline__ void packed_ij_fast(int t, int m, int& i, int& j) {
    const float b = 2.0f * m + 1.0f;
    int r = (int)((b - sqrtf(fmaxf(b * b - 8.0f * (float)t, 0.0f))) * 0.5f);
    r = r < 0 ? 0 : (r > m - 1 ? m - 1 : r);
    const int s0 = r * m - r * (r - 1) / 2;
    if (s0 > t) --r;
    else if (t >= s0 + (m - r)) ++r;
    i = r;
    j = r + (t - (r * m - r * (r - 1) / 2));
}

// sum_{q < n} p[q * stride] in q order with sc1 loads issued 24 at a time (one memory round
// trip for the group sizes of a few hundred to ~600 photos)
__device__ __forceinline__ double sum_sc1(const double* p, int n, size_t stride) {
    constexpr int B = 24;
    double v = 0.0;
    for (int q0 = 0; q0 < n; q0 += B) {
        double b[B];
#pragma unroll
        for (int u = 0; u < B; ++u) b[u] = ld_sc1(p + (size_t)min(q0 + u, n - 1) * stride);
#pragma unroll
        for (int u = 0; u < B; ++u) v += q0 + u < n ? b[u] : 0.0;
    }
    return v;
}

// ---------------------------------------------------------------- peer transport (PeerCtx)
// System-scope relaxed 8-B stores / loads (global_store / global_load sc0 sc1): write-through to
// the owner's memory over xGMI, reads from memory (the inbox is uncached besides).  No fence: an
// LL word is valid on its own once its epoch half matches.
__device__ __forceinline__ void st_sys(unsigned long long* p, unsigned long long w) {
    __hip_atomic_store((gu64*)p, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ unsigned long long ld_sys(const unsigned long long* p) {
    return __hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ size_t peer_word(const PeerCtx& pc, unsigned ep, int src, int t) {
    return ((size_t)(ep & 1u) * pc.nranks + src) * 2 * (size_t)pc.Lc + 2 * (size_t)t;
}
// value t of this rank -> every peer's inbox (two LL words: low and high 32 bits)
__device__ __forceinline__ void peer_send(const PeerCtx& pc, unsigned ep, int t, double v) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v), e = (unsigned long long)ep << 32;
    const size_t w = peer_word(pc, ep, pc.rank, t);
    for (int q = 0; q < pc.nranks; ++q) {
        if (q == pc.rank) continue;
        unsigned long long* d = pc.peers[q] + w;
        st_sys(d, e | (b & 0xffffffffull));
        st_sys(d + 1, e | (b >> 32));
    }
}
// value t of rank q from this rank's inbox; spins until both words carry epoch ep, or gives up
// (timeout set, returns 0) once t0 + pc.timeout has passed
__device__ __forceinline__ double peer_recv(const PeerCtx& pc, unsigned ep, int q, int t, long long t0, bool& timeout) {
    const unsigned long long* s = pc.inbox + peer_word(pc, ep, q, t);
    for (;;) {
        const unsigned long long a = ld_sys(s), b = ld_sys(s + 1);
        if ((unsigned)(a >> 32) == ep && (unsigned)(b >> 32) == ep)
            return __longlong_as_double((long long)(((b & 0xffffffffull) << 32) | (a & 0xffffffffull)));
        if (timeout || (long long)__builtin_amdgcn_s_memrealtime() - t0 > pc.timeout) {
            timeout = true;
            return 0.0;
        }
        __builtin_amdgcn_s_sleep(2);
    }
}
// sum over ranks in rank order (identical bits on every rank); own = this rank's value
__device__ __forceinline__ double peer_sum(const PeerCtx& pc, unsigned ep, int t, double own, long long t0, bool& timeout) {
    double s = 0.0;
    for (int q = 0; q < pc.nranks; ++q) s += q == pc.rank ? own : peer_recv(pc, ep, q, t, t0, timeout);
    return s;
}
// The exchange of the packed system held in vals[0, Lc) (global, this workgroup's own copy):
// every thread sends its entries, then replaces them with the rank-ordered sums.  Returns false
// (state error bit 2, done) when a peer did not deliver within the timeout.  Whole workgroup.
__device__ __forceinline__ bool peer_exchange(const PeerCtx& pc, State* st, double* vals, bool send = true) {
    __shared__ unsigned ep_s;
    __shared__ int to_s;
    const int tid = threadIdx.x;
    const long long tx0 = (long long)__builtin_amdgcn_s_memrealtime();   // exchange time (thread 0's)
    if (tid == 0) {
        ep_s = st->epoch + 1u;
        to_s = 0;
    }
    __syncthreads();
    const unsigned ep = ep_s;
    if (send)
        for (int t = tid; t < pc.Lc; t += blockDim.x) peer_send(pc, ep, t, vals[t]);
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    bool timeout = false;
    for (int t = tid; t < pc.Lc; t += blockDim.x) vals[t] = peer_sum(pc, ep, t, vals[t], t0, timeout);
    if (timeout) to_s = 1;
    __syncthreads();
    if (tid == 0) {
        st->epoch = ep;
        st->xchg_ticks += (long long)__builtin_amdgcn_s_memrealtime() - tx0;   // mcc_timing_exchange
        if (to_s) {
            st->error |= kErrPeerTimeout;
            st->done = 1;
        }
    }
    return !to_s;
}

// The stop-test norm slot w (0: normG2, 1: normX2) the final arriver writes into the packed system.
// A photo block that was not positive definite on THIS rank (its workgroup set kErrPhotoNotPD before
// its ticket) turns normX2 into a NaN: the exchange's sum (peer transport or RCCL) carries the NaN to
// every rank, and every rank's solve_global stops on the same step with the same error, so the
// ranks' replicated camera blocks never diverge (a rank-local stop would leave the other ranks
// solving a system without its shard).  normX2 is a sum of squared float32 parameters, NaN only
// when the state itself is, which is an error too.
// err: State::error, loaded by the caller with its other loads (photo_error), so the flag costs no
// round trip of its own on the final arriver's path
__device__ __forceinline__ int photo_error(State* st) {
    return __hip_atomic_load(&st->error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double photo_flag_norm(int err, int w, double v) {
    return w == 1 && (err & kErrPhotoNotPD) ? __builtin_nan("") : v;
}

template <bool LARGE>
__device__ __forceinline__ void solve_global(const SolveCtx& a, double* S, double* r, double normG2, double normX2,
                                             const WarmCtx* warm = nullptr, const double* Iv = nullptr);

__device__ __forceinline__ unsigned ld_agent_u32(const unsigned* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// The fused step's final arriver, each thread before its first write of the packed system: the
// spare's acknowledgement (ack, loaded with the thread's batch) must be this update launch's (want =
// the iteration every workgroup of the launch read + 1).  Polls (sc1 loads) up to LinArgs::spare_wait; the
// spare is the grid's last workgroup and the other photos have exited, so it runs unless the device is
// held by others.  false: gave up (*to = 1; the step fails at the next barrier, spare_failed).
__device__ __forceinline__ bool spare_wait(const LinArgs& a, unsigned ack, unsigned want, int* to) {
    if (ack == want) return true;
    if (threadIdx.x == 0 && a.solve.sstats)   // (statistics: a step that waited)
        atomicAdd(reinterpret_cast<unsigned long long*>(a.solve.sstats + 4), 1ull);
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    do {
        __builtin_amdgcn_s_sleep(2);
        if (ld_agent_u32(&a.state->spare_ack) == want) return true;
    } while ((long long)__builtin_amdgcn_s_memrealtime() - t0 < a.spare_wait);
    *to = 1;
    return false;
}
// after a barrier behind every thread's spare_wait: the spare never acknowledged -> fail the step
// (MCC_ETIMEOUT), stop the loop.  Neither the state nor the solve is written.  The packed system may be:
// each thread writes its entries as soon as its own spare_wait returns, so when the acknowledgement
// lands at the bound some threads have written theirs and the others gave up.  That copy is read only
// as the next update launch's spare input (a pending update); a new optimisation (mcc_set_params)
// starts with none, so a failed step's packed system is never inverted
// (tests/test_warm_solve.py::test_fused_spare_timeout_fails_the_step runs one on the same handle)
__device__ __forceinline__ bool spare_failed(State* st, int ack_to) {
    if (!ack_to) return false;
    if (threadIdx.x == 0) {
        atomicOr(&st->error, kErrWarmTimeout);
        st->done = 1;
    }
    return true;
}
__device__ __forceinline__ void small_inverse(const LinArgs& a, double* A, bool ack);

// ---------------------------------------------------------------- k_linearize
// Diagnostic builds (-DMCC_DIAG, libmcc_diag.so only) stamp s_memtime at phase boundaries.
// The m <= 30 single-kernel step (a.fused); m > 30 takes the split step below.
template <int MODEL, bool RATIONAL, int PRISM>
__global__ __launch_bounds__(256, 2) void k_linearize(LinArgs a) {
    static_assert(PRISM != 2, "the tilted sensor takes the split step (mcc_create)");
    State* st = a.state;
    const int photo = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    if (photo == a.n_photos) {   // the spare workgroup (a.ssinv): the previous system's inverse
        small_inverse(a, smem, true);
        return;
    }
    // ---- round trip 1: everything indexed by the photo alone
    const int done = st->done, pending = st->pending;
    const double alpha_prev = st->alpha;   // step factor of the pending update
    const int e0 = a.photo_ptr[photo];
    const int ne = a.photo_ptr[photo + 1] - e0;
    if (done) return;
    STAMP(0);
    RSTAMP(14);
#ifdef MCC_DIAG
    if (tid == 0 && a.stamps) {   // placement: HW_ID (cu/se/simd/wave), XCC_ID; and the edge count
        const unsigned hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));
        const unsigned xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11));
        a.stamps[kStampStride * (size_t)photo + 25] = ((long long)xcc << 32) | hw;
        a.stamps[kStampStride * (size_t)photo + 27] = ne;
    }
#endif
    EdgeLds* el = reinterpret_cast<EdgeLds*>(smem);
    PhotoLds& P = *reinterpret_cast<PhotoLds*>(smem + (size_t)ne * (sizeof(EdgeLds) / sizeof(double)));
    double* ctab = reinterpret_cast<double*>(&P + 1);   // [C][kCamStride] = {R, Jl, T}
    double* ktab = ctab + kCamStride * a.n_cams;         // [C][kIntrStride] intrinsics
    float* cs = reinterpret_cast<float*>(ktab + kIntrStride * a.n_cams);   // [5][max_cpp] corners
    const int c0 = a.photo_corner[photo];
    const int ncs = a.photo_corner[photo + 1] - c0;
    float* xg = a.x + a.global_dim + 6 * (size_t)photo;

    // ---- phase 0.  wave 0: photo parameters, pending-update operands (registers);
    // wave 1: camera / double-side / intrinsics tables; waves 2-3: the photo's corners -> LDS;
    // every thread < ne: its edge record
    double part = 0.0, lov = 0.0;
    float xov = 0.f;
    if (wave == 0) {
        if (lane < 6) xov = xg[lane];
        else if (lane < 8) P.nrm[lane - 6] = a.photo_norm[2 * (size_t)photo + lane - 6];   // k_backsub flush
        else if (lane < 10) P.cn[lane - 8] = lane == 8 ? st->cam_normG2 : st->cam_normX2;
        else if (lane == 10) P.iter0 = st->iter;
        if (pending) {
            if (lane < 6) lov = a.zp[6 * (size_t)photo + lane];   // z' = Hpp^-1 gp
            // lane l < 60: k = l % 6, columns l / 6 + 10 u (m <= 30): sum_col W[k][col] dg[col].
            // W (written by the previous step) is indexed by the photo alone, so every operand
            // of the pending update arrives in this first round trip.
            const int k = lane % 6, c = lane / 6, m = a.global_dim;
            if (lane < 60) {
                const double* Wk = a.W + (size_t)photo * 6 * m + (size_t)k * m;
                double w[3], d[3];
#pragma unroll
                for (int u = 0; u < 3; ++u) {
                    const int col = c + 10 * u;
                    w[u] = col < m ? Wk[col] : 0.0;
                    d[u] = col < m ? a.dg[col] : 0.0;
                }
#pragma unroll
                for (int u = 0; u < 3; ++u) part += w[u] * d[u];
            }
        }
    } else if (wave == 1) {
        if (lane < a.n_cams) {
            const int c = lane;
            double om2[3], T2[3];
            if (MODEL == MCC_MODEL_DOUBLESIDE) {
#pragma unroll
                for (int k = 0; k < 3; ++k) { om2[k] = a.cam_rt[6 * c + k]; T2[k] = a.cam_rt[6 * c + 3 + k]; }
            } else if (c == 0) {
#pragma unroll
                for (int k = 0; k < 3; ++k) { om2[k] = 0.0; T2[k] = 0.0; }   // src/mymulticalib.cpp:721-725
            } else {
#pragma unroll
                for (int k = 0; k < 3; ++k) { om2[k] = a.x[6 * (c - 1) + k]; T2[k] = a.x[6 * (c - 1) + 3 + k]; }
            }
            double* kt = ktab + kIntrStride * c;
            const float* Kc = a.K + 9 * c;
            kt[0] = Kc[0]; kt[1] = Kc[4]; kt[2] = Kc[2]; kt[3] = Kc[5]; kt[4] = Kc[1];
            kt[5] = MODEL == MCC_MODEL_OMNI ? (double)a.xi[c] : 0.0;
            const int nd = a.nd;
#pragma unroll
            for (int q = 0; q < 12; ++q) kt[6 + q] = q < nd ? (double)a.D[nd * c + q] : 0.0;
            Rot r2;
            rodrigues_v2m(om2, r2);
            double J[9];
            so3_jac(om2, r2, +1.0, J);
            double* ct = ctab + kCamStride * c;
#pragma unroll
            for (int k = 0; k < 9; ++k) { ct[k] = r2.R[k]; ct[9 + k] = J[k]; }
#pragma unroll
            for (int k = 0; k < 3; ++k) ct[18 + k] = T2[k];
        } else if (lane == 63 && a.has_back) {
            double dsr[3];
            if (MODEL == MCC_MODEL_DOUBLESIDE) {
#pragma unroll
                for (int k = 0; k < 3; ++k) { dsr[k] = a.x[k]; P.dst[k] = a.x[3 + k]; }
            } else {
#pragma unroll
                for (int k = 0; k < 3; ++k) { dsr[k] = a.ds_rt[k]; P.dst[k] = a.ds_rt[3 + k]; }
            }
            Rot rd;
            rodrigues_v2m(dsr, rd);
            double J[9];
            so3_jac(dsr, rd, -1.0, J);
#pragma unroll
            for (int k = 0; k < 9; ++k) { P.Rds[k] = rd.R[k]; P.Jrds[k] = J[k]; }
        }
    } else {
        // wave 2 lanes < ne: the edge records (off wave 0's pending-update path)
        for (int le = tid - 128; le < ne; le += 64) {
            const int4 info = a.edge_info[e0 + le];
            EdgeLds& L = el[le];
            L.cam = info.x; L.side = info.y; L.off = info.z - c0; L.n = info.w; L.edge = e0 + le;
        }
        // the photo's corners are contiguous (photo-major layout): stage all five streams
        for (int q = tid - 128; q < ncs; q += 128) {
            const size_t c = (size_t)c0 + q;
            cs[q] = a.obj_x[c];
            cs[a.max_cpp + q] = a.obj_y[c];
            cs[2 * a.max_cpp + q] = a.obj_z[c];
            cs[3 * a.max_cpp + q] = a.img_u[c];
            cs[4 * a.max_cpp + q] = a.img_v[c];
        }
    }
    STAMP(16);
    if (wave == 0) {
        if (pending) {
            // fused back-substitution of the previous step: dp_k = z'_k - sum_c part(k, c),
            // the ten partials of component k summed in c order through LDS by lane k
            if (lane < 60) P.dgl[lane] = part;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (lane < 6) {
                double tq = lov;
#pragma unroll
                for (int c = 0; c < 10; ++c) tq -= P.dgl[6 * c + lane];
                const float G = (float)(alpha_prev * tq);   // G = alpha*delta -> CV_32F (:491-496)
                const float xn = xov + G;                   // x = x + G (:501)
                xg[lane] = xn;
                P.xp[lane] = xn;
                P.dgl[64 + lane] = (double)G;
            }
        } else if (lane < 6) {
            P.xp[lane] = xov;
        }
        STAMP(18);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        if (lane == 0) {   // photo Rodrigues, shared by every edge of the photo
            if (pending) {   // norms of the applied update (independent of the Rodrigues chain)
                double g2 = 0.0, x2 = 0.0;
#pragma unroll
                for (int q = 0; q < 6; ++q) {
                    g2 += P.dgl[64 + q] * P.dgl[64 + q];
                    x2 += P.xp[q] * P.xp[q];
                }
                a.photo_norm[2 * (size_t)photo] = g2;
                a.photo_norm[2 * (size_t)photo + 1] = x2;
                P.nrm[0] = g2;
                P.nrm[1] = x2;
            }
            const double om1[3] = {P.xp[0], P.xp[1], P.xp[2]};
            Rot r1;
            rodrigues_v2m(om1, r1);
            double J[9];
            so3_jac(om1, r1, -1.0, J);
#pragma unroll
            for (int k = 0; k < 9; ++k) { P.R1[k] = r1.R[k]; P.Jr1[k] = J[k]; }
        }
        STAMP(19);
    }
    __syncthreads();
    STAMP(1);


    // ---- phase B/C: corner sweep + reduction + chain products, one wave per edge
    for (int base = 0; base < ne; base += 4) {
        const int le = base + wave;
        if (le < ne) {
            EdgeLds& L = el[le];
            // ---- phase A: the wave's edge prologue
            edge_prologue_wave<MODEL>(P, ctab, L, lane);
            wave_sync_lds();
            if (base == 0) STAMP(2);
            const int cam = L.cam, off = L.off, n = L.n;
            double R[9], T[3], kd[12];
#pragma unroll
            for (int q = 0; q < 9; ++q) R[q] = L.R[q];
#pragma unroll
            for (int q = 0; q < 3; ++q) T[q] = L.T[q];
            const double* kt = ktab + kIntrStride * cam;
#pragma unroll
            for (int q = 0; q < 12; ++q) kd[q] = kt[6 + q];
            const double fx = kt[0], fy = kt[1], cx = kt[2], cy = kt[3], sk = kt[4];
            const double xi = kt[5];
            double acc[32];
#pragma unroll
            for (int q = 0; q < 32; ++q) acc[q] = 0.0;
            for (int i = lane; i < n; i += 64) {
                const int c = off + i;   // photo-local corner (staged in LDS)
                const double X = cs[c], Y = cs[a.max_cpp + c], Z = cs[2 * a.max_cpp + c];
                const float ou = cs[3 * a.max_cpp + c], ov = cs[4 * a.max_cpp + c];
                double Yr[3], D[6];
                float u, v;
                if (MODEL == MCC_MODEL_OMNI)
                    omni_corner(R, T, kd, fx, fy, cx, cy, sk, xi, X, Y, Z, Yr, u, v, D);
                else
                    pinhole_corner<RATIONAL, PRISM>(R, T, kd, fx, fy, cx, cy, X, Y, Z, Yr, u, v, D);
                const float euf = ou - u, evf = ov - v;   // fl32(imagePoints - imagePoints2)
                if (a.resid) { a.resid[2 * ((size_t)c0 + c)] = euf; a.resid[2 * ((size_t)c0 + c) + 1] = evf; }
                const double eu = euf, ev = evf;
                double ju[6], jv[6];   // J' rows: [Y x d, d]
                ju[0] = Yr[1] * D[2] - Yr[2] * D[1];
                ju[1] = Yr[2] * D[0] - Yr[0] * D[2];
                ju[2] = Yr[0] * D[1] - Yr[1] * D[0];
                ju[3] = D[0]; ju[4] = D[1]; ju[5] = D[2];
                jv[0] = Yr[1] * D[5] - Yr[2] * D[4];
                jv[1] = Yr[2] * D[3] - Yr[0] * D[5];
                jv[2] = Yr[0] * D[4] - Yr[1] * D[3];
                jv[3] = D[3]; jv[4] = D[4]; jv[5] = D[5];
                int q = 0;
#pragma unroll
                for (int r = 0; r < 6; ++r)
#pragma unroll
                    for (int s = r; s < 6; ++s, ++q) acc[q] = fma(jv[r], jv[s], fma(ju[r], ju[s], acc[q]));
#pragma unroll
                for (int r = 0; r < 6; ++r) acc[21 + r] = fma(jv[r], ev, fma(ju[r], eu, acc[21 + r]));
            }
            if (wave == 0) STAMP(3);
            const double sum = wave_reduce_scatter32(acc, lane);
            const int idx = bfly_index(lane);
            if ((lane & 1) == 0 && idx < 27) {
                if (idx < 21) {
                    int r = 0, rem = idx;
                    while (rem >= 6 - r) { rem -= 6 - r; ++r; }
                    const int s = r + rem;
                    L.A[r * 6 + s] = sum;
                    L.A[s * 6 + r] = sum;
                } else {
                    L.b[idx - 21] = sum;
                }
            }
        }
        // each wave owns its edge: wave-local ordering of the LDS records is enough
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        STAMP(4);
        if (le < ne) {   // X = A' G  (A' symmetric)
            EdgeLds& L = el[le];
            for (int t = lane; t < 72; t += 64) {
                const int w = t / 36, ij = t % 36, i = ij / 6, j = ij % 6;
                const double* G = w ? L.Gg : L.Gp;
                double s = 0.0;
#pragma unroll
                for (int k = 0; k < 6; ++k) s += L.A[i * 6 + k] * G[k * 6 + j];
                (w ? L.Xg : L.Xp)[ij] = s;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (le < ne) {   // H = G^T X, g = G^T b'
            EdgeLds& L = el[le];
            for (int t = lane; t < 120; t += 64) {
                if (t < 108) {
                    const int w = t / 36, ij = t % 36, i = ij / 6, j = ij % 6;
                    const double* Gl = (w == 0) ? L.Gp : L.Gg;
                    const double* X = (w == 1) ? L.Xg : L.Xp;
                    double s = 0.0;
#pragma unroll
                    for (int k = 0; k < 6; ++k) s += Gl[k * 6 + i] * X[k * 6 + j];
                    (w == 0 ? L.Hpp : (w == 1 ? L.Hgg : L.Hgp))[ij] = s;
                } else {
                    const int w = (t - 108) / 6, i = (t - 108) % 6;
                    const double* Gl = w ? L.Gg : L.Gp;
                    double s = 0.0;
#pragma unroll
                    for (int k = 0; k < 6; ++k) s += Gl[k * 6 + i] * L.b[k];
                    (w ? L.gg : L.gp)[i] = s;
                }
            }
        }
    }
    __syncthreads();

    // ---- phase D: photo block Hpp = sum_e Hpp_e, its inverse (register Gauss-Jordan on wave 0,
    // Hpp is SPD), z' = Hpp^-1 gp and the Schur factors Y'_e = Hgp_e Hpp^-1: the reduced camera
    // system is S = sum (Hgg - Y'_a Hgp_b^T), r = sum (gg - Y'_a gp), and the photo step of a
    // global step dg is dp = z' - sum_e Y'_e^T dg_e (no triangular solves anywhere)
    STAMP(5);
    double* gs = P.gs;
    double* Hi = P.Lm;   // Hpp^-1
    double* z = P.z;
    if (wave == 0) {
        // lane i < 6 owns row i of [Hpp | I] (summed over the photo's edges in edge order);
        // lanes >= 6 sum row 0 and stay idle; lanes 6..11 also sum gp
        const int li = lane < 6 ? lane : 0;
        double row[12];
#pragma unroll
        for (int j = 0; j < 6; ++j) { row[j] = 0.0; row[6 + j] = li == j ? 1.0 : 0.0; }
        double gsum = 0.0;
        for (int le = 0; le < ne; ++le) {
#pragma unroll
            for (int j = 0; j < 6; ++j) row[j] += el[le].Hpp[li * 6 + j];
            if (lane >= 6 && lane < 12) gsum += el[le].gp[lane - 6];
        }
        if (lane >= 6 && lane < 12) gs[lane - 6] = gsum;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        double dii = 1.0;
        bool bad = false;
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            const double piv = readlane_f64(row[k], k);
            bad |= !(piv > 0.0);
            const double pv = piv > 0.0 ? piv : 1.0;
            double ip = __builtin_amdgcn_rcp(pv);
            ip = fma(ip, fma(-pv, ip, 1.0), ip);
            if (lane == k) dii = pv;
            const double f = lane == k ? 0.0 : row[k] * ip;
            double pr[12];
#pragma unroll
            for (int j = k + 1; j < 12; ++j) pr[j] = readlane_f64(row[j], k);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int j = k + 1; j < 12; ++j) row[j] -= f * pr[j];
        }
        if (lane < 6) {
            const double id = 1.0 / dii;
            double zi = 0.0;
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                const double h = row[6 + j] * id;
                Hi[lane * 6 + j] = h;
                zi += h * gs[j];
            }
            z[lane] = zi;
        }
        if ((bad || photo == a.fault_photo) && lane == 0) atomicOr(&st->error, kErrPhotoNotPD);
    }
    __syncthreads();
    STAMP(6);
    if (tid >= 36 && tid < 42) a.zp[6 * (size_t)photo + tid - 36] = z[tid - 36];
    else if (tid >= 42 && tid < 48) a.gp_tot[6 * (size_t)photo + tid - 42] = gs[tid - 42];
    for (int t = tid; t < 36 * ne; t += blockDim.x) {
        const int le = t / 36, ij = t % 36, i = ij / 6, j = ij % 6;
        EdgeLds& L = el[le];
        double y = 0.0;
        if (L.has_global) {
#pragma unroll
            for (int k = 0; k < 6; ++k) y += L.Hgp[i * 6 + k] * Hi[k * 6 + j];
        }
        L.Xg[ij] = y;   // Xg (A' Gg scratch) is dead: Y'_e for the products below (W replaces the edge-indexed Y')
    }
    if (tid >= 192 && tid < 197) {   // per camera block (m <= 30: at most 5) the photo's edges in edge order
        const int b = tid - 192;
        int cnt = 0;
        for (int e = 0; e < ne; ++e) {
            const EdgeLds& L = el[e];
            const int g = L.has_global ? (MODEL == MCC_MODEL_DOUBLESIDE ? 0 : L.cam - 1) : -1;
            if (g == b) P.bl[b][min(cnt++, 63)] = e;
        }
        P.bn[b] = min(cnt, 64);
    }
    // ---- phase E (fused step, m <= 30): this photo's packed contribution
    //   S[i][j] (i <= j) = sum_{a: g_a = i/6} sum_{b: g_b = j/6} ([a == b] Hgg_a - Y_a Y_b^T)[i%6][j%6]
    //   r[i] = sum_{a: g_a = i/6} (gg_a - Y_a z)[i%6],  jte_g[i] = sum gg_a[i%6],  norms of the update
    // (k_schur's pair sums, src/multicalib.cpp:565-579 normal equations reduced onto the cameras)
    __syncthreads();
    STAMP(7);
    const int m = a.global_dim, ntri = m * (m + 1) / 2, Lc = ntri + 2 * m + 2, Lcp = (Lc + 1) & ~1;
    double* cv = a.contrib + (size_t)photo * Lcp;   // rows of Lcp (even): 16-B stores of value pairs
    for (int tb = 0; tb < Lcp; tb += blockDim.x) {
        const int t = tb + tid;
        double v = 0.0;
        if (t >= Lc) {
        } else if (t < ntri) {
            int i, j;
            packed_ij(t, m, i, j);
            const int bi = i / 6, bj = j / 6, ii = i % 6, jj = j % 6;
            const int na = P.bn[bi], nb2 = P.bn[bj];
            for (int qa = 0; qa < na; ++qa) {
                const int ea = P.bl[bi][qa];
                const EdgeLds& La = el[ea];
                for (int qb = 0; qb < nb2; ++qb) {
                    const int eb = P.bl[bj][qb];
                    const EdgeLds& Lb = el[eb];
                    double d = 0.0;
#pragma unroll
                    for (int k = 0; k < 6; ++k) d += La.Xg[ii * 6 + k] * Lb.Hgp[jj * 6 + k];
                    v -= d;
                    if (ea == eb) v += La.Hgg[ii * 6 + jj];
                }
            }
        } else if (t < ntri + 2 * m) {
            const int u = t - ntri, w = u / m, i = u % m, bi = i / 6, ii = i % 6;
            for (int qa = 0; qa < P.bn[bi]; ++qa) {
                const EdgeLds& La = el[P.bl[bi][qa]];
                if (w == 0) {
                    double d = 0.0;
#pragma unroll
                    for (int k = 0; k < 6; ++k) d += La.Xg[ii * 6 + k] * gs[k];
                    v += La.gg[ii] - d;
                } else {
                    v += La.gg[ii];
                }
            }
        } else {
            v = P.nrm[t - ntri - 2 * m];
        }
        const double vn = dpp_f64<kDppXor1>(v);   // the odd partner's value (same wave)
        if ((t & 1) == 0 && t < Lcp) st_sc1_x2(cv + t, v, vn);
    }
    STAMP(8);
    RSTAMP(29);
    // ---- level 1: the last photo of a group sums the group in photo order
    const int G = a.group_size, grp = photo / G, g0 = grp * G;
    const int gn = min(G, a.n_photos - g0);   // (the grid may carry the warm solve's spare workgroup)
    const bool grp_last = arrive_last_sc1(a.cnt + grp, gn, a.stamps ? a.stamps + kStampStride * (size_t)photo + 28 : nullptr);
    // the next step's pending-update matrix of this photo (after the ticket: off its drain),
    // W[k][6g + i] = sum over the photo's edges e of camera block g of Y'_e[i][k]
    for (int t = tid; t < 6 * m; t += blockDim.x) {
        const int k = t / m, col = t % m, g = col / 6, i = col % 6;
        double w = 0.0;
        for (int q = 0; q < P.bn[g]; ++q) w += el[P.bl[g][q]].Xg[i * 6 + k];
        a.W[(size_t)photo * 6 * m + t] = w;
    }
    if (!grp_last) {
        RSTAMP(15);
        return;
    }
    STAMP(9);
    for (int tb = 0; tb < Lcp; tb += blockDim.x) {
        const int t = tb + tid;
        const double v = t < Lc ? sum_sc1(a.contrib + (size_t)g0 * Lcp + t, gn, Lcp) : 0.0;
        const double vn = dpp_f64<kDppXor1>(v);
        if ((t & 1) == 0 && t < Lcp) st_sc1_x2(a.gsum + (size_t)grp * Lcp + t, v, vn);
    }
    STAMP(10);
    RSTAMP(30);
    // ---- level 2: the last group sums the groups in order -> packed system
    if (!arrive_last_sc1(a.cnt + a.n_groups, a.n_groups)) { RSTAMP(15); return; }
    STAMP(11);
    RSTAMP(31);
    double* S = smem;            // the edge records are dead: m*m + m doubles for the solve
    double* rr = smem + m * m;
    __shared__ double nrm2[2];
    const int iter0 = P.iter0;   // read before S overwrites the photo record
    const double cnG = P.cn[0], cnX = P.cn[1];
    // the spare's acknowledgement of this launch (small_inverse): no thread writes its packed entries or
    // the state before it has seen it; a thread that gave up (spare_wait's bound) sets ack_to, and the
    // step then fails after the next barrier instead of solving (spare_failed: what a failed step leaves)
#ifdef MCC_NO_SPARE_ACK   // (A/B builds only: the round-4 race, for pricing the acknowledgement)
    const bool spare = false;
#else
    const bool spare = a.ssinv != nullptr;   // (update launches only: enqueue_step)
#endif
    const unsigned want = (unsigned)P.iter0 + 1u;   // (update launches only: spare_wait)
    __shared__ int ack_to;
    if (tid == 0) ack_to = 0;
    __syncthreads();
    auto place = [&](int t, double v) {
        if (t < ntri) {
            int i, j;
            packed_ij_fast(t, m, i, j);
            S[i * m + j] = v;
            S[j * m + i] = v;
        } else if (t < ntri + m) {
            rr[t - ntri] = v;
        } else if (t >= ntri + 2 * m) {
            nrm2[t - ntri - 2 * m] = v;
        }
    };
    const bool peer = a.peer.nranks > 0;
    // the m <= 30 warm solve: the inverse the previous launch's spare workgroup formed (of the system
    // two updates back: this launch's spare is still inverting the last one), loaded with the group
    // sums; used when its tag says which iteration made it (small_inverse)
    constexpr int kIvF = 4;   // m^2 <= 900 doubles over 256 threads
    double ivv[kIvF];
    int ivtag = 0;
    const bool ivuse = a.ssinv && a.fuse_solve && iter0 >= 1;
    if (ivuse) {
        const double* src = a.ssinv + (size_t)((iter0 - 1) & 1) * m * m;
        ivtag = a.ssinv_ok[(iter0 - 1) & 1];
#pragma unroll
        for (int u = 0; u < kIvF; ++u) ivv[u] = src[min(u * (int)blockDim.x + tid, m * m - 1)];
    }
    // entry t's final value (the stop-test norms: photos of every rank + the camera block once), placed
    // in the solve's LDS -- the packed system's global copy is written after the spare's acknowledgement
    auto finish_value = [&](int t, double v, int err) {
        if (t >= ntri + 2 * m) {
            const int w = t - ntri - 2 * m;
            if (iter0 > 0) {
                if (a.rank == 0) v += w ? cnX : cnG;
            } else {
                v = 0.0;
            }
            v = photo_flag_norm(err, w, v);
        }
        if (!peer) place(t, v);
        return v;
    };
    if (Lc <= (int)blockDim.x && a.n_groups <= 24) {
        // one entry per thread (m <= 18), its column of group sums in one batch of loads with no
        // loop around it: a loop's head would wait for the inverse's loads above first
        const int ng = a.n_groups, tt = min(tid, Lc - 1);
        double b[24];
#pragma unroll
        for (int q = 0; q < 24; ++q) b[q] = ld_sc1(a.gsum + (size_t)min(q, ng - 1) * Lcp + tt);
        // the error word after the sums' loads: the compiler makes it uniform (v_readfirstlane) and
        // waits for it at once, which in front of the batch would be a memory round trip of its own;
        // the spare's acknowledgement likewise (normally long there: the spare reads its inputs first)
        const int err_now = photo_error(st);
        // (unconditional: a load under `spare ?` joins the branch with a wait for every load in flight)
        const unsigned ack = ld_agent_u32(&st->spare_ack);
        double v = 0.0;
#pragma unroll
        for (int q = 0; q < 24; ++q) v += q < ng ? b[q] : 0.0;   // group order (sum_sc1's additions)
        if (tid < Lc) v = finish_value(tid, v, err_now);
        // the acknowledgement, loaded with the batch, is tested only now: ahead of the sums its compare
        // held them until every load had landed (+0.4 us per config2 step)
        if (spare_wait(a, spare ? ack : want, want, &ack_to) && tid < Lc) a.packed[tid] = v;
    } else if (spare_wait(a, spare ? ld_agent_u32(&st->spare_ack) : want, want, &ack_to)) {
        for (int t = tid; t < Lc; t += blockDim.x) {
            const double v = sum_sc1(a.gsum + t, a.n_groups, Lcp);
            a.packed[t] = finish_value(t, v, photo_error(st));
        }
    }
    STAMP(17);   // thread 0's share of the assembly done (MCC_DIAG)
    if (peer) {   // multi-GPU: rank-ordered sum of every rank's system, then this rank solves
        if (spare) {
            __syncthreads();
            if (spare_failed(st, ack_to)) { RSTAMP(15); return; }
        }
        if (!peer_exchange(a.peer, st, a.packed)) { RSTAMP(15); return; }
        for (int t = tid; t < Lc; t += blockDim.x) place(t, a.packed[t]);
    }
    if (!a.fuse_solve) { RSTAMP(15); return; }
    double* Iv = smem + m * m + m;   // after S and rr (the host sizes the LDS for it)
    __shared__ int iv_ok;
    if (ivuse) {
#pragma unroll
        for (int u = 0; u < kIvF; ++u) {
            const int t = u * (int)blockDim.x + tid;
            if (t < m * m) Iv[t] = ivv[u];
        }
        if (tid == 0) iv_ok = ivtag == iter0;
    }
    __syncthreads();
    if (spare && spare_failed(st, ack_to)) { RSTAMP(15); return; }
    STAMP(12);
    SolveCtx sc = a.solve;
#ifdef MCC_DIAG
    sc.stamps = a.stamps ? a.stamps + kStampStride * (size_t)photo + 20 : nullptr;   // slots 20..26
#endif
    solve_global<false>(sc, S, rr, nrm2[0], nrm2[1], nullptr, ivuse && iv_ok ? Iv : nullptr);
    STAMP(13);
    RSTAMP(15);
}

// ================================================================ split step (m > 30)
// The large-m step as three kernels, each over its natural unit, so that no workgroup carries a
// long serial chain at low occupancy ("split step"):
//   k_prep   one 16-lane group per photo vertex: the previous step's pending photo update, then
//            one LANE per edge: photo / camera Rodrigues, compose_motion (+ the double-side compose
//            of BACK edges), the float32 composed pose and its Rodrigues, the chain maps ->
//            per-edge records erec (R, T) and echain (Gp, Gg blocks);
//   k_edge   L lanes per edge (64 / L edges per wave): the corner sweep (FP64 projection + 2x6
//            J' rows, float32 residual), the L-lane butterfly of the 27 normal-equation sums, and
//            the chain H = G^T A' G, g = G^T b' -> eh;
//   k_photo  one wave per photo vertex: Hpp = sum_e Hpp_e, its inverse, z', the Schur factors
//            Y'_e = Hgp_e Hpp^-1 and the photo's Schur pair products (k_schur sums them).
// (src/mymulticalib.cpp:468-614, 668-818; src/multicalib.cpp:593-824; src/doubleSide.cpp:288-581)

// float32 composed pose -> R (Rodrigues of the float32 vector, for the projection), T, Jl(fl32 om)
__device__ __forceinline__ void prep_finish(const double* om, const double* Tc, double th, double sn, double cs,
                                            double* R, double* T, double* Jl) {
    double rf[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) { rf[k] = (double)(float)om[k]; T[k] = (double)(float)Tc[k]; }   // :546-553
    Rot rp;
    rodrigues_near(rf, th, sn, cs, rp);
#pragma unroll
    for (int k = 0; k < 9; ++k) R[k] = rp.R[k];
    so3_jac(rf, rp, +1.0, Jl);
}

// One edge's prologue (one lane).  gb: the chain maps' nonzero 3x3 blocks, row-major:
// [0..26]  Gp11, Gp21, Gp22 with Gp = [[Gp11, 0], [Gp21, Gp22]] (photo: J_photo = J' Gp)
// [27..53] Gg11, Gg21, Gg22 with Gg likewise (camera or double-side block)
template <int MODEL, bool BACK>
__device__ __forceinline__ void prep_edge(const double* R1, const double* Jr1, const double* T1, const double* R2,
                                          const double* Jl2, const double* T2, const double* Rds, const double* Jrds,
                                          const double* dst, int side, double* er, double* gb) {
    double* R = er;
    double* T = er + 9;
    Motion f;
    double th3, s3, c3;
    compose(R1, Jr1, T1, R2, Jl2, T2, f, th3, s3, c3);   // compose_motion(photo, camera), :498-500
    double Jl[9], t9[9];
    if (BACK && side == MCC_BACK) {
        // compose_motion(ds, photofront), src/mymulticalib.cpp:503-506 / src/doubleSide.cpp:320-322;
        // R(om_front) is the FP64 composed rotation itself (Rodrigues(om_front) to rounding)
        Rot rf0;
        rf0.th = th3; rf0.s = s3; rf0.c = c3;
        double Jlf[9];
        so3_jac(f.om, rf0, +1.0, Jlf);
        Motion b;
        double th, sn, cs;
        compose(Rds, Jrds, dst, f.R, Jlf, f.T, b, th, sn, cs);
        prep_finish(b.om, b.T, th, sn, cs, R, T, Jl);
        mat3_mul(b.A2, f.A1, t9);          // photo: [[Jl A2b A1, 0], [B2b A1, R2]]  (:509-512)
        mat3_mul(Jl, t9, gb);
        mat3_mul(b.B2, f.A1, gb + 9);
#pragma unroll
        for (int k = 0; k < 9; ++k) gb[18 + k] = R2[k];
        if (MODEL == MCC_MODEL_DOUBLESIDE) {   // ds block: [[Jl A1b, 0], [0, R_front]]  (doubleSide.cpp:398-399)
            mat3_mul(Jl, b.A1, gb + 27);
#pragma unroll
            for (int k = 0; k < 9; ++k) { gb[36 + k] = 0.0; gb[45 + k] = f.R[k]; }
        } else {   // camera block as the reference chains it, omitting dTt/dTf dTf/dRc (:516, hazard A12)
            mat3_mul(b.A2, f.A2, t9);
            mat3_mul(Jl, t9, gb + 27);
            mat3_mul(b.B2, f.A2, gb + 36);
#pragma unroll
            for (int k = 0; k < 9; ++k) gb[45 + k] = (k % 4 == 0) ? 1.0 : 0.0;
        }
    } else {
        prep_finish(f.om, f.T, th3, s3, c3, R, T, Jl);
        mat3_mul(Jl, f.A1, gb);             // photo: [[Jl A1, 0], [0, R2]]
#pragma unroll
        for (int k = 0; k < 9; ++k) { gb[9 + k] = 0.0; gb[18 + k] = R2[k]; }
        if (MODEL == MCC_MODEL_DOUBLESIDE) {   // front edges carry a zero ds block (doubleSide.cpp:335-336)
#pragma unroll
            for (int k = 0; k < 27; ++k) gb[27 + k] = 0.0;
        } else {                               // camera: [[Jl A2, 0], [B2, I]]
            mat3_mul(Jl, f.A2, gb + 27);
#pragma unroll
            for (int k = 0; k < 9; ++k) { gb[36 + k] = f.B2[k]; gb[45 + k] = (k % 4 == 0) ? 1.0 : 0.0; }
        }
    }
}

#ifndef MCC_PREP_GROUP
#define MCC_PREP_GROUP 16
#endif
constexpr int kPrepGroup = MCC_PREP_GROUP;   // lanes per photo vertex in k_prep (64 / kPrepGroup photos per wave)
static_assert(kPrepGroup >= 8 && kPrepGroup <= 64 && (kPrepGroup & (kPrepGroup - 1)) == 0, "k_prep group");
constexpr int kMaxEdgesPerPhoto = 64;   // split step (k_prep's LDS; mcc_create checks)
#ifndef MCC_PREP_WAVES
#define MCC_PREP_WAVES 2           // k_prep waves per SIMD
#endif
// camera vertex c's pose (om, T): DoubleSide's fixed cameras, camera 0 = identity, else x
__device__ __forceinline__ void camera_pose_lds(const double* cam6, int cam, double* om2, double* T2) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        om2[k] = cam6[6 * cam + k];
        T2[k] = cam6[6 * cam + 3 + k];
    }
}
// BACK: the problem has back-side edges (MyMulti doubleSideTransform / DoubleSide), so the
// front-only instantiation carries no second compose
template <int MODEL, bool BACK>
__global__ __launch_bounds__(64, MCC_PREP_WAVES) void k_prep(LinArgs a) {
    const State* st = a.state;
    const int done = st->done;   // tested after the first round trip's loads are issued
    const int tid = threadIdx.x, grp = tid / kPrepGroup, l = tid % kPrepGroup;
    const int photo = blockIdx.x * (64 / kPrepGroup) + grp;
    long long* stp = a.stamps ? a.stamps + kStampStride * (size_t)blockIdx.x + 8 : nullptr;   // MCC_DIAG
    SSTAMP(stp, 0, 0);
    __shared__ double s_v[64 / kPrepGroup][16];
    __shared__ double s_part[64 / kPrepGroup][kMaxEdgesPerPhoto][6];
    __shared__ double s_ph[64 / kPrepGroup][44];   // R1, Jr1, T1, Rds, Jrds, dst (the group's photo)
    // camera poses (rvec, tvec per camera), the previous step's dg and the double-side transform,
    // staged in the first round trip with the photo ranges (no dependent load for them later)
    __shared__ double s_cam[6 * 64], s_dg[128], s_ds[6];   // <= 63 cameras, m <= 128 (mcc_create)
    const bool valid = photo < a.n_photos;
    const int e0 = valid ? a.photo_ptr[photo] : 0;
    const int ne = valid ? a.photo_ptr[photo + 1] - e0 : 0;
    const int pending = st->pending;
    const double alpha_prev = st->alpha;   // step factor of the pending update
    for (int q = tid; q < 6 * a.n_cams; q += 64) {
        const int c = q / 6, k = q % 6;
        s_cam[q] = MODEL == MCC_MODEL_DOUBLESIDE ? (double)a.cam_rt[q]
                                                 : (c == 0 ? 0.0 : (double)a.x[6 * (c - 1) + k]);   // src/mymulticalib.cpp:721-725
    }
    for (int q = tid; q < a.global_dim; q += 64) s_dg[q] = a.dg[q];
    if (BACK && tid < 6) s_ds[tid] = MODEL == MCC_MODEL_DOUBLESIDE ? (double)a.x[tid] : a.ds_rt[tid];
    wave_sync_lds();
    if (done) return;
    float* xg = a.x + a.global_dim + 6 * (size_t)photo;
    // the camera of the lane's first edge: Rodrigues + Jl, independent of the photo update
    int4 info0 = make_int4(0, 0, 0, 0);
    Rot r2;
    double Jl2[9], T2[3];
    if (l < ne) {
        info0 = a.edge_info[e0 + l];
        double om2[3];
        camera_pose_lds(s_cam, info0.x, om2, T2);
        rodrigues_v2m(om2, r2);
        so3_jac(om2, r2, +1.0, Jl2);
    }
    // ---- the previous step's photo update: dp_k = z'_k - sum_e (Y'_e^T dg_g(e))_k in edge order
    // (k_backsub's photo_delta), G = fl32(alpha dp), x = fl32(x + G).  Lane l forms the 6-vector
    // Y'_e^T dg of edges l, l + 16, ... (every load of the photo in flight at once), lane k < 6
    // sums component k over the edges in order.
    float xo = 0.f;
    double zk = 0.0;
    if (valid && l < 6) {
        xo = xg[l];
        if (pending) zk = a.zp[6 * (size_t)photo + l];
    }
    if (valid && pending) {
        for (int le = l; le < ne; le += kPrepGroup) {
            const int g = a.gblock[e0 + le];
            const double* Ye = a.Y + 36 * (size_t)(e0 + le);
            double y[36];
#pragma unroll
            for (int q = 0; q < 36; ++q) y[q] = Ye[q];
            const double* d = s_dg + 6 * (g < 0 ? 0 : g);
            double dv[6];
#pragma unroll
            for (int i = 0; i < 6; ++i) dv[i] = d[i];
#pragma unroll
            for (int k = 0; k < 6; ++k) {
                double sk = 0.0;
#pragma unroll
                for (int i = 0; i < 6; ++i) sk += y[6 * i + k] * dv[i];
                s_part[grp][le][k] = g < 0 ? 0.0 : sk;
            }
        }
    }
    wave_sync_lds();
    double xk = 0.0, Gk = 0.0;
    if (valid && l < 6) {
        float xn = xo;
        if (pending) {
            double t = zk;
            for (int le = 0; le < ne; ++le) t -= s_part[grp][le][l];   // (0 for edges without a global block)
            const float G = (float)(alpha_prev * t);   // G = alpha*delta -> CV_32F (:491-496)
            xn = xo + G;                                // x = x + G (:501)
            xg[l] = xn;
            Gk = (double)G;
        }
        xk = (double)xn;
    }
    if (l < 6) {
        s_v[grp][l] = xk;
        s_v[grp][8 + l] = Gk;
    }
    wave_sync_lds();
    SSTAMP(stp, 1, 0);
    if (!valid) return;
    double* ph = s_ph[grp];
    if (l == 0) {   // ||G||^2, ||x||^2 partials of the applied update (stop test); photo Rodrigues
        if (pending) {
            double g2 = 0.0, x2 = 0.0;
#pragma unroll
            for (int q = 0; q < 6; ++q) {
                g2 += s_v[grp][8 + q] * s_v[grp][8 + q];
                x2 += s_v[grp][q] * s_v[grp][q];
            }
            a.photo_norm[2 * (size_t)photo] = g2;
            a.photo_norm[2 * (size_t)photo + 1] = x2;
        }
        const double om1[3] = {s_v[grp][0], s_v[grp][1], s_v[grp][2]};
        Rot r1;
        rodrigues_v2m(om1, r1);
        so3_jac(om1, r1, -1.0, ph + 9);
#pragma unroll
        for (int k = 0; k < 9; ++k) ph[k] = r1.R[k];
#pragma unroll
        for (int k = 0; k < 3; ++k) ph[18 + k] = s_v[grp][3 + k];
    } else if (BACK && l == 1) {   // the double-side transform (BACK edges; DoubleSide's global block)
        double dsr[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            dsr[k] = s_ds[k];
            ph[39 + k] = s_ds[3 + k];
        }
        Rot rd;
        rodrigues_v2m(dsr, rd);
        so3_jac(dsr, rd, -1.0, ph + 30);
#pragma unroll
        for (int k = 0; k < 9; ++k) ph[21 + k] = rd.R[k];
    }
    wave_sync_lds();
    SSTAMP(stp, 2, 0);
    // ---- one lane per edge
    for (int le = l; le < ne; le += kPrepGroup) {
        const int e = e0 + le;
        int4 info = info0;
        if (le >= kPrepGroup) {   // more edges than lanes: this edge's camera
            info = a.edge_info[e];
            double om2[3];
            camera_pose_lds(s_cam, info.x, om2, T2);
            rodrigues_v2m(om2, r2);
            so3_jac(om2, r2, +1.0, Jl2);
        }
        prep_edge<MODEL, BACK>(ph, ph + 9, ph + 18, r2.R, Jl2, T2, ph + 21, ph + 30, ph + 39, info.y,
                               a.erec + 12 * (size_t)e, a.echain + 54 * (size_t)e);
    }
#ifdef MCC_DIAG
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    SSTAMP(stp, 3, 0);
}

// Reduce-scatter of 32 per-lane values over the L lanes {g, g + 64/L, ...} of one edge (k_edge's
// strided lane map, g = lane % (64/L)): xor 32 and 16 as whole half-wave / row swaps
// (v_permlane32_swap, v_permlane16_swap: two instructions and an add per value pair instead of
// selects around DPP), xor 8 and 4 by DPP inside a row.  In the edge's own numbering
// (sub = lane / (64/L)) this is the fixed tree sub ^ (L/2), ..., ^ 1.  Afterwards the lane holds
// the edge's sums of value indices strided_rs_base<L>(lane) + {0 .. 32/L - 1}.
template <int CTRL>
__device__ __forceinline__ double dpp_f64u(double v) {   // no 'old' operand to initialise
    const unsigned long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)(unsigned)b, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(unsigned)(b >> 32), CTRL, 0xF, 0xF, false);
    return ull_f64((unsigned)lo, (unsigned)hi);
}
template <int L>
__device__ __forceinline__ void strided_reduce_scatter(double* v, int lane) {
    static_assert(L == 32 || L == 16 || L == 8, "lanes per edge");
#pragma unroll
    for (int j = 0; j < 16; ++j) { double p = v[j], q = v[j + 16]; pl32_swap(p, q); v[j] = p + q; }   // lane ^ 32
#pragma unroll
    for (int j = 0; j < 8; ++j) { double p = v[j], q = v[j + 8]; pl16_swap(p, q); v[j] = p + q; }     // lane ^ 16
    {   // lane ^ 8: rotate a row by 8
        const bool hi = (lane & 8) != 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const double send = hi ? v[j] : v[j + 4], keep = hi ? v[j + 4] : v[j];
            v[j] = keep + dpp_f64u<kDppRor8>(send);
        }
    }
    if (L >= 16) {   // lane ^ 4: i - 4 for the upper, i + 4 = i - 12 for the lower
        const bool hi = (lane & 4) != 0;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const double send = hi ? v[j] : v[j + 2], keep = hi ? v[j + 2] : v[j];
            const double p4 = dpp_f64u<kDppRor4>(send), p12 = dpp_f64u<kDppRor12>(send);
            v[j] = keep + (hi ? p4 : p12);
        }
    }
    if (L == 32) {   // lane ^ 2: a quad permutation
        const bool hi = (lane & 2) != 0;
        const double send = hi ? v[0] : v[1], keep = hi ? v[1] : v[0];
        v[0] = keep + dpp_f64u<kDppXor2>(send);
    }
}
template <int L>
__device__ __forceinline__ int strided_rs_base(int lane) {
    return 16 * ((lane >> 5) & 1) + 8 * ((lane >> 4) & 1) + 4 * ((lane >> 3) & 1) + (L >= 16 ? 2 * ((lane >> 2) & 1) : 0) +
           (L == 32 ? ((lane >> 1) & 1) : 0);
}
// packed upper index t < 21 -> (r, s), r <= s, without a loop: r from a 3-bit-per-entry table
__device__ __forceinline__ void tri6(int t, int& r, int& s) {
    constexpr unsigned long long kRow = 0ull | (1ull << 18) | (1ull << 21) | (1ull << 24) | (1ull << 27) |
                                        (1ull << 30) | (2ull << 33) | (2ull << 36) | (2ull << 39) | (2ull << 42) |
                                        (3ull << 45) | (3ull << 48) | (3ull << 51) | (4ull << 54) | (4ull << 57) |
                                        (5ull << 60);
    r = (int)((kRow >> (3 * t)) & 7);
    s = t - 6 * r + r * (r - 1) / 2 + r;   // t - (row start 6r - r(r-1)/2) + r
}

// One edge's chain H = G^T A' G, g = G^T b' from its LDS record (A', b', the chain maps' nonzero
// blocks), by the edge's 16 lanes sq = 0 .. 15 (every lane of the wave calls it: wave-level syncs).
struct EdgeChain {
    double A[36], B[8];
    double Gb[2][28];   // [photo | global] nonzero 3x3 blocks G11, G21, G22 (27 + pad)
    double X[2][6][8];  // X_p = [A' Gp | b'], X_g = A' Gg (rows of 8: 16-B aligned)
};
__device__ __forceinline__ void edge_chain_xh(EdgeChain& CH, int sq, int eq, bool valid, const LinArgs& a) {
    // X_w = A' G_w with G_w = [[G11, 0], [G21, G22]] (A' symmetric): lane (w, i) < 12 forms row i,
    // the zero block skipped (the same FMA sequence as the dense 6 x 6 product minus its exact-zero
    // terms); X_p carries b' as a seventh column, so that G^T X_p also yields g = G^T b'
    if (sq < 12) {
        const int w = sq / 6, i = sq % 6;
        double ar[6], gm[28], xr[8];
        const double2* A2 = reinterpret_cast<const double2*>(CH.A + 6 * i);
        const double2* G2 = reinterpret_cast<const double2*>(CH.Gb[w]);
#pragma unroll
        for (int q = 0; q < 3; ++q) { const double2 v = A2[q]; ar[2 * q] = v.x; ar[2 * q + 1] = v.y; }
#pragma unroll
        for (int q = 0; q < 14; ++q) { const double2 v = G2[q]; gm[2 * q] = v.x; gm[2 * q + 1] = v.y; }
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            double s2 = 0.0;
#pragma unroll
            for (int k = 0; k < 3; ++k) s2 += ar[k] * gm[k * 3 + j];            // G11
#pragma unroll
            for (int k = 0; k < 3; ++k) s2 += ar[3 + k] * gm[9 + k * 3 + j];   // G21
            xr[j] = s2;
            double s3 = 0.0;
#pragma unroll
            for (int k = 0; k < 3; ++k) s3 += ar[3 + k] * gm[18 + k * 3 + j];  // G22
            xr[3 + j] = s3;
        }
        xr[6] = w == 0 ? CH.B[i] : 0.0;
        xr[7] = 0.0;
        double2* X2 = reinterpret_cast<double2*>(CH.X[w][i]);
#pragma unroll
        for (int q = 0; q < 4; ++q) X2[q] = make_double2(xr[2 * q], xr[2 * q + 1]);
    }
    wave_sync_lds();
    // H = G_l^T X_r: eh = [Hpp upper 21 | Hgg upper 21 | Hgp 36 | gp 6 | gg 6].  Lane (T, i) < 9
    // forms rows i and i + 3 of (T = 0) Gp^T [Xp | b'] -> Hpp, gp; (1) Gg^T [Xp | b'] -> Hgp, gg;
    // (2) Gg^T Xg -> Hgg.  Row i < 3 takes G11 and G21, row i + 3 only G22 (zero block skipped).
    if (sq < 9 && valid) {
        const int T = sq / 3, i = sq % 3;
        const double* Gl = CH.Gb[T == 0 ? 0 : 1];
        const double2* X2 = reinterpret_cast<const double2*>(CH.X[T == 2 ? 1 : 0][0]);
        double c11[3], c21[3], c22[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            c11[k] = Gl[k * 3 + i];
            c21[k] = Gl[9 + k * 3 + i];
            c22[k] = Gl[18 + k * 3 + i];
        }
        double h[7], h2[7];
#pragma unroll
        for (int j = 0; j < 7; ++j) { h[j] = 0.0; h2[j] = 0.0; }
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            double xk[8];
#pragma unroll
            for (int q = 0; q < 4; ++q) { const double2 v = X2[4 * k + q]; xk[2 * q] = v.x; xk[2 * q + 1] = v.y; }
            const double c = k < 3 ? c11[k] : c21[k - 3];
#pragma unroll
            for (int j = 0; j < 7; ++j) h[j] += c * xk[j];
            if (k >= 3) {
#pragma unroll
                for (int j = 0; j < 7; ++j) h2[j] += c22[k - 3] * xk[j];
            }
        }
        double* out = a.eh + 90 * (size_t)eq;
        const bool tri = T != 1;
        const int i2 = i + 3;
        const int blk = T == 2 ? 21 : 0;
        double* o1 = tri ? out + blk + 6 * i - i * (i - 1) / 2 - i : out + 42 + 6 * i;
        double* o2 = tri ? out + blk + 6 * i2 - i2 * (i2 - 1) / 2 - i2 : out + 42 + 6 * i2;
#pragma unroll
        for (int j = 0; j < 6; ++j) {
            if (!tri || j >= i) o1[j] = h[j];
            if (!tri || j >= i2) o2[j] = h2[j];
        }
        if (T < 2) {
            out[78 + 6 * T + i] = h[6];
            out[78 + 6 * T + i2] = h2[6];
        }
    }
}

constexpr int kEdgeChunk = 96;    // corners of one edge staged in LDS at a time (k_edge)
#ifndef MCC_EDGE_WAVES
#define MCC_EDGE_WAVES 4            // k_edge waves per SIMD (register budget 128 VGPRs)
#endif
// L lanes per edge (16 or 8), 64 / L edges per one-wave workgroup, lanes strided: edge
// g = lane % (64/L) owns lanes g, g + 64/L, ... (sub = lane / (64/L)), so the butterfly's widest
// exchanges are permlane swaps and the staged corners are read at consecutive LDS addresses.
// L = 8 sweeps an 88-corner edge in 11 full rounds (16 lanes: 5.5), halves the butterfly per
// edge, and stages corners in 48-corner chunks; the chain then runs in passes of 4 edges with 16
// lanes each (edge_chain_xh) so that its LDS fits in the corner area.
template <int MODEL, bool RATIONAL, int PRISM, int L>
__global__ __launch_bounds__(64, (MODEL == MCC_MODEL_OMNI || RATIONAL || PRISM) ? 3 : MCC_EDGE_WAVES) void k_edge(LinArgs a) {
    static_assert(L == 16 || L == 8, "k_edge: 16 or 8 lanes per edge");
    if (a.state->done) return;
    constexpr int GPB = 64 / L;   // edges per workgroup (one wave)
    constexpr int CHK = kEdgeChunk * L / 16;   // corners per staged chunk
    const int tid = threadIdx.x, g = tid % GPB, sub = tid / GPB;
    const int e = blockIdx.x * GPB + g;
    long long* stp = (a.stamps && (int)(blockIdx.x / 2) < a.n_photos)
                         ? a.stamps + kStampStride * (size_t)(blockIdx.x / 2) + 16 + 8 * (blockIdx.x & 1) : nullptr;
    SSTAMP(stp, 0, 0);
    // LDS per wave: the staged corners [stream][corner][edge], reused after the sweep for the chain
    // (A', b', the chain maps' nonzero blocks, X = A' G), and the edge's pose / camera (8.6 KB: 4
    // waves per SIMD)
    __shared__ __attribute__((aligned(16))) union { float C[5][CHK][GPB]; EdgeChain H[4]; } sU;
    __shared__ double sP[GPB][PRISM == 2 ? 40 : 30];   // + matTilt (the tilted sensor)
    __shared__ int sI[GPB][2];   // corner offset and count, re-read per chunk (nothing stays live through the sweep)
    auto& sC = sU.C;
    // a workgroup's edges past the last are swept as empty (no early exit: the chain passes map
    // lanes to edges differently from the sweep when L = 8)
    const bool ev = e < a.n_edges;
    const int4 info = ev ? a.edge_info[e] : make_int4(0, 0, 0, 0);
    const int cam = info.x, off = info.z, n = info.w;
    if (sub == 0) {
        sI[g][0] = off;
        sI[g][1] = n;
    }
    // the edge's corners (contiguous in all five streams) -> LDS, every load in flight at once
    auto stage = [&](int eoff, int c0, int cn) {   // every load of the chunk issued before the first LDS store
        constexpr int PER = CHK / L;
        float v[PER][5];
        int sb = sub;   // opaque: the lane's chunk offsets are recomputed per chunk, not kept live (spilled)
        asm volatile("" : "+v"(sb));
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int i = sb + L * u;
            // 32-bit element index: SGPR base + one VGPR offset per load (saddr form), not a 64-bit
            // address pair per stream, which spilled to scratch
            const unsigned c = (unsigned)(eoff + c0 + (i < cn ? i : 0));
            v[u][0] = a.obj_x[c];
            v[u][1] = a.obj_y[c];
            v[u][2] = a.obj_z[c];
            v[u][3] = a.img_u[c];
            v[u][4] = a.img_v[c];
        }
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int i = sb + L * u;
            if (i < cn) {
#pragma unroll
                for (int f = 0; f < 5; ++f) sC[f][i][g] = v[u][f];
            }
        }
    };
    stage(off, 0, min(n, CHK));
    SSTAMP(stp, 1, 0);
    // the edge's pose and camera (R, T, fx, fy, cx, cy, skew, xi, k[12]) in LDS, re-read by every
    // corner (an opaque offset keeps the compiler from hoisting them into ~50 more VGPRs, which
    // would halve the waves per SIMD)
    {
        double* P = sP[g];
        const double* er = a.erec + 12 * (size_t)(ev ? e : 0);
        const float* Kc = a.K + 9 * cam;
        const int nd = a.nd;
        for (int t = sub; t < (PRISM == 2 ? 39 : 30); t += L) {
            double v;
            if (t >= 30) v = a.tilt[9 * cam + (t - 30)];
            else if (t < 12) v = er[t];
            else if (t < 17) v = (double)Kc[t == 12 ? 0 : t == 13 ? 4 : t == 14 ? 2 : t == 15 ? 5 : 1];
            else if (t == 17) v = MODEL == MCC_MODEL_OMNI ? (double)a.xi[cam] : 0.0;
            else v = t - 18 < nd ? (double)a.D[nd * cam + (t - 18)] : 0.0;
            P[t] = v;
        }
    }
    double acc[32];
#pragma unroll
    for (int q = 0; q < 32; ++q) acc[q] = 0.0;
    wave_sync_lds();
    for (int c0 = 0;; c0 += CHK) {
        const int nn = sI[g][1];
        if (c0 >= nn) break;
        const int cn = min(nn - c0, CHK);
        if (c0 > 0) {
            wave_sync_lds();   // the previous chunk is consumed
            stage(sI[g][0], c0, cn);
        }
        wave_sync_lds();
#pragma unroll 1
        for (int i = sub; i < cn; i += L) {
            int po = 0;
            asm volatile("" : "+v"(po));
            const double* P = sP[g] + po;
            double R[9], T[3], kd[12];
#pragma unroll
            for (int q = 0; q < 9; ++q) R[q] = P[q];
#pragma unroll
            for (int q = 0; q < 3; ++q) T[q] = P[9 + q];
#pragma unroll
            for (int q = 0; q < 12; ++q) kd[q] = P[18 + q];
            const double fx = P[12], fy = P[13], cx = P[14], cy = P[15], sk = P[16], xi = P[17];
            const double X = sC[0][i][g], Y = sC[1][i][g], Z = sC[2][i][g];
            const float ou = sC[3][i][g], ov = sC[4][i][g];
            double Yr[3], D[6];
            float u, v;
            if (MODEL == MCC_MODEL_OMNI)
                omni_corner(R, T, kd, fx, fy, cx, cy, sk, xi, X, Y, Z, Yr, u, v, D);
            else
                pinhole_corner<RATIONAL, PRISM>(R, T, kd, fx, fy, cx, cy, X, Y, Z, Yr, u, v, D, P + 30);
            const float euf = ou - u, evf = ov - v;   // fl32(imagePoints - imagePoints2)
            if (a.resid) {
                const size_t c = (size_t)off + c0 + i;
                a.resid[2 * c] = euf;
                a.resid[2 * c + 1] = evf;
            }
            const double eu = euf, ev = evf;
            double ju[6], jv[6];   // J' rows: [Y x d, d]
            ju[0] = Yr[1] * D[2] - Yr[2] * D[1];
            ju[1] = Yr[2] * D[0] - Yr[0] * D[2];
            ju[2] = Yr[0] * D[1] - Yr[1] * D[0];
            ju[3] = D[0]; ju[4] = D[1]; ju[5] = D[2];
            jv[0] = Yr[1] * D[5] - Yr[2] * D[4];
            jv[1] = Yr[2] * D[3] - Yr[0] * D[5];
            jv[2] = Yr[0] * D[4] - Yr[1] * D[3];
            jv[3] = D[3]; jv[4] = D[4]; jv[5] = D[5];
            int q = 0;
#pragma unroll
            for (int r = 0; r < 6; ++r)
#pragma unroll
                for (int s2 = r; s2 < 6; ++s2, ++q) acc[q] = fma(jv[r], jv[s2], fma(ju[r], ju[s2], acc[q]));
#pragma unroll
            for (int r = 0; r < 6; ++r) acc[21 + r] = fma(jv[r], ev, fma(ju[r], eu, acc[21 + r]));
        }
    }
    SSTAMP(stp, 2, 0);
    // after the sweep: lane indices re-derived from one opaque copy of the thread id, so that only it
    // (not e, g, sub and their addresses) stays live through the sweep at 128 VGPRs
    int tq = tid;
    asm volatile("" : "+v"(tq));
    // the chain in passes of 4 edges, 16 lanes each: pass p takes edges 4p .. 4p + 3 of the
    // workgroup, edge slot gq = tq & 3 with chain lane sq = tq >> 2 (for L = 16 the sweep's own map)
    const int gq = tq & 3, sq = tq >> 2;
    // the chain maps' nonzero blocks (echain: Gp11, Gp21, Gp22, Gg11, Gg21, Gg22) of the first
    // pass, loaded before the butterfly so that it covers their latency
    double gv[4];
    auto load_g = [&](int eq) {
        const double* ec = a.echain + 54 * (size_t)(eq < a.n_edges ? eq : 0);
#pragma unroll
        for (int u = 0; u < 4; ++u) gv[u] = sq + 16 * u < 54 ? ec[sq + 16 * u] : 0.0;
    };
    load_g(blockIdx.x * GPB + gq);
    strided_reduce_scatter<L>(acc, tq);
    SSTAMP(stp, 3, 0);
    const int gs = tq % GPB, base = strided_rs_base<L>(tq);
#pragma unroll
    for (int pass = 0; pass < GPB / 4; ++pass) {
        const int eq = blockIdx.x * GPB + 4 * pass + gq;
        if (pass > 0) load_g(eq);
        wave_sync_lds();   // the corners (pass 0) / the previous pass's records are consumed
        EdgeChain& CH = sU.H[gq];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int t = sq + 16 * u;
            if (t < 54) CH.Gb[t / 27][t % 27] = gv[u];
        }
        if (gs / 4 == pass) {   // this lane's reduced sums belong to an edge of the pass
            EdgeChain& CW = sU.H[gs % 4];
#pragma unroll
            for (int q = 0; q < 32 / L; ++q) {
                const int idx = base + q;
                if (idx < 21) {
                    int r, s2;
                    tri6(idx, r, s2);
                    CW.A[r * 6 + s2] = acc[q];
                    CW.A[s2 * 6 + r] = acc[q];
                } else if (idx < 27) {
                    CW.B[idx - 21] = acc[q];
                }
            }
        }
        wave_sync_lds();
        edge_chain_xh(CH, sq, eq, eq < a.n_edges, a);
    }
#ifdef MCC_DIAG
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    SSTAMP(stp, 4, 0);
}

// One workgroup per group of consecutive photo vertices (at most kPhotoGroup photos and
// kPhotoGroupEdges edges, host-built).  Per photo: Hpp = sum_e Hpp_e and gp (edge order), the
// Cholesky factor Hpp = L L^T and Li = L^-1 (so Hpp^-1 = Li^T Li), z' = Hpp^-1 gp; per edge
// U_e = Hgp_e Li^T (in place of Hgp) and Y'_e = Hgp_e Hpp^-1 = U_e Li (-> Y, the next step's photo
// update).  Then per camera-pair block the group touches: the sum over its photos' edge pairs of
// the Schur pair products ([self] Hgg_a - Y'_a Hgp_b^T = U_a U_b^T, [self] (gg_a - U_a v),
// [self] gg_a), written once per group at the block's slot (k_schur sums the slots).  Summing in
// the group first cuts the slots (and k_schur's reads) to ~40% at 8 photos per group on config3.
#ifndef MCC_PHOTO_RPT
#define MCC_PHOTO_RPT 1   // rows of a camera-pair block per k_photo pair task (2, 3: fewer waves, slower)
#endif
#if MCC_IN(4)
#ifdef MCC_PHOTO_OCC
__global__ __launch_bounds__(256, MCC_PHOTO_OCC) void k_photo(LinArgs a) {
#else
__global__ __launch_bounds__(256) void k_photo(LinArgs a) {
#endif
    State* st = a.state;
    const int grp = blockIdx.x, tid = threadIdx.x;
    long long* stp = a.stamps ? a.stamps + kStampStride * (size_t)grp : nullptr;   // MCC_DIAG: slots 0..7
    SSTAMP(stp, 0, 0);
    // one round trip: the state and every per-group range (the stop test after the loads are issued)
    const int done = st->done;
    const int p0 = a.pgrp_ptr[grp], np = a.pgrp_ptr[grp + 1] - p0;
    const int ge0 = a.pgrp_edge[grp], gne = a.pgrp_edge[grp + 1] - ge0;   // the group's edges are contiguous
    const int q0 = a.gpair_ptr[grp], nq = a.gpair_ptr[grp + 1] - q0;
    const int c0 = a.gcon_ptr[grp], nc = a.gcon_ptr[grp + 1] - c0;
    if (done) return;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    constexpr int ES = 64;                      // per edge: Hgg upper [0, 21), pad, U [22, 58), gg [58, 64)
    double* sE = smem;                          // [gne][ES]
    double* s27 = sE + ES * gne;                // [kPhotoGroup][28]: Hpp upper 21, gp 6
    double* sLi = s27 + 28 * kPhotoGroup;       // [kPhotoGroup][36]: Li = L^-1 (lower, zeros above)
    double* sv = sLi + 36 * kPhotoGroup;        // [kPhotoGroup][6]: v = Li gp
    int* sgb = reinterpret_cast<int*>(smem + photo_lds_doubles(gne));   // [gne] gblock
    int* seq = sgb + gne;                                               // [gne] group-local photo
    int4* spq = reinterpret_cast<int4*>(sgb + ((2 * gne + 3) & ~3));   // [nq] (16-B aligned)
    unsigned* scn = reinterpret_cast<unsigned*>(spq + nq);              // [nc]
    const double* src = a.eh + 90 * (size_t)ge0;   // eh = [Hpp 21 | Hgg 21 | Hgp 36 | gp 6 | gg 6]
    {
        // every load of the staging issued before the first LDS store: the rest of eh -> LDS
        // (16 per thread: one round up to 64 edges); threads < 27 np: photo q's Hpp / gp column
        // sums in edge order, straight to registers
        constexpr int U = 16;
        const int tot = ES * gne;
        double v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int t = tid + 256 * u, le = t >> 6, c = t & 63;
            const int sc = c < 21 ? c + 21 : (c < 58 ? c + 20 : c + 26);
            v[u] = src[t < tot ? 90 * le + sc : 0];
        }
        const int sq = tid / 27, col27 = tid % 27;
        const bool sl = sq < np;
        int pe0 = 0, pne = 0;
        if (sl) {
            pe0 = a.photo_ptr[p0 + sq] - ge0;
            pne = a.photo_ptr[p0 + sq + 1] - ge0 - pe0;
        }
        const int col = col27 < 21 ? col27 : 78 + (col27 - 21);
        constexpr int SB = 16;
        double sv0[SB];
#pragma unroll
        for (int u = 0; u < SB; ++u) sv0[u] = (sl && u < pne) ? src[90 * (pe0 + u) + col] : 0.0;
        const int gbv = tid < gne ? a.gblock[ge0 + tid] : -1;
        const int lpv = tid < gne ? a.edge_lphoto[ge0 + tid] : 0;
        const int4 pqv = tid < nq ? a.gpairs[q0 + tid] : make_int4(0, 0, 0, 0);
        const unsigned cnv = tid < nc ? a.gcon[c0 + tid] : 0u;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int t = tid + 256 * u;
            if (t < tot) sE[t] = v[u];
        }
        for (int t0 = 256 * U; t0 < tot; t0 += 256) {   // beyond 64 edges (host bounds the groups)
            const int t = t0 + tid, le = t >> 6, c = t & 63;
            const int sc = c < 21 ? c + 21 : (c < 58 ? c + 20 : c + 26);
            if (t < tot) sE[t] = src[90 * le + sc];
        }
        double s = 0.0;
#pragma unroll
        for (int u = 0; u < SB; ++u) s += sv0[u];
        if (sl) {
            for (int le = SB; le < pne; ++le) s += src[90 * (pe0 + le) + col];
            s27[28 * sq + col27] = s;
        }
        if (tid < gne) sgb[tid] = gbv;
        for (int t = tid + 256; t < gne; t += 256) sgb[t] = a.gblock[ge0 + t];
        if (tid < gne) seq[tid] = lpv;   // edge -> group-local photo (host-built, first round trip)
        for (int t = tid + 256; t < gne; t += 256) seq[t] = a.edge_lphoto[ge0 + t];
        if (tid < nq) spq[tid] = pqv;
        for (int t = tid + 256; t < nq; t += 256) spq[t] = a.gpairs[q0 + t];
        if (tid < nc) scn[tid] = cnv;
        for (int t = tid + 256; t < nc; t += 256) scn[t] = a.gcon[c0 + t];
    }
    __syncthreads();
    SSTAMP(stp, 1, 0);
    if (tid < np) {   // one lane per photo: Cholesky Hpp = L L^T, Li = L^-1, v = Li gp, z' = Li^T v
        const int q = tid, photo = p0 + q;
        double A[21], gs[6], Lm[6][6], Li[6][6];
        const double2* S2 = reinterpret_cast<const double2*>(s27 + 28 * q);
#pragma unroll
        for (int k = 0; k < 14; ++k) {
            const double2 w = S2[k];
            if (2 * k < 21) A[2 * k] = w.x; else gs[2 * k - 21] = w.x;
            if (2 * k + 1 < 21) A[2 * k + 1] = w.y; else if (2 * k + 1 < 27) gs[2 * k + 1 - 21] = w.y;
        }
        bool bad = false;
        double idg[6];
#pragma unroll
        for (int j = 0; j < 6; ++j) {
            double d = A[6 * j - j * (j - 1) / 2];
#pragma unroll
            for (int k = 0; k < j; ++k) d -= Lm[j][k] * Lm[j][k];
            bad |= !(d > 0.0);
            const double sd = sqrt(d > 0.0 ? d : 1.0);
            const double is = 1.0 / sd;
            Lm[j][j] = sd;
            idg[j] = is;
#pragma unroll
            for (int i = j + 1; i < 6; ++i) {
                double t = A[6 * j - j * (j - 1) / 2 + (i - j)];   // Hpp(j, i) = Hpp(i, j)
#pragma unroll
                for (int k = 0; k < j; ++k) t -= Lm[i][k] * Lm[j][k];
                Lm[i][j] = t * is;
            }
        }
#pragma unroll
        for (int j = 0; j < 6; ++j) {   // column j of Li: forward substitution of L x = e_j
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                if (i < j) { Li[i][j] = 0.0; continue; }
                double t = i == j ? 1.0 : 0.0;
#pragma unroll
                for (int k = j; k < i; ++k) t -= Lm[i][k] * Li[k][j];
                Li[i][j] = t * idg[i];
            }
        }
        double vv[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            double t = 0.0;
#pragma unroll
            for (int k = 0; k <= i; ++k) t += Li[i][k] * gs[k];
            vv[i] = t;
        }
#pragma unroll
        for (int j = 0; j < 6; ++j) {
            double t = 0.0;
#pragma unroll
            for (int i = j; i < 6; ++i) t += Li[i][j] * vv[i];
            a.zp[6 * (size_t)photo + j] = t;
            a.gp_tot[6 * (size_t)photo + j] = gs[j];
            sv[6 * q + j] = vv[j];
        }
        double2* L2 = reinterpret_cast<double2*>(sLi + 36 * q);
#pragma unroll
        for (int k = 0; k < 18; ++k) L2[k] = make_double2(Li[(2 * k) / 6][(2 * k) % 6], Li[(2 * k + 1) / 6][(2 * k + 1) % 6]);
        if (bad || photo == a.fault_photo) atomicOr(&st->error, kErrPhotoNotPD);
    }
    __syncthreads();
    SSTAMP(stp, 3, 0);
    for (int t = tid; t < 6 * gne; t += 256) {   // task (edge, row i): U row i in place of Hgp row i, Y' row i
        const int le = t / 6, i = t % 6;
        double h[6], li[36], u[6], y[6];
        double2* H2 = reinterpret_cast<double2*>(sE + ES * le + 22 + 6 * i);
        const double2* I2 = reinterpret_cast<const double2*>(sLi + 36 * seq[le]);
#pragma unroll
        for (int q = 0; q < 3; ++q) { const double2 w = H2[q]; h[2 * q] = w.x; h[2 * q + 1] = w.y; }
#pragma unroll
        for (int q = 0; q < 18; ++q) { const double2 w = I2[q]; li[2 * q] = w.x; li[2 * q + 1] = w.y; }
        const bool gl = sgb[le] >= 0;
#pragma unroll
        for (int j = 0; j < 6; ++j) {   // U[i][j] = sum_{k <= j} Hgp[i][k] Li[j][k]
            double w = 0.0;
#pragma unroll
            for (int k = 0; k <= j; ++k) w += h[k] * li[6 * j + k];
            u[j] = gl ? w : 0.0;
        }
#pragma unroll
        for (int j = 0; j < 6; ++j) {   // Y'[i][j] = sum_{k >= j} U[i][k] Li[k][j]
            double w = 0.0;
#pragma unroll
            for (int k = j; k < 6; ++k) w += u[k] * li[6 * k + j];
            y[j] = w;
        }
        double2* G2 = reinterpret_cast<double2*>(a.Y + 36 * (size_t)(ge0 + le) + 6 * i);
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            H2[q] = make_double2(u[2 * q], u[2 * q + 1]);
            G2[q] = make_double2(y[2 * q], y[2 * q + 1]);
        }
    }
    __syncthreads();
    SSTAMP(stp, 4, 0);
    // task (block pair k, rows i0 .. i0 + RPT - 1, part h of H): the group's contributions c = h, h + H,
    // ... (photo, then edge pair order) summed by each part, the H parts (consecutive lanes)
    // combined by a fixed xor butterfly.  RPT = 2 rows per task: U_b is read once for both (three
    // tasks per block pair; three rows would spill at 3 waves per SIMD), and each entry keeps its
    // summation order.  H > 1 only when the group has few block
    // pairs (a one-block rig: DoubleSide, every edge pair of the group lands in one slot) so the
    // threads stay busy.
    constexpr int RPT = MCC_PHOTO_RPT, NT = 6 / RPT;
    int H = 1;
    while (H < 32 && NT * nq * 2 * H <= 256) H *= 2;
    for (int t = tid; t < NT * nq * H; t += 256) {
        const int h = t % H, k = t / H / NT, i0 = RPT * ((t / H) % NT);
        const int4 pq = spq[k];   // {first contribution, count, diagonal block << 1, slot offset}
        const bool diag = (pq.z & 2) != 0;
        double acc[RPT][6], racc[RPT], jacc[RPT];
#pragma unroll
        for (int r = 0; r < RPT; ++r) {
            racc[r] = 0.0;
            jacc[r] = 0.0;
#pragma unroll
            for (int j = 0; j < 6; ++j) acc[r][j] = 0.0;
        }
#pragma unroll 1
        for (int c = pq.x + h; c < pq.x + pq.y; c += H) {
            const unsigned w = scn[c];
            const int ea = w & 255, eb = (w >> 8) & 255, q = w >> 17;
            const bool self = (w >> 16) & 1;
            const double2* Y2 = reinterpret_cast<const double2*>(sE + ES * ea + 22 + 6 * i0);
            const double2* B2 = reinterpret_cast<const double2*>(sE + ES * eb + 22);
            double y[6 * RPT];
#pragma unroll
            for (int qq = 0; qq < 3 * RPT; ++qq) { const double2 v = Y2[qq]; y[2 * qq] = v.x; y[2 * qq + 1] = v.y; }
            const double* Hgg = sE + ES * ea;
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                double hb[6];
#pragma unroll
                for (int qq = 0; qq < 3; ++qq) { const double2 v = B2[3 * j + qq]; hb[2 * qq] = v.x; hb[2 * qq + 1] = v.y; }
#pragma unroll
                for (int r = 0; r < RPT; ++r) {
                    const int i = i0 + r;
                    double d = 0.0;
#pragma unroll
                    for (int kk = 0; kk < 6; ++kk) d += y[6 * r + kk] * hb[kk];
                    double hv = 0.0;
                    if (self) {
                        const int rr = i < j ? i : j, cc = i < j ? j : i;
                        hv = Hgg[rr * 6 - rr * (rr - 1) / 2 + (cc - rr)];
                    }
                    acc[r][j] += self ? hv - d : -d;
                }
            }
            if (diag && self) {
#pragma unroll
                for (int r = 0; r < RPT; ++r) {
                    double d = 0.0;
#pragma unroll
                    for (int kk = 0; kk < 6; ++kk) d += y[6 * r + kk] * sv[6 * q + kk];
                    const double gg = sE[ES * ea + 58 + i0 + r];
                    racc[r] += gg - d;
                    jacc[r] += gg;
                }
            }
        }
        for (int o = 1; o < H; o <<= 1) {   // the H parts are lanes t - h .. t - h + H - 1 (H | 64)
#pragma unroll
            for (int r = 0; r < RPT; ++r) {
#pragma unroll
                for (int j = 0; j < 6; ++j) acc[r][j] += __shfl_xor(acc[r][j], o);
                racc[r] += __shfl_xor(racc[r], o);
                jacc[r] += __shfl_xor(jacc[r], o);
            }
        }
        if (h == 0) {
            double* out = a.pairprod + (size_t)pq.w;
#pragma unroll
            for (int r = 0; r < RPT; ++r) {
#pragma unroll
                for (int j = 0; j < 6; ++j) out[(i0 + r) * 6 + j] = acc[r][j];
                if (diag) {
                    out[36 + i0 + r] = racc[r];
                    out[42 + i0 + r] = jacc[r];
                }
            }
        }
    }
#ifdef MCC_DIAG
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    SSTAMP(stp, 5, 0);
}
#endif  // MCC_IN(4)

// ---------------------------------------------------------------- global solve (one workgroup)
// Stop test (src/multicalib.cpp:475-477), elimination of the reduced camera system (m <= 128),
// global-block delta and float32 update.  S (m x m) and r (m) are in LDS and are overwritten.
__device__ __forceinline__ double sub_sum(double v, int tpr) {
    for (int o = 1; o < tpr; o <<= 1) v += __shfl_xor(v, o);
    return v;
}

// Gauss-Jordan of [S | r] (m x (m+1), m <= 30) by one wavefront with the matrix in registers:
// lane i owns row i.  Step k broadcasts only row k right of the pivot (m - k values, v_readlane
// with a compile-time lane) -- about m^2/2 broadcasts in all -- and every lane i != k eliminates
// its column-k entry.  S is SPD: no pivoting.  Writes delta_i = r_i / S_ii into r[].

template <int MM>
__device__ __forceinline__ void gj_rows(const double* S, double* r, int m, int lane, int* err, int* bad_lds) {
    // every load address is in range for every lane: lanes >= m read row 0 and stay idle
    const int li = lane < m ? lane : 0;
    double row[MM];
#pragma unroll
    for (int j = 0; j < MM; ++j) row[j] = S[li * m + (j < m ? j : 0)];
    double rr = r[li], dii = 1.0;
    bool bad = false;
#pragma unroll
    for (int k = 0; k < MM; ++k) {
        if (k >= m) break;
        const double piv = readlane_f64(row[k], k);
        bad |= !(piv > 0.0);
        const double pv = piv > 0.0 ? piv : 1.0;
        double ip = __builtin_amdgcn_rcp(pv);   // v_rcp_f64 (~2^-26 rel), one Newton step -> ~1 ulp
        ip = fma(ip, fma(-pv, ip, 1.0), ip);
        if (lane == k) dii = piv;
        const double f = lane == k ? 0.0 : row[k] * ip;
        // broadcast the whole pivot row first (distinct SGPR pairs, back-to-back v_readlane),
        // then the updates: no readlane -> use -> readlane reuse of one SGPR pair per column
        double pr[MM + 1];
#pragma unroll
        for (int j = k + 1; j < MM; ++j) pr[j] = j < m ? readlane_f64(row[j], k) : 0.0;
        pr[MM] = readlane_f64(rr, k);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = k + 1; j < MM; ++j) {
            if (j >= m) break;
            row[j] -= f * pr[j];
        }
        rr -= f * pr[MM];
    }
    if (bad && lane == 0) atomicOr(err, 2);
    if (bad_lds && lane == 0) *bad_lds = bad ? 1 : 0;   // every call writes it (no initialisation race)
    if (lane < m) r[lane] = rr / dii;
}


__device__ __forceinline__ int packed_index(int i, int j, int m) {   // i <= j
    return i * m - i * (i - 1) / 2 + (j - i);
}

// Blocked Gauss-Jordan of [S | r] for m > 30 (m <= 128; k_solve), 16 x 16 blocks in LDS:
// A = S padded with the identity to M = 16 nb rows (stride M + 1: odd, conflict-free columns),
// x = r.  Per pivot block kb: (1) wave 0 inverts A[kb][kb] (register Gauss-Jordan, lane i owns
// row i of [P | I]); (2) the pivot block row is scaled by the inverse, A[kb][j] <- P^-1 A[kb][j]
// (j > kb) and x_kb <- P^-1 x_kb; (3) the block column is eliminated from every other block row,
// A[i][j] -= A[i][kb] A[kb][j], x_i -= A[i][kb] x_kb.  Every 16 x 16 x 16 block product is four
// v_mfma_f64_16x16x4_f64 (operands straight from LDS, items dealt round-robin to the 4 waves).
// S is SPD: no pivoting.  x ends as the solution.
typedef double v4f64_t __attribute__((ext_vector_type(4)));
constexpr int kBlkLd = 17;   // stride of the 16 x 16 pivot-inverse scratch
#ifndef MCC_SOLVE_THREADS
#define MCC_SOLVE_THREADS 512
#endif
constexpr int kSolveThreads = MCC_SOLVE_THREADS;   // k_solve's workgroup for m > 30
__device__ __forceinline__ int gjb_ld(int m) { return 16 * ((m + 15) / 16) + 1; }
__device__ __forceinline__ void blk_mfma(double* C, int ldc, const double* Ap, int lda, const double* Bp, int ldb,
                                         bool sub, bool zero_c) {
    const int lane = threadIdx.x & 63, i = lane & 15, kq = lane >> 4;
    v4f64_t acc;
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[r] = zero_c ? 0.0 : C[(kq + 4 * r) * ldc + i];
    double av[4], bv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        av[q] = Ap[i * lda + 4 * q + kq];   // A[i][k], k = 4q + kq
        bv[q] = Bp[(4 * q + kq) * ldb + i];  // B[k][j], j = i
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(sub ? -av[q] : av[q], bv[q], acc, 0, 0, 0);
#pragma unroll
    for (int r = 0; r < 4; ++r) C[(kq + 4 * r) * ldc + i] = acc[r];   // C[row = kq + 4r][col = i]
}
// 16 x 16 SPD inverse by one wave, all 64 lanes (GjbStep below).  Writes P^-1 to PV (stride
// kBlkLd); returns false if a pivot is not > 0.
template <int K>
__device__ __forceinline__ double gjb_bcast16(double v) {
    const long long u = __double_as_longlong(v);
    // all rows / banks enabled: every lane is written, so no 'old' operand needs materialising
    const int lo = __builtin_amdgcn_mov_dpp((int)u, 0x150 + K, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_mov_dpp((int)(u >> 32), 0x150 + K, 0xF, 0xF, true);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
// In-place Gauss-Jordan inversion (no identity half): lane l holds row i = l & 15, columns
// 4g .. 4g+3 (g = l >> 4).  Pivot K: p = A[K][K] by v_readlane, ip = 1/p; the pivot row's columns of
// every lane by DPP row_newbcast:K inside each 16-lane row (the lanes of one column group), A[i][K]
// of each row by one bpermute; then A[i][j] -= f A[K][j] with f = A[i][K] ip, the pivot row is
// scaled by ip, and column K becomes -f (ip on the diagonal).
// Row group GK (16 lanes) of x copied to every row group: lane (i, g) gets x(i, GK).  Two VALU
// swaps (v_permlane16_swap: odd rows <-> even rows, v_permlane32_swap: halves), no LDS path.
template <int GK>
__device__ __forceinline__ double bcast_group(double x) {
    double a = x, b = x;
    pl16_swap(a, b);                      // a(i, g) = x(i, g & ~1), b(i, g) = x(i, g | 1)
    double c = (GK & 1) ? b : a;          // c(i, g) = x(i, (g & 2) | (GK & 1))
    double d = c, e = c;
    pl32_swap(d, e);                      // d(i, g) = c(i, g & 1), e(i, g) = c(i, 2 | (g & 1))
    return (GK & 2) ? e : d;
}
#ifndef MCC_GJB_IDLE4
#define MCC_GJB_IDLE4 0
#endif
#ifndef MCC_GJB_SWAP
#define MCC_GJB_SWAP 0   // 1: the pivot column by permlane16/32 swaps, the pivot by DPP (m = 90: 19.2 vs 18.7 us, slower)
#endif
template <int K>
struct GjbStep {
    __device__ __forceinline__ static void run(double (&v)[4], int lane, bool& ok) {
        constexpr int gk = K >> 2, ck = K & 3;
        const int i = lane & 15, g = lane >> 4;
#if MCC_GJB_SWAP
        const double rik = bcast_group<gk>(v[ck]);     // row i's column-K entry
        const double piv = gjb_bcast16<K>(rik);          // row K's: the pivot
#else
        const double piv = readlane_f64(v[ck], K + 16 * gk);
        const double rik = __shfl(v[ck], i + 16 * gk);   // row i's column-K entry
#endif
        ok &= piv > 0.0;
        const double pv = piv > 0.0 ? piv : 1.0;
        double ip = __builtin_amdgcn_rcp(pv);
        ip = fma(ip, fma(-pv, ip, 1.0), ip);
        const bool prow = i == K;
        // other rows: v - f pr with f = A[i][K] ip; the pivot row (pr = its own v): fma(ip, v, 0), an
        // exactly rounded v ip (1 - ip and a difference would cancel when ip is tiny)
        const double f = prow ? -ip : rik * ip;
        const double keep = prow ? 0.0 : 1.0;
        double pr[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) pr[c] = gjb_bcast16<K>(v[c]);
#pragma unroll
        for (int c = 0; c < 4; ++c) v[c] = fma(-f, pr[c], v[c] * keep);
        if (g == gk) v[ck] = prow ? ip : -f;
        GjbStep<K + 1>::run(v, lane, ok);
    }
};
template <>
struct GjbStep<16> {
    __device__ __forceinline__ static void run(double (&)[4], int, bool&) {}
};
// Two pivots per step (K even: columns K, K + 1 share a lane's column group): the 2 x 2 pivot block
// P = [[a, b], [c, d]] inverted in closed form, Q = P^-1 (one reciprocal of det), then
// rows i outside {K, K+1}: A[i][j] -= [A[i][K] A[i][K+1]] Q [A[K][j]; A[K+1][j]], columns K, K+1 <-
// -[A[i][K] A[i][K+1]] Q; the pivot rows <- Q times them; the pivot block <- Q.  The same result as
// two single pivots in exact arithmetic (SPD: a > 0 and det = a d' > 0), with about 3/4 of their
// instructions (one reciprocal chain, one set of multipliers).
#ifndef MCC_GJB_PAIR
#define MCC_GJB_PAIR 0   // 1: pairs of pivots (m = 90: 18.72 vs 18.63 us per solve, m = 126: 28.4 vs 29.8)
#endif
template <int K>
struct GjbPair {
    __device__ __forceinline__ static void run(double (&v)[4], int lane, bool& ok) {
        constexpr int gk = K >> 2, c0 = K & 3, c1 = c0 + 1;
        const int i = lane & 15, g = lane >> 4;
        const double a = readlane_f64(v[c0], K + 16 * gk), b = readlane_f64(v[c1], K + 16 * gk);
        const double c = readlane_f64(v[c0], K + 1 + 16 * gk), d = readlane_f64(v[c1], K + 1 + 16 * gk);
        const double r0 = __shfl(v[c0], i + 16 * gk), r1 = __shfl(v[c1], i + 16 * gk);   // A[i][K], A[i][K+1]
        const double det = fma(a, d, -(b * c));
        ok &= a > 0.0 && det > 0.0;
        const double pd = det > 0.0 ? det : 1.0;
        double id = __builtin_amdgcn_rcp(pd);
        id = fma(id, fma(-pd, id, 1.0), id);
        const double q00 = d * id, q01 = -b * id, q10 = -c * id, q11 = a * id;
        const bool p0 = i == K, p1 = i == K + 1;
        double m0 = fma(r0, q00, r1 * q10), m1 = fma(r0, q01, r1 * q11);
        m0 = p0 ? -q00 : (p1 ? -q10 : m0);
        m1 = p0 ? -q01 : (p1 ? -q11 : m1);
        const double keep = (p0 || p1) ? 0.0 : 1.0;
        double pa[4], pb[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            pa[q] = gjb_bcast16<K>(v[q]);
            pb[q] = gjb_bcast16<K + 1>(v[q]);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = fma(-m1, pb[q], fma(-m0, pa[q], v[q] * keep));
        if (g == gk) {
            v[c0] = p0 ? q00 : (p1 ? q10 : -m0);
            v[c1] = p0 ? q01 : (p1 ? q11 : -m1);
        }
        GjbPair<K + 2>::run(v, lane, ok);
    }
};
template <>
struct GjbPair<16> {
    __device__ __forceinline__ static void run(double (&)[4], int, bool&) {}
};
__device__ __forceinline__ bool gjb_inverse16_regs(double (&v)[4], double* PV, int lane) {
    const int i = lane & 15, g = lane >> 4;
    bool ok = true;
#if MCC_GJB_PAIR
    GjbPair<0>::run(v, lane, ok);
#else
    GjbStep<0>::run(v, lane, ok);
#endif
#pragma unroll
    for (int c = 0; c < 4; ++c) PV[i * kBlkLd + 4 * g + c] = v[c];
    return ok;
}
__device__ __forceinline__ bool gjb_inverse16(const double* Pk, int ld, double* PV, int lane) {
    const int i = lane & 15, g = lane >> 4;
    double v[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) v[c] = Pk[i * ld + 4 * g + c];
    return gjb_inverse16_regs(v, PV, lane);
}
// gst (mcc_debug_solve only; null in the step kernels): s_memtime of thread 0 at the phase
// boundaries, slot 0 after the loads, 1 + 3 kb .. 3 + 3 kb per pivot block step
#define GJB_STAMP(k) do { if (gst && threadIdx.x == 0) gst[k] = (long long)__builtin_amdgcn_s_memtime(); } while (0)
__device__ __forceinline__ void gj_blocked(const double* packed, double* x, double* A, double* PV, int m, int* err,
                                           long long* gst, int* bad_lds = nullptr) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
    const int nb = (m + 15) / 16, M = 16 * nb, ld = M + 1, ntri = m * (m + 1) / 2;
    // rhs, padding and the packed triangle: every global load is issued before the first LDS store
    const double xr = tid < m ? packed[ntri + tid] : 0.0;   // M <= 128 <= blockDim.x
    // the packed upper triangle: thread t takes the sixteen contiguous entries 16t .. 16t+15
    // (eight 16-B loads in flight, one memory round trip up to m = 90); the row of the first from
    // the quadratic's root with a one-step fix-up, the rest by stepping along the row; (i, j) and
    // (j, i) written
    // Wave 0 meanwhile gathers the first pivot block (rows / columns 0..15, inside the matrix since
    // m > 30) straight from the packed system and inverts it, off the load's critical path.
    const int nt = m * (m + 1) / 2;
    constexpr int PB = 16;
    bool bad = false;
    if (wave == 0) {
        const int i = lane & 15, g = lane >> 4;
        double v0[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int col = 4 * g + c;
            v0[c] = packed[i <= col ? packed_index(i, col, m) : packed_index(col, i, m)];
        }
        bad |= !gjb_inverse16_regs(v0, PV, lane);
    } else {
        const int lt = tid - 64, nlt = (int)blockDim.x - 64;
        for (int t0 = PB * lt; t0 < nt; t0 += PB * nlt) {
            double v[PB];
            if (t0 + PB <= nt) {
                const double2* p2 = reinterpret_cast<const double2*>(packed + t0);   // t0 even: 16-B aligned
#pragma unroll
                for (int u = 0; u < PB / 2; ++u) { const double2 w = p2[u]; v[2 * u] = w.x; v[2 * u + 1] = w.y; }
            } else {
#pragma unroll
                for (int u = 0; u < PB; ++u) v[u] = packed[min(t0 + u, nt - 1)];
            }
            const double b = 2.0 * m + 1.0;
            int i = (int)((b - sqrt(b * b - 8.0 * t0)) * 0.5);
            i = max(0, min(i, m - 1));
            if (packed_index(i, i, m) > t0) --i;
            else if (i + 1 < m && packed_index(i + 1, i + 1, m) <= t0) ++i;
            int j = i + (t0 - packed_index(i, i, m));
#pragma unroll
            for (int u = 0; u < PB; ++u) {
                if (t0 + u < nt) {
                    A[i * ld + j] = v[u];
                    A[j * ld + i] = v[u];
                }
                if (++j == m) { ++i; j = i; }
            }
        }
        // padding: rows m .. M-1 (every column) and columns m .. M-1 of rows < m
        for (int i = m + wave - 1; i < M; i += nw - 1)
            for (int j = lane; j < M; j += 64) A[i * ld + j] = i == j ? 1.0 : 0.0;
        for (int i = lt; i < m; i += nlt)
            for (int j = m; j < M; ++j) A[i * ld + j] = 0.0;
    }
    if (tid < M) x[tid] = xr;
    __syncthreads();
    GJB_STAMP(0);
    // later pivots are inverted one step ahead (look-ahead): in step kb, wave 0 first eliminates
    // block (kb+1, kb+1) and inverts it while the other waves eliminate the rest; PV holds two
    // 16 x 17 buffers (step parity)
    for (int kb = 0; kb < nb; ++kb) {
        GJB_STAMP(1 + 3 * kb);
        const double* PVk = PV + (kb & 1) * 16 * kBlkLd;
        // (2) scale the pivot block row: items j = kb+1 .. nb-1 (MFMA), then the rhs block
        {
            const int n2 = nb - 1 - kb;
            for (int it = wave; it <= n2; it += nw) {
                if (it < n2) {
                    double* Ckj = A + 16 * kb * ld + 16 * (kb + 1 + it);
                    blk_mfma(Ckj, ld, PVk, kBlkLd, Ckj, ld, false, true);
                } else {
                    double v = 0.0;
                    if (lane < 16) {
#pragma unroll
                        for (int k = 0; k < 16; ++k) v += PVk[lane * kBlkLd + k] * x[16 * kb + k];
                    }
                    __builtin_amdgcn_wave_barrier();
                    if (lane < 16) x[16 * kb + lane] = v;
                }
            }
        }
        __syncthreads();
        GJB_STAMP(2 + 3 * kb);
        // (3) eliminate block column kb from the other block rows: items (ib, j), then the rhs
        {
            const int nj = nb - 1 - kb, n3 = (nb - 1) * nj;
            const bool ahead = kb + 1 < nb && nw > 1;
            const int it0 = kb * nj;   // item of block (kb+1, kb+1): row index r = kb, column c = 0
            auto item = [&](int it) {
                if (it < n3) {
                    const int r = it / max(nj, 1), c = it % max(nj, 1);
                    const int ib = r < kb ? r : r + 1, jb = kb + 1 + c;
                    blk_mfma(A + 16 * ib * ld + 16 * jb, ld, A + 16 * ib * ld + 16 * kb, ld, A + 16 * kb * ld + 16 * jb, ld,
                             true, false);
                } else {
                    for (int i = lane; i < M; i += 64) {
                        if ((i >> 4) == kb) continue;
                        double v = x[i];
#pragma unroll
                        for (int k = 0; k < 16; ++k) v -= A[i * ld + 16 * kb + k] * x[16 * kb + k];
                        x[i] = v;
                    }
                }
            };
            if (!ahead) {
                for (int it = wave; it <= n3; it += nw) item(it);
            } else if (wave == 0) {
                item(it0);
                if (gst && tid == 0) gst[40 + kb] = (long long)__builtin_amdgcn_s_memtime();
                const int kn = kb + 1;
                bad |= !gjb_inverse16(A + 16 * kn * ld + 16 * kn, ld, PV + (kn & 1) * 16 * kBlkLd, lane);
                if (gst && tid == 0) gst[48 + kb] = (long long)__builtin_amdgcn_s_memtime();
            } else {
#if MCC_GJB_IDLE4
                // wave 4 shares wave 0's SIMD: it sits out, so the pivot chain has the SIMD alone
                if (nw > 5 && wave == 4) {
                } else {
                    const int wid = nw > 5 && wave > 4 ? wave - 2 : wave - 1, nwk = nw > 5 ? nw - 2 : nw - 1;
                    for (int q = wid; q < n3; q += nwk) item(q < it0 ? q : q + 1);
                }
#else
                for (int q = wave - 1; q < n3; q += nw - 1) item(q < it0 ? q : q + 1);   // n3 - 1 blocks + rhs
#endif
                if (gst && tid == 64) gst[56 + kb] = (long long)__builtin_amdgcn_s_memtime();
            }
        }
        __syncthreads();
        GJB_STAMP(3 + 3 * kb);
    }
    if (bad && lane == 0) {
        atomicOr(err, 2);
        if (bad_lds) *bad_lds = 1;
    }
}

// ---------------------------------------------------------------- warm solve (m > 30, k_solve)
// S_{t+1} x = r by iterative refinement with the inverse of the previous step's system, which the
// resident helper k_sinv_helper computed while this step linearised:
//   x_0 = S_t^-1 r,  x_{k+1} = x_k + S_t^-1 (r - S_{t+1} x_k).
// Hand-off with the helper through uncached memory (every access goes to HBM, so no cache holds a
// stale copy): k_solve publishes S_t (sprev, then sync[0] = t's epoch, after its stores drained);
// the helper inverts it into sinv and publishes sync[1] = that epoch; the next k_solve waits for
// sync[1] == sync[0] before it reads sinv or overwrites sprev.  It always refines with exactly the
// previous step's inverse, so the result does not depend on timing: there is no "helper late ->
// direct elimination" switch (a helper that has not delivered after WarmCtx::wait_ticks fails the
// step with kErrWarmTimeout), and on a sharded problem every rank takes the same branch on the same
// bits (tests/test_warm_solve.py: a delayed helper, one rank delayed at world 2).
// Thread t holds row i = t >> 2 of S_{t+1} and of S_t^-1, columns [24 g, 24 g + 24) (g = t & 3; zero
// beyond m), in registers; a product A v is the quad's four partial dot products (v from LDS, six
// 16-B reads in flight) added by two DPP quad permutes.  (Measured, not kept: 4 x 6 blocks per
// thread with a 16-lane butterfly per row -- 4x less LDS traffic per product, but ~5.6k instead of
// ~3.3k cycles per correction.)
// Converged when every equation holds to its own scale, |r - S x|_i <= 64 eps (|S| |x| + |r|)_i
// (tested before each correction, so a preconditioner as good as the systems' step-to-step change
// costs none); otherwise (kWarmMaxIters corrections, a NaN) the direct elimination runs.
constexpr int kWarmQ = 24;                 // M <= 96 (m <= 96): the staged S and S^-1 fit in LDS
constexpr int kWarmN = 4 * kWarmQ;
__device__ __forceinline__ double wave_max(double v) {
    {
        double a = v, b = v;
        pl32_swap(a, b);
        v = fmax(a, b);
    }
    {
        double a = v, b = v;
        pl16_swap(a, b);
        v = fmax(a, b);
    }
    v = fmax(v, dpp_f64<kDppRor8>(v));
    v = fmax(v, dpp_f64<kDppRor4>(v));
    v = fmax(v, dpp_f64<kDppXor2>(v));
    v = fmax(v, dpp_f64<kDppXor1>(v));
    return v;
}
// a workgroup barrier that orders LDS only (no wait for outstanding global stores)
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}
// the quad's dot product of row i with v over its chunk (no guards, so every 16-B LDS read is in
// flight at once), summed over the quad
__device__ __forceinline__ double warm_dot(const double (&a)[kWarmQ], const double* v) {
    double2 w[kWarmQ / 2];
#pragma unroll
    for (int c = 0; c < kWarmQ / 2; ++c) w[c] = reinterpret_cast<const double2*>(v)[c];
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
#pragma unroll
    for (int c = 0; c < kWarmQ / 2; c += 2) {
        s0 = fma(a[2 * c], w[c].x, s0);
        s1 = fma(a[2 * c + 1], w[c].y, s1);
        s2 = fma(a[2 * c + 2], w[c + 1].x, s2);
        s3 = fma(a[2 * c + 3], w[c + 1].y, s3);
    }
    double s = (s0 + s1) + (s2 + s3);
    s += dpp_f64<kDppXor1>(s);
    s += dpp_f64<kDppXor2>(s);
    return s;
}
// the same for A v and |A| |v| together (the residual and its componentwise scale)
__device__ __forceinline__ double warm_dot_abs(const double (&a)[kWarmQ], const double* v, double& sa) {
    double2 w[kWarmQ / 2];
#pragma unroll
    for (int c = 0; c < kWarmQ / 2; ++c) w[c] = reinterpret_cast<const double2*>(v)[c];
    double s0 = 0.0, s1 = 0.0, t0 = 0.0, t1 = 0.0;
#pragma unroll
    for (int c = 0; c < kWarmQ / 2; ++c) {
        s0 = fma(a[2 * c], w[c].x, s0);
        s1 = fma(a[2 * c + 1], w[c].y, s1);
        t0 = fma(fabs(a[2 * c]), fabs(w[c].x), t0);
        t1 = fma(fabs(a[2 * c + 1]), fabs(w[c].y), t1);
    }
    double s = s0 + s1, t = t0 + t1;
    s += dpp_f64<kDppXor1>(s);
    t += dpp_f64<kDppXor1>(t);
    s += dpp_f64<kDppXor2>(s);
    t += dpp_f64<kDppXor2>(t);
    sa = t;
    return s;
}
__host__ __device__ __forceinline__ int warm_lc2(int m) { return (m * (m + 1) / 2 + m + 1) / 2; }   // packed [S | r] in double2
// the helper's LDS: the elimination [M x (M + 1)] and its pivot scratch; refine: the staged [S | r],
// the solution and warm_refine's work area
__host__ __device__ __forceinline__ size_t helper_shmem_doubles(int m, bool refine) {
    const size_t M = 16 * (size_t)((m + 15) / 16);
    return M * (M + 1) + 16 * kBlkLd + (refine ? 2 * (size_t)warm_lc2(m) + 2 * kWarmN + 8 : 16 * kBlkLd);
}
// LDS doubles of the warm path behind x (kWarmN): packed [S | r] (even length), S^-1 (M x (M + 2)),
// the residual (kWarmN), wave maxima
__host__ __device__ __forceinline__ size_t warm_shmem_doubles(int m) {
    const int M = 16 * ((m + 15) / 16);
    return 2 * (size_t)((m * (m + 1) / 2 + m + 1) / 2) + (size_t)M * (M + 2) + kWarmN + 48;
}
// row i's chunk of S_{t+1} from the staged packed upper triangle (zero beyond m)
__device__ __forceinline__ void warm_gather_s(const double* Pk, int m, double (&Sr)[kWarmQ]) {
    const int i = threadIdx.x >> 2, g = threadIdx.x & 3;
    const bool row = i < m;
    const int ic = row ? i : 0;
#pragma unroll
    for (int c = 0; c < kWarmQ; ++c) {
        const int j = min(g * kWarmQ + c, m - 1);
        const int lo = min(ic, j), hi = max(ic, j);
        const double v = Pk[lo * m - lo * (lo - 1) / 2 + (hi - lo)];
        Sr[c] = row && g * kWarmQ + c < m ? v : 0.0;
    }
}
// the refinement: Sr (registers), Iv = S_t^-1 (LDS, row stride ivld: k_solve's M + 2, the helper's
// elimination layout M + 1), Pk = packed [S | r] (LDS); x[kWarmN] receives the solution (zero beyond
// m).  stats (k_solve): the counters; corr (the helper): the corrections run
template <bool ODD_LD>
__device__ __forceinline__ bool warm_refine(const double (&Sr)[kWarmQ], const double* Iv, int ivld, const double* Pk,
                                            double* x, double* work, int m, long long* stats, int* corr = nullptr) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr int nw = kSolveThreads / 64;
    const int i = tid >> 2, g = tid & 3;
    constexpr int Qp = kWarmQ, nv = kWarmN;
    const int ntri = m * (m + 1) / 2, M = 16 * ((m + 15) / 16);
    const bool row = i < m;
    const int ic = row ? i : 0;
    double Ir[kWarmQ];
    if (!ODD_LD) {   // 16-B aligned rows
#pragma unroll
        for (int c = 0; c < kWarmQ; c += 2) {
            const int j = g * Qp + c;
            const double2 v = *reinterpret_cast<const double2*>(Iv + ic * ivld + min(j, M - 2));
            Ir[c] = row && j < m ? v.x : 0.0;
            Ir[c + 1] = row && j + 1 < m ? v.y : 0.0;
        }
    } else {
#pragma unroll
        for (int c = 0; c < kWarmQ; ++c) {
            const int j = g * Qp + c;
            Ir[c] = row && j < m ? Iv[ic * ivld + j] : 0.0;
        }
    }
    const double rr = row ? Pk[ntri + i] : 0.0;
    double* rv = work;            // [nv] right-hand side, then the residual
    double* red = work + nv;      // [nw] per-wave max of the scaled residual
    if (g == 0 && i < nv) rv[i] = rr;
    lds_barrier();
    // stop when every equation is satisfied to its own scale (componentwise backward error,
    // Oettli-Prager): |r - S x|_i <= 64 eps (|S| |x| + |r|)_i -- the level of the residual's own
    // rounding; a normwise test lets the small (rotation) components of a badly scaled system drift.
    // (A fallback wastes the corrections it ran: it stops at kWarmMaxIters or at the first
    // correction that does not cut the error fourfold.)
    constexpr double kTol = 64.0 * 1.1102230246251565e-16;
    double xi = warm_dot(Ir, rv + g * Qp);   // x_0 = S_t^-1 r
    bool conv = false;
    int it = 0;
    double qprev = 0.0;
    for (;;) {
        if (g == 0 && i < nv) x[i] = row ? xi : 0.0;
        lds_barrier();
        double sa;
        const double res = rr - warm_dot_abs(Sr, x + g * Qp, sa);
        // row i's componentwise backward error |r - S x|_i / (|S| |x| + |r|)_i (NaN: 1)
        const double q = fabs(res) / fmax(sa + fabs(rr), 1e-300);
        const double qm = wave_max(row ? (q == q ? q : 1.0) : 0.0);
        if (g == 0 && i < nv) rv[i] = row ? res : 0.0;
        if (lane == 0) red[wave] = qm;
        lds_barrier();
        {
            double rd[nw];
#pragma unroll
            for (int k = 0; k < nw; ++k) rd[k] = red[k];
            double qn = rd[0];
#pragma unroll
            for (int k = 1; k < nw; ++k) qn = fmax(qn, rd[k]);
            conv = qn <= kTol;
            // give up early when a correction does not shrink the error fourfold (the systems moved
            // too far for the stale inverse: the first Gauss-Newton steps from a rough start)
            if (!conv && it > 0 && !(qn <= 0.25 * qprev)) it = kWarmMaxIters;
            qprev = qn;
        }
        if (conv || it >= kWarmMaxIters) break;
        xi += warm_dot(Ir, rv + g * Qp);
        ++it;
    }
    if (tid == 0 && stats) {
        stats[0] += 1;
        stats[1] += it;
        if (!conv) stats[2] += 1;
    }
    if (corr) *corr = it;
    return conv;
}
// The warm buffers are uncached device memory: plain loads and stores go to HBM whatever their
// cache bits (so many loads stay in flight under the compiler's own waits); the epochs are read
// and written with system-scope atomics so the spin loops re-load them.  The data loads follow
// the epoch check through a workgroup barrier.
__device__ __forceinline__ double2 ld_sys_x2(const double* p) { return *reinterpret_cast<const double2*>(p); }
// 5 x 16 bytes past every cache (sc0 sc1), all in flight before one wait: the resident helper's staging
// of prev2 (plain loads of the uncached buffer were served stale copies, see ld_sys_f64)
__device__ __forceinline__ void ld_nc_x2_5(const double* p0, const double* p1, const double* p2, const double* p3,
                                           const double* p4, f64x2_t (&v)[5]) {
    asm volatile(
        "global_load_dwordx4 %0, %5, off sc0 sc1\n\t"
        "global_load_dwordx4 %1, %6, off sc0 sc1\n\t"
        "global_load_dwordx4 %2, %7, off sc0 sc1\n\t"
        "global_load_dwordx4 %3, %8, off sc0 sc1\n\t"
        "global_load_dwordx4 %4, %9, off sc0 sc1\n\t"
        "s_waitcnt vmcnt(0)"
        : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4])
        : "v"(p0), "v"(p1), "v"(p2), "v"(p3), "v"(p4)
        : "memory");
}
// 16 bytes of epoch words past every cache, waited for (k_solve's poll of the helper's {epoch, status,
// corrections}: one request, so the status words written before the epoch arrive with it)
__device__ __forceinline__ uint4 ld_nc_u32x4(const unsigned* p) {
    uint4 v;
    asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=&v"(v) : "v"(p) : "memory");
    return v;
}
__device__ __forceinline__ void st_sys_x2(double* p, double a, double b) {
    f64x2_t v;
    v.x = a;
    v.y = b;
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");   // (st_sc1_x2's hazard)
}
// prev2 in the resident helper: system-scope loads.  Plain loads of the uncached buffer were served
// stale copies in a helper that runs for many systems (round 5: the previous use of the same parity
// buffer, two systems back -- every refinement with the carried inverse then fell back)
__device__ __forceinline__ double ld_sys_f64(const double* p) {
    return __longlong_as_double(
        (long long)__hip_atomic_load(reinterpret_cast<const unsigned long long*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
}
__device__ __forceinline__ unsigned ld_sys_u32(const unsigned* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys_u32(unsigned* p, unsigned v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// no system will follow from this step (the loop stopped, a failed step): the helper may exit
__device__ __forceinline__ void warm_stop(const WarmCtx& w) {
    if (w.sync && threadIdx.x == 0) st_sys_u32(w.sync + 2, 1u);
}

// k_solve's m > 30 elimination with the warm path, in three pieces around solve_global's stop test
// (so that its memory round trips overlap the state's):
//   warm_issue  (every thread, before the stop test): this step's packed [S | r] into registers;
//   warm_check  (thread 64, meanwhile): the epochs {published, inverted, stop, PD} in one 16-B load,
//               a wait for the helper only if it has not inverted the last published system;
//   warm_finish (after the stop test): stage [S | r] in LDS and publish it as sprev for the helper,
//               load S_t^-1 (uncached) into LDS, refine; the direct elimination (gj_blocked) when
//               there is no inverse yet, the last system was not positive definite, or the
//               refinement does not converge; then the new epoch.  Barriers that only order LDS are raw s_barriers, so the sprev
//               stores drain behind the refinement instead of at each barrier.
// x: LDS (the solution), followed by the work area (mcc_solve_shmem).
constexpr int kWarmPer = 8;   // double2 of [S | r] per thread: one pass up to m = 90 (2 093 double2 at 512 threads)
struct WarmStage {
    double2 v[kWarmPer];
};
__device__ __forceinline__ bool warm_on(const WarmCtx* w, int m) { return w && w->sync && m <= kWarmN; }
__device__ __forceinline__ void warm_issue(const double* packed, int m, WarmStage& ws) {
    const int n2 = warm_lc2(m), tid = threadIdx.x;
#pragma unroll
    for (int u = 0; u < kWarmPer; ++u) {
        const int q = u * (int)blockDim.x + tid;
        ws.v[u] = q < n2 ? reinterpret_cast<const double2*>(packed)[q] : make_double2(0.0, 0.0);
    }
}
// use: 1 refine with the helper's inverse, 0 the direct elimination (no system inverted yet, or the
// helper found the last one not positive definite -- both functions of the systems alone), -1 the
// helper did not deliver within wait_ticks (the step fails: kErrWarmTimeout)
__device__ __forceinline__ void warm_check(const WarmCtx& w, int* use_s, unsigned* e_s) {
    if (w.refine) {
        // the helper solves: wait for its solution of the system k_schur published (epoch e); 2: use
        // it, 0: eliminate (no inverse of the previous system, or the refinement did not converge)
        const unsigned e = ld_sys_u32(w.sync);
        // {solved epoch, status, corrections, -} in one 16-byte load per poll (round 6: the status words
        // were re-read after the epoch matched, one more memory round trip on every waited step)
        uint4 hy = ld_nc_u32x4(w.sync + 4);
        if (hy.x != e) {
            w.stats[4] += 1;
            const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
            while (hy.x != e && (long long)__builtin_amdgcn_s_memrealtime() - t0 < w.wait_ticks) {
                __builtin_amdgcn_s_sleep(2);
                hy = ld_nc_u32x4(w.sync + 4);
            }
        }
        // use: -1 the helper did not deliver; else (corrections << 3) | (0 no inverse, 1 refined, not
        // converged, 2 converged: x is the helper's); counted by warm_finish, when the solve is used
        *use_s = hy.x == e ? (int)((hy.z << 3) | (hy.y == 0u ? 0u : hy.y == 1u ? 2u : 1u)) : -1;
        *e_s = e;
        return;
    }
    uint4 sy = ld_nc_u32x4(w.sync);   // {published, inverted, stop, PD}: as above, one load per poll
    const unsigned e = sy.x;
    int use = 0;
    if (e == 0) {
        w.stats[3] += 1;
    } else {
        if (sy.y != e) {
            w.stats[4] += 1;   // waited for the helper (the branch taken below does not depend on it)
            const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
            while (sy.y != e && (long long)__builtin_amdgcn_s_memrealtime() - t0 < w.wait_ticks) {
                __builtin_amdgcn_s_sleep(2);
                sy = ld_nc_u32x4(w.sync);
            }
        }
        const unsigned h = sy.y, ok = sy.w;
        use = h != e ? -1 : ok ? 1 : 0;
        if (use == 0) w.stats[3] += 1;
    }
    *use_s = use;
    *e_s = e;
}
__device__ void warm_finish(const double* packed, const WarmCtx& w, double* x, int m, int* err, const WarmStage& ws,
                            int use, unsigned e, int* bad_lds, long long* stp = nullptr) {
    const int tid = threadIdx.x, M = 16 * ((m + 15) / 16), n2 = warm_lc2(m);
    double* Pk = x + kWarmN;                         // staged packed [S | r] (x: kWarmN doubles)
    double* Iv = Pk + 2 * n2;                        // staged S_t^-1
    double* work = Iv + (size_t)M * (M + 2);
    double* prev = w.prev2 + (size_t)(e & 1u) * w.prev_stride;   // iteration e's copy
    if (w.refine) {   // the helper's solution (use 2), else the direct elimination; k_schur published
        if (tid == 0) {
            if ((use & 7) == 0) {
                w.stats[3] += 1;
            } else {
                w.stats[0] += 1;
                w.stats[1] += use >> 3;
                if ((use & 7) == 1) w.stats[2] += 1;
            }
        }
        if ((use & 7) == 2) {
            for (int t = tid; t < kWarmN; t += blockDim.x)
                x[t] = t < m ? __longlong_as_double((long long)__hip_atomic_load(reinterpret_cast<unsigned long long*>(w.xsol + t),
                                                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM))
                             : 0.0;
            lds_barrier();
        } else {
            gj_blocked(packed, x, x + M, x + M + M * (M + 1), m, err, nullptr, bad_lds);
        }
        SSTAMP(stp, 11, 0);
        return;
    }
#pragma unroll
    for (int u = 0; u < kWarmPer; ++u) {
        const int q = u * (int)blockDim.x + tid;
        if (q < n2) {
            reinterpret_cast<double2*>(Pk)[q] = ws.v[u];
            if (w.copy_prev) st_sys_x2(prev + 2 * q, ws.v[u].x, ws.v[u].y);   // sharded: the summed system
        }
    }
    SSTAMP(stp, 8, 0);   // [S | r] staged
    // single GPU: publish this step's system (k_schur left it in prev2[e & 1]) for the helper as soon
    // as this k_solve no longer needs S_t^-1 -- at once on the direct path, after S_t^-1 is in LDS
    // otherwise; sharded: after this k_solve's own copy has drained (at the end)
    const bool early = !w.copy_prev;
    if (early && use <= 0 && tid == 0) st_sys_u32(w.sync, e + 1u);
    bool solved = false;
    if (use > 0) {
        // S_t^-1 (one memory round trip) into registers; meanwhile the refinement gathers its
        // rows of S_{t+1} from the staged packed system; then S_t^-1 into LDS, rows padded to
        // M + 2 (16 rows of a wave would otherwise share banks).  (Its packed upper triangle, half
        // the bytes, was slower: mirroring it into LDS cost more than the saved load, round 4.)
        constexpr int kIvPer = 9;   // double2 per thread: M x M / 2 <= 4 608 at 512 threads
        const int n2i = M * M / 2;
        double2 iv[kIvPer];
#pragma unroll
        for (int u = 0; u < kIvPer; ++u) {
            const int q = u * (int)blockDim.x + tid;
            iv[u] = q < n2i ? reinterpret_cast<const double2*>(w.sinv)[q] : make_double2(0.0, 0.0);
        }
        lds_barrier();   // the staged packed system
        double Sr[kWarmQ];
        warm_gather_s(Pk, m, Sr);
#pragma unroll
        for (int u = 0; u < kIvPer; ++u) {
            const int q = u * (int)blockDim.x + tid;
            if (q < n2i) {
                const int t = 2 * q, r = t / M, c = t % M;
                *reinterpret_cast<double2*>(Iv + r * (M + 2) + c) = iv[u];
            }
        }
        lds_barrier();
        if (early && tid == 0) st_sys_u32(w.sync, e + 1u);
        SSTAMP(stp, 9, 0);   // S_t^-1 in LDS, the rows of S_{t+1} gathered
        solved = warm_refine<false>(Sr, Iv, M + 2, Pk, x, work, m, w.stats);
        SSTAMP(stp, 10, 0);   // refined
    }
    if (!solved) gj_blocked(packed, x, x + M, x + M + M * (M + 1), m, err, nullptr, bad_lds);
    SSTAMP(stp, 11, 0);
    if (!early) {   // sharded: publish after the copy's stores drained
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        lds_barrier();
        if (tid == 0) st_sys_u32(w.sync, e + 1u);
    }
}

// In-place blocked Gauss-Jordan inverse of the padded SPD system in LDS (A: M x M, stride ld = M + 1,
// 16 x 16 blocks; the helper).  Per pivot block kb: P^-1 (gjb_inverse16); the pivot block row
// A[kb][j] <- P^-1 A[kb][j]; every other block A[i][j] -= A[i][kb] A[kb][j]; the pivot block column
// A[i][kb] <- -A[i][kb] P^-1 and A[kb][kb] <- P^-1.  Scheduled with a look-ahead (round 6): in kb's
// block update wave 0 takes the next pivot block (kb + 1, kb + 1) first and inverts it while the
// other waves update the rest, and the pivot column of kb shares one phase with the pivot row of
// kb + 1 (block (kb + 1, kb) goes through both, in that order, on one wave) -- two barriers per pivot
// block instead of four, and the serial 16 x 16 inverse (1.65 us of the 4.9 us per block) off the
// critical path except its own chain.  The same products in the same order: bitwise the round-5
// schedule's inverse.  m = 90: 29.1 -> 22.8 us alone on a CU (tools/inv_bench.hip; 19.1 with the first
// pivot block as a separate prologue, which spilled the helper).  PV0, PV1: the
// 16 x kBlkLd scratch of the even and odd pivot blocks.  Returns false (every thread) if a pivot is not > 0.
// LA = false: the round-5 schedule (four phases per pivot block, PV0 only).  WarmCtx::inv_la picks:
// the look-ahead where the helper's cycle bounds the step (k_group's short steps: the config3 x8 shard
// 45.0 -> 41.1 us), round 5's where the inversion overlaps a long linearisation -- there the denser
// look-ahead slowed the co-resident linearisation workgroups (config3 107.8 -> 109.3 us per step).
template <bool LA>
__device__ bool gj_inverse_blocked(double* A, double* PV0, double* PV1, int M) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
    const int nb = M / 16, n1 = nb - 1, ld = M + 1;
    __shared__ int bad_s;
    if (tid == 0) bad_s = 0;
    auto blk = [&](int ib, int jb) { return A + 16 * ib * ld + 16 * jb; };
    auto pvb = [&](int kb) { return kb & 1 ? PV1 : PV0; };
    if (!LA) {
        for (int kb = 0; kb < nb; ++kb) {
            if (wave == 0 && !gjb_inverse16(blk(kb, kb), ld, PV0, lane) && lane == 0) bad_s = 1;
            __syncthreads();
            for (int it = wave; it < n1; it += nw) {   // pivot block row
                double* C = blk(kb, it < kb ? it : it + 1);
                blk_mfma(C, ld, PV0, kBlkLd, C, ld, false, true);
            }
            __syncthreads();
            for (int it = wave; it < n1 * n1; it += nw) {   // the other blocks
                const int r = it / n1, c = it % n1;
                const int ib = r < kb ? r : r + 1, jb = c < kb ? c : c + 1;
                blk_mfma(blk(ib, jb), ld, blk(ib, kb), ld, blk(kb, jb), ld, true, false);
            }
            __syncthreads();
            for (int it = wave; it < nb; it += nw) {   // the pivot block column, and the pivot block
                double* C = blk(it, kb);
                if (it != kb) {
                    blk_mfma(C, ld, C, ld, PV0, kBlkLd, true, true);
                } else {
                    const int i = lane & 15, g = lane >> 4;
#pragma unroll
                    for (int c = 0; c < 4; ++c) C[i * ld + 4 * g + c] = PV0[i * kBlkLd + 4 * g + c];
                }
            }
            __syncthreads();
        }
        return bad_s == 0;
    }
    // kb = -1: the first pivot block's inverse, then its pivot block row
    for (int kb = -1; kb < nb; ++kb) {
        const bool next = kb + 1 < nb;
        if (next && wave == 0) {   // the next pivot block first, then its inverse
            if (kb >= 0) blk_mfma(blk(kb + 1, kb + 1), ld, blk(kb + 1, kb), ld, blk(kb, kb + 1), ld, true, false);
            if (!gjb_inverse16(blk(kb + 1, kb + 1), ld, pvb(kb + 1), lane) && lane == 0) bad_s = 1;
        } else if (kb >= 0) {
            const int w0 = next ? wave - 1 : wave, nws = next ? nw - 1 : nw;
            const int skip = next ? kb * n1 + kb : n1 * n1;   // (kb + 1, kb + 1): wave 0's
            for (int it = w0; it < n1 * n1 - (next ? 1 : 0); it += nws) {
                const int t = it < skip ? it : it + 1;
                const int r = t / n1, c = t % n1;
                const int ib = r < kb ? r : r + 1, jb = c < kb ? c : c + 1;
                blk_mfma(blk(ib, jb), ld, blk(ib, kb), ld, blk(kb, jb), ld, true, false);
            }
        }
        __syncthreads();
        // items < ncol: the pivot block column of kb (item kb + 1, dealt first, also takes its block
        // through the pivot row of kb + 1); the rest: that row's other blocks (columns other than kb, kb + 1)
        const int ncol = kb >= 0 ? nb : 0;
        const int nrow = next ? (kb >= 0 ? nb - 2 : nb - 1) : 0;
        for (int it0 = wave; it0 < ncol + nrow; it0 += nw) {
            if (it0 < ncol) {
                const int it = next && it0 <= kb + 1 ? (it0 == 0 ? kb + 1 : it0 - 1) : it0;
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
                const int q = it0 - ncol;
                const int jb = kb < 0 ? q + 1 : (q < kb ? q : q + 2);
                double* C = blk(kb + 1, jb);
                blk_mfma(C, ld, pvb(kb + 1), kBlkLd, C, ld, false, true);
            }
        }
        __syncthreads();
    }
    return bad_s == 0;
}

// The resident helper (one workgroup on a side stream, launched with each batch of update steps):
// for each system k_solve publishes (sync[0] past the last one inverted), copy sprev into LDS,
// invert it (gj_inverse_blocked), store S^-1 (uncached), drain, publish sync[1].  It exits after
// n_systems systems, when a k_solve reports that no more systems follow (sync[2]: the loop
// stopped, a failed step, a peer timeout), or after kHelperIdleTicks without a new system: every
// wave reaches the exit.
#if MCC_IN(5)
// With WarmCtx::refine (single GPU) the helper also SOLVES each system: k_schur's final arriver
// publishes the system as soon as its copy in prev2 is complete (sync[0] = iteration + 1), the helper
// stages it, refines with the inverse of the previous system it still holds in LDS (the same
// warm_refine, the same bits k_solve would form), publishes x (xsol, then sync[5] status, sync[6]
// corrections, sync[4] = the epoch) and only then inverts the new system in place.  k_solve waits for
// sync[4] instead of loading S_t^-1 (74 KB) and refining: 3.1 + 3.4 us of its 10.5 us at m = 90
// (tools/diag_solve.py), which now run while k_schur ends and k_solve starts.  The refinement runs
// only with the inverse of system e - 1 (a batch's helper starts from sinv and the epoch sync[1]
// names), so its branch is a function of the systems alone, as before.
// LA: the look-ahead inversion (WarmCtx::inv_la; a template, as both schedules inlined into one kernel
// spilled it)
template <bool LA>
__global__ __launch_bounds__(kSolveThreads) void k_sinv_helper(WarmCtx w, int m, int n_systems) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    __shared__ unsigned ep_s;
    __shared__ int quit_s, have_s;
    const int tid = threadIdx.x, M = 16 * ((m + 15) / 16), ld = M + 1;
    double* A = sm;
    double* PV = sm + M * ld;
    const int n2 = warm_lc2(m);
    double* Pk = PV + 16 * kBlkLd;   // refine: the staged packed [S | r] (even length)
    double* xs = Pk + 2 * n2;        // refine: the solution [kWarmN]
    double* work = xs + kWarmN;      // refine: warm_refine's residual and wave maxima
    unsigned seen = ld_sys_u32(w.sync + 1);
    unsigned held = 0u;   // refine: the epoch whose inverse A holds
    // A -> sinv (ordinary, cached memory: this XCD's L2 written back before an epoch says it is there;
    // its readers run in later launches, whose start drops stale lines from their own caches)
    auto dump_inverse = [&]() {
        for (int q = tid; q < M * M / 2; q += blockDim.x) {
            const int t = 2 * q, i = t / M, j = t % M;
            *reinterpret_cast<double2*>(w.sinv + t) =
                w.poison ? make_double2(__builtin_nan(""), __builtin_nan("")) : make_double2(A[i * ld + j], A[i * ld + j + 1]);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    };
    if (w.refine) {
        // the inverse the previous batch's helper left (sinv, for epoch sync[1], positive definite)
        const bool have = seen != 0u && ld_sys_u32(w.sync + 3) != 0u;
        if (have) {
            for (int t = tid; t < M * M; t += blockDim.x) A[(t / M) * ld + t % M] = w.sinv[t];
            held = seen;
        }
        if (tid == 0) have_s = have;
    }
    for (int k = 0; k < n_systems; ++k) {
        if (tid == 0) {
            const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
            unsigned e = ld_sys_u32(w.sync);
            int quit = 0;
            while (e == seen) {
                if (ld_sys_u32(w.sync + 2) || (long long)__builtin_amdgcn_s_memrealtime() - t0 > w.idle_ticks) {
                    quit = 1;
                    break;
                }
                __builtin_amdgcn_s_sleep(8);
                e = ld_sys_u32(w.sync);
            }
            ep_s = e;
            quit_s = quit;
        }
        __syncthreads();
        if (quit_s) {
            if (w.refine && held != 0u) {   // the next batch's helper starts from it (sync[1], sync[3])
                dump_inverse();
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            return;
        }
        const unsigned e = ep_s;
#ifdef MCC_DIAG   // (the helper's phases: seen, staged, S gathered, refined, x published, inverted; [6] the
                  // corrections, [7] the epoch; [15] stays -1, the host's marker)
#define HSTAMP(k) do { if (tid == 0 && w.hst) w.hst[(e & 3u) * 16 + (k)] = (long long)MCC_DIAG_CLOCK(); } while (0)
        if (tid == 0 && w.hst) w.hst[(e & 3u) * 16 + 7] = e;
#else
#define HSTAMP(k) do { } while (0)
#endif
        HSTAMP(0);
        // system e (solved by the update step whose iteration counter was e - 1: k_schur wrote it to
        // prev2[(e - 1) & 1]) -> the full symmetric matrix in LDS (padding: identity)
        const int ntri = m * (m + 1) / 2;
        const double* src = w.prev2 + (size_t)((e - 1u) & 1u) * w.prev_stride;
        if (w.refine) {
            // [S | r] staged, x = S^-1 r refined with the held inverse of system e - 1, published.
            // k_schur publishes e when it STARTS (round 6; it used to after its second hand-off level), and
            // every word of prev2 is its own flag (kFoldEmpty until its block's sc1 store lands; the helper
            // empties the buffer again once it has refined), so the staging polls the words as the blocks
            // land instead of starting after the last one: 5 x 16-byte loads per thread (the landed ones
            // re-read at the buffer's first word), a short sleep between passes.  The pad word of an odd
            // packed length is 0 for good (mcc_create).  (n2 <= 2 093 at m = 90: one batch of 512 x 5)
            if (!w.poll) {   // (published complete: round 5's one batch -- the polling loop below cost the
                             // 8-rank shard, whose step the helper's cycle bounds, 0.9 us even in one pass)
                for (int q0 = 0; q0 < n2; q0 += 5 * (int)blockDim.x) {
                    const double* pq[5];
#pragma unroll
                    for (int u = 0; u < 5; ++u) pq[u] = src + 2 * min(q0 + u * (int)blockDim.x + tid, n2 - 1);
                    f64x2_t v[5];
                    ld_nc_x2_5(pq[0], pq[1], pq[2], pq[3], pq[4], v);
#pragma unroll
                    for (int u = 0; u < 5; ++u) {
                        const int q = q0 + u * (int)blockDim.x + tid;
                        if (q < n2) reinterpret_cast<double2*>(Pk)[q] = make_double2(v[u].x, v[u].y);
                    }
                }
                __syncthreads();
            } else {
                unsigned got = 0u;
                const long long tp = (long long)__builtin_amdgcn_s_memrealtime();
                for (;;) {
                    const double* pq[5];
#pragma unroll
                    for (int u = 0; u < 5; ++u) {
                        const int q = u * (int)blockDim.x + tid;
                        pq[u] = src + ((got >> u) & 1u || q >= n2 ? 0 : 2 * q);
                    }
                    f64x2_t v[5];
                    ld_nc_x2_5(pq[0], pq[1], pq[2], pq[3], pq[4], v);
                    int pend = 0;
#pragma unroll
                    for (int u = 0; u < 5; ++u) {
                        const int q = u * (int)blockDim.x + tid;
                        if (q >= n2 || ((got >> u) & 1u)) continue;
                        if (__double_as_longlong(v[u].x) != kFoldEmpty && __double_as_longlong(v[u].y) != kFoldEmpty) {
                            reinterpret_cast<double2*>(Pk)[q] = make_double2(v[u].x, v[u].y);
                            got |= 1u << u;
                        } else {
                            ++pend;
                        }
                    }
                    if (!__syncthreads_or(pend)) break;
                    if (tid == 0)   // (a failed step or the loop's end: no more words will land)
                        quit_s = ld_sys_u32(w.sync + 2) || (long long)__builtin_amdgcn_s_memrealtime() - tp > w.idle_ticks;
                    __syncthreads();
                    if (quit_s) {   // (as below: the next batch's helper starts from the inverse this one holds)
                        if (held != 0u) {
                            dump_inverse();
                            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        }
                        return;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
            }
            HSTAMP(1);
            int status = 0, corr = 0;
#ifdef MCC_HELPER_RELOAD   // (A/B debug builds only)
            if (have_s && held == e - 1u) {
                for (int t = tid; t < M * M; t += blockDim.x) A[(t / M) * ld + t % M] = w.sinv[t];
                __syncthreads();
            }
#endif
#ifdef MCC_HELPER_BARRIER   // (A/B debug builds only)
            __syncthreads();
#endif
            if (have_s && held == e - 1u) {
                // (m and the LDS bases re-derived per system: hoisted out of the system loop, the
                // refinement's addresses held ~160 SGPRs for the whole kernel and spilled)
                int mo = m;
                asm volatile("" : "+s"(mo));
                const int Mo = 16 * ((mo + 15) / 16), ldo = Mo + 1;
                double* Ao = sm;
                double* Pko = sm + Mo * ldo + 16 * kBlkLd;
                double* xso = Pko + 2 * warm_lc2(mo);
                double Sr[kWarmQ];
                warm_gather_s(Pko, mo, Sr);
                HSTAMP(2);
                const bool conv = warm_refine<true>(Sr, Ao, ldo, Pko, xso, xso + kWarmN, mo, nullptr, &corr);
                status = conv && !w.poison ? 1 : 2;   // (test: a poisoned helper's solves all fall back)
            }
            HSTAMP(3);
#ifdef MCC_DIAG
            if (tid == 0 && w.hst) w.hst[(e & 3u) * 16 + 6] = corr;
#endif
            if (status == 1)
                for (int t = tid; t < m; t += blockDim.x)
                    __hip_atomic_store(reinterpret_cast<unsigned long long*>(w.xsol + t), (unsigned long long)__double_as_longlong(xs[t]),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if (tid == 0) {   // (with x: k_solve trusts them only once the epoch below matches, and the
                              // previous system's k_solve has ended before this system was published)
                st_sys_u32(w.sync + 5, (unsigned)status);
                st_sys_u32(w.sync + 6, (unsigned)corr);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0 && w.delay_ticks > 0) {   // test: a slow helper (k_solve must wait, not switch)
                const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
                while ((long long)__builtin_amdgcn_s_memrealtime() - t0 < w.delay_ticks) __builtin_amdgcn_s_sleep(8);
            }
            if (tid == 0) st_sys_u32(w.sync + 4, e);
            HSTAMP(4);
            // (the words go back to kFoldEmpty in the next step's k_schur, schur_block_store: 33 KB of
            // stores here lengthened the helper's cycle, which bounds the 8-rank shard's step)
            for (int t = tid; t < ntri; t += blockDim.x) {
                int i, j;
                packed_ij(t, m, i, j);
                const double x = Pk[t];
                A[i * ld + j] = x;
                A[j * ld + i] = x;
            }
        } else {
            for (int t = tid; t < ntri; t += blockDim.x) {
                int i, j;
                packed_ij(t, m, i, j);
                const double x = ld_sys_f64(src + t);
                A[i * ld + j] = x;
                A[j * ld + i] = x;
            }
        }
        for (int t = tid; t < M * M; t += blockDim.x) {
            const int i = t / M, j = t % M;
            if (i >= m || j >= m) A[i * ld + j] = i == j ? 1.0 : 0.0;
        }
        __syncthreads();
        // (the odd pivot blocks' scratch: refine, the staged system, copied into A by now; else its own)
        const bool ok = gj_inverse_blocked<LA>(A, PV, PV + 16 * kBlkLd, M);
        HSTAMP(5);
#undef HSTAMP
#ifdef MCC_HELPER_RELOAD
        dump_inverse();
#else
        if (!w.refine) dump_inverse();   // (refine: the inverse stays in LDS; sinv only when the helper exits)
#endif
#ifdef MCC_HELPER_RELOAD_END   // (A/B debug builds only)
        dump_inverse();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        for (int t = tid; t < M * M; t += blockDim.x) A[(t / M) * ld + t % M] = w.sinv[t];
#endif
        if (tid == 0) st_sys_u32(reinterpret_cast<unsigned*>(w.sinv_ok_sys), ok ? 1u : 0u);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (!w.refine && tid == 0 && w.delay_ticks > 0) {   // test: a slow helper (k_solve must wait, not switch)
            const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
            while ((long long)__builtin_amdgcn_s_memrealtime() - t0 < w.delay_ticks) __builtin_amdgcn_s_sleep(8);
        }
        if (tid == 0) st_sys_u32(w.sync + 1, e);
        seen = e;
        held = e;
        if (tid == 0) have_s = ok;   // (read after the next system's barrier)
    }
    if (w.refine && held != 0u) {
        dump_inverse();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
}
#endif  // MCC_IN(5)

__device__ void gj_dispatch(const double* S, double* r, int m, int lane, int* err, int* bad_lds = nullptr) {
    switch (m) {
#define GJ(M) case M: gj_rows<M>(S, r, m, lane, err, bad_lds); break;
        GJ(6) GJ(12) GJ(18) GJ(24) GJ(30)
#undef GJ
        default: break;
    }
}

// ---------------------------------------------------------------- the m <= 30 warm solve
// The previous Gauss-Newton step's reduced system changes little by the next step, so its inverse is
// a preconditioner good enough that iterative refinement reaches the elimination's accuracy in one or
// two corrections -- a few 18 x 18 products on one wave against the 18-pivot register Gauss-Jordan's
// chain of broadcasts (~5.4 k cycles).  The inverse is formed OFF the critical
// path: k_group launches one spare workgroup beyond its groups (250 groups on 256 CUs at config4), which
// inverts the packed system the previous step's k_schur left (gj_inverse_rows) while the groups
// linearise; k_schur's final arriver reads it after the kernel boundary.  The fused step (k_linearize)
// appends the spare to the same launch whose final arriver rewrites the packed system and the state, so
// there the spare acknowledges (State::spare_ack = iteration + 1) once it holds its inputs in LDS, and
// the final arriver writes neither before it has seen that (spare_wait): the spare always inverts the
// previous launch's system and tags it with this launch's iteration, however late it is scheduled.
// Every step forms it, so the branch a step takes -- refinement, or the elimination when there is no
// previous system (an optimisation's first step, a linearisation-only step) or the refinement does not
// converge -- is a function of the systems alone, never of timing.

// Gauss-Jordan on [S | I] in LDS by the whole workgroup (S from the packed upper triangle in global
// memory; thread-per-element updates, two barriers per pivot: ~2 us at m = 18, off the critical path,
// and no register arrays that would raise k_group's register pressure); Sinv row i = (E row i) / d_i.
// ok = 0 when a pivot is not > 0.  ack: the fused step's spare (above).
__device__ __forceinline__ void small_inverse(const LinArgs& a, double* A, bool ack) {
    State* st = a.state;
    const int tid = threadIdx.x, nt = blockDim.x, m = a.global_dim, W = 2 * m;
    if ((ack || a.fold) && a.spare_delay > 0) {   // test (MCC_SPARE_DELAY_US): a spare scheduled late
        if (tid == 0) {
            const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
            while ((long long)__builtin_amdgcn_s_memrealtime() - t0 < a.spare_delay) __builtin_amdgcn_s_sleep(8);
        }
        __syncthreads();
    }
    // buffer iteration & 1, tagged iteration + 1 (0: none): k_schur of this step reads it, the fused
    // step's final arriver of the NEXT launch does (this launch's is still inverting).  A fused launch
    // that updates nothing (linearisation only) has no spare (enqueue_step).
    const int done = st->done, it = st->iter, pend = st->pending;
    if (done) return;   // (the photos see the same word)
    const unsigned seq = (unsigned)it;
    // k_group's folded step (a.fold): the final workgroup of THIS launch reads the inverse -- sc1
    // stores into fiv, each word its own flag, and the status word +(it + 1) (an inverse) or -(it + 1)
    // (none) as a double, written after this workgroup read the packed system and the state: the final workgroup
    // writes neither before it has seen the status
    const bool fold = a.fold != 0;
    double* out = fold ? a.fiv : a.ssinv + (size_t)(it & 1) * m * m;
    int* okp = a.ssinv_ok + (it & 1);
    __shared__ int ok_s;
    if (!pend) {   // no update step before this one: no system to precondition with
        if (tid == 0) {
            if (fold) st_sc1(a.fiv + m * m, -(double)(it + 1));   // (a double: -1 as bits would read as empty)
            else *okp = 0;
            if (ack) __hip_atomic_store(&st->spare_ack, seq + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        return;
    }
    for (int t = tid; t < m * W; t += nt) {
        const int i = t / W, j = t % W;
        double v;
        if (j < m) {
            const int lo = i < j ? i : j, hi = i < j ? j : i;
            v = a.packed[lo * m - lo * (lo - 1) / 2 + (hi - lo)];
        } else {
            v = j - m == i ? 1.0 : 0.0;
        }
        A[t] = v;
    }
    if (tid == 0) ok_s = 1;
    __syncthreads();   // every thread's loads have landed in LDS (and the state words in registers)
    if (ack && tid == 0) __hip_atomic_store(&st->spare_ack, seq + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int k = 0; k < m; ++k) {
        const double piv = A[k * W + k];
        if (!(piv > 0.0)) {
            if (tid == 0) ok_s = 0;
            break;   // uniform: every thread read the same pivot
        }
        const double ip = 1.0 / piv;
        double nv[8];   // <= 8 elements per thread: 30 x 60 over 256 threads (k_group's 16-lane form)
        int nn = 0;
        for (int t = tid; t < m * W; t += nt, ++nn) {
            const int i = t / W, j = t % W;
            nv[nn & 7] = i == k ? A[t] : A[t] - A[i * W + k] * ip * A[k * W + j];
        }
        __syncthreads();
        nn = 0;
        for (int t = tid; t < m * W; t += nt, ++nn) A[t] = nv[nn & 7];
        __syncthreads();
    }
    __syncthreads();
    const bool ok = ok_s != 0;
    if (ok)
        for (int t = tid; t < m * m; t += nt) {
            const int i = t / m, j = t % m;
            const double v = A[i * W + m + j] / A[i * W + i];
            if (fold) st_sc1(out + t, v);
            else out[t] = v;
        }
    if (tid == 0) {
        if (fold) st_sc1(a.fiv + m * m, ok ? (double)(it + 1) : -(double)(it + 1));
        else *okp = ok ? it + 1 : 0;
    }
}

// x = S^-1 r by refinement with Iv (m x m) on one wave: x0 = Iv r, x += Iv (r - S x) until every
// equation holds to its own scale, |r - S x|_i <= 64 eps (|S| |x| + |r|)_i (the warm solve's test),
// at most kWarmMaxIters corrections, each cutting the error fourfold.  Two lanes share row i (lanes
// 2i, 2i+1, m <= 30): each holds half of the row of S and of Iv in registers (read once) and takes
// the matching half of the vector from a 32-entry LDS slot that the even lanes write, so a product
// is m/2 LDS reads and FMAs per lane plus one DPP exchange of the two half sums.  Round 4 broadcast
// the vector by m v_readlane pairs per product (~1.9 us of refinement at m = 18); round 4's first
// form read S and Iv from LDS per product (~3 us).  On success r holds x.
template <int MM>
__device__ __forceinline__ bool small_refine_reg(const double* S, double* r, const double* Iv, int m, int lane, int* corr,
                                                 double* vb) {
    constexpr int H = MM / 2;
    // a necessary condition for S > 0 that the direct elimination's pivots would test: a non-positive
    // (or NaN) diagonal entry sends the system to gj_rows, which reports it (MCC_ENOTPD)
    const int li = lane < m ? lane : 0;
    if (__builtin_amdgcn_ballot_w64(lane < m && !(S[li * m + li] > 0.0))) return false;
    const int i = lane >> 1, c0 = (lane & 1) * H;
    const bool act = i < MM, wr = act && (lane & 1) == 0;
    const int ri = act ? i : 0;
    double sr[H], ir[H], w[H];
#pragma unroll
    for (int k = 0; k < H; ++k) {
        sr[k] = S[ri * MM + c0 + k];
        ir[k] = Iv[ri * MM + c0 + k];
        w[k] = r[c0 + k];
    }
    const double rr = r[ri];
    double p = 0.0;
#pragma unroll
    for (int k = 0; k < H; ++k) p = fma(ir[k], w[k], p);
    double x = p + dpp_f64<kDppXor1>(p);   // both lanes of the row: the same sum, the same rounding
    constexpr double kTol = 64.0 * 1.1102230246251565e-16;
    bool conv = false;
    double qprev = 0.0;
    for (int it = 0;; ++it) {
        if (wr) vb[i] = x;
        wave_sync_lds();
        double ps = 0.0, pa = 0.0;
#pragma unroll
        for (int k = 0; k < H; ++k) {
            const double xj = vb[c0 + k];
            ps = fma(sr[k], xj, ps);
            pa = fma(fabs(sr[k]), fabs(xj), pa);
        }
        wave_sync_lds();
        const double res = rr - (ps + dpp_f64<kDppXor1>(ps));
        const double sa = fabs(rr) + (pa + dpp_f64<kDppXor1>(pa));
        const double q = act ? (fabs(res) / fmax(sa, 1e-300)) : 0.0;
        const double qm = wave_max(q == q ? q : 1.0);
        conv = qm <= kTol;
        if (conv || it >= kWarmMaxIters || (it > 0 && !(qm <= 0.25 * qprev))) break;
        qprev = qm;
        *corr = it + 1;
        if (wr) vb[i] = res;
        wave_sync_lds();
        double pd = 0.0;
#pragma unroll
        for (int k = 0; k < H; ++k) pd = fma(ir[k], vb[c0 + k], pd);
        wave_sync_lds();
        x += pd + dpp_f64<kDppXor1>(pd);
    }
    if (conv && wr) r[i] = x;   // r was read by every lane above (one wave: in order)
    return conv;
}
__device__ __forceinline__ bool small_refine(const double* S, double* r, const double* Iv, int m, int lane, int* corr,
                                             double* vb) {
    switch (m) {
#define SR(M) case M: return small_refine_reg<M>(S, r, Iv, m, lane, corr, vb);
        SR(6) SR(12) SR(18) SR(24) SR(30)
#undef SR
        default: return false;
    }
}

// LARGE: m > 30 (k_solve only: the register-tiled elimination needs the whole workgroup's registers)
template <bool LARGE>
__device__ __forceinline__ void solve_global(const SolveCtx& a, double* S, double* r, double normG2, double normX2,
                                             const WarmCtx* warm, const double* Iv) {
    State* st = a.state;
    const int m = a.m, tid = threadIdx.x;
    __shared__ int stop, s_iter;
    __shared__ double s_alpha;
    __shared__ float s_x[128];
    __shared__ int s_use, s_bad, s_bad_rows, s_err0;
    __shared__ unsigned s_ep;
    SSTAMP(a.stamps, 0, 0);
    const bool wrm = LARGE && warm_on(warm, m);
    __shared__ int s_sm_ok, s_sm_corr;   // m <= 30: the refinement converged, with this many corrections
    __shared__ double s_rv[32];          // m <= 30: the refinement's vector exchange
    WarmStage ws;
    if (wrm && !warm->refine) warm_issue(S, m, ws);
    if (wrm && tid == 64) warm_check(*warm, &s_use, &s_ep);
    if (tid == 0) {
        // the error bits the step's photo work set (bit 0), read with the state so that the stop
        // at the end needs no further round trip.  On a sharded problem a photo block that is not
        // positive definite on ANY rank arrives here as a NaN in the summed normX2 slot
        // (photo_flag_norm): every rank then stops on the same step with the same error
        s_err0 = __hip_atomic_load(&st->error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (!(normX2 == normX2)) s_err0 |= kErrPhotoNotPD;
        s_bad = 0;
        const int k = st->iter;
        double change = 1.0;
        if (k > 0) {
            change = sqrt(normG2) / sqrt(normX2);   // change = norm(G) / norm(x) (:504)
            st->change = change;
        }
        const int ty = st->crit_type;
        int s = (ty == 1 && k >= st->max_count) || (ty == 2 && change <= st->eps) ||
                (ty == 3 && (change <= st->eps || k >= st->max_count));
        if (!a.do_update) s = 0;
        stop = s;
        if (s) st->done = 1;
        st->pending = 0;   // this step's k_linearize has applied the previous update
        const double alpha = a.do_update ? (k < a.n_alpha ? a.alpha[k] : pow(0.95, (double)k + 1.0)) : 0.0;
        st->alpha = alpha;
        s_alpha = alpha;
        s_iter = k;
    } else if (tid >= 128 && tid < 128 + m) {
        s_x[tid - 128] = a.x[tid - 128];   // global-block parameters, fetched while wave 1 eliminates
    } else if (!LARGE && tid >= 64 && tid < 128) {
        // speculative: the elimination does not depend on the stop test (its result is unused
        // when the loop stops), so wave 1 runs it while wave 0 loads the state
        SSTAMP(a.stamps, 1, 64);
        if (tid == 64) s_bad_rows = 0;   // (this wave's own write below follows in program order)
        // with the previous system's inverse (k_schur, m <= 30): refinement, else / on failure the
        // register Gauss-Jordan
        int corr = 0;
        const bool ok = Iv && small_refine(S, r, Iv, m, tid - 64, &corr, s_rv);
        if (tid == 64) {   // (statistics, read after the barriers below)
            s_sm_ok = ok;
            s_sm_corr = corr;
        }
        if (!ok) gj_dispatch(S, r, m, tid - 64, &st->error, &s_bad_rows);
        SSTAMP(a.stamps, 2, 64);
    }
    __syncthreads();
    if (stop) {
        if (warm) warm_stop(*warm);
        return;
    }
    if (wrm && s_use < 0) {   // the helper did not deliver: fail the step rather than switch algorithms
        if (tid == 0) {
            atomicOr(&st->error, kErrWarmTimeout);
            st->done = 1;
        }
        warm_stop(*warm);
        return;
    }
    SSTAMP(a.stamps, 4, 0);
    if (LARGE) {   // S is the packed system itself (global); r (LDS) is followed by the block work area
        const int M = 16 * ((m + 15) / 16);
        if (wrm) warm_finish(S, *warm, r, m, &st->error, ws, s_use, s_ep, &s_bad, a.stamps);
        else gj_blocked(S, r, r + M, r + M + M * (M + 1), m, &st->error, nullptr, &s_bad);
    }
    SSTAMP(a.stamps, 5, 0);
    if (tid < 64) {
        const int lane = tid;
        // global block: delta, update, norm partials (identical on every rank)
        const double alpha = s_alpha;
        double g2 = 0.0, x2 = 0.0;
        for (int i = lane; i < m; i += 64) {
            const double d = r[i];
            a.dg[i] = d;
            a.delta[i] = d;
            if (a.do_update) {
                const float G = (float)(alpha * d);   // G = alpha*delta -> CV_32F (:491-496)
                const float xn = s_x[i] + G;          // x = x + G (:501)
                a.x[i] = xn;
                g2 += (double)G * (double)G;
                x2 += (double)xn * (double)xn;
            }
        }
        SSTAMP(a.stamps, 6, 0);
        g2 = wave_sum(g2);
        x2 = wave_sum(x2);
        if (lane == 0 && a.do_update) {
            st->cam_normG2 = g2;
            st->cam_normX2 = x2;
            st->iter = s_iter + 1;
            st->pending = 1;
        }
    }
    // a step that hit a not-positive-definite block (a photo's: bit 0, set by the photo workgroups
    // before their tickets; the reduced system's: bit 1, set by this workgroup's elimination) stops
    // the steps after it, as mcc_check documents; the kernels test `done` only at their entry, so
    // no launch in flight loses a workgroup's ticket
    __syncthreads();
    if (tid == 0 && ((s_err0 & 3) || s_bad || (!LARGE && s_bad_rows))) {
        if (s_err0 & kErrPhotoNotPD) atomicOr(&st->error, kErrPhotoNotPD);   // another rank's photo
        st->done = 1;
        if (warm) warm_stop(*warm);
    }
#ifndef MCC_NO_SSTATS   // (A/B builds only)
    if (!LARGE && tid == 64 && a.sstats) {   // m <= 30 warm-solve statistics, last (nothing waits on them)
        unsigned long long* ss = reinterpret_cast<unsigned long long*>(a.sstats);
        if (Iv) {
            atomicAdd(ss + 0, 1ull);
            atomicAdd(ss + 1, (unsigned long long)s_sm_corr);
            if (!s_sm_ok) atomicAdd(ss + 2, 1ull);
        } else {
            atomicAdd(ss + 3, 1ull);
        }
    }
#endif
}

// ---------------------------------------------------------------- k_schur
// Work item {block, offset of its first slot in doubles, slot count, slot size 48 | 36}: a run of
// consecutive slots of one camera-pair block.  k_photo wrote one slot per (photo group, block):
// the group's sum of the block's pair products (48 doubles: sum of [self] Hgg_a - Y'_a Hgp_b^T,
// [self] (gg_a - Y'_a gp), [self] gg_a; 36 on an off-diagonal block, which has no self pair), so
// an item streams and sums them.  Thread t < 240: entry q = t % 48 (0..35: S entry, 36..41: r entry,
// 42..47: JTE of the global block), sub-chunk s = t / 48.
// Norm items sum 256 photos' norm partials.  Hand-off in two write-through levels (sc1 stores,
// tickets, no fences): the last item of each camera-pair block sums the block's items in item
// order into the packed system [S upper (m(m+1)/2) | r (m) | jte_g (m) | normG2 | normX2]; the
// last of the blocks and norm chunks adds the norms and, with fuse_solve (single GPU), solves.
// (One last-arriver assembling every block alone took ~56 us at m = 90.)
constexpr int kSub = 5;
constexpr int kSchurThreads = 256;   // k_schur's workgroup (mcc_launch_schur)
// entry tid < 48 of camera-pair block blk's sum -> the packed system (write-through)
// prev: the warm solve's copy of [S | r] for the helper (prev2[iteration & 1], uncached), or null;
// with the helper's polled staging (a.wpub_early) the same entries of the OTHER buffer go back to kFoldEmpty: it
// held the previous system, which the helper consumed before the previous step's k_solve could take
// its solution and end, and the system after this one lands there (its words are their own flags)
__device__ __forceinline__ void schur_block_store(const SchurArgs& a, int blk, int tid, double v, double* prev) {
    double* other = prev && a.wpub && a.wpub_early ? prev + (prev == a.prev2 ? a.prev_stride : -a.prev_stride) : nullptr;
    const double empty = __longlong_as_double(kFoldEmpty);
    const int m = a.m, nb = m / 6, ntri = m * (m + 1) / 2;
    int b1 = 0;
    while (b1 + 1 < nb && (b1 + 1) * nb - (b1 + 1) * b1 / 2 <= blk) ++b1;
    const int b2 = b1 + (blk - (b1 * nb - b1 * (b1 - 1) / 2));
    if (tid < 36) {
        const int ii = tid / 6, jj = tid % 6;
        if (b1 != b2 || ii <= jj) {
            const int k = packed_index(6 * b1 + ii, 6 * b2 + jj, m);
            st_sc1(a.packed + k, v);
            if (prev) st_sc1(prev + k, v);
            if (other) st_sc1(other + k, empty);
        }
    } else if (b1 == b2) {
        const int w = (tid - 36) / 6, i = 6 * b1 + (tid - 36) % 6;
        st_sc1(a.packed + ntri + w * m + i, v);   // r (w = 0), JTE of the global block (w = 1)
        if (prev && w == 0) st_sc1(prev + ntri + i, v);
        if (other && w == 0) st_sc1(other + ntri + i, empty);
    }
}
constexpr int kMaxItemsPerBlock = 24;   // host splits each block's pairs into <= 24 items

// m <= 30 (at most 15 camera-pair blocks, a few dozen items): ONE hand-off level.  Every item and
// norm chunk has written its partial (sc1) and takes one ticket; the last arriver sums each block's
// items in item order -- the sums level 1 forms, so the bits are those of the two-level form -- and
// places them straight into the solve's LDS matrix as well as the packed system (plain stores: the
// peer exchange / all-reduce / host read it), instead of a second ticket over the blocks and a reload
// of the packed system.  Round 3 measured the two levels at ~1.8 us each on config4's step tail.
// Every value the final arriver needs -- the partials of all items and norm chunks, the block ranges,
// the warm solve's inverse, the state -- is loaded in ONE round trip into LDS (batches of
// independent unconditional loads: a load under a per-item condition, or a loop whose stores wait
// on its loads, costs a round trip per load or iteration: 5 us at config4 in the first form), and
// the sums are formed from LDS.
__device__ __forceinline__ void schur_finish(const SchurArgs& a, int nparts, int iter, double cn0, double cn1,
                                             int err_now, bool iv, long long* srow);
__device__ __forceinline__ void schur_one_level(const SchurArgs& a, int iter_e) {
    State* st = a.state;
    const int tid = threadIdx.x;
    if (!arrive_last_sc1(a.counter, (int)gridDim.x)) return;
    STAMPP(a.stamps, kSchurStampStride, 2);
    const int m = a.m;
    extern __shared__ __attribute__((aligned(16))) double sm[];
    // the previous system's inverse from k_group's spare workgroup
    double* Iv = a.ssinv && a.fuse_solve ? sm + m * m + m : nullptr;
    double* itm = sm + schur_items_offset(m, a.fuse_solve, a.ssinv != nullptr);   // [grid][48]
    int* sbi = reinterpret_cast<int*>(itm + 48 * (size_t)gridDim.x);                // [nblk + 1]
    __shared__ int iv_ok;
    // ---- the round trip: every load unconditional (uniform words as scalar loads, no branch for
    // the compiler to wait at), consumed only after the barrier
    const int bi = a.block_items[tid < a.nblk ? tid : a.nblk];
    const int iter = st->iter;
    const double cn0 = st->cam_normG2, cn1 = st->cam_normX2;
    const int err_now = photo_error(st);
    // this step's spare workgroup inverted the previous system into buffer iter & 1, tagged iter + 1
    const double* ivsrc = a.ssinv ? a.ssinv + (size_t)(iter_e & 1) * m * m : nullptr;
    const int ivok = Iv ? a.ssinv_ok[iter_e & 1] == iter_e + 1 : 0;
    {
        // one batch of U loads per thread, no loop (a loop's header waits for the previous iteration's
        // loads, and so for the state loads above), U the smallest of 4 / 8 / 16 that covers n: a
        // lane past n re-reads element n - 1, and rows of such loads -- many requests for one
        // address -- cost ~1.5 us at config4 when U was 16 for n = 912.  The host keeps 48 grid + m^2
        // <= kSchurOneLevelLoads * 256.
        const int nI = 48 * (int)gridDim.x, nV = Iv ? m * m : 0, n = nI + nV;
        auto batch = [&](auto UC) {
            constexpr int U = decltype(UC)::value;
            double v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                int t = u * kSchurThreads + tid;
                t = t < n ? t : n - 1;
                v[u] = ld_sc1(t < nI ? a.item_out + t : ivsrc + (t - nI));
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int t = u * kSchurThreads + tid;
                if (t < nI) itm[t] = v[u];
                else if (t < n) Iv[t - nI] = v[u];
            }
        };
        static_assert(kSchurOneLevelLoads == 16, "k_schur one-level batch sizes");
        if (n <= 4 * kSchurThreads) batch(std::integral_constant<int, 4>{});
        else if (n <= 8 * kSchurThreads) batch(std::integral_constant<int, 8>{});
        else batch(std::integral_constant<int, 16>{});
    }
    if (tid <= a.nblk) sbi[tid] = bi;
    if (tid == 0) iv_ok = ivok;
    __syncthreads();
    STAMPP(a.stamps, kSchurStampStride, 8);   // the batch landed in LDS
    schur_finish(a, (int)gridDim.x, iter, cn0, cn1, err_now, Iv && iv_ok,
                 a.stamps ? a.stamps + kSchurStampStride * (size_t)blockIdx.x : nullptr);
}
// The final sums of the one-level hand-off and the solve, from LDS: every partial (48 per item or norm
// chunk, nparts of them) in itm, the block ranges in sbi, the inverse (iv) after S and r -- k_schur's
// last arriver (schur_one_level) and k_group's folded final workgroup (fold_final) both land them there
// srow: this workgroup's MCC_DIAG stamp row (k_schur's by grid index, the folded final's after the items)
__device__ __forceinline__ void schur_finish(const SchurArgs& a, int nparts, int iter, double cn0, double cn1,
                                             int err_now, bool iv, long long* srow) {
    State* st = a.state;
    const int tid = threadIdx.x;
    const int m = a.m, nb = m / 6, ntri = m * (m + 1) / 2;
    extern __shared__ __attribute__((aligned(16))) double sm[];
    double* S = sm;          // m*m
    double* r = sm + m * m;  // m
    __shared__ double norms[2];
    const bool lds = a.fuse_solve && a.peer.nranks == 0;   // single GPU: solve from the sums directly
    double* Iv = iv ? sm + m * m + m : nullptr;
    const double* itm = sm + schur_items_offset(m, a.fuse_solve, a.ssinv != nullptr);   // [nparts][48]
    const int* sbi = reinterpret_cast<const int*>(itm + 48 * (size_t)nparts);          // [nblk + 1]
    // the sums first, every global store after them: a loop entered with a store in flight gets
    // an s_waitcnt vmcnt(0) at its head (the compiler's pre-loop flush), which waits for the store's
    // completion -- 1.5 us at config4 when the packed stores sat between the sums' loops
    constexpr int EU = (15 * 48 + kSchurThreads - 1) / kSchurThreads;   // entries per thread (m <= 30)
    const int nent = a.nblk * 48;
    double ev[EU];
    const bool sl = tid < kSchurThreads;   // (the folded final workgroup has k_group's 256 or 512 threads)
#pragma unroll
    for (int u = 0; u < EU; ++u) {
        const int t = tid + u * kSchurThreads;
        double v = 0.0;
        if (sl && t < nent) {
            const int blk = t / 48, e = t % 48;
            const int k0 = sbi[blk], nk = sbi[blk + 1] - k0;
            // item order (level 1's sums); the first 8 items' words read in one go (a loop with a
            // runtime bound waited for each LDS read in turn: ~1.8 us from the batch to the placed sums)
            double w[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) w[q] = itm[48 * (k0 + (q < nk ? q : 0)) + e];
#pragma unroll
            for (int q = 0; q < 8; ++q)
                if (q < nk) v += w[q];
            for (int q = 8; q < nk; ++q) v += itm[48 * (k0 + q) + e];
        }
        ev[u] = v;
    }
    double nrm = 0.0;
    if (tid < 2) {
        const int w = tid;   // 0: normG2, 1: normX2 of the last update
        const int nc = nparts - a.n_items;
        double cw[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) cw[q] = itm[48 * (a.n_items + (q < nc ? q : 0)) + w];
#pragma unroll
        for (int q = 0; q < 8; ++q)
            if (q < nc) nrm += cw[q];   // chunk order
        for (int k = a.n_items + 8; k < nparts; ++k) nrm += itm[48 * k + w];
        if (a.rank == 0) nrm += w ? cn1 : cn0;
        if (iter <= 0) nrm = 0.0;
        nrm = photo_flag_norm(err_now, w, nrm);
        norms[w] = nrm;
    }
#pragma unroll
    for (int u = 0; u < EU; ++u) {
        const int t = tid + u * kSchurThreads;
        if (!sl || t >= nent) continue;
        const int blk = t / 48, e = t % 48;
        int b1 = 0;   // the block's row: the last b with first_block(b) <= blk (nb <= 5)
#pragma unroll
        for (int b = 1; b < 5; ++b)
            if (b < nb && b * nb - b * (b - 1) / 2 <= blk) b1 = b;
        const int b2 = b1 + (blk - (b1 * nb - b1 * (b1 - 1) / 2));
        if (e >= 36 && b1 != b2) continue;   // off-diagonal blocks: 36 entries, no r / JTE
        const double v = ev[u];
        if (e < 36) {
            const int ii = e / 6, jj = e % 6, i = 6 * b1 + ii, j = 6 * b2 + jj;
            if (b1 != b2 || ii <= jj) {
                a.packed[packed_index(i, j, m)] = v;
                if (lds) {
                    S[i * m + j] = v;
                    S[j * m + i] = v;
                }
            }
        } else {
            const int w = (e - 36) / 6, i = 6 * b1 + (e - 36) % 6;
            a.packed[ntri + w * m + i] = v;   // r (w = 0), JTE of the global block (w = 1)
            if (lds && w == 0) r[i] = v;
        }
    }
    if (tid < 2) a.packed[ntri + 2 * m + tid] = nrm;
    SSTAMP(srow, 9, 0);   // sums placed (thread 0)
    if (!a.fuse_solve) return;
    __syncthreads();   // the packed system and the norms (this workgroup's global stores and LDS)
    if (a.peer.nranks > 0) {
        // multi-GPU: the rank-ordered sum of every rank's system, then this rank solves it
        if (!peer_exchange(a.peer, st, a.packed)) return;
        for (int t = tid; t < ntri + m; t += blockDim.x) {
            const double v = a.packed[t];
            if (t < ntri) {
                int i, j;
                packed_ij(t, m, i, j);
                S[i * m + j] = v;
                S[j * m + i] = v;
            } else {
                r[t - ntri] = v;
            }
        }
        if (tid < 2) norms[tid] = a.packed[ntri + 2 * m + tid];
        __syncthreads();
    }
    SSTAMP(srow, 3, 0);
    SolveCtx sc = a.solve;
    sc.stamps = srow;   // slots 4..6 of this row
    solve_global<false>(sc, S, r, norms[0], norms[1], nullptr, Iv);
    SSTAMP(srow, 7, 0);
}
#ifndef MCC_SCHUR_LOADS
#define MCC_SCHUR_LOADS 32
#endif
#if MCC_IN(5)
__global__ __launch_bounds__(kSchurThreads) void k_schur(SchurArgs a) {
    State* st = a.state;
    if (st->done) return;
    // the warm solve's copy of this step's [S | r] (m > 30): prev2[iteration & 1] (same cache line as done)
    const int iter_e = st->iter;
    double* prev = a.prev2 ? a.prev2 + (size_t)(iter_e & 1) * a.prev_stride : nullptr;
    // the helper solves this system (WarmCtx::refine): publish it now (sync[0] = iteration + 1), the
    // helper stages prev2's words as the blocks write them (each word its own flag)
    if (a.wpub && a.wpub_early && blockIdx.x == 0 && threadIdx.x == 0) st_sys_u32(a.wpub, (unsigned)iter_e + 1u);
    STAMPP(a.stamps, kSchurStampStride, 0);
    const int item = blockIdx.x;
    const int tid = threadIdx.x;
    __shared__ double part[kSub][48];
    if (item < a.n_items) {
        const int4 it = a.items[item];   // {block, first slot's offset (doubles), slots, slot size 48 | 36 [| single]}
        const int q = tid % 48, sub = tid / 48, sz = it.w & (kItemSingle - 1);
        double s = 0.0;
        if (sub < kSub) {
            // the group sums k_photo wrote at the block's slots: independent coalesced loads,
            // eight in flight per thread (entries >= 36 of an off-diagonal block: none, zeros)
            if (q < sz) {
                // slots sub, sub + kSub, ... summed in that order; MCC_SCHUR_LOADS loads per thread in
                // flight per round (the summation order does not depend on it)
                const double* pp = a.pairprod + (size_t)it.y + q;
                constexpr int U = MCC_SCHUR_LOADS;
                for (int p0 = sub; p0 < it.z; p0 += U * kSub) {
                    double v[U];
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const int p = p0 + u * kSub;
                        v[u] = p < it.z ? pp[(size_t)sz * p] : 0.0;
                    }
#pragma unroll
                    for (int u = 0; u < U; ++u) s += v[u];
                }
            }
            part[sub][q] = s;
        }
        __syncthreads();
        if (tid < 48) {
            double t = part[0][tid];
            for (int c = 1; c < kSub; ++c) t += part[c][tid];
            if ((it.w & kItemSingle) && !a.one_level) schur_block_store(a, it.x, tid, 0.0 + t, prev);   // as level 1 over one item
            else st_sc1(a.item_out + 48 * (size_t)item + tid, t);
        }
    } else {
        // a norm chunk: 256 photos' ||G||^2, ||x||^2 partials, both in one round trip and a fixed
        // butterfly per wave (wave_sum), the four waves in order (round 3's LDS tree took 18 barriers)
        const int c = item - a.n_items;
        const int p = c * 256 + tid, pc = min(p, a.n_photos - 1);
        const double2 gx = *reinterpret_cast<const double2*>(a.photo_norm + 2 * (size_t)pc);
        const double g = wave_sum(p < a.n_photos ? gx.x : 0.0), x = wave_sum(p < a.n_photos ? gx.y : 0.0);
        __shared__ double wred[2][kSchurThreads / 64];
        if ((tid & 63) == 0) {
            wred[0][tid >> 6] = g;
            wred[1][tid >> 6] = x;
        }
        __syncthreads();
        if (tid < 2) {
            double v = 0.0;
#pragma unroll
            for (int w = 0; w < kSchurThreads / 64; ++w) v += wred[tid][w];
            st_sc1(a.item_out + 48 * (size_t)item + tid, v);
        }
    }
    STAMPP(a.stamps, kSchurStampStride, 1);
    if (a.one_level) {
        schur_one_level(a, iter_e);
        return;
    }
    const int m = a.m, nb = m / 6, ntri = m * (m + 1) / 2;
    // ---- level 1 (write-through hand-off, no fences): the last item of a camera-pair block sums
    // the block's items in item order and writes the block's entries of the packed system
    if (item < a.n_items && !(a.items[item].w & kItemSingle)) {
        const int blk = a.items[item].x;
        const int k0 = a.block_items[blk], nk = a.block_items[blk + 1] - k0;
        if (!arrive_last_sc1(a.cnt_blk + blk, nk)) return;
        if (tid < 48) {
            // unconditional loads (item_out is padded by kMaxItemsPerBlock zeroed items), masked adds
            double pv[kMaxItemsPerBlock];
#pragma unroll
            for (int q = 0; q < kMaxItemsPerBlock; ++q) pv[q] = ld_sc1(a.item_out + 48 * (size_t)(k0 + q) + tid);
            double v = 0.0;
#pragma unroll
            for (int q = 0; q < kMaxItemsPerBlock; ++q) v += q < nk ? pv[q] : 0.0;
            schur_block_store(a, blk, tid, v, prev);
        }
    }
    STAMPP(a.stamps, kSchurStampStride, 2);
    // ---- level 2: the last of the blocks and norm chunks adds the stop-test norms
    if (!arrive_last_sc1(a.counter, a.nblk + (int)gridDim.x - a.n_items)) return;
    STAMPP(a.stamps, kSchurStampStride, 4);   // (MCC_DIAG: level 2 reached)
    extern __shared__ __attribute__((aligned(16))) double sm[];
    double* S = sm;          // m*m
    double* r = sm + m * m;  // m
    __shared__ double norms[2];
    if (tid < 2) {
        // every load in one memory round trip (the iteration count, the camera norm and the norm
        // chunks' partials are independent), then the sums in chunk order as before
        const int w = tid;   // 0: normG2, 1: normX2 of the last update
        const int iter = st->iter;
        const double cn = w ? st->cam_normX2 : st->cam_normG2;
        const int err_now = photo_error(st);
        constexpr int B = 32;
        double v = 0.0;
        for (int k0 = a.n_items; k0 < (int)gridDim.x; k0 += B) {
            double pv[B];
#pragma unroll
            for (int u = 0; u < B; ++u)
                pv[u] = k0 + u < (int)gridDim.x ? ld_sc1(a.item_out + 48 * (size_t)(k0 + u) + w) : 0.0;
#pragma unroll
            for (int u = 0; u < B; ++u)
                if (k0 + u < (int)gridDim.x) v += pv[u];
        }
        if (a.rank == 0) v += cn;
        if (iter <= 0) v = 0.0;
        v = photo_flag_norm(err_now, w, v);
        norms[w] = v;
        a.packed[ntri + 2 * m + w] = v;
    } else if (tid == 64 && a.wpub && !a.wpub_early) {
        // (without the polled staging: publish once prev2 is complete -- the blocks' sc1 stores drained
        // before their tickets -- as round 5 did; the helper's first pass then finds every word current)
        st_sys_u32(a.wpub, (unsigned)iter_e + 1u);
    }
    if (!a.fuse_solve) return;
    if (a.peer.nranks > 0) {
        // multi-GPU, m <= 30: the rank-ordered sum of every rank's system right here (one launch
        // fewer than k_peer_push + k_solve), then this rank solves it like the fused step does
        __syncthreads();   // the norms above
        if (!peer_exchange(a.peer, st, a.packed)) return;
        if (tid < 2) norms[tid] = a.packed[ntri + 2 * m + tid];
    }
    STAMPP(a.stamps, kSchurStampStride, 3);
    for (int t = tid; t < ntri + m; t += blockDim.x) {
        const double v = ld_sc1(a.packed + t);
        if (t < ntri) {
            int i, j;
            packed_ij(t, m, i, j);
            S[i * m + j] = v;
            S[j * m + i] = v;
        } else {
            r[t - ntri] = v;
        }
    }
    __syncthreads();
    SolveCtx sc = a.solve;
    sc.stamps = a.stamps ? a.stamps + kSchurStampStride * (size_t)blockIdx.x : nullptr;   // slots 4..6 of this row
    solve_global<false>(sc, S, r, norms[0], norms[1]);
    STAMPP(a.stamps, kSchurStampStride, 7);
}
#endif  // MCC_IN(5)

// ---------------------------------------------------------------- k_solve (multi-GPU: after the all-reduce)
#if MCC_IN(5)
__global__ __launch_bounds__(kSolveThreads) void k_solve(SolveArgs a) {
    if (a.ctx.state->done) {
        warm_stop(a.warm);
        return;
    }
    const int m = a.ctx.m, tid = threadIdx.x, ntri = m * (m + 1) / 2;
    extern __shared__ __attribute__((aligned(16))) double sm[];
    double* S = sm;
    double* r = sm + m * m;
    if (a.peer.nranks > 0 && !peer_exchange(a.peer, a.ctx.state, a.packed, !a.pushed)) {
        warm_stop(a.warm);
        return;
    }
    if (m > 30) {   // the blocked elimination reads the packed system directly (LDS: x, A, pivot inverse)
        solve_global<true>(a.ctx, a.packed, sm, a.packed[ntri + 2 * m], a.packed[ntri + 2 * m + 1], &a.warm);
        return;
    }
    for (int t = tid; t < ntri; t += blockDim.x) {
        int i = 0, rem = t;
        while (rem >= m - i) { rem -= m - i; ++i; }
        const int j = i + rem;
        const double v = a.packed[t];
        S[i * m + j] = v;
        S[j * m + i] = v;
    }
    for (int t = tid; t < m; t += blockDim.x) r[t] = a.packed[ntri + t];
    __syncthreads();
    solve_global<false>(a.ctx, S, r, a.packed[ntri + 2 * m], a.packed[ntri + 2 * m + 1]);
}
#endif  // MCC_IN(5)

// This rank's packed system -> every peer's inbox from many workgroups (the m > 30 split step, in
// front of k_solve, which then only receives): 2 Lc LL words per peer -- 68 KB at m = 90, ~480 KB
// per rank at 8 ranks -- are too many 8-B system-scope stores for one workgroup's store issue.
// The epoch is read here and advanced only by k_solve's exchange after this kernel has ended.
#if MCC_IN(0)
__global__ __launch_bounds__(256) void k_peer_push(PeerCtx pc, const State* st, const double* vals) {
    if (st->done) return;
    const unsigned ep = st->epoch + 1u;
    for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < pc.Lc; t += gridDim.x * blockDim.x)
        peer_send(pc, ep, t, vals[t]);
}
#endif  // MCC_IN(0)

// ---------------------------------------------------------------- mcc_debug_solve
// The m > 30 dense solve alone (k_solve's elimination on a packed SPD system [S upper | r]):
// x = S^-1 r, the error bits, and per-phase stamps.  Test and measurement only.
#if MCC_IN(5)
__global__ __launch_bounds__(1024) void k_debug_solve(const double* packed, double* xout, int m, int* err,
                                                       long long* gst) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    const int M = 16 * ((m + 15) / 16);
    gj_blocked(packed, sm, sm + M, sm + M + M * (M + 1), m, err, gst);
    __syncthreads();
    GJB_STAMP(63);
    for (int t = threadIdx.x; t < m; t += blockDim.x) xout[t] = sm[t];
}
#endif  // MCC_IN(5)

// ---------------------------------------------------------------- peer transport: handshake, max
// k_peer_handshake: round 1 sends a (rank, index) pattern over the whole inbox width and checks
// every peer's; round 2 sends each rank's verdict, so all ranks reach the same one (out[0] = 1 only
// if every rank saw every peer's pattern intact).  out = {all_ok, mismatches, round-1 timeout,
// round-2 timeout}.  One workgroup.
__device__ __forceinline__ double peer_pattern(int rank, int t) {
    return (double)(rank + 1) * 1.0e6 + (double)t * 0.123456789 + 1.0 / 3.0;
}
#if MCC_IN(0)
__global__ __launch_bounds__(256) void k_peer_handshake(PeerCtx pc, State* st, double* out) {
    __shared__ unsigned ep_s;
    __shared__ int bad_s, to_s;
    const int tid = threadIdx.x;
    if (tid == 0) {
        ep_s = st->epoch + 1u;
        bad_s = 0;
        to_s = 0;
    }
    __syncthreads();
    const unsigned ep = ep_s;
    for (int t = tid; t < pc.Lc; t += blockDim.x) peer_send(pc, ep, t, peer_pattern(pc.rank, t));
    long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    bool to = false;
    int bad = 0;
    for (int q = 0; q < pc.nranks; ++q) {
        if (q == pc.rank) continue;
        for (int t = tid; t < pc.Lc; t += blockDim.x) {
            const double v = peer_recv(pc, ep, q, t, t0, to);
            if (!to && v != peer_pattern(q, t)) ++bad;
        }
    }
    if (bad) atomicAdd(&bad_s, bad);
    if (to) to_s = 1;
    __syncthreads();
    if (tid == 0) {
        const unsigned ep2 = ep + 1u;
        const double ok = (bad_s == 0 && to_s == 0) ? 1.0 : 0.0;
        peer_send(pc, ep2, 0, ok);
        bool to2 = false;
        double all = ok;
        t0 = (long long)__builtin_amdgcn_s_memrealtime();
        for (int q = 0; q < pc.nranks; ++q)
            if (q != pc.rank) all = fmin(all, peer_recv(pc, ep2, q, 0, t0, to2));
        out[0] = to2 ? 0.0 : all;
        out[1] = (double)bad_s;
        out[2] = (double)to_s;
        out[3] = to2 ? 1.0 : 0.0;
        st->epoch = ep2;
    }
}
#endif  // MCC_IN(0)

// k_peer_max: v[0] <- max over ranks (the bench's max-over-ranks timing and the barrier when no
// RCCL communicator exists, e.g. several ranks on one device).  One thread.
#if MCC_IN(0)
__global__ void k_peer_max(PeerCtx pc, State* st, double* v) {
    if (threadIdx.x != 0) return;
    const unsigned ep = st->epoch + 1u;
    peer_send(pc, ep, 0, v[0]);
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    bool to = false;
    double mx = v[0];
    for (int q = 0; q < pc.nranks; ++q)
        if (q != pc.rank) mx = fmax(mx, peer_recv(pc, ep, q, 0, t0, to));
    v[0] = mx;
    st->epoch = ep;
    if (to) st->error |= 4;
}
#endif  // MCC_IN(0)

// ---------------------------------------------------------------- k_backsub
// one thread per photo: dp = L^-T (z - sum_e Y_e^T dg_e); with do_update the float32 update
// (flush of a pending update), otherwise only deltaX.
#if MCC_IN(0)
__global__ __launch_bounds__(256) void k_backsub(BacksubArgs a) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= a.n_photos) return;
    double t[6];
    if (a.W) photo_delta_w(a.W, a.m, a.zp, a.dg, p, t);
    else photo_delta(a.photo_ptr, a.gblock, a.Y, a.zp, a.dg, p, t);
    const int col = a.m + 6 * p;
    const double alpha = a.state->alpha;
    double g2 = 0.0, x2 = 0.0;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        a.delta[col + k] = t[k];
        if (a.do_update) {
            const float G = (float)(alpha * t[k]);
            const float xn = a.x[col + k] + G;
            a.x[col + k] = xn;
            g2 += (double)G * (double)G;
            x2 += (double)xn * (double)xn;
        }
    }
    if (a.do_update) {
        a.photo_norm[2 * p] = g2;
        a.photo_norm[2 * p + 1] = x2;
    }
}
#endif  // MCC_IN(0)

// ---------------------------------------------------------------- k_project_error
// computeProjectError (src/mymulticalib.cpp:820-939, src/multicalib.cpp:895-1006,
// src/doubleSide.cpp:640-769): float32 Rodrigues + float32 gemm, Rodrigues back, float
// projection, ferror = sqrtf(ex*ex + ey*ey), per-edge sequential float sum.  One wave per edge.
__device__ __forceinline__ void rod_f32(const float* r, float* Rf) {
    double rd[3] = {r[0], r[1], r[2]};
    Rot o;
    rodrigues_v2m(rd, o);
#pragma unroll
    for (int k = 0; k < 9; ++k) Rf[k] = (float)o.R[k];
}

template <int MODEL, bool RATIONAL, int PRISM>
__global__ __launch_bounds__(64) void k_project_error(ErrArgs a) {
#pragma clang fp contract(off)
    const int e = blockIdx.x;   // photo-major edge index
    const int lane = threadIdx.x;
    const int4 info = a.edge_info[e];
    const int cam = info.x, side = info.y, off = info.z, n = info.w;
    const int photo = a.edge_photo[e];
    __shared__ double Rs[9], Ts[3];
    __shared__ float ferr[1024];
    if (lane == 0) {
        const float* xp = a.x + a.m + 6 * photo;
        float Rp[9], Rt[9], Tt[3];
        rod_f32(xp, Rp);
        if (MODEL == MCC_MODEL_DOUBLESIDE) {
            float P4[16], C4[16], T4[16];
            for (int i = 0; i < 16; ++i) { P4[i] = 0.f; C4[i] = a.cam_pose[16 * cam + i]; }
            for (int i = 0; i < 3; ++i) {
                for (int j = 0; j < 3; ++j) P4[i * 4 + j] = Rp[i * 3 + j];
                P4[i * 4 + 3] = xp[3 + i];
            }
            P4[15] = 1.f;
            auto mm4 = [](const float* A, const float* B, float* Cc) {
                for (int i = 0; i < 4; ++i)
                    for (int j = 0; j < 4; ++j) {
                        float t = A[i * 4] * B[j];
                        t = t + A[i * 4 + 1] * B[4 + j];
                        t = t + A[i * 4 + 2] * B[8 + j];
                        t = t + A[i * 4 + 3] * B[12 + j];
                        Cc[i * 4 + j] = (float)((double)t * 1.0);
                    }
            };
            mm4(C4, P4, T4);
            if (side == MCC_BACK) {
                float D4[16], Rd[9], T5[16];
                rod_f32(a.x, Rd);
                for (int i = 0; i < 16; ++i) D4[i] = 0.f;
                for (int i = 0; i < 3; ++i) {
                    for (int j = 0; j < 3; ++j) D4[i * 4 + j] = Rd[i * 3 + j];
                    D4[i * 4 + 3] = a.x[3 + i];
                }
                D4[15] = 1.f;
                mm4(T4, D4, T5);
                for (int i = 0; i < 16; ++i) T4[i] = T5[i];
            }
            for (int i = 0; i < 3; ++i) {
                for (int j = 0; j < 3; ++j) Rt[i * 3 + j] = T4[i * 4 + j];
                Tt[i] = T4[i * 4 + 3];
            }
        } else if (cam == 0) {
            for (int k = 0; k < 9; ++k) Rt[k] = Rp[k];
            for (int k = 0; k < 3; ++k) Tt[k] = xp[3 + k];
        } else {
            const float* xc = a.x + 6 * (cam - 1);
            float Rc[9];
            rod_f32(xc, Rc);
            for (int i = 0; i < 3; ++i) {
                for (int j = 0; j < 3; ++j) {
                    float t = Rc[i * 3] * Rp[j];
                    t = t + Rc[i * 3 + 1] * Rp[3 + j];
                    t = t + Rc[i * 3 + 2] * Rp[6 + j];
                    Rt[i * 3 + j] = (float)((double)t * 1.0);
                }
                float t = Rc[i * 3] * xp[3];
                t = t + Rc[i * 3 + 1] * xp[4];
                t = t + Rc[i * 3 + 2] * xp[5];
                Tt[i] = (float)((double)t * 1.0 + (double)xc[3 + i] * 1.0);
            }
        }
        double Rd[9], rv[3], th, s, c;
        for (int k = 0; k < 9; ++k) Rd[k] = Rt[k];
        polar3(Rd);
        rodrigues_m2v(Rd, rv, th, s, c);
        double rf[3] = {(double)(float)rv[0], (double)(float)rv[1], (double)(float)rv[2]};
        Rot rr;
        rodrigues_v2m(rf, rr);
        for (int k = 0; k < 9; ++k) Rs[k] = rr.R[k];
        for (int k = 0; k < 3; ++k) Ts[k] = Tt[k];
    }
    __syncthreads();
    double R[9], T[3], kd[12];
    for (int q = 0; q < 9; ++q) R[q] = Rs[q];
    for (int q = 0; q < 3; ++q) T[q] = Ts[q];
    const int nd = a.nd;
    for (int q = 0; q < 12; ++q) kd[q] = q < nd ? (double)a.D[nd * cam + q] : 0.0;
    const float* Kc = a.K + 9 * cam;
    const double fx = Kc[0], fy = Kc[4], cx = Kc[2], cy = Kc[5], sk = Kc[1];
    for (int i = lane; i < n; i += 64) {
        const int c = off + i;
        double Yr[3], D[6];
        float u, v;
        if (MODEL == MCC_MODEL_OMNI)
            omni_corner(R, T, kd, fx, fy, cx, cy, sk, (double)a.xi[cam], a.obj_x[c], a.obj_y[c], a.obj_z[c], Yr, u, v, D);
        else
            pinhole_corner<RATIONAL, PRISM>(R, T, kd, fx, fy, cx, cy, a.obj_x[c], a.obj_y[c], a.obj_z[c], Yr, u, v, D,
                                            PRISM == 2 ? a.tilt + 9 * cam : nullptr);
        const float ex = a.img_u[c] - u, ey = a.img_v[c] - v;
        float s2 = ex * ex;
        s2 = s2 + ey * ey;
        ferr[i] = sqrtf(s2);
        if (a.corner_err) a.corner_err[c] = ferr[i];
    }
    __syncthreads();
    if (lane == 0) {
        float s = 0.f;
        for (int i = 0; i < n; ++i) s += ferr[i];
        a.edge_sum[e] = s;
    }
}

#include "mcc_group.hpp"

}  // namespace mcc

// ---------------------------------------------------------------- launch wrappers
using namespace mcc;

#if MCC_IN(1)
template <int MODEL>
static hipError_t launch_lin_model(const LinArgs& a, int n_photos, size_t shmem, hipStream_t s, bool rational, int prism) {
    const dim3 grid(n_photos + (a.ssinv ? 1 : 0));   // + the m <= 30 warm solve's spare workgroup
    if (prism == 2) return hipErrorInvalidValue;   // the tilted sensor takes the split step (mcc_create)
    if (rational && prism) hipLaunchKernelGGL((k_linearize<MODEL, true, true>), grid, dim3(256), shmem, s, a);
    else if (rational) hipLaunchKernelGGL((k_linearize<MODEL, true, false>), grid, dim3(256), shmem, s, a);
    else if (prism) hipLaunchKernelGGL((k_linearize<MODEL, false, true>), grid, dim3(256), shmem, s, a);
    else hipLaunchKernelGGL((k_linearize<MODEL, false, false>), grid, dim3(256), shmem, s, a);
    return hipGetLastError();
}
hipError_t mcc_launch_linearize(const LinArgs& a, int model, int n_photos, int max_epp, bool rational, int prism, hipStream_t s) {
    const size_t shmem = mcc_lin_shmem(max_epp, a.n_cams, a.global_dim, a.max_cpp);
    switch (model) {
        case MCC_MODEL_OMNI: return launch_lin_model<MCC_MODEL_OMNI>(a, n_photos, shmem, s, false, false);
        case MCC_MODEL_DOUBLESIDE: return launch_lin_model<MCC_MODEL_DOUBLESIDE>(a, n_photos, shmem, s, rational, prism);
        default: return launch_lin_model<MCC_MODEL_PINHOLE>(a, n_photos, shmem, s, rational, prism);
    }
}
hipError_t mcc_attrs_linearize(size_t shmem) {
    hipError_t err = hipSuccess;
#define SETA(M, R, P) hipFuncSetAttribute((const void*)&k_linearize<M, R, P>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shmem)
    for (hipError_t e : {SETA(0, false, false), SETA(0, true, false), SETA(0, false, true), SETA(0, true, true),
                         SETA(1, false, false), SETA(2, false, false), SETA(2, true, false), SETA(2, false, true),
                         SETA(2, true, true)})
        if (e != hipSuccess) err = e;
#undef SETA
    return err;
}
#endif  // MCC_IN(1)

#if MCC_IN(4)
// split step: lanes per edge of k_edge (88-corner edges: 6 passes at 92% lane use, the 27-value
// butterfly over 16 lanes is a quarter of a wave's)
#ifndef MCC_EDGE_LANES
#define MCC_EDGE_LANES 16
#endif
constexpr int kEdgeLanes = MCC_EDGE_LANES;   // lanes per edge in k_edge (16 or 8)
template <int MODEL, bool RATIONAL, int PRISM>
static void launch_edge(const LinArgs& a, hipStream_t s) {
    constexpr int per = 64 / kEdgeLanes;
    hipLaunchKernelGGL((k_edge<MODEL, RATIONAL, PRISM, kEdgeLanes>), dim3((a.n_edges + per - 1) / per), dim3(64), 0, s, a);
}
hipError_t mcc_launch_split(const LinArgs& a, int model, bool rational, int prism, size_t photo_shmem,
                            hipStream_t s) {
    if (a.n_photos <= 0 || a.n_edges <= 0) return hipSuccess;
    const dim3 gp((a.n_photos + 64 / kPrepGroup - 1) / (64 / kPrepGroup));
    const bool p4 = a.prep_lanes == 4;
    const bool back = model == MCC_MODEL_DOUBLESIDE || (model == MCC_MODEL_PINHOLE && a.has_back);
    const size_t p4shm = prep_lds_bytes(a.n_cams, back);
    const dim3 g4(a.n_prep);
    if (model == MCC_MODEL_OMNI) {
        if (p4) hipLaunchKernelGGL((k_prep4<MCC_MODEL_OMNI, false>), g4, dim3(64), p4shm, s, a);
        else hipLaunchKernelGGL((k_prep<MCC_MODEL_OMNI, false>), gp, dim3(64), 0, s, a);
        launch_edge<MCC_MODEL_OMNI, false, false>(a, s);
    } else if (model == MCC_MODEL_DOUBLESIDE) {
        if (p4) hipLaunchKernelGGL((k_prep4<MCC_MODEL_DOUBLESIDE, true>), g4, dim3(64), p4shm, s, a);
        else hipLaunchKernelGGL((k_prep<MCC_MODEL_DOUBLESIDE, true>), gp, dim3(64), 0, s, a);
        if (prism == 2) launch_edge<MCC_MODEL_DOUBLESIDE, true, 2>(a, s);
        else if (rational && prism) launch_edge<MCC_MODEL_DOUBLESIDE, true, true>(a, s);
        else if (rational) launch_edge<MCC_MODEL_DOUBLESIDE, true, false>(a, s);
        else if (prism) launch_edge<MCC_MODEL_DOUBLESIDE, false, true>(a, s);
        else launch_edge<MCC_MODEL_DOUBLESIDE, false, false>(a, s);
    } else {
        if (p4 && a.has_back) hipLaunchKernelGGL((k_prep4<MCC_MODEL_PINHOLE, true>), g4, dim3(64), p4shm, s, a);
        else if (p4) hipLaunchKernelGGL((k_prep4<MCC_MODEL_PINHOLE, false>), g4, dim3(64), p4shm, s, a);
        else if (a.has_back) hipLaunchKernelGGL((k_prep<MCC_MODEL_PINHOLE, true>), gp, dim3(64), 0, s, a);
        else hipLaunchKernelGGL((k_prep<MCC_MODEL_PINHOLE, false>), gp, dim3(64), 0, s, a);
        if (prism == 2) launch_edge<MCC_MODEL_PINHOLE, true, 2>(a, s);
        else if (rational && prism) launch_edge<MCC_MODEL_PINHOLE, true, true>(a, s);
        else if (rational) launch_edge<MCC_MODEL_PINHOLE, true, false>(a, s);
        else if (prism) launch_edge<MCC_MODEL_PINHOLE, false, true>(a, s);
        else launch_edge<MCC_MODEL_PINHOLE, false, false>(a, s);
    }
    hipLaunchKernelGGL(k_photo, dim3(a.n_pgroups), dim3(256), photo_shmem, s, a);
    return hipGetLastError();
}
hipError_t mcc_attrs_photo(size_t shmem) {
    return hipFuncSetAttribute((const void*)&k_photo, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shmem);
}
#endif  // MCC_IN(4)

#if MCC_IN(0)

size_t mcc_lin_shmem(int max_edges_per_photo, int n_cams, int m, int max_cpp) {
    const size_t lin = (size_t)max_edges_per_photo * sizeof(EdgeLds) + sizeof(PhotoLds) +
                       (kCamStride + kIntrStride) * sizeof(double) * (size_t)n_cams +
                       ((5 * sizeof(float) * (size_t)max_cpp + 15) & ~(size_t)15);
    // the final arriver's S, r and (m <= 30, the fused step) the warm solve's inverse; the spare
    // workgroup's [S | I]
    return std::max(lin, (size_t)((m <= 30 ? 2 : 1) * m * m + m) * sizeof(double));
}

size_t mcc_solve_shmem(int m) {
    const size_t M = 16 * (size_t)((m + 15) / 16);
    const size_t blocked = M + M * (M + 1) + 2 * 16 * kBlkLd;   // gj_blocked (m > 30, k_solve)
    const size_t warm = M <= kWarmN ? kWarmN + warm_shmem_doubles(m) : 0;   // warm_finish
    const size_t helper = M <= kWarmN ? helper_shmem_doubles(m, true) : 0;   // k_sinv_helper (refine)
    return std::max((size_t)(m * m + m), m > 30 ? std::max(std::max(blocked, warm), helper) : 0) * sizeof(double);
}

#endif  // MCC_IN(0)

#if MCC_IN(2) || MCC_IN(3)
template <int MODEL, bool RATIONAL, int PRISM, bool BACK, int L>
static hipError_t launch_group_t(const LinArgs& a, size_t shmem, hipStream_t s) {
    // + the spare workgroup of the m <= 30 warm solve (small_inverse)
    // (+ the folded reduction's item, norm-chunk and final workgroups)
    const dim3 grid(a.n_pgroups + (a.ssinv ? 1 : 0) + (a.fold && !a.fold_dyn ? a.fold_parts + 1 : 0));
    if (a.fold_first) {   // (test layout, omnidir only: mcc_create)
        if (MODEL != MCC_MODEL_OMNI) return hipErrorInvalidValue;
        hipLaunchKernelGGL((k_group<MCC_MODEL_OMNI, false, false, false, L, true>), grid, dim3(kGroupRound * L), shmem, s, a);
        return hipGetLastError();
    }
    hipLaunchKernelGGL((k_group<MODEL, RATIONAL, PRISM, BACK, L>), grid, dim3(kGroupRound * L), shmem, s, a);
    return hipGetLastError();
}
template <int L>
static hipError_t launch_group_l(const LinArgs& a, int model, bool rational, int prism, size_t shmem, hipStream_t s) {
    if (model == MCC_MODEL_OMNI) return launch_group_t<MCC_MODEL_OMNI, false, false, false, L>(a, shmem, s);
    if (model == MCC_MODEL_DOUBLESIDE) {
        if (prism == 2) return launch_group_t<MCC_MODEL_DOUBLESIDE, true, 2, true, L>(a, shmem, s);
        if (rational && prism) return launch_group_t<MCC_MODEL_DOUBLESIDE, true, true, true, L>(a, shmem, s);
        if (rational) return launch_group_t<MCC_MODEL_DOUBLESIDE, true, false, true, L>(a, shmem, s);
        if (prism) return launch_group_t<MCC_MODEL_DOUBLESIDE, false, true, true, L>(a, shmem, s);
        return launch_group_t<MCC_MODEL_DOUBLESIDE, false, false, true, L>(a, shmem, s);
    }
    if (a.has_back) {
        if (prism == 2) return launch_group_t<MCC_MODEL_PINHOLE, true, 2, true, L>(a, shmem, s);
        if (rational && prism) return launch_group_t<MCC_MODEL_PINHOLE, true, true, true, L>(a, shmem, s);
        if (rational) return launch_group_t<MCC_MODEL_PINHOLE, true, false, true, L>(a, shmem, s);
        if (prism) return launch_group_t<MCC_MODEL_PINHOLE, false, true, true, L>(a, shmem, s);
        return launch_group_t<MCC_MODEL_PINHOLE, false, false, true, L>(a, shmem, s);
    }
    if (prism == 2) return launch_group_t<MCC_MODEL_PINHOLE, true, 2, false, L>(a, shmem, s);
    if (rational && prism) return launch_group_t<MCC_MODEL_PINHOLE, true, true, false, L>(a, shmem, s);
    if (rational) return launch_group_t<MCC_MODEL_PINHOLE, true, false, false, L>(a, shmem, s);
    if (prism) return launch_group_t<MCC_MODEL_PINHOLE, false, true, false, L>(a, shmem, s);
    return launch_group_t<MCC_MODEL_PINHOLE, false, false, false, L>(a, shmem, s);
}
template <int L>
static hipError_t set_group_attrs(size_t group_shmem) {
    hipError_t err = hipSuccess;
#define SETG(M, R, P, B) hipFuncSetAttribute((const void*)&k_group<M, R, P, B, L>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)group_shmem)
    for (hipError_t e : {SETG(1, false, false, false), SETG(2, true, true, true), SETG(2, true, false, true),
                         SETG(2, false, true, true), SETG(2, false, false, true), SETG(0, true, true, true),
                         SETG(0, true, false, true), SETG(0, false, true, true), SETG(0, false, false, true),
                         SETG(0, true, true, false), SETG(0, true, false, false), SETG(0, false, true, false),
                         SETG(0, false, false, false), SETG(2, true, 2, true), SETG(0, true, 2, true),
                         SETG(0, true, 2, false),
                         hipFuncSetAttribute((const void*)&k_group<1, false, false, false, L, true>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)group_shmem)})
        if (e != hipSuccess) err = e;
#undef SETG
    return err;
}
#endif  // MCC_IN(2) || MCC_IN(3)
#if MCC_IN(3)
hipError_t mcc_launch_group32(const LinArgs& a, int model, bool rational, int prism, size_t shmem, hipStream_t s) {
    return launch_group_l<32>(a, model, rational, prism, shmem, s);
}
hipError_t mcc_attrs_group32(size_t shmem) { return set_group_attrs<32>(shmem); }
#endif
#if MCC_IN(2)
hipError_t mcc_launch_group32(const LinArgs& a, int model, bool rational, int prism, size_t shmem, hipStream_t s);
hipError_t mcc_launch_group(const LinArgs& a, int model, bool rational, int prism, int lanes, size_t shmem,
                            hipStream_t s) {
    if (a.n_photos <= 0 || a.n_edges <= 0) return hipSuccess;
    return lanes == 32 ? mcc_launch_group32(a, model, rational, prism, shmem, s)
                       : launch_group_l<16>(a, model, rational, prism, shmem, s);
}
hipError_t mcc_attrs_group16(size_t shmem) { return set_group_attrs<16>(shmem); }
#endif

#if MCC_IN(0)

// The dynamic-LDS limits only ever grow within a process (per device): a graph captured for an
// earlier, larger problem keeps launching with the LDS it was captured with after a smaller problem
// is created.
hipError_t mcc_set_kernel_attrs(int max_epp, int n_cams, int m, int max_cpp, size_t photo_shmem, size_t group_shmem) {
    hipError_t err = hipSuccess;
    static std::mutex mu;
    static std::map<int, std::array<size_t, 4>> high;   // device -> {group, linearize, photo, solve}
    std::lock_guard<std::mutex> lock(mu);
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = -1;
    auto& hw = high[dev];
    size_t shmem = mcc_lin_shmem(max_epp, n_cams, m, max_cpp), ss = mcc_solve_shmem(m);
    group_shmem = hw[0] = std::max(hw[0], group_shmem);
    shmem = hw[1] = std::max(hw[1], shmem);
    photo_shmem = hw[2] = std::max(hw[2], photo_shmem);
    ss = hw[3] = std::max(hw[3], ss);
    if (group_shmem > 64 * 1024) {
        for (hipError_t e : {mcc_attrs_group16(group_shmem), mcc_attrs_group32(group_shmem)})
            if (e != hipSuccess) err = e;
    }
    if (shmem > 64 * 1024) {
        hipError_t e = mcc_attrs_linearize(shmem);
        if (e != hipSuccess) err = e;
    }
    if (photo_shmem > 64 * 1024) {
        hipError_t e = mcc_attrs_photo(photo_shmem);
        if (e != hipSuccess) err = e;
    }
    if (ss > 60 * 1024) {
        hipError_t e = mcc_attrs_solve(ss);
        if (e != hipSuccess) err = e;
    }
    return err;
}
#endif  // MCC_IN(0)

#if MCC_IN(5)
hipError_t mcc_attrs_solve(size_t ss) {
    hipError_t err = hipSuccess;
    for (hipError_t e : {hipFuncSetAttribute((const void*)&k_schur, hipFuncAttributeMaxDynamicSharedMemorySize, (int)ss),
                         hipFuncSetAttribute((const void*)&k_solve, hipFuncAttributeMaxDynamicSharedMemorySize, (int)ss),
                         hipFuncSetAttribute((const void*)&k_sinv_helper<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)ss),
                         hipFuncSetAttribute((const void*)&k_sinv_helper<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)ss)})
        if (e != hipSuccess) err = e;
    return err;
}

hipError_t mcc_launch_schur(const SchurArgs& a, int grid, hipStream_t s) {
    // LDS for the solve only when this launch solves (single GPU, m <= 30): the item workgroups
    // keep their occupancy
    const size_t shm = schur_lds_bytes(a.m, a.fuse_solve, a.ssinv != nullptr, a.one_level, grid, a.nblk);
    hipLaunchKernelGGL(k_schur, dim3(grid), dim3(kSchurThreads), shm, s, a);
    return hipGetLastError();
}
hipError_t mcc_launch_solve(const SolveArgs& a, hipStream_t s) {
    // m > 30: 8 waves, so the block eliminations of a pivot step (up to (nb - 1)^2 16 x 16 MFMA
    // products) are not what waits on the next pivot inverse
    hipLaunchKernelGGL(k_solve, dim3(1), dim3(a.ctx.m > 30 ? kSolveThreads : 256), mcc_solve_shmem(a.ctx.m), s, a);
    return hipGetLastError();
}
hipError_t mcc_launch_debug_solve(const double* packed, double* x, int m, int* err, long long* stamps, hipStream_t s) {
    const size_t shm = mcc_solve_shmem(m);
    hipError_t e = hipFuncSetAttribute((const void*)&k_debug_solve, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_debug_solve, dim3(1), dim3(kSolveThreads), shm, s, packed, x, m, err, stamps);
    return hipGetLastError();
}
hipError_t mcc_launch_sinv_helper(const WarmCtx& w, int m, int n_systems, hipStream_t s) {
    const size_t shm = helper_shmem_doubles(m, w.refine != 0) * sizeof(double);
    if (w.inv_la)
        hipLaunchKernelGGL(k_sinv_helper<true>, dim3(1), dim3(kSolveThreads), shm, s, w, m, n_systems);
    else
        hipLaunchKernelGGL(k_sinv_helper<false>, dim3(1), dim3(kSolveThreads), shm, s, w, m, n_systems);
    return hipGetLastError();
}
#endif  // MCC_IN(5)

#if MCC_IN(0)
hipError_t mcc_launch_peer_push(const PeerCtx& pc, const State* st, const double* vals, hipStream_t s) {
    // ~16 KB of words per workgroup: 8 ranks at m = 90 -> 30 workgroups
    const long long bytes = 16LL * pc.Lc * (pc.nranks - 1);
    const int grid = (int)std::min<long long>(64, std::max<long long>(1, (bytes + 16383) / 16384));
    hipLaunchKernelGGL(k_peer_push, dim3(grid), dim3(256), 0, s, pc, st, vals);
    return hipGetLastError();
}
hipError_t mcc_launch_peer_handshake(const PeerCtx& pc, State* st, double* out, hipStream_t s) {
    hipLaunchKernelGGL(k_peer_handshake, dim3(1), dim3(256), 0, s, pc, st, out);
    return hipGetLastError();
}
hipError_t mcc_launch_peer_max(const PeerCtx& pc, State* st, double* v, hipStream_t s) {
    hipLaunchKernelGGL(k_peer_max, dim3(1), dim3(64), 0, s, pc, st, v);
    return hipGetLastError();
}
// one wave that waits `ticks` of the 100 MHz clock (vector-free, no memory traffic): the timing
// window's head, so the host can enqueue the window before the GPU reaches it
__global__ __launch_bounds__(64) void k_delay(long long ticks) {
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    while ((long long)__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(64);
}
hipError_t mcc_launch_delay(long long ticks, hipStream_t s) {
    hipLaunchKernelGGL(k_delay, dim3(1), dim3(64), 0, s, ticks);
    return hipGetLastError();
}

hipError_t mcc_launch_backsub(const BacksubArgs& a, hipStream_t s) {
    if (a.n_photos > 0) hipLaunchKernelGGL(k_backsub, dim3((a.n_photos + 255) / 256), dim3(256), 0, s, a);
    return hipGetLastError();
}
hipError_t mcc_launch_project_error(const ErrArgs& a, int model, int n_edges, bool rational, int prism, hipStream_t s) {
#define PE(M, R, P) hipLaunchKernelGGL((k_project_error<M, R, P>), dim3(n_edges), dim3(64), 0, s, a)
    if (model == MCC_MODEL_OMNI) PE(1, false, false);
    else if (model == MCC_MODEL_DOUBLESIDE) {
        if (prism == 2) PE(2, true, 2); else if (rational && prism) PE(2, true, true); else if (rational) PE(2, true, false); else if (prism) PE(2, false, true); else PE(2, false, false);
    } else {
        if (prism == 2) PE(0, true, 2); else if (rational && prism) PE(0, true, true); else if (rational) PE(0, true, false); else if (prism) PE(0, false, true); else PE(0, false, false);
    }
#undef PE
    return hipGetLastError();
}
#endif  // MCC_IN(0)
