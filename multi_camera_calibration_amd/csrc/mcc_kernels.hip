// mcc_kernels.hip -- CDNA4 (gfx950) kernels of one Gauss-Newton step of the reference's
// multi-camera extrinsic BA (MultiCameraCalibration::optimizeExtrinsics, src/multicalib.cpp:462-514).
//
// Step dataflow:
//   k_linearize   one workgroup per photo vertex, one wavefront per edge (camera observing it):
//                 edge prologue (compose_motion + fl32 pose, one lane per edge), corner sweep
//                 (lanes over corners, FP64 projection + 2x6 Jacobian strips, float32 residual),
//                 butterfly reduce-scatter of the 27 normal-equation sums, chain rule to the
//                 photo / global blocks, 6x6 photo Cholesky and the Schur factors Y_e = H_gp L^-T.
//   k_schur       camera-pair blocks of S = sum H_gg - sum Y_e Y_e'^T and r, per work item.
//   k_assemble    deterministic sum of the work items + norm partials into the packed buffer
//                 that multi-GPU runs all-reduce over RCCL.
//   k_solve       stop test (src/multicalib.cpp:475-477), Cholesky of S, global-block update.
//   k_backsub     photo back-substitution and float32 update x = fl32(x + fl32(a*delta)).
// No MFMA: the largest dense block is 6x6; the path is FP64-VALU and
// latency bound.  All reductions are fixed-order, so a run is bitwise reproducible.
#include <hip/hip_runtime.h>

#include "mcc_device.hpp"
#include "mcc_internal.h"

namespace mcc {

// ---------------------------------------------------------------- wave reduction
// Reduce-scatter butterfly of NV (<= 32) per-lane doubles across the 64 lanes: 32 shuffles of
// 64-bit values instead of 6*NV.  Afterwards lane l (and l^1) holds the full sum of value
// index idx(l) = 16*b5 + 8*b4 + 4*b3 + 2*b2 + b1.
template <int W>
__device__ __forceinline__ void bfly_step(double* v, int lane) {
    const bool hi = (lane & (2 * W)) != 0;
#pragma unroll
    for (int j = 0; j < W; ++j) {
        double send = hi ? v[j] : v[j + W];
        double keep = hi ? v[j + W] : v[j];
        v[j] = keep + __shfl_xor(send, 2 * W);
    }
}
__device__ __forceinline__ double wave_reduce_scatter32(double* v, int lane) {
    bfly_step<16>(v, lane);
    bfly_step<8>(v, lane);
    bfly_step<4>(v, lane);
    bfly_step<2>(v, lane);
    bfly_step<1>(v, lane);
    return v[0] + __shfl_xor(v[0], 1);
}
__device__ __forceinline__ int bfly_index(int lane) {
    return ((lane >> 5) & 1) * 16 + ((lane >> 4) & 1) * 8 + ((lane >> 3) & 1) * 4 +
           ((lane >> 2) & 1) * 2 + ((lane >> 1) & 1);
}

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

// ---------------------------------------------------------------- edge prologue (one lane)
template <int MODEL>
__device__ void edge_prologue(const LinArgs& a, int photo, int e, EdgeLds& L) {
    const int4 info = a.edge_info[e];
    const int cam = info.x, side = info.y;
    const float* x = a.x;
    const int pc = a.global_dim + 6 * photo;
    double om1[3], T1[3], om2[3], T2[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) { om1[k] = x[pc + k]; T1[k] = x[pc + 3 + k]; }
    if (MODEL == MCC_MODEL_DOUBLESIDE) {
#pragma unroll
        for (int k = 0; k < 3; ++k) { om2[k] = a.cam_rt[6 * cam + k]; T2[k] = a.cam_rt[6 * cam + 3 + k]; }
    } else if (cam == 0) {
#pragma unroll
        for (int k = 0; k < 3; ++k) { om2[k] = 0.0; T2[k] = 0.0; }
    } else {
        const int cc = 6 * (cam - 1);
#pragma unroll
        for (int k = 0; k < 3; ++k) { om2[k] = x[cc + k]; T2[k] = x[cc + 3 + k]; }
    }
    Motion f;
    compose_motion(om1, T1, om2, T2, f);
    double Mp[36], Mg[36];
#pragma unroll
    for (int k = 0; k < 36; ++k) { Mp[k] = 0.0; Mg[k] = 0.0; }
    double om[3], T[3];
    int has_global;
    if (side == MCC_BACK) {
        double dsr[3], dst[3];
        if (MODEL == MCC_MODEL_DOUBLESIDE) {
#pragma unroll
            for (int k = 0; k < 3; ++k) { dsr[k] = x[k]; dst[k] = x[3 + k]; }
        } else {
#pragma unroll
            for (int k = 0; k < 3; ++k) { dsr[k] = a.ds_rt[k]; dst[k] = a.ds_rt[3 + k]; }
        }
        Motion b;   // compose_motion(ds, photofront), src/mymulticalib.cpp:503-506
        compose_motion(dsr, dst, f.om, f.T, b);
#pragma unroll
        for (int k = 0; k < 3; ++k) { om[k] = b.om[k]; T[k] = b.T[k]; }
        // photo: E2 * D1 = [[A2b A1, 0], [B2b A1, R2]]
        double t[9];
        mat3_mul(b.A2, f.A1, t);
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) Mp[i * 6 + j] = t[i * 3 + j];
        mat3_mul(b.B2, f.A1, t);
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) { Mp[(3 + i) * 6 + j] = t[i * 3 + j]; Mp[(3 + i) * 6 + 3 + j] = f.R2[i * 3 + j]; }
        if (MODEL == MCC_MODEL_DOUBLESIDE) {
            // ds block: [[A1b, 0], [0, R_front]]  (src/doubleSide.cpp:398-399)
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) { Mg[i * 6 + j] = b.A1[i * 3 + j]; Mg[(3 + i) * 6 + 3 + j] = f.R[i * 3 + j]; }
            has_global = 1;
        } else {
            // camera block as the reference chains it (src/mymulticalib.cpp:514-517), which
            // omits dTt/dTf * dTf/dRc at :516 (hazard A12): [[A2b A2, 0], [B2b A2, I]]
            mat3_mul(b.A2, f.A2, t);
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) Mg[i * 6 + j] = t[i * 3 + j];
            mat3_mul(b.B2, f.A2, t);
            for (int i = 0; i < 3; ++i) {
                for (int j = 0; j < 3; ++j) Mg[(3 + i) * 6 + j] = t[i * 3 + j];
                Mg[(3 + i) * 6 + 3 + i] = 1.0;
            }
            has_global = cam != 0;
        }
    } else {
#pragma unroll
        for (int k = 0; k < 3; ++k) { om[k] = f.om[k]; T[k] = f.T[k]; }
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) { Mp[i * 6 + j] = f.A1[i * 3 + j]; Mp[(3 + i) * 6 + 3 + j] = f.R2[i * 3 + j]; }
        if (MODEL == MCC_MODEL_DOUBLESIDE) {
            has_global = 0;   // zero double-side jacobian on the front side (doubleSide.cpp:335-336)
        } else {
            for (int i = 0; i < 3; ++i) {
                for (int j = 0; j < 3; ++j) { Mg[i * 6 + j] = f.A2[i * 3 + j]; Mg[(3 + i) * 6 + j] = f.B2[i * 3 + j]; }
                Mg[(3 + i) * 6 + 3 + i] = 1.0;
            }
            has_global = cam != 0;
        }
    }
    // Rvectran1 / Tvectran1 -> float32 (src/mymulticalib.cpp:546-553)
    double rf[3], Jl[9];
#pragma unroll
    for (int k = 0; k < 3; ++k) { rf[k] = (double)(float)om[k]; L.T[k] = (double)(float)T[k]; }
    rodrigues_v2m(rf, L.R);
    so3_jl(rf, Jl);
    // G = blockdiag(Jl, I) * M
    for (int j = 0; j < 6; ++j) {
        for (int i = 0; i < 3; ++i) {
            L.Gp[i * 6 + j] = Jl[i * 3] * Mp[j] + Jl[i * 3 + 1] * Mp[6 + j] + Jl[i * 3 + 2] * Mp[12 + j];
            L.Gg[i * 6 + j] = Jl[i * 3] * Mg[j] + Jl[i * 3 + 1] * Mg[6 + j] + Jl[i * 3 + 2] * Mg[12 + j];
            L.Gp[(3 + i) * 6 + j] = Mp[(3 + i) * 6 + j];
            L.Gg[(3 + i) * 6 + j] = Mg[(3 + i) * 6 + j];
        }
    }
    L.cam = cam;
    L.side = side;
    L.off = info.z;
    L.n = info.w;
    L.has_global = has_global;
    L.edge = e;
}

// ---------------------------------------------------------------- per-corner models
// Pinhole (cvProjectPoints2Internal order).  Returns float32 pixel and D = d(u,v)/dXc (2x3).
template <bool RATIONAL, bool PRISM>
__device__ __forceinline__ void pinhole_corner(const double* R, const double* T, const double* k,
                                               double fx, double fy, double cx, double cy,
                                               double X, double Y, double Z, double* Yr,
                                               float& u, float& v, double* D) {
    double x, y, z, r2, r4, r6, cdist, icdist2;
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
        double a1 = 2 * x * y, a2 = r2 + 2 * x * x, a3 = r2 + 2 * y * y;
        cdist = 1 + k[0] * r2 + k[1] * r4 + k[4] * r6;
        icdist2 = RATIONAL ? 1. / (1 + k[5] * r2 + k[6] * r4 + k[7] * r6) : 1.0;
        double xd = (RATIONAL ? x * cdist * icdist2 : x * cdist) + k[2] * a1 + k[3] * a2;
        double yd = (RATIONAL ? y * cdist * icdist2 : y * cdist) + k[2] * a3 + k[3] * a1;
        if (PRISM) {
            xd = xd + k[8] * r2 + k[9] * r4;
            yd = yd + k[10] * r2 + k[11] * r4;
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
    const double m00 = cc + 2 * x * x * g + 2 * k[2] * y + 6 * k[3] * x + 2 * x * P1;
    const double m01 = xy2g + 2 * k[2] * x + 2 * k[3] * y + 2 * y * P1;
    const double m10 = xy2g + 2 * k[2] * x + 2 * k[3] * y + 2 * x * P2;
    const double m11 = cc + 2 * y * y * g + 6 * k[2] * y + 2 * k[3] * x + 2 * y * P2;
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
        double inrm = 1. / nrm;
        Xs[0] = Xc[0] * inrm;
        Xs[1] = Xc[1] * inrm;
        Xs[2] = Xc[2] * inrm;
        xu0 = Xs[0] / (Xs[2] + xi);
        xu1 = Xs[1] / (Xs[2] + xi);
        r2 = xu0 * xu0 + xu1 * xu1;
        r4 = r2 * r2;
        const double k1 = k[0], k2 = k[1], p1 = k[2], p2 = k[3];
        double xd0 = xu0 * (1 + k1 * r2 + k2 * r4) + 2 * p1 * xu0 * xu1 + p2 * (r2 + 2 * xu0 * xu0);
        double xd1 = xu1 * (1 + k1 * r2 + k2 * r4) + p1 * (r2 + 2 * xu1 * xu1) + 2 * p2 * xu0 * xu1;
        u = (float)(f0 * xd0 + s * xd1 + c0);
        v = (float)(f1 * xd1 + c1);
    }
    const double k1 = k[0], k2 = k[1], p1 = k[2], p2 = k[3];
    const double r_1 = 1.0 / nrm, r_3 = r_1 * r_1 * r_1;
    const double den = 1.0 / (Xs[2] + xi);
    // dxu/dXs (2x3)
    const double a00 = den, a02 = -Xs[0] * den * den, a11 = den, a12 = -Xs[1] * den * den;
    const double t1 = 2 * k1 * xu0 + 4 * k2 * xu0 * r2;
    const double t2 = 2 * k1 * xu1 + 4 * k2 * xu1 * r2;
    const double b00 = k2 * r4 + 6 * p2 * xu0 + 2 * p1 * xu1 + xu0 * t1 + k1 * r2 + 1;
    const double b01 = 2 * p1 * xu0 + 2 * p2 * xu1 + xu0 * t2;
    const double b10 = 2 * p1 * xu0 + 2 * p2 * xu1 + xu1 * t1;
    const double b11 = k2 * r4 + 2 * p2 * xu0 + 6 * p1 * xu1 + xu1 * t2 + k1 * r2 + 1;
    // P = dxpd/dxd * dxd/dxu (2x2)
    const double q00 = f0 * b00 + s * b10, q01 = f0 * b01 + s * b11;
    const double q10 = f1 * b10, q11 = f1 * b11;
    // Q = P * dxu/dXs (2x3)
    const double w00 = q00 * a00, w01 = q01 * a11, w02 = q00 * a02 + q01 * a12;
    const double w10 = q10 * a00, w11 = q11 * a11, w12 = q10 * a02 + q11 * a12;
    // D = Q * dXs/dXc,  dXs/dXc = r_1 I - r_3 Xc Xc^T
    const double d0 = w00 * Xc[0] + w01 * Xc[1] + w02 * Xc[2];
    const double d1 = w10 * Xc[0] + w11 * Xc[1] + w12 * Xc[2];
    D[0] = w00 * r_1 - d0 * r_3 * Xc[0];
    D[1] = w01 * r_1 - d0 * r_3 * Xc[1];
    D[2] = w02 * r_1 - d0 * r_3 * Xc[2];
    D[3] = w10 * r_1 - d1 * r_3 * Xc[0];
    D[4] = w11 * r_1 - d1 * r_3 * Xc[1];
    D[5] = w12 * r_1 - d1 * r_3 * Xc[2];
}

// ---------------------------------------------------------------- k_linearize
template <int MODEL, bool RATIONAL, bool PRISM>
__global__ __launch_bounds__(256) void k_linearize(LinArgs a) {
    if (a.state->done) return;
    const int photo = blockIdx.x;
    const int e0 = a.photo_ptr[photo];
    const int ne = a.photo_ptr[photo + 1] - e0;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    EdgeLds* el = reinterpret_cast<EdgeLds*>(smem);
    double* ph = smem + (size_t)ne * (sizeof(EdgeLds) / sizeof(double));   // photo scratch
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

    // ---- phase A: edge prologues, one lane per edge
    for (int le = tid; le < ne; le += blockDim.x) edge_prologue<MODEL>(a, photo, e0 + le, el[le]);
    __syncthreads();

    // ---- phase B/C: corner sweep + reduction + chain products, one wave per edge
    for (int base = 0; base < ne; base += 4) {
        const int le = base + wave;
        if (le < ne) {
            EdgeLds& L = el[le];
            const int cam = L.cam, off = L.off, n = L.n;
            double R[9], T[3], kd[12];
#pragma unroll
            for (int q = 0; q < 9; ++q) R[q] = L.R[q];
#pragma unroll
            for (int q = 0; q < 3; ++q) T[q] = L.T[q];
            const int nd = a.nd;
#pragma unroll
            for (int q = 0; q < 12; ++q) kd[q] = q < nd ? (double)a.D[nd * cam + q] : 0.0;
            const float* Kc = a.K + 9 * cam;
            const double fx = Kc[0], fy = Kc[4], cx = Kc[2], cy = Kc[5], sk = Kc[1];
            const double xi = MODEL == MCC_MODEL_OMNI ? (double)a.xi[cam] : 0.0;
            double acc[32];
#pragma unroll
            for (int q = 0; q < 32; ++q) acc[q] = 0.0;
            for (int i = lane; i < n; i += 64) {
                const int c = off + i;
                const double X = a.obj_x[c], Y = a.obj_y[c], Z = a.obj_z[c];
                const float ou = a.img_u[c], ov = a.img_v[c];
                double Yr[3], D[6];
                float u, v;
                if (MODEL == MCC_MODEL_OMNI)
                    omni_corner(R, T, kd, fx, fy, cx, cy, sk, xi, X, Y, Z, Yr, u, v, D);
                else
                    pinhole_corner<RATIONAL, PRISM>(R, T, kd, fx, fy, cx, cy, X, Y, Z, Yr, u, v, D);
                const float euf = ou - u, evf = ov - v;
                if (a.resid) { a.resid[2 * c] = euf; a.resid[2 * c + 1] = evf; }
                const double eu = euf, ev = evf;
                // J' rows: [Y x d, d]
                double ju[6], jv[6];
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
                    for (int s = r; s < 6; ++s) acc[q++] += ju[r] * ju[s] + jv[r] * jv[s];
#pragma unroll
                for (int r = 0; r < 6; ++r) acc[21 + r] += ju[r] * eu + jv[r] * ev;
            }
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
        __syncthreads();
        // X = A' G  (A' symmetric)
        if (le < ne) {
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
        __syncthreads();
        // H = G^T X, g = G^T b'
        if (le < ne) {
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
        __syncthreads();
    }

    // ---- phase D: photo block: Hpp = sum_e, Cholesky, z = L^-1 gp, Y_e = Hgp_e L^-T
    double* Hs = ph;        // 36
    double* gs = ph + 36;   // 6
    double* Lm = ph + 48;   // 36 (lower)
    double* z = ph + 84;    // 6
    if (tid < 42) {
        double s = 0.0;
        for (int le = 0; le < ne; ++le) s += tid < 36 ? el[le].Hpp[tid] : el[le].gp[tid - 36];
        if (tid < 36) Hs[tid] = s; else gs[tid - 36] = s;
    }
    __syncthreads();
    if (tid == 0) {
        int ok = 1;
        for (int j = 0; j < 6; ++j) {
            double s = Hs[j * 6 + j];
            for (int k = 0; k < j; ++k) s -= Lm[j * 6 + k] * Lm[j * 6 + k];
            if (!(s > 0.0)) { ok = 0; s = 1.0; }
            const double l = sqrt(s), il = 1.0 / l;
            Lm[j * 6 + j] = l;
            for (int i = j + 1; i < 6; ++i) {
                double t = Hs[i * 6 + j];
                for (int k = 0; k < j; ++k) t -= Lm[i * 6 + k] * Lm[j * 6 + k];
                Lm[i * 6 + j] = t * il;
            }
            for (int i = 0; i < j; ++i) Lm[i * 6 + j] = 0.0;
        }
        for (int i = 0; i < 6; ++i) {
            double s = gs[i];
            for (int k = 0; k < i; ++k) s -= Lm[i * 6 + k] * z[k];
            z[i] = s / Lm[i * 6 + i];
        }
        if (!ok) atomicOr(&a.state->error, 1);
    }
    __syncthreads();
    double* Lg = a.Lp + 36 * (size_t)photo;
    if (tid < 36) Lg[tid] = Lm[tid];
    else if (tid < 42) a.zp[6 * (size_t)photo + tid - 36] = z[tid - 36];
    else if (tid < 48) a.gp_tot[6 * (size_t)photo + tid - 42] = gs[tid - 42];
    // Y rows: (edge, row i of Hgp) -> forward substitution with L
    for (int t = tid; t < 6 * ne; t += blockDim.x) {
        const int le = t / 6, i = t % 6;
        const EdgeLds& L = el[le];
        const int e = e0 + le;
        double y[6];
        if (L.has_global) {
            for (int j = 0; j < 6; ++j) {
                double s = L.Hgp[i * 6 + j];
                for (int k = 0; k < j; ++k) s -= Lm[j * 6 + k] * y[k];
                y[j] = s / Lm[j * 6 + j];
            }
        } else {
            for (int j = 0; j < 6; ++j) y[j] = 0.0;
        }
        double* Yo = a.Y + 36 * (size_t)e + 6 * i;
        for (int j = 0; j < 6; ++j) Yo[j] = y[j];
        double* Ho = a.Hgg + 36 * (size_t)e + 6 * i;
        for (int j = 0; j < 6; ++j) Ho[j] = L.has_global ? L.Hgg[i * 6 + j] : 0.0;
        a.gg[6 * (size_t)e + i] = L.has_global ? L.gg[i] : 0.0;
    }
}

// ---------------------------------------------------------------- k_schur
// Work item: pairs [begin, end) of one camera-pair block (gb1, gb2).  Thread t < 252:
// entry q = t % 42 (0..35: S block entry, 36..41: r entry), chunk = t / 42 (6 chunks).
__global__ __launch_bounds__(256) void k_schur(SchurArgs a) {
    if (a.state->done) return;
    const int item = blockIdx.x;
    const int4 it = a.items[item];   // {block, begin, end, diag}
    __shared__ double part[6][42];
    const int tid = threadIdx.x;
    const int q = tid % 42, chunk = tid / 42;
    double s = 0.0;
    if (chunk < 6) {
        for (int p = it.y + chunk; p < it.z; p += 6) {
            const int4 pr = a.pairs[p];   // {e1, e2, photo, self}
            const double* Y1 = a.Y + 36 * (size_t)pr.x;
            if (q < 36) {
                const int i = q / 6, j = q % 6;
                const double* Y2 = a.Y + 36 * (size_t)pr.y;
                double t = 0.0;
#pragma unroll
                for (int k = 0; k < 6; ++k) t += Y1[i * 6 + k] * Y2[j * 6 + k];
                s -= t;
                if (pr.w) s += a.Hgg[36 * (size_t)pr.x + q];
            } else if (pr.w) {
                const int i = q - 36;
                const double* zp = a.zp + 6 * (size_t)pr.z;
                double t = 0.0;
#pragma unroll
                for (int k = 0; k < 6; ++k) t += Y1[i * 6 + k] * zp[k];
                s += a.gg[6 * (size_t)pr.x + i] - t;
            }
        }
        part[chunk][q] = s;
    }
    __syncthreads();
    if (tid < 42) {
        double t = part[0][tid];
        for (int c = 1; c < 6; ++c) t += part[c][tid];
        a.item_out[42 * (size_t)item + tid] = t;
    }
}

// ---------------------------------------------------------------- k_assemble (1 workgroup)
// packed layout: [S upper triangle m(m+1)/2][r m][jte_g m][normG2][normX2]
__global__ __launch_bounds__(256) void k_assemble(AsmArgs a) {
    if (a.state->done) return;
    const int m = a.m, nb = m / 6;
    const int tid = threadIdx.x;
    const int ntri = m * (m + 1) / 2;
    for (int t = tid; t < ntri + 2 * m + 2; t += blockDim.x) {
        double v = 0.0;
        if (t < ntri) {
            // (i, j) with i <= j from packed index
            int i = 0, rem = t;
            while (rem >= m - i) { rem -= m - i; ++i; }
            const int j = i + rem;
            int b1 = i / 6, b2 = j / 6, ii = i % 6, jj = j % 6;
            const int blk = b1 * nb - b1 * (b1 - 1) / 2 + (b2 - b1);
            for (int k = a.block_items[blk]; k < a.block_items[blk + 1]; ++k)
                v += a.item_out[42 * (size_t)k + ii * 6 + jj];
        } else if (t < ntri + m) {
            const int g = t - ntri, b = g / 6;
            const int blk = b * nb - b * (b - 1) / 2;
            for (int k = a.block_items[blk]; k < a.block_items[blk + 1]; ++k)
                v += a.item_out[42 * (size_t)k + 36 + g % 6];
        } else if (t < ntri + 2 * m) {
            // JTE of the global block: sum over edges of gg (edge order = photo-major)
            const int g = t - ntri - m, b = g / 6;
            for (int k = a.gblock_ptr[b]; k < a.gblock_ptr[b + 1]; ++k)
                v += a.gg[6 * (size_t)a.gblock_edges[k] + g % 6];
        } else {
            const int w = t - ntri - 2 * m;   // 0: normG2, 1: normX2 (partials of the last update)
            if (a.state->iter > 0) {
                for (int p = 0; p < a.n_photos; ++p) v += a.photo_norm[2 * p + w];
                if (a.rank == 0) v += w ? a.state->cam_normX2 : a.state->cam_normG2;
            }
        }
        a.packed[t] = v;
    }
}

// ---------------------------------------------------------------- k_solve (1 workgroup)
// Stop test, Cholesky of S (one wavefront, LDS), global-block solve and float32 update.
__global__ __launch_bounds__(256) void k_solve(SolveArgs a) {
    State* st = a.state;
    if (st->done) return;
    const int m = a.m, tid = threadIdx.x;
    const int ntri = m * (m + 1) / 2;
    extern __shared__ __attribute__((aligned(16))) double sm[];
    double* S = sm;            // m*m
    double* r = sm + m * m;    // m
    __shared__ int stop;
    if (tid == 0) {
        const int k = st->iter;
        double change = 1.0;
        if (k > 0) change = sqrt(a.packed[ntri + 2 * m]) / sqrt(a.packed[ntri + 2 * m + 1]);
        if (k > 0) st->change = change;
        const int ty = st->crit_type;
        int s = (ty == 1 && k >= st->max_count) || (ty == 2 && change <= st->eps) ||
                (ty == 3 && (change <= st->eps || k >= st->max_count));
        if (!a.do_update) s = 0;
        stop = s;
        if (s) st->done = 1;
        st->alpha = a.do_update ? (k < a.n_alpha ? a.alpha[k] : pow(0.95, (double)k + 1.0)) : 0.0;
    }
    __syncthreads();
    if (stop) return;
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
    if (tid < 64) {
        const int lane = tid;
        // right-looking Cholesky, lower triangle, one wavefront (LDS ops of one wave are ordered)
        for (int j = 0; j < m; ++j) {
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            const double d = S[j * m + j];
            if (!(d > 0.0) && lane == 0) atomicOr(&st->error, 2);
            const double l = sqrt(d > 0.0 ? d : 1.0), il = 1.0 / l;
            for (int i = j + 1 + lane; i < m; i += 64) S[i * m + j] *= il;
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            if (lane == 0) S[j * m + j] = l;
            // trailing update of the lower triangle
            const int w = m - j - 1;
            for (int t = lane; t < w * (w + 1) / 2; t += 64) {
                int ii = 0, rem = t;
                while (rem > ii) { rem -= ii + 1; ++ii; }
                const int i = j + 1 + ii, k = j + 1 + rem;
                S[i * m + k] -= S[i * m + j] * S[k * m + j];
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        if (lane == 0) {
            for (int i = 0; i < m; ++i) {
                double s = r[i];
                for (int k = 0; k < i; ++k) s -= S[i * m + k] * r[k];
                r[i] = s / S[i * m + i];
            }
            for (int i = m - 1; i >= 0; --i) {
                double s = r[i];
                for (int k = i + 1; k < m; ++k) s -= S[k * m + i] * r[k];
                r[i] = s / S[i * m + i];
            }
        }
    }
    __syncthreads();
    // global block: delta, update, norm partials (identical on every rank)
    if (tid == 0) {
        const double alpha = st->alpha;
        double g2 = 0.0, x2 = 0.0;
        for (int i = 0; i < m; ++i) {
            a.dg[i] = r[i];
            a.delta[i] = r[i];
            if (a.do_update) {
                const float G = (float)(alpha * r[i]);
                const float xn = a.x[i] + G;
                a.x[i] = xn;
                g2 += (double)G * (double)G;
                x2 += (double)xn * (double)xn;
            }
        }
        if (a.do_update) {
            st->cam_normG2 = g2;
            st->cam_normX2 = x2;
            st->iter = st->iter + 1;
        }
    }
}

// ---------------------------------------------------------------- k_backsub
// one thread per photo: dp = L^-T (z - sum_e Y_e^T dg_e), x_p = fl32(x_p + fl32(a dp))
__global__ __launch_bounds__(256) void k_backsub(BacksubArgs a) {
    const State* st = a.state;
    if (st->done) return;
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= a.n_photos) return;
    double t[6];
    const double* z = a.zp + 6 * (size_t)p;
#pragma unroll
    for (int k = 0; k < 6; ++k) t[k] = z[k];
    for (int e = a.photo_ptr[p]; e < a.photo_ptr[p + 1]; ++e) {
        const int g = a.edge_gblock[e];
        if (g < 0) continue;
        const double* Y = a.Y + 36 * (size_t)e;
        const double* dg = a.dg + 6 * g;
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            double s = 0.0;
#pragma unroll
            for (int i = 0; i < 6; ++i) s += Y[i * 6 + k] * dg[i];
            t[k] -= s;
        }
    }
    const double* Lm = a.Lp + 36 * (size_t)p;
#pragma unroll
    for (int i = 5; i >= 0; --i) {
        double s = t[i];
#pragma unroll
        for (int k = i + 1; k < 6; ++k) s -= Lm[k * 6 + i] * t[k];
        t[i] = s / Lm[i * 6 + i];
    }
    const int col = a.m + 6 * p;
    double g2 = 0.0, x2 = 0.0;
    const double alpha = st->alpha;
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

// ---------------------------------------------------------------- k_project_error
// computeProjectError (src/mymulticalib.cpp:820-939, src/multicalib.cpp:895-1006,
// src/doubleSide.cpp:640-769): float32 Rodrigues + float32 gemm, Rodrigues back, float
// projection, ferror = sqrtf(ex*ex + ey*ey), per-edge sequential float sum.  One wave per edge.
__device__ __forceinline__ void rod_f32(const float* r, float* Rf) {
    double rd[3] = {r[0], r[1], r[2]}, Rd[9];
    rodrigues_v2m(rd, Rd);
#pragma unroll
    for (int k = 0; k < 9; ++k) Rf[k] = (float)Rd[k];
}

template <int MODEL, bool RATIONAL, bool PRISM>
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
        double Rd[9], rv[3];
        for (int k = 0; k < 9; ++k) Rd[k] = Rt[k];
        polar3(Rd);
        rodrigues_m2v(Rd, rv);
        double rf[3] = {(double)(float)rv[0], (double)(float)rv[1], (double)(float)rv[2]};
        double Rr[9];
        rodrigues_v2m(rf, Rr);
        for (int k = 0; k < 9; ++k) Rs[k] = Rr[k];
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
            pinhole_corner<RATIONAL, PRISM>(R, T, kd, fx, fy, cx, cy, a.obj_x[c], a.obj_y[c], a.obj_z[c], Yr, u, v, D);
        const float ex = a.img_u[c] - u, ey = a.img_v[c] - v;
        float s2 = ex * ex;
        s2 = s2 + ey * ey;
        ferr[i] = sqrtf(s2);
    }
    __syncthreads();
    if (lane == 0) {
        float s = 0.f;
        for (int i = 0; i < n; ++i) s += ferr[i];
        a.edge_sum[e] = s;
    }
}

}  // namespace mcc

// ---------------------------------------------------------------- launch wrappers
using namespace mcc;

template <int MODEL>
static hipError_t launch_lin_model(const LinArgs& a, int n_photos, size_t shmem, hipStream_t s, bool rational, bool prism) {
    if (rational && prism) hipLaunchKernelGGL((k_linearize<MODEL, true, true>), dim3(n_photos), dim3(256), shmem, s, a);
    else if (rational) hipLaunchKernelGGL((k_linearize<MODEL, true, false>), dim3(n_photos), dim3(256), shmem, s, a);
    else if (prism) hipLaunchKernelGGL((k_linearize<MODEL, false, true>), dim3(n_photos), dim3(256), shmem, s, a);
    else hipLaunchKernelGGL((k_linearize<MODEL, false, false>), dim3(n_photos), dim3(256), shmem, s, a);
    return hipGetLastError();
}

size_t mcc_lin_shmem(int max_edges_per_photo) {
    return (size_t)max_edges_per_photo * sizeof(EdgeLds) + 96 * sizeof(double);
}

hipError_t mcc_launch_linearize(const LinArgs& a, int model, int n_photos, int max_epp, bool rational, bool prism, hipStream_t s) {
    const size_t shmem = mcc_lin_shmem(max_epp);
    switch (model) {
        case MCC_MODEL_OMNI: return launch_lin_model<MCC_MODEL_OMNI>(a, n_photos, shmem, s, false, false);
        case MCC_MODEL_DOUBLESIDE: return launch_lin_model<MCC_MODEL_DOUBLESIDE>(a, n_photos, shmem, s, rational, prism);
        default: return launch_lin_model<MCC_MODEL_PINHOLE>(a, n_photos, shmem, s, rational, prism);
    }
}

hipError_t mcc_set_lin_attrs(int max_epp) {
    const size_t shmem = mcc_lin_shmem(max_epp);
    if (shmem <= 64 * 1024) return hipSuccess;
#define SETA(M, R, P) hipFuncSetAttribute((const void*)&k_linearize<M, R, P>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shmem)
    hipError_t err = hipSuccess;
    for (hipError_t e : {SETA(0, false, false), SETA(0, true, false), SETA(0, false, true), SETA(0, true, true),
                         SETA(1, false, false), SETA(2, false, false), SETA(2, true, false), SETA(2, false, true), SETA(2, true, true)})
        if (e != hipSuccess) err = e;
#undef SETA
    return err;
}

hipError_t mcc_launch_schur(const SchurArgs& a, int n_items, hipStream_t s) {
    if (n_items > 0) hipLaunchKernelGGL(k_schur, dim3(n_items), dim3(256), 0, s, a);
    return hipGetLastError();
}
hipError_t mcc_launch_assemble(const AsmArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_assemble, dim3(1), dim3(256), 0, s, a);
    return hipGetLastError();
}
hipError_t mcc_launch_solve(const SolveArgs& a, hipStream_t s) {
    const size_t shmem = (size_t)(a.m * a.m + a.m) * sizeof(double);
    if (shmem > 64 * 1024) (void)hipFuncSetAttribute((const void*)&k_solve, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shmem);
    hipLaunchKernelGGL(k_solve, dim3(1), dim3(256), shmem, s, a);
    return hipGetLastError();
}
hipError_t mcc_launch_backsub(const BacksubArgs& a, hipStream_t s) {
    if (a.n_photos > 0) hipLaunchKernelGGL(k_backsub, dim3((a.n_photos + 255) / 256), dim3(256), 0, s, a);
    return hipGetLastError();
}
hipError_t mcc_launch_project_error(const ErrArgs& a, int model, int n_edges, bool rational, bool prism, hipStream_t s) {
#define PE(M, R, P) hipLaunchKernelGGL((k_project_error<M, R, P>), dim3(n_edges), dim3(64), 0, s, a)
    if (model == MCC_MODEL_OMNI) PE(1, false, false);
    else if (model == MCC_MODEL_DOUBLESIDE) {
        if (rational && prism) PE(2, true, true); else if (rational) PE(2, true, false); else if (prism) PE(2, false, true); else PE(2, false, false);
    } else {
        if (rational && prism) PE(0, true, true); else if (rational) PE(0, true, false); else if (prism) PE(0, false, true); else PE(0, false, false);
    }
#undef PE
    return hipGetLastError();
}
