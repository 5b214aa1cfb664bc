// mcc_device.hpp -- device math for the MI355X BA hot path.
//
// Two kinds of arithmetic live here:
//  * value paths whose float32 rounding is observable in the reference (composed pose -> fl32,
//    projected pixel -> fl32, residual fl32(obs - proj)): evaluated with FMA contraction OFF in
//    the reference's operation order (OpenCV 4.x cvRodrigues2 / cvProjectPoints2Internal,
//    src/omnidir.cpp:141-170), so the float32 residuals match the CPU oracle bit for bit except
//    at float32 rounding ties of FP64 values that differ in the last ulp (transcendentals);
//  * derivative paths (normal equations): closed-form SO(3) Jacobians instead of OpenCV's
//    3x9 / 9x9 chains (compose_motion, src/multicalib.cpp:1008-1056).  They are the same
//    derivatives (exact rotations), evaluated in FP64 with FMA and with every sin/cos/acos
//    computed once; parity vs the oracle is at FP64 rounding level (tests/test_gpu_parity.py).
#pragma once
#include <hip/hip_runtime.h>

namespace mcc {

// ---------------------------------------------------------------- small 3x3 helpers (row-major)
__device__ __forceinline__ void mat3_mul(const double* A, const double* B, double* C) {
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
            C[i * 3 + j] = A[i * 3] * B[j] + A[i * 3 + 1] * B[3 + j] + A[i * 3 + 2] * B[6 + j];
}

// I + s1*[w]x + s2*[w]x^2
__device__ __forceinline__ void so3_poly(const double w[3], double s1, double s2, double* M) {
    const double x = w[0], y = w[1], z = w[2];
    const double xx = x * x, yy = y * y, zz = z * z;
    M[0] = 1.0 + s2 * (-yy - zz);
    M[4] = 1.0 + s2 * (-xx - zz);
    M[8] = 1.0 + s2 * (-xx - yy);
    M[1] = -s1 * z + s2 * x * y;
    M[3] = s1 * z + s2 * x * y;
    M[2] = s1 * y + s2 * x * z;
    M[6] = -s1 * y + s2 * x * z;
    M[5] = -s1 * x + s2 * y * z;
    M[7] = s1 * x + s2 * y * z;
}

// Rotation with the trigonometry of its angle kept for the Jacobians.
struct Rot {
    double R[9];
    double th, s, c;
};

// cvRodrigues2 vector -> matrix in OpenCV's operation order (contraction off).
__device__ __forceinline__ void rodrigues_v2m(const double r[3], Rot& o) {
#pragma clang fp contract(off)
    double rx = r[0], ry = r[1], rz = r[2];
    const double theta = sqrt(rx * rx + ry * ry + rz * rz);
    o.th = theta;
    if (theta < 2.220446049250313e-16) {
        o.s = 0.0; o.c = 1.0;
        o.R[0] = 1; o.R[1] = 0; o.R[2] = 0; o.R[3] = 0; o.R[4] = 1; o.R[5] = 0; o.R[6] = 0; o.R[7] = 0; o.R[8] = 1;
        return;
    }
    double s, c;
    sincos(theta, &s, &c);
    o.s = s; o.c = c;
    const double c1 = 1. - c;
    const double itheta = theta ? 1. / theta : 0.;
    rx *= itheta; ry *= itheta; rz *= itheta;
    const double rrt[9] = {rx * rx, rx * ry, rx * rz, rx * ry, ry * ry, ry * rz, rx * rz, ry * rz, rz * rz};
    const double r_x[9] = {0, -rz, ry, rz, 0, -rx, -ry, rx, 0};
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        const double I = (k == 0 || k == 4 || k == 8) ? 1.0 : 0.0;
        o.R[k] = c * I + c1 * rrt[k] + s * r_x[k];
    }
}

// Left (sign = +1) / right (sign = -1) SO(3) Jacobian from the angle's trig:
//   J = I + sign*a*[w]x + b*[w]x^2,  a = (1-cos)/th^2, b = (th-sin)/th^3.
__device__ __forceinline__ void so3_jac(const double w[3], const Rot& o, double sign, double* J) {
    const double th = o.th, t2 = th * th;
    double a, b;
    if (th < 1e-2) {
        a = 0.5 - t2 * (1.0 / 24.0) + t2 * t2 * (1.0 / 720.0);
        b = 1.0 / 6.0 - t2 * (1.0 / 120.0) + t2 * t2 * (1.0 / 5040.0);
    } else {
        a = (1.0 - o.c) / t2;
        b = (th - o.s) / (t2 * th);
    }
    so3_poly(w, sign * a, b, J);
}

// Inverse left (sign = +1) / right (sign = -1) Jacobian: I - sign*0.5*[w]x + ci*[w]x^2,
// ci = 1/th^2 - (1+cos)/(2 th sin).
__device__ __forceinline__ void so3_jac_inv(const double w[3], double th, double s, double c, double sign, double* J) {
    const double t2 = th * th;
    double ci;
    if (th < 1e-2) ci = 1.0 / 12.0 + t2 * (1.0 / 720.0) + t2 * t2 * (1.0 / 30240.0);
    else ci = 1.0 / t2 - (1.0 + c) / (2.0 * th * s);
    so3_poly(w, -sign * 0.5, ci, J);
}

// The oracle's restatement of the re-orthonormalisation cvRodrigues2 applies first (SVD, U V^T), as a
// Newton iteration X <- (X + X^-T) / 2 in its operation order (oracle/mcc_oracle.c polar3).
__device__ __forceinline__ void polar3_ora(double* R) {
#pragma clang fp contract(off)
    for (int it = 0; it < 40; ++it) {
        const double d = R[0] * (R[4] * R[8] - R[5] * R[7]) - R[1] * (R[3] * R[8] - R[5] * R[6]) +
                         R[2] * (R[3] * R[7] - R[4] * R[6]);
        if (!(fabs(d) > 1e-300)) break;
        double cof[9];
        cof[0] = R[4] * R[8] - R[5] * R[7];
        cof[1] = -(R[3] * R[8] - R[5] * R[6]);
        cof[2] = R[3] * R[7] - R[4] * R[6];
        cof[3] = -(R[1] * R[8] - R[2] * R[7]);
        cof[4] = R[0] * R[8] - R[2] * R[6];
        cof[5] = -(R[0] * R[7] - R[1] * R[6]);
        cof[6] = R[1] * R[5] - R[2] * R[4];
        cof[7] = -(R[0] * R[5] - R[2] * R[3]);
        cof[8] = R[0] * R[4] - R[1] * R[3];
        double delta = 0;
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            const double v = 0.5 * (R[k] + cof[k] / d);
            const double df = fabs(v - R[k]);
            if (df > delta) delta = df;
            R[k] = v;
        }
        if (delta < 1e-15) break;
    }
}

// cvRodrigues2 matrix -> vector (acos branch and the s < 1e-5 branches), returning the angle's
// trig (th, s, c) for the inverse Jacobians.  The SVD re-orthonormalisation OpenCV applies first
// changes an FP64 product of two rotations only at the 1e-16 level, and the vector by ~1e-16 / s.
// It is skipped: near theta = 0 or pi the vector's float32 rounding can follow it (in the s < 1e-5
// branch near pi, which reads the axis from the diagonal, by up to ~1e-16 / |axis component|), but
// the restated polar step (polar3_ora, as the oracle and the host edge Jacobian run it) cost config4
// 0.5 us per step in instruction-cache misses even untaken (SQC_ICACHE_MISSES +24 %, round 6), for a
// value that is rounding noise of an ill-conditioned formula there (OpenCV's SVD gives other last
// bits than either restatement).  tests/test_rodrigues_branch.py holds the pi-branch edge's residuals
// to a float32-noise bar instead.
__device__ __forceinline__ void rodrigues_m2v(const double* Rin, double* r, double& th_o, double& s_o, double& c_o,
                                              int& jz) {
#pragma clang fp contract(off)
    jz = 0;
    const double* R = Rin;
    double rx = R[7] - R[5], ry = R[2] - R[6], rz = R[3] - R[1];
    double s = sqrt((rx * rx + ry * ry + rz * rz) * 0.25);
    double c = (R[0] + R[4] + R[8] - 1) * 0.5;
    c = c > 1. ? 1. : c < -1. ? -1. : c;
    double theta = acos(c);
    th_o = theta; s_o = s; c_o = c;
    if (s < 1e-5) {
        if (c > 0) {
            rx = ry = rz = 0;
        } else {
            jz = 1;   // (rot_jzero)
            double t;
            t = (R[0] + 1) * 0.5; rx = sqrt(t > 0 ? t : 0.);
            t = (R[4] + 1) * 0.5; ry = sqrt(t > 0 ? t : 0.) * (R[1] < 0 ? -1. : 1.);
            t = (R[8] + 1) * 0.5; rz = sqrt(t > 0 ? t : 0.) * (R[2] < 0 ? -1. : 1.);
            if (fabs(rx) < fabs(ry) && fabs(rx) < fabs(rz) && (R[5] > 0) != (ry * rz > 0)) rz = -rz;
            theta /= sqrt(rx * rx + ry * ry + rz * rz);
            rx *= theta; ry *= theta; rz *= theta;
        }
    } else {
        double vth = 1 / (2 * s);
        vth *= theta;
        rx *= vth; ry *= vth; rz *= vth;
    }
    r[0] = rx; r[1] = ry; r[2] = rz;
}
// (jz: 1 in the theta ~ pi branch, where cvRodrigues2's d om / d R is zero -- rot_jzero's case)
__device__ __forceinline__ void rodrigues_m2v(const double* R, double* r, double& th_o, double& s_o, double& c_o) {
    int jz;
    rodrigues_m2v(R, r, th_o, s_o, c_o, jz);
}

// cvRodrigues2's derivative d om / d R in its s < 1e-5 branch near theta = pi (c <= 0) is ZERO (it
// fills the 3 x 9 Jacobian only for c > 0), so compose_motion's d om3 / d om1 and d om3 / d om2 vanish
// for a composed rotation within ~1e-5 rad of pi (DoubleSide rigs: a camera facing the board's back;
// config5's rig has one such edge after its first update).  The closed-form inverse Jacobians below
// would give the true derivative there; the reference gives 0, and so do we (rot_jzero).  (Near
// theta = 0, c > 0, OpenCV's fixed 0.5 pattern equals the closed form to O(theta) < 1e-5.)
#ifdef MCC_NO_JZERO   // (A/B builds only)
__device__ __forceinline__ bool rot_jzero(double, double) { return false; }
#else
__device__ __forceinline__ bool rot_jzero(double s, double c) { return s < 1e-5 && !(c > 0); }
#endif

// Polar factor (U V^T) by Newton iteration, for float32 products of rotations (metric path).
__device__ __forceinline__ void polar3(double* R) {
    for (int it = 0; it < 8; ++it) {
        double cof[9];
        cof[0] = R[4] * R[8] - R[5] * R[7];
        cof[1] = -(R[3] * R[8] - R[5] * R[6]);
        cof[2] = R[3] * R[7] - R[4] * R[6];
        cof[3] = -(R[1] * R[8] - R[2] * R[7]);
        cof[4] = R[0] * R[8] - R[2] * R[6];
        cof[5] = -(R[0] * R[7] - R[1] * R[6]);
        cof[6] = R[1] * R[5] - R[2] * R[4];
        cof[7] = -(R[0] * R[5] - R[2] * R[3]);
        cof[8] = R[0] * R[4] - R[1] * R[3];
        const double d = R[0] * cof[0] + R[1] * cof[1] + R[2] * cof[2];
        const double id = 1.0 / d;
        double delta = 0;
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            const double v = 0.5 * (R[k] + cof[k] * id);
            delta = fmax(delta, fabs(v - R[k]));
            R[k] = v;
        }
        if (delta < 1e-15) break;
    }
}

// ---------------------------------------------------------------- compose_motion
// R3 = R2 R1, T3 = R2 T1 + T2 (src/multicalib.cpp:1030-1051, OpenCV small-gemm order) and
//   A1 = d om3/d om1 = Jr(om3)^-1 Jr(om1),  A2 = d om3/d om2 = Jl(om3)^-1 Jl(om2),
//   B2 = d T3/d om2 = -[R2 T1]x Jl(om2);   d T3/d T1 = R2, d T3/d T2 = I, other blocks 0.
// r1 / r2 are the Rodrigues of om1 / om2 (with trig); Jr1 = Jr(om1), Jl2 = Jl(om2).
struct Motion {
    double om[3], T[3], R[9];
    double A1[9], A2[9], B2[9];
};

// th / s / c: the composed angle's trig from the matrix -> vector formula (for Jacobians and
// the Rodrigues of the float32-rounded vector).
__device__ __forceinline__ void compose(const double* R1, const double* Jr1, const double* T1,
                                        const double* R2, const double* Jl2, const double* T2, Motion& m,
                                        double& th, double& s, double& c) {
    double* R3 = m.R;
    double q[3];
    {
#pragma clang fp contract(off)
#pragma unroll
        for (int i = 0; i < 3; ++i) {
#pragma unroll
            for (int j = 0; j < 3; ++j)
                R3[i * 3 + j] = R2[i * 3] * R1[j] + R2[i * 3 + 1] * R1[3 + j] + R2[i * 3 + 2] * R1[6 + j];
            q[i] = R2[i * 3] * T1[0] + R2[i * 3 + 1] * T1[1] + R2[i * 3 + 2] * T1[2];
            m.T[i] = q[i] + T2[i];
        }
    }
    double Ji[9];
    rodrigues_m2v(R3, m.om, th, s, c);
    so3_jac_inv(m.om, th, s, c, -1.0, Ji);   // Jr^-1(om3)
    mat3_mul(Ji, Jr1, m.A1);
    so3_jac_inv(m.om, th, s, c, +1.0, Ji);   // Jl^-1(om3)
    mat3_mul(Ji, Jl2, m.A2);
    if (rot_jzero(s, c)) {   // (cvRodrigues2's theta ~ pi branch)
#pragma unroll
        for (int k = 0; k < 9; ++k) m.A1[k] = m.A2[k] = 0.0;
    }
    const double qx[9] = {0, q[2], -q[1], -q[2], 0, q[0], q[1], -q[0], 0};   // -[q]x
    mat3_mul(qx, Jl2, m.B2);
}

}  // namespace mcc
