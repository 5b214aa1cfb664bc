// mcc_device.hpp -- device math for the MI355X BA hot path.
//
// Two kinds of arithmetic live here:
//  * value paths whose float32 rounding is observable in the reference (composed pose -> fl32,
//    projected pixel -> fl32, residual fl32(obs - proj)): evaluated with FMA contraction OFF in
//    the reference's operation order (OpenCV 4.x cvRodrigues2 / cvProjectPoints2Internal,
//    src/omnidir.cpp:141-170), so the float32 residuals match the CPU oracle bit for bit except
//    at float32 rounding ties of FP64 values that differ in the last ulp (transcendentals);
//  * derivative paths (normal equations): closed-form SO(3) Jacobians instead of OpenCV's
//    3x9 / 9x9 chains.  They are the same derivatives (exact rotations), evaluated in FP64 with
//    FMA; parity vs the oracle is at FP64 rounding level (tests/test_gpu_parity.py).
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
    // [w]x^2 = w w^T - |w|^2 I
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

// Coefficients of the SO(3) Jacobians at angle th:
//   a = (1-cos)/th^2, b = (th-sin)/th^3, c = 1/th^2 - (1+cos)/(2 th sin)
__device__ __forceinline__ void so3_coeffs(double th, double& a, double& b, double& c) {
    const double t2 = th * th;
    if (th < 1e-2) {
        a = 0.5 - t2 * (1.0 / 24.0) + t2 * t2 * (1.0 / 720.0);
        b = 1.0 / 6.0 - t2 * (1.0 / 120.0) + t2 * t2 * (1.0 / 5040.0);
        c = 1.0 / 12.0 + t2 * (1.0 / 720.0) + t2 * t2 * (1.0 / 30240.0);
    } else {
        double s, co;
        sincos(th, &s, &co);
        a = (1.0 - co) / t2;
        b = (th - s) / (t2 * th);
        c = 1.0 / t2 - (1.0 + co) / (2.0 * th * s);
    }
}

// left Jacobian J_l(w) (d Exp(w) / dw as left perturbation) and inverses.
__device__ __forceinline__ void so3_jl(const double w[3], double* J) {
    double th = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]), a, b, c;
    so3_coeffs(th, a, b, c);
    so3_poly(w, a, b, J);
}
__device__ __forceinline__ void so3_jr(const double w[3], double* J) {
    double th = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]), a, b, c;
    so3_coeffs(th, a, b, c);
    so3_poly(w, -a, b, J);
}
__device__ __forceinline__ void so3_jl_inv(const double w[3], double* J) {
    double th = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]), a, b, c;
    so3_coeffs(th, a, b, c);
    so3_poly(w, -0.5, c, J);
}
__device__ __forceinline__ void so3_jr_inv(const double w[3], double* J) {
    double th = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]), a, b, c;
    so3_coeffs(th, a, b, c);
    so3_poly(w, 0.5, c, J);
}

// ---------------------------------------------------------------- Rodrigues (value paths)
// cvRodrigues2 vector -> matrix in OpenCV's operation order (contraction off).
__device__ __forceinline__ void rodrigues_v2m(const double r[3], double* R) {
#pragma clang fp contract(off)
    double rx = r[0], ry = r[1], rz = r[2];
    double theta = sqrt(rx * rx + ry * ry + rz * rz);
    if (theta < 2.220446049250313e-16) {
        R[0] = 1; R[1] = 0; R[2] = 0; R[3] = 0; R[4] = 1; R[5] = 0; R[6] = 0; R[7] = 0; R[8] = 1;
        return;
    }
    double s, c;
    sincos(theta, &s, &c);
    double c1 = 1. - c;
    double itheta = theta ? 1. / theta : 0.;
    rx *= itheta; ry *= itheta; rz *= itheta;
    const double rrt[9] = {rx * rx, rx * ry, rx * rz, rx * ry, ry * ry, ry * rz, rx * rz, ry * rz, rz * rz};
    const double r_x[9] = {0, -rz, ry, rz, 0, -rx, -ry, rx, 0};
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        double I = (k == 0 || k == 4 || k == 8) ? 1.0 : 0.0;
        R[k] = c * I + c1 * rrt[k] + s * r_x[k];
    }
}

// rotation vector of an (orthonormal to FP64 precision) matrix: cvRodrigues2 matrix -> vector
// formula (acos branch; the s < 1e-5 branches follow OpenCV too).  The SVD re-orthonormalisation
// OpenCV applies first changes an FP64 product of two rotations only at the 1e-16 level.
__device__ __forceinline__ void rodrigues_m2v(const double* R, double* r) {
#pragma clang fp contract(off)
    double rx = R[7] - R[5], ry = R[2] - R[6], rz = R[3] - R[1];
    double s = sqrt((rx * rx + ry * ry + rz * rz) * 0.25);
    double c = (R[0] + R[4] + R[8] - 1) * 0.5;
    c = c > 1. ? 1. : c < -1. ? -1. : c;
    double theta = acos(c);
    if (s < 1e-5) {
        if (c > 0) {
            rx = ry = rz = 0;
        } else {
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
        double d = R[0] * cof[0] + R[1] * cof[1] + R[2] * cof[2];
        double id = 1.0 / d, delta = 0;
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            double v = 0.5 * (R[k] + cof[k] * id);
            delta = fmax(delta, fabs(v - R[k]));
            R[k] = v;
        }
        if (delta < 1e-15) break;
    }
}

// ---------------------------------------------------------------- compose_motion derivatives
// Pose composition (src/multicalib.cpp:1008-1056): R3 = R2 R1, T3 = R2 T1 + T2 and
//   A1 = d om3/d om1 = Jr(om3)^-1 Jr(om1),  A2 = d om3/d om2 = Jl(om3)^-1 Jl(om2),
//   B2 = d T3/d om2 = -[R2 T1]x Jl(om2),    d T3/d T1 = R2, d T3/d T2 = I, other blocks 0.
struct Motion {
    double om[3], T[3], R[9];   // composed
    double A1[9], A2[9], B2[9], R2[9];
};

__device__ __forceinline__ void compose_motion(const double om1[3], const double T1[3],
                                               const double om2[3], const double T2[3], Motion& m) {
    double R1[9];
    rodrigues_v2m(om1, R1);
    rodrigues_v2m(om2, m.R2);
    {
#pragma clang fp contract(off)
        // R3 = R2 * R1 and T3t = R2 * T1 in OpenCV's small-gemm order, T3 = T3t + T2
#pragma unroll
        for (int i = 0; i < 3; ++i) {
#pragma unroll
            for (int j = 0; j < 3; ++j)
                m.R[i * 3 + j] = m.R2[i * 3] * R1[j] + m.R2[i * 3 + 1] * R1[3 + j] + m.R2[i * 3 + 2] * R1[6 + j];
            double t = m.R2[i * 3] * T1[0] + m.R2[i * 3 + 1] * T1[1] + m.R2[i * 3 + 2] * T1[2];
            m.T[i] = t + T2[i];
        }
    }
    rodrigues_m2v(m.R, m.om);
    double Ji[9], J[9];
    so3_jr_inv(m.om, Ji);
    so3_jr(om1, J);
    mat3_mul(Ji, J, m.A1);
    so3_jl_inv(m.om, Ji);
    double Jl2[9];
    so3_jl(om2, Jl2);
    mat3_mul(Ji, Jl2, m.A2);
    double q[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) q[i] = m.R2[i * 3] * T1[0] + m.R2[i * 3 + 1] * T1[1] + m.R2[i * 3 + 2] * T1[2];
    // -[q]x Jl2
    const double qx[9] = {0, q[2], -q[1], -q[2], 0, q[0], q[1], -q[0], 0};
    mat3_mul(qx, Jl2, m.B2);
}

}  // namespace mcc
