// edge_jacobian.cpp -- one edge's linearisation on the host: the reference's per-edge
// computePhotoCameraJacobian, for callers of the cv::Mat seam that assemble their own normal
// equations the way the reference's computeJacobianExtrinsic does (a subclass that reuses that
// body; the library itself linearises whole steps on the GPU and never calls this).
//
//   base class   src/multicalib.cpp:717-824    compose(photo, camera), then the camera model
//   MyMulti      src/mymulticalib.cpp:468-614  BACK views: compose(ds, photofront) and the chain,
//                                              without dT/dTpf * dTpf/dRc (:516, SURVEY hazard A12)
//   DoubleSide   src/doubleSide.cpp:288-430    the global block is ds; FRONT views: zero (:335-336)
//
// The composed pose is rounded to float32 before it is projected (mymulticalib.cpp:546-553); the
// residual is fl32(obs - proj) widened to double, rows [u0, v0, u1, v1, ...] (:578-586).  The value
// path (rotation of the float pose, projection) follows OpenCV's operation order -- the order the
// device kernels use (mcc_device.hpp), so the float32 residuals agree with the GPU's bit for bit
// except at rare FP64 rounding ties of a transcendental.  The derivatives are the closed-form SO(3)
// chain the device uses (d(R X)/dr = -[R X]x Jl(r); compose_motion's partials in composeMotion),
// the same derivatives OpenCV's 3x9 Rodrigues / matMulDeriv chains evaluate.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <stdexcept>

#include "../../include/mcc_multicalib.hpp"

namespace mcc {
namespace multicalib {

namespace {

void mat3(const double* A, const double* B, double* C) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) C[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
}

// I + s1 [w]x + s2 [w]x^2
void so3_poly(const double w[3], double s1, double s2, double M[9]) {
    const double x = w[0], y = w[1], z = w[2];
    M[0] = 1.0 + s2 * (-y * y - z * z);
    M[4] = 1.0 + s2 * (-x * x - z * z);
    M[8] = 1.0 + s2 * (-x * x - y * y);
    M[1] = -s1 * z + s2 * x * y;
    M[3] = s1 * z + s2 * x * y;
    M[2] = s1 * y + s2 * x * z;
    M[6] = -s1 * y + s2 * x * z;
    M[5] = -s1 * x + s2 * y * z;
    M[7] = s1 * x + s2 * y * z;
}

// left (sign +1) / right (sign -1) SO(3) Jacobian of w, or its inverse
void so3_jac(const double w[3], double sign, bool inverse, double J[9]) {
    const double th = std::sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]), t2 = th * th;
    if (inverse) {
        const double ci = th < 1e-2 ? 1.0 / 12.0 + t2 / 720.0 + t2 * t2 / 30240.0
                                    : 1.0 / t2 - (1.0 + std::cos(th)) / (2.0 * th * std::sin(th));
        so3_poly(w, -sign * 0.5, ci, J);
    } else {
        const double a = th < 1e-2 ? 0.5 - t2 / 24.0 + t2 * t2 / 720.0 : (1.0 - std::cos(th)) / t2;
        const double b = th < 1e-2 ? 1.0 / 6.0 - t2 / 120.0 + t2 * t2 / 5040.0 : (th - std::sin(th)) / (t2 * th);
        so3_poly(w, sign * a, b, J);
    }
}

// cvRodrigues2 vector -> matrix in OpenCV's order (cos / sin of the angle, the normalised axis)
void rot_of(const double r[3], double R[9]) {
    const double th = std::sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
    if (th < 2.220446049250313e-16) {
        for (int k = 0; k < 9; ++k) R[k] = k % 4 == 0 ? 1.0 : 0.0;
        return;
    }
    const double c = std::cos(th), s = std::sin(th), c1 = 1. - c, it = 1. / th;
    const double x = r[0] * it, y = r[1] * it, z = r[2] * it;
    const double rrt[9] = {x * x, x * y, x * z, x * y, y * y, y * z, x * z, y * z, z * z};
    const double rx[9] = {0, -z, y, z, 0, -x, -y, x, 0};
    for (int k = 0; k < 9; ++k) R[k] = c * (k % 4 == 0 ? 1.0 : 0.0) + c1 * rrt[k] + s * rx[k];
}

// the SVD re-orthonormalisation cvRodrigues2 applies first, as the oracle restates it (Newton
// iteration X <- (X + X^-T) / 2, oracle/mcc_oracle.c polar3; the device's polar3_ora)
void polar_of(const double* Rin, double* R) {
    std::memcpy(R, Rin, 9 * sizeof(double));
    for (int it = 0; it < 40; ++it) {
        const double d = R[0] * (R[4] * R[8] - R[5] * R[7]) - R[1] * (R[3] * R[8] - R[5] * R[6]) +
                         R[2] * (R[3] * R[7] - R[4] * R[6]);
        if (!(std::fabs(d) > 1e-300)) break;
        const double cof[9] = {R[4] * R[8] - R[5] * R[7], -(R[3] * R[8] - R[5] * R[6]), R[3] * R[7] - R[4] * R[6],
                               -(R[1] * R[8] - R[2] * R[7]), R[0] * R[8] - R[2] * R[6], -(R[0] * R[7] - R[1] * R[6]),
                               R[1] * R[5] - R[2] * R[4], -(R[0] * R[5] - R[2] * R[3]), R[0] * R[4] - R[1] * R[3]};
        double delta = 0;
        for (int k = 0; k < 9; ++k) {
            const double v = 0.5 * (R[k] + cof[k] / d);
            delta = std::max(delta, std::fabs(v - R[k]));
            R[k] = v;
        }
        if (delta < 1e-15) break;
    }
}

// cvRodrigues2 matrix -> vector (the acos branch and the s < 1e-5 branches near 0 and pi); the
// re-orthonormalisation only where the vector's float32 rounding follows it, s < 1e-3 (the device's
// rodrigues_m2v)
void log_of(const double* Rin, double r[3]) {
    const double* R = Rin;
    double rx = R[7] - R[5], ry = R[2] - R[6], rz = R[3] - R[1];
    double s = std::sqrt((rx * rx + ry * ry + rz * rz) * 0.25);
    double Rp[9];
    if (s < 1e-3) {
        polar_of(Rin, Rp);
        R = Rp;
        rx = R[7] - R[5]; ry = R[2] - R[6]; rz = R[3] - R[1];
        s = std::sqrt((rx * rx + ry * ry + rz * rz) * 0.25);
    }
    double c = (R[0] + R[4] + R[8] - 1) * 0.5;
    c = c > 1. ? 1. : c < -1. ? -1. : c;
    double theta = std::acos(c);
    if (s < 1e-5) {
        if (c > 0) {
            rx = ry = rz = 0;
        } else {
            double t = (R[0] + 1) * 0.5;
            rx = std::sqrt(t > 0 ? t : 0.);
            t = (R[4] + 1) * 0.5;
            ry = std::sqrt(t > 0 ? t : 0.) * (R[1] < 0 ? -1. : 1.);
            t = (R[8] + 1) * 0.5;
            rz = std::sqrt(t > 0 ? t : 0.) * (R[2] < 0 ? -1. : 1.);
            if (std::fabs(rx) < std::fabs(ry) && std::fabs(rx) < std::fabs(rz) && (R[5] > 0) != (ry * rz > 0)) rz = -rz;
            theta /= std::sqrt(rx * rx + ry * ry + rz * rz);
            rx *= theta; ry *= theta; rz *= theta;
        }
    } else {
        double vth = 1 / (2 * s);
        vth *= theta;
        rx *= vth; ry *= vth; rz *= vth;
    }
    r[0] = rx; r[1] = ry; r[2] = rz;
}

// computeTiltProjectionMatrix (OpenCV calib3d): matTilt = matProjZ * (matRotY(tau_y) * matRotX(tau_x))
void tilt_of(double tx, double ty, double M[9]) {
    const double cx = std::cos(tx), sx = std::sin(tx), cy = std::cos(ty), sy = std::sin(ty);
    const double rx[9] = {1, 0, 0, 0, cx, sx, 0, -sx, cx}, ry[9] = {cy, 0, -sy, 0, 1, 0, sy, 0, cy};
    double rxy[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double s = 0;
            for (int q = 0; q < 3; ++q) s += ry[3 * i + q] * rx[3 * q + j];
            rxy[3 * i + j] = s;
        }
    const double pz[9] = {rxy[8], 0, -rxy[2], 0, rxy[8], -rxy[5], 0, 0, 1};
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double s = 0;
            for (int q = 0; q < 3; ++q) s += pz[3 * i + q] * rxy[3 * q + j];
            M[3 * i + j] = s;
        }
}

// One corner through cv::projectPoints' pinhole model (cvProjectPoints2Internal, k1 k2 p1 p2 [k3
// [k4 k5 k6 [s1 s2 s3 s4 [tau_x tau_y]]]]): the float32 pixel and D = d(u, v)/dXc (2 x 3).  mt: the
// tilted sensor's matTilt (null: none) -- vecTilt = mt (xd0, yd0, 1), (xd, yd) = vecTilt(0..1) / vecTilt(2)
void pinhole_point(const double* R, const double* T, const double* k, const float* Kf, const float* P, float& u,
                   float& v, double* Yr, double* D, const double* mt) {
    const double fx = Kf[0], fy = Kf[4], cx = Kf[2], cy = Kf[5];
    const double X = P[0], Y = P[1], Z = P[2];
    Yr[0] = R[0] * X + R[1] * Y + R[2] * Z;
    Yr[1] = R[3] * X + R[4] * Y + R[5] * Z;
    Yr[2] = R[6] * X + R[7] * Y + R[8] * Z;
    double x = Yr[0] + T[0], y = Yr[1] + T[1], z = Yr[2] + T[2];
    z = z ? 1. / z : 1;
    x *= z;
    y *= z;
    const double r2 = x * x + y * y, r4 = r2 * r2, r6 = r4 * r2;
    const double a1 = 2 * x * y, a2 = r2 + 2 * x * x, a3 = r2 + 2 * y * y;
    const double cdist = 1 + k[0] * r2 + k[1] * r4 + k[4] * r6;
    const double icdist2 = 1. / (1 + k[5] * r2 + k[6] * r4 + k[7] * r6);
    double xd = x * cdist * icdist2 + k[2] * a1 + k[3] * a2 + k[8] * r2 + k[9] * r4;
    double yd = y * cdist * icdist2 + k[2] * a3 + k[3] * a1 + k[10] * r2 + k[11] * r4;
    double t0 = 0, t1 = 0, t2 = 1, ip = 1;
    if (mt) {
        t0 = mt[0] * xd + mt[1] * yd + mt[2];
        t1 = mt[3] * xd + mt[4] * yd + mt[5];
        t2 = mt[6] * xd + mt[7] * yd + mt[8];
        ip = t2 ? 1. / t2 : 1;
        xd = ip * t0;
        yd = ip * t1;
    }
    u = (float)(xd * fx + cx);
    v = (float)(yd * fy + cy);
    // the distortion map's derivative w.r.t. the normalised point, then d(x, y)/dXc
    const double cc = cdist * icdist2;
    const double g = (k[0] + 2 * k[1] * r2 + 3 * k[4] * r4) * icdist2 -
                     cdist * icdist2 * icdist2 * (k[5] + 2 * k[6] * r2 + 3 * k[7] * r4);
    const double P1 = k[8] + 2 * r2 * k[9], P2 = k[10] + 2 * r2 * k[11];
    double m00 = cc + 2 * x * x * g + 2 * k[2] * y + 6 * k[3] * x + 2 * x * P1;
    double m01 = 2 * x * y * g + 2 * k[2] * x + 2 * k[3] * y + 2 * y * P1;
    double m10 = 2 * x * y * g + 2 * k[2] * x + 2 * k[3] * y + 2 * x * P2;
    double m11 = cc + 2 * y * y * g + 6 * k[2] * y + 2 * k[3] * x + 2 * y * P2;
    if (mt) {   // dMatTilt (2 x 2) after the distortion map
        const double ip2 = ip * ip;
        const double d00 = (mt[0] * t2 - mt[6] * t0) * ip2, d01 = (mt[1] * t2 - mt[7] * t0) * ip2;
        const double d10 = (mt[3] * t2 - mt[6] * t1) * ip2, d11 = (mt[4] * t2 - mt[7] * t1) * ip2;
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

// One corner through cv::omnidir::projectPoints (Mei model, src/omnidir.cpp:141-208)
void omni_point(const double* R, const double* T, const double* k, const float* Kf, double xi, const float* P,
                float& u, float& v, double* Yr, double* D) {
    const double f0 = Kf[0], f1 = Kf[4], c0 = Kf[2], c1 = Kf[5], s = Kf[1];
    const double X = P[0], Y = P[1], Z = P[2];
    Yr[0] = R[0] * X + R[1] * Y + R[2] * Z;
    Yr[1] = R[3] * X + R[4] * Y + R[5] * Z;
    Yr[2] = R[6] * X + R[7] * Y + R[8] * Z;
    const double Xc[3] = {Yr[0] + T[0], Yr[1] + T[1], Yr[2] + T[2]};
    const double nrm = std::sqrt(Xc[0] * Xc[0] + Xc[1] * Xc[1] + Xc[2] * Xc[2]), inrm = 1. / nrm;
    const double Xs[3] = {Xc[0] * inrm, Xc[1] * inrm, Xc[2] * inrm};
    const double xu0 = Xs[0] / (Xs[2] + xi), xu1 = Xs[1] / (Xs[2] + xi);
    const double r2 = xu0 * xu0 + xu1 * xu1, r4 = r2 * r2;
    const double k1 = k[0], k2 = k[1], p1 = k[2], p2 = k[3];
    const double xd0 = xu0 * (1 + k1 * r2 + k2 * r4) + 2 * p1 * xu0 * xu1 + p2 * (r2 + 2 * xu0 * xu0);
    const double xd1 = xu1 * (1 + k1 * r2 + k2 * r4) + p1 * (r2 + 2 * xu1 * xu1) + 2 * p2 * xu0 * xu1;
    u = (float)(f0 * xd0 + s * xd1 + c0);
    v = (float)(f1 * xd1 + c1);
    // d pixel / d xd (2 x 2) * d xd / d xu (2 x 2) * d xu / d Xs (2 x 3) * d Xs / d Xc (3 x 3)
    const double den = 1.0 / (Xs[2] + xi);
    const double a00 = den, a02 = -Xs[0] * den * den, a11 = den, a12 = -Xs[1] * den * den;
    const double t1 = 2 * k1 * xu0 + 4 * k2 * xu0 * r2, t2 = 2 * k1 * xu1 + 4 * k2 * xu1 * r2;
    const double b00 = k2 * r4 + 6 * p2 * xu0 + 2 * p1 * xu1 + xu0 * t1 + k1 * r2 + 1;
    const double b01 = 2 * p1 * xu0 + 2 * p2 * xu1 + xu0 * t2;
    const double b10 = 2 * p1 * xu0 + 2 * p2 * xu1 + xu1 * t1;
    const double b11 = k2 * r4 + 2 * p2 * xu0 + 6 * p1 * xu1 + xu1 * t2 + k1 * r2 + 1;
    const double q00 = f0 * b00 + s * b10, q01 = f0 * b01 + s * b11, q10 = f1 * b10, q11 = f1 * b11;
    const double w[2][3] = {{q00 * a00, q01 * a11, q00 * a02 + q01 * a12}, {q10 * a00, q11 * a11, q10 * a02 + q11 * a12}};
    const double r_1 = 1.0 / nrm, r_3 = r_1 * r_1 * r_1;
    for (int i = 0; i < 2; ++i) {
        const double d = w[i][0] * Xc[0] + w[i][1] * Xc[1] + w[i][2] * Xc[2];
        for (int j = 0; j < 3; ++j) D[3 * i + j] = w[i][j] * r_1 - d * r_3 * Xc[j];
    }
}

}  // namespace

void composeMotion(const double om1[3], const double T1[3], const double om2[3], const double T2[3], double om3[3],
                   double T3[3], double d[8][9]) {
    double R1[9], R2[9], R3[9], q[3];
    rot_of(om1, R1);
    rot_of(om2, R2);
    mat3(R2, R1, R3);
    for (int i = 0; i < 3; ++i) {
        q[i] = R2[3 * i] * T1[0] + R2[3 * i + 1] * T1[1] + R2[3 * i + 2] * T1[2];
        T3[i] = q[i] + T2[i];
    }
    log_of(R3, om3);
    double Jr1[9], Jl2[9], Ji[9];
    so3_jac(om1, -1.0, false, Jr1);
    so3_jac(om2, +1.0, false, Jl2);
    so3_jac(om3, -1.0, true, Ji);
    mat3(Ji, Jr1, d[0]);                                   // dom3/dom1 = Jr(om3)^-1 Jr(om1)
    so3_jac(om3, +1.0, true, Ji);
    mat3(Ji, Jl2, d[2]);                                   // dom3/dom2 = Jl(om3)^-1 Jl(om2)
    {
        // cvRodrigues2's s < 1e-5 branch near theta = pi: d om / d R is zero there, so are both
        // partials (mcc_device.hpp rot_jzero)
        const double sx = R3[7] - R3[5], sy = R3[2] - R3[6], sz = R3[3] - R3[1];
        const double s = std::sqrt((sx * sx + sy * sy + sz * sz) * 0.25);
        double c = (R3[0] + R3[4] + R3[8] - 1) * 0.5;
        c = c > 1. ? 1. : c < -1. ? -1. : c;
        if (s < 1e-5 && !(c > 0))
            for (int k = 0; k < 9; ++k) d[0][k] = d[2][k] = 0.0;
    }
    const double qx[9] = {0, q[2], -q[1], -q[2], 0, q[0], q[1], -q[0], 0};   // -[R2 T1]x
    mat3(qx, Jl2, d[6]);                                   // dT3/dom2
    std::memcpy(d[5], R2, sizeof(R2));                     // dT3/dT1
    for (int k = 0; k < 9; ++k) {
        d[1][k] = d[3][k] = d[4][k] = 0.0;                 // dom3/dT1, dom3/dT2, dT3/dom1
        d[7][k] = k % 4 == 0 ? 1.0 : 0.0;                  // dT3/dT2
    }
}

void edgeJacobian(int edgeClass, bool omni, int patternSide, const double rP[3], const double tP[3],
                  const double rC[3], const double tC[3], const double* rDs, const double* tDs, int n,
                  const float* obj, const float* img, const float K[9], const float* D, int nd, float xi,
                  EdgeLinearization& out) {
    if (n < 0 || (n && (!obj || !img))) throw std::invalid_argument("edgeJacobian: bad corner arrays");
    if (!omni && !(nd == 4 || nd == 5 || nd == 8 || nd == 12 || nd == 14))
        throw std::invalid_argument("edgeJacobian: pinhole distortion must have 4, 5, 8, 12 or 14 terms");
    if (omni && nd != 4) throw std::invalid_argument("edgeJacobian: omnidir distortion must have 4 terms");
    const bool back = patternSide == MultiCameraCalibration::BACK_PATTERN && edgeClass != EDGE_BASE;
    if (back && (!rDs || !tDs)) throw std::invalid_argument("edgeJacobian: a BACK view needs the double-side transform");

    // photofront = camera * photo (src/mymulticalib.cpp:498-500, src/multicalib.cpp:737-739)
    double omf[3], Tf[3], df[8][9];
    composeMotion(rP, tP, rC, tC, omf, Tf, df);
    // chain maps of the projected pose: photo [dR/dRp, dR/dTp, dT/dRp, dT/dTp], global block alike
    double cp[4][9], cg[4][9];
    double om[3], T[3];
    if (back) {
        double db[8][9];
        composeMotion(rDs, tDs, omf, Tf, om, T, db);   // compose_motion(ds, photofront) (:503-506)
        mat3(db[2], df[0], cp[0]);                      // dRt/dRp = dRt/dRf dRf/dRp        (:509)
        mat3(db[3], df[5], cp[1]);                      // dRt/dTp = dRt/dTf dTf/dTp (= 0)  (:510)
        mat3(db[6], df[0], cp[2]);                      // dTt/dRp = dTt/dRf dRf/dRp        (:511)
        mat3(db[7], df[5], cp[3]);                      // dTt/dTp = dTt/dTf dTf/dTp        (:512)
        if (edgeClass == EDGE_DOUBLESIDE) {             // the global block is ds (src/doubleSide.cpp:320-328)
            std::memcpy(cg[0], db[0], sizeof(cg[0]));
            std::memcpy(cg[1], db[1], sizeof(cg[1]));
            std::memcpy(cg[2], db[4], sizeof(cg[2]));
            std::memcpy(cg[3], db[5], sizeof(cg[3]));
        } else {                                        // the camera, as :514-517 chain it (:516 omits
            mat3(db[2], df[2], cg[0]);                  // + dTt/dTf dTf/dRc: hazard A12)
            mat3(db[3], df[7], cg[1]);
            mat3(db[6], df[2], cg[2]);
            mat3(db[7], df[7], cg[3]);
        }
    } else {
        std::memcpy(om, omf, sizeof(om));
        std::memcpy(T, Tf, sizeof(T));
        std::memcpy(cp[0], df[0], sizeof(cp[0]));
        std::memcpy(cp[1], df[1], sizeof(cp[1]));
        std::memcpy(cp[2], df[4], sizeof(cp[2]));
        std::memcpy(cp[3], df[5], sizeof(cp[3]));
        if (edgeClass == EDGE_DOUBLESIDE) {             // FRONT views carry a zero ds block (:335-336)
            for (auto& c : cg) std::memset(c, 0, sizeof(c));
        } else {
            std::memcpy(cg[0], df[2], sizeof(cg[0]));
            std::memcpy(cg[1], df[3], sizeof(cg[1]));
            std::memcpy(cg[2], df[6], sizeof(cg[2]));
            std::memcpy(cg[3], df[7], sizeof(cg[3]));
        }
    }
    for (int k = 0; k < 3; ++k) {
        out.rvecTran[k] = om[k];
        out.tvecTran[k] = T[k];
        out.rvecTranF[k] = (float)om[k];   // Rvectran1 / Tvectran1 -> CV_32F (:546-553)
        out.tvecTranF[k] = (float)T[k];
    }
    // the projected pose: Rodrigues of the float32 vector, in double
    const double rf[3] = {out.rvecTranF[0], out.rvecTranF[1], out.rvecTranF[2]};
    const double tf[3] = {out.tvecTranF[0], out.tvecTranF[1], out.tvecTranF[2]};
    double R[9], Jl[9];
    rot_of(rf, R);
    so3_jac(rf, +1.0, false, Jl);
    double kd[12] = {0};
    for (int q = 0; q < nd && q < 12; ++q) kd[q] = D[q];
    double mt[9];   // the tilted sensor (14 terms, tau != 0)
    const bool tilt = !omni && nd == 14 && (D[12] != 0.f || D[13] != 0.f);
    if (tilt) tilt_of(D[12], D[13], mt);

    out.jacPhoto.assign(12 * (size_t)n, 0.0);
    out.jacGlobal.assign(12 * (size_t)n, 0.0);
    out.E.assign(2 * (size_t)n, 0.0);
    out.proj.assign(2 * (size_t)n, 0.f);
    for (int i = 0; i < n; ++i) {
        float u, v;
        double Yr[3], Dp[6];
        if (omni) omni_point(R, tf, kd, K, (double)xi, obj + 3 * (size_t)i, u, v, Yr, Dp);
        else pinhole_point(R, tf, kd, K, obj + 3 * (size_t)i, u, v, Yr, Dp, tilt ? mt : nullptr);
        out.proj[2 * (size_t)i] = u;
        out.proj[2 * (size_t)i + 1] = v;
        const float eu = img[2 * (size_t)i] - u, ev = img[2 * (size_t)i + 1] - v;   // fl32(obs - proj)
        out.E[2 * (size_t)i] = eu;
        out.E[2 * (size_t)i + 1] = ev;
        // projectPoints' columns for the pose: d/dr = -D [R X]x Jl(r), d/dt = D
        const double yx[9] = {0, Yr[2], -Yr[1], -Yr[2], 0, Yr[0], Yr[1], -Yr[0], 0};   // -[R X]x
        for (int row = 0; row < 2; ++row) {
            const double* d = Dp + 3 * row;
            double jr[3], jt[3] = {d[0], d[1], d[2]}, dy[3];
            for (int j = 0; j < 3; ++j) dy[j] = d[0] * yx[j] + d[1] * yx[3 + j] + d[2] * yx[6 + j];
            for (int j = 0; j < 3; ++j) jr[j] = dy[0] * Jl[j] + dy[1] * Jl[3 + j] + dy[2] * Jl[6 + j];
            // dx/dq = jacobian.colRange(0, 3) * dRt/dq + jacobian.colRange(3, 6) * dTt/dq (:588-604)
            double* jp = out.jacPhoto.data() + 6 * (2 * (size_t)i + row);
            double* jg = out.jacGlobal.data() + 6 * (2 * (size_t)i + row);
            for (int j = 0; j < 3; ++j) {
                jp[j] = jr[0] * cp[0][j] + jr[1] * cp[0][3 + j] + jr[2] * cp[0][6 + j] +
                        (jt[0] * cp[2][j] + jt[1] * cp[2][3 + j] + jt[2] * cp[2][6 + j]);
                jp[3 + j] = jr[0] * cp[1][j] + jr[1] * cp[1][3 + j] + jr[2] * cp[1][6 + j] +
                            (jt[0] * cp[3][j] + jt[1] * cp[3][3 + j] + jt[2] * cp[3][6 + j]);
                jg[j] = jr[0] * cg[0][j] + jr[1] * cg[0][3 + j] + jr[2] * cg[0][6 + j] +
                        (jt[0] * cg[2][j] + jt[1] * cg[2][3 + j] + jt[2] * cg[2][6 + j]);
                jg[3 + j] = jr[0] * cg[1][j] + jr[1] * cg[1][3 + j] + jr[2] * cg[1][6 + j] +
                            (jt[0] * cg[3][j] + jt[1] * cg[3][3 + j] + jt[2] * cg[3][6 + j]);
            }
        }
    }
}

}  // namespace multicalib
}  // namespace mcc

// C entry of edgeJacobian for non-C++ callers (ctypes: tests/test_edge_jacobian.py): 0, or
// MCC_EINVAL for arguments the reference's per-edge Jacobian does not accept
extern "C" int mcc_host_edge_jacobian(int edge_class, int omni, int pattern_side, const double* rP, const double* tP,
                                      const double* rC, const double* tC, const double* rDs, const double* tDs, int n,
                                      const float* obj, const float* img, const float* K, const float* D, int nd,
                                      float xi, double* jac_photo, double* jac_global, double* E, float* pose_f32) {
    try {
        mcc::multicalib::EdgeLinearization L;
        mcc::multicalib::edgeJacobian(edge_class, omni != 0, pattern_side, rP, tP, rC, tC, rDs, tDs, n, obj, img, K, D,
                                      nd, xi, L);
        if (jac_photo) std::memcpy(jac_photo, L.jacPhoto.data(), L.jacPhoto.size() * sizeof(double));
        if (jac_global) std::memcpy(jac_global, L.jacGlobal.data(), L.jacGlobal.size() * sizeof(double));
        if (E) std::memcpy(E, L.E.data(), L.E.size() * sizeof(double));
        if (pose_f32) {
            std::memcpy(pose_f32, L.rvecTranF, 3 * sizeof(float));
            std::memcpy(pose_f32 + 3, L.tvecTranF, 3 * sizeof(float));
        }
        return MCC_OK;
    } catch (const std::exception&) {
        return MCC_EINVAL;
    }
}
