/*
 * mcc_oracle.c -- CPU restatement of the reference BA hot path (TEST INFRASTRUCTURE ONLY).
 * See mcc_oracle.h for the header comment, the reference file:line map and the rules on who
 * may call this code.  Every function cites the reference code (or the OpenCV 4.x formula it
 * follows).  Arithmetic order mirrors the reference where it is observable (float32 rounding
 * points F1-F8 / M1-M7 of SURVEY.md Appendix B); built with -ffp-contract=off.
 */
#include "mcc_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

int ora_num_threads(void)
{
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* ------------------------------------------------------------------ small dense helpers */

/* C(m x n) = A(m x k) * B(k x n), row-major, k summed left to right (OpenCV gemmImpl's
 * small-matrix branch for k = 2..4 and its generic single-thread loop order otherwise). */
static void mm(const double *A, const double *B, double *C, int m, int k, int n)
{
    for (int i = 0; i < m; ++i)
        for (int j = 0; j < n; ++j) {
            double s = A[i * k] * B[j];
            for (int t = 1; t < k; ++t) s = s + A[i * k + t] * B[t * n + j];
            C[i * n + j] = s;
        }
}

static void transpose(const double *A, double *At, int m, int n)
{
    for (int i = 0; i < m; ++i)
        for (int j = 0; j < n; ++j) At[j * m + i] = A[i * n + j];
}

/* float32 3x3 * 3xn gemm, OpenCV gemmImpl small branch (len == 3, CV_32F):
 * t = a0*b0 + a1*b1 + a2*b2 in float, then d = (float)(t*alpha + c*beta) in double. */
static void mm3f(const float *A, const float *B, float *C, int n, const float *Cadd)
{
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < n; ++j) {
            float t = A[i * 3] * B[j];
            t = t + A[i * 3 + 1] * B[n + j];
            t = t + A[i * 3 + 2] * B[2 * n + j];
            double c = Cadd ? (double)Cadd[i * n + j] : 0.0;
            C[i * n + j] = (float)((double)t * 1.0 + c * (Cadd ? 1.0 : 0.0));
        }
}

/* float32 4x4 gemm, OpenCV gemmImpl small branch (len == 4, CV_32F). */
static void mm4f(const float *A, const float *B, float *C)
{
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            float t = A[i * 4] * B[j];
            t = t + A[i * 4 + 1] * B[4 + j];
            t = t + A[i * 4 + 2] * B[8 + j];
            t = t + A[i * 4 + 3] * B[12 + j];
            C[i * 4 + j] = (float)((double)t * 1.0);
        }
}

static double det3(const double *A)
{
    return A[0] * (A[4] * A[8] - A[5] * A[7]) - A[1] * (A[3] * A[8] - A[5] * A[6]) +
           A[2] * (A[3] * A[7] - A[4] * A[6]);
}

/* Polar factor U*Vt of a 3x3 matrix (what cvRodrigues2 obtains from SVD::compute + U*Vt
 * before extracting the rotation vector).  Newton iteration X <- (X + X^-T)/2 converges
 * quadratically to the same factor for det > 0. */
static void polar3(const double *Rin, double *R)
{
    memcpy(R, Rin, 9 * sizeof(double));
    for (int it = 0; it < 40; ++it) {
        double d = det3(R);
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
        for (int k = 0; k < 9; ++k) {
            double v = 0.5 * (R[k] + cof[k] / d);   /* inverse-transpose = cofactor / det */
            double df = fabs(v - R[k]);
            if (df > delta) delta = df;
            R[k] = v;
        }
        if (delta < 1e-15) break;
    }
}

/* ------------------------------------------------------------------ Rodrigues (OpenCV) */

void ora_rodrigues_v2m(const double rin[3], double R[9], double J[27])
{
    /* cvRodrigues2 vector -> matrix (OpenCV 4.x calib3d/src/calibration.cpp). */
    double rx = rin[0], ry = rin[1], rz = rin[2];
    double theta = sqrt(rx * rx + ry * ry + rz * rz);
    if (theta < DBL_EPSILON) {
        static const double I9[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
        memcpy(R, I9, sizeof(I9));
        if (J) {
            memset(J, 0, 27 * sizeof(double));
            J[5] = J[15] = J[19] = -1;
            J[7] = J[11] = J[21] = 1;
        }
        return;
    }
    double c = cos(theta), s = sin(theta), c1 = 1. - c;
    double itheta = theta ? 1. / theta : 0.;
    rx *= itheta; ry *= itheta; rz *= itheta;
    double rrt[9] = {rx * rx, rx * ry, rx * rz, rx * ry, ry * ry, ry * rz, rx * rz, ry * rz, rz * rz};
    double r_x[9] = {0, -rz, ry, rz, 0, -rx, -ry, rx, 0};
    static const double I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    for (int k = 0; k < 9; ++k) R[k] = c * I[k] + c1 * rrt[k] + s * r_x[k];
    if (J) {
        double drrt[27] = {rx + rx, ry, rz, ry, 0, 0, rz, 0, 0,
                           0, rx, 0, rx, ry + ry, rz, 0, rz, 0,
                           0, 0, rx, 0, 0, ry, rx, ry, rz + rz};
        static const double d_r_x_[27] = {0, 0, 0, 0, 0, -1, 0, 1, 0,
                                          0, 0, 1, 0, 0, 0, -1, 0, 0,
                                          0, -1, 0, 1, 0, 0, 0, 0, 0};
        for (int i = 0; i < 3; ++i) {
            double ri = i == 0 ? rx : i == 1 ? ry : rz;
            double a0 = -s * ri, a1 = (s - 2 * c1 * itheta) * ri, a2 = c1 * itheta;
            double a3 = (c - s * itheta) * ri, a4 = s * itheta;
            for (int k = 0; k < 9; ++k)
                J[i * 9 + k] = a0 * I[k] + a1 * rrt[k] + a2 * drrt[i * 9 + k] + a3 * r_x[k] +
                               a4 * d_r_x_[i * 9 + k];
        }
    }
}

void ora_rodrigues_m2v(const double Rin[9], double rout[3], double Jout[27])
{
    /* cvRodrigues2 matrix -> vector (OpenCV 4.x); jacobian returned 9x3 (the C++ API
     * creates Size(3,9) and transposes the internal 3x9). */
    double R[9];
    polar3(Rin, R);
    double rx = R[7] - R[5], ry = R[2] - R[6], rz = R[3] - R[1];
    double s = sqrt((rx * rx + ry * ry + rz * rz) * 0.25);
    double c = (R[0] + R[4] + R[8] - 1) * 0.5;
    c = c > 1. ? 1. : c < -1. ? -1. : c;
    double theta = acos(c);
    double J[27];
    memset(J, 0, sizeof(J));
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
        if (c > 0) {
            J[5] = J[15] = J[19] = -0.5;
            J[7] = J[11] = J[21] = 0.5;
        }
    } else {
        double vth = 1 / (2 * s);
        double dtheta_dtr = -1. / s;
        double dvth_dtheta = -vth * c / s;
        double d1 = 0.5 * dvth_dtheta * dtheta_dtr;
        double d2 = 0.5 * dtheta_dtr;
        double dvardR[45] = {0, 0, 0, 0, 0, 1, 0, -1, 0,
                             0, 0, -1, 0, 0, 0, 1, 0, 0,
                             0, 1, 0, -1, 0, 0, 0, 0, 0,
                             d1, 0, 0, 0, d1, 0, 0, 0, d1,
                             d2, 0, 0, 0, d2, 0, 0, 0, d2};
        double dvar2dvar[20] = {vth, 0, 0, rx, 0,
                                0, vth, 0, ry, 0,
                                0, 0, vth, rz, 0,
                                0, 0, 0, 0, 1};
        double domegadvar2[12] = {theta, 0, 0, rx * vth,
                                  0, theta, 0, ry * vth,
                                  0, 0, theta, rz * vth};
        double t0[15];
        mm(domegadvar2, dvar2dvar, t0, 3, 4, 5);
        mm(t0, dvardR, J, 3, 5, 9);
        double t;
#define SWP(a, b) (t = J[a], J[a] = J[b], J[b] = t)
        SWP(1, 3); SWP(2, 6); SWP(5, 7);
        SWP(10, 12); SWP(11, 15); SWP(14, 16);
        SWP(19, 21); SWP(20, 24); SWP(23, 25);
#undef SWP
        vth *= theta;
        rx *= vth; ry *= vth; rz *= vth;
    }
    rout[0] = rx; rout[1] = ry; rout[2] = rz;
    if (Jout) transpose(J, Jout, 3, 9); /* 9x3 */
}

/* cv::matMulDeriv(A (m x n), B (n x p)): dABdA ((m*p) x (m*n)), dABdB ((m*p) x (n*p)). */
static void matmul_deriv(const double *A, const double *B, int m, int n, int p,
                         double *dABdA, double *dABdB)
{
    memset(dABdA, 0, (size_t)m * p * m * n * sizeof(double));
    memset(dABdB, 0, (size_t)m * p * n * p * sizeof(double));
    for (int i = 0; i < m; ++i)
        for (int j = 0; j < p; ++j) {
            double *dcda = dABdA + (size_t)(i * p + j) * (m * n);
            double *dcdb = dABdB + (size_t)(i * p + j) * (n * p);
            for (int k = 0; k < n; ++k) {
                dcda[i * n + k] = B[k * p + j];
                dcdb[k * p + j] = A[i * n + k];
            }
        }
}

/* ------------------------------------------------------------------ compose_motion */

void ora_compose_motion(const double om1[3], const double T1[3], const double om2[3],
                        const double T2[3], double om3[3], double T3[3], double d[8][9])
{
    /* src/multicalib.cpp:1008-1056 */
    double R1[9], R2[9], R3[9], dR1dom1_39[27], dR2dom2_39[27], dR1dom1[27], dR2dom2[27];
    ora_rodrigues_v2m(om1, R1, dR1dom1_39);
    ora_rodrigues_v2m(om2, R2, dR2dom2_39);
    transpose(dR1dom1_39, dR1dom1, 3, 9); /* dR1dom1 = dR1dom1.t()  (9x3) */
    transpose(dR2dom2_39, dR2dom2, 3, 9);
    mm(R2, R1, R3, 3, 3, 3); /* R3 = R2 * R1 */
    double dR3dR2[81], dR3dR1[81];
    matmul_deriv(R2, R1, 3, 3, 3, dR3dR2, dR3dR1);
    double dom3dR3_93[27], dom3dR3[27];
    ora_rodrigues_m2v(R3, om3, dom3dR3_93);
    transpose(dom3dR3_93, dom3dR3, 9, 3); /* dom3dR3 = dom3dR3.t()  (3x9) */
    double tmp[27];
    mm(dom3dR3, dR3dR1, tmp, 3, 9, 9);
    mm(tmp, dR1dom1, d[0], 3, 9, 3);  /* dom3dom1 */
    mm(dom3dR3, dR3dR2, tmp, 3, 9, 9);
    mm(tmp, dR2dom2, d[2], 3, 9, 3);  /* dom3dom2 */
    memset(d[1], 0, 9 * sizeof(double)); /* dom3dT1 */
    memset(d[3], 0, 9 * sizeof(double)); /* dom3dT2 */
    double T3t[3];
    mm(R2, T1, T3t, 3, 3, 1);          /* T3t = R2 * T1 */
    double dT3tdR2[27], dT3tdT1[9];
    matmul_deriv(R2, T1, 3, 3, 1, dT3tdR2, dT3tdT1);
    mm(dT3tdR2, dR2dom2, d[6], 3, 9, 3); /* dT3dom2 = dT3tdR2 * dR2dom2 */
    for (int i = 0; i < 3; ++i) T3[i] = T3t[i] + T2[i];
    memcpy(d[5], dT3tdT1, 9 * sizeof(double));    /* dT3dT1 */
    static const double I9[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    memcpy(d[7], I9, sizeof(I9));                /* dT3dT2 */
    memset(d[4], 0, 9 * sizeof(double));          /* dT3dom1 */
}

/* ------------------------------------------------------------------ projection models */

/* computeTiltProjectionMatrix (OpenCV calib3d distortion_model.hpp): matTilt = matProjZ * matRotXY,
 * matRotXY = matRotY(tauY) * matRotX(tauX), matProjZ = [[r22, 0, -r02], [0, r22, -r12], [0, 0, 1]]
 * (r = matRotXY); cv::Matx products sum from 0, left to right. */
void ora_tilt_matrix(double tauX, double tauY, double M[9])
{
    double cTauX = cos(tauX), sTauX = sin(tauX), cTauY = cos(tauY), sTauY = sin(tauY);
    double rx[9] = {1, 0, 0, 0, cTauX, sTauX, 0, -sTauX, cTauX};
    double ry[9] = {cTauY, 0, -sTauY, 0, 1, 0, sTauY, 0, cTauY};
    double rxy[9], pz[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double s = 0;
            for (int q = 0; q < 3; ++q) s += ry[3 * i + q] * rx[3 * q + j];
            rxy[3 * i + j] = s;
        }
    pz[0] = rxy[8]; pz[1] = 0; pz[2] = -rxy[2];
    pz[3] = 0; pz[4] = rxy[8]; pz[5] = -rxy[5];
    pz[6] = 0; pz[7] = 0; pz[8] = 1;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double s = 0;
            for (int q = 0; q < 3; ++q) s += pz[3 * i + q] * rxy[3 * q + j];
            M[3 * i + j] = s;
        }
}

int ora_project_pinhole(int n, const float *obj, const float rvec[3], const float tvec[3],
                        const float Kf[9], const float *Df, int nd, float *img, double *jac)
{
    /* cv::projectPoints -> cvProjectPoints2Internal (OpenCV 4.x), aspectRatio = 0.  With 14
     * coefficients the tilted-sensor projection follows the distortion: vecTilt = matTilt *
     * (xd0, yd0, 1), invProj = 1 / vecTilt(2), (xd, yd) = invProj * vecTilt(0..1); the derivatives
     * pass through dMatTilt(r, c) = (matTilt(r, c) vecTilt(2) - matTilt(2, c) vecTilt(r)) invProj^2. */
    double k[14] = {0};
    for (int i = 0; i < nd && i < 14; ++i) k[i] = Df[i];
    double mt[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    if (nd == 14) ora_tilt_matrix(k[12], k[13], mt);
    double r[3] = {rvec[0], rvec[1], rvec[2]}, t[3] = {tvec[0], tvec[1], tvec[2]};
    double R[9], dRdr[27];
    ora_rodrigues_v2m(r, R, dRdr);
    double fx = Kf[0], fy = Kf[4], cx = Kf[2], cy = Kf[5];
    for (int i = 0; i < n; ++i) {
        double X = obj[3 * i], Y = obj[3 * i + 1], Z = obj[3 * i + 2];
        double x = R[0] * X + R[1] * Y + R[2] * Z + t[0];
        double y = R[3] * X + R[4] * Y + R[5] * Z + t[1];
        double z = R[6] * X + R[7] * Y + R[8] * Z + t[2];
        z = z ? 1. / z : 1;
        x *= z; y *= z;
        double r2 = x * x + y * y, r4 = r2 * r2, r6 = r4 * r2;
        double a1 = 2 * x * y, a2 = r2 + 2 * x * x, a3 = r2 + 2 * y * y;
        double cdist = 1 + k[0] * r2 + k[1] * r4 + k[4] * r6;
        double icdist2 = 1. / (1 + k[5] * r2 + k[6] * r4 + k[7] * r6);
        double xd0 = x * cdist * icdist2 + k[2] * a1 + k[3] * a2 + k[8] * r2 + k[9] * r4;
        double yd0 = y * cdist * icdist2 + k[2] * a3 + k[3] * a1 + k[10] * r2 + k[11] * r4;
        double vt0 = 0, vt1 = 0, vt2 = 0;
        vt0 += mt[0] * xd0; vt0 += mt[1] * yd0; vt0 += mt[2] * 1.0;
        vt1 += mt[3] * xd0; vt1 += mt[4] * yd0; vt1 += mt[5] * 1.0;
        vt2 += mt[6] * xd0; vt2 += mt[7] * yd0; vt2 += mt[8] * 1.0;
        double invProj = vt2 ? 1. / vt2 : 1;
        double xd = invProj * vt0, yd = invProj * vt1;
        double dmt[4];   /* dMatTilt (2 x 2, row-major) */
        for (int row = 0; row < 2; ++row)
            for (int col = 0; col < 2; ++col)
                dmt[2 * row + col] = mt[3 * row + col] * vt2 - mt[6 + col] * (row ? vt1 : vt0);
        double ips = invProj * invProj;
        for (int q = 0; q < 4; ++q) dmt[q] *= ips;
        img[2 * i] = (float)(xd * fx + cx);
        img[2 * i + 1] = (float)(yd * fy + cy);
        if (jac) {
            double *ju = jac + (size_t)(2 * i) * 6, *jv = ju + 6;
            double dx0dr[3], dy0dr[3], dz0dr[3];
            for (int j = 0; j < 3; ++j) {
                dx0dr[j] = X * dRdr[j * 9 + 0] + Y * dRdr[j * 9 + 1] + Z * dRdr[j * 9 + 2];
                dy0dr[j] = X * dRdr[j * 9 + 3] + Y * dRdr[j * 9 + 4] + Z * dRdr[j * 9 + 5];
                dz0dr[j] = X * dRdr[j * 9 + 6] + Y * dRdr[j * 9 + 7] + Z * dRdr[j * 9 + 8];
            }
            for (int j = 0; j < 3; ++j) {
                double dxdr = z * (dx0dr[j] - x * dz0dr[j]);
                double dydr = z * (dy0dr[j] - y * dz0dr[j]);
                double dr2dr = 2 * x * dxdr + 2 * y * dydr;
                double dcdist_dr = (k[0] + 2 * k[1] * r2 + 3 * k[4] * r4) * dr2dr;
                double dicdist2_dr = -icdist2 * icdist2 * (k[5] + 2 * k[6] * r2 + 3 * k[7] * r4) * dr2dr;
                double da1dr = 2 * (x * dydr + y * dxdr);
                double dmxdr = (dxdr * cdist * icdist2 + x * dcdist_dr * icdist2 + x * cdist * dicdist2_dr +
                                k[2] * da1dr + k[3] * (dr2dr + 4 * x * dxdr) + (k[8] + 2 * r2 * k[9]) * dr2dr);
                double dmydr = (dydr * cdist * icdist2 + y * dcdist_dr * icdist2 + y * cdist * dicdist2_dr +
                                k[2] * (dr2dr + 4 * y * dydr) + k[3] * da1dr + (k[10] + 2 * r2 * k[11]) * dr2dr);
                ju[j] = fx * (dmt[0] * dmxdr + dmt[1] * dmydr);
                jv[j] = fy * (dmt[2] * dmxdr + dmt[3] * dmydr);
            }
            double dxdt[3] = {z, 0, -x * z}, dydt[3] = {0, z, -y * z};
            for (int j = 0; j < 3; ++j) {
                double dr2dt = 2 * x * dxdt[j] + 2 * y * dydt[j];
                double dcdist_dt = (k[0] + 2 * k[1] * r2 + 3 * k[4] * r4) * dr2dt;
                double dicdist2_dt = -icdist2 * icdist2 * (k[5] + 2 * k[6] * r2 + 3 * k[7] * r4) * dr2dt;
                double da1dt = 2 * (x * dydt[j] + y * dxdt[j]);
                double dmxdt = (dxdt[j] * cdist * icdist2 + x * dcdist_dt * icdist2 + x * cdist * dicdist2_dt +
                                k[2] * da1dt + k[3] * (dr2dt + 4 * x * dxdt[j]) + (k[8] + 2 * r2 * k[9]) * dr2dt);
                double dmydt = (dydt[j] * cdist * icdist2 + y * dcdist_dt * icdist2 + y * cdist * dicdist2_dt +
                                k[2] * (dr2dt + 4 * y * dydt[j]) + k[3] * da1dt + (k[10] + 2 * r2 * k[11]) * dr2dt);
                ju[3 + j] = fx * (dmt[0] * dmxdt + dmt[1] * dmydt);
                jv[3 + j] = fy * (dmt[2] * dmxdt + dmt[3] * dmydt);
            }
        }
    }
    return 0;
}

void ora_project_omni(int n, const float *obj, const float rvec[3], const float tvec[3],
                      const float Kf[9], double xi, const float Df[4], float *img, double *jac)
{
    /* src/omnidir.cpp:84-245 (CV_32F object points, CV_32F K and D). */
    double om[3] = {rvec[0], rvec[1], rvec[2]}, T[3] = {tvec[0], tvec[1], tvec[2]};
    double f0 = Kf[0], f1 = Kf[4], c0 = Kf[2], c1 = Kf[5], s = (double)Kf[1];
    double k1 = Df[0], k2 = Df[1], p1 = Df[2], p2 = Df[3];
    double R[9], dRdom[27];
    ora_rodrigues_v2m(om, R, dRdom); /* Rodrigues(om, R, dRdom): Matx<double,3,9> */
    for (int i = 0; i < n; ++i) {
        double Xw[3] = {obj[3 * i], obj[3 * i + 1], obj[3 * i + 2]};
        double Xc[3];
        for (int a = 0; a < 3; ++a) {
            double acc = 0;
            for (int b = 0; b < 3; ++b) acc = acc + R[a * 3 + b] * Xw[b];
            Xc[a] = acc + T[a];
        }
        double nrm = sqrt(0 + Xc[0] * Xc[0] + Xc[1] * Xc[1] + Xc[2] * Xc[2]);
        double inrm = 1. / nrm;
        double Xs[3] = {Xc[0] * inrm, Xc[1] * inrm, Xc[2] * inrm};
        double xu[2] = {Xs[0] / (Xs[2] + xi), Xs[1] / (Xs[2] + xi)};
        double r2 = xu[0] * xu[0] + xu[1] * xu[1];
        double r4 = r2 * r2;
        double xd[2];
        xd[0] = xu[0] * (1 + k1 * r2 + k2 * r4) + 2 * p1 * xu[0] * xu[1] + p2 * (r2 + 2 * xu[0] * xu[0]);
        xd[1] = xu[1] * (1 + k1 * r2 + k2 * r4) + p1 * (r2 + 2 * xu[1] * xu[1]) + 2 * p2 * xu[0] * xu[1];
        double fin0 = f0 * xd[0] + s * xd[1] + c0;
        double fin1 = f1 * xd[1] + c1;
        img[2 * i] = (float)fin0;
        img[2 * i + 1] = (float)fin1;
        if (jac) {
            double dXcdR[27] = {Xw[0], Xw[1], Xw[2], 0, 0, 0, 0, 0, 0,
                                0, 0, 0, Xw[0], Xw[1], Xw[2], 0, 0, 0,
                                0, 0, 0, 0, 0, 0, Xw[0], Xw[1], Xw[2]};
            double dRdomT[27], dXcdom[9];
            transpose(dRdom, dRdomT, 3, 9);
            mm(dXcdR, dRdomT, dXcdom, 3, 9, 3);
            double r_1 = 1.0 / nrm;
            double r_3 = pow(r_1, 3);
            double dXsdXc[9] = {r_1 - Xc[0] * Xc[0] * r_3, -(Xc[0] * Xc[1]) * r_3, -(Xc[0] * Xc[2]) * r_3,
                                -(Xc[0] * Xc[1]) * r_3, r_1 - Xc[1] * Xc[1] * r_3, -(Xc[1] * Xc[2]) * r_3,
                                -(Xc[0] * Xc[2]) * r_3, -(Xc[1] * Xc[2]) * r_3, r_1 - Xc[2] * Xc[2] * r_3};
            double dxudXs[6] = {1 / (Xs[2] + xi), 0, -Xs[0] / (Xs[2] + xi) / (Xs[2] + xi),
                                0, 1 / (Xs[2] + xi), -Xs[1] / (Xs[2] + xi) / (Xs[2] + xi)};
            double temp1 = 2 * k1 * xu[0] + 4 * k2 * xu[0] * r2;
            double temp2 = 2 * k1 * xu[1] + 4 * k2 * xu[1] * r2;
            double dxddxu[4] = {k2 * r4 + 6 * p2 * xu[0] + 2 * p1 * xu[1] + xu[0] * temp1 + k1 * r2 + 1,
                                2 * p1 * xu[0] + 2 * p2 * xu[1] + xu[0] * temp2,
                                2 * p1 * xu[0] + 2 * p2 * xu[1] + xu[1] * temp1,
                                k2 * r4 + 2 * p2 * xu[0] + 6 * p1 * xu[1] + xu[1] * temp2 + k1 * r2 + 1};
            double dxpddxd[4] = {f0, s, 0, f1};
            double t22[4], t23[6], dxpddXc[6], dxpddom[6];
            mm(dxpddxd, dxddxu, t22, 2, 2, 2);
            mm(t22, dxudXs, t23, 2, 2, 3);
            mm(t23, dXsdXc, dxpddXc, 2, 3, 3);
            mm(dxpddXc, dXcdom, dxpddom, 2, 3, 3);
            static const double I3[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
            double dxpddT[6];
            mm(dxpddXc, I3, dxpddT, 2, 3, 3);
            double *ju = jac + (size_t)(2 * i) * 6, *jv = ju + 6;
            for (int j = 0; j < 3; ++j) {
                ju[j] = dxpddom[j];
                jv[j] = dxpddom[3 + j];
                ju[3 + j] = dxpddT[j];
                jv[3 + j] = dxpddT[3 + j];
            }
        }
    }
}

/* ------------------------------------------------------------------ problem layout */

int ora_nparams(const ora_problem *p)
{
    if (p->model == ORA_DOUBLESIDE) return 6 * (1 + p->n_photos);
    return 6 * (p->n_cams - 1 + p->n_photos);
}

int ora_global_dim(const ora_problem *p)
{
    return p->model == ORA_DOUBLESIDE ? 6 : 6 * (p->n_cams - 1);
}

int ora_param_col_photo(const ora_problem *p, int photo)
{
    /* buildParas src/multicalib.cpp:422-440 (vertex v at (v-1)*6, v = C + photo);
     * DoubleSide::buildParas src/doubleSide.cpp:233-261 (ds first, photo at (v-C+1)*6). */
    if (p->model == ORA_DOUBLESIDE) return 6 * (1 + photo);
    return 6 * (p->n_cams - 1 + photo);
}

int ora_param_col_cam(const ora_problem *p, int cam)
{
    if (p->model == ORA_DOUBLESIDE || cam == 0) return -1;
    return 6 * (cam - 1);
}

/* rvec/tvec (float) of a camera vertex as the reference slices them from x. */
static void cam_params(const ora_problem *p, const float *x, int cam, float r[3], float t[3])
{
    if (p->model == ORA_DOUBLESIDE) {
        /* cameraPose2vec src/doubleSide.cpp:262-275: Rodrigues of the float pose -> float. */
        double R[9], rv[3];
        const float *P = p->cam_pose + 16 * cam;
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) R[a * 3 + b] = P[a * 4 + b];
        ora_rodrigues_m2v(R, rv, NULL);
        for (int a = 0; a < 3; ++a) { r[a] = (float)rv[a]; t[a] = P[a * 4 + 3]; }
        return;
    }
    if (cam == 0) { /* src/mymulticalib.cpp:721-725: zeros */
        r[0] = r[1] = r[2] = 0.f;
        t[0] = t[1] = t[2] = 0.f;
        return;
    }
    int c = ora_param_col_cam(p, cam);
    for (int a = 0; a < 3; ++a) { r[a] = x[c + a]; t[a] = x[c + 3 + a]; }
}

/* ------------------------------------------------------------------ edge linearisation */

/* out(2N x 3) = Jr(2N x 3, cols 0..2 of jac) * A + Jt(2N x 3, cols 3..5) * B  (two small
 * gemms then a Mat add, src/mymulticalib.cpp:588-604). */
static void chain_cols(const double *jac, int n2, const double *A, const double *B,
                       double *out, int out_stride, int out_col)
{
    for (int r = 0; r < n2; ++r) {
        const double *a = jac + (size_t)r * 6;
        for (int j = 0; j < 3; ++j) {
            double t1 = a[0] * A[j] + a[1] * A[3 + j] + a[2] * A[6 + j];
            double t2 = a[3] * B[j] + a[4] * B[3 + j] + a[5] * B[6 + j];
            out[(size_t)r * out_stride + out_col + j] = t1 + t2;
        }
    }
}

int ora_edge_linearize(const ora_problem *p, const float *x, int e, double *jc, double *jp,
                       double *E, float *proj)
{
    int cam = p->edge_cam[e], photo = p->edge_photo[e], side = p->edge_side[e];
    int n = p->edge_n[e], off = p->edge_off[e];
    int pc = ora_param_col_photo(p, photo);
    float rp[3], tp[3], rc[3], tc[3];
    for (int a = 0; a < 3; ++a) { rp[a] = x[pc + a]; tp[a] = x[pc + 3 + a]; }
    cam_params(p, x, cam, rc, tc);

    /* compose_motion(photo, camera) -> "photofront"  (src/mymulticalib.cpp:498-500) */
    double om1[3] = {rp[0], rp[1], rp[2]}, T1[3] = {tp[0], tp[1], tp[2]};
    double om2[3] = {rc[0], rc[1], rc[2]}, T2[3] = {tc[0], tc[1], tc[2]};
    double omf[3], Tf[3], df[8][9];
    ora_compose_motion(om1, T1, om2, T2, omf, Tf, df);
    /* df: 0 dRf/dRp 1 dRf/dTp 2 dRf/dRc 3 dRf/dTc 4 dTf/dRp 5 dTf/dTp 6 dTf/dRc 7 dTf/dTc */

    double om[3], T[3];
    /* chain matrices to the composed transform: [dRt/dRp, dRt/dTp, dTt/dRp, dTt/dTp] and the
     * global block [dRt/dRg, dRt/dTg, dTt/dRg, dTt/dTg] (camera, or ds for DoubleSide). */
    double cp[4][9], cg[4][9];
    static const double Z9[9] = {0};
    int have_global = 1;
    if (side == ORA_BACK) {
        double ds_r[3], ds_t[3];
        if (p->model == ORA_DOUBLESIDE) {
            for (int a = 0; a < 3; ++a) { ds_r[a] = x[a]; ds_t[a] = x[3 + a]; } /* float -> double */
        } else {
            if (!p->ds_pose) return -2;
            /* doublesideTransform2vec src/mymulticalib.cpp:105-117 (CV_64F) */
            double R[9];
            for (int a = 0; a < 3; ++a)
                for (int b = 0; b < 3; ++b) R[a * 3 + b] = p->ds_pose[a * 4 + b];
            ora_rodrigues_m2v(R, ds_r, NULL);
            for (int a = 0; a < 3; ++a) ds_t[a] = p->ds_pose[a * 4 + 3];
        }
        double db[8][9];
        /* compose_motion(ds, photofront) src/mymulticalib.cpp:503-506, doubleSide.cpp:319-322 */
        ora_compose_motion(ds_r, ds_t, omf, Tf, om, T, db);
        /* db: 0 dRt/dRds 1 dRt/dTds 2 dRt/dRf 3 dRt/dTf 4 dTt/dRds 5 dTt/dTds 6 dTt/dRf 7 dTt/dTf */
        mm(db[2], df[0], cp[0], 3, 3, 3); /* dRvectran_dRvecPhoto = dRt/dRf * dRf/dRp   (:509) */
        mm(db[3], df[5], cp[1], 3, 3, 3); /* dRvectran_dTvecPhoto = dRt/dTf * dTf/dTp   (:510) */
        mm(db[6], df[0], cp[2], 3, 3, 3); /* dTvectran_dRvecPhoto = dTt/dRf * dRf/dRp   (:511) */
        mm(db[7], df[5], cp[3], 3, 3, 3); /* dTvectran_dTvecPhoto = dTt/dTf * dTf/dTp   (:512) */
        if (p->model == ORA_DOUBLESIDE) {
            memcpy(cg[0], db[0], sizeof(cg[0])); /* dRvectran_dRvecDoubleside */
            memcpy(cg[1], db[1], sizeof(cg[1])); /* dRvectran_dTvecDoubleside */
            memcpy(cg[2], db[4], sizeof(cg[2])); /* dTvectran_dRvecDoubleside */
            memcpy(cg[3], db[5], sizeof(cg[3])); /* dTvectran_dTvecDoubleside */
        } else {
            /* src/mymulticalib.cpp:514-517; :516 omits + dTt/dTf * dTf/dRc (hazard A12). */
            mm(db[2], df[2], cg[0], 3, 3, 3);
            mm(db[3], df[7], cg[1], 3, 3, 3);
            mm(db[6], df[2], cg[2], 3, 3, 3);
            mm(db[7], df[7], cg[3], 3, 3, 3);
        }
    } else {
        memcpy(om, omf, sizeof(om));
        memcpy(T, Tf, sizeof(T));
        memcpy(cp[0], df[0], sizeof(cp[0]));
        memcpy(cp[1], df[1], sizeof(cp[1]));
        memcpy(cp[2], df[4], sizeof(cp[2]));
        memcpy(cp[3], df[5], sizeof(cp[3]));
        if (p->model == ORA_DOUBLESIDE) {
            /* src/doubleSide.cpp:335-336: zero double-side jacobian for the front side */
            for (int k = 0; k < 4; ++k) memcpy(cg[k], Z9, sizeof(Z9));
        } else {
            memcpy(cg[0], df[2], sizeof(cg[0]));
            memcpy(cg[1], df[3], sizeof(cg[1]));
            memcpy(cg[2], df[6], sizeof(cg[2]));
            memcpy(cg[3], df[7], sizeof(cg[3]));
        }
    }
    (void)have_global;

    /* Rvectran1/Tvectran1 -> CV_32F (src/mymulticalib.cpp:546-553) */
    float rf[3] = {(float)om[0], (float)om[1], (float)om[2]};
    float tf[3] = {(float)T[0], (float)T[1], (float)T[2]};

    const float *obj = p->obj + 3 * (size_t)off;
    const float *img = p->img + 2 * (size_t)off;
    double *jac = (double *)malloc(sizeof(double) * 12 * (size_t)n);
    float *pr = (float *)malloc(sizeof(float) * 2 * (size_t)n);
    if (!jac || !pr) { free(jac); free(pr); return -3; }
    if (p->model == ORA_OMNI) {
        ora_project_omni(n, obj, rf, tf, p->K + 9 * cam, (double)p->xi[cam], p->D + p->nd * cam, pr, jac);
    } else {
        if (ora_project_pinhole(n, obj, rf, tf, p->K + 9 * cam, p->D + p->nd * cam, p->nd, pr, jac)) {
            free(jac); free(pr);
            return -4;
        }
    }
    /* E = fl32(imagePoints - imagePoints2) -> CV_64F, reshaped 2N x 1 (:578-586) */
    for (int i = 0; i < 2 * n; ++i) {
        float ef = img[i] - pr[i];
        E[i] = (double)ef;
        if (proj) proj[i] = pr[i];
    }
    chain_cols(jac, 2 * n, cg[0], cg[2], jc, 6, 0); /* dx_dRvecCamera */
    chain_cols(jac, 2 * n, cg[1], cg[3], jc, 6, 3); /* dx_dTvecCamera */
    chain_cols(jac, 2 * n, cp[0], cp[2], jp, 6, 0); /* dx_dRvecPhoto  */
    chain_cols(jac, 2 * n, cp[1], cp[3], jp, 6, 3); /* dx_dTvecPhoto  */
    free(jac);
    free(pr);
    return 0;
}

/* ------------------------------------------------------------------ dense faithful path */

static int global_col(const ora_problem *p, int e)
{
    if (p->model == ORA_DOUBLESIDE) return 0;
    return ora_param_col_cam(p, p->edge_cam[e]);
}

int ora_normal_dense(const ora_problem *p, const float *x, double *JTJ, double *JTE)
{
    /* src/mymulticalib.cpp:668-803: J (2 sum N) x P dense, JTJ = J.t()*J, JTE = J.t()*E. */
    int P = ora_nparams(p);
    memset(JTJ, 0, sizeof(double) * (size_t)P * P);
    memset(JTE, 0, sizeof(double) * (size_t)P);
    int maxn = 0;
    for (int e = 0; e < p->n_edges; ++e) if (p->edge_n[e] > maxn) maxn = p->edge_n[e];
    double *jc = (double *)malloc(sizeof(double) * 12 * (size_t)maxn);
    double *jp = (double *)malloc(sizeof(double) * 12 * (size_t)maxn);
    double *E = (double *)malloc(sizeof(double) * 2 * (size_t)maxn);
    double *row = (double *)malloc(sizeof(double) * (size_t)P);
    int *cols = (int *)malloc(sizeof(int) * 12);
    int rc = 0;
    if (!jc || !jp || !E || !row || !cols) { rc = -3; goto out; }
    for (int e = 0; e < p->n_edges; ++e) {
        if ((rc = ora_edge_linearize(p, x, e, jc, jp, E, NULL))) goto out;
        int gc = global_col(p, e), pc = ora_param_col_photo(p, p->edge_photo[e]);
        int nz = 0;
        if (gc >= 0) for (int j = 0; j < 6; ++j) cols[nz++] = gc + j;
        for (int j = 0; j < 6; ++j) cols[nz++] = pc + j;
        for (int r = 0; r < 2 * p->edge_n[e]; ++r) {
            double v[12];
            int q = 0;
            if (gc >= 0) for (int j = 0; j < 6; ++j) v[q++] = jc[r * 6 + j];
            for (int j = 0; j < 6; ++j) v[q++] = jp[r * 6 + j];
            for (int a = 0; a < nz; ++a) {
                JTE[cols[a]] += v[a] * E[r];
                for (int b = 0; b < nz; ++b) JTJ[(size_t)cols[a] * P + cols[b]] += v[a] * v[b];
            }
        }
    }
out:
    free(jc); free(jp); free(E); free(row); free(cols);
    return rc;
}

int ora_cg(int P, const double *A, const double *b, double *xout)
{
    /* Eigen 3 conjugate_gradient (IterativeLinearSolvers/ConjugateGradient.h) with a Jacobi
     * preconditioner (DiagonalPreconditioner: 1/diag, 1 where diag == 0), x0 = 0,
     * tol = NumTraits<double>::epsilon(), maxIters = 2*cols.  sparseSolver calls solve()
     * twice with identical inputs (src/multicalib.cpp:573,577): the second result is returned. */
    double *x = xout;
    double *res = (double *)malloc(sizeof(double) * P * 4);
    double *pdir = res + P, *z = pdir + P, *tmp = z + P;
    double *invd = (double *)malloc(sizeof(double) * P);
    int iters = 0;
    for (int i = 0; i < P; ++i) {
        double d = A[(size_t)i * P + i];
        invd[i] = d == 0 ? 1.0 : 1.0 / d;
    }
    for (int pass = 0; pass < 2; ++pass) {
        const double tol = DBL_EPSILON;
        int maxIters = 2 * P;
        for (int i = 0; i < P; ++i) x[i] = 0;
        for (int i = 0; i < P; ++i) res[i] = b[i]; /* residual = rhs - A*0 */
        double rhsNorm2 = 0;
        for (int i = 0; i < P; ++i) rhsNorm2 += b[i] * b[i];
        if (rhsNorm2 == 0) { iters = 0; continue; }
        double considerAsZero = DBL_MIN;
        double threshold = tol * tol * rhsNorm2;
        if (threshold < considerAsZero) threshold = considerAsZero;
        double residualNorm2 = 0;
        for (int i = 0; i < P; ++i) residualNorm2 += res[i] * res[i];
        if (residualNorm2 < threshold) { iters = 0; continue; }
        for (int i = 0; i < P; ++i) pdir[i] = invd[i] * res[i];
        double absNew = 0;
        for (int i = 0; i < P; ++i) absNew += res[i] * pdir[i];
        int it = 0;
        while (it < maxIters) {
            for (int i = 0; i < P; ++i) {
                double s = 0;
                const double *Ai = A + (size_t)i * P;
                for (int j = 0; j < P; ++j) s += Ai[j] * pdir[j];
                tmp[i] = s;
            }
            double pt = 0;
            for (int i = 0; i < P; ++i) pt += pdir[i] * tmp[i];
            double alpha = absNew / pt;
            for (int i = 0; i < P; ++i) x[i] += alpha * pdir[i];
            for (int i = 0; i < P; ++i) res[i] -= alpha * tmp[i];
            residualNorm2 = 0;
            for (int i = 0; i < P; ++i) residualNorm2 += res[i] * res[i];
            if (residualNorm2 < threshold) break;
            for (int i = 0; i < P; ++i) z[i] = invd[i] * res[i];
            double absOld = absNew;
            absNew = 0;
            for (int i = 0; i < P; ++i) absNew += res[i] * z[i];
            double beta = absNew / absOld;
            for (int i = 0; i < P; ++i) pdir[i] = z[i] + beta * pdir[i];
            it++;
        }
        iters = it;
    }
    free(res);
    free(invd);
    return iters;
}

/* ------------------------------------------------------------------ block-sparse exact path */

/* per-edge blocks: Hgg (6x6), Hpp (6x6), Hgp (6x6), gg (6), gp (6) */
typedef struct { double Hgg[36], Hpp[36], Hgp[36], gg[6], gp[6]; } edge_blk;

static int edge_blocks(const ora_problem *p, const float *x, int e, edge_blk *b, double *wk)
{
    int n = p->edge_n[e];
    double *jc = wk, *jp = wk + 12 * (size_t)n, *E = wk + 24 * (size_t)n;
    int rc = ora_edge_linearize(p, x, e, jc, jp, E, NULL);
    if (rc) return rc;
    memset(b, 0, sizeof(*b));
    for (int r = 0; r < 2 * n; ++r) {
        const double *c = jc + r * 6, *q = jp + r * 6;
        for (int a = 0; a < 6; ++a) {
            b->gg[a] += c[a] * E[r];
            b->gp[a] += q[a] * E[r];
            for (int k = 0; k < 6; ++k) {
                b->Hgg[a * 6 + k] += c[a] * c[k];
                b->Hpp[a * 6 + k] += q[a] * q[k];
                b->Hgp[a * 6 + k] += c[a] * q[k];
            }
        }
    }
    return 0;
}

/* Cholesky A = L L^T in place (lower), n x n. Returns nonzero if not positive definite. */
static int cholesky(double *A, int n)
{
    for (int j = 0; j < n; ++j) {
        double s = A[j * n + j];
        for (int k = 0; k < j; ++k) s -= A[j * n + k] * A[j * n + k];
        if (!(s > 0)) return -1;
        double l = sqrt(s);
        A[j * n + j] = l;
        for (int i = j + 1; i < n; ++i) {
            double t = A[i * n + j];
            for (int k = 0; k < j; ++k) t -= A[i * n + k] * A[j * n + k];
            A[i * n + j] = t / l;
        }
        for (int i = 0; i < j; ++i) A[i * n + j] = 0;
    }
    return 0;
}

static void chol_solve(const double *L, int n, double *b)
{
    for (int i = 0; i < n; ++i) {
        double s = b[i];
        for (int k = 0; k < i; ++k) s -= L[i * n + k] * b[k];
        b[i] = s / L[i * n + i];
    }
    for (int i = n - 1; i >= 0; --i) {
        double s = b[i];
        for (int k = i + 1; k < n; ++k) s -= L[k * n + i] * b[k];
        b[i] = s / L[i * n + i];
    }
}

typedef struct {
    int *ptr, *idx;     /* photo -> edges CSR, edges in reference order */
    edge_blk *blk;      /* per edge */
} sparse_ws;

static int build_ws(const ora_problem *p, const float *x, sparse_ws *w)
{
    int V = p->n_photos, E = p->n_edges;
    w->ptr = (int *)calloc((size_t)V + 1, sizeof(int));
    w->idx = (int *)malloc(sizeof(int) * (size_t)(E ? E : 1));
    w->blk = (edge_blk *)malloc(sizeof(edge_blk) * (size_t)(E ? E : 1));
    if (!w->ptr || !w->idx || !w->blk) return -3;
    for (int e = 0; e < E; ++e) w->ptr[p->edge_photo[e] + 1]++;
    for (int v = 0; v < V; ++v) w->ptr[v + 1] += w->ptr[v];
    int *fill = (int *)calloc((size_t)V, sizeof(int));
    for (int e = 0; e < E; ++e) {
        int v = p->edge_photo[e];
        w->idx[w->ptr[v] + fill[v]++] = e;
    }
    free(fill);
    int maxn = 0;
    for (int e = 0; e < E; ++e) if (p->edge_n[e] > maxn) maxn = p->edge_n[e];
    int rc = 0;
#pragma omp parallel
    {
        double *wk = (double *)malloc(sizeof(double) * 26 * (size_t)(maxn ? maxn : 1));
#pragma omp for schedule(dynamic, 16)
        for (int e = 0; e < E; ++e) {
            int r = edge_blocks(p, x, e, &w->blk[e], wk);
            if (r) {
#pragma omp critical
                rc = r;
            }
        }
        free(wk);
    }
    return rc;
}

static void free_ws(sparse_ws *w)
{
    free(w->ptr); free(w->idx); free(w->blk);
}

/* global block index (0-based block of 6) of an edge, or -1 */
static int gblock(const ora_problem *p, int e)
{
    if (p->model == ORA_DOUBLESIDE) return 0;
    return p->edge_cam[e] - 1;
}

/* Per photo: Hpp = sum, L = chol(Hpp); for each edge Y_e = Hgp_e * Hpp^-1 (6x6), w = Hpp^-1 gp */
static int photo_reduce(const ora_problem *p, const sparse_ws *w, int v, double *S, double *r,
                        int m, double *Lout, double *zout)
{
    double Hpp[36] = {0}, gp[6] = {0};
    for (int q = w->ptr[v]; q < w->ptr[v + 1]; ++q) {
        const edge_blk *b = &w->blk[w->idx[q]];
        for (int k = 0; k < 36; ++k) Hpp[k] += b->Hpp[k];
        for (int k = 0; k < 6; ++k) gp[k] += b->gp[k];
    }
    double L[36];
    memcpy(L, Hpp, sizeof(L));
    if (cholesky(L, 6)) return -5;
    if (Lout) memcpy(Lout, L, sizeof(L));
    double z[6];
    memcpy(z, gp, sizeof(z));
    chol_solve(L, 6, z); /* Hpp^-1 gp */
    if (zout) memcpy(zout, z, sizeof(z));
    int ne = w->ptr[v + 1] - w->ptr[v];
    double *Y = (double *)malloc(sizeof(double) * 36 * (size_t)(ne ? ne : 1));
    for (int a = 0; a < ne; ++a) {
        const edge_blk *b = &w->blk[w->idx[w->ptr[v] + a]];
        /* Y = Hgp * Hpp^-1 : solve Hpp Y^T = Hgp^T row by row */
        for (int i = 0; i < 6; ++i) {
            double rowv[6];
            for (int k = 0; k < 6; ++k) rowv[k] = b->Hgp[i * 6 + k];
            chol_solve(L, 6, rowv);
            for (int k = 0; k < 6; ++k) Y[a * 36 + i * 6 + k] = rowv[k];
        }
    }
    for (int a = 0; a < ne; ++a) {
        int ea = w->idx[w->ptr[v] + a], ga = gblock(p, ea);
        if (ga < 0) continue;
        const edge_blk *ba = &w->blk[ea];
        for (int i = 0; i < 6; ++i) {
            double acc = ba->gg[i];
            for (int k = 0; k < 6; ++k) acc -= Y[a * 36 + i * 6 + k] * gp[k];
            r[ga * 6 + i] += acc;
            for (int j = 0; j < 6; ++j) S[(size_t)(ga * 6 + i) * m + ga * 6 + j] += ba->Hgg[i * 6 + j];
        }
        for (int b2 = 0; b2 < ne; ++b2) {
            int eb = w->idx[w->ptr[v] + b2], gbk = gblock(p, eb);
            if (gbk < 0) continue;
            const edge_blk *bb = &w->blk[eb];
            /* S[ga,gb] -= Y_a * Hgp_b^T */
            for (int i = 0; i < 6; ++i)
                for (int j = 0; j < 6; ++j) {
                    double acc = 0;
                    for (int k = 0; k < 6; ++k) acc += Y[a * 36 + i * 6 + k] * bb->Hgp[j * 6 + k];
                    S[(size_t)(ga * 6 + i) * m + gbk * 6 + j] -= acc;
                }
        }
    }
    free(Y);
    return 0;
}

int ora_schur_partial(const ora_problem *p, const float *x, int lo, int hi, double *S, double *r)
{
    int m = ora_global_dim(p);
    memset(S, 0, sizeof(double) * (size_t)m * m);
    memset(r, 0, sizeof(double) * (size_t)m);
    sparse_ws w;
    int rc = build_ws(p, x, &w);
    if (!rc)
        for (int v = lo; v < hi && !rc; ++v) rc = photo_reduce(p, &w, v, S, r, m, NULL, NULL);
    free_ws(&w);
    return rc;
}

static int solve_schur(const ora_problem *p, const float *x, double *delta, double *jte)
{
    int m = ora_global_dim(p), V = p->n_photos;
    sparse_ws w;
    int rc = build_ws(p, x, &w);
    double *S = (double *)calloc((size_t)m * m + 1, sizeof(double));
    double *r = (double *)calloc((size_t)m + 1, sizeof(double));
    double *L = (double *)malloc(sizeof(double) * 36 * (size_t)(V ? V : 1));
    double *z = (double *)malloc(sizeof(double) * 6 * (size_t)(V ? V : 1));
    if (rc) goto out;
    for (int v = 0; v < V && !rc; ++v) rc = photo_reduce(p, &w, v, S, r, m, L + 36 * v, z + 6 * v);
    if (rc) goto out;
    if (jte) {
        memset(jte, 0, sizeof(double) * (size_t)ora_nparams(p));
        for (int e = 0; e < p->n_edges; ++e) {
            int g = gblock(p, e), pc = ora_param_col_photo(p, p->edge_photo[e]);
            for (int k = 0; k < 6; ++k) {
                if (g >= 0) jte[g * 6 + k] += w.blk[e].gg[k];
                jte[pc + k] += w.blk[e].gp[k];
            }
        }
    }
    if (cholesky(S, m)) { rc = -6; goto out; }
    chol_solve(S, m, r);
    for (int i = 0; i < m; ++i) delta[i] = r[i];
    /* back-substitution: dp = Hpp^-1 (gp - sum Hgp^T dg) = z - Hpp^-1 sum Hgp^T dg */
    for (int v = 0; v < V; ++v) {
        double t[6] = {0};
        for (int q = w.ptr[v]; q < w.ptr[v + 1]; ++q) {
            int e = w.idx[q], g = gblock(p, e);
            if (g < 0) continue;
            for (int k = 0; k < 6; ++k)
                for (int i = 0; i < 6; ++i) t[k] += w.blk[e].Hgp[i * 6 + k] * r[g * 6 + i];
        }
        chol_solve(L + 36 * v, 6, t);
        int pc = ora_param_col_photo(p, v);
        for (int k = 0; k < 6; ++k) delta[pc + k] = z[6 * v + k] - t[k];
    }
out:
    free(S); free(r); free(L); free(z);
    free_ws(&w);
    return rc;
}

/* Photo back-substitution for a given global step dg (m): dp_v = Hpp^-1 (gp - sum_e Hgp_e^T dg_e)
 * for photos [lo, hi), written to dphoto[6 * (v - lo)] (the rank-local half of a sharded step). */
int ora_photo_backsub(const ora_problem *p, const float *x, int lo, int hi, const double *dg,
                      double *dphoto)
{
    sparse_ws w;
    int rc = build_ws(p, x, &w);
    for (int v = lo; v < hi && !rc; ++v) {
        double L[36] = {0}, gp[6] = {0}, t[6] = {0};
        for (int q = w.ptr[v]; q < w.ptr[v + 1]; ++q) {
            const edge_blk *b = &w.blk[w.idx[q]];
            for (int k = 0; k < 36; ++k) L[k] += b->Hpp[k];
            for (int k = 0; k < 6; ++k) gp[k] += b->gp[k];
            int g = gblock(p, w.idx[q]);
            if (g < 0) continue;
            for (int k = 0; k < 6; ++k)
                for (int i = 0; i < 6; ++i) t[k] += b->Hgp[i * 6 + k] * dg[g * 6 + i];
        }
        if (cholesky(L, 6)) { rc = -5; break; }
        chol_solve(L, 6, gp);
        chol_solve(L, 6, t);
        for (int k = 0; k < 6; ++k) dphoto[6 * (v - lo) + k] = gp[k] - t[k];
    }
    free_ws(&w);
    return rc;
}

int ora_normal_dense_j(const ora_problem *p, const float *x, double *JTJ, double *JTE)
{
    /* src/mymulticalib.cpp:680-803 literally, one thread: J = zeros(2 sum N, P) (:683), each
     * edge's 2N x 6 blocks copied in at the camera / photo columns (:776-786), E stacked (:784),
     * then JTJ = J.t() * J and JTE = J.t() * E as dense products (:802-803).  The product runs
     * over the transpose (P rows of length 2 sum N), so each entry is one contiguous dot. */
    int P = ora_nparams(p);
    long long rows = 0;
    int maxn = 0;
    for (int e = 0; e < p->n_edges; ++e) {
        rows += 2LL * p->edge_n[e];
        if (p->edge_n[e] > maxn) maxn = p->edge_n[e];
    }
    double *Jt = (double *)calloc((size_t)P * (size_t)rows, sizeof(double));
    double *E = (double *)malloc(sizeof(double) * (size_t)rows);
    double *jc = (double *)malloc(sizeof(double) * 12 * (size_t)maxn);
    double *jp = (double *)malloc(sizeof(double) * 12 * (size_t)maxn);
    int rc = 0;
    if (!Jt || !E || !jc || !jp) { rc = -3; goto out; }
    long long r0 = 0;
    for (int e = 0; e < p->n_edges; ++e) {
        if ((rc = ora_edge_linearize(p, x, e, jc, jp, E + r0, NULL))) goto out;
        int gc = global_col(p, e), pc = ora_param_col_photo(p, p->edge_photo[e]);
        for (int r = 0; r < 2 * p->edge_n[e]; ++r)
            for (int j = 0; j < 6; ++j) {
                if (gc >= 0) Jt[(size_t)(gc + j) * rows + r0 + r] = jc[r * 6 + j];
                Jt[(size_t)(pc + j) * rows + r0 + r] = jp[r * 6 + j];
            }
        r0 += 2LL * p->edge_n[e];
    }
    for (int a = 0; a < P; ++a) {
        const double *ja = Jt + (size_t)a * rows;
        for (int b = a; b < P; ++b) {
            const double *jb = Jt + (size_t)b * rows;
            double s = 0;
            for (long long r = 0; r < rows; ++r) s += ja[r] * jb[r];
            JTJ[(size_t)a * P + b] = s;
            JTJ[(size_t)b * P + a] = s;
        }
        double s = 0;
        for (long long r = 0; r < rows; ++r) s += ja[r] * E[r];
        JTE[a] = s;
    }
out:
    free(Jt); free(E); free(jc); free(jp);
    return rc;
}

int ora_linearize_solve(const ora_problem *p, const float *x, int solver, double *delta,
                        double *jte)
{
    int P = ora_nparams(p);
    if (solver == ORA_SOLVER_SCHUR) return solve_schur(p, x, delta, jte);
    double *JTJ = (double *)malloc(sizeof(double) * (size_t)P * P);
    double *JTE = (double *)malloc(sizeof(double) * (size_t)P);
    if (!JTJ || !JTE) { free(JTJ); free(JTE); return -3; }
    int rc = solver == ORA_SOLVER_DENSE_J ? ora_normal_dense_j(p, x, JTJ, JTE) : ora_normal_dense(p, x, JTJ, JTE);
    if (!rc) {
        ora_cg(P, JTJ, JTE, delta);
        if (jte) memcpy(jte, JTE, sizeof(double) * (size_t)P);
    }
    free(JTJ); free(JTE);
    return rc;
}

/* cv::norm(CV_32F, NORM_L2): double accumulation, CV_ENABLE_UNROLLED order. */
static double norm_l2f(const float *a, int n)
{
    double s = 0;
    int i = 0;
    for (; i <= n - 4; i += 4) {
        double v0 = a[i], v1 = a[i + 1], v2 = a[i + 2], v3 = a[i + 3];
        s += v0 * v0 + v1 * v1 + v2 * v2 + v3 * v3;
    }
    for (; i < n; ++i) { double v = a[i]; s += v * v; }
    return sqrt(s);
}

double ora_optimize(const ora_problem *p, int crit_type, int max_count, double eps, int solver,
                    float *x, int *iters, double *last_change)
{
    /* MultiCameraCalibration::optimizeExtrinsics, src/multicalib.cpp:462-514 */
    int P = ora_nparams(p);
    double *delta = (double *)malloc(sizeof(double) * (size_t)P);
    float *G = (float *)malloc(sizeof(float) * (size_t)P);
    double change = 1;
    int iter;
    for (iter = 0;; ++iter) {
        if ((crit_type == 1 && iter >= max_count) || (crit_type == 2 && change <= eps) ||
            (crit_type == 3 && (change <= eps || iter >= max_count)))
            break;
        const double alpha_smooth = 0.95;
        double alpha_smooth2 = pow(alpha_smooth, (double)iter + 1.0);
        if (ora_linearize_solve(p, x, solver, delta, NULL)) {
            free(delta); free(G);
            return -1.0;
        }
        for (int i = 0; i < P; ++i) G[i] = (float)(alpha_smooth2 * delta[i]);
        for (int i = 0; i < P; ++i) x[i] = x[i] + G[i];
        change = norm_l2f(G, P) / norm_l2f(x, P);
    }
    if (iters) *iters = iter;
    if (last_change) *last_change = change;
    free(delta); free(G);
    double mean = -1;
    if (ora_project_error(p, x, NULL, &mean)) return -1.0;
    return mean;
}

/* ------------------------------------------------------------------ computeProjectError */

/* cv::Rodrigues(Vec3f) -> CV_32F 3x3 (double internally, converted to float). */
static void rod_v2m_f(const float r[3], float R[9])
{
    double rd[3] = {r[0], r[1], r[2]}, Rd[9];
    ora_rodrigues_v2m(rd, Rd, NULL);
    for (int k = 0; k < 9; ++k) R[k] = (float)Rd[k];
}

int ora_project_error(const ora_problem *p, const float *x, float *edge_err, double *mean)
{
    /* src/mymulticalib.cpp:820-939 (pinhole), src/multicalib.cpp:895-1006 (omni),
     * src/doubleSide.cpp:640-769 (double side; the C == 2 CV_Assert at :643 is not restated). */
    float totalError = 0;
    long totalNPoints = 0;
    int maxn = 0;
    for (int e = 0; e < p->n_edges; ++e) if (p->edge_n[e] > maxn) maxn = p->edge_n[e];
    float *pr = (float *)malloc(sizeof(float) * 2 * (size_t)(maxn ? maxn : 1));
    float ds4[16];
    if (p->model == ORA_DOUBLESIDE) {
        float R[9];
        rod_v2m_f(x, R); /* doubleSideTransform1 from Rodrigues(RvecVertex[0]) */
        memset(ds4, 0, sizeof(ds4));
        for (int a = 0; a < 3; ++a) {
            for (int b = 0; b < 3; ++b) ds4[a * 4 + b] = R[a * 3 + b];
            ds4[a * 4 + 3] = x[3 + a];
        }
        ds4[15] = 1;
    }
    for (int e = 0; e < p->n_edges; ++e) {
        int cam = p->edge_cam[e], n = p->edge_n[e], off = p->edge_off[e];
        int pc = ora_param_col_photo(p, p->edge_photo[e]);
        float Rp[9], Rt[9], Tt[3];
        const float *tp = x + pc + 3;
        rod_v2m_f(x + pc, Rp);
        if (p->model == ORA_DOUBLESIDE) {
            float P4[16] = {0}, T4[16], T5[16];
            for (int a = 0; a < 3; ++a) {
                for (int b = 0; b < 3; ++b) P4[a * 4 + b] = Rp[a * 3 + b];
                P4[a * 4 + 3] = tp[a];
            }
            P4[15] = 1;
            mm4f(p->cam_pose + 16 * cam, P4, T4);
            if (p->edge_side[e] == ORA_BACK) {
                mm4f(T4, ds4, T5);
                memcpy(T4, T5, sizeof(T4));
            }
            for (int a = 0; a < 3; ++a) {
                for (int b = 0; b < 3; ++b) Rt[a * 3 + b] = T4[a * 4 + b];
                Tt[a] = T4[a * 4 + 3];
            }
        } else if (cam == 0) {
            memcpy(Rt, Rp, sizeof(Rt));
            memcpy(Tt, tp, sizeof(Tt));
        } else {
            int cc = ora_param_col_cam(p, cam);
            float Rc[9];
            rod_v2m_f(x + cc, Rc);
            mm3f(Rc, Rp, Rt, 3, NULL);           /* RCamera*RPhoto              */
            mm3f(Rc, tp, Tt, 1, x + cc + 3);     /* RCamera * TPhoto + TCamera  */
        }
        double Rd[9], rv[3];
        for (int k = 0; k < 9; ++k) Rd[k] = Rt[k];
        ora_rodrigues_m2v(Rd, rv, NULL);
        float rvec[3] = {(float)rv[0], (float)rv[1], (float)rv[2]};
        const float *obj = p->obj + 3 * (size_t)off, *img = p->img + 2 * (size_t)off;
        if (p->model == ORA_OMNI)
            ora_project_omni(n, obj, rvec, Tt, p->K + 9 * cam, (double)p->xi[cam], p->D + p->nd * cam, pr, NULL);
        else if (ora_project_pinhole(n, obj, rvec, Tt, p->K + 9 * cam, p->D + p->nd * cam, p->nd, pr, NULL)) {
            free(pr);
            return -4;
        }
        float errorPerImage = 0;
        for (int i = 0; i < n; ++i) {
            float ex = img[2 * i] - pr[2 * i];
            float ey = img[2 * i + 1] - pr[2 * i + 1];
            float s2 = ex * ex;
            s2 = s2 + ey * ey;
            float ferror = sqrtf(s2);
            errorPerImage += ferror;
        }
        if (edge_err) edge_err[e] = errorPerImage / n;
        totalError += errorPerImage;
        totalNPoints += (p->model == ORA_OMNI) ? n : 2 * n; /* error.total() (hazard H2) */
    }
    free(pr);
    if (mean) *mean = (double)totalError / (double)totalNPoints;
    return 0;
}
