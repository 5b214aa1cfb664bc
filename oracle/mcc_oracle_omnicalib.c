/*
 * mcc_oracle_omnicalib.c -- CPU restatement of cv::omnidir::calibrate, the per-camera intrinsic
 * Levenberg-Marquardt-style loop of the reference.
 *
 * TEST INFRASTRUCTURE ONLY (see mcc_oracle.h): the parity checker of the product's
 * mcc_omnidir_* path (include/mcc_omnidir.h).  The product never links or calls it.
 *
 * Restates (file:line under the reference):
 *   cv::omnidir::projectPoints with the 2x16 Jacobian ........ src/omnidir.cpp:84-245
 *   cv::omnidir::internal::initializeCalibration .............. src/omnidir.cpp:551-748
 *   cv::omnidir::internal::computeJacobian (dense JTJ, blocks
 *     as written, subMatrix by flags, JTJ + epsilon, inv()) .. src/omnidir.cpp:851-935
 *   cv::omnidir::calibrate's loop (alpha_smooth2, epsilon,
 *     fillFixed, change = |G| / |x|) ............................ src/omnidir.cpp:1067-1211
 *   encodeParameters layout [om_i, T_i]..., fx, fy, s, cx, cy,
 *     xi, k1, k2, p1, p2 ....................................... src/omnidir.cpp:1541-1568
 *   estimateUncertainties' rms ................................ src/omnidir.cpp:1734-1804
 *   computeMeanReproErr ....................................... src/omnidir.cpp:1892-1955
 *   flags2idx / fillFixed / subMatrix ......................... src/omnidir.cpp:2003-2153
 * OpenCV core pieces it calls (not vendored, version unpinned): Mat::inv() = DECOMP_LU (Gaussian
 * elimination with partial pivoting), SVD::compute (restated as one-sided Jacobi), solvePoly for
 * the quadratic (restated in closed form), Rodrigues (mcc_oracle.c).
 */
#include "mcc_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

static void mmd(const double *A, const double *B, double *C, int m, int k, int n)
{
    for (int i = 0; i < m; ++i)
        for (int j = 0; j < n; ++j) {
            double s = A[i * k] * B[j];
            for (int t = 1; t < k; ++t) s = s + A[i * k + t] * B[t * n + j];
            C[i * n + j] = s;
        }
}

/* ------------------------------------------------------------------ projection + 2x16 J */

void ora_omni_project_full(int n, const double *obj, const double om[3], const double T[3],
                           const double kin[5], double xi, const double D[4], double *img, double *jac)
{
    /* src/omnidir.cpp:84-245, CV_64F object points.  kin = fx, fy, s, cx, cy.  jac rows
     * (u_i, v_i) x 16 columns in JacobianRow order (:65-73): dom(3) dT(3) df(2) ds dc(2) dxi dkp(4). */
    const double f0 = kin[0], f1 = kin[1], s = kin[2], c0 = kin[3], c1 = kin[4];
    const double k1 = D[0], k2 = D[1], p1 = D[2], p2 = D[3];
    double R[9], dRdom[27];
    ora_rodrigues_v2m(om, R, dRdom);
    for (int i = 0; i < n; ++i) {
        const double Xw[3] = {obj[3 * i], obj[3 * i + 1], obj[3 * i + 2]};
        double Xc[3];
        for (int a = 0; a < 3; ++a) {
            double acc = R[a * 3] * Xw[0];
            acc = acc + R[a * 3 + 1] * Xw[1];
            acc = acc + R[a * 3 + 2] * Xw[2];
            Xc[a] = acc + T[a];
        }
        const double nrm = sqrt(Xc[0] * Xc[0] + Xc[1] * Xc[1] + Xc[2] * Xc[2]);
        const double Xs[3] = {Xc[0] / nrm, Xc[1] / nrm, Xc[2] / nrm};
        const double xu[2] = {Xs[0] / (Xs[2] + xi), Xs[1] / (Xs[2] + xi)};
        const double r2 = xu[0] * xu[0] + xu[1] * xu[1];
        const double r4 = r2 * r2;
        double xd[2];
        xd[0] = xu[0] * (1 + k1 * r2 + k2 * r4) + 2 * p1 * xu[0] * xu[1] + p2 * (r2 + 2 * xu[0] * xu[0]);
        xd[1] = xu[1] * (1 + k1 * r2 + k2 * r4) + p1 * (r2 + 2 * xu[1] * xu[1]) + 2 * p2 * xu[0] * xu[1];
        img[2 * i] = f0 * xd[0] + s * xd[1] + c0;
        img[2 * i + 1] = f1 * xd[1] + c1;
        if (!jac) continue;
        double dXcdom[9];
        for (int a = 0; a < 3; ++a)        /* dXcdR (3x9) * dRdom^T (9x3) */
            for (int b = 0; b < 3; ++b) {
                double acc = 0;
                for (int c = 0; c < 3; ++c) acc = acc + Xw[c] * dRdom[b * 9 + a * 3 + c];
                dXcdom[a * 3 + b] = acc;
            }
        const double r_1 = 1.0 / nrm, r_3 = pow(r_1, 3);
        const double dXsdXc[9] = {r_1 - Xc[0] * Xc[0] * r_3, -(Xc[0] * Xc[1]) * r_3, -(Xc[0] * Xc[2]) * r_3,
                                  -(Xc[0] * Xc[1]) * r_3, r_1 - Xc[1] * Xc[1] * r_3, -(Xc[1] * Xc[2]) * r_3,
                                  -(Xc[0] * Xc[2]) * r_3, -(Xc[1] * Xc[2]) * r_3, r_1 - Xc[2] * Xc[2] * r_3};
        const double den = Xs[2] + xi;
        const double dxudXs[6] = {1 / den, 0, -Xs[0] / den / den, 0, 1 / den, -Xs[1] / den / den};
        const double temp1 = 2 * k1 * xu[0] + 4 * k2 * xu[0] * r2;
        const double temp2 = 2 * k1 * xu[1] + 4 * k2 * xu[1] * r2;
        const double dxddxu[4] = {k2 * r4 + 6 * p2 * xu[0] + 2 * p1 * xu[1] + xu[0] * temp1 + k1 * r2 + 1,
                                  2 * p1 * xu[0] + 2 * p2 * xu[1] + xu[0] * temp2,
                                  2 * p1 * xu[0] + 2 * p2 * xu[1] + xu[1] * temp1,
                                  k2 * r4 + 2 * p2 * xu[0] + 6 * p1 * xu[1] + xu[1] * temp2 + k1 * r2 + 1};
        const double dxpddxd[4] = {f0, s, 0, f1};
        double t22[4], t23[6], dxpddXc[6], dxpddom[6];
        mmd(dxpddxd, dxddxu, t22, 2, 2, 2);
        mmd(t22, dxudXs, t23, 2, 2, 3);
        mmd(t23, dXsdXc, dxpddXc, 2, 3, 3);
        mmd(dxpddXc, dXcdom, dxpddom, 2, 3, 3);
        const double dxudxi[2] = {-Xs[0] / den / den, -Xs[1] / den / den};
        double dxpddxi[2];
        mmd(t22, dxudxi, dxpddxi, 2, 2, 1);
        const double dxddkp[8] = {xu[0] * r2, xu[0] * r4, 2 * xu[0] * xu[1], r2 + 2 * xu[0] * xu[0],
                                  xu[1] * r2, xu[1] * r4, r2 + 2 * xu[1] * xu[1], 2 * xu[0] * xu[1]};
        double dxpddkp[8];
        mmd(dxpddxd, dxddkp, dxpddkp, 2, 2, 4);
        double *ju = jac + (size_t)(2 * i) * 16, *jv = ju + 16;
        for (int j = 0; j < 3; ++j) {
            ju[j] = dxpddom[j];
            jv[j] = dxpddom[3 + j];
            ju[3 + j] = dxpddXc[j];   /* dxpddT = dxpddXc * I */
            jv[3 + j] = dxpddXc[3 + j];
        }
        ju[6] = xd[0]; ju[7] = 0;     jv[6] = 0; jv[7] = xd[1];     /* df */
        ju[8] = xd[1];                jv[8] = 0;                    /* ds */
        ju[9] = 1; ju[10] = 0;        jv[9] = 0; jv[10] = 1;        /* dc */
        ju[11] = dxpddxi[0];          jv[11] = dxpddxi[1];          /* dxi */
        for (int j = 0; j < 4; ++j) {
            ju[12 + j] = dxpddkp[j];
            jv[12 + j] = dxpddkp[4 + j];
        }
    }
}

/* kin / xi / D from the parameter vector (encodeParameters, src/omnidir.cpp:1541-1568) */
static void decode_intr(const double *para, int n, double kin[5], double *xi, double D[4])
{
    const double *q = para + 6 * n;
    kin[0] = q[0]; kin[1] = q[1]; kin[2] = q[2]; kin[3] = q[3]; kin[4] = q[4];
    *xi = q[5];
    D[0] = q[6]; D[1] = q[7]; D[2] = q[8]; D[3] = q[9];
}

/* flags2idx, src/omnidir.cpp:2031-2076 (the cascade of >= tests, CALIB_USE_GUESS unhandled) */
void ora_omni_flags2idx(int flags, int n, int *idx)
{
    const int P = 6 * n + 10;
    for (int i = 0; i < P; ++i) idx[i] = 1;
    int f = flags;
    if (f >= 256) { idx[6 * n + 3] = 0; idx[6 * n + 4] = 0; f -= 256; }   /* CALIB_FIX_CENTER */
    if (f >= 128) { idx[6 * n] = 0; idx[6 * n + 1] = 0; f -= 128; }       /* CALIB_FIX_GAMMA  */
    if (f >= 64) { idx[6 * n + 5] = 0; f -= 64; }                         /* CALIB_FIX_XI     */
    if (f >= 32) { idx[6 * n + 9] = 0; f -= 32; }                         /* CALIB_FIX_P2     */
    if (f >= 16) { idx[6 * n + 8] = 0; f -= 16; }                         /* CALIB_FIX_P1     */
    if (f >= 8) { idx[6 * n + 7] = 0; f -= 8; }                           /* CALIB_FIX_K2     */
    if (f >= 4) { idx[6 * n + 6] = 0; f -= 4; }                           /* CALIB_FIX_K1     */
    if (f >= 2) { idx[6 * n + 2] = 0; }                                   /* CALIB_FIX_SKEW   */
}

/* Mat::inv() (DECOMP_LU): Gauss-Jordan with partial pivoting on [A | I].  Returns 0, or -1
 * when a pivot is exactly zero (OpenCV then returns a zero matrix). */
static int lu_inverse(const double *A, double *Ai, int n)
{
    double *M = (double *)malloc(sizeof(double) * (size_t)n * 2 * n);
    if (!M) return -2;
    const int w = 2 * n;
    for (int i = 0; i < n; ++i) {
        for (int j = 0; j < n; ++j) {
            M[(size_t)i * w + j] = A[(size_t)i * n + j];
            M[(size_t)i * w + n + j] = i == j ? 1.0 : 0.0;
        }
    }
    int rc = 0;
    for (int k = 0; k < n && !rc; ++k) {
        int p = k;
        for (int i = k + 1; i < n; ++i)
            if (fabs(M[(size_t)i * w + k]) > fabs(M[(size_t)p * w + k])) p = i;
        if (M[(size_t)p * w + k] == 0.0) { rc = -1; break; }
        if (p != k)
            for (int j = 0; j < w; ++j) {
                double t = M[(size_t)k * w + j];
                M[(size_t)k * w + j] = M[(size_t)p * w + j];
                M[(size_t)p * w + j] = t;
            }
        const double ip = 1.0 / M[(size_t)k * w + k];
        for (int j = 0; j < w; ++j) M[(size_t)k * w + j] *= ip;
        for (int i = 0; i < n; ++i) {
            if (i == k) continue;
            const double f = M[(size_t)i * w + k];
            if (f == 0.0) continue;
            for (int j = 0; j < w; ++j) M[(size_t)i * w + j] -= f * M[(size_t)k * w + j];
        }
    }
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) Ai[(size_t)i * n + j] = rc ? 0.0 : M[(size_t)i * w + n + j];
    free(M);
    return rc;
}

/* ------------------------------------------------------------------ computeJacobian */

int ora_omni_jacobian(int n, const int *off, const double *obj, const double *img, const double *para,
                      int flags, double epsilon, double *JTJ_inv, double *JTE_full, double *JTE_sub, int *n_free)
{
    /* src/omnidir.cpp:851-935.  JTE_full (P, optional): the JTE before subMatrix.  JTJ_inv
     * (optional, n_free^2) and JTE_sub (optional, n_free): the outputs after subMatrix by the
     * flags, with JTJ + epsilon inverted. */
    const int P = 6 * n + 10;
    double kin[5], xi, D[4];
    decode_intr(para, n, kin, &xi, D);
    double *JTJ = (double *)calloc((size_t)P * P, sizeof(double));
    double *JTE = (double *)calloc((size_t)P, sizeof(double));
    int maxn = 0;
    for (int i = 0; i < n; ++i) maxn = off[i + 1] - off[i] > maxn ? off[i + 1] - off[i] : maxn;
    double *proj = (double *)malloc(sizeof(double) * 2 * (size_t)(maxn > 0 ? maxn : 1));
    double *jac = (double *)malloc(sizeof(double) * 32 * (size_t)(maxn > 0 ? maxn : 1));
    if (!JTJ || !JTE || !proj || !jac) {
        free(JTJ); free(JTE); free(proj); free(jac);
        return -2;
    }
    for (int i = 0; i < n; ++i) {
        const int np = off[i + 1] - off[i];
        ora_omni_project_full(np, obj + 3 * (size_t)off[i], para + 6 * i, para + 6 * i + 3, kin, xi, D, proj, jac);
        /* JIn = jacobian cols 6..15, JEx = cols 0..5; projError = img - proj (2N x 1) */
        const double *ob = img + 2 * (size_t)off[i];
        double JInTJIn[100] = {0}, JExTJEx[36] = {0}, JExTJIn[60] = {0}, JInTe[10] = {0}, JExTe[6] = {0};
        for (int a = 0; a < 16; ++a) {
            for (int b = 0; b < 16; ++b) {
                if ((a < 6) != (b < 6) && a >= 6) continue;   /* JIn^T JEx is the transpose below */
                double acc = 0;
                for (int r = 0; r < 2 * np; ++r) acc = acc + jac[(size_t)r * 16 + a] * jac[(size_t)r * 16 + b];
                if (a < 6 && b < 6) JExTJEx[a * 6 + b] = acc;
                else if (a < 6) JExTJIn[a * 10 + b - 6] = acc;
                else JInTJIn[(a - 6) * 10 + b - 6] = acc;
            }
            double acc = 0;
            for (int r = 0; r < 2 * np; ++r) acc = acc + jac[(size_t)r * 16 + a] * (ob[r] - proj[r]);
            if (a < 6) JExTe[a] = acc;
            else JInTe[a - 6] = acc;
        }
        const int c = 6 * n;
        for (int a = 0; a < 10; ++a)
            for (int b = 0; b < 10; ++b) JTJ[(size_t)(c + a) * P + c + b] += JInTJIn[a * 10 + b];
        for (int a = 0; a < 6; ++a)
            for (int b = 0; b < 6; ++b) JTJ[(size_t)(6 * i + a) * P + 6 * i + b] = JExTJEx[a * 6 + b];
        for (int a = 0; a < 6; ++a)
            for (int b = 0; b < 10; ++b) {
                JTJ[(size_t)(6 * i + a) * P + c + b] = JExTJIn[a * 10 + b];   /* JTJ(Rect(6n, 6i, 10, 6)) */
                JTJ[(size_t)(c + b) * P + 6 * i + a] = JExTJIn[a * 10 + b];   /* JTJ(Rect(6i, 6n, 6, 10)) */
            }
        for (int a = 0; a < 10; ++a) JTE[c + a] += JInTe[a];
        for (int a = 0; a < 6; ++a) JTE[6 * i + a] = JExTe[a];
    }
    free(proj);
    free(jac);
    if (JTE_full) memcpy(JTE_full, JTE, sizeof(double) * P);
    int *idx = (int *)malloc(sizeof(int) * P);
    ora_omni_flags2idx(flags, n, idx);
    int nf = 0;
    for (int i = 0; i < P; ++i) nf += idx[i];
    if (n_free) *n_free = nf;
    int rc = 0;
    if (JTJ_inv || JTE_sub) {
        double *S = (double *)malloc(sizeof(double) * (size_t)nf * nf);
        int ii = 0;
        for (int i = 0; i < P; ++i) {
            if (!idx[i]) continue;
            int jj = 0;
            for (int j = 0; j < P; ++j) {
                if (!idx[j]) continue;
                S[(size_t)ii * nf + jj] = JTJ[(size_t)i * P + j] + epsilon;   /* JTJ + epsilon: every entry */
                ++jj;
            }
            if (JTE_sub) JTE_sub[ii] = JTE[i];
            ++ii;
        }
        if (JTJ_inv) rc = lu_inverse(S, JTJ_inv, nf);
        free(S);
    }
    free(idx);
    free(JTJ);
    free(JTE);
    return rc == -2 ? -2 : 0;
}

/* One G of calibrate's loop at iteration iter (src/omnidir.cpp:1134-1148): alpha_smooth2 *
 * JTJ_inv * JTError, fillFixed.  G is P long. */
int ora_omni_step(int n, const int *off, const double *obj, const double *img, const double *para,
                  int flags, int iter, double *G)
{
    const int P = 6 * n + 10;
    const double alpha_smooth = 0.01;
    const double alpha_smooth2 = 1 - pow(1 - alpha_smooth, (double)iter + 1.0);
    const double epsilon = 0.01 * pow(0.9, (double)iter / 10);
    int nf = 0;
    double *Ji = (double *)malloc(sizeof(double) * (size_t)P * P);
    double *Je = (double *)malloc(sizeof(double) * P);
    int *idx = (int *)malloc(sizeof(int) * P);
    if (!Ji || !Je || !idx) { free(Ji); free(Je); free(idx); return -2; }
    int rc = ora_omni_jacobian(n, off, obj, img, para, flags, epsilon, Ji, NULL, Je, &nf);
    if (!rc) {
        ora_omni_flags2idx(flags, n, idx);
        for (int i = 0, j = 0; i < P; ++i) {
            if (!idx[i]) { G[i] = 0.0; continue; }
            /* (alpha_smooth2 * JTJ_inv) * JTError */
            double acc = (alpha_smooth2 * Ji[(size_t)j * nf]) * Je[0];
            for (int k = 1; k < nf; ++k) acc = acc + (alpha_smooth2 * Ji[(size_t)j * nf + k]) * Je[k];
            G[i] = acc;
            ++j;
        }
    }
    free(Ji); free(Je); free(idx);
    return rc;
}

static double norm2(const double *a, int n)
{
    double s = 0;
    for (int i = 0; i < n; ++i) s = s + a[i] * a[i];
    return sqrt(s);
}

int ora_omni_optimize(int n, const int *off, const double *obj, const double *img, double *para, int flags,
                      int crit_type, int max_count, double eps, int *iters, double *last_change)
{
    /* calibrate's loop, src/omnidir.cpp:1126-1149 */
    const int P = 6 * n + 10;
    double *G = (double *)malloc(sizeof(double) * P);
    if (!G) return -2;
    double change = 1;
    int iter = 0;
    for (;; ++iter) {
        if ((crit_type == 1 && iter >= max_count) || (crit_type == 2 && change <= eps) ||
            (crit_type == 3 && (change <= eps || iter >= max_count)))
            break;
        int rc = ora_omni_step(n, off, obj, img, para, flags, iter, G);
        if (rc) { free(G); return rc; }
        change = norm2(G, P) / norm2(para, P);
        for (int i = 0; i < P; ++i) para[i] = para[i] + G[i];
    }
    free(G);
    if (iters) *iters = iter;
    if (last_change) *last_change = change;
    return 0;
}

double ora_omni_rms(int n, const int *off, const double *obj, const double *img, const double *para)
{
    /* estimateUncertainties' rms, src/omnidir.cpp:1791-1803 */
    double kin[5], xi, D[4];
    decode_intr(para, n, kin, &xi, D);
    double rms = 0;
    long long tot = 0;
    for (int i = 0; i < n; ++i) {
        const int np = off[i + 1] - off[i];
        double *proj = (double *)malloc(sizeof(double) * 2 * (size_t)(np > 0 ? np : 1));
        ora_omni_project_full(np, obj + 3 * (size_t)off[i], para + 6 * i, para + 6 * i + 3, kin, xi, D, proj, NULL);
        const double *ob = img + 2 * (size_t)off[i];
        for (int k = 0; k < np; ++k) {
            const double ex = ob[2 * k] - proj[2 * k], ey = ob[2 * k + 1] - proj[2 * k + 1];
            rms += ex * ex + ey * ey;
        }
        tot += np;
        free(proj);
    }
    rms /= (double)tot;
    return sqrt(rms);
}

/* ------------------------------------------------------------------ initializeCalibration */

/* One-sided Jacobi SVD of A (m x k, row-major, destroyed): V (k x k, columns = right singular
 * vectors) and sv[k] (unsorted). */
static void jacobi_svd(double *A, int m, int k, double *V, double *sv)
{
    for (int i = 0; i < k; ++i)
        for (int j = 0; j < k; ++j) V[i * k + j] = i == j ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 60; ++sweep) {
        double off = 0;
        for (int p = 0; p < k - 1; ++p)
            for (int q = p + 1; q < k; ++q) {
                double a = 0, b = 0, g = 0;
                for (int r = 0; r < m; ++r) {
                    a += A[r * k + p] * A[r * k + p];
                    b += A[r * k + q] * A[r * k + q];
                    g += A[r * k + p] * A[r * k + q];
                }
                if (a == 0 || b == 0) continue;
                const double rel = fabs(g) / sqrt(a * b);
                if (rel > off) off = rel;
                if (rel < 1e-15) continue;
                const double zeta = (b - a) / (2 * g);
                const double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1 + zeta * zeta));
                const double c = 1 / sqrt(1 + t * t), s = c * t;
                for (int r = 0; r < m; ++r) {
                    const double x = A[r * k + p], y = A[r * k + q];
                    A[r * k + p] = c * x - s * y;
                    A[r * k + q] = s * x + c * y;
                }
                for (int r = 0; r < k; ++r) {
                    const double x = V[r * k + p], y = V[r * k + q];
                    V[r * k + p] = c * x - s * y;
                    V[r * k + q] = s * x + c * y;
                }
            }
        if (off < 1e-15) break;
    }
    for (int j = 0; j < k; ++j) {
        double s = 0;
        for (int r = 0; r < m; ++r) s += A[r * k + j] * A[r * k + j];
        sv[j] = sqrt(s);
    }
}

static double mean_repro(int np, const double *img, const double *proj)
{
    /* computeMeanReproErr(imagePoints, proImagePoints), src/omnidir.cpp:1892-1934 */
    double e = 0;
    for (int j = 0; j < np; ++j) {
        const double dx = img[2 * j] - proj[2 * j], dy = img[2 * j + 1] - proj[2 * j + 1];
        e += sqrt(dx * dx + dy * dy);
    }
    return e / np;
}

static int cmp_double(const void *a, const void *b)
{
    const double x = *(const double *)a, y = *(const double *)b;
    return x < y ? -1 : x > y ? 1 : 0;
}

int ora_omni_init(int n_img, const int *off, const double *obj, const double *img, int width, int height,
                  double *om_out, double *t_out, double *K, double *xi, int *idx, int *n_idx)
{
    /* src/omnidir.cpp:551-748.  om_out / t_out: [3 * n_idx] of the kept views (idx order). */
    const double u0 = width / 2, v0 = height / 2;   /* int division, as Size::width / 2 */
    double *omA = (double *)calloc(3 * (size_t)n_img + 3, sizeof(double));
    double *tA = (double *)calloc(3 * (size_t)n_img + 3, sizeof(double));
    double *gammaAll = (double *)calloc((size_t)n_img + 1, sizeof(double));
    int maxn = 1;
    for (int i = 0; i < n_img; ++i) maxn = off[i + 1] - off[i] > maxn ? off[i + 1] - off[i] : maxn;
    double *M = (double *)malloc(sizeof(double) * 6 * (size_t)maxn);
    double *A = (double *)malloc(sizeof(double) * 6 * (size_t)maxn);
    double *B = (double *)malloc(sizeof(double) * 2 * (size_t)maxn);
    double *proj = (double *)malloc(sizeof(double) * 2 * (size_t)maxn);
    const double zeroD[4] = {0, 0, 0, 0};
    for (int im = 0; im < n_img; ++im) {
        const int np = off[im + 1] - off[im];
        const double *ob = obj + 3 * (size_t)off[im];
        const double *ip = img + 2 * (size_t)off[im];
        for (int j = 0; j < np; ++j) {
            const double x = ob[3 * j], y = ob[3 * j + 1], u = ip[2 * j] - u0, v = ip[2 * j + 1] - v0;
            double *row = M + 6 * (size_t)j;
            row[0] = -v * x; row[1] = -v * y; row[2] = u * x; row[3] = u * y; row[4] = -v; row[5] = u;
        }
        double V[36], sv[6];
        jacobi_svd(M, np, 6, V, sv);
        int jmin = 0;   /* the smallest singular value (OpenCV's V column 5) */
        for (int j = 1; j < 6; ++j) if (sv[j] < sv[jmin]) jmin = j;
        double best = 1e5;
        for (int coef = 1; coef >= -1; coef -= 2) {
            const double r11 = V[0 * 6 + jmin] * coef, r12 = V[1 * 6 + jmin] * coef;
            const double r21 = V[2 * 6 + jmin] * coef, r22 = V[3 * 6 + jmin] * coef;
            const double t1 = V[4 * 6 + jmin] * coef, t2 = V[5 * 6 + jmin] * coef;
            /* solvePoly(z^2 + bq z + cq): the reference takes root 0 if > 0 else root 1, i.e. the
             * positive root of this quadratic (cq <= 0) */
            const double q = r11 * r12 + r21 * r22;
            const double bq = r11 * r11 + r21 * r21 - r12 * r12 - r22 * r22, cq = -q * q;
            const double disc = sqrt(bq * bq - 4 * cq);
            const double zp = bq > 0 ? (-2 * cq) / (bq + disc) : (-bq + disc) / 2;
            const double r31s = sqrt(zp);
            for (int coef2 = 1; coef2 >= -1; coef2 -= 2) {
                const double r31 = r31s * coef2;
                const double r32 = -(r11 * r12 + r21 * r22) / r31;
                double r1[3] = {r11, r21, r31}, r2[3] = {r12, r22, r32}, t[3] = {t1, t2, 0};
                const double scale = 1 / sqrt(r1[0] * r1[0] + r1[1] * r1[1] + r1[2] * r1[2]);
                for (int k = 0; k < 3; ++k) { r1[k] *= scale; r2[k] *= scale; t[k] *= scale; }
                /* Scaramuzza's equations: A (2np x 3), B (2np) */
                for (int j = 0; j < np; ++j) {
                    const double x = ob[3 * j], y = ob[3 * j + 1], u = ip[2 * j] - u0, v = ip[2 * j + 1] - v0;
                    const double rho2 = u * u + v * v;
                    const double a0 = (r1[1] * x + r2[1] * y + t[1]) / 2;
                    const double a1 = (r1[0] * x + r2[0] * y + t[0]) / 2;
                    A[3 * j] = a0; A[3 * j + 1] = -a0 * rho2; A[3 * j + 2] = -v;
                    A[3 * (np + j)] = a1; A[3 * (np + j) + 1] = -a1 * rho2; A[3 * (np + j) + 2] = -u;
                    B[j] = v * (r1[2] * x + r2[2] * y);
                    B[np + j] = u * (r1[2] * x + r2[2] * y);
                }
                double maxA[3] = {0, 0, 0};
                for (int r = 0; r < 2 * np; ++r)
                    for (int c = 0; c < 3; ++c) if (fabs(A[3 * r + c]) > maxA[c]) maxA[c] = fabs(A[3 * r + c]);
                for (int r = 0; r < 2 * np; ++r)
                    for (int c = 0; c < 3; ++c) A[3 * r + c] /= maxA[c];
                /* A.inv(DECOMP_SVD) * B: the minimum-norm least-squares solution */
                double Va[9], sa[3];
                jacobi_svd(A, 2 * np, 3, Va, sa);   /* A <- U * diag(sa) */
                double res[3] = {0, 0, 0};
                const double smax = fmax(sa[0], fmax(sa[1], sa[2]));
                for (int c = 0; c < 3; ++c) {
                    if (!(sa[c] > smax * DBL_EPSILON * 2 * np)) continue;
                    double ub = 0;
                    for (int r = 0; r < 2 * np; ++r) ub += A[3 * r + c] * B[r];
                    ub /= sa[c] * sa[c];   /* (U_c . B) / sigma_c with U_c = A_c / sigma_c */
                    for (int k = 0; k < 3; ++k) res[k] += Va[k * 3 + c] * ub;
                }
                for (int k = 0; k < 3; ++k) res[k] *= 1 / maxA[k];
                const double gamma = sqrt(res[0] / res[1]);
                t[2] = res[2];
                const double r3[3] = {r1[1] * r2[2] - r1[2] * r2[1], r1[2] * r2[0] - r1[0] * r2[2],
                                      r1[0] * r2[1] - r1[1] * r2[0]};
                const double R[9] = {r1[0], r2[0], r3[0], r1[1], r2[1], r3[1], r1[2], r2[2], r3[2]};
                double om[3];
                ora_rodrigues_m2v(R, om, NULL);
                const double kin[5] = {gamma, gamma, 0, u0, v0};
                ora_omni_project_full(np, ob, om, t, kin, 1.0, zeroD, proj, NULL);
                const double err = mean_repro(np, ip, proj);
                if (err < best) {
                    best = err;
                    memcpy(omA + 3 * im, om, sizeof(om));
                    memcpy(tA + 3 * im, t, sizeof(t));
                    gammaAll[im] = gamma;
                }
            }
        }
    }
    /* median gamma: nth_element at n/2 */
    double *sorted = (double *)malloc(sizeof(double) * ((size_t)n_img + 1));
    memcpy(sorted, gammaAll, sizeof(double) * n_img);
    qsort(sorted, n_img, sizeof(double), cmp_double);
    const double gammaFinal = sorted[n_img / 2];
    free(sorted);
    const double Kf[9] = {gammaFinal, 0, u0, 0, gammaFinal, v0, 0, 0, 1};
    memcpy(K, Kf, sizeof(Kf));
    const double kin[5] = {gammaFinal, gammaFinal, 0, u0, v0};
    int nk = 0;
    for (int i = 0; i < n_img; ++i) {
        const int np = off[i + 1] - off[i];
        ora_omni_project_full(np, obj + 3 * (size_t)off[i], omA + 3 * i, tA + 3 * i, kin, 1.0, zeroD, proj, NULL);
        const double err = mean_repro(np, img + 2 * (size_t)off[i], proj);
        if (err < 100) {
            idx[nk] = i;
            memcpy(om_out + 3 * nk, omA + 3 * i, 3 * sizeof(double));
            memcpy(t_out + 3 * nk, tA + 3 * i, 3 * sizeof(double));
            ++nk;
        }
    }
    *n_idx = nk;
    *xi = 1;
    free(omA); free(tA); free(gammaAll); free(M); free(A); free(B); free(proj);
    return 0;
}

double ora_omni_calibrate(int n_img, const int *off, const double *obj, const double *img, int width, int height,
                          int flags, int crit_type, int max_count, double eps, double *K, double *xi, double *D,
                          double *om, double *t, int *idx, int *n_idx, int *iters)
{
    /* src/omnidir.cpp:1067-1211: initialise, keep idx views, encodeParameters with D = 0, loop,
     * decode, rms of estimateUncertainties.  Returns rms (negative on failure). */
    double *om0 = (double *)malloc(sizeof(double) * 3 * ((size_t)n_img + 1));
    double *t0 = (double *)malloc(sizeof(double) * 3 * ((size_t)n_img + 1));
    double K0[9], xi0;
    int nk = 0;
    ora_omni_init(n_img, off, obj, img, width, height, om0, t0, K0, &xi0, idx, &nk);
    *n_idx = nk;
    int *o2 = (int *)malloc(sizeof(int) * ((size_t)nk + 1));
    o2[0] = 0;
    for (int i = 0; i < nk; ++i) o2[i + 1] = o2[i] + off[idx[i] + 1] - off[idx[i]];
    double *ob2 = (double *)malloc(sizeof(double) * 3 * ((size_t)o2[nk] + 1));
    double *im2 = (double *)malloc(sizeof(double) * 2 * ((size_t)o2[nk] + 1));
    for (int i = 0; i < nk; ++i) {
        const int np = o2[i + 1] - o2[i];
        memcpy(ob2 + 3 * (size_t)o2[i], obj + 3 * (size_t)off[idx[i]], sizeof(double) * 3 * np);
        memcpy(im2 + 2 * (size_t)o2[i], img + 2 * (size_t)off[idx[i]], sizeof(double) * 2 * np);
    }
    const int P = 6 * nk + 10;
    double *para = (double *)malloc(sizeof(double) * P);
    for (int i = 0; i < nk; ++i) {
        memcpy(para + 6 * i, om0 + 3 * i, 3 * sizeof(double));
        memcpy(para + 6 * i + 3, t0 + 3 * i, 3 * sizeof(double));
    }
    double *q = para + 6 * nk;
    q[0] = K0[0]; q[1] = K0[4]; q[2] = K0[1]; q[3] = K0[2]; q[4] = K0[5]; q[5] = xi0;
    q[6] = q[7] = q[8] = q[9] = 0;
    double rms = -1;
    if (ora_omni_optimize(nk, o2, ob2, im2, para, flags, crit_type, max_count, eps, iters, NULL) == 0) {
        rms = ora_omni_rms(nk, o2, ob2, im2, para);
        const double Kd[9] = {q[0], q[2], q[3], 0, q[1], q[4], 0, 0, 1};
        memcpy(K, Kd, sizeof(Kd));
        *xi = q[5];
        memcpy(D, q + 6, 4 * sizeof(double));
        for (int i = 0; i < nk; ++i) {
            memcpy(om + 3 * i, para + 6 * i, 3 * sizeof(double));
            memcpy(t + 3 * i, para + 6 * i + 3, 3 * sizeof(double));
        }
    }
    free(om0); free(t0); free(o2); free(ob2); free(im2); free(para);
    return rms;
}
