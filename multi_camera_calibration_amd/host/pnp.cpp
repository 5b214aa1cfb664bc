// pnp.cpp -- cv::solvePnP (SOLVEPNP_ITERATIVE) restated for the loaders' pose initialisation
// (include/mcc_pnp.hpp; reference call site src/mymulticalib.cpp:203-211).
#include "mcc_pnp.hpp"

#include <algorithm>
#include <cmath>
#include <cstring>

namespace mcc {
namespace pnp {

namespace {

// Jacobi eigen-decomposition of a symmetric n x n matrix (row-major, n <= 12): eigenvalues in
// w (ascending), eigenvectors in the columns of V
void jacobi_eig(const double* A0, int n, double* w, double* V) {
    double A[144];
    std::memcpy(A, A0, sizeof(double) * n * n);
    for (int i = 0; i < n * n; ++i) V[i] = 0.0;
    for (int i = 0; i < n; ++i) V[i * n + i] = 1.0;
    for (int sweep = 0; sweep < 100; ++sweep) {
        double off = 0.0;
        for (int i = 0; i < n; ++i)
            for (int j = i + 1; j < n; ++j) off += A[i * n + j] * A[i * n + j];
        if (off < 1e-300) break;
        for (int p = 0; p < n; ++p)
            for (int q = p + 1; q < n; ++q) {
                const double apq = A[p * n + q];
                if (std::fabs(apq) < 1e-300) continue;
                const double theta = (A[q * n + q] - A[p * n + p]) / (2.0 * apq);
                const double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1.0));
                const double c = 1.0 / std::sqrt(t * t + 1.0), s = t * c;
                for (int k = 0; k < n; ++k) {   // A <- J^T A J
                    const double akp = A[k * n + p], akq = A[k * n + q];
                    A[k * n + p] = c * akp - s * akq;
                    A[k * n + q] = s * akp + c * akq;
                }
                for (int k = 0; k < n; ++k) {
                    const double apk = A[p * n + k], aqk = A[q * n + k];
                    A[p * n + k] = c * apk - s * aqk;
                    A[q * n + k] = s * apk + c * aqk;
                }
                for (int k = 0; k < n; ++k) {
                    const double vkp = V[k * n + p], vkq = V[k * n + q];
                    V[k * n + p] = c * vkp - s * vkq;
                    V[k * n + q] = s * vkp + c * vkq;
                }
            }
    }
    // sort ascending
    int idx[12];
    for (int i = 0; i < n; ++i) idx[i] = i;
    std::sort(idx, idx + n, [&](int a, int b) { return A[a * n + a] < A[b * n + b]; });
    double Vs[144];
    for (int i = 0; i < n; ++i) {
        w[i] = A[idx[i] * n + idx[i]];
        for (int k = 0; k < n; ++k) Vs[k * n + i] = V[k * n + idx[i]];
    }
    std::memcpy(V, Vs, sizeof(double) * n * n);
}

// nearest rotation to M (polar factor, det +1): R = M (M^T M)^-1/2
void nearest_rotation(const double* M, double* R) {
    double MtM[9], w[3], V[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double s = 0.0;
            for (int k = 0; k < 3; ++k) s += M[k * 3 + i] * M[k * 3 + j];
            MtM[i * 3 + j] = s;
        }
    jacobi_eig(MtM, 3, w, V);
    double Si[9];   // V diag(1/sqrt w) V^T
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double s = 0.0;
            for (int k = 0; k < 3; ++k) s += V[i * 3 + k] * V[j * 3 + k] / std::sqrt(std::max(w[k], 1e-300));
            Si[i * 3 + j] = s;
        }
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double s = 0.0;
            for (int k = 0; k < 3; ++k) s += M[i * 3 + k] * Si[k * 3 + j];
            R[i * 3 + j] = s;
        }
    const double det = R[0] * (R[4] * R[8] - R[5] * R[7]) - R[1] * (R[3] * R[8] - R[5] * R[6]) +
                       R[2] * (R[3] * R[7] - R[4] * R[6]);
    if (det < 0)
        for (int i = 0; i < 3; ++i) R[i * 3 + 2] = -R[i * 3 + 2];
}

bool solve6(double* A, double* b) {   // A x = b (6 x 6, SPD-ish), Gaussian elimination with pivoting
    const int n = 6;
    for (int k = 0; k < n; ++k) {
        int p = k;
        for (int i = k + 1; i < n; ++i)
            if (std::fabs(A[i * n + k]) > std::fabs(A[p * n + k])) p = i;
        if (std::fabs(A[p * n + k]) < 1e-300) return false;
        if (p != k) {
            for (int j = 0; j < n; ++j) std::swap(A[k * n + j], A[p * n + j]);
            std::swap(b[k], b[p]);
        }
        for (int i = k + 1; i < n; ++i) {
            const double f = A[i * n + k] / A[k * n + k];
            for (int j = k; j < n; ++j) A[i * n + j] -= f * A[k * n + j];
            b[i] -= f * b[k];
        }
    }
    for (int i = n - 1; i >= 0; --i) {
        double s = b[i];
        for (int j = i + 1; j < n; ++j) s -= A[i * n + j] * b[j];
        b[i] = s / A[i * n + i];
    }
    return true;
}

double dcoef(const std::vector<double>& D, int i) { return i < (int)D.size() ? D[i] : 0.0; }

void distort(double x, double y, const std::vector<double>& D, double& xd, double& yd) {
    const double k1 = dcoef(D, 0), k2 = dcoef(D, 1), p1 = dcoef(D, 2), p2 = dcoef(D, 3), k3 = dcoef(D, 4);
    const double k4 = dcoef(D, 5), k5 = dcoef(D, 6), k6 = dcoef(D, 7);
    const double s1 = dcoef(D, 8), s2 = dcoef(D, 9), s3 = dcoef(D, 10), s4 = dcoef(D, 11);
    const double r2 = x * x + y * y, r4 = r2 * r2, r6 = r4 * r2;
    const double cd = (1 + k1 * r2 + k2 * r4 + k3 * r6) / (1 + k4 * r2 + k5 * r4 + k6 * r6);
    xd = x * cd + 2 * p1 * x * y + p2 * (r2 + 2 * x * x) + s1 * r2 + s2 * r4;
    yd = y * cd + p1 * (r2 + 2 * y * y) + 2 * p2 * x * y + s3 * r2 + s4 * r4;
}

// homography H (3 x 3, row-major) with H [X Y 1]^T ~ [x y 1]^T, normalised DLT
void homography(const double* XY, const double* xy, int n, double* H) {
    double mx = 0, my = 0, mu = 0, mv = 0;
    for (int i = 0; i < n; ++i) {
        mx += XY[2 * i]; my += XY[2 * i + 1];
        mu += xy[2 * i]; mv += xy[2 * i + 1];
    }
    mx /= n; my /= n; mu /= n; mv /= n;
    double sx = 0, su = 0;
    for (int i = 0; i < n; ++i) {
        sx += std::hypot(XY[2 * i] - mx, XY[2 * i + 1] - my);
        su += std::hypot(xy[2 * i] - mu, xy[2 * i + 1] - mv);
    }
    sx = std::sqrt(2.0) * n / std::max(sx, 1e-300);
    su = std::sqrt(2.0) * n / std::max(su, 1e-300);
    double AtA[81] = {0};
    for (int i = 0; i < n; ++i) {
        const double X = (XY[2 * i] - mx) * sx, Y = (XY[2 * i + 1] - my) * sx;
        const double u = (xy[2 * i] - mu) * su, v = (xy[2 * i + 1] - mv) * su;
        const double r1[9] = {X, Y, 1, 0, 0, 0, -u * X, -u * Y, -u};
        const double r2[9] = {0, 0, 0, X, Y, 1, -v * X, -v * Y, -v};
        for (int a = 0; a < 9; ++a)
            for (int b = 0; b < 9; ++b) AtA[a * 9 + b] += r1[a] * r1[b] + r2[a] * r2[b];
    }
    double w[9], V[81];
    jacobi_eig(AtA, 9, w, V);
    double Hn[9];
    for (int k = 0; k < 9; ++k) Hn[k] = V[k * 9 + 0];
    // H = Tu^-1 Hn Tx
    const double Tx[9] = {sx, 0, -sx * mx, 0, sx, -sx * my, 0, 0, 1};
    const double Tui[9] = {1 / su, 0, mu, 0, 1 / su, mv, 0, 0, 1};
    double T1[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double s = 0;
            for (int k = 0; k < 3; ++k) s += Hn[i * 3 + k] * Tx[k * 3 + j];
            T1[i * 3 + j] = s;
        }
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double s = 0;
            for (int k = 0; k < 3; ++k) s += Tui[i * 3 + k] * T1[k * 3 + j];
            H[i * 3 + j] = s;
        }
}

double rms_error(const double* object, const double* image, int n, const double* r, const double* t, const double* K,
                 const std::vector<double>& D, std::vector<double>& buf) {
    buf.resize(2 * (size_t)n);
    projectPoints(object, n, r, t, K, D, buf.data());
    double s = 0;
    for (int i = 0; i < 2 * n; ++i) s += (buf[i] - image[i]) * (buf[i] - image[i]);
    return std::sqrt(s / std::max(n, 1));
}

}  // namespace

void rodrigues(const double r[3], double R[9]) {
    const double th = std::sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
    if (th < 2.220446049250313e-16) {
        for (int k = 0; k < 9; ++k) R[k] = (k % 4 == 0) ? 1.0 : 0.0;
        return;
    }
    const double c = std::cos(th), s = std::sin(th), c1 = 1 - c;
    const double x = r[0] / th, y = r[1] / th, z = r[2] / th;
    const double rrt[9] = {x * x, x * y, x * z, x * y, y * y, y * z, x * z, y * z, z * z};
    const double rx[9] = {0, -z, y, z, 0, -x, -y, x, 0};
    for (int k = 0; k < 9; ++k) R[k] = c * ((k % 4 == 0) ? 1.0 : 0.0) + c1 * rrt[k] + s * rx[k];
}

void rodriguesInv(const double R[9], double r[3]) {
    double rx = R[7] - R[5], ry = R[2] - R[6], rz = R[3] - R[1];
    const double s = std::sqrt((rx * rx + ry * ry + rz * rz) * 0.25);
    double c = (R[0] + R[4] + R[8] - 1) * 0.5;
    c = c > 1. ? 1. : c < -1. ? -1. : c;
    double th = std::acos(c);
    if (s < 1e-5) {
        if (c > 0) {
            rx = ry = rz = 0;
        } else {
            double t = (R[0] + 1) * 0.5; rx = std::sqrt(std::max(t, 0.));
            t = (R[4] + 1) * 0.5; ry = std::sqrt(std::max(t, 0.)) * (R[1] < 0 ? -1. : 1.);
            t = (R[8] + 1) * 0.5; rz = std::sqrt(std::max(t, 0.)) * (R[2] < 0 ? -1. : 1.);
            if (std::fabs(rx) < std::fabs(ry) && std::fabs(rx) < std::fabs(rz) && (R[5] > 0) != (ry * rz > 0)) rz = -rz;
            th /= std::sqrt(rx * rx + ry * ry + rz * rz);
            rx *= th; ry *= th; rz *= th;
        }
    } else {
        const double v = th / (2 * s);
        rx *= v; ry *= v; rz *= v;
    }
    r[0] = rx; r[1] = ry; r[2] = rz;
}

void projectPoints(const double* object, int n, const double rvec[3], const double tvec[3], const double K[9],
                   const std::vector<double>& D, double* image) {
    double R[9];
    rodrigues(rvec, R);
    for (int i = 0; i < n; ++i) {
        const double* X = object + 3 * i;
        const double Xc = R[0] * X[0] + R[1] * X[1] + R[2] * X[2] + tvec[0];
        const double Yc = R[3] * X[0] + R[4] * X[1] + R[5] * X[2] + tvec[1];
        const double Zc = R[6] * X[0] + R[7] * X[1] + R[8] * X[2] + tvec[2];
        const double z = Zc != 0.0 ? 1.0 / Zc : 1.0;
        double xd, yd;
        distort(Xc * z, Yc * z, D, xd, yd);
        image[2 * i] = K[0] * xd + K[2];       // cv::projectPoints: fx, fy, cx, cy (no skew)
        image[2 * i + 1] = K[4] * yd + K[5];
    }
}

void undistortPoints(const double* image, int n, const double K[9], const std::vector<double>& D, double* xy,
                     int iterations) {
    const double k1 = dcoef(D, 0), k2 = dcoef(D, 1), p1 = dcoef(D, 2), p2 = dcoef(D, 3), k3 = dcoef(D, 4);
    const double k4 = dcoef(D, 5), k5 = dcoef(D, 6), k6 = dcoef(D, 7);
    const double s1 = dcoef(D, 8), s2 = dcoef(D, 9), s3 = dcoef(D, 10), s4 = dcoef(D, 11);
    for (int i = 0; i < n; ++i) {
        const double x0 = (image[2 * i] - K[2]) / K[0], y0 = (image[2 * i + 1] - K[5]) / K[4];
        double x = x0, y = y0;
        for (int it = 0; it < iterations; ++it) {
            const double r2 = x * x + y * y, r4 = r2 * r2, r6 = r4 * r2;
            const double icd = (1 + k4 * r2 + k5 * r4 + k6 * r6) / (1 + k1 * r2 + k2 * r4 + k3 * r6);
            const double dx = 2 * p1 * x * y + p2 * (r2 + 2 * x * x) + s1 * r2 + s2 * r4;
            const double dy = p1 * (r2 + 2 * y * y) + 2 * p2 * x * y + s3 * r2 + s4 * r4;
            x = (x0 - dx) * icd;
            y = (y0 - dy) * icd;
        }
        xy[2 * i] = x;
        xy[2 * i + 1] = y;
    }
}

double solvePnP(const double* object, const double* image, int n, const double K[9], const std::vector<double>& D,
                double rvec[3], double tvec[3]) {
    if (n < 4) return -1.0;
    std::vector<double> xy(2 * (size_t)n);
    undistortPoints(image, n, K, D, xy.data());
    // plane of the object points: centroid and the covariance's smallest eigenvector
    double c[3] = {0, 0, 0};
    for (int i = 0; i < n; ++i)
        for (int k = 0; k < 3; ++k) c[k] += object[3 * i + k] / n;
    double C[9] = {0};
    for (int i = 0; i < n; ++i)
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) C[a * 3 + b] += (object[3 * i + a] - c[a]) * (object[3 * i + b] - c[b]);
    double w[3], V[9];
    jacobi_eig(C, 3, w, V);
    double R[9], t[3];
    const bool planar = w[0] <= 1e-9 * std::max(w[2], 1e-300);
    if (planar) {
        // plane frame: Rp rows = (e2, e1, e0) (e0 = normal), X_plane = Rp (X - c)
        double Rp[9];
        for (int k = 0; k < 3; ++k) {
            Rp[0 * 3 + k] = V[k * 3 + 2];
            Rp[1 * 3 + k] = V[k * 3 + 1];
            Rp[2 * 3 + k] = V[k * 3 + 0];
        }
        const double det = Rp[0] * (Rp[4] * Rp[8] - Rp[5] * Rp[7]) - Rp[1] * (Rp[3] * Rp[8] - Rp[5] * Rp[6]) +
                           Rp[2] * (Rp[3] * Rp[7] - Rp[4] * Rp[6]);
        if (det < 0)
            for (int k = 0; k < 3; ++k) Rp[2 * 3 + k] = -Rp[2 * 3 + k];
        std::vector<double> XY(2 * (size_t)n);
        for (int i = 0; i < n; ++i) {
            const double d[3] = {object[3 * i] - c[0], object[3 * i + 1] - c[1], object[3 * i + 2] - c[2]};
            XY[2 * i] = Rp[0] * d[0] + Rp[1] * d[1] + Rp[2] * d[2];
            XY[2 * i + 1] = Rp[3] * d[0] + Rp[4] * d[1] + Rp[5] * d[2];
        }
        double H[9];
        homography(XY.data(), xy.data(), n, H);
        const double n1 = std::sqrt(H[0] * H[0] + H[3] * H[3] + H[6] * H[6]);
        const double n2 = std::sqrt(H[1] * H[1] + H[4] * H[4] + H[7] * H[7]);
        double lam = 1.0 / std::sqrt(n1 * n2);
        if (H[8] * lam < 0) lam = -lam;   // the plane origin in front of the camera
        double M[9];
        const double h1[3] = {H[0] * lam, H[3] * lam, H[6] * lam}, h2[3] = {H[1] * lam, H[4] * lam, H[7] * lam};
        const double h3[3] = {h1[1] * h2[2] - h1[2] * h2[1], h1[2] * h2[0] - h1[0] * h2[2], h1[0] * h2[1] - h1[1] * h2[0]};
        for (int k = 0; k < 3; ++k) {
            M[k * 3 + 0] = h1[k];
            M[k * 3 + 1] = h2[k];
            M[k * 3 + 2] = h3[k];
        }
        double Rh[9];
        nearest_rotation(M, Rh);
        const double th[3] = {H[2] * lam, H[5] * lam, H[8] * lam};
        // X_cam = Rh Rp (X - c) + th  ->  R = Rh Rp, t = th - R c
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) {
                double s = 0;
                for (int k = 0; k < 3; ++k) s += Rh[i * 3 + k] * Rp[k * 3 + j];
                R[i * 3 + j] = s;
            }
        for (int i = 0; i < 3; ++i) t[i] = th[i] - (R[i * 3] * c[0] + R[i * 3 + 1] * c[1] + R[i * 3 + 2] * c[2]);
    } else {
        if (n < 6) return -1.0;
        // DLT of P = [R | t] on normalized coordinates
        double AtA[144] = {0};
        for (int i = 0; i < n; ++i) {
            const double X = object[3 * i] - c[0], Y = object[3 * i + 1] - c[1], Z = object[3 * i + 2] - c[2];
            const double u = xy[2 * i], v = xy[2 * i + 1];
            const double r1[12] = {X, Y, Z, 1, 0, 0, 0, 0, -u * X, -u * Y, -u * Z, -u};
            const double r2[12] = {0, 0, 0, 0, X, Y, Z, 1, -v * X, -v * Y, -v * Z, -v};
            for (int a = 0; a < 12; ++a)
                for (int b = 0; b < 12; ++b) AtA[a * 12 + b] += r1[a] * r1[b] + r2[a] * r2[b];
        }
        double w12[12], V12[144];
        jacobi_eig(AtA, 12, w12, V12);
        double P[12];
        for (int k = 0; k < 12; ++k) P[k] = V12[k * 12];
        const double M[9] = {P[0], P[1], P[2], P[4], P[5], P[6], P[8], P[9], P[10]};
        double sc = std::cbrt(M[0] * (M[4] * M[8] - M[5] * M[7]) - M[1] * (M[3] * M[8] - M[5] * M[6]) +
                              M[2] * (M[3] * M[7] - M[4] * M[6]));
        if (sc == 0) return -1.0;
        double Ms[9];
        for (int k = 0; k < 9; ++k) Ms[k] = M[k] / sc;
        nearest_rotation(Ms, R);
        const double tc[3] = {P[3] / sc, P[7] / sc, P[11] / sc};
        for (int i = 0; i < 3; ++i) t[i] = tc[i] - (R[i * 3] * c[0] + R[i * 3 + 1] * c[1] + R[i * 3 + 2] * c[2]);
    }
    double r[3];
    rodriguesInv(R, r);
    // Levenberg-Marquardt on the reprojection error (numeric central-difference Jacobian)
    std::vector<double> buf, p0(2 * (size_t)n), pp(2 * (size_t)n), pm(2 * (size_t)n);
    double lambda = 1e-3;
    double err = rms_error(object, image, n, r, t, K, D, buf);
    for (int it = 0; it < 50; ++it) {
        double x[6] = {r[0], r[1], r[2], t[0], t[1], t[2]};
        projectPoints(object, n, x, x + 3, K, D, p0.data());
        std::vector<double> J(12 * (size_t)n);
        for (int k = 0; k < 6; ++k) {
            const double h = 1e-7 * std::max(1.0, std::fabs(x[k]));
            double xp[6], xm[6];
            std::memcpy(xp, x, sizeof xp);
            std::memcpy(xm, x, sizeof xm);
            xp[k] += h;
            xm[k] -= h;
            projectPoints(object, n, xp, xp + 3, K, D, pp.data());
            projectPoints(object, n, xm, xm + 3, K, D, pm.data());
            for (int i = 0; i < 2 * n; ++i) J[(size_t)i * 6 + k] = (pp[i] - pm[i]) / (2 * h);
        }
        double JtJ[36] = {0}, Jte[6] = {0};
        for (int i = 0; i < 2 * n; ++i) {
            const double e = image[i] - p0[i];
            for (int a = 0; a < 6; ++a) {
                Jte[a] += J[(size_t)i * 6 + a] * e;
                for (int b = 0; b < 6; ++b) JtJ[a * 6 + b] += J[(size_t)i * 6 + a] * J[(size_t)i * 6 + b];
            }
        }
        bool improved = false;
        for (int tries = 0; tries < 10 && !improved; ++tries) {
            double A[36], d[6];
            std::memcpy(A, JtJ, sizeof A);
            std::memcpy(d, Jte, sizeof d);
            for (int a = 0; a < 6; ++a) A[a * 6 + a] *= 1.0 + lambda;
            if (!solve6(A, d)) break;
            const double rn[3] = {r[0] + d[0], r[1] + d[1], r[2] + d[2]};
            const double tn[3] = {t[0] + d[3], t[1] + d[4], t[2] + d[5]};
            const double en = rms_error(object, image, n, rn, tn, K, D, buf);
            if (en <= err) {
                const double rel = (err - en) / std::max(err, 1e-300);
                std::memcpy(r, rn, sizeof r);
                std::memcpy(t, tn, sizeof t);
                err = en;
                lambda = std::max(lambda * 0.1, 1e-12);
                improved = true;
                if (rel < 1e-14) it = 1000;   // converged
            } else {
                lambda *= 10.0;
            }
        }
        if (!improved) break;
    }
    std::memcpy(rvec, r, sizeof r);
    std::memcpy(tvec, t, sizeof t);
    return err;
}

}  // namespace pnp
}  // namespace mcc
