/*
 * opencv2/ccalib/multicalib.hpp -- source-compatible stand-in for the reference's header of the
 * same path (include/opencv2/ccalib/multicalib.hpp:73-252): cv::multicalib::MultiCameraCalibration
 * and the OpenCV value types its callers name (cv::Size, cv::TermCriteria, cv::Mat -- the minimal
 * cv::Mat of mcc_cvmat.hpp), so code written against the reference compiles against this build and
 * runs the bundle adjustment on the MI355X: its sample samples/multi_cameras_calibration.cpp byte
 * for byte, and subclasses written the way the reference writes MyMultiCameraCalibration and
 * DoubleSideCalibration, through the reference's cv::Mat-typed extension seam.
 *
 * The names resolve to the C++ host layer over the C ABI (mcc_multicalib.hpp -> libmcc_host.so,
 * libmcc.so).  Constructors, methods and defaults follow the reference:
 *   MultiCameraCalibration(cameraType, nCameras, fileName, patternWidth, patternHeight, verbose,
 *       showExtration, nMiniMatches, flags, TermCriteria(COUNT, 20, 1e-7))  multicalib.hpp:138-143
 *   loadImages() :147, initialize() :151, optimizeExtrinsics() :155, conjungate() :157, run() :161,
 *   reset() :162, writeParameters(const std::string&) :165
 *   protected, virtual: computeJacobianExtrinsic(const Mat&, Mat&, Mat&, Mat&) :176,
 *   computePhotoCameraJacobian(...) :178-180, computeProjectError(Mat&) :188,
 *   vector2parameters(...) :190, buildParas() :239, paras2vertex(const Mat&) :241;
 *   non-virtual: compose_motion(...) :182-183, parameters2vector(...) :191, isValidPose(...),
 *   IsvalidImagePoints(...).
 * (The feature detector / descriptor / matcher arguments are dropped: image feature matching is
 * outside this build, which reads pre-detected corners.)  Errors throw std::runtime_error where the
 * reference's CV_Assert / CV_Error throw cv::Exception; its asserts abort in strict-reference mode
 * (strictReference = true or MCC_STRICT_REFERENCE=1).
 *
 * optimizeExtrinsics: on the library's own classes it is the device loop (mcc_optimize: the whole
 * Gauss-Newton loop on the GPU).  On a subclass -- whose overrides of the seam must be honoured --
 * and in strict-reference mode it is the reference's loop (src/multicalib.cpp:462-514) on the host,
 * calling this object's virtual computeJacobianExtrinsic (by default one GPU linearisation + solve),
 * computeProjectError, buildParas and paras2vertex exactly where the reference does.
 * computePhotoCameraJacobian is the reference's per-edge CPU Jacobian (base :717-824, MyMulti
 * src/mymulticalib.cpp:468-614, DoubleSide src/doubleSide.cpp:288-430), restated on the host
 * (mcc::multicalib::edgeJacobian, libmcc_host.so): the library's own loop linearises whole steps on
 * the GPU and never calls it, but a subclass whose computeJacobianExtrinsic assembles the dense J
 * edge by edge the way the reference's does gets the reference's per-edge blocks from it.  The
 * per-view state such a body reads is offered as cv::Mat too (objectPointsMat, imagePointsMat,
 * cameraMatrixMat, distortCoeffsMat, xiMat, transformMat; MyMulti's doubleSideTransform_rvec /
 * _tvec, DoubleSide's camerasPose_rvec / _tvec as functions).  Build: -I<repo>/include/opencv2/ccalib
 * -I<repo>/include, link -lmcc_host -lmcc.
 */
#ifndef MCC_CV_MULTICALIB_HPP
#define MCC_CV_MULTICALIB_HPP

#if defined(OPENCV_CORE_HPP) || defined(OPENCV_CORE_MAT_HPP)
// the seam reads cv::Mat through the in-repo shim's accessors (mcc_cvmat.hpp): it is this build's
// stand-in for OpenCV, not an extension of it
#error "include/opencv2/ccalib/*.hpp replace OpenCV's cv::multicalib headers; do not include OpenCV before them"
#endif

#include <cstdio>
#include <iostream>
#include <set>
#include <stdexcept>
#include <string>
#include <typeinfo>
#include <vector>

#include "../../mcc_cvmat.hpp"
#include "../../mcc_multicalib.hpp"

namespace cv {

using Size = mcc::multicalib::Size;                 // cv::Size(width, height)
using TermCriteria = mcc::multicalib::TermCriteria;   // COUNT = MAX_ITER = 1, EPS = 2

namespace multicalib {
namespace detail {

inline Mat row_f32(const std::vector<float>& v) {   // 1 x P CV_32F (buildParas' shape)
    Mat m(1, (int)v.size(), CV_32F);
    for (size_t i = 0; i < v.size(); ++i) m.at<float>(0, (int)i) = v[i];
    return m;
}
inline Mat col_f64(const std::vector<double>& v) {   // P x 1 CV_64F (deltaX / JTE shape)
    Mat m((int)v.size(), 1, CV_64F);
    for (size_t i = 0; i < v.size(); ++i) m.at<double>((int)i, 0) = v[i];
    return m;
}
inline std::vector<float> to_f32(const Mat& m) {   // any 1 x P / P x 1 parameter vector
    std::vector<float> v;
    v.reserve(m.total());
    for (int r = 0; r < m.rows; ++r)
        for (int c = 0; c < m.cols; ++c) v.push_back((float)m.get(r, c));
    return v;
}

// small dense helpers of compose_motion (row-major 3 x 3, double)
inline void so3_poly(const double w[3], double s1, double s2, double M[9]) {   // I + s1 [w]x + s2 [w]x^2
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
inline void mat3(const double* A, const double* B, double* C) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) C[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
}
// left / right SO(3) Jacobian of w: I +- a [w]x + b [w]x^2, and their inverses
inline void so3_jac(const double w[3], double sign, bool inverse, double J[9]) {
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
inline Mat mat33(const double* v) {
    Mat m(3, 3, CV_64F);
    for (int k = 0; k < 9; ++k) m.at<double>(k / 3, k % 3) = v[k];
    return m;
}
inline void vec3(const Mat& m, double v[3]) {
    for (int k = 0; k < 3; ++k) v[k] = m.rows == 1 ? m.get(0, k) : m.get(k, 0);
}
// every scalar of a matrix (any channel count) in row-major order, as float
inline std::vector<float> flat_f32(const Mat& m) {
    std::vector<float> v;
    v.reserve(m.total() * m.channels());
    for (int r = 0; r < m.rows; ++r)
        for (int c = 0; c < m.cols * m.channels(); ++c)
            v.push_back(m.depth() == CV_64F ? (float)m.ptr<double>(r)[c] : m.ptr<float>(r)[c]);
    return v;
}
inline Mat rows_f32(const std::vector<float>& v, int width) {   // n x width CV_32F
    Mat m((int)(v.size() / width), width, CV_32F);
    for (size_t i = 0; i < v.size(); ++i) m.at<float>((int)(i / width), (int)(i % width)) = v[i];
    return m;
}
// the reference's per-edge computePhotoCameraJacobian on cv::Mat arguments: jacobianPhoto /
// jacobianGlobal (2N x 6 CV_64F), E (2N x 1 CV_64F, rows u0, v0, u1, ...); rvecTran / tvecTran
// (3 x 1 CV_32F) when given (the base class's version assigns them, MyMulti's and DoubleSide's do not)
inline void edge_jacobian_mats(int edgeClass, bool omni, int patternSide, const Mat& rP, const Mat& tP, const Mat& rC,
                               const Mat& tC, const Mat* rDs, const Mat* tDs, const Mat& objectPoints,
                               const Mat& imagePoints, const Mat& K, const Mat& distort, const Mat& xi,
                               Mat& jacobianPhoto, Mat& jacobianGlobal, Mat& E, Mat* rvecTran, Mat* tvecTran) {
    double rp[3], tp[3], rc[3], tc[3], rd[3] = {0, 0, 0}, td[3] = {0, 0, 0};
    vec3(rP, rp); vec3(tP, tp); vec3(rC, rc); vec3(tC, tc);
    const bool ds = rDs && tDs && !rDs->empty() && !tDs->empty();
    if (ds) { vec3(*rDs, rd); vec3(*tDs, td); }
    const std::vector<float> obj = flat_f32(objectPoints), img = flat_f32(imagePoints), k = flat_f32(K);
    const std::vector<float> d = flat_f32(distort);
    const int n = (int)(obj.size() / 3);
    if (obj.size() != 3 * (size_t)n || img.size() != 2 * (size_t)n || k.size() != 9)
        throw std::runtime_error("computePhotoCameraJacobian: objectPoints N x 3, imagePoints N x 2, K 3 x 3");
    const float xif = omni && !xi.empty() ? flat_f32(xi)[0] : 0.f;
    mcc::multicalib::EdgeLinearization L;
    mcc::multicalib::edgeJacobian(edgeClass, omni, patternSide, rp, tp, rc, tc, ds ? rd : nullptr, ds ? td : nullptr, n,
                                  obj.data(), img.data(), k.data(), d.data(), (int)d.size(), xif, L);
    jacobianPhoto = Mat(2 * n, 6, CV_64F);
    jacobianGlobal = Mat(2 * n, 6, CV_64F);
    E = Mat(2 * n, 1, CV_64F);
    for (int r = 0; r < 2 * n; ++r) {
        for (int c = 0; c < 6; ++c) {
            jacobianPhoto.at<double>(r, c) = L.jacPhoto[6 * (size_t)r + c];
            jacobianGlobal.at<double>(r, c) = L.jacGlobal[6 * (size_t)r + c];
        }
        E.at<double>(r, 0) = L.E[r];
    }
    if (rvecTran && tvecTran) {
        *rvecTran = Mat(3, 1, CV_32F);
        *tvecTran = Mat(3, 1, CV_32F);
        for (int q = 0; q < 3; ++q) {
            rvecTran->at<float>(q, 0) = L.rvecTranF[q];
            tvecTran->at<float>(q, 0) = L.tvecTranF[q];
        }
    }
}

// The reference's cv::Mat-typed seam over one of the host layer's classes (Impl), for the
// cv::multicalib class Self that derives from it.
template <class Impl, class Self>
class Seam : public Impl {
public:
    using Impl::Impl;

    // optimizeExtrinsics (multicalib.hpp:155, src/multicalib.cpp:462-514): the device loop for the
    // library's own class; the reference's host loop through the virtual seam for a subclass
    double optimizeExtrinsics() {
        if (typeid(*this) == typeid(Self) && !this->strictReference) return Impl::optimizeExtrinsics();
        if (this->strictReference)
            for (const auto& e : this->_edgeList) {
                const float t[3] = {e.transform[3], e.transform[7], e.transform[11]};
                if (!mcc::multicalib::valid_pose(t)) mcc::multicalib::strict_abort("isValidPose(Tvectran)", "src/mymulticalib.cpp:706");
            }
        Mat extrinParam = buildParas();
        double change = 1;
        int iter = 0;
        const TermCriteria& cr = this->_criteria;
        for (;; ++iter) {
            if ((cr.type == 1 && iter >= cr.maxCount) || (cr.type == 2 && change <= cr.epsilon) ||
                (cr.type == 3 && (change <= cr.epsilon || iter >= cr.maxCount)))
                break;
            if (this->strictReference) this->checkIterate(detail::to_f32(extrinParam));
            const double alpha_smooth2 = std::pow(0.95, (double)iter + 1.0);
            Mat JTJ_inv, JTError, deltx;
            this->computeJacobianExtrinsic(extrinParam, JTJ_inv, JTError, deltx);
            Mat G = alpha_smooth2 * deltx;
            if (G.depth() == CV_64F) G.convertTo(G, CV_32F);
            const Mat Gt = G.reshape(1, 1);
            const bool print = this->verboseOn();   // src/multicalib.cpp:492, 499-500, 506
            if (print) {
                std::printf("alpha_smooth2:%s \n", this->cout_str(alpha_smooth2).c_str());
                this->print_row("extrinParam:", detail::to_f32(extrinParam));
                this->print_row("Gt:", detail::to_f32(Gt));
            }
            extrinParam = extrinParam + Gt;
            change = norm(G) / norm(extrinParam);
            if (print) std::printf("iter:%d" "change:%s\n", iter, this->cout_str(change).c_str());
        }
        this->_iters = iter;
        this->_change = change;
        const double error = computeProjectError(extrinParam);
        paras2vertex(extrinParam);
        this->_error = error;
        return error;
    }

    // conjungate (multicalib.hpp:157, src/multicalib.cpp:580-592): x = a^-1 b for the symmetric
    // positive definite a (JTJ) and right-hand side(s) b, in CV_64F.  The reference runs Eigen's
    // Jacobi-preconditioned CG to DBL_EPSILON (twice, sparseSolver :565-579); this is the exact
    // solution by a host Cholesky factorisation, the same to within the CG's tolerance.
    Mat conjungate(const Mat& a, const Mat& b) {
        const int n = a.rows;
        if (a.cols != n || b.rows != n) throw std::runtime_error("conjungate: a must be n x n and b n x k");
        std::vector<double> L((size_t)n * n, 0.0);
        for (int j = 0; j < n; ++j) {
            double d = a.get(j, j);
            for (int k = 0; k < j; ++k) d -= L[(size_t)j * n + k] * L[(size_t)j * n + k];
            if (!(d > 0.0)) throw std::runtime_error("conjungate: the matrix is not positive definite");
            const double s = std::sqrt(d);
            L[(size_t)j * n + j] = s;
            for (int i = j + 1; i < n; ++i) {
                double v = a.get(i, j);
                for (int k = 0; k < j; ++k) v -= L[(size_t)i * n + k] * L[(size_t)j * n + k];
                L[(size_t)i * n + j] = v / s;
            }
        }
        Mat x(n, b.cols, CV_64F);
        for (int c = 0; c < b.cols; ++c) {
            std::vector<double> y(n);
            for (int i = 0; i < n; ++i) {
                double v = b.get(i, c);
                for (int k = 0; k < i; ++k) v -= L[(size_t)i * n + k] * y[k];
                y[i] = v / L[(size_t)i * n + i];
            }
            for (int i = n - 1; i >= 0; --i) {
                double v = y[i];
                for (int k = i + 1; k < n; ++k) v -= L[(size_t)k * n + i] * x.at<double>(k, c);
                x.at<double>(i, c) = v / L[(size_t)i * n + i];
            }
        }
        return x;
    }

protected:
    // computeJacobianExtrinsic (multicalib.hpp:176): deltaX and JTE (P x 1, CV_64F) at the 1 x P
    // CV_32F parameters; JTJ_inv stays empty (the reference allocates it and never reads it,
    // src/mymulticalib.cpp:680).  One linearisation + normal-equation solve on the GPU.
    virtual void computeJacobianExtrinsic(const Mat& extrinsicParams, Mat& JTJ_inv, Mat& JTE, Mat& deltaX) {
        std::vector<double> jinv, jte, dx;
        Impl::computeJacobianExtrinsic(detail::to_f32(extrinsicParams), jinv, jte, dx);
        JTJ_inv = Mat();
        JTE = detail::col_f64(jte);
        deltaX = detail::col_f64(dx);
    }
    // computeProjectError (multicalib.hpp:188): every edge's reprojecterror and the mean
    virtual double computeProjectError(Mat& parameters) {
        std::vector<float> x = detail::to_f32(parameters);
        return Impl::computeProjectError(x);
    }
    // buildParas / paras2vertex (multicalib.hpp:239-241; src/multicalib.cpp:422-459)
    virtual Mat buildParas() { return detail::row_f32(Impl::buildParaVector()); }
    virtual void paras2vertex(const Mat& extrinParam) { Impl::paras2vertex(detail::to_f32(extrinParam)); }
    // vector2parameters / parameters2vector (multicalib.hpp:190-191, src/multicalib.cpp:1058-1090):
    // the 1 x P row <-> per-vertex (rvec, tvec)
    virtual void vector2parameters(const Mat& parameters, std::vector<Vec3f>& rvecVertex, std::vector<Vec3f>& tvecVertexs) {
        const std::vector<float> x = detail::to_f32(parameters);
        if (x.size() % 6) throw std::runtime_error("vector2parameters: the parameter count is not a multiple of 6");
        rvecVertex.assign(x.size() / 6, Vec3f());
        tvecVertexs.assign(x.size() / 6, Vec3f());
        for (size_t i = 0; i < x.size() / 6; ++i)
            for (int k = 0; k < 3; ++k) {
                rvecVertex[i][k] = x[6 * i + k];
                tvecVertexs[i][k] = x[6 * i + 3 + k];
            }
    }
    void parameters2vector(const std::vector<Vec3f>& rvecVertex, const std::vector<Vec3f>& tvecVertex, Mat& parameters) {
        if (rvecVertex.size() != tvecVertex.size()) throw std::runtime_error("parameters2vector: sizes differ");
        parameters = Mat(1, (int)(6 * rvecVertex.size()), CV_32F);
        for (size_t i = 0; i < rvecVertex.size(); ++i)
            for (int k = 0; k < 3; ++k) {
                parameters.at<float>(0, (int)(6 * i + k)) = rvecVertex[i][k];
                parameters.at<float>(0, (int)(6 * i + 3 + k)) = tvecVertex[i][k];
            }
    }
    // compose_motion (multicalib.hpp:182-183, src/multicalib.cpp:1008-1056): R3 = R2 R1,
    // T3 = R2 T1 + T2 and the eight 3 x 3 partials; the rotation partials in closed form
    // (dom3/dom1 = Jr^-1(om3) Jr(om1), dom3/dom2 = Jl^-1(om3) Jl(om2), dT3/dom2 = -[R2 T1]x Jl(om2)),
    // the derivatives the reference's Rodrigues / matMulDeriv chains evaluate numerically
    void compose_motion(InputArray _om1, InputArray _T1, InputArray _om2, InputArray _T2, Mat& om3, Mat& T3,
                        Mat& dom3dom1, Mat& dom3dT1, Mat& dom3dom2, Mat& dom3dT2, Mat& dT3dom1, Mat& dT3dT1,
                        Mat& dT3dom2, Mat& dT3dT2) {
        double om1[3], T1[3], om2[3], T2[3];
        detail::vec3(_om1, om1);
        detail::vec3(_T1, T1);
        detail::vec3(_om2, om2);
        detail::vec3(_T2, T2);
        auto rod = [](const double w[3], double R[9]) {
            const double th = std::sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
            if (th < 2.220446049250313e-16) {
                for (int k = 0; k < 9; ++k) R[k] = k % 4 == 0 ? 1.0 : 0.0;
                return;
            }
            const double c = std::cos(th), s = std::sin(th), c1 = 1.0 - c;
            const double x = w[0] / th, y = w[1] / th, z = w[2] / th;
            const double rrt[9] = {x * x, x * y, x * z, x * y, y * y, y * z, x * z, y * z, z * z};
            const double rx[9] = {0, -z, y, z, 0, -x, -y, x, 0};
            for (int k = 0; k < 9; ++k) R[k] = c * (k % 4 == 0 ? 1.0 : 0.0) + c1 * rrt[k] + s * rx[k];
        };
        double R1[9], R2[9], R3[9], q[3], T[3];
        rod(om1, R1);
        rod(om2, R2);
        detail::mat3(R2, R1, R3);
        for (int i = 0; i < 3; ++i) {
            q[i] = R2[3 * i] * T1[0] + R2[3 * i + 1] * T1[1] + R2[3 * i + 2] * T1[2];
            T[i] = q[i] + T2[i];
        }
        float Rf[9], r3f[3];
        for (int k = 0; k < 9; ++k) Rf[k] = (float)R3[k];
        double om[3];
        {   // cvRodrigues2 matrix -> vector in double
            const double rx = R3[7] - R3[5], ry = R3[2] - R3[6], rz = R3[3] - R3[1];
            const double s = std::sqrt((rx * rx + ry * ry + rz * rz) * 0.25);
            double c = (R3[0] + R3[4] + R3[8] - 1) * 0.5;
            c = c > 1. ? 1. : c < -1. ? -1. : c;
            const double th = std::acos(c);
            if (s < 1e-5) {   // the ~0 / ~pi branches: the float helper's branch logic
                mcc::multicalib::rodrigues_m2v(Rf, r3f);
                for (int k = 0; k < 3; ++k) om[k] = r3f[k];
            } else {
                const double v = th / (2 * s);
                om[0] = rx * v; om[1] = ry * v; om[2] = rz * v;
            }
        }
        double Jr1[9], Jl2[9], Jri3[9], Jli3[9], A1[9], A2[9], B2[9];
        detail::so3_jac(om1, -1.0, false, Jr1);
        detail::so3_jac(om2, +1.0, false, Jl2);
        detail::so3_jac(om, -1.0, true, Jri3);
        detail::so3_jac(om, +1.0, true, Jli3);
        detail::mat3(Jri3, Jr1, A1);
        detail::mat3(Jli3, Jl2, A2);
        const double qx[9] = {0, q[2], -q[1], -q[2], 0, q[0], q[1], -q[0], 0};   // -[q]x
        detail::mat3(qx, Jl2, B2);
        const double Z[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
        om3 = Mat(3, 1, CV_64F);
        T3 = Mat(3, 1, CV_64F);
        for (int k = 0; k < 3; ++k) {
            om3.at<double>(k, 0) = om[k];
            T3.at<double>(k, 0) = T[k];
        }
        dom3dom1 = detail::mat33(A1);
        dom3dT1 = detail::mat33(Z);
        dom3dom2 = detail::mat33(A2);
        dom3dT2 = detail::mat33(Z);
        dT3dom1 = detail::mat33(Z);
        dT3dT1 = detail::mat33(R2);
        dT3dom2 = detail::mat33(B2);
        dT3dT2 = detail::mat33(I);
    }
    // isValidPose (src/multicalib.cpp:107-126) and IsvalidImagePoints (:704-715, which asserts)
    bool isValidPose(const Mat& tvec) {
        const float t[3] = {(float)tvec.at<float>(0), (float)tvec.at<float>(1), (float)tvec.at<float>(2)};
        return mcc::multicalib::valid_pose(t);
    }
    bool isValidPose(const Vec3f& tvecVertex) {
        const float t[3] = {tvecVertex[0], tvecVertex[1], tvecVertex[2]};
        return mcc::multicalib::valid_pose(t);
    }
    bool IsvalidImagePoints(const Mat& imagePoints2) {
        for (int r = 0; r < imagePoints2.rows; r++) {
            const float x = imagePoints2.at<float>(r, 0), y = imagePoints2.at<float>(r, 1);
            if (!(x >= 0 && y >= 0)) mcc::multicalib::strict_abort("x >= 0 && y >= 0", "src/multicalib.cpp:711");
            if (!(x < 1920 && y < 1080)) mcc::multicalib::strict_abort("x < 1920 && y < 1080", "src/multicalib.cpp:712");
        }
        return true;
    }
    // the per-view state (multicalib.hpp:207-214) as the reference's cv::Mat types, for a subclass
    // body written against them: corners N x 3 / N x 2 CV_32F, K 3 x 3, distortion 1 x nd, xi 1 x 1,
    // an edge's transform 4 x 4 (all CV_32F, copies)
    Mat objectPointsMat(int camera, int photoIndex) const {
        return rows_f32(this->_objectPointsForEachCamera.at(camera).at(photoIndex), 3);
    }
    Mat imagePointsMat(int camera, int photoIndex) const {
        return rows_f32(this->_imagePointsForEachCamera.at(camera).at(photoIndex), 2);
    }
    Mat cameraMatrixMat(int camera) const {
        const auto& k = this->_cameraMatrix.at(camera);
        return rows_f32(std::vector<float>(k.begin(), k.end()), 3);
    }
    Mat distortCoeffsMat(int camera) const {
        const auto& d = this->_distortCoeffs.at(camera);
        return rows_f32(d, (int)std::max<size_t>(d.size(), 1));
    }
    Mat xiMat(int camera) const { return rows_f32(std::vector<float>(1, this->_xi.at(camera)), 1); }
    template <class Edge>
    Mat transformMat(const Edge& e) const { return rows_f32(std::vector<float>(e.transform.begin(), e.transform.end()), 4); }
};

}  // namespace detail

class MultiCameraCalibration
    : public detail::Seam<mcc::multicalib::MultiCameraCalibration, MultiCameraCalibration> {
public:
    using detail::Seam<mcc::multicalib::MultiCameraCalibration, MultiCameraCalibration>::Seam;

protected:
    // computePhotoCameraJacobian (multicalib.hpp:178-180, src/multicalib.cpp:717-824): one edge's
    // Jacobians w.r.t. the photo and the camera, the residual, and the composed pose (CV_32F) in
    // rvecTran / tvecTran; the camera model is _camType's (projectPoints / omnidir::projectPoints)
    virtual void computePhotoCameraJacobian(const Mat& rvecPhoto, const Mat& tvecPhoto, const Mat& rvecCamera,
                                            const Mat& tvecCamera, Mat& rvecTran, Mat& tvecTran,
                                            const Mat& objectPoints, const Mat& imagePoints, const Mat& K,
                                            const Mat& distort, const Mat& xi, Mat& jacobianPhoto,
                                            Mat& jacobianCamera, Mat& E) {
        detail::edge_jacobian_mats(mcc::multicalib::EDGE_BASE, this->_camType == OMNIDIRECTIONAL, FRONT_PATTERN,
                                   rvecPhoto, tvecPhoto, rvecCamera, tvecCamera, nullptr, nullptr, objectPoints,
                                   imagePoints, K, distort, xi, jacobianPhoto, jacobianCamera, E, &rvecTran, &tvecTran);
    }
};

}  // namespace multicalib
}  // namespace cv

#endif
