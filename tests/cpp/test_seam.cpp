// The reference's cv::Mat-typed extension seam, compiled against this build's source-compatible
// headers (include/opencv2/ccalib/*.hpp over include/mcc_cvmat.hpp): subclasses written the way the
// reference writes MyMultiCameraCalibration and DoubleSideCalibration (overriding the protected
// virtuals of mymulticalib.hpp:164-172 / doubleSide.hpp:133-165 with their cv::Mat signatures).
// Built and run by tests/test_cpp_host.py:
//
//   test_seam selftest              host only (no GPU): the cv::Mat shim, conjungate (public,
//                                   multicalib.hpp:157) against a direct solve, compose_motion's
//                                   partials against central differences, the per-edge Jacobian
//                                   (shapes, the FRONT / BACK / DoubleSide block structure), and
//                                   that the subclasses construct
//   test_seam strict                strict-reference mode: an edge whose stored transform fails
//                                   isValidPose aborts optimizeExtrinsics (src/mymulticalib.cpp:706)
//   test_seam run <in.bin>          (GPU) a fixture problem (tests/cpp blob, see test_multicalib.cpp)
//                                   optimised by the library class (the device loop) and by the
//                                   counting subclass (the reference's host loop through the
//                                   overridden virtuals): same iterations, parameters, error; the
//                                   overrides called where the reference calls them
//   test_seam refstyle <in.bin>     (GPU) a subclass whose computeJacobianExtrinsic is the
//                                   reference's body (src/mymulticalib.cpp:668-818,
//                                   src/doubleSide.cpp:434-581): the dense J assembled edge by edge
//                                   from computePhotoCameraJacobian, J^T J, J^T E, conjungate -- all
//                                   on the host -- against the library's GPU linearisation (deltaX,
//                                   JTE) and, through the reference's host loop, its device loop
#include "opencv2/ccalib/doubleSide.hpp"

#include <cstdio>
#include <cstring>
#include <fstream>
#include <memory>
#include <random>
#include <type_traits>

static int g_fail = 0;
#define EXPECT(c)                                                              \
    do {                                                                       \
        if (!(c)) {                                                            \
            std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
            ++g_fail;                                                          \
        }                                                                      \
    } while (0)

// ---- subclasses as the reference writes them (mymulticalib.hpp:164-172, doubleSide.hpp:133-165)
struct Calls {
    int jac = 0, err = 0, build = 0, p2v = 0, edge = 0;
};
class CountingMyMulti : public cv::multicalib::MyMultiCameraCalibration {
public:
    using MyMultiCameraCalibration::MyMultiCameraCalibration;
    Calls calls;
    // expose the protected helpers for the host-only checks
    void composeMotion(const Mat& om1, const Mat& T1, const Mat& om2, const Mat& T2, std::vector<Mat>& out) {
        out.assign(10, Mat());
        compose_motion(om1, T1, om2, T2, out[0], out[1], out[2], out[3], out[4], out[5], out[6], out[7], out[8], out[9]);
    }
    void edgeJacobian(int side, const Mat& rP, const Mat& tP, const Mat& rC, const Mat& tC, const Mat& rD, const Mat& tD,
                      Mat& rt, Mat& tt, const Mat& obj, const Mat& img, const Mat& K, const Mat& D, const Mat& xi,
                      Mat& jp, Mat& jc, Mat& e) {
        MyMultiCameraCalibration::computePhotoCameraJacobian(side, rP, tP, rC, tC, rD, tD, rt, tt, obj, img, K, D, xi, jp,
                                                             jc, e);
    }

protected:
    virtual void computeJacobianExtrinsic(const Mat& extrinsicParams, Mat& JTJ_inv, Mat& JTE, Mat& deltaX) override {
        ++calls.jac;
        MyMultiCameraCalibration::computeJacobianExtrinsic(extrinsicParams, JTJ_inv, JTE, deltaX);
        EXPECT(deltaX.rows == (int)extrinsicParams.total() && deltaX.cols == 1 && deltaX.type() == CV_64F);
        EXPECT(JTE.rows == deltaX.rows && JTJ_inv.empty());
    }
    virtual void computePhotoCameraJacobian(int patternSide, const Mat& RvecPhoto, const Mat& TvecPhoto,
                                            const Mat& RvecCamera, const Mat& TvecCamera, const Mat& RvecDoubleside,
                                            const Mat& TvecDoubleside, Mat& Rvectran, Mat& Tvectran,
                                            const Mat& objectPoints, const Mat& imagePoints, const Mat& K,
                                            const Mat& distort, const Mat& xi, Mat& jacobianPhoto,
                                            Mat& jacobianDoubleside, Mat& E) override {
        ++calls.edge;
        (void)patternSide; (void)RvecPhoto; (void)TvecPhoto; (void)RvecCamera; (void)TvecCamera; (void)RvecDoubleside;
        (void)TvecDoubleside; (void)Rvectran; (void)Tvectran; (void)objectPoints; (void)imagePoints; (void)K;
        (void)distort; (void)xi; (void)jacobianPhoto; (void)jacobianDoubleside; (void)E;
    }
    virtual double computeProjectError(Mat& parameters) override {
        ++calls.err;
        return MyMultiCameraCalibration::computeProjectError(parameters);
    }
    virtual cv::Mat buildParas() override {
        ++calls.build;
        return MyMultiCameraCalibration::buildParas();
    }
    virtual void paras2vertex(const cv::Mat& extrinParam) override {
        ++calls.p2v;
        MyMultiCameraCalibration::paras2vertex(extrinParam);
    }
};
class CountingDoubleSide : public cv::multicalib::DoubleSideCalibration {
public:
    using DoubleSideCalibration::DoubleSideCalibration;
    Calls calls;
    void edgeJacobian(int side, const Mat& rP, const Mat& tP, const Mat& rC, const Mat& tC, const Mat& rD, const Mat& tD,
                      Mat& rt, Mat& tt, const Mat& obj, const Mat& img, const Mat& K, const Mat& D, const Mat& xi,
                      Mat& jp, Mat& jg, Mat& e) {
        DoubleSideCalibration::computePhotoCameraJacobian(side, rP, tP, rC, tC, rD, tD, rt, tt, obj, img, K, D, xi, jp,
                                                          jg, e);
    }

protected:
    virtual void computeJacobianExtrinsic(const Mat& extrinsicParams, Mat& JTJ_inv, Mat& JTE, Mat& deltaX) override {
        ++calls.jac;
        DoubleSideCalibration::computeJacobianExtrinsic(extrinsicParams, JTJ_inv, JTE, deltaX);
    }
    virtual double computeProjectError(Mat& parameters) override {
        ++calls.err;
        return DoubleSideCalibration::computeProjectError(parameters);
    }
    virtual cv::Mat buildParas() override {
        ++calls.build;
        return DoubleSideCalibration::buildParas();
    }
    virtual void paras2vertex(const cv::Mat& extrinParam) override {
        ++calls.p2v;
        DoubleSideCalibration::paras2vertex(extrinParam);
    }
};
// the reference's public interface on a subclass pointer, as its sample uses it
class PublicConjungate : public cv::multicalib::MultiCameraCalibration {
public:
    using MultiCameraCalibration::MultiCameraCalibration;
};

// computeJacobianExtrinsic written as the reference writes it (src/mymulticalib.cpp:668-818 for
// MyMulti, src/doubleSide.cpp:434-581 for DoubleSide): per edge, slice the photo and camera (or ds)
// parameters, call the per-edge computePhotoCameraJacobian, copy its blocks into the dense J and E;
// then JTJ = J^T J, JTE = J^T E, deltaX = conjungate(JTJ, JTE).  Everything on the host: the per-edge
// Jacobian is the build's host restatement, the product and the solve the cv::Mat shim's.
template <class Base>
class RefStyle : public Base {
public:
    using Base::Base;
    int edgeCalls = 0;
    void jacobianAt(const Mat& x, Mat& JTE, Mat& deltaX) {
        Mat jinv;
        this->computeJacobianExtrinsic(x, jinv, JTE, deltaX);
    }
    void libraryJacobianAt(const Mat& x, Mat& JTE, Mat& deltaX) {   // the GPU linearisation (the seam's default)
        Mat jinv;
        Base::computeJacobianExtrinsic(x, jinv, JTE, deltaX);
    }
    Mat params() { return this->buildParas(); }

protected:
    static constexpr bool kDoubleSide = std::is_base_of<cv::multicalib::DoubleSideCalibration, Base>::value ||
                                        std::is_same<cv::multicalib::DoubleSideCalibration, Base>::value;
    void computePhotoCameraJacobian(int patternSide, const Mat& rvecPhoto, const Mat& tvecPhoto, const Mat& rvecCamera,
                                    const Mat& tvecCamera, const Mat& rvecDoubleside, const Mat& tvecDoubleside,
                                    Mat& rvecTran, Mat& tvecTran, const Mat& objectPoints, const Mat& imagePoints,
                                    const Mat& K, const Mat& distort, const Mat& xi, Mat& jacobianPhoto,
                                    Mat& jacobianGlobal, Mat& E) override {
        ++edgeCalls;
        Base::computePhotoCameraJacobian(patternSide, rvecPhoto, tvecPhoto, rvecCamera, tvecCamera, rvecDoubleside,
                                         tvecDoubleside, rvecTran, tvecTran, objectPoints, imagePoints, K, distort, xi,
                                         jacobianPhoto, jacobianGlobal, E);
    }
    void computeJacobianExtrinsic(const Mat& extrinsicParams, Mat& JTJ_inv, Mat& JTE, Mat& deltaX) override {
        const int nParam = (int)extrinsicParams.total();
        const int nEdge = (int)this->_edgeList.size();
        std::vector<int> pointsLocation(nEdge + 1, 0);
        for (int edgeIdx = 0; edgeIdx < nEdge; ++edgeIdx) {
            const int nPoints = this->objectPointsMat(this->_edgeList[edgeIdx].cameraVertex, this->_edgeList[edgeIdx].photoIndex).rows;
            pointsLocation[edgeIdx + 1] = pointsLocation[edgeIdx] + nPoints * 2;
        }
        JTJ_inv = Mat();
        Mat J = Mat::zeros(pointsLocation[nEdge], nParam, CV_64F);
        Mat E = Mat::zeros(pointsLocation[nEdge], 1, CV_64F);
        Mat RvecDoubleSide, TvecDoubleSide;
        if constexpr (kDoubleSide) {   // the global block is the first six parameters (doubleSide.cpp:450-451)
            RvecDoubleSide = extrinsicParams.colRange(0, 3);
            TvecDoubleSide = extrinsicParams.colRange(3, 6);
        } else {
            RvecDoubleSide = this->doubleSideTransform_rvec();
            TvecDoubleSide = this->doubleSideTransform_tvec();
        }
        for (int edgeIdx = 0; edgeIdx < nEdge; ++edgeIdx) {
            const auto& eg = this->_edgeList[edgeIdx];
            const int photoVertex = eg.photoVertex, photoIndex = eg.photoIndex, cameraVertex = eg.cameraVertex;
            const Mat objectPoints = this->objectPointsMat(cameraVertex, photoIndex);
            const Mat imagePoints = this->imagePointsMat(cameraVertex, photoIndex);
            const int paraRow = kDoubleSide ? photoVertex - this->_nCamera + 1 : photoVertex - 1;
            const Mat RvecPhoto = extrinsicParams.colRange(paraRow * 6, paraRow * 6 + 3);
            const Mat TvecPhoto = extrinsicParams.colRange(paraRow * 6 + 3, paraRow * 6 + 6);
            Mat RvecCamera, TvecCamera;
            if constexpr (kDoubleSide) {
                RvecCamera = this->camerasPose_rvec(cameraVertex);
                TvecCamera = this->camerasPose_tvec(cameraVertex);
            } else if (cameraVertex > 0) {
                RvecCamera = extrinsicParams.colRange((cameraVertex - 1) * 6, (cameraVertex - 1) * 6 + 3);
                TvecCamera = extrinsicParams.colRange((cameraVertex - 1) * 6 + 3, (cameraVertex - 1) * 6 + 6);
            } else {
                RvecCamera = Mat::zeros(3, 1, CV_32F);
                TvecCamera = Mat::zeros(3, 1, CV_32F);
            }
            Mat Rvectran, Tvectran, jacobianPhoto, jacobianGlobal, error;
            computePhotoCameraJacobian(eg.patternSide, RvecPhoto, TvecPhoto, RvecCamera, TvecCamera, RvecDoubleSide,
                                       TvecDoubleSide, Rvectran, Tvectran, objectPoints, imagePoints,
                                       this->cameraMatrixMat(cameraVertex), this->distortCoeffsMat(cameraVertex),
                                       this->xiMat(cameraVertex), jacobianPhoto, jacobianGlobal, error);
            const int rowBegin = pointsLocation[edgeIdx], rowEnd = pointsLocation[edgeIdx + 1];
            if constexpr (kDoubleSide) {
                jacobianGlobal.copyTo(J.rowRange(rowBegin, rowEnd).colRange(0, 6));
            } else if (cameraVertex > 0) {
                jacobianGlobal.copyTo(J.rowRange(rowBegin, rowEnd).colRange((cameraVertex - 1) * 6, cameraVertex * 6));
            }
            jacobianPhoto.copyTo(J.rowRange(rowBegin, rowEnd).colRange(paraRow * 6, (paraRow + 1) * 6));
            error.copyTo(E.rowRange(rowBegin, rowEnd));
        }
        const Mat Jt = J.t();
        const Mat JTJ = Jt * J;
        JTE = Jt * E;
        deltaX = this->conjungate(JTJ, JTE);
    }
};
using RefMyMulti = RefStyle<cv::multicalib::MyMultiCameraCalibration>;
using RefDoubleSide = RefStyle<cv::multicalib::DoubleSideCalibration>;

static Mat vec3m(double a, double b, double c) {
    Mat m(3, 1, CV_64F);
    m.at<double>(0) = a;
    m.at<double>(1) = b;
    m.at<double>(2) = c;
    return m;
}

static int selftest() {
    // ---- the cv::Mat shim
    {
        Mat a = Mat::zeros(3, 4, CV_32F);
        a.at<float>(1, 2) = 5.f;
        Mat v = a.rowRange(1, 3).colRange(2, 4);   // a view
        EXPECT(v.rows == 2 && v.cols == 2 && v.at<float>(0, 0) == 5.f);
        v.at<float>(1, 1) = 7.f;
        EXPECT(a.at<float>(2, 3) == 7.f);
        Mat c = a.clone();
        c.at<float>(0, 0) = 1.f;
        EXPECT(a.at<float>(0, 0) == 0.f);
        Mat d;
        a.convertTo(d, CV_64F);
        EXPECT(d.type() == CV_64F && d.at<double>(1, 2) == 5.0);
        const Mat r = d.reshape(1, 1);
        EXPECT(r.rows == 1 && r.cols == 12 && r.at<double>(0, 6) == 5.0);
        Mat p = d.t() * d;   // 4 x 4
        EXPECT(p.rows == 4 && p.cols == 4 && p.at<double>(2, 2) == 25.0 && p.at<double>(3, 3) == 49.0);
        EXPECT(std::fabs(cv::norm(d) - std::sqrt(74.0)) < 1e-12);
        bool threw = false;
        try {
            (void)a.at<float>(3, 0);
        } catch (const std::out_of_range&) {
            threw = true;
        }
        EXPECT(threw);
    }
    // ---- conjungate (multicalib.hpp:157): a^-1 b for SPD a
    {
        PublicConjungate mc(cv::multicalib::MultiCameraCalibration::PINHOLE, 2);
        const int n = 12;
        std::mt19937 rng(3);
        std::normal_distribution<double> nd;
        Mat B(n, n, CV_64F), b(n, 2, CV_64F);
        for (int i = 0; i < n; ++i)
            for (int j = 0; j < n; ++j) B.at<double>(i, j) = nd(rng);
        for (int i = 0; i < n; ++i)
            for (int j = 0; j < 2; ++j) b.at<double>(i, j) = nd(rng);
        const Mat A = B.t() * B + 0.5 * Mat::eye(n, CV_64F);
        const Mat x = mc.conjungate(A, b);
        const Mat res = A * x - b;
        EXPECT(x.rows == n && x.cols == 2 && cv::norm(res) < 1e-10 * cv::norm(b));
    }
    // ---- compose_motion's partials against central differences (src/multicalib.cpp:1008-1056)
    {
        CountingMyMulti mc(2);
        const double om1[3] = {0.4, -0.7, 1.1}, T1[3] = {120.0, -40.0, 900.0};
        const double om2[3] = {-0.3, 0.2, 0.5}, T2[3] = {-250.0, 30.0, 60.0};
        std::vector<Mat> o;
        mc.composeMotion(vec3m(om1[0], om1[1], om1[2]), vec3m(T1[0], T1[1], T1[2]), vec3m(om2[0], om2[1], om2[2]),
                         vec3m(T2[0], T2[1], T2[2]), o);
        const double h = 1e-6;
        double worst = 0.0;
        for (int which = 0; which < 4; ++which)   // om1, T1, om2, T2
            for (int k = 0; k < 3; ++k) {
                double a[4][3] = {{om1[0], om1[1], om1[2]}, {T1[0], T1[1], T1[2]}, {om2[0], om2[1], om2[2]}, {T2[0], T2[1], T2[2]}};
                double b2[4][3];
                std::memcpy(b2, a, sizeof a);
                const double s = which % 2 ? 1e-3 : h;   // translations in mm
                a[which][k] += s;
                b2[which][k] -= s;
                std::vector<Mat> p, m;
                mc.composeMotion(vec3m(a[0][0], a[0][1], a[0][2]), vec3m(a[1][0], a[1][1], a[1][2]), vec3m(a[2][0], a[2][1], a[2][2]),
                                 vec3m(a[3][0], a[3][1], a[3][2]), p);
                mc.composeMotion(vec3m(b2[0][0], b2[0][1], b2[0][2]), vec3m(b2[1][0], b2[1][1], b2[1][2]),
                                 vec3m(b2[2][0], b2[2][1], b2[2][2]), vec3m(b2[3][0], b2[3][1], b2[3][2]), m);
                // partial order of compose_motion: dom3dom1, dom3dT1, dom3dom2, dom3dT2, dT3dom1, dT3dT1, dT3dom2, dT3dT2
                const Mat& dom = o[2 + which];
                const Mat& dT = o[6 + which];
                for (int i = 0; i < 3; ++i) {
                    const double fom = (p[0].at<double>(i) - m[0].at<double>(i)) / (2 * s);
                    const double fT = (p[1].at<double>(i) - m[1].at<double>(i)) / (2 * s);
                    worst = std::max(worst, std::fabs(fom - dom.at<double>(i, k)));
                    worst = std::max(worst, std::fabs(fT - dT.at<double>(i, k)) / std::max(1.0, std::fabs(fT)));
                }
            }
        EXPECT(worst < 1e-6);
    }
    // ---- the per-edge Jacobian (computePhotoCameraJacobian): shapes, and the block structure of
    // MyMulti's FRONT / BACK chains and DoubleSide's zero ds block for FRONT views
    {
        CountingMyMulti mc(2);
        Mat obj(4, 3, CV_32F), img(4, 2, CV_32F), K = Mat::zeros(3, 3, CV_32F), D = Mat::zeros(1, 5, CV_32F), xi;
        for (int i = 0; i < 4; ++i) {
            obj.at<float>(i, 0) = 40.f * (i % 2);
            obj.at<float>(i, 1) = 40.f * (i / 2);
            obj.at<float>(i, 2) = 0.f;
            img.at<float>(i, 0) = 900.f + 10.f * i;
            img.at<float>(i, 1) = 500.f;
        }
        K.at<float>(0, 0) = K.at<float>(1, 1) = 1200.f;
        K.at<float>(0, 2) = 960.f;
        K.at<float>(1, 2) = 540.f;
        K.at<float>(2, 2) = 1.f;
        D.at<float>(0, 0) = -0.1f;
        const Mat rP = vec3m(0.3, -0.2, 0.1), tP = vec3m(-20, 10, 1200), rC = vec3m(0.05, 0.2, -0.1),
                  tC = vec3m(-300, 5, 40), rD = vec3m(0.0, 3.1, 0.0), tD = vec3m(10, 0, -25);
        Mat jpF, jcF, eF, jpB, jcB, eB, rt, tt;
        mc.edgeJacobian(0, rP, tP, rC, tC, rD, tD, rt, tt, obj, img, K, D, xi, jpF, jcF, eF);
        mc.edgeJacobian(1, rP, tP, rC, tC, rD, tD, rt, tt, obj, img, K, D, xi, jpB, jcB, eB);
        EXPECT(jpF.rows == 8 && jpF.cols == 6 && jcF.rows == 8 && eF.rows == 8 && eF.cols == 1 && eF.type() == CV_64F);
        EXPECT(rt.empty() && tt.empty());   // MyMulti leaves Rvectran / Tvectran alone
        bool finite = true;
        for (int r = 0; r < 8; ++r) {
            finite = finite && std::isfinite(eF.at<double>(r)) && std::isfinite(eB.at<double>(r));
            for (int c = 0; c < 6; ++c)
                finite = finite && std::isfinite(jpF.at<double>(r, c)) && std::isfinite(jcB.at<double>(r, c));
        }
        EXPECT(finite);
        EXPECT(cv::norm(eF - eB) > 1.0);   // the BACK pose differs by the double-side transform
        CountingDoubleSide ds(2);
        Mat jp2, jg2, e2;
        ds.edgeJacobian(0, rP, tP, rC, tC, rD, tD, rt, tt, obj, img, K, D, xi, jp2, jg2, e2);
        EXPECT(cv::norm(jg2) == 0.0 && cv::norm(jp2 - jpF) == 0.0 && cv::norm(e2 - eF) == 0.0);
        ds.edgeJacobian(1, rP, tP, rC, tC, rD, tD, rt, tt, obj, img, K, D, xi, jp2, jg2, e2);
        EXPECT(cv::norm(jg2) > 0.0 && cv::norm(jp2 - jpB) == 0.0 && cv::norm(e2 - eB) == 0.0);
        EXPECT(ds.calls.jac == 0);
    }
    std::printf("selftest %s (%d failures)\n", g_fail ? "FAILED" : "ok", g_fail);
    return g_fail ? 1 : 0;
}

// strict-reference mode: the reference asserts isValidPose on every edge's stored transform in every
// linearisation (src/mymulticalib.cpp:706); an identity transform (|t| = 0) aborts before any GPU work
static int strict() {
    cv::multicalib::MyMultiCameraCalibration mc(2);
    mc.strictReference = true;
    mc.addPhotoVertex(0, mcc::multicalib::eye4());
    mc._edgeList.emplace_back(0, 2, 0, mcc::multicalib::eye4());
    mc.optimizeExtrinsics();
    std::printf("strict mode did not abort\n");
    return 1;
}

template <class T>
static std::vector<T> rd(std::ifstream& f, size_t n) {
    std::vector<T> v(n);
    f.read(reinterpret_cast<char*>(v.data()), (std::streamsize)(n * sizeof(T)));
    if (!f) throw std::runtime_error("truncated input");
    return v;
}

// the fixture problem (tests/cpp blob) into a host-layer object's state, as test_multicalib.cpp does
struct Blob {
    int model, C, V, E, nd, corners, crit_type, crit_max;
    bool has_ds, has_cp;
    double eps;
    std::vector<int> ecam, ephoto, eside, eoff, en;
    std::vector<float> obj, img, K, D, xi, cp, x0;
    std::vector<double> dsp;
};
static Blob read_blob(const char* in) {
    std::ifstream f(in, std::ios::binary);
    if (!f) throw std::runtime_error("cannot open input");
    const auto h = rd<int>(f, 11);
    if (h[0] != 0x4d434331) throw std::runtime_error("bad magic");
    Blob b;
    b.model = h[1]; b.C = h[2]; b.V = h[3]; b.E = h[4]; b.nd = h[5]; b.corners = h[6];
    b.has_ds = h[7] != 0; b.has_cp = h[8] != 0; b.crit_type = h[9]; b.crit_max = h[10];
    b.eps = rd<double>(f, 1)[0];
    b.ecam = rd<int>(f, b.E); b.ephoto = rd<int>(f, b.E); b.eside = rd<int>(f, b.E);
    b.eoff = rd<int>(f, b.E); b.en = rd<int>(f, b.E);
    b.obj = rd<float>(f, 3 * (size_t)b.corners); b.img = rd<float>(f, 2 * (size_t)b.corners);
    b.K = rd<float>(f, 9 * (size_t)b.C); b.D = rd<float>(f, (size_t)b.nd * b.C); b.xi = rd<float>(f, b.C);
    if (b.has_ds) b.dsp = rd<double>(f, 16);
    if (b.has_cp) b.cp = rd<float>(f, 16 * (size_t)b.C);
    const int P = (b.model == MCC_MODEL_DOUBLESIDE ? 6 : 6 * (b.C - 1)) + 6 * b.V;
    b.x0 = rd<float>(f, P);
    return b;
}
template <class MC>
static void fill(MC& mc, const Blob& b) {
    for (int c = 0; c < b.C; ++c) {
        std::copy(b.K.begin() + 9 * c, b.K.begin() + 9 * (c + 1), mc._cameraMatrix[c].begin());
        mc._distortCoeffs[c].assign(b.D.begin() + b.nd * c, b.D.begin() + b.nd * (c + 1));
        mc._xi[c] = b.xi[c];
    }
    for (int v = 0; v < b.V; ++v) mc.addPhotoVertex(v, mcc::multicalib::eye4());
    for (int e = 0; e < b.E; ++e) {
        const int c = b.ecam[e];
        const int pi = (int)mc._objectPointsForEachCamera[c].size();
        mc._objectPointsForEachCamera[c].emplace_back(b.obj.begin() + 3 * (size_t)b.eoff[e], b.obj.begin() + 3 * (size_t)(b.eoff[e] + b.en[e]));
        mc._imagePointsForEachCamera[c].emplace_back(b.img.begin() + 2 * (size_t)b.eoff[e], b.img.begin() + 2 * (size_t)(b.eoff[e] + b.en[e]));
        mc._edgeList.emplace_back(c, b.C + b.ephoto[e], pi, mcc::multicalib::eye4());
        mc._edgeList.back().patternSide = b.eside[e];
    }
    // the host layer's paras2vertex(vector) by virtual dispatch: DoubleSide's layout is [ds | photos]
    // (a qualified call would run the base class's [cameras | photos] on every model)
    static_cast<mcc::multicalib::MultiCameraCalibration&>(mc).paras2vertex(b.x0);
}

static long long ulp_diff(float a, float b) {
    int ia, ib;
    std::memcpy(&ia, &a, 4);
    std::memcpy(&ib, &b, 4);
    const long long oa = ia < 0 ? -(long long)(ia & 0x7fffffff) : ia, ob = ib < 0 ? -(long long)(ib & 0x7fffffff) : ib;
    return oa > ob ? oa - ob : ob - oa;
}

template <class Lib, class Sub>
static int compare(const Blob& b, Lib& lib, Sub& sub) {
    fill(lib, b);
    fill(sub, b);
    double e_lib = 0.0, e_sub = 0.0;
    try {
        e_lib = lib.optimizeExtrinsics();   // the device loop (the library's own class)
    } catch (const std::exception& e) {
        std::fprintf(stderr, "library class: %s\n", e.what());
        throw;
    }
    try {
        e_sub = sub.optimizeExtrinsics();   // the reference's host loop through the overrides
    } catch (const std::exception& e) {
        std::fprintf(stderr, "subclass, after %d linearisations: %s\n", sub.calls.jac, e.what());
        throw;
    }
    const std::vector<float> x_lib = lib.buildParaVector(), x_sub = sub.buildParaVector();
    long long worst = 0;
    for (size_t i = 0; i < x_lib.size(); ++i) worst = std::max(worst, ulp_diff(x_lib[i], x_sub[i]));
    std::printf("library: %d iterations, error %.12g; subclass: %d iterations, error %.12g; max %lld ulp; "
                "calls jac %d err %d build %d p2v %d\n",
                lib.iterations(), e_lib, sub.iterations(), e_sub, worst, sub.calls.jac, sub.calls.err,
                sub.calls.build, sub.calls.p2v);
    EXPECT(lib.iterations() == sub.iterations());
    EXPECT(std::fabs(e_lib - e_sub) <= 1e-6);
    EXPECT(worst <= 1);
    EXPECT(sub.calls.jac == sub.iterations());   // once per step (src/multicalib.cpp:489)
    EXPECT(sub.calls.err == 1 && sub.calls.build == 1 && sub.calls.p2v == 1);   // :464, :509, :512
    return g_fail ? 1 : 0;
}

static int run(const char* in) {
    const Blob b = read_blob(in);
    const mcc::multicalib::TermCriteria crit(b.crit_type, b.crit_max, b.eps);
    int rc = 0;
    if (b.model == MCC_MODEL_PINHOLE) {
        cv::multicalib::MyMultiCameraCalibration lib(b.C, crit);
        CountingMyMulti sub(b.C, crit);
        if (b.has_ds) {
            std::copy(b.dsp.begin(), b.dsp.end(), lib.doubleSideTransform.begin());
            std::copy(b.dsp.begin(), b.dsp.end(), sub.doubleSideTransform.begin());
        }
        rc = compare(b, lib, sub);
    } else if (b.model == MCC_MODEL_DOUBLESIDE) {
        cv::multicalib::DoubleSideCalibration lib(b.C, crit);
        CountingDoubleSide sub(b.C, crit);
        for (int c = 0; c < b.C; ++c) {
            std::copy(b.cp.begin() + 16 * c, b.cp.begin() + 16 * (c + 1), lib.camerasPose[c].begin());
            std::copy(b.cp.begin() + 16 * c, b.cp.begin() + 16 * (c + 1), sub.camerasPose[c].begin());
        }
        rc = compare(b, lib, sub);
    } else {
        std::printf("seam: omnidirectional fixture skipped (the MyMulti / DoubleSide seam)\n");
    }
    std::printf("seam %s\n", rc ? "FAILED" : "ok");
    return rc;
}

// the reference-style subclass against the library: its host linearisation at x0 against the GPU's
// (deltaX within 1e-6, JTE within 1e-9 of the largest entry), then its host loop (one host
// linearisation per step) against the library class's device loop
template <class Ref, class Lib>
static int refstyle_compare(const Blob& b, Lib& lib, Ref& ref) {
    fill(lib, b);
    fill(ref, b);
    const Mat x0 = ref.params();
    Mat jte_h, dx_h, jte_g, dx_g;
    ref.jacobianAt(x0, jte_h, dx_h);
    const int nEdgeCalls = ref.edgeCalls;
    ref.libraryJacobianAt(x0, jte_g, dx_g);
    double jmax = 0, dmax = 0, jdiff = 0, ddiff = 0;
    for (int i = 0; i < dx_h.rows; ++i) {
        jmax = std::max(jmax, std::fabs(jte_g.at<double>(i)));
        dmax = std::max(dmax, std::fabs(dx_g.at<double>(i)));
        jdiff = std::max(jdiff, std::fabs(jte_h.at<double>(i) - jte_g.at<double>(i)));
        ddiff = std::max(ddiff, std::fabs(dx_h.at<double>(i) - dx_g.at<double>(i)));
    }
    std::printf("refstyle: %d edges, JTE diff %.3g of %.3g, deltaX diff %.3g of %.3g\n", nEdgeCalls, jdiff, jmax, ddiff, dmax);
    EXPECT(nEdgeCalls == (int)ref._edgeList.size());
    EXPECT(jdiff <= 1e-9 * jmax);
    EXPECT(ddiff <= 1e-6 * dmax);
    const double e_lib = lib.optimizeExtrinsics();
    const double e_ref = ref.optimizeExtrinsics();
    const std::vector<float> x_lib = lib.buildParaVector(), x_ref = ref.buildParaVector();
    long long worst = 0;
    for (size_t i = 0; i < x_lib.size(); ++i) worst = std::max(worst, ulp_diff(x_lib[i], x_ref[i]));
    std::printf("refstyle loop: library %d iterations, error %.12g; host %d iterations, error %.12g; max %lld ulp\n",
                lib.iterations(), e_lib, ref.iterations(), e_ref, worst);
    EXPECT(lib.iterations() == ref.iterations());
    EXPECT(std::fabs(e_lib - e_ref) <= 1e-6);
    EXPECT(worst <= 1);
    return g_fail ? 1 : 0;
}

static int refstyle(const char* in) {
    const Blob b = read_blob(in);
    const mcc::multicalib::TermCriteria crit(b.crit_type, b.crit_max, b.eps);
    int rc = 0;
    if (b.model == MCC_MODEL_PINHOLE) {
        cv::multicalib::MyMultiCameraCalibration lib(b.C, crit);
        RefMyMulti ref(b.C, crit);
        if (b.has_ds) {
            std::copy(b.dsp.begin(), b.dsp.end(), lib.doubleSideTransform.begin());
            std::copy(b.dsp.begin(), b.dsp.end(), ref.doubleSideTransform.begin());
        }
        rc = refstyle_compare(b, lib, ref);
    } else if (b.model == MCC_MODEL_DOUBLESIDE) {
        cv::multicalib::DoubleSideCalibration lib(b.C, crit);
        RefDoubleSide ref(b.C, crit);
        for (int c = 0; c < b.C; ++c) {
            std::copy(b.cp.begin() + 16 * c, b.cp.begin() + 16 * (c + 1), lib.camerasPose[c].begin());
            std::copy(b.cp.begin() + 16 * c, b.cp.begin() + 16 * (c + 1), ref.camerasPose[c].begin());
        }
        rc = refstyle_compare(b, lib, ref);
    } else {
        std::printf("refstyle: omnidirectional fixture skipped (the MyMulti / DoubleSide bodies)\n");
    }
    std::printf("refstyle %s\n", rc ? "FAILED" : "ok");
    return rc;
}

int main(int argc, char** argv) {
    try {
        if (argc >= 2 && !std::strcmp(argv[1], "selftest")) return selftest();
        if (argc >= 2 && !std::strcmp(argv[1], "strict")) return strict();
        if (argc >= 3 && !std::strcmp(argv[1], "run")) return run(argv[2]);
        if (argc >= 3 && !std::strcmp(argv[1], "refstyle")) return refstyle(argv[2]);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 2;
    }
    std::fprintf(stderr, "usage: test_seam selftest | strict | run <in.bin> | refstyle <in.bin>\n");
    return 2;
}
