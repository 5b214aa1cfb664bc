/*
 * opencv2/ccalib/doubleSide.hpp -- source-compatible stand-in for the reference's
 * include/opencv2/ccalib/doubleSide.hpp:80-170: cv::multicalib::DoubleSideCalibration (fixed
 * camera poses from each config's CameraMatrix, the front->back board transform as the only
 * global block), resolved to the host layer's class (mcc_multicalib.hpp) under the reference's
 * cv::Mat-typed seam (multicalib.hpp in this directory).
 *   DoubleSideCalibration(cameraSerials, cameraType, nCameras, dataFolder, cameraConfigFolder,
 *       frontPatternSize, backPatternSize, patternWidth, patternHeight, verbose = 0,
 *       showExtration = 0, nMiniMatches = 20, flags = 0,
 *       TermCriteria(COUNT + EPS, 200, 1e-8))                        doubleSide.hpp:99-105
 *   initialize() :119, writeParameters(const std::string&) :120;
 *   protected, virtual: computeJacobianExtrinsic(const Mat&, Mat&, Mat&, Mat&) :133, buildParas()
 *   :135, computePhotoCameraJacobian(int patternSide, ...) :153-157, paras2vertex(const Mat&) :161,
 *   computeProjectError(Mat&) :163, vector2parameters(...) :165.
 * The reference's class runs only with two cameras (src/doubleSide.cpp:44-50, 643); this one
 * generalises its initialisation past that.
 */
#ifndef MCC_CV_DOUBLESIDE_HPP
#define MCC_CV_DOUBLESIDE_HPP

#include "mymulticalib.hpp"

namespace cv {
namespace multicalib {

class DoubleSideCalibration
    : public detail::Seam<mcc::multicalib::DoubleSideCalibration, DoubleSideCalibration> {
public:
    using detail::Seam<mcc::multicalib::DoubleSideCalibration, DoubleSideCalibration>::Seam;

protected:
    // computePhotoCameraJacobian (doubleSide.hpp:153-157, src/doubleSide.cpp:288-430): one edge's
    // Jacobians w.r.t. the photo and the double-side transform (zero for FRONT views, :335-336),
    // the residual; rvecTran / tvecTran are left as they are
    virtual void computePhotoCameraJacobian(int patternSide, const Mat& rvecPhoto, const Mat& tvecPhoto,
                                            const Mat& rvecCamera, const Mat& tvecCamera,
                                            const Mat& rvecDoubleside, const Mat& tvecDoubleside, Mat& rvecTran,
                                            Mat& tvecTran, const Mat& objectPoints, const Mat& imagePoints,
                                            const Mat& K, const Mat& distort, const Mat& xi, Mat& jacobianPhoto,
                                            Mat& jacobianDoubleside, Mat& E) {
        (void)rvecTran; (void)tvecTran;
        detail::edge_jacobian_mats(mcc::multicalib::EDGE_DOUBLESIDE, false, patternSide, rvecPhoto, tvecPhoto,
                                   rvecCamera, tvecCamera, &rvecDoubleside, &tvecDoubleside, objectPoints, imagePoints,
                                   K, distort, xi, jacobianPhoto, jacobianDoubleside, E, nullptr, nullptr);
    }
    // camerasPose_rvec[c] / camerasPose_tvec[c] (doubleSide.hpp:124-125; cameraPose2vec,
    // src/doubleSide.cpp:262-275): the fixed CV_32F camera pose as rvec, tvec (3 x 1 CV_32F)
    Mat camerasPose_rvec(int camera) const {
        float r[3];
        mcc::multicalib::rodrigues_m2v(rotation_of(this->camerasPose.at(camera)).data(), r);
        Mat m(3, 1, CV_32F);
        for (int k = 0; k < 3; ++k) m.at<float>(k, 0) = r[k];
        return m;
    }
    Mat camerasPose_tvec(int camera) const {
        Mat m(3, 1, CV_32F);
        for (int k = 0; k < 3; ++k) m.at<float>(k, 0) = this->camerasPose.at(camera)[4 * k + 3];
        return m;
    }

private:
    static std::array<float, 9> rotation_of(const mcc::multicalib::Pose& P) {
        std::array<float, 9> R;
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) R[3 * i + j] = P[4 * i + j];
        return R;
    }
};

}  // namespace multicalib
}  // namespace cv

#endif
