/*
 * opencv2/ccalib/mymulticalib.hpp -- source-compatible stand-in for the reference's
 * include/opencv2/ccalib/mymulticalib.hpp:72-176: cv::multicalib::MyMultiCameraCalibration
 * (pinhole cameras from per-serial configs, pre-detected corner files, solvePnP seeding, the
 * two-pass outlier flow), resolved to the host layer's class (mcc_multicalib.hpp) under the
 * reference's cv::Mat-typed seam (multicalib.hpp in this directory).
 *   MyMultiCameraCalibration(cameraSerials, cameraType, nCameras, dataFolder, cameraConfigFolder,
 *       doubleSideConfig, frontPatternSize, backPatternSize, patternWidth, patternHeight,
 *       verbose = 0, showExtration = 0, nMiniMatches = 20, flags = 0,
 *       TermCriteria(COUNT + EPS, 200, 1e-7))                        mymulticalib.hpp:91-96
 *   loadImages(const std::set<std::string>& outliers = {}) :100, initialize() :105,
 *   removeOutlier() :109, writeParameters(const std::string&) :110, plus the base class's
 *   optimizeExtrinsics(), conjungate(), reset(), run();
 *   protected, virtual: computeJacobianExtrinsic(const Mat&, Mat&, Mat&, Mat&) :164,
 *   computePhotoCameraJacobian(int patternSide, ...) :166-170, computeProjectError(Mat&) :172.
 * Like the reference header (mymulticalib.hpp:50) it brings namespace cv into scope.
 */
#ifndef MCC_CV_MYMULTICALIB_HPP
#define MCC_CV_MYMULTICALIB_HPP

#include "multicalib.hpp"
#include "../../mcc_pnp.hpp"

using namespace cv;

namespace cv {
namespace multicalib {

class MyMultiCameraCalibration
    : public detail::Seam<mcc::multicalib::MyMultiCameraCalibration, MyMultiCameraCalibration> {
public:
    using detail::Seam<mcc::multicalib::MyMultiCameraCalibration, MyMultiCameraCalibration>::Seam;

protected:
    // computePhotoCameraJacobian (mymulticalib.hpp:166-170, src/mymulticalib.cpp:468-614): one edge's
    // Jacobians w.r.t. the photo and the camera (BACK views through compose(ds, photofront), chained
    // as :509-517 chain them), the residual; Rvectran / Tvectran are left as they are (the reference
    // projects local copies)
    virtual void computePhotoCameraJacobian(int patternSide, const Mat& RvecPhoto, const Mat& TvecPhoto,
                                            const Mat& RvecCamera, const Mat& TvecCamera,
                                            const Mat& RvecDoubleside, const Mat& TvecDoubleside, Mat& Rvectran,
                                            Mat& Tvectran, const Mat& objectPoints, const Mat& imagePoints,
                                            const Mat& K, const Mat& distort, const Mat& xi, Mat& jacobianPhoto,
                                            Mat& jacobianDoubleside, Mat& E) {
        (void)Rvectran; (void)Tvectran;
        detail::edge_jacobian_mats(mcc::multicalib::EDGE_MYMULTI, false, patternSide, RvecPhoto, TvecPhoto, RvecCamera,
                                   TvecCamera, &RvecDoubleside, &TvecDoubleside, objectPoints, imagePoints, K, distort,
                                   xi, jacobianPhoto, jacobianDoubleside, E, nullptr, nullptr);
    }
    // doubleSideTransform_rvec / _tvec (mymulticalib.hpp:123; doublesideTransform2vec,
    // src/mymulticalib.cpp:105-117): the CV_64F transform as rvec, tvec (3 x 1 CV_64F)
    Mat doubleSideTransform_rvec() const {
        double R[9], r[3];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) R[3 * i + j] = this->doubleSideTransform[4 * i + j];
        mcc::multicalib::polar_orthonormalise(R);   // cv::Rodrigues' SVD step
        mcc::pnp::rodriguesInv(R, r);
        Mat m(3, 1, CV_64F);
        for (int k = 0; k < 3; ++k) m.at<double>(k, 0) = r[k];
        return m;
    }
    Mat doubleSideTransform_tvec() const {
        Mat m(3, 1, CV_64F);
        for (int k = 0; k < 3; ++k) m.at<double>(k, 0) = this->doubleSideTransform[4 * k + 3];
        return m;
    }
};

}  // namespace multicalib
}  // namespace cv

#endif
