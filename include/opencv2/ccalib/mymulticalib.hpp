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

using namespace cv;

namespace cv {
namespace multicalib {

class MyMultiCameraCalibration
    : public detail::Seam<mcc::multicalib::MyMultiCameraCalibration, MyMultiCameraCalibration> {
public:
    using detail::Seam<mcc::multicalib::MyMultiCameraCalibration, MyMultiCameraCalibration>::Seam;

protected:
    // computePhotoCameraJacobian (mymulticalib.hpp:166-170): one edge's Jacobians with the
    // double-side transform of BACK views (src/mymulticalib.cpp:468-614); see multicalib.hpp
    virtual void computePhotoCameraJacobian(int patternSide, const Mat& RvecPhoto, const Mat& TvecPhoto,
                                            const Mat& RvecCamera, const Mat& TvecCamera,
                                            const Mat& RvecDoubleside, const Mat& TvecDoubleside, Mat& Rvectran,
                                            Mat& Tvectran, const Mat& objectPoints, const Mat& imagePoints,
                                            const Mat& K, const Mat& distort, const Mat& xi, Mat& jacobianPhoto,
                                            Mat& jacobianDoubleside, Mat& E) {
        (void)patternSide; (void)RvecPhoto; (void)TvecPhoto; (void)RvecCamera; (void)TvecCamera;
        (void)RvecDoubleside; (void)TvecDoubleside; (void)Rvectran; (void)Tvectran; (void)objectPoints;
        (void)imagePoints; (void)K; (void)distort; (void)xi; (void)jacobianPhoto; (void)jacobianDoubleside; (void)E;
        no_per_edge_jacobian();
    }
};

}  // namespace multicalib
}  // namespace cv

#endif
