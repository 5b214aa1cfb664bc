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
    // computePhotoCameraJacobian (doubleSide.hpp:153-157, src/doubleSide.cpp:288-430); see multicalib.hpp
    virtual void computePhotoCameraJacobian(int patternSide, const Mat& rvecPhoto, const Mat& tvecPhoto,
                                            const Mat& rvecCamera, const Mat& tvecCamera,
                                            const Mat& rvecDoubleside, const Mat& tvecDoubleside, Mat& rvecTran,
                                            Mat& tvecTran, const Mat& objectPoints, const Mat& imagePoints,
                                            const Mat& K, const Mat& distort, const Mat& xi, Mat& jacobianPhoto,
                                            Mat& jacobianDoubleside, Mat& E) {
        (void)patternSide; (void)rvecPhoto; (void)tvecPhoto; (void)rvecCamera; (void)tvecCamera;
        (void)rvecDoubleside; (void)tvecDoubleside; (void)rvecTran; (void)tvecTran; (void)objectPoints;
        (void)imagePoints; (void)K; (void)distort; (void)xi; (void)jacobianPhoto; (void)jacobianDoubleside; (void)E;
        no_per_edge_jacobian();
    }
};

}  // namespace multicalib
}  // namespace cv

#endif
