/*
 * opencv2/ccalib/mymulticalib.hpp -- source-compatible stand-in for the reference's
 * include/opencv2/ccalib/mymulticalib.hpp:72-176: cv::multicalib::MyMultiCameraCalibration
 * (pinhole cameras from per-serial configs, pre-detected corner files, solvePnP seeding, the
 * two-pass outlier flow), resolved to the host layer's class (mcc_multicalib.hpp).
 *   MyMultiCameraCalibration(cameraSerials, cameraType, nCameras, dataFolder, cameraConfigFolder,
 *       doubleSideConfig, frontPatternSize, backPatternSize, patternWidth, patternHeight,
 *       verbose = 0, showExtration = 0, nMiniMatches = 20, flags = 0,
 *       TermCriteria(COUNT + EPS, 200, 1e-7))                        mymulticalib.hpp:91-96
 *   loadImages(const std::set<std::string>& outliers = {}) :100, initialize() :105,
 *   removeOutlier() :109, writeParameters(const std::string&) :110, plus the base class's
 *   optimizeExtrinsics(), reset(), run().
 * Like the reference header (mymulticalib.hpp:50) it brings namespace cv into scope.
 */
#ifndef MCC_CV_MYMULTICALIB_HPP
#define MCC_CV_MYMULTICALIB_HPP

#include "multicalib.hpp"

using namespace cv;

namespace cv {
namespace multicalib {

using mcc::multicalib::MyMultiCameraCalibration;

}  // namespace multicalib
}  // namespace cv

#endif
