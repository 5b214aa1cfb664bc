/*
 * opencv2/ccalib/doubleSide.hpp -- source-compatible stand-in for the reference's
 * include/opencv2/ccalib/doubleSide.hpp:80-170: cv::multicalib::DoubleSideCalibration (fixed
 * camera poses from each config's CameraMatrix, the front->back board transform as the only
 * global block), resolved to the host layer's class (mcc_multicalib.hpp).
 *   DoubleSideCalibration(cameraSerials, cameraType, nCameras, dataFolder, cameraConfigFolder,
 *       frontPatternSize, backPatternSize, patternWidth, patternHeight, verbose = 0,
 *       showExtration = 0, nMiniMatches = 20, flags = 0,
 *       TermCriteria(COUNT + EPS, 200, 1e-8))                        doubleSide.hpp:99-105
 * The reference's class runs only with two cameras (src/doubleSide.cpp:44-50, 643); this one
 * generalises its initialisation past that.
 */
#ifndef MCC_CV_DOUBLESIDE_HPP
#define MCC_CV_DOUBLESIDE_HPP

#include "mymulticalib.hpp"

namespace cv {
namespace multicalib {

using mcc::multicalib::DoubleSideCalibration;

}  // namespace multicalib
}  // namespace cv

#endif
