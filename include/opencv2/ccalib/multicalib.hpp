/*
 * opencv2/ccalib/multicalib.hpp -- source-compatible stand-in for the reference's header of the
 * same path (include/opencv2/ccalib/multicalib.hpp:73-252): cv::multicalib::MultiCameraCalibration
 * and the OpenCV value types its callers name (cv::Size, cv::TermCriteria), so code written
 * against the reference -- its sample samples/multi_cameras_calibration.cpp included, byte for
 * byte -- compiles against this build and runs the bundle adjustment on the MI355X.
 *
 * The names resolve to the C++ host layer over the C ABI (mcc_multicalib.hpp -> libmcc_host.so,
 * libmcc.so).  Constructors, methods and defaults follow the reference:
 *   MultiCameraCalibration(cameraType, nCameras, fileName, patternWidth, patternHeight, verbose,
 *       showExtration, nMiniMatches, flags, TermCriteria(COUNT, 20, 1e-7))  multicalib.hpp:138-143
 *   loadImages() :147, initialize() :151, optimizeExtrinsics() :155, run() :161, reset() :162,
 *   writeParameters(const std::string&) :165
 * (the feature detector / descriptor / matcher arguments are dropped: image feature matching is
 * outside this build, which reads pre-detected corners).  Errors throw std::runtime_error where
 * the reference's CV_Assert / CV_Error throw cv::Exception.  Build: -I<repo>/include/opencv2/ccalib
 * -I<repo>/include, link -lmcc_host -lmcc.
 */
#ifndef MCC_CV_MULTICALIB_HPP
#define MCC_CV_MULTICALIB_HPP

#include <cstdio>
#include <iostream>
#include <set>
#include <string>
#include <vector>

#include "../../mcc_multicalib.hpp"

namespace cv {

using Size = mcc::multicalib::Size;                 // cv::Size(width, height)
using TermCriteria = mcc::multicalib::TermCriteria;   // COUNT = MAX_ITER = 1, EPS = 2

namespace multicalib {

using mcc::multicalib::MultiCameraCalibration;

}  // namespace multicalib
}  // namespace cv

#endif
