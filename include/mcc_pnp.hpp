/*
 * mcc_pnp.hpp -- host-side pose initialisation for the loaders (no OpenCV in this build).
 *
 * The reference initialises every corner view with cv::solvePnP (SOLVEPNP_ITERATIVE) in
 * MyMultiCameraCalibration::calcPatternPose (src/mymulticalib.cpp:203-211).  This restates that
 * method's published algorithm (OpenCV 4.x calib3d, cvFindExtrinsicCameraParams2): undistort the
 * corners, an initial pose from the plane homography (planar targets) or a DLT (non-planar),
 * then Levenberg-Marquardt on the reprojection error through the full distortion model.  The
 * pose only initialises the Gauss-Newton (which converges to the same least-squares minimum), so
 * parity with OpenCV's solvePnP is not required bit for bit.
 *
 * Pinhole model of cv::projectPoints: D = k1 k2 p1 p2 [k3 [k4 k5 k6 [s1 s2 s3 s4]]].
 */
#ifndef MCC_PNP_HPP
#define MCC_PNP_HPP

#include <vector>

namespace mcc {
namespace pnp {

// image[2n] of object[3n] (float64) for pose (rvec, tvec)
void projectPoints(const double* object, int n, const double rvec[3], const double tvec[3], const double K[9],
                   const std::vector<double>& D, double* image);

// normalized, undistorted coordinates (x, y) of pixel points (cv::undistortPoints, iterative)
void undistortPoints(const double* image, int n, const double K[9], const std::vector<double>& D, double* xy,
                     int iterations = 20);

// cv::solvePnP(..., SOLVEPNP_ITERATIVE); returns the final RMS reprojection error (px), or a
// negative value when fewer than 4 points (planar) / 6 points (non-planar) are given
double solvePnP(const double* object, const double* image, int n, const double K[9], const std::vector<double>& D,
                double rvec[3], double tvec[3]);

// cvRodrigues2 in double
void rodrigues(const double r[3], double R[9]);
void rodriguesInv(const double R[9], double r[3]);

}  // namespace pnp
}  // namespace mcc

#endif
