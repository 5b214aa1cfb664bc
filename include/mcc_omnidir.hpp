/*
 * mcc_omnidir.hpp -- C++ mirror of cv::omnidir::calibrate over the C ABI (mcc_omnidir.h):
 * the same name, argument order and meaning as include/opencv2/ccalib/omnidir.hpp's
 *
 *   double calibrate(InputArrayOfArrays objectPoints, InputArrayOfArrays imagePoints, Size size,
 *                    InputOutputArray K, InputOutputArray xi, InputOutputArray D,
 *                    OutputArrayOfArrays rvecs, OutputArrayOfArrays tvecs, int flags,
 *                    TermCriteria criteria, OutputArray idx = noArray());
 *
 * (src/omnidir.cpp:1067-1211) with std containers in place of cv::Mat: per-view point lists in,
 * K (3x3 row-major), xi, D (k1, k2, p1, p2), the kept views' rvecs / tvecs and their indices out,
 * the rms reprojection error returned.  The loop runs on the GPU (libmcc.so); the CV_Assert
 * checks of the reference (:1071-1079) throw std::invalid_argument, device / numerical failures
 * std::runtime_error with mcc_last_error().
 */
#ifndef MCC_OMNIDIR_HPP
#define MCC_OMNIDIR_HPP

#include <array>
#include <stdexcept>
#include <string>
#include <vector>

#include "mcc_multicalib.hpp"
#include "mcc_omnidir.h"

namespace mcc {
namespace omnidir {

enum {
    CALIB_USE_GUESS = MCC_OMNI_CALIB_USE_GUESS,
    CALIB_FIX_SKEW = MCC_OMNI_CALIB_FIX_SKEW,
    CALIB_FIX_K1 = MCC_OMNI_CALIB_FIX_K1,
    CALIB_FIX_K2 = MCC_OMNI_CALIB_FIX_K2,
    CALIB_FIX_P1 = MCC_OMNI_CALIB_FIX_P1,
    CALIB_FIX_P2 = MCC_OMNI_CALIB_FIX_P2,
    CALIB_FIX_XI = MCC_OMNI_CALIB_FIX_XI,
    CALIB_FIX_GAMMA = MCC_OMNI_CALIB_FIX_GAMMA,
    CALIB_FIX_CENTER = MCC_OMNI_CALIB_FIX_CENTER
};

using Vec3d = std::array<double, 3>;
using Vec2d = std::array<double, 2>;
using Size = multicalib::Size;
using TermCriteria = multicalib::TermCriteria;

inline double calibrate(const std::vector<std::vector<Vec3d>>& objectPoints,
                        const std::vector<std::vector<Vec2d>>& imagePoints, Size size, std::array<double, 9>& K,
                        double& xi, std::array<double, 4>& D, std::vector<Vec3d>& rvecs, std::vector<Vec3d>& tvecs,
                        int flags, TermCriteria criteria, std::vector<int>* idx = nullptr, int device = 0) {
    if (objectPoints.empty() || imagePoints.empty() || objectPoints.size() != imagePoints.size())
        throw std::invalid_argument("omnidir::calibrate: objectPoints and imagePoints must be non-empty and of equal count");
    const int n = (int)objectPoints.size();
    std::vector<int> off(n + 1, 0);
    for (int i = 0; i < n; ++i) {
        if (objectPoints[i].size() != imagePoints[i].size())
            throw std::invalid_argument("omnidir::calibrate: view " + std::to_string(i) + " has mismatched point counts");
        off[i + 1] = off[i] + (int)objectPoints[i].size();
    }
    std::vector<double> obj(3 * (size_t)off[n]), img(2 * (size_t)off[n]);
    for (int i = 0; i < n; ++i)
        for (size_t j = 0; j < objectPoints[i].size(); ++j) {
            for (int k = 0; k < 3; ++k) obj[3 * (off[i] + j) + k] = objectPoints[i][j][k];
            for (int k = 0; k < 2; ++k) img[2 * (off[i] + j) + k] = imagePoints[i][j][k];
        }
    std::vector<double> om(3 * (size_t)n), t(3 * (size_t)n);
    std::vector<int> kept(n);
    int nk = 0, iters = 0;
    double rms = 0;
    const int rc = mcc_omnidir_calibrate(n, off.data(), obj.data(), img.data(), size.width, size.height, flags,
                                         criteria.type, criteria.maxCount, criteria.epsilon, device, K.data(), &xi,
                                         D.data(), om.data(), t.data(), kept.data(), &nk, &rms, &iters);
    if (rc != MCC_OK) throw std::runtime_error(std::string("omnidir::calibrate: ") + mcc_last_error());
    rvecs.assign(nk, Vec3d{});
    tvecs.assign(nk, Vec3d{});
    for (int i = 0; i < nk; ++i)
        for (int k = 0; k < 3; ++k) {
            rvecs[i][k] = om[3 * i + k];
            tvecs[i][k] = t[3 * i + k];
        }
    if (idx) idx->assign(kept.begin(), kept.begin() + nk);
    return rms;
}

}  // namespace omnidir
}  // namespace mcc

#endif
