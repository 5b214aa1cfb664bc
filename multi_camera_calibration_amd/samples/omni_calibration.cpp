// omni_calibration -- the reference's samples/omni_calibration.cpp flow on pre-detected corners:
// read per-view pattern / image points, cv::omnidir::calibrate with TermCriteria(3, 200, 1e-8)
// (samples/omni_calibration.cpp:216-217), and write the camera parameters in the sample's
// saveCameraParams layout (:75-146).  Chessboard detection in images is out of scope (the input
// is the tutorial data format, tutorials/data/omni_calib_data.xml: objectPoints, imagePoints,
// imageSize); the calibration loop runs on the GPU through mcc::omnidir::calibrate.
//
//   omni_calibration [-fs] [-fp] [-o out_camera_params.xml] input.xml
#include <cstdio>
#include <cstring>
#include <ctime>
#include <iostream>
#include <string>
#include <vector>

#include "mcc_omnidir.hpp"
#include "mcc_storage.hpp"

using mcc::storage::FileStorage;
using mcc::storage::Mat;
using mcc::storage::Node;

namespace {

std::vector<Mat> mats(const Node& n) {
    std::vector<Mat> out;
    if (n.type == Node::MAT) out.push_back(n.mat);
    for (const Node& k : n.seq)
        if (k.type == Node::MAT) out.push_back(k.mat);
    return out;
}

}  // namespace

int main(int argc, char** argv) {
    std::string input, output = "out_camera_params.xml";
    int flags = 0;
    for (int i = 1; i < argc; ++i) {
        if (!std::strcmp(argv[i], "-fs")) flags |= mcc::omnidir::CALIB_FIX_SKEW;
        else if (!std::strcmp(argv[i], "-fp")) flags |= mcc::omnidir::CALIB_FIX_CENTER;
        else if (!std::strcmp(argv[i], "-o") && i + 1 < argc) output = argv[++i];
        else input = argv[i];
    }
    if (input.empty()) {
        std::cout << "usage: omni_calibration [-fs] [-fp] [-o out_camera_params.xml] corners.xml\n";
        return 0;
    }
    FileStorage fs(input, FileStorage::READ);
    if (!fs.isOpened()) {
        std::cout << "Can not read " << input << std::endl;
        return -1;
    }
    const std::vector<Mat> obj = mats(fs["objectPoints"]), img = mats(fs["imagePoints"]);
    const Node& sz = fs["imageSize"];
    if (obj.empty() || obj.size() != img.size() || sz.seq.size() != 2) {
        std::cout << "input needs objectPoints, imagePoints (one matrix per view) and imageSize" << std::endl;
        return -1;
    }
    std::vector<std::vector<mcc::omnidir::Vec3d>> objectPoints(obj.size());
    std::vector<std::vector<mcc::omnidir::Vec2d>> imagePoints(img.size());
    for (size_t v = 0; v < obj.size(); ++v) {
        const size_t n = obj[v].total();
        for (size_t j = 0; j < n; ++j) {
            objectPoints[v].push_back({obj[v].data[3 * j], obj[v].data[3 * j + 1], obj[v].data[3 * j + 2]});
            imagePoints[v].push_back({img[v].data[2 * j], img[v].data[2 * j + 1]});
        }
    }
    const mcc::omnidir::Size imageSize(sz.seq[0].toInt(), sz.seq[1].toInt());
    std::array<double, 9> K{};
    std::array<double, 4> D{};
    double xi = 0;
    std::vector<mcc::omnidir::Vec3d> rvecs, tvecs;
    std::vector<int> idx;
    const mcc::omnidir::TermCriteria criteria(3, 200, 1e-8);
    double rms = 0;
    try {
        rms = mcc::omnidir::calibrate(objectPoints, imagePoints, imageSize, K, xi, D, rvecs, tvecs, flags, criteria,
                                      &idx);
    } catch (const std::exception& e) {
        std::cout << e.what() << std::endl;
        return -1;
    }
    std::cout << "Saving camera params to " << output << std::endl;
    FileStorage out(output, FileStorage::WRITE);
    char buf[256];
    std::time_t tt = std::time(nullptr);
    std::strftime(buf, sizeof(buf) - 1, "%c", std::localtime(&tt));
    out.write("calibration_time", std::string(buf));
    out.write("nFrames", (int)rvecs.size());
    out.write("flags", flags);
    Mat Km(3, 3, 'd'), Dm(1, 4, 'd'), ext((int)rvecs.size(), 6, 'd'), used(1, (int)idx.size(), 'i');
    for (int k = 0; k < 9; ++k) Km.data[k] = K[k];
    for (int k = 0; k < 4; ++k) Dm.data[k] = D[k];
    for (size_t i = 0; i < rvecs.size(); ++i)
        for (int k = 0; k < 3; ++k) {
            ext.at((int)i, k) = rvecs[i][k];
            ext.at((int)i, 3 + k) = tvecs[i][k];
        }
    for (size_t i = 0; i < idx.size(); ++i) used.data[i] = idx[i];
    out.write("camera_matrix", Km);
    out.write("distortion_coefficients", Dm);
    out.write("xi", xi);
    out.write("used_imgs", used);   // indices of the views kept (the sample writes their image names)
    out.write("extrinsic_parameters", ext);
    out.write("rms", rms);
    out.release();
    std::printf("rms %.9f  fx %.6f fy %.6f s %.6f cx %.6f cy %.6f xi %.9f  D %.9f %.9f %.9f %.9f  views %zu\n", rms,
                K[0], K[4], K[1], K[2], K[5], xi, D[0], D[1], D[2], D[3], rvecs.size());
    return 0;
}
