// multi_cameras_calibration -- the reference sample's flow (samples/multi_cameras_calibration.cpp:
// 46-83) on the MI355X optimiser: MyMultiCameraCalibration over pre-detected corner files, two
// passes with outlier removal, results written as the reference does.  The reference hard-codes
// its folders; here they are arguments.
//
//   multi_cameras_calibration --serials S0,S1,... --data DIR --config DIR [--doubleside FILE]
//       [--front 8x11] [--back 7x10] [--out multi-camera-results.xml] [--single-pass]
//       [--double-side] [--init-only] [--dump-problem FILE] [--dump-result FILE] [--device N]
//       [--verbose]
//
// --double-side runs DoubleSideCalibration instead (the reference sample's #else branch: fixed
// camera poses from the configs' CameraMatrix, the double-side transform optimised; its
// writeParameters writes doublesideTransform.yaml in the working directory).
//
// --list FILE runs the base MultiCameraCalibration instead, as the reference's multi-camera
// tutorial does (tutorials/multi_camera_tutorial.markdown: construct, run(), writeParameters):
// FILE is an imagelist_creator list whose entries after the first are per-view corner files
// "cameraIdx-timestamp.yaml" (imagePoints, objectPoints, imageSize); with --omni (the only camera
// type whose intrinsics are restated) every camera is first calibrated by cv::omnidir::calibrate
// on the GPU.  --cameras N (required), --min-matches K (nMiniMatches, default 20).
//
// --init-only stops after loadImages + initialize (no GPU needed).  --dump-problem writes the
// problem of the last pass (tests/cpp blob format + photo timestamps) with x0 = buildParaVector(),
// --dump-result the optimised parameters, error, iterations and the outlier files.
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <memory>
#include <sstream>

#include "mcc_multicalib.hpp"

using namespace mcc::multicalib;

namespace {

std::vector<std::string> split(const std::string& s, char sep) {
    std::vector<std::string> out;
    std::stringstream ss(s);
    std::string tok;
    while (std::getline(ss, tok, sep))
        if (!tok.empty()) out.push_back(tok);
    return out;
}

Size parse_size(const std::string& s) {
    const auto p = split(s, 'x');
    if (p.size() != 2) throw std::runtime_error("size must be WxH: " + s);
    return Size(std::stoi(p[0]), std::stoi(p[1]));
}

template <class T>
void wr(std::ofstream& f, const T* p, size_t n) {
    f.write(reinterpret_cast<const char*>(p), (std::streamsize)(n * sizeof(T)));
}

// the problem as the C ABI sees it (edge order, photo index = vertex - C), x0 = buildParaVector()
void dump_problem(MultiCameraCalibration& mc, const std::string& path) {
    const int C = mc._nCamera, V = (int)mc._vertexList.size() - C, E = (int)mc._edgeList.size();
    const int nd = (int)mc._distortCoeffs[0].size();
    std::vector<int> ecam, ephoto, eside, eoff, en;
    std::vector<float> obj, img;
    int corners = 0;
    for (const auto& e : mc._edgeList) {
        const auto& o = mc._objectPointsForEachCamera[e.cameraVertex][e.photoIndex];
        const auto& im = mc._imagePointsForEachCamera[e.cameraVertex][e.photoIndex];
        ecam.push_back(e.cameraVertex);
        ephoto.push_back(e.photoVertex - C);
        eside.push_back(e.patternSide);
        eoff.push_back(corners);
        en.push_back((int)o.size() / 3);
        obj.insert(obj.end(), o.begin(), o.end());
        img.insert(img.end(), im.begin(), im.end());
        corners += (int)o.size() / 3;
    }
    auto* dsc = dynamic_cast<DoubleSideCalibration*>(&mc);
    auto* my = dynamic_cast<MyMultiCameraCalibration*>(&mc);
    bool has_ds = false;
    if (!dsc && my)
        for (double v : my->doubleSideTransform) has_ds = has_ds || v != 0.0;
    const int model = dsc ? MCC_MODEL_DOUBLESIDE
                          : (mc._camType == MultiCameraCalibration::OMNIDIRECTIONAL ? MCC_MODEL_OMNI : MCC_MODEL_PINHOLE);
    const int hdr[11] = {0x4d434331, model, C, V, E, nd, corners,
                         has_ds ? 1 : 0, dsc ? 1 : 0, mc._criteria.type, mc._criteria.maxCount};
    std::ofstream f(path, std::ios::binary);
    wr(f, hdr, 11);
    wr(f, &mc._criteria.epsilon, 1);
    wr(f, ecam.data(), E); wr(f, ephoto.data(), E); wr(f, eside.data(), E); wr(f, eoff.data(), E); wr(f, en.data(), E);
    wr(f, obj.data(), obj.size());
    wr(f, img.data(), img.size());
    for (int c = 0; c < C; ++c) wr(f, mc._cameraMatrix[c].data(), 9);
    for (int c = 0; c < C; ++c) wr(f, mc._distortCoeffs[c].data(), nd);
    wr(f, mc._xi.data(), C);
    if (has_ds) wr(f, my->doubleSideTransform.data(), 16);
    if (dsc)
        for (int c = 0; c < C; ++c) wr(f, dsc->camerasPose[c].data(), 16);
    const std::vector<float> x0 = mc.buildParaVector();
    wr(f, x0.data(), x0.size());
    std::vector<int> ts;
    for (int v = C; v < C + V; ++v) ts.push_back(mc._vertexList[v].timestamp);
    wr(f, ts.data(), ts.size());
    if (!f) throw std::runtime_error("cannot write " + path);
}

}  // namespace

int main(int argc, char** argv) {
    std::string serials, data, config, ds, out = "multi-camera-results.xml", dump_p, dump_r, list;
    Size front(8, 11), back(7, 10);
    bool single = false, init_only = false, double_side = false, omni = false;
    int device = 0, verbose = 0, ncams = 0, min_matches = 20;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        auto next = [&]() -> std::string {
            if (i + 1 >= argc) throw std::runtime_error("missing value for " + a);
            return argv[++i];
        };
        if (a == "--serials") serials = next();
        else if (a == "--data") data = next();
        else if (a == "--config") config = next();
        else if (a == "--doubleside") ds = next();
        else if (a == "--front") front = parse_size(next());
        else if (a == "--back") back = parse_size(next());
        else if (a == "--out") out = next();
        else if (a == "--single-pass") single = true;
        else if (a == "--init-only") init_only = true;
        else if (a == "--double-side") double_side = true;
        else if (a == "--dump-problem") dump_p = next();
        else if (a == "--dump-result") dump_r = next();
        else if (a == "--device") device = std::stoi(next());
        else if (a == "--verbose") verbose = 1;
        else if (a == "--list") list = next();
        else if (a == "--omni") omni = true;
        else if (a == "--cameras") ncams = std::stoi(next());
        else if (a == "--min-matches") min_matches = std::stoi(next());
        else {
            std::fprintf(stderr, "unknown argument %s\n", a.c_str());
            return 2;
        }
    }
    try {
        if (!list.empty()) {   // the multi-camera tutorial's flow on the base class
            if (ncams < 1) throw std::runtime_error("--list needs --cameras N");
            MultiCameraCalibration multiCalib(omni ? MultiCameraCalibration::OMNIDIRECTIONAL
                                                   : MultiCameraCalibration::PINHOLE,
                                              ncams, list, 0.f, 0.f, verbose, 0, min_matches, 0,
                                              TermCriteria(TermCriteria::COUNT, 20, 1e-7), device);
            multiCalib.loadImages();
            multiCalib.initialize();
            if (!dump_p.empty()) dump_problem(multiCalib, dump_p);
            if (init_only) {
                std::printf("loaded: %zu edges, %zu vertices\n", multiCalib._edgeList.size(),
                            multiCalib._vertexList.size());
                return 0;
            }
            const double err = multiCalib.optimizeExtrinsics();
            multiCalib.writeParameters(out);
            if (!dump_r.empty()) {
                std::ofstream r(dump_r);
                char b[40];
                std::snprintf(b, sizeof b, "%.17g", err);
                r << "error_exact " << b << "\niterations " << multiCalib.iterations() << "\nx";
                for (float v : multiCalib.buildParaVector()) {
                    std::snprintf(b, sizeof b, " %.9g", v);
                    r << b;
                }
                r << "\n";
            }
            std::printf("meanReprojectError %.9g after %d iterations\n", err, multiCalib.iterations());
            return 0;
        }
        const std::vector<std::string> cams = split(serials, ',');
        if (cams.empty() || data.empty() || config.empty()) {
            std::fprintf(stderr, "usage: %s --serials S0,S1,... --data DIR --config DIR [options]\n", argv[0]);
            return 2;
        }
        std::unique_ptr<MyMultiCameraCalibration> mc;
        if (double_side)
            mc.reset(new DoubleSideCalibration(cams, MultiCameraCalibration::PINHOLE, (int)cams.size(), data, config,
                                               front, back, 0.f, 0.f, verbose, 0, 0, 0,
                                               TermCriteria(TermCriteria::COUNT + TermCriteria::EPS, 200, 1e-8),
                                               device));
        else
            mc.reset(new MyMultiCameraCalibration(cams, MultiCameraCalibration::PINHOLE, (int)cams.size(), data,
                                                  config, ds, front, back, 0.f, 0.f, verbose, 0, 0, 0,
                                                  TermCriteria(TermCriteria::COUNT + TermCriteria::EPS, 200, 1e-7),
                                                  device));
        MyMultiCameraCalibration& multiCalib = *mc;
        multiCalib.loadImages();
        multiCalib.initialize();
        if (init_only) {
            if (!dump_p.empty()) dump_problem(multiCalib, dump_p);
            std::printf("loaded: %zu edges, %zu vertices\n", multiCalib._edgeList.size(), multiCalib._vertexList.size());
            return 0;
        }
        double err = multiCalib.optimizeExtrinsics();
        std::set<std::string> outliers;
        if (!single) {
            outliers = multiCalib.removeOutlier();
            std::cout << "number of outliers: " << outliers.size() << std::endl;
            multiCalib.reset();
            multiCalib.loadImages(outliers);
            multiCalib.initialize();
            if (!dump_p.empty()) dump_problem(multiCalib, dump_p);
            err = multiCalib.optimizeExtrinsics();
        } else if (!dump_p.empty()) {
            throw std::runtime_error("--dump-problem with --single-pass: dump before optimising with --init-only");
        }
        multiCalib.writeParameters(out);
        if (!dump_r.empty()) {
            std::ofstream r(dump_r);
            char b[40];
            r << "error " << std::to_string(err) << "\n";
            std::snprintf(b, sizeof b, "%.17g", err);
            r << "error_exact " << b << "\niterations " << multiCalib.iterations() << "\nx";
            for (float v : multiCalib.buildParaVector()) {
                std::snprintf(b, sizeof b, " %.9g", v);
                r << b;
            }
            r << "\n";
            for (const auto& o : outliers) r << "outlier " << o << "\n";
        }
        std::printf("meanReprojectError %.9g after %d iterations, %zu outliers\n", err, multiCalib.iterations(),
                    outliers.size());
    } catch (const std::exception& e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 1;
    }
    return 0;
}
