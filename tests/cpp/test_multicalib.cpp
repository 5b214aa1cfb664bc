// Drives the C++ host layer (include/mcc_multicalib.hpp) the way the reference's sample drives
// cv::multicalib (samples/multi_cameras_calibration.cpp: construct, loadImages + initialize,
// optimizeExtrinsics).  Built and run by tests/test_cpp_host.py:
//
//   test_multicalib selftest              host-only checks (no GPU): Rodrigues round trips,
//                                         buildParas / paras2vertex layouts, error behaviour
//   test_multicalib run <in.bin> <out.txt>  fixture problem (written by the test from a golden
//                                         npz): seam at x0, computeProjectError, optimizeExtrinsics
//   test_multicalib storage <file>        FileStorage read: one line per top-level key
//                                         (kind, rows x cols x channels / sequence length)
//
// The input blob: int32 header [magic, model, C, V, E, nd, corners, has_ds, has_campose,
// crit_type, crit_max], float64 eps, then edge_cam, edge_photo, edge_side, edge_off, edge_n
// (int32 [E]), obj [3 corners], img [2 corners], K [9C], D [nd C], xi [C] (float32),
// ds_pose [16] float64 (if has_ds), cam_pose [16 C] float32 (if has_campose), x0 [P] float32.
#include "mcc_multicalib.hpp"
#include "mcc_pnp.hpp"
#include "mcc_storage.hpp"

#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <memory>

using namespace mcc::multicalib;

static int g_fail = 0;
#define EXPECT(c)                                                              \
    do {                                                                       \
        if (!(c)) {                                                            \
            std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
            ++g_fail;                                                          \
        }                                                                      \
    } while (0)

template <class F>
static bool throws(F f) {
    try {
        f();
    } catch (const std::runtime_error&) {
        return true;
    }
    return false;
}

static double maxdiff(const std::vector<float>& a, const std::vector<float>& b) {
    double m = a.size() == b.size() ? 0.0 : 1e30;
    for (size_t i = 0; i < a.size() && i < b.size(); ++i) m = std::max(m, (double)std::fabs(a[i] - b[i]));
    return m;
}

static int selftest() {
    // Rodrigues: vector -> matrix -> vector, including the small-angle and ~pi branches
    const float cases[][3] = {{0.1f, -0.2f, 0.3f}, {1e-9f, 0.f, 0.f}, {0.f, 0.f, 0.f}, {3.1f, 0.05f, -0.02f},
                              {-0.7f, 1.2f, 0.4f}};
    for (const auto& r : cases) {
        float R[9], back[3];
        rodrigues_v2m(r, R);
        double orth = 0;   // R R^T = I
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) {
                double s = 0;
                for (int k = 0; k < 3; ++k) s += (double)R[3 * i + k] * R[3 * j + k];
                orth = std::max(orth, std::fabs(s - (i == j)));
            }
        EXPECT(orth < 1e-6);
        rodrigues_m2v(R, back);
        for (int k = 0; k < 3; ++k) EXPECT(std::fabs(back[k] - r[k]) < 2e-5);
    }
    {   // a rotation by pi about x: the ~pi branch must return (+-pi, 0, 0)
        const float R[9] = {1, 0, 0, 0, -1, 0, 0, 0, -1};
        float r[3];
        rodrigues_m2v(R, r);
        EXPECT(std::fabs(std::fabs(r[0]) - 3.14159265f) < 1e-5 && std::fabs(r[1]) < 1e-6 && std::fabs(r[2]) < 1e-6);
    }
    // buildParas / paras2vertex layouts: base class [cams 1..C-1, photos], DoubleSide [ds, photos]
    {
        MyMultiCameraCalibration mc(3);
        for (int v = 0; v < 2; ++v) mc.addPhotoVertex(v, eye4());
        std::vector<float> x(6 * 4);
        for (size_t i = 0; i < x.size(); ++i) x[i] = 0.01f * (float)(i % 6 + 1) * ((i / 6) % 2 ? -1.f : 1.f) + (i % 6 >= 3 ? 0.5f * (float)i : 0.f);
        mc.paras2vertex(x);
        EXPECT(mc._vertexList[0].pose == eye4());                    // camera 0 is the world frame
        EXPECT(maxdiff(mc.buildParaVector(), x) < 1e-6);
        EXPECT(mc._vertexList[4].pose[3] == x[6 * 3 + 3]);           // photo vertex 4 -> columns 18..23
    }
    {
        DoubleSideCalibration ds(2);
        for (int v = 0; v < 3; ++v) ds.addPhotoVertex(v, eye4());
        std::vector<float> x(6 * 4);
        for (size_t i = 0; i < x.size(); ++i) x[i] = 0.02f * (float)(i % 6) - 0.03f + (i % 6 >= 3 ? 0.25f * (float)i : 0.f);
        ds.paras2vertex(x);
        EXPECT(maxdiff(ds.buildParaVector(), x) < 1e-6);
        EXPECT(ds.doubleSide[11] == x[5]);                           // ds tvec first
        EXPECT(ds._vertexList[2].pose[3] == x[6 + 3]);               // first photo vertex after ds
    }
    // error behaviour: counts that disagree throw before any device work (CV_Assert analogue)
    {
        MyMultiCameraCalibration mc(1);
        mc.addPhotoVertex(0, eye4());
        mc._cameraMatrix[0] = {500, 0, 320, 0, 500, 240, 0, 0, 1};
        mc._distortCoeffs[0] = {0, 0, 0, 0, 0};
        mc._objectPointsForEachCamera[0].push_back(std::vector<float>(3 * 4, 0.f));
        mc._imagePointsForEachCamera[0].push_back(std::vector<float>(2 * 3, 0.f));   // 3 != 4
        mc._edgeList.emplace_back(0, 1, 0, eye4());
        std::vector<float> x(6, 0.f), err;
        EXPECT(throws([&] { mc.computeProjectError(x); }));
        MyMultiCameraCalibration mc2(2);
        mc2._distortCoeffs[0] = {0, 0, 0, 0, 0};
        mc2._distortCoeffs[1] = {0, 0, 0, 0};                        // cameras differ in terms
        mc2.addPhotoVertex(0, eye4());
        mc2._objectPointsForEachCamera[0].push_back(std::vector<float>(3, 0.f));
        mc2._imagePointsForEachCamera[0].push_back(std::vector<float>(2, 0.f));
        mc2._edgeList.emplace_back(0, 2, 0, eye4());
        EXPECT(throws([&] { mc2.optimizeExtrinsics(); }));
        MyMultiCameraCalibration mc3(1);                             // edge to a missing photo slot
        mc3._edgeList.emplace_back(0, 1, 5, eye4());
        EXPECT(throws([&] { mc3.optimizeExtrinsics(); }));
    }
    // solvePnP (cv::solvePnP restated): exact synthetic views, planar and non-planar, with
    // Brown-Conrady and rational distortion, recover the pose
    {
        const double K[9] = {1200, 0, 960, 0, 1180, 540, 0, 0, 1};
        const std::vector<std::vector<double>> Ds = {{-0.1, 0.05, 1e-4, -2e-4, 0.0}, {-0.12, 0.08, 2e-4, 1e-4, 0.01, 0.002, -0.001, 0.003}};
        for (const auto& D : Ds)
            for (int planar = 0; planar < 2; ++planar) {
                std::vector<double> obj;
                for (int i = 0; i < 8; ++i)
                    for (int j = 0; j < 11; ++j)
                        obj.insert(obj.end(), {40.0 * j, 40.0 * i, planar ? 0.0 : 15.0 * std::sin(0.7 * i + 0.3 * j)});
                const int n = (int)obj.size() / 3;
                const double r[3] = {0.3, -0.4, 0.2}, t[3] = {-150.0, -90.0, 1300.0};
                std::vector<double> img(2 * n);
                mcc::pnp::projectPoints(obj.data(), n, r, t, K, D, img.data());
                double rr[3], tt[3];
                const double rms = mcc::pnp::solvePnP(obj.data(), img.data(), n, K, D, rr, tt);
                EXPECT(rms >= 0 && rms < 1e-6);
                for (int k = 0; k < 3; ++k) {
                    EXPECT(std::fabs(rr[k] - r[k]) < 1e-7);
                    EXPECT(std::fabs(tt[k] - t[k]) < 1e-4);
                }
            }
    }
    // FileStorage: write XML and YAML, read back every kind
    for (const char* ext : {".xml", ".yaml"}) {
        const std::string fn = std::string("/tmp/mcc_storage_selftest") + ext;
        {
            mcc::storage::FileStorage fs(fn, mcc::storage::FileStorage::WRITE);
            fs.write("nCameras", 3);
            fs.write("meanReprojectError", 0.123456789012345);
            fs.write("name", std::string("rig"));
            mcc::storage::Mat m(2, 3, 'd');
            for (int k = 0; k < 6; ++k) m.data[k] = 0.1 * k - 0.25;
            fs.write("M", m);
            mcc::storage::Mat pts(4, 1, 'f', 2);
            for (int k = 0; k < 8; ++k) pts.data[k] = (double)(float)(1.5f * k + 0.3f);
            fs.write("pts", pts);
        }
        mcc::storage::FileStorage in(fn, mcc::storage::FileStorage::READ);
        EXPECT(in.isOpened());
        EXPECT(in["nCameras"].toInt() == 3);
        EXPECT(std::fabs(in["meanReprojectError"].toReal() - 0.123456789012345) < 1e-15);
        EXPECT(in["name"].str == "rig");
        EXPECT(in["M"].type == mcc::storage::Node::MAT && in["M"].mat.rows == 2 && in["M"].mat.cols == 3);
        EXPECT(in["M"].mat.data[5] == 0.1 * 5 - 0.25);
        EXPECT(in["pts"].mat.channels == 2 && in["pts"].mat.depth == 'f' && in["pts"].mat.data[7] == (double)(float)(1.5f * 7 + 0.3f));
        EXPECT(in["missing"].empty());
        EXPECT(in.keys().size() == 5);
    }
    std::printf("selftest %s (%d failures)\n", g_fail ? "FAILED" : "ok", g_fail);
    return g_fail ? 1 : 0;
}

template <class T>
static std::vector<T> rd(std::ifstream& f, size_t n) {
    std::vector<T> v(n);
    f.read(reinterpret_cast<char*>(v.data()), (std::streamsize)(n * sizeof(T)));
    if (!f) throw std::runtime_error("truncated input");
    return v;
}

static void put(std::ofstream& o, const char* key, const std::vector<double>& v) {
    o << key << ' ' << v.size();
    char b[40];
    for (double d : v) {
        std::snprintf(b, sizeof b, " %.17g", d);
        o << b;
    }
    o << '\n';
}

static int run(const char* in, const char* outp) {
    std::ifstream f(in, std::ios::binary);
    if (!f) throw std::runtime_error("cannot open input");
    const auto h = rd<int>(f, 11);
    if (h[0] != 0x4d434331) throw std::runtime_error("bad magic");
    const int model = h[1], C = h[2], V = h[3], E = h[4], nd = h[5], corners = h[6];
    const bool has_ds = h[7] != 0, has_cp = h[8] != 0;
    const double eps = rd<double>(f, 1)[0];
    const auto ecam = rd<int>(f, E), ephoto = rd<int>(f, E), eside = rd<int>(f, E), eoff = rd<int>(f, E),
               en = rd<int>(f, E);
    const auto obj = rd<float>(f, 3 * (size_t)corners), img = rd<float>(f, 2 * (size_t)corners);
    const auto K = rd<float>(f, 9 * (size_t)C), D = rd<float>(f, (size_t)nd * C), xi = rd<float>(f, C);
    std::vector<double> dsp;
    std::vector<float> cp;
    if (has_ds) dsp = rd<double>(f, 16);
    if (has_cp) cp = rd<float>(f, 16 * (size_t)C);
    const int P = (model == MCC_MODEL_DOUBLESIDE ? 6 : 6 * (C - 1)) + 6 * V;
    const auto x0 = rd<float>(f, P);

    const TermCriteria crit(h[9], h[10], eps);
    std::unique_ptr<MultiCameraCalibration> mc;
    if (model == MCC_MODEL_OMNI) {
        mc.reset(new MultiCameraCalibration(MultiCameraCalibration::OMNIDIRECTIONAL, C, crit));
    } else if (model == MCC_MODEL_PINHOLE) {
        auto* m = new MyMultiCameraCalibration(C, crit);
        if (has_ds) std::copy(dsp.begin(), dsp.end(), m->doubleSideTransform.begin());
        mc.reset(m);
    } else {
        auto* m = new DoubleSideCalibration(C, crit);
        for (int c = 0; c < C; ++c) std::copy(cp.begin() + 16 * c, cp.begin() + 16 * (c + 1), m->camerasPose[c].begin());
        mc.reset(m);
    }
    // the state initialize() leaves behind: intrinsics, photo vertices, edges with per-camera
    // photo indices into _objectPointsForEachCamera / _imagePointsForEachCamera
    for (int c = 0; c < C; ++c) {
        std::copy(K.begin() + 9 * c, K.begin() + 9 * (c + 1), mc->_cameraMatrix[c].begin());
        mc->_distortCoeffs[c].assign(D.begin() + nd * c, D.begin() + nd * (c + 1));
        mc->_xi[c] = xi[c];
    }
    for (int v = 0; v < V; ++v) mc->addPhotoVertex(v, eye4());
    for (int e = 0; e < E; ++e) {
        const int c = ecam[e];
        const int pi = (int)mc->_objectPointsForEachCamera[c].size();
        mc->_objectPointsForEachCamera[c].emplace_back(obj.begin() + 3 * (size_t)eoff[e], obj.begin() + 3 * (size_t)(eoff[e] + en[e]));
        mc->_imagePointsForEachCamera[c].emplace_back(img.begin() + 2 * (size_t)eoff[e], img.begin() + 2 * (size_t)(eoff[e] + en[e]));
        mc->_edgeList.emplace_back(c, C + ephoto[e], pi, eye4());
        mc->_edgeList.back().patternSide = eside[e];
    }

    std::ofstream o(outp);
    // the seam at x0 (exact parameters, no pose round trip)
    std::vector<double> jinv, jte, delta;
    mc->computeJacobianExtrinsic(x0, jinv, jte, delta);
    put(o, "delta", delta);
    put(o, "jte", jte);
    put(o, "jtj_inv_size", {(double)jinv.size()});
    std::vector<float> xe(x0);
    const double pe = mc->computeProjectError(xe);
    std::vector<double> ee;
    for (const auto& ed : mc->_edgeList) ee.push_back(ed.reprojecterror);
    put(o, "pe_mean", {pe});
    put(o, "pe_edge", ee);
    // the reference's flow: poses -> buildParas -> optimizeExtrinsics -> paras2vertex
    mc->paras2vertex(x0);
    const auto xb = mc->buildParaVector();
    put(o, "x_built", std::vector<double>(xb.begin(), xb.end()));
    const double err = mc->optimizeExtrinsics();
    const auto xo = mc->buildParaVector();
    put(o, "opt_error", {err});
    put(o, "opt_iters", {(double)mc->iterations()});
    put(o, "opt_change", {mc->lastChange()});
    put(o, "x_opt_built", std::vector<double>(xo.begin(), xo.end()));
    // a second run on the same object reuses the device problem (and converges immediately)
    const double err2 = mc->optimizeExtrinsics();
    put(o, "opt2_error", {err2});
    put(o, "opt2_iters", {(double)mc->iterations()});
    o.close();
    std::printf("run ok: P=%d iters=%d err=%.9g\n", P, mc->iterations(), err);
    return 0;
}

int main(int argc, char** argv) {
    try {
        if (argc >= 2 && !std::strcmp(argv[1], "selftest")) return selftest();
        if (argc >= 4 && !std::strcmp(argv[1], "run")) return run(argv[2], argv[3]);
        if (argc >= 3 && !std::strcmp(argv[1], "storage")) {
            mcc::storage::FileStorage fs(argv[2], mcc::storage::FileStorage::READ);
            if (!fs.isOpened()) throw std::runtime_error("cannot open");
            for (const std::string& k : fs.keys()) {
                const mcc::storage::Node& n = fs[k];
                if (n.type == mcc::storage::Node::MAT)
                    std::printf("%s mat %d %d %d\n", k.c_str(), n.mat.rows, n.mat.cols, n.mat.channels);
                else if (n.type == mcc::storage::Node::SEQ)
                    std::printf("%s seq %zu %s\n", k.c_str(), n.seq.size(),
                                n.seq.empty() ? "-" : (n.seq[0].type == mcc::storage::Node::MAT ? "mat" : "scalar"));
                else
                    std::printf("%s scalar\n", k.c_str());
            }
            return 0;
        }
    } catch (const std::exception& e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 2;
    }
    std::fprintf(stderr, "usage: %s selftest | run <in.bin> <out.txt>\n", argv[0]);
    return 2;
}
