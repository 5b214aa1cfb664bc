// multicalib.cpp -- the reference sample's problem construction and driver around the GPU
// optimiser (include/mcc_multicalib.hpp):
//   MyMultiCameraCalibration(...)   src/mymulticalib.cpp:72-131  (camera configs, double side)
//   loadImages(outliers)            src/mymulticalib.cpp:182-405 (corner files, solvePnP, filter)
//   initialize()                    src/mymulticalib.cpp:615-666 (graph BFS pose chaining)
//   removeOutlier()                 src/mymulticalib.cpp:406-423
//   reset() / run()                 src/multicalib.cpp:127-152
//   writeParameters(...)            src/multicalib.cpp:1092-1127, src/mymulticalib.cpp:424-456
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <filesystem>
#include <iostream>

#include "mcc_multicalib.hpp"
#include "mcc_omnidir.hpp"
#include "mcc_pnp.hpp"
#include "mcc_storage.hpp"

namespace mcc {
namespace multicalib {

namespace {

namespace stg = mcc::storage;
constexpr int INVALID = -2;

// pose algebra in double, results rounded to the reference's CV_32F poses
void to_d(const Pose& P, double* D) {
    for (int k = 0; k < 16; ++k) D[k] = P[k];
}
Pose to_f(const double* D) {
    Pose P;
    for (int k = 0; k < 16; ++k) P[k] = (float)D[k];
    return P;
}
void mul4(const double* A, const double* B, double* C) {
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            double s = 0.0;
            for (int k = 0; k < 4; ++k) s += A[4 * i + k] * B[4 * k + j];
            C[4 * i + j] = s;
        }
}
// Mat::inv of a 4 x 4 (Gauss-Jordan with partial pivoting, as DECOMP_LU would)
void inv4(const double* A, double* X) {
    double M[4][8];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 8; ++j) M[i][j] = j < 4 ? A[4 * i + j] : (j - 4 == i ? 1.0 : 0.0);
    for (int k = 0; k < 4; ++k) {
        int p = k;
        for (int i = k + 1; i < 4; ++i)
            if (std::fabs(M[i][k]) > std::fabs(M[p][k])) p = i;
        if (M[p][k] == 0.0) throw std::runtime_error("singular pose in initialize()");
        if (p != k)
            for (int j = 0; j < 8; ++j) std::swap(M[k][j], M[p][j]);
        const double d = M[k][k];
        for (int j = 0; j < 8; ++j) M[k][j] /= d;
        for (int i = 0; i < 4; ++i) {
            if (i == k) continue;
            const double f = M[i][k];
            for (int j = 0; j < 8; ++j) M[i][j] -= f * M[k][j];
        }
    }
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) X[4 * i + j] = M[i][4 + j];
}

stg::Mat pose_mat(const Pose& P) {
    stg::Mat m(4, 4, 'f');
    for (int k = 0; k < 16; ++k) m.data[k] = P[k];
    return m;
}

// cv::Mat -> flat values of a points matrix: N x k (1 channel) or N x 1 (k channels)
std::vector<double> points_of(const stg::Node& n, int k, const std::string& file, const char* key) {
    if (n.type != stg::Node::MAT) throw std::runtime_error(file + ": no matrix '" + key + "'");
    const stg::Mat& m = n.mat;
    if ((m.cols * m.channels) % k != 0 && (m.rows * m.cols * m.channels) % k != 0)
        throw std::runtime_error(file + ": '" + key + "' is not a list of " + std::to_string(k) + "-vectors");
    return m.data;
}

bool is_valid_pose(const float t[3]) {   // isValidPose (src/multicalib.cpp:104-126): 300 < |t| < 3000 mm
    const float r = std::sqrt(t[0] * t[0] + t[1] * t[1] + t[2] * t[2]);
    return r < 3000.f && r > 300.f;
}

}  // namespace

// ---------------------------------------------------------------- base class
double MultiCameraCalibration::run() {
    loadImages();
    initialize();
    return optimizeExtrinsics();
}

std::vector<std::string> MultiCameraCalibration::readStringList() const {
    stg::FileStorage fs(_filename, stg::FileStorage::READ);
    if (!fs.isOpened()) throw std::runtime_error("cannot read the image list " + _filename);
    const std::vector<std::string> keys = fs.keys();
    if (keys.empty()) throw std::runtime_error(_filename + ": empty image list");
    const stg::Node& n = fs[keys[0]];   // getFirstTopLevelNode
    std::vector<std::string> l;
    for (const stg::Node& k : n.seq) {
        if (k.type != stg::Node::STRING) throw std::runtime_error(_filename + ": list entries must be file names");
        l.push_back(k.str);
    }
    return l;
}

void MultiCameraCalibration::loadImages() {
    namespace fsys = std::filesystem;
    const std::vector<std::string> file_list = readStringList();
    if (file_list.size() < 2) throw std::runtime_error(_filename + ": the list holds no view after the pattern");
    const fsys::path base = fsys::path(_filename).parent_path();
    // entry 0 is the pattern image (only the feature matcher reads it); the others are
    // "cameraIdx-timestamp.*" (src/multicalib.cpp:199-218)
    for (size_t i = 1; i < file_list.size(); ++i) {
        fsys::path f(file_list[i]);
        if (f.is_relative() && !base.empty() && !fsys::exists(f)) f = base / f;
        const std::string ext = f.extension().string();
        if (ext != ".yaml" && ext != ".yml" && ext != ".xml") f.replace_extension(".yaml");   // image -> its corners
        int cameraVertex = -1, timestamp = 0;
        if (std::sscanf(f.stem().string().c_str(), "%d-%d", &cameraVertex, &timestamp) != 2 || cameraVertex < 0 ||
            cameraVertex >= _nCamera)
            throw std::runtime_error(file_list[i] + ": expected a 'cameraIdx-timestamp' name with cameraIdx < " +
                                     std::to_string(_nCamera));
        filesEachCameraFull[cameraVertex].push_back(f.string());
        timestampFull[cameraVertex].push_back(timestamp);
    }
    for (int camera = 0; camera < _nCamera; ++camera) {   // calibrate each camera individually
        Size size;
        std::vector<std::vector<mcc::omnidir::Vec3d>> objs;
        std::vector<std::vector<mcc::omnidir::Vec2d>> imgs;
        for (size_t imgIdx = 0; imgIdx < filesEachCameraFull[camera].size(); ++imgIdx) {
            const std::string& file = filesEachCameraFull[camera][imgIdx];
            stg::FileStorage fs(file, stg::FileStorage::READ);
            if (!fs.isOpened()) throw std::runtime_error("cannot read " + file);
            const bool tut = !fs["imagePoints"].empty();
            const std::vector<double> img = points_of(fs[tut ? "imagePoints" : "corners"], 2, file, "imagePoints");
            const std::vector<double> obj = points_of(fs[tut ? "objectPoints" : "objects"], 3, file, "objectPoints");
            const int n = (int)img.size() / 2;
            if ((int)obj.size() != 3 * n) throw std::runtime_error(file + ": image and object points differ in count");
            const stg::Node& sz = fs["imageSize"];
            if (sz.seq.size() == 2) size = Size(sz.seq[0].toInt(), sz.seq[1].toInt());   // image.size()
            if (n > _nMiniMatches) {   // (int)imgObj[0].total() > _nMiniMatches
                std::vector<float> fi(img.size()), fo(obj.size());   // the finder's CV_32F points
                for (size_t k = 0; k < img.size(); ++k) fi[k] = (float)img[k];
                for (size_t k = 0; k < obj.size(); ++k) fo[k] = (float)obj[k];
                std::vector<mcc::omnidir::Vec3d> o3(n);
                std::vector<mcc::omnidir::Vec2d> i2(n);
                for (int k = 0; k < n; ++k) {   // calibrate converts CV_32F to CV_64F
                    o3[k] = {(double)fo[3 * k], (double)fo[3 * k + 1], (double)fo[3 * k + 2]};
                    i2[k] = {(double)fi[2 * k], (double)fi[2 * k + 1]};
                }
                objs.push_back(std::move(o3));
                imgs.push_back(std::move(i2));
                _imagePointsForEachCamera[camera].push_back(std::move(fi));
                _objectPointsForEachCamera[camera].push_back(std::move(fo));
                timestampAvailable[camera].push_back(timestampFull[camera][imgIdx]);
            } else if (_verbose) {
                std::cout << "image " << file << " has too few matched points " << std::endl;
            }
        }
        if (objs.empty()) throw std::runtime_error("camera " + std::to_string(camera) + " has no usable view");
        if (size.width <= 0 || size.height <= 0)
            throw std::runtime_error("camera " + std::to_string(camera) + ": no imageSize in its corner files");
        if (_camType != OMNIDIRECTIONAL)
            throw std::runtime_error(
                "MultiCameraCalibration::loadImages: PINHOLE intrinsics need cv::calibrateCamera, which is not "
                "restated here; use MyMultiCameraCalibration with camera configs");
        std::array<double, 9> K{};
        std::array<double, 4> D{};
        double xi = 0;
        std::vector<mcc::omnidir::Vec3d> om, t;
        std::vector<int> idx;
        const double rms = mcc::omnidir::calibrate(objs, imgs, size, K, xi, D, om, t, _flags,
                                                   TermCriteria(TermCriteria::COUNT + TermCriteria::EPS, 300, 1e-7),
                                                   &idx, _device);
        for (int k = 0; k < 9; ++k) _cameraMatrix[camera][k] = (float)K[k];   // convertTo(CV_32F)
        _distortCoeffs[camera].assign({(float)D[0], (float)D[1], (float)D[2], (float)D[3]});
        _xi[camera] = (float)xi;
        for (size_t i = 0; i < om.size(); ++i) {   // edges from the calibration's view poses (:296-312)
            const std::array<float, 3> r{(float)om[i][0], (float)om[i][1], (float)om[i][2]};
            const std::array<float, 3> tv{(float)t[i][0], (float)t[i][1], (float)t[i][2]};
            _omEachCamera[camera].push_back(r);
            _tEachCamera[camera].push_back(tv);
            const int timestamp = timestampAvailable[camera][idx[i]];
            const int photoVertex = getPhotoVertex(timestamp);
            _edgeList.push_back(edge(camera, photoVertex, idx[i], rt_to_pose(r.data(), tv.data())));
        }
        if (_verbose) {
            std::cout << "initialized for camera " << camera << " rms = " << rms << std::endl;
            std::cout << "xi for camera " << camera << " is " << _xi[camera] << std::endl;
        }
    }
    release();
}

void MultiCameraCalibration::graphTraverse(int begin, std::vector<int>& order, std::vector<int>& pre,
                                           std::vector<std::vector<std::pair<int, int>>>* adjacency) const {
    const int nV = (int)_vertexList.size();
    // buildGraph: G(c, p) = G(p, c) = edgeIdx + 1, a later edge of the same pair overwrites
    std::vector<std::vector<std::pair<int, int>>> adj(nV);
    auto link = [&](int a, int b, int e) {
        for (auto& q : adj[a])
            if (q.first == b) {
                q.second = e;
                return;
            }
        adj[a].push_back({b, e});
    };
    for (int e = 0; e < (int)_edgeList.size(); ++e) {
        const int c = _edgeList[e].cameraVertex, p = _edgeList[e].photoVertex;
        if (c < 0 || c >= nV || p < 0 || p >= nV) throw std::runtime_error("edge refers to a missing vertex");
        link(c, p, e);
        link(p, c, e);
    }
    for (auto& a : adj) std::sort(a.begin(), a.end());   // findRowNonZero: increasing index
    order.clear();
    pre.assign(nV, INVALID);
    if (begin < 0 || begin >= nV) throw std::runtime_error("graphTraverse: bad start vertex");
    std::vector<char> visited(nV, 0);
    std::vector<int> queue{begin};
    visited[begin] = 1;
    pre[begin] = -1;
    order.push_back(begin);
    for (size_t h = 0; h < queue.size(); ++h) {
        const int v = queue[h];
        for (const auto& q : adj[v])
            if (!visited[q.first]) {
                visited[q.first] = 1;
                queue.push_back(q.first);
                order.push_back(q.first);
                pre[q.first] = v;
            }
    }
    if (adjacency) *adjacency = std::move(adj);
}

void MultiCameraCalibration::initialize() { chainPoses(true); }

void MultiCameraCalibration::chainPoses(bool setCameras) {
    std::vector<int> order, pre;
    std::vector<std::vector<std::pair<int, int>>> adj;
    graphTraverse(0, order, pre, &adj);
    for (int i = 0; i < _nCamera; ++i)
        if (pre[i] == INVALID) std::cout << "camera" << i << "is not connected" << std::endl;
    const double* dsInv = nullptr;
    double dsi[16];
    if (auto* my = dynamic_cast<MyMultiCameraCalibration*>(this)) {
        bool any = false;
        for (double v : my->doubleSideTransform) any = any || v != 0.0;
        if (any) {
            inv4(my->doubleSideTransform.data(), dsi);
            dsInv = dsi;
        }
    }
    for (size_t i = 1; i < order.size(); ++i) {
        const int v = order[i], pv = pre[v];
        int e = -1;
        for (const auto& q : adj[v])
            if (q.first == pv) e = q.second;
        const edge& eg = _edgeList[e];
        double prePose[16], preInv[16], T[16], out[16];
        to_d(_vertexList[pv].pose, prePose);
        inv4(prePose, preInv);
        to_d(eg.transform, T);
        if (eg.patternSide == BACK_PATTERN) {   // front pose = back pose * doubleSideTransform^-1
            if (!dsInv) throw std::runtime_error("BACK edge without doubleSideTransform");
            double t2[16];
            mul4(T, dsInv, t2);
            std::copy(t2, t2 + 16, T);
        }
        if (v < _nCamera) {
            if (!setCameras) continue;             // DoubleSide: fixed cameras
            mul4(T, preInv, out);                  // camera: transform * prePose^-1
        } else {
            mul4(preInv, T, out);                  // photo:  prePose^-1 * transform
        }
        _vertexList[v].pose = to_f(out);
        if (_verbose && v < _nCamera) std::cout << "initial pose for camera " << v << " set" << std::endl;
    }
    release();
}

void MultiCameraCalibration::reset() {
    _edgeList.clear();
    _vertexList.clear();
    for (int i = 0; i < _nCamera; ++i) _vertexList.emplace_back();
    for (int i = 0; i < _nCamera; ++i) {
        filesEachCameraFull[i].clear();
        timestampFull[i].clear();
        timestampAvailable[i].clear();
        _objectPointsForEachCamera[i].clear();
        _imagePointsForEachCamera[i].clear();
        _omEachCamera[i].clear();
        _tEachCamera[i].clear();
    }
    release();
}

void MultiCameraCalibration::writeParameters(const std::string& filename) {
    stg::FileStorage fs(filename, stg::FileStorage::WRITE);
    if (!fs.isOpened()) throw std::runtime_error("cannot open " + filename + " for writing");
    fs.write("nCameras", _nCamera);
    for (int c = 0; c < _nCamera; ++c) {
        const std::string i = std::to_string(c);
        stg::Mat K(3, 3, 'f');
        for (int k = 0; k < 9; ++k) K.data[k] = _cameraMatrix[c][k];
        stg::Mat D(1, (int)_distortCoeffs[c].size(), 'f');
        for (size_t k = 0; k < _distortCoeffs[c].size(); ++k) D.data[k] = _distortCoeffs[c][k];
        fs.write("camera_matrix_" + i, K);
        fs.write("camera_distortion_" + i, D);
        if (_camType == OMNIDIRECTIONAL) fs.write("xi_" + i, (double)_xi[c]);
        fs.write("camera_pose_" + i, pose_mat(_vertexList[c].pose));
    }
    fs.write("meanReprojectError", _error);
    for (size_t v = _nCamera; v < _vertexList.size(); ++v)
        fs.write("pose_timestamp_" + std::to_string(_vertexList[v].timestamp), pose_mat(_vertexList[v].pose));
    fs.release();
}

// ---------------------------------------------------------------- MyMultiCameraCalibration
MyMultiCameraCalibration::MyMultiCameraCalibration(const std::vector<std::string>& serials, int cameraType,
                                                   int nCameras, const std::string& dataFolder_,
                                                   const std::string& cameraConfigFolder_,
                                                   const std::string& doubleSideConfig, Size frontPatternSize,
                                                   Size backPatternSize, float, float, int verbose, int, int, int,
                                                   TermCriteria criteria, int device)
    : MultiCameraCalibration(cameraType, nCameras, criteria, device), cameraSerials(serials), dataFolder(dataFolder_),
      cameraConfigFolder(cameraConfigFolder_), _FrontPatternSize(frontPatternSize), _BackPatternSize(backPatternSize),
      timestampIsMulticamera(nCameras) {
    if ((int)serials.size() != nCameras) throw std::runtime_error("one camera serial per camera is required");
    _verbose = verbose;
    // readcameraIntrinsics (src/mymulticalib.cpp:118-131)
    for (int c = 0; c < nCameras; ++c) {
        const std::string fn = cameraConfigFolder + "/" + serials[c] + ".xml";
        stg::FileStorage fs(fn, stg::FileStorage::READ);
        if (!fs.isOpened()) throw std::runtime_error("cannot read camera config " + fn);
        const stg::Node& K = fs["Intrinsics"];
        const stg::Node& D = fs["Distortion"];
        if (K.type != stg::Node::MAT || K.mat.data.size() != 9) throw std::runtime_error(fn + ": Intrinsics must be 3x3");
        if (D.type != stg::Node::MAT) throw std::runtime_error(fn + ": no Distortion");
        for (int k = 0; k < 9; ++k) _cameraMatrix[c][k] = (float)K.mat.data[k];
        _distortCoeffs[c].assign(D.mat.data.begin(), D.mat.data.end());
    }
    // readDoubleSide (src/mymulticalib.cpp:99-103)
    if (!doubleSideConfig.empty()) {
        stg::FileStorage fs(doubleSideConfig, stg::FileStorage::READ);
        if (!fs.isOpened()) throw std::runtime_error("cannot read " + doubleSideConfig);
        const stg::Node& T = fs["transform"];
        if (T.type != stg::Node::MAT || T.mat.data.size() != 16)
            throw std::runtime_error(doubleSideConfig + ": transform must be 4x4");
        std::copy(T.mat.data.begin(), T.mat.data.end(), doubleSideTransform.begin());
    }
}

void MyMultiCameraCalibration::loadImages(const std::set<std::string>& outliers) {
    namespace fsys = std::filesystem;
    if (!outliers.empty()) m_outliers = outliers;
    const int backN = _BackPatternSize.width * _BackPatternSize.height;
    for (int cam = 0; cam < _nCamera; ++cam) {   // loadOneSerial (src/mymulticalib.cpp:262-301)
        const std::string folder = stg::resolve_path(dataFolder + "/" + cameraSerials[cam]);
        std::vector<std::string> files;
        if (fsys::is_directory(folder))
            for (const auto& de : fsys::directory_iterator(folder))
                if (de.path().extension() == ".yaml") files.push_back(de.path().string());
        std::sort(files.begin(), files.end());   // cv::glob returns sorted paths
        double K[9];
        for (int k = 0; k < 9; ++k) K[k] = _cameraMatrix[cam][k];
        const std::vector<double> D(_distortCoeffs[cam].begin(), _distortCoeffs[cam].end());
        for (const std::string& file : files) {
            if (m_outliers.count(file)) {
                std::cout << "outlier:" << file << " skipped: " << std::endl;
                continue;
            }
            const int timestamp = std::stoi(fsys::path(file).stem().string());   // readTimestamps
            stg::FileStorage fs(file, stg::FileStorage::READ);                    // readCorners
            if (!fs.isOpened()) throw std::runtime_error("cannot read " + file);
            const std::vector<double> img = points_of(fs["corners"], 2, file, "corners");
            const std::vector<double> objd = points_of(fs["objects"], 3, file, "objects");
            const int n = (int)img.size() / 2;
            if ((int)objd.size() != 3 * n) throw std::runtime_error(file + ": corners and objects differ in count");
            std::vector<double> obj(objd.size());   // objectPoints.convertTo(CV_32F)
            for (size_t k = 0; k < objd.size(); ++k) obj[k] = (double)(float)objd[k];
            double r[3], t[3];   // calcPatternPose: cv::solvePnP
            if (mcc::pnp::solvePnP(obj.data(), img.data(), n, K, D, r, t) < 0)
                throw std::runtime_error(file + ": too few corners for solvePnP");
            const std::array<float, 3> om{(float)r[0], (float)r[1], (float)r[2]};
            const std::array<float, 3> tv{(float)t[0], (float)t[1], (float)t[2]};
            if (!is_valid_pose(tv.data())) {   // the reference asserts (src/mymulticalib.cpp:210, :297)
                if (strictReference) strict_abort("isValidPose(tvec)", "src/mymulticalib.cpp:210 (calcPatternPose)");
                ++invalidPoseCount;
                std::cout << "invalid pattern :" << invalidPoseCount << ", " << file << std::endl;
                continue;
            }
            if (!keepView(n)) continue;   // storeReaded: MyMulti keeps front-pattern views only (:237)
            filesEachCameraFull[cam].push_back(file);
            timestampFull[cam].push_back(timestamp);
            timestampAvailable[cam].push_back(timestamp);
            _omEachCamera[cam].push_back(om);
            _tEachCamera[cam].push_back(tv);
            std::vector<float> fi(img.size()), fo(obj.size());
            for (size_t k = 0; k < img.size(); ++k) fi[k] = (float)img[k];
            for (size_t k = 0; k < obj.size(); ++k) fo[k] = (float)obj[k];
            _imagePointsForEachCamera[cam].push_back(std::move(fi));
            _objectPointsForEachCamera[cam].push_back(std::move(fo));
        }
    }
    // identifyMultiCameraTimestamps (src/mymulticalib.cpp:314-347)
    setOfTimestampIsMulticamera.clear();
    for (int cam = 0; cam < _nCamera; ++cam) {
        timestampIsMulticamera[cam].clear();
        for (size_t i = 0; i < timestampAvailable[cam].size(); ++i) {
            const int ts = timestampAvailable[cam][i];
            const int n = (int)_imagePointsForEachCamera[cam][i].size() / 2;
            bool found = false;
            for (int c2 = 0; c2 < _nCamera && !found; ++c2) {
                if (c2 == cam) continue;
                for (size_t j = 0; j < timestampAvailable[c2].size() && !found; ++j)
                    found = timestampAvailable[c2][j] == ts &&
                            sameTimestampMatches(n, (int)_imagePointsForEachCamera[c2][j].size() / 2);
            }
            timestampIsMulticamera[cam].push_back(found);
            if (found) setOfTimestampIsMulticamera.insert(ts);
        }
    }
    // edges (src/mymulticalib.cpp:362-403)
    for (int cam = 0; cam < _nCamera; ++cam)
        for (int i = 0; i < (int)_omEachCamera[cam].size(); ++i) {
            const int ts = timestampAvailable[cam][i];
            if (!setOfTimestampIsMulticamera.count(ts)) continue;
            const int pv = getPhotoVertex(ts);
            Pose T = rt_to_pose(_omEachCamera[cam][i].data(), _tEachCamera[cam][i].data());
            edge eg(cam, pv, i, T);
            if ((int)_imagePointsForEachCamera[cam][i].size() / 2 == backN) eg.patternSide = BACK_PATTERN;
            _edgeList.push_back(eg);
        }
    release();
}

void MyMultiCameraCalibration::initialize() { MultiCameraCalibration::initialize(); }

std::set<std::string> MyMultiCameraCalibration::removeOutlier() {
    std::vector<edge> kept;
    std::set<std::string> names;
    int cnt = 0;
    for (const edge& eg : _edgeList) {
        if (eg.reprojecterror > 0.5f) {
            const std::string& f = filesEachCameraFull[eg.cameraVertex][eg.photoIndex];
            std::cout << "outlier:" << eg.reprojecterror << ":" << f << " removed" << std::endl;
            names.insert(f);
            ++cnt;
        } else {
            kept.push_back(eg);
        }
    }
    std::cout << "Totally " << cnt << " outlier removed" << std::endl;
    _edgeList = kept;
    release();
    return names;
}

void MyMultiCameraCalibration::reset() {
    MultiCameraCalibration::reset();
    for (auto& v : timestampIsMulticamera) v.clear();
    setOfTimestampIsMulticamera.clear();
}

void MyMultiCameraCalibration::writeParameters(const std::string& filename) {
    MultiCameraCalibration::writeParameters(filename);
    // writeParameters2config (src/mymulticalib.cpp:424-449): rewrite each camera config with
    // CameraMatrix = the camera's optimised pose
    const char* scalarNames[2] = {"depth_scale", "height"};
    const char* matNames[3] = {"CameraMatrix", "Intrinsics", "Distortion"};
    for (int c = 0; c < _nCamera; ++c) {
        const std::string fn = cameraConfigFolder + "/" + cameraSerials[c] + ".xml";
        double scalars[2] = {0.0, 0.0};
        stg::Mat mats[3];
        {
            stg::FileStorage in(fn, stg::FileStorage::READ);
            if (!in.isOpened()) throw std::runtime_error("cannot read camera config " + fn);
            for (int i = 0; i < 2; ++i)
                if (!in[scalarNames[i]].empty()) scalars[i] = in[scalarNames[i]].toReal();
            for (int i = 0; i < 3; ++i)
                if (in[matNames[i]].type == stg::Node::MAT) mats[i] = in[matNames[i]].mat;
        }
        mats[0] = pose_mat(_vertexList[c].pose);
        stg::FileStorage out(fn, stg::FileStorage::WRITE);
        for (int i = 0; i < 2; ++i) out.write(scalarNames[i], (double)(float)scalars[i]);
        for (int i = 0; i < 3; ++i)
            if (!mats[i].empty()) out.write(matNames[i], mats[i]);
        out.release();
    }
}

// ---------------------------------------------------------------- DoubleSideCalibration
DoubleSideCalibration::DoubleSideCalibration(const std::vector<std::string>& serials, int cameraType, int nCameras,
                                             const std::string& dataFolder_, const std::string& cameraConfigFolder_,
                                             Size frontPatternSize, Size backPatternSize, float pw, float ph,
                                             int verbose, int showExtration, int nMiniMatches, int flags,
                                             TermCriteria criteria, int device)
    : MyMultiCameraCalibration(serials, cameraType, nCameras, dataFolder_, cameraConfigFolder_, "", frontPatternSize,
                               backPatternSize, pw, ph, verbose, showExtration, nMiniMatches, flags, criteria, device),
      camerasPose(nCameras, eye4()) {
    for (int c = 0; c < nCameras; ++c) {   // loadCameraPose (src/doubleSide.cpp:276-287)
        const std::string fn = cameraConfigFolder + "/" + serials[c] + ".xml";
        stg::FileStorage fs(fn, stg::FileStorage::READ);
        const stg::Node& P = fs["CameraMatrix"];
        if (P.type != stg::Node::MAT || P.mat.data.size() != 16) throw std::runtime_error(fn + ": CameraMatrix must be 4x4");
        for (int k = 0; k < 16; ++k) camerasPose[c][k] = (float)P.mat.data[k];
        _vertexList[c].pose = camerasPose[c];
    }
}

void DoubleSideCalibration::initialize() {
    // initializeDoublesideTransform: the first photo vertex with a FRONT and a BACK edge
    int ef = -1, eb = -1;
    for (size_t v = _nCamera; v < _vertexList.size() && (ef < 0 || eb < 0); ++v) {
        ef = eb = -1;
        for (size_t e = 0; e < _edgeList.size(); ++e) {
            if (_edgeList[e].photoVertex != (int)v) continue;
            if (_edgeList[e].patternSide == BACK_PATTERN) {
                if (eb < 0) eb = (int)e;
            } else if (ef < 0) {
                ef = (int)e;
            }
        }
    }
    if (ef < 0 || eb < 0) throw std::runtime_error("DoubleSide initialize: no photo is seen from both sides");
    // findTransformOfTwoEdge: frontpose = camPose_f^-1 T_f, backpose = camPose_b^-1 T_b,
    // doubleSideTransform = frontpose^-1 backpose
    double cf[16], cb[16], tf[16], tb[16], cfi[16], cbi[16], fp[16], bp[16], fpi[16], ds[16];
    to_d(camerasPose[_edgeList[ef].cameraVertex], cf);
    to_d(camerasPose[_edgeList[eb].cameraVertex], cb);
    to_d(_edgeList[ef].transform, tf);
    to_d(_edgeList[eb].transform, tb);
    inv4(cf, cfi);
    inv4(cb, cbi);
    mul4(cfi, tf, fp);
    mul4(cbi, tb, bp);
    inv4(fp, fpi);
    mul4(fpi, bp, ds);
    for (int k = 0; k < 16; ++k) doubleSideTransform[k] = (double)(float)ds[k];   // CV_32F pose product
    doubleSide = to_f(ds);
    for (int c = 0; c < _nCamera; ++c) _vertexList[c].pose = camerasPose[c];
    chainPoses(false);
}

void DoubleSideCalibration::writeParameters(const std::string&) {
    stg::FileStorage fs("doublesideTransform.yaml", stg::FileStorage::WRITE);
    stg::Mat T(4, 4, 'f');
    for (int k = 0; k < 16; ++k) T.data[k] = doubleSide[k];
    fs.write("transform", T);
    fs.release();
}

void DoubleSideCalibration::reset() {
    MyMultiCameraCalibration::reset();
    for (int c = 0; c < _nCamera; ++c) _vertexList[c].pose = camerasPose[c];
}

}  // namespace multicalib
}  // namespace mcc
