/*
 * mcc_storage.hpp -- the subset of cv::FileStorage the reference's loaders and writers use, in
 * plain C++ (no OpenCV in this build).
 *
 * Read (XML `<opencv_storage>` or YAML `%YAML:1.0`): top-level keys holding an int, a real, a
 * string, an `opencv-matrix` (rows, cols, dt, data) or a sequence of those.  That covers
 *   - the corner files `fs["corners"] >> imagePoints; fs["objects"] >> objectPoints`
 *     (src/mymulticalib.cpp:182-192),
 *   - the camera configs `fs["Intrinsics"]`, `fs["Distortion"]`, `depth_scale`, `height`,
 *     `CameraMatrix` (src/mymulticalib.cpp:118-131, 424-449),
 *   - the double-side transform `fs["transform"]` (src/mymulticalib.cpp:100-103),
 *   - the tutorial data (tutorials/data/omni_calib_data.xml: sequences of matrices).
 * Write: the same kinds, XML or YAML chosen by the file extension (.xml / .yml / .yaml), in
 * OpenCV's layout (writeParameters, src/multicalib.cpp:1092-1127).
 *
 * Errors throw std::runtime_error (cv::Exception analogue).
 */
#ifndef MCC_STORAGE_HPP
#define MCC_STORAGE_HPP

#include <map>
#include <string>
#include <vector>

namespace mcc {
namespace storage {

// dense matrix: rows x cols x channels, row-major with interleaved channels; depth is the
// OpenCV dt letter ('u','c','w','s','i','f','d')
struct Mat {
    int rows = 0, cols = 0, channels = 1;
    char depth = 'd';
    std::vector<double> data;
    Mat() = default;
    Mat(int r, int c, char dt = 'd', int ch = 1) : rows(r), cols(c), channels(ch), depth(dt), data((size_t)r * c * ch, 0.0) {}
    bool empty() const { return data.empty(); }
    size_t total() const { return (size_t)rows * cols; }
    double& at(int r, int c, int ch = 0) { return data[((size_t)r * cols + c) * channels + ch]; }
    double at(int r, int c, int ch = 0) const { return data[((size_t)r * cols + c) * channels + ch]; }
};

struct Node {
    enum Type { NONE, INT, REAL, STRING, MAT, SEQ };
    Type type = NONE;
    double real = 0.0;
    long long integer = 0;
    std::string str;
    Mat mat;
    std::vector<Node> seq;
    bool empty() const { return type == NONE; }
    double toReal() const;       // INT or REAL
    int toInt() const;
};

// Path remapping for callers that hard-code their data and config locations (the reference
// sample does: samples/multi_cameras_calibration.cpp:50-52).  MCC_PATH_MAP="from=to[;from=to...]"
// rewrites a path that starts with `from` (the first matching entry, once) to start with `to`;
// without the variable a path is returned unchanged.  Every file the loaders and writers open and
// every folder they list goes through it.
std::string resolve_path(const std::string& path);

class FileStorage {
public:
    enum { READ = 0, WRITE = 1 };
    FileStorage(const std::string& path, int flags);
    ~FileStorage();
    FileStorage(const FileStorage&) = delete;
    FileStorage& operator=(const FileStorage&) = delete;

    bool isOpened() const { return opened_; }
    // READ: the top-level node `key` (type NONE when absent)
    const Node& operator[](const std::string& key) const;
    std::vector<std::string> keys() const { return order_; }

    // WRITE (kept in insertion order, flushed by release() / the destructor)
    void write(const std::string& key, int v);
    void write(const std::string& key, double v);
    void write(const std::string& key, const std::string& v);
    void write(const std::string& key, const Mat& m);
    void release();

private:
    std::string path_;
    int flags_;
    bool opened_ = false, xml_ = true;
    std::map<std::string, Node> nodes_;
    std::vector<std::string> order_;
    void put(const std::string& key, Node n);
};

}  // namespace storage
}  // namespace mcc

#endif
