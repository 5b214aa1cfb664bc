/*
 * mcc_cvmat.hpp -- the minimal cv::Mat this build's source-compatible headers need (SURVEY.md §7:
 * "a minimal in-repo shim [of] cv::Mat"), so that the reference's cv::Mat-typed extension seam
 * (include/opencv2/ccalib/multicalib.hpp:157, :176-191; mymulticalib.hpp:164-172;
 * doubleSide.hpp:133-164) can be declared with its own signatures, and a subclass written the way
 * the reference writes MyMultiCameraCalibration / DoubleSideCalibration compiles against it.
 *
 * What it is: a reference-counted 2-D matrix of CV_32F / CV_64F elements (1-4 channels), with
 * OpenCV's header semantics (copies share data; clone() deep-copies; rowRange / colRange / row /
 * col are views into the parent), element access (at, ptr), convertTo, t(), matrix products,
 * element-wise + / -, scalar scaling and cv::norm.  Type codes follow OpenCV (CV_32F = 5,
 * CV_64F = 6, CV_MAKETYPE(depth, cn) = depth + ((cn - 1) << 3)).  No OpenCV code is used or
 * needed.  It replaces OpenCV: include/opencv2/ccalib/multicalib.hpp refuses to compile after the real
 * OpenCV headers (#error), since the seam reads matrices through this shim's accessors.
 */
#ifndef MCC_CVMAT_HPP
#define MCC_CVMAT_HPP

#include <algorithm>
#include <cmath>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#if defined(OPENCV_CORE_HPP) || defined(OPENCV_CORE_MAT_HPP)
#define MCC_HAVE_OPENCV 1
#endif

#ifndef MCC_HAVE_OPENCV
#define CV_32F 5
#define CV_64F 6
#define CV_CN_SHIFT 3
#define CV_MAKETYPE(depth, cn) ((depth) + (((cn)-1) << CV_CN_SHIFT))
#define CV_32FC1 CV_MAKETYPE(CV_32F, 1)
#define CV_32FC2 CV_MAKETYPE(CV_32F, 2)
#define CV_32FC3 CV_MAKETYPE(CV_32F, 3)
#define CV_64FC1 CV_MAKETYPE(CV_64F, 1)
#define CV_64FC2 CV_MAKETYPE(CV_64F, 2)
#define CV_64FC3 CV_MAKETYPE(CV_64F, 3)

namespace cv {

template <typename T, int n>
struct Vec {
    T val[n] = {};
    Vec() = default;
    Vec(T a, T b, T c = T(), T d = T()) {
        const T v[4] = {a, b, c, d};
        for (int i = 0; i < n && i < 4; ++i) val[i] = v[i];
    }
    T& operator[](int i) { return val[i]; }
    const T& operator[](int i) const { return val[i]; }
};
using Vec2f = Vec<float, 2>;
using Vec3f = Vec<float, 3>;
using Vec3d = Vec<double, 3>;

class Mat {
public:
    int rows = 0, cols = 0;

    Mat() = default;
    Mat(int r, int c, int type) { create(r, c, type); }
    Mat(int r, int c, int type, double value) {
        create(r, c, type);
        setTo(value);
    }
    static Mat zeros(int r, int c, int type) { return Mat(r, c, type, 0.0); }
    static Mat ones(int r, int c, int type) { return Mat(r, c, type, 1.0); }
    static Mat eye(int n, int type) {
        Mat m = zeros(n, n, type);
        for (int i = 0; i < n; ++i) m.set(i, i, 1.0);
        return m;
    }

    void create(int r, int c, int type) {
        if (r < 0 || c < 0) throw std::invalid_argument("cv::Mat: negative size");
        if ((type & 7) != CV_32F && (type & 7) != CV_64F) throw std::invalid_argument("cv::Mat: CV_32F / CV_64F only");
        rows = r;
        cols = c;
        type_ = type;
        step_ = (size_t)c * elemSize();
        buf_ = std::make_shared<std::vector<unsigned char>>(std::max<size_t>(step_ * r, 1), 0);
        data = buf_->data();
    }
    int type() const { return type_; }
    int depth() const { return type_ & 7; }
    int channels() const { return 1 + (type_ >> CV_CN_SHIFT); }
    size_t elemSize1() const { return depth() == CV_64F ? 8 : 4; }
    size_t elemSize() const { return elemSize1() * channels(); }
    size_t total() const { return (size_t)rows * cols; }
    bool empty() const { return total() == 0; }
    bool isContinuous() const { return step_ == (size_t)cols * elemSize() || rows <= 1; }
    size_t step() const { return step_; }

    template <typename T>
    T* ptr(int r = 0) { return reinterpret_cast<T*>(data + (size_t)r * step_); }
    template <typename T>
    const T* ptr(int r = 0) const { return reinterpret_cast<const T*>(data + (size_t)r * step_); }
    // at<T>(i): i-th element of a row or column vector (OpenCV's 1-index form)
    template <typename T>
    T& at(int i) { return rows == 1 ? at<T>(0, i) : at<T>(i, 0); }
    template <typename T>
    const T& at(int i) const { return rows == 1 ? at<T>(0, i) : at<T>(i, 0); }
    template <typename T>
    T& at(int r, int c) {
        check_at<T>(r, c);
        return ptr<T>(r)[c];
    }
    template <typename T>
    const T& at(int r, int c) const {
        check_at<T>(r, c);
        return ptr<T>(r)[c];
    }

    // element (r, c) of a single-channel matrix as double, whatever the depth
    double get(int r, int c) const {
        return depth() == CV_64F ? (double)ptr<double>(r)[c] : (double)ptr<float>(r)[c];
    }
    void set(int r, int c, double v) {
        if (depth() == CV_64F) ptr<double>(r)[c] = v;
        else ptr<float>(r)[c] = (float)v;
    }
    Mat& setTo(double v) {
        const int cn = channels();
        for (int r = 0; r < rows; ++r)
            for (int c = 0; c < cols * cn; ++c) {
                if (depth() == CV_64F) ptr<double>(r)[c] = v;
                else ptr<float>(r)[c] = (float)v;
            }
        return *this;
    }

    // views (share the data, OpenCV semantics)
    Mat rowRange(int a, int b) const {
        range_check(a, b, rows);
        Mat m = *this;
        m.data = data + (size_t)a * step_;
        m.rows = b - a;
        return m;
    }
    Mat colRange(int a, int b) const {
        range_check(a, b, cols);
        Mat m = *this;
        m.data = data + (size_t)a * elemSize();
        m.cols = b - a;
        return m;
    }
    Mat row(int r) const { return rowRange(r, r + 1); }
    Mat col(int c) const { return colRange(c, c + 1); }

    Mat clone() const {
        Mat m(rows, cols, type_);
        for (int r = 0; r < rows; ++r) std::memcpy(m.ptr<unsigned char>(r), ptr<unsigned char>(r), (size_t)cols * elemSize());
        return m;
    }
    // copyTo: a destination of the same size and type receives the values in place (so views of a
    // larger matrix are written through); anything else is re-created
    void copyTo(Mat& dst) const {
        if (dst.data == data && dst.rows == rows && dst.cols == cols && dst.type_ == type_) return;
        if (dst.rows != rows || dst.cols != cols || dst.type_ != type_ || !dst.buf_) dst.create(rows, cols, type_);
        for (int r = 0; r < rows; ++r) std::memcpy(dst.ptr<unsigned char>(r), ptr<unsigned char>(r), (size_t)cols * elemSize());
    }
    // into a temporary view, as OpenCV's OutputArray allows: m.copyTo(J.rowRange(a, b).colRange(c, d))
    void copyTo(Mat&& dst) const {
        Mat d = dst;
        copyTo(d);
    }
    void convertTo(Mat& dst, int rtype, double alpha = 1.0) const {
        const int cn = channels();
        Mat out(rows, cols, CV_MAKETYPE(rtype & 7, cn));
        for (int r = 0; r < rows; ++r)
            for (int c = 0; c < cols * cn; ++c) {
                const double v = alpha * (depth() == CV_64F ? ptr<double>(r)[c] : (double)ptr<float>(r)[c]);
                if (out.depth() == CV_64F) out.ptr<double>(r)[c] = v;
                else out.ptr<float>(r)[c] = (float)v;
            }
        dst = out;
    }
    // a continuous matrix with cn channels and r rows over the same data (OpenCV's reshape)
    Mat reshape(int cn, int r = 0) const {
        if (!isContinuous()) throw std::invalid_argument("cv::Mat::reshape: not continuous");
        const size_t scalars = total() * channels();
        if (cn <= 0) cn = channels();
        if (r <= 0) r = rows;
        if (scalars % ((size_t)cn * r)) throw std::invalid_argument("cv::Mat::reshape: bad size");
        Mat m = *this;
        m.type_ = CV_MAKETYPE(depth(), cn);
        m.rows = r;
        m.cols = (int)(scalars / ((size_t)cn * r));
        m.step_ = (size_t)m.cols * m.elemSize();
        return m;
    }
    Mat t() const {
        one_channel();
        Mat m(cols, rows, type_);
        for (int r = 0; r < rows; ++r)
            for (int c = 0; c < cols; ++c) m.set(c, r, get(r, c));
        return m;
    }

    friend Mat operator*(const Mat& a, const Mat& b) {
        a.one_channel();
        b.one_channel();
        if (a.cols != b.rows || a.depth() != b.depth()) throw std::invalid_argument("cv::Mat: product size / type");
        Mat m(a.rows, b.cols, a.type_);
        if (a.depth() == CV_64F) {   // row-major i-k-j: each output row accumulates over k in order
            std::vector<double> acc(b.cols);
            for (int i = 0; i < a.rows; ++i) {
                std::fill(acc.begin(), acc.end(), 0.0);
                const double* ai = a.ptr<double>(i);
                for (int k = 0; k < a.cols; ++k) {
                    const double aik = ai[k];
                    if (aik == 0.0) continue;   // exact: the dense J of a BA problem is mostly zeros
                    const double* bk = b.ptr<double>(k);
                    for (int j = 0; j < b.cols; ++j) acc[j] += aik * bk[j];
                }
                std::copy(acc.begin(), acc.end(), m.ptr<double>(i));
            }
            return m;
        }
        for (int i = 0; i < a.rows; ++i)
            for (int j = 0; j < b.cols; ++j) {
                double s = 0.0;
                for (int k = 0; k < a.cols; ++k) s += a.get(i, k) * b.get(k, j);
                m.set(i, j, s);
            }
        return m;
    }
    friend Mat operator*(double s, const Mat& a) { return a.map([s](double v) { return s * v; }); }
    friend Mat operator*(const Mat& a, double s) { return s * a; }
    friend Mat operator+(const Mat& a, const Mat& b) { return a.zip(b, [](double x, double y) { return x + y; }); }
    friend Mat operator-(const Mat& a, const Mat& b) { return a.zip(b, [](double x, double y) { return x - y; }); }
    friend Mat operator-(const Mat& a) { return a.map([](double v) { return -v; }); }

    unsigned char* data = nullptr;

private:
    template <typename T>
    void check_at(int r, int c) const {
        if (r < 0 || r >= rows || c < 0 || (size_t)c * sizeof(T) >= (size_t)cols * elemSize())
            throw std::out_of_range("cv::Mat::at: index out of range");
    }
    static void range_check(int a, int b, int n) {
        if (a < 0 || b < a || b > n) throw std::out_of_range("cv::Mat: range out of bounds");
    }
    void one_channel() const {
        if (channels() != 1) throw std::invalid_argument("cv::Mat: single-channel matrices only");
    }
    template <typename F>
    Mat map(F f) const {
        Mat m(rows, cols, type_);
        const int cn = channels();
        for (int r = 0; r < rows; ++r)
            for (int c = 0; c < cols * cn; ++c) {
                const double v = depth() == CV_64F ? ptr<double>(r)[c] : (double)ptr<float>(r)[c];
                if (depth() == CV_64F) m.ptr<double>(r)[c] = f(v);
                else m.ptr<float>(r)[c] = (float)f(v);
            }
        return m;
    }
    template <typename F>
    Mat zip(const Mat& b, F f) const {
        if (b.rows != rows || b.cols != cols || b.type_ != type_) throw std::invalid_argument("cv::Mat: operand size / type");
        Mat m(rows, cols, type_);
        const int cn = channels();
        for (int r = 0; r < rows; ++r)
            for (int c = 0; c < cols * cn; ++c) {
                const double x = depth() == CV_64F ? ptr<double>(r)[c] : (double)ptr<float>(r)[c];
                const double y = depth() == CV_64F ? b.ptr<double>(r)[c] : (double)b.ptr<float>(r)[c];
                if (depth() == CV_64F) m.ptr<double>(r)[c] = f(x, y);
                else m.ptr<float>(r)[c] = (float)f(x, y);
            }
        return m;
    }

    int type_ = CV_32F;
    size_t step_ = 0;
    std::shared_ptr<std::vector<unsigned char>> buf_;
};

using InputArray = const Mat&;
using OutputArray = Mat&;

// cv::norm (NORM_L2) of every element, accumulated in double
inline double norm(const Mat& m) {
    double s = 0.0;
    const int cn = m.channels();
    for (int r = 0; r < m.rows; ++r)
        for (int c = 0; c < m.cols * cn; ++c) {
            const double v = m.depth() == CV_64F ? m.ptr<double>(r)[c] : (double)m.ptr<float>(r)[c];
            s += v * v;
        }
    return std::sqrt(s);
}

}  // namespace cv
#endif  // MCC_HAVE_OPENCV

#endif
