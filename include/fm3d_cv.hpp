/*
 * fm3d_cv.hpp -- drop-in stand-ins for the includes of the reference's main.cpp (main.cpp:8-20):
 *
 *   #include <lmmin.h>                                  (lmfit: the LM runs inside the GPU kernel)
 *   #include <opencv2/opencv.hpp>                       -> namespace cv below (the types and the few
 *   #include <opencv2/nonfree/features2d.hpp>              functions main.cpp calls)
 *   #include "DescriptorsMatcher/descriptorsmatcher.h"  -> class DescriptorsMatcher
 *   #include "Triangulator/singlecameratriangulator.h"  -> class SingleCameraTriangulator
 *   #include "Triangulator/normaloptimizer.h"           -> class NormalOptimizer
 *   #include "Triangulator/neighborhoodsgenerator.h"    -> class NeighborhoodsGenerator
 *   #include "pclvisualizerthread.h" / "tools.h"        -> drawMatches, drawBackProjectedPoints,
 *                                                          pcl::PointCloud / pcl::Normal and the
 *                                                          view* functions (no-op viewers)
 *
 * Replacing those lines by `#include "fm3d_cv.hpp"` lets the reference main.cpp compile unchanged:
 * tests/test_compat_main.py::test_reference_main_compiles_with_includes_swapped does exactly that
 * to /root/reference/main.cpp when it is readable, and compiles examples/main_dropin.cpp (the same
 * call sequence written for this repository), whose outputs it checks against the Python mirror of
 * the classes.  The classes keep
 * the reference's names, constructors, method signatures and out-parameter semantics and run the
 * hot path through the C ABI (fm3d.h) on GPU 0:
 *   DescriptorsMatcher        descriptorsmatcher.h:39-111   (ctor :47, compare / crosscompare /
 *                                                             compareWithNNDR :55-77)
 *   SingleCameraTriangulator  singlecameratriangulator.h:52-93
 *   NormalOptimizer           normaloptimizer.h:43-59
 *   NeighborhoodsGenerator    neighborhoodsgenerator.h:78-97 (square and circular methods)
 *   MOSAIC                    mosaic.h:47-70 (the pipeline as a descriptor extractor)
 *
 * What differs, and why:
 *   - feature detection/description (descriptorsmatcher.cpp:110-115): when main.cpp:94 passes
 *     empty vectors, the settings' detector / extractor runs on the GPU (SURF of
 *     build/settings.yml, fm3d_surf_detect; ORB, SIFT, FAST, STAR, MSER, ADAPTIVE and the BRISK
 *     and FREAK extractors too, any pair of them, see fm3d.h); a type the reference does not build
 *     (FM3D_FEAT_OTHER) falls back to the image's feature side files:
 *     <image>.kpts.f32 (N x 2 float32 positions) and <image>.desc.u8 (N x 128 uint8) or
 *     <image>.desc.f32 (N x 128 float32) -- FeatureOptions.ExtractorType ORB / BRISK / FREAK
 *     selects Hamming matching on <image>.desc.u8 rows of 32 / 64 bytes (descriptorsmatcher.cpp:64-71);
 *   - the matcher is exact brute force, ties to the lowest train index;
 *   - extractDescriptorsFromPatches runs the settings' SURF, SIFT, ORB, BRISK or FREAK extractor on the GPU;
 *   - the PCL viewer is visual only: start/stopVisualizerThread and the view* functions are
 *     no-ops; drawMatches / drawBackProjectedPoints draw with plain loops, in the reference's
 *     colours (cv::RNG(0xFFF0FF0F), random_color);
 *   - errors throw fm3d::compat::Error where the reference exit()s.
 */
#ifndef FM3D_CV_HPP
#define FM3D_CV_HPP

#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "fm3d_compat.hpp"

#ifndef CV_8U
#define CV_8U 0
#define CV_32F 5
#define CV_64F 6
#define CV_8UC1 0
#define CV_8UC3 16
#define CV_32FC1 5
#define CV_64FC1 6
#define CV_64FC2 14
#define CV_64FC3 22
#endif
#ifndef CV_LOAD_IMAGE_GRAYSCALE
#define CV_LOAD_IMAGE_GRAYSCALE 0
#endif

namespace cv {

typedef unsigned char uchar;

struct Point2f {
    float x = 0, y = 0;
    Point2f() {}
    Point2f(float x_, float y_) : x(x_), y(y_) {}
};

struct KeyPoint {
    Point2f pt;
    float size = 0, angle = -1, response = 0;
    int octave = 0, class_id = -1;
    KeyPoint() {}
    KeyPoint(float x, float y, float size_, float angle_ = -1, float response_ = 0, int octave_ = 0, int class_id_ = -1)
        : pt(x, y), size(size_), angle(angle_), response(response_), octave(octave_), class_id(class_id_) {}
};

struct DMatch {  // the field layout of fm3d_dmatch (the ABI writes these directly)
    int queryIdx = -1, trainIdx = -1, imgIdx = -1;
    float distance = 0;
};
static_assert(sizeof(DMatch) == sizeof(fm3d_dmatch), "DMatch layout");

template <typename T, int n>
struct Vec {
    T val[n];
    Vec() {
        for (int i = 0; i < n; i++) val[i] = T(0);
    }
    Vec(T a, T b) : Vec() {
        val[0] = a;
        if (n > 1) val[1] = b;
    }
    Vec(T a, T b, T c) : Vec() {
        val[0] = a;
        if (n > 1) val[1] = b;
        if (n > 2) val[2] = c;
    }
    T& operator[](int i) { return val[i]; }
    const T& operator[](int i) const { return val[i]; }
};
typedef Vec<double, 2> Vec2d;
typedef Vec<double, 3> Vec3d;
typedef Vec<uchar, 3> Vec3b;

template <typename T, int n>
inline std::ostream& operator<<(std::ostream& o, const Vec<T, n>& v) {
    o << "[";
    for (int i = 0; i < n; i++) o << (i ? ", " : "") << +v.val[i];
    return o << "]";
}

struct Matx44d {  // row major
    double val[16];
    Matx44d() {
        for (double& v : val) v = 0;
    }
    double& operator()(int r, int c) { return val[4 * r + c]; }
    double operator()(int r, int c) const { return val[4 * r + c]; }
};
inline std::ostream& operator<<(std::ostream& o, const Matx44d& m) {
    o << "[";
    for (int i = 0; i < 16; i++) o << m.val[i] << (i == 15 ? "]" : (i % 4 == 3 ? ";\n " : ", "));
    return o;
}

struct Scalar {
    double val[4];
    Scalar(double a = 0, double b = 0, double c = 0, double d = 0) : val{a, b, c, d} {}
    double operator[](int i) const { return val[i]; }
    double& operator[](int i) { return val[i]; }
};

struct Size {
    int width = 0, height = 0;
    Size() {}
    Size(int w, int h) : width(w), height(h) {}
};

// cv::RNG (OpenCV 2.4 core): multiply-with-carry, next() = the low 32 bits of the new state
class RNG {
public:
    explicit RNG(uint64_t state = 0xffffffffULL) : state_(state ? state : 0xffffffffULL) {}
    unsigned next() {
        state_ = (uint64_t)(unsigned)state_ * 4164903690U + (unsigned)(state_ >> 32);
        return (unsigned)state_;
    }
    operator unsigned() { return next(); }

private:
    uint64_t state_;
};

// CV_RGB(r, g, b) is Scalar(b, g, r, 0); random_color (tools.cpp:116-120)
inline Scalar random_color(RNG& rng) {
    const int color = (int)rng.next();
    return Scalar((color >> 16) & 255, (color >> 8) & 255, color & 255, 0);
}

// cv::Mat: 2-D, continuous, reference-counted storage (the element types main.cpp's path uses)
class Mat {
public:
    int rows = 0, cols = 0;
    uchar* data = nullptr;
    Mat() {}
    Mat(int rows_, int cols_, int type_) { create(rows_, cols_, type_); }
    Mat(Size s, int type_, const Scalar& v = Scalar()) {
        create(s.height, s.width, type_);
        if (v[0] != 0 || v[1] != 0 || v[2] != 0) fill(v);
    }
    static Mat zeros(Size s, int type_) { return Mat(s, type_); }
    static Mat zeros(int rows_, int cols_, int type_) { return Mat(rows_, cols_, type_); }
    void create(int rows_, int cols_, int type_) {
        rows = rows_;
        cols = cols_;
        type__ = type_;
        buf_ = std::make_shared<std::vector<uchar> >((size_t)rows * cols * elemSize(), 0);
        data = buf_->data();
    }
    int type() const { return type__; }
    int depth() const { return type__ & 7; }
    int channels() const { return (type__ >> 3) + 1; }
    size_t elemSize1() const { return depth() == CV_8U ? 1 : depth() == CV_32F ? 4 : 8; }
    size_t elemSize() const { return elemSize1() * channels(); }
    size_t step() const { return (size_t)cols * elemSize(); }
    bool empty() const { return data == nullptr || rows == 0 || cols == 0; }
    size_t total() const { return (size_t)rows * cols; }
    Mat clone() const {
        Mat m;
        m.rows = rows;
        m.cols = cols;
        m.type__ = type__;
        m.source_ = source_;
        if (buf_) {
            m.buf_ = std::make_shared<std::vector<uchar> >(*buf_);
            m.data = m.buf_->data();
        }
        return m;
    }
    uchar* ptr(int r) { return data + (size_t)r * step(); }
    const uchar* ptr(int r) const { return data + (size_t)r * step(); }
    template <typename T>
    T& at(int r, int c) {
        return reinterpret_cast<T*>(ptr(r))[c];
    }
    template <typename T>
    const T& at(int r, int c) const {
        return reinterpret_cast<const T*>(ptr(r))[c];
    }
    template <typename T>
    T& at(int i) {  // element i of a row or column vector
        return reinterpret_cast<T*>(data)[i];
    }
    template <typename T>
    const T& at(int i) const {
        return reinterpret_cast<const T*>(data)[i];
    }
    // the file an image was read from (imread): the feature side files sit next to it
    const std::string& source() const { return source_; }
    void set_source(const std::string& s) { source_ = s; }

private:
    void fill(const Scalar& v) {
        for (size_t i = 0; i < total(); i++)
            for (int ch = 0; ch < channels(); ch++) {
                uchar* p = data + i * elemSize() + ch * elemSize1();
                if (depth() == CV_8U)
                    *p = (uchar)v[ch];
                else if (depth() == CV_32F)
                    *reinterpret_cast<float*>(p) = (float)v[ch];
                else
                    *reinterpret_cast<double*>(p) = v[ch];
            }
    }
    int type__ = 0;
    std::shared_ptr<std::vector<uchar> > buf_;
    std::string source_;
};

namespace detail {
inline std::vector<char> slurp(const std::string& path, bool& ok) {
    std::ifstream f(path, std::ios::binary);
    ok = (bool)f;
    if (!ok) return {};
    return std::vector<char>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}
// PGM / PPM header: magic, width, height, maxval, '#' comments between tokens
inline bool pnm_header(const std::vector<char>& b, std::string& magic, int& w, int& h, int& maxval, size_t& off) {
    size_t i = 0;
    auto token = [&](std::string& t) {
        t.clear();
        while (i < b.size()) {
            const char c = b[i];
            if (c == '#' && t.empty()) {
                while (i < b.size() && b[i] != '\n') i++;
            } else if (std::isspace((unsigned char)c)) {
                if (!t.empty()) break;
                i++;
            } else {
                if (t.size() > 16) return false;
                t += c;
                i++;
            }
        }
        return !t.empty();
    };
    std::string tw, th, tm;
    if (!token(magic) || !token(tw) || !token(th) || !token(tm)) return false;
    char* e = nullptr;
    const long lw = std::strtol(tw.c_str(), &e, 10);
    if (*e) return false;
    const long lh = std::strtol(th.c_str(), &e, 10);
    if (*e) return false;
    const long lm = std::strtol(tm.c_str(), &e, 10);
    if (*e) return false;
    if (lw <= 0 || lh <= 0 || lw > (1 << 20) || lh > (1 << 20) || lm <= 0 || lm > 255) return false;
    w = (int)lw;
    h = (int)lh;
    maxval = (int)lm;
    off = i + 1;  // one whitespace byte after maxval
    return off <= b.size();
}
}  // namespace detail

// cv::imread of 8-bit PGM (P5) / PPM (P6) files; flags CV_LOAD_IMAGE_GRAYSCALE (0) converts P6 to
// gray with OpenCV's weights.  An unreadable or malformed file gives an empty Mat, as in OpenCV.
inline Mat imread(const std::string& path, int flags = 1) {
    bool ok;
    std::vector<char> b = detail::slurp(path, ok);
    std::string magic;
    int w = 0, h = 0, maxval = 0;
    size_t off = 0;
    if (!ok || !detail::pnm_header(b, magic, w, h, maxval, off) || (magic != "P5" && magic != "P6")) return Mat();
    const int ch = magic == "P5" ? 1 : 3;
    if (b.size() - off < (size_t)w * h * ch) return Mat();
    const uchar* src = reinterpret_cast<const uchar*>(b.data() + off);
    Mat m;
    if (ch == 1) {
        m.create(h, w, CV_8UC1);
        std::memcpy(m.data, src, (size_t)w * h);
    } else if (flags == CV_LOAD_IMAGE_GRAYSCALE) {
        m.create(h, w, CV_8UC1);
        for (size_t i = 0; i < (size_t)w * h; i++)  // RGB file order; cvtColor BGR2GRAY weights
            m.data[i] = (uchar)std::lround(0.299 * src[3 * i] + 0.587 * src[3 * i + 1] + 0.114 * src[3 * i + 2]);
    } else {
        m.create(h, w, CV_8UC3);
        for (size_t i = 0; i < (size_t)w * h; i++)  // stored BGR, like OpenCV
            for (int k = 0; k < 3; k++) m.data[3 * i + k] = src[3 * i + 2 - k];
    }
    m.set_source(path);
    return m;
}

// cv::imwrite: CV_8UC1 -> P5, CV_8UC3 (BGR) -> P6
inline bool imwrite(const std::string& path, const Mat& m) {
    if (m.empty() || m.depth() != CV_8U || (m.channels() != 1 && m.channels() != 3)) return false;
    std::ofstream f(path, std::ios::binary);
    if (!f) return false;
    f << (m.channels() == 1 ? "P5" : "P6") << "\n" << m.cols << " " << m.rows << "\n255\n";
    if (m.channels() == 1) {
        f.write(reinterpret_cast<const char*>(m.data), (std::streamsize)m.total());
    } else {
        std::vector<uchar> rgb(m.total() * 3);
        for (size_t i = 0; i < m.total(); i++)
            for (int k = 0; k < 3; k++) rgb[3 * i + k] = m.data[3 * i + 2 - k];
        f.write(reinterpret_cast<const char*>(rgb.data()), (std::streamsize)rgb.size());
    }
    return (bool)f;
}

// cv::FileNode / cv::FileStorage over fm3d_settings_lookup (the %YAML:1.0 subset settings.yml uses)
class FileNode {
public:
    FileNode() {}
    FileNode(const std::string& path, const std::string& key) : path_(path), key_(key) {}
    FileNode operator[](const std::string& name) const { return FileNode(path_, key_.empty() ? name : key_ + "." + name); }
    FileNode operator[](const char* name) const { return (*this)[std::string(name)]; }
    bool empty() const {
        int len = 0;
        return fm3d_settings_lookup(path_.c_str(), key_.c_str(), nullptr, 0, &len) != FM3D_OK;
    }
    std::string text() const {
        int len = 0;
        if (fm3d_settings_lookup(path_.c_str(), key_.c_str(), nullptr, 0, &len) != FM3D_OK) return std::string();
        std::vector<char> b((size_t)len + 1);
        fm3d_settings_lookup(path_.c_str(), key_.c_str(), b.data(), len + 1, &len);
        return std::string(b.data(), (size_t)len);
    }
    operator double() const { return std::strtod(text().c_str(), nullptr); }
    operator float() const { return (float)(double)*this; }
    operator int() const { return (int)(double)*this; }
    operator std::string() const { return text(); }

private:
    std::string path_, key_;
};
inline void operator>>(const FileNode& n, std::string& v) { v = n.text(); }
inline void operator>>(const FileNode& n, double& v) { v = (double)n; }
inline void operator>>(const FileNode& n, float& v) { v = (float)n; }
inline void operator>>(const FileNode& n, int& v) { v = (int)n; }
inline void operator>>(const FileNode& n, std::vector<double>& v) {
    std::string t = n.text();
    for (char& c : t)
        if (c == '[' || c == ']' || c == ',') c = ' ';
    std::istringstream ss(t);
    v.clear();
    double x;
    while (ss >> x) v.push_back(x);
}

class FileStorage {
public:
    enum { READ = 0 };
    FileStorage() {}
    FileStorage(const std::string& path, int flags) { open(path, flags); }
    bool open(const std::string& path, int /*flags*/) {
        path_ = path;
        fm3d_settings s;
        opened_ = fm3d_settings_load(path.c_str(), &s) == FM3D_OK;
        return opened_;
    }
    bool isOpened() const { return opened_; }
    void release() { opened_ = false; }
    FileNode operator[](const std::string& name) const { return FileNode(path_, name); }
    FileNode operator[](const char* name) const { return FileNode(path_, name); }
    // fm3d: the settings of the hot path, read once
    fm3d_settings settings() const {
        fm3d_settings s;
        fm3d::compat::check(nullptr, fm3d_settings_load(path_.c_str(), &s));
        return s;
    }
    const std::string& path() const { return path_; }

private:
    std::string path_;
    bool opened_ = false;
};

}  // namespace cv

namespace fm3d {
namespace cvshim {

template <class T>
inline std::vector<T> read_side(const std::string& path, bool& ok) {
    std::vector<char> b = cv::detail::slurp(path, ok);
    std::vector<T> v(ok ? b.size() / sizeof(T) : 0);
    if (!v.empty()) std::memcpy(v.data(), b.data(), v.size() * sizeof(T));
    return v;
}

// OpenCV's data tables that the library cannot ship: ORB's bit_pattern_31_ (orb.cpp) and FREAK's
// DEF_PAIRS (freak.cpp).  FM3D_ORB_PATTERN names a raw file of 512 (x, y) int32 test points,
// FM3D_FREAK_PAIRS one of 512 int32 pair indices; without them the drop-in's ORB at patchSize 31
// runs on makeRandomPattern(31) and FREAK on the library's restated table, and one warning per
// process says so (the descriptors then differ from OpenCV's).
inline void load_tables(fm3d_ctx* c, const fm3d_settings& s) {
    bool ok = false;
    if (const char* p = std::getenv("FM3D_ORB_PATTERN")) {
        std::vector<int32_t> v = read_side<int32_t>(p, ok);
        ok = ok && v.size() == 1024;
        if (ok)
            fm3d::compat::check(c, fm3d_orb_set_pattern(c, v.data(), 512));
        else
            std::fprintf(stderr, "fm3d: FM3D_ORB_PATTERN=%s is not 512 int32 (x, y) points: ignored\n", p);
    }
    if (!ok && s.orbPatchSize == 31 && (s.detectorType == FM3D_FEAT_ORB || s.extractorType == FM3D_FEAT_ORB))
        std::fprintf(stderr, "fm3d: ORB runs on makeRandomPattern(31), not OpenCV's bit_pattern_31_: its descriptors "
                             "differ from OpenCV's (FM3D_ORB_PATTERN: a file of the table's 512 int32 (x, y) "
                             "points)\n");
    ok = false;
    if (const char* p = std::getenv("FM3D_FREAK_PAIRS")) {
        std::vector<int32_t> v = read_side<int32_t>(p, ok);
        ok = ok && v.size() == 512;
        if (ok)
            fm3d::compat::check(c, fm3d_freak_set_pairs(c, v.data(), 512));
        else
            std::fprintf(stderr, "fm3d: FM3D_FREAK_PAIRS=%s is not 512 int32 pair indices: ignored\n", p);
    }
    if (!ok && s.extractorType == FM3D_FEAT_FREAK)
        std::fprintf(stderr, "fm3d: FREAK runs on the library's restated DEF_PAIRS table, unverified against "
                             "OpenCV's (FM3D_FREAK_PAIRS: a file of OpenCV's 512 int32 pair indices)\n");
}

// one GPU context per process, shared by the reference classes (the reference's classes share
// state through the SingleCameraTriangulator pointer and the images they are given)
inline fm3d::compat::Device& device(const fm3d_settings& s) {
    static std::unique_ptr<fm3d::compat::Device> dev;
    if (!dev) {
        dev.reset(new fm3d::compat::Device(s, 0));
        load_tables(dev->ctx(), s);
    }
    return *dev;
}

inline std::string upper(std::string s) {
    for (char& c : s) c = (char)std::toupper((unsigned char)c);
    return s;
}

}  // namespace cvshim
}  // namespace fm3d

// ---------------------------------------------------------------- DescriptorsMatcher
class DescriptorsMatcher {
public:
    DescriptorsMatcher(cv::FileStorage& fs, cv::Mat& frame_a, cv::Mat& frame_b)
        : s_(fs.settings()), image_a_(frame_a), image_b_(frame_b) {
        std::string ex;
        fs["FeatureOptions"]["ExtractorType"] >> ex;
        ex = fm3d::cvshim::upper(ex);
        binary_ = ex == "ORB" || ex == "BRISK" || ex == "FREAK";  // LSH matcher in the reference (:64-71)
        fm3d::cvshim::device(s_);
    }
    // descriptorsmatcher.cpp:74-87
    void crosscompare(std::vector<std::vector<cv::DMatch> >& matchesAB, std::vector<std::vector<cv::DMatch> >& matchesBA,
                      std::vector<cv::KeyPoint>& kpts_a, std::vector<cv::KeyPoint>& kpts_b,
                      cv::Mat& completeDescriptors_a, cv::Mat& completeDescriptors_b) {
        features(image_a_, kpts_a, completeDescriptors_a);
        features(image_b_, kpts_b, completeDescriptors_b);
        knn(completeDescriptors_a, completeDescriptors_b, matchesAB);
        knn(completeDescriptors_b, completeDescriptors_a, matchesBA);
    }
    // descriptorsmatcher.cpp:89-105
    void compare(std::vector<std::vector<cv::DMatch> >& matches, std::vector<cv::KeyPoint>& kpts_a,
                 std::vector<cv::KeyPoint>& kpts_b, cv::Mat& completeDescriptors_a, cv::Mat& completeDescriptors_b) {
        features(image_a_, kpts_a, completeDescriptors_a);
        features(image_b_, kpts_b, completeDescriptors_b);
        knn(completeDescriptors_a, completeDescriptors_b, matches);
    }
    // descriptorsmatcher.cpp:107-131: matches are APPENDED (m[0] iff d0 <= eps * d1)
    void compareWithNNDR(double epsilon, std::vector<cv::DMatch>& matches, std::vector<cv::KeyPoint>& kpts_a,
                         std::vector<cv::KeyPoint>& kpts_b, cv::Mat& completeDescriptors_a,
                         cv::Mat& completeDescriptors_b) {
        features(image_a_, kpts_a, completeDescriptors_a);
        features(image_b_, kpts_b, completeDescriptors_b);
        const fm3d::compat::DescMat A = desc(completeDescriptors_a), B = desc(completeDescriptors_b);
        std::vector<fm3d_dmatch> tmp(A.rows > 0 ? A.rows : 1);
        int n = 0;
        fm3d_ctx* c = fm3d::cvshim::device(s_).ctx();
        fm3d::compat::check(c, fm3d_match_nndr(c, A.data, A.rows, B.data, B.rows, A.cols, A.type, epsilon, tmp.data(), &n));
        for (int i = 0; i < n; i++) matches.push_back(reinterpret_cast<const cv::DMatch&>(tmp[i]));
    }
    // descriptorsmatcher.cpp:133-174: per patch one keypoint at its centre, size = the patch edge,
    // described by the settings' SURF or SIFT extractor on the GPU; one descriptor row per patch
    void extractDescriptorsFromPatches(const std::vector<cv::Mat>& patchesVector, cv::Mat& descriptors) {
        if (patchesVector.empty()) throw fm3d::compat::Error(FM3D_ERR_INVALID, "no patches");  // descriptorsVector[0]
        const int size = patchesVector[0].rows;
        std::vector<uint8_t> all((size_t)patchesVector.size() * size * size);
        for (size_t i = 0; i < patchesVector.size(); i++) {
            const cv::Mat& m = patchesVector[i];
            if (m.rows != size || m.cols != size || m.type() != CV_8UC1)
                throw fm3d::compat::Error(FM3D_ERR_INVALID, "patches must be equal-size square 8-bit images");
            std::memcpy(&all[i * (size_t)size * size], m.data, (size_t)size * size);
        }
        fm3d_ctx* c = fm3d::cvshim::device(s_).ctx();
        int cols = 0, type = 0;
        fm3d::compat::check(c, fm3d_descriptor_info(c, &cols, &type));
        descriptors.create((int)patchesVector.size(), cols, type == FM3D_DESC_BITS ? CV_8UC1 : CV_32FC1);
        fm3d::compat::check(c, fm3d_extract_descriptors_from_patches_any(c, all.data(), (int)patchesVector.size(), size,
                                                                         descriptors.data));
    }

private:
    // the detector + extractor (:110-115): the settings' pair on the GPU (SURF, ORB, SIFT, FAST, STAR, MSER,
    // ADAPTIVE, the BRISK and FREAK extractors, mixed pairs); a type the reference does not build takes its
    // output from the images' side files
    // (<image>.kpts.f32 and <image>.desc.u8 / .desc.f32), or from the caller's keypoints + descriptors
    void features(const cv::Mat& img, std::vector<cv::KeyPoint>& kpts, cv::Mat& d) {
        if (s_.detectorType == FM3D_FEAT_SURF && s_.extractorType == FM3D_FEAT_SURF) {
            static_assert(sizeof(cv::KeyPoint) == sizeof(fm3d_keypoint), "cv::KeyPoint layout");
            fm3d_ctx* c = fm3d::cvshim::device(s_).ctx();
            const int dsize = s_.surfExtended ? 128 : 64;
            // one detection with room for one keypoint per 64 pixels; again only if more were found
            int cap = std::max(4096, img.cols * img.rows / 64), n = 0;
            std::vector<fm3d_keypoint> k;
            std::vector<float> f;
            for (;;) {
                k.resize(cap);
                f.resize((size_t)cap * dsize);
                fm3d::compat::check(c, fm3d_surf_detect(c, img.data, img.cols, img.rows, k.data(), cap, &n, f.data()));
                if (n <= cap) break;
                cap = n;
            }
            kpts.assign(n, cv::KeyPoint());
            if (n > 0) std::memcpy(static_cast<void*>(kpts.data()), k.data(), (size_t)n * sizeof(fm3d_keypoint));
            d.create(n, dsize, CV_32FC1);
            if (n > 0) std::memcpy(d.data, f.data(), (size_t)n * dsize * sizeof(float));
            return;
        }
        if (s_.detectorType == FM3D_FEAT_ORB && s_.extractorType == FM3D_FEAT_ORB) {
            // the reference's two calls (:110-115): detect, then compute on the detected keypoints
            fm3d_ctx* c = fm3d::cvshim::device(s_).ctx();
            int cap = std::max(1024, 2 * s_.orbNumFeatures), n = 0;
            std::vector<fm3d_keypoint> k;
            for (;;) {
                k.resize(cap);
                fm3d::compat::check(c, fm3d_orb_detect(c, img.data, img.cols, img.rows, k.data(), cap, &n, nullptr));
                if (n <= cap) break;
                cap = n;
            }
            std::vector<fm3d_keypoint> ko(n > 0 ? n : 1);
            std::vector<uint8_t> desc((size_t)(n > 0 ? n : 1) * 32);
            int m = 0;
            if (n > 0)
                fm3d::compat::check(c, fm3d_orb_compute(c, img.data, img.cols, img.rows, k.data(), n, ko.data(), nullptr,
                                                        &m, desc.data()));
            kpts.assign(m, cv::KeyPoint());
            if (m > 0) std::memcpy(static_cast<void*>(kpts.data()), ko.data(), (size_t)m * sizeof(fm3d_keypoint));
            d.create(m, 32, CV_8UC1);
            if (m > 0) std::memcpy(d.data, desc.data(), (size_t)m * 32);
            return;
        }
        if (s_.detectorType == FM3D_FEAT_SIFT && s_.extractorType == FM3D_FEAT_SIFT) {
            // the reference's two calls (:110-115): detect, then compute on the detected keypoints;
            // SIFT's descriptors are CV_32F rows holding integers 0..255
            fm3d_ctx* c = fm3d::cvshim::device(s_).ctx();
            int cap = std::max(4096, 2 * s_.siftNumFeatures), n = 0;
            std::vector<fm3d_keypoint> k;
            for (;;) {
                k.resize(cap);
                fm3d::compat::check(c, fm3d_sift_detect(c, img.data, img.cols, img.rows, k.data(), cap, &n, nullptr));
                if (n <= cap) break;
                cap = n;
            }
            std::vector<fm3d_keypoint> ko(n > 0 ? n : 1);
            std::vector<float> desc((size_t)(n > 0 ? n : 1) * 128);
            int m = 0;
            if (n > 0)
                fm3d::compat::check(c, fm3d_sift_compute(c, img.data, img.cols, img.rows, k.data(), n, ko.data(), nullptr,
                                                         &m, desc.data()));
            kpts.assign(m, cv::KeyPoint());
            if (m > 0) std::memcpy(static_cast<void*>(kpts.data()), ko.data(), (size_t)m * sizeof(fm3d_keypoint));
            d.create(m, 128, CV_32FC1);
            if (m > 0) std::memcpy(d.data, desc.data(), (size_t)m * 128 * sizeof(float));
            return;
        }
        if (s_.detectorType != FM3D_FEAT_OTHER && s_.extractorType != FM3D_FEAT_OTHER) {
            // any other pair built here (FAST, STAR, the ADAPTIVE mode, a detector of one type with an
            // extractor of another): the reference's two calls through fm3d_detect / fm3d_compute
            fm3d_ctx* c = fm3d::cvshim::device(s_).ctx();
            int cap = std::max(4096, img.cols * img.rows / 64), n = 0;
            std::vector<fm3d_keypoint> k;
            for (;;) {
                k.resize(cap);
                fm3d::compat::check(c, fm3d_detect(c, img.data, img.cols, img.rows, k.data(), cap, &n));
                if (n <= cap) break;
                cap = n;
            }
            int cols = 0, type = 0;
            fm3d::compat::check(c, fm3d_descriptor_info(c, &cols, &type));
            const size_t esz = type == FM3D_DESC_BITS ? 1 : sizeof(float);
            std::vector<fm3d_keypoint> ko(n > 0 ? n : 1);
            std::vector<uint8_t> desc((size_t)(n > 0 ? n : 1) * cols * esz);
            int m = 0;
            if (n > 0)
                fm3d::compat::check(c, fm3d_compute(c, img.data, img.cols, img.rows, k.data(), n, ko.data(), nullptr, &m,
                                                    desc.data()));
            kpts.assign(m, cv::KeyPoint());
            if (m > 0) std::memcpy(static_cast<void*>(kpts.data()), ko.data(), (size_t)m * sizeof(fm3d_keypoint));
            d.create(m, cols, type == FM3D_DESC_BITS ? CV_8UC1 : CV_32FC1);
            if (m > 0) std::memcpy(d.data, desc.data(), (size_t)m * cols * esz);
            return;
        }
        if (!kpts.empty() && !d.empty()) return;
        const std::string base = img.source();
        if (base.empty())
            throw fm3d::compat::Error(FM3D_ERR_INVALID, "no keypoints/descriptors given and the image has no file");
        bool ok;
        std::vector<float> xy = fm3d::cvshim::read_side<float>(base + ".kpts.f32", ok);
        if (!ok) throw fm3d::compat::Error(FM3D_ERR_INVALID, "feature detection is upstream: missing " + base + ".kpts.f32");
        const int n = (int)(xy.size() / 2);
        kpts.assign(n, cv::KeyPoint());
        for (int i = 0; i < n; i++) kpts[i].pt = cv::Point2f(xy[2 * i], xy[2 * i + 1]);
        std::vector<uint8_t> u8 = fm3d::cvshim::read_side<uint8_t>(base + ".desc.u8", ok);
        if (ok) {
            const int cols = n ? (int)(u8.size() / n) : (binary_ ? 32 : 128);
            if ((size_t)cols * n != u8.size()) throw fm3d::compat::Error(FM3D_ERR_INVALID, base + ".desc.u8: bad size");
            d.create(n, cols, CV_8UC1);
            if (!u8.empty()) std::memcpy(d.data, u8.data(), u8.size());
            return;
        }
        std::vector<float> f32 = fm3d::cvshim::read_side<float>(base + ".desc.f32", ok);
        if (!ok) throw fm3d::compat::Error(FM3D_ERR_INVALID, "feature detection is upstream: missing " + base + ".desc.u8/.f32");
        const int cols = n ? (int)(f32.size() / n) : 128;
        if ((size_t)cols * n != f32.size()) throw fm3d::compat::Error(FM3D_ERR_INVALID, base + ".desc.f32: bad size");
        d.create(n, cols, CV_32FC1);
        if (!f32.empty()) std::memcpy(d.data, f32.data(), f32.size() * 4);
    }
    fm3d::compat::DescMat desc(const cv::Mat& m) const {
        fm3d_desc_type t = binary_ ? FM3D_DESC_BITS : (m.depth() == CV_32F ? FM3D_DESC_F32 : FM3D_DESC_U8);
        if (m.depth() != CV_8U && m.depth() != CV_32F) throw fm3d::compat::Error(FM3D_ERR_INVALID, "descriptor type");
        return fm3d::compat::DescMat{m.rows, m.cols, t, m.data};
    }
    // knnMatch(k = 2): per query the neighbours that exist (two, or fewer for tiny train sets)
    void knn(const cv::Mat& a, const cv::Mat& b, std::vector<std::vector<cv::DMatch> >& out) {
        const fm3d::compat::DescMat A = desc(a), B = desc(b);
        if (A.cols != B.cols || A.type != B.type) throw fm3d::compat::Error(FM3D_ERR_INVALID, "descriptor matrices differ");
        std::vector<fm3d_dmatch> r((size_t)2 * (A.rows > 0 ? A.rows : 1));
        fm3d_ctx* c = fm3d::cvshim::device(s_).ctx();
        fm3d::compat::check(c, fm3d_knn2(c, A.data, A.rows, B.data, B.rows, A.cols, A.type, r.data()));
        out.assign(A.rows, std::vector<cv::DMatch>());
        for (int i = 0; i < A.rows; i++)
            for (int k = 0; k < 2; k++)
                if (r[2 * i + k].trainIdx >= 0) out[i].push_back(reinterpret_cast<const cv::DMatch&>(r[2 * i + k]));
    }
    fm3d_settings s_;
    cv::Mat image_a_, image_b_;
    bool binary_ = false;
};

// ---------------------------------------------------------------- SingleCameraTriangulator
class SingleCameraTriangulator {
public:
    explicit SingleCameraTriangulator(cv::FileStorage& settings)
        : s_(settings.settings()), dev_(fm3d::cvshim::device(s_)), sct_(dev_) {}
    // :116-121 (the images of the patch export)
    void setImages(const cv::Mat& img1, const cv::Mat& img2) { set_images(dev_, img1, img2); }
    // :123-143
    void setg12(const cv::Vec3d& T1, const cv::Vec3d& T2, const cv::Vec3d& rodrigues1, const cv::Vec3d& rodrigues2,
                cv::Matx44d& g12) {
        fm3d::compat::Matx44d g;
        sct_.setg12(v3(T1), v3(T2), v3(rodrigues1), v3(rodrigues2), g);
        for (int i = 0; i < 16; i++) g12.val[i] = g[i];
    }
    // :145-171
    void setKeypoints(const std::vector<cv::KeyPoint>& kpts1, const std::vector<cv::KeyPoint>& kpts2,
                      const std::vector<cv::DMatch>& matches) {
        std::vector<fm3d::compat::KeyPoint> k1(kpts1.size()), k2(kpts2.size());
        for (size_t i = 0; i < kpts1.size(); i++) k1[i].pt = fm3d::compat::Point2f{kpts1[i].pt.x, kpts1[i].pt.y};
        for (size_t i = 0; i < kpts2.size(); i++) k2[i].pt = fm3d::compat::Point2f{kpts2[i].pt.x, kpts2[i].pt.y};
        std::vector<fm3d_dmatch> m(matches.size());
        if (!m.empty()) std::memcpy(m.data(), matches.data(), m.size() * sizeof(fm3d_dmatch));
        sct_.setKeypoints(k1, k2, m);
    }
    // :173-230: triangulatedPoints cleared then filled; outliersMask APPENDED
    void triangulate(std::vector<cv::Vec3d>& triangulatedPoints, std::vector<bool>& outliersMask) {
        std::vector<fm3d::compat::Vec3d> p;
        sct_.triangulate(p, outliersMask);
        triangulatedPoints.clear();
        for (const auto& x : p) triangulatedPoints.push_back(cv::Vec3d(x[0], x[1], x[2]));
    }
    // :806-849: patchesVector / imagePointsVector cleared, then per frame a size x size CV_8UC1
    // patch and a (size*size) x 1 CV_64FC2 Mat of projected points
    void projectReferencePointsToImageWithFrames(const std::vector<cv::Vec3d>& referenceNeighborhood,
                                                 const std::vector<cv::Matx44d>& featureFrames,
                                                 std::vector<cv::Mat>& patchesVector,
                                                 std::vector<cv::Mat>& imagePointsVector) {
        std::vector<fm3d::compat::Vec3d> ref(referenceNeighborhood.size());
        for (size_t i = 0; i < ref.size(); i++) ref[i] = v3(referenceNeighborhood[i]);
        std::vector<fm3d::compat::Matx44d> ff(featureFrames.size());
        for (size_t i = 0; i < ff.size(); i++)
            for (int k = 0; k < 16; k++) ff[i][k] = featureFrames[i].val[k];
        std::vector<fm3d::compat::Patch8u> patches;
        std::vector<std::vector<double> > pts;
        sct_.projectReferencePointsToImageWithFrames(ref, ff, patches, pts);
        patchesVector.clear();
        imagePointsVector.clear();
        for (size_t f = 0; f < patches.size(); f++) {
            cv::Mat p(patches[f].rows, patches[f].cols, CV_8UC1);
            std::memcpy(p.data, patches[f].data.data(), patches[f].data.size());
            patchesVector.push_back(p);
            cv::Mat q((int)(pts[f].size() / 2), 1, CV_64FC2);
            std::memcpy(q.data, pts[f].data(), pts[f].size() * sizeof(double));
            imagePointsVector.push_back(q);
        }
    }
    fm3d::compat::Device& device() { return dev_; }
    static void set_images(fm3d::compat::Device& d, const cv::Mat& img1, const cv::Mat& img2) {
        if (img1.empty() || img2.empty() || img1.type() != CV_8UC1 || img2.type() != CV_8UC1 || img1.rows != img2.rows ||
            img1.cols != img2.cols)
            throw fm3d::compat::Error(FM3D_ERR_INVALID, "two gray images of the same size expected");
        fm3d::compat::check(d.ctx(), fm3d_set_images(d.ctx(), img1.data, img2.data, img1.cols, img1.rows, img1.cols));
    }

private:
    static fm3d::compat::Vec3d v3(const cv::Vec3d& v) { return fm3d::compat::Vec3d{v[0], v[1], v[2]}; }
    fm3d_settings s_;
    fm3d::compat::Device& dev_;
    fm3d::compat::SingleCameraTriangulator sct_;
};

// ---------------------------------------------------------------- NormalOptimizer
class NormalOptimizer {
public:
    NormalOptimizer(const cv::FileStorage settings, SingleCameraTriangulator* sct)
        : sct_(sct), no_(sct->device(), nullptr) {
        (void)settings;  // the same settings file the triangulator was built from
    }
    // :191-221
    void setImages(const cv::Mat& img1, const cv::Mat& img2) { SingleCameraTriangulator::set_images(sct_->device(), img1, img2); }
    // :294-452: failed points ERASED from points3D, one normal per kept point APPENDED
    void computeOptimizedNormals(std::vector<cv::Vec3d>& points3D, std::vector<cv::Vec3d>& normalsVector) {
        std::vector<fm3d::compat::Vec3d> p(points3D.size()), n;
        for (size_t i = 0; i < p.size(); i++) p[i] = fm3d::compat::Vec3d{points3D[i][0], points3D[i][1], points3D[i][2]};
        no_.computeOptimizedNormals(p, n);
        points3D.clear();
        for (const auto& x : p) points3D.push_back(cv::Vec3d(x[0], x[1], x[2]));
        for (const auto& x : n) normalsVector.push_back(cv::Vec3d(x[0], x[1], x[2]));
    }
    // colors feed the PCL viewer only (:372)
    void computeOptimizedNormals(std::vector<cv::Vec3d>& points3D, std::vector<cv::Vec3d>& normalsVector,
                                 std::vector<cv::Scalar>& /*colors*/) {
        computeOptimizedNormals(points3D, normalsVector);
    }
    // :454-504: one frame per (point, normal), APPENDED
    void computeFeaturesFrames(std::vector<cv::Vec3d>& points3D, std::vector<cv::Vec3d>& normalsVector,
                               std::vector<cv::Matx44d>& featuresFrames) {
        std::vector<fm3d::compat::Vec3d> p(points3D.size()), n(normalsVector.size());
        for (size_t i = 0; i < p.size(); i++) p[i] = fm3d::compat::Vec3d{points3D[i][0], points3D[i][1], points3D[i][2]};
        for (size_t i = 0; i < n.size(); i++)
            n[i] = fm3d::compat::Vec3d{normalsVector[i][0], normalsVector[i][1], normalsVector[i][2]};
        std::vector<fm3d::compat::Matx44d> f;
        no_.computeFeaturesFrames(p, n, f);
        for (const auto& x : f) {
            cv::Matx44d m;
            for (int k = 0; k < 16; k++) m.val[k] = x[k];
            featuresFrames.push_back(m);
        }
    }
    void startVisualizerThread() {}
    void stopVisualizerThread() {}
    // :185-188
    cv::Vec3d getGravity() {
        const fm3d::compat::Vec3d g = no_.getGravity();
        return cv::Vec3d(g[0], g[1], g[2]);
    }
    const std::vector<int32_t>& lastStatus() const { return no_.lastStatus(); }

private:
    SingleCameraTriangulator* sct_;
    fm3d::compat::NormalOptimizer no_;
};

// ---------------------------------------------------------------- NeighborhoodsGenerator
class NeighborhoodsGenerator {
public:
    explicit NeighborhoodsGenerator(cv::FileStorage settings) : s_(settings.settings()), ng_(s_) {}
    // neighborhoodsgenerator.cpp:134-158
    void getReferenceSquaredNeighborhood(std::vector<cv::Vec3d>& neighborhood) {
        std::vector<fm3d::compat::Vec3d> r;
        ng_.getReferenceSquaredNeighborhood(r);
        neighborhood.clear();
        for (const auto& x : r) neighborhood.push_back(cv::Vec3d(x[0], x[1], x[2]));
    }
    // neighborhoodsgenerator.cpp:76-132 (main.cpp:187)
    void computeSquareNeighborhoodsByNormals(const std::vector<cv::Matx44d>& featuresFrames,
                                             std::vector<std::vector<cv::Vec3d> >& neighborhoodsVector) {
        std::vector<fm3d::compat::Matx44d> ff(featuresFrames.size());
        for (size_t i = 0; i < ff.size(); i++)
            for (int k = 0; k < 16; k++) ff[i][k] = featuresFrames[i].val[k];
        std::vector<std::vector<fm3d::compat::Vec3d> > out;
        ng_.computeSquareNeighborhoodsByNormals(fm3d::cvshim::device(s_), ff, out);
        neighborhoodsVector.clear();
        for (const auto& nb : out) {
            std::vector<cv::Vec3d> v;
            v.reserve(nb.size());
            for (const auto& x : nb) v.push_back(cv::Vec3d(x[0], x[1], x[2]));
            neighborhoodsVector.push_back(v);
        }
    }

    // neighborhoodsgenerator.cpp:160-224: points / normals are 3 x N CV_64F Mats (column = point);
    // an empty normals Mat is filled with the initial guess; one 1 x (thetas*rays) CV_64FC3 Mat per
    // point is appended
    void computeCircularNeighborhoodsByNormals(const cv::Mat& points, cv::Mat& normals,
                                               std::vector<cv::Mat>& neighborhoodsVector) {
        const int n = points.cols;
        std::vector<fm3d::compat::Vec3d> P(n), N;
        for (int i = 0; i < n; i++)
            for (int k = 0; k < 3; k++) P[i][k] = points.at<double>(k, i);
        if (!normals.empty()) {
            N.resize(n);
            for (int i = 0; i < n; i++)
                for (int k = 0; k < 3; k++) N[i][k] = normals.at<double>(k, i);
        }
        std::vector<std::vector<fm3d::compat::Vec3d> > out;
        ng_.computeCircularNeighborhoodsByNormals(fm3d::cvshim::device(s_), P, N, out);
        if (normals.empty()) {
            normals = cv::Mat::zeros(cv::Size(n, 3), CV_64FC1);
            for (int i = 0; i < n; i++)
                for (int k = 0; k < 3; k++) normals.at<double>(k, i) = N[i][k];
        }
        for (const auto& nb : out) neighborhoodsVector.push_back(to_mat(nb));
    }
    // neighborhoodsgenerator.cpp:226-277
    void computeCircularNeighborhoodByNormal(const cv::Vec3d& point, cv::Vec3d& normal, cv::Mat& neighborhood) {
        fm3d::compat::Vec3d X{point[0], point[1], point[2]}, nn{normal[0], normal[1], normal[2]};
        std::vector<fm3d::compat::Vec3d> nb;
        ng_.computeCircularNeighborhoodByNormal(fm3d::cvshim::device(s_), X, nn, nb);
        normal = cv::Vec3d(nn[0], nn[1], nn[2]);
        neighborhood = to_mat(nb);
    }

private:
    static cv::Mat to_mat(const std::vector<fm3d::compat::Vec3d>& nb) {
        cv::Mat m = cv::Mat::zeros(cv::Size((int)nb.size(), 1), CV_64FC3);
        for (size_t s = 0; s < nb.size(); s++)
            for (int k = 0; k < 3; k++) reinterpret_cast<double*>(m.data)[3 * s + k] = nb[s][k];
        return m;
    }
    fm3d_settings s_;
    fm3d::compat::NeighborhoodsGenerator ng_;
};

// ---------------------------------------------------------------- MOSAIC (mosaic.h:47-70)
// The constructor runs mosaic.cpp:32-73's seven steps (on the GPU); the reference's computeImpl is
// empty, compute() describes the patches as main.cpp:182-183 does (extractDescriptorsFromPatches).
class MOSAIC {
public:
    MOSAIC(cv::FileStorage fs, cv::Mat& imgA, cv::Mat& imgB, const cv::Vec3d tA, const cv::Vec3d tB,
           const cv::Vec3d rA, const cv::Vec3d rB)
        : imgA_(imgA), imgB_(imgB), dm_(fs, imgA, imgB), sct_(fs), no_(fs, &sct_), ng_(fs) {
        cv::Mat desc1, desc2;
        dm_.compareWithNNDR(fs["NNDR"]["epsilon"], matches_, kptsA_, kptsB_, desc1, desc2);
        sct_.setg12(tA, tB, rA, rB, gAB_);
        std::vector<bool> outliersMask;
        sct_.setKeypoints(kptsA_, kptsB_, matches_);
        sct_.triangulate(triangulated_points_, outliersMask);
        no_.setImages(imgA_, imgB_);
        no_.computeOptimizedNormals(triangulated_points_, normals_vector_, colors_);
        no_.computeFeaturesFrames(triangulated_points_, normals_vector_, features_frames_);
        ng_.getReferenceSquaredNeighborhood(reference_neighborhood_);
        sct_.setImages(imgA_, imgB_);
        sct_.projectReferencePointsToImageWithFrames(reference_neighborhood_, features_frames_, patches_vector_,
                                                     image_points_vector_);
    }
    int descriptorType() { return CV_32F; }
    int descriptorSize() { return 128; }
    // one descriptor row per kept feature (the patches' SURF descriptors)
    void compute(cv::Mat& descriptors) {
        if (patches_vector_.empty()) {
            descriptors = cv::Mat();
            return;
        }
        dm_.extractDescriptorsFromPatches(patches_vector_, descriptors);
    }
    const std::vector<cv::DMatch>& matches() const { return matches_; }
    const std::vector<cv::Vec3d>& points() const { return triangulated_points_; }
    const std::vector<cv::Vec3d>& normals() const { return normals_vector_; }
    const std::vector<cv::Mat>& patches() const { return patches_vector_; }

private:
    cv::Mat imgA_, imgB_;
    DescriptorsMatcher dm_;
    std::vector<cv::KeyPoint> kptsA_, kptsB_;
    std::vector<cv::DMatch> matches_;
    std::vector<cv::Vec3d> triangulated_points_;
    SingleCameraTriangulator sct_;
    cv::Matx44d gAB_;
    std::vector<cv::Mat> patches_vector_, image_points_vector_;
    NormalOptimizer no_;
    std::vector<cv::Vec3d> normals_vector_;
    std::vector<cv::Matx44d> features_frames_;
    NeighborhoodsGenerator ng_;
    std::vector<cv::Vec3d> reference_neighborhood_;
    std::vector<cv::Scalar> colors_;
};

// ---------------------------------------------------------------- tools.cpp drawing (visual only)
// drawMatches (tools.cpp:146-191): side-by-side BGR window, per inlier match a circle at both
// keypoints and a line between them; one color per drawn match is APPENDED to colors
inline void drawMatches(const cv::Mat& img1, const cv::Mat& img2, cv::Mat& window, const std::vector<cv::KeyPoint>& kpts1,
                        const std::vector<cv::KeyPoint>& kpts2, const std::vector<cv::DMatch>& matches,
                        std::vector<cv::Scalar>& colors, const std::vector<bool> outliersMask) {
    window = cv::Mat(cv::Size(img1.cols * 2, img1.rows), CV_8UC3);
    for (int r = 0; r < img1.rows; r++)
        for (int c = 0; c < img1.cols; c++)
            for (int k = 0; k < 3; k++) {
                window.at<cv::uchar>(r, 3 * c + k) = img1.at<cv::uchar>(r, c);
                if (r < img2.rows && c < img2.cols) window.at<cv::uchar>(r, 3 * (c + img1.cols) + k) = img2.at<cv::uchar>(r, c);
            }
    auto put = [&](int x, int y, const cv::Scalar& col) {
        if (x < 0 || y < 0 || x >= window.cols || y >= window.rows) return;
        for (int k = 0; k < 3; k++) window.at<cv::uchar>(y, 3 * x + k) = (cv::uchar)col[k];
    };
    auto line = [&](double x0, double y0, double x1, double y1, const cv::Scalar& col) {
        const int n = (int)std::ceil(std::max(std::fabs(x1 - x0), std::fabs(y1 - y0))) + 1;
        for (int i = 0; i <= n; i++) put((int)std::lround(x0 + (x1 - x0) * i / n), (int)std::lround(y0 + (y1 - y0) * i / n), col);
    };
    auto circle = [&](double x, double y, const cv::Scalar& col) {
        for (int a = 0; a < 64; a++) put((int)std::lround(x + 4 * std::cos(a * M_PI / 32)), (int)std::lround(y + 4 * std::sin(a * M_PI / 32)), col);
    };
    // cv::RNG rng(0xFFF0FF0F) and random_color (tools.cpp:116-120, 159-167): the same colour sequence
    // as the reference, so results/*/image{1,2}pixels.pgm and projectedPatches.pgm colours line up
    cv::RNG rng(0xFFF0FF0FULL);
    for (size_t i = 0; i < matches.size() && i < outliersMask.size(); i++) {
        if (!outliersMask[i]) continue;
        const cv::Scalar col = cv::random_color(rng);
        colors.push_back(col);
        const cv::Point2f p1 = kpts1.at(matches[i].queryIdx).pt, p2 = kpts2.at(matches[i].trainIdx).pt;
        circle(p1.x, p1.y, col);
        circle(p2.x + img1.cols, p2.y, col);
        line(p1.x, p1.y, p2.x + img1.cols, p2.y, col);
    }
}

// drawBackProjectedPoints (tools.cpp:193-221): the gray image as BGR, each patch's projected points
// painted in its color (pixels inside the image)
inline void drawBackProjectedPoints(const cv::Mat& input, cv::Mat& output, const std::vector<cv::Mat>& points,
                                    const std::vector<cv::Scalar>& colors) {
    output = cv::Mat(cv::Size(input.cols, input.rows), CV_8UC3);
    for (size_t i = 0; i < input.total(); i++)
        for (int k = 0; k < 3; k++) output.data[3 * i + k] = input.data[i];
    for (size_t i = 0; i < points.size() && i < colors.size(); i++)
        for (int k = 0; k < points[i].rows; k++) {
            const cv::Vec2d p = points[i].at<cv::Vec2d>(k);
            const int x = (int)std::lround(p[0]), y = (int)std::lround(p[1]);
            if (x < 0 || y < 0 || x >= output.cols || y >= output.rows) continue;
            for (int ch = 0; ch < 3; ch++) output.at<cv::uchar>(y, 3 * x + ch) = (cv::uchar)colors[i][ch];
        }
}

// ---------------------------------------------------------------- PCL stand-ins (visual only)
// main.cpp:199-217 collects the normals into a pcl::PointCloud<pcl::Normal> and opens a PCL viewer
// (tools.h:79-91).  The viewer is out of scope: the cloud types hold the data, the
// view* functions return at once.
namespace pcl {
struct Normal {  // pcl::Normal's fields (PCL 1.x point_types.h)
    float normal_x = 0, normal_y = 0, normal_z = 0, curvature = 0;
    Normal() {}
    Normal(float nx, float ny, float nz, float c = 0) : normal_x(nx), normal_y(ny), normal_z(nz), curvature(c) {}
};
template <class PointT>
class PointCloud {
public:
    typedef std::shared_ptr<PointCloud<PointT> > Ptr;
    typedef std::shared_ptr<const PointCloud<PointT> > ConstPtr;
    std::vector<PointT> points;
    uint32_t width = 0, height = 1;
    bool is_dense = true;
    size_t size() const { return points.size(); }
    bool empty() const { return points.empty(); }
    void push_back(const PointT& p) {
        points.push_back(p);
        width = (uint32_t)points.size();
        height = 1;
    }
};
}  // namespace pcl

// tools.h:79-91: the PCL viewers (blocking windows in the reference), no-ops here
inline void viewPointCloud(const cv::Mat&, const std::vector<cv::Scalar>&) {}
inline void viewPointCloud(const std::vector<cv::Vec3d>&) {}
inline void viewPointCloud(const std::vector<cv::Vec3d>&, const cv::Vec3d&) {}
inline void viewPointCloudAndNormals(const std::vector<cv::Vec3d>&, pcl::PointCloud<pcl::Normal>::ConstPtr,
                                     const std::vector<cv::Scalar>&) {}
inline void viewPointCloudNormalsAndFrames(const std::vector<cv::Vec3d>&, pcl::PointCloud<pcl::Normal>::ConstPtr,
                                           const std::vector<cv::Scalar>&, std::vector<cv::Matx44d>&) {}
inline void viewPointCloudNeighborhood(const cv::Mat&, std::vector<cv::Mat>&, const std::vector<cv::Scalar>&) {}
inline void viewPointCloudNormalsFramesAndNeighborhood(const std::vector<std::vector<cv::Vec3d> >&,
                                                       std::vector<cv::Vec3d>&, const std::vector<cv::Scalar>&,
                                                       std::vector<cv::Matx44d>&) {}
inline void viewPointCloudNormalsFramesNeighborhoodAndGravity(const std::vector<std::vector<cv::Vec3d> >&,
                                                              std::vector<cv::Vec3d>&, const std::vector<cv::Scalar>&,
                                                              std::vector<cv::Matx44d>&, cv::Vec3d&) {}

#endif  // FM3D_CV_HPP
