/*
 * fm3d_compat.hpp -- header-only C++ shim that re-exposes the reference's class
 * interface for the hot path on top of the C ABI (fm3d.h).
 *
 * The reference calls its three classes from main.cpp:91-155:
 *   DescriptorsMatcher        DescriptorsMatcher/descriptorsmatcher.h:39-111
 *   SingleCameraTriangulator  Triangulator/singlecameratriangulator.h:52-93
 *   NormalOptimizer           Triangulator/normaloptimizer.h:43-59
 * The classes below keep those names, method names, argument order, argument meaning
 * and out-parameter semantics (appended matches, erased points, appended normals).
 * Two deliberate differences, both outside the hot path:
 *   - compareWithNNDR takes the descriptor matrices: feature detection/description
 *     (descriptorsmatcher.cpp:110-115) is upstream and out of scope;
 *   - the OpenCV value types are replaced by the small PODs below (Mat8u, DescMat,
 *     KeyPoint, DMatch, Vec3d, Matx44d) with the same fields the path reads, and
 *     cv::FileStorage by the settings.yml reader fm3d_settings_load.
 * Errors: every ABI failure throws fm3d::compat::Error (the reference exit()s).
 */
#ifndef FM3D_COMPAT_HPP
#define FM3D_COMPAT_HPP

#include <array>
#include <cmath>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <cstdlib>
#include <cstdio>
#include <vector>

#include "fm3d.h"

namespace fm3d {
namespace compat {

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& what) : std::runtime_error(what), code(c) {}
};

struct Point2f {
    float x, y;
};
struct KeyPoint {  // cv::KeyPoint: the path reads .pt only (singlecameratriangulator.cpp:152-164)
    Point2f pt;
    float size, angle, response;
    int octave, class_id;
};
typedef fm3d_dmatch DMatch;  // cv::DMatch field layout: queryIdx, trainIdx, imgIdx, distance
typedef std::array<double, 3> Vec3d;
typedef std::array<double, 16> Matx44d;  // row major

struct Mat8u {  // CV_8UC1 image (rows x cols, row stride `step` bytes)
    int rows, cols;
    const uint8_t* data;
    int step;
};
struct Patch8u {  // an owned CV_8UC1 patch (rows x cols, continuous)
    int rows = 0, cols = 0;
    std::vector<uint8_t> data;
};
struct DescMat {  // descriptor matrix: CV_32F rows, CV_8U rows, or binary strings
    int rows, cols;
    fm3d_desc_type type;  // FM3D_DESC_F32 / FM3D_DESC_U8 / FM3D_DESC_BITS (cols = bytes)
    const void* data;
};

inline void check(fm3d_ctx* ctx, int rc) {
    if (rc != FM3D_OK) throw Error(rc, ctx ? fm3d_last_error(ctx) : "fm3d error");
}

// Owns the device context (settings + one HIP stream on one GPU).
class Device {
public:
    explicit Device(const fm3d_settings& s, int device = 0) : settings_(s) {
        check(nullptr, fm3d_ctx_create(&s, device, &ctx_));
    }
    // cv::FileStorage fs(path) stand-in: the %YAML:1.0 subset build/settings.yml uses
    static fm3d_settings load_settings(const std::string& path) {
        fm3d_settings s;
        check(nullptr, fm3d_settings_load(path.c_str(), &s));
        return s;
    }
    ~Device() { fm3d_ctx_destroy(ctx_); }
    Device(const Device&) = delete;
    Device& operator=(const Device&) = delete;
    fm3d_ctx* ctx() const { return ctx_; }
    const fm3d_settings& settings() const { return settings_; }

private:
    fm3d_ctx* ctx_ = nullptr;
    fm3d_settings settings_;
};

// NeighborhoodsGenerator (neighborhoodsgenerator.h:78-97), the square and the circular methods
class NeighborhoodsGenerator {
public:
    // neighborhoodsgenerator.cpp:36-74: an unsupported Neighborhoods.method ends the program with -10
    explicit NeighborhoodsGenerator(const fm3d_settings& s) : s_(s) {
        if (s_.neighMethod != 0 && s_.neighMethod != 1) {
            std::fprintf(stderr, "Unsupported method for plane neighborhood extraction\n");
            std::exit(-10);
        }
    }
    // computeCircularNeighborhoodsByNormals (neighborhoodsgenerator.cpp:160-224): per point
    // thetas*rays samples (ray outer, angle inner) on d's GPU; empty normals are filled with the
    // initial guess X/|X| as the reference does (its normals Mat is an in/out parameter)
    void computeCircularNeighborhoodsByNormals(Device& d, const std::vector<Vec3d>& points, std::vector<Vec3d>& normals,
                                               std::vector<std::vector<Vec3d> >& neighborhoodsVector) const {
        const size_t S = (size_t)s_.neighThetas * s_.neighRays;
        if (normals.empty())
            for (const Vec3d& X : points) {
                double q = 0;
                for (int i = 0; i < 3; i++) q += X[i] * X[i];
                const double inv = 1. / std::sqrt(q);
                normals.push_back(Vec3d{X[0] * inv, X[1] * inv, X[2] * inv});
            }
        std::vector<Vec3d> all(points.size() * S);
        if (!points.empty())
            check(d.ctx(), fm3d_circular_neighborhoods(d.ctx(), points.data()->data(), normals.data()->data(),
                                                       (int)points.size(), all.data()->data()));
        for (size_t p = 0; p < points.size(); p++)  // appended, as the reference push_backs
            neighborhoodsVector.emplace_back(all.begin() + p * S, all.begin() + (p + 1) * S);
    }
    // computeCircularNeighborhoodByNormal (neighborhoodsgenerator.cpp:226-277): a zero normal is
    // replaced by X/|X| (in/out), then the samples of that one point
    void computeCircularNeighborhoodByNormal(Device& d, const Vec3d& point, Vec3d& normal,
                                             std::vector<Vec3d>& neighborhood) const {
        std::vector<Vec3d> pts{point}, nrm;
        if (!(normal[0] == 0 && normal[1] == 0 && normal[2] == 0)) nrm.push_back(normal);
        std::vector<std::vector<Vec3d> > out;
        computeCircularNeighborhoodsByNormals(d, pts, nrm, out);
        normal = nrm[0];
        neighborhood = out[0];
    }
    // getReferenceSquaredNeighborhood (neighborhoodsgenerator.cpp:134-158): cleared, then size^2
    // points (-epsilon + inc*i, -epsilon + inc*j, 0), i outer
    void getReferenceSquaredNeighborhood(std::vector<Vec3d>& neighborhood) const {
        const int n = fm3d_patch_size(&s_);
        const double inc = s_.cmPerPixel * 0.01;
        neighborhood.clear();
        for (int i = 0; i < n; i++)
            for (int j = 0; j < n; j++) neighborhood.push_back(Vec3d{-s_.neighEpsilon + inc * i, -s_.neighEpsilon + inc * j, 0});
    }
    // computeSquareNeighborhoodsByNormals (neighborhoodsgenerator.cpp:76-132, main.cpp:187): cleared,
    // then per frame the size^2 grid points moved by the frame, computed on d's GPU
    void computeSquareNeighborhoodsByNormals(Device& d, const std::vector<Matx44d>& featuresFrames,
                                             std::vector<std::vector<Vec3d> >& neighborhoodsVector) const {
        const size_t per = (size_t)fm3d_patch_size(&s_) * fm3d_patch_size(&s_);
        std::vector<Vec3d> all(featuresFrames.size() * per);
        neighborhoodsVector.clear();
        if (featuresFrames.empty()) return;
        check(d.ctx(), fm3d_square_neighborhoods(d.ctx(), featuresFrames.data()->data(), (int)featuresFrames.size(),
                                                 all.data()->data()));
        for (size_t f = 0; f < featuresFrames.size(); f++)
            neighborhoodsVector.emplace_back(all.begin() + f * per, all.begin() + (f + 1) * per);
    }

private:
    fm3d_settings s_;
};

// DescriptorsMatcher (descriptorsmatcher.h:39-111)
class DescriptorsMatcher {
public:
    explicit DescriptorsMatcher(Device& d) : d_(d) {}
    // knnMatch(k=2) of compare (descriptorsmatcher.cpp:89-105): nA x 2 neighbours
    void knnMatch(const DescMat& A, const DescMat& B, std::vector<std::array<DMatch, 2> >& out) {
        require_same(A, B);
        out.resize(A.rows);
        check(d_.ctx(), fm3d_knn2(d_.ctx(), A.data, A.rows, B.data, B.rows, A.cols, A.type,
                                  reinterpret_cast<fm3d_dmatch*>(out.data())));
    }
    // compareWithNNDR (descriptorsmatcher.cpp:107-131): matches are APPENDED, in query order
    void compareWithNNDR(double epsilon, std::vector<DMatch>& matches, const DescMat& A, const DescMat& B) {
        require_same(A, B);
        std::vector<DMatch> tmp(A.rows > 0 ? A.rows : 1);
        int n = 0;
        check(d_.ctx(), fm3d_match_nndr(d_.ctx(), A.data, A.rows, B.data, B.rows, A.cols, A.type, epsilon,
                                        tmp.data(), &n));
        matches.insert(matches.end(), tmp.begin(), tmp.begin() + n);
    }

private:
    static void require_same(const DescMat& A, const DescMat& B) {
        if (A.cols != B.cols || A.type != B.type) throw Error(FM3D_ERR_INVALID, "descriptor matrices differ");
    }
    Device& d_;
};

// SingleCameraTriangulator (singlecameratriangulator.h:52-93), hot-path methods
class SingleCameraTriangulator {
public:
    explicit SingleCameraTriangulator(Device& d) : d_(d) {}
    // setg12 (:123-143): g12 = gIC^-1 g2^-1 g1 gIC, also installed for triangulation
    void setg12(const Vec3d& T1, const Vec3d& T2, const Vec3d& r1, const Vec3d& r2, Matx44d& g12) {
        check(d_.ctx(), fm3d_setg12(d_.ctx(), T1.data(), T2.data(), r1.data(), r2.data(), g12.data()));
    }
    void setg12(const Matx44d& g12) { check(d_.ctx(), fm3d_set_g12(d_.ctx(), g12.data())); }
    // projectReferencePointsToImageWithFrames (:769-849) on image 1 of NormalOptimizer::setImages:
    // patchesVector / imagePointsVector are cleared, then one size x size patch (and its 2*size*size
    // projected coordinates) per frame; patch row j, column i = reference point (i, j)
    void projectReferencePointsToImageWithFrames(const std::vector<Vec3d>& referenceNeighborhood,
                                                 const std::vector<Matx44d>& featuresFrames,
                                                 std::vector<Patch8u>& patchesVector,
                                                 std::vector<std::vector<double> >& imagePointsVector) {
        patchesVector.clear();
        imagePointsVector.clear();
        const int P = (int)featuresFrames.size();
        const int size = fm3d_patch_size(&d_.settings());  // the square neighbourhood the ABI rebuilds
        if ((size_t)size * size != referenceNeighborhood.size())
            throw Error(FM3D_ERR_INVALID, "reference neighbourhood is not the square one of the settings");
        if (P == 0 || size == 0) return;
        std::vector<uint8_t> patches((size_t)P * size * size);
        std::vector<double> pts((size_t)P * size * size * 2);
        check(d_.ctx(), fm3d_export_patches(d_.ctx(), featuresFrames.data()->data(), P, patches.data(), pts.data()));
        for (int p = 0; p < P; p++) {
            Patch8u m;
            m.rows = m.cols = size;
            m.data.assign(patches.begin() + (size_t)p * size * size, patches.begin() + (size_t)(p + 1) * size * size);
            patchesVector.push_back(m);
            imagePointsVector.push_back(std::vector<double>(pts.begin() + (size_t)p * size * size * 2,
                                                            pts.begin() + (size_t)(p + 1) * size * size * 2));
        }
    }
    // setKeypoints (:145-171)
    void setKeypoints(const std::vector<KeyPoint>& k1, const std::vector<KeyPoint>& k2,
                      const std::vector<DMatch>& matches) {
        kp1_.resize(k1.size());
        kp2_.resize(k2.size());
        for (size_t i = 0; i < k1.size(); i++) kp1_[i] = fm3d_point2f{k1[i].pt.x, k1[i].pt.y};
        for (size_t i = 0; i < k2.size(); i++) kp2_[i] = fm3d_point2f{k2[i].pt.x, k2[i].pt.y};
        matches_ = matches;
    }
    // triangulate (:173-230): points3D is cleared then filled (inliers, match order);
    // outliersMask is APPENDED (one flag per match, true = kept), as in the reference
    void triangulate(std::vector<Vec3d>& points3D, std::vector<bool>& outliersMask) {
        const int K = (int)matches_.size();
        std::vector<double> pts((size_t)3 * (K > 0 ? K : 1));
        std::vector<uint8_t> mask(K > 0 ? K : 1);
        int n = 0;
        check(d_.ctx(), fm3d_triangulate(d_.ctx(), kp1_.data(), (int)kp1_.size(), kp2_.data(), (int)kp2_.size(),
                                         matches_.data(), K, pts.data(), mask.data(), &n));
        points3D.clear();
        for (int i = 0; i < n; i++) points3D.push_back(Vec3d{pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]});
        for (int i = 0; i < K; i++) outliersMask.push_back(mask[i] != 0);
    }
    Device& device() const { return d_; }

private:
    Device& d_;
    std::vector<fm3d_point2f> kp1_, kp2_;
    std::vector<DMatch> matches_;
};

// NormalOptimizer (normaloptimizer.h:43-59), hot-path methods
class NormalOptimizer {
public:
    NormalOptimizer(Device& d, SingleCameraTriangulator* sct) : d_(d), sct_(sct), settings_(d.settings()) {}
    // setImages (normaloptimizer.cpp:191-221): both gray images, builds the pyramids
    void setImages(const Mat8u& img1, const Mat8u& img2) {
        if (img1.rows != img2.rows || img1.cols != img2.cols || img1.step != img2.step)
            throw Error(FM3D_ERR_INVALID, "images differ in size");
        check(d_.ctx(), fm3d_set_images(d_.ctx(), img1.data, img2.data, img1.cols, img1.rows, img1.step));
    }
    // computeOptimizedNormals (:321-452): failed points are ERASED from points3D (order
    // kept); one normal per kept point is APPENDED to normalsVector
    void computeOptimizedNormals(std::vector<Vec3d>& points3D, std::vector<Vec3d>& normalsVector) {
        const int P = (int)points3D.size();
        std::vector<double> pts((size_t)3 * (P > 0 ? P : 1)), nrm((size_t)3 * (P > 0 ? P : 1));
        for (int i = 0; i < P; i++)
            for (int k = 0; k < 3; k++) pts[3 * i + k] = points3D[i][k];
        status_.assign(P > 0 ? P : 1, 0);
        int kept = 0;
        check(d_.ctx(), fm3d_optimize_normals(d_.ctx(), pts.data(), P, nrm.data(), status_.data(), nullptr, nullptr,
                                              &kept, &stats_));
        status_.resize(P);
        points3D.resize(kept);
        for (int i = 0; i < kept; i++) {
            points3D[i] = Vec3d{pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]};
            normalsVector.push_back(Vec3d{nrm[3 * i], nrm[3 * i + 1], nrm[3 * i + 2]});
        }
    }
    // getGravity (normaloptimizer.cpp:185-188)
    Vec3d getGravity() const {
        fm3d_settings s;
        settings(s);
        Vec3d g;
        check(d_.ctx(), fm3d_gravity(&s, g.data()));
        return g;
    }
    // computeFeaturesFrames (normaloptimizer.cpp:454-504): one frame per (point, normal), APPENDED
    void computeFeaturesFrames(const std::vector<Vec3d>& points3D, const std::vector<Vec3d>& normalsVector,
                               std::vector<Matx44d>& featuresFrames) {
        const size_t n = points3D.size() < normalsVector.size() ? points3D.size() : normalsVector.size();
        if (n == 0) return;
        std::vector<Matx44d> f(n);
        check(d_.ctx(), fm3d_features_frames(d_.ctx(), points3D.data()->data(), normalsVector.data()->data(), (int)n,
                                             f.data()->data()));
        featuresFrames.insert(featuresFrames.end(), f.begin(), f.end());
    }
    // the PCL viewer thread (pclvisualizerthread.cpp) is visual only: no-ops
    void startVisualizerThread() {}
    void stopVisualizerThread() {}
    // per input point outcome of the last call (FM3D_ST_*) and its counters
    const std::vector<int32_t>& lastStatus() const { return status_; }
    const fm3d_lm_stats& lastStats() const { return stats_; }

private:
    void settings(fm3d_settings& s) const { s = settings_; }
    Device& d_;
    SingleCameraTriangulator* sct_;
    fm3d_settings settings_;
    std::vector<int32_t> status_;
    fm3d_lm_stats stats_{};
};

}  // namespace compat
}  // namespace fm3d

#endif  // FM3D_COMPAT_HPP
