// fm3d_main.cpp -- the hot-path part of the reference's main.cpp:91-155, written
// against the compat shim (include/fm3d_compat.hpp): settings.yml -> match + NNDR ->
// setg12/setKeypoints/triangulate -> setImages -> computeOptimizedNormals.
//
// Detection/description is upstream (out of scope), so keypoints and descriptors
// come from side files next to the images:
//   <dir>/img1.pgm img2.pgm   8-bit P5 images
//   <dir>/kp1.f32 kp2.f32     N x 2 float32 keypoint positions
//   <dir>/desc1.u8 desc2.u8   N x 128 uint8 descriptors (SIFT saturated to uchar)
// Writes <dir>/out_matches.bin (DMatch), out_points.f64, out_normals.f64 and, like main.cpp:160-180,
// the normal-rectified patches of the first 16 points as patch_<i>.pgm.
// Usage: fm3d_main -s settings.yml -d <dir>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "fm3d_compat.hpp"

using namespace fm3d::compat;

static std::vector<char> slurp(const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw Error(FM3D_ERR_INVALID, "cannot open " + path);
    return std::vector<char>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

// P5 (binary 8-bit gray) PGM reader: header tokens with '#' comments, maxval <= 255
static std::vector<uint8_t> read_pgm(const std::string& path, int& w, int& h) {
    std::vector<char> b = slurp(path);
    size_t i = 0;
    auto token = [&]() {
        std::string t;
        while (i < b.size()) {
            if (b[i] == '#') {
                while (i < b.size() && b[i] != '\n') i++;
            } else if (isspace((unsigned char)b[i])) {
                if (!t.empty()) break;
                i++;
            } else {
                t += b[i++];
            }
        }
        return t;
    };
    if (token() != "P5") throw Error(FM3D_ERR_INVALID, path + ": not a P5 PGM");
    w = std::stoi(token());
    h = std::stoi(token());
    int maxval = std::stoi(token());
    i++;  // single whitespace after maxval
    if (maxval > 255 || b.size() < i + (size_t)w * h) throw Error(FM3D_ERR_INVALID, path + ": bad PGM");
    return std::vector<uint8_t>(b.begin() + i, b.begin() + i + (size_t)w * h);
}

template <class T>
static std::vector<T> read_raw(const std::string& path) {
    std::vector<char> b = slurp(path);
    std::vector<T> v(b.size() / sizeof(T));
    std::memcpy(v.data(), b.data(), v.size() * sizeof(T));
    return v;
}

// P5 writer (cv::imwrite of the patches, singlecameratriangulator.cpp:799-802)
static void write_pgm(const std::string& path, const Patch8u& m) {
    std::ofstream f(path, std::ios::binary);
    f << "P5\n" << m.cols << " " << m.rows << "\n255\n";
    f.write(reinterpret_cast<const char*>(m.data.data()), (std::streamsize)m.data.size());
}

template <class T>
static void write_raw(const std::string& path, const T* p, size_t n) {
    std::ofstream f(path, std::ios::binary);
    f.write(reinterpret_cast<const char*>(p), n * sizeof(T));
}

int main(int argc, char** argv) {
    std::string settingsPath, dir;
    for (int a = 1; a + 1 < argc; a += 2) {
        if (!strcmp(argv[a], "-s")) settingsPath = argv[a + 1];
        if (!strcmp(argv[a], "-d")) dir = argv[a + 1];
    }
    if (settingsPath.empty() || dir.empty()) {
        std::cerr << "usage: fm3d_main -s settings.yml -d <dir>\n";
        return -1;  // main.cpp:48
    }
    try {
        fm3d_settings s = Device::load_settings(settingsPath);  // main.cpp:62-71
        Device dev(s, 0);
        int w = 0, h = 0, w2 = 0, h2 = 0;
        std::vector<uint8_t> img1 = read_pgm(dir + "/img1.pgm", w, h);  // main.cpp:79-81
        std::vector<uint8_t> img2 = read_pgm(dir + "/img2.pgm", w2, h2);
        std::vector<float> kp1f = read_raw<float>(dir + "/kp1.f32"), kp2f = read_raw<float>(dir + "/kp2.f32");
        std::vector<uint8_t> d1 = read_raw<uint8_t>(dir + "/desc1.u8"), d2 = read_raw<uint8_t>(dir + "/desc2.u8");
        std::vector<KeyPoint> k1(kp1f.size() / 2), k2(kp2f.size() / 2);
        for (size_t i = 0; i < k1.size(); i++) k1[i].pt = Point2f{kp1f[2 * i], kp1f[2 * i + 1]};
        for (size_t i = 0; i < k2.size(); i++) k2[i].pt = Point2f{kp2f[2 * i], kp2f[2 * i + 1]};

        DescriptorsMatcher dm(dev);  // main.cpp:91-92
        std::vector<DMatch> matches;
        DescMat A{(int)k1.size(), 128, FM3D_DESC_U8, d1.data()}, B{(int)k2.size(), 128, FM3D_DESC_U8, d2.data()};
        dm.compareWithNNDR(s.nndrEpsilon, matches, A, B);  // main.cpp:94

        SingleCameraTriangulator sct(dev);  // main.cpp:126-131
        Matx44d g12;
        Vec3d T1{s.pos1[0], s.pos1[1], s.pos1[2]}, r1{s.pos1[3], s.pos1[4], s.pos1[5]};
        Vec3d T2{s.pos2[0], s.pos2[1], s.pos2[2]}, r2{s.pos2[3], s.pos2[4], s.pos2[5]};
        sct.setg12(T1, T2, r1, r2, g12);
        sct.setKeypoints(k1, k2, matches);
        std::vector<Vec3d> points3D;
        std::vector<bool> outliersMask;
        sct.triangulate(points3D, outliersMask);

        NormalOptimizer no(dev, &sct);  // main.cpp:146-155
        no.setImages(Mat8u{h, w, img1.data(), w}, Mat8u{h2, w2, img2.data(), w2});
        no.startVisualizerThread();
        std::vector<Vec3d> normals;
        no.computeOptimizedNormals(points3D, normals);
        no.stopVisualizerThread();

        // main.cpp:157-180: feature frames, reference neighbourhood, normal-rectified patches
        std::vector<Matx44d> featuresFrames;
        no.computeFeaturesFrames(points3D, normals, featuresFrames);
        NeighborhoodsGenerator ng(s);
        std::vector<Vec3d> referenceNeighborhood;
        ng.getReferenceSquaredNeighborhood(referenceNeighborhood);
        std::vector<Patch8u> patchesVector;
        std::vector<std::vector<double> > imagePointsVector;
        sct.projectReferencePointsToImageWithFrames(referenceNeighborhood, featuresFrames, patchesVector,
                                                    imagePointsVector);
        for (size_t i = 0; i < patchesVector.size() && i < 16; i++)
            write_pgm(dir + "/patch_" + std::to_string(i) + ".pgm", patchesVector[i]);

        write_raw(dir + "/out_matches.bin", matches.data(), matches.size());
        write_raw(dir + "/out_points.f64", points3D.data()->data(), points3D.size() * 3);
        write_raw(dir + "/out_normals.f64", normals.data()->data(), normals.size() * 3);
        std::cout << matches.size() << " matches, " << outliersMask.size() << " triangulated ("
                  << points3D.size() << " kept after normal optimisation)\n";
    } catch (const Error& e) {
        std::cerr << "fm3d error " << e.code << ": " << e.what() << "\n";
        return e.code;
    }
    return 0;
}
