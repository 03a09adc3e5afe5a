// main_dropin.cpp -- the reference's main() call sequence (main.cpp:36-194) written against
// include/fm3d_cv.hpp, to show that main.cpp compiles with only its include lines changed:
//
//   main.cpp:8-20  (#include <lmmin.h>, <opencv2/...>, the project headers)
//     ->  #include "fm3d_cv.hpp"
//
// Everything below the includes uses the reference's own types and calls (cv::FileStorage,
// cv::imread, DescriptorsMatcher(fs, img1, img2).compareWithNNDR(...), SingleCameraTriangulator(fs),
// NormalOptimizer(fs, &sct), NeighborhoodsGenerator(fs), drawMatches, ...).  The PCL viewers are
// left out (visual only).  With the reference's SURF detector / extractor the features are detected
// and described on the GPU; with another detector type (no GPU implementation) the keypoints /
// descriptors come from the images' side files <image>.kpts.f32 / <image>.desc.u8.
//
// Usage: main_dropin -s settings.yml    (the reference's command line)
// Writes matches.pgm, patch_<i>.pgm (via the patch export), projectedPatches.pgm like the
// reference, plus out_matches.bin / out_points.f64 / out_normals.f64 for the tests.
#include <fstream>
#include <iomanip>
#include <iostream>
#include <vector>

#include "fm3d_cv.hpp"

static void dump(const std::string& path, const void* p, size_t bytes) {
    std::ofstream f(path, std::ios::binary);
    f.write(static_cast<const char*>(p), (std::streamsize)bytes);
}

int main(int argc, char** argv) {
    std::cout << std::fixed << std::setprecision(12);
    if (argc != 3 || std::string(argv[1]) != "-s") {
        std::cout << "Usage: main_dropin -s <settings.yml>" << std::endl;
        return -1;  // main.cpp:46-56 exit(-1)
    }
    try {
        cv::FileStorage fs;
        fs.open(argv[2], cv::FileStorage::READ);
        if (!fs.isOpened()) {
            std::cerr << "Could not open settings file: " << argv[2] << std::endl;
            return -1;
        }
        std::string IMG_1, IMG_2;
        fs["IMAGES"]["img1"] >> IMG_1;
        fs["IMAGES"]["img2"] >> IMG_2;
        cv::Mat img1 = cv::imread(IMG_1, CV_LOAD_IMAGE_GRAYSCALE), img2 = cv::imread(IMG_2, CV_LOAD_IMAGE_GRAYSCALE);
        if (img1.empty() || img2.empty()) {
            std::cerr << "Could not read the images" << std::endl;
            return -1;
        }

        // feature match (main.cpp:85-94)
        std::vector<cv::KeyPoint> kpts1, kpts2;
        cv::Mat desc1, desc2;
        std::vector<cv::DMatch> matches;
        DescriptorsMatcher dm(fs, img1, img2);
        dm.compareWithNNDR(fs["NNDR"]["epsilon"], matches, kpts1, kpts2, desc1, desc2);

        // poses, g12, triangulation (main.cpp:96-131)
        std::vector<double> pos1, pos2;
        fs["IMAGES"]["pos1"] >> pos1;
        fs["IMAGES"]["pos2"] >> pos2;
        cv::Vec3d translation1(pos1[0], pos1[1], pos1[2]), translation2(pos2[0], pos2[1], pos2[2]);
        cv::Vec3d rodrigues1(pos1[3], pos1[4], pos1[5]), rodrigues2(pos2[3], pos2[4], pos2[5]);
        cv::Matx44d g12;
        std::vector<cv::Vec3d> triagulated;
        std::vector<bool> outliersMask;
        SingleCameraTriangulator sct(fs);
        sct.setKeypoints(kpts1, kpts2, matches);
        sct.setg12(translation1, translation2, rodrigues1, rodrigues2, g12);
        sct.triangulate(triagulated, outliersMask);

        // matches.pgm (main.cpp:135-141)
        cv::Mat window;
        std::vector<cv::Scalar> colors;
        drawMatches(img1, img2, window, kpts1, kpts2, matches, colors, outliersMask);
        cv::imwrite("matches.pgm", window);

        // normals (main.cpp:146-155)
        NormalOptimizer no(fs, &sct);
        std::vector<cv::Vec3d> normalsVector;
        no.setImages(img1, img2);
        no.startVisualizerThread();
        no.computeOptimizedNormals(triagulated, normalsVector, colors);

        // feature frames, neighbourhoods, patches (main.cpp:157-194)
        std::vector<cv::Matx44d> featuresFrames;
        no.computeFeaturesFrames(triagulated, normalsVector, featuresFrames);
        NeighborhoodsGenerator ng(fs);
        std::vector<std::vector<cv::Vec3d> > neighborhoodsVector;
        std::vector<cv::Vec3d> referenceNeighborhood;
        ng.getReferenceSquaredNeighborhood(referenceNeighborhood);
        std::vector<cv::Mat> patchesVector, imagePointsVector;
        sct.setImages(img1, img2);
        sct.projectReferencePointsToImageWithFrames(referenceNeighborhood, featuresFrames, patchesVector,
                                                    imagePointsVector);
        for (size_t i = 0; i < patchesVector.size(); i++)  // singlecameratriangulator.cpp:843-846
            cv::imwrite("patch_" + std::to_string(i) + ".pgm", patchesVector[i]);
        // main.cpp:182-183 (the settings' extractor on the GPU: SURF, SIFT, ORB or BRISK)
        cv::Mat descriptors;
        if (!patchesVector.empty()) {
            try {
                dm.extractDescriptorsFromPatches(patchesVector, descriptors);
            } catch (const fm3d::compat::Error& e) {
                if (e.code != FM3D_ERR_UNSUPPORTED) throw;
                std::cout << "extractDescriptorsFromPatches: " << e.what() << std::endl;
            }
        }
        ng.computeSquareNeighborhoodsByNormals(featuresFrames, neighborhoodsVector);
        cv::Mat img1_points;
        drawBackProjectedPoints(img1, img1_points, imagePointsVector, colors);
        cv::imwrite("projectedPatches.pgm", img1_points);
        no.stopVisualizerThread();
        cv::Vec3d gravity(no.getGravity());

        dump("out_matches.bin", matches.data(), matches.size() * sizeof(cv::DMatch));
        dump("out_points.f64", triagulated.data(), triagulated.size() * sizeof(cv::Vec3d));
        dump("out_normals.f64", normalsVector.data(), normalsVector.size() * sizeof(cv::Vec3d));
        dump(descriptors.depth() == CV_8U ? "out_patch_desc.u8" : "out_patch_desc.f32", descriptors.data,
             descriptors.empty() ? 0 : (size_t)descriptors.rows * descriptors.cols * descriptors.elemSize());
        dump("out_neighborhoods.f64", neighborhoodsVector.empty() ? nullptr : neighborhoodsVector[0].data(),
             neighborhoodsVector.empty() ? 0 : neighborhoodsVector[0].size() * sizeof(cv::Vec3d));
        std::cout << matches.size() << " matches, " << triagulated.size() << " points with normals, gravity "
                  << gravity << std::endl;
    } catch (const fm3d::compat::Error& e) {
        std::cerr << "fm3d error " << e.code << ": " << e.what() << std::endl;
        return e.code;
    }
    return 0;
}
