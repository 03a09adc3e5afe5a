// mosaic_demo.cpp -- the reference's MOSAIC descriptor extractor (mosaic.h:47-70) through
// include/fm3d_cv.hpp: MOSAIC(fs, imgA, imgB, tA, tB, rA, rB) runs the whole pipeline on the GPU,
// compute() describes the normal-rectified patches.
// Usage: mosaic_demo -s settings.yml  -> mosaic_desc.f32 (rows x 128), mosaic_points.f64
#include <fstream>
#include <iostream>
#include <vector>

#include "fm3d_cv.hpp"

int main(int argc, char** argv) {
    if (argc != 3 || std::string(argv[1]) != "-s") {
        std::cout << "Usage: mosaic_demo -s <settings.yml>" << std::endl;
        return -1;
    }
    try {
        cv::FileStorage fs;
        fs.open(argv[2], cv::FileStorage::READ);
        if (!fs.isOpened()) return -1;
        std::string IMG_1, IMG_2;
        fs["IMAGES"]["img1"] >> IMG_1;
        fs["IMAGES"]["img2"] >> IMG_2;
        cv::Mat imgA = cv::imread(IMG_1, CV_LOAD_IMAGE_GRAYSCALE), imgB = cv::imread(IMG_2, CV_LOAD_IMAGE_GRAYSCALE);
        if (imgA.empty() || imgB.empty()) return -1;
        std::vector<double> pos1, pos2;
        fs["IMAGES"]["pos1"] >> pos1;
        fs["IMAGES"]["pos2"] >> pos2;
        MOSAIC mosaic(fs, imgA, imgB, cv::Vec3d(pos1[0], pos1[1], pos1[2]), cv::Vec3d(pos2[0], pos2[1], pos2[2]),
                      cv::Vec3d(pos1[3], pos1[4], pos1[5]), cv::Vec3d(pos2[3], pos2[4], pos2[5]));
        cv::Mat descriptors;
        mosaic.compute(descriptors);
        std::ofstream d("mosaic_desc.f32", std::ios::binary);
        if (!descriptors.empty()) d.write((const char*)descriptors.data, (std::streamsize)descriptors.rows * descriptors.cols * 4);
        std::ofstream p("mosaic_points.f64", std::ios::binary);
        p.write((const char*)mosaic.points().data(), (std::streamsize)(mosaic.points().size() * sizeof(cv::Vec3d)));
        std::cout << mosaic.matches().size() << " matches, " << mosaic.points().size() << " features, "
                  << descriptors.rows << " x " << mosaic.descriptorSize() << " descriptors" << std::endl;
    } catch (const fm3d::compat::Error& e) {
        std::cerr << "fm3d error " << e.code << ": " << e.what() << std::endl;
        return e.code;
    }
    return 0;
}
