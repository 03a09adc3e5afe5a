// san_parse.cpp -- the settings.yml reader (csrc/fm3d_settings.cpp: fm3d_settings_load /
// fm3d_settings_lookup) and the PGM reader/writer of the cv:: stand-ins (include/fm3d_cv.hpp:
// imread / imwrite / FileStorage) under AddressSanitizer + UndefinedBehaviorSanitizer, on
// well-formed and malformed inputs (empty, truncated, binary garbage, huge or negative sizes,
// overlong lines and tokens, unterminated sequences, deep nesting).  Malformed inputs must be
// rejected (error code / empty Mat), never read out of bounds.  Run by tests/test_sanitizers.py.
#include <cstdio>
#include <fstream>
#include <random>
#include <string>

#include "fm3d_cv.hpp"

static int fails = 0;
#define EXPECT(c)                                                             \
    do {                                                                      \
        if (!(c)) {                                                           \
            std::fprintf(stderr, "%s:%d: expectation failed: %s\n", __FILE__, __LINE__, #c); \
            fails++;                                                          \
        }                                                                     \
    } while (0)

static std::string dir;
static std::string put(const std::string& name, const std::string& bytes) {
    const std::string p = dir + "/" + name;
    std::ofstream(p, std::ios::binary) << bytes;
    return p;
}

static void probe_yaml(const std::string& path) {
    fm3d_settings s;
    const int rc = fm3d_settings_load(path.c_str(), &s);
    EXPECT(rc == FM3D_OK || rc == FM3D_ERR_PARSE);
    const char* keys[] = {"IMAGES.img1", "IMAGES.pos1", "NNDR.epsilon", "Neighborhoods.pixelsRay", "A.B.C.D", "", "x"};
    for (const char* k : keys) {
        int len = -1;
        char small[4];
        if (fm3d_settings_lookup(path.c_str(), k, nullptr, 0, &len) == FM3D_OK) EXPECT(len >= 0);
        if (fm3d_settings_lookup(path.c_str(), k, small, sizeof(small), &len) == FM3D_OK) EXPECT(std::strlen(small) < 4);
    }
    cv::FileStorage fs(path, cv::FileStorage::READ);
    std::vector<double> v;
    std::string str;
    fs["IMAGES"]["pos1"] >> v;
    fs["IMAGES"]["img1"] >> str;
    double e = fs["NNDR"]["epsilon"];
    (void)e;
}

int main(int argc, char** argv) {
    dir = argc > 1 ? argv[1] : "/tmp";
    std::mt19937 rng(7);
    // ---- YAML
    const std::string good =
        "%YAML:1.0\nIMAGES:\n#TIME : 1 POS : 1 2 3\n\n   img1: /a/b.pgm\n   img2: c:d.pgm\n"
        "   pos1: [5.301099, 8.031408, 1.977258, 0.153433, 0.149941, -2.658648]\n"
        "NNDR:\n   epsilon: 0.55\nNeighborhoods:\n   pixelsRay: 64\n   pyramids: 3\n";
    probe_yaml(put("good.yml", good));
    {
        fm3d_settings s;
        EXPECT(fm3d_settings_load((dir + "/good.yml").c_str(), &s) == FM3D_OK && s.pixelsRay == 64 && s.pos1[5] == -2.658648);
        cv::FileStorage fs(dir + "/good.yml", cv::FileStorage::READ);
        std::string img;
        fs["IMAGES"]["img2"] >> img;
        EXPECT(img == "c:d.pgm");
    }
    probe_yaml(dir + "/missing.yml");
    probe_yaml(put("empty.yml", ""));
    probe_yaml(put("header.yml", "%YAML:1.0\n"));
    std::string garbage(4096, 0);
    for (char& c : garbage) c = (char)rng();
    probe_yaml(put("garbage.yml", garbage));
    probe_yaml(put("longline.yml", "%YAML:1.0\nA: " + std::string(1 << 20, 'x')));
    std::string deep = "%YAML:1.0\n";
    for (int i = 0; i < 300; i++) deep += std::string(i, ' ') + "k" + std::to_string(i) + ":\n";
    probe_yaml(put("deep.yml", deep));
    probe_yaml(put("bad_values.yml",
                   "%YAML:1.0\nIMAGES:\n   pos1: [1, 2\n   pos2: ]]]\nNNDR:\n   epsilon: 1e400\n"
                   "Neighborhoods:\n   pixelsRay: abc\n   pyramids: -99999999999999999999\n"
                   "CameraSettings:\n   Fx: nan\n   Fy:\n   rodriguesIC: [,,,]\n   :\n  ::: :\n\t\r\n"));
    probe_yaml(put("crlf.yml", "%YAML:1.0\r\nNNDR:\r\n   epsilon: 0.6\r\n"));
    // ---- PGM / PPM
    cv::Mat m = cv::imread(dir + "/missing.pgm", 0);
    EXPECT(m.empty());
    const char* bad[] = {"", "P5", "P5 10", "P5 10 10", "P5 10 10 255", "P5 10 10 255\nabc", "P5 -3 4 255\n\xff",
                         "P5 1048577 2 255\n", "P5 100000 100000 255\n", "P5 4 4 65535\n", "P5 11111111111111111111 1 255\n",
                         "P2 2 2 255\n1 2 3 4\n", "P5 2 2 255", "# only a comment\n", "P5 2 2 0\n\x01\x02\x03\x04"};
    for (const char* b : bad) {
        cv::Mat x = cv::imread(put("bad.pgm", std::string(b)), 0);
        EXPECT(x.empty());
    }
    {
        std::string g2 = "P5\n# c1\n3 # c2\n2\n255\n";
        g2 += std::string("\x01\x02\x03\x04\x05\x06", 6);
        cv::Mat x = cv::imread(put("ok.pgm", g2), 0);
        EXPECT(!x.empty() && x.rows == 2 && x.cols == 3 && x.data[5] == 6);
        EXPECT(cv::imwrite(dir + "/rt.pgm", x));
        cv::Mat y = cv::imread(dir + "/rt.pgm", 0);
        EXPECT(!y.empty() && std::memcmp(x.data, y.data, 6) == 0);
        std::string p6 = "P6 2 1 255\n";
        p6 += std::string("\xff\x00\x00\x00\x00\xff", 6);
        cv::Mat c = cv::imread(put("ok.ppm", p6), 1);
        EXPECT(!c.empty() && c.channels() == 3 && c.data[2] == 255 && c.data[3] == 255);  // stored BGR
        cv::Mat gray = cv::imread(dir + "/ok.ppm", CV_LOAD_IMAGE_GRAYSCALE);
        EXPECT(!gray.empty() && gray.data[0] == 76 && gray.data[1] == 29);
        EXPECT(cv::imwrite(dir + "/rt.ppm", c));
        EXPECT(!cv::imwrite(dir + "/x.pgm", cv::Mat()));
    }
    for (int trial = 0; trial < 200; trial++) {  // random headers and truncations
        std::string b = "P5 " + std::to_string((int)(rng() % 40) - 5) + " " + std::to_string((int)(rng() % 40) - 5) +
                        " " + std::to_string((int)(rng() % 300)) + "\n";
        b += std::string(rng() % 900, (char)rng());
        cv::Mat x = cv::imread(put("fuzz.pgm", b.substr(0, rng() % (b.size() + 1))), 0);
        if (!x.empty()) EXPECT(x.rows > 0 && x.cols > 0 && x.total() <= b.size());
    }
    std::printf("san_parse: %s\n", fails ? "FAILED" : "ok");
    return fails ? 1 : 0;
}
