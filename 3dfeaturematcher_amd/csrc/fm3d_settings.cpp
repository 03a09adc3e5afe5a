// fm3d_settings.cpp -- settings.yml reader (cv::FileStorage %YAML:1.0 subset).
//
// The reference reads build/settings.yml through cv::FileStorage with ad-hoc keys
// (main.cpp:62-98, singlecameratriangulator.cpp:45-112, normaloptimizer.cpp:154-164).
// This parser accepts the subset that file uses: "%YAML:1.0" header, nested maps by
// indentation, scalars, flow sequences "[a, b, c]", '#' comments.
#include <algorithm>
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "fm3d.h"

namespace {

std::string trim(const std::string& s) {
    size_t a = 0, b = s.size();
    while (a < b && std::isspace((unsigned char)s[a])) a++;
    while (b > a && std::isspace((unsigned char)s[b - 1])) b--;
    return s.substr(a, b - a);
}

bool parse_yaml(const char* path, std::map<std::string, std::string>& kv) {
    std::ifstream in(path);
    if (!in) return false;
    std::string line;
    std::vector<std::pair<int, std::string>> stack;  // (indent, key)
    bool first = true;
    while (std::getline(in, line)) {
        if (first) {
            first = false;
            if (line.rfind("%YAML", 0) == 0) continue;
        }
        // strip comments (not inside quotes; settings.yml has none)
        size_t hash = line.find('#');
        if (hash != std::string::npos) line = line.substr(0, hash);
        if (trim(line).empty()) continue;
        int indent = 0;
        while (indent < (int)line.size() && line[indent] == ' ') indent++;
        std::string body = trim(line);
        size_t colon = body.find(':');
        if (colon == std::string::npos) continue;
        std::string key = trim(body.substr(0, colon));
        std::string val = trim(body.substr(colon + 1));
        while (!stack.empty() && stack.back().first >= indent) stack.pop_back();
        std::string full;
        for (auto& e : stack) full += e.second + ".";
        full += key;
        if (val.empty()) {
            stack.push_back({indent, key});
        } else {
            if (val.size() >= 2 && (val[0] == '"' || val[0] == '\'')) val = val.substr(1, val.size() - 2);
            kv[full] = val;
        }
    }
    return true;
}

bool get_d(const std::map<std::string, std::string>& kv, const char* k, double* out) {
    auto it = kv.find(k);
    if (it == kv.end()) return false;
    *out = std::strtod(it->second.c_str(), nullptr);
    return true;
}

bool get_i(const std::map<std::string, std::string>& kv, const char* k, int* out) {
    double d;
    if (!get_d(kv, k, &d)) return false;
    *out = (int)d;
    return true;
}

bool get_vec(const std::map<std::string, std::string>& kv, const char* k, double* out, int n) {
    auto it = kv.find(k);
    if (it == kv.end()) return false;
    std::string v = it->second;
    for (char& c : v)
        if (c == '[' || c == ']' || c == ',') c = ' ';
    std::istringstream ss(v);
    for (int i = 0; i < n; i++)
        if (!(ss >> out[i])) return false;
    return true;
}

}  // namespace

extern "C" int fm3d_settings_default(fm3d_settings* s) {
    if (!s) return FM3D_ERR_INVALID;
    std::memset(s, 0, sizeof(*s));
    // build/settings.yml
    s->Fx = 572.4765;
    s->Fy = 572.69354;
    s->Cx = 549.75189;
    s->Cy = 411.68039;
    s->p1 = -6.6e-05;
    s->p2 = 0.000567;
    s->k0 = -0.299957;
    s->k1 = 0.124129;
    s->k2 = -0.028357;
    s->rodriguesIC[0] = -1.2005;
    s->rodriguesIC[1] = 1.1981;
    s->rodriguesIC[2] = -1.2041;
    s->translationIC[0] = 0.0;
    s->translationIC[1] = 0.015;
    s->translationIC[2] = -0.051;
    s->zThresholdMin = 1.5;
    s->zThresholdMax = 2.4;
    s->epsilonLMMIN = 1e-10;
    s->pixelsRay = 64;
    s->pyramids = 3;
    s->nndrEpsilon = 0.55;
    const double p1[6] = {5.301099, 8.031408, 1.977258, 0.153433, 0.149941, -2.658648};
    const double p2[6] = {4.735536, 7.691893, 1.913166, 0.252828, 0.048977, -2.676886};
    for (int i = 0; i < 6; i++) {
        s->pos1[i] = p1[i];
        s->pos2[i] = p2[i];
    }
    s->boundWidth = 1024;
    s->boundHeight = 768;
    s->strictNanExit = 0;
    s->lmWaves = 0;
    s->neighEpsilon = 0.16;  // build/settings.yml Neighborhoods
    s->cmPerPixel = 0.25;
    s->neighMethod = 0;      // method: square
    s->neighThetas = 15;     // the commented-out circular values of build/settings.yml
    s->neighRays = 5;
    s->detectorType = FM3D_FEAT_SURF;  // FeatureOptions: STATIC SURF detector + extractor
    s->extractorType = FM3D_FEAT_SURF;
    s->surfHessianThreshold = 400;
    s->surfOctaves = 4;
    s->surfOctaveLayers = 2;
    s->surfExtended = 1;
    s->surfUpright = 1;
    s->orbNumFeatures = 500;  // cv::ORB's defaults (FeatureOptions.OrbDetector, absent from settings.yml)
    s->orbScaleFactor = 1.2;
    s->orbNumLevels = 8;
    s->orbEdgeThreshold = 31;
    s->orbPatchSize = 31;
    s->orbFastThreshold = 20;
    s->siftNumFeatures = 0;  // cv::SIFT's defaults (FeatureOptions.SiftDetector, absent from settings.yml)
    s->siftOctaveLayers = 3;
    s->siftContrastThreshold = 0.04;
    s->siftEdgeThreshold = 10;
    s->siftSigma = 1.6;
    s->detectorMode = 0;
    s->fastThreshold = 10;  // cv::FastFeatureDetector's defaults
    s->fastNonmax = 1;
    s->adaptiveMinFeatures = 400;  // cv::DynamicAdaptedFeatureDetector's defaults
    s->adaptiveMaxFeatures = 500;
    s->adaptiveMaxIters = 5;
    s->starMaxSize = 45;  // cv::StarDetector's defaults
    s->starResponse = 30;
    s->starLineThreshold = 10;
    s->starLineBinarized = 8;
    s->starSuppression = 5;
    s->briskThreshold = 30;  // cv::BRISK's defaults
    s->briskOctaves = 3;
    s->mserDelta = 5;  // cv::MSER's defaults
    s->mserMinArea = 60;
    s->mserMaxArea = 14400;
    s->mserMaxVariation = 0.25;
    s->mserMinDiversity = 0.2;
    s->mserMaxEvolution = 200;
    s->mserAreaThreshold = 1.01;
    s->mserMinMargin = 0.003;
    s->mserEdgeBlurSize = 5;
    s->lmReduction = 0;  // pixel-order sums (the reference's)
    s->dltSolver = 0;    // OpenCV 2.4 cvSVD (the reference's)
    return FM3D_OK;
}

extern "C" int fm3d_settings_load(const char* path, fm3d_settings* s) {
    if (!path || !s) return FM3D_ERR_INVALID;
    std::map<std::string, std::string> kv;
    if (!parse_yaml(path, kv)) return FM3D_ERR_PARSE;
    fm3d_settings_default(s);
    get_d(kv, "CameraSettings.Fx", &s->Fx);
    get_d(kv, "CameraSettings.Fy", &s->Fy);
    get_d(kv, "CameraSettings.Cx", &s->Cx);
    get_d(kv, "CameraSettings.Cy", &s->Cy);
    get_d(kv, "CameraSettings.p1", &s->p1);
    get_d(kv, "CameraSettings.p2", &s->p2);
    get_d(kv, "CameraSettings.k0", &s->k0);
    get_d(kv, "CameraSettings.k1", &s->k1);
    get_d(kv, "CameraSettings.k2", &s->k2);
    get_vec(kv, "CameraSettings.rodriguesIC", s->rodriguesIC, 3);
    get_vec(kv, "CameraSettings.translationIC", s->translationIC, 3);
    get_d(kv, "CameraSettings.zThresholdMin", &s->zThresholdMin);
    get_d(kv, "CameraSettings.zThresholdMax", &s->zThresholdMax);
    get_d(kv, "Neighborhoods.epsilonLMMIN", &s->epsilonLMMIN);
    get_i(kv, "Neighborhoods.pixelsRay", &s->pixelsRay);
    get_i(kv, "Neighborhoods.pyramids", &s->pyramids);
    get_d(kv, "NNDR.epsilon", &s->nndrEpsilon);
    get_d(kv, "Neighborhoods.epsilon", &s->neighEpsilon);
    get_d(kv, "Neighborhoods.cmPerPixel", &s->cmPerPixel);
    {
        auto it = kv.find("Neighborhoods.method");
        if (it != kv.end()) {
            std::string m = it->second;
            if (m.size() >= 2 && (m[0] == '"' || m[0] == '\'') && m.back() == m[0]) m = m.substr(1, m.size() - 2);
            s->neighMethod = m == "square" ? 0 : (m == "circular" ? 1 : -1);
        }
    }
    {
        auto str = [&](const char* k, std::string& v) {
            auto it = kv.find(k);
            if (it == kv.end()) return false;
            v = it->second;
            if (v.size() >= 2 && (v[0] == '"' || v[0] == '\'') && v.back() == v[0]) v = v.substr(1, v.size() - 2);
            return true;
        };
        std::string mode = "STATIC", det, ex;
        str("FeatureOptions.DetectorMode", mode);
        s->detectorMode = mode == "ADAPTIVE" ? 1 : 0;
        if (str("FeatureOptions.DetectorType", det)) {
            if (mode == "STATIC")
                s->detectorType = det == "SURF"   ? FM3D_FEAT_SURF
                                  : det == "ORB"  ? FM3D_FEAT_ORB
                                  : det == "SIFT" ? FM3D_FEAT_SIFT
                                  : det == "FAST" ? FM3D_FEAT_FAST
                                  : det == "STAR" ? FM3D_FEAT_STAR
                                  : det == "MSER" ? FM3D_FEAT_MSER
                                                  : FM3D_FEAT_OTHER;
            else  // ADAPTIVE: the FAST / SURF / STAR adjusters
                s->detectorType = mode != "ADAPTIVE" ? FM3D_FEAT_OTHER
                                  : det == "SURF"    ? FM3D_FEAT_SURF
                                  : det == "FAST"    ? FM3D_FEAT_FAST
                                  : det == "STAR"    ? FM3D_FEAT_STAR
                                                     : FM3D_FEAT_OTHER;
        }
        {
            int nm = s->fastNonmax;
            get_i(kv, "FeatureOptions.FastDetector.Threshold", &s->fastThreshold);
            get_i(kv, "FeatureOptions.FastDetector.NonMaxSuppression", &nm);
            s->fastNonmax = nm > 0;  // (int)fs[...] > 0
        }
        get_i(kv, "FeatureOptions.StarDetector.MaxSize", &s->starMaxSize);
        get_i(kv, "FeatureOptions.StarDetector.Response", &s->starResponse);
        get_i(kv, "FeatureOptions.StarDetector.LineThreshold", &s->starLineThreshold);
        get_i(kv, "FeatureOptions.StarDetector.LineBinarized", &s->starLineBinarized);
        get_i(kv, "FeatureOptions.StarDetector.Suppression", &s->starSuppression);
        get_i(kv, "FeatureOptions.MSERDetector.Delta", &s->mserDelta);
        get_i(kv, "FeatureOptions.MSERDetector.MinArea", &s->mserMinArea);
        get_i(kv, "FeatureOptions.MSERDetector.MaxArea", &s->mserMaxArea);
        get_d(kv, "FeatureOptions.MSERDetector.MaxVariation", &s->mserMaxVariation);
        get_d(kv, "FeatureOptions.MSERDetector.MinDiversity", &s->mserMinDiversity);
        get_i(kv, "FeatureOptions.MSERDetector.MaxEvolution", &s->mserMaxEvolution);
        get_d(kv, "FeatureOptions.MSERDetector.AreaThreshold", &s->mserAreaThreshold);
        get_d(kv, "FeatureOptions.MSERDetector.MinMargin", &s->mserMinMargin);
        get_i(kv, "FeatureOptions.MSERDetector.EdgeBlurSize", &s->mserEdgeBlurSize);
        get_i(kv, "FeatureOptions.Adaptive.MinFeatures", &s->adaptiveMinFeatures);
        get_i(kv, "FeatureOptions.Adaptive.MaxFeatures", &s->adaptiveMaxFeatures);
        get_i(kv, "FeatureOptions.Adaptive.MaxIters", &s->adaptiveMaxIters);
        if (str("FeatureOptions.ExtractorType", ex))
            s->extractorType = ex == "SURF"    ? FM3D_FEAT_SURF
                               : ex == "ORB"   ? FM3D_FEAT_ORB
                               : ex == "SIFT"  ? FM3D_FEAT_SIFT
                               : ex == "BRISK" ? FM3D_FEAT_BRISK
                               : ex == "FREAK" ? FM3D_FEAT_FREAK
                                               : FM3D_FEAT_OTHER;
        get_i(kv, "FeatureOptions.BriskDetector.Threshold", &s->briskThreshold);
        get_i(kv, "FeatureOptions.BriskDetector.Octaves", &s->briskOctaves);
        get_i(kv, "FeatureOptions.SiftDetector.NumFeatures", &s->siftNumFeatures);
        get_i(kv, "FeatureOptions.SiftDetector.NumOctaveLayers", &s->siftOctaveLayers);
        get_d(kv, "FeatureOptions.SiftDetector.ContrastThreshold", &s->siftContrastThreshold);
        get_d(kv, "FeatureOptions.SiftDetector.EdgeThreshold", &s->siftEdgeThreshold);
        get_d(kv, "FeatureOptions.SiftDetector.Sigma", &s->siftSigma);
        get_i(kv, "FeatureOptions.OrbDetector.NumFeatures", &s->orbNumFeatures);
        get_d(kv, "FeatureOptions.OrbDetector.ScaleFactor", &s->orbScaleFactor);
        get_i(kv, "FeatureOptions.OrbDetector.NumLevels", &s->orbNumLevels);
        get_d(kv, "FeatureOptions.SurfDetector.HessianThreshold", &s->surfHessianThreshold);
        get_i(kv, "FeatureOptions.SurfDetector.NumOctaves", &s->surfOctaves);
        get_i(kv, "FeatureOptions.SurfDetector.NumOctaveLayers", &s->surfOctaveLayers);
        int e = s->surfExtended, u = s->surfUpright;
        get_i(kv, "FeatureOptions.SurfDetector.Extended", &e);
        get_i(kv, "FeatureOptions.SurfDetector.Upright", &u);
        s->surfExtended = e > 0;  // (int)fs[...] > 0
        s->surfUpright = u > 0;
    }
    get_i(kv, "Neighborhoods.thetas", &s->neighThetas);
    get_i(kv, "Neighborhoods.rays", &s->neighRays);
    get_vec(kv, "IMAGES.pos1", s->pos1, 6);
    get_vec(kv, "IMAGES.pos2", s->pos2, 6);
    // extensions (optional section)
    get_i(kv, "Fm3d.boundWidth", &s->boundWidth);
    get_i(kv, "Fm3d.boundHeight", &s->boundHeight);
    get_i(kv, "Fm3d.strictNanExit", &s->strictNanExit);
    get_i(kv, "Fm3d.lmWaves", &s->lmWaves);
    get_i(kv, "Fm3d.lmReduction", &s->lmReduction);
    get_i(kv, "Fm3d.dltSolver", &s->dltSolver);
    return FM3D_OK;
}

extern "C" int fm3d_settings_lookup(const char* path, const char* key, char* out, int cap, int* len) {
    if (!path || !key || !len || cap < 0 || (cap > 0 && !out)) return FM3D_ERR_INVALID;
    std::map<std::string, std::string> kv;
    if (!parse_yaml(path, kv)) return FM3D_ERR_PARSE;
    auto it = kv.find(key);
    if (it == kv.end()) return FM3D_ERR_INVALID;
    *len = (int)it->second.size();
    if (cap > 0) {
        const size_t n = std::min((size_t)cap - 1, it->second.size());
        std::memcpy(out, it->second.data(), n);
        out[n] = 0;
    }
    return FM3D_OK;
}
