// The real libstdc++ of this image behind a C ABI, for tests/test_orb_oracle.py: the oracle's C
// restatement of std::nth_element / std::partition (oracle/orc_orb.c, what KeyPointsFilter::retainBest
// calls in OpenCV's ORB) must reorder keypoints exactly as these do.
#include <algorithm>
#include <vector>

struct Kp {  // cv::KeyPoint layout
    float x, y, size, angle, response;
    int octave, class_id;
};
struct Greater {  // KeypointResponseGreater
    bool operator()(const Kp& a, const Kp& b) const { return a.response > b.response; }
};
struct GreaterThanThreshold {  // KeypointResponseGreaterThanThreshold
    float v;
    bool operator()(const Kp& k) const { return k.response >= v; }
};

extern "C" {
void cxx_nth_element(Kp* k, long nth, long n) { std::nth_element(k, k + nth, k + n, Greater()); }
long cxx_partition_ge(Kp* k, long lo, long hi, float thr) {
    return std::partition(k + lo, k + hi, GreaterThanThreshold{thr}) - k;
}
void cxx_heap_select(Kp* k, long mid, long n) {
    std::__heap_select(k, k + mid, k + n, __gnu_cxx::__ops::__iter_comp_iter(Greater()));
}
int cxx_retain_best(Kp* k, int n, int npts) {  // KeyPointsFilter::retainBest (OpenCV 2.4.9)
    if (npts >= 0 && n > npts) {
        if (npts == 0) return 0;
        std::nth_element(k, k + npts, k + n, Greater());
        const float amb = k[npts - 1].response;
        return (int)(std::partition(k + npts, k + n, GreaterThanThreshold{amb}) - k);
    }
    return n;
}
}
