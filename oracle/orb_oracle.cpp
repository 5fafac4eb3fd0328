// ============================================================================================
// orb_oracle.cpp — CPU ORACLE (test infrastructure only; NOT part of the product path).
//
// A plain C++ restatement of the ORB-SLAM3 front-end hot path as vendored in
// giltchcity/orb_slam3_ros, used (a) as the bit-exact checker for the HIP kernels in
// orb_slam3_ros_amd/csrc and (b) as the timed CPU baseline ("kind": "port") in bench.py.
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
//
// Follows (file:line are under /root/reference/orb_slam3/):
//   src/ORBextractor.cc:76-103    IC_Angle                       -> ic_angle()
//   src/ORBextractor.cc:106-146   computeOrbDescriptor           -> orb_descriptor()
//   src/ORBextractor.cc:409-469   ORBextractor ctor (tables)     -> Extractor::Extractor()
//   src/ORBextractor.cc:480-553   DivideNode / compareNodes      -> Node::divide(), compare_nodes()
//   src/ORBextractor.cc:555-779   DistributeOctTree              -> Extractor::distribute_octtree()
//   src/ORBextractor.cc:781-896   ComputeKeyPointsOctTree        -> Extractor::compute_keypoints()
//   src/ORBextractor.cc:1086-1168 operator()                     -> Extractor::extract()
//   src/ORBextractor.cc:1170-1195 ComputePyramid                 -> Extractor::compute_pyramid()
//   src/Frame.cc:811-981          Frame::ComputeStereoMatches    -> oro_stereo_match()
//   src/ORBmatcher.cc:2058-2074   DescriptorDistance             -> hamming()
//
// PARITY STATUS: "parity unpinned" w.r.t. the real reference. The reference cannot be built
// here (OpenCV 4.2 / Eigen / Boost absent, no network) and ships no tests, golden vectors or
// fixtures for this path. The OpenCV 4.2 primitives it calls are restated
// from their published algorithms; every assumption is a switch recorded in fixture metadata:
//   * cv::resize INTER_LINEAR 8U: fixed-point (11-bit coefs); vertical pass modelled with the
//     universal-intrinsic split (`resize_simd_lanes`, default 16 = SSE baseline; 0 = scalar).
//   * cv::GaussianBlur 7x7 sigma 2 8U: bit-exact fixed-point path; kernel quantisation
//     `blur_kernel` 0 = error-diffusion [18,34,48,56,48,34,18] (default), 1 = per-tap rounding.
//   * cv::FAST TYPE_9_16 with non-max suppression, cornerScore<16>.
//   * cv::fastAtan2 (OpenCV 4.x atan_f32 polynomial), no FMA contraction.
//   * cos/sin of the float angle: glibc cosf/sinf of the host (what the reference calls).
//   * std::sort in DistributeOctTree: the host libstdc++ introsort (what the reference calls).
// Built with -ffp-contract=off (see oracle/Makefile).
// ============================================================================================
#include <algorithm>
#include <chrono>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <list>
#include <thread>
#include <vector>

#include "../orb_slam3_ros_amd/csrc/brief_pattern.h"

namespace oracle {

// ---- OpenCV scalar helpers (core/fast_math.hpp semantics on x86-64 SSE2) ----
static inline int cv_round(float v) { return (int)std::lrintf(v); }   // half-to-even
static inline int cv_round(double v) { return (int)std::lrint(v); }
static inline int cv_floor(float v) { int i = (int)v; return i - (i > v); }
static inline int cv_floor(double v) { int i = (int)v; return i - (i > v); }
static inline int cv_ceil(float v) { int i = (int)v; return i + (i < v); }
static inline uint8_t sat_u8(int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }
static inline short sat_s16_from_float(float v) {
    int iv = cv_round(v);
    return (short)(iv < -32768 ? -32768 : (iv > 32767 ? 32767 : iv));
}

struct KeyPoint {          // byte layout of cv::KeyPoint (28 B)
    float x, y, size, angle, response;
    int octave, class_id;
};

struct Image {             // tightly packed u8 plane
    int w = 0, h = 0;
    std::vector<uint8_t> px;
    uint8_t at(int x, int y) const { return px[(size_t)y * w + x]; }
    const uint8_t* row(int y) const { return px.data() + (size_t)y * w; }
};

// OpenCV's own code is compiled into libopencv_* with OpenCV's flags, not the reference's
// -march=native: in the reference-flags build of this file (liborb_oracle_contract.so,
// tests/test_oracle_contraction.py) these restatements stay uncontracted while the code the
// reference owns (computeOrbDescriptor, ComputeStereoMatches, ...) is contracted as g++ does.
#define ORO_OPENCV __attribute__((optimize("fp-contract=off")))

// ---- cv::fastAtan2 (OpenCV 4.x mathfuncs atan_f32) ----
static const float kAtanP1 = 0.9997878412794807f * (float)(180 / M_PI);
static const float kAtanP3 = -0.3258083974640975f * (float)(180 / M_PI);
static const float kAtanP5 = 0.1555786518463281f * (float)(180 / M_PI);
static const float kAtanP7 = -0.04432655554792128f * (float)(180 / M_PI);
ORO_OPENCV float fast_atan2(float y, float x) {
    float ax = std::fabs(x), ay = std::fabs(y), a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + (float)DBL_EPSILON);
        c2 = c * c;
        a = (((kAtanP7 * c2 + kAtanP5) * c2 + kAtanP3) * c2 + kAtanP1) * c;
    } else {
        c = ax / (ay + (float)DBL_EPSILON);
        c2 = c * c;
        a = 90.f - (((kAtanP7 * c2 + kAtanP5) * c2 + kAtanP3) * c2 + kAtanP1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

// ---- cv::resize(src, dst, dsize, 0, 0, INTER_LINEAR), CV_8UC1 (imgproc/resize.cpp) ----
ORO_OPENCV void resize_linear(const Image& src, Image& dst, int dw, int dh, int simd_lanes) {
    dst.w = dw; dst.h = dh; dst.px.assign((size_t)dw * dh, 0);
    if (dw == src.w && dh == src.h) { dst.px = src.px; return; }
    const double inv_x = (double)dw / src.w, inv_y = (double)dh / src.h;
    const double scale_x = 1. / inv_x, scale_y = 1. / inv_y;
    const int ONE = 2048;
    std::vector<int> xofs(dw);
    std::vector<short> ialpha(2 * dw);
    int xmax = dw;
    for (int dx = 0; dx < dw; dx++) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = cv_floor(fx);
        fx -= sx;
        if (sx < 0) { fx = 0; sx = 0; }
        if (sx + 1 >= src.w) {
            xmax = std::min(xmax, dx);
            if (sx >= src.w - 1) { fx = 0; sx = src.w - 1; }
        }
        xofs[dx] = sx;
        ialpha[2 * dx] = sat_s16_from_float((1.f - fx) * ONE);
        ialpha[2 * dx + 1] = sat_s16_from_float(fx * ONE);
    }
    std::vector<int> H0(dw), H1(dw);
    auto hresize = [&](int sy, std::vector<int>& D) {
        const uint8_t* S = src.row(sy);
        for (int dx = 0; dx < dw; dx++) {
            int sx = xofs[dx];
            D[dx] = dx < xmax ? S[sx] * ialpha[2 * dx] + S[sx + 1] * ialpha[2 * dx + 1] : S[sx] * ONE;
        }
    };
    for (int dy = 0; dy < dh; dy++) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        int sy = cv_floor(fy);
        fy -= sy;
        const int b0 = sat_s16_from_float((1.f - fy) * ONE);
        const int b1 = sat_s16_from_float(fy * ONE);
        auto clip = [&](int v) { return v < 0 ? 0 : (v >= src.h ? src.h - 1 : v); };
        hresize(clip(sy), H0);
        hresize(clip(sy + 1), H1);
        uint8_t* D = dst.px.data() + (size_t)dy * dw;
        int x = 0;
        if (simd_lanes > 0) {  // VResizeLinearVec_32s8u (universal intrinsics, v_uint8 = simd_lanes)
            const int half = simd_lanes / 2;
            auto vec = [&](int xx) {
                int a = (int)(((int64_t)(int16_t)(H0[xx] >> 4) * b0) >> 16);
                int b = (int)(((int64_t)(int16_t)(H1[xx] >> 4) * b1) >> 16);
                D[xx] = sat_u8((a + b + 2) >> 2);
            };
            for (; x <= dw - simd_lanes; x += simd_lanes)
                for (int k = 0; k < simd_lanes; k++) vec(x + k);
            for (; x < dw - half; x += half)
                for (int k = 0; k < half; k++) vec(x + k);
        }
        for (; x < dw; x++) D[x] = sat_u8((H0[x] * b0 + H1[x] * b1 + (1 << 21)) >> 22);
    }
}

// ---- cv::GaussianBlur(img, img, Size(7,7), 2, 2, BORDER_REFLECT_101), CV_8U fixed point ----
static const int kBlurED[7] = {18, 34, 48, 56, 48, 34, 18};
static const int kBlurRound[7] = {18, 34, 49, 55, 49, 34, 18};
static inline int reflect101(int p, int n) {
    if (n == 1) return 0;
    while (p < 0 || p >= n) p = p < 0 ? -p : 2 * n - 2 - p;
    return p;
}
ORO_OPENCV void gaussian_blur7(const Image& src, Image& dst, int variant) {
    const int* k = variant == 1 ? kBlurRound : kBlurED;
    const int w = src.w, h = src.h;
    std::vector<uint32_t> rowq((size_t)w * h);   // Q8 row-pass values
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            uint32_t s = 0;
            for (int i = -3; i <= 3; i++) s += (uint32_t)k[i + 3] * src.at(reflect101(x + i, w), y);
            rowq[(size_t)y * w + x] = s;
        }
    dst.w = w; dst.h = h; dst.px.assign((size_t)w * h, 0);
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            uint32_t s = 0;
            for (int j = -3; j <= 3; j++) s += (uint32_t)k[j + 3] * rowq[(size_t)reflect101(y + j, h) * w + x];
            uint32_t v = (s + 32768u) >> 16;
            dst.px[(size_t)y * w + x] = (uint8_t)(v > 255 ? 255 : v);
        }
}

// ---- cv::FAST(roi, kps, th, nonmax=true), TYPE_9_16 (features2d/fast.cpp FAST_t<16>) ----
static const int kRing[16][2] = {{0, 3}, {1, 3}, {2, 2}, {3, 1}, {3, 0}, {3, -1}, {2, -2}, {1, -3},
                                 {0, -3}, {-1, -3}, {-2, -2}, {-3, -1}, {-3, 0}, {-3, 1}, {-2, 2}, {-1, 3}};

ORO_OPENCV static int corner_score16(const uint8_t* p, const int* pixel, int threshold) {
    const int K = 8, N = 25;
    int v = p[0];
    int d[N];
    for (int k = 0; k < N; k++) d[k] = v - p[pixel[k]];
    int a0 = threshold;
    for (int k = 0; k < 16; k += 2) {
        int a = std::min(d[k + 1], d[k + 2]);
        a = std::min(a, d[k + 3]);
        if (a <= a0) continue;
        a = std::min(a, d[k + 4]); a = std::min(a, d[k + 5]); a = std::min(a, d[k + 6]);
        a = std::min(a, d[k + 7]); a = std::min(a, d[k + 8]);
        a0 = std::max(a0, std::min(a, d[k]));
        a0 = std::max(a0, std::min(a, d[k + 9]));
    }
    int b0 = -a0;
    for (int k = 0; k < 16; k += 2) {
        int b = std::max(d[k + 1], d[k + 2]);
        b = std::max(b, d[k + 3]); b = std::max(b, d[k + 4]); b = std::max(b, d[k + 5]);
        if (b >= b0) continue;
        b = std::max(b, d[k + 6]); b = std::max(b, d[k + 7]); b = std::max(b, d[k + 8]);
        b0 = std::min(b0, std::max(b, d[k]));
        b0 = std::min(b0, std::max(b, d[k + 9]));
    }
    (void)K;
    return -b0 - 1;
}

// roi: pointer to top-left, step = row stride, rows x cols.
ORO_OPENCV void fast9(const uint8_t* roi, int step, int rows, int cols, int threshold, std::vector<KeyPoint>& kps) {
    const int K = 8, N = 25;
    int pixel[25];
    for (int k = 0; k < 16; k++) pixel[k] = kRing[k][0] + kRing[k][1] * step;
    for (int k = 16; k < 25; k++) pixel[k] = pixel[k - 16];
    kps.clear();
    threshold = std::min(std::max(threshold, 0), 255);
    uint8_t tab[512];
    for (int i = -255; i <= 255; i++) tab[i + 255] = (uint8_t)(i < -threshold ? 1 : i > threshold ? 2 : 0);
    if (cols < 1) return;
    std::vector<uint8_t> bufv((size_t)cols * 3, 0);
    std::vector<int> cpv((size_t)(cols + 1) * 3, 0);
    uint8_t* buf[3] = {bufv.data(), bufv.data() + cols, bufv.data() + 2 * cols};
    int* cpbuf[3] = {cpv.data() + 1, cpv.data() + 1 + (cols + 1), cpv.data() + 1 + 2 * (cols + 1)};
    for (int i = 3; i < rows - 2; i++) {
        const uint8_t* ptr = roi + (size_t)i * step + 3;
        uint8_t* curr = buf[(i - 3) % 3];
        int* cornerpos = cpbuf[(i - 3) % 3];
        memset(curr, 0, cols);
        int ncorners = 0;
        if (i < rows - 3) {
            for (int j = 3; j < cols - 3; j++, ptr++) {
                int v = ptr[0];
                const uint8_t* t = &tab[0] - v + 255;
                int d = t[ptr[pixel[0]]] | t[ptr[pixel[8]]];
                if (d == 0) continue;
                d &= t[ptr[pixel[2]]] | t[ptr[pixel[10]]];
                d &= t[ptr[pixel[4]]] | t[ptr[pixel[12]]];
                d &= t[ptr[pixel[6]]] | t[ptr[pixel[14]]];
                if (d == 0) continue;
                d &= t[ptr[pixel[1]]] | t[ptr[pixel[9]]];
                d &= t[ptr[pixel[3]]] | t[ptr[pixel[11]]];
                d &= t[ptr[pixel[5]]] | t[ptr[pixel[13]]];
                d &= t[ptr[pixel[7]]] | t[ptr[pixel[15]]];
                if (d & 1) {
                    int vt = v - threshold, count = 0;
                    for (int k = 0; k < N; k++) {
                        int x = ptr[pixel[k]];
                        if (x < vt) {
                            if (++count > K) {
                                cornerpos[ncorners++] = j;
                                curr[j] = (uint8_t)corner_score16(ptr, pixel, threshold);
                                break;
                            }
                        } else count = 0;
                    }
                }
                if (d & 2) {
                    int vt = v + threshold, count = 0;
                    for (int k = 0; k < N; k++) {
                        int x = ptr[pixel[k]];
                        if (x > vt) {
                            if (++count > K) {
                                cornerpos[ncorners++] = j;
                                curr[j] = (uint8_t)corner_score16(ptr, pixel, threshold);
                                break;
                            }
                        } else count = 0;
                    }
                }
            }
        }
        cornerpos[-1] = ncorners;
        if (i == 3) continue;
        const uint8_t* prev = buf[(i - 4 + 3) % 3];
        const uint8_t* pprev = buf[(i - 5 + 3) % 3];
        cornerpos = cpbuf[(i - 4 + 3) % 3];
        ncorners = cornerpos[-1];
        for (int k = 0; k < ncorners; k++) {
            int j = cornerpos[k];
            int score = prev[j];
            if (score > prev[j + 1] && score > prev[j - 1] && score > pprev[j - 1] && score > pprev[j] &&
                score > pprev[j + 1] && score > curr[j - 1] && score > curr[j] && score > curr[j + 1])
                kps.push_back(KeyPoint{(float)j, (float)(i - 1), 7.f, -1.f, (float)score, 0, -1});
        }
    }
}

// ---- ExtractorNode (ORBextractor.h:30-41, ORBextractor.cc:480-536) ----
struct Node {
    std::vector<KeyPoint> keys;
    int ulx = 0, uly = 0, urx = 0, ury = 0, blx = 0, bly = 0, brx = 0, bry = 0;
    std::list<Node>::iterator lit;
    bool no_more = false;
    void divide(Node& n1, Node& n2, Node& n3, Node& n4) const {
        const int halfX = (int)std::ceil((float)(urx - ulx) / 2);
        const int halfY = (int)std::ceil((float)(bry - uly) / 2);
        n1.ulx = ulx; n1.uly = uly; n1.urx = ulx + halfX; n1.ury = uly;
        n1.blx = ulx; n1.bly = uly + halfY; n1.brx = ulx + halfX; n1.bry = uly + halfY;
        n2.ulx = n1.urx; n2.uly = n1.ury; n2.urx = urx; n2.ury = ury;
        n2.blx = n1.brx; n2.bly = n1.bry; n2.brx = urx; n2.bry = uly + halfY;
        n3.ulx = n1.blx; n3.uly = n1.bly; n3.urx = n1.brx; n3.ury = n1.bry;
        n3.blx = blx; n3.bly = bly; n3.brx = n1.brx; n3.bry = bly;
        n4.ulx = n3.urx; n4.uly = n3.ury; n4.urx = n2.brx; n4.ury = n2.bry;
        n4.blx = n3.brx; n4.bly = n3.bry; n4.brx = brx; n4.bry = bry;
        for (const KeyPoint& kp : keys) {
            if (kp.x < n1.urx) {
                if (kp.y < n1.bry) n1.keys.push_back(kp); else n3.keys.push_back(kp);
            } else if (kp.y < n1.bry) n2.keys.push_back(kp);
            else n4.keys.push_back(kp);
        }
        if (n1.keys.size() == 1) n1.no_more = true;
        if (n2.keys.size() == 1) n2.no_more = true;
        if (n3.keys.size() == 1) n3.no_more = true;
        if (n4.keys.size() == 1) n4.no_more = true;
    }
};
typedef std::pair<int, Node*> SizeNode;
static bool compare_nodes(const SizeNode& e1, const SizeNode& e2) {
    if (e1.first < e2.first) return true;
    if (e1.first > e2.first) return false;
    return e1.second->ulx < e2.second->ulx;
}

struct Extractor {
    int nfeatures, nlevels, iniTh, minTh;
    double scaleFactor;
    int resize_simd_lanes = 16, blur_variant = 0;
    std::vector<float> scale, inv_scale, sigma2, inv_sigma2;
    std::vector<int> per_level, umax;
    std::vector<Image> pyramid;
    // debug captures of the last call
    std::vector<std::vector<KeyPoint>> raw_keys, level_keys;

    Extractor(int nf, float sf, int nl, int ini, int mn)
        : nfeatures(nf), nlevels(nl), iniTh(ini), minTh(mn), scaleFactor(sf) {
        scale.resize(nl); sigma2.resize(nl);
        scale[0] = 1.0f; sigma2[0] = 1.0f;
        for (int i = 1; i < nl; i++) {
            scale[i] = scale[i - 1] * scaleFactor;
            sigma2[i] = scale[i] * scale[i];
        }
        inv_scale.resize(nl); inv_sigma2.resize(nl);
        for (int i = 0; i < nl; i++) { inv_scale[i] = 1.0f / scale[i]; inv_sigma2[i] = 1.0f / sigma2[i]; }
        pyramid.resize(nl);
        per_level.resize(nl);
        float factor = 1.0f / scaleFactor;
        float nDesired = nf * (1 - factor) / (1 - (float)pow((double)factor, (double)nl));
        int sum = 0;
        for (int l = 0; l < nl - 1; l++) {
            per_level[l] = cv_round(nDesired);
            sum += per_level[l];
            nDesired *= factor;
        }
        per_level[nl - 1] = std::max(nf - sum, 0);
        umax.resize(16);
        int v, v0, vmax = cv_floor(15 * std::sqrt(2.f) / 2 + 1);
        int vmin = cv_ceil(15 * std::sqrt(2.f) / 2);
        const double hp2 = 15 * 15;
        for (v = 0; v <= vmax; ++v) umax[v] = cv_round(std::sqrt(hp2 - v * v));
        for (v = 15, v0 = 0; v >= vmin; --v) {
            while (umax[v0] == umax[v0 + 1]) ++v0;
            umax[v] = v0;
            ++v0;
        }
    }

    void compute_pyramid(const Image& img) {
        for (int l = 0; l < nlevels; l++) {
            const float s = inv_scale[l];
            const int w = cv_round((float)img.w * s), h = cv_round((float)img.h * s);
            if (l == 0) pyramid[0] = img;
            else resize_linear(pyramid[l - 1], pyramid[l], w, h, resize_simd_lanes);
        }
    }

    std::vector<KeyPoint> distribute_octtree(const std::vector<KeyPoint>& toDistribute, int minX, int maxX,
                                             int minY, int maxY, int N) {
        const int nIni = (int)std::round((float)(maxX - minX) / (maxY - minY));
        const float hX = (float)(maxX - minX) / nIni;
        std::list<Node> lNodes;
        std::vector<Node*> ini(nIni);
        for (int i = 0; i < nIni; i++) {
            Node ni;
            ni.ulx = (int)(hX * (float)i); ni.uly = 0;
            ni.urx = (int)(hX * (float)(i + 1)); ni.ury = 0;
            ni.blx = ni.ulx; ni.bly = maxY - minY;
            ni.brx = ni.urx; ni.bry = maxY - minY;
            lNodes.push_back(ni);
            ini[i] = &lNodes.back();
        }
        for (const KeyPoint& kp : toDistribute) ini[(size_t)(kp.x / hX)]->keys.push_back(kp);
        auto lit = lNodes.begin();
        while (lit != lNodes.end()) {
            if (lit->keys.size() == 1) { lit->no_more = true; lit++; }
            else if (lit->keys.empty()) lit = lNodes.erase(lit);
            else lit++;
        }
        bool finish = false;
        std::vector<SizeNode> vSize;
        vSize.reserve(lNodes.size() * 4);
        auto push_children = [&](Node& n1, Node& n2, Node& n3, Node& n4, int* nToExpand) {
            Node* ch[4] = {&n1, &n2, &n3, &n4};
            for (int c = 0; c < 4; c++) {
                if (ch[c]->keys.size() > 0) {
                    lNodes.push_front(*ch[c]);
                    if (ch[c]->keys.size() > 1) {
                        if (nToExpand) (*nToExpand)++;
                        vSize.push_back(std::make_pair((int)ch[c]->keys.size(), &lNodes.front()));
                        lNodes.front().lit = lNodes.begin();
                    }
                }
            }
        };
        while (!finish) {
            int prevSize = (int)lNodes.size();
            lit = lNodes.begin();
            int nToExpand = 0;
            vSize.clear();
            while (lit != lNodes.end()) {
                if (lit->no_more) { lit++; continue; }
                Node n1, n2, n3, n4;
                lit->divide(n1, n2, n3, n4);
                push_children(n1, n2, n3, n4, &nToExpand);
                lit = lNodes.erase(lit);
            }
            if ((int)lNodes.size() >= N || (int)lNodes.size() == prevSize) {
                finish = true;
            } else if (((int)lNodes.size() + nToExpand * 3) > N) {
                while (!finish) {
                    prevSize = (int)lNodes.size();
                    std::vector<SizeNode> vPrev = vSize;
                    vSize.clear();
                    std::sort(vPrev.begin(), vPrev.end(), compare_nodes);
                    for (int j = (int)vPrev.size() - 1; j >= 0; j--) {
                        Node n1, n2, n3, n4;
                        vPrev[j].second->divide(n1, n2, n3, n4);
                        push_children(n1, n2, n3, n4, nullptr);
                        lNodes.erase(vPrev[j].second->lit);
                        if ((int)lNodes.size() >= N) break;
                    }
                    if ((int)lNodes.size() >= N || (int)lNodes.size() == prevSize) finish = true;
                }
            }
        }
        std::vector<KeyPoint> result;
        for (auto it = lNodes.begin(); it != lNodes.end(); it++) {
            const std::vector<KeyPoint>& k = it->keys;
            const KeyPoint* best = &k[0];
            float maxResponse = best->response;
            for (size_t i = 1; i < k.size(); i++)
                if (k[i].response > maxResponse) { best = &k[i]; maxResponse = k[i].response; }
            result.push_back(*best);
        }
        return result;
    }

    float ic_angle(const Image& im, float px, float py) const {
        int m01 = 0, m10 = 0;
        const uint8_t* center = im.px.data() + (size_t)cv_round(py) * im.w + cv_round(px);
        for (int u = -15; u <= 15; ++u) m10 += u * center[u];
        const int step = im.w;
        for (int v = 1; v <= 15; ++v) {
            int v_sum = 0;
            int d = umax[v];
            for (int u = -d; u <= d; ++u) {
                int vp = center[u + v * step], vm = center[u - v * step];
                v_sum += (vp - vm);
                m10 += u * (vp + vm);
            }
            m01 += v * v_sum;
        }
        return fast_atan2((float)m01, (float)m10);
    }

    void compute_keypoints(std::vector<std::vector<KeyPoint>>& all) {
        all.assign(nlevels, {});
        raw_keys.assign(nlevels, {});
        const float W = 35;
        for (int level = 0; level < nlevels; ++level) {
            const Image& im = pyramid[level];
            const int minBX = 16, minBY = 16;
            const int maxBX = im.w - 16, maxBY = im.h - 16;
            std::vector<KeyPoint> toDist;
            const float width = (float)(maxBX - minBX), height = (float)(maxBY - minBY);
            const int nCols = (int)(width / W), nRows = (int)(height / W);
            const int wCell = (int)std::ceil(width / nCols), hCell = (int)std::ceil(height / nRows);
            std::vector<KeyPoint> cell;
            for (int i = 0; i < nRows; i++) {
                const float iniY = (float)(minBY + i * hCell);
                float maxY = iniY + hCell + 6;
                if (iniY >= maxBY - 3) continue;
                if (maxY > maxBY) maxY = (float)maxBY;
                for (int j = 0; j < nCols; j++) {
                    const float iniX = (float)(minBX + j * wCell);
                    float maxX = iniX + wCell + 6;
                    if (iniX >= maxBX - 6) continue;
                    if (maxX > maxBX) maxX = (float)maxBX;
                    const int r0 = (int)iniY, r1 = (int)maxY, c0 = (int)iniX, c1 = (int)maxX;
                    const uint8_t* roi = im.px.data() + (size_t)r0 * im.w + c0;
                    fast9(roi, im.w, r1 - r0, c1 - c0, iniTh, cell);
                    if (cell.empty()) fast9(roi, im.w, r1 - r0, c1 - c0, minTh, cell);
                    for (KeyPoint kp : cell) {
                        kp.x += j * wCell;
                        kp.y += i * hCell;
                        toDist.push_back(kp);
                    }
                }
            }
            raw_keys[level] = toDist;
            std::vector<KeyPoint>& kps = all[level];
            kps = distribute_octtree(toDist, minBX, maxBX, minBY, maxBY, per_level[level]);
            const int scaledPatch = (int)(31 * scale[level]);
            for (KeyPoint& kp : kps) {
                kp.x += minBX; kp.y += minBY;
                kp.octave = level;
                kp.size = (float)scaledPatch;
            }
        }
        for (int level = 0; level < nlevels; ++level)
            for (KeyPoint& kp : all[level]) kp.angle = ic_angle(pyramid[level], kp.x, kp.y);
    }

    static void orb_descriptor(const KeyPoint& kpt, const Image& img, uint8_t* desc) {
        const float factorPI = (float)(M_PI / 180.f);
        float angle = (float)kpt.angle * factorPI;
        float a = (float)std::cos(angle), b = (float)std::sin(angle);   // float overloads -> cosf/sinf
        const uint8_t* center = img.px.data() + (size_t)cv_round(kpt.y) * img.w + cv_round(kpt.x);
        const int step = img.w;
        const signed char* pattern = ORBFE_BRIEF_PATTERN;
        auto val = [&](int idx) -> int {
            const float px = (float)pattern[2 * idx], py = (float)pattern[2 * idx + 1];
            return center[cv_round(px * b + py * a) * step + cv_round(px * a - py * b)];
        };
        for (int i = 0; i < 32; ++i) {
            int v = 0;
            for (int k = 0; k < 8; k++) {
                int t0 = val(16 * i + 2 * k), t1 = val(16 * i + 2 * k + 1);
                v |= (t0 < t1) << k;
            }
            desc[i] = (uint8_t)v;
        }
    }

    // operator() (ORBextractor.cc:1086-1168). Returns monoIndex, -1 on empty image.
    int extract(const Image& img, int lap0, int lap1, std::vector<KeyPoint>& out, std::vector<uint8_t>& desc) {
        if (img.w == 0 || img.h == 0) return -1;
        compute_pyramid(img);
        std::vector<std::vector<KeyPoint>> all;
        compute_keypoints(all);
        level_keys = all;
        int n = 0;
        for (auto& v : all) n += (int)v.size();
        out.assign(n, KeyPoint{});
        desc.assign((size_t)n * 32, 0);
        int monoIndex = 0, stereoIndex = n - 1;
        Image blurred;
        std::vector<uint8_t> d(32);
        for (int level = 0; level < nlevels; ++level) {
            std::vector<KeyPoint>& kps = all[level];
            if (kps.empty()) continue;
            gaussian_blur7(pyramid[level], blurred, blur_variant);
            const float s = scale[level];
            for (KeyPoint kp : kps) {
                orb_descriptor(kp, blurred, d.data());
                if (level != 0) { kp.x *= s; kp.y *= s; }
                int slot;
                if (kp.x >= lap0 && kp.x <= lap1) slot = stereoIndex--;
                else slot = monoIndex++;
                out[slot] = kp;
                memcpy(&desc[(size_t)slot * 32], d.data(), 32);
            }
        }
        return monoIndex;
    }
};

int hamming(const uint8_t* a, const uint8_t* b) {
    int dist = 0;
    for (int i = 0; i < 8; i++) {
        uint32_t v = 0, u = 0;
        memcpy(&v, a + 4 * i, 4); memcpy(&u, b + 4 * i, 4);
        v ^= u;
        v = v - ((v >> 1) & 0x55555555);
        v = (v & 0x33333333) + ((v >> 2) & 0x33333333);
        dist += (((v + (v >> 4)) & 0xF0F0F0F) * 0x1010101) >> 24;
    }
    return dist;
}

}  // namespace oracle

using oracle::Extractor;
using oracle::Image;
using oracle::KeyPoint;

// ================================ C API (ctypes) =============================================
extern "C" {

void* oro_create(int nfeatures, float scaleFactor, int nlevels, int iniTh, int minTh) {
    return new Extractor(nfeatures, scaleFactor, nlevels, iniTh, minTh);
}
void oro_destroy(void* h) { delete (Extractor*)h; }
void oro_set_model(void* h, int resize_simd_lanes, int blur_variant) {
    ((Extractor*)h)->resize_simd_lanes = resize_simd_lanes;
    ((Extractor*)h)->blur_variant = blur_variant;
}
void oro_level_info(void* h, float* scale, float* inv_scale, float* sigma2, float* inv_sigma2, int* per_level,
                    int* umax16) {
    Extractor* e = (Extractor*)h;
    for (int l = 0; l < e->nlevels; l++) {
        if (scale) scale[l] = e->scale[l];
        if (inv_scale) inv_scale[l] = e->inv_scale[l];
        if (sigma2) sigma2[l] = e->sigma2[l];
        if (inv_sigma2) inv_sigma2[l] = e->inv_sigma2[l];
        if (per_level) per_level[l] = e->per_level[l];
    }
    if (umax16) for (int v = 0; v < 16; v++) umax16[v] = e->umax[v];
}

// kps: cap x 7 floats? no: cap KeyPoint records (28 B each, cv::KeyPoint layout).
int oro_extract(void* h, const uint8_t* img, int w, int hgt, int stride, int lap0, int lap1, KeyPoint* kps,
                int cap, uint8_t* desc, int* n_out) {
    Extractor* e = (Extractor*)h;
    Image im;
    im.w = w; im.h = hgt; im.px.resize((size_t)w * hgt);
    for (int y = 0; y < hgt; y++) memcpy(&im.px[(size_t)y * w], img + (size_t)y * stride, w);
    std::vector<KeyPoint> out;
    std::vector<uint8_t> d;
    int mono = e->extract(im, lap0, lap1, out, d);
    int n = (int)out.size();
    *n_out = n;
    if (n > cap) return -4;
    if (n) { memcpy(kps, out.data(), sizeof(KeyPoint) * n); memcpy(desc, d.data(), (size_t)n * 32); }
    return mono;
}

int oro_pyramid_level(void* h, int level, uint8_t* dst, int cap, int* w, int* hgt) {
    Extractor* e = (Extractor*)h;
    const Image& im = e->pyramid[level];
    *w = im.w; *hgt = im.h;
    if (dst) {
        if ((int)im.px.size() > cap) return -4;
        memcpy(dst, im.px.data(), im.px.size());
    }
    return 0;
}
// debug: raw FAST keys (vToDistributeKeys, relative coords) or octree output (final per-level, pre-scale)
int oro_debug_keys(void* h, int level, int which, KeyPoint* out, int cap) {
    Extractor* e = (Extractor*)h;
    const std::vector<KeyPoint>& v = which == 0 ? e->raw_keys[level] : e->level_keys[level];
    int n = (int)v.size();
    if (out && n <= cap) memcpy(out, v.data(), sizeof(KeyPoint) * n);
    return n;
}

void oro_resize(const uint8_t* src, int sw, int sh, uint8_t* dst, int dw, int dh, int simd_lanes) {
    Image s; s.w = sw; s.h = sh; s.px.assign(src, src + (size_t)sw * sh);
    Image d;
    oracle::resize_linear(s, d, dw, dh, simd_lanes);
    memcpy(dst, d.px.data(), (size_t)dw * dh);
}
void oro_blur(const uint8_t* src, int w, int h, uint8_t* dst, int variant) {
    Image s; s.w = w; s.h = h; s.px.assign(src, src + (size_t)w * h);
    Image d;
    oracle::gaussian_blur7(s, d, variant);
    memcpy(dst, d.px.data(), (size_t)w * h);
}
int oro_fast(const uint8_t* roi, int step, int rows, int cols, int th, KeyPoint* out, int cap) {
    std::vector<KeyPoint> k;
    oracle::fast9(roi, step, rows, cols, th, k);
    int n = (int)k.size();
    if (out && n <= cap) memcpy(out, k.data(), sizeof(KeyPoint) * n);
    return n;
}
float oro_fast_atan2(float y, float x) { return oracle::fast_atan2(y, x); }
int oro_hamming(const uint8_t* a, const uint8_t* b) { return oracle::hamming(a, b); }

// Frame::ComputeStereoMatches (Frame.cc:811-981) for a rectified pinhole stereo pair extracted by
// hL / hR (pyramids of the last extract call). bf = mbf, fx = K(0,0). Outputs uRight[N], depth[N].
int oro_stereo_match(void* hL, void* hR, const KeyPoint* kL, const uint8_t* dL, int N, const KeyPoint* kR,
                     const uint8_t* dR, int Nr, float bf, float fx, float* uRight, float* depth) {
    Extractor* eL = (Extractor*)hL;
    Extractor* eR = (Extractor*)hR;
    for (int i = 0; i < N; i++) { uRight[i] = -1.0f; depth[i] = -1.0f; }
    const int TH_HIGH = 100, TH_LOW = 50;
    const int thOrbDist = (TH_HIGH + TH_LOW) / 2;
    const int nRows = eL->pyramid[0].h;
    std::vector<std::vector<size_t>> rows(nRows);
    for (int iR = 0; iR < Nr; iR++) {
        const float kpY = kR[iR].y;
        const float r = 2.0f * eL->scale[kR[iR].octave];
        const int maxr = (int)std::ceil(kpY + r), minr = (int)std::floor(kpY - r);
        for (int yi = minr; yi <= maxr; yi++)
            if (yi >= 0 && yi < nRows) rows[yi].push_back(iR);   // reference: unguarded (never hit for kp.y>=19)
    }
    // The reference reads the member `mb` here BEFORE the Frame ctor assigns it (Frame.cc:141 vs :174),
    // i.e. an indeterminate value; we use the intended mb = mbf/fx (maxD = fx), see DESIGN.md.
    const float mb = bf / fx;
    const float minZ = mb, minD = 0, maxD = bf / minZ;
    std::vector<std::pair<int, int>> distIdx;
    for (int iL = 0; iL < N; iL++) {
        const KeyPoint& kpL = kL[iL];
        const int levelL = kpL.octave;
        const float vL = kpL.y, uL = kpL.x;
        const std::vector<size_t>& cand = rows[(size_t)vL];
        if (cand.empty()) continue;
        const float minU = uL - maxD, maxU = uL - minD;
        if (maxU < 0) continue;
        int bestDist = TH_HIGH;
        size_t bestIdxR = 0;
        for (size_t iC = 0; iC < cand.size(); iC++) {
            const size_t iR = cand[iC];
            const KeyPoint& kpR = kR[iR];
            if (kpR.octave < levelL - 1 || kpR.octave > levelL + 1) continue;
            const float uR = kpR.x;
            if (uR >= minU && uR <= maxU) {
                const int dist = oracle::hamming(dL + (size_t)iL * 32, dR + iR * 32);
                if (dist < bestDist) { bestDist = dist; bestIdxR = iR; }
            }
        }
        if (bestDist < thOrbDist) {
            const float uR0 = kR[bestIdxR].x;
            const float scaleFactor = eL->inv_scale[kpL.octave];
            const float scaleduL = std::round(kpL.x * scaleFactor);
            const float scaledvL = std::round(kpL.y * scaleFactor);
            const float scaleduR0 = std::round(uR0 * scaleFactor);
            const int w = 5, L = 5;
            const Image& IL = eL->pyramid[kpL.octave];
            const Image& IRimg = eR->pyramid[kpL.octave];
            int bestD = INT32_MAX;
            int bestincR = 0;
            float vDists[11];
            const float iniu = scaleduR0 + L - w;
            const float endu = scaleduR0 + L + w + 1;
            if (iniu < 0 || endu >= IRimg.w) continue;
            const int r0 = (int)(scaledvL - w), c0L = (int)(scaleduL - w);
            for (int incR = -L; incR <= L; incR++) {
                const int c0R = (int)(scaleduR0 + incR - w);
                double s = 0;
                int si = 0;
                for (int yy = 0; yy < 2 * w + 1; yy++)
                    for (int xx = 0; xx < 2 * w + 1; xx++)
                        si += std::abs((int)IL.at(c0L + xx, r0 + yy) - (int)IRimg.at(c0R + xx, r0 + yy));
                s = si;
                float dist = (float)s;
                if (dist < bestD) { bestD = (int)dist; bestincR = incR; }
                vDists[L + incR] = dist;
            }
            if (bestincR == -L || bestincR == L) continue;
            const float dist1 = vDists[L + bestincR - 1], dist2 = vDists[L + bestincR], dist3 = vDists[L + bestincR + 1];
            const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
            if (deltaR < -1 || deltaR > 1) continue;
            float bestuR = eL->scale[kpL.octave] * ((float)scaleduR0 + (float)bestincR + deltaR);
            float disparity = (uL - bestuR);
            if (disparity >= minD && disparity < maxD) {
                if (disparity <= 0) { disparity = 0.01; bestuR = uL - 0.01; }
                depth[iL] = bf / disparity;
                uRight[iL] = bestuR;
                distIdx.push_back(std::make_pair(bestD, iL));
            }
        }
    }
    if (distIdx.empty()) return 0;   // the reference indexes vDistIdx[size/2] unguarded here
    std::sort(distIdx.begin(), distIdx.end());
    const float median = (float)distIdx[distIdx.size() / 2].first;
    const float thDist = 1.5f * 1.4f * median;
    for (int i = (int)distIdx.size() - 1; i >= 0; i--) {
        if (distIdx[i].first < thDist) break;
        uRight[distIdx[i].second] = -1;
        depth[distIdx[i].second] = -1;
    }
    return (int)distIdx.size();
}

// Throughput helper for the CPU baseline: extract nimg images with nthreads threads, one image
// per task (independent Extractor instances, like the reference's per-camera extractors).
double oro_bench_extract(const uint8_t* imgs, int nimg, int w, int h, int nfeatures, float sf, int nlevels,
                         int ini, int mn, int nthreads, int* total_kps) {
    std::vector<std::thread> th;
    std::vector<int> counts(nthreads, 0);
    for (int t = 0; t < nthreads; t++) {
        th.emplace_back([&, t]() {
            Extractor e(nfeatures, sf, nlevels, ini, mn);
            std::vector<KeyPoint> out;
            std::vector<uint8_t> d;
            for (int i = t; i < nimg; i += nthreads) {
                Image im; im.w = w; im.h = h;
                im.px.assign(imgs + (size_t)i * w * h, imgs + (size_t)(i + 1) * w * h);
                e.extract(im, 0, 0, out, d);
                counts[t] += (int)out.size();
            }
        });
    }
    for (auto& t : th) t.join();
    int tot = 0;
    for (int c : counts) tot += c;
    if (total_kps) *total_kps = tot;
    return 0.0;
}

// std::sort of u64 values by their high 32 bits (the shape of DistributeOctTree's
// compareNodes sort, ORBextractor.cc:700) — checker for the device block-parallel replica.
void oro_std_sort_u64_hi(uint64_t* a, int n) {
    std::sort(a, a + n, [](uint64_t x, uint64_t y) { return (x >> 32) < (y >> 32); });
}

// CPU baseline for the bench's workload (config 2): per frame extract(L) + extract(R) on two
// threads (Frame.cc:122-125) then ComputeStereoMatches, with `nthreads` frames in flight.
// Returns the total number of stereo matches (so the work cannot be optimised away).
long oro_bench_stereo(const uint8_t* L, const uint8_t* R, int nframes, int w, int h, int nfeatures, float sf,
                      int nlevels, int ini, int mn, float bf, float fx, int nthreads) {
    std::vector<std::thread> th;
    std::vector<long> tot(nthreads, 0);
    for (int t = 0; t < nthreads; t++) {
        th.emplace_back([&, t]() {
            Extractor el(nfeatures, sf, nlevels, ini, mn), er(nfeatures, sf, nlevels, ini, mn);
            std::vector<KeyPoint> kl, kr;
            std::vector<uint8_t> dl, dr;
            std::vector<float> ur, dp;
            for (int f = t; f < nframes; f += nthreads) {
                Image a, b;
                a.w = b.w = w; a.h = b.h = h;
                a.px.assign(L + (size_t)f * w * h, L + (size_t)(f + 1) * w * h);
                b.px.assign(R + (size_t)f * w * h, R + (size_t)(f + 1) * w * h);
                el.extract(a, 0, 0, kl, dl);
                er.extract(b, 0, 0, kr, dr);
                ur.resize(kl.size() + 1); dp.resize(kl.size() + 1);
                tot[t] += oro_stereo_match(&el, &er, kl.data(), dl.data(), (int)kl.size(), kr.data(), dr.data(),
                                           (int)kr.size(), bf, fx, ur.data(), dp.data());
            }
        });
    }
    for (auto& x : th) x.join();
    long s = 0;
    for (long v : tot) s += v;
    return s;
}

// CPU latency modes of SURVEY §8(d), one frame at a time on the calling thread:
//   lr_split = 0: extract(L), extract(R), ComputeStereoMatches, all on one thread (frame-serial);
//   lr_split = 1: the reference's split (Frame.cc:122-125): two std::threads per frame run
//                 ExtractORB(left) / ExtractORB(right) on separate extractor instances, joined, then
//                 ComputeStereoMatches on the calling thread.
// *ms_per_frame = mean wall time per frame. Returns the total stereo matches.
long oro_bench_stereo_latency(const uint8_t* L, const uint8_t* R, int nframes, int w, int h, int nfeatures,
                              float sf, int nlevels, int ini, int mn, float bf, float fx, int lr_split,
                              double* ms_per_frame) {
    Extractor el(nfeatures, sf, nlevels, ini, mn), er(nfeatures, sf, nlevels, ini, mn);
    std::vector<KeyPoint> kl, kr;
    std::vector<uint8_t> dl, dr;
    std::vector<float> ur, dp;
    long tot = 0;
    const auto t0 = std::chrono::steady_clock::now();
    for (int f = 0; f < nframes; f++) {
        Image a, b;
        a.w = b.w = w; a.h = b.h = h;
        a.px.assign(L + (size_t)f * w * h, L + (size_t)(f + 1) * w * h);
        b.px.assign(R + (size_t)f * w * h, R + (size_t)(f + 1) * w * h);
        if (lr_split) {
            std::thread tl([&]() { el.extract(a, 0, 0, kl, dl); });
            std::thread tr([&]() { er.extract(b, 0, 0, kr, dr); });
            tl.join();
            tr.join();
        } else {
            el.extract(a, 0, 0, kl, dl);
            er.extract(b, 0, 0, kr, dr);
        }
        ur.resize(kl.size() + 1); dp.resize(kl.size() + 1);
        tot += oro_stereo_match(&el, &er, kl.data(), dl.data(), (int)kl.size(), kr.data(), dr.data(), (int)kr.size(),
                                bf, fx, ur.data(), dp.data());
    }
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (ms_per_frame) *ms_per_frame = nframes > 0 ? ms / nframes : 0.0;
    return tot;
}

// Monocular frames (config 1): ORBextractor::operator() with the mono Frame's vLappingArea
// (Frame.cc:311 passes {0, 1000}), `nthreads` frames in flight (1 = frame-serial latency).
// Returns the total keypoints; *ms_total = wall time.
long oro_bench_mono(const uint8_t* imgs, int nimg, int w, int h, int nfeatures, float sf, int nlevels, int ini, int mn,
                    int lap0, int lap1, int nthreads, double* ms_total) {
    std::vector<std::thread> th;
    std::vector<long> counts(nthreads, 0);
    const auto t0 = std::chrono::steady_clock::now();
    for (int t = 0; t < nthreads; t++) {
        th.emplace_back([&, t]() {
            Extractor e(nfeatures, sf, nlevels, ini, mn);
            std::vector<KeyPoint> out;
            std::vector<uint8_t> d;
            for (int i = t; i < nimg; i += nthreads) {
                Image im; im.w = w; im.h = h;
                im.px.assign(imgs + (size_t)i * w * h, imgs + (size_t)(i + 1) * w * h);
                e.extract(im, lap0, lap1, out, d);
                counts[t] += (long)out.size();
            }
        });
    }
    for (auto& t : th) t.join();
    if (ms_total) *ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    long tot = 0;
    for (long c : counts) tot += c;
    return tot;
}

}  // extern "C"
