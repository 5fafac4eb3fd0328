// Frame-side drop-in on top of liborbfe.so (include/orbfe.h): the stereo Frame's extraction +
// ComputeStereoMatches in one library call, and ComputeStereoMatches itself (orb_slam3/src/Frame.cc).
// Built inside the ORB-SLAM3 tree with OpenCV 4.2 / Eigen / Sophus; this repository compiles it with
// -fsyntax-only against stand-in headers (tests/shim_stubs/, tests/test_shim_compile.py), so a drift
// between include/orbfe.h and this file fails a test. INTEGRATION.md §2 lists the Frame.h / Frame.cc
// edits: the member declarations below, the original ComputeStereoMatches body renamed
// ComputeStereoMatches_cpu, and the constructor's six-line change:
//
//   Frame::Frame(imLeft, imRight, ...) (Frame.cc:101-197), lines 122-141 become
//       const bool fused = ExtractStereoOrbfe(imLeft, imRight);   // ExtractORB x 2 + ComputeStereoMatches
//       if (!fused) { thread threadLeft(...); thread threadRight(...); threadLeft.join(); threadRight.join(); }
//       N = mvKeys.size();
//       if (mvKeys.empty()) return;
//       UndistortKeyPoints();
//       if (!fused) ComputeStereoMatches();
#include "Frame.h"

#include <cstdio>
#include <mutex>
#include <set>
#include <string>

#include <orbfe.h>

#include "ORBextractor.h"
#include "orbfe_glue.h"

using namespace std;

namespace ORB_SLAM3 {

// Referenced by shim/ORBextractor_orbfe.cc: an ORBextractor.cc replaced without this file (the
// ComputeStereoMatches below, the only reader of mvImagePyramid in the reference, Frame.cc:818-923)
// fails to link instead of leaving Frame.cc reading the pyramid the shim no longer fills.
extern const int kOrbfeStereoRerouted = 1;

namespace {

// One log line per (call site, error code), as the matcher shims.
void log_fallback(int rc, const char* what) {
    static std::mutex mu;
    static std::set<std::pair<std::string, int>> seen;
    bool first;
    {
        std::lock_guard<std::mutex> lk(mu);
        first = seen.emplace(what, rc).second;
    }
    if (first) fprintf(stderr, "[orbfe] %s returned %d; running the CPU implementation\n", what, rc);
}

// A cv::Mat descriptor sink for orbfe_glue::frame_stereo: a continuous cap x 32 CV_8U block, cut to
// its first n rows (a row-range header: no copy).
struct MatRows {
    cv::Mat m;
    uint8_t* rows(int cap) {
        m.create(cap, 32, CV_8U);
        return m.data;
    }
    void keep(int n) { m = n > 0 ? m.rowRange(0, n) : cv::Mat(); }
};

orbfe_extractor* handle_of(ORBextractor* e) { return static_cast<orbfe_extractor*>(e->OrbfeHandle()); }

}  // namespace

// Frame.cc:122-141 in one call (the members INTEGRATION.md §2 adds to Frame.h). Fills mvKeys,
// mvKeysRight, mDescriptors, mDescriptorsRight, mvuRight and mvDepth exactly as the two ExtractORB
// threads and ComputeStereoMatches do, with mb = mbf / fx taken from mK (the reference's body reads
// the member mb before the constructor assigns it, Frame.cc:141 vs :174). Returns false
// after one logged line when the library cannot (no device, a capacity limit): the constructor then
// runs its original two threads and ComputeStereoMatches().
bool Frame::ExtractStereoOrbfe(const cv::Mat& imLeft, const cv::Mat& imRight) {
    if (imLeft.type() != CV_8UC1 || imRight.type() != CV_8UC1 || imLeft.size() != imRight.size() ||
        imLeft.step != imRight.step)
        return false;
    MatRows dl, dr;
    const float fxK = mK.at<float>(0, 0);
    const int ns = orbfe_glue::frame_stereo(handle_of(mpORBextractorLeft), handle_of(mpORBextractorRight), imLeft.data,
                                            imRight.data, imLeft.cols, imLeft.rows, (int)imLeft.step, mbf, fxK, mvKeys,
                                            dl, &monoLeft, mvKeysRight, dr, &monoRight, mvuRight, mvDepth);
    if (ns < 0) {
        log_fallback(ns, "orbfe_frame_stereo");
        return false;
    }
    mDescriptors = dl.m;
    mDescriptorsRight = dr.m;
    // Tracking's searches on this frame read it in HBM while the left handle still holds it
    // (orbfe_frame_device_view); rectified stereo only: mvKeysUn == mvKeys (no distortion)
    mnOrbfeFrameId = mDistCoef.at<float>(0) == 0.f ? orbfe_extractor_frame_id(handle_of(mpORBextractorLeft)) : 0;
    mpORBextractorLeft->mvImagePyramid.clear();
    mpORBextractorRight->mvImagePyramid.clear();
    return true;
}

// Frame::ComputeStereoMatches (Frame.cc:811-981) over the last extraction of both handles (the
// separate-thread path: ExtractORB x 2, then this). The original body stays in Frame.cc as
// ComputeStereoMatches_cpu: it runs, after the host pyramids are materialised, when the library
// refuses (e.g. more keypoints per image than k_stereo stages in LDS).
void Frame::ComputeStereoMatches() {
    mvuRight = vector<float>(N, -1.0f);
    mvDepth = vector<float>(N, -1.0f);
    if (N == 0) return;
    const int rc = orbfe_stereo_match(handle_of(mpORBextractorLeft), handle_of(mpORBextractorRight), mbf,
                                      mK.at<float>(0, 0), mvuRight.data(), mvDepth.data());
    if (rc < 0) {
        log_fallback(rc, "orbfe_stereo_match");
        mpORBextractorLeft->MaterialisePyramid();
        mpORBextractorRight->MaterialisePyramid();
        ComputeStereoMatches_cpu();
    }
}

}  // namespace ORB_SLAM3
