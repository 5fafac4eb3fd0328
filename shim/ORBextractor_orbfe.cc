// Drop-in replacement for orb_slam3/src/ORBextractor.cc on top of liborbfe.so (include/orbfe.h).
// Built inside the ORB-SLAM3 tree (OpenCV 4.2 and the ORB-SLAM3 headers); this repository compiles
// it with -fsyntax-only against stand-in headers (tests/shim_stubs/, tests/test_shim_compile.py).
// ORBextractor.h keeps its public interface; the header changes are one private member
//     void* mpOrbfe = nullptr;   // orbfe_extractor*
// its public accessor void* OrbfeHandle() const { return mpOrbfe; } (the Frame shim's handle), a
// non-inline destructor declaration and void MaterialisePyramid().
#include "ORBextractor.h"

#include <cassert>
#include <cstring>
#include <stdexcept>
#include <string>

#include <orbfe.h>

using namespace cv;
using namespace std;

namespace ORB_SLAM3 {

// Defined by shim/Frame_orbfe.cc next to the ComputeStereoMatches replacement: the only
// reader of mvImagePyramid in the reference (Frame.cc:818-923), which this file no longer fills.
// Replacing ORBextractor.cc without that rerouting is a link error, not a silent wrong read.
extern const int kOrbfeStereoRerouted;

static_assert(sizeof(cv::KeyPoint) == sizeof(orbfe_keypoint), "cv::KeyPoint layout (28 B) expected");

// ORBextractor::ORBextractor (ORBextractor.cc:409-469): tables come from the library, which
// derives them with the reference's float/double expressions.
ORBextractor::ORBextractor(int _nfeatures, float _scaleFactor, int _nlevels, int _iniThFAST, int _minThFAST)
    : nfeatures(_nfeatures), scaleFactor(_scaleFactor), nlevels(_nlevels), iniThFAST(_iniThFAST),
      minThFAST(_minThFAST) {
    orbfe_extractor* h = nullptr;
    if (orbfe_extractor_create(nfeatures, _scaleFactor, nlevels, iniThFAST, minThFAST, &h) != ORBFE_OK)
        throw std::runtime_error("orbfe_extractor_create failed (no HIP device?)");
    mpOrbfe = h;
    if (kOrbfeStereoRerouted != 1) throw std::logic_error("ComputeStereoMatches is not routed to orbfe_stereo_match");
    mvScaleFactor.resize(nlevels);
    mvInvScaleFactor.resize(nlevels);
    mvLevelSigma2.resize(nlevels);
    mvInvLevelSigma2.resize(nlevels);
    mnFeaturesPerLevel.resize(nlevels);
    orbfe_extractor_scale_info(h, mvScaleFactor.data(), mvInvScaleFactor.data(), mvLevelSigma2.data(),
                               mvInvLevelSigma2.data(), mnFeaturesPerLevel.data());
}

ORBextractor::~ORBextractor() { orbfe_extractor_destroy(static_cast<orbfe_extractor*>(mpOrbfe)); }

// int ORBextractor::operator() (ORBextractor.cc:1086-1168)
int ORBextractor::operator()(InputArray _image, InputArray _mask, vector<KeyPoint>& _keypoints,
                             OutputArray _descriptors, std::vector<int>& vLappingArea) {
    (void)_mask;   // ignored, as in the reference
    if (_image.empty()) return -1;
    Mat image = _image.getMat();
    assert(image.type() == CV_8UC1);
    orbfe_extractor* h = static_cast<orbfe_extractor*>(mpOrbfe);
    const int cap = orbfe_extractor_capacity(h, image.cols, image.rows);
    if (cap < 0) throw std::runtime_error("orbfe_extractor_capacity failed");
    _keypoints.resize(cap);
    Mat desc(cap, 32, CV_8U);
    int n = 0;
    const int monoIndex = orbfe_extract(h, image.data, image.cols, image.rows, (int)image.step, vLappingArea[0],
                                        vLappingArea[1], reinterpret_cast<orbfe_keypoint*>(_keypoints.data()),
                                        desc.data, cap, &n);
    if (monoIndex == ORBFE_E_EMPTY) { _keypoints.clear(); return -1; }
    if (monoIndex < 0)   // device error or a capacity limit: no CPU extractor is linked to fall back to
        throw std::runtime_error("orbfe_extract failed with code " + std::to_string(monoIndex));
    _keypoints.resize(n);
    if (n == 0) {
        _descriptors.release();
    } else {
        _descriptors.create(n, 32, CV_8U);
        desc.rowRange(0, n).copyTo(_descriptors.getMat());
    }
    // mvImagePyramid is read only by Frame::ComputeStereoMatches, which the Frame shim routes to
    // orbfe_stereo_match (kOrbfeStereoRerouted above makes that a link-time requirement); call
    // MaterialisePyramid() when host levels are needed elsewhere (the CPU stereo fallback does).
    mvImagePyramid.clear();
    return monoIndex;
}

// Optional host copy of the pyramid of the last call (1.1 MB D2H at 752x480).
void ORBextractor::MaterialisePyramid() {
    orbfe_extractor* h = static_cast<orbfe_extractor*>(mpOrbfe);
    mvImagePyramid.resize(nlevels);
    for (int l = 0; l < nlevels; l++) {
        int w = 0, hh = 0;
        orbfe_pyramid_level(h, 0, l, nullptr, 0, &w, &hh);
        mvImagePyramid[l].create(hh, w, CV_8U);
        orbfe_pyramid_level(h, 0, l, mvImagePyramid[l].data, (int)mvImagePyramid[l].step, &w, &hh);
    }
}

}  // namespace ORB_SLAM3
