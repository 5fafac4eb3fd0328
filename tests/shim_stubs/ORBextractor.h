// TEST INFRASTRUCTURE: ORB_SLAM3::ORBextractor as include/ORBextractor.h declares it, plus the members
// INTEGRATION.md §2 adds (mpOrbfe, OrbfeHandle, MaterialisePyramid, non-inline destructor).
#pragma once
#include <vector>
#include "stub_types.h"
namespace ORB_SLAM3 {
class ORBextractor {
public:
    ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST);
    ~ORBextractor();
    int operator()(cv::InputArray _image, cv::InputArray _mask, std::vector<cv::KeyPoint>& _keypoints,
                   cv::OutputArray _descriptors, std::vector<int>& vLappingArea);
    int inline GetLevels() { return nlevels; }
    void* OrbfeHandle() const { return mpOrbfe; }
    void MaterialisePyramid();
    std::vector<cv::Mat> mvImagePyramid;

protected:
    std::vector<int> mnFeaturesPerLevel;
    int nfeatures;
    double scaleFactor;
    int nlevels;
    int iniThFAST;
    int minThFAST;
    std::vector<float> mvScaleFactor, mvInvScaleFactor, mvLevelSigma2, mvInvLevelSigma2;
    void* mpOrbfe = nullptr;
};
}  // namespace ORB_SLAM3
