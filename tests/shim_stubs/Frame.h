// TEST INFRASTRUCTURE: the ORB_SLAM3::Frame members the shims read / write (include/Frame.h), plus
// ExtractStereoOrbfe and ComputeStereoMatches_cpu, which INTEGRATION.md §2 adds.
#pragma once
#include <map>
#include <vector>
#include "stub_types.h"
namespace ORB_SLAM3 {
class Frame {
public:
    void ExtractORB(int flag, const cv::Mat& im, const int x0, const int x1);
    bool ExtractStereoOrbfe(const cv::Mat& imLeft, const cv::Mat& imRight);
    void ComputeStereoMatches();
    void ComputeStereoMatches_cpu();
    bool isInFrustum(MapPoint* pMP, float viewingCosLimit);
    Sophus::SE3f GetRelativePoseTrl();
    Sophus::SE3f GetRelativePoseTlr();
    Eigen::Vector3f GetCameraCenter();
    Eigen::Matrix3f GetRotationInverse();
    Sophus::SE3<float> GetPose() const;
    ORBextractor *mpORBextractorLeft, *mpORBextractorRight;
    cv::Mat mK;
    cv::Mat mDistCoef;
    uint64_t mnOrbfeFrameId = 0;   // orbfe_extractor_frame_id after ExtractStereoOrbfe
    float mbf, mb;
    int N;
    std::vector<cv::KeyPoint> mvKeys, mvKeysRight, mvKeysUn;
    std::vector<float> mvuRight, mvDepth;
    DBoW2::FeatureVector mFeatVec;
    cv::Mat mDescriptors, mDescriptorsRight;
    std::vector<MapPoint*> mvpMapPoints;
    std::vector<bool> mvbOutlier;
    long unsigned int mnId;
    int mnScaleLevels;
    float mfLogScaleFactor;
    std::vector<float> mvScaleFactors;
    static float mnMinX, mnMaxX, mnMinY, mnMaxY;
    std::map<long unsigned int, cv::Point2f> mmProjectPoints;
    GeometricCamera *mpCamera, *mpCamera2;
    int Nleft, Nright;
    int monoLeft, monoRight;
    std::vector<int> mvLeftToRightMatch, mvRightToLeftMatch;
};
}  // namespace ORB_SLAM3
