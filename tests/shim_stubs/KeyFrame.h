// TEST INFRASTRUCTURE: the ORB_SLAM3::KeyFrame members the matcher shims read (include/KeyFrame.h).
#pragma once
#include <set>
#include <vector>
#include "stub_types.h"
namespace ORB_SLAM3 {
class KeyFrame {
public:
    Sophus::SE3f GetPose();
    Sophus::SE3f GetPoseInverse();
    Sophus::SE3f GetRightPose();
    Sophus::SE3f GetRightPoseInverse();
    Eigen::Vector3f GetCameraCenter();
    Eigen::Vector3f GetRightCameraCenter();
    std::vector<MapPoint*> GetMapPointMatches();
    std::set<MapPoint*> GetMapPoints();
    MapPoint* GetMapPoint(const size_t& idx);
    void AddMapPoint(MapPoint* pMP, const size_t& idx);
    bool isBad();
    const int N;
    int NLeft;
    const std::vector<cv::KeyPoint> mvKeys, mvKeysUn;
    const std::vector<cv::KeyPoint> mvKeysRight;
    const std::vector<float> mvuRight;
    const cv::Mat mDescriptors;
    DBoW2::FeatureVector mFeatVec;
    const int mnScaleLevels;
    const float mfLogScaleFactor;
    const std::vector<float> mvScaleFactors, mvLevelSigma2, mvInvLevelSigma2;
    const int mnMinX, mnMinY, mnMaxX, mnMaxY;
    const float fx, fy, cx, cy, mbf;
    std::vector<int> mvLeftToRightMatch, mvRightToLeftMatch;
    GeometricCamera *mpCamera, *mpCamera2;
};
}  // namespace ORB_SLAM3
