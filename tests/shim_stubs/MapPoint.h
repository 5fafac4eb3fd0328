// TEST INFRASTRUCTURE: the ORB_SLAM3::MapPoint members the shim reads / writes (include/MapPoint.h),
// plus GetMinDistance / GetMaxDistance / SetDescriptor, which INTEGRATION.md §2 adds.
#pragma once
#include <map>
#include <tuple>
#include "stub_types.h"
namespace ORB_SLAM3 {
class MapPoint {
public:
    Eigen::Vector3f GetWorldPos();
    Eigen::Vector3f GetNormal();
    std::map<KeyFrame*, std::tuple<int, int>> GetObservations();
    int Observations();
    std::tuple<int, int> GetIndexInKeyFrame(KeyFrame* pKF);
    bool IsInKeyFrame(KeyFrame* pKF);
    void AddObservation(KeyFrame* pKF, int idx);
    void Replace(MapPoint* pMP);
    bool isBad();
    void IncreaseVisible(int n = 1);
    void ComputeDistinctiveDescriptors();
    cv::Mat GetDescriptor();
    void SetDescriptor(const uint8_t* desc32);
    float GetMinDistanceInvariance();
    float GetMaxDistanceInvariance();
    float GetMinDistance();
    float GetMaxDistance();
    int PredictScale(const float& currentDist, Frame* pF);
    long unsigned int mnId;
    float mTrackProjX, mTrackProjY, mTrackDepth, mTrackDepthR, mTrackProjXR, mTrackProjYR;
    bool mbTrackInView, mbTrackInViewR;
    int mnTrackScaleLevel, mnTrackScaleLevelR;
    float mTrackViewCos, mTrackViewCosR;
    long unsigned int mnLastFrameSeen;
};
}  // namespace ORB_SLAM3
