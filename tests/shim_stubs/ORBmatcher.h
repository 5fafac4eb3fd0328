// TEST INFRASTRUCTURE: ORB_SLAM3::ORBmatcher as include/ORBmatcher.h declares it, plus the *_cpu
// renames of the replaced bodies, which INTEGRATION.md §2 adds.
#pragma once
#include <set>
#include <utility>
#include <vector>
#include "stub_types.h"
#include "Frame.h"
#include "KeyFrame.h"
#include "MapPoint.h"
namespace ORB_SLAM3 {
class ORBmatcher {
public:
    ORBmatcher(float nnratio = 0.6, bool checkOri = true);
    static int DescriptorDistance(const cv::Mat& a, const cv::Mat& b);
    int SearchByProjection(Frame& F, const std::vector<MapPoint*>& vpMapPoints, const float th = 3,
                           const bool bFarPoints = false, const float thFarPoints = 50.0f);
    int SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, const float th, const bool bMono);
    int SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF, const std::set<MapPoint*>& sAlreadyFound,
                           const float th, const int ORBdist);
    int SearchByProjection(KeyFrame* pKF, Sophus::Sim3<float>& Scw, const std::vector<MapPoint*>& vpPoints,
                           std::vector<MapPoint*>& vpMatched, int th, float ratioHamming = 1.0);
    int SearchByBoW(KeyFrame* pKF, Frame& F, std::vector<MapPoint*>& vpMapPointMatches);
    int SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2, std::vector<MapPoint*>& vpMatches12);
    int SearchForInitialization(Frame& F1, Frame& F2, std::vector<cv::Point2f>& vbPrevMatched,
                                std::vector<int>& vnMatches12, int windowSize = 10);
    int SearchForTriangulation(KeyFrame* pKF1, KeyFrame* pKF2, std::vector<std::pair<size_t, size_t>>& vMatchedPairs,
                               const bool bOnlyStereo, const bool bCoarse = false);
    int SearchBySim3(KeyFrame* pKF1, KeyFrame* pKF2, std::vector<MapPoint*>& vpMatches12, const Sophus::Sim3f& S12,
                     const float th);
    int Fuse(KeyFrame* pKF, const std::vector<MapPoint*>& vpMapPoints, const float th = 3.0, const bool bRight = false);
    int Fuse(KeyFrame* pKF, Sophus::Sim3f& Scw, const std::vector<MapPoint*>& vpPoints, float th,
             std::vector<MapPoint*>& vpReplacePoint);
    // the original bodies, renamed
    int SearchByProjection_cpu(Frame& F, const std::vector<MapPoint*>& vpMapPoints, const float th,
                               const bool bFarPoints, const float thFarPoints);
    int SearchByProjection_cpu(Frame& CurrentFrame, const Frame& LastFrame, const float th, const bool bMono);
    int SearchByProjection_cpu(Frame& CurrentFrame, KeyFrame* pKF, const std::set<MapPoint*>& sAlreadyFound,
                               const float th, const int ORBdist);
    int SearchByProjection_cpu(KeyFrame* pKF, Sophus::Sim3<float>& Scw, const std::vector<MapPoint*>& vpPoints,
                               std::vector<MapPoint*>& vpMatched, int th, float ratioHamming);
    int SearchByBoW_cpu(KeyFrame* pKF, Frame& F, std::vector<MapPoint*>& vpMapPointMatches);
    int SearchByBoW_cpu(KeyFrame* pKF1, KeyFrame* pKF2, std::vector<MapPoint*>& vpMatches12);
    int SearchForInitialization_cpu(Frame& F1, Frame& F2, std::vector<cv::Point2f>& vbPrevMatched,
                                    std::vector<int>& vnMatches12, int windowSize);
    int SearchForTriangulation_cpu(KeyFrame* pKF1, KeyFrame* pKF2,
                                   std::vector<std::pair<size_t, size_t>>& vMatchedPairs, const bool bOnlyStereo,
                                   const bool bCoarse);
    int SearchBySim3_cpu(KeyFrame* pKF1, KeyFrame* pKF2, std::vector<MapPoint*>& vpMatches12, const Sophus::Sim3f& S12,
                         const float th);
    int Fuse_cpu(KeyFrame* pKF, const std::vector<MapPoint*>& vpMapPoints, const float th, const bool bRight);
    int Fuse_cpu(KeyFrame* pKF, Sophus::Sim3f& Scw, const std::vector<MapPoint*>& vpPoints, float th,
                 std::vector<MapPoint*>& vpReplacePoint);

protected:
    float mfNNratio;
    bool mbCheckOrientation;
};
}  // namespace ORB_SLAM3
