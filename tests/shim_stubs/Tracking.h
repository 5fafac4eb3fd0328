// TEST INFRASTRUCTURE: the ORB_SLAM3::Tracking members SearchLocalPoints uses (include/Tracking.h), plus
// the SearchLocalPoints_cpu rename INTEGRATION.md §2 adds.
#pragma once
#include <vector>
#include "stub_types.h"
#include "Frame.h"
namespace ORB_SLAM3 {
class Atlas;
class LocalMapping;
class Tracking {
public:
    enum eTrackingState { SYSTEM_NOT_READY = -1, NO_IMAGES_YET = 0, NOT_INITIALIZED = 1, OK = 2, RECENTLY_LOST = 3,
                          LOST = 4, OK_KLT = 5 };
    eTrackingState mState;
    int mSensor;
    Frame mCurrentFrame;

protected:
    void SearchLocalPoints();
    void SearchLocalPoints_cpu();
    LocalMapping* mpLocalMapper;
    std::vector<MapPoint*> mvpLocalMapPoints;
    Atlas* mpAtlas;
    unsigned int mnLastRelocFrameId;
};
}  // namespace ORB_SLAM3
