// TEST INFRASTRUCTURE: the Atlas / Map queries Tracking::SearchLocalPoints makes (include/Atlas.h, Map.h).
#pragma once
#include "stub_types.h"
namespace ORB_SLAM3 {
class Map {
public:
    bool GetIniertialBA2();
};
class Atlas {
public:
    bool isImuInitialized();
    Map* GetCurrentMap();
};
}  // namespace ORB_SLAM3
