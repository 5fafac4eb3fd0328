// TEST INFRASTRUCTURE: the LocalMapping fields Tracking::SearchLocalPoints reads (include/LocalMapping.h).
#pragma once
#include "stub_types.h"
namespace ORB_SLAM3 {
class LocalMapping {
public:
    bool mbFarPoints;
    float mThFarPoints;
};
}  // namespace ORB_SLAM3
