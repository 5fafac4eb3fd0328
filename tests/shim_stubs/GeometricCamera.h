// TEST INFRASTRUCTURE: ORB_SLAM3::GeometricCamera (include/CameraModels/GeometricCamera.h) for the
// shim's -fsyntax-only compile; declared in stub_types.h with the other stand-ins.
#pragma once
#include "stub_types.h"
