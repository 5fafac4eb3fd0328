// ORB-SLAM3 / Sophus types -> include/orbfe.h records, shared by the shim files that need them (built
// inside the ORB-SLAM3 tree; tests/test_shim_compile.py compiles them against stand-in headers).
#pragma once
#include <cstring>

#include <orbfe.h>

#include "GeometricCamera.h"

namespace ORB_SLAM3 {
namespace orbfe_shim {

// a Sophus pose as the library applies it (include/orbfe.h orbfe_pose: sophus/so3.hpp:358-367)
inline orbfe_pose pose_of(const Sophus::SE3f& T) {
    orbfe_pose p;
    const Eigen::Quaternionf& q = T.unit_quaternion();
    p.q[0] = q.x(); p.q[1] = q.y(); p.q[2] = q.z(); p.q[3] = q.w();
    const Eigen::Vector3f t = T.translation();
    p.t[0] = t(0); p.t[1] = t(1); p.t[2] = t(2);
    p.kind = ORBFE_SE3;
    return p;
}

inline orbfe_pose pose_of(const Sophus::Sim3f& S) {
    orbfe_pose p;
    const Eigen::Quaternionf& q = S.quaternion();   // RxSO3: non-unit, |q|^2 = scale
    p.q[0] = q.x(); p.q[1] = q.y(); p.q[2] = q.z(); p.q[3] = q.w();
    const Eigen::Vector3f t = S.translation();
    p.t[0] = t(0); p.t[1] = t(1); p.t[2] = t(2);
    p.kind = ORBFE_SIM3;
    return p;
}

// GeometricCamera -> orbfe_camera_model (mnType, mvParameters)
inline orbfe_camera_model model_of(GeometricCamera* c) {
    orbfe_camera_model m;
    memset(&m, 0, sizeof(m));
    m.type = c->GetType() == GeometricCamera::CAM_PINHOLE ? ORBFE_CAM_PINHOLE : ORBFE_CAM_KANNALA_BRANDT8;
    const int np = m.type == ORBFE_CAM_PINHOLE ? 4 : 8;
    for (int k = 0; k < np; k++) m.params[k] = c->getParameter(k);
    return m;
}

}  // namespace orbfe_shim
}  // namespace ORB_SLAM3
