// TEST INFRASTRUCTURE (tests/test_shim_compile.py): minimal stand-ins for the OpenCV 4.2 / Eigen 3 /
// Sophus / DBoW2 types and the ORB-SLAM3 classes that the drop-in shim (shim/*.cc) touches, so the shim
// compiles with -fsyntax-only in a container that has none of those libraries. Declarations only, of
// the members the shim uses, with the reference's names and argument types (orb_slam3/include/*.h);
// nothing here is linked or run.
#pragma once
#include <cstddef>
#include <cstdint>
#include <list>
#include <map>
#include <set>
#include <tuple>
#include <utility>
#include <vector>

#define EIGEN_MAKE_ALIGNED_OPERATOR_NEW

namespace cv {
enum { CV_8U_ = 0 };
struct Size {
    int width = 0, height = 0;
    bool operator==(const Size& o) const { return width == o.width && height == o.height; }
    bool operator!=(const Size& o) const { return !(*this == o); }
};
template <class T> struct Point_ { T x, y; Point_() : x(0), y(0) {} Point_(T a, T b) : x(a), y(b) {} };
typedef Point_<float> Point2f;
struct KeyPoint {
    Point2f pt;
    float size, angle, response;
    int octave, class_id;
};
struct Range {};
class Mat {
public:
    int rows = 0, cols = 0;
    size_t step = 0;
    uint8_t* data = nullptr;
    Mat();
    Mat(int rows, int cols, int type);
    void create(int rows, int cols, int type);
    bool empty() const;
    int type() const;
    Size size() const;
    Mat rowRange(int a, int b) const;
    Mat clone() const;
    void copyTo(const Mat& dst) const;
    void release();
    template <class T> T* ptr(int row = 0);
    template <class T> const T* ptr(int row = 0) const;
    template <class T> T& at(int i0);
    template <class T> const T& at(int i0) const;
    template <class T> T& at(int r, int c);
    template <class T> const T& at(int r, int c) const;
};
class _InputArray {
public:
    Mat getMat() const;
    bool empty() const;
};
class _OutputArray : public _InputArray {
public:
    void create(int rows, int cols, int type) const;
    void release() const;
};
typedef const _InputArray& InputArray;
typedef const _OutputArray& OutputArray;
}  // namespace cv
#define CV_8U 0
#define CV_8UC1 0

namespace Eigen {
template <class S, int R, int C>
class Matrix {
public:
    Matrix();
    S& operator()(int i);
    S operator()(int i) const;
    S& operator()(int r, int c);
    S operator()(int r, int c) const;
    Matrix operator-(const Matrix& o) const;
    Matrix operator+(const Matrix& o) const;
    Matrix operator/(S s) const;
    template <int C2> Matrix<S, R, C2> operator*(const Matrix<S, C, C2>& o) const;
    Matrix<S, C, R> transpose() const;
    Matrix inverse() const;
    S norm() const;
    S dot(const Matrix& o) const;
    void setZero();
};
typedef Matrix<float, 3, 1> Vector3f;
typedef Matrix<float, 2, 1> Vector2f;
typedef Matrix<float, 3, 3> Matrix3f;
template <class S>
class Quaternion {
public:
    S x() const; S y() const; S z() const; S w() const;
};
typedef Quaternion<float> Quaternionf;
}  // namespace Eigen

namespace Sophus {
template <class S>
class SO3 {
public:
    static Eigen::Matrix<S, 3, 3> hat(const Eigen::Matrix<S, 3, 1>& v);
};
typedef SO3<float> SO3f;
template <class S>
class SE3 {
public:
    SE3();
    SE3(const Eigen::Matrix<S, 3, 3>& R, const Eigen::Matrix<S, 3, 1>& t);
    SE3 inverse() const;
    Eigen::Matrix<S, 3, 1> translation() const;
    Eigen::Matrix<S, 3, 3> rotationMatrix() const;
    const Eigen::Quaternion<S>& unit_quaternion() const;
    SE3 operator*(const SE3& o) const;
    Eigen::Matrix<S, 3, 1> operator*(const Eigen::Matrix<S, 3, 1>& p) const;
};
typedef SE3<float> SE3f;
template <class S>
class Sim3 {
public:
    Sim3 inverse() const;
    Eigen::Matrix<S, 3, 1> translation() const;
    Eigen::Matrix<S, 3, 3> rotationMatrix() const;
    S scale() const;
    const Eigen::Quaternion<S>& quaternion() const;
};
typedef Sim3<float> Sim3f;
}  // namespace Sophus

namespace DBoW2 {
typedef unsigned int NodeId;
class FeatureVector : public std::map<NodeId, std::vector<unsigned int>> {};
}  // namespace DBoW2

namespace ORB_SLAM3 {
class GeometricCamera {
public:
    enum { CAM_PINHOLE = 0, CAM_FISHEYE = 1 };
    unsigned int GetType();
    float getParameter(const int i);
    Eigen::Vector2f project(const Eigen::Vector3f& v3D);
    Eigen::Matrix3f toK_();
    bool epipolarConstrain(GeometricCamera* otherCamera, const cv::KeyPoint& kp1, const cv::KeyPoint& kp2,
                           const Eigen::Matrix3f& R12, const Eigen::Vector3f& t12, const float sigmaLevel,
                           const float unc);
};
class System {
public:
    enum eSensor { MONOCULAR = 0, STEREO = 1, RGBD = 2, IMU_MONOCULAR = 3, IMU_STEREO = 4, IMU_RGBD = 5 };
};
class Frame;
class KeyFrame;
class MapPoint;
class ORBextractor;
}  // namespace ORB_SLAM3

using std::pair;
using std::vector;
