// tests/compile/shim/lorb_cv_shim.hpp -- declaration-only stand-ins for the OpenCV / Ceres types
// that the reference's headers (include/*.h of abstract-liu/LORB_SLAM) and its caller
// src/visual_odometry.cpp name.  Used ONLY by tests/test_compile_boundary.py to run
// `g++ -fsyntax-only` over the drop-ins and the reference's unchanged callers (OpenCV and Ceres are
// not installed in this image).  Nothing here is linked or executed; bodies are minimal so that
// the expressions the callers write type-check.  Written from the call sites, not from OpenCV.
#pragma once

#include <cstddef>
#include <cstdint>
#include <initializer_list>
#include <vector>
// standard headers the real OpenCV / Ceres headers bring in transitively (the reference relies on
// them: include/matcher.h and include/map.h name std::set without including <set>)
#include <algorithm>
#include <cmath>
#include <map>
#include <set>
#include <string>

#define CV_8U 0
#define CV_8UC1 0
#define CV_32F 5
#define CV_64F 6

namespace cv {

template <class T> struct Point_ {
  T x{}, y{};
  Point_() = default;
  Point_(T x_, T y_) : x(x_), y(y_) {}
};
template <class T> struct Point3_ {
  T x{}, y{}, z{};
  Point3_() = default;
  Point3_(T x_, T y_, T z_) : x(x_), y(y_), z(z_) {}
};
typedef Point_<float> Point2f;
typedef Point_<int> Point2i;
typedef Point2i Point;
typedef Point3_<float> Point3f;

struct KeyPoint {
  Point2f pt;
  float size = 0, angle = -1, response = 0;
  int octave = 0, class_id = -1;
};

struct DMatch {
  int queryIdx = -1, trainIdx = -1, imgIdx = -1;
  float distance = 0;
};

class Mat {
 public:
  int rows = 0, cols = 0;
  size_t step = 0;
  unsigned char* data = nullptr;
  Mat() = default;
  Mat(int r, int c, int /*type*/) : rows(r), cols(c) {}
  static Mat eye(int r, int c, int type) { return Mat(r, c, type); }
  static Mat zeros(int r, int c, int type) { return Mat(r, c, type); }
  Mat clone() const { return *this; }
  Mat inv() const { return *this; }
  Mat t() const { return *this; }
  bool empty() const { return rows == 0; }
  void push_back(const Mat&) {}
  Mat row(int) const { return *this; }
  Mat rowRange(int, int) const { return *this; }
  Mat colRange(int, int) const { return *this; }
  void copyTo(Mat&) const {}
  template <class T> T* ptr(int = 0) { return reinterpret_cast<T*>(data); }
  template <class T> const T* ptr(int = 0) const { return reinterpret_cast<const T*>(data); }
  template <class T> T& at(int i) { return ptr<T>()[i]; }
  template <class T> const T& at(int i) const { return ptr<T>()[i]; }
  template <class T> T& at(int r, int c) { return ptr<T>()[r * cols + c]; }
  template <class T> const T& at(int r, int c) const { return ptr<T>()[r * cols + c]; }
};
inline Mat operator*(const Mat& a, const Mat&) { return a; }
inline Mat operator+(const Mat& a, const Mat&) { return a; }
inline Mat operator-(const Mat& a, const Mat&) { return a; }
inline Mat operator-(const Mat& a) { return a; }

template <class T> struct MatCommaInitializer_ {
  Mat m;
  MatCommaInitializer_& operator,(T) { return *this; }
  operator Mat() const { return m; }
};
template <class T> struct Mat_ : Mat {
  Mat_(int r, int c) : Mat(r, c, CV_32F) {}
  MatCommaInitializer_<T> operator<<(T) const { return MatCommaInitializer_<T>{*this}; }
};

typedef const Mat& InputArray;
typedef Mat& OutputArray;
typedef Mat& InputOutputArray;

enum { SOLVEPNP_ITERATIVE = 0 };
bool solvePnPRansac(const std::vector<Point3f>& objectPoints, const std::vector<Point2f>& imagePoints,
                    InputArray cameraMatrix, InputArray distCoeffs, OutputArray rvec, OutputArray tvec,
                    bool useExtrinsicGuess, int iterationsCount, float reprojectionError, double confidence,
                    std::vector<int>& inliers, int flags);
bool solvePnP(const std::vector<Point3f>& objectPoints, const std::vector<Point2f>& imagePoints,
              InputArray cameraMatrix, InputArray distCoeffs, OutputArray rvec, OutputArray tvec,
              bool useExtrinsicGuess = false, int flags = SOLVEPNP_ITERATIVE);
void Rodrigues(InputArray src, OutputArray dst);

}  // namespace cv

namespace ceres {
class Problem;
struct Solver {
  struct Options {};
  struct Summary {};
};
}  // namespace ceres
