// cv_compat.hpp -- the cv:: point/vector types the reference API uses.
//
// The reference headers (P/DistanceCalculator.hpp:5, P/Main.cpp) pull these
// from <opencv2/opencv.hpp> (OpenCV 3.0.0).  When OpenCV is installed we use
// it; otherwise this header supplies layout- and operator-compatible types so
// the drop-in API (Match.hpp, DistanceCalculator.hpp, Matching.hpp) compiles
// without OpenCV.  Semantics kept from OpenCV 3.0 where the reference's
// arithmetic depends on them:
//   * Point_<T> {x, y}; Point3_<T> {x, y, z}; Vec<T, n> {val[n]} -- same layout;
//   * Point_ +, -, +=, -= element-wise; * and / by a float/double/int scalar are
//     element-wise in the scalar's promoted type, then cast back to T
//     (Point2f / float stays a float operation);
//   * Vec<T, n>(T v0) is non-explicit and zero-fills the tail, and
//     Point3_(const Vec<T,3>&) is non-explicit, so (Point3i)(unsigned u) is
//     (u, 0, 0) -- the conversion P/Main.cpp:492 relies on;
//   * RotatedRect {center, size, angle(deg)} and points() in OpenCV's corner order
//     (the centroid step, P/Main.cpp:1129-1139).
#pragma once

#if defined(__has_include)
#if __has_include(<opencv2/opencv.hpp>) && !defined(USV_NO_OPENCV)
#define USV_HAVE_OPENCV 1
#endif
#endif

#ifdef USV_HAVE_OPENCV
#include <opencv2/opencv.hpp>
#else
#include <cmath>
#include <cstddef>

namespace cv {

template <typename T, int n>
class Vec {
public:
    T val[n];
    Vec() {
        for (int i = 0; i < n; ++i) val[i] = T(0);
    }
    Vec(T v0) {  // non-explicit, as in OpenCV 3.0
        val[0] = v0;
        for (int i = 1; i < n; ++i) val[i] = T(0);
    }
    Vec(T v0, T v1) {
        static_assert(n >= 2, "Vec(v0, v1) needs n >= 2");
        val[0] = v0;
        val[1] = v1;
        for (int i = 2; i < n; ++i) val[i] = T(0);
    }
    Vec(T v0, T v1, T v2) {
        static_assert(n >= 3, "Vec(v0, v1, v2) needs n >= 3");
        val[0] = v0;
        val[1] = v1;
        val[2] = v2;
        for (int i = 3; i < n; ++i) val[i] = T(0);
    }
    T& operator[](int i) { return val[i]; }
    const T& operator[](int i) const { return val[i]; }
};
typedef Vec<int, 2> Vec2i;
typedef Vec<int, 3> Vec3i;
typedef Vec<int, 4> Vec4i;
typedef Vec<float, 2> Vec2f;
typedef Vec<float, 3> Vec3f;
typedef Vec<double, 3> Vec3d;

template <typename T>
class Point_ {
public:
    T x, y;
    Point_() : x(0), y(0) {}
    Point_(T x_, T y_) : x(x_), y(y_) {}
    Point_(const Vec<T, 2>& v) : x(v.val[0]), y(v.val[1]) {}
    template <typename U>
    operator Point_<U>() const {
        return Point_<U>(static_cast<U>(x), static_cast<U>(y));
    }
    T dot(const Point_& p) const { return x * p.x + y * p.y; }
};

template <typename T>
class Point3_ {
public:
    T x, y, z;
    Point3_() : x(0), y(0), z(0) {}
    Point3_(T x_, T y_, T z_) : x(x_), y(y_), z(z_) {}
    Point3_(const Vec<T, 3>& v) : x(v.val[0]), y(v.val[1]), z(v.val[2]) {}  // non-explicit
    explicit Point3_(const Point_<T>& p) : x(p.x), y(p.y), z(0) {}
};

typedef Point_<int> Point2i;
typedef Point2i Point;
typedef Point_<float> Point2f;
typedef Point_<double> Point2d;
typedef Point3_<int> Point3i;
typedef Point3_<float> Point3f;
typedef Point3_<double> Point3d;

template <typename T> inline Point_<T> operator+(const Point_<T>& a, const Point_<T>& b) { return Point_<T>(static_cast<T>(a.x + b.x), static_cast<T>(a.y + b.y)); }
template <typename T> inline Point_<T> operator-(const Point_<T>& a, const Point_<T>& b) { return Point_<T>(static_cast<T>(a.x - b.x), static_cast<T>(a.y - b.y)); }
template <typename T> inline Point_<T> operator-(const Point_<T>& a) { return Point_<T>(static_cast<T>(-a.x), static_cast<T>(-a.y)); }
template <typename T> inline Point_<T>& operator+=(Point_<T>& a, const Point_<T>& b) { a.x = static_cast<T>(a.x + b.x); a.y = static_cast<T>(a.y + b.y); return a; }
template <typename T> inline Point_<T>& operator-=(Point_<T>& a, const Point_<T>& b) { a.x = static_cast<T>(a.x - b.x); a.y = static_cast<T>(a.y - b.y); return a; }
template <typename T> inline bool operator==(const Point_<T>& a, const Point_<T>& b) { return a.x == b.x && a.y == b.y; }
template <typename T> inline bool operator!=(const Point_<T>& a, const Point_<T>& b) { return !(a == b); }

// scalar * and / : the operation runs in the promoted type of (T, S).
#define USV_CV_SCALAR_OPS(S)                                                                       \
    template <typename T> inline Point_<T> operator*(const Point_<T>& a, S b) { return Point_<T>(static_cast<T>(a.x * b), static_cast<T>(a.y * b)); } \
    template <typename T> inline Point_<T> operator*(S b, const Point_<T>& a) { return Point_<T>(static_cast<T>(a.x * b), static_cast<T>(a.y * b)); } \
    template <typename T> inline Point_<T> operator/(const Point_<T>& a, S b) { return Point_<T>(static_cast<T>(a.x / b), static_cast<T>(a.y / b)); } \
    template <typename T> inline Point_<T>& operator*=(Point_<T>& a, S b) { a.x = static_cast<T>(a.x * b); a.y = static_cast<T>(a.y * b); return a; } \
    template <typename T> inline Point_<T>& operator/=(Point_<T>& a, S b) { a.x = static_cast<T>(a.x / b); a.y = static_cast<T>(a.y / b); return a; }
USV_CV_SCALAR_OPS(int)
USV_CV_SCALAR_OPS(float)
USV_CV_SCALAR_OPS(double)
#undef USV_CV_SCALAR_OPS


template <typename T>
class Size_ {
public:
    T width, height;
    Size_() : width(0), height(0) {}
    Size_(T w, T h) : width(w), height(h) {}
};
typedef Size_<float> Size2f;

// OpenCV 3.0 RotatedRect: centre, (width, height), angle in degrees.
class RotatedRect {
public:
    Point2f center;
    Size2f size;
    float angle;
    RotatedRect() : center(), size(), angle(0) {}
    RotatedRect(const Point2f& c, const Size2f& s, float a) : center(c), size(s), angle(a) {}
    // The four corners, OpenCV's order and float arithmetic (double angle -> float cos/sin * 0.5f).
    void points(Point2f pt[]) const {
        const double a_rad = angle * 3.14159265358979323846 / 180.;
        const float b = (float)std::cos(a_rad) * 0.5f;
        const float a = (float)std::sin(a_rad) * 0.5f;
        pt[0].x = center.x - a * size.height - b * size.width;
        pt[0].y = center.y + b * size.height - a * size.width;
        pt[1].x = center.x + a * size.height - b * size.width;
        pt[1].y = center.y - b * size.height - a * size.width;
        pt[2].x = 2 * center.x - pt[0].x;
        pt[2].y = 2 * center.y - pt[0].y;
        pt[3].x = 2 * center.x - pt[1].x;
        pt[3].y = 2 * center.y - pt[1].y;
    }
};

}  // namespace cv
#endif  // USV_HAVE_OPENCV
