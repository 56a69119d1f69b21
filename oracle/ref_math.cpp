// ORACLE -- TEST INFRASTRUCTURE ONLY (see ref_common.h).
//
// Numeric primitives the reference obtains from its dependencies:
//   * cv::fastAtan2 (OpenCV 2.4 core/src/mathfuncs.cpp), called from
//     IC_Angle (src/ORBextractor.cc:150).
//   * cos/sin on a float angle (src/ORBextractor.cc:160).  With `using
//     namespace std` these resolve to std::cos(float)/std::sin(float), i.e.
//     libm cosf/sinf.  libm versions differ (glibc 2.15/2.19 of the
//     reference era vs 2.35 here, which is not correctly rounded on ~0.1% of
//     [0, 2pi]); the pinned semantics is the correctly rounded value, which
//     every libm approximates.  It is computed from double cos/sin and, when
//     the double result lies within 16 ulp of a float rounding midpoint, from
//     binary128 (libquadmath).
#include "ref_common.h"

#include <cfloat>
#include <cmath>
#include <cstring>
#include <quadmath.h>

namespace orbref {

// OpenCV 2.4 polynomial atan2 in degrees.  Constants are float products
// evaluated exactly as the static initialisers do.
static const float kP1 = 0.9997878412794807f * (float)(180 / M_PI);
static const float kP3 = -0.3258083974640975f * (float)(180 / M_PI);
static const float kP5 = 0.1555786518463281f * (float)(180 / M_PI);
static const float kP7 = -0.04432655554792128f * (float)(180 / M_PI);

float fast_atan2_cv24(float y, float x)
{
    const float ax = std::fabs(x), ay = std::fabs(y);
    float a;
    if (ax >= ay) {
        const float c = ay / (ax + (float)DBL_EPSILON);
        const float c2 = c * c;
        a = (((kP7 * c2 + kP5) * c2 + kP3) * c2 + kP1) * c;
    } else {
        const float c = ax / (ay + (float)DBL_EPSILON);
        const float c2 = c * c;
        a = 90.f - (((kP7 * c2 + kP5) * c2 + kP3) * c2 + kP1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

// True when double d lies within 16 double-ulps of the midpoint between the
// two floats that bracket it (so rounding d to float may be wrong).
static bool near_midpoint(double d)
{
    const float f = (float)d;
    if ((double)f == d) return false;
    const float g = std::nextafter(f, d > (double)f ? INFINITY : -INFINITY);
    const double mid = 0.5 * ((double)f + (double)g);
    return std::fabs(d - mid) <= 16.0 * std::fabs(d) * DBL_EPSILON;
}

float cr_cosf(float x)
{
    const double d = std::cos((double)x);
    if (near_midpoint(d)) return (float)cosq((__float128)x);
    return (float)d;
}

float cr_sinf(float x)
{
    const double d = std::sin((double)x);
    if (near_midpoint(d)) return (float)sinq((__float128)x);
    return (float)d;
}

}  // namespace orbref
