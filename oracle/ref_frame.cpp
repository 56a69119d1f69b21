// ORACLE -- TEST INFRASTRUCTURE ONLY (see ref_common.h).
//
// Frame::UndistortKeyPoints (src/Frame.cc:288-318) and
// Frame::ComputeImageBounds (:320-348) through cv::undistortPoints with
// P = K, restated from OpenCV 2.4's cvUndistortPoints (un-vendored): the
// normalised point x0 = (u - cx) / fx is refined 5 times in double,
//   icdist = (1 + ((k6 r2 + k5) r2 + k4) r2) / (1 + ((k3 r2 + k2) r2 + k1) r2)
//   x = (x0 - 2 p1 x y - p2 (r2 + 2 x^2)) icdist,
// then re-projected with RR = P (= K): (P00 x + P01 y + P02) / (P20 x + P21 y
// + P22).  Parity with OpenCV itself is unpinned (no OpenCV here).
#include <algorithm>
#include <cmath>
#include <cstdint>

#include "../include/orbx.h"

namespace {

void undistort(const float* K, const float* dist, float px, float py, float* ox, float* oy)
{
    const double fx = K[0], fy = K[1], cx = K[2], cy = K[3];
    const double ifx = 1. / fx, ify = 1. / fy;
    double k[8] = {dist[0], dist[1], dist[2], dist[3], dist[4], 0, 0, 0};
    double x = ((double)px - cx) * ifx, y = ((double)py - cy) * ify;
    const double x0 = x, y0 = y;
    for (int j = 0; j < 5; j++) {
        const double r2 = x * x + y * y;
        const double icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
        const double deltaX = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x);
        const double deltaY = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y;
        x = (x0 - deltaX) * icdist;
        y = (y0 - deltaY) * icdist;
    }
    const double xx = fx * x + 0.0 * y + cx;
    const double yy = 0.0 * x + fy * y + cy;
    const double ww = 1. / (0.0 * x + 0.0 * y + 1.0);
    *ox = (float)(xx * ww);
    *oy = (float)(yy * ww);
}

}  // namespace

extern "C" int orbx_ref_undistort_keypoints(int n, const orbx_keypoint* keys, const float* K, const float* dist,
                                            orbx_keypoint* keys_un)
{
    for (int i = 0; i < n; i++) {
        keys_un[i] = keys[i];
        if (dist[0] == 0.0f) continue;   // mvKeysUn = mvKeys (:290-294)
        undistort(K, dist, keys[i].x, keys[i].y, &keys_un[i].x, &keys_un[i].y);
    }
    return ORBX_OK;
}

extern "C" int orbx_ref_compute_image_bounds(int w, int h, const float* K, const float* dist, float* b)
{
    if (dist[0] == 0.0f) {
        b[0] = 0.f;
        b[1] = (float)w;
        b[2] = 0.f;
        b[3] = (float)h;
        return ORBX_OK;
    }
    const float cx[4] = {0.f, (float)w, 0.f, (float)w}, cy[4] = {0.f, 0.f, (float)h, (float)h};
    float ux[4], uy[4];
    for (int i = 0; i < 4; i++) undistort(K, dist, cx[i], cy[i], &ux[i], &uy[i]);
    b[0] = std::min(std::floor(ux[0]), std::floor(ux[2]));
    b[1] = std::max(std::ceil(ux[1]), std::ceil(ux[3]));
    b[2] = std::min(std::floor(uy[0]), std::floor(uy[1]));
    b[3] = std::max(std::ceil(uy[2]), std::ceil(uy[3]));
    return ORBX_OK;
}
