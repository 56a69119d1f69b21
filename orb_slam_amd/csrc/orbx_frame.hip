// Frame construction on the device: keypoint
// undistortion (Frame::UndistortKeyPoints, src/Frame.cc:288-318) and the
// undistorted image bounds (Frame::ComputeImageBounds, :320-348), both
// through cv::undistortPoints with P = K (OpenCV 2.4 cvUndistortPoints,
// un-vendored, restated: the normalised point iterated 5 times in double
// against k1 k2 p1 p2 k3, then re-projected with K; a zero k1 copies the
// keypoints as the reference does).  One thread per keypoint; the
// device-resident form rewrites the keypoints of extracted frame slots in
// place so the matchers read mvKeysUn.
#include <algorithm>
#include <cmath>

#include "orbx_device.h"
#include "orbx_internal.h"

namespace orbx {

struct Undistort {
    double fx, fy, cx, cy, ifx, ify;
    double k[8];   // k1 k2 p1 p2 k3 k4 k5 k6
    double p0, p2, p4, p5;   // RR = P (= K): rows [fx 0 cx; 0 fy cy; 0 0 1]
};

__host__ __device__ inline void undistort_point(const Undistort& U, float px, float py, float* ox, float* oy)
{
    double x = ((double)px - U.cx) * U.ifx, y = ((double)py - U.cy) * U.ify;
    const double x0 = x, y0 = y;
    const double* k = U.k;
    for (int j = 0; j < 5; j++) {
        const double r2 = x * x + y * y;
        const double icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
        const double deltaX = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x);
        const double deltaY = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y;
        x = (x0 - deltaX) * icdist;
        y = (y0 - deltaY) * icdist;
    }
    // RR = P * I: xx = P00 x + P01 y + P02, ww = 1 / (0 x + 0 y + 1)
    const double xx = U.p0 * x + 0.0 * y + U.cx;
    const double yy = 0.0 * x + U.p4 * y + U.cy;
    const double ww = 1. / (0.0 * x + 0.0 * y + 1.0);
    *ox = (float)(xx * ww);
    *oy = (float)(yy * ww);
}

__global__ __launch_bounds__(256) void k_undistort(Undistort U, orbx_keypoint* kps, const int32_t* counts, int stride,
                                                   int n_single)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int slot = blockIdx.y;
    const int n = counts ? counts[slot] : n_single;
    if (i >= n) return;
    orbx_keypoint& k = kps[(size_t)slot * stride + i];
    float x, y;
    undistort_point(U, k.x, k.y, &x, &y);
    k.x = x;
    k.y = y;
}

namespace {
bool make_undistort(const float* K, const float* dist, Undistort& U)
{
    if (!K || !dist || !(K[0] != 0.0f) || !(K[1] != 0.0f)) return false;
    U.fx = K[0];
    U.fy = K[1];
    U.cx = K[2];
    U.cy = K[3];
    U.ifx = 1. / U.fx;
    U.ify = 1. / U.fy;
    for (int i = 0; i < 8; i++) U.k[i] = 0;
    for (int i = 0; i < 5; i++) U.k[i] = dist[i];   // k1 k2 p1 p2 k3
    U.p0 = U.fx;
    U.p2 = U.cx;
    U.p4 = U.fy;
    U.p5 = U.cy;
    return true;
}
}  // namespace
}  // namespace orbx

using namespace orbx;

extern "C" int orbx_undistort_keypoints(orbx_ctx* ctx, int n, const orbx_keypoint* keys, const float* K,
                                        const float* dist, orbx_keypoint* keys_un)
{
    Undistort U;
    if (!ctx || n < 0 || (n > 0 && (!keys || !keys_un)) || !make_undistort(K, dist, U)) return ORBX_ERR_ARG;
    if (n == 0) return ORBX_OK;
    if (dist[0] == 0.0f) {   // mDistCoef.at<float>(0)==0.0: mvKeysUn = mvKeys (:290-294)
        std::copy(keys, keys + n, keys_un);
        return ORBX_OK;
    }
    ctx_enter(ctx);
    int r = ensure_scratch(ctx, (size_t)n * sizeof(orbx_keypoint));
    if (r != ORBX_OK) return r;
    orbx_keypoint* d = static_cast<orbx_keypoint*>(ctx->scratch);
    ORBX_HIP_CHECK(hipMemcpyAsync(d, keys, (size_t)n * sizeof(orbx_keypoint), hipMemcpyHostToDevice, ctx->stream));
    hipLaunchKernelGGL(k_undistort, dim3((n + 255) / 256, 1), dim3(256), 0, ctx->stream, U, d, nullptr, 0, n);
    ORBX_HIP_CHECK(hipGetLastError());
    ORBX_HIP_CHECK(hipMemcpyAsync(keys_un, d, (size_t)n * sizeof(orbx_keypoint), hipMemcpyDeviceToHost, ctx->stream));
    ORBX_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    return ORBX_OK;
}

extern "C" int orbx_compute_image_bounds(int w, int h, const float* K, const float* dist, float* bounds)
{
    Undistort U;
    if (w <= 0 || h <= 0 || !bounds || !make_undistort(K, dist, U)) return ORBX_ERR_ARG;
    if (dist[0] == 0.0f) {
        bounds[0] = 0.f;
        bounds[1] = (float)w;
        bounds[2] = 0.f;
        bounds[3] = (float)h;
        return ORBX_OK;
    }
    // the four corners (:324-334); host evaluation of the same routine the
    // keypoint kernel runs (four points do not warrant a launch)
    const float cx[4] = {0.f, (float)w, 0.f, (float)w}, cy[4] = {0.f, 0.f, (float)h, (float)h};
    float ux[4], uy[4];
    for (int i = 0; i < 4; i++) undistort_point(U, cx[i], cy[i], &ux[i], &uy[i]);
    bounds[0] = std::min(std::floor(ux[0]), std::floor(ux[2]));   // mnMinX
    bounds[1] = std::max(std::ceil(ux[1]), std::ceil(ux[3]));     // mnMaxX
    bounds[2] = std::min(std::floor(uy[0]), std::floor(uy[1]));   // mnMinY
    bounds[3] = std::max(std::ceil(uy[2]), std::ceil(uy[3]));     // mnMaxY
    return ORBX_OK;
}

extern "C" int orbx_dev_undistort(orbx_ctx* ctx, int first, int count, const float* K, const float* dist)
{
    Undistort U;
    if (!ctx || first < 0 || count < 0 || first + count > ctx->slots || !make_undistort(K, dist, U))
        return ORBX_ERR_ARG;
    if (count == 0 || dist[0] == 0.0f) return ORBX_OK;
    ctx_enter(ctx);
    const int nf = ctx->geom.nfeatures;
    hipLaunchKernelGGL(k_undistort, dim3((nf + 255) / 256, count), dim3(256), 0, ctx->stream, U,
                       ctx->out_kps + (size_t)first * nf, ctx->out_n + first, nf, 0);
    ORBX_HIP_CHECK(hipGetLastError());
    return ORBX_OK;
}
