// SE3 / quaternion device primitives shared by the local-BA and
// pose-optimisation kernels: g2o's SE3Quat (types/slam3d/se3quat.h) with
// Eigen's quaternion formulas (Quaternion::_transformVector,
// toRotationMatrix, quaternionbase_assign_impl<3x3>), FP64.
#pragma once

#include <hip/hip_runtime.h>

namespace orbx {

struct Q { double x, y, z, w; };

__device__ inline void qrot(const Q& q, const double v[3], double o[3])
{
    double uv[3] = {q.y * v[2] - q.z * v[1], q.z * v[0] - q.x * v[2], q.x * v[1] - q.y * v[0]};
    for (int i = 0; i < 3; i++) uv[i] += uv[i];
    const double c[3] = {q.y * uv[2] - q.z * uv[1], q.z * uv[0] - q.x * uv[2], q.x * uv[1] - q.y * uv[0]};
    for (int i = 0; i < 3; i++) o[i] = v[i] + q.w * uv[i] + c[i];
}

__device__ inline Q qmul(const Q& a, const Q& b)
{
    Q r;
    r.w = a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z;
    r.x = a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y;
    r.y = a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z;
    r.z = a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x;
    return r;
}

__device__ inline void qmat(const Q& q, double R[9])
{
    const double tx = 2 * q.x, ty = 2 * q.y, tz = 2 * q.z;
    const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
    const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
    const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
    R[0] = 1 - (tyy + tzz); R[1] = txy - twz;       R[2] = txz + twy;
    R[3] = txy + twz;       R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;       R[7] = tyz + twx;       R[8] = 1 - (txx + tyy);
}

__device__ inline Q qfrom(const double m[9])
{
    Q q;
    double t = m[0] + m[4] + m[8];
    if (t > 0) {
        t = sqrt(t + 1.0);
        q.w = 0.5 * t;
        t = 0.5 / t;
        q.x = (m[7] - m[5]) * t;
        q.y = (m[2] - m[6]) * t;
        q.z = (m[3] - m[1]) * t;
    } else {
        // Eigen's branch on the largest diagonal entry, spelled out per case
        // (no dynamically indexed private arrays)
        int i = 0;
        if (m[4] > m[0]) i = 1;
        if (m[8] > m[i * 4]) i = 2;
        if (i == 0) {
            t = sqrt(m[0] - m[4] - m[8] + 1.0);
            q.x = 0.5 * t;
            t = 0.5 / t;
            q.w = (m[7] - m[5]) * t;
            q.y = (m[3] + m[1]) * t;
            q.z = (m[6] + m[2]) * t;
        } else if (i == 1) {
            t = sqrt(m[4] - m[8] - m[0] + 1.0);
            q.y = 0.5 * t;
            t = 0.5 / t;
            q.w = (m[2] - m[6]) * t;
            q.z = (m[7] + m[5]) * t;
            q.x = (m[1] + m[3]) * t;
        } else {
            t = sqrt(m[8] - m[0] - m[4] + 1.0);
            q.z = 0.5 * t;
            t = 0.5 / t;
            q.w = (m[3] - m[1]) * t;
            q.x = (m[2] + m[6]) * t;
            q.y = (m[5] + m[7]) * t;
        }
    }
    return q;
}

__device__ inline void qnormalize(Q& q)
{
    if (q.w < 0) {
        q.x = -q.x; q.y = -q.y; q.z = -q.z; q.w = -q.w;
    }
    const double n = sqrt(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
    q.x /= n; q.y /= n; q.z /= n; q.w /= n;
}

// VertexSE3Expmap::oplusImpl: estimate = SE3Quat::exp(update) * estimate
__device__ inline void se3_oplus(double* pose, const double* u)
{
    const double om[3] = {u[0], u[1], u[2]}, up[3] = {u[3], u[4], u[5]};
    const double theta = sqrt(om[0] * om[0] + om[1] * om[1] + om[2] * om[2]);
    const double O[9] = {0, -om[2], om[1], om[2], 0, -om[0], -om[1], om[0], 0};
    double O2[9], R[9], V[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) O2[i * 3 + j] = O[i * 3] * O[j] + O[i * 3 + 1] * O[3 + j] + O[i * 3 + 2] * O[6 + j];
    if (theta < 0.00001) {
        for (int i = 0; i < 9; i++) R[i] = (i % 4 == 0 ? 1.0 : 0.0) + O[i] + O2[i];
        for (int i = 0; i < 9; i++) V[i] = R[i];
    } else {
        const double s = sin(theta), c = cos(theta);
        const double a = s / theta, b = (1 - c) / (theta * theta), d = (theta - s) / pow(theta, 3);
        for (int i = 0; i < 9; i++) {
            const double I = (i % 4 == 0 ? 1.0 : 0.0);
            R[i] = I + a * O[i] + b * O2[i];
            V[i] = I + b * O[i] + d * O2[i];
        }
    }
    Q eq = qfrom(R);
    double et[3];
    for (int i = 0; i < 3; i++) et[i] = V[i * 3] * up[0] + V[i * 3 + 1] * up[1] + V[i * 3 + 2] * up[2];
    qnormalize(eq);
    // (exp) * estimate  (SE3Quat::operator*)
    const Q pq{pose[0], pose[1], pose[2], pose[3]};
    const double pt[3] = {pose[4], pose[5], pose[6]};
    double rt[3];
    qrot(eq, pt, rt);
    Q nq = qmul(eq, pq);
    qnormalize(nq);
    pose[0] = nq.x; pose[1] = nq.y; pose[2] = nq.z; pose[3] = nq.w;
    for (int i = 0; i < 3; i++) pose[4 + i] = et[i] + rt[i];
}

__device__ inline void se3_map(const double* pose, const double* p, double* o)
{
    const Q q{pose[0], pose[1], pose[2], pose[3]};
    qrot(q, p, o);
    for (int i = 0; i < 3; i++) o[i] += pose[4 + i];
}

}  // namespace orbx
