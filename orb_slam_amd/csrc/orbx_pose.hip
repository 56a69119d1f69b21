// Motion-only pose optimisation on MI355X (FP64): Optimizer::PoseOptimization
// (src/Optimizer.cc:154-285) for batches of frames.
//
// g2o subset (as the reference configures it): one VertexSE3Expmap against
// fixed VertexSBAPointXYZ vertices through EdgeSE3ProjectXYZ edges with a
// Huber kernel, BlockSolverX + LinearSolverDense (Eigen LDLT, diagonal
// pivoting) and OptimizationAlgorithmLevenberg with ORB-SLAM's stop rule.
// The points are fixed, so the Schur complement is empty and every LM trial
// is a 6x6 solve.
//
// Mapping: one wavefront per frame, four frames per 256-thread workgroup,
// the whole four-round robust optimisation (up to 32 LM iterations of up to
// 10 trials) in ONE launch, no workgroup barriers.  The frame's first
// kPoseLdsEdges edges are copied into the wavefront's LDS area once (a
// wavefront-scope fence, no barrier: each wave reads only its own area) and
// every pass reads them there; edges past them are read from global memory.
// Lanes stride the edges: edge a < nL on lane a % 64, edge a >= nL on lane
// (a - nL) % 64, the same lane for the whole run, so an edge's level
// (outlier) flag is lane-private.  Per LM iteration one fused pass computes the errors, the
// robust chi2, the Jacobians and the 21 lower entries of H plus b; per trial
// one pass computes the trial errors.  Sums are wave reductions whose result
// is bitwise identical on every lane, so the LDLT, the exp-map update and
// the accept/reject logic run redundantly on uniform data (no broadcast).
//
// Stored-error semantics: g2o's outlier test reads each edge's _error as
// left by the LAST computeActiveErrors -- the final trial's state even when
// that trial was rejected and the estimate popped.  The kernel keeps that
// pose ("errpose") and re-evaluates active edges there; edges already
// classified as outliers are recomputed at the current pose
// (src/Optimizer.cc:250-251).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <thread>
#include <type_traits>
#include <vector>

#include "orbx_device.h"
#include "orbx_internal.h"
#include "orbx_pose_dev.h"
#include "orbx_se3.h"

namespace orbx {


constexpr int kPoseThreads = 256;   // 4 frames (wavefronts) per workgroup
// Edges per frame kept in LDS (6 floats + the outlier flag, 25 B each):
// 4 frames x 800 edges = 80 KB per workgroup, 2 workgroups per CU of
// gfx950's 160 KB -- the occupancy the kernel's 250 VGPRs allow anyway.  The passes over the edges
// (one per LM iteration, one per trial, one per robust round) then read LDS
// instead of re-fetching the frame from HBM; edges past the first 800 are
// read from global memory.
constexpr int kPoseLdsEdges = 800;
// edges a one-frame workgroup (the kW > 1 instances) keeps in LDS: 75 KB
constexpr int kPoseLdsEdgesWide = 3072;
// active-edge list capacity of the exact-sum batch kernel (u16 indices, 4 KB
// per frame); frames with more edges walk all of them every pass
constexpr int kPoseActCap = 2048;
#ifndef ORBX_POSE_WIDE
#define ORBX_POSE_WIDE 4
#endif
constexpr int kPoseWideWaves = ORBX_POSE_WIDE;    // wavefronts per frame of the one-call kernel
static_assert((kPoseThreads / 64) * kPoseLdsEdges * (6 * sizeof(float) + 1) <= 80 * 1024,
              "two pose workgroups per CU need <= 80 KB of LDS each (gfx950: 160 KB per CU)");

// Wave sum whose result is the same double on every lane: DPP butterflies
// inside each row of 16 (xor 1, xor 2 by quad_perm; the half-row and row
// mirrors pair lanes symmetrically), then the four row sums combined by
// readlane in a fixed order.
__device__ inline double dpp_f64(double v, int ctrl_sel)
{
    const int lo = __double2loint(v), hi = __double2hiint(v);
    int rlo, rhi;
    switch (ctrl_sel) {
    case 0:
        rlo = __builtin_amdgcn_update_dpp(lo, lo, 0xB1, 0xf, 0xf, false);   // quad_perm [1,0,3,2]
        rhi = __builtin_amdgcn_update_dpp(hi, hi, 0xB1, 0xf, 0xf, false);
        break;
    case 1:
        rlo = __builtin_amdgcn_update_dpp(lo, lo, 0x4E, 0xf, 0xf, false);   // quad_perm [2,3,0,1]
        rhi = __builtin_amdgcn_update_dpp(hi, hi, 0x4E, 0xf, 0xf, false);
        break;
    case 2:
        rlo = __builtin_amdgcn_update_dpp(lo, lo, 0x141, 0xf, 0xf, false);  // row_half_mirror
        rhi = __builtin_amdgcn_update_dpp(hi, hi, 0x141, 0xf, 0xf, false);
        break;
    default:
        rlo = __builtin_amdgcn_update_dpp(lo, lo, 0x140, 0xf, 0xf, false);  // row_mirror
        rhi = __builtin_amdgcn_update_dpp(hi, hi, 0x140, 0xf, 0xf, false);
        break;
    }
    return __hiloint2double(rhi, rlo);
}

__device__ inline double lane_f64(double v, int lane)
{
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
    return __hiloint2double(hi, lo);
}

__device__ inline double wave_sum_uniform(double v)
{
    v += dpp_f64(v, 0);
    v += dpp_f64(v, 1);
    v += dpp_f64(v, 2);
    v += dpp_f64(v, 3);
    return (lane_f64(v, 0) + lane_f64(v, 16)) + (lane_f64(v, 32) + lane_f64(v, 48));
}

__device__ inline int wave_sum_int(int v)
{
    v += __builtin_amdgcn_update_dpp(v, v, 0xB1, 0xf, 0xf, false);
    v += __builtin_amdgcn_update_dpp(v, v, 0x4E, 0xf, 0xf, false);
    v += __builtin_amdgcn_update_dpp(v, v, 0x141, 0xf, 0xf, false);
    v += __builtin_amdgcn_update_dpp(v, v, 0x140, 0xf, 0xf, false);
    return __builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16) + __builtin_amdgcn_readlane(v, 32) +
           __builtin_amdgcn_readlane(v, 48);
}

// Eigen::LDLT<MatrixXd> of the lower triangle of m (row-major 6x6) and the
// solve of m x = b: the restatement of oracle/ref_pose.cpp ldlt_solve with
// every index a compile-time constant (the runtime pivot selects among
// unrolled swap variants), so the matrix stays in registers.
__device__ inline void swap_d(double& a, double& b)
{
    const double t = a;
    a = b;
    b = t;
}

// Packed lower triangle: entry (i, j), j <= i, at i (i + 1) / 2 + j.
#define LT(i, j) ((i) * ((i) + 1) / 2 + (j))

__device__ inline bool ldlt6_solve(double m[21], const double b[6], double x[6])
{
    int tr[6];
    double temp[6];
    int sign = 0;   // 0 zero, 1 positive semidefinite, 2 negative semidefinite, 3 indefinite
#pragma unroll
    for (int k = 0; k < 6; k++) {
        int big = k;
        double bv = fabs(m[LT(k, k)]);
#pragma unroll
        for (int i = k + 1; i < 6; i++)
            if (fabs(m[LT(i, i)]) > bv) {
                bv = fabs(m[LT(i, i)]);
                big = i;
            }
        tr[k] = big;
#pragma unroll
        for (int q = k + 1; q < 6; q++) {
            if (big == q) {
#pragma unroll
                for (int j = 0; j < k; j++) swap_d(m[LT(k, j)], m[LT(q, j)]);
#pragma unroll
                for (int i = q + 1; i < 6; i++) swap_d(m[LT(i, k)], m[LT(i, q)]);
                swap_d(m[LT(k, k)], m[LT(q, q)]);
#pragma unroll
                for (int i = k + 1; i < q; i++) swap_d(m[LT(i, k)], m[LT(q, i)]);
            }
        }
        if (k > 0) {
#pragma unroll
            for (int j = 0; j < k; j++) temp[j] = m[LT(j, j)] * m[LT(k, j)];
            double acc = m[LT(k, 0)] * temp[0];
#pragma unroll
            for (int j = 1; j < k; j++) acc += m[LT(k, j)] * temp[j];
            m[LT(k, k)] -= acc;
#pragma unroll
            for (int i = k + 1; i < 6; i++)
#pragma unroll
                for (int j = 0; j < k; j++) m[LT(i, k)] -= m[LT(i, j)] * temp[j];
        }
        const double akk = m[LT(k, k)];
        if (k < 5 && fabs(akk) > 0.0) {
#pragma unroll
            for (int i = k + 1; i < 6; i++) m[LT(i, k)] /= akk;
        }
        if (sign == 1) {
            if (akk < 0) sign = 3;
        } else if (sign == 2) {
            if (akk > 0) sign = 3;
        } else if (sign == 0) {
            if (akk > 0) sign = 1;
            else if (akk < 0) sign = 2;
        }
    }
#pragma unroll
    for (int i = 0; i < 6; i++) x[i] = b[i];
#pragma unroll
    for (int k = 0; k < 6; k++)
#pragma unroll
        for (int q = k + 1; q < 6; q++)
            if (tr[k] == q) swap_d(x[k], x[q]);
#pragma unroll
    for (int i = 0; i < 6; i++)
#pragma unroll
        for (int j = 0; j < i; j++) x[i] -= m[LT(i, j)] * x[j];
#pragma unroll
    for (int i = 0; i < 6; i++) {
        if (fabs(m[LT(i, i)]) > 2.2250738585072014e-308) x[i] /= m[LT(i, i)];
        else x[i] = 0.0;
    }
#pragma unroll
    for (int i = 4; i >= 0; i--) {
        double s = m[LT(i + 1, i)] * x[i + 1];
#pragma unroll
        for (int j = i + 2; j < 6; j++) s += m[LT(j, i)] * x[j];
        x[i] -= s;
    }
#pragma unroll
    for (int k = 5; k >= 0; k--)
#pragma unroll
        for (int q = k + 1; q < 6; q++)
            if (tr[k] == q) swap_d(x[k], x[q]);
    return sign == 1 || sign == 0;
}


struct Cam {
    double fx, fy, cx, cy;
};

// EdgeSE3ProjectXYZ::computeError (types_six_dof_expmap.h:172-177) at pose
// (q x y z w, t): e = obs - (fx X/Z + cx, fy Y/Z + cy), Xc = q Xw + t.
__device__ inline bool div_safe(double x, double y, double z);
__device__ inline double div_rcp(double d);
__device__ inline double div_by(double n, double d, double y);
__device__ inline void pose_edge_error(const double* pose, const double X[3], double o0, double o1, const Cam& c,
                                       double pc[3], double& e0, double& e1)
{
    se3_map(pose, X, pc);
    double u, v;
    if (div_safe(pc[0], pc[1], pc[2])) {   // the two quotients by z through one reciprocal (below)
        const double y = div_rcp(pc[2]);
        u = div_by(pc[0], pc[2], y) * c.fx + c.cx;
        v = div_by(pc[1], pc[2], y) * c.fy + c.cy;
    } else {
        u = pc[0] / pc[2] * c.fx + c.cx;
        v = pc[1] / pc[2] * c.fy + c.cy;
    }
    e0 = o0 - u;
    e1 = o1 - v;
}

// RobustKernelHuber::robustify (robust_kernel_impl.cpp:78-91)
__device__ inline void huber2(double e2, double delta, double& rho0, double& rho1)
{
    const double dsqr = delta * delta;
    if (e2 <= dsqr) {
        rho0 = e2;
        rho1 = 1.;
    } else {
        const double sq = sqrt(e2);
        rho0 = 2 * sq * delta - dsqr;
        rho1 = delta / sq;
    }
}

// Double division with the reciprocal shared between quotients of one
// denominator.  The compiler's f64 division is v_div_scale (operands
// rescaled only near the exponent range's ends), y = v_rcp_f64 refined by two
// Newton steps fma(y, fma(-d, y, 1), y), then q = n y, r = fma(-d, q, n),
// v_div_fmas = fma(r, y, q) and v_div_fixup (special values only) -- the
// correctly rounded n / d.  y depends on d alone, so where v_div_scale leaves
// both operands alone (div_safe below) div_by returns the same bits as n / d
// (up to the sign of a zero quotient, which only ever reaches sums and
// products here, where it changes nothing) for 3 instructions instead of 11.
__device__ inline double div_rcp(double d)
{
    double y = __builtin_amdgcn_rcp(d);
    y = __fma_rn(y, __fma_rn(-d, y, 1.0), y);
    return __fma_rn(y, __fma_rn(-d, y, 1.0), y);
}
__device__ inline double div_by(double n, double d, double y)
{
    const double q = n * y;
    return __fma_rn(__fma_rn(-d, q, n), y, q);
}
// The camera-frame point (x, y, z) of an edge keeps every division of
// computeError and linearizeOplus away from v_div_scale's rescaling: |x|, |y|
// zero or in [2^-150, 2^150], |z| in [2^-150, 2^150] bound every numerator
// (x, y, 1, x y, x^2, y^2) by 2^+-300, every denominator (z, z^2) likewise,
// so the exponent gap stays below 768 and no operand, reciprocal or quotient
// is denormal or tiny.  NaN and infinity fail the comparisons.
__device__ inline bool div_safe(double x, double y, double z)
{
    constexpr double lo = 0x1p-150, hi = 0x1p150;
    const double ax = fabs(x), ay = fabs(y), az = fabs(z);
    return (ax <= hi) & ((ax >= lo) | (ax == 0.0)) & (ay <= hi) & ((ay >= lo) | (ay == 0.0)) & (az <= hi) &
           (az >= lo);
}

// The per-edge terms of one LM linearisation (computeActiveErrors +
// buildSystem): c[0] the robust chi2, c[1..21] the lower entries of
// J^T W J, c[22..27] b -- each the value g2o adds for this edge.
// Fast form (div_safe): the quotients of computeError and linearizeOplus by
// z and z^2 through two shared reciprocals, and the structural zeros
// B(0, 4) = B(1, 3) = 0 of the pose Jacobian left out of the products: a
// left-out product is +-0, and x + (+-0) = x for every x the sums can hold
// (they start at +0.0, and round-to-nearest never makes -0.0 of it), so each
// term adds the same value to every sum as g2o's.  Elsewhere the original
// expressions, division by division.
__device__ inline void pose_edge_terms(const double* pose, const Cam& cam, double delta, float fo0, float fo1, float fis,
                                       float fx_, float fy_, float fz_, double (&c)[28])
{
    const double X[3] = {(double)fx_, (double)fy_, (double)fz_};
    const double s = (double)fis;
    double pc[3], er0, er1;
    se3_map(pose, X, pc);
    if (div_safe(pc[0], pc[1], pc[2])) {
        const double x = pc[0], y = pc[1], z = pc[2], z_2 = z * z;
        const double yz = div_rcp(z), yz2 = div_rcp(z_2);
        const double x_z = div_by(x, z, yz), y_z = div_by(y, z, yz);
        const double i_z = __fma_rn(__fma_rn(-z, yz, 1.0), yz, yz);   // div_by(1, z, yz)
        er0 = (double)fo0 - (x_z * cam.fx + cam.cx);
        er1 = (double)fo1 - (y_z * cam.fy + cam.cy);
        double rho0, rho1;
        huber2(er0 * (s * er0) + er1 * (s * er1), delta, rho0, rho1);
        c[0] = rho0;
        const double fx = cam.fx, fy = cam.fy;
        const double xy_z2 = div_by(x * y, z_2, yz2);
        double B[12];
        B[0] = xy_z2 * fx;
        B[1] = -(1 + div_by(x * x, z_2, yz2)) * fx;
        B[2] = y_z * fx;
        B[3] = -i_z * fx;    // -1. / z = -(1 / z)
        B[4] = 0;
        B[5] = div_by(x, z_2, yz2) * fx;
        B[6] = (1 + div_by(y * y, z_2, yz2)) * fy;
        B[7] = -xy_z2 * fy;  // -x * y / z_2 = -(x y / z_2)
        B[8] = -x_z * fy;
        B[9] = 0;
        B[10] = -i_z * fy;
        B[11] = div_by(y, z_2, yz2) * fy;
        const double w = rho1 * s;
        const double om0 = -(s * er0) * rho1, om1 = -(s * er1) * rho1;
        int k = 1;
#pragma unroll
        for (int i = 0; i < 6; i++)
#pragma unroll
            for (int j = 0; j <= i; j++, k++) {
                const bool p0 = i == 4 || j == 4, q0 = i == 3 || j == 3;   // B(0, 4), B(1, 3) factors
                const double P = (B[i] * w) * B[j], Q = (B[6 + i] * w) * B[6 + j];
                c[k] = p0 ? (q0 ? 0.0 : Q) : (q0 ? P : P + Q);
            }
#pragma unroll
        for (int i = 0; i < 6; i++)
            c[22 + i] = i == 3 ? B[3] * om0 : (i == 4 ? B[10] * om1 : B[i] * om0 + B[6 + i] * om1);
        return;
    }
    {
        const double u = pc[0] / pc[2] * cam.fx + cam.cx;
        const double v = pc[1] / pc[2] * cam.fy + cam.cy;
        er0 = (double)fo0 - u;
        er1 = (double)fo1 - v;
    }
    double rho0, rho1;
    huber2(er0 * (s * er0) + er1 * (s * er1), delta, rho0, rho1);
    c[0] = rho0;
    const double x = pc[0], y = pc[1], z = pc[2], z_2 = z * z;
    const double fx = cam.fx, fy = cam.fy;
    double B[12];
    B[0] = x * y / z_2 * fx;
    B[1] = -(1 + (x * x / z_2)) * fx;
    B[2] = y / z * fx;
    B[3] = -1. / z * fx;
    B[4] = 0;
    B[5] = x / z_2 * fx;
    B[6] = (1 + y * y / z_2) * fy;
    B[7] = -x * y / z_2 * fy;
    B[8] = -x / z * fy;
    B[9] = 0;
    B[10] = -1. / z * fy;
    B[11] = y / z_2 * fy;
    const double w = rho1 * s;
    const double om0 = -(s * er0) * rho1, om1 = -(s * er1) * rho1;
    int k = 1;
#pragma unroll
    for (int i = 0; i < 6; i++)
#pragma unroll
        for (int j = 0; j <= i; j++, k++) c[k] = (B[i] * w) * B[j] + (B[6 + i] * w) * B[6 + j];
#pragma unroll
    for (int i = 0; i < 6; i++) c[22 + i] = B[i] * om0 + B[6 + i] * om1;
}

// kExact: every chi2, H and b sum is accumulated sequentially in g2o's
// active-edge order (OptimizationAlgorithmLevenberg / BlockSolver add edge
// by edge in insertion order): per group of 64 edges each lane writes its
// edge's terms to an LDS row, then lane q adds column q over the rows in
// edge order.  The sums -- and so every accept / reject decision and the
// whole LM trajectory -- are then those of the sequential restatement
// (oracle/ref_pose.cpp), at the cost of a 64-step dependent chain per group
// (the default; orbx_pose_set_exact(ctx, 0) selects the reassociated sums).
// An inactive edge contributes
// +0.0: the sum starts at +0.0 and round-to-nearest never yields -0.0 from
// it, so adding +0.0 leaves every bit as skipping the edge would.  The term
// rows (57 KB per workgroup) sit beside the edge cache: one workgroup per CU.
//
// kW > 1 (a single frame or a few, orbx_pose_optimization's one call): a
// workgroup of kW wavefronts per frame, the edges strided over all of its
// threads, each sum formed per wave (the DPP tree) and then over the waves in
// wave order through LDS -- deterministic, and the same LM logic on the
// same uniform data, but another summation order than the one-wave kernel.
template <bool kExact, int kW = 1>
__global__ __launch_bounds__(kW == 1 ? kPoseThreads : 64 * kW) void k_pose_opt(const PoseHdr* __restrict__ hdrs,
                                                                              PoseEdgeArrays ed,
                                                                              uint8_t* __restrict__ eflag,
                                                                              PoseOut* __restrict__ outs, int P,
                                                                              double delta)
{
    static_assert(kW == 1 || !kExact, "the exact sums run one wave per frame");
    constexpr int kT = 64 * kW;                          // threads striding one frame's edges
    constexpr int kFrames = kW == 1 ? kPoseThreads / 64 : 1;
    // kExact keeps no edges in LDS: the term rows (57 KB) and the active-edge
    // lists (16 KB) let two workgroups share a CU, so a wave's add chain
    // overlaps another's terms
    constexpr int kCache = kExact ? 1 : (kW == 1 ? kPoseLdsEdges : kPoseLdsEdgesWide);
    const int prob = kW == 1 ? blockIdx.x * (kPoseThreads / 64) + (threadIdx.x >> 6) : blockIdx.x;
    if (prob >= P) return;   // whole wavefront (kW > 1: whole workgroup)
    const int lane = kW == 1 ? threadIdx.x & 63 : threadIdx.x;   // position among the frame's threads
    const PoseHdr& H = hdrs[prob];
    const long long e0 = H.e0;
    const int nE = H.nE;
    const Cam cam{(double)H.cam[0], (double)H.cam[1], (double)H.cam[2], (double)H.cam[3]};
    // Converter::toSE3Quat (src/Converter.cc:38-48)
    double pose[7], errpose[7];
    {
        double R[9];
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int j = 0; j < 3; j++) R[i * 3 + j] = (double)H.T[i * 4 + j];
        Q q = qfrom(R);
        qnormalize(q);
        pose[0] = q.x; pose[1] = q.y; pose[2] = q.z; pose[3] = q.w;
#pragma unroll
        for (int i = 0; i < 3; i++) pose[4 + i] = (double)H.T[i * 4 + 3];
    }
#pragma unroll
    for (int i = 0; i < 7; i++) errpose[i] = pose[i];
    const float* ox = ed.ox + e0;
    const float* oy = ed.oy + e0;
    const float* isg = ed.isig + e0;
    const float* px = ed.px + e0;
    const float* py = ed.py + e0;
    const float* pz = ed.pz + e0;
    uint8_t* flag = eflag + e0;
    __shared__ float s_e[kFrames][6][kCache];
    __shared__ uint8_t s_f[kFrames][kCache];
    __shared__ double s_rows[kExact ? kPoseThreads / 64 : 1][kExact ? 64 : 1][28];   // per-edge terms
    // kExact, robust rounds 2-4: the active edges (flag 0) in edge order, so
    // the passes walk only them; an outlier adds +0.0 to every sum, so
    // leaving it out changes no bit, and ~16 % fewer groups run
    __shared__ uint16_t s_act[kExact ? kPoseThreads / 64 : 1][kExact ? kPoseActCap : 1];
    int n_list = -1;   // -1: walk every edge (round 1, or a frame over kPoseActCap edges)
    // kW > 1: per-wave sums and the solver's broadcast, in two buffers used
    // in turn, so each exchange needs one barrier (a buffer is written again
    // only after the barrier of the exchange that used the other one, which
    // every thread passes after its reads of this one)
    __shared__ double s_red[2][kW][28];
    int rb = 0;
    const int wq = kW == 1 ? threadIdx.x >> 6 : 0;
    const int nL = kExact ? 0 : min(nE, kCache);
    // sums over the frame's threads, the same double on every thread: the
    // wave's DPP tree, then (kW > 1) the waves' sums in wave order
    auto frame_sums = [&](double* v, const int n) {
#pragma unroll
        for (int k = 0; k < n; k++) v[k] = wave_sum_uniform(v[k]);
        if constexpr (kW > 1) {
            if ((threadIdx.x & 63) == 0)
#pragma unroll
                for (int k = 0; k < n; k++) s_red[rb][threadIdx.x >> 6][k] = v[k];
            __syncthreads();
#pragma unroll
            for (int k = 0; k < n; k++) {
                double t = s_red[rb][0][k];
#pragma unroll
                for (int w = 1; w < kW; w++) t += s_red[rb][w][k];
                v[k] = t;
            }
            rb ^= 1;
        }
    };
    auto frame_sum_int = [&](int v) {
        v = wave_sum_int(v);
        if constexpr (kW > 1) {
            if ((threadIdx.x & 63) == 0) s_red[rb][threadIdx.x >> 6][0] = (double)v;
            __syncthreads();
            int t = 0;
#pragma unroll
            for (int w = 0; w < kW; w++) t += (int)s_red[rb][w][0];
            rb ^= 1;
            return t;
        }
        return v;
    };
    float* lox = s_e[wq][0];
    float* loy = s_e[wq][1];
    float* lis = s_e[wq][2];
    float* lpx = s_e[wq][3];
    float* lpy = s_e[wq][4];
    float* lpz = s_e[wq][5];
    uint8_t* lfl = s_f[wq];
#pragma unroll 1
    for (int a = lane; a < nL; a += kT) {
        const float v0 = ox[a], v1 = oy[a], v2 = isg[a], v3 = px[a], v4 = py[a], v5 = pz[a];
        lox[a] = v0;
        loy[a] = v1;
        lis[a] = v2;
        lpx[a] = v3;
        lpy[a] = v4;
        lpz[a] = v5;
        lfl[a] = 0;
    }
    for (int a = nL + lane; a < nE; a += kT) flag[a] = 0;
    if constexpr (kW == 1) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    } else {
        __syncthreads();
    }
    // the frame's edges: LDS part [0, nL), global part [nL, nE); an edge
    // stays on one thread for the whole run, so its flag is thread-private
    auto for_edges = [&](auto&& body) {
#pragma unroll 1
        for (int a = lane; a < nL; a += kT)
            if (!lfl[a]) body(lox[a], loy[a], lis[a], lpx[a], lpy[a], lpz[a]);
#pragma unroll 1
        for (int a = nL + lane; a < nE; a += kT)
            if (!flag[a]) body(ox[a], oy[a], isg[a], px[a], py[a], pz[a]);
    };

    // kExact: the sequential sums of Q per-edge terms over the active edges
    // in edge order; lane q < Q returns sum q
    auto seq_sums = [&](int Q, auto&& terms) -> double {
        double acc = 0;
        double(*rows)[28] = s_rows[kExact ? wq : 0];
        const int cnt = n_list >= 0 ? n_list : nE;
#pragma unroll 1
        for (int g = 0; g < cnt; g += 64) {
            const int i = g + lane;
            double c[28];
            bool act;
            int a;
            if (n_list >= 0) {   // uniform
                act = i < cnt;
                a = act ? (int)s_act[kExact ? wq : 0][i] : 0;
            } else {
                a = i;
                act = a < nE && !flag[a];
            }
            if (act) terms(ox[a], oy[a], isg[a], px[a], py[a], pz[a], c);
            // stores in two branches, not 56 selects on every lane (the
            // empty asm keeps the compiler from merging them back into
            // selects); the zero branch runs only when some lane is idle
            if (act) {
                for (int q = 0; q < Q; q++) rows[lane][q] = c[q];
            } else {
                asm volatile("" ::: "memory");
                for (int q = 0; q < Q; q++) rows[lane][q] = 0.0;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (lane < Q) {
                // all 64 rows in two register buffers of 16, each refilled
                // right after its adds, so 16 loads are in flight while 16
                // adds run (no copies between buffers; a third buffer would
                // take the kernel past 256 VGPRs).  Rows past the frame's
                // last edge hold +0.0, which leaves the sum's bits as they
                // are (a frame's last group is nearly always full).  The
                // sched_barriers keep the compiler's scheduler from sinking
                // each load next to its add.
                double A[16], Bf[16];
#pragma unroll
                for (int k = 0; k < 16; k++) A[k] = rows[k][lane];
#pragma unroll
                for (int k = 0; k < 16; k++) Bf[k] = rows[16 + k][lane];
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int k = 0; k < 16; k++) acc += A[k];
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int k = 0; k < 16; k++) A[k] = rows[32 + k][lane];
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int k = 0; k < 16; k++) acc += Bf[k];
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int k = 0; k < 16; k++) Bf[k] = rows[48 + k][lane];
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int k = 0; k < 16; k++) acc += A[k];
#pragma unroll
                for (int k = 0; k < 16; k++) acc += Bf[k];
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        return acc;
    };

    PoseOut& out = outs[prob];
    int not_posdef = 0, rounds = 0;
    int n_active = nE;
    int nBadOut = 0;
#pragma unroll 1
    for (int it = 0; it < 4; it++) {
        // const float chi2[4]={9.210,7.378,5.991,5.991}; const int its[4]={10,10,7,5}; (:236-237)
        const float chi2th = it == 0 ? 9.210f : (it == 1 ? 7.378f : 5.991f);
        const int its = it < 2 ? 10 : (it == 2 ? 7 : 5);
        int r_iters = 0, r_trials = 0;
        double r_chi = 0;
        rounds = it + 1;
        if (n_active > 0) {
            double lambda = 0, ni = 2;
            int nBadLM = 0;
            // kExact: a trial pass sums the whole system at the trial pose
            // (lane q holds sum q), which the next iteration takes when the
            // trial is accepted -- the sums computeActiveErrors + buildSystem
            // would form there, in the same order
            double sys_sum = 0;
            bool have_sys = false;
#pragma unroll 1
            for (int iter = 0; iter < its; iter++) {
                // computeActiveErrors + activeRobustChi2 + buildSystem (fused)
                double h[21], bv[6], chi = 0;
#pragma unroll
                for (int k = 0; k < 21; k++) h[k] = 0;
#pragma unroll
                for (int k = 0; k < 6; k++) bv[k] = 0;
                double currentChi;
                if constexpr (kExact) {
                    if (!have_sys)
                        sys_sum = seq_sums(28, [&](float fo0, float fo1, float fis, float fx_, float fy_, float fz_,
                                                   double (&c)[28]) {
                            pose_edge_terms(pose, cam, delta, fo0, fo1, fis, fx_, fy_, fz_, c);
                        });
                    have_sys = false;
                    currentChi = lane_f64(sys_sum, 0);
#pragma unroll
                    for (int k = 0; k < 21; k++) h[k] = lane_f64(sys_sum, 1 + k);
#pragma unroll
                    for (int k = 0; k < 6; k++) bv[k] = lane_f64(sys_sum, 22 + k);
                } else {
                for_edges([&](float fo0, float fo1, float fis, float fx_, float fy_, float fz_) {
                    // computeError, the Huber kernel, linearizeOplus's pose
                    // block (types_six_dof_expmap.cpp:384-420) and
                    // constructQuadraticForm's toNotFixed branch
                    // (base_binary_edge.hpp:96-113): the edge's terms, added
                    double c[28];
                    pose_edge_terms(pose, cam, delta, fo0, fo1, fis, fx_, fy_, fz_, c);
                    chi += c[0];
#pragma unroll
                    for (int k = 0; k < 21; k++) h[k] += c[1 + k];
#pragma unroll
                    for (int i = 0; i < 6; i++) bv[i] += c[22 + i];
                });
                {   // chi, H and b in one exchange (each sum in the same order as alone)
                    double v[28];
                    v[0] = chi;
#pragma unroll
                    for (int k = 0; k < 21; k++) v[1 + k] = h[k];
#pragma unroll
                    for (int k = 0; k < 6; k++) v[22 + k] = bv[k];
                    frame_sums(v, 28);
                    chi = v[0];
#pragma unroll
                    for (int k = 0; k < 21; k++) h[k] = v[1 + k];
#pragma unroll
                    for (int k = 0; k < 6; k++) bv[k] = v[22 + k];
                }
                currentChi = chi;
                }
                const double iniChi = currentChi;
                if (iter == 0) {   // computeLambdaInit (levenberg.cpp:166-180)
                    double mx = 0;
#pragma unroll
                    for (int j = 0; j < 6; j++) mx = fmax(fabs(h[LT(j, j)]), mx);
                    lambda = 1e-5 * mx;
                    ni = 2;
                    nBadLM = 0;
                }
                double rho = 0;
                int qmax = 0;
                do {
                    double m[21], xs[6], tp[7];
                    bool ok2 = false;
                    // kW > 1: wave 0 alone solves and steps (the other waves
                    // would only compete for the SIMDs), then shares the result
                    if (kW == 1 || threadIdx.x < 64) {
#pragma unroll
                        for (int k = 0; k < 21; k++) m[k] = h[k];
#pragma unroll
                        for (int j = 0; j < 6; j++) m[LT(j, j)] += lambda;
                        ok2 = ldlt6_solve(m, bv, xs);
#pragma unroll
                        for (int i = 0; i < 7; i++) tp[i] = pose[i];
                        if (ok2) {
                            se3_oplus(tp, xs);
                        } else {
#pragma unroll
                            for (int i = 0; i < 6; i++) xs[i] = 0.0;
                        }
                    }
                    if constexpr (kW > 1) {
                        if (threadIdx.x == 0) {
#pragma unroll
                            for (int i = 0; i < 6; i++) s_red[rb][0][i] = xs[i];
#pragma unroll
                            for (int i = 0; i < 7; i++) s_red[rb][0][6 + i] = tp[i];
                            s_red[rb][0][13] = ok2 ? 1.0 : 0.0;
                        }
                        __syncthreads();
#pragma unroll
                        for (int i = 0; i < 6; i++) xs[i] = s_red[rb][0][i];
#pragma unroll
                        for (int i = 0; i < 7; i++) tp[i] = s_red[rb][0][6 + i];
                        ok2 = s_red[rb][0][13] != 0.0;
                        rb ^= 1;
                    }
                    if (!ok2) not_posdef++;
                    // computeActiveErrors at the trial estimate
                    auto trial_chi = [&](float fo0, float fo1, float fis, float fx_, float fy_, float fz_) {
                        const double X[3] = {(double)fx_, (double)fy_, (double)fz_};
                        const double s = (double)fis;
                        double pc[3], er0, er1;
                        pose_edge_error(tp, X, (double)fo0, (double)fo1, cam, pc, er0, er1);
                        double rho0, rho1;
                        huber2(er0 * (s * er0) + er1 * (s * er1), delta, rho0, rho1);
                        return rho0;
                    };
                    double tempChi, tsum = 0;
                    if constexpr (kExact) {
                        tsum = seq_sums(28, [&](float fo0, float fo1, float fis, float fx_, float fy_, float fz_,
                                                double (&c)[28]) {
                            pose_edge_terms(tp, cam, delta, fo0, fo1, fis, fx_, fy_, fz_, c);
                        });
                        tempChi = lane_f64(tsum, 0);
                    } else {
                        double tchi = 0;
                        for_edges([&](float fo0, float fo1, float fis, float fx_, float fy_, float fz_) {
                            tchi += trial_chi(fo0, fo1, fis, fx_, fy_, fz_);
                        });
                        frame_sums(&tchi, 1);
                        tempChi = tchi;
                    }
#pragma unroll
                    for (int i = 0; i < 7; i++) errpose[i] = tp[i];
                    if (!ok2) tempChi = 1.79769313486231570815e+308;
                    double scale = 0;
#pragma unroll
                    for (int j = 0; j < 6; j++) scale += xs[j] * (lambda * xs[j] + bv[j]);
                    scale += 1e-3;
                    rho = (currentChi - tempChi) / scale;
                    if (rho > 0 && isfinite(tempChi)) {
                        double alpha = 1. - pow((2 * rho - 1), 3);
                        alpha = fmin(alpha, 2. / 3.);
                        lambda *= fmax(1. / 3., alpha);
                        ni = 2;
                        currentChi = tempChi;
#pragma unroll
                        for (int i = 0; i < 7; i++) pose[i] = tp[i];
                        if constexpr (kExact) {
                            sys_sum = tsum;
                            have_sys = true;
                        }
                    } else {
                        lambda *= ni;
                        ni *= 2;
                    }
                    qmax++;
                } while (rho < 0 && qmax < 10);
                r_iters++;
                r_trials += qmax;
                r_chi = currentChi;
                if (qmax == 10 || rho == 0) break;
                if ((iniChi - currentChi) * 1e3 < iniChi) nBadLM++;
                else nBadLM = 0;
                if (nBadLM >= 3) break;
            }
        }
        // outlier classification (src/Optimizer.cc:243-265)
        int bad = 0, act = 0;
        const double th = (double)chi2th;
        auto classify = [&](uint8_t f, float fo0, float fo1, float fis, float fx_, float fy_, float fz_) {
            const double X[3] = {(double)fx_, (double)fy_, (double)fz_};
            const double s = (double)fis;
            double pc[3], er0, er1;
            pose_edge_error(f ? pose : errpose, X, (double)fo0, (double)fo1, cam, pc, er0, er1);
            const double c2 = er0 * (s * er0) + er1 * (s * er1);
            uint8_t nf = f;
            if (c2 > th) {
                nf = 1;
                bad++;
            } else if (c2 <= th) {
                nf = 0;
            }
            act += nf == 0;
            return nf;
        };
#pragma unroll 1
        for (int a = lane; a < nL; a += kT) lfl[a] = classify(lfl[a], lox[a], loy[a], lis[a], lpx[a], lpy[a], lpz[a]);
#pragma unroll 1
        for (int a = nL + lane; a < nE; a += kT) flag[a] = classify(flag[a], ox[a], oy[a], isg[a], px[a], py[a], pz[a]);
        nBadOut = frame_sum_int(bad);
        n_active = frame_sum_int(act);
        if constexpr (kExact) {
            // the next round's active edges, in edge order (each lane reads
            // the flags it has just written)
            if (nE <= kPoseActCap) {
                int base = 0;
#pragma unroll 1
                for (int c0 = 0; c0 < nE; c0 += 64) {
                    const int a = c0 + lane;
                    const bool on = a < nE && flag[a] == 0;
                    const uint64_t m = __builtin_amdgcn_ballot_w64(on);
                    const int r = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                    if (on) s_act[wq][base + r] = (uint16_t)a;
                    base += __popcll(m);
                }
                n_list = base;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
        }
        if (lane == 0) {
            out.iterations[it] = r_iters;
            out.trials[it] = r_trials;
            out.chi2_final[it] = r_chi;
            out.n_bad[it] = nBadOut;
        }
        if (nE < 10) break;
    }
    for (int a = lane; a < nL; a += kT) flag[a] = lfl[a];   // mvbOutlier of the LDS part
    if (lane == 0) {
        double R[9];
        qmat(Q{pose[0], pose[1], pose[2], pose[3]}, R);
#pragma unroll
        for (int i = 0; i < 3; i++) {
#pragma unroll
            for (int j = 0; j < 3; j++) out.T[i * 4 + j] = (float)R[i * 3 + j];
            out.T[i * 4 + 3] = (float)pose[4 + i];
        }
        out.n_inliers = nE - nBadOut;
        out.rounds = rounds;
        for (int r = rounds; r < 4; r++) {
            out.iterations[r] = 0;
            out.trials[r] = 0;
            out.chi2_final[r] = 0;
            out.n_bad[r] = 0;
        }
        out.not_posdef = not_posdef;
    }
}

// The exact sums (g2o's sequential edge order, bit for bit the restatement)
// for one frame per workgroup, fast.  Every sum of a pass is a chain of
// dependent FP64 adds in edge order -- the part no reassociation may
// shorten -- so the kernel keeps that chain busy and hides everything else
// behind it.  Wave 0 adds; waves 1..7 compute the per-edge terms (28
// doubles per edge: chi2, the 21 lower entries of J^T W J, b) of groups of
// 64 edges, group g on worker g % 7, into a ring of kPxSlots LDS slots
// (column-major, one column per sum, padded so lanes 0..27 of wave 0 read
// 28 different bank pairs).  Producer and consumer meet through LDS
// counters, not workgroup barriers: a worker waits until its slot's
// previous group was consumed, wave 0 until its next group is ready -- so
// seven groups are in flight while the chain runs.  A trial pass computes
// the full system at the trial pose (the next iteration's build when the
// trial is accepted).  The LM control runs on uniform values broadcast
// through LDS, the 6x6 LDLT and the exp-map step on wave 0 alone
// (orbx_pose_set_exact; see k_pose_opt for the g2o semantics every line
// below follows).
#ifdef ORBX_POSE_PROFILE
// phase stamps of k_pose_exact_wide (block 0, thread 0; wall clock, 100 MHz):
// 0 round-start builds, 1 solves, 2 trial passes, 3 classification, 4 the
// whole kernel, 5 builds, 6 trials, 7 the LDLT part of the solves
__device__ unsigned long long g_pose_prof[8];
// (accumulated in registers, written once at the kernel's end: a global
// read-modify-write per stamp would stall the wave it measures)
#define PX_T0() const unsigned long long _px_t0 = wall_clock64()
#define PX_ACC(k, t0) (px_acc[k] += wall_clock64() - (t0))
#define PX_CNT(k) (px_acc[k] += 1)
#else
#define PX_T0() (void)0
#define PX_ACC(k, t0) (void)0
#define PX_CNT(k) (void)0
#endif
constexpr int kPxWaves = 8;                   // two per SIMD (255 VGPRs)
constexpr int kPxThreads = 64 * kPxWaves;
constexpr int kPxWorkers = kPxWaves - 1;
constexpr int kPxCache = 1024;                // edges kept in LDS (25 KB)
constexpr int kPxStride = 65;                 // doubles per column of a slot (64 edges + 1 pad)
constexpr int kPxSlot = 28 * kPxStride;       // doubles per slot
constexpr int kPxSlots = 8;                   // ring depth (114 KB)

__global__ __launch_bounds__(kPxThreads) void k_pose_exact_wide(const PoseHdr* __restrict__ hdrs, PoseEdgeArrays ed,
                                                               uint8_t* __restrict__ eflag,
                                                               PoseOut* __restrict__ outs, int P, double delta)
{
    const int prob = blockIdx.x;
    if (prob >= P) return;   // whole workgroup
#ifdef ORBX_POSE_PROFILE
    const unsigned long long t_kernel = wall_clock64();
    unsigned long long px_acc[8] = {};
#endif
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const PoseHdr& H = hdrs[prob];
    const long long e0 = H.e0;
    const int nE = H.nE;
    const Cam cam{(double)H.cam[0], (double)H.cam[1], (double)H.cam[2], (double)H.cam[3]};
    double pose[7], errpose[7];
    {
        double R[9];
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int j = 0; j < 3; j++) R[i * 3 + j] = (double)H.T[i * 4 + j];
        Q q = qfrom(R);
        qnormalize(q);
        pose[0] = q.x; pose[1] = q.y; pose[2] = q.z; pose[3] = q.w;
#pragma unroll
        for (int i = 0; i < 3; i++) pose[4 + i] = (double)H.T[i * 4 + 3];
    }
#pragma unroll
    for (int i = 0; i < 7; i++) errpose[i] = pose[i];
    const float* ox = ed.ox + e0;
    const float* oy = ed.oy + e0;
    const float* isg = ed.isig + e0;
    const float* px = ed.px + e0;
    const float* py = ed.py + e0;
    const float* pz = ed.pz + e0;
    uint8_t* flag = eflag + e0;
    __shared__ float s_e[6][kPxCache];
    __shared__ uint8_t s_f[kPxCache];
    __shared__ double s_ring[kPxSlots * kPxSlot];
    __shared__ int s_ready[kPxSlots];   // ticket + 1 of the group a slot holds
    __shared__ int s_done;              // tickets consumed so far (all passes)
    __shared__ double s_sum[28];        // the pass's sums (written by wave 0 after the chain)
    __shared__ double s_sol[14];        // wave 0's step: xs, trial pose, ok
    __shared__ int s_cnt[kPxWaves][2];
    // robust rounds 2-4: the active edges in edge order (an outlier adds
    // +0.0 to every sum, so the chain skips it without changing a bit)
    __shared__ uint16_t s_act[kPoseActCap];
    int n_list = -1;   // -1: every edge (round 1, or over kPoseActCap edges)
    const int nL = min(nE, kPxCache);
    for (int a = tid; a < nL; a += kPxThreads) {
        s_e[0][a] = ox[a];
        s_e[1][a] = oy[a];
        s_e[2][a] = isg[a];
        s_e[3][a] = px[a];
        s_e[4][a] = py[a];
        s_e[5][a] = pz[a];
        s_f[a] = 0;
    }
    for (int a = nL + tid; a < nE; a += kPxThreads) flag[a] = 0;
    if (tid < kPxSlots) s_ready[tid] = 0;
    if (tid == 0) s_done = 0;
    __syncthreads();
    int ticket = 0;   // groups of all passes so far (uniform: every wave counts every pass)
    // the edge's inputs and whether it is active (not an outlier)
    auto edge = [&](int a, float& o0, float& o1, float& is, float& X, float& Y, float& Z) -> bool {
        if (a < nL) {
            o0 = s_e[0][a]; o1 = s_e[1][a]; is = s_e[2][a]; X = s_e[3][a]; Y = s_e[4][a]; Z = s_e[5][a];
            return !s_f[a];
        }
        o0 = ox[a]; o1 = oy[a]; is = isg[a]; X = px[a]; Y = py[a]; Z = pz[a];
        return !flag[a];
    };
    // Q sequential sums over the active edges in edge order (an inactive
    // edge adds +0.0, which leaves every bit: the sums start at +0.0 and
    // round-to-nearest never yields -0.0 from there); the results land in
    // s_sum[0, Q) for every thread
    auto seq_sums = [&](auto Qc, auto&& terms) {
        constexpr int Qn = decltype(Qc)::value;
        const int cnt = n_list >= 0 ? n_list : nE;
        const int G = (cnt + 63) >> 6;   // groups of 64 edges (the last padded with +0.0 rows)
        if (wave > 0) {
#pragma unroll 1
            for (int g = wave - 1; g < G; g += kPxWorkers) {
                const int tk = ticket + g, slot = tk % kPxSlots;
                // the slot's previous group (ticket tk - kPxSlots) is consumed
                // (bounded: a wait that never ends would hang the device;
                // after ~0.1 s the pass goes on with wrong sums instead)
                for (int spin = 0; *(volatile int*)&s_done < tk - kPxSlots + 1 && spin < (1 << 22); spin++)
                    __builtin_amdgcn_s_sleep(1);
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                double* buf = s_ring + slot * kPxSlot;
                const int i = g * 64 + lane;
                double t[Qn];
                float o0, o1, is, X, Y, Z;
                bool act;
                if (n_list >= 0) {   // uniform
                    act = i < cnt;
                    if (act) edge((int)s_act[i], o0, o1, is, X, Y, Z);
                } else {
                    act = i < nE && edge(i, o0, o1, is, X, Y, Z);
                }
                if (act) terms(o0, o1, is, X, Y, Z, t);
#pragma unroll
                for (int q = 0; q < Qn; q++) buf[q * kPxStride + lane] = act ? t[q] : 0.0;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                if (lane == 0) *(volatile int*)&s_ready[slot] = tk + 1;
            }
        } else {
            double acc = 0.0;
#pragma unroll 1
            for (int g = 0; g < G; g++) {
                const int tk = ticket + g, slot = tk % kPxSlots;
                for (int spin = 0; *(volatile int*)&s_ready[slot] != tk + 1 && spin < (1 << 22); spin++)
                    __builtin_amdgcn_s_sleep(1);
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                if (lane < Qn) {
                    // the chain: blocks of 8 (the group's last edge rounded
                    // up), the next block's loads issued before this block's adds
                    const double* col = s_ring + slot * kPxSlot + lane * kPxStride;
                    const int nb = min(8, (cnt - g * 64 + 7) >> 3);
                    double cur[8];
#pragma unroll
                    for (int k = 0; k < 8; k++) cur[k] = col[k];
#pragma unroll
                    for (int bk = 1; bk < 8; bk++) {
                        if (bk >= nb) break;
                        double nxt[8];
#pragma unroll
                        for (int k = 0; k < 8; k++) nxt[k] = col[8 * bk + k];
#pragma unroll
                        for (int k = 0; k < 8; k++) acc += cur[k];
#pragma unroll
                        for (int k = 0; k < 8; k++) cur[k] = nxt[k];
                    }
#pragma unroll
                    for (int k = 0; k < 8; k++) acc += cur[k];
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");   // the slot's reads are done
                if (lane == 0) *(volatile int*)&s_done = tk + 1;
            }
            if (lane < Qn) s_sum[lane] = acc;
        }
        ticket += G;
        __syncthreads();
    };
    auto block_counts = [&](int a0, int a1, int& r0, int& r1) {
        a0 = wave_sum_int(a0);
        a1 = wave_sum_int(a1);
        if (lane == 0) {
            s_cnt[wave][0] = a0;
            s_cnt[wave][1] = a1;
        }
        __syncthreads();
        r0 = r1 = 0;
#pragma unroll
        for (int w = 0; w < kPxWaves; w++) {
            r0 += s_cnt[w][0];
            r1 += s_cnt[w][1];
        }
        __syncthreads();   // s_cnt is written again by the next round
    };

    PoseOut& out = outs[prob];
    int not_posdef = 0, rounds = 0;
    int n_active = nE;
    int nBadOut = 0;
#pragma unroll 1
    for (int it = 0; it < 4; it++) {
        const float chi2th = it == 0 ? 9.210f : (it == 1 ? 7.378f : 5.991f);
        const int its = it < 2 ? 10 : (it == 2 ? 7 : 5);
        int r_iters = 0, r_trials = 0;
        double r_chi = 0;
        rounds = it + 1;
        if (n_active > 0) {
            double lambda = 0, ni = 2;
            int nBadLM = 0;
            // the system at `pose` (chi2, H, b): built at the round's start; a
            // trial pass builds it at the trial pose too, which the next
            // iteration uses when the trial is accepted -- the same sums in
            // the same order as computeActiveErrors + buildSystem there
            double h[21], bv[6], currentChi = 0;
            bool have_sys = false;
#pragma unroll 1
            for (int iter = 0; iter < its; iter++) {
                if (!have_sys) {
                    PX_T0();
                    PX_CNT(5);
                    seq_sums(std::integral_constant<int, 28>{},
                             [&](float fo0, float fo1, float fis, float fx_, float fy_, float fz_, double(&c)[28]) {
                                 pose_edge_terms(pose, cam, delta, fo0, fo1, fis, fx_, fy_, fz_, c);
                             });
                    currentChi = s_sum[0];
#pragma unroll
                    for (int k = 0; k < 21; k++) h[k] = s_sum[1 + k];
#pragma unroll
                    for (int k = 0; k < 6; k++) bv[k] = s_sum[22 + k];
                    PX_ACC(0, _px_t0);
                }
                have_sys = false;
                const double iniChi = currentChi;
                if (iter == 0) {   // computeLambdaInit (levenberg.cpp:166-180)
                    double mx = 0;
#pragma unroll
                    for (int j = 0; j < 6; j++) mx = fmax(fabs(h[LT(j, j)]), mx);
                    lambda = 1e-5 * mx;
                    ni = 2;
                    nBadLM = 0;
                }
                double rho = 0;
                int qmax = 0;
                do {
                    double xs[6], tp[7];
#ifdef ORBX_POSE_PROFILE
                    const unsigned long long t_solve = wall_clock64();
#endif
                    if (wave == 0) {
                        double m[21];
#pragma unroll
                        for (int k = 0; k < 21; k++) m[k] = h[k];
#pragma unroll
                        for (int j = 0; j < 6; j++) m[LT(j, j)] += lambda;
#ifdef ORBX_POSE_PROFILE
                        const unsigned long long t_l0 = wall_clock64();
#endif
                        const bool ok = ldlt6_solve(m, bv, xs);
#pragma unroll
                        for (int i = 0; i < 7; i++) tp[i] = pose[i];
#ifdef ORBX_POSE_PROFILE
                        PX_ACC(7, t_l0);
#endif
                        if (ok) {
                            se3_oplus(tp, xs);
                        } else {
#pragma unroll
                            for (int i = 0; i < 6; i++) xs[i] = 0.0;
                        }
                        if (lane == 0) {
#pragma unroll
                            for (int i = 0; i < 6; i++) s_sol[i] = xs[i];
#pragma unroll
                            for (int i = 0; i < 7; i++) s_sol[6 + i] = tp[i];
                            s_sol[13] = ok ? 1.0 : 0.0;
                        }
                    }
                    __syncthreads();
#pragma unroll
                    for (int i = 0; i < 6; i++) xs[i] = s_sol[i];
#pragma unroll
                    for (int i = 0; i < 7; i++) tp[i] = s_sol[6 + i];
                    const bool ok2 = s_sol[13] != 0.0;
                    PX_ACC(1, t_solve);
                    PX_T0();
                    PX_CNT(6);
                    if (!ok2) not_posdef++;
                    // computeActiveErrors at the trial estimate, with the
                    // system there (s_sol is written again only after this
                    // pass's barriers)
                    seq_sums(std::integral_constant<int, 28>{},
                             [&](float fo0, float fo1, float fis, float fx_, float fy_, float fz_, double(&c)[28]) {
                                 pose_edge_terms(tp, cam, delta, fo0, fo1, fis, fx_, fy_, fz_, c);
                             });
                    double tempChi = s_sum[0];
                    PX_ACC(2, _px_t0);
#pragma unroll
                    for (int i = 0; i < 7; i++) errpose[i] = tp[i];
                    if (!ok2) tempChi = 1.79769313486231570815e+308;
                    double scale = 0;
#pragma unroll
                    for (int j = 0; j < 6; j++) scale += xs[j] * (lambda * xs[j] + bv[j]);
                    scale += 1e-3;
                    rho = (currentChi - tempChi) / scale;
                    if (rho > 0 && isfinite(tempChi)) {
                        double alpha = 1. - pow((2 * rho - 1), 3);
                        alpha = fmin(alpha, 2. / 3.);
                        lambda *= fmax(1. / 3., alpha);
                        ni = 2;
                        currentChi = tempChi;
#pragma unroll
                        for (int i = 0; i < 7; i++) pose[i] = tp[i];
                        // the trial pass's system (s_sum stays until the
                        // next pass's last barrier)
#pragma unroll
                        for (int k = 0; k < 21; k++) h[k] = s_sum[1 + k];
#pragma unroll
                        for (int k = 0; k < 6; k++) bv[k] = s_sum[22 + k];
                        have_sys = true;
                    } else {
                        lambda *= ni;
                        ni *= 2;
                    }
                    qmax++;
                } while (rho < 0 && qmax < 10);
                r_iters++;
                r_trials += qmax;
                r_chi = currentChi;
                if (qmax == 10 || rho == 0) break;
                if ((iniChi - currentChi) * 1e3 < iniChi) nBadLM++;
                else nBadLM = 0;
                if (nBadLM >= 3) break;
            }
        }
        // outlier classification (src/Optimizer.cc:243-265)
        PX_T0();
        int bad = 0, act = 0;
        const double th = (double)chi2th;
#pragma unroll 1
        for (int a = tid; a < nE; a += kPxThreads) {
            float o0, o1, is, X, Y, Z;
            const uint8_t f = edge(a, o0, o1, is, X, Y, Z) ? 0 : 1;
            const double Xw[3] = {(double)X, (double)Y, (double)Z};
            const double sg = (double)is;
            double pc[3], er0, er1;
            pose_edge_error(f ? pose : errpose, Xw, (double)o0, (double)o1, cam, pc, er0, er1);
            const double c2 = er0 * (sg * er0) + er1 * (sg * er1);
            uint8_t nf = f;
            if (c2 > th) {
                nf = 1;
                bad++;
            } else if (c2 <= th) {
                nf = 0;
            }
            act += nf == 0;
            if (a < nL) s_f[a] = nf;
            else flag[a] = nf;
        }
        block_counts(bad, act, nBadOut, n_active);
        if (nE <= kPoseActCap) {   // uniform: the next round's list, by wave 0
            if (wave == 0) {
                int base = 0;
#pragma unroll 1
                for (int c0 = 0; c0 < nE; c0 += 64) {
                    const int a = c0 + lane;
                    const bool on = a < nE && (a < nL ? s_f[a] : flag[a]) == 0;
                    const uint64_t m = __builtin_amdgcn_ballot_w64(on);
                    const int r = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                    if (on) s_act[base + r] = (uint16_t)a;
                    base += __popcll(m);
                }
            }
            n_list = n_active;   // the same count (block_counts)
            __syncthreads();
        }
        PX_ACC(3, _px_t0);
        if (tid == 0) {
            out.iterations[it] = r_iters;
            out.trials[it] = r_trials;
            out.chi2_final[it] = r_chi;
            out.n_bad[it] = nBadOut;
        }
        if (nE < 10) break;
    }
    for (int a = tid; a < nL; a += kPxThreads) flag[a] = s_f[a];   // mvbOutlier of the LDS part
    if (tid == 0) {
        double R[9];
        qmat(Q{pose[0], pose[1], pose[2], pose[3]}, R);
#pragma unroll
        for (int i = 0; i < 3; i++) {
#pragma unroll
            for (int j = 0; j < 3; j++) out.T[i * 4 + j] = (float)R[i * 3 + j];
            out.T[i * 4 + 3] = (float)pose[4 + i];
        }
        out.n_inliers = nE - nBadOut;
        out.rounds = rounds;
        for (int r = rounds; r < 4; r++) {
            out.iterations[r] = 0;
            out.trials[r] = 0;
            out.chi2_final[r] = 0;
            out.n_bad[r] = 0;
        }
        out.not_posdef = not_posdef;
    }
#ifdef ORBX_POSE_PROFILE
    PX_ACC(4, t_kernel);
    if (blockIdx.x == 0 && threadIdx.x == 0)
        for (int k = 0; k < 8; k++) g_pose_prof[k] += px_acc[k];
#endif
}

namespace {
inline size_t align256(size_t b) { return (b + 255) & ~size_t(255); }

template <typename Fn>
void pose_parallel(int n, Fn fn)
{
    const int nth = std::max(1, std::min<int>(n / 64 + 1, std::min(16u, std::max(1u, std::thread::hardware_concurrency()))));
    if (nth == 1) {
        for (int i = 0; i < n; i++) fn(i);
        return;
    }
    std::vector<std::thread> pool;
    for (int t = 0; t < nth; t++)
        pool.emplace_back([&, t]() {
            for (int i = t; i < n; i += nth) fn(i);
        });
    for (auto& th : pool) th.join();
}
}  // namespace

}  // namespace orbx

using namespace orbx;

// sync: wait for the upload (orbx_pose_stage: the caller may stage again
// before running; the one-call batch below runs and fetches on the same
// stream, which orders the copies, and its host threads touch the buffer
// only after the fetch's synchronisation)
static int pose_stage_impl(orbx_ctx* ctx, int P, const orbx_pose_frame* frames, bool sync)
{
    if (!ctx || P < 0 || (P > 0 && !frames)) return ORBX_ERR_ARG;
    std::vector<long long> e0(P + 1, 0);
    for (int i = 0; i < P; i++) {
        const orbx_pose_frame& f = frames[i];
        if (f.n < 0 || (f.n > 0 && (!f.kp_un || !f.octave || !f.has_mp || !f.mp_xyz || !f.outlier)) ||
            f.nlevels <= 0 || !f.inv_level_sigma2)
            return ORBX_ERR_ARG;
        long long c = 0;
        for (int k = 0; k < f.n; k++)
            if (f.has_mp[k]) {
                if (f.octave[k] < 0 || f.octave[k] >= f.nlevels) return ORBX_ERR_ARG;
                c++;
            }
        e0[i + 1] = e0[i] + c;
    }
    const long long E = e0[P];
    ctx_enter(ctx);
    // layout: hdr[P] | 6 float edge arrays [E] | flags u8 [E] | out[P]
    const size_t o_hdr = 0;
    const size_t o_edges = align256(sizeof(PoseHdr) * (size_t)std::max(P, 1));
    const size_t arr = align256(4 * (size_t)std::max<long long>(E, 1));
    const size_t o_flags = o_edges + 6 * arr;
    const size_t o_out = o_flags + align256((size_t)std::max<long long>(E, 1));
    const size_t out_bytes = sizeof(PoseOut) * (size_t)std::max(P, 1);
    const size_t total = o_out + align256(out_bytes);
    const size_t staged = o_flags;                                  // copied H2D
    const size_t host_need = std::max(staged, o_out - o_flags + out_bytes);   // fetch: flags | outputs, one copy
    if (total > ctx->pose_dev_bytes) {
        if (ctx->pose_dev) (void)hipFree(ctx->pose_dev);
        ctx->pose_dev = nullptr;
        ctx->pose_dev_bytes = 0;
        if (hipMalloc(&ctx->pose_dev, total) != hipSuccess) return ORBX_ERR_NOMEM;
        ctx->pose_dev_bytes = total;
    }
    if (host_need > ctx->pose_host_bytes) {
        if (ctx->pose_host) (void)hipHostFree(ctx->pose_host);
        ctx->pose_host = nullptr;
        ctx->pose_host_bytes = 0;
        if (hipHostMalloc(&ctx->pose_host, host_need, hipHostMallocDefault) != hipSuccess) return ORBX_ERR_NOMEM;
        ctx->pose_host_bytes = host_need;
    }
    uint8_t* hb = static_cast<uint8_t*>(ctx->pose_host);
    ctx->pose_edge_kp.assign((size_t)E, 0);
    PoseHdr* hd = reinterpret_cast<PoseHdr*>(hb + o_hdr);
    float* arrs[6];
    for (int k = 0; k < 6; k++) arrs[k] = reinterpret_cast<float*>(hb + o_edges + k * arr);
    pose_parallel(P, [&](int i) {
        const orbx_pose_frame& f = frames[i];
        PoseHdr& h = hd[i];
        h.e0 = e0[i];
        h.nE = (int)(e0[i + 1] - e0[i]);
        h.pad = 0;
        for (int r = 0; r < 3; r++)
            for (int c = 0; c < 4; c++) h.T[r * 4 + c] = f.Tcw[r * 4 + c];
        for (int c = 0; c < 4; c++) h.cam[c] = f.cam[c];
        long long e = e0[i];
        for (int k = 0; k < f.n; k++) {
            if (!f.has_mp[k]) continue;
            arrs[0][e] = f.kp_un[2 * k];
            arrs[1][e] = f.kp_un[2 * k + 1];
            arrs[2][e] = f.inv_level_sigma2[f.octave[k]];
            arrs[3][e] = f.mp_xyz[3 * k];
            arrs[4][e] = f.mp_xyz[3 * k + 1];
            arrs[5][e] = f.mp_xyz[3 * k + 2];
            ctx->pose_edge_kp[e] = k;
            e++;
        }
    });
    ORBX_HIP_CHECK(hipMemcpyAsync(ctx->pose_dev, hb, staged, hipMemcpyHostToDevice, ctx->stream));
    if (sync) ORBX_HIP_CHECK(hipStreamSynchronize(ctx->stream));   // the pinned buffer is reused by fetch
    ctx->pose_P = P;
    ctx->pose_E = E;
    ctx->pose_o_flags = o_flags;
    ctx->pose_o_out = o_out;
    ctx->pose_out_bytes = out_bytes;
    ctx->pose_e0 = e0;
    ctx->pose_ran = false;
    return ORBX_OK;
}

extern "C" int orbx_pose_stage(orbx_ctx* ctx, int P, const orbx_pose_frame* frames)
{
    return pose_stage_impl(ctx, P, frames, true);
}

namespace orbx {
// P frames whose headers, edges, flags and outputs are already in device
// memory (the tracking chain builds them on the device): the launch
// orbx_pose_run makes (the same kernel selection).
int launch_pose_device(orbx_ctx* ctx, const PoseHdr* hdrs, const PoseEdgeArrays& ed, uint8_t* flags, PoseOut* outs,
                       int P)
{
    const double delta = (double)(float)std::sqrt(5.991);   // const float delta = sqrt(5.991) (:188)
    const int per = kPoseThreads / 64;
    const bool wide = P <= ctx->pose_wide_max;
    if (ctx->pose_exact && wide) {
        k_pose_exact_wide<<<P, kPxThreads, 0, ctx->stream>>>(hdrs, ed, flags, outs, P, delta);
    } else {
        auto kern = ctx->pose_exact ? k_pose_opt<true>
                                    : (wide ? k_pose_opt<false, kPoseWideWaves> : k_pose_opt<false>);
        const int blocks = wide && !ctx->pose_exact ? P : (P + per - 1) / per;
        const int threads = wide && !ctx->pose_exact ? 64 * kPoseWideWaves : kPoseThreads;
        kern<<<blocks, threads, 0, ctx->stream>>>(hdrs, ed, flags, outs, P, delta);
    }
    ORBX_HIP_CHECK(hipGetLastError());
    return ORBX_OK;
}
}  // namespace orbx

#ifdef ORBX_POSE_PROFILE
extern "C" int orbx_debug_pose_prof(unsigned long long* out, int reset)
{
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pose_prof), sizeof(unsigned long long) * 8) != hipSuccess) return -2;
    if (reset) {
        const unsigned long long z[8] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_pose_prof), z, sizeof(z)) != hipSuccess) return -2;
    }
    return 0;
}
#endif

extern "C" int orbx_pose_run(orbx_ctx* ctx)
{
    if (!ctx || !ctx->pose_dev) return ORBX_ERR_ARG;
    ctx_enter(ctx);
    const int P = ctx->pose_P;
    ctx->pose_ran = true;
    if (P == 0) return ORBX_OK;
    uint8_t* d = static_cast<uint8_t*>(ctx->pose_dev);
    const size_t arr = align256(4 * (size_t)std::max<long long>(ctx->pose_E, 1));
    const size_t o_edges = align256(sizeof(PoseHdr) * (size_t)std::max(P, 1));
    PoseEdgeArrays ed;
    ed.ox = reinterpret_cast<const float*>(d + o_edges);
    ed.oy = reinterpret_cast<const float*>(d + o_edges + arr);
    ed.isig = reinterpret_cast<const float*>(d + o_edges + 2 * arr);
    ed.px = reinterpret_cast<const float*>(d + o_edges + 3 * arr);
    ed.py = reinterpret_cast<const float*>(d + o_edges + 4 * arr);
    ed.pz = reinterpret_cast<const float*>(d + o_edges + 5 * arr);
    timer_begin(ctx, "pose");
    // a lone frame (the reference's one call per frame) gets a workgroup of
    // several wavefronts; batches a wavefront per frame
    const int lr = launch_pose_device(ctx, reinterpret_cast<const PoseHdr*>(d), ed, d + ctx->pose_o_flags,
                                      reinterpret_cast<PoseOut*>(d + ctx->pose_o_out), P);
    if (lr != ORBX_OK) return lr;
    timer_end(ctx, "pose");
    ORBX_HIP_CHECK(hipGetLastError());
    return ORBX_OK;
}

extern "C" int orbx_pose_fetch(orbx_ctx* ctx, orbx_pose_frame* frames, int32_t* n_inliers, orbx_pose_stats* stats)
{
    if (!ctx || !ctx->pose_ran || (ctx->pose_P > 0 && !frames)) return ORBX_ERR_ARG;
    ctx_enter(ctx);
    const int P = ctx->pose_P;
    if (P == 0) return ORBX_OK;
    uint8_t* hb = static_cast<uint8_t*>(ctx->pose_host);
    uint8_t* d = static_cast<uint8_t*>(ctx->pose_dev);
    // flags and outputs are adjacent on the device: one copy
    const size_t span = ctx->pose_o_out - ctx->pose_o_flags + ctx->pose_out_bytes;
    ORBX_HIP_CHECK(hipMemcpyAsync(hb, d + ctx->pose_o_flags, span, hipMemcpyDeviceToHost, ctx->stream));
    ORBX_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    const PoseOut* outs = reinterpret_cast<const PoseOut*>(hb + (ctx->pose_o_out - ctx->pose_o_flags));
    const uint8_t* flags = hb;
    pose_parallel(P, [&](int i) {
        orbx_pose_frame& f = frames[i];
        const PoseOut& o = outs[i];
        for (int r = 0; r < 3; r++)
            for (int c = 0; c < 4; c++) f.Tcw[r * 4 + c] = o.T[r * 4 + c];
        f.Tcw[12] = 0.f;
        f.Tcw[13] = 0.f;
        f.Tcw[14] = 0.f;
        f.Tcw[15] = 1.f;
        for (long long e = ctx->pose_e0[i]; e < ctx->pose_e0[i + 1]; e++) f.outlier[ctx->pose_edge_kp[e]] = flags[e];
        if (n_inliers) n_inliers[i] = o.n_inliers;
        if (stats) {
            orbx_pose_stats& s = stats[i];
            s.rounds = o.rounds;
            for (int r = 0; r < 4; r++) {
                s.iterations[r] = o.iterations[r];
                s.levenberg_trials[r] = o.trials[r];
                s.n_bad[r] = o.n_bad[r];
                s.chi2_final[r] = o.chi2_final[r];
            }
            s.not_posdef = o.not_posdef;
        }
    });
    return ORBX_OK;
}

extern "C" int orbx_pose_optimization_batch(orbx_ctx* ctx, int P, orbx_pose_frame* frames, int32_t* n_inliers,
                                            orbx_pose_stats* stats)
{
    int r = pose_stage_impl(ctx, P, frames, false);
    if (r != ORBX_OK) return r;
    if ((r = orbx_pose_run(ctx)) != ORBX_OK) return r;
    return orbx_pose_fetch(ctx, frames, n_inliers, stats);
}

extern "C" int orbx_pose_set_exact(orbx_ctx* ctx, int exact)
{
    if (!ctx || exact < 0 || exact > 1) return ORBX_ERR_ARG;
    ctx->pose_exact = exact != 0;
    return ORBX_OK;
}

extern "C" int orbx_pose_get_exact(const orbx_ctx* ctx)
{
    return ctx ? (ctx->pose_exact ? 1 : 0) : ORBX_ERR_ARG;
}

extern "C" int orbx_pose_optimization(orbx_ctx* ctx, orbx_pose_frame* f, int* n_inliers, orbx_pose_stats* stats)
{
    if (!f) return ORBX_ERR_ARG;
    int32_t n = 0;
    const int r = orbx_pose_optimization_batch(ctx, 1, f, &n, stats);
    if (r == ORBX_OK && n_inliers) *n_inliers = n;
    return r;
}
