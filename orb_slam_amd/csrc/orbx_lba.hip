// Local bundle adjustment on MI355X (FP64): the inner loop of
// Optimizer::LocalBundleAdjustment (src/Optimizer.cc:287-536) on the g2o
// subset it uses (BlockSolverX + Schur over the points, Levenberg).
//
// Layout.  A problem's active edges are stored point-major: each active
// point's edges contiguous, in the caller's edge order, as 16-byte records
// (observation and information as the floats the reference has --
// cv::KeyPoint::pt, KeyFrame::mvInvLevelSigma2 -- whenever every value of the
// batch is a float, else 32-byte double records), so the passes that walk a
// point's edges (errors, linearisation, Schur complement, back-substitution)
// stream them; a per-free-pose list of (record, point) pairs serves the pose
// blocks of the linearisation.  The poses (quaternion, translation, rotation
// matrix, camera) of the problem live in LDS for the whole launch.
//
// Device work per LM iteration (one 512-thread workgroup per problem; one
// launch per iteration when the caller passes abort flags, polled between
// iterations exactly where SparseOptimizer::optimize polls terminate(), else
// one launch per optimize() pass):
//   errors    EdgeSE3ProjectXYZ::computeError per edge, Huber robust chi2 --
//             only in an optimize() call's first iteration: every later
//             iteration starts at the state the previous iteration's accepted
//             trial just evaluated, bit for bit
//   linearize EdgeSE3ProjectXYZ::linearizeOplus + constructQuadraticForm: per
//             point (Hll, bl) one thread in edge order; per pose (Hpp, bp)
//             one wave with a fixed butterfly reduction
//   trial     Schur point by point (thread per point, its free-pose edges):
//             Dinv, db, then bs -= W_i db and S(i,j) -= W_i Dinv W_j^T for
//             every pair, W_i = B_i^T w A_i never formed (the pair's 6x6
//             block as (w B_i)^T [(A_i Dinv) A_j^T] (w B_j)).  The reduced
//             camera system is accumulated in scaled fixed point with 64-bit
//             integer atomics (two limbs per entry, packed lower triangle in
//             LDS): integer sums do not depend on the order the points arrive
//             in, so the result is bitwise reproducible (g2o sums the points
//             sequentially in double; the two differ by rounding only).
//             Dense LLT on the packed triangle; one-wave triangular solves;
//             exp-map update of the poses; then one pass per point does the
//             back-substitution, the point update and the trial's errors
//             (computeActiveErrors) together; accept / reject with g2o's rho
//             rule
//   Raul stop rule (levenberg.cpp:154-161)
// Index structures (g2o's initializeOptimization / buildStructure) are built
// on the device: k_lba_build for the first optimize() call, k_lba_rebuild
// (order-preserving filters) for the second.
#include <algorithm>
#include <cmath>
#include <cstddef>
#include <cstring>
#include <thread>
#include <vector>

#include "orbx_device.h"
#include "orbx_internal.h"
#include "orbx_se3.h"

namespace orbx {

// Race / call-boundary checks (diagnostic builds, tools/lba_race_check.py):
//  -DORBX_LBA_NOINLINE: every device function of this file is a real call
//   (the form in which round 4's dropped pose-pair Schur went wrong);
//  -DORBX_LBA_PERTURB: after every workgroup barrier each wave sleeps a
//   pseudo-random 0..~2k cycles (wave, workgroup and clock hashed), so the
//   phases between barriers run in other interleavings.  A missing barrier or
//   an LDS overlap between phases then changes bits; the product build and
//   both variants must give the same bits.
#ifdef ORBX_LBA_NOINLINE
#define LBA_FN __device__ __noinline__
#else
#define LBA_FN __device__ __forceinline__
#endif
#ifdef ORBX_LBA_PERTURB
__device__ __forceinline__ void lba_perturb()
{
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t));
    unsigned h = (unsigned)t * 2654435761u ^ (threadIdx.x >> 6) * 40503u ^ blockIdx.x * 9973u;
    h ^= h >> 13;
    for (unsigned k = h & 31; k > 0; k--) __builtin_amdgcn_s_sleep(1);
}
#define LBA_SYNC()      \
    do {                \
        __syncthreads(); \
        lba_perturb();  \
    } while (0)
#else
#define LBA_SYNC() __syncthreads()
#endif

// Active edge, point-major.  pose: index into the problem's poses; ph: its
// pose block (free poses in g2o id order) or -1 for a fixed pose.
struct EdgeRecF {
    float ox, oy, isig;
    uint16_t pose;
    int16_t ph;
};
struct EdgeRecD {
    double ox, oy, isig;
    uint16_t pose;
    int16_t ph;
    int32_t pad;
};
static_assert(sizeof(EdgeRecF) == 16 && sizeof(EdgeRecD) == 32, "edge record layout");

struct LbaDev {
    int nP, nL, nE;                // free poses, active points, active edges
    int nposes_all, npoints_all, nedges_all;
    int dim_p;                     // 6 * nP
    double* pose;                  // [nposes_all][7]: qx qy qz qw tx ty tz
    double* point;                 // [npoints_all][3]
    double* point_bk;              // [nL][3] active points before the trial
    const double* cam;             // [nposes_all][4]
    // active edges, point-major (active point l's edges: le_ptr[l] .. le_ptr[l + 1])
    const void* rec;               // EdgeRecF / EdgeRecD [nE]
    const int* e_orig;             // [nE] caller's edge index
    const int* iv_pose;            // [nP] pose index of each free pose block
    const int* iv_point;           // [nL] point index of each active point (g2o id order)
    const int* le_ptr;             // [nL + 1]
    const int* pe_ptr;             // [nP + 1]
    const int2* pe_idx;            // per free pose, its edges in edge order: (record, point index)
    double* err;                   // [nedges_all][2] last computed errors (caller's index)
    double* ew;                    // [nE] robust weight rho' * invSigma2 of the linearisation
    // scratch
    int* ce;                       // points by edge count (iteration kernel); build / rebuild maps
    double* hp;                    // [nP][27]: Hpp upper 21 | bp 6
    double* hl;                    // [nL][9]: Hll upper 6 | bl 3
    double* dl;                    // [nL][12]: Dinv | db of the trial
    double* S;                     // reduced system, lba_sys_doubles(dim_p) (global fallback of the LDS copy)
    // the caller's problem arrays (staged; read by k_lba_build only)
    const int* r_edge_pose;
    const int* r_edge_point;
    const double* r_edge_obs;
    const double* r_edge_isig;
    const uint8_t* r_pose_fixed;
    const long long* r_pose_id;
    const long long* r_point_id;
    double huber_delta;
    // LM state
    double lambda, ni, current_chi, last_chi, chi2_initial;
    double hmax, bmax;             // this linearisation's max Hpp diagonal and max |b| (fixed-point scales)
    int nBad, status, iterations, trials, not_posdef;
    int abort;
};

enum { kRunning = 0, kTerminated = 1 };

// One optimize() pass's statistics of one problem, written by k_lba_outliers
// after the pass into the readback block (one copy brings back the results,
// the flags and these).
struct LbaStatRec {
    int iterations, trials, not_posdef, pad;
    double chi2_initial, last_chi;
};

// Phase timing of block 0 (diagnostic build only: -DORBX_LBA_PROFILE).
#ifdef ORBX_LBA_PROFILE
__device__ unsigned long long g_lba_prof[32];
LBA_FN unsigned long long lba_stamp()
{
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
// per-wave phase stamps of llt_solve (k_llt_bench, block 0): work / barrier
// wait of the panel phase, work / wait of the trailing phase
__device__ unsigned long long g_llt_wave[8][4];
#define LLT_W0() unsigned long long _w = lba_stamp()
#define LLT_W(k)                                                                                \
    do {                                                                                        \
        const unsigned long long _n = lba_stamp();                                              \
        if (blockIdx.x == 0 && (threadIdx.x & 63) == 0) atomicAdd(&g_llt_wave[threadIdx.x >> 6][k], _n - _w); \
        _w = _n;                                                                                \
    } while (0)
#ifdef ORBX_LBA_NOMARKS   // the microbenchmarks without the phase marks
#define LBA_T0()
#define LBA_MARK(k)
#else
#define LBA_T0() unsigned long long _t = lba_stamp()
#define LBA_MARK(k)                                                         \
    do {                                                                    \
        LBA_SYNC();                                                    \
        const unsigned long long _n = lba_stamp();                          \
        if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&g_lba_prof[k], _n - _t); \
        _t = _n;                                                            \
    } while (0)
#endif
#else
#define LBA_T0()
#define LBA_MARK(k)
#define LLT_W0()
#define LLT_W(k)
#endif

constexpr int kLbaThreads = 512;               // one workgroup (8 waves) per problem: the phases need up to 255 VGPRs
constexpr int kLbaWaves = kLbaThreads / 64;
constexpr int kPz = 20;                        // LDS doubles per pose: q(4) t(3) R(9) cam(4)
constexpr int kPbk = 16;                       // LDS doubles per free-pose backup: q(4) t(3) R(9)

// ---------------------------------------------------------------------------
// Block reductions in double
// ---------------------------------------------------------------------------
struct DScratch {
    double w[kLbaWaves];
};

LBA_FN double wave_sum_d(double v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

LBA_FN double wave_max_d(double v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
    return v;
}

LBA_FN double block_sum_d(double v, DScratch& s)
{
    v = wave_sum_d(v);
    LBA_SYNC();
    if ((threadIdx.x & 63) == 0) s.w[threadIdx.x >> 6] = v;
    LBA_SYNC();
    double t = 0;
    for (int i = 0; i < kLbaWaves; i++) t += s.w[i];
    return t;
}

LBA_FN double block_max_d(double v, DScratch& s)
{
    v = wave_max_d(v);
    LBA_SYNC();
    if ((threadIdx.x & 63) == 0) s.w[threadIdx.x >> 6] = v;
    LBA_SYNC();
    double t = s.w[0];
    for (int i = 1; i < kLbaWaves; i++) t = fmax(t, s.w[i]);
    return t;
}

// ---------------------------------------------------------------------------
// Edge algebra (pose z in the LDS layout: q at z[0..3], t at z[4..6], the
// rotation matrix at z[7..15], fx fy cx cy at z[16..19])
// ---------------------------------------------------------------------------
LBA_FN void huber(double e2, double delta, double* rho0, double* rho1)
{
    const double dsqr = delta * delta;
    if (e2 <= dsqr) {
        *rho0 = e2;
        *rho1 = 1.;
    } else {
        const double sq = sqrt(e2);
        *rho0 = 2 * sq * delta - dsqr;
        *rho1 = delta / sq;
    }
}

// EdgeSE3ProjectXYZ::computeError (types_six_dof_expmap.h:172-177) with
// cam_project (.cpp:422-428): e = obs - (fx X / Z + cx, fy Y / Z + cy)
LBA_FN void residual(const double* c, const double (&pc)[3], double ox, double oy, double& e0, double& e1)
{
    e0 = ox - (pc[0] / pc[2] * c[0] + c[2]);
    e1 = oy - (pc[1] / pc[2] * c[1] + c[3]);
}

// EdgeSE3ProjectXYZ::linearizeOplus (types_six_dof_expmap.cpp:384-420) at
// camera-frame point pc: A = d e / d point (2x3) with the pose's rotation R,
// the reference's divisions by z and z^2 as products with 1/z (one division
// per edge; the values differ from g2o's in rounding only).
LBA_FN void jac_point(const double* c, const double* R, const double (&pc)[3], double (&A)[6])
{
    const double iz = 1. / pc[2];
    const double fx = c[0], fy = c[1];
    const double s = -iz;
    const double t0 = s * fx, t2 = s * (-(pc[0] * iz) * fx), t4 = s * fy, t5 = s * (-(pc[1] * iz) * fy);
#pragma unroll
    for (int j = 0; j < 3; j++) {
        A[j] = t0 * R[j] + t2 * R[6 + j];
        A[3 + j] = t4 * R[3 + j] + t5 * R[6 + j];
    }
}

// B = d e / d pose (2x6), update order [omega(3), upsilon(3)]
LBA_FN void jac_pose(const double* c, const double (&pc)[3], double (&B)[12])
{
    const double x = pc[0], y = pc[1];
    const double iz = 1. / pc[2], iz2 = iz * iz;
    const double fx = c[0], fy = c[1];
    B[0] = x * y * iz2 * fx;
    B[1] = -(1 + (x * x * iz2)) * fx;
    B[2] = y * iz * fx;
    B[3] = -iz * fx;
    B[4] = 0;
    B[5] = x * iz2 * fx;
    B[6] = (1 + y * y * iz2) * fy;
    B[7] = -x * y * iz2 * fy;
    B[8] = -x * iz * fy;
    B[9] = 0;
    B[10] = -iz * fy;
    B[11] = y * iz2 * fy;
}

template <class Rec>
LBA_FN Rec load_rec(const LbaDev& P, int j)
{
    return reinterpret_cast<const Rec*>(P.rec)[j];
}

LBA_FN void load_point(const double* p, double (&v)[3])
{
    v[0] = p[0];
    v[1] = p[1];
    v[2] = p[2];
}

LBA_FN void map_point(const double* z, const double (&p)[3], double (&pc)[3])
{
    se3_map(z, p, pc);   // SE3Quat::map: q p + t
}

// Errors of point l's edges at the current poses (LDS) and the point value
// pt; writes P.err, returns the summed robust chi2 (computeActiveErrors +
// activeRobustChi2 of these edges)
template <class Rec>
LBA_FN double point_errors(LbaDev& P, const double* pz, int l, const double (&pt)[3])
{
    double part = 0;
    for (int j = P.le_ptr[l]; j < P.le_ptr[l + 1]; j++) {
        const Rec r = load_rec<Rec>(P, j);
        const double* z = pz + kPz * r.pose;
        double pc[3], e0, e1;
        map_point(z, pt, pc);
        residual(z + 16, pc, (double)r.ox, (double)r.oy, e0, e1);
        const int e = P.e_orig[j];
        P.err[2 * e] = e0;
        P.err[2 * e + 1] = e1;
        const double s = (double)r.isig;
        double r0, r1;
        huber(e0 * (s * e0) + e1 * (s * e1), P.huber_delta, &r0, &r1);
        part += r0;
    }
    return part;
}

// computeActiveErrors + activeRobustChi2 over every active point.  Points
// in index order, a fixed share per thread: the double sum is the same on
// every run (the count-sorted order of the Schur pass is not fixed within a
// count).
template <class Rec>
LBA_FN double compute_errors(LbaDev& P, const double* pz, DScratch& sc)
{
    double part = 0;
    for (int l = threadIdx.x; l < P.nL; l += kLbaThreads) {
        double pt[3];
        load_point(P.point + 3 * P.iv_point[l], pt);
        part += point_errors<Rec>(P, pz, l, pt);
    }
    return block_sum_d(part, sc);
}

LBA_FN int up6(int i, int j) { return i * 6 - (i * (i - 1)) / 2 + (j - i); }   // i <= j
LBA_FN int up3(int i, int j) { return i * 3 - (i * (i - 1)) / 2 + (j - i); }
// packed lower triangle: element (i, j), j <= i
LBA_FN int pk(int i, int j) { return i * (i + 1) / 2 + j; }

// constructQuadraticForm (base_binary_edge.hpp:55-120) split by owner:
//  - per point (one thread, its edges in edge order): Hll += A^T W A,
//    bl += A^T (-Omega e); the robust weight W = rho' Omega kept per edge for
//    the trial (ew)
//  - per free pose (one wave, lanes stride the pose's edges in edge order,
//    fixed butterfly reduction): Hpp += B^T W B, bp += B^T (-Omega e).
// The errors are recomputed from the state (the values compute_errors left
// in P.err, bit for bit).  Also the largest |Hpp| diagonal and |b| entry
// (the fixed-point scales of the trials).
// One point's share (thread per point, its edges in edge order): Hll, bl
// into P.hl, the robust weights into P.ew; returns max |bl|.
template <class Rec>
LBA_FN double point_linearize(LbaDev& P, const double* pz, int l, double (&acc)[9])
{
    double pt[3];
    load_point(P.point + 3 * P.iv_point[l], pt);
#pragma unroll
    for (int v = 0; v < 9; v++) acc[v] = 0.0;
    for (int j = P.le_ptr[l]; j < P.le_ptr[l + 1]; j++) {
        const Rec r = load_rec<Rec>(P, j);
        const double* z = pz + kPz * r.pose;
        double pc[3], e0, e1, A[6];
        map_point(z, pt, pc);
        residual(z + 16, pc, (double)r.ox, (double)r.oy, e0, e1);
        jac_point(z + 16, z + 7, pc, A);
        const double sg = (double)r.isig;
        double r0, r1;
        huber(e0 * (sg * e0) + e1 * (sg * e1), P.huber_delta, &r0, &r1);
        const double w = r1 * sg, om0 = -(sg * e0) * r1, om1 = -(sg * e1) * r1;
        P.ew[j] = w;
        int k = 0;
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int c = i; c < 3; c++) acc[k++] += (A[i] * w) * A[c] + (A[3 + i] * w) * A[3 + c];
#pragma unroll
        for (int i = 0; i < 3; i++) acc[6 + i] += A[i] * om0 + A[3 + i] * om1;
    }
#pragma unroll
    for (int v = 0; v < 9; v++) P.hl[9 * l + v] = acc[v];
    return fmax(fabs(acc[6]), fmax(fabs(acc[7]), fabs(acc[8])));
}

// One free pose's share (one wave, lanes stride the pose's edges in edge
// order, fixed butterfly reduction): Hpp, bp into P.hp.  hm / bm take the
// largest |diagonal| and |bp|; every lane ends with the same values.
template <class Rec>
LBA_FN void pose_linearize(LbaDev& P, const double* pz, int p, double& hm, double& bm)
{
    const int lane = threadIdx.x & 63;
    const double* z = pz + kPz * P.iv_pose[p];
    double acc[27];
#pragma unroll
    for (int v = 0; v < 27; v++) acc[v] = 0.0;
    for (int q = P.pe_ptr[p] + lane; q < P.pe_ptr[p + 1]; q += 64) {
        const int2 ent = P.pe_idx[q];
        const Rec r = load_rec<Rec>(P, ent.x);
        double pt[3];
        load_point(P.point + 3 * ent.y, pt);
        double pc[3], e0, e1, B[12];
        map_point(z, pt, pc);
        residual(z + 16, pc, (double)r.ox, (double)r.oy, e0, e1);
        jac_pose(z + 16, pc, B);
        const double sg = (double)r.isig;
        double r0, r1;
        huber(e0 * (sg * e0) + e1 * (sg * e1), P.huber_delta, &r0, &r1);
        const double w = r1 * sg, om0 = -(sg * e0) * r1, om1 = -(sg * e1) * r1;
        int k = 0;
#pragma unroll
        for (int i = 0; i < 6; i++)
#pragma unroll
            for (int c = i; c < 6; c++) acc[k++] += (B[i] * w) * B[c] + (B[6 + i] * w) * B[6 + c];
#pragma unroll
        for (int i = 0; i < 6; i++) acc[21 + i] += B[i] * om0 + B[6 + i] * om1;
    }
#pragma unroll
    for (int v = 0; v < 27; v++) {
        const double t = wave_sum_d(acc[v]);
        if (lane == 0) P.hp[27 * p + v] = t;
        // diagonal of the packed upper 6x6 (row-major): 0, 6, 11, 15, 18, 20
        if (v == 0 || v == 6 || v == 11 || v == 15 || v == 18 || v == 20) hm = fmax(hm, fabs(t));
        else if (v >= 21) bm = fmax(bm, fabs(t));
    }
}

// constructQuadraticForm (base_binary_edge.hpp:55-120) split by owner:
//  - per point (one thread, its edges in edge order): Hll += A^T W A,
//    bl += A^T (-Omega e); the robust weight W = rho' Omega kept per edge for
//    the trial (ew)
//  - per free pose (one wave, lanes stride the pose's edges in edge order,
//    fixed butterfly reduction): Hpp += B^T W B, bp += B^T (-Omega e).
// The errors are recomputed from the state (the values compute_errors left
// in P.err, bit for bit).  Also the largest |Hpp| diagonal and |b| entry
// (the fixed-point scales of the trials).
template <class Rec>
LBA_FN void linearize(LbaDev& P, const double* pz, DScratch& sc)
{
    const int wv = threadIdx.x >> 6;
    double hm = 0, bm = 0;
    const int* order = P.ce;
    for (int t = threadIdx.x; t < P.nL; t += kLbaThreads) {
        double acc[9];
        bm = fmax(bm, point_linearize<Rec>(P, pz, order[t], acc));
    }
    for (int p = wv; p < P.nP; p += kLbaWaves) pose_linearize<Rec>(P, pz, p, hm, bm);
    hm = block_max_d(hm, sc);
    bm = block_max_d(bm, sc);
    if (threadIdx.x == 0) {
        P.hmax = hm;
        P.bmax = bm;
    }
    LBA_SYNC();
}

// Fixed-point accumulation of the reduced camera system.  Every value v is
// first scaled by a power of two s chosen per problem and trial (exact), so
// that the largest diagonal entry of Hpp + lambda I lands in [2^29, 2^30)
// (and the largest |b| entry in [2^23, 2^24) for the right-hand side).  The
// scaled value x = v s is split as x * 2^51 ~= hi * 2^40 + lo:
// hi = round(x * 2^11), lo = round((x * 2^11 - hi) * 2^40), |lo| <= 2^39 (the
// split of a given x is always the same; bits below 2^-51 of x, i.e. 2^-80 of
// the largest diagonal, are rounded off, far below the double rounding of
// the entries), and both limbs are added with 64-bit integer atomics.
// Integer addition is associative, so the accumulated limbs, and the double
// made from them, do not depend on the order in which threads add: the
// reduced system is bitwise reproducible.  Every Schur contribution
// (W_i Dinv W_j^T)_rc is bounded by sqrt(S_rr S_cc) <= the largest diagonal
// of Hpp + lambda I (a point's block [Hpp_l W; W^T Hll] is positive
// semi-definite), so the scaled contributions stay below 2^30 whatever the
// camera model or information weights (pixels, normalised coordinates,
// huge or tiny weights: tests/test_lba_gpu.py).  The limb sums stay exact for
// 2^22 contributions per entry (the host refuses problems with more points);
// a contribution with |x| >= 2^40 (possible only for b, whose bound involves
// 1/lambda) makes the trial retry at a 2^-24 smaller scale, and a non-finite
// one rejects the trial, as CHOLMOD's failure would.  Integerisation by the
// 1.5 * 2^52 magic-number addition (exact round-to-nearest for |x| < 2^51).
constexpr double kFxHi = 2048.0;                           // 2^11
constexpr double kFxLo = 1099511627776.0;                  // 2^40
constexpr double kFxInvHi = 1.0 / 2048.0;                  // 2^-11
constexpr double kFxInvLo = 1.0 / 2251799813685248.0;      // 2^-51
constexpr double kFxMax = 2251799813685248.0;              // 2^51 (of x * 2^11)
constexpr double kFxMagic = 6755399441055744.0;            // 1.5 * 2^52

typedef unsigned long long fx_t;

// (t = x * 2^11, already scaled)
LBA_FN void fx_split_scaled(double t, fx_t& hi, fx_t& lo, int& bad)
{
    bad |= !(fabs(t) < kFxMax);
    const double th = t + kFxMagic;                 // round(t) in the low mantissa bits
    const double r = t - (th - kFxMagic);           // exact, |r| <= 1/2
    // round(r * 2^40) likewise: the product is exact (a power of two), so the
    // multiply-then-add rounds exactly as fma(r, 2^40, M) -- in two
    // instructions, where the fma's accumulator needs M copied in first
    const double tl = r * kFxLo + kFxMagic;
    const long long m = __double_as_longlong(kFxMagic);
    hi = (fx_t)(__double_as_longlong(th) - m);
    lo = (fx_t)(__double_as_longlong(tl) - m);
}

// 64-bit integer atomic add into the reduced system, with the address space
// explicit (LDS, or global for the kLds = false fallback): on a generic
// pointer the compiler tests the address space at run time, and that test
// has tripped its instruction selection here
template <bool kLds>
LBA_FN void fx_atomic(fx_t* p, fx_t v)
{
#if defined(ORBX_LBA_DIAG_NOATOMIC)   // timing diagnostics only (wrong sums): a plain LDS add
    if constexpr (kLds) {
        *p += v;
        return;
    }
#elif defined(ORBX_LBA_DIAG_NOSTORE)  // timing diagnostics only: the contribution is computed, not stored
    if constexpr (kLds) {
        asm volatile("" ::"v"(v));
        return;
    }
#endif
    if constexpr (kLds) {
        atomicAdd(p, v);
    } else {
        auto* g = (__attribute__((address_space(1))) fx_t*)p;
        __hip_atomic_fetch_add(g, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
}

template <bool kLds>
LBA_FN void fx_add_scaled(fx_t* hi, fx_t* lo, int idx, double t, int& bad)
{
    fx_t h, l;
    fx_split_scaled(t, h, l, bad);
    fx_atomic<kLds>(hi + idx, h);
    fx_atomic<kLds>(lo + idx, l);
}

LBA_FN double fx_value(fx_t hi, fx_t lo)
{
    return (double)(long long)hi * kFxInvHi + (double)(long long)lo * kFxInvLo;
}

// Reduced-system storage of one problem (LDS or its global fallback), in
// doubles: limbs hi[M] | lo[M] | bhi[n] | blo[n] with M = n (n + 1) / 2;
// after accumulation hi[] holds the packed lower triangle as doubles and
// bhi[] the right-hand side.
__host__ __device__ constexpr long long lba_sys_doubles(long long n) { return n * (n + 1) + 2 * n; }

// Dinv = (Hll + lambda I)^-1 of a point (Eigen's 3x3 cofactor inverse:
// d[i*3+j] = cof(j, i) / det)
LBA_FN void point_dinv(const double* h, double lambda, double (&d)[9])
{
    double m[9];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) m[i * 3 + j] = h[i <= j ? up3(i, j) : up3(j, i)] + (i == j ? lambda : 0.0);
    const double c00 = m[4] * m[8] - m[5] * m[7], c10 = m[7] * m[2] - m[8] * m[1], c20 = m[1] * m[5] - m[2] * m[4];
    const double c01 = m[5] * m[6] - m[3] * m[8], c11 = m[8] * m[0] - m[6] * m[2], c21 = m[2] * m[3] - m[0] * m[5];
    const double c02 = m[3] * m[7] - m[4] * m[6], c12 = m[6] * m[1] - m[7] * m[0], c22 = m[0] * m[4] - m[1] * m[3];
    const double det = c00 * m[0] + c10 * m[3] + c20 * m[6];
    const double inv = 1.0 / det;
    d[0] = c00 * inv; d[1] = c10 * inv; d[2] = c20 * inv;
    d[3] = c01 * inv; d[4] = c11 * inv; d[5] = c21 * inv;
    d[6] = c02 * inv; d[7] = c12 * inv; d[8] = c22 * inv;
}

// One point's Schur contributions: D = Hll + lambda I, Dinv, db = Dinv bl;
// for each free-pose edge u: bs -= W_u db and, for every later edge v of the
// point (and v = u), S(p_u, p_v) -= W_u Dinv W_v^T as fixed-point limbs.
// With W = (w B)^T A the 6x6 block is (w B_u)^T G (w B_v), G = (A_u Dinv)
// A_v^T 2x2: W is never formed.
// (w B)(0, k) a0 + (w B)(1, k) a1 as fma((w B)(1, k), a1, (w B)(0, k) a0),
// with jac_pose's structural zeros B(0, 4) = B(1, 3) = 0 left out: the fused
// form's zero product adds only a signed zero, so the value is the same (a
// non-finite a0 / a1 still reaches the other columns, which reject the
// trial as before).
LBA_FN double wb_dot(const double (&wB)[12], int k, double a0, double a1)
{
    if (k == 3) return wB[3] * a0;
    if (k == 4) return wB[10] * a1;
    return __fma_rn(wB[6 + k], a1, wB[k] * a0);
}

template <bool kLds>
LBA_FN void schur_block(const double (&AD)[6], const double (&wBu)[12], const double (&Av)[6],
                                   const double (&wBv)[12], int pu, int pv, bool diag, double kS, fx_t* hi, fx_t* lo,
                                   int& bad)
{
    // G = AD Av^T (2x2); Q = -kS (w B_u)^T G (6x2): element (r, c) of the
    // block is Q[r] . (w B_v)[:, c]
    double G[4];
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++)
            G[2 * a + b] = __fma_rn(AD[3 * a + 2], Av[3 * b + 2], __fma_rn(AD[3 * a + 1], Av[3 * b + 1], AD[3 * a] * Av[3 * b]));
    double Q0[6], Q1[6];
#pragma unroll
    for (int r = 0; r < 6; r++) {
        Q0[r] = -kS * wb_dot(wBu, r, G[0], G[2]);
        Q1[r] = -kS * wb_dot(wBu, r, G[1], G[3]);
    }
    // element (r, c) belongs at S(6 pu + r, 6 pv + c): stored at the packed
    // lower index of that position or of its mirror
    const bool upper = pu < pv;
    const int ihi = upper ? pv : pu, ilo = upper ? pu : pv;
    const int base = pk(6 * ihi, 0) + 6 * ilo;
    if (pu != pv) {
        // Storage element (s, t) of the lower block is the block's (s, t)
        // when pu > pv and its (t, s) when pu < pv.  Both are
        // fma(P1[s], W1[t], P0[s] W0[t]) with (P, W) = (Q, w B_v) for the
        // first and (w B_v, Q) for the second -- wb_dot's value either way
        // (products commute; its structural zeros w B(0, 4) = w B(1, 3) = 0
        // enter here as +-0 terms, whose limbs are 0 all the same) -- so the
        // operands are swapped once per block, each storage row is one base
        // address and its six columns are immediate offsets (the per-element
        // index arithmetic cost more than the element's own arithmetic).
        double P0[6], P1[6], W0[6], W1[6];
#pragma unroll
        for (int k = 0; k < 6; k++) {
            P0[k] = upper ? wBv[k] : Q0[k];
            P1[k] = upper ? wBv[6 + k] : Q1[k];
            W0[k] = upper ? Q0[k] : wBv[k];
            W1[k] = upper ? Q1[k] : wBv[6 + k];
        }
        // odd lanes take the storage rows in the order 3, 4, 5, 0, 1, 2: lanes
        // of a wave that land on the same block then add to different rows
        // at the same instruction (fewer LDS address conflicts); the integer
        // limb sums do not depend on the order
        const bool rot = threadIdx.x & 1;
#pragma unroll
        for (int k = 0; k < 6; k++) {
            const int sa = k, sb = (k + 3) % 6;
            const int s = rot ? sb : sa;
            const double p0 = rot ? P0[sb] : P0[sa], p1 = rot ? P1[sb] : P1[sa];
            const int row = base + 6 * ihi * s + (rot ? sb * (sb + 1) / 2 : sa * (sa + 1) / 2);
            fx_t* hr = hi + row;
            fx_t* lr = lo + row;
#pragma unroll
            for (int t = 0; t < 6; t++) fx_add_scaled<kLds>(hr, lr, t, __fma_rn(p1, W1[t], p0 * W0[t]), bad);
        }
    } else {
        // one edge (diag): the lower triangle of its own block; two edges of
        // one point on the same pose (not made by LocalBundleAdjustment,
        // handled for completeness): the block plus its transpose
#pragma unroll
        for (int r = 0; r < 6; r++) {
            const int row = base + 6 * ihi * r + r * (r + 1) / 2;   // one base per row, immediate columns
            fx_t* hr = hi + row;
            fx_t* lr = lo + row;
#pragma unroll
            for (int c = 0; c <= r; c++) {
                double t = wb_dot(wBv, c, Q0[r], Q1[r]);
                if (!diag) t += wb_dot(wBv, r, Q0[c], Q1[c]);
                fx_add_scaled<kLds>(hr, lr, c, t, bad);
            }
        }
    }
}

// the edge's A (2x3) and w B (2x6) at point pt (pose z in LDS)
LBA_FN void edge_aw(const LbaDev& P, const double* z, int j, const double (&pt)[3], double (&A)[6],
                               double (&wB)[12])
{
    double pc[3], B[12];
    map_point(z, pt, pc);
    jac_point(z + 16, z + 7, pc, A);
    jac_pose(z + 16, pc, B);
    const double w = P.ew[j];
#pragma unroll
    for (int i = 0; i < 12; i++) wB[i] = (i == 4 || i == 9) ? 0.0 : B[i] * w;   // wb_dot skips them
}

template <class Rec, bool kLds>
LBA_FN void schur_point(LbaDev& P, const double* pz, int l, double lambda, double kS, double kB, fx_t* hi,
                                   fx_t* lo, fx_t* bhi, fx_t* blo, int& bad)
{
    double* dlo = P.dl + 12 * l;
    {
        const double* h = P.hl + 9 * l;
        double d[9];
        point_dinv(h, lambda, d);
#pragma unroll
        for (int i = 0; i < 9; i++) dlo[i] = d[i];
        dlo[9] = d[0] * h[6] + d[1] * h[7] + d[2] * h[8];
        dlo[10] = d[3] * h[6] + d[4] * h[7] + d[5] * h[8];
        dlo[11] = d[6] * h[6] + d[7] * h[7] + d[8] * h[8];
    }
    double pt[3];
    load_point(P.point + 3 * P.iv_point[l], pt);
    const int j0 = P.le_ptr[l], j1 = P.le_ptr[l + 1];
    for (int ju = j0; ju < j1; ju++) {
        const Rec ru = load_rec<Rec>(P, ju);
        if (ru.ph < 0) continue;
        const int pu = ru.ph;
        double AD[6], wBu[12];
        {
            double Au[6];
            edge_aw(P, pz + kPz * ru.pose, ju, pt, Au, wBu);
            // AD = A_u Dinv (2x3); bs -= W_u db = (w B_u)^T (A_u db)
            const double* d = dlo;
#pragma unroll
            for (int a = 0; a < 2; a++)
#pragma unroll
                for (int k = 0; k < 3; k++)
                    AD[3 * a + k] = __fma_rn(Au[3 * a + 2], d[6 + k], __fma_rn(Au[3 * a + 1], d[3 + k], Au[3 * a] * d[k]));
            const double adb0 = __fma_rn(Au[2], d[11], __fma_rn(Au[1], d[10], Au[0] * d[9]));
            const double adb1 = __fma_rn(Au[5], d[11], __fma_rn(Au[4], d[10], Au[3] * d[9]));
#pragma unroll
            for (int r = 0; r < 6; r++)
                fx_add_scaled<kLds>(bhi, blo, 6 * pu + r, -wb_dot(wBu, r, adb0, adb1) * kB, bad);
            schur_block<kLds>(AD, wBu, Au, wBu, pu, pu, true, kS, hi, lo, bad);   // v = u
        }
        for (int jv = ju + 1; jv < j1; jv++) {
            const Rec rv = load_rec<Rec>(P, jv);
            if (rv.ph < 0) continue;
            double Av[6], wBv[12];
            edge_aw(P, pz + kPz * rv.pose, jv, pt, Av, wBv);
            schur_block<kLds>(AD, wBu, Av, wBv, pu, rv.ph, false, kS, hi, lo, bad);
        }
    }
}

// 1 / sqrt(x) for x > 0: the hardware estimate (v_rsq_f64) refined by two
// Newton steps, r <- r (3/2 - x/2 r^2), to within a few ulps.  The LLT below
// scales by it instead of dividing by sqrt(x): a dependent double sqrt and
// division cost several times its latency on the pivot chain.
LBA_FN double rsqrt_nr(double x)
{
    double r = __builtin_amdgcn_rsq(x);
    const double h = 0.5 * x;
    r = r * __fma_rn(-h * r, r, 1.5);
    r = r * __fma_rn(-h * r, r, 1.5);
    return r;
}

// Dense LLT of the reduced system S (packed lower triangle, n x n, with the
// right-hand side as its row n: bs = S + n (n + 1) / 2) and the pose solve
// into xp; every thread of the workgroup takes part.  Returns false when S
// is not positive definite (uniform).  The reciprocals 1 / L_jj live at
// S + M + n (the free half of the limb region).
LBA_FN bool llt_solve(double* S, double* xp, const int n)
{
    __shared__ int s_fail;
    LBA_T0();
    const int M = n * (n + 1) / 2;
    double* bs = S + M;
    double* inv = bs + n;
    // dense LLT on the packed lower triangle, right-looking in 6x6 blocks
    // (the pose blocks): one lane factors a diagonal block in registers, the
    // panel rows solve against it (multiplying by the pivots' reciprocals),
    // the trailing triangle takes the rank-6 update.  Look-ahead: during block
    // column kb's trailing update wave 0 first updates the next diagonal block
    // itself and factors it at once, so each block column costs two barriers
    // and the factorisations hide behind the trailing updates.
    const int nb = n / 6;
    auto factor_diag = [&](int k0) {   // lane 0 of wave 0
        double a[21];                  // packed lower 6x6, a[i (i + 1) / 2 + j]
#pragma unroll
        for (int i = 0; i < 6; i++)
#pragma unroll
            for (int j = 0; j <= i; j++) a[i * (i + 1) / 2 + j] = S[pk(k0 + i, k0 + j)];
        int fail = 0;
#pragma unroll
        for (int j = 0; j < 6; j++) {
            const double piv = a[j * (j + 1) / 2 + j];
            fail |= !(piv > 0);
            const double r = rsqrt_nr(piv);
            a[j * (j + 1) / 2 + j] = piv * r;   // L_jj = sqrt(piv)
            inv[k0 + j] = r;
#pragma unroll
            for (int i = j + 1; i < 6; i++) a[i * (i + 1) / 2 + j] *= r;
#pragma unroll
            for (int i = j + 1; i < 6; i++)
#pragma unroll
                for (int q = j + 1; q <= i; q++) a[i * (i + 1) / 2 + q] -= a[i * (i + 1) / 2 + j] * a[q * (q + 1) / 2 + j];
        }
#pragma unroll
        for (int i = 0; i < 6; i++)
#pragma unroll
            for (int j = 0; j <= i; j++) S[pk(k0 + i, k0 + j)] = a[i * (i + 1) / 2 + j];
        s_fail = fail;
    };
    // S(i, j) -= L(i, block) . L(j, block) of block column k0
    auto trail = [&](int k0, int i, int j) {
        const double* Li = S + pk(i, k0);
        const double* Lj = S + pk(j, k0);
        S[pk(i, j)] -= ((((Li[0] * Lj[0] + Li[1] * Lj[1]) + Li[2] * Lj[2]) + Li[3] * Lj[3]) + Li[4] * Lj[4]) +
                       Li[5] * Lj[5];
    };
    if (nb > 0) {
        if (threadIdx.x == 0) factor_diag(0);
        LBA_SYNC();
        if (s_fail) return false;   // not positive definite (uniform)
    }
    LLT_W0();
    for (int kb = 0; kb < nb; kb++) {
        const int k0 = 6 * kb, k1 = k0 + 6;
        // panel: row r below the block solves x L_kk^T = A(r, block)
        for (int r = k1 + threadIdx.x; r <= n; r += kLbaThreads) {   // row n: the forward solve of b
            double x[6];
            double* Sr = S + pk(r, k0);
#pragma unroll
            for (int j = 0; j < 6; j++) x[j] = Sr[j];
#pragma unroll
            for (int j = 0; j < 6; j++) {
                const double* Lj = S + pk(k0 + j, k0);
#pragma unroll
                for (int q = 0; q < j; q++) x[j] -= x[q] * Lj[q];
                x[j] = x[j] * inv[k0 + j];
            }
#pragma unroll
            for (int j = 0; j < 6; j++) Sr[j] = x[j];
        }
        LLT_W(0);
        LBA_SYNC();
        LLT_W(1);
        LBA_MARK(26);
        const bool ahead = kb + 1 < nb;
        if (ahead && threadIdx.x < 64) {
            // the next diagonal block's 21 elements, then its factorisation
            const int t = threadIdx.x;
            if (t < 21) {
                int r = 0;
                while ((r + 1) * (r + 2) / 2 <= t) r++;
                trail(k0, k1 + r, k1 + (t - r * (r + 1) / 2));
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            if (t == 0) factor_diag(k1);
        } else {
            // the rest of the trailing triangle (and the b row): a half-wave
            // per pair of rows, each L(j, block) loaded once for both rows
            // (the next diagonal block, rows k1 .. k1 + 5, is wave 0's)
            const int t = ahead ? threadIdx.x - 64 : threadIdx.x;
            const int nhw = (ahead ? kLbaThreads - 64 : kLbaThreads) / 32;
            const int r0 = ahead ? k1 + 6 : k1;
            for (int i = r0 + 2 * (t >> 5); i <= n; i += 2 * nhw) {
                const bool two = i + 1 <= n;
                const double* Li = S + pk(i, k0);
                const double* Lk = S + pk(two ? i + 1 : i, k0);
                const double l0 = Li[0], l1 = Li[1], l2 = Li[2], l3 = Li[3], l4 = Li[4], l5 = Li[5];
                const double m0 = Lk[0], m1 = Lk[1], m2 = Lk[2], m3 = Lk[3], m4 = Lk[4], m5 = Lk[5];
                double* Si = S + pk(i, 0);
                double* Sk = S + pk(i + 1, 0);
                const int ji = min(i, n - 1), jk = two ? min(i + 1, n - 1) : ji;
                for (int j = k1 + (t & 31); j <= jk; j += 32) {
                    const double* Lj = S + pk(j, k0);
                    const double a0 = Lj[0], a1 = Lj[1], a2 = Lj[2], a3 = Lj[3], a4 = Lj[4], a5 = Lj[5];
                    if (j <= ji) Si[j] -= ((((l0 * a0 + l1 * a1) + l2 * a2) + l3 * a3) + l4 * a4) + l5 * a5;
                    if (two) Sk[j] -= ((((m0 * a0 + m1 * a1) + m2 * a2) + m3 * a3) + m4 * a4) + m5 * a5;
                }
            }
        }
        LLT_W(2);
        LBA_SYNC();
        LLT_W(3);
        LBA_MARK(27);
        if (s_fail) return false;
    }
    LBA_MARK(3);
    // the factorisation above solved L y = b in its row n (the panel step is
    // the forward substitution's block solve, the trailing update its update
    // of the later rows, in the same operation order); backward substitution
    // by one wave, in 6-row blocks: lane 0 solves the block's triangle in
    // registers, then every lane updates the earlier rows with its six values
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        for (int i = lane; i < n; i += 64) xp[i] = bs[i];
        auto wave_fence = [] {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        };
        wave_fence();
        for (int kb = nb - 1; kb >= 0; kb--) {   // L^T x = y
            const int k0 = 6 * kb;
            if (lane == 0) {
                double y[6], iv[6], Lb[21];   // the block's values loaded before the chain
#pragma unroll
                for (int p = 0; p < 6; p++) {
                    y[p] = xp[k0 + p];
                    iv[p] = inv[k0 + p];
                }
#pragma unroll
                for (int j = 1; j < 6; j++)
#pragma unroll
                    for (int p = 0; p < j; p++) Lb[j * (j + 1) / 2 + p] = S[pk(k0 + j, k0 + p)];
#pragma unroll
                for (int j = 5; j >= 0; j--) {
                    y[j] = y[j] * iv[j];
#pragma unroll
                    for (int p = 0; p < j; p++) y[p] -= Lb[j * (j + 1) / 2 + p] * y[j];
                }
#pragma unroll
                for (int p = 0; p < 6; p++) xp[k0 + p] = y[p];
            }
            wave_fence();
            double x[6];
#pragma unroll
            for (int p = 0; p < 6; p++) x[p] = xp[k0 + p];
            for (int i = lane; i < k0; i += 64)
                xp[i] -= ((((S[pk(k0, i)] * x[0] + S[pk(k0 + 1, i)] * x[1]) + S[pk(k0 + 2, i)] * x[2]) +
                           S[pk(k0 + 3, i)] * x[3]) + S[pk(k0 + 4, i)] * x[4]) + S[pk(k0 + 5, i)] * x[5];
            wave_fence();
        }
    }
    LBA_SYNC();
    LBA_MARK(4);
    return true;
}

// One Levenberg trial's linear algebra: Schur complement, LLT, the pose
// solve into xp (LDS).  Returns false when the reduced system is not
// positive definite (or its accumulation not finite).
// kLds: the reduced system lives in the dynamic LDS block (its accesses then
// compile to ds_* instructions instead of flat ones), else in P.S.
template <class Rec, bool kLds>
LBA_FN bool trial_solve(LbaDev& P, double* lds, const double* pz, double* xp, double lambda)
{
    __shared__ int s_bad;
    LBA_T0();
    const int n = P.dim_p;
    const int M = n * (n + 1) / 2;
    fx_t* hi = reinterpret_cast<fx_t*>(kLds ? lds : P.S);
    fx_t* lo = hi + M;
    fx_t* bhi = lo + M;
    fx_t* blo = bhi + n;
    // after conversion: the packed lower triangle S, and the right-hand side
    // as its row n (S + M, over the dead lo limbs), which the factorisation
    // below carries through the forward substitution
    double* S = reinterpret_cast<double*>(hi);
    double* bs = S + M;
    // the power-of-two scales of the fixed point (see fx_split_scaled):
    // largest diagonal of Hpp + lambda I into [2^29, 2^30), largest |b| into
    // [2^23, 2^24); exact, and the same on every thread
    const double hmax = P.hmax + lambda, bmax = P.bmax;
    double sS = (hmax > 0 && isfinite(hmax)) ? ldexp(1.0, 29 - ilogb(hmax)) : 1.0;
    double sB = (bmax > 0 && isfinite(bmax)) ? ldexp(1.0, 23 - ilogb(bmax)) : 1.0;
    const int* order = P.ce;
    for (int attempt = 0;; attempt++) {
        const double kS = sS * kFxHi, kB = sB * kFxHi;   // value -> fixed-point scale (x 2^11)
        int bad = 0;
        // the diagonal blocks Hpp + lambda I, zero elsewhere; bs <- bp
        for (int k = threadIdx.x; k < M; k += kLbaThreads) {
            hi[k] = 0;
            lo[k] = 0;
        }
        if (threadIdx.x == 0) s_bad = 0;
        LBA_SYNC();
        for (int item = threadIdx.x; item < P.nP * 21; item += kLbaThreads) {
            const int p = item / 21, u = item - p * 21;
            int r = 0;
            while (up6(r, 5) < u) r++;
            const int c = r + (u - up6(r, r));   // upper element (r, c), c >= r
            const int idx = pk(6 * p + c, 6 * p + r);
            fx_split_scaled((P.hp[27 * p + u] + (r == c ? lambda : 0.0)) * kS, hi[idx], lo[idx], bad);
        }
        for (int i = threadIdx.x; i < n; i += kLbaThreads)
            fx_split_scaled(P.hp[27 * (i / 6) + 21 + (i % 6)] * kB, bhi[i], blo[i], bad);
        LBA_SYNC();
        LBA_MARK(1);
        // points in the order of their edge counts: the lanes of a wave run
        // loops of similar length; with order-independent sums this changes
        // no bit of the result
        for (int t = threadIdx.x; t < P.nL; t += kLbaThreads)
            schur_point<Rec, kLds>(P, pz, order[t], lambda, kS, kB, hi, lo, bhi, blo, bad);
        if (bad) s_bad = 1;
        LBA_SYNC();
        if (!s_bad) break;                  // uniform
        if (attempt == 1) return false;     // still out of range (or non-finite): rejected
        sS *= 0x1p-24;                      // a contribution reached 2^40: once more at a smaller scale
        sB *= 0x1p-24;
        LBA_SYNC();                    // every thread has read s_bad before it is reset
    }
    // limbs -> doubles in place (element k's double overwrites its own hi),
    // scaled back (exact)
    const double iS = 1.0 / sS, iB = 1.0 / sB;
    for (int k = threadIdx.x; k < M; k += kLbaThreads) S[k] = fx_value(hi[k], lo[k]) * iS;
    LBA_SYNC();   // the lo limbs are read before row n overwrites them
    for (int i = threadIdx.x; i < n; i += kLbaThreads) bs[i] = fx_value(bhi[i], blo[i]) * iB;
    LBA_SYNC();
    LBA_MARK(2);
    return llt_solve(S, xp, n);
}

// The points of a pass by decreasing count of edges (counting sort; the
// order within a count is arbitrary and does not matter) into P.ce.
LBA_FN void point_order(LbaDev& P)
{
    __shared__ int hist[64], off[64];
    int* order = P.ce;
    for (int b = threadIdx.x; b < 64; b += kLbaThreads) hist[b] = 0;
    LBA_SYNC();
    auto bucket = [&](int l) { return 63 - min(P.le_ptr[l + 1] - P.le_ptr[l], 63); };
    for (int l = threadIdx.x; l < P.nL; l += kLbaThreads) atomicAdd(&hist[bucket(l)], 1);
    LBA_SYNC();
    if (threadIdx.x == 0) {
        int acc = 0;
        for (int b = 0; b < 64; b++) {
            off[b] = acc;
            acc += hist[b];
        }
    }
    LBA_SYNC();
    for (int l = threadIdx.x; l < P.nL; l += kLbaThreads) order[atomicAdd(&off[bucket(l)], 1)] = l;
    LBA_SYNC();
}

// rotation matrix of pose z (q at z[0..3]) into z[7..15] (Eigen's
// toRotationMatrix, the R of linearizeOplus)
LBA_FN void pz_rot(double* z) { qmat(Q{z[0], z[1], z[2], z[3]}, z + 7); }

// Back-substitution of point l with the W_i of the linearisation state (the
// saved poses pbk, the point before its update pt): xl = Dinv (bl - sum_i
// W_i^T xp_i) (block_solver.hpp:461-486)
template <class Rec>
LBA_FN void point_backsub(const LbaDev& P, const double* pz, const double* pbk, const double* xp, int l,
                                     const double (&pt)[3], double (&xl)[3])
{
    const double* h = P.hl + 9 * l;
    double cl[3] = {h[6], h[7], h[8]};
    for (int j = P.le_ptr[l]; j < P.le_ptr[l + 1]; j++) {
        const Rec r = load_rec<Rec>(P, j);
        if (r.ph < 0) continue;
        const double* zo = pbk + kPbk * r.ph;          // the pose (and rotation) before the update
        const double* cam = pz + kPz * r.pose + 16;
        double pc[3], A[6], B[12];
        map_point(zo, pt, pc);
        jac_point(cam, zo + 7, pc, A);
        jac_pose(cam, pc, B);
        const double w = P.ew[j];
        const double* x6 = xp + 6 * r.ph;
        double bx0 = 0, bx1 = 0;
#pragma unroll
        for (int k = 0; k < 6; k++) {
            bx0 += B[k] * x6[k];
            bx1 += B[6 + k] * x6[k];
        }
#pragma unroll
        for (int k = 0; k < 3; k++) cl[k] -= w * (A[k] * bx0 + A[3 + k] * bx1);
    }
    const double* d = P.dl + 12 * l;
#pragma unroll
    for (int i = 0; i < 3; i++) xl[i] = d[3 * i] * cl[0] + d[3 * i + 1] * cl[1] + d[3 * i + 2] * cl[2];
}

// Dynamic LDS layout of k_lba_iteration (doubles): [S region][poses][pose
// backups][xp]; the S region is empty when the batch's systems live in
// global memory.
struct LbaLds {
    int s_doubles, pz_off, pbk_off, xp_off;
    int bp_off;     // k_lba_split only: bp of the current linearisation (n doubles after xp)
    int stage_off;  // k_lba_split only: the staged Schur's slots (lba_staged_bytes())
};

// OptimizationAlgorithmLevenberg::solve for one problem (levenberg.cpp:61-164),
// iterations [iteration, iteration + iters) of SparseOptimizer::optimize
// (sparse_optimizer.cpp:380-402): one launch per iteration when the caller
// polls an abort flag between iterations, else all of a pass's iterations in
// one launch, so a problem whose trials take longer does not hold the others
// at every iteration.  The LM state (lambda, ni, chi2, the Raul counter) is
// the same on every thread (it follows block sums) and stays in registers
// across the iterations of a launch.
template <class Rec, bool kLds>
__global__ __launch_bounds__(kLbaThreads) void k_lba_iteration(LbaDev* probs, int iteration, int iters, LbaLds lay)
{
    extern __shared__ __attribute__((aligned(16))) double lds[];
    __shared__ DScratch sc;
    LbaDev& P = probs[blockIdx.x];
    if (P.status != kRunning || P.abort) return;
    if (P.nE == 0 || P.nP + P.nL == 0) {
        if (threadIdx.x == 0) P.status = kTerminated;
        return;
    }
    const int n = P.dim_p;
    double* pz = lds + lay.pz_off;
    double* pbk = lds + lay.pbk_off;
    double* xp = lds + lay.xp_off;
    // the problem's poses and cameras into LDS, rotation matrices beside them
    for (int i = threadIdx.x; i < P.nposes_all * 11; i += kLbaThreads) {
        const int p = i / 11, k = i - 11 * p;
        pz[kPz * p + (k < 7 ? k : 9 + k)] = k < 7 ? P.pose[7 * p + k] : P.cam[4 * p + (k - 7)];
    }
    LBA_SYNC();
    for (int p = threadIdx.x; p < P.nposes_all; p += kLbaThreads) pz_rot(pz + kPz * p);
    if (iteration == 0) point_order(P);
    LBA_SYNC();
    // the LM state carried from iteration to iteration of this launch, in
    // LDS: kept in registers across the iteration loop it spilled the Schur
    // pass (every thread computes the same values; thread 0 stores them)
    __shared__ double s_lm[3];   // lambda, ni, currentChi
    __shared__ int s_it[4];      // nBad, status, iterations done, trials
    if (threadIdx.x == 0) {
        s_lm[0] = P.lambda;
        s_lm[1] = P.ni;
        s_lm[2] = P.current_chi;
        s_it[0] = P.nBad;
        s_it[1] = kRunning;
        s_it[2] = 0;
        s_it[3] = 0;
    }
    LBA_SYNC();
    for (int it = iteration; it < iteration + iters && s_it[1] == kRunning; it++) {
    double lambda = s_lm[0], ni = s_lm[1], currentChi = s_lm[2];
    int nBad = s_it[0];
    LBA_T0();
    // computeActiveErrors at the start of the iteration: after the first
    // iteration the state is the previous iteration's accepted trial state,
    // whose errors (P.err) and robust chi2 that trial computed, bit for bit
    if (it == 0) currentChi = compute_errors<Rec>(P, pz, sc);
    const double iniChi = currentChi;
    if (it == 0 && threadIdx.x == 0) P.chi2_initial = currentChi;
    LBA_MARK(6);
    linearize<Rec>(P, pz, sc);
    LBA_MARK(7);
    if (it == 0) {
        double m = 0;
        for (int item = threadIdx.x; item < P.nP * 6; item += kLbaThreads)
            m = fmax(m, fabs(P.hp[27 * (item / 6) + up6(item % 6, item % 6)]));
        for (int item = threadIdx.x; item < P.nL * 3; item += kLbaThreads)
            m = fmax(m, fabs(P.hl[9 * (item / 3) + up3(item % 3, item % 3)]));
        m = block_max_d(m, sc);
        lambda = 1e-5 * m;
        ni = 2;
        nBad = 0;
    }
    double rho = 0;
    int qmax = 0;
    do {
        // push: the free poses (with their rotation matrices) into LDS; the
        // points are saved by the update pass below
        for (int i = threadIdx.x; i < P.nP * kPbk; i += kLbaThreads) {
            const int p = i / kPbk, k = i - kPbk * p;
            pbk[i] = pz[kPz * P.iv_pose[p] + k];
        }
        LBA_SYNC();
        const bool ok2 = trial_solve<Rec, kLds>(P, lds, pz, xp, lambda);
        if (ok2)
            for (int p = threadIdx.x; p < P.nP; p += kLbaThreads) {
                double* z = pz + kPz * P.iv_pose[p];
                se3_oplus(z, xp + 6 * p);
                pz_rot(z);
            }
        LBA_SYNC();
        LBA_T0();
        // per point: back-substitution, the update (VertexSBAPointXYZ::
        // oplusImpl) and the errors of its edges at the new state;
        // computeScale's sum_j x_j (lambda x_j + b_j) beside it.  A failed
        // solve leaves the state as it was (x = 0) and only evaluates the
        // errors.
        // (points in index order: a fixed share per thread, so the double
        // sums are the same on every run)
        double chi_part = 0, scale_part = 0;
        for (int l = threadIdx.x; l < P.nL; l += kLbaThreads) {
            double* pw = P.point + 3 * P.iv_point[l];
            double pt[3];
            load_point(pw, pt);
            if (ok2) {
                double xl[3];
                point_backsub<Rec>(P, pz, pbk, xp, l, pt, xl);
                const double* h = P.hl + 9 * l;
                double* bk = P.point_bk + 3 * l;
#pragma unroll
                for (int i = 0; i < 3; i++) {
                    bk[i] = pt[i];
                    scale_part += xl[i] * (lambda * xl[i] + h[6 + i]);
                    pt[i] += xl[i];
                    pw[i] = pt[i];
                }
            }
            chi_part += point_errors<Rec>(P, pz, l, pt);
        }
        if (ok2)
            for (int j = threadIdx.x; j < n; j += kLbaThreads)
                scale_part += xp[j] * (lambda * xp[j] + P.hp[27 * (j / 6) + 21 + (j % 6)]);
        double tempChi = block_sum_d(chi_part, sc);
        LBA_MARK(8);
        if (!ok2) {
            tempChi = 1.79769313486231570815e+308;
            if (threadIdx.x == 0) P.not_posdef++;
        }
        double scale = block_sum_d(scale_part, sc);
        scale += 1e-3;
        rho = (currentChi - tempChi) / scale;
        const bool accept = rho > 0 && isfinite(tempChi);
        if (accept) {
            double alpha = 1. - pow((2 * rho - 1), 3);
            alpha = fmin(alpha, 2. / 3.);
            lambda *= fmax(1. / 3., alpha);
            ni = 2;
            currentChi = tempChi;
        } else {
            lambda *= ni;
            ni *= 2;
            if (ok2) {   // pop: the saved poses and points
                for (int i = threadIdx.x; i < P.nP * kPbk; i += kLbaThreads) {
                    const int p = i / kPbk, k = i - kPbk * p;
                    pz[kPz * P.iv_pose[p] + k] = pbk[i];
                }
                for (int i = threadIdx.x; i < P.nL * 3; i += kLbaThreads) {
                    const int l = i / 3, k = i - 3 * l;
                    P.point[3 * P.iv_point[l] + k] = P.point_bk[i];
                }
            }
        }
        LBA_SYNC();
        qmax++;
    } while (rho < 0 && qmax < 10 && !P.abort);
    int status = kRunning;
    if (qmax == 10 || rho == 0) {
        status = kTerminated;
    } else {
        if ((iniChi - currentChi) * 1e3 < iniChi) nBad++;
        else nBad = 0;
        if (nBad >= 3) status = kTerminated;
    }
    if (threadIdx.x == 0) {
        s_lm[0] = lambda;
        s_lm[1] = ni;
        s_lm[2] = currentChi;
        s_it[0] = nBad;
        s_it[1] = status;
        s_it[2]++;
        s_it[3] += qmax;
    }
    LBA_SYNC();
    }
    // the free poses back to global memory (the next launch and the outlier
    // pass read them there)
    for (int i = threadIdx.x; i < P.nP * 7; i += kLbaThreads) {
        const int p = i / 7, k = i - 7 * p;
        P.pose[7 * P.iv_pose[p] + k] = pz[kPz * P.iv_pose[p] + k];
    }
    if (threadIdx.x == 0) {
        P.lambda = s_lm[0];
        P.ni = s_lm[1];
        P.trials += s_it[3];
        P.iterations += s_it[2];
        P.last_chi = s_lm[2];
        P.current_chi = s_lm[2];
        P.nBad = s_it[0];
        P.status = s_it[1];
    }
}

// ---------------------------------------------------------------------------
// One problem over G workgroups (orbx_lba_solve, and batches of one): the
// latency form of k_lba_iteration for the LocalMapping thread's single call
// (src/LocalMapping.cc:83).  Point l belongs to workgroup l mod G, free pose
// p's wave to workgroup p mod G; every workgroup keeps all the poses in its
// own LDS and applies the identical updates.  Per trial:
//   Schur     each workgroup accumulates its points' contributions (and
//             workgroup 0 the diagonal blocks Hpp + lambda I and bp) into its
//             own fixed-point limbs in LDS, stores them as its slab;
//             barrier; workgroup g sums slice g of the limbs over all slabs
//             (integer sums: the same total as k_lba_iteration's atomics);
//             barrier
//   solve     every workgroup converts the total and runs the same dense
//             LLT and solve (llt_solve) on its own copy: identical pose steps
//             everywhere, no broadcast
//   update    poses in every workgroup's LDS; back-substitution, point update
//             and errors per point, their robust chi2 and computeScale terms
//             stored per point; barrier; every workgroup sums them in
//             k_lba_iteration's thread order (thread t takes points t, t +
//             512, ..., then a block sum): the same bits, the same LM decision
//             everywhere
// and per iteration the linearisation (points and pose waves spread over the
// workgroups) with one barrier before its maxima are combined.  Results are
// bit-identical to k_lba_iteration (tests/test_lba_gpu.py compares the single
// call with the batch bit for bit).  Barriers: one monotonic arrival counter
// (zeroed before each launch) polled with relaxed agent-scope loads, an
// agent-scope release before the arrival and an acquire after it
// (MI355X_MICROARCH.md, inter-workgroup visibility); a barrier that waits
// past its bound marks the run failed instead of hanging, and the host
// reports ORBX_ERR_HIP.
// ---------------------------------------------------------------------------
// The Schur contributions of one workgroup's points (l = g + G k) in three
// stages, so that a point's work spreads over lanes instead of one thread
// (the split kernel has ~32 points per workgroup: thread per point left one
// point's ~1500 dependent contributions on the critical path).  Per chunk of
// up to kSP points whose free edges fit kSE slots:
//   points  Dinv and db (schur_point's arithmetic, into P.dl and LDS), the
//           free records into consecutive edge slots
//   edges   A, w B and A Dinv of each free edge, its bs contribution
//   pairs   one (u <= v) edge pair of a point per thread: schur_block
// The values are schur_point's, bit for bit; the limbs are integer sums, so
// the order of the atomics does not matter.
constexpr int kSP = 64;    // points per chunk (one wave's scan)
constexpr int kSE = 128;   // free-edge slots per chunk
constexpr int kSEd = 24;   // doubles per slot: A (6), w B (12), A Dinv (6)
// LDS bytes of the staged Schur (after k_lba_split's layout)
__host__ __device__ constexpr int lba_staged_bytes() { return kSE * kSEd * 8 + kSP * 12 * 8 + (3 * kSE + 3 * kSP + 2) * 4; }

template <class Rec>
LBA_FN void schur_staged(LbaDev& P, const double* pz, const int g, const int G, const double lambda,
                                             const double kS, const double kB, fx_t* hi, fx_t* lo, fx_t* bhi,
                                             fx_t* blo, int& bad, double* eA, double* pD, int* tab)
{
    __shared__ int s_m, s_ne, s_np;
    int* f = tab;               // [kSP] free edges per chunk point
    int* eb = f + kSP;          // [kSP + 1] first slot of each point
    int* pb = eb + kSP + 1;     // [kSP + 1] first pair of each point
    int* erec = pb + kSP + 1;   // [kSE] record of each slot
    int* epnt = erec + kSE;     // [kSE] chunk point of each slot
    int* eph = epnt + kSE;      // [kSE] pose block of each slot
    const int t = threadIdx.x;
    const int nk = g < P.nL ? (P.nL - g + G - 1) / G : 0;
    for (int k0 = 0; k0 < nk;) {
        if (t < kSP) {
            int c = 0;
            if (k0 + t < nk) {
                const int l = g + G * (k0 + t);
                for (int j = P.le_ptr[l]; j < P.le_ptr[l + 1]; j++) c += load_rec<Rec>(P, j).ph >= 0;
            }
            f[t] = c;
        }
        LBA_SYNC();
        if (t < 64) {
            const int c = f[t];
            const int inc = wave_inclusive_scan(c), pinc = wave_inclusive_scan(c * (c + 1) / 2);
            eb[t + 1] = inc;
            pb[t + 1] = pinc;
            if (t == 0) eb[0] = pb[0] = 0;
            // the slot counts grow with t: the chunk is the prefix that fits
            const unsigned long long fit = __ballot(inc <= kSE && k0 + t < nk);
            const int m = __popcll(fit);
            if (t == 0) s_m = m;
            if (m > 0 && t == m - 1) {
                s_ne = inc;
                s_np = pinc;
            }
        }
        LBA_SYNC();
        const int m = s_m;
        if (m == 0) {   // a point with more than kSE edges: the host does not split such problems
            bad = 1;
            break;
        }
        const int ne = s_ne, np = s_np;
        if (t < m) {
            const int l = g + G * (k0 + t);
            double* dlo = P.dl + 12 * l;
            double* pd = pD + 12 * t;
            const double* h = P.hl + 9 * l;
            double d[9];
            point_dinv(h, lambda, d);
#pragma unroll
            for (int i = 0; i < 9; i++) dlo[i] = pd[i] = d[i];
            dlo[9] = pd[9] = d[0] * h[6] + d[1] * h[7] + d[2] * h[8];
            dlo[10] = pd[10] = d[3] * h[6] + d[4] * h[7] + d[5] * h[8];
            dlo[11] = pd[11] = d[6] * h[6] + d[7] * h[7] + d[8] * h[8];
            int sl = eb[t];
            for (int j = P.le_ptr[l]; j < P.le_ptr[l + 1]; j++) {
                const int ph = load_rec<Rec>(P, j).ph;
                if (ph < 0) continue;
                erec[sl] = j;
                epnt[sl] = t;
                eph[sl] = ph;
                sl++;
            }
        }
        LBA_SYNC();
        for (int e = t; e < ne; e += kLbaThreads) {
            const int j = erec[e], i = epnt[e];
            const int l = g + G * (k0 + i);
            double pt[3];
            load_point(P.point + 3 * P.iv_point[l], pt);
            const Rec ru = load_rec<Rec>(P, j);
            double Au[6], wBu[12], AD[6];
            edge_aw(P, pz + kPz * ru.pose, j, pt, Au, wBu);
            const double* d = pD + 12 * i;
#pragma unroll
            for (int a = 0; a < 2; a++)
#pragma unroll
                for (int k = 0; k < 3; k++)
                    AD[3 * a + k] = __fma_rn(Au[3 * a + 2], d[6 + k], __fma_rn(Au[3 * a + 1], d[3 + k], Au[3 * a] * d[k]));
            const double adb0 = __fma_rn(Au[2], d[11], __fma_rn(Au[1], d[10], Au[0] * d[9]));
            const double adb1 = __fma_rn(Au[5], d[11], __fma_rn(Au[4], d[10], Au[3] * d[9]));
#pragma unroll
            for (int r = 0; r < 6; r++)
                fx_add_scaled<true>(bhi, blo, 6 * ru.ph + r, -wb_dot(wBu, r, adb0, adb1) * kB, bad);
            double* o = eA + kSEd * e;
#pragma unroll
            for (int k = 0; k < 6; k++) {
                o[k] = Au[k];
                o[18 + k] = AD[k];
            }
#pragma unroll
            for (int k = 0; k < 12; k++) o[6 + k] = wBu[k];
        }
        LBA_SYNC();
        for (int q = t; q < np; q += kLbaThreads) {
            int i = 0;
            while (pb[i + 1] <= q) i++;          // the chunk point of pair q
            const int fi = f[i];
            int r = q - pb[i], u = 0;
            while (r >= fi - u) {                // pairs (u, v), v = u .. fi - 1, u ascending
                r -= fi - u;
                u++;
            }
            const int eu = eb[i] + u, ev = eu + r;
            const double* ou = eA + kSEd * eu;
            const double* ov = eA + kSEd * ev;
            double ADu[6], wBu[12], Av[6], wBv[12];
#pragma unroll
            for (int k = 0; k < 6; k++) {
                ADu[k] = ou[18 + k];
                Av[k] = ov[k];
            }
#pragma unroll
            for (int k = 0; k < 12; k++) {
                wBu[k] = ou[6 + k];
                wBv[k] = ov[6 + k];
            }
            schur_block<true>(ADu, wBu, Av, wBv, eph[eu], eph[ev], eu == ev, kS, hi, lo, bad);
        }
        LBA_SYNC();
        k0 += m;
    }
}

struct LbaSplit {
    unsigned* bar;    // [0] arrivals, [1] failed (zeroed before each launch)
    fx_t* slabs;      // G x limbs
    fx_t* total;      // limbs
    double* chi_pt;   // nL: robust chi2 of each point's edges (last error pass)
    double* sc_pt;    // 3 nL: computeScale terms of each point's update
    double* wmax;     // G x 4: per-workgroup maxima (|Hpp| diagonal, |b|, lambda-init)
    int* wbad;        // 2 G: per-workgroup fixed-point range flags, per attempt
    int G, limbs;     // limbs = lba_sys_doubles(dim_p): hi M | lo M | bhi n | blo n
};

LBA_FN bool grid_sync(const LbaSplit& X, unsigned& epoch)
{
    __shared__ int s_ok;
    epoch++;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave's stores drained
    LBA_SYNC();
    if (threadIdx.x == 0) {
        auto* bar = (__attribute__((address_space(1))) unsigned*)X.bar;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned target = epoch * (unsigned)X.G;
        int ok = 1;
        for (unsigned spins = 0;; spins++) {
            if (__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) break;
            if (__hip_atomic_load(bar + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u || spins > (1u << 22)) {
                __hip_atomic_store(bar + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok = 0;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        s_ok = ok;
    }
    LBA_SYNC();
    return s_ok != 0;
}

// k_lba_split's back-substitution, point update and errors with the per-edge
// work spread over the workgroup's threads.  Per point (one thread, as
// k_lba_iteration does it) the workgroup's longest point -- up to ~20 edges of
// Jacobians in a row -- set the phase's length.  Here, in four steps:
//  1. per free edge (a thread each) its W^T x term (point_backsub's loop body),
//  2. per point (a thread each) the terms subtracted in edge order, Dinv, the
//     update,
//  3. per edge the error at the updated point (point_errors' loop body),
//  4. per point the robust chi2 summed in edge order.
// Every value and every sum is formed as point_backsub / point_errors form
// it, so the bits are those of the per-point loop (and of k_lba_iteration).
// The scratch is the staged Schur's LDS (free here): returns false, having
// done nothing, when the workgroup's points or edges exceed it.
constexpr int kBsPoints = 64;                                    // one wave's prefix
constexpr int kBsEdges = (kSE * kSEd - 3 * kBsPoints) / 3;       // 3 doubles per edge
template <class Rec>
LBA_FN bool backsub_edgewise(LbaDev& P, const double* pz, const double* pbk, const double* xp, const int g, const int G,
                             const bool ok2, const double lambda, const LbaSplit& X, double* es, int* pre)
{
    __shared__ int s_ne;
    const int t = threadIdx.x;
    const int np = g < P.nL ? (P.nL - g + G - 1) / G : 0;
    if (np > kBsPoints) return false;   // uniform
    double* npt = es + 3 * kBsEdges;    // the updated points
    if (t < 64) {
        const int c = t < np ? P.le_ptr[g + G * t + 1] - P.le_ptr[g + G * t] : 0;
        const int inc = wave_inclusive_scan(c);
        pre[t + 1] = inc;
        if (t == 0) pre[0] = 0;
        if (t == 63) s_ne = inc;
    }
    LBA_SYNC();
    const int ne = s_ne;
    if (ne > kBsEdges) return false;    // uniform
    // the workgroup point of edge slot e: the last t with pre[t] <= e
    auto point_of = [&](int e) {
        int a = 0, b = np - 1;
        while (a < b) {
            const int m = (a + b + 1) >> 1;
            if (pre[m] <= e) a = m;
            else b = m - 1;
        }
        return a;
    };
    if (ok2)
        for (int e = t; e < ne; e += kLbaThreads) {
            const int tp = point_of(e), l = g + G * tp, j = P.le_ptr[l] + (e - pre[tp]);
            const Rec r = load_rec<Rec>(P, j);
            if (r.ph < 0) continue;
            double pt[3];
            load_point(P.point + 3 * P.iv_point[l], pt);
            const double* zo = pbk + kPbk * r.ph;
            const double* cam = pz + kPz * r.pose + 16;
            double pc[3], A[6], B[12];
            map_point(zo, pt, pc);
            jac_point(cam, zo + 7, pc, A);
            jac_pose(cam, pc, B);
            const double w = P.ew[j];
            const double* x6 = xp + 6 * r.ph;
            double bx0 = 0, bx1 = 0;
#pragma unroll
            for (int k = 0; k < 6; k++) {
                bx0 += B[k] * x6[k];
                bx1 += B[6 + k] * x6[k];
            }
#pragma unroll
            for (int k = 0; k < 3; k++) es[3 * e + k] = w * (A[k] * bx0 + A[3 + k] * bx1);
        }
    LBA_SYNC();
    if (t < np) {
        const int l = g + G * t;
        double* pw = P.point + 3 * P.iv_point[l];
        double pt[3];
        load_point(pw, pt);
        double s3[3] = {0.0, 0.0, 0.0};
        if (ok2) {
            const double* h = P.hl + 9 * l;
            double cl[3] = {h[6], h[7], h[8]};
            const int j0 = P.le_ptr[l] - pre[t];
            for (int e = pre[t]; e < pre[t + 1]; e++) {
                if (load_rec<Rec>(P, j0 + e).ph < 0) continue;
#pragma unroll
                for (int k = 0; k < 3; k++) cl[k] -= es[3 * e + k];
            }
            const double* d = P.dl + 12 * l;
            double xl[3];
#pragma unroll
            for (int i = 0; i < 3; i++) xl[i] = d[3 * i] * cl[0] + d[3 * i + 1] * cl[1] + d[3 * i + 2] * cl[2];
            double* bk = P.point_bk + 3 * l;
#pragma unroll
            for (int i = 0; i < 3; i++) {
                bk[i] = pt[i];
                s3[i] = xl[i] * (lambda * xl[i] + h[6 + i]);
                pt[i] += xl[i];
                pw[i] = pt[i];
            }
        }
#pragma unroll
        for (int i = 0; i < 3; i++) {
            npt[3 * t + i] = pt[i];
            X.sc_pt[3 * l + i] = s3[i];
        }
    }
    LBA_SYNC();
    for (int e = t; e < ne; e += kLbaThreads) {
        const int tp = point_of(e), l = g + G * tp, j = P.le_ptr[l] + (e - pre[tp]);
        const Rec r = load_rec<Rec>(P, j);
        const double* z = pz + kPz * r.pose;
        const double pt[3] = {npt[3 * tp], npt[3 * tp + 1], npt[3 * tp + 2]};
        double pc[3], e0, e1;
        map_point(z, pt, pc);
        residual(z + 16, pc, (double)r.ox, (double)r.oy, e0, e1);
        const int eo = P.e_orig[j];
        P.err[2 * eo] = e0;
        P.err[2 * eo + 1] = e1;
        const double s = (double)r.isig;
        double r0, r1;
        huber(e0 * (s * e0) + e1 * (s * e1), P.huber_delta, &r0, &r1);
        es[e] = r0;   // the terms of step 1 are dead: step 2 is behind the barrier
    }
    LBA_SYNC();
    if (t < np) {
        double part = 0;
        for (int e = pre[t]; e < pre[t + 1]; e++) part += es[e];
        X.chi_pt[g + G * t] = part;
    }
    return true;
}

// k_lba_split's linearisation of the workgroup's points (point_linearize) and,
// in a pass's first iteration, their errors (point_errors), edge-parallel the
// same way: per edge (a thread each) its 9 Hll / bl terms, its robust weight
// and chi2 term -- computeError's values are the same in both functions, so
// one residual serves both; per point (a thread each) the sums in edge order.
// Returns false, having done nothing, when the workgroup's points or edges
// exceed the staged Schur's LDS (10 doubles per edge).
constexpr int kLinEdges = (kSE * kSEd) / 10;
template <class Rec>
LBA_FN bool linearize_edgewise(LbaDev& P, const double* pz, const int g, const int G, const bool errors,
                               const LbaSplit& X, double* es, int* pre, double& bm, double& hlm)
{
    __shared__ int s_ne;
    const int t = threadIdx.x;
    const int np = g < P.nL ? (P.nL - g + G - 1) / G : 0;
    if (np > kBsPoints) return false;   // uniform
    if (t < 64) {
        const int c = t < np ? P.le_ptr[g + G * t + 1] - P.le_ptr[g + G * t] : 0;
        const int inc = wave_inclusive_scan(c);
        pre[t + 1] = inc;
        if (t == 0) pre[0] = 0;
        if (t == 63) s_ne = inc;
    }
    LBA_SYNC();
    const int ne = s_ne;
    if (ne > kLinEdges) return false;   // uniform
    double* chi = es + 9 * ne;          // per-edge robust chi2 terms
    for (int e = t; e < ne; e += kLbaThreads) {
        int a = 0, b = np - 1;   // the workgroup point of edge slot e
        while (a < b) {
            const int m = (a + b + 1) >> 1;
            if (pre[m] <= e) a = m;
            else b = m - 1;
        }
        const int l = g + G * a, j = P.le_ptr[l] + (e - pre[a]);
        double pt[3];
        load_point(P.point + 3 * P.iv_point[l], pt);
        const Rec r = load_rec<Rec>(P, j);
        const double* z = pz + kPz * r.pose;
        double pc[3], e0, e1, A[6];
        map_point(z, pt, pc);
        residual(z + 16, pc, (double)r.ox, (double)r.oy, e0, e1);
        if (errors) {
            const int eo = P.e_orig[j];
            P.err[2 * eo] = e0;
            P.err[2 * eo + 1] = e1;
        }
        jac_point(z + 16, z + 7, pc, A);
        const double sg = (double)r.isig;
        double r0, r1;
        huber(e0 * (sg * e0) + e1 * (sg * e1), P.huber_delta, &r0, &r1);
        const double w = r1 * sg, om0 = -(sg * e0) * r1, om1 = -(sg * e1) * r1;
        P.ew[j] = w;
        double* o = es + 9 * e;
        int k = 0;
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int c = i; c < 3; c++) o[k++] = (A[i] * w) * A[c] + (A[3 + i] * w) * A[3 + c];
#pragma unroll
        for (int i = 0; i < 3; i++) o[6 + i] = A[i] * om0 + A[3 + i] * om1;
        chi[e] = r0;
    }
    LBA_SYNC();
    if (t < np) {
        const int l = g + G * t;
        double acc[9], part = 0;
#pragma unroll
        for (int v = 0; v < 9; v++) acc[v] = 0.0;
        for (int e = pre[t]; e < pre[t + 1]; e++) {
#pragma unroll
            for (int v = 0; v < 9; v++) acc[v] += es[9 * e + v];
            part += chi[e];
        }
#pragma unroll
        for (int v = 0; v < 9; v++) P.hl[9 * l + v] = acc[v];
        if (errors) X.chi_pt[l] = part;
        bm = fmax(bm, fmax(fabs(acc[6]), fmax(fabs(acc[7]), fabs(acc[8]))));
        hlm = fmax(hlm, fmax(fabs(acc[0]), fmax(fabs(acc[3]), fabs(acc[5]))));
    }
    return true;
}

// sum over l of v[l] in k_lba_iteration's order (thread t: l = t, t + 512,
// ... sequentially, then the block sum); every workgroup gets the same bits
LBA_FN double canon_sum(const double* v, int nL, DScratch& sc)
{
    double part = 0;
    for (int l = threadIdx.x; l < nL; l += kLbaThreads) part += v[l];
    return block_sum_d(part, sc);
}

// The LM state of k_lba_split, identical in every workgroup: in LDS, so that
// no register holds it across the Schur, solve and update stages (kept in
// registers it spilled them).  Every thread computes the same values; thread
// 0 stores them before a barrier.
struct SplitLM {
    double lambda, ni, currentChi, chi2_ini, iniChi, hm, bm, sS, sB, rho;
    int nBad, status, done, trials, not_posdef, ok, ok2, qmax;
};

template <class Rec>
__global__ __launch_bounds__(kLbaThreads) void k_lba_split(LbaDev* probs, int iteration, int iters, LbaLds lay,
                                                           LbaSplit X)
{
    extern __shared__ __attribute__((aligned(16))) double lds[];
    __shared__ DScratch sc;
    __shared__ int s_bad;
    __shared__ SplitLM st;
    LbaDev& P = probs[0];
    const int g = blockIdx.x, G = X.G;
    if (P.status != kRunning || P.abort) return;   // uniform: P is rewritten only after the last barrier
    if (P.nE == 0 || P.nP + P.nL == 0) {
        unsigned e = 0;
        grid_sync(X, e);                           // every workgroup has read P.status
        if (g == 0 && threadIdx.x == 0) P.status = kTerminated;
        return;
    }
    unsigned epoch = 0;
    const int n = P.dim_p, M = n * (n + 1) / 2;
    const int wv = threadIdx.x >> 6;
    double* pz = lds + lay.pz_off;
    double* pbk = lds + lay.pbk_off;
    double* xp = lds + lay.xp_off;
    double* bpl = lds + lay.bp_off;
    fx_t* hi = reinterpret_cast<fx_t*>(lds);
    fx_t* lo = hi + M;
    fx_t* bhi = lo + M;
    fx_t* blo = bhi + n;
    double* S = lds;
    double* bs = S + M;
    // the staged Schur's LDS after the layout (lay.stage_off doubles)
    double* eA = lds + lay.stage_off;
    double* pD = eA + kSE * kSEd;
    int* etab = reinterpret_cast<int*>(pD + kSP * 12);
    for (int i = threadIdx.x; i < P.nposes_all * 11; i += kLbaThreads) {
        const int p = i / 11, k = i - 11 * p;
        pz[kPz * p + (k < 7 ? k : 9 + k)] = k < 7 ? P.pose[7 * p + k] : P.cam[4 * p + (k - 7)];
    }
    if (threadIdx.x == 0) {
        st.lambda = P.lambda;
        st.ni = P.ni;
        st.currentChi = P.current_chi;
        st.chi2_ini = P.chi2_initial;
        st.nBad = P.nBad;
        st.status = kRunning;
        st.done = st.trials = st.not_posdef = 0;
        st.ok = 1;
    }
    LBA_SYNC();
    for (int p = threadIdx.x; p < P.nposes_all; p += kLbaThreads) pz_rot(pz + kPz * p);
    LBA_SYNC();
    for (int it = iteration; it < iteration + iters && st.status == kRunning && st.ok; it++) {
        LBA_T0();
        {   // linearisation (and, in a pass's first iteration, computeActiveErrors)
            double hm = 0, bm = 0, hlm = 0;
            // edge-parallel when the workgroup's points fit the scratch, else
            // a thread per point (the same bits either way)
            const bool edgewise = linearize_edgewise<Rec>(P, pz, g, G, it == 0, X, eA, etab, bm, hlm);
            for (int t = threadIdx.x; !edgewise; t += kLbaThreads) {
                const int l = g + G * t;
                if (l >= P.nL) break;
                if (it == 0) {
                    double pt[3];
                    load_point(P.point + 3 * P.iv_point[l], pt);
                    X.chi_pt[l] = point_errors<Rec>(P, pz, l, pt);
                }
                double acc[9];
                bm = fmax(bm, point_linearize<Rec>(P, pz, l, acc));
                hlm = fmax(hlm, fmax(fabs(acc[0]), fmax(fabs(acc[3]), fabs(acc[5]))));
            }
            for (int p = g + G * wv; p < P.nP; p += G * kLbaWaves) pose_linearize<Rec>(P, pz, p, hm, bm);
            hm = block_max_d(hm, sc);
            bm = block_max_d(bm, sc);
            hlm = block_max_d(hlm, sc);
            LBA_MARK(16);
            if (threadIdx.x == 0) {
                X.wmax[4 * g] = hm;
                X.wmax[4 * g + 1] = bm;
                X.wmax[4 * g + 2] = hlm;
            }
        }
        const bool ok1 = grid_sync(X, epoch);
        {
            double a = 0, b = 0, c = 0;
            for (int q = threadIdx.x; q < G; q += kLbaThreads) {
                a = fmax(a, X.wmax[4 * q]);
                b = fmax(b, X.wmax[4 * q + 1]);
                c = fmax(c, X.wmax[4 * q + 2]);
            }
            a = block_max_d(a, sc);
            b = block_max_d(b, sc);
            c = block_max_d(c, sc);
            // bp for computeScale: a copy, since a workgroup that is done with
            // this iteration's last trial may already write the next linearisation
            for (int j = threadIdx.x; j < n; j += kLbaThreads) bpl[j] = P.hp[27 * (j / 6) + 21 + (j % 6)];
            const double chi0 = it == 0 ? canon_sum(X.chi_pt, P.nL, sc) : 0.0;
            if (threadIdx.x == 0) {
                st.ok = st.ok && ok1;
                st.hm = a;
                st.bm = b;
                if (it == 0) {
                    st.currentChi = chi0;
                    st.chi2_ini = chi0;
                    st.lambda = 1e-5 * fmax(a, c);
                    st.ni = 2;
                    st.nBad = 0;
                }
                st.iniChi = st.currentChi;
                st.rho = 0;
                st.qmax = 0;
            }
            LBA_SYNC();
        }
        LBA_MARK(17);
        do {
            for (int i = threadIdx.x; i < P.nP * kPbk; i += kLbaThreads) {
                const int p = i / kPbk, k = i - kPbk * p;
                pbk[i] = pz[kPz * P.iv_pose[p] + k];
            }
            // --- Schur complement, summed over the workgroups
            if (threadIdx.x == 0) {
                const double hmax = st.hm + st.lambda, bmax = st.bm;
                st.sS = (hmax > 0 && isfinite(hmax)) ? ldexp(1.0, 29 - ilogb(hmax)) : 1.0;
                st.sB = (bmax > 0 && isfinite(bmax)) ? ldexp(1.0, 23 - ilogb(bmax)) : 1.0;
                st.ok2 = 1;
            }
            for (int attempt = 0;; attempt++) {
                int bad = 0;
                for (int k = threadIdx.x; k < X.limbs; k += kLbaThreads) hi[k] = 0;
                if (threadIdx.x == 0) s_bad = 0;
                LBA_SYNC();
                const double lambda = st.lambda, kS = st.sS * kFxHi, kB = st.sB * kFxHi;
                if (g == 0) {
                    for (int item = threadIdx.x; item < P.nP * 21; item += kLbaThreads) {
                        const int p = item / 21, u = item - p * 21;
                        int r = 0;
                        while (up6(r, 5) < u) r++;
                        const int c = r + (u - up6(r, r));
                        const int idx = pk(6 * p + c, 6 * p + r);
                        fx_split_scaled((P.hp[27 * p + u] + (r == c ? lambda : 0.0)) * kS, hi[idx], lo[idx], bad);
                    }
                    for (int i = threadIdx.x; i < n; i += kLbaThreads)
                        fx_split_scaled(P.hp[27 * (i / 6) + 21 + (i % 6)] * kB, bhi[i], blo[i], bad);
                }
                LBA_SYNC();
                schur_staged<Rec>(P, pz, g, G, lambda, kS, kB, hi, lo, bhi, blo, bad, eA, pD, etab);
                if (bad) s_bad = 1;
                LBA_SYNC();
                LBA_MARK(18);
                fx_t* slab = X.slabs + (size_t)g * X.limbs;
                for (int k = threadIdx.x; k < X.limbs; k += kLbaThreads) slab[k] = hi[k];
                if (threadIdx.x == 0) X.wbad[attempt * G + g] = s_bad;
                const bool oka = grid_sync(X, epoch);
                LBA_MARK(19);
                int anyb = 0;
                for (int q = threadIdx.x; q < G; q += kLbaThreads) anyb |= X.wbad[attempt * G + q];
                anyb = __syncthreads_or(anyb);
                if (threadIdx.x == 0) st.ok = st.ok && oka;
                if (anyb) {
                    LBA_SYNC();   // every thread has read st before thread 0 updates it
                    if (threadIdx.x == 0) {
                        if (attempt == 1) st.ok2 = 0;   // still out of range (or non-finite): rejected
                        st.sS *= 0x1p-24;
                        st.sB *= 0x1p-24;
                    }
                    LBA_SYNC();
                    if (attempt == 1) break;
                    continue;
                }
                // slice g of the limbs summed over the slabs: 16-byte units
                // (two limbs), the slabs split into groups so that every
                // thread keeps several independent loads in flight; group sums
                // meet in LDS (integer adds: any order)
                {
                    const int u0 = (int)((long long)(X.limbs / 2) * g / G), u1 = (int)((long long)(X.limbs / 2) * (g + 1) / G);
                    const int nu = u1 - u0, t = threadIdx.x;
                    const ulonglong2* sl = reinterpret_cast<const ulonglong2*>(X.slabs);
                    const size_t ustride = (size_t)(X.limbs / 2);
                    if (nu >= kLbaThreads / 2) {   // few workgroups: a thread per unit, every slab
                        for (int k = t; k < nu; k += kLbaThreads) {
                            fx_t a = 0, b = 0;
                            for (int q = 0; q < G; q++) {
                                const ulonglong2 v = sl[(size_t)q * ustride + u0 + k];
                                a += v.x;
                                b += v.y;
                            }
                            reinterpret_cast<ulonglong2*>(X.total)[u0 + k] = make_ulonglong2(a, b);
                        }
                    } else if (nu > 0) {
                        const int ngrp = min(kLbaThreads / nu, G);
                        fx_t* part = reinterpret_cast<fx_t*>(eA);   // the staged Schur's slots are free here
                        const int grp = t / nu, u = u0 + (t - grp * nu);
                        if (grp < ngrp) {
                            fx_t a = 0, b = 0;
                            for (int q = grp; q < G; q += ngrp) {
                                const ulonglong2 v = sl[(size_t)q * ustride + u];
                                a += v.x;
                                b += v.y;
                            }
                            part[2 * t] = a;
                            part[2 * t + 1] = b;
                        }
                        LBA_SYNC();
                        for (int k = t; k < nu; k += kLbaThreads) {
                            fx_t a = 0, b = 0;
                            for (int q = 0; q < ngrp; q++) {
                                a += part[2 * (q * nu + k)];
                                b += part[2 * (q * nu + k) + 1];
                            }
                            reinterpret_cast<ulonglong2*>(X.total)[u0 + k] = make_ulonglong2(a, b);
                        }
                    }
                }
                const bool okb = grid_sync(X, epoch);
                LBA_MARK(20);
                const double iS = 1.0 / st.sS, iB = 1.0 / st.sB;
                const fx_t* T = X.total;
                for (int k = threadIdx.x; k < M; k += kLbaThreads) S[k] = fx_value(T[k], T[M + k]) * iS;
                for (int i = threadIdx.x; i < n; i += kLbaThreads)
                    bs[i] = fx_value(T[2 * M + i], T[2 * M + n + i]) * iB;
                if (threadIdx.x == 0) st.ok = st.ok && okb;
                LBA_SYNC();
                break;
            }
            LBA_MARK(21);
            {
                const bool ok2 = st.ok2 && llt_solve(S, xp, n);
                LBA_MARK(22);
                if (ok2)
                    for (int p = threadIdx.x; p < P.nP; p += kLbaThreads) {
                        double* z = pz + kPz * P.iv_pose[p];
                        se3_oplus(z, xp + 6 * p);
                        pz_rot(z);
                    }
                LBA_SYNC();
                if (threadIdx.x == 0) st.ok2 = ok2;
            }
            {   // --- back-substitution, point update, errors of this workgroup's points
                const bool ok2 = st.ok2;
                const double lambda = st.lambda;
                // edge-parallel when the workgroup's points fit the scratch,
                // else a thread per point (the same bits either way)
                const bool edgewise = backsub_edgewise<Rec>(P, pz, pbk, xp, g, G, ok2, lambda, X, eA, etab);
                for (int t = threadIdx.x; !edgewise; t += kLbaThreads) {
                    const int l = g + G * t;
                    if (l >= P.nL) break;
                    double* pw = P.point + 3 * P.iv_point[l];
                    double pt[3];
                    load_point(pw, pt);
                    double s3[3] = {0.0, 0.0, 0.0};
                    if (ok2) {
                        double xl[3];
                        point_backsub<Rec>(P, pz, pbk, xp, l, pt, xl);
                        const double* h = P.hl + 9 * l;
                        double* bk = P.point_bk + 3 * l;
#pragma unroll
                        for (int i = 0; i < 3; i++) {
                            bk[i] = pt[i];
                            s3[i] = xl[i] * (lambda * xl[i] + h[6 + i]);
                            pt[i] += xl[i];
                            pw[i] = pt[i];
                        }
                    }
                    X.chi_pt[l] = point_errors<Rec>(P, pz, l, pt);
#pragma unroll
                    for (int i = 0; i < 3; i++) X.sc_pt[3 * l + i] = s3[i];
                }
            }
            LBA_MARK(23);
            const bool ok3 = grid_sync(X, epoch);
            LBA_MARK(24);
            {   // k_lba_iteration's sums, in its order, and its LM decision
                const bool ok2 = st.ok2;
                const double lambda = st.lambda, ni = st.ni, currentChi = st.currentChi;
                double tempChi = canon_sum(X.chi_pt, P.nL, sc);
                double scale_part = 0;
                if (ok2) {
                    for (int l = threadIdx.x; l < P.nL; l += kLbaThreads) {
                        scale_part += X.sc_pt[3 * l];
                        scale_part += X.sc_pt[3 * l + 1];
                        scale_part += X.sc_pt[3 * l + 2];
                    }
                    for (int j = threadIdx.x; j < n; j += kLbaThreads) scale_part += xp[j] * (lambda * xp[j] + bpl[j]);
                }
                if (!ok2) tempChi = 1.79769313486231570815e+308;
                double scale = block_sum_d(scale_part, sc);
                scale += 1e-3;
                const double rho = (currentChi - tempChi) / scale;
                const bool accept = rho > 0 && isfinite(tempChi);
                if (!accept && ok2) {   // pop: the saved poses (every workgroup) and this workgroup's points
                    for (int i = threadIdx.x; i < P.nP * kPbk; i += kLbaThreads) {
                        const int p = i / kPbk, k = i - kPbk * p;
                        pz[kPz * P.iv_pose[p] + k] = pbk[i];
                    }
                    for (int t = threadIdx.x;; t += kLbaThreads) {
                        const int l = g + G * t;
                        if (l >= P.nL) break;
#pragma unroll
                        for (int k = 0; k < 3; k++) P.point[3 * P.iv_point[l] + k] = P.point_bk[3 * l + k];
                    }
                }
                LBA_SYNC();   // every thread has read st
                if (threadIdx.x == 0) {
                    if (accept) {
                        double alpha = 1. - pow((2 * rho - 1), 3);
                        alpha = fmin(alpha, 2. / 3.);
                        st.lambda = lambda * fmax(1. / 3., alpha);
                        st.ni = 2;
                        st.currentChi = tempChi;
                    } else {
                        st.lambda = lambda * ni;
                        st.ni = ni * 2;
                    }
                    if (!ok2) st.not_posdef++;
                    st.rho = rho;
                    st.qmax++;
                    st.ok = st.ok && ok3;
                }
                LBA_SYNC();
            }
            LBA_MARK(25);
        } while (st.rho < 0 && st.qmax < 10 && !P.abort && st.ok);
        LBA_SYNC();   // every thread has evaluated the loop condition
        if (threadIdx.x == 0) {
            if (st.qmax == 10 || st.rho == 0) {
                st.status = kTerminated;
            } else {
                if ((st.iniChi - st.currentChi) * 1e3 < st.iniChi) st.nBad++;
                else st.nBad = 0;
                if (st.nBad >= 3) st.status = kTerminated;
            }
            st.done++;
            st.trials += st.qmax;
        }
        LBA_SYNC();
    }
    // every workgroup is past its last read of P and of the shared buffers
    const bool okf = grid_sync(X, epoch);
    if (g != 0) return;
    for (int i = threadIdx.x; i < P.nP * 7; i += kLbaThreads) {
        const int p = i / 7, k = i - 7 * p;
        P.pose[7 * P.iv_pose[p] + k] = pz[kPz * P.iv_pose[p] + k];
    }
    if (threadIdx.x == 0) {
        if (iteration == 0) P.chi2_initial = st.chi2_ini;
        P.lambda = st.lambda;
        P.ni = st.ni;
        P.trials += st.trials;
        P.iterations += st.done;
        P.last_chi = st.currentChi;
        P.current_chi = st.currentChi;
        P.nBad = st.nBad;
        P.status = (st.ok && okf) ? st.status : kTerminated;
        P.not_posdef += st.not_posdef;
    }
}

// Outlier passes of LocalBundleAdjustment (src/Optimizer.cc:452-470,
// :497-515).  The reference walks the edges in order; an edge's outcome
// depends only on earlier edges of the same map point (EraseObservation ->
// SetBadFlag), so each point's active edges are walked in edge order by one
// thread, points in parallel.  chi2() reads the errors of the last
// computeActiveErrors (P.err: the last trial's, accepted or not).
template <class Rec>
__global__ __launch_bounds__(256) void k_lba_outliers(LbaDev* probs, int* nobs_all, uint8_t* status_all,
                                                      uint8_t* bad_all, int pass, double thr, int* n_out,
                                                      const long long* offs, LbaStatRec* stat, unsigned* split_bar,
                                                      int* split_failed)
{
    __shared__ int s_cnt;
    LbaDev& P = probs[blockIdx.x];
    const long long eo = offs[3 * blockIdx.x], po = offs[3 * blockIdx.x + 1];
    int* nobs = nobs_all + po;
    uint8_t* st = status_all + eo;
    uint8_t* bad = bad_all + po;
    if (threadIdx.x == 0) s_cnt = 0;
    LBA_SYNC();
    int cnt = 0;
    // points spread over gridDim.y workgroups (a single problem's call:
    // several; a batch: one per problem)
    for (int l = threadIdx.x + blockDim.x * blockIdx.y; l < P.nL; l += blockDim.x * gridDim.y) {
        const int p = P.iv_point[l];
        double pt[3];
        load_point(P.point + 3 * p, pt);
        for (int j = P.le_ptr[l]; j < P.le_ptr[l + 1]; j++) {
            if (bad[p]) break;
            const Rec r = load_rec<Rec>(P, j);
            const int e = P.e_orig[j];
            const double s = (double)r.isig;
            const double e0 = P.err[2 * e], e1 = P.err[2 * e + 1];
            const double chi2 = e0 * (s * e0) + e1 * (s * e1);
            double pc[3];
            map_point(P.pose + 7 * r.pose, pt, pc);
            if (chi2 > thr || !(pc[2] > 0.0)) {
                if (--nobs[p] <= 2) bad[p] = 1;
                st[e] = (uint8_t)pass;
                cnt++;
            }
        }
    }
    atomicAdd(&s_cnt, cnt);
    LBA_SYNC();
    if (threadIdx.x == 0) atomicAdd(&n_out[blockIdx.x], s_cnt);   // zeroed by k_lba_build
    if (threadIdx.x == 0 && blockIdx.y == 0) {
        LbaStatRec& o = stat[blockIdx.x];
        o.iterations = P.iterations;
        o.trials = P.trials;
        o.not_posdef = P.not_posdef;
        o.pad = 0;
        o.chi2_initial = P.chi2_initial;
        o.last_chi = P.last_chi;
        // k_lba_split's barrier words (one problem): note a timed-out barrier,
        // re-arm the arrival counter for the next pass's launch
        if (split_bar && blockIdx.x == 0) {
            if (split_bar[1]) *split_failed = 1;
            split_bar[0] = 0;
        }
    }
}

// Structures of the first optimize() built on the device from the caller's
// arrays: g2o's initializeOptimization + BlockSolver::buildStructure
// (sparse_optimizer.cpp:166-267, block_solver.hpp:143-295) on the subset
// LocalBundleAdjustment uses.  Every edge is active; the free poses with an
// edge and the points with an edge are ordered by g2o vertex id (ties by
// index: a stable sort), which fixes the Hessian block order.  The edges are
// laid out point-major (each point's edges in edge order) as records; per
// free pose the (record, point) list of its edges in edge order.  Ranks come
// from a scan when the ids are already increasing (the caller's usual order)
// and from pairwise counts otherwise.  One workgroup per problem; the maps
// live in the ce scratch.
LBA_FN void lba_rank(const long long* id, const int* act, int n, int* rank, int* count,
                                BlockScratchN<kLbaWaves>& bs)
{
    const int tid = threadIdx.x;
    int unsorted = 0;
    for (int i = tid; i + 1 < n; i += kLbaThreads) unsorted |= !(id[i] < id[i + 1]);
    unsorted = block_sum<kLbaWaves>(unsorted, bs, 0);
    LBA_SYNC();
    int total = 0;
    if (!unsorted) {
        int base = 0;
        for (int c = 0; c < n; c += kLbaThreads) {
            const int i = c + tid;
            const int a = i < n ? act[i] : 0;
            int tot;
            const int off = block_exclusive_scan<kLbaWaves>(a, &tot, bs, (c / kLbaThreads) & 1);
            if (i < n) rank[i] = a ? base + off : -1;
            base += tot;
        }
        total = base;
    } else {
        int cnt = 0;
        for (int i = tid; i < n; i += kLbaThreads) {
            if (!act[i]) {
                rank[i] = -1;
                continue;
            }
            cnt++;
            const long long v = id[i];
            int r = 0;
            for (int j = 0; j < n; j++) r += act[j] && (id[j] < v || (id[j] == v && j < i));
            rank[i] = r;
        }
        total = block_sum<kLbaWaves>(cnt, bs, 1);
    }
    LBA_SYNC();
    *count = total;
}

// counts in ptr[1 .. n] -> offsets (block scans); ptr[0] = 0
LBA_FN void lba_offsets(int* ptr, int n, BlockScratchN<kLbaWaves>& bs)
{
    const int tid = threadIdx.x;
    int base = 0;
    for (int c = 0; c < n; c += kLbaThreads) {
        const int i = c + tid;
        const int v = i < n ? ptr[i + 1] : 0;
        int tot;
        const int inc = block_exclusive_scan<kLbaWaves>(v, &tot, bs, (c / kLbaThreads) & 1) + v;
        LBA_SYNC();
        if (i < n) ptr[i + 1] = base + inc;
        base += tot;
        LBA_SYNC();
    }
    if (tid == 0) ptr[0] = 0;
    LBA_SYNC();
}

// The edges of each free pose in edge order, as a stable counting scatter:
// the block walks the edges in chunks of kLbaThreads; in each chunk every
// wave ranks its lanes among the lanes of the same pose block (one ballot per
// distinct pose block of the wave) and stores its per-pose counts, then a
// prefix over the waves (in wave order) and the running per-pose base give
// each edge its place.  counts != nullptr: only count (the totals land in
// counts[q]); else write pe_idx[ptr[q] + place] = (point-major record, point).
constexpr int kBuildPoses = 128;   // free poses the LDS tables hold (else the per-pose scan)
constexpr int kBuildPoints = 8192; // active points whose counts / cursors k_lba_build keeps in LDS

LBA_FN void pose_chunks(const LbaDev& A, const int* ph, int nP, int (*wcnt)[kBuildPoses],
                                            int* base, int* ptr, const int* pos, int2* pe_idx)
{
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, E = A.nedges_all;
    const bool count_only = pe_idx == nullptr;
    for (int q = tid; q < nP; q += kLbaThreads) base[q] = 0;
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    for (int a0 = 0; a0 < E; a0 += kLbaThreads) {
        for (int q = lane; q < nP; q += 64) wcnt[wv][q] = 0;
        LBA_SYNC();
        const int a = a0 + tid;
        const int q = a < E ? ph[A.r_edge_pose[a]] : -1;
        int rank = 0;
        uint64_t act = __builtin_amdgcn_ballot_w64(q >= 0);
        while (act) {
            const int lead = (int)__builtin_ctzll(act);
            const int qq = __builtin_amdgcn_readlane(q, lead);
            const uint64_t m = __builtin_amdgcn_ballot_w64(q == qq);
            if (q == qq) rank = (int)__popcll(m & lt);
            if (lane == lead) wcnt[wv][qq] = (int)__popcll(m);
            act &= ~m;
        }
        LBA_SYNC();
        for (int qq = tid; qq < nP; qq += kLbaThreads) {   // wave-order prefix per pose
            int sum = base[qq];
#pragma unroll
            for (int w = 0; w < kLbaWaves; w++) {
                const int c = wcnt[w][qq];
                wcnt[w][qq] = sum;
                sum += c;
            }
            base[qq] = sum;
        }
        LBA_SYNC();
        if (!count_only && q >= 0) pe_idx[ptr[q] + wcnt[wv][q] + rank] = make_int2(pos[a], A.r_edge_point[a]);
    }
    LBA_SYNC();
    if (count_only)
        for (int qq = tid; qq < nP; qq += kLbaThreads) ptr[qq] = base[qq];
    LBA_SYNC();
}

template <class Rec>
__global__ __launch_bounds__(kLbaThreads) void k_lba_build(LbaDev* probs, int* n_out, int P_all, unsigned* split_bar,
                                                           int* split_failed)
{
    __shared__ BlockScratchN<kLbaWaves> bs;
    __shared__ int s_wcnt[kLbaWaves][kBuildPoses], s_base[kBuildPoses];
    __shared__ int s_pt[kBuildPoints];   // per active point: edge counts, then list cursors
    LbaDev& A = probs[blockIdx.x];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int NP = A.nposes_all, NL = A.npoints_all, E = A.nedges_all;
    int* pflag = A.ce;           // [NP] pose has an edge and is free
    int* lflag = pflag + NP;     // [NL] point has an edge
    int* ph = lflag + NL;        // [NP] pose block or -1
    int* lh = ph + NP;           // [NL] point block or -1
    int* cur = lh + NL;          // [NL] list cursors
    int* pos = cur + NL;         // [E] point-major position of each edge
    LBA_T0();
    // the solve's zero state: per-edge errors, both passes' outlier counts,
    // k_lba_split's barrier words and failed flag
    for (int i = tid; i < 2 * E; i += kLbaThreads) A.err[i] = 0.0;
    if (tid < 2) n_out[tid * P_all + blockIdx.x] = 0;
    if (blockIdx.x == 0 && split_bar && tid < 16) split_bar[tid] = 0;
    if (blockIdx.x == 0 && tid == 0) *split_failed = 0;
    for (int i = tid; i < NP; i += kLbaThreads) pflag[i] = 0;
    for (int i = tid; i < NL; i += kLbaThreads) lflag[i] = 0;
    LBA_SYNC();
    for (int a = tid; a < E; a += kLbaThreads) {
        const int p = A.r_edge_pose[a];
        if (!A.r_pose_fixed[p]) pflag[p] = 1;
        lflag[A.r_edge_point[a]] = 1;
    }
    LBA_SYNC();
    LBA_MARK(9);
    int nP, nL;
    lba_rank(A.r_pose_id, pflag, NP, ph, &nP, bs);
    lba_rank(A.r_point_id, lflag, NL, lh, &nL, bs);
    LBA_MARK(10);
    int* iv_pose = const_cast<int*>(A.iv_pose);
    int* iv_point = const_cast<int*>(A.iv_point);
    for (int i = tid; i < NP; i += kLbaThreads)
        if (ph[i] >= 0) iv_pose[ph[i]] = i;
    for (int i = tid; i < NL; i += kLbaThreads)
        if (lh[i] >= 0) iv_point[lh[i]] = i;
    int* pe_ptr = const_cast<int*>(A.pe_ptr);
    int* le_ptr = const_cast<int*>(A.le_ptr);
    for (int i = tid; i <= nP; i += kLbaThreads) pe_ptr[i] = 0;
    for (int i = tid; i <= nL; i += kLbaThreads) le_ptr[i] = 0;
    LBA_SYNC();
    // the free poses' edge counts come from the chunked pass below when the
    // batch's free poses fit its LDS tables (kBuildPoses), else from atomics
    const bool chunked = nP <= kBuildPoses;
    if (chunked) pose_chunks(A, ph, nP, s_wcnt, s_base, pe_ptr + 1, nullptr, nullptr);
    // the points' edge counts and list cursors in LDS when they fit
    const bool pts_lds = nL <= kBuildPoints;
    if (pts_lds) {
        for (int l = tid; l < nL; l += kLbaThreads) s_pt[l] = 0;
        LBA_SYNC();
    }
    for (int a = tid; a < E; a += kLbaThreads) {
        if (!chunked) {
            const int eph = ph[A.r_edge_pose[a]];
            if (eph >= 0) atomicAdd(&pe_ptr[eph + 1], 1);
        }
        const int l = lh[A.r_edge_point[a]];
        if (pts_lds) atomicAdd(&s_pt[l], 1);
        else atomicAdd(&le_ptr[l + 1], 1);
    }
    LBA_SYNC();
    if (pts_lds)
        for (int l = tid; l < nL; l += kLbaThreads) le_ptr[l + 1] = s_pt[l];
    LBA_SYNC();
    LBA_MARK(11);
    lba_offsets(pe_ptr, nP, bs);
    lba_offsets(le_ptr, nL, bs);
    // point-major slots, then each point's edges put in edge order (few)
    int* e_orig = const_cast<int*>(A.e_orig);
    int* cursor = pts_lds ? s_pt : cur;
    for (int l = tid; l < nL; l += kLbaThreads) cursor[l] = le_ptr[l];
    LBA_SYNC();
    for (int a = tid; a < E; a += kLbaThreads) e_orig[atomicAdd(&cursor[lh[A.r_edge_point[a]]], 1)] = a;
    LBA_SYNC();
    LBA_MARK(12);
    for (int l = tid; l < nL; l += kLbaThreads) {
        const int q0 = le_ptr[l], q1 = le_ptr[l + 1];
        for (int i = q0 + 1; i < q1; i++) {   // insertion sort by edge index
            const int x = e_orig[i];
            int j = i - 1;
            while (j >= q0 && e_orig[j] > x) {
                e_orig[j + 1] = e_orig[j];
                j--;
            }
            e_orig[j + 1] = x;
        }
    }
    LBA_SYNC();
    LBA_MARK(13);
    // the records (float fields only when the host found every value exact)
    Rec* rec = reinterpret_cast<Rec*>(const_cast<void*>(A.rec));
    for (int j = tid; j < E; j += kLbaThreads) {
        const int a = e_orig[j];
        const int p = A.r_edge_pose[a];
        Rec r{};
        r.ox = A.r_edge_obs[2 * a];
        r.oy = A.r_edge_obs[2 * a + 1];
        r.isig = A.r_edge_isig[a];
        r.pose = (uint16_t)p;
        r.ph = (int16_t)ph[p];
        rec[j] = r;
        pos[a] = j;
    }
    LBA_SYNC();
    LBA_MARK(14);
    // per free pose, its edges in edge order: the chunked stable scatter, or
    // (more free poses than its tables) a wave per pose with ballot compaction
    int2* pe_idx = const_cast<int2*>(A.pe_idx);
    if (chunked) pose_chunks(A, ph, nP, s_wcnt, s_base, pe_ptr, pos, pe_idx);
    else
    for (int p1 = wv; p1 < nP; p1 += kLbaWaves) {
        const int pose = iv_pose[p1];
        int w = pe_ptr[p1];
        for (int a0 = 0; a0 < E; a0 += 64) {
            const int a = a0 + lane;
            const bool mine = a < E && A.r_edge_pose[a] == pose;
            const unsigned long long bal = __ballot(mine);
            if (mine)
                pe_idx[w + __popcll(bal & (lane ? (~0ull >> (64 - lane)) : 0ull))] = make_int2(pos[a], A.r_edge_point[a]);
            w += __popcll(bal);
        }
    }
    LBA_MARK(15);
    if (tid == 0) {
        A.nP = nP;
        A.nL = nL;
        A.nE = E;
        A.dim_p = 6 * nP;
    }
}

// Structures of the second optimize() (src/Optimizer.cc:472-478: the edges
// the first outlier pass set to level 1 leave the graph) built on the device
// from the first pass's: g2o's initializeOptimization / buildStructure
// restated as order-preserving filters of the first pass's lists (the kept
// records keep their point-major order, free poses / points their id order,
// the pose lists their edge order), so the result equals the first-pass
// build (k_lba_build) on the reduced edge set.  One workgroup per problem;
// the maps live in the shared ce scratch (the first pass's point order is
// dead by then).  B's pointer fields are set by the host.
template <class Rec>
__global__ __launch_bounds__(kLbaThreads) void k_lba_rebuild(const LbaDev* d0s, LbaDev* d1s, const uint8_t* status_all,
                                                             const long long* offs)
{
    __shared__ BlockScratchN<kLbaWaves> bs;
    const LbaDev& A = d0s[blockIdx.x];
    LbaDev& B = d1s[blockIdx.x];
    const uint8_t* st = status_all + offs[3 * blockIdx.x];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int nE0 = A.nE, nP0 = A.nP, nL0 = A.nL;
    int* nj = A.ce;              // [nE0] new record index or -1
    int* ph1 = nj + nE0;         // [nP0] new pose block or -1
    int* cp = ph1 + nP0;         // [nP0] kept edges per free pose
    int* lh1 = cp + nP0;         // [nL0] new point index or -1
    int* cl = lh1 + nL0;         // [nL0] kept edges per point
    auto kept = [&](int j) { return st[A.e_orig[j]] == 0; };
    // 1. records: new index by a block scan over the kept flags (point-major order)
    int base = 0;
    for (int c = 0; c < nE0; c += kLbaThreads) {
        const int j = c + tid;
        const int k = j < nE0 && kept(j) ? 1 : 0;
        int tot;
        const int off = block_exclusive_scan<kLbaWaves>(k, &tot, bs, (c / kLbaThreads) & 1);
        if (j < nE0) nj[j] = k ? base + off : -1;
        base += tot;
    }
    const int nE1 = base;
    LBA_SYNC();
    // 2. kept edges per pose (wave per pose) and per point (thread per point)
    for (int p = wv; p < nP0; p += kLbaWaves) {
        int cnt = 0;
        for (int q = A.pe_ptr[p] + lane; q < A.pe_ptr[p + 1]; q += 64) cnt += nj[A.pe_idx[q].x] >= 0;
        cnt = wave_sum(cnt);
        if (lane == 0) cp[p] = cnt;
    }
    for (int l = tid; l < nL0; l += kLbaThreads) {
        int c1 = 0;
        for (int j = A.le_ptr[l]; j < A.le_ptr[l + 1]; j++) c1 += nj[j] >= 0;
        cl[l] = c1;
    }
    LBA_SYNC();
    // 3. new pose / point indices and list offsets: scans over the active ones
    int nP1 = 0, pe_base = 0;
    for (int c = 0; c < nP0; c += kLbaThreads) {
        const int p = c + tid;
        const int act = p < nP0 && cp[p] > 0 ? 1 : 0;
        int tot, tot2;
        const int idx = block_exclusive_scan<kLbaWaves>(act, &tot, bs, 0);
        const int eo = block_exclusive_scan<kLbaWaves>(act ? cp[p] : 0, &tot2, bs, 1);
        if (p < nP0) {
            const int p1 = act ? nP1 + idx : -1;
            if (act) {
                const_cast<int*>(B.iv_pose)[p1] = A.iv_pose[p];
                const_cast<int*>(B.pe_ptr)[p1] = pe_base + eo;
            }
            ph1[p] = p1;
        }
        nP1 += tot;
        pe_base += tot2;
        LBA_SYNC();   // bs reads done before the next round's scans
    }
    int nL1 = 0, le_base = 0;
    for (int c = 0; c < nL0; c += kLbaThreads) {
        const int l = c + tid;
        const int act = l < nL0 && cl[l] > 0 ? 1 : 0;
        int tot, tot2;
        const int idx = block_exclusive_scan<kLbaWaves>(act, &tot, bs, 0);
        const int eo = block_exclusive_scan<kLbaWaves>(act ? cl[l] : 0, &tot2, bs, 1);
        if (l < nL0) {
            const int l1 = act ? nL1 + idx : -1;
            if (act) {
                const_cast<int*>(B.iv_point)[l1] = A.iv_point[l];
                const_cast<int*>(B.le_ptr)[l1] = le_base + eo;
            }
            lh1[l] = l1;
        }
        nL1 += tot;
        le_base += tot2;
        LBA_SYNC();   // bs reads done before the next round's scans
    }
    if (tid == 0) {
        const_cast<int*>(B.pe_ptr)[nP1] = pe_base;
        const_cast<int*>(B.le_ptr)[nL1] = le_base;
    }
    LBA_SYNC();
    // 4. the kept records, pose blocks remapped
    const Rec* ra = reinterpret_cast<const Rec*>(A.rec);
    Rec* rb = reinterpret_cast<Rec*>(const_cast<void*>(B.rec));
    for (int j = tid; j < nE0; j += kLbaThreads) {
        const int j1 = nj[j];
        if (j1 < 0) continue;
        Rec r = ra[j];
        r.ph = (int16_t)(r.ph >= 0 ? ph1[r.ph] : -1);
        rb[j1] = r;
        const_cast<int*>(B.e_orig)[j1] = A.e_orig[j];
    }
    // 5. pose lists: filters of the first pass's lists (wave per pose, ballot compaction)
    for (int p = wv; p < nP0; p += kLbaWaves) {
        const int p1 = ph1[p];
        if (p1 < 0) continue;
        int w = B.pe_ptr[p1];
        for (int q0 = A.pe_ptr[p]; q0 < A.pe_ptr[p + 1]; q0 += 64) {
            const int q = q0 + lane;
            int2 ent = make_int2(-1, 0);
            if (q < A.pe_ptr[p + 1]) {
                ent = A.pe_idx[q];
                ent.x = nj[ent.x];
            }
            const unsigned long long bal = __ballot(ent.x >= 0);
            if (ent.x >= 0) {
                const unsigned long long lt = lane ? (~0ull >> (64 - lane)) : 0ull;
                const_cast<int2*>(B.pe_idx)[w + __popcll(bal & lt)] = ent;
            }
            w += __popcll(bal);
        }
    }
    if (tid == 0) {
        B.nP = nP1;
        B.nL = nL1;
        B.nE = nE1;
        B.dim_p = 6 * nP1;
        B.lambda = 0;
        B.ni = 2;
        B.current_chi = B.last_chi = B.chi2_initial = 0;
        B.nBad = 0;
        B.status = kRunning;
        B.iterations = B.trials = B.not_posdef = 0;
        B.abort = A.abort;
    }
}

// ---------------------------------------------------------------------------
// Host: structure build (initializeOptimization + buildStructure) and driver
// ---------------------------------------------------------------------------
namespace {

// doubles of dynamic LDS for k_lba_iteration (160 KB less its static LDS)
constexpr int kLdsCap = (160 * 1024 - 2048) / 8;

// Runs fn(i) for i in [0, n) on up to 16 host threads (independent problems).
template <typename Fn>
void host_parallel(int n, Fn fn)
{
    const int nth = std::max(1, std::min<int>(n, std::min(16u, std::max(1u, std::thread::hardware_concurrency()))));
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

inline size_t align256(size_t b) { return (b + 255) & ~size_t(255); }
}  // namespace

// Device layout of one batch of P problems (planned on the host from the
// problems' sizes): the staged block [0, staged_end) that the host fills --
// the persistent part [0, base_bytes) (poses, points, cameras, per-point
// observation counts, edge / point flags, offsets, outlier counts; poses
// and points first, so the results copy reads back a prefix), the callers'
// raw edge / id arrays, and both passes' LbaDev arrays -- then device-only:
// the LM backups, the per-edge errors, both passes' structure arrays and the
// scratch.
struct LbaPlay {
    size_t pose, point, pointbk, cam, err;
};
struct LbaPlan {
    int P = 0;
    uint8_t* d = nullptr;   // device base the LbaDev pointers were packed against
    bool float_rec = true;  // every observation / information is a float: 16-byte edge records
    LbaLds lay{};           // k_lba_iteration's dynamic LDS
    size_t lds_bytes = 0;
    size_t lds_split_bytes = 0;   // k_lba_split's (the layout plus bp)
    int nfree0 = 0;               // free poses of problem 0 (k_lba_split's reduced system)
    int max_obs0 = 0;             // most edges on one point of problem 0 (k_lba_split stages <= kSE)
    std::vector<LbaPlay> pl;
    std::vector<long long> offs;   // per problem: first edge, first point (global flag arrays)
    std::vector<int> n_poses, n_points, n_edges;
    long long eacc = 0, pacc = 0;
    size_t result_bytes = 0, base_bytes = 0, o_all_nobs = 0, o_all_st = 0, o_all_bad = 0, o_offs = 0, o_nout = 0;
    size_t o_stats = 0, o_failed = 0;   // LbaStatRec [2][P], k_lba_split's failed flag: the end of the readback block
    size_t o_devs = 0, o_devs1 = 0, staged_end = 0, o_err = 0, err_bytes = 0, dev_end = 0;
    double chi2_threshold = 0;
};

// Plans the layout of P problems at device base d (nullptr: plan only, to
// learn dev_end) and, with d set, packs the staged block into the pinned
// buffer and queues its upload on the context stream.
static int lba_plan_stage(orbx_ctx* ctx, int P, const orbx_ba_problem* probs, uint8_t* d, LbaPlan& L)
{
    for (int i = 0; i < P; i++) {
        const orbx_ba_problem& p = probs[i];
        if (p.n_poses < 0 || p.n_points < 0 || p.n_edges < 0) return ORBX_ERR_ARG;
        // the fixed-point limb sums are exact for < 2^22 contributions per
        // entry of the reduced system (one per point); edge records hold the
        // pose index in 16 bits and its block in 15
        if (p.n_points >= (1 << 22) || p.n_poses > 32767) return ORBX_ERR_UNSUPPORTED;
    }
    // the sizes-only call before this one (lba_run: plan, allocate, stage)
    // checked the same batch: reuse its verdicts
    const bool checked = d && L.P == P && L.d == nullptr && L.n_edges.size() == (size_t)P;
    const bool prev_float = L.float_rec;
    std::vector<uint8_t> bad_edge(P, 0), not_float(P, 0);
    if (!checked)
    host_parallel(P, [&](int i) {
        const orbx_ba_problem& p = probs[i];
        for (int e = 0; e < p.n_edges; e++) {
            if (p.edge_point[e] < 0 || p.edge_point[e] >= p.n_points || p.edge_pose[e] < 0 || p.edge_pose[e] >= p.n_poses)
                bad_edge[i] = 1;
            // the reference's observations (cv::KeyPoint::pt) and information
            // (mvInvLevelSigma2) are floats: stored as such when exact
            const double v[3] = {p.edge_obs[2 * e], p.edge_obs[2 * e + 1], p.edge_inv_sigma2[e]};
            for (double x : v) not_float[i] |= (double)(float)x != x;
        }
    });
    bool float_rec = checked ? prev_float : true;
    for (int i = 0; i < P && !checked; i++) {
        if (bad_edge[i]) return ORBX_ERR_ARG;
        float_rec = float_rec && !not_float[i];
    }
    L = LbaPlan{};
    L.float_rec = float_rec;
    const size_t rec_bytes = float_rec ? sizeof(EdgeRecF) : sizeof(EdgeRecD);
    L.P = P;
    L.d = d;
    L.chi2_threshold = P > 0 ? probs[0].chi2_threshold : 0;
    L.pl.resize(P);
    L.offs.assign(3 * (size_t)P, 0);
    L.n_poses.resize(P);
    L.n_points.resize(P);
    L.n_edges.resize(P);
    std::vector<LbaPlay>& pl = L.pl;
    size_t at = 0;
    for (int i = 0; i < P; i++) {
        const orbx_ba_problem& p = probs[i];
        L.n_poses[i] = p.n_poses;
        L.n_points[i] = p.n_points;
        L.n_edges[i] = p.n_edges;
        pl[i].pose = at;    at += align256(7 * (size_t)p.n_poses * 8);
        pl[i].point = at;   at += align256(3 * (size_t)p.n_points * 8);
    }
    L.result_bytes = at;
    for (int i = 0; i < P; i++) {
        const orbx_ba_problem& p = probs[i];
        pl[i].cam = at;     at += align256(4 * (size_t)p.n_poses * 8);
        L.offs[3 * i] = L.eacc;
        L.offs[3 * i + 1] = L.pacc;
        L.eacc += p.n_edges;
        L.pacc += p.n_points;
    }
    L.o_all_nobs = at; at += align256(4 * (size_t)L.pacc);
    L.o_all_st = at;   at += align256((size_t)L.eacc);
    L.o_all_bad = at;  at += align256((size_t)L.pacc);
    L.o_offs = at;     at += align256(L.offs.size() * 8);
    L.o_nout = at;     at += 8 * (size_t)P;             // outliers per problem, per pass
    L.o_stats = at;    at += sizeof(LbaStatRec) * 2 * (size_t)P;
    L.o_failed = at;   at += align256(8);
    L.base_bytes = at;
    // Both optimize() calls' structures are built on the device: the first
    // from the caller's arrays (k_lba_build), the second from the first's
    // after the first outlier pass (k_lba_rebuild), so the host only stages
    // the problems, and both passes run back to back after one upload.
    constexpr int kRaw = 7, kArr = 7;
    std::vector<size_t> so_raw(kRaw * (size_t)P), so(kArr * (size_t)P), so1(kArr * (size_t)P);
    std::vector<int> nfree(P, 0);
    host_parallel(P, [&](int i) {
        int c = 0;
        for (int k = 0; k < probs[i].n_poses; k++) c += !probs[i].pose_fixed[k];
        nfree[i] = c;
    });
    auto raw_bytes = [&](const orbx_ba_problem& p, size_t (&bytes)[kRaw]) {
        const size_t E = p.n_edges, NP = p.n_poses, NL = p.n_points;
        const size_t b[kRaw] = {E * 4, E * 4, E * 16, E * 8, NP, NP * 8, NL * 8};
        for (int k = 0; k < kRaw; k++) bytes[k] = b[k];
    };
    // per pass: records, e_orig, iv_pose, iv_point, le_ptr, pe_ptr, pe_idx
    auto arr_bytes = [&](int i, size_t (&bytes)[kArr]) {
        const orbx_ba_problem& p = probs[i];
        const size_t E = p.n_edges, NP = nfree[i], NL = p.n_points;
        const size_t b[kArr] = {E * rec_bytes, E * 4, NP * 4, NL * 4, (NL + 1) * 4, (NP + 1) * 4, E * 8};
        for (int k = 0; k < kArr; k++) bytes[k] = b[k];
    };
    size_t end = L.base_bytes;
    for (int i = 0; i < P; i++) {
        size_t bytes[kRaw];
        raw_bytes(probs[i], bytes);
        for (int k = 0; k < kRaw; k++) {
            so_raw[kRaw * i + k] = end;
            end += align256(bytes[k]);
        }
    }
    L.o_devs = end;
    end += align256(sizeof(LbaDev) * P);
    L.o_devs1 = end;
    end += align256(sizeof(LbaDev) * P);
    L.staged_end = end;
    // device-only: the points' LM backups and the per-edge errors (zeroed
    // on the device); the poses' backups live in LDS
    for (int i = 0; i < P; i++) {
        const orbx_ba_problem& p = probs[i];
        pl[i].pointbk = end; end += align256(3 * (size_t)p.n_points * 8);
    }
    L.o_err = end;
    for (int i = 0; i < P; i++) {
        pl[i].err = end;
        end += align256(2 * (size_t)probs[i].n_edges * 8);
    }
    L.err_bytes = end - L.o_err;
    for (int pass = 0; pass < 2; pass++)
        for (int i = 0; i < P; i++) {
            size_t bytes[kArr];
            arr_bytes(i, bytes);
            for (int k = 0; k < kArr; k++) {
                (pass == 0 ? so : so1)[kArr * i + k] = end;
                end += align256(bytes[k]);
            }
        }
    // k_lba_iteration's dynamic LDS for the batch: the poses (q, t, R,
    // camera), the free poses' backups and the pose solution, and the reduced
    // system in front of them when the largest one fits beside them
    int np_max = 0, nf_max = 0;
    for (int i = 0; i < P; i++) {
        np_max = std::max(np_max, probs[i].n_poses);
        nf_max = std::max(nf_max, nfree[i]);
    }
    const long long non_s = (long long)np_max * kPz + (long long)nf_max * kPbk + 6LL * nf_max;
    if (non_s > kLdsCap) return ORBX_ERR_UNSUPPORTED;   // hundreds of keyframes: not a local BA
    const long long sys_max = lba_sys_doubles(6LL * nf_max);
    const bool s_in_lds = sys_max + non_s <= kLdsCap;
    L.lay.s_doubles = s_in_lds ? (int)sys_max : 0;
    L.lay.pz_off = L.lay.s_doubles;
    L.lay.pbk_off = L.lay.pz_off + np_max * kPz;
    L.lay.xp_off = L.lay.pbk_off + nf_max * kPbk;
    L.lds_bytes = (size_t)(L.lay.xp_off + 6 * nf_max + 1) * 8;
    L.lay.bp_off = L.lay.xp_off + 6 * nf_max;
    L.lay.stage_off = L.lay.bp_off + 6 * nf_max + 1;
    L.lds_split_bytes = (size_t)L.lay.stage_off * 8 + lba_staged_bytes();
    L.nfree0 = P > 0 ? nfree[0] : 0;
    if (P == 1 && d) {
        std::vector<int> obs(probs[0].n_points, 0);
        for (int e = 0; e < probs[0].n_edges; e++) L.max_obs0 = std::max(L.max_obs0, ++obs[probs[0].edge_point[e]]);
    }
    // device-only scratch, sized by the free poses, every point and edge:
    // ce (k_lba_build / k_lba_rebuild maps, then the point order), hp, hl,
    // dl, S (the reduced system when it lives in global memory), ew
    constexpr int kSc = 6;
    std::vector<size_t> sc(kSc * (size_t)P);
    for (int i = 0; i < P; i++) {
        const orbx_ba_problem& p = probs[i];
        const size_t nE = p.n_edges, nL = p.n_points, n = 6 * (size_t)nfree[i];
        const size_t sys = (size_t)lba_sys_doubles((long long)n);
        const size_t bytes[kSc] = {(nE + 2 * (size_t)p.n_poses + 3 * nL + 8) * 4, 27 * (size_t)nfree[i] * 8,
                                   9 * nL * 8, 12 * nL * 8, s_in_lds ? 8 : sys * 8, nE * 8};
        for (int k = 0; k < kSc; k++) {
            sc[kSc * i + k] = end;
            end += align256(bytes[k]);
        }
    }
    L.dev_end = end;
    if (!d) return ORBX_OK;
    int r;
    if ((r = ensure_pinned(ctx, L.staged_end)) != ORBX_OK) return r;
    uint8_t* hb = static_cast<uint8_t*>(ctx->host_pinned);
    std::vector<LbaDev> devs(P), devs1(P);
    // fill the staged bytes on host threads
    host_parallel(P, [&](int i) {
        const orbx_ba_problem& p = probs[i];
        double* pose = reinterpret_cast<double*>(hb + pl[i].pose);
        for (int k = 0; k < p.n_poses; k++) {
            for (int j = 0; j < 4; j++) pose[7 * k + j] = p.pose_q[4 * k + j];
            for (int j = 0; j < 3; j++) pose[7 * k + 4 + j] = p.pose_t[3 * k + j];
        }
        std::memcpy(hb + pl[i].point, p.points, 3 * (size_t)p.n_points * 8);
        std::memcpy(hb + pl[i].cam, p.pose_cam, 4 * (size_t)p.n_poses * 8);
        std::memcpy(hb + L.o_all_nobs + 4 * (size_t)L.offs[3 * i + 1], p.point_nobs, 4 * (size_t)p.n_points);
        std::memset(hb + L.o_all_st + L.offs[3 * i], 0, (size_t)p.n_edges);
        std::memset(hb + L.o_all_bad + L.offs[3 * i + 1], 0, (size_t)p.n_points);
        const void* src[kRaw] = {p.edge_pose, p.edge_point, p.edge_obs, p.edge_inv_sigma2,
                                 p.pose_fixed, p.pose_id, p.point_id};
        size_t rb[kRaw];
        raw_bytes(p, rb);
        for (int k = 0; k < kRaw; k++)
            if (rb[k]) std::memcpy(hb + so_raw[kRaw * i + k], src[k], rb[k]);
        auto fill = [&](LbaDev& D, const size_t* o) {
            D = LbaDev{};
            D.nposes_all = p.n_poses;
            D.npoints_all = p.n_points;
            D.nedges_all = p.n_edges;
            D.pose = reinterpret_cast<double*>(d + pl[i].pose);
            D.point = reinterpret_cast<double*>(d + pl[i].point);
            D.point_bk = reinterpret_cast<double*>(d + pl[i].pointbk);
            D.cam = reinterpret_cast<const double*>(d + pl[i].cam);
            D.err = reinterpret_cast<double*>(d + pl[i].err);
            D.rec = d + o[0];
            D.e_orig = reinterpret_cast<const int*>(d + o[1]);
            D.iv_pose = reinterpret_cast<const int*>(d + o[2]);
            D.iv_point = reinterpret_cast<const int*>(d + o[3]);
            D.le_ptr = reinterpret_cast<const int*>(d + o[4]);
            D.pe_ptr = reinterpret_cast<const int*>(d + o[5]);
            D.pe_idx = reinterpret_cast<const int2*>(d + o[6]);
            const size_t* c = &sc[kSc * i];
            D.ce = reinterpret_cast<int*>(d + c[0]);
            D.hp = reinterpret_cast<double*>(d + c[1]);
            D.hl = reinterpret_cast<double*>(d + c[2]);
            D.dl = reinterpret_cast<double*>(d + c[3]);
            D.S = reinterpret_cast<double*>(d + c[4]);
            D.ew = reinterpret_cast<double*>(d + c[5]);
            const size_t* q = &so_raw[kRaw * i];
            D.r_edge_pose = reinterpret_cast<const int*>(d + q[0]);
            D.r_edge_point = reinterpret_cast<const int*>(d + q[1]);
            D.r_edge_obs = reinterpret_cast<const double*>(d + q[2]);
            D.r_edge_isig = reinterpret_cast<const double*>(d + q[3]);
            D.r_pose_fixed = d + q[4];
            D.r_pose_id = reinterpret_cast<const long long*>(d + q[5]);
            D.r_point_id = reinterpret_cast<const long long*>(d + q[6]);
            D.huber_delta = p.huber_delta;
            D.status = kRunning;
            D.ni = 2;
        };
        fill(devs[i], &so[kArr * i]);     // counts and contents: k_lba_build
        fill(devs1[i], &so1[kArr * i]);   // counts and contents: k_lba_rebuild
    });
    std::memcpy(hb + L.o_offs, L.offs.data(), L.offs.size() * 8);
    std::memset(hb + L.o_nout, 0, L.base_bytes - L.o_nout);   // counts, statistics, flag (k_lba_build zeroes them too)
    std::memcpy(hb + L.o_devs, devs.data(), sizeof(LbaDev) * P);
    std::memcpy(hb + L.o_devs1, devs1.data(), sizeof(LbaDev) * P);
    ORBX_HIP_CHECK(hipMemcpyAsync(d, hb, L.staged_end, hipMemcpyHostToDevice, ctx->stream));
    return ORBX_OK;
}

// Workgroups for a batch of one problem (orbx_lba_set_workgroups): 1 for
// batches, for reduced systems too large for LDS, for a point seen by more
// than kSE keyframes (schur_staged's chunk) and for problems with few
// points; else the context's setting, or by default one workgroup per 32
// points, at most 64 (each workgroup's share of the Schur complement then
// costs less than the solve every workgroup repeats).
static int lba_split_workgroups(const orbx_ctx* ctx, const LbaPlan& L)
{
    if (L.P != 1 || L.lay.s_doubles == 0 || ctx->lba_workgroups == 1 || ctx->lba_force_single) return 1;
    if (L.lds_split_bytes + 2048 > 160 * 1024 || L.max_obs0 > kSE) return 1;
    const int nL = L.n_points[0];
    if (ctx->lba_workgroups > 1) return std::min(ctx->lba_workgroups, 256);
    if (nL < 128) return 1;
    return std::min(64, (nL + 31) / 32);
}

// How many k_lba_split<Rec> workgroups of `lds` dynamic LDS bytes the device
// holds at once (occupancy per CU x CUs): the grid barrier waits for all G,
// so G above this would spin until the barrier's bound.  Cached per record
// type and LDS size; 0 when the query fails.
template <class Rec>
static int lba_split_capacity(orbx_ctx* ctx, size_t lds)
{
    const int k = std::is_same<Rec, EdgeRecF>::value ? 1 : 0;
    if (ctx->lba_split_cap_lds[k] != lds || ctx->lba_split_cap[k] == 0) {
        int per_cu = 0, cus = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_lba_split<Rec>, kLbaThreads, lds) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device) != hipSuccess)
            return 0;
        ctx->lba_split_cap[k] = per_cu * cus;
        ctx->lba_split_cap_lds[k] = lds;
    }
    int cap = ctx->lba_split_cap[k];
    if (ctx->lba_dbg_cap > 0) cap = std::min(cap, ctx->lba_dbg_cap);
    return cap;
}

// Cooperative launches where the device offers them (the runtime then
// refuses a grid that cannot be co-resident instead of starting it).
static bool lba_split_coop(orbx_ctx* ctx)
{
    if (ctx->lba_split_coop < 0) {
        int v = 0;
        ctx->lba_split_coop =
            hipDeviceGetAttribute(&v, hipDeviceAttributeCooperativeLaunch, ctx->device) == hipSuccess && v ? 1 : 0;
    }
    return ctx->lba_split_coop != 0;
}

// Queues both optimize() passes of a staged batch on the context stream:
// k_lba_build, iterations, outliers, k_lba_rebuild, iterations, outliers.
// With abort flags (per problem, entries may be null) each iteration is a
// launch and the host polls the flags (and the problems' status) between
// them, which synchronises; an aborted problem's later iterations return at
// once (g2o's force-stop flag, sparse_optimizer.cpp:394-396).  Without flags
// each pass is one launch of all its iterations and nothing waits.
template <class Rec>
static int lba_launch_t(orbx_ctx* ctx, const LbaPlan& L, int iters0, int iters1,
                        const volatile uint8_t* const* aborts)
{
    const int P = L.P;
    uint8_t* d = L.d;
    // k_lba_split's buffers (a batch of one problem over G workgroups)
    LbaSplit X{};
    int G = lba_split_workgroups(ctx, L);
    if (G > 1) {
        // no more workgroups than the device holds at once (a partitioned
        // device, a large setting): fewer give the same bits
        const int cap = lba_split_capacity<Rec>(ctx, L.lds_split_bytes);
        G = std::min(G, cap);
        if (G < 2) G = 1;
    }
    ctx->lba_last_workgroups = G;
    if (G > 1) {
        const long long nL = L.n_points[0], limbs = lba_sys_doubles(6LL * L.nfree0);
        size_t o = 0;
        auto take = [&](size_t bytes) {
            const size_t at = o;
            o += align256(bytes);
            return at;
        };
        const size_t o_bar = take(64), o_wmax = take(32 * (size_t)G), o_wbad = take(8 * (size_t)G),
                     o_chi = take(8 * (size_t)nL), o_sc = take(24 * (size_t)nL), o_tot = take(8 * (size_t)limbs),
                     o_slabs = take(8 * (size_t)limbs * G);
        if (o > ctx->lba_split_bytes) {
            if (ctx->lba_split) (void)hipFree(ctx->lba_split);
            ctx->lba_split = nullptr;
            ctx->lba_split_bytes = 0;
            if (hipMalloc(&ctx->lba_split, o) != hipSuccess) return ORBX_ERR_NOMEM;
            ctx->lba_split_bytes = o;
        }
        uint8_t* b = static_cast<uint8_t*>(ctx->lba_split);
        X.bar = reinterpret_cast<unsigned*>(b + o_bar);
        X.wmax = reinterpret_cast<double*>(b + o_wmax);
        X.wbad = reinterpret_cast<int*>(b + o_wbad);
        X.chi_pt = reinterpret_cast<double*>(b + o_chi);
        X.sc_pt = reinterpret_cast<double*>(b + o_sc);
        X.total = reinterpret_cast<fx_t*>(b + o_tot);
        X.slabs = reinterpret_cast<fx_t*>(b + o_slabs);
        X.G = G;
        X.limbs = (int)limbs;
    }
    // k_lba_build also zeroes the errors, the outlier counts and (G > 1) the
    // barrier words; k_lba_outliers re-arms the arrival counter after a pass
    int* n_out = reinterpret_cast<int*>(d + L.o_nout);
    int* failed = reinterpret_cast<int*>(d + L.o_failed);
    timer_begin(ctx, "lba_build");
    hipLaunchKernelGGL(k_lba_build<Rec>, dim3(P), dim3(kLbaThreads), 0, ctx->stream,
                       reinterpret_cast<LbaDev*>(d + L.o_devs), n_out, P, X.bar, failed);
    timer_end(ctx, "lba_build");
    ORBX_HIP_CHECK(hipGetLastError());
    if (G > 1 && ctx->lba_dbg_fail > 0) {   // test hook: every barrier of this solve reports a timeout
        ORBX_HIP_CHECK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(X.bar + 1), 1, 1, ctx->stream));
        ctx->lba_dbg_fail--;
    }
    const bool coop = G > 1 && lba_split_coop(ctx);
    // one layout for both passes: the second pass's systems are no larger
    const size_t lds = L.lds_bytes;
    // the reduced systems in LDS (when the batch's largest fits) or in global memory
    auto kern = L.lay.s_doubles > 0 ? k_lba_iteration<Rec, true> : k_lba_iteration<Rec, false>;
    bool polled = false;
    for (int i = 0; aborts && i < P; i++) polled |= aborts[i] != nullptr;
    std::vector<LbaDev> hv(polled ? P : 0);
    std::vector<uint8_t> stopped(P, 0);   // abort written to the device
    for (int pass = 0; pass < 2; pass++) {
        LbaDev* dd = reinterpret_cast<LbaDev*>(d + (pass == 0 ? L.o_devs : L.o_devs1));
        if (pass == 1) {
            timer_begin(ctx, "lba_rebuild");
            hipLaunchKernelGGL(k_lba_rebuild<Rec>, dim3(P), dim3(kLbaThreads), 0, ctx->stream,
                               reinterpret_cast<const LbaDev*>(d + L.o_devs), dd, d + L.o_all_st,
                               reinterpret_cast<const long long*>(d + L.o_offs));
            timer_end(ctx, "lba_rebuild");
            ORBX_HIP_CHECK(hipGetLastError());
        }
        const int iters = pass == 0 ? iters0 : iters1;
        if (pass == 1)   // k_lba_rebuild carries each problem's abort into the second pass
            for (int i = 0; i < P; i++) stopped[i] = 0;
        for (int it = 0; it < iters; it++) {
            if (polled) {
                const int one = 1;
                bool any = false, all = true;
                for (int i = 0; i < P; i++) {
                    const bool stop = aborts[i] && *aborts[i];
                    if (stop && !stopped[i]) {
                        ORBX_HIP_CHECK(hipMemcpyAsync(reinterpret_cast<uint8_t*>(dd + i) + offsetof(LbaDev, abort),
                                                      &one, 4, hipMemcpyHostToDevice, ctx->stream));
                        stopped[i] = 1;
                        any = true;
                    }
                    all &= stop;
                }
                if (any) ORBX_HIP_CHECK(hipStreamSynchronize(ctx->stream));   // &one outlives the copy
                if (all) break;
            }
            timer_begin(ctx, "lba_iter");
            // without abort flags a pass's iterations run in one launch
            const int n_it = polled ? 1 : iters;
            if (G > 1) {
                if (polled && it > 0)   // a launch per iteration: re-arm the arrival counter
                    ORBX_HIP_CHECK(hipMemsetAsync(X.bar, 0, 4, ctx->stream));
                if (coop) {
                    int it_arg = it, n_arg = n_it;
                    LbaLds lay = L.lay;
                    void* args[] = {&dd, &it_arg, &n_arg, &lay, &X};
                    ORBX_HIP_CHECK(hipLaunchCooperativeKernel(reinterpret_cast<const void*>(k_lba_split<Rec>), dim3(G),
                                                              dim3(kLbaThreads), args, L.lds_split_bytes, ctx->stream));
                } else {
                    hipLaunchKernelGGL(k_lba_split<Rec>, dim3(G), dim3(kLbaThreads), L.lds_split_bytes, ctx->stream,
                                       dd, it, n_it, L.lay, X);
                }
            } else {
                hipLaunchKernelGGL(kern, dim3(P), dim3(kLbaThreads), lds, ctx->stream, dd, it, n_it, L.lay);
            }
            timer_end(ctx, "lba_iter");
            ORBX_HIP_CHECK(hipGetLastError());
            // With an abort flag the host polls it between iterations (where
            // g2o polls its force-stop flag), which needs the device state;
            // without one, the launch above ran the whole pass.
            if (!polled) break;
            {
                ORBX_HIP_CHECK(hipMemcpyAsync(hv.data(), dd, sizeof(LbaDev) * P, hipMemcpyDeviceToHost, ctx->stream));
                ORBX_HIP_CHECK(hipStreamSynchronize(ctx->stream));
                bool running = false;
                for (int i = 0; i < P; i++) running |= hv[i].status == kRunning && !hv[i].abort;
                if (!running) break;
            }
        }
        timer_begin(ctx, "lba_outliers");
        hipLaunchKernelGGL(k_lba_outliers<Rec>, dim3(P, G > 1 ? 16 : 1), dim3(256), 0, ctx->stream, dd,
                           reinterpret_cast<int*>(d + L.o_all_nobs), d + L.o_all_st, d + L.o_all_bad, pass + 1,
                           L.chi2_threshold, n_out + pass * P, reinterpret_cast<const long long*>(d + L.o_offs),
                           reinterpret_cast<LbaStatRec*>(d + L.o_stats) + pass * P, X.bar, failed);
        timer_end(ctx, "lba_outliers");
        ORBX_HIP_CHECK(hipGetLastError());
    }
    return ORBX_OK;
}

static int lba_launch(orbx_ctx* ctx, const LbaPlan& L, int iters0, int iters1, const volatile uint8_t* const* aborts)
{
    return L.float_rec ? lba_launch_t<EdgeRecF>(ctx, L, iters0, iters1, aborts)
                       : lba_launch_t<EdgeRecD>(ctx, L, iters0, iters1, aborts);
}

// Reads a solved batch back (synchronising the context stream): poses and
// points into the problems' arrays, edge / point flags, statistics.
static int lba_readback(orbx_ctx* ctx, const LbaPlan& L, orbx_ba_problem* probs, uint8_t* const* edge_status,
                        uint8_t* const* point_bad, orbx_ba_stats* stats)
{
    const int P = L.P;
    uint8_t* d = L.d;
    int r;
    if ((r = ensure_pinned(ctx, L.base_bytes)) != ORBX_OK) return r;
    uint8_t* hb = static_cast<uint8_t*>(ctx->host_pinned);
    // one copy: poses, points, cameras, observation counts, edge status,
    // point flags, offsets, outlier counts, per-pass statistics, failed flag
    ORBX_HIP_CHECK(hipMemcpyAsync(hb, d, L.base_bytes, hipMemcpyDeviceToHost, ctx->stream));
    ORBX_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    // a k_lba_split barrier timed out: nothing is written back (the caller's
    // arrays keep their input) and the callers below re-run on one workgroup
    ctx->lba_split_timed_out = *reinterpret_cast<const int*>(hb + L.o_failed) != 0;
    if (ctx->lba_split_timed_out) return ORBX_ERR_HIP;
    const int* nout = reinterpret_cast<const int*>(hb + L.o_nout);
    const LbaStatRec* sr = reinterpret_cast<const LbaStatRec*>(hb + L.o_stats);
    const uint8_t* all_st = hb + L.o_all_st;
    if (stats)
        for (int pass = 0; pass < 2; pass++)
            for (int i = 0; i < P; i++) {
                const LbaStatRec& o = sr[pass * (size_t)P + i];
                stats[i].iterations[pass] = o.iterations;
                stats[i].levenberg_trials[pass] = o.trials;
                stats[i].chi2_initial[pass] = o.chi2_initial;
                stats[i].chi2_final[pass] = o.last_chi;
                stats[i].n_outliers[pass] = nout[pass * (size_t)P + i];
                stats[i].not_posdef += o.not_posdef;
            }
    host_parallel(P, [&](int i) {
        orbx_ba_problem& p = probs[i];
        const double* pose = reinterpret_cast<const double*>(hb + L.pl[i].pose);
        for (int k = 0; k < p.n_poses; k++) {
            for (int j = 0; j < 4; j++) p.pose_q[4 * k + j] = pose[7 * k + j];
            for (int j = 0; j < 3; j++) p.pose_t[3 * k + j] = pose[7 * k + 4 + j];
        }
        std::memcpy(p.points, hb + L.pl[i].point, 3 * (size_t)p.n_points * 8);
        if (edge_status && edge_status[i]) std::memcpy(edge_status[i], all_st + L.offs[3 * i], p.n_edges);
        if (point_bad && point_bad[i]) std::memcpy(point_bad[i], hb + L.o_all_bad + L.offs[3 * i + 1], p.n_points);
    });
    return ORBX_OK;
}

// Solves P problems from host arrays; per problem a workgroup.  The
// problems' pose/point arrays are updated in place.  One planned layout in
// the context scratch, filled by host threads straight into the pinned
// buffer, one copy each way.
static int lba_run(orbx_ctx* ctx, int P, orbx_ba_problem* probs, int iters0, int iters1,
                   const volatile uint8_t* const* aborts, uint8_t* const* edge_status, uint8_t* const* point_bad,
                   orbx_ba_stats* stats)
{
    ctx_enter(ctx);
    LbaPlan L;
    int r = lba_plan_stage(ctx, P, probs, nullptr, L);   // sizes only
    if (r != ORBX_OK) return r;
    if (L.dev_end > ctx->scratch_bytes && (r = ensure_scratch(ctx, L.dev_end)) != ORBX_OK) return r;
    if ((r = lba_plan_stage(ctx, P, probs, static_cast<uint8_t*>(ctx->scratch), L)) != ORBX_OK) return r;
    if ((r = lba_launch(ctx, L, iters0, iters1, aborts)) != ORBX_OK) return r;
    r = lba_readback(ctx, L, probs, edge_status, point_bad, stats);
    if (r == ORBX_ERR_HIP && ctx->lba_split_timed_out && ctx->lba_split_fallback && !ctx->lba_force_single) {
        // the split kernel's workgroups were not all resident (another
        // context's kernels held the CUs): the same solve on one workgroup,
        // restaged from the untouched input; same bits
        ctx->lba_force_single = true;
        r = lba_run(ctx, P, probs, iters0, iters1, aborts, edge_status, point_bad, stats);
        ctx->lba_force_single = false;
    }
    return r;
}

// Device-resident form (orbx_lba_stage / _run / _fetch): the batch lives in
// a buffer of its own, with a copy of the staged block's mutable parts
// (poses, points, counts and flags; both LbaDev arrays) that every run
// restores first, so each run starts from the staged problems.
struct LbaResident {
    LbaPlan plan;
    void* dev = nullptr;
    void* image = nullptr;
    size_t dev_bytes = 0, image_bytes = 0;
    bool solved = false;
};

void lba_resident_free(orbx_ctx* ctx)
{
    if (!ctx->lba_res) return;
    if (ctx->lba_res->dev) (void)hipFree(ctx->lba_res->dev);
    if (ctx->lba_res->image) (void)hipFree(ctx->lba_res->image);
    delete ctx->lba_res;
    ctx->lba_res = nullptr;
}

static int lba_stage_resident(orbx_ctx* ctx, int P, const orbx_ba_problem* probs)
{
    ctx_enter(ctx);
    if (!ctx->lba_res) ctx->lba_res = new (std::nothrow) LbaResident();
    if (!ctx->lba_res) return ORBX_ERR_NOMEM;
    LbaResident& R = *ctx->lba_res;
    // the previous staging is dropped before anything is freed: a stage that
    // fails part-way leaves no plan pointing into released buffers, and
    // orbx_lba_run / _fetch refuse the context until a stage succeeds
    ORBX_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    R.plan = LbaPlan{};
    R.solved = false;
    LbaPlan L;
    int r = lba_plan_stage(ctx, P, probs, nullptr, L);
    if (r != ORBX_OK) return r;
    if (L.dev_end > R.dev_bytes) {
        if (R.dev) (void)hipFree(R.dev);
        R.dev = nullptr;
        R.dev_bytes = 0;
        if (hipMalloc(&R.dev, L.dev_end) != hipSuccess) return ORBX_ERR_NOMEM;
        R.dev_bytes = L.dev_end;
    }
    if (L.staged_end > R.image_bytes) {
        if (R.image) (void)hipFree(R.image);
        R.image = nullptr;
        R.image_bytes = 0;
        if (hipMalloc(&R.image, L.staged_end) != hipSuccess) return ORBX_ERR_NOMEM;
        R.image_bytes = L.staged_end;
    }
    if ((r = lba_plan_stage(ctx, P, probs, static_cast<uint8_t*>(R.dev), L)) != ORBX_OK) return r;
    ORBX_HIP_CHECK(hipMemcpyAsync(R.image, R.dev, L.staged_end, hipMemcpyDeviceToDevice, ctx->stream));
    ORBX_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    R.plan = std::move(L);
    return ORBX_OK;
}

static int lba_run_resident(orbx_ctx* ctx, int iters0, int iters1, const volatile uint8_t* const* aborts)
{
    if (!ctx->lba_res || ctx->lba_res->plan.P == 0) return ORBX_ERR_ARG;
    ctx_enter(ctx);
    ctx->lba_res_iters[0] = iters0;
    ctx->lba_res_iters[1] = iters1;
    LbaResident& R = *ctx->lba_res;
    const LbaPlan& L = R.plan;
    uint8_t* d = static_cast<uint8_t*>(R.dev);
    const uint8_t* img = static_cast<const uint8_t*>(R.image);
    // mutable parts of the staged block: [0, base_bytes) and the LbaDev
    // arrays (the raw edge / id arrays between them are only read)
    ORBX_HIP_CHECK(hipMemcpyAsync(d, img, L.base_bytes, hipMemcpyDeviceToDevice, ctx->stream));
    ORBX_HIP_CHECK(hipMemcpyAsync(d + L.o_devs, img + L.o_devs, L.staged_end - L.o_devs, hipMemcpyDeviceToDevice,
                                  ctx->stream));
    R.solved = true;
    return lba_launch(ctx, L, iters0, iters1, aborts);
}

#ifdef ORBX_LBA_PROFILE
// llt_solve alone (diagnostic build): reps factorisations of the packed
// system Sin (n x n plus the right-hand-side row) in LDS, cycles summed
__global__ void __launch_bounds__(kLbaThreads) k_llt_bench(const double* Sin, int n, int reps, double* xout,
                                                            unsigned long long* cyc, int mode)
{
    extern __shared__ double lds[];
    const int M = n * (n + 1) / 2;
    double* S = lds;
    double* xp = lds + M + 2 * n;
    unsigned long long tot = 0;
    if (mode >= 2) {   // latency probes: 1000 dependent f64 multiplies (2) or rsqrt_nr (3); raw v_rsq_f64 (4)
        if (mode == 4) {
            for (int k = threadIdx.x; k < n; k += kLbaThreads) xout[k] = __builtin_amdgcn_rsq(Sin[k]);
            return;
        }
        double v = Sin[threadIdx.x], a = Sin[n + threadIdx.x];
        if (mode == 5 || mode == 6) {   // 1000 workgroup barriers (5); 1000 dependent LDS loads (6)
            int* q = reinterpret_cast<int*>(lds);
            for (int k = threadIdx.x; k < 1024; k += kLbaThreads) q[k] = (k + 1) & 1023;
            LBA_SYNC();
            int j = threadIdx.x & 63;
            const unsigned long long t0 = lba_stamp();
            if (mode == 5)
                for (int i = 0; i < 1000; i++) LBA_SYNC();
            else
                for (int i = 0; i < 1000; i++) j = q[j];
            const unsigned long long t1 = lba_stamp();
            if (threadIdx.x == 0) {
                *cyc = t1 - t0;
                xout[0] = j;
            }
            return;
        }
        const unsigned long long t0 = lba_stamp();
        if (mode == 2)
            for (int i = 0; i < 1000; i++) v = v * a;
        else
            for (int i = 0; i < 1000; i++) v = rsqrt_nr(v);
        const unsigned long long t1 = lba_stamp();
        if (threadIdx.x == 0) {
            *cyc = t1 - t0;
            xout[0] = v;
        }
        return;
    }
    for (int r = 0; r < reps; r++) {
        for (int k = threadIdx.x; k < M + n; k += kLbaThreads) S[k] = Sin[k];
        LBA_SYNC();
        const unsigned long long t0 = lba_stamp();
        const bool ok = llt_solve(S, xp, n);
        const unsigned long long t1 = lba_stamp();
        tot += t1 - t0;
        if (!ok) break;
    }
    for (int k = threadIdx.x; k < n; k += kLbaThreads) xout[k] = xp[k];
    if (threadIdx.x == 0) *cyc = tot;
}
#endif

}  // namespace orbx

extern "C" {

#ifdef ORBX_LBA_PROFILE
int orbx_debug_llt_waves(unsigned long long* out)
{
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(orbx::g_llt_wave), sizeof(unsigned long long) * 32) == hipSuccess ? 0 : -2;
}

int orbx_debug_lba_prof(unsigned long long* out)
{
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(orbx::g_lba_prof), sizeof(unsigned long long) * 32) == hipSuccess ? 0 : -2;
}

int orbx_debug_llt_bench(const double* Sin_host, int n, int reps, double* x_host, unsigned long long* cycles, int mode)
{
    const int M = n * (n + 1) / 2;
    double *dS = nullptr, *dx = nullptr;
    unsigned long long* dc = nullptr;
    if (hipMalloc(&dS, (M + n) * 8) != hipSuccess || hipMalloc(&dx, n * 8) != hipSuccess || hipMalloc(&dc, 8) != hipSuccess)
        return -2;
    (void)hipMemcpy(dS, Sin_host, (M + n) * 8, hipMemcpyHostToDevice);
    const size_t lds = (size_t)(M + 3 * n) * 8;
    hipLaunchKernelGGL(orbx::k_llt_bench, dim3(1), dim3(orbx::kLbaThreads), lds, 0, dS, n, reps, dx, dc, mode);
    const bool ok = hipDeviceSynchronize() == hipSuccess;
    (void)hipMemcpy(x_host, dx, n * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(cycles, dc, 8, hipMemcpyDeviceToHost);
    (void)hipFree(dS);
    (void)hipFree(dx);
    (void)hipFree(dc);
    return ok ? 0 : -2;
}
#endif

int orbx_lba_solve(orbx_ctx* ctx, orbx_ba_problem* p, int iters0, int iters1, const volatile uint8_t* abort,
                   uint8_t* edge_status, uint8_t* point_bad, orbx_ba_stats* stats)
{
    if (!ctx || !p || iters0 < 0 || iters1 < 0) return ORBX_ERR_ARG;
    if (stats) std::memset(stats, 0, sizeof(*stats));
    uint8_t* es[1] = {edge_status};
    uint8_t* pb[1] = {point_bad};
    const volatile uint8_t* ab[1] = {abort};
    return orbx::lba_run(ctx, 1, p, iters0, iters1, ab, es, pb, stats);
}

int orbx_lba_solve_batch(orbx_ctx* ctx, int P, orbx_ba_problem* problems, int iters0, int iters1,
                         const volatile uint8_t* const* aborts, uint8_t* const* edge_status,
                         uint8_t* const* point_bad, orbx_ba_stats* stats)
{
    if (!ctx || P <= 0 || !problems || iters0 < 0 || iters1 < 0) return ORBX_ERR_ARG;
    if (stats) std::memset(stats, 0, sizeof(*stats) * P);
    return orbx::lba_run(ctx, P, problems, iters0, iters1, aborts, edge_status, point_bad, stats);
}

int orbx_lba_set_workgroups(orbx_ctx* ctx, int n)
{
    if (!ctx || n < 0 || n > 256) return ORBX_ERR_ARG;
    ctx_enter(ctx);
    ctx->lba_workgroups = n;
    return ORBX_OK;
}

int orbx_lba_get_workgroups(const orbx_ctx* ctx) { return ctx ? ctx->lba_workgroups : ORBX_ERR_ARG; }

int orbx_lba_stage(orbx_ctx* ctx, int P, const orbx_ba_problem* problems)
{
    if (!ctx || P <= 0 || !problems) return ORBX_ERR_ARG;
    return orbx::lba_stage_resident(ctx, P, problems);
}

int orbx_lba_run(orbx_ctx* ctx, int iters0, int iters1, const volatile uint8_t* const* aborts)
{
    if (!ctx || iters0 < 0 || iters1 < 0) return ORBX_ERR_ARG;
    return orbx::lba_run_resident(ctx, iters0, iters1, aborts);
}

int orbx_lba_fetch(orbx_ctx* ctx, orbx_ba_problem* problems, uint8_t* const* edge_status, uint8_t* const* point_bad,
                   orbx_ba_stats* stats)
{
    if (!ctx || !problems || !ctx->lba_res || !ctx->lba_res->solved || ctx->lba_res->plan.P == 0) return ORBX_ERR_ARG;
    const orbx::LbaPlan& L = ctx->lba_res->plan;
    for (int i = 0; i < L.P; i++)
        if (problems[i].n_poses != L.n_poses[i] || problems[i].n_points != L.n_points[i] ||
            problems[i].n_edges != L.n_edges[i])
            return ORBX_ERR_ARG;
    if (stats) std::memset(stats, 0, sizeof(*stats) * L.P);
    ctx_enter(ctx);
    int r = orbx::lba_readback(ctx, L, problems, edge_status, point_bad, stats);
    if (r == ORBX_ERR_HIP && ctx->lba_split_timed_out && ctx->lba_split_fallback) {
        // a timed-out split run (orbx::lba_run's fallback): the staged batch
        // again from its image on one workgroup, without abort polling
        ctx->lba_force_single = true;
        r = orbx::lba_run_resident(ctx, ctx->lba_res_iters[0], ctx->lba_res_iters[1], nullptr);
        ctx->lba_force_single = false;
        if (r == ORBX_OK) r = orbx::lba_readback(ctx, L, problems, edge_status, point_bad, stats);
    }
    return r;
}

/* Test hooks of the split kernel's residency handling: fail > 0 makes the
 * barriers of the next `fail` split launches report a timeout; fallback 0
 * turns the one-workgroup re-run off (the call then returns ORBX_ERR_HIP with
 * the caller's arrays untouched); cap > 0 caps the residency capacity; coop
 * -1 leaves the cooperative-launch choice to the device, 0 / 1 force it.
 * Every argument < 0 (coop < -1) leaves that setting unchanged. */
int orbx_debug_lba_split(orbx_ctx* ctx, int fail, int fallback, int cap, int coop)
{
    if (!ctx) return ORBX_ERR_ARG;
    if (fail >= 0) ctx->lba_dbg_fail = fail;
    if (fallback >= 0) ctx->lba_split_fallback = fallback != 0;
    if (cap >= 0) ctx->lba_dbg_cap = cap;
    if (coop >= -1) ctx->lba_split_coop = coop;
    return ORBX_OK;
}

int orbx_lba_last_workgroups(const orbx_ctx* ctx) { return ctx ? ctx->lba_last_workgroups : ORBX_ERR_ARG; }

}  // extern "C"
