// Local bundle adjustment on MI355X (FP64): the inner loop of
// Optimizer::LocalBundleAdjustment (src/Optimizer.cc:287-536) on the g2o
// subset it uses (BlockSolverX + Schur over the points, Levenberg).
//
// Device work per LM iteration (one 512-thread workgroup per problem, one
// launch per iteration so the caller's abort flag is polled between
// iterations exactly where SparseOptimizer::optimize polls terminate()):
//   errors    EdgeSE3ProjectXYZ::computeError per edge, Huber robust chi2
//   linearize EdgeSE3ProjectXYZ::linearizeOplus + constructQuadraticForm per
//             edge into component-major (SoA) rows; per pose (Hpp, bp) one
//             wave with a fixed butterfly reduction, per point (Hll, bl) one
//             thread in edge order
//   trial     Schur point by point (a point's edges are contiguous): Dinv,
//             db, then bs -= W_i db and S(i,j) -= W_i Dinv W_j^T for every
//             pair of its edges.  The W_i = Hpl blocks are rebuilt from the
//             edge's inputs (pose, point, observation) where they are used
//             instead of being stored per edge and re-read from HBM.  The
//             reduced camera system is accumulated in 2^-51 fixed point with
//             64-bit integer atomics (two limbs per entry, packed lower
//             triangle in LDS): integer sums do not depend on the order the
//             points arrive in, so the result is bitwise reproducible
//             (g2o sums the points sequentially in double; the two differ by
//             rounding only).  Dense LLT on the packed triangle; one-wave
//             triangular solves; back-substitution for the points; exp-map
//             update; accept / reject with g2o's rho rule
//   Raul stop rule (levenberg.cpp:154-161)
// Index structures (g2o's initializeOptimization / buildStructure) are built
// on the host once per optimize() call.
#include <algorithm>
#include <cmath>
#include <cstddef>
#include <cstring>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "orbx_device.h"
#include "orbx_internal.h"
#include "orbx_se3.h"

namespace orbx {

struct LbaDev {
    int nP, nL, nE;                // free poses, active points, active edges
    int nposes_all, npoints_all, nedges_all;
    int dim_p;                     // 6 * nP
    double* pose;                  // [nposes_all][7]: qx qy qz qw tx ty tz
    double* point;                 // [npoints_all][3]
    double* pose_bk;
    double* point_bk;
    const double* cam;             // [nposes_all][4]
    // active edges in g2o order (SoA over active index)
    const int* e_orig;             // original edge index
    const int* e_pose;             // pose index
    const int* e_point;            // point index
    const int* e_ph;               // pose hessian index or -1 (fixed)
    const int* e_lh;               // point hessian index
    const double* e_obs;           // [nE][2]
    const double* e_isig;          // [nE]
    double* err;                   // [nedges_all][2] last computed errors (original index)
    const int* iv_pose;            // [nP]
    const int* iv_point;           // [nL]
    const int* pe_ptr; const int* pe_idx;   // per free pose: active edges, edge order
    const int* le_ptr; const int* le_idx;   // per point: active edges, edge order
    const int* lc_ptr; const int* lc_idx;   // per point: Schur column (free poses, pose order)
    // scratch
    double* ce;                    // index maps of k_lba_build / k_lba_rebuild (no Hpl blocks are stored)
    double* hp;                    // [nP][27]: Hpp upper 21 | bp 6
    double* hl;                    // [nL][9]: Hll upper 6 | bl 3
    double* dl;                    // [nL][12]: Dinv 9 | db 3
    double* S;                     // reduced system, lba_sys_doubles(dim_p) (global fallback of the LDS copy)
    double* x;                     // [dim_p + 3 nL]
    double* bs;                    // [dim_p]
    double* ew;                    // [nE] robust weight rho' * invSigma2 of the linearisation
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
    int nBad, status, iterations, trials, not_posdef;
    int abort;
};

enum { kRunning = 0, kTerminated = 1 };

// Phase timing of block 0 (diagnostic build only: -DORBX_LBA_PROFILE).
#ifdef ORBX_LBA_PROFILE
__device__ unsigned long long g_lba_prof[16];
__device__ inline unsigned long long lba_stamp()
{
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
#define LBA_T0() unsigned long long _t = lba_stamp()
#define LBA_MARK(k)                                                         \
    do {                                                                    \
        __syncthreads();                                                    \
        const unsigned long long _n = lba_stamp();                          \
        if (blockIdx.x == 0 && threadIdx.x == 0) g_lba_prof[k] += _n - _t;  \
        _t = _n;                                                            \
    } while (0)
#else
#define LBA_T0()
#define LBA_MARK(k)
#endif

constexpr int kLbaThreads = 512;               // one workgroup (8 waves) per problem
constexpr int kLbaWaves = kLbaThreads / 64;
constexpr int kSchurEdges = 8;                 // per-thread LDS edge table of the Schur pass (32 KB)
#ifndef ORBX_SCHUR_GROUP
#define ORBX_SCHUR_GROUP 2
#endif
constexpr int kSchurGroup = ORBX_SCHUR_GROUP;  // edges whose W_i Dinv share one pass over the later W_j



// ---------------------------------------------------------------------------
// Block reductions in double
// ---------------------------------------------------------------------------
struct DScratch {
    double w[kLbaWaves];
    double v[4];
    int iv[4];
};

__device__ inline double wave_sum_d(double v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ inline double wave_max_d(double v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
    return v;
}

__device__ inline double block_sum_d(double v, DScratch& s)
{
    v = wave_sum_d(v);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) s.w[threadIdx.x >> 6] = v;
    __syncthreads();
    double t = 0;
    for (int i = 0; i < kLbaWaves; i++) t += s.w[i];
    return t;
}

__device__ inline double block_max_d(double v, DScratch& s)
{
    v = wave_max_d(v);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) s.w[threadIdx.x >> 6] = v;
    __syncthreads();
    double t = s.w[0];
    for (int i = 1; i < kLbaWaves; i++) t = fmax(t, s.w[i]);
    return t;
}

// ---------------------------------------------------------------------------
// Phases
// ---------------------------------------------------------------------------
__device__ inline void huber(double e2, double delta, double* rho0, double* rho1)
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

__device__ inline double edge_chi2(const LbaDev& P, int a)
{
    const int e = P.e_orig[a];
    const double s = P.e_isig[a];
    const double e0 = P.err[2 * e], e1 = P.err[2 * e + 1];
    return e0 * (s * e0) + e1 * (s * e1);
}

// EdgeSE3ProjectXYZ::computeError (types_six_dof_expmap.h:172-177) of
// active edge a at the current pose / point, with the camera-frame point
__device__ inline void edge_residual(const LbaDev& P, int a, double (&pc)[3], double& e0, double& e1)
{
    se3_map(P.pose + 7 * P.e_pose[a], P.point + 3 * P.e_point[a], pc);
    const double* c = P.cam + 4 * P.e_pose[a];
    const double u = pc[0] / pc[2] * c[0] + c[2];
    const double v = pc[1] / pc[2] * c[1] + c[3];
    e0 = P.e_obs[2 * a] - u;
    e1 = P.e_obs[2 * a + 1] - v;
}

// computeActiveErrors + activeRobustChi2
__device__ double compute_errors(LbaDev& P, DScratch& sc)
{
    double part = 0;
    for (int a = threadIdx.x; a < P.nE; a += kLbaThreads) {
        const int e = P.e_orig[a];
        double pc[3];
        edge_residual(P, a, pc, P.err[2 * e], P.err[2 * e + 1]);
        double r0, r1;
        huber(edge_chi2(P, a), P.huber_delta, &r0, &r1);
        part += r0;
    }
    __syncthreads();
    return block_sum_d(part, sc);
}

// EdgeSE3ProjectXYZ::linearizeOplus (types_six_dof_expmap.cpp:384-420) for
// active edge a: A = d e / d point (2x3), B = d e / d pose (2x6); plus the
// robust weight w = rho' * invSigma2 and the weighted error -Omega e rho'.
struct EdgeLin {
    double A[6], B[12], w, om0, om1;
};

// The Jacobians of linearizeOplus at camera-frame point pc: the
// reference's divisions by z and z^2 as products with 1/z (one division per
// edge; the values differ from g2o's in rounding only).
__device__ inline void edge_jacobians(const LbaDev& P, int a, const double (&pc)[3], double (&A)[6], double (&B)[12])
{
    const double* T = P.pose + 7 * P.e_pose[a];
    const double x = pc[0], y = pc[1];
    const double iz = 1. / pc[2], iz2 = iz * iz;
    const double* c = P.cam + 4 * P.e_pose[a];
    const double fx = c[0], fy = c[1];
    const double tmp[6] = {fx, 0, -(x * iz) * fx, 0, fy, -(y * iz) * fy};
    double R[9];
    qmat(Q{T[0], T[1], T[2], T[3]}, R);
    const double s = -iz;
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
        for (int j = 0; j < 3; j++)
            A[i * 3 + j] = (s * tmp[i * 3]) * R[j] + (s * tmp[i * 3 + 1]) * R[3 + j] + (s * tmp[i * 3 + 2]) * R[6 + j];
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

// (pc: the camera-frame point, e0 / e1 the edge's error, both at the
// linearisation point)
__device__ inline void edge_linearize_at(const LbaDev& P, int a, const double (&pc)[3], double e0, double e1, EdgeLin& L)
{
    edge_jacobians(P, a, pc, L.A, L.B);
    const double sg = P.e_isig[a];
    double r0, r1;
    huber(e0 * (sg * e0) + e1 * (sg * e1), P.huber_delta, &r0, &r1);
    L.w = r1 * sg;
    L.om0 = -(sg * e0) * r1;
    L.om1 = -(sg * e1) * r1;
}

// linearizeOplus at the errors computeActiveErrors left in P.err
__device__ inline void edge_linearize(const LbaDev& P, int a, EdgeLin& L)
{
    double pc[3];
    se3_map(P.pose + 7 * P.e_pose[a], P.point + 3 * P.e_point[a], pc);
    const int e = P.e_orig[a];
    edge_linearize_at(P, a, pc, P.err[2 * e], P.err[2 * e + 1], L);
}

// Hpl = B^T W A (6x3, row-major) of active edge a, rebuilt at the current
// pose / point with the weight linearize() stored: inside trial_solve these
// are the iteration's linearisation point (a rejected trial is undone before
// the next), so the blocks are the ones g2o's linearisation would store.
__device__ inline void edge_hpl(const LbaDev& P, int a, double (&hpl)[18])
{
    double pc[3];
    se3_map(P.pose + 7 * P.e_pose[a], P.point + 3 * P.e_point[a], pc);
    double A[6], B[12];
    edge_jacobians(P, a, pc, A, B);
    const double w = P.ew[a];   // the robust weight linearize() used
#pragma unroll
    for (int i = 0; i < 6; i++) {
        const double b0 = B[i] * w, b1 = B[6 + i] * w;
#pragma unroll
        for (int j = 0; j < 3; j++) hpl[i * 3 + j] = __fma_rn(b1, A[3 + j], b0 * A[j]);
    }
}

// constructQuadraticForm (base_binary_edge.hpp:55-120) split by owner:
//  - per free pose (one wave, lanes stride the pose's edges in edge order,
//    fixed butterfly reduction): Hpp += B^T W B, bp += B^T (-Omega e)
//  - per point (one thread, its edges in order): Hll += A^T W A,
//    bl += A^T (-Omega e).  The edges' Hpl = B^T W A blocks are not stored:
//    the Schur pass and the back-substitution rebuild them (edge_hpl).
__device__ void linearize(LbaDev& P)
{
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int p = wv; p < P.nP; p += kLbaWaves) {
        double acc[27];
#pragma unroll
        for (int v = 0; v < 27; v++) acc[v] = 0.0;
        for (int q = P.pe_ptr[p] + lane; q < P.pe_ptr[p + 1]; q += 64) {
            EdgeLin L;
            edge_linearize(P, P.pe_idx[q], L);
            int k = 0;
#pragma unroll
            for (int i = 0; i < 6; i++)
#pragma unroll
                for (int j = i; j < 6; j++) acc[k++] += (L.B[i] * L.w) * L.B[j] + (L.B[6 + i] * L.w) * L.B[6 + j];
#pragma unroll
            for (int i = 0; i < 6; i++) acc[21 + i] += L.B[i] * L.om0 + L.B[6 + i] * L.om1;
        }
#pragma unroll
        for (int v = 0; v < 27; v++) {
            const double t = wave_sum_d(acc[v]);
            if (lane == 0) P.hp[27 * p + v] = t;
        }
    }
    for (int l = threadIdx.x; l < P.nL; l += kLbaThreads) {
        double acc[9];
#pragma unroll
        for (int v = 0; v < 9; v++) acc[v] = 0.0;
        for (int q = P.le_ptr[l]; q < P.le_ptr[l + 1]; q++) {
            const int a = P.le_idx[q];
            EdgeLin L;
            edge_linearize(P, a, L);
            P.ew[a] = L.w;
            int k = 0;
#pragma unroll
            for (int i = 0; i < 3; i++)
#pragma unroll
                for (int j = i; j < 3; j++) acc[k++] += (L.A[i] * L.w) * L.A[j] + (L.A[3 + i] * L.w) * L.A[3 + j];
#pragma unroll
            for (int i = 0; i < 3; i++) acc[6 + i] += L.A[i] * L.om0 + L.A[3 + i] * L.om1;
        }
#pragma unroll
        for (int v = 0; v < 9; v++) P.hl[9 * l + v] = acc[v];
    }
    __syncthreads();
}

__device__ inline int up6(int i, int j) { return i * 6 - (i * (i - 1)) / 2 + (j - i); }   // i <= j
__device__ inline int up3(int i, int j) { return i * 3 - (i * (i - 1)) / 2 + (j - i); }
// packed lower triangle: element (i, j), j <= i
__device__ inline int pk(int i, int j) { return i * (i + 1) / 2 + j; }

// Fixed-point accumulation of the reduced camera system.  A contribution v
// (|v| < 2^40) is split as v * 2^51 ~= hi * 2^40 + lo: hi = round(v * 2^11),
// lo = round((v * 2^11 - hi) * 2^40), |lo| <= 2^39 (the split of a given v is
// always the same; bits below 2^-51 are rounded off, far below the double
// rounding of the entries, whose natural scale is >= 1 here), and both limbs
// are added with 64-bit integer atomics.  Integer addition is associative,
// so the accumulated limbs, and the double made from them, do not depend on
// the order in which threads add: the reduced system is bitwise
// reproducible.  lo sums stay exact for 2^23 contributions per entry; a
// contribution with |v| >= 2^40 (or non-finite) flags the trial, which is
// then rejected as CHOLMOD's failure would be.  Integerisation by the
// 1.5 * 2^52 magic-number addition (exact round-to-nearest for |x| < 2^51).
constexpr double kFxHi = 2048.0;                           // 2^11
constexpr double kFxLo = 1099511627776.0;                  // 2^40
constexpr double kFxInvHi = 1.0 / 2048.0;                  // 2^-11
constexpr double kFxInvLo = 1.0 / 2251799813685248.0;      // 2^-51
constexpr double kFxMax = 2251799813685248.0;              // 2^51 (of v * 2^11)
constexpr double kFxMagic = 6755399441055744.0;            // 1.5 * 2^52

typedef unsigned long long fx_t;

// (t = v * 2^11, already scaled)
__device__ inline void fx_split_scaled(double t, fx_t& hi, fx_t& lo, int& bad)
{
    bad |= !(fabs(t) < kFxMax);
    const double th = t + kFxMagic;                 // round(t) in the low mantissa bits
    const double r = t - (th - kFxMagic);           // exact, |r| <= 1/2
    const double tl = __fma_rn(r, kFxLo, kFxMagic); // round(r * 2^40) likewise
    const long long m = __double_as_longlong(kFxMagic);
    hi = (fx_t)(__double_as_longlong(th) - m);
    lo = (fx_t)(__double_as_longlong(tl) - m);
}

__device__ inline void fx_split(double v, fx_t& hi, fx_t& lo, int& bad)
{
    fx_split_scaled(v * kFxHi, hi, lo, bad);   // the scaling is exact
}

// 64-bit integer atomic add into the reduced system, with the address space
// explicit (LDS, or global for the kLds = false fallback): on a generic
// pointer the compiler tests the address space at run time, and that test
// has tripped its instruction selection here
template <bool kLds>
__device__ inline void fx_atomic(fx_t* p, fx_t v)
{
    if constexpr (kLds) {
        atomicAdd(p, v);
    } else {
        auto* g = (__attribute__((address_space(1))) fx_t*)p;
        __hip_atomic_fetch_add(g, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
}

template <bool kLds>
__device__ inline void fx_add_scaled(fx_t* hi, fx_t* lo, int idx, double t, int& bad)
{
    fx_t h, l;
    fx_split_scaled(t, h, l, bad);
    fx_atomic<kLds>(hi + idx, h);
    fx_atomic<kLds>(lo + idx, l);
}

template <bool kLds>
__device__ inline void fx_add(fx_t* hi, fx_t* lo, int idx, double v, int& bad)
{
    fx_add_scaled<kLds>(hi, lo, idx, v * kFxHi, bad);   // the scaling is exact
}

__device__ inline void fx_set(fx_t* hi, fx_t* lo, int idx, double v, int& bad)
{
    fx_split(v, hi[idx], lo[idx], bad);
}

__device__ inline double fx_value(fx_t hi, fx_t lo)
{
    return (double)(long long)hi * kFxInvHi + (double)(long long)lo * kFxInvLo;
}

// Reduced-system storage of one problem (LDS or its global fallback), in
// doubles: limbs hi[M] | lo[M] | bhi[n] | blo[n] with M = n (n + 1) / 2;
// after accumulation hi[] holds the packed lower triangle as doubles and
// bhi[] the right-hand side.
__host__ __device__ constexpr long long lba_sys_doubles(long long n) { return n * (n + 1) + 2 * n; }

// One Levenberg trial: Schur complement, LLT, back-substitution, update.
// Returns false when the reduced system is not positive definite.
// per-thread edge table of the Schur pass (one allocation for both
// instantiations below)
__shared__ int2 s_edges[kLbaThreads][kSchurEdges];

// kLds: the reduced system lives in the dynamic LDS block (its accesses then
// compile to ds_* instructions instead of flat ones), else in P.S.
template <bool kLds>
__device__ bool trial_solve(LbaDev& P, double lambda, DScratch& sc)
{
    extern __shared__ __attribute__((aligned(16))) double s_S[];
    __shared__ int s_bad;
    LBA_T0();
    const int n = P.dim_p;
    const int M = n * (n + 1) / 2;
    fx_t* hi = reinterpret_cast<fx_t*>(kLds ? s_S : P.S);
    fx_t* lo = hi + M;
    fx_t* bhi = lo + M;
    fx_t* blo = bhi + n;
    double* S = reinterpret_cast<double*>(hi);     // packed lower triangle, after conversion
    double* bs = reinterpret_cast<double*>(bhi);
    int bad = 0;
    // the diagonal blocks Hpp + lambda I, zero elsewhere; bs <- bp
    for (int k = threadIdx.x; k < M; k += kLbaThreads) {
        hi[k] = 0;
        lo[k] = 0;
    }
    if (threadIdx.x == 0) s_bad = 0;
    __syncthreads();
    for (int item = threadIdx.x; item < P.nP * 21; item += kLbaThreads) {
        const int p = item / 21, u = item - p * 21;
        int r = 0;
        while (up6(r, 5) < u) r++;
        const int c = r + (u - up6(r, r));   // upper element (r, c), c >= r
        fx_set(hi, lo, pk(6 * p + c, 6 * p + r), P.hp[27 * p + u] + (r == c ? lambda : 0.0), bad);
    }
    for (int i = threadIdx.x; i < n; i += kLbaThreads) fx_set(bhi, blo, i, P.hp[27 * (i / 6) + 21 + (i % 6)], bad);
    __syncthreads();
    LBA_MARK(1);
    // Schur complement, point by point (one thread per point, its edges are
    // contiguous): D = Hll + lambda I, Dinv (Eigen 3x3 cofactor inverse),
    // db; then bs -= W_i db and S(i, j) -= (W_i Dinv) W_j^T for every pair of
    // the point's free-pose edges (upper blocks; diagonal blocks upper
    // triangle), as fixed-point limbs.  Points are taken in the order of
    // their edge counts (P.ce, point_order): the lanes of a wave run loops of
    // similar length and every thread gets a similar share; with
    // order-independent sums this changes no bit of the result.
    const int* order = reinterpret_cast<const int*>(P.ce);
#ifdef ORBX_DIAG_SCHUR
    double diag_sink = 0;
#endif
    for (int t = threadIdx.x; t < P.nL; t += kLbaThreads) {
        const int l = order[t];
        const double* h = P.hl + 9 * l;
        double m[9];
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int j = 0; j < 3; j++) m[i * 3 + j] = h[i <= j ? up3(i, j) : up3(j, i)] + (i == j ? lambda : 0.0);
        double d[12];
        {
            const double c00 = m[4] * m[8] - m[5] * m[7], c10 = m[7] * m[2] - m[8] * m[1], c20 = m[1] * m[5] - m[2] * m[4];
            const double c01 = m[5] * m[6] - m[3] * m[8], c11 = m[8] * m[0] - m[6] * m[2], c21 = m[2] * m[3] - m[0] * m[5];
            const double c02 = m[3] * m[7] - m[4] * m[6], c12 = m[6] * m[1] - m[7] * m[0], c22 = m[0] * m[4] - m[1] * m[3];
            const double det = c00 * m[0] + c10 * m[3] + c20 * m[6];
            const double inv = 1.0 / det;
            d[0] = c00 * inv; d[1] = c10 * inv; d[2] = c20 * inv;   // d[i*3+j] = cof(j, i) / det
            d[3] = c01 * inv; d[4] = c11 * inv; d[5] = c21 * inv;
            d[6] = c02 * inv; d[7] = c12 * inv; d[8] = c22 * inv;
        }
        const double* bl = h + 6;
#pragma unroll
        for (int i = 0; i < 3; i++) d[9 + i] = d[3 * i] * bl[0] + d[3 * i + 1] * bl[1] + d[3 * i + 2] * bl[2];
        double* dl = P.dl + 12 * l;
#pragma unroll
        for (int i = 0; i < 12; i++) dl[i] = d[i];
        const int q0 = P.lc_ptr[l], q1 = P.lc_ptr[l + 1], k = q1 - q0;
        // the point's free-pose edges (edge, pose block) in this thread's LDS
        // row; points with more than kSchurEdges such edges read the lists
        // from global memory
        int2* te = s_edges[threadIdx.x];
        const bool tab = k <= kSchurEdges;
        if (tab)
            for (int j = 0; j < k; j++) {
                const int a = P.lc_idx[q0 + j];
                te[j] = make_int2(a, P.e_ph[a]);
            }
        auto edge_at = [&](int j) { return tab ? te[j] : make_int2(P.lc_idx[q0 + j], P.e_ph[P.lc_idx[q0 + j]]); };
        // The point's edges in groups of kSchurGroup: the group's W_i Dinv
        // blocks stay in registers while every later edge's W_j is rebuilt
        // once for the whole group (k + ~k^2 / (2 G) rebuilds per point).
        constexpr int G = kSchurGroup;
        // S(i1, i2) -= (W_i Dinv) W_j^T over the 6x6 block (upper triangle of
        // a diagonal block), stored as the lower element (6 i2 + c, 6 i1 + r)
        // (w = -2^11 W_i Dinv: the element's contribution already negated and
        // in fixed-point scale; fused multiply-adds)
        auto pair_update = [&](const double (&w)[18], int i1, const double (&bj)[18], int i2) {
#pragma unroll
            for (int r = 0; r < 6; r++)
#pragma unroll
                for (int c = 0; c < 6; c++) {
                    if (i1 == i2 && c < r) continue;
                    const double t =
                        __fma_rn(w[r * 3 + 2], bj[c * 3 + 2], __fma_rn(w[r * 3 + 1], bj[c * 3 + 1], w[r * 3] * bj[c * 3]));
#if defined(ORBX_DIAG_SCHUR) && ORBX_DIAG_SCHUR == 1   // timing diagnostics only (wrong results)
                    diag_sink += t;
#elif defined(ORBX_DIAG_SCHUR) && ORBX_DIAG_SCHUR == 2
                    if (r == 0 && c == 0) diag_sink += t;
#else
                    fx_add_scaled<kLds>(hi, lo, pk(6 * i2 + c, 6 * i1 + r), t, bad);
#endif
                }
        };
        for (int g = 0; g < k; g += G) {
            double wd[G][18];   // W_i Dinv (6x3) of the group's edges
            int pi[G];
            double cur[18];
            // the group's own W blocks: W_i Dinv, bs, and the pairs among the
            // group's edges
#pragma unroll
            for (int u = 0; u < G; u++) {
                pi[u] = -1;
                if (g + u < k) {
                    const int2 ei = edge_at(g + u);
                    pi[u] = ei.y;
                    edge_hpl(P, ei.x, cur);
#pragma unroll
                    for (int r = 0; r < 6; r++) {
                        const double b0 = cur[3 * r], b1 = cur[3 * r + 1], b2 = cur[3 * r + 2];
#pragma unroll
                        for (int c = 0; c < 3; c++)
                            wd[u][r * 3 + c] = -kFxHi * __fma_rn(b2, d[6 + c], __fma_rn(b1, d[3 + c], b0 * d[c]));
                        fx_add<kLds>(bhi, blo, 6 * ei.y + r, -(b0 * d[9] + b1 * d[10] + b2 * d[11]), bad);
                    }
#pragma unroll
                    for (int v = 0; v <= u; v++) pair_update(wd[v], pi[v], cur, ei.y);
                }
            }
            // every later edge's W_j, rebuilt once for the whole group
            for (int qj = g + G; qj < k; qj++) {
                const int2 ej = edge_at(qj);
                edge_hpl(P, ej.x, cur);
#pragma unroll
                for (int u = 0; u < G; u++) pair_update(wd[u], pi[u], cur, ej.y);
            }
        }
    }
#ifdef ORBX_DIAG_SCHUR
    if (diag_sink == 1.2345) bad = 1;
#endif
    if (bad) s_bad = 1;
    __syncthreads();
    if (s_bad) return false;   // uniform
    // limbs -> doubles in place (element k's double overwrites its own hi)
    for (int k = threadIdx.x; k < M; k += kLbaThreads) S[k] = fx_value(hi[k], lo[k]);
    for (int i = threadIdx.x; i < n; i += kLbaThreads) bs[i] = fx_value(bhi[i], blo[i]);
    __syncthreads();
    LBA_MARK(2);
    // dense LLT on the packed lower triangle, right-looking in 6x6 blocks
    // (the pose blocks): per block column one wave factors the diagonal block
    // in registers (rows on lanes 0..5, shuffles), the panel rows solve
    // against it, the trailing triangle takes the rank-6 update; three
    // barriers per block column instead of three per column.
    const int nb = n / 6;
    for (int kb = 0; kb < nb; kb++) {
        const int k0 = 6 * kb;
        if (threadIdx.x < 64) {
            const int i = threadIdx.x;
            const bool row = i < 6;
            double a[6];
#pragma unroll
            for (int j = 0; j < 6; j++) a[j] = (row && j <= i) ? S[pk(k0 + i, k0 + j)] : 0.0;
            int fail = 0;
#pragma unroll
            for (int j = 0; j < 6; j++) {
                const double piv = __shfl(a[j], j, 64);   // a_jj after the previous columns
                fail |= !(piv > 0);
                const double ljj = sqrt(piv);
                if (i == j) a[j] = ljj;
                else if (row && i > j) a[j] = a[j] / ljj;
#pragma unroll
                for (int q = j + 1; q < 6; q++) {
                    const double lqj = __shfl(a[j], q, 64);
                    if (row && i >= q) a[q] -= a[j] * lqj;
                }
            }
            if (row)
#pragma unroll
                for (int j = 0; j < 6; j++)
                    if (j <= i) S[pk(k0 + i, k0 + j)] = a[j];
            if (i == 0) s_bad = fail;
        }
        __syncthreads();
        if (s_bad) return false;   // not positive definite (uniform)
        // panel: row r below the block solves x L_kk^T = A(r, block)
        for (int r = k0 + 6 + threadIdx.x; r < n; r += kLbaThreads) {
            double x[6];
            double* Sr = S + pk(r, k0);
#pragma unroll
            for (int j = 0; j < 6; j++) x[j] = Sr[j];
#pragma unroll
            for (int j = 0; j < 6; j++) {
                const double* Lj = S + pk(k0 + j, k0);
#pragma unroll
                for (int q = 0; q < j; q++) x[j] -= x[q] * Lj[q];
                x[j] = x[j] / Lj[j];
            }
#pragma unroll
            for (int j = 0; j < 6; j++) Sr[j] = x[j];
        }
        __syncthreads();
        // trailing triangle: S(i, j) -= L(i, block) . L(j, block)
        for (int i = k0 + 6 + (threadIdx.x >> 5); i < n; i += kLbaThreads / 32) {
            const double* Li = S + pk(i, k0);
            const double l0 = Li[0], l1 = Li[1], l2 = Li[2], l3 = Li[3], l4 = Li[4], l5 = Li[5];
            double* Si = S + pk(i, 0);
            for (int j = k0 + 6 + (threadIdx.x & 31); j <= i; j += 32) {
                const double* Lj = S + pk(j, k0);
                Si[j] -= ((((l0 * Lj[0] + l1 * Lj[1]) + l2 * Lj[2]) + l3 * Lj[3]) + l4 * Lj[4]) + l5 * Lj[5];
            }
        }
        __syncthreads();
    }
    LBA_MARK(3);
    // forward / backward substitution by one wave, in 6-row blocks: the
    // block's triangle on lanes 0..5 with shuffles, then the other rows
    // updated with the block's six values; one wave barrier per block
    double* xp = P.x;
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        for (int i = lane; i < n; i += 64) xp[i] = bs[i];
        auto wave_fence = [] {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        };
        wave_fence();
        for (int kb = 0; kb < nb; kb++) {   // L y = b
            const int k0 = 6 * kb;
            double yi = lane < 6 ? xp[k0 + lane] : 0.0;
#pragma unroll
            for (int j = 0; j < 6; j++) {
                const double yj = __shfl(yi, j, 64) / S[pk(k0 + j, k0 + j)];
                if (lane == j) yi = yj;
                else if (lane > j && lane < 6) yi -= S[pk(k0 + lane, k0 + j)] * yj;
            }
            if (lane < 6) xp[k0 + lane] = yi;
            double y[6];
#pragma unroll
            for (int p = 0; p < 6; p++) y[p] = __shfl(yi, p, 64);
            for (int i = k0 + 6 + lane; i < n; i += 64) {
                const double* Li = S + pk(i, k0);
                xp[i] -= ((((Li[0] * y[0] + Li[1] * y[1]) + Li[2] * y[2]) + Li[3] * y[3]) + Li[4] * y[4]) + Li[5] * y[5];
            }
            wave_fence();
        }
        for (int kb = nb - 1; kb >= 0; kb--) {   // L^T x = y
            const int k0 = 6 * kb;
            double xi = lane < 6 ? xp[k0 + lane] : 0.0;
#pragma unroll
            for (int j = 5; j >= 0; j--) {
                const double xj = __shfl(xi, j, 64) / S[pk(k0 + j, k0 + j)];
                if (lane == j) xi = xj;
                else if (lane < j) xi -= S[pk(k0 + j, k0 + lane)] * xj;
            }
            if (lane < 6) xp[k0 + lane] = xi;
            double x[6];
#pragma unroll
            for (int p = 0; p < 6; p++) x[p] = __shfl(xi, p, 64);
            for (int i = lane; i < k0; i += 64)
                xp[i] -= ((((S[pk(k0, i)] * x[0] + S[pk(k0 + 1, i)] * x[1]) + S[pk(k0 + 2, i)] * x[2]) +
                           S[pk(k0 + 3, i)] * x[3]) + S[pk(k0 + 4, i)] * x[4]) + S[pk(k0 + 5, i)] * x[5];
            wave_fence();
        }
    }
    __syncthreads();
    LBA_MARK(4);
    // landmarks: xl = Dinv (bl - sum_i B_i^T xp_i), the W_i rebuilt
    for (int t = threadIdx.x; t < P.nL; t += kLbaThreads) {
        const int l = order[t];
        const double* h = P.hl + 9 * l;
        double cl[3] = {h[6], h[7], h[8]};
        for (int q = P.lc_ptr[l]; q < P.lc_ptr[l + 1]; q++) {
            const int a = P.lc_idx[q];
            const int i1 = P.e_ph[a];
            double w[18];
            edge_hpl(P, a, w);
#pragma unroll
            for (int c = 0; c < 3; c++) {
                double acc = 0;
#pragma unroll
                for (int r = 0; r < 6; r++) acc += w[r * 3 + c] * (-xp[6 * i1 + r]);
                cl[c] += acc;
            }
        }
        const double* d = P.dl + 12 * l;
        for (int i = 0; i < 3; i++) P.x[n + 3 * l + i] = d[3 * i] * cl[0] + d[3 * i + 1] * cl[1] + d[3 * i + 2] * cl[2];
    }
    __syncthreads();
    LBA_MARK(5);
    return true;
}

// The points of a pass by decreasing count of free-pose edges (counting
// sort; the order within a count is arbitrary and does not matter) into
// P.ce, which is free scratch once the pass's structure is built.
__device__ void point_order(LbaDev& P)
{
    __shared__ int hist[64], off[64];
    int* order = reinterpret_cast<int*>(P.ce);
    for (int b = threadIdx.x; b < 64; b += kLbaThreads) hist[b] = 0;
    __syncthreads();
    auto bucket = [&](int l) { return 63 - min(P.lc_ptr[l + 1] - P.lc_ptr[l], 63); };
    for (int l = threadIdx.x; l < P.nL; l += kLbaThreads) atomicAdd(&hist[bucket(l)], 1);
    __syncthreads();
    if (threadIdx.x == 0) {
        int acc = 0;
        for (int b = 0; b < 64; b++) {
            off[b] = acc;
            acc += hist[b];
        }
    }
    __syncthreads();
    for (int l = threadIdx.x; l < P.nL; l += kLbaThreads) order[atomicAdd(&off[bucket(l)], 1)] = l;
    __syncthreads();
}

// OptimizationAlgorithmLevenberg::solve for one problem (levenberg.cpp:61-164)
__global__ __launch_bounds__(kLbaThreads) void k_lba_iteration(LbaDev* probs, int iteration, int lds_S_cap)
{
    __shared__ DScratch sc;
    LbaDev& P = probs[blockIdx.x];
    if (P.status != kRunning || P.abort) return;
    if (P.nE == 0 || P.nP + P.nL == 0) {
        if (threadIdx.x == 0) P.status = kTerminated;
        return;
    }
    const int n = P.dim_p;
    const bool in_lds = lba_sys_doubles(n) <= lds_S_cap;
    if (iteration == 0) point_order(P);
    LBA_T0();
    double currentChi = compute_errors(P, sc);
    const double iniChi = currentChi;
    if (iteration == 0 && threadIdx.x == 0) P.chi2_initial = currentChi;
    LBA_MARK(6);
    linearize(P);
    LBA_MARK(7);
    double lambda = P.lambda, ni = P.ni;
    if (iteration == 0) {
        double m = 0;
        for (int item = threadIdx.x; item < P.nP * 6; item += kLbaThreads)
            m = fmax(m, fabs(P.hp[27 * (item / 6) + up6(item % 6, item % 6)]));
        for (int item = threadIdx.x; item < P.nL * 3; item += kLbaThreads)
            m = fmax(m, fabs(P.hl[9 * (item / 3) + up3(item % 3, item % 3)]));
        m = block_max_d(m, sc);
        lambda = 1e-5 * m;
        ni = 2;
        if (threadIdx.x == 0) P.nBad = 0;
    }
    const int nx = n + 3 * P.nL;
    double rho = 0;
    int qmax = 0;
    do {
        // push
        for (int i = threadIdx.x; i < P.nposes_all * 7; i += kLbaThreads) P.pose_bk[i] = P.pose[i];
        for (int i = threadIdx.x; i < P.npoints_all * 3; i += kLbaThreads) P.point_bk[i] = P.point[i];
        __syncthreads();
        const bool ok2 = in_lds ? trial_solve<true>(P, lambda, sc) : trial_solve<false>(P, lambda, sc);
        if (ok2) {
            for (int p = threadIdx.x; p < P.nP; p += kLbaThreads) se3_oplus(P.pose + 7 * P.iv_pose[p], P.x + 6 * p);
            for (int item = threadIdx.x; item < P.nL * 3; item += kLbaThreads) {
                const int l = item / 3, i = item - l * 3;
                P.point[3 * P.iv_point[l] + i] += P.x[n + item];
            }
        } else {
            for (int i = threadIdx.x; i < nx; i += kLbaThreads) P.x[i] = 0.0;
            if (threadIdx.x == 0) P.not_posdef++;
        }
        __syncthreads();
        LBA_T0();
        double tempChi = compute_errors(P, sc);
        LBA_MARK(8);
        if (!ok2) tempChi = 1.79769313486231570815e+308;
        // computeScale: sum_j x_j (lambda x_j + b_j)
        double part = 0;
        for (int j = threadIdx.x; j < nx; j += kLbaThreads) {
            const double bj = j < n ? P.hp[27 * (j / 6) + 21 + (j % 6)] : P.hl[9 * ((j - n) / 3) + 6 + ((j - n) % 3)];
            part += P.x[j] * (lambda * P.x[j] + bj);
        }
        double scale = block_sum_d(part, sc);
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
            for (int i = threadIdx.x; i < P.nposes_all * 7; i += kLbaThreads) P.pose[i] = P.pose_bk[i];
            for (int i = threadIdx.x; i < P.npoints_all * 3; i += kLbaThreads) P.point[i] = P.point_bk[i];
        }
        __syncthreads();
        qmax++;
    } while (rho < 0 && qmax < 10 && !P.abort);
    if (threadIdx.x == 0) {
        P.lambda = lambda;
        P.ni = ni;
        P.trials += qmax;
        P.iterations++;
        P.last_chi = currentChi;
        int status = kRunning;
        if (qmax == 10 || rho == 0) {
            status = kTerminated;
        } else {
            if ((iniChi - currentChi) * 1e3 < iniChi) P.nBad++;
            else P.nBad = 0;
            if (P.nBad >= 3) status = kTerminated;
        }
        P.status = status;
    }
}

// Outlier passes of LocalBundleAdjustment (src/Optimizer.cc:452-470,
// :497-515).  The reference walks the edges in order; an edge's outcome
// depends only on earlier edges of the same map point (EraseObservation ->
// SetBadFlag), so each point's active edges are walked in edge order by one
// thread, points in parallel.
__global__ __launch_bounds__(256) void k_lba_outliers(LbaDev* probs, int* nobs_all, uint8_t* status_all,
                                                      uint8_t* bad_all, int pass, double thr, int* n_out,
                                                      const long long* offs)
{
    __shared__ int s_cnt;
    LbaDev& P = probs[blockIdx.x];
    const long long eo = offs[3 * blockIdx.x], po = offs[3 * blockIdx.x + 1];
    int* nobs = nobs_all + po;
    uint8_t* st = status_all + eo;
    uint8_t* bad = bad_all + po;
    if (threadIdx.x == 0) s_cnt = 0;
    __syncthreads();
    int cnt = 0;
    for (int l = threadIdx.x; l < P.nL; l += blockDim.x) {
        const int p = P.iv_point[l];
        for (int q = P.le_ptr[l]; q < P.le_ptr[l + 1]; q++) {
            if (bad[p]) break;
            const int a = P.le_idx[q];
            const int e = P.e_orig[a];
            const double s = P.e_isig[a];
            const double e0 = P.err[2 * e], e1 = P.err[2 * e + 1];
            const double chi2 = e0 * (s * e0) + e1 * (s * e1);
            double pc[3];
            se3_map(P.pose + 7 * P.e_pose[a], P.point + 3 * p, pc);
            if (chi2 > thr || !(pc[2] > 0.0)) {
                if (--nobs[p] <= 2) bad[p] = 1;
                st[e] = (uint8_t)pass;
                cnt++;
            }
        }
    }
    atomicAdd(&s_cnt, cnt);
    __syncthreads();
    if (threadIdx.x == 0) n_out[blockIdx.x] = s_cnt;
}

// Structures of the first optimize() built on the device from the caller's
// arrays: g2o's initializeOptimization + BlockSolver::buildStructure
// (sparse_optimizer.cpp:166-267, block_solver.hpp:143-295) on the subset
// LocalBundleAdjustment uses.  Every edge is active; the free poses with an
// edge and the points with an edge are ordered by g2o vertex id (ties by
// index: a stable sort), which fixes the Hessian block order; per free pose
// and per point the active edges in edge order (CSR); per point its edges to
// free poses in pose-block order (the Schur columns).  Ranks come from a
// scan when the ids are already increasing (the caller's usual order) and
// from pairwise counts otherwise.  One workgroup per problem; the Hpl
// scratch (dead until linearisation) holds the index maps.
__device__ inline void lba_rank(const long long* id, const int* act, int n, int* rank, int* count,
                                BlockScratchN<kLbaWaves>& bs)
{
    const int tid = threadIdx.x;
    int unsorted = 0;
    for (int i = tid; i + 1 < n; i += kLbaThreads) unsorted |= !(id[i] < id[i + 1]);
    unsorted = block_sum<kLbaWaves>(unsorted, bs, 0);
    __syncthreads();
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
    __syncthreads();
    *count = total;
}

__global__ __launch_bounds__(kLbaThreads) void k_lba_build(LbaDev* probs)
{
    __shared__ BlockScratchN<kLbaWaves> bs;
    LbaDev& A = probs[blockIdx.x];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int NP = A.nposes_all, NL = A.npoints_all, E = A.nedges_all;
    int* pflag = reinterpret_cast<int*>(A.ce);   // [NP] pose has an edge and is free
    int* lflag = pflag + NP;                     // [NL] point has an edge
    int* ph = lflag + NL;                        // [NP] pose block or -1
    int* lh = ph + NP;                           // [NL] point block or -1
    int* cur = lh + NL;                          // [NL] list cursors
    for (int i = tid; i < NP; i += kLbaThreads) pflag[i] = 0;
    for (int i = tid; i < NL; i += kLbaThreads) lflag[i] = 0;
    __syncthreads();
    for (int a = tid; a < E; a += kLbaThreads) {
        const int p = A.r_edge_pose[a];
        if (!A.r_pose_fixed[p]) pflag[p] = 1;
        lflag[A.r_edge_point[a]] = 1;
    }
    __syncthreads();
    int nP, nL;
    lba_rank(A.r_pose_id, pflag, NP, ph, &nP, bs);
    lba_rank(A.r_point_id, lflag, NL, lh, &nL, bs);
    int* iv_pose = const_cast<int*>(A.iv_pose);
    int* iv_point = const_cast<int*>(A.iv_point);
    for (int i = tid; i < NP; i += kLbaThreads)
        if (ph[i] >= 0) iv_pose[ph[i]] = i;
    for (int i = tid; i < NL; i += kLbaThreads)
        if (lh[i] >= 0) iv_point[lh[i]] = i;
    // edge records (every edge active, original order)
    int* pe_ptr = const_cast<int*>(A.pe_ptr);
    int* le_ptr = const_cast<int*>(A.le_ptr);
    int* lc_ptr = const_cast<int*>(A.lc_ptr);
    for (int i = tid; i <= nP; i += kLbaThreads) pe_ptr[i] = 0;
    for (int i = tid; i <= nL; i += kLbaThreads) {
        le_ptr[i] = 0;
        lc_ptr[i] = 0;
    }
    __syncthreads();
    for (int a = tid; a < E; a += kLbaThreads) {
        const int p = A.r_edge_pose[a], l = A.r_edge_point[a];
        const int eph = ph[p], elh = lh[l];
        const_cast<int*>(A.e_orig)[a] = a;
        const_cast<int*>(A.e_pose)[a] = p;
        const_cast<int*>(A.e_point)[a] = l;
        const_cast<int*>(A.e_ph)[a] = eph;
        const_cast<int*>(A.e_lh)[a] = elh;
        const_cast<double*>(A.e_obs)[2 * a] = A.r_edge_obs[2 * a];
        const_cast<double*>(A.e_obs)[2 * a + 1] = A.r_edge_obs[2 * a + 1];
        const_cast<double*>(A.e_isig)[a] = A.r_edge_isig[a];
        if (eph >= 0) {
            atomicAdd(&pe_ptr[eph + 1], 1);
            atomicAdd(&lc_ptr[elh + 1], 1);
        }
        atomicAdd(&le_ptr[elh + 1], 1);
    }
    __syncthreads();
    // counts -> offsets (block scans)
    auto offsets = [&](int* ptr, int n) {
        int base = 0;
        for (int c = 0; c < n; c += kLbaThreads) {
            const int i = c + tid;
            const int v = i < n ? ptr[i + 1] : 0;
            int tot;
            const int inc = block_exclusive_scan<kLbaWaves>(v, &tot, bs, (c / kLbaThreads) & 1) + v;
            __syncthreads();
            if (i < n) ptr[i + 1] = base + inc;
            base += tot;
            __syncthreads();
        }
    };
    offsets(pe_ptr, nP);
    offsets(le_ptr, nL);
    offsets(lc_ptr, nL);
    __syncthreads();
    // per free pose, its edges in edge order (wave per pose, ballot compaction)
    int* pe_idx = const_cast<int*>(A.pe_idx);
    for (int p1 = wv; p1 < nP; p1 += kLbaWaves) {
        const int pose = iv_pose[p1];
        int w = pe_ptr[p1];
        for (int a0 = 0; a0 < E; a0 += 64) {
            const int a = a0 + lane;
            const bool mine = a < E && A.r_edge_pose[a] == pose;
            const unsigned long long bal = __ballot(mine);
            if (mine) pe_idx[w + __popcll(bal & (lane ? (~0ull >> (64 - lane)) : 0ull))] = a;
            w += __popcll(bal);
        }
    }
    // per point: its edges appended, then put in edge order (few per point);
    // its Schur columns: the edges to free poses, in pose-block order
    int* le_idx = const_cast<int*>(A.le_idx);
    int* lc_idx = const_cast<int*>(A.lc_idx);
    for (int l1 = tid; l1 < nL; l1 += kLbaThreads) cur[l1] = le_ptr[l1];
    __syncthreads();
    for (int a = tid; a < E; a += kLbaThreads) le_idx[atomicAdd(&cur[lh[A.r_edge_point[a]]], 1)] = a;
    __syncthreads();
    for (int l1 = tid; l1 < nL; l1 += kLbaThreads) {
        const int q0 = le_ptr[l1], q1 = le_ptr[l1 + 1];
        for (int i = q0 + 1; i < q1; i++) {   // insertion sort by edge index
            const int x = le_idx[i];
            int j = i - 1;
            while (j >= q0 && le_idx[j] > x) {
                le_idx[j + 1] = le_idx[j];
                j--;
            }
            le_idx[j + 1] = x;
        }
        int w = lc_ptr[l1];
        const int c0 = w;
        for (int q = q0; q < q1; q++) {
            const int a = le_idx[q];
            const int eph = ph[A.r_edge_pose[a]];
            if (eph < 0) continue;
            int j = w - 1;   // stable insertion by pose block
            while (j >= c0 && ph[A.r_edge_pose[lc_idx[j]]] > eph) {
                lc_idx[j + 1] = lc_idx[j];
                j--;
            }
            lc_idx[j + 1] = a;
            w++;
        }
    }
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
// restated as order-preserving filters of the first pass's sorted lists
// (active edges keep their original order, free poses / points their id
// order, every CSR list its edge or pose order), so the result equals the
// first-pass build (k_lba_build) on the reduced edge set.  One workgroup per problem;
// the first pass's Hpl and Hll scratch (dead until the second pass
// linearises) hold the index maps.  B's pointer fields are set by the host.
__global__ __launch_bounds__(kLbaThreads) void k_lba_rebuild(const LbaDev* d0s, LbaDev* d1s, const uint8_t* status_all,
                                                             const long long* offs)
{
    __shared__ BlockScratchN<kLbaWaves> bs;
    const LbaDev& A = d0s[blockIdx.x];
    LbaDev& B = d1s[blockIdx.x];
    const uint8_t* st = status_all + offs[3 * blockIdx.x];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int nE0 = A.nE, nP0 = A.nP, nL0 = A.nL;
    int* na = reinterpret_cast<int*>(A.ce);     // [nE0] new edge index or -1
    int* ph1 = reinterpret_cast<int*>(A.hp);    // [nP0] new pose hessian index or -1, then counts
    int* cp = ph1 + nP0;                        // [nP0] kept edges per pose
    int* lh1 = reinterpret_cast<int*>(A.hl);    // [nL0] new point index or -1
    int* cl = lh1 + nL0;                        // [nL0] kept edges per point
    int* cc = cl + nL0;                         // [nL0] kept Schur-column edges per point
    auto kept = [&](int a0) { return st[A.e_orig[a0]] == 0; };
    // 1. edges: new index by a block scan over the kept flags (edge order)
    int base = 0;
    for (int c = 0; c < nE0; c += kLbaThreads) {
        const int a0 = c + tid;
        const int k = a0 < nE0 && kept(a0) ? 1 : 0;
        int tot;
        const int off = block_exclusive_scan<kLbaWaves>(k, &tot, bs, (c / kLbaThreads) & 1);
        if (a0 < nE0) na[a0] = k ? base + off : -1;
        base += tot;
    }
    const int nE1 = base;
    __syncthreads();
    // 2. kept edges per pose (wave per pose) and per point (thread per point)
    for (int p = wv; p < nP0; p += kLbaWaves) {
        int cnt = 0;
        for (int q = A.pe_ptr[p] + lane; q < A.pe_ptr[p + 1]; q += 64) cnt += na[A.pe_idx[q]] >= 0;
        cnt = wave_sum(cnt);
        if (lane == 0) cp[p] = cnt;
    }
    for (int l = tid; l < nL0; l += kLbaThreads) {
        int c1 = 0, c2 = 0;
        for (int q = A.le_ptr[l]; q < A.le_ptr[l + 1]; q++) c1 += na[A.le_idx[q]] >= 0;
        for (int q = A.lc_ptr[l]; q < A.lc_ptr[l + 1]; q++) c2 += na[A.lc_idx[q]] >= 0;
        cl[l] = c1;
        cc[l] = c2;
    }
    __syncthreads();
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
        __syncthreads();   // bs reads done before the next round's scans
    }
    int nL1 = 0, le_base = 0, lc_base = 0;
    for (int c = 0; c < nL0; c += kLbaThreads) {
        const int l = c + tid;
        const int act = l < nL0 && cl[l] > 0 ? 1 : 0;
        int tot, tot2, tot3;
        const int idx = block_exclusive_scan<kLbaWaves>(act, &tot, bs, 0);
        const int eo = block_exclusive_scan<kLbaWaves>(act ? cl[l] : 0, &tot2, bs, 1);
        const int co = block_exclusive_scan<kLbaWaves>(act ? cc[l] : 0, &tot3, bs, 0);
        if (l < nL0) {
            const int l1 = act ? nL1 + idx : -1;
            if (act) {
                const_cast<int*>(B.iv_point)[l1] = A.iv_point[l];
                const_cast<int*>(B.le_ptr)[l1] = le_base + eo;
                const_cast<int*>(B.lc_ptr)[l1] = lc_base + co;
            }
            lh1[l] = l1;
        }
        nL1 += tot;
        le_base += tot2;
        lc_base += tot3;
        __syncthreads();   // bs reads done before the next round's scans
    }
    if (tid == 0) {
        const_cast<int*>(B.pe_ptr)[nP1] = pe_base;
        const_cast<int*>(B.le_ptr)[nL1] = le_base;
        const_cast<int*>(B.lc_ptr)[nL1] = lc_base;
    }
    __syncthreads();
    // 4. the kept edges' records, remapped
    for (int a0 = tid; a0 < nE0; a0 += kLbaThreads) {
        const int a1 = na[a0];
        if (a1 < 0) continue;
        const int ph = A.e_ph[a0];
        const_cast<int*>(B.e_orig)[a1] = A.e_orig[a0];
        const_cast<int*>(B.e_pose)[a1] = A.e_pose[a0];
        const_cast<int*>(B.e_point)[a1] = A.e_point[a0];
        const_cast<int*>(B.e_ph)[a1] = ph >= 0 ? ph1[ph] : -1;
        const_cast<int*>(B.e_lh)[a1] = lh1[A.e_lh[a0]];
        const_cast<double*>(B.e_obs)[2 * a1] = A.e_obs[2 * a0];
        const_cast<double*>(B.e_obs)[2 * a1 + 1] = A.e_obs[2 * a0 + 1];
        const_cast<double*>(B.e_isig)[a1] = A.e_isig[a0];
    }
    // 5. CSR lists: filters of the first pass's lists (wave per pose, with a
    //    ballot compaction; thread per point)
    for (int p = wv; p < nP0; p += kLbaWaves) {
        const int p1 = ph1[p];
        if (p1 < 0) continue;
        int w = B.pe_ptr[p1];
        for (int q0 = A.pe_ptr[p]; q0 < A.pe_ptr[p + 1]; q0 += 64) {
            const int q = q0 + lane;
            const int a1 = q < A.pe_ptr[p + 1] ? na[A.pe_idx[q]] : -1;
            const unsigned long long bal = __ballot(a1 >= 0);
            if (a1 >= 0) {
                const unsigned long long lt = lane ? (~0ull >> (64 - lane)) : 0ull;
                const_cast<int*>(B.pe_idx)[w + __popcll(bal & lt)] = a1;
            }
            w += __popcll(bal);
        }
    }
    for (int l = tid; l < nL0; l += kLbaThreads) {
        const int l1 = lh1[l];
        if (l1 < 0) continue;
        int w = B.le_ptr[l1];
        for (int q = A.le_ptr[l]; q < A.le_ptr[l + 1]; q++) {
            const int a1 = na[A.le_idx[q]];
            if (a1 >= 0) const_cast<int*>(B.le_idx)[w++] = a1;
        }
        w = B.lc_ptr[l1];
        for (int q = A.lc_ptr[l]; q < A.lc_ptr[l + 1]; q++) {
            const int a1 = na[A.lc_idx[q]];
            if (a1 >= 0) const_cast<int*>(B.lc_idx)[w++] = a1;
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

// doubles of LDS for the reduced system (160 KB less the Schur edge table)
constexpr int kLdsSCap = (160 * 1024 - kLbaThreads * kSchurEdges * 8 - 1024) / 8;

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
    size_t pose, point, posebk, pointbk, cam, err;
};
struct LbaPlan {
    int P = 0;
    uint8_t* d = nullptr;   // device base the LbaDev pointers were packed against
    std::vector<LbaPlay> pl;
    std::vector<long long> offs;   // per problem: first edge, first point (global flag arrays)
    std::vector<int> n_poses, n_points, n_edges;
    long long eacc = 0, pacc = 0;
    size_t result_bytes = 0, base_bytes = 0, o_all_nobs = 0, o_all_st = 0, o_all_bad = 0, o_offs = 0, o_nout = 0;
    size_t o_devs = 0, o_devs1 = 0, staged_end = 0, o_err = 0, err_bytes = 0, dev_end = 0, max_n2 = 0;
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
    }
    std::vector<uint8_t> bad_edge(P, 0);
    host_parallel(P, [&](int i) {
        const orbx_ba_problem& p = probs[i];
        for (int e = 0; e < p.n_edges; e++)
            if (p.edge_point[e] < 0 || p.edge_point[e] >= p.n_points || p.edge_pose[e] < 0 || p.edge_pose[e] >= p.n_poses)
                bad_edge[i] = 1;
    });
    for (int i = 0; i < P; i++)
        if (bad_edge[i]) return ORBX_ERR_ARG;
    L = LbaPlan{};
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
    L.o_nout = at;     at += align256(8 * (size_t)P);   // outliers per problem, per pass
    L.base_bytes = at;
    // Both optimize() calls' structures are built on the device: the first
    // from the caller's arrays (k_lba_build), the second from the first's
    // after the first outlier pass (k_lba_rebuild), so the host only stages
    // the problems, and both passes run back to back after one upload.
    constexpr int kRaw = 7, kArr = 15;
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
    auto arr_bytes = [&](int i, size_t (&bytes)[kArr]) {
        const orbx_ba_problem& p = probs[i];
        const size_t E = p.n_edges, NP = nfree[i], NL = p.n_points;
        const size_t b[kArr] = {E * 4,  E * 4,        E * 4,  E * 4,        E * 4,  E * 16,       E * 8, NP * 4,
                                NL * 4, (NP + 1) * 4, E * 4, (NL + 1) * 4, E * 4, (NL + 1) * 4, E * 4};
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
    // device-only: the LM backups and the per-edge errors (zeroed on the device)
    for (int i = 0; i < P; i++) {
        const orbx_ba_problem& p = probs[i];
        pl[i].posebk = end;  end += align256(7 * (size_t)p.n_poses * 8);
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
    // device-only scratch, sized by the free poses, every point and edge
    // (the Hpl scratch also holds k_lba_build's and k_lba_rebuild's maps)
    std::vector<size_t> sc(8 * (size_t)P);
    for (int i = 0; i < P; i++) {
        const orbx_ba_problem& p = probs[i];
        const size_t nE = p.n_edges, nL = p.n_points, n = 6 * (size_t)nfree[i];
        const size_t sys = (size_t)lba_sys_doubles((long long)n);
        L.max_n2 = std::max(L.max_n2, sys);
        // ce: index maps of k_lba_build / k_lba_rebuild only (no Hpl blocks
        // are stored); S: the reduced system when it does not fit LDS
        const size_t bytes[8] = {std::max(nE * 4, (2 * (size_t)p.n_poses + 3 * nL) * 4), 27 * (size_t)nfree[i] * 8,
                                 9 * nL * 8, 12 * nL * 8, sys > (size_t)kLdsSCap ? sys * 8 : 8, (n + 3 * nL) * 8,
                                 n * 8 + 8, nE * 8};
        for (int k = 0; k < 8; k++) {
            sc[8 * i + k] = end;
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
            D.pose_bk = reinterpret_cast<double*>(d + pl[i].posebk);
            D.point_bk = reinterpret_cast<double*>(d + pl[i].pointbk);
            D.cam = reinterpret_cast<const double*>(d + pl[i].cam);
            D.err = reinterpret_cast<double*>(d + pl[i].err);
            D.e_orig = reinterpret_cast<const int*>(d + o[0]);
            D.e_pose = reinterpret_cast<const int*>(d + o[1]);
            D.e_point = reinterpret_cast<const int*>(d + o[2]);
            D.e_ph = reinterpret_cast<const int*>(d + o[3]);
            D.e_lh = reinterpret_cast<const int*>(d + o[4]);
            D.e_obs = reinterpret_cast<const double*>(d + o[5]);
            D.e_isig = reinterpret_cast<const double*>(d + o[6]);
            D.iv_pose = reinterpret_cast<const int*>(d + o[7]);
            D.iv_point = reinterpret_cast<const int*>(d + o[8]);
            D.pe_ptr = reinterpret_cast<const int*>(d + o[9]);
            D.pe_idx = reinterpret_cast<const int*>(d + o[10]);
            D.le_ptr = reinterpret_cast<const int*>(d + o[11]);
            D.le_idx = reinterpret_cast<const int*>(d + o[12]);
            D.lc_ptr = reinterpret_cast<const int*>(d + o[13]);
            D.lc_idx = reinterpret_cast<const int*>(d + o[14]);
            const size_t* c = &sc[8 * i];
            D.ce = reinterpret_cast<double*>(d + c[0]);
            D.hp = reinterpret_cast<double*>(d + c[1]);
            D.hl = reinterpret_cast<double*>(d + c[2]);
            D.dl = reinterpret_cast<double*>(d + c[3]);
            D.S = reinterpret_cast<double*>(d + c[4]);
            D.x = reinterpret_cast<double*>(d + c[5]);
            D.bs = reinterpret_cast<double*>(d + c[6]);
            D.ew = reinterpret_cast<double*>(d + c[7]);
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
    std::memcpy(hb + L.o_devs, devs.data(), sizeof(LbaDev) * P);
    std::memcpy(hb + L.o_devs1, devs1.data(), sizeof(LbaDev) * P);
    ORBX_HIP_CHECK(hipMemcpyAsync(d, hb, L.staged_end, hipMemcpyHostToDevice, ctx->stream));
    return ORBX_OK;
}

// Queues both optimize() passes of a staged batch on the context stream:
// k_lba_build, iterations, outliers, k_lba_rebuild, iterations, outliers.
// With abort flags (per problem, entries may be null) the host polls them
// (and the problems' status) between iterations, which synchronises; an
// aborted problem's later iterations return at once (g2o's force-stop flag,
// sparse_optimizer.cpp:394-396); without flags nothing waits.
static int lba_launch(orbx_ctx* ctx, const LbaPlan& L, int iters0, int iters1,
                      const volatile uint8_t* const* aborts)
{
    const int P = L.P;
    uint8_t* d = L.d;
    ORBX_HIP_CHECK(hipMemsetAsync(d + L.o_err, 0, L.err_bytes, ctx->stream));
    timer_begin(ctx, "lba_build");
    hipLaunchKernelGGL(k_lba_build, dim3(P), dim3(kLbaThreads), 0, ctx->stream, reinterpret_cast<LbaDev*>(d + L.o_devs));
    timer_end(ctx, "lba_build");
    ORBX_HIP_CHECK(hipGetLastError());
    const size_t lds = std::min(L.max_n2, (size_t)kLdsSCap) * 8;   // the second pass's systems are no larger
    const int lds_cap = (int)(lds / 8);
    bool polled = false;
    for (int i = 0; aborts && i < P; i++) polled |= aborts[i] != nullptr;
    std::vector<LbaDev> hv(polled ? P : 0);
    std::vector<uint8_t> stopped(P, 0);   // abort written to the device
    for (int pass = 0; pass < 2; pass++) {
        LbaDev* dd = reinterpret_cast<LbaDev*>(d + (pass == 0 ? L.o_devs : L.o_devs1));
        if (pass == 1) {
            timer_begin(ctx, "lba_rebuild");
            hipLaunchKernelGGL(k_lba_rebuild, dim3(P), dim3(kLbaThreads), 0, ctx->stream,
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
            hipLaunchKernelGGL(k_lba_iteration, dim3(P), dim3(kLbaThreads), lds, ctx->stream, dd, it, lds_cap);
            timer_end(ctx, "lba_iter");
            ORBX_HIP_CHECK(hipGetLastError());
            // With an abort flag the host polls it between iterations (where
            // g2o polls its force-stop flag), which needs the device state;
            // without one, iterations are queued back to back and a
            // terminated problem's later launches return immediately.
            if (polled) {
                ORBX_HIP_CHECK(hipMemcpyAsync(hv.data(), dd, sizeof(LbaDev) * P, hipMemcpyDeviceToHost, ctx->stream));
                ORBX_HIP_CHECK(hipStreamSynchronize(ctx->stream));
                bool running = false;
                for (int i = 0; i < P; i++) running |= hv[i].status == kRunning && !hv[i].abort;
                if (!running) break;
            }
        }
        timer_begin(ctx, "lba_outliers");
        hipLaunchKernelGGL(k_lba_outliers, dim3(P), dim3(256), 0, ctx->stream, dd,
                           reinterpret_cast<int*>(d + L.o_all_nobs), d + L.o_all_st, d + L.o_all_bad, pass + 1,
                           L.chi2_threshold, reinterpret_cast<int*>(d + L.o_nout) + pass * P,
                           reinterpret_cast<const long long*>(d + L.o_offs));
        timer_end(ctx, "lba_outliers");
        ORBX_HIP_CHECK(hipGetLastError());
    }
    return ORBX_OK;
}

// Reads a solved batch back (synchronising the context stream): poses and
// points into the problems' arrays, edge / point flags, statistics.
static int lba_readback(orbx_ctx* ctx, const LbaPlan& L, orbx_ba_problem* probs, uint8_t* const* edge_status,
                        uint8_t* const* point_bad, orbx_ba_stats* stats)
{
    const int P = L.P;
    uint8_t* d = L.d;
    int r;
    if ((r = ensure_pinned(ctx, std::max(L.result_bytes, L.o_all_bad + (size_t)L.pacc))) != ORBX_OK) return r;
    uint8_t* hb = static_cast<uint8_t*>(ctx->host_pinned);
    std::vector<LbaDev> devs(P), devs1(P);
    std::vector<uint8_t> all_st((size_t)L.eacc, 0);
    std::vector<int> nout(2 * (size_t)P);
    ORBX_HIP_CHECK(hipMemcpyAsync(devs.data(), d + L.o_devs, sizeof(LbaDev) * P, hipMemcpyDeviceToHost, ctx->stream));
    ORBX_HIP_CHECK(hipMemcpyAsync(devs1.data(), d + L.o_devs1, sizeof(LbaDev) * P, hipMemcpyDeviceToHost, ctx->stream));
    if (L.eacc)
        ORBX_HIP_CHECK(hipMemcpyAsync(all_st.data(), d + L.o_all_st, all_st.size(), hipMemcpyDeviceToHost, ctx->stream));
    ORBX_HIP_CHECK(hipMemcpyAsync(nout.data(), d + L.o_nout, 8 * (size_t)P, hipMemcpyDeviceToHost, ctx->stream));
    // results: poses and points in one copy, scattered on host threads below
    ORBX_HIP_CHECK(hipMemcpyAsync(hb, d, L.result_bytes, hipMemcpyDeviceToHost, ctx->stream));
    if (L.pacc)
        ORBX_HIP_CHECK(hipMemcpyAsync(hb + L.o_all_bad, d + L.o_all_bad, (size_t)L.pacc, hipMemcpyDeviceToHost,
                                      ctx->stream));
    ORBX_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    if (stats)
        for (int pass = 0; pass < 2; pass++) {
            const std::vector<LbaDev>& hv = pass == 0 ? devs : devs1;
            for (int i = 0; i < P; i++) {
                stats[i].iterations[pass] = hv[i].iterations;
                stats[i].levenberg_trials[pass] = hv[i].trials;
                stats[i].chi2_initial[pass] = hv[i].chi2_initial;
                stats[i].chi2_final[pass] = hv[i].last_chi;
                stats[i].n_outliers[pass] = nout[pass * (size_t)P + i];
                stats[i].not_posdef += hv[i].not_posdef;
            }
        }
    host_parallel(P, [&](int i) {
        orbx_ba_problem& p = probs[i];
        const double* pose = reinterpret_cast<const double*>(hb + L.pl[i].pose);
        for (int k = 0; k < p.n_poses; k++) {
            for (int j = 0; j < 4; j++) p.pose_q[4 * k + j] = pose[7 * k + j];
            for (int j = 0; j < 3; j++) p.pose_t[3 * k + j] = pose[7 * k + 4 + j];
        }
        std::memcpy(p.points, hb + L.pl[i].point, 3 * (size_t)p.n_points * 8);
        if (edge_status && edge_status[i]) std::memcpy(edge_status[i], all_st.data() + L.offs[3 * i], p.n_edges);
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
    return lba_readback(ctx, L, probs, edge_status, point_bad, stats);
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

}  // namespace orbx

extern "C" {

#ifdef ORBX_LBA_PROFILE
int orbx_debug_lba_prof(unsigned long long* out)
{
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(orbx::g_lba_prof), sizeof(unsigned long long) * 16) == hipSuccess ? 0 : -2;
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
    return orbx::lba_readback(ctx, L, problems, edge_status, point_bad, stats);
}

}  // extern "C"
