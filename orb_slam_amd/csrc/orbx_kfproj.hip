// Keyframe projection searches on MI355X: the state-free part of
// ORBmatcher::Fuse (both overloads, src/ORBmatcher.cc:1016-1265),
// SearchBySim3 (:1267-1505) and MapPoint::ComputeDistinctiveDescriptors
// (src/MapPoint.cc:185-250).
//
// Projection: one wavefront per map point, four per 256-thread workgroup.
// The keyframe's keypoint table (position, grid cell, octave) is staged in
// LDS once per workgroup; each wavefront computes its point's projection
// and gates redundantly on every lane (uniform), then the lanes stride the
// keyframe's keypoints with the GetFeaturesInArea cell/box test and the
// level window, and one 64-bit min reduction over (distance, cell, index)
// gives the reference's first strict minimum in GetFeaturesInArea order.
// cv::Mat arithmetic is restated as in oracle/ref_proj.cpp (float products
// summed left to right, scalar scaling by a double factor, cv::norm and
// Mat::dot accumulated in double).
//
// Distinctive descriptors: one wavefront per map point; lane i takes
// descriptor i and finds the median of its distance row by a binary search
// on the value (9 counting passes over the row), then a (median, i) min
// reduction picks the first least median.
#include <algorithm>
#include <climits>
#include <cmath>
#include <vector>

#include "orbx_device.h"
#include "orbx_internal.h"
#include "orbx_match_common.h"

namespace orbx {

struct KfProjArgs {
    FrameDev K;                 // searched keyframe
    float scales[kMaxLevels];
    int nlevels;
    float cam[4];
    float Ra[9], ta[3];         // p = Ra X + ta
    float Rb[9], tb[3];         // then p = Rb p + tb (two_stage)
    float Ow[3];
    int two_stage;
    int mode;                   // 0 Fuse (1/z float), 1 Fuse Scw (1.0/z double), 2 SearchBySim3
    float th;
    int nq;
    const float* pos;
    const float* normal;
    const float* dmin;
    const float* dmax;
    const uint8_t* qdesc;
    const uint8_t* qvalid;      // may be null
    int32_t* best_idx;
    int32_t* best_dist;
};

__device__ inline void xform3(const float* R, const float* t, const float* X, float* o)
{
#pragma unroll
    for (int r = 0; r < 3; r++)
        o[r] = __fadd_rn(__fadd_rn(__fadd_rn(__fmul_rn(R[3 * r], X[0]), __fmul_rn(R[3 * r + 1], X[1])),
                                   __fmul_rn(R[3 * r + 2], X[2])),
                         t[r]);
}

__device__ inline float norm3_cv(const float* v)
{
    double s = 0;
#pragma unroll
    for (int i = 0; i < 3; i++) s += (double)v[i] * (double)v[i];
    return (float)sqrt(s);
}

__device__ inline double dot3_cv(const float* a, const float* b)
{
    double s = 0;
#pragma unroll
    for (int i = 0; i < 3; i++) s += (double)a[i] * (double)b[i];
    return s;
}

__device__ inline void kf_project_block(const KfProjArgs& a, uint8_t* smem, int mblock)
{
    float* tx = reinterpret_cast<float*>(smem);
    float* ty = tx + a.K.n;
    int* tco = reinterpret_cast<int*>(ty + a.K.n);   // cell | octave << 16
    for (int i = threadIdx.x; i < a.K.n; i += kBlock) {
        const orbx_keypoint k = a.K.kps[i];
        tx[i] = k.x;
        ty[i] = k.y;
        const int cell = grid_cell(a.K, k.x, k.y);
        tco[i] = (cell & 0xFFFF) | (k.octave << 16);
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int m = mblock * (kBlock / 64) + (threadIdx.x >> 6);
    if (m >= a.nq) return;
    int best_idx = -1, best_dist = INT_MAX;
    do {
        if (a.qvalid && !a.qvalid[m]) break;
        const float Xw[3] = {a.pos[3 * m], a.pos[3 * m + 1], a.pos[3 * m + 2]};
        float pc[3];
        xform3(a.Ra, a.ta, Xw, pc);
        if (a.two_stage) {
            const float p1[3] = {pc[0], pc[1], pc[2]};
            xform3(a.Rb, a.tb, p1, pc);
        }
        if (pc[2] < 0.0f) break;
        const float invz = a.mode == 0 ? __fdiv_rn(1.0f, pc[2]) : (float)(1.0 / (double)pc[2]);
        const float x = __fmul_rn(pc[0], invz), y = __fmul_rn(pc[1], invz);
        const float u = __fadd_rn(__fmul_rn(a.cam[0], x), a.cam[2]);
        const float v = __fadd_rn(__fmul_rn(a.cam[1], y), a.cam[3]);
        if (!(u >= a.K.min_x && u < a.K.max_x && v >= a.K.min_y && v < a.K.max_y)) break;   // IsInImage
        const float maxDistance = a.dmax[m], minDistance = a.dmin[m];
        float dist3D;
        if (a.mode == 2) {
            dist3D = norm3_cv(pc);   // SearchBySim3: norm of the camera point
        } else {
            const float PO[3] = {__fsub_rn(Xw[0], a.Ow[0]), __fsub_rn(Xw[1], a.Ow[1]), __fsub_rn(Xw[2], a.Ow[2])};
            dist3D = norm3_cv(PO);
            if (dist3D < minDistance || dist3D > maxDistance) break;
            const float Pn[3] = {a.normal[3 * m], a.normal[3 * m + 1], a.normal[3 * m + 2]};
            if (dot3_cv(PO, Pn) < 0.5 * (double)dist3D) break;
        }
        if (dist3D < minDistance || dist3D > maxDistance) break;
        const float ratio = __fdiv_rn(dist3D, minDistance);
        int pred = 0;
        while (pred < a.nlevels && a.scales[pred] < ratio) pred++;   // lower_bound
        pred = min(pred, a.nlevels - 1);
        const float radius = __fmul_rn(a.th, a.scales[pred]);
        const AreaQuery q = area_cells(a.K, u, v, radius);
        if (q.empty) break;
        uint4 d0, d1;
        load_desc(a.qdesc + (size_t)m * 32, d0, d1);
        unsigned long long bk = ~0ull;
        for (int j = lane; j < a.K.n; j += 64) {
            const int co = tco[j];
            const int oct = co >> 16;
            if (oct < pred - 1 || oct > pred) continue;
            const int cell = (co & 0xFFFF) == 0xFFFF ? -1 : (co & 0xFFFF);
            if (!in_area(q, cell, tx[j], ty[j], u, v, radius)) continue;
            uint4 b0, b1;
            load_desc(a.K.desc + (size_t)j * 32, b0, b1);
            const unsigned long long key = ((unsigned long long)hamming256(d0, d1, b0, b1) << 32) |
                                           ((unsigned long long)cell << 12) | (unsigned long long)j;
            bk = key < bk ? key : bk;
        }
        bk = wave_min_u64(bk);
        if (bk != ~0ull) {
            best_idx = (int)(bk & 0xFFF);
            best_dist = (int)(bk >> 32);
        }
    } while (false);
    if (lane == 0) {
        a.best_idx[m] = best_idx;
        a.best_dist[m] = best_dist;
    }
}

__global__ __launch_bounds__(256) void k_kf_project(KfProjArgs a)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    kf_project_block(a, smem, blockIdx.x);
}

// Batched form: grid.y = keyframe job (each with its own keypoint table,
// pose and map points), grid.x = blocks of four map points.
__global__ __launch_bounds__(256) void k_kf_project_jobs(const KfProjArgs* jobs)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const KfProjArgs& a = jobs[blockIdx.y];
    if ((int)blockIdx.x * (kBlock / 64) >= a.nq) return;   // uniform per block
    kf_project_block(a, smem, blockIdx.x);
}

// MapPoint::ComputeDistinctiveDescriptors, one wavefront per map point.
__global__ __launch_bounds__(256) void k_distinctive(const int32_t* ptr, const uint8_t* desc, int n_mp, int32_t* best)
{
    const int lane = threadIdx.x & 63;
    const int m = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    if (m >= n_mp) return;
    const int b0 = ptr[m], N = ptr[m + 1] - b0;
    if (N <= 0) {
        if (lane == 0) best[m] = -1;
        return;
    }
    const uint8_t* D = desc + (size_t)b0 * 32;
    const int k = (N - 1) / 2;                     // vDists[0.5*(N-1)]
    uint32_t key = 0xFFFFFFFFu;
    for (int i = lane; i < N; i += 64) {
        uint4 a0, a1;
        load_desc(D + (size_t)i * 32, a0, a1);
        int lo = 0, hi = 256;                       // smallest v with #{d(i,l) <= v} > k
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            int cnt = 0;
            for (int l = 0; l < N; l++) {
                uint4 c0, c1;
                load_desc(D + (size_t)l * 32, c0, c1);
                cnt += hamming256(a0, a1, c0, c1) <= mid;
            }
            if (cnt > k) hi = mid;
            else lo = mid + 1;
        }
        const uint32_t kk = ((uint32_t)lo << 20) | (uint32_t)i;
        key = kk < key ? kk : key;
    }
    key = wave_min_u32(key);
    if (lane == 0) best[m] = (int)(key & 0xFFFFF);
}


// Sequential projection searches (the candidate exclusion depends on the
// earlier points' assignments): one wavefront replays the reference's loop
// over the points in order; per point the lanes stride the searched
// frame's keypoints (LDS table) and one min reduction gives the first
// strict minimum in GetFeaturesInArea order.
//  variant 0: SearchByProjection(KeyFrame*, Scw, vpPoints, vpMatched, th)
//             (src/ORBmatcher.cc:286-407)
//  variant 1: SearchByProjection(Frame&, KeyFrame*, sAlreadyFound, th,
//             ORBdist) (:1622-1746), with the rotation-consistency filter
struct SeqProjArgs {
    FrameDev T;                 // searched keyframe (variant 0) / frame (variant 1)
    float scales[kMaxLevels];
    int nlevels;
    float cam[4];
    float R[9], t[3], Ow[3];
    float th;
    int orb_dist, check_ori, variant;
    int nq;
    const float* pos;
    const float* normal;
    const float* dmin;
    const float* dmax;
    const uint8_t* qdesc;
    const uint8_t* qskip;       // variant 0: isBad || already found; variant 1: !valid
    const orbx_keypoint* qkps;  // variant 1: the KF keypoints (angles)
    const uint8_t* assigned;    // variant 1: CurrentFrame.mvpMapPoints[i] != NULL
    int32_t* out;               // variant 0: vpMatched (in/out); variant 1: matches_f
    int32_t* out_n;
};

__global__ __launch_bounds__(64) void k_proj_seq(SeqProjArgs a)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int n = a.T.n, lane = threadIdx.x;
    float* tx = reinterpret_cast<float*>(smem);
    float* ty = tx + n;
    int* tco = reinterpret_cast<int*>(ty + n);
    int* taken = tco + n;
    int* keys = taken + n;
    int* hist = keys + n;
    signed char* bins = reinterpret_cast<signed char*>(hist + 32);
    for (int i = lane; i < n; i += 64) {
        const orbx_keypoint k = a.T.kps[i];
        tx[i] = k.x;
        ty[i] = k.y;
        const int cell = grid_cell(a.T, k.x, k.y);
        tco[i] = (cell & 0xFFFF) | (k.octave << 16);
        taken[i] = a.variant == 0 ? (a.out[i] >= 0) : (int)a.assigned[i];
    }
    wave_sync();
    int nmatches = 0, npushed = 0;
    for (int m = 0; m < a.nq; m++) {
        if (a.qskip[m]) continue;
        const float Xw[3] = {a.pos[3 * m], a.pos[3 * m + 1], a.pos[3 * m + 2]};
        float pc[3];
        xform3(a.R, a.t, Xw, pc);
        float u, v;
        int pred, lo, hi, accept;
        const float PO[3] = {__fsub_rn(Xw[0], a.Ow[0]), __fsub_rn(Xw[1], a.Ow[1]), __fsub_rn(Xw[2], a.Ow[2])};
        const float dist3D = norm3_cv(PO);
        const float minDistance = a.dmin[m];
        if (a.variant == 0) {
            if (pc[2] < 0.0f) continue;
            const float invz = __fdiv_rn(1.0f, pc[2]);
            u = __fadd_rn(__fmul_rn(a.cam[0], __fmul_rn(pc[0], invz)), a.cam[2]);
            v = __fadd_rn(__fmul_rn(a.cam[1], __fmul_rn(pc[1], invz)), a.cam[3]);
            if (!(u >= a.T.min_x && u < a.T.max_x && v >= a.T.min_y && v < a.T.max_y)) continue;
            if (dist3D < minDistance || dist3D > a.dmax[m]) continue;
            const float Pn[3] = {a.normal[3 * m], a.normal[3 * m + 1], a.normal[3 * m + 2]};
            if (dot3_cv(PO, Pn) < 0.5 * (double)dist3D) continue;
        } else {
            const float invzc = (float)(1.0 / (double)pc[2]);
            u = __fadd_rn(__fmul_rn(__fmul_rn(a.cam[0], pc[0]), invzc), a.cam[2]);
            v = __fadd_rn(__fmul_rn(__fmul_rn(a.cam[1], pc[1]), invzc), a.cam[3]);
            if (u < a.T.min_x || u > a.T.max_x) continue;
            if (v < a.T.min_y || v > a.T.max_y) continue;
        }
        const float ratio = __fdiv_rn(dist3D, minDistance);
        pred = 0;
        while (pred < a.nlevels && a.scales[pred] < ratio) pred++;
        pred = min(pred, a.nlevels - 1);
        const float radius = __fmul_rn(a.th, a.scales[pred]);
        if (a.variant == 0) {
            lo = pred - 1;
            hi = pred;
            accept = kTHLow;
        } else {
            lo = pred - 1;
            hi = pred + 1;
            accept = a.orb_dist;
        }
        const AreaQuery q = area_cells(a.T, u, v, radius);
        if (q.empty) continue;
        uint4 d0, d1;
        load_desc(a.qdesc + (size_t)m * 32, d0, d1);
        unsigned long long bk = ~0ull;
        for (int j = lane; j < n; j += 64) {
            const int co = tco[j];
            const int oct = co >> 16;
            if (oct < lo || oct > hi) continue;
            const int cell = (co & 0xFFFF) == 0xFFFF ? -1 : (co & 0xFFFF);
            if (!in_area(q, cell, tx[j], ty[j], u, v, radius)) continue;
            if (taken[j]) continue;
            uint4 b0, b1;
            load_desc(a.T.desc + (size_t)j * 32, b0, b1);
            const unsigned long long key = ((unsigned long long)hamming256(d0, d1, b0, b1) << 32) |
                                           ((unsigned long long)cell << 12) | (unsigned long long)j;
            bk = key < bk ? key : bk;
        }
        bk = wave_min_u64(bk);
        if (bk == ~0ull || (int)(bk >> 32) > accept) continue;
        const int j = (int)(bk & 0xFFF);
        if (lane == 0) {
            taken[j] = 1;
            a.out[j] = m;
            if (a.variant == 1 && a.check_ori) {
                bins[npushed] = (signed char)rot_bin(a.qkps[m].angle, a.T.kps[j].angle);
                keys[npushed] = j;
            }
        }
        if (a.variant == 1 && a.check_ori) npushed++;
        nmatches++;
        wave_sync();
    }
    wave_sync();
    if (lane == 0) {
        if (npushed) {
            for (int b = 0; b < kHistoLength; b++) hist[b] = 0;
            for (int i = 0; i < npushed; i++) hist[bins[i]]++;
            int i1, i2, i3;
            three_maxima(hist, i1, i2, i3);
            for (int i = 0; i < npushed; i++) {
                const int b = bins[i];
                if (b == i1 || b == i2 || b == i3) continue;
                a.out[keys[i]] = -1;
                nmatches--;
            }
        }
        *a.out_n = nmatches;
    }
}

namespace {

inline size_t al256(size_t b) { return (b + 255) & ~size_t(255); }

bool valid_kf(const orbx_frame_view* v)
{
    return v && v->n >= 0 && v->n <= kMaxFeatures && (v->n == 0 || (v->keys_un && v->desc)) && v->max_x > v->min_x &&
           v->max_y > v->min_y && v->nlevels > 0 && v->nlevels <= kMaxLevels;
}

bool valid_mps(const orbx_mappoint_view* p, bool need_normal)
{
    return p && p->n >= 0 &&
           (p->n == 0 || (p->pos && p->min_dist && p->max_dist && p->desc && (!need_normal || p->normal)));
}

// Same arithmetic as oracle/ref_proj.cpp pose_parts (src/ORBmatcher.cc:
// 1145-1149; KeyFrame::SetPose's Ow = -Rwc * tcw).
void pose_parts(const float* T, int sim3, float* R, float* t, float* Ow)
{
    if (sim3) {
        double s = 0;
        for (int c = 0; c < 3; c++) s += (double)T[c] * (double)T[c];
        const float scw = (float)std::sqrt(s);
        const double inv = 1.0 / (double)scw;
        for (int r = 0; r < 3; r++) {
            for (int c = 0; c < 3; c++) R[3 * r + c] = (float)((double)T[4 * r + c] * inv);
            t[r] = (float)((double)T[4 * r + 3] * inv);
        }
    } else {
        for (int r = 0; r < 3; r++) {
            for (int c = 0; c < 3; c++) R[3 * r + c] = T[4 * r + c];
            t[r] = T[4 * r + 3];
        }
    }
    for (int c = 0; c < 3; c++) Ow[c] = -(R[c] * t[0] + R[3 + c] * t[1] + R[6 + c] * t[2]);
}

FrameDev kf_dev(const orbx_frame_view* v, const uint8_t* base, size_t kp_off, size_t desc_off)
{
    FrameDev F;
    F.kps = reinterpret_cast<const orbx_keypoint*>(base + kp_off);
    F.desc = base + desc_off;
    F.n = v->n;
    F.min_x = v->min_x;
    F.max_x = v->max_x;
    F.min_y = v->min_y;
    F.max_y = v->max_y;
    F.grid_w_inv = static_cast<float>(kGridCols) / (v->max_x - v->min_x);   // src/Frame.cc:76-77
    F.grid_h_inv = static_cast<float>(kGridRows) / (v->max_y - v->min_y);
    return F;
}

struct Staging {
    orbx_ctx* ctx;
    size_t at = 0;
    std::vector<std::pair<size_t, std::pair<const void*, size_t>>> puts;
    size_t res(size_t bytes, const void* src = nullptr)
    {
        const size_t o = at;
        at += al256(std::max<size_t>(bytes, 1));
        if (src && bytes) puts.push_back({o, {src, bytes}});
        return o;
    }
    int upload()
    {
        int r = ensure_scratch(ctx, at);
        if (r != ORBX_OK) return r;
        uint8_t* d = static_cast<uint8_t*>(ctx->scratch);
        for (auto& p : puts)
            ORBX_HIP_CHECK(hipMemcpyAsync(d + p.first, p.second.first, p.second.second, hipMemcpyHostToDevice,
                                          ctx->stream));
        return ORBX_OK;
    }
    uint8_t* base() const { return static_cast<uint8_t*>(ctx->scratch); }
};

// Stages the keyframe and the map points, fills the common fields.
struct ProjStage {
    size_t kp, kd, pos, nrm, dmin, dmax, qd, qv, bi, bd;
};

ProjStage stage_proj(Staging& s, const orbx_frame_view* K, const orbx_mappoint_view* P, const uint8_t* qvalid)
{
    ProjStage o;
    o.kp = s.res((size_t)K->n * sizeof(orbx_keypoint), K->keys_un);
    o.kd = s.res((size_t)K->n * 32, K->desc);
    o.pos = s.res((size_t)P->n * 12, P->pos);
    o.nrm = s.res((size_t)P->n * 12, P->normal);
    o.dmin = s.res((size_t)P->n * 4, P->min_dist);
    o.dmax = s.res((size_t)P->n * 4, P->max_dist);
    o.qd = s.res((size_t)P->n * 32, P->desc);
    o.qv = s.res((size_t)P->n, qvalid);
    o.bi = s.res((size_t)P->n * 4);
    o.bd = s.res((size_t)P->n * 4);
    return o;
}

void fill_proj(KfProjArgs& a, const Staging& s, const ProjStage& o, const orbx_frame_view* K,
               const orbx_mappoint_view* P, bool has_valid)
{
    uint8_t* d = s.base();
    a.K = kf_dev(K, d, o.kp, o.kd);
    a.nlevels = K->nlevels;
    a.scales[0] = 1.0f;
    for (int l = 1; l < K->nlevels; l++) a.scales[l] = a.scales[l - 1] * K->scale_factor;   // src/Frame.cc:98-102
    a.nq = P->n;
    a.pos = reinterpret_cast<const float*>(d + o.pos);
    a.normal = reinterpret_cast<const float*>(d + o.nrm);
    a.dmin = reinterpret_cast<const float*>(d + o.dmin);
    a.dmax = reinterpret_cast<const float*>(d + o.dmax);
    a.qdesc = d + o.qd;
    a.qvalid = has_valid ? d + o.qv : nullptr;
    a.best_idx = reinterpret_cast<int32_t*>(d + o.bi);
    a.best_dist = reinterpret_cast<int32_t*>(d + o.bd);
}

int launch_proj(orbx_ctx* ctx, const KfProjArgs& a)
{
    if (a.nq == 0) return ORBX_OK;
    const int per = kBlock / 64;
    const size_t lds = (size_t)std::max(a.K.n, 1) * 12;
    hipLaunchKernelGGL(k_kf_project, dim3((a.nq + per - 1) / per), dim3(kBlock), lds, ctx->stream, a);
    ORBX_HIP_CHECK(hipGetLastError());
    return ORBX_OK;
}

}  // namespace
}  // namespace orbx

using namespace orbx;

extern "C" int orbx_fuse_candidates(orbx_ctx* ctx, const orbx_frame_view* KF, const float* cam,
                                    const orbx_mappoint_view* mps, const float* T, int sim3, float th,
                                    int32_t* best_idx, int32_t* best_dist)
{
    if (!ctx || !valid_kf(KF) || !cam || !valid_mps(mps, true) || !T || (mps->n > 0 && (!best_idx || !best_dist)))
        return ORBX_ERR_ARG;
    ctx_enter(ctx);
    Staging s{ctx};
    const ProjStage o = stage_proj(s, KF, mps, nullptr);
    int r = s.upload();
    if (r != ORBX_OK) return r;
    KfProjArgs a{};
    fill_proj(a, s, o, KF, mps, false);
    for (int k = 0; k < 4; k++) a.cam[k] = cam[k];
    pose_parts(T, sim3, a.Ra, a.ta, a.Ow);
    a.two_stage = 0;
    a.mode = sim3 ? 1 : 0;
    a.th = th;
    if ((r = launch_proj(ctx, a)) != ORBX_OK) return r;
    if (mps->n) {
        ORBX_HIP_CHECK(hipMemcpyAsync(best_idx, s.base() + o.bi, (size_t)mps->n * 4, hipMemcpyDeviceToHost, ctx->stream));
        ORBX_HIP_CHECK(hipMemcpyAsync(best_dist, s.base() + o.bd, (size_t)mps->n * 4, hipMemcpyDeviceToHost, ctx->stream));
    }
    ORBX_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    return ORBX_OK;
}

// SearchInNeighbors' first loop (src/LocalMapping.cc:403-416: Fuse of the
// current keyframe's map points into every target keyframe) in one upload,
// one launch and one readback.  Map-point views that are the same object are
// uploaded once.
extern "C" int orbx_fuse_candidates_batch(orbx_ctx* ctx, int n_kf, const orbx_frame_view* KFs, const float* cams,
                                          const orbx_mappoint_view* const* mps, const float* Ts, int sim3, float th,
                                          int32_t* const* best_idx, int32_t* const* best_dist)
{
    if (!ctx || n_kf < 0 || (n_kf > 0 && (!KFs || !cams || !mps || !Ts || !best_idx || !best_dist))) return ORBX_ERR_ARG;
    for (int k = 0; k < n_kf; k++)
        if (!valid_kf(&KFs[k]) || !valid_mps(mps[k], true) || (mps[k]->n > 0 && (!best_idx[k] || !best_dist[k])))
            return ORBX_ERR_ARG;
    if (n_kf == 0) return ORBX_OK;
    ctx_enter(ctx);
    Staging s{ctx};
    struct Off {
        size_t kp, kd, pos, nrm, dmin, dmax, qd, bi, bd;
    };
    std::vector<Off> o(n_kf);
    int max_n = 1, max_q = 0;
    for (int k = 0; k < n_kf; k++) {
        const orbx_frame_view* K = &KFs[k];
        const orbx_mappoint_view* P = mps[k];
        o[k].kp = s.res((size_t)K->n * sizeof(orbx_keypoint), K->keys_un);
        o[k].kd = s.res((size_t)K->n * 32, K->desc);
        int same = -1;
        for (int j = 0; j < k && same < 0; j++)
            if (mps[j] == P) same = j;
        if (same >= 0) {   // the same map points: reuse their upload
            o[k].pos = o[same].pos;
            o[k].nrm = o[same].nrm;
            o[k].dmin = o[same].dmin;
            o[k].dmax = o[same].dmax;
            o[k].qd = o[same].qd;
        } else {
            o[k].pos = s.res((size_t)P->n * 12, P->pos);
            o[k].nrm = s.res((size_t)P->n * 12, P->normal);
            o[k].dmin = s.res((size_t)P->n * 4, P->min_dist);
            o[k].dmax = s.res((size_t)P->n * 4, P->max_dist);
            o[k].qd = s.res((size_t)P->n * 32, P->desc);
        }
        o[k].bi = s.res((size_t)P->n * 4);
        o[k].bd = s.res((size_t)P->n * 4);
        max_n = std::max(max_n, K->n);
        max_q = std::max(max_q, P->n);
    }
    const size_t o_jobs = s.res(sizeof(KfProjArgs) * (size_t)n_kf);
    std::vector<KfProjArgs> jobs(n_kf);
    uint8_t* d = nullptr;
    int r = ensure_scratch(ctx, s.at);
    if (r != ORBX_OK) return r;
    d = s.base();
    for (int k = 0; k < n_kf; k++) {
        const orbx_frame_view* K = &KFs[k];
        KfProjArgs& a = jobs[k];
        a = KfProjArgs{};
        a.K = kf_dev(K, d, o[k].kp, o[k].kd);
        a.nlevels = K->nlevels;
        a.scales[0] = 1.0f;
        for (int l = 1; l < K->nlevels; l++) a.scales[l] = a.scales[l - 1] * K->scale_factor;   // src/Frame.cc:98-102
        a.nq = mps[k]->n;
        a.pos = reinterpret_cast<const float*>(d + o[k].pos);
        a.normal = reinterpret_cast<const float*>(d + o[k].nrm);
        a.dmin = reinterpret_cast<const float*>(d + o[k].dmin);
        a.dmax = reinterpret_cast<const float*>(d + o[k].dmax);
        a.qdesc = d + o[k].qd;
        a.qvalid = nullptr;
        a.best_idx = reinterpret_cast<int32_t*>(d + o[k].bi);
        a.best_dist = reinterpret_cast<int32_t*>(d + o[k].bd);
        for (int c = 0; c < 4; c++) a.cam[c] = cams[4 * k + c];
        pose_parts(Ts + 16 * k, sim3, a.Ra, a.ta, a.Ow);
        a.two_stage = 0;
        a.mode = sim3 ? 1 : 0;
        a.th = th;
    }
    s.puts.push_back({o_jobs, {jobs.data(), sizeof(KfProjArgs) * (size_t)n_kf}});
    if ((r = s.upload()) != ORBX_OK) return r;
    if (max_q > 0) {
        const int per = kBlock / 64;
        hipLaunchKernelGGL(k_kf_project_jobs, dim3((max_q + per - 1) / per, n_kf), dim3(kBlock), (size_t)max_n * 12,
                           ctx->stream, reinterpret_cast<const KfProjArgs*>(d + o_jobs));
        ORBX_HIP_CHECK(hipGetLastError());
    }
    for (int k = 0; k < n_kf; k++)
        if (mps[k]->n) {
            ORBX_HIP_CHECK(hipMemcpyAsync(best_idx[k], d + o[k].bi, (size_t)mps[k]->n * 4, hipMemcpyDeviceToHost,
                                          ctx->stream));
            ORBX_HIP_CHECK(hipMemcpyAsync(best_dist[k], d + o[k].bd, (size_t)mps[k]->n * 4, hipMemcpyDeviceToHost,
                                          ctx->stream));
        }
    ORBX_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    return ORBX_OK;
}

// LocalMapping::SearchInNeighbors' Fuse loop against keyframes that stay in
// their extraction slots: the keyframes' keypoints (mvKeysUn after
// orbx_dev_undistort) and descriptors are read where orbx_dev_extract left
// them; only the map points, poses and cameras travel.
extern "C" int orbx_dev_fuse_candidates(orbx_ctx* ctx, int n_kf, const int* slots, const float* bounds,
                                        const float* cams, const orbx_mappoint_view* const* mps, const float* Ts,
                                        int sim3, float th, int32_t* const* best_idx, int32_t* const* best_dist)
{
    if (!ctx || n_kf < 0 || (n_kf > 0 && (!slots || !cams || !mps || !Ts || !best_idx || !best_dist)))
        return ORBX_ERR_ARG;
    if (ctx->geom_w <= 0) return ORBX_ERR_ARG;
    for (int k = 0; k < n_kf; k++) {
        if (slots[k] < 0 || slots[k] >= ctx->slots || !valid_mps(mps[k], true) ||
            (mps[k]->n > 0 && (!best_idx[k] || !best_dist[k])))
            return ORBX_ERR_ARG;
        if (bounds && !(bounds[4 * k + 1] > bounds[4 * k] && bounds[4 * k + 3] > bounds[4 * k + 2])) return ORBX_ERR_ARG;
    }
    if (n_kf == 0) return ORBX_OK;
    ctx_enter(ctx);
    // the slots' keypoint counts size the kernel's LDS grid
    std::vector<int32_t> cnt(ctx->slots);
    ORBX_HIP_CHECK(hipMemcpyAsync(cnt.data(), ctx->out_n, sizeof(int32_t) * ctx->slots, hipMemcpyDeviceToHost,
                                  ctx->stream));
    ORBX_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    const Geometry& g = ctx->geom;
    const size_t nf = g.nfeatures;
    Staging s{ctx};
    struct Off {
        size_t pos, nrm, dmin, dmax, qd, bi, bd;
    };
    std::vector<Off> o(n_kf);
    int max_n = 1, max_q = 0;
    for (int k = 0; k < n_kf; k++) {
        const orbx_mappoint_view* P = mps[k];
        int same = -1;
        for (int j = 0; j < k && same < 0; j++)
            if (mps[j] == P) same = j;
        if (same >= 0) {
            o[k] = o[same];
        } else {
            o[k].pos = s.res((size_t)P->n * 12, P->pos);
            o[k].nrm = s.res((size_t)P->n * 12, P->normal);
            o[k].dmin = s.res((size_t)P->n * 4, P->min_dist);
            o[k].dmax = s.res((size_t)P->n * 4, P->max_dist);
            o[k].qd = s.res((size_t)P->n * 32, P->desc);
        }
        o[k].bi = s.res((size_t)P->n * 4);
        o[k].bd = s.res((size_t)P->n * 4);
        max_n = std::max(max_n, std::min<int>(cnt[slots[k]], (int)nf));
        max_q = std::max(max_q, P->n);
    }
    const size_t o_jobs = s.res(sizeof(KfProjArgs) * (size_t)n_kf);
    std::vector<KfProjArgs> jobs(n_kf);
    int r = ensure_scratch(ctx, s.at);
    if (r != ORBX_OK) return r;
    uint8_t* d = s.base();
    for (int k = 0; k < n_kf; k++) {
        const int sl = slots[k];
        // the extracted frame as a keyframe view (bounds: the caller's
        // ComputeImageBounds, or the undistorted image 0..w, 0..h)
        orbx_frame_view v{};
        v.n = std::min<int>(cnt[sl], (int)nf);
        v.min_x = bounds ? bounds[4 * k] : 0.f;
        v.max_x = bounds ? bounds[4 * k + 1] : (float)g.w;
        v.min_y = bounds ? bounds[4 * k + 2] : 0.f;
        v.max_y = bounds ? bounds[4 * k + 3] : (float)g.h;
        KfProjArgs& a = jobs[k];
        a = KfProjArgs{};
        a.K = kf_dev(&v, nullptr, 0, 0);
        a.K.kps = ctx->out_kps + (size_t)sl * nf;
        a.K.desc = ctx->out_desc + (size_t)sl * nf * 32;
        a.nlevels = g.nlevels;
        a.scales[0] = 1.0f;
        for (int l = 1; l < g.nlevels; l++) a.scales[l] = a.scales[l - 1] * g.scale_factor;   // src/Frame.cc:98-102
        a.nq = mps[k]->n;
        a.pos = reinterpret_cast<const float*>(d + o[k].pos);
        a.normal = reinterpret_cast<const float*>(d + o[k].nrm);
        a.dmin = reinterpret_cast<const float*>(d + o[k].dmin);
        a.dmax = reinterpret_cast<const float*>(d + o[k].dmax);
        a.qdesc = d + o[k].qd;
        a.qvalid = nullptr;
        a.best_idx = reinterpret_cast<int32_t*>(d + o[k].bi);
        a.best_dist = reinterpret_cast<int32_t*>(d + o[k].bd);
        for (int c = 0; c < 4; c++) a.cam[c] = cams[4 * k + c];
        pose_parts(Ts + 16 * k, sim3, a.Ra, a.ta, a.Ow);
        a.two_stage = 0;
        a.mode = sim3 ? 1 : 0;
        a.th = th;
    }
    s.puts.push_back({o_jobs, {jobs.data(), sizeof(KfProjArgs) * (size_t)n_kf}});
    if ((r = s.upload()) != ORBX_OK) return r;
    if (max_q > 0) {
        const int per = kBlock / 64;
        hipLaunchKernelGGL(k_kf_project_jobs, dim3((max_q + per - 1) / per, n_kf), dim3(kBlock), (size_t)max_n * 12,
                           ctx->stream, reinterpret_cast<const KfProjArgs*>(d + o_jobs));
        ORBX_HIP_CHECK(hipGetLastError());
    }
    for (int k = 0; k < n_kf; k++)
        if (mps[k]->n) {
            ORBX_HIP_CHECK(hipMemcpyAsync(best_idx[k], d + o[k].bi, (size_t)mps[k]->n * 4, hipMemcpyDeviceToHost,
                                          ctx->stream));
            ORBX_HIP_CHECK(hipMemcpyAsync(best_dist[k], d + o[k].bd, (size_t)mps[k]->n * 4, hipMemcpyDeviceToHost,
                                          ctx->stream));
        }
    ORBX_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    return ORBX_OK;
}

// SearchBySim3 for keyframe views whose keypoints and descriptors are on
// the host (dev1 / dev2 null: staged) or already on the device (the slot
// arrays: the views then carry only counts, bounds and the scale pyramid).
static int run_sim3(orbx_ctx* ctx, const orbx_frame_view* KF1, const orbx_frame_view* KF2,
                    const orbx_keypoint* dk1, const uint8_t* dd1, const orbx_keypoint* dk2, const uint8_t* dd2,
                    const float* cam, const orbx_mappoint_view* mp1, const uint8_t* valid1,
                    const orbx_mappoint_view* mp2, const uint8_t* valid2, const float* T1w, const float* T2w,
                    float s12, const float* R12, const float* t12, float th, const int32_t* prior12, int32_t* new12,
                    int* n_found)
{
    const int N1 = KF1->n, N2 = KF2->n;
    // vbAlreadyMatched1/2 (:1300-1313) folded into the query masks
    std::vector<uint8_t> q1(N1), q2(N2);
    std::vector<uint8_t> already2(N2, 0);
    for (int i = 0; i < N1; i++)
        if (prior12[i] >= 0 && prior12[i] < N2) already2[prior12[i]] = 1;
    for (int i = 0; i < N1; i++) q1[i] = valid1[i] && prior12[i] == -2;
    for (int i = 0; i < N2; i++) q2[i] = valid2[i] && !already2[i];
    // sR12 = s12*R12, sR21 = (1.0/s12)*R12.t(), t21 = -sR21*t12 (:1284-1286)
    float R1w[9], t1w[3], R2w[9], t2w[3], sR12[9], sR21[9], t21[3];
    for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 3; c++) {
            R1w[3 * r + c] = T1w[4 * r + c];
            R2w[3 * r + c] = T2w[4 * r + c];
        }
        t1w[r] = T1w[4 * r + 3];
        t2w[r] = T2w[4 * r + 3];
    }
    const double inv_s = 1.0 / (double)s12;
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) {
            sR12[3 * r + c] = (float)((double)s12 * (double)R12[3 * r + c]);
            sR21[3 * r + c] = (float)(inv_s * (double)R12[3 * c + r]);
        }
    for (int r = 0; r < 3; r++) t21[r] = -(sR21[3 * r] * t12[0] + sR21[3 * r + 1] * t12[1] + sR21[3 * r + 2] * t12[2]);
    ctx_enter(ctx);
    Staging s{ctx};
    const ProjStage o1 = stage_proj(s, KF2, mp1, q1.data());   // KF1 points searched in KF2
    const ProjStage o2 = stage_proj(s, KF1, mp2, q2.data());   // KF2 points searched in KF1
    int r = s.upload();
    if (r != ORBX_OK) return r;
    KfProjArgs a{};
    fill_proj(a, s, o1, KF2, mp1, true);
    if (dk2) {
        a.K.kps = dk2;
        a.K.desc = dd2;
    }
    for (int k = 0; k < 4; k++) a.cam[k] = cam[k];
    std::copy(R1w, R1w + 9, a.Ra);
    std::copy(t1w, t1w + 3, a.ta);
    std::copy(sR21, sR21 + 9, a.Rb);
    std::copy(t21, t21 + 3, a.tb);
    a.two_stage = 1;
    a.mode = 2;
    a.th = th;
    if ((r = launch_proj(ctx, a)) != ORBX_OK) return r;
    KfProjArgs b{};
    fill_proj(b, s, o2, KF1, mp2, true);
    if (dk1) {
        b.K.kps = dk1;
        b.K.desc = dd1;
    }
    for (int k = 0; k < 4; k++) b.cam[k] = cam[k];
    std::copy(R2w, R2w + 9, b.Ra);
    std::copy(t2w, t2w + 3, b.ta);
    std::copy(sR12, sR12 + 9, b.Rb);
    std::copy(t12, t12 + 3, b.tb);
    b.two_stage = 1;
    b.mode = 2;
    b.th = th;
    if ((r = launch_proj(ctx, b)) != ORBX_OK) return r;
    std::vector<int32_t> bi1(N1), bd1(N1), bi2(N2), bd2(N2);
    if (N1) {
        ORBX_HIP_CHECK(hipMemcpyAsync(bi1.data(), s.base() + o1.bi, (size_t)N1 * 4, hipMemcpyDeviceToHost, ctx->stream));
        ORBX_HIP_CHECK(hipMemcpyAsync(bd1.data(), s.base() + o1.bd, (size_t)N1 * 4, hipMemcpyDeviceToHost, ctx->stream));
    }
    if (N2) {
        ORBX_HIP_CHECK(hipMemcpyAsync(bi2.data(), s.base() + o2.bi, (size_t)N2 * 4, hipMemcpyDeviceToHost, ctx->stream));
        ORBX_HIP_CHECK(hipMemcpyAsync(bd2.data(), s.base() + o2.bd, (size_t)N2 * 4, hipMemcpyDeviceToHost, ctx->stream));
    }
    ORBX_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    // bestDist <= TH_HIGH (:1395, :1480), then the agreement check (:1486-1502)
    int nFound = 0;
    for (int i1 = 0; i1 < N1; i1++) {
        new12[i1] = -1;
        const int idx2 = bd1[i1] <= kTHHigh ? bi1[i1] : -1;
        if (idx2 >= 0 && bd2[idx2] <= kTHHigh && bi2[idx2] == i1) {
            new12[i1] = idx2;
            nFound++;
        }
    }
    *n_found = nFound;
    return ORBX_OK;
}

extern "C" int orbx_search_by_sim3(orbx_ctx* ctx, const orbx_frame_view* KF1, const orbx_frame_view* KF2,
                                   const float* cam, const orbx_mappoint_view* mp1, const uint8_t* valid1,
                                   const orbx_mappoint_view* mp2, const uint8_t* valid2, const float* T1w,
                                   const float* T2w, float s12, const float* R12, const float* t12, float th,
                                   const int32_t* prior12, int32_t* new12, int* n_found)
{
    if (!ctx || !valid_kf(KF1) || !valid_kf(KF2) || !cam || !valid_mps(mp1, false) || !valid_mps(mp2, false) ||
        mp1->n != KF1->n || mp2->n != KF2->n || (KF1->n && (!valid1 || !prior12 || !new12)) ||
        (KF2->n && !valid2) || !T1w || !T2w || !R12 || !t12 || !n_found)
        return ORBX_ERR_ARG;
    return run_sim3(ctx, KF1, KF2, nullptr, nullptr, nullptr, nullptr, cam, mp1, valid1, mp2, valid2, T1w, T2w, s12,
                    R12, t12, th, prior12, new12, n_found);
}

// LoopClosing::ComputeSim3's SearchBySim3 with both keyframes resident in
// their extraction slots.
extern "C" int orbx_dev_search_by_sim3(orbx_ctx* ctx, int slot1, const float* bounds1, int slot2,
                                       const float* bounds2, const float* cam, const orbx_mappoint_view* mp1,
                                       const uint8_t* valid1, const orbx_mappoint_view* mp2, const uint8_t* valid2,
                                       const float* T1w, const float* T2w, float s12, const float* R12,
                                       const float* t12, float th, const int32_t* prior12, int32_t* new12, int cap,
                                       int* n_found)
{
    if (!ctx || slot1 < 0 || slot1 >= ctx->slots || slot2 < 0 || slot2 >= ctx->slots || ctx->geom_w <= 0 || !cam ||
        !valid_mps(mp1, false) || !valid_mps(mp2, false) || !T1w || !T2w || !R12 || !t12 || !n_found || !new12)
        return ORBX_ERR_ARG;
    for (const float* b : {bounds1, bounds2})
        if (b && !(b[1] > b[0] && b[3] > b[2])) return ORBX_ERR_ARG;
    ctx_enter(ctx);
    std::vector<int32_t> cnt(ctx->slots);
    ORBX_HIP_CHECK(hipMemcpyAsync(cnt.data(), ctx->out_n, sizeof(int32_t) * ctx->slots, hipMemcpyDeviceToHost,
                                  ctx->stream));
    ORBX_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    const Geometry& g = ctx->geom;
    const size_t nf = g.nfeatures;
    const int N1 = std::min<int>(cnt[slot1], (int)nf), N2 = std::min<int>(cnt[slot2], (int)nf);
    if (mp1->n != N1 || mp2->n != N2 || (N1 && (!valid1 || !prior12)) || (N2 && !valid2)) return ORBX_ERR_ARG;
    if (cap < N1) return ORBX_ERR_CAPACITY;
    auto view = [&](int n, const float* b) {
        orbx_frame_view v{};
        v.n = n;
        v.min_x = b ? b[0] : 0.f;
        v.max_x = b ? b[1] : (float)g.w;
        v.min_y = b ? b[2] : 0.f;
        v.max_y = b ? b[3] : (float)g.h;
        v.nlevels = g.nlevels;
        v.scale_factor = g.scale_factor;
        return v;
    };
    const orbx_frame_view K1 = view(N1, bounds1), K2 = view(N2, bounds2);
    return run_sim3(ctx, &K1, &K2, ctx->out_kps + (size_t)slot1 * nf, ctx->out_desc + (size_t)slot1 * nf * 32,
                    ctx->out_kps + (size_t)slot2 * nf, ctx->out_desc + (size_t)slot2 * nf * 32, cam, mp1, valid1, mp2,
                    valid2, T1w, T2w, s12, R12, t12, th, prior12, new12, n_found);
}

extern "C" int orbx_distinctive_descriptors(orbx_ctx* ctx, int n_mp, const int32_t* obs_ptr, const uint8_t* desc,
                                            int32_t* best)
{
    if (!ctx || n_mp < 0 || (n_mp > 0 && (!obs_ptr || !best))) return ORBX_ERR_ARG;
    if (n_mp == 0) return ORBX_OK;
    if (obs_ptr[0] < 0) return ORBX_ERR_ARG;
    for (int m = 0; m < n_mp; m++)
        if (obs_ptr[m + 1] < obs_ptr[m] || obs_ptr[m + 1] - obs_ptr[m] >= (1 << 20)) return ORBX_ERR_ARG;
    const size_t rows = (size_t)obs_ptr[n_mp];
    if (rows && !desc) return ORBX_ERR_ARG;
    ctx_enter(ctx);
    Staging s{ctx};
    const size_t o_ptr = s.res((size_t)(n_mp + 1) * 4, obs_ptr), o_d = s.res(rows * 32, desc),
                 o_b = s.res((size_t)n_mp * 4);
    int r = s.upload();
    if (r != ORBX_OK) return r;
    const int per = kBlock / 64;
    hipLaunchKernelGGL(k_distinctive, dim3((n_mp + per - 1) / per), dim3(kBlock), 0, ctx->stream,
                       reinterpret_cast<const int32_t*>(s.base() + o_ptr), s.base() + o_d, n_mp,
                       reinterpret_cast<int32_t*>(s.base() + o_b));
    ORBX_HIP_CHECK(hipGetLastError());
    ORBX_HIP_CHECK(hipMemcpyAsync(best, s.base() + o_b, (size_t)n_mp * 4, hipMemcpyDeviceToHost, ctx->stream));
    ORBX_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    return ORBX_OK;
}

extern "C" int orbx_search_by_projection_kf_sim3(orbx_ctx* ctx, const orbx_frame_view* KF, const float* cam,
                                                 const orbx_mappoint_view* mps, const uint8_t* mp_skip,
                                                 const float* Scw, int th, int32_t* matched, int* n_matches)
{
    if (!ctx || !valid_kf(KF) || !cam || !valid_mps(mps, true) || !Scw || !n_matches || (mps->n && !mp_skip) ||
        (KF->n && !matched))
        return ORBX_ERR_ARG;
    ctx_enter(ctx);
    Staging s{ctx};
    const size_t o_kp = s.res((size_t)KF->n * sizeof(orbx_keypoint), KF->keys_un), o_kd = s.res((size_t)KF->n * 32, KF->desc);
    const size_t o_pos = s.res((size_t)mps->n * 12, mps->pos), o_nrm = s.res((size_t)mps->n * 12, mps->normal),
                 o_mn = s.res((size_t)mps->n * 4, mps->min_dist), o_mx = s.res((size_t)mps->n * 4, mps->max_dist),
                 o_qd = s.res((size_t)mps->n * 32, mps->desc), o_sk = s.res(mps->n, mp_skip),
                 o_out = s.res((size_t)KF->n * 4, matched), o_n = s.res(4);
    int r = s.upload();
    if (r != ORBX_OK) return r;
    uint8_t* d = s.base();
    SeqProjArgs a{};
    a.T = kf_dev(KF, d, o_kp, o_kd);
    a.nlevels = KF->nlevels;
    a.scales[0] = 1.0f;
    for (int l = 1; l < KF->nlevels; l++) a.scales[l] = a.scales[l - 1] * KF->scale_factor;
    for (int k = 0; k < 4; k++) a.cam[k] = cam[k];
    pose_parts(Scw, 1, a.R, a.t, a.Ow);
    a.th = (float)th;
    a.variant = 0;
    a.nq = mps->n;
    a.pos = reinterpret_cast<const float*>(d + o_pos);
    a.normal = reinterpret_cast<const float*>(d + o_nrm);
    a.dmin = reinterpret_cast<const float*>(d + o_mn);
    a.dmax = reinterpret_cast<const float*>(d + o_mx);
    a.qdesc = d + o_qd;
    a.qskip = d + o_sk;
    a.out = reinterpret_cast<int32_t*>(d + o_out);
    a.out_n = reinterpret_cast<int32_t*>(d + o_n);
    const size_t lds = (size_t)std::max(KF->n, 1) * 21 + 32 * 4 + 64;
    hipLaunchKernelGGL(k_proj_seq, dim3(1), dim3(64), lds, ctx->stream, a);
    ORBX_HIP_CHECK(hipGetLastError());
    if (KF->n) ORBX_HIP_CHECK(hipMemcpyAsync(matched, d + o_out, (size_t)KF->n * 4, hipMemcpyDeviceToHost, ctx->stream));
    ORBX_HIP_CHECK(hipMemcpyAsync(n_matches, d + o_n, 4, hipMemcpyDeviceToHost, ctx->stream));
    ORBX_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    return ORBX_OK;
}

// LoopClosing::ComputeSim3 / CorrectLoop's SearchByProjection(pKF, Scw, ...)
// against a keyframe resident in its extraction slot.
extern "C" int orbx_dev_search_by_projection_kf_sim3(orbx_ctx* ctx, int slot, const float* bounds, const float* cam,
                                                     const orbx_mappoint_view* mps, const uint8_t* mp_skip,
                                                     const float* Scw, int th, int32_t* matched, int cap,
                                                     int* n_matches)
{
    if (!ctx || slot < 0 || slot >= ctx->slots || ctx->geom_w <= 0 || !cam || !valid_mps(mps, true) || !Scw ||
        !n_matches || (mps->n && !mp_skip) || !matched)
        return ORBX_ERR_ARG;
    if (bounds && !(bounds[1] > bounds[0] && bounds[3] > bounds[2])) return ORBX_ERR_ARG;
    ctx_enter(ctx);
    int32_t cnt = 0;
    ORBX_HIP_CHECK(hipMemcpyAsync(&cnt, ctx->out_n + slot, 4, hipMemcpyDeviceToHost, ctx->stream));
    ORBX_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    const Geometry& g = ctx->geom;
    const size_t nf = g.nfeatures;
    const int n = std::min<int>(cnt, (int)nf);
    if (cap < n) return ORBX_ERR_CAPACITY;
    Staging s{ctx};
    const size_t o_pos = s.res((size_t)mps->n * 12, mps->pos), o_nrm = s.res((size_t)mps->n * 12, mps->normal),
                 o_mn = s.res((size_t)mps->n * 4, mps->min_dist), o_mx = s.res((size_t)mps->n * 4, mps->max_dist),
                 o_qd = s.res((size_t)mps->n * 32, mps->desc), o_sk = s.res(mps->n, mp_skip),
                 o_out = s.res((size_t)n * 4, matched), o_n = s.res(4);
    int r = s.upload();
    if (r != ORBX_OK) return r;
    uint8_t* d = s.base();
    orbx_frame_view v{};
    v.n = n;
    v.min_x = bounds ? bounds[0] : 0.f;
    v.max_x = bounds ? bounds[1] : (float)g.w;
    v.min_y = bounds ? bounds[2] : 0.f;
    v.max_y = bounds ? bounds[3] : (float)g.h;
    SeqProjArgs a{};
    a.T = kf_dev(&v, nullptr, 0, 0);
    a.T.kps = ctx->out_kps + (size_t)slot * nf;
    a.T.desc = ctx->out_desc + (size_t)slot * nf * 32;
    a.nlevels = g.nlevels;
    a.scales[0] = 1.0f;
    for (int l = 1; l < g.nlevels; l++) a.scales[l] = a.scales[l - 1] * g.scale_factor;
    for (int k = 0; k < 4; k++) a.cam[k] = cam[k];
    pose_parts(Scw, 1, a.R, a.t, a.Ow);
    a.th = (float)th;
    a.variant = 0;
    a.nq = mps->n;
    a.pos = reinterpret_cast<const float*>(d + o_pos);
    a.normal = reinterpret_cast<const float*>(d + o_nrm);
    a.dmin = reinterpret_cast<const float*>(d + o_mn);
    a.dmax = reinterpret_cast<const float*>(d + o_mx);
    a.qdesc = d + o_qd;
    a.qskip = d + o_sk;
    a.out = reinterpret_cast<int32_t*>(d + o_out);
    a.out_n = reinterpret_cast<int32_t*>(d + o_n);
    const size_t lds = (size_t)std::max(n, 1) * 21 + 32 * 4 + 64;
    hipLaunchKernelGGL(k_proj_seq, dim3(1), dim3(64), lds, ctx->stream, a);
    ORBX_HIP_CHECK(hipGetLastError());
    if (n) ORBX_HIP_CHECK(hipMemcpyAsync(matched, d + o_out, (size_t)n * 4, hipMemcpyDeviceToHost, ctx->stream));
    ORBX_HIP_CHECK(hipMemcpyAsync(n_matches, d + o_n, 4, hipMemcpyDeviceToHost, ctx->stream));
    ORBX_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    return ORBX_OK;
}

extern "C" int orbx_search_by_projection_frame_kf(orbx_ctx* ctx, const orbx_frame_view* F, const orbx_frame_view* KF,
                                                  const float* cam, const orbx_mappoint_view* kf_mps,
                                                  const uint8_t* kf_valid, const uint8_t* f_assigned,
                                                  const float* Tcw, float th, int orb_dist, int check_ori,
                                                  int32_t* matches_f, int* n_matches)
{
    if (!ctx || !valid_kf(F) || !valid_kf(KF) || !cam || !valid_mps(kf_mps, false) || kf_mps->n != KF->n || !Tcw ||
        !n_matches || (KF->n && !kf_valid) || (F->n && (!f_assigned || !matches_f)))
        return ORBX_ERR_ARG;
    ctx_enter(ctx);
    Staging s{ctx};
    const size_t o_kp = s.res((size_t)F->n * sizeof(orbx_keypoint), F->keys_un), o_kd = s.res((size_t)F->n * 32, F->desc);
    const size_t o_qk = s.res((size_t)KF->n * sizeof(orbx_keypoint), KF->keys_un),
                 o_pos = s.res((size_t)KF->n * 12, kf_mps->pos), o_mn = s.res((size_t)KF->n * 4, kf_mps->min_dist),
                 o_qd = s.res((size_t)KF->n * 32, kf_mps->desc), o_sk = s.res(KF->n), o_as = s.res(F->n, f_assigned),
                 o_out = s.res((size_t)F->n * 4), o_n = s.res(4);
    std::vector<uint8_t> skip(KF->n);
    for (int i = 0; i < KF->n; i++) skip[i] = !kf_valid[i];
    if (KF->n) s.puts.push_back({o_sk, {skip.data(), (size_t)KF->n}});
    int r = s.upload();
    if (r != ORBX_OK) return r;
    uint8_t* d = s.base();
    ORBX_HIP_CHECK(hipMemsetAsync(d + o_out, 0xFF, (size_t)std::max(F->n, 1) * 4, ctx->stream));
    SeqProjArgs a{};
    a.T = kf_dev(F, d, o_kp, o_kd);
    a.nlevels = F->nlevels;
    a.scales[0] = 1.0f;
    for (int l = 1; l < F->nlevels; l++) a.scales[l] = a.scales[l - 1] * F->scale_factor;
    for (int k = 0; k < 4; k++) a.cam[k] = cam[k];
    pose_parts(Tcw, 0, a.R, a.t, a.Ow);
    a.th = th;
    a.orb_dist = orb_dist;
    a.check_ori = check_ori;
    a.variant = 1;
    a.nq = KF->n;
    a.pos = reinterpret_cast<const float*>(d + o_pos);
    a.dmin = reinterpret_cast<const float*>(d + o_mn);
    a.qdesc = d + o_qd;
    a.qskip = d + o_sk;
    a.qkps = reinterpret_cast<const orbx_keypoint*>(d + o_qk);
    a.assigned = d + o_as;
    a.out = reinterpret_cast<int32_t*>(d + o_out);
    a.out_n = reinterpret_cast<int32_t*>(d + o_n);
    const size_t lds = (size_t)std::max(F->n, 1) * 21 + 32 * 4 + 64;
    hipLaunchKernelGGL(k_proj_seq, dim3(1), dim3(64), lds, ctx->stream, a);
    ORBX_HIP_CHECK(hipGetLastError());
    if (F->n) ORBX_HIP_CHECK(hipMemcpyAsync(matches_f, d + o_out, (size_t)F->n * 4, hipMemcpyDeviceToHost, ctx->stream));
    ORBX_HIP_CHECK(hipMemcpyAsync(n_matches, d + o_n, 4, hipMemcpyDeviceToHost, ctx->stream));
    ORBX_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    return ORBX_OK;
}

// Tracking::Relocalisation's second search, SearchByProjection(CurrentFrame,
// pKF, sAlreadyFound, th, ORBdist), with the current frame and the candidate
// keyframe both resident in their extraction slots: the frame's keypoints
// and descriptors and the keyframe's keypoints are read in HBM; the
// keyframe's map points and the flags are uploaded.
extern "C" int orbx_dev_search_by_projection_frame_kf(orbx_ctx* ctx, int f_slot, const float* f_bounds, int kf_slot,
                                                      const float* cam, const orbx_mappoint_view* kf_mps,
                                                      const uint8_t* kf_valid, const uint8_t* f_assigned,
                                                      const float* Tcw, float th, int orb_dist, int check_ori,
                                                      int32_t* matches_f, int cap, int* n_matches)
{
    if (!ctx || f_slot < 0 || f_slot >= ctx->slots || kf_slot < 0 || kf_slot >= ctx->slots || ctx->geom_w <= 0 ||
        !cam || !valid_mps(kf_mps, false) || !Tcw || !n_matches || !matches_f || !f_assigned ||
        (kf_mps->n && !kf_valid))
        return ORBX_ERR_ARG;
    if (f_bounds && !(f_bounds[1] > f_bounds[0] && f_bounds[3] > f_bounds[2])) return ORBX_ERR_ARG;
    ctx_enter(ctx);
    std::vector<int32_t> cnt(ctx->slots);
    ORBX_HIP_CHECK(hipMemcpyAsync(cnt.data(), ctx->out_n, sizeof(int32_t) * ctx->slots, hipMemcpyDeviceToHost,
                                  ctx->stream));
    ORBX_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    const Geometry& g = ctx->geom;
    const size_t nf = g.nfeatures;
    const int nF = std::min<int>(cnt[f_slot], (int)nf), nK = std::min<int>(cnt[kf_slot], (int)nf);
    if (kf_mps->n != nK) return ORBX_ERR_ARG;   // one map-point entry per keyframe keypoint
    if (cap < nF) return ORBX_ERR_CAPACITY;
    Staging s{ctx};
    const size_t o_pos = s.res((size_t)nK * 12, kf_mps->pos), o_mn = s.res((size_t)nK * 4, kf_mps->min_dist),
                 o_qd = s.res((size_t)nK * 32, kf_mps->desc), o_sk = s.res(nK), o_as = s.res(nF, f_assigned),
                 o_out = s.res((size_t)nF * 4), o_n = s.res(4);
    std::vector<uint8_t> skip(nK);
    for (int i = 0; i < nK; i++) skip[i] = !kf_valid[i];
    if (nK) s.puts.push_back({o_sk, {skip.data(), (size_t)nK}});
    int r = s.upload();
    if (r != ORBX_OK) return r;
    uint8_t* d = s.base();
    ORBX_HIP_CHECK(hipMemsetAsync(d + o_out, 0xFF, (size_t)std::max(nF, 1) * 4, ctx->stream));
    orbx_frame_view v{};
    v.n = nF;
    v.min_x = f_bounds ? f_bounds[0] : 0.f;
    v.max_x = f_bounds ? f_bounds[1] : (float)g.w;
    v.min_y = f_bounds ? f_bounds[2] : 0.f;
    v.max_y = f_bounds ? f_bounds[3] : (float)g.h;
    SeqProjArgs a{};
    a.T = kf_dev(&v, nullptr, 0, 0);
    a.T.kps = ctx->out_kps + (size_t)f_slot * nf;
    a.T.desc = ctx->out_desc + (size_t)f_slot * nf * 32;
    a.nlevels = g.nlevels;
    a.scales[0] = 1.0f;
    for (int l = 1; l < g.nlevels; l++) a.scales[l] = a.scales[l - 1] * g.scale_factor;
    for (int k = 0; k < 4; k++) a.cam[k] = cam[k];
    pose_parts(Tcw, 0, a.R, a.t, a.Ow);
    a.th = th;
    a.orb_dist = orb_dist;
    a.check_ori = check_ori;
    a.variant = 1;
    a.nq = nK;
    a.pos = reinterpret_cast<const float*>(d + o_pos);
    a.dmin = reinterpret_cast<const float*>(d + o_mn);
    a.qdesc = d + o_qd;
    a.qskip = d + o_sk;
    a.qkps = ctx->out_kps + (size_t)kf_slot * nf;
    a.assigned = d + o_as;
    a.out = reinterpret_cast<int32_t*>(d + o_out);
    a.out_n = reinterpret_cast<int32_t*>(d + o_n);
    const size_t lds = (size_t)std::max(nF, 1) * 21 + 32 * 4 + 64;
    hipLaunchKernelGGL(k_proj_seq, dim3(1), dim3(64), lds, ctx->stream, a);
    ORBX_HIP_CHECK(hipGetLastError());
    if (nF) ORBX_HIP_CHECK(hipMemcpyAsync(matches_f, d + o_out, (size_t)nF * 4, hipMemcpyDeviceToHost, ctx->stream));
    ORBX_HIP_CHECK(hipMemcpyAsync(n_matches, d + o_n, 4, hipMemcpyDeviceToHost, ctx->stream));
    ORBX_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    return ORBX_OK;
}
