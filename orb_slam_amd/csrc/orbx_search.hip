// Host-pointer entry points of the ORBmatcher searches (include/orbx.h,
// section B): frames are uploaded, one wave replays the reference's greedy
// query loop on the device, results come back.  Also the all-pairs Hamming
// kernel (brute-force matching, C3).
//
// Candidate order everywhere is Frame::GetFeaturesInArea order (cell x, then
// cell y, then keypoint index; src/Frame.cc:232-257) and ties resolve to the
// earliest candidate, as the reference's strict `<` comparisons do.  The
// second-best of a query is the earliest candidate holding the minimum over
// all admissible candidates except the best one.
#include <algorithm>
#include <cstring>
#include <vector>

#include "orbx_match_common.h"
#include "orbx_pose_dev.h"

namespace orbx {

// LDS candidate table over all keypoints of the searched frame.
struct CandTab {
    float* x;
    float* y;
    int* cell_oct;   // cell (or -1) | octave << 16
    int* taken;      // assignment state (-1 free)
};

__device__ inline void carve_tab(uint8_t* base, int cap, CandTab& t)
{
    t.x = reinterpret_cast<float*>(base);
    t.y = t.x + cap;
    t.cell_oct = reinterpret_cast<int*>(t.y + cap);
    t.taken = t.cell_oct + cap;
}

__device__ inline void fill_tab(const FrameDev& F, const uint8_t* assigned, CandTab& t)
{
    for (int i = threadIdx.x; i < F.n; i += 64) {
        const orbx_keypoint k = F.kps[i];
        t.x[i] = k.x;
        t.y[i] = k.y;
        const int cell = grid_cell(F, k.x, k.y);
        t.cell_oct[i] = (cell & 0xFFFF) | (k.octave << 16);
        t.taken[i] = (assigned && assigned[i]) ? -2 : -1;
    }
    wave_sync();
}

struct LevelFilter {
    bool check, same;
    int lo, hi;
};

__device__ inline LevelFilter level_filter(int minLevel, int maxLevel)
{
    LevelFilter f;
    f.check = !(minLevel == -1 && maxLevel == -1);
    f.same = f.check && (minLevel == maxLevel);
    f.lo = minLevel;
    f.hi = maxLevel;
    return f;
}

__device__ inline bool level_ok(const LevelFilter& f, int oct)
{
    if (f.check && !f.same) return !(oct < f.lo || oct > f.hi);
    if (f.same) return oct == f.lo;
    return true;
}

// best and second keys (dist << 32 | cell << 12 | index) over admissible
// candidates: inside the area, level filter passed, not taken.
struct Best2 {
    unsigned long long best, second;
    bool any;   // GetFeaturesInArea returned something (before `taken`)
};

__device__ inline Best2 eval_query(const CandTab& t, int n, const AreaQuery& q, float qx, float qy, float r,
                                   const LevelFilter& lf, const uint4& d1a, const uint4& d1b,
                                   const uint8_t* desc2)
{
    Best2 res;
    unsigned long long best = ~0ull;
    int any = 0;
    for (int j = threadIdx.x; j < n; j += 64) {
        const int co = t.cell_oct[j];
        const int cell = (co & 0xFFFF) == 0xFFFF ? -1 : (co & 0xFFFF);
        if (!level_ok(lf, co >> 16)) continue;
        if (!in_area(q, cell, t.x[j], t.y[j], qx, qy, r)) continue;
        any = 1;
        if (t.taken[j] != -1) continue;
        uint4 a, b;
        load_desc(desc2 + (size_t)j * 32, a, b);
        const unsigned long long key = ((unsigned long long)hamming256(d1a, d1b, a, b) << 32) |
                                       ((unsigned long long)cell << 12) | (unsigned long long)j;
        best = key < best ? key : best;
    }
    res.any = __any(any);
    best = wave_min_u64(best);
    unsigned long long second = ~0ull;
    if (best != ~0ull) {
        const int bj = (int)(best & 0xFFF);
        for (int j = threadIdx.x; j < n; j += 64) {
            if (j == bj) continue;
            const int co = t.cell_oct[j];
            const int cell = (co & 0xFFFF) == 0xFFFF ? -1 : (co & 0xFFFF);
            if (!level_ok(lf, co >> 16)) continue;
            if (!in_area(q, cell, t.x[j], t.y[j], qx, qy, r)) continue;
            if (t.taken[j] != -1) continue;
            uint4 a, b;
            load_desc(desc2 + (size_t)j * 32, a, b);
            const unsigned long long key = ((unsigned long long)hamming256(d1a, d1b, a, b) << 32) |
                                           ((unsigned long long)cell << 12) | (unsigned long long)j;
            second = key < second ? key : second;
        }
        second = wave_min_u64(second);
    }
    res.best = best;
    res.second = second;
    return res;
}

__device__ inline int key_dist(unsigned long long k) { return k == ~0ull ? 0x7fffffff : (int)(k >> 32); }
__device__ inline int key_idx(unsigned long long k) { return k == ~0ull ? -1 : (int)(k & 0xFFF); }

// x3Dc = R * x3Dw + t in float, left-to-right sums; u = fx*xc*invzc + cx
// with invzc = 1.0/zc evaluated in double (src/ORBmatcher.cc:541-549).
__device__ inline void project(const float* T, const float* cam, const float* X, float* u, float* v, float* zc)
{
    float c[3];
#pragma unroll
    for (int r = 0; r < 3; r++)
        c[r] = __fadd_rn(__fadd_rn(__fadd_rn(__fmul_rn(T[4 * r], X[0]), __fmul_rn(T[4 * r + 1], X[1])),
                                   __fmul_rn(T[4 * r + 2], X[2])),
                         T[4 * r + 3]);
    const float invzc = (float)(1.0 / (double)c[2]);
    *u = __fadd_rn(__fmul_rn(__fmul_rn(cam[0], c[0]), invzc), cam[2]);
    *v = __fadd_rn(__fmul_rn(__fmul_rn(cam[1], c[1]), invzc), cam[3]);
    *zc = c[2];
}

// Rotation-consistency filter over entries pushed[i] = bin (or -1) of the
// keys listed in order; resets out[key[i]] when its bin is not a top-3 bin.
__device__ inline int rotation_filter(const signed char* bins, const int* keys, int npushed, int32_t* out,
                                      int* hist)
{
    int removed = 0;
    for (int b = 0; b < kHistoLength; b++) hist[b] = 0;
    for (int i = 0; i < npushed; i++) hist[bins[i]]++;
    int ind1, ind2, ind3;
    three_maxima(hist, ind1, ind2, ind3);
    for (int i = 0; i < npushed; i++) {
        const int b = bins[i];
        if (b == ind1 || b == ind2 || b == ind3) continue;
        out[keys[i]] = -1;
        removed++;
    }
    return removed;
}

struct SearchArgs {
    FrameDev F1, F2;              // query frame, searched frame
    const uint8_t* q_valid;       // per query
    const float* q_xyz;           // per query world point (projection searches)
    const uint8_t* f2_assigned;
    const float* prev_xy;         // SearchForInitialization
    float* prev_out;
    const float* proj_xy;         // local map
    const int32_t* pred_level;
    const float* view_cos;
    const uint8_t* q_desc;        // local map: map point descriptors
    int nq;
    float T[12];
    float cam[4];
    float scale[kMaxLevels];
    int window, min_level, max_level;
    float nnratio, th;
    int check_ori;
    int32_t* out;                 // result array
    int32_t* out_n;
    // Frame::isInFrustum inputs / outputs (local-map search from raw points)
    const float* mp_normal;       // n x 3
    const float* mp_dist;         // n x 2: min, max distance invariance
    const uint8_t* mp_skip;       // n or null
    float Rcw[9], tcw[3], Ow[3];
    float view_cos_limit;
    int nlevels;
    uint8_t* fr_in_view;          // n
    float* fr_proj;               // n x 2
    int32_t* fr_pred;             // n
    float* fr_cos;                // n
    int32_t* fr_count;            // points in view
    // frames resident in slots (orbx_track_frame): keypoint counts on the
    // device (F1.n / F2.n are then capacities)
    const int32_t* F1_cnt;
    const int32_t* F2_cnt;
};

// ORBmatcher::SearchByProjection(Frame& F, const vector<MapPoint*>&, float)
// (src/ORBmatcher.cc:49-125) with RadiusByViewingCos (:127-133).
__device__ inline void proj_local_wave(const SearchArgs& a, uint8_t* smem)
{
    CandTab t;
    carve_tab(smem, a.F2.n, t);
    fill_tab(a.F2, a.f2_assigned, t);
    const bool bFactor = a.th != 1.0f;
    int nmatches = 0;
    for (int m = 0; m < a.nq; m++) {
        if (!a.q_valid[m]) continue;
        const int pred = a.pred_level[m];
        float r = ((double)a.view_cos[m] > 0.998) ? 2.5f : 4.0f;
        if (bFactor) r = __fmul_rn(r, a.th);
        const float radius = __fmul_rn(r, a.scale[pred]);
        const float qx = a.proj_xy[2 * m], qy = a.proj_xy[2 * m + 1];
        const AreaQuery q = area_cells(a.F2, qx, qy, radius);
        if (q.empty) continue;
        uint4 d1a, d1b;
        load_desc(a.q_desc + (size_t)m * 32, d1a, d1b);
        const Best2 b = eval_query(t, a.F2.n, q, qx, qy, radius, level_filter(pred - 1, pred), d1a, d1b, a.F2.desc);
        if (!b.any) continue;
        const int bestDist = key_dist(b.best), bestDist2 = key_dist(b.second), bestIdx = key_idx(b.best);
        if (bestDist <= kTHHigh) {
            const int bestLevel = (t.cell_oct[bestIdx] >> 16);
            const int j2 = key_idx(b.second);
            const int bestLevel2 = j2 >= 0 ? (t.cell_oct[j2] >> 16) : -1;
            if (bestLevel == bestLevel2 && (float)bestDist > __fmul_rn(a.nnratio, (float)bestDist2)) continue;
            if (threadIdx.x == 0) {
                t.taken[bestIdx] = m;
                a.out[bestIdx] = m;
            }
            nmatches++;
            wave_sync();
        }
    }
    if (threadIdx.x == 0) *a.out_n = nmatches;
}

// ---------------------------------------------------------------------------
// Two-phase form of the greedy window / projection searches (the calls
// Tracking makes per frame: WindowSearch :409-516, SearchByProjection
// :1507-1620 (motion), :519-594 (pair), :49-125 (local map)).
//
// The one-wave kernels above scan every candidate of the searched frame for
// every query, twice, in the reference's sequential order: ~5 us per query.
// But the only state a query reads from the earlier ones is which candidates
// are taken (`if(F.mvpMapPoints[i2]) continue`).  So:
//  1. k_area_lists (state-free, one wave per query across the chip): the
//     query's area, level filter and candidate keys (distance, then
//     GetFeaturesInArea order: cell x, cell y, index) -- the list sorted
//     when it holds <= 64 keys, else in index order;
//  2. k_area_replay (one wave, sequential): per query the first two
//     admissible (untaken) keys of the sorted list -- one LDS lookup and
//     one ballot -- or wave minima over a longer list; a list that
//     overflowed its slot is evaluated in full as before.  Then each
//     search's own acceptance rule, the `taken` update and the rotation
//     filter, exactly as the one-wave kernels.
// Best and second are the same keys eval_query finds (the minimum key, and
// the minimum over the others), so the results are identical.
// ---------------------------------------------------------------------------
enum QueryKind { kQWindow = 0, kQPair = 1, kQMotion = 2, kQLocal = 3 };
constexpr int kAreaListWaves = 16;
constexpr int kAreaCap = 128;   // list entries per query (dist << 16 | index)

struct QuerySetup {
    bool active;
    float qx, qy, r;
    AreaQuery q;
    LevelFilter lf;
    const uint8_t* desc;
};

// The reference's per-query preamble of each search, up to
// GetFeaturesInArea.  nq: queries of the search.
template <int K>
__device__ inline int query_count(const SearchArgs& a)
{
    return K == kQLocal ? a.nq : (a.F1_cnt ? *a.F1_cnt : a.F1.n);
}

template <int K>
__device__ inline QuerySetup query_setup(const SearchArgs& a, int i)
{
    QuerySetup s;
    s.active = false;
    s.qx = s.qy = s.r = 0.f;
    s.desc = nullptr;
    if (!a.q_valid[i]) return s;
    if constexpr (K == kQWindow) {
        const orbx_keypoint k1 = a.F1.kps[i];
        const int level1 = k1.octave;
        if (a.min_level > 0 && level1 < a.min_level) return s;
        if (a.max_level < 0x7fffffff && level1 > a.max_level) return s;
        s.qx = k1.x;
        s.qy = k1.y;
        s.r = (float)a.window;
        s.lf = level_filter(level1, level1);
        s.desc = a.F1.desc + (size_t)i * 32;
    } else if constexpr (K == kQPair) {
        const int level1 = a.F1.kps[i].octave;
        float zc;
        project(a.T, a.cam, a.q_xyz + 3 * i, &s.qx, &s.qy, &zc);
        s.r = (float)a.window;
        s.lf = level_filter(level1, level1);
        s.desc = a.F1.desc + (size_t)i * 32;
    } else if constexpr (K == kQMotion) {
        float zc;
        project(a.T, a.cam, a.q_xyz + 3 * i, &s.qx, &s.qy, &zc);
        if (s.qx < a.F2.min_x || s.qx > a.F2.max_x) return s;
        if (s.qy < a.F2.min_y || s.qy > a.F2.max_y) return s;
        const int oct = a.F1.kps[i].octave;
        s.r = __fmul_rn(a.th, a.scale[oct]);
        s.lf = level_filter(oct - 1, oct + 1);
        s.desc = a.F1.desc + (size_t)i * 32;
    } else {
        const int pred = a.pred_level[i];
        float r = ((double)a.view_cos[i] > 0.998) ? 2.5f : 4.0f;
        if (a.th != 1.0f) r = __fmul_rn(r, a.th);
        s.r = __fmul_rn(r, a.scale[pred]);
        s.qx = a.proj_xy[2 * i];
        s.qy = a.proj_xy[2 * i + 1];
        s.lf = level_filter(pred - 1, pred);
        s.desc = a.q_desc + (size_t)i * 32;
    }
    s.q = area_cells(a.F2, s.qx, s.qy, s.r);
    s.active = !s.q.empty;
    return s;
}

// LDS of k_area_lists: per searched keypoint x, y and code (cx | cy << 8 |
// octave << 16, -1 outside the grid), then a 64-key sort buffer per wave
__host__ __device__ inline size_t area_lists_lds(int n2) { return (size_t)((n2 * 12 + 15) & ~15) + kAreaListWaves * 64 * 8; }

// grid.x: groups of kAreaListWaves queries; grid.y: job.  cnt[i]: -1 for a
// query the preamble skips, else its candidate count (admissible before
// `taken`; 0 = GetFeaturesInArea empty).
template <int K>
__global__ __launch_bounds__(kAreaListWaves * 64) void k_area_lists(const SearchArgs* jobs, int cap_q,
                                                                    uint32_t* lists_all, int32_t* cnt_all)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const SearchArgs& a = jobs[blockIdx.y];
    const int nq = query_count<K>(a);
    if ((int)blockIdx.x * kAreaListWaves >= nq) return;   // uniform
    if constexpr (K == kQLocal) {   // after k_frustum (fr_count set): no point in view, the replay skips the job
        if (a.fr_count && *a.fr_count == 0) return;
    }
    const FrameDev& F2 = a.F2;
    const int n2 = a.F2_cnt ? *a.F2_cnt : F2.n;
    float* sx = reinterpret_cast<float*>(smem);
    float* sy = sx + n2;
    int* scode = reinterpret_cast<int*>(sy + n2);
    unsigned long long* sortbuf = reinterpret_cast<unsigned long long*>(smem + ((n2 * 12 + 15) & ~15));
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    for (int j = tid; j < n2; j += kAreaListWaves * 64) {
        const orbx_keypoint k = F2.kps[j];
        const int cell = grid_cell(F2, k.x, k.y);
        sx[j] = k.x;
        sy[j] = k.y;
        scode[j] = cell < 0 ? -1 : ((cell / kGridRows) | ((cell % kGridRows) << 8) | (k.octave << 16));
    }
    __syncthreads();
    const int i = blockIdx.x * kAreaListWaves + wv;
    if (i >= nq) return;   // whole waves; no barrier below
    uint32_t* lists = lists_all + (size_t)blockIdx.y * cap_q * kAreaCap;
    int32_t* cnt = cnt_all + (size_t)blockIdx.y * cap_q;
    const QuerySetup s = query_setup<K>(a, i);
    int n = -1;
    if (s.active) {
        uint4 d1a, d1b;
        load_desc(s.desc, d1a, d1b);
        unsigned long long* sb = sortbuf + 64 * wv;
        uint32_t* out = lists + (size_t)i * kAreaCap;
        const unsigned long long lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
        n = 0;
        for (int j0 = 0; j0 < n2; j0 += 64) {
            const int j = j0 + lane;
            bool ok = false;
            int cx = 0, cy = 0;
            if (j < n2) {
                const int code = scode[j];
                cx = code & 0xFF;
                cy = (code >> 8) & 0xFF;
                ok = code >= 0 && level_ok(s.lf, code >> 16) && cx >= s.q.min_cx && cx <= s.q.max_cx &&
                     cy >= s.q.min_cy && cy <= s.q.max_cy && !(fabsf(__fsub_rn(sx[j], s.qx)) > s.r) &&
                     !(fabsf(__fsub_rn(sy[j], s.qy)) > s.r);
            }
            const unsigned long long bal = __ballot(ok);
            if (ok) {
                uint4 a2, b2;
                load_desc(F2.desc + (size_t)j * 32, a2, b2);
                const uint32_t dist = (uint32_t)hamming256(d1a, d1b, a2, b2);
                const int pos = n + __popcll(bal & lt_mask);
                if (pos < 64)
                    sb[pos] = ((unsigned long long)dist << 32) |
                              ((unsigned long long)(cx * kGridRows + cy) << 12) | (unsigned long long)j;
                if (pos < kAreaCap) out[pos] = dist << 16 | (uint32_t)j;   // index order
            }
            n += __popcll(bal);
        }
        if (n > 1 && n <= 64) {   // sorted by key: each lane's rank
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const unsigned long long mine = lane < n ? sb[lane] : ~0ull;
            int rank = 0;
            for (int k = 0; k < n; k++) {
                const unsigned long long o =
                    ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(mine >> 32), k) << 32) |
                    (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)mine, k);
                rank += o < mine;
            }
            if (lane < n) out[rank] = (uint32_t)(mine >> 32) << 16 | (uint32_t)(mine & 0xFFF);
        }
    }
    if (lane == 0) cnt[i] = n;
}

// The greedy resolution, in parallel rounds.  A query's result depends on
// the earlier queries only through the candidates they took, so with
//   R_t(i) = query i decided with the candidates that queries k < i took
//            in round t - 1 excluded (claim_{t-1}[j] < i),
//   claim_t[j] = the smallest query that takes j in round t,
// round t reproduces the sequential result for every query whose earlier
// queries were already right in round t - 1 (query 0 always is), and the
// rounds reach the sequential result -- its unique fixed point -- when no
// query changes.  Conflicts (two queries wanting one candidate) are rare, so
// that takes a few rounds of all queries at once instead of nq dependent
// steps of one wave; after kMaxRounds the sequential replay takes over.
//
// One workgroup per job (16 waves): the candidate table, the searched
// keypoints' angles, every query's count / short list (<= 64 keys, up to an
// LDS budget; the rest stay in global memory) and angle are staged first.
constexpr int kReplayThreads = 1024;
constexpr int kReplayWaves = kReplayThreads / 64;
constexpr int kReplayEntries = 8192;   // short-list entries staged in LDS (32 KB), at most
constexpr int kMaxRounds = 24;
// rounds used and sequential fallbacks, summed over replays (orbx_debug_area_rounds)
__device__ unsigned long long g_area_rounds[2];
// LDS: table (x, y, cell_oct, taken), bins, keys, hist, angles, two claim
// arrays; per query count, offset, angle, state (nq_lds of them: 0 when the
// per-query arrays live in global memory); ent_cap short-list entries
__host__ __device__ inline size_t area_replay_lds(int n2, int nq_lds, int ent_cap)
{
    return (size_t)n2 * 16 + ((n2 + 15) & ~15) + (size_t)n2 * 4 + 48 * 4 + (size_t)n2 * 4 + (size_t)n2 * 8 +
           (size_t)nq_lds * 20 + (size_t)ent_cap * 4;
}

// qglob: per job 5 cap_q ints (count, offset, angle, state, long-list
// queries) when the per-query arrays do not fit LDS (q_lds 0), else unused
template <int K>
__global__ __launch_bounds__(kReplayThreads) void k_area_replay(const SearchArgs* jobs, int cap_q,
                                                                const uint32_t* lists_all, const int32_t* cnt_all,
                                                                int q_lds, int ent_cap, int* qglob)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    __shared__ BlockScratchN<kReplayWaves> bs, bs2;
    __shared__ int s_changed[2], s_removed;
    const SearchArgs& a = jobs[blockIdx.x];
    if constexpr (K == kQLocal) {
        if (a.fr_count && *a.fr_count == 0) {
            if (threadIdx.x == 0) *a.out_n = 0;
            return;
        }
    }
    const int n2 = a.F2_cnt ? *a.F2_cnt : a.F2.n, nq = query_count<K>(a), tid = threadIdx.x, lane = tid & 63,
              wv = tid >> 6;
    CandTab t;
    carve_tab(smem, n2, t);
    signed char* bins = reinterpret_cast<signed char*>(t.taken + n2);
    int* keys = reinterpret_cast<int*>(bins + ((n2 + 15) & ~15));
    int* hist = keys + n2;
    float* ang2 = reinterpret_cast<float*>(hist + 48);
    int* claim0 = reinterpret_cast<int*>(ang2 + n2);
    int* claim1 = claim0 + n2;
    int* qbase = q_lds ? claim1 + n2 : qglob + (size_t)blockIdx.x * 5 * cap_q;
    int* q_cnt = qbase;
    int* q_off = q_cnt + cap_q;                                // entry offset of the short list, -1: global
    float* q_ang = reinterpret_cast<float*>(q_off + cap_q);
    int* q_state = reinterpret_cast<int*>(q_ang + cap_q);      // accepted candidate, or -1
    int* q_long = q_state + cap_q;                             // the queries with more than 64 candidates
    uint32_t* ent = reinterpret_cast<uint32_t*>(claim1 + n2 + (q_lds ? 5 * cap_q : 0));
    const uint32_t* lists = lists_all + (size_t)blockIdx.x * cap_q * kAreaCap;
    const int32_t* cnt = cnt_all + (size_t)blockIdx.x * cap_q;
    constexpr bool kRot = K == kQWindow || K == kQMotion;
    constexpr int kBig = 0x7fffffff;
    for (int i = tid; i < n2; i += kReplayThreads) {
        const orbx_keypoint k = a.F2.kps[i];
        ang2[i] = k.angle;
        t.x[i] = k.x;
        t.y[i] = k.y;
        const int cell = grid_cell(a.F2, k.x, k.y);
        t.cell_oct[i] = (cell & 0xFFFF) | (k.octave << 16);
        t.taken[i] = (a.f2_assigned && a.f2_assigned[i]) ? -2 : -1;
        claim0[i] = kBig;
    }
    // short lists into LDS: block prefix over the queries (in chunks of the
    // block), while the budget lasts
    int used = 0, nlong = 0;
    for (int q0 = 0; q0 < nq; q0 += kReplayThreads) {
        const int i = q0 + tid;
        const int c = i < nq ? cnt[i] : -1;
        const int w = (c > 0 && c <= 64) ? c : 0;
        int total, tl;
        const int off = used + block_exclusive_scan(w, &total, bs, (q0 / kReplayThreads) & 1);
        const int pl = nlong + block_exclusive_scan(c > 64 ? 1 : 0, &tl, bs2, (q0 / kReplayThreads) & 1);
        if (c > 64) q_long[pl] = i;
        nlong += tl;
        if (i < nq) {
            const bool fits = w > 0 && off + w <= ent_cap;
            q_cnt[i] = c;
            q_off[i] = fits ? off : -1;
            q_state[i] = -2;
            if (kRot) q_ang[i] = a.F1.kps[i].angle;
            if (fits) {
                const uint32_t* L = lists + (size_t)i * kAreaCap;
                for (int e = 0; e < w; e++) ent[off + e] = L[e];
            }
        }
        used = min(used + total, ent_cap);
    }
    __syncthreads();

    // best and second keys of query i (one wave) among the candidates with
    // is_free(j)
    auto best2 = [&](const int i, auto is_free, unsigned long long& best, unsigned long long& second) {
        best = ~0ull;
        second = ~0ull;
        const int c = q_cnt[i];
        if (c <= 64) {
            const int off = q_off[i];
            const uint32_t e = lane < c ? (off >= 0 ? ent[off + lane] : lists[(size_t)i * kAreaCap + lane]) : 0u;
            const int j = lane < c ? (int)(e & 0xFFFF) : 0;
            const bool adm = lane < c && is_free(j);
            const unsigned long long bal = __ballot(adm);
            if (bal) {
                const uint32_t e1 = (uint32_t)__builtin_amdgcn_readlane((int)e, __builtin_ctzll(bal));
                best = ((unsigned long long)(e1 >> 16) << 32) | (e1 & 0xFFFF);
                const unsigned long long bal2 = bal & (bal - 1);
                if (bal2) {
                    const uint32_t e2 = (uint32_t)__builtin_amdgcn_readlane((int)e, __builtin_ctzll(bal2));
                    second = ((unsigned long long)(e2 >> 16) << 32) | (e2 & 0xFFFF);
                }
            }
            return;
        }
        // longer lists: minima over full keys (distance, cell, index)
        unsigned long long b = ~0ull;
        if (c <= kAreaCap) {
            const uint32_t* L = lists + (size_t)i * kAreaCap;
            for (int k = lane; k < c; k += 64) {
                const uint32_t ek = L[k];
                const int j = (int)(ek & 0xFFFF);
                if (!is_free(j)) continue;
                const unsigned long long kk = ((unsigned long long)(ek >> 16) << 32) |
                                              ((unsigned long long)(t.cell_oct[j] & 0xFFFF) << 12) | (unsigned long long)j;
                b = kk < b ? kk : b;
            }
            best = wave_min_u64(b);
            if (best == ~0ull) return;
            b = ~0ull;
            for (int k = lane; k < c; k += 64) {
                const uint32_t ek = L[k];
                const int j = (int)(ek & 0xFFFF);
                if (j == key_idx(best) || !is_free(j)) continue;
                const unsigned long long kk = ((unsigned long long)(ek >> 16) << 32) |
                                              ((unsigned long long)(t.cell_oct[j] & 0xFFFF) << 12) | (unsigned long long)j;
                b = kk < b ? kk : b;
            }
            second = wave_min_u64(b);
            return;
        }
        // more candidates than the slot holds: every keypoint of the frame
        const QuerySetup s = query_setup<K>(a, i);
        uint4 d1a, d1b;
        load_desc(s.desc, d1a, d1b);
        for (int pass = 0; pass < 2; pass++) {
            b = ~0ull;
            for (int j = lane; j < n2; j += 64) {
                const int co = t.cell_oct[j];
                const int cell = (co & 0xFFFF) == 0xFFFF ? -1 : (co & 0xFFFF);
                if (!level_ok(s.lf, co >> 16)) continue;
                if (!in_area(s.q, cell, t.x[j], t.y[j], s.qx, s.qy, s.r)) continue;
                if (!is_free(j) || (pass == 1 && j == key_idx(best))) continue;
                uint4 a2, b2;
                load_desc(a.F2.desc + (size_t)j * 32, a2, b2);
                const unsigned long long kk = ((unsigned long long)hamming256(d1a, d1b, a2, b2) << 32) |
                                              ((unsigned long long)cell << 12) | (unsigned long long)j;
                b = kk < b ? kk : b;
            }
            b = wave_min_u64(b);
            if (pass == 0) {
                best = b;
                if (best == ~0ull) return;
            } else {
                second = b;
            }
        }
    };
    // each search's acceptance rule; returns the candidate taken, or -1
    auto decide = [&](const unsigned long long best, const unsigned long long second) {
        const int bestDist = key_dist(best), bestDist2 = key_dist(second), bestIdx = key_idx(best);
        bool accept;
        if constexpr (K == kQWindow || K == kQPair) {
            accept = (float)bestDist <= __fmul_rn((float)bestDist2, a.nnratio) && bestDist <= kTHHigh;
        } else if constexpr (K == kQMotion) {
            accept = bestDist <= kTHHigh;
        } else {
            accept = bestDist <= kTHHigh;
            if (accept) {
                const int bestLevel = (t.cell_oct[bestIdx] >> 16);
                const int j2 = key_idx(second);
                const int bestLevel2 = j2 >= 0 ? (t.cell_oct[j2] >> 16) : -1;
                if (bestLevel == bestLevel2 && (float)bestDist > __fmul_rn(a.nnratio, (float)bestDist2)) accept = false;
            }
        }
        return accept ? bestIdx : -1;
    };

    // parallel rounds: a thread per query with a short sorted list (the first
    // two free keys of the list), a wave per query with a longer one
    int* claim_prev = claim0;
    int* claim_next = claim1;
    bool converged = false;
    for (int round = 0; round < kMaxRounds; round++) {
        for (int j = tid; j < n2; j += kReplayThreads) claim_next[j] = kBig;
        // a flag per round parity: a thread still reading the last round's
        // flag must not see this round's reset
        if (tid == 0) s_changed[round & 1] = 0;
        __syncthreads();
        int changed = 0;
        for (int i = tid; i < nq; i += kReplayThreads) {
            const int c = q_cnt[i];
            if (c > 64) continue;
            int st = -1;
            if (c > 0) {
                const int off = q_off[i];
                const uint32_t* L = off >= 0 ? ent + off : lists + (size_t)i * kAreaCap;
                unsigned long long best = ~0ull, second = ~0ull;
                for (int k = 0; k < c; k++) {
                    const uint32_t e = L[k];
                    const int j = (int)(e & 0xFFFF);
                    if (t.taken[j] != -1 || claim_prev[j] < i) continue;
                    const unsigned long long kk = ((unsigned long long)(e >> 16) << 32) | (unsigned long long)j;
                    if (best == ~0ull) {
                        best = kk;
                    } else {
                        second = kk;
                        break;
                    }
                }
                st = decide(best, second);
            }
            changed |= st != q_state[i];
            q_state[i] = st;
            if (st >= 0) atomicMin(&claim_next[st], i);
        }
        for (int l = wv; l < nlong; l += kReplayWaves) {
            const int i = q_long[l];
            unsigned long long best, second;
            best2(i, [&](int j) { return t.taken[j] == -1 && claim_prev[j] >= i; }, best, second);
            const int st = decide(best, second);
            if (lane == 0) {
                changed |= st != q_state[i];
                q_state[i] = st;
                if (st >= 0) atomicMin(&claim_next[st], i);
            }
        }
        if (__any(changed) && lane == 0) s_changed[round & 1] = 1;
        __syncthreads();
        if (!s_changed[round & 1]) {
            if (tid == 0) atomicAdd(&g_area_rounds[0], (unsigned long long)(round + 1));
            converged = true;
            break;
        }
        int* tmp = claim_prev;
        claim_prev = claim_next;
        claim_next = tmp;
    }
    if (!converged && tid == 0) atomicAdd(&g_area_rounds[1], 1ull);
    if (!converged && tid < 64) {   // the sequential replay (taken: -1 free, >= 0 / -2 not)
        for (int i = 0; i < nq; i++) {
            int st = -1;
            if (q_cnt[i] > 0) {
                unsigned long long best, second;
                best2(i, [&](int j) { return t.taken[j] == -1; }, best, second);
                st = decide(best, second);
                if (st >= 0 && lane == 0) t.taken[st] = i;
            }
            if (lane == 0) q_state[i] = st;
            wave_sync();
        }
    }
    __syncthreads();
    // matches, rotation histogram (the reference pushes every match of
    // WindowSearch, and of the motion search with its check on; the filter
    // runs with the check on)
    const bool filter = kRot && a.check_ori;
    if (tid < 32) hist[tid] = 0;
    if (tid == 0) s_removed = 0;
    for (int j = tid; j < n2; j += kReplayThreads) keys[j] = -1;   // out of the searched keypoint
    __syncthreads();
    int acc = 0;
    for (int i = tid; i < nq; i += kReplayThreads) {
        const int st = q_state[i];
        if (st < 0) continue;
        acc++;
        keys[st] = i;
        if (filter) {
            const int b = rot_bin(q_ang[i], ang2[st]);
            bins[st] = (signed char)b;
            atomicAdd(&hist[b], 1);
        }
    }
    const int nacc = block_sum(acc, bs, 0);
    __syncthreads();
    if (filter && tid == 0) {
        int ind1, ind2, ind3;
        three_maxima(hist, ind1, ind2, ind3);
        hist[32] = ind1;
        hist[33] = ind2;
        hist[34] = ind3;
    }
    __syncthreads();
    int removed = 0;
    for (int j = tid; j < n2; j += kReplayThreads) {
        int m = keys[j];
        if (m >= 0 && filter) {
            const int b = bins[j];
            if (b != hist[32] && b != hist[33] && b != hist[34]) {
                m = -1;
                removed++;
            }
        }
        a.out[j] = m;
    }
    const int nrem = block_sum(removed, bs, 1);
    if (tid == 0) *a.out_n = nacc - nrem;
}

// Frame::isInFrustum (src/Frame.cc:136-197) for map point m of job a:
// Pc = mRcw*P + mtcw as OpenCV 2.4's small-matrix gemm evaluates it (float
// products summed left to right, + t); invz = 1.0/PcZ in double; cv::norm
// and Mat::dot of the float vectors accumulated in double.  Every float
// operation rounded on its own (ISO evaluation, -ffp-contract=off).
__device__ inline void frustum_point(const SearchArgs& a, int m)
{
    uint8_t in = 0;
    float u = 0.f, v = 0.f, vc = 0.f;
    int pred = 0;
    if (!(a.mp_skip && a.mp_skip[m])) {
        const float P[3] = {a.q_xyz[3 * m], a.q_xyz[3 * m + 1], a.q_xyz[3 * m + 2]};
        float Pc[3];
#pragma unroll
        for (int r = 0; r < 3; r++)
            Pc[r] = __fadd_rn(__fadd_rn(__fadd_rn(__fmul_rn(a.Rcw[3 * r], P[0]), __fmul_rn(a.Rcw[3 * r + 1], P[1])),
                                        __fmul_rn(a.Rcw[3 * r + 2], P[2])),
                              a.tcw[r]);
        if (!(Pc[2] < 0.0f)) {
            const float invz = (float)(1.0 / (double)Pc[2]);
            u = __fadd_rn(__fmul_rn(__fmul_rn(a.cam[0], Pc[0]), invz), a.cam[2]);
            v = __fadd_rn(__fmul_rn(__fmul_rn(a.cam[1], Pc[1]), invz), a.cam[3]);
            if (!(u < a.F2.min_x || u > a.F2.max_x || v < a.F2.min_y || v > a.F2.max_y)) {
                const float minD = a.mp_dist[2 * m], maxD = a.mp_dist[2 * m + 1];
                const float PO[3] = {__fsub_rn(P[0], a.Ow[0]), __fsub_rn(P[1], a.Ow[1]), __fsub_rn(P[2], a.Ow[2])};
                double s2 = 0.0;
#pragma unroll
                for (int i = 0; i < 3; i++) s2 = __dadd_rn(s2, __dmul_rn((double)PO[i], (double)PO[i]));
                const float dist = (float)__dsqrt_rn(s2);
                if (!(dist < minD || dist > maxD)) {
                    const float* Pn = a.mp_normal + 3 * m;
                    double d = 0.0;
#pragma unroll
                    for (int i = 0; i < 3; i++) d = __dadd_rn(d, __dmul_rn((double)PO[i], (double)Pn[i]));
                    vc = (float)__ddiv_rn(d, (double)dist);
                    if (!(vc < a.view_cos_limit)) {
                        const float ratio = __fdiv_rn(dist, minD);
                        // lower_bound(mvScaleFactors, ratio), clamped to the last level
                        pred = 0;
                        while (pred < a.nlevels && a.scale[pred] < ratio) pred++;
                        if (pred >= a.nlevels) pred = a.nlevels - 1;
                        in = 1;
                    }
                }
            }
        }
    }
    a.fr_in_view[m] = in;
    if (in) {
        a.fr_proj[2 * m] = u;
        a.fr_proj[2 * m + 1] = v;
        a.fr_pred[m] = pred;
        a.fr_cos[m] = vc;
    } else {
        a.fr_proj[2 * m] = 0.f;
        a.fr_proj[2 * m + 1] = 0.f;
        a.fr_pred[m] = 0;
        a.fr_cos[m] = 0.f;
    }
    const unsigned long long b = __ballot(in);
    if (__lane_id() == 0 && b) atomicAdd(a.fr_count, (int)__popcll(b));
}

// One thread per local map point; grid.y = job (independent frames).
__global__ __launch_bounds__(256) void k_frustum(const SearchArgs* jobs)
{
    const SearchArgs& a = jobs[blockIdx.y];
    const int m = blockIdx.x * 256 + threadIdx.x;
    // a wave's lane 0 holds its smallest index, so lane 0 is active
    // whenever any lane is (the in-view count is added by lane 0)
    if (m < a.nq) frustum_point(a, m);
}

// SearchByProjection(F, local map) per job after k_frustum: one wavefront per
// frame, skipped when no point is in view (`if(nToMatch>0)`,
// src/Tracking.cc:742).
__global__ __launch_bounds__(64) void k_proj_local_jobs(const SearchArgs* jobs)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const SearchArgs& a = jobs[blockIdx.x];
    if (*a.fr_count == 0) {
        if (threadIdx.x == 0) *a.out_n = 0;
        return;
    }
    proj_local_wave(a, smem);
}

// SearchForInitialization with host inputs (prev_xy in/out), one pair, in
// two launches: k_sfi_lists builds every query's candidate list across the
// chip (one wave per F1 octave-0 keypoint, 16 per workgroup), then one
// workgroup of kInitOneThreads copies them into LDS and replays the greedy
// assignment (one wave; the rest stage and finish).
constexpr int kInitOneThreads = 1024;
constexpr int kListWaves = 16;

// LDS of k_sfi_lists: candidate records and descriptors (cap_c each) and a
// 64-key sort buffer per wave
__host__ __device__ inline size_t sfi_lists_lds(int cap_c) { return (size_t)cap_c * 48 + kListWaves * 64 * 4; }

__global__ __launch_bounds__(kListWaves * 64) void k_sfi_lists(SearchArgs a, int cap_c, int n1q, uint32_t* keys,
                                                               int32_t* cnt)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    __shared__ BlockScratchN<kListWaves> bs;
    InitLDS s{};
    s.desc = reinterpret_cast<uint4*>(smem);
    s.rec = reinterpret_cast<float4*>(s.desc + 2 * cap_c);
    uint32_t* sortbuf = reinterpret_cast<uint32_t*>(s.rec + cap_c);
    s.cap_c = cap_c;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const FrameDev& F2 = a.F2;
    // F2 octave-0 keypoints in index order -> candidate slots (as
    // search_for_init_block stages them)
    int nc = 0;
    for (int base = 0; base < F2.n; base += kListWaves * 64) {
        const int i2 = base + tid;
        orbx_keypoint k;
        bool ok = false;
        if (i2 < F2.n) {
            k = F2.kps[i2];
            ok = (k.octave == 0);
        }
        int tot;
        const int pos = nc + block_exclusive_scan(ok ? 1 : 0, &tot, bs, (base / (kListWaves * 64)) & 1);
        if (ok && pos < cap_c) {
            const int cell = grid_cell(F2, k.x, k.y);
            s.rec[pos] = make_float4(k.x, k.y, __int_as_float(cell < 0 ? -1 : ((cell / kGridRows) | ((cell % kGridRows) << 8))),
                                     __int_as_float(cell));
            const uint4* d = reinterpret_cast<const uint4*>(F2.desc + (size_t)i2 * 32);
            s.desc[2 * pos] = d[0];
            s.desc[2 * pos + 1] = d[1];
        }
        nc += tot;
    }
    __syncthreads();
    nc = min(nc, cap_c);   // the replay kernel reports an overflow
    const int i1 = blockIdx.x * kListWaves + wv;
    if (i1 >= n1q) return;   // whole waves; no barrier below
    const orbx_keypoint k1 = a.F1.kps[i1];
    int n = 0;
    int4 qa = make_int4(1, 0, 1, 0);
    float2 qp = make_float2(0.f, 0.f);
    const float r = (float)a.window;
    if (k1.octave == 0) {
        qp = make_float2(a.prev_xy[2 * i1], a.prev_xy[2 * i1 + 1]);
        const AreaQuery q = area_cells(F2, qp.x, qp.y, r);
        if (!q.empty) qa = make_int4(q.min_cx, q.max_cx, q.min_cy, q.max_cy);
        n = sfi_query_count(s, nc, qa, qp, r, lane);
    }
    if (n > 0) {
        uint4 d1a, d1b;
        load_desc(a.F1.desc + (size_t)i1 * 32, d1a, d1b);
        uint32_t* out = keys + (size_t)i1 * cap_c;
        if (n <= 64) {   // sorted through this wave's LDS buffer
            uint32_t* sb = sortbuf + 64 * wv;
            sfi_query_fill(s, nc, qa, qp, d1a, d1b, r, sb, lane);
            sfi_sort_short(sb, out, n, lane);
        } else {
            sfi_query_fill(s, nc, qa, qp, d1a, d1b, r, out, lane);
        }
    }
    if (lane == 0) cnt[i1] = n;
}

__global__ __launch_bounds__(kInitOneThreads) void k_search_init_one(SearchArgs a, int cap_c, int cap_keys,
                                                                      int32_t* error_flags, const uint32_t* keys,
                                                                      const int32_t* cnt)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    __shared__ BlockScratchN<kInitOneThreads / 64> bs;
    const InitLDS L = carve_init(smem, cap_c, max(a.F1.n, 1), cap_keys);
    search_for_init_block<kInitOneThreads, true>(a.F1, a.F2, a.prev_xy, a.window, a.nnratio, a.check_ori != 0,
                                                 a.out, a.out_n, a.prev_out, L, bs, error_flags, keys, cnt);
}

// ---------------------------------------------------------------------------
// All-pairs Hamming (B8): one thread per query row, B streamed through LDS
// in chunks of 256 descriptors; ascending b with strict `<` keeps the
// reference's first-index tie rule.  grid.y indexes independent pairs.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_hamming_bf(const uint8_t* dA, int nA, const uint8_t* dB, int nB,
                                                    int32_t* best_idx, int32_t* best, int32_t* second,
                                                    int32_t* m12, int th_low, float nnratio)
{
    __shared__ uint4 sb[256][2];
    const int a = blockIdx.x * 256 + threadIdx.x;
    uint4 qa = make_uint4(0, 0, 0, 0), qb = qa;
    if (a < nA) load_desc(dA + (size_t)a * 32, qa, qb);
    int b1 = 0x7fffffff, b2 = 0x7fffffff, bi = -1;
    for (int base = 0; base < nB; base += 256) {
        __syncthreads();
        const int j = base + threadIdx.x;
        if (j < nB) load_desc(dB + (size_t)j * 32, sb[threadIdx.x][0], sb[threadIdx.x][1]);
        __syncthreads();
        const int cnt = min(256, nB - base);
        for (int k = 0; k < cnt; k++) {
            const int d = hamming256(qa, qb, sb[k][0], sb[k][1]);
            if (d < b1) {
                b2 = b1;
                b1 = d;
                bi = base + k;
            } else if (d < b2) {
                b2 = d;
            }
        }
    }
    if (a < nA) {
        best_idx[a] = bi;
        best[a] = b1;
        second[a] = b2;
        // C3 acceptance: best <= TH_LOW and best < nnratio * second
        if (m12) m12[a] = (b1 <= th_low && (float)b1 < __fmul_rn((float)b2, nnratio)) ? bi : -1;
    }
}

// ---------------------------------------------------------------------------
// The tracking chain's glue (orbx_track_frame): one 1024-thread workgroup
// between the searches and the PoseOptimization launches, reading and writing
// the chain's state in device memory (no host round trip).
// ---------------------------------------------------------------------------
struct TrackOut {
    float T[12];
    int n_cur, status, n_motion, n_pair, n_after_pose, n_in_view, n_local, n_inliers, err, pad[3];
};

struct TrackDev {
    const orbx_keypoint* cur_kps;   // the current frame's slot
    const int32_t* cur_cnt;
    const int32_t* last_mp;
    const uint8_t* last_outlier;
    int n_last, n_mp, n_local, cap; // n_last: entries of last_mp / last_outlier; n_local: frustum search's points
    const int32_t* last_cnt;        // LastFrame in a slot: its keypoint count (else null)
    const int32_t* err;             // the context's error flags (read back with the outputs)
    const float* mp_pos;
    const uint8_t* mp_skip_in;      // or null
    const float* isig;
    float Tpred[12], cam[4];
    float* q_xyz;                   // motion search queries (last frame's points)
    uint8_t* q_valid;
    const int32_t* motion_out;      // k_area_replay<kQMotion>: last-frame index per current keypoint
    const int32_t* motion_n;
    int32_t* motion_out_w;          // the same, initialised by stage 0
    int32_t* motion_n_w;
    int32_t* local_out_w;           // the local search's, initialised by stage 2
    int32_t* local_n_w;
    const int32_t* local_out;       // k_area_replay<kQLocal>: local-map index per current keypoint
    const int32_t* local_n;
    int32_t* cur_mp;
    uint8_t* f_assigned;
    uint8_t* mp_skip;
    SearchArgs* local_job;
    PoseHdr* hdr;                   // 3 problems: before the local map, after it, TrackPreviousFrame's first
    float* edges;                   // 6 arrays x 3 cap
    int32_t* edge_kp;               // 3 cap
    const uint8_t* flags;           // 3 cap (k_pose_opt's outlier flags)
    const PoseOut* pout;            // 3
    int32_t* st;                    // status, matches before pose 0, left after it, first search's, pair's
    // TrackPreviousFrame (mode 1): the two WindowSearch jobs and the pair
    // search's, their outputs, the window and pair queries' validity
    int mode, min_octave;
    SearchArgs* win_job[2];
    SearchArgs* pair_job;
    int32_t* win_out[2];
    int32_t* win_n[2];
    int32_t* pair_out;
    int32_t* pair_n;
    uint8_t* w_valid;
    uint8_t* p_valid;
    TrackOut* out;                  // read-back block: TrackOut, cur_mp[cap], cur_outlier[cap]
};

constexpr int kTrackThreads = 1024;

// PoseOptimization problem p from the current matches (edges in keypoint
// order: g2o's insertion order, src/Optimizer.cc:187-231), initial pose T
template <int kT>
__device__ inline void track_build_pose(const TrackDev& d, int p, const float* T, bool run, int n,
                                        BlockScratchN<kT / 64>& bs)
{
    const int tid = threadIdx.x;
    float* ox = d.edges;
    const size_t arr = (size_t)3 * d.cap;
    int base = 0;
    for (int c0 = 0; c0 < n; c0 += kT) {
        const int i = c0 + tid;
        const int m = (run && i < n) ? d.cur_mp[i] : -1;
        int tot;
        const int pos = base + block_exclusive_scan(m >= 0 ? 1 : 0, &tot, bs, (c0 / kT) & 1);
        if (m >= 0) {
            const size_t e = (size_t)p * d.cap + pos;
            const orbx_keypoint k = d.cur_kps[i];
            ox[e] = k.x;
            ox[arr + e] = k.y;
            ox[2 * arr + e] = d.isig[k.octave];
            ox[3 * arr + e] = d.mp_pos[3 * m];
            ox[4 * arr + e] = d.mp_pos[3 * m + 1];
            ox[5 * arr + e] = d.mp_pos[3 * m + 2];
            d.edge_kp[e] = i;
        }
        base += tot;
    }
    if (tid == 0) {
        PoseHdr& h = d.hdr[p];
        h.e0 = (long long)p * d.cap;
        h.nE = base;
        h.pad = 0;
        for (int k = 0; k < 12; k++) h.T[k] = T[k];
        for (int k = 0; k < 4; k++) h.cam[k] = d.cam[k];
    }
}

// stage 0: motion queries; 1: after the motion search; 2: after the first
// PoseOptimization; 3: after the local-map search; 4: outputs
__global__ __launch_bounds__(kTrackThreads) void k_track_stage(TrackDev d, int stage)
{
    __shared__ BlockScratchN<kTrackThreads / 64> bs;
    __shared__ int s_cnt;
    const int tid = threadIdx.x;
    const int n = *d.cur_cnt;
    if (stage == 0) {
        const int nl = d.last_cnt ? min(*d.last_cnt, d.n_last) : d.n_last;
        for (int i = tid; i < d.n_last; i += kTrackThreads) {
            const int m = i < nl ? d.last_mp[i] : -1;
            const bool v = m >= 0 && m < d.n_mp && !d.last_outlier[i];
            d.q_valid[i] = v;
            d.q_xyz[3 * i] = v ? d.mp_pos[3 * m] : 0.f;
            d.q_xyz[3 * i + 1] = v ? d.mp_pos[3 * m + 1] : 0.f;
            d.q_xyz[3 * i + 2] = v ? d.mp_pos[3 * m + 2] : 0.f;
        }
        // SearchByProjection's outputs; the current frame's mvpMapPoints are
        // cleared (src/Tracking.cc:581), nothing is assigned yet
        for (int i = tid; i < d.cap; i += kTrackThreads) {
            d.motion_out_w[i] = -1;
            d.f_assigned[i] = 0;
        }
        if (tid == 0) {
            d.st[0] = d.st[1] = d.st[2] = 0;
            *d.motion_n_w = 0;
        }
        return;
    }
    const int status = d.st[0];
    if (stage == 10) {
        // TrackPreviousFrame (src/Tracking.cc:497-569): WindowSearch queries
        // are the last frame's points that are not bad (no outlier test,
        // src/ORBmatcher.cc:424-430); all outputs cleared
        const int nl = d.last_cnt ? min(*d.last_cnt, d.n_last) : d.n_last;
        for (int i = tid; i < d.n_last; i += kTrackThreads) {
            const int m = i < nl ? d.last_mp[i] : -1;
            d.w_valid[i] = m >= 0 && m < d.n_mp && !(d.mp_skip_in && d.mp_skip_in[m]);
        }
        for (int i = tid; i < d.cap; i += kTrackThreads) {
            d.win_out[0][i] = d.win_out[1][i] = d.pair_out[i] = -1;
            d.f_assigned[i] = 0;
        }
        if (tid == 0) {
            for (int k = 0; k < 5; k++) d.st[k] = 0;
            *d.win_n[0] = *d.win_n[1] = *d.pair_n = 0;
        }
        return;
    }
    if (stage == 11) {   // < 10: WindowSearch(100) without the scale constraint (:514-517)
        // (F1.n is the window kind's query count: 0 makes the launch a no-op)
        if (tid == 0 && *d.win_n[0] >= 10) d.win_job[1]->F1.n = 0;
        return;
    }
    if (stage == 12) {
        // the window matches taken (< 10 after both: none, :518-522);
        // mCurrentFrame.mTcw = mLastFrame.mTcw; >= 10: PoseOptimization
        const int n0 = *d.win_n[0], n1 = *d.win_n[1];
        const int src = n0 >= 10 ? 0 : (n1 >= 10 ? 1 : -1);
        const int nm = src < 0 ? 0 : (src == 0 ? n0 : n1);
        for (int i = tid; i < n; i += kTrackThreads) {
            const int m = src < 0 ? -1 : d.win_out[src][i];
            d.cur_mp[i] = m >= 0 ? d.last_mp[m] : -1;
        }
        __syncthreads();
        track_build_pose<kTrackThreads>(d, 2, d.Tpred, nm >= 10, n, bs);
        if (tid == 0) {
            d.st[1] = nm;
            d.st[3] = nm;
        }
        return;
    }
    if (stage == 13) {
        // >= 10: outliers discarded, SearchByProjection(last, current, 15) at
        // the optimised pose; else (none kept) at mLastFrame.mTcw with 50
        // (:531-547).  Its queries: the last frame's points that are not bad
        // and not already among the current frame's (:530-534); candidates:
        // the current keypoints without a point
        const int nm = d.st[1];
        const bool posed = nm >= 10;
        if (tid == 0) s_cnt = 0;
        for (int m = tid; m < d.n_mp; m += kTrackThreads) d.mp_skip[m] = 0;   // "already found" set
        __syncthreads();
        int nout = 0;
        if (posed) {
            const int nE = d.hdr[2].nE;
            for (int e = tid; e < nE; e += kTrackThreads)
                if (d.flags[(size_t)2 * d.cap + e]) {
                    d.cur_mp[d.edge_kp[(size_t)2 * d.cap + e]] = -1;
                    nout++;
                }
            if (nout) atomicAdd(&s_cnt, nout);
        }
        __syncthreads();
        for (int i = tid; i < d.cap; i += kTrackThreads) {
            const int m = i < n ? d.cur_mp[i] : -1;
            d.f_assigned[i] = m >= 0;
            if (m >= 0) d.mp_skip[m] = 1;
        }
        __syncthreads();
        const int nl = d.last_cnt ? min(*d.last_cnt, d.n_last) : d.n_last;
        for (int i = tid; i < d.n_last; i += kTrackThreads) {
            const int m = i < nl ? d.last_mp[i] : -1;
            const bool v = d.w_valid[i] && !d.mp_skip[m];
            d.p_valid[i] = v;
            d.q_xyz[3 * i] = v ? d.mp_pos[3 * m] : 0.f;
            d.q_xyz[3 * i + 1] = v ? d.mp_pos[3 * m + 1] : 0.f;
            d.q_xyz[3 * i + 2] = v ? d.mp_pos[3 * m + 2] : 0.f;
        }
        if (tid == 0) {
            SearchArgs& j = *d.pair_job;
            const float* T = posed ? d.pout[2].T : d.Tpred;
            for (int k = 0; k < 12; k++) j.T[k] = T[k];
            j.window = posed ? 15 : 50;
            d.st[1] = posed ? nm - s_cnt : 0;   // nmatches before the pair search
        }
        return;
    }
    if (stage == 14) {
        // the pair search's matches added (vpMapPointMatches, :548); < 10:
        // fail; else PoseOptimization from the pose the search used (:553-556)
        for (int i = tid; i < n; i += kTrackThreads) {
            const int m = d.pair_out[i];
            if (m >= 0) d.cur_mp[i] = d.last_mp[m];
        }
        const int np = *d.pair_n, total = d.st[1] + np;
        __syncthreads();
        track_build_pose<kTrackThreads>(d, 0, d.pair_job->T, total >= 10, n, bs);
        if (tid == 0) {
            d.st[4] = np;
            d.st[1] = total;
            d.st[0] = total >= 10 ? 0 : 3;
        }
        return;
    }
    if (stage == 1) {
        // mvpMapPoints of the current frame = the last frame's points found
        // (src/ORBmatcher.cc:1575); < 20 matches: TrackWithMotionModel fails
        for (int i = tid; i < n; i += kTrackThreads) {
            const int m = d.motion_out[i];
            d.cur_mp[i] = m >= 0 ? d.last_mp[m] : -1;
        }
        const int nm = *d.motion_n;
        const bool run = nm >= 20;
        __syncthreads();
        track_build_pose<kTrackThreads>(d, 0, d.Tpred, run, n, bs);
        if (tid == 0) {
            d.st[0] = run ? 0 : 1;
            d.st[1] = nm;
        }
        return;
    }
    if (stage == 2) {
        // discard the outliers (src/Tracking.cc:592-603); < 10 left: fail
        if (tid == 0) s_cnt = 0;
        __syncthreads();
        int nout = 0;
        if (status == 0) {
            const int nE = d.hdr[0].nE;
            for (int e = tid; e < nE; e += kTrackThreads)
                if (d.flags[e]) {
                    d.cur_mp[d.edge_kp[e]] = -1;
                    nout++;
                }
            if (nout) atomicAdd(&s_cnt, nout);
        }
        __syncthreads();
        const int left = d.st[1] - s_cnt;
        const bool ok = status == 0 && left >= 10;
        // SearchReferencePointsInFrustum (src/Tracking.cc:701-752) with the
        // pose just found: points matched already are not projected
        for (int m = tid; m < d.n_mp; m += kTrackThreads) d.mp_skip[m] = d.mp_skip_in ? d.mp_skip_in[m] : 0;
        for (int i = tid; i < d.cap; i += kTrackThreads) {
            d.f_assigned[i] = 0;
            d.local_out_w[i] = -1;
        }
        __syncthreads();
        // matched points: bad ones are dropped, the others marked seen
        // (mnLastFrameSeen, src/Tracking.cc:704-718)
        if (ok)
            for (int i = tid; i < n; i += kTrackThreads) {
                const int m = d.cur_mp[i];
                if (m < 0) continue;
                if (d.mp_skip_in && d.mp_skip_in[m]) {
                    d.cur_mp[i] = -1;
                } else {
                    d.f_assigned[i] = 1;
                    d.mp_skip[m] = 1;
                }
            }
        if (tid == 0) {
            *d.local_n_w = 0;
            SearchArgs& j = *d.local_job;
            *j.fr_count = 0;
            j.nq = ok ? d.n_local : 0;
            if (ok) {
                // Frame::UpdatePoseMatrices (src/Frame.cc:129-134): Rcw, tcw,
                // Ow = -Rcw^T tcw (float, left to right)
                const float* T = d.pout[0].T;
                for (int r = 0; r < 3; r++) {
                    for (int c = 0; c < 3; c++) j.Rcw[3 * r + c] = T[4 * r + c];
                    j.tcw[r] = T[4 * r + 3];
                }
                for (int c = 0; c < 3; c++)
                    j.Ow[c] = -__fadd_rn(__fadd_rn(__fmul_rn(T[c], T[3]), __fmul_rn(T[4 + c], T[7])),
                                         __fmul_rn(T[8 + c], T[11]));
            }
            d.st[0] = status != 0 ? status : (ok ? 0 : (d.mode ? 4 : 2));
            d.st[2] = left;
        }
        return;
    }
    if (stage == 3) {
        // the local-map matches join the frame's (SearchByProjection writes
        // F.mvpMapPoints, src/ORBmatcher.cc:115); PoseOptimization again from
        // the pose found (src/Tracking.cc:627)
        const bool ok = status == 0;
        if (ok && *d.local_job->fr_count > 0)
            for (int i = tid; i < n; i += kTrackThreads) {
                const int m = d.local_out[i];
                if (m >= 0) d.cur_mp[i] = m;
            }
        __syncthreads();
        track_build_pose<kTrackThreads>(d, 1, d.pout[0].T, ok, n, bs);
        return;
    }
    // stage 4: outputs of the last PoseOptimization that ran
    int32_t* cur_mp_out = reinterpret_cast<int32_t*>(d.out + 1);
    uint8_t* cur_out = reinterpret_cast<uint8_t*>(cur_mp_out + d.cap);
    for (int i = tid; i < d.cap; i += kTrackThreads) {
        cur_mp_out[i] = i < n ? d.cur_mp[i] : -1;
        cur_out[i] = 0;
    }
    __syncthreads();
    if (status == 0) {
        const int nE = d.hdr[1].nE;
        for (int e = tid; e < nE; e += kTrackThreads) cur_out[d.edge_kp[(size_t)d.cap + e]] = d.flags[(size_t)d.cap + e];
    }
    if (tid == 0) {
        TrackOut& o = *d.out;
        // the pose of the last PoseOptimization that ran (status 3: the pair
        // search's pose, i.e. the first one's or mLastFrame.mTcw)
        const float* T = status == 0 ? d.pout[1].T
                         : (status == 2 || status == 4) ? d.pout[0].T
                         : status == 3 ? d.pair_job->T : d.Tpred;
        for (int k = 0; k < 12; k++) o.T[k] = T[k];
        o.n_cur = n;
        o.status = status;
        o.n_motion = d.mode ? d.st[3] : d.st[1];
        o.n_pair = d.mode ? d.st[4] : 0;
        o.n_after_pose = (status == 0 || status == 2 || status == 4) ? d.st[2] : 0;
        o.n_in_view = status == 0 ? *d.local_job->fr_count : 0;
        o.n_local = (status == 0 && *d.local_job->fr_count > 0) ? *d.local_n : 0;
        o.n_inliers = status == 0 ? d.pout[1].n_inliers : (status == 2 || status == 4) ? d.pout[0].n_inliers : 0;
        o.pad[0] = o.pad[1] = o.pad[2] = 0;
        o.err = *d.err;
    }
}

// ---------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------
namespace {

struct Uploader {
    orbx_ctx* ctx;
    std::vector<std::pair<size_t, size_t>> parts;   // offset, bytes
    size_t total = 0;
    size_t reserve(size_t bytes)
    {
        const size_t off = total;
        total += (bytes + 255) & ~size_t(255);
        return off;
    }
    uint8_t* base() const { return static_cast<uint8_t*>(ctx->scratch); }
};

// One call's device block staged through the context's page-locked buffer:
// inputs (and initialised outputs) are written at their device offsets into
// the pinned copy and go over in ONE copy, the outputs come back in ONE copy
// from out_begin -- instead of a copy per array, each of which costs a
// DMA setup (and, from pageable memory, a staging kernel).
struct Pinned {
    orbx_ctx* ctx;
    uint8_t* h = nullptr;
    int open(size_t total)
    {
        const int r = ensure_pinned(ctx, total);
        h = static_cast<uint8_t*>(ctx->host_pinned);
        return r;
    }
    void put(size_t off, const void* src, size_t bytes)
    {
        if (bytes && src) std::memcpy(h + off, src, bytes);
    }
    void fill(size_t off, int v, size_t bytes) { std::memset(h + off, v, bytes); }
    int upload(size_t bytes)
    {
        ORBX_HIP_CHECK(hipMemcpyAsync(ctx->scratch, h, bytes, hipMemcpyHostToDevice, ctx->stream));
        return ORBX_OK;
    }
    int download(size_t begin, size_t end)
    {
        ORBX_HIP_CHECK(hipMemcpyAsync(h + begin, static_cast<uint8_t*>(ctx->scratch) + begin, end - begin,
                                      hipMemcpyDeviceToHost, ctx->stream));
        ORBX_HIP_CHECK(hipStreamSynchronize(ctx->stream));
        return ORBX_OK;
    }
    void get(void* dst, size_t off, size_t bytes) const
    {
        if (bytes && dst) std::memcpy(dst, h + off, bytes);
    }
};

bool valid_view(const orbx_frame_view* v)
{
    return v && v->n >= 0 && v->n <= kMaxFeatures && (v->n == 0 || (v->keys_un && v->desc)) && v->max_x > v->min_x &&
           v->max_y > v->min_y && v->nlevels > 0 && v->nlevels <= kMaxLevels;
}

FrameDev dev_frame(const orbx_frame_view* v, const uint8_t* base, size_t kp_off, size_t desc_off)
{
    FrameDev F;
    F.kps = reinterpret_cast<const orbx_keypoint*>(base + kp_off);
    F.desc = base + desc_off;
    F.n = v->n;
    F.min_x = v->min_x;
    F.max_x = v->max_x;
    F.min_y = v->min_y;
    F.max_y = v->max_y;
    // src/Frame.cc:76-77: FRAME_GRID_COLS / (mnMaxX - mnMinX) in float
    F.grid_w_inv = static_cast<float>(kGridCols) / (v->max_x - v->min_x);
    F.grid_h_inv = static_cast<float>(kGridRows) / (v->max_y - v->min_y);
    return F;
}

void frame_scales(const orbx_frame_view* v, float* s)
{
    s[0] = 1.0f;
    for (int i = 1; i < v->nlevels; i++) s[i] = s[i - 1] * v->scale_factor;   // src/Frame.cc:98-102
}

// Uploads a frame view; returns offsets.
struct FrameOffs { size_t kp, desc; };

FrameOffs reserve_frame(Uploader& u, const orbx_frame_view* v)
{
    FrameOffs o;
    o.kp = u.reserve((size_t)v->n * sizeof(orbx_keypoint));
    o.desc = u.reserve((size_t)v->n * 32);
    return o;
}

void put_frame(Pinned& pin, const FrameOffs& o, const orbx_frame_view* v)
{
    pin.put(o.kp, v->keys_un, (size_t)v->n * sizeof(orbx_keypoint));
    pin.put(o.desc, v->desc, (size_t)v->n * 32);
}

size_t tab_lds(int n) { return (size_t)n * 16 + ((n + 15) & ~15) + (size_t)n * 4 + 32 * 4 + 64; }

// Device space of the two-phase searches' candidate lists: B jobs of up to
// nq queries (reserved after the read-back range; never copied).
struct AreaBufs {
    size_t lists, cnt, qglob;
};
AreaBufs reserve_area(Uploader& u, int B, int nq)
{
    AreaBufs o;
    o.lists = u.reserve((size_t)B * std::max(nq, 1) * kAreaCap * 4);
    o.cnt = u.reserve((size_t)B * std::max(nq, 1) * 4);
    o.qglob = u.reserve((size_t)B * std::max(nq, 1) * 16);
    return o;
}

// The two launches of a search of kind K over B jobs whose SearchArgs are
// in device memory at dj (nq_max queries, n2_max searched keypoints at most).
template <int K>
int launch_area_search(orbx_ctx* ctx, const SearchArgs* dj, int B, int nq_max, int n2_max, const Uploader& u,
                       const AreaBufs& o)
{
    uint32_t* lists = reinterpret_cast<uint32_t*>(u.base() + o.lists);
    int32_t* cnt = reinterpret_cast<int32_t*>(u.base() + o.cnt);
    const int cap_q = std::max(nq_max, 1);
    n2_max = std::max(n2_max, 1);
    // the replay's per-query arrays in LDS when they fit beside the table
    // and a full entry budget, else in global memory; the entry budget
    // shrinks to what is left
    constexpr size_t kLds = 160 * 1024 - 1024;   // static LDS of the kernel aside
    int q_lds = area_replay_lds(n2_max, cap_q, kReplayEntries) <= kLds;
    const size_t fixed = area_replay_lds(n2_max, q_lds ? cap_q : 0, 0);
    if (fixed > kLds) return ORBX_ERR_UNSUPPORTED;
    const int ent_cap = (int)std::min<size_t>(kReplayEntries, (kLds - fixed) / 4);
    if (nq_max > 0)
        hipLaunchKernelGGL(k_area_lists<K>, dim3((nq_max + kAreaListWaves - 1) / kAreaListWaves, B),
                           dim3(kAreaListWaves * 64), area_lists_lds(n2_max), ctx->stream, dj, cap_q, lists, cnt);
    hipLaunchKernelGGL(k_area_replay<K>, dim3(B), dim3(kReplayThreads), area_replay_lds(n2_max, q_lds ? cap_q : 0, ent_cap),
                       ctx->stream, dj, cap_q, lists, cnt, q_lds, ent_cap, reinterpret_cast<int*>(u.base() + o.qglob));
    ORBX_HIP_CHECK(hipGetLastError());
    return ORBX_OK;
}

}  // namespace
}  // namespace orbx

using namespace orbx;

extern "C" {

// Diagnostics: rounds of the two-phase searches' parallel replay summed over
// calls, and how many fell back to the sequential replay.
int orbx_debug_area_rounds(unsigned long long* out)
{
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(orbx::g_area_rounds), sizeof(unsigned long long) * 2) == hipSuccess
               ? ORBX_OK
               : ORBX_ERR_HIP;
}

int orbx_search_for_initialization(orbx_ctx* ctx, const orbx_frame_view* F1, const orbx_frame_view* F2,
                                   float* prev_matched, int32_t* matches12, int window, float nnratio,
                                   int check_ori, int* n_matches)
{
    if (!ctx || !valid_view(F1) || !valid_view(F2) || !prev_matched || !matches12 || !n_matches || window < 0)
        return ORBX_ERR_ARG;
    ctx_enter(ctx);
    // inputs, then the outputs (prev_out starts as a copy of prev_matched)
    Uploader u{ctx};
    const FrameOffs o1 = reserve_frame(u, F1), o2 = reserve_frame(u, F2);
    const size_t op = u.reserve((size_t)F1->n * 8);
    const size_t opo = u.reserve((size_t)F1->n * 8), oo = u.reserve((size_t)F1->n * 4 + 4), on = u.reserve(4);
    // candidate slots = F2 keypoints of octave 0; queries = F1's up to its
    // last octave-0 keypoint
    int cap_c = 0, n1q = 0;
    for (int i = 0; i < F2->n; i++) cap_c += F2->keys_un[i].octave == 0;
    for (int i = 0; i < F1->n; i++)
        if (F1->keys_un[i].octave == 0) n1q = i + 1;
    cap_c = std::max(cap_c, 1);
    if (cap_c > kInitMaxCand) return ORBX_ERR_UNSUPPORTED;
    // k_sfi_lists' output (device only, after the read-back range)
    const size_t out_end = on + 4;
    const size_t okeys = u.reserve((size_t)std::max(n1q, 1) * cap_c * 4), ocnt = u.reserve((size_t)std::max(n1q, 1) * 4);
    const int cap1 = std::max(F1->n, 1);
    const size_t fixed = init_lds_bytes(cap_c, cap1, 0);
    const int cap_keys = std::max<int>(cap_c, (int)((kInitLdsBudget - std::min(fixed, kInitLdsBudget)) / 4));
    const size_t lds = init_lds_bytes(cap_c, cap1, cap_keys);
    if (lds > 160 * 1024) return ORBX_ERR_UNSUPPORTED;
    int r = ensure_scratch(ctx, u.total);
    Pinned pin{ctx};
    if (r == ORBX_OK) r = pin.open(out_end);
    if (r != ORBX_OK) return r;
    put_frame(pin, o1, F1);
    put_frame(pin, o2, F2);
    pin.put(op, prev_matched, (size_t)F1->n * 8);
    pin.put(opo, prev_matched, (size_t)F1->n * 8);
    if ((r = pin.upload(oo)) != ORBX_OK) return r;
    SearchArgs a{};
    a.F1 = dev_frame(F1, u.base(), o1.kp, o1.desc);
    a.F2 = dev_frame(F2, u.base(), o2.kp, o2.desc);
    a.prev_xy = reinterpret_cast<const float*>(u.base() + op);
    a.prev_out = reinterpret_cast<float*>(u.base() + opo);
    a.window = window;
    a.nnratio = nnratio;
    a.check_ori = check_ori;
    a.out = reinterpret_cast<int32_t*>(u.base() + oo);
    a.out_n = reinterpret_cast<int32_t*>(u.base() + on);
    uint32_t* dkeys = reinterpret_cast<uint32_t*>(u.base() + okeys);
    int32_t* dcnt = reinterpret_cast<int32_t*>(u.base() + ocnt);
    if (n1q > 0)
        hipLaunchKernelGGL(k_sfi_lists, dim3((n1q + kListWaves - 1) / kListWaves), dim3(kListWaves * 64),
                           sfi_lists_lds(cap_c), ctx->stream, a, cap_c, n1q, dkeys, dcnt);
    hipLaunchKernelGGL(k_search_init_one, dim3(1), dim3(kInitOneThreads), lds, ctx->stream, a, cap_c, cap_keys,
                       ctx->error_flags, dkeys, dcnt);
    ORBX_HIP_CHECK(hipGetLastError());
    if ((r = pin.download(opo, out_end)) != ORBX_OK) return r;
    pin.get(matches12, oo, (size_t)F1->n * 4);
    pin.get(n_matches, on, 4);
    pin.get(prev_matched, opo, (size_t)F1->n * 8);
    return *n_matches < 0 ? *n_matches : ORBX_OK;
}

int orbx_window_search(orbx_ctx* ctx, const orbx_frame_view* F1, const orbx_frame_view* F2, const uint8_t* f1_mp,
                       int window, int min_level, int max_level, float nnratio, int check_ori, int32_t* matches21,
                       int* n_matches)
{
    if (!ctx || !valid_view(F1) || !valid_view(F2) || !f1_mp || !matches21 || !n_matches || window < 0)
        return ORBX_ERR_ARG;
    ctx_enter(ctx);
    Uploader u{ctx};
    const FrameOffs o1 = reserve_frame(u, F1), o2 = reserve_frame(u, F2);
    const size_t ov = u.reserve(F1->n), oarg = u.reserve(sizeof(SearchArgs));
    const size_t oo = u.reserve((size_t)F2->n * 4 + 4), on = u.reserve(4), io_end = on + 4;
    const AreaBufs ol = reserve_area(u, 1, F1->n);
    int r = ensure_scratch(ctx, u.total);
    Pinned pin{ctx};
    if (r == ORBX_OK) r = pin.open(io_end);
    if (r != ORBX_OK) return r;
    put_frame(pin, o1, F1);
    put_frame(pin, o2, F2);
    pin.put(ov, f1_mp, F1->n);
    pin.fill(oo, 0xFF, (size_t)F2->n * 4 + 4);
    SearchArgs a{};
    a.F1 = dev_frame(F1, u.base(), o1.kp, o1.desc);
    a.F2 = dev_frame(F2, u.base(), o2.kp, o2.desc);
    a.q_valid = u.base() + ov;
    a.window = window;
    a.min_level = min_level;
    a.max_level = max_level < 0 ? 0x7fffffff : max_level;
    a.nnratio = nnratio;
    a.check_ori = check_ori;
    a.out = reinterpret_cast<int32_t*>(u.base() + oo);
    a.out_n = reinterpret_cast<int32_t*>(u.base() + on);
    pin.put(oarg, &a, sizeof(a));
    if ((r = pin.upload(io_end)) != ORBX_OK) return r;
    const SearchArgs* da = reinterpret_cast<const SearchArgs*>(u.base() + oarg);
    if ((r = launch_area_search<kQWindow>(ctx, da, 1, F1->n, F2->n, u, ol)) != ORBX_OK) return r;
    if ((r = pin.download(oo, io_end)) != ORBX_OK) return r;
    pin.get(matches21, oo, (size_t)F2->n * 4);
    pin.get(n_matches, on, 4);
    return ORBX_OK;
}

int orbx_search_by_projection_pair(orbx_ctx* ctx, const orbx_frame_view* F1, const orbx_frame_view* F2,
                                   const float* f1_mp_xyz, const uint8_t* f1_mp_valid, const uint8_t* f2_assigned,
                                   const float* Tcw2, const float* cam, int window, float nnratio, int32_t* matches21,
                                   int* n_matches)
{
    if (!ctx || !valid_view(F1) || !valid_view(F2) || !f1_mp_xyz || !f1_mp_valid || !f2_assigned || !Tcw2 || !cam ||
        !matches21 || !n_matches || window < 0)
        return ORBX_ERR_ARG;
    ctx_enter(ctx);
    Uploader u{ctx};
    const FrameOffs o1 = reserve_frame(u, F1), o2 = reserve_frame(u, F2);
    const size_t ox = u.reserve((size_t)F1->n * 12), ov = u.reserve(F1->n), oa = u.reserve(F2->n);
    const size_t oarg = u.reserve(sizeof(SearchArgs));
    const size_t oo = u.reserve((size_t)F2->n * 4 + 4), on = u.reserve(4), io_end = on + 4;
    const AreaBufs ol = reserve_area(u, 1, F1->n);
    int r = ensure_scratch(ctx, u.total);
    Pinned pin{ctx};
    if (r == ORBX_OK) r = pin.open(io_end);
    if (r != ORBX_OK) return r;
    put_frame(pin, o1, F1);
    put_frame(pin, o2, F2);
    pin.put(ox, f1_mp_xyz, (size_t)F1->n * 12);
    pin.put(ov, f1_mp_valid, F1->n);
    pin.put(oa, f2_assigned, F2->n);
    pin.fill(oo, 0xFF, (size_t)F2->n * 4 + 4);
    SearchArgs a{};
    a.F1 = dev_frame(F1, u.base(), o1.kp, o1.desc);
    a.F2 = dev_frame(F2, u.base(), o2.kp, o2.desc);
    a.q_xyz = reinterpret_cast<const float*>(u.base() + ox);
    a.q_valid = u.base() + ov;
    a.f2_assigned = u.base() + oa;
    for (int i = 0; i < 12; i++) a.T[i] = Tcw2[i];
    for (int i = 0; i < 4; i++) a.cam[i] = cam[i];
    a.window = window;
    a.nnratio = nnratio;
    a.out = reinterpret_cast<int32_t*>(u.base() + oo);
    a.out_n = reinterpret_cast<int32_t*>(u.base() + on);
    pin.put(oarg, &a, sizeof(a));
    if ((r = pin.upload(io_end)) != ORBX_OK) return r;
    const SearchArgs* da = reinterpret_cast<const SearchArgs*>(u.base() + oarg);
    if ((r = launch_area_search<kQPair>(ctx, da, 1, F1->n, F2->n, u, ol)) != ORBX_OK) return r;
    if ((r = pin.download(oo, io_end)) != ORBX_OK) return r;
    pin.get(matches21, oo, (size_t)F2->n * 4);
    pin.get(n_matches, on, 4);
    return ORBX_OK;
}

int orbx_search_by_projection_motion(orbx_ctx* ctx, const orbx_frame_view* Cur, const orbx_frame_view* Last,
                                     const float* last_mp_xyz, const uint8_t* last_mp_valid,
                                     const uint8_t* cur_assigned, const float* Tcw, const float* cam, float th,
                                     int check_ori, int32_t* matches_cur, int* n_matches)
{
    if (!ctx || !valid_view(Cur) || !valid_view(Last) || !last_mp_xyz || !last_mp_valid || !cur_assigned || !Tcw ||
        !cam || !matches_cur || !n_matches)
        return ORBX_ERR_ARG;
    ctx_enter(ctx);
    Uploader u{ctx};
    const FrameOffs oL = reserve_frame(u, Last), oC = reserve_frame(u, Cur);
    const size_t ox = u.reserve((size_t)Last->n * 12), ov = u.reserve(Last->n), oa = u.reserve(Cur->n);
    const size_t oarg = u.reserve(sizeof(SearchArgs));
    const size_t oo = u.reserve((size_t)Cur->n * 4 + 4), on = u.reserve(4), io_end = on + 4;
    const AreaBufs ol = reserve_area(u, 1, Last->n);
    int r = ensure_scratch(ctx, u.total);
    Pinned pin{ctx};
    if (r == ORBX_OK) r = pin.open(io_end);
    if (r != ORBX_OK) return r;
    put_frame(pin, oL, Last);
    put_frame(pin, oC, Cur);
    pin.put(ox, last_mp_xyz, (size_t)Last->n * 12);
    pin.put(ov, last_mp_valid, Last->n);
    pin.put(oa, cur_assigned, Cur->n);
    pin.fill(oo, 0xFF, (size_t)Cur->n * 4 + 4);
    SearchArgs a{};
    a.F1 = dev_frame(Last, u.base(), oL.kp, oL.desc);
    a.F2 = dev_frame(Cur, u.base(), oC.kp, oC.desc);
    a.q_xyz = reinterpret_cast<const float*>(u.base() + ox);
    a.q_valid = u.base() + ov;
    a.f2_assigned = u.base() + oa;
    for (int i = 0; i < 12; i++) a.T[i] = Tcw[i];
    for (int i = 0; i < 4; i++) a.cam[i] = cam[i];
    frame_scales(Cur, a.scale);
    a.th = th;
    a.check_ori = check_ori;
    a.out = reinterpret_cast<int32_t*>(u.base() + oo);
    a.out_n = reinterpret_cast<int32_t*>(u.base() + on);
    pin.put(oarg, &a, sizeof(a));
    if ((r = pin.upload(io_end)) != ORBX_OK) return r;
    const SearchArgs* da = reinterpret_cast<const SearchArgs*>(u.base() + oarg);
    if ((r = launch_area_search<kQMotion>(ctx, da, 1, Last->n, Cur->n, u, ol)) != ORBX_OK) return r;
    if ((r = pin.download(oo, io_end)) != ORBX_OK) return r;
    pin.get(matches_cur, oo, (size_t)Cur->n * 4);
    pin.get(n_matches, on, 4);
    return ORBX_OK;
}

int orbx_search_by_projection_local(orbx_ctx* ctx, const orbx_frame_view* F, int n_mp, const uint8_t* in_view,
                                    const float* proj_xy, const int32_t* pred_level, const float* view_cos,
                                    const uint8_t* mp_desc, const uint8_t* f_assigned, float th, float nnratio,
                                    int32_t* matches_f, int* n_matches)
{
    if (!ctx || !valid_view(F) || n_mp < 0 || (n_mp > 0 && (!in_view || !proj_xy || !pred_level || !view_cos || !mp_desc)) ||
        !f_assigned || !matches_f || !n_matches)
        return ORBX_ERR_ARG;
    for (int m = 0; m < n_mp; m++)
        if (in_view[m] && (pred_level[m] < 0 || pred_level[m] >= F->nlevels)) return ORBX_ERR_ARG;
    ctx_enter(ctx);
    Uploader u{ctx};
    const FrameOffs oF = reserve_frame(u, F);
    const size_t ov = u.reserve(n_mp), op = u.reserve((size_t)n_mp * 8), ol = u.reserve((size_t)n_mp * 4);
    const size_t oc = u.reserve((size_t)n_mp * 4), od = u.reserve((size_t)n_mp * 32), oa = u.reserve(F->n);
    const size_t oarg = u.reserve(sizeof(SearchArgs));
    const size_t oo = u.reserve((size_t)F->n * 4 + 4), on = u.reserve(4), io_end = on + 4;
    const AreaBufs oli = reserve_area(u, 1, n_mp);
    int r = ensure_scratch(ctx, u.total);
    Pinned pin{ctx};
    if (r == ORBX_OK) r = pin.open(io_end);
    if (r != ORBX_OK) return r;
    put_frame(pin, oF, F);
    pin.put(ov, in_view, n_mp);
    pin.put(op, proj_xy, (size_t)n_mp * 8);
    pin.put(ol, pred_level, (size_t)n_mp * 4);
    pin.put(oc, view_cos, (size_t)n_mp * 4);
    pin.put(od, mp_desc, (size_t)n_mp * 32);
    pin.put(oa, f_assigned, F->n);
    pin.fill(oo, 0xFF, (size_t)F->n * 4 + 4);
    SearchArgs a{};
    a.F2 = dev_frame(F, u.base(), oF.kp, oF.desc);
    a.nq = n_mp;
    a.q_valid = u.base() + ov;
    a.proj_xy = reinterpret_cast<const float*>(u.base() + op);
    a.pred_level = reinterpret_cast<const int32_t*>(u.base() + ol);
    a.view_cos = reinterpret_cast<const float*>(u.base() + oc);
    a.q_desc = u.base() + od;
    a.f2_assigned = u.base() + oa;
    frame_scales(F, a.scale);
    a.th = th;
    a.nnratio = nnratio;
    a.out = reinterpret_cast<int32_t*>(u.base() + oo);
    a.out_n = reinterpret_cast<int32_t*>(u.base() + on);
    pin.put(oarg, &a, sizeof(a));
    if ((r = pin.upload(io_end)) != ORBX_OK) return r;
    const SearchArgs* da = reinterpret_cast<const SearchArgs*>(u.base() + oarg);
    if ((r = launch_area_search<kQLocal>(ctx, da, 1, n_mp, F->n, u, oli)) != ORBX_OK) return r;
    if ((r = pin.download(oo, io_end)) != ORBX_OK) return r;
    pin.get(matches_f, oo, (size_t)F->n * 4);
    pin.get(n_matches, on, 4);
    return ORBX_OK;
}

// Tracking::SearchReferencePointsInFrustum for B frames: one packed upload
// (pinned staging), k_frustum over every job's points, k_proj_local_jobs one
// wavefront per frame, one packed readback.
static int search_local_map_impl(orbx_ctx* ctx, int B, orbx_local_map_query* qs)
{
    if (!ctx || B <= 0 || !qs) return ORBX_ERR_ARG;
    int max_n = 1, max_mp = 0;
    for (int b = 0; b < B; b++) {
        const orbx_local_map_query& q = qs[b];
        const orbx_frame_view* F = q.frame;
        if (!valid_view(F) || q.n_mp < 0 || !q.Rcw || !q.tcw || !q.Ow || !q.cam || !q.f_assigned || !q.matches_f ||
            (q.n_mp > 0 && (!q.mp_pos || !q.mp_normal || !q.mp_dist || !q.mp_desc)))
            return ORBX_ERR_ARG;
        max_n = std::max(max_n, F->n);
        max_mp = std::max(max_mp, q.n_mp);
    }
    ctx_enter(ctx);
    // layout: [inputs of every job | SearchArgs[B] | outputs of every job]
    struct Offs {
        FrameOffs f;
        size_t assigned, pos, normal, dist, skip, desc;        // inputs
        size_t in_view, proj, pred, cos, out, out_n, count;    // outputs
    };
    std::vector<Offs> o(B);
    Uploader u{ctx};
    for (int b = 0; b < B; b++) {
        const orbx_local_map_query& q = qs[b];
        const size_t n = q.frame->n, m = q.n_mp;
        o[b].f = reserve_frame(u, q.frame);
        o[b].assigned = u.reserve(n);
        o[b].pos = u.reserve(m * 12);
        o[b].normal = u.reserve(m * 12);
        o[b].dist = u.reserve(m * 8);
        o[b].skip = u.reserve(m);
        o[b].desc = u.reserve(m * 32);
    }
    const size_t o_jobs = u.reserve((size_t)B * sizeof(SearchArgs));
    const size_t o_outputs = u.total;
    size_t o_end = 0;
    for (int b = 0; b < B; b++) {
        const orbx_local_map_query& q = qs[b];
        const size_t n = q.frame->n, m = q.n_mp;
        o[b].out = u.reserve(n * 4);
        o[b].out_n = u.reserve(4);
        o[b].count = u.reserve(4);
        o[b].in_view = u.reserve(m);
        o[b].proj = u.reserve(m * 8);
        o[b].pred = u.reserve(m * 4);
        o[b].cos = u.reserve(m * 4);
    }
    o_end = u.total;
    // one frame (Tracking's per-frame call): the two-phase search; batches of
    // frames keep one wave per frame (k_proj_local_jobs)
    const AreaBufs oa = reserve_area(u, 1, B == 1 ? max_mp : 0);
    int r = ensure_scratch(ctx, u.total);
    if (r == ORBX_OK) r = ensure_pinned(ctx, o_end);
    if (r != ORBX_OK) return r;
    uint8_t* h = static_cast<uint8_t*>(ctx->host_pinned);
    uint8_t* d = u.base();
    auto cp = [&](size_t off, const void* src, size_t bytes) {
        if (bytes && src) std::memcpy(h + off, src, bytes);
    };
    std::vector<SearchArgs> jobs(B);
    for (int b = 0; b < B; b++) {
        const orbx_local_map_query& q = qs[b];
        const orbx_frame_view* F = q.frame;
        const size_t n = F->n, m = q.n_mp;
        cp(o[b].f.kp, F->keys_un, n * sizeof(orbx_keypoint));
        cp(o[b].f.desc, F->desc, n * 32);
        cp(o[b].assigned, q.f_assigned, n);
        cp(o[b].pos, q.mp_pos, m * 12);
        cp(o[b].normal, q.mp_normal, m * 12);
        cp(o[b].dist, q.mp_dist, m * 8);
        if (q.mp_skip) cp(o[b].skip, q.mp_skip, m);
        else if (m) std::memset(h + o[b].skip, 0, m);
        cp(o[b].desc, q.mp_desc, m * 32);
        std::memset(h + o[b].out, 0xFF, n * 4);   // matches_f: -1 unless assigned here
        std::memset(h + o[b].out_n, 0, 8);        // out_n, count
        SearchArgs& a = jobs[b];
        a = SearchArgs{};
        a.F2 = dev_frame(F, d, o[b].f.kp, o[b].f.desc);
        a.nq = q.n_mp;
        a.q_xyz = reinterpret_cast<const float*>(d + o[b].pos);
        a.mp_normal = reinterpret_cast<const float*>(d + o[b].normal);
        a.mp_dist = reinterpret_cast<const float*>(d + o[b].dist);
        a.mp_skip = d + o[b].skip;
        a.q_desc = d + o[b].desc;
        a.f2_assigned = d + o[b].assigned;
        for (int i = 0; i < 9; i++) a.Rcw[i] = q.Rcw[i];
        for (int i = 0; i < 3; i++) {
            a.tcw[i] = q.tcw[i];
            a.Ow[i] = q.Ow[i];
        }
        for (int i = 0; i < 4; i++) a.cam[i] = q.cam[i];
        frame_scales(F, a.scale);
        a.nlevels = F->nlevels;
        a.view_cos_limit = q.view_cos_limit;
        a.th = q.th;
        a.nnratio = q.nnratio;
        a.fr_in_view = d + o[b].in_view;
        a.fr_proj = reinterpret_cast<float*>(d + o[b].proj);
        a.fr_pred = reinterpret_cast<int32_t*>(d + o[b].pred);
        a.fr_cos = reinterpret_cast<float*>(d + o[b].cos);
        a.fr_count = reinterpret_cast<int32_t*>(d + o[b].count);
        // the search reads the frustum results as its per-point inputs
        a.q_valid = a.fr_in_view;
        a.proj_xy = a.fr_proj;
        a.pred_level = a.fr_pred;
        a.view_cos = a.fr_cos;
        a.out = reinterpret_cast<int32_t*>(d + o[b].out);
        a.out_n = reinterpret_cast<int32_t*>(d + o[b].out_n);
    }
    cp(o_jobs, jobs.data(), (size_t)B * sizeof(SearchArgs));
    // inputs and the job table in one copy, then each job's -1 match vector
    // and zero counters (contiguous per job)
    ORBX_HIP_CHECK(hipMemcpyAsync(d, h, o_outputs, hipMemcpyHostToDevice, ctx->stream));
    for (int b = 0; b < B; b++)
        ORBX_HIP_CHECK(hipMemcpyAsync(d + o[b].out, h + o[b].out, o[b].count + 4 - o[b].out, hipMemcpyHostToDevice,
                                      ctx->stream));
    const SearchArgs* dj = reinterpret_cast<const SearchArgs*>(d + o_jobs);
    if (max_mp > 0)
        hipLaunchKernelGGL(k_frustum, dim3((max_mp + 255) / 256, B), dim3(256), 0, ctx->stream, dj);
    if (B == 1) {
        if ((r = launch_area_search<kQLocal>(ctx, dj, 1, max_mp, max_n, u, oa)) != ORBX_OK) return r;
    } else {
        hipLaunchKernelGGL(k_proj_local_jobs, dim3(B), dim3(64), tab_lds(max_n), ctx->stream, dj);
    }
    ORBX_HIP_CHECK(hipGetLastError());
    ORBX_HIP_CHECK(hipMemcpyAsync(h + o_outputs, d + o_outputs, o_end - o_outputs, hipMemcpyDeviceToHost, ctx->stream));
    ORBX_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    for (int b = 0; b < B; b++) {
        orbx_local_map_query& q = qs[b];
        const size_t n = q.frame->n, m = q.n_mp;
        std::memcpy(q.matches_f, h + o[b].out, n * 4);
        std::memcpy(&q.n_matches, h + o[b].out_n, 4);
        std::memcpy(&q.n_in_view, h + o[b].count, 4);
        if (q.in_view) std::memcpy(q.in_view, h + o[b].in_view, m);
        if (q.proj_xy) std::memcpy(q.proj_xy, h + o[b].proj, m * 8);
        if (q.pred_level) std::memcpy(q.pred_level, h + o[b].pred, m * 4);
        if (q.view_cos) std::memcpy(q.view_cos, h + o[b].cos, m * 4);
    }
    return ORBX_OK;
}

static int hamming_bf_impl(orbx_ctx* ctx, const uint8_t* dA, int nA, const uint8_t* dB, int nB, int32_t* best_idx,
                           int32_t* best, int32_t* second, int32_t* m12, int th_low, float nnratio)
{
    if (!ctx || nA < 0 || nB < 0 || (nA && (!dA || !best_idx || !best || !second)) || (nB && !dB)) return ORBX_ERR_ARG;
    if (nA == 0) return ORBX_OK;
    ctx_enter(ctx);
    Uploader u{ctx};
    const size_t oa = u.reserve((size_t)nA * 32), ob = u.reserve((size_t)nB * 32);
    const size_t oi = u.reserve((size_t)nA * 4), o1 = u.reserve((size_t)nA * 4), o2 = u.reserve((size_t)nA * 4);
    const size_t om = u.reserve((size_t)nA * 4);
    int r = ensure_scratch(ctx, u.total);
    Pinned pin{ctx};
    if (r == ORBX_OK) r = pin.open(u.total);
    if (r != ORBX_OK) return r;
    pin.put(oa, dA, (size_t)nA * 32);
    pin.put(ob, dB, (size_t)nB * 32);
    if ((r = pin.upload(oi)) != ORBX_OK) return r;
    uint8_t* base = u.base();
    hipLaunchKernelGGL(k_hamming_bf, dim3((nA + 255) / 256), dim3(256), 0, ctx->stream, base + oa, nA, base + ob, nB,
                       reinterpret_cast<int32_t*>(base + oi), reinterpret_cast<int32_t*>(base + o1),
                       reinterpret_cast<int32_t*>(base + o2), m12 ? reinterpret_cast<int32_t*>(base + om) : nullptr,
                       th_low, nnratio);
    ORBX_HIP_CHECK(hipGetLastError());
    if ((r = pin.download(oi, u.total)) != ORBX_OK) return r;
    pin.get(best_idx, oi, (size_t)nA * 4);
    pin.get(best, o1, (size_t)nA * 4);
    pin.get(second, o2, (size_t)nA * 4);
    pin.get(m12, om, (size_t)nA * 4);
    return ORBX_OK;
}

// Tracking::TrackWithMotionModel + TrackLocalMap on the device (see
// include/orbx.h): one upload, the extraction of the slot, nine launches
// (glue, two-phase motion search, glue, PoseOptimization, glue, frustum,
// two-phase local search, glue, PoseOptimization, glue), one read-back.
int orbx_track_frame(orbx_ctx* ctx, orbx_track_query* q)
{
    if (!ctx || !q) return ORBX_ERR_ARG;
    const bool from_slot = q->last_slot >= 0;
    if (q->slot < 0 || q->slot >= ctx->slots || q->last_slot >= ctx->slots || q->last_slot == q->slot ||
        (!from_slot && !valid_view(q->last)) || (from_slot && q->last_cap < 0) || q->n_mp < 0 ||
        (q->n_mp > 0 && (!q->mp_pos || !q->mp_normal || !q->mp_dist || !q->mp_desc)) || !q->Tcw_pred || !q->cam ||
        !q->inv_level_sigma2 || !q->cur_mp || !q->cur_outlier || q->cap < 0 || q->nlevels <= 0 ||
        q->nlevels > kMaxLevels || q->mode < 0 || q->mode > 1 || q->min_octave < 0)
        return ORBX_ERR_ARG;
    const bool prev = q->mode == 1;   // TrackPreviousFrame
    const int n1 = from_slot ? q->last_cap : q->last->n;
    if (from_slot && n1 > ctx->geom.nfeatures) return ORBX_ERR_ARG;
    if (n1 > 0 && (!q->last_mp || !q->last_outlier)) return ORBX_ERR_ARG;
    if (q->image && (q->w <= 0 || q->h <= 0 || q->stride < (size_t)q->w)) return ORBX_ERR_ARG;
    ctx_enter(ctx);
    int r = ORBX_OK;
    if (q->image && (r = ensure_geometry(ctx, q->w, q->h)) != ORBX_OK) return r;
    if (ctx->geom_w <= 0 || q->nlevels != ctx->geom.nlevels) return ORBX_ERR_ARG;
    for (int i = 0; i < n1; i++)
        if (q->last_mp[i] >= q->n_mp) return ORBX_ERR_ARG;
    const Geometry& g = ctx->geom;
    const int nf = g.nfeatures, m = q->n_mp, cap = std::max(nf, 1);
    const int m_local = q->n_local_mp > 0 ? std::min(q->n_local_mp, m) : m;   // the frustum search's points
    const size_t img_bytes = q->image ? (size_t)q->w * q->h : 0;
    // [inputs | SearchArgs x2 | read-back block | device-only state]
    Uploader u{ctx};
    FrameOffs oL{};
    if (!from_slot) oL = reserve_frame(u, q->last);
    const size_t o_lmp = u.reserve((size_t)n1 * 4), o_lout = u.reserve(n1);
    const size_t o_pos = u.reserve((size_t)m * 12), o_nrm = u.reserve((size_t)m * 12), o_dist = u.reserve((size_t)m * 8);
    const size_t o_desc = u.reserve((size_t)m * 32), o_skin = u.reserve(m), o_isig = u.reserve(4 * kMaxLevels);
    const size_t o_img = u.reserve(img_bytes);
    const size_t o_jm = u.reserve(sizeof(SearchArgs)), o_jl = u.reserve(sizeof(SearchArgs));
    // mode 1: the two WindowSearch jobs and the pair search's
    const size_t o_jw = u.reserve(prev ? 2 * sizeof(SearchArgs) : 0), o_jp = u.reserve(prev ? sizeof(SearchArgs) : 0);
    const size_t in_end = u.total;
    const size_t o_out = u.reserve(sizeof(TrackOut) + (size_t)cap * 5), out_end = u.total;
    const size_t o_qxyz = u.reserve((size_t)n1 * 12), o_qv = u.reserve(n1);
    const size_t o_mout = u.reserve((size_t)cap * 4 + 4), o_mn = u.reserve(4);
    const size_t o_lo = u.reserve((size_t)cap * 4 + 4), o_ln = u.reserve(4), o_cnt = u.reserve(4);
    const size_t o_fiv = u.reserve(m), o_fpr = u.reserve((size_t)m * 8), o_fpl = u.reserve((size_t)m * 4);
    const size_t o_fcos = u.reserve((size_t)m * 4), o_cmp = u.reserve((size_t)cap * 4), o_fas = u.reserve(cap);
    const size_t o_skip = u.reserve(m), o_hdr = u.reserve(3 * sizeof(PoseHdr)), o_edg = u.reserve((size_t)cap * 72);
    const size_t o_ekp = u.reserve((size_t)cap * 12), o_flg = u.reserve((size_t)cap * 3);
    const size_t o_pout = u.reserve(3 * sizeof(PoseOut)), o_st = u.reserve(32);
    size_t o_wout[2] = {0, 0}, o_wn[2] = {0, 0}, o_pout2 = 0, o_pn = 0, o_wv = 0, o_pv = 0;
    if (prev) {
        for (int k = 0; k < 2; k++) {
            o_wout[k] = u.reserve((size_t)cap * 4 + 4);
            o_wn[k] = u.reserve(4);
        }
        o_pout2 = u.reserve((size_t)cap * 4 + 4);
        o_pn = u.reserve(4);
        o_wv = u.reserve(n1);
        o_pv = u.reserve(n1);
    }
    const AreaBufs am = reserve_area(u, 1, n1), al = reserve_area(u, 1, m_local);
    r = ensure_scratch(ctx, u.total);
    Pinned pin{ctx};
    if (r == ORBX_OK) r = pin.open(out_end);
    if (r != ORBX_OK) return r;
    uint8_t* d = u.base();
    if (!from_slot) put_frame(pin, oL, q->last);
    pin.put(o_lmp, q->last_mp, (size_t)n1 * 4);
    pin.put(o_lout, q->last_outlier, n1);
    pin.put(o_pos, q->mp_pos, (size_t)m * 12);
    pin.put(o_nrm, q->mp_normal, (size_t)m * 12);
    pin.put(o_dist, q->mp_dist, (size_t)m * 8);
    pin.put(o_desc, q->mp_desc, (size_t)m * 32);
    if (q->mp_skip) pin.put(o_skin, q->mp_skip, m);
    pin.put(o_isig, q->inv_level_sigma2, (size_t)q->nlevels * 4);
    if (q->image) {
        if (q->stride == (size_t)q->w) {
            pin.put(o_img, q->image, img_bytes);
        } else {
            for (int y = 0; y < q->h; y++) pin.put(o_img + (size_t)y * q->w, q->image + (size_t)y * q->stride, q->w);
        }
    }
    // the slots' frames: keypoints where extraction left them, the count on
    // the device, bounds of orbx_dev_set_image_bounds (default the image)
    auto slot_frame = [&](int slot) {
        FrameDev F;
        F.kps = ctx->out_kps + (size_t)slot * nf;
        F.desc = ctx->out_desc + (size_t)slot * nf * 32;
        F.n = nf;
        F.min_x = ctx->has_bounds ? ctx->bounds[0] : 0.f;
        F.max_x = ctx->has_bounds ? ctx->bounds[1] : (float)g.w;
        F.min_y = ctx->has_bounds ? ctx->bounds[2] : 0.f;
        F.max_y = ctx->has_bounds ? ctx->bounds[3] : (float)g.h;
        F.grid_w_inv = static_cast<float>(kGridCols) / (F.max_x - F.min_x);
        F.grid_h_inv = static_cast<float>(kGridRows) / (F.max_y - F.min_y);
        return F;
    };
    float scale[kMaxLevels] = {};
    scale[0] = 1.0f;
    for (int i = 1; i < g.nlevels; i++) scale[i] = scale[i - 1] * g.scale_factor;   // src/Frame.cc:98-102
    // SearchByProjection(mCurrentFrame, mLastFrame, 15), ORBmatcher(0.9, true)
    // (src/Tracking.cc:574-584): queries = the last frame's keypoints
    SearchArgs jm{};
    jm.F1 = from_slot ? slot_frame(q->last_slot) : dev_frame(q->last, d, oL.kp, oL.desc);
    jm.F2 = slot_frame(q->slot);
    jm.F2_cnt = ctx->out_n + q->slot;
    if (from_slot) jm.F1.n = n1;   // queries past the slot's count are not valid (k_track_stage 0)
    jm.q_xyz = reinterpret_cast<const float*>(d + o_qxyz);
    jm.q_valid = d + o_qv;
    jm.f2_assigned = d + o_fas;
    for (int i = 0; i < 12; i++) jm.T[i] = q->Tcw_pred[i];
    for (int i = 0; i < 4; i++) jm.cam[i] = q->cam[i];
    std::memcpy(jm.scale, scale, sizeof(scale));
    jm.th = 15.f;
    jm.check_ori = 1;
    jm.out = reinterpret_cast<int32_t*>(d + o_mout);
    jm.out_n = reinterpret_cast<int32_t*>(d + o_mn);
    // SearchReferencePointsInFrustum (src/Tracking.cc:701-752): the pose and
    // the query count are filled in on the device (k_track_stage 2)
    SearchArgs jl{};
    jl.F2 = slot_frame(q->slot);
    jl.F2_cnt = ctx->out_n + q->slot;
    jl.nq = 0;
    jl.q_xyz = reinterpret_cast<const float*>(d + o_pos);
    jl.mp_normal = reinterpret_cast<const float*>(d + o_nrm);
    jl.mp_dist = reinterpret_cast<const float*>(d + o_dist);
    jl.mp_skip = d + o_skip;
    jl.q_desc = d + o_desc;
    jl.f2_assigned = d + o_fas;
    for (int i = 0; i < 4; i++) jl.cam[i] = q->cam[i];
    std::memcpy(jl.scale, scale, sizeof(scale));
    jl.nlevels = g.nlevels;
    jl.view_cos_limit = 0.5f;
    jl.th = q->th_local;
    jl.nnratio = 0.8f;
    jl.fr_in_view = d + o_fiv;
    jl.fr_proj = reinterpret_cast<float*>(d + o_fpr);
    jl.fr_pred = reinterpret_cast<int32_t*>(d + o_fpl);
    jl.fr_cos = reinterpret_cast<float*>(d + o_fcos);
    jl.fr_count = reinterpret_cast<int32_t*>(d + o_cnt);
    jl.q_valid = jl.fr_in_view;
    jl.proj_xy = jl.fr_proj;
    jl.pred_level = jl.fr_pred;
    jl.view_cos = jl.fr_cos;
    jl.out = reinterpret_cast<int32_t*>(d + o_lo);
    jl.out_n = reinterpret_cast<int32_t*>(d + o_ln);
    pin.put(o_jm, &jm, sizeof(jm));
    pin.put(o_jl, &jl, sizeof(jl));
    if (prev) {
        // WindowSearch(mLastFrame, mCurrentFrame, 200, minOctave) and (100, 0),
        // ORBmatcher(0.9, true) (src/Tracking.cc:500-517)
        for (int k = 0; k < 2; k++) {
            SearchArgs jw{};
            jw.F1 = jm.F1;
            jw.F2 = jm.F2;
            jw.F2_cnt = jm.F2_cnt;
            jw.q_valid = d + o_wv;
            jw.window = k == 0 ? 200 : 100;
            jw.min_level = k == 0 ? q->min_octave : 0;
            jw.max_level = 0x7fffffff;
            jw.nnratio = 0.9f;
            jw.check_ori = 1;
            jw.out = reinterpret_cast<int32_t*>(d + o_wout[k]);
            jw.out_n = reinterpret_cast<int32_t*>(d + o_wn[k]);
            pin.put(o_jw + k * sizeof(SearchArgs), &jw, sizeof(jw));
        }
        // SearchByProjection(mLastFrame, mCurrentFrame, 15 or 50) (:544, :547):
        // pose and window set on the device
        SearchArgs jp{};
        jp.F1 = jm.F1;
        jp.F2 = jm.F2;
        jp.F2_cnt = jm.F2_cnt;
        jp.q_xyz = jm.q_xyz;
        jp.q_valid = d + o_pv;
        jp.f2_assigned = d + o_fas;
        for (int i = 0; i < 4; i++) jp.cam[i] = q->cam[i];
        jp.nnratio = 0.9f;
        jp.out = reinterpret_cast<int32_t*>(d + o_pout2);
        jp.out_n = reinterpret_cast<int32_t*>(d + o_pn);
        pin.put(o_jp, &jp, sizeof(jp));
    }
    TrackDev td{};
    td.cur_kps = jm.F2.kps;
    td.cur_cnt = jm.F2_cnt;
    td.last_mp = reinterpret_cast<const int32_t*>(d + o_lmp);
    td.last_outlier = d + o_lout;
    td.n_last = n1;
    td.last_cnt = from_slot ? ctx->out_n + q->last_slot : nullptr;
    td.err = ctx->error_flags;
    td.n_mp = m;
    td.n_local = m_local;
    td.cap = cap;
    td.mp_pos = jl.q_xyz;
    td.mp_skip_in = q->mp_skip ? d + o_skin : nullptr;
    td.isig = reinterpret_cast<const float*>(d + o_isig);
    for (int i = 0; i < 12; i++) td.Tpred[i] = q->Tcw_pred[i];
    for (int i = 0; i < 4; i++) td.cam[i] = q->cam[i];
    td.q_xyz = reinterpret_cast<float*>(d + o_qxyz);
    td.q_valid = d + o_qv;
    td.motion_out = jm.out;
    td.motion_n = jm.out_n;
    td.local_out = jl.out;
    td.local_n = jl.out_n;
    td.motion_out_w = jm.out;
    td.motion_n_w = jm.out_n;
    td.local_out_w = jl.out;
    td.local_n_w = jl.out_n;
    td.cur_mp = reinterpret_cast<int32_t*>(d + o_cmp);
    td.f_assigned = d + o_fas;
    td.mp_skip = d + o_skip;
    td.local_job = reinterpret_cast<SearchArgs*>(d + o_jl);
    td.hdr = reinterpret_cast<PoseHdr*>(d + o_hdr);
    td.edges = reinterpret_cast<float*>(d + o_edg);
    td.edge_kp = reinterpret_cast<int32_t*>(d + o_ekp);
    td.flags = d + o_flg;
    td.pout = reinterpret_cast<const PoseOut*>(d + o_pout);
    td.st = reinterpret_cast<int32_t*>(d + o_st);
    td.out = reinterpret_cast<TrackOut*>(d + o_out);
    td.mode = q->mode;
    td.min_octave = q->min_octave;
    if (prev) {
        for (int k = 0; k < 2; k++) {
            td.win_job[k] = reinterpret_cast<SearchArgs*>(d + o_jw + k * sizeof(SearchArgs));
            td.win_out[k] = reinterpret_cast<int32_t*>(d + o_wout[k]);
            td.win_n[k] = reinterpret_cast<int32_t*>(d + o_wn[k]);
        }
        td.pair_job = reinterpret_cast<SearchArgs*>(d + o_jp);
        td.pair_out = reinterpret_cast<int32_t*>(d + o_pout2);
        td.pair_n = reinterpret_cast<int32_t*>(d + o_pn);
        td.w_valid = d + o_wv;
        td.p_valid = d + o_pv;
    } else {
        td.pair_job = reinterpret_cast<SearchArgs*>(d + o_jm);   // stage 4 reads its T only for status 3
    }
    // one upload; the image into its slot and the slot's extraction
    if ((r = pin.upload(in_end)) != ORBX_OK) return r;
    if (q->image) {
        ORBX_HIP_CHECK(hipMemcpyAsync(ctx->frames + (size_t)q->slot * img_bytes, d + o_img, img_bytes,
                                      hipMemcpyDeviceToDevice, ctx->stream));
        ctx->last_first = q->slot;
        ctx->last_count = 1;
        ctx->single_frame = true;   // the latency-first single-frame launches
        r = launch_extract(ctx, q->slot, 1);
        ctx->single_frame = false;
        if (r != ORBX_OK) return r;
    }
    PoseEdgeArrays ed;
    const size_t arr = (size_t)3 * cap;
    ed.ox = td.edges;
    ed.oy = td.edges + arr;
    ed.isig = td.edges + 2 * arr;
    ed.px = td.edges + 3 * arr;
    ed.py = td.edges + 4 * arr;
    ed.pz = td.edges + 5 * arr;
    uint8_t* flags = d + o_flg;
    PoseOut* pout = reinterpret_cast<PoseOut*>(d + o_pout);
    const SearchArgs* dm = reinterpret_cast<const SearchArgs*>(d + o_jm);
    const SearchArgs* dl = reinterpret_cast<const SearchArgs*>(d + o_jl);
    auto stage = [&](int s) { hipLaunchKernelGGL(k_track_stage, dim3(1), dim3(kTrackThreads), 0, ctx->stream, td, s); };
    if (!prev) {
        stage(0);
        if ((r = launch_area_search<kQMotion>(ctx, dm, 1, n1, nf, u, am)) != ORBX_OK) return r;
        stage(1);
    } else {
        const SearchArgs* dw = reinterpret_cast<const SearchArgs*>(d + o_jw);
        stage(10);
        if ((r = launch_area_search<kQWindow>(ctx, dw, 1, n1, nf, u, am)) != ORBX_OK) return r;
        stage(11);
        if ((r = launch_area_search<kQWindow>(ctx, dw + 1, 1, n1, nf, u, am)) != ORBX_OK) return r;
        stage(12);
        if ((r = launch_pose_device(ctx, td.hdr + 2, ed, flags, pout + 2, 1)) != ORBX_OK) return r;
        stage(13);
        if ((r = launch_area_search<kQPair>(ctx, reinterpret_cast<const SearchArgs*>(d + o_jp), 1, n1, nf, u, am)) !=
            ORBX_OK)
            return r;
        stage(14);
    }
    if ((r = launch_pose_device(ctx, td.hdr, ed, flags, pout, 1)) != ORBX_OK) return r;
    stage(2);
    if (m_local > 0) hipLaunchKernelGGL(k_frustum, dim3((m_local + 255) / 256, 1), dim3(256), 0, ctx->stream, dl);
    if ((r = launch_area_search<kQLocal>(ctx, dl, 1, m_local, nf, u, al)) != ORBX_OK) return r;
    stage(3);
    if ((r = launch_pose_device(ctx, td.hdr + 1, ed, flags, pout + 1, 1)) != ORBX_OK) return r;
    stage(4);
    ORBX_HIP_CHECK(hipGetLastError());
    if ((r = pin.download(o_out, out_end)) != ORBX_OK) return r;
    TrackOut o;
    pin.get(&o, o_out, sizeof(o));
    for (int i = 0; i < 12; i++) q->Tcw[i] = o.T[i];
    q->n_cur = o.n_cur;
    q->status = o.status;
    q->n_motion = o.n_motion;
    q->n_pair = o.n_pair;
    q->n_after_pose = o.n_after_pose;
    q->n_in_view = o.n_in_view;
    q->n_local = o.n_local;
    q->n_inliers = o.n_inliers;
    const int nc = std::min(o.n_cur, q->cap);
    pin.get(q->cur_mp, o_out + sizeof(TrackOut), (size_t)nc * 4);
    pin.get(q->cur_outlier, o_out + sizeof(TrackOut) + (size_t)cap * 4, nc);
    if (o.err) {   // an extraction overflow (k_track_stage read the flags)
        ORBX_HIP_CHECK(hipMemsetAsync(ctx->error_flags, 0, sizeof(int32_t), ctx->stream));
        return ORBX_ERR_CAPACITY;
    }
    return o.n_cur > q->cap ? ORBX_ERR_CAPACITY : ORBX_OK;
}

int orbx_search_local_map(orbx_ctx* ctx, orbx_local_map_query* q)
{
    return search_local_map_impl(ctx, 1, q);
}

int orbx_search_local_map_batch(orbx_ctx* ctx, int B, orbx_local_map_query* qs)
{
    return search_local_map_impl(ctx, B, qs);
}

int orbx_hamming_bf(orbx_ctx* ctx, const uint8_t* dA, int nA, const uint8_t* dB, int nB, int32_t* best_idx,
                    int32_t* best, int32_t* second)
{
    return hamming_bf_impl(ctx, dA, nA, dB, nB, best_idx, best, second, nullptr, 0, 0.f);
}

// Brute-force matcher (C3): best <= th_low && best < nnratio * second.
int orbx_match_bf(orbx_ctx* ctx, const uint8_t* dA, int nA, const uint8_t* dB, int nB, int th_low, float nnratio,
                  int32_t* m12, int* n_matches)
{
    if (!m12 || !n_matches || nA < 0) return ORBX_ERR_ARG;
    std::vector<int32_t> bi(nA), b1(nA), b2(nA);
    int r = hamming_bf_impl(ctx, dA, nA, dB, nB, bi.data(), b1.data(), b2.data(), m12, th_low, nnratio);
    if (r != ORBX_OK) return r;
    int n = 0;
    for (int a = 0; a < nA; a++) n += m12[a] >= 0;
    *n_matches = n;
    return ORBX_OK;
}

}  // extern "C"

#ifdef ORBX_MATCH_PROFILE
// this file's copy of the stamp sums (k_search_init_one's block 0, wave 0)
extern "C" int orbx_debug_search_prof(unsigned long long* out, int reset)
{
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_match_prof), sizeof(unsigned long long) * 12) != hipSuccess) return -2;
    if (reset) {
        const unsigned long long z[12] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_match_prof), z, sizeof(z)) != hipSuccess) return -2;
    }
    return 0;
}
#endif
