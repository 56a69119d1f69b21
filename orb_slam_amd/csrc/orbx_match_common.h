// Shared device code of the ORBmatcher kernels (orbx_match.hip,
// orbx_search.hip): Frame grid queries (src/Frame.cc:199-276), rotation
// histogram (src/ORBmatcher.cc:1748-1789), wave reductions, and the
// SearchForInitialization block routine.
#pragma once
#include "orbx_device.h"
#include "orbx_internal.h"

namespace orbx {

constexpr int kTHHigh = 100;      // ORBmatcher::TH_HIGH (src/ORBmatcher.cc:40)
constexpr int kTHLow = 50;        // TH_LOW (:41)
constexpr int kHistoLength = 30;  // HISTO_LENGTH (:42)

struct FrameDev {
    const orbx_keypoint* kps;
    const uint8_t* desc;
    int n;
    float min_x, max_x, min_y, max_y;
    float grid_w_inv, grid_h_inv;   // FRAME_GRID_COLS / (maxX - minX) etc.
};

__device__ inline void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

__device__ inline unsigned long long wave_min_u64(unsigned long long v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long t = __shfl_xor(v, o, 64);
        v = t < v ? t : v;
    }
    return v;
}

// Wave-wide min through DPP row shifts and row broadcasts (gfx9 wave64)
// instead of ds_bpermute shuffles: a handful of VALU ops, no LDS round trips.
// Lanes whose DPP source is out of range keep their own value, so the
// partial results stay correct for min.  Result broadcast from lane 63.
__device__ inline uint32_t wave_min_u32(uint32_t v)
{
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x111, 0xf, 0xf, false));   // row_shr:1
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x112, 0xf, 0xf, false));   // row_shr:2
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x114, 0xf, 0xf, false));   // row_shr:4
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x118, 0xf, 0xf, false));   // row_shr:8
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x142, 0xa, 0xf, false));   // row_bcast:15
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x143, 0xc, 0xf, false));   // row_bcast:31
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// Wave-wide (best key, second-best distance) over 64 lanes' partial
// results: (a1, a2) + (b1, b2) -> (min(a1, b1), min(a2, b2, dist(max(a1, b1)))),
// keys being distinct.  DPP scan pattern; result broadcast from lane 63.
template <int kCtrl, int kRowMask>
__device__ inline void best_second_step(uint32_t& m1, int& m2)
{
    const uint32_t p1 = (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)m1, kCtrl, kRowMask, 0xf, false);
    const int p2 = __builtin_amdgcn_update_dpp(511, m2, kCtrl, kRowMask, 0xf, false);
    m2 = min(min(m2, p2), (int)(max(m1, p1) >> 23));
    m1 = min(m1, p1);
}

__device__ inline void best_second_reduce(uint32_t& m1, int& m2)
{
    best_second_step<0x111, 0xf>(m1, m2);
    best_second_step<0x112, 0xf>(m1, m2);
    best_second_step<0x114, 0xf>(m1, m2);
    best_second_step<0x118, 0xf>(m1, m2);
    best_second_step<0x142, 0xa>(m1, m2);
    best_second_step<0x143, 0xc>(m1, m2);
    m1 = (uint32_t)__builtin_amdgcn_readlane((int)m1, 63);
    m2 = __builtin_amdgcn_readlane(m2, 63);
}

__device__ inline int wave_min_i32(int v)
{
    v = min(v, __builtin_amdgcn_update_dpp(v, v, 0x111, 0xf, 0xf, false));
    v = min(v, __builtin_amdgcn_update_dpp(v, v, 0x112, 0xf, 0xf, false));
    v = min(v, __builtin_amdgcn_update_dpp(v, v, 0x114, 0xf, 0xf, false));
    v = min(v, __builtin_amdgcn_update_dpp(v, v, 0x118, 0xf, 0xf, false));
    v = min(v, __builtin_amdgcn_update_dpp(v, v, 0x142, 0xa, 0xf, false));
    v = min(v, __builtin_amdgcn_update_dpp(v, v, 0x143, 0xc, 0xf, false));
    return __builtin_amdgcn_readlane(v, 63);
}

// Frame::PosInGrid (src/Frame.cc:266-276): cell or -1.
__device__ inline int grid_cell(const FrameDev& F, float x, float y)
{
    const int px = (int)roundf(__fmul_rn(__fsub_rn(x, F.min_x), F.grid_w_inv));
    const int py = (int)roundf(__fmul_rn(__fsub_rn(y, F.min_y), F.grid_h_inv));
    if (px < 0 || px >= kGridCols || py < 0 || py >= kGridRows) return -1;
    return px * kGridRows + py;
}

struct AreaQuery {
    int min_cx, max_cx, min_cy, max_cy;
    bool empty;
};

// Frame::GetFeaturesInArea cell range (src/Frame.cc:204-222).
__device__ inline AreaQuery area_cells(const FrameDev& F, float x, float y, float r)
{
    AreaQuery q;
    q.empty = false;
    q.min_cx = max(0, (int)floorf(__fmul_rn(__fsub_rn(__fsub_rn(x, F.min_x), r), F.grid_w_inv)));
    q.max_cx = min(kGridCols - 1, (int)ceilf(__fmul_rn(__fadd_rn(__fsub_rn(x, F.min_x), r), F.grid_w_inv)));
    q.min_cy = max(0, (int)floorf(__fmul_rn(__fsub_rn(__fsub_rn(y, F.min_y), r), F.grid_h_inv)));
    q.max_cy = min(kGridRows - 1, (int)ceilf(__fmul_rn(__fadd_rn(__fsub_rn(y, F.min_y), r), F.grid_h_inv)));
    if (q.min_cx >= kGridCols || q.max_cx < 0 || q.min_cy >= kGridRows || q.max_cy < 0) q.empty = true;
    return q;
}

__device__ inline bool in_area(const AreaQuery& q, int cell, float kx, float ky, float x, float y, float r)
{
    if (cell < 0) return false;
    const int cx = cell / kGridRows, cy = cell - cx * kGridRows;
    if (cx < q.min_cx || cx > q.max_cx || cy < q.min_cy || cy > q.max_cy) return false;
    return !(fabsf(__fsub_rn(kx, x)) > r || fabsf(__fsub_rn(ky, y)) > r);
}

__device__ inline int rot_bin(float a1, float a2)
{
    constexpr float factor = 1.0f / kHistoLength;   // compile-time float division, as the reference
    float rot = __fsub_rn(a1, a2);
    if (rot < 0.0f) rot = __fadd_rn(rot, 360.0f);
    int bin = (int)roundf(__fmul_rn(rot, factor));   // round half away from zero
    if (bin == kHistoLength) bin = 0;
    return bin;
}

// ORBmatcher::ComputeThreeMaxima (src/ORBmatcher.cc:1748-1789), sequential.
__device__ inline void three_maxima(const int* histo, int& ind1, int& ind2, int& ind3)
{
    int max1 = 0, max2 = 0, max3 = 0;
    ind1 = ind2 = ind3 = -1;
    for (int i = 0; i < kHistoLength; i++) {
        const int s = histo[i];
        if (s > max1) {
            max3 = max2; max2 = max1; max1 = s;
            ind3 = ind2; ind2 = ind1; ind1 = i;
        } else if (s > max2) {
            max3 = max2; max2 = s;
            ind3 = ind2; ind2 = i;
        } else if (s > max3) {
            max3 = s;
            ind3 = i;
        }
    }
    if ((float)max2 < __fmul_rn(0.1f, (float)max1)) {
        ind2 = -1;
        ind3 = -1;
    } else if ((float)max3 < __fmul_rn(0.1f, (float)max1)) {
        ind3 = -1;
    }
}

__device__ inline void load_desc(const uint8_t* d, uint4& a, uint4& b)
{
    a = *reinterpret_cast<const uint4*>(d);
    b = *reinterpret_cast<const uint4*>(d + 16);
}

// ---------------------------------------------------------------------------
// SearchForInitialization (src/ORBmatcher.cc:598-713) for one pair, one
// 256-thread block, in two phases per group of 256 F1 keypoints:
//
//  1. (all threads, state-free) each F1 octave-0 keypoint gathers its
//     candidate window -- F2 octave-0 keypoints passing GetFeaturesInArea's
//     cell and box tests -- and stores one 32-bit key per candidate:
//     dist (9 bits) << 23 | grid cell (12 bits) << 11 | candidate slot.
//     Keys order candidates by (distance, GetFeaturesInArea order), so the
//     minimum key is the reference's first strict minimum.
//     In the single-pair kernel a list of at most 64 keys is then sorted
//     (each lane's rank).
//  2. (wave 0, sequential in i1 order) the greedy replay: admissible keys
//     (vMatchedDistance[i2] > dist) -> best key and second-best distance:
//     on a sorted list the first two admissible lanes of one ballot, else
//     wave reductions; then the accept / steal update in LDS.
//
// Descriptors of the candidates are staged in LDS.  The rotation histogram
// (with the reference's stale entries of stolen matches) is built with LDS
// atomics and filtered in parallel after ComputeThreeMaxima.
// ---------------------------------------------------------------------------
constexpr int kInitMaxCand = 2048;     // slot field of the key (11 bits)

// Frame::GetFeaturesInArea membership (src/Frame.cc:222-257) on a packed
// candidate record, branch-free: the candidate loops stream 16-byte records.
__device__ inline bool in_area_rec(const AreaQuery& q, const float4& rc, float qx, float qy, float r)
{
    const int cxcy = __float_as_int(rc.z);
    const int cx = cxcy & 0xFF, cy = (cxcy >> 8) & 0xFF;
    return (cxcy >= 0) & (cx >= q.min_cx) & (cx <= q.max_cx) & (cy >= q.min_cy) & (cy <= q.max_cy) &
           !(fabsf(__fsub_rn(rc.x, qx)) > r) & !(fabsf(__fsub_rn(rc.y, qy)) > r);
}

#ifdef ORBX_MATCH_PROFILE
__device__ unsigned long long g_match_prof[12];   // 0-7 cycles, 8-10 replay counts
__device__ inline unsigned long long match_stamp()
{
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
#define MP_T0() unsigned long long _mt = match_stamp()
#define MP_COUNT(k, v)                                                           \
    do {                                                                         \
        if (blockIdx.x == 0 && threadIdx.x == 0) g_match_prof[k] += (v);         \
    } while (0)
#define MP_MARK(k)                                                               \
    do {                                                                         \
        const unsigned long long _n = match_stamp();                             \
        if (blockIdx.x == 0 && threadIdx.x == 0) g_match_prof[k] += _n - _mt;     \
        _mt = _n;                                                                \
    } while (0)
#else
#define MP_T0()
#define MP_COUNT(k, v)
#define MP_MARK(k)
#endif
// LDS of a SearchForInitialization block: its fixed tables (~40 KB at 1000
// features) plus candidate keys up to this budget.  The blocks stay resident
// for the whole match (~0.3 ms per batch, overlapping the next batch's
// extraction on another stream), so every KB here is taken from the
// extraction kernels on the same CUs: 64 KB -> 44 KB measured c2 207-210k
// -> 214.7k frames/s at the same match time (41 KB: match +6 %, no gain).
constexpr size_t kInitLdsBudget = 44 * 1024;

struct InitLDS {
    float* x;
    float* y;
    float* ang;
    int* cell;
    int* idx;
    int* mdist;
    int* m21;
    uint4* desc;        // 2 per candidate
    int* m12;           // per F1 keypoint
    float* ang1;        // per F1 keypoint: angle (rotation check)
    signed char* pushed;
    int* offs;          // 257 list offsets of the current group
    int* hist;          // 32 bins + 3 maxima indices
    uint32_t* keys;     // candidate lists
    float4* rec;        // per candidate: x, y, (cx | cy << 8) or -1, grid cell (as int bits)
    uint4* qdesc;       // per query of the current group (256): descriptor (2 x uint4)
    float2* qxy;        // query position
    int4* qarea;        // cell range (min_cx, max_cx, min_cy, max_cy); min_cx > max_cx when inactive
    int cap_c, cap1, cap_keys;
};

__host__ __device__ inline size_t init_lds_bytes(int cap_c, int cap1, int cap_keys)
{
    return (size_t)cap_c * (7 * 4 + 32 + 16) + (size_t)cap1 * 8 + (size_t)((cap1 + 15) & ~15) + 257 * 4 + 36 * 4 +
           (size_t)cap_keys * 4 + 256 * (32 + 8 + 16) + 64;
}

__device__ inline InitLDS carve_init(uint8_t* base, int cap_c, int cap1, int cap_keys)
{
    InitLDS s;
    s.cap_c = cap_c;
    s.cap1 = cap1;
    s.cap_keys = cap_keys;
    s.desc = reinterpret_cast<uint4*>(base);
    s.qdesc = s.desc + 2 * cap_c;
    s.qarea = reinterpret_cast<int4*>(s.qdesc + 2 * 256);
    s.qxy = reinterpret_cast<float2*>(s.qarea + 256);
    s.rec = reinterpret_cast<float4*>(s.qxy + 256);
    s.x = reinterpret_cast<float*>(s.rec + cap_c);
    s.y = s.x + cap_c;
    s.ang = s.y + cap_c;
    s.cell = reinterpret_cast<int*>(s.ang + cap_c);
    s.idx = s.cell + cap_c;
    s.mdist = s.idx + cap_c;
    s.m21 = s.mdist + cap_c;
    s.m12 = s.m21 + cap_c;
    s.ang1 = reinterpret_cast<float*>(s.m12 + cap1);
    s.offs = reinterpret_cast<int*>(s.ang1 + cap1);
    s.hist = s.offs + 257;
    s.keys = reinterpret_cast<uint32_t*>(s.hist + 36);
    s.pushed = reinterpret_cast<signed char*>(s.keys + cap_keys);
    return s;
}

//
// One query's candidate count and keys (one wave, lanes over the nc
// candidate records): the count pass and the fill pass of the routine
// below, shared with k_sfi_lists.
__device__ inline AreaQuery area_of(const int4 qa)
{
    AreaQuery q;
    q.min_cx = qa.x; q.max_cx = qa.y; q.min_cy = qa.z; q.max_cy = qa.w; q.empty = false;
    return q;
}

__device__ inline int sfi_query_count(const InitLDS& s, int nc, int4 qa, float2 qp, float r, int lane)
{
    if (qa.x > qa.y) return 0;
    const AreaQuery q = area_of(qa);
    int cnt = 0;
    for (int j = lane; j < nc; j += 64) cnt += in_area_rec(q, s.rec[j], qp.x, qp.y, r);
    return wave_sum(cnt);
}

// keys of the in-area candidates, compacted in candidate order into out[]
__device__ inline void sfi_query_fill(const InitLDS& s, int nc, int4 qa, float2 qp, uint4 d1a, uint4 d1b, float r,
                                      uint32_t* out, int lane)
{
    const AreaQuery q = area_of(qa);
    const unsigned long long lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    int w = 0;
    for (int j0 = 0; j0 < nc; j0 += 64) {
        const int j = j0 + lane;
        bool ok = false;
        float4 rc;
        if (j < nc) {
            rc = s.rec[j];
            ok = in_area_rec(q, rc, qp.x, qp.y, r);
        }
        const unsigned long long bal = __ballot(ok);
        if (ok) {
            const int dist = hamming256(d1a, d1b, s.desc[2 * j], s.desc[2 * j + 1]);
            out[w + __popcll(bal & lt_mask)] = ((uint32_t)dist << 23) | ((uint32_t)__float_as_int(rc.w) << 11) | (uint32_t)j;
        }
        w += __popcll(bal);
    }
}

// a list of w <= 64 distinct keys into ascending order (each lane's rank),
// from src to dst (may be the same array)
__device__ inline void sfi_sort_short(const uint32_t* src, uint32_t* dst, int w, int lane)
{
    const uint32_t mine = lane < w ? src[lane] : 0xFFFFFFFFu;
    int rank = 0;
    for (int i = 0; i < w; i++) rank += (uint32_t)__builtin_amdgcn_readlane((int)mine, i) < mine;
    if (lane < w) dst[rank] = mine;
}

// kT threads (a multiple of 64, >= kBlock): the batch kernel runs 256 per
// pair; the single-pair call 1024, so the count and fill passes (one wave per
// query) have 16 waves instead of 4.  Queries are staged in groups of kBlock
// whatever kT is.
// kPre: the candidate lists were built by k_sfi_lists (pre_cnt[i1] keys at
// pre_keys + i1 * cap_c, sorted when <= 64): the count and fill passes
// become a copy into LDS.
template <int kT = kBlock, bool kPre = false>
__device__ inline void search_for_init_block(const FrameDev& F1, const FrameDev& F2, const float* prev_xy,
                                             int window, float nnratio, bool check_ori, int32_t* out_m12,
                                             int32_t* out_n, float* out_prev_xy, InitLDS s,
                                             BlockScratchN<kT / 64>& bs, int32_t* error_flags,
                                             const uint32_t* pre_keys = nullptr, const int32_t* pre_cnt = nullptr)
{
    static_assert(kT % 64 == 0 && kT >= kBlock, "whole waves, at least one query group");
    constexpr int kW = kT / 64;
    // sorted candidate lists and the ballot replay for the single-pair
    // kernel (latency: one pair on the chip); the batch kernel keeps the
    // unsorted lists and the reduction replay (throughput: its extra fill
    // work cost c2 1.2 % while matching overlaps extraction)
    constexpr bool kSortLists = kT > kBlock;
    const int tid = threadIdx.x, lane = tid & 63;
    MP_T0();
    // F2 octave-0 keypoints in index order -> candidate slots
    int nc = 0;
    for (int base = 0; base < F2.n; base += kT) {
        const int i2 = base + tid;
        orbx_keypoint k;
        bool ok = false;
        if (i2 < F2.n) {
            k = F2.kps[i2];
            ok = (k.octave == 0);
        }
        int tot;
        const int pos = nc + block_exclusive_scan(ok ? 1 : 0, &tot, bs, (base / kT) & 1);
        if (ok && pos < s.cap_c) {
            s.x[pos] = k.x;
            s.y[pos] = k.y;
            s.ang[pos] = k.angle;
            const int cell = grid_cell(F2, k.x, k.y);
            s.cell[pos] = cell;
            s.rec[pos] = make_float4(k.x, k.y, __int_as_float(cell < 0 ? -1 : ((cell / kGridRows) | ((cell % kGridRows) << 8))),
                                     __int_as_float(cell));
            s.idx[pos] = i2;
            s.mdist[pos] = 0x7fffffff;
            s.m21[pos] = -1;
            const uint4* d = reinterpret_cast<const uint4*>(F2.desc + (size_t)i2 * 32);
            s.desc[2 * pos] = d[0];
            s.desc[2 * pos + 1] = d[1];
        }
        nc += tot;
    }
    if (nc > s.cap_c) {
        if (tid == 0) {
            atomicOr(error_flags, 4);
            *out_n = ORBX_ERR_CAPACITY;
        }
        return;
    }
    // queries are the F1 octave-0 keypoints: the groups below stop after the
    // last one (extractor output is level-major, so they are a prefix)
    int last0 = -1;
    for (int i = tid; i < F1.n; i += kT) {
        const orbx_keypoint k1 = F1.kps[i];
        s.m12[i] = -1;
        s.pushed[i] = -1;
        s.ang1[i] = k1.angle;
        if (k1.octave == 0) last0 = i;
    }
    if (tid < 36) s.hist[tid] = 0;
    __syncthreads();   // the staging scans' reads of bs are done
    const int n1q = block_max(last0, bs, 0) + 1;
    __syncthreads();
    MP_MARK(0);
    const float r = (float)window;
    const int wv = tid >> 6;
    for (int g0 = 0; g0 < n1q; g0 += kBlock) {
        const int gn = min(kBlock, n1q - g0);
        // stage the group's queries (one thread each): position, cell range,
        // descriptor; inactive (octave > 0 or empty area) get an empty range
        if (!kPre) {
            const int i1 = g0 + tid;
            int4 qa = make_int4(1, 0, 1, 0);
            float2 qp = make_float2(0.f, 0.f);
            if (tid < gn) {   // gn <= kBlock
                const orbx_keypoint k1 = F1.kps[i1];
                if (k1.octave == 0) {
                    qp = make_float2(prev_xy ? prev_xy[2 * i1] : k1.x, prev_xy ? prev_xy[2 * i1 + 1] : k1.y);
                    const AreaQuery q = area_cells(F2, qp.x, qp.y, r);
                    if (!q.empty) qa = make_int4(q.min_cx, q.max_cx, q.min_cy, q.max_cy);
                    load_desc(F1.desc + (size_t)i1 * 32, s.qdesc[2 * tid], s.qdesc[2 * tid + 1]);
                }
            }
            if (tid < kBlock) {
                s.qarea[tid] = qa;
                s.qxy[tid] = qp;
            }
        }
        __syncthreads();
        // count pass, one wave per query (lanes over the candidates): balanced
        // whatever the window population of individual queries
        for (int t = wv; t < gn; t += kW) {
            const int cnt = kPre ? pre_cnt[g0 + t] : sfi_query_count(s, nc, s.qarea[t], s.qxy[t], r, lane);
            if (lane == 0) s.offs[t] = cnt;
        }
        if (g0 == 0) MP_MARK(4);
        __syncthreads();
        const int cnt = tid < gn ? s.offs[tid] : 0;
        if (g0 == 0) MP_MARK(5);
        int total;
        const int off = block_exclusive_scan(cnt, &total, bs, 0);
        if (tid < kBlock) s.offs[tid] = off;
        if (tid == kBlock - 1) s.offs[kBlock] = total;
        __syncthreads();
        for (int lo = 0; lo < kBlock;) {
            // largest hi with offs[hi] - offs[lo] <= cap_keys (one list always fits: cnt <= nc <= cap)
            const int base_off = s.offs[lo];
            const int fits = (tid >= lo && tid < kBlock && s.offs[tid + 1] - base_off <= s.cap_keys) ? 1 : 0;
            const int hi = lo + block_sum(fits, bs, 1);
            // fill pass, one wave per query: keys of the in-area candidates
            if (kPre) {
                // flat copy of the chunk's keys: key e belongs to the last
                // query t with offs[t] - base_off <= e
                const int tot = s.offs[hi] - base_off;
                for (int e = tid; e < tot; e += kT) {
                    int qa = lo, qb = hi - 1;
                    while (qa < qb) {
                        const int m = (qa + qb + 1) >> 1;
                        if (s.offs[m] - base_off <= e) qa = m;
                        else qb = m - 1;
                    }
                    s.keys[e] = pre_keys[(size_t)(g0 + qa) * s.cap_c + (e - (s.offs[qa] - base_off))];
                }
            }
            for (int t = lo + wv; !kPre && t < hi; t += kW) {
                const int n = s.offs[t + 1] - s.offs[t];
                if (n == 0) continue;
                uint32_t* out = s.keys + (s.offs[t] - base_off);
                sfi_query_fill(s, nc, s.qarea[t], s.qxy[t], s.qdesc[2 * t], s.qdesc[2 * t + 1], r, out, lane);
                // a list that fits one wave is left in ascending key order
                // (rank of each key among the list; keys are distinct)
                if (kSortLists && n <= 64) sfi_sort_short(out, out, n, lane);
            }
            if (g0 == 0) MP_MARK(6);
            __syncthreads();
            MP_MARK(1);
            if (kSortLists && tid < 64) {
                // nnratio in a register for the whole replay (not re-read
                // from the kernel arguments per accepted query)
                float nr = nnratio;
                asm volatile("" : "+v"(nr));
                for (int w0 = lo; w0 < hi; w0 += 64) {
                    // a window of up to 64 queries, one per lane: list offset
                    // and length, read per query with readlane instead of
                    // dependent LDS loads
                    const int wn = min(64, hi - w0);
                    const int tq = w0 + lane;
                    const int q_b = lane < wn ? s.offs[tq] - base_off : 0;
                    const int q_n = lane < wn ? s.offs[tq + 1] - s.offs[tq] : 0;
                    // keys of query i+1 are loaded while i is decided: only the
                    // mdist reads depend on the previous query's outcome
                    int b = __builtin_amdgcn_readlane(q_b, 0), n = __builtin_amdgcn_readlane(q_n, 0);
                    uint32_t kn = lane < n ? s.keys[b + lane] : 0xFFFFFFFFu;
                    for (int i = 0; i < wn; i++) {
                        const int t = w0 + i;
                        const int bc = b, nc1 = n;
                        const uint32_t k0 = kn;
                        if (i + 1 < wn) {
                            b = __builtin_amdgcn_readlane(q_b, i + 1);
                            n = __builtin_amdgcn_readlane(q_n, i + 1);
                            kn = lane < n ? s.keys[b + lane] : 0xFFFFFFFFu;
                        }
                        if (nc1 == 0) continue;   // vIndices2.empty(), or not an octave-0 query
                        const int d0 = (int)(k0 >> 23);
                        const bool adm0 = lane < nc1 && s.mdist[k0 & 0x7FF] > d0;   // vMatchedDistance[i2] > dist
                        uint32_t m1;
                        int m2;
                        if (nc1 <= 64) {
                            // the list is in key order: the best admissible
                            // key is the first admissible lane, the second-best
                            // distance the next one's
                            const unsigned long long am = __ballot(adm0);
                            if (am == 0) continue;
                            const unsigned long long am2 = am & (am - 1);
                            m1 = (uint32_t)__builtin_amdgcn_readlane((int)k0, __builtin_ctzll(am));
                            m2 = am2 ? (int)((uint32_t)__builtin_amdgcn_readlane((int)k0, __builtin_ctzll(am2)) >> 23)
                                     : 511;
                        } else {
                            // one pass over the admissible candidates, as the
                            // reference's loop
                            m1 = adm0 ? k0 : 0xFFFFFFFFu;
                            m2 = 511;   // "none" (> any Hamming distance)
                            for (int e = lane + 64; e < nc1; e += 64) {   // lists longer than a wave
                                const uint32_t key = s.keys[bc + e];
                                const int dist = (int)(key >> 23);
                                if (s.mdist[key & 0x7FF] > dist) {
                                    if (key < m1) {
                                        m2 = min(m2, (int)(m1 >> 23));
                                        m1 = key;
                                    } else {
                                        m2 = min(m2, dist);
                                    }
                                }
                            }
                            best_second_reduce(m1, m2);
                        }
                        if (m1 == 0xFFFFFFFFu) continue;
                        const int bestDist = (int)(m1 >> 23);
                        const int second = m2 >= 511 ? 0x7fffffff : m2;
                        if (bestDist <= kTHLow && (float)bestDist < __fmul_rn((float)second, nr)) {
                            // accept: the slot now belongs to ii1.  A steal needs no
                            // read-modify-write here: m12 is rebuilt at the end from
                            // "ii1 still owns the slot it took" (m21[slot] == ii1),
                            // and the rotation bin from the slot ii1 took.
                            if (lane == 0) {
                                const int slot = (int)(m1 & 0x7FF);
                                s.m12[g0 + t] = slot;
                                s.m21[slot] = g0 + t;
                                s.mdist[slot] = bestDist;
                            }
                            // LDS operations of one wave complete in order: the next
                            // query's mdist reads see these writes; only keep the
                            // compiler from moving memory operations across
                            __atomic_signal_fence(__ATOMIC_SEQ_CST);
                            __builtin_amdgcn_wave_barrier();
                        }
                    }
                }
            }
            if (!kSortLists && tid < 64) {
                // keys of query t+1 are loaded while t is decided: only the
                // mdist reads depend on the previous query's outcome
                int oa = s.offs[lo], ob = s.offs[lo + 1];
                uint32_t kn = lane < ob - oa ? s.keys[oa - base_off + lane] : 0xFFFFFFFFu;
                for (int t = lo; t < hi; t++) {
                    const int n = ob - oa;
                    const int b = oa - base_off;
                    const uint32_t k0 = kn;
                    if (t + 1 < hi) {
                        const int oc = s.offs[t + 2];
                        kn = lane < oc - ob ? s.keys[ob - base_off + lane] : 0xFFFFFFFFu;
                        oa = ob;
                        ob = oc;
                    }
                    if (n == 0) continue;   // vIndices2.empty(), or not an octave-0 query
                    // one pass: lane-local best key and second-best distance
                    // over the admissible candidates (vMatchedDistance > dist)
                    uint32_t m1 = 0xFFFFFFFFu;
                    int m2 = 511;   // "none" (> any Hamming distance)
                    if (lane < n && s.mdist[k0 & 0x7FF] > (int)(k0 >> 23)) m1 = k0;
                    for (int e = lane + 64; e < n; e += 64) {   // lists longer than a wave
                        const uint32_t key = s.keys[b + e];
                        const int dist = (int)(key >> 23);
                        if (s.mdist[key & 0x7FF] > dist) {
                            if (key < m1) {
                                m2 = min(m2, (int)(m1 >> 23));
                                m1 = key;
                            } else {
                                m2 = min(m2, dist);
                            }
                        }
                    }
                    best_second_reduce(m1, m2);
                    if (m1 == 0xFFFFFFFFu) continue;
                    const int bestDist = (int)(m1 >> 23);
                    const int second = m2 >= 511 ? 0x7fffffff : m2;
                    if (bestDist <= kTHLow && (float)bestDist < __fmul_rn((float)second, nnratio)) {
                        // accept: the slot now belongs to ii1.  A steal needs no
                        // read-modify-write here: m12 is rebuilt at the end from
                        // "ii1 still owns the slot it took" (m21[slot] == ii1),
                        // and the rotation bin from the slot ii1 took.
                        if (lane == 0) {
                            const int slot = (int)(m1 & 0x7FF);
                            s.m12[g0 + t] = slot;
                            s.m21[slot] = g0 + t;
                            s.mdist[slot] = bestDist;
                        }
                        // LDS operations of one wave complete in order: the next
                        // query's mdist reads see these writes; only keep the
                        // compiler from moving memory operations across
                        __atomic_signal_fence(__ATOMIC_SEQ_CST);
                        __builtin_amdgcn_wave_barrier();
                    }
                }
            }
            MP_MARK(7);   // wave 0: the replay of this chunk
            __syncthreads();
            lo = hi;
        }
    }
    MP_MARK(2);
    __syncthreads();
    // m12[i] held the slot i took; keep it only if i still owns that slot
    // (rotHist keeps the entries of stolen matches too: src/ORBmatcher.cc:675, 688-703)
    for (int i = tid; i < F1.n; i += kT) {
        const int sl = s.m12[i];
        if (check_ori && sl >= 0) s.pushed[i] = (signed char)rot_bin(s.ang1[i], s.ang[sl]);
        s.m12[i] = (sl >= 0 && s.m21[sl] == i) ? s.idx[sl] : -1;
    }
    __syncthreads();
    if (check_ori) {
        for (int i = tid; i < F1.n; i += kT)
            if (s.pushed[i] >= 0) atomicAdd(&s.hist[s.pushed[i]], 1);
        __syncthreads();
        if (tid == 0) three_maxima(s.hist, s.hist[32], s.hist[33], s.hist[34]);
        __syncthreads();
        const int ind1 = s.hist[32], ind2 = s.hist[33], ind3 = s.hist[34];
        for (int i = tid; i < F1.n; i += kT) {
            const int b = s.pushed[i];
            if (b < 0 || b == ind1 || b == ind2 || b == ind3) continue;
            s.m12[i] = -1;
        }
        __syncthreads();
    }
    int nm = 0;
    for (int i = tid; i < F1.n; i += kT) {
        const int m = s.m12[i];
        out_m12[i] = m;
        nm += m >= 0;
        if (out_prev_xy && m >= 0) {
            out_prev_xy[2 * i] = F2.kps[m].x;
            out_prev_xy[2 * i + 1] = F2.kps[m].y;
        }
    }
    nm = block_sum(nm, bs, 0);
    if (tid == 0) *out_n = nm;
    MP_MARK(3);
}

}  // namespace orbx
