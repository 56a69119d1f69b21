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
    const float factor = __fdiv_rn(1.0f, (float)kHistoLength);
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
//  2. (wave 0, sequential in i1 order) the greedy replay: admissible keys
//     (vMatchedDistance[i2] > dist) -> best key and second-best distance by
//     wave reductions, then the accept / steal update in LDS.
//
// Descriptors of the candidates are staged in LDS.  The rotation histogram
// (with the reference's stale entries of stolen matches) is built with LDS
// atomics and filtered in parallel after ComputeThreeMaxima.
// ---------------------------------------------------------------------------
constexpr int kInitMaxCand = 2048;     // slot field of the key (11 bits)
constexpr size_t kInitLdsBudget = 64 * 1024;

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
    int cap_c, cap1, cap_keys;
};

__host__ __device__ inline size_t init_lds_bytes(int cap_c, int cap1, int cap_keys)
{
    return (size_t)cap_c * (7 * 4 + 32) + (size_t)cap1 * 8 + (size_t)((cap1 + 15) & ~15) + 257 * 4 + 36 * 4 +
           (size_t)cap_keys * 4 + 64;
}

__device__ inline InitLDS carve_init(uint8_t* base, int cap_c, int cap1, int cap_keys)
{
    InitLDS s;
    s.cap_c = cap_c;
    s.cap1 = cap1;
    s.cap_keys = cap_keys;
    s.desc = reinterpret_cast<uint4*>(base);
    s.x = reinterpret_cast<float*>(s.desc + 2 * cap_c);
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

__device__ inline void search_for_init_block(const FrameDev& F1, const FrameDev& F2, const float* prev_xy,
                                             int window, float nnratio, bool check_ori, int32_t* out_m12,
                                             int32_t* out_n, float* out_prev_xy, InitLDS s, BlockScratch& bs,
                                             int32_t* error_flags)
{
    const int tid = threadIdx.x, lane = tid & 63;
    // F2 octave-0 keypoints in index order -> candidate slots
    int nc = 0;
    for (int base = 0; base < F2.n; base += kBlock) {
        const int i2 = base + tid;
        orbx_keypoint k;
        bool ok = false;
        if (i2 < F2.n) {
            k = F2.kps[i2];
            ok = (k.octave == 0);
        }
        int tot;
        const int pos = nc + block_exclusive_scan(ok ? 1 : 0, &tot, bs, (base / kBlock) & 1);
        if (ok && pos < s.cap_c) {
            s.x[pos] = k.x;
            s.y[pos] = k.y;
            s.ang[pos] = k.angle;
            s.cell[pos] = grid_cell(F2, k.x, k.y);
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
    for (int i = tid; i < F1.n; i += kBlock) {
        s.m12[i] = -1;
        s.pushed[i] = -1;
        s.ang1[i] = F1.kps[i].angle;
    }
    if (tid < 36) s.hist[tid] = 0;
    __syncthreads();
    const float r = (float)window;
    for (int g0 = 0; g0 < F1.n; g0 += kBlock) {
        const int i1 = g0 + tid;
        bool act = false;
        float qx = 0.f, qy = 0.f;
        AreaQuery q;
        q.empty = true;
        uint4 d1a = make_uint4(0, 0, 0, 0), d1b = d1a;
        if (i1 < F1.n) {
            const orbx_keypoint k1 = F1.kps[i1];
            if (k1.octave == 0) {
                qx = prev_xy ? prev_xy[2 * i1] : k1.x;
                qy = prev_xy ? prev_xy[2 * i1 + 1] : k1.y;
                q = area_cells(F2, qx, qy, r);
                act = !q.empty;
                if (act) load_desc(F1.desc + (size_t)i1 * 32, d1a, d1b);
            }
        }
        int cnt = 0;
        if (act)
            for (int j = 0; j < nc; j++) cnt += in_area(q, s.cell[j], s.x[j], s.y[j], qx, qy, r);
        int total;
        const int off = block_exclusive_scan(cnt, &total, bs, 0);
        s.offs[tid] = off;
        if (tid == kBlock - 1) s.offs[kBlock] = total;
        __syncthreads();
        for (int lo = 0; lo < kBlock;) {
            // largest hi with offs[hi] - offs[lo] <= cap_keys (one list always fits: cnt <= nc <= cap)
            const int base_off = s.offs[lo];
            const int fits = (tid >= lo && s.offs[tid + 1] - base_off <= s.cap_keys) ? 1 : 0;
            const int hi = lo + block_sum(fits, bs, 1);
            if (tid >= lo && tid < hi && cnt > 0) {
                uint32_t* out = s.keys + (off - base_off);
                int w = 0;
                for (int j = 0; j < nc; j++) {
                    const int cell = s.cell[j];
                    if (!in_area(q, cell, s.x[j], s.y[j], qx, qy, r)) continue;
                    const int dist = hamming256(d1a, d1b, s.desc[2 * j], s.desc[2 * j + 1]);
                    out[w++] = ((uint32_t)dist << 23) | ((uint32_t)cell << 11) | (uint32_t)j;
                }
            }
            __syncthreads();
            if (tid < 64) {
                for (int t = lo; t < hi; t++) {
                    const int b = s.offs[t] - base_off, n = s.offs[t + 1] - s.offs[t];
                    if (n == 0) continue;   // vIndices2.empty(), or not an octave-0 query
                    uint32_t best = 0xFFFFFFFFu;
                    for (int e = lane; e < n; e += 64) {
                        const uint32_t key = s.keys[b + e];
                        const int dist = (int)(key >> 23);
                        if (s.mdist[key & 0x7FF] > dist) best = min(best, key);
                    }
                    best = wave_min_u32(best);
                    if (best == 0xFFFFFFFFu) continue;
                    const int bestDist = (int)(best >> 23);
                    int second = 0x7fffffff;
                    for (int e = lane; e < n; e += 64) {
                        const uint32_t key = s.keys[b + e];
                        const int dist = (int)(key >> 23);
                        if (key != best && s.mdist[key & 0x7FF] > dist) second = min(second, dist);
                    }
                    second = wave_min_i32(second);
                    if (bestDist <= kTHLow && (float)bestDist < __fmul_rn((float)second, nnratio)) {
                        if (lane == 0) {
                            const int slot = (int)(best & 0x7FF);
                            const int ii1 = g0 + t;
                            const int prev = s.m21[slot];
                            if (prev >= 0) s.m12[prev] = -1;
                            s.m12[ii1] = s.idx[slot];
                            s.m21[slot] = ii1;
                            s.mdist[slot] = bestDist;
                            if (check_ori) s.pushed[ii1] = (signed char)rot_bin(s.ang1[ii1], s.ang[slot]);
                        }
                        wave_sync();
                    }
                }
            }
            __syncthreads();
            lo = hi;
        }
    }
    if (check_ori) {
        for (int i = tid; i < F1.n; i += kBlock)
            if (s.pushed[i] >= 0) atomicAdd(&s.hist[s.pushed[i]], 1);
        __syncthreads();
        if (tid == 0) three_maxima(s.hist, s.hist[32], s.hist[33], s.hist[34]);
        __syncthreads();
        const int ind1 = s.hist[32], ind2 = s.hist[33], ind3 = s.hist[34];
        for (int i = tid; i < F1.n; i += kBlock) {
            const int b = s.pushed[i];
            if (b < 0 || b == ind1 || b == ind2 || b == ind3) continue;
            s.m12[i] = -1;
        }
        __syncthreads();
    }
    int nm = 0;
    for (int i = tid; i < F1.n; i += kBlock) {
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
}

}  // namespace orbx
