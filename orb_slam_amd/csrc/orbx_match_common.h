// Shared device code of the ORBmatcher kernels (orbx_match.hip,
// orbx_search.hip): Frame grid queries (src/Frame.cc:199-276), rotation
// histogram (src/ORBmatcher.cc:1748-1789), wave reductions, and the
// SearchForInitialization wave routine.
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

__device__ inline int wave_min_i32(int v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
    return v;
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
// SearchForInitialization (src/ORBmatcher.cc:598-713) for one pair, one wave.
// LDS (per wave): candidate table of F2's octave-0 keypoints in index order
// {x, y, cell, vMatchedDistance, vnMatches21, index} and, per F1 keypoint,
// vnMatches12 and the rotation bin it was pushed to.
// ---------------------------------------------------------------------------
struct CandLDS {
    float* x;
    float* y;
    int* cell;
    int* mdist;
    int* m21;
    int* idx;
};

__device__ inline void search_for_init_wave(const FrameDev& F1, const FrameDev& F2, const float* prev_xy,
                                     int window, float nnratio, bool check_ori, int32_t* out_m12,
                                     int32_t* out_n, float* out_prev_xy, CandLDS c, int* m12,
                                     signed char* pushed, int* hist)
{
    const int lane = threadIdx.x & 63;
    // compact F2 octave-0 keypoints (index order)
    int nc = 0;
    for (int base = 0; base < F2.n; base += 64) {
        const int i2 = base + lane;
        bool ok = false;
        orbx_keypoint k;
        if (i2 < F2.n) {
            k = F2.kps[i2];
            ok = (k.octave == 0);
        }
        const unsigned long long bal = __ballot(ok);
        if (ok) {
            const int pos = nc + __popcll(bal & ((1ull << lane) - 1ull));
            c.x[pos] = k.x;
            c.y[pos] = k.y;
            c.cell[pos] = grid_cell(F2, k.x, k.y);
            c.mdist[pos] = 0x7fffffff;
            c.m21[pos] = -1;
            c.idx[pos] = i2;
        }
        nc += __popcll(bal);
    }
    for (int i = lane; i < F1.n; i += 64) {
        m12[i] = -1;
        pushed[i] = -1;
    }
    wave_sync();
    const float r = (float)window;
    int nmatches = 0;
    for (int i1 = 0; i1 < F1.n; i1++) {
        const orbx_keypoint k1 = F1.kps[i1];
        if (k1.octave > 0) continue;
        const float qx = prev_xy ? prev_xy[2 * i1] : k1.x;
        const float qy = prev_xy ? prev_xy[2 * i1 + 1] : k1.y;
        const AreaQuery q = area_cells(F2, qx, qy, r);
        if (q.empty) continue;
        uint4 d1a, d1b;
        load_desc(F1.desc + (size_t)i1 * 32, d1a, d1b);
        unsigned long long best = ~0ull;
        int any = 0;
        for (int j = lane; j < nc; j += 64) {
            const int cell = c.cell[j];
            if (!in_area(q, cell, c.x[j], c.y[j], qx, qy, r)) continue;
            any = 1;
            uint4 d2a, d2b;
            load_desc(F2.desc + (size_t)c.idx[j] * 32, d2a, d2b);
            const int dist = hamming256(d1a, d1b, d2a, d2b);
            if (c.mdist[j] <= dist) continue;
            const unsigned long long key = ((unsigned long long)dist << 32) |
                                           ((unsigned long long)cell << 12) | (unsigned long long)c.idx[j];
            best = key < best ? key : best;
        }
        if (!__any(any)) continue;   // vIndices2.empty()
        best = wave_min_u64(best);
        if (best == ~0ull) continue;
        const int bestDist = (int)(best >> 32);
        const int bestIdx2 = (int)(best & 0xFFF);
        // second smallest of the multiset of admissible distances
        int second = 0x7fffffff;
        for (int j = lane; j < nc; j += 64) {
            const int cell = c.cell[j];
            if (c.idx[j] == bestIdx2) continue;
            if (!in_area(q, cell, c.x[j], c.y[j], qx, qy, r)) continue;
            uint4 d2a, d2b;
            load_desc(F2.desc + (size_t)c.idx[j] * 32, d2a, d2b);
            const int dist = hamming256(d1a, d1b, d2a, d2b);
            if (c.mdist[j] <= dist) continue;
            second = min(second, dist);
        }
        second = wave_min_i32(second);
        if (bestDist <= kTHLow && (float)bestDist < __fmul_rn((float)second, nnratio)) {
            // locate bestIdx2's candidate slot (unique)
            int slot = -1;
            for (int j = lane; j < nc; j += 64)
                if (c.idx[j] == bestIdx2) slot = j;
            slot = wave_max(slot);
            if (lane == 0) {
                const int prev = c.m21[slot];
                if (prev >= 0) {
                    m12[prev] = -1;
                    nmatches--;
                }
                m12[i1] = bestIdx2;
                c.m21[slot] = i1;
                c.mdist[slot] = bestDist;
                nmatches++;
                if (check_ori) pushed[i1] = (signed char)rot_bin(k1.angle, F2.kps[bestIdx2].angle);
            }
            wave_sync();
        }
    }
    wave_sync();
    if (lane == 0) {
        if (check_ori) {
            for (int b = 0; b < kHistoLength; b++) hist[b] = 0;
            for (int i = 0; i < F1.n; i++)
                if (pushed[i] >= 0) hist[pushed[i]]++;
            int ind1, ind2, ind3;
            three_maxima(hist, ind1, ind2, ind3);
            for (int i = 0; i < F1.n; i++) {
                const int b = pushed[i];
                if (b < 0 || b == ind1 || b == ind2 || b == ind3) continue;
                if (m12[i] >= 0) {
                    m12[i] = -1;
                    nmatches--;
                }
            }
        }
        *out_n = nmatches;
    }
    wave_sync();
    for (int i = lane; i < F1.n; i += 64) {
        const int m = m12[i];
        out_m12[i] = m;
        if (out_prev_xy && m >= 0) {
            out_prev_xy[2 * i] = F2.kps[m].x;
            out_prev_xy[2 * i + 1] = F2.kps[m].y;
        }
    }
}

// Shared-memory carve for one wave: 6 candidate arrays of cap_c, m12 of cap1,
// pushed bins of cap1, histogram of 32.
__device__ inline void carve(uint8_t* base, int cap_c, int cap1, CandLDS& c, int*& m12,
                             signed char*& pushed, int*& hist)
{
    c.x = reinterpret_cast<float*>(base);
    c.y = c.x + cap_c;
    c.cell = reinterpret_cast<int*>(c.y + cap_c);
    c.mdist = c.cell + cap_c;
    c.m21 = c.mdist + cap_c;
    c.idx = c.m21 + cap_c;
    m12 = c.idx + cap_c;
    hist = m12 + cap1;
    pushed = reinterpret_cast<signed char*>(hist + 32);
}

__host__ __device__ inline size_t search_init_lds_bytes(int cap_c, int cap1)
{
    return (size_t)cap_c * 24 + (size_t)cap1 * 4 + 32 * 4 + (size_t)((cap1 + 15) & ~15);
}

}  // namespace orbx
