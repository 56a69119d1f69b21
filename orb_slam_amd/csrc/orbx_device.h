// Device-side building blocks shared by the orbx kernels (gfx950, wave64).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "orbx_sincos.h"

namespace orbx {

#include "orbx_sincos_table.inc"

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;

// --------------------------------------------------------------------------
// cv::fastAtan2 (OpenCV 2.4 mathfuncs.cpp), degrees in [0, 360].
// Called by IC_Angle (src/ORBextractor.cc:150).  Division is IEEE (built
// with -fhip-fp32-correctly-rounded-divide-sqrt) and no FMA contraction.
// --------------------------------------------------------------------------
__device__ inline float fast_atan2_deg(float y, float x)
{
    const float p1 = 0.9997878412794807f * (float)(180 / M_PI);
    const float p3 = -0.3258083974640975f * (float)(180 / M_PI);
    const float p5 = 0.1555786518463281f * (float)(180 / M_PI);
    const float p7 = -0.04432655554792128f * (float)(180 / M_PI);
    const float eps = (float)2.220446049250313e-16;   // (float)DBL_EPSILON
    const float ax = fabsf(x), ay = fabsf(y);
    float a;
    if (ax >= ay) {
        const float c = __fdiv_rn(ay, __fadd_rn(ax, eps));
        const float c2 = __fmul_rn(c, c);
        a = __fmul_rn(__fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(p7, c2), p5), c2), p3), c2), p1), c);
    } else {
        const float c = __fdiv_rn(ax, __fadd_rn(ay, eps));
        const float c2 = __fmul_rn(c, c);
        a = __fsub_rn(90.f, __fmul_rn(__fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(p7, c2), p5), c2), p3), c2), p1), c));
    }
    if (x < 0) a = __fsub_rn(180.f, a);
    if (y < 0) a = __fsub_rn(360.f, a);
    return a;
}

// Correctly rounded sinf/cosf of a float angle (see orbx_sincos.h).
__device__ inline float hard_case(float x, int kind, float fallback)
{
    uint32_t xb = __float_as_uint(x);
    int lo = 0, hi = ORBX_SINCOS_HARD_N - 1;
    while (lo <= hi) {
        const int mid = (lo + hi) >> 1;
        const uint32_t mb = kSincosHard[mid][0];
        const int mk = (int)kSincosHard[mid][1];
        if (mb == xb && mk == kind) return __uint_as_float(kSincosHard[mid][2]);
        if (mb < xb || (mb == xb && mk < kind)) lo = mid + 1;
        else hi = mid - 1;
    }
    return fallback;
}

__device__ inline void cr_sincosf(float x, float* s, float* c)
{
    double ds, dc;
    sincos_double(x, &ds, &dc);
    float fs = (float)ds, fc = (float)dc;
    if (near_float_midpoint(ds)) fs = hard_case(x, 0, fs);
    if (near_float_midpoint(dc)) fc = hard_case(x, 1, fc);
    *s = fs;
    *c = fc;
}

// BORDER_REFLECT_101 index (cv::borderInterpolate).
__host__ __device__ inline int reflect101(int p, int len)
{
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    do {
        if (p < 0) p = -p;
        else p = 2 * len - 2 - p;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}

// GaussianBlur 7x7 sigma 2 (OpenCV 2.4 8U fixed point, kernel {18,34,49,55,49,34,18}):
// Horizontal 7-tap sums of the 4 pixels of dword wc (wl / wr: the dwords to
// its left / right): taps j-3..j as one v_dot4_u32_u8 with {18,34,49,55},
// taps j+1..j+3 as a second with {49,34,18,0}.
__device__ inline void blur_hsum_w(uint32_t wl, uint32_t wc, uint32_t wr, int hs[4])
{
    constexpr uint32_t kWA = 0x37312212u, kWB = 0x00122231u;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t A = j == 3 ? wc : __builtin_amdgcn_alignbyte(wc, wl, j + 1);   // bytes j-3 .. j
        const uint32_t B = j == 3 ? wr : __builtin_amdgcn_alignbyte(wr, wc, j + 1);   // bytes j+1 .. j+4
        hs[j] = (int)__builtin_amdgcn_udot4(B, kWB, __builtin_amdgcn_udot4(A, kWA, 0u, false), false);
    }
}

// cvRound of a float (SSE2 cvtsd2si, round half to even).
__device__ inline int cv_round(float v) { return __float2int_rn(v); }

// ORBmatcher::DescriptorDistance (src/ORBmatcher.cc:1794-1810): Hamming
// distance of two 256-bit descriptors = popcount of XOR.
// (one chain of v_bcnt_u32_b32 accumulations, which add their second
// operand; the compiler rebalances a summed form into separate counts and
// add3s: 11 instead of 8 VALU after the xors)
__device__ inline uint32_t bcnt_acc(uint32_t x, uint32_t acc)
{
    uint32_t r;
    asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(acc));
    return r;
}
__device__ inline int hamming256(const uint4& a0, const uint4& a1, const uint4& b0, const uint4& b1)
{
    uint32_t c = __builtin_popcount(a0.x ^ b0.x);
    c = bcnt_acc(a0.y ^ b0.y, c);
    c = bcnt_acc(a0.z ^ b0.z, c);
    c = bcnt_acc(a0.w ^ b0.w, c);
    c = bcnt_acc(a1.x ^ b1.x, c);
    c = bcnt_acc(a1.y ^ b1.y, c);
    c = bcnt_acc(a1.z ^ b1.z, c);
    c = bcnt_acc(a1.w ^ b1.w, c);
    return (int)c;
}

// --------------------------------------------------------------------------
// Block-wide scans / reductions for 256-thread blocks (4 waves).
// --------------------------------------------------------------------------
template <int kW>
struct BlockScratchN {
    int wave[2][kW];
    int vars[8];
};
using BlockScratch = BlockScratchN<kWaves>;

// Wave64 scans / reductions on DPP row shifts + row broadcasts (gfx9):
// VALU-only, no ds_bpermute round trips.  All 64 lanes must be active.
template <int kCtrl, int kRowMask>
__device__ inline int dpp_or0(int v)
{
    return __builtin_amdgcn_update_dpp(0, v, kCtrl, kRowMask, 0xf, false);
}

__device__ inline int wave_inclusive_scan(int v)
{
    v += dpp_or0<0x111, 0xf>(v);   // row_shr:1
    v += dpp_or0<0x112, 0xf>(v);   // row_shr:2
    v += dpp_or0<0x114, 0xf>(v);   // row_shr:4
    v += dpp_or0<0x118, 0xf>(v);   // row_shr:8
    v += dpp_or0<0x142, 0xa>(v);   // row_bcast:15 -> rows 1, 3
    v += dpp_or0<0x143, 0xc>(v);   // row_bcast:31 -> rows 2, 3
    return v;
}

__device__ inline int wave_sum(int v)
{
    return __builtin_amdgcn_readlane(wave_inclusive_scan(v), 63);
}

__device__ inline int wave_max(int v)
{
    v = max(v, __builtin_amdgcn_update_dpp(v, v, 0x111, 0xf, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(v, v, 0x112, 0xf, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(v, v, 0x114, 0xf, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(v, v, 0x118, 0xf, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(v, v, 0x142, 0xa, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(v, v, 0x143, 0xc, 0xf, false));
    return __builtin_amdgcn_readlane(v, 63);
}

// Exclusive prefix of v over threadIdx order; *total = block sum.
template <int kW>
__device__ inline int block_exclusive_scan(int v, int* total, BlockScratchN<kW>& s, int buf)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int inc = wave_inclusive_scan(v);
    if (lane == 63) s.wave[buf][w] = inc;
    __syncthreads();
    int base = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < kW; i++) {
        const int x = s.wave[buf][i];
        base += (i < w) ? x : 0;
        tot += x;
    }
    *total = tot;
    return base + inc - v;
}

template <int kW>
__device__ inline int block_sum(int v, BlockScratchN<kW>& s, int buf)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    v = wave_sum(v);
    if (lane == 0) s.wave[buf][w] = v;
    __syncthreads();
    int t = 0;
#pragma unroll
    for (int i = 0; i < kW; i++) t += s.wave[buf][i];
    return t;
}

template <int kW>
__device__ inline int block_max(int v, BlockScratchN<kW>& s, int buf)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    v = wave_max(v);
    if (lane == 0) s.wave[buf][w] = v;
    __syncthreads();
    int t = s.wave[buf][0];
#pragma unroll
    for (int i = 1; i < kW; i++) t = max(t, s.wave[buf][i]);
    return t;
}

// --------------------------------------------------------------------------
// std::nth_element (libstdc++ 11, bits/stl_algo.h:1964-1986 __introselect)
// replayed exactly on a keypoint list, with the comparator of OpenCV's
// KeyPointsFilter::retainBest (response greater).  Elements are packed
// score<<24 | y<<12 | x; only the score takes part in comparisons, so the
// permutation equals the one libstdc++ applies to the cv::KeyPoint vector
// (src/ORBextractor.cc:683, :699).
//
// The Hoare partition (__unguarded_partition, stl_algo.h:1880-1896) is
// computed block-parallel: with L = ascending positions whose key <= pivot
// and R = descending positions whose key >= pivot, it swaps (L_k, R_k) for
// k = 1..m where m = max_s min(#L before s, #R at/after s), and returns
// L_1 (m == 0) or min(L_{m+1}, R_m).
// --------------------------------------------------------------------------
// XCD-aware block order for a (chunk, frame) grid launched as C x
// roundup(nframes, 8) blocks.  Blocks are dealt round-robin over the 8 XCDs
// (blocks p and p + 8 share one L2; MI355X_MICROARCH.md, workgroup
// dispatch), so frame f's chunks are taken by the blocks p = 8 j + f % 8,
// j = (f / 8) C .. (f / 8 + 1) C - 1: one frame's chunks share an L2 and the
// data they have in common (overlapping rows, patches) is fetched once.
// frame >= nframes marks a padding block (return before any barrier).
struct XcdBlock {
    int chunk, frame;
};
__device__ inline XcdBlock xcd_block()
{
    const int C = gridDim.x;
    const int p = blockIdx.x + C * blockIdx.y, j = p >> 3, g = j / C;
    return {j - g * C, 8 * g + (p & 7)};
}
__host__ inline int xcd_frames(int nframes) { return (nframes + 7) & ~7; }

// Harris entries (scoreType == HARRIS_SCORE) are u64: the order-preserving
// bit image of the float response (harris_key) in the high word, y<<12 | x
// in the low word.
__device__ inline uint32_t kp_key(uint32_t e) { return e >> 24; }
__device__ inline uint32_t kp_key(uint64_t e) { return (uint32_t)(e >> 32); }
template <typename E>
__device__ inline bool kp_greater(E a, E b) { return kp_key(a) > kp_key(b); }
// float -> u32 with a < b (as floats) <=> key(a) < key(b) for finite values
// (-0 is folded onto +0, which compares equal to it)
__host__ __device__ inline uint32_t harris_key(float r)
{
    uint32_t u;
    const float z = r + 0.0f;
    __builtin_memcpy(&u, &z, 4);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__host__ __device__ inline float harris_response(uint32_t k)
{
    const uint32_t u = (k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k;
    float r;
    __builtin_memcpy(&r, &u, 4);
    return r;
}

// libstdc++ bits/stl_heap.h helpers (sequential, thread 0 only).
template <typename E>
__device__ inline void heap_push(E* first, int hole, int top, E value)
{
    int parent = (hole - 1) / 2;
    while (hole > top && kp_greater(first[parent], value)) {
        first[hole] = first[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    first[hole] = value;
}

template <typename E>
__device__ inline void heap_adjust(E* first, int hole, int len, E value)
{
    const int top = hole;
    int second = hole;
    while (second < (len - 1) / 2) {
        second = 2 * (second + 1);
        if (kp_greater(first[second], first[second - 1])) second--;
        first[hole] = first[second];
        hole = second;
    }
    if ((len & 1) == 0 && second == (len - 2) / 2) {
        second = 2 * (second + 1);
        first[hole] = first[second - 1];
        hole = second - 1;
    }
    heap_push(first, hole, top, value);
}

template <typename E>
__device__ inline void heap_select(E* first, int middle, int last)
{
    // __make_heap(first, first+middle)
    if (middle >= 2) {
        int parent = (middle - 2) / 2;
        while (true) {
            heap_adjust(first, parent, middle, first[parent]);
            if (parent == 0) break;
            parent--;
        }
    }
    for (int i = middle; i < last; ++i) {
        if (kp_greater(first[i], first[0])) {
            // __pop_heap(first, first+middle, first+i)
            const E value = first[i];
            first[i] = first[0];
            heap_adjust(first, 0, middle, value);
        }
    }
}

template <typename E>
__device__ inline void insertion_sort(E* a, int first, int last)
{
    if (first == last) return;
    for (int i = first + 1; i < last; ++i) {
        const E val = a[i];
        if (kp_greater(val, a[first])) {
            for (int k = i; k > first; --k) a[k] = a[k - 1];
            a[first] = val;
        } else {
            int k = i;
            while (kp_greater(val, a[k - 1])) {
                a[k] = a[k - 1];
                --k;
            }
            a[k] = val;
        }
    }
}

template <typename E>
__device__ inline void move_median_to_first(E* a, int result, int x, int y, int z)
{
    int t;
    if (kp_greater(a[x], a[y])) {
        if (kp_greater(a[y], a[z])) t = y;
        else if (kp_greater(a[x], a[z])) t = z;
        else t = x;
    } else if (kp_greater(a[x], a[z])) {
        t = x;
    } else if (kp_greater(a[y], a[z])) {
        t = z;
    } else {
        t = y;
    }
    const E tmp = a[result];
    a[result] = a[t];
    a[t] = tmp;
}

// GCC 4.6 .. 4.8's __move_median_first(a, b, c): the median of (a, b, c)
// moved to a, a left in place when it is the median (before PR
// libstdc++/58437; the reference's era).
template <typename E>
__device__ inline void move_median_first_gcc48(E* a, int x, int y, int z)
{
    int t;
    if (kp_greater(a[x], a[y])) {
        if (kp_greater(a[y], a[z])) t = y;
        else if (kp_greater(a[x], a[z])) t = z;
        else return;
    } else if (kp_greater(a[x], a[z])) {
        return;
    } else if (kp_greater(a[y], a[z])) {
        t = z;
    } else {
        t = y;
    }
    const E tmp = a[x];
    a[x] = a[t];
    a[t] = tmp;
}

// introselect's pivot step for [first, last): pivot_mode 0 = libstdc++ >=
// 4.9 (median of first + 1, mid, last - 1 swapped to first), 1 = GCC 4.6 ..
// 4.8 (median of first, mid, last - 1 moved to first); orbx_set_nth_pivot.
template <typename E>
__device__ inline void nth_pivot_step(E* a, int first, int last, int pivot_mode)
{
    const int mid = first + (last - first) / 2;
    if (pivot_mode == 1) move_median_first_gcc48(a, first, mid, last - 1);
    else move_median_to_first(a, first, first + 1, mid, last - 1);
}

// Partition [lo+1, hi) around the pivot key at a[lo]; returns the cut.
// pos: scratch of 2 * ((hi-lo)/2 + 1) ints.  Must be called by all threads.
__device__ inline int block_hoare_partition(uint32_t* a, int lo, int hi, int* pos, BlockScratch& s)
{
    int* posR = pos;
    int* posL = pos + (hi - lo) / 2 + 1;
    const int tid = threadIdx.x;
    const uint32_t P = kp_key(a[lo]);
    const int len = hi - lo - 1;
    const int chunk = (len + kBlock - 1) / kBlock;
    const int s0 = min(lo + 1 + tid * chunk, hi), s1 = min(s0 + chunk, hi);
    int nle = 0, nge = 0;
    for (int x = s0; x < s1; x++) {
        const uint32_t k = kp_key(a[x]);
        nle += (k <= P);
        nge += (k >= P);
    }
    int tot_le, tot_ge;
    const int le_before = block_exclusive_scan(nle, &tot_le, s, 0);
    const int ge_before = block_exclusive_scan(nge, &tot_ge, s, 1);
    const int ge_after_chunk = tot_ge - ge_before - nge;   // #ge in chunks after this one
    // m = max over splits of min(CL, CR)
    int cl = le_before, cr = ge_after_chunk + nge, best = 0;
    for (int x = s0; x < s1; x++) {
        best = max(best, min(cl, cr));
        const uint32_t k = kp_key(a[x]);
        cl += (k <= P);
        cr -= (k >= P);
    }
    best = max(best, min(cl, cr));
    __syncthreads();   // scan scratch reuse
    const int m = block_max(best, s, 0);
    // locate R_k (k <= m), L_{m+1}, R_m, L_1
    if (tid == 0) {
        s.vars[0] = 0x7fffffff;   // L_{m+1}
        s.vars[1] = -1;           // R_m
        s.vars[2] = 0x7fffffff;   // L_1
    }
    __syncthreads();
    cl = le_before;
    cr = ge_after_chunk + nge;
    for (int x = s0; x < s1; x++) {
        const uint32_t k = kp_key(a[x]);
        if (k <= P) {
            cl++;
            if (cl <= m) posL[cl - 1] = x;
            if (cl == m + 1) s.vars[0] = x;
            if (cl == 1) s.vars[2] = x;
        }
        if (k >= P) {
            if (cr <= m) posR[cr - 1] = x;
            if (cr == m) s.vars[1] = x;
            cr--;
        }
    }
    __syncthreads();
    // swaps (L_k, R_k), k = 1..m: disjoint pairs, positions fixed above
    for (int k = tid; k < m; k += kBlock) {
        const int i = posL[k], j = posR[k];
        const uint32_t t = a[i];
        a[i] = a[j];
        a[j] = t;
    }
    const int cut = (m == 0) ? s.vars[2] : min(s.vars[0], s.vars[1]);
    __syncthreads();
    return cut;
}

__device__ inline int floor_log2(int n)
{
    return 31 - __clz(n);
}

// std::nth_element(a, a + nth, a + n, greater-by-response).
// pos: scratch of n + 4 ints.
__device__ inline void block_nth_element(uint32_t* a, int n, int nth, int* pos, BlockScratch& s, int pivot_mode = 0)
{
    if (n == 0 || nth == n) return;
    int first = 0, last = n;
    int depth = 2 * floor_log2(n);
    while (last - first > 3) {
        if (depth == 0) {
            if (threadIdx.x == 0) {
                heap_select(a + first, nth + 1 - first, last - first);
                const uint32_t t = a[first];
                a[first] = a[nth];
                a[nth] = t;
            }
            __syncthreads();
            return;
        }
        --depth;
        if (threadIdx.x == 0) nth_pivot_step(a, first, last, pivot_mode);
        __syncthreads();
        const int cut = block_hoare_partition(a, first, last, pos, s);
        if (cut <= nth) first = cut;
        else last = cut;
    }
    if (threadIdx.x == 0) insertion_sort(a, first, last);
    __syncthreads();
}

// --------------------------------------------------------------------------
// Wave-level (64 lanes, no block barriers) variants of the partition and
// nth_element above, for lists held in a wave-private LDS buffer.
// --------------------------------------------------------------------------
__device__ inline void lds_wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Ordering point for a wave working on a list in global memory (same CU:
// workgroup scope keeps the CU's L1 coherent with its own stores).
__device__ inline void global_wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

template <bool kGlobal>
__device__ inline void nth_sync()
{
    if constexpr (kGlobal) global_wave_sync();
    else lds_wave_sync();
}

__device__ inline int wave_min_int(int v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
    return v;
}

template <bool kGlobal = false, typename E>
__device__ inline int wave_hoare_partition(E* a, int lo, int hi, int* pos)
{
    int* posR = pos;
    int* posL = pos + (hi - lo) / 2 + 1;
    const int lane = threadIdx.x & 63;
    const uint32_t P = kp_key(a[lo]);
    const int len = hi - lo - 1;
    const int chunk = (len + 63) / 64;
    const int s0 = min(lo + 1 + lane * chunk, hi), s1 = min(s0 + chunk, hi);
    int nle = 0, nge = 0;
    for (int x = s0; x < s1; x++) {
        const uint32_t k = kp_key(a[x]);
        nle += (k <= P);
        nge += (k >= P);
    }
    // both prefix counts in one scan (16-bit halves) when they fit
    int le_incl, ge_incl;
    if (len < 65536) {
        const int both = wave_inclusive_scan(nle | (nge << 16));
        le_incl = both & 0xFFFF;
        ge_incl = (int)((uint32_t)both >> 16);
    } else {
        le_incl = wave_inclusive_scan(nle);
        ge_incl = wave_inclusive_scan(nge);
    }
    const int tot_ge = __builtin_amdgcn_readlane(ge_incl, 63);
    const int le_before = le_incl - nle;
    const int ge_after_chunk = tot_ge - ge_incl;
    int cl = le_before, cr = ge_after_chunk + nge, best = 0;
    for (int x = s0; x < s1; x++) {
        best = max(best, min(cl, cr));
        const uint32_t k = kp_key(a[x]);
        cl += (k <= P);
        cr -= (k >= P);
    }
    best = max(best, min(cl, cr));
    const int m = wave_max(best);
    int lm1 = 0x7fffffff, rm = -1, l1 = 0x7fffffff;
    cl = le_before;
    cr = ge_after_chunk + nge;
    for (int x = s0; x < s1; x++) {
        const uint32_t k = kp_key(a[x]);
        if (k <= P) {
            cl++;
            if (cl <= m) posL[cl - 1] = x;
            if (cl == m + 1) lm1 = x;
            if (cl == 1) l1 = x;
        }
        if (k >= P) {
            if (cr <= m) posR[cr - 1] = x;
            if (cr == m) rm = x;
            cr--;
        }
    }
    // L_{m+1}, L_1 and R_m each lie in exactly one lane's chunk (or none):
    // read them from that lane instead of reducing over the wave
    auto from_lane = [](int v, bool have, int none) {
        const unsigned long long b = __ballot(have);
        return b ? __builtin_amdgcn_readlane(v, (int)__builtin_ctzll(b)) : none;
    };
    lm1 = from_lane(lm1, lm1 != 0x7fffffff, 0x7fffffff);
    l1 = from_lane(l1, l1 != 0x7fffffff, 0x7fffffff);
    rm = from_lane(rm, rm >= 0, -1);
    nth_sync<kGlobal>();
    for (int k = lane; k < m; k += 64) {
        const int i = posL[k], j = posR[k];
        const E t = a[i];
        a[i] = a[j];
        a[j] = t;
    }
    nth_sync<kGlobal>();
    return (m == 0) ? l1 : min(lm1, rm);
}

// std::nth_element(a, a + nth, a + n, greater-by-response), one wave.
// kGlobal: list and scratch in global memory (lists too long for LDS).
template <bool kGlobal = false, typename E>
__device__ inline void wave_nth_element(E* a, int n, int nth, int* pos, int pivot_mode = 0)
{
    if (n == 0 || nth == n) return;
    const int lane = threadIdx.x & 63;
    int first = 0, last = n;
    int depth = 2 * floor_log2(n);
    while (last - first > 3) {
        if (depth == 0) {
            if (lane == 0) {
                heap_select(a + first, nth + 1 - first, last - first);
                const E t = a[first];
                a[first] = a[nth];
                a[nth] = t;
            }
            nth_sync<kGlobal>();
            return;
        }
        --depth;
        if (lane == 0) nth_pivot_step(a, first, last, pivot_mode);
        nth_sync<kGlobal>();
        const int cut = wave_hoare_partition<kGlobal>(a, first, last, pos);
        if (cut <= nth) first = cut;
        else last = cut;
    }
    if (lane == 0) insertion_sort(a, first, last);
    nth_sync<kGlobal>();
}

}  // namespace orbx
