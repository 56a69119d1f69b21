// ORB extraction on MI355X (gfx950): ORBextractor::operator()
// (src/ORBextractor.cc:718-779) for a batch of frames, one launch per stage:
//
//   k_pyr_level0   copyMakeBorder(REFLECT_101) of the input   (:814)
//   k_pyr_resize   resize INTER_LINEAR + border, level l      (:800, :806)
//   k_fast_cells   FAST-9/16 + cell-local NMS + threshold-7
//                  fallback + raster-order compaction, one
//                  workgroup per grid cell                    (:599-614)
//   k_harris_cells HarrisResponses of every FAST corner (HARRIS_SCORE
//                  only), u64 entries keyed by the float response (:616-620)
//   k_retain_cells per-level quota redistribution + cell retainBest,
//                  one wave per cell (libstdc++ introselect)  (:622-694)
//   k_retain_levels level retainBest, one wave per level      (:697-701)
//   k_blur         GaussianBlur 7x7 sigma 2 on each level     (:760)
//   k_describe     IC_Angle + rBRIEF + coordinate scaling,
//                  one wave per keypoint                      (:124-194, :705,
//                                                              :764-777)
//
// All integer / byte work; the bounds are HBM or latency, never MFMA.
#include <algorithm>
#include <type_traits>

#include "orbx_device.h"
#include "orbx_internal.h"

namespace orbx {

constexpr size_t kRetainLds = 128 * 1024;   // LDS budget of a retain block
constexpr int kRetainCellCap = 512;         // cell lists up to this length sort in LDS
constexpr int kSplitMinFrames = 16;         // batches >= 2x this run as two concurrent halves
constexpr size_t kResizeLds = 96 * 1024;    // LDS budget of a staged resize strip

__constant__ __attribute__((aligned(4))) int8_t c_pattern[256][4] = {
#include "orbx_pattern.inc"
};

#ifdef ORBX_FAST_PROFILE
__device__ unsigned long long g_fast_prof[16];
__device__ inline unsigned long long fp_stamp()
{
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
#define FP_T0() unsigned long long _ft = fp_stamp()
#define FP_MARK(k)                                                                  \
    do {                                                                            \
        const unsigned long long _n = fp_stamp();                                   \
        if (threadIdx.x == 0) atomicAdd(&g_fast_prof[k], _n - _ft);                 \
        _ft = _n;                                                                   \
    } while (0)
#define FP_ADD(k, v) atomicAdd(&g_fast_prof[k], (unsigned long long)(v))
extern "C" int orbx_debug_fast_prof(unsigned long long* out)
{
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fast_prof), sizeof(unsigned long long) * 16) == hipSuccess ? 0 : -2;
}
#else
#define FP_T0()
#define FP_MARK(k)
#define FP_ADD(k, v)
#endif

struct ExtractArgs {
    const LevelGeom* levels;
    const CellGeom* cells;
    const ResizeCol* res_cols;
    const ResizeRow* res_rows;
    const int* umax;
    const uint8_t* frames;
    uint8_t* pyr_raw;
    uint8_t* pyr_blur;
    uint32_t* cell_lists;
    int32_t* cell_count;
    uint32_t* level_keys;
    int32_t* level_count;
    orbx_keypoint* out_kps;
    uint8_t* out_desc;
    int32_t* out_n;
    int32_t* error_flags;
    // orbx_extract's single frame: k_describe also writes the page-locked
    // read-back block (count and flags at 0, records at 64, descriptors
    // after nfeatures records), in place of a pack launch; else null
    uint8_t* host_out;
    int32_t* retain_scratch;        // slots x (list_entries + 4 ncells): global nth_element scratch
    const int4* blur_tiles;         // k_blur work blocks (also the blur tail of k_fast_cells<..., true>)
    uint64_t* cell_keys64;          // HARRIS_SCORE: Harris-keyed cell lists (as cell_lists)
    uint64_t* level_keys64;         // HARRIS_SCORE: Harris-keyed level lists (as level_keys)
    int harris;                     // scoreType == HARRIS_SCORE
    int fp_contract;                // orbx_set_fp_contract: FMA-contracted reference build
    int nth_pivot;                  // orbx_set_nth_pivot: retainBest's libstdc++ era
    long long frame_pyr_bytes;
    int first_slot;
    int w, h;
    int nlevels, ncells, list_entries, level_entries, nfeatures;
    int fast_th, fast_th_low;       // FAST thresholds (fastTh, 7), clamped
    int max_list_cap, max_level_cap;
};

// The geometry tables (cells, levels, ...) are never written by a kernel:
// read through the constant address space, a wave-uniform read is a scalar
// load (scalar cache hit once warm) instead of a vector load + readfirstlane,
// so the dependent table reads in front of a workgroup's first data loads
// cost cache hits rather than L2 round trips.
template <class T>
__device__ __forceinline__ T cget(const T* p, int i)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return ((const __attribute__((address_space(4))) T*)p)[i];
#else
    return p[i];   // host pass: parsed, never called
#endif
}

__device__ inline uint8_t sat_u8(int v) { return (uint8_t)min(max(v, 0), 255); }
__device__ inline int sat_s16(int v) { return min(max(v, -32768), 32767); }

// (row, column) walk of a row-major index advancing by a fixed stride,
// without a division per step.
struct RowWalk {
    int r, q, dr, dq, nq;
    __device__ RowWalk(int start, int stride, int n_q) : nq(n_q)
    {
        // callers never pass n_q == 0 (integer division by zero is undefined
        // behaviour, which the compiler may assume away)
        r = start / n_q;
        q = start - r * n_q;
        dr = stride / n_q;
        dq = stride - dr * n_q;
    }
    __device__ void next()
    {
        r += dr;
        q += dq;
        if (q >= nq) {
            q -= nq;
            r++;
        }
    }
};


// Copy n items into LDS, kBatch per thread per round: the loads are
// unconditional (index clamped to n - 1, whose entry out-of-range lanes
// rewrite with its own value), so no branch separates them and all kBatch
// are in flight before the first wait.
template <int kBatch, typename T, typename Load>
__device__ inline void stage_to_lds(T* dst, int n, int tid, int nthr, Load load)
{
    for (int u0 = 0; u0 < n; u0 += kBatch * nthr) {
        T v[kBatch];
#pragma unroll
        for (int k = 0; k < kBatch; k++) v[k] = load(min(u0 + k * nthr + tid, n - 1));
#pragma unroll
        for (int k = 0; k < kBatch; k++) dst[min(u0 + k * nthr + tid, n - 1)] = v[k];
    }
}

// ---------------------------------------------------------------------------
// Level 0: padded copy with BORDER_REFLECT_101.  16 output bytes per thread
// and row: interior words are two aligned 16-byte loads funnel-shifted by
// the border offset; words touching the border gather reflected bytes.
// ---------------------------------------------------------------------------
// One thread per (16-byte column, strip of kPyrRows rows): the strip's
// independent row loads are in flight together.
constexpr int kPyrRows = 8;
constexpr int kPyr0Shift = (16 - kEdge % 16) % 16;   // (16q - kEdge) mod 16

// Work items: first the interior words (q_lo .. q_lo + nint - 1) in strips of
// kPyrRows rows, then the border words one (word, row) each, so border
// gathers run in waves of their own.
__global__ __launch_bounds__(256) void k_pyr_level0(ExtractArgs a, int q_lo, int nint)
{
    const int f = blockIdx.y;
    const LevelGeom L = cget(a.levels, 0);
    const int qpr = L.stride >> 4, nstrips = (L.ph + kPyrRows - 1) / kPyrRows;
    const int nbord = qpr - nint;
    int idx = blockIdx.x * blockDim.x + threadIdx.x;
    const uint8_t* src = a.frames + (size_t)(a.first_slot + f) * a.w * a.h;
    uint8_t* dst = a.pyr_raw + (size_t)f * a.frame_pyr_bytes + L.off;
    if (idx < nint * nstrips) {
        const int strip = idx / nint, q = q_lo + (idx - strip * nint), px0 = 16 * q;
        const int al = px0 - kEdge - kPyr0Shift;   // 16-byte aligned source column
        const int py_first = strip * kPyrRows;
        // all the strip's loads first (rows past the level repeat the last
        // one, their stores are skipped), then the funnel shifts and stores
        uint4 lo[kPyrRows], hi[kPyrRows];
#pragma unroll
        for (int rr = 0; rr < kPyrRows; rr++) {
            const int py = min(py_first + rr, L.ph - 1);
            const uint8_t* row = src + (size_t)reflect101(py - kEdge, L.h) * a.w + al;
            lo[rr] = *reinterpret_cast<const uint4*>(row);
            hi[rr] = *reinterpret_cast<const uint4*>(row + 16);
        }
#pragma unroll
        for (int rr = 0; rr < kPyrRows; rr++) {
            const uint32_t w[8] = {lo[rr].x, lo[rr].y, lo[rr].z, lo[rr].w, hi[rr].x, hi[rr].y, hi[rr].z, hi[rr].w};
            constexpr int d = kPyr0Shift >> 2, b = kPyr0Shift & 3;
            uint32_t o[4];
#pragma unroll
            for (int k = 0; k < 4; k++)
                o[k] = b ? __builtin_amdgcn_alignbyte(w[k + d + 1], w[k + d], b) : w[k + d];
            if (py_first + rr < L.ph)
                *reinterpret_cast<uint4*>(dst + (size_t)(py_first + rr) * L.stride + px0) = make_uint4(o[0], o[1], o[2], o[3]);
        }
        return;
    }
    idx -= nint * nstrips;
    if (idx >= nbord * L.ph) return;
    const int py = idx / nbord, k = idx - py * nbord;
    const int q = k < q_lo ? k : k + nint, px0 = 16 * q;
    const uint8_t* row = src + (size_t)reflect101(py - kEdge, L.h) * a.w;
    if (kEdge == 16 && a.w % 16 == 0 && a.w >= 32) {
        // aligned rows: the left border word is frame bytes 16 .. 1, the word
        // after the last 16 interior bytes is bytes w-2 .. w-17 (byte permutes
        // of two aligned loads), the rest of the row is zero
        const int w16 = a.w >> 4;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (q == 0) {
            const uint4 A = *reinterpret_cast<const uint4*>(row), B = *reinterpret_cast<const uint4*>(row + 16);
            v.x = __builtin_amdgcn_perm(B.x, A.w, 0x01020304u);
            v.y = __builtin_amdgcn_perm(A.w, A.z, 0x01020304u);
            v.z = __builtin_amdgcn_perm(A.z, A.y, 0x01020304u);
            v.w = __builtin_amdgcn_perm(A.y, A.x, 0x01020304u);
        } else if (q <= w16) {
            v = *reinterpret_cast<const uint4*>(row + 16 * (q - 1));
        } else if (q == w16 + 1) {
            const uint4 A = *reinterpret_cast<const uint4*>(row + a.w - 32), B = *reinterpret_cast<const uint4*>(row + a.w - 16);
            v.x = __builtin_amdgcn_perm(B.w, B.z, 0x03040506u);
            v.y = __builtin_amdgcn_perm(B.z, B.y, 0x03040506u);
            v.z = __builtin_amdgcn_perm(B.y, B.x, 0x03040506u);
            v.w = __builtin_amdgcn_perm(B.x, A.w, 0x03040506u);
        }
        *reinterpret_cast<uint4*>(dst + (size_t)py * L.stride + px0) = v;
        return;
    }
    uint8_t v[16];
#pragma unroll
    for (int i = 0; i < 16; i++) v[i] = px0 + i < L.pw ? row[reflect101(px0 + i - kEdge, L.w)] : 0;
    uint32_t o[4];
#pragma unroll
    for (int i = 0; i < 4; i++)
        o[i] = v[4 * i] | (uint32_t)v[4 * i + 1] << 8 | (uint32_t)v[4 * i + 2] << 16 | (uint32_t)v[4 * i + 3] << 24;
    *reinterpret_cast<uint4*>(dst + (size_t)py * L.stride + px0) = make_uint4(o[0], o[1], o[2], o[3]);
}

// ---------------------------------------------------------------------------
// Level l >= 1: cv::resize INTER_LINEAR from level l-1 (fixed point, 11-bit
// weights; columns < nvec use the SSE2 VResizeLinearVec_32s8u arithmetic,
// the rest the scalar FixedPtCast<int,uchar,22>), then copyMakeBorder
// REFLECT_101 of the level itself (border pixels recompute their source).
// ---------------------------------------------------------------------------
__device__ inline uint8_t resize_pixel(const uint8_t* prev, int pstride, const ResizeCol& c,
                                       const ResizeRow& r, bool vec)
{
    const uint8_t* r0 = prev + (size_t)r.sy0 * pstride;
    const uint8_t* r1 = prev + (size_t)r.sy1 * pstride;
    const int S0 = r0[c.sx0] * c.a0 + r0[c.sx1] * c.a1;
    const int S1 = r1[c.sx0] * c.a0 + r1[c.sx1] * c.a1;
    if (vec) {
        const int x0 = sat_s16(S0 >> 4), y0 = sat_s16(S1 >> 4);
        int v = sat_s16(((x0 * r.b0) >> 16) + ((y0 * r.b1) >> 16));
        v = sat_s16(v + 2) >> 2;
        return sat_u8(v);
    }
    return sat_u8((S0 * r.b0 + S1 * r.b1 + (1 << 21)) >> 22);
}

__global__ __launch_bounds__(256) void k_pyr_resize(ExtractArgs a, int level)
{
    const int f = blockIdx.y;
    const LevelGeom L = cget(a.levels, level);
    const LevelGeom P = cget(a.levels, level - 1);
    const int wpr = L.stride >> 2, nstrips = (L.ph + kPyrRows - 1) / kPyrRows;
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= wpr * nstrips) return;
    const int strip = idx / wpr, q = idx - strip * wpr, px0 = 4 * q;
    const uint8_t* prev = a.pyr_raw + (size_t)f * a.frame_pyr_bytes + P.off + (size_t)kEdge * P.stride + kEdge;
    uint8_t* dst = a.pyr_raw + (size_t)f * a.frame_pyr_bytes + L.off;
    ResizeCol c[4];
    bool vec[4], on[4];
#pragma unroll
    for (int b = 0; b < 4; b++) {
        on[b] = px0 + b < L.pw;
        const int x = on[b] ? reflect101(px0 + b - kEdge, L.w) : 0;
        c[b] = a.res_cols[L.res_col_off + x];
        vec[b] = x < L.nvec_resize;
    }
#pragma unroll
    for (int rr = 0; rr < kPyrRows; rr++) {
        const int py = min(strip * kPyrRows + rr, L.ph - 1);
        const ResizeRow r = a.res_rows[L.res_row_off + reflect101(py - kEdge, L.h)];
        uint32_t word = 0;
#pragma unroll
        for (int b = 0; b < 4; b++)
            if (on[b]) word |= (uint32_t)resize_pixel(prev, P.stride, c[b], r, vec[b]) << (8 * b);
        if (strip * kPyrRows + rr < L.ph) *reinterpret_cast<uint32_t*>(dst + (size_t)py * L.stride + px0) = word;
    }
}

// The same resize with the strip's source rows staged in LDS: one
// workgroup per (strip of kResRows output rows, frame).  The previous
// level's rows [lo, hi] feeding the strip are copied with 16-byte loads
// (padded columns 0 .. kEdge + P.w), together with the level's column and
// row tables; every output pixel then reads its 2x2 sources from LDS.
// The host guarantees hi - lo + 1 <= L.res_span (computed from the tables).
// The level's and its parent's geometry, passed by value: no dependent
// table read before the staging loads.
struct ResizeLevel {
    long long off, poff;                 // level / parent offsets in a frame's pyramid
    int stride, pstride, w, h, pw, ph, ph_parent_h, nvec, span, strip_off, row_off, col_off;
    int packed;                          // every interior word's taps lie within 8 bytes (the packed form applies)
};

__global__ __launch_bounds__(256) void k_pyr_resize_lds(ExtractArgs a, ResizeLevel L, int pitch)
{
    extern __shared__ uint4 s_dyn[];
    __shared__ ResizeRow s_rows[kResRows];
    const int f = blockIdx.y, tid = threadIdx.x;
    const int py0 = blockIdx.x * kResRows, nrows = min(kResRows, L.ph - py0);
    const int nch = pitch >> 4;
    ResizeCol* s_cols = reinterpret_cast<ResizeCol*>(s_dyn + (size_t)L.span * nch);
    uint8_t* s_src = reinterpret_cast<uint8_t*>(s_dyn);
    // the strip's first source row comes from a host table (uniform scalar
    // load), so the staging loads go out together with the row/column tables
    const int lo = a.res_rows[L.strip_off + blockIdx.x].sy0;
    if (tid < nrows) s_rows[tid] = a.res_rows[L.row_off + reflect101(py0 + tid - kEdge, L.h)];
    stage_to_lds<4>(s_cols, L.w, tid, (int)blockDim.x, [&](int x) { return a.res_cols[L.col_off + x]; });
    const int nsrc = min(L.span, L.ph_parent_h - lo);
    const uint8_t* pbase = a.pyr_raw + (size_t)f * a.frame_pyr_bytes + L.poff + (size_t)(lo + kEdge) * L.pstride;
#ifndef RES_NO_STAGE
    {
        // u / nch as a float product: (u + 1/2) / nch lies at least 1/(2 nch)
        // from an integer and the product errs by < 2^-21 (u + 1) for
        // u < 2^16 (no integer division per item)
        const float inv = 1.0f / (float)nch;
        stage_to_lds<8>(s_dyn, nsrc * nch, tid, (int)blockDim.x, [&](int u) {
            const int r = (int)(((float)u + 0.5f) * inv), c = u - r * nch;
            return *reinterpret_cast<const uint4*>(pbase + (size_t)r * L.pstride + 16 * c);
        });
    }
#endif
    __syncthreads();
    uint8_t* dst = a.pyr_raw + (size_t)f * a.frame_pyr_bytes + L.off + (size_t)py0 * L.stride;
#ifdef RES_NO_COMPUTE
    if (tid < 64) reinterpret_cast<uint32_t*>(dst)[tid] = s_src[tid * 7];
    return;
#endif
    // Output words split by form (no wave runs both):
    //  * interior words [q_lo, q_hi) whose four columns are on the SSE2 path
    //    (x < nvec): the packed form below, one thread per word sliding
    //    down the strip's rows;
    //  * the rest -- the reflected border words, the scalar-tail columns
    //    x >= nvec and the row padding -- one (row, word) item per thread,
    //    in the general form.
    // sx1 is sx0 + 1, or sx0 with a1 = 0 (HResizeLinear tail), so the
    // second tap is always read at offset +1.
    const int nq = L.stride >> 2;
    const int q_lo = (kEdge + 3) >> 2, q_hi = L.packed ? max(q_lo, (kEdge + min(L.w, L.nvec)) >> 2) : q_lo;
    const int nfast = q_hi - q_lo;
    // Packed form: a word's four source taps lie in 8 bytes (source step
    // < 2, so sx0(x + 3) - sx0(x) <= 6); three dword reads aligned to the
    // word's first tap (alignbyte) hold them, each column's (p0, p1) pair is
    // one v_perm into 16-bit halves and its 2-tap sum one v_dot2_u32_u16 with
    // weights (16 a0, 16 a1) -- 16 S, whose bits 8..23 are (S >> 4) << 8 --
    // and VResizeLinearVec_32s8u's (S >> 4) * b >> 16 is one
    // v_mul_hi_u32_u24 of that with b << 8.  S >> 4 <= 32640 and the
    // weights are <= 2048, so none of its 16-bit saturations can trigger;
    // the rounded row weights sum to 2048 +- 1 (cvRound of complementary
    // values), so the two terms sum to <= 32640 * 2049 / 2^16 < 1021, the
    // final (t + 2) >> 2 is <= 255 and its u8 saturation is a no-op.
    typedef unsigned short orbx_us2 __attribute__((ext_vector_type(2)));
    auto mh = [](uint32_t x, uint32_t y) {   // bits 32..47 of the 24 x 24-bit product
        return (uint32_t)(((unsigned long long)(x & 0xFFFFFFu) * (unsigned long long)(y & 0xFFFFFFu)) >> 32);
    };
    for (int t = tid; t < nfast; t += blockDim.x) {
        const int q = q_lo + t, x0 = 4 * q - kEdge;
        int ca[4];
        uint32_t sel[4], wgt[4];
#pragma unroll
        for (int b = 0; b < 4; b++) {
            const ResizeCol c = s_cols[x0 + b];
            ca[b] = kEdge + c.sx0;
            wgt[b] = (uint32_t)(16 * c.a0) | (uint32_t)(16 * c.a1) << 16;
        }
        const int qa = ca[0] & ~3, sh = ca[0] & 3;
#pragma unroll
        for (int b = 0; b < 4; b++) {
            const uint32_t r = (uint32_t)(ca[b] - ca[0]);   // tap bytes r, r + 1 of the aligned 8 (L.packed)
            sel[b] = r | 0x0C00u | (r + 1) << 16 | 0x0C000000u;
        }
        auto hrow = [&](int sy, uint32_t (&S)[4]) {
            const uint32_t* d = reinterpret_cast<const uint32_t*>(s_src + (sy - lo) * pitch + qa);
            const uint32_t d0 = d[0], d1 = d[1], d2 = d[2];
            const uint32_t w0 = __builtin_amdgcn_alignbyte(d1, d0, sh), w1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
#pragma unroll
            for (int b = 0; b < 4; b++)
                S[b] = __builtin_amdgcn_udot2(__builtin_bit_cast(orbx_us2, __builtin_amdgcn_perm(w1, w0, sel[b])),
                                              __builtin_bit_cast(orbx_us2, wgt[b]), 0u, false) &
                       0x00FFFF00u;
        };
        uint32_t H0[4], H1[4];
        int c0 = -1, c1 = -1;
        // the next row's table entry is read while this row is computed
        uint2 nxt = reinterpret_cast<const uint2*>(s_rows)[0];
        for (int rr = 0; rr < nrows; rr++) {
            const uint2 cur = nxt;
            if (rr + 1 < nrows) nxt = reinterpret_cast<const uint2*>(s_rows)[rr + 1];
            const uint32_t w0 = __builtin_amdgcn_readfirstlane(cur.x), w1 = __builtin_amdgcn_readfirstlane(cur.y);
            const int sy0 = (int)(int16_t)(w0 & 0xFFFF), sy1 = (int)(int16_t)(w0 >> 16);
            const uint32_t B0 = (w1 & 0xFFFFu) << 8, B1 = (w1 >> 16) << 8;
            uint32_t A[4], B[4];
            if (sy0 == c1) {
#pragma unroll
                for (int b = 0; b < 4; b++) A[b] = H1[b];
            } else if (sy0 == c0) {
#pragma unroll
                for (int b = 0; b < 4; b++) A[b] = H0[b];
            } else {
                hrow(sy0, A);
            }
            if (sy1 == sy0) {
#pragma unroll
                for (int b = 0; b < 4; b++) B[b] = A[b];
            } else if (sy1 == c1) {
#pragma unroll
                for (int b = 0; b < 4; b++) B[b] = H1[b];
            } else {
                hrow(sy1, B);
            }
#pragma unroll
            for (int b = 0; b < 4; b++) {
                H0[b] = A[b];
                H1[b] = B[b];
            }
            c0 = sy0;
            c1 = sy1;
            uint32_t word = 0;
#pragma unroll
            for (int b = 0; b < 4; b++) word |= ((mh(A[b], B0) + mh(B[b], B1) + 2) >> 2) << (8 * b);
            *reinterpret_cast<uint32_t*>(dst + (size_t)rr * L.stride + 4 * q) = word;
        }
    }
    // the other words, one (row, word) each
    const int nslow = nq - nfast;
    for (int item = tid; item < nrows * nslow; item += blockDim.x) {
        const int rr = item / nslow, k = item - rr * nslow;
        const int q = k < q_lo ? k : k + nfast, px0 = 4 * q;
        const ResizeRow R = s_rows[rr];
        uint32_t word = 0;
#pragma unroll
        for (int b = 0; b < 4; b++) {
            if (px0 + b >= L.pw) continue;   // row padding: zero
            const int x = reflect101(px0 + b - kEdge, L.w);
            const ResizeCol c = s_cols[x];
            const uint8_t* r0 = s_src + (R.sy0 - lo) * pitch + kEdge + c.sx0;
            const uint8_t* r1 = s_src + (R.sy1 - lo) * pitch + kEdge + c.sx0;
            const int S0 = r0[0] * c.a0 + r0[1] * c.a1, S1 = r1[0] * c.a0 + r1[1] * c.a1;
            int v;
            if (x < L.nvec)
                v = (((S0 >> 4) * R.b0 >> 16) + ((S1 >> 4) * R.b1 >> 16) + 2) >> 2;
            else   // FixedPtCast<int, uchar, 22>
                v = (S0 * R.b0 + S1 * R.b1 + (1 << 21)) >> 22;
            word |= (uint32_t)sat_u8(v) << (8 * b);
        }
        *reinterpret_cast<uint32_t*>(dst + (size_t)rr * L.stride + px0) = word;
    }
}

// ---------------------------------------------------------------------------
// The whole raw pyramid in one launch: ComputePyramid (src/ORBextractor.cc:
// 781-822) as a cascade of row bands.  One workgroup per (band, frame) walks
// the levels: level 0's rows come from the frame, level l's from level
// l - 1's rows in LDS (ping-pong buffers, each row in the padded layout), so
// no level waits for another launch.  Per (band, level) the host plan gives
// the padded rows the band writes (a partition of the level) and the ROI
// rows it computes: those rows' sources plus every ROI row the band's share
// of the next level reads (a few halo rows are computed by two bands, with
// the same arithmetic).  Each ROI pixel is the staged resize's (the row /
// column tables, the SSE2 column path and the scalar tail), the border
// pixels copyMakeBorder's REFLECT_101 copies of it, bytes past the padded
// width zero: the buffers equal the staged launches', byte for byte.
// plan[band * nlevels + l] = (first owned ROI row, end, first computed ROI
// row, last computed ROI row); a band writes its owned rows' padded rows and
// the border rows that reflect to them.
// ---------------------------------------------------------------------------
// T threads per workgroup: 256 in batches (several bands per CU), 1024 for
// orbx_extract's single frame, whose ~23 bands leave most CUs idle: more
// threads per band shorten each level's row loop.
#ifndef ORBX_CASCADE_SINGLE_THREADS
#define ORBX_CASCADE_SINGLE_THREADS 1024
#endif
#ifdef ORBX_CASC_PROFILE
// diagnostic: band 0's cycles per (level, phase): 0 resize or level-0 load,
// 1 first barrier, 2 border pass + second barrier, 3 pyramid stores
__device__ unsigned long long g_casc_prof[kMaxLevels][4];
#define CASC_T0() unsigned long long _ct = __builtin_readcyclecounter()
#define CASC_MARK(l, k)                                                          \
    do {                                                                         \
        const unsigned long long _n = __builtin_readcyclecounter();              \
        if (blockIdx.x == 0 && threadIdx.x == 0) g_casc_prof[l][k] += _n - _ct;  \
        _ct = _n;                                                                \
    } while (0)
extern "C" int orbx_debug_casc_prof(unsigned long long* out)
{
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_casc_prof), sizeof(g_casc_prof)) == hipSuccess ? 0 : -2;
}
#else
#define CASC_T0()
#define CASC_MARK(l, k)
#endif
// kTab (the single-frame instance): every level's column table and the
// band's row-table slices are staged in LDS at tab_off (tab_cols entries,
// then the rows) with the level-0 loads, so no level's row loop waits on a
// global table load per row (band 0's stamps: 4-5 dependent ~2 k-cycle
// loads per group at levels 1-3 before).
template <int T>
__global__ __launch_bounds__(T) void k_pyr_cascade(ExtractArgs a, const int4* plan, int buf_x, int tab_off,
                                                   int tab_cols)
{
    CASC_T0();
    const bool kTab = T >= 1024 && tab_off > 0;   // tab_off 0: tables too large for LDS, read from HBM
    extern __shared__ uint4 s_dyn[];
    uint8_t* const lds = reinterpret_cast<uint8_t*>(s_dyn);   // buffers: [0, buf_x) even levels, then odd
    const int band = blockIdx.x, f = blockIdx.y, tid = threadIdx.x;
    uint8_t* pyr = a.pyr_raw + (size_t)f * a.frame_pyr_bytes;
    const uint8_t* img = a.frames + (size_t)(a.first_slot + f) * a.w * a.h;
    ResizeCol* const t_cols = reinterpret_cast<ResizeCol*>(lds + tab_off);
    ResizeRow* const t_rows = reinterpret_cast<ResizeRow*>(t_cols + tab_cols);
    if (kTab) {
        // flat index over the levels' column tables, then the band's row
        // slices; four loads in flight per thread before the stores
        int ncol = 0, nrow = 0;
        for (int l = 1; l < a.nlevels; l++) {
            const int4 pl = plan[band * a.nlevels + l];
            ncol += cget(a.levels, l).w;
            nrow += max(0, pl.w - pl.z + 1);
        }
        const int n = ncol + nrow;
        for (int u0 = 0; u0 < n; u0 += 4 * T) {
            uint2 v[4];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                int e = u0 + k * T + tid;
                v[k] = make_uint2(0, 0);
                if (e >= n) continue;
                if (e < ncol) {
                    int l = 1, w;
                    while (e >= (w = cget(a.levels, l).w)) {
                        e -= w;
                        l++;
                    }
                    v[k] = *reinterpret_cast<const uint2*>(a.res_cols + cget(a.levels, l).res_col_off + e);
                } else {
                    e -= ncol;
                    int l = 1, m;
                    int4 pl = plan[band * a.nlevels + 1];
                    while (e >= (m = max(0, pl.w - pl.z + 1))) {
                        e -= m;
                        l++;
                        pl = plan[band * a.nlevels + l];
                    }
                    v[k] = *reinterpret_cast<const uint2*>(a.res_rows + cget(a.levels, l).res_row_off + pl.z + e);
                }
            }
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int e = u0 + k * T + tid;
                if (e < ncol) reinterpret_cast<uint2*>(t_cols)[e] = v[k];
                else if (e < n) reinterpret_cast<uint2*>(t_rows)[e - ncol] = v[k];
            }
        }
    }
    int sc0 = 0, sstride = 0;   // the previous level's first computed ROI row and row pitch
    int tcol = 0, trow = 0;     // this level's offsets in the staged tables (kTab)
    for (int l = 0; l < a.nlevels; l++) {
        const int4 pl = plan[band * a.nlevels + l];
        const LevelGeom L = cget(a.levels, l);
        const int stride = L.stride, c0 = pl.z, nrows = pl.w - pl.z + 1;
        uint8_t* dst = lds + (l & 1) * buf_x;
        // 1. the ROI rows [c0, c0 + nrows) into dst at byte kEdge of each row
        if (l == 0) {
            // the frame's rows, 16-byte loads (w % 16 == 0: host), four in
            // flight per thread before the first store
            const int n16 = a.w >> 4, n = nrows * n16;
            for (int u0 = 0; u0 < n; u0 += 4 * T) {
                uint4 v[4];
                int o[4];
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const int u = min(u0 + k * T + tid, n - 1), r = u / n16, q = u - r * n16;
                    v[k] = *reinterpret_cast<const uint4*>(img + (size_t)(c0 + r) * a.w + 16 * q);
                    o[k] = r * stride + kEdge + 16 * q;
                }
#pragma unroll
                for (int k = 0; k < 4; k++) *reinterpret_cast<uint4*>(dst + o[k]) = v[k];
            }
        } else if (nrows > 0) {
            const uint8_t* src = lds + ((l - 1) & 1) * buf_x;
            // one thread per 4-pixel word and group of rows (G groups when the
            // row is at most T / G words wide; wider rows loop over words)
            const int nw = (L.w + 3) >> 2;
            const int G = max(1, T / nw), g = tid / nw;
            for (int q = tid - min(g, G - 1) * nw; g < G && q < nw; q += T) {
                const int r_lo = g * nrows / G, r_hi = (g + 1) * nrows / G;
                const int px0 = 4 * q;
                int ca[4], a0[4], a1[4];
                bool vb[4], vec = true;
#pragma unroll
                for (int b = 0; b < 4; b++) {
                    const bool on = px0 + b < L.w;
                    const ResizeCol c = kTab ? t_cols[tcol + (on ? px0 + b : 0)] : a.res_cols[L.res_col_off + (on ? px0 + b : 0)];
                    ca[b] = kEdge + c.sx0;
                    a0[b] = on ? c.a0 : 0;
                    a1[b] = on ? c.a1 : 0;
                    vb[b] = px0 + b < L.nvec_resize;
                    vec = vec && (!on || vb[b]);
                }
                auto hrow = [&](int sy, int (&S)[4]) {
                    const uint8_t* base = src + (sy - sc0) * sstride;
#pragma unroll
                    for (int b = 0; b < 4; b++) S[b] = base[ca[b]] * a0[b] + base[ca[b] + 1] * a1[b];
                };
                int H0[4], H1[4], cs0 = -1, cs1 = -1;
                for (int r = r_lo; r < r_hi; r++) {
                    const ResizeRow rw = kTab ? t_rows[trow + r] : a.res_rows[L.res_row_off + c0 + r];
                    const int sy0 = rw.sy0, sy1 = rw.sy1, b0 = rw.b0, b1 = rw.b1;
                    int A[4], B[4];
                    if (sy0 == cs1) {
#pragma unroll
                        for (int b = 0; b < 4; b++) A[b] = H1[b];
                    } else if (sy0 == cs0) {
#pragma unroll
                        for (int b = 0; b < 4; b++) A[b] = H0[b];
                    } else {
                        hrow(sy0, A);
                    }
                    if (sy1 == sy0) {
#pragma unroll
                        for (int b = 0; b < 4; b++) B[b] = A[b];
                    } else if (sy1 == cs1) {
#pragma unroll
                        for (int b = 0; b < 4; b++) B[b] = H1[b];
                    } else {
                        hrow(sy1, B);
                    }
#pragma unroll
                    for (int b = 0; b < 4; b++) {
                        H0[b] = A[b];
                        H1[b] = B[b];
                    }
                    cs0 = sy0;
                    cs1 = sy1;
                    uint32_t word = 0;
                    if (vec) {
                        // VResizeLinearVec_32s8u (its 16-bit saturations cannot trigger
                        // for 11-bit weights, k_pyr_resize_lds)
#pragma unroll
                        for (int b = 0; b < 4; b++) {
                            const int v = (((A[b] >> 4) * b0 >> 16) + ((B[b] >> 4) * b1 >> 16) + 2) >> 2;
                            word |= (uint32_t)min(v, 255) << (8 * b);
                        }
                    } else {
#pragma unroll
                        for (int b = 0; b < 4; b++) {
                            int v;
                            if (vb[b])
                                v = (((A[b] >> 4) * b0 >> 16) + ((B[b] >> 4) * b1 >> 16) + 2) >> 2;
                            else   // FixedPtCast<int, uchar, 22>
                                v = (A[b] * b0 + B[b] * b1 + (1 << 21)) >> 22;
                            word |= (uint32_t)sat_u8(v) << (8 * b);
                        }
                    }
                    // bytes past the ROI (the last word) are overwritten by the border pass
                    *reinterpret_cast<uint32_t*>(dst + r * stride + kEdge + px0) = word;
                }
            }
        }
        CASC_MARK(l, 0);
        __syncthreads();
        CASC_MARK(l, 1);
        // 2. border columns (REFLECT_101 of the row's own pixels) and the zero
        //    tail past the padded width, per computed row
        const int tail = stride - L.pw;
        for (int i = tid; i < nrows * (2 * kEdge + tail); i += T) {
            const int r = i / (2 * kEdge + tail), k = i - r * (2 * kEdge + tail);
            uint8_t* row = dst + r * stride;
            if (k < 2 * kEdge) {
                const int px = k < kEdge ? k : L.w + k;   // 0 .. 15, then kEdge + w .. kEdge + w + 15
                row[px] = row[kEdge + reflect101(px - kEdge, L.w)];
            } else {
                row[L.pw + (k - 2 * kEdge)] = 0;
            }
        }
        __syncthreads();
        CASC_MARK(l, 2);
        // 3. the band's rows to the pyramid, 16-byte stores: its owned ROI
        //    rows, then the border rows whose reflection it owns
        {
            const int n16 = stride >> 4, nown = pl.y - pl.x;
            uint8_t* out = pyr + L.off;
            for (int i = tid; i < nown * n16; i += T) {
                const int rr = i / n16, q = i - rr * n16, r = pl.x + rr;
                *reinterpret_cast<uint4*>(out + (size_t)(kEdge + r) * stride + 16 * q) =
                    *reinterpret_cast<const uint4*>(dst + (r - c0) * stride + 16 * q);
            }
            for (int i = tid; i < 2 * kEdge * n16; i += T) {
                const int k = i / n16, q = i - k * n16;
                const int py = k < kEdge ? k : L.h + k;   // 0 .. 15, then kEdge + h .. kEdge + h + 15
                const int r = reflect101(py - kEdge, L.h);
                if (r >= pl.x && r < pl.y)
                    *reinterpret_cast<uint4*>(out + (size_t)py * stride + 16 * q) =
                        *reinterpret_cast<const uint4*>(dst + (r - c0) * stride + 16 * q);
            }
        }
        CASC_MARK(l, 3);
        if (l > 0) {
            tcol += L.w;
            trow += max(0, nrows);
        }
        // the next level reads dst's ROI bytes (final since the first barrier)
        // and writes the other buffer, which nobody reads any more
        sc0 = c0;
        sstride = stride;
    }
}

// ---------------------------------------------------------------------------
// FAST-9/16 score map.  For a pixel with value v and ring d_k = v - p_k
// (k = 0..15, OpenCV offsets), S = max(M_dark, M_bright) - 1 where M_dark is
// the best 9-arc minimum of d and M_bright that of -d.  FAST at threshold t
// classifies the pixel as a corner iff S >= t, and cornerScore<16> returns
// exactly S (OpenCV 2.4 fast.cpp / fast_score.cpp).  A pixel whose compass
// pre-test passes in one direction only has S = that direction's arc - 1.
// ---------------------------------------------------------------------------
// Two candidates per lane (a, b) on packed fp16 halves: the 8-bit pixels
// become the exact fp16 integers 1024 + p (bits 0x6400 | p), so the ring
// differences d_k = v - p_k (|d| <= 255) are exact in fp16 and the 3-way
// windows are single v_pk_minimum3_f16 / v_pk_maximum3_f16 instructions
// (gfx950) for both candidates.  Returns max(dark, bright) (= S + 1) per
// candidate.
typedef _Float16 orbx_h2 __attribute__((ext_vector_type(2)));
typedef unsigned short orbx_u16x2 __attribute__((ext_vector_type(2)));
__device__ inline orbx_h2 h2_min3(orbx_h2 a, orbx_h2 b, orbx_h2 c)
{
    return __builtin_elementwise_minimum(__builtin_elementwise_minimum(a, b), c);
}
__device__ inline orbx_h2 h2_max3(orbx_h2 a, orbx_h2 b, orbx_h2 c)
{
    return __builtin_elementwise_maximum(__builtin_elementwise_maximum(a, b), c);
}
__device__ inline void fast_arc2(const uint8_t* t, int pa, int pb, int pitch, int& Sa, int& Sb)
{
    const int off[16] = {3 * pitch,      1 + 3 * pitch, 2 + 2 * pitch,  3 + pitch,
                         3,              3 - pitch,     2 - 2 * pitch,  1 - 3 * pitch,
                         -3 * pitch,     -1 - 3 * pitch, -2 - 2 * pitch, -3 - pitch,
                         -3,             -3 + pitch,    -2 + 2 * pitch, -1 + 3 * pitch};
    // bases at the ring's top-left corner: every offset is a non-negative
    // ds_read immediate (no address arithmetic per ring point)
    const int o = 3 * pitch + 3;
    int ba = pa - o, bb = pb - o;
    asm("" : "+v"(ba), "+v"(bb));   // opaque: keeps the constant offsets out of the bases
    const uint8_t* ta = t + ba;
    const uint8_t* tb = t + bb;
    // (a, b) byte pairs assembled as 16-bit halves (ds_read_u8_d16 /
    // _d16_hi), then the fp16 exponent bits
    auto pair = [&](int k) {
        orbx_u16x2 pv;
        pv.x = ta[k];
        pv.y = tb[k];
        return __builtin_bit_cast(uint32_t, pv) | 0x64006400u;
    };
    const orbx_h2 v = __builtin_bit_cast(orbx_h2, pair(o));
    orbx_h2 d[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const uint32_t w = pair(off[k] + o);
        d[k] = v - __builtin_bit_cast(orbx_h2, w);
    }
    orbx_h2 lo3[16], hi3[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {
        lo3[k] = h2_min3(d[k], d[(k + 1) & 15], d[(k + 2) & 15]);
        hi3[k] = h2_max3(d[k], d[(k + 1) & 15], d[(k + 2) & 15]);
    }
    orbx_h2 m9[16], x9[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {
        m9[k] = h2_min3(lo3[k], lo3[(k + 3) & 15], lo3[(k + 6) & 15]);
        x9[k] = h2_max3(hi3[k], hi3[(k + 3) & 15], hi3[(k + 6) & 15]);
    }
    // dark = max_k m9[k], bright = min_k x9[k] (3-way trees)
    orbx_h2 dk = h2_max3(m9[0], m9[1], m9[2]), br = h2_min3(x9[0], x9[1], x9[2]);
#pragma unroll
    for (int k = 3; k < 15; k += 2) {
        dk = h2_max3(dk, m9[k], m9[k + 1]);
        br = h2_min3(br, x9[k], x9[k + 1]);
    }
    dk = __builtin_elementwise_maximum(dk, m9[15]);
    br = __builtin_elementwise_minimum(br, x9[15]);
    const orbx_h2 r = __builtin_elementwise_maximum(dk, -br);
    Sa = (int)(float)r.x;
    Sb = (int)(float)r.y;
}

// One workgroup per (cell, frame).  LDS (dynamic): the cell ROI with
// 16-byte aligned rows (tile), its S' map (sm), and two bitmaps: `nz` (one
// bit per tile dword whose S' word is nonzero) and `kept` (one bit per tile
// byte that survives NMS), which reuses the tile's first bytes once the
// score pass is done (the threshold-7 rescore reloads the tile).
//  1. compass pre-test, 4 pixels per thread: a 9-arc covers two adjacent
//     compass points, so S >= tmin needs d > tmin (or < -tmin) on both;
//     survivors are compacted per wave and scored with all lanes busy; a
//     nonzero S' sets its dword's `nz` bit;
//  2. non-max suppression on the `nz` dwords only (listed with one block
//     scan), kept pixels set their `kept` bit;
//  3. raster-order compaction of the `kept` bitmap (tile byte order is
//     raster order), one block scan over ~2 bitmap words per thread.
// ---------------------------------------------------------------------------
__device__ inline int byte_of(uint32_t w, int k) { return (int)((w >> (8 * k)) & 0xFF); }

// Packed 16-bit lanes (v_pk_sub_i16 / v_pk_max_i16).
typedef short orbx_s16x2 __attribute__((ext_vector_type(2)));
__device__ inline uint32_t pk_sub16(uint32_t a, uint32_t b)
{
    return __builtin_bit_cast(uint32_t, (orbx_s16x2)(__builtin_bit_cast(orbx_s16x2, a) - __builtin_bit_cast(orbx_s16x2, b)));
}
__device__ inline uint32_t pk_max16(uint32_t a, uint32_t b)
{
    return __builtin_bit_cast(uint32_t,
                              __builtin_elementwise_max(__builtin_bit_cast(orbx_s16x2, a), __builtin_bit_cast(orbx_s16x2, b)));
}
// bytes (b0, b2) or (b1, b3) of w as the packed fp16 pair (1024 + b, 1024 + b')
// (exact integers): one v_perm with the 0x64 exponent bytes from k64
__device__ inline orbx_h2 h2_bytes(uint32_t w, uint32_t k64, uint32_t sel)
{
    return __builtin_bit_cast(orbx_h2, __builtin_amdgcn_perm(k64, w, sel));
}

constexpr int kFastWideThreads = 256;   // workgroup of the wide-tile FAST instances
// Dynamic LDS of a FAST workgroup for tiles of `bytes` (host and device).
__host__ __device__ constexpr int fast_tile_bytes(int hy_max, int pitch) { return (hy_max * pitch + 511) & ~511; }
__host__ __device__ constexpr int fast_lds_bytes(int tile_bytes) { return 2 * tile_bytes + tile_bytes / 32; }
// static LDS of a 256-thread FAST workgroup: 4 survivor queues of 384
// entries (u16, or u32 for the runtime-pitch instance) + block scratch
__host__ __device__ constexpr int fast_static_lds(bool u32_entries) { return 4 * 384 * (u32_entries ? 4 : 2) + 64; }
#ifndef ORBX_FAST_LDS_TARGET
#define ORBX_FAST_LDS_TARGET (40 * 1024)   // 4 workgroups per CU
#endif
constexpr int kFastLdsTarget = ORBX_FAST_LDS_TARGET;
// Diagnostic builds only (-DORBX_DIAG_REPEAT=r,b,d,f): launch resize, blur,
// describe or FAST that many times (idempotent kernels) to price each
// stage's marginal cost inside the pipelined bench.
#ifndef ORBX_DIAG_REPEAT
#define ORBX_DIAG_REPEAT 1, 1, 1, 1
#endif
constexpr int kDiagRepeat[4] = {ORBX_DIAG_REPEAT};

// kP > 0: compile-time tile pitch (>= every cell's aligned row), so ring
// offsets and row strides are immediates; kP == 0: per-cell pitch.
// kThreads: 256 for cells up to 208-byte rows; the wide tiles of large
// frames (1920x1080: 336-byte rows, 75 KB of LDS, two workgroups per CU)
// get more waves per workgroup instead.
__device__ __forceinline__ void blur_block(const ExtractArgs& a, const int4* tiles, int bx, int f);

// kBlurTail (orbx_extract's single-frame graph): the grid carries the blur's
// work blocks after the cells (blockIdx.x >= ncells), so FAST and the blur,
// which both read only the raw pyramid, are one launch.
template <int kP, int kThreads = 256, bool kBanded = false, bool kBlurTail = false>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(kThreads > 256 ? 6 : 4))) void k_fast_cells(
    ExtractArgs a, int tile_bytes, int band_rows)
{
    static_assert(!kBlurTail || kThreads == kBlurItems, "the blur tail runs 256-thread blur blocks");
    if constexpr (kBlurTail) {
        if ((int)blockIdx.x >= a.ncells) {
            blur_block(a, a.blur_tiles, (int)blockIdx.x - a.ncells, (int)blockIdx.y);
            return;
        }
    }
    constexpr int kBlock = kThreads, kWaves = kThreads / 64;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    __shared__ BlockScratchN<kWaves> bs;
    // Per-wave queue of compass survivors (tile positions): u16 for the
    // templated pitches (the host sends tiles over 64 KB to kP = 0), u32 for
    // kP = 0.  Linear, not a ring: after each scoring round the < 128 left
    // over move to the front, so an iteration's <= 256 new entries always fit.
    using QEntry = typename std::conditional<kP != 0, uint16_t, uint32_t>::type;
    constexpr int kQueue = 128 + 256;
    constexpr int kQueueWords = kWaves * kQueue * (int)sizeof(QEntry) / 4;
    constexpr int kUnitCap = 2 * kQueueWords;   // u16 NMS unit list aliasing the queues
    __shared__ __attribute__((aligned(16))) uint32_t qbuf[kQueueWords];
    __shared__ int s_left[kWaves];   // each wave's queue length at the end of a score pass
    uint16_t* ulist = reinterpret_cast<uint16_t*>(qbuf);
    const int f = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    QEntry* cand = reinterpret_cast<QEntry*>(qbuf) + wv * kQueue;
    // S' (0 where not scored) and nz start at zero (contiguous: tile_bytes *
    // (1 + 1/32), a multiple of 16); kept is cleared after the score pass
    const int clear16 = (tile_bytes + tile_bytes / 32) >> 4;
    auto clear_maps_at = [&](uint8_t* sm) {
        for (int i = tid; i < clear16; i += kBlock) reinterpret_cast<uint4*>(sm)[i] = make_uint4(0, 0, 0, 0);
    };
    // One cell.  tile / sm: its tile buffer and the S' map (nz follows sm).
    auto process = [&](const int cell, uint8_t* const tile, uint8_t* const sm) {
    const CellGeom C = cget(a.cells, cell);
    int32_t* count_out = a.cell_count + (size_t)f * a.ncells + cell;
    if (!C.valid) {
        if (tid == 0) *count_out = 0;
        return;
    }
    const LevelGeom L = cget(a.levels, C.level);
    const int roi_x = kEdge + C.ini_x, x_al = roi_x & ~15, sh = roi_x - x_al;
    const int hx = C.hx, hy = C.hy;
    const int nq16 = (sh + hx + 15) >> 4;               // 16-byte words loaded per row
    const int P = kP ? kP : 16 * nq16, nq = P >> 2;     // tile pitch, dwords per row
    const uint8_t* src = a.pyr_raw + (size_t)f * a.frame_pyr_bytes + L.off + (size_t)(kEdge + C.ini_y) * L.stride + x_al;
    uint32_t* tile32 = reinterpret_cast<uint32_t*>(tile);
    uint32_t* sm32 = reinterpret_cast<uint32_t*>(sm);
    uint32_t* kept = tile32;                                      // bit per tile byte (after scoring)
    uint32_t* nz = reinterpret_cast<uint32_t*>(sm + tile_bytes);  // bit per tile dword
    FP_T0();
    // the cell's rows [w0, w0 + wh) into tile rows 0 .. wh - 1
    auto load_tile = [&](int w0, int wh) {
        uint4* t16 = reinterpret_cast<uint4*>(tile32);
        const uint8_t* src_w = src + (size_t)w0 * L.stride;
        const int n = wh * nq16;
        // i / nq16 as a float product: (i + 1/2) / nq16 is at least 1/(2 nq16)
        // from an integer and the product's error is < 2^-21 (i + 1) for
        // i < 2^16, nq16 < 2^8 -- four integer divisions cost ~80 VALU
        const float inv16 = 1.0f / (float)nq16;
        auto row_of = [&](int i) { return (int)(((float)i + 0.5f) * inv16); };
        // four independent loads per round (named registers: an array here
        // was kept in scratch memory), then the LDS stores
        for (int u0 = 0; u0 < n; u0 += 4 * kBlock) {
            const int i0 = min(u0 + tid, n - 1), i1 = min(u0 + kBlock + tid, n - 1);
            const int i2 = min(u0 + 2 * kBlock + tid, n - 1), i3 = min(u0 + 3 * kBlock + tid, n - 1);
            const int r0 = row_of(i0), r1 = row_of(i1), r2 = row_of(i2), r3 = row_of(i3);
            const int c0 = i0 - r0 * nq16, c1 = i1 - r1 * nq16, c2 = i2 - r2 * nq16, c3 = i3 - r3 * nq16;
            // 32-bit offsets from the uniform tile origin (saddr loads)
            const uint4 v0 = *reinterpret_cast<const uint4*>(src_w + (uint32_t)(r0 * L.stride + 16 * c0));
            const uint4 v1 = *reinterpret_cast<const uint4*>(src_w + (uint32_t)(r1 * L.stride + 16 * c1));
            const uint4 v2 = *reinterpret_cast<const uint4*>(src_w + (uint32_t)(r2 * L.stride + 16 * c2));
            const uint4 v3 = *reinterpret_cast<const uint4*>(src_w + (uint32_t)(r3 * L.stride + 16 * c3));
            t16[r0 * (P >> 4) + c0] = v0;
            t16[r1 * (P >> 4) + c1] = v1;
            t16[r2 * (P >> 4) + c2] = v2;
            t16[r3 * (P >> 4) + c3] = v3;
        }
    };
    auto clear_maps = [&]() { clear_maps_at(sm); };
    auto clear_kept = [&]() {
        for (int i = tid; i < (tile_bytes >> 7); i += kBlock) reinterpret_cast<uint4*>(kept)[i] = make_uint4(0, 0, 0, 0);
    };
    const int c_lo = 3 + sh, c_hi = hx - 4 + sh;         // interior tile columns
    // dwords holding them; none when the ROI has no interior (hx < 7: a
    // degenerate cell of a tiny level, where c_hi < c_lo and, with a large
    // alignment shift, (c_hi >> 2) - q0 + 1 would go negative)
    const int q0 = c_lo >> 2, nqe = c_hi >= c_lo ? (c_hi >> 2) - q0 + 1 : 0;
    const int q_last = q0 + nqe - 1;
    const int j_lo = c_lo & 3, j_hi = c_hi & 3;           // pixels j >= j_lo of dword q0, j <= j_hi of q_last
    const uint32_t k64 = 0x64646464u;
    // S' map at threshold tmin over the window rows [sr0, sr0 + nrows):
    // S' = S where S >= tmin, else 0
    auto score_pass = [&](const int tmin, const int sr0, const int nrows) {
        const int nunits = max(nrows, 0) * nqe;
        // no interior dwords (a degenerate cell of a tiny level): nothing to
        // score, and RowWalk must not divide by nqe == 0
        if (nunits <= 0) return;
        // per-wave queue cand[0, qt) of compass survivors, scored 128 at a
        // time (two per lane) with every lane busy
        int qt = 0;
        auto set_nz = [&](int p) { atomicOr(&nz[p >> 7], 1u << ((p >> 2) & 31)); };
        auto score_pair = [&](int pa, int pb, bool has_a, bool has_b) {
            if (!has_a) return;
            int Sa, Sb;
            fast_arc2(tile, pa, pb, P, Sa, Sb);
            Sa -= 1;
            Sb -= 1;
            if (Sa >= tmin) {
                sm[pa] = (uint8_t)Sa;
                set_nz(pa);
            }
            if (has_b && Sb >= tmin) {
                sm[pb] = (uint8_t)Sb;
                set_nz(pb);
            }
        };
        // pass <=> max(v - A, B - v) >= tmin + 1 with A = min of the four
        // adjacent compass-pair maxima, B = max of the pair minima (exact
        // on the fp16 integers 1024 + p; the sign bit of the difference
        // is clear exactly when the test passes)
        const orbx_h2 T1 = {(_Float16)(tmin + 1), (_Float16)(tmin + 1)};
        RowWalk cw_(wv * 64 + lane, kBlock, nqe);
        for (int u0 = wv * 64; u0 < nunits; u0 += kBlock, cw_.next()) {
            const int u = u0 + lane;
            const int r = sr0 + cw_.r, q = q0 + cw_.q;
            // per pixel j: the sign bit of x_j = max(v - A, B - v) - tmin - 1
            // is set where the pixel fails (even half: j = 0, 2; odd: 1, 3)
            uint32_t xw0 = 0xBC00BC00u, xw1 = 0xBC00BC00u;   // -1.0: fails both tests (not -0)
            if (u < nunits) {
                const uint32_t* row = tile32 + r * nq + q;
                const uint32_t mid = row[0];
                // row[-1] / row[1] past the row ends are the neighbouring rows'
                // dwords (r is an interior row): only pixels outside the
                // interior columns read them, and those are masked below
                const uint32_t lo = row[-1], hi = row[1];
                const uint32_t up = row[-3 * nq], dn = row[3 * nq];
                // 4 pixels at once: even / odd bytes as two packed fp16 halves
                const uint32_t p4w = __builtin_amdgcn_alignbyte(hi, mid, 3);    // bytes j+3
                const uint32_t p12w = __builtin_amdgcn_alignbyte(mid, lo, 1);   // bytes j-3
                uint32_t xw[2];
#pragma unroll
                for (int hf = 0; hf < 2; hf++) {
                    const uint32_t sel = hf ? 0x04030401u : 0x04020400u;   // bytes 1,3 or 0,2 | 0x64
                    const orbx_h2 v = h2_bytes(mid, k64, sel);
                    // compass points in ring order 0, 4, 8, 12
                    const orbx_h2 p0 = h2_bytes(dn, k64, sel), p4 = h2_bytes(p4w, k64, sel);
                    const orbx_h2 p8 = h2_bytes(up, k64, sel), p12 = h2_bytes(p12w, k64, sel);
                    // IEEE maximum / minimum: no canonicalising moves (the
                    // operands are finite).  A = min over the adjacent pairs
                    // (0,4), (4,8), (8,12), (12,0) of the pair maximum; by
                    // distributivity min(max(a, x), max(b, x)) = max(x, min(a, b))
                    // that is max(min(p4, p12), min(p0, p8)); likewise
                    // B = max over the pairs of the pair minimum
                    // = min(max(p4, p12), max(p0, p8)).
                    const orbx_h2 A = __builtin_elementwise_maximum(__builtin_elementwise_minimum(p4, p12),
                                                                    __builtin_elementwise_minimum(p0, p8));
                    const orbx_h2 B = __builtin_elementwise_minimum(__builtin_elementwise_maximum(p4, p12),
                                                                    __builtin_elementwise_maximum(p0, p8));
                    const orbx_h2 x = __builtin_elementwise_maximum(v - A, B - v) - T1;
                    xw[hf] = __builtin_bit_cast(uint32_t, x);
                }
                xw0 = xw[0];
                xw1 = xw[1];
            }
            // pass flags as lane masks (bit 15 / 31 clear: a 16-bit and a
            // 32-bit signed compare each); the partial dwords q0 and q_last
            // drop the pixels outside the interior columns (uniform j tests;
            // bitwise on the lane masks, no short-circuit branches)
            const bool at_q0 = q == q0, at_ql = q == q_last;
            const bool cut0 = at_q0 & (j_lo > 0), cut1 = (at_q0 & (j_lo > 1)) | (at_ql & (j_hi < 1));
            const bool cut2 = (at_q0 & (j_lo > 2)) | (at_ql & (j_hi < 2)), cut3 = at_ql & (j_hi < 3);
            // (low halves as fp16 >= 0: no -0 or NaN arises from these exact
            // integer differences)
            const bool ok0 = (__builtin_bit_cast(orbx_h2, xw0).x >= (_Float16)0) & !cut0;
            const bool ok1 = (__builtin_bit_cast(orbx_h2, xw1).x >= (_Float16)0) & !cut1;
            const bool ok2 = ((int32_t)xw0 >= 0) & !cut2, ok3 = ((int32_t)xw1 >= 0) & !cut3;
            const uint64_t b0 = __builtin_amdgcn_ballot_w64(ok0), b1 = __builtin_amdgcn_ballot_w64(ok1);
            const uint64_t b2 = __builtin_amdgcn_ballot_w64(ok2), b3 = __builtin_amdgcn_ballot_w64(ok3);
            const int n0 = __popcll(b0), n1 = __popcll(b1), n2 = __popcll(b2);
            const int ntot = n0 + n1 + n2 + __popcll(b3);
#ifdef ORBX_FAST_PROFILE
            if (lane == 0) FP_ADD(10 + (tmin < 10), ntot);
            if (lane == 0) FP_ADD(12, 1);
#endif
            // plane-major order: each plane's survivors at their lane rank
            // (mbcnt, which adds the plane's start) after the earlier planes'
            const int pbase = r * P + 4 * q;
            auto slot = [&](uint64_t bm, int start) {
                return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32),
                                                      __builtin_amdgcn_mbcnt_lo((uint32_t)bm, (uint32_t)start));
            };
            if (ok0) cand[slot(b0, qt)] = (QEntry)pbase;
            if (ok1) cand[slot(b1, qt + n0)] = (QEntry)(pbase + 1);
            if (ok2) cand[slot(b2, qt + n0 + n1)] = (QEntry)(pbase + 2);
            if (ok3) cand[slot(b3, qt + n0 + n1 + n2)] = (QEntry)(pbase + 3);
            qt = __builtin_amdgcn_readfirstlane(qt + ntot);   // wave-uniform
            if (qt >= 128) {   // uniform: score full batches, move the rest to the front
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                int qh = 0;
                for (; qt - qh >= 128; qh += 128)
                    score_pair(cand[qh + lane], cand[qh + 64 + lane], true, true);
                const int rest = qt - qh;   // < 128
                const QEntry e0 = lane < rest ? cand[qh + lane] : (QEntry)0;
                const QEntry e1 = lane + 64 < rest ? cand[qh + 64 + lane] : (QEntry)0;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                if (lane < rest) cand[lane] = e0;
                if (lane + 64 < rest) cand[lane + 64] = e1;
                qt = __builtin_amdgcn_readfirstlane(rest);
            }
            // no fence here: the next iteration appends at >= qt (the moved
            // rest lies below it), and the queue is read only after the
            // fence above
        }
        // the waves' leftovers (< 128 each) scored together, in full batches
        // of 128 where they add up (one partly filled batch per wave would
        // run the whole scoring code for a few pixels)
        if (lane == 0) s_left[wv] = qt;
        __syncthreads();
        int pre[kWaves + 1];
        pre[0] = 0;
#pragma unroll
        for (int w = 0; w < kWaves; w++) pre[w + 1] = pre[w] + s_left[w];
        const int T = pre[kWaves];
        auto entry = [&](int g) {
            int w = 0;
#pragma unroll
            for (int k = 1; k < kWaves; k++) w += g >= pre[k];
            return (int)(reinterpret_cast<const QEntry*>(qbuf) + w * kQueue)[g - pre[w]];
        };
        for (int b0 = wv * 128; b0 < T; b0 += kWaves * 128) {
            const int ga = b0 + lane, gb = b0 + 64 + lane;
            score_pair(ga < T ? entry(ga) : 0, gb < T ? entry(gb) : 0, ga < T, gb < T);
        }
    };
    // non-max suppression over the S' map: a pixel is kept if its S' beats
    // all 8 neighbours' S'.  Only dwords whose `nz` bit is set can keep
    // anything; they are listed (u16 tile dword indices, in windows of
    // kUnitCap) with one block scan and shared by all 256 threads.
    // Only the window rows [rb0, rb1) (the band's own rows) keep anything;
    // the halo rows' S' serve as their neighbours.
    // Returns this thread's count of kept corners at fastTh.
    auto nms_pass = [&](const int rb0, const int rb1, const int wh) {
        int c1 = 0;
        const uint32_t FT = (uint32_t)max(a.fast_th, 1) * 0x00010001u;
        auto nms_unit = [&](int idx) {
            const int rw = idx / nq, q = idx - rw * nq;
            if (rw < rb0 || rw >= rb1) return;
            const uint32_t* m = sm32 + idx;
            const uint32_t mid = m[0];
            // the 8 neighbours of the 4 pixels as dwords (bytes j-1, j, j+1 of
            // rows r-1, r, r+1), byte-wise max on even / odd u16x2 halves
            uint32_t nb[8];
            int k = 0;
#pragma unroll
            for (int dr = 0; dr < 3; dr++) {
                const uint32_t* mr = m + (dr - 1) * nq;
                const uint32_t lo = q > 0 ? mr[-1] : 0u, mm = mr[0], hi = q + 1 < nq ? mr[1] : 0u;
                nb[k++] = __builtin_amdgcn_alignbyte(mm, lo, 3);   // j-1
                if (dr != 1) nb[k++] = mm;
                nb[k++] = __builtin_amdgcn_alignbyte(hi, mm, 1);   // j+1
            }
            uint32_t bits = 0;
#pragma unroll
            for (int hf = 0; hf < 2; hf++) {
                const uint32_t sel = hf ? 0x0c030c01u : 0x0c020c00u;
                uint32_t mx = __builtin_amdgcn_perm(0u, nb[0], sel);
#pragma unroll
                for (int i = 1; i < 8; i++) mx = pk_max16(mx, __builtin_amdgcn_perm(0u, nb[i], sel));
                const uint32_t sv = __builtin_amdgcn_perm(0u, mid, sel);
                // keep where mx - s < 0 (s > every neighbour)
                const uint32_t keep = pk_sub16(mx, sv) & 0x80008000u;
                // pixel j -> bit j (even half: j = 0, 2; odd half: j = 1, 3)
                bits |= ((keep >> 15) & 1) << hf | ((keep >> 31) & 1) << (2 + hf);
                // corners at fastTh among the kept (kept >= max(fastTh, 1))
                const uint32_t kept16 = sv & ((keep >> 15) * 0xFFFFu);
                c1 += __popc(~pk_sub16(kept16, FT) & keep);
            }
            if (bits) atomicOr(&kept[idx >> 3], bits << (4 * (idx & 7)));
        };
        const int nw = (wh * nq + 31) >> 5;                  // nz words
        const int pw = (nw + kBlock - 1) / kBlock;
        const int w0 = min(tid * pw, nw), w1 = min(w0 + pw, nw);
        int cnt = 0;
        for (int w = w0; w < w1; w++) cnt += __popc(nz[w]);
        int total;
        const int off0 = block_exclusive_scan(cnt, &total, bs, 1);
        for (int base = 0; base < total; base += kUnitCap) {
            if (base > 0) __syncthreads();                   // previous window consumed
            if (cnt && off0 < base + kUnitCap && off0 + cnt > base) {
                int off = off0;
                for (int w = w0; w < w1; w++) {
                    uint32_t b = nz[w];
                    while (b) {
                        const int bit = __builtin_ctz(b);
                        b &= b - 1;
                        if (off >= base && off < base + kUnitCap) ulist[off - base] = (uint16_t)(32 * w + bit);
                        off++;
                    }
                }
            }
            __syncthreads();
            const int n = min(total - base, kUnitCap);
            for (int i = tid; i < n; i += kBlock) nms_unit((int)ulist[i]);
        }
        return c1;
    };
    uint32_t* out = a.cell_lists + (size_t)f * a.list_entries + C.list_off;
    // Raster-order compaction of the kept bitmap into the cell's list at
    // out_base: thread tid owns the contiguous bitmap words [ka, kb); kept
    // bytes are S' >= tmin of the pass, and t == tmin unless fastTh < 7 fell
    // back to 7 (then each byte is compared).  Returns the entries written.
    auto compact = [&](const int t, const int tmin, const int w0, const int wh, const int out_base) {
        const int nkw = (wh * P + 31) >> 5;
        const int per = (nkw + kBlock - 1) / kBlock;
        const int ka = min(tid * per, nkw), kb = min(ka + per, nkw);
        const bool all_kept = t == tmin;
        int cnt = 0;
        for (int k = ka; k < kb; k++) {
            uint32_t b = kept[k];
            if (all_kept) {
                cnt += __popc(b);
            } else {
                while (b) {
                    const int bit = __builtin_ctz(b);
                    b &= b - 1;
                    cnt += sm[32 * k + bit] >= t;
                }
            }
        }
        int total;
        int off = out_base + block_exclusive_scan(cnt, &total, bs, 1);
        if (cnt) {
            // entries go straight to the cell's list (each thread's run is
            // contiguous; the tile area holds the kept bitmap being read)
            for (int k = ka; k < kb; k++) {
                uint32_t b = kept[k];
                while (b) {
                    const int bit = __builtin_ctz(b);
                    b &= b - 1;
                    const int pos = 32 * k + bit;
                    const int s = sm[pos];
                    if (s >= t) {
                        if (off < C.list_cap) {
                            const int r = w0 + pos / P, cc = pos % P - sh;   // cell row, ROI column
                            out[off] = ((uint32_t)s << 24) | ((uint32_t)(C.ini_y + r) << 12) | (uint32_t)(C.ini_x + cc);
                        }
                        off++;
                    }
                }
            }
        }
        return total;
    };
    // One band: the cell rows [b0, b1) (interior rows 3 .. hy - 4).  Its
    // window holds the rows [b0 - 4, b1 + 4) (clipped to the cell): FAST's
    // 3-pixel radius around the rows b0 - 1 .. b1 whose S' the band's NMS
    // reads.  Scores, suppresses and (emit) appends the band's kept corners
    // at out_base; returns the band's kept corners at fastTh.  A whole cell
    // is one band unless the host splits tall cells (band_rows) so that a
    // workgroup's LDS stays small (1920x1080: 4 workgroups per CU instead of
    // 2); S' of a row depends only on the rows within 3 of it, so the split
    // is exact.
    auto band = [&](const int b0, const int b1, const int tmin, const bool loaded = false) {
        const int w0 = max(0, b0 - 4), wh = min(hy, b1 + 4) - w0;
        const int s0 = max(3, b0 - 1), s1 = min(hy - 4, b1);   // scored rows (inclusive)
        if (!loaded) {
            FP_MARK(7);
            load_tile(w0, wh);
            FP_MARK(5);
            clear_maps();
            FP_MARK(6);
            __syncthreads();
        }
        FP_MARK(0);
        score_pass(tmin, s0 - w0, s1 - s0 + 1);
        __syncthreads();
        FP_MARK(1);
        clear_kept();   // the tile is dead until the next band reloads it
        __syncthreads();
        const int n1 = block_sum(nms_pass(b0 - w0, b1 - w0, wh), bs, 0);
        __syncthreads();
        return n1;
    };
    // Thresholds (:599-614): FAST(fastTh), and FAST(7) when that finds <= 3
    // corners.  The S' map at threshold t gives both answers for t <= min
    // (NMS against S' equals NMS against the t-score map for corners >= t),
    // so a cell is scored at fastTh first (far fewer compass survivors) and
    // rescored at 7 only when it needs the fallback.
    int n1 = 0, written = 0;
    if constexpr (kBanded) {
        // each band is emitted at fastTh as it is done; a cell whose kept
        // corners at fastTh number <= 3 is scored again band by band (at 7,
        // or at fastTh < 7 and filtered to >= 7) and re-emitted
        const int brows = band_rows > 0 ? band_rows : hy;
        for (int b0 = 3; b0 < hy - 3; b0 += brows) {
            const int b1 = min(b0 + brows, hy - 3);
            n1 += band(b0, b1, a.fast_th);
            written += compact(a.fast_th, a.fast_th, max(0, b0 - 4), min(hy, b1 + 4) - max(0, b0 - 4), written);
            __syncthreads();   // kept / S' reused by the next band
        }
        if (n1 <= 3) {   // uniform over the block
            const int tmin2 = a.fast_th > a.fast_th_low ? a.fast_th_low : a.fast_th;
            written = 0;
            for (int b0 = 3; b0 < hy - 3; b0 += brows) {
                const int b1 = min(b0 + brows, hy - 3);
                band(b0, b1, tmin2);
                written += compact(a.fast_th_low, tmin2, max(0, b0 - 4), min(hy, b1 + 4) - max(0, b0 - 4), written);
                __syncthreads();
            }
        }
    } else if (hy > 6) {   // the whole cell as one band (the host sends band_rows = 0)
        int tmin_final = a.fast_th;
        n1 = band(3, hy - 3, a.fast_th);
        FP_MARK(2);
        if (a.fast_th > a.fast_th_low && n1 <= 3) {   // uniform over the block
            if (threadIdx.x == 0) FP_ADD(8, 1);
            tmin_final = a.fast_th_low;
            band(3, hy - 3, a.fast_th_low);
            FP_MARK(3);
        }
        // threshold choice: FAST(fastTh); if <= 3 corners, FAST(7) (:607-614)
        written = compact(n1 <= 3 ? a.fast_th_low : a.fast_th, tmin_final, 0, hy, 0);
    }
    if (tid == 0) {
        *count_out = written;
        if (written > C.list_cap) atomicOr(a.error_flags, 1);
    }
    FP_MARK(4);
    if (tid == 0) FP_ADD(9, 1);
    };
    process(blockIdx.x, smem, smem + tile_bytes);
}

// ---------------------------------------------------------------------------
// retainBest, in two launches (src/ORBextractor.cc:622-701):
//  k_retain_cells   one wave per (cell, frame): the level's quota
//                   redistribution (:622-670, wave-parallel over cells),
//                   nth_element of the cell list in a wave-private LDS
//                   buffer (:683-685), and the retained prefix written to
//                   the cell's slot of the level list (cell order, :687-694);
//  k_retain_levels  one wave per (level, frame): nth_element of the level
//                   list when it exceeds the level quota (:697-701).
// ---------------------------------------------------------------------------
__device__ inline void level_quota(const ExtractArgs& a, const LevelGeom& L, const int32_t* counts, int cell,
                                   int* keep_c, int* pre_c, int* level_total)
{
    const int lane = threadIdx.x & 63;
    const int nCells = L.n_cells, nfc = L.nfeatures_cell;
    constexpr int kPer = 4;   // cells per lane (<= 256 cells per level)
    int tot[kPer], ret[kPer];
    bool nomore[kPer];
    int toDist = 0, nNoMore = 0;
    // slots past the level's cells are skipped (a uniform branch): C2's
    // levels have <= 30 cells, so one slot of 64 does all the work
#pragma unroll
    for (int k = 0; k < kPer; k++) {
        const int c = lane + 64 * k;
        tot[k] = 0;
        ret[k] = 0;
        nomore[k] = false;
        if (64 * k < nCells && c < nCells) {
            tot[k] = counts[c];
            if (a.cells[L.cell_base + c].valid) {
                if (tot[k] > nfc) {
                    ret[k] = nfc;
                } else {
                    ret[k] = tot[k];
                    toDist += nfc - tot[k];
                    nomore[k] = true;
                    nNoMore++;
                }
            }
        }
    }
    toDist = wave_sum(toDist);
    nNoMore = wave_sum(nNoMore);
    while (toDist > 0 && nNoMore < nCells) {
        const int nNew = nfc + (int)ceilf(__fdiv_rn((float)toDist, (float)(nCells - nNoMore)));
        int td = 0, nm = 0;
#pragma unroll
        for (int k = 0; k < kPer; k++) {
            if (64 * k >= nCells) break;
            const int c = lane + 64 * k;
            if (c < nCells && !nomore[k]) {
                if (tot[k] > nNew) {
                    ret[k] = nNew;
                } else {
                    ret[k] = tot[k];
                    td += nNew - tot[k];
                    nomore[k] = true;
                    nm++;
                }
            }
        }
        toDist = wave_sum(td);
        nNoMore += wave_sum(nm);
    }
    int base = 0, my_keep = 0, my_pre = 0;
#pragma unroll
    for (int k = 0; k < kPer; k++) {
        if (64 * k >= nCells) break;
        const int c = lane + 64 * k;
        const int take = (c < nCells && tot[k] > 0 && ret[k] > 0) ? min(tot[k], ret[k]) : 0;
        const int incl = wave_inclusive_scan(take);
        const int kk = __builtin_amdgcn_readlane(ret[k], cell & 63), pp = __builtin_amdgcn_readlane(base + incl - take, cell & 63);
        if ((cell >> 6) == k) {
            my_keep = kk;
            my_pre = pp;
        }
        base += __builtin_amdgcn_readlane(incl, 63);
    }
    *keep_c = my_keep;
    *pre_c = my_pre;
    *level_total = base;
}

// ---------------------------------------------------------------------------
// HarrisResponses(cellImage, cellKeyPoints, 7, HARRIS_K) (:79-120, :616-620)
// on each cell's FAST list, one thread per corner: the 7x7 block of 3x3
// Sobel products around the corner (9x9 pixels of the unblurred level,
// three rows live in registers), integer sums, then the float response in
// the source's evaluation order with every operation rounded on its own
// (no contraction).  The entry becomes harris_key(response) << 32 | y << 12
// | x, so the retain kernels compare responses exactly as retainBest does.
// ---------------------------------------------------------------------------
constexpr float kHarrisK = 0.04f;                                  // HARRIS_K (:73)
constexpr float kHarrisScale = 1.0f / ((1 << 2) * 7 * 255.0f);     // 1 / ((1<<2) blockSize 255)  (:90-91)
constexpr float kHarrisScale4 = kHarrisScale * kHarrisScale * kHarrisScale * kHarrisScale;   // (:92)

__global__ __launch_bounds__(256) void k_harris_cells(ExtractArgs a)
{
    const int cell = blockIdx.x, f = blockIdx.y;
    const CellGeom C = cget(a.cells, cell);
    if (!C.valid) return;
    const int n = min(a.cell_count[(size_t)f * a.ncells + cell], C.list_cap);
    const LevelGeom L = cget(a.levels, C.level);
    const int stride = L.stride;
    const uint8_t* img = a.pyr_raw + (size_t)f * a.frame_pyr_bytes + L.off + (size_t)kEdge * stride + kEdge;
    const uint32_t* src = a.cell_lists + (size_t)f * a.list_entries + C.list_off;
    uint64_t* dst = a.cell_keys64 + (size_t)f * a.list_entries + C.list_off;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const uint32_t e = src[i];
        const int y = (int)((e >> 12) & 0xFFF), x = (int)(e & 0xFFF);
        const uint8_t* p0 = img + (ptrdiff_t)(y - 4) * stride + (x - 4);
        int r0[9], r1[9], r2[9];
#pragma unroll
        for (int j = 0; j < 9; j++) {
            r0[j] = p0[j];
            r1[j] = p0[stride + j];
        }
        int sa = 0, sb = 0, sc = 0;
#pragma unroll
        for (int rr = 2; rr < 9; rr++) {
#pragma unroll
            for (int j = 0; j < 9; j++) r2[j] = p0[(ptrdiff_t)rr * stride + j];
#pragma unroll
            for (int j = 1; j < 8; j++) {
                const int Ix = (r1[j + 1] - r1[j - 1]) * 2 + (r0[j + 1] - r0[j - 1]) + (r2[j + 1] - r2[j - 1]);
                const int Iy = (r2[j] - r0[j]) * 2 + (r2[j - 1] - r0[j - 1]) + (r2[j + 1] - r0[j + 1]);
                sa += Ix * Ix;
                sb += Iy * Iy;
                sc += Ix * Iy;
            }
#pragma unroll
            for (int j = 0; j < 9; j++) {
                r0[j] = r1[j];
                r1[j] = r2[j];
            }
        }
        const float fa = (float)sa, fb = (float)sb, fc = (float)sc;
        const float s2 = __fadd_rn(fa, fb);
        // (a*b - c*c) - (k*(a+b))*(a+b), each operation rounded (ISO), or as
        // GCC contracts it on an FMA host: fma(a, b, -(c*c)), then
        // fma(-(k*(a+b)), a+b, that) (oracle/ref_orbsites.cpp)
        const float t = a.fp_contract
                            ? __fmaf_rn(-__fmul_rn(kHarrisK, s2), s2, __fmaf_rn(fa, fb, -__fmul_rn(fc, fc)))
                            : __fsub_rn(__fsub_rn(__fmul_rn(fa, fb), __fmul_rn(fc, fc)),
                                        __fmul_rn(__fmul_rn(kHarrisK, s2), s2));
        const float resp = __fmul_rn(t, kHarrisScale4);
        dst[i] = (uint64_t)harris_key(resp) << 32 | (e & 0xFFFFFFu);
    }
}

// E = uint32_t (FAST score entries) or uint64_t (Harris-keyed entries)
template <typename E>
__device__ inline E* cell_entries(const ExtractArgs& a)
{
    if constexpr (sizeof(E) == 8) return a.cell_keys64;
    else return a.cell_lists;
}
template <typename E>
__device__ inline E* level_entries(const ExtractArgs& a)
{
    if constexpr (sizeof(E) == 8) return a.level_keys64;
    else return a.level_keys;
}

template <typename E>
__global__ __launch_bounds__(256) void k_retain_cells(ExtractArgs a, int waves_per_block, int wave_words)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t sbuf[];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int cell = blockIdx.x * waves_per_block + wv, f = blockIdx.y;
    if (cell >= a.ncells) return;
    E* list = reinterpret_cast<E*>(sbuf + (size_t)wv * wave_words);
    int* pos = reinterpret_cast<int*>(list + kRetainCellCap);
    const CellGeom C = cget(a.cells, cell);
    const LevelGeom L = cget(a.levels, C.level);
    const int c = cell - L.cell_base;
    const int32_t* counts = a.cell_count + (size_t)f * a.ncells + L.cell_base;
    int k, pre, level_total;
    level_quota(a, L, counts, c, &k, &pre, &level_total);
    if (c == 0 && lane == 0) a.level_count[(size_t)f * a.nlevels + C.level] = min(level_total, L.level_cap);
    if (level_total > L.level_cap) {
        if (lane == 0) atomicOr(a.error_flags, 2);
        return;
    }
    const int n = counts[c];
    if (n == 0 || k == 0) return;
    const int take = min(n, k);
    E* src = cell_entries<E>(a) + (size_t)f * a.list_entries + C.list_off;
    E* dst = level_entries<E>(a) + (size_t)f * a.level_entries + L.level_off + pre;
    if (n > k && n <= kRetainCellCap) {
        stage_to_lds<8>(list, n, lane, 64, [&](int i) { return src[i]; });
        lds_wave_sync();
        wave_nth_element(list, n, k, pos, a.nth_pivot);
        for (int i = lane; i < take; i += 64) dst[i] = list[i];
    } else if (n > k) {
        // long list: replay in place in global memory
        int* gpos = a.retain_scratch + (size_t)f * (a.list_entries + 4 * a.ncells) + C.list_off + 4 * cell;
        wave_nth_element<true>(src, n, k, gpos, a.nth_pivot);
        for (int i = lane; i < take; i += 64) dst[i] = src[i];
    } else {
        for (int i = lane; i < take; i += 64) dst[i] = src[i];
    }
}

template <typename E>
__global__ __launch_bounds__(256) void k_retain_levels(ExtractArgs a, int waves_per_block, int wave_words)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t sbuf[];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int level = blockIdx.x * waves_per_block + wv, f = blockIdx.y;
    if (level >= a.nlevels) return;
    const LevelGeom L = cget(a.levels, level);
    int32_t* cnt = a.level_count + (size_t)f * a.nlevels + level;
    const int nlev = *cnt;
    if (nlev <= L.n_desired) return;
    E* list = reinterpret_cast<E*>(sbuf + (size_t)wv * wave_words);
    int* pos = reinterpret_cast<int*>(list + a.max_level_cap);
    E* g = level_entries<E>(a) + (size_t)f * a.level_entries + L.level_off;
    stage_to_lds<8>(list, nlev, lane, 64, [&](int i) { return g[i]; });
    lds_wave_sync();
    wave_nth_element(list, nlev, L.n_desired, pos, a.nth_pivot);
    for (int i = lane; i < L.n_desired; i += 64) g[i] = list[i];
    if (lane == 0) *cnt = L.n_desired;
}

// ---------------------------------------------------------------------------
// GaussianBlur 7x7, sigma 2, BORDER_REFLECT_101 on the level ROI with the
// parent border as context (OpenCV 2.4 8U fixed-point separable filter:
// taps {18,34,49,55,49,34,18}/256 per pass).  Column pass rounding: columns
// < nvec follow SymmColumnVec_32s8u (float, round-half-even), the tail
// FixedPtCastEx (+2^15 >> 16).  The padded border is copied unblurred.
// Each thread owns one dword column (4 pixels) of a kBlurStrip-row strip and
// slides a 7-row window of horizontal sums down it in registers: one pass
// over the input rows it needs, one dword store per output row, no LDS.
// ---------------------------------------------------------------------------
__device__ inline void blur_hsum(const uint8_t* row, int x, int hs[4])
{
    const uint32_t* w = reinterpret_cast<const uint32_t*>(row + x);
    blur_hsum_w(w[-1], w[0], w[1], hs);
}

// One blur work block (bx) of frame f.
__device__ __forceinline__ void blur_block(const ExtractArgs& a, const int4* tiles, const int bx, const int f)
{
    // One wave per (row strip, chunk of kBlurChunkCols dword columns): lane
    // l holds dword 62 c - 1 + l of each row, lanes 0 and 63 only as halo.
    // A row is one dword load per lane; the left / right neighbour dwords of
    // the horizontal taps come from the adjacent lanes (DPP wave_shr:1 /
    // wave_shl:1) instead of two more loads.
    const int4 tl = cget(tiles, bx);   // level, first wave item, chunks per row, strips
    const int wi = tl.y + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (wi >= tl.z * tl.w) return;       // whole waves
    const LevelGeom L = cget(a.levels, tl.x);
    const int strip = wi / tl.z, chunk = wi - strip * tl.z;
    const int ndw = L.stride >> 2;
    const int dw = kBlurChunkCols * chunk - 1 + lane;
    const bool out = lane >= 1 && lane <= kBlurChunkCols && dw < ndw;
    const int x = 4 * min(max(dw, 0), ndw - 1);
    const int y0 = strip * kBlurStrip, y1 = min(y0 + kBlurStrip, L.ph);
    // uniform level bases + 32-bit per-lane offsets (saddr + voffset loads)
    const uint8_t* src = a.pyr_raw + (size_t)f * a.frame_pyr_bytes + L.off;
    uint8_t* dst = a.pyr_blur + (size_t)f * a.frame_pyr_bytes + L.off;
    const uint32_t stride = (uint32_t)L.stride;
    auto ld = [&](int y) { return *reinterpret_cast<const uint32_t*>(src + ((uint32_t)y * stride + (uint32_t)x)); };
    auto st = [&](int y, uint32_t v) {
        if (out) *reinterpret_cast<uint32_t*>(dst + ((uint32_t)y * stride + (uint32_t)x)) = v;
    };
    // neighbours' words (lane - 1 / lane + 1): the DPP reads need every lane
    // of the wave active, so all lanes run the same rows
    auto left = [&](uint32_t v) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xf, 0xf, false); };
    auto right = [&](uint32_t v) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xf, 0xf, false); };
    // interior rows of this level in padded coordinates: rows [ya, yb) of the
    // strip are blurred (border columns keep their raw bytes), the rest copied
    const int iy0 = kEdge, iy1 = kEdge + L.h;
    const int ya = min(max(y0, iy0), y1), yb = max(min(y1, iy1), ya);
    // bytes beyond the padded width (row pitch padding) are zero
    uint32_t keep_mask = 0;
#pragma unroll
    for (int j = 0; j < 4; j++)
        if (x + j < L.pw) keep_mask |= 0xFFu << (8 * j);
    // copied (border) rows, 4 loads in flight per round
    auto copy_rows = [&](int ylo, int yhi) {
        for (int yc = ylo; yc < yhi; yc += 4) {
            uint32_t v[4];
#pragma unroll
            for (int k = 0; k < 4; k++) v[k] = ld(min(yc + k, yhi - 1));
#pragma unroll
            for (int k = 0; k < 4; k++)
                if (yc + k < yhi) st(yc + k, v[k] & keep_mask);
        }
    };
    copy_rows(y0, ya);
    if (ya < yb) {
        // per column: float path (round half to even) below nvec, else +2^15
        int half_even[4];
        bool inside[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int xi = x + j - kEdge;
            inside[j] = xi >= 0 && xi < L.w;
            half_even[j] = xi < L.nvec_blur;
        }
        // Vertical pass in packed FP32 (two pixels per v_pk_fma_f32): the row
        // sums are integers <= 255 * 257 and N <= 255 * 257^2; every partial
        // sum below 2^24 is exact, and an N beyond 2^24 saturates to 255 either
        // way.  Rounding and saturation by v_cvt_pk_u8_f32 (round half to even
        // = cvtps2dq of SymmColumnVec_32s8u); the scalar tail columns
        // (FixedPtCastEx, +2^15 >> 16) pass floor((N + 2^15) / 2^16).
        typedef float f2 __attribute__((ext_vector_type(2)));
        constexpr float kInv = 1.0f / 65536.0f;
        bool tail_col[4], any_tail = false;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            tail_col[j] = inside[j] && !half_even[j];
            any_tail = any_tail || tail_col[j];
        }
        f2 R[7][2];
        auto hrow = [&](uint32_t c, f2 (&o)[2]) {
            int hs[4];
            blur_hsum_w(left(c), c, right(c), hs);
            o[0] = f2{(float)hs[0], (float)hs[1]};
            o[1] = f2{(float)hs[2], (float)hs[3]};
        };
        uint32_t C[3];   // raw centre words of rows y, y+1, y+2 (loaded as rows y'+3 earlier)
        {
            uint32_t w0[6];
#pragma unroll
            for (int k = 0; k < 6; k++) w0[k] = ld(ya - 3 + k);
#pragma unroll
            for (int k = 0; k < 6; k++) {
                hrow(w0[k], R[k]);
                if (k >= 3) C[k - 3] = w0[k];
            }
        }
        // chunks of 7 output rows (the window's period: the register
        // rotation needs no moves); the chunk's input rows y + 3 are loaded
        // together, then filtered from registers
        constexpr int kBlurChunk = 7;
        for (int yc = ya; yc < yb; yc += kBlurChunk) {
            uint32_t wc[kBlurChunk];
#pragma unroll
            for (int k = 0; k < kBlurChunk; k++) wc[k] = ld(min(yc + k, yb - 1) + 3);   // rows past yb + 2 repeat
#pragma unroll
            for (int k = 0; k < kBlurChunk; k++) {
                // rows past yb are computed on repeated input and not stored:
                // no early exit, so the window rotation stays straight-line
                const int y = yc + k;
                hrow(wc[k], R[6]);
                float sv[4];
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    f2 N = R[3][h] * 55.0f;
                    N = __builtin_elementwise_fma(R[2][h] + R[4][h], f2{49.0f, 49.0f}, N);
                    N = __builtin_elementwise_fma(R[1][h] + R[5][h], f2{34.0f, 34.0f}, N);
                    N = __builtin_elementwise_fma(R[0][h] + R[6][h], f2{18.0f, 18.0f}, N);
                    const f2 sc = N * kInv;
                    sv[2 * h] = sc.x;
                    sv[2 * h + 1] = sc.y;
                    if (any_tail) {
                        const f2 tl2 = (N + 32768.0f) * kInv;
                        if (tail_col[2 * h]) sv[2 * h] = floorf(tl2.x);
                        if (tail_col[2 * h + 1]) sv[2 * h + 1] = floorf(tl2.y);
                    }
                }
                uint32_t word = C[0];   // border columns keep the raw byte
#pragma unroll
                for (int j = 0; j < 4; j++)
                    if (inside[j]) word = __builtin_amdgcn_cvt_pk_u8_f32(sv[j], j, word);
                if (y < yb) st(y, word & keep_mask);
#pragma unroll
                for (int kk = 0; kk < 6; kk++)
#pragma unroll
                    for (int h = 0; h < 2; h++) R[kk][h] = R[kk + 1][h];
                C[0] = C[1];
                C[1] = C[2];
                C[2] = wc[k];
            }
        }
    }
    copy_rows(yb, y1);
}

__global__ __launch_bounds__(256) void k_blur(ExtractArgs a, const int4* tiles)
{
    blur_block(a, tiles, (int)blockIdx.x, (int)blockIdx.y);
}

// ---------------------------------------------------------------------------
// IC_Angle + computeOrbDescriptor + output assembly, one wave per keypoint.
// The wave first stages, with independent dword loads, the 31x31 unblurred
// patch (IC_Angle reads radius 15) and the 37x37 blurred patch (rotated
// pattern points reach cvRound(13*sqrt(2)) = 18) in LDS, so the gathers
// cost one memory round trip instead of a dependent chain.
// ---------------------------------------------------------------------------
constexpr int kIcRows = 2 * kHalfPatch + 1;          // 31
constexpr int kIcPitch = 36;                         // 9 dwords: 31 bytes + alignment
constexpr int kBrR = 18;                             // pattern reach
constexpr int kBrRows = 2 * kBrR + 1;                // 37
constexpr int kBrPitch = 40;                         // 10 dwords: 37 bytes + alignment
constexpr int kDescWaveBytes = kIcRows * kIcPitch + kBrRows * kBrPitch;

// Half-wave (32-lane) sums: DPP row shifts inside each 16-lane row, then
// row_bcast:15 folds row 0 into row 1 and row 2 into row 3; lane 31 holds the
// lower half's sum, lane 63 the upper half's.
__device__ inline int half_wave_sum(int v)
{
    v += dpp_or0<0x111, 0xf>(v);
    v += dpp_or0<0x112, 0xf>(v);
    v += dpp_or0<0x114, 0xf>(v);
    v += dpp_or0<0x118, 0xf>(v);
    v += dpp_or0<0x142, 0xa>(v);
    const int lo = __builtin_amdgcn_readlane(v, 31), hi = __builtin_amdgcn_readlane(v, 63);
    return (threadIdx.x & 32) ? hi : lo;
}

// Two keypoints per wave, one per 32-lane half: every per-keypoint scalar
// step (fastAtan2, the correctly rounded sin/cos) is shared by two
// keypoints per instruction, and the pattern's 256 tests map onto 8 rounds
// of 32 lanes (ballot halves = 32 descriptor bits each).
// GET_VALUE's sample coordinates (src/ORBextractor.cc:165-167): row
// x*b + y*a and column x*a - y*b.  kFma: as GCC contracts them on an FMA host
// (-O3 -march=native, CMakeLists.txt:12-13): fma(x, b, y*a), fma(x, a, -(y*b)).
template <bool kFma>
__device__ inline int orb_sample_offset(float px, float py, float sa, float ca)
{
    const float fy = kFma ? __fmaf_rn(px, sa, __fmul_rn(py, ca)) : __fadd_rn(__fmul_rn(px, sa), __fmul_rn(py, ca));
    const float fx = kFma ? __fmaf_rn(px, ca, -__fmul_rn(py, sa)) : __fsub_rn(__fmul_rn(px, ca), __fmul_rn(py, sa));
    return cv_round(fy) * kBrPitch + cv_round(fx);
}

// Both points of a pattern pair at once on packed fp32 (v_pk_mul_f32 /
// v_pk_add_f32 / v_pk_fma_f32: each lane rounds exactly as the scalar
// operation).  cvRound (round half to even, OpenCV 2.4's cvtsd2si) is the
// 1.5 * 2^23 magic-number round trip: |coordinate| <= 18, so fy + M rounds fy
// to its nearest-even integer and subtracting M again is exact.  The patch
// offset row * kBrPitch + col (+ base, folded into the column's round trip)
// is then an exact float fma on integers below 2^24.  Returns the two LDS
// byte addresses.
typedef float orbx_f2 __attribute__((ext_vector_type(2)));
template <bool kFma>
__device__ inline void orb_sample_addr2(orbx_f2 px, orbx_f2 py, float sa, float ca, float base, uint32_t& a1,
                                        uint32_t& a2)
{
    const orbx_f2 SA = {sa, sa}, CA = {ca, ca};
    orbx_f2 fy, fx;
    if constexpr (kFma) {
        fy = __builtin_elementwise_fma(px, SA, py * CA);
        fx = __builtin_elementwise_fma(px, CA, -(py * SA));
    } else {
        fy = px * SA + py * CA;
        fx = px * CA - py * SA;
    }
    const orbx_f2 M = {12582912.0f, 12582912.0f}, MB = {12582912.0f - base, 12582912.0f - base};
    const orbx_f2 P = {(float)kBrPitch, (float)kBrPitch};
    const orbx_f2 ry = (fy + M) - M, rxb = (fx + M) - MB;
    const orbx_f2 ad = __builtin_elementwise_fma(ry, P, rxb);
    a1 = (uint32_t)ad.x;
    a2 = (uint32_t)ad.y;
}

template <bool kFma>
__global__ __launch_bounds__(256) void k_describe(ExtractArgs a, int nframes)
{
    __shared__ __attribute__((aligned(16))) uint8_t s_patch[2 * kWaves][kDescWaveBytes];
    // XCD-aware order (xcd_block): a frame's keypoint patches, which overlap,
    // are fetched into one XCD's L2
    const XcdBlock xb = xcd_block();
    const int f = xb.frame, chunk = xb.chunk;
    if (f >= nframes) return;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, half = lane >> 5, hl = lane & 31;
    const int slot = wv * 2 + half;
    const int k = chunk * (2 * kWaves) + slot;
    // tables needed later, loaded up front (independent of the keypoint):
    // umax[0..15] one entry per lane, this lane's 8 pattern pairs
    const int umax_l = a.umax[min(lane, kHalfPatch)];
    uint32_t pat[8];
#pragma unroll
    for (int r = 0; r < 8; r++) pat[r] = *reinterpret_cast<const uint32_t*>(c_pattern[r * 32 + hl]);
    // per-level data, one level per lane, fetched in the same round trip as
    // the tables above: keypoint count, offsets, stride, scale, patch size
    const int ll = min(lane, a.nlevels - 1);
    const int cnt_l = lane < a.nlevels ? a.level_count[(size_t)f * a.nlevels + lane] : 0;
    const long long off_l = a.levels[ll].off;
    const int stride_l = a.levels[ll].stride, loff_l = a.levels[ll].level_off;
    const float scale_l = a.levels[ll].scale, psize_l = a.levels[ll].patch_size;
    int total = 0, level = -1, local = 0;
    for (int l = 0; l < a.nlevels; l++) {
        const int c = __builtin_amdgcn_readlane(cnt_l, l);
        if (level < 0 && k < total + c) {
            level = l;
            local = k - total;
        }
        total += c;
    }
    if (k == 0 && lane == 0) {
        a.out_n[a.first_slot + f] = total;
        if (a.host_out) {   // every earlier kernel's error flags are final here
            reinterpret_cast<int32_t*>(a.host_out)[0] = total;
            reinterpret_cast<int32_t*>(a.host_out)[1] = *a.error_flags;
        }
    }
    // a wave keeps running while either half has a keypoint (DPP/ballot need
    // the whole wave); an empty half works on level 0 / key 0 and stores nothing
    const bool valid = level >= 0;
    if (!__any(valid)) return;
    if (!valid) {
        level = 0;
        local = 0;
    }
    // this half's level data, read back from lane `level`
    const int lv0 = __builtin_amdgcn_readlane(level, 0), lv1 = __builtin_amdgcn_readlane(level, 32);
    auto pick = [&](int v) {
        const int a0 = __builtin_amdgcn_readlane(v, lv0), a1 = __builtin_amdgcn_readlane(v, lv1);
        return half ? a1 : a0;
    };
    const long long lev_off = (long long)(((unsigned long long)(uint32_t)pick((int)(off_l >> 32)) << 32) |
                                          (uint32_t)pick((int)off_l));
    const int lev_stride = pick(stride_l), lev_loff = pick(loff_l);
    const float lev_scale = __int_as_float(pick(__float_as_int(scale_l)));
    const float lev_psize = __int_as_float(pick(__float_as_int(psize_l)));
    uint32_t e;
    float response;
    if (a.harris) {
        const uint64_t e64 = a.level_keys64[(size_t)f * a.level_entries + lev_loff + local];
        e = (uint32_t)e64;
        response = harris_response((uint32_t)(e64 >> 32));
    } else {
        e = a.level_keys[(size_t)f * a.level_entries + lev_loff + local];
        response = (float)(e >> 24);   // FAST score
    }
    const int y = (int)((e >> 12) & 0xFFF), x = (int)(e & 0xFFF);
    const int X = kEdge + (valid ? x : kHalfPatch + 8), Y = kEdge + (valid ? y : kHalfPatch + 8);
    uint8_t* ic = s_patch[slot];
    uint8_t* br = ic + kIcRows * kIcPitch;
    {
        const uint8_t* raw = a.pyr_raw + (size_t)f * a.frame_pyr_bytes + lev_off;
        const uint8_t* blr = a.pyr_blur + (size_t)f * a.frame_pyr_bytes + lev_off;
        const int ix0 = (X - kHalfPatch) & ~3, bx0 = (X - kBrR) & ~3;
        uint32_t* ic32 = reinterpret_cast<uint32_t*>(ic);
        uint32_t* br32 = reinterpret_cast<uint32_t*>(br);
        // both patches' loads (9 + 12 per lane) in flight together; 32-bit
        // offsets from the patches' first rows, (row, dword) stepped per load
        constexpr int nic = kIcRows * (kIcPitch / 4), nbr = kBrRows * (kBrPitch / 4);
        constexpr int qi = kIcPitch / 4, qb = kBrPitch / 4;
        const uint8_t* ri = raw + (long long)(Y - kHalfPatch) * lev_stride + ix0;
        const uint8_t* rb = blr + (long long)(Y - kBrR) * lev_stride + bx0;
        const uint32_t stride = (uint32_t)lev_stride;
        uint32_t vi[(nic + 31) / 32], vb[(nbr + 31) / 32];
        {
            int r = hl / qi, q = hl - (hl / qi) * qi;
#pragma unroll
            for (int k = 0; k < (nic + 31) / 32; k++) {
                const bool in = hl + 32 * k < nic;
                // lanes past the patch re-load (and below re-store) its last dword
                vi[k] = *reinterpret_cast<const uint32_t*>(
                    ri + (in ? (uint32_t)r * stride + 4u * (uint32_t)q : (uint32_t)(kIcRows - 1) * stride + 4u * (qi - 1)));
                r += 32 / qi;
                q += 32 % qi;
                if (q >= qi) {
                    q -= qi;
                    r++;
                }
            }
        }
        {
            int r = hl / qb, q = hl - (hl / qb) * qb;
#pragma unroll
            for (int k = 0; k < (nbr + 31) / 32; k++) {
                const bool in = hl + 32 * k < nbr;
                vb[k] = *reinterpret_cast<const uint32_t*>(
                    rb + (in ? (uint32_t)r * stride + 4u * (uint32_t)q : (uint32_t)(kBrRows - 1) * stride + 4u * (qb - 1)));
                r += 32 / qb;
                q += 32 % qb;
                if (q >= qb) {
                    q -= qb;
                    r++;
                }
            }
        }
#pragma unroll
        for (int k = 0; k < (nic + 31) / 32; k++) ic32[min(hl + 32 * k, nic - 1)] = vi[k];
#pragma unroll
        for (int k = 0; k < (nbr + 31) / 32; k++) br32[min(hl + 32 * k, nbr - 1)] = vb[k];
        ic += (X - kHalfPatch) - ix0 + kHalfPatch * kIcPitch + kHalfPatch;   // -> patch center
        br += (X - kBrR) - bx0 + kBrR * kBrPitch + kBrR;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // IC_Angle on the unblurred level (src/ORBextractor.cc:124-151): lane u
    // of the half takes column u - 15 over all rows of the circular patch
    int m01 = 0, m10 = 0;
    // umax read back from the lanes with readlane: no table loads in the loop
    if (hl < kIcRows) {
        const int u = hl - kHalfPatch;
        m10 = u * ic[u];
#pragma unroll
        for (int v = 1; v <= kHalfPatch; v++) {
            const int d = __builtin_amdgcn_readlane(umax_l, v);
            if (u >= -d && u <= d) {
                const int vp = ic[u + v * kIcPitch], vm = ic[u - v * kIcPitch];
                m01 += v * (vp - vm);
                m10 += u * (vp + vm);
            }
        }
    }
    m01 = half_wave_sum(m01);
    m10 = half_wave_sum(m10);
    const float angle = fast_atan2_deg((float)m01, (float)m10);
    // computeOrbDescriptor on the blurred level (src/ORBextractor.cc:155-194)
    const float factorPI = (float)(M_PI / 180.f);
    float sa, ca;
    cr_sincosf(__fmul_rn(angle, factorPI), &sa, &ca);
    uint8_t* desc = a.out_desc + ((size_t)(a.first_slot + f) * a.nfeatures + k) * 32;
    // the blurred patch centre as an offset into the block's LDS (exact in float)
    const uint8_t* lds_bytes = &s_patch[0][0];
    const float brf = (float)(int)(br - lds_bytes);
#pragma unroll
    for (int r = 0; r < 8; r++) {
        const orbx_f2 px = {(float)(int8_t)(pat[r] & 0xFF), (float)(int8_t)((pat[r] >> 16) & 0xFF)};
        const orbx_f2 py = {(float)(int8_t)((pat[r] >> 8) & 0xFF), (float)(int8_t)(pat[r] >> 24)};
        uint32_t a1, a2;
        orb_sample_addr2<kFma>(px, py, sa, ca, brf, a1, a2);
        const int t0 = lds_bytes[a1];
        const int t1 = lds_bytes[a2];
        const unsigned long long bits = __ballot(t0 < t1);
        // this half's 32 bits are descriptor bits 32r .. 32r+31 (bytes 4r .. 4r+3)
        if (valid && hl == r) {
            reinterpret_cast<uint32_t*>(desc)[r] = (uint32_t)(bits >> (32 * half));
            if (a.host_out)
                reinterpret_cast<uint32_t*>(a.host_out + 64 + (size_t)a.nfeatures * sizeof(orbx_keypoint) +
                                            (size_t)k * 32)[r] = (uint32_t)(bits >> (32 * half));
        }
    }
    if (valid && hl == 0) {
        orbx_keypoint kp;
        kp.x = (float)x;
        kp.y = (float)y;
        if (level != 0) {
            kp.x = __fmul_rn(kp.x, lev_scale);
            kp.y = __fmul_rn(kp.y, lev_scale);
        }
        kp.size = lev_psize;
        kp.angle = angle;
        kp.response = response;
        kp.octave = level;
        kp.class_id = -1;
        a.out_kps[(size_t)(a.first_slot + f) * a.nfeatures + k] = kp;
        if (a.host_out) reinterpret_cast<orbx_keypoint*>(a.host_out + 64)[k] = kp;
    }
}

// Diagnostics: the LDS introselect replay of k_retain_cells on one list of
// u32 entries (key << 24 | payload), one wavefront; also the global-memory
// replay of long lists (out_glb).
__global__ __launch_bounds__(64) void k_debug_nth(const uint32_t* in, int n, int nth, uint32_t* out_glb,
                                                  uint32_t* out_lds, int* gpos, int pivot_mode)
{
    __shared__ uint32_t list[kRetainCellCap];
    __shared__ int pos[kRetainCellCap + 8];
    const int lane = threadIdx.x;
    for (int i = lane; i < n; i += 64) out_glb[i] = in[i];
    global_wave_sync();
    wave_nth_element<true>(out_glb, n, nth, gpos, pivot_mode);
    for (int i = lane; i < n; i += 64) list[i] = in[i];
    lds_wave_sync();
    wave_nth_element(list, n, nth, pos, pivot_mode);
    for (int i = lane; i < n; i += 64) out_lds[i] = list[i];
}

}  // namespace orbx

extern "C" int orbx_debug_nth_pivot(const uint32_t* entries, int n, int nth, int pivot_mode, uint32_t* out_glb,
                                    uint32_t* out_lds)
{
    using namespace orbx;
    if (!entries || !out_glb || !out_lds || n < 0 || n > kRetainCellCap || nth < 0 || nth > n ||
        (pivot_mode != 0 && pivot_mode != 1))
        return ORBX_ERR_ARG;
    uint32_t* d = nullptr;
    if (hipMalloc(&d, 4 * sizeof(uint32_t) * (n + 8)) != hipSuccess) return ORBX_ERR_NOMEM;
    int r = ORBX_OK;
    if (hipMemcpy(d, entries, sizeof(uint32_t) * n, hipMemcpyHostToDevice) != hipSuccess) r = ORBX_ERR_HIP;
    if (r == ORBX_OK) {
        hipLaunchKernelGGL(k_debug_nth, dim3(1), dim3(64), 0, 0, d, n, nth, d + (n + 8), d + 2 * (n + 8),
                           reinterpret_cast<int*>(d + 3 * (n + 8)), pivot_mode);
        if (hipDeviceSynchronize() != hipSuccess ||
            hipMemcpy(out_glb, d + (n + 8), sizeof(uint32_t) * n, hipMemcpyDeviceToHost) != hipSuccess ||
            hipMemcpy(out_lds, d + 2 * (n + 8), sizeof(uint32_t) * n, hipMemcpyDeviceToHost) != hipSuccess)
            r = ORBX_ERR_HIP;
    }
    (void)hipFree(d);
    return r;
}

extern "C" int orbx_debug_nth(const uint32_t* entries, int n, int nth, uint32_t* out_glb, uint32_t* out_lds)
{
    return orbx_debug_nth_pivot(entries, n, nth, ORBX_NTH_PIVOT_GCC48, out_glb, out_lds);   // the default era
}

namespace orbx {

// ---------------------------------------------------------------------------
// Host launcher
// ---------------------------------------------------------------------------
int launch_extract(orbx_ctx* ctx, int first, int count, const MatchSpec* m)
{
    const Geometry& g = ctx->geom;
    if (count > 1 || (m && m->kind != 0 && ctx->async_match)) {   // the batch pipeline's streams
        const int r = ensure_aux_streams(ctx);
        if (r != ORBX_OK) return r;
    }
    for (int sl = first; sl < first + count && sl < (int)ctx->bow_ready.size(); sl++) ctx->bow_ready[sl] = 0;
    // frames still being uploaded (orbx_dev_upload_async): every part and
    // half below starts on, or is released from, the context stream
    wait_uploads_overlap(ctx, first, count, ctx->stream);
    ExtractArgs a;
    a.levels = ctx->dgeom.levels;
    a.cells = ctx->dgeom.cells;
    a.res_cols = ctx->dgeom.res_cols;
    a.res_rows = ctx->dgeom.res_rows;
    a.umax = ctx->dgeom.umax;
    a.frames = ctx->frames;
    // work buffers are per slot (frame f of this pass uses slot first + f):
    // batches on disjoint slots can be in flight at the same time
    a.pyr_raw = ctx->pyr_raw + (size_t)first * g.frame_pyr_bytes;
    a.pyr_blur = ctx->pyr_blur + (size_t)first * g.frame_pyr_bytes;
    a.cell_lists = ctx->cell_lists + (size_t)first * g.list_entries;
    a.cell_count = ctx->cell_count + (size_t)first * g.cells.size();
    a.level_keys = ctx->level_keys + (size_t)first * g.level_entries;
    a.level_count = ctx->level_count + (size_t)first * g.nlevels;
    a.out_kps = ctx->out_kps;
    a.out_desc = ctx->out_desc;
    a.out_n = ctx->out_n;
    a.error_flags = ctx->error_flags;
    a.host_out = ctx->single_frame ? ctx->single_out : nullptr;
    a.retain_scratch = ctx->retain_scratch + (size_t)first * (g.list_entries + 4 * g.cells.size());
    a.blur_tiles = ctx->blur_tiles;
    a.harris = ctx->harris;
    a.fp_contract = ctx->fp_contract;
    a.nth_pivot = ctx->nth_pivot;
    // the level retain holds a whole level list (+ scratch) in one block's LDS
    if ((size_t)((ctx->harris ? 3 : 2) * g.max_level_cap + 8) * 4 > 160 * 1024) return ORBX_ERR_UNSUPPORTED;
    a.cell_keys64 = ctx->harris ? ctx->cell_keys64 + (size_t)first * g.list_entries : nullptr;
    a.level_keys64 = ctx->harris ? ctx->level_keys64 + (size_t)first * g.level_entries : nullptr;
    a.frame_pyr_bytes = g.frame_pyr_bytes;
    a.w = g.w;
    a.h = g.h;
    a.nlevels = g.nlevels;
    a.ncells = (int)g.cells.size();
    a.list_entries = g.list_entries;
    a.level_entries = g.level_entries;
    a.nfeatures = g.nfeatures;
    a.fast_th = min(max(g.fast_th, 0), 255);
    a.fast_th_low = 7;
    a.max_list_cap = g.max_list_cap;
    a.max_level_cap = g.max_level_cap;

    // The pyramid stages over nb frames on stream st.
    auto run_pyramid = [&](const ExtractArgs& x, int nb, hipStream_t st) {
        // orbx_extract's single-frame graph: the whole raw pyramid in one
        // launch (its lowest latency; batches fill the chip with the staged
        // per-level launches below, which measured faster there)
        if (ctx->single_frame && g.cascade_bands > 0) {
            timer_begin(ctx, "resize", st);
            for (int rep = 0; rep < kDiagRepeat[0]; rep++) {
                {
                    int tab_off = (g.cascade_lds + 15) & ~15;
                    size_t lds = (size_t)tab_off + 8 * (size_t)(g.cascade_tab_cols + g.cascade_tab_rows);
                    if (lds > 160 * 1024) {   // very wide frames: the tables stay in HBM
                        tab_off = 0;
                        lds = g.cascade_lds;
                    }
                    hipLaunchKernelGGL(k_pyr_cascade<ORBX_CASCADE_SINGLE_THREADS>, dim3(g.cascade_bands, nb),
                                       dim3(ORBX_CASCADE_SINGLE_THREADS), lds, st, x, ctx->cascade, g.cascade_buf_x,
                                       tab_off, g.cascade_tab_cols);
                }
            }
            timer_end(ctx, "resize", st);
            return;
        }
        timer_begin(ctx, "pyr0", st);
        {
            const LevelGeom& L = g.levels[0];
            // interior 16-byte words: two aligned source loads cover them
            // (frames rows are 16-byte aligned when w % 16 == 0)
            const int qpr = L.stride / 16;
            int q_lo = (kEdge + 15) / 16, q_hi = (L.w + kEdge + kPyr0Shift - 32) / 16;
            q_hi = std::min(q_hi, qpr - 1);
            const int nint = (g.w % 16 == 0 && q_hi >= q_lo) ? q_hi - q_lo + 1 : 0;
            if (nint == 0) q_lo = 0;
            const int items = nint * ((L.ph + kPyrRows - 1) / kPyrRows) + (qpr - nint) * L.ph;
            hipLaunchKernelGGL(k_pyr_level0, dim3((items + 255) / 256, nb), dim3(256), 0, st, x, q_lo, nint);
        }
        timer_end(ctx, "pyr0", st);
        for (int l = 1; l < g.nlevels; l++) {
            const LevelGeom& L = g.levels[l];
            const LevelGeom& P = g.levels[l - 1];
            const int pitch = (kEdge + P.w + 15) & ~15;
            const size_t lds = (size_t)L.res_span * pitch + (size_t)L.w * sizeof(ResizeCol);
            timer_begin(ctx, "resize", st);
            if (lds <= kResizeLds) {
                const int threads = std::min(256, ((L.stride / 4) + 63) & ~63);
                // the packed form needs each interior word's taps within 8
                // bytes (source step < 2 keeps them within 7; a level just
                // over 2x, e.g. 333 -> 166, may not)
                int packed = 1;
                for (int x0 = 0; x0 + 3 < L.w; x0 += 4)
                    if (g.res_cols[L.res_col_off + x0 + 3].sx0 - g.res_cols[L.res_col_off + x0].sx0 > 6) packed = 0;
                const ResizeLevel rl{L.off, P.off, L.stride, P.stride, L.w, L.h, L.pw, L.ph, P.h, L.nvec_resize,
                                     L.res_span, L.res_strip_off, L.res_row_off, L.res_col_off, packed};
                for (int rep = 0; rep < kDiagRepeat[0]; rep++)
                    hipLaunchKernelGGL(k_pyr_resize_lds, dim3((L.ph + kResRows - 1) / kResRows, nb), dim3(threads), lds,
                                       st, x, rl, pitch);
            } else {   // very wide levels: per-pixel gathers from global memory
                const int items = (L.stride / 4) * ((L.ph + kPyrRows - 1) / kPyrRows);
                hipLaunchKernelGGL(k_pyr_resize, dim3((items + 255) / 256, nb), dim3(256), 0, st, x, l);
            }
            timer_end(ctx, "resize", st);
        }
    };
    // FAST .. describe over nb frames on stream st (after their pyramid).
    // parts: 1 = FAST, 2 = retain, 4 = blur, 8 = describe
    // 16 = FAST with the blur's blocks in the same launch where the FAST
    // instance takes them (whole cells at a template pitch), else FAST then blur
    auto run_rest = [&](const ExtractArgs& x, int nb, hipStream_t st, int parts) {
        const bool tail = (parts & 16) != 0;
        bool tail_done = false;
        if (parts & (1 | 16)) {
        timer_begin(ctx, "fast", st);
        {
            // widest aligned cell row and tallest cell pick the tile pitch
            int wmax = 0, hmax = 0;
            for (const CellGeom& c : g.cells) {
                if (!c.valid) continue;
                wmax = std::max(wmax, (15 + c.hx + 15) & ~15);
                hmax = std::max(hmax, c.hy);
            }
            const dim3 grid((int)g.cells.size(), nb);
            // Whole cells when a workgroup's LDS (tile + S' + nz + the static
            // survivor queues) stays within kFastLdsTarget (4 workgroups per
            // CU); taller cells are split into the fewest equal row bands
            // whose windows (band + 8 halo rows) fit.
            auto plan = [&](int P, int static_lds, int& band_rows) {
                band_rows = 0;
                const int whole = fast_tile_bytes(hmax, P);
                if (fast_lds_bytes(whole) + static_lds <= kFastLdsTarget || hmax <= 9) return whole;
                int wh = hmax;
                while (wh > 9 && fast_lds_bytes(fast_tile_bytes(wh, P)) + static_lds > kFastLdsTarget) wh--;
                const int nint = hmax - 6, bmax = wh - 8;
                const int nbands = (nint + bmax - 1) / bmax;
                band_rows = (nint + nbands - 1) / nbands;
                return fast_tile_bytes(std::min(hmax, band_rows + 8), P);
            };
            auto fast = [&](auto kern, int bytes, int band_rows, int threads) {
                const int lds = fast_lds_bytes(bytes);
                hipLaunchKernelGGL(kern, grid, dim3(threads), lds, st, x, bytes, band_rows);
            };
            auto fast_tail = [&](auto kern, int bytes) {
                const int lds = fast_lds_bytes(bytes);
                hipLaunchKernelGGL(kern, dim3((int)g.cells.size() + ctx->blur_tiles_n, nb), dim3(256), lds, st, x, bytes,
                                   0);
                tail_done = true;
            };
            // the templated instances queue u16 tile positions: windows of up
            // to 64 KB (larger ones take the runtime-pitch instance)
            // whole cells at the 96 / 144 / 208 pitches (their tiles fit four
            // workgroups per CU at the frame sizes of interest), row bands
            // where needed at 336 (1920x1080) and the runtime pitch
            int br = 0, bytes = 0;
            auto fits = [&](int P) {
                if (wmax > P) return false;
                bytes = fast_tile_bytes(hmax, P);
                return bytes <= 65536;
            };
            auto fits_banded = [&](int P) {
                if (wmax > P) return false;
                bytes = plan(P, fast_static_lds(false), br);
                return bytes <= 65536;
            };
            if (fits(96)) {
                if (tail) fast_tail(k_fast_cells<96, 256, false, true>, bytes);
                else fast(k_fast_cells<96>, bytes, 0, 256);
            } else if (fits(144)) {
                if (tail) fast_tail(k_fast_cells<144, 256, false, true>, bytes);
                else
                for (int rep = 0; rep < kDiagRepeat[3]; rep++) fast(k_fast_cells<144>, bytes, 0, 256);
            } else if (fits(208)) {
                if (tail) fast_tail(k_fast_cells<208, 256, false, true>, bytes);
                else fast(k_fast_cells<208>, bytes, 0, 256);
            }
            else if (fits_banded(336)) fast(k_fast_cells<336, kFastWideThreads, true>, bytes, br, kFastWideThreads);
            else {
                bytes = plan(wmax, fast_static_lds(true), br);
                fast(k_fast_cells<0, kFastWideThreads, true>, bytes, br, kFastWideThreads);
            }
        }
        timer_end(ctx, "fast", st);
        }
        if (parts & 2) {
        timer_begin(ctx, "retain", st);
        {
            // wave-private LDS (u32 words): cell list + partition scratch
            // (longer lists are replayed in global memory)
            const int ew = x.harris ? 2 : 1;   // u32 words per entry
            const int cw = (ew + 1) * kRetainCellCap + 8;
            const int cwaves = 4;
            const int lw = (ew + 1) * g.max_level_cap + 8;
            const int lwaves = 1;   // one level per block: small LDS blocks fit beside the other stream's kernels
            const dim3 cgrid(((int)g.cells.size() + cwaves - 1) / cwaves, nb), lgrid((g.nlevels + lwaves - 1) / lwaves, nb);
            if (x.harris) {
                hipLaunchKernelGGL(k_harris_cells, dim3((int)g.cells.size(), nb), dim3(256), 0, st, x);
                hipLaunchKernelGGL(k_retain_cells<uint64_t>, cgrid, dim3(64 * cwaves), (size_t)cwaves * cw * 4, st, x,
                                   cwaves, cw);
                hipLaunchKernelGGL(k_retain_levels<uint64_t>, lgrid, dim3(64 * lwaves), (size_t)lwaves * lw * 4, st, x,
                                   lwaves, lw);
            } else {
                hipLaunchKernelGGL(k_retain_cells<uint32_t>, cgrid, dim3(64 * cwaves), (size_t)cwaves * cw * 4, st, x,
                                   cwaves, cw);
                hipLaunchKernelGGL(k_retain_levels<uint32_t>, lgrid, dim3(64 * lwaves), (size_t)lwaves * lw * 4, st, x,
                                   lwaves, lw);
            }
        }
        timer_end(ctx, "retain", st);
        }
        if (parts & 4 || (tail && !tail_done)) {
            timer_begin(ctx, "blur", st);
            for (int rep = 0; rep < kDiagRepeat[1]; rep++)
                hipLaunchKernelGGL(k_blur, dim3(ctx->blur_tiles_n, nb), dim3(kBlurItems), 0, st, x, ctx->blur_tiles);
            timer_end(ctx, "blur", st);
        }
        if (!(parts & 8)) return;
        timer_begin(ctx, "describe", st);
        const dim3 dgrid((g.nfeatures + 2 * kWaves - 1) / (2 * kWaves), xcd_frames(nb));
        for (int rep = 0; rep < kDiagRepeat[2]; rep++) {
            if (x.fp_contract)
                hipLaunchKernelGGL(k_describe<true>, dgrid, dim3(256), 0, st, x, nb);
            else
                hipLaunchKernelGGL(k_describe<false>, dgrid, dim3(256), 0, st, x, nb);
        }
        timer_end(ctx, "describe", st);
    };
    auto run = [&](const ExtractArgs& x, int nb, hipStream_t st) {
        run_pyramid(x, nb, st);
        run_rest(x, nb, st, 15);
    };
    // Matching of slot s against prev(s) (the rule of orbx_dev_match_prev),
    // for the slots of [lo, hi) whose predecessor lies in [plo, phi) (all of
    // them when phi < 0), launched as contiguous runs on stream st.
    int err = ORBX_OK;
    auto match_runs = [&](int lo, int hi, int plo, int phi, hipStream_t st) {
        if (!m || m->kind == 0) return;
        auto prev = [&](int sl) { return (sl % m->seq_len == 0) ? sl + m->seq_len - 1 : sl - 1; };
        auto take = [&](int sl) {
            const int p = prev(sl);
            return phi < 0 || (p >= plo && p < phi);
        };
        for (int s0 = lo; s0 < hi;) {
            if (!take(s0)) {
                s0++;
                continue;
            }
            int s1 = s0 + 1;
            while (s1 < hi && take(s1)) s1++;
            const int r = m->kind == 1 ? launch_match_prev(ctx, s0, s1 - s0, m->seq_len, m->window, m->nnratio,
                                                           m->check_ori, st)
                                       : launch_match_bf_prev(ctx, s0, s1 - s0, m->seq_len, m->th_low, m->nnratio, st);
            if (r != ORBX_OK) err = r;
            s0 = s1;
        }
    };
    // Every buffer is indexed by slot: the frame store and outputs, and the
    // work buffers too (a.pyr_raw, cell_lists, retain_scratch, the key lists
    // are offset by `first`, and by a part's first slot below), so calls on
    // disjoint slot ranges never share scratch.  Parts launched on stream2 /
    // xstreams are never joined back to ctx->stream: later calls are ordered
    // after them only through the pending-match events that ctx_enter and
    // wait_pending_overlap wait on (the match stream waits for every part).
    // Large batches run
    // as two halves on two streams so that the VALU-bound FAST pass of one
    // half overlaps the latency-bound passes of the other; each half's
    // internal frame pairs are matched on its own stream, the pairs that
    // straddle the halves after the join.
    a.first_slot = first;
    const bool async = m && m->kind != 0 && ctx->async_match && ctx->mstream;
    // outputs of [first, first + count) are rewritten: a pending match that
    // reads any of them must finish first
    if (!async) {
        wait_pending_overlap(ctx, first, count, ctx->stream);
        ctx->stream_dirty = true;
    }
    if (async) {
        // Extraction, then the batch's matching on mstream, which overlaps
        // the next call's extraction of other slots.  Batches large enough
        // to split run as a software pipeline over two streams: the first
        // half's pyramid + FAST on the context stream, then its retain ..
        // describe while the second half (stream2, started at that point)
        // runs its pyramid + FAST; the next call's first half follows on the
        // context stream during the second half's tail.  The VALU-bound FAST
        // of one half thus overlaps the latency-bound stages of the other,
        // in steady state.  mstream's match waits for both halves.
        const int ways = std::min(ctx->split_ways, count / kSplitMinFrames);
        if (ctx->split && ways >= 2 && ctx->stream2) {
            // outputs of [first, first + count) are rewritten: pending matches
            // reading them finish first (the other parts' streams inherit it
            // through the release chain)
            wait_pending_overlap(ctx, first, count, ctx->stream);
            const hipStream_t S[orbx_ctx::kMaxWays] = {ctx->stream, ctx->stream2, ctx->xstreams[0], ctx->xstreams[1]};
            for (int i = 0; i < ways; i++) {
                const int lo = count * i / ways, n = count * (i + 1) / ways - lo;
                ExtractArgs b = a;
                b.first_slot = first + lo;
                b.pyr_raw += (size_t)lo * a.frame_pyr_bytes;
                b.pyr_blur += (size_t)lo * a.frame_pyr_bytes;
                b.cell_lists += (size_t)lo * a.list_entries;
                b.retain_scratch += (size_t)lo * (a.list_entries + 4 * a.ncells);
                b.cell_count += (size_t)lo * a.ncells;
                b.level_keys += (size_t)lo * a.level_entries;
                if (a.harris) {
                    b.cell_keys64 += (size_t)lo * a.list_entries;
                    b.level_keys64 += (size_t)lo * a.level_entries;
                }
                b.level_count += (size_t)lo * a.nlevels;
                // part i starts once part i - 1 is past its FAST pass
                if (i > 0) ORBX_HIP_CHECK(hipStreamWaitEvent(S[i], ctx->ev_part_fast[i - 1], 0));
                run_pyramid(b, n, S[i]);
                run_rest(b, n, S[i], 1);
                ORBX_HIP_CHECK(hipEventRecord(ctx->ev_part_fast[i], S[i]));
                run_rest(b, n, S[i], 14);
                ORBX_HIP_CHECK(hipEventRecord(ctx->ev_part_done[i], S[i]));
                ORBX_HIP_CHECK(hipStreamWaitEvent(ctx->mstream, ctx->ev_part_done[i], 0));
            }
        } else {
            const int r = launch_extract(ctx, first, count, nullptr);
            if (r != ORBX_OK) return r;
            ORBX_HIP_CHECK(hipEventRecord(ctx->ev_extracted, ctx->stream));
            ORBX_HIP_CHECK(hipStreamWaitEvent(ctx->mstream, ctx->ev_extracted, 0));
        }
        match_runs(first, first + count, 0, -1, ctx->mstream);
        // the match reads the outputs of the batch's sequences
        const int q = m->seq_len;
        const int lo = (first / q) * q, hi = ((first + count + q - 1) / q) * q;
        ORBX_HIP_CHECK(push_pending(ctx, lo, hi));
        if (err != ORBX_OK) return err;
        if (hipGetLastError() != hipSuccess) return ORBX_ERR_HIP;
        return ORBX_OK;
    }
    if (ctx->split && count >= 2 * kSplitMinFrames && ctx->stream2) {
        const int n0 = count / 2, n1 = count - n0;
        ExtractArgs b = a;
        b.first_slot = first + n0;
        b.pyr_raw += (size_t)n0 * a.frame_pyr_bytes;
        b.pyr_blur += (size_t)n0 * a.frame_pyr_bytes;
        b.cell_lists += (size_t)n0 * a.list_entries;
        b.retain_scratch += (size_t)n0 * (a.list_entries + 4 * a.ncells);
        b.cell_count += (size_t)n0 * a.ncells;
        b.level_keys += (size_t)n0 * a.level_entries;
        if (a.harris) {
            b.cell_keys64 += (size_t)n0 * a.list_entries;
            b.level_keys64 += (size_t)n0 * a.level_entries;
        }
        b.level_count += (size_t)n0 * a.nlevels;
        ORBX_HIP_CHECK(hipEventRecord(ctx->ev_fork, ctx->stream));
        ORBX_HIP_CHECK(hipStreamWaitEvent(ctx->stream2, ctx->ev_fork, 0));
        run(a, n0, ctx->stream);
        match_runs(first, first + n0, first, first + n0, ctx->stream);
        run(b, n1, ctx->stream2);
        match_runs(first + n0, first + count, first + n0, first + count, ctx->stream2);
        ORBX_HIP_CHECK(hipEventRecord(ctx->ev_join, ctx->stream2));
        ORBX_HIP_CHECK(hipStreamWaitEvent(ctx->stream, ctx->ev_join, 0));
        // straddling pairs (predecessor in the other half, or outside the batch)
        match_runs(first, first + n0, first + n0, 0x7fffffff, ctx->stream);
        match_runs(first, first + n0, -0x7fffffff, first, ctx->stream);
        match_runs(first + n0, first + count, first, first + n0, ctx->stream);
        match_runs(first + n0, first + count, first + count, 0x7fffffff, ctx->stream);
        match_runs(first + n0, first + count, -0x7fffffff, first, ctx->stream);
    } else if (ctx->single_frame && count == 1) {
        // one frame (orbx_extract's captured graph), for latency: the raw
        // pyramid as one cascade launch, FAST with the blur's blocks in its
        // grid (a branch for the blur measured slower: the cross-queue join
        // cost more than the blur), then retain and describe
        run_pyramid(a, 1, ctx->stream);
        run_rest(a, 1, ctx->stream, 16 | 2 | 8);
        match_runs(first, first + count, 0, -1, ctx->stream);
    } else {
        run(a, count, ctx->stream);
        match_runs(first, first + count, 0, -1, ctx->stream);
    }
    if (err != ORBX_OK) return err;
    if (hipGetLastError() != hipSuccess) return ORBX_ERR_HIP;
    return ORBX_OK;
}


}  // namespace orbx
