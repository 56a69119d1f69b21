// ORB extraction on MI355X (gfx950): ORBextractor::operator()
// (src/ORBextractor.cc:718-779) for a batch of frames, one launch per stage:
//
//   k_pyr_level0   copyMakeBorder(REFLECT_101) of the input   (:814)
//   k_pyr_resize   resize INTER_LINEAR + border, level l      (:800, :806)
//   k_fast_cells   FAST-9/16 + cell-local NMS + threshold-7
//                  fallback + raster-order compaction, one
//                  workgroup per grid cell                    (:599-614)
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

#include "orbx_device.h"
#include "orbx_internal.h"

namespace orbx {

constexpr size_t kRetainLds = 128 * 1024;   // LDS budget of a retain block
constexpr int kRetainCellCap = 1024;        // cell lists up to this length sort in LDS
constexpr int kSplitMinFrames = 16;         // batches >= 2x this run as two concurrent halves

__constant__ int8_t c_pattern[256][4] = {
#include "orbx_pattern.inc"
};

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
    int32_t* retain_scratch;        // slots x (list_entries + 4 ncells): global nth_element scratch
    long long frame_pyr_bytes;
    int first_slot;
    int w, h;
    int nlevels, ncells, list_entries, level_entries, nfeatures;
    int fast_th, fast_th_low;       // FAST thresholds (fastTh, 7), clamped
    int max_list_cap, max_level_cap;
};

__device__ inline int reflect101(int p, int len)
{
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    do {
        if (p < 0) p = -p;
        else p = 2 * len - 2 - p;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}

__device__ inline uint8_t sat_u8(int v) { return (uint8_t)min(max(v, 0), 255); }
__device__ inline int sat_s16(int v) { return min(max(v, -32768), 32767); }

// (row, column) walk of a row-major index advancing by a fixed stride,
// without a division per step.
struct RowWalk {
    int r, q, dr, dq, nq;
    __device__ RowWalk(int start, int stride, int n_q) : nq(n_q)
    {
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


// ---------------------------------------------------------------------------
// Level 0: padded copy with BORDER_REFLECT_101.  4 output bytes per thread.
// ---------------------------------------------------------------------------
// One thread per (dword column, strip of kPyrRows rows): the column's
// reflected source offsets are computed once and the strip's independent
// row loads are in flight together.
constexpr int kPyrRows = 8;

__global__ __launch_bounds__(256) void k_pyr_level0(ExtractArgs a)
{
    const int f = blockIdx.y;
    const LevelGeom L = a.levels[0];
    const int wpr = L.stride >> 2, nstrips = (L.ph + kPyrRows - 1) / kPyrRows;
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= wpr * nstrips) return;
    const int strip = idx / wpr, q = idx - strip * wpr, px0 = 4 * q;
    const uint8_t* src = a.frames + (size_t)(a.first_slot + f) * a.w * a.h;
    uint8_t* dst = a.pyr_raw + (size_t)f * a.frame_pyr_bytes + L.off;
    const bool aligned = (px0 - kEdge) >= 0 && (px0 - kEdge + 3) < L.w && (a.w & 3) == 0;
    int sx[4];
#pragma unroll
    for (int b = 0; b < 4; b++) sx[b] = (px0 + b < L.pw) ? reflect101(px0 + b - kEdge, L.w) : -1;
#pragma unroll
    for (int rr = 0; rr < kPyrRows; rr++) {
        // rows past the level repeat the last one (loads stay in bounds and
        // can all be issued up front); their stores are skipped
        const int py = min(strip * kPyrRows + rr, L.ph - 1);
        const uint8_t* row = src + (size_t)reflect101(py - kEdge, L.h) * a.w;
        uint32_t word;
        if (aligned) {
            word = *reinterpret_cast<const uint32_t*>(row + px0 - kEdge);
        } else {
            word = 0;
#pragma unroll
            for (int b = 0; b < 4; b++)
                if (sx[b] >= 0) word |= (uint32_t)row[sx[b]] << (8 * b);
        }
        if (strip * kPyrRows + rr < L.ph) *reinterpret_cast<uint32_t*>(dst + (size_t)py * L.stride + px0) = word;
    }
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
    const LevelGeom L = a.levels[level];
    const LevelGeom P = a.levels[level - 1];
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

// ---------------------------------------------------------------------------
// FAST-9/16 score map.  For a pixel with value v and ring d_k = v - p_k
// (k = 0..15, OpenCV offsets), S = max(M_dark, M_bright) - 1 where M_dark is
// the best 9-arc minimum of d and M_bright that of -d.  FAST at threshold t
// classifies the pixel as a corner iff S >= t, and cornerScore<16> returns
// exactly S (OpenCV 2.4 fast.cpp / fast_score.cpp).  A pixel whose compass
// pre-test passes in one direction only has S = that direction's arc - 1.
// ---------------------------------------------------------------------------
// Best 9-arc minimum of sgn * (v - p_k) (the "dark" arc for sgn = +1, the
// "bright" arc for sgn = -1).
__device__ inline int fast_arc(const uint8_t* t, int pitch, int sgn)
{
    const int off[16] = {3 * pitch,      1 + 3 * pitch, 2 + 2 * pitch,  3 + pitch,
                         3,              3 - pitch,     2 - 2 * pitch,  1 - 3 * pitch,
                         -3 * pitch,     -1 - 3 * pitch, -2 - 2 * pitch, -3 - pitch,
                         -3,             -3 + pitch,    -2 + 2 * pitch, -1 + 3 * pitch};
    // x_k = sgn * (v - p_k) as one 24-bit multiply-add per ring pixel
    const int c = sgn * (int)t[0], s = -sgn;
    int x[16], m3[16];
#pragma unroll
    for (int k = 0; k < 16; k++) x[k] = (int)t[off[k]] * s + c;
    // min over 9 consecutive = min of three consecutive 3-minima
#pragma unroll
    for (int k = 0; k < 16; k++) m3[k] = min(min(x[k], x[(k + 1) & 15]), x[(k + 2) & 15]);
    int best = -1000;
#pragma unroll
    for (int k = 0; k < 16; k++) best = max(best, min(min(m3[k], m3[(k + 3) & 15]), m3[(k + 6) & 15]));
    return best;
}

// One workgroup per (cell, frame).  LDS: the cell ROI with dword-aligned rows
// (tile), its S' map (sm), and one candidate buffer per wave.
//  1. compass pre-test, 4 pixels per thread: a 9-arc covers two adjacent
//     compass points, so S >= tmin needs d > tmin (or < -tmin) on both;
//     survivors are compacted per wave and scored with all lanes busy;
//  2. non-max suppression, 4 pixels per thread (result kept over `tile`);
//  3. raster-order compaction of the corners at the chosen threshold.
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

// byte k (0..11) of the 12-byte window lo|mid|hi
__device__ inline int byte12(uint32_t lo, uint32_t mid, uint32_t hi, int k)
{
    return k < 4 ? byte_of(lo, k) : (k < 8 ? byte_of(mid, k - 4) : byte_of(hi, k - 8));
}

__global__ __launch_bounds__(256) void k_fast_cells(ExtractArgs a, int tile_pitch_bytes)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    __shared__ BlockScratch bs;
    __shared__ uint32_t cand[kWaves][256];   // tile position | direction flags << 16
    const int cell = blockIdx.x, f = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const CellGeom C = a.cells[cell];
    int32_t* count_out = a.cell_count + (size_t)f * a.ncells + cell;
    if (!C.valid) {
        if (tid == 0) *count_out = 0;
        return;
    }
    const LevelGeom L = a.levels[C.level];
    const int roi_x = kEdge + C.ini_x, x_al = roi_x & ~3, sh = roi_x - x_al;
    const int hx = C.hx, hy = C.hy;
    const int P = (sh + hx + 3) & ~3, nq = P >> 2;     // tile pitch, dwords per row
    const uint8_t* src = a.pyr_raw + (size_t)f * a.frame_pyr_bytes + L.off + (size_t)(kEdge + C.ini_y) * L.stride + x_al;
    uint8_t* tile = smem;
    uint8_t* sm = smem + tile_pitch_bytes;
    uint32_t* tile32 = reinterpret_cast<uint32_t*>(tile);
    uint32_t* sm32 = reinterpret_cast<uint32_t*>(sm);
    {
        RowWalk w(tid, kBlock, nq);
        for (int i = tid; i < hy * nq; i += kBlock, w.next())
            tile32[i] = *reinterpret_cast<const uint32_t*>(src + (size_t)w.r * L.stride + 4 * w.q);
    }
    // S' is 0 outside the interior rows [3, hy-4]; the interior rows are
    // fully rewritten below
    for (int i = tid; i < nq; i += kBlock) {
        sm32[2 * nq + i] = 0;
        sm32[(hy - 3) * nq + i] = 0;
    }
    __syncthreads();
    const int tmin = min(a.fast_th, a.fast_th_low);
    const int c_lo = 3 + sh, c_hi = hx - 4 + sh;         // interior tile columns
    const int nunits = (hy - 6) * nq;
    RowWalk cw_(wv * 64 + lane, kBlock, nq);
    for (int u0 = wv * 64; u0 < nunits; u0 += kBlock, cw_.next()) {
        const int u = u0 + lane;
        const int r = 3 + cw_.r, q = cw_.q;
        int mask = 0;
        if (u < nunits) {
            const uint32_t* row = tile32 + r * nq + q;
            const uint32_t mid = row[0];
            const uint32_t lo = q > 0 ? row[-1] : 0u, hi = q + 1 < nq ? row[1] : 0u;
            const uint32_t up = row[-3 * nq], dn = row[3 * nq];
            // 4 pixels at once: even / odd bytes as two u16x2 halves, packed
            // 16-bit arithmetic; a lane's sign bit set = "test fails"
            const uint32_t p4w = __builtin_amdgcn_alignbyte(hi, mid, 3);    // bytes j+3
            const uint32_t p12w = __builtin_amdgcn_alignbyte(mid, lo, 1);   // bytes j-3
            const uint32_t T1 = (uint32_t)(tmin + 1) * 0x00010001u;
            const uint32_t NT1 = (uint32_t)(-(tmin + 1) & 0xFFFF) * 0x00010001u;
            int ok[2][2];   // [half][dark, bright] sign-bit masks of passing lanes
#pragma unroll
            for (int hf = 0; hf < 2; hf++) {
                const uint32_t sel = hf ? 0x0c030c01u : 0x0c020c00u;   // bytes 1,3 or 0,2 -> u16x2
                const uint32_t v = __builtin_amdgcn_perm(0u, mid, sel);
                const uint32_t pk[4] = {__builtin_amdgcn_perm(0u, dn, sel), __builtin_amdgcn_perm(0u, p4w, sel),
                                        __builtin_amdgcn_perm(0u, up, sel), __builtin_amdgcn_perm(0u, p12w, sel)};
                uint32_t xd[4], xb[4];
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const uint32_t d = pk_sub16(v, pk[k]);     // v - p
                    xd[k] = pk_sub16(d, T1);                   // >= 0 <=> v - p > t
                    xb[k] = pk_sub16(NT1, d);                  // >= 0 <=> p - v > t
                }
                const uint32_t failD = (xd[0] | xd[1]) & (xd[1] | xd[2]) & (xd[2] | xd[3]) & (xd[3] | xd[0]);
                const uint32_t failB = (xb[0] | xb[1]) & (xb[1] | xb[2]) & (xb[2] | xb[3]) & (xb[3] | xb[0]);
                ok[hf][0] = (int)(~failD & 0x80008000u);
                ok[hf][1] = (int)(~failB & 0x80008000u);
            }
            // pixel j: bit 2j dark, 2j+1 bright (even half: j = 0, 2; odd: 1, 3)
            mask = ((ok[0][0] >> 15) & 1) | ((ok[0][1] >> 14) & 2) |                          // j = 0
                   (((ok[1][0] >> 15) & 1) << 2) | (((ok[1][1] >> 14) & 2) << 2) |              // j = 1
                   (((ok[0][0] >> 31) & 1) << 4) | ((((unsigned)ok[0][1] >> 30) & 2) << 4) |     // j = 2
                   (((ok[1][0] >> 31) & 1) << 6) | ((((unsigned)ok[1][1] >> 30) & 2) << 6);     // j = 3
            // interior columns only
            const int j0 = max(c_lo - 4 * q, 0), j1 = min(c_hi - 4 * q, 3);
            mask = (j1 < j0) ? 0 : (mask & (((1 << (2 * (j1 + 1))) - 1) & ~((1 << (2 * j0)) - 1)));
            sm32[r * nq + q] = 0;
        }
        const int cnt = __popc((mask | (mask >> 1)) & 0x55);
        const int incl = wave_inclusive_scan(cnt);
        const int ntot = __builtin_amdgcn_readlane(incl, 63);
        int w = incl - cnt;
        if (mask) {
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int fl = (mask >> (2 * j)) & 3;
                if (fl) cand[wv][w++] = (uint32_t)(r * P + 4 * q + j) | ((uint32_t)fl << 16);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (int i0 = 0; i0 < ntot; i0 += 64) {
            const int i = i0 + lane;
            const uint32_t cw = i < ntot ? cand[wv][i] : 0u;
            const int pos = (int)(cw & 0xFFFF), fl = (int)(cw >> 16);
            int S = 0;
            if (fl) S = fast_arc(tile + pos, P, (fl & 1) ? 1 : -1);
            if (__any(fl == 3) && fl == 3) S = max(S, fast_arc(tile + pos, P, -1));
            S -= 1;
            if (fl) sm[pos] = (uint8_t)(S >= tmin ? S : 0);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    __syncthreads();
    // non-max suppression: keep S' if it beats all 8 neighbours' S'
    int c1 = 0;
    RowWalk nw(tid, kBlock, nq);
    for (int u = tid; u < nunits; u += kBlock, nw.next()) {
        const int r = 3 + nw.r, q = nw.q;
        uint32_t word = 0;
        const uint32_t* m = sm32 + r * nq + q;
        const uint32_t mid = m[0];
        if (mid) {
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
            const uint32_t FT = (uint32_t)max(a.fast_th, 1) * 0x00010001u;
#pragma unroll
            for (int hf = 0; hf < 2; hf++) {
                const uint32_t sel = hf ? 0x0c030c01u : 0x0c020c00u;
                uint32_t mx = __builtin_amdgcn_perm(0u, nb[0], sel);
#pragma unroll
                for (int i = 1; i < 8; i++) mx = pk_max16(mx, __builtin_amdgcn_perm(0u, nb[i], sel));
                const uint32_t sv = __builtin_amdgcn_perm(0u, mid, sel);
                // keep where mx - s < 0 (s > every neighbour)
                const uint32_t keep = ((pk_sub16(mx, sv) & 0x80008000u) >> 15) * 0xFFu;
                const uint32_t kept = sv & keep;
                word |= kept << (8 * hf);
                // corners at fastTh among the kept (kept >= max(fastTh, 1))
                c1 += __popc(~pk_sub16(kept, FT) & 0x80008000u);
            }
        }
        tile32[r * nq + q] = word;
    }
    // threshold choice: FAST(fastTh); if <= 3 corners, FAST(7) (:607-614)
    const int n1 = block_sum(c1, bs, 0);
    const int t = (n1 <= 3) ? a.fast_th_low : a.fast_th;
    uint32_t* out = a.cell_lists + (size_t)f * a.list_entries + C.list_off;
    int base = 0, buf = 1;
    RowWalk ow(tid, kBlock, nq);
    for (int u0 = 0; u0 < nunits; u0 += kBlock, ow.next()) {
        const int u = u0 + tid;
        uint32_t word = 0;
        int cnt = 0;
        if (u < nunits) {
            word = tile32[(3 + ow.r) * nq + ow.q];
#pragma unroll
            for (int j = 0; j < 4; j++) cnt += byte_of(word, j) >= t && byte_of(word, j) > 0;
        }
        int total;
        int off = base + block_exclusive_scan(cnt, &total, bs, buf);
        buf ^= 1;
        if (cnt) {
            const int r = 3 + ow.r, q = ow.q;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int s = byte_of(word, j);
                if (s >= t && s > 0 && off < C.list_cap) {
                    const int cc = 4 * q + j - sh;   // ROI column
                    out[off] = ((uint32_t)s << 24) | ((uint32_t)(C.ini_y + r) << 12) | (uint32_t)(C.ini_x + cc);
                }
                off += (s >= t && s > 0);
            }
        }
        base += total;
    }
    if (tid == 0) {
        *count_out = base;
        if (base > C.list_cap) atomicOr(a.error_flags, 1);
    }
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
#pragma unroll
    for (int k = 0; k < kPer; k++) {
        const int c = lane + 64 * k;
        tot[k] = 0;
        ret[k] = 0;
        nomore[k] = false;
        if (c < nCells) {
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

__global__ __launch_bounds__(256) void k_retain_cells(ExtractArgs a, int waves_per_block, int wave_words)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t sbuf[];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int cell = blockIdx.x * waves_per_block + wv, f = blockIdx.y;
    if (cell >= a.ncells) return;
    uint32_t* list = sbuf + (size_t)wv * wave_words;
    int* pos = reinterpret_cast<int*>(list + kRetainCellCap);
    const CellGeom C = a.cells[cell];
    const LevelGeom L = a.levels[C.level];
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
    uint32_t* src = a.cell_lists + (size_t)f * a.list_entries + C.list_off;
    uint32_t* dst = a.level_keys + (size_t)f * a.level_entries + L.level_off + pre;
    if (n > k && n <= kRetainCellCap) {
        for (int i = lane; i < n; i += 64) list[i] = src[i];
        lds_wave_sync();
        wave_nth_element(list, n, k, pos);
        for (int i = lane; i < take; i += 64) dst[i] = list[i];
    } else if (n > k) {
        // long list: replay in place in global memory
        int* gpos = a.retain_scratch + (size_t)f * (a.list_entries + 4 * a.ncells) + C.list_off + 4 * cell;
        wave_nth_element<true>(src, n, k, gpos);
        for (int i = lane; i < take; i += 64) dst[i] = src[i];
    } else {
        for (int i = lane; i < take; i += 64) dst[i] = src[i];
    }
}

__global__ __launch_bounds__(256) void k_retain_levels(ExtractArgs a, int waves_per_block, int wave_words)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t sbuf[];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int level = blockIdx.x * waves_per_block + wv, f = blockIdx.y;
    if (level >= a.nlevels) return;
    const LevelGeom L = a.levels[level];
    int32_t* cnt = a.level_count + (size_t)f * a.nlevels + level;
    const int nlev = *cnt;
    if (nlev <= L.n_desired) return;
    uint32_t* list = sbuf + (size_t)wv * wave_words;
    int* pos = reinterpret_cast<int*>(list + a.max_level_cap);
    uint32_t* g = a.level_keys + (size_t)f * a.level_entries + L.level_off;
    for (int i = lane; i < nlev; i += 64) list[i] = g[i];
    lds_wave_sync();
    wave_nth_element(list, nlev, L.n_desired, pos);
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
    const uint32_t wl = w[-1], wc = w[0], wr = w[1];
    int b[12];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        b[k] = (wl >> (8 * k)) & 0xFF;
        b[4 + k] = (wc >> (8 * k)) & 0xFF;
        b[8 + k] = (wr >> (8 * k)) & 0xFF;
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const int c = 4 + j;
        hs[j] = 55 * b[c] + 49 * (b[c - 1] + b[c + 1]) + 34 * (b[c - 2] + b[c + 2]) + 18 * (b[c - 3] + b[c + 3]);
    }
}

__global__ __launch_bounds__(256) void k_blur(ExtractArgs a, const int4* tiles)
{
    const int f = blockIdx.y;
    const int4 tl = tiles[blockIdx.x];   // level, first item, dwords per row, strips
    const int item = tl.y + threadIdx.x;
    if (item >= tl.z * tl.w) return;
    const LevelGeom L = a.levels[tl.x];
    const int strip = item / tl.z, dw = item - strip * tl.z;
    const int x = dw * 4;
    const int y0 = strip * kBlurStrip, y1 = min(y0 + kBlurStrip, L.ph);
    const uint8_t* src = a.pyr_raw + (size_t)f * a.frame_pyr_bytes + L.off;
    uint8_t* dst = a.pyr_blur + (size_t)f * a.frame_pyr_bytes + L.off;
    // interior columns / rows of this level in padded coordinates
    const int ix0 = kEdge, ix1 = kEdge + L.w, iy0 = kEdge, iy1 = kEdge + L.h;
    const bool col_interior = (x + 3 >= ix0) && (x < ix1);
    // rows [ya, yb) of this strip are blurred, the rest copied
    const int ya = col_interior ? max(y0, iy0) : y1;
    const int yb = col_interior ? min(y1, iy1) : y1;
    // bytes beyond the padded width (row pitch padding) are zero
    uint32_t keep_mask = 0;
#pragma unroll
    for (int j = 0; j < 4; j++)
        if (x + j < L.pw) keep_mask |= 0xFFu << (8 * j);
    for (int y = y0; y < min(ya, y1); y++)
        *reinterpret_cast<uint32_t*>(dst + (size_t)y * L.stride + x) =
            *reinterpret_cast<const uint32_t*>(src + (size_t)y * L.stride + x) & keep_mask;
    if (ya < yb) {
        int R[7][4];
#pragma unroll
        for (int k = 0; k < 6; k++) blur_hsum(src + (size_t)(ya - 3 + k) * L.stride, x, R[k]);
        for (int y = ya; y < yb; y++) {
            blur_hsum(src + (size_t)(y + 3) * L.stride, x, R[6]);
            const uint32_t raw = *reinterpret_cast<const uint32_t*>(src + (size_t)y * L.stride + x);
            uint32_t word = 0;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int xi = x + j - kEdge;
                uint32_t v = (raw >> (8 * j)) & 0xFF;
                if (xi >= 0 && xi < L.w) {
                    const int N = 55 * R[3][j] + 49 * (R[2][j] + R[4][j]) + 34 * (R[1][j] + R[5][j]) +
                                  18 * (R[0][j] + R[6][j]);
                    int q;
                    if (xi < L.nvec_blur) {   // float path: exact N/2^16, cvtps2dq rounding
                        q = N >> 16;
                        const int rem = N & 0xFFFF;
                        if (rem > 0x8000 || (rem == 0x8000 && (q & 1))) q++;
                    } else {
                        q = (N + (1 << 15)) >> 16;
                    }
                    v = (uint32_t)sat_u8(q);
                }
                word |= v << (8 * j);
            }
            *reinterpret_cast<uint32_t*>(dst + (size_t)y * L.stride + x) = word & keep_mask;
#pragma unroll
            for (int k = 0; k < 6; k++)
#pragma unroll
                for (int j = 0; j < 4; j++) R[k][j] = R[k + 1][j];
        }
    }
    for (int y = max(yb, ya); y < y1; y++)
        *reinterpret_cast<uint32_t*>(dst + (size_t)y * L.stride + x) =
            *reinterpret_cast<const uint32_t*>(src + (size_t)y * L.stride + x) & keep_mask;
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
__global__ __launch_bounds__(256) void k_describe(ExtractArgs a)
{
    __shared__ __attribute__((aligned(16))) uint8_t s_patch[2 * kWaves][kDescWaveBytes];
    const int f = blockIdx.y;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, half = lane >> 5, hl = lane & 31;
    const int slot = wv * 2 + half;
    const int k = blockIdx.x * (2 * kWaves) + slot;
    const int32_t* lc = a.level_count + (size_t)f * a.nlevels;
    int total = 0, level = -1, local = 0;
    for (int l = 0; l < a.nlevels; l++) {
        const int c = lc[l];
        if (level < 0 && k < total + c) {
            level = l;
            local = k - total;
        }
        total += c;
    }
    if (k == 0 && lane == 0) a.out_n[a.first_slot + f] = total;
    // a wave keeps running while either half has a keypoint (DPP/ballot need
    // the whole wave); an empty half works on level 0 / key 0 and stores nothing
    const bool valid = level >= 0;
    if (!__any(valid)) return;
    if (!valid) {
        level = 0;
        local = 0;
    }
    const LevelGeom L = a.levels[level];
    const uint32_t e = a.level_keys[(size_t)f * a.level_entries + L.level_off + local];
    const int score = (int)(e >> 24), y = (int)((e >> 12) & 0xFFF), x = (int)(e & 0xFFF);
    const int X = kEdge + (valid ? x : kHalfPatch + 8), Y = kEdge + (valid ? y : kHalfPatch + 8);
    uint8_t* ic = s_patch[slot];
    uint8_t* br = ic + kIcRows * kIcPitch;
    {
        const uint8_t* raw = a.pyr_raw + (size_t)f * a.frame_pyr_bytes + L.off;
        const uint8_t* blr = a.pyr_blur + (size_t)f * a.frame_pyr_bytes + L.off;
        const int ix0 = (X - kHalfPatch) & ~3, bx0 = (X - kBrR) & ~3;
        uint32_t* ic32 = reinterpret_cast<uint32_t*>(ic);
        uint32_t* br32 = reinterpret_cast<uint32_t*>(br);
        for (int i = hl; i < kIcRows * (kIcPitch / 4); i += 32) {
            const int r = i / (kIcPitch / 4), q = i - r * (kIcPitch / 4);
            ic32[i] = *reinterpret_cast<const uint32_t*>(raw + (size_t)(Y - kHalfPatch + r) * L.stride + ix0 + 4 * q);
        }
        for (int i = hl; i < kBrRows * (kBrPitch / 4); i += 32) {
            const int r = i / (kBrPitch / 4), q = i - r * (kBrPitch / 4);
            br32[i] = *reinterpret_cast<const uint32_t*>(blr + (size_t)(Y - kBrR + r) * L.stride + bx0 + 4 * q);
        }
        ic += (X - kHalfPatch) - ix0 + kHalfPatch * kIcPitch + kHalfPatch;   // -> patch center
        br += (X - kBrR) - bx0 + kBrR * kBrPitch + kBrR;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // IC_Angle on the unblurred level (src/ORBextractor.cc:124-151): lane u
    // of the half takes column u - 15 over all rows of the circular patch
    int m01 = 0, m10 = 0;
    if (hl < kIcRows) {
        const int u = hl - kHalfPatch;
        m10 = u * ic[u];
        for (int v = 1; v <= kHalfPatch; v++) {
            const int d = a.umax[v];
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
#pragma unroll
    for (int r = 0; r < 8; r++) {
        const int q = r * 32 + hl;
        const float px1 = c_pattern[q][0], py1 = c_pattern[q][1];
        const float px2 = c_pattern[q][2], py2 = c_pattern[q][3];
        const int t0 = br[cv_round(__fadd_rn(__fmul_rn(px1, sa), __fmul_rn(py1, ca))) * kBrPitch +
                          cv_round(__fsub_rn(__fmul_rn(px1, ca), __fmul_rn(py1, sa)))];
        const int t1 = br[cv_round(__fadd_rn(__fmul_rn(px2, sa), __fmul_rn(py2, ca))) * kBrPitch +
                          cv_round(__fsub_rn(__fmul_rn(px2, ca), __fmul_rn(py2, sa)))];
        const unsigned long long bits = __ballot(t0 < t1);
        // this half's 32 bits are descriptor bits 32r .. 32r+31 (bytes 4r .. 4r+3)
        if (valid && hl == r) reinterpret_cast<uint32_t*>(desc)[r] = (uint32_t)(bits >> (32 * half));
    }
    if (valid && hl == 0) {
        orbx_keypoint kp;
        kp.x = (float)x;
        kp.y = (float)y;
        if (level != 0) {
            kp.x = __fmul_rn(kp.x, L.scale);
            kp.y = __fmul_rn(kp.y, L.scale);
        }
        kp.size = L.patch_size;
        kp.angle = angle;
        kp.response = (float)score;
        kp.octave = level;
        kp.class_id = -1;
        a.out_kps[(size_t)(a.first_slot + f) * a.nfeatures + k] = kp;
    }
}

// ---------------------------------------------------------------------------
// Host launcher
// ---------------------------------------------------------------------------
int launch_extract(orbx_ctx* ctx, int first, int count)
{
    const Geometry& g = ctx->geom;
    ExtractArgs a;
    a.levels = ctx->dgeom.levels;
    a.cells = ctx->dgeom.cells;
    a.res_cols = ctx->dgeom.res_cols;
    a.res_rows = ctx->dgeom.res_rows;
    a.umax = ctx->dgeom.umax;
    a.frames = ctx->frames;
    a.pyr_raw = ctx->pyr_raw;
    a.pyr_blur = ctx->pyr_blur;
    a.cell_lists = ctx->cell_lists;
    a.cell_count = ctx->cell_count;
    a.level_keys = ctx->level_keys;
    a.level_count = ctx->level_count;
    a.out_kps = ctx->out_kps;
    a.out_desc = ctx->out_desc;
    a.out_n = ctx->out_n;
    a.error_flags = ctx->error_flags;
    a.retain_scratch = ctx->retain_scratch;
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

    // One pass of the stage sequence over nb frames on stream st.
    auto run = [&](const ExtractArgs& x, int nb, hipStream_t st) {
        timer_begin(ctx, "pyr0", st);
        {
            const LevelGeom& L = g.levels[0];
            const int items = (L.stride / 4) * ((L.ph + kPyrRows - 1) / kPyrRows);
            hipLaunchKernelGGL(k_pyr_level0, dim3((items + 255) / 256, nb), dim3(256), 0, st, x);
        }
        timer_end(ctx, "pyr0", st);
        for (int l = 1; l < g.nlevels; l++) {
            const LevelGeom& L = g.levels[l];
            const int items = (L.stride / 4) * ((L.ph + kPyrRows - 1) / kPyrRows);
            timer_begin(ctx, "resize", st);
            hipLaunchKernelGGL(k_pyr_resize, dim3((items + 255) / 256, nb), dim3(256), 0, st, x, l);
            timer_end(ctx, "resize", st);
        }
        timer_begin(ctx, "fast", st);
        {
            const int pitch = (g.max_tile_bytes + 15) & ~15;
            hipLaunchKernelGGL(k_fast_cells, dim3((int)g.cells.size(), nb), dim3(256), 2 * pitch, st, x, pitch);
        }
        timer_end(ctx, "fast", st);
        timer_begin(ctx, "retain", st);
        {
            // wave-private LDS: cell list + partition scratch (longer lists
            // are replayed in global memory)
            const int cw = 2 * kRetainCellCap + 8;
            const int cwaves = 4;
            hipLaunchKernelGGL(k_retain_cells, dim3(((int)g.cells.size() + cwaves - 1) / cwaves, nb), dim3(64 * cwaves),
                               (size_t)cwaves * cw * 4, st, x, cwaves, cw);
            const int lw = 2 * g.max_level_cap + 8;
            const int lwaves = std::max(1, std::min(4, (int)(kRetainLds / (4 * (size_t)lw))));
            hipLaunchKernelGGL(k_retain_levels, dim3((g.nlevels + lwaves - 1) / lwaves, nb), dim3(64 * lwaves),
                               (size_t)lwaves * lw * 4, st, x, lwaves, lw);
        }
        timer_end(ctx, "retain", st);
        timer_begin(ctx, "blur", st);
        hipLaunchKernelGGL(k_blur, dim3(ctx->blur_tiles_n, nb), dim3(kBlurItems), 0, st, x, ctx->blur_tiles);
        timer_end(ctx, "blur", st);
        timer_begin(ctx, "describe", st);
        hipLaunchKernelGGL(k_describe, dim3((g.nfeatures + 2 * kWaves - 1) / (2 * kWaves), nb), dim3(256), 0, st, x);
        timer_end(ctx, "describe", st);
    };
    // Work buffers are indexed by batch position (frame f of a pass uses
    // work slot f); the frame store and outputs by slot.  Large batches run
    // as two halves on two streams so that the VALU-bound FAST pass of one
    // half overlaps the latency-bound passes of the other.
    a.first_slot = first;
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
        b.level_count += (size_t)n0 * a.nlevels;
        ORBX_HIP_CHECK(hipEventRecord(ctx->ev_fork, ctx->stream));
        ORBX_HIP_CHECK(hipStreamWaitEvent(ctx->stream2, ctx->ev_fork, 0));
        run(a, n0, ctx->stream);
        run(b, n1, ctx->stream2);
        ORBX_HIP_CHECK(hipEventRecord(ctx->ev_join, ctx->stream2));
        ORBX_HIP_CHECK(hipStreamWaitEvent(ctx->stream, ctx->ev_join, 0));
    } else {
        run(a, count, ctx->stream);
    }
    if (hipGetLastError() != hipSuccess) return ORBX_ERR_HIP;
    return ORBX_OK;
}

}  // namespace orbx
