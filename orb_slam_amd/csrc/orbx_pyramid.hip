// Fused image pyramid + GaussianBlur on MI355X (gfx950): the ComputePyramid
// stage of ORBextractor::operator() (src/ORBextractor.cc:781-822: level 0
// copyMakeBorder REFLECT_101 (:814), level l = resize INTER_LINEAR of level
// l-1 (:800) + copyMakeBorder (:806)) together with the per-level
// GaussianBlur(7x7, sigma 2, REFLECT_101) of :760, in one launch.
//
// One 1024-thread workgroup per frame streams the frame top to bottom in
// steps of T level-0 rows.  Every level keeps its most recent interior rows
// (as full padded rows) in an LDS ring; in step s
//   * level-0 load items write the T rows loaded during step s-1 (16-byte
//     words, REFLECT_101 columns by byte permutes) and load the next T;
//   * the resize jobs of level l >= 1 produce the rows whose two source rows
//     of level l-1 were in the ring by the end of step s-1;
//   * the blur jobs of level l blur the rows whose 7-row window was in the
//     ring by the end of step s-1 (a 7-row window of horizontal sums slides
//     down each dword column in registers across the whole frame);
// and one barrier ends the step.  Rows are written to HBM once when
// produced (raw interior row + its REFLECT_101 mirror rows in both buffers;
// blurred interior rows), so the frame is read from HBM once and each
// pyramid byte written once.  The host plan (plan_pyramid) computes, per
// level and step, the rows produced and blurred, the smallest ring that is
// never overwritten while read, and the wave -> job assignment.
//
// Arithmetic is that of the staged kernels (orbx_extract.hip): OpenCV 2.4
// resize 8U (SSE2 VResizeLinearVec_32s8u columns / scalar FixedPtCast tail)
// and the 8U separable blur (SymmColumnVec_32s8u float rounding / scalar
// FixedPtCastEx tail).  Integer byte work: HBM / VALU bound, no MFMA.
#include <algorithm>
#include <utility>
#include <cstdio>
#include <cstdlib>

#include "orbx_device.h"
#include "orbx_internal.h"

namespace orbx {

struct PyrArgs {
    const uint8_t* frames;
    uint8_t* pyr_raw;
    uint8_t* pyr_blur;
    const LevelGeom* levels;
    const PyrLevel* plv;
    const ResizeCol* res_cols;
    const ResizeRow* res_rows;
    const int32_t* sched;
    const PyrWave* waves;
    long long frame_pyr_bytes;
    int first_slot, w, h, nlevels, T, S, l0_items, nq16;
    int rows_first, rows_count, rows_lds, sched_lds, l0_fast;
};

#ifdef ORBX_PYR_PROFILE
// diagnostic build: per wave index, cycles (s_memtime) summed over the
// workgroups in setup / level-0 items / resize / blur / barrier wait
__device__ unsigned long long g_pyr_prof[kPyrWaves][5];
__device__ inline unsigned long long pp_stamp()
{
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
#define PP_T0() unsigned long long _pt = pp_stamp(), _pacc[5] = {0, 0, 0, 0, 0}
#define PP_MARK(k)                                 \
    do {                                           \
        const unsigned long long _n = pp_stamp();  \
        _pacc[k] += _n - _pt;                      \
        _pt = _n;                                  \
    } while (0)
#define PP_FLUSH()                                                                      \
    do {                                                                                \
        if (lane == 0)                                                                  \
            for (int k = 0; k < 5; k++) atomicAdd(&g_pyr_prof[wv][k], _pacc[k]);        \
    } while (0)
extern "C" int orbx_debug_pyr_prof(unsigned long long* out)
{
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pyr_prof), sizeof(g_pyr_prof)) == hipSuccess ? 0 : -2;
}
#else
#define PP_T0()
#define PP_MARK(k)
#define PP_FLUSH()
#endif

typedef unsigned short orbx_u16x2_t __attribute__((ext_vector_type(2)));

// wave-uniform copy of a level's ring description (scalar registers)
__device__ inline PyrLevel uniform_level(const PyrLevel& p)
{
    return PyrLevel{__builtin_amdgcn_readfirstlane(p.ring_off), __builtin_amdgcn_readfirstlane(p.ring),
                    __builtin_amdgcn_readfirstlane(p.rp), (uint32_t)__builtin_amdgcn_readfirstlane((int)p.mul)};
}

__device__ inline int ring_slot(int r, const PyrLevel& p)
{
    return r - p.ring * (int)(((uint32_t)r * p.mul) >> 20);
}

// Per-level values a job keeps: where its rows go in HBM and in the ring.
struct PyrLv {
    long long off;   // level offset in a frame's pyramid
    int stride, h;
};

// kL0Fast: w % 16 == 0 (level-0 words are aligned frame words or permutes
// of two); otherwise level-0 bytes are gathered one by one.
template <bool kL0Fast>
__global__ __launch_bounds__(kPyrThreads) void k_pyramid(PyrArgs a)
{
    extern __shared__ uint4 s_pyr[];
    uint8_t* lds = reinterpret_cast<uint8_t*>(s_pyr);
    const int f = blockIdx.x, tid = threadIdx.x;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const size_t fo = (size_t)f * a.frame_pyr_bytes;
    uint8_t* raw = a.pyr_raw + fo;
    uint8_t* blr = a.pyr_blur + fo;
    const uint8_t* src = a.frames + (size_t)(a.first_slot + f) * a.w * a.h;
    PP_T0();
    ResizeRow* s_rows = reinterpret_cast<ResizeRow*>(lds + a.rows_lds);
    int32_t* s_sched = reinterpret_cast<int32_t*>(lds + a.sched_lds);
    {   // stage the row tables and the schedule, independent loads in flight together
        const int nsched = a.S * a.nlevels;
        for (int i0 = 0; i0 < a.rows_count; i0 += 4 * kPyrThreads) {
            ResizeRow v[4];
#pragma unroll
            for (int k = 0; k < 4; k++) v[k] = a.res_rows[a.rows_first + min(i0 + k * kPyrThreads + tid, a.rows_count - 1)];
#pragma unroll
            for (int k = 0; k < 4; k++)
                if (i0 + k * kPyrThreads + tid < a.rows_count) s_rows[i0 + k * kPyrThreads + tid] = v[k];
        }
        for (int i0 = 0; i0 < nsched; i0 += 4 * kPyrThreads) {
            int32_t v[4];
#pragma unroll
            for (int k = 0; k < 4; k++) v[k] = a.sched[min(i0 + k * kPyrThreads + tid, nsched - 1)];
#pragma unroll
            for (int k = 0; k < 4; k++)
                if (i0 + k * kPyrThreads + tid < nsched) s_sched[i0 + k * kPyrThreads + tid] = v[k];
        }
    }
    const PyrWave W = a.waves[wv];
    const int nl = a.nlevels;

    // ---- level-0 load item: 16-byte column c0 of row k0 of every step ----
    const PyrLv L0{a.levels[0].off, a.levels[0].stride, a.h};
    const PyrLevel R0 = uniform_level(a.plv[0]);
    const int l0_item = W.l0_base >= 0 ? W.l0_base + lane : a.l0_items;
    const bool l0_on = l0_item < a.l0_items;
    const int k0 = l0_item / a.nq16, c0 = l0_item - k0 * a.nq16;
    const int w16 = a.w >> 4;
    // byte offsets of the two aligned source words of the item (fast path,
    // w % 16 == 0): interior words are one frame word, the two border words
    // are byte permutes of two
    const int oa = c0 == 0 ? 0 : (c0 <= w16 ? 16 * (c0 - 1) : a.w - 32);
    const int ob = c0 == 0 ? 16 : (c0 <= w16 ? 16 * (c0 - 1) : a.w - 16);
    uint4 pA = make_uint4(0, 0, 0, 0), pB = pA;
    auto l0_load = [&](int s) {
        const int r = min(a.T * s + k0, a.h - 1);
        const uint8_t* row = src + (size_t)r * a.w;
        pA = *reinterpret_cast<const uint4*>(row + oa);
        pB = *reinterpret_cast<const uint4*>(row + ob);
    };
    if (kL0Fast && l0_on) l0_load(0);

    // Row r of a level is stored to padded row kEdge + r, and to its
    // REFLECT_101 mirror rows (levels with h >= 17: rows 1..16 mirror above,
    // rows h-17..h-2 below) in both buffers.  Row bases are uniform; lanes
    // add a 32-bit byte offset.
    auto store_row = [&](const PyrLv& L, int r, uint32_t byte, auto v) {
        typedef decltype(v) V;
        uint8_t* rb = raw + (L.off + (long long)(kEdge + r) * L.stride);
        *reinterpret_cast<V*>(rb + byte) = v;
        if (r >= 1 && r <= kEdge) {
            const long long o = L.off + (long long)(kEdge - r) * L.stride;
            *reinterpret_cast<V*>(raw + o + byte) = v;
            *reinterpret_cast<V*>(blr + o + byte) = v;
        }
        if (r >= L.h - kEdge - 1 && r <= L.h - 2) {
            const long long o = L.off + (long long)(kEdge + 2 * L.h - 2 - r) * L.stride;
            *reinterpret_cast<V*>(raw + o + byte) = v;
            *reinterpret_cast<V*>(blr + o + byte) = v;
        }
    };

    // ---- resize job: dword column rq of level lr >= 1 ----
    // Per column: the byte offset of its first source pixel in the parent's
    // ring row (one unaligned ds_read_b32 fetches both taps) and the packed
    // 11-bit weights a0 | a1 << 16 for v_dot2_u32_u16 (zero off the row).
    const int lr = W.res_level;
    PyrLv Lr{0, 0, 0};
    PyrLevel Rr{}, Rp{};
    int rq = 0, rrow0 = 0;
    uint32_t roff[4] = {0, 0, 0, 0}, rw[4] = {0, 0, 0, 0};
    bool rvb[4] = {true, true, true, true}, rvec = true, r_on = false;
    if (lr >= 1) {
        const LevelGeom& G = a.levels[lr];
        Lr = PyrLv{G.off, G.stride, G.h};
        rrow0 = G.res_row_off - a.rows_first;
        Rr = uniform_level(a.plv[lr]);
        Rp = uniform_level(a.plv[lr - 1]);
        rq = W.res_q0 + lane;
        r_on = rq < (G.stride >> 2);
        const int pw = G.pw, lw = G.w, nvec = G.nvec_resize, col_off = G.res_col_off;
#pragma unroll
        for (int b = 0; b < 4; b++) {
            const bool on = 4 * rq + b < pw;
            const int x = on ? reflect101(4 * rq + b - kEdge, lw) : 0;
            const ResizeCol c = a.res_cols[col_off + x];
            roff[b] = (uint32_t)(kEdge + c.sx0);
            rw[b] = on ? ((uint32_t)(uint16_t)c.a0 | (uint32_t)(uint16_t)c.a1 << 16) : 0u;
            rvb[b] = x < nvec;
            rvec = rvec && (!on || rvb[b]);
        }
    }

    // ---- blur job: dword column bq of level lb ----
    // The 7-row window of horizontal sums lives in registers as 7 slots (row
    // y in slot y % 7, two float pairs), so the window never moves: the row
    // body is instantiated for the 7 phases.  Border columns keep the raw
    // centre word, re-read from the ring.
    const int lb = W.blur_level;
    PyrLv Lb{0, 0, 0};
    PyrLevel Rb{};
    int bq = 0, qm = 0, qc = 0, qp = 0;
    bool inside[4] = {false, false, false, false}, tail_col[4] = {false, false, false, false}, any_tail = false;
    bool b_on = false;
    uint32_t keep_mask = 0, in_mask = 0, out_mask = 0;   // bytes inside the row / blurred / kept raw
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 Wa[7], Wb[7];
#pragma unroll
    for (int k = 0; k < 7; k++) Wa[k] = Wb[k] = f2{0.f, 0.f};
    if (lb >= 0) {
        const LevelGeom& G = a.levels[lb];
        Lb = PyrLv{G.off, G.stride, G.h};
        Rb = uniform_level(a.plv[lb]);
        bq = W.blur_q0 + lane;
        b_on = bq < (G.stride >> 2);
        const int rpd = Rb.rp >> 2, lw = G.w, pw = G.pw, nvec = G.nvec_blur;
        qm = min(max(bq - 1, 0), rpd - 1);
        qc = min(bq, rpd - 1);
        qp = min(bq + 1, rpd - 1);
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int xi = 4 * bq + j - kEdge;
            inside[j] = xi >= 0 && xi < lw;
            tail_col[j] = inside[j] && xi >= nvec;
            any_tail = any_tail || tail_col[j];
            if (4 * bq + j < pw) keep_mask |= 0xFFu << (8 * j);
        }
#pragma unroll
        for (int j = 0; j < 4; j++)
            if (inside[j]) in_mask |= 0xFFu << (8 * j);
        out_mask = keep_mask & ~in_mask;
    }
    __syncthreads();
    PP_MARK(4);

    for (int s = 0; s < a.S; s++) {
        // -- level 0: the rows of step s (loaded during step s - 1) --
        if (l0_on) {
            const int r = a.T * s + k0;
            if (r < a.h) {
                uint4 v;
                if (kL0Fast) {
                    if (c0 == 0) {
                        v.x = __builtin_amdgcn_perm(pB.x, pA.w, 0x01020304u);
                        v.y = __builtin_amdgcn_perm(pA.w, pA.z, 0x01020304u);
                        v.z = __builtin_amdgcn_perm(pA.z, pA.y, 0x01020304u);
                        v.w = __builtin_amdgcn_perm(pA.y, pA.x, 0x01020304u);
                    } else if (c0 <= w16) {
                        v = pA;
                    } else if (c0 == w16 + 1) {
                        v.x = __builtin_amdgcn_perm(pB.w, pB.z, 0x03040506u);
                        v.y = __builtin_amdgcn_perm(pB.z, pB.y, 0x03040506u);
                        v.z = __builtin_amdgcn_perm(pB.y, pB.x, 0x03040506u);
                        v.w = __builtin_amdgcn_perm(pB.x, pA.w, 0x03040506u);
                    } else {
                        v = make_uint4(0, 0, 0, 0);
                    }
                } else {   // any width: byte gathers
                    const uint8_t* row = src + (size_t)r * a.w;
                    uint32_t o[4] = {0, 0, 0, 0};
#pragma unroll
                    for (int i = 0; i < 16; i++) {
                        const int px = 16 * c0 + i;
                        const uint32_t b = px < a.w + 2 * kEdge ? row[reflect101(px - kEdge, a.w)] : 0u;
                        o[i >> 2] |= b << (8 * (i & 3));
                    }
                    v = make_uint4(o[0], o[1], o[2], o[3]);
                }
                if (16 * c0 < R0.rp)
                    *reinterpret_cast<uint4*>(lds + R0.ring_off + ring_slot(r, R0) * R0.rp + 16 * c0) = v;
                store_row(L0, r, 16u * c0, v);
            }
            if (kL0Fast && s + 1 < a.S) l0_load(s + 1);
        }
        PP_MARK(0);
        // -- resize: rows of level lr whose sources were ready by step s - 1 --
        if (lr >= 1) {
            const int p0 = s > 0 ? s_sched[(s - 1) * nl + lr] & 0xFFFF : 0;
            const int p1 = s_sched[s * nl + lr] & 0xFFFF;
            const uint8_t* pring = lds + Rp.ring_off;
            // horizontal pass of source rows: S = p[sx0] a0 + p[sx0 + 1] a1;
            // the byte reads of every row are issued before the sums
            auto hrows = [&](auto... rows) {
                constexpr int n = sizeof...(rows);
                const int sy[n] = {rows.first...};
                uint32_t p0[n][4], p1[n][4];
#pragma unroll
                for (int i = 0; i < n; i++) {
                    const uint8_t* base = pring + ring_slot(sy[i], Rp) * Rp.rp;
#pragma unroll
                    for (int b = 0; b < 4; b++) {
                        p0[i][b] = base[roff[b]];
                        p1[i][b] = base[roff[b] + 1];
                    }
                }
                uint32_t* out[n] = {rows.second...};
#pragma unroll
                for (int i = 0; i < n; i++)
#pragma unroll
                    for (int b = 0; b < 4; b++)
                        out[i][b] = __builtin_amdgcn_udot2(__builtin_bit_cast(orbx_u16x2_t, p0[i][b] | p1[i][b] << 16),
                                                           __builtin_bit_cast(orbx_u16x2_t, rw[b]), 0u, false);
            };
            // the step's row-table entries, one per lane (rows step down by
            // 1.2, so a step produces far fewer than 64 rows)
            const int2 rrow = *reinterpret_cast<const int2*>(&s_rows[rrow0 + min(p0 + lane, max(p1 - 1, 0))]);
            // the previous row's second source row is this row's first one
            // whenever the rows step down by 1.2 (recomputed otherwise)
            uint32_t H1[4];
            int cy1 = -1;
            for (int r = p0; r < p1; r++) {
                const int ys = __builtin_amdgcn_readlane(rrow.x, r - p0);
                const int bs = __builtin_amdgcn_readlane(rrow.y, r - p0);
                const int sy0 = (int)(int16_t)(ys & 0xFFFF), sy1 = ys >> 16;
                const uint32_t b0 = (uint32_t)(bs & 0xFFFF), b1 = (uint32_t)bs >> 16;
                uint32_t A[4], B[4];
                if (sy0 == cy1) {
#pragma unroll
                    for (int b = 0; b < 4; b++) A[b] = H1[b];
                    if (sy1 == sy0) {
#pragma unroll
                        for (int b = 0; b < 4; b++) B[b] = A[b];
                    } else {
                        hrows(std::pair<int, uint32_t*>{sy1, B});
                    }
                } else if (sy1 == sy0) {
                    hrows(std::pair<int, uint32_t*>{sy0, A});
#pragma unroll
                    for (int b = 0; b < 4; b++) B[b] = A[b];
                } else {
                    hrows(std::pair<int, uint32_t*>{sy0, A}, std::pair<int, uint32_t*>{sy1, B});
                }
#pragma unroll
                for (int b = 0; b < 4; b++) H1[b] = B[b];
                cy1 = sy1;
                // VResizeLinearVec_32s8u (its 16-bit saturations cannot trigger
                // for 11-bit weights); products below 2^27 on 24-bit multiplies
                uint32_t word = 0;
#pragma unroll
                for (int b = 0; b < 4; b++) {
                    const uint32_t v = ((__umul24(A[b] >> 4, b0) >> 16) + (__umul24(B[b] >> 4, b1) >> 16) + 2) >> 2;
                    word |= min(v, 255u) << (8 * b);
                }
                if (!rvec) {   // the row's scalar tail: FixedPtCast<int, uchar, 22>
                    word = 0;
#pragma unroll
                    for (int b = 0; b < 4; b++) {
                        uint32_t v;
                        if (rvb[b])
                            v = ((__umul24(A[b] >> 4, b0) >> 16) + (__umul24(B[b] >> 4, b1) >> 16) + 2) >> 2;
                        else
                            v = (__umul24(A[b], b0) + __umul24(B[b], b1) + (1u << 21)) >> 22;
                        word |= min(v, 255u) << (8 * b);
                    }
                }
                if (r_on) {
                    if (4 * rq < Rr.rp)
                        *reinterpret_cast<uint32_t*>(lds + Rr.ring_off + ring_slot(r, Rr) * Rr.rp + 4 * rq) = word;
                    store_row(Lr, r, 4u * rq, word);
                }
            }
        }
        PP_MARK(1);
        // -- blur: rows of level lb whose 7-row window was ready by step s - 1 --
        if (lb >= 0) {
            const int e0 = s > 0 ? s_sched[(s - 1) * nl + lb] >> 16 : 0;
            const int e1 = s_sched[s * nl + lb] >> 16;
            const uint8_t* ring = lds + Rb.ring_off;
            const uint32_t boff = 4u * bq;
            // row y's horizontal sums and centre word into window slot K
#define ORBX_BLUR_LOAD(K, y)                                                                       \
    {                                                                                              \
        const uint32_t* row_ = reinterpret_cast<const uint32_t*>(ring + ring_slot((y), Rb) * Rb.rp); \
        int hs_[4];                                                                                \
        blur_hsum_w(row_[qm], row_[qc], row_[qp], hs_);                                            \
        Wa[K] = f2{(float)hs_[0], (float)hs_[1]};                                                  \
        Wb[K] = f2{(float)hs_[2], (float)hs_[3]};                                                  \
    }
            if (e0 == 0 && e1 > 0) {   // rows -3 .. 2 (reflected) into slots 4, 5, 6, 0, 1, 2
                ORBX_BLUR_LOAD(4, 3);
                ORBX_BLUR_LOAD(5, 2);
                ORBX_BLUR_LOAD(6, 1);
                ORBX_BLUR_LOAD(0, 0);
                ORBX_BLUR_LOAD(1, 1);
                ORBX_BLUR_LOAD(2, 2);
            }
            // one output row in phase K = r % 7: row r + 3 enters slot (K + 3) % 7
#define ORBX_BLUR_ROW(K)                                                                                      \
    {                                                                                                         \
        const int yn = r + 3 < Lb.h ? r + 3 : 2 * Lb.h - 5 - r;                                               \
        const uint32_t centre = reinterpret_cast<const uint32_t*>(ring + ring_slot(r, Rb) * Rb.rp)[qc];      \
        ORBX_BLUR_LOAD((K + 3) % 7, yn);                                                                      \
        constexpr float kInv = 1.0f / 65536.0f;                                                               \
        f2 Na = Wa[K] * 55.0f, Nb = Wb[K] * 55.0f;                                                            \
        Na = __builtin_elementwise_fma(Wa[(K + 6) % 7] + Wa[(K + 1) % 7], f2{49.0f, 49.0f}, Na);              \
        Nb = __builtin_elementwise_fma(Wb[(K + 6) % 7] + Wb[(K + 1) % 7], f2{49.0f, 49.0f}, Nb);              \
        Na = __builtin_elementwise_fma(Wa[(K + 5) % 7] + Wa[(K + 2) % 7], f2{34.0f, 34.0f}, Na);              \
        Nb = __builtin_elementwise_fma(Wb[(K + 5) % 7] + Wb[(K + 2) % 7], f2{34.0f, 34.0f}, Nb);              \
        Na = __builtin_elementwise_fma(Wa[(K + 4) % 7] + Wa[(K + 3) % 7], f2{18.0f, 18.0f}, Na);              \
        Nb = __builtin_elementwise_fma(Wb[(K + 4) % 7] + Wb[(K + 3) % 7], f2{18.0f, 18.0f}, Nb);              \
        const f2 sa = Na * kInv, sb = Nb * kInv;                                                              \
        float sv[4] = {sa.x, sa.y, sb.x, sb.y};                                                               \
        if (any_tail) {                                                                                       \
            const f2 ta = (Na + 32768.0f) * kInv, tb = (Nb + 32768.0f) * kInv;                                \
            const float tv[4] = {ta.x, ta.y, tb.x, tb.y};                                                     \
            _Pragma("unroll") for (int j = 0; j < 4; j++) if (tail_col[j]) sv[j] = floorf(tv[j]);             \
        }                                                                                                     \
        uint32_t word = 0;                                                                                    \
        _Pragma("unroll") for (int j = 0; j < 4; j++) word = __builtin_amdgcn_cvt_pk_u8_f32(sv[j], j, word);  \
        word = (word & in_mask) | (centre & out_mask);                                                        \
        if (b_on) *reinterpret_cast<uint32_t*>(blr + (Lb.off + (long long)(kEdge + r) * Lb.stride) + boff) = word; \
    }
            for (int r = e0; r < e1; r++) {
                switch (r % 7) {
                case 0: ORBX_BLUR_ROW(0); break;
                case 1: ORBX_BLUR_ROW(1); break;
                case 2: ORBX_BLUR_ROW(2); break;
                case 3: ORBX_BLUR_ROW(3); break;
                case 4: ORBX_BLUR_ROW(4); break;
                case 5: ORBX_BLUR_ROW(5); break;
                default: ORBX_BLUR_ROW(6); break;
                }
            }
#undef ORBX_BLUR_ROW
#undef ORBX_BLUR_LOAD
        }
        PP_MARK(2);
        __syncthreads();
        PP_MARK(3);
    }
    PP_FLUSH();
}

// ---------------------------------------------------------------------------
// Host plan
// ---------------------------------------------------------------------------
void plan_pyramid(const Geometry& g, int T, PyrPlan& p)
{
    p = PyrPlan{};
    const int nl = g.nlevels;
    if (nl < 1 || T < 1) return;
    for (int l = 0; l < nl; l++)   // single REFLECT_101 mirror rows/columns
        if (g.levels[l].h <= kEdge || g.levels[l].w <= kEdge) return;
    auto rrow = [&](int l, int r) { return g.res_rows[g.levels[l].res_row_off + r]; };
    // rows produced (P) / blurred (B) by the end of each step
    std::vector<std::vector<int>> P(nl), B(nl);
    for (int s = 0;; s++) {
        bool done = true;
        for (int l = 0; l < nl; l++) {
            const LevelGeom& L = g.levels[l];
            int pr = s > 0 ? P[l][s - 1] : 0;
            if (l == 0) {
                pr = std::min(T * (s + 1), L.h);
            } else {
                const int src = s > 0 ? P[l - 1][s - 1] : 0;
                while (pr < L.h && std::max(rrow(l, pr).sy0, rrow(l, pr).sy1) < src) pr++;
            }
            int bl = s > 0 ? B[l][s - 1] : 0;
            const int have = s > 0 ? P[l][s - 1] : 0;
            while (bl < L.h && std::min(bl + 4, L.h) <= have) bl++;
            P[l].push_back(pr);
            B[l].push_back(bl);
            done = done && bl == L.h;
        }
        if (done) {
            p.S = s + 1;
            break;
        }
        if (s > 8 * 4096) return;
    }
    const int S = p.S;
    for (int l = 0; l < nl; l++)   // the resize reads a step's row-table entries one per lane
        for (int s = 0; s < S; s++)
            if (P[l][s] - (s > 0 ? P[l][s - 1] : 0) > 64) return;
    // ring rows: every row read in step s must survive the rows written up to
    // the end of step s (reads see rows of earlier steps only)
    p.levels.assign(nl, PyrLevel{});
    int off = 0;
    for (int l = 0; l < nl; l++) {
        const LevelGeom& L = g.levels[l];
        int need = 1;
        for (int s = 0; s < S; s++) {
            int lo = 1 << 30;
            const int b0 = s > 0 ? B[l][s - 1] : 0, b1 = B[l][s];
            if (b1 > b0) {
                if (b0 == 0)
                    for (int k = 0; k < 6; k++) lo = std::min(lo, reflect101(k - 3, L.h));
                for (int r = b0; r < b1; r++) lo = std::min(lo, std::min(r, reflect101(r + 3, L.h)));
            }
            if (l + 1 < nl) {
                const int p0 = s > 0 ? P[l + 1][s - 1] : 0, p1 = P[l + 1][s];
                for (int r = p0; r < p1; r++) lo = std::min(lo, (int)std::min(rrow(l + 1, r).sy0, rrow(l + 1, r).sy1));
            }
            if (lo < (1 << 30)) need = std::max(need, P[l][s] - lo);
        }
        PyrLevel& q = p.levels[l];
        q.ring = need;
        q.rp = (L.pw + 15) & ~15;
        q.mul = (uint32_t)(((1u << 20) + need - 1) / need);
        for (int r = 0; r < L.h; r++)
            if (r - need * (int)(((uint32_t)r * q.mul) >> 20) != r % need) return;
        q.ring_off = off;
        off += need * q.rp;
    }
    p.rows_first = nl > 1 ? g.levels[1].res_row_off : 0;
    p.rows_count = nl > 1 ? g.levels[nl - 1].res_row_off + g.levels[nl - 1].h - p.rows_first : 0;
    p.rows_lds = off;
    off += ((p.rows_count * (int)sizeof(ResizeRow)) + 15) & ~15;
    p.sched_lds = off;
    off += S * nl * 4;
    p.lds_bytes = off;
    if (p.lds_bytes > 160 * 1024) return;
    p.sched.resize((size_t)S * nl);
    for (int s = 0; s < S; s++)
        for (int l = 0; l < nl; l++) p.sched[(size_t)s * nl + l] = P[l][s] | (B[l][s] << 16);
    // jobs, costed by the rows each processes over the frame; greedy onto the
    // waves (at most one job of each kind per wave)
    p.T = T;
    p.nq16 = g.levels[0].stride / 16;
    p.l0_items = T * p.nq16;
    struct Job {
        int kind, level, q0;
        double cost;
    };
    std::vector<Job> jobs;
    for (int l = 0; l < nl; l++) {
        const int nq = g.levels[l].stride / 4;
        for (int q0 = 0; q0 < nq; q0 += 64) {
            jobs.push_back(Job{0, l, q0, 1.0 * g.levels[l].h});
            if (l >= 1) jobs.push_back(Job{1, l, q0, 0.35 * g.levels[l].h});
        }
    }
    for (int i0 = 0; i0 < p.l0_items; i0 += 64) jobs.push_back(Job{2, 0, i0, 0.2 * g.levels[0].h});
    std::stable_sort(jobs.begin(), jobs.end(), [](const Job& x, const Job& y) { return x.cost > y.cost; });
    double load[kPyrWaves] = {};
    for (int wv = 0; wv < kPyrWaves; wv++) p.waves[wv] = PyrWave{-1, 0, -1, 0, -1, 0};
    for (const Job& j : jobs) {
        int best = -1;
        for (int wv = 0; wv < kPyrWaves; wv++) {
            const PyrWave& W = p.waves[wv];
            const bool free = j.kind == 0 ? W.blur_level < 0 : j.kind == 1 ? W.res_level < 0 : W.l0_base < 0;
            if (free && (best < 0 || load[wv] < load[best])) best = wv;
        }
        if (best < 0) return;   // more jobs than waves
        PyrWave& W = p.waves[best];
        if (j.kind == 0) {
            W.blur_level = (int16_t)j.level;
            W.blur_q0 = (int16_t)j.q0;
        } else if (j.kind == 1) {
            W.res_level = (int16_t)j.level;
            W.res_q0 = (int16_t)j.q0;
        } else {
            W.l0_base = (int16_t)j.q0;
        }
        load[best] += j.cost;
    }
    p.ok = true;
}

template <typename T>
static int ensure_dev(T*& ptr, size_t count)
{
    if (ptr) (void)hipFree(ptr);
    ptr = nullptr;
    return hipMalloc(reinterpret_cast<void**>(&ptr), std::max<size_t>(count, 1) * sizeof(T)) == hipSuccess ? ORBX_OK
                                                                                                          : ORBX_ERR_NOMEM;
}

int upload_pyramid_plan(orbx_ctx* ctx)
{
    constexpr int T = 8;   // level-0 rows per step (4 / 8 / 16 measured equal)
    plan_pyramid(ctx->geom, T, ctx->pyr);
    const PyrPlan& p = ctx->pyr;
    if (!p.ok) return ORBX_OK;
    int r;
    if (!ctx->d_pyr_levels && (r = ensure_dev(ctx->d_pyr_levels, kMaxLevels)) != ORBX_OK) return r;
    if (!ctx->d_pyr_waves && (r = ensure_dev(ctx->d_pyr_waves, kPyrWaves)) != ORBX_OK) return r;
    if ((int)p.sched.size() > ctx->cap_pyr_sched) {
        if ((r = ensure_dev(ctx->d_pyr_sched, p.sched.size())) != ORBX_OK) return r;
        ctx->cap_pyr_sched = (int)p.sched.size();
    }
    ORBX_HIP_CHECK(hipMemcpy(ctx->d_pyr_levels, p.levels.data(), p.levels.size() * sizeof(PyrLevel), hipMemcpyHostToDevice));
    ORBX_HIP_CHECK(hipMemcpy(ctx->d_pyr_waves, p.waves, sizeof(p.waves), hipMemcpyHostToDevice));
    ORBX_HIP_CHECK(hipMemcpy(ctx->d_pyr_sched, p.sched.data(), p.sched.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    return ORBX_OK;
}

bool ensure_pyramid_plan(orbx_ctx* ctx)
{
    if (!ctx->pyr_planned) {
        ctx->pyr_planned = true;
        // a failed upload only disables the optional fused path
        if (upload_pyramid_plan(ctx) != ORBX_OK) ctx->pyr.ok = false;
    }
    return ctx->pyr.ok;
}

int launch_pyramid(orbx_ctx* ctx, int first_slot, uint8_t* pyr_raw, uint8_t* pyr_blur, int nb, hipStream_t st)
{
    const Geometry& g = ctx->geom;
    const PyrPlan& p = ctx->pyr;
    PyrArgs a;
    a.frames = ctx->frames_src ? ctx->frames_src : ctx->frames;
    a.pyr_raw = pyr_raw;
    a.pyr_blur = pyr_blur;
    a.levels = ctx->dgeom.levels;
    a.plv = ctx->d_pyr_levels;
    a.res_cols = ctx->dgeom.res_cols;
    a.res_rows = ctx->dgeom.res_rows;
    a.sched = ctx->d_pyr_sched;
    a.waves = ctx->d_pyr_waves;
    a.frame_pyr_bytes = g.frame_pyr_bytes;
    a.first_slot = first_slot;
    a.w = g.w;
    a.h = g.h;
    a.nlevels = g.nlevels;
    a.T = p.T;
    a.S = p.S;
    a.l0_items = p.l0_items;
    a.nq16 = p.nq16;
    a.rows_first = p.rows_first;
    a.rows_count = p.rows_count;
    a.rows_lds = p.rows_lds;
    a.sched_lds = p.sched_lds;
    a.l0_fast = (g.w % 16 == 0 && g.w >= 32) ? 1 : 0;
    if (a.l0_fast)
        hipLaunchKernelGGL(k_pyramid<true>, dim3(nb), dim3(kPyrThreads), p.lds_bytes, st, a);
    else
        hipLaunchKernelGGL(k_pyramid<false>, dim3(nb), dim3(kPyrThreads), p.lds_bytes, st, a);
    return ORBX_OK;
}

}  // namespace orbx
