// ORB matching on MI355X: the ORBmatcher searches on the per-frame hot path.
//
// The reference matchers are sequential greedy loops (each accepted match
// changes the state the next query sees: vMatchedDistance / vnMatches21 in
// SearchForInitialization, F.mvpMapPoints in the projection searches).  The
// GPU form keeps that order exactly: ONE wave owns one frame pair, walks the
// queries in reference order, and evaluates each query's candidate window
// with all 64 lanes (Hamming distance = popcount of XOR, 8 x 32-bit per
// descriptor), reducing best / second-best with wave shuffles.  Ties resolve
// to the first candidate in GetFeaturesInArea order (cell x, cell y, index:
// src/Frame.cc:232-257), as the reference's strict `<` does.
#include <algorithm>

#include "orbx_match_common.h"

namespace orbx {

struct MatchPrevArgs {
    const orbx_keypoint* kps;
    const uint8_t* desc;
    const int32_t* nkp;
    int32_t* match12;
    int32_t* match_n;
    int nfeatures;
    int first, seq_len, window;
    float nnratio;
    int check_ori;
    int cap_c, cap_keys;
    int32_t* error_flags;
    float min_x, max_x, min_y, max_y, gw_inv, gh_inv;
};

// One 256-thread block per frame pair: slot s vs its predecessor in a
// cyclic sequence of seq_len slots.
__global__ __launch_bounds__(256) void k_match_prev(MatchPrevArgs a)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    __shared__ BlockScratch bs;
    const int s = a.first + blockIdx.x;
    const int prev = (s % a.seq_len == 0) ? s + a.seq_len - 1 : s - 1;
    FrameDev F1, F2;
    F1.kps = a.kps + (size_t)prev * a.nfeatures;
    F1.desc = a.desc + (size_t)prev * a.nfeatures * 32;
    F1.n = a.nkp[prev];
    F2.kps = a.kps + (size_t)s * a.nfeatures;
    F2.desc = a.desc + (size_t)s * a.nfeatures * 32;
    F2.n = a.nkp[s];
    F1.min_x = F2.min_x = a.min_x;
    F1.max_x = F2.max_x = a.max_x;
    F1.min_y = F2.min_y = a.min_y;
    F1.max_y = F2.max_y = a.max_y;
    F1.grid_w_inv = F2.grid_w_inv = a.gw_inv;
    F1.grid_h_inv = F2.grid_h_inv = a.gh_inv;
    const InitLDS L = carve_init(smem, a.cap_c, a.nfeatures, a.cap_keys);
    search_for_init_block(F1, F2, nullptr, a.window, a.nnratio, a.check_ori != 0,
                          a.match12 + (size_t)s * a.nfeatures, a.match_n + s, nullptr, L, bs, a.error_flags);
}

// Brute-force matching of slot s against its predecessor (config C3): for
// each keypoint a of the previous frame, the first index of the smallest
// Hamming distance over all keypoints of frame s and the second smallest
// value; accept best <= th_low && best < nnratio * second (the B3 rule of
// src/ORBmatcher.cc:640-654 applied to all pairs).  grid = (query blocks of
// 256, pairs); candidates stream through LDS 512 descriptors at a time, each
// of the 8 waves scanning its own 64 for 4 queries per lane.
constexpr int kBfWaves = 8;   // candidate splits (k_match_bf_prev)
constexpr int kBfQ = 4;       // queries per lane

__global__ __launch_bounds__(64 * kBfWaves) void k_match_bf_prev(MatchPrevArgs a, int th_low)
{
    // 64 kBfQ queries per workgroup, kBfQ per lane (one LDS read of a
    // candidate serves kBfQ distances: the broadcast ds_read_b128 pair per
    // candidate, not the VALU, bounded the one-query-per-lane form); wave w
    // scans the candidates [64 w, 64 w + 64) of every LDS chunk (an
    // increasing subset, first strict minimum kept), then the waves'
    // (best, index, second) merge in wave order: the two smallest values of
    // the union are the two smallest of the waves' pairs, and an equal best
    // keeps the lower index, as the one sequential scan does
    constexpr int kT = 64 * kBfWaves, kQB = 64 * kBfQ;
    __shared__ uint4 sb[kT][2];
    __shared__ uint32_t mk1[kBfWaves][kQB], mk2[kBfWaves][kQB];
    const int s = a.first + blockIdx.y;
    const int prev = (s % a.seq_len == 0) ? s + a.seq_len - 1 : s - 1;
    const int nA = a.nkp[prev], nB = a.nkp[s];
    const uint8_t* dA = a.desc + (size_t)prev * a.nfeatures * 32;
    const uint8_t* dB = a.desc + (size_t)s * a.nfeatures * 32;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int q0 = blockIdx.x * kQB;
    if (q0 >= nA) return;   // block-uniform
    uint4 qa[kBfQ], qb[kBfQ];
    uint32_t kb1[kBfQ], kb2[kBfQ];
#pragma unroll
    for (int u = 0; u < kBfQ; u++) {
        const int q = q0 + 64 * u + lane;
        qa[u] = qb[u] = make_uint4(0, 0, 0, 0);
        if (q < nA) load_desc(dA + (size_t)q * 32, qa[u], qb[u]);
        kb1[u] = kb2[u] = 0xFFFFFFFFu;
    }
    for (int base = 0; base < nB; base += kT) {
        __syncthreads();
        const int j = base + threadIdx.x;
        if (j < nB) load_desc(dB + (size_t)j * 32, sb[threadIdx.x][0], sb[threadIdx.x][1]);
        __syncthreads();
        const int k0 = 64 * wv, k1 = min(k0 + 64, nB - base);   // wave-uniform
        for (int k = k0; k < k1; k++) {
            const uint4 c0 = sb[k][0], c1 = sb[k][1];
            const uint32_t idx = (uint32_t)(base + k);
#pragma unroll
            for (int u = 0; u < kBfQ; u++) {
                // (distance << 16 | index) keys: the best is the smallest key
                // (first index of the smallest distance), the second
                // smallest distance of the multiset is min(second, max(best,
                // this)) taken on keys (equal distances differ in the index
                // only)
                const uint32_t key = ((uint32_t)hamming256(qa[u], qb[u], c0, c1) << 16) | idx;
                kb2[u] = min(kb2[u], max(kb1[u], key));
                kb1[u] = min(kb1[u], key);
            }
        }
    }
#pragma unroll
    for (int u = 0; u < kBfQ; u++) {
        mk1[wv][64 * u + lane] = kb1[u];
        mk2[wv][64 * u + lane] = kb2[u];
    }
    __syncthreads();
    // merge: thread t < kQB finalises query q0 + t
    int ok = 0;
    const int t = threadIdx.x;
    if (t < kQB) {
        uint32_t r1 = mk1[0][t], r2 = mk2[0][t];
#pragma unroll
        for (int w = 1; w < kBfWaves; w++) {
            const uint32_t c1 = mk1[w][t], c2 = mk2[w][t];
            r2 = min(min(r2, c2), max(r1, c1));
            r1 = min(r1, c1);
        }
        const int q = q0 + t;
        if (q < nA) {
            // no candidate: key ~0 (distance 0xFFFF, never accepted)
            const int d1 = (int)(r1 >> 16), d2 = r2 == 0xFFFFFFFFu ? 0x7fffffff : (int)(r2 >> 16);
            ok = (d1 <= th_low && (float)d1 < __fmul_rn((float)d2, a.nnratio));
            a.match12[(size_t)s * a.nfeatures + q] = ok ? (int)(r1 & 0xFFFF) : -1;
        }
    }
    ok = wave_sum(ok);
    if (lane == 0 && ok) atomicAdd(a.match_n + s, ok);
}

// The same brute-force rule on the i8 matrix cores.  popc(a ^ b) =
// popc(a) + popc(b) - 2 a.b with the 256 descriptor bits as 0/1 bytes, so a
// 32x32 block of distances is eight v_mfma_i32_32x32x32_i8 over the bit
// planes (exact integer sums).  Queries sit on the A rows (bits expanded
// once into registers), candidates on the B columns (expanded per
// 128-candidate chunk into LDS, rows padded to 272 B; the next chunk's dwords
// load into registers while the current one is scored).  Any k order serves
// as long as A and B share it: 16-bit group 2t + h of a descriptor is k-step t of lane
// half h, bit j its byte j.  For a fixed query popc(a) is a constant, so
// the per-lane key is C_col - (a.b << 17) with C_col = (popc(b) + 256) << 16
// | index: one multiply-add per distance, ordered as (distance, index); an
// absent candidate has C_col = ~0 and zero bits (key ~0, never chosen).
constexpr int kBfmWaves = 8;                  // query tiles of 32 per workgroup
constexpr int kBfmQ = 32 * kBfmWaves;
constexpr int kBfmChunk = 128;                // candidates per LDS chunk
constexpr int kBfmPitch = 17;                 // uint4 per expanded candidate row

using orbx_i8x16 = __attribute__((ext_vector_type(16))) signed char;
using orbx_i32x16 = __attribute__((ext_vector_type(16))) int;

__device__ inline uint32_t nibble_bytes(uint32_t nib)   // bit j of nib -> byte j (0/1)
{
    return (nib * 0x00204081u) & 0x01010101u;
}

__device__ inline uint4 expand_bits16(uint32_t g)
{
    return make_uint4(nibble_bytes(g & 15u), nibble_bytes((g >> 4) & 15u), nibble_bytes((g >> 8) & 15u),
                      nibble_bytes((g >> 12) & 15u));
}

__device__ inline int popc_desc(const uint4& x, const uint4& y)
{
    return __popc(x.x) + __popc(x.y) + __popc(x.z) + __popc(x.w) + __popc(y.x) + __popc(y.y) + __popc(y.z) +
           __popc(y.w);
}

__global__ __launch_bounds__(64 * kBfmWaves) void k_match_bf_prev_mfma(MatchPrevArgs a, int th_low)
{
    __shared__ uint4 bx[kBfmChunk][kBfmPitch];
    __shared__ uint32_t cval[kBfmChunk];
    __shared__ uint32_t fk1[kBfmQ], fk2[kBfmQ];
    const int s = a.first + blockIdx.y;
    const int prev = (s % a.seq_len == 0) ? s + a.seq_len - 1 : s - 1;
    const int nA = a.nkp[prev], nB = a.nkp[s];
    const uint8_t* dA = a.desc + (size_t)prev * a.nfeatures * 32;
    const uint8_t* dB = a.desc + (size_t)s * a.nfeatures * 32;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, r = lane & 31, h = lane >> 5;
    const int q0 = blockIdx.x * kBfmQ;
    if (q0 >= nA) return;   // block-uniform
    // A fragments of query q0 + 32 wv + r: k-step t holds 16-bit group 2t + h
    orbx_i8x16 af[8];
    {
        const int q = q0 + 32 * wv + r;
        uint4 x = make_uint4(0, 0, 0, 0), y = make_uint4(0, 0, 0, 0);
        if (q < nA) load_desc(dA + (size_t)q * 32, x, y);
        const uint32_t w[8] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
#pragma unroll
        for (int t = 0; t < 8; t++) af[t] = __builtin_bit_cast(orbx_i8x16, expand_bits16(w[t] >> (16 * h) & 0xFFFFu));
    }
    uint32_t k1[16], k2[16];
#pragma unroll
    for (int i = 0; i < 16; i++) k1[i] = k2[i] = 0xFFFFFFFFu;
    // candidate dwords of a chunk: thread tid holds dword i = tid + kT m
    // (candidate i >> 3, word i & 7), loaded one chunk ahead
    constexpr int kT = 64 * kBfmWaves, kPer = kBfmChunk * 8 / kT;
    const uint32_t* dB32 = reinterpret_cast<const uint32_t*>(dB);
    uint32_t raw[kPer];
    auto fetch = [&](int base) {
#pragma unroll
        for (int m = 0; m < kPer; m++) {
            const int i = tid + kT * m, j = base + (i >> 3);
            raw[m] = j < nB ? dB32[(size_t)j * 8 + (i & 7)] : 0u;
        }
    };
    fetch(0);
    for (int base = 0; base < nB; base += kBfmChunk) {
        __syncthreads();   // previous chunk consumed
#pragma unroll
        for (int m = 0; m < kPer; m++) {
            const int i = tid + kT * m, c = i >> 3, w = i & 7, j = base + c;
            bx[c][2 * w] = expand_bits16(raw[m] & 0xFFFFu);
            bx[c][2 * w + 1] = expand_bits16(raw[m] >> 16);
            // popc of the candidate over its 8 consecutive lanes
            int p = __popc(raw[m]);
            p += __shfl_xor(p, 1);
            p += __shfl_xor(p, 2);
            p += __shfl_xor(p, 4);
            if (w == 0) cval[c] = j < nB ? ((uint32_t)(p + 256) << 16) | (uint32_t)j : 0xFFFFFFFFu;
        }
        __syncthreads();
        if (base + kBfmChunk < nB) fetch(base + kBfmChunk);   // block-uniform; lands during the tiles
        const int ntiles = min(kBfmChunk / 32, (nB - base + 31) >> 5);   // block-uniform
        for (int tile = 0; tile < ntiles; tile++) {
            orbx_i32x16 acc = {};
            const uint4* brow = bx[32 * tile + r];
#pragma unroll
            for (int t = 0; t < 8; t++)
                acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[t], __builtin_bit_cast(orbx_i8x16, brow[2 * t + h]), acc,
                                                            0, 0, 0);
            // D[row][col]: col = lane & 31 (candidate), row = (i & 3) + 8 (i >> 2) + 4 h (query)
            const uint32_t C = cval[32 * tile + r];
#pragma unroll
            for (int i = 0; i < 16; i++) {
                const uint32_t key = C - ((uint32_t)acc[i] << 17);
                k2[i] = min(k2[i], max(k1[i], key));
                k1[i] = min(k1[i], key);
            }
        }
    }
    // merge the 32 columns of each lane half (keys are unique: order-free)
#pragma unroll
    for (int off = 1; off < 32; off <<= 1) {
#pragma unroll
        for (int i = 0; i < 16; i++) {
            const uint32_t c1 = (uint32_t)__shfl_xor((int)k1[i], off), c2 = (uint32_t)__shfl_xor((int)k2[i], off);
            k2[i] = min(min(k2[i], c2), max(k1[i], c1));
            k1[i] = min(k1[i], c1);
        }
    }
    if (r == 0) {
#pragma unroll
        for (int i = 0; i < 16; i++) {
            const int row = (i & 3) + 8 * (i >> 2) + 4 * h;
            fk1[32 * wv + row] = k1[i];
            fk2[32 * wv + row] = k2[i];
        }
    }
    __syncthreads();
    int ok = 0;
    const int q = q0 + tid;
    if (tid < kBfmQ && q < nA) {
        uint4 x, y;
        load_desc(dA + (size_t)q * 32, x, y);
        const int pa = popc_desc(x, y) - 256;
        const uint32_t r1 = fk1[tid], r2 = fk2[tid];
        const int d1 = r1 == 0xFFFFFFFFu ? 0x7fffffff : (int)(r1 >> 16) + pa;
        const int d2 = r2 == 0xFFFFFFFFu ? 0x7fffffff : (int)(r2 >> 16) + pa;
        ok = (d1 <= th_low && (float)d1 < __fmul_rn((float)d2, a.nnratio));
        a.match12[(size_t)s * a.nfeatures + q] = ok ? (int)(r1 & 0xFFFF) : -1;
    }
    ok = wave_sum(ok);
    if (lane == 0 && ok) atomicAdd(a.match_n + s, ok);
}

#ifdef ORBX_MATCH_PROFILE
extern "C" int orbx_debug_match_prof(unsigned long long* out)
{
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_match_prof), sizeof(unsigned long long) * 8) == hipSuccess ? 0 : -2;
}
#endif

// Both brute-force kernels pack the candidate index into the low 16 bits of
// their (distance, index) keys.
static_assert(kMaxFeatures <= 0xFFFF, "brute-force keys hold the candidate index in 16 bits");

int launch_match_bf_prev(orbx_ctx* ctx, int first, int count, int seq_len, int th_low, float nnratio,
                         hipStream_t st)
{
    if (!st) st = ctx->stream;
    const Geometry& g = ctx->geom;
    if (g.nfeatures > 0xFFFF) return ORBX_ERR_UNSUPPORTED;   // the 16-bit index field of the keys
    MatchPrevArgs a{};
    a.kps = ctx->out_kps;
    a.desc = ctx->out_desc;
    a.nkp = ctx->out_n;
    a.match12 = ctx->match12;
    a.match_n = ctx->match_n;
    a.nfeatures = g.nfeatures;
    a.first = first;
    a.seq_len = seq_len;
    a.nnratio = nnratio;
    ORBX_HIP_CHECK(hipMemsetAsync(ctx->match_n + first, 0, sizeof(int32_t) * count, st));
    timer_begin(ctx, "match", st);
#ifdef ORBX_BF_VALU   // A/B builds only: the VALU popcount form
    hipLaunchKernelGGL(k_match_bf_prev, dim3((g.nfeatures + 64 * kBfQ - 1) / (64 * kBfQ), count), dim3(64 * kBfWaves), 0,
                       st, a, th_low);
#else
    hipLaunchKernelGGL(k_match_bf_prev_mfma, dim3((g.nfeatures + kBfmQ - 1) / kBfmQ, count), dim3(64 * kBfmWaves), 0,
                       st, a, th_low);
#endif
    timer_end(ctx, "match", st);
    if (hipGetLastError() != hipSuccess) return ORBX_ERR_HIP;
    return ORBX_OK;
}

int launch_match_prev(orbx_ctx* ctx, int first, int count, int seq_len, int window, float nnratio,
                      int check_ori, hipStream_t st)
{
    if (!st) st = ctx->stream;
    const Geometry& g = ctx->geom;
    MatchPrevArgs a;
    a.kps = ctx->out_kps;
    a.desc = ctx->out_desc;
    a.nkp = ctx->out_n;
    a.match12 = ctx->match12;
    a.match_n = ctx->match_n;
    a.nfeatures = g.nfeatures;
    a.first = first;
    a.seq_len = seq_len;
    a.window = window;
    a.nnratio = nnratio;
    a.check_ori = check_ori;
    // Frame::ComputeImageBounds (src/Frame.cc:320-348): the context's bounds
    // of undistorted keypoints (orbx_dev_set_image_bounds), else the image
    // (:341-347); the grid cell scales of src/Frame.cc:76-77
    a.min_x = ctx->has_bounds ? ctx->bounds[0] : 0.f;
    a.max_x = ctx->has_bounds ? ctx->bounds[1] : (float)g.w;
    a.min_y = ctx->has_bounds ? ctx->bounds[2] : 0.f;
    a.max_y = ctx->has_bounds ? ctx->bounds[3] : (float)g.h;
    a.gw_inv = static_cast<float>(kGridCols) / (a.max_x - a.min_x);
    a.gh_inv = static_cast<float>(kGridRows) / (a.max_y - a.min_y);
    // candidates = keypoints of octave 0, at most the level-0 quota
    a.cap_c = std::min(g.levels[0].n_desired, g.nfeatures);
    if (a.cap_c > kInitMaxCand) return ORBX_ERR_UNSUPPORTED;
    a.error_flags = ctx->error_flags;
    const size_t fixed = init_lds_bytes(a.cap_c, g.nfeatures, 0);
    a.cap_keys = std::max<int>(a.cap_c, (int)((kInitLdsBudget - std::min(fixed, kInitLdsBudget)) / 4));
    const size_t lds = init_lds_bytes(a.cap_c, g.nfeatures, a.cap_keys);
    timer_begin(ctx, "match", st);
    hipLaunchKernelGGL(k_match_prev, dim3(count), dim3(256), lds, st, a);
    timer_end(ctx, "match", st);
    if (hipGetLastError() != hipSuccess) return ORBX_ERR_HIP;
    return ORBX_OK;
}

}  // namespace orbx
