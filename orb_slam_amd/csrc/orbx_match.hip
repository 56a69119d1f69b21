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

#ifdef ORBX_MATCH_PROFILE
extern "C" int orbx_debug_match_prof(unsigned long long* out)
{
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_match_prof), sizeof(unsigned long long) * 8) == hipSuccess ? 0 : -2;
}
#endif

int launch_match_bf_prev(orbx_ctx* ctx, int first, int count, int seq_len, int th_low, float nnratio,
                         hipStream_t st)
{
    if (!st) st = ctx->stream;
    const Geometry& g = ctx->geom;
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
    hipLaunchKernelGGL(k_match_bf_prev, dim3((g.nfeatures + 64 * kBfQ - 1) / (64 * kBfQ), count), dim3(64 * kBfWaves), 0,
                       st, a, th_low);
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
    // Frame::ComputeImageBounds without distortion (src/Frame.cc:341-347)
    a.min_x = 0.f;
    a.max_x = (float)g.w;
    a.min_y = 0.f;
    a.max_y = (float)g.h;
    a.gw_inv = static_cast<float>(kGridCols) / static_cast<float>(g.w - 0);
    a.gh_inv = static_cast<float>(kGridRows) / static_cast<float>(g.h - 0);
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
