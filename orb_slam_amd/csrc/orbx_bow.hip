// Vocabulary-node searches of ORBmatcher on MI355X: SearchByBoW(KF, F)
// (src/ORBmatcher.cc:155-283), SearchByBoW(KF1, KF2) (:715-850) and
// SearchForTriangulation (:852-1014).
//
// The reference walks the DBoW2 FeatureVector nodes both frames share and,
// inside a node, replays a greedy loop over the first frame's features: each
// takes its best still-unmatched candidate of the same node in the second
// frame.  A feature belongs to one node only, so nodes are independent: one
// workgroup per call, its four wavefronts take the common nodes round-robin.
// Inside a node the wavefront replays the greedy loop in order with the
// node's second-frame features spread over the lanes (lane j owns list
// entries j, j + 64, ...; their "already matched" flags are a register
// bitmask): each step is one Hamming distance per lane and one DPP
// best/second reduction (SearchForTriangulation: a min-distance reduction,
// then the first (distance, index) candidate passing the epipolar test).
// The rotation histogram (ComputeThreeMaxima, :1748-1789) is built after all
// nodes with LDS atomics and filtered in parallel.
#include <algorithm>
#include <vector>

#include "orbx_device.h"
#include "orbx_internal.h"
#include "orbx_match_common.h"

namespace orbx {

constexpr int kBowMaxChunks = 32;   // second-frame features per node <= 64 * 32

struct BowSideDev {
    const orbx_keypoint* kps;
    const uint8_t* desc;
    const uint8_t* mp;
    const int32_t* feat;
};

struct BowArgs {
    BowSideDev s1, s2;
    const int4* nodes;      // (first1, count1, first2, count2) per common node
    int n_common;
    int mode;               // 0 SearchByBoW(KF, F), 1 SearchByBoW(KF1, KF2), 2 SearchForTriangulation
    float nnratio;
    int check_ori;
    float F12[9];
    float sigma2[kMaxLevels];
    int32_t* out;           // mode 0: [F.n] (KF index); modes 1, 2: [KF1.n] (KF2 index)
    int out_len;
    signed char* bins;      // rotation bin per out entry, -1 when none
    int32_t* out_n;
};

// ORBmatcher::CheckDistEpipolarLine (src/ORBmatcher.cc:136-153): float line
// coefficients summed left to right, threshold 3.84 * sigma2 in double.
__device__ inline bool epipolar_ok(const orbx_keypoint& k1, const orbx_keypoint& k2, const float* F,
                                   const float* sigma2)
{
    const float a = __fadd_rn(__fadd_rn(__fmul_rn(k1.x, F[0]), __fmul_rn(k1.y, F[3])), F[6]);
    const float b = __fadd_rn(__fadd_rn(__fmul_rn(k1.x, F[1]), __fmul_rn(k1.y, F[4])), F[7]);
    const float c = __fadd_rn(__fadd_rn(__fmul_rn(k1.x, F[2]), __fmul_rn(k1.y, F[5])), F[8]);
    const float num = __fadd_rn(__fadd_rn(__fmul_rn(a, k2.x), __fmul_rn(b, k2.y)), c);
    const float den = __fadd_rn(__fmul_rn(a, a), __fmul_rn(b, b));
    if (den == 0.0f) return false;
    const float dsqr = __fdiv_rn(__fmul_rn(num, num), den);
    return (double)dsqr < 3.84 * (double)sigma2[k2.octave];
}

__device__ void bow_match_block(const BowArgs& a)
{
    __shared__ int hist[kHistoLength];
    __shared__ int s_acc, s_removed, s_ind[3];
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
    if (tid < kHistoLength) hist[tid] = 0;
    if (tid == 0) {
        s_acc = 0;
        s_removed = 0;
    }
    __syncthreads();
    int accepted = 0;
    for (int k = wv; k < a.n_common; k += kBlock / 64) {
        const int4 nd = a.nodes[k];
        const int nch = (nd.w + 63) >> 6;
        uint32_t taken = 0;   // bit c: list entry lane + 64 c already matched
        for (int i = 0; i < nd.y; i++) {
            const int idx1 = a.s1.feat[nd.x + i];
            const int m1 = a.s1.mp[idx1];
            if (a.mode == 2 ? m1 != 0 : m1 != 1) continue;   // uniform
            uint4 d1a, d1b;
            load_desc(a.s1.desc + (size_t)idx1 * 32, d1a, d1b);
            int best_j;
            if (a.mode < 2) {
                // best (first strict minimum in list order) and second distance
                uint32_t m1k = 0xFFFFFFFFu;
                int m2d = 511;
                for (int c = 0; c < nch; c++) {
                    const int j = c * 64 + lane;
                    if (j >= nd.w || ((taken >> c) & 1)) continue;
                    const int idx2 = a.s2.feat[nd.z + j];
                    if (a.mode == 1 && a.s2.mp[idx2] != 1) continue;
                    uint4 b0, b1;
                    load_desc(a.s2.desc + (size_t)idx2 * 32, b0, b1);
                    const int dist = hamming256(d1a, d1b, b0, b1);
                    const uint32_t key = ((uint32_t)dist << 23) | (uint32_t)j;
                    if (key < m1k) {
                        m2d = min(m2d, (int)(m1k >> 23));
                        m1k = key;
                    } else {
                        m2d = min(m2d, dist);
                    }
                }
                best_second_reduce(m1k, m2d);
                if (m1k == 0xFFFFFFFFu) continue;
                const int d1 = (int)(m1k >> 23);
                const float second = m2d >= 511 ? 2147483648.0f : (float)m2d;   // (float)INT_MAX
                const bool ok = (a.mode == 0 ? d1 <= kTHLow : d1 < kTHLow) && (float)d1 < __fmul_rn(a.nnratio, second);
                if (!ok) continue;
                best_j = (int)(m1k & 0x7FFFFF);
            } else {
                // vDistIndex: candidates with dist <= TH_LOW sorted by
                // (dist, index); the first within 2 * best passing the
                // epipolar test wins
                int bd = 0x7fffffff;
                for (int c = 0; c < nch; c++) {
                    const int j = c * 64 + lane;
                    if (j >= nd.w || ((taken >> c) & 1)) continue;
                    const int idx2 = a.s2.feat[nd.z + j];
                    if (a.s2.mp[idx2] != 0) continue;
                    uint4 b0, b1;
                    load_desc(a.s2.desc + (size_t)idx2 * 32, b0, b1);
                    const int dist = hamming256(d1a, d1b, b0, b1);
                    if (dist <= kTHLow) bd = min(bd, dist);
                }
                bd = wave_min_i32(bd);
                if (bd > kTHLow) continue;
                const int th = 2 * bd;   // round(2*BestDist)
                const orbx_keypoint kp1 = a.s1.kps[idx1];
                unsigned long long kb = ~0ull;
                for (int c = 0; c < nch; c++) {
                    const int j = c * 64 + lane;
                    if (j >= nd.w || ((taken >> c) & 1)) continue;
                    const int idx2 = a.s2.feat[nd.z + j];
                    if (a.s2.mp[idx2] != 0) continue;
                    uint4 b0, b1;
                    load_desc(a.s2.desc + (size_t)idx2 * 32, b0, b1);
                    const int dist = hamming256(d1a, d1b, b0, b1);
                    if (dist > kTHLow || dist > th) continue;
                    if (!epipolar_ok(kp1, a.s2.kps[idx2], a.F12, a.sigma2)) continue;
                    const unsigned long long key = ((unsigned long long)dist << 48) |
                                                   ((unsigned long long)(uint32_t)idx2 << 16) | (unsigned long long)j;
                    kb = key < kb ? key : kb;
                }
                kb = wave_min_u64(kb);
                if (kb == ~0ull) continue;
                best_j = (int)(kb & 0xFFFF);
            }
            if ((best_j & 63) == lane) taken |= 1u << (best_j >> 6);
            if (lane == 0) {
                const int idx2 = a.s2.feat[nd.z + best_j];
                const int slot = a.mode == 0 ? idx2 : idx1;
                a.out[slot] = a.mode == 0 ? idx1 : idx2;
                if (a.check_ori) a.bins[slot] = (signed char)rot_bin(a.s1.kps[idx1].angle, a.s2.kps[idx2].angle);
            }
            accepted++;
        }
    }
    if (lane == 0 && accepted) atomicAdd(&s_acc, accepted);
    __syncthreads();
    if (a.check_ori) {
        for (int i = tid; i < a.out_len; i += kBlock) {
            const int b = a.bins[i];
            if (b >= 0) atomicAdd(&hist[b], 1);
        }
        __syncthreads();
        if (tid == 0) three_maxima(hist, s_ind[0], s_ind[1], s_ind[2]);
        __syncthreads();
        int rem = 0;
        for (int i = tid; i < a.out_len; i += kBlock) {
            const int b = a.bins[i];
            if (b >= 0 && b != s_ind[0] && b != s_ind[1] && b != s_ind[2]) {
                a.out[i] = -1;
                rem++;
            }
        }
        rem = wave_sum(rem);
        if (lane == 0 && rem) atomicAdd(&s_removed, rem);
        __syncthreads();
    }
    if (tid == 0) *a.out_n = s_acc - s_removed;
}

__global__ __launch_bounds__(256) void k_bow_match(BowArgs a) { bow_match_block(a); }

// One workgroup per job (one keyframe pair each).
__global__ __launch_bounds__(256) void k_bow_match_jobs(const BowArgs* jobs) { bow_match_block(jobs[blockIdx.x]); }

// SearchByBoW(KF, F) against a device-resident frame (orbx_dev_search_by_bow),
// and the keyframe-pair searches between device-resident frames
// (orbx_dev_search_by_bow_kf, orbx_dev_search_for_triangulation): the
// slots' FeatureVectors come from k_bow_build, so the common nodes are found
// here.  Each KF node binary-searches F's ascending node ids; hits are
// compacted in KF node order (the reference's merge order), then the job
// runs as bow_match_block.
struct BowSlotJob {
    BowArgs a;                 // s1 = KF, s2 = the slot; nodes / n_common / out_len filled here
    const uint32_t* kf_node_id;
    const int32_t* kf_node_ptr;
    int kf_n_nodes;
    const int32_t* kf_counts;  // side 1 a slot too: its (n_words, n_fv_nodes), else null
    const uint32_t* f_node_id;
    const int32_t* f_node_ptr;
    const int32_t* f_counts;   // (n_words, n_fv_nodes)
    const int32_t* out_count;  // feature count of the side the output is indexed by
    int nf;
    int4* nodes;               // [side-1 nodes] scratch
};

__global__ __launch_bounds__(256) void k_bow_match_slot(const BowSlotJob* jobs)
{
    __shared__ BlockScratch bs;
    __shared__ int s_bad;
    const BowSlotJob& j = jobs[blockIdx.x];
    const int tid = threadIdx.x, nfv = j.f_counts[1], nkf = j.kf_counts ? j.kf_counts[1] : j.kf_n_nodes;
    if (tid == 0) s_bad = 0;
    const int per = (nkf + kBlock - 1) / kBlock, k0 = tid * per, k1 = min(k0 + per, nkf);
    auto find = [&](uint32_t id) {
        int lo = 0, hi = nfv;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (j.f_node_id[mid] < id) lo = mid + 1;
            else hi = mid;
        }
        return lo < nfv && j.f_node_id[lo] == id ? lo : -1;
    };
    int hits = 0;
    for (int k = k0; k < k1; k++) hits += find(j.kf_node_id[k]) >= 0;
    int total;
    int at = block_exclusive_scan(hits, &total, bs, 0);
    for (int k = k0; k < k1; k++) {
        const int f = find(j.kf_node_id[k]);
        if (f < 0) continue;
        const int c2 = j.f_node_ptr[f + 1] - j.f_node_ptr[f];
        if (c2 > 64 * kBowMaxChunks) s_bad = 1;
        j.nodes[at++] = make_int4(j.kf_node_ptr[k], j.kf_node_ptr[k + 1] - j.kf_node_ptr[k], j.f_node_ptr[f], c2);
    }
    __threadfence_block();
    __syncthreads();
    if (s_bad) {
        if (tid == 0) *j.a.out_n = -1;   // a node wider than the taken-mask covers: ORBX_ERR_UNSUPPORTED
        return;
    }
    BowArgs a = j.a;
    a.nodes = j.nodes;
    a.n_common = total;
    a.out_len = min(*j.out_count, j.nf);
    bow_match_block(a);
}

namespace {

bool valid_bow(const orbx_bow_view* v, int max_octave)
{
    if (!v || v->n < 0 || v->n_nodes < 0) return false;
    if (v->n > 0 && (!v->keys || !v->desc || !v->mp)) return false;
    if (v->n_nodes == 0) return true;
    if (!v->node_id || !v->node_ptr || !v->feat_idx || v->node_ptr[0] < 0) return false;
    std::vector<uint8_t> seen(v->n, 0);
    for (int k = 0; k < v->n_nodes; k++) {
        if (v->node_ptr[k + 1] < v->node_ptr[k]) return false;
        if (k > 0 && v->node_id[k] <= v->node_id[k - 1]) return false;
        for (int e = v->node_ptr[k]; e < v->node_ptr[k + 1]; e++) {
            const int f = v->feat_idx[e];
            if (f < 0 || f >= v->n || seen[f]) return false;
            seen[f] = 1;
        }
    }
    if (max_octave > 0)
        for (int i = 0; i < v->n; i++)
            if (v->keys[i].octave < 0 || v->keys[i].octave >= max_octave) return false;
    return true;
}

// The common node ids in ascending order (the reference's merge loop).
std::vector<int4> common_nodes(const orbx_bow_view& a, const orbx_bow_view& b)
{
    std::vector<int4> out;
    int i = 0, j = 0;
    while (i < a.n_nodes && j < b.n_nodes) {
        if (a.node_id[i] == b.node_id[j]) {
            out.push_back(make_int4(a.node_ptr[i], a.node_ptr[i + 1] - a.node_ptr[i], b.node_ptr[j],
                                    b.node_ptr[j + 1] - b.node_ptr[j]));
            i++;
            j++;
        } else if (a.node_id[i] < b.node_id[j]) {
            i = (int)(std::lower_bound(a.node_id + i, a.node_id + a.n_nodes, b.node_id[j]) - a.node_id);
        } else {
            j = (int)(std::lower_bound(b.node_id + j, b.node_id + b.n_nodes, a.node_id[i]) - b.node_id);
        }
    }
    return out;
}

inline size_t al256(size_t b) { return (b + 255) & ~size_t(255); }

int run_bow(orbx_ctx* ctx, const orbx_bow_view* V1, const orbx_bow_view* V2, int mode, float nnratio, int check_ori,
            const float* F12, const float* sigma2, int nlevels, int32_t* out, int* n_out)
{
    if (!ctx || !out || !n_out) return ORBX_ERR_ARG;
    if (mode == 2 && (!F12 || !sigma2 || nlevels <= 0 || nlevels > kMaxLevels)) return ORBX_ERR_ARG;
    if (!valid_bow(V1, 0) || !valid_bow(V2, mode == 2 ? nlevels : 0)) return ORBX_ERR_ARG;
    const std::vector<int4> nodes = common_nodes(*V1, *V2);
    for (const int4& nd : nodes)
        if (nd.w > 64 * kBowMaxChunks) return ORBX_ERR_UNSUPPORTED;
    const int out_len = mode == 0 ? V2->n : V1->n;
    ctx_enter(ctx);
    const int nf1 = V1->n_nodes ? V1->node_ptr[V1->n_nodes] : 0, nf2 = V2->n_nodes ? V2->node_ptr[V2->n_nodes] : 0;
    // layout in the context scratch
    size_t at = 0;
    auto res = [&](size_t bytes) {
        const size_t o = at;
        at += al256(std::max<size_t>(bytes, 1));
        return o;
    };
    const size_t o_k1 = res((size_t)V1->n * sizeof(orbx_keypoint)), o_d1 = res((size_t)V1->n * 32),
                 o_m1 = res(V1->n), o_f1 = res((size_t)nf1 * 4);
    const size_t o_k2 = res((size_t)V2->n * sizeof(orbx_keypoint)), o_d2 = res((size_t)V2->n * 32),
                 o_m2 = res(V2->n), o_f2 = res((size_t)nf2 * 4);
    const size_t o_nd = res(nodes.size() * sizeof(int4)), o_out = res((size_t)out_len * 4), o_bin = res(out_len),
                 o_n = res(4);
    int r = ensure_scratch(ctx, at);
    if (r != ORBX_OK) return r;
    uint8_t* d = static_cast<uint8_t*>(ctx->scratch);
    auto put = [&](size_t off, const void* src, size_t bytes) -> int {
        if (bytes == 0 || !src) return ORBX_OK;
        ORBX_HIP_CHECK(hipMemcpyAsync(d + off, src, bytes, hipMemcpyHostToDevice, ctx->stream));
        return ORBX_OK;
    };
    if ((r = put(o_k1, V1->keys, (size_t)V1->n * sizeof(orbx_keypoint))) ||
        (r = put(o_d1, V1->desc, (size_t)V1->n * 32)) || (r = put(o_m1, V1->mp, V1->n)) ||
        (r = put(o_f1, V1->n_nodes ? V1->feat_idx : nullptr, (size_t)nf1 * 4)) ||
        (r = put(o_k2, V2->keys, (size_t)V2->n * sizeof(orbx_keypoint))) ||
        (r = put(o_d2, V2->desc, (size_t)V2->n * 32)) || (r = put(o_m2, V2->mp, V2->n)) ||
        (r = put(o_f2, V2->n_nodes ? V2->feat_idx : nullptr, (size_t)nf2 * 4)) ||
        (r = put(o_nd, nodes.data(), nodes.size() * sizeof(int4))))
        return r;
    ORBX_HIP_CHECK(hipMemsetAsync(d + o_out, 0xFF, (size_t)out_len * 4, ctx->stream));
    ORBX_HIP_CHECK(hipMemsetAsync(d + o_bin, 0xFF, (size_t)out_len, ctx->stream));
    BowArgs a{};
    a.s1 = {reinterpret_cast<const orbx_keypoint*>(d + o_k1), d + o_d1, d + o_m1,
            reinterpret_cast<const int32_t*>(d + o_f1)};
    a.s2 = {reinterpret_cast<const orbx_keypoint*>(d + o_k2), d + o_d2, d + o_m2,
            reinterpret_cast<const int32_t*>(d + o_f2)};
    a.nodes = reinterpret_cast<const int4*>(d + o_nd);
    a.n_common = (int)nodes.size();
    a.mode = mode;
    a.nnratio = nnratio;
    a.check_ori = check_ori;
    if (mode == 2) {
        for (int k = 0; k < 9; k++) a.F12[k] = F12[k];
        for (int l = 0; l < nlevels; l++) a.sigma2[l] = sigma2[l];
    }
    a.out = reinterpret_cast<int32_t*>(d + o_out);
    a.out_len = out_len;
    a.bins = reinterpret_cast<signed char*>(d + o_bin);
    a.out_n = reinterpret_cast<int32_t*>(d + o_n);
    hipLaunchKernelGGL(k_bow_match, dim3(1), dim3(kBlock), 0, ctx->stream, a);
    ORBX_HIP_CHECK(hipGetLastError());
    if (out_len) ORBX_HIP_CHECK(hipMemcpyAsync(out, d + o_out, (size_t)out_len * 4, hipMemcpyDeviceToHost, ctx->stream));
    ORBX_HIP_CHECK(hipMemcpyAsync(n_out, d + o_n, 4, hipMemcpyDeviceToHost, ctx->stream));
    ORBX_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    return ORBX_OK;
}

// One keyframe against n others (modes 1, 2): KF1 uploaded once, each pair's
// common nodes, one launch of n workgroups, one readback.
int run_bow_batch(orbx_ctx* ctx, const orbx_bow_view* V1, int n, const orbx_bow_view* V2s, int mode, float nnratio,
                  int check_ori, const float* F12s, const float* sigma2s, int nlevels, int32_t* const* outs,
                  int* n_outs)
{
    if (!ctx || n < 0 || (n > 0 && (!V2s || !outs || !n_outs))) return ORBX_ERR_ARG;
    if (mode == 2 && n > 0 && (!F12s || !sigma2s || nlevels <= 0 || nlevels > kMaxLevels)) return ORBX_ERR_ARG;
    if (!valid_bow(V1, 0)) return ORBX_ERR_ARG;
    for (int k = 0; k < n; k++)
        if (!valid_bow(&V2s[k], mode == 2 ? nlevels : 0) || (V1->n > 0 && !outs[k])) return ORBX_ERR_ARG;
    if (n == 0) return ORBX_OK;
    std::vector<std::vector<int4>> nodes(n);
    for (int k = 0; k < n; k++) {
        nodes[k] = common_nodes(*V1, V2s[k]);
        for (const int4& nd : nodes[k])
            if (nd.w > 64 * kBowMaxChunks) return ORBX_ERR_UNSUPPORTED;
    }
    ctx_enter(ctx);
    const int out_len = V1->n;
    size_t at = 0;
    auto res = [&](size_t bytes) {
        const size_t o = at;
        at += al256(std::max<size_t>(bytes, 1));
        return o;
    };
    const int nf1 = V1->n_nodes ? V1->node_ptr[V1->n_nodes] : 0;
    const size_t o_k1 = res((size_t)V1->n * sizeof(orbx_keypoint)), o_d1 = res((size_t)V1->n * 32),
                 o_m1 = res(V1->n), o_f1 = res((size_t)nf1 * 4);
    struct Off {
        size_t k2, d2, m2, f2, nd, out, bin, n;
    };
    std::vector<Off> o(n);
    for (int k = 0; k < n; k++) {
        const orbx_bow_view& V2 = V2s[k];
        const int nf2 = V2.n_nodes ? V2.node_ptr[V2.n_nodes] : 0;
        o[k].k2 = res((size_t)V2.n * sizeof(orbx_keypoint));
        o[k].d2 = res((size_t)V2.n * 32);
        o[k].m2 = res(V2.n);
        o[k].f2 = res((size_t)nf2 * 4);
        o[k].nd = res(nodes[k].size() * sizeof(int4));
        o[k].out = res((size_t)out_len * 4);
        o[k].bin = res(out_len);
        o[k].n = res(4);
    }
    const size_t o_jobs = res(sizeof(BowArgs) * (size_t)n);
    int r = ensure_scratch(ctx, at);
    if (r != ORBX_OK) return r;
    uint8_t* d = static_cast<uint8_t*>(ctx->scratch);
    auto put = [&](size_t off, const void* src, size_t bytes) -> int {
        if (bytes == 0 || !src) return ORBX_OK;
        ORBX_HIP_CHECK(hipMemcpyAsync(d + off, src, bytes, hipMemcpyHostToDevice, ctx->stream));
        return ORBX_OK;
    };
    if ((r = put(o_k1, V1->keys, (size_t)V1->n * sizeof(orbx_keypoint))) ||
        (r = put(o_d1, V1->desc, (size_t)V1->n * 32)) || (r = put(o_m1, V1->mp, V1->n)) ||
        (r = put(o_f1, V1->n_nodes ? V1->feat_idx : nullptr, (size_t)nf1 * 4)))
        return r;
    std::vector<BowArgs> jobs(n);
    for (int k = 0; k < n; k++) {
        const orbx_bow_view& V2 = V2s[k];
        const int nf2 = V2.n_nodes ? V2.node_ptr[V2.n_nodes] : 0;
        if ((r = put(o[k].k2, V2.keys, (size_t)V2.n * sizeof(orbx_keypoint))) ||
            (r = put(o[k].d2, V2.desc, (size_t)V2.n * 32)) || (r = put(o[k].m2, V2.mp, V2.n)) ||
            (r = put(o[k].f2, V2.n_nodes ? V2.feat_idx : nullptr, (size_t)nf2 * 4)) ||
            (r = put(o[k].nd, nodes[k].data(), nodes[k].size() * sizeof(int4))))
            return r;
        ORBX_HIP_CHECK(hipMemsetAsync(d + o[k].out, 0xFF, (size_t)out_len * 4, ctx->stream));
        ORBX_HIP_CHECK(hipMemsetAsync(d + o[k].bin, 0xFF, (size_t)out_len, ctx->stream));
        BowArgs& a = jobs[k];
        a = BowArgs{};
        a.s1 = {reinterpret_cast<const orbx_keypoint*>(d + o_k1), d + o_d1, d + o_m1,
                reinterpret_cast<const int32_t*>(d + o_f1)};
        a.s2 = {reinterpret_cast<const orbx_keypoint*>(d + o[k].k2), d + o[k].d2, d + o[k].m2,
                reinterpret_cast<const int32_t*>(d + o[k].f2)};
        a.nodes = reinterpret_cast<const int4*>(d + o[k].nd);
        a.n_common = (int)nodes[k].size();
        a.mode = mode;
        a.nnratio = nnratio;
        a.check_ori = check_ori;
        if (mode == 2) {
            for (int c = 0; c < 9; c++) a.F12[c] = F12s[9 * k + c];
            for (int l = 0; l < nlevels; l++) a.sigma2[l] = sigma2s[(size_t)nlevels * k + l];
        }
        a.out = reinterpret_cast<int32_t*>(d + o[k].out);
        a.out_len = out_len;
        a.bins = reinterpret_cast<signed char*>(d + o[k].bin);
        a.out_n = reinterpret_cast<int32_t*>(d + o[k].n);
    }
    if ((r = put(o_jobs, jobs.data(), sizeof(BowArgs) * (size_t)n))) return r;
    hipLaunchKernelGGL(k_bow_match_jobs, dim3(n), dim3(kBlock), 0, ctx->stream,
                       reinterpret_cast<const BowArgs*>(d + o_jobs));
    ORBX_HIP_CHECK(hipGetLastError());
    for (int k = 0; k < n; k++) {
        if (out_len)
            ORBX_HIP_CHECK(hipMemcpyAsync(outs[k], d + o[k].out, (size_t)out_len * 4, hipMemcpyDeviceToHost, ctx->stream));
        ORBX_HIP_CHECK(hipMemcpyAsync(&n_outs[k], d + o[k].n, 4, hipMemcpyDeviceToHost, ctx->stream));
    }
    ORBX_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    return ORBX_OK;
}

}  // namespace
}  // namespace orbx

using namespace orbx;

extern "C" int orbx_search_by_bow_frame(orbx_ctx* ctx, const orbx_bow_view* KF, const orbx_bow_view* F,
                                        float nnratio, int check_ori, int32_t* matches_f, int* n_matches)
{
    return run_bow(ctx, KF, F, 0, nnratio, check_ori, nullptr, nullptr, 0, matches_f, n_matches);
}

extern "C" int orbx_search_by_bow_kf(orbx_ctx* ctx, const orbx_bow_view* KF1, const orbx_bow_view* KF2,
                                     float nnratio, int check_ori, int32_t* matches12, int* n_matches)
{
    return run_bow(ctx, KF1, KF2, 1, nnratio, check_ori, nullptr, nullptr, 0, matches12, n_matches);
}

extern "C" int orbx_search_for_triangulation(orbx_ctx* ctx, const orbx_bow_view* KF1, const orbx_bow_view* KF2,
                                             const float* F12, const float* sigma2_2, int nlevels, int check_ori,
                                             int32_t* matches12, int* n_matches)
{
    return run_bow(ctx, KF1, KF2, 2, 0.f, check_ori, F12, sigma2_2, nlevels, matches12, n_matches);
}

extern "C" int orbx_search_by_bow_kf_batch(orbx_ctx* ctx, const orbx_bow_view* KF1, int n, const orbx_bow_view* KF2s,
                                           float nnratio, int check_ori, int32_t* const* matches12, int* n_matches)
{
    return run_bow_batch(ctx, KF1, n, KF2s, 1, nnratio, check_ori, nullptr, nullptr, 0, matches12, n_matches);
}

extern "C" int orbx_search_for_triangulation_batch(orbx_ctx* ctx, const orbx_bow_view* KF1, int n,
                                                   const orbx_bow_view* KF2s, const float* F12s,
                                                   const float* sigma2_2s, int nlevels, int check_ori,
                                                   int32_t* const* matches12, int* n_matches)
{
    return run_bow_batch(ctx, KF1, n, KF2s, 2, 0.f, check_ori, F12s, sigma2_2s, nlevels, matches12, n_matches);
}

// Tracking::Relocalisation's loop (src/Tracking.cc:904-925): SearchByBoW(KF,
// F) of each candidate keyframe against the extracted frame in `slot`, whose
// BoW orbx_dev_compute_bow left in HBM.  One upload of the n keyframes, one
// launch of n workgroups, one readback.
extern "C" int orbx_dev_search_by_bow(orbx_ctx* ctx, int slot, int n, const orbx_bow_view* KFs, float nnratio,
                                      int check_ori, int32_t* const* matches_f, int cap, int* n_matches)
{
    if (!ctx || slot < 0 || slot >= ctx->slots || n < 0 || (n > 0 && (!KFs || !matches_f || !n_matches)))
        return ORBX_ERR_ARG;
    if (!ctx->bow_dev || slot >= (int)ctx->bow_ready.size() || !ctx->bow_ready[slot]) return ORBX_ERR_ARG;
    const int nf = ctx->bow_nf;
    if (n > 0 && cap < nf) return ORBX_ERR_CAPACITY;
    for (int k = 0; k < n; k++)
        if (!valid_bow(&KFs[k], 0) || !matches_f[k]) return ORBX_ERR_ARG;
    if (n == 0) return ORBX_OK;
    ctx_enter(ctx);
    size_t at = 0;
    auto res = [&](size_t bytes) {
        const size_t o = at;
        at += al256(std::max<size_t>(bytes, 1));
        return o;
    };
    struct Off {
        size_t k1, d1, m1, f1, nid, nptr, nd, out, bin, n;
    };
    std::vector<Off> o(n);
    for (int k = 0; k < n; k++) {
        const orbx_bow_view& V = KFs[k];
        const int nf1 = V.n_nodes ? V.node_ptr[V.n_nodes] : 0;
        o[k].k1 = res((size_t)V.n * sizeof(orbx_keypoint));
        o[k].d1 = res((size_t)V.n * 32);
        o[k].m1 = res(V.n);
        o[k].f1 = res((size_t)nf1 * 4);
        o[k].nid = res((size_t)V.n_nodes * 4);
        o[k].nptr = res((size_t)(V.n_nodes + 1) * 4);
        o[k].nd = res((size_t)V.n_nodes * sizeof(int4));
        o[k].out = res((size_t)nf * 4);
        o[k].bin = res(nf);
        o[k].n = res(4);
    }
    const size_t o_jobs = res(sizeof(BowSlotJob) * (size_t)n);
    int r = ensure_scratch(ctx, at);
    if (r != ORBX_OK) return r;
    uint8_t* d = static_cast<uint8_t*>(ctx->scratch);
    auto put = [&](size_t off, const void* src, size_t bytes) -> int {
        if (bytes == 0 || !src) return ORBX_OK;
        ORBX_HIP_CHECK(hipMemcpyAsync(d + off, src, bytes, hipMemcpyHostToDevice, ctx->stream));
        return ORBX_OK;
    };
    const SlotBowDev& b = ctx->bow;
    std::vector<BowSlotJob> jobs(n);
    for (int k = 0; k < n; k++) {
        const orbx_bow_view& V = KFs[k];
        const int nf1 = V.n_nodes ? V.node_ptr[V.n_nodes] : 0;
        if ((r = put(o[k].k1, V.keys, (size_t)V.n * sizeof(orbx_keypoint))) ||
            (r = put(o[k].d1, V.desc, (size_t)V.n * 32)) || (r = put(o[k].m1, V.mp, V.n)) ||
            (r = put(o[k].f1, V.n_nodes ? V.feat_idx : nullptr, (size_t)nf1 * 4)) ||
            (r = put(o[k].nid, V.n_nodes ? V.node_id : nullptr, (size_t)V.n_nodes * 4)) ||
            (r = put(o[k].nptr, V.n_nodes ? V.node_ptr : nullptr, (size_t)(V.n_nodes + 1) * 4)))
            return r;
        ORBX_HIP_CHECK(hipMemsetAsync(d + o[k].out, 0xFF, (size_t)nf * 4, ctx->stream));
        ORBX_HIP_CHECK(hipMemsetAsync(d + o[k].bin, 0xFF, (size_t)nf, ctx->stream));
        BowSlotJob& j = jobs[k];
        j = BowSlotJob{};
        BowArgs& a = j.a;
        a.s1 = {reinterpret_cast<const orbx_keypoint*>(d + o[k].k1), d + o[k].d1, d + o[k].m1,
                reinterpret_cast<const int32_t*>(d + o[k].f1)};
        a.s2 = {ctx->out_kps + (size_t)slot * nf, ctx->out_desc + (size_t)slot * nf * 32, nullptr,
                b.fv_feat + (size_t)slot * nf};
        a.mode = 0;
        a.nnratio = nnratio;
        a.check_ori = check_ori;
        a.out = reinterpret_cast<int32_t*>(d + o[k].out);
        a.bins = reinterpret_cast<signed char*>(d + o[k].bin);
        a.out_n = reinterpret_cast<int32_t*>(d + o[k].n);
        j.kf_node_id = reinterpret_cast<const uint32_t*>(d + o[k].nid);
        j.kf_node_ptr = reinterpret_cast<const int32_t*>(d + o[k].nptr);
        j.kf_n_nodes = V.n_nodes;
        j.f_node_id = b.fv_nodes + (size_t)slot * nf;
        j.f_node_ptr = b.fv_ptr + (size_t)slot * (nf + 1);
        j.f_counts = b.counts + 2 * slot;
        j.out_count = ctx->out_n + slot;
        j.nf = nf;
        j.nodes = reinterpret_cast<int4*>(d + o[k].nd);
    }
    if ((r = put(o_jobs, jobs.data(), sizeof(BowSlotJob) * (size_t)n))) return r;
    timer_begin(ctx, "bow_match_slot");
    hipLaunchKernelGGL(k_bow_match_slot, dim3(n), dim3(kBlock), 0, ctx->stream,
                       reinterpret_cast<const BowSlotJob*>(d + o_jobs));
    timer_end(ctx, "bow_match_slot");
    ORBX_HIP_CHECK(hipGetLastError());
    for (int k = 0; k < n; k++) {
        ORBX_HIP_CHECK(hipMemcpyAsync(matches_f[k], d + o[k].out, (size_t)nf * 4, hipMemcpyDeviceToHost, ctx->stream));
        ORBX_HIP_CHECK(hipMemcpyAsync(&n_matches[k], d + o[k].n, 4, hipMemcpyDeviceToHost, ctx->stream));
    }
    ORBX_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    for (int k = 0; k < n; k++)
        if (n_matches[k] < 0) return ORBX_ERR_UNSUPPORTED;
    return ORBX_OK;
}

namespace {

// SearchByBoW(KF1, KF2) (mode 1) / SearchForTriangulation (mode 2) of the
// frame in slot1 against the frames in slots2[0, n): keypoints, descriptors
// and FeatureVectors where orbx_dev_extract / orbx_dev_undistort /
// orbx_dev_compute_bow left them; only the map-point states travel.
int run_bow_slots(orbx_ctx* ctx, int mode, int slot1, const uint8_t* mp1, int n, const int* slots2,
                  const uint8_t* const* mp2s, float nnratio, int check_ori, const float* F12s, const float* sigma2s,
                  int nlevels, int32_t* const* outs, int cap, int* n_outs)
{
    auto ready = [&](int s) {
        return s >= 0 && s < ctx->slots && ctx->bow_dev && s < (int)ctx->bow_ready.size() && ctx->bow_ready[s];
    };
    if (n < 0 || (n > 0 && (!slots2 || !mp2s || !outs || !n_outs || !mp1))) return ORBX_ERR_ARG;
    if (mode == 2 && n > 0 && (!F12s || !sigma2s || nlevels <= 0 || nlevels > kMaxLevels)) return ORBX_ERR_ARG;
    if (!ready(slot1)) return ORBX_ERR_ARG;
    for (int k = 0; k < n; k++)
        if (!ready(slots2[k]) || !mp2s[k] || !outs[k]) return ORBX_ERR_ARG;
    const int nf = ctx->bow_nf;
    if (n > 0 && cap < nf) return ORBX_ERR_CAPACITY;
    if (n == 0) return ORBX_OK;
    ctx_enter(ctx);
    // the slots' feature counts bound the map-point arrays the caller passes
    std::vector<int32_t> cnt(ctx->slots);
    ORBX_HIP_CHECK(hipMemcpyAsync(cnt.data(), ctx->out_n, sizeof(int32_t) * ctx->slots, hipMemcpyDeviceToHost,
                                  ctx->stream));
    ORBX_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    auto count = [&](int s) { return std::min<int>(cnt[s], nf); };
    size_t at = 0;
    auto res = [&](size_t bytes) {
        const size_t o = at;
        at += al256(std::max<size_t>(bytes, 1));
        return o;
    };
    const size_t o_m1 = res(nf);
    struct Off {
        size_t m2, nd, out, bin, n;
    };
    std::vector<Off> o(n);
    for (int k = 0; k < n; k++) {
        o[k].m2 = res(nf);
        o[k].nd = res((size_t)nf * sizeof(int4));
        o[k].out = res((size_t)nf * 4);
        o[k].bin = res(nf);
        o[k].n = res(4);
    }
    const size_t o_jobs = res(sizeof(BowSlotJob) * (size_t)n);
    int r = ensure_scratch(ctx, at);
    if (r != ORBX_OK) return r;
    uint8_t* d = static_cast<uint8_t*>(ctx->scratch);
    if (count(slot1) > 0)
        ORBX_HIP_CHECK(hipMemcpyAsync(d + o_m1, mp1, count(slot1), hipMemcpyHostToDevice, ctx->stream));
    const SlotBowDev& b = ctx->bow;
    std::vector<BowSlotJob> jobs(n);
    for (int k = 0; k < n; k++) {
        const int s2 = slots2[k];
        if (count(s2) > 0)
            ORBX_HIP_CHECK(hipMemcpyAsync(d + o[k].m2, mp2s[k], count(s2), hipMemcpyHostToDevice, ctx->stream));
        ORBX_HIP_CHECK(hipMemsetAsync(d + o[k].out, 0xFF, (size_t)nf * 4, ctx->stream));
        ORBX_HIP_CHECK(hipMemsetAsync(d + o[k].bin, 0xFF, (size_t)nf, ctx->stream));
        BowSlotJob& j = jobs[k];
        j = BowSlotJob{};
        BowArgs& a = j.a;
        a.s1 = {ctx->out_kps + (size_t)slot1 * nf, ctx->out_desc + (size_t)slot1 * nf * 32, d + o_m1,
                b.fv_feat + (size_t)slot1 * nf};
        a.s2 = {ctx->out_kps + (size_t)s2 * nf, ctx->out_desc + (size_t)s2 * nf * 32, d + o[k].m2,
                b.fv_feat + (size_t)s2 * nf};
        a.mode = mode;
        a.nnratio = nnratio;
        a.check_ori = check_ori;
        if (mode == 2) {
            for (int c = 0; c < 9; c++) a.F12[c] = F12s[9 * k + c];
            for (int l = 0; l < nlevels; l++) a.sigma2[l] = sigma2s[(size_t)nlevels * k + l];
        }
        a.out = reinterpret_cast<int32_t*>(d + o[k].out);
        a.bins = reinterpret_cast<signed char*>(d + o[k].bin);
        a.out_n = reinterpret_cast<int32_t*>(d + o[k].n);
        j.kf_node_id = b.fv_nodes + (size_t)slot1 * nf;
        j.kf_node_ptr = b.fv_ptr + (size_t)slot1 * (nf + 1);
        j.kf_counts = b.counts + 2 * slot1;
        j.f_node_id = b.fv_nodes + (size_t)s2 * nf;
        j.f_node_ptr = b.fv_ptr + (size_t)s2 * (nf + 1);
        j.f_counts = b.counts + 2 * s2;
        j.out_count = ctx->out_n + slot1;
        j.nf = nf;
        j.nodes = reinterpret_cast<int4*>(d + o[k].nd);
    }
    ORBX_HIP_CHECK(hipMemcpyAsync(d + o_jobs, jobs.data(), sizeof(BowSlotJob) * (size_t)n, hipMemcpyHostToDevice,
                                  ctx->stream));
    timer_begin(ctx, "bow_match_slot");
    hipLaunchKernelGGL(k_bow_match_slot, dim3(n), dim3(kBlock), 0, ctx->stream,
                       reinterpret_cast<const BowSlotJob*>(d + o_jobs));
    timer_end(ctx, "bow_match_slot");
    ORBX_HIP_CHECK(hipGetLastError());
    for (int k = 0; k < n; k++) {
        ORBX_HIP_CHECK(hipMemcpyAsync(outs[k], d + o[k].out, (size_t)nf * 4, hipMemcpyDeviceToHost, ctx->stream));
        ORBX_HIP_CHECK(hipMemcpyAsync(&n_outs[k], d + o[k].n, 4, hipMemcpyDeviceToHost, ctx->stream));
    }
    ORBX_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    for (int k = 0; k < n; k++)
        if (n_outs[k] < 0) return ORBX_ERR_UNSUPPORTED;
    return ORBX_OK;
}

}  // namespace

extern "C" int orbx_dev_search_by_bow_kf(orbx_ctx* ctx, int slot1, const uint8_t* mp1, int n, const int* slots2,
                                         const uint8_t* const* mp2s, float nnratio, int check_ori,
                                         int32_t* const* matches12, int cap, int* n_matches)
{
    if (!ctx) return ORBX_ERR_ARG;
    return run_bow_slots(ctx, 1, slot1, mp1, n, slots2, mp2s, nnratio, check_ori, nullptr, nullptr, 0, matches12, cap,
                         n_matches);
}

extern "C" int orbx_dev_search_for_triangulation(orbx_ctx* ctx, int slot1, const uint8_t* mp1, int n,
                                                 const int* slots2, const uint8_t* const* mp2s, const float* F12s,
                                                 const float* sigma2_2s, int nlevels, int check_ori,
                                                 int32_t* const* matches12, int cap, int* n_matches)
{
    if (!ctx) return ORBX_ERR_ARG;
    if (n > 0 && nlevels != ctx->geom.nlevels) return ORBX_ERR_ARG;   // octaves index sigma2_2
    return run_bow_slots(ctx, 2, slot1, mp1, n, slots2, mp2s, 0.f, check_ori, F12s, sigma2_2s, nlevels, matches12,
                         cap, n_matches);
}
