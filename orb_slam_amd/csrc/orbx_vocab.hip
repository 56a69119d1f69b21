// DBoW2 vocabulary-tree descent on MI355X: TemplatedVocabulary::transform
// (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1127-1259) for ORB
// descriptors, as Frame::ComputeBoW calls it (src/Frame.cc:279-286).
//
// The tree lives in HBM as a children CSR (children in increasing id order,
// as loadFromTextFile appends them) with 32-byte node descriptors stored as
// two 16-byte words, word ids and weights.  One thread per feature walks
// from the root: at each level it loads the child list and the children's
// descriptors (independent 16-byte loads issued back to back) and keeps the
// first strict minimum Hamming distance, recording the level-(L - levelsup)
// node for the FeatureVector.  The upper levels (the first 111 nodes of a
// k = 10 tree) are shared by every feature and stay in L2.  The BowVector /
// FeatureVector maps are assembled from the per-feature results in the
// reference's order (std::map iteration, addWeight sums in feature order, L1
// normalisation over ascending word ids): on the host for the one-shot
// orbx_vocab_transform, on the device (k_bow_build, one workgroup per frame)
// for extracted slots (orbx_dev_compute_bow), whose FeatureVector then feeds
// orbx_dev_search_by_bow without leaving HBM.
#include <algorithm>
#include <cmath>
#include <map>
#include <vector>

#include "orbx_device.h"
#include "orbx_internal.h"

struct orbx_vocab {
    int device = 0;
    int k = 0, L = 0, n_nodes = 0, n_words = 0;
    int32_t* child_ptr = nullptr;   // [n_nodes + 1]
    int32_t* child_idx = nullptr;   // [n_nodes - 1]
    uint4* desc = nullptr;          // [n_nodes][2]
    double* weight = nullptr;       // [n_nodes]
    int32_t* word_id = nullptr;     // [n_nodes]
};

namespace orbx {

struct VocabDev {
    const int32_t* child_ptr;
    const int32_t* child_idx;
    const uint4* desc;
    const double* weight;
    const int32_t* word_id;
};

// One feature's descent from the root (TemplatedVocabulary::transform's
// per-feature loop, :1205-1240): the first strict minimum child per level.
__device__ inline void vocab_descend(const VocabDev& v, uint4 f0, uint4 f1, int nid_level, int32_t& word, double& w,
                                     int32_t& nid)
{
    int final_id = 0, level = 0, out_nid = nid_level <= 0 ? 0 : -1;
    int c0 = v.child_ptr[0], c1 = v.child_ptr[1];
    while (c0 < c1) {
        ++level;
        int best = v.child_idx[c0];
        int bd = hamming256(f0, f1, v.desc[2 * best], v.desc[2 * best + 1]);
        for (int c = c0 + 1; c < c1; c++) {
            const int id = v.child_idx[c];
            const int d = hamming256(f0, f1, v.desc[2 * id], v.desc[2 * id + 1]);
            if (d < bd) {
                bd = d;
                best = id;
            }
        }
        final_id = best;
        if (level == nid_level) out_nid = final_id;
        c0 = v.child_ptr[final_id];
        c1 = v.child_ptr[final_id + 1];
    }
    word = v.word_id[final_id];
    w = v.weight[final_id];
    nid = out_nid;
}

__global__ __launch_bounds__(256) void k_vocab_transform(VocabDev v, const uint4* feat, int n, int nid_level,
                                                         int32_t* word, double* w, int32_t* nid)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    vocab_descend(v, feat[2 * i], feat[2 * i + 1], nid_level, word[i], w[i], nid[i]);
}

// Device-resident frames (orbx_dev_compute_bow): the descent of every
// extracted feature of slots [first, first + gridDim.y), each slot's count
// read on the device.
__global__ __launch_bounds__(256) void k_vocab_transform_slots(VocabDev v, const uint4* desc, const int32_t* n_feat,
                                                               int nf, int nid_level, SlotBowDev b)
{
    const int s = blockIdx.y, i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= min(n_feat[s], nf)) return;
    const size_t e = (size_t)s * nf + i;
    vocab_descend(v, desc[2 * e], desc[2 * e + 1], nid_level, b.word[e], b.weight[e], b.node[e]);
}

// Bitonic sort of keys[0, N) (N a power of two <= kBowSortMax) by the block.
template <int kThreads>
__device__ inline void block_bitonic_sort(uint64_t* keys, int N)
{
    for (int k = 2; k <= N; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int t = threadIdx.x; t < N / 2; t += kThreads) {
                const int lo = 2 * t - (t & (j - 1)), hi = lo + j;
                const uint64_t a = keys[lo], c = keys[hi];
                const bool up = (lo & k) == 0;
                if ((a > c) == up) {
                    keys[lo] = c;
                    keys[hi] = a;
                }
            }
            __syncthreads();
        }
}

// One slot's FeatureVector and BowVector from the per-feature descent
// results, in the reference's std::map order (TemplatedVocabulary.h:
// 1145-1193): features with weight > 0 only; FeatureVector nodes ascending
// with their features ascending; BowVector words ascending, each value the
// sum of its features' weights in feature order (addWeight), then L1
// normalised by the sum of |value| over ascending words (BowVector::
// normalize).  Sorting (id << 32 | feature) keys gives both orders; the
// sums are sequential per word and the norm sequential over words, so the
// doubles are those of the map code.
constexpr int kBowBuildThreads = 1024;

__global__ __launch_bounds__(kBowBuildThreads) void k_bow_build(const int32_t* n_feat, int nf, SlotBowDev b)
{
    __shared__ uint64_t keys[kBowSortMax];
    __shared__ BlockScratchN<kBowBuildThreads / 64> bs;
    __shared__ double s_norm;
    const int s = blockIdx.x, tid = threadIdx.x;
    const int n = min(n_feat[s], nf);
    const size_t o = (size_t)s * nf;
    int N = 1;
    while (N < n) N <<= 1;
    const int per = (N + kBowBuildThreads - 1) / kBowBuildThreads, p0 = tid * per;
    for (int pass = 0; pass < 2; pass++) {
        // pass 0: (node, feature) -> FeatureVector; pass 1: (word, feature) -> BowVector
        int valid = 0;
        for (int p = tid; p < N; p += kBowBuildThreads) {
            // entries past n (the power-of-two padding) belong to the next
            // slot or past the array: only p < n is read
            const bool ok = p < n && b.weight[o + p] > 0.0;
            uint64_t key = ~0ull;
            if (ok) key = (uint64_t)(uint32_t)(pass == 0 ? b.node[o + p] : b.word[o + p]) << 32 | (uint32_t)p;
            keys[p] = key;
            valid += ok;
        }
        const int m = block_sum(valid, bs, 0);   // includes the barrier after the fill
        block_bitonic_sort<kBowBuildThreads>(keys, N);
        // group heads, compacted in key order
        int heads = 0;
        for (int p = p0; p < min(p0 + per, m); p++) heads += p == 0 || (keys[p] >> 32) != (keys[p - 1] >> 32);
        int nh;
        int h = block_exclusive_scan(heads, &nh, bs, 1);
        if (pass == 0) {
            for (int p = p0; p < min(p0 + per, m); p++) {
                b.fv_feat[o + p] = (int32_t)(uint32_t)keys[p];
                if (p == 0 || (keys[p] >> 32) != (keys[p - 1] >> 32)) {
                    b.fv_nodes[o + h] = (uint32_t)(keys[p] >> 32);
                    b.fv_ptr[(size_t)s * (nf + 1) + h] = p;
                    h++;
                }
            }
            if (tid == 0) {
                b.fv_ptr[(size_t)s * (nf + 1) + nh] = m;
                b.counts[2 * s + 1] = nh;
            }
            __syncthreads();   // keys are refilled by pass 1
        } else {
            // per-word sums in feature order, kept in registers until the
            // keys are no longer needed, then staged in the keys array
            double sum[4];
            int nsum = 0;
            for (int p = p0; p < min(p0 + per, m); p++) {
                if (!(p == 0 || (keys[p] >> 32) != (keys[p - 1] >> 32))) continue;
                double acc = 0.0;
                for (int q = p; q < m && (keys[q] >> 32) == (keys[p] >> 32); q++)
                    acc += b.weight[o + (uint32_t)keys[q]];
                b.bow_words[o + h + nsum] = (uint32_t)(keys[p] >> 32);
                sum[nsum++] = acc;
            }
            __syncthreads();
            double* vals = reinterpret_cast<double*>(keys);
            for (int q = 0; q < nsum; q++) vals[h + q] = sum[q];
            __syncthreads();
            if (tid == 0) {
                double norm = 0.0;
                for (int q = 0; q < nh; q++) norm += fabs(vals[q]);
                s_norm = norm;
                b.counts[2 * s] = nh;
            }
            __syncthreads();
            const double norm = s_norm;
            for (int q = tid; q < nh; q += kBowBuildThreads)
                b.bow_values[o + q] = norm > 0.0 ? vals[q] / norm : vals[q];
        }
    }
}

}  // namespace orbx

using namespace orbx;

extern "C" int orbx_vocab_create(orbx_ctx* ctx, int k, int L, int n_nodes, const int32_t* parent,
                                 const uint8_t* is_leaf, const uint8_t* desc, const double* weight, orbx_vocab** out)
{
    if (!ctx || !out || k < 1 || L < 1 || n_nodes < 2 || !parent || !is_leaf || !desc || !weight)
        return ORBX_ERR_ARG;
    *out = nullptr;
    // children CSR in increasing id order; word ids for the leaf-flagged nodes
    std::vector<int32_t> cnt(n_nodes + 1, 0), word(n_nodes, 0);
    int wid = 0;
    for (int i = 1; i < n_nodes; i++) {
        if (parent[i] < 0 || parent[i] >= n_nodes || parent[i] == i) return ORBX_ERR_ARG;
        cnt[parent[i] + 1]++;
        if (is_leaf[i]) word[i] = wid++;
    }
    for (int i = 0; i < n_nodes; i++) cnt[i + 1] += cnt[i];
    std::vector<int32_t> idx(std::max(n_nodes - 1, 1)), fill(cnt.begin(), cnt.end() - 1);
    for (int i = 1; i < n_nodes; i++) idx[fill[parent[i]]++] = i;
    // loadFromTextFile's files list a parent before its children; requiring
    // it also rules out cycles, so every descent ends at a childless node
    for (int i = 1; i < n_nodes; i++)
        if (parent[i] >= i) return ORBX_ERR_ARG;
    ctx_enter(ctx);
    orbx_vocab* v = new orbx_vocab;
    v->device = ctx->device;
    v->k = k;
    v->L = L;
    v->n_nodes = n_nodes;
    v->n_words = wid;
    auto fail = [&](int code) {
        orbx_vocab_destroy(v);
        return code;
    };
    if (hipMalloc(&v->child_ptr, (size_t)(n_nodes + 1) * 4) != hipSuccess ||
        hipMalloc(&v->child_idx, idx.size() * 4) != hipSuccess ||
        hipMalloc(&v->desc, (size_t)n_nodes * 32) != hipSuccess ||
        hipMalloc(&v->weight, (size_t)n_nodes * 8) != hipSuccess ||
        hipMalloc(&v->word_id, (size_t)n_nodes * 4) != hipSuccess)
        return fail(ORBX_ERR_NOMEM);
    if (hipMemcpyAsync(v->child_ptr, cnt.data(), (size_t)(n_nodes + 1) * 4, hipMemcpyHostToDevice, ctx->stream) ||
        hipMemcpyAsync(v->child_idx, idx.data(), idx.size() * 4, hipMemcpyHostToDevice, ctx->stream) ||
        hipMemcpyAsync(v->desc, desc, (size_t)n_nodes * 32, hipMemcpyHostToDevice, ctx->stream) ||
        hipMemcpyAsync(v->weight, weight, (size_t)n_nodes * 8, hipMemcpyHostToDevice, ctx->stream) ||
        hipMemcpyAsync(v->word_id, word.data(), (size_t)n_nodes * 4, hipMemcpyHostToDevice, ctx->stream) ||
        hipStreamSynchronize(ctx->stream))
        return fail(ORBX_ERR_HIP);
    *out = v;
    return ORBX_OK;
}

extern "C" void orbx_vocab_destroy(orbx_vocab* v)
{
    if (!v) return;
    (void)hipSetDevice(v->device);
    void* ptrs[] = {v->child_ptr, v->child_idx, v->desc, v->weight, v->word_id};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    delete v;
}

extern "C" int orbx_vocab_n_words(const orbx_vocab* v) { return v ? v->n_words : 0; }

extern "C" int orbx_vocab_transform(orbx_ctx* ctx, const orbx_vocab* voc, int n, const uint8_t* desc, int levelsup,
                                    int32_t* word_id, double* weight, int32_t* node_id, uint32_t* bow_words,
                                    double* bow_values, int* n_words, uint32_t* fv_nodes, int32_t* fv_ptr,
                                    int32_t* fv_feat, int* n_fv_nodes)
{
    if (!ctx || !voc || n < 0 || (n > 0 && (!desc || !word_id || !weight || !node_id || !bow_words || !bow_values ||
                                          !fv_nodes || !fv_feat)) ||
        !n_words || !fv_ptr || !n_fv_nodes || voc->device != ctx->device)
        return ORBX_ERR_ARG;
    ctx_enter(ctx);
    if (n > 0) {
        const size_t o_f = 0, o_w = ((size_t)n * 32 + 255) & ~size_t(255), o_d = o_w + (((size_t)n * 4 + 255) & ~size_t(255)),
                     o_n = o_d + (((size_t)n * 8 + 255) & ~size_t(255)), total = o_n + (size_t)n * 4;
        int r = ensure_scratch(ctx, total);
        if (r != ORBX_OK) return r;
        uint8_t* d = static_cast<uint8_t*>(ctx->scratch);
        ORBX_HIP_CHECK(hipMemcpyAsync(d + o_f, desc, (size_t)n * 32, hipMemcpyHostToDevice, ctx->stream));
        VocabDev v{voc->child_ptr, voc->child_idx, voc->desc, voc->weight, voc->word_id};
        timer_begin(ctx, "vocab");
        hipLaunchKernelGGL(k_vocab_transform, dim3((n + 255) / 256), dim3(256), 0, ctx->stream, v,
                           reinterpret_cast<const uint4*>(d + o_f), n, voc->L - levelsup,
                           reinterpret_cast<int32_t*>(d + o_w), reinterpret_cast<double*>(d + o_d),
                           reinterpret_cast<int32_t*>(d + o_n));
        timer_end(ctx, "vocab");
        ORBX_HIP_CHECK(hipGetLastError());
        ORBX_HIP_CHECK(hipMemcpyAsync(word_id, d + o_w, (size_t)n * 4, hipMemcpyDeviceToHost, ctx->stream));
        ORBX_HIP_CHECK(hipMemcpyAsync(weight, d + o_d, (size_t)n * 8, hipMemcpyDeviceToHost, ctx->stream));
        ORBX_HIP_CHECK(hipMemcpyAsync(node_id, d + o_n, (size_t)n * 4, hipMemcpyDeviceToHost, ctx->stream));
        ORBX_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    }
    // BowVector / FeatureVector in the reference's map order (:1145-1193)
    std::map<uint32_t, double> bow;
    std::map<uint32_t, std::vector<int32_t>> fv;
    for (int i = 0; i < n; i++) {
        if (!(weight[i] > 0)) continue;
        bow[(uint32_t)word_id[i]] += weight[i];
        fv[(uint32_t)node_id[i]].push_back(i);
    }
    double norm = 0.0;
    for (auto& e : bow) norm += std::fabs(e.second);
    int c = 0;
    for (auto& e : bow) {
        bow_words[c] = e.first;
        bow_values[c] = norm > 0.0 ? e.second / norm : e.second;
        c++;
    }
    *n_words = c;
    int nn = 0, at = 0;
    for (auto& e : fv) {
        fv_nodes[nn] = e.first;
        fv_ptr[nn] = at;
        for (int32_t f : e.second) fv_feat[at++] = f;
        nn++;
    }
    fv_ptr[nn] = at;
    *n_fv_nodes = nn;
    return ORBX_OK;
}

namespace {

// The per-slot BoW buffer for the context's slots x nfeatures.
int ensure_slot_bow(orbx_ctx* ctx)
{
    const int nf = ctx->geom.nfeatures;
    if (ctx->bow_dev && ctx->bow_nf == nf) return ORBX_OK;
    if (ctx->bow_dev) {
        (void)hipStreamSynchronize(ctx->stream);
        (void)hipFree(ctx->bow_dev);
        ctx->bow_dev = nullptr;
    }
    const size_t S = (size_t)ctx->slots, e = S * nf;
    auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
    const size_t o_word = 0, o_w = o_word + al(e * 4), o_node = o_w + al(e * 8), o_fvn = o_node + al(e * 4),
                 o_fvp = o_fvn + al(e * 4), o_fvf = o_fvp + al(S * (nf + 1) * 4), o_bw = o_fvf + al(e * 4),
                 o_bv = o_bw + al(e * 4), o_c = o_bv + al(e * 8), total = o_c + al(S * 8);
    if (hipMalloc(&ctx->bow_dev, total) != hipSuccess) {
        ctx->bow_dev = nullptr;
        return ORBX_ERR_NOMEM;
    }
    uint8_t* d = static_cast<uint8_t*>(ctx->bow_dev);
    ctx->bow = SlotBowDev{reinterpret_cast<int32_t*>(d + o_word), reinterpret_cast<double*>(d + o_w),
                          reinterpret_cast<int32_t*>(d + o_node), reinterpret_cast<uint32_t*>(d + o_fvn),
                          reinterpret_cast<int32_t*>(d + o_fvp), reinterpret_cast<int32_t*>(d + o_fvf),
                          reinterpret_cast<uint32_t*>(d + o_bw), reinterpret_cast<double*>(d + o_bv),
                          reinterpret_cast<int32_t*>(d + o_c)};
    ctx->bow_nf = nf;
    ctx->bow_ready.assign(ctx->slots, 0);
    return ORBX_OK;
}

}  // namespace

extern "C" int orbx_dev_compute_bow(orbx_ctx* ctx, const orbx_vocab* voc, int first, int count, int levelsup)
{
    if (!ctx || !voc || count <= 0 || first < 0 || first + count > ctx->slots || ctx->geom_w <= 0 ||
        voc->device != ctx->device)
        return ORBX_ERR_ARG;
    const int nf = ctx->geom.nfeatures;
    if (nf > kBowSortMax) return ORBX_ERR_UNSUPPORTED;
    ctx_enter(ctx);
    int r = ensure_slot_bow(ctx);
    if (r != ORBX_OK) return r;
    SlotBowDev b = ctx->bow;
    const size_t o = (size_t)first * nf;
    b.word += o;
    b.weight += o;
    b.node += o;
    b.fv_nodes += o;
    b.fv_ptr += (size_t)first * (nf + 1);
    b.fv_feat += o;
    b.bow_words += o;
    b.bow_values += o;
    b.counts += 2 * first;
    VocabDev v{voc->child_ptr, voc->child_idx, voc->desc, voc->weight, voc->word_id};
    timer_begin(ctx, "vocab");
    hipLaunchKernelGGL(k_vocab_transform_slots, dim3((nf + 255) / 256, count), dim3(256), 0, ctx->stream, v,
                       reinterpret_cast<const uint4*>(ctx->out_desc + o * 32), ctx->out_n + first, nf,
                       voc->L - levelsup, b);
    timer_end(ctx, "vocab");
    ORBX_HIP_CHECK(hipGetLastError());
    timer_begin(ctx, "bow_build");
    hipLaunchKernelGGL(k_bow_build, dim3(count), dim3(kBowBuildThreads), 0, ctx->stream, ctx->out_n + first, nf, b);
    timer_end(ctx, "bow_build");
    ORBX_HIP_CHECK(hipGetLastError());
    for (int s = first; s < first + count; s++) ctx->bow_ready[s] = 1;
    return ORBX_OK;
}

extern "C" int orbx_dev_read_bow(orbx_ctx* ctx, int slot, int cap, int32_t* word_id, double* weight, int32_t* node_id,
                                 uint32_t* bow_words, double* bow_values, int* n_words, uint32_t* fv_nodes,
                                 int32_t* fv_ptr, int32_t* fv_feat, int* n_fv_nodes)
{
    if (!ctx || slot < 0 || slot >= ctx->slots || cap < 0) return ORBX_ERR_ARG;
    if (!ctx->bow_dev || slot >= (int)ctx->bow_ready.size() || !ctx->bow_ready[slot]) return ORBX_ERR_ARG;
    ctx_enter(ctx);
    ORBX_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    const size_t nf = ctx->bow_nf, o = (size_t)slot * nf;
    int32_t n = 0, c[2] = {0, 0};
    ORBX_HIP_CHECK(hipMemcpy(&n, ctx->out_n + slot, 4, hipMemcpyDeviceToHost));
    ORBX_HIP_CHECK(hipMemcpy(c, ctx->bow.counts + 2 * slot, 8, hipMemcpyDeviceToHost));
    n = std::min<int32_t>(n, (int32_t)nf);
    if (n_words) *n_words = c[0];
    if (n_fv_nodes) *n_fv_nodes = c[1];
    if (n > cap) return ORBX_ERR_CAPACITY;
    auto get = [&](void* dst, const void* src, size_t bytes) -> int {
        if (dst && bytes) ORBX_HIP_CHECK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
        return ORBX_OK;
    };
    int32_t m = 0;   // features in the FeatureVector
    ORBX_HIP_CHECK(hipMemcpy(&m, ctx->bow.fv_ptr + slot * (nf + 1) + c[1], 4, hipMemcpyDeviceToHost));
    int r;
    if ((r = get(word_id, ctx->bow.word + o, (size_t)n * 4)) || (r = get(weight, ctx->bow.weight + o, (size_t)n * 8)) ||
        (r = get(node_id, ctx->bow.node + o, (size_t)n * 4)) ||
        (r = get(bow_words, ctx->bow.bow_words + o, (size_t)c[0] * 4)) ||
        (r = get(bow_values, ctx->bow.bow_values + o, (size_t)c[0] * 8)) ||
        (r = get(fv_nodes, ctx->bow.fv_nodes + o, (size_t)c[1] * 4)) ||
        (r = get(fv_ptr, ctx->bow.fv_ptr + slot * (nf + 1), (size_t)(c[1] + 1) * 4)) ||
        (r = get(fv_feat, ctx->bow.fv_feat + o, (size_t)m * 4)))
        return r;
    return ORBX_OK;
}
