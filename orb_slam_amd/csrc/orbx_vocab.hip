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
// FeatureVector maps are assembled on the host from the per-feature results
// in the reference's order (std::map iteration, addWeight sums in feature
// order, L1 normalisation over ascending word ids).
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

__global__ __launch_bounds__(256) void k_vocab_transform(VocabDev v, const uint4* feat, int n, int nid_level,
                                                         int32_t* word, double* w, int32_t* nid)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint4 f0 = feat[2 * i], f1 = feat[2 * i + 1];
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
    word[i] = v.word_id[final_id];
    w[i] = v.weight[final_id];
    nid[i] = out_nid;
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
