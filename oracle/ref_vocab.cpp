// ORACLE -- TEST INFRASTRUCTURE ONLY (see ref_common.h).
//
// Sequential CPU restatement of DBoW2's TemplatedVocabulary::transform
// (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1127-1259) for ORB
// descriptors (FORB::distance = Hamming, Thirdparty/DBoW2/DBoW2/FORB.cpp),
// as Frame::ComputeBoW calls it (src/Frame.cc:279-286, levelsup 4), with the
// TF-IDF weighting and L1 scoring ORB-SLAM's vocabulary uses:
// BowVector::addWeight / normalize(L1) (BowVector.cpp:34-46, 60-90) and
// FeatureVector::addFeature (FeatureVector.cpp:31-45).
//
// The tree is given as loadFromTextFile builds it (TemplatedVocabulary.h:
// 1338-1420): node 0 the root, node i's parent parent[i], children in
// increasing id (file) order, word ids assigned to the nodes flagged leaf in
// id order.  The vocabulary file itself is absent (.MISSING_LARGE_BLOBS:1),
// so the tests run on synthetic trees of the same shape.
#include <cmath>
#include <cstdint>
#include <map>
#include <vector>

#include "../include/orbx.h"
#include "ref_common.h"

namespace orbref {

struct VocabRef {
    int k = 0, L = 0;
    std::vector<std::vector<int>> children;
    std::vector<uint8_t> desc;
    std::vector<double> weight;
    std::vector<int> word_id;
};

static void vocab_build(VocabRef& v, int k, int L, int n, const int32_t* parent, const uint8_t* is_leaf,
                        const uint8_t* desc, const double* weight)
{
    v.k = k;
    v.L = L;
    v.children.assign(n, {});
    v.desc.assign(desc, desc + (size_t)n * 32);
    v.weight.assign(weight, weight + n);
    v.word_id.assign(n, 0);
    int wid = 0;
    for (int i = 1; i < n; i++) {
        v.children[parent[i]].push_back(i);
        if (is_leaf[i]) v.word_id[i] = wid++;
    }
}

// transform(feature, word_id, weight, nid, levelsup) (:1218-1259)
static void transform_one(const VocabRef& v, const uint8_t* f, int levelsup, int& word, double& w, int& nid)
{
    const int nid_level = v.L - levelsup;
    nid = -1;
    if (nid_level <= 0) nid = 0;
    int final_id = 0, current_level = 0;
    do {
        ++current_level;
        const std::vector<int>& nodes = v.children[final_id];
        final_id = nodes[0];
        double best_d = descriptor_distance(f, v.desc.data() + (size_t)final_id * 32);
        for (size_t c = 1; c < nodes.size(); c++) {
            const int id = nodes[c];
            const double d = descriptor_distance(f, v.desc.data() + (size_t)id * 32);
            if (d < best_d) {
                best_d = d;
                final_id = id;
            }
        }
        if (current_level == nid_level) nid = final_id;
    } while (!v.children[final_id].empty());
    word = v.word_id[final_id];
    w = v.weight[final_id];
}

}  // namespace orbref

using namespace orbref;

extern "C" int orbx_ref_vocab_transform(int k, int L, int n_nodes, const int32_t* parent, const uint8_t* is_leaf,
                                        const uint8_t* vdesc, const double* vweight, int n, const uint8_t* desc,
                                        int levelsup, int32_t* word_id, double* weight, int32_t* node_id,
                                        uint32_t* bow_words, double* bow_values, int* n_words, uint32_t* fv_nodes,
                                        int32_t* fv_ptr, int32_t* fv_feat, int* n_fv_nodes)
{
    static thread_local VocabRef v;
    vocab_build(v, k, L, n_nodes, parent, is_leaf, vdesc, vweight);
    std::map<uint32_t, double> bow;                       // BowVector
    std::map<uint32_t, std::vector<int>> fv;              // FeatureVector
    for (int i = 0; i < n; i++) {
        int wd, nd;
        double w;
        transform_one(v, desc + (size_t)i * 32, levelsup, wd, w, nd);
        word_id[i] = wd;
        weight[i] = w;
        node_id[i] = nd;
        if (w > 0) {                                      // not stopped (:1157-1161)
            bow[(uint32_t)wd] += w;                       // BowVector::addWeight
            fv[(uint32_t)nd].push_back(i);                // FeatureVector::addFeature
        }
    }
    double norm = 0.0;                                    // BowVector::normalize(L1)
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
        for (int f : e.second) fv_feat[at++] = f;
        nn++;
    }
    fv_ptr[nn] = at;
    *n_fv_nodes = nn;
    return ORBX_OK;
}
