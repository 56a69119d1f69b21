// ORACLE -- TEST INFRASTRUCTURE ONLY (see ref_common.h).
//
// Sequential CPU restatement of the vocabulary-node searches of
// ORBmatcher (src/ORBmatcher.cc): SearchByBoW(KeyFrame*, Frame&) (:155-283),
// SearchByBoW(KeyFrame*, KeyFrame*) (:715-850) and SearchForTriangulation
// (:852-1014) with CheckDistEpipolarLine (:136-153), on flattened keyframe
// views (include/orbx.h orbx_bow_view).  DBoW2::FeatureVector is a
// std::map<NodeId, vector<unsigned>>; its CSR form keeps the map order, and
// the reference's lower_bound merge visits exactly the common node ids in
// ascending order.
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <utility>
#include <vector>

#include "../include/orbx.h"
#include "ref_common.h"

namespace orbref {
namespace {

const int TH_LOW = 50;        // src/ORBmatcher.cc:41
const int HISTO_LENGTH = 30;  // :42

void three_maxima(const std::vector<int>* histo, int L, int& ind1, int& ind2, int& ind3)
{
    int max1 = 0, max2 = 0, max3 = 0;
    for (int i = 0; i < L; i++) {
        const int s = (int)histo[i].size();
        if (s > max1) {
            max3 = max2; max2 = max1; max1 = s;
            ind3 = ind2; ind2 = ind1; ind1 = i;
        } else if (s > max2) {
            max3 = max2; max2 = s;
            ind3 = ind2; ind2 = i;
        } else if (s > max3) {
            max3 = s;
            ind3 = i;
        }
    }
    if (max2 < 0.1f * (float)max1) {
        ind2 = -1;
        ind3 = -1;
    } else if (max3 < 0.1f * (float)max1) {
        ind3 = -1;
    }
}

int rot_bin(float a1, float a2)
{
    const float factor = 1.0f / HISTO_LENGTH;
    float rot = a1 - a2;
    if (rot < 0.0) rot += 360.0f;
    int bin = (int)std::round(rot * factor);
    if (bin == HISTO_LENGTH) bin = 0;
    return bin;
}

struct NodePair {
    int first1, count1, first2, count2;
};

// Common FeatureVector nodes, in the order of the reference's merge loop.
std::vector<NodePair> common_nodes(const orbx_bow_view& a, const orbx_bow_view& b)
{
    std::vector<NodePair> out;
    int i = 0, j = 0;
    while (i < a.n_nodes && j < b.n_nodes) {
        if (a.node_id[i] == b.node_id[j]) {
            out.push_back({a.node_ptr[i], a.node_ptr[i + 1] - a.node_ptr[i], b.node_ptr[j],
                           b.node_ptr[j + 1] - b.node_ptr[j]});
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

// The ComputeThreeMaxima pass shared by the three searches; returns the
// number of matches removed.
int rotation_filter(std::vector<int>* rotHist, std::vector<int>& out)
{
    int ind1 = -1, ind2 = -1, ind3 = -1;
    three_maxima(rotHist, HISTO_LENGTH, ind1, ind2, ind3);
    int removed = 0;
    for (int i = 0; i < HISTO_LENGTH; i++) {
        if (i == ind1 || i == ind2 || i == ind3) continue;
        for (int k : rotHist[i]) {
            out[k] = -1;
            removed++;
        }
    }
    return removed;
}

}  // namespace

// ORBmatcher::SearchByBoW(KeyFrame*, Frame&) (src/ORBmatcher.cc:155-283)
int search_by_bow_frame(const orbx_bow_view& KF, const orbx_bow_view& F, float nnratio, bool checkOri,
                        std::vector<int>& matchesF)
{
    matchesF.assign(F.n, -1);
    std::vector<int> rotHist[HISTO_LENGTH];
    int nmatches = 0;
    for (const NodePair& nd : common_nodes(KF, F)) {
        for (int a = 0; a < nd.count1; a++) {
            const int realIdxKF = KF.feat_idx[nd.first1 + a];
            if (KF.mp[realIdxKF] != 1) continue;   // !pMP || pMP->isBad()
            const uint8_t* dKF = KF.desc + (size_t)realIdxKF * 32;
            int bestDist1 = INT_MAX, bestIdxF = -1, bestDist2 = INT_MAX;
            for (int b = 0; b < nd.count2; b++) {
                const int realIdxF = F.feat_idx[nd.first2 + b];
                if (matchesF[realIdxF] >= 0) continue;
                const int dist = descriptor_distance(dKF, F.desc + (size_t)realIdxF * 32);
                if (dist < bestDist1) {
                    bestDist2 = bestDist1;
                    bestDist1 = dist;
                    bestIdxF = realIdxF;
                } else if (dist < bestDist2) {
                    bestDist2 = dist;
                }
            }
            if (bestDist1 <= TH_LOW && static_cast<float>(bestDist1) < nnratio * static_cast<float>(bestDist2)) {
                matchesF[bestIdxF] = realIdxKF;
                if (checkOri) rotHist[rot_bin(KF.keys[realIdxKF].angle, F.keys[bestIdxF].angle)].push_back(bestIdxF);
                nmatches++;
            }
        }
    }
    if (checkOri) nmatches -= rotation_filter(rotHist, matchesF);
    return nmatches;
}

// ORBmatcher::SearchByBoW(KeyFrame*, KeyFrame*) (src/ORBmatcher.cc:715-850)
int search_by_bow_kf(const orbx_bow_view& K1, const orbx_bow_view& K2, float nnratio, bool checkOri,
                     std::vector<int>& matches12)
{
    matches12.assign(K1.n, -1);
    std::vector<uint8_t> matched2(K2.n, 0);
    std::vector<int> rotHist[HISTO_LENGTH];
    int nmatches = 0;
    for (const NodePair& nd : common_nodes(K1, K2)) {
        for (int a = 0; a < nd.count1; a++) {
            const int idx1 = K1.feat_idx[nd.first1 + a];
            if (K1.mp[idx1] != 1) continue;
            const uint8_t* d1 = K1.desc + (size_t)idx1 * 32;
            int bestDist1 = INT_MAX, bestIdx2 = -1, bestDist2 = INT_MAX;
            for (int b = 0; b < nd.count2; b++) {
                const int idx2 = K2.feat_idx[nd.first2 + b];
                if (matched2[idx2] || K2.mp[idx2] == 0) continue;
                if (K2.mp[idx2] == 2) continue;
                const int dist = descriptor_distance(d1, K2.desc + (size_t)idx2 * 32);
                if (dist < bestDist1) {
                    bestDist2 = bestDist1;
                    bestDist1 = dist;
                    bestIdx2 = idx2;
                } else if (dist < bestDist2) {
                    bestDist2 = dist;
                }
            }
            if (bestDist1 < TH_LOW && static_cast<float>(bestDist1) < nnratio * static_cast<float>(bestDist2)) {
                matches12[idx1] = bestIdx2;
                matched2[bestIdx2] = 1;
                if (checkOri) rotHist[rot_bin(K1.keys[idx1].angle, K2.keys[bestIdx2].angle)].push_back(idx1);
                nmatches++;
            }
        }
    }
    if (checkOri) nmatches -= rotation_filter(rotHist, matches12);
    return nmatches;
}

// ORBmatcher::CheckDistEpipolarLine (src/ORBmatcher.cc:136-153): float
// line coefficients, the threshold 3.84 * sigma2 in double.
static bool check_dist_epipolar(const orbx_keypoint& kp1, const orbx_keypoint& kp2, const float* F12,
                                const float* sigma2)
{
    const float a = kp1.x * F12[0] + kp1.y * F12[3] + F12[6];
    const float b = kp1.x * F12[1] + kp1.y * F12[4] + F12[7];
    const float c = kp1.x * F12[2] + kp1.y * F12[5] + F12[8];
    const float num = a * kp2.x + b * kp2.y + c;
    const float den = a * a + b * b;
    if (den == 0) return false;
    const float dsqr = num * num / den;
    return dsqr < 3.84 * sigma2[kp2.octave];
}

// ORBmatcher::SearchForTriangulation (src/ORBmatcher.cc:852-1014)
int search_for_triangulation(const orbx_bow_view& K1, const orbx_bow_view& K2, const float* F12,
                             const float* sigma2_2, bool checkOri, std::vector<int>& matches12)
{
    matches12.assign(K1.n, -1);
    std::vector<uint8_t> matched2(K2.n, 0);
    std::vector<int> rotHist[HISTO_LENGTH];
    int nmatches = 0;
    for (const NodePair& nd : common_nodes(K1, K2)) {
        for (int a = 0; a < nd.count1; a++) {
            const int idx1 = K1.feat_idx[nd.first1 + a];
            if (K1.mp[idx1] != 0) continue;   // already has a MapPoint (bad or not)
            const orbx_keypoint& kp1 = K1.keys[idx1];
            const uint8_t* d1 = K1.desc + (size_t)idx1 * 32;
            std::vector<std::pair<int, int>> vDistIndex;
            for (int b = 0; b < nd.count2; b++) {
                const int idx2 = K2.feat_idx[nd.first2 + b];
                if (matched2[idx2] || K2.mp[idx2] != 0) continue;
                const int dist = descriptor_distance(d1, K2.desc + (size_t)idx2 * 32);
                if (dist > TH_LOW) continue;
                vDistIndex.push_back({dist, idx2});
            }
            if (vDistIndex.empty()) continue;
            std::sort(vDistIndex.begin(), vDistIndex.end());
            const int DistTh = (int)std::round(2 * vDistIndex.front().first);
            for (const auto& di : vDistIndex) {
                if (di.first > DistTh) break;
                const int idx2 = di.second;
                const orbx_keypoint& kp2 = K2.keys[idx2];
                if (check_dist_epipolar(kp1, kp2, F12, sigma2_2)) {
                    matched2[idx2] = 1;
                    matches12[idx1] = idx2;
                    nmatches++;
                    if (checkOri) rotHist[rot_bin(kp1.angle, kp2.angle)].push_back(idx1);
                    break;
                }
            }
        }
    }
    if (checkOri) nmatches -= rotation_filter(rotHist, matches12);
    return nmatches;
}

}  // namespace orbref

using namespace orbref;

extern "C" int orbx_ref_search_by_bow_frame(const orbx_bow_view* KF, const orbx_bow_view* F, float nnratio,
                                            int check_ori, int32_t* matches_f, int* n_matches)
{
    std::vector<int> m;
    *n_matches = search_by_bow_frame(*KF, *F, nnratio, check_ori != 0, m);
    std::copy(m.begin(), m.end(), matches_f);
    return ORBX_OK;
}

extern "C" int orbx_ref_search_by_bow_kf(const orbx_bow_view* K1, const orbx_bow_view* K2, float nnratio,
                                         int check_ori, int32_t* matches12, int* n_matches)
{
    std::vector<int> m;
    *n_matches = search_by_bow_kf(*K1, *K2, nnratio, check_ori != 0, m);
    std::copy(m.begin(), m.end(), matches12);
    return ORBX_OK;
}

extern "C" int orbx_ref_search_for_triangulation(const orbx_bow_view* K1, const orbx_bow_view* K2, const float* F12,
                                                 const float* sigma2_2, int check_ori, int32_t* matches12,
                                                 int* n_matches)
{
    std::vector<int> m;
    *n_matches = search_for_triangulation(*K1, *K2, F12, sigma2_2, check_ori != 0, m);
    std::copy(m.begin(), m.end(), matches12);
    return ORBX_OK;
}
