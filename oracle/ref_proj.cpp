// ORACLE -- TEST INFRASTRUCTURE ONLY (see ref_common.h).
//
// Sequential CPU restatement of the keyframe projection searches of
// ORBmatcher and of MapPoint::ComputeDistinctiveDescriptors:
//   Fuse(KeyFrame*, vector<MapPoint*>&, th)          src/ORBmatcher.cc:1016-1134
//   Fuse(KeyFrame*, cv::Mat Scw, vector<MapPoint*>&) src/ORBmatcher.cc:1136-1265
//   SearchBySim3                                     src/ORBmatcher.cc:1267-1505
//   ComputeDistinctiveDescriptors                    src/MapPoint.cc:185-250
// Fuse is restated as its state-free part -- the best keyframe keypoint of
// every map point (the caller replays the graph updates in map-point
// order, as the reference's loop does).
//
// cv::Mat arithmetic (OpenCV 2.4, un-vendored, restated): small float
// matrix products sum the float products left to right; a Mat divided or
// multiplied by a scalar is scaled by a double factor and rounded to float;
// cv::norm and Mat::dot of float vectors accumulate in double.
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <vector>

#include "../include/orbx.h"
#include "ref_common.h"

namespace orbref {
namespace {

const int TH_LOW = 50;     // src/ORBmatcher.cc:41
const int TH_HIGH = 100;   // :40

// x = R * X + t, float products summed left to right
void xform(const float* R, const float* t, const float* X, float* o)
{
    for (int r = 0; r < 3; r++) o[r] = R[3 * r] * X[0] + R[3 * r + 1] * X[1] + R[3 * r + 2] * X[2] + t[r];
}

// cv::norm(float 3-vector): squares accumulated in double
float norm3(const float* v)
{
    double s = 0;
    for (int i = 0; i < 3; i++) {
        const double x = v[i];
        s += x * x;
    }
    return (float)std::sqrt(s);
}

// Mat::dot of float 3-vectors, in double
double dot3(const float* a, const float* b)
{
    double s = 0;
    for (int i = 0; i < 3; i++) s += (double)a[i] * b[i];
    return s;
}

int predicted_level(const std::vector<float>& scales, float ratio)
{
    const int it = (int)(std::lower_bound(scales.begin(), scales.end(), ratio) - scales.begin());
    return std::min(it, (int)scales.size() - 1);
}

// Best keypoint of KF within `radius` of (u, v) whose octave lies in
// [pred - 1, pred] (first strict minimum in GetFeaturesInArea order).
void best_in_area(const FrameRef& KF, float u, float v, float radius, int pred, const uint8_t* d, int& bestIdx,
                  int& bestDist)
{
    bestIdx = -1;
    bestDist = INT_MAX;
    for (size_t idx : KF.featuresInArea(u, v, radius, -1, -1)) {
        const int lvl = KF.keys[idx].octave;
        if (lvl < pred - 1 || lvl > pred) continue;
        const int dist = descriptor_distance(d, KF.desc.data() + idx * 32);
        if (dist < bestDist) {
            bestDist = dist;
            bestIdx = (int)idx;
        }
    }
}

}  // namespace

// Rcw, tcw, Ow from a 4x4 float pose (sim3 = 0: Tcw, KeyFrame::SetPose's
// Ow = -Rcw^T tcw) or similarity (sim3 = 1: the Scw decomposition of
// src/ORBmatcher.cc:1145-1149).
void pose_parts(const float* T, int sim3, float* R, float* t, float* Ow)
{
    if (sim3) {
        const float srow[3] = {T[0], T[1], T[2]};
        const float scw = (float)std::sqrt(dot3(srow, srow));
        const double inv = 1.0 / (double)scw;
        for (int r = 0; r < 3; r++) {
            for (int c = 0; c < 3; c++) R[3 * r + c] = (float)((double)T[4 * r + c] * inv);
            t[r] = (float)((double)T[4 * r + 3] * inv);
        }
    } else {
        for (int r = 0; r < 3; r++) {
            for (int c = 0; c < 3; c++) R[3 * r + c] = T[4 * r + c];
            t[r] = T[4 * r + 3];
        }
    }
    for (int c = 0; c < 3; c++) Ow[c] = -(R[c] * t[0] + R[3 + c] * t[1] + R[6 + c] * t[2]);
}

// The state-free part of ORBmatcher::Fuse (both overloads) for every map
// point: geometric gates, predicted level, best keypoint in the radius.
void fuse_candidates(const FrameRef& KF, const float* cam, int n_mp, const float* pos, const float* normal,
                     const float* dmin, const float* dmax, const uint8_t* desc, const float* T, int sim3, float th,
                     int32_t* best_idx, int32_t* best_dist)
{
    float R[9], t[3], Ow[3];
    pose_parts(T, sim3, R, t, Ow);
    const int nMaxLevel = (int)KF.scaleFactors.size() - 1;
    for (int m = 0; m < n_mp; m++) {
        best_idx[m] = -1;
        best_dist[m] = INT_MAX;
        const float* Xw = pos + 3 * m;
        float p3Dc[3];
        xform(R, t, Xw, p3Dc);
        if (p3Dc[2] < 0.0f) continue;
        // Fuse(KF, vpMapPoints): 1/z in float (:1050); Fuse(KF, Scw): 1.0/z in double (:1179)
        const float invz = sim3 ? (float)(1.0 / (double)p3Dc[2]) : 1 / p3Dc[2];
        const float x = p3Dc[0] * invz, y = p3Dc[1] * invz;
        const float u = cam[0] * x + cam[2], v = cam[1] * y + cam[3];
        if (!(u >= KF.minX && u < KF.maxX && v >= KF.minY && v < KF.maxY)) continue;   // KeyFrame::IsInImage
        const float maxDistance = dmax[m], minDistance = dmin[m];
        const float PO[3] = {Xw[0] - Ow[0], Xw[1] - Ow[1], Xw[2] - Ow[2]};
        const float dist3D = norm3(PO);
        if (dist3D < minDistance || dist3D > maxDistance) continue;
        if (dot3(PO, normal + 3 * m) < 0.5 * dist3D) continue;
        const float ratio = dist3D / minDistance;
        const int nPredictedLevel = std::min(predicted_level(KF.scaleFactors, ratio), nMaxLevel);
        const float radius = th * KF.scaleFactors[nPredictedLevel];
        int bi, bd;
        best_in_area(KF, u, v, radius, nPredictedLevel, desc + (size_t)m * 32, bi, bd);
        best_idx[m] = bi;
        best_dist[m] = bd;
    }
}

// ORBmatcher::SearchBySim3 (src/ORBmatcher.cc:1267-1505).  prior12 per KF1
// keypoint: -2 no match (vpMatches12[i] == NULL), -1 matched to a map point
// not observed in KF2, >= 0 its index in KF2.  new12 (out): the KF2 index
// matched by this call, or -1.
int search_by_sim3(const FrameRef& K1, const FrameRef& K2, const float* cam, const float* pos1, const float* dmin1,
                   const float* dmax1, const uint8_t* desc1, const uint8_t* valid1, const float* pos2,
                   const float* dmin2, const float* dmax2, const uint8_t* desc2, const uint8_t* valid2,
                   const float* T1w, const float* T2w, float s12, const float* R12, const float* t12, float th,
                   const int32_t* prior12, int32_t* new12)
{
    const int N1 = (int)K1.keys.size(), N2 = (int)K2.keys.size();
    float R1w[9], t1w[3], R2w[9], t2w[3], sR12[9], sR21[9], t21[3];
    for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 3; c++) {
            R1w[3 * r + c] = T1w[4 * r + c];
            R2w[3 * r + c] = T2w[4 * r + c];
        }
        t1w[r] = T1w[4 * r + 3];
        t2w[r] = T2w[4 * r + 3];
    }
    const double inv_s = 1.0 / (double)s12;
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) {
            sR12[3 * r + c] = (float)((double)s12 * (double)R12[3 * r + c]);   // s12*R12
            sR21[3 * r + c] = (float)(inv_s * (double)R12[3 * c + r]);         // (1.0/s12)*R12.t()
        }
    for (int r = 0; r < 3; r++) t21[r] = -(sR21[3 * r] * t12[0] + sR21[3 * r + 1] * t12[1] + sR21[3 * r + 2] * t12[2]);
    std::vector<uint8_t> already1(N1, 0), already2(N2, 0);
    for (int i = 0; i < N1; i++) {
        if (prior12[i] == -2) continue;
        already1[i] = 1;
        if (prior12[i] >= 0 && prior12[i] < N2) already2[prior12[i]] = 1;
    }
    std::vector<int> match1(N1, -1), match2(N2, -1);
    auto search = [&](const FrameRef& Kd, const float* pos, const float* dmin, const float* dmax,
                      const uint8_t* desc, const float* Rw, const float* tw, const float* sR, const float* tt,
                      int i) -> int {
        float pc1[3], pc2[3];
        xform(Rw, tw, pos + 3 * i, pc1);
        xform(sR, tt, pc1, pc2);
        if (pc2[2] < 0.0) return -1;
        const float invz = (float)(1.0 / (double)pc2[2]);
        const float x = pc2[0] * invz, y = pc2[1] * invz;
        const float u = cam[0] * x + cam[2], v = cam[1] * y + cam[3];
        if (!(u >= Kd.minX && u < Kd.maxX && v >= Kd.minY && v < Kd.maxY)) return -1;
        const float maxDistance = dmax[i], minDistance = dmin[i];
        const float dist3D = norm3(pc2);
        if (dist3D < minDistance || dist3D > maxDistance) return -1;
        const float ratio = dist3D / minDistance;
        const int pred = std::min(predicted_level(Kd.scaleFactors, ratio), (int)Kd.scaleFactors.size() - 1);
        const float radius = th * Kd.scaleFactors[pred];
        int bi, bd;
        best_in_area(Kd, u, v, radius, pred, desc + (size_t)i * 32, bi, bd);
        return bd <= TH_HIGH ? bi : -1;
    };
    for (int i1 = 0; i1 < N1; i1++) {
        if (!valid1[i1] || already1[i1]) continue;
        match1[i1] = search(K2, pos1, dmin1, dmax1, desc1, R1w, t1w, sR21, t21, i1);
    }
    for (int i2 = 0; i2 < N2; i2++) {
        if (!valid2[i2] || already2[i2]) continue;
        match2[i2] = search(K1, pos2, dmin2, dmax2, desc2, R2w, t2w, sR12, t12, i2);
    }
    int nFound = 0;
    for (int i1 = 0; i1 < N1; i1++) {
        new12[i1] = -1;
        const int idx2 = match1[i1];
        if (idx2 >= 0 && match2[idx2] == i1) {
            new12[i1] = idx2;
            nFound++;
        }
    }
    return nFound;
}

// ORBmatcher::SearchByProjection(KeyFrame*, Scw, vpPoints, vpMatched, th)
// (src/ORBmatcher.cc:286-407).  matched: per KF keypoint, the vpPoints
// index assigned (or any value >= 0 for an entry already set), -1 empty.
int search_by_projection_kf_sim3(const FrameRef& KF, const float* cam, int n_mp, const float* pos,
                                 const float* normal, const float* dmin, const float* dmax, const uint8_t* desc,
                                 const uint8_t* skip, const float* Scw, int th, int32_t* matched)
{
    float R[9], t[3], Ow[3];
    pose_parts(Scw, 1, R, t, Ow);
    const int nMaxLevel = (int)KF.scaleFactors.size() - 1;
    int nmatches = 0;
    for (int m = 0; m < n_mp; m++) {
        if (skip[m]) continue;   // isBad() || spAlreadyFound.count(pMP)
        const float* Xw = pos + 3 * m;
        float p3Dc[3];
        xform(R, t, Xw, p3Dc);
        if (p3Dc[2] < 0.0) continue;
        const float invz = 1 / p3Dc[2];
        const float x = p3Dc[0] * invz, y = p3Dc[1] * invz;
        const float u = cam[0] * x + cam[2], v = cam[1] * y + cam[3];
        if (!(u >= KF.minX && u < KF.maxX && v >= KF.minY && v < KF.maxY)) continue;
        const float maxDistance = dmax[m], minDistance = dmin[m];
        const float PO[3] = {Xw[0] - Ow[0], Xw[1] - Ow[1], Xw[2] - Ow[2]};
        const float dist = norm3(PO);
        if (dist < minDistance || dist > maxDistance) continue;
        if (dot3(PO, normal + 3 * m) < 0.5 * dist) continue;
        const float ratio = dist / minDistance;
        const int pred = std::min(predicted_level(KF.scaleFactors, ratio), nMaxLevel);
        const float radius = th * KF.scaleFactors[pred];
        int bestDist = INT_MAX, bestIdx = -1;
        for (size_t idx : KF.featuresInArea(u, v, radius, -1, -1)) {
            if (matched[idx] >= 0) continue;
            const int lvl = KF.keys[idx].octave;
            if (lvl < pred - 1 || lvl > pred) continue;
            const int d = descriptor_distance(desc + (size_t)m * 32, KF.desc.data() + idx * 32);
            if (d < bestDist) {
                bestDist = d;
                bestIdx = (int)idx;
            }
        }
        if (bestDist <= TH_LOW) {
            matched[bestIdx] = m;
            nmatches++;
        }
    }
    return nmatches;
}

// ORBmatcher::SearchByProjection(Frame&, KeyFrame*, sAlreadyFound, th,
// ORBdist) (src/ORBmatcher.cc:1622-1746).  kf_valid: pMP && !isBad() &&
// !sAlreadyFound.count(pMP); f_assigned: CurrentFrame.mvpMapPoints[i].
// matches_f: the KF keypoint whose map point this call assigns, or -1.
int search_by_projection_frame_kf(const FrameRef& F, const FrameRef& KF, const float* cam, const float* pos,
                                  const float* dmin, const uint8_t* desc, const uint8_t* kf_valid,
                                  const uint8_t* f_assigned, const float* Tcw, float th, int ORBdist, bool checkOri,
                                  int32_t* matches_f)
{
    float R[9], t[3], Ow[3];
    pose_parts(Tcw, 0, R, t, Ow);
    const int NF = (int)F.keys.size();
    std::vector<uint8_t> taken(f_assigned, f_assigned + NF);
    for (int i = 0; i < NF; i++) matches_f[i] = -1;
    std::vector<int> rotHist[30];
    int nmatches = 0;
    const int nLevels = (int)F.scaleFactors.size();
    for (int i = 0; i < (int)KF.keys.size(); i++) {
        if (!kf_valid[i]) continue;
        const float* Xw = pos + 3 * i;
        float x3Dc[3];
        xform(R, t, Xw, x3Dc);
        const float xc = x3Dc[0], yc = x3Dc[1];
        const float invzc = (float)(1.0 / (double)x3Dc[2]);
        const float u = cam[0] * xc * invzc + cam[2];
        const float v = cam[1] * yc * invzc + cam[3];
        if (u < F.minX || u > F.maxX) continue;
        if (v < F.minY || v > F.maxY) continue;
        const float minDistance = dmin[i];
        const float PO[3] = {Xw[0] - Ow[0], Xw[1] - Ow[1], Xw[2] - Ow[2]};
        const float dist3D = norm3(PO);
        const float ratio = dist3D / minDistance;
        const int pred = std::min(predicted_level(F.scaleFactors, ratio), nLevels - 1);
        const float radius = th * F.scaleFactors[pred];
        const std::vector<size_t> idx2 = F.featuresInArea(u, v, radius, pred - 1, pred + 1);
        if (idx2.empty()) continue;
        int bestDist = INT_MAX, bestIdx2 = -1;
        for (size_t i2 : idx2) {
            if (taken[i2]) continue;
            const int d = descriptor_distance(desc + (size_t)i * 32, F.desc.data() + i2 * 32);
            if (d < bestDist) {
                bestDist = d;
                bestIdx2 = (int)i2;
            }
        }
        if (bestDist <= ORBdist) {
            taken[bestIdx2] = 1;
            matches_f[bestIdx2] = i;
            nmatches++;
            if (checkOri) {
                const float factor = 1.0f / 30;
                float rot = KF.keys[i].angle - F.keys[bestIdx2].angle;
                if (rot < 0.0) rot += 360.0f;
                int bin = (int)std::round(rot * factor);
                if (bin == 30) bin = 0;
                rotHist[bin].push_back(bestIdx2);
            }
        }
    }
    if (checkOri) {
        int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
        for (int b = 0; b < 30; b++) {   // ComputeThreeMaxima (:1748-1789)
            const int s = (int)rotHist[b].size();
            if (s > max1) {
                max3 = max2; max2 = max1; max1 = s;
                ind3 = ind2; ind2 = ind1; ind1 = b;
            } else if (s > max2) {
                max3 = max2; max2 = s;
                ind3 = ind2; ind2 = b;
            } else if (s > max3) {
                max3 = s;
                ind3 = b;
            }
        }
        if (max2 < 0.1f * (float)max1) {
            ind2 = -1;
            ind3 = -1;
        } else if (max3 < 0.1f * (float)max1) {
            ind3 = -1;
        }
        for (int b = 0; b < 30; b++) {
            if (b == ind1 || b == ind2 || b == ind3) continue;
            for (int k : rotHist[b]) {
                matches_f[k] = -1;
                nmatches--;
            }
        }
    }
    return nmatches;
}

// MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cc:185-250): the
// descriptor with the least median distance to the others.
int distinctive_descriptor(const uint8_t* desc, int N)
{
    if (N <= 0) return -1;
    std::vector<int> D((size_t)N * N, 0);
    for (int i = 0; i < N; i++)
        for (int j = i + 1; j < N; j++) {
            const int d = descriptor_distance(desc + (size_t)i * 32, desc + (size_t)j * 32);
            D[(size_t)i * N + j] = d;
            D[(size_t)j * N + i] = d;
        }
    int BestMedian = INT_MAX, BestIdx = 0;
    for (int i = 0; i < N; i++) {
        std::vector<int> v(D.begin() + (size_t)i * N, D.begin() + (size_t)(i + 1) * N);
        std::sort(v.begin(), v.end());
        const int median = v[(size_t)(0.5 * (N - 1))];
        if (median < BestMedian) {
            BestMedian = median;
            BestIdx = i;
        }
    }
    return BestIdx;
}

}  // namespace orbref

using namespace orbref;

static void frame_ref(const orbx_frame_view* v, FrameRef& F)
{
    F.build(reinterpret_cast<const KeyPoint*>(v->keys_un), v->desc, v->n, v->min_x, v->max_x, v->min_y, v->max_y,
            v->nlevels, v->scale_factor);
}

extern "C" int orbx_ref_fuse_candidates(const orbx_frame_view* KF, const float* cam, int n_mp, const float* pos,
                                        const float* normal, const float* dmin, const float* dmax,
                                        const uint8_t* desc, const float* T, int sim3, float th, int32_t* best_idx,
                                        int32_t* best_dist)
{
    static thread_local FrameRef F;
    frame_ref(KF, F);
    fuse_candidates(F, cam, n_mp, pos, normal, dmin, dmax, desc, T, sim3, th, best_idx, best_dist);
    return ORBX_OK;
}

extern "C" int orbx_ref_search_by_sim3(const orbx_frame_view* KF1, const orbx_frame_view* KF2, const float* cam,
                                       const float* pos1, const float* dmin1, const float* dmax1,
                                       const uint8_t* desc1, const uint8_t* valid1, const float* pos2,
                                       const float* dmin2, const float* dmax2, const uint8_t* desc2,
                                       const uint8_t* valid2, const float* T1w, const float* T2w, float s12,
                                       const float* R12, const float* t12, float th, const int32_t* prior12,
                                       int32_t* new12, int* n_found)
{
    static thread_local FrameRef A, B;
    frame_ref(KF1, A);
    frame_ref(KF2, B);
    *n_found = search_by_sim3(A, B, cam, pos1, dmin1, dmax1, desc1, valid1, pos2, dmin2, dmax2, desc2, valid2, T1w,
                              T2w, s12, R12, t12, th, prior12, new12);
    return ORBX_OK;
}

extern "C" int orbx_ref_distinctive_descriptors(int n_mp, const int32_t* obs_ptr, const uint8_t* desc,
                                                int32_t* best)
{
    for (int m = 0; m < n_mp; m++)
        best[m] = distinctive_descriptor(desc + (size_t)obs_ptr[m] * 32, obs_ptr[m + 1] - obs_ptr[m]);
    return ORBX_OK;
}

extern "C" int orbx_ref_search_by_projection_kf_sim3(const orbx_frame_view* KF, const float* cam, int n_mp,
                                                     const float* pos, const float* normal, const float* dmin,
                                                     const float* dmax, const uint8_t* desc, const uint8_t* skip,
                                                     const float* Scw, int th, int32_t* matched, int* n_matches)
{
    static thread_local FrameRef F;
    frame_ref(KF, F);
    *n_matches = search_by_projection_kf_sim3(F, cam, n_mp, pos, normal, dmin, dmax, desc, skip, Scw, th, matched);
    return ORBX_OK;
}

extern "C" int orbx_ref_search_by_projection_frame_kf(const orbx_frame_view* Fv, const orbx_frame_view* KFv,
                                                      const float* cam, const float* pos, const float* dmin,
                                                      const uint8_t* desc, const uint8_t* kf_valid,
                                                      const uint8_t* f_assigned, const float* Tcw, float th,
                                                      int orb_dist, int check_ori, int32_t* matches_f,
                                                      int* n_matches)
{
    static thread_local FrameRef F, K;
    frame_ref(Fv, F);
    frame_ref(KFv, K);
    *n_matches = search_by_projection_frame_kf(F, K, cam, pos, dmin, desc, kf_valid, f_assigned, Tcw, th, orb_dist,
                                               check_ori != 0, matches_f);
    return ORBX_OK;
}
