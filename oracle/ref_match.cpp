// ORACLE -- TEST INFRASTRUCTURE ONLY (see ref_common.h).
//
// CPU restatement of the ORBmatcher searches on the hot path
// (src/ORBmatcher.cc) and of the Frame grid they query (src/Frame.cc).
// Map-point state is passed as flat arrays; the sequential greedy order of the
// reference loops is kept exactly.
#include "ref_common.h"

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstring>

namespace orbref {

namespace {
const int TH_HIGH = 100;      // src/ORBmatcher.cc:40
const int TH_LOW = 50;        // :41
const int HISTO_LENGTH = 30;  // :42
const int GRID_COLS = 64;     // include/Frame.h:35
const int GRID_ROWS = 48;     // include/Frame.h:36

// ORBmatcher::ComputeThreeMaxima (src/ORBmatcher.cc:1748-1789)
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

// Rotation-histogram bin (e.g. src/ORBmatcher.cc:668-673).  factor is
// 1/HISTO_LENGTH, so only bins 0..12 are reachable; the reference bug is kept.
int rot_bin(float angle1, float angle2)
{
    const float factor = 1.0f / HISTO_LENGTH;
    float rot = angle1 - angle2;
    if (rot < 0.0) rot += 360.0f;
    int bin = (int)std::round(rot * factor);
    if (bin == HISTO_LENGTH) bin = 0;
    return bin;
}

// x3Dc = R*x3Dw + t in float, components summed left to right.
void transform(const float* T, const float* X, float* out)
{
    for (int r = 0; r < 3; r++) out[r] = T[4 * r] * X[0] + T[4 * r + 1] * X[1] + T[4 * r + 2] * X[2] + T[4 * r + 3];
}
}  // namespace

// ORBmatcher::DescriptorDistance (src/ORBmatcher.cc:1794-1810), SWAR popcount.
int descriptor_distance(const uint8_t* a, const uint8_t* b)
{
    int dist = 0;
    for (int i = 0; i < 8; i++) {
        uint32_t pa, pb;
        std::memcpy(&pa, a + 4 * i, 4);
        std::memcpy(&pb, b + 4 * i, 4);
        uint32_t v = pa ^ pb;
        v = v - ((v >> 1) & 0x55555555u);
        v = (v & 0x33333333u) + ((v >> 2) & 0x33333333u);
        dist += (int)((((v + (v >> 4)) & 0xF0F0F0Fu) * 0x1010101u) >> 24);
    }
    return dist;
}

// Frame constructor grid part (src/Frame.cc:76-77, 94-122) and PosInGrid
// (:266-276).  mvKeysUn == mvKeys (distortion k1 == 0, :290-294).
void FrameRef::build(const KeyPoint* k, const uint8_t* d, int n, float minx, float maxx,
                     float miny, float maxy, int nlevels, float scale)
{
    keys.assign(k, k + n);
    desc.assign(d, d + (size_t)n * 32);
    minX = minx; maxX = maxx; minY = miny; maxY = maxy;
    gridWInv = static_cast<float>(GRID_COLS) / static_cast<float>(maxX - minX);
    gridHInv = static_cast<float>(GRID_ROWS) / static_cast<float>(maxY - minY);
    scaleFactors.assign(nlevels, 1.0f);
    for (int i = 1; i < nlevels; i++) scaleFactors[i] = scaleFactors[i - 1] * scale;
    for (int i = 0; i < GRID_COLS; i++)
        for (int j = 0; j < GRID_ROWS; j++) grid[i][j].clear();
    for (int i = 0; i < n; i++) {
        const int posX = (int)std::round((keys[i].x - minX) * gridWInv);
        const int posY = (int)std::round((keys[i].y - minY) * gridHInv);
        if (posX < 0 || posX >= GRID_COLS || posY < 0 || posY >= GRID_ROWS) continue;
        grid[posX][posY].push_back(i);
    }
}

// Frame::GetFeaturesInArea (src/Frame.cc:199-264)
std::vector<size_t> FrameRef::featuresInArea(float x, float y, float r, int minLevel, int maxLevel) const
{
    std::vector<size_t> idx;
    int nMinCellX = (int)std::floor((x - minX - r) * gridWInv);
    nMinCellX = std::max(0, nMinCellX);
    if (nMinCellX >= GRID_COLS) return idx;
    int nMaxCellX = (int)std::ceil((x - minX + r) * gridWInv);
    nMaxCellX = std::min(GRID_COLS - 1, nMaxCellX);
    if (nMaxCellX < 0) return idx;
    int nMinCellY = (int)std::floor((y - minY - r) * gridHInv);
    nMinCellY = std::max(0, nMinCellY);
    if (nMinCellY >= GRID_ROWS) return idx;
    int nMaxCellY = (int)std::ceil((y - minY + r) * gridHInv);
    nMaxCellY = std::min(GRID_ROWS - 1, nMaxCellY);
    if (nMaxCellY < 0) return idx;
    bool bCheckLevels = true, bSameLevel = false;
    if (minLevel == -1 && maxLevel == -1) bCheckLevels = false;
    else if (minLevel == maxLevel) bSameLevel = true;
    for (int ix = nMinCellX; ix <= nMaxCellX; ix++) {
        for (int iy = nMinCellY; iy <= nMaxCellY; iy++) {
            const std::vector<int>& cell = grid[ix][iy];
            for (int j : cell) {
                const KeyPoint& kp = keys[j];
                if (bCheckLevels && !bSameLevel) {
                    if (kp.octave < minLevel || kp.octave > maxLevel) continue;
                } else if (bSameLevel) {
                    if (kp.octave != minLevel) continue;
                }
                if (std::fabs(kp.x - x) > r || std::fabs(kp.y - y) > r) continue;
                idx.push_back(j);
            }
        }
    }
    return idx;
}

// ORBmatcher::SearchForInitialization (src/ORBmatcher.cc:598-713)
int search_for_initialization(const FrameRef& F1, const FrameRef& F2,
                              std::vector<float>& prevMatched, std::vector<int>& matches12,
                              int windowSize, float nnratio, bool checkOri)
{
    int nmatches = 0;
    const int N1 = (int)F1.keys.size(), N2 = (int)F2.keys.size();
    matches12.assign(N1, -1);
    std::vector<int> rotHist[HISTO_LENGTH];
    std::vector<int> vMatchedDistance(N2, INT_MAX);
    std::vector<int> vnMatches21(N2, -1);
    for (int i1 = 0; i1 < N1; i1++) {
        const KeyPoint& kp1 = F1.keys[i1];
        const int level1 = kp1.octave;
        if (level1 > 0) continue;
        std::vector<size_t> v2 = F2.featuresInArea(prevMatched[2 * i1], prevMatched[2 * i1 + 1],
                                                   (float)windowSize, level1, level1);
        if (v2.empty()) continue;
        const uint8_t* d1 = &F1.desc[(size_t)i1 * 32];
        int bestDist = INT_MAX, bestDist2 = INT_MAX, bestIdx2 = -1;
        for (size_t i2 : v2) {
            const int dist = descriptor_distance(d1, &F2.desc[i2 * 32]);
            if (vMatchedDistance[i2] <= dist) continue;
            if (dist < bestDist) {
                bestDist2 = bestDist;
                bestDist = dist;
                bestIdx2 = (int)i2;
            } else if (dist < bestDist2) {
                bestDist2 = dist;
            }
        }
        if (bestDist <= TH_LOW) {
            if (bestDist < (float)bestDist2 * nnratio) {
                if (vnMatches21[bestIdx2] >= 0) {
                    matches12[vnMatches21[bestIdx2]] = -1;
                    nmatches--;
                }
                matches12[i1] = bestIdx2;
                vnMatches21[bestIdx2] = i1;
                vMatchedDistance[bestIdx2] = bestDist;
                nmatches++;
                if (checkOri) rotHist[rot_bin(F1.keys[i1].angle, F2.keys[bestIdx2].angle)].push_back(i1);
            }
        }
    }
    if (checkOri) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        three_maxima(rotHist, HISTO_LENGTH, ind1, ind2, ind3);
        for (int i = 0; i < HISTO_LENGTH; i++) {
            if (i == ind1 || i == ind2 || i == ind3) continue;
            for (int idx1 : rotHist[i]) {
                if (matches12[idx1] >= 0) {
                    matches12[idx1] = -1;
                    nmatches--;
                }
            }
        }
    }
    for (int i1 = 0; i1 < N1; i1++) {
        if (matches12[i1] >= 0) {
            prevMatched[2 * i1] = F2.keys[matches12[i1]].x;
            prevMatched[2 * i1 + 1] = F2.keys[matches12[i1]].y;
        }
    }
    return nmatches;
}

// ORBmatcher::WindowSearch (src/ORBmatcher.cc:409-516)
int window_search(const FrameRef& F1, const FrameRef& F2, const uint8_t* f1_mp,
                  int windowSize, int minLevel, int maxLevel, float nnratio,
                  bool checkOri, std::vector<int>& matches21)
{
    int nmatches = 0;
    const int N1 = (int)F1.keys.size(), N2 = (int)F2.keys.size();
    matches21.assign(N2, -1);  // vpMapPointMatches2 (as F1 index) == vnMatches21
    std::vector<int> rotHist[HISTO_LENGTH];
    const bool bMinLevel = minLevel > 0;
    const bool bMaxLevel = maxLevel < INT_MAX;
    for (int i1 = 0; i1 < N1; i1++) {
        if (!f1_mp[i1]) continue;
        const KeyPoint& kp1 = F1.keys[i1];
        const int level1 = kp1.octave;
        if (bMinLevel && level1 < minLevel) continue;
        if (bMaxLevel && level1 > maxLevel) continue;
        std::vector<size_t> v2 = F2.featuresInArea(kp1.x, kp1.y, (float)windowSize, level1, level1);
        if (v2.empty()) continue;
        const uint8_t* d1 = &F1.desc[(size_t)i1 * 32];
        int bestDist = INT_MAX, bestDist2 = INT_MAX, bestIdx2 = -1;
        for (size_t i2 : v2) {
            if (matches21[i2] >= 0) continue;
            const int dist = descriptor_distance(d1, &F2.desc[i2 * 32]);
            if (dist < bestDist) {
                bestDist2 = bestDist;
                bestDist = dist;
                bestIdx2 = (int)i2;
            } else if (dist < bestDist2) {
                bestDist2 = dist;
            }
        }
        if (bestDist <= bestDist2 * nnratio && bestDist <= TH_HIGH) {
            matches21[bestIdx2] = i1;
            nmatches++;
            rotHist[rot_bin(F1.keys[i1].angle, F2.keys[bestIdx2].angle)].push_back(bestIdx2);
        }
    }
    if (checkOri) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        three_maxima(rotHist, HISTO_LENGTH, ind1, ind2, ind3);
        for (int i = 0; i < HISTO_LENGTH; i++) {
            if (i != ind1 && i != ind2 && i != ind3) {
                for (int i2 : rotHist[i]) {
                    matches21[i2] = -1;
                    nmatches--;
                }
            }
        }
    }
    return nmatches;
}

// ORBmatcher::SearchByProjection(Frame&, Frame&, int, vector<MapPoint*>&)
// (src/ORBmatcher.cc:519-594).  matches21 holds only assignments made here.
int search_by_projection_pair(const FrameRef& F1, const FrameRef& F2,
                              const float* mp_xyz, const uint8_t* mp_valid,
                              const uint8_t* f2_assigned, const float* Tcw,
                              const float* cam, int windowSize, float nnratio,
                              std::vector<int>& matches21)
{
    int nmatches = 0;
    const int N1 = (int)F1.keys.size(), N2 = (int)F2.keys.size();
    matches21.assign(N2, -1);
    std::vector<uint8_t> taken(f2_assigned, f2_assigned + N2);
    for (int i1 = 0; i1 < N1; i1++) {
        if (!mp_valid[i1]) continue;
        const int level1 = F1.keys[i1].octave;
        float xc[3];
        transform(Tcw, &mp_xyz[3 * i1], xc);
        const float invzc = (float)(1.0 / xc[2]);
        const float u2 = cam[0] * xc[0] * invzc + cam[2];
        const float v2 = cam[1] * xc[1] * invzc + cam[3];
        std::vector<size_t> vi = F2.featuresInArea(u2, v2, (float)windowSize, level1, level1);
        if (vi.empty()) continue;
        const uint8_t* d1 = &F1.desc[(size_t)i1 * 32];
        int bestDist = INT_MAX, bestDist2 = INT_MAX, bestIdx2 = -1;
        for (size_t i2 : vi) {
            if (taken[i2]) continue;
            const int dist = descriptor_distance(d1, &F2.desc[i2 * 32]);
            if (dist < bestDist) {
                bestDist2 = bestDist;
                bestDist = dist;
                bestIdx2 = (int)i2;
            } else if (dist < bestDist2) {
                bestDist2 = dist;
            }
        }
        if (static_cast<float>(bestDist) <= static_cast<float>(bestDist2) * nnratio && bestDist <= TH_HIGH) {
            taken[bestIdx2] = 1;
            matches21[bestIdx2] = i1;
            nmatches++;
        }
    }
    return nmatches;
}

// ORBmatcher::SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame,
// float th) (src/ORBmatcher.cc:1507-1620).
int search_by_projection_motion(const FrameRef& Cur, const FrameRef& Last,
                                const float* mp_xyz, const uint8_t* mp_valid,
                                const uint8_t* cur_assigned, const float* Tcw,
                                const float* cam, float th, bool checkOri,
                                std::vector<int>& matchesCur)
{
    int nmatches = 0;
    const int NL = (int)Last.keys.size(), NC = (int)Cur.keys.size();
    matchesCur.assign(NC, -1);
    std::vector<uint8_t> taken(cur_assigned, cur_assigned + NC);
    std::vector<int> rotHist[HISTO_LENGTH];
    for (int i = 0; i < NL; i++) {
        if (!mp_valid[i]) continue;
        float xc[3];
        transform(Tcw, &mp_xyz[3 * i], xc);
        const float invzc = (float)(1.0 / xc[2]);
        const float u = cam[0] * xc[0] * invzc + cam[2];
        const float v = cam[1] * xc[1] * invzc + cam[3];
        if (u < Cur.minX || u > Cur.maxX) continue;
        if (v < Cur.minY || v > Cur.maxY) continue;
        const int nPredictedOctave = Last.keys[i].octave;
        const float radius = th * Cur.scaleFactors[nPredictedOctave];
        std::vector<size_t> vi = Cur.featuresInArea(u, v, radius, nPredictedOctave - 1, nPredictedOctave + 1);
        if (vi.empty()) continue;
        const uint8_t* dMP = &Last.desc[(size_t)i * 32];
        int bestDist = INT_MAX, bestIdx2 = -1;
        for (size_t i2 : vi) {
            if (taken[i2]) continue;
            const int dist = descriptor_distance(dMP, &Cur.desc[i2 * 32]);
            if (dist < bestDist) {
                bestDist = dist;
                bestIdx2 = (int)i2;
            }
        }
        if (bestDist <= TH_HIGH) {
            taken[bestIdx2] = 1;
            matchesCur[bestIdx2] = i;
            nmatches++;
            if (checkOri) rotHist[rot_bin(Last.keys[i].angle, Cur.keys[bestIdx2].angle)].push_back(bestIdx2);
        }
    }
    if (checkOri) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        three_maxima(rotHist, HISTO_LENGTH, ind1, ind2, ind3);
        for (int i = 0; i < HISTO_LENGTH; i++) {
            if (i != ind1 && i != ind2 && i != ind3) {
                for (int i2 : rotHist[i]) {
                    matchesCur[i2] = -1;
                    nmatches--;
                }
            }
        }
    }
    return nmatches;
}

// ORBmatcher::SearchByProjection(Frame& F, const vector<MapPoint*>&, float th)
// (src/ORBmatcher.cc:49-125) with RadiusByViewingCos (:127-133).
int search_by_projection_local(const FrameRef& F, int n_mp, const uint8_t* in_view,
                               const float* proj_xy, const int32_t* pred_level,
                               const float* view_cos, const uint8_t* mp_desc,
                               const uint8_t* f_assigned, float th, float nnratio,
                               std::vector<int>& matchesF)
{
    int nmatches = 0;
    const int N = (int)F.keys.size();
    matchesF.assign(N, -1);
    std::vector<uint8_t> taken(f_assigned, f_assigned + N);
    const bool bFactor = th != 1.0;
    for (int m = 0; m < n_mp; m++) {
        if (!in_view[m]) continue;
        const int nPredictedLevel = pred_level[m];
        float r = view_cos[m] > 0.998 ? 2.5f : 4.0f;
        if (bFactor) r *= th;
        std::vector<size_t> vi = F.featuresInArea(proj_xy[2 * m], proj_xy[2 * m + 1],
                                                  r * F.scaleFactors[nPredictedLevel],
                                                  nPredictedLevel - 1, nPredictedLevel);
        if (vi.empty()) continue;
        const uint8_t* dMP = &mp_desc[(size_t)m * 32];
        int bestDist = INT_MAX, bestLevel = -1, bestDist2 = INT_MAX, bestLevel2 = -1, bestIdx = -1;
        for (size_t idx : vi) {
            if (taken[idx]) continue;
            const int dist = descriptor_distance(dMP, &F.desc[idx * 32]);
            if (dist < bestDist) {
                bestDist2 = bestDist;
                bestDist = dist;
                bestLevel2 = bestLevel;
                bestLevel = F.keys[idx].octave;
                bestIdx = (int)idx;
            } else if (dist < bestDist2) {
                bestLevel2 = F.keys[idx].octave;
                bestDist2 = dist;
            }
        }
        if (bestDist <= TH_HIGH) {
            if (bestLevel == bestLevel2 && bestDist > nnratio * bestDist2) continue;
            taken[bestIdx] = 1;
            matchesF[bestIdx] = m;
            nmatches++;
        }
    }
    return nmatches;
}

// Frame::isInFrustum (src/Frame.cc:136-197).  cv::Mat arithmetic as OpenCV
// 2.4 evaluates it (un-vendored, restated; the same conventions as
// ref_proj.cpp): Pc = mRcw*P + mtcw through gemm's small-matrix path (float
// products summed left to right, + t); cv::norm and Mat::dot of float
// vectors accumulate in double.  Rcw / tcw / Ow are the Frame's own members.
bool is_in_frustum(const FrameRef& F, const float* Rcw, const float* tcw, const float* Ow, const float* cam,
                   const float* P, const float* Pn, float minDistance, float maxDistance, float viewingCosLimit,
                   float& u_out, float& v_out, int& level_out, float& cos_out)
{
    float Pc[3];
    for (int r = 0; r < 3; r++) Pc[r] = Rcw[3 * r] * P[0] + Rcw[3 * r + 1] * P[1] + Rcw[3 * r + 2] * P[2] + tcw[r];
    if (Pc[2] < 0.0) return false;                                   // :150-151
    const float invz = (float)(1.0 / Pc[2]);                         // :154
    const float u = cam[0] * Pc[0] * invz + cam[2];
    const float v = cam[1] * Pc[1] * invz + cam[3];
    if (u < F.minX || u > F.maxX) return false;                      // :158-161
    if (v < F.minY || v > F.maxY) return false;
    const float PO[3] = {P[0] - Ow[0], P[1] - Ow[1], P[2] - Ow[2]};   // :166
    double s = 0;
    for (int i = 0; i < 3; i++) s += (double)PO[i] * PO[i];
    const float dist = (float)std::sqrt(s);                          // cv::norm
    if (dist < minDistance || dist > maxDistance) return false;       // :169-170
    double d = 0;
    for (int i = 0; i < 3; i++) d += (double)PO[i] * Pn[i];           // Mat::dot
    const float viewCos = (float)(d / dist);                         // :175
    if (viewCos < viewingCosLimit) return false;
    const float ratio = dist / minDistance;                          // :181
    int level = (int)(std::lower_bound(F.scaleFactors.begin(), F.scaleFactors.end(), ratio) - F.scaleFactors.begin());
    if (level >= (int)F.scaleFactors.size()) level = (int)F.scaleFactors.size() - 1;
    u_out = u;
    v_out = v;
    level_out = level;
    cos_out = viewCos;
    return true;
}

// All-pairs best / second (B8 primitive; rule of src/ORBmatcher.cc:640-649).
void hamming_bf(const uint8_t* dA, int nA, const uint8_t* dB, int nB,
                int32_t* best_idx, int32_t* best, int32_t* second)
{
    for (int a = 0; a < nA; a++) {
        int b1 = INT_MAX, b2 = INT_MAX, bi = -1;
        for (int b = 0; b < nB; b++) {
            const int d = descriptor_distance(dA + (size_t)a * 32, dB + (size_t)b * 32);
            if (d < b1) {
                b2 = b1;
                b1 = d;
                bi = b;
            } else if (d < b2) {
                b2 = d;
            }
        }
        best_idx[a] = bi;
        best[a] = b1;
        second[a] = b2;
    }
}

}  // namespace orbref
