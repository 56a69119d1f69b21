// Exercises the C++ adapter (orbx_adapters.hpp) the way ORB-SLAM's Tracking
// and LocalMapping would: extract two frames of a shifted synthetic image,
// SearchForInitialization between them, brute-force matching, and one local
// BA on a tiny synthetic problem.  Prints one JSON line.  Exit codes: 0 ok,
// 3 device path unavailable (orbx_error), 1 other failure.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "orbx_adapters.hpp"

using namespace ORB_SLAM_AMD;

static std::vector<uint8_t> make_image(int w, int h, int dx, uint32_t seed)
{
    // box-filtered LCG noise + rectangles, shifted by dx columns
    const int W = w + 64;
    std::vector<uint8_t> big((size_t)W * h);
    uint32_t s = seed;
    for (auto& v : big) {
        s = s * 1664525u + 1013904223u;
        v = (uint8_t)(s >> 24);
    }
    std::vector<uint8_t> sm(big.size());
    for (int y = 0; y < h; y++)
        for (int x = 0; x < W; x++) {
            int acc = 0, n = 0;
            for (int j = -2; j <= 2; j++)
                for (int i = -2; i <= 2; i++) {
                    const int yy = y + j, xx = x + i;
                    if (yy >= 0 && yy < h && xx >= 0 && xx < W) {
                        acc += big[(size_t)yy * W + xx];
                        n++;
                    }
                }
            sm[(size_t)y * W + x] = (uint8_t)(acc / n);
        }
    for (int r = 0; r < 120; r++) {
        s = s * 1664525u + 1013904223u;
        const int x0 = (int)(s % (uint32_t)(W - 40)), y0 = (int)((s >> 8) % (uint32_t)(h - 30));
        const uint8_t val = (uint8_t)(s >> 16);
        for (int y = y0; y < y0 + 24; y++)
            for (int x = x0; x < x0 + 36; x++) sm[(size_t)y * W + x] = val;
    }
    std::vector<uint8_t> img((size_t)w * h);
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) img[(size_t)y * w + x] = sm[(size_t)y * W + x + dx];
    return img;
}

int main()
{
    try {
        const int w = 640, h = 480;
        ORBextractor ex(1000, 1.2f, 8, ORBextractor::FAST_SCORE, 20, w, h);
        FrameData F1, F2;
        for (FrameData* F : {&F1, &F2}) {
            const auto img = make_image(w, h, F == &F1 ? 0 : 2, 7);
            ex(img.data(), w, h, w, F->keys_un, F->desc);
            F->max_x = (float)w;
            F->max_y = (float)h;
        }
        ORBmatcher matcher(0.9f, true, ex.context());
        std::vector<Point2f> prev(F1.keys_un.size());
        for (size_t i = 0; i < prev.size(); i++) prev[i] = {F1.keys_un[i].x, F1.keys_un[i].y};
        std::vector<int> m12;
        const int n_init = matcher.SearchForInitialization(F1, F2, prev, m12, 100);
        std::vector<int> mbf;
        const int n_bf = matcher.MatchBruteForce(F1.desc, F2.desc, mbf);
        // tiny BA: 3 keyframes (first fixed) observing 60 points
        LocalBAProblem P;
        const int nk = 3, np = 60;
        for (int k = 0; k < nk; k++) {
            const double ang = 0.02 * k;
            P.pose_q.insert(P.pose_q.end(), {0.0, std::sin(ang / 2), 0.0, std::cos(ang / 2)});
            P.pose_t.insert(P.pose_t.end(), {-0.1 * k + (k ? 0.01 : 0.0), 0.0, 0.0});
            P.pose_fixed.push_back(k == 0);
            P.pose_id.push_back(k);
            P.pose_cam.insert(P.pose_cam.end(), {500.0, 500.0, 320.0, 240.0});
        }
        uint32_t s = 11;
        for (int p = 0; p < np; p++) {
            s = s * 1664525u + 1013904223u;
            const double X = ((s >> 8) % 2000) / 1000.0 - 1.0, Y = ((s >> 4) % 1500) / 1000.0 - 0.75,
                         Z = 3.0 + ((s >> 12) % 2000) / 1000.0;
            P.points.insert(P.points.end(), {X + 0.01, Y - 0.01, Z});
            P.point_id.push_back(nk + p);
            P.point_nobs.push_back(nk);
            for (int k = 0; k < nk; k++) {
                const double ang = 0.02 * k, c = std::cos(ang), sn = std::sin(ang);
                const double xc = c * X + sn * Z - 0.1 * k, yc = Y, zc = -sn * X + c * Z;
                P.edge_point.push_back(p);
                P.edge_pose.push_back(k);
                P.edge_obs.push_back(500.0 * xc / zc + 320.0);
                P.edge_obs.push_back(500.0 * yc / zc + 240.0);
                P.edge_inv_sigma2.push_back(1.0);
            }
        }
        Optimizer::LocalBundleAdjustment(ex.context(), P);
        // PoseOptimization of F2: every other keypoint gets a map point 3-5 m
        // in front of the identity camera; the initial pose is off by 2 cm
        PoseFrame PF;
        PF.keys_un = F2.keys_un;
        PF.fx = PF.fy = 500.f;
        PF.cx = 320.f;
        PF.cy = 240.f;
        float sc = 1.f;
        for (int l = 0; l < 8; l++, sc *= 1.2f) PF.inv_level_sigma2.push_back(1.f / (sc * sc));
        for (size_t i = 0; i < PF.keys_un.size(); i++) {
            const bool mp = (i % 2) == 0;
            PF.has_mp.push_back(mp);
            const float z = 3.f + (float)(i % 7) * 0.3f;
            PF.mp_xyz.insert(PF.mp_xyz.end(), {(PF.keys_un[i].x - 320.f) / 500.f * z,
                                               (PF.keys_un[i].y - 240.f) / 500.f * z, z});
        }
        PF.Tcw[3] = 0.02f;
        const int n_pose_inliers = Optimizer::PoseOptimization(ex.context(), PF);
        int n_mp = 0;
        for (uint8_t m : PF.has_mp) n_mp += m;
        std::printf("{\"n1\": %zu, \"n2\": %zu, \"levels\": %d, \"scale\": %.3f, \"init_matches\": %d, "
                    "\"bf_matches\": %d, \"ba_iterations\": [%d, %d], \"ba_chi2\": [%.6g, %.6g], "
                    "\"pose_inliers\": %d, \"pose_edges\": %d, \"pose_tx\": %.6g}\n",
                    F1.keys_un.size(), F2.keys_un.size(), ex.GetLevels(), ex.GetScaleFactor(), n_init, n_bf,
                    P.stats.iterations[0], P.stats.iterations[1], P.stats.chi2_initial[0], P.stats.chi2_final[1],
                    n_pose_inliers, n_mp, PF.Tcw[3]);
        return 0;
    } catch (const orbx_error& e) {
        std::fprintf(stderr, "%s\n", e.what());
        return 3;
    } catch (const std::exception& e) {
        std::fprintf(stderr, "%s\n", e.what());
        return 1;
    }
}
