// C++ adapter over the orbx C ABI (include/orbx.h) that keeps the reference's
// class and function signatures for the hot path, so ORB-SLAM's callers
// (Frame, Tracking, LocalMapping) need only a type swap.  OpenCV-free: images
// are (pointer, w, h, stride) and descriptors N x 32 byte buffers; the
// cv::Mat glue a maintainer adds inside the reference is in INTEGRATION.md.
//
//   ORB_SLAM_AMD::ORBextractor   <- ORB_SLAM::ORBextractor   include/ORBextractor.h:32-77
//   ORB_SLAM_AMD::ORBmatcher     <- ORB_SLAM::ORBmatcher     include/ORBmatcher.h:37-107
//   ORB_SLAM_AMD::Optimizer      <- ORB_SLAM::Optimizer::LocalBundleAdjustment
//                                                           include/Optimizer.h:42
//
// Error behaviour: the reference has no error codes.  Like the reference, an
// empty image returns without touching the outputs (src/ORBextractor.cc:
// 721-722); every other failure of the device path throws orbx_error (there
// is no CPU fallback).
#pragma once

#include <cstdint>
#include <climits>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/orbx.h"

namespace ORB_SLAM_AMD {

struct orbx_error : std::runtime_error {
    int code;
    orbx_error(int c, const char* where)
        : std::runtime_error(std::string(where) + ": orbx error " + std::to_string(c)), code(c) {}
};

inline void check(int code, const char* where)
{
    if (code != ORBX_OK) throw orbx_error(code, where);
}

using KeyPoint = orbx_keypoint;   // layout of cv::KeyPoint (28 bytes)

// One device context per calling thread (the reference gives each thread its
// own extractor / matcher instances).
class Context {
public:
    Context(int nfeatures, float scale_factor, int nlevels, int score_type, int fast_th, int max_w, int max_h,
            int max_batch = 1, int device = 0)
    {
        // a library of another ABI revision may have changed a signature this
        // header calls through (include/orbx.h, ORBX_ABI_VERSION)
        if (orbx_abi_version() != ORBX_ABI_VERSION) throw orbx_error(ORBX_ERR_UNSUPPORTED, "orbx_abi_version");
        check(orbx_create(&ctx_, device, nfeatures, scale_factor, nlevels, score_type, fast_th, max_w, max_h, max_batch),
              "orbx_create");
    }
    ~Context() { orbx_destroy(ctx_); }
    Context(const Context&) = delete;
    Context& operator=(const Context&) = delete;
    orbx_ctx* get() const { return ctx_; }

private:
    orbx_ctx* ctx_ = nullptr;
};

// ---------------------------------------------------------------------------
// ORBextractor (src/ORBextractor.cc:457-779)
// ---------------------------------------------------------------------------
class ORBextractor {
public:
    enum { HARRIS_SCORE = 0, FAST_SCORE = 1 };

    ORBextractor(int nfeatures = 1000, float scaleFactor = 1.2f, int nlevels = 8, int scoreType = FAST_SCORE,
                 int fastTh = 20, int max_w = 1920, int max_h = 1080, int device = 0)
        : nfeatures_(nfeatures), ctx_(nfeatures, scaleFactor, nlevels, scoreType, fastTh, max_w, max_h, 1, device)
    {
    }

    // operator()(image, mask, keypoints, descriptors): keypoints cleared and
    // filled; descriptors resized to N*32 bytes (released when N == 0).
    void operator()(const uint8_t* image, int w, int h, size_t stride, std::vector<KeyPoint>& keypoints,
                    std::vector<uint8_t>& descriptors)
    {
        if (image == nullptr || w == 0 || h == 0) return;   // :721-722
        keypoints.resize(nfeatures_);
        descriptors.resize((size_t)nfeatures_ * 32);
        int n = 0;
        check(orbx_extract(ctx_.get(), image, w, h, stride, keypoints.data(), descriptors.data(), nfeatures_, &n),
              "ORBextractor::operator()");
        keypoints.resize(n);
        descriptors.resize((size_t)n * 32);
    }

    // With a mask (any size / content): the reference builds mvMaskPyramid
    // from it (:792-812) but FAST never reads the cell mask (:601-613), so
    // the outputs are those of the unmasked call.
    void operator()(const uint8_t* image, int w, int h, size_t stride, const uint8_t* /*mask*/,
                    std::vector<KeyPoint>& keypoints, std::vector<uint8_t>& descriptors)
    {
        (*this)(image, w, h, stride, keypoints, descriptors);
    }

    int GetLevels() const { return orbx_get_levels(ctx_.get()); }
    float GetScaleFactor() const { return orbx_get_scale_factor(ctx_.get()); }
    std::vector<int> GetFeaturesPerLevel() const
    {
        std::vector<int> v(64);
        v.resize(orbx_get_features_per_level(ctx_.get(), v.data(), 64));
        return v;
    }
    orbx_ctx* context() const { return ctx_.get(); }
    // Match a reference binary built with FMA contraction (GCC -O3
    // -march=native on an FMA host; orbx_set_fp_contract).
    void SetFpContract(bool enable) { check(orbx_set_fp_contract(ctx_.get(), enable ? 1 : 0), "SetFpContract"); }
    // retainBest's std::nth_element as the libstdc++ the reference was built
    // against implements it: gcc48 = GCC 4.6 .. 4.8 (orbx_set_nth_pivot).
    // The constructor leaves the default, GCC 4.6 .. 4.8: the reference
    // documents Ubuntu 12.04 / 14.04 (README.md:46), whose OpenCV 2.4
    // packages were built with those compilers; SetNthElementEra(false)
    // matches an OpenCV built with GCC >= 4.9.
    void SetNthElementEra(bool gcc48)
    {
        check(orbx_set_nth_pivot(ctx_.get(), gcc48 ? ORBX_NTH_PIVOT_GCC48 : ORBX_NTH_PIVOT_GCC49), "SetNthElementEra");
    }

private:
    int nfeatures_;
    Context ctx_;
};

// ---------------------------------------------------------------------------
// Frame data the matchers read (Frame::mvKeysUn, mDescriptors, image bounds,
// scale pyramid: src/Frame.cc:59-122, 320-348).
// ---------------------------------------------------------------------------
struct FrameData {
    std::vector<KeyPoint> keys_un;
    std::vector<uint8_t> desc;   // N x 32
    float min_x = 0, max_x = 0, min_y = 0, max_y = 0;
    int nlevels = 8;
    float scale_factor = 1.2f;

    orbx_frame_view view() const
    {
        orbx_frame_view v;
        v.keys_un = keys_un.data();
        v.desc = desc.data();
        v.n = (int)keys_un.size();
        v.min_x = min_x;
        v.max_x = max_x;
        v.min_y = min_y;
        v.max_y = max_y;
        v.nlevels = nlevels;
        v.scale_factor = scale_factor;
        return v;
    }
};

struct Point2f {
    float x, y;
};

// ---------------------------------------------------------------------------
// ORBmatcher (src/ORBmatcher.cc): the searches on the per-frame hot path.
// ---------------------------------------------------------------------------
class ORBmatcher {
public:
    static const int TH_LOW = 50;
    static const int TH_HIGH = 100;
    static const int HISTO_LENGTH = 30;

    // The matcher needs a device context; share the extractor's or own one.
    explicit ORBmatcher(float nnratio = 0.6f, bool checkOri = true, orbx_ctx* ctx = nullptr)
        : mfNNratio(nnratio), mbCheckOrientation(checkOri), ctx_(ctx)
    {
        if (!ctx_) {
            own_.reset(new Context(1000, 1.2f, 8, 1, 20, 64, 64));
            ctx_ = own_->get();
        }
    }

    // :1794-1810
    static int DescriptorDistance(const uint8_t* a, const uint8_t* b) { return orbx_descriptor_distance(a, b); }

    // :598-713
    int SearchForInitialization(const FrameData& F1, const FrameData& F2, std::vector<Point2f>& vbPrevMatched,
                                std::vector<int>& vnMatches12, int windowSize = 10)
    {
        const orbx_frame_view v1 = F1.view(), v2 = F2.view();
        vnMatches12.assign(v1.n, -1);
        int n = 0;
        check(orbx_search_for_initialization(ctx_, &v1, &v2, reinterpret_cast<float*>(vbPrevMatched.data()),
                                             vnMatches12.data(), windowSize, mfNNratio, mbCheckOrientation, &n),
              "ORBmatcher::SearchForInitialization");
        return n;
    }

    // :409-516.  f1_has_mp[i1]: F1.mvpMapPoints[i1] set and not bad.
    // vnMatches21[i2]: F1 index whose map point F2 keypoint i2 received, or -1.
    int WindowSearch(const FrameData& F1, const FrameData& F2, int windowSize, const std::vector<uint8_t>& f1_has_mp,
                     std::vector<int>& vnMatches21, int minOctave = -1, int maxOctave = INT32_MAX)
    {
        const orbx_frame_view v1 = F1.view(), v2 = F2.view();
        vnMatches21.assign(v2.n, -1);
        int n = 0;
        check(orbx_window_search(ctx_, &v1, &v2, f1_has_mp.data(), windowSize, minOctave,
                                 maxOctave == INT32_MAX ? -1 : maxOctave, mfNNratio, mbCheckOrientation,
                                 vnMatches21.data(), &n),
              "ORBmatcher::WindowSearch");
        return n;
    }

    // :49-125, local-map tracking (per map point: in_view, projection,
    // predicted level, viewing cosine, descriptor).
    int SearchByProjection(const FrameData& F, int n_mp, const uint8_t* in_view, const float* proj_xy,
                           const int32_t* pred_level, const float* view_cos, const uint8_t* mp_desc,
                           const uint8_t* f_assigned, float th, std::vector<int>& matches_f)
    {
        const orbx_frame_view v = F.view();
        matches_f.assign(v.n, -1);
        int n = 0;
        check(orbx_search_by_projection_local(ctx_, &v, n_mp, in_view, proj_xy, pred_level, view_cos, mp_desc,
                                              f_assigned, th, mfNNratio, matches_f.data(), &n),
              "ORBmatcher::SearchByProjection(local map)");
        return n;
    }

    // Tracking::SearchReferencePointsInFrustum (src/Tracking.cc:701-752):
    // Frame::isInFrustum for every local map point, then the local-map search
    // above, both on the device (no host pass over the local map).  The
    // per-point frustum results come back for IncreaseVisible() and the
    // MapPoint tracking fields; q.frame / q.matches_f are set here.
    int SearchLocalMap(const FrameData& F, orbx_local_map_query& q, std::vector<int>& matches_f)
    {
        const orbx_frame_view v = F.view();
        matches_f.assign(v.n, -1);
        q.frame = &v;
        q.matches_f = matches_f.data();
        q.nnratio = mfNNratio;
        check(orbx_search_local_map(ctx_, &q), "Tracking::SearchReferencePointsInFrustum");
        q.frame = nullptr;
        q.matches_f = nullptr;
        return q.n_matches;
    }

    // :1507-1620, motion-model tracking.
    int SearchByProjection(const FrameData& Cur, const FrameData& Last, const float* last_mp_xyz,
                           const uint8_t* last_mp_valid, const uint8_t* cur_assigned, const float* Tcw,
                           const float* cam, float th, std::vector<int>& matches_cur)
    {
        const orbx_frame_view vc = Cur.view(), vl = Last.view();
        matches_cur.assign(vc.n, -1);
        int n = 0;
        check(orbx_search_by_projection_motion(ctx_, &vc, &vl, last_mp_xyz, last_mp_valid, cur_assigned, Tcw, cam, th,
                                               mbCheckOrientation, matches_cur.data(), &n),
              "ORBmatcher::SearchByProjection(motion)");
        return n;
    }

    // :519-594, refinement after pose optimisation.
    int SearchByProjection(const FrameData& F1, const FrameData& F2, int windowSize, const float* f1_mp_xyz,
                           const uint8_t* f1_mp_valid, const uint8_t* f2_assigned, const float* Tcw2,
                           const float* cam, std::vector<int>& matches21)
    {
        const orbx_frame_view v1 = F1.view(), v2 = F2.view();
        matches21.assign(v2.n, -1);
        int n = 0;
        check(orbx_search_by_projection_pair(ctx_, &v1, &v2, f1_mp_xyz, f1_mp_valid, f2_assigned, Tcw2, cam,
                                             windowSize, mfNNratio, matches21.data(), &n),
              "ORBmatcher::SearchByProjection(pair)");
        return n;
    }

    // Brute-force matching of two descriptor sets (config C3: the B3 rule over
    // all pairs).
    int MatchBruteForce(const std::vector<uint8_t>& dA, const std::vector<uint8_t>& dB, std::vector<int>& m12,
                        int th_low = TH_LOW)
    {
        const int nA = (int)(dA.size() / 32), nB = (int)(dB.size() / 32);
        m12.assign(nA, -1);
        int n = 0;
        check(orbx_match_bf(ctx_, dA.data(), nA, dB.data(), nB, th_low, mfNNratio, m12.data(), &n),
              "ORBmatcher::MatchBruteForce");
        return n;
    }

    float mfNNratio;
    bool mbCheckOrientation;

private:
    orbx_ctx* ctx_;
    std::unique_ptr<Context> own_;
};

// ---------------------------------------------------------------------------
// Optimizer::LocalBundleAdjustment (src/Optimizer.cc:287-536).  The caller
// packs the local window (local keyframes, fixed covisible keyframes, local
// map points and their observations, in g2o insertion order) into a
// LocalBAProblem, runs it, then applies the results the way the reference
// does: erase the observations flagged in edge_status, write poses/points
// back for keyframes and non-bad points.
// ---------------------------------------------------------------------------
struct LocalBAProblem {
    std::vector<double> pose_q, pose_t, pose_cam, points, edge_obs, edge_inv_sigma2;
    std::vector<uint8_t> pose_fixed;
    std::vector<int64_t> pose_id, point_id;
    std::vector<int32_t> point_nobs, edge_point, edge_pose;
    double huber_delta = (double)(float)2.4476519;   // sqrt(5.991) as float
    double chi2_threshold = 5.991;
    // results
    std::vector<uint8_t> edge_status, point_bad;
    orbx_ba_stats stats{};

    orbx_ba_problem view()
    {
        orbx_ba_problem p;
        p.n_poses = (int)pose_fixed.size();
        p.n_points = (int)point_id.size();
        p.n_edges = (int)edge_point.size();
        p.pose_q = pose_q.data();
        p.pose_t = pose_t.data();
        p.pose_fixed = pose_fixed.data();
        p.pose_id = pose_id.data();
        p.pose_cam = pose_cam.data();
        p.points = points.data();
        p.point_id = point_id.data();
        p.point_nobs = point_nobs.data();
        p.edge_point = edge_point.data();
        p.edge_pose = edge_pose.data();
        p.edge_obs = edge_obs.data();
        p.edge_inv_sigma2 = edge_inv_sigma2.data();
        p.huber_delta = huber_delta;
        p.chi2_threshold = chi2_threshold;
        return p;
    }
};

// ---------------------------------------------------------------------------
// Optimizer::PoseOptimization(Frame*) (src/Optimizer.cc:154-285): the fields
// of Frame it reads and writes.  mp_xyz holds pMP->GetWorldPos() for the
// keypoints whose mvpMapPoints entry is set (has_mp).
// ---------------------------------------------------------------------------
struct PoseFrame {
    std::vector<KeyPoint> keys_un;          // mvKeysUn
    std::vector<float> inv_level_sigma2;    // mvInvLevelSigma2
    std::vector<uint8_t> has_mp;            // mvpMapPoints[i] != NULL
    std::vector<float> mp_xyz;              // 3 per keypoint
    float fx = 0, fy = 0, cx = 0, cy = 0;
    float Tcw[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};   // mTcw, row-major
    std::vector<uint8_t> outlier;           // mvbOutlier
    orbx_pose_stats stats{};
};

class Optimizer {
public:
    // Returns nInitialCorrespondences - nBad, updates F.Tcw and F.outlier.
    static int PoseOptimization(orbx_ctx* ctx, PoseFrame& F)
    {
        const int n = (int)F.keys_un.size();
        std::vector<float> kp(2 * (size_t)n);
        std::vector<int32_t> oct(n);
        for (int i = 0; i < n; i++) {
            kp[2 * i] = F.keys_un[i].x;
            kp[2 * i + 1] = F.keys_un[i].y;
            oct[i] = F.keys_un[i].octave;
        }
        F.outlier.resize(n, 0);
        orbx_pose_frame f;
        f.n = n;
        f.kp_un = kp.data();
        f.octave = oct.data();
        f.inv_level_sigma2 = F.inv_level_sigma2.data();
        f.nlevels = (int)F.inv_level_sigma2.size();
        f.has_mp = F.has_mp.data();
        f.mp_xyz = F.mp_xyz.data();
        f.cam[0] = F.fx;
        f.cam[1] = F.fy;
        f.cam[2] = F.cx;
        f.cam[3] = F.cy;
        for (int k = 0; k < 16; k++) f.Tcw[k] = F.Tcw[k];
        f.outlier = F.outlier.data();
        int inl = 0;
        check(orbx_pose_optimization(ctx, &f, &inl, &F.stats), "Optimizer::PoseOptimization");
        for (int k = 0; k < 16; k++) F.Tcw[k] = f.Tcw[k];
        return inl;
    }

    // pbStopFlag: LocalMapping's mbAbortBA, polled between LM iterations.
    static void LocalBundleAdjustment(orbx_ctx* ctx, LocalBAProblem& prob, bool* pbStopFlag = nullptr)
    {
        orbx_ba_problem p = prob.view();
        prob.edge_status.assign(p.n_edges, 0);
        prob.point_bad.assign(p.n_points, 0);
        check(orbx_lba_solve(ctx, &p, 5, 10, reinterpret_cast<const volatile uint8_t*>(pbStopFlag),
                             prob.edge_status.data(), prob.point_bad.data(), &prob.stats),
              "Optimizer::LocalBundleAdjustment");
    }
};

}  // namespace ORB_SLAM_AMD
