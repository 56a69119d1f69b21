// ORACLE -- TEST INFRASTRUCTURE ONLY (see ref_common.h).
//
// extern "C" surface of the CPU restatement, loaded by tests/ and bench.py
// (cpu_baseline) through ctypes.  Mirrors include/orbx.h with an orbx_ref_
// prefix; frame/keypoint structs are the public ABI ones.
#include "ref_common.h"
#include "../include/orbx.h"

#include <algorithm>
#include <chrono>
#include <cstring>
#include <exception>
#include <memory>

using namespace orbref;

// memcpy that accepts the empty vectors' null data() (n == 0), which
// std::memcpy does not (UBSan: nonnull arguments)
static inline void copy_bytes(void* dst, const void* src, size_t n)
{
    if (n) std::memcpy(dst, src, n);
}

extern "C" {

struct orbx_ref_extractor {
    std::unique_ptr<ORBextractorRef> ex;
};

orbx_ref_extractor* orbx_ref_extractor_create(int nfeatures, float scale, int nlevels,
                                              int score_type, int fast_th)
{
    if (nfeatures <= 0 || nlevels <= 0 || nlevels > 32 || !(scale > 1.0f))
        return nullptr;
    auto* r = new orbx_ref_extractor;
    r->ex.reset(new ORBextractorRef(nfeatures, scale, nlevels, score_type, fast_th));
    return r;
}

void orbx_ref_extractor_destroy(orbx_ref_extractor* r) { delete r; }

int orbx_ref_extract(orbx_ref_extractor* r, const uint8_t* img, int w, int h, size_t stride,
                     orbx_keypoint* kps, uint8_t* desc, int cap, int* n_out)
{
    try {
        std::vector<KeyPoint> k;
        std::vector<uint8_t> d;
        if (!r->ex->extract(img, w, h, stride, k, d)) {
            *n_out = 0;
            return ORBX_OK;
        }
        *n_out = (int)k.size();
        if ((int)k.size() > cap) return ORBX_ERR_CAPACITY;
        copy_bytes(kps, k.data(), k.size() * sizeof(KeyPoint));
        copy_bytes(desc, d.data(), d.size());
        return ORBX_OK;
    } catch (const std::exception&) {
        return ORBX_ERR_UNSUPPORTED;
    }
}

// Debug tap: padded level (raw or blurred) of the last extract() call.
int orbx_ref_level(orbx_ref_extractor* r, int level, int blurred, uint8_t* out, int cap,
                   int* pw, int* ph)
{
    auto& v = blurred ? r->ex->blurred : r->ex->pyramid;
    if (level < 0 || level >= (int)v.size()) return ORBX_ERR_ARG;
    const PaddedImage& L = v[level];
    *pw = L.pw;
    *ph = L.ph;
    if ((int)L.buf.size() > cap) return ORBX_ERR_CAPACITY;
    copy_bytes(out, L.buf.data(), L.buf.size());
    return ORBX_OK;
}

// Debug tap: level keypoints (level coordinates, pre-scaling) of the last call.
int orbx_ref_level_keys(orbx_ref_extractor* r, int level, orbx_keypoint* out, int cap, int* n)
{
    if (level < 0 || level >= (int)r->ex->levelKeys.size()) return ORBX_ERR_ARG;
    const auto& v = r->ex->levelKeys[level];
    *n = (int)v.size();
    if ((int)v.size() > cap) return ORBX_ERR_CAPACITY;
    copy_bytes(out, v.data(), v.size() * sizeof(KeyPoint));
    return ORBX_OK;
}

int orbx_ref_features_per_level(orbx_ref_extractor* r, int32_t* out, int cap)
{
    const auto& v = r->ex->mnFeaturesPerLevel;
    for (int i = 0; i < (int)v.size() && i < cap; i++) out[i] = v[i];
    return (int)v.size();
}

int orbx_ref_umax(orbx_ref_extractor* r, int32_t* out, int cap)
{
    const auto& v = r->ex->umax;
    for (int i = 0; i < (int)v.size() && i < cap; i++) out[i] = v[i];
    return (int)v.size();
}

int orbx_ref_scale_factors(orbx_ref_extractor* r, float* out, float* inv, int cap)
{
    const int n = r->ex->nlevels;
    for (int i = 0; i < n && i < cap; i++) {
        out[i] = r->ex->mvScaleFactor[i];
        inv[i] = r->ex->mvInvScaleFactor[i];
    }
    return n;
}

// Times `iters` extract() calls on one core; returns seconds.
double orbx_ref_time_extract(orbx_ref_extractor* r, const uint8_t* imgs, int nimg, int w, int h,
                             size_t stride, int iters)
{
    std::vector<KeyPoint> k;
    std::vector<uint8_t> d;
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < iters; i++)
        r->ex->extract(imgs + (size_t)(i % nimg) * h * stride, w, h, stride, k, d);
    auto t1 = std::chrono::steady_clock::now();
    return std::chrono::duration<double>(t1 - t0).count();
}

// ---- primitives ----
float orbx_ref_fast_atan2(float y, float x) { return fast_atan2_cv24(y, x); }
float orbx_ref_cosf(float x) { return cr_cosf(x); }
/* 1 when this library's reference-compiled float sites (ref_orbsites.cpp)
 * were built with GCC's FMA contraction (liborbx_ref_contract.so) */
int orbx_ref_fp_contract(void) { return orbsites_contracted(); }
float orbx_ref_sinf(float x) { return cr_sinf(x); }
int orbx_ref_descriptor_distance(const uint8_t* a, const uint8_t* b) { return descriptor_distance(a, b); }

int orbx_ref_fast_cell(const uint8_t* img, int step, int rows, int cols, int threshold,
                       orbx_keypoint* out, int cap, int* n)
{
    std::vector<KeyPoint> k;
    cv24_fast16(img, step, rows, cols, threshold, true, k);
    *n = (int)k.size();
    if ((int)k.size() > cap) return ORBX_ERR_CAPACITY;
    copy_bytes(out, k.data(), k.size() * sizeof(KeyPoint));
    return ORBX_OK;
}

int orbx_ref_resize(const uint8_t* src, int sstep, int sw, int sh, uint8_t* dst, int dstep,
                    int dw, int dh)
{
    try {
        cv24_resize_linear_u8(src, sstep, sw, sh, dst, dstep, dw, dh);
        return ORBX_OK;
    } catch (const std::exception&) {
        return ORBX_ERR_UNSUPPORTED;
    }
}

/* libstdc++ era of retainBest's std::nth_element pivot step
 * (ref_extract.cpp): 0 = GCC >= 4.9 (this image's), 1 = GCC 4.6 .. 4.8 */
int orbx_ref_set_nth_pivot(int mode)
{
    if (mode != NTH_PIVOT_GCC49 && mode != NTH_PIVOT_GCC48) return ORBX_ERR_ARG;
    set_nth_pivot(mode);
    return ORBX_OK;
}
int orbx_ref_get_nth_pivot(void) { return get_nth_pivot(); }

/* Permutation nth_element(a, a + nth, a + n, greater) leaves on n float
 * keys: the restatement with the given pivot era (std_impl = 0), or this
 * image's std::nth_element (std_impl = 1), for checking the restatement. */
static bool kp_response_greater(const KeyPoint& a, const KeyPoint& b) { return a.response > b.response; }

int orbx_ref_nth_element_perm(const float* keys, int n, int nth, int mode, int std_impl, int32_t* perm)
{
    if (n < 0 || nth < 0 || nth > n) return ORBX_ERR_ARG;
    std::vector<KeyPoint> v(n);
    for (int i = 0; i < n; i++) {
        std::memset(&v[i], 0, sizeof(KeyPoint));
        v[i].response = keys[i];
        v[i].class_id = i;
    }
    if (std_impl) std::nth_element(v.begin(), v.begin() + nth, v.end(), kp_response_greater);
    else libstdcxx_nth_element(v.data(), v.data() + nth, v.data() + n, kp_response_greater, mode);
    for (int i = 0; i < n; i++) perm[i] = v[i].class_id;
    return ORBX_OK;
}

// retainBest over a list of responses; writes the surviving original indices.
int orbx_ref_retain_best(const float* responses, int n, int n_points, int32_t* out_idx)
{
    std::vector<KeyPoint> k(n);
    for (int i = 0; i < n; i++) {
        std::memset(&k[i], 0, sizeof(KeyPoint));
        k[i].response = responses[i];
        k[i].class_id = i;
    }
    cv24_retain_best(k, n_points);
    if ((int)k.size() > n_points && n_points >= 0) k.resize(n_points);
    for (size_t i = 0; i < k.size(); i++) out_idx[i] = k[i].class_id;
    return (int)k.size();
}

// ---- matchers ----
static void to_frame(const orbx_frame_view* v, FrameRef& F)
{
    F.build(reinterpret_cast<const KeyPoint*>(v->keys_un), v->desc, v->n, v->min_x, v->max_x,
            v->min_y, v->max_y, v->nlevels, v->scale_factor);
}

int orbx_ref_search_for_initialization(const orbx_frame_view* F1v, const orbx_frame_view* F2v,
                                       float* prev_matched, int32_t* matches12, int window,
                                       float nnratio, int check_ori, int* n_matches)
{
    static thread_local FrameRef F1, F2;
    to_frame(F1v, F1);
    to_frame(F2v, F2);
    std::vector<float> pm(prev_matched, prev_matched + 2 * F1v->n);
    std::vector<int> m;
    *n_matches = search_for_initialization(F1, F2, pm, m, window, nnratio, check_ori != 0);
    copy_bytes(prev_matched, pm.data(), pm.size() * sizeof(float));
    for (int i = 0; i < F1v->n; i++) matches12[i] = m[i];
    return ORBX_OK;
}

int orbx_ref_window_search(const orbx_frame_view* F1v, const orbx_frame_view* F2v,
                           const uint8_t* f1_mp, int window, int min_level, int max_level,
                           float nnratio, int check_ori, int32_t* matches21, int* n_matches)
{
    static thread_local FrameRef F1, F2;
    to_frame(F1v, F1);
    to_frame(F2v, F2);
    std::vector<int> m;
    *n_matches = window_search(F1, F2, f1_mp, window, min_level, max_level < 0 ? 2147483647 : max_level,
                               nnratio, check_ori != 0, m);
    for (int i = 0; i < F2v->n; i++) matches21[i] = m[i];
    return ORBX_OK;
}

int orbx_ref_search_by_projection_pair(const orbx_frame_view* F1v, const orbx_frame_view* F2v,
                                       const float* xyz, const uint8_t* valid,
                                       const uint8_t* f2_assigned, const float* Tcw,
                                       const float* cam, int window, float nnratio,
                                       int32_t* matches21, int* n_matches)
{
    static thread_local FrameRef F1, F2;
    to_frame(F1v, F1);
    to_frame(F2v, F2);
    std::vector<int> m;
    *n_matches = search_by_projection_pair(F1, F2, xyz, valid, f2_assigned, Tcw, cam, window, nnratio, m);
    for (int i = 0; i < F2v->n; i++) matches21[i] = m[i];
    return ORBX_OK;
}

int orbx_ref_search_by_projection_motion(const orbx_frame_view* Cv, const orbx_frame_view* Lv,
                                         const float* xyz, const uint8_t* valid,
                                         const uint8_t* cur_assigned, const float* Tcw,
                                         const float* cam, float th, int check_ori,
                                         int32_t* matches_cur, int* n_matches)
{
    static thread_local FrameRef C, L;
    to_frame(Cv, C);
    to_frame(Lv, L);
    std::vector<int> m;
    *n_matches = search_by_projection_motion(C, L, xyz, valid, cur_assigned, Tcw, cam, th, check_ori != 0, m);
    for (int i = 0; i < Cv->n; i++) matches_cur[i] = m[i];
    return ORBX_OK;
}

int orbx_ref_search_by_projection_local(const orbx_frame_view* Fv, int n_mp, const uint8_t* in_view,
                                        const float* proj_xy, const int32_t* pred_level,
                                        const float* view_cos, const uint8_t* mp_desc,
                                        const uint8_t* f_assigned, float th, float nnratio,
                                        int32_t* matches_f, int* n_matches)
{
    static thread_local FrameRef F;
    to_frame(Fv, F);
    std::vector<int> m;
    *n_matches = search_by_projection_local(F, n_mp, in_view, proj_xy, pred_level, view_cos, mp_desc,
                                            f_assigned, th, nnratio, m);
    for (int i = 0; i < Fv->n; i++) matches_f[i] = m[i];
    return ORBX_OK;
}

// Tracking::SearchReferencePointsInFrustum (src/Tracking.cc:701-752):
// isInFrustum per local map point, in list order, then the local-map
// SearchByProjection over the points in view.
int orbx_ref_search_local_map(orbx_local_map_query* q)
{
    if (!q || !q->frame) return ORBX_ERR_ARG;
    static thread_local FrameRef F;
    to_frame(q->frame, F);
    const int n = q->n_mp;
    std::vector<uint8_t> in(n, 0);
    std::vector<float> xy(2 * (size_t)n, 0.f), vc(n, 0.f);
    std::vector<int32_t> lv(n, 0);
    int n_in = 0;
    for (int m = 0; m < n; m++) {
        if (q->mp_skip && q->mp_skip[m]) continue;
        float u, v, c;
        int l;
        if (is_in_frustum(F, q->Rcw, q->tcw, q->Ow, q->cam, q->mp_pos + 3 * m, q->mp_normal + 3 * m,
                          q->mp_dist[2 * m], q->mp_dist[2 * m + 1], q->view_cos_limit, u, v, l, c)) {
            in[m] = 1;
            xy[2 * m] = u;
            xy[2 * m + 1] = v;
            lv[m] = l;
            vc[m] = c;
            n_in++;
        }
    }
    for (int m = 0; m < n; m++) {
        if (q->in_view) q->in_view[m] = in[m];
        if (q->proj_xy) {
            q->proj_xy[2 * m] = xy[2 * m];
            q->proj_xy[2 * m + 1] = xy[2 * m + 1];
        }
        if (q->pred_level) q->pred_level[m] = lv[m];
        if (q->view_cos) q->view_cos[m] = vc[m];
    }
    q->n_in_view = n_in;
    std::vector<int> mf;
    q->n_matches = n_in > 0 ? search_by_projection_local(F, n, in.data(), xy.data(), lv.data(), vc.data(), q->mp_desc,
                                                         q->f_assigned, q->th, q->nnratio, mf)
                            : 0;
    for (int i = 0; i < q->frame->n; i++) q->matches_f[i] = n_in > 0 ? mf[i] : -1;
    return ORBX_OK;
}

int orbx_ref_hamming_bf(const uint8_t* dA, int nA, const uint8_t* dB, int nB, int32_t* best_idx,
                        int32_t* best, int32_t* second)
{
    hamming_bf(dA, nA, dB, nB, best_idx, best, second);
    return ORBX_OK;
}

}  // extern "C"

// ---- local BA ----
#include "ref_lba.h"

extern "C" int orbx_ref_lba(orbx_ba_problem* p, int iters0, int iters1, uint8_t* edge_status, uint8_t* point_bad,
                            orbx_ba_stats* stats)
{
    LBAInput in;
    in.n_poses = p->n_poses;
    in.n_points = p->n_points;
    in.n_edges = p->n_edges;
    in.poses.resize(p->n_poses);
    for (int i = 0; i < p->n_poses; i++) {
        in.poses[i].q = {p->pose_q[4 * i], p->pose_q[4 * i + 1], p->pose_q[4 * i + 2], p->pose_q[4 * i + 3]};
        for (int k = 0; k < 3; k++) in.poses[i].t[k] = p->pose_t[3 * i + k];
    }
    in.pose_fixed.assign(p->pose_fixed, p->pose_fixed + p->n_poses);
    in.pose_id.assign(p->pose_id, p->pose_id + p->n_poses);
    in.pose_cam.assign(p->pose_cam, p->pose_cam + 4 * p->n_poses);
    in.points.assign(p->points, p->points + 3 * p->n_points);
    in.point_id.assign(p->point_id, p->point_id + p->n_points);
    in.point_nobs.assign(p->point_nobs, p->point_nobs + p->n_points);
    in.edge_point.assign(p->edge_point, p->edge_point + p->n_edges);
    in.edge_pose.assign(p->edge_pose, p->edge_pose + p->n_edges);
    in.edge_obs.assign(p->edge_obs, p->edge_obs + 2 * p->n_edges);
    in.edge_inv_sigma2.assign(p->edge_inv_sigma2, p->edge_inv_sigma2 + p->n_edges);
    in.huber_delta = p->huber_delta;
    in.chi2_threshold = p->chi2_threshold;
    std::vector<uint8_t> es, pb;
    LBAStats st;
    local_ba(in, iters0, iters1, es, pb, st);
    for (int i = 0; i < p->n_poses; i++) {
        p->pose_q[4 * i] = in.poses[i].q.x;
        p->pose_q[4 * i + 1] = in.poses[i].q.y;
        p->pose_q[4 * i + 2] = in.poses[i].q.z;
        p->pose_q[4 * i + 3] = in.poses[i].q.w;
        for (int k = 0; k < 3; k++) p->pose_t[3 * i + k] = in.poses[i].t[k];
    }
    copy_bytes(p->points, in.points.data(), in.points.size() * sizeof(double));
    copy_bytes(edge_status, es.data(), es.size());
    copy_bytes(point_bad, pb.data(), pb.size());
    if (stats) {
        for (int k = 0; k < 2; k++) {
            stats->iterations[k] = st.iterations[k];
            stats->levenberg_trials[k] = st.trials[k];
            stats->chi2_initial[k] = st.chi2_initial[k];
            stats->chi2_final[k] = st.chi2_final[k];
            stats->n_outliers[k] = st.n_outliers[k];
        }
        stats->not_posdef = st.not_posdef;
    }
    return ORBX_OK;
}

// SE3 primitives for unit tests
extern "C" void orbx_ref_se3_exp(const double* u, double* q, double* t)
{
    SE3 s = se3_exp(u);
    q[0] = s.q.x; q[1] = s.q.y; q[2] = s.q.z; q[3] = s.q.w;
    for (int k = 0; k < 3; k++) t[k] = s.t[k];
}

extern "C" void orbx_ref_quat_from_matrix(const double* R, double* q)
{
    Quat r = quat_from_matrix(R);
    q[0] = r.x; q[1] = r.y; q[2] = r.z; q[3] = r.w;
}

// EdgeSE3ProjectXYZ error and analytic Jacobians for a single observation
// (unit tests against finite differences).  pose: q(4) t(3); A: 2x3, B: 2x6.
extern "C" void orbx_ref_edge_linearize(const double* pose, const double* point, const double* cam,
                                        const double* obs, double* err, double* A, double* B)
{
    LBAInput in;
    in.n_poses = 1;
    in.n_points = 1;
    in.n_edges = 1;
    in.poses.resize(1);
    in.poses[0].q = {pose[0], pose[1], pose[2], pose[3]};
    for (int k = 0; k < 3; k++) in.poses[0].t[k] = pose[4 + k];
    in.pose_fixed = {0};
    in.pose_id = {0};
    in.pose_cam.assign(cam, cam + 4);
    in.points.assign(point, point + 3);
    in.point_id = {1};
    in.point_nobs = {3};
    in.edge_point = {0};
    in.edge_pose = {0};
    in.edge_obs.assign(obs, obs + 2);
    in.edge_inv_sigma2 = {1.0};
    in.huber_delta = 1e9;
    in.chi2_threshold = 1e9;
    edge_linearize_for_test(in, err, A, B);
}

// ---- motion-only pose optimisation ----
#include "ref_pose.h"

extern "C" int orbx_ref_pose_optimization(orbx_pose_frame* f, int* n_inliers, orbx_pose_stats* stats)
{
    if (!f || f->n < 0 || f->nlevels <= 0) return ORBX_ERR_ARG;
    std::vector<float> isig(f->n > 0 ? f->n : 1, 0.f);
    for (int i = 0; i < f->n; i++) {
        if (!f->has_mp[i]) continue;
        if (f->octave[i] < 0 || f->octave[i] >= f->nlevels) return ORBX_ERR_ARG;
        isig[i] = f->inv_level_sigma2[f->octave[i]];   // pFrame->mvInvLevelSigma2[kpUn.octave] (:212)
    }
    PoseStats st;
    const int r = pose_optimization(f->Tcw, f->cam, f->n, f->kp_un, isig.data(), f->has_mp, f->mp_xyz, f->outlier, &st);
    if (n_inliers) *n_inliers = r;
    if (stats) {
        stats->rounds = st.rounds;
        for (int k = 0; k < 4; k++) {
            stats->iterations[k] = st.iterations[k];
            stats->levenberg_trials[k] = st.trials[k];
            stats->n_bad[k] = st.n_bad[k];
            stats->chi2_final[k] = st.chi2_final[k];
        }
        stats->not_posdef = st.not_posdef;
    }
    return ORBX_OK;
}

// Eigen LDLT restatement (unit test against numpy's solve)
extern "C" int orbx_ref_ldlt_solve(int n, const double* a, const double* b, double* x)
{
    return ldlt_solve(n, a, b, x) ? 1 : 0;
}
