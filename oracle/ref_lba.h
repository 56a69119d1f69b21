// ORACLE -- TEST INFRASTRUCTURE ONLY (see ref_common.h).
//
// Sequential CPU restatement of Optimizer::LocalBundleAdjustment's
// optimisation core (src/Optimizer.cc:287-536) on the g2o subset it uses:
// VertexSE3Expmap / VertexSBAPointXYZ / EdgeSE3ProjectXYZ
// (types_six_dof_expmap.{h,cpp}), RobustKernelHuber, SparseOptimizer,
// BlockSolverX with Schur complement over the points, and
// OptimizationAlgorithmLevenberg with ORB-SLAM's stop rule.  The reduced
// camera system is solved with a dense Cholesky (LLT) where the reference
// uses CHOLMOD (SuiteSparse, absent here); both are exact LLT
// factorisations of the same SPD matrix, differing only in rounding.
#pragma once
#include <cstdint>
#include <vector>

namespace orbref {

struct Quat { double x, y, z, w; };
struct SE3 { Quat q; double t[3]; };

// Eigen/g2o primitives restated (se3quat.h, Eigen Quaternion).
Quat quat_mul(const Quat& a, const Quat& b);
void quat_rotate(const Quat& q, const double v[3], double out[3]);
void quat_to_matrix(const Quat& q, double R[9]);
Quat quat_from_matrix(const double R[9]);
void se3_normalize(SE3& s);
SE3 se3_exp(const double update[6]);
SE3 se3_mul(const SE3& a, const SE3& b);

struct LBAInput {
    int n_poses, n_points, n_edges;
    std::vector<SE3> poses;
    std::vector<uint8_t> pose_fixed;
    std::vector<int64_t> pose_id;
    std::vector<double> pose_cam;      // 4 per pose
    std::vector<double> points;        // 3 per point
    std::vector<int64_t> point_id;
    std::vector<int> point_nobs;
    std::vector<int> edge_point, edge_pose;
    std::vector<double> edge_obs;      // 2 per edge
    std::vector<double> edge_inv_sigma2;
    double huber_delta, chi2_threshold;
};

struct LBAStats {
    int iterations[2] = {0, 0};
    int trials[2] = {0, 0};
    double chi2_initial[2] = {0, 0};
    double chi2_final[2] = {0, 0};
    int n_outliers[2] = {0, 0};
    int not_posdef = 0;
};

// Error and analytic Jacobians of edge 0 of `in` at the current estimate.
void edge_linearize_for_test(LBAInput& in, double err[2], double A[6], double B[12]);

// Runs optimize(iters0), outlier pass 1, optimize(iters1), outlier pass 2.
// edge_status: 0 inlier, 1 erased in pass 1, 2 erased in pass 2.
void local_ba(LBAInput& in, int iters0, int iters1, std::vector<uint8_t>& edge_status,
              std::vector<uint8_t>& point_bad, LBAStats& stats);

}  // namespace orbref
