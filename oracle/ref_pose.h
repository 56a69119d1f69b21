// ORACLE -- TEST INFRASTRUCTURE ONLY (see ref_common.h).
//
// Sequential CPU restatement of Optimizer::PoseOptimization
// (src/Optimizer.cc:154-285): one VertexSE3Expmap (id 0) against fixed
// VertexSBAPointXYZ vertices through EdgeSE3ProjectXYZ edges with a Huber
// kernel, BlockSolverX + LinearSolverDense (Eigen LDLT with diagonal
// pivoting, solvers/dense/linear_solver_dense.h:70-113) and
// OptimizationAlgorithmLevenberg with ORB-SLAM's stop rule
// (optimization_algorithm_levenberg.cpp:61-164).  Four robust rounds classify
// outliers (chi2 9.210 / 7.378 / 5.991 / 5.991, iterations 10 / 10 / 7 / 5).
// Pose conversions follow Converter::toSE3Quat / toCvMat (src/Converter.cc:
// 38-72).
#pragma once
#include <cstdint>

namespace orbref {

struct PoseStats {
    int rounds = 0;             // robust rounds run (break when < 10 edges)
    int iterations[4] = {0, 0, 0, 0};
    int trials[4] = {0, 0, 0, 0};
    int n_bad[4] = {0, 0, 0, 0};
    double chi2_final[4] = {0, 0, 0, 0};
    int not_posdef = 0;
};

// Eigen::LDLT<MatrixXd> (lower, diagonal pivoting) of the n x n row-major
// matrix `a` (read: lower triangle) and solve a x = b.  Returns
// LDLT::isPositive().  Shared with the unit tests.
bool ldlt_solve(int n, const double* a, const double* b, double* x);

// Optimizer::PoseOptimization on one frame.  Tcw: row-major 4x4 float
// (in/out).  Per keypoint i: kp_un (2), inv_sigma2 (mvInvLevelSigma2 of its
// octave), has_mp, mp_xyz (3).  outlier (in/out): mvbOutlier, written for
// keypoints with a map point.  Returns nInitialCorrespondences - nBad.
int pose_optimization(float Tcw[16], const float cam[4], int n, const float* kp_un,
                      const float* inv_sigma2, const uint8_t* has_mp, const float* mp_xyz,
                      uint8_t* outlier, PoseStats* stats);

}  // namespace orbref
