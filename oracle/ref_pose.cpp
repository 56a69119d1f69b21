// ORACLE -- TEST INFRASTRUCTURE ONLY (see ref_common.h, ref_pose.h).
#include "ref_pose.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <limits>
#include <utility>
#include <vector>

#include "ref_lba.h"

namespace orbref {

// Eigen::LDLT<MatrixXd>::compute (ldlt_inplace<Lower>::unblocked: largest
// remaining diagonal pivot, first index on ties) and LDLT::solve
// (transpositions, unit-lower forward solve, pseudo-inverse of D, unit-upper
// backward solve with a row dot product, inverse transpositions).
bool ldlt_solve(int n, const double* a, const double* b, double* x)
{
    std::vector<double> m(a, a + (size_t)n * n);
    std::vector<int> tr(n);
    std::vector<double> temp(n);
    enum { kZero, kPos, kNeg, kIndef } sign = kZero;
    auto M = [&](int i, int j) -> double& { return m[(size_t)i * n + j]; };
    for (int k = 0; k < n; k++) {
        int big = k;
        double bv = std::fabs(M(k, k));
        for (int i = k + 1; i < n; i++)
            if (std::fabs(M(i, i)) > bv) {
                bv = std::fabs(M(i, i));
                big = i;
            }
        tr[k] = big;
        if (k != big) {
            for (int j = 0; j < k; j++) std::swap(M(k, j), M(big, j));
            for (int i = big + 1; i < n; i++) std::swap(M(i, k), M(i, big));
            std::swap(M(k, k), M(big, big));
            for (int i = k + 1; i < big; i++) {
                const double t = M(i, k);
                M(i, k) = M(big, i);
                M(big, i) = t;
            }
        }
        const int rs = n - k - 1;
        if (k > 0) {
            for (int j = 0; j < k; j++) temp[j] = M(j, j) * M(k, j);
            double acc = M(k, 0) * temp[0];
            for (int j = 1; j < k; j++) acc += M(k, j) * temp[j];
            M(k, k) -= acc;
            for (int i = k + 1; i < n; i++)
                for (int j = 0; j < k; j++) M(i, k) -= M(i, j) * temp[j];
        }
        const double akk = M(k, k);
        if (rs > 0 && std::fabs(akk) > 0.0)
            for (int i = k + 1; i < n; i++) M(i, k) /= akk;
        if (sign == kPos) {
            if (akk < 0) sign = kIndef;
        } else if (sign == kNeg) {
            if (akk > 0) sign = kIndef;
        } else if (sign == kZero) {
            if (akk > 0) sign = kPos;
            else if (akk < 0) sign = kNeg;
        }
    }
    for (int i = 0; i < n; i++) x[i] = b[i];
    for (int k = 0; k < n; k++) std::swap(x[k], x[tr[k]]);
    for (int i = 0; i < n; i++)
        for (int j = 0; j < i; j++) x[i] -= M(i, j) * x[j];
    for (int i = 0; i < n; i++) {
        if (std::fabs(M(i, i)) > DBL_MIN) x[i] /= M(i, i);
        else x[i] = 0.0;
    }
    for (int i = n - 1; i >= 0; i--) {
        if (i == n - 1) continue;
        double s = M(i + 1, i) * x[i + 1];
        for (int j = i + 2; j < n; j++) s += M(j, i) * x[j];
        x[i] -= s;
    }
    for (int k = n - 1; k >= 0; k--) std::swap(x[k], x[tr[k]]);
    return sign == kPos || sign == kZero;
}

namespace {

struct PoseEdge {
    double obs[2];
    double isig;
    double X[3];
    int kp;
};

struct PoseOpt {
    SE3 pose;
    double fx, fy, cx, cy;
    double delta;
    std::vector<PoseEdge> edges;
    std::vector<uint8_t> level;          // g2o edge level (0 active, 1 outlier)
    std::vector<double> err;             // last computed error per edge
    std::vector<int> active;
    double H[36], b[6], x[6];
    double lambda = 0, ni = 2;
    int nBad = 0;

    void compute_error(int e)
    {
        const PoseEdge& E = edges[e];
        double pc[3];
        quat_rotate(pose.q, E.X, pc);
        for (int i = 0; i < 3; i++) pc[i] += pose.t[i];
        const double u = pc[0] / pc[2] * fx + cx;
        const double v = pc[1] / pc[2] * fy + cy;
        err[2 * e] = E.obs[0] - u;
        err[2 * e + 1] = E.obs[1] - v;
    }

    double chi2(int e) const
    {
        const double s = edges[e].isig, e0 = err[2 * e], e1 = err[2 * e + 1];
        return e0 * (s * e0) + e1 * (s * e1);
    }

    // RobustKernelHuber::robustify (robust_kernel_impl.cpp:78-91)
    void robustify(double e2, double rho[2]) const
    {
        const double dsqr = delta * delta;
        if (e2 <= dsqr) {
            rho[0] = e2;
            rho[1] = 1.;
        } else {
            const double sq = std::sqrt(e2);
            rho[0] = 2 * sq * delta - dsqr;
            rho[1] = delta / sq;
        }
    }

    double active_errors()
    {
        double chi = 0;
        for (int e : active) {
            compute_error(e);
            double rho[2];
            robustify(chi2(e), rho);
            chi += rho[0];
        }
        return chi;
    }

    // BlockSolver::buildSystem: EdgeSE3ProjectXYZ::linearizeOplus
    // (types_six_dof_expmap.cpp:384-420, the pose Jacobian; the point is
    // fixed) + BaseBinaryEdge::constructQuadraticForm (base_binary_edge.hpp:
    // 55-120, toNotFixed branch).
    void build_system()
    {
        for (int i = 0; i < 36; i++) H[i] = 0;
        for (int i = 0; i < 6; i++) b[i] = 0;
        for (int e : active) {
            const PoseEdge& E = edges[e];
            double pc[3];
            quat_rotate(pose.q, E.X, pc);
            for (int i = 0; i < 3; i++) pc[i] += pose.t[i];
            const double xx = pc[0], y = pc[1], z = pc[2], z_2 = z * z;
            double B[12];
            B[0] = xx * y / z_2 * fx;
            B[1] = -(1 + (xx * xx / z_2)) * fx;
            B[2] = y / z * fx;
            B[3] = -1. / z * fx;
            B[4] = 0;
            B[5] = xx / z_2 * fx;
            B[6] = (1 + y * y / z_2) * fy;
            B[7] = -xx * y / z_2 * fy;
            B[8] = -xx / z * fy;
            B[9] = 0;
            B[10] = -1. / z * fy;
            B[11] = y / z_2 * fy;
            double rho[2];
            robustify(chi2(e), rho);
            const double s = E.isig, w = rho[1] * s;
            const double om0 = -(s * err[2 * e]) * rho[1], om1 = -(s * err[2 * e + 1]) * rho[1];
            for (int i = 0; i < 6; i++) b[i] += B[i] * om0 + B[6 + i] * om1;
            for (int i = 0; i < 6; i++)
                for (int j = 0; j < 6; j++) H[i * 6 + j] += (B[i] * w) * B[j] + (B[6 + i] * w) * B[6 + j];
        }
    }

    enum Result { OK, TERMINATE };

    // OptimizationAlgorithmLevenberg::solve (levenberg.cpp:61-164) for the
    // single free vertex: the Schur complement is empty, so the reduced
    // system is Hpp + lambda I solved by LinearSolverDense.
    Result solve(int iteration, int& trials, PoseStats& st, double& last_chi)
    {
        double currentChi = active_errors();
        const double iniChi = currentChi;
        build_system();
        if (iteration == 0) {
            double m = 0;
            for (int j = 0; j < 6; j++) m = std::max(std::fabs(H[7 * j]), m);
            lambda = 1e-5 * m;
            ni = 2;
            nBad = 0;
        }
        double rho = 0;
        int qmax = 0;
        do {
            const SE3 backup = pose;
            double Hs[36];
            for (int i = 0; i < 36; i++) Hs[i] = H[i];
            for (int j = 0; j < 6; j++) Hs[7 * j] += lambda;
            const bool ok2 = ldlt_solve(6, Hs, b, x);
            if (!ok2) {
                // LinearSolverDense leaves x untouched on failure; the step
                // is rejected below (tempChi = DBL_MAX), taken here as x = 0.
                st.not_posdef++;
                for (int i = 0; i < 6; i++) x[i] = 0;
            } else {
                pose = se3_mul(se3_exp(x), pose);
            }
            double tempChi = active_errors();
            if (!ok2) tempChi = std::numeric_limits<double>::max();
            rho = currentChi - tempChi;
            double scale = 0;
            for (int j = 0; j < 6; j++) scale += x[j] * (lambda * x[j] + b[j]);
            scale += 1e-3;
            rho /= scale;
            if (rho > 0 && std::isfinite(tempChi)) {
                double alpha = 1. - std::pow((2 * rho - 1), 3);
                alpha = std::min(alpha, 2. / 3.);
                lambda *= std::max(1. / 3., alpha);
                ni = 2;
                currentChi = tempChi;
            } else {
                lambda *= ni;
                ni *= 2;
                pose = backup;   // pop(); the edges keep the trial's errors
            }
            qmax++;
            trials++;
        } while (rho < 0 && qmax < 10);
        last_chi = currentChi;
        if (qmax == 10 || rho == 0) return TERMINATE;
        if ((iniChi - currentChi) * 1e3 < iniChi) nBad++;
        else nBad = 0;
        if (nBad >= 3) return TERMINATE;
        return OK;
    }
};

}  // namespace

int pose_optimization(float Tcw[16], const float cam[4], int n, const float* kp_un, const float* inv_sigma2,
                      const uint8_t* has_mp, const float* mp_xyz, uint8_t* outlier, PoseStats* stats)
{
    PoseStats st;
    PoseOpt o;
    // Converter::toSE3Quat (src/Converter.cc:38-48): SE3Quat(R, t) =
    // Quaterniond(R) then normalizeRotation().
    double R[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) R[i * 3 + j] = Tcw[i * 4 + j];
    o.pose.q = quat_from_matrix(R);
    for (int i = 0; i < 3; i++) o.pose.t[i] = Tcw[i * 4 + 3];
    se3_normalize(o.pose);
    o.fx = cam[0];
    o.fy = cam[1];
    o.cx = cam[2];
    o.cy = cam[3];
    o.delta = (double)(float)std::sqrt(5.991);   // const float delta = sqrt(5.991)  (:188)
    int nInitial = 0;
    for (int i = 0; i < n; i++) {
        if (!has_mp[i]) continue;
        PoseEdge E;
        E.obs[0] = kp_un[2 * i];
        E.obs[1] = kp_un[2 * i + 1];
        E.isig = inv_sigma2[i];
        for (int k = 0; k < 3; k++) E.X[k] = mp_xyz[3 * i + k];
        E.kp = i;
        o.edges.push_back(E);
        outlier[i] = 0;
        nInitial++;
    }
    const int nE = (int)o.edges.size();
    o.level.assign(nE, 0);
    o.err.assign(2 * nE, 0.0);
    const float chi2th[4] = {9.210f, 7.378f, 5.991f, 5.991f};
    const int its[4] = {10, 10, 7, 5};
    int nBad = 0;
    for (int it = 0; it < 4; it++) {
        st.rounds = it + 1;
        // initializeOptimization(0): the level-0 edges, insertion order
        o.active.clear();
        for (int e = 0; e < nE; e++)
            if (o.level[e] == 0) o.active.push_back(e);
        // optimize(its[it]); with no active edge the pose is not in the
        // index map and optimize() returns -1 without touching anything
        if (!o.active.empty()) {
            for (int i = 0; i < its[it]; i++) {
                int trials = 0;
                double last = 0;
                const auto r = o.solve(i, trials, st, last);
                st.iterations[it]++;
                st.trials[it] += trials;
                st.chi2_final[it] = last;
                if (r != PoseOpt::OK) break;
            }
        }
        nBad = 0;
        for (int e = 0; e < nE; e++) {
            const int idx = o.edges[e].kp;
            if (outlier[idx]) o.compute_error(e);
            const double c2 = o.chi2(e);
            if (c2 > chi2th[it]) {
                outlier[idx] = 1;
                o.level[e] = 1;
                nBad++;
            } else if (c2 <= chi2th[it]) {
                outlier[idx] = 0;
                o.level[e] = 0;
            }
        }
        st.n_bad[it] = nBad;
        if (nE < 10) break;
    }
    // Converter::toCvMat(SE3Quat) (src/Converter.cc:50-72)
    double Rq[9];
    quat_to_matrix(o.pose.q, Rq);
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) Tcw[i * 4 + j] = (float)Rq[i * 3 + j];
        Tcw[i * 4 + 3] = (float)o.pose.t[i];
    }
    Tcw[12] = 0.f;
    Tcw[13] = 0.f;
    Tcw[14] = 0.f;
    Tcw[15] = 1.f;
    if (stats) *stats = st;
    return nInitial - nBad;
}

}  // namespace orbref
