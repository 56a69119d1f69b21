// ORACLE -- TEST INFRASTRUCTURE ONLY (see ref_common.h, ref_lba.h).
#include "ref_lba.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>
#include <numeric>

namespace orbref {

// ---------------------------------------------------------------------------
// Eigen quaternion / matrix primitives used by g2o's SE3Quat (se3quat.h).
// ---------------------------------------------------------------------------
Quat quat_mul(const Quat& a, const Quat& b)
{
    Quat r;
    r.w = a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z;
    r.x = a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y;
    r.y = a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z;
    r.z = a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x;
    return r;
}

static void cross(const double a[3], const double b[3], double o[3])
{
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}

// Eigen Quaternion::_transformVector: uv = 2 q.vec x v; v + w uv + q.vec x uv
void quat_rotate(const Quat& q, const double v[3], double out[3])
{
    const double qv[3] = {q.x, q.y, q.z};
    double uv[3], uv2[3];
    cross(qv, v, uv);
    for (int i = 0; i < 3; i++) uv[i] += uv[i];
    cross(qv, uv, uv2);
    for (int i = 0; i < 3; i++) out[i] = v[i] + q.w * uv[i] + uv2[i];
}

void quat_to_matrix(const Quat& q, double R[9])
{
    const double tx = 2 * q.x, ty = 2 * q.y, tz = 2 * q.z;
    const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
    const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
    const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
    R[0] = 1 - (tyy + tzz); R[1] = txy - twz;       R[2] = txz + twy;
    R[3] = txy + twz;       R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;       R[7] = tyz + twx;       R[8] = 1 - (txx + tyy);
}

// Eigen quaternionbase_assign_impl<3x3>
Quat quat_from_matrix(const double m[9])
{
    Quat q;
    double t = m[0] + m[4] + m[8];
    if (t > 0) {
        t = std::sqrt(t + 1.0);
        q.w = 0.5 * t;
        t = 0.5 / t;
        q.x = (m[7] - m[5]) * t;
        q.y = (m[2] - m[6]) * t;
        q.z = (m[3] - m[1]) * t;
    } else {
        int i = 0;
        if (m[4] > m[0]) i = 1;
        if (m[8] > m[i * 4]) i = 2;
        const int j = (i + 1) % 3, k = (j + 1) % 3;
        t = std::sqrt(m[i * 4] - m[j * 4] - m[k * 4] + 1.0);
        double c[3];
        c[i] = 0.5 * t;
        t = 0.5 / t;
        q.w = (m[k * 3 + j] - m[j * 3 + k]) * t;
        c[j] = (m[j * 3 + i] + m[i * 3 + j]) * t;
        c[k] = (m[k * 3 + i] + m[i * 3 + k]) * t;
        q.x = c[0];
        q.y = c[1];
        q.z = c[2];
    }
    return q;
}

void se3_normalize(SE3& s)
{
    if (s.q.w < 0) {
        s.q.x = -s.q.x;
        s.q.y = -s.q.y;
        s.q.z = -s.q.z;
        s.q.w = -s.q.w;
    }
    const double n = std::sqrt(s.q.x * s.q.x + s.q.y * s.q.y + s.q.z * s.q.z + s.q.w * s.q.w);
    s.q.x /= n;
    s.q.y /= n;
    s.q.z /= n;
    s.q.w /= n;
}

static void mat3_mul(const double A[9], const double B[9], double C[9])
{
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) C[i * 3 + j] = A[i * 3] * B[j] + A[i * 3 + 1] * B[3 + j] + A[i * 3 + 2] * B[6 + j];
}

// SE3Quat::exp (se3quat.h:223-257)
SE3 se3_exp(const double u[6])
{
    const double om[3] = {u[0], u[1], u[2]}, up[3] = {u[3], u[4], u[5]};
    const double theta = std::sqrt(om[0] * om[0] + om[1] * om[1] + om[2] * om[2]);
    const double Om[9] = {0, -om[2], om[1], om[2], 0, -om[0], -om[1], om[0], 0};
    double Om2[9], R[9], V[9];
    mat3_mul(Om, Om, Om2);
    if (theta < 0.00001) {
        for (int i = 0; i < 9; i++) R[i] = (i % 4 == 0 ? 1.0 : 0.0) + Om[i] + Om2[i];
        std::memcpy(V, R, sizeof(R));
    } else {
        const double s = std::sin(theta), c = std::cos(theta);
        const double a = s / theta, b = (1 - c) / (theta * theta), d = (theta - s) / std::pow(theta, 3);
        for (int i = 0; i < 9; i++) {
            const double I = (i % 4 == 0 ? 1.0 : 0.0);
            R[i] = I + a * Om[i] + b * Om2[i];
            V[i] = I + b * Om[i] + d * Om2[i];
        }
    }
    SE3 r;
    r.q = quat_from_matrix(R);
    for (int i = 0; i < 3; i++) r.t[i] = V[i * 3] * up[0] + V[i * 3 + 1] * up[1] + V[i * 3 + 2] * up[2];
    se3_normalize(r);
    return r;
}

// SE3Quat::operator* (se3quat.h:104-110)
SE3 se3_mul(const SE3& a, const SE3& b)
{
    SE3 r = a;
    double rt[3];
    quat_rotate(a.q, b.t, rt);
    for (int i = 0; i < 3; i++) r.t[i] += rt[i];
    r.q = quat_mul(a.q, b.q);
    se3_normalize(r);
    return r;
}

static void se3_map(const SE3& s, const double p[3], double out[3])
{
    quat_rotate(s.q, p, out);
    for (int i = 0; i < 3; i++) out[i] += s.t[i];
}

// Eigen compute_inverse<3x3> (cofactors, result(i,j) = cof(j,i)/det)
static void inverse3(const double m[9], double r[9])
{
    auto M = [&](int i, int j) { return m[i * 3 + j]; };
    auto cof = [&](int i, int j) {
        const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
        return M(i1, j1) * M(i2, j2) - M(i1, j2) * M(i2, j1);
    };
    const double c0 = cof(0, 0), c1 = cof(1, 0), c2 = cof(2, 0);
    const double det = c0 * M(0, 0) + c1 * M(1, 0) + c2 * M(2, 0);
    const double inv = 1.0 / det;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) r[i * 3 + j] = cof(j, i) * inv;
}

// ---------------------------------------------------------------------------
// Sparse optimiser restatement
// ---------------------------------------------------------------------------
namespace {

struct Optimizer {
    LBAInput& in;
    std::vector<uint8_t> edge_removed;
    // initializeOptimization state
    std::vector<int> active_edges;       // insertion (id) order
    std::vector<int> pose_h, point_h;    // hessian index or -1
    std::vector<int> iv_poses, iv_points;
    std::vector<std::vector<int>> point_edges;   // per point hessian idx: edges sorted by pose hessian idx
    // per-edge last computed error
    std::vector<double> err;
    // system
    std::vector<double> Hpp, Hll, Hpl, b, x, coef;   // Hpp: 36/pose, Hll: 9/point, Hpl: 18/edge (6x3)
    int nP = 0, nL = 0;
    double lambda = 0, ni = 2;
    int nBad = 0;
    bool abort_flag = false;

    explicit Optimizer(LBAInput& i) : in(i), edge_removed(i.n_edges, 0), err(2 * i.n_edges, 0.0) {}

    void initialize()
    {
        active_edges.clear();
        std::vector<uint8_t> pose_act(in.n_poses, 0), pt_act(in.n_points, 0);
        for (int e = 0; e < in.n_edges; e++) {
            if (edge_removed[e]) continue;
            active_edges.push_back(e);   // the point vertex is never fixed
            pose_act[in.edge_pose[e]] = 1;
            pt_act[in.edge_point[e]] = 1;
        }
        std::vector<int> ps, ls;
        for (int p = 0; p < in.n_poses; p++)
            if (pose_act[p] && !in.pose_fixed[p]) ps.push_back(p);
        for (int l = 0; l < in.n_points; l++)
            if (pt_act[l]) ls.push_back(l);
        std::stable_sort(ps.begin(), ps.end(), [&](int a, int b2) { return in.pose_id[a] < in.pose_id[b2]; });
        std::stable_sort(ls.begin(), ls.end(), [&](int a, int b2) { return in.point_id[a] < in.point_id[b2]; });
        iv_poses = ps;
        iv_points = ls;
        pose_h.assign(in.n_poses, -1);
        point_h.assign(in.n_points, -1);
        for (size_t i = 0; i < ps.size(); i++) pose_h[ps[i]] = (int)i;
        for (size_t i = 0; i < ls.size(); i++) point_h[ls[i]] = (int)i;
        nP = (int)ps.size();
        nL = (int)ls.size();
        point_edges.assign(nL, {});
        for (int e : active_edges) {
            const int l = point_h[in.edge_point[e]];
            if (pose_h[in.edge_pose[e]] >= 0) point_edges[l].push_back(e);
        }
        for (auto& v : point_edges)
            std::stable_sort(v.begin(), v.end(), [&](int a, int b2) { return pose_h[in.edge_pose[a]] < pose_h[in.edge_pose[b2]]; });
    }

    const double* cam(int e) const { return &in.pose_cam[4 * in.edge_pose[e]]; }

    void compute_error(int e)
    {
        double pc[3];
        se3_map(in.poses[in.edge_pose[e]], &in.points[3 * in.edge_point[e]], pc);
        const double* c = cam(e);
        const double u = pc[0] / pc[2] * c[0] + c[2];
        const double v = pc[1] / pc[2] * c[1] + c[3];
        err[2 * e] = in.edge_obs[2 * e] - u;
        err[2 * e + 1] = in.edge_obs[2 * e + 1] - v;
    }

    void compute_active_errors()
    {
        for (int e : active_edges) compute_error(e);
    }

    double chi2(int e) const
    {
        const double s = in.edge_inv_sigma2[e];
        const double e0 = err[2 * e], e1 = err[2 * e + 1];
        return e0 * (s * e0) + e1 * (s * e1);
    }

    void robustify(double e2, double rho[2]) const
    {
        const double delta = in.huber_delta, dsqr = delta * delta;
        if (e2 <= dsqr) {
            rho[0] = e2;
            rho[1] = 1.;
        } else {
            const double sqrte = std::sqrt(e2);
            rho[0] = 2 * sqrte * delta - dsqr;
            rho[1] = delta / sqrte;
        }
    }

    double robust_chi2() const
    {
        double chi = 0;
        for (int e : active_edges) {
            double rho[2];
            robustify(chi2(e), rho);
            chi += rho[0];
        }
        return chi;
    }

    bool depth_positive(int e) const
    {
        double pc[3];
        se3_map(in.poses[in.edge_pose[e]], &in.points[3 * in.edge_point[e]], pc);
        return pc[2] > 0.0;
    }

    // EdgeSE3ProjectXYZ::linearizeOplus (types_six_dof_expmap.cpp:384-420)
    void linearize(int e, double A[6], double B[12]) const
    {
        const SE3& T = in.poses[in.edge_pose[e]];
        double pc[3];
        se3_map(T, &in.points[3 * in.edge_point[e]], pc);
        const double x = pc[0], y = pc[1], z = pc[2], z_2 = z * z;
        const double* c = cam(e);
        const double fx = c[0], fy = c[1];
        const double tmp[6] = {fx, 0, -x / z * fx, 0, fy, -y / z * fy};
        double R[9];
        quat_to_matrix(T.q, R);
        const double s = -1. / z;
        for (int i = 0; i < 2; i++)
            for (int j = 0; j < 3; j++)
                A[i * 3 + j] = (s * tmp[i * 3]) * R[j] + (s * tmp[i * 3 + 1]) * R[3 + j] + (s * tmp[i * 3 + 2]) * R[6 + j];
        B[0] = x * y / z_2 * fx;
        B[1] = -(1 + (x * x / z_2)) * fx;
        B[2] = y / z * fx;
        B[3] = -1. / z * fx;
        B[4] = 0;
        B[5] = x / z_2 * fx;
        B[6] = (1 + y * y / z_2) * fy;
        B[7] = -x * y / z_2 * fy;
        B[8] = -x / z * fy;
        B[9] = 0;
        B[10] = -1. / z * fy;
        B[11] = y / z_2 * fy;
    }

    // BlockSolver::buildSystem + BaseBinaryEdge::constructQuadraticForm
    void build_system()
    {
        Hpp.assign(36 * nP, 0.0);
        Hll.assign(9 * nL, 0.0);
        Hpl.assign(18 * (size_t)in.n_edges, 0.0);
        b.assign(6 * nP + 3 * nL, 0.0);
        for (int e : active_edges) {
            double A[6], Bm[12];
            linearize(e, A, Bm);
            const double s = in.edge_inv_sigma2[e];
            double rho[2];
            robustify(chi2(e), rho);
            const double w = rho[1] * s;   // weightedOmega = rho1 * I * invSigma2
            const double om_r[2] = {-(s * err[2 * e]) * rho[1], -(s * err[2 * e + 1]) * rho[1]};
            const int lh = point_h[in.edge_point[e]], ph = pose_h[in.edge_pose[e]];
            double* bl = &b[6 * nP + 3 * lh];
            double* hl = &Hll[9 * lh];
            for (int i = 0; i < 3; i++) bl[i] += A[i] * om_r[0] + A[3 + i] * om_r[1];
            for (int i = 0; i < 3; i++)
                for (int j = 0; j < 3; j++) hl[i * 3 + j] += (A[i] * w) * A[j] + (A[3 + i] * w) * A[3 + j];
            if (ph >= 0) {
                double* hpl = &Hpl[18 * (size_t)e];
                for (int i = 0; i < 6; i++)
                    for (int j = 0; j < 3; j++) hpl[i * 3 + j] += (Bm[i] * w) * A[j] + (Bm[6 + i] * w) * A[3 + j];
                double* bp = &b[6 * ph];
                double* hp = &Hpp[36 * ph];
                for (int i = 0; i < 6; i++) bp[i] += Bm[i] * om_r[0] + Bm[6 + i] * om_r[1];
                for (int i = 0; i < 6; i++)
                    for (int j = 0; j < 6; j++) hp[i * 6 + j] += (Bm[i] * w) * Bm[j] + (Bm[6 + i] * w) * Bm[6 + j];
            }
        }
    }

    double lambda_init() const
    {
        double m = 0;
        for (int p = 0; p < nP; p++)
            for (int j = 0; j < 6; j++) m = std::max(std::fabs(Hpp[36 * p + 7 * j]), m);
        for (int l = 0; l < nL; l++)
            for (int j = 0; j < 3; j++) m = std::max(std::fabs(Hll[9 * l + 4 * j]), m);
        return 1e-5 * m;
    }

    // BlockSolver::solve (block_solver.hpp:354-486) with lambda on the diagonals.
    bool solve_schur()
    {
        const int dp = 6 * nP;
        std::vector<double> S((size_t)dp * dp, 0.0);
        for (int p = 0; p < nP; p++)
            for (int i = 0; i < 6; i++)
                for (int j = 0; j < 6; j++)
                    S[(size_t)(6 * p + i) * dp + 6 * p + j] = Hpp[36 * p + 6 * i + j] + (i == j ? lambda : 0.0);
        coef.assign(dp, 0.0);
        std::vector<double> Dinv(9 * nL);
        for (int l = 0; l < nL; l++) {
            double D[9];
            for (int k = 0; k < 9; k++) D[k] = Hll[9 * l + k] + (k % 4 == 0 ? lambda : 0.0);
            inverse3(D, &Dinv[9 * l]);
            const double* Di = &Dinv[9 * l];
            const double* bl = &b[dp + 3 * l];
            double db[3];
            for (int i = 0; i < 3; i++) db[i] = Di[3 * i] * bl[0] + Di[3 * i + 1] * bl[1] + Di[3 * i + 2] * bl[2];
            const auto& col = point_edges[l];
            for (size_t a = 0; a < col.size(); a++) {
                const int e1 = col[a];
                const int i1 = pose_h[in.edge_pose[e1]];
                const double* Bi = &Hpl[18 * (size_t)e1];
                double BD[18];
                for (int r = 0; r < 6; r++)
                    for (int c = 0; c < 3; c++)
                        BD[r * 3 + c] = Bi[r * 3] * Di[c] + Bi[r * 3 + 1] * Di[3 + c] + Bi[r * 3 + 2] * Di[6 + c];
                for (int r = 0; r < 6; r++) coef[6 * i1 + r] += Bi[r * 3] * db[0] + Bi[r * 3 + 1] * db[1] + Bi[r * 3 + 2] * db[2];
                for (size_t bb = a; bb < col.size(); bb++) {
                    const int e2 = col[bb];
                    const int i2 = pose_h[in.edge_pose[e2]];
                    const double* Bj = &Hpl[18 * (size_t)e2];
                    for (int r = 0; r < 6; r++)
                        for (int c = 0; c < 6; c++)
                            S[(size_t)(6 * i1 + r) * dp + 6 * i2 + c] -=
                                BD[r * 3] * Bj[c * 3] + BD[r * 3 + 1] * Bj[c * 3 + 1] + BD[r * 3 + 2] * Bj[c * 3 + 2];
                }
            }
        }
        std::vector<double> bs(dp);
        for (int i = 0; i < dp; i++) bs[i] = b[i] - coef[i];
        // symmetric fill from the upper blocks, dense LLT (stands in for CHOLMOD)
        for (int i = 0; i < dp; i++)
            for (int j = 0; j < i; j++) S[(size_t)i * dp + j] = S[(size_t)j * dp + i];
        std::vector<double> L((size_t)dp * dp, 0.0);
        for (int i = 0; i < dp; i++) {
            for (int j = 0; j <= i; j++) {
                double s = S[(size_t)i * dp + j];
                for (int k = 0; k < j; k++) s -= L[(size_t)i * dp + k] * L[(size_t)j * dp + k];
                if (i == j) {
                    if (!(s > 0)) return false;
                    L[(size_t)i * dp + i] = std::sqrt(s);
                } else {
                    L[(size_t)i * dp + j] = s / L[(size_t)j * dp + j];
                }
            }
        }
        x.assign(dp + 3 * nL, 0.0);
        std::vector<double> y(dp);
        for (int i = 0; i < dp; i++) {
            double s = bs[i];
            for (int k = 0; k < i; k++) s -= L[(size_t)i * dp + k] * y[k];
            y[i] = s / L[(size_t)i * dp + i];
        }
        for (int i = dp - 1; i >= 0; i--) {
            double s = y[i];
            for (int k = i + 1; k < dp; k++) s -= L[(size_t)k * dp + i] * x[k];
            x[i] = s / L[(size_t)i * dp + i];
        }
        // landmarks: xl = Dinv (bl - B^T xp)   (HplCCS->rightMultiply, DInv multiply)
        for (int l = 0; l < nL; l++) {
            double cl[3] = {b[dp + 3 * l], b[dp + 3 * l + 1], b[dp + 3 * l + 2]};
            for (int e : point_edges[l]) {
                const int i1 = pose_h[in.edge_pose[e]];
                const double* Bi = &Hpl[18 * (size_t)e];
                for (int c = 0; c < 3; c++) {
                    double acc = 0;
                    for (int r = 0; r < 6; r++) acc += Bi[r * 3 + c] * (-x[6 * i1 + r]);
                    cl[c] += acc;
                }
            }
            const double* Di = &Dinv[9 * l];
            for (int i = 0; i < 3; i++) x[dp + 3 * l + i] = Di[3 * i] * cl[0] + Di[3 * i + 1] * cl[1] + Di[3 * i + 2] * cl[2];
        }
        return true;
    }

    void apply_update()
    {
        for (int p = 0; p < nP; p++) {
            const int v = iv_poses[p];
            in.poses[v] = se3_mul(se3_exp(&x[6 * p]), in.poses[v]);
        }
        const int dp = 6 * nP;
        for (int l = 0; l < nL; l++) {
            const int v = iv_points[l];
            for (int i = 0; i < 3; i++) in.points[3 * v + i] += x[dp + 3 * l + i];
        }
    }

    double compute_scale() const
    {
        double s = 0;
        for (size_t j = 0; j < x.size(); j++) s += x[j] * (lambda * x[j] + b[j]);
        return s;
    }

    enum Result { OK, TERMINATE, FAIL };

    // OptimizationAlgorithmLevenberg::solve (levenberg.cpp:61-164)
    Result solve(int iteration, int& trials, LBAStats& st)
    {
        compute_active_errors();
        double currentChi = robust_chi2();
        const double iniChi = currentChi;
        build_system();
        if (iteration == 0) {
            lambda = lambda_init();
            ni = 2;
            nBad = 0;
        }
        double rho = 0;
        int qmax = 0;
        do {
            std::vector<SE3> bp(in.poses);
            std::vector<double> bpt(in.points);
            const bool ok2 = solve_schur();
            if (!ok2) {
                st.not_posdef++;
                x.assign(6 * nP + 3 * nL, 0.0);
            }
            if (ok2) apply_update();
            compute_active_errors();
            double tempChi = robust_chi2();
            if (!ok2) tempChi = std::numeric_limits<double>::max();
            rho = currentChi - tempChi;
            double scale = compute_scale();
            scale += 1e-3;
            rho /= scale;
            if (rho > 0 && std::isfinite(tempChi)) {
                double alpha = 1. - std::pow((2 * rho - 1), 3);
                alpha = std::min(alpha, 2. / 3.);
                const double scaleFactor = std::max(1. / 3., alpha);
                lambda *= scaleFactor;
                ni = 2;
                currentChi = tempChi;
            } else {
                lambda *= ni;
                ni *= 2;
                in.poses = bp;
                in.points = bpt;
            }
            qmax++;
            trials++;
        } while (rho < 0 && qmax < 10 && !abort_flag);
        st_last_chi = currentChi;
        if (qmax == 10 || rho == 0) return TERMINATE;
        if ((iniChi - currentChi) * 1e3 < iniChi) nBad++;
        else nBad = 0;
        if (nBad >= 3) return TERMINATE;
        return OK;
    }
    double st_last_chi = 0;

    // SparseOptimizer::optimize (sparse_optimizer.cpp:354-419)
    void optimize(int iterations, int pass, LBAStats& st)
    {
        initialize();
        if (active_edges.empty() || (nP + nL) == 0) return;
        bool ok = true;
        int it = 0;
        for (int i = 0; i < iterations && ok; i++) {
            int trials = 0;
            if (i == 0) {
                compute_active_errors();
                st.chi2_initial[pass] = robust_chi2();
            }
            const Result r = solve(i, trials, st);
            st.trials[pass] += trials;
            ok = (r == OK);
            it++;
        }
        st.iterations[pass] = it;
        st.chi2_final[pass] = st_last_chi;
    }
};

}  // namespace

void edge_linearize_for_test(LBAInput& in, double err[2], double A[6], double B[12])
{
    Optimizer opt(in);
    opt.compute_error(0);
    err[0] = opt.err[0];
    err[1] = opt.err[1];
    opt.linearize(0, A, B);
}

// Optimizer::LocalBundleAdjustment core (src/Optimizer.cc:449-535).
void local_ba(LBAInput& in, int iters0, int iters1, std::vector<uint8_t>& edge_status,
              std::vector<uint8_t>& point_bad, LBAStats& st)
{
    Optimizer opt(in);
    edge_status.assign(in.n_edges, 0);
    point_bad.assign(in.n_points, 0);
    std::vector<int> nobs(in.point_nobs);
    opt.optimize(iters0, 0, st);
    // outlier pass 1 (:452-470): erase observation, remove edge
    for (int e = 0; e < in.n_edges; e++) {
        const int p = in.edge_point[e];
        if (point_bad[p]) continue;
        if (opt.chi2(e) > in.chi2_threshold || !opt.depth_positive(e)) {
            if (--nobs[p] <= 2) point_bad[p] = 1;   // MapPoint::EraseObservation -> SetBadFlag
            opt.edge_removed[e] = 1;
            edge_status[e] = 1;
            st.n_outliers[0]++;
        }
    }
    opt.optimize(iters1, 1, st);
    // outlier pass 2 (:497-515): erase observation only
    for (int e = 0; e < in.n_edges; e++) {
        if (opt.edge_removed[e]) continue;
        const int p = in.edge_point[e];
        if (point_bad[p]) continue;
        if (opt.chi2(e) > in.chi2_threshold || !opt.depth_positive(e)) {
            if (--nobs[p] <= 2) point_bad[p] = 1;
            edge_status[e] = 2;
            st.n_outliers[1]++;
        }
    }
}

}  // namespace orbref
