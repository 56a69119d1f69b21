"""An independent numpy restatement of Optimizer::LocalBundleAdjustment's
solver core (src/Optimizer.cc:449-535 with the g2o it links), against the
oracle's restatement (oracle/ref_lba.cpp) on small problems.

Written from the reference and g2o's published code paths, not from the
oracle's code, and deliberately in a different form: the full (dense) normal
equations solved by a Cholesky factorisation instead of the Schur complement
over the points, the quaternion rotation of SE3Quat::map as Eigen evaluates
it, Eigen's rotation-matrix-to-quaternion conversion.  The two agree to
rounding, so the bar is 1e-8 on poses and points, identical LM iteration and
trial counts, identical outlier decisions and MapPoint bad flags.

* EdgeSE3ProjectXYZ (types_six_dof_expmap.h / .cpp): e = obs - (fx X/Z + cx,
  fy Y/Z + cy) at the camera-frame point q p + t; Jacobians of linearizeOplus
  (point: -1/Z [fx 0 -X fx/Z; 0 fy -Y fy/Z] R; pose: [omega, upsilon] order);
* RobustKernelHuber: rho = (e2, 1) inside delta^2, (2 sqrt(e2) delta -
  delta^2, delta / sqrt(e2)) outside; the quadratic form uses rho' Omega;
* OptimizationAlgorithmLevenberg::solve (levenberg.cpp): lambda = 1e-5 max
  diag(H) at an optimize() call's first iteration, lambda added to the whole
  diagonal, rho = (chi2 - chi2_new) / (x . (lambda x + b) + 1e-3), the
  1 - (2 rho - 1)^3 rule cropped to [1/3, 2/3], ni doubling, at most 10
  trials, the nBad (Raul) stop after three iterations with less than 1e-3
  relative gain;
* VertexSE3Expmap::oplusImpl: SE3Quat::exp(update) * estimate (Rodrigues
  with the theta < 1e-5 branch, normalizeRotation after the product);
  VertexSBAPointXYZ: additive;
* the two outlier passes: chi2 of the last computeActiveErrors (the last
  trial's errors, accepted or not) above 5.991 or a non-positive depth at the
  current estimate; MapPoint::EraseObservation drops the point at <= 2
  observations and later edges of a bad point are skipped; the first pass's
  outliers leave the graph, then optimize(10).
"""
import ctypes

import numpy as np
import pytest

from orb_slam_amd import synth_ba as sb
from oracle_lib import load

CHI2_TH = 5.991


def quat_mul(a, b):   # Eigen order (x, y, z, w)
    av, aw, bv, bw = a[:3], a[3], b[:3], b[3]
    v = aw * bv + bw * av + np.cross(av, bv)
    return np.array([v[0], v[1], v[2], aw * bw - av @ bv])


def quat_rotate(q, p):   # Eigen's Quaternion * Vector3
    u, w = q[:3], q[3]
    uv = np.cross(u, p)
    uv = uv + uv
    return p + w * uv + np.cross(u, uv)


def quat_matrix(q):
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def matrix_quat(m):   # Eigen's Quaternion(const Matrix3&)
    q = np.zeros(4)
    t = np.trace(m)
    if t > 0:
        t = np.sqrt(t + 1.0)
        q[3] = 0.5 * t
        t = 0.5 / t
        q[0] = (m[2, 1] - m[1, 2]) * t
        q[1] = (m[0, 2] - m[2, 0]) * t
        q[2] = (m[1, 0] - m[0, 1]) * t
    else:
        i = 0
        if m[1, 1] > m[0, 0]:
            i = 1
        if m[2, 2] > m[i, i]:
            i = 2
        j, k = (i + 1) % 3, (i + 2) % 3
        t = np.sqrt(m[i, i] - m[j, j] - m[k, k] + 1.0)
        q[i] = 0.5 * t
        t = 0.5 / t
        q[3] = (m[k, j] - m[j, k]) * t
        q[j] = (m[j, i] + m[i, j]) * t
        q[k] = (m[k, i] + m[i, k]) * t
    return q


def normalize_rotation(q):
    if q[3] < 0:
        q = -q
    return q / np.linalg.norm(q)


def skew(v):
    return np.array([[0, -v[2], v[1]], [v[2], 0, -v[0]], [-v[1], v[0], 0]])


def se3_exp(d):
    omega, upsilon = d[:3], d[3:]
    theta = np.linalg.norm(omega)
    Om = skew(omega)
    if theta < 0.00001:
        R = np.eye(3) + Om + Om @ Om
        V = R
    else:
        Om2 = Om @ Om
        R = np.eye(3) + np.sin(theta) / theta * Om + (1 - np.cos(theta)) / (theta * theta) * Om2
        V = np.eye(3) + (1 - np.cos(theta)) / (theta * theta) * Om + (theta - np.sin(theta)) / theta ** 3 * Om2
    return normalize_rotation(matrix_quat(R)), V @ upsilon


def se3_oplus(q, t, d):   # exp(d) * (q, t)
    qe, te = se3_exp(d)
    t2 = te + quat_rotate(qe, t)
    return normalize_rotation(quat_mul(qe, q)), t2


class Graph:
    def __init__(self, prob):
        self.q = prob["pose_q"].copy()
        self.t = prob["pose_t"].copy()
        self.X = prob["points"].copy()
        self.cam = prob["pose_cam"]
        self.fixed = prob["pose_fixed"]
        self.ep, self.ek = prob["edge_point"], prob["edge_pose"]
        self.obs, self.isig = prob["edge_obs"], prob["edge_inv_sigma2"]
        self.delta = prob["huber_delta"]
        self.err = np.zeros((len(self.ep), 2))

    def pc(self, e):
        k = self.ek[e]
        return quat_rotate(self.q[k], self.X[self.ep[e]]) + self.t[k]

    def error(self, e):
        c = self.cam[self.ek[e]]
        p = self.pc(e)
        return self.obs[e] - np.array([p[0] / p[2] * c[0] + c[2], p[1] / p[2] * c[1] + c[3]])

    def robust(self, e2):
        d = self.delta
        if e2 <= d * d:
            return e2, 1.0
        s = np.sqrt(e2)
        return 2 * s * d - d * d, d / s

    def chi2(self, e):
        return self.isig[e] * (self.err[e] @ self.err[e])

    def compute_errors(self, active):
        tot = 0.0
        for e in active:
            self.err[e] = self.error(e)
            tot += self.robust(self.chi2(e))[0]
        return tot

    def optimize(self, active, iters):
        """SparseOptimizer::optimize(iters) over the active edges; returns
        (iterations run, Levenberg trials)."""
        poses = sorted({int(self.ek[e]) for e in active if not self.fixed[self.ek[e]]})
        points = sorted({int(self.ep[e]) for e in active})
        pi = {k: 6 * i for i, k in enumerate(poses)}
        li = {p: 6 * len(poses) + 3 * i for i, p in enumerate(points)}
        n = 6 * len(poses) + 3 * len(points)
        lam = ni = 0.0
        nbad = 0
        trials = 0
        it = 0
        while it < iters:
            chi = self.compute_errors(active)
            ini = chi
            H = np.zeros((n, n))
            b = np.zeros(n)
            for e in active:
                k, p = int(self.ek[e]), int(self.ep[e])
                c = self.cam[k]
                R = quat_matrix(self.q[k])
                x, y, z = quat_rotate(self.q[k], self.X[p]) + self.t[k]
                A = -1.0 / z * np.array([[c[0], 0, -x / z * c[0]], [0, c[1], -y / z * c[1]]]) @ R
                z2 = z * z
                B = np.array([[x * y / z2 * c[0], -(1 + x * x / z2) * c[0], y / z * c[0], -1 / z * c[0], 0,
                               x / z2 * c[0]],
                              [(1 + y * y / z2) * c[1], -x * y / z2 * c[1], -x / z * c[1], 0, -1 / z * c[1],
                               y / z2 * c[1]]])
                r1 = self.robust(self.chi2(e))[1]
                W = r1 * self.isig[e]
                J = np.zeros((2, n))
                J[:, li[p]:li[p] + 3] = A
                if k in pi:
                    J[:, pi[k]:pi[k] + 6] = B
                H += W * (J.T @ J)
                b += -W * (J.T @ self.err[e])
            if it == 0:
                lam = 1e-5 * np.max(np.diag(H))
                ni = 2.0
                nbad = 0
            q = 0
            while True:
                saved = (self.q.copy(), self.t.copy(), self.X.copy())
                try:
                    L = np.linalg.cholesky(H + lam * np.eye(n))
                    dx = np.linalg.solve(L.T, np.linalg.solve(L, b))
                    ok = True
                except np.linalg.LinAlgError:
                    dx, ok = np.zeros(n), False
                if ok:
                    for k in poses:
                        self.q[k], self.t[k] = se3_oplus(self.q[k], self.t[k], dx[pi[k]:pi[k] + 6])
                    for p in points:
                        self.X[p] = self.X[p] + dx[li[p]:li[p] + 3]
                tmp = self.compute_errors(active)
                if not ok:
                    tmp = np.finfo(np.float64).max
                rho = (chi - tmp) / (dx @ (lam * dx + b) + 1e-3)
                if rho > 0 and np.isfinite(tmp):
                    alpha = min(1.0 - (2 * rho - 1) ** 3, 2.0 / 3.0)
                    lam *= max(1.0 / 3.0, alpha)
                    ni = 2.0
                    chi = tmp
                else:
                    lam *= ni
                    ni *= 2
                    self.q, self.t, self.X = saved
                q += 1
                if not (rho < 0 and q < 10):
                    break
            trials += q
            it += 1
            if q == 10 or rho == 0:
                break
            nbad = nbad + 1 if (ini - chi) * 1e3 < ini else 0
            if nbad >= 3:
                break
        return it, trials


def local_ba(prob, i0=5, i1=10):
    g = Graph(prob)
    ne = len(g.ep)
    nobs = prob["point_nobs"].astype(np.int64).copy()
    bad = np.zeros(len(nobs), np.uint8)
    status = np.zeros(ne, np.uint8)
    stats = []
    active = list(range(ne))
    for pss, iters in ((1, i0), (2, i1)):
        stats.append(g.optimize(active, iters))
        for e in active:
            p = g.ep[e]
            if bad[p]:
                continue
            if g.chi2(e) > CHI2_TH or not g.pc(e)[2] > 0.0:
                nobs[p] -= 1
                if nobs[p] <= 2:
                    bad[p] = 1
                status[e] = pss
        active = [e for e in active if status[e] == 0]
    return g, status, bad, stats


def run_ref(prob, i0=5, i1=10):
    L = load()
    L.orbx_ref_lba.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                               ctypes.c_void_p]
    p, arrs = sb.to_ctypes(prob)
    es = np.zeros(p.n_edges, np.uint8)
    pb = np.zeros(p.n_points, np.uint8)
    st = sb.BAStats()
    assert L.orbx_ref_lba(ctypes.byref(p), i0, i1, es.ctypes.data, pb.ctypes.data, ctypes.byref(st)) == 0
    return arrs, es, pb, st


@pytest.mark.parametrize("kw", [
    dict(n_kf=5, n_points=90, seed=3, outlier_frac=0.06),
    dict(n_kf=4, n_points=70, seed=11, outlier_frac=0.1, pix_noise=2.0),
    dict(n_kf=4, n_points=60, seed=5, outlier_frac=0.05, normalized=True, info_scale=500.0 ** 2),
    # far from the solution: rejected Levenberg trials (pop, lambda * ni) in pass 2 / pass 1
    dict(n_kf=3, n_points=30, seed=1, outlier_frac=0.1, pose_noise=(0.4, 1.0), point_noise=1.0, pix_noise=1.5),
    dict(n_kf=3, n_points=30, seed=2, outlier_frac=0.1, pose_noise=(0.4, 1.0), point_noise=1.0, pix_noise=1.5),
])
def test_local_ba_matches_oracle(kw):
    prob = sb.make_problem(n_fixed_extra=1, **kw)
    g, status, bad, stats = local_ba(prob)
    ra, res, rpb, rst = run_ref(prob)
    assert np.abs(g.q - ra["pose_q"]).max() <= 1e-8
    assert np.abs(g.t - ra["pose_t"]).max() <= 1e-8
    assert np.abs(g.X - ra["points"]).max() <= 1e-8
    assert np.array_equal(status, res), (np.count_nonzero(status), np.count_nonzero(res))
    assert np.array_equal(bad, rpb)
    assert [s[0] for s in stats] == list(rst.iterations)
    assert [s[1] for s in stats] == list(rst.levenberg_trials)
    assert list(rst.n_outliers) == [int(np.count_nonzero(status == 1)), int(np.count_nonzero(status == 2))]
    assert np.count_nonzero(status) > 0   # the outlier passes did something
