"""Synthetic local-BA problems.

Keyframes on a 2 m arc look at a point cloud 2-6 m away; each point is seen
by 3-10 keyframes.  Observations = true projection + N(0, 1 px) * 1.2^octave
(octave uniform 0..7), information = invSigma2(octave) computed in float the
way Frame/KeyFrame do (src/Frame.cc:94-106).  A few gross outliers exercise
the two outlier passes.  Initial poses are perturbed by ~0.01 rad / 0.02 m and
points by 0.02 m.  KF 0 and `n_fixed_extra` further keyframes are fixed
(the "fixed cameras" of src/Optimizer.cc:322-338).

Returns numpy arrays laid out as include/orbx.h's orbx_ba_problem.
"""
import ctypes

import numpy as np


def _rot_to_quat(R):
    """Eigen Quaterniond(R) (quaternionbase_assign_impl), returns x,y,z,w."""
    t = np.trace(R)
    if t > 0:
        t = np.sqrt(t + 1.0)
        w = 0.5 * t
        t = 0.5 / t
        return np.array([(R[2, 1] - R[1, 2]) * t, (R[0, 2] - R[2, 0]) * t, (R[1, 0] - R[0, 1]) * t, w])
    i = 0
    if R[1, 1] > R[0, 0]:
        i = 1
    if R[2, 2] > R[i, i]:
        i = 2
    j, k = (i + 1) % 3, (i + 2) % 3
    t = np.sqrt(R[i, i] - R[j, j] - R[k, k] + 1.0)
    c = np.zeros(3)
    c[i] = 0.5 * t
    t = 0.5 / t
    w = (R[k, j] - R[j, k]) * t
    c[j] = (R[j, i] + R[i, j]) * t
    c[k] = (R[k, i] + R[i, k]) * t
    return np.array([c[0], c[1], c[2], w])


def _normalize_q(q):
    if q[3] < 0:
        q = -q
    return q / np.linalg.norm(q)


def _exp_so3(w):
    th = np.linalg.norm(w)
    K = np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]])
    if th < 1e-12:
        return np.eye(3) + K
    return np.eye(3) + np.sin(th) / th * K + (1 - np.cos(th)) / th ** 2 * K @ K


def inv_sigma2_table(nlevels=8, scale=1.2):
    s = np.float32(1.0)
    out = []
    for i in range(nlevels):
        if i > 0:
            s = np.float32(s * np.float32(scale))
        sig2 = np.float32(s * s)
        out.append(float(np.float32(np.float32(1.0) / sig2)))
    return np.array(out)


def make_problem(n_kf=20, n_points=2000, n_fixed_extra=2, seed=0, outlier_frac=0.01,
                 w=640, h=480, fx=500.0, fy=500.0, cx=320.0, cy=240.0,
                 pose_noise=(0.01, 0.02), point_noise=0.02, pix_noise=1.0,
                 normalized=False, info_scale=1.0, near_points=0):
    """normalized: observations and camera in normalised image coordinates
    ((u - cx) / fx, (v - cy) / fy, camera fx = fy = 1, cx = cy = 0) instead
    of pixels; info_scale multiplies every edge's information (with a
    normalised camera, fx^2 keeps the chi2 of the pixel problem);
    near_points: that many points moved to 2-8 cm in front of keyframe 1
    (large Jacobians).  These exercise the reduced system outside the pixel
    regime."""
    rng = np.random.default_rng(seed)
    n_poses = n_kf + n_fixed_extra
    center = np.array([0.0, 0.0, 4.0])
    poses_true = []
    for k in range(n_poses):
        ang = -0.25 + 0.5 * k / max(1, n_poses - 1)            # 2 m arc at radius 4
        c = center + 4.0 * np.array([np.sin(ang), 0.05 * np.cos(3 * ang), -np.cos(ang)])
        fwd = center - c
        fwd /= np.linalg.norm(fwd)
        right = np.cross([0.0, 1.0, 0.0], fwd)
        right /= np.linalg.norm(right)
        down = np.cross(fwd, right)
        Rwc = np.stack([right, down, fwd], 1)
        Rcw = Rwc.T
        poses_true.append((Rcw, -Rcw @ c))
    pts = center + rng.uniform([-2.0, -1.5, -2.0], [2.0, 1.5, 2.0], size=(n_points, 3))
    if near_points:
        R1, t1 = poses_true[1]
        for i in range(near_points):   # camera-frame point 2-8 cm ahead, back to world
            pc = np.array([rng.uniform(-0.01, 0.01), rng.uniform(-0.01, 0.01), rng.uniform(0.02, 0.08)])
            pts[i] = R1.T @ (pc - t1)
    isig = inv_sigma2_table()
    e_point, e_pose, e_obs, e_isig = [], [], [], []
    nobs = np.zeros(n_points, np.int32)
    for p in range(n_points):
        vis = []
        for k, (R, t) in enumerate(poses_true):
            pc = R @ pts[p] + t
            if pc[2] <= (0.01 if near_points else 0.5):
                continue
            u, v = fx * pc[0] / pc[2] + cx, fy * pc[1] / pc[2] + cy
            if 0 <= u < w and 0 <= v < h:
                vis.append((k, u, v))
        if len(vis) < (2 if p < near_points else 3):
            continue
        m = int(rng.integers(3, min(10, len(vis)) + 1))
        chosen = sorted(rng.choice(len(vis), m, replace=False))
        for ci in chosen:
            k, u, v = vis[ci]
            octave = int(rng.integers(0, 8))
            sd = pix_noise * 1.2 ** octave
            ou, ov = u + rng.normal(0, sd), v + rng.normal(0, sd)
            if rng.random() < outlier_frac:
                ou += rng.choice([-1, 1]) * rng.uniform(20, 60)
                ov += rng.choice([-1, 1]) * rng.uniform(20, 60)
            e_point.append(p)
            e_pose.append(k)
            if normalized:
                ou, ov = (ou - cx) / fx, (ov - cy) / fy
            e_obs.append((np.float32(ou), np.float32(ov)))   # cv::KeyPoint coords are float
            e_isig.append(isig[octave] * info_scale)
            nobs[p] += 1
    # keep only observed points, re-index
    used = np.nonzero(nobs)[0]
    remap = -np.ones(n_points, np.int64)
    remap[used] = np.arange(len(used))
    pts = pts[used]
    nobs = nobs[used]
    e_point = remap[np.array(e_point)].astype(np.int32)
    # perturbed initial state (float32 like cv::Mat poses/points, widened)
    q = np.zeros((n_poses, 4))
    t = np.zeros((n_poses, 3))
    fixed = np.zeros(n_poses, np.uint8)
    fixed[0] = 1
    fixed[n_kf:] = 1
    for k, (R, tt) in enumerate(poses_true):
        if not fixed[k]:
            dR = _exp_so3(rng.normal(0, pose_noise[0], 3))
            R = dR @ R
            tt = tt + rng.normal(0, pose_noise[1], 3)
        R32 = R.astype(np.float32).astype(np.float64)
        q[k] = _normalize_q(_rot_to_quat(R32))
        t[k] = tt.astype(np.float32).astype(np.float64)
    pts0 = (pts + rng.normal(0, point_noise, pts.shape)).astype(np.float32).astype(np.float64)
    maxkf = n_poses - 1
    prob = {
        "pose_q": q, "pose_t": t, "pose_fixed": fixed,
        "pose_id": np.arange(n_poses, dtype=np.int64),
        "pose_cam": np.tile([1.0, 1.0, 0.0, 0.0] if normalized else [fx, fy, cx, cy], (n_poses, 1)).astype(np.float64),
        "points": pts0, "point_id": (np.arange(len(pts0)) + maxkf + 1).astype(np.int64),
        "point_nobs": nobs.astype(np.int32),
        "edge_point": e_point, "edge_pose": np.array(e_pose, np.int32),
        "edge_obs": np.array(e_obs, np.float64), "edge_inv_sigma2": np.array(e_isig, np.float64),
        "huber_delta": float(np.float32(np.sqrt(5.991))), "chi2_threshold": 5.991,
        "points_true": pts, "poses_true": poses_true,
    }
    for k in ["pose_q", "pose_t", "pose_cam", "points", "edge_obs", "edge_inv_sigma2"]:
        prob[k] = np.ascontiguousarray(prob[k], np.float64)
    return prob


class BAProblem(ctypes.Structure):
    _fields_ = [("n_poses", ctypes.c_int), ("n_points", ctypes.c_int), ("n_edges", ctypes.c_int),
                ("pose_q", ctypes.c_void_p), ("pose_t", ctypes.c_void_p), ("pose_fixed", ctypes.c_void_p),
                ("pose_id", ctypes.c_void_p), ("pose_cam", ctypes.c_void_p), ("points", ctypes.c_void_p),
                ("point_id", ctypes.c_void_p), ("point_nobs", ctypes.c_void_p), ("edge_point", ctypes.c_void_p),
                ("edge_pose", ctypes.c_void_p), ("edge_obs", ctypes.c_void_p),
                ("edge_inv_sigma2", ctypes.c_void_p), ("huber_delta", ctypes.c_double),
                ("chi2_threshold", ctypes.c_double)]


class BAStats(ctypes.Structure):
    _fields_ = [("iterations", ctypes.c_int * 2), ("levenberg_trials", ctypes.c_int * 2),
                ("chi2_initial", ctypes.c_double * 2), ("chi2_final", ctypes.c_double * 2),
                ("n_outliers", ctypes.c_int * 2), ("not_posdef", ctypes.c_int)]


def to_ctypes(prob):
    """orbx_ba_problem over copies of the arrays (returned dict keeps them alive)."""
    arrs = {k: np.ascontiguousarray(prob[k]).copy() for k in
            ["pose_q", "pose_t", "pose_fixed", "pose_id", "pose_cam", "points", "point_id", "point_nobs",
             "edge_point", "edge_pose", "edge_obs", "edge_inv_sigma2"]}
    p = BAProblem()
    p.n_poses = len(arrs["pose_fixed"])
    p.n_points = len(arrs["point_id"])
    p.n_edges = len(arrs["edge_point"])
    for k, a in arrs.items():
        setattr(p, k, a.ctypes.data)
    p.huber_delta = prob["huber_delta"]
    p.chi2_threshold = prob["chi2_threshold"]
    return p, arrs
