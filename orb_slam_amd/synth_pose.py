"""Synthetic tracking frames for Optimizer::PoseOptimization
(src/Optimizer.cc:154-285).

A 640x480 frame with `n_kp` keypoints (octave uniform 0..7, mvKeysUn in
float); a fraction `mp_frac` carries a map point 2-6 m in front of the true
camera.  Observations = true projection + N(0, 1 px) * 1.2^octave; a
fraction `outlier_frac` of the map-point keypoints are gross outliers (the
wrong-match case the robust rounds exist for).  The initial mTcw is the
true pose perturbed by ~0.01 rad / 0.02 m (a motion-model prediction), in
float like the reference's cv::Mat.

Returns numpy arrays laid out as include/orbx.h's orbx_pose_frame.
"""
import ctypes

import numpy as np

from .synth_ba import _exp_so3, inv_sigma2_table


def make_frame(n_kp=1000, mp_frac=0.7, outlier_frac=0.1, seed=0, w=640, h=480, fx=500.0, fy=500.0, cx=320.0,
               cy=240.0, pose_noise=(0.01, 0.02), pix_noise=1.0, nlevels=8):
    rng = np.random.default_rng(seed)
    R = _exp_so3(rng.normal(0, 0.3, 3))
    t = rng.normal(0, 1.0, 3)
    octave = rng.integers(0, nlevels, n_kp).astype(np.int32)
    has_mp = (rng.random(n_kp) < mp_frac).astype(np.uint8)
    u = rng.uniform(0, w, n_kp)
    v = rng.uniform(0, h, n_kp)
    depth = rng.uniform(2.0, 6.0, n_kp)
    Xc = np.stack([(u - cx) / fx * depth, (v - cy) / fy * depth, depth], 1)
    Xw = (Xc - t) @ R                               # R^T (Xc - t), row-wise
    sd = pix_noise * 1.2 ** octave
    ou = u + rng.normal(0, 1, n_kp) * sd
    ov = v + rng.normal(0, 1, n_kp) * sd
    bad = rng.random(n_kp) < outlier_frac
    ou[bad] += rng.choice([-1, 1], bad.sum()) * rng.uniform(15, 60, bad.sum())
    ov[bad] += rng.choice([-1, 1], bad.sum()) * rng.uniform(15, 60, bad.sum())
    dR = _exp_so3(rng.normal(0, pose_noise[0], 3))
    T = np.eye(4)
    T[:3, :3] = dR @ R
    T[:3, 3] = t + rng.normal(0, pose_noise[1], 3)
    T_true = np.eye(4)
    T_true[:3, :3] = R
    T_true[:3, 3] = t
    return {
        "kp_un": np.ascontiguousarray(np.stack([ou, ov], 1), np.float32),
        "octave": octave,
        "inv_level_sigma2": inv_sigma2_table(nlevels).astype(np.float32),
        "has_mp": has_mp,
        "mp_xyz": np.ascontiguousarray(Xw, np.float32),
        "cam": np.array([fx, fy, cx, cy], np.float32),
        "Tcw": np.ascontiguousarray(T, np.float32),
        "outlier": np.zeros(n_kp, np.uint8),
        "Tcw_true": T_true,
    }


class PoseFrame(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int), ("kp_un", ctypes.c_void_p), ("octave", ctypes.c_void_p),
                ("inv_level_sigma2", ctypes.c_void_p), ("nlevels", ctypes.c_int), ("has_mp", ctypes.c_void_p),
                ("mp_xyz", ctypes.c_void_p), ("cam", ctypes.c_float * 4), ("Tcw", ctypes.c_float * 16),
                ("outlier", ctypes.c_void_p)]


class PoseStats(ctypes.Structure):
    _fields_ = [("rounds", ctypes.c_int), ("iterations", ctypes.c_int * 4), ("levenberg_trials", ctypes.c_int * 4),
                ("n_bad", ctypes.c_int * 4), ("chi2_final", ctypes.c_double * 4), ("not_posdef", ctypes.c_int)]


def to_ctypes(fr):
    """orbx_pose_frame over copies of the frame's arrays; returns (struct,
    arrays) -- the arrays dict keeps the memory alive and receives the
    outlier flags."""
    arrs = {k: np.ascontiguousarray(fr[k]).copy() for k in
            ["kp_un", "octave", "inv_level_sigma2", "has_mp", "mp_xyz", "outlier"]}
    p = PoseFrame()
    p.n = len(arrs["octave"])
    p.nlevels = len(arrs["inv_level_sigma2"])
    for k in ["kp_un", "octave", "inv_level_sigma2", "has_mp", "mp_xyz", "outlier"]:
        setattr(p, k, arrs[k].ctypes.data)
    for i in range(4):
        p.cam[i] = float(fr["cam"][i])
    for i, val in enumerate(np.asarray(fr["Tcw"], np.float32).reshape(-1)):
        p.Tcw[i] = float(val)
    return p, arrs


def pose_of(p):
    return np.frombuffer(bytes(p.Tcw), np.float32).reshape(4, 4).copy()
