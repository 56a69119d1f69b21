"""CPU checks of the Optimizer::PoseOptimization restatement
(oracle/ref_pose.cpp; src/Optimizer.cc:154-285) -- the checker the GPU
parity tests in test_pose_gpu.py compare against.

Known answers: Eigen's pivoted LDLT solve equals numpy's dense solve; a
noise-free frame converges to the true pose with no outliers; gross outliers
are classified as outliers; the < 10 edges rule stops after round 0; a frame
without map points leaves the pose (up to the SE3Quat round trip) and the
untouched mvbOutlier entries alone.
"""
import ctypes

import numpy as np
import pytest

from orb_slam_amd import synth_pose as sp
from oracle_lib import load


def ref_pose(fr):
    L = load()
    L.orbx_ref_pose_optimization.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    p, arrs = sp.to_ctypes(fr)
    n = ctypes.c_int()
    st = sp.PoseStats()
    assert L.orbx_ref_pose_optimization(ctypes.byref(p), ctypes.byref(n), ctypes.byref(st)) == 0
    return sp.pose_of(p), arrs["outlier"], n.value, st


@pytest.mark.parametrize("seed", range(6))
def test_ldlt_matches_dense_solve(seed):
    L = load()
    L.orbx_ref_ldlt_solve.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    rng = np.random.default_rng(seed)
    J = rng.normal(size=(40, 6)) * rng.uniform(0.01, 100, 6)   # badly scaled columns: pivoting matters
    A = J.T @ J + 1e-3 * np.eye(6)
    b = rng.normal(size=6)
    x = np.zeros(6)
    A = np.ascontiguousarray(A)
    assert L.orbx_ref_ldlt_solve(6, A.ctypes.data, b.ctypes.data, x.ctypes.data) == 1
    np.testing.assert_allclose(A @ x, b, rtol=0, atol=1e-9 * np.abs(b).max() * np.linalg.cond(A) ** 0.5)
    np.testing.assert_allclose(x, np.linalg.solve(A, b), rtol=1e-8, atol=1e-12)


def test_ldlt_reports_indefinite():
    L = load()
    L.orbx_ref_ldlt_solve.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    A = np.diag([1.0, -2.0, 3.0])
    b = np.ones(3)
    x = np.zeros(3)
    assert L.orbx_ref_ldlt_solve(3, A.ctypes.data, b.ctypes.data, x.ctypes.data) == 0


def test_noise_free_frame_recovers_true_pose():
    fr = sp.make_frame(n_kp=400, pix_noise=0.0, outlier_frac=0.0, seed=11)
    T, out, n, st = ref_pose(fr)
    assert n == int(fr["has_mp"].sum()) and out.sum() == 0
    assert np.abs(T[:3] - fr["Tcw_true"][:3]).max() < 2e-4
    assert st.rounds == 4


def test_gross_outliers_are_rejected():
    fr = sp.make_frame(n_kp=600, outlier_frac=0.15, seed=3)
    T, out, n, st = ref_pose(fr)
    Tt = fr["Tcw_true"]
    # reprojection error at the true pose decides which keypoints are gross outliers
    m = fr["has_mp"].astype(bool)
    X = fr["mp_xyz"][m].astype(np.float64)
    pc = X @ Tt[:3, :3].T + Tt[:3, 3]
    uv = pc[:, :2] / pc[:, 2:] * fr["cam"][:2] + fr["cam"][2:]
    r = np.linalg.norm(fr["kp_un"][m] - uv, axis=1)
    sd = 1.2 ** fr["octave"][m]
    gross = r > 10 * sd
    assert gross.sum() > 20
    assert out[m][gross].all()
    assert n == m.sum() - out[m].sum() == m.sum() - st.n_bad[st.rounds - 1]


def test_fewer_than_ten_edges_stop_after_round_zero():
    fr = sp.make_frame(n_kp=12, mp_frac=0.6, seed=5)
    fr["has_mp"][:] = 0
    fr["has_mp"][:7] = 1
    T, out, n, st = ref_pose(fr)
    assert st.rounds == 1 and st.iterations[0] > 0


def test_no_map_points_leaves_outputs_alone():
    fr = sp.make_frame(n_kp=50, seed=6)
    fr["has_mp"][:] = 0
    fr["outlier"][:] = 7
    T, out, n, st = ref_pose(fr)
    assert n == 0 and st.rounds == 1 and st.iterations[0] == 0
    assert (out == 7).all()
    # SE3Quat round trip of the float pose only
    assert np.abs(T - fr["Tcw"]).max() < 1e-6
