"""The Tracking chain restated over the oracle (tests/track_data.py), on the
CPU: on the synthetic plane scene the chain must recover the camera that
rendered the current image -- a known answer for the restatement the GPU
chain is compared with (tests/test_track_gpu.py)."""
import numpy as np
import pytest

import track_data as td
from oracle_lib import RefExtractor, load

W, H = 640, 480


@pytest.fixture(scope="module")
def ex():
    return RefExtractor(1000)


@pytest.mark.parametrize("shift,pred_err", [(6, 1.5), (14, -3.0)])
def test_motion_model_chain_recovers_camera(ex, shift, pred_err):
    last, cur = td.images(W, H, shift, 1)
    kl, dl = ex(last)
    kc, dc = ex(cur)
    scene = td.make_scene(kl, dl, 1)
    px = td.DEPTH / float(td.CAM[0])
    out = td.ref_chain(load(), kl, dl, kc, dc, scene, td.pose_x((shift + pred_err) * px))
    assert out["status"] == 0 and out["n_motion"] >= 20 and out["n_inliers"] > 300
    T = out["Tcw"].reshape(3, 4)
    assert np.abs(T[:, :3] - np.eye(3)).max() < 2e-3          # no rotation
    assert abs(T[0, 3] + shift * px) < 0.25 * px               # within a quarter pixel of the true shift
    assert np.abs(T[1:, 3]).max() < 0.01


def test_previous_frame_chain_recovers_camera(ex):
    shift = 10
    last, cur = td.images(W, H, shift, 2)
    kl, dl = ex(last)
    kc, dc = ex(cur)
    scene = td.make_scene(kl, dl, 2)
    px = td.DEPTH / float(td.CAM[0])
    out = td.ref_chain_prev(load(), kl, dl, kc, dc, scene, td.pose_x(0.0))
    assert out["status"] == 0 and out["n_pair"] >= 0
    T = out["Tcw"].reshape(3, 4)
    assert abs(T[0, 3] + shift * px) < 0.25 * px


def test_chain_failure_statuses(ex):
    last, cur = td.images(W, H, 6, 11)
    kl, dl = ex(last)
    kc, dc = ex(cur)
    few = td.make_scene(kl, dl, 11, observed=0.004)
    assert td.ref_chain(load(), kl, dl, kc, dc, few, td.pose_x(6 * td.DEPTH / 500))["status"] == 1
    assert td.ref_chain_prev(load(), kl, dl, kc, dc, few, td.pose_x(0.0))["status"] == 3
