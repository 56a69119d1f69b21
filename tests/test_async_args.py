"""Argument checks of Context.upload_async / download_async (host side,
before any device call: runs without a GPU)."""
import numpy as np
import pytest

import orb_slam_amd as ox


def bare_ctx(nf=100):
    c = ox.Context.__new__(ox.Context)   # no device context: the checks run first
    c.nfeatures = nf
    c._h = None
    return c


def test_upload_async_rejects_bad_frames():
    c = bare_ctx()
    with pytest.raises(TypeError):
        c.upload_async(np.zeros((1, 8, 8), np.float32))
    with pytest.raises(ValueError):
        c.upload_async(np.zeros((8, 8), np.uint8))
    with pytest.raises(ValueError):
        c.upload_async(np.zeros((1, 8, 16), np.uint8)[:, :, ::2])
    with pytest.raises(TypeError):
        c.upload_async([[0]])


def test_download_async_rejects_short_or_wrong_arrays():
    c = bare_ctx(nf=100)
    with pytest.raises(ValueError):
        c.download_async(0, 2, kps=np.zeros(150, ox.KEYPOINT))
    with pytest.raises(TypeError):
        c.download_async(0, 1, n_kps=np.zeros(1, np.int64))
    with pytest.raises(ValueError):
        c.download_async(0, 1, desc=np.zeros((100, 32), np.uint8)[:, :16])
    with pytest.raises(ValueError):
        c.download_async(0, 1, m12=np.zeros(99, np.int32))
