"""The C++ adapter (orb_slam_amd/adapters/orbx_adapters.hpp) that keeps the
reference's ORBextractor / ORBmatcher / Optimizer signatures over the C ABI.
The demo program is built by orb_slam_amd.build (g++ against liborbx.so)."""
import json
import subprocess
from pathlib import Path

import pytest

import orb_slam_amd as ox

DEMO = Path(ox.__file__).resolve().parent / "adapters" / "adapter_demo"


@pytest.fixture(scope="module")
def demo():
    if not DEMO.exists():
        from orb_slam_amd import build
        build.build()
    assert DEMO.exists()
    return DEMO


def test_adapter_fails_loudly_without_device(demo, tmp_path):
    import os
    if os.path.exists("/dev/kfd"):
        pytest.skip("GPU present")
    p = subprocess.run([str(demo)], capture_output=True, text=True, timeout=120)
    assert p.returncode == 3, (p.returncode, p.stderr)
    assert "orbx" in p.stderr


@pytest.mark.gpu
def test_adapter_end_to_end(demo):
    p = subprocess.run([str(demo)], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["levels"] == 8 and abs(r["scale"] - 1.2) < 1e-6
    assert r["n1"] > 500 and r["n2"] > 500
    assert r["init_matches"] > 50 and r["bf_matches"] > 50
    assert r["ba_iterations"][0] >= 1
    assert r["ba_chi2"][1] < r["ba_chi2"][0]
    # noise-free map points: every edge an inlier, the 2 cm offset removed
    assert r["pose_inliers"] == r["pose_edges"] > 100
    assert abs(r["pose_tx"]) < 1e-3
