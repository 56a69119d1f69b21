"""bench.py's CPU-baseline helpers (no GPU): thread count selection, the
thread runner, and the all-cores oracle baseline on tiny frames."""
import sys
from pathlib import Path

import pytest

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
from orb_slam_amd import synth  # noqa: E402


def test_cpu_threads_env(monkeypatch):
    monkeypatch.setenv("ORBX_CPU_THREADS", "3")
    assert bench.cpu_threads() == 3
    monkeypatch.delenv("ORBX_CPU_THREADS")
    monkeypatch.setenv("OMP_NUM_THREADS", "5")
    assert bench.cpu_threads() == 5


def test_run_threads_sums_workers():
    n, dt = bench.run_threads(4, 0.05, lambda t, deadline: t + 1)
    assert n == 10 and dt >= 0


@pytest.mark.parametrize("bf", [False, True])
def test_cpu_all_cores_frames(monkeypatch, bf):
    monkeypatch.setenv("ORBX_CPU_THREADS", "2")
    frames = synth.sequence(96, 80, 4, seed=3)
    r = bench.cpu_all_cores_frames(frames, 100, 0.5, bf=bf)
    assert r["cores"] == 2 and r["value"] > 0 and r["kind"] == "port"
    assert r["unit"] == ("pairs/s" if bf else "frames/s")
