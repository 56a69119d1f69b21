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


def test_native_oracle_builds_for_this_host():
    """The timed CPU baseline's library: the oracle built here with the
    reference's -O3 -march=native (CMakeLists.txt:12-13)."""
    L, desc = bench.native_oracle()
    assert "march=native" in desc, desc
    assert L.orbx_ref_descriptor_distance is not None


@pytest.mark.parametrize("bf", [False, True])
def test_cpu_baseline_frames_protocol(bf):
    """Warm-up frames, then the median / p90 of the timed frames' times."""
    frames = synth.sequence(96, 80, 4, seed=3)
    r = bench.cpu_baseline_frames(frames, 100, (2, 5), bf=bf)
    assert r["timed_units"] == 5 and r["cores"] == 1 and r["kind"] == "port"
    assert r["p90_ms"] >= r["median_ms"] > 0 and abs(r["value"] - 1e3 / r["median_ms"]) / r["value"] < 1e-3
    assert "2 warm-up + 5 timed" in r["sample"]


def test_sequence_has_300_distinct_frames():
    """a 300-frame sequence without repeated frames."""
    offs = {synth.sequence_offset(k) for k in range(synth.SEQ_PERIOD)}
    assert len(offs) == synth.SEQ_PERIOD
    seq = synth.sequence(64, 48, 300, seed=1)
    assert len({f.tobytes() for f in seq}) == 300
    # consecutive frames move by at most 2 px (the matcher's window is 100)
    for k in range(1, 300):
        (x0, y0), (x1, y1) = synth.sequence_offset(k - 1), synth.sequence_offset(k)
        assert abs(x1 - x0) <= 2 and abs(y1 - y0) <= 1
