"""`bench.py --gpus N` end to end on CPU (BASELINE configs[3]).

The real harness runs through tests/bench_stub.py, which only swaps the orbx
context for an oracle-backed CPU stand-in: the launcher starts N rank
processes, they meet over gloo, run the warm-up / serialised / timed steps,
gather their stats before rank 0's CPU legs, and rank 0 prints the one JSON
line with value = units of all ranks / the slowest rank's seconds.
"""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def _run(args, env_extra=None, timeout=300):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, str(ROOT / "tests" / "bench_stub.py"), *args], cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=timeout)


def _line(p):
    assert p.returncode == 0, p.stderr[-3000:]
    lines = p.stdout.splitlines()
    assert len(lines) == 1 and lines[0].startswith("{"), p.stdout   # rank 0's JSON line, nothing else
    return json.loads(lines[0])


@pytest.mark.parametrize("world,workload,batch", [(2, "c2", 6), (3, "c2", 4), (2, "c3", 2)])
def test_bench_gpus_n_end_to_end(world, workload, batch):
    steps = 2 if workload == "c2" else 1
    out = _line(_run(["--gpus", str(world), "--workload", workload, "--steps", str(steps), "--warmup", "1",
                      "--batch", str(batch), "--cpu-budget", "1", "--cpu-protocol", "1,3"]))
    assert out["n_gpus"] == world and out["steps"] == steps
    r = out["ranks"]
    assert r["backend"] == "gloo" and len(r["elapsed_s"]) == world
    assert r["units"] == [batch * steps] * world            # weak scaling: fixed work per rank
    want = sum(r["units"]) / max(r["elapsed_s"])
    assert out["value"] == pytest.approx(want, rel=1e-3)
    assert out["ms_per_step"] == pytest.approx(1e3 * max(r["elapsed_s"]) / steps, rel=1e-3)
    # rank 0 keeps the CPU baseline and the parity check of its last step in N > 1 lines
    assert out["cpu_baseline"]["cores"] == 1 and out["cpu_baseline"]["value"] > 0
    assert out["cpu_baseline_all_cores"]["value"] > 0
    assert out["check"]["parity_last_step"]["bit_exact"] is True
    assert out["check"]["parity_last_step"]["nth_element_era"].startswith("GCC 4.6-4.8")
    assert out["roofline"]["kernel"] == "fast"
    # the host-fed leg's read-back equals the device outputs (stubbed here)
    hi = out["check"]["host_inclusive"]
    assert hi["host_buffers_equal_device_outputs"] is True and hi["frames_per_s"] > 0
    # the whole-path figure counts every rank's frames
    per = out["path_roofline"]["algorithmic_bytes_per_frame"]
    assert out["path_roofline"]["algorithmic_bytes_per_step"] == per * batch * world


def test_bench_rejects_world_size_mismatch():
    p = _run(["--gpus", "4", "--steps", "1", "--warmup", "0", "--batch", "2", "--no-cpu-baseline"],
             env_extra={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"}, timeout=120)
    assert p.returncode == 2 and "WORLD_SIZE=2 but --gpus 4" in p.stderr


def test_bench_single_rank_has_no_ranks_block():
    out = _line(_run(["--steps", "1", "--warmup", "0", "--batch", "3", "--no-cpu-baseline", "--no-isolated"]))
    assert out["n_gpus"] == 1 and "ranks" not in out
