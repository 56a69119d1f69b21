"""bench.py with a CPU stand-in for the orbx context (TEST INFRASTRUCTURE).

Run as `python tests/bench_stub.py <bench.py arguments>`.  It installs
StubContext in place of orb_slam_amd.Context and enters bench.main(), so the
real harness runs end to end on a host without a GPU: the `--gpus N`
launcher (which re-enters this wrapper for every rank, since it starts
sys.argv[0]), the process group, the warm-up / serialised / timed steps with
their barriers, the stats gather before rank 0's CPU legs, the parity check of
the last step and the JSON line.

The stand-in "extracts" with the oracle and matches with the oracle's
SearchForInitialization / brute force, and reports its wall times under the
bench's kernel names, so the parity leg compares the oracle with itself: this
tests the harness, not the kernels (those are the -m gpu tests).
"""
import ctypes
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

import bench  # noqa: E402
import oracle_lib  # noqa: E402
import orb_slam_amd as ox  # noqa: E402


class StubContext:
    """The subset of orb_slam_amd.Context that bench.run_frames calls."""

    def __init__(self, nfeatures=1000, max_w=640, max_h=480, slots=1, device=0, **_):
        self.nfeatures, self.slots, self.device = nfeatures, slots, device
        self.w, self.h = max_w, max_h
        self.L = oracle_lib.load()
        self.ex = oracle_lib.RefExtractor(nfeatures, lib=self.L)
        self.frames, self.out, self.match = {}, {}, {}
        self.enabled, self.only, self.acc = False, None, {}

    def upload(self, frames, first=0):
        for i, f in enumerate(np.asarray(frames, np.uint8)):
            self.frames[first + i] = f.copy()

    def upload_async(self, frames, first=0):
        self.upload(frames, first)

    def download_async(self, first, count, kps=None, desc=None, n_kps=None, m12=None, n_m=None):
        nf = self.nfeatures
        for i in range(count):
            k, d = self.out[first + i]
            m, nm = self.match[first + i]
            kps[i * nf:i * nf + len(k)] = k
            desc[i * nf:i * nf + len(k)] = d
            n_kps[i] = len(k)
            m12[i * nf:(i + 1) * nf] = m
            n_m[i] = nm

    def set_split(self, n):
        pass

    def set_async_match(self, enable):
        pass

    def nth_pivot(self):
        return self.ex.nth_pivot

    def _record(self, name, dt):
        if self.enabled and (self.only is None or self.only == name):
            n, tot = self.acc.get(name, (0, 0.0))
            self.acc[name] = (n + 1, tot + 1e3 * dt)

    def extract(self, first, count):
        t0 = time.perf_counter()
        for s in range(first, first + count):
            self.out[s] = self.ex(self.frames[s])
        self._record("fast", time.perf_counter() - t0)

    def _match(self, first, count, seq_len, bf):
        t0 = time.perf_counter()
        for i in range(count):
            s, p = first + i, first + (i - 1) % seq_len
            (pk, pd), (k, d) = self.out[p], self.out[s]
            m = np.full(self.nfeatures, -1, np.int32)
            if bf:
                bi, b1, b2 = (np.zeros(len(pd), np.int32) for _ in range(3))
                self.L.orbx_ref_hamming_bf(oracle_lib.ptr(pd), len(pd), oracle_lib.ptr(d), len(d),
                                           oracle_lib.ptr(bi), oracle_lib.ptr(b1), oracle_lib.ptr(b2))
                want = np.where((b1 <= 50) & (b1.astype(np.float32) < b2.astype(np.float32) * np.float32(0.9)),
                                bi, -1)
                m[:len(pd)] = want
                nm = int((want >= 0).sum())
            else:
                F1, F2 = ox.frame_view(pk, pd, self.w, self.h), ox.frame_view(k, d, self.w, self.h)
                pm = np.stack([pk["x"], pk["y"]], 1).astype(np.float32).copy()
                mm = np.zeros(len(pk), np.int32)
                c = ctypes.c_int()
                self.L.orbx_ref_search_for_initialization(ctypes.byref(F1), ctypes.byref(F2), oracle_lib.ptr(pm),
                                                          oracle_lib.ptr(mm), 100, 0.9, 1, ctypes.byref(c))
                m[:len(pk)] = mm
                nm = c.value
            self.match[s] = (m, nm)
        self._record("match", time.perf_counter() - t0)

    def match_prev(self, first, count, seq_len, **_):
        self._match(first, count, seq_len, False)

    def match_bf_prev(self, first, count, seq_len, **_):
        self._match(first, count, seq_len, True)

    def extract_match(self, first, count, seq_len, mode="init", **_):
        self.extract(first, count)
        self._match(first, count, seq_len, mode == "bf")

    def sync(self):
        pass

    def timing(self, enable=True, only=None):
        self.enabled, self.only, self.acc = bool(enable), only, {}

    def kernel_time(self, name):
        n, tot = self.acc.get(name, (0, 0.0))
        return n, (tot / n if n else 0.0), tot

    def features(self, slot):
        return self.out[slot]

    def matches(self, slot):
        return self.match[slot]

    def close(self):
        pass


class StubHostArray:
    """orb_slam_amd.HostArray without page-locking (no device here)."""

    def __init__(self, shape, dtype):
        self.array = np.zeros(shape, dtype)

    def close(self):
        self.array = None


if __name__ == "__main__":
    bench.ox.Context = StubContext
    bench.ox.HostArray = StubHostArray
    bench.main()
