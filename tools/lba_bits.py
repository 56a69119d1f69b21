"""Writes the poses and points of local-BA solves (c5-shaped problems and the
normalised-camera case) to an .npz, so two library builds can be compared
bit for bit: ORBX_LIBRARY=<lib> python3 tools/lba_bits.py out.npz"""
import ctypes
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import orb_slam_amd as ox
from orb_slam_amd import synth_ba as sb

ctx = ox.Context(nfeatures=100, max_w=64, max_h=64, slots=1)
out = {}
cases = [dict(n_kf=20, n_points=2000, seed=s) for s in range(3)] + [
    dict(n_kf=8, n_points=400, seed=3, normalized=True, info_scale=500.0 ** 2)]
for k, kw in enumerate(cases):
    prob = sb.make_problem(**kw)
    p, arrs = sb.to_ctypes(prob)
    es = np.zeros(p.n_edges, np.uint8)
    pb = np.zeros(p.n_points, np.uint8)
    st = sb.BAStats()
    assert ox.lib().orbx_lba_solve(ctx.handle, ctypes.byref(p), 5, 10, None, es.ctypes.data, pb.ctypes.data,
                                   ctypes.byref(st)) == 0
    for key in ("pose_q", "pose_t", "points"):
        out[f"{k}_{key}"] = arrs[key]
    out[f"{k}_status"] = es
    out[f"{k}_stats"] = np.array(list(st.iterations) + list(st.levenberg_trials))
np.savez(sys.argv[1], **out)
print("saved", sys.argv[1], len(out))
