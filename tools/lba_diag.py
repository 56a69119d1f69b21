"""Diagnostic: one local-BA problem solved with several workgroup counts,
each twice, against the oracle (poses, LM statistics)."""
import ctypes
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import orb_slam_amd as ox  # noqa: E402
from orb_slam_amd import synth_ba as sb  # noqa: E402
from test_lba_gpu import run_ref  # noqa: E402

prob = sb.make_problem(n_kf=20, n_points=2000, seed=0)
ctx = ox.Context(nfeatures=100, max_w=64, max_h=64, slots=1)
ref = run_ref(prob)
print("oracle", list(ref[3].iterations), list(ref[3].levenberg_trials), list(ref[3].n_outliers))
for wg in (1, 1, 0, 0, 2, 2):
    assert ox.lib().orbx_lba_set_workgroups(ctx.handle, wg) == 0
    p, arrs = sb.to_ctypes(prob)
    es = np.zeros(p.n_edges, np.uint8)
    pb = np.zeros(p.n_points, np.uint8)
    st = sb.BAStats()
    r = ox.lib().orbx_lba_solve(ctx.handle, ctypes.byref(p), 5, 10, None, es.ctypes.data, pb.ctypes.data,
                                ctypes.byref(st))
    d = float(np.abs(arrs["pose_q"] - ref[0]["pose_q"]).max())
    print(wg, r, "dq", d, list(st.iterations), list(st.levenberg_trials), list(st.n_outliers), st.not_posdef,
          "es", int((es != ref[1]).sum()), float(arrs["pose_q"].sum()), list(st.chi2_final))
