"""Local-BA race / call-boundary check.

Runs the same local-BA solves through a library build and stores every output
bit; `compare` then asserts that several builds agree bit for bit.  The
builds: the product library, -DORBX_LBA_NOINLINE (every device function of
orbx_lba.hip a real call, the form in which round 4's dropped pose-pair
Schur went wrong) and -DORBX_LBA_PERTURB (each wave sleeps a pseudo-random
0..~2k cycles after every workgroup barrier, so the phases run in other
interleavings).  A missing barrier, an LDS region shared by two phases or a
call-boundary miscompile changes bits in one of them.

  python -m orb_slam_amd.build -DORBX_LBA_NOINLINE --out=orb_slam_amd/liborbx_lbanoinline.so
  python -m orb_slam_amd.build -DORBX_LBA_PERTURB --out=orb_slam_amd/liborbx_lbaperturb.so
  ORBX_LIBRARY=<lib> python3 tools/lba_race_check.py dump <out.npz> [repeats]
  python3 tools/lba_race_check.py compare a.npz b.npz ..."""
import ctypes
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

KINDS = [dict(n_kf=20, n_points=2000, seed=0), dict(n_kf=20, n_points=2000, seed=77, outlier_frac=0.02),
         dict(n_kf=10, n_points=600, seed=3, outlier_frac=0.05), dict(n_kf=8, n_points=400, seed=3, normalized=True),
         dict(n_kf=8, n_points=400, seed=3, info_scale=1e8), dict(n_kf=8, n_points=400, seed=3, near_points=40),
         dict(n_kf=8, n_points=400, n_fixed_extra=0, seed=7), dict(n_kf=24, n_points=3000, seed=11, outlier_frac=0.1)]


def outputs(arrs, es, pb, st):
    return [arrs["pose_q"].copy(), arrs["pose_t"].copy(), arrs["points"].copy(), es.copy(), pb.copy(),
            np.array(list(st.iterations) + list(st.levenberg_trials) + list(st.n_outliers), np.int64),
            np.array(list(st.chi2_initial) + list(st.chi2_final), np.float64)]


def dump(path, repeats):
    import orb_slam_amd as ox
    from orb_slam_amd import synth_ba as sb
    L = ox.lib()
    ctx = ox.Context(nfeatures=100, max_w=64, max_h=64, slots=1)
    res = {}
    probs = [sb.make_problem(**k) for k in KINDS]
    for rep in range(repeats):
        # single problems: one workgroup, the automatic split, 7 workgroups
        for wg in (1, 0, 7):
            assert L.orbx_lba_set_workgroups(ctx.handle, wg) == 0
            for i, prob in enumerate(probs):
                p, arrs = sb.to_ctypes(prob)
                es = np.zeros(p.n_edges, np.uint8)
                pb = np.zeros(p.n_points, np.uint8)
                st = sb.BAStats()
                assert L.orbx_lba_solve(ctx.handle, ctypes.byref(p), 5, 10, None, es.ctypes.data, pb.ctypes.data,
                                        ctypes.byref(st)) == 0
                for k, a in enumerate(outputs(arrs, es, pb, st)):
                    res[f"r{rep}_wg{wg}_p{i}_{k}"] = a
        # one batch of all kinds (one workgroup per problem)
        cps = [sb.to_ctypes(pr) for pr in probs]
        P = len(cps)
        arr = (sb.BAProblem * P)(*[c[0] for c in cps])
        es = [np.zeros(c[0].n_edges, np.uint8) for c in cps]
        pb = [np.zeros(c[0].n_points, np.uint8) for c in cps]
        st = (sb.BAStats * P)()
        assert L.orbx_lba_solve_batch(ctx.handle, P, arr, 5, 10, None, (ctypes.c_void_p * P)(*[e.ctypes.data for e in es]),
                                      (ctypes.c_void_p * P)(*[b.ctypes.data for b in pb]), st) == 0
        for i in range(P):
            for k, a in enumerate(outputs(cps[i][1], es[i], pb[i], st[i])):
                res[f"r{rep}_batch_p{i}_{k}"] = a
    ctx.close()
    np.savez(path, **res)
    print(f"{path}: {len(res)} arrays from {ox.LIB_PATH}")


def compare(paths):
    base = np.load(paths[0])
    # every array of every build (each repeat, each workgroup count) equal to
    # the first build's repeat 0 (single problems: its one-workgroup solve)
    bad, n = [], 0
    for path in paths:
        other = np.load(path)
        for k in sorted(other.files):
            ref_key = "r0_wg1_" + k.split("_", 2)[2] if "_wg" in k else "r0_" + k.split("_", 1)[1]
            n += 1
            if not np.array_equal(other[k], base[ref_key]):
                bad.append((path, k))
    print(f"{n} arrays over {len(paths)} builds compared; {len(bad)} differ")
    for b in bad[:20]:
        print("  differs:", b)
    return not bad


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 2)
    else:
        sys.exit(0 if compare(sys.argv[2:]) else 1)
