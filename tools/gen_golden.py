"""Generate tests/golden/*.npz: input/output vectors of the CPU restatement.

The reference has no tests, fixtures or buildable binary for this path
(it needs OpenCV 2.4, Eigen, g2o/CHOLMOD and ROS), so
these vectors are produced by the oracle (oracle/liborbx_ref.so), whose
semantics are pinned by tests/test_oracle_kat.py.  They freeze the oracle's
outputs so that (a) any later change to the oracle is caught on CPU and
(b) GPU tests can check the product against data alone.

Run from the repo root:  python tools/gen_golden.py
"""
import ctypes
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

import orb_slam_amd as ox  # noqa: E402
from orb_slam_amd import synth, synth_ba as sb  # noqa: E402
from oracle_lib import RefExtractor, load, ptr  # noqa: E402

OUT = ROOT / "tests" / "golden"


def extract_cases():
    """(name, image, nfeatures) -- small enough to keep the fixtures tiny."""
    return [
        ("extract_texture_320x240", synth.texture_frame(320, 240, 101), 500),
        ("extract_noise_160x120", synth.noise_frame(160, 120, 102), 300),
        ("extract_ragged_97x71", synth.texture_frame(97, 71, 103, n_rects=80), 120),
    ]


# retainBest's libstdc++ era (orbx_ref_set_nth_pivot): 1 = GCC 4.6 .. 4.8,
# the default (`<name>.npz`); 0 = GCC >= 4.9 (`<name>_gcc49.npz`)
ERAS = {1: "", 0: "_gcc49"}


def gen_extract():
    for name, img, nf in extract_cases():
        for era, suffix in ERAS.items():
            e = RefExtractor(nf, 1.2, 8, 20, nth_pivot=era)
            k, d = e(img)
            np.savez_compressed(OUT / f"{name}{suffix}.npz", image=img, nfeatures=nf, nth_pivot=era,
                                keypoints=k.view(np.uint8).reshape(-1, 28), descriptors=d)
            print(name + suffix, len(k))


def gen_init_match():
    W, H = 320, 240
    frames = synth.sequence(W, H, 2, seed=104)
    e = RefExtractor(500)
    (k1, d1), (k2, d2) = e(frames[0]), e(frames[1])
    F1, F2 = ox.frame_view(k1, d1, W, H), ox.frame_view(k2, d2, W, H)
    prev = np.stack([k1["x"], k1["y"]], 1).astype(np.float32)
    prev_in = prev.copy()
    m = np.zeros(len(k1), np.int32)
    n = ctypes.c_int()
    L = load()
    assert L.orbx_ref_search_for_initialization(ctypes.byref(F1), ctypes.byref(F2), ptr(prev), ptr(m), 100, 0.9, 1,
                                                ctypes.byref(n)) == 0
    np.savez_compressed(OUT / "search_init_320x240.npz", w=W, h=H,
                        kps1=k1.view(np.uint8).reshape(-1, 28), desc1=d1,
                        kps2=k2.view(np.uint8).reshape(-1, 28), desc2=d2, prev_in=prev_in,
                        window=100, nnratio=0.9, check_ori=1, matches12=m, n_matches=n.value, prev_out=prev)
    print("search_init", n.value)


def gen_hamming():
    r = np.random.default_rng(105)
    base = r.integers(0, 256, (96, 32), dtype=np.uint8)
    dA = base.copy()
    flip = r.integers(0, 256, (96, 32), dtype=np.uint8) & r.integers(0, 256, (96, 32), dtype=np.uint8) \
        & r.integers(0, 256, (96, 32), dtype=np.uint8)
    dB = np.concatenate([base ^ flip, r.integers(0, 256, (40, 32), dtype=np.uint8)])[r.permutation(136)]
    dB[5] = dB[7]                              # duplicate candidates: ties resolve to the lower index
    bi, b, s = (np.zeros(96, np.int32) for _ in range(3))
    L = load()
    assert L.orbx_ref_hamming_bf(ptr(dA), 96, ptr(dB), len(dB), ptr(bi), ptr(b), ptr(s)) == 0
    np.savez_compressed(OUT / "hamming_bf.npz", desc_a=dA, desc_b=dB, best_idx=bi, best=b, second=s)
    print("hamming", int((b < 50).sum()))


def gen_lba():
    prob = sb.make_problem(n_kf=5, n_points=160, n_fixed_extra=1, seed=106, outlier_frac=0.03)
    p, arrs = sb.to_ctypes(prob)
    es = np.zeros(p.n_edges, np.uint8)
    pb = np.zeros(p.n_points, np.uint8)
    st = sb.BAStats()
    L = load()
    L.orbx_ref_lba.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                               ctypes.c_void_p]
    assert L.orbx_ref_lba(ctypes.byref(p), 5, 10, ptr(es), ptr(pb), ctypes.byref(st)) == 0
    inputs = {f"in_{k}": prob[k] for k in ["pose_q", "pose_t", "pose_fixed", "pose_id", "pose_cam", "points",
                                            "point_id", "point_nobs", "edge_point", "edge_pose", "edge_obs",
                                            "edge_inv_sigma2"]}
    np.savez_compressed(OUT / "lba_small.npz", **inputs, huber_delta=prob["huber_delta"],
                        chi2_threshold=prob["chi2_threshold"], iters0=5, iters1=10,
                        out_pose_q=arrs["pose_q"], out_pose_t=arrs["pose_t"], out_points=arrs["points"],
                        edge_status=es, point_bad=pb, iterations=np.array(st.iterations),
                        levenberg_trials=np.array(st.levenberg_trials), n_outliers=np.array(st.n_outliers),
                        chi2_final=np.array(st.chi2_final))
    print("lba", list(st.iterations), list(st.n_outliers))


def gen_pose():
    from orb_slam_amd import synth_pose as sp
    fr = sp.make_frame(n_kp=300, seed=107, outlier_frac=0.15)
    fr["outlier"][:] = 9
    p, arrs = sp.to_ctypes(fr)
    n = ctypes.c_int()
    st = sp.PoseStats()
    L = load()
    L.orbx_ref_pose_optimization.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    assert L.orbx_ref_pose_optimization(ctypes.byref(p), ctypes.byref(n), ctypes.byref(st)) == 0
    inputs = {f"in_{k}": fr[k] for k in ["kp_un", "octave", "inv_level_sigma2", "has_mp", "mp_xyz", "cam", "Tcw",
                                          "outlier"]}
    np.savez_compressed(OUT / "pose_frame.npz", **inputs, out_Tcw=sp.pose_of(p), out_outlier=arrs["outlier"],
                        n_inliers=n.value, rounds=st.rounds, iterations=np.array(st.iterations),
                        n_bad=np.array(st.n_bad))
    print("pose", n.value, list(st.iterations), list(st.n_bad))


def gen_bow():
    from bow_data import make_pair
    from test_bow_oracle import run_ref
    P = make_pair(n1=300, n2=300, n_nodes=25, seed=108)
    a1, a2 = P["keep"]
    out = {}
    for mode, name in [(0, "bow_frame"), (1, "bow_kf"), (2, "triangulation")]:
        m, n = run_ref(mode, P, 0.75, 1)
        out[f"{name}_matches"] = m
        out[f"{name}_n"] = n
    side = {}
    for tag, a in (("a", a1), ("b", a2)):
        for k in ["kps", "desc", "mp", "ids", "ptr", "feat"]:
            side[f"{tag}_{k}"] = a[k] if k != "kps" else a[k].view(np.uint8).reshape(-1, 28)
    np.savez_compressed(OUT / "bow_pair.npz", **side, F12=P["F12"], sigma2=P["sigma2"], **out)
    print("bow", out["bow_frame_n"], out["bow_kf_n"], out["triangulation_n"])


def gen_vocab():
    from vocab_data import features, make_vocab, run_ref
    V = make_vocab(k=6, L=4, seed=109, irregular=True)
    d = features(V, n=400, seed=110)
    r = run_ref(V, d, 2)
    np.savez_compressed(OUT / "vocab_small.npz", k=V["k"], L=V["L"], parent=V["parent"], is_leaf=V["is_leaf"],
                        vdesc=V["desc"], weight=V["weight"], desc=d, levelsup=2, word=r["word"], w=r["weight"],
                        nid=r["nid"], bow_words=r["bw"][:r["nw"]], bow_values=r["bv"][:r["nw"]],
                        fv_nodes=r["fn"][:r["nf"]], fv_ptr=r["fp"][:r["nf"] + 1], fv_feat=r["ff"][:r["fp"][r["nf"]]])
    print("vocab", r["nw"], r["nf"])


if __name__ == "__main__":
    if sys.argv[1:] == ["extract"]:   # only the extraction vectors (both eras)
        gen_extract()
        sys.exit(0)
    OUT.mkdir(parents=True, exist_ok=True)
    gen_extract()
    gen_init_match()
    gen_hamming()
    gen_lba()
    gen_pose()
    gen_bow()
    gen_vocab()
