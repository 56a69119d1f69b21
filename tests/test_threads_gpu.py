"""ORB-SLAM's threading model on one GPU.

The reference runs Tracking, LocalMapping and LoopClosing as three
concurrent threads (src/main.cc:122-133), each with its own extractor and
matcher instances: LocalMapping's local BA
(src/LocalMapping.cc:83) and triangulation search (:220-260) run while
Tracking extracts and optimises poses (src/Tracking.cc:203-206, 533, 556,
584) and LoopClosing searches candidate keyframes (src/LoopClosing.cc:240,
574).  Here each thread owns an orbx_ctx and calls the C ABI from its own
host thread (ctypes releases the GIL), all three at once, for several
rounds:

* Tracking:     orbx_extract -> orbx_search_by_projection_motion ->
                orbx_pose_optimization
* LocalMapping: orbx_lba_solve (the multi-workgroup k_lba_split, whose grid
                barrier needs its workgroups co-resident while the other
                threads' kernels share the CUs) -> orbx_search_for_triangulation
* LoopClosing:  orbx_search_by_bow_kf -> orbx_search_by_sim3

Every output under contention must be bit-identical to the same calls run
one at a time, and those match the CPU restatement (the per-call parity
tests' rules)."""
import numpy as np
import pytest

import orb_slam_amd as ox
from oracle_lib import load
from test_bow_oracle import run_ref as bow_ref
from test_lba_gpu import compare as lba_compare
from test_lba_gpu import run_ref as lba_ref
from test_pose_gpu import compare_exact as pose_compare
from test_pose_oracle import ref_pose
from threads_work import WORK, _medians, _motion, _sim3, make_contexts, make_inputs, run_threads, same

pytestmark = pytest.mark.gpu

ROUNDS = 6


@pytest.fixture(scope="module")
def inputs():
    return make_inputs()


@pytest.fixture(scope="module")
def contexts():
    cs = make_contexts()
    yield cs
    for c in cs.values():
        c.close()


@pytest.fixture(scope="module")
def serial(contexts, inputs):
    """Each thread's calls one at a time (reference outputs of this test),
    checked against the CPU restatement."""
    out = {k: [WORK[k](contexts[k], inputs, r)[0] for r in range(len(inputs["frames"]))] for k in WORK}
    L = load()
    for r, (kps, desc, m, n, pose) in enumerate(out["tracking"]):
        rk, rd = inputs["ref_feats"][r]
        assert kps.tobytes() == rk.tobytes() and desc.tobytes() == rd.tobytes()
        rm, rn = _motion(None, rk, rd, inputs, L)
        assert n == rn and rn > 0 and np.array_equal(m, rm)
        pose_compare(ref_pose(inputs["pose_frame"]), pose)
    (ba, tri) = out["local_mapping"][0]
    lba_compare(lba_ref(inputs["lba"]), ba)
    ro, rn = bow_ref(2, inputs["tri"], 0.6, 1)
    assert tri[1] == rn and rn > 0 and np.array_equal(tri[0], ro)
    (bkf, s3) = out["loop_closing"][0]
    ro, rn = bow_ref(1, inputs["bowkf"], 0.75, 1)
    assert bkf[1] == rn and rn > 0 and np.array_equal(bkf[0], ro)
    rn3, rc3 = _sim3(None, inputs, L)
    assert s3[1] == rc3 and rc3 > 0 and np.array_equal(s3[0], rn3)
    for k in ("local_mapping", "loop_closing"):   # the same inputs every round
        for o in out[k][1:]:
            assert same(o, out[k][0]), k
    return out


def _medians(times):
    return {k: {c: round(float(np.median([t[c] for t in times[k]])) * 1e3, 4) for c in times[k][0]} for k in times}


@pytest.mark.parametrize("coop", [1, 0], ids=["cooperative", "plain"])
def test_three_threads_concurrent_equal_serial(contexts, inputs, serial, coop):
    """All three threads at once for ROUNDS rounds each: every output equals
    its serial run bit for bit (so also the oracle), and the local BA really
    ran over several workgroups beside the other threads' kernels (launched
    cooperatively, and plainly)."""
    assert ox.lib().orbx_debug_lba_split(contexts["local_mapping"].handle, -1, -1, -1, coop) == 0
    alone = {k: [WORK[k](contexts[k], inputs, r)[1] for r in range(ROUNDS)] for k in WORK}
    results, times, errors = run_threads(contexts, inputs, ROUNDS)
    assert not errors, errors
    for k in WORK:
        ser = serial[k]
        for r, o in enumerate(results[k]):
            assert same(o, ser[r % len(ser)]), (k, r)
    assert ox.lib().orbx_lba_last_workgroups(contexts["local_mapping"].handle) > 1
    ox.lib().orbx_debug_lba_split(contexts["local_mapping"].handle, -1, -1, -1, 0)   # the default again
    print(f"coop {coop}: median ms one thread at a time:", _medians(alone))
    print(f"coop {coop}: median ms under contention:", _medians(times))
