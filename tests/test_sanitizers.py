"""Sanitizer leg ("Race detection / sanitizers"): the
host C++ runs under AddressSanitizer, driven by the existing CPU tests.

* The oracle (oracle/, g++) built with ASan + UBSan (`make -C oracle asan`),
  loaded in place of liborbx_ref.so (ORBX_REF_LIBRARY) with gcc's libasan
  preloaded, runs the oracle's known-answer, golden-vector and restatement
  tests.
* The product library's host code (C ABI argument checks, extractor tables,
  geometry, adapters' marshalling; orbx_api.cpp, orbx_geometry.cpp and the
  host side of every .hip file) built with -Xarch_host -fsanitize=address
  (orb_slam_amd.build(sanitize=True); device code is not instrumented) and
  loaded through ORBX_LIBRARY with clang's runtime preloaded, runs the ABI,
  quota-bound, KAT, adapter and undistortion tests.
Each leg runs in its own process (the two ASan runtimes cannot share one).
"""
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]

ORACLE_TESTS = ["tests/test_oracle_kat.py", "tests/test_golden.py", "tests/test_local_map.py",
                "tests/test_proj_oracle.py", "tests/test_pose_oracle.py", "tests/test_harris_oracle.py",
                "tests/test_bow_oracle.py", "tests/test_vocab_oracle.py", "tests/test_quota_bound.py",
                "tests/test_fp_contract.py"]
PRODUCT_TESTS = ["tests/test_abi.py", "tests/test_quota_bound.py", "tests/test_oracle_kat.py",
                 "tests/test_adapters.py", "tests/test_frame_undistort.py"]


def run_pytest(env, files):
    cmd = [sys.executable, "-m", "pytest", "-x", "-q", "-m", "not gpu", "-p", "no:cacheprovider", *files]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    out = p.stdout + p.stderr
    assert p.returncode == 0 and "passed" in out and "ERROR: AddressSanitizer" not in out \
        and "runtime error:" not in out, out[-4000:]
    return out


def instrumented(lib):
    syms = subprocess.run(["nm", "-D", "--undefined-only", str(lib)], capture_output=True, text=True).stdout
    return "__asan_report" in syms or "__asan_init" in syms


def test_oracle_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", str(ROOT / "oracle"), "-j8", "asan"], check=True)
    lib = ROOT / "oracle" / "_asan" / "liborbx_ref_asan.so"
    assert instrumented(lib)
    libasan = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    env = dict(os.environ, LD_PRELOAD=libasan, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", ORBX_REF_LIBRARY=str(lib))
    run_pytest(env, ORACLE_TESTS)


def test_product_host_code_under_asan():
    sys.path.insert(0, str(ROOT))
    from orb_slam_amd import build
    lib = build.build(sanitize=True)
    assert instrumented(lib)
    env = dict(os.environ, LD_PRELOAD=str(build.asan_runtime()), ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               ORBX_LIBRARY=str(lib))
    run_pytest(env, PRODUCT_TESTS)
