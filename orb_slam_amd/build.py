"""Build liborbx.so (HIP kernels + C ABI) in-tree for gfx950.

Usage: python -m orb_slam_amd.build  (or orb_slam_amd.build.build()).
Compiles every orb_slam_amd/csrc/*.hip and *.cpp with hipcc in parallel and
links orb_slam_amd/liborbx.so.  Objects go to orb_slam_amd/build/ and are
rebuilt only when a source or header is newer.
"""
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
OBJ = PKG / "build"
LIB = PKG / "liborbx.so"
ARCH = os.environ.get("ORBX_ARCH", "gfx950")
if ARCH != "gfx950":
    # the kernels are written for gfx950 only: 160 KB of LDS per CU (the pose
    # and local-BA kernels size their LDS for it), v_pk_minimum3_f16, 32-lane SIMDs
    raise RuntimeError(f"ORBX_ARCH={ARCH}: liborbx targets gfx950 (MI355X) only")

COMMON = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
          "-fhip-fp32-correctly-rounded-divide-sqrt", "-Wall", "-Wno-unused-function", "-Wno-unused-result", "-Wno-unused-value",
          f"-I{PKG.parent / 'include'}", f"-I{CSRC}"]


def hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and Path(c).exists():
            return c
    raise RuntimeError("hipcc not found (ROCm required to build liborbx)")


def _needs(obj, src, headers):
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    return src.stat().st_mtime > t or any(h.stat().st_mtime > t for h in headers)


ASAN_DIR = PKG / "build_asan"
ASAN_LIB = ASAN_DIR / "liborbx_asan.so"


def asan_runtime():
    """clang's AddressSanitizer runtime (preloaded to run the ASan build)."""
    hits = sorted(Path("/opt/rocm/lib/llvm/lib/clang").glob("*/lib/linux/libclang_rt.asan-x86_64.so"))
    if not hits:
        raise RuntimeError("libclang_rt.asan-x86_64.so not found under /opt/rocm/lib/llvm")
    return hits[-1]


def build(verbose=False, jobs=None, defines=(), lib=None, sanitize=False):
    """defines: extra -D flags for an instrumented variant (e.g.
    ORBX_MATCH_PROFILE); such a variant is linked to `lib` with its own
    object directory and loaded through ORBX_LIBRARY.
    sanitize: the host-code AddressSanitizer build:
    host code of every file instrumented, device code untouched (-Xarch_host),
    linked to build_asan/liborbx_asan.so; run it with the runtime of
    asan_runtime() preloaded (tests/test_sanitizers.py).  GPU-side ASan is
    not used."""
    cc = hipcc()
    if sanitize:
        obj_dir, out = ASAN_DIR, ASAN_LIB
    else:
        obj_dir = OBJ if not defines else OBJ.parent / ("build_" + "_".join(d.lower() for d in defines))
        out = Path(lib) if lib else LIB
    obj_dir.mkdir(exist_ok=True)
    headers = list(CSRC.glob("*.h")) + list(CSRC.glob("*.inc")) + [PKG.parent / "include" / "orbx.h"]
    srcs = sorted(CSRC.glob("*.hip")) + sorted(CSRC.glob("*.cpp"))
    cmds = []
    objs = []
    for s in srcs:
        o = obj_dir / (s.name + ".o")
        objs.append(o)
        if _needs(o, s, headers):
            lang = ["-x", "hip", f"--offload-arch={ARCH}"] if s.suffix == ".hip" else ["-D__HIP_PLATFORM_AMD__"]
            san = []
            if sanitize:
                san = (["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fno-omit-frame-pointer", "-g"]
                       if s.suffix == ".hip" else ["-fsanitize=address", "-fno-omit-frame-pointer", "-g"])
            cmds.append([cc, *lang, *COMMON, *san, *(f"-D{d}" for d in defines), "-c", str(s), "-o", str(o)])

    def run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        p = subprocess.run(cmd, capture_output=True, text=True)
        if p.returncode != 0:
            raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{p.stdout}\n{p.stderr}")
        return p.stderr

    with cf.ThreadPoolExecutor(max_workers=jobs or min(8, os.cpu_count() or 4)) as ex:
        for err in ex.map(run, cmds):
            if err and verbose:
                print(err, file=sys.stderr)
    if cmds or not out.exists():
        link = [cc, f"--offload-arch={ARCH}", "-shared", "-pthread", "-o", str(out), *map(str, objs)]
        run(link)
    if defines or sanitize:
        return out
    # C++ adapter demo (the reference-style C++ binding)
    demo_src = PKG / "adapters" / "adapter_demo.cpp"
    demo = PKG / "adapters" / "adapter_demo"
    adapter_hdr = PKG / "adapters" / "orbx_adapters.hpp"
    if demo_src.exists() and (not demo.exists() or _needs(demo, demo_src, [adapter_hdr, LIB])):
        run(["g++", "-O2", "-std=c++17", "-Wall", f"-I{PKG.parent / 'include'}", str(demo_src), "-o", str(demo),
             f"-L{PKG}", "-lorbx", "-Wl,-rpath,$ORIGIN/.."])
    return LIB


if __name__ == "__main__":
    defs = [a[2:] for a in sys.argv[1:] if a.startswith("-D")]
    outs = [a[6:] for a in sys.argv[1:] if a.startswith("--out=")]
    print(build(verbose="-v" in sys.argv, defines=defs, lib=outs[0] if outs else None, sanitize="--asan" in sys.argv))
