"""Where the host-inclusive c2 leg (bench.py host_inclusive_frames) spends
its time: the same double-buffered step with parts left out.

  python3 tools/host_leg.py [B] [steps]

Variants: resident (extract + match only), up (uploads only), down
(downloads only), up+ex, ex+down, full."""
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import orb_slam_amd as ox  # noqa: E402
from orb_slam_amd import synth  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    w, h, nf = 640, 480, 1000
    frames = synth.sequence(w, h, B, seed=2000)
    ctx = ox.Context(nfeatures=nf, max_w=w, max_h=h, slots=2 * B)
    ctx.upload(frames, first=0)
    ctx.upload(frames, first=B)
    ctx.set_split(1)
    ctx.set_async_match(True)
    src = ox.HostArray((B, h, w), np.uint8)
    src.array[:] = frames
    o = dict(kps=ox.HostArray((B * nf,), ox.KEYPOINT), desc=ox.HostArray((B * nf, 32), np.uint8),
             n=ox.HostArray((B,), np.int32), m12=ox.HostArray((B * nf,), np.int32), nm=ox.HostArray((B,), np.int32))
    res = {}
    for name, up, ex, down in (("resident", 0, 1, 0), ("up", 1, 0, 0), ("down", 0, 0, 1), ("up+ex", 1, 1, 0),
                               ("ex+down", 0, 1, 1), ("full", 1, 1, 1)):
        it = [0]

        def step():
            k = it[0]
            it[0] += 1
            first, nxt = (k % 2) * B, ((k + 1) % 2) * B
            if up:
                ctx.upload_async(src.array, first=nxt)
            if ex:
                ctx.extract_match(first, B, B, mode="init", window=100, th_low=50, nnratio=0.9, check_ori=True)
            if down:
                ctx.download_async(first, B, o["kps"].array, o["desc"].array, o["n"].array, o["m12"].array,
                                   o["nm"].array)

        for _ in range(3):
            step()
        ctx.sync()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        ctx.sync()
        res[name + "_ms"] = round(1e3 * (time.perf_counter() - t0) / steps, 3)
        print(name, res[name + "_ms"], flush=True)
    res["in_MB"] = round(B * h * w / 1e6, 1)
    res["out_MB"] = round(B * (nf * 64 + 8) / 1e6, 1)
    print(json.dumps(res))
    for v in o.values():
        v.close()
    src.close()
    ctx.close()


if __name__ == "__main__":
    main()
