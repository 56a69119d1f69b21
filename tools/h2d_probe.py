"""Host<->device copy probe for the host-inclusive c2 leg (bench.py
host_inclusive_frames): page-locked H2D / D2H rates for one copy on one
stream against the same bytes split over several streams, and both
directions at once.  Plain torch copies, no library code.

  python3 tools/h2d_probe.py [MB_in] [MB_out]"""
import json
import sys
import time

import torch


def rate(fn, nbytes, reps=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return round(nbytes * reps / (time.perf_counter() - t0) / 1e9, 2)


def split_copy(dst, src, streams):
    n = len(streams)
    step = (src.numel() + n - 1) // n
    cur = torch.cuda.current_stream()
    for i, s in enumerate(streams):
        s.wait_stream(cur)
        with torch.cuda.stream(s):
            dst[i * step:(i + 1) * step].copy_(src[i * step:(i + 1) * step], non_blocking=True)
    for s in streams:
        cur.wait_stream(s)


def main():
    mb_in = int(sys.argv[1]) if len(sys.argv) > 1 else 315
    mb_out = int(sys.argv[2]) if len(sys.argv) > 2 else 66
    hin = torch.empty(mb_in << 20, dtype=torch.uint8).pin_memory()
    din = torch.empty(mb_in << 20, dtype=torch.uint8, device="cuda")
    hout = torch.empty(mb_out << 20, dtype=torch.uint8).pin_memory()
    dout = torch.empty(mb_out << 20, dtype=torch.uint8, device="cuda")
    res = {}
    for n in (1, 2, 4, 8):
        ss = [torch.cuda.Stream() for _ in range(n)]
        res[f"h2d_{n}streams_GBps"] = rate(lambda: split_copy(din, hin, ss), din.numel())
        res[f"d2h_{n}streams_GBps"] = rate(lambda: split_copy(hout, dout, ss), dout.numel())
    a, b = torch.cuda.Stream(), torch.cuda.Stream()

    def both():
        cur = torch.cuda.current_stream()
        for s in (a, b):
            s.wait_stream(cur)
        with torch.cuda.stream(a):
            din.copy_(hin, non_blocking=True)
        with torch.cuda.stream(b):
            hout.copy_(dout, non_blocking=True)
        for s in (a, b):
            cur.wait_stream(s)

    res["both_directions_total_GBps"] = rate(both, din.numel() + dout.numel())
    print(json.dumps(res))


if __name__ == "__main__":
    main()
