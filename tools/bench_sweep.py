"""Time the D=64 plane-sweep cost volume (bench.py's roofline_plane_sweep) alone,
next to the write-bandwidth references of the same output size: ATen's
fill_ (a pure write stream) and copy_ (read + write).  The cost volume is
126 MB written from 4 MB read, so the fill is its practical ceiling.
usage: python tools/bench_sweep.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def _time(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    res = {"plane_sweep": bench.roofline_plane_sweep(dev, iters=50)}
    n = 64 * 2 * 128 * 24 * 80
    out = torch.empty(n, device=dev)
    src = torch.empty(n, device=dev).normal_()
    ms = _time(lambda: out.fill_(1.0))
    res["fill_same_size"] = {"ms": round(ms, 5), "GB/s": round(4 * n / ms / 1e6, 1)}
    ms = _time(lambda: out.copy_(src))
    res["copy_same_size"] = {"ms": round(ms, 5), "GB/s (read+write)": round(8 * n / ms / 1e6, 1)}
    print(json.dumps(res))
