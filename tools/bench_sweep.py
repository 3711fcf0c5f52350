"""Time the D=64 plane-sweep cost volume (bench.py's roofline_plane_sweep) alone.
usage: python tools/bench_sweep.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    print(json.dumps(bench.roofline_plane_sweep(dev, iters=50)))
