"""Warp-cost backward under scatter contention.

The fmap_ref gradient is a bilinear scatter with fp32 atomics.  Where a warp
compresses the reference (consecutive target pixels sampling one cell), a
wave's atomics hit the same addresses and serialise in L2.  This times one
metric-config cost call's backward (B=2, C=128, 24x80, N=2, depth-mean
reduction, as DepthPoseNet.depth_cost_calc) for an ordinary warp and for warps
compressing the reference 2x / 5x / 10x, on the kernel's stream with HIP events.

usage: python tools/bench_warp_contention.py [iters]
"""
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
import torch  # noqa: E402

import dro_sfm_amd.hip as hip  # noqa: E402
from common import kitti_K  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    dev = "cuda"
    g = torch.Generator().manual_seed(3)
    B, C, h, w, N = 2, 128, 24, 80, 2
    K = kitti_K(B).to(dev)
    fmap = torch.randn(B, C, h, w, generator=g).to(dev).requires_grad_(True)
    frefs = torch.randn(N, B, C, h, w, generator=g).to(dev).requires_grad_(True)
    depth = (1.0 + 0.01 * torch.rand(B, 1, h, w, generator=g)).to(dev).requires_grad_(True)
    G = torch.randn(B, C, h, w, generator=g).to(dev)
    for name, tz in (("ordinary", 0.1), ("2x", 1.0), ("5x", 4.0), ("10x", 9.0)):
        pose = torch.zeros(N, B, 6)
        pose[:, :, 2] = tz
        pose[:, :, 3:] = 0.01 * torch.randn(N, B, 3, generator=g)
        pose = pose.to(dev)
        cost = hip.warp_cost(fmap, frefs, depth, pose, K, reduce_mean=True)
        for _ in range(3):
            torch.autograd.grad(cost, (fmap, frefs, depth), G, retain_graph=True)
        torch.cuda.synchronize()
        st = torch.cuda.current_stream()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record(st)
        for _ in range(iters):
            torch.autograd.grad(cost, (fmap, frefs, depth), G, retain_graph=True)
        t1.record(st)
        torch.cuda.synchronize()
        print(f"{name:9s} tz={tz:4.1f}: backward {1e3 * t0.elapsed_time(t1) / iters:7.1f} us per call "
              f"(feature + geometry kernels, gradient zero-fills)", flush=True)


if __name__ == "__main__":
    main()
