"""Depth evaluation metrics: hip.depth_metrics (csrc/metrics.hip) against the
reference algorithm (compute_depth_metrics, dro_sfm/utils/depth.py:259-343, as
restated by oracle/dro_oracle.py) run through ATen on the same GPU and on the
host CPU.  KITTI eval shape: B=4, 375x1242 LiDAR-like ground truth (5 % valid),
192x640 prediction, garg crop, median scaling.
usage: python tools/bench_metrics.py [--iters 20]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import dro_sfm_amd.hip as hip  # noqa: E402
from oracle import dro_oracle as O  # noqa: E402  (the reference algorithm, timed as the comparison)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    B, H, W, h, w, lo, hi = 4, 375, 1242, 192, 640, 1e-3, 80.0
    g = torch.Generator().manual_seed(3)
    gt = torch.zeros(B, 1, H, W)
    keep = torch.rand(B, 1, H, W, generator=g) < 0.05
    gt[keep] = (1.0 + 79.0 * torch.rand(B, 1, H, W, generator=g))[keep]
    pred = 1.0 + 40.0 * torch.rand(B, 1, h, w, generator=g)
    gd, pd = gt.cuda(), pred.cuda()

    def timed(fn, iters, sync):
        fn()
        sync()
        t0 = time.perf_counter()
        for _ in range(iters):
            out = fn()
        sync()
        return out, 1e3 * (time.perf_counter() - t0) / iters

    hs = torch.cuda.synchronize
    out, t_hip = timed(lambda: hip.depth_metrics(gd, pd, lo, hi, crop="garg"), args.iters, hs)
    ref_gpu, t_aten = timed(lambda: O.depth_metrics(gd, pd, lo, hi, "garg"), args.iters, hs)
    ref_cpu, t_cpu = timed(lambda: O.depth_metrics(gt, pred, lo, hi, "garg"), max(2, args.iters // 4),
                           lambda: None)
    err = float(((out.cpu().double() - ref_cpu.double()).abs() / ref_cpu.double().abs().clamp(min=1e-12)).max())
    print(f"depth metrics B={B} gt {H}x{W} pred {h}x{w} garg+median: hip {t_hip:.3f} ms, "
          f"reference algorithm on ATen/GPU {t_aten:.3f} ms, on CPU ({torch.get_num_threads()} threads) "
          f"{t_cpu:.3f} ms; max rel diff vs CPU {err:.2e}")


if __name__ == "__main__":
    main()
