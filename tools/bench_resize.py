"""GPU resize + ToTensor of KITTI frames (csrc/resize.hip) against the
reference's CPU path: PIL BILINEAR resize + ToTensor per frame (what each
data-loader worker does, datasets/augmentations.py:69-160).  One training
step's frames at the metric config: B=2 targets + 2x2 context = 6 frames,
375x1242 -> 192x640.  usage: python tools/bench_resize.py [--iters 50]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
from PIL import Image  # noqa: E402

from dro_sfm_amd.datasets.gpu_transforms import resize_to_tensor, train_transforms  # noqa: E402
from oracle import dro_oracle as O  # noqa: E402  (Pillow jitter chain, timed as the CPU baseline)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    N, h0, w0, H, W = 6, 375, 1242, 192, 640
    frames = np.random.default_rng(0).integers(0, 256, (N, h0, w0, 3), dtype=np.uint8)
    fd = torch.from_numpy(frames).cuda()
    resize_to_tensor(fd, (H, W))
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.iters):
        out = resize_to_tensor(fd, (H, W))
    e1.record()
    torch.cuda.synchronize()
    gpu_ms = e0.elapsed_time(e1) / args.iters
    pil = [Image.fromarray(f) for f in frames]
    t0 = time.perf_counter()
    reps = 5
    for _ in range(reps):
        ref = [torch.from_numpy(np.asarray(p.resize((W, H), Image.BILINEAR)).copy()).permute(2, 0, 1).float().div(255)
               for p in pil]
    cpu_ms = 1e3 * (time.perf_counter() - t0) / reps
    same = all(torch.equal(out[i].cpu(), ref[i]) for i in range(N))
    mb = (N * h0 * w0 * 3 + 2 * N * h0 * W * 3 + N * 3 * H * W * 4) / 1e6
    # full train_transforms (resize -> duplicate -> jitter (0.2, 0.2, 0.2, 0.05) -> to_tensor), B=2, 2 refs
    batch = {"rgb": fd[:2], "rgb_context": [fd[2:4], fd[4:6]]}
    train_transforms(batch, (H, W), (0.2, 0.2, 0.2, 0.05))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.iters):
        train_transforms(batch, (H, W), (0.2, 0.2, 0.2, 0.05))
    torch.cuda.synchronize()
    tt_ms = 1e3 * (time.perf_counter() - t0) / args.iters
    t0 = time.perf_counter()
    for _ in range(2):
        for p in pil:
            r = np.asarray(p.resize((W, H), Image.BILINEAR))
            torch.from_numpy(r.copy()).permute(2, 0, 1).float().div(255)
            j = O.color_jitter_pil(r, [3, 0, 2, 1], [1.1, 0.9, 1.15], 0.03)
            torch.from_numpy(j.copy()).permute(2, 0, 1).float().div(255)
    pil_tt_ms = 1e3 * (time.perf_counter() - t0) / 2
    print(f"train_transforms {N} frames (resize + jitter + to_tensor, originals kept): gpu {tt_ms:.3f} ms wall "
          f"(incl. host parameter draws), Pillow chain on 1 CPU thread {pil_tt_ms:.1f} ms")
    print(f"resize+to_tensor {N} frames {h0}x{w0} -> {H}x{W}: gpu {gpu_ms * 1e3:.1f} us "
          f"({mb / gpu_ms:.0f} GB/s algorithmic over {mb:.1f} MB), PIL on 1 CPU thread {cpu_ms:.2f} ms; "
          f"bit-identical: {same}")


if __name__ == "__main__":
    main()
