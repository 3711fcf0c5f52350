"""Would launching the depth and the pose update block's convolutions as one
grid pay?  Per update-block conv shape (KITTI it8: hd 64, 24x80), times the
depth launch (B=2), the pose launch (B=N*B=4) and ONE launch over B=6 (the
same instantiation over the union of both blocks' pixels approximates a paired
launch), forward and data gradient, as hipGraph replays.

usage: python tools/bench_pairing.py [--iters N]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import dro_sfm_amd.hip as hip  # noqa: E402
sys.path.insert(0, os.path.join(ROOT, "tools"))
from bench_encoder_conv import timeit  # noqa: E402

# (name, Cin, Cout, kh, kw, act)
SHAPES = [
    ("convc1 1x1", 128, 64, 1, 1, "relu"),
    ("convc2 3x3", 64, 64, 3, 3, "relu"),
    ("conv 3x3 fuse", 128, 63, 3, 3, "relu"),
    ("gru zr 1x5", 160, 128, 1, 5, "sigmoid"),
    ("gru q 5x1", 160, 64, 5, 1, "tanh"),
    ("head 3x3", 64, 192, 3, 3, "relu"),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    H, W = 24, 80
    tot = {}
    for name, Cin, Cout, kh, kw, act in SHAPES:
        res = {}
        for B in (2, 4, 6):
            g = torch.Generator(device=dev).manual_seed(B)
            x = torch.randn(B, Cin, H, W, device=dev, generator=g).requires_grad_()
            w = (torch.randn(Cout, Cin, kh, kw, device=dev, generator=g) / (Cin * kh * kw) ** 0.5)
            b = torch.zeros(Cout, device=dev)
            gout = torch.randn(B, Cout, H, W, device=dev, generator=g)

            def fwd():
                with torch.no_grad():
                    return hip.conv2d(x, w, b, act=act)

            def fb():
                x.grad = None
                hip.conv2d(x, w, b, act=act).backward(gout)
            tf = timeit(fwd, args.iters)
            tb = timeit(fb, args.iters) - tf
            res[B] = (tf, tb)
        sep = tuple(res[2][i] + res[4][i] for i in range(2))
        print(f"{name:14s} fwd: B2 {res[2][0]:6.1f} + B4 {res[4][0]:6.1f} = {sep[0]:6.1f} us vs B6 {res[6][0]:6.1f} | "
              f"dgrad: {res[2][1]:6.1f} + {res[4][1]:6.1f} = {sep[1]:6.1f} vs {res[6][1]:6.1f}", flush=True)
        for i, k in enumerate(("fwd", "dgrad")):
            tot.setdefault(k, [0.0, 0.0])
            tot[k][0] += sep[i]
            tot[k][1] += res[6][i]
    for k, (s, p) in tot.items():
        print(f"total {k}: separate {s:.1f} us, one launch {p:.1f} us ({100 * (1 - p / s):.0f} % less)")


if __name__ == "__main__":
    main()
