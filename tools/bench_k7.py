"""Weight-gradient kernel time of the 7x7 convs: the encoders' stems (stride 2)
and the update blocks' state convs (stride 1) at the KITTI step's shapes,
wgrad_k7_kernel vs wgrad_kernel (DRO_K7_WGRAD_OFF=1, read once per process).
usage: [DRO_K7_WGRAD_OFF=1] [DRO_K7_FWD=1] python tools/bench_k7.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import dro_sfm_amd.hip  # noqa: F401  (registers torch.ops.dro)
    from dro_sfm_amd.hip.conv import _conv_bwd
    dev = torch.device("cuda")
    tag = "wgrad_kernel" if os.environ.get("DRO_K7_WGRAD_OFF") else "wgrad_k7_kernel"
    g = torch.Generator(device=dev).manual_seed(0)
    cases = [("fnet stem", 6, 3, 64, 192, 640, 2), ("cnet_pose stem", 4, 6, 64, 192, 640, 2),
             ("cnet_depth stem", 2, 3, 64, 192, 640, 2), ("convd1 (stride 1)", 2, 1, 128, 24, 80, 1),
             ("convp1 (stride 1)", 4, 6, 128, 24, 80, 1)]
    for name, B, Cin, Cout, H, W, s in cases:
        x = torch.randn(B, Cin, H, W, device=dev, generator=g)
        w = torch.randn(Cout, Cin, 7, 7, device=dev, generator=g)
        Ho, Wo = (H - 1) // s + 1, (W - 1) // s + 1
        gout = torch.randn(B, Cout, Ho, Wo, device=dev, generator=g)
        gw = torch.empty_like(w)
        gb = torch.empty(Cout, device=dev)
        if s == 2:
            fn = lambda: torch.ops.dro.conv2d_strided_backward(x, w, gout, 2, 3, None, gw, None, 0)  # noqa: E731
        else:
            fn = lambda: _conv_bwd([x], w, None, gout, 0, 1.0, [None], [0], gw, gb, 0)  # noqa: E731
        gf = 2.0 * Cout * Cin * 49 * B * Ho * Wo / 1e9
        us = _time(fn)
        print(f"{tag:16s} {name:20s} {us:8.1f} us  {gf / us * 1e3:6.1f} TF/s (incl. finish)", flush=True)
        if s == 2:
            ftag = "fwd_k7s2_kernel" if os.environ.get("DRO_K7_FWD") == "1" else "igemm_kernel"
            us = _time(lambda: torch.ops.dro.conv2d_strided(x, w, None, 2, 3, 0))
            print(f"{ftag:16s} {name:20s} {us:8.1f} us  {gf / us * 1e3:6.1f} TF/s (forward)", flush=True)


def _time(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


if __name__ == "__main__":
    main()
