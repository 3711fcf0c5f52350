"""Encoder weight gradients: MIOpen (aten convolution_backward, weight only)
against the native halo weight-gradient kernel (dro_conv2d_backward with only
grad_weight), at the ResNet-18 encoder 3x3 stride-1 shapes of the KITTI
192x640 bench (fnet: 6 images, cnet_pose: 4, cnet_depth: 2).

usage: python tools/bench_enc_wgrad.py [--iters N]
Set DRO_WH_MAX_SPLITS / DRO_WH_TARGET_BLOCKS to try other split policies.
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from dro_sfm_amd.hip import _lib  # noqa: E402
from dro_sfm_amd.hip.conv import _slices, _workspace  # noqa: E402

# (name, images, Cin, Cout, H, W)
SHAPES = [("layer1", 6, 64, 64, 48, 160), ("layer2", 6, 128, 128, 24, 80), ("layer3", 6, 256, 256, 12, 40),
          ("upconv1", 6, 256, 128, 24, 80), ("out_conv", 6, 128, 128, 24, 80),
          ("layer1 pose", 4, 64, 64, 48, 160), ("layer1 depth", 2, 64, 64, 48, 160)]


def timeit(fn, iters):
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    for name, B, Cin, Cout, H, W in SHAPES:
        g = torch.Generator(device=dev).manual_seed(0)
        x = torch.randn(B, Cin, H, W, device=dev, generator=g)
        w = torch.randn(Cout, Cin, 3, 3, device=dev, generator=g) * 0.05
        go = torch.randn(B, Cout, H, W, device=dev, generator=g)
        gw = torch.empty_like(w)
        ws, nws = _workspace(B, H, W, Cin, Cout, 3, 3, dev)
        sl = _slices([x])

        def miopen():
            return torch.ops.aten.convolution_backward(go, x, w, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1,
                                                       [False, True, False])[1]

        def native():
            _lib.check(lib.dro_conv2d_backward(sl, 1, _lib.ptr(w), B, H, W, Cout, 3, 3, 0, ctypes.c_float(1.0),
                                               None, _lib.ptr(go), None, None, None, None, _lib.ptr(gw), None, 0,
                                               None, _lib.ptr(ws), nws,
                                               ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)),
                       "wgrad")
        tm = timeit(miopen, args.iters)
        tn = timeit(native, args.iters)
        ref = torch.ops.aten.convolution_backward(go.double(), x.double(), w.double(), None, [1, 1], [1, 1],
                                                  [1, 1], False, [0, 0], 1, [False, True, False])[1]
        native()
        torch.cuda.synchronize()
        err_n = ((gw.double() - ref).abs().max() / ref.abs().max()).item()
        err_m = ((miopen().double() - ref).abs().max() / ref.abs().max()).item()
        fl = 2.0 * Cout * Cin * 9 * B * H * W
        print(f"{name:13s} B{B} {Cin:3d}->{Cout:3d} {H}x{W}: MIOpen {tm:7.1f} us ({fl / tm / 1e6:5.1f} TF/s, "
              f"err {err_m:.1e})  native {tn:7.1f} us ({fl / tn / 1e6:5.1f} TF/s, err {err_n:.1e})", flush=True)


if __name__ == "__main__":
    main()
