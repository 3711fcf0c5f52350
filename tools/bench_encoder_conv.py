"""Encoder 3x3 stride-1 convolutions (ResNet-18 trunk + fusion head of the
KITTI fnet/cnet encoders): MIOpen (what the encoders run on) against the
native engines -- split-bf16 (xconv) and f32 MFMA (dconv) -- for forward,
data gradient and weight gradient, each timed as a hipGraph replay of --iters
calls (device time per call), with the max relative error against MIOpen.

usage: python tools/bench_encoder_conv.py [--iters N]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import dro_sfm_amd.hip as hip  # noqa: E402
from dro_sfm_amd.hip import conv as hconv  # noqa: E402

# (name, B, Cin, Cout, H, W)
SHAPES = [
    ("layer1 fnet", 6, 64, 64, 48, 160),
    ("layer2 fnet", 6, 128, 128, 24, 80),
    ("layer3 fnet", 6, 256, 256, 12, 40),
    ("upconv1 fnet", 6, 256, 128, 24, 80),
    ("out_conv fnet", 6, 128, 128, 24, 80),
    ("layer1 cnet", 2, 64, 64, 48, 160),
    ("layer3 cnet", 2, 256, 256, 12, 40),
]


def timeit(fn, iters):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=s):
            for _ in range(iters):
                fn()
    torch.cuda.current_stream().wait_stream(s)
    graph.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    graph.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def rel(a, b):
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    for name, B, Cin, Cout, H, W in SHAPES:
        g = torch.Generator(device=dev).manual_seed(5)
        x = torch.randn(B, Cin, H, W, device=dev, generator=g)
        w = torch.randn(Cout, Cin, 3, 3, device=dev, generator=g) / (Cin * 9) ** 0.5
        gout = torch.randn(B, Cout, H, W, device=dev, generator=g)
        flops = 2.0 * B * Cout * Cin * 9 * H * W
        conv_bwd = torch.ops.aten.convolution_backward

        def mi_fwd():
            return F.conv2d(x, w, padding=1)

        def mi_dgrad():
            return conv_bwd(gout, x, w, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1, [True, False, False])[0]

        def mi_wgrad():
            return conv_bwd(gout, x, w, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1, [False, True, False])[1]

        t = {"miopen": (timeit(mi_fwd, args.iters), timeit(mi_dgrad, args.iters), timeit(mi_wgrad, args.iters))}
        y_ref, dx_ref, dw_ref = mi_fwd(), mi_dgrad(), mi_wgrad()
        err = {}
        xg = x.clone().requires_grad_()
        wg = w.clone().requires_grad_()
        for eng in ("split", "f32"):
            hconv.set_split_engine(eng == "split")
            with hconv.weight_grad_scope():
                def fwd():
                    with torch.no_grad():
                        return hip.conv2d(x, w)

                def fb_data():
                    xg.grad = None
                    hip.conv2d(xg, w).backward(gout)

                def fb_weight():
                    wg.grad = None
                    hip.conv2d(x, wg).backward(gout)
                tf = timeit(fwd, args.iters)
                td = timeit(fb_data, args.iters) - tf
                tw = timeit(fb_weight, args.iters) - tf
                t[eng] = (tf, td, tw)
            with hconv.weight_grad_scope():   # fresh scope: the first use returns its gradient
                y = fwd()
                fb_data()
                fb_weight()
                err[eng] = (rel(y, y_ref), rel(xg.grad, dx_ref), rel(wg.grad, dw_ref))
        hconv.set_split_engine(False)
        print(f"== {name}: B{B} Cin {Cin} Cout {Cout} {H}x{W} ({flops / 1e9:.2f} GFLOP per pass)", flush=True)
        for eng, (tf, td, tw) in t.items():
            e = err.get(eng)
            es = f"  rel err vs miopen y {e[0]:.1e} dx {e[1]:.1e} dw {e[2]:.1e}" if e else ""
            print(f"   {eng:6s} fwd {tf:7.1f} us ({flops / tf / 1e6:5.1f} TF/s)  dgrad {td:7.1f} us "
                  f"({flops / max(td, 1e-3) / 1e6:5.1f})  wgrad {tw:7.1f} us ({flops / max(tw, 1e-3) / 1e6:5.1f})"
                  + es, flush=True)


if __name__ == "__main__":
    main()
