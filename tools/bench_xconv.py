"""A/B micro-benchmark: split-bf16 engine (xconv) vs f32-MFMA engine (dconv) at
the update-block conv shapes of the KITTI it8 / it12-h workloads.

usage: python tools/bench_xconv.py [--iters N] [--rounds R]
Per shape: forward and data-gradient times of both engines (HIP events around a
hipGraph replay of the calls, interleaved rounds in one process, median), TFLOP/s of the
algorithmic work, and the max relative difference between the engines and
against an fp64 CPU reference.
"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import dro_sfm_amd.hip as hip  # noqa: E402
from dro_sfm_amd.hip import conv as hconv  # noqa: E402

# (name, source channels, Cout, (KH, KW), act, B, H, W)
SHAPES = [
    ("gru zr 1x5 depth", [64, 32, 63, 1], 128, (1, 5), "sigmoid", 2, 24, 80),
    ("gru q 1x5 depth", [64, 32, 63, 1], 64, (1, 5), "tanh", 2, 24, 80),
    ("gru zr 5x1 pose", [64, 32, 58, 6], 128, (5, 1), "sigmoid", 4, 24, 80),
    ("gru zr 1x5 h128", [128, 32, 127, 1], 256, (1, 5), "sigmoid", 8, 30, 40),
    ("proj 3x3 cost", [64], 64, (3, 3), "relu", 2, 24, 80),
    ("proj 3x3 fuse", [64, 64], 63, (3, 3), "relu", 2, 24, 80),
    ("head 3x3", [64], 128, (3, 3), "relu", 2, 24, 80),
    ("mask 1x1", [256], 576, (1, 1), None, 2, 24, 80),
    ("convc1 1x1", [128], 128, (1, 1), "relu", 2, 24, 80),
]


def timeit(fn, iters):
    """Device time per call: `iters` calls captured in one hipGraph and replayed
    (no Python / launch overhead in the measurement)."""
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
    return e0.elapsed_time(e1) / iters * 1e3   # us


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    for name, chans, Cout, (KH, KW), act, B, H, W in SHAPES:
        g = torch.Generator(device="cuda").manual_seed(3)
        srcs = [torch.randn(B, c, H, W, device="cuda", generator=g) for c in chans]
        Cin = sum(chans)
        w = torch.randn(Cout, Cin, KH, KW, device="cuda", generator=g) / (Cin * KH * KW) ** 0.5
        bias = 0.1 * torch.randn(Cout, device="cuda", generator=g)
        gout = torch.randn(B, Cout, H, W, device="cuda", generator=g)
        flops = 2.0 * Cout * Cin * KH * KW * B * H * W
        xs = [s.clone().requires_grad_() for s in srcs]

        def fwd():
            with torch.no_grad():
                return hip.conv2d(srcs, w, bias, act=act)

        def fb():
            for x in xs:
                x.grad = None
            y = hip.conv2d(xs, w, bias, act=act)
            y.backward(gout)

        res = {True: ([], []), False: ([], [])}
        outs = {}
        for _ in range(args.rounds):
            for split in (True, False):
                hconv.set_split_engine(split)
                # one weight generation: the weight is split once, as in a training forward
                with hconv.weight_grad_scope():
                    tf = timeit(fwd, args.iters)
                    tfb = timeit(fb, args.iters)
                    res[split][0].append(tf)
                    res[split][1].append(tfb - tf)
                    outs[split] = (fwd(), [x.grad.clone() for x in xs])
        hconv.set_split_engine(False)
        # fp64 reference
        xr = torch.cat([s.double().cpu() for s in srcs], 1).requires_grad_()
        pre = F.conv2d(xr, w.double().cpu(), bias.double().cpu(), padding=(KH // 2, KW // 2))
        yr = {None: pre, "relu": torch.relu(pre), "sigmoid": torch.sigmoid(pre), "tanh": torch.tanh(pre)}[act]
        yr.backward(gout.double().cpu())
        gx_ref = torch.cat([x.grad for x in xs], 1) if False else xr.grad
        line = f"{name:18s} B{B} {H}x{W} Cin {Cin:3d} Cout {Cout:3d}:"
        for split in (True, False):
            tf = statistics.median(res[split][0])
            tb = statistics.median(res[split][1])
            y, gx = outs[split]
            gcat = torch.cat(gx, 1)
            line += (f"  [{'split' if split else 'f32  '}] fwd {tf:6.1f} us {flops / tf / 1e6:6.1f} TF/s"
                     f" dgrad {tb:6.1f} us ({flops / max(tb, 1e-3) / 1e6:6.1f} TF/s)"
                     f" err y {rel(y, yr):.1e} dx {rel(gcat, gx_ref):.1e}")
        print(line, flush=True)


if __name__ == "__main__":
    main()
