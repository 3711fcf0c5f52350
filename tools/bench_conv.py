"""Micro-benchmark of the conv engine at the KITTI it8 update-block shapes.

usage: python tools/bench_conv.py [--iters N] [--op gates|blend|gru|all]
Prints per-launch times (HIP events on the current stream) and TFLOP/s.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import dro_sfm_amd.hip as hip  # noqa: E402


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
    return e0.elapsed_time(e1) / iters * 1e3   # us


def gru_inputs(B, pose, hd=64, cd=32, H=24, W=80):
    g = torch.Generator(device="cuda").manual_seed(0)
    h = torch.randn(B, hd, H, W, device="cuda", generator=g).tanh().requires_grad_()
    ctx = torch.randn(B, cd, H, W, device="cuda", generator=g).requires_grad_()
    if pose:
        out = torch.randn(B, hd - 6, H, W, device="cuda", generator=g).requires_grad_()
        pm = torch.randn(B, 6, 1, 1, device="cuda", generator=g).requires_grad_()
        xs = [ctx, out, pm.expand(B, 6, H, W)]
    else:
        out = torch.randn(B, hd - 1, H, W, device="cuda", generator=g).requires_grad_()
        d = torch.rand(B, 1, H, W, device="cuda", generator=g).requires_grad_()
        xs = [ctx, out, d]
    return h, xs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    hd, cin = 64, 64 + 32 + 64
    for name, B, pose in (("depth", 2, False), ("pose", 4, True)):
        h, xs = gru_inputs(B, pose)
        H, W = h.shape[2:]
        P = B * H * W
        for k in ((1, 5), (5, 1)):
            convs = [torch.nn.Conv2d(cin, hd, k, padding=(k[0] // 2, k[1] // 2)).cuda() for _ in range(3)]
            fl_g = 2 * 2 * hd * cin * 5 * P
            fl_q = 2 * hd * cin * 5 * P

            def fwd():
                with torch.no_grad():
                    hip.sepconvgru_half(h, *convs, xs)

            def fwdbwd():
                out = hip.sepconvgru_half(h, *convs, xs)
                out.backward(torch.ones_like(out))

            t_f = timeit(fwd, args.iters)
            t_fb = timeit(fwdbwd, args.iters)
            fl_f = fl_g + fl_q
            print(f"{name} {k}: GRU half fwd {t_f:7.1f} us ({fl_f / t_f / 1e6:6.1f} TF/s)  "
                  f"fwd+bwd {t_fb:7.1f} us ({3 * fl_f / t_fb / 1e6:6.1f} TF/s)", flush=True)
            # single convs
            wzr = torch.cat([convs[0].weight, convs[1].weight], 0).detach()
            bzr = torch.cat([convs[0].bias, convs[1].bias], 0).detach()
            srcs = [h.detach(), *[x.detach() for x in xs]]
            t = timeit(lambda: hip.conv2d(srcs, wzr, bzr, act="sigmoid"), args.iters)
            print(f"   gates conv (Cout {2 * hd}) fwd {t:7.1f} us ({fl_g / t / 1e6:6.1f} TF/s)", flush=True)
            wq = convs[2].weight.detach()
            t = timeit(lambda: hip.conv2d(srcs, wq, convs[2].bias.detach(), act="tanh"), args.iters)
            print(f"   q conv (Cout {hd}) fwd {t:7.1f} us ({fl_q / t / 1e6:6.1f} TF/s)", flush=True)
            ws = [x.detach().requires_grad_() for x in srcs]
            wr = wzr.clone().requires_grad_()

            def cbwd():
                y = hip.conv2d(ws, wr, None, act=None)
                y.backward(torch.ones_like(y))

            t2 = timeit(cbwd, args.iters)
            print(f"   gates conv fwd+bwd {t2:7.1f} us (bwd ~{t2 - t:7.1f} us, "
                  f"{2 * fl_g / max(t2 - t, 1e-3) / 1e6:6.1f} TF/s)", flush=True)


if __name__ == "__main__":
    main()
