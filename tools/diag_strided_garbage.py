"""Does hip.conv2d_strided write every element of its outputs?  The caching
allocator is first filled with NaN blocks of the sizes the op will ask for
and released, so any element the kernels leave unwritten shows up as NaN
(a fresh allocation is often zero by luck).  Runs the encoder's strided
shapes (tests/test_conv_engine.py) forward and backward against fp64
F.conv2d.  usage: python tools/diag_strided_garbage.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import dro_sfm_amd.hip as hip  # noqa: E402

CASES = [
    (2, 64, 128, 48, 160, 3, 2, 1), (2, 128, 256, 24, 80, 3, 2, 1), (2, 64, 128, 48, 160, 1, 2, 0),
    (2, 3, 64, 64, 96, 7, 2, 3), (1, 6, 64, 47, 81, 7, 2, 3), (5, 64, 128, 16, 24, 3, 2, 1),
    (5, 64, 128, 16, 24, 1, 2, 0), (5, 128, 256, 8, 12, 3, 2, 1), (3, 64, 128, 16, 24, 3, 2, 1),
    (3, 64, 128, 16, 24, 1, 2, 0), (2, 128, 256, 8, 12, 1, 2, 0), (1, 64, 128, 30, 40, 3, 2, 1),
    (1, 128, 256, 15, 20, 3, 2, 1), (1, 128, 256, 15, 20, 1, 2, 0),
]


def poison(numels):
    keep = [torch.full((n,), float("nan"), device="cuda") for n in numels for _ in range(3)]
    torch.cuda.synchronize()
    del keep


def main():
    dev = torch.device("cuda", 0)
    for B, Cin, Cout, Hi, Wi, k, s, p in CASES:
        g = torch.Generator().manual_seed(Cin + Cout + Hi)
        x = torch.randn(B, Cin, Hi, Wi, generator=g)
        w = torch.randn(Cout, Cin, k, k, generator=g) / (Cin * k * k) ** 0.5
        xr, wr = x.double().requires_grad_(), w.double().requires_grad_()
        ref = F.conv2d(xr, wr, stride=s, padding=p)
        G = torch.randn(ref.shape, generator=g)
        (ref * G.double()).sum().backward()
        poison([x.numel(), w.numel(), ref.numel(), 4 * ref.numel(), 4 * x.numel()])
        xd, wd = x.to(dev).requires_grad_(), w.to(dev).requires_grad_()
        out = hip.conv2d_strided(xd, wd, None, s, p)
        (out * G.to(dev)).sum().backward()
        torch.cuda.synchronize()
        res = []
        for name, a, b in (("out", out, ref), ("dx", xd.grad, xr.grad), ("dw", wd.grad, wr.grad)):
            a = a.detach().double().cpu()
            nan = int(torch.isnan(a).sum())
            err = float((a - b.detach()).abs().nan_to_num(1e30).max() / b.detach().abs().max())
            res.append(f"{name} rel {err:.2e} nan {nan}")
        print((B, Cin, Cout, Hi, Wi, k, s, p), " | ".join(res), flush=True)


if __name__ == "__main__":
    main()
