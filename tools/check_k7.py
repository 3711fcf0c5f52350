"""Diagnostic: the 7x7 stem kernels (fwd_k7s2_kernel, wgrad_k7_kernel) against
float64 PyTorch at the step shapes (KITTI and ScanNet batches).
usage: python tools/check_k7.py"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import dro_sfm_amd.hip  # noqa: F401
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    for B, Cin, H, W in [(6, 3, 192, 640), (4, 6, 192, 640), (2, 3, 192, 640), (5, 3, 240, 320), (20, 3, 240, 320),
                         (16, 6, 240, 320), (4, 3, 240, 320), (4, 6, 240, 320), (8, 3, 240, 320)]:
        x = torch.randn(B, Cin, H, W, device=dev, generator=g)
        w = 0.1 * torch.randn(64, Cin, 7, 7, device=dev, generator=g)
        y = torch.ops.dro.conv2d_strided(x, w, None, 2, 3, 0)
        ref = F.conv2d(x.double(), w.double(), stride=2, padding=3)
        ef = float((y.double() - ref).abs().max() / ref.abs().max())
        gout = torch.randn_like(y)
        gw = torch.empty_like(w)
        torch.ops.dro.conv2d_strided_backward(x, w, gout, 2, 3, None, gw, None, 0)
        rw = torch.nn.grad.conv2d_weight(x.double(), w.shape, gout.double(), stride=2, padding=3)
        ew = float((gw.double() - rw).abs().max() / rw.abs().max())
        bad = int(((y.double() - ref).abs() > 1e-3 * ref.abs().max()).sum())
        print(f"B={B:2d} Cin={Cin} {H}x{W}: forward max rel {ef:.2e} ({bad} bad), weight grad {ew:.2e}", flush=True)


if __name__ == "__main__":
    main()
