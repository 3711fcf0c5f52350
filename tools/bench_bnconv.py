"""Kernel times of the BN-fused 3x3 convs (csrc/conv.hip BnFuse) against the
plain conv at the encoders' shapes: EPI 5 (statistics epilogue + last-block
fold), XF 1 (BN + ReLU staged, owner stores), both, and the data-gradient
variants EPI 6 / XF 3.  DRO_BN_ABLATE (read once by the library) switches
parts of the statistics off for timing (results invalid): 1 no arrival /
fold, 2 no partial stores, 4 no row sums.
usage: [DRO_BN_ABLATE=n] python tools/bench_bnconv.py"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    from dro_sfm_amd.hip import _lib, bnconv
    from dro_sfm_amd.hip._lib import ptr, stream_of
    from dro_sfm_amd.hip.conv import _workspace
    lib = _lib.load()
    dev = torch.device("cuda")
    tag = os.environ.get("DRO_BN_ABLATE", "0")
    for (B, C, H, W) in [(6, 64, 48, 160), (6, 128, 24, 80), (2, 256, 12, 40)]:
        g = torch.Generator(device=dev).manual_seed(0)
        x = torch.randn(B, C, H, W, device=dev, generator=g)
        w = 0.05 * torch.randn(C, C, 3, 3, device=dev, generator=g)
        z = torch.empty_like(x)
        y = torch.empty_like(x)
        gx = torch.empty_like(x)
        bn = torch.nn.BatchNorm2d(C).to(dev)
        st_in = bnconv.BnSite(bn, (B, C, H, W), dev)
        st_out = bnconv.BnSite(bn, (B, C, H, W), dev)
        smean, sinv = torch.empty(C, device=dev), torch.empty(C, device=dev)
        prm = st_out.params(bn, smean, sinv)
        ws, nws = _workspace(B, H, W, C, C, 3, 3, dev)
        s = stream_of(x)

        def fwd(xf, stats):
            return lib.dro_conv2d_bn_forward(ptr(x), B, H, W, C, ptr(w), C, ptr(st_in.fwd) if xf else None, None,
                                             ptr(y) if xf else None, ctypes.byref(prm) if stats else None,
                                             ptr(st_out.fwd) if stats else None, ptr(z), ptr(ws), nws, s)

        gp = bnconv.DroBnGradParams(y.data_ptr(), x.data_ptr(), None, smean.data_ptr(), sinv.data_ptr(), None, None)

        def bwd(mode):
            if mode == "epi6":
                return lib.dro_conv2d_bn_backward_data(ptr(w), B, H, W, C, C, ptr(x), None, None, None,
                                                       ctypes.byref(gp), ptr(st_in.bwd), ptr(gx), 0, ptr(ws), nws, s)
            if mode == "xf3":
                return lib.dro_conv2d_bn_backward_data(ptr(w), B, H, W, C, C, ptr(x), ptr(st_in.bwd), ptr(x),
                                                       ptr(y), None, None, ptr(gx), 0, ptr(ws), nws, s)
            return lib.dro_conv2d_bn_backward_data(ptr(w), B, H, W, C, C, ptr(x), None, None, None, None, None,
                                                   ptr(gx), 0, ptr(ws), nws, s)

        cases = [("fwd plain", lambda: fwd(False, False)), ("fwd EPI5", lambda: fwd(False, True)),
                 ("fwd XF1", lambda: fwd(True, False)), ("fwd XF1+EPI5", lambda: fwd(True, True)),
                 ("dgrad plain", lambda: bwd("plain")), ("dgrad EPI6", lambda: bwd("epi6")),
                 ("dgrad XF3", lambda: bwd("xf3"))]
        fwd(False, True)   # coefficients for XF 1
        bwd("epi6")        # and XF 3
        torch.cuda.synchronize()
        for name, fn in cases:
            for _ in range(5):
                assert fn() == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(50):
                fn()
            e1.record()
            torch.cuda.synchronize()
            print(f"ablate={tag} B={B} C={C} {H}x{W} {name:14s} {e0.elapsed_time(e1) / 50 * 1e3:8.1f} us", flush=True)


if __name__ == "__main__":
    main()
