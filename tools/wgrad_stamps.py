"""Per-phase timing of one batched weight-gradient launch (wgrad_halo_kernel
<..., MULTI>, dro_conv2d_weight_grad_multi) from in-kernel s_memtime stamps:
set-up -> first tile staged -> prologue -> each pixel tile -> loop done -> end.

usage: python tools/wgrad_stamps.py     (STAMP_DBG=0,1,2,4 for the ablations:
                                          1 no loads, 2 no MFMAs, 4 no LDS stores;
                                          they need a diagnostic build:
                                          make -C dro-sfm_amd/csrc clean all EXTRA=-DDRO_CONV_ABLATE=1)
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from dro_sfm_amd.hip import _lib  # noqa: E402
from dro_sfm_amd.hip.conv import DroWgradUse, _slices  # noqa: E402

# (name, source channels, Cout, (KH, KW), act, uses, B, H, W)
CASES = [("convc2 3x3 depth", [64], 64, (3, 3), 1, 8, 2, 24, 80),
         ("head conv_cat 3x3", [64], 192, (3, 3), 1, 8, 2, 24, 80),
         ("fuse 3x3 pose", [64, 64], 58, (3, 3), 1, 8, 4, 24, 80),
         ("gru zr 1x5 depth", [64, 32, 63, 1], 128, (1, 5), 0, 8, 2, 24, 80)]


def run(name, chans, Cout, k, act, uses, B, H, W, reps=3):
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1)
    KH, KW = k
    Cin = sum(chans)
    keep, arr = [], (DroWgradUse * uses)()
    for u in range(uses):
        srcs = [torch.randn(B, c, H, W, device=dev, generator=g) for c in chans]
        dout = torch.randn(B, Cout, H, W, device=dev, generator=g)
        y = torch.rand(B, Cout, H, W, device=dev, generator=g) if act else None
        sl = _slices(srcs)
        keep.append((srcs, dout, y, sl))
        arr[u].srcs = ctypes.cast(sl, ctypes.c_void_p)
        arr[u].dout = dout.data_ptr()
        arr[u].y = y.data_ptr() if y is not None else None
    gw = torch.zeros(Cout, Cin, KH, KW, device=dev)
    gb = torch.zeros(Cout, device=dev)
    nb = int(lib.dro_conv2d_weight_grad_multi_workspace_bytes(uses, B, H, W, Cin, Cout, KH, KW))
    ws = torch.empty(max(nb, 1), dtype=torch.uint8, device=dev)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def launch():
        _lib.check(lib.dro_conv2d_weight_grad_multi(arr, uses, len(chans), B, H, W, Cout, KH, KW, act,
                                                    ctypes.c_float(1.0), _lib.ptr(gw), _lib.ptr(gb), 1,
                                                    _lib.ptr(ws), nb, st), "wgrad multi")
    for _ in range(3):
        launch()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        launch()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 100.0
    stamps = torch.zeros(65536 * 16, dtype=torch.int64, device=dev)
    lib.dro_debug_conv_stamps(_lib.ptr(stamps))
    stamps.zero_()
    launch()
    torch.cuda.synchronize()
    lib.dro_debug_conv_stamps(None)
    s = stamps.view(-1, 16).cpu()
    s = s[s[:, 0] > 0]
    fl = 2.0 * Cout * Cin * KH * KW * uses * B * H * W
    print(f"== {name}: {s.shape[0]} blocks, {us:.1f} us per launch (with finish), {fl / us / 1e6:.1f} TF/s")
    t0 = int(s[:, 0].min())
    end = (s[:, 14] - t0).float()
    print(f"   block start spread: median {float((s[:, 0] - t0).float().median()):.0f}, "
          f"last end {float(end.max()):.0f} cycles")
    prev = s[:, 0]
    for kk, label in ((12, "first tile staged"), (1, "prologue"), (2, "tile 0"), (3, "tile 1"), (4, "tile 2"),
                      (5, "tile 3"), (13, "loop done"), (14, "epilogue")):
        if not bool((s[:, kk] > 0).all()):
            continue
        d = (s[:, kk] - prev).float()
        print(f"   {label:18s}: median {float(d.median()):7.0f}  max {float(d.max()):7.0f} cycles")
        prev = s[:, kk]
    ntiles = uses * B * ((H + 7) // 8) * ((W + 7) // 8)
    print(f"   (tiles per block ~ {ntiles * s.shape[0] / max(s.shape[0], 1) / s.shape[0]:.1f})")


def main():
    for c in CASES:
        run(*c)


if __name__ == "__main__":
    for dbg in os.environ.get("STAMP_DBG", "0").split(","):
        os.environ["DRO_CONV_DBG"] = dbg
        print(f"######## DRO_CONV_DBG={dbg} (1 no loads, 2 no MFMAs, 4 no LDS stores)")
        main()
