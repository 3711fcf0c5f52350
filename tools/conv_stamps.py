"""Per-phase timing of one halo-conv launch from in-kernel s_memtime stamps
(dro_debug_conv_stamps): kernel start -> prologue done -> each K iteration ->
reductions -> epilogue, per block, in shader-clock cycles.

usage: python tools/conv_stamps.py    (runs the bench roofline shape and a 1x1)
Ablations (STAMP_DBG=1,2,4) need a diagnostic build:
make -C dro-sfm_amd/csrc clean all EXTRA=-DDRO_CONV_ABLATE=1
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from dro_sfm_amd.hip import _lib  # noqa: E402
from dro_sfm_amd.hip import conv as hconv  # noqa: E402
from dro_sfm_amd.hip.conv import _slices, _workspace  # noqa: E402

SPLIT = [True]   # STAMP_ENGINE=f32 for the f32-MFMA engine


def run(name, B, hd, H, W, cins, KH, KW, gates=True, reps=5):
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(3)
    h = torch.randn(B, hd, H, W, generator=g, device=dev)
    srcs = [h] + [torch.randn(B, c, H, W, generator=g, device=dev) for c in cins]
    cin = hd + sum(cins)
    cout = 2 * hd if gates else hd
    w = 0.05 * torch.randn(cout, cin, KH, KW, generator=g, device=dev)
    bias = torch.zeros(cout, device=dev)
    out = torch.empty(B, cout, H, W, device=dev)
    rh = torch.empty_like(h)
    ws, nws = _workspace(B, H, W, cin, cout, KH, KW, dev)
    st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    stamps = torch.zeros(4096 * 16, dtype=torch.int64, device=dev)
    sl = _slices(srcs)
    wf = hconv._wsplit(w)[0] if SPLIT[0] else None

    def launch():
        if gates:
            _lib.check(lib.dro_convgru_gates_forward(sl, len(srcs), _lib.ptr(w), _lib.ptr(bias), B, H, W, hd,
                                                     KH, KW, _lib.ptr(out), _lib.ptr(rh), _lib.ptr(wf), _lib.ptr(ws), nws,
                                                     st),
                       "gates")
        else:
            _lib.check(lib.dro_conv2d_forward(sl, len(srcs), _lib.ptr(w), _lib.ptr(bias), B, H, W, cout, KH, KW,
                                              1, ctypes.c_float(1.0), _lib.ptr(out), cout, 0, _lib.ptr(wf), _lib.ptr(ws),
                                              nws, st), "conv")
    for _ in range(3):
        launch()
    torch.cuda.synchronize()
    lib.dro_debug_conv_stamps(_lib.ptr(stamps))
    res = []
    for _ in range(reps):
        stamps.zero_()
        launch()
        torch.cuda.synchronize()
        res.append(stamps.view(-1, 16).cpu().clone())
    lib.dro_debug_conv_stamps(None)
    s = res[-1]
    s = s[s[:, 0] > 0]
    t0 = int(s[:, 0].min())
    print(f"== {name}: {s.shape[0]} blocks")
    start = (s[:, 0] - t0).float()
    print(f"   block start: min 0  median {start.median():.0f}  max {start.max():.0f} cycles")
    setup = (s[:, 0] - s[:, 10]).float()
    espread = (s[:, 11] - s[:, 10]).float()
    print(f"   wave 0 set-up {setup.median():.0f} cycles; last wave enters {espread.median():.0f}"
          f" (max {espread.max():.0f}) after wave 0")
    spread = (s[:, 15] - s[:, 0]).float()
    staged = (s[:, 12] - s[:, 0]).float()
    print(f"   last wave starts {spread.median():.0f} (max {spread.max():.0f}) cycles after wave 0;"
          f" wave 0's first chunk staged after {staged.median():.0f}")
    cols = [k for k in (1, 2, 3, 4, 5, 6, 7, 8, 9, 13, 14) if bool((s[:, k] > 0).all())]
    prev = s[:, 0]
    for k in cols:
        d = (s[:, k] - prev).float()
        label = {1: "prologue", 13: "reductions", 14: "epilogue"}.get(k, f"iter {k - 2}")
        print(f"   {label:11s}: median {d.median():7.0f}  max {d.max():7.0f} cycles")
        prev = s[:, k]
    end = (s[:, cols[-1]] - t0).float()
    print(f"   last block done at {end.max():.0f} cycles after the first start")


def main():
    run("gates 1x5 (roofline shape)", 2, 64, 24, 80, (32, 63, 1), 1, 5, gates=True)
    run("relu 1x1 Cin 128 -> 64", 2, 64, 24, 80, (64,), 1, 1, gates=False)
    run("relu 3x3 Cin 128 -> 64", 2, 64, 24, 80, (64,), 3, 3, gates=False)


if __name__ == "__main__":
    SPLIT[0] = os.environ.get("STAMP_ENGINE", "split") == "split"
    hconv.set_split_engine(SPLIT[0])
    for dbg in os.environ.get("STAMP_DBG", "0").split(","):
        os.environ["DRO_CONV_DBG"] = dbg
        print(f"######## engine {'split-bf16' if SPLIT[0] else 'f32'}, DRO_CONV_DBG={dbg} "
              "(1 no loads, 2 no MFMA, 4 no LDS stores in the K loop)")
        main()
