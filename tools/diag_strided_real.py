"""Native stride-2 convs vs MIOpen vs fp64 on the REAL operands of a training
step (the view5 fixture, SelfSupModelMF it12-h-out, N=4): every stride-2
encoder conv's input x and output gradient G are captured from one backward
(HIP model, MIOpen strided path), then the data and weight gradients are
recomputed by (a) the native strided HIP path, (b) MIOpen (F.conv2d on the
GPU, autograd), (c) fp64 on the CPU; prints max-rel errors of (a) and (b)
against (c) per conv.  usage: python tools/diag_strided_real.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import test_hip_parity as T  # noqa: E402
from dro_sfm_amd import hip  # noqa: E402
from dro_sfm_amd.networks.optim import extractor  # noqa: E402


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def main():
    from dro_sfm_amd.hip import _lib
    _lib.load()
    f = T.fx("train_step_it12h_selfsup_n4")
    mind, maxd = T.fval(f["min_depth"]), T.fval(f["max_depth"])
    batch = {"rgb": f["image"], "rgb_context": list(f["refs"]), "rgb_original": f["image"],
             "rgb_context_original": list(f["refs"]), "intrinsics": f["K"].clone()}
    model = T._selfsup_model(mind, maxd, "it12h", "it12-h-out")
    captured = []
    orig = extractor.conv3x3

    def spy(m, srcs, act=None):
        srcs_l = list(srcs) if isinstance(srcs, (list, tuple)) else [srcs]
        y = orig(m, srcs, act)
        if m.stride != (1, 1) and y.requires_grad:
            x = srcs_l[0]
            rec = {"m": m, "x": x.detach().clone()}
            y.register_hook(lambda g, rec=rec: rec.__setitem__("G", g.detach().clone()))
            captured.append(rec)
        return y
    extractor.conv3x3 = spy
    out = model(batch)
    out["loss"].sum().backward()
    torch.cuda.synchronize()
    extractor.conv3x3 = orig
    print(f"{len(captured)} stride-2 convs captured")
    for i, rec in enumerate(captured):
        m, x, G = rec["m"], rec["x"], rec.get("G")
        if G is None:
            continue
        s, p = m.stride[0], m.padding[0]
        w = m.weight.detach()
        # fp64 reference
        xr = x.double().cpu().requires_grad_(True)
        wr = w.double().cpu().requires_grad_(True)
        (F.conv2d(xr, wr, None, s, p) * G.double().cpu()).sum().backward()
        # MIOpen
        xm = x.clone().requires_grad_(True)
        wm = w.clone().requires_grad_(True)
        (F.conv2d(xm, wm, None, s, p) * G).sum().backward()
        # native
        xn = x.clone().requires_grad_(True)
        wn = w.clone().requires_grad_(True)
        (hip.conv2d_strided(xn, wn, None, s, p) * G).sum().backward()
        torch.cuda.synchronize()
        print(f"[{i}] {tuple(w.shape)} s{s} p{p} x{tuple(x.shape)}: "
              f"dX miopen {rel(xm.grad, xr.grad):.2e} native {rel(xn.grad, xr.grad):.2e} | "
              f"dW miopen {rel(wm.grad, wr.grad):.2e} native {rel(wn.grad, wr.grad):.2e}",
              flush=True)


if __name__ == "__main__":
    main()
