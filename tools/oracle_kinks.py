"""Which kinks make the training step discontinuous?  The fp64 oracle (CPU) on
the view5 fixture, plain and with its stem outputs multiplied by
(1 + 1e-6 N(0,1)) -- selection and bilinear cells of the plain run pinned, as
in tools/oracle_sensitivity.py -- and, in addition, the branch of every call
of one class of non-smooth function pinned to the plain run's at near-kinks:
  relu   F.relu / torch.relu (update-block and decoder convs, GRU inputs)
  abs    Tensor.abs on tensors that carry a gradient (L1 residuals, smoothness)
  clamp  torch.clamp on tensors that carry a gradient (SSIM, depth range)
The class whose pinning brings the gradient change back to ~1e-6 is the one
the native / MIOpen stem realisations fall on different sides of (DESIGN.md
2b).  usage: python tools/oracle_kinks.py [relu,abs,clamp]"""
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]
import test_hip_parity as T  # noqa: E402

T.DEV = "cpu"
from oracle import dro_oracle as O  # noqa: E402

TOL = float(os.environ.get("KINK_TOL", "1e-5"))    # near-kink margin, relative to the tensor's max |value|
BOOK = {"far_calls": [], "mode": None, "pin": set(), "rec": {}, "i": {}, "moved": {}}
_relu, _trelu, _abs, _clamp, _tclamp = F.relu, torch.relu, torch.Tensor.abs, torch.clamp, torch.Tensor.clamp


def _key(kind):
    i = BOOK["i"].get(kind, 0)
    BOOK["i"][kind] = i + 1
    return kind, i


def _pinned(kind, v, natural_mask, apply):
    """natural result, or -- in force mode for a pinned class -- the recorded
    branch at elements within TOL of the kink where it differs."""
    k = _key(kind)
    m = natural_mask(v.detach())
    if BOOK["mode"] == "record":
        BOOK["rec"][k] = m
    elif BOOK["mode"] == "force" and kind in BOOK["pin"] and k in BOOK["rec"]:
        f = BOOK["rec"][k]
        scale = v.detach().abs().max().clamp_min(1e-300)
        near = _kdist(kind, v.detach()) <= TOL * scale
        use = (f != m) & near
        BOOK["moved"][kind] = BOOK["moved"].get(kind, 0) + int(use.sum())
        far = int(((f != m) & ~near).sum())
        if far:
            BOOK["moved"][kind + "_far"] = BOOK["moved"].get(kind + "_far", 0) + far
            BOOK["far_calls"].append((k, far, float((_kdist(kind, v.detach())[(f != m) & ~near] / scale).min())))
        if use.any():
            return apply(v, torch.where(use, f, m))
    return apply(v, m)


def _kdist(kind, v):
    if kind == "clamp":
        lo, hi = BOOK["clamp_bounds"]
        d = torch.full_like(v, float("inf"))
        if lo is not None:
            d = torch.minimum(d, (v - lo).abs())
        if hi is not None:
            d = torch.minimum(d, (v - hi).abs())
        return d
    return v.abs()


def relu(v, inplace=False):
    if not v.requires_grad:
        return _relu(v)
    return _pinned("relu", v, lambda d: d > 0, lambda x, m: x * m.to(x.dtype))


def t_abs(v):
    if not v.requires_grad:
        return _abs(v)
    return _pinned("abs", v, lambda d: d >= 0, lambda x, m: x * (2 * m.to(x.dtype) - 1))


def clamp(v, min=None, max=None):
    if not v.requires_grad or (min is None and max is None) or torch.is_tensor(min) or torch.is_tensor(max):
        return _clamp(v, min, max)
    BOOK["clamp_bounds"] = (min, max)

    def region(d):   # 0 below, 1 inside, 2 above
        r = torch.ones_like(d, dtype=torch.uint8)
        if min is not None:
            r = torch.where(d < min, torch.zeros_like(r), r)
        if max is not None:
            r = torch.where(d > max, torch.full_like(r, 2), r)
        return r

    def apply(x, r):
        out = x
        if min is not None:
            out = torch.where(r == 0, torch.full_like(x, min) + 0 * x, out)
        if max is not None:
            out = torch.where(r == 2, torch.full_like(x, max) + 0 * x, out)
        return out
    return _pinned("clamp", v, region, apply)


def t_clamp(v, min=None, max=None):
    return clamp(v, min, max)


F.relu = relu
torch.relu = relu
torch.Tensor.abs = t_abs
torch.clamp = clamp
torch.Tensor.clamp = t_clamp

f = T.fx("train_step_it12h_selfsup_n4")
mind, maxd = T.fval(f["min_depth"]), T.fval(f["max_depth"])
spec = T.load_spec(os.path.join(T.G, "depthposenet_it12h_keys.json"))
batch = {"rgb": f["image"], "rgb_context": list(f["refs"]), "rgb_original": f["image"],
         "rgb_context_original": list(f["refs"]), "intrinsics": f["K"].clone()}
orig_conv = O._conv
NOISE = [0.0, 0]


def noisy_conv(p, name, x, stride=1, pad=0):
    y = orig_conv(p, name, x, stride, pad)
    if name.endswith("conv1") and "layer" not in name and NOISE[0] > 0:
        g = torch.Generator().manual_seed(NOISE[1])
        y = y * (1 + NOISE[0] * torch.randn(y.shape, generator=g, dtype=y.dtype))
    return y


O._conv = noisy_conv


def run(sel=None, book=None):
    BOOK["i"] = {}
    p = T.params_from_spec(spec)
    p = {k: (v.double().requires_grad_(True) if v.is_floating_point() and "running" not in k
             else (v.double() if v.is_floating_point() else v)) for k, v in p.items()}
    b = {k: (v.clone().double() if torch.is_tensor(v) else [t.double() for t in v]) for k, v in batch.items()}
    out = O.train_step_loss(p, "it12-h-out", mind, maxd, b, kind="selfsup", forced_selection=sel, cells=book)
    out["loss"].sum().backward()
    return {k: v.grad for k, v in p.items() if getattr(v, "grad", None) is not None}


def main():
    pins = [s for s in (sys.argv[1] if len(sys.argv) > 1 else "relu,abs,clamp").split(",") if s]
    run()
    sel0 = torch.stack(list(O.LAST_SELECTION), 0).unsqueeze(2)
    rec = O.Cells(record=True)
    BOOK["mode"] = "record"
    g0 = run(sel0, rec)
    print("calls recorded:", {k: sum(1 for kk in BOOK["rec"] if kk[0] == k) for k in ("relu", "abs", "clamp")})
    for pin in [pins]:
        for n, seed in ((1e-6, 0), (1e-6, 1)):
            NOISE[:] = [n, seed]
            BOOK.update(mode="force", pin=set(pin), moved={}, far_calls=[])
            for k_ in list(O.PIN_STATS):
                O.PIN_STATS[k_] = 0
            g1 = run(sel0, O.Cells(forced=rec.recorded))
            per, l2 = T._grad_check_vs(g1, g0)
            worst = sorted(per.items(), key=lambda kv: -kv[1])[:3]
            print(f"pin {'+'.join(pin) or 'none':16s} noise {n:g} seed {seed}: L2 {l2:.2e} worst "
                  + ", ".join(f"{k} {e:.1e}" for k, e in worst) + f"  moved {BOOK['moved']} oracle {dict(O.PIN_STATS)}", flush=True)
            if BOOK["far_calls"]:
                print("   first far flips (call, count, min distance / max):", BOOK["far_calls"][:6])


if __name__ == "__main__":
    main()
