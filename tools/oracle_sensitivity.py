"""How discontinuous is the training step itself?  The fp64 oracle (CPU) on the
view5 fixture, once plain and then with its three stem convolutions' outputs
multiplied by (1 + noise * N(0,1)) -- with the min-selection and the bilinear
cells of the plain run pinned -- and the relative change of the parameter
gradients.  A smooth function would move by ~noise; this one moves by 0.5-1 %
at noise 1e-6 (one tensor 17 %): kinks that neither the selection nor the cells
cover.  usage: python tools/oracle_sensitivity.py"""
import sys, os, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]
import test_hip_parity as T
T.DEV = "cpu"
from oracle import dro_oracle as O
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
    p = T.params_from_spec(spec)
    p = {k: (v.double().requires_grad_(True) if v.is_floating_point() and "running" not in k else (v.double() if v.is_floating_point() else v)) for k, v in p.items()}
    b = {k: (v.clone().double() if torch.is_tensor(v) else [t.double() for t in v]) for k, v in batch.items()}
    out = O.train_step_loss(p, "it12-h-out", mind, maxd, b, kind="selfsup", forced_selection=sel, cells=book)
    out["loss"].sum().backward()
    return {k: v.grad for k, v in p.items() if getattr(v, "grad", None) is not None}
g0 = run()
sel0 = torch.stack(list(O.LAST_SELECTION), 0).unsqueeze(2)    # [n,B,1,H,W]
rec = O.Cells(record=True)
g0 = run(sel0, rec)
for n, seed in ((1e-6, 0), (1e-6, 1), (1e-7, 0)):
    NOISE[:] = [n, seed]
    for k_ in list(O.PIN_STATS):
        O.PIN_STATS[k_] = 0
    g1 = run(sel0, O.Cells(forced=rec.recorded))
    print("moved", dict(O.PIN_STATS))
    per, l2 = T._grad_check_vs(g1, g0)
    print(n, seed, "L2", l2, sorted(per.items(), key=lambda kv: -kv[1])[:4])
