"""Locate the photometric pose-gradient deviation on the golden fixtures:
HIP vs the fp64 oracle per loss term (L1 only, SSIM only, full; smoothness
off), per (b, ref, prediction) pose, and the reference fp32 fixture's own
distance for scale."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
import torch  # noqa: E402
from common import load_fixture  # noqa: E402
from oracle import dro_oracle as O  # noqa: E402
import dro_sfm_amd.hip as hip  # noqa: E402

for name in ("photo_loss_mean", "photo_loss_noauto", "photo_loss"):
    d = load_fixture(os.path.join(ROOT, "tests", "golden", name + ".npz"))
    n, B, _, H, W = d["inv_depths"].shape
    N = d["poses"].shape[1]
    auto, rmin = bool(int(d["automask"])), bool(int(d["reduce_min"]))
    for ssim_w, smooth_w in ((0.85, 0.001), (0.0, 0.0), (1.0, 0.0), (0.85, 0.0)):
        ig = d["inv_depths"].cuda().requires_grad_(True)
        vg = d["poses"].cuda().requires_grad_(True)
        loss, _, sel = hip.photometric_loss(d["image"].cuda(), d["context"].cuda(), ig, vg.permute(1, 2, 0, 3),
                                            d["K"].cuda(), ssim_w=ssim_w, smooth_w=smooth_w, automask=auto,
                                            reduce_min=rmin, return_selection=True)
        loss.sum().backward()
        res = {}
        for dt in (torch.float32, torch.float64):
            ic = d["inv_depths"].to(dt).clone().requires_grad_(True)
            vc = d["poses"].to(dt).clone().requires_grad_(True)
            out = O.photometric_decay_loss(d["image"].to(dt), list(d["context"].to(dt)), list(ic), d["K"].to(dt),
                                           d["K"].to(dt), [[vc[:, j, i] for i in range(n)] for j in range(N)],
                                           ssim_w=ssim_w, smooth_w=smooth_w, automask=auto,
                                           reduce="min" if rmin else "mean",
                                           forced_selection=sel.cpu().unsqueeze(2) if rmin else None)
            out["loss"].sum().backward()
            res[dt] = (float(out["loss"]), ic.grad.double(), vc.grad.double())
        l64, gi64, gv64 = res[torch.float64]
        _, gi32, gv32 = res[torch.float32]
        m = gv64.abs().max()
        eh = (vg.grad.cpu().double() - gv64).abs()
        e32 = (gv32 - gv64).abs()
        print(f"{name} ssim_w={ssim_w} smooth={smooth_w}: loss rel {abs(float(loss) - l64) / abs(l64):.2e}; "
              f"pose max-rel hip {float(eh.max() / m):.2e} fp32-oracle {float(e32.max() / m):.2e}; "
              f"inv max-rel hip {float((ig.grad.cpu().double() - gi64).abs().max() / gi64.abs().max()):.2e} "
              f"fp32-oracle {float((gi32 - gi64).abs().max() / gi64.abs().max()):.2e}")
        worst = eh.flatten().argsort(descending=True)[:4]
        for f in worst.tolist():
            b, j, i, k = (int(v) for v in torch.unravel_index(torch.tensor(f), eh.shape))
            print(f"    b{b} j{j} i{i} k{k}: hip {float(vg.grad[b, j, i, k]):+.6e} o64 {float(gv64[b, j, i, k]):+.6e} "
                  f"o32 {float(gv32[b, j, i, k]):+.6e}")
