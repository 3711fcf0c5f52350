"""Where do the train-step gradient deviations come from?  For each case:
loss (HIP, fp32 oracle, fp64 oracle) and per-tensor max-rel of HIP and of
the fp32 oracle against the fp64 oracle (kernel's min-selection forced), with
the encoders on MIOpen and on PyTorch's native convolutions.

usage: python tools/diag_train_steps.py [case ...]
cases: it8flip view5golden scannet_sup scannet_view5
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

import test_hip_parity as T  # noqa: E402
from common import fval, load_spec, smooth_images  # noqa: E402
from oracle import dro_oracle as O  # noqa: E402


def run(case, cudnn):
    G = T.G
    flip = False
    if case == "it8flip":
        d, dn = T.fx("train_step_it8"), T.fx("depthposenet_it8")
        tag, version, kind, flip = "it8", "it8-seq4-inter-out", "selfsup", True
        mind, maxd = fval(dn["min_depth"]), fval(dn["max_depth"])
        N = d["refs"].shape[0]
        batch = {"rgb": d["image"], "rgb_context": list(d["refs"]), "rgb_original": d["image"],
                 "rgb_context_original": list(d["refs"]), "intrinsics": d["K"].clone()}
    elif case == "view5golden":
        f = T.fx("train_step_it12h_selfsup_n4")
        tag, version, kind = "it12h", "it12-h-out", "selfsup"
        mind, maxd = fval(f["min_depth"]), fval(f["max_depth"])
        batch = {"rgb": f["image"], "rgb_context": list(f["refs"]), "rgb_original": f["image"],
                 "rgb_context_original": list(f["refs"]), "intrinsics": f["K"].clone()}
    else:
        tag, version = "it12h", "it12-h-out"
        kind = "sup" if case == "scannet_sup" else "selfsup"
        N = 2 if kind == "sup" else 4
        B, H, W = 1, 240, 320
        mind, maxd = 0.2, 10.0
        img = smooth_images(B, H, W, 81, detail=0.3)
        refs = [torch.roll(img, 2 * (j + 1), 3) * 0.9 + 0.1 * smooth_images(B, H, W, 82 + j, detail=0.3)
                for j in range(N)]
        batch = {"rgb": img, "rgb_context": refs, "rgb_original": img, "rgb_context_original": refs,
                 "intrinsics": T._scannet_K(B)}
        if kind == "sup":
            g = torch.Generator().manual_seed(83)
            batch["depth"] = 0.5 + 9.5 * torch.rand(B, 1, H, W, generator=g)
            batch["pose_context"] = [O.vec_to_transform(torch.cat([0.05 * torch.randn(B, 3, generator=g),
                                                                  0.01 * torch.randn(B, 3, generator=g)], 1))
                                     for _ in range(N)]
    spec = load_spec(os.path.join(G, f"depthposenet_{tag}_keys.json"))
    cpu_batch = {k: (v.cpu().clone() if torch.is_tensor(v) else [t.cpu().clone() for t in v]) for k, v in batch.items()}
    gb = {k: (v.cuda() if torch.is_tensor(v) else [t.cuda() for t in v]) for k, v in batch.items()}
    with torch.backends.cudnn.flags(enabled=cudnn):
        model = (T._selfsup_model if kind == "selfsup" else T._sup_model)(mind, maxd, tag, version)
        out = model(gb, flip=flip)
        out["loss"].sum().backward()
    forced = model._photometric_loss.last_selection.cpu().unsqueeze(2) if kind == "selfsup" else None
    l64, g64 = T._oracle_grads(spec, version, mind, maxd, cpu_batch, kind, torch.float64, forced, flip)
    l32, g32 = T._oracle_grads(spec, version, mind, maxd, cpu_batch, kind, torch.float32, forced, flip)
    lh = float(out["loss"])
    print(f"== {case} cudnn={cudnn}: loss hip {lh:.7f} o32 {float(l32):.7f} o64 {float(l64):.7f} "
          f"rel hip {abs(lh - float(l64)) / abs(float(l64)):.2e} o32 {abs(float(l32) - float(l64)) / abs(float(l64)):.2e}")
    if "metrics" in out:
        print("   hip metrics", {k: round(float(v), 7) for k, v in out["metrics"].items() if torch.is_tensor(v) and v.numel() == 1})
    rows = []
    for k, v in model.depth_net.named_parameters():
        if k in g64 and v.grad is not None:
            rows.append((T.rel(v.grad, g64[k]), T.rel(g32[k], g64[k]), k))
    rows.sort(reverse=True)
    for eh, e32, k in rows[:8]:
        print(f"   {k:55s} hip {eh:.2e}  o32 {e32:.2e}  ratio {eh / max(e32, 1e-12):.1f}")
    groups = {}
    for eh, e32, k in rows:
        top = k.split(".")[0]
        groups.setdefault(top, []).append(eh)
    print("   max per module:", {k: f"{max(v):.1e}" for k, v in groups.items()})


def view5_loss_isolation():
    """view5 golden step: the HIP photometric loss on the HIP net's own outputs
    vs the fp64 oracle loss on the same tensors (isolates the loss kernel), and
    the whole step with the smoothness term off (loss_kw smooth_w=0)."""
    f = T.fx("train_step_it12h_selfsup_n4")
    mind, maxd = fval(f["min_depth"]), fval(f["max_depth"])
    batch = {"rgb": f["image"], "rgb_context": list(f["refs"]), "rgb_original": f["image"],
             "rgb_context_original": list(f["refs"]), "intrinsics": f["K"].clone()}
    model = T._selfsup_model(mind, maxd, "it12h", "it12-h-out")
    out = model(batch)
    invs = torch.stack(out["inv_depths"]).detach()                 # [n,B,1,H,W]
    pv = model.depth_net(batch["rgb"], batch["rgb_context"], batch["intrinsics"])[1].detach()  # [B,N,n,6]
    print("inv range", float(invs.min()), float(invs.max()), "means per pred", invs.mean((1, 2, 3, 4)).tolist())
    import dro_sfm_amd.hip as hip
    for smooth in (0.001, 0.0):
        ig = invs.clone().requires_grad_(True)
        vg = pv.clone().requires_grad_(True)
        loss, metrics, sel = hip.photometric_loss(batch["rgb"], torch.stack(batch["rgb_context"]), ig,
                                                  vg.permute(1, 2, 0, 3), batch["intrinsics"], smooth_w=smooth,
                                                  return_selection=True)
        loss.sum().backward()
        dt = torch.float64
        ic = invs.cpu().to(dt).requires_grad_(True)
        vc = pv.cpu().to(dt).requires_grad_(True)
        N, n = vc.shape[1], vc.shape[2]
        o = O.photometric_decay_loss(batch["rgb"].cpu().to(dt), [c.cpu().to(dt) for c in batch["rgb_context"]],
                                     list(ic), batch["intrinsics"].cpu().to(dt), batch["intrinsics"].cpu().to(dt),
                                     [[vc[:, j, i] for i in range(n)] for j in range(N)], smooth_w=smooth,
                                     forced_selection=sel.cpu().unsqueeze(2))
        o["loss"].sum().backward()
        print(f"loss-only smooth={smooth}: loss rel {abs(float(loss) - float(o['loss'])) / float(o['loss']):.2e} "
              f"inv max-rel {T.rel(ig.grad, ic.grad):.2e} pose max-rel {T.rel(vg.grad, vc.grad):.2e}")


if __name__ == "__main__":
    torch.set_num_threads(16)
    if sys.argv[1:] == ["view5iso"]:
        view5_loss_isolation()
        sys.exit(0)
    for case in sys.argv[1:] or ["it8flip", "view5golden", "scannet_sup"]:
        for cudnn in (True, False):
            run(case, cudnn)
