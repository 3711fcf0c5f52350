"""Localise the view5 (N=4, B=1, it12-h self-sup) gradient deviation:
(a) warp_cost at that shape vs the fp64 oracle (depth mean over 4 refs and
per-ref pose cost), (b) the DepthPoseNet forward outputs vs the fp64 oracle,
(c) gradients of a random linear functional of the net outputs (no loss)
vs the fp64 oracle, per module."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

import test_hip_parity as T  # noqa: E402
from common import fval, load_spec, params_from_spec  # noqa: E402
from oracle import dro_oracle as O  # noqa: E402
import dro_sfm_amd.hip as hip  # noqa: E402

torch.set_num_threads(16)
f = T.fx("train_step_it12h_selfsup_n4")
mind, maxd = fval(f["min_depth"]), fval(f["max_depth"])
img, refs, K = f["image"], list(f["refs"]), f["K"]
B, N, H, W = img.shape[0], len(refs), img.shape[2], img.shape[3]

# (a) warp cost at the feature shape
g = torch.Generator().manual_seed(1)
for (B_, N_, C, h, w) in ((1, 4, 128, 8, 12), (1, 4, 128, 12, 20), (2, 2, 128, 8, 12), (1, 2, 128, 8, 12)):
    Kc = K[:1].repeat(B_, 1, 1).cpu()
    fmap, frefs = torch.randn(B_, C, h, w, generator=g), torch.randn(N_, B_, C, h, w, generator=g)
    disp = torch.rand(B_, 1, h, w, generator=g)
    poses = torch.cat([0.05 * torch.randn(N_, B_, 3, generator=g), 0.02 * torch.randn(N_, B_, 3, generator=g)], 2)
    G = torch.randn(B_, C, h, w, generator=g)
    dt = torch.float64
    dc, fc, rc = (t.to(dt).requires_grad_(True) for t in (disp, fmap, frefs))
    inv = O.disp_to_depth(dc, mind, maxd)
    cm = O.depth_cost_calc(inv, fc, list(rc), list(poses.to(dt)), Kc.to(dt), Kc.to(dt), 1 / 8)
    (cm * G.to(dt)).sum().backward()
    dg, fg, rg = (t.cuda().requires_grad_(True) for t in (disp, fmap, frefs))
    hm = hip.warp_cost(fg, rg, dg, poses.cuda(), Kc.cuda(), depth_mode=hip.DEPTH_DISP, min_depth=mind,
                       max_depth=maxd, reduce_mean=True)
    (hm * G.cuda()).sum().backward()
    print(f"warp_cost B{B_} N{N_} {h}x{w}: cost {T.rel(hm, cm):.2e} g_disp {T.rel(dg.grad, dc.grad):.2e} "
          f"g_fmap {T.rel(fg.grad, fc.grad):.2e} g_fref {T.rel(rg.grad, rc.grad):.2e}")

# (b)/(c) the net alone
spec = load_spec(os.path.join(T.G, "depthposenet_it12h_keys.json"))
net = T._load_net("it12h", "it12-h-out", mind, maxd).train()
invs, poses = net(img, refs, K.clone())
gi = torch.randn(torch.stack(invs).shape, generator=torch.Generator().manual_seed(2)).cuda()
gp = torch.randn(poses.shape, generator=torch.Generator().manual_seed(3)).cuda()
((torch.stack(invs) * gi).sum() + (poses * gp).sum()).backward()
dt = torch.float64
p = {k: (v.to(dt).requires_grad_(True) if v.is_floating_point() and "running" not in k else
         (v.to(dt) if v.is_floating_point() else v)) for k, v in params_from_spec(spec).items()}
oi, op = O.depth_pose_net(p, "it12-h-out", mind, maxd, img.cpu().to(dt), [r.cpu().to(dt) for r in refs],
                          K.cpu().to(dt), training=True)
print(f"net fwd: inv {T.rel(torch.stack(invs), torch.stack(oi)):.2e} poses {T.rel(poses, op):.2e}")
((torch.stack(oi) * gi.cpu().to(dt)).sum() + (op * gp.cpu().to(dt)).sum()).backward()
rows = sorted(((T.rel(v.grad, p[k].grad), k) for k, v in net.named_parameters()
               if v.grad is not None and p[k].grad is not None), reverse=True)
groups = {}
for e, k in rows:
    groups.setdefault(k.split(".")[0], []).append(e)
print("net grads max per module:", {k: f"{max(v):.1e}" for k, v in groups.items()})
print("worst:", [(k, f"{e:.1e}") for e, k in rows[:6]])
