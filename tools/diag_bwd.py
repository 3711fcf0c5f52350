"""Backward error localisation: grads at the loss boundary and at the feature maps."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
import torch
from common import load_fixture, load_spec, params_from_spec
from oracle import dro_oracle as O
from dro_sfm_amd.networks.depth_pose.DepthPoseNet import DepthPoseNet
from dro_sfm_amd.losses.multiview_photometric_loss_mf import MultiViewPhotometricDecayLoss
from dro_sfm_amd.geometry.pose import Pose

tag, version = "it8", "it8-seq4-inter-out"
d = load_fixture(os.path.join(ROOT, f"tests/golden/train_step_{tag}.npz"))
spec = load_spec(os.path.join(ROOT, f"tests/golden/depthposenet_{tag}_keys.json"))
img, refs, K = d["image"], list(d["refs"]), d["K"]


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max())


# fp64 oracle with intermediate grads
dt = torch.float64
p = {k: (v.to(dt) if v.is_floating_point() else v) for k, v in params_from_spec(spec).items()}
invs64, pose64 = O.depth_pose_net(p, version, 0.5, 80.0, img.to(dt), [r.to(dt) for r in refs], K.to(dt), True)
invs64 = [i.detach().requires_grad_(True) for i in invs64]
pose64 = pose64.detach().requires_grad_(True)
N, n = pose64.shape[1], pose64.shape[2]
out = O.photometric_decay_loss(img.to(dt), [r.to(dt) for r in refs], invs64, K.to(dt), K.to(dt),
                               [[pose64[:, j, i] for i in range(n)] for j in range(N)])
out["loss"].sum().backward()
# GPU loss on the same (fp64-rounded-to-fp32) network outputs
inv32 = [i.detach().float().cuda().requires_grad_(True) for i in invs64]
pose32 = pose64.detach().float().cuda().requires_grad_(True)
loss_fn = MultiViewPhotometricDecayLoss(ssim_loss_weight=0.85, smooth_loss_weight=0.001, photometric_reduce_op="min",
                                        clip_loss=0.0, automask_loss=True)
res = loss_fn(img.cuda(), [r.cuda() for r in refs], inv32, K.cuda(), K.cuda(),
              [[Pose.from_vec(pose32[:, j, i], "euler") for i in range(n)] for j in range(N)])
res["loss"].sum().backward()
print("loss rel", rel(res["loss"], out["loss"]))
for i in range(n):
    print(f"  dL/dinv[{i}] rel {rel(inv32[i].grad, invs64[i].grad):.2e}   dL/dpose[:,:,{i}] rel {rel(pose32.grad[:, :, i], pose64.grad[:, :, i]):.2e}")
# oracle fp32 for the same boundary
inv_o = [i.detach().float().requires_grad_(True) for i in invs64]
pose_o = pose64.detach().float().requires_grad_(True)
o32 = O.photometric_decay_loss(img, refs, inv_o, K, K, [[pose_o[:, j, i] for i in range(n)] for j in range(N)])
o32["loss"].sum().backward()
for i in range(n):
    print(f"  oracle32 dL/dinv[{i}] rel {rel(inv_o[i].grad, invs64[i].grad):.2e}   dpose rel {rel(pose_o.grad[:, :, i], pose64.grad[:, :, i]):.2e}")
