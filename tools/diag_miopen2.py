"""Which MIOpen piece loses gradient accuracy?  it12h supervised step, per-param
grad error vs the fp64 oracle, with BN or conv selectively routed off MIOpen."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
import torch, torch.nn as nn, torch.nn.functional as F
from common import load_fixture, load_spec, params_from_spec
from oracle import dro_oracle as O
from dro_sfm_amd.models.SupModelMF import SupModelMF
from dro_sfm_amd.networks.depth_pose.DepthPoseNet import DepthPoseNet

tag, version, kind = "it12h", "it12-h-out", "sup"
d = load_fixture(os.path.join(ROOT, f"tests/golden/train_step_{tag}.npz"))
dn = load_fixture(os.path.join(ROOT, f"tests/golden/depthposenet_{tag}.npz"))
mind, maxd = float(dn["min_depth"]), float(dn["max_depth"])
spec = load_spec(os.path.join(ROOT, f"tests/golden/depthposenet_{tag}_keys.json"))
N = d["refs"].shape[0]
batch = {"rgb": d["image"], "rgb_context": list(d["refs"]), "rgb_original": d["image"],
         "rgb_context_original": list(d["refs"]), "intrinsics": d["K"], "depth": d["gt_depth"],
         "pose_context": [d["gt_poses"][:, j] for j in range(N)]}
p = params_from_spec(spec)
p = {k: (v.double().requires_grad_(True) if v.is_floating_point() and "running" not in k else (v.double() if v.is_floating_point() else v)) for k, v in p.items()}
b64 = {k: (v.double() if torch.is_tensor(v) and v.is_floating_point() else ([t.double() for t in v] if isinstance(v, list) else v)) for k, v in batch.items()}
o = O.train_step_loss(p, version, mind, maxd, b64, kind=kind); o["loss"].sum().backward()
g64 = {k: v.grad for k, v in p.items() if getattr(v, "grad", None) is not None}

orig_bn, orig_conv = nn.BatchNorm2d.forward, nn.Conv2d._conv_forward


def bn_native(self, x):
    with torch.backends.cudnn.flags(enabled=False):
        return orig_bn(self, x)


def conv_native(self, x, w, bias):
    with torch.backends.cudnn.flags(enabled=False):
        return orig_conv(self, x, w, bias)


def run(label, bn_off, conv_off, env=None):
    nn.BatchNorm2d.forward = bn_native if bn_off else orig_bn
    nn.Conv2d._conv_forward = conv_native if conv_off else orig_conv
    torch.backends.cudnn.enabled = True
    net = DepthPoseNet(version=version, min_depth=mind, max_depth=maxd)
    net.load_state_dict(params_from_spec(spec))
    model = SupModelMF(flip_lr_prob=0.0, min_depth=mind, max_depth=maxd)
    model.add_depth_net(net.cuda()); model.train()
    gb = {k: (v.cuda() if torch.is_tensor(v) else [t.cuda() for t in v]) for k, v in batch.items()}
    out = model(gb); out["loss"].sum().backward()
    rows = sorted(((O.rel_err(v.grad.cpu(), g64[k]), k) for k, v in model.depth_net.named_parameters()
                   if k in g64 and v.grad is not None), reverse=True)
    print(label, ["%.2e %s" % r for r in rows[:3]], flush=True)


run("all-miopen   ", False, False)
run("bn-native    ", True, False)
run("conv-native  ", False, True)
run("both-native  ", True, True)
