"""it12h supervised train step: per-param grad error vs fp64 oracle, MIOpen on/off."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
import torch
from common import load_fixture, load_spec, params_from_spec
from oracle import dro_oracle as O
from dro_sfm_amd.models.SupModelMF import SupModelMF
from dro_sfm_amd.models.SelfSupModelMF import SelfSupModelMF
from dro_sfm_amd.networks.depth_pose.DepthPoseNet import DepthPoseNet

for tag, version, kind in (("it12h", "it12-h-out", "sup"), ("it8", "it8-seq4-inter-out", "selfsup")):
    d = load_fixture(os.path.join(ROOT, f"tests/golden/train_step_{tag}.npz"))
    dn = load_fixture(os.path.join(ROOT, f"tests/golden/depthposenet_{tag}.npz"))
    mind, maxd = float(dn["min_depth"]), float(dn["max_depth"])
    spec = load_spec(os.path.join(ROOT, f"tests/golden/depthposenet_{tag}_keys.json"))
    N = d["refs"].shape[0]
    batch = {"rgb": d["image"], "rgb_context": list(d["refs"]), "rgb_original": d["image"],
             "rgb_context_original": list(d["refs"]), "intrinsics": d["K"], "depth": d["gt_depth"],
             "pose_context": [d["gt_poses"][:, j] for j in range(N)]}
    for miopen in (True, False):
        torch.backends.cudnn.enabled = miopen
        net = DepthPoseNet(version=version, min_depth=mind, max_depth=maxd)
        net.load_state_dict(params_from_spec(spec))
        if kind == "sup":
            model = SupModelMF(flip_lr_prob=0.0, min_depth=mind, max_depth=maxd)
        else:
            model = SelfSupModelMF(flip_lr_prob=0.0, automask_loss=True, photometric_reduce_op="min", clip_loss=0.0,
                                   smooth_loss_weight=0.001, min_depth=mind, max_depth=maxd)
            model._photometric_loss.keep_selection = True
        model.add_depth_net(net.cuda()); model.train()
        gb = {k: (v.cuda() if torch.is_tensor(v) else [t.cuda() for t in v]) for k, v in batch.items()}
        out = model(gb); out["loss"].sum().backward()
        forced = model._photometric_loss.last_selection.cpu() if kind == "selfsup" else None
        res = {}
        for dt in (torch.float32, torch.float64):
            p = params_from_spec(spec)
            p = {k: (v.to(dt).requires_grad_(True) if v.is_floating_point() and "running" not in k else (v.to(dt) if v.is_floating_point() else v)) for k, v in p.items()}
            b = {k: (v.to(dt) if torch.is_tensor(v) and v.is_floating_point() else ([t.to(dt) for t in v] if isinstance(v, list) else v)) for k, v in batch.items()}
            o = O.train_step_loss(p, version, mind, maxd, b, kind=kind, forced_selection=forced)
            o["loss"].sum().backward()
            res[dt] = {k: v.grad for k, v in p.items() if getattr(v, "grad", None) is not None}
        rows = []
        for k, v in model.depth_net.named_parameters():
            if k in res[torch.float64] and v.grad is not None:
                rows.append((O.rel_err(v.grad.cpu(), res[torch.float64][k]), O.rel_err(res[torch.float32][k], res[torch.float64][k]), k))
        rows.sort(reverse=True)
        print(tag, "miopen", miopen, "loss gpu", float(out["loss"].detach()))
        for r in rows[:6]:
            print("   gpu %.2e  cpu32 %.2e  %s" % r)
        by = sorted(rows, key=lambda r: -r[1])[:3]
        print("   (worst cpu32:", ["%.2e %s" % (r[1], r[2]) for r in by], ")", flush=True)
