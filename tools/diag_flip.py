"""Diagnose test_train_step_golden[it8-...-selfsup-True] (flipped it8 step):
per-tensor gradient errors of HIP, the fp32 oracle and the sensitivity probes
against the fp64 oracle, with the HIP PoseHead (hip.pose_mean) and with the
ATen restatement of PoseHead.forward (mean(3).mean(2) * scale [+ pose])."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)

import torch  # noqa: E402

import test_hip_parity as T  # noqa: E402
from dro_sfm_amd.networks.optim import update as U  # noqa: E402


def aten_posehead(self, x_p, pose=None):
    y = U.conv(U.conv(x_p, self.conv1_pose.weight, self.conv1_pose.bias, "relu"),
               self.conv2_pose.weight, self.conv2_pose.bias)
    d = y.mean(3).mean(2) * self._scale
    return d if pose is None else pose + d


def run(flip, label):
    tag, version, kind = "it8", "it8-seq4-inter-out", "selfsup"
    d = T.fx(f"train_step_{tag}")
    dn = T.fx(f"depthposenet_{tag}")
    mind, maxd = T.fval(dn["min_depth"]), T.fval(dn["max_depth"])
    spec = T.load_spec(os.path.join(T.G, f"depthposenet_{tag}_keys.json"))
    N = d["refs"].shape[0]
    batch = {"rgb": d["image"], "rgb_context": list(d["refs"]), "rgb_original": d["image"],
             "rgb_context_original": list(d["refs"]), "intrinsics": d["K"].clone()}
    cpu_batch = {k: (v.cpu().clone() if torch.is_tensor(v) else [t.cpu() for t in v]) for k, v in batch.items()}
    model = T._selfsup_model(mind, maxd, tag, version)
    out = model(batch, flip=flip)
    out["loss"].sum().backward()
    forced = model._photometric_loss.last_selection.cpu().unsqueeze(2)
    args = (spec, version, mind, maxd, cpu_batch, kind, torch.float64, forced, flip)
    _, g64, p64 = T._oracle_grads(*args, want_preds=True)
    _, g32, p32 = T._oracle_grads(*args[:6], torch.float32, forced, flip, want_preds=True)
    gs, sinfo = T._matched_sensitivity(model, out, p64, (args, {}))
    bad, ok, info = T._grad_check(model, g64, g32, gsens=gs)
    print(f"== {label} flip={flip}: ok_global={ok} info={info} sinfo={sinfo}", flush=True)
    grads = dict(model.depth_net.named_parameters())
    rows = []
    for k in g64:
        if k not in grads or grads[k].grad is None:
            continue
        e = T.rel(grads[k].grad, g64[k])
        e32 = T.rel(g32[k], g64[k])
        es = max(T.rel(g[k], g64[k]) for g in gs)
        rows.append((e, k, e32, es))
    rows.sort(reverse=True)
    for e, k, e32, es in rows[:12]:
        print(f"   {k:60s} hip {e:.3e}  o32 {e32:.3e}  sens {es:.3e}", flush=True)
    print(f"   bad: {[(k, round(e, 4), round(t, 4)) for k, e, t in bad]}", flush=True)


if __name__ == "__main__":
    T.hip.__wrapped__() if hasattr(T.hip, "__wrapped__") else None
    from dro_sfm_amd.hip import _lib
    _lib.load()
    run(True, "hip posehead")
    U.PoseHead.forward = aten_posehead
    run(True, "aten posehead")
    run(False, "aten posehead")
