"""The fp32 floor of the train-step gradients (tests/test_hip_parity.py's
GRAD_* bounds): the reference algorithm (oracle/dro_oracle.py) evaluated in
fp32 against itself in fp64, on the same branch -- the fp64 run records its
bilinear cells and the fp32 run takes them.  CPU only (test infrastructure:
reads the golden fixtures and the oracle).

usage: python tools/grad_floor.py it8 it8-seq4-inter-out selfsup [flip]
       python tools/grad_floor.py kitti          (metric config 192x640, B=2, N=2)
       python tools/grad_floor.py view5          (ScanNet view5 fixture, it12-h, N=4)
"""
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]
import torch  # noqa: E402

import test_hip_parity as T  # noqa: E402
from oracle import dro_oracle as O  # noqa: E402

T.DEV = "cpu"


def golden_case(tag, version, kind):
    d, dn = T.fx(f"train_step_{tag}"), T.fx(f"depthposenet_{tag}")
    N = d["refs"].shape[0]
    batch = {"rgb": d["image"], "rgb_context": list(d["refs"]), "rgb_original": d["image"],
             "rgb_context_original": list(d["refs"]), "intrinsics": d["K"].clone(),
             "depth": d["gt_depth"], "pose_context": [d["gt_poses"][:, j] for j in range(N)]}
    return tag, version, kind, T.fval(dn["min_depth"]), T.fval(dn["max_depth"]), batch


def view5_case():
    d = T.fx("train_step_it12h_selfsup_n4")
    batch = {"rgb": d["image"], "rgb_context": list(d["refs"]), "rgb_original": d["image"],
             "rgb_context_original": list(d["refs"]), "intrinsics": d["K"].clone()}
    return "it12h", "it12-h-out", "selfsup", T.fval(d["min_depth"]), T.fval(d["max_depth"]), batch


def kitti_case():
    B, N, H, W = 2, 2, 192, 640
    img = T.smooth_images(B, H, W, 51, detail=0.3)
    refs = [torch.roll(img, 3 * (j + 1), 3) * 0.9 + 0.1 * T.smooth_images(B, H, W, 52 + j, detail=0.3)
            for j in range(N)]
    batch = {"rgb": img, "rgb_context": refs, "rgb_original": img, "rgb_context_original": refs,
             "intrinsics": T.kitti_K(B)}
    return "it8", "it8-seq4-inter-out", "selfsup", 0.5, 80.0, batch


def run(spec, version, kind, mind, maxd, batch, dt, book, flip):
    p = T.params_from_spec(spec)
    p = {k: (v.to(dt).requires_grad_(True) if v.is_floating_point() and "running" not in k
             else (v.to(dt) if v.is_floating_point() else v)) for k, v in p.items()}
    b = {k: (v.clone().to(dt) if torch.is_tensor(v) and v.is_floating_point() else
             ([t.to(dt) for t in v] if isinstance(v, list) else v)) for k, v in batch.items()}
    out = O.train_step_loss(p, version, mind, maxd, b, kind=kind, flip=flip, cells=book)
    out["loss"].sum().backward()
    return out, {k: v.grad for k, v in p.items() if getattr(v, "grad", None) is not None}


def main():
    a = sys.argv[1:]
    tag, version, kind, mind, maxd, batch = (kitti_case() if a[0] == "kitti" else view5_case() if a[0] == "view5"
                                             else golden_case(*a[:3]))
    flip = "flip" in a
    spec = T.load_spec(os.path.join(T.G, f"depthposenet_{tag}_keys.json"))
    batch = {k: (v.cpu().clone() if torch.is_tensor(v) else [t.cpu() for t in v]) for k, v in batch.items()}
    rec = O.Cells(record=True)
    o64, g64 = run(spec, version, kind, mind, maxd, batch, torch.float64, rec, flip)
    o32, g32 = run(spec, version, kind, mind, maxd, batch, torch.float32, O.Cells(forced=rec.recorded), flip)
    per, l2 = T._grad_check_vs(g32, g64)
    worst = sorted(per.items(), key=lambda kv: -kv[1])[:5]
    print(f"{' '.join(a)}: loss rel {T.rel(o32['loss'], o64['loss']):.2e}  gradient L2 {l2:.3e}  worst "
          + ", ".join(f"{k} {e:.2e}" for k, e in worst))


if __name__ == "__main__":
    main()
