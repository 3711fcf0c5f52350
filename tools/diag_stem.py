"""The 7x7/s2 stem convolution on the view5 fixture's frames: native (HIP
flattened implicit GEMM) and MIOpen against fp64, with the error measured
where training-mode BatchNorm sees it -- per output channel, max|err| over
that channel's standard deviation (BN divides by it).  usage:
python tools/diag_stem.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import dro_sfm_amd.hip as hip  # noqa: E402
import test_hip_parity as T  # noqa: E402


def main():
    f = T.fx("train_step_it12h_selfsup_n4")
    p = T.params_from_spec(T.load_spec(os.path.join(T.G, "depthposenet_it12h_keys.json")))
    x = torch.cat([f["image"]] + list(f["refs"]), 0).float()
    w = p["fnet.conv1.weight"].cuda().float()
    ref = F.conv2d(x.double(), w.double(), stride=2, padding=3)
    std = ref.std(dim=(0, 2, 3))
    for name, y in (("native", hip.conv2d_strided(x, w, None, 2, 3)),
                    ("miopen", F.conv2d(x, w, stride=2, padding=3))):
        err = (y.double() - ref).abs()
        per = err.amax(dim=(0, 2, 3)) / std
        rel_max = float(err.max() / ref.abs().max())
        worst = torch.argsort(per, descending=True)[:5]
        print(f"{name}: max-rel {rel_max:.2e}; max|err|/std per channel: median {float(per.median()):.2e} "
              f"worst " + ", ".join(f"c{int(c)} {float(per[c]):.2e} (std {float(std[c]):.2e})" for c in worst))
        print(f"   mean signed error (bias) over all outputs: {float((y.double() - ref).mean()):.3e}, "
              f"channel std range {float(std.min()):.2e}..{float(std.max()):.2e}")


if __name__ == "__main__":
    main()
