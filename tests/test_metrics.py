"""Depth evaluation metrics on the GPU (hip.depth_metrics, csrc/metrics.hip)
against the reference's compute_depth_metrics (dro_sfm/utils/depth.py:259-343):
the golden outputs of the reference itself, and the CPU oracle at KITTI and
NYU ground-truth sizes.  Tolerance: 1e-4 relative per metric (the kernels sum
in fp64 where the reference's torch.mean sums in fp32)."""
import os
from types import SimpleNamespace

import pytest
import torch

from common import fval, load_fixture
from oracle import dro_oracle as O

G = os.path.join(os.path.dirname(__file__), "golden")
TOL = 1e-4


def close(a, b, tol=TOL):
    a, b = a.double().cpu(), b.double().cpu()
    return bool(((a - b).abs() <= tol * b.abs() + 1e-7).all())


def sparse_gt(B, H, W, lo, hi, frac, seed):
    g = torch.Generator().manual_seed(seed)
    gt = torch.zeros(B, 1, H, W)
    keep = torch.rand(B, 1, H, W, generator=g) < frac
    gt[keep] = (lo + 0.5 + (hi - lo - 0.5) * torch.rand(B, 1, H, W, generator=g))[keep]
    return gt, g


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["metrics_garg", "metrics_nocrop"])
@pytest.mark.parametrize("scaled", [True, False])
def test_depth_metrics_golden(name, scaled):
    from dro_sfm_amd.utils.depth import compute_depth_metrics
    d = load_fixture(os.path.join(G, name + ".npz"))
    cfg = SimpleNamespace(crop={0: "", 1: "garg", 2: "eigen_nyu"}[int(d["crop"])],
                          min_depth=fval(d["min_depth"]), max_depth=fval(d["max_depth"]))
    out = compute_depth_metrics(cfg, d["gt"].cuda(), d["pred"].cuda(), use_gt_scale=scaled)
    want = d["metrics_scaled" if scaled else "metrics_unscaled"]
    assert out.is_cuda and out.shape == (9,)
    assert close(out, want), (out.cpu(), want)


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["kitti_garg", "nyu_eigen", "same_res"])
def test_depth_metrics_vs_oracle(case):
    import dro_sfm_amd.hip as hip
    if case == "kitti_garg":        # KITTI eval: 375x1242 LiDAR gt, 192x640 prediction
        (B, H, W), (h, w), lo, hi, crop, frac = (4, 375, 1242), (192, 640), 1e-3, 80.0, "garg", 0.05
    elif case == "nyu_eigen":       # NYU/ScanNet-style dense gt with the eigen crop
        (B, H, W), (h, w), lo, hi, crop, frac = (2, 480, 640), (240, 320), 0.2, 10.0, "eigen_nyu", 0.9
    else:
        (B, H, W), (h, w), lo, hi, crop, frac = (3, 240, 320), (240, 320), 0.2, 10.0, "", 0.9
    gt, g = sparse_gt(B, H, W, lo, hi, frac, 5)
    pred = gt.clone()
    if (h, w) != (H, W):
        pred = torch.nn.functional.interpolate(gt.clamp(min=lo + 0.5), size=(h, w), mode="area")
    pred = pred.clamp(min=lo + 0.5) * (1.0 + 0.2 * torch.randn(B, 1, h, w, generator=g)).abs()
    for scaled in (True, False):
        ref = O.depth_metrics(gt, pred, lo, hi, crop, scaled)
        out = hip.depth_metrics(gt.cuda(), pred.cuda(), lo, hi, crop=crop, use_gt_scale=scaled)
        assert close(out, ref), (case, scaled, out.cpu(), ref)
        again = hip.depth_metrics(gt.cuda(), pred.cuda(), lo, hi, crop=crop, use_gt_scale=scaled)
        assert torch.equal(out, again)                  # fixed-order fp64 sums: deterministic


@pytest.mark.gpu
def test_depth_metrics_no_valid_pixels():
    import dro_sfm_amd.hip as hip
    gt = torch.zeros(2, 1, 16, 24).cuda()
    pred = torch.ones(2, 1, 8, 12).cuda()
    out = hip.depth_metrics(gt, pred, 0.1, 80.0, crop="garg")
    assert torch.equal(out.cpu(), torch.zeros(9))


def test_depth_metrics_rejects_cpu():
    import dro_sfm_amd.hip as hip
    with pytest.raises(RuntimeError):
        hip.depth_metrics(torch.ones(1, 1, 4, 4), torch.ones(1, 1, 4, 4), 0.1, 80.0)
