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


def _angle_tol(deg, rel=1e-4):
    """|error| allowed on an arccos angle: the reference computes cos in
    numpy float32 (a few ulp of cos), and d(arccos)/d(cos) = -1/sin."""
    import math
    s = max(math.sin(math.radians(abs(deg))), 1e-4)
    return math.degrees(4e-7 / s) + rel * abs(deg)


@pytest.mark.gpu
@pytest.mark.parametrize("scaled", [True, False])
def test_depth_metrics_demon_golden(scaled):
    """compute_depth_metrics_demon (utils/depth.py:343-398; configs[4]'s ScanNet
    evaluation) against the reference's own outputs: gt normalised by the first
    reference's gt translation, median scaling, no clamps; 1e-4."""
    from dro_sfm_amd.utils.depth import compute_depth_metrics_demon
    d = load_fixture(os.path.join(G, "metrics_demon.npz"))
    cfg = SimpleNamespace(min_depth=fval(d["min_depth"]), max_depth=fval(d["max_depth"]))
    out = compute_depth_metrics_demon(cfg, d["gt"].cuda(), d["gt_pose"].cuda(), d["pred"].cuda(),
                                      use_gt_scale=scaled)
    want = d["metrics_scaled" if scaled else "metrics_unscaled"]
    assert out.is_cuda and out.shape == (9,)
    assert close(out, want), (out.cpu(), want)


@pytest.mark.gpu
def test_depth_metrics_demon_scannet_size_vs_oracle():
    """ScanNet evaluation size (480x640 dense gt, 240x320 prediction, B=4, N=2
    gt poses) against the oracle restatement; 1e-4."""
    import dro_sfm_amd.hip as hip
    B, H, W, h, w = 4, 480, 640, 240, 320
    gt, g = sparse_gt(B, H, W, 0.2, 10.0, 0.9, 12)
    pred = torch.nn.functional.interpolate(gt.clamp(min=0.7), size=(h, w), mode="area")
    pred = pred * (1.0 + 0.2 * torch.randn(B, 1, h, w, generator=g)).abs() + 0.05
    vec = torch.cat([0.3 * torch.randn(B * 2, 3, generator=g), 0.05 * torch.randn(B * 2, 3, generator=g)], 1)
    pose = O.vec_to_transform(vec).view(B, 2, 4, 4)
    for scaled in (True, False):
        want = O.depth_metrics_demon(gt, pose, pred, 0.2, 10.0, scaled)
        out = hip.depth_metrics_demon(gt.cuda(), pose.cuda(), pred.cuda(), 0.2, 10.0, use_gt_scale=scaled)
        assert close(out, want), (scaled, out.cpu(), want)


def test_pose_metrics_golden():
    """compute_pose_metrics (utils/depth.py:400-421) against the reference's
    outputs on six near pose pairs (CPU tensors here; the function runs on the
    pair's device): angles within the float32 conditioning of arccos, the
    translation error at 1e-4."""
    from dro_sfm_amd.utils.depth import compute_pose_metrics
    d = load_fixture(os.path.join(G, "metrics_pose.npz"))
    for k in range(d["gt"].shape[0]):
        out = compute_pose_metrics(None, [d["gt"][k:k + 1]], [d["pred"][k:k + 1]])
        want = d["metrics"][k]
        assert abs(float(out[0] - want[0])) <= _angle_tol(float(want[0])), (k, out, want)
        assert abs(float(out[1] - want[1])) <= _angle_tol(float(want[1])), (k, out, want)
        assert abs(float(out[2] - want[2])) <= 1e-4 * abs(float(want[2])) + 1e-5, (k, out, want)
