"""Depth encodings (dro_sfm/utils/depth.py:102-144, networks/layers/resnet/layers.py:11-20).

Written with torch.where instead of the reference's boolean index_put so
they never synchronise with the host (graph-capturable).
"""
import math

import torch


def inv2depth(inv_depth):
    if isinstance(inv_depth, (list, tuple)):
        return [inv2depth(x) for x in inv_depth]
    d = 1.0 / inv_depth.clamp(min=1e-6)
    return torch.where(inv_depth <= 0.0, torch.zeros_like(d), d)


def depth2inv(depth):
    if isinstance(depth, (list, tuple)):
        return [depth2inv(x) for x in depth]
    i = 1.0 / depth.clamp(min=1e-6)
    return torch.where(depth <= 0.0, torch.zeros_like(i), i)


def disp_to_depth(disp, min_depth, max_depth):
    lo, hi = 1.0 / max_depth, 1.0 / min_depth
    scaled = lo + (hi - lo) * disp
    return scaled, 1.0 / scaled


def compute_depth_metrics(config, gt, pred, use_gt_scale=True):
    """compute_depth_metrics (dro_sfm/utils/depth.py:259-343 of the reference),
    same signature and return value: a tensor [9] of abs_rel, sq_rel, rmse,
    rmse_log, a1, a2, a3, SILog, iabs_diff averaged over the batch.  `config`
    needs .crop ('garg', 'eigen_nyu' or other), .min_depth and .max_depth.
    Computed by the HIP metrics kernels (csrc/metrics.hip); GPU tensors only."""
    from .. import hip
    return hip.depth_metrics(gt, pred, config.min_depth, config.max_depth, crop=config.crop,
                             use_gt_scale=use_gt_scale).type_as(gt)


def _first_ref_poses(gt_pose, B):
    """The per-image transform the reference's loop pairs with image b
    (`zip(pred, gt, gt_pose)`, utils/depth.py:353): a [B,N,4,4] tensor gives
    image b its first reference; a list of N [B,4,4] tensors (the collated
    batch['pose_context']) gives image b element 0 of reference b, and images
    b >= N are not evaluated (they still count in the batch mean)."""
    if torch.is_tensor(gt_pose):
        return gt_pose, B
    n = min(B, len(gt_pose))
    return torch.stack([gt_pose[b][0] for b in range(n)]).unsqueeze(1), n


def compute_depth_metrics_demon(config, gt, gt_pose, pred, use_gt_scale=True):
    """compute_depth_metrics_demon (dro_sfm/utils/depth.py:343-398 of the
    reference), same signature and return value: tensor [9] of abs_rel, sq_rel,
    rmse, rmse_log, a1, a2, a3, SILog, iabs_diff.  `config` needs .min_depth
    and .max_depth.  HIP metrics kernels (csrc/metrics.hip); GPU tensors only."""
    from .. import hip
    B = gt.shape[0]
    poses, n = _first_ref_poses(gt_pose, B)
    out = hip.depth_metrics_demon(gt[:n], poses.to(gt.device), pred[:n], config.min_depth, config.max_depth,
                                  use_gt_scale=use_gt_scale)
    if n != B:
        out = out * (n / B)
    return out.type_as(gt)


def compute_pose_metrics(config, gt, pred):
    """compute_pose_metrics (dro_sfm/utils/depth.py:400-421 of the reference):
    [rotation error (deg), translation direction error (deg), scale-fitted
    translation error (cm)] of the first reference's pose (gt[0], pred[0] a
    Pose or a [1,4,4] tensor).  The reference takes the pair to the host and
    computes in numpy float32; here the same formulas run in float64 on the
    pair's device (no host synchronisation), returned as float32."""
    pm = pred[0].mat if hasattr(pred[0], "mat") else pred[0]
    pr = pm.detach().squeeze().double()
    g = gt[0].detach().squeeze().to(pr.device).double()
    R1, t1, R2, t2 = g[:3, :3], g[:3, 3], pr[:3, :3], pr[:3, 3]
    cos_r = torch.clamp_max(((R1 * R2).sum() - 1.0) / 2.0, 1.0)          # trace(R1^T R2)
    rdeg = torch.arccos(cos_r) * (180.0 / math.pi)
    cos_t = (t1 * t2).sum() / (t1.norm() * t2.norm())
    tdeg = torch.arccos(cos_t) * (180.0 / math.pi)
    a = (t1 * t2).sum() / (t2 * t2).sum()
    tcm = 100.0 * torch.sqrt(((t1 - a * t2) ** 2).sum())
    return torch.stack([rdeg, tdeg, tcm]).float()
