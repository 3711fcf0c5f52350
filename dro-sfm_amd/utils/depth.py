"""Depth encodings (dro_sfm/utils/depth.py:102-144, networks/layers/resnet/layers.py:11-20).

Written with torch.where instead of the reference's boolean index_put so
they never synchronise with the host (graph-capturable).
"""
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
