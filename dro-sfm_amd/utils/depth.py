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
