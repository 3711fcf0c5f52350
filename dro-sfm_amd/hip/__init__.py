"""Autograd-aware wrappers of the gfx950 kernels (libdro_amd.so).

Every op launches on torch's current HIP stream, allocates only through the
PyTorch caching allocator and never synchronises, so whole training steps can
be captured into a hipGraph.
"""
from .ops import (DEPTH_DISP, DEPTH_INV, DEPTH_METRIC, POSE_EULER, POSE_MATRIX,
                  batchnorm_act, bilinear_upsample2x, grad_sink, maxpool3x3s2, depth_metrics, depth_metrics_demon,
                  pose_mean, convex_upsample, convex_upsample_many, stacked_view, photometric_loss, plane_sweep_cost,
                  record_bilinear_cells, supervised_loss, view_synthesis, warp_cost)
from .conv import cached_cat, conv2d, conv2d_strided, sepconvgru_half, weight_grad_scope

__all__ = ["conv2d", "conv2d_strided", "sepconvgru_half", "weight_grad_scope", "cached_cat", "warp_cost",
           "view_synthesis", "plane_sweep_cost", "photometric_loss", "supervised_loss",
           "convex_upsample", "convex_upsample_many", "stacked_view",
           "bilinear_upsample2x", "maxpool3x3s2", "depth_metrics", "depth_metrics_demon", "pose_mean", "batchnorm_act",
           "grad_sink", "record_bilinear_cells",
           "POSE_EULER", "POSE_MATRIX", "DEPTH_METRIC", "DEPTH_INV", "DEPTH_DISP"]
