"""ctypes binding of libdro_amd.so (C ABI: include/dro_amd.h).

The library is loaded AFTER torch so that its NEEDED libamdhip64.so.7 resolves
to the HIP runtime torch already mapped (one runtime, one device context).
There is deliberately no fallback: if the library is missing, or the tensors
are not on a ROCm device, the ops raise.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# DRO_LIB_PATH: an alternative build of the same library (A/B measurements)
LIB_PATH = os.environ.get("DRO_LIB_PATH") or os.path.normpath(os.path.join(_HERE, "..", "libdro_amd.so"))

_c_float_p = ctypes.c_void_p
_lib = None


def _sig(fn, *argtypes, restype=ctypes.c_int):
    fn.argtypes = list(argtypes)
    fn.restype = restype


def load():
    """Load and type the library once; raise loudly if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"dro_sfm_amd: native library not found at {LIB_PATH}; build it with "
            "`make -C dro-sfm_amd/csrc` (or __graft_entry__.build()).  There is no CPU fallback.")
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    P, I, F, S, Z = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_void_p, ctypes.c_size_t
    LL = ctypes.c_longlong
    _sig(lib.dro_last_error, restype=ctypes.c_char_p)
    _sig(lib.dro_abi_version)
    _sig(lib.dro_timestamp, P, I, S)
    _sig(lib.dro_wall_clock_hz, P)
    _sig(lib.dro_warp_cost_forward, P, P, P, I, F, F, P, P, F, P, I, I, I, I, I, I, I, I, P, S)
    _sig(lib.dro_warp_cost_workspace_bytes, I, I, I, I, restype=Z)
    _sig(lib.dro_warp_cost_backward, P, P, P, I, F, F, P, P, F, P, I, I, I, I, I, I, I, I,
         P, P, P, P, P, I, P, P, S)
    _sig(lib.dro_view_synthesis_forward, P, P, I, F, F, P, P, F, P, I, I, I, I, I, I, P, S)
    _sig(lib.dro_view_synthesis_backward, P, P, I, F, F, P, P, F, P, I, I, I, I, I, I, P, P, P, P, P, P, S)
    _sig(lib.dro_plane_sweep_forward, P, P, P, I, F, F, P, P, F, P, I, I, I, I, I, P, S)
    _sig(lib.dro_photometric_workspace_bytes, I, I, I, I, I, F, restype=Z)
    _sig(lib.dro_photometric_forward, P, P, P, P, P, P, I, I, I, I, I, I, F, F, F, F, I, I, F,
         P, P, S)
    _sig(lib.dro_photometric_clip_offset, I, I, I, I, I, I, restype=Z)
    _sig(lib.dro_photometric_backward, P, P, P, P, P, P, I, I, I, I, I, I, F, F, F, F, I, I, F,
         P, P, P, P, P, P, S)
    _sig(lib.dro_supervised_workspace_bytes, I, I, I, I, I, restype=Z)
    _sig(lib.dro_supervised_forward, P, P, P, P, P, P, I, I, I, I, I, I, F, F, P, P, S)
    _sig(lib.dro_supervised_backward, P, P, P, P, P, P, I, I, I, I, I, I, F, F, P, P, P, P, S)
    _sig(lib.dro_convex_upsample_forward, P, P, I, I, I, I, F, F, P, S)
    _sig(lib.dro_convex_upsample_backward, P, P, P, I, I, I, I, F, P, P, S)
    _sig(lib.dro_convex_upsample_many_forward, P, P, I, I, I, I, I, F, F, P, S)
    _sig(lib.dro_convex_upsample_many_workspace_bytes, I, I, I, I, restype=Z)
    _sig(lib.dro_convex_upsample_many_backward, P, P, P, I, I, I, I, I, F, P, P, P, Z, S)
    _sig(lib.dro_bilinear_upsample2x_forward, P, ctypes.c_longlong, I, I, P, S)
    _sig(lib.dro_bilinear_upsample2x_backward, P, ctypes.c_longlong, I, I, P, S)
    _sig(lib.dro_maxpool3x3s2_forward, P, ctypes.c_longlong, I, I, P, P, S)
    _sig(lib.dro_maxpool3x3s2_backward, P, P, ctypes.c_longlong, I, I, P, S)
    _sig(lib.dro_depth_metrics_blocks, I, I)
    _sig(lib.dro_depth_metrics_workspace_bytes, I, restype=Z)
    _sig(lib.dro_depth_metrics_prepare, P, P, I, I, I, I, I, F, F, I, I, I, I, P, P, P, S)
    _sig(lib.dro_depth_metrics_reduce, P, P, P, I, I, I, F, F, I, I, I, I, P, P, S)
    _sig(lib.dro_depth_metrics_median_workspace_bytes, I, restype=Z)
    _sig(lib.dro_depth_metrics_median, P, P, I, I, I, P, P, S)
    _sig(lib.dro_pose_mean_forward, P, P, P, I, I, I, F, S)
    _sig(lib.dro_pose_mean_backward, P, P, I, I, I, F, S)
    _sig(lib.dro_conv2d_strided_workspace_bytes, I, I, I, I, I, I, I, I, I, restype=Z)
    _sig(lib.dro_conv2d_strided_forward, P, P, P, I, I, I, I, I, I, I, I, I, I, P, P, Z, S)
    _sig(lib.dro_conv2d_strided_backward, P, P, P, I, I, I, I, I, I, I, I, I, P, I, P, P, I, P, Z, S)
    _sig(lib.dro_depth_metrics_demon_prepare, P, P, P, LL, I, I, I, I, I, F, F, P, P, P, S)
    _sig(lib.dro_depth_metrics_demon_reduce, P, P, P, P, LL, I, I, I, F, F, P, P, S)
    _sig(lib.dro_resize_rgb8_to_tensor, P, I, I, I, I, I, P, P, I, P, P, I, P, P, S)
    _sig(lib.dro_color_jitter_rgb8, P, I, I, I, P, P, S)
    _sig(lib.dro_resize_rgb8, P, I, I, I, I, I, P, P, I, P, P, I, P, P, S)
    _sig(lib.dro_rgb8_to_tensor, P, I, I, I, P, S)
    _sig(lib.dro_png_filtered_bytes, I, I, I, restype=Z)
    _sig(lib.dro_png_decode, P, P, I, I, I, I, P, P, P, S)
    _sig(lib.dro_batchnorm_workspace_bytes, I, I, I, restype=Z)
    _sig(lib.dro_batchnorm_relu_forward, P, P, P, P, I, I, I, I, F, F, P, P, P, P, P, P, P, Z, S)
    _sig(lib.dro_batchnorm_relu_backward, P, P, P, P, P, P, I, I, I, I, P, P, P, P, P, Z, S)
    _sig(lib.dro_conv2d_workspace_bytes, I, I, I, I, I, I, I, restype=Z)
    _sig(lib.dro_conv2d_plan, I, I, I, I, I, I, I, P)
    _sig(lib.dro_debug_conv_stamps, P)
    _sig(lib.dro_conv_log, I)
    _sig(lib.dro_conv_log_read, ctypes.c_char_p, ctypes.c_longlong, restype=ctypes.c_longlong)
    _sig(lib.dro_weight_split_bytes, I, I, I, I, I, restype=Z)
    _sig(lib.dro_weight_split, P, I, I, I, I, P, P, S)
    _sig(lib.dro_conv2d_forward, P, I, P, P, I, I, I, I, I, I, I, F, P, I, I, P, P, Z, S)
    _sig(lib.dro_convgru_gates_forward, P, I, P, P, I, I, I, I, I, I, P, P, P, P, Z, S)
    _sig(lib.dro_convgru_blend_forward, P, I, P, P, I, I, I, I, I, I, P, P, P, P, I, I, P, P, Z, S)
    _sig(lib.dro_conv2d_backward, P, I, P, I, I, I, I, I, I, I, F, P, P, P, P, P, P, P, P, I, P, P, Z, S)
    _sig(lib.dro_conv2d_weight_grad_multi_workspace_bytes, I, I, I, I, I, I, I, I, restype=Z)
    _sig(lib.dro_conv2d_weight_grad_multi, P, I, I, I, I, I, I, I, I, I, F, P, P, I, P, Z, S)
    _sig(lib.dro_adam_step, P, P, P, P, ctypes.c_longlong, P, P, S)
    _sig(lib.dro_gru_backward_elem, I, I, I, I, I, P, P, P, P, P, P, P, P, S)
    _sig(lib.dro_convgru_candidate_backward, P, I, P, I, I, I, I, I, I, P, P, P, P, P, P, P, P, P, P, Z, S)
    _sig(lib.dro_convgru_gates_backward, P, I, P, I, I, I, I, I, I, P, P, P, P, P, P, P, P, P, P, P, I, P, Z, S)
    _sig(lib.dro_bn_state_bytes, I, I, I, I, restype=Z)
    _sig(lib.dro_bn_apply, P, P, I, I, I, I, I, P, P, S)
    _sig(lib.dro_bn_backward_apply, P, P, I, I, I, I, P, P, S)
    _sig(lib.dro_conv2d_bn_forward, P, I, I, I, I, P, I, P, P, P, P, P, P, P, Z, S)
    _sig(lib.dro_conv2d_bn_backward_data, P, I, I, I, I, I, P, P, P, P, P, P, P, I, P, Z, S)
    _lib = lib
    return lib


# names every consumer can check against include/dro_amd.h
EXPORTED = (
    "dro_last_error", "dro_abi_version", "dro_timestamp", "dro_wall_clock_hz",
    "dro_warp_cost_forward", "dro_warp_cost_workspace_bytes", "dro_warp_cost_backward",
    "dro_view_synthesis_forward", "dro_view_synthesis_backward",
    "dro_plane_sweep_forward",
    "dro_photometric_workspace_bytes", "dro_photometric_clip_offset", "dro_photometric_forward", "dro_photometric_backward",
    "dro_supervised_workspace_bytes", "dro_supervised_forward", "dro_supervised_backward",
    "dro_convex_upsample_forward", "dro_convex_upsample_backward",
    "dro_convex_upsample_many_forward", "dro_convex_upsample_many_workspace_bytes",
    "dro_convex_upsample_many_backward",
    "dro_bilinear_upsample2x_forward", "dro_bilinear_upsample2x_backward",
    "dro_maxpool3x3s2_forward", "dro_maxpool3x3s2_backward",
    "dro_depth_metrics_blocks", "dro_depth_metrics_workspace_bytes", "dro_depth_metrics_prepare",
    "dro_depth_metrics_reduce", "dro_depth_metrics_median_workspace_bytes", "dro_depth_metrics_median",
    "dro_depth_metrics_demon_prepare", "dro_depth_metrics_demon_reduce",
    "dro_conv2d_strided_workspace_bytes", "dro_conv2d_strided_forward", "dro_conv2d_strided_backward",
    "dro_pose_mean_forward", "dro_pose_mean_backward",
    "dro_resize_rgb8_to_tensor", "dro_color_jitter_rgb8", "dro_resize_rgb8", "dro_rgb8_to_tensor",
    "dro_png_filtered_bytes", "dro_png_decode",
    "dro_batchnorm_workspace_bytes", "dro_batchnorm_relu_forward", "dro_batchnorm_relu_backward",
    "dro_weight_split_bytes", "dro_weight_split",
    "dro_conv2d_workspace_bytes", "dro_conv2d_plan", "dro_debug_conv_stamps", "dro_conv_log", "dro_conv_log_read", "dro_conv2d_forward", "dro_convgru_gates_forward",
    "dro_convgru_blend_forward", "dro_conv2d_backward",
    "dro_conv2d_weight_grad_multi_workspace_bytes", "dro_conv2d_weight_grad_multi",
    "dro_gru_backward_elem", "dro_convgru_candidate_backward", "dro_convgru_gates_backward", "dro_adam_step",
    "dro_bn_state_bytes", "dro_bn_apply", "dro_bn_backward_apply", "dro_conv2d_bn_forward", "dro_conv2d_bn_backward_data",
)


def check(status, what):
    if status != 0:
        msg = load().dro_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed (status {status}): {msg}")


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def stream_of(t):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def require_device(*tensors, what="op"):
    for t in tensors:
        if t is None:
            continue
        if not t.is_cuda:
            raise RuntimeError(f"dro_sfm_amd.{what}: tensors must live on a ROCm device "
                               "(no CPU fallback)")
        if t.dtype != torch.float32:
            raise RuntimeError(f"dro_sfm_amd.{what}: expected float32, got {t.dtype}")
