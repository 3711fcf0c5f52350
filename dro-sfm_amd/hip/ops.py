"""torch.library custom ops (namespace `dro`, torch.ops.dro.*) over the C ABI
of libdro_amd.so, and the Python entry points the drop-in modules call.

Each op checks dtype/device/shape up front (RuntimeError, as the reference's
ATen ops would raise), allocates outputs through the caching allocator, and
launches on the current stream.  Differentiable ops register their backward
(itself a registered op) with torch.library.register_autograd and a fake
kernel with the output shapes; tests/test_library.py checks the schemas.
"""
import contextlib
import os
import ctypes
from typing import Optional

import torch

from . import _lib
from ._lib import check, ptr, require_device, stream_of

POSE_EULER, POSE_MATRIX = 0, 1
DEPTH_METRIC, DEPTH_INV, DEPTH_DISP = 0, 1, 2


def _pose_layout(pose, lead):
    """Return (flat pose [*lead, 6|12] contiguous, mode).  The flattening is
    differentiable torch indexing, so a matrix pose's gradient reaches it
    through autograd."""
    if pose.shape[-1] == 6 and pose.dim() == len(lead) + 1:
        return pose.contiguous(), POSE_EULER
    if pose.shape[-2:] in ((3, 4), (4, 4)) and pose.dim() == len(lead) + 2:
        return pose[..., :3, :].contiguous().view(*lead, 12), POSE_MATRIX
    raise RuntimeError(f"pose must be [...,6] (euler) or [...,3|4,4] matrices, got {tuple(pose.shape)}")


def _disp_range(min_depth, max_depth):
    if min_depth is None or max_depth is None:
        return 0.0, 0.0
    return 1.0 / max_depth, 1.0 / min_depth


# ------------------------------------------------------------------------- warp + feature cost
class GradSinkState:
    """A sink's dense gradient buffer and whether a consumer has written it yet
    (the first consumer to run overwrites, the later ones add: no zero-fill)."""
    __slots__ = ("buf", "written")

    def __init__(self, like):
        # channels-last reference maps keep their layout (the cost kernels
        # scatter into it); everything else gets a dense NCHW buffer
        self.buf = (torch.empty_like(like) if _is_channels_last_refs(like)
                    else torch.empty(like.shape, device=like.device, dtype=like.dtype))
        self.written = False

    def target(self):
        """(buffer, accumulate flag) for the calling consumer's backward."""
        acc = 1 if self.written else 0
        self.written = True
        return self.buf, acc


class _GradSink(torch.autograd.Function):
    """Identity whose gradient is a buffer that consumers write into in place.

    A tensor read by several ops of one step (the feature maps of every cost
    call, the context features of every GRU step, the state and projection
    features every GRU half and 7x7 conv read) otherwise gets one gradient per
    use and autograd sums them with one add launch each.  Ops that know the
    sink (hip.warp_cost, hip.sepconvgru_half, hip.conv2d) write straight into
    it and return None; autograd runs this node only after all of them, so the
    buffer is complete when it is handed on (plus any gradient other ops
    returned)."""

    @staticmethod
    def forward(ctx, x, state):
        ctx.state = state
        ctx.set_materialize_grads(False)
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        st = ctx.state
        if not st.written:
            return g, None
        st.written = False
        return (st.buf if g is None else st.buf + g), None


_SINKS = [True]
# A/B: DRO_DEPTH_SINK=0 returns the cost's depth gradient to autograd instead
# of adding it into the depth state's sink
_DEPTH_SINK = os.environ.get("DRO_DEPTH_SINK", "1") != "0"


def set_grad_sinks(enabled):
    """grad_sink on (default) / off (identity: autograd sums per use).  Measured
    (round 2, sinks covering the 5-D reference feature maps, one box, two
    interleaved rounds of 40 steps): 20.92 / 20.81 ms/step on against 21.28 /
    21.04 off.  (Round 1, before the feature maps were covered: 21.79 on vs
    21.24 off.)"""
    _SINKS[0] = bool(enabled)


def grad_sink(x):
    """x (aliased) with an in-place gradient sink; x itself when no gradient flows.
    One backward per forward.  x may be a dense tensor of any rank or a 4-D
    broadcast view (an expanded pose map): the sink buffer is dense, the view's
    own backward reduces it once."""
    if not (_SINKS[0] and torch.is_grad_enabled() and x.requires_grad and x.is_cuda):
        return x
    if not x.is_contiguous() and x.dim() != 4 and not _is_channels_last_refs(x):
        # broadcast (expanded) views: only the 4-D pose maps the convs read; dense
        # tensors of any rank (the [N,B,C,h,w] reference feature maps) qualify
        return x
    st = GradSinkState(x)
    y = _GradSink.apply(x, st)
    y._dro_gsink = st
    return y


def _sink_of(t):
    return getattr(t, "_dro_gsink", None)


# ------------------------------------------------------------------------- bilinear-cell record
class CellRecord:
    """Test hook (parity tests only): the bilinear cell every warp's backward
    used per pixel -- grid_sample's derivative is piecewise constant in the
    sampling position and jumps where a coordinate crosses an integer, so an
    fp32 and an fp64 evaluation can land on different branches.  Each op call
    made inside record_bilinear_cells() allocates an int32 map (-1 = not
    recorded) that its backward kernel fills (pack_cell, csrc/dro_common.hpp);
    `calls` holds (tag, map) in forward call order."""

    def __init__(self):
        self.calls = []

    def new(self, tag, shape, device, dtype=torch.int32, fill=-1):
        cells = torch.full(shape, fill, dtype=dtype, device=device)
        self.calls.append((tag, cells))
        return cells


_CELLS = [None]


@contextlib.contextmanager
def record_bilinear_cells():
    """Record the bilinear cells of every warp_cost / photometric_loss /
    view_synthesis backward run for ops called inside the block."""
    prev = _CELLS[0]
    _CELLS[0] = rec = CellRecord()
    try:
        yield rec
    finally:
        _CELLS[0] = prev


def record_branch(tag, mask, *inputs):
    """Inside record_bilinear_cells(): keep a branch map an op already has --
    the ReLU mask y > 0 of a BatchNorm+ReLU site, the stem pooling's argmax --
    under `tag` (tests pin the oracle to it; nothing is computed when not
    recording)."""
    rec = _CELLS[0]
    if rec is not None and torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in inputs):
        rec.calls.append((tag, mask() if callable(mask) else mask))


def record_relu(y, mod):
    """y (the ReLU output of module `mod`'s convolution) unchanged; inside
    record_bilinear_cells() its branch y > 0 is kept under ("relu_seq",
    mod._dro_tag), one entry per call of the site."""
    record_branch(("relu_seq", getattr(mod, "_dro_tag", None)), lambda: (y > 0).to(torch.uint8), y)
    return y


def _new_cells(tag, shape, device, *inputs, dtype=torch.int32, fill=-1):
    """A cell map (-1 filled) when recording and a backward will run."""
    rec = _CELLS[0]
    if rec is None or not torch.is_grad_enabled() or not any(t is not None and t.requires_grad for t in inputs):
        return None
    return rec.new(tag, shape, device, dtype, fill)


def _opt(t):
    """Empty-tensor placeholder -> None (custom ops return tensors only)."""
    return None if t is None or t.numel() == 0 and t.dim() == 1 and t.shape[0] == 0 else t


def _none_like(device):
    return torch.empty(0, device=device)


# =========================================================================== torch.library ops
# Every kernel entry point of libdro_amd.so is a torch.library custom op in the
# `dro` namespace (torch.ops.dro.*), with a fake (meta) kernel giving output
# shapes and, for the differentiable ones, register_autograd over a
# registered backward op.  The implementations launch through the C ABI on
# the current stream; there is no CPU kernel (a CPU tensor raises).
Tensor = torch.Tensor


# ------------------------------------------------------------------------- warp + feature cost
def _is_channels_last_refs(t):
    """[N,B,C,h,w] stored as a dense [N,B,h,w,C] (channels_last_refs)."""
    return t.dim() == 5 and not t.is_contiguous() and t.permute(0, 1, 3, 4, 2).is_contiguous()


def _ref_layout(t):
    """(tensor, ref_layout) for the C ABI: channels-last reference maps pass
    as they are (1), anything else as a contiguous NCHW tensor (0)."""
    return (t, 1) if _is_channels_last_refs(t) else (t.contiguous(), 0)


def channels_last_refs(fmap_ref):
    """The [N,B,C,h,w] reference feature maps re-laid channel-contiguous
    ([N,B,h,w,C] memory, same shape): the cost kernels then gather and scatter
    whole channel rows (dro_warp_cost_forward ref_layout 1).  One copy each
    way per training step, shared by every cost call."""
    return fmap_ref.permute(0, 1, 3, 4, 2).contiguous().permute(0, 1, 4, 2, 3)


@torch.library.custom_op("dro::warp_cost", mutates_args=())
def _warp_cost_op(fmap: Tensor, fmap_ref: Tensor, depth: Tensor, pose: Tensor, K: Tensor, ref_K: Tensor,
                  depth_mode: int, min_disp: float, max_disp: float, scale: float, pose_mode: int,
                  reduce_mean: bool, cells: Optional[Tensor]) -> Tensor:
    """get_cost_each / depth_cost_calc (DepthPoseNet.py:76-105): fmap [B,C,h,w],
    fmap_ref [N,B,C,h,w], depth [B,1,h,w], pose [N,B,6|12] -> cost [B,C,h,w]
    (reduce_mean) or [N,B,C,h,w].  `cells` (int32 [N,B,h,w] or None) is the
    test hook the backward fills."""
    lib = _lib.load()
    require_device(fmap, fmap_ref, depth, pose, K, ref_K, what="warp_cost")
    B, C, h, w = fmap.shape
    N = fmap_ref.shape[0]
    fmap, depth = fmap.contiguous(), depth.contiguous()
    fmap_ref, layout = _ref_layout(fmap_ref)
    cost = torch.empty((B, C, h, w) if reduce_mean else (N, B, C, h, w), device=fmap.device)
    check(lib.dro_warp_cost_forward(ptr(fmap), ptr(fmap_ref), ptr(depth), depth_mode, min_disp, max_disp,
                                    ptr(K.contiguous()), ptr(ref_K.contiguous()), scale, ptr(pose.contiguous()),
                                    pose_mode, B, N, C, h, w, int(reduce_mean), layout, ptr(cost),
                                    stream_of(fmap)),
          "dro_warp_cost_forward")
    return cost


@_warp_cost_op.register_fake
def _(fmap, fmap_ref, depth, pose, K, ref_K, depth_mode, min_disp, max_disp, scale, pose_mode, reduce_mean,
      cells):
    B, C, h, w = fmap.shape
    return fmap.new_empty((B, C, h, w) if reduce_mean else (fmap_ref.shape[0], B, C, h, w))


@torch.library.custom_op("dro::warp_cost_backward",
                         mutates_args=("grad_fmap_out", "grad_fmap_ref_out", "cells", "grad_depth_out"))
def _warp_cost_bwd_op(fmap: Tensor, fmap_ref: Tensor, depth: Tensor, pose: Tensor, K: Tensor, ref_K: Tensor,
                      grad_cost: Tensor, depth_mode: int, min_disp: float, max_disp: float, scale: float,
                      pose_mode: int, reduce_mean: bool, need_fmap: bool, need_fmap_ref: bool, need_depth: bool,
                      need_pose: bool, grad_fmap_out: Optional[Tensor], grad_fmap_ref_out: Optional[Tensor],
                      accumulate: int, cells: Optional[Tensor],
                      grad_depth_out: Optional[Tensor]) -> list[Tensor]:
    """Backward of dro::warp_cost.  grad_fmap_out / grad_fmap_ref_out /
    grad_depth_out: buffers the feature / depth gradients are written
    (accumulate bit 0 / 1 / 2: added) into in place -- the gradient sinks of
    maps every cost call of a step shares and of the depth state; the returned
    gradient of such an input is empty.  Returns [g_fmap, g_fmap_ref, g_depth,
    g_pose] (empty where not needed)."""
    lib = _lib.load()
    B, C, h, w = fmap.shape
    N = fmap_ref.shape[0]
    dev = fmap.device
    fmap, depth, pose = fmap.contiguous(), depth.contiguous(), pose.contiguous()
    fmap_ref, layout = _ref_layout(fmap_ref)
    K, ref_K = K.contiguous(), ref_K.contiguous()
    if grad_fmap_ref_out is not None and _is_channels_last_refs(grad_fmap_ref_out) != bool(layout):
        raise RuntimeError("warp_cost backward: the fmap_ref gradient sink's layout differs from fmap_ref's")
    g_f = grad_fmap_out if grad_fmap_out is not None else (torch.empty_like(fmap) if need_fmap else None)
    g_r = grad_fmap_ref_out if grad_fmap_ref_out is not None else (
        torch.empty_like(fmap_ref) if need_fmap_ref else None)
    g_d = grad_depth_out if grad_depth_out is not None else (torch.empty_like(depth) if need_depth else None)
    g_p = torch.empty_like(pose) if need_pose else None
    ws = None
    if g_d is not None or g_p is not None or cells is not None:
        ws = torch.empty(lib.dro_warp_cost_workspace_bytes(B, N, h, w) // 4 + 1, device=dev)
    check(lib.dro_warp_cost_backward(ptr(fmap), ptr(fmap_ref), ptr(depth), depth_mode, min_disp, max_disp,
                                     ptr(K), ptr(ref_K), scale, ptr(pose), pose_mode, B, N, C, h, w,
                                     int(reduce_mean), layout, ptr(grad_cost.contiguous()), ptr(g_f), ptr(g_r),
                                     ptr(g_d),
                                     ptr(g_p), accumulate, ptr(ws), ptr(cells), stream_of(fmap)),
          "dro_warp_cost_backward")
    out = lambda g, own: g if (g is not None and not own) else _none_like(dev)
    return [out(g_f, grad_fmap_out is not None), out(g_r, grad_fmap_ref_out is not None),
            out(g_d, grad_depth_out is not None), out(g_p, False)]


@_warp_cost_bwd_op.register_fake
def _(fmap, fmap_ref, depth, pose, K, ref_K, grad_cost, depth_mode, min_disp, max_disp, scale, pose_mode,
      reduce_mean, need_fmap, need_fmap_ref, need_depth, need_pose, grad_fmap_out, grad_fmap_ref_out, accumulate,
      cells, grad_depth_out):
    e = fmap.new_empty(0)
    return [fmap.new_empty(fmap.shape) if need_fmap and grad_fmap_out is None else e,
            fmap_ref.new_empty(fmap_ref.shape) if need_fmap_ref and grad_fmap_ref_out is None else e,
            depth.new_empty(depth.shape) if need_depth and grad_depth_out is None else e,
            pose.new_empty(pose.shape) if need_pose else e]


def _warp_cost_setup(ctx, inputs, output):
    fmap, fmap_ref, depth, pose, K, ref_K, depth_mode, min_disp, max_disp, scale, pose_mode, reduce_mean, cells = inputs
    ctx.save_for_backward(fmap, fmap_ref, depth, pose, K, ref_K, cells)
    ctx.cfg = (depth_mode, min_disp, max_disp, scale, pose_mode, reduce_mean)
    ctx.need = (fmap.requires_grad, fmap_ref.requires_grad, depth.requires_grad, pose.requires_grad)
    # maps shared by every cost call of a step (and the depth state): gradients
    # summed in their sinks
    ctx.sinks = (_sink_of(fmap) if ctx.need[0] else None, _sink_of(fmap_ref) if ctx.need[1] else None,
                 _sink_of(depth) if ctx.need[2] and _DEPTH_SINK else None)


def _warp_cost_backward(ctx, gcost):
    fmap, fmap_ref, depth, pose, K, ref_K, cells = ctx.saved_tensors
    depth_mode, min_disp, max_disp, scale, pose_mode, reduce_mean = ctx.cfg
    sf, sr, sd = ctx.sinks
    acc, bf, br, bd = 0, None, None, None
    if sf is not None:
        bf, a = sf.target()
        acc |= a
    if sr is not None:
        br, a = sr.target()
        acc |= 2 * a
    if sd is not None:
        bd, a = sd.target()
        acc |= 4 * a
    g = torch.ops.dro.warp_cost_backward(fmap, fmap_ref, depth, pose, K, ref_K, gcost, depth_mode, min_disp,
                                         max_disp, scale, pose_mode, reduce_mean, *ctx.need, bf, br, acc, cells, bd)
    return (*[_opt(t) for t in g], None, None, None, None, None, None, None, None, None)


torch.library.register_autograd("dro::warp_cost", _warp_cost_backward, setup_context=_warp_cost_setup)


def warp_cost(fmap, fmap_ref, depth, pose, K, ref_K=None, *, depth_mode=DEPTH_METRIC,
              min_depth=None, max_depth=None, scale=1.0 / 8, reduce_mean=True, tag=None):
    """Fused get_cost_each / depth_cost_calc (DepthPoseNet.py:76-105).

    fmap [B,C,h,w]; fmap_ref [N,B,C,h,w]; depth [B,1,h,w] encoded per depth_mode
    (DEPTH_DISP applies disp_to_depth(min_depth, max_depth) then inv2depth);
    pose [N,B,6] euler vectors or [N,B,3|4,4] matrices; K/ref_K full-res [B,3,3].
    Returns the mean cost over refs [B,C,h,w] (reduce_mean) or [N,B,C,h,w].
    `tag` names the call in a record_bilinear_cells() record (tests).
    torch.ops.dro.warp_cost underneath.
    """
    if fmap_ref.dim() == 4:
        fmap_ref = fmap_ref.unsqueeze(0)
        pose = pose.unsqueeze(0)
    require_device(fmap, fmap_ref, depth, K, what="warp_cost")
    B, C, h, w = fmap.shape
    N = fmap_ref.shape[0]
    if fmap_ref.shape != (N, B, C, h, w) or depth.shape != (B, 1, h, w) or K.shape != (B, 3, 3):
        raise RuntimeError("warp_cost: shape mismatch (fmap [B,C,h,w], fmap_ref [N,B,C,h,w], "
                           "depth [B,1,h,w], K [B,3,3])")
    if depth_mode == DEPTH_DISP and (min_depth is None or max_depth is None):
        raise RuntimeError("warp_cost: DEPTH_DISP needs min_depth and max_depth")
    pose_flat, pose_mode = _pose_layout(pose, (N, B))
    require_device(pose_flat, what="warp_cost")
    min_disp, max_disp = _disp_range(min_depth, max_depth)
    ref_K = K if ref_K is None else ref_K
    cells = _new_cells(tag, (N, B, h, w), fmap.device, fmap, fmap_ref, depth, pose_flat)
    return torch.ops.dro.warp_cost(fmap, fmap_ref, depth, pose_flat, K, ref_K, depth_mode, float(min_disp),
                                   float(max_disp), float(scale), pose_mode, bool(reduce_mean), cells)


# ------------------------------------------------------------------------- view synthesis
@torch.library.custom_op("dro::view_synthesis", mutates_args=())
def _view_synthesis_op(ref_image: Tensor, depth: Tensor, pose: Tensor, K: Tensor, ref_K: Tensor, depth_mode: int,
                       min_disp: float, max_disp: float, scale: float, pose_mode: int,
                       cells: Optional[Tensor]) -> Tensor:
    """view_synthesis (camera_utils.py:23-56) of N views: ref_image [N,B,C,H,W],
    depth [B,1,H,W], pose [N,B,6|12] -> warped [N,B,C,H,W]."""
    lib = _lib.load()
    require_device(ref_image, depth, pose, K, ref_K, what="view_synthesis")
    N, B, C, H, W = ref_image.shape
    ref_image = ref_image.contiguous()
    warped = torch.empty_like(ref_image)
    check(lib.dro_view_synthesis_forward(ptr(ref_image), ptr(depth.contiguous()), depth_mode, min_disp, max_disp,
                                         ptr(K.contiguous()), ptr(ref_K.contiguous()), scale, ptr(pose.contiguous()),
                                         pose_mode, B, N, C, H, W, ptr(warped), stream_of(ref_image)),
          "dro_view_synthesis_forward")
    return warped


@_view_synthesis_op.register_fake
def _(ref_image, depth, pose, K, ref_K, depth_mode, min_disp, max_disp, scale, pose_mode, cells):
    return ref_image.new_empty(ref_image.shape)


@torch.library.custom_op("dro::view_synthesis_backward", mutates_args=("cells",))
def _view_synthesis_bwd_op(ref_image: Tensor, depth: Tensor, pose: Tensor, K: Tensor, ref_K: Tensor,
                           grad_warped: Tensor, depth_mode: int, min_disp: float, max_disp: float, scale: float,
                           pose_mode: int, need_ref: bool, need_depth: bool, need_pose: bool,
                           cells: Optional[Tensor]) -> list[Tensor]:
    """Backward of dro::view_synthesis: [g_ref_image, g_depth (summed over the
    views), g_pose] (empty where not needed)."""
    lib = _lib.load()
    N, B, C, H, W = ref_image.shape
    dev = depth.device
    ref_image, depth, pose = ref_image.contiguous(), depth.contiguous(), pose.contiguous()
    K, ref_K = K.contiguous(), ref_K.contiguous()
    g_r = torch.empty_like(ref_image) if need_ref else None
    g_d = torch.empty_like(depth) if need_depth else None
    g_p = torch.empty_like(pose) if need_pose else None
    ws = torch.empty(lib.dro_warp_cost_workspace_bytes(B, N, H, W) // 4 + 1, device=dev)
    check(lib.dro_view_synthesis_backward(ptr(ref_image), ptr(depth), depth_mode, min_disp, max_disp, ptr(K),
                                          ptr(ref_K), scale, ptr(pose), pose_mode, B, N, C, H, W,
                                          ptr(grad_warped.contiguous()), ptr(g_r), ptr(g_d), ptr(g_p), ptr(ws),
                                          ptr(cells), stream_of(depth)), "dro_view_synthesis_backward")
    return [t if t is not None else _none_like(dev) for t in (g_r, g_d, g_p)]


@_view_synthesis_bwd_op.register_fake
def _(ref_image, depth, pose, K, ref_K, grad_warped, depth_mode, min_disp, max_disp, scale, pose_mode, need_ref,
      need_depth, need_pose, cells):
    e = depth.new_empty(0)
    return [ref_image.new_empty(ref_image.shape) if need_ref else e, depth.new_empty(depth.shape) if need_depth else e,
            pose.new_empty(pose.shape) if need_pose else e]


def _view_synthesis_setup(ctx, inputs, output):
    ref_image, depth, pose, K, ref_K, depth_mode, min_disp, max_disp, scale, pose_mode, cells = inputs
    ctx.save_for_backward(ref_image, depth, pose, K, ref_K, cells)
    ctx.cfg = (depth_mode, min_disp, max_disp, scale, pose_mode)
    ctx.need = (ref_image.requires_grad, depth.requires_grad, pose.requires_grad)


def _view_synthesis_backward(ctx, gw):
    ref_image, depth, pose, K, ref_K, cells = ctx.saved_tensors
    g = torch.ops.dro.view_synthesis_backward(ref_image, depth, pose, K, ref_K, gw, *ctx.cfg, *ctx.need, cells)
    return (*[_opt(t) for t in g], None, None, None, None, None, None, None, None)


torch.library.register_autograd("dro::view_synthesis", _view_synthesis_backward, setup_context=_view_synthesis_setup)


def view_synthesis(ref_image, depth, pose, K, ref_K=None, *, depth_mode=DEPTH_METRIC, min_depth=None,
                   max_depth=None, scale=1.0):
    """view_synthesis (geometry/camera_utils.py:23-56) of N reference images in one
    launch: ref_image [N,B,C,H,W] (or [B,C,H,W] for one view), depth [B,1,H,W]
    in `depth_mode`, pose [N,B,6] euler vectors or [N,B,3|4,4] matrices (target
    -> reference, Camera(ref_K, Tcw=pose)), K/ref_K [B,3,3] scaled by `scale`
    (scale_intrinsics).  Returns the warped references, same shape as ref_image.
    The kernels are the cost's (warp_cost_fwd/bwd_feat/bwd_geo in SAMPLE mode);
    torch.ops.dro.view_synthesis underneath."""
    single = ref_image.dim() == 4
    if single:
        ref_image, pose = ref_image.unsqueeze(0), pose.unsqueeze(0)
    if depth_mode == DEPTH_DISP and (min_depth is None or max_depth is None):
        raise RuntimeError("view_synthesis: DEPTH_DISP needs min_depth and max_depth")
    require_device(ref_image, depth, K, what="view_synthesis")
    N, B, C, H, W = ref_image.shape
    if depth.shape != (B, 1, H, W) or K.shape != (B, 3, 3):
        raise RuntimeError("view_synthesis: ref_image [N,B,C,H,W], depth [B,1,H,W], K/ref_K [B,3,3]")
    pose_flat, pose_mode = _pose_layout(pose, (N, B))
    min_disp, max_disp = _disp_range(min_depth, max_depth)
    cells = _new_cells("view_synthesis", (N, B, H, W), depth.device, ref_image, depth, pose_flat)
    out = torch.ops.dro.view_synthesis(ref_image, depth, pose_flat, K, K if ref_K is None else ref_K, depth_mode,
                                       float(min_disp), float(max_disp), float(scale), pose_mode, cells)
    return out[0] if single else out


# ------------------------------------------------------------------------- plane sweep (forward only)
@torch.library.custom_op("dro::plane_sweep", mutates_args=())
def _plane_sweep_op(fmap: Tensor, fmap_ref: Tensor, disp: Tensor, pose: Tensor, K: Tensor, ref_K: Tensor,
                    min_disp: float, max_disp: float, scale: float, pose_mode: int) -> Tensor:
    """D fronto-parallel planes: fmap/fmap_ref [B,C,h,w], disp [D] (sigmoid
    space), pose [B,6|12] -> cost volume [B,D,C,h,w]."""
    lib = _lib.load()
    require_device(fmap, fmap_ref, disp, pose, K, ref_K, what="plane_sweep_cost")
    B, C, h, w = fmap.shape
    D = disp.numel()
    cost = torch.empty(B, D, C, h, w, device=fmap.device)
    check(lib.dro_plane_sweep_forward(ptr(fmap.contiguous()), ptr(fmap_ref.contiguous()), ptr(disp.contiguous()), D,
                                      min_disp, max_disp, ptr(K.contiguous()), ptr(ref_K.contiguous()), scale,
                                      ptr(pose.contiguous()), pose_mode, B, C, h, w, ptr(cost), stream_of(fmap)),
          "dro_plane_sweep_forward")
    return cost


@_plane_sweep_op.register_fake
def _(fmap, fmap_ref, disp, pose, K, ref_K, min_disp, max_disp, scale, pose_mode):
    B, C, h, w = fmap.shape
    return fmap.new_empty((B, disp.numel(), C, h, w))


def plane_sweep_cost(fmap, fmap_ref, disp, pose, K, ref_K=None, *, min_depth, max_depth,
                     scale=1.0 / 8):
    """Cost of D fronto-parallel planes (disp [D] in sigmoid space): [B,D,C,h,w]."""
    require_device(fmap, fmap_ref, disp, K, what="plane_sweep_cost")
    B = fmap.shape[0]
    pose_flat, pose_mode = _pose_layout(pose, (B,))
    min_disp, max_disp = _disp_range(min_depth, max_depth)
    return torch.ops.dro.plane_sweep(fmap, fmap_ref, disp, pose_flat, K, K if ref_K is None else ref_K,
                                     float(min_disp), float(max_disp), float(scale), pose_mode)


# ------------------------------------------------------------------------- photometric loss
@torch.library.custom_op("dro::photometric_loss", mutates_args=())
def _photometric_op(image: Tensor, context: Tensor, inv_depths: Tensor, pose: Tensor, K: Tensor, ref_K: Tensor,
                    pose_mode: int, ssim_w: float, C1: float, C2: float, smooth_w: float, automask: bool,
                    reduce_min: bool, clip_loss: float, cells: Optional[Tensor],
                    l1_signs: Optional[Tensor]) -> tuple[Tensor, Tensor, Tensor]:
    """MultiViewPhotometricDecayLoss (multiview_photometric_loss_mf.py:303-361):
    image [B,3,H,W], context [N,B,3,H,W], inv_depths [n,B,1,H,W], pose
    [N,n,B,6|12] -> (loss [1], metrics [2] (photometric, smoothness), the
    forward state [bytes] the backward reads; its first n*B*H*W bytes are the
    per-pixel min selection).  clip_loss > 0: every candidate map clamped at
    mean + clip_loss * std of itself (:223-227).  `cells` (int32 [N,n,B,H,W])
    and `l1_signs` (int8 [N,n,B,3,H,W]), or None: the backward's test hooks
    (the clip thresholds are in the state: photometric_clip_thresholds)."""
    lib = _lib.load()
    require_device(image, context, inv_depths, pose, K, ref_K, what="photometric_loss")
    n, B, _, H, W = inv_depths.shape
    N = context.shape[0]
    ws = torch.empty(lib.dro_photometric_workspace_bytes(B, N, n, H, W, clip_loss), device=image.device,
                     dtype=torch.uint8)
    out = torch.empty(3, device=image.device)
    check(lib.dro_photometric_forward(ptr(image.contiguous()), ptr(context.contiguous()), ptr(inv_depths.contiguous()),
                                      ptr(K.contiguous()), ptr(ref_K.contiguous()), ptr(pose.contiguous()), pose_mode,
                                      B, N, n, H, W, ssim_w, C1, C2, smooth_w, int(automask), int(reduce_min),
                                      clip_loss, ptr(out), ptr(ws), stream_of(image)), "dro_photometric_forward")
    return out[0:1].clone(), out[1:].clone(), ws


@_photometric_op.register_fake
def _(image, context, inv_depths, pose, K, ref_K, pose_mode, ssim_w, C1, C2, smooth_w, automask, reduce_min,
      clip_loss, cells, l1_signs):
    n, B, _, H, W = inv_depths.shape
    nb = _lib.load().dro_photometric_workspace_bytes(B, context.shape[0], n, H, W, clip_loss)
    return image.new_empty(1), image.new_empty(2), image.new_empty(nb, dtype=torch.uint8)


@torch.library.custom_op("dro::photometric_loss_backward", mutates_args=("cells", "l1_signs"))
def _photometric_bwd_op(image: Tensor, context: Tensor, inv_depths: Tensor, pose: Tensor, K: Tensor,
                        ref_K: Tensor, state: Tensor, grad_loss: Tensor, pose_mode: int, ssim_w: float, C1: float,
                        C2: float, smooth_w: float, automask: bool, reduce_min: bool, clip_loss: float,
                        need_pose: bool, cells: Optional[Tensor], l1_signs: Optional[Tensor]) -> list[Tensor]:
    """Backward of dro::photometric_loss: [g_inv_depths, g_pose (empty unless need_pose)]."""
    lib = _lib.load()
    n, B, _, H, W = inv_depths.shape
    N = context.shape[0]
    image, context, inv_depths, pose = image.contiguous(), context.contiguous(), inv_depths.contiguous(), pose.contiguous()
    K, ref_K = K.contiguous(), ref_K.contiguous()
    g_inv = torch.empty_like(inv_depths)
    g_pose = torch.empty_like(pose) if need_pose else None
    check(lib.dro_photometric_backward(ptr(image), ptr(context), ptr(inv_depths), ptr(K), ptr(ref_K), ptr(pose),
                                       pose_mode, B, N, n, H, W, ssim_w, C1, C2, smooth_w, int(automask),
                                       int(reduce_min), clip_loss, ptr(grad_loss.contiguous()), ptr(g_inv),
                                       ptr(g_pose), ptr(state), ptr(cells), ptr(l1_signs), stream_of(image)),
          "dro_photometric_backward")
    return [g_inv, g_pose if g_pose is not None else _none_like(image.device)]


@_photometric_bwd_op.register_fake
def _(image, context, inv_depths, pose, K, ref_K, state, grad_loss, pose_mode, ssim_w, C1, C2, smooth_w, automask,
      reduce_min, clip_loss, need_pose, cells, l1_signs):
    return [inv_depths.new_empty(inv_depths.shape), pose.new_empty(pose.shape) if need_pose else pose.new_empty(0)]


def _photometric_setup(ctx, inputs, output):
    (image, context, inv_depths, pose, K, ref_K, pose_mode, ssim_w, C1, C2, smooth_w, automask, reduce_min, clip_loss,
     cells, l1_signs) = inputs
    _, metrics, state = output
    ctx.save_for_backward(image, context, inv_depths, pose, K, ref_K, state, cells, l1_signs)
    ctx.cfg = (pose_mode, ssim_w, C1, C2, smooth_w, automask, reduce_min, clip_loss)
    ctx.need = (inv_depths.requires_grad, pose.requires_grad)
    ctx.mark_non_differentiable(metrics, state)
    ctx.set_materialize_grads(False)     # no zero-filled gradients for the non-differentiable outputs


def _photometric_backward(ctx, gloss, _gmetrics, _gstate):
    if gloss is None:
        return (None,) * 16
    image, context, inv_depths, pose, K, ref_K, state, cells, l1_signs = ctx.saved_tensors
    g_inv, g_pose = torch.ops.dro.photometric_loss_backward(image, context, inv_depths, pose, K, ref_K, state, gloss,
                                                            *ctx.cfg, ctx.need[1], cells, l1_signs)
    # one entry per forward input: image, context, inv_depths, pose, then twelve non-differentiable ones
    return (None, None, g_inv if ctx.need[0] else None, _opt(g_pose)) + (None,) * 12


torch.library.register_autograd("dro::photometric_loss", _photometric_backward, setup_context=_photometric_setup)


def photometric_loss(image, context, inv_depths, pose, K, ref_K=None, *, ssim_w=0.85, C1=1e-4,
                     C2=9e-4, smooth_w=0.001, automask=True, reduce_min=True, clip_loss=0.0,
                     return_selection=False):
    """Fused MultiViewPhotometricDecayLoss (multiview_photometric_loss_mf.py:303-361).
    clip_loss > 0: each candidate map is clamped at float(mean + clip_loss * std)
    of itself before the reduction (:223-227).

    image [B,3,H,W]; context [N,B,3,H,W]; inv_depths [n,B,1,H,W];
    pose [N,n,B,6] euler vectors or [N,n,B,3|4,4] matrices.
    Returns (loss [1], detached metrics [2] = (photometric_loss, smoothness_loss))
    and, with return_selection, the per-pixel min-candidate index uint8 [n,B,H,W]
    (candidate order of the reference's torch.cat: warped_0, unwarped_0, ...).
    torch.ops.dro.photometric_loss underneath.
    """
    require_device(image, context, inv_depths, K, what="photometric_loss")
    n, B, _, H, W = inv_depths.shape
    N = context.shape[0]
    if image.shape != (B, 3, H, W) or context.shape != (N, B, 3, H, W):
        raise RuntimeError("photometric_loss: image [B,3,H,W], context [N,B,3,H,W] and "
                           "inv_depths [n,B,1,H,W] must share B,H,W (full-res predictions)")
    pose_flat, pose_mode = _pose_layout(pose, (N, n, B))
    require_device(pose_flat, what="photometric_loss")
    cells = _new_cells("photo", (N, n, B, H, W), image.device, inv_depths, pose_flat)
    signs = _new_cells("photo_l1", (N, n, B, 3, H, W), image.device, inv_depths, pose_flat, dtype=torch.int8, fill=0)
    loss, metrics, state = torch.ops.dro.photometric_loss(
        image, context, inv_depths, pose_flat, K, K if ref_K is None else ref_K, pose_mode, float(ssim_w),
        float(C1), float(C2), float(smooth_w), bool(automask), bool(reduce_min), float(clip_loss), cells, signs)
    if clip_loss > 0 and _CELLS[0] is not None:
        # the forward's clip thresholds and clamp decisions (in its state), for
        # the oracle's branch
        lib = _lib.load()
        o_pm, o_thr = (lib.dro_photometric_clip_offset(B, N, n, H, W, w) for w in (0, 1))
        thr = state[o_thr:o_thr + 4 * (N * n + N)].view(torch.float32).clone()
        pm = state[o_pm:o_pm + 4 * N * n * B * H * W].view(torch.float32).view(N, n, B, H, W)
        keep = (pm <= thr[:N * n].view(N, n, 1, 1, 1)).to(torch.uint8)
        _CELLS[0].calls.append(("photo_clip", thr))
        _CELLS[0].calls.append(("photo_clipmask", keep))
    if return_selection:
        return loss, metrics, state[:n * B * H * W].view(n, B, H, W)
    return loss, metrics


# ------------------------------------------------------------------------- supervised loss
@torch.library.custom_op("dro::supervised_loss", mutates_args=())
def _supervised_op(gt_inv: Tensor, inv_depths: Tensor, pose: Tensor, gt_pose: Tensor, K: Tensor, ref_K: Tensor,
                   pose_mode: int, min_depth: float, max_depth: float) -> tuple[Tensor, Tensor]:
    """SupervisedDepthPoseLoss (supervised_loss.py:343-371, 'sparse-l1'):
    gt_inv [B,1,H,W], inv_depths [n,B,1,H,W], pose [N,n,B,6|12], gt_pose
    [N,B,12] -> (loss [1], metrics [2] (depth_loss, pose_loss))."""
    lib = _lib.load()
    require_device(gt_inv, inv_depths, pose, gt_pose, K, ref_K, what="supervised_loss")
    n, B, _, H, W = inv_depths.shape
    N = gt_pose.shape[0]
    ws = torch.empty(lib.dro_supervised_workspace_bytes(B, N, n, H, W) // 4 + 1, device=gt_inv.device)
    out = torch.empty(3, device=gt_inv.device)
    check(lib.dro_supervised_forward(ptr(gt_inv.contiguous()), ptr(inv_depths.contiguous()), ptr(K.contiguous()),
                                     ptr(ref_K.contiguous()), ptr(gt_pose.contiguous()), ptr(pose.contiguous()),
                                     pose_mode, B, N, n, H, W, min_depth, max_depth, ptr(out), ptr(ws),
                                     stream_of(gt_inv)), "dro_supervised_forward")
    return out[0:1].clone(), out[1:].clone()


@_supervised_op.register_fake
def _(gt_inv, inv_depths, pose, gt_pose, K, ref_K, pose_mode, min_depth, max_depth):
    return gt_inv.new_empty(1), gt_inv.new_empty(2)


@torch.library.custom_op("dro::supervised_loss_backward", mutates_args=())
def _supervised_bwd_op(gt_inv: Tensor, inv_depths: Tensor, pose: Tensor, gt_pose: Tensor, K: Tensor, ref_K: Tensor,
                       grad_loss: Tensor, pose_mode: int, min_depth: float, max_depth: float) -> list[Tensor]:
    """Backward of dro::supervised_loss: [g_inv_depths, g_pose]."""
    lib = _lib.load()
    n, B, _, H, W = inv_depths.shape
    N = gt_pose.shape[0]
    gt_inv, inv_depths, pose, gt_pose = gt_inv.contiguous(), inv_depths.contiguous(), pose.contiguous(), gt_pose.contiguous()
    K, ref_K = K.contiguous(), ref_K.contiguous()
    g_inv, g_pose = torch.empty_like(inv_depths), torch.empty_like(pose)
    ws = torch.empty(lib.dro_supervised_workspace_bytes(B, N, n, H, W) // 4 + 1, device=gt_inv.device)
    check(lib.dro_supervised_backward(ptr(gt_inv), ptr(inv_depths), ptr(K), ptr(ref_K), ptr(gt_pose), ptr(pose),
                                      pose_mode, B, N, n, H, W, min_depth, max_depth, ptr(grad_loss.contiguous()),
                                      ptr(g_inv), ptr(g_pose), ptr(ws), stream_of(gt_inv)), "dro_supervised_backward")
    return [g_inv, g_pose]


@_supervised_bwd_op.register_fake
def _(gt_inv, inv_depths, pose, gt_pose, K, ref_K, grad_loss, pose_mode, min_depth, max_depth):
    return [inv_depths.new_empty(inv_depths.shape), pose.new_empty(pose.shape)]


def _supervised_setup(ctx, inputs, output):
    gt_inv, inv_depths, pose, gt_pose, K, ref_K, pose_mode, min_depth, max_depth = inputs
    ctx.save_for_backward(gt_inv, inv_depths, pose, gt_pose, K, ref_K)
    ctx.cfg = (pose_mode, min_depth, max_depth)
    ctx.need = (inv_depths.requires_grad, pose.requires_grad)
    ctx.mark_non_differentiable(output[1])
    ctx.set_materialize_grads(False)     # no zero-filled gradients for the non-differentiable outputs


def _supervised_backward(ctx, gloss, _gmetrics):
    if gloss is None:
        return (None,) * 9
    gt_inv, inv_depths, pose, gt_pose, K, ref_K = ctx.saved_tensors
    g_inv, g_pose = torch.ops.dro.supervised_loss_backward(gt_inv, inv_depths, pose, gt_pose, K, ref_K, gloss,
                                                           *ctx.cfg)
    return (None, g_inv if ctx.need[0] else None, g_pose if ctx.need[1] else None, None, None, None, None, None,
            None)


torch.library.register_autograd("dro::supervised_loss", _supervised_backward, setup_context=_supervised_setup)


def supervised_loss(gt_inv, inv_depths, pose, gt_pose, K, ref_K=None, *, min_depth, max_depth):
    """Fused SupervisedDepthPoseLoss (supervised_loss.py:343-371, 'sparse-l1').

    gt_inv [B,1,H,W]; inv_depths [n,B,1,H,W]; pose [N,n,B,6] euler vectors or
    [N,n,B,3|4,4] matrices; gt_pose [N,B,3|4,4].  Returns (loss [1], detached
    metrics [2] = (depth_loss, pose_loss)).  torch.ops.dro.supervised_loss.
    """
    require_device(gt_inv, inv_depths, gt_pose, K, what="supervised_loss")
    n, B, _, H, W = inv_depths.shape
    N = gt_pose.shape[0]
    ref_K = K if ref_K is None else ref_K
    if gt_inv.shape != (B, 1, H, W) or K.shape != (B, 3, 3) or ref_K.shape != (B, 3, 3):
        raise RuntimeError("supervised_loss: gt_inv [B,1,H,W] and inv_depths [n,B,1,H,W] must "
                           "share B,H,W; K/ref_K [B,3,3]")
    pose_flat, pose_mode = _pose_layout(pose, (N, n, B))
    gt_flat, gt_mode = _pose_layout(gt_pose, (N, B))
    if gt_mode != POSE_MATRIX:
        raise RuntimeError("supervised_loss: gt_pose must be [N,B,3|4,4] matrices")
    require_device(pose_flat, what="supervised_loss")
    return torch.ops.dro.supervised_loss(gt_inv, inv_depths, pose_flat, gt_flat.detach(), K, ref_K, pose_mode,
                                         float(min_depth), float(max_depth))


# ------------------------------------------------------------------------- convex upsample
@torch.library.custom_op("dro::convex_upsample", mutates_args=())
def _convex_upsample_op(inv: Tensor, mask: Tensor, ratio: int, add: float, mul: float) -> Tensor:
    """DepthPoseNet.upsample_depth (DepthPoseNet.py:63-74): inv [B,1,h,w], mask
    [B,9*r*r,h,w] -> add + mul * up [B,1,r*h,r*w]."""
    lib = _lib.load()
    require_device(inv, mask, what="convex_upsample")
    B, _, h, w = inv.shape
    out = torch.empty(B, 1, h * ratio, w * ratio, device=inv.device)
    check(lib.dro_convex_upsample_forward(ptr(inv.contiguous()), ptr(mask.contiguous()), B, h, w, ratio,
                                          ctypes.c_float(add), ctypes.c_float(mul), ptr(out), stream_of(inv)),
          "dro_convex_upsample_forward")
    return out


@_convex_upsample_op.register_fake
def _(inv, mask, ratio, add, mul):
    B, _, h, w = inv.shape
    return inv.new_empty((B, 1, h * ratio, w * ratio))


@torch.library.custom_op("dro::convex_upsample_backward", mutates_args=())
def _convex_upsample_bwd_op(inv: Tensor, mask: Tensor, grad_out: Tensor, ratio: int, mul: float,
                            need_inv: bool) -> list[Tensor]:
    """Backward of dro::convex_upsample: [g_inv (empty unless need_inv), g_mask]."""
    lib = _lib.load()
    B, _, h, w = inv.shape
    g_inv = torch.empty_like(inv) if need_inv else None
    g_mask = torch.empty_like(mask)
    check(lib.dro_convex_upsample_backward(ptr(inv), ptr(mask), ptr(grad_out.contiguous()), B, h, w, ratio,
                                           ctypes.c_float(mul), ptr(g_inv), ptr(g_mask), stream_of(inv)),
          "dro_convex_upsample_backward")
    return [g_inv if g_inv is not None else _none_like(inv.device), g_mask]


@_convex_upsample_bwd_op.register_fake
def _(inv, mask, grad_out, ratio, mul, need_inv):
    return [inv.new_empty(inv.shape) if need_inv else inv.new_empty(0), mask.new_empty(mask.shape)]


def _convex_upsample_setup(ctx, inputs, output):
    inv, mask, ratio, add, mul = inputs
    ctx.save_for_backward(inv.contiguous(), mask.contiguous())
    ctx.cfg = (ratio, mul, inv.requires_grad, mask.requires_grad)


def _convex_upsample_backward(ctx, gout):
    inv, mask = ctx.saved_tensors
    ratio, mul, need_inv, need_mask = ctx.cfg
    g_inv, g_mask = torch.ops.dro.convex_upsample_backward(inv, mask, gout, ratio, mul, need_inv)
    return _opt(g_inv), g_mask if need_mask else None, None, None, None


torch.library.register_autograd("dro::convex_upsample", _convex_upsample_backward,
                                setup_context=_convex_upsample_setup)


def convex_upsample(inv, mask, ratio=8, affine=None):
    """DepthPoseNet.upsample_depth (DepthPoseNet.py:63-74): [B,1,h,w] -> [B,1,rh,rw];
    affine=(add, mul) folds `add + mul * out` (scale_inv_depth) into the kernel."""
    require_device(inv, mask, what="convex_upsample")
    B, _, h, w = inv.shape
    if mask.shape != (B, 9 * ratio * ratio, h, w):
        raise RuntimeError("convex_upsample: mask must be [B, 9*r*r, h, w]")
    add, mul = affine if affine is not None else (0.0, 1.0)
    return torch.ops.dro.convex_upsample(inv, mask, int(ratio), float(add), float(mul))


def _ptr_table(ts):
    arr = (ctypes.c_void_p * len(ts))()
    for i, t in enumerate(ts):
        arr[i] = t.data_ptr() if t is not None else None
    return arr


@torch.library.custom_op("dro::convex_upsample_many", mutates_args=())
def _convex_upsample_many_op(invs: list[Tensor], masks: list[Tensor], ratio: int, add: float,
                             mul: float) -> Tensor:
    """n convex upsamples in one launch: invs n x [B,1,h,w], masks n x
    [B,9*r*r,h,w] -> [n,B,1,r*h,r*w]."""
    lib = _lib.load()
    invs = [t.contiguous() for t in invs]
    masks = [t.contiguous() for t in masks]
    require_device(*invs, *masks, what="convex_upsample_many")
    n = len(invs)
    B, _, h, w = invs[0].shape
    out = torch.empty(n, B, 1, h * ratio, w * ratio, device=invs[0].device)
    check(lib.dro_convex_upsample_many_forward(_ptr_table(invs), _ptr_table(masks), n, B, h, w, ratio,
                                               ctypes.c_float(add), ctypes.c_float(mul), ptr(out), stream_of(out)),
          "dro_convex_upsample_many_forward")
    return out


@_convex_upsample_many_op.register_fake
def _(invs, masks, ratio, add, mul):
    B, _, h, w = invs[0].shape
    return invs[0].new_empty((len(invs), B, 1, h * ratio, w * ratio))


@torch.library.custom_op("dro::convex_upsample_many_backward", mutates_args=())
def _convex_upsample_many_bwd_op(invs: list[Tensor], masks: list[Tensor], grad_out: Tensor, ratio: int, mul: float,
                                 need_inv: list[bool]) -> list[Tensor]:
    """Backward of dro::convex_upsample_many: the n inverse-depth gradients
    (empty where not needed) followed by the n mask gradients; deterministic
    (two passes, no atomics)."""
    lib = _lib.load()
    n = len(invs)
    B, _, h, w = invs[0].shape
    g_inv = [torch.empty_like(t) if need_inv[i] else None for i, t in enumerate(invs)]
    g_mask = [torch.empty_like(m) for m in masks]
    nb = int(lib.dro_convex_upsample_many_workspace_bytes(n, B, h, w))
    ws = torch.empty(nb, dtype=torch.uint8, device=grad_out.device)
    check(lib.dro_convex_upsample_many_backward(_ptr_table(invs), _ptr_table(masks), ptr(grad_out.contiguous()),
                                                n, B, h, w, ratio, ctypes.c_float(mul), _ptr_table(g_inv),
                                                _ptr_table(g_mask), ptr(ws), nb, stream_of(grad_out)),
          "dro_convex_upsample_many_backward")
    return [g if g is not None else _none_like(grad_out.device) for g in g_inv] + g_mask


@_convex_upsample_many_bwd_op.register_fake
def _(invs, masks, grad_out, ratio, mul, need_inv):
    return ([t.new_empty(t.shape) if need_inv[i] else t.new_empty(0) for i, t in enumerate(invs)] +
            [m.new_empty(m.shape) for m in masks])


def _convex_upsample_many_setup(ctx, inputs, output):
    invs, masks, ratio, add, mul = inputs
    invs = [t.contiguous() for t in invs]
    masks = [t.contiguous() for t in masks]
    ctx.save_for_backward(*invs, *masks)
    ctx.cfg = (len(invs), ratio, mul, [t.requires_grad for t in invs], [m.requires_grad for m in masks])


def _convex_upsample_many_backward(ctx, gout):
    n, ratio, mul, need_inv, need_mask = ctx.cfg
    saved = ctx.saved_tensors
    g = torch.ops.dro.convex_upsample_many_backward(list(saved[:n]), list(saved[n:]), gout, ratio, mul, need_inv)
    g_inv = [_opt(t) for t in g[:n]]
    g_mask = [t if need_mask[i] else None for i, t in enumerate(g[n:])]
    return g_inv, g_mask, None, None, None


torch.library.register_autograd("dro::convex_upsample_many", _convex_upsample_many_backward,
                                setup_context=_convex_upsample_many_setup)


def convex_upsample_many(invs, masks, ratio=8, affine=None):
    """convex_upsample of n (inv, mask) pairs in one launch each way: returns the
    stacked [n, B, 1, rh, rw] (the losses read the predictions stacked;
    stacked_view() recovers it from its unbind() views).  Deterministic
    backward (no atomics).  torch.ops.dro.convex_upsample_many underneath."""
    if not 1 <= len(invs) == len(masks) <= 32:
        raise RuntimeError("convex_upsample_many: 1..32 (inv, mask) pairs")
    require_device(*invs, *masks, what="convex_upsample_many")
    B, _, h, w = invs[0].shape
    for i, m in zip(invs, masks):
        if i.shape != (B, 1, h, w) or m.shape != (B, 9 * ratio * ratio, h, w):
            raise RuntimeError("convex_upsample_many: every inv must be [B,1,h,w] and mask [B,9*r*r,h,w]")
    add, mul = affine if affine is not None else (0.0, 1.0)
    return torch.ops.dro.convex_upsample_many(list(invs), list(masks), int(ratio), float(add), float(mul))


def stacked_view(ts):
    """torch.stack(ts) without the copy when ts are, in order, the unbind()
    views of one contiguous [n, ...] tensor (convex_upsample_many's output);
    otherwise torch.stack(ts)."""
    ts = list(ts)
    base = ts[0]._base if ts else None
    if (base is not None and base.is_contiguous() and base.dim() == ts[0].dim() + 1 and base.shape[0] == len(ts)
            and all(t._base is base and t.shape == base.shape[1:] and
                    t.storage_offset() == base.storage_offset() + i * base.stride(0) for i, t in enumerate(ts))):
        return base
    return torch.stack(ts, 0)


# ------------------------------------------------------------------ bilinear 2x upsample
@torch.library.custom_op("dro::bilinear_upsample2x", mutates_args=())
def _bilinear2x_op(x: Tensor) -> Tensor:
    """F.interpolate(x, scale_factor=2, bilinear, align_corners=False), float32 NCHW."""
    lib = _lib.load()
    require_device(x, what="bilinear_upsample2x")
    N, C, h, w = x.shape
    out = torch.empty(N, C, 2 * h, 2 * w, device=x.device)
    check(lib.dro_bilinear_upsample2x_forward(ptr(x.contiguous()), N * C, h, w, ptr(out), stream_of(x)),
          "dro_bilinear_upsample2x_forward")
    return out


@_bilinear2x_op.register_fake
def _(x):
    N, C, h, w = x.shape
    return x.new_empty((N, C, 2 * h, 2 * w))


@torch.library.custom_op("dro::bilinear_upsample2x_backward", mutates_args=())
def _bilinear2x_bwd_op(grad_out: Tensor) -> Tensor:
    lib = _lib.load()
    N, C, H2, W2 = grad_out.shape
    h, w = H2 // 2, W2 // 2
    gx = torch.empty(N, C, h, w, device=grad_out.device)
    check(lib.dro_bilinear_upsample2x_backward(ptr(grad_out.contiguous()), N * C, h, w, ptr(gx), stream_of(grad_out)),
          "dro_bilinear_upsample2x_backward")
    return gx


@_bilinear2x_bwd_op.register_fake
def _(grad_out):
    N, C, H2, W2 = grad_out.shape
    return grad_out.new_empty((N, C, H2 // 2, W2 // 2))


torch.library.register_autograd("dro::bilinear_upsample2x",
                                lambda ctx, g: torch.ops.dro.bilinear_upsample2x_backward(g),
                                setup_context=lambda ctx, inputs, output: None)


def bilinear_upsample2x(x):
    """F.interpolate(x, scale_factor=2, mode="bilinear", align_corners=False) for float32
    NCHW (reference networks/optim/extractor.py:91-97); deterministic backward."""
    if x.dtype != torch.float32 or x.dim() != 4:
        raise RuntimeError("bilinear_upsample2x: expects a float32 NCHW tensor")
    return torch.ops.dro.bilinear_upsample2x(x)


# ------------------------------------------------------------------ ResNet stem max pooling
@torch.library.custom_op("dro::maxpool3x3s2", mutates_args=())
def _maxpool_op(x: Tensor) -> tuple[Tensor, Tensor]:
    """F.max_pool2d(x, 3, 2, 1): (y, argmax uint8 in the 3x3 window)."""
    lib = _lib.load()
    require_device(x, what="maxpool3x3s2")
    N, C, H, W = x.shape
    Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    y = torch.empty(N, C, Ho, Wo, device=x.device)
    arg = torch.empty(N, C, Ho, Wo, device=x.device, dtype=torch.uint8)
    check(lib.dro_maxpool3x3s2_forward(ptr(x.contiguous()), N * C, H, W, ptr(y), ptr(arg), stream_of(x)),
          "dro_maxpool3x3s2_forward")
    return y, arg


@_maxpool_op.register_fake
def _(x):
    N, C, H, W = x.shape
    sh = (N, C, (H - 1) // 2 + 1, (W - 1) // 2 + 1)
    return x.new_empty(sh), x.new_empty(sh, dtype=torch.uint8)


@torch.library.custom_op("dro::maxpool3x3s2_backward", mutates_args=())
def _maxpool_bwd_op(grad_out: Tensor, argmax: Tensor, H: int, W: int) -> Tensor:
    lib = _lib.load()
    N, C = grad_out.shape[:2]
    gx = torch.empty(N, C, H, W, device=grad_out.device)
    check(lib.dro_maxpool3x3s2_backward(ptr(grad_out.contiguous()), ptr(argmax), N * C, H, W, ptr(gx),
                                        stream_of(grad_out)), "dro_maxpool3x3s2_backward")
    return gx


@_maxpool_bwd_op.register_fake
def _(grad_out, argmax, H, W):
    return grad_out.new_empty((grad_out.shape[0], grad_out.shape[1], H, W))


def _maxpool_setup(ctx, inputs, output):
    ctx.save_for_backward(output[1])
    ctx.hw = inputs[0].shape[2:]
    ctx.mark_non_differentiable(output[1])
    ctx.set_materialize_grads(False)     # no zero-filled gradients for the non-differentiable outputs


torch.library.register_autograd(
    "dro::maxpool3x3s2", lambda ctx, gy, _garg: torch.ops.dro.maxpool3x3s2_backward(gy, ctx.saved_tensors[0], *ctx.hw),
    setup_context=_maxpool_setup)


def maxpool3x3s2(x, tag=None):
    """F.max_pool2d(x, 3, 2, 1) for float32 NCHW on the GPU (ResNet stem,
    reference networks/optim/extractor.py:60-66); bit-identical forward and
    backward, one argmax byte per output instead of int64 indices.  Inside
    record_bilinear_cells() the argmax map (dy * 3 + dx per output, the window
    the backward routes to) is recorded as ("maxpool", tag): near-ties of a
    window are a branch of the step like bilinear cells (tests only)."""
    if x.dtype != torch.float32 or x.dim() != 4:
        raise RuntimeError("maxpool3x3s2: expects a float32 NCHW tensor")
    y, arg = torch.ops.dro.maxpool3x3s2(x)
    record_branch(("maxpool", tag), arg, x)
    return y


# ------------------------------------------------------------------ PoseHead mean
@torch.library.custom_op("dro::pose_mean", mutates_args=())
def _pose_mean_op(y: Tensor, pose: Optional[Tensor], rot_scale: float) -> Tensor:
    """PoseHead's output (update.py:16-28): y.mean((2, 3)) [B,C] with channels
    3..5 scaled by rot_scale, plus `pose` [B,C] when given."""
    lib = _lib.load()
    require_device(y, pose, what="pose_mean")
    B, C, H, W = y.shape
    out = torch.empty(B, C, device=y.device)
    check(lib.dro_pose_mean_forward(ptr(y.contiguous()), ptr(pose.contiguous() if pose is not None else None),
                                    ptr(out), B, C, H * W, float(rot_scale), stream_of(y)), "dro_pose_mean_forward")
    return out


@_pose_mean_op.register_fake
def _(y, pose, rot_scale):
    return y.new_empty(y.shape[:2])


@torch.library.custom_op("dro::pose_mean_backward", mutates_args=())
def _pose_mean_bwd_op(grad_out: Tensor, H: int, W: int, rot_scale: float) -> Tensor:
    lib = _lib.load()
    B, C = grad_out.shape
    gy = torch.empty(B, C, H, W, device=grad_out.device)
    check(lib.dro_pose_mean_backward(ptr(grad_out.contiguous()), ptr(gy), B, C, H * W, float(rot_scale),
                                     stream_of(grad_out)), "dro_pose_mean_backward")
    return gy


@_pose_mean_bwd_op.register_fake
def _(grad_out, H, W, rot_scale):
    return grad_out.new_empty((*grad_out.shape, H, W))


def _pose_mean_setup(ctx, inputs, output):
    y, pose, rot_scale = inputs
    ctx.cfg = (y.shape[2], y.shape[3], rot_scale, pose is not None and pose.requires_grad)


def _pose_mean_backward(ctx, gout):
    H, W, rs, pose_grad = ctx.cfg
    return torch.ops.dro.pose_mean_backward(gout, H, W, rs), (gout if pose_grad else None), None


torch.library.register_autograd("dro::pose_mean", _pose_mean_backward, setup_context=_pose_mean_setup)


def pose_mean(y, rot_scale=0.01, pose=None):
    """PoseHead's output (update.py:16-28) -- y.mean((2, 3)) with the rotation
    channels (3..5) scaled by rot_scale -- plus `pose` when given (the update
    `pose + pose_head(net)`, update.py:189-197): one launch forward, one
    backward.  y [B, C, H, W], pose [B, C].  torch.ops.dro.pose_mean."""
    require_device(y, pose, what="pose_mean")
    return torch.ops.dro.pose_mean(y, pose, float(rot_scale))


# ------------------------------------------------------------------ training-mode BatchNorm (+ skip) (+ ReLU)
# Not a torch.library op: its launch updates the running statistics in place
# (fused into the statistics pass), and torch.library refuses an autograd
# formula for an op that mutates inputs; splitting the update out would add
# two launches per BN site (~120 per step).
class _BatchNormAct(torch.autograd.Function):
    """Training-mode BN (+ skip) (+ ReLU) in two launches each way (csrc/batchnorm.hip)."""

    @staticmethod
    def forward(ctx, x, weight, bias, skip, running_mean, running_var, num_batches, relu, eps,
                momentum):
        lib = _lib.load()
        require_device(x, what="batchnorm_act")
        N, C, H, W = x.shape
        x = x.contiguous()
        skip = skip.contiguous() if skip is not None else None
        y = torch.empty_like(x)
        smean = torch.empty(C, device=x.device, dtype=torch.float32)
        sinv = torch.empty(C, device=x.device, dtype=torch.float32)
        nws = lib.dro_batchnorm_workspace_bytes(N, C, H * W)
        ws = torch.empty(max(nws, 16), device=x.device, dtype=torch.uint8)
        check(lib.dro_batchnorm_relu_forward(
            ptr(x), ptr(weight), ptr(bias), ptr(skip), int(relu), N, C, H * W, float(eps),
            float(momentum), ptr(running_mean), ptr(running_var), ptr(num_batches), ptr(y),
            ptr(smean), ptr(sinv), ptr(ws), nws, stream_of(x)), "dro_batchnorm_relu_forward")
        ctx.save_for_backward(x, y, weight, smean, sinv)
        ctx.relu, ctx.has_skip = int(relu), skip is not None
        # a skip input with a gradient sink (a ResNet block's input, also read
        # by the block's conv1): this backward runs before conv1's, so it writes
        # the sink first -- straight into its buffer, no add launch
        ctx.skipsink = _sink_of(skip) if skip is not None and skip.requires_grad else None
        ctx.affine = (weight is not None, bias is not None)
        return y

    @staticmethod
    def backward(ctx, gy):
        lib = _lib.load()
        x, y, weight, smean, sinv = ctx.saved_tensors
        N, C, H, W = x.shape
        gy = gy.contiguous()
        gx = torch.empty_like(x)
        gw = torch.empty(C, device=x.device, dtype=torch.float32) if ctx.affine[0] else None
        gb = torch.empty(C, device=x.device, dtype=torch.float32) if ctx.affine[1] else None
        gs = torch.empty_like(x) if ctx.has_skip and ctx.needs_input_grad[3] else None
        in_sink = gs is not None and ctx.skipsink is not None and not ctx.skipsink.written
        if in_sink:
            gs = ctx.skipsink.target()[0]
        nws = lib.dro_batchnorm_workspace_bytes(N, C, H * W)
        ws = torch.empty(max(nws, 16), device=x.device, dtype=torch.uint8)
        check(lib.dro_batchnorm_relu_backward(
            ptr(gy), ptr(x), ptr(y), ptr(weight), ptr(smean), ptr(sinv), ctx.relu, N, C, H * W,
            ptr(gx), ptr(gw), ptr(gb), ptr(gs), ptr(ws), nws, stream_of(gy)),
            "dro_batchnorm_relu_backward")
        return gx, gw, gb, (None if in_sink else gs), None, None, None, None, None, None


def batchnorm_act(x, bn, skip=None, relu=True):
    """act(bn(x) + skip) for a training-mode nn.BatchNorm2d `bn` (float32 NCHW):
    torch.nn.functional.batch_norm(training=True) semantics, including the
    running-statistics update and num_batches_tracked (reference
    networks/optim/extractor.py:7-107 via torchvision's BasicBlock)."""
    if x.dtype != torch.float32 or x.dim() != 4:
        raise RuntimeError("batchnorm_act: expects a float32 NCHW tensor")
    if bn.momentum is None:
        raise NotImplementedError("batchnorm_act: cumulative averaging (momentum=None)")
    track = bn.track_running_stats and bn.running_mean is not None
    return _BatchNormAct.apply(
        x, bn.weight, bn.bias, skip, bn.running_mean if track else None,
        bn.running_var if track else None, bn.num_batches_tracked if track else None,
        1 if relu else 0, bn.eps, bn.momentum)


# ------------------------------------------------------------------ depth evaluation metrics
def crop_rect(crop, H, W):
    """Crop rectangle (y1, y2, x1, x2) of compute_depth_metrics
    (dro_sfm/utils/depth.py:287-298): 'garg' (KITTI, fractions of the gt size,
    Python float products truncated by int()), 'eigen_nyu' (fixed), else none."""
    if crop == "garg":
        return (int(0.40810811 * H), int(0.99189189 * H), int(0.03594771 * W), int(0.96405229 * W))
    if crop == "eigen_nyu":
        return (20, 459, 24, 615)
    return (-1, -1, -1, -1)


def depth_metrics(gt, pred, min_depth, max_depth, crop="", use_gt_scale=True):
    """compute_depth_metrics (dro_sfm/utils/depth.py:259-343) on the GPU.

    gt [B,1,H,W], pred [B,1,h,w] depths (float32).  Returns a float32 tensor [9]:
    abs_rel, sq_rel, rmse, rmse_log, a1, a2, a3, SILog, iabs_diff (batch means).
    One prepare pass (upsample, validity, ratios), the per-image median of the
    valid gt/pred ratios by an on-device radix select (the reference's
    torch.median: the lower middle element), one reduce pass.  No host
    synchronisation (the reference synchronises per image)."""
    lib = _lib.load()
    require_device(gt, pred, what="depth_metrics")
    if gt.dim() != 4 or pred.dim() != 4 or gt.shape[1] != 1 or pred.shape[1] != 1 or gt.shape[0] != pred.shape[0]:
        raise RuntimeError("depth_metrics: gt [B,1,H,W] and pred [B,1,h,w] expected")
    B, _, H, W = gt.shape
    h, w = pred.shape[-2:]
    y1, y2, x1, x2 = crop_rect(crop, H, W)
    gt, pred = gt.contiguous(), pred.contiguous()
    nblk = lib.dro_depth_metrics_blocks(H, W)
    pred_up = torch.empty(B, H * W, device=gt.device, dtype=torch.float32)
    ratio = torch.empty_like(pred_up)
    counts = torch.empty(B, nblk, device=gt.device, dtype=torch.int32)
    st = stream_of(gt)
    check(lib.dro_depth_metrics_prepare(ptr(gt), ptr(pred), B, H, W, h, w, float(min_depth), float(max_depth),
                                        y1, y2, x1, x2, ptr(pred_up), ptr(ratio), ptr(counts), st),
          "dro_depth_metrics_prepare")
    scale = None
    if use_gt_scale:
        scale = torch.empty(B, device=gt.device, dtype=torch.float32)
        mws = torch.empty(lib.dro_depth_metrics_median_workspace_bytes(B) // 4 + 1, device=gt.device,
                          dtype=torch.int32)
        check(lib.dro_depth_metrics_median(ptr(ratio), ptr(counts), B, H, W, ptr(scale), ptr(mws), st),
              "dro_depth_metrics_median")
    ws = torch.empty(lib.dro_depth_metrics_workspace_bytes(B) // 8 + 1, device=gt.device, dtype=torch.float64)
    out = torch.empty(9, device=gt.device, dtype=torch.float32)
    check(lib.dro_depth_metrics_reduce(ptr(gt), ptr(pred_up), ptr(scale), B, H, W, float(min_depth),
                                       float(max_depth), y1, y2, x1, x2, ptr(out), ptr(ws), st),
          "dro_depth_metrics_reduce")
    return out


def depth_metrics_demon(gt, gt_pose, pred, min_depth, max_depth, use_gt_scale=True):
    """compute_depth_metrics_demon (dro_sfm/utils/depth.py:343-398) on the GPU.

    gt [B,1,H,W], pred [B,1,h,w] depths; gt_pose [B,N,3|4,4] ground-truth
    transforms (image b's FIRST reference normalises its ground truth when
    use_gt_scale).  Returns float32 [9] like depth_metrics.  Same three passes
    (prepare, on-device median, reduce), no crop, no clamp of the scaled
    prediction to the depth range."""
    lib = _lib.load()
    require_device(gt, pred, gt_pose, what="depth_metrics_demon")
    if gt.dim() != 4 or pred.dim() != 4 or gt.shape[1] != 1 or pred.shape[1] != 1 or gt.shape[0] != pred.shape[0]:
        raise RuntimeError("depth_metrics_demon: gt [B,1,H,W] and pred [B,1,h,w] expected")
    B, _, H, W = gt.shape
    if gt_pose.dim() != 4 or gt_pose.shape[0] != B or gt_pose.shape[-1] != 4 or gt_pose.shape[-2] not in (3, 4):
        raise RuntimeError("depth_metrics_demon: gt_pose [B,N,3|4,4] expected")
    h, w = pred.shape[-2:]
    gt, pred = gt.contiguous(), pred.contiguous()
    first = gt_pose[:, 0].float().contiguous()                 # [B,3|4,4]
    pose_stride = first.shape[1] * 4
    nblk = lib.dro_depth_metrics_blocks(H, W)
    pred_up = torch.empty(B, H * W, device=gt.device, dtype=torch.float32)
    ratio = torch.empty_like(pred_up)
    counts = torch.empty(B, nblk, device=gt.device, dtype=torch.int32)
    st = stream_of(gt)
    pose_p = ptr(first) if use_gt_scale else None
    check(lib.dro_depth_metrics_demon_prepare(ptr(gt), ptr(pred), pose_p, pose_stride, B, H, W, h, w,
                                              float(min_depth), float(max_depth), ptr(pred_up), ptr(ratio),
                                              ptr(counts), st), "dro_depth_metrics_demon_prepare")
    scale = None
    if use_gt_scale:
        scale = torch.empty(B, device=gt.device, dtype=torch.float32)
        mws = torch.empty(lib.dro_depth_metrics_median_workspace_bytes(B) // 4 + 1, device=gt.device,
                          dtype=torch.int32)
        check(lib.dro_depth_metrics_median(ptr(ratio), ptr(counts), B, H, W, ptr(scale), ptr(mws), st),
              "dro_depth_metrics_median")
    ws = torch.empty(lib.dro_depth_metrics_workspace_bytes(B) // 8 + 1, device=gt.device, dtype=torch.float64)
    out = torch.empty(9, device=gt.device, dtype=torch.float32)
    check(lib.dro_depth_metrics_demon_reduce(ptr(gt), ptr(pred_up), ptr(scale), pose_p, pose_stride, B, H, W,
                                             float(min_depth), float(max_depth), ptr(out), ptr(ws), st),
          "dro_depth_metrics_demon_reduce")
    return out


