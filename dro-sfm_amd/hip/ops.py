"""torch.autograd.Function wrappers over the C ABI of libdro_amd.so.

Each Function checks dtype/device/shape up front (RuntimeError, as the
reference's ATen ops would raise), allocates outputs through the caching
allocator, and launches on the current stream.
"""
import contextlib
import ctypes

import torch

from . import _lib
from ._lib import check, ptr, require_device, stream_of

POSE_EULER, POSE_MATRIX = 0, 1
DEPTH_METRIC, DEPTH_INV, DEPTH_DISP = 0, 1, 2


def _pose_layout(pose, lead):
    """Return (flat pose [*lead, 6|12] contiguous, mode, restore-fn for its grad)."""
    if pose.shape[-1] == 6 and pose.dim() == len(lead) + 1:
        return pose.contiguous(), POSE_EULER, lambda g: g
    if pose.shape[-2:] in ((3, 4), (4, 4)) and pose.dim() == len(lead) + 2:
        rows = pose.shape[-2]
        flat = pose[..., :3, :].contiguous().view(*lead, 12)

        def restore(g):
            g = g.view(*lead, 3, 4)
            if rows == 4:
                g = torch.cat([g, g.new_zeros(*lead, 1, 4)], dim=-2)
            return g
        return flat, POSE_MATRIX, restore
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
        self.buf = torch.empty(like.shape, device=like.device, dtype=like.dtype)
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
    if not x.is_contiguous() and x.dim() != 4:
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

    def new(self, tag, shape, device):
        cells = torch.full(shape, -1, dtype=torch.int32, device=device)
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


def _cell_map(tag, shape, device):
    rec = _CELLS[0]
    return rec.new(tag, shape, device) if rec is not None and torch.is_grad_enabled() else None


class _WarpCost(torch.autograd.Function):
    @staticmethod
    def forward(ctx, fmap, fmap_ref, depth, pose, K, ref_K, depth_mode, min_disp, max_disp, scale,
                reduce_mean, tag):
        lib = _lib.load()
        require_device(fmap, fmap_ref, depth, K, ref_K, what="warp_cost")
        B, C, h, w = fmap.shape
        N = fmap_ref.shape[0]
        if fmap_ref.shape != (N, B, C, h, w) or depth.shape != (B, 1, h, w) or K.shape != (B, 3, 3):
            raise RuntimeError("warp_cost: shape mismatch (fmap [B,C,h,w], fmap_ref [N,B,C,h,w], "
                               "depth [B,1,h,w], K [B,3,3])")
        pose_flat, pose_mode, restore = _pose_layout(pose, (N, B))
        require_device(pose_flat, what="warp_cost")
        sinks = (_sink_of(fmap), _sink_of(fmap_ref))
        fmap, fmap_ref, depth = fmap.contiguous(), fmap_ref.contiguous(), depth.contiguous()
        K, ref_K = K.contiguous(), ref_K.contiguous()
        out_shape = (B, C, h, w) if reduce_mean else (N, B, C, h, w)
        cost = torch.empty(out_shape, device=fmap.device, dtype=torch.float32)
        check(lib.dro_warp_cost_forward(ptr(fmap), ptr(fmap_ref), ptr(depth), depth_mode,
                                        min_disp, max_disp, ptr(K), ptr(ref_K), scale,
                                        ptr(pose_flat), pose_mode, B, N, C, h, w, int(reduce_mean),
                                        ptr(cost), stream_of(fmap)), "dro_warp_cost_forward")
        ctx.save_for_backward(fmap, fmap_ref, depth, pose_flat, K, ref_K)
        ctx.sinks = sinks
        ctx.cfg = (depth_mode, min_disp, max_disp, scale, pose_mode, int(reduce_mean))
        ctx.restore = restore
        ctx.cells = _cell_map(tag, (N, B, h, w), fmap.device)
        return cost

    @staticmethod
    def backward(ctx, gcost):
        lib = _lib.load()
        fmap, fmap_ref, depth, pose_flat, K, ref_K = ctx.saved_tensors
        depth_mode, min_disp, max_disp, scale, pose_mode, reduce_mean = ctx.cfg
        B, C, h, w = fmap.shape
        N = fmap_ref.shape[0]
        need = ctx.needs_input_grad
        gcost = gcost.contiguous()
        # feature maps shared by all cost calls of a step: summed in their sinks
        sf, sr = ctx.sinks
        sf = sf if need[0] else None
        sr = sr if need[1] else None
        accumulate = 0
        if sf is not None:
            g_f, af = sf.target()
            accumulate |= af
        else:
            g_f = torch.empty_like(fmap) if need[0] else None
        if sr is not None:
            g_r, ar = sr.target()
            accumulate |= 2 * ar
        else:
            g_r = torch.empty_like(fmap_ref) if need[1] else None
        g_d = torch.empty_like(depth) if need[2] else None
        g_p = torch.empty_like(pose_flat) if need[3] else None
        ws = None
        if g_d is not None or g_p is not None or ctx.cells is not None:
            nbytes = lib.dro_warp_cost_workspace_bytes(B, N, h, w)
            ws = torch.empty(nbytes // 4 + 1, device=fmap.device, dtype=torch.float32)
        check(lib.dro_warp_cost_backward(ptr(fmap), ptr(fmap_ref), ptr(depth), depth_mode,
                                         min_disp, max_disp, ptr(K), ptr(ref_K), scale,
                                         ptr(pose_flat), pose_mode, B, N, C, h, w, reduce_mean,
                                         ptr(gcost), ptr(g_f), ptr(g_r), ptr(g_d), ptr(g_p),
                                         accumulate, ptr(ws), ptr(ctx.cells), stream_of(fmap)),
              "dro_warp_cost_backward")
        if g_p is not None:
            g_p = ctx.restore(g_p)
        if sf is not None:
            g_f = None
        if sr is not None:
            g_r = None
        return g_f, g_r, g_d, g_p, None, None, None, None, None, None, None, None


def warp_cost(fmap, fmap_ref, depth, pose, K, ref_K=None, *, depth_mode=DEPTH_METRIC,
              min_depth=None, max_depth=None, scale=1.0 / 8, reduce_mean=True, tag=None):
    """Fused get_cost_each / depth_cost_calc (DepthPoseNet.py:76-105).

    fmap [B,C,h,w]; fmap_ref [N,B,C,h,w]; depth [B,1,h,w] encoded per depth_mode
    (DEPTH_DISP applies disp_to_depth(min_depth, max_depth) then inv2depth);
    pose [N,B,6] euler vectors or [N,B,3|4,4] matrices; K/ref_K full-res [B,3,3].
    Returns the mean cost over refs [B,C,h,w] (reduce_mean) or [N,B,C,h,w].
    `tag` names the call in a record_bilinear_cells() record (tests).
    """
    if fmap_ref.dim() == 4:
        fmap_ref = fmap_ref.unsqueeze(0)
        pose = pose.unsqueeze(0)
    min_disp, max_disp = _disp_range(min_depth, max_depth)
    if depth_mode == DEPTH_DISP and (min_depth is None or max_depth is None):
        raise RuntimeError("warp_cost: DEPTH_DISP needs min_depth and max_depth")
    return _WarpCost.apply(fmap, fmap_ref, depth, pose, K, K if ref_K is None else ref_K,
                           depth_mode, float(min_disp), float(max_disp), float(scale), reduce_mean, tag)


class _ViewSynthesis(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ref_image, depth, pose, K, ref_K, depth_mode, min_disp, max_disp, scale):
        lib = _lib.load()
        require_device(ref_image, depth, K, ref_K, what="view_synthesis")
        N, B, C, H, W = ref_image.shape
        if depth.shape != (B, 1, H, W) or K.shape != (B, 3, 3) or ref_K.shape != (B, 3, 3):
            raise RuntimeError("view_synthesis: ref_image [N,B,C,H,W], depth [B,1,H,W], K/ref_K [B,3,3]")
        pose_flat, pose_mode, restore = _pose_layout(pose, (N, B))
        require_device(pose_flat, what="view_synthesis")
        ref_image, depth, K, ref_K = ref_image.contiguous(), depth.contiguous(), K.contiguous(), ref_K.contiguous()
        warped = torch.empty_like(ref_image)
        check(lib.dro_view_synthesis_forward(ptr(ref_image), ptr(depth), depth_mode, min_disp, max_disp, ptr(K),
                                             ptr(ref_K), scale, ptr(pose_flat), pose_mode, B, N, C, H, W,
                                             ptr(warped), stream_of(ref_image)), "dro_view_synthesis_forward")
        ctx.save_for_backward(ref_image, depth, pose_flat, K, ref_K)
        ctx.cfg = (depth_mode, min_disp, max_disp, scale, pose_mode)
        ctx.restore = restore
        ctx.cells = _cell_map("view_synthesis", (N, B, H, W), ref_image.device)
        return warped

    @staticmethod
    def backward(ctx, gw):
        lib = _lib.load()
        ref_image, depth, pose_flat, K, ref_K = ctx.saved_tensors
        depth_mode, min_disp, max_disp, scale, pose_mode = ctx.cfg
        N, B, C, H, W = ref_image.shape
        need = ctx.needs_input_grad
        g_r = torch.empty_like(ref_image) if need[0] else None
        g_d = torch.empty_like(depth) if need[1] else None
        g_p = torch.empty_like(pose_flat) if need[2] else None
        ws = torch.empty(lib.dro_warp_cost_workspace_bytes(B, N, H, W) // 4 + 1, device=depth.device)
        check(lib.dro_view_synthesis_backward(ptr(ref_image), ptr(depth), depth_mode, min_disp, max_disp, ptr(K),
                                              ptr(ref_K), scale, ptr(pose_flat), pose_mode, B, N, C, H, W,
                                              ptr(gw.contiguous()), ptr(g_r), ptr(g_d), ptr(g_p), ptr(ws),
                                              ptr(ctx.cells), stream_of(depth)), "dro_view_synthesis_backward")
        return g_r, g_d, (ctx.restore(g_p) if g_p is not None else None), None, None, None, None, None, None


def view_synthesis(ref_image, depth, pose, K, ref_K=None, *, depth_mode=DEPTH_METRIC, min_depth=None,
                   max_depth=None, scale=1.0):
    """view_synthesis (geometry/camera_utils.py:23-56) of N reference images in one
    launch: ref_image [N,B,C,H,W] (or [B,C,H,W] for one view), depth [B,1,H,W]
    in `depth_mode`, pose [N,B,6] euler vectors or [N,B,3|4,4] matrices (target
    -> reference, Camera(ref_K, Tcw=pose)), K/ref_K [B,3,3] scaled by `scale`
    (scale_intrinsics).  Returns the warped references, same shape as ref_image.
    The kernels are the cost's (warp_cost_fwd/bwd_feat/bwd_geo in SAMPLE mode)."""
    single = ref_image.dim() == 4
    if single:
        ref_image, pose = ref_image.unsqueeze(0), pose.unsqueeze(0)
    if depth_mode == DEPTH_DISP and (min_depth is None or max_depth is None):
        raise RuntimeError("view_synthesis: DEPTH_DISP needs min_depth and max_depth")
    min_disp, max_disp = _disp_range(min_depth, max_depth)
    out = _ViewSynthesis.apply(ref_image, depth, pose, K, K if ref_K is None else ref_K, depth_mode,
                               float(min_disp), float(max_disp), float(scale))
    return out[0] if single else out


def plane_sweep_cost(fmap, fmap_ref, disp, pose, K, ref_K=None, *, min_depth, max_depth,
                     scale=1.0 / 8):
    """Cost of D fronto-parallel planes (disp [D] in sigmoid space): [B,D,C,h,w]."""
    lib = _lib.load()
    require_device(fmap, fmap_ref, disp, K, what="plane_sweep_cost")
    B, C, h, w = fmap.shape
    D = disp.numel()
    pose_flat, pose_mode, _ = _pose_layout(pose, (B,))
    ref_K = K if ref_K is None else ref_K
    min_disp, max_disp = _disp_range(min_depth, max_depth)
    fmap, fmap_ref, disp = fmap.contiguous(), fmap_ref.contiguous(), disp.contiguous()
    K, ref_K = K.contiguous(), ref_K.contiguous()
    cost = torch.empty(B, D, C, h, w, device=fmap.device, dtype=torch.float32)
    check(lib.dro_plane_sweep_forward(ptr(fmap), ptr(fmap_ref), ptr(disp), D, float(min_disp),
                                      float(max_disp), ptr(K), ptr(ref_K), float(scale),
                                      ptr(pose_flat), pose_mode, B, C, h, w, ptr(cost),
                                      stream_of(fmap)), "dro_plane_sweep_forward")
    return cost


# ------------------------------------------------------------------------- photometric loss
class _Photometric(torch.autograd.Function):
    @staticmethod
    def forward(ctx, image, context, inv_depths, pose, K, ref_K, opts):
        lib = _lib.load()
        require_device(image, context, inv_depths, K, ref_K, what="photometric_loss")
        n, B, _, H, W = inv_depths.shape
        N = context.shape[0]
        if image.shape != (B, 3, H, W) or context.shape != (N, B, 3, H, W):
            raise RuntimeError("photometric_loss: image [B,3,H,W], context [N,B,3,H,W] and "
                               "inv_depths [n,B,1,H,W] must share B,H,W (full-res predictions)")
        pose_flat, pose_mode, restore = _pose_layout(pose, (N, n, B))
        ssim_w, C1, C2, smooth_w, automask, reduce_min = opts
        image, context, inv_depths = image.contiguous(), context.contiguous(), inv_depths.contiguous()
        K, ref_K = K.contiguous(), ref_K.contiguous()
        nbytes = lib.dro_photometric_workspace_bytes(B, N, n, H, W)
        ws = torch.empty(nbytes, device=image.device, dtype=torch.uint8)
        out = torch.empty(3, device=image.device, dtype=torch.float32)
        check(lib.dro_photometric_forward(ptr(image), ptr(context), ptr(inv_depths), ptr(K),
                                          ptr(ref_K), ptr(pose_flat), pose_mode, B, N, n, H, W,
                                          ssim_w, C1, C2, smooth_w, automask, reduce_min,
                                          ptr(out), ptr(ws), stream_of(image)),
              "dro_photometric_forward")
        ctx.save_for_backward(image, context, inv_depths, pose_flat, K, ref_K, ws)
        ctx.cfg = (pose_mode, opts)
        ctx.restore = restore
        ctx.cells = _cell_map("photo", (N, n, B, H, W), image.device)
        metrics = out[1:].detach()
        # per-pixel argmin over the candidate maps (uint8 [n,B,H,W], the first
        # region of the workspace); exposed for parity tests
        sel = ws[:n * B * H * W].view(n, B, H, W)
        ctx.mark_non_differentiable(metrics, sel)
        return out[0:1], metrics, sel

    @staticmethod
    def backward(ctx, gloss, _gmetrics, _gsel):
        lib = _lib.load()
        image, context, inv_depths, pose_flat, K, ref_K, ws = ctx.saved_tensors
        pose_mode, (ssim_w, C1, C2, smooth_w, automask, reduce_min) = ctx.cfg
        n, B, _, H, W = inv_depths.shape
        N = context.shape[0]
        gloss = gloss.contiguous()
        g_inv = torch.empty_like(inv_depths)
        g_pose = torch.empty_like(pose_flat) if ctx.needs_input_grad[3] else None
        check(lib.dro_photometric_backward(ptr(image), ptr(context), ptr(inv_depths), ptr(K),
                                           ptr(ref_K), ptr(pose_flat), pose_mode, B, N, n, H, W,
                                           ssim_w, C1, C2, smooth_w, automask, reduce_min,
                                           ptr(gloss), ptr(g_inv), ptr(g_pose), ptr(ws), ptr(ctx.cells),
                                           stream_of(image)), "dro_photometric_backward")
        if g_pose is not None:
            g_pose = ctx.restore(g_pose)
        return None, None, g_inv if ctx.needs_input_grad[2] else None, g_pose, None, None, None


def photometric_loss(image, context, inv_depths, pose, K, ref_K=None, *, ssim_w=0.85, C1=1e-4,
                     C2=9e-4, smooth_w=0.001, automask=True, reduce_min=True,
                     return_selection=False):
    """Fused MultiViewPhotometricDecayLoss (multiview_photometric_loss_mf.py:303-361).

    image [B,3,H,W]; context [N,B,3,H,W]; inv_depths [n,B,1,H,W];
    pose [N,n,B,6] euler vectors or [N,n,B,3|4,4] matrices.
    Returns (loss [1], detached metrics [2] = (photometric_loss, smoothness_loss))
    and, with return_selection, the per-pixel min-candidate index uint8 [n,B,H,W]
    (candidate order of the reference's torch.cat: warped_0, unwarped_0, ...).
    """
    opts = (float(ssim_w), float(C1), float(C2), float(smooth_w), int(bool(automask)),
            int(bool(reduce_min)))
    loss, metrics, sel = _Photometric.apply(image, context, inv_depths, pose, K,
                                            K if ref_K is None else ref_K, opts)
    return (loss, metrics, sel) if return_selection else (loss, metrics)


# ------------------------------------------------------------------------- supervised loss
class _Supervised(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gt_inv, inv_depths, pose, gt_pose, K, ref_K, min_depth, max_depth):
        lib = _lib.load()
        require_device(gt_inv, inv_depths, gt_pose, K, ref_K, what="supervised_loss")
        n, B, _, H, W = inv_depths.shape
        N = gt_pose.shape[0]
        if gt_inv.shape != (B, 1, H, W) or K.shape != (B, 3, 3) or ref_K.shape != (B, 3, 3):
            raise RuntimeError("supervised_loss: gt_inv [B,1,H,W] and inv_depths [n,B,1,H,W] must "
                               "share B,H,W; K/ref_K [B,3,3]")
        pose_flat, pose_mode, restore = _pose_layout(pose, (N, n, B))
        gt_flat, gt_mode, _ = _pose_layout(gt_pose, (N, B))
        if gt_mode != POSE_MATRIX:
            raise RuntimeError("supervised_loss: gt_pose must be [N,B,3|4,4] matrices")
        require_device(pose_flat, what="supervised_loss")
        gt_inv, inv_depths = gt_inv.contiguous(), inv_depths.contiguous()
        K, ref_K = K.contiguous(), ref_K.contiguous()
        ws = torch.empty(lib.dro_supervised_workspace_bytes(B, N, n, H, W) // 4 + 1,
                         device=gt_inv.device, dtype=torch.float32)
        out = torch.empty(3, device=gt_inv.device, dtype=torch.float32)
        check(lib.dro_supervised_forward(ptr(gt_inv), ptr(inv_depths), ptr(K), ptr(ref_K),
                                         ptr(gt_flat), ptr(pose_flat), pose_mode, B, N, n, H, W,
                                         min_depth, max_depth, ptr(out), ptr(ws),
                                         stream_of(gt_inv)), "dro_supervised_forward")
        ctx.save_for_backward(gt_inv, inv_depths, pose_flat, gt_flat, K, ref_K)
        ctx.cfg = (pose_mode, min_depth, max_depth)
        ctx.restore = restore
        metrics = out[1:].detach()
        ctx.mark_non_differentiable(metrics)
        return out[0:1], metrics

    @staticmethod
    def backward(ctx, gloss, _gmetrics):
        lib = _lib.load()
        gt_inv, inv_depths, pose_flat, gt_flat, K, ref_K = ctx.saved_tensors
        pose_mode, min_depth, max_depth = ctx.cfg
        n, B, _, H, W = inv_depths.shape
        N = gt_flat.shape[0]
        gloss = gloss.contiguous()
        g_inv = torch.empty_like(inv_depths)
        g_pose = torch.empty_like(pose_flat)
        ws = torch.empty(lib.dro_supervised_workspace_bytes(B, N, n, H, W) // 4 + 1,
                         device=gt_inv.device, dtype=torch.float32)
        check(lib.dro_supervised_backward(ptr(gt_inv), ptr(inv_depths), ptr(K), ptr(ref_K),
                                          ptr(gt_flat), ptr(pose_flat), pose_mode, B, N, n, H, W,
                                          min_depth, max_depth, ptr(gloss), ptr(g_inv),
                                          ptr(g_pose), ptr(ws), stream_of(gt_inv)),
              "dro_supervised_backward")
        need = ctx.needs_input_grad
        return (None, g_inv if need[1] else None, ctx.restore(g_pose) if need[2] else None,
                None, None, None, None, None)


def supervised_loss(gt_inv, inv_depths, pose, gt_pose, K, ref_K=None, *, min_depth, max_depth):
    """Fused SupervisedDepthPoseLoss (supervised_loss.py:343-371, 'sparse-l1').

    gt_inv [B,1,H,W]; inv_depths [n,B,1,H,W]; pose [N,n,B,6] euler vectors or
    [N,n,B,3|4,4] matrices; gt_pose [N,B,3|4,4].  Returns (loss [1], detached
    metrics [2] = (depth_loss, pose_loss)).
    """
    return _Supervised.apply(gt_inv, inv_depths, pose, gt_pose, K, K if ref_K is None else ref_K,
                             float(min_depth), float(max_depth))


# ------------------------------------------------------------------------- convex upsample
class _ConvexUpsample(torch.autograd.Function):
    @staticmethod
    def forward(ctx, inv, mask, ratio, add, mul):
        lib = _lib.load()
        require_device(inv, mask, what="convex_upsample")
        B, _, h, w = inv.shape
        if mask.shape != (B, 9 * ratio * ratio, h, w):
            raise RuntimeError("convex_upsample: mask must be [B, 9*r*r, h, w]")
        inv, mask = inv.contiguous(), mask.contiguous()
        out = torch.empty(B, 1, h * ratio, w * ratio, device=inv.device, dtype=torch.float32)
        check(lib.dro_convex_upsample_forward(ptr(inv), ptr(mask), B, h, w, ratio, ctypes.c_float(add),
                                              ctypes.c_float(mul), ptr(out), stream_of(inv)),
              "dro_convex_upsample_forward")
        ctx.save_for_backward(inv, mask)
        ctx.ratio, ctx.mul = ratio, mul
        return out

    @staticmethod
    def backward(ctx, gout):
        lib = _lib.load()
        inv, mask = ctx.saved_tensors
        B, _, h, w = inv.shape
        g_inv = torch.empty_like(inv) if ctx.needs_input_grad[0] else None
        g_mask = torch.empty_like(mask)
        check(lib.dro_convex_upsample_backward(ptr(inv), ptr(mask), ptr(gout.contiguous()), B, h, w,
                                               ctx.ratio, ctypes.c_float(ctx.mul), ptr(g_inv), ptr(g_mask),
                                               stream_of(inv)), "dro_convex_upsample_backward")
        return g_inv, g_mask if ctx.needs_input_grad[1] else None, None, None, None


def convex_upsample(inv, mask, ratio=8, affine=None):
    """DepthPoseNet.upsample_depth (DepthPoseNet.py:63-74): [B,1,h,w] -> [B,1,rh,rw];
    affine=(add, mul) folds `add + mul * out` (scale_inv_depth) into the kernel."""
    add, mul = affine if affine is not None else (0.0, 1.0)
    return _ConvexUpsample.apply(inv, mask, int(ratio), float(add), float(mul))


def _ptr_table(ts):
    arr = (ctypes.c_void_p * len(ts))()
    for i, t in enumerate(ts):
        arr[i] = t.data_ptr() if t is not None else None
    return arr


class _ConvexUpsampleMany(torch.autograd.Function):
    """n convex upsamples in one launch each way -> [n, B, 1, rh, rw]."""

    @staticmethod
    def forward(ctx, ratio, add, mul, n, *tensors):
        lib = _lib.load()
        invs = [t.contiguous() for t in tensors[:n]]
        masks = [t.contiguous() for t in tensors[n:]]
        require_device(*invs, *masks, what="convex_upsample_many")
        B, _, h, w = invs[0].shape
        for i, m in zip(invs, masks):
            if i.shape != (B, 1, h, w) or m.shape != (B, 9 * ratio * ratio, h, w):
                raise RuntimeError("convex_upsample_many: every inv must be [B,1,h,w] and mask [B,9*r*r,h,w]")
        out = torch.empty(n, B, 1, h * ratio, w * ratio, device=invs[0].device, dtype=torch.float32)
        check(lib.dro_convex_upsample_many_forward(_ptr_table(invs), _ptr_table(masks), n, B, h, w, ratio,
                                                   ctypes.c_float(add), ctypes.c_float(mul), ptr(out),
                                                   stream_of(out)), "dro_convex_upsample_many_forward")
        ctx.save_for_backward(*invs, *masks)
        ctx.n, ctx.ratio, ctx.mul = n, ratio, mul
        return out

    @staticmethod
    def backward(ctx, gout):
        lib = _lib.load()
        n = ctx.n
        saved = ctx.saved_tensors
        invs, masks = saved[:n], saved[n:]
        B, _, h, w = invs[0].shape
        g_inv = [torch.empty_like(t) if ctx.needs_input_grad[4 + i] else None for i, t in enumerate(invs)]
        g_mask = [torch.empty_like(m) for m in masks]
        nb = int(lib.dro_convex_upsample_many_workspace_bytes(n, B, h, w))
        ws = torch.empty(nb, dtype=torch.uint8, device=gout.device)
        check(lib.dro_convex_upsample_many_backward(_ptr_table(invs), _ptr_table(masks), ptr(gout.contiguous()),
                                                    n, B, h, w, ctx.ratio, ctypes.c_float(ctx.mul),
                                                    _ptr_table(g_inv), _ptr_table(g_mask), ptr(ws), nb,
                                                    stream_of(gout)), "dro_convex_upsample_many_backward")
        g_mask = [g if ctx.needs_input_grad[4 + n + i] else None for i, g in enumerate(g_mask)]
        return (None, None, None, None, *g_inv, *g_mask)


def convex_upsample_many(invs, masks, ratio=8, affine=None):
    """convex_upsample of n (inv, mask) pairs in one launch each way: returns the
    stacked [n, B, 1, rh, rw] (the losses read the predictions stacked;
    stacked_view() recovers it from its unbind() views).  Deterministic
    backward (no atomics)."""
    if not 1 <= len(invs) == len(masks) <= 32:
        raise RuntimeError("convex_upsample_many: 1..32 (inv, mask) pairs")
    add, mul = affine if affine is not None else (0.0, 1.0)
    return _ConvexUpsampleMany.apply(int(ratio), float(add), float(mul), len(invs), *invs, *masks)


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
class _Bilinear2x(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        lib = _lib.load()
        require_device(x, what="bilinear_upsample2x")
        N, C, h, w = x.shape
        x = x.contiguous()
        out = torch.empty(N, C, 2 * h, 2 * w, device=x.device, dtype=torch.float32)
        check(lib.dro_bilinear_upsample2x_forward(ptr(x), N * C, h, w, ptr(out), stream_of(x)),
              "dro_bilinear_upsample2x_forward")
        ctx.shape = (N, C, h, w)
        return out

    @staticmethod
    def backward(ctx, gout):
        lib = _lib.load()
        N, C, h, w = ctx.shape
        gout = gout.contiguous()
        gx = torch.empty(N, C, h, w, device=gout.device, dtype=torch.float32)
        check(lib.dro_bilinear_upsample2x_backward(ptr(gout), N * C, h, w, ptr(gx), stream_of(gout)),
              "dro_bilinear_upsample2x_backward")
        return gx


def bilinear_upsample2x(x):
    """F.interpolate(x, scale_factor=2, mode="bilinear", align_corners=False) for float32
    NCHW (reference networks/optim/extractor.py:91-97); deterministic backward."""
    if x.dtype != torch.float32 or x.dim() != 4:
        raise RuntimeError("bilinear_upsample2x: expects a float32 NCHW tensor")
    return _Bilinear2x.apply(x)


# ------------------------------------------------------------------ ResNet stem max pooling
class _MaxPool3s2(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        lib = _lib.load()
        require_device(x, what="maxpool3x3s2")
        N, C, H, W = x.shape
        Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
        x = x.contiguous()
        y = torch.empty(N, C, Ho, Wo, device=x.device, dtype=torch.float32)
        arg = torch.empty(N, C, Ho, Wo, device=x.device, dtype=torch.uint8)
        check(lib.dro_maxpool3x3s2_forward(ptr(x), N * C, H, W, ptr(y), ptr(arg), stream_of(x)),
              "dro_maxpool3x3s2_forward")
        ctx.save_for_backward(arg)
        ctx.shape = (N, C, H, W)
        ctx.mark_non_differentiable(arg)
        return y

    @staticmethod
    def backward(ctx, gy):
        lib = _lib.load()
        (arg,) = ctx.saved_tensors
        N, C, H, W = ctx.shape
        gy = gy.contiguous()
        gx = torch.empty(N, C, H, W, device=gy.device, dtype=torch.float32)
        check(lib.dro_maxpool3x3s2_backward(ptr(gy), ptr(arg), N * C, H, W, ptr(gx), stream_of(gy)),
              "dro_maxpool3x3s2_backward")
        return gx


def maxpool3x3s2(x):
    """F.max_pool2d(x, 3, 2, 1) for float32 NCHW on the GPU (ResNet stem,
    reference networks/optim/extractor.py:60-66); bit-identical forward and
    backward, one argmax byte per output instead of int64 indices."""
    if x.dtype != torch.float32 or x.dim() != 4:
        raise RuntimeError("maxpool3x3s2: expects a float32 NCHW tensor")
    return _MaxPool3s2.apply(x)


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


class _PoseMean(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, pose, rot_scale):
        lib = _lib.load()
        require_device(y, pose, what="pose_mean")
        B, C, H, W = y.shape
        y = y.contiguous()
        p = pose.contiguous() if pose is not None else None
        out = torch.empty(B, C, device=y.device, dtype=torch.float32)
        check(lib.dro_pose_mean_forward(ptr(y), ptr(p), ptr(out), B, C, H * W, float(rot_scale), stream_of(y)),
              "dro_pose_mean_forward")
        ctx.meta = (B, C, H, W, float(rot_scale), pose is not None)
        return out

    @staticmethod
    def backward(ctx, gout):
        lib = _lib.load()
        B, C, H, W, rs, has_pose = ctx.meta
        gout = gout.contiguous()
        gy = torch.empty(B, C, H, W, device=gout.device, dtype=torch.float32)
        check(lib.dro_pose_mean_backward(ptr(gout), ptr(gy), B, C, H * W, rs, stream_of(gout)),
              "dro_pose_mean_backward")
        return gy, (gout if has_pose and ctx.needs_input_grad[1] else None), None


def pose_mean(y, rot_scale=0.01, pose=None):
    """PoseHead's output (update.py:16-28) -- y.mean((2, 3)) with the rotation
    channels (3..5) scaled by rot_scale -- plus `pose` when given (the update
    `pose + pose_head(net)`, update.py:189-197): one launch forward, one
    backward.  y [B, C, H, W], pose [B, C]."""
    return _PoseMean.apply(y, pose, rot_scale)


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
        nws = lib.dro_batchnorm_workspace_bytes(N, C, H * W)
        ws = torch.empty(max(nws, 16), device=x.device, dtype=torch.uint8)
        check(lib.dro_batchnorm_relu_backward(
            ptr(gy), ptr(x), ptr(y), ptr(weight), ptr(smean), ptr(sinv), ctx.relu, N, C, H * W,
            ptr(gx), ptr(gw), ptr(gb), ptr(gs), ptr(ws), nws, stream_of(gy)),
            "dro_batchnorm_relu_backward")
        return gx, gw, gb, gs, None, None, None, None, None, None


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
