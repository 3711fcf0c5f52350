"""Training-mode BatchNorm fused into the encoders' 3x3 stride-1 convolutions
(csrc/conv.hip BnFuse; include/dro_amd.h ABI 10).

The reference's BasicBlock (dro_sfm/networks/optim/extractor.py:67-107, via
torchvision's ResNet-18) runs conv1 -> bn1 -> relu -> conv2 -> bn2 (+ skip)
-> relu.  hip.batchnorm_act ran every BN site as its own launches (statistics
+ apply forward, reduce + apply backward: 1-2 each way).  Here, at the sites a
3x3 stride-1 halo conv produces:

  conv_bn_stats(x, conv, bn)            z = conv(x); the conv's epilogue takes
                                        bn's batch statistics of z (per pixel
                                        tile, folded by the last block: no
                                        statistics launch)
  bn_relu_conv_stats(z1, bn1, conv2, bn2)
                                        z2 = conv2(relu(bn1(z1))): conv2 stages
                                        the BN + ReLU of z1 from the statistics
                                        and stores y1 = relu(bn1(z1)) once per
                                        pixel (no apply launch); its epilogue
                                        takes bn2's statistics of z2
  bn_apply(z2, bn2, skip)               relu(bn2(z2) + skip) from the
                                        statistics conv2 left: one launch
                                        (statistics + apply before)

Backward of the inner site (bn1): conv2's data gradient takes g1 = dy1 [y1 >
0] and the BN backward's sums of g1 and g1 xhat in its epilogue (no reduce
launch) and hands g1 on as "the gradient of z1"; conv1's data gradient stages
dz1 = k (g1 - mean(g1) - xhat mean(g1 xhat)) and stores it for conv1's weight
gradient (no apply launch).  bn2's backward stays dro_batchnorm_relu_backward.

Each BN module keeps one pair of states per activation geometry (zero-filled
once; the kernels reset their counters), so a module must not run twice
concurrently -- the encoders run each module once per step.
"""
import ctypes
import os

import torch

from . import _lib
from ._lib import check, ptr, require_device, stream_of
from .ops import _sink_of, record_branch
from .conv import _workspace, _direct_targets, _queue_weight_grad, _conv_bwd, _grad_buffers, current_scope

# "large" (default): fused where a channel holds more than 16 K elements
# (B*H*W > 16384: there hip.batchnorm_act takes two launches each way; below
# it one, and the fused path's finalize launch and epilogue cost as much --
# measured); "all": every 3x3 stride-1 site; "0": never
_MODE = [{"0": "0", "1": "large", "large": "large", "all": "all"}.get(os.environ.get("DRO_BN_FUSION", "large"),
                                                                      "large")]
_LARGE = 16384


def set_bn_fusion(mode):
    """True / "large" (default), "all" or False: which BN sites run inside the
    3x3 stride-1 convs (A/B runs; DRO_BN_FUSION=0|large|all at start-up)."""
    _MODE[0] = "large" if mode is True else ("0" if mode is False else str(mode))


def bn_fusion_enabled():
    return _MODE[0] != "0"


class DroBnParams(ctypes.Structure):
    _fields_ = [("gamma", ctypes.c_void_p), ("beta", ctypes.c_void_p), ("running_mean", ctypes.c_void_p),
                ("running_var", ctypes.c_void_p), ("num_batches_tracked", ctypes.c_void_p),
                ("eps", ctypes.c_float), ("momentum", ctypes.c_float),
                ("save_mean", ctypes.c_void_p), ("save_invstd", ctypes.c_void_p)]


class DroBnGradParams(ctypes.Structure):
    _fields_ = [("y", ctypes.c_void_p), ("z", ctypes.c_void_p), ("gamma", ctypes.c_void_p),
                ("save_mean", ctypes.c_void_p), ("save_invstd", ctypes.c_void_p),
                ("grad_gamma", ctypes.c_void_p), ("grad_beta", ctypes.c_void_p)]


def _p(t):
    return t.data_ptr() if t is not None else None


class BnSite:
    """A BN module's fused-path states for one activation geometry: `fwd`
    (statistics of the forward, coefficients for the consumer) and `bwd`
    (the backward's sums, coefficients for the producer's data gradient),
    plus the last forward's save_mean / save_invstd."""

    def __init__(self, bn, shape, device):
        B, C, H, W = shape
        n = int(_lib.load().dro_bn_state_bytes(B, H, W, C))
        if n == 0:
            raise RuntimeError(f"BN fusion: unsupported geometry {tuple(shape)}")
        self.fwd = torch.zeros(n, dtype=torch.uint8, device=device)
        self.bwd = torch.zeros(n, dtype=torch.uint8, device=device)
        self.saved = None
        self.g_ready = False

    def params(self, bn, smean, sinv):
        track = bn.track_running_stats and bn.running_mean is not None
        return DroBnParams(_p(bn.weight), _p(bn.bias), _p(bn.running_mean) if track else None,
                           _p(bn.running_var) if track else None,
                           _p(bn.num_batches_tracked) if track else None, float(bn.eps), float(bn.momentum),
                           smean.data_ptr(), sinv.data_ptr())


def site_of(bn, shape, device):
    sites = bn.__dict__.get("_dro_sites")
    if sites is None:
        sites = {}
        object.__setattr__(bn, "_dro_sites", sites)
    key = (tuple(shape), str(device))
    s = sites.get(key)
    if s is None:
        s = sites[key] = BnSite(bn, shape, device)
    return s


def supported(bn, conv, x, elems=None):
    """The fused path applies: a training-mode BN with momentum after a 3x3
    stride-1 'same' conv without bias on a float32 CUDA tensor, with `elems`
    (the BN's elements per channel, B*H*W) above the size policy's bound."""
    if _MODE[0] == "0" or (_MODE[0] == "large" and (elems if elems is not None else
                                                    x.shape[0] * x.shape[2] * x.shape[3]) <= _LARGE):
        return False
    return (x.is_cuda and x.dtype == torch.float32 and x.dim() == 4 and bn.training
            and bn.momentum is not None and conv.kernel_size == (3, 3) and conv.stride == (1, 1)
            and conv.padding == (1, 1) and conv.dilation == (1, 1) and conv.groups == 1 and conv.bias is None
            and conv.padding_mode == "zeros")


_PLANS = {}


def _stage_dz(B, H, W, Cin, Cout):
    """The producer's data gradient stages the BN backward (XF 3) when its
    plan has one row tile: every row tile re-reads z and the coefficients
    (measured at the encoders' shapes, tools/bench_bnconv.py: +8 us over the
    plain data gradient with one row tile, +19 / +40 us with 4 / 8, against
    ~6-12 us for dro_bn_backward_apply)."""
    key = (B, H, W, Cin, Cout)
    v = _PLANS.get(key)
    if v is None:
        info = (ctypes.c_longlong * 16)()
        check(_lib.load().dro_conv2d_plan(Cin, Cout, 3, 3, B, H, W, info), "dro_conv2d_plan")
        v = _PLANS[key] = bool(info[0]) and int(info[2]) == 1
    return v


def _weight_grad(ctx, srcs, w, dout):
    """conv3x3(srcs)'s weight gradient for `dout`: in place into the flat .grad
    view (direct path, returns None) or a buffer (returned on first use)."""
    if ctx.direct is not None:
        gw = ctx.direct[2]
        if not _queue_weight_grad(srcs, w.shape, 0, 1.0, dout, None, gw, None, w):
            _conv_bwd(srcs, w, None, dout, 0, 1.0, [None] * len(srcs), [0] * len(srcs), gw, None, 1)
        return None
    if not ctx.need_w:
        return None
    gw, _, wacc, first = _grad_buffers(ctx.scope, ("conv", w.data_ptr(), w.shape[0]), w, 0, dout.device)
    _conv_bwd(srcs, w, None, dout, 0, 1.0, [None] * len(srcs), [0] * len(srcs), gw, None, wacc)
    return gw if first else None


def _grad_target(ctx, x):
    """(buffer, accumulate) for x's data gradient: its sink, else a new tensor."""
    if ctx.xsink is not None:
        return ctx.xsink.target()
    return torch.empty(x.shape, device=x.device, dtype=x.dtype), 0


class _ConvBnStats(torch.autograd.Function):
    """z = conv3x3(x) with bn's batch statistics of z taken in the epilogue."""

    @staticmethod
    def forward(ctx, x, w, gamma, beta, bn, site, direct):
        lib = _lib.load()
        x = x.contiguous()
        B, Cin, H, W = x.shape
        Cout = w.shape[0]
        z = torch.empty(B, Cout, H, W, device=x.device, dtype=torch.float32)
        smean = torch.empty(Cout, device=x.device, dtype=torch.float32)
        sinv = torch.empty(Cout, device=x.device, dtype=torch.float32)
        prm = site.params(bn, smean, sinv)
        ws, nws = _workspace(B, H, W, Cin, Cout, 3, 3, x.device)
        check(lib.dro_conv2d_bn_forward(ptr(x), B, H, W, Cin, ptr(w), Cout, None, None, None, ctypes.byref(prm),
                                        ptr(site.fwd), ptr(z), ptr(ws), nws, stream_of(x)),
              "dro_conv2d_bn_forward")
        site.saved = (smean, sinv)
        ctx.save_for_backward(x, w, z)
        ctx.site, ctx.direct, ctx.scope = site, direct, current_scope()
        ctx.need_w = w.requires_grad
        ctx.xsink = _sink_of(x) if x.requires_grad else None
        return z

    @staticmethod
    def backward(ctx, gz):
        x, w, z = ctx.saved_tensors
        site = ctx.site
        B, Cin, H, W = x.shape
        Cout = w.shape[0]
        gz = gz.contiguous()
        need_x = ctx.needs_input_grad[0]
        gx, gx_ret = None, None
        if need_x:
            gx, acc = _grad_target(ctx, x)
            gx_ret = None if ctx.xsink is not None else gx
        if site.g_ready and _stage_dz(B, H, W, Cin, Cout):
            # gz is the consumer's g (bn_relu_conv_stats' backward): the BN
            # backward's dz is formed in this data gradient's staging and stored
            site.g_ready = False
            lib = _lib.load()
            dz = torch.empty_like(z)
            if gx is None:
                gx, acc = torch.empty(x.shape, device=x.device), 0
            ws, nws = _workspace(B, H, W, Cin, Cout, 3, 3, x.device)
            check(lib.dro_conv2d_bn_backward_data(ptr(w), B, H, W, Cin, Cout, ptr(gz), ptr(site.bwd), ptr(z),
                                                  ptr(dz), None, None, ptr(gx), acc, ptr(ws), nws, stream_of(gz)),
                  "dro_conv2d_bn_backward_data")
        elif site.g_ready:
            # several row tiles: one pass forms dz (each tile would re-read z)
            site.g_ready = False
            dz = torch.empty_like(z)
            check(_lib.load().dro_bn_backward_apply(ptr(gz), ptr(z), B, Cout, H, W, ptr(site.bwd), ptr(dz),
                                                    stream_of(gz)), "dro_bn_backward_apply")
            if gx is not None:
                _conv_bwd([x], w, None, dz, 0, 1.0, [gx], [acc])
        else:
            dz = gz
            if gx is not None:
                _conv_bwd([x], w, None, dz, 0, 1.0, [gx], [acc])
        gw = _weight_grad(ctx, [x], w, dz)
        return gx_ret, gw, None, None, None, None, None


class _BnReluConvStats(torch.autograd.Function):
    """z2 = conv3x3(relu(bn1(z1))) staged from bn1's statistics (y1 stored by
    the conv), with bn2's statistics of z2 taken in the epilogue when bn2 is
    given."""

    @staticmethod
    def forward(ctx, z1, gamma1, beta1, w2, bn1, site1, bn2, site2, direct):
        lib = _lib.load()
        B, C1, H, W = z1.shape
        C2 = w2.shape[0]
        y1 = torch.empty_like(z1)
        z2 = torch.empty(B, C2, H, W, device=z1.device, dtype=torch.float32)
        prm = None
        if bn2 is not None:
            smean2 = torch.empty(C2, device=z1.device, dtype=torch.float32)
            sinv2 = torch.empty(C2, device=z1.device, dtype=torch.float32)
            prm = site2.params(bn2, smean2, sinv2)
        ws, nws = _workspace(B, H, W, C1, C2, 3, 3, z1.device)
        check(lib.dro_conv2d_bn_forward(ptr(z1), B, H, W, C1, ptr(w2), C2, ptr(site1.fwd), None, ptr(y1),
                                        ctypes.byref(prm) if prm is not None else None,
                                        ptr(site2.fwd) if prm is not None else None, ptr(z2), ptr(ws), nws,
                                        stream_of(z1)), "dro_conv2d_bn_forward")
        if prm is not None:
            site2.saved = (smean2, sinv2)
        smean1, sinv1 = site1.saved
        ctx.save_for_backward(z1, y1, w2, gamma1, smean1, sinv1)
        ctx.site1, ctx.direct, ctx.scope = site1, direct, current_scope()
        ctx.need_w = w2.requires_grad
        ctx.y1 = y1     # the parity tests' ReLU branch record (bn_relu_conv_stats)
        return z2

    @staticmethod
    def backward(ctx, gz2):
        z1, y1, w2, gamma1, smean1, sinv1 = ctx.saved_tensors
        lib = _lib.load()
        B, C1, H, W = z1.shape
        C2 = w2.shape[0]
        gz2 = gz2.contiguous()
        g1 = torch.empty_like(z1)
        dg = torch.empty(C1, device=z1.device) if ctx.needs_input_grad[1] else None
        db = torch.empty(C1, device=z1.device) if ctx.needs_input_grad[2] else None
        gp = DroBnGradParams(y1.data_ptr(), z1.data_ptr(), _p(gamma1), smean1.data_ptr(), sinv1.data_ptr(),
                             _p(dg), _p(db))
        ws, nws = _workspace(B, H, W, C1, C2, 3, 3, z1.device)
        check(lib.dro_conv2d_bn_backward_data(ptr(w2), B, H, W, C1, C2, ptr(gz2), None, None, None,
                                              ctypes.byref(gp), ptr(ctx.site1.bwd), ptr(g1), 0, ptr(ws), nws,
                                              stream_of(gz2)), "dro_conv2d_bn_backward_data")
        ctx.site1.g_ready = True       # the producer's backward receives g1, not dz1
        gw = _weight_grad(ctx, [y1], w2, gz2)
        return g1, dg, db, gw, None, None, None, None, None


def _bn_relu_backward(dy, z, y, gamma, smean, sinv, need_gamma, need_beta, gs):
    """hip.batchnorm_act's backward (relu, skip gradient into gs when given):
    (dz, dgamma, dbeta)."""
    lib = _lib.load()
    N, C, H, W = z.shape
    gx = torch.empty_like(z)
    gw = torch.empty(C, device=z.device) if need_gamma else None
    gb = torch.empty(C, device=z.device) if need_beta else None
    nws = lib.dro_batchnorm_workspace_bytes(N, C, H * W)
    ws = torch.empty(max(nws, 16), device=z.device, dtype=torch.uint8)
    check(lib.dro_batchnorm_relu_backward(
        ptr(dy), ptr(z), ptr(y), ptr(gamma), ptr(smean), ptr(sinv), 1, N, C, H * W,
        ptr(gx), ptr(gw), ptr(gb), ptr(gs), ptr(ws), nws, stream_of(dy)), "dro_batchnorm_relu_backward")
    return gx, gw, gb


class _BnAddReluConvStats(torch.autograd.Function):
    """(y, z1) = (relu(bn2(z2) + skip), conv1(y)): a BasicBlock's output
    staged by the NEXT block's conv1 from bn2's statistics (XF 2; y stored
    once per pixel by the conv: it is that block's skip), with bn1's
    statistics of z1 in conv1's epilogue.  Backward: conv1's data gradient
    adds into dy (the skip's gradient the next bn2 returned), then bn2's
    backward (dro_batchnorm_relu_backward)."""

    @staticmethod
    def forward(ctx, z2, gamma2, beta2, skip, w1, bn2, site2, bn1, site1, direct):
        lib = _lib.load()
        B, C, H, W = z2.shape
        C1 = w1.shape[0]
        skip = skip.contiguous()
        y = torch.empty_like(z2)
        z1 = torch.empty(B, C1, H, W, device=z2.device, dtype=torch.float32)
        smean1 = torch.empty(C1, device=z2.device, dtype=torch.float32)
        sinv1 = torch.empty(C1, device=z2.device, dtype=torch.float32)
        prm = site1.params(bn1, smean1, sinv1)
        ws, nws = _workspace(B, H, W, C, C1, 3, 3, z2.device)
        check(lib.dro_conv2d_bn_forward(ptr(z2), B, H, W, C, ptr(w1), C1, ptr(site2.fwd), ptr(skip), ptr(y),
                                        ctypes.byref(prm), ptr(site1.fwd), ptr(z1), ptr(ws), nws, stream_of(z2)),
              "dro_conv2d_bn_forward")
        site1.saved = (smean1, sinv1)
        smean2, sinv2 = site2.saved
        ctx.save_for_backward(z2, y, gamma2, smean2, sinv2, w1, z1)
        ctx.site1, ctx.direct, ctx.scope = site1, direct, current_scope()
        ctx.need_w = w1.requires_grad
        ctx.skipsink = _sink_of(skip) if skip.requires_grad else None
        return y, z1

    @staticmethod
    def backward(ctx, gy, gz1):
        z2, y, gamma2, smean2, sinv2, w1, z1 = ctx.saved_tensors
        B, C, H, W = z2.shape
        C1 = w1.shape[0]
        site1 = ctx.site1
        # the block output's gradient: what its other reader (the next bn2's
        # skip) returned, plus conv1's data gradient added in place
        if gy is not None:
            dy, acc = gy.contiguous(), 1
        else:
            dy, acc = torch.empty_like(y), 0
        gw1 = None
        if gz1 is not None:
            gz1 = gz1.contiguous()
            if site1.g_ready and _stage_dz(B, H, W, C, C1):
                site1.g_ready = False
                dz1 = torch.empty_like(z1)
                ws, nws = _workspace(B, H, W, C, C1, 3, 3, z2.device)
                check(_lib.load().dro_conv2d_bn_backward_data(ptr(w1), B, H, W, C, C1, ptr(gz1), ptr(site1.bwd),
                                                              ptr(z1), ptr(dz1), None, None, ptr(dy), acc, ptr(ws),
                                                              nws, stream_of(gz1)), "dro_conv2d_bn_backward_data")
            else:
                if site1.g_ready:
                    site1.g_ready = False
                    dz1 = torch.empty_like(z1)
                    check(_lib.load().dro_bn_backward_apply(ptr(gz1), ptr(z1), B, C1, H, W, ptr(site1.bwd),
                                                            ptr(dz1), stream_of(gz1)), "dro_bn_backward_apply")
                else:
                    dz1 = gz1
                _conv_bwd([y], w1, None, dz1, 0, 1.0, [dy], [acc])
            gw1 = _weight_grad(ctx, [y], w1, dz1)
        elif gy is None:
            return (None,) * 10
        gs, in_sink = None, False
        if ctx.needs_input_grad[3]:
            if ctx.skipsink is not None and not ctx.skipsink.written:
                gs, in_sink = ctx.skipsink.target()[0], True
            else:
                gs = torch.empty_like(z2)
        gx, gg, gb = _bn_relu_backward(dy, z2, y, gamma2, smean2, sinv2, ctx.needs_input_grad[1],
                                       ctx.needs_input_grad[2], gs)
        return gx, gg, gb, (None if in_sink else gs), gw1, None, None, None, None, None


class _BnApply(torch.autograd.Function):
    """relu(bn(z) [+ skip]) from the statistics the producing conv left; the
    backward is hip.batchnorm_act's (dro_batchnorm_relu_backward)."""

    @staticmethod
    def forward(ctx, z, gamma, beta, skip, bn, site, relu):
        lib = _lib.load()
        B, C, H, W = z.shape
        skip = skip.contiguous() if skip is not None else None
        y = torch.empty_like(z)
        check(lib.dro_bn_apply(ptr(z), ptr(skip), int(relu), B, C, H, W, ptr(site.fwd), ptr(y), stream_of(z)),
              "dro_bn_apply")
        smean, sinv = site.saved
        ctx.save_for_backward(z, y, gamma, smean, sinv)
        ctx.relu, ctx.has_skip = int(relu), skip is not None
        ctx.skipsink = _sink_of(skip) if skip is not None and skip.requires_grad else None
        ctx.affine = (gamma is not None, beta is not None)
        return y

    @staticmethod
    def backward(ctx, gy):
        lib = _lib.load()
        x, y, weight, smean, sinv = ctx.saved_tensors
        N, C, H, W = x.shape
        gy = gy.contiguous()
        gx = torch.empty_like(x)
        gw = torch.empty(C, device=x.device) if ctx.affine[0] else None
        gb = torch.empty(C, device=x.device) if ctx.affine[1] else None
        gs = torch.empty_like(x) if ctx.has_skip and ctx.needs_input_grad[3] else None
        in_sink = gs is not None and ctx.skipsink is not None and not ctx.skipsink.written
        if in_sink:
            gs = ctx.skipsink.target()[0]
        nws = lib.dro_batchnorm_workspace_bytes(N, C, H * W)
        ws = torch.empty(max(nws, 16), device=x.device, dtype=torch.uint8)
        check(lib.dro_batchnorm_relu_backward(
            ptr(gy), ptr(x), ptr(y), ptr(weight), ptr(smean), ptr(sinv), ctx.relu, N, C, H * W,
            ptr(gx), ptr(gw), ptr(gb), ptr(gs), ptr(ws), nws, stream_of(gy)), "dro_batchnorm_relu_backward")
        return gx, gw, gb, (None if in_sink else gs), None, None, None


def bn_add_relu_conv_stats(z2, bn2, skip, conv1, bn1):
    """(relu(bn2(z2) + skip), conv1 of it) with z2 from a conv that took
    bn2's statistics: the block output is staged (and stored) by the next
    block's conv1, whose epilogue takes bn1's statistics."""
    site2 = site_of(bn2, z2.shape, z2.device)
    if site2.saved is None:
        raise RuntimeError("bn_add_relu_conv_stats: z2 must come from a conv that took bn2's statistics")
    site1 = site_of(bn1, (z2.shape[0], conv1.weight.shape[0], z2.shape[2], z2.shape[3]), z2.device)
    y, z1 = _BnAddReluConvStats.apply(z2, bn2.weight, bn2.bias, skip, conv1.weight, bn2, site2, bn1, site1,
                                      _direct(conv1.weight))
    record_branch(("relu", getattr(bn2, "_dro_tag", None)), lambda: (y > 0).to(torch.uint8), z2)
    return y, z1


def _direct(w):
    d = _direct_targets((w,), ())          # marks w as written in place
    return d


def conv_bn_stats(x, conv, bn):
    """z = conv(x) (3x3 stride 1) with bn's training statistics of z taken in
    the conv's epilogue (running statistics updated); feed z to
    bn_relu_conv_stats or bn_apply."""
    require_device(x, conv.weight, what="conv_bn_stats")
    site = site_of(bn, (x.shape[0], conv.weight.shape[0], x.shape[2], x.shape[3]), x.device)
    return _ConvBnStats.apply(x, conv.weight, bn.weight, bn.bias, bn, site, _direct(conv.weight))


def bn_relu_conv_stats(z1, bn1, conv2, bn2=None):
    """conv2(relu(bn1(z1))) with z1 from conv_bn_stats(.., bn1); bn2's
    statistics of the result taken in conv2's epilogue when given."""
    site1 = site_of(bn1, z1.shape, z1.device)
    if site1.saved is None:
        raise RuntimeError("bn_relu_conv_stats: z1 must come from conv_bn_stats with the same BN")
    site2 = site_of(bn2, (z1.shape[0], conv2.weight.shape[0], z1.shape[2], z1.shape[3]), z1.device) \
        if bn2 is not None else None
    z2 = _BnReluConvStats.apply(z1, bn1.weight, bn1.bias, conv2.weight, bn1, site1, bn2, site2,
                                _direct(conv2.weight))
    record_branch(("relu", getattr(bn1, "_dro_tag", None)), lambda: _relu_mask_of(z2), z1)
    return z2


def _relu_mask_of(z2):
    # the y1 the conv stored (kept on the autograd node, i.e. the op's ctx)
    return (z2.grad_fn.y1 > 0).to(torch.uint8)


def bn_apply(z, bn, skip=None, relu=True):
    """relu(bn(z) [+ skip]) with z from conv_bn_stats / bn_relu_conv_stats(..,
    bn): the statistics are already taken."""
    site = site_of(bn, z.shape, z.device)
    if site.saved is None:
        raise RuntimeError("bn_apply: z must come from a conv that took this BN's statistics")
    y = _BnApply.apply(z, bn.weight, bn.bias, skip, bn, site, 1 if relu else 0)
    if relu:
        record_branch(("relu", getattr(bn, "_dro_tag", None)), lambda: (y > 0).to(torch.uint8), z)
    return y
