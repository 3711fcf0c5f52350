"""Autograd wrappers of the f32-MFMA convolution engine (csrc/conv.hip).

`conv2d(srcs, weight, bias, act, alpha)` computes act(conv(cat(srcs))) * alpha
for stride-1 'same' convolutions without materialising the concatenation:
each source may be a dense NCHW tensor, a channel-slice view of one, or a
[B,C,1,1] tensor expanded over H x W (a constant map).  `sepconvgru_half`
is one direction of SepConvGRU (update.py:47-74) in two launches forward.
"""
import ctypes

import torch

from . import _lib
from ._lib import check, ptr, require_device, stream_of

ACT = {None: 0, "none": 0, "relu": 1, "sigmoid": 2, "tanh": 3}


class DroSlice(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("channels", ctypes.c_int),
                ("total_channels", ctypes.c_int), ("channel_offset", ctypes.c_int),
                ("broadcast", ctypes.c_int)]


def _slice(t):
    B, C, H, W = t.shape
    s0, s1, s2, s3 = t.stride()
    if s2 == 0 and s3 == 0 and s1 == 1:                       # expanded [B,C,1,1]
        return DroSlice(t.data_ptr(), C, s0 if B > 1 else C, 0, 1)
    HW = H * W
    if s3 == 1 and s2 == W and s1 == HW and (B == 1 or (s0 % HW == 0 and s0 >= C * HW)):
        return DroSlice(t.data_ptr(), C, s0 // HW if B > 1 else C, 0, 0)
    raise RuntimeError(f"conv2d: unsupported source layout {tuple(t.shape)} strides {t.stride()}"
                       " (need NCHW, a channel slice of NCHW, or an expanded [B,C,1,1])")


def _slices(srcs):
    arr = (DroSlice * len(srcs))()
    for i, t in enumerate(srcs):
        arr[i] = _slice(t)
    return arr


def _grad_targets(bufs):
    n = len(bufs)
    ptrs = (ctypes.c_void_p * n)(*[b.data_ptr() if b is not None else None for b in bufs])
    ctot = (ctypes.c_int * n)(*[b.shape[1] if b is not None else 0 for b in bufs])
    coff = (ctypes.c_int * n)(*([0] * n))
    return ptrs, ctot, coff


_WS = {}


def _workspace(B, H, W, Cin, Cout, KH, KW, device):
    """Scratch for one conv call (torch caching allocator: graph-capture safe)."""
    key = (B, H, W, Cin, Cout, KH, KW)
    n = _WS.get(key)
    if n is None:
        n = _WS[key] = int(_lib.load().dro_conv2d_workspace_bytes(B, H, W, Cin, Cout, KH, KW))
    return torch.empty(max(n, 1), dtype=torch.uint8, device=device), n


def _dense_out(srcs, C):
    B, _, H, W = srcs[0].shape
    return torch.empty(B, C, H, W, device=srcs[0].device, dtype=torch.float32)


class _Conv2d(torch.autograd.Function):
    @staticmethod
    def forward(ctx, weight, bias, act, alpha, *srcs):
        lib = _lib.load()
        require_device(weight, bias, *srcs, what="conv2d")
        Cout, Cin, KH, KW = weight.shape
        if sum(s.shape[1] for s in srcs) != Cin:
            raise RuntimeError("conv2d: source channels do not add up to the weight's Cin")
        B, _, H, W = srcs[0].shape
        weight = weight.contiguous()
        out = _dense_out(srcs, Cout)
        ws, nws = _workspace(B, H, W, Cin, Cout, KH, KW, out.device)
        check(lib.dro_conv2d_forward(_slices(srcs), len(srcs), ptr(weight), ptr(bias), B, H, W, Cout, KH, KW,
                                     act, ctypes.c_float(alpha), ptr(out), Cout, 0, ptr(ws), nws,
                                     stream_of(out)), "dro_conv2d_forward")
        ctx.save_for_backward(weight, out if act else None, *srcs)
        ctx.meta = (act, alpha, bias is not None)
        return out

    @staticmethod
    def backward(ctx, gout):
        lib = _lib.load()
        weight, y, *srcs = ctx.saved_tensors
        act, alpha, has_bias = ctx.meta
        Cout, Cin, KH, KW = weight.shape
        B, _, H, W = srcs[0].shape
        need = ctx.needs_input_grad
        gout = gout.contiguous()
        gsrc = [torch.empty(B, s.shape[1], H, W, device=gout.device) if need[4 + i] else None
                for i, s in enumerate(srcs)]
        gw = torch.empty_like(weight) if (need[0] or (has_bias and need[1])) else None
        gb = torch.empty(Cout, device=gout.device) if (has_bias and need[1]) else None
        ptrs, ctot, coff = _grad_targets(gsrc)
        acc = (ctypes.c_int * len(srcs))()
        ys = DroSlice(y.data_ptr(), Cout, Cout, 0, 0) if y is not None else None
        ws, nws = _workspace(B, H, W, Cin, Cout, KH, KW, gout.device)
        check(lib.dro_conv2d_backward(_slices(srcs), len(srcs), ptr(weight), B, H, W, Cout, KH, KW,
                                      act, ctypes.c_float(alpha), ctypes.byref(ys) if ys else None,
                                      ptr(gout), ptrs, ctot, coff, acc, ptr(gw), ptr(gb), ptr(ws), nws,
                                      stream_of(gout)), "dro_conv2d_backward")
        return (gw if need[0] else None, gb, None, None, *gsrc)


def conv2d(srcs, weight, bias=None, act=None, alpha=1.0):
    """act(conv2d(cat(srcs, 1), weight, bias, padding=k//2)) * alpha on f32 MFMA."""
    if torch.is_tensor(srcs):
        srcs = [srcs]
    return _Conv2d.apply(weight, bias, ACT[act], float(alpha), *srcs)


class _SepGRUHalf(torch.autograd.Function):
    """One direction of SepConvGRU (update.py:59-70): z, r = sigmoid(conv([h; x]));
    q = tanh(conv([r*h; x])); h' = (1-z) h + z q.  x given as sources.
    Forward: 2 launches (gates + r*h; candidate + blend)."""

    @staticmethod
    def forward(ctx, h, wz, bz, wr, br, wq, bq, *xs):
        lib = _lib.load()
        require_device(h, wz, wq, *xs, what="sepconvgru")
        h = h.contiguous()
        B, hd, H, W = h.shape
        KH, KW = wz.shape[2:]
        cin = wz.shape[1]
        wzr = torch.cat([wz, wr], 0).contiguous()
        bzr = torch.cat([bz, br], 0).contiguous()
        st = stream_of(h)
        zr = torch.empty(B, 2 * hd, H, W, device=h.device)
        rh = torch.empty_like(h)
        ws, nws = _workspace(B, H, W, cin, 2 * hd, KH, KW, h.device)
        check(lib.dro_convgru_gates_forward(_slices([h, *xs]), 1 + len(xs), ptr(wzr), ptr(bzr), B, H, W, hd,
                                            KH, KW, ptr(zr), ptr(rh), ptr(ws), nws, st),
              "dro_convgru_gates_forward")
        q = torch.empty_like(h)
        hn = torch.empty_like(h)
        z_sl = DroSlice(zr.data_ptr(), hd, 2 * hd, 0, 0)
        h_sl = DroSlice(h.data_ptr(), hd, hd, 0, 0)
        wsq, nwsq = _workspace(B, H, W, cin, hd, KH, KW, h.device)
        check(lib.dro_convgru_blend_forward(_slices([rh, *xs]), 1 + len(xs), ptr(wq.contiguous()), ptr(bq),
                                            B, H, W, hd, KH, KW, ctypes.byref(z_sl), ctypes.byref(h_sl),
                                            ptr(q), ptr(hn), hd, 0, ptr(wsq), nwsq, st),
              "dro_convgru_blend_forward")
        ctx.save_for_backward(h, rh, wzr, wq, zr, q, *xs)
        return hn

    @staticmethod
    def backward(ctx, dhn):
        lib = _lib.load()
        h, rh, wzr, wq, zr, q, *xs = ctx.saved_tensors
        B, hd, H, W = h.shape
        KH, KW = wq.shape[2:]
        cin = wq.shape[1]
        st = stream_of(h)
        dhn = dhn.contiguous()
        need = ctx.needs_input_grad
        n = 1 + len(xs)
        # stage 1: pre-activation grads of q and z, dh = dh' (1-z)
        dq, dh = torch.empty_like(h), torch.empty_like(h)
        dzr = torch.empty_like(zr)
        check(lib.dro_gru_backward_elem(1, B, hd, H, W, ptr(dhn), ptr(zr), ptr(q), ptr(h), None, ptr(dq),
                                        ptr(dzr), ptr(dh), st), "dro_gru_backward_elem(1)")
        # candidate conv over [r*h, x]: d(r*h), dx (overwrite), dWq, dbq
        drh = torch.empty_like(h)
        dxs = [torch.empty(B, x.shape[1], H, W, device=h.device) if need[7 + i] else None
               for i, x in enumerate(xs)]
        gwq, gbq = torch.empty_like(wq), torch.empty(hd, device=h.device)
        ptrs, ctot, coff = _grad_targets([drh, *dxs])
        acc = (ctypes.c_int * n)()
        ws, nws = _workspace(B, H, W, cin, hd, KH, KW, h.device)
        check(lib.dro_conv2d_backward(_slices([rh, *xs]), n, ptr(wq.contiguous()), B, H, W, hd, KH, KW,
                                      0, ctypes.c_float(1.0), None, ptr(dq), ptrs, ctot, coff, acc,
                                      ptr(gwq), ptr(gbq), ptr(ws), nws, st), "dro_conv2d_backward(q)")
        # stage 2: pre-activation grad of r, dh += d(r*h) r
        check(lib.dro_gru_backward_elem(2, B, hd, H, W, None, ptr(zr), None, ptr(h), ptr(drh), None,
                                        ptr(dzr), ptr(dh), st), "dro_gru_backward_elem(2)")
        # gate conv over [h, x]: dh, dx accumulate; dWz|dWr, dbz|dbr
        gwzr, gbzr = torch.empty_like(wzr), torch.empty(2 * hd, device=h.device)
        ptrs, ctot, coff = _grad_targets([dh, *dxs])
        acc = (ctypes.c_int * n)(*([1] * n))
        ws, nws = _workspace(B, H, W, cin, 2 * hd, KH, KW, h.device)
        check(lib.dro_conv2d_backward(_slices([h, *xs]), n, ptr(wzr), B, H, W, 2 * hd, KH, KW,
                                      0, ctypes.c_float(1.0), None, ptr(dzr), ptrs, ctot, coff, acc,
                                      ptr(gwzr), ptr(gbzr), ptr(ws), nws, st), "dro_conv2d_backward(zr)")
        return (dh if need[0] else None, gwzr[:hd], gbzr[:hd], gwzr[hd:], gbzr[hd:], gwq, gbq, *dxs)


def sepconvgru_half(h, convz, convr, convq, xs):
    """h' for one SepConvGRU direction; xs: the input sources (virtual concat)."""
    return _SepGRUHalf.apply(h, convz.weight, convz.bias, convr.weight, convr.bias, convq.weight,
                             convq.bias, *xs)
