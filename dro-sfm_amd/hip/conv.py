"""Autograd wrappers of the f32-MFMA convolution engine (csrc/conv.hip).

`conv2d(srcs, weight, bias, act, alpha)` computes act(conv(cat(srcs))) * alpha
for stride-1 'same' convolutions without materialising the concatenation:
each source may be a dense NCHW tensor, a channel-slice view of one, or a
[B,C,1,1] tensor expanded over H x W (a constant map).  `sepconvgru_half`
is one direction of SepConvGRU (update.py:47-74) in two launches forward.

`weight_grad_scope()`: inside it (one forward of the recurrent net), a weight
used by several convs gets its gradient summed IN the backward kernels (the
first backward call of that weight returns the buffer, later ones add into it
and return None; autograd consumes it only after every producer has run), and
weight concatenations are built once.  Without the scope every call returns
its own gradient, as plain autograd would.

Direct weight gradients (the trainer's path): when the parameters a conv reads
are flagged `_dro_direct` and their `.grad` tensors are back-to-back views of
one flat buffer (trainers/dp_trainer.GradBuckets lays fused groups out
adjacently), the weight/bias gradient kernels accumulate straight into those
views, in stream order; autograd receives None for the parameters.  Fused
weights (z|r gates, shared-input heads) are then views of the flat parameter
buffer instead of per-forward concatenations.  (Round 3 measured two
side-stream variants -- per-call weight gradients forked onto a side stream,
and the batched flushes on a stream of their own -- both slower under hipGraph
replay; they were removed in round 4.)

Batched weight gradients (direct path, default on): the recurrent update
blocks apply every weight once per iteration, so instead of one weight-gradient
launch + one split reduction per use, each use is queued (sources, output
gradient, saved output kept alive) and all uses of a weight are reduced by ONE
dro_conv2d_weight_grad_multi launch: from the parameter's post-accumulate hook
(flush_param_grads, called by the trainer's gradient buckets -- autograd runs
it once the last use has been back-propagated, so the bucket's all-reduce
overlaps the rest of the backward), or at the end of backward (engine final
callback) for whatever is still queued.  set_batched_weight_grads.

Split-bf16 engine (set_split_engine, default off): the 1x5 / 5x1 / 3x3 / 1x1
forward and data-gradient GEMMs run on bf16 MFMA over operands split into three
bf16 terms (csrc/xconv.hip, f32 accuracy at 2.67x the f32 MFMA rate).  Each
weight is split (both GEMM layouts) at its first use in a forward pass of the
network (one split per weight_grad_scope; every call outside a scope splits
afresh) and the split buffers are saved for the backward.
"""
import contextlib
import ctypes
import os
from typing import Optional

import torch

from . import _lib
from ._lib import check, ptr, require_device, stream_of
from .ops import _sink_of

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


class WeightGradScope:
    def __init__(self):
        self.grads = {}     # key -> [gw, gb] accumulation buffers
        self.cats = {}      # key -> concatenated (weight, bias)


_SCOPE = [None]
_GEN = [0, 0]      # [weight generation, open scopes]: splits are reused within one generation


@contextlib.contextmanager
def weight_grad_scope():
    prev = _SCOPE[0]
    _SCOPE[0] = WeightGradScope() if torch.is_grad_enabled() else None
    if _GEN[1] == 0:
        _GEN[0] += 1       # a new forward pass: weights may have changed since the last one
    _GEN[1] += 1
    try:
        yield _SCOPE[0]
    finally:
        _SCOPE[0] = prev
        _GEN[1] -= 1


# measured: not faster than the f32 engine at the step's shapes;
# DRO_SPLIT_ENGINE=all|3x3fwd turns it on for A/B runs
_XCONV = [os.environ.get("DRO_SPLIT_ENGINE", "") in ("all", "3x3fwd")]
_XSHAPES = {(1, 5), (5, 1), (3, 3), (1, 1)}
# "all": every xconv shape, fwd + data grad; "3x3fwd": 3x3 forwards only
_XPOLICY = [os.environ.get("DRO_SPLIT_ENGINE", "") or "all"]
_SPLITS = {}       # (data_ptr, shape, device) -> [generation, fwd split, bwd split]


def set_split_engine(enabled, policy="all"):
    """Split-bf16 MFMA engine for the halo convs (True) or the f32-MFMA engine
    (False, default: the faster of the two at the update-block shapes).
    policy "3x3fwd" limits it to the forward of the 3x3 convs."""
    _XCONV[0] = bool(enabled)
    _XPOLICY[0] = policy


def _wsplit(weight):
    """(fwd, bwd) split-bf16 copies of a contiguous weight for the xconv engine,
    or (None, None) when the f32 engine runs this conv."""
    if not _XCONV[0] or tuple(weight.shape[2:]) not in _XSHAPES:
        return None, None
    if _XPOLICY[0] == "3x3fwd" and tuple(weight.shape[2:]) != (3, 3):
        return None, None
    lib = _lib.load()
    Cout, Cin, KH, KW = weight.shape
    key = (weight.data_ptr(), tuple(weight.shape), weight.device)
    ent = _SPLITS.get(key)
    if ent is None:
        if len(_SPLITS) > 512:   # drop splits of weights unused for two forward passes
            for k in [k for k, v in _SPLITS.items() if v[0] < _GEN[0] - 1]:
                del _SPLITS[k]
        nf = int(lib.dro_weight_split_bytes(Cout, Cin, KH, KW, 0))
        nb = int(lib.dro_weight_split_bytes(Cout, Cin, KH, KW, 1))
        ent = _SPLITS[key] = [-1, torch.empty(nf // 2, dtype=torch.int16, device=weight.device),
                              torch.empty(nb // 2, dtype=torch.int16, device=weight.device)]
    if ent[0] != _GEN[0] or _GEN[1] == 0:
        check(lib.dro_weight_split(ptr(weight), Cout, Cin, KH, KW, ptr(ent[1]), ptr(ent[2]),
                                   stream_of(weight)), "dro_weight_split")
        ent[0] = _GEN[0]
    if _XPOLICY[0] == "3x3fwd":
        return ent[1], None
    return ent[1], ent[2]


def _wsplit_bwd(weight):
    """The backward split copy `_wsplit` made for this weight in the forward
    (a cache lookup: no launch), or None -- the backward then runs the f32
    engine.  setup_context reads it here instead of from the forward's
    side channel (a module-global hand-off breaks when tracing
    runs a setup without its implementation)."""
    if not _XCONV[0] or _XPOLICY[0] == "3x3fwd" or not weight.is_contiguous():
        return None
    ent = _SPLITS.get((weight.data_ptr(), tuple(weight.shape), weight.device))
    return ent[2] if ent is not None and ent[0] == _GEN[0] else None


def current_scope():
    return _SCOPE[0]


def cached_cat(key, make):
    """make() once per scope (e.g. torch.cat of conv weights); uncached outside."""
    sc = _SCOPE[0]
    if sc is None:
        return make()
    v = sc.cats.get(key)
    if v is None:
        v = sc.cats[key] = make()
    return v


_DIRECT = [True]


def set_direct_weight_grads(enabled):
    """Enable/disable the side-stream direct weight-gradient path (A/B runs)."""
    _DIRECT[0] = bool(enabled)


def _flat_view(tensors):
    """[sum(dim 0), *rest] view over tensors stored back to back (contiguous, same
    trailing shape) in one storage, or None.  Never tracked by autograd."""
    t0 = tensors[0]
    base, off, n = t0.untyped_storage().data_ptr(), t0.storage_offset(), 0
    for t in tensors:
        if (not t.is_contiguous() or t.untyped_storage().data_ptr() != base or t.storage_offset() != off + n
                or t.shape[1:] != t0.shape[1:] or t.dtype != t0.dtype):
            return None
        n += t.numel()
    shape = (sum(t.shape[0] for t in tensors),) + tuple(t0.shape[1:])
    if len(tensors) == 1:
        return t0.detach()
    return t0.detach().as_strided(shape, torch.empty(shape, device="meta").stride(), off)


def _direct_targets(wparts, bparts, mark=True, in_setup=False):
    """(fused weight, fused bias, grad-weight view, grad-bias view) when the
    direct path applies to these parameters, else None.  in_setup: called from
    an op's setup_context, which runs with grad mode off (inside the op's
    autograd.Function forward): the grad-mode test was the caller's."""
    if not _DIRECT[0] or not (in_setup or torch.is_grad_enabled()):
        return None
    ps = list(wparts) + list(bparts or ())
    for p in ps:
        if not (getattr(p, "_dro_direct", False) and p.requires_grad and p.grad is not None):
            return None
    gw = _flat_view([p.grad for p in wparts])
    gb = _flat_view([p.grad for p in bparts]) if bparts else None
    w = _flat_view(list(wparts))
    b = _flat_view(list(bparts)) if bparts else None
    if gw is None or w is None or (bparts and (gb is None or b is None)):
        return None
    if mark:
        _mark_direct(ps)
    return w, b, gw, gb


def _mark_direct(params):
    for p in params:
        p._dro_direct_used = True


def _grad_buffers(scope, key, weight, nbias, device):
    """(gw, gb, accumulate, first) for one backward call."""
    if scope is None:
        return (torch.empty_like(weight), torch.empty(nbias, device=device) if nbias else None, 0, True)
    ent = scope.grads.get(key)
    if ent is None:
        gw = torch.empty_like(weight)
        gb = torch.empty(nbias, device=device) if nbias else None
        scope.grads[key] = (gw, gb)
        return gw, gb, 0, True
    return ent[0], ent[1], 1, False


class DroWgradUse(ctypes.Structure):
    _fields_ = [("srcs", ctypes.c_void_p), ("dout", ctypes.c_void_p), ("y", ctypes.c_void_p)]


_BATCH = [True]
_PENDING = {}
_PENDING_CB = [False]
_MULTI_SHAPES = {(1, 1), (1, 5), (5, 1), (3, 3)}
# shapes whose queued uses are stacked on the batch axis and reduced by ONE
# single-use weight gradient (no multi-use kernel for them): the update blocks'
# 7x7 state convs (convd1 / convp1, one source of 1 or 6 channels) -- 8 uses per
# step each, 48 MFLOP per use, ~28 us + a split sum per launch when alone
# (DRO_CAT_WGRAD=0: per use, A/B)
_CAT_SHAPES = {(7, 7)} if os.environ.get("DRO_CAT_WGRAD", "1") != "0" else set()
_MAX_USES = 16


def set_batched_weight_grads(enabled):
    """Batch the direct-path weight gradients of each weight over a backward
    pass (True, default) or launch them per use (False, A/B runs)."""
    _BATCH[0] = bool(enabled)


def _queue_weight_grad(srcs, wshape, act, alpha, dout, y, gw, gb, weight=None):
    """Queue one use's weight(+bias) gradient for the end-of-backward batch;
    False when this conv shape is not batched (the caller launches it)."""
    Cout, Cin, KH, KW = wshape
    if not _BATCH[0] or not ((KH, KW) in _MULTI_SHAPES or ((KH, KW) in _CAT_SHAPES and len(srcs) == 1)):
        return False
    B, _, H, W = srcs[0].shape
    key = (gw.data_ptr(), gb.data_ptr() if gb is not None else 0, B, H, W, act, float(alpha),
           tuple(t.shape[1] for t in srcs))
    ent = _PENDING.get(key)
    cur = torch.cuda.current_stream()
    if ent is None:
        ent = _PENDING[key] = ((B, H, W, Cin, Cout, KH, KW, act, float(alpha), gw, gb, len(srcs), weight), [], [])
    ent[1].append((list(srcs), dout, y))
    if all(s != cur for s in ent[2]):
        ent[2].append(cur)
    if not _PENDING_CB[0]:
        _PENDING_CB[0] = True
        stream = torch.cuda.current_stream()
        torch.autograd.Variable._execution_engine.queue_callback(lambda: flush_weight_grads(stream))
    return True


def _covers(t, ptr_):
    return t is not None and t.data_ptr() <= ptr_ < t.data_ptr() + t.numel() * t.element_size()


def flush_param_grads(param):
    """Launch now the queued weight gradients that write into `param.grad`
    (trainers/dp_trainer.GradBuckets calls this from the parameter's
    post-accumulate hook: autograd runs that hook once every use of the
    parameter has been back-propagated, so the queue holds all of its uses and
    its bucket's all-reduce can start while the rest of the backward runs).
    Returns the stream the launches were queued on, or None."""
    g = param.grad
    if g is None or not _PENDING:
        return None
    p0 = g.data_ptr()
    keys = [k for k, (meta, _, _) in _PENDING.items() if _covers(meta[9], p0) or _covers(meta[10], p0)]
    if not keys:
        return None
    items = [_PENDING.pop(k) for k in keys]
    return _launch_weight_grads(items, items[0][2][0])


def flush_weight_grads(stream=None):
    """Launch every queued weight gradient (one launch + one reduction per
    weight per 16 uses), in first-use order; releases the kept tensors."""
    _PENDING_CB[0] = False
    if not _PENDING:
        return
    items = list(_PENDING.values())
    _PENDING.clear()
    _launch_weight_grads(items, stream or torch.cuda.current_stream())


def _launch_weight_grads(items, stream):
    lib = _lib.load()
    side = any(s != stream for _, _, streams in items for s in streams)
    for _, uses, streams in items:       # uses queued from other streams (concurrent blocks)
        for s in streams:
            if s != stream:
                stream.wait_stream(s)
    if side:
        for _, uses, streams in items:
            for srcs, dout, y in uses:
                for x in (*srcs, dout, y):
                    if x is not None:
                        x.record_stream(stream)
    with torch.cuda.stream(stream):
        for meta, uses, _ in items:
            B, H, W, Cin, Cout, KH, KW, act, alpha, gw, gb, nsrc, weight = meta
            if (KH, KW) in _CAT_SHAPES:
                # every use on the batch axis (broadcast sources materialise),
                # one weight-gradient launch + one split sum for all of them
                xs = torch.cat([srcs[0].expand(B, Cin, H, W) for srcs, _, _ in uses], 0)
                g = torch.cat([d for _, d, _ in uses], 0)
                yy = torch.cat([t for _, _, t in uses], 0) if act else None
                _conv_bwd([xs], weight, yy, g, act, alpha, [None], [0], gw, gb, 1)
                continue
            for c0 in range(0, len(uses), _MAX_USES):
                chunk = uses[c0:c0 + _MAX_USES]
                n = len(chunk)
                sl = [_slices(srcs) for srcs, _, _ in chunk]
                arr = (DroWgradUse * n)()
                for i, (_, dout, y) in enumerate(chunk):
                    arr[i].srcs = ctypes.cast(sl[i], ctypes.c_void_p)
                    arr[i].dout = dout.data_ptr()
                    arr[i].y = y.data_ptr() if y is not None else None
                nb = int(lib.dro_conv2d_weight_grad_multi_workspace_bytes(n, B, H, W, Cin, Cout, KH, KW))
                ws = torch.empty(max(nb, 1), dtype=torch.uint8, device=gw.device)
                check(lib.dro_conv2d_weight_grad_multi(arr, n, nsrc, B, H, W, Cout, KH, KW, act,
                                                       ctypes.c_float(alpha), ptr(gw), ptr(gb), 1,
                                                       ptr(ws), nb, stream_of(gw)),
                      "dro_conv2d_weight_grad_multi")
    return stream


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


Tensor = torch.Tensor


def _placeholder(t, device):
    return t if t is not None else torch.empty(0, device=device)


# ------------------------------------------------------------------ dro::conv2d_backward (data + weight gradients)
@torch.library.custom_op("dro::conv2d_backward", mutates_args=("grad_srcs", "grad_weight", "grad_bias"))
def _conv2d_bwd_op(srcs: list[Tensor], weight: Tensor, y: Optional[Tensor], grad_out: Tensor, act: int,
                   alpha: float, grad_srcs: list[Tensor], accumulate: list[int], grad_weight: Optional[Tensor],
                   grad_bias: Optional[Tensor], weight_accumulate: int, wsplit: Optional[Tensor]) -> None:
    """Gradients of act(conv(cat(srcs), weight) + b) * alpha: the data gradient of
    source i into grad_srcs[i] (empty = not wanted; accumulate[i] = 1 adds),
    the weight (+ bias) gradient into grad_weight / grad_bias (added when
    weight_accumulate).  y: the saved output when act != none (its derivative
    is folded into the staging).  One launch per gradient kind."""
    lib = _lib.load()
    Cout, Cin, KH, KW = weight.shape
    B, _, H, W = srcs[0].shape
    tgt = [g if g.numel() else None for g in grad_srcs]
    ys = DroSlice(y.data_ptr(), Cout, Cout, 0, 0) if y is not None else None
    ws, nws = _workspace(B, H, W, Cin, Cout, KH, KW, grad_out.device)
    ptrs, ctot, coff = _grad_targets(tgt) if any(t is not None for t in tgt) else (None, None, None)
    acc = (ctypes.c_int * len(srcs))(*accumulate) if ptrs is not None else None
    if ptrs is None and grad_weight is None:
        return
    check(lib.dro_conv2d_backward(_slices(srcs), len(srcs), ptr(weight), B, H, W, Cout, KH, KW, act,
                                  ctypes.c_float(alpha), ctypes.byref(ys) if ys else None, ptr(grad_out.contiguous()),
                                  ptrs, ctot, coff, acc, ptr(grad_weight), ptr(grad_bias), weight_accumulate,
                                  ptr(wsplit), ptr(ws), nws, stream_of(grad_out)), "dro_conv2d_backward")


@_conv2d_bwd_op.register_fake
def _(srcs, weight, y, grad_out, act, alpha, grad_srcs, accumulate, grad_weight, grad_bias, weight_accumulate,
      wsplit):
    return None


def _conv_bwd(srcs, weight, y, gout, act, alpha, tgt, dacc, gw=None, gb=None, wacc=0, wsplit=None):
    dev = gout.device
    torch.ops.dro.conv2d_backward(list(srcs), weight, y, gout, act, float(alpha),
                                  [_placeholder(t, dev) for t in tgt], [int(a) for a in dacc], gw, gb, int(wacc),
                                  wsplit)


# ------------------------------------------------------------------ dro::conv2d
@torch.library.custom_op("dro::conv2d", mutates_args=())
def _conv2d_op(srcs: list[Tensor], weight: Tensor, bias: Optional[Tensor], act: int, alpha: float,
               params: list[Tensor], nweight: int) -> Tensor:
    """act(conv2d(cat(srcs, 1), weight, bias, stride 1, padding k//2)) * alpha
    without materialising the concatenation (each source: NCHW, a channel
    slice of one, or a [B,C,1,1] map expanded over H x W).  params: the
    parameters weight/bias are the fused flat-buffer views of when the
    trainer's in-place weight gradients apply (params[:nweight] weights,
    the rest biases), else empty."""
    lib = _lib.load()
    require_device(weight, bias, *srcs, what="conv2d")
    Cout, Cin, KH, KW = weight.shape
    if sum(t.shape[1] for t in srcs) != Cin:
        raise RuntimeError("conv2d: source channels do not add up to the weight's Cin")
    B, _, H, W = srcs[0].shape
    weight = weight.contiguous()
    out = _dense_out(srcs, Cout)
    ws, nws = _workspace(B, H, W, Cin, Cout, KH, KW, out.device)
    wf, wb = _wsplit(weight)
    check(lib.dro_conv2d_forward(_slices(srcs), len(srcs), ptr(weight), ptr(bias), B, H, W, Cout, KH, KW, act,
                                 ctypes.c_float(alpha), ptr(out), Cout, 0, ptr(wf), ptr(ws), nws, stream_of(out)),
          "dro_conv2d_forward")
    return out


@_conv2d_op.register_fake
def _(srcs, weight, bias, act, alpha, params, nweight):
    B, _, H, W = srcs[0].shape
    return srcs[0].new_empty((B, weight.shape[0], H, W))


def _conv2d_setup(ctx, inputs, output):
    srcs, weight, bias, act, alpha, params, nweight = inputs
    ctx.wsplit = _wsplit_bwd(weight)
    ctx.save_for_backward(weight.contiguous(), output if act else None, *srcs)
    ctx.sinks = [_sink_of(x) if x.requires_grad else None for x in srcs]
    ctx.need_src = [x.requires_grad for x in srcs]
    ctx.meta = (act, alpha, bias is not None, weight.requires_grad, bias is not None and bias.requires_grad)
    ctx.direct = _direct_targets(params[:nweight], params[nweight:], mark=False, in_setup=True) if params else None
    ctx.scope = None if params else current_scope()
    ctx.nparams = len(params)


def _conv2d_backward(ctx, gout):
    weight, y, *srcs = ctx.saved_tensors
    act, alpha, has_bias, need_w, need_b = ctx.meta
    Cout, Cin, KH, KW = weight.shape
    B, _, H, W = srcs[0].shape
    gout = gout.contiguous()
    # sources with a gradient sink are written in place (and get None)
    sinks = ctx.sinks
    gsrc = [torch.empty(B, x.shape[1], H, W, device=gout.device) if ctx.need_src[i] and sinks[i] is None
            else None for i, x in enumerate(srcs)]
    sk = [sn.target() if sn is not None else (None, 0) for sn in sinks]
    tgt = [t if sn is not None else g for (t, _), sn, g in zip(sk, sinks, gsrc)]
    dacc = [a for _, a in sk]
    none_params = [None] * ctx.nparams
    if ctx.direct is not None:
        # data gradients here; the weight gradients in place into the flat .grad
        # views, queued for one batched launch per weight (or launched now)
        gw, gb = ctx.direct[2], ctx.direct[3]
        if any(g is not None for g in tgt):
            _conv_bwd(srcs, weight, y, gout, act, alpha, tgt, dacc, wsplit=ctx.wsplit)
        if not _queue_weight_grad(srcs, weight.shape, act, alpha, gout, y, gw, gb if has_bias else None, weight):
            _conv_bwd(srcs, weight, y, gout, act, alpha, [None] * len(srcs), [0] * len(srcs), gw,
                      gb if has_bias else None, 1)
        return gsrc, None, None, None, None, none_params, None
    want_w = need_w or (has_bias and need_b)
    if want_w:
        gw, gb, wacc, first = _grad_buffers(ctx.scope, ("conv", weight.data_ptr(), Cout),
                                            weight, Cout if has_bias else 0, gout.device)
    else:
        gw, gb, wacc, first = None, None, 0, False
    _conv_bwd(srcs, weight, y, gout, act, alpha, tgt, dacc, gw, gb, wacc, ctx.wsplit)
    rw = gw if (first and need_w) else None
    rb = gb if (first and has_bias and need_b) else None
    return gsrc, rw, rb, None, None, none_params, None


torch.library.register_autograd("dro::conv2d", _conv2d_backward, setup_context=_conv2d_setup)


def conv2d(srcs, weight, bias=None, act=None, alpha=1.0, parts=None):
    """act(conv2d(cat(srcs, 1), weight, bias, padding=k//2)) * alpha on f32 MFMA
    (torch.ops.dro.conv2d).

    parts=(weights, biases): the weight/bias are the dim-0 concatenation of these
    parameters (weight/bias may then be None: built here, as a flat-buffer view
    on the direct path or a torch.cat otherwise)."""
    if torch.is_tensor(srcs):
        srcs = [srcs]
    if parts is None:
        parts = ((weight,), (bias,) if bias is not None else ())
    wparts, bparts = parts
    direct = _direct_targets(wparts, bparts)
    if direct is not None:
        return torch.ops.dro.conv2d(list(srcs), direct[0], direct[1], ACT[act], float(alpha),
                                    [*wparts, *bparts], len(wparts))
    if weight is None:
        key = ("cat",) + tuple(id(p) for p in wparts)
        weight, bias = cached_cat(key, lambda: (torch.cat(list(wparts), 0),
                                                torch.cat(list(bparts), 0) if bparts else None))
    return torch.ops.dro.conv2d(list(srcs), weight, bias, ACT[act], float(alpha), [], 0)


# ------------------------------------------------------------------ dro::conv2d_strided
@torch.library.custom_op("dro::conv2d_strided", mutates_args=())
def _conv2d_strided_op(x: Tensor, weight: Tensor, bias: Optional[Tensor], stride: int, pad: int,
                       act: int) -> Tensor:
    """act(F.conv2d(x, weight, bias, stride, pad)) on the flattened implicit GEMM
    (csrc/conv.hip dro_conv2d_strided_*): the encoders' stride-2 convs."""
    lib = _lib.load()
    require_device(x, weight, bias, what="conv2d_strided")
    B, Cin, Hi, Wi = x.shape
    Cout, cin_w, KH, KW = weight.shape
    if cin_w != Cin:
        raise RuntimeError("conv2d_strided: input channels do not match the weight")
    Ho, Wo = (Hi + 2 * pad - KH) // stride + 1, (Wi + 2 * pad - KW) // stride + 1
    x, weight = x.contiguous(), weight.contiguous()
    out = torch.empty(B, Cout, Ho, Wo, device=x.device, dtype=torch.float32)
    nws = int(lib.dro_conv2d_strided_workspace_bytes(B, Hi, Wi, Cin, Cout, KH, KW, stride, pad))
    ws = torch.empty(max(nws, 1), dtype=torch.uint8, device=x.device)
    check(lib.dro_conv2d_strided_forward(ptr(x), ptr(weight), ptr(bias), B, Hi, Wi, Cin, Cout, KH, KW, stride, pad,
                                         act, ptr(out), ptr(ws), nws, stream_of(out)), "dro_conv2d_strided_forward")
    return out


@_conv2d_strided_op.register_fake
def _(x, weight, bias, stride, pad, act):
    B, _, Hi, Wi = x.shape
    Cout, _, KH, KW = weight.shape
    return x.new_empty((B, Cout, (Hi + 2 * pad - KH) // stride + 1, (Wi + 2 * pad - KW) // stride + 1))


@torch.library.custom_op("dro::conv2d_strided_backward", mutates_args=("grad_x", "grad_weight", "grad_bias"))
def _conv2d_strided_bwd_op(x: Tensor, weight: Tensor, grad_out: Tensor, stride: int, pad: int,
                           grad_x: Optional[Tensor], grad_weight: Optional[Tensor], grad_bias: Optional[Tensor],
                           weight_accumulate: int, grad_x_accumulate: int = 0) -> None:
    """Data gradient into grad_x (added when grad_x_accumulate), weight (+ bias)
    gradient into grad_weight / grad_bias (added when weight_accumulate); act
    none only."""
    lib = _lib.load()
    B, Cin, Hi, Wi = x.shape
    Cout, _, KH, KW = weight.shape
    nws = int(lib.dro_conv2d_strided_workspace_bytes(B, Hi, Wi, Cin, Cout, KH, KW, stride, pad))
    ws = torch.empty(max(nws, 1), dtype=torch.uint8, device=x.device)
    check(lib.dro_conv2d_strided_backward(ptr(x.contiguous()), ptr(weight.contiguous()), ptr(grad_out.contiguous()),
                                          B, Hi, Wi, Cin, Cout, KH, KW, stride, pad, ptr(grad_x), int(grad_x_accumulate),
                                          ptr(grad_weight),
                                          ptr(grad_bias), weight_accumulate, ptr(ws), nws, stream_of(grad_out)),
          "dro_conv2d_strided_backward")


@_conv2d_strided_bwd_op.register_fake
def _(x, weight, grad_out, stride, pad, grad_x, grad_weight, grad_bias, weight_accumulate, grad_x_accumulate=0):
    return None


def _conv2d_strided_setup(ctx, inputs, output):
    x, weight, bias, stride, pad, act = inputs
    ctx.save_for_backward(x, weight)
    has_bias = bias is not None
    ctx.meta = (stride, pad, act, has_bias, x.requires_grad, weight.requires_grad,
                has_bias and bias.requires_grad)
    ctx.direct = _direct_targets((weight,), (bias,) if has_bias else (), mark=False, in_setup=True)
    ctx.xsink = _sink_of(x) if x.requires_grad else None


def _conv2d_strided_backward(ctx, gout):
    x, weight = ctx.saved_tensors
    stride, pad, act, has_bias, need_x, need_w, need_b = ctx.meta
    if act:
        raise RuntimeError("conv2d_strided: backward through a fused activation is not supported")
    Cout = weight.shape[0]
    # an input with a gradient sink (a ResNet block's input: its stride-2 conv1
    # and downsample both read it) is written / added in place and gets None
    xacc = 0
    if ctx.xsink is not None:
        gx, xacc = ctx.xsink.target()
    else:
        gx = torch.empty_like(x) if need_x else None
    direct = ctx.direct
    if direct is not None:                 # in place into the trainer's flat .grad views
        gw, gb, wacc = direct[2], direct[3] if has_bias else None, 1
    else:
        gw = torch.empty_like(weight) if need_w else None
        gb = torch.empty(Cout, device=x.device) if (has_bias and need_b) else None
        wacc = 0
    if gw is None and gb is not None:
        gw = torch.empty_like(weight)
    torch.ops.dro.conv2d_strided_backward(x, weight, gout, stride, pad, gx, gw, gb, wacc, xacc)
    if ctx.xsink is not None:
        gx = None
    if direct is not None:
        return gx, None, None, None, None, None
    return gx, (gw if need_w else None), (gb if has_bias and need_b else None), None, None, None


torch.library.register_autograd("dro::conv2d_strided", _conv2d_strided_backward, setup_context=_conv2d_strided_setup)


def conv2d_strided(x, weight, bias=None, stride=2, padding=1, act=None):
    """act(F.conv2d(x, weight, bias, stride, padding)) on the HIP conv engine
    (stride 1 or 2, any kernel size, one dense input; torch.ops.dro.conv2d_strided).
    Weight gradients go in place into the trainer's flat buffer when the
    parameters are flagged for it (as hip.conv2d does)."""
    _direct_targets((weight,), (bias,) if bias is not None else ())      # marks them as written in place
    return torch.ops.dro.conv2d_strided(x, weight, bias, int(stride), int(padding), ACT[act])


# ------------------------------------------------------------------ dro::gru_backward_elem
@torch.library.custom_op("dro::gru_backward_elem", mutates_args=("dq", "dzr", "dh"))
def _gru_elem_op(stage: int, dhn: Optional[Tensor], zr: Tensor, q: Optional[Tensor], h: Tensor,
                 drh: Optional[Tensor], dq: Optional[Tensor], dzr: Tensor, dh: Tensor) -> None:
    """SepConvGRU elementwise backward (csrc/conv.hip gru_backward_elem):
    stage 1 -- from dL/dh' the pre-activation gradients of q and z and
    dh = dh' (1 - z); stage 2 -- the pre-activation gradient of r and dh +=
    d(r*h) r."""
    lib = _lib.load()
    B, hd, H, W = h.shape
    check(lib.dro_gru_backward_elem(stage, B, hd, H, W, ptr(dhn), ptr(zr), ptr(q), ptr(h), ptr(drh), ptr(dq),
                                    ptr(dzr), ptr(dh), stream_of(h)), f"dro_gru_backward_elem({stage})")


@_gru_elem_op.register_fake
def _(stage, dhn, zr, q, h, drh, dq, dzr, dh):
    return None


@torch.library.custom_op("dro::convgru_candidate_backward", mutates_args=("dzr", "dh", "grad_srcs"))
def _gru_cand_bwd_op(srcs: list[Tensor], weight: Tensor, dq: Tensor, zr: Tensor, h: Tensor, dzr: Tensor,
                     dh: Tensor, grad_srcs: list[Tensor], accumulate: list[int]) -> None:
    """The candidate conv's data gradient with SepConvGRU stage 2 in its
    epilogue (csrc/conv.hip dro_convgru_candidate_backward): srcs = [r*h, x...],
    d(r*h) is not stored but turned into dzr[:, hd:] = d h r (1-r) and
    dh += d r; grad_srcs[1:] / accumulate[1:] as in conv2d_backward
    (grad_srcs[0] unused)."""
    lib = _lib.load()
    hd, Cin, KH, KW = weight.shape
    B, _, H, W = srcs[0].shape
    tgt = [None] + [g if g.numel() else None for g in grad_srcs[1:]]
    ws, nws = _workspace(B, H, W, Cin, hd, KH, KW, dq.device)
    ptrs, ctot, coff = _grad_targets(tgt) if any(t is not None for t in tgt) else (None, None, None)
    acc = (ctypes.c_int * len(srcs))(*accumulate) if ptrs is not None else None
    check(lib.dro_convgru_candidate_backward(_slices(srcs), len(srcs), ptr(weight), B, H, W, hd, KH, KW,
                                             ptr(dq.contiguous()), ptr(zr), ptr(h), ptr(dzr), ptr(dh), ptrs, ctot,
                                             coff, acc, ptr(ws), nws, stream_of(dq)),
          "dro_convgru_candidate_backward")


@_gru_cand_bwd_op.register_fake
def _(srcs, weight, dq, zr, h, dzr, dh, grad_srcs, accumulate):
    return None


@torch.library.custom_op("dro::convgru_gates_backward",
                         mutates_args=("grad_srcs", "prev_dq", "prev_dzr", "prev_dh"))
def _gru_gates_bwd_op(srcs: list[Tensor], weight: Tensor, dzr: Tensor, grad_srcs: list[Tensor],
                      accumulate: list[int], prev_zr: Tensor, prev_q: Tensor, prev_h: Tensor, prev_dq: Tensor,
                      prev_dzr: Tensor, prev_dh: Tensor, prev_dh_accumulate: int) -> None:
    """The gate conv's data gradient of a SepConvGRU's second half with the
    first half's stage 1 in its epilogue (csrc/conv.hip
    dro_convgru_gates_backward): srcs = [h, x...] (h = the first half's
    output), grad_srcs[0] its dense gradient (accumulated; the finished value
    is the first half's dh'), the first half's dq, dzr[:, :hd] and dh written
    (dh added into when prev_dh_accumulate)."""
    lib = _lib.load()
    C2, Cin, KH, KW = weight.shape
    B, hd, H, W = srcs[0].shape
    # the first half's tensors are read as dense [B, hd|2hd, H, W] arrays
    for name, t in (("prev_zr", prev_zr), ("prev_q", prev_q), ("prev_h", prev_h), ("prev_dq", prev_dq),
                    ("prev_dzr", prev_dzr), ("prev_dh", prev_dh)):
        if not t.is_contiguous():
            raise RuntimeError(f"convgru_gates_backward: {name} must be contiguous")
    tgt = [g if g.numel() else None for g in grad_srcs]
    ws, nws = _workspace(B, H, W, Cin, C2, KH, KW, dzr.device)
    ptrs, ctot, coff = _grad_targets(tgt)
    acc = (ctypes.c_int * len(srcs))(*accumulate)
    check(lib.dro_convgru_gates_backward(_slices(srcs), len(srcs), ptr(weight), B, H, W, hd, KH, KW,
                                         ptr(dzr.contiguous()), ptrs, ctot, coff, acc, ptr(prev_zr), ptr(prev_q),
                                         ptr(prev_h), ptr(prev_dq), ptr(prev_dzr), ptr(prev_dh),
                                         int(prev_dh_accumulate), ptr(ws), nws, stream_of(dzr)),
          "dro_convgru_gates_backward")


@_gru_gates_bwd_op.register_fake
def _(srcs, weight, dzr, grad_srcs, accumulate, prev_zr, prev_q, prev_h, prev_dq, prev_dzr, prev_dh,
      prev_dh_accumulate):
    return None


_GRU_FOLD = os.environ.get("DRO_GRU_FOLD", "1") != "0"   # A/B: 0 keeps the separate stage-2 launch
# A/B: 0 keeps the first half's stage-1 launch (DRO_GRU_FOLD=0 implies it)
_GRU_CHAIN = _GRU_FOLD and os.environ.get("DRO_GRU_CHAIN", "1") != "0"


class GruChain:
    """Links the two halves of one SepConvGRU (SepConvGRU.forward): the second
    half's gate-conv data gradient finishes d h = the first half's dh' and runs
    the first half's stage 1 in its epilogue.  Only built for the two halves of
    one GRU, whose middle state nothing else reads."""
    __slots__ = ("first", "hn_ptr", "direct", "zr", "q", "h", "hsink", "done", "dq", "dzr", "dh", "h_in_sink")
    folded = 0   # backward passes that ran a first half's stage 1 in the epilogue (tests)
    stats = {"first": 0, "second": 0, "linked": 0, "bwd_linked": 0}   # (tests: why a link did not form)

    def __init__(self):
        self.first = False
        self.done = False
        self.hn_ptr = None


_SEPGRU_CHAIN = []   # the GruChain of the call being set up (sepconvgru_half)


# ------------------------------------------------------------------ dro::sepconvgru_half
@torch.library.custom_op("dro::sepconvgru_half", mutates_args=())
def _sepgru_op(h: Tensor, wz: Tensor, bz: Tensor, wr: Tensor, br: Tensor, wq: Tensor, bq: Tensor, xs: list[Tensor],
               wzr: Optional[Tensor], bzr: Optional[Tensor]) -> tuple[Tensor, Tensor, Tensor, Tensor]:
    """One direction of SepConvGRU (update.py:59-70): z, r = sigmoid(conv([h; x]));
    q = tanh(conv([r*h; x])); h' = (1-z) h + z q, x given as sources (virtual
    concat).  wzr/bzr: the fused z|r weight/bias when the caller has them (a
    flat-buffer view or a per-forward concatenation), else built here.
    Returns (h', z|r, r*h, q); the last three are saved for the backward."""
    lib = _lib.load()
    require_device(h, wz, wq, *xs, what="sepconvgru")
    h = h.contiguous()
    B, hd, H, W = h.shape
    KH, KW = wz.shape[2:]
    cin = wz.shape[1]
    if wzr is None:
        wzr = torch.cat([wz, wr], 0).contiguous()
        bzr = torch.cat([bz, br], 0).contiguous()
    st = stream_of(h)
    zr = torch.empty(B, 2 * hd, H, W, device=h.device)
    rh = torch.empty_like(h)
    ws, nws = _workspace(B, H, W, cin, 2 * hd, KH, KW, h.device)
    wq = wq.contiguous()
    zf, zb = _wsplit(wzr)
    qf, qb = _wsplit(wq)
    check(lib.dro_convgru_gates_forward(_slices([h, *xs]), 1 + len(xs), ptr(wzr), ptr(bzr), B, H, W, hd,
                                        KH, KW, ptr(zr), ptr(rh), ptr(zf), ptr(ws), nws, st),
          "dro_convgru_gates_forward")
    q = torch.empty_like(h)
    hn = torch.empty_like(h)
    z_sl = DroSlice(zr.data_ptr(), hd, 2 * hd, 0, 0)
    h_sl = DroSlice(h.data_ptr(), hd, hd, 0, 0)
    wsq, nwsq = _workspace(B, H, W, cin, hd, KH, KW, h.device)
    check(lib.dro_convgru_blend_forward(_slices([rh, *xs]), 1 + len(xs), ptr(wq), ptr(bq),
                                        B, H, W, hd, KH, KW, ctypes.byref(z_sl), ctypes.byref(h_sl),
                                        ptr(q), ptr(hn), hd, 0, ptr(qf), ptr(wsq), nwsq, st),
          "dro_convgru_blend_forward")
    return hn, zr, rh, q


@_sepgru_op.register_fake
def _(h, wz, bz, wr, br, wq, bq, xs, wzr, bzr):
    B, hd, H, W = h.shape
    return h.new_empty(h.shape), h.new_empty((B, 2 * hd, H, W)), h.new_empty(h.shape), h.new_empty(h.shape)


def _sepgru_setup(ctx, inputs, output):
    h, wz, bz, wr, br, wq, bq, xs, wzr_in, bzr_in = inputs
    hn, zr, rh, q = output
    # the fused z|r weight the implementation ran with (sepconvgru_half always
    # passes one; a direct op call without it gets the same concatenation)
    wzr = wzr_in if wzr_in is not None else torch.cat([wz, wr], 0).detach().contiguous()
    ctx.wsplit = (_wsplit_bwd(wzr), _wsplit_bwd(wq.contiguous()))
    hc = h.contiguous()    # the dense state both this half's and a linked second half's backward read
    ctx.save_for_backward(hc, rh, wzr, wq.contiguous(), zr, q, *xs)
    ctx.mark_non_differentiable(zr, rh, q)
    ctx.set_materialize_grads(False)     # no zero-filled gradients for the three saved outputs
    ctx.sinks = [_sink_of(x) if x.requires_grad else None for x in xs]
    ctx.hsink = _sink_of(h) if h.requires_grad else None
    ctx.need = (h.requires_grad, [x.requires_grad for x in xs],
                any(t.requires_grad for t in (wz, bz, wr, br)), any(t.requires_grad for t in (wq, bq)))
    ctx.scope = current_scope()
    ctx.keys = (("zr", wz.data_ptr(), wr.data_ptr()), ("q", wq.data_ptr()))
    ctx.direct = _SEPGRU_DIRECT.pop() if _SEPGRU_DIRECT else None
    chain = _SEPGRU_CHAIN.pop() if _SEPGRU_CHAIN else None
    ctx.chain_first = ctx.chain_prev = None
    if chain is not None and _GRU_CHAIN:
        GruChain.stats["second" if chain.first else "first"] += 1
        if not chain.first:
            chain.first = True
            chain.hn_ptr = hn.data_ptr()
            chain.direct = ctx.direct is not None
            chain.zr, chain.q, chain.h, chain.hsink = zr, q, hc, ctx.hsink
            ctx.chain_first = chain
        elif chain.hn_ptr == h.data_ptr() and chain.direct and ctx.direct is not None and h.requires_grad:
            ctx.chain_prev = chain
            GruChain.stats["linked"] += 1


_SEPGRU_DIRECT = []   # the in-place weight-gradient targets of the call being set up (sepconvgru_half)


def _sepgru_backward(ctx, dhn, _gzr, _grh, _gq):
    h, rh, wzr, wq, zr, q, *xs = ctx.saved_tensors
    B, hd, H, W = h.shape
    need_h, need_x, need_zr_w, need_q_w = ctx.need
    if dhn is None:
        return (None,) * 7 + ([None] * len(xs), None, None)
    dhn = dhn.contiguous()
    first = ctx.chain_first
    if first is not None and first.done:
        # stage 1 already ran in the second half's gate-conv epilogue; the link is
        # one-shot: a second backward through the graph (retain_graph) finds the
        # chain's tensors released and runs both halves unlinked
        dq, dzr, dh, h_in_sink = first.dq, first.dzr, first.dh, first.h_in_sink
        first.dq = first.dzr = first.dh = first.zr = first.q = first.h = first.hsink = None
        first.done = False
    else:
        # stage 1: pre-activation grads of q and z, dh = dh' (1-z).  When h has a
        # gradient sink that no consumer has written yet (the next GRU step runs its
        # backward before the heads that also read this state), dh is built right in
        # the sink and autograd gets None for h (no add launch)
        dq = torch.empty_like(h)
        h_in_sink = ctx.hsink is not None and not ctx.hsink.written
        dh = ctx.hsink.target()[0] if h_in_sink else torch.empty_like(h)
        dzr = torch.empty_like(zr)
        torch.ops.dro.gru_backward_elem(1, dhn, zr, q, h, None, dq, dzr, dh)
    # candidate conv over [r*h, x]: d(r*h), dx (overwrite); sources with a
    # gradient sink are accumulated in place and get None from autograd
    drh = torch.empty_like(h)
    sinks = ctx.sinks
    dxs = [torch.empty(B, x.shape[1], H, W, device=h.device) if need_x[i] and sinks[i] is None
           else None for i, x in enumerate(xs)]
    sk = [sn.target() if sn is not None else (None, 0) for sn in sinks]
    tg = [t if sn is not None else d for (t, _), sn, d in zip(sk, sinks, dxs)]
    qacc0 = [0] + [a for _, a in sk]
    zb, qb = ctx.wsplit
    nones = (None,) * 6
    if ctx.direct is not None:
        (_, _), (gwzr, gbzr), (gwq, gbq) = ctx.direct
        if _GRU_FOLD and qb is None:
            # d(r*h) goes straight into stage 2 in the data gradient's epilogue
            torch.ops.dro.convgru_candidate_backward([rh, *xs], wq, dq, zr, h, dzr, dh,
                                                     [_placeholder(t, h.device) for t in [None, *tg]], qacc0)
        else:
            _conv_bwd([rh, *xs], wq, None, dq, 0, 1.0, [drh, *tg], qacc0, wsplit=qb)
        if not _queue_weight_grad([rh, *xs], wq.shape, 0, 1.0, dq, None, gwq, gbq):
            _conv_bwd([rh, *xs], wq, None, dq, 0, 1.0, [None] * (1 + len(xs)), [0] * (1 + len(xs)), gwq, gbq, 1)
        if not (_GRU_FOLD and qb is None):
            torch.ops.dro.gru_backward_elem(2, None, zr, None, h, drh, None, dzr, dh)
        p = ctx.chain_prev
        if p is not None:
            GruChain.stats["bwd_linked"] += 1
        if p is not None and p.h is None:
            p = None           # the chain was consumed by an earlier backward pass
        if p is not None and zb is None:
            # this half's d h, once finished, is the first half's dh': its stage 1
            # runs in the gate conv's epilogue (dq, dzr, dh of the first half; dh
            # straight into the first half's input sink when it has one)
            p.dq, p.dzr = torch.empty_like(p.h), torch.empty_like(p.zr)
            if p.hsink is not None:
                p.dh, pacc = p.hsink.target()
                p.h_in_sink = True
            else:
                p.dh, pacc, p.h_in_sink = torch.empty_like(p.h), 0, False
            torch.ops.dro.convgru_gates_backward([h, *xs], wzr, dzr, [dh, *[_placeholder(t, h.device) for t in tg]],
                                                 [1] * (1 + len(xs)), p.zr, p.q, p.h, p.dq, p.dzr, p.dh, pacc)
            p.done = True
            GruChain.folded += 1
        else:
            _conv_bwd([h, *xs], wzr, None, dzr, 0, 1.0, [dh, *tg], [1] * (1 + len(xs)), wsplit=zb)
        if not _queue_weight_grad([h, *xs], wzr.shape, 0, 1.0, dzr, None, gwzr, gbzr):
            _conv_bwd([h, *xs], wzr, None, dzr, 0, 1.0, [None] * (1 + len(xs)), [0] * (1 + len(xs)), gwzr, gbzr, 1)
        return (dh if need_h and not h_in_sink else None, *nones, dxs, None, None)
    gwq, gbq, qacc, qfirst = _grad_buffers(ctx.scope, ctx.keys[1], wq, hd, h.device)
    _conv_bwd([rh, *xs], wq, None, dq, 0, 1.0, [drh, *tg], qacc0, gwq, gbq, qacc, qb)
    # stage 2: pre-activation grad of r, dh += d(r*h) r
    torch.ops.dro.gru_backward_elem(2, None, zr, None, h, drh, None, dzr, dh)
    # gate conv over [h, x]: dh, dx accumulate; dWz|dWr, dbz|dbr
    gwzr, gbzr, zacc, zfirst = _grad_buffers(ctx.scope, ctx.keys[0], wzr, 2 * hd, h.device)
    _conv_bwd([h, *xs], wzr, None, dzr, 0, 1.0, [dh, *tg], [1] * (1 + len(xs)), gwzr, gbzr, zacc, zb)
    gz = (gwzr[:hd], gbzr[:hd], gwzr[hd:], gbzr[hd:]) if (zfirst and need_zr_w) else (None,) * 4
    gq = (gwq, gbq) if (qfirst and need_q_w) else (None, None)
    return (dh if need_h and not h_in_sink else None, *gz, *gq, dxs, None, None)


torch.library.register_autograd("dro::sepconvgru_half", _sepgru_backward, setup_context=_sepgru_setup)


def sepconvgru_half(h, convz, convr, convq, xs, chain=None):
    """h' for one SepConvGRU direction; xs: the input sources (virtual concat).
    chain: one GruChain shared by the two halves of one SepConvGRU (the
    second half's backward then runs the first half's stage 1).
    torch.ops.dro.sepconvgru_half."""
    direct = None
    zr = _direct_targets((convz.weight, convr.weight), (convz.bias, convr.bias), mark=False)
    if zr is not None:
        qd = _direct_targets((convq.weight,), (convq.bias,), mark=False)
        if qd is not None:
            direct = ((zr[0], zr[1]), (zr[2], zr[3]), (qd[2], qd[3]))
            _mark_direct([convz.weight, convz.bias, convr.weight, convr.bias, convq.weight, convq.bias])
    scope = current_scope()
    if direct is not None:
        wzr, bzr = direct[0]
    else:
        key = ("zr", convz.weight.data_ptr(), convr.weight.data_ptr())
        ent = scope.cats.get(key) if scope is not None else None
        if ent is None:
            ent = (torch.cat([convz.weight, convr.weight], 0).detach().contiguous(),
                   torch.cat([convz.bias, convr.bias], 0).detach().contiguous())
            if scope is not None:
                scope.cats[key] = ent
        wzr, bzr = ent
    _SEPGRU_DIRECT[:] = [direct] if direct is not None else []
    _SEPGRU_CHAIN[:] = [chain] if chain is not None else []
    try:
        return torch.ops.dro.sepconvgru_half(h, convz.weight, convz.bias, convr.weight, convr.bias, convq.weight,
                                             convq.bias, list(xs), wzr, bzr)[0]
    finally:
        _SEPGRU_DIRECT.clear()
        _SEPGRU_CHAIN.clear()
