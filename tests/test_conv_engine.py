"""GPU parity of the f32-MFMA convolution engine (csrc/conv.hip) against
torch.nn.functional.conv2d evaluated in fp64 on the CPU.

Shapes are the update-block convolutions of networks/optim/update.py
(reference dro_sfm/networks/optim/update.py:5-199) at a reduced pixel count:
SepConvGRU 1x5 / 5x1 gates over [h, context, projection, depth|pose-map]
virtual concatenations, projection-encoder 7x7/3x3/1x1 convs, heads, the
0.25-scaled mask conv.  Tolerance 1e-4 relative (max|a-b| / max|b|), the
north_star bound; f32 MFMA accumulates in exact fp32, the split-bf16 engine
sums six bf16 products per term (dropped terms < 2^-24 |ab|) in fp32.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL = 1e-4


@pytest.fixture(scope="module")
def hip():
    import dro_sfm_amd.hip as H
    from dro_sfm_amd.hip import _lib
    _lib.load()
    return H


@pytest.fixture(params=["split", "f32"])
def engine(request, hip):
    """Both engines: split-bf16 MFMA (csrc/xconv.hip, 1x5/5x1/3x3/1x1) and f32 MFMA
    (csrc/conv.hip, the default); the same f32-level tolerance for both."""
    from dro_sfm_amd.hip import conv as C
    C.set_split_engine(request.param == "split")
    prev = C._XCONV[0]
    yield request.param
    C.set_split_engine(prev)


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


ACTS = {None: lambda x: x, "relu": torch.relu, "sigmoid": torch.sigmoid, "tanh": torch.tanh}


def make_src(kind, B, C, H, W, g):
    """kind: 'dense' | 'slice' (channel slice of a wider tensor) | 'bcast' ([B,C,1,1] expanded)."""
    if kind == "bcast":
        base = torch.randn(B, C, 1, 1, generator=g)
        return base, lambda t: t.expand(B, C, H, W)
    if kind == "slice":
        base = torch.randn(B, C + 5, H, W, generator=g)
        return base, lambda t: t[:, 3:3 + C]
    base = torch.randn(B, C, H, W, generator=g)
    return base, lambda t: t


CASES = [
    # (sources [(kind, C)], Cout, (KH, KW), act, alpha, B, H, W)
    ([("dense", 128), ("dense", 128), ("dense", 63), ("dense", 1)], 256, (1, 5), "sigmoid", 1.0, 2, 24, 80),
    ([("dense", 128), ("slice", 128), ("dense", 58), ("bcast", 6)], 128, (5, 1), "tanh", 1.0, 2, 24, 80),
    ([("slice", 64)], 64, (3, 3), "relu", 1.0, 2, 24, 80),
    ([("dense", 1)], 128, (7, 7), "relu", 1.0, 2, 24, 80),
    ([("bcast", 6)], 128, (7, 7), "relu", 1.0, 2, 24, 80),
    ([("dense", 64), ("dense", 64)], 63, (3, 3), "relu", 1.0, 2, 24, 80),
    ([("slice", 128)], 576, (1, 1), None, 0.25, 2, 24, 80),
    ([("dense", 128)], 1, (3, 3), "tanh", 1.0, 2, 24, 80),
    ([("dense", 128)], 6, (3, 3), None, 1.0, 4, 24, 80),
    ([("dense", 37), ("slice", 11)], 45, (5, 3), "sigmoid", 1.0, 3, 7, 13),
    # thin 7x7 path (<= 8 input channels): ragged tiles, Cout not a multiple of 16
    ([("dense", 3)], 20, (7, 7), "tanh", 1.0, 3, 13, 21),
    ([("slice", 8)], 64, (7, 7), None, 0.5, 2, 9, 11),
]


@pytest.mark.parametrize("case", range(len(CASES)))
def test_conv2d_fwd_bwd(hip, engine, case):
    srcs_spec, Cout, (KH, KW), act, alpha, B, H, W = CASES[case]
    g = torch.Generator().manual_seed(100 + case)
    bases, views = zip(*[make_src(k, B, C, H, W, g) for k, C in srcs_spec])
    Cin = sum(C for _, C in srcs_spec)
    w = torch.randn(Cout, Cin, KH, KW, generator=g) / (Cin * KH * KW) ** 0.5
    b = torch.randn(Cout, generator=g) * 0.1
    gout = torch.randn(B, Cout, H, W, generator=g)

    # fp64 reference on the CPU
    rb = [x.double().requires_grad_() for x in bases]
    rw, rbias = w.double().requires_grad_(), b.double().requires_grad_()
    db = [x.to(DEV).requires_grad_() for x in bases]
    dw, dbias = w.to(DEV).requires_grad_(), b.to(DEV).requires_grad_()
    out = hip.conv2d([v(t) for v, t in zip(views, db)], dw, dbias, act=act, alpha=alpha)
    out.backward(gout.to(DEV))
    torch.cuda.synchronize()

    x = torch.cat([v(t) for v, t in zip(views, rb)], 1)
    pre = F.conv2d(x, rw, rbias, padding=(KH // 2, KW // 2))
    if act == "relu":   # take relu's on/off decision from the fp32 result: a pre-activation
        ref = pre * (out.detach().cpu() > 0).double()   # within fp32 rounding of 0 may flip
    else:
        ref = ACTS[act](pre) * alpha
    ref.backward(gout.double())
    assert rel(out, ref) < TOL
    assert rel(dw.grad, rw.grad) < TOL
    assert rel(dbias.grad, rbias.grad) < TOL
    for i, (a, r) in enumerate(zip(db, rb)):
        assert rel(a.grad, r.grad) < TOL, f"source {i}"


def _gru_ref(h, xs, wz, bz, wr, br, wq, bq, pad):
    hx = torch.cat([h, *xs], 1)
    z = torch.sigmoid(F.conv2d(hx, wz, bz, padding=pad))
    r = torch.sigmoid(F.conv2d(hx, wr, br, padding=pad))
    q = torch.tanh(F.conv2d(torch.cat([r * h, *xs], 1), wq, bq, padding=pad))
    return (1 - z) * h + z * q


@pytest.mark.parametrize("kernel", [(1, 5), (5, 1)])
@pytest.mark.parametrize("pose", [False, True])
def test_sepconvgru_half(hip, engine, kernel, pose):
    """One SepConvGRU direction (update.py:59-70) fused: 2 launches forward."""
    B, hd, H, W = 2, 64, 24, 40
    g = torch.Generator().manual_seed(7 + pose)
    KH, KW = kernel
    pad = (KH // 2, KW // 2)
    spec = [("slice", 64), ("dense", 58), ("bcast", 6)] if pose else [("dense", 64), ("dense", 63), ("dense", 1)]
    bases, views = zip(*[make_src(k, B, C, H, W, g) for k, C in spec])
    h = torch.randn(B, hd, H, W, generator=g).tanh()
    cin = hd + sum(C for _, C in spec)
    ws = [torch.randn(hd, cin, KH, KW, generator=g) / (cin * KH * KW) ** 0.5 for _ in range(3)]
    bs = [torch.randn(hd, generator=g) * 0.1 for _ in range(3)]
    gout = torch.randn(B, hd, H, W, generator=g)

    rp = [t.double().requires_grad_() for t in (h, *bases, *ws, *bs)]
    rh, rbases, rws, rbs = rp[0], rp[1:1 + len(bases)], rp[1 + len(bases):4 + len(bases)], rp[4 + len(bases):]
    ref = _gru_ref(rh, [v(t) for v, t in zip(views, rbases)], rws[0], rbs[0], rws[1], rbs[1], rws[2], rbs[2], pad)
    ref.backward(gout.double())

    dp = [t.to(DEV).requires_grad_() for t in (h, *bases, *ws, *bs)]
    dh, dbases, dws, dbs = dp[0], dp[1:1 + len(bases)], dp[1 + len(bases):4 + len(bases)], dp[4 + len(bases):]
    convs = [torch.nn.Conv2d(cin, hd, kernel, padding=pad).to(DEV) for _ in range(3)]
    for c, w_, b_ in zip(convs, dws, dbs):     # route the leaves through conv-shaped holders
        c.weight, c.bias = torch.nn.Parameter(w_), torch.nn.Parameter(b_)
    out = hip.sepconvgru_half(dh, convs[0], convs[1], convs[2], [v(t) for v, t in zip(views, dbases)])
    out.backward(gout.to(DEV))
    torch.cuda.synchronize()
    assert rel(out, ref) < TOL
    assert rel(dh.grad, rh.grad) < TOL
    for i, (a, r) in enumerate(zip(dbases, rbases)):
        assert rel(a.grad, r.grad) < TOL, f"x{i}"
    for i, (c, rw, rb) in enumerate(zip(convs, rws, rbs)):
        assert rel(c.weight.grad, rw.grad) < TOL, f"W{i}"
        assert rel(c.bias.grad, rb.grad) < TOL, f"b{i}"


def test_conv2d_rejects_bad_layout(hip):
    x = torch.randn(2, 8, 6, 10, device=DEV).permute(0, 1, 3, 2)
    w = torch.randn(4, 8, 3, 3, device=DEV)
    with pytest.raises(RuntimeError):
        hip.conv2d([x], w)
    with pytest.raises(RuntimeError):
        hip.conv2d([torch.randn(2, 7, 6, 6, device=DEV)], w)


def test_weight_grad_scope_matches_autograd(hip):
    """A weight shared by several convs / GRU steps of one forward: summing its
    gradient in-kernel (weight_grad_scope) equals autograd's own accumulation."""
    g = torch.Generator(device=DEV).manual_seed(11)
    B, hd, H, W = 2, 64, 12, 20
    convs = [torch.nn.Conv2d(hd + 32, hd, (1, 5), padding=(0, 2)).to(DEV) for _ in range(3)]
    head = torch.nn.Conv2d(hd, hd, 3, padding=1).to(DEV)
    h0 = torch.randn(B, hd, H, W, device=DEV, generator=g).tanh()
    x = torch.randn(B, 32, H, W, device=DEV, generator=g)
    params = [p for c in convs + [head] for p in c.parameters()]

    def run(scoped):
        for p in params:
            p.grad = None
        ctxm = hip.weight_grad_scope() if scoped else torch.enable_grad()
        with ctxm:
            h = h0
            for _ in range(3):
                h = hip.sepconvgru_half(h, *convs, [x])
                h = hip.conv2d([h], head.weight, head.bias, act="tanh")
            loss = (h * h).sum()
        loss.backward()
        torch.cuda.synchronize()
        return [p.grad.detach().clone() for p in params]

    ref, got = run(False), run(True)
    for i, (a, r) in enumerate(zip(got, ref)):
        assert rel(a, r) < 1e-5, f"param {i}"


MULTI_CASES = [
    # (sources [(kind, C)], Cout, (KH, KW), act, alpha, uses, B, H, W)
    ([("dense", 64), ("dense", 32), ("dense", 63), ("dense", 1)], 128, (1, 5), None, 1.0, 8, 2, 24, 80),
    ([("dense", 64), ("slice", 32), ("dense", 58), ("bcast", 6)], 64, (5, 1), None, 1.0, 3, 4, 24, 80),
    ([("slice", 64)], 96, (3, 3), "relu", 1.0, 5, 2, 24, 80),
    ([("dense", 128)], 6, (3, 3), "tanh", 1.0, 17, 2, 12, 20),
    ([("slice", 128)], 576, (1, 1), None, 0.25, 4, 2, 24, 80),
    ([("dense", 37), ("slice", 11)], 45, (3, 3), "sigmoid", 1.0, 2, 3, 7, 13),
    # the encoders' shapes: fnet layer1 at the KITTI metric batch (the bench
    # roofline call), layer3 with 64-row output tiles
    ([("dense", 64)], 64, (3, 3), None, 1.0, 1, 6, 48, 160),
    ([("dense", 256)], 256, (3, 3), "relu", 1.0, 2, 2, 12, 40),
]


@pytest.mark.parametrize("case", range(len(MULTI_CASES)))
def test_weight_grad_multi(hip, case):
    """dro_conv2d_weight_grad_multi: the weight + bias gradient of ONE weight over
    several uses (own sources, output gradients and saved outputs) in one
    launch, accumulated onto the existing gradient, equals the fp64 sum of the
    per-use autograd gradients (more than 16 uses: chunked by the caller)."""
    import ctypes
    from dro_sfm_amd.hip import _lib
    from dro_sfm_amd.hip.conv import DroWgradUse, _slices
    lib = _lib.load()
    spec, Cout, (KH, KW), act, alpha, uses, B, H, W = MULTI_CASES[case]
    g = torch.Generator().manual_seed(100 + case)
    Cin = sum(c for _, c in spec)
    w = 0.1 * torch.randn(Cout, Cin, KH, KW, generator=g)
    b = 0.1 * torch.randn(Cout, generator=g)
    gw_ref = torch.zeros(Cout, Cin, KH, KW, dtype=torch.float64)
    gb_ref = torch.zeros(Cout, dtype=torch.float64)
    dev_uses = []
    for _ in range(uses):
        bases, views = zip(*[make_src(k, B, c, H, W, g) for k, c in spec])
        dout = torch.randn(B, Cout, H, W, generator=g)
        wd = w.double().requires_grad_(True)
        bd = b.double().requires_grad_(True)
        x = torch.cat([v(t.double()) for v, t in zip(views, bases)], 1)
        y = alpha * ACTS[act](F.conv2d(x, wd, bd, padding=(KH // 2, KW // 2)))
        (y * dout.double()).sum().backward()
        gw_ref += wd.grad
        gb_ref += bd.grad
        srcs = [v(t.to(DEV)) for v, t in zip(views, bases)]
        dev_uses.append((srcs, dout.to(DEV), y.detach().float().to(DEV) if act else None))
    init_w = torch.randn(Cout, Cin, KH, KW, generator=g)
    init_b = torch.randn(Cout, generator=g)
    gw, gb = init_w.to(DEV), init_b.to(DEV)
    keep = []
    for c0 in range(0, uses, 16):
        chunk = dev_uses[c0:c0 + 16]
        arr = (DroWgradUse * len(chunk))()
        for i, (srcs, dout, y) in enumerate(chunk):
            sl = _slices(srcs)
            keep.append(sl)
            arr[i].srcs = ctypes.cast(sl, ctypes.c_void_p)
            arr[i].dout = dout.data_ptr()
            arr[i].y = y.data_ptr() if y is not None else None
        nb = lib.dro_conv2d_weight_grad_multi_workspace_bytes(len(chunk), B, H, W, Cin, Cout, KH, KW)
        ws = torch.empty(nb, dtype=torch.uint8, device=DEV)
        st = lib.dro_conv2d_weight_grad_multi(arr, len(chunk), len(spec), B, H, W, Cout, KH, KW,
                                              {None: 0, "relu": 1, "sigmoid": 2, "tanh": 3}[act],
                                              ctypes.c_float(alpha), gw.data_ptr(), gb.data_ptr(), 1,
                                              ws.data_ptr(), nb, None)
        assert st == 0, lib.dro_last_error()
    torch.cuda.synchronize()
    assert rel(gw - init_w.to(DEV), gw_ref) < TOL
    assert rel(gb - init_b.to(DEV), gb_ref) < TOL


def test_weight_grad_multi_rejects(hip):
    import ctypes
    from dro_sfm_amd.hip import _lib
    from dro_sfm_amd.hip.conv import DroWgradUse, _slices
    lib = _lib.load()
    B, H, W = 1, 8, 8
    x1 = torch.randn(B, 8, H, W, device=DEV)
    a, b_ = torch.randn(B, 3, H, W, device=DEV), torch.randn(B, 5, H, W, device=DEV)
    dout = torch.randn(B, 4, H, W, device=DEV)
    gw = torch.zeros(4, 8, 3, 3, device=DEV)
    s1, s2 = _slices([x1]), _slices([a, b_])
    arr = (DroWgradUse * 17)()
    for i in range(17):
        arr[i].srcs = ctypes.cast(s1, ctypes.c_void_p)
        arr[i].dout = dout.data_ptr()
    args = (B, H, W, 4, 3, 3, 0, ctypes.c_float(1.0), gw.data_ptr(), None, 1, None, 0, None)
    assert lib.dro_conv2d_weight_grad_multi(arr, 17, 1, *args) == -2          # > 16 uses
    assert lib.dro_conv2d_weight_grad_multi(arr, 1, 1, B, H, W, 4, 7, 7, 0, ctypes.c_float(1.0),
                                            gw.data_ptr(), None, 1, None, 0, None) == -2   # 7x7
    two = (DroWgradUse * 2)()
    two[0].srcs, two[0].dout = ctypes.cast(s2, ctypes.c_void_p), dout.data_ptr()
    two[1].srcs, two[1].dout = ctypes.cast(s2, ctypes.c_void_p), dout.data_ptr()
    assert lib.dro_conv2d_weight_grad_multi(two, 2, 2, *args) == -2           # no workspace
    assert lib.dro_conv2d_weight_grad_multi(arr, 1, 1, B, H, W, 4, 3, 3, 1, ctypes.c_float(1.0),
                                            gw.data_ptr(), None, 1, None, 0, None) == -1   # relu, no y


def test_weight_split_exact(hip):
    """dro_weight_split: the three bf16 planes sum back to the f32 weight (within
    2^-24 relative per element, the f32 rounding unit) in both layouts; padded
    channels are zero; the data-gradient layout is the transposed, tap-flipped
    weight."""
    import ctypes  # noqa: F401
    from dro_sfm_amd.hip import _lib
    lib = _lib.load()
    g = torch.Generator().manual_seed(5)
    Cout, Cin, KH, KW = 45, 37, 3, 3
    T = KH * KW
    w = torch.randn(Cout, Cin, KH, KW, generator=g) * torch.logspace(-6, 3, Cout).view(-1, 1, 1, 1)
    wd = w.to(DEV)
    nf = lib.dro_weight_split_bytes(Cout, Cin, KH, KW, 0)
    nb = lib.dro_weight_split_bytes(Cout, Cin, KH, KW, 1)
    fw = torch.empty(nf // 2, dtype=torch.int16, device=DEV)
    bw = torch.empty(nb // 2, dtype=torch.int16, device=DEV)
    assert lib.dro_weight_split(_lib.ptr(wd), Cout, Cin, KH, KW, _lib.ptr(fw), _lib.ptr(bw), None) == 0
    torch.cuda.synchronize()

    def planes(buf, rows, kc):
        nch = (kc + 31) // 32
        p = buf.cpu().view(torch.bfloat16).float().view(3, rows, nch, T, 32)
        return (p[0].double() + p[1].double() + p[2].double()), p
    s, p = planes(fw, Cout, Cin)
    ref = w.permute(0, 1, 2, 3).reshape(Cout, Cin, T).double()
    got = s.permute(0, 1, 3, 2).reshape(Cout, -1, T)[:, :Cin]        # [Cout][c][tap]
    assert ((got - ref).abs() <= ref.abs() * 2.0 ** -24).all()
    assert (s.permute(0, 1, 3, 2).reshape(Cout, -1, T)[:, Cin:] == 0).all()
    s, _ = planes(bw, Cin, Cout)
    refb = w.reshape(Cout, Cin, T).flip(2).permute(1, 0, 2).double()  # [Cin][o][flipped tap]
    gotb = s.permute(0, 1, 3, 2).reshape(Cin, -1, T)[:, :Cout]
    assert ((gotb - refb).abs() <= refb.abs() * 2.0 ** -24).all()


@pytest.mark.parametrize("case", [
    # (B, Cin, Cout, Hi, Wi, k, stride, pad, bias, act): the encoders' strided convs
    (2, 64, 128, 48, 160, 3, 2, 1, False, None),     # layer2 stage entry (KITTI cnet_depth)
    (2, 128, 256, 24, 80, 3, 2, 1, False, None),     # layer3 stage entry
    (2, 64, 128, 48, 160, 1, 2, 0, False, None),     # 1x1/s2 downsample
    (2, 3, 64, 64, 96, 7, 2, 3, False, None),        # 7x7/s2 stem (3 channels)
    (1, 6, 64, 47, 81, 7, 2, 3, False, None),        # cnet_pose stem, odd input size
    (2, 6, 64, 192, 640, 7, 2, 3, False, None),      # KITTI-size stem (wgrad_k7_kernel: 240 tiles per image)
    (2, 20, 24, 17, 23, 3, 2, 1, True, "relu"),      # odd sizes, bias + relu forward
    (2, 16, 40, 12, 20, 3, 1, 0, True, None),        # stride 1, no padding
    (2, 20, 24, 17, 23, 3, 2, 1, True, None),        # odd sizes: parity classes of unequal size
    (3, 10, 12, 9, 7, 1, 2, 0, False, None),         # 1x1/s2, odd: three classes get no tap
    (2, 5, 8, 10, 13, 4, 2, 1, False, None),         # even kernel: every class has 2x2 taps
    # the ScanNet view5 fixture's fnet (5 frames of 64x96)
    (5, 3, 64, 64, 96, 7, 2, 3, False, None),
    (5, 64, 128, 16, 24, 3, 2, 1, False, None),
    (5, 64, 128, 16, 24, 1, 2, 0, False, None),
    (5, 128, 256, 8, 12, 3, 2, 1, False, None),
])
def test_conv2d_strided(hip, case):
    """hip.conv2d_strided (dro_conv2d_strided_*: flattened implicit GEMM with
    the stride, generic weight gradient) against fp64 F.conv2d: output, input
    gradient, weight and bias gradients; 1e-4."""
    B, Cin, Cout, Hi, Wi, k, stride, pad, use_bias, act = case
    g = torch.Generator().manual_seed(Cin * 7 + Cout)
    x = torch.randn(B, Cin, Hi, Wi, generator=g)
    w = torch.randn(Cout, Cin, k, k, generator=g) / (Cin * k * k) ** 0.5
    b = torch.randn(Cout, generator=g) if use_bias else None
    xr, wr = x.double().requires_grad_(), w.double().requires_grad_()
    br = b.double().requires_grad_() if use_bias else None
    ref = ACTS[act](F.conv2d(xr, wr, br, stride=stride, padding=pad))
    G = torch.randn(ref.shape, generator=g)
    xd, wd = x.to(DEV).requires_grad_(), w.to(DEV).requires_grad_()
    bd = b.to(DEV).requires_grad_() if use_bias else None
    if act is None:
        out = hip.conv2d_strided(xd, wd, bd, stride, pad)
        assert out.shape == ref.shape and rel(out, ref) < TOL
        (ref * G.double()).sum().backward()
        (out * G.to(DEV)).sum().backward()
        assert rel(xd.grad, xr.grad) < TOL
        assert rel(wd.grad, wr.grad) < TOL
        if use_bias:
            assert rel(bd.grad, br.grad) < TOL
    else:
        with torch.no_grad():
            out = hip.conv2d_strided(xd, wd, bd, stride, pad, act=act)
        assert out.shape == ref.shape and rel(out, ref) < TOL


def test_pose_mean(hip):
    """hip.pose_mean (PoseHead spatial mean + rotation scale + pose update,
    update.py:16-28, 189-197) against fp64 torch: value and both gradients."""
    g = torch.Generator().manual_seed(4)
    y = torch.randn(4, 6, 24, 80, generator=g)
    pose = torch.randn(4, 6, generator=g)
    G = torch.randn(4, 6, generator=g)
    scale = torch.tensor([1.0, 1.0, 1.0, 0.01, 0.01, 0.01], dtype=torch.float64)
    yr, pr = y.double().requires_grad_(), pose.double().requires_grad_()
    ref = pr + yr.mean(dim=(2, 3)) * scale
    (ref * G.double()).sum().backward()
    yd, pd = y.to(DEV).requires_grad_(), pose.to(DEV).requires_grad_()
    out = hip.pose_mean(yd, 0.01, pd)
    (out * G.to(DEV)).sum().backward()
    assert rel(out, ref) < TOL and rel(yd.grad, yr.grad) < TOL and rel(pd.grad, pr.grad) < TOL
    assert rel(hip.pose_mean(yd.detach(), 0.01), yr.detach().mean(dim=(2, 3)) * scale) < TOL


@pytest.mark.parametrize("kernel,B,hd,H,W", [((1, 5), 2, 32, 24, 80), ((5, 1), 4, 32, 24, 80),
                                              ((3, 3), 2, 64, 13, 37), ((1, 5), 1, 8, 5, 7)])
def test_convgru_candidate_backward_matches_unfused(hip, kernel, B, hd, H, W):
    """The candidate conv's data gradient with SepConvGRU stage 2 in its
    epilogue (dro_convgru_candidate_backward, ABI 8) against the two-launch
    form (conv2d_backward into d(r*h), then gru_backward_elem stage 2): dzr
    (both halves), dh (accumulated into) and the other sources' gradients
    (one overwritten, one accumulated) bit for bit."""
    g = torch.Generator(device=DEV).manual_seed(5)
    KH, KW = kernel
    cx = (24, 10)
    rh = torch.randn(B, hd, H, W, device=DEV, generator=g)
    xs = [torch.randn(B, c, H, W, device=DEV, generator=g) for c in cx]
    wq = torch.randn(hd, hd + sum(cx), KH, KW, device=DEV, generator=g) * 0.05
    dq = torch.randn(B, hd, H, W, device=DEV, generator=g)
    zr = torch.sigmoid(torch.randn(B, 2 * hd, H, W, device=DEV, generator=g))
    h = torch.randn(B, hd, H, W, device=DEV, generator=g)
    dh0 = torch.randn(B, hd, H, W, device=DEV, generator=g)
    dzr0 = torch.randn(B, 2 * hd, H, W, device=DEV, generator=g)
    gx0 = [torch.randn(B, c, H, W, device=DEV, generator=g) for c in cx]
    acc = [0, 0, 1]
    # two launches
    drh = torch.empty_like(h)
    dh_a, dzr_a, gx_a = dh0.clone(), dzr0.clone(), [t.clone() for t in gx0]
    torch.ops.dro.conv2d_backward([rh, *xs], wq, None, dq, 0, 1.0, [drh, *gx_a], acc, None, None, 0, None)
    torch.ops.dro.gru_backward_elem(2, None, zr, None, h, drh, None, dzr_a, dh_a)
    # folded
    dh_b, dzr_b, gx_b = dh0.clone(), dzr0.clone(), [t.clone() for t in gx0]
    torch.ops.dro.convgru_candidate_backward([rh, *xs], wq, dq, zr, h, dzr_b, dh_b,
                                             [torch.empty(0, device=DEV), *gx_b], acc)
    torch.cuda.synchronize()
    assert torch.equal(dzr_a, dzr_b)
    assert torch.equal(dh_a, dh_b)
    for a, b in zip(gx_a, gx_b):
        assert torch.equal(a, b)
    assert torch.equal(dzr_b[:, :hd], dzr0[:, :hd])     # the z half untouched


def test_convgru_candidate_backward_rejects(hip):
    from dro_sfm_amd.hip import _lib
    lib = _lib.load()
    assert lib.dro_convgru_candidate_backward(None, 0, None, 1, 1, 1, 1, 1, 5, None, None, None, None, None,
                                              None, None, None, None, None, 0, None) != 0


@pytest.mark.parametrize("kernel,B,hd,H,W,dh_acc", [((5, 1), 2, 32, 24, 80, 0), ((1, 5), 4, 32, 24, 80, 1),
                                                     ((3, 3), 1, 16, 13, 37, 0), ((5, 1), 1, 8, 5, 7, 1)])
def test_convgru_gates_backward_matches_unfused(hip, kernel, B, hd, H, W, dh_acc):
    """The second GRU half's gate-conv data gradient with the first half's
    stage 1 in its epilogue (dro_convgru_gates_backward, ABI 8) against
    conv2d_backward (d h accumulated) followed by gru_backward_elem stage 1 on
    the finished d h: d h, the other sources' gradients, the first half's dq
    and dzr (z half; r half untouched) bit for bit; its dh bit for bit when
    written, to one rounding when added into (dh_acc)."""
    g = torch.Generator(device=DEV).manual_seed(9)
    KH, KW = kernel
    cx = (24, 10)
    h2 = torch.randn(B, hd, H, W, device=DEV, generator=g)
    xs = [torch.randn(B, c, H, W, device=DEV, generator=g) for c in cx]
    wzr = torch.randn(2 * hd, hd + sum(cx), KH, KW, device=DEV, generator=g) * 0.05
    dzr2 = torch.randn(B, 2 * hd, H, W, device=DEV, generator=g)
    dh2_0 = torch.randn(B, hd, H, W, device=DEV, generator=g)
    gx0 = [torch.randn(B, c, H, W, device=DEV, generator=g) for c in cx]
    zr1 = torch.sigmoid(torch.randn(B, 2 * hd, H, W, device=DEV, generator=g))
    q1 = torch.tanh(torch.randn(B, hd, H, W, device=DEV, generator=g))
    h1 = torch.randn(B, hd, H, W, device=DEV, generator=g)
    dzr1_0 = torch.randn(B, 2 * hd, H, W, device=DEV, generator=g)
    dh1_0 = torch.randn(B, hd, H, W, device=DEV, generator=g)
    acc = [1, 0, 1]
    # two launches
    dh2_a, gx_a = dh2_0.clone(), [t.clone() for t in gx0]
    dq1_a, dzr1_a, dh1_a = torch.empty_like(h1), dzr1_0.clone(), torch.empty_like(h1)
    torch.ops.dro.conv2d_backward([h2, *xs], wzr, None, dzr2, 0, 1.0, [dh2_a, *gx_a], acc, None, None, 0, None)
    torch.ops.dro.gru_backward_elem(1, dh2_a, zr1, q1, h1, None, dq1_a, dzr1_a, dh1_a)
    if dh_acc:
        dh1_a = dh1_0 + dh1_a
    # folded
    dh2_b, gx_b = dh2_0.clone(), [t.clone() for t in gx0]
    dq1_b, dzr1_b = torch.empty_like(h1), dzr1_0.clone()
    dh1_b = dh1_0.clone() if dh_acc else torch.empty_like(h1)
    torch.ops.dro.convgru_gates_backward([h2, *xs], wzr, dzr2, [dh2_b, *gx_b], acc, zr1, q1, h1, dq1_b, dzr1_b,
                                         dh1_b, dh_acc)
    torch.cuda.synchronize()
    assert torch.equal(dh2_a, dh2_b)
    for a, b in zip(gx_a, gx_b):
        assert torch.equal(a, b)
    assert torch.equal(dq1_a, dq1_b)
    assert torch.equal(dzr1_a, dzr1_b)
    assert torch.equal(dzr1_b[:, hd:], dzr1_0[:, hd:])
    if dh_acc:
        assert rel(dh1_b, dh1_a) < 1e-6
    else:
        assert torch.equal(dh1_a, dh1_b)


def test_convgru_gates_backward_rejects_strided_state(hip):
    """the first half's tensors are read as dense arrays; a strided
    one is refused instead of being read at the wrong elements."""
    B, hd, H, W = 2, 8, 5, 7
    h2 = torch.randn(B, hd, H, W, device=DEV)
    wzr = torch.randn(2 * hd, hd, 1, 5, device=DEV)
    dzr2 = torch.randn(B, 2 * hd, H, W, device=DEV)
    zr1 = torch.rand(B, 2 * hd, H, W, device=DEV)
    q1 = torch.rand(B, hd, H, W, device=DEV)
    h1 = torch.randn(B, 2 * hd, H, W, device=DEV)[:, :hd]          # a channel slice
    with pytest.raises(RuntimeError, match="contiguous"):
        torch.ops.dro.convgru_gates_backward([h2], wzr, dzr2, [torch.zeros_like(h2)], [1], zr1, q1, h1,
                                             torch.empty_like(q1), torch.empty_like(zr1), torch.empty_like(q1), 0)


def test_gru_chain_second_backward(hip):
    """the GruChain link is one-shot.  A second backward through the
    same graph (retain_graph) runs both halves unlinked and adds the same
    gradients again (2x the first pass, to fp32 reassociation)."""
    from dro_sfm_amd.hip import conv as C
    from dro_sfm_amd.networks.optim.update import SepConvGRU
    from dro_sfm_amd.trainers.dp_trainer import GradBuckets, flatten_parameters
    if not C._GRU_CHAIN:
        pytest.skip("GRU chain disabled (DRO_GRU_CHAIN=0)")
    torch.manual_seed(3)
    B, hd, cx, H, W = 2, 32, 48, 12, 20
    gru = SepConvGRU(hidden_dim=hd, input_dim=cx).to(DEV)
    with torch.no_grad():
        for p in gru.parameters():
            p.mul_(0.5)
    buckets = GradBuckets(list(gru.parameters()), groups=gru.dro_param_groups())
    # the trainer's layout: fused weights are views of one flat parameter buffer
    flatten_parameters(buckets.params, buckets.offsets, buckets.flat.numel(), buckets.flat.device)
    h = torch.randn(B, hd, H, W, device=DEV).tanh().requires_grad_()
    x = torch.randn(B, cx, H, W, device=DEV).requires_grad_()
    gout = torch.randn(B, hd, H, W, device=DEV)
    with C.weight_grad_scope():
        out = gru(h, x)
    n0 = C.GruChain.folded
    (out * gout).sum().backward(retain_graph=True)
    torch.cuda.synchronize()
    assert C.GruChain.folded == n0 + 1               # the first pass ran linked
    g1 = [buckets.flat.clone(), h.grad.clone(), x.grad.clone()]
    (out * gout).sum().backward()
    torch.cuda.synchronize()
    assert C.GruChain.folded == n0 + 1               # the second pass ran unlinked
    for a, b in zip([buckets.flat, h.grad, x.grad], g1):
        assert rel(a, 2 * b) < 1e-5
