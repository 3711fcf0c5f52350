"""BatchNorm fused into the encoders' 3x3 stride-1 convolutions (hip.bnconv,
csrc/conv.hip BnFuse, ABI 10) against the same ResNet-18 BasicBlock
(reference networks/optim/extractor.py:67-107 via torchvision) computed in fp64
by PyTorch on the CPU -- conv2d + batch_norm(training=True) + skip + relu --
and against the unfused HIP path (hip.batchnorm_act after each conv).

Checked: block output, running_mean / running_var / num_batches_tracked, and
the gradients of the input, both conv weights and the four BN affine
parameters, for stride-1 blocks (bn1 fused both ways, bn2's statistics in
conv2's epilogue) and stride-2 entry blocks (bn2's statistics only), at a
site with hundreds of pixel tiles (two-level fold of the partial sums) and at
small ones; repeated calls (the self-resetting counters) and a captured hipGraph
replay.  Tolerances: 1e-5 relative on outputs and statistics, 1e-4 on
gradients (channel means of O(N H W) terms), as tests/test_batchnorm.py.
"""
import pytest
import torch
import torch.nn.functional as F

from dro_sfm_amd.hip import _lib, bnconv
from dro_sfm_amd.hip.ops import record_bilinear_cells
from dro_sfm_amd.networks.optim import extractor


def _block(cin, cout, stride, seed):
    torch.manual_seed(seed)
    blk = extractor.BasicBlock(cin, cout, stride)
    with torch.no_grad():
        for m in blk.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.3, 0.3)
                m.running_mean.uniform_(-0.2, 0.2)
                m.running_var.uniform_(0.8, 1.2)
    return blk.train()


def _reference(blk, x, gout, masks):
    """fp64 CPU forward + backward of the block (torch ops only); each ReLU
    takes its on/off decision from the product's mask (a BN output within
    fp32 rounding of 0 may fall on either side: the kink is pinned, as in the
    train-step parity tests)."""
    p = {n: t.detach().double().cpu().requires_grad_(t.requires_grad) for n, t in blk.named_parameters()}
    bufs = {n: t.detach().double().cpu() for n, t in blk.named_buffers() if "running" in n}
    xr = x.detach().double().cpu().requires_grad_()

    def bn(z, name):
        return F.batch_norm(z, bufs[name + ".running_mean"], bufs[name + ".running_var"], p[name + ".weight"],
                            p[name + ".bias"], training=True, momentum=0.1, eps=1e-5)

    def relu(v, tag):
        return v * masks[tag].to(v.device, torch.float64)

    s = blk.conv1.stride[0]
    y = relu(bn(F.conv2d(xr, p["conv1.weight"], stride=s, padding=1), "bn1"), "bn1")
    z2 = bn(F.conv2d(y, p["conv2.weight"], padding=1), "bn2")
    skip = xr if blk.downsample is None else \
        bn(F.conv2d(xr, p["downsample.0.weight"], stride=s), "downsample.1")
    out = relu(z2 + skip, "bn2")
    out.backward(gout.double().cpu())
    return out.detach(), xr.grad, {n: t.grad for n, t in p.items()}, bufs


def _run(blk, x, gout, fused, masks=None):
    """Forward + backward on the GPU; masks (dict) receives each BN site's ReLU
    mask y > 0 (the product's branch record, hip.ops.record_branch)."""
    for name in ("bn1", "bn2"):
        object.__setattr__(getattr(blk, name), "_dro_tag", name)
    bnconv.set_bn_fusion("all" if fused else False)
    try:
        xd = x.clone().requires_grad_()
        with record_bilinear_cells() as rec:
            out = blk(xd)
        out.backward(gout)
        torch.cuda.synchronize()
        if masks is not None:
            masks.update({tag[1]: m.bool().cpu() for tag, m in rec.calls if tag[0] == "relu"})
        return out.detach(), xd.grad, {n: t.grad.clone() for n, t in blk.named_parameters()}
    finally:
        bnconv.set_bn_fusion(True)


@pytest.fixture
def all_sites():
    bnconv.set_bn_fusion("all")
    yield
    bnconv.set_bn_fusion(True)


CASES = [  # (cin, cout, stride, B, H, W): KITTI layer1 / layer2 / layer3, ragged, batch 1
    (64, 64, 1, 6, 48, 160),
    (128, 128, 1, 6, 24, 80),
    (256, 256, 1, 2, 12, 40),
    (32, 32, 1, 3, 13, 29),
    (64, 128, 2, 6, 48, 160),
    (128, 256, 2, 1, 30, 40),
]


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=lambda c: "x".join(map(str, c)))
def test_fused_block_matches_fp64(case):
    cin, cout, stride, B, H, W = case
    blk = _block(cin, cout, stride, seed=3).cuda()
    g = torch.Generator().manual_seed(4)
    x = (0.5 + torch.randn(B, cin, H, W, generator=g)).cuda()
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    gout = torch.randn(B, cout, Ho, Wo, generator=g).cuda()
    _lib.load()
    bufs0 = {n: t.clone() for n, t in blk.named_buffers()}
    masks = {}
    out, gx, gp = _run(blk, x, gout, True, masks)
    assert set(masks) == {"bn1", "bn2"}
    fused_bufs = {n: t.clone() for n, t in blk.named_buffers()}
    with torch.no_grad():
        for n, t in blk.named_buffers():
            t.copy_(bufs0[n])
    ref_out, ref_gx, ref_gp, ref_bufs = _reference(blk, x, gout, masks)
    torch.testing.assert_close(out.double().cpu(), ref_out, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(gx.double().cpu(), ref_gx, rtol=1e-4, atol=1e-4)
    for n, t in gp.items():
        scale = max(1.0, float(ref_gp[n].abs().max()))
        torch.testing.assert_close(t.double().cpu(), ref_gp[n], rtol=1e-4, atol=1e-4 * scale, msg=n)
    for n, t in fused_bufs.items():
        if "running" in n:
            torch.testing.assert_close(t.double().cpu(), ref_bufs[n], rtol=1e-5, atol=1e-6, msg=n)
        if "num_batches" in n:
            assert int(t) == 1, n


def _stage_reference(stage, x, gout, masks):
    """fp64 CPU forward + backward of a two-block stage, ReLUs pinned to the
    product's masks (tags b<i>.bn<j>)."""
    p = {n: t.detach().double().cpu().requires_grad_() for n, t in stage.named_parameters()}
    bufs = {n: t.detach().double().cpu() for n, t in stage.named_buffers() if "running" in n}
    xr = x.detach().double().cpu().requires_grad_()

    def bn(z, name):
        return F.batch_norm(z, bufs[name + ".running_mean"], bufs[name + ".running_var"], p[name + ".weight"],
                            p[name + ".bias"], training=True, momentum=0.1, eps=1e-5)

    h = xr
    for i in range(2):
        blk = stage[i]
        s = blk.conv1.stride[0]
        y = bn(F.conv2d(h, p[f"{i}.conv1.weight"], stride=s, padding=1), f"{i}.bn1") * masks[f"b{i}.bn1"].double()
        z2 = bn(F.conv2d(y, p[f"{i}.conv2.weight"], padding=1), f"{i}.bn2")
        skip = h if blk.downsample is None else bn(F.conv2d(h, p[f"{i}.downsample.0.weight"], stride=s),
                                                    f"{i}.downsample.1")
        h = (z2 + skip) * masks[f"b{i}.bn2"].double()
    h.backward(gout.double().cpu())
    return h.detach(), xr.grad, {n: t.grad for n, t in p.items()}, bufs


@pytest.mark.gpu
@pytest.mark.parametrize("case", [(64, 64, 1, 6, 48, 160), (64, 128, 2, 6, 48, 160), (128, 256, 2, 2, 24, 80)],
                         ids=lambda c: "x".join(map(str, c)))
def test_fused_stage_matches_fp64(case, all_sites):
    """extractor.run_stage: the first block's output staged (and stored) by
    the second block's conv1 (bn_add_relu_conv_stats), against fp64."""
    cin, cout, stride, B, H, W = case
    torch.manual_seed(9)
    stage = extractor._stage(cin, cout, stride)
    with torch.no_grad():
        for m in stage.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.3, 0.3)
    stage = stage.cuda().train()
    for i in range(2):
        for name in ("bn1", "bn2"):
            object.__setattr__(getattr(stage[i], name), "_dro_tag", f"b{i}.{name}")
    g = torch.Generator().manual_seed(10)
    x = (0.5 + torch.randn(B, cin, H, W, generator=g)).cuda()
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    gout = torch.randn(B, cout, Ho, Wo, generator=g).cuda()
    bufs0 = {n: t.clone() for n, t in stage.named_buffers()}
    xd = x.clone().requires_grad_()
    with record_bilinear_cells() as rec:
        out = extractor.run_stage(stage, xd)
    out.backward(gout)
    masks = {tag[1]: m.bool().cpu() for tag, m in rec.calls if tag[0] == "relu"}
    assert {"b0.bn1", "b0.bn2", "b1.bn1", "b1.bn2"} <= set(masks)
    fused_bufs = {n: t.clone() for n, t in stage.named_buffers()}
    with torch.no_grad():
        for n, t in stage.named_buffers():
            t.copy_(bufs0[n])
    ref_out, ref_gx, ref_gp, ref_bufs = _stage_reference(stage, x, gout, masks)
    torch.testing.assert_close(out.detach().double().cpu(), ref_out, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(xd.grad.double().cpu(), ref_gx, rtol=1e-4, atol=1e-4)
    for n, t in stage.named_parameters():
        scale = max(1.0, float(ref_gp[n].abs().max()))
        torch.testing.assert_close(t.grad.double().cpu(), ref_gp[n], rtol=1e-4, atol=1e-4 * scale, msg=n)
    for n, t in fused_bufs.items():
        if "running" in n:
            torch.testing.assert_close(t.double().cpu(), ref_bufs[n], rtol=1e-5, atol=1e-6, msg=n)


@pytest.mark.gpu
@pytest.mark.parametrize("case", [CASES[0], CASES[2], CASES[4]], ids=lambda c: "x".join(map(str, c)))
def test_fused_block_equals_unfused_hip(case):
    """Same block, same inputs: the fused path against hip.batchnorm_act after
    each conv -- identical up to the statistics' fp64 summation order."""
    cin, cout, stride, B, H, W = case
    blk = _block(cin, cout, stride, seed=5).cuda()
    g = torch.Generator().manual_seed(6)
    x = torch.randn(B, cin, H, W, generator=g).cuda()
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    gout = torch.randn(B, cout, Ho, Wo, generator=g).cuda()
    state = {k: v.clone() for k, v in blk.state_dict().items()}
    o1, gx1, gp1 = _run(blk, x, gout, True)
    blk.load_state_dict(state)
    for p in blk.parameters():
        p.grad = None
    o0, gx0, gp0 = _run(blk, x, gout, False)
    torch.testing.assert_close(o1, o0, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(gx1, gx0, rtol=1e-5, atol=1e-5)
    for n in gp0:
        torch.testing.assert_close(gp1[n], gp0[n], rtol=1e-5, atol=1e-5 * max(1.0, float(gp0[n].abs().max())), msg=n)


@pytest.mark.gpu
def test_fused_block_repeat_and_graph_replay(all_sites):
    """Repeated calls reuse the per-site states (counters reset by the kernels):
    every call equals the first, eager and replayed from a captured graph."""
    blk = _block(64, 64, 1, seed=7).cuda()
    for m in blk.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.momentum = 0.0          # running statistics stay put: calls are comparable
    g = torch.Generator().manual_seed(8)
    x = torch.randn(6, 64, 48, 160, generator=g).cuda().requires_grad_()
    gout = torch.randn(6, 64, 48, 160, generator=g).cuda()

    def step():
        for p in blk.parameters():
            p.grad = None
        x.grad = None
        out = blk(x)
        out.backward(gout)
        return out.detach().clone(), x.grad.clone(), blk.conv1.weight.grad.clone(), blk.bn1.weight.grad.clone()

    first = step()
    for _ in range(3):
        again = step()
        for a, b in zip(first, again):
            assert torch.equal(a, b)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()
    torch.cuda.current_stream().wait_stream(s)
    for p in blk.parameters():
        p.grad = None
    x.grad = None
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out = blk(x)
        out.backward(gout)
    for _ in range(2):
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, first[0])
        assert torch.equal(x.grad, first[1])


def test_bn_state_bytes_cpu():
    lib = _lib.load()
    n = lib.dro_bn_state_bytes(6, 48, 160, 64)
    # counters + 720 tiles x 64 channels x 16 B partials + 23 groups + 5 x 64 coefficients
    assert n >= 720 * 64 * 16 + 23 * 64 * 16 + 5 * 64 * 4
    assert lib.dro_bn_state_bytes(0, 48, 160, 64) == 0
    assert lib.dro_bn_state_bytes(6, 48, 160, 0) == 0


def test_size_policy_cpu():
    """Default policy: fused only where a channel holds > 16 K elements."""
    blk = extractor.BasicBlock(64, 64, 1).train()
    x = torch.empty(6, 64, 48, 160, device="meta")
    conv, bn = blk.conv2, blk.bn2
    assert not bnconv.supported(bn, conv, x)            # meta tensors are not CUDA
    bnconv.set_bn_fusion(False)
    try:
        assert not bnconv.bn_fusion_enabled()
    finally:
        bnconv.set_bn_fusion(True)
    assert bnconv.bn_fusion_enabled()
