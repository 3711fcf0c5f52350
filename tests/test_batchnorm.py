"""Fused training-mode BatchNorm + residual + ReLU (hip.batchnorm_act,
csrc/batchnorm.hip) against torch.nn.functional.batch_norm(training=True) + add
+ relu in fp64 on the CPU (the encoder sites of reference
networks/optim/extractor.py:7-107, torchvision BasicBlock).  Checked: output,
save statistics through the backward, running_mean / running_var / num_batches_tracked
updates, and the gradients of x, gamma, beta and skip.  Tolerance 1e-5 relative
(1e-4 for gradients: they subtract channel means of O(N*HW) terms)."""
import ctypes

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

import dro_sfm_amd.hip as hip
from dro_sfm_amd.hip import _lib
from dro_sfm_amd.networks.optim import extractor

# one-launch path (a channel's N*H*W <= 16 K: bn_fused_*_kernel, every EPT) and
# the two-launch path (> 16 K: partial sums + apply)
SHAPES = [(6, 64, 24, 80), (2, 3, 5, 7), (1, 16, 12, 40), (4, 1, 3, 4), (2, 32, 48, 160), (3, 8, 37, 29),
          (2, 8, 96, 100), (5, 4, 61, 67)]


def _reference(x, w, b, skip, rm, rv, relu, eps, momentum):
    y = F.batch_norm(x, rm, rv, w, b, training=True, momentum=momentum, eps=eps)
    if skip is not None:
        y = y + skip
    return F.relu(y) if relu else y


@pytest.mark.gpu
@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("variant", ["relu", "skip_relu", "plain"])
def test_batchnorm_act_matches_torch(shape, variant):
    relu = variant != "plain"
    use_skip = variant == "skip_relu"
    g = torch.Generator().manual_seed(1)
    N, C, H, W = shape
    x = 3.0 + 2.0 * torch.randn(*shape, generator=g, dtype=torch.float64)
    w = 1.0 + 0.1 * torch.randn(C, generator=g, dtype=torch.float64)
    b = 0.1 * torch.randn(C, generator=g, dtype=torch.float64)
    skip = torch.randn(*shape, generator=g, dtype=torch.float64) if use_skip else None
    gout = torch.randn(*shape, generator=g, dtype=torch.float64)
    rm0 = 0.1 * torch.randn(C, generator=g, dtype=torch.float64)
    rv0 = 1.0 + 0.1 * torch.rand(C, generator=g, dtype=torch.float64)

    xr, wr, br = (t.clone().requires_grad_() for t in (x, w, b))
    sr = skip.clone().requires_grad_() if use_skip else None
    rm, rv = rm0.clone(), rv0.clone()
    ref = _reference(xr, wr, br, sr, rm, rv, relu, 1e-5, 0.1)
    ref.backward(gout)

    bn = extractor.BatchNorm2d(C).cuda()
    with torch.no_grad():
        bn.weight.copy_(w.float())
        bn.bias.copy_(b.float())
        bn.running_mean.copy_(rm0.float())
        bn.running_var.copy_(rv0.float())
    bn.train()
    xd = x.float().cuda().requires_grad_()
    sd = skip.float().cuda().requires_grad_() if use_skip else None
    out = hip.batchnorm_act(xd, bn, skip=sd, relu=relu)
    out.backward(gout.float().cuda())

    torch.testing.assert_close(out.double().cpu(), ref.detach(), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(bn.running_mean.double().cpu(), rm, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(bn.running_var.double().cpu(), rv, rtol=1e-5, atol=1e-6)
    assert int(bn.num_batches_tracked) == 1
    torch.testing.assert_close(xd.grad.double().cpu(), xr.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(bn.weight.grad.double().cpu(), wr.grad, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(bn.bias.grad.double().cpu(), br.grad, rtol=1e-4, atol=1e-3)
    if use_skip:
        torch.testing.assert_close(sd.grad.double().cpu(), sr.grad, rtol=1e-6, atol=1e-6)


@pytest.mark.gpu
def test_batchnorm_act_deterministic():
    g = torch.Generator().manual_seed(2)
    x = torch.randn(6, 64, 48, 160, generator=g).cuda()
    gout = torch.randn(6, 64, 48, 160, generator=g).cuda()
    grads = []
    for _ in range(2):
        bn = extractor.BatchNorm2d(64).cuda().train()
        xd = x.clone().requires_grad_()
        hip.batchnorm_act(xd, bn).backward(gout)
        grads.append((xd.grad, bn.weight.grad, bn.bias.grad, bn.running_var.clone()))
    for a, b in zip(*grads):
        assert torch.equal(a, b)


@pytest.mark.gpu
def test_encoder_fused_bn_matches_unfused():
    """ResNetEncoder forward + backward with the fused sites vs PyTorch's BN/ReLU."""
    torch.manual_seed(0)
    enc = extractor.ResNetEncoder(out_chs=96, stride=8).cuda().train()
    x = torch.randn(2, 3, 64, 96, device="cuda")
    outs = []
    for fused in (True, False):
        extractor.set_fused_batchnorm(fused)
        e = extractor.ResNetEncoder(out_chs=96, stride=8).cuda().train()
        e.load_state_dict(enc.state_dict())
        e.zero_grad()
        y = e(x)
        y.square().mean().backward()
        outs.append((y.detach(), {k: p.grad.clone() for k, p in e.named_parameters()},
                     {k: v.clone() for k, v in e.state_dict().items()}))
    extractor.set_fused_batchnorm(True)
    (y1, g1, s1), (y2, g2, s2) = outs
    # fp32 rounding of the statistics (fp64 here, Welford fp32 in PyTorch) carried
    # through 17 MIOpen convolutions
    torch.testing.assert_close(y1, y2, rtol=1e-3, atol=1e-4)
    for k in g1:
        torch.testing.assert_close(g1[k], g2[k], rtol=5e-3, atol=1e-5, msg=k)
    for k in s1:
        torch.testing.assert_close(s1[k].double(), s2[k].double(), rtol=1e-5, atol=1e-6, msg=k)


def test_batchnorm_abi_rejects_bad_arguments():
    """C-ABI argument checks (no launch happens on these paths)."""
    lib = _lib.load()
    assert lib.dro_batchnorm_workspace_bytes(2, 4, 16) > 0
    assert lib.dro_batchnorm_workspace_bytes(0, 4, 16) == 0
    null = ctypes.c_void_p(0)
    one = ctypes.c_void_p(16)
    st = lib.dro_batchnorm_relu_forward(null, null, null, null, 1, 2, 4, 16, 1e-5, 0.1, null, null,
                                        null, one, one, one, one, 1 << 20, null)
    assert st == -1
    st = lib.dro_batchnorm_relu_forward(one, null, null, null, 2, 2, 4, 16, 1e-5, 0.1, null, null,
                                        null, one, one, one, one, 1 << 20, null)
    assert st == -3
    st = lib.dro_batchnorm_relu_forward(one, null, null, null, 1, 2, 4, 16, 1e-5, 0.1, null, null,
                                        null, one, one, one, one, 1, null)
    assert st == -2
    st = lib.dro_batchnorm_relu_backward(one, one, null, null, one, one, 1, 2, 4, 16, one, null, null,
                                         null, one, 1 << 20, null)
    assert st == -1


def test_batchnorm_act_rejects_cpu():
    bn = nn.BatchNorm2d(2)
    with pytest.raises(RuntimeError):
        hip.batchnorm_act(torch.zeros(1, 2, 2, 2), bn)
