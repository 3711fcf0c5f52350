"""Bilinear 2x upsampling of the feature trunk (hip.bilinear_upsample2x) against
F.interpolate(scale_factor=2, mode="bilinear", align_corners=False) in fp64
(reference networks/optim/extractor.py:91-97).  Tolerance: 1e-5 relative."""
import pytest
import torch
import torch.nn.functional as F

import dro_sfm_amd.hip as hip

SHAPES = [(6, 256, 12, 40), (2, 3, 1, 1), (1, 5, 7, 3), (3, 2, 1, 9)]


@pytest.mark.gpu
@pytest.mark.parametrize("shape", SHAPES)
def test_bilinear_upsample2x_matches_interpolate(shape):
    g = torch.Generator().manual_seed(0)
    x = torch.randn(*shape, generator=g, dtype=torch.float64)
    gout = torch.randn(shape[0], shape[1], 2 * shape[2], 2 * shape[3], generator=g, dtype=torch.float64)
    xr = x.clone().requires_grad_()
    ref = F.interpolate(xr, scale_factor=2, mode="bilinear", align_corners=False)
    ref.backward(gout)
    xd = x.float().cuda().requires_grad_()
    out = hip.bilinear_upsample2x(xd)
    out.backward(gout.float().cuda())
    torch.testing.assert_close(out.double().cpu(), ref.detach(), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(xd.grad.double().cpu(), xr.grad, rtol=1e-5, atol=1e-5)
    # the backward gathers in a fixed order: run-to-run identical
    xd2 = x.float().cuda().requires_grad_()
    hip.bilinear_upsample2x(xd2).backward(gout.float().cuda())
    assert torch.equal(xd.grad, xd2.grad)


def test_bilinear_upsample2x_rejects_cpu():
    with pytest.raises(RuntimeError):
        hip.bilinear_upsample2x(torch.zeros(1, 1, 2, 2))


@pytest.mark.gpu
def test_bilinear_upsample2x_more_than_65535_planes():
    """Planes ride grid.y (<= 65535 per launch); larger batches are launched in
    chunks: forward and backward equal to F.interpolate."""
    import dro_sfm_amd.hip as hip
    g = torch.Generator(device="cuda").manual_seed(5)
    x = torch.rand(1, 70001, 3, 5, device="cuda", generator=g).requires_grad_(True)
    y = hip.bilinear_upsample2x(x)
    gy = torch.rand(y.shape, device="cuda", generator=g)
    (y * gy).sum().backward()
    x2 = x.detach().clone().requires_grad_(True)
    y2 = torch.nn.functional.interpolate(x2, scale_factor=2, mode="bilinear", align_corners=False)
    (y2 * gy).sum().backward()
    torch.testing.assert_close(y, y2, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(x.grad, x2.grad, rtol=1e-5, atol=1e-6)
