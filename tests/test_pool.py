"""ResNet stem max pooling (hip.maxpool3x3s2) against F.max_pool2d(x, 3, 2, 1)
(reference networks/optim/extractor.py:60-66, torchvision's ResNet stem).
Bit-identical: the forward takes ATen's first maximum in scan order and the
backward sums each input's windows in ATen's order.  Shapes include odd sizes,
1-pixel planes and ties (post-ReLU zeros, repeated values)."""
import pytest
import torch
import torch.nn.functional as F

import dro_sfm_amd.hip as hip

SHAPES = [(6, 64, 96, 320), (2, 3, 7, 5), (1, 2, 1, 1), (3, 4, 2, 9), (1, 1, 33, 17)]


@pytest.mark.gpu
@pytest.mark.parametrize("shape", SHAPES)
def test_maxpool3x3s2_matches_max_pool2d(shape):
    g = torch.Generator().manual_seed(3)
    x = torch.randn(*shape, generator=g).relu()            # post-ReLU: many tied zeros
    x[..., ::3, ::2] = 0.5                                  # and tied positive values
    ref_x = x.cuda().requires_grad_()
    ref = F.max_pool2d(ref_x, 3, 2, 1)
    gout = torch.randn(ref.shape, generator=g).cuda()
    ref.backward(gout)
    xd = x.cuda().requires_grad_()
    out = hip.maxpool3x3s2(xd)
    out.backward(gout)
    assert out.shape == ref.shape
    assert torch.equal(out, ref.detach())
    assert torch.equal(xd.grad, ref_x.grad)


@pytest.mark.gpu
def test_maxpool3x3s2_nan_propagates_like_aten():
    x = torch.zeros(1, 1, 5, 5)
    x[0, 0, 2, 2] = float("nan")
    xd = x.cuda()
    assert torch.equal(torch.isnan(hip.maxpool3x3s2(xd)), torch.isnan(F.max_pool2d(xd, 3, 2, 1)))


def test_maxpool3x3s2_rejects_cpu_and_dtype():
    with pytest.raises(RuntimeError):
        hip.maxpool3x3s2(torch.zeros(1, 1, 4, 4, dtype=torch.float64))
    with pytest.raises(RuntimeError):
        hip.maxpool3x3s2(torch.zeros(1, 1, 4, 4))


@pytest.mark.gpu
def test_maxpool_more_than_65535_planes():
    """Chunked launches beyond 65535 planes: bit-identical to
    F.max_pool2d forward and backward."""
    import dro_sfm_amd.hip as hip
    g = torch.Generator(device="cuda").manual_seed(6)
    x = torch.rand(2, 35000, 6, 7, device="cuda", generator=g).requires_grad_(True)
    y = hip.maxpool3x3s2(x)
    gy = torch.rand(y.shape, device="cuda", generator=g)
    (y * gy).sum().backward()
    x2 = x.detach().clone().requires_grad_(True)
    y2 = torch.nn.functional.max_pool2d(x2, 3, 2, 1)
    (y2 * gy).sum().backward()
    assert torch.equal(y, y2) and torch.equal(x.grad, x2.grad)
