"""GPU resize + ToTensor (dro_sfm_amd.datasets.gpu_transforms, csrc/resize.hip)
against Pillow's BILINEAR resize + torchvision-style ToTensor (value / 255),
as the reference's training transforms apply them
(datasets/augmentations.py:69-160).  Bit-identical."""
import numpy as np
import pytest
import torch

SHAPES = [((375, 1242), (192, 640)), ((370, 1226), (192, 640)), ((480, 640), (240, 320)), ((50, 40), (96, 81))]


@pytest.mark.gpu
@pytest.mark.parametrize("shape", SHAPES)
def test_resize_to_tensor_matches_pillow(shape):
    from PIL import Image
    from dro_sfm_amd.datasets.gpu_transforms import resize_to_tensor
    (h0, w0), (H, W) = shape
    rng = np.random.default_rng(w0)
    frames = rng.integers(0, 256, (3, h0, w0, 3), dtype=np.uint8)
    out = resize_to_tensor(torch.from_numpy(frames).cuda(), (H, W)).cpu()
    for n in range(3):
        ref = np.asarray(Image.fromarray(frames[n]).resize((W, H), Image.BILINEAR))
        want = torch.from_numpy(ref.copy()).permute(2, 0, 1).float().div(255)
        assert torch.equal(out[n], want)


@pytest.mark.gpu
def test_resize_sample_scales_intrinsics():
    from dro_sfm_amd.datasets.gpu_transforms import resize_sample_to_tensor
    B, h0, w0 = 2, 375, 1242
    rgb = torch.randint(0, 256, (B, h0, w0, 3), dtype=torch.uint8).cuda()
    ctx = [torch.randint(0, 256, (B, h0, w0, 3), dtype=torch.uint8).cuda() for _ in range(2)]
    K = torch.tensor([[721.5, 0.0, 609.6], [0.0, 721.5, 172.9], [0.0, 0.0, 1.0]]).repeat(B, 1, 1).cuda()
    out = resize_sample_to_tensor({"rgb": rgb, "rgb_context": ctx, "intrinsics": K}, (192, 640))
    assert out["rgb"].shape == (B, 3, 192, 640) and len(out["rgb_context"]) == 2
    assert torch.equal(out["rgb_original"], out["rgb"])
    Kw = K.clone()
    Kw[:, 0] *= 640 / 1242
    Kw[:, 1] *= 192 / 375
    assert torch.equal(out["intrinsics"], Kw)


def test_resize_rejects_cpu_and_layout():
    from dro_sfm_amd.datasets.gpu_transforms import resize_to_tensor
    with pytest.raises(RuntimeError):
        resize_to_tensor(torch.zeros(1, 4, 4, 3, dtype=torch.uint8), (2, 2))
    with pytest.raises(RuntimeError):
        resize_to_tensor(torch.zeros(1, 3, 4, 4, dtype=torch.uint8), (2, 2))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_color_jitter_matches_pillow(seed):
    """colorjitter_sample (augmentations.py:213-258) with the reference default
    jittering (0.2, 0.2, 0.2, 0.05) and wider factors (clipping branch):
    every frame's random order / factors applied through Pillow (oracle) vs the
    GPU kernels, bit for bit."""
    from oracle import dro_oracle as O
    from dro_sfm_amd.datasets.gpu_transforms import color_jitter_, colorjitter_params
    g = torch.Generator().manual_seed(seed)
    jit = (0.2, 0.2, 0.2, 0.05) if seed < 2 else (0.9, 0.9, 0.9, 0.5)
    frames = np.random.default_rng(seed).integers(0, 256, (4, 57, 83, 3), dtype=np.uint8)
    orders, factors, hues = colorjitter_params(jit, 4, g)
    out = color_jitter_(torch.from_numpy(frames.copy()).cuda(), orders, factors, hues).cpu().numpy()
    for n in range(4):
        ref = O.color_jitter_pil(frames[n], orders[n], factors[n], hues[n])
        assert np.array_equal(out[n], ref), (n, orders[n], factors[n], hues[n], int((out[n] != ref).sum()))


@pytest.mark.gpu
def test_train_transforms_pipeline_matches_pillow():
    """resize -> duplicate -> jitter -> to_tensor on a KITTI-size batch against
    the same chain through Pillow with the same random draws."""
    from PIL import Image
    from oracle import dro_oracle as O
    from dro_sfm_amd.datasets.gpu_transforms import train_transforms
    B, h0, w0, H, W = 2, 375, 1242, 192, 640
    rng = np.random.default_rng(7)
    rgb = rng.integers(0, 256, (B, h0, w0, 3), dtype=np.uint8)
    ctx = [rng.integers(0, 256, (B, h0, w0, 3), dtype=np.uint8) for _ in range(2)]
    out = train_transforms({"rgb": torch.from_numpy(rgb).cuda(), "rgb_context": [torch.from_numpy(c).cuda() for c in ctx]},
                           (H, W), (0.2, 0.2, 0.2, 0.05), generator=torch.Generator().manual_seed(3))
    # the reference's draw order (colorjitter_sample, augmentations.py:226-256): per
    # sample one discarded get_params draw, then rgb, ctx0, ctx1
    g = torch.Generator().manual_seed(3)
    from dro_sfm_amd.datasets.gpu_transforms import colorjitter_params
    draws = {}
    for n in range(B):
        colorjitter_params((0.2, 0.2, 0.2, 0.05), 1, g)
        for f in range(3):
            o, fa, hu = colorjitter_params((0.2, 0.2, 0.2, 0.05), 1, g)
            draws[f, n] = (o[0], fa[0], hu[0])
    cases = [(out["rgb"], out["rgb_original"], rgb)] + \
        [(out["rgb_context"][j], out["rgb_context_original"][j], ctx[j]) for j in range(2)]
    for f, (got, got_orig, src) in enumerate(cases):
        for n in range(B):
            rs = np.asarray(Image.fromarray(src[n]).resize((W, H), Image.BILINEAR))
            want_o = torch.from_numpy(rs.copy()).permute(2, 0, 1).float().div(255)
            jt = O.color_jitter_pil(rs, *draws[f, n])
            want = torch.from_numpy(jt.copy()).permute(2, 0, 1).float().div(255)
            assert torch.equal(got_orig[n].cpu(), want_o)
            assert torch.equal(got[n].cpu(), want)
