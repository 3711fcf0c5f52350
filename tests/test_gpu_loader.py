"""The GPU data path hooked to reference-style samples (datasets/gpu_loader.py):
collate of decoded frames on the host, then train_transforms on the GPU --
equal to the reference's CPU data_transform chain (Pillow resize, ColorJitter
with the same draws, ToTensor) sample by sample, with KITTI drives' differing
raw sizes in one batch."""
import numpy as np
import pytest
import torch

JIT = (0.2, 0.2, 0.2, 0.05)


def _samples(sizes, seed=11, n_ctx=2):
    from PIL import Image
    rng = np.random.default_rng(seed)
    out = []
    for i, (h0, w0) in enumerate(sizes):
        img = lambda: Image.fromarray(rng.integers(0, 256, (h0, w0, 3), dtype=np.uint8))
        K = np.array([[721.5, 0.0, w0 / 2], [0.0, 721.5, h0 / 2], [0.0, 0.0, 1.0]], np.float32)
        poses = [np.eye(4, dtype=np.float32) + 0.01 * j for j in range(n_ctx)]
        out.append({"idx": i, "filename": f"s{i}", "rgb": img(), "rgb_context": [img() for _ in range(n_ctx)],
                    "intrinsics": K, "pose_context": poses})
    return out


def test_collate_decoded_layout():
    """Host collate: uint8 HWC frames per sample (raw sizes may differ),
    stacked float32 intrinsics and per-reference poses, other keys as lists."""
    from dro_sfm_amd.datasets.gpu_loader import collate_decoded
    s = _samples([(12, 20), (12, 20), (10, 18)])
    b = collate_decoded(s)
    assert len(b["rgb"]) == 3 and b["rgb"][2].shape == (10, 18, 3) and b["rgb"][0].dtype == torch.uint8
    assert np.array_equal(b["rgb"][1].numpy(), np.asarray(s[1]["rgb"]))
    assert len(b["rgb_context"]) == 2 and np.array_equal(b["rgb_context"][1][0].numpy(),
                                                           np.asarray(s[0]["rgb_context"][1]))
    assert b["intrinsics"].shape == (3, 3, 3) and b["intrinsics"].dtype == torch.float32
    assert len(b["pose_context"]) == 2 and b["pose_context"][1].shape == (3, 4, 4)
    assert b["idx"] == [0, 1, 2] and b["filename"][2] == "s2"


@pytest.mark.gpu
def test_gpu_pipeline_matches_reference_chain():
    """GPUTrainPipeline on a batch of two 375x1242 samples and one 370x1226
    sample (two KITTI drives) == per sample: Pillow resize to 192x640, the
    reference's ColorJitter draws in its order, ToTensor; intrinsics scaled by
    each sample's own raw size (augmentations.py:93-99)."""
    from PIL import Image
    from oracle import dro_oracle as O
    from dro_sfm_amd.datasets.gpu_loader import GPUTrainPipeline, collate_decoded
    from dro_sfm_amd.datasets.gpu_transforms import colorjitter_params
    H, W = 192, 640
    sizes = [(375, 1242), (375, 1242), (370, 1226)]
    s = _samples(sizes)
    out = GPUTrainPipeline((H, W), JIT, generator=torch.Generator().manual_seed(5))(collate_decoded(s))
    g = torch.Generator().manual_seed(5)
    for n, (h0, w0) in enumerate(sizes):
        colorjitter_params(JIT, 1, g)                       # the draw the reference discards
        frames = [s[n]["rgb"]] + s[n]["rgb_context"]
        got = [out["rgb"]] + out["rgb_context"]
        got_o = [out["rgb_original"]] + out["rgb_context_original"]
        for f, im in enumerate(frames):
            o, fa, hu = colorjitter_params(JIT, 1, g)
            rs = np.asarray(im.resize((W, H), Image.BILINEAR))
            want_o = torch.from_numpy(rs.copy()).permute(2, 0, 1).float().div(255)
            want = torch.from_numpy(O.color_jitter_pil(rs, o[0], fa[0], hu[0]).copy()).permute(2, 0, 1).float().div(255)
            assert torch.equal(got_o[f][n].cpu(), want_o), (n, f)
            assert torch.equal(got[f][n].cpu(), want), (n, f)
        K = torch.from_numpy(s[n]["intrinsics"]).clone()
        K[0] *= W / w0
        K[1] *= H / h0
        assert torch.allclose(out["intrinsics"][n].cpu(), K, rtol=0, atol=1e-4)
    assert out["pose_context"][1].is_cuda and out["pose_context"][1].shape == (3, 4, 4)
