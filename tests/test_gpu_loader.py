"""The GPU data path hooked to reference-style samples (datasets/gpu_loader.py):
collate of decoded frames on the host, then train_transforms on the GPU --
equal to the reference's CPU data_transform chain (Pillow resize, ColorJitter
with the same draws, ToTensor) sample by sample, with KITTI drives' differing
raw sizes in one batch."""
import numpy as np
import pytest
import torch

JIT = (0.2, 0.2, 0.2, 0.05)


def _samples(sizes, seed=11, n_ctx=2, depth=False):
    from PIL import Image
    rng = np.random.default_rng(seed)
    out = []
    for i, (h0, w0) in enumerate(sizes):
        img = lambda: Image.fromarray(rng.integers(0, 256, (h0, w0, 3), dtype=np.uint8))
        K = np.array([[721.5, 0.0, w0 / 2], [0.0, 721.5, h0 / 2], [0.0, 0.0, 1.0]], np.float32)
        poses = [np.eye(4, dtype=np.float32) + 0.01 * j for j in range(n_ctx)]
        s = {"idx": i, "filename": f"s{i}", "rgb": img(), "rgb_context": [img() for _ in range(n_ctx)],
             "intrinsics": K, "pose_context": poses}
        if depth:
            # sparse LiDAR-like depth (KITTI velodyne projection: ~5 % valid)
            dmap = lambda: (rng.uniform(1, 80, (h0, w0)) * (rng.random((h0, w0)) < 0.05)).astype(np.float32)
            s["depth"] = dmap()
            s["depth_context"] = [dmap()[..., None] for _ in range(n_ctx)]
        out.append(s)
    return out


def test_resize_depth_nearest_matches_cv2_restatement():
    """The gather used on the GPU (run here on CPU tensors) == the oracle's
    OpenCV INTER_NEAREST restatement, for KITTI raw sizes -> 192x640 and an
    upscaling case."""
    from oracle import dro_oracle as O
    from dro_sfm_amd.datasets.gpu_loader import resize_depth_nearest
    rng = np.random.default_rng(3)
    for (h, w), shape in [((375, 1242), (192, 640)), ((370, 1226), (192, 640)), ((7, 9), (16, 20))]:
        d = rng.uniform(0, 80, (2, h, w)).astype(np.float32)
        got = resize_depth_nearest(torch.from_numpy(d), shape)
        assert got.shape == (2, 1) + shape
        for b in range(2):
            want = O.resize_depth_cv2_nearest(d[b], shape)[..., 0]
            assert np.array_equal(got[b, 0].numpy(), want)


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
    d = collate_decoded(_samples([(12, 20), (10, 18)], depth=True))
    assert [t.shape for t in d["depth"]] == [(12, 20), (10, 18)] and d["depth"][0].dtype == torch.float32
    assert len(d["depth_context"]) == 2 and d["depth_context"][1][1].shape == (10, 18)


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


@pytest.mark.gpu
def test_gpu_pipeline_depth_two_raw_sizes():
    """Supervised batches: 'depth' and 'depth_context' of samples
    from two KITTI drives (375x1242, 370x1226) come out [B, 1, 192, 640] on the
    device, each sample equal to resize_depth (cv2 INTER_NEAREST restated in
    the oracle) + ToTensor -- the resolution SupervisedDepthPoseLoss needs."""
    from oracle import dro_oracle as O
    from dro_sfm_amd.datasets.gpu_loader import GPUTrainPipeline, collate_decoded
    H, W = 192, 640
    sizes = [(375, 1242), (370, 1226), (370, 1226)]
    s = _samples(sizes, depth=True)
    out = GPUTrainPipeline((H, W), JIT, generator=torch.Generator().manual_seed(5))(collate_decoded(s))
    assert out["depth"].shape == (3, 1, H, W) and out["depth"].is_cuda
    assert len(out["depth_context"]) == 2 and out["depth_context"][0].shape == (3, 1, H, W)
    for n in range(3):
        want = O.resize_depth_cv2_nearest(s[n]["depth"], (H, W))[..., 0]
        assert np.array_equal(out["depth"][n, 0].cpu().numpy(), want), n
        for j in range(2):
            want = O.resize_depth_cv2_nearest(s[n]["depth_context"][j], (H, W))[..., 0]
            assert np.array_equal(out["depth_context"][j][n, 0].cpu().numpy(), want), (n, j)


def _png_samples(tmp_path, sizes, seed=21, n_ctx=2):
    """Samples whose frames are lazily opened PNG files (load_image =
    Image.open, utils/image.py:13-27), textured so the encoder uses every
    filter and real Huffman blocks."""
    from PIL import Image
    rng = np.random.default_rng(seed)
    out = []
    for i, (h0, w0) in enumerate(sizes):
        def img(tag):
            y, x = np.mgrid[0:h0, 0:w0]
            a = np.stack([(x * (2 + c) + y * 3 + rng.integers(0, 9)) % 256 for c in range(3)], -1)
            a = (a + rng.integers(0, 24, a.shape)).clip(0, 255).astype(np.uint8)
            fn = str(tmp_path / f"s{i}_{tag}.png")
            Image.fromarray(a).save(fn)
            return Image.open(fn)
        K = np.array([[721.5, 0.0, w0 / 2], [0.0, 721.5, h0 / 2], [0.0, 0.0, 1.0]], np.float32)
        out.append({"idx": i, "rgb": img("t"), "rgb_context": [img(f"c{j}") for j in range(n_ctx)],
                    "intrinsics": K, "pose_context": [np.eye(4, dtype=np.float32)] * n_ctx})
    return out


def test_collate_encoded_keeps_png_streams(tmp_path):
    """With GPU decoding the workers do not decode PNG frames: they pass the
    parsed streams (PngInfo); in-memory (non-file) frames are decoded as before."""
    from dro_sfm_amd.datasets.gpu_loader import collate_encoded
    from dro_sfm_amd.datasets.png import PngInfo
    s = _png_samples(tmp_path, [(12, 20), (10, 18)])
    s[1]["rgb"] = s[1]["rgb"].copy()                      # an in-memory image: no file behind it
    b = collate_encoded(s)
    assert isinstance(b["rgb"][0], PngInfo) and b["rgb"][0].key == (12, 20, 2)
    assert torch.is_tensor(b["rgb"][1]) and b["rgb"][1].shape == (10, 18, 3)
    assert isinstance(b["rgb_context"][1][1], PngInfo) and b["rgb_context"][1][1].key == (10, 18, 2)


@pytest.mark.gpu
def test_gpu_pipeline_with_gpu_decode_equals_host_decode(tmp_path):
    """The whole GPU pipeline fed encoded PNG frames (decoded on the GPU, two
    raw sizes in one batch) == the same pipeline fed Pillow-decoded frames:
    every output tensor bit-identical."""
    from dro_sfm_amd.datasets.gpu_loader import GPUTrainPipeline, collate_decoded, collate_encoded
    s = _png_samples(tmp_path, [(375, 1242), (370, 1226), (370, 1226)])
    a = GPUTrainPipeline((192, 640), JIT, generator=torch.Generator().manual_seed(7))(collate_encoded(s))
    b = GPUTrainPipeline((192, 640), JIT, generator=torch.Generator().manual_seed(7))(collate_decoded(s))
    for key in ("rgb", "rgb_original", "intrinsics"):
        assert torch.equal(a[key], b[key]), key
    for key in ("rgb_context", "rgb_context_original"):
        for x, y in zip(a[key], b[key]):
            assert torch.equal(x, y), key
