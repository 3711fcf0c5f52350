"""GPU-side resize + to-tensor for the training transforms.

The reference's train_transforms (dro_sfm/datasets/transforms.py:8-31) run on
CPU data-loader workers over PIL images: resize_sample (augmentations.py:69-
133: torchvision Resize((H, W), BILINEAR) of 'rgb' / 'rgb_context' and the
intrinsics scaled by out/in), duplicate_sample (:186-211), colorjitter_sample
(:213-258) and to_tensor_sample (:149-184).  At 8 GPUs x ~100 frames/s each
the PIL resize of 375x1242 KITTI frames on the host becomes the bottleneck.
Here decoded frames travel to the GPU as uint8 (a quarter of the float
bytes) and csrc/resize.hip resamples them bit-identically to Pillow, applies
torchvision's ColorJitter (the reference default jittering = (0.2, 0.2, 0.2,
0.05), configs/default_config.py:145) bit-identically to Pillow's
ImageEnhance / HSV arithmetic, and writes the float CHW tensors.  The
jitter's random order and factors are drawn on the host from torch's
generator in the reference's exact order per sample (colorjitter_sample,
augmentations.py:226-256): its Python `random.random()` gate, one get_params
draw that the reference discards, then one ColorJitter draw per image --
'rgb', then each 'rgb_context' frame -- so a seeded run reproduces the
reference's augmentations, not only their distribution.  Decoding stays on
the host.
"""
import ctypes
import random
from functools import lru_cache

import numpy as np
import torch

from ..hip import _lib
from ..hip._lib import check, ptr, require_device, stream_of

_PREC = 22   # Pillow Resample.c PRECISION_BITS for 8-bit images (32 - 8 - 2)


@lru_cache(maxsize=64)
def pil_bilinear_coeffs(in_size, out_size):
    """Pillow's precompute_coeffs + normalize_coeffs_8bpc for the bilinear
    (triangle, support 1) filter: per output index (xmin, count) and the
    fixed-point weights, padded to a common width.  Host arithmetic in double,
    as Pillow does."""
    scale = in_size / out_size
    filterscale = max(scale, 1.0)
    support = filterscale
    ss = 1.0 / filterscale
    bounds, coefs = [], []
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), in_size) - xmin
        ws = []
        for x in range(xmax):
            t = abs((x + xmin - center + 0.5) * ss)
            ws.append(1.0 - t if t < 1.0 else 0.0)
        total = sum(ws)
        if total != 0.0:
            ws = [w / total for w in ws]
        coefs.append([int(w * (1 << _PREC) + (0.5 if w >= 0 else -0.5)) for w in ws])
        bounds.append((xmin, xmax))
    K = max(len(c) for c in coefs)
    table = np.zeros((out_size, K), np.int32)
    for i, c in enumerate(coefs):
        table[i, :len(c)] = c
    return np.asarray(bounds, np.int32), table


_DEV_TABLES = {}


def _tables(in_size, out_size, device):
    key = (in_size, out_size, str(device))
    if key not in _DEV_TABLES:
        b, c = pil_bilinear_coeffs(in_size, out_size)
        _DEV_TABLES[key] = (torch.from_numpy(b).to(device), torch.from_numpy(c).to(device), c.shape[1])
    return _DEV_TABLES[key]


def resize_to_tensor(frames, shape):
    """frames: uint8 [N, H0, W0, 3] (decoded RGB, HWC) on the GPU -> float32
    [N, 3, H, W] = ToTensor(Resize(shape, BILINEAR)(frame)) for every frame."""
    lib = _lib.load()
    if frames.dtype != torch.uint8 or frames.dim() != 4 or frames.shape[-1] != 3:
        raise RuntimeError("resize_to_tensor: expects uint8 [N, H0, W0, 3] frames")
    if not frames.is_cuda:
        raise RuntimeError("dro_sfm_amd.resize_to_tensor: tensors must live on a ROCm device (no CPU fallback)")
    N, H0, W0, _ = frames.shape
    H, W = int(shape[0]), int(shape[1])
    frames = frames.contiguous()
    xb, xk, KX = _tables(W0, W, frames.device)
    yb, yk, KY = _tables(H0, H, frames.device)
    tmp = torch.empty(N, H0, W, 3, device=frames.device, dtype=torch.uint8)
    out = torch.empty(N, 3, H, W, device=frames.device, dtype=torch.float32)
    check(lib.dro_resize_rgb8_to_tensor(ptr(frames), N, H0, W0, H, W, ptr(xb), ptr(xk), KX, ptr(yb), ptr(yk),
                                        KY, ptr(tmp), ptr(out), stream_of(out)),
          "dro_resize_rgb8_to_tensor")
    return out


def resize_sample_to_tensor(sample, shape):
    """resize_sample + duplicate_sample + to_tensor_sample of a batch whose
    'rgb' is uint8 [B, H0, W0, 3] and 'rgb_context' a list of those, on the
    GPU; 'intrinsics' [B, 3, 3] (or [3, 3]) scaled as augmentations.py:93-99.
    Returns a new dict with float32 'rgb', 'rgb_context' and the '_original'
    copies (no colour jitter: identical tensors)."""
    out = dict(sample)
    H0, W0 = sample["rgb"].shape[1:3]
    H, W = int(shape[0]), int(shape[1])
    out["rgb"] = resize_to_tensor(sample["rgb"], shape)
    out["rgb_context"] = [resize_to_tensor(c, shape) for c in sample["rgb_context"]]
    out["rgb_original"] = out["rgb"]
    out["rgb_context_original"] = list(out["rgb_context"])
    if "intrinsics" in sample:
        K = sample["intrinsics"].clone()
        K[..., 0, :] *= W / W0
        K[..., 1, :] *= H / H0
        out["intrinsics"] = K
    return out


def _check_frames(frames, what):
    if frames.dtype != torch.uint8 or frames.dim() != 4 or frames.shape[-1] != 3:
        raise RuntimeError(f"{what}: expects uint8 [N, H, W, 3] frames")
    if not frames.is_cuda:
        raise RuntimeError(f"dro_sfm_amd.{what}: tensors must live on a ROCm device (no CPU fallback)")


def resize_rgb8(frames, shape):
    """uint8 [N, H0, W0, 3] -> uint8 [N, H, W, 3], Pillow BILINEAR (the resized PIL image)."""
    lib = _lib.load()
    _check_frames(frames, "resize_rgb8")
    N, H0, W0, _ = frames.shape
    H, W = int(shape[0]), int(shape[1])
    frames = frames.contiguous()
    xb, xk, KX = _tables(W0, W, frames.device)
    yb, yk, KY = _tables(H0, H, frames.device)
    tmp = torch.empty(N, H0, W, 3, device=frames.device, dtype=torch.uint8)
    out = torch.empty(N, H, W, 3, device=frames.device, dtype=torch.uint8)
    check(lib.dro_resize_rgb8(ptr(frames), N, H0, W0, H, W, ptr(xb), ptr(xk), KX, ptr(yb), ptr(yk), KY,
                              ptr(tmp), ptr(out), stream_of(out)), "dro_resize_rgb8")
    return out


def rgb8_to_tensor(frames):
    """ToTensor of uint8 [N, H, W, 3] frames -> float32 [N, 3, H, W] (value / 255)."""
    lib = _lib.load()
    _check_frames(frames, "rgb8_to_tensor")
    N, H, W, _ = frames.shape
    frames = frames.contiguous()
    out = torch.empty(N, 3, H, W, device=frames.device, dtype=torch.float32)
    check(lib.dro_rgb8_to_tensor(ptr(frames), N, H, W, ptr(out), stream_of(out)), "dro_rgb8_to_tensor")
    return out


def colorjitter_params(jittering, n, generator=None):
    """torchvision ColorJitter.get_params for n frames (one draw per frame, as
    the reference applies its transform object per image):
    (brightness, contrast, saturation, hue) -> ranges [max(0, 1 - x), 1 + x]
    and [-hue, hue] (augmentations.py:236-245); per frame randperm(4), then
    uniform brightness, contrast, saturation, hue factors.  Returns
    (order [n, 4] int, factors [n, 3] float, hue [n] float)."""
    b, c, s, h = jittering
    rng = [(max(0.0, 1 - b), 1 + b), (max(0.0, 1 - c), 1 + c), (max(0.0, 1 - s), 1 + s)]
    orders, factors, hues = [], [], []
    for _ in range(n):
        orders.append(torch.randperm(4, generator=generator).tolist())
        factors.append([float(torch.empty(1).uniform_(lo, hi, generator=generator)) for lo, hi in rng])
        hues.append(float(torch.empty(1).uniform_(-h, h, generator=generator)))
    return orders, factors, hues


def color_jitter_(frames, orders, factors, hues):
    """In-place ColorJitter of uint8 [N, H, W, 3] frames on the GPU with the
    given per-frame order / factors / hue factors (colorjitter_params)."""
    lib = _lib.load()
    _check_frames(frames, "color_jitter")
    if not frames.is_contiguous():
        raise RuntimeError("color_jitter_: frames must be contiguous (in place)")
    N, H, W, _ = frames.shape
    prm = np.zeros((N, 8), np.int32)
    for i in range(N):
        prm[i, :4] = orders[i]
        prm[i, 4:7] = np.asarray(factors[i], np.float32).view(np.int32)
        prm[i, 7] = int(hues[i] * 255) & 255        # np.array(h * 255).astype(np.uint8): trunc, wrap
    prm_d = torch.from_numpy(prm).to(frames.device)
    ws = torch.empty(N, device=frames.device, dtype=torch.int64)
    check(lib.dro_color_jitter_rgb8(ptr(frames), N, H, W, ptr(prm_d), ptr(ws), stream_of(frames)),
          "dro_color_jitter_rgb8")
    return frames


def train_transforms(sample, image_shape, jittering, generator=None):
    """train_transforms (reference datasets/transforms.py:8-31) on the GPU for a
    batch whose 'rgb' is uint8 [B, H0, W0, 3] and 'rgb_context' a list of
    those: resize_sample -> duplicate_sample -> colorjitter_sample ->
    to_tensor_sample.  colorjitter_sample's own `random.random() < prob`
    gate has prob = 1.0 in the reference, so every batch is jittered."""
    out = dict(sample)
    frames = [sample["rgb"]] + list(sample["rgb_context"])
    H0, W0 = sample["rgb"].shape[1:3]
    resized = [resize_rgb8(f, image_shape) if len(image_shape) else f.contiguous() for f in frames]
    originals = [rgb8_to_tensor(r) for r in resized]
    if len(jittering) > 0:
        # per sample, in colorjitter_sample's order (augmentations.py:226-256)
        B, F = resized[0].shape[0], len(resized)
        per = [[None] * B for _ in range(F)]
        for b in range(B):
            random.random()                                  # `random.random() < prob` (prob 1.0)
            colorjitter_params(jittering, 1, generator)      # get_params result the reference discards
            for f in range(F):                               # 'rgb', then 'rgb_context' in order
                o, fa, hu = colorjitter_params(jittering, 1, generator)
                per[f][b] = (o[0], fa[0], hu[0])
        for f, r in enumerate(resized):
            color_jitter_(r, [p[0] for p in per[f]], [p[1] for p in per[f]], [p[2] for p in per[f]])
    tensors = [rgb8_to_tensor(r) for r in resized]
    out["rgb"], out["rgb_context"] = tensors[0], tensors[1:]
    out["rgb_original"], out["rgb_context_original"] = originals[0], originals[1:]
    if "intrinsics" in sample and len(image_shape):
        K = sample["intrinsics"].clone()
        K[..., 0, :] *= image_shape[1] / W0
        K[..., 1, :] *= image_shape[0] / H0
        out["intrinsics"] = K
    return out
