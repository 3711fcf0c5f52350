"""GPU-side resize + to-tensor for the training transforms.

The reference's train_transforms (dro_sfm/datasets/transforms.py:8-31) run on
CPU data-loader workers over PIL images: resize_sample (augmentations.py:69-
133: torchvision Resize((H, W), BILINEAR) of 'rgb' / 'rgb_context' and the
intrinsics scaled by out/in), duplicate_sample (:186-211), colorjitter_sample
(:213-258) and to_tensor_sample (:149-184).  At 8 GPUs x ~100 frames/s each
the PIL resize of 375x1242 KITTI frames on the host becomes the bottleneck.
Here decoded frames travel to the GPU as uint8 (a quarter of the float
bytes) and csrc/resize.hip resamples them bit-identically to Pillow and
writes the float CHW tensors directly.  Colour jittering stays out (the
reference's yamls for the metric config train without it -- jittering is a
data-loader option); decoding stays on the host.
"""
import ctypes
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
