"""Shared, dependency-free helpers for the golden generator and the tests.

Test infrastructure only.  Nothing in the product package imports this file.

* ``det_init``   -- deterministic, name-keyed parameter fill.  The reference
  initialises its nets with kaiming draws in construction order
  (``dro_sfm/networks/optim/extractor.py:49-54``) and a torchvision download
  (``extractor.py:56-57``, never run here).  Golden fixtures instead fill every
  parameter from a generator seeded by ``crc32(state_dict key)``, so any
  implementation that keeps the reference ``state_dict`` key names
   reproduces the exact same weights without shipping them.
* ``smooth_images`` / ``kitti_K`` -- the synthetic inputs of SURVEY.md §8(d).
"""
import zlib

import numpy as np
import torch

KITTI_K_640 = [[371.8, 0.0, 314.1], [0.0, 369.4, 88.5], [0.0, 0.0, 1.0]]
SCANNET_K_320 = [[289.0, 0.0, 160.0], [0.0, 290.0, 120.0], [0.0, 0.0, 1.0]]


def kitti_K(B, W=640, H=192):
    """KITTI P_rect_02 intrinsics rescaled to a W-wide image."""
    s = W / 640.0
    sy = H / 192.0
    K = torch.tensor(KITTI_K_640, dtype=torch.float32)
    K[0, 0] *= s
    K[0, 2] *= s
    K[1, 1] *= sy
    K[1, 2] *= sy
    return K.unsqueeze(0).repeat(B, 1, 1).contiguous()


def _gen(name, salt=0):
    g = torch.Generator()
    g.manual_seed((zlib.crc32(name.encode()) + 7919 * salt) & 0x7FFFFFFF)
    return g


def fill_tensor(name, t, salt=0, gain=1.0):
    """Deterministic value of one state_dict entry, keyed by its name."""
    with torch.no_grad():
        if name.endswith("num_batches_tracked"):
            t.zero_()
        elif name.endswith("running_mean"):
            t.zero_()
        elif name.endswith("running_var"):
            t.fill_(1.0)
        elif t.dim() >= 2:
            fan_in = t[0].numel()
            w = torch.randn(t.shape, generator=_gen(name, salt))
            t.copy_(w * (gain / fan_in) ** 0.5)
        elif name.endswith("bias"):
            t.copy_(0.05 * torch.randn(t.shape, generator=_gen(name, salt)))
        else:  # 1-d weights: norm-layer affine
            t.copy_(1.0 + 0.1 * torch.randn(t.shape, generator=_gen(name, salt)))
    return t


def det_init(module, salt=0, gain=1.0):
    """Fill every parameter/buffer of ``module`` from its state_dict key."""
    for name, t in module.state_dict().items():
        fill_tensor(name, t, salt, gain)
    return module


def params_from_spec(spec, salt=0):
    """{name: shape} (e.g. a *_keys.json fixture) -> {name: filled fp32 tensor}."""
    out = {}
    for name, shape in spec.items():
        dt = torch.int64 if name.endswith("num_batches_tracked") else torch.float32
        out[name] = fill_tensor(name, torch.empty(tuple(shape), dtype=dt), salt)
    return out


def load_spec(path):
    import json
    with open(path) as f:
        return json.load(f)


def smooth_images(n, H, W, seed, detail=0.1):
    """Bilinear-upsampled U[0,1) noise at 1/8 res + `detail` x U[0,1) detail, clamped."""
    g = torch.Generator()
    g.manual_seed(seed)
    lo = torch.rand(n, 3, max(H // 8, 2), max(W // 8, 2), generator=g)
    up = torch.nn.functional.interpolate(lo, size=(H, W), mode="bilinear", align_corners=False)
    img = up + detail * torch.rand(n, 3, H, W, generator=g)
    return img.clamp(0.0, 1.0).contiguous()


def to_np(x):
    if isinstance(x, torch.Tensor):
        return x.detach().cpu().numpy()
    return np.asarray(x)


def load_fixture(path):
    with np.load(path, allow_pickle=False) as z:
        return {k: torch.from_numpy(z[k].copy()) for k in z.files}
