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


# the update heads' output convolutions: the per-step inverse-depth / pose
# increments of the recurrence (reference networks/optim/update.py DepthHead.conv2,
# PoseHead.conv2_pose)
DAMPED = ("update_block_depth.depth_head.conv2.", "update_block_pose.pose_head.conv2_pose.", "pose_head.conv2_pose.")


def condition_params(params, damp):
    """The documented damping of the full-size train-step parity tests
    (tests/test_hip_parity.py): the update heads' output
    convolutions (weight and bias) scaled by `damp`.  At random init those
    increments are large and the it8 / it12-h recurrences amplify fp32
    rounding by orders of magnitude at 192x640 and 240x320
    (tools/conditioning.py); damped, the recurrence is a small perturbation of
    its start and an fp32 evaluation of the reference algorithm stays within
    ~1e-5 of fp64, so fixed bounds can fail.  Every parameter still gets a
    gradient through the same graph.  damp = 1: unchanged."""
    if damp == 1.0:
        return params
    out = dict(params)
    for k, v in params.items():
        if k.startswith(DAMPED) and v.is_floating_point():
            out[k] = v * damp
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


GRAD_SAMPLE = 2048


def grad_sample_index(name, numel, k=GRAD_SAMPLE):
    """Deterministic sample of k flat indices of parameter `name`'s gradient
    (the train-step fixtures store gradients of large encoder tensors at these
    indices; the tests read the same entries).  None: the tensor is small
    enough to be stored whole."""
    if numel <= k:
        return None
    return torch.randperm(numel, generator=_gen("gidx:" + name))[:k].sort().values


def grad_fixture(named_grads, full_prefixes=()):
    """{'gfull.<name>': whole gradient} for parameters under `full_prefixes` or
    with <= GRAD_SAMPLE entries, else {'gsamp.<name>': gradient at
    grad_sample_index(name)} -- per-element values, not checksums."""
    out = {}
    for name, g in named_grads:
        if g is None:
            continue
        idx = grad_sample_index(name, g.numel())
        if idx is None or name.split(".")[0] in full_prefixes:
            out["gfull." + name] = g.detach().clone()
        else:
            out["gsamp." + name] = g.detach().flatten()[idx].clone()
    return out


def grad_errors(named_grads, fixture):
    """Per parameter: max|g - g_ref| / max|g_ref| over the fixture's stored
    entries (whole tensors 'gfull.*' or the sampled 'gsamp.*').  Returns
    {name: error}; every stored gradient must be present in named_grads."""
    got = dict(named_grads)
    out = {}
    for key, ref in fixture.items():
        if not key.startswith(("gfull.", "gsamp.")):
            continue
        name = key.split(".", 1)[1]
        g = got[name]
        assert g is not None, f"no gradient for {name}"
        g = g.detach().cpu()
        if key.startswith("gsamp."):
            g = g.flatten()[grad_sample_index(name, g.numel())]
        else:
            g = g.reshape(ref.shape)
        ref = ref.double()
        out[name] = float((g.double() - ref).abs().max() / ref.abs().max().clamp_min(1e-30))
    return out


def fval(t):
    """A scalar fixture entry (stored as float32) back as the Python float the
    generator passed to the reference (shortest float32 repr: 0.2, not
    0.2000000030): depth ranges enter 1/min_depth and the validity masks."""
    return float(np.format_float_positional(np.float32(float(t)), unique=True))
