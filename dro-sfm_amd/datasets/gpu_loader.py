"""The GPU data path hooked to the reference's datasets.

The reference's datasets decode frames on CPU workers and then apply
`data_transform` = train_transforms (resize, duplicate, colour jitter,
to_tensor; dro_sfm/datasets/transforms.py:8-31) there too
(KITTIDataset.__getitem__, kitti_dataset.py:348-404, `self.data_transform(sample)`
at :399).  Here the same dataset classes are built with `data_transform=None`
(their __getitem__ then returns the decoded PIL frames, the intrinsics and
the context poses untouched), and:

  * `collate_decoded` (DataLoader collate_fn, CPU worker) stacks the decoded
    uint8 HWC frames into pinned host tensors -- one quarter of the bytes the
    float tensors of the reference's path would move;
  * `GPUTrainPipeline` (training process) copies them to the GPU
    (non_blocking) and runs train_transforms there
    (datasets/gpu_transforms.py: Pillow-exact resize, torchvision-exact
    ColorJitter in the reference's draw order, ToTensor), intrinsics scaled per
    sample by its own raw size.  KITTI drives differ in raw size (375x1242,
    370x1226, 374x1238, ...): samples of one size are resized in one launch,
    per size group, and the batch is reassembled in sample order.

With gpu_decode=True (round 6) PNG frames are decoded on the GPU as well
(datasets/png.py, csrc/png.hip: inflate + row filters, bit-identical to
Pillow): the workers only open the files (PIL's Image.open is lazy), read their
bytes and walk the PNG chunks; GPUTrainPipeline decodes every frame of the
batch in one launch pair per geometry before the transforms.  JPEG frames (no
GPU decoder here) are decoded by the workers as before.
"""
import numpy as np
import torch

from .gpu_transforms import train_transforms


def _png_source(img):
    """The PNG file behind a lazily opened PIL image (load_image), or None."""
    fn = getattr(img, "filename", None)
    return fn if getattr(img, "format", None) == "PNG" and fn else None


def _frame(img, gpu_decode):
    """A worker-side frame: PngInfo (the compressed stream; decoded on the GPU)
    when gpu_decode and the image is a PNG file, else uint8 HWC pixels."""
    if gpu_decode:
        fn = _png_source(img)
        if fn is not None:
            from .png import parse_png
            with open(fn, "rb") as f:
                return parse_png(f.read())
    return _as_uint8(img)


def _as_uint8(img):
    a = np.asarray(img)
    if a.dtype != np.uint8 or a.ndim != 3 or a.shape[2] != 3:
        a = np.asarray(img.convert("RGB") if hasattr(img, "convert") else a, dtype=np.uint8)
    return torch.from_numpy(np.ascontiguousarray(a))


def _depth_map(d):
    """A decoded depth map (np [h,w] or [h,w,1]) as float32 [h, w]."""
    a = np.asarray(d, dtype=np.float32)
    if a.ndim == 3:
        a = a[..., 0]
    return torch.from_numpy(np.ascontiguousarray(a))


def nearest_indices(src, dst):
    """cv2.resize(..., INTER_NEAREST) source index per destination index along one
    axis (OpenCV resizeNN: ifx = 1 / (dst / src) in double, floor(x * ifx),
    clamped to src - 1)."""
    ifx = 1.0 / (float(dst) / float(src))
    return np.minimum(np.floor(np.arange(dst, dtype=np.float64) * ifx).astype(np.int64), src - 1)


def resize_depth_nearest(depth, shape):
    """augmentations.resize_depth (augmentations.py:47-65: cv2 INTER_NEAREST to
    dsize=shape[::-1]) + ToTensor for a batch of depth maps of one raw size on
    the GPU: [B, h, w] -> [B, 1, H, W], a pure gather (bit-exact)."""
    H, W = shape
    h, w = depth.shape[-2:]
    iy = torch.from_numpy(nearest_indices(h, H)).to(depth.device, non_blocking=True)
    ix = torch.from_numpy(nearest_indices(w, W)).to(depth.device, non_blocking=True)
    return depth.index_select(-2, iy).index_select(-1, ix).unsqueeze(1)


def collate_encoded(samples):
    """collate_decoded with PNG frames left encoded (datasets/png.PngInfo):
    GPUTrainPipeline decodes them on the GPU."""
    return collate_decoded(samples, gpu_decode=True)


def collate_decoded(samples, gpu_decode=False):
    """Collate reference samples built WITHOUT data_transform: 'rgb' and
    'rgb_context' (PIL images or uint8 HWC arrays) become lists of uint8
    [H0, W0, 3] tensors (pinned when a GPU is present; per sample, raw sizes
    may differ); 'intrinsics' float32 [B, 3, 3]; 'pose_context' a list over
    references of float32 [B, 4, 4]; 'depth' a list of float32 [h0, w0] raw
    maps ('depth_context' a list over references of such lists) when present;
    other keys as lists."""
    pin = torch.cuda.is_available()
    out = {}

    def host(img):
        t = _frame(img, gpu_decode)
        return t.pin_memory() if pin and torch.is_tensor(t) else t

    out["rgb"] = [host(s["rgb"]) for s in samples]
    if "rgb_context" in samples[0]:
        n = len(samples[0]["rgb_context"])
        out["rgb_context"] = [[host(s["rgb_context"][j]) for s in samples] for j in range(n)]
    if "intrinsics" in samples[0]:
        out["intrinsics"] = torch.stack([torch.as_tensor(np.asarray(s["intrinsics"]), dtype=torch.float32)
                                         for s in samples])
    if "pose_context" in samples[0]:
        n = len(samples[0]["pose_context"])
        out["pose_context"] = [torch.stack([torch.as_tensor(np.asarray(s["pose_context"][j]), dtype=torch.float32)
                                            for s in samples]) for j in range(n)]
    if "depth" in samples[0]:
        # per sample, at the raw size (drives differ); resized on the GPU
        out["depth"] = [_depth_map(s["depth"]) for s in samples]
    if "depth_context" in samples[0]:
        n = len(samples[0]["depth_context"])
        out["depth_context"] = [[_depth_map(s["depth_context"][j]) for s in samples] for j in range(n)]
    for k in samples[0]:
        if k not in out:
            out[k] = [s[k] for s in samples]
    return out


class GPUTrainPipeline:
    """Host batch from `collate_decoded` -> the model's training batch on the
    GPU: train_transforms(image_shape, jittering) exactly as the reference's
    data_transform would have produced it on the CPU workers (same random
    draws from `generator`, in the reference's per-sample order)."""

    def __init__(self, image_shape, jittering=(0.2, 0.2, 0.2, 0.05), device=None, generator=None):
        self.image_shape = tuple(int(v) for v in image_shape)
        self.jittering = tuple(jittering)
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.generator = generator

    def __call__(self, host):
        dev = self.device
        B = len(host["rgb"])
        N = len(host.get("rgb_context", []))
        frames = self._frames([host["rgb"]] + [host["rgb_context"][j] for j in range(N)])
        K = host["intrinsics"].to(dev, non_blocking=True) if "intrinsics" in host else None
        sizes = [tuple(f.shape[:2]) for f in frames[0]]
        # jitter draws must follow sample order: group only consecutive equal sizes
        groups, start = [], 0
        for b in range(1, B + 1):
            if b == B or sizes[b] != sizes[start]:
                groups.append((start, b))
                start = b
        parts = []
        for lo, hi in groups:
            sub = {"rgb": torch.stack(frames[0][lo:hi]),
                   "rgb_context": [torch.stack(frames[1 + j][lo:hi]) for j in range(N)]}
            if K is not None:
                sub["intrinsics"] = K[lo:hi]
            parts.append(train_transforms(sub, self.image_shape, self.jittering, self.generator))
        cat = lambda key: torch.cat([p[key] for p in parts]) if len(parts) > 1 else parts[0][key]
        out = {k: v for k, v in host.items() if k not in ("rgb", "rgb_context", "intrinsics")}
        out["rgb"], out["rgb_original"] = cat("rgb"), cat("rgb_original")
        out["rgb_context"] = [torch.cat([p["rgb_context"][j] for p in parts]) for j in range(N)]
        out["rgb_context_original"] = [torch.cat([p["rgb_context_original"][j] for p in parts])
                                       for j in range(N)]
        if K is not None:
            out["intrinsics"] = cat("intrinsics")
        if "pose_context" in host:
            out["pose_context"] = [p.to(dev, non_blocking=True) for p in host["pose_context"]]
        if "depth" in host:
            out["depth"] = self._depths(host["depth"])
        if "depth_context" in host:
            out["depth_context"] = [self._depths(d) for d in host["depth_context"]]
        return out

    def _frames(self, lists):
        """Host frames (uint8 tensors, or PngInfo streams from collate_encoded)
        -> uint8 [H0, W0, 3] device tensors; every encoded frame of the batch is
        decoded on the GPU in one launch pair per geometry."""
        dev = self.device
        flat = [f for lst in lists for f in lst]
        enc = [i for i, f in enumerate(flat) if not torch.is_tensor(f)]
        dec = {}
        if enc:
            from .png import decode_pngs
            for i, t in zip(enc, decode_pngs([flat[i] for i in enc], dev)):
                if t.dim() != 3:
                    raise RuntimeError("GPUTrainPipeline: a 16-bit PNG among the RGB frames")
                dec[i] = t
        out, k = [], 0
        for lst in lists:
            row = []
            for f in lst:
                row.append(dec[k] if k in dec else f.to(dev, non_blocking=True))
                k += 1
            out.append(row)
        return out

    def _depths(self, maps):
        """Per-sample raw depth maps -> [B, 1, H, W] on the device (nearest
        neighbour, resize_sample's depth branch, augmentations.py:135-143),
        one gather per run of equal raw sizes."""
        dev = self.device
        maps = [m.to(dev, non_blocking=True) for m in maps]
        parts, start = [], 0
        for b in range(1, len(maps) + 1):
            if b == len(maps) or maps[b].shape != maps[start].shape:
                parts.append(resize_depth_nearest(torch.stack(maps[start:b]), self.image_shape))
                start = b
        return torch.cat(parts) if len(parts) > 1 else parts[0]


def gpu_data_loader(dataset, batch_size, image_shape, jittering=(0.2, 0.2, 0.2, 0.05), num_workers=4,
                    shuffle=True, generator=None, device=None, gpu_decode=False, **loader_kw):
    """Iterate a reference dataset built with data_transform=None through the
    GPU pipeline: a DataLoader over collate_decoded (workers decode and stack
    uint8 frames; with gpu_decode, collate_encoded: PNG frames stay encoded and
    are decoded on the GPU) whose batches GPUTrainPipeline transforms on the GPU."""
    loader = torch.utils.data.DataLoader(dataset, batch_size=batch_size, shuffle=shuffle, num_workers=num_workers,
                                         collate_fn=collate_encoded if gpu_decode else collate_decoded, **loader_kw)
    pipe = GPUTrainPipeline(image_shape, jittering, device=device, generator=generator)
    for host in loader:
        yield pipe(host)
