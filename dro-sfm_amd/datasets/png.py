"""PNG decoding on the GPU (csrc/png.hip), the decode step of the reference's
data pipeline: utils/image.py:13-27 `load_image` (PIL.Image.open) of the KITTI
frames (datasets/kitti_dataset.py:354, :387) and of its 16-bit ground-truth
depth maps (kitti_dataset.py:38-44 `read_png_depth`).

The host only walks the PNG chunks (IHDR, the concatenated IDAT payload);
inflate and the row filters run on the device, one workgroup per image, all
images of one geometry in one launch each way.  Results are bit-identical to
Pillow: frames as uint8 [N, H, W, 3] (Image.convert("RGB")), depth maps as
float32 [N, H, W] = value / 256 with -1 where the value is 0 (read_png_depth).
Supported: non-interlaced 8-bit grey / RGB / RGBA and 16-bit grey -- every
PNG the reference's KITTI / NYU / ScanNet readers open; anything else raises
(no CPU fallback).
"""
import struct
import zlib

import numpy as np
import torch

from ..hip import _lib
from ..hip._lib import check, ptr, stream_of

_SIG = b"\x89PNG\r\n\x1a\n"
# (bit depth, colour type) -> kernel kind
KINDS = {(8, 0): 0, (8, 2): 2, (8, 6): 6, (16, 0): 16}
ERRORS = {1: "bad zlib header", 2: "bad block type / stored length", 3: "bad code lengths", 4: "invalid code",
          5: "distance beyond the output", 6: "output overrun", 7: "compressed stream overrun",
          8: "bad filter type", 9: "short output"}


class PngInfo:
    __slots__ = ("width", "height", "kind", "idat")

    def __init__(self, width, height, kind, idat):
        self.width, self.height, self.kind, self.idat = width, height, kind, idat

    @property
    def key(self):
        return (self.height, self.width, self.kind)


def parse_png(data):
    """(width, height, kind, zlib stream) of a PNG file's bytes.  Chunk CRCs are
    checked; the zlib stream itself is decoded on the device."""
    data = bytes(data)
    if data[:8] != _SIG:
        raise ValueError("not a PNG file")
    pos, ihdr, idat = 8, None, []
    while pos + 8 <= len(data):
        n, typ = struct.unpack(">I4s", data[pos:pos + 8])
        body = data[pos + 8:pos + 8 + n]
        if len(body) != n or pos + 12 + n > len(data):
            raise ValueError("truncated PNG chunk")
        crc = struct.unpack(">I", data[pos + 8 + n:pos + 12 + n])[0]
        if zlib.crc32(typ + body) & 0xFFFFFFFF != crc:
            raise ValueError(f"PNG chunk {typ!r}: CRC mismatch")
        if typ == b"IHDR":
            ihdr = struct.unpack(">IIBBBBB", body)
        elif typ == b"IDAT":
            idat.append(body)
        elif typ == b"IEND":
            break
        pos += 12 + n
    if ihdr is None or not idat:
        raise ValueError("PNG without IHDR / IDAT")
    w, h, depth, ctype, comp, filt, interlace = ihdr
    kind = KINDS.get((depth, ctype))
    if kind is None or comp != 0 or filt != 0 or interlace != 0:
        raise NotImplementedError(f"PNG bit depth {depth}, colour type {ctype}, interlace {interlace}: only "
                                  "non-interlaced 8-bit grey / RGB / RGBA and 16-bit grey are decoded on the GPU")
    return PngInfo(w, h, kind, b"".join(idat))


def _bpp(kind):
    return {0: 1, 2: 3, 6: 4, 16: 2}[kind]


def decode_png_batch(infos, device=None, check_status=True):
    """Decode PNGs of ONE geometry (same height, width and kind) on the GPU.
    infos: PngInfo (parse_png) or raw file bytes.  Returns uint8 [N, H, W, 3]
    (8-bit kinds) or float32 [N, H, W] depth (16-bit grey), on `device`.
    check_status: synchronise and raise on a malformed stream (else the
    per-image int32 status is returned too: 0 = decoded)."""
    infos = [i if isinstance(i, PngInfo) else parse_png(i) for i in infos]
    if not infos:
        raise ValueError("decode_png_batch: no images")
    key = infos[0].key
    if any(i.key != key for i in infos):
        raise ValueError("decode_png_batch: images of one geometry per call (group by PngInfo.key)")
    H, W, kind = key
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    if dev.type != "cuda":
        raise RuntimeError("decode_png_batch: decodes on a ROCm device only (no CPU fallback)")
    lib = _lib.load()
    # the streams back to back, each 4-byte aligned (the kernel reads words)
    sizes = [len(i.idat) for i in infos]
    offs = np.zeros(len(infos) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([(s + 3) // 4 * 4 for s in sizes])
    host = torch.zeros(int(offs[-1]), dtype=torch.uint8)
    hv = host.numpy()
    for i, inf in enumerate(infos):
        hv[offs[i]:offs[i] + sizes[i]] = np.frombuffer(inf.idat, dtype=np.uint8)
    if torch.cuda.is_available():
        host = host.pin_memory()
    zdata = host.to(dev, non_blocking=True)
    # stream i occupies [zoff[i], zoff[i+1]): its bytes, then up to 3 zero pad
    # bytes (after the zlib trailer, never reached by a well-formed stream)
    zoff = torch.from_numpy(offs).to(dev, non_blocking=True)
    N = len(infos)
    flen = int(lib.dro_png_filtered_bytes(H, W, _bpp(kind)))
    filt = torch.empty(N * flen, dtype=torch.uint8, device=dev)
    out = (torch.empty(N, H, W, dtype=torch.float32, device=dev) if kind == 16
           else torch.empty(N, H, W, 3, dtype=torch.uint8, device=dev))
    status = torch.full((N,), -1, dtype=torch.int32, device=dev)
    check(lib.dro_png_decode(ptr(zdata), ptr(zoff), N, H, W, kind, ptr(filt), ptr(out), ptr(status),
                             stream_of(out)), "dro_png_decode")
    if check_status:
        st = status.cpu()
        bad = [(i, int(v)) for i, v in enumerate(st.tolist()) if v != 0]
        if bad:
            raise RuntimeError("decode_png_batch: " + "; ".join(f"image {i}: {ERRORS.get(v, v)}" for i, v in bad))
        return out
    return out, status


def decode_pngs(blobs, device=None):
    """Decode a list of PNG files (bytes / PngInfo) of any geometries: one launch
    pair per geometry; returns the decoded tensors in input order."""
    infos = [b if isinstance(b, PngInfo) else parse_png(b) for b in blobs]
    groups = {}
    for i, inf in enumerate(infos):
        groups.setdefault(inf.key, []).append(i)
    out = [None] * len(infos)
    for idx in groups.values():
        dec = decode_png_batch([infos[i] for i in idx], device)
        for j, i in enumerate(idx):
            out[i] = dec[j]
    return out
