"""CPU ORACLE for the GPU PNG decoder (csrc/png.hip) -- TEST INFRASTRUCTURE ONLY.

The reference decodes its frames with Pillow (utils/image.py:13-27
load_image = PIL.Image.open; datasets/kitti_dataset.py:38-44 read_png_depth).
Pillow's PNG decoding lives in a third-party dependency absent from
/root/reference (Pillow 12.2 is installed here; its C decoder inflates with
zlib, then undoes the per-row filters of the PNG specification, ISO/IEC
15948 section 9).  This module restates that algorithm:

  * inflate: Python's zlib.decompress (the same zlib Pillow links against);
  * unfilter: the five row filters (None, Sub, Up, Average, Paeth) in numpy,
    one row at a time, vectorised over the bytes that do not depend on each
    other (Up, and each of a row's bpp byte lanes for the others);
  * output conventions: Image.convert("RGB") for 8-bit grey / RGB / RGBA,
    read_png_depth's value / 256 (-1 where 0) for 16-bit grey.

Pinned against Pillow itself on the committed fixtures and on generated images
(tests/test_png.py).  Only tests/ import it; the product decodes on the GPU.
"""
import struct
import zlib

import numpy as np


def parse(data):
    """(width, height, bit depth, colour type, concatenated IDAT) of PNG bytes."""
    assert data[:8] == b"\x89PNG\r\n\x1a\n", "not a PNG"
    pos, ihdr, idat = 8, None, []
    while pos < len(data):
        n, typ = struct.unpack(">I4s", data[pos:pos + 8])
        body = data[pos + 8:pos + 8 + n]
        if typ == b"IHDR":
            ihdr = struct.unpack(">IIBBBBB", body)
        elif typ == b"IDAT":
            idat.append(body)
        elif typ == b"IEND":
            break
        pos += 12 + n
    w, h, depth, ctype, _, _, interlace = ihdr
    assert interlace == 0
    return w, h, depth, ctype, b"".join(idat)


def _paeth(a, b, c):
    p = a + b - c
    pa, pb, pc = np.abs(p - a), np.abs(p - b), np.abs(p - c)
    return np.where((pa <= pb) & (pa <= pc), a, np.where(pb <= pc, b, c))


def unfilter(raw, h, w, bpp):
    """PNG filters undone (ISO/IEC 15948 section 9.2): raw = h rows of
    (filter byte + w * bpp bytes) -> uint8 [h, w * bpp]."""
    stride = 1 + w * bpp
    buf = np.frombuffer(raw, dtype=np.uint8)
    assert buf.size == h * stride, (buf.size, h * stride)
    out = np.zeros((h, w * bpp), dtype=np.int32)
    prev = np.zeros(w * bpp, dtype=np.int32)
    for r in range(h):
        ft = int(buf[r * stride])
        x = buf[r * stride + 1:(r + 1) * stride].astype(np.int32)
        if ft == 0:
            cur = x
        elif ft == 2:
            cur = (x + prev) & 255
        elif ft in (1, 3, 4):
            cur = np.zeros_like(x)
            for i in range(0, w * bpp, bpp):        # left neighbour: bpp bytes back
                a = cur[i - bpp:i] if i else np.zeros(bpp, dtype=np.int32)
                b = prev[i:i + bpp]
                c = prev[i - bpp:i] if i else np.zeros(bpp, dtype=np.int32)
                pred = a if ft == 1 else ((a + b) >> 1 if ft == 3 else _paeth(a, b, c))
                cur[i:i + bpp] = (x[i:i + bpp] + pred) & 255
        else:
            raise ValueError(f"row {r}: filter type {ft}")
        out[r] = cur
        prev = cur
    return out.astype(np.uint8)


def decode(data):
    """PNG bytes -> uint8 [H, W, 3] (8-bit grey / RGB / RGBA, as
    Image.convert("RGB")) or float32 [H, W] depth (16-bit grey, as
    read_png_depth: value / 256, -1 where 0)."""
    w, h, depth, ctype, idat = parse(data)
    bpp = {(8, 0): 1, (8, 2): 3, (8, 6): 4, (16, 0): 2}[(depth, ctype)]
    px = unfilter(zlib.decompress(idat), h, w, bpp).reshape(h, w, bpp)
    if depth == 16:
        v = (px[..., 0].astype(np.int32) << 8) | px[..., 1]
        return np.where(v == 0, -1.0, v / 256.0).astype(np.float32)
    if ctype == 0:
        return np.repeat(px, 3, axis=2)
    return np.ascontiguousarray(px[..., :3])
