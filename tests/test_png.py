"""GPU PNG decoding (csrc/png.hip, dro_sfm_amd/datasets/png.py) against Pillow,
the decoder behind the reference's load_image / read_png_depth
(utils/image.py:13-27, datasets/kitti_dataset.py:38-44, :354, :387).

Bit-exact: the decoded uint8 frames equal np.asarray(Image.open(f).convert("RGB"))
and the depth maps equal read_png_depth's value / 256 (-1 where 0), on the
committed KITTI-size fixtures (tests/golden/gen_png.py) and on PNGs built here
with every row filter and every DEFLATE block type (stored, fixed, dynamic;
long overlapping matches, incompressible rows).  CPU tests pin the oracle
(oracle/png_oracle.py) to Pillow and check the host-side chunk parsing.
"""
import io
import os
import struct
import zlib

import numpy as np
import pytest
import torch
from PIL import Image

from oracle import png_oracle as PO

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FIXTURES = ["png_kitti_rgb.png", "png_kitti_depth16.png"]


def pillow_decode(data):
    im = Image.open(io.BytesIO(data))
    if im.mode in ("I;16", "I;16B", "I"):
        v = np.array(im, dtype=int)                      # read_png_depth
        return np.where(v == 0, -1.0, v / 256.0).astype(np.float32)
    return np.asarray(im.convert("RGB"))


def _chunk(typ, body):
    return struct.pack(">I", len(body)) + typ + body + struct.pack(">I", zlib.crc32(typ + body) & 0xFFFFFFFF)


def encode_png(px, depth, ctype, filters, compressor, idat_split=0):
    """A PNG of px ([h, w, bpp-bytes] uint8, big-endian words for 16-bit) with
    the given per-row filter types and a zlib compressor (compressobj)."""
    h, w = px.shape[:2]
    rowb = px.reshape(h, -1).astype(np.int32)
    bpp = {(8, 0): 1, (8, 2): 3, (8, 6): 4, (16, 0): 2}[(depth, ctype)]
    raw = bytearray()
    prev = np.zeros(rowb.shape[1], dtype=np.int32)
    for r in range(h):
        ft = filters[r % len(filters)]
        x = rowb[r]
        a = np.concatenate([np.zeros(bpp, np.int32), x[:-bpp]])
        c = np.concatenate([np.zeros(bpp, np.int32), prev[:-bpp]])
        pred = {0: 0 * x, 1: a, 2: prev, 3: (a + prev) >> 1, 4: PO._paeth(a, prev, c)}[ft]
        raw.append(ft)
        raw += ((x - pred) & 255).astype(np.uint8).tobytes()
        prev = x
    z = compressor.compress(bytes(raw)) + compressor.flush()
    parts = [z] if not idat_split else [z[i:i + idat_split] for i in range(0, len(z), idat_split)]
    out = b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, depth, ctype, 0, 0, 0))
    for p in parts:
        out += _chunk(b"IDAT", p)
    return out + _chunk(b"IEND", b"")


def _image(h, w, bpp, seed, kind="mixed"):
    rng = np.random.default_rng(seed)
    if kind == "random":
        return rng.integers(0, 256, size=(h, w, bpp), dtype=np.uint8)
    y, x = np.mgrid[0:h, 0:w]
    base = np.stack([(x * (3 + c) + y * (5 - c) + (x * y) // 7) % 256 for c in range(bpp)], -1)
    base[h // 3: h // 2] = 77                                          # long runs: overlapping matches
    base[:, : max(1, w // 9)] = rng.integers(0, 256, size=(h, max(1, w // 9), bpp))
    return base.astype(np.uint8)


COMPRESSORS = {
    "stored": lambda: zlib.compressobj(0),
    "fixed": lambda: zlib.compressobj(6, zlib.DEFLATED, 15, 9, zlib.Z_FIXED),
    "rle": lambda: zlib.compressobj(6, zlib.DEFLATED, 15, 9, zlib.Z_RLE),
    "dynamic": lambda: zlib.compressobj(9),
    "fast": lambda: zlib.compressobj(1),
}
CASES = [  # (h, w, depth, ctype, filters, compressor, image kind)
    (37, 53, 8, 2, [0, 1, 2, 3, 4], "dynamic", "mixed"),
    (130, 97, 8, 2, [3, 4, 1, 2, 0], "fixed", "mixed"),
    (70, 1242, 8, 2, [4, 3], "rle", "mixed"),
    (65, 33, 8, 6, [1, 3, 4], "dynamic", "mixed"),
    (64, 64, 8, 0, [2, 4, 3, 1], "fast", "mixed"),
    (129, 211, 16, 0, [4, 1, 3, 2], "dynamic", "mixed"),
    (9, 1, 8, 2, [0, 1, 2, 3, 4], "dynamic", "mixed"),
    (33, 41, 8, 2, [4], "stored", "random"),
    (200, 300, 8, 2, [1, 4], "dynamic", "random"),
]


def _case_png(i):
    h, w, depth, ctype, filters, comp, kind = CASES[i]
    bpp = {(8, 0): 1, (8, 2): 3, (8, 6): 4, (16, 0): 2}[(depth, ctype)]
    return encode_png(_image(h, w, bpp, 10 + i, kind), depth, ctype, filters, COMPRESSORS[comp](),
                      idat_split=1000 if i % 2 else 0)


# ------------------------------------------------------------------ CPU: oracle and host parsing
@pytest.mark.parametrize("name", FIXTURES)
def test_oracle_matches_pillow_on_fixtures(name):
    data = open(os.path.join(G, name), "rb").read()
    assert np.array_equal(PO.decode(data), pillow_decode(data))


@pytest.mark.parametrize("i", range(len(CASES)))
def test_oracle_matches_pillow_generated(i):
    data = _case_png(i)
    assert np.array_equal(PO.decode(data), pillow_decode(data))


def test_parse_png_host_side():
    from dro_sfm_amd.datasets.png import parse_png
    data = open(os.path.join(G, FIXTURES[0]), "rb").read()
    info = parse_png(data)
    assert info.key == (375, 1242, 2)
    assert zlib.decompress(info.idat)[:1] in (b"\x00", b"\x01", b"\x02", b"\x03", b"\x04")
    assert parse_png(_case_png(1)).key == (130, 97, 2)          # several IDAT chunks, concatenated
    pal = io.BytesIO()
    Image.fromarray(np.zeros((4, 4, 3), np.uint8)).convert("P").save(pal, format="PNG")
    with pytest.raises(NotImplementedError):
        parse_png(pal.getvalue())
    inter = b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", struct.pack(">IIBBBBB", 8, 8, 8, 2, 0, 0, 1)) + \
        _chunk(b"IDAT", zlib.compress(b"\x00" * 8)) + _chunk(b"IEND", b"")   # Adam7 interlaced
    with pytest.raises(NotImplementedError):
        parse_png(inter)
    bad = bytearray(data[:200])
    bad[40] ^= 0xFF
    with pytest.raises(ValueError):
        parse_png(bytes(bad))


# ------------------------------------------------------------------ GPU: bit-exact to Pillow
@pytest.fixture(scope="module")
def png():
    from dro_sfm_amd.datasets import png as P
    from dro_sfm_amd.hip import _lib
    _lib.load()
    return P


@pytest.mark.gpu
@pytest.mark.parametrize("name", FIXTURES)
def test_gpu_decode_fixture(png, name):
    """The committed KITTI-size frame (375 x 1242 RGB) and 16-bit depth map."""
    data = open(os.path.join(G, name), "rb").read()
    got = png.decode_png_batch([data, data], "cuda").cpu().numpy()
    ref = pillow_decode(data)
    assert got.dtype == ref.dtype and got.shape[1:] == ref.shape
    for k in range(2):
        assert np.array_equal(got[k], ref)


@pytest.mark.gpu
def test_gpu_decode_generated(png):
    """Every row filter, stored / fixed / dynamic blocks, RLE matches, split
    IDATs, grey / RGB / RGBA / 16-bit grey, widths 1 .. 1242, heights across
    the 64-row bands; several geometries in one call (decode_pngs groups)."""
    blobs = [_case_png(i) for i in range(len(CASES))]
    got = png.decode_pngs(blobs, "cuda")
    for i, (b, g) in enumerate(zip(blobs, got)):
        assert np.array_equal(g.cpu().numpy(), pillow_decode(b)), CASES[i]


@pytest.mark.gpu
def test_gpu_decode_batch_of_distinct_frames(png):
    """Six different frames of one geometry in one launch pair (a training
    step's target + context frames): each equals its own Pillow decode."""
    blobs = []
    for s in range(6):
        buf = io.BytesIO()
        Image.fromarray(_image(96, 320, 3, 40 + s)).save(buf, format="PNG", compress_level=1 + s)
        blobs.append(buf.getvalue())
    got = png.decode_png_batch(blobs, "cuda").cpu().numpy()
    for k, b in enumerate(blobs):
        assert np.array_equal(got[k], pillow_decode(b))


@pytest.mark.gpu
def test_gpu_decode_rejects_corrupt_stream(png):
    data = _case_png(0)
    info = png.parse_png(data)
    z = bytearray(info.idat)
    z[0] = 0x79                                         # bad zlib header (CM != 8)
    bad = png.PngInfo(info.width, info.height, info.kind, bytes(z))
    with pytest.raises(RuntimeError, match="zlib header"):
        png.decode_png_batch([bad], "cuda")
    trunc = png.PngInfo(info.width, info.height, info.kind, info.idat[: len(info.idat) // 2])
    with pytest.raises(RuntimeError):
        png.decode_png_batch([trunc], "cuda")
    out, status = png.decode_png_batch([info, bad], "cuda", check_status=False)
    assert status.cpu().tolist()[0] == 0 and status.cpu().tolist()[1] != 0
