"""One GPU inflate of the literal-only (Z_HUFFMAN_ONLY) re-encoding of the
KITTI fixture, for rocprofv3 --pmc counter passes (tools/bench_png_modes.py:
the literal path dominates the per-image time)."""
import os
import sys
import zlib

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from dro_sfm_amd.datasets import png as P  # noqa: E402

path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden", "png_kitti_rgb.png")
info = P.parse_png(open(path, "rb").read())
raw = zlib.decompress(info.idat)
c = zlib.compressobj(6, zlib.DEFLATED, 15, 9, zlib.Z_HUFFMAN_ONLY)
z = c.compress(raw) + c.flush()
out = P.decode_png_batch([P.PngInfo(info.width, info.height, info.kind, z)], "cuda")
torch.cuda.synchronize()
print("literals", len(raw), "compressed", len(z))
