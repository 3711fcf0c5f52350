"""GPU inflate time by DEFLATE content (tools/bench_png.py's frame re-encoded):
stored blocks, literals only (Huffman only), RLE matches, fixed codes, zlib
levels 1 / 6 / 9 -- which part of the stream the per-image time goes to.
usage: python tools/bench_png_modes.py"""
import os
import sys
import zlib

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    from dro_sfm_amd.datasets import png as P
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden", "png_kitti_rgb.png")
    info = P.parse_png(open(path, "rb").read())
    raw = zlib.decompress(info.idat)
    modes = {"stored": zlib.compressobj(0), "huffman-only": zlib.compressobj(6, zlib.DEFLATED, 15, 9, zlib.Z_HUFFMAN_ONLY),
             "rle": zlib.compressobj(6, zlib.DEFLATED, 15, 9, zlib.Z_RLE),
             "fixed": zlib.compressobj(6, zlib.DEFLATED, 15, 9, zlib.Z_FIXED),
             "level1": zlib.compressobj(1), "level6": zlib.compressobj(6), "level9": zlib.compressobj(9)}
    for name, c in modes.items():
        z = c.compress(raw) + c.flush()
        inf = P.PngInfo(info.width, info.height, info.kind, z)
        out = P.decode_png_batch([inf], "cuda")
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        P.decode_png_batch([inf], "cuda", check_status=False)
        e1.record()
        torch.cuda.synchronize()
        print(f"{name:13s} {len(z) / 1e3:8.0f} KB compressed  {e0.elapsed_time(e1):8.2f} ms per frame", flush=True)


if __name__ == "__main__":
    main()
