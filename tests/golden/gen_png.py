"""Writes the committed PNG fixtures of tests/test_png.py with Pillow (the
encoder the reference's datasets were written with): a KITTI-like RGB frame
(375 x 1242, the raw KITTI size; smooth gradients + texture + flat regions so
the encoder picks every row filter and both literal-heavy and match-heavy
Huffman blocks) and a KITTI-like 16-bit sparse depth map (mostly zeros,
values * 256 as in the KITTI depth benchmark).
usage: python tests/golden/gen_png.py   (writes tests/golden/png_*.png)"""
import os

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))


def kitti_like_rgb(h=375, w=1242, seed=0):
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w].astype(np.float64)
    img = np.stack([128 + 90 * np.sin(x / 37.0 + c) * np.cos(y / 23.0 - c) for c in range(3)], -1)
    img[h // 2:] += rng.normal(0, 12, size=(h - h // 2, w, 3))         # textured road
    img[: h // 6] = [200, 210, 230]                                     # flat sky
    img[:, w // 3: w // 3 + 40] = rng.integers(0, 256, size=(h, 40, 3))  # incompressible strip
    return np.clip(img, 0, 255).astype(np.uint8)


def kitti_like_depth(h=375, w=1242, seed=1):
    rng = np.random.default_rng(seed)
    d = np.zeros((h, w), dtype=np.uint16)
    rows = rng.random((h, w)) < 0.05
    rows[: h // 3] = False
    d[rows] = (rng.uniform(1.0, 80.0, size=int(rows.sum())) * 256).astype(np.uint16)
    return d


def main():
    Image.fromarray(kitti_like_rgb()).save(os.path.join(HERE, "png_kitti_rgb.png"))
    Image.fromarray(kitti_like_depth()).save(os.path.join(HERE, "png_kitti_depth16.png"))


if __name__ == "__main__":
    main()
