"""GPU PNG decode (csrc/png.hip) vs Pillow on the host: the committed
KITTI-size frame (375 x 1242 RGB, tests/golden/png_kitti_rgb.png) decoded N
at a time (one workgroup per image), per-kernel times from HIP events, and
Pillow's decode of the same file on one host thread.
usage: python tools/bench_png.py [N ...]   (default 6 48 256)"""
import io
import os
import sys
import time

import numpy as np
import torch
from PIL import Image

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    from dro_sfm_amd.datasets import png as P
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden", "png_kitti_rgb.png")
    data = open(path, "rb").read()
    info = P.parse_png(data)
    ns = [int(a) for a in sys.argv[1:]] or [6, 48, 256]
    t0 = time.perf_counter()
    for _ in range(5):
        ref = np.asarray(Image.open(io.BytesIO(data)).convert("RGB"))
    cpu_ms = (time.perf_counter() - t0) / 5 * 1e3
    print(f"Pillow decode, one host thread: {cpu_ms:.2f} ms per frame ({len(data) / 1e3:.0f} KB PNG, "
          f"{ref.nbytes / 1e6:.2f} MB RGB)", flush=True)
    for n in ns:
        out = P.decode_png_batch([info] * n, "cuda")
        torch.cuda.synchronize()
        assert all(np.array_equal(out[k].cpu().numpy(), ref) for k in (0, n - 1))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 3
        e0.record()
        for _ in range(reps):
            P.decode_png_batch([info] * n, "cuda", check_status=False)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        print(f"GPU decode of {n} frames: {ms:.2f} ms per call (incl. H2D of the streams) = "
              f"{n / ms * 1e3:.0f} frames/s; Pillow on one thread {1e3 / cpu_ms:.0f} frames/s", flush=True)


if __name__ == "__main__":
    main()
