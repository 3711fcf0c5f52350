"""Encoder (ResNet-18 trunk, fnet shape: 6 x 3 x 192 x 640) forward + backward
with NCHW against channels_last (NHWC) activations, PyTorch batch norm in both
(the fused HIP BN is NCHW only), to see what MIOpen's NHWC kernels are worth
without the NCHW<->NHWC transposes it wraps around its weight-gradient kernels.

usage: python tools/bench_encoder_layout.py [--iters N]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from dro_sfm_amd.networks.optim import extractor  # noqa: E402


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    for fused in (True, False):
        extractor.set_fused_batchnorm(fused)
        for cl in (False, True):
            if fused and cl:
                continue
            enc = extractor.ResNetEncoder(out_chs=128, stride=8).to(dev).train()
            x = torch.rand(6, 3, 192, 640, device=dev)
            if cl:
                enc = enc.to(memory_format=torch.channels_last)
                x = x.contiguous(memory_format=torch.channels_last)

            def step():
                enc.zero_grad(set_to_none=True)
                y = enc(x)
                y.float().square().mean().backward()
            ms = timeit(step, args.iters)
            print(f"BN {'fused hip' if fused else 'pytorch  '} layout {'NHWC' if cl else 'NCHW'}: "
                  f"{ms:.3f} ms fwd+bwd", flush=True)


if __name__ == "__main__":
    main()
