"""Cost of cross-stream edges inside a captured hipGraph: two chains of K
kernels (each a 128 x 128 x D matmul accumulate, a small grid with work) on two
streams, with the chains made to wait for each other every M nodes
(s1.wait_stream(s2) and s2.wait_stream(s1): two edges), M = inf for none.
The step graph has two chains joined by many such edges (the pose block's
stream and the autograd backward's stream crossings).
usage: python tools/graph_sync_cost.py [K=256] [D=4096]
"""
import sys

import torch


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    D = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    dev = torch.device("cuda", 0)
    A = torch.randn(128, D, device=dev) * 1e-3
    Bm = torch.randn(D, 128, device=dev) * 1e-3
    x = torch.zeros(128, 128, device=dev)
    y = torch.zeros(128, 128, device=dev)
    x.addmm_(A, Bm)
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    for M in (0, 64, 16, 4, 1):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s1):
            s2.wait_stream(s1)
            for k in range(K // 2):
                x.addmm_(A, Bm)
                with torch.cuda.stream(s2):
                    y.addmm_(A, Bm)
                if M and (k + 1) % M == 0:
                    s1.wait_stream(s2)
                    s2.wait_stream(s1)
            s1.wait_stream(s2)
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        us = 1e3 * e0.elapsed_time(e1) / 10
        nsync = 0 if not M else (K // 2) // M
        print(f"K={K} D={D} sync every {M if M else 'never'}: {us:.1f} us per replay ({nsync} sync pairs), "
              f"{us / (K // 2):.2f} us per node along a chain", flush=True)
    # the same kernels on one stream (serial reference)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s1):
        for k in range(K):
            x.addmm_(A, Bm)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    us = 1e3 * e0.elapsed_time(e1) / 10
    print(f"K={K} D={D} one stream: {us:.1f} us per replay, {us / K:.2f} us per node", flush=True)


if __name__ == "__main__":
    main()
