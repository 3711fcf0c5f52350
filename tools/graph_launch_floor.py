"""Per-node cost of a hipGraph replay on this box: a graph of K dependent
launches of a tiny kernel (one-element add, ATen) on one stream, and the same
K split over two streams (two independent chains), replayed and timed with
events.  The step graph is ~1130 kernel nodes on two streams: this is the
floor a node costs beyond its own work.
usage: python tools/graph_launch_floor.py [K=512] [elements=1]
(elements > 1: each node adds over that many floats, a kernel with real work)
"""
import sys

import torch


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    E = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    dev = torch.device("cuda", 0)
    x = torch.zeros(max(E, 1), device=dev)
    y = torch.zeros(max(E, 1), device=dev)
    # E < 0: each node a 128 x 128 x |E| matmul (a small grid with real work)
    if E < 0:
        A = torch.randn(128, -E, device=dev) * 1e-3
        Bm = torch.randn(-E, 128, device=dev) * 1e-3
        x = torch.zeros(128, 128, device=dev)
        y = torch.zeros(128, 128, device=dev)
    s1 = torch.cuda.Stream(dev)
    s2 = torch.cuda.Stream(dev)

    def chain(t, n):
        for _ in range(n):
            if E < 0:
                t.addmm_(A, Bm)
            else:
                t.add_(1.0)

    chain(x, 1)                       # library handles created outside any capture
    torch.cuda.synchronize()
    for name, two in (("one stream", False), ("two streams", True)):
        g = torch.cuda.CUDAGraph()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s1):
            if two:
                s2.wait_stream(s1)
                chain(x, K // 2)
                with torch.cuda.stream(s2):
                    chain(y, K // 2)
                s1.wait_stream(s2)
            else:
                chain(x, K)
        for _ in range(5):
            g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 20
        e0.record()
        for _ in range(reps):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        print(f"{name}: {K} nodes of {E} elements, {1e3 * ms:.1f} us per replay, {1e3 * ms / (K / (2 if two else 1)):.2f} us "
              f"per node along a chain", flush=True)

    # the two chains as two linear (single-stream) graphs, replayed on two
    # streams side by side
    ga, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    with torch.cuda.graph(ga, stream=s1):
        chain(x, K // 2)
    with torch.cuda.graph(gb, stream=s2):
        chain(y, K // 2)
    torch.cuda.synchronize()
    main = torch.cuda.current_stream(dev)

    def both():
        s1.wait_stream(main)
        s2.wait_stream(main)
        with torch.cuda.stream(s1):
            ga.replay()
        with torch.cuda.stream(s2):
            gb.replay()
        main.wait_stream(s1)
        main.wait_stream(s2)

    for _ in range(5):
        both()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        both()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    print(f"two linear graphs on two streams: {K} nodes of {E} elements, {1e3 * ms:.1f} us per replay, "
          f"{1e3 * ms / (K / 2):.2f} us per node along a chain", flush=True)


if __name__ == "__main__":
    main()
