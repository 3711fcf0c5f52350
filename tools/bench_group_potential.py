"""What would one launch per conv shape over the depth (B=2) and pose (N*B=4)
update blocks buy?  For each pairable update-block conv a
hipGraph of R dependent repetitions of

  serial   the B=2 conv, then the B=4 conv, on one stream
  streams  the B=2 chain on one stream beside the B=4 chain on another (the
           step's structure today: depth block on S0, pose block on S1)
  merged   ONE conv over B=6 (the same work in one launch: the duration a
           grouped launch over both problems would approach)

forward and data gradient, timed per repetition with events around the
replays.  usage: python tools/bench_group_potential.py [R=64]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

H, W = 24, 80
# (name, sources' channels, Cout, kernel, act)
SHAPES = [("c1 1x1 128->64", [128], 64, (1, 1), "relu"),
          ("c2 3x3 64->64", [64], 64, (3, 3), "relu"),
          ("fuse 3x3 128->63", [64, 64], 63, (3, 3), "relu"),
          ("gates 1x5 160->128", [64, 32, 63, 1], 128, (1, 5), "sigmoid"),
          ("gates 5x1 160->128", [64, 32, 63, 1], 128, (5, 1), "sigmoid"),
          ("cand 1x5 160->64", [64, 32, 63, 1], 64, (1, 5), "tanh"),
          ("head 3x3 64->192", [64], 192, (3, 3), "relu")]


def main():
    import dro_sfm_amd.hip as hip
    from dro_sfm_amd.hip import _lib
    _lib.load()
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    dev = torch.device("cuda", 0)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    print(f"{'shape':22s} {'pass':5s} {'serial':>8s} {'streams':>8s} {'merged':>8s}  us per repetition")
    for name, cs, Cout, k, act in SHAPES:
        Cin = sum(cs)
        w = torch.randn(Cout, Cin, *k, device=dev) * 0.05
        b = torch.randn(Cout, device=dev) * 0.1
        xs = {B: [torch.randn(B, c, H, W, device=dev) for c in cs] for B in (2, 4, 6)}
        gy = {B: torch.randn(B, Cout, H, W, device=dev) for B in (2, 4, 6)}
        y = {B: hip.conv2d(xs[B], w, b, act=act) for B in (2, 4, 6)}
        gx = {B: [torch.empty_like(x) for x in xs[B]] for B in (2, 4, 6)}
        from dro_sfm_amd.hip.conv import ACT

        def fwd(B):
            return torch.ops.dro.conv2d(xs[B], w, b, ACT[act], 1.0, [], 0)

        def bwd(B):
            torch.ops.dro.conv2d_backward(xs[B], w, y[B], gy[B], ACT[act], 1.0, gx[B], [0] * len(cs), None, None,
                                          0, None)

        for pname, fn in (("fwd", fwd), ("dgrad", bwd)):
            res = {}
            for mode in ("serial", "streams", "merged"):
                fn(2), fn(4), fn(6)
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=s1):
                    if mode == "serial":
                        for _ in range(R):
                            fn(2)
                            fn(4)
                    elif mode == "merged":
                        for _ in range(R):
                            fn(6)
                    else:
                        s2.wait_stream(s1)
                        for _ in range(R):
                            fn(2)
                        with torch.cuda.stream(s2):
                            for _ in range(R):
                                fn(4)
                        s1.wait_stream(s2)
                for _ in range(3):
                    g.replay()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    g.replay()
                e1.record()
                torch.cuda.synchronize()
                res[mode] = e0.elapsed_time(e1) * 1000 / 5 / R
                del g
            print(f"{name:22s} {pname:5s} {res['serial']:8.1f} {res['streams']:8.1f} {res['merged']:8.1f}", flush=True)


if __name__ == "__main__":
    main()
