"""Warp-cost kernel timing on the inputs the training step actually produces.

Trains the bench model (KITTI 192x640 self-sup, B=2) for --steps eager steps,
records the arguments of every hip.warp_cost call of one more forward, then
times forward and backward of the recorded depth-cost and pose-cost calls
(hipGraph replay, device time per call) next to synthetic near-identity warps.
Also prints how concentrated the bilinear taps are (the atomic scatter's
worst-case contention: max taps landing on one source pixel).

usage: python tools/bench_warp.py [--steps N] [--iters N]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
import dro_sfm_amd.hip as hip  # noqa: E402
from dro_sfm_amd.hip import ops as hops  # noqa: E402


def graph_time(fn, iters):
    """Wall time per call (HIP events; includes launch overhead -- run under
    rocprofv3 --kernel-trace --stats for the kernels' own durations)."""
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def tap_histogram(depth, pose, K, h, w, scale):
    """max / mean number of bilinear taps per source pixel (CPU, per ref)."""
    from dro_sfm_amd.geometry.pose import euler2mat
    B = depth.shape[0]
    Ks = K.clone()
    Ks[:, 0, :] *= scale
    Ks[:, 1, :] *= scale
    Ks[:, 0, 2] = (K[:, 0, 2] + 0.5) * scale - 0.5
    Ks[:, 1, 2] = (K[:, 1, 2] + 0.5) * scale - 0.5
    ys, xs = torch.meshgrid(torch.arange(h, dtype=torch.float32), torch.arange(w, dtype=torch.float32),
                            indexing="ij")
    pix = torch.stack([xs, ys, torch.ones_like(xs)], 0).view(3, -1)
    out = []
    for n in range(pose.shape[0]):
        for b in range(B):
            X = torch.linalg.inv(Ks[b]) @ pix * depth[b].view(1, -1)
            R = euler2mat(pose[n, b, 3:].view(1, 3))[0]
            t = pose[n, b, :3].view(3, 1)
            x = Ks[b] @ (R @ X + t)
            u = (x[0] / x[2].clamp_min(1e-5)).round().long().clamp(0, w - 1)
            v = (x[1] / x[2].clamp_min(1e-5)).round().long().clamp(0, h - 1)
            cnt = torch.bincount(v * w + u, minlength=h * w).float()
            out.append((cnt.max().item(), (cnt[cnt > 0]).mean().item()))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=25)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--mode", choices=("real", "synth"), default="real")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    if args.mode == "synth":
        return synth(args, dev)
    torch.manual_seed(42)
    model = bench.build_model(dev, 0.0)
    model.seed(42)
    from dro_sfm_amd.trainers.dp_trainer import DataParallelTrainer
    trainer = DataParallelTrainer(model, lr=2e-4, bucket_mb=25.0, capturable=False)
    batch = bench.make_batch(2, 7, dev)
    for _ in range(args.steps):
        batch["intrinsics"].copy_(batch["_K0"])
        trainer.step(batch)
    torch.cuda.synchronize()
    calls = []
    orig = hops.warp_cost

    def rec(*a, **k):
        calls.append((a, k))
        return orig(*a, **k)
    hip.warp_cost = rec
    import dro_sfm_amd.networks.depth_pose.DepthPoseNet as dpn
    dpn.hip.warp_cost = rec
    batch["intrinsics"].copy_(batch["_K0"])
    with torch.no_grad():
        model(batch)
    hip.warp_cost = orig
    dpn.hip.warp_cost = orig
    print(f"{len(calls)} warp_cost calls per forward", flush=True)
    for idx in (0, len(calls) - 1):
        a, k = calls[idx]
        fmap, fref, depth, pose, K = [x.detach() if torch.is_tensor(x) else x for x in a[:5]]
        fmap = fmap.clone().requires_grad_()
        fref = fref.clone().requires_grad_()
        depth = depth.clone().requires_grad_()
        pose = pose.clone().requires_grad_()
        cost = orig(fmap, fref, depth, pose, K, *a[5:], **k)
        gc = torch.randn_like(cost)

        def fwd():
            with torch.no_grad():
                orig(fmap, fref, depth, pose, K, *a[5:], **k)

        def fb():
            fmap.grad = fref.grad = depth.grad = pose.grad = None
            c = orig(fmap, fref, depth, pose, K, *a[5:], **k)
            c.backward(gc)
        tf = graph_time(fwd, args.iters)
        tfb = graph_time(fb, args.iters)
        print(f"call {idx}: fmap {tuple(fmap.shape)} refs {tuple(fref.shape)} pose {tuple(pose.shape)} "
              f"kwargs {sorted(k)}: fwd {tf:.1f} us, bwd {tfb - tf:.1f} us", flush=True)
        print(f"   pose values: {pose.detach().flatten()[:12].tolist()}", flush=True)
        print(f"   depth range: {depth.min().item():.4g} .. {depth.max().item():.4g}", flush=True)


def synth(args, dev):
    """synthetic near-identity warps"""
    B, C, h, w, N = 2, 128, 24, 80, 2
    g = torch.Generator(device=dev).manual_seed(1)
    fmap = torch.randn(B, C, h, w, device=dev, generator=g).requires_grad_()
    fref = torch.randn(N, B, C, h, w, device=dev, generator=g).requires_grad_()
    depth = (5 + 10 * torch.rand(B, 1, h, w, device=dev, generator=g)).requires_grad_()
    pose = torch.cat([0.1 * torch.randn(N, B, 3, device=dev, generator=g),
                      0.01 * torch.randn(N, B, 3, device=dev, generator=g)], 2).requires_grad_()
    K = torch.tensor(bench.KITTI_K, device=dev).unsqueeze(0).repeat(B, 1, 1)
    gc = torch.randn(B, C, h, w, device=dev, generator=g)

    def fwd2():
        with torch.no_grad():
            hip.warp_cost(fmap, fref, depth, pose, K)

    def fb2():
        fmap.grad = fref.grad = depth.grad = pose.grad = None
        hip.warp_cost(fmap, fref, depth, pose, K).backward(gc)
    tf = graph_time(fwd2, args.iters)
    tfb = graph_time(fb2, args.iters)
    print(f"synthetic near-identity: fwd {tf:.1f} us, bwd {tfb - tf:.1f} us", flush=True)
    print(f"   taps per source pixel (max, mean): "
          f"{tap_histogram(depth.detach().cpu(), pose.detach().cpu(), K.cpu(), h, w, 1 / 8)}", flush=True)


if __name__ == "__main__":
    main()
