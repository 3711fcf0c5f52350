"""Warp-cost backward on the cost calls of a real training state.

Trains the bench model (KITTI self-sup workload) eagerly for a few steps,
records the inputs of every warp_cost call of one more forward, and replays
each call's backward in isolation: per call, the bilinear-cell statistics of
its sampling (how strongly the warp compresses the reference: pixels per
occupied cell, distinct cells per 64-pixel wave) and the backward's time.  Run
under `rocprofv3 --kernel-trace` for per-kernel durations (each call: one
recording launch, then `iters` timed ones).

usage: python tools/warp_state_probe.py [train_steps] [iters]
"""
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT]
import torch  # noqa: E402

import bench  # noqa: E402
import dro_sfm_amd.hip as hip  # noqa: E402
from dro_sfm_amd.hip import ops  # noqa: E402


def cell_stats(cells):
    """cells int32 [N,B,h,w] packed ((y0+32768)<<16)|(x0+32768), -1 unrecorded."""
    N, B, h, w = cells.shape
    raw = cells.reshape(N * B, h * w)
    c = raw.long() & 0xFFFFFFFF
    x0 = (c & 0xFFFF) - 32768
    y0 = (c >> 16) - 32768
    inside = (raw != -1) & (x0 >= -1) & (x0 < w) & (y0 >= -1) & (y0 < h)
    key = torch.where(inside, (y0 + 1) * (w + 1) + x0 + 1, torch.full_like(c, -1))
    maxc, occ, runs = 0, 0, []
    for i in range(N * B):
        k = key[i][key[i] >= 0]
        if k.numel():
            _, cnt = torch.unique(k, return_counts=True)
            maxc = max(maxc, int(cnt.max()))
            occ += int(cnt.numel())
        kw = key[i][: (h * w) // 64 * 64].reshape(-1, 64)
        runs.append(torch.tensor([torch.unique(r[r >= 0]).numel() for r in kw]).float().mean())
    return dict(inside=float(inside.float().mean()), px_per_cell=float(inside.sum()) / max(occ, 1),
                max_per_cell=maxc, cells_per_wave=float(torch.stack(runs).mean()))


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from dro_sfm_amd.trainers.dp_trainer import DataParallelTrainer, init_distributed
    init_distributed()
    bench.set_workload("kitti_selfsup")
    torch.manual_seed(42)
    model = bench.build_model(dev, 0.0)
    model.seed(42)
    trainer = DataParallelTrainer(model, lr=2e-4, bucket_mb=25.0, capturable=False)
    batches = [bench.make_batch(bench.WL["batch"], i, dev) for i in range(4)]
    for i in range(steps):
        trainer.step(batches[i % 4])
    recs, orig = [], hip.warp_cost

    def recording(fmap, fmap_ref, depth, pose, K, ref_K=None, **kw):
        recs.append((fmap.detach().clone(), fmap_ref.detach().clone(), depth.detach().clone(),
                     pose.detach().clone(), K.clone(), kw))
        return orig(fmap, fmap_ref, depth, pose, K, ref_K, **kw)

    hip.warp_cost = recording
    model(batches[steps % 4])
    hip.warp_cost = orig
    torch.cuda.synchronize()
    print(f"{len(recs)} cost calls recorded after {steps} steps", flush=True)
    for i, (fmap, fref, depth, pose, K, kw) in enumerate(recs):
        kw = {k: v for k, v in kw.items() if k != "tag"}
        leaves = [t.requires_grad_(True) for t in (fmap, fref, depth, pose)]
        with ops.record_bilinear_cells() as rec:
            cost = orig(*leaves, K, **kw)
        G = torch.randn_like(cost)
        torch.autograd.grad(cost, leaves, G, retain_graph=True)
        st = cell_stats(rec.calls[0][1])
        cost = orig(*leaves, K, **kw)           # without the (mutated) cell map
        torch.autograd.grad(cost, leaves, G, retain_graph=True)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            torch.autograd.grad(cost, leaves, G, retain_graph=True)
        e1.record()
        torch.cuda.synchronize()
        print(f"call {i:2d} N={fref.shape[0]} mean={kw.get('reduce_mean')} "
              f"depth[{float(depth.detach().min()):.3g},{float(depth.detach().max()):.3g}] "
              f"inside={st['inside']:.2f} px/cell={st['px_per_cell']:.2f} max/cell={st['max_per_cell']} "
              f"cells/wave={st['cells_per_wave']:.1f} backward={1e3 * e0.elapsed_time(e1) / iters:.1f} us",
              flush=True)


if __name__ == "__main__":
    main()
