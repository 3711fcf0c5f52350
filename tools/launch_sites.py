"""Where do the step's non-engine launches come from?  One eager training step
of the bench workload under torch.profiler: every ATen op that launched a GPU
kernel, grouped by op and by its innermost Python frames in this repository.

usage: python tools/launch_sites.py [--top 40]
"""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--top", type=int, default=40)
    args = ap.parse_args()
    import bench
    from dro_sfm_amd.trainers.dp_trainer import DataParallelTrainer
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(42)
    model = bench.build_model(dev, 0.0)
    tr = DataParallelTrainer(model, lr=2e-4, bucket_mb=25.0)
    batch = bench.make_batch(2, 7, dev)

    def step():
        batch["intrinsics"].copy_(batch["_K0"])
        tr.step(batch, flip=False)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        step()
        torch.cuda.synchronize()
    sites = collections.Counter()
    ops = collections.Counter()
    for ev in prof.events():
        if ev.device_type != torch.autograd.DeviceType.CPU or not ev.name.startswith("aten::"):
            continue
        nk = sum(1 for k in ev.kernels) if hasattr(ev, "kernels") else 0
        if nk == 0:
            continue
        frames = [f for f in (ev.stack or []) if ROOT in f or "dro_sfm_amd" in f or "dro-sfm_amd" in f]
        site = " <- ".join(f.replace(ROOT + "/", "")[:90] for f in frames[:2]) or "(autograd engine / no repo frame)"
        sites[(ev.name, site)] += nk
        ops[ev.name] += nk
    print("== kernels launched by ATen ops, per op")
    for k, v in ops.most_common(args.top):
        print(f"{v:5d}  {k}")
    print("== per (op, call site)")
    for (name, site), v in sites.most_common(args.top):
        print(f"{v:5d}  {name:32s} {site}")


if __name__ == "__main__":
    main()
