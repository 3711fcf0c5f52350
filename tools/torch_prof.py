"""Attribute the small PyTorch kernels of one eager training step to ops/shapes
(torch.profiler on the GPU).  usage: python tools/torch_prof.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

import bench  # noqa: E402
from dro_sfm_amd.trainers.dp_trainer import DataParallelTrainer  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    model = bench.build_model(dev, 0.0)
    tr = DataParallelTrainer(model, lr=2e-4, bucket_mb=25.0, capturable=False)
    batch = bench.make_batch(2, 0, dev)
    for _ in range(3):
        batch["intrinsics"].copy_(batch["_K0"])
        tr.step(batch, flip=False)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True, with_stack=True) as prof:
        batch["intrinsics"].copy_(batch["_K0"])
        tr.step(batch, flip=False)
        torch.cuda.synchronize()
    rows = [e for e in prof.key_averages(group_by_input_shape=True) if e.key.startswith("aten::")]
    rows.sort(key=lambda e: -e.count)
    print(f"{'op':28s} {'calls':>6s} {'dev us':>9s}  shapes")
    for e in rows[:70]:
        print(f"{e.key[:28]:28s} {e.count:6d} {e.device_time_total:9.0f}  {str(e.input_shapes)[:150]}")
    st = [e for e in prof.key_averages(group_by_stack_n=6) if e.key in ("aten::add_", "aten::add", "aten::mul", "aten::zeros", "aten::fill_", "aten::copy_")]
    st.sort(key=lambda e: -e.count)
    for e in st[:25]:
        print(f"== {e.key} x{e.count} dev {e.device_time_total:.0f}us")
        for fr in (e.stack or [])[:6]:
            print("     ", fr[:150])
    fns = [e for e in prof.key_averages() if "Backward" in e.key or "evaluate_function" in e.key]
    fns.sort(key=lambda e: -e.count)
    for e in fns[:30]:
        print(f"{e.key[:70]:70s} {e.count:6d} {e.device_time_total:9.0f}")


if __name__ == "__main__":
    main()
