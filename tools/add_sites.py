"""Which autograd nodes launch the step's accumulation adds?  One eager
training step of the bench workload under a TorchDispatchMode that records
every aten add / add_ issued during backward with the autograd node running.
usage: python tools/add_sites.py"""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

CNT = collections.Counter()


class Rec(TorchDispatchMode):
    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = str(func.overloadpacket.__name__)
        if name in ("add", "add_", "mul", "copy_", "sum", "mean", "cat", "fill_", "div"):
            node = torch._C._current_autograd_node()
            shp = tuple(args[0].shape) if args and torch.is_tensor(args[0]) else ()
            CNT[(name, type(node).__name__ if node is not None else "-", shp)] += 1
        return func(*args, **(kwargs or {}))


def main():
    import bench
    from dro_sfm_amd.trainers.dp_trainer import DataParallelTrainer
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(42)
    model = bench.build_model(dev, 0.0)
    tr = DataParallelTrainer(model, lr=2e-4, bucket_mb=25.0)
    batch = bench.make_batch(2, 7, dev)
    for _ in range(2):
        batch["intrinsics"].copy_(batch["_K0"])
        tr.step(batch, flip=False)
    torch.cuda.synchronize()
    batch["intrinsics"].copy_(batch["_K0"])
    with Rec():
        tr.step(batch, flip=False)
    torch.cuda.synchronize()
    for (name, node, shp), v in CNT.most_common(60):
        print(f"{v:4d}  {name:6s} {node:40s} {shp}")


if __name__ == "__main__":
    main()
