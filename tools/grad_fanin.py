"""Where does autograd still sum gradients with ATen add kernels?  One eager
forward of the bench model, then a walk of the autograd graph from the loss:
every (node, output) consumed by more than one node gets its gradients summed
by the engine (one add per extra consumer).  Lists them by node type and
shape, most adds first.  usage: python tools/grad_fanin.py"""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    model = bench.build_model(dev, 0.0)
    batch = bench.make_batch(2, 0, dev)
    out = model(batch)
    loss = out["loss"].sum()
    uses = collections.Counter()
    names = {}
    seen, stack = set(), [loss.grad_fn]
    while stack:
        fn = stack.pop()
        if fn is None or fn in seen:
            continue
        seen.add(fn)
        for nxt, nr in fn.next_functions:
            if nxt is None:
                continue
            uses[(nxt, nr)] += 1
            names[(nxt, nr)] = nxt
            stack.append(nxt)
    agg = collections.Counter()
    for (fn, nr), n in uses.items():
        if n > 1 and type(fn).__name__ != "AccumulateGrad":
            meta = getattr(fn, "_input_metadata", None)
            shape = tuple(meta[nr].shape) if meta is not None and nr < len(meta) else None
            agg[(type(fn).__name__, nr, shape)] += n - 1
    acc = sum(n - 1 for (fn, nr), n in uses.items() if n > 1 and type(fn).__name__ == "AccumulateGrad")
    print(f"engine adds (non-leaf fan-in): {sum(agg.values())}; leaf (AccumulateGrad) fan-in extra: {acc}")
    for k, v in agg.most_common(40):
        print(f"  {v:4d}  {k}")


if __name__ == "__main__":
    main()
