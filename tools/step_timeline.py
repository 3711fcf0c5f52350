"""In-graph timeline of the KITTI metric training step.

Builds bench.py's model and trainer, captures the step into a hipGraph with
the timeline active (hip/timeline.py: stamps on the stream that reaches each
point, captured like any launch), replays it, and prints every stamp of the
last replay with its stream and time, plus the phase durations.  No profiler
is attached, so the streams overlap as they do in bench.py.
usage: python tools/step_timeline.py [--replays 20] [--batch 2]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from dro_sfm_amd.hip.timeline import Timeline  # noqa: E402
from dro_sfm_amd.trainers.dp_trainer import DataParallelTrainer, GraphedTrainStep  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--replays", type=int, default=20)
    ap.add_argument("--batch", type=int, default=2)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(42)
    model = bench.build_model(dev, 0.0)
    trainer = DataParallelTrainer(model, lr=2e-4, bucket_mb=25.0, capturable=True)
    batch = bench.make_batch(args.batch, 0, dev)
    with Timeline(dev) as tl:
        gs = GraphedTrainStep(trainer, batch, warmup=3, flips=(False,))
    first = max(i for i, (n, _) in enumerate(tl.names) if n == "step:begin")   # the captured step
    for _ in range(args.replays):
        gs.step(batch, flip=False)
    torch.cuda.synchronize()
    ev = tl.read(first)
    streams = {}
    for _, s, _ in ev:
        streams.setdefault(s, f"S{len(streams)}")
    print(f"in-graph timeline of one replayed step (last of {args.replays}); wall clock "
          f"{tl.hz / 1e6:.0f} MHz; streams: " + ", ".join(f"{v}=id {k}" for k, v in streams.items()))
    by_name = {}
    for n, s, t in sorted(ev, key=lambda e: e[2]):
        by_name[n] = t
        print(f"  {t:9.1f} us  {streams[s]:3s} {n}")
    total = by_name["step:end"] - by_name["step:begin"]

    def span(a, b):
        return by_name[b] - by_name[a] if a in by_name and b in by_name else float("nan")
    iters = sorted({int(n[len("fwd:depth_iter"):]) for n in by_name if n.startswith("fwd:depth_iter")})
    last = iters[-1] if iters else None
    print("phases (us):")
    rows = [("encoders + initial heads (fwd)", "step:begin", "fwd:init_heads"),
            ("update blocks (fwd, to the last depth iteration)", "fwd:init_heads", f"fwd:depth_iter{last}"),
            ("update blocks (fwd, to the last pose iteration)", "fwd:init_heads", f"fwd:pose_iter{last}"),
            ("upsample + loss (fwd)", f"fwd:depth_iter{last}", "fwd:loss"),
            ("loss backward", "bwd:begin", "bwd:loss_done"),
            ("update blocks (bwd, depth chain)", "bwd:loss_done", "bwd:depth_iter0"),
            ("update blocks (bwd, pose chain)", "bwd:loss_done", "bwd:pose_iter0"),
            ("to the initial depth head's backward", "bwd:begin", "bwd:init_depth_head"),
            ("cnet_depth backward begins", "bwd:begin", "bwd:cnet_depth_begin"),
            ("cnet_pose backward begins", "bwd:begin", "bwd:cnet_pose_begin"),
            ("fnet backward begins", "bwd:begin", "bwd:fnet_begin"),
            ("encoders (bwd) to the end of backward", "bwd:fnet_begin", "bwd:end"),
            ("all-reduce (world 1: none) + Adam", "bwd:end", "step:end")]
    for label, a, b in rows:
        print(f"  {span(a, b):9.1f}  {label}  [{a} -> {b}]")
    print(f"  {total:9.1f}  whole step (step:begin -> step:end)")


if __name__ == "__main__":
    main()
