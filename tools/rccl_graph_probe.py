"""Minimal RCCL-in-hipGraph probes (the step's capture with
bucketed all-reduces inside crashed at capture_end).  One world-size-1 "nccl"
(RCCL) group per process, no model; each mode isolates one ingredient of the
trainer's in-graph exchange:

  plain      eager warm-up all_reduce, then capture one all_reduce on the
             capture stream; replay twice
  async      the same with async_op=True and work.wait() inside the capture
  side       the collective issued from a second stream forked from and joined
             back into the capture stream (the trainer's comm stream)
  lazy       NO eager collective before the capture (communicator created
             inside the capture)

usage: python tools/rccl_graph_probe.py MODE [--port P]
Prints one line per stage (stderr, unbuffered) so a crash names its stage.
"""
import faulthandler
import os
import sys

import torch
import torch.distributed as dist


def stage(msg):
    print(f"[rccl-probe {MODE}] {msg}", file=sys.stderr, flush=True)


MODE = sys.argv[1] if len(sys.argv) > 1 else "plain"


def main():
    faulthandler.enable()
    port = sys.argv[sys.argv.index("--port") + 1] if "--port" in sys.argv else "29611"
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    stage(f"group up (torch {torch.__version__}, nccl {torch.cuda.nccl.version()})")
    x = torch.ones(1 << 20, device=dev)
    if MODE != "lazy":
        dist.all_reduce(x)
        torch.cuda.synchronize()
        stage("eager all_reduce ok")
    side = torch.cuda.Stream(device=dev)
    g = torch.cuda.CUDAGraph()
    stage("capture begin")
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        x.mul_(2.0)
        if MODE in ("plain", "lazy"):
            dist.all_reduce(x)
        elif MODE == "async":
            w = dist.all_reduce(x, async_op=True)
            w.wait()
        elif MODE == "side":
            cur = torch.cuda.current_stream()
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                w = dist.all_reduce(x, async_op=True)
            w.wait()
            cur.wait_stream(side)
        x.add_(1.0)
    stage("capture end ok")
    x.fill_(1.0)
    g.replay()
    g.replay()
    torch.cuda.synchronize()
    stage(f"replay ok: x[0] = {float(x[0])} (expect 7.0)")
    assert float(x[0]) == 7.0
    del g
    torch.cuda.synchronize()
    dist.destroy_process_group()
    stage("done")


if __name__ == "__main__":
    main()
