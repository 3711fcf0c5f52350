"""Probe for the RCCL watchdog abort during a step capture (VERDICT r5 weak 6,
next 3): `hipErrorCapturedEvent` in WorkNCCL::finishedGPUExecutionInternal,
thrown from the ProcessGroupNCCL watchdog thread while GraphedTrainStep was
capturing with collectives inside the graph.

Hypothesis under test: the watchdog still tracks the LAST EAGER collectives of
the warm-up steps when the capture begins (it retires completed works only on
its next poll, up to its sleep interval later).  Their end events were recorded
eagerly on RCCL's internal stream; the first captured collective pulls that
same stream into the capture, and the watchdog's next hipEventQuery of the old
eager event then fails with hipErrorCapturedEvent -- the query sees an event
whose recording stream is capturing.  Timing decides whether a poll lands in
that window: "about 1 run in 7".

Each mode runs in a child process (world-size-1 "nccl" group, watchdog errors
rethrown, i.e. torch's default):
  race   eager all_reduce, sync, capture at once: a captured all_reduce, then
         the host waits 1 s inside the capture (the watchdog polls the eager
         work while RCCL's stream is capturing)
  drain  the same after waiting for the watchdog to retire the eager work
         (dp_trainer.drain_watchdog) before the capture begins
  recycle / recycle_nocache  with torch's CUDA event cache on (off): a
         captured all_reduce whose work object is then released (its events
         go back to the cache), then eager all_reduces (which may take those
         events) polled by the watchdog for 1 s
usage: python tools/rccl_watchdog_probe.py [race drain ...]
One line per mode: its exit code (-6 = the watchdog's abort).
"""
import os
import subprocess
import sys
import time


def child(mode, port):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    x = torch.ones(1 << 20, device=dev)
    for _ in range(3):
        dist.all_reduce(x)                     # eager: tracked by the watchdog
    torch.cuda.synchronize()
    if mode.startswith("recycle"):
        import dro_sfm_amd.trainers.dp_trainer as T
        T.drain_watchdog()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            y = x * 2
            w = dist.all_reduce(y, async_op=True)
            w.wait()
        del w                                   # the captured work's events back to the cache
        torch.cuda.synchronize()
        for _ in range(8):
            dist.all_reduce(x)                  # eager works: recycled events?
        time.sleep(1.0)
        g.replay()
        torch.cuda.synchronize()
        print(f"[{mode}] survived: x[0] = {float(x[0])}", flush=True)
        del g
        dist.destroy_process_group()
        return
    if mode == "drain":
        import dro_sfm_amd.trainers.dp_trainer as T
        T.drain_watchdog()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        y = x * 2
        dist.all_reduce(y)                     # RCCL's stream joins the capture
        time.sleep(1.0)                        # several watchdog polls inside the capture
        y += 1
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    print(f"[{mode}] replayed: y[0] = {float(y[0])}", flush=True)
    del g
    dist.destroy_process_group()


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(sys.argv[2], int(sys.argv[3]))
        return
    modes = sys.argv[1:] or ["race", "drain", "recycle", "recycle_nocache", "race_fr", "recycle_fr"]
    for i, m in enumerate(modes):
        # *_fr: the flight recorder on (2000 entries), as torch's default was
        env = dict(os.environ, TORCH_NCCL_RETHROW_CUDA_ERRORS="1",
                   TORCH_NCCL_CUDA_EVENT_CACHE="1" if m in ("recycle", "recycle_fr") else "0",
                   TORCH_NCCL_TRACE_BUFFER_SIZE="2000" if m.endswith("_fr") else "0")
        name, m = m, (m[:-3] if m.endswith("_fr") else m)
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", m, str(29711 + i)], env=env,
                           stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=240)
        tail = [ln for ln in r.stdout.splitlines() if "replayed" in ln or "survived" in ln or "hipError" in ln
                or "terminate" in ln]
        print(f"mode {name}: exit {r.returncode}; " + " | ".join(tail[:3]), flush=True)


if __name__ == "__main__":
    main()
