"""Per-kernel roofline table of the conv engine over one training step
(VERDICT round 2, item 7).

  run:     rocprofv3 --kernel-trace --stats -d OUT -o run -- python tools/conv_roofline.py run OUT
           (optionally again under --pmc FETCH_SIZE / WRITE_SIZE / SQ_VALU_MFMA_BUSY_CYCLES)
  table:   python tools/conv_roofline.py table OUT [--pmc-dirs D1 D2 ...]

`run` builds the bench workload (KITTI it8, B=2, flip off), runs W eager
steps, then ONE eager step with the library's launch log on (dro_conv_log:
kernel instantiation -> launches, algorithmic FLOPs 2*Cout*Cin*KH*KW*B*H*W per
use), then K eager steps, and writes OUT/conv_log.json.  Every step launches the
same kernels with the same shapes, so rocprof's per-kernel totals / (W+1+K)
are per-step times.  `table` joins them: per instantiation launches/step,
GFLOP/step, us/launch, TFLOP/s, fraction of the 157.3 TF/s f32 MFMA peak,
and -- from the PMC passes -- HBM bytes per launch (FETCH_SIZE x 2 per the
gfx950 note, WRITE_SIZE) and MFMA busy fraction.
"""
import csv
import ctypes
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PEAK = 157.3   # TF/s, f32 MFMA dense (MI355X_MICROARCH.md)
W_STEPS, K_STEPS = 3, 5


def run(out):
    import torch
    import bench
    from dro_sfm_amd.hip import _lib
    from dro_sfm_amd.trainers.dp_trainer import DataParallelTrainer
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(42)
    model = bench.build_model(dev, 0.0)
    tr = DataParallelTrainer(model, lr=2e-4, bucket_mb=25.0)
    batch = bench.make_batch(2, 7, dev)

    def step():
        batch["intrinsics"].copy_(batch["_K0"])
        tr.step(batch, flip=False)

    for _ in range(W_STEPS):
        step()
    torch.cuda.synchronize()
    lib.dro_conv_log(1)
    step()
    torch.cuda.synchronize()
    lib.dro_conv_log(0)
    n = lib.dro_conv_log_read(None, 0)
    buf = ctypes.create_string_buffer(int(n) + 1)
    lib.dro_conv_log_read(buf, n + 1)
    for _ in range(K_STEPS):
        step()
    torch.cuda.synchronize()
    rows = {}
    for line in buf.value.decode().splitlines():
        name, launches, flops = line.split("\t")
        rows[name] = {"launches": int(launches), "flops": float(flops)}
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, "conv_log.json"), "w") as f:
        json.dump({"steps_total": W_STEPS + 1 + K_STEPS, "kernels": rows}, f, indent=1)
    print(f"logged {len(rows)} conv kernel instantiations")


def _find(pattern):
    hits = glob.glob(pattern, recursive=True)
    return hits[0] if hits else None


def _match(kname, name):
    return name in kname.replace("dro::", "") and (name.endswith("(") or f"{name}(" in kname.replace("dro::", ""))


def table(out, pmc_dirs):
    log = json.load(open(os.path.join(out, "conv_log.json")))
    steps = log["steps_total"]
    stats = _find(os.path.join(out, "**", "*kernel_stats.csv"))
    times = {}
    with open(stats) as f:
        for r in csv.DictReader(f):
            times[r["Name"]] = (int(r["Calls"]), float(r["TotalDurationNs"]))
    pmc = {}
    for d in pmc_dirs:
        cc = _find(os.path.join(d, "**", "*counter_collection.csv"))
        if not cc:
            continue
        with open(cc) as f:
            for r in csv.DictReader(f):
                key = (r["Kernel_Name"], r["Counter_Name"])
                v = pmc.setdefault(key, [0.0, 0])
                v[0] += float(r["Counter_Value"])
                v[1] += 1
    lines, total_ms, total_gf = [], 0.0, 0.0
    for name, e in sorted(log["kernels"].items(), key=lambda kv: -kv[1]["flops"]):
        hit = [(k, v) for k, v in times.items() if _match(k, name)]
        if not hit:
            continue
        kname, (calls, ns) = hit[0]
        per_step_ms = ns / steps / 1e6
        per_launch_us = ns / calls / 1e3
        per_step_calls = calls / steps
        tfs = e["flops"] / (per_step_ms * 1e-3) / 1e12
        row = {"kernel": name, "launches_per_step": round(per_step_calls, 2),
               "logged_launches": e["launches"], "gflop_per_step": round(e["flops"] / 1e9, 3),
               "gflop_per_launch": round(e["flops"] / e["launches"] / 1e9, 4),
               "us_per_launch": round(per_launch_us, 2), "ms_per_step": round(per_step_ms, 4),
               "tflops": round(tfs, 2), "frac_f32_mfma_peak": round(tfs / PEAK, 4)}
        for cname, label, scale in (("FETCH_SIZE", "fetch_bytes_per_launch", 2 * 1024.0),
                                    ("WRITE_SIZE", "write_bytes_per_launch", 1024.0),
                                    ("SQ_VALU_MFMA_BUSY_CYCLES", "mfma_busy_cycles_per_launch", 1.0),
                                    ("GRBM_GUI_ACTIVE", "gui_active_cycles_per_launch", 1.0)):
            v = pmc.get((kname, cname))
            if v:
                row[label] = round(v[0] / v[1] * scale, 1)
        if "mfma_busy_cycles_per_launch" in row and "gui_active_cycles_per_launch" in row:
            # busy cycles are summed over the 256 CUs x 4 SIMDs; GRBM_GUI_ACTIVE is
            # the sum over the 8 XCDs (MI355X_MICROARCH.md, DVFS note): /8 = kernel cycles
            row["mfma_busy_frac"] = round(row["mfma_busy_cycles_per_launch"] /
                                          (row["gui_active_cycles_per_launch"] / 8 * 256 * 4), 4)
        lines.append(row)
        total_ms += per_step_ms
        total_gf += e["flops"] / 1e9
    summary = {"steps_profiled": steps, "conv_ms_per_step": round(total_ms, 3),
               "conv_gflop_per_step": round(total_gf, 2),
               "conv_tflops": round(total_gf / total_ms, 2) if total_ms else None}
    json.dump({"summary": summary, "kernels": lines}, open(os.path.join(out, "conv_roofline.json"), "w"),
              indent=1)
    print(json.dumps(summary))
    hdr = f"{'kernel':45s} {'L/step':>6s} {'GF/step':>8s} {'us/L':>7s} {'ms/step':>7s} {'TF/s':>6s} {'frac':>6s}"
    print(hdr)
    for r in lines:
        print(f"{r['kernel']:45s} {r['launches_per_step']:6.1f} {r['gflop_per_step']:8.2f} "
              f"{r['us_per_launch']:7.1f} {r['ms_per_step']:7.3f} {r['tflops']:6.1f} {r['frac_f32_mfma_peak']:6.3f}"
              + (f"  fetch {r['fetch_bytes_per_launch'] / 1e6:.2f}MB" if "fetch_bytes_per_launch" in r else "")
              + (f" write {r['write_bytes_per_launch'] / 1e6:.2f}MB" if "write_bytes_per_launch" in r else "")
              + (f" mfma {r['mfma_busy_frac']:.3f}" if "mfma_busy_frac" in r else ""))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2])
    else:
        dirs = sys.argv[sys.argv.index("--pmc-dirs") + 1:] if "--pmc-dirs" in sys.argv else []
        table(sys.argv[2], dirs)
