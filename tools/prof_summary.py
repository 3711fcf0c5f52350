"""Per-step kernel breakdown of a rocprofv3 kernel trace (steady state only).

Steps are delimited by consecutive launches of a marker kernel that runs once
per training step (default: photo_fwd_kernel); the last --steps intervals are
averaged, so MIOpen's find/tuning launches during warmup are excluded.
usage: python tools/prof_summary.py run_kernel_trace.csv [--steps 5] [--top 40]
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--marker", default="photo_fwd_kernel")
    args = ap.parse_args()
    rows = list(csv.DictReader(open(args.trace)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
    marks = [s for s, _, n in ks if args.marker in n]
    if len(marks) < args.steps + 1:
        raise SystemExit(f"only {len(marks)} marker launches")
    t0, t1 = marks[-args.steps - 1], marks[-1]
    per = collections.defaultdict(lambda: [0, 0])
    busy = 0
    for s, e, n in ks:
        if t0 <= s < t1:
            per[n][0] += e - s
            per[n][1] += 1
            busy += e - s
    S = args.steps
    wall = (t1 - t0) / S / 1e6
    print(f"steady state: {S} steps, wall {wall:.3f} ms/step, kernel busy {busy / S / 1e6:.3f} ms/step, "
          f"{sum(c for _, c in per.values()) / S:.0f} launches/step")
    groups = collections.defaultdict(float)
    for n, (d, c) in per.items():
        key = ("dro::" + n.split("dro::")[1].split("(")[0].split("<")[0]) if "dro::" in n else \
              "miopen/ck/blas" if any(t in n for t in ("miopen", "Cijk", "ck::", "igemm", "naive_conv", "Im2d", "Col2Im",
                                                       "batched_transpose", "SubTensor", "_ZN2ck")) else \
              "aten " + n.split("at::native::")[1].split("<")[0].split("(")[0] if "at::native::" in n else n[:40]
        groups[key] += d
    print("-- groups (ms/step)")
    for k, d in sorted(groups.items(), key=lambda kv: -kv[1])[:25]:
        print(f"{d / S / 1e6:8.3f}  {k}")
    print("-- kernels (ms/step, launches/step, us/launch)")
    for n, (d, c) in sorted(per.items(), key=lambda kv: -kv[1][0])[:args.top]:
        print(f"{d / S / 1e6:8.3f} {c / S:6.0f} {d / c / 1e3:8.1f}  {n[:120]}")


if __name__ == "__main__":
    main()
