"""HBM traffic per launch of the bench roofline kernel from two rocprofv3 PMC
passes (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950):

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d OUT/pmc_fetch -o run -- python bench.py --roofline-only
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d OUT/pmc_write -o run -- python bench.py --roofline-only
    python tools/pmc_traffic.py OUT [dest.json]

Both counters are kilobytes (counter_defs.yaml).  Per MI355X_MICROARCH.md §HBM,
FETCH_SIZE reads 1/2 of the bytes of wide streaming reads on gfx950, so it is
doubled; WRITE_SIZE is taken as is.  The conv kernel's loads are 4 B/lane
(uncalibrated width per the guide): treat the absolute as approximate."""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

KERNELS = tuple(bench.roofline_kernels()[0])


def per_launch(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    vals = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            for k in KERNELS:
                if k in r["Kernel_Name"] and r["Counter_Name"] == counter:
                    key = (f, r.get("Dispatch_Id") or r.get("Correlation_Id"))
                    vals.setdefault(k, {})
                    vals[k][key] = vals[k].get(key, 0.0) + float(r["Counter_Value"])
    if len(vals) != len(KERNELS):
        raise SystemExit(f"no {counter} rows for {KERNELS} under {d}")
    # per call = sum over the kernels of their per-launch means
    means = {k: sum(v.values()) / len(v) for k, v in vals.items()}
    return sum(means.values()), {k: len(v) for k, v in vals.items()}, means


def main():
    out = sys.argv[1]
    dest = sys.argv[2] if len(sys.argv) > 2 else os.path.join(out, "roofline_traffic.json")
    fkb, nf, fmed = per_launch(os.path.join(out, "pmc_fetch"), "FETCH_SIZE")
    wkb, nw, wmed = per_launch(os.path.join(out, "pmc_write"), "WRITE_SIZE")
    res = {"kernels": list(KERNELS), "fetch_size_kb_per_launch": fkb, "write_size_kb_per_launch": wkb,
           "fetch_bytes_corrected": 2 * fkb * 1024, "write_bytes": wkb * 1024,
           "hbm_bytes_per_launch": int(2 * fkb * 1024 + wkb * 1024), "launches": [nf, nw],
           "unit": "per call (every kernel the call launches)",
           "per_kernel_kb": [fmed, wmed],
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over "
                     "`bench.py --roofline-only`; FETCH_SIZE x2 (gfx950 correction)"}
    with open(dest, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
