"""Per-launch-configuration timing of selected kernels in the steady state of a
rocprofv3 kernel trace.  usage: prof_configs.py trace.csv [substr ...]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
keys = sys.argv[2:] or ["igemm", "wgrad"]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
marks = [int(r["Start_Timestamp"]) for r in rows if "photo_fwd_kernel" in r["Kernel_Name"]]
t0, t1 = marks[-5], marks[-1]
c = collections.defaultdict(list)
for r in rows:
    s = int(r["Start_Timestamp"])
    if t0 <= s < t1 and any(k in r["Kernel_Name"] for k in keys):
        k = (r["Kernel_Name"].split("(")[0].replace("void dro::", "")[:48], int(r["Grid_Size_X"]) // 256,
             int(r["Grid_Size_Y"]))
        c[k].append((int(r["End_Timestamp"]) - s) / 1000)
for k, v in sorted(c.items(), key=lambda kv: -sum(kv[1]))[:40]:
    print(f"{sum(v) / 4:8.0f} us/step {len(v) / 4:5.1f}/step avg {sum(v) / len(v):6.1f} us  {k}")
