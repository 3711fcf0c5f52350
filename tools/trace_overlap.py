"""Busy/overlap/idle breakdown of a rocprofv3 kernel trace (steady-state tail).
usage: python tools/trace_overlap.py <run_kernel_trace.csv> [tail_fraction]"""
import csv
import sys
from collections import Counter


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    frac = float(sys.argv[2]) if len(sys.argv) > 2 else 0.3
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"]) for r in rows)
    ev = ev[int(len(ev) * (1 - frac)):]
    tot = sum(e - s for s, e, _ in ev)
    union, cs, ce = 0, None, None
    for s, e, _ in ev:
        if ce is None or s > ce:
            if ce is not None:
                union += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    union += ce - cs
    span = ev[-1][1] - ev[0][0]
    print(f"{len(ev)} kernels: sum {tot / 1e6:.2f} ms, busy(union) {union / 1e6:.2f} ms, "
          f"span {span / 1e6:.2f} ms, idle {(span - union) / 1e6:.2f} ms, queues {dict(Counter(q for *_, q in ev))}")


if __name__ == "__main__":
    main()
