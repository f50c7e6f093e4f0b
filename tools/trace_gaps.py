#!/usr/bin/env python3
"""Per-kernel averages and the idle time between consecutive kernels of a rocprofv3 kernel trace
(`--kernel-trace --output-format csv`): where a simulation step's wall time goes beyond the kernels.

usage: trace_gaps.py <rocprofv3 output dir>"""
import csv
import glob
import sys
from collections import defaultdict


def main(d):
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)
    rows = list(csv.DictReader(open(f[0])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = defaultdict(list)
    gap_before = defaultdict(list)
    prev = None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].split("(")[0][:48]
        dur[name].append((e - s) / 1e3)
        if prev is not None and s - prev < 50_000:          # gaps inside a move (host syncs excluded)
            gap_before[name].append((s - prev) / 1e3)
        prev = e
    print(f"{'kernel':48s} {'calls':>7s} {'avg us':>9s} {'gap before (avg us)':>20s}")
    for name, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        g = gap_before[name]
        print(f"{name:48s} {len(v):7d} {sum(v) / len(v):9.2f} {sum(g) / max(1, len(g)):20.2f}")
    span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e6
    busy = sum(sum(v) for v in dur.values()) / 1e3
    print(f"trace span {span:.1f} ms, kernels busy {busy:.1f} ms ({100 * busy / span:.1f}%)")


if __name__ == "__main__":
    main(sys.argv[1])
