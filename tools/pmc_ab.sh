#!/bin/bash
# SQ/GRBM PMC pass over the C3 trunk (tools/net_bench.py) for each conv flag set in FLAGS (decimal,
# AZ_CONV_FLAGS), plus a kernel-trace stats pass each.  Output: gpurun_out/pmcab_<flags>/
set -e
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for F in ${FLAGS:-516 772}; do
  OUT=gpurun_out/pmcab_$F
  mkdir -p $OUT
  AZ_CONV_FLAGS=$F timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 tools/net_bench.py --batch ${BATCH:-2048} --iters 5 > $OUT/trace.log 2>&1
  AZ_CONV_FLAGS=$F timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq -o run -- python3 tools/net_bench.py --batch ${BATCH:-2048} --iters 3 > $OUT/sq.log 2>&1
  python3 - $OUT <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
for f in glob.glob(d + "/trace/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "conv3x3" in r["Name"] and float(r["Calls"]) > 20:
            print(r["Name"][:60], "avg us", float(r["AverageNs"]) / 1e3, "calls", r["Calls"])
vals = collections.defaultdict(list)
for f in glob.glob(d + "/sq/**/*counter_collection.csv", recursive=True):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for r in csv.DictReader(open(f)):
        if "conv3x3" in r["Kernel_Name"]:
            per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = r["Kernel_Name"]
    big = [k for k in per if per[k].get("SQ_INSTS_MFMA", 0) > 1e6]
    for k in big:
        for c, v in per[k].items():
            vals[c].append(v)
avg = {c: sum(v) / len(v) for c, v in vals.items()}
for c in sorted(avg):
    print(f"  {c} {avg[c]:.4g}")
g = avg.get("GRBM_GUI_ACTIVE", 0) / 8
if g:
    print("  mfma busy frac", avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (g * 1024), "gui cycles/XCD", g)
PY
done
