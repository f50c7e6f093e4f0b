# conv3x3_v8 vs v7 (AZ_CONV_FLAGS 516 = default, 131588 = v7 forced) on the C3 trunk: kernel trace,
# one SQ busy/wait pass and one LDS pass per flag set.  Output: gpurun_out/v8pmc_<flags>/
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for F in ${FLAGS:-516 131588}; do
  OUT=gpurun_out/v8pmc_$F
  mkdir -p $OUT
  AZ_CONV_FLAGS=$F timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 tools/net_bench.py --batch 2048 --iters 5 > $OUT/trace.log 2>&1 || exit 1
  AZ_CONV_FLAGS=$F timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq -o run -- python3 tools/net_bench.py --batch 2048 --iters 3 > $OUT/sq.log 2>&1 || exit 1
  AZ_CONV_FLAGS=$F timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $OUT/lds -o run -- python3 tools/net_bench.py --batch 2048 --iters 3 > $OUT/lds.log 2>&1 || exit 1
  python3 - $OUT <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
for f in glob.glob(d + "/trace/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "conv3x3" in r["Name"] and float(r["Calls"]) > 20:
            print(r["Name"][:60], "avg us", float(r["AverageNs"]) / 1e3, "calls", r["Calls"])
for sub in ("sq", "lds"):
    vals = collections.defaultdict(list)
    for f in glob.glob(d + "/" + sub + "/**/*counter_collection.csv", recursive=True):
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(f)):
            if "conv3x3" in r["Kernel_Name"]:
                per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        big = [k for k in per if per[k].get("GRBM_GUI_ACTIVE", 0) > 4e6]
        for k in big:
            for c, v in per[k].items():
                vals[c].append(v)
    avg = {c: sum(v) / len(v) for c, v in vals.items()}
    for c in sorted(avg):
        print(f"  {sub} {c} {avg[c]:.5g} (n={len(vals[c])})")
    g = avg.get("GRBM_GUI_ACTIVE", 0) / 8
    if g and "SQ_VALU_MFMA_BUSY_CYCLES" in avg:
        print("  mfma busy frac", avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (g * 1024), "gui cycles/XCD", g)
PY
done
