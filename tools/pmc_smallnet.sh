#!/bin/bash
# SQ counters of k_smallnet (C2 net, 256 boards): MFMA busy, LDS activity / bank conflicts / waits.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-pmc_sm}
mkdir -p $O
for w in ${WAVES:-8 4}; do
AZ_SM_WAVES=$w timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv -d $O/sq$w -o run -- python3 tools/net_bench.py --channels 64 --blocks 6 --batch 256 --iters 3 > $O/sq$w.log 2>&1 || { echo PMC_FAIL; tail -5 $O/sq$w.log; exit 1; }
O=$O W=$w python3 - <<'PY'
import collections, csv, glob, os
O, W = os.environ["O"], os.environ["W"]
vals = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(f"{O}/sq{W}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_smallnet" in r["Kernel_Name"]:
            vals[(f, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
n = len(vals)
avg = {k: sum(d[k] for d in vals.values()) / n for k in next(iter(vals.values()))}
print(f"== {W} waves, dispatches", n)
for k, v in sorted(avg.items()):
    print(f"{k:28s} {v:16.0f}")
g = avg["GRBM_GUI_ACTIVE"] / 8
print("MFMA busy frac (per SIMD, 256 CUs used)", avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (256 * 4) / g)
PY
done
