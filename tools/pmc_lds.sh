#!/bin/bash
# One SQ counter pass on the C3 trunk: LDS bank conflicts / activity, waits, MFMA busy.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmc_lds
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv -d $O/sq -o run -- python3 tools/net_bench.py --iters 2 > $O/sq.log 2>&1 || { echo PMC_FAIL; tail -5 $O/sq.log; exit 1; }
python3 - <<'PY'
import collections, csv, glob
vals = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob("gpurun_out/pmc_lds/sq/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "conv3x3_v6" in r["Kernel_Name"]:
            vals[(f, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
n = len(vals)
avg = {k: sum(d[k] for d in vals.values()) / n for k in next(iter(vals.values()))}
print("dispatches", n)
for k, v in sorted(avg.items()):
    print(f"{k:28s} {v:16.0f}")
PY
