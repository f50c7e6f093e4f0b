#!/bin/bash
# Row f3 measurement: tools/dataset_bench.py (k_dataset_extract, 2048 x 60-ply 15x15 records,
# 8-fold augmentation, shuffled slots), the same under rocprofv3 kernel trace, and the HBM PMC
# passes (FETCH_SIZE, WRITE_SIZE in separate runs).  Output: gpurun_out/ds/
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ds
mkdir -p $O
timeout -k 10 200 python3 tools/dataset_bench.py > $O/dataset.json 2> $O/dataset.err || { echo FAIL bench; tail -5 $O/dataset.err; exit 1; }
cat $O/dataset.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/dataset_bench.py > $O/trace.log 2>&1 || { echo FAIL trace; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 tools/dataset_bench.py > $O/fetch.log 2>&1 || { echo FAIL fetch; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 tools/dataset_bench.py > $O/write.log 2>&1 || { echo FAIL write; exit 1; }
python3 - <<'PY'
import collections, csv, glob, json
def per(sub, name):
    vals = collections.defaultdict(float); n = set()
    for f in glob.glob(f"gpurun_out/ds/{sub}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_dataset_extract" in r["Kernel_Name"]:
                vals[r["Dispatch_Id"]] += float(r["Counter_Value"])
    return sum(vals.values()) / max(1, len(vals)), len(vals)
fs, nf = per("fetch", "FETCH_SIZE"); ws, nw = per("write", "WRITE_SIZE")
st = [r for f in glob.glob("gpurun_out/ds/trace/**/*kernel_stats.csv", recursive=True) for r in csv.DictReader(open(f))
      if "k_dataset_extract" in r["Name"]]
out = {"kernel": "k_dataset_extract", "dispatches": nf, "avg_duration_ns": float(st[0]["AverageNs"]) if st else None,
       "hbm_read_bytes_per_launch": fs * 1024 * 2, "hbm_write_bytes_per_launch": ws * 1024,
       "note": "FETCH_SIZE x2 (gfx950 correction) and WRITE_SIZE are KiB per dispatch, averaged"}
json.dump(out, open("gpurun_out/ds/dataset_pmc.json", "w"), indent=1)
print(json.dumps(out))
PY
