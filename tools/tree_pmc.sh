# rocprofv3 HBM traffic of the tree kernels (k_select, k_expand_backup, k_scan, k_gather_planes) over
# one C3-shaped move (2048 games, 64 sims: an 800-sim move under --pmc crashed the profiler on the host): kernel trace, then FETCH_SIZE and WRITE_SIZE in separate passes.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/tree
mkdir -p $O
CMD="python3 bench.py --cpu-baseline 0 --steps 1 --warmup 0 --sims ${SIMS:-64}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $CMD > $O/trace.log 2>&1 || { echo FAIL trace; tail -3 $O/trace.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $CMD > $O/fetch.log 2>&1 || { echo FAIL fetch; tail -3 $O/fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $CMD > $O/write.log 2>&1 || { echo FAIL write; tail -3 $O/write.log; exit 1; }
python3 - <<'PY'
import collections, csv, glob, json
K = ["k_select", "k_expand_backup", "k_scan", "k_gather_planes"]
def per(sub):
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(f"gpurun_out/tree/{sub}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            for k in K:
                if r["Kernel_Name"].startswith(k + "("):
                    vals[k][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {k: (sum(v.values()) / len(v), len(v)) for k, v in vals.items()}
fe, wr = per("fetch"), per("write")
dur = {}
for f in glob.glob("gpurun_out/tree/trace/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        for k in K:
            if r["Name"].startswith(k + "("):
                dur[k] = float(r["AverageNs"])
out = {"workload": "python3 bench.py --cpu-baseline 0 --steps 1 --warmup 0 (C3 games and net, --sims 64: one move; the full 800-sim move crashed rocprofv3 counter collection on the host)",
       "note": "per dispatch: FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE (KiB), average duration from the kernel trace pass"}
for k in K:
    if k in fe and k in wr and k in dur:
        rd, w = fe[k][0] * 1024 * 2, wr[k][0] * 1024
        out[k] = {"dispatches": fe[k][1], "avg_duration_us": dur[k] / 1e3, "hbm_read_bytes": rd, "hbm_write_bytes": w,
                  "hbm_GB_per_s": (rd + w) / dur[k], "frac_of_hbm_peak": (rd + w) / dur[k] / 8000.0}
json.dump(out, open("gpurun_out/tree/tree_pmc.json", "w"), indent=1)
print(json.dumps(out, indent=1))
PY
