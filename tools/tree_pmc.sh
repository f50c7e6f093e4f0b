# rocprofv3 HBM traffic of the tree kernels (k_select, k_expand_backup, k_scan) and the record ->
# g8 input kernel (k_rec_to_g8) over one full C3 move (2048 games, 800 sims): a kernel-trace pass,
# then FETCH_SIZE and WRITE_SIZE in separate passes.  The net is cut to 2 residual blocks (tree
# traffic does not depend on the trunk's depth): counters over the full 20-block run's 64k trunk
# dispatches crash rocprofv3 on the host, and so does --kernel-include-regex (SIGSEGV in the
# profiler's launch hook at the first conv dispatch).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-tree}
mkdir -p $O
CMD="python3 bench.py --cpu-baseline 0 --steps 1 --warmup 0 --sims ${SIMS:-800} --blocks ${BLOCKS:-2}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $CMD > $O/trace.log 2>&1 || { echo FAIL trace; tail -3 $O/trace.log; exit 1; }
( while sleep 30; do echo "pmc pass running ($(date +%T))"; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -s KILL ${PMC_TIMEOUT:-240} rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $CMD > $O/fetch.log 2>&1 || { echo FAIL fetch; tail -3 $O/fetch.log; exit 1; }
timeout -s KILL ${PMC_TIMEOUT:-240} rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $CMD > $O/write.log 2>&1 || { echo FAIL write; tail -3 $O/write.log; exit 1; }
kill $HB 2>/dev/null
O=$O SIMS=${SIMS:-800} BLOCKS=${BLOCKS:-2} python3 - <<'PY'
import collections, csv, glob, json, os, re
O = os.environ["O"]
K = ["k_select", "k_expand_backup", "k_scan", "k_rec_to_g8"]
def key(name):
    for k in K:
        if re.search(r"\b" + k + r"\b", name):
            return k
def per(sub):
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(f"{O}/{sub}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = key(r["Kernel_Name"])
            if k:
                vals[k][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {k: (sum(v.values()) / len(v), len(v)) for k, v in vals.items()}
fe, wr = per("fetch"), per("write")
dur = {}
for f in glob.glob(f"{O}/trace/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = key(r["Name"])
        if k:
            dur[k] = float(r["AverageNs"])
out = {"workload": f"python3 bench.py --cpu-baseline 0 --steps 1 --warmup 0 --sims {os.environ['SIMS']} --blocks {os.environ['BLOCKS']} (C3 games: 2048, 15x15, 256-filter fp16 net cut to {os.environ['BLOCKS']} blocks; one full move)",
       "note": "per dispatch: FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE (KiB -> bytes); average duration from the kernel-trace pass (all dispatches incl. the per-move root steps)"}
for k in K:
    if k in fe and k in wr and k in dur:
        rd, w = fe[k][0] * 1024 * 2, wr[k][0] * 1024
        out[k] = {"dispatches": fe[k][1], "avg_duration_us": dur[k] / 1e3, "hbm_read_bytes": rd, "hbm_write_bytes": w,
                  "hbm_GB_per_s": (rd + w) / dur[k], "frac_of_hbm_peak": (rd + w) / dur[k] / 8000.0}
json.dump(out, open(f"{O}/tree_pmc.json", "w"), indent=1)
print(json.dumps(out, indent=1))
PY
