#!/bin/bash
# rocprofv3 HBM traffic of the tree kernels (k_select, k_expand_backup, the fused k_expand_select,
# k_scan) and the record -> g8 input kernel (k_rec_to_g8) over one full C3 move (2048 games, 800
# sims, BLOCKS residual blocks, default 20 = the bench config): a kernel-trace pass (bench.py's own
# kernel timing on, so its JSON line carries the kernels' algorithmic bytes), then FETCH_SIZE and
# WRITE_SIZE in separate passes.  Rounds 2-3 had to pass --kernel-timing 0 there: a search that
# recorded HIP events hung under counter collection (tools/pmc_hang_probe2.sh); since round 4 the
# timing uses device clock-stamp kernels instead of events (engine.hip ProfClock), and KT (default 1)
# keeps the bench's timing on in the counter passes too.
# --kernel-include-regex is not used (round 2: SIGSEGV in the profiler's launch hook).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-tree}
mkdir -p $O
# CONFIG=c2: BASELINE configs[1] as the bench runs it (256 games, 400 sims, the 6x64 net: every
# kernel at its own bench config); default c3 with BLOCKS (default 20, the bench's net)
# SYNC (default 10): a host sync every SYNC simulation steps.  rocprofv3 --pmc stalls (round 4) or
# crashes in its own thread (SIGSEGV at a page-aligned address, rounds 3-5) when a selfplay move
# queues thousands of dispatches without a host synchronisation: BLOCKS=2 passes at SYNC=100 (~600
# queued dispatches), BLOCKS=20 crashes at SYNC=100 (~4,300: 41 per simulation step) with the 560-byte
# TreeDev kernargs (r04) and with the round-5 8-byte device-resident TreeDev alike -- so not the
# kernarg size -- and passes at SYNC=10 (~430; profiles/r05_tree_pmc_c3.json).  The counter passes
# run with --crash-report: a crash leaves $O/crash_<pass>.txt (thread name, PC, /proc/self/maps)
if [ "${CONFIG:-c3}" = c2 ]; then
  CMD="python3 bench.py --config c2 --cpu-baseline 0 --parity-steps 0 --steps 1 --warmup 0 --sync-every ${SYNC:-10}"
else
  CMD="python3 bench.py --cpu-baseline 0 --parity-steps 0 --steps 1 --warmup 0 --sims ${SIMS:-800} --blocks ${BLOCKS:-20} --sync-every ${SYNC:-10}"
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $CMD > $O/trace.log 2>&1 || { echo FAIL trace; tail -3 $O/trace.log; exit 1; }
( while sleep 30; do echo "pmc pass running ($(date +%T))"; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -s KILL ${PMC_TIMEOUT:-240} rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $CMD --kernel-timing ${KT:-1} --crash-report $O/crash_fetch.txt > $O/fetch.log 2>&1 || { echo FAIL fetch; tail -3 $O/fetch.log; exit 1; }
timeout -s KILL ${PMC_TIMEOUT:-240} rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $CMD --kernel-timing ${KT:-1} --crash-report $O/crash_write.txt > $O/write.log 2>&1 || { echo FAIL write; tail -3 $O/write.log; exit 1; }
kill $HB 2>/dev/null
O=$O SIMS=${SIMS:-800} BLOCKS=${BLOCKS:-20} CONFIG=${CONFIG:-c3} python3 - <<'PY'
import collections, csv, glob, json, os, re
O = os.environ["O"]
K = ["k_select", "k_expand_backup", "k_expand_select", "k_scan", "k_rec_to_g8"]
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
wl = ("bench.py --config c2 (C2: 256 games, 400 sims, 6x64 fp16 net; one full move)" if os.environ["CONFIG"] == "c2" else
      f"bench.py --sims {os.environ['SIMS']} --blocks {os.environ['BLOCKS']} (C3 games: 2048, 15x15, 256-filter fp16 net with {os.environ['BLOCKS']} blocks; one full move)")
out = {"workload": wl,
       "note": "per dispatch: FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE (KiB -> bytes), counter passes with the bench kernel timing as KT (1: clock-stamp kernels on); average duration from the kernel-trace pass (all dispatches incl. the per-move root steps); algorithmic bytes: the bench line of the trace pass (kernel-counted, sampled steps)"}
bl = [l for l in open(f"{O}/trace.log") if l.startswith('{"metric"')]
if bl:
    tk = json.loads(bl[-1]).get("tree_kernels", {})
    alg = {k: tk[k]["bytes_per_launch"] for k in ("k_select", "k_expand_backup") if k in tk}
    if len(alg) == 2:
        alg["k_expand_select"] = alg["k_select"] + alg["k_expand_backup"]
    out["algorithmic_bytes_per_launch"] = alg
for k in K:
    if k in fe and k in wr and k in dur:
        rd, w = fe[k][0] * 1024 * 2, wr[k][0] * 1024
        out[k] = {"dispatches": fe[k][1], "avg_duration_us": dur[k] / 1e3, "hbm_read_bytes": rd, "hbm_write_bytes": w,
                  "hbm_GB_per_s": (rd + w) / dur[k], "frac_of_hbm_peak": (rd + w) / dur[k] / 8000.0}
        a = out.get("algorithmic_bytes_per_launch", {}).get(k)
        if a:
            out[k]["traffic_over_algorithmic"] = (rd + w) / a
json.dump(out, open(f"{O}/tree_pmc.json", "w"), indent=1)
print(json.dumps(out, indent=1))
PY
