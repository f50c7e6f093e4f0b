# Round-1 (re-entry) measurement: C3 bench under rocprofv3 kernel trace, C4 Go bench, g8 net
# benches (flattened tiles), and the dataset extraction kernel (trace + HBM PMC passes).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r01b
mkdir -p $O
step() { echo "== $1"; }
step c3-rocprof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --cpu-baseline 0 --steps 1 --warmup 1 > $O/bench_under_rocprof.json 2> $O/rocprof.err || { echo FAIL c3-rocprof; tail -5 $O/rocprof.err; exit 1; }
cat $O/bench_under_rocprof.json
step net-go19
timeout -k 10 200 python3 tools/net_bench.py --game go19 --batch 1024 --iters 5 > $O/net_go19.txt 2>&1 || { echo FAIL net-go19; tail -5 $O/net_go19.txt; exit 1; }
tail -2 $O/net_go19.txt
step net-chess
timeout -k 10 200 python3 tools/net_bench.py --game chess --batch 1024 --iters 5 > $O/net_chess.txt 2>&1 || { echo FAIL net-chess; tail -5 $O/net_chess.txt; exit 1; }
tail -2 $O/net_chess.txt
step go-c4
timeout -k 10 500 python3 bench.py --game go --steps 1 --warmup 1 > $O/bench_go.json 2> $O/bench_go.err || { echo FAIL go-c4; tail -5 $O/bench_go.err; exit 1; }
cat $O/bench_go.json
step dataset
timeout -k 10 200 python3 tools/dataset_bench.py > $O/dataset.json 2> $O/dataset.err || { echo FAIL dataset; tail -5 $O/dataset.err; exit 1; }
cat $O/dataset.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ds_trace -o run -- python3 tools/dataset_bench.py > $O/ds_trace.log 2>&1 || { echo FAIL ds-trace; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/ds_fetch -o run -- python3 tools/dataset_bench.py > $O/ds_fetch.log 2>&1 || { echo FAIL ds-fetch; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/ds_write -o run -- python3 tools/dataset_bench.py > $O/ds_write.log 2>&1 || { echo FAIL ds-write; exit 1; }
echo all-done
