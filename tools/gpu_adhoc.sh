set -o pipefail
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/c2
mkdir -p $O
AZ_DIAG_HIP_LIB=$R/alphazero-multi-game_amd/build_old/libaz_hip.so timeout -k 10 150 python3 -u tools/upload_race.py 45 > $O/race_old.txt 2>&1 && tail -1 $O/race_old.txt &&
timeout -k 10 150 python3 -u tools/upload_race.py 45 > $O/race_new.txt 2>&1 && tail -1 $O/race_new.txt &&
TAG=c2/tree FILES="tests/test_gpu_search.py tests/test_gpu_go.py tests/test_gpu_host_api.py tests/test_gpu_api.py tests/test_gpu_callback_eval.py tests/test_gpu_selfplay_net.py" bash tools/gpu_tests.sh &&
timeout -k 10 200 python3 bench.py --config c2 --steps 4 --warmup 1 --cpu-baseline 0 --parity-steps 0 > $O/bench_c2.json 2> $O/bench_c2.err && cat $O/bench_c2.json | cut -c1-400 &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o run -- python3 $R/bench.py --steps 1 --warmup 1 --cpu-baseline 0 --parity-steps 0 > $O/bench_c3_prof.json 2>&1 && cut -c1-300 $O/bench_c3_prof.json | tail -2
