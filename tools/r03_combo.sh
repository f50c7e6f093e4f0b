set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/combo
timeout -k 10 200 python -u -m pytest tests/test_gpu_host_api.py -q -k "keep_the_tree or rng" --timeout 120 --timeout-method thread > gpurun_out/combo/host.log 2>&1; tail -2 gpurun_out/combo/host.log
bash tools/pmc_smallnet.sh > gpurun_out/combo/pmcsm.txt 2>&1; cat gpurun_out/combo/pmcsm.txt
for w in 4 8; do echo "== $w waves"; AZ_SM_WAVES=$w AZ_HIP_LIB=$PWD/alphazero-multi-game_amd/build_smdiag/libaz_hip.so timeout -k 10 60 python3 tools/sm_stamps.py 256 | sed -n "1,4p;13,17p"; done
TAG=combo/pmclim bash tools/pmc_limit.sh
