set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/smscan
for bl in 1 2 6 12; do
  timeout -k 10 120 python tools/net_bench.py --channels 64 --blocks $bl --batch 256 --iters 50 2>&1 | tail -1
done
for B in 64 512 1024; do
  timeout -k 10 120 python tools/net_bench.py --channels 64 --blocks 6 --batch $B --iters 50 2>&1 | tail -1
done
