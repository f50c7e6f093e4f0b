# A/B of conv3x3_v4<0,64> with one board per block (build) vs two (build_ab): bitwise outputs, forward timing
# of the C2 net in bf16x3, and the GPU tests that run that kernel.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03l_v4b1
mkdir -p $O
for lib in build_ab build; do
  AZ_HIP_LIB=$PWD/alphazero-multi-game_amd/$lib/libaz_hip.so timeout -k 10 120 python3 tools/r03_v4b1_check.py --out $O/$lib.npz || { echo CHECK_FAIL $lib; exit 1; }
done
python3 -c "
import numpy as np
a=np.load('$O/build_ab.npz'); b=np.load('$O/build.npz')
print('bitwise equal:', all(np.array_equal(a[k], b[k]) for k in a.files), {k: float(np.abs(a[k]-b[k]).max()) for k in a.files})"
ROUNDS=3 ABTAG=r03l_v4b1_ab NBARGS="--channels 64 --blocks 6 --batch 256 --iters 30 --precision bf16x3" bash tools/r03_smab.sh || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_trained_scale.py tests/test_gpu_net.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
