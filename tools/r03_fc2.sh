# k_fc_heads with every K chunk of a slice loaded up front (build) vs the committed kernel
# (build_ab): C2 net outputs bitwise, then the C2 bench under rocprofv3 --kernel-trace --stats.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03fc2
mkdir -p $O
for lib in build_ab build; do
  AZ_HIP_LIB=$PWD/alphazero-multi-game_amd/$lib/libaz_hip.so timeout -k 10 120 python3 - $O/$lib.npz <<'PY' || exit 1
import sys, numpy as np
sys.path.insert(0, "alphazero-multi-game_amd")
import az_amd
eng = az_amd.Engine(0)
out = {}
for B in (256, 37):
    net = az_amd.HipNeuralNetwork(eng, az_amd.NetDesc(15, 11, 64, 6, 225, 32, 8, 256, 1, 0, az_amd.AZ_PREC_FP16, 256))
    net.init_random(7)
    x = (np.random.default_rng(B).random((B, 11, 15, 15)) < 0.2).astype(np.float32)
    l, v = net.forward(x)
    out[f"l{B}"], out[f"v{B}"] = l, v
    net.close()
np.savez(sys.argv[1], **out)
print("saved", sys.argv[1])
PY
done
python3 - $O <<'PY' || exit 1
import sys, numpy as np
a, b = np.load(sys.argv[1] + "/build_ab.npz"), np.load(sys.argv[1] + "/build.npz")
for k in a.files:
    print(k, "bitwise equal" if np.array_equal(a[k], b[k]) else f"DIFF max {np.abs(a[k]-b[k]).max()}")
    assert np.array_equal(a[k], b[k])
PY
for lib in build_ab build; do
  AZ_HIP_LIB=$PWD/alphazero-multi-game_amd/$lib/libaz_hip.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$lib -o run -- python3 bench.py --config c2 --steps 2 --warmup 1 > $O/bench_$lib.json 2> $O/bench_$lib.err || { tail -5 $O/bench_$lib.err; exit 1; }
  python3 - $O/prof_$lib <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if float(r["Calls"]) > 100:
            print(f'{r["Name"][:60]:60s} {r["Calls"]:>6s} {float(r["AverageNs"])/1e3:8.2f} us')
PY
  tail -1 $O/bench_$lib.json | cut -c1-200
done
