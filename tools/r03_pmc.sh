#!/bin/bash
# Round 3 trunk PMC on the final tree: tools/pmc_conv.sh for the fp16 trunk (conv3x3_v7) and the
# fp32-faithful trunk (conv3x3_v7x3, bench.py's parity_mode), folded into profiles/r03l_*_trunk_pmc.json
# (bench.py reads the newest matching summary for roofline.traffic).
set -eo pipefail
bash tools/pmc_conv.sh fp16 r03l_fp16
python3 tools/pmc_summary.py gpurun_out/pmc_r03l_fp16 --kernel conv3x3_v7 --precision fp16 --out gpurun_out/r03l_fp16_v7_trunk_pmc.json > /dev/null
bash tools/pmc_conv.sh bf16x3 r03l_x3
python3 tools/pmc_summary.py gpurun_out/pmc_r03l_x3 --kernel conv3x3_v7x3 --precision bf16x3 --out gpurun_out/r03l_bf16x3_v7x3_trunk_pmc.json > /dev/null
python3 - <<'PY'
import json
for f in ("gpurun_out/r03l_fp16_v7_trunk_pmc.json", "gpurun_out/r03l_bf16x3_v7x3_trunk_pmc.json"):
    d = json.load(open(f))
    alg = sum(d["algorithmic_bytes_per_launch"].values())
    print(f, d["kernel"], f"{d['avg_duration_ns'] / 1e3:.1f} us", f"{d.get('clock_ghz_effective', 0):.2f} GHz",
          f"MFMA busy {d.get('mfma_busy_frac', 0):.3f}", f"HBM {d['hbm_bytes_per_launch'] / 1e6:.0f} MB vs {alg / 1e6:.0f} MB algorithmic")
PY
