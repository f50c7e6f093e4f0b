#!/usr/bin/env python3
"""Bitwise A/B of two library builds on the C2 net in bf16x3 (conv3x3_v4<0,64>: two boards per block
vs one): forward of the same planes / weights, outputs saved to --out (run once per AZ_HIP_LIB)."""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "alphazero-multi-game_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)
import az_amd  # noqa: E402
import net_oracle  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--out", required=True)
ap.add_argument("--batch", type=int, default=256)
a = ap.parse_args()
eng = az_amd.Engine(0)
outs = {}
for B in (a.batch, 37, 1):
    desc = az_amd.NetDesc(15, 11, 64, 6, 225, 32, 8, 256, 1, 0, az_amd.AZ_PREC_BF16X3, a.batch)
    rng = np.random.default_rng(B)
    x = (rng.random((B, 11, 15, 15)) < 0.3).astype(np.float32)
    net = az_amd.HipNeuralNetwork(eng, desc)
    net.load_weights(net_oracle.init_blob(desc, 99))
    lo, v = net.forward(x)
    outs[f"l{B}"], outs[f"v{B}"] = lo, v
    if B == 37:
        rl, rv = net_oracle.forward(desc, net_oracle.init_blob(desc, 99), x[:4])
        print(f"B={B}: max|dlogit| vs fp32 oracle {np.abs(lo[:4] - rl).max():.3e}, max|dvalue| {np.abs(v[:4] - rv).max():.3e}")
    net.close()
np.savez(a.out, **outs)
print("saved", a.out)
