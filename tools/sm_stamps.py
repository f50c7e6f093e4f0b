#!/usr/bin/env python3
"""Phase stamps of k_smallnet's block 0 (AZ_SM_STAMPS=1): prologue, each layer, pool, head convs (us)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-multi-game_amd"))
import az_amd  # noqa: E402
from az_amd import _lib  # noqa: E402

B, blocks = int(sys.argv[1]) if len(sys.argv) > 1 else 256, 6
if os.environ.get("AZ_SM_WAVES"):      # measurement-only kernel variant (diag entry point)
    from az_amd import _lib as _l
    _l.lib().az_diag_set_smallnet_waves(int(os.environ["AZ_SM_WAVES"]))
if os.environ.get("AZ_CONV_FLAGS"):
    from az_amd import _lib as _l
    _l.lib().az_diag_set_conv_flags(int(os.environ["AZ_CONV_FLAGS"], 0))
_lib.lib().az_diag_set_smallnet_stamps(int(os.environ.get("AZ_SM_STAMPS", "1")))
if os.environ.get("AZ_SM_KERNEL"):
    _lib.lib().az_diag_set_smallnet_kernel(int(os.environ["AZ_SM_KERNEL"]))
eng = az_amd.Engine(0)
net = az_amd.HipNeuralNetwork(eng, az_amd.NetDesc(15, 11, 64, blocks, 225, 32, 8, 256, 1, 0, az_amd.AZ_PREC_FP16, B))
net.init_random(1)
x = (np.random.default_rng(0).random((B, 11, 15, 15)) < 0.2).astype(np.float32)
for _ in range(5):
    net.forward(x)
buf = (ctypes.c_ulonglong * 128)()
_lib.lib().az_diag_smallnet_stamps(buf, 128)
st = list(buf)
t0 = st[0]
names = {1: "prologue"} | {2 + i: f"layer {i}" for i in range(2 * blocks + 1)} | {40: "stream->LDS, wt", 41: "pool", 42: "head convs"}
if os.environ.get("SM_TAIL"):    # the tail: ring drain, barrier, stream / weight staging, pool, head MFMAs
    names = {2 * blocks + 2: f"layer {2 * blocks}", 54: "ring drained", 55: "barrier", 56: "stream + wt to LDS",
             40: "barrier", 57: "pool", 41: "barrier", 58: "head MFMAs", 42: "head stores"}
if os.environ.get("SM_INNER"):   # inside layer 5: from the end of layer 4, each tap's MFMAs issued, the epilogue
    names = {6: "layer 4 end"} | {43 + t: f"L5 tap {t} issued" for t in range(8)} | {52: "L5 tap 8 issued", 53: "L5 epilogue", 7: "L5 end"}
prev, prevk = t0, 0
for i in sorted(names):
    dt = (st[i] - prev) / 100.0
    cyc = st[64 + i] - st[64 + prevk]
    print(f"{names[i]:16s} {dt:8.2f} us {cyc:8d} cyc {cyc / max(dt, 1e-9) / 1e3:5.2f} GHz  (t = {(st[i] - t0) / 100.0:8.2f})")
    prev, prevk = st[i], i
