#!/usr/bin/env python3
"""Per-block phase timing of the trunk conv (diagnostic build with -DAZ_V4_STAMPS):
  make -C alphazero-multi-game_amd OUT=build_diag EXTRA=-DAZ_V4_STAMPS
  python3 tools/v4_stamps.py [--precision fp16]
Stamps (s_memrealtime, 100 MHz) of the LAST conv launch of one C3 forward at B=2048."""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["AZ_DIAG_HIP_LIB"] = os.path.join(ROOT, "alphazero-multi-game_amd", os.environ.get("AZ_DIAG_DIR", "build_diag"), "libaz_hip.so")
sys.path.insert(0, os.path.join(ROOT, "alphazero-multi-game_amd"))
import az_amd  # noqa: E402
from az_amd import _lib  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--precision", default="fp16")
ap.add_argument("--batch", type=int, default=2048)
a = ap.parse_args()
P = {"fp16": az_amd.AZ_PREC_FP16, "bf16": az_amd.AZ_PREC_BF16, "bf16x3": az_amd.AZ_PREC_BF16X3}[a.precision]
eng = az_amd.Engine(0)
net = az_amd.HipNeuralNetwork(eng, az_amd.gomoku_net_desc(15, 256, 20, precision=P, max_batch=a.batch))
net.init_random(1234)
x = (np.random.default_rng(0).random((a.batch, 11, 15, 15)) < 0.2).astype(np.float32)
for _ in range(3):
    net.forward(x)
nblk = a.batch // 2 * 2
SLOTS, MAXBLK = 48, 4096
buf = (ctypes.c_ulonglong * (SLOTS * MAXBLK * 8))()
assert _lib.lib().az_diag_v4_stamps(buf, SLOTS * MAXBLK * 8) == 0
allst4 = np.frombuffer(buf, np.uint64).reshape(SLOTS, MAXBLK, 8)[:, :nblk, :].astype(np.int64)
allst = allst4[:, :, :3]
rows = []
for slot in range(40):
    st = allst[slot]
    if st[:, 0].max() == 0:
        continue
    st = (st - st[:, 0].min()) * 10                  # ns
    rows.append((slot, st[:, 2].max() / 1e3, (st[:, 1] - st[:, 0]).mean() / 1e3, (st[:, 2] - st[:, 1]).mean() / 1e3,
                 allst4[slot, :, 3].mean(), allst4[slot, :, 4].mean(),
                 ((allst4[slot, :, 6] - allst4[slot, :, 5]) / np.maximum(1, allst4[slot, :, 1] - allst4[slot, :, 0])).mean() * 0.1))
print(f"{a.precision}: launches stamped {len(rows)}")
for name, sel in (("conv1 (even)", [r for r in rows if r[0] % 2 == 0 and r[0] < 38]),
                  ("conv2 (odd) ", [r for r in rows if r[0] % 2 == 1 and r[0] < 39]),
                  ("last launch ", rows[-1:])):
    if sel:
        sp, mn, ep, wt, it, ck = (np.mean([r[i] for r in sel]) for i in (1, 2, 3, 4, 5, 6))
        print(f"  {name}: span {sp:7.1f} us   main/block {mn:6.2f} us   epilogue/block {ep:6.2f} us   "
              f"wave0 wait+barrier {wt:7.0f} cyc  DMA issue {it:7.0f} cyc  clock {ck:.2f} GHz  (n={len(sel)})")
