#!/usr/bin/env python3
"""Per-block phases of the v6 trunk conv across CUs (diagnostic build with -DAZ_V4_STAMPS):
  make -C alphazero-multi-game_amd OUT=build_diag EXTRA=-DAZ_V4_STAMPS build_diag/libaz_hip.so
  python3 tools/v6_phases.py --flags 0x4,0x40a04
For each flag set: the last conv1 and conv2 launch of one C3 forward at B=2048 -- launch span,
per-block stagger / main loop / epilogue, idle gaps between consecutive blocks on one CU, and how
many CUs are in their epilogue at once (the HBM-burst picture)."""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["AZ_HIP_LIB"] = os.path.join(ROOT, "alphazero-multi-game_amd", os.environ.get("AZ_DIAG_DIR", "build_diag"), "libaz_hip.so")
sys.path.insert(0, os.path.join(ROOT, "alphazero-multi-game_amd"))
import az_amd  # noqa: E402
from az_amd import _lib  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--flags", default="0x4")
ap.add_argument("--batch", type=int, default=2048)
a = ap.parse_args()
eng = az_amd.Engine(0)
net = az_amd.HipNeuralNetwork(eng, az_amd.gomoku_net_desc(15, 256, 20, precision=az_amd.AZ_PREC_FP16, max_batch=a.batch))
net.init_random(1234)
x = (np.random.default_rng(0).random((a.batch, 11, 15, 15)) < 0.2).astype(np.float32)
SLOTS, MAXBLK = 48, 4096
nblk = a.batch // 2 * 2
for f in [int(v, 0) for v in a.flags.split(",")]:
    _lib.lib().az_diag_set_conv_flags(f)
    for _ in range(3):
        net.forward(x)
    buf = (ctypes.c_ulonglong * (SLOTS * MAXBLK * 8))()
    assert _lib.lib().az_diag_v4_stamps(buf, SLOTS * MAXBLK * 8) == 0
    st = np.frombuffer(buf, np.uint64).reshape(SLOTS, MAXBLK, 8)[:, :nblk, :]
    for slot, name in ((38, "conv1"), (39, "conv2")):
        s = st[slot].astype(np.int64)
        t0 = s[:, 0].min()
        beg, stag, mainend, end = [(s[:, k] - t0) * 10 / 1e3 for k in (0, 3, 1, 2)]   # us
        hw = st[slot][:, 7]
        cu = ((hw >> np.uint64(32)) & np.uint64(0xF)) * np.uint64(1 << 16) + ((hw >> np.uint64(8)) & np.uint64(0xF)) * np.uint64(16) \
            + ((hw >> np.uint64(13)) & np.uint64(0x7)) * np.uint64(256)          # xcc, cu_id, se_id
        gaps, nper = [], []
        for c in np.unique(cu):
            idx = np.where(cu == c)[0]
            o = idx[np.argsort(beg[idx])]
            nper.append(len(o))
            gaps += list(beg[o[1:]] - end[o[:-1]])
        ep = end - mainend
        first = np.argsort(beg)[:256]
        grid = np.linspace(0, end.max(), 2000)
        conc = np.array([((mainend <= t) & (end > t)).sum() for t in grid])
        print(f"flags={f:#x} {name}: span {end.max():6.1f} us  CUs {len(nper)} blocks/CU {np.mean(nper):.2f} "
              f"(max {max(nper)})  stagger {np.mean(stag - beg):5.2f}  main {np.mean(mainend - stag):6.2f}  "
              f"epilogue {ep.mean():6.2f} (round1 {ep[first].mean():6.2f}, rest {np.delete(ep, first).mean():6.2f})  "
              f"gap {np.mean(gaps):5.2f} (max {np.max(gaps):5.2f})  CUs in epilogue: mean {conc.mean():5.1f} "
              f"p90 {np.percentile(conc, 90):5.0f}")
