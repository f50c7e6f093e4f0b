#!/usr/bin/env python3
"""Phase timeline of one conv3x3_v9x3 launch (diagnostic build: make EXTRA=-DAZ_V9_STAMPS
OUT=build_stamps, loaded with AZ_DIAG_HIP_LIB).  Wave 0 of every block stamps s_memrealtime
(100 MHz) at its start, after the prologue barrier, after the main loop, after the epilogue's
stores issue and after they complete; HW_ID / XCC_ID name the CU.  Prints the per-block phase
averages, the launch span, and per CU the share of the span its blocks spent in each phase and in
gaps between blocks."""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-multi-game_amd"))
import az_amd  # noqa: E402
from az_amd import _lib  # noqa: E402

GAMES = {"gomoku15": (15, 11, 225), "go19": (19, 8, 362), "chess": (8, 111, 4672)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--game", default="gomoku15", choices=list(GAMES))
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--precision", default="f16x3", choices=["f16x3", "bf16x3"])
    ap.add_argument("--launch", type=int, default=21, help="trunk launch index (2 i + 1: block i's second conv)")
    ap.add_argument("--flags", type=lambda s: int(s, 0), default=None)
    a = ap.parse_args()
    bs, planes, A = GAMES[a.game]
    L = _lib.lib()
    f = L.az_diag_v9_stamps
    f.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    if f(-1, None, None, 0) != 0:
        raise SystemExit("not a stamp build (make EXTRA=-DAZ_V9_STAMPS OUT=build_stamps; AZ_DIAG_HIP_LIB)")
    if a.flags is not None:
        L.az_diag_set_conv_flags(a.flags)
    eng = az_amd.Engine(0)
    prec = {"f16x3": az_amd.AZ_PREC_F16X3, "bf16x3": az_amd.AZ_PREC_BF16X3}[a.precision]
    net = az_amd.HipNeuralNetwork(eng, az_amd.NetDesc(bs, planes, 256, 20, A, 32, 8, 256, 1, 0, prec, a.batch))
    net.init_random(1234)
    x = (np.random.default_rng(0).random((a.batch, planes, bs, bs)) < 0.2).astype(np.float32)
    net.forward(x)
    grid = a.batch if bs == 15 else (a.batch * bs * bs + 255) // 256
    st = np.zeros((grid, 5), np.uint64)
    hw = np.zeros((grid, 2), np.uint32)
    rows = []
    for rep in range(3):
        f(a.launch, None, None, 0)
        net.forward(x)
        assert f(-2, st.ctypes.data, hw.ctypes.data, grid) == 0
        t = st.astype(np.int64)
        assert (t[:, 0] > 0).all(), "missing stamps"
        t0 = t[:, 0].min()
        span = (t[:, 4].max() - t0) / 100.0                 # us
        ph = np.diff(t, axis=1) / 100.0                      # pro, main, epi issue, epi drain (us)
        cu = (hw[:, 1].astype(np.int64) << 16) | ((hw[:, 0] >> 8) & 0xFF)
        ucu = np.unique(cu)
        busy = np.zeros(4)
        gaps, first, tail = [], [], []
        per_cu = []
        for c in ucu:
            idx = np.where(cu == c)[0]
            o = idx[np.argsort(t[idx, 0])]
            per_cu.append(len(o))
            first.append((t[o[0], 0] - t0) / 100.0)
            tail.append((t[:, 4].max() - t[o[-1], 4]) / 100.0)
            gaps += list((t[o[1:], 0] - t[o[:-1], 4]) / 100.0)
            busy += ph[o].sum(axis=0)
        tot = span * len(ucu)
        rows.append(span)
        print(f"rep {rep}: span {span:.1f} us over {len(ucu)} CUs ({grid} blocks, {np.mean(per_cu):.2f} per CU, "
              f"max {max(per_cu)}); per block (us) prologue {ph[:, 0].mean():.2f}, main {ph[:, 1].mean():.2f}, "
              f"epilogue issue {ph[:, 2].mean():.2f}, drain {ph[:, 3].mean():.2f}")
        print(f"   share of CU-time: prologue {busy[0] / tot:.3f} main {busy[1] / tot:.3f} epilogue {busy[2] / tot:.3f} "
              f"drain {busy[3] / tot:.3f} gaps {sum(gaps) / tot:.3f} (mean gap {np.mean(gaps):.2f} us) "
              f"first-start {np.mean(first) / span:.3f} idle-tail {np.mean(tail) / span:.3f}")
        mm = ph[:, 1]
        print(f"   main loop per block: min {mm.min():.1f} median {np.median(mm):.1f} max {mm.max():.1f} us")
    print(f"span median {np.median(rows):.1f} us")


if __name__ == "__main__":
    main()
