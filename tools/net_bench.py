#!/usr/bin/env python3
"""Trunk-conv microbenchmark: C3 net (15x15, 20 blocks x 256 filters) forward at batch B
(--game go19 / chess: the C4 / C5 nets).  Prints the average trunk-conv launch time (HIP events
on the engine stream) and the algorithmic TFLOP/s (2*9*C*C*H*W FLOP per board per conv).  Used for kernel iteration and
for rocprofv3 PMC passes (the conv kernel is the only MFMA kernel of note)."""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-multi-game_amd"))
import az_amd  # noqa: E402

GAMES = {"gomoku15": (15, 11, 225), "go19": (19, 8, 362), "chess": (8, 111, 4672), "gomoku9": (9, 11, 81),
         "go13": (13, 8, 170), "go9": (9, 8, 82)}   # board, planes, actions
PREC = {"f32": az_amd.AZ_PREC_F32, "bf16x3": az_amd.AZ_PREC_BF16X3, "bf16": az_amd.AZ_PREC_BF16,
        "fp16": az_amd.AZ_PREC_FP16, "f16x3": az_amd.AZ_PREC_F16X3}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--precision", default="fp16", choices=list(PREC))
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--channels", type=int, default=256)
    ap.add_argument("--blocks", type=int, default=20)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--flags", default="", help="comma list of conv variant flag sets to A/B (alternating rounds)")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--sm-kernels", default="", help="comma list of k_smallnet kernels to A/B (0 = current, 1 = round 2; "
                                                     "optionally :4 / :8 waves, e.g. 0:8,0:4,1:8)")
    ap.add_argument("--game", default="gomoku15", choices=list(GAMES))
    a = ap.parse_args()
    bs, planes, actions = GAMES[a.game]
    if os.environ.get("AZ_SM_WAVES"):      # measurement-only kernel variants (diag entry points)
        from az_amd import _lib as _l
        _l.lib().az_diag_set_smallnet_waves(int(os.environ["AZ_SM_WAVES"]))
    if os.environ.get("AZ_CONV_FLAGS"):
        from az_amd import _lib as _l
        _l.lib().az_diag_set_conv_flags(int(os.environ["AZ_CONV_FLAGS"], 0))
    if os.environ.get("AZ_V9_STAGGER"):
        from az_amd import _lib as _l
        _l.lib().az_diag_set_v9_stagger(int(os.environ["AZ_V9_STAGGER"]))
    eng = az_amd.Engine(int(os.environ.get("LOCAL_RANK", 0)))
    desc = az_amd.NetDesc(bs, planes, a.channels, a.blocks, actions, 32, 8, 256, 1, 0, PREC[a.precision], a.batch)
    net = az_amd.HipNeuralNetwork(eng, desc)
    net.init_random(1234)
    x = (np.random.default_rng(0).random((a.batch, planes, bs, bs)) < (0.05 if planes > 16 else 0.2)).astype(np.float32)
    net.forward(x)
    if a.sm_kernels:
        from az_amd import _lib
        sets = a.sm_kernels.split(",")
        res = {f: [] for f in sets}
        flops = a.batch * 2 * 9 * a.channels * a.channels * bs * bs
        for _ in range(a.rounds):
            for f in sets:
                k, _, w = f.partition(":")
                _lib.lib().az_diag_set_smallnet_kernel(int(k))
                _lib.lib().az_diag_set_smallnet_waves(int(w or 8))
                net.forward(x)
                net.profile(True)
                for _ in range(a.iters):
                    net.forward(x)
                ms, launches, fw = net.profile_read()
                res[f].append(ms / fw)
        for f in sets:
            v = np.array(res[f])
            print(f"k_smallnet kernel {f}: {1e3 * np.median(v):.1f} us/forward (min {1e3 * v.min():.1f} max {1e3 * v.max():.1f}), "
                  f"{2 * a.blocks * flops / np.median(v) / 1e9:.1f} TFLOP/s trunk")
        return
    if a.flags:
        from az_amd import _lib
        sets = [int(f, 0) for f in a.flags.split(",")]
        res = {f: [] for f in sets}
        flops = a.batch * 2 * 9 * a.channels * a.channels * bs * bs
        for _ in range(a.rounds):
            for f in sets:
                _lib.lib().az_diag_set_conv_flags(f)
                net.forward(x)
                net.profile(True)
                for _ in range(a.iters):
                    net.forward(x)
                ms, launches, _ = net.profile_read()
                res[f].append(ms / launches)
        for f in sets:
            v = np.array(res[f])
            print(f"{a.precision} flags={f:#x}: trunk {np.median(v):.4f} ms/launch (min {v.min():.4f} max {v.max():.4f}), "
                  f"{flops / np.median(v) / 1e9:.1f} TFLOP/s")
        return
    net.profile(True)
    t0 = time.perf_counter()
    for _ in range(a.iters):
        net.forward(x)
    wall = (time.perf_counter() - t0) / a.iters
    ms, launches, fw = net.profile_read()
    per = ms / launches
    flops = a.batch * 2 * 9 * a.channels * a.channels * bs * bs
    print(f"{a.game} {a.precision} B={a.batch}: trunk {per:.4f} ms/launch, {flops / per / 1e9:.1f} TFLOP/s algorithmic, "
          f"forward wall {wall * 1e3:.2f} ms (incl. H2D/D2H)")


if __name__ == "__main__":
    main()
