#!/usr/bin/env python3
"""DDW-RandWire forward benchmark (row f4): the reference's default DDWRandWireResNet(11, 225,
channels=128, num_blocks=20) on 15x15 (src/nn/ddw_randwire_resnet.cpp:387-468) at batch B through
az_net_forward (device-resident weights; planes in / logits + value out over PCIe, small).
Prints one JSON line: ms per forward (wall, synchronous), boards/s, and the algorithmic FLOP rate
of the whole forward against the MFMA peak of the precision (MI355X_MICROARCH.md): f32-input MFMA
157.3 TFLOP/s for --precision f32 (the reference module's arithmetic), dense bf16 / fp16 2.5 PFLOP/s
for --precision bf16x3 (fp32-faithful split operands: three MFMAs per product, FLOPs counted once)
and --precision fp16 (node convs on conv3x3_v4; SE and the residual stream stay fp32).  FLOPs counted: every 3x3 conv and router /
output-router 1x1 conv (2 * K * N per pixel), the input conv; heads and SE excluded (< 0.1 %)."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-multi-game_amd"))
import az_amd  # noqa: E402


def flops_per_board(bs, C, nb, inp):
    HW = bs * bs
    f = 2 * 9 * inp * C * HW
    for i in range(nb):
        g = az_amd.randwire_graph(i)
        for v in range(32):
            deg = len(g["preds"][v])
            f += 2 * (2 * 9 * C * C * HW)
            if deg > 1:
                f += 2 * deg * C * C * HW
        if len(g["output_nodes"]) > 1:
            f += 2 * len(g["output_nodes"]) * C * C * HW
    return f


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--channels", type=int, default=128)
    ap.add_argument("--blocks", type=int, default=20)
    ap.add_argument("--board", type=int, default=15)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--precision", default="f32", choices=["f32", "bf16x3", "fp16"])
    a = ap.parse_args()
    eng = az_amd.Engine(int(os.environ.get("LOCAL_RANK", 0)))
    net = az_amd.createDDWRandWireResNet(eng, 11, a.board * a.board, a.channels, a.blocks, a.board, a.batch)
    if a.precision != "f32":
        net.set_precision(az_amd.AZ_PREC_FP16 if a.precision == "fp16" else az_amd.AZ_PREC_BF16X3)
    net.init_random(7)
    x = (np.random.default_rng(0).random((a.batch, 11, a.board, a.board)) < 0.2).astype(np.float32)
    net.forward(x)
    t0 = time.perf_counter()
    for _ in range(a.iters):
        net.forward(x)
    ms = (time.perf_counter() - t0) * 1e3 / a.iters
    fl = flops_per_board(a.board, a.channels, a.blocks, 11) * a.batch
    tf = fl / (ms * 1e-3) / 1e12
    print(json.dumps({"net": f"DDWRandWireResNet(11, {a.board * a.board}, {a.channels}, {a.blocks})", "board": a.board,
                      "precision": a.precision,
                      "batch": a.batch, "ms_per_forward": round(ms, 3), "boards_per_s": round(a.batch / ms * 1e3, 1),
                      "gflop_per_board": round(fl / a.batch / 1e9, 2), "tflops": round(tf, 2),
                      "frac_peak": round(tf / (157.3 if a.precision == "f32" else 2500.0), 4),
                      "peak_tflops": 157.3 if a.precision == "f32" else 2500.0}), flush=True)
    net.close()
    eng.close()


if __name__ == "__main__":
    main()
