#!/usr/bin/env python3
"""Small-batch DENSE diagnosis: one net (19x19 Go shape unless AZ_SB_GEO, 1 block) at B boards in fp16 / bf16,
forwarded by conv3x3_v6 and by conv3x3_v7 at every tile size; max differences between them and
against the fp32 oracle."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "alphazero-multi-game_amd"), os.path.join(ROOT, "oracle")]
import az_amd  # noqa: E402
import net_oracle  # noqa: E402
from az_amd import _lib  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 130
# AZ_SB_FLAGS="name=0xflags,...": the routings to compare (the first one is the reference, v6)
FLAGS = [(kv.split("=")[0], int(kv.split("=")[1], 16)) for kv in os.environ.get(
    "AZ_SB_FLAGS", "v6=0x904,v7_256=0x10804,v7_128=0x20804,v7_64=0x30804,v7_auto=0x804").split(",")]
# AZ_SB_GEO="board,in_planes,actions": the net's geometry (default the 19x19 Go net)
BS, CI, NACT = (int(v) for v in os.environ.get("AZ_SB_GEO", "19,8,362").split(","))
eng = az_amd.Engine(0)
for mode, prec in (("fp16", az_amd.AZ_PREC_FP16), ("bf16", az_amd.AZ_PREC_BF16)):
    desc = az_amd.NetDesc(BS, CI, 256, 1, NACT, 32, 8, 256, 1, 0, prec, B)
    net = az_amd.HipNeuralNetwork(eng, desc)
    blob = net_oracle.init_blob(desc, seed=31)
    net.load_weights(blob)
    rng = np.random.default_rng(19 * 7 + B)
    x = (rng.random((B, CI, BS, BS)) < (0.05 if CI > 16 else 0.25)).astype(np.float32)
    outs = {}
    for name, fl in FLAGS:
        _lib.lib().az_diag_set_conv_flags(fl)
        outs[name] = net.forward(x)
        print(f"{mode} {name}: {net.trunk_kernel()}", flush=True)
        outs[name + "_again"] = net.forward(x)
    _lib.lib().az_diag_set_conv_flags(0x204)
    idx = np.unique(np.concatenate([[0, B - 1], rng.choice(B, 6, replace=False)]))
    rl, rv = net_oracle.forward(desc, blob, x[idx])
    for k, (l, v) in outs.items():
        dl = np.abs(l - outs[FLAGS[0][0]][0])
        bad = np.where(dl.max(axis=1) > 0)[0]
        print(f"{mode} {k:12s}: vs v6 {dl.max():.3e} (boards {bad[:8].tolist()}{'...' if len(bad) > 8 else ''}, "
              f"{len(bad)} differ), vs fp32 {np.abs(l[idx] - rl).max():.3e}", flush=True)
    net.close()
