#!/usr/bin/env python3
"""Golden vectors of the reference's C++ DDW-RandWire network (row f4), generated HERE where
/root/reference exists (the GPU box never reads it):

  ref_randwire_graphs.json  the 20 rand-wire graphs (RandWireBlock(C, 32, 0.75, seed=i),
                            src/nn/ddw_randwire_resnet.cpp:399) as the reference builds them:
                            nodes() order, inputs / outputs, predecessors, topological order, edges
  randwire_golden.npz       per case: the input planes and the reference module's forward
                            (logits, value) in eval() mode with every state entry overwritten by
                            the counter-based blob (oracle/randwire_oracle.init_blob, the same as
                            az_net_init_random); the harness's state_dict names / shapes are
                            checked against randwire_oracle.param_shapes (the blob order)

Needs oracle/_ref/ref_randwire (oracle/build_ref_randwire.sh).  Usage: python3 gen_randwire_golden.py
"""
import json
import os
import subprocess
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import randwire_oracle as RW  # noqa: E402

EXE = os.path.join(ROOT, "oracle", "_ref", "ref_randwire")
N_GRAPHS = 20   # the reference's default num_blocks (python/alphazero/models/ddw_randwire_cpp.py:27)

CASES = [  # name, in_planes, board, channels, blocks, batch, seed
    ("c16_b1_h9", 11, 9, 16, 1, 3, 11),
    ("c32_b2_h15", 11, 15, 32, 2, 2, 12),
    ("c16_b3_h8", 11, 8, 16, 3, 2, 13),
]


def desc(inp, bs, ch, nb):
    return types.SimpleNamespace(board_size=bs, in_planes=inp, channels=ch, blocks=nb, action_size=bs * bs,
                                 head_channels=32, pool=8, fc_hidden=256)


def main():
    out = subprocess.run([EXE, "graphs", str(N_GRAPHS)], check=True, capture_output=True, text=True, timeout=120).stdout
    with open(RW.GRAPHS, "w") as f:
        f.write(out)
    graphs = RW.load_graphs()
    arrays = {}
    for name, inp, bs, ch, nb, B, seed in CASES:
        d = desc(inp, bs, ch, nb)
        blob = RW.init_blob(d, graphs, seed)
        rng = np.random.default_rng(seed)
        planes = (rng.random((B, inp, bs, bs)) < 0.3).astype(np.float32)
        with tempfile.TemporaryDirectory() as td:
            bp, pp, op = (os.path.join(td, x) for x in ("blob.f32", "planes.f32", "out.f32"))
            blob.tofile(bp)
            planes.tofile(pp)
            res = subprocess.run([EXE, "forward", str(inp), str(bs * bs), str(ch), str(nb), str(bs), str(B), bp, pp, op],
                                 check=True, capture_output=True, text=True, timeout=600)
            o = np.fromfile(op, np.float32)
        entries = [json.loads(line) for line in res.stdout.splitlines() if line.startswith("{")]
        spec = RW.param_shapes(d, graphs)
        assert [(e["name"], tuple(e["shape"])) for e in entries] == [(n, s) for n, s, _, _ in spec], name
        logits, value = o[:B * bs * bs].reshape(B, bs * bs), o[B * bs * bs:]
        ol, ov = RW.forward(d, graphs, blob, planes)
        print(f"{name}: {len(entries)} state entries, {blob.size} floats; oracle max|dlogit| "
              f"{np.abs(ol - logits).max():.3g} (|logit| max {np.abs(logits).max():.3g}), max|dvalue| {np.abs(ov - value).max():.3g}")
        arrays[name + "_planes"] = planes
        arrays[name + "_logits"] = logits
        arrays[name + "_value"] = value
        arrays[name + "_cfg"] = np.array([inp, bs, ch, nb, B, seed], np.int64)
    np.savez_compressed(os.path.join(HERE, "randwire_golden.npz"), **arrays)


if __name__ == "__main__":
    main()
