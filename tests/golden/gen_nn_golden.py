#!/usr/bin/env python3
"""Golden input/output vectors of the reference's own Python network classes
(run here, where /root/reference exists; the GPU box never reads it):

  simple8   SimplifiedModel(11, 64, channels=16, blocks=2)  python/simple_export.py:12-66
            (heads flatten 32x8x8 directly: only 8x8 boards fit it)
  fallback15  exporter fallback DDWRandWireResNet(11, 225, channels=16, blocks=2)
            python/scripts/simple_export.py:40-96 (plain conv stack, adaptive 8x8 pool)

Weights come from the counter-based generator (oracle/net_oracle.init_blob, the
same as az_net_init_random), copied into the reference modules' state_dict in
order; inputs are feature planes of random legal positions.  Only the seeds, the
inputs and the outputs are stored (tests/golden/nn_golden.npz)."""
import importlib.util
import os
import sys
import types

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "alphazero-multi-game_amd")]
REF = "/root/reference/python"

import az_oracle as O  # noqa: E402
import net_oracle  # noqa: E402
from az_amd._lib import NetDesc  # noqa: E402


def load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def planes(bs, B, seed):
    rng = np.random.default_rng(seed)
    out = np.zeros((B, 11, bs, bs), np.float32)
    for b in range(B):
        k = int(rng.integers(0, bs * bs // 2))
        out[b] = O.position(bs, rng.permutation(bs * bs)[:k].tolist())[0]
    return out


def run(model, desc, seed, x):
    blob = net_oracle.init_blob(desc, seed)
    sd = model.state_dict()
    keys = [k for k in sd if not k.endswith("num_batches_tracked")]
    shapes = net_oracle.param_shapes(desc)
    assert len(keys) == len(shapes), (len(keys), len(shapes))
    off = 0
    new = {}
    for k, (_, shp, _, _) in zip(keys, shapes):
        assert tuple(sd[k].shape) == tuple(shp), (k, sd[k].shape, shp)
        n = int(np.prod(shp))
        new[k] = torch.from_numpy(blob[off:off + n].reshape(shp).copy())
        off += n
    assert off == blob.size
    model.load_state_dict(new, strict=False)
    model.eval()
    with torch.no_grad():
        p, v = model(torch.from_numpy(x))
    return p.numpy(), v.reshape(-1).numpy()


def main():
    out = {}
    se = load("ref_simple_export", os.path.join(REF, "simple_export.py"))
    d = NetDesc(8, 11, 16, 2, 64, 32, 8, 256, 1, 1, 0, 4)
    x = planes(8, 4, 1)
    p, v = run(se.SimplifiedModel(11, 64, channels=16, blocks=2), d, 21, x)
    out.update(simple8_x=x, simple8_logits=p, simple8_value=v, simple8_seed=21)
    # the exporter script falls back to its own plain stack when the alphazero package
    # cannot be imported (python/scripts/simple_export.py:30-40); make that import fail
    sys.modules["alphazero"] = types.ModuleType("alphazero")
    sx = load("ref_scripts_simple_export", os.path.join(REF, "scripts", "simple_export.py"))
    d = NetDesc(15, 11, 16, 2, 225, 32, 8, 256, 0, 0, 0, 4)
    x = planes(15, 4, 2)
    p, v = run(sx.DDWRandWireResNet(11, 225, channels=16, blocks=2), d, 22, x)
    out.update(fallback15_x=x, fallback15_logits=p, fallback15_value=v, fallback15_seed=22)
    np.savez_compressed(os.path.join(os.path.dirname(os.path.abspath(__file__)), "nn_golden.npz"), **out)
    print({k: np.asarray(v).shape for k, v in out.items()})


if __name__ == "__main__":
    main()
