#!/usr/bin/env python3
"""Per-layer precision table of the C3 trunk (VERDICT r05 'next' 3): how much of the fp16 trunk's
logit / value error each 3x3 conv contributes, on the trained-like suites of
tests/test_gpu_trained_scale.py, by a CPU emulation of the kernels' arithmetic.

The emulation: BN folded into the conv weights (as az_net_load_weights folds them), the layer's
MFMA operands rounded to fp16 (round to nearest: the fp16 trunk's activation planes and weight
pieces), products exact and accumulated in float64 (the kernels accumulate in fp32: ~1e-7
relative, far below the effects measured), the residual stream exact (the fp16 trunk carries it
as fp16 + int8 remainder, ~2^-20).  Every other layer and the heads run in float64.  The reference
is the float64 network.  A layer in 'f16x3' is exact here (its 22-bit pieces hold the operands to
~2^-22: measured 1.0e-5 for the whole C3 trunk on the GPU).

Output: for each suite, max|dlogit| / max|dvalue| with (a) every layer fp16 (checks the emulation
against the GPU figure), (b) layer i alone fp16, the rest exact -- the floor of any per-layer mixed
mode that runs at least one trunk conv in single-pass fp16, (c) every layer with one operand split
into hi + lo pieces and the other single fp16 (the two-MFMA products hi*hi + hi*lo).

  python3 tools/layer_precision.py [--boards 16] [--out profiles/r06_layer_precision.json]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "alphazero-multi-game_amd")):
    sys.path.insert(0, p)


def fold(p, conv, bn):
    """(W * scale, bias) in float64: the conv + eval BN folded as the engine folds it."""
    w = p[conv + ".weight"].double()
    g, b = p[bn + ".weight"].double(), p[bn + ".bias"].double()
    mu, var = p[bn + ".running_mean"].double(), p[bn + ".running_var"].double()
    scale = g / torch.sqrt(var + 1e-5)
    cb = p[conv + ".bias"].double() if (conv + ".bias") in p else torch.zeros_like(mu)
    return w * scale[:, None, None, None], (cb - mu) * scale + b


def r16(t):
    return t.to(torch.float16).double()


def r16_scaled(w):
    """fp16 rounding of each output channel scaled by 2^s (max |w| in [2^13, 2^14)), as the F16X3
    weight pieces are scaled: a relative 2^-12 whatever the channel's magnitude (no subnormals)."""
    m = w.abs().amax(dim=(1, 2, 3))
    s = torch.where(m > 0, 13 - torch.floor(torch.log2(m)), torch.zeros_like(m))
    up = torch.pow(2.0, s)[:, None, None, None]
    return (w * up).to(torch.float16).double() / up


class Net:
    def __init__(self, desc, blob):
        import net_oracle
        self.d = desc
        self.p = net_oracle.unpack(desc, blob)
        self.layers = [fold(self.p, "input_conv", "input_bn")]
        for i in range(desc.blocks):
            self.layers.append(fold(self.p, f"blocks.{i}.0", f"blocks.{i}.1"))
            self.layers.append(fold(self.p, f"blocks.{i}.3", f"blocks.{i}.4"))

    mode = "both"     # which operands an fp16 layer rounds: both (single-pass fp16), x or w only (two MFMAs)

    def conv(self, l, x, fp16):
        w, b = self.layers[l]
        if fp16:
            if self.mode in ("both", "x"):
                x = r16(x)
            if self.mode in ("both", "w"):
                w = r16(w)
            if self.mode in ("both_s", "ws"):
                w = r16_scaled(w)
            if self.mode == "both_s":
                x = r16(x)
        return F.conv2d(x, w, b, padding=1)

    def trunk_from(self, l0, state, fp16, cache=None):
        """The trunk from conv l0 (0: the input conv; 1 + 2i / 2 + 2i: block i's first / second conv)
        given that conv's input state (a tensor; for a second conv the pair (y, residual)), with the
        convs in `fp16` rounded; cache[l] keeps every conv's input state of this run."""
        d = self.d
        l = l0
        h = state
        if l == 0:
            h = torch.relu(self.conv(0, state, 0 in fp16))
            l = 1
        while l <= 2 * d.blocks:
            if cache is not None:
                cache[l] = h
            if l % 2 == 1:
                h = (torch.relu(self.conv(l, h, l in fp16)), h)
            else:
                y, r = h
                z = self.conv(l, y, l in fp16)
                h = torch.relu(z + r) if d.residual else torch.relu(z)
            l += 1
        return h

    def heads(self, h):
        d, p = self.d, self.p
        x = F.adaptive_avg_pool2d(h, (d.pool, d.pool))

        def cbn(x, conv, bn):
            w, b = fold(p, conv, bn)
            return F.conv2d(x, w, b)
        pol = torch.relu(cbn(x, "policy_conv", "policy_bn")).reshape(x.shape[0], -1)
        pol = F.linear(pol, p["policy_fc.weight"].double(), p["policy_fc.bias"].double())
        v = torch.relu(cbn(x, "value_conv", "value_bn")).reshape(x.shape[0], -1)
        v = torch.relu(F.linear(v, p["value_fc1.weight"].double(), p["value_fc1.bias"].double()))
        v = torch.tanh(F.linear(v, p["value_fc2.weight"].double(), p["value_fc2.bias"].double()))
        return pol.numpy(), v.reshape(-1).numpy()


def table(name, desc, blob, x):
    net = Net(desc, blob)
    x = torch.from_numpy(np.ascontiguousarray(x, np.float64))
    t0 = time.time()
    cache = {}
    with torch.no_grad():
        ref_l, ref_v = net.heads(net.trunk_from(0, x, set(), cache))
        L = 1 + 2 * desc.blocks

        def err(fp16):
            lo = min(fp16)
            h = net.trunk_from(lo, x if lo == 0 else cache[lo], fp16)
            lg, v = net.heads(h)
            return float(np.abs(lg - ref_l).max()), float(np.abs(v - ref_v).max())
        all16 = err(set(range(L)))
        # two-MFMA splits, every layer: activations single fp16 with weights hi + lo (x only), or
        # weights single fp16 with activations hi + lo (w only)
        net.mode = "x"
        x_only = err(set(range(L)))
        net.mode = "w"
        w_only = err(set(range(L)))
        # the same with the weights scaled per output channel before rounding (as F16X3's pieces)
        net.mode = "ws"
        ws_only = err(set(range(L)))
        net.mode = "both_s"
        both_s = err(set(range(L)))
        net.mode = "both"
        per = []
        for l in range(L):
            el, ev = err({l})
            per.append({"layer": l, "conv": "input" if l == 0 else f"block {(l - 1) // 2} conv {(l - 1) % 2 + 1}",
                        "max_dlogit": el, "max_dvalue": ev})
            print(f"  {name} layer {l:2d}: {el:.3e} {ev:.3e}", flush=True)
    order = sorted(per, key=lambda r: max(r["max_dlogit"], r["max_dvalue"]))
    return {"suite": name, "boards": int(x.shape[0]), "logit_max": float(np.abs(ref_l).max()),
            "value_max": float(np.abs(ref_v).max()),
            "all_layers_fp16": {"max_dlogit": all16[0], "max_dvalue": all16[1]},
            "all_layers_two_mfma_x_rounded": {"max_dlogit": x_only[0], "max_dvalue": x_only[1]},
            "all_layers_two_mfma_w_rounded": {"max_dlogit": w_only[0], "max_dvalue": w_only[1]},
            "all_layers_two_mfma_w_rounded_scaled": {"max_dlogit": ws_only[0], "max_dvalue": ws_only[1]},
            "all_layers_fp16_w_scaled": {"max_dlogit": both_s[0], "max_dvalue": both_s[1]},
            "single_layer_fp16": per,
            "smallest_single_layer": order[0], "largest_single_layer": order[-1],
            "layers_within_5e-5": [r["layer"] for r in per if max(r["max_dlogit"], r["max_dvalue"]) <= 5e-5],
            "seconds": time.time() - t0}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--boards", type=int, default=16)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r06_layer_precision.json"))
    a = ap.parse_args()
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    import az_amd  # noqa: F401  (NetDesc)
    from az_amd import NetDesc
    import test_gpu_trained_scale as T
    bs, ci, ch, blocks, A = T.NETS["c3"]
    desc = NetDesc(bs, ci, ch, blocks, A, 32, 8, 256, 1, 0, 3, a.boards)
    out = {"workload": "C3 net (15x15, 20 blocks x 256 filters), trained-like suites of tests/test_gpu_trained_scale.py",
           "method": __doc__.split("\n\n")[1].replace("\n", " "), "suites": []}
    x = T._planes("c3", a.boards, seed=17)
    out["suites"].append(table("trained_heads (trained_scale_blob, seed 1234)", desc, T.trained_scale_blob(desc, 1234, x), x))
    x = T._planes("c3", a.boards, seed=31)
    blob, amax = T.trunk_scaled_blob(desc, 2468, x)
    r = table("trained_trunk (trunk_scaled_blob, seed 2468)", desc, blob, x)
    r["activation_max"] = amax
    out["suites"].append(r)
    json.dump(out, open(a.out, "w"), indent=1)
    for s in out["suites"]:
        print(s["suite"], "all fp16:", s["all_layers_fp16"], "smallest single layer:", s["smallest_single_layer"],
              "within 5e-5:", s["layers_within_5e-5"])


if __name__ == "__main__":
    main()
