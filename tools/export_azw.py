#!/usr/bin/env python3
"""Convert the reference's plain ResNet (python/simple_export.py SimplifiedModel / the exporter
fallback stack) into the engine's .azw weight file, which HipNeuralNetwork::load /
createNeuralNetwork read.  The input is either

  * the reference's TorchScript model file (torch.jit.save, python/scripts/self_play.py:139-193):
    read by the host module's TorchScript reader (cpp/src/torchscript_reader.cpp: zip directory +
    restricted pickle machine, nothing executed), layout and shape recognised there; or
  * a PyTorch state_dict, loaded with torch.load(weights_only=True) (tensors only, nothing executed).

  python tools/export_azw.py model.pt model.azw [--precision fp16] [--max-batch 2048] [--game go]

The blob is the state_dict values in order, num_batches_tracked dropped; the net shape is read from
the tensor shapes.  (createNeuralNetwork also takes the TorchScript file directly.)  File layout: b"AZW1", 12 int32 (board, in_planes, channels, blocks,
action_size, head_channels, pool, fc_hidden, residual, conv_bias, precision, max_batch),
uint64 count, float32[count]."""
import argparse
import math
import os
import re
import struct
import sys
import zipfile

import numpy as np

PREC = {"f32": 0, "bf16x3": 1, "bf16": 2, "fp16": 3}


def shape_of(sd, residual=None):
    w = sd["input_conv.weight"]
    F, cin = int(w.shape[0]), int(w.shape[1])
    blocks = len({int(m.group(1)) for k in sd for m in [re.match(r"(?:res_blocks|middle_layers|blocks)\.(\d+)\.", k)] if m})
    A = int(sd["policy_fc.weight"].shape[0])
    hc = int(sd["policy_conv.weight"].shape[0])
    pp = int(sd["policy_fc.weight"].shape[1]) // hc
    bs = int(round(math.sqrt(A)))
    assert bs * bs == A, "policy size must be a square board"
    return dict(board=bs, in_planes=cin, channels=F, blocks=blocks, action_size=A, head_channels=hc,
                pool=int(round(math.sqrt(pp))), fc_hidden=int(sd["value_fc1.weight"].shape[0]),
                residual=1 if residual is None else int(residual), conv_bias=int("input_conv.bias" in sd))


def is_torchscript(path):
    """torch.jit.save archives carry compiled code next to data.pkl; torch.save state dicts do not."""
    if not zipfile.is_zipfile(path):
        return False
    with zipfile.ZipFile(path) as z:
        names = z.namelist()
    return any(n.endswith("/constants.pkl") or "/code/" in n for n in names)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("dst")
    ap.add_argument("--precision", default="fp16", choices=list(PREC))
    ap.add_argument("--max-batch", type=int, default=2048)
    ap.add_argument("--residual", type=int, default=1, help="1: SimplifiedModel residual blocks; 0: plain stack")
    ap.add_argument("--game", default="gomoku", choices=["gomoku", "go"], help="TorchScript input: policy size -> board")
    ap.add_argument("--board", type=int, default=0, help="TorchScript input: board size (0: from the policy size)")
    a = ap.parse_args()
    if is_torchscript(a.src):
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                        "alphazero-multi-game_amd"))
        import _alphazero_cpp as az
        gt = az.GameType.GO if a.game == "go" else az.GameType.GOMOKU
        s, blob = az.torchScriptResNet(a.src, gt, a.board)
        blob = np.asarray(blob, np.float32)
    else:
        import torch
        sd = torch.load(a.src, map_location="cpu", weights_only=True)
        if "state_dict" in sd:
            sd = sd["state_dict"]
        s = shape_of(sd, a.residual)
        blob = np.concatenate([v.detach().float().numpy().ravel() for k, v in sd.items()
                               if not k.endswith("num_batches_tracked")]).astype(np.float32)
    hdr = [s["board"], s["in_planes"], s["channels"], s["blocks"], s["action_size"], s["head_channels"], s["pool"],
           s["fc_hidden"], s["residual"], s["conv_bias"], PREC[a.precision], a.max_batch]
    with open(a.dst, "wb") as f:
        f.write(b"AZW1")
        f.write(struct.pack("<12i", *hdr))
        f.write(struct.pack("<Q", blob.size))
        f.write(blob.tobytes())
    print(f"{a.dst}: {s} {blob.size} parameters, trunk {a.precision}")


if __name__ == "__main__":
    main()
