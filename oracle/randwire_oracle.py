"""oracle/randwire_oracle.py -- TEST INFRASTRUCTURE ONLY (row f4, DDW-RandWire).

fp32 PyTorch-CPU restatement of the reference's C++ DDWRandWireResNet
(src/nn/ddw_randwire_resnet.cpp) over the canonical parameter blob of
az_net_create_randwire (torch state_dict order, num_batches_tracked dropped, BN in eval form):

  input_conv (3x3, no bias) + input_bn + ReLU                          :391-394, :431
  per rand-wire block i (RandWireBlock(C, 32, 0.75, seed=i), :399):
      router_<v> for every node with in-degree > 0, nodes() order        :225-232
          (1x1 conv over in_degree*C channels, no bias, + BN + ReLU)     :64-75
      block_<v> for every node, nodes() order                            :235-239
          conv1 3x3 + bn1 + ReLU, conv2 3x3 + bn2, SE(C, 16), + x, ReLU  :35-61
          SE: mean over H x W -> Linear(C, C/16) -> ReLU -> Linear -> sigmoid, x * s   :10-32
      output_router when more than one sink                              :242-245
      forward: input nodes on the block input, the rest in topological order; a node
      with several predecessors takes router(concat(preds in insertion order)),
      one predecessor is passed through; output = output router over the sinks'
      concat, or the single sink                                          :321-384
  adaptive_avg_pool2d to min(8, H) (identity at 8), policy / value heads  :438-467

The graphs are NOT regenerated here: they come from tests/golden/ref_randwire_graphs.json,
dumped by the reference itself (oracle/ref_randwire, built by oracle/build_ref_randwire.sh with
the P10 fix of its undefined-behaviour duplicate-edge test).  The whole restatement is pinned
by tests/golden/randwire_golden.npz (forward outputs of the reference C++ module).
"""
import json
import os

import numpy as np
import torch
import torch.nn.functional as F

from net_oracle import _splitmix64

GRAPHS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                      "ref_randwire_graphs.json")


def load_graphs(path=GRAPHS):
    out = []
    with open(path) as f:
        for line in f:
            g = json.loads(line)
            g["preds"] = {int(k): v for k, v in g["preds"].items()}
            out.append(g)
    return out


def param_shapes(desc, graphs):
    """[(name, shape, kind, fan_in)] in blob order (kinds as az_net_init_random)."""
    C, Ci, HC, A, Hd = desc.channels, desc.in_planes, desc.head_channels, desc.action_size, desc.fc_hidden
    PP = desc.pool * desc.pool
    R = C // 16
    out = []

    def conv(name, co, ci, k):
        out.append((name + ".weight", (co, ci, k, k), 0, ci * k * k))

    def bn(name, co):
        out.extend([(name + ".weight", (co,), 2, 1), (name + ".bias", (co,), 3, 1),
                    (name + ".running_mean", (co,), 4, 1), (name + ".running_var", (co,), 5, 1)])

    def linear(name, o, i):
        out.extend([(name + ".weight", (o, i), 0, i), (name + ".bias", (o,), 1, i)])

    conv("input_conv", C, Ci, 3)
    bn("input_bn", C)
    for i in range(desc.blocks):
        g = graphs[i]
        pre = f"rand_wire_blocks.{i}."
        for v in g["nodes"]:
            deg = len(g["preds"][v])
            if deg > 0:
                conv(pre + f"router_{v}.conv", C, deg * C, 1)
                bn(pre + f"router_{v}.bn", C)
        for v in g["nodes"]:
            b = pre + f"block_{v}."
            conv(b + "conv1", C, C, 3)
            bn(b + "bn1", C)
            conv(b + "conv2", C, C, 3)
            bn(b + "bn2", C)
            linear(b + "se.excitation.0", R, C)
            linear(b + "se.excitation.2", C, R)
        if len(g["output_nodes"]) > 1:
            conv(pre + "output_router.conv", C, len(g["output_nodes"]) * C, 1)
            bn(pre + "output_router.bn", C)
    conv("policy_conv", HC, C, 1)
    bn("policy_bn", HC)
    linear("policy_fc", A, HC * PP)
    conv("value_conv", HC, C, 1)
    bn("value_bn", HC)
    linear("value_fc1", Hd, HC * PP)
    linear("value_fc2", 1, Hd)
    return out


def init_blob(desc, graphs, seed):
    """az_net_init_random for a rand-wire net: the counter-based generator over this blob order."""
    parts = []
    seed = np.uint64(seed)
    for t, (_, shape, kind, fan_in) in enumerate(param_shapes(desc, graphs)):
        n = int(np.prod(shape))
        i = np.arange(n, dtype=np.uint64)
        r = _splitmix64(seed ^ (np.uint64(t) << np.uint64(40)) ^ i)
        u = (r >> np.uint64(40)).astype(np.int32).astype(np.float32) * np.float32(1.0 / 8388608.0) - np.float32(1.0)
        bound = np.float32(1.0) / np.sqrt(np.float32(fan_in))
        if kind in (0, 1):
            v = u * bound
        elif kind == 2:
            v = np.float32(1.0) + np.float32(0.1) * u
        elif kind in (3, 4):
            v = np.float32(0.1) * u
        else:
            v = np.float32(1.0) + np.float32(0.25) * (u + np.float32(1.0))
        parts.append(v.astype(np.float32))
    return np.concatenate(parts)


def unpack(desc, graphs, blob):
    out, off = {}, 0
    for name, shape, _, _ in param_shapes(desc, graphs):
        n = int(np.prod(shape))
        out[name] = torch.from_numpy(np.asarray(blob[off:off + n], np.float32).reshape(shape).copy())
        off += n
    assert off == blob.size, (off, blob.size)
    return out


def forward(desc, graphs, blob, planes):
    """planes [B, C_in, H, W] -> (logits [B, A], value [B]), fp32 on the CPU."""
    p = unpack(desc, graphs, blob)
    x = torch.from_numpy(np.ascontiguousarray(planes, np.float32))

    def bn(x, name):
        return F.batch_norm(x, p[name + ".running_mean"], p[name + ".running_var"], p[name + ".weight"],
                            p[name + ".bias"], training=False, eps=1e-5)

    def conv(x, name, pad):
        return F.conv2d(x, p[name + ".weight"], None, padding=pad)

    def router(x, name):
        return torch.relu(bn(conv(x, name + ".conv", 0), name + ".bn"))

    def resblock(x, name):
        y = torch.relu(bn(conv(x, name + "conv1", 1), name + "bn1"))
        y = bn(conv(y, name + "conv2", 1), name + "bn2")
        s = y.mean(dim=(2, 3))
        s = torch.relu(F.linear(s, p[name + "se.excitation.0.weight"], p[name + "se.excitation.0.bias"]))
        s = torch.sigmoid(F.linear(s, p[name + "se.excitation.2.weight"], p[name + "se.excitation.2.bias"]))
        return torch.relu(y * s[:, :, None, None] + x)

    with torch.no_grad():
        x = torch.relu(bn(conv(x, "input_conv", 1), "input_bn"))
        for i in range(desc.blocks):
            g = graphs[i]
            pre = f"rand_wire_blocks.{i}."
            outs = {}
            for v in g["input_nodes"]:
                outs[v] = resblock(x, pre + f"block_{v}.")
            for v in g["topo"]:
                if v in g["input_nodes"] or not g["preds"][v]:
                    continue
                ins = [outs[u] for u in g["preds"][v]]
                routed = router(torch.cat(ins, 1), pre + f"router_{v}") if len(ins) > 1 else ins[0]
                outs[v] = resblock(routed, pre + f"block_{v}.")
            if len(g["output_nodes"]) > 1:
                x = router(torch.cat([outs[v] for v in g["output_nodes"]], 1), pre + "output_router")
            else:
                x = outs[g["output_nodes"][0]]
        t = min(8, x.shape[2], x.shape[3])
        if x.shape[2] != t or x.shape[3] != t:
            x = F.adaptive_avg_pool2d(x, (t, t))
        pol = torch.relu(bn(conv(x, "policy_conv", 0), "policy_bn")).reshape(x.shape[0], -1)
        pol = F.linear(pol, p["policy_fc.weight"], p["policy_fc.bias"])
        v = torch.relu(bn(conv(x, "value_conv", 0), "value_bn")).reshape(x.shape[0], -1)
        v = torch.relu(F.linear(v, p["value_fc1.weight"], p["value_fc1.bias"]))
        v = torch.tanh(F.linear(v, p["value_fc2.weight"], p["value_fc2.bias"]))
    return pol.numpy(), v.reshape(-1).numpy()
