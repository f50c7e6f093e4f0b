"""oracle/net_oracle.py -- TEST INFRASTRUCTURE ONLY.

fp32 restatement of the reference policy/value ConvNet on PyTorch CPU, taking the
canonical parameter blob of include/az_engine.h (torch state_dict order):
  * residual=1, conv_bias=1, pool=identity  == SimplifiedModel (python/simple_export.py:12-66)
  * residual=0, conv_bias=0, adaptive pool  == exporter fallback DDWRandWireResNet
                                               (python/scripts/simple_export.py:40-96)
  * residual=1 + adaptive pool (BASELINE.json's "20-block x 256-filter ResNet")
Pinned against golden outputs of the reference's own Python classes
(tests/golden/gen_nn_golden.py).  Also restates az_net_init_random (the
counter-based weight generator) in numpy with identical fp32 operations.
"""
import numpy as np
import torch
import torch.nn.functional as F

MASK64 = (1 << 64) - 1


def _splitmix64(x):
    """Vectorised SplitMix64 over uint64 numpy arrays."""
    x = (x + np.uint64(0x9E3779B97F4A7C15)) & np.uint64(MASK64)
    x = ((x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & np.uint64(MASK64)
    x = ((x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & np.uint64(MASK64)
    return x ^ (x >> np.uint64(31))


def param_shapes(desc):
    """[(name, shape, kind, fan_in)] in blob order; kinds as az_net_init_random."""
    d = desc
    Fc, Ci, HC, PP, A, Hd = d.channels, d.in_planes, d.head_channels, d.pool * d.pool, d.action_size, d.fc_hidden
    out = []

    def conv(name, co, ci, k):
        out.append((name + ".weight", (co, ci, k, k), 0, ci * k * k))
        if d.conv_bias:
            out.append((name + ".bias", (co,), 1, ci * k * k))

    def bn(name, co):
        out.extend([(name + ".weight", (co,), 2, 1), (name + ".bias", (co,), 3, 1),
                    (name + ".running_mean", (co,), 4, 1), (name + ".running_var", (co,), 5, 1)])

    conv("input_conv", Fc, Ci, 3)
    bn("input_bn", Fc)
    for i in range(d.blocks):
        conv(f"blocks.{i}.0", Fc, Fc, 3)
        bn(f"blocks.{i}.1", Fc)
        conv(f"blocks.{i}.3", Fc, Fc, 3)
        bn(f"blocks.{i}.4", Fc)
    conv("policy_conv", HC, Fc, 1)
    bn("policy_bn", HC)
    out += [("policy_fc.weight", (A, HC * PP), 0, HC * PP), ("policy_fc.bias", (A,), 1, HC * PP)]
    conv("value_conv", HC, Fc, 1)
    bn("value_bn", HC)
    out += [("value_fc1.weight", (Hd, HC * PP), 0, HC * PP), ("value_fc1.bias", (Hd,), 1, HC * PP),
            ("value_fc2.weight", (1, Hd), 0, Hd), ("value_fc2.bias", (1,), 1, Hd)]
    return out


def init_blob(desc, seed):
    """Numpy restatement of az_net_init_random (engine.hip), bit-identical."""
    parts = []
    seed = np.uint64(seed)
    for t, (_, shape, kind, fan_in) in enumerate(param_shapes(desc)):
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


def unpack(desc, blob):
    out = {}
    off = 0
    for name, shape, _, _ in param_shapes(desc):
        n = int(np.prod(shape))
        out[name] = torch.from_numpy(np.asarray(blob[off:off + n], np.float32).reshape(shape).copy())
        off += n
    assert off == blob.size, (off, blob.size)
    return out


def forward(desc, blob, planes):
    """planes [B, C_in, H, W] -> (logits [B, A], value [B]) in fp32 on the CPU."""
    p = unpack(desc, blob)
    x = torch.from_numpy(np.ascontiguousarray(planes, np.float32))

    def conv_bn(x, conv, bn, pad):
        x = F.conv2d(x, p[conv + ".weight"], p.get(conv + ".bias"), padding=pad)
        return F.batch_norm(x, p[bn + ".running_mean"], p[bn + ".running_var"], p[bn + ".weight"], p[bn + ".bias"],
                            training=False, eps=1e-5)

    with torch.no_grad():
        x = torch.relu(conv_bn(x, "input_conv", "input_bn", 1))
        for i in range(desc.blocks):
            r = x
            y = torch.relu(conv_bn(x, f"blocks.{i}.0", f"blocks.{i}.1", 1))
            y = conv_bn(y, f"blocks.{i}.3", f"blocks.{i}.4", 1)
            x = torch.relu(y + r) if desc.residual else torch.relu(y)
        x = F.adaptive_avg_pool2d(x, (desc.pool, desc.pool))
        pol = torch.relu(conv_bn(x, "policy_conv", "policy_bn", 0)).reshape(x.shape[0], -1)
        pol = F.linear(pol, p["policy_fc.weight"], p["policy_fc.bias"])
        v = torch.relu(conv_bn(x, "value_conv", "value_bn", 0)).reshape(x.shape[0], -1)
        v = torch.relu(F.linear(v, p["value_fc1.weight"], p["value_fc1.bias"]))
        v = torch.tanh(F.linear(v, p["value_fc2.weight"], p["value_fc2.bias"]))
    return pol.numpy(), v.reshape(-1).numpy()


def softmax_policy(logits):
    """TorchNeuralNetwork::predictBatch softmax (torch_neural_network.cpp:296-316), per row."""
    out = np.empty_like(logits)
    for b in range(logits.shape[0]):
        row = logits[b]
        e = np.exp(row - row.max()).astype(np.float32)
        s = np.float32(0.0)
        for v in e:
            s = np.float32(s + v)
        out[b] = e / s if s > 0 else e
    return out


class Model:
    """Cached fp32 CPU model (weights unpacked once) for repeated single-state evaluations."""

    def __init__(self, desc, blob):
        self.desc = desc
        self.p = unpack(desc, blob)

    def __call__(self, planes):
        d, p = self.desc, self.p
        x = torch.from_numpy(np.ascontiguousarray(planes, np.float32))

        def conv_bn(x, conv, bn, pad):
            x = F.conv2d(x, p[conv + ".weight"], p.get(conv + ".bias"), padding=pad)
            return F.batch_norm(x, p[bn + ".running_mean"], p[bn + ".running_var"], p[bn + ".weight"],
                                p[bn + ".bias"], training=False, eps=1e-5)

        with torch.no_grad():
            x = torch.relu(conv_bn(x, "input_conv", "input_bn", 1))
            for i in range(d.blocks):
                r = x
                y = torch.relu(conv_bn(x, f"blocks.{i}.0", f"blocks.{i}.1", 1))
                y = conv_bn(y, f"blocks.{i}.3", f"blocks.{i}.4", 1)
                x = torch.relu(y + r) if d.residual else torch.relu(y)
            x = F.adaptive_avg_pool2d(x, (d.pool, d.pool))
            pol = torch.relu(conv_bn(x, "policy_conv", "policy_bn", 0)).reshape(x.shape[0], -1)
            pol = F.linear(pol, p["policy_fc.weight"], p["policy_fc.bias"])
            v = torch.relu(conv_bn(x, "value_conv", "value_bn", 0)).reshape(x.shape[0], -1)
            v = torch.relu(F.linear(v, p["value_fc1.weight"], p["value_fc1.bias"]))
            v = torch.tanh(F.linear(v, p["value_fc2.weight"], p["value_fc2.bias"]))
        return pol.numpy(), v.reshape(-1).numpy()
