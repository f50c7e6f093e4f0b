"""Network parity on weights scaled like a trained net's outputs (VERDICT r01 'What's weak' 1):
the counter-based init gives |logit| <= 0.4, where an absolute error bound says little.  Here the
policy FC (weight + bias) is scaled so the largest |logit| over the test positions is 8, and the
value FC2 so the largest |pre-tanh value| is 1.5 (|value| ~ 0.9): the heads carry the magnitudes
a trained AlphaZero net emits while the trunk keeps the same activations.

Tolerance (BASELINE.json north_star, 1e-4 absolute on logits and value):
  * AZ_PREC_F32 and AZ_PREC_F16X3 (the parity precisions: exact fp32 products, and fp16 hi + lo
    pieces carrying 22 significant bits) must hold it;
  * AZ_PREC_BF16X3 (bf16 hi + lo pieces: 16-17 significant bits, the full fp32 range -- the
    precision for nets whose activations leave the fp16 range) holds it on trained-scale heads, and
    on trained-like trunks is held to 2.5e-5 of the largest logit (C5's 20-block trunk reaches
    1.4e-4 at |logit| 8: the bf16 pieces' own representation error, reproduced by a CPU emulation
    of the same arithmetic);
  * AZ_PREC_FP16 (the throughput precision, the reference's useFp16) cannot at this scale -- its
    operands carry 11 significant bits, so the error grows with the logit scale; it is held to a
    bound relative to the largest logit (3e-4) and the measured figures are printed."""
import numpy as np
import pytest

TOL = 1e-4
FP16_REL = 3e-4
BF16X3_REL = 2.5e-5     # AZ_PREC_BF16X3 on trained-like trunks, relative to the largest logit
PRECS = {"f16x3": 4, "bf16x3": 1, "fp16": 3}


@pytest.fixture(scope="module")
def engine():
    import az_amd
    return az_amd.Engine(0)


def _offsets(desc):
    import net_oracle
    off, out = 0, {}
    for name, shape, _, _ in net_oracle.param_shapes(desc):
        n = int(np.prod(shape))
        out[name] = (off, n)
        off += n
    return out


def trained_scale_blob(desc, seed, x, logit_max=8.0, value_pre_max=1.5):
    """init_blob with the policy FC and value FC2 rescaled (see module docstring)."""
    import net_oracle
    blob = net_oracle.init_blob(desc, seed)
    rl, rv = net_oracle.forward(desc, blob, x)
    o = _offsets(desc)
    kp = logit_max / float(np.abs(rl).max())
    kv = value_pre_max / float(np.abs(np.arctanh(np.clip(rv, -0.999999, 0.999999))).max())
    for name, k in (("policy_fc.weight", kp), ("policy_fc.bias", kp), ("value_fc2.weight", kv),
                    ("value_fc2.bias", kv)):
        a, n = o[name]
        blob[a:a + n] *= np.float32(k)
    return blob


def trunk_scaled_blob(desc, seed, x, act_max=64.0, spread=4.0, logit_max=8.0, value_pre_max=1.5):
    """init_blob reshaped like a TRAINED trunk, not only trained heads: every
    BN of the trunk gets per-channel output scales drawn log-uniform in [1/spread, spread] (channel
    magnitudes a decade or two apart, so every dot product mixes large and small terms), and each
    block's second BN a global gain calibrated on the fp32 network so that the largest activation
    after block i grows geometrically from 4 to `act_max` over the trunk (O(10-100), the range of a
    trained AlphaZero trunk; the init weights stay near 1-2).  Then the heads as trained_scale_blob
    (|logit|max = logit_max, |pre-tanh value| = value_pre_max).  Returns (blob, largest trunk activation)."""
    import torch
    import torch.nn.functional as Fn
    import net_oracle
    blob = net_oracle.init_blob(desc, seed)
    o = _offsets(desc)
    rng = np.random.default_rng(seed + 7)
    C = desc.channels
    xt = torch.from_numpy(np.ascontiguousarray(x, np.float32))

    def scale_bn(name, k):
        for f in ("weight", "bias"):
            a, n = o[f"{name}.{f}"]
            blob[a:a + n] *= np.asarray(k, np.float32)

    def conv_bn(h, conv, bn, pad):
        p = net_oracle.unpack(desc, blob)
        h = Fn.conv2d(h, p[conv + ".weight"], p.get(conv + ".bias"), padding=pad)
        return Fn.batch_norm(h, p[bn + ".running_mean"], p[bn + ".running_var"], p[bn + ".weight"], p[bn + ".bias"],
                             training=False, eps=1e-5)

    spreadk = lambda: np.exp(rng.uniform(-np.log(spread), np.log(spread), C))
    targets = np.geomspace(4.0, act_max, desc.blocks + 1)
    amax = 0.0
    with torch.no_grad():
        scale_bn("input_bn", spreadk())
        h = torch.relu(conv_bn(xt, "input_conv", "input_bn", 1))
        scale_bn("input_bn", np.full(C, targets[0] / float(h.max())))
        h = torch.relu(conv_bn(xt, "input_conv", "input_bn", 1))
        amax = float(h.max())
        for i in range(desc.blocks):
            scale_bn(f"blocks.{i}.1", spreadk())
            scale_bn(f"blocks.{i}.4", spreadk())
            y = torch.relu(conv_bn(h, f"blocks.{i}.0", f"blocks.{i}.1", 1))
            z = conv_bn(y, f"blocks.{i}.3", f"blocks.{i}.4", 1)
            for _ in range(4):                     # gain g on the block's branch: max relu(g z + h) -> target
                cur = float(torch.relu(z + h).max()) if desc.residual else float(torch.relu(z).max())
                g = targets[i + 1] / max(cur, 1e-6)
                scale_bn(f"blocks.{i}.4", np.full(C, g))
                z = z * g
            h = torch.relu(z + h) if desc.residual else torch.relu(z)
            amax = max(amax, float(h.max()), float(y.max()))
    rl, rv = net_oracle.forward(desc, blob, x)
    kp = logit_max / float(np.abs(rl).max())
    kv = value_pre_max / float(np.abs(np.arctanh(np.clip(rv, -0.999999, 0.999999))).max())
    for name, k in (("policy_fc.weight", kp), ("policy_fc.bias", kp), ("value_fc2.weight", kv),
                    ("value_fc2.bias", kv)):
        a, n = o[name]
        blob[a:a + n] *= np.float32(k)
    return blob, amax


def _planes(shape, B, seed):
    rng = np.random.default_rng(seed)
    if shape == "c3" or shape == "c2":
        import az_oracle as O
        out = np.zeros((B, 11, 15, 15), np.float32)
        for b in range(B):
            k = int(rng.integers(0, 75))
            out[b] = O.position(15, rng.permutation(225)[:k].tolist())[0]
        return out
    if shape == "c4":
        return (rng.random((B, 8, 19, 19)) < 0.3).astype(np.float32)
    return (rng.random((B, 111, 8, 8)) < 0.05).astype(np.float32)


NETS = {  # board, in_planes, channels, blocks, actions
    "c2": (15, 11, 64, 6, 225),
    "c3": (15, 11, 256, 20, 225),
    "c4": (19, 8, 256, 20, 362),
    "c5": (8, 111, 256, 20, 4672),
}


@pytest.mark.gpu
@pytest.mark.parametrize("prec", list(PRECS))
@pytest.mark.parametrize("shape", list(NETS))
def test_gpu_trained_scale_outputs(engine, shape, prec):
    import az_amd
    import net_oracle
    bs, ci, ch, blocks, A = NETS[shape]
    p = PRECS[prec]
    B = 16
    desc = az_amd.NetDesc(bs, ci, ch, blocks, A, 32, 8, 256, 1, 0, p, B)
    x = _planes(shape, B, seed=17)
    blob = trained_scale_blob(desc, 1234, x)
    net = az_amd.HipNeuralNetwork(engine, desc)
    net.load_weights(blob)
    lo, v = net.forward(x)
    rl, rv = net_oracle.forward(desc, blob, x)
    lmax = float(np.abs(rl).max())
    el, ev = float(np.abs(lo - rl).max()), float(np.abs(v - rv).max())
    print(f"{shape} {prec}: |logit|max {lmax:.3f} |value|max {np.abs(rv).max():.3f}  max|dlogit|={el:.3e} "
          f"({el / lmax:.2e} of |logit|max) max|dvalue|={ev:.3e}")
    assert 7.9 < lmax < 8.1
    if prec == "fp16":
        assert el <= FP16_REL * lmax and ev <= FP16_REL
    else:
        assert el <= TOL and ev <= TOL
    net.close()


@pytest.mark.gpu
@pytest.mark.parametrize("prec", ["f16x3", "bf16x3"])
@pytest.mark.parametrize("shape,B", [("c4", 1024), ("c5", 1024)])
def test_gpu_trained_scale_production_batch_x3(engine, shape, B, prec):
    """The split precisions at the BASELINE configs' production batch (C4 / C5: 1024 boards per
    forward, the batch the self-play search hands the net), trained-scale heads: 16 sampled boards
    (first, last, and 14 in between) against the fp32 oracle within the north-star 1e-4.  (C3's
    2048-board batch: tests/test_gpu_selfplay_net.py::test_gpu_c3_full_size_replay_x3.)"""
    import az_amd
    import net_oracle
    bs, ci, ch, blocks, A = NETS[shape]
    desc = az_amd.NetDesc(bs, ci, ch, blocks, A, 32, 8, 256, 1, 0, PRECS[prec], B)
    x = _planes(shape, B, seed=29)
    pick = np.unique(np.concatenate([[0, B - 1], np.random.default_rng(5).choice(B, 14, replace=False)]))
    blob = trained_scale_blob(desc, 4321, x[pick])
    net = az_amd.HipNeuralNetwork(engine, desc)
    net.load_weights(blob)
    lo, v = net.forward(x)
    rl, rv = net_oracle.forward(desc, blob, x[pick])
    lmax = float(np.abs(rl).max())
    el, ev = float(np.abs(lo[pick] - rl).max()), float(np.abs(v[pick] - rv).max())
    print(f"{shape} {prec} B={B}: |logit|max {lmax:.3f} max|dlogit|={el:.3e} max|dvalue|={ev:.3e}")
    assert 7.9 < lmax < 8.1
    assert el <= TOL and ev <= TOL
    net.close()


# the BASELINE configs' batch per forward: N = 1 (C2 256, C3 2048, C4 / C5 1024) and the per-rank
# shards of the multi-GPU configs (python/scripts/orchestrate_selfplay.py:303-311 splits the games over
# the GPUs): C3 at N = 8 (256 games per GPU), C4 / C5 at N = 8 (128) and C4 at N = 4 (256).  The shard
# batches take other kernels: fp16 15x15 below 1024 boards conv3x3_v6, 19x19 / 8x8 below 1024 boards the
# small-tile conv3x3_v7 (192 / 64-row tiles); F16X3 conv3x3_v9x3 with less than one round of blocks.
PROD_B = [("c2", 256), ("c3", 2048), ("c4", 1024), ("c5", 1024),
          ("c3", 256), ("c4", 128), ("c4", 256), ("c5", 128)]
SHARD_KERNEL = {("c3", 256, "fp16"): "conv3x3_v6<2, 15>", ("c4", 128, "fp16"): "conv3x3_v7<2, 19, DENSE, 128, 3>",
                ("c4", 256, "fp16"): "conv3x3_v7<2, 19, DENSE, 128, 3>", ("c5", 128, "fp16"): "conv3x3_v7<2, 8, DENSE, 64>",
                ("c3", 256, "f16x3"): "conv3x3_v9x3<15, SLIM, f16>", ("c4", 128, "f16x3"): "conv3x3_v9x3<19, DENSE, f16>",
                ("c5", 128, "f16x3"): "conv3x3_v9x3<8, DENSE, f16>"}


@pytest.mark.gpu
@pytest.mark.parametrize("prec", list(PRECS))
@pytest.mark.parametrize("shape,B", PROD_B, ids=[f"{s}-B{b}" for s, b in PROD_B])
def test_gpu_trunk_scaled_production_batch(engine, shape, B, prec):
    """A trained-like TRUNK (trunk_scaled_blob: per-channel BN scales a decade apart, activations
    growing to O(64) through the blocks) plus trained-scale heads, at each config's production batch
    (C2 256 on k_smallnet_x3, C3 2048, C4 / C5 1024 on conv3x3_v9x3) and at the per-rank shard batches
    of the multi-GPU configs (C3 256, C4 128 / 256, C5 128): 16 sampled boards (first, last, 14
    between) against the fp32 oracle on RAW logits and values.  f16x3 must hold the north-star
    1e-4; bf16x3 (16-17 significant bits) is held to BF16X3_REL of the largest logit; fp16's error is
    reported (its 11-bit operands cannot hold 1e-4 at |logit| 8) and bounded relative to the
    largest logit."""
    import az_amd
    import net_oracle
    bs, ci, ch, blocks, A = NETS[shape]
    p = PRECS[prec]
    desc = az_amd.NetDesc(bs, ci, ch, blocks, A, 32, 8, 256, 1, 0, p, B)
    x = _planes(shape, B, seed=31)
    pick = np.unique(np.concatenate([[0, B - 1], np.random.default_rng(6).choice(B, 14, replace=False)]))
    blob, amax = trunk_scaled_blob(desc, 2468, x[pick])
    net = az_amd.HipNeuralNetwork(engine, desc)
    if (shape, B, prec) in SHARD_KERNEL:
        assert net.trunk_kernel() == SHARD_KERNEL[(shape, B, prec)]
    net.load_weights(blob)
    lo, v = net.forward(x)
    rl, rv = net_oracle.forward(desc, blob, x[pick])
    lmax = float(np.abs(rl).max())
    el, ev = float(np.abs(lo[pick] - rl).max()), float(np.abs(v[pick] - rv).max())
    print(f"{shape} {prec} B={B} [{net.trunk_kernel()}] trunk-scaled (max activation {amax:.1f}): |logit|max {lmax:.3f} "
          f"max|dlogit|={el:.3e} ({el / lmax:.2e} of |logit|max) max|dvalue|={ev:.3e}")
    assert amax > 30.0 and 7.9 < lmax < 8.1
    if prec == "fp16":
        assert el <= 2e-3 * lmax and ev <= 2e-3
    elif prec == "bf16x3":
        assert el <= BF16X3_REL * lmax and ev <= TOL
    else:
        assert el <= TOL and ev <= TOL
    net.close()


OVF_CASES = [  # (board, in_planes, channels, blocks, actions, B, conv flags, precision): every fp16 kernel
    (15, 11, 64, 2, 225, 8, 0x204, "fp16"),       # k_smallnet_g (C2 shape)
    (15, 11, 256, 2, 225, 8, 0x204, "fp16"),      # conv3x3_v6 (below 1024 boards)
    (15, 11, 256, 2, 225, 8, 0xa04, "fp16"),      # conv3x3_v7 (flag 0x800 forces it at any batch)
    (19, 8, 256, 2, 362, 4, 0x204, "fp16"),       # conv3x3_v6 DENSE (Go)
    (15, 11, 64, 2, 225, 8, 0x204, "f16x3"),      # k_smallnet_x3<15, 8, true, 2>
    (15, 11, 256, 2, 225, 8, 0x204, "f16x3"),     # conv3x3_v9x3 SLIM, fp16 pieces (+ k_to_g8x3<2>)
    (15, 11, 128, 2, 225, 8, 0x204, "f16x3"),     # conv3x3_v7x3 SLIM, fp16 pieces (N = 128)
    (19, 8, 256, 2, 362, 4, 0x204, "f16x3"),      # conv3x3_v9x3 DENSE, fp16 pieces
]


@pytest.mark.gpu
@pytest.mark.parametrize("case", OVF_CASES, ids=[str(c) for c in OVF_CASES])
def test_gpu_fp16_overflow_fails_loudly(engine, case):
    """The fp16 range guard: a trunk whose activations exceed the fp16 range (65504) must not
    return silently wrong outputs -- the forward fails with AZ_ERR_RANGE (AzError) -- while the same
    trunk at O(64) activations runs, the flag is cleared after it is reported, and the parity
    bf16-piece precision (bf16x3) takes the overflowing trunk within 1e-4."""
    import az_amd
    import net_oracle
    from az_amd import _lib
    bs, ci, ch, blocks, A, B, fl, prec = case
    shape = "c4" if bs == 19 else "c3"
    x = _planes(shape, B, seed=3)
    try:
        _lib.lib().az_diag_set_conv_flags(fl)
        for act_max, ok in ((64.0, True), (3.0e5, False), (64.0, True)):
            desc = az_amd.NetDesc(bs, ci, ch, blocks, A, 32, 8, 256, 1, 0, PRECS[prec], B)
            blob, amax = trunk_scaled_blob(desc, 99, x, act_max=act_max)
            net = az_amd.HipNeuralNetwork(engine, desc)
            net.load_weights(blob)
            if ok:
                lo, v = net.forward(x)
                assert np.isfinite(lo).all() and np.isfinite(v).all()
            else:
                with pytest.raises(az_amd.AzError, match="fp16 activation overflow") as ei:
                    net.forward(x)
                assert ei.value.code == _lib.AZ_ERR_RANGE and amax > 65504
                with pytest.raises(az_amd.AzError, match="fp16 activation overflow"):
                    net.forward(x)                       # every overflowing forward is reported
                dx = az_amd.NetDesc(bs, ci, ch, blocks, A, 32, 8, 256, 1, 0, az_amd.AZ_PREC_BF16X3, B)
                n3 = az_amd.HipNeuralNetwork(engine, dx)
                n3.load_weights(blob)
                l3, v3 = n3.forward(x)
                rl, rv = net_oracle.forward(dx, blob, x)
                assert np.abs(l3 - rl).max() <= TOL and np.abs(v3 - rv).max() <= TOL
                n3.close()
            net.close()
    finally:
        _lib.lib().az_diag_set_conv_flags(0x204)
