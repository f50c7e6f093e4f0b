"""Network parity on weights scaled like a trained net's outputs (VERDICT r01 'What's weak' 1):
the counter-based init gives |logit| <= 0.4, where an absolute error bound says little.  Here the
policy FC (weight + bias) is scaled so the largest |logit| over the test positions is 8, and the
value FC2 so the largest |pre-tanh value| is 1.5 (|value| ~ 0.9): the heads carry the magnitudes
a trained AlphaZero net emits while the trunk keeps the same activations.

Tolerance (BASELINE.json north_star, 1e-4 absolute on logits and value):
  * AZ_PREC_F32 and AZ_PREC_BF16X3 (the parity precisions) must hold it;
  * AZ_PREC_FP16 (the throughput precision, the reference's useFp16) cannot at this scale -- its
    operands carry 11 significant bits, so the error grows with the logit scale; it is held to a
    bound relative to the largest logit (3e-4) and the measured figures are printed."""
import numpy as np
import pytest

TOL = 1e-4
FP16_REL = 3e-4


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
@pytest.mark.parametrize("prec", ["bf16x3", "fp16"])
@pytest.mark.parametrize("shape", list(NETS))
def test_gpu_trained_scale_outputs(engine, shape, prec):
    import az_amd
    import net_oracle
    bs, ci, ch, blocks, A = NETS[shape]
    p = {"bf16x3": az_amd.AZ_PREC_BF16X3, "fp16": az_amd.AZ_PREC_FP16}[prec]
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
@pytest.mark.parametrize("shape,B", [("c4", 1024), ("c5", 1024)])
def test_gpu_trained_scale_production_batch_bf16x3(engine, shape, B):
    """The parity precision at the BASELINE configs' production batch (C4 / C5: 1024 boards per
    forward, the batch the self-play search hands the net), trained-scale heads: 16 sampled boards
    (first, last, and 14 in between) against the fp32 oracle within the north-star 1e-4.  (C3's
    2048-board batch: tests/test_gpu_selfplay_net.py::test_gpu_c3_full_size_replay_bf16x3.)"""
    import az_amd
    import net_oracle
    bs, ci, ch, blocks, A = NETS[shape]
    desc = az_amd.NetDesc(bs, ci, ch, blocks, A, 32, 8, 256, 1, 0, az_amd.AZ_PREC_BF16X3, B)
    x = _planes(shape, B, seed=29)
    pick = np.unique(np.concatenate([[0, B - 1], np.random.default_rng(5).choice(B, 14, replace=False)]))
    blob = trained_scale_blob(desc, 4321, x[pick])
    net = az_amd.HipNeuralNetwork(engine, desc)
    net.load_weights(blob)
    lo, v = net.forward(x)
    rl, rv = net_oracle.forward(desc, blob, x[pick])
    lmax = float(np.abs(rl).max())
    el, ev = float(np.abs(lo[pick] - rl).max()), float(np.abs(v[pick] - rv).max())
    print(f"{shape} bf16x3 B={B}: |logit|max {lmax:.3f} max|dlogit|={el:.3e} max|dvalue|={ev:.3e}")
    assert 7.9 < lmax < 8.1
    assert el <= TOL and ev <= TOL
    net.close()
