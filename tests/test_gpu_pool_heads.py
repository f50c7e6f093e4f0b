"""k_pool_heads_g8 (csrc/conv_bf16.hip): the trunk's tail -- adaptive average pool of the g8 trunk
output and both head 1x1 convs -- in one launch.  It must be BITWISE what the two-launch tail gives
(k_pool_g8 + gemm_f32<64>: same pooling order, same v_mfma_f32_32x32x2_f32 chain over k), which conv
flag 0x400000 selects: every logit and value of the whole network is compared, in every trunk
precision that runs on the g8 planes, on every board size, at ragged and production batches."""
import numpy as np
import pytest

PREC = {"bf16": 2, "fp16": 3, "bf16x3": 1, "f16x3": 4}

CASES = [  # board, in_planes, actions, channels, blocks, B, precision
    (15, 11, 225, 256, 2, 37, "fp16"),      # C3 shape, ragged batch
    (15, 11, 225, 256, 1, 1, "bf16"),       # a single board
    (15, 11, 225, 256, 2, 2048, "fp16"),    # the C3 production batch
    (15, 11, 225, 256, 1, 64, "f16x3"),     # the parity precision (conv3x3_v9x3 trunk, lo planes)
    (15, 11, 225, 256, 1, 13, "bf16x3"),
    (19, 8, 362, 256, 2, 128, "fp16"),      # the C4 per-rank shard
    (19, 8, 362, 256, 1, 130, "f16x3"),
    (9, 11, 81, 256, 1, 29, "fp16"),        # pool windows of 2 (9 -> 8)
    (13, 8, 170, 256, 1, 400, "bf16"),
    (8, 111, 4672, 256, 1, 128, "fp16"),    # the C5 net: 8 -> 8, windows of 1
]


@pytest.fixture(scope="module")
def engine():
    import az_amd
    return az_amd.Engine(0)


def _flags(f):
    from az_amd import _lib
    _lib.lib().az_diag_set_conv_flags(int(f))


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=[f"{c[0]}x{c[0]}-B{c[5]}-{c[6]}" for c in CASES])
def test_gpu_fused_tail_bitwise(engine, case):
    import az_amd
    import net_oracle
    bs, ci, A, ch, blocks, B, prec = case
    desc = az_amd.NetDesc(bs, ci, ch, blocks, A, 32, 8, 256, 1, 0, PREC[prec], B)
    net = az_amd.HipNeuralNetwork(engine, desc)
    net.load_weights(net_oracle.init_blob(desc, seed=23))
    rng = np.random.default_rng(bs * 11 + B)
    x = (rng.random((B, ci, bs, bs)) < (0.05 if ci > 16 else 0.25)).astype(np.float32)
    try:
        _flags(0x204)
        lf, vf = net.forward(x)                 # the fused tail (library default)
        _flags(0x204 | 0x400000)
        ls, vs = net.forward(x)                 # k_pool_g8 + gemm_f32
    finally:
        _flags(0x204)
    bad = np.where((lf != ls).any(axis=1) | (vf != vs))[0]
    print(f"{case}: max|dlogit| {np.abs(lf - ls).max():.3e} max|dvalue| {np.abs(vf - vs).max():.3e}, "
          f"boards differing {bad.tolist()[:16]}")
    assert np.isfinite(lf).all() and np.abs(lf).max() > 0
    assert np.array_equal(lf, ls) and np.array_equal(vf, vs)
    net.close()
