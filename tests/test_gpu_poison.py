"""Read-before-write check of every production forward routing.

az_diag_set_poison(byte) fills every activation, remainder, workspace and input buffer of a net
with `byte` before each forward (the zeroed halo tails and the weights excepted).  A kernel that
reads memory its forward never wrote -- a halo row past the last board, a remainder plane a
previous net left behind, a split-K slice no block wrote -- then returns a result that depends on
the byte.  Each routing below runs clean, under 0xff (NaN in every float format, -1 in int8) and
under 0x55, and all three must be bitwise equal.

The routings are the ones production takes (net_forward / g8_choice / az_conv_v7_tm at the
capacity of the net): the per-rank shard batches of the 8-GPU configs (C3 256 boards of 15x15, C4
128 of 19x19, C5 128 of 8x8) and the N = 1 batches, in the throughput (fp16) and parity (F16X3)
precisions, plus the C2 fused small net."""
import numpy as np
import pytest

PREC = {"f32": 0, "bf16x3": 1, "bf16": 2, "fp16": 3, "f16x3": 4}

CASES = [  # board, in_planes, actions, channels, blocks, B, precision, trunk kernel it must take
    (15, 11, 225, 256, 2, 1024, "fp16", "conv3x3_v7<2, 15, SLIM>"),
    (15, 11, 225, 256, 2, 256, "fp16", "conv3x3_v6<2, 15>"),
    (15, 11, 225, 256, 2, 256, "f16x3", "conv3x3_v9x3<15, SLIM, f16>"),
    (19, 8, 362, 256, 2, 1024, "fp16", "conv3x3_v6<2, 19, DENSE>"),
    (19, 8, 362, 256, 2, 128, "fp16", "conv3x3_v7<2, 19, DENSE, 128, 3>"),
    (19, 8, 362, 256, 2, 130, "bf16", "conv3x3_v7<1, 19, DENSE, 128, 3>"),
    (19, 8, 362, 256, 2, 128, "f16x3", "conv3x3_v9x3<19, DENSE, f16>"),
    (8, 111, 4672, 256, 2, 128, "fp16", "conv3x3_v7<2, 8, DENSE, 64>"),
    (8, 111, 4672, 256, 2, 128, "f16x3", "conv3x3_v9x3<8, DENSE, f16>"),
    (15, 11, 225, 64, 6, 256, "fp16", "k_smallnet_g<15, 8, true>"),
    (15, 11, 225, 64, 6, 256, "f16x3", "k_smallnet_x3<15, 8, true, 2>"),
    (9, 11, 81, 64, 2, 130, "f32", "gemm_f32"),
]


@pytest.fixture(scope="module")
def engine():
    import az_amd
    return az_amd.Engine(0)


def _poison(byte):
    from az_amd import _lib
    _lib.lib().az_diag_set_poison(int(byte))


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=[f"{c[0]}x{c[0]}-{c[3]}ch-B{c[5]}-{c[6]}" for c in CASES])
def test_gpu_forward_reads_only_what_it_wrote(engine, case):
    import az_amd
    import net_oracle
    bs, ci, A, ch, blocks, B, prec, kernel = case
    desc = az_amd.NetDesc(bs, ci, ch, blocks, A, 32, 8, 256, 1, 0, PREC[prec], B)
    net = az_amd.HipNeuralNetwork(engine, desc)
    assert net.trunk_kernel() == kernel
    net.load_weights(net_oracle.init_blob(desc, seed=77))
    rng = np.random.default_rng(bs * 13 + B)
    x = (rng.random((B, ci, bs, bs)) < (0.05 if ci > 16 else 0.25)).astype(np.float32)
    outs = {}
    try:
        for byte in (0xff, 0x55, -1):
            _poison(byte)
            outs[byte] = net.forward(x)
    finally:
        _poison(-1)
    lc, vc = outs[-1]
    assert np.isfinite(lc).all() and np.isfinite(vc).all() and np.abs(lc).max() > 0
    for byte, (l, v) in outs.items():
        bad = np.where((l != lc).any(axis=1) | (v != vc))[0]
        print(f"{case} poison {byte:#x}: max|d logit| {np.abs(l - lc).max():.3e}, boards differing {bad.tolist()[:16]}")
        assert np.array_equal(l, lc) and np.array_equal(v, vc), byte
    net.close()
