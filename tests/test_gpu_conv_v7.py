"""conv3x3_v7 (csrc/conv_v7.hip: two 256-thread blocks per CU, swapped MFMA operands, epilogue from
registers; the default for batches of >= 1024 boards on 15x15) against conv3x3_v6 (csrc/conv_bf16.hip): same products in the same accumulation order,
so every output of the whole network must be BITWISE equal -- on the SLIM and padded 15x15 tiles, on DENSE
tiles of every board, for ragged batches and in both 16-bit modes.  Both kernels are also pinned to
the fp32 reference by tests/test_gpu_net.py (v7 is the default kernel there)."""
import numpy as np
import pytest


@pytest.fixture(scope="module")
def engine():
    import az_amd
    return az_amd.Engine(0)


def _flags(f):
    from az_amd import _lib
    _lib.lib().az_diag_set_conv_flags(int(f))


def _poison(byte):
    """az_diag_set_poison: every activation / workspace buffer of a net is filled with `byte` before
    each forward (-1: off), so a read of memory the forward never wrote shows up as a bitwise change"""
    from az_amd import _lib
    _lib.lib().az_diag_set_poison(int(byte))


CASES = [  # board, in_planes, actions, channels, blocks, B, flags selecting v7 (v6 = flags | 0x100)
    (15, 11, 225, 256, 2, 37, 0xa04),     # SLIM 15x16 tile (the default), ragged batch
    (15, 11, 225, 256, 1, 1, 0xa04),      # a single board
    (15, 11, 225, 128, 2, 64, 0xa04),     # 128 channels (one channel half)
    (15, 11, 225, 256, 2, 37, 0xe04),     # padded 15x17 tile
    (15, 11, 225, 256, 2, 37, 0xa0c),     # DENSE 15x15 tiles
    (19, 8, 362, 256, 2, 13, 0x804),      # DENSE 19x19 (Go)
    (9, 11, 81, 128, 2, 29, 0x804),       # DENSE 9x9
    (13, 8, 170, 256, 1, 7, 0x804),       # DENSE 13x13
    (8, 111, 4672, 256, 2, 33, 0x804),    # DENSE 8x8 chess: the 128-channel input conv runs on v7 too
    # small-batch DENSE tiles (conv flag bits 0x70000 force the tile rows: 1 = 256, 2 = 128, 3 = 64,
    # 4 = 192; without them az_conv_v7_tm picks by the board and the launch's block count)
    (19, 8, 362, 256, 2, 13, 0x10804),    # 256-row tiles at a small batch
    (19, 8, 362, 256, 2, 13, 0x20804),    # 128-row tiles
    (19, 8, 362, 256, 2, 13, 0x30804),    # 64-row tiles
    (19, 8, 362, 256, 2, 13, 0x40804),    # 192-row tiles (two A register sets of 3 fragments)
    (8, 111, 4672, 256, 2, 33, 0x40804),  # 8x8, 192-row tiles
    (8, 111, 4672, 256, 2, 33, 0x20804),  # 8x8, 128-row tiles: tiles span 2 boards
    (15, 11, 225, 256, 2, 37, 0x20a0c),   # 15x15 DENSE, 128-row tiles
    (13, 8, 170, 256, 1, 7, 0x30804),     # 13x13, 64-row tiles (a tile holds < 1 board)
    (19, 8, 362, 256, 1, 130, 0x804),     # C4 shard-sized batch, the automatic choice
    # conv flag 0x80000: the 3-slot weight ring with three blocks per CU (128 / 64-row tiles)
    (19, 8, 362, 256, 2, 13, 0xa0804),    # 128-row tiles, 3-slot ring
    (8, 111, 4672, 256, 2, 33, 0xb0804),  # 8x8, 64-row tiles, 3-slot ring
    (13, 8, 170, 256, 1, 7, 0xb0804),     # 13x13, 64-row tiles (a tile holds < 1 board), 3-slot ring
    (19, 8, 362, 256, 1, 130, 0xa0804),   # C4 shard-sized batch, 128-row tiles, 3-slot ring
    # several blocks per CU over several rounds (LDS contention: a fragment read still in flight at
    # the loop exit used to land in a reused register -- tools/lds_hazards.py; these gave wrong
    # boards or an illegal address before the drains)
    (19, 8, 362, 256, 1, 130, 0x20804),   # 128-row tiles, two blocks per CU
    (8, 111, 4672, 256, 1, 1024, 0x20804),  # 8x8, 128-row tiles, 1024 boards
    (13, 8, 170, 256, 1, 400, 0x804),     # 13x13 at 400 boards: the automatic choice (128-row tiles)
    (9, 11, 81, 256, 1, 700, 0x804),      # 9x9 at 700 boards: the automatic choice (128-row tiles)
    (19, 8, 362, 256, 1, 400, 0x30804),   # 64-row tiles, three blocks per CU
    (8, 111, 4672, 256, 1, 512, 0x804),   # 8x8 at 512 boards: the automatic 128-row tiles on the 3-slot ring
    (19, 8, 362, 256, 1, 256, 0x804),     # the C4 N = 4 shard: 128-row tiles, 3-slot ring, two rounds
]


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["fp16", "bf16"])
@pytest.mark.parametrize("case", CASES, ids=[str(c) for c in CASES])
def test_gpu_v7_bitwise_equals_v6(engine, case, mode):
    import az_amd
    import net_oracle
    bs, ci, A, ch, blocks, B, fl = case
    prec = az_amd.AZ_PREC_FP16 if mode == "fp16" else az_amd.AZ_PREC_BF16
    desc = az_amd.NetDesc(bs, ci, ch, blocks, A, 32, 8, 256, 1, 0, prec, B)
    net = az_amd.HipNeuralNetwork(engine, desc)
    net.load_weights(net_oracle.init_blob(desc, seed=31))
    rng = np.random.default_rng(bs * 7 + B)
    x = (rng.random((B, ci, bs, bs)) < (0.05 if ci > 16 else 0.25)).astype(np.float32)
    # v6 and v7 each run under two poisons (NaN bytes, then 0x55) and v7 once clean: a kernel that
    # reads activation / remainder / workspace memory its forward never wrote cannot pass
    outs = {}
    try:
        for name, f, byte in (("v6/ff", fl | 0x100, 0xff), ("v6/55", fl | 0x100, 0x55),
                              ("v7/ff", fl, 0xff), ("v7/55", fl, 0x55), ("v7", fl, -1)):
            _flags(f)
            _poison(byte)
            outs[name] = net.forward(x)
    finally:
        _poison(-1)
        _flags(0x204)                     # the library default
    l6, v6 = outs["v6/ff"]
    for name, (l7, v7) in outs.items():
        bad = np.where((l7 != l6).any(axis=1) | (v7 != v6))[0]
        print(f"{case} {mode} {name}: max|. - v6| logits {np.abs(l7 - l6).max():.3e} value {np.abs(v7 - v6).max():.3e}, "
              f"boards differing {bad.tolist()[:16]} of {B}")
    for name, (l7, v7) in outs.items():
        assert np.isfinite(l7).all() and np.isfinite(v7).all(), name
        assert np.array_equal(l7, l6) and np.array_equal(v7, v6), name
    net.close()


X3W_CASES = [  # board, in_planes, actions, channels, blocks, residual, B: conv3x3_v9x3 geometries (N % 256 == 0)
    (15, 11, 225, 256, 2, 1, 37),     # SLIM tile, ragged batch
    (15, 11, 225, 256, 1, 1, 1),      # a single board
    (15, 11, 225, 256, 2, 0, 5),      # plain stack (no residual planes)
    (19, 8, 362, 256, 2, 1, 13),      # DENSE 19x19 (Go), tiles spanning boards
    (9, 11, 81, 256, 1, 1, 29),       # DENSE 9x9
    (13, 8, 170, 256, 1, 1, 7),       # DENSE 13x13
    (8, 111, 4672, 256, 2, 1, 33),    # DENSE 8x8 chess shape
    (15, 11, 225, 512, 1, 1, 3),      # two 256-channel output blocks per tile
]


V9_VARIANTS = [0x204, 0x20000204, 0x40000204, 0x60000204]   # default; tap-start barrier; no fragment skip; both


@pytest.mark.gpu
@pytest.mark.parametrize("prec", ["bf16x3", "f16x3"])
@pytest.mark.parametrize("case", X3W_CASES, ids=[str(c) for c in X3W_CASES])
def test_gpu_v9x3_bitwise_equals_v7x3(engine, case, prec):
    """conv3x3_v9x3 (one 512-thread block per CU owning all 256 output channels of a tile) gives
    every accumulator the same products in the same order as conv3x3_v7x3 (Bh*Ah, Bl*Ah, Bh*Al per
    tap), so the whole split-precision network must be BITWISE equal on every geometry and batch
    shape, for bf16 pieces (and every v9x3 A/B variant) and fp16 pieces (the default variant)."""
    import az_amd
    import net_oracle
    bs, ci, A, ch, blocks, res, B = case
    p = {"bf16x3": az_amd.AZ_PREC_BF16X3, "f16x3": az_amd.AZ_PREC_F16X3}[prec]
    desc = az_amd.NetDesc(bs, ci, ch, blocks, A, 32, 8, 256, res, 0, p, B)
    net = az_amd.HipNeuralNetwork(engine, desc)
    assert net.trunk_kernel().startswith("conv3x3_v9x3<")
    net.load_weights(net_oracle.init_blob(desc, seed=57))
    rng = np.random.default_rng(bs * 11 + B)
    x = (rng.random((B, ci, bs, bs)) < (0.05 if ci > 16 else 0.25)).astype(np.float32)
    try:
        _flags(0x10000204)                # conv3x3_v7x3
        _poison(0xff)
        l7, v7 = net.forward(x)
        outs = {}
        for fl in (V9_VARIANTS if prec == "bf16x3" else V9_VARIANTS[:1]):   # 0x204: the library default
            _flags(fl)
            _poison(0x55)
            outs[fl] = net.forward(x)
        _poison(-1)
        outs["clean"] = net.forward(x)
    finally:
        _poison(-1)
        _flags(0x204)
    for fl, (l9, v9) in outs.items():
        print(f"{case} flags {fl}: max|v9x3 - v7x3| logits {np.abs(l9 - l7).max():.3e} value {np.abs(v9 - v7).max():.3e}")
        assert np.isfinite(l9).all() and np.abs(l9).max() > 0
        assert np.array_equal(l9, l7) and np.array_equal(v9, v7), fl
    net.close()
