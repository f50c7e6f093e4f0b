"""GPU parity of the HIP ConvNet (through the C-ABI) against the fp32 PyTorch-CPU
restatement (oracle/net_oracle.py), itself pinned to the reference's Python classes
(tests/test_nn_golden.py).

Tolerance (BASELINE.json north_star): |logit - ref| <= 1e-4 and |value - ref| <= 1e-4
for the parity precisions (AZ_PREC_F32, AZ_PREC_F16X3, AZ_PREC_BF16X3) and the throughput
precision AZ_PREC_FP16 on init-scale weights (trained scale: tests/test_gpu_trained_scale.py).
Plain bf16 is a throughput variant and only gets a loose sanity bound."""
import numpy as np
import pytest

TOL = 1e-4
PREC = {"f32": 0, "bf16x3": 1, "bf16": 2, "fp16": 3, "f16x3": 4}


def f16x3_ok(bs, ch, blocks):
    """AZ_PREC_F16X3's kernels: conv3x3_v9x3 / v7x3 or the 15x15 64-channel k_smallnet_x3."""
    return (bs in (8, 9, 13, 15, 19) and ch % 128 == 0) or (bs == 15 and ch == 64 and blocks <= 15)


@pytest.fixture(scope="module")
def engine():
    import az_amd
    return az_amd.Engine(0)


def _planes(B, bs, seed):
    """Feature planes of random legal positions (0/1 stone planes, coords), like the search emits."""
    import az_oracle as O
    rng = np.random.default_rng(seed)
    out = np.zeros((B, 11, bs, bs), np.float32)
    for b in range(B):
        k = int(rng.integers(0, bs * bs // 3))
        moves = rng.permutation(bs * bs)[:k].tolist()
        out[b] = O.position(bs, moves)[0]
    return out


CASES = [  # (board, channels, blocks, residual, conv_bias, B)
    (15, 64, 6, 1, 0, 16),     # C2 net
    (15, 256, 20, 1, 0, 8),    # C3 net
    (15, 32, 3, 0, 0, 5),      # exporter fallback (plain stack)
    (8, 16, 2, 1, 1, 3),       # SimplifiedModel shape (pool 8x8 = identity)
    (9, 64, 2, 1, 0, 130),     # ragged batch (> one 128-row tile of samples)
]


@pytest.mark.gpu
@pytest.mark.parametrize("prec", ["f32", "f16x3", "bf16x3", "fp16"])
@pytest.mark.parametrize("case", CASES, ids=[str(c) for c in CASES])
def test_gpu_net_matches_fp32_reference(engine, case, prec):
    import az_amd
    import net_oracle
    bs, ch, blocks, res, bias, B = case
    p = PREC[prec]
    if p != az_amd.AZ_PREC_F32 and ch % 32:
        pytest.skip("bf16 trunk needs channels % 32 == 0")
    if p == az_amd.AZ_PREC_FP16 and (bs != 15 or ch % 64):
        pytest.skip("fp16 trunk: 15x15 boards, channels % 64 == 0")
    desc = az_amd.gomoku_net_desc(board_size=bs, channels=ch, blocks=blocks, residual=res, conv_bias=bias,
                                  precision=p, max_batch=B)
    if prec == "f16x3" and not f16x3_ok(bs, ch, blocks):
        with pytest.raises(az_amd.AzError, match="AZ_PREC_F16X3"):     # refused at creation, not run elsewhere
            az_amd.HipNeuralNetwork(engine, desc)
        return
    net = az_amd.HipNeuralNetwork(engine, desc)
    blob = net_oracle.init_blob(desc, seed=11)
    net.load_weights(blob)
    x = _planes(B, bs, seed=1)
    lo, v = net.forward(x)
    rl, rv = net_oracle.forward(desc, blob, x)
    err_l = float(np.abs(lo - rl).max())
    err_v = float(np.abs(v - rv).max())
    print(f"{case} {prec}: max|dlogit|={err_l:.3e} (|logit|max {np.abs(rl).max():.3f}) max|dvalue|={err_v:.3e}")
    assert err_l <= TOL and err_v <= TOL
    # predictBatch semantics: softmax over A
    pp, pv = net.predictBatch(x)
    assert np.abs(pp - net_oracle.softmax_policy(rl)).max() <= 1e-5
    assert np.array_equal(pv, v)
    net.close()


@pytest.mark.gpu
def test_gpu_net_bf16_sanity(engine):
    import az_amd
    import net_oracle
    desc = az_amd.gomoku_net_desc(board_size=15, channels=64, blocks=6, precision=az_amd.AZ_PREC_BF16, max_batch=8)
    net = az_amd.HipNeuralNetwork(engine, desc)
    blob = net_oracle.init_blob(desc, seed=11)
    net.load_weights(blob)
    x = _planes(8, 15, seed=2)
    lo, v = net.forward(x)
    rl, rv = net_oracle.forward(desc, blob, x)
    print("bf16 max|dlogit|", np.abs(lo - rl).max(), "max|dvalue|", np.abs(v - rv).max())
    assert np.abs(lo - rl).max() < 5e-2 * max(1.0, np.abs(rl).max())
    net.close()


@pytest.mark.gpu
@pytest.mark.parametrize("prec", [0, 1, 3, 4])
def test_gpu_net_batch_position_independent(engine, prec):
    """A sample's output does not depend on its position or batch-mates (bitwise)."""
    import az_amd
    import net_oracle
    desc = az_amd.gomoku_net_desc(board_size=15, channels=64, blocks=2, precision=prec, max_batch=40)
    net = az_amd.HipNeuralNetwork(engine, desc)
    net.load_weights(net_oracle.init_blob(desc, seed=5))
    x = _planes(40, 15, seed=3)
    lo, v = net.forward(x)
    perm = np.random.default_rng(0).permutation(40)
    lo2, v2 = net.forward(x[perm])
    assert np.array_equal(lo2, lo[perm]) and np.array_equal(v2, v[perm])
    lo3, v3 = net.forward(x[7:9])
    assert np.array_equal(lo3, lo[7:9]) and np.array_equal(v3, v[7:9])
    net.close()


@pytest.mark.gpu
def test_gpu_net_init_random_matches_numpy(engine):
    """az_net_init_random == oracle/net_oracle.init_blob (same counter-based generator)."""
    import az_amd
    import net_oracle
    desc = az_amd.gomoku_net_desc(board_size=9, channels=32, blocks=1, max_batch=4)
    a = az_amd.HipNeuralNetwork(engine, desc)
    a.init_random(77)
    b = az_amd.HipNeuralNetwork(engine, desc)
    b.load_weights(net_oracle.init_blob(desc, seed=77))
    x = _planes(4, 9, seed=4)
    la, va = a.forward(x)
    lb, vb = b.forward(x)
    assert np.array_equal(la, lb) and np.array_equal(va, vb)
    a.close()
    b.close()


@pytest.mark.gpu
@pytest.mark.parametrize("prec", ["f16x3", "bf16x3", "fp16"])
def test_gpu_c3_net_error_over_many_positions(engine, prec):
    """The C3 net (20 blocks x 256 filters) on 96 random positions: every logit and value
    within 1e-4 of the fp32 reference (the bench precisions)."""
    import az_amd
    import net_oracle
    p = PREC[prec]
    desc = az_amd.gomoku_net_desc(board_size=15, channels=256, blocks=20, precision=p, max_batch=96)
    net = az_amd.HipNeuralNetwork(engine, desc)
    blob = net_oracle.init_blob(desc, seed=1234)      # bench.py's weights
    net.load_weights(blob)
    x = _planes(96, 15, seed=7)
    lo, v = net.forward(x)
    rl, rv = net_oracle.forward(desc, blob, x)
    el, ev = float(np.abs(lo - rl).max()), float(np.abs(v - rv).max())
    print(f"C3 {prec}: max|dlogit|={el:.3e} max|dvalue|={ev:.3e} (|logit|max {np.abs(rl).max():.3f})")
    assert el <= TOL and ev <= TOL
    net.close()


X3_CASES = [  # (board, in_planes, action_size, channels, blocks, residual, B): conv3x3_v7x3 geometries
    (15, 11, 225, 128, 2, 1, 9),     # SLIM tile, one board per tile
    (15, 11, 225, 128, 2, 0, 3),     # plain stack (no residual planes)
    (19, 8, 362, 128, 2, 1, 5),      # Go: DENSE tiles spanning boards, ragged last tile
    (9, 11, 81, 256, 1, 1, 7),       # 9x9 DENSE, both channel halves
    (13, 8, 170, 128, 2, 1, 4),      # 13x13 DENSE
    (8, 111, 4672, 128, 1, 1, 6),    # Chess shape: the 111-plane input conv on the f32 GEMM
]


@pytest.mark.gpu
@pytest.mark.parametrize("prec", ["f16x3", "bf16x3"])
@pytest.mark.parametrize("case", X3_CASES, ids=[str(c) for c in X3_CASES])
def test_gpu_x3_trunk_geometries(engine, case, prec):
    """The split-precision trunks (AZ_PREC_F16X3 / BF16X3 on conv3x3_v7x3 / v9x3, g8 hi / lo planes)
    on every tile geometry they are instantiated for: within 1e-4 of the fp32 reference, and a
    board's outputs bitwise the same whatever its batch position and tile-mates."""
    import az_amd
    import net_oracle
    bs, ci, A, ch, blocks, res, B = case
    desc = az_amd.NetDesc(bs, ci, ch, blocks, A, 32, 8, 256, res, 0, PREC[prec], B)
    net = az_amd.HipNeuralNetwork(engine, desc)
    if ch % 64 == 0:
        assert net.trunk_kernel().startswith("conv3x3_v9x3<" if ch % 256 == 0 else "conv3x3_v7x3<")
    blob = net_oracle.init_blob(desc, seed=31)
    net.load_weights(blob)
    x = _rand_planes(B, ci, bs, seed=40 + bs, p=0.05 if ci > 16 else 0.25)
    lo, v = net.forward(x)
    rl, rv = net_oracle.forward(desc, blob, x)
    el, ev = float(np.abs(lo - rl).max()), float(np.abs(v - rv).max())
    print(f"{case} {prec}: max|dlogit|={el:.3e} (|logit|max {np.abs(rl).max():.3f}) max|dvalue|={ev:.3e}")
    assert el <= TOL and ev <= TOL
    perm = np.random.default_rng(bs).permutation(B)
    lo2, v2 = net.forward(x[perm])
    assert np.array_equal(lo2, lo[perm]) and np.array_equal(v2, v[perm])
    lo3, v3 = net.forward(x[B - 2:])
    assert np.array_equal(lo3, lo[B - 2:]) and np.array_equal(v3, v[B - 2:])
    net.close()


G8_CASES = [  # (board, in_planes, action_size, channels, blocks, B): the g8 conv3x3_v6 board geometries
    (19, 8, 362, 128, 2, 5),      # Go shape (C4: 8 planes, 361 + pass); flattened tiles span boards
    (8, 111, 4672, 128, 2, 9),    # Chess shape (C5: 111 planes, 4672 moves); flattened tiles, v6 input conv
    (9, 11, 81, 128, 2, 6),       # Gomoku 9x9 (C1 board)
    (13, 11, 169, 256, 1, 3),     # Go 13x13
    (15, 20, 225, 128, 1, 4),     # 15x15 with > 16 planes: the input conv runs on v6 (32-channel chunks)
]


def _rand_planes(B, ci, bs, seed, p=0.2):
    rng = np.random.default_rng(seed)
    return (rng.random((B, ci, bs, bs)) < p).astype(np.float32)


@pytest.mark.gpu
@pytest.mark.parametrize("bs,ci", [(8, 32), (9, 11), (13, 8), (15, 11), (19, 8)])
def test_gpu_g8_batch_position_independent(engine, bs, ci):
    """g8 trunk (DENSE tiles on 8/9/13/19, where a 512-row tile spans boards and the batch's last
    tile is partial; the padded two-board tile on 15x15): a board's output is bitwise the same
    whatever its position in the batch, its tile-mates and the batch size."""
    import az_amd
    import net_oracle
    B = 23
    desc = az_amd.NetDesc(bs, ci, 128, 2, bs * bs, 32, 8, 256, 1, 0, az_amd.AZ_PREC_FP16, B)
    net = az_amd.HipNeuralNetwork(engine, desc)
    net.load_weights(net_oracle.init_blob(desc, seed=9))
    x = _rand_planes(B, ci, bs, seed=100 + bs)
    lo, v = net.forward(x)
    perm = np.random.default_rng(bs).permutation(B)
    lo2, v2 = net.forward(x[perm])
    assert np.array_equal(lo2, lo[perm]) and np.array_equal(v2, v[perm])
    for a, b in ((0, 1), (5, 12), (22, 23)):
        lo3, v3 = net.forward(x[a:b])
        assert np.array_equal(lo3, lo[a:b]) and np.array_equal(v3, v[a:b]), (a, b)
    net.close()


@pytest.mark.gpu
@pytest.mark.parametrize("prec", ["fp16", "bf16"])
@pytest.mark.parametrize("case", G8_CASES, ids=[str(c) for c in G8_CASES])
def test_gpu_g8_boards_match_fp32_reference(engine, case, prec):
    """conv3x3_v6 on every board geometry it is instantiated for (8, 9, 13, 15, 19), through the
    whole net against the fp32 reference: fp16 within the 1e-4 tolerance, bf16 a sanity bound."""
    import az_amd
    import net_oracle
    bs, ci, A, ch, blocks, B = case
    p = {"fp16": az_amd.AZ_PREC_FP16, "bf16": az_amd.AZ_PREC_BF16}[prec]
    desc = az_amd.NetDesc(bs, ci, ch, blocks, A, 32, 8, 256, 1, 0, p, B)
    net = az_amd.HipNeuralNetwork(engine, desc)
    blob = net_oracle.init_blob(desc, seed=21)
    net.load_weights(blob)
    x = _rand_planes(B, ci, bs, seed=bs, p=0.05 if ci > 16 else 0.2)
    lo, v = net.forward(x)
    rl, rv = net_oracle.forward(desc, blob, x)
    el, ev = float(np.abs(lo - rl).max()), float(np.abs(v - rv).max())
    print(f"{case} {prec}: max|dlogit|={el:.3e} (|logit|max {np.abs(rl).max():.3f}) max|dvalue|={ev:.3e}")
    if prec == "fp16":
        assert el <= TOL and ev <= TOL
    else:
        assert el < 5e-2 * max(1.0, np.abs(rl).max()) and ev < 5e-2
    # a sample's output does not depend on the batch it rides in (ragged tiles of BOARDS boards)
    lo1, v1 = net.forward(x[B - 1:])
    assert np.array_equal(lo1, lo[B - 1:]) and np.array_equal(v1, v[B - 1:])
    net.close()


@pytest.mark.gpu
@pytest.mark.parametrize("shape", ["go19", "chess"])
def test_gpu_c4_c5_nets_fp16_within_tolerance(engine, shape):
    """The C4 (Go 19x19) and C5 (Chess 8x8x111 -> 4672) 20-block x 256-filter nets in fp16: every
    logit and value within 1e-4 of the fp32 reference."""
    import az_amd
    import net_oracle
    if shape == "go19":
        desc = az_amd.NetDesc(19, 8, 256, 20, 362, 32, 8, 256, 1, 0, az_amd.AZ_PREC_FP16, 24)
        x = _rand_planes(24, 8, 19, seed=3, p=0.3)
    else:
        desc = az_amd.NetDesc(8, 111, 256, 20, 4672, 32, 8, 256, 1, 0, az_amd.AZ_PREC_FP16, 48)
        x = _rand_planes(48, 111, 8, seed=4, p=0.05)
    net = az_amd.HipNeuralNetwork(engine, desc)
    blob = net_oracle.init_blob(desc, seed=1234)
    net.load_weights(blob)
    lo, v = net.forward(x)
    rl, rv = net_oracle.forward(desc, blob, x)
    el, ev = float(np.abs(lo - rl).max()), float(np.abs(v - rv).max())
    print(f"{shape} fp16: max|dlogit|={el:.3e} max|dvalue|={ev:.3e} (|logit|max {np.abs(rl).max():.3f})")
    assert el <= TOL and ev <= TOL
    net.close()


@pytest.mark.gpu
def test_gpu_c5_net_full_batch(engine):
    """C5 at its full per-GPU batch (BASELINE.json configs[4]: 8x8x111 planes -> 4672-way policy, 20 x
    256 net, B = 1024 -- the chess rules are not runnable in the reference): a
    sample of the 1024 outputs within 1e-4 of the fp32 network, and a board's outputs bitwise the
    same in a sub-batch (DENSE tiles of 8 boards, full last round)."""
    import az_amd
    import net_oracle
    B = 1024
    desc = az_amd.NetDesc(8, 111, 256, 20, 4672, 32, 8, 256, 1, 0, az_amd.AZ_PREC_FP16, B)
    net = az_amd.HipNeuralNetwork(engine, desc)
    blob = net_oracle.init_blob(desc, seed=1234)
    net.load_weights(blob)
    x = _rand_planes(B, 111, 8, seed=11, p=0.05)
    lo, v = net.forward(x)
    idx = np.random.default_rng(5).choice(B, 24, replace=False)
    rl, rv = net_oracle.forward(desc, blob, x[idx])
    assert np.abs(lo[idx] - rl).max() <= TOL and np.abs(v[idx] - rv).max() <= TOL
    lo2, v2 = net.forward(x[517:530])
    assert np.array_equal(lo2, lo[517:530]) and np.array_equal(v2, v[517:530])
    net.close()


@pytest.mark.gpu
@pytest.mark.parametrize("case", [
    # (board, in_planes, channels, blocks, actions, precision, max_batch) -> trunk kernel prefix
    ((15, 11, 256, 20, 225, "fp16", 2048), "conv3x3_v7<2, 15, SLIM>"),   # C3 at N = 1, 2
    ((15, 11, 256, 20, 225, "fp16", 256), "conv3x3_v6<2, 15>"),          # C3 shard at N = 8
    ((15, 11, 64, 6, 225, "fp16", 256), "k_smallnet_g<15, 8, true>"),    # C2: the fused 64-filter forward
    ((15, 11, 64, 6, 225, "f16x3", 256), "k_smallnet_x3<15, 8, true, 2>"),   # C2 in the parity precision
    ((15, 11, 64, 6, 225, "bf16x3", 256), "k_smallnet_x3<15, 8, true, 1>"),
    ((15, 11, 256, 20, 225, "f16x3", 2048), "conv3x3_v9x3<15, SLIM, f16>"),   # the parity precision at C3
    ((15, 11, 256, 20, 225, "bf16x3", 64), "conv3x3_v9x3<15, SLIM>"),
    ((15, 11, 256, 20, 225, "bf16x3", 2048), "conv3x3_v9x3<15, SLIM>"),
    ((15, 11, 128, 2, 225, "bf16x3", 64), "conv3x3_v7x3<15, SLIM>"),    # 128 channels: the v7 tile
    ((15, 11, 128, 2, 225, "f16x3", 64), "conv3x3_v7x3<15, SLIM, f16>"),
    ((19, 8, 256, 20, 362, "bf16x3", 1024), "conv3x3_v9x3<19, DENSE>"),
    ((19, 8, 256, 20, 362, "f16x3", 1024), "conv3x3_v9x3<19, DENSE, f16>"),
    ((19, 8, 256, 20, 362, "fp16", 1024), "conv3x3_v6<2, 19, DENSE>"),   # C4
    ((19, 8, 256, 20, 362, "fp16", 128), "conv3x3_v7<2, 19, DENSE, 128, 3>"),   # C4 shard at N = 8: small tiles
    ((19, 8, 256, 20, 362, "fp16", 256), "conv3x3_v7<2, 19, DENSE, 128, 3>"),   # C4 shard at N = 4
    ((8, 111, 256, 20, 4672, "fp16", 128), "conv3x3_v7<2, 8, DENSE, 64>"),   # C5 shard at N = 8
    ((8, 111, 256, 20, 4672, "fp16", 1024), "conv3x3_v6<2, 8, DENSE>"),      # C5 at N = 1
    ((15, 11, 32, 2, 225, "f32", 4), "gemm_f32"),
])
def test_gpu_trunk_kernel_name(engine, case):
    """az_net_trunk_kernel names the kernel the trunk actually dispatches (bench.py's roofline label)."""
    import az_amd
    (bs, ci, ch, blocks, A, prec, B), want = case
    p = PREC[prec]
    net = az_amd.HipNeuralNetwork(engine, az_amd.NetDesc(bs, ci, ch, blocks, A, 32, 8, 256, 1, 0, p, B))
    assert net.trunk_kernel() == want
    net.close()


@pytest.mark.gpu
@pytest.mark.parametrize("residual", [1, 0])
@pytest.mark.parametrize("B", [256, 37])
def test_gpu_smallnet_matches_round2_kernel(engine, residual, B):
    """k_smallnet_g (round 3: offset-addressed activation fragments, weights streamed into registers,
    layer pairs, med3 epilogue) runs the round-2 kernel's arithmetic: the same MFMA sequence,
    residual stream and fp16 rounding, so both kernels (and both of the round-2 kernel's wave
    shapes) give bitwise equal outputs on C2-shape nets."""
    import az_amd
    from az_amd import _lib
    d = az_amd.NetDesc(15, 11, 64, 6, 225, 32, 8, 256, residual, 0, az_amd.AZ_PREC_FP16, 256)
    net = az_amd.HipNeuralNetwork(engine, d)
    net.init_random(77 + residual)
    x = _rand_planes(B, 11, 15, 5 + B)
    outs = {}
    try:
        for k, w in ((1, 8), (0, 8), (1, 4)):
            _lib.lib().az_diag_set_smallnet_kernel(k)
            _lib.lib().az_diag_set_smallnet_waves(w)
            outs[(k, w)] = net.forward(x)
    finally:
        _lib.lib().az_diag_set_smallnet_kernel(0)
        _lib.lib().az_diag_set_smallnet_waves(8)
    ref_p, ref_v = outs[(1, 8)]
    assert np.isfinite(ref_p).all() and np.abs(ref_p).max() > 0
    for kw, (pl, v) in outs.items():
        np.testing.assert_array_equal(pl, ref_p, err_msg=f"kernel {kw}")
        np.testing.assert_array_equal(v, ref_v, err_msg=f"kernel {kw}")


@pytest.mark.gpu
@pytest.mark.parametrize("prec", ["f16x3", "bf16x3"])
@pytest.mark.parametrize("residual", [1, 0])
@pytest.mark.parametrize("B", [256, 37])
def test_gpu_smallnet_x3_matches_oracle(engine, residual, B, prec):
    """k_smallnet_x3 (the fused 64-filter forward in the split precisions: hi / lo activation planes
    of fp16 or bf16 pieces updated in place in LDS, three MFMAs per product) on C2-shape nets: within
    the north-star 1e-4 of the fp32 network on sampled boards, and a board's outputs bitwise the same
    whatever its batch position (permuted batch, a tail slice)."""
    import az_amd
    import net_oracle
    d = az_amd.NetDesc(15, 11, 64, 6, 225, 32, 8, 256, residual, 0, PREC[prec], 256)
    net = az_amd.HipNeuralNetwork(engine, d)
    pt = 2 if prec == "f16x3" else 1
    assert net.trunk_kernel() == f"k_smallnet_x3<15, 8, {'true' if residual else 'false'}, {pt}>"
    blob = net_oracle.init_blob(d, seed=91 + residual)
    net.load_weights(blob)
    x = _rand_planes(B, 11, 15, 15 + B)
    lo, v = net.forward(x)
    pick = np.unique(np.concatenate([[0, B - 1], np.random.default_rng(B).choice(B, 10, replace=False)]))
    rl, rv = net_oracle.forward(d, blob, x[pick])
    el, ev = float(np.abs(lo[pick] - rl).max()), float(np.abs(v[pick] - rv).max())
    print(f"smallnet_x3 {prec} residual={residual} B={B}: max|dlogit|={el:.3e} max|dvalue|={ev:.3e}")
    assert el <= TOL and ev <= TOL
    perm = np.random.default_rng(3).permutation(B)
    lo2, v2 = net.forward(x[perm])
    assert np.array_equal(lo2, lo[perm]) and np.array_equal(v2, v[perm])
    lo3, v3 = net.forward(x[B - 5:])
    assert np.array_equal(lo3, lo[B - 5:]) and np.array_equal(v3, v[B - 5:])
    net.close()
