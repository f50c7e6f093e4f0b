"""GPU parity of the batched HIP search on Go (GoState on device --
captures, ko, positional superko, pass, area scoring, the 8 feature planes) against
  (1) golden games of the patched REFERENCE search on GoState (tests/golden/ref_go_games.json.gz),
  (2) the CPU restatement (oracle/az_oracle.cpp, GoState) for multi-game runs with per-game seeds.
Bit-exact, as tests/test_gpu_search.py."""
import gzip
import json
import os

import numpy as np
import pytest

from test_gpu_search import bits, children_rows, play_and_compare

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
with gzip.open(os.path.join(GOLD, "ref_go_games.json.gz"), "rt") as _f:
    GO_GAMES = json.load(_f)


@pytest.fixture(scope="module")
def engine():
    import az_amd
    return az_amd.Engine(0)


@pytest.mark.gpu
@pytest.mark.parametrize("idx", range(len(GO_GAMES)), ids=[str(g["case"]) for g in GO_GAMES])
def test_gpu_go_search_matches_reference_golden(engine, idx):
    import az_amd
    ref = GO_GAMES[idx]
    bs, sims, mm, ev, es, nes, cp, fpu = ref["case"]
    m = az_amd.ParallelMCTS(engine, n_games=1, board_size=bs, num_simulations=sims, c_puct=cp, fpu_reduction=fpu,
                            evaluator=az_amd.AZ_EVAL_HASH, eval_seed=es, use_dirichlet_each_search=bool(nes),
                            game=az_amd.AZ_GAME_GO)
    try:
        play_and_compare(m, [ref], 1)
    finally:
        m.close()


@pytest.mark.gpu
@pytest.mark.parametrize("bs,sims,games,ev,max_moves", [(9, 120, 12, "hash", 60), (9, 90, 6, "uniform", 40),
                                                         (13, 200, 4, "hash", 12)])
def test_gpu_go_multigame_matches_oracle(engine, bs, sims, games, ev, max_moves):
    """G independent Go games with per-game noise seeds (42 + g)."""
    import az_amd
    import az_oracle as O
    kind = {"hash": O.EVAL_HASH, "uniform": O.EVAL_UNIFORM}[ev]
    dev = {"hash": az_amd.AZ_EVAL_HASH, "uniform": az_amd.AZ_EVAL_UNIFORM}[ev]
    refs = O.play(seed_stride=1, bs=bs, sims=sims, max_moves=max_moves, eval_kind=kind, eval_seed=5, n_games=games,
                  game=O.GAME_GO)
    m = az_amd.ParallelMCTS(engine, n_games=games, board_size=bs, num_simulations=sims, evaluator=dev, eval_seed=5,
                            noise_seed=42, noise_seed_stride=1, game=az_amd.AZ_GAME_GO)
    try:
        play_and_compare(m, refs, games, max_moves)
    finally:
        m.close()


@pytest.mark.gpu
def test_gpu_go_small_tt(engine):
    """2^6 TT slots: collisions, replacement, and Go TT hits re-gathering the cached policy over the
    current legal set."""
    import az_amd
    import az_oracle as O
    bs, sims, mm = 9, 150, 30
    refs = O.play(bs=bs, sims=sims, max_moves=mm, eval_kind=O.EVAL_HASH, tt_log2=6, game=O.GAME_GO)
    m = az_amd.ParallelMCTS(engine, n_games=1, board_size=bs, num_simulations=sims, evaluator=az_amd.AZ_EVAL_HASH,
                            tt_log2=6, game=az_amd.AZ_GAME_GO)
    try:
        play_and_compare(m, refs, 1, mm)
    finally:
        m.close()


@pytest.mark.gpu
@pytest.mark.parametrize("prec", [0, 3])
def test_gpu_go_net_selfplay_matches_oracle_replay(engine, prec):
    """Go with the ConvNet evaluator: the device's 8 GoState feature planes of every evaluated leaf
    equal the oracle's for the same search, and replaying the logged network outputs through the
    oracle reproduces the device search bit for bit (as tests/test_gpu_selfplay_net.py)."""
    import az_amd
    import az_oracle as O
    import net_oracle
    bs, sims, G, moves, logged = 9, 100, 3, 8, 1
    ch = 128 if prec == 3 else 32
    desc = az_amd.NetDesc(bs, 8, ch, 2, bs * bs + 1, 32, 8, 256, 1, 0, prec, G)
    net = az_amd.HipNeuralNetwork(engine, desc)
    blob = net_oracle.init_blob(desc, seed=9)
    net.load_weights(blob)
    m = az_amd.ParallelMCTS(engine, n_games=G, board_size=bs, num_simulations=sims, evaluator=az_amd.AZ_EVAL_NET,
                            net=net, noise_seed=42, noise_seed_stride=1, game=az_amd.AZ_GAME_GO)
    cap = (sims + 2) * (moves + 1)
    m.enableEvalLog(logged, cap)
    m.newGames()
    m.addDirichletNoise(0.03, 0.25)
    dev = []
    try:
        for ply in range(moves):
            m.search()
            act, val, probs, cact, nch = m.select(True, 1.0 if ply < 30 else 0.0)
            a, N, VL, W, P = m.rootChildren(logged)
            dev.append(dict(action=int(act[logged]), N=N.tolist(), VL=VL.tolist(), W=W.view(np.uint32).tolist(),
                            P=P.view(np.uint32).tolist(), probs=probs[logged, :nch[logged]].view(np.uint32).tolist()))
            term, _ = m.updateWithMove(act)
            if ply % 2 == 0:
                m.addDirichletNoise(0.03, 0.25)
            if term[logged]:
                break
        pol, valv, planes = m.readEvalLog(cap)
    finally:
        m.close()
    assert len(pol) > sims and planes.shape[1] == 8

    k = [0]

    def replay(game, x):
        i = k[0]
        k[0] += 1
        assert np.array_equal(x, planes[i]), f"feature planes differ at evaluation {i}"
        return pol[i], float(valv[i])

    ref = O.play(bs=bs, sims=sims, max_moves=len(dev), eval_kind=O.EVAL_REPLAY, evaluator=replay,
                 noise_seed=42 + logged, game=O.GAME_GO)[0]
    assert k[0] == len(pol)
    for ply, (d, r) in enumerate(zip(dev, ref["moves"])):
        kids = r["children"]
        assert d["N"] == [c[1] for c in kids] and d["VL"] == [c[2] for c in kids], ply
        assert d["W"] == [c[3] for c in kids] and d["P"] == [c[4] for c in kids], ply
        assert d["probs"] == r["probs"] and d["action"] == r["action"], ply
    # the logged network outputs against the fp32 reference network on the same planes
    rl, rv = net_oracle.forward(desc, blob, planes[:64])
    sm = net_oracle.softmax_policy(rl)
    assert np.abs(sm - pol[:64]).max() <= 1e-4 and np.abs(rv - valv[:64]).max() <= 1e-4
    net.close()


C4_REPLAYS = [  # games per GPU, the logged game, trunk precision, the trunk kernel that batch takes
    (1024, 777, "fp16", "conv3x3_v6<2, 19, DENSE>"),          # C4 on one GPU
    (128, 77, "fp16", "conv3x3_v7<2, 19, DENSE, 128, 3>"),       # the per-rank shard of C4 on 8 GPUs
    (128, 101, "f16x3", "conv3x3_v9x3<19, DENSE, f16>"),      # the same shard in the parity precision
]


@pytest.mark.gpu
@pytest.mark.parametrize("G,logged,prec,kernel", C4_REPLAYS, ids=[f"G{c[0]}-{c[2]}" for c in C4_REPLAYS])
def test_gpu_c4_full_size_replay(engine, G, logged, prec, kernel):
    """C4 at full per-GPU size (BASELINE.json configs[3]: Go 19x19, 1024 games, 800 sims, the 20 x 256
    net with 8 planes / 362 actions, fp16 trunk on DENSE tiles) and at the per-rank shard of its 8-GPU
    run (128 games: the small-tile trunk; python/scripts/orchestrate_selfplay.py:303-311 shards the
    games over the GPUs), fp16 and F16X3: the first two moves of every game, one game replayed bit for
    bit through the CPU restatement, sampled network outputs within 1e-4 of the fp32 reference
    network, and every root's probabilities summing to 1."""
    import az_amd
    import az_oracle as O
    import net_oracle
    bs, sims, moves = 19, 800, 2
    p = {"fp16": az_amd.AZ_PREC_FP16, "f16x3": az_amd.AZ_PREC_F16X3}[prec]
    desc = az_amd.NetDesc(bs, 8, 256, 20, bs * bs + 1, 32, 8, 256, 1, 0, p, G)
    net = az_amd.HipNeuralNetwork(engine, desc)
    assert net.trunk_kernel() == kernel
    blob = net_oracle.init_blob(desc, seed=1234)
    net.load_weights(blob)
    m = az_amd.ParallelMCTS(engine, n_games=G, board_size=bs, num_simulations=sims, evaluator=az_amd.AZ_EVAL_NET,
                            net=net, noise_seed=42, noise_seed_stride=1, game=az_amd.AZ_GAME_GO)
    cap = (sims + 2) * (moves + 1)
    m.enableEvalLog(logged, cap)
    m.newGames()
    m.addDirichletNoise(0.03, 0.25)
    dev = []
    try:
        for ply in range(moves):
            m.search()
            act, val, probs, cact, nch = m.select(True, 1.0)
            sums = np.array([probs[g, :nch[g]].astype(np.float64).sum() for g in range(G)])
            assert np.abs(sums - 1.0).max() < 1e-5
            a, N, VL, W, P = m.rootChildren(logged)
            dev.append(dict(action=int(act[logged]), N=N.tolist(), VL=VL.tolist(), W=W.view(np.uint32).tolist(),
                            P=P.view(np.uint32).tolist(), probs=probs[logged, :nch[logged]].view(np.uint32).tolist()))
            m.updateWithMove(act)
            if ply % 2 == 0:
                m.addDirichletNoise(0.03, 0.25)
        pol, valv, planes = m.readEvalLog(cap)
    finally:
        m.close()
    k = [0]

    def replay(game, x):
        i = k[0]
        k[0] += 1
        assert np.array_equal(x, planes[i]), f"feature planes differ at evaluation {i}"
        return pol[i], float(valv[i])

    ref = O.play(bs=bs, sims=sims, max_moves=moves, eval_kind=O.EVAL_REPLAY, evaluator=replay,
                 noise_seed=42 + logged, game=O.GAME_GO)[0]
    assert k[0] == len(pol)
    for ply, (d, r) in enumerate(zip(dev, ref["moves"])):
        kids = r["children"]
        assert d["N"] == [c[1] for c in kids] and d["VL"] == [c[2] for c in kids], ply
        assert d["W"] == [c[3] for c in kids] and d["P"] == [c[4] for c in kids], ply
        assert d["probs"] == r["probs"] and d["action"] == r["action"], ply
    idx = np.random.default_rng(1).choice(len(pol), 32, replace=False)
    rl, rv = net_oracle.forward(desc, blob, planes[idx])
    assert np.abs(net_oracle.softmax_policy(rl) - pol[idx]).max() <= 1e-4 and np.abs(rv - valv[idx]).max() <= 1e-4
    # RAW logits / values of a full B = G forward of the logged leaves (cycled): 16 boards vs fp32
    xb = planes[np.arange(G) % len(planes)]
    lo, v = net.forward(xb)
    jdx = np.unique(np.concatenate([[0, G - 1], np.random.default_rng(2).choice(G, 14, replace=False)]))
    jl, jv = net_oracle.forward(desc, blob, xb[jdx])
    el, ev = float(np.abs(lo[jdx] - jl).max()), float(np.abs(v[jdx] - jv).max())
    print(f"C4 G={G} {prec} raw outputs: |logit|max {np.abs(jl).max():.3f} max|dlogit|={el:.3e} max|dvalue|={ev:.3e}")
    assert el <= 1e-4 and ev <= 1e-4
    net.close()
