"""Full hot path with the ConvNet evaluator: device feature planes -> HIP ConvNet ->
softmax -> TT/expand/backup.  The engine logs every evaluation of one game; the CPU
restatement replays those (policy, value) outputs and must reproduce the device
search bit for bit, and must have asked for exactly the logged feature planes.
The logged network outputs are separately checked against the fp32 reference
network (tolerance 1e-4, BASELINE.json north_star)."""
import numpy as np
import pytest


@pytest.mark.gpu
@pytest.mark.parametrize("prec", [0, 1])
@pytest.mark.parametrize("logged", [0, 3])
def test_gpu_net_selfplay_matches_oracle_replay(prec, logged):
    import az_amd
    import az_oracle as O
    import net_oracle
    bs, sims, G, moves = 9, 48, 4, 6
    eng = az_amd.Engine(0)
    desc = az_amd.gomoku_net_desc(board_size=bs, channels=32, blocks=2, precision=prec, max_batch=G)
    net = az_amd.HipNeuralNetwork(eng, desc)
    blob = net_oracle.init_blob(desc, seed=9)
    net.load_weights(blob)
    m = az_amd.ParallelMCTS(eng, n_games=G, board_size=bs, num_simulations=sims, evaluator=az_amd.AZ_EVAL_NET,
                            net=net, noise_seed=42, noise_seed_stride=1)
    cap = (sims + 2) * (moves + 1)
    m.enableEvalLog(logged, cap)
    m.newGames()
    m.addDirichletNoise(0.03, 0.25)
    dev = []
    for ply in range(moves):
        m.search()
        T = 1.0 if ply < 30 else 0.0
        act, val, probs, cact, nch = m.select(True, T)
        a, N, VL, W, P = m.rootChildren(logged)
        dev.append(dict(action=int(act[logged]), value=float(val[logged]), N=N.tolist(), VL=VL.tolist(),
                        W=W.view(np.uint32).tolist(), P=P.view(np.uint32).tolist(),
                        probs=probs[logged, :nch[logged]].view(np.uint32).tolist()))
        term, _ = m.updateWithMove(act)
        if ply % 2 == 0:
            m.addDirichletNoise(0.03, 0.25)
        if term[logged]:
            break
    pol, valv, planes = m.readEvalLog(cap)
    assert len(pol) > sims

    k = [0]

    def replay(game, x):
        i = k[0]
        k[0] += 1
        assert np.array_equal(x, planes[i]), f"feature planes differ at evaluation {i}"
        return pol[i], float(valv[i])

    ref = O.play(bs=bs, sims=sims, max_moves=len(dev), eval_kind=O.EVAL_REPLAY, evaluator=replay,
                 noise_seed=42 + logged)[0]
    assert k[0] == len(pol)
    for ply, (d, r) in enumerate(zip(dev, ref["moves"])):
        kids = r["children"]
        assert d["N"] == [c[1] for c in kids] and d["VL"] == [c[2] for c in kids], ply
        assert d["W"] == [c[3] for c in kids] and d["P"] == [c[4] for c in kids], ply
        assert d["probs"] == r["probs"] and d["action"] == r["action"], ply
        assert np.float32(d["value"]).view(np.uint32) == r["value"], ply
    # the logged network outputs against the fp32 reference network
    rl, rv = net_oracle.forward(desc, blob, planes)
    assert np.abs(valv - rv).max() <= 1e-4
    assert np.abs(pol - net_oracle.softmax_policy(rl)).max() <= 1e-4
    m.close()
    net.close()


def _full_size_replay(bs, sims, G, moves, logged, channels, blocks, prec=None, trained=False):
    """Play `moves` moves of G games at a BASELINE.json size (fp16 trunk unless `prec`), log game
    `logged` and replay it through the CPU restatement bit for bit; check a sample of its logged
    network outputs against the fp32 reference network (1e-4) and size-independent properties of
    every game's root (one child per empty cell, visit sum, probability sum, value range).
    trained: heads scaled to a trained net's output magnitudes (|logit|max 8, |value| ~0.9,
    test_gpu_trained_scale.trained_scale_blob), and the raw logits of a full B = G forward of the
    logged leaves checked against the fp32 network too."""
    import az_amd
    import az_oracle as O
    import net_oracle
    eng = az_amd.Engine(0)
    desc = az_amd.gomoku_net_desc(board_size=bs, channels=channels, blocks=blocks,
                                  precision=az_amd.AZ_PREC_FP16 if prec is None else prec, max_batch=G)
    net = az_amd.HipNeuralNetwork(eng, desc)
    if trained:
        from test_gpu_trained_scale import _planes as ts_planes, trained_scale_blob
        blob = trained_scale_blob(desc, 1234, ts_planes("c3", 16, seed=17))
    else:
        blob = net_oracle.init_blob(desc, seed=1234)
    net.load_weights(blob)
    m = az_amd.ParallelMCTS(eng, n_games=G, board_size=bs, num_simulations=sims, evaluator=az_amd.AZ_EVAL_NET,
                            net=net, noise_seed=42, noise_seed_stride=1)
    cap = (sims + 2) * (moves + 1)
    m.enableEvalLog(logged, cap)
    m.newGames()
    m.addDirichletNoise(0.03, 0.25)
    dev = []
    for ply in range(moves):
        m.search()
        act, val, probs, cact, nch = m.select(True, 1.0)
        # every game: one child per empty cell, probabilities sum to 1, values within [-1, 1]
        assert (nch == bs * bs - ply).all()
        sums = np.array([probs[g, :nch[g]].astype(np.float64).sum() for g in range(G)])
        assert np.abs(sums - 1.0).max() < 1e-5
        assert (np.abs(val) <= 1.0 + 1e-6).all()
        a, N, VL, W, P = m.rootChildren(logged)
        assert int(np.sum(N)) >= sims - 1
        dev.append(dict(action=int(act[logged]), value=float(val[logged]), N=N.tolist(), VL=VL.tolist(),
                        W=W.view(np.uint32).tolist(), P=P.view(np.uint32).tolist(),
                        probs=probs[logged, :nch[logged]].view(np.uint32).tolist()))
        m.updateWithMove(act)
        if ply % 2 == 0:
            m.addDirichletNoise(0.03, 0.25)
    pol, valv, planes = m.readEvalLog(cap)
    assert len(pol) > sims   # TT hits and terminal leaves are not evaluated
    k = [0]

    def replay(game, x):
        i = k[0]
        k[0] += 1
        assert np.array_equal(x, planes[i]), f"feature planes differ at evaluation {i}"
        return pol[i], float(valv[i])

    ref = O.play(bs=bs, sims=sims, max_moves=moves, eval_kind=O.EVAL_REPLAY, evaluator=replay,
                 noise_seed=42 + logged)[0]
    assert k[0] == len(pol)
    for ply, (d, r) in enumerate(zip(dev, ref["moves"])):
        kids = r["children"]
        assert d["N"] == [c[1] for c in kids] and d["VL"] == [c[2] for c in kids], ply
        assert d["W"] == [c[3] for c in kids] and d["P"] == [c[4] for c in kids], ply
        assert d["probs"] == r["probs"] and d["action"] == r["action"], ply
        assert np.float32(d["value"]).view(np.uint32) == r["value"], ply
    idx = np.random.default_rng(0).choice(len(pol), 48, replace=False)
    rl, rv = net_oracle.forward(desc, blob, planes[idx])
    assert np.abs(valv[idx] - rv).max() <= 1e-4
    assert np.abs(pol[idx] - net_oracle.softmax_policy(rl)).max() <= 1e-4
    # RAW logits and values of a full-capacity forward (B = G boards: the logged leaves, cycled) --
    # post-softmax probabilities of ~1/A each would hide a logit error A times larger
    xb = planes[np.arange(G) % len(planes)]
    lo, v = net.forward(xb)
    jdx = np.unique(np.concatenate([[0, G - 1], np.random.default_rng(1).choice(G, 14, replace=False)]))
    jl, jv = net_oracle.forward(desc, blob, xb[jdx])
    el = float(np.abs(lo[jdx] - jl).max())
    ev = float(np.abs(v[jdx] - jv).max())
    print(f"full-size raw outputs ({'trained-scale' if trained else 'init'} weights): |logit|max "
          f"{np.abs(jl).max():.3f} max|dlogit|={el:.3e} max|dvalue|={ev:.3e} over {len(jdx)} boards of B = {G}")
    assert el <= 1e-4 and ev <= 1e-4
    if trained:
        assert np.abs(jl).max() > 2.0
    m.close()
    net.close()


@pytest.mark.gpu
def test_gpu_c3_full_size_replay():
    """C3 at full size (BASELINE.json configs[2]: 2048 games, 15x15, 800 sims, the 20 x 256 net):
    the first two moves of every game, game 1337 (in the middle of the batch) replayed."""
    _full_size_replay(bs=15, sims=800, G=2048, moves=2, logged=1337, channels=256, blocks=20)


@pytest.mark.gpu
@pytest.mark.parametrize("prec", ["f16x3", "bf16x3"])
def test_gpu_c3_full_size_replay_x3(prec):
    """C3 at full size in the split precisions (AZ_PREC_F16X3 -- the parity precision -- and
    AZ_PREC_BF16X3, both on conv3x3_v9x3) with trained-scale heads: two moves of all 2048 games, game
    1337 replayed bit for bit, sampled logits / values of the logged leaves and of a B = 2048 forward
    within 1e-4 of the fp32 network."""
    _full_size_replay(bs=15, sims=800, G=2048, moves=2, logged=1337, channels=256, blocks=20,
                      prec={"f16x3": 4, "bf16x3": 1}[prec], trained=True)


@pytest.mark.gpu
def test_gpu_c2_full_size_replay():
    """C2 at full size (BASELINE.json configs[1]: 256 games, 15x15, 400 sims, the 6 x 64 net of
    python/simple_export.py's shape family): the first four moves of every game (noise after plies
    0 and 2, subtree reuse across three moves), game 137 replayed."""
    _full_size_replay(bs=15, sims=400, G=256, moves=4, logged=137, channels=64, blocks=6)


@pytest.mark.gpu
@pytest.mark.parametrize("prec", ["f16x3", "bf16x3"])
def test_gpu_c2_full_size_replay_x3(prec):
    """C2 at full size in the split precisions (k_smallnet_x3 with fp16 / bf16 pieces, fed the
    search's leaf records) with trained-scale heads: four moves of all 256 games, game 137 replayed
    bit for bit, sampled outputs of the logged leaves and of a B = 256 forward within 1e-4 of fp32."""
    _full_size_replay(bs=15, sims=400, G=256, moves=4, logged=137, channels=64, blocks=6,
                      prec={"f16x3": 4, "bf16x3": 1}[prec], trained=True)
