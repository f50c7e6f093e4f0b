"""A host evaluator driving the device search (AZ_EVAL_CALLBACK: the path a custom NeuralNetwork
subclass takes, parallel_mcts.cpp:886-901):
  (1) az_amd with a callback over the feature planes, three games at once, against the CPU
      restatement running the same function over the same planes (oracle EVAL_REPLAY): bit-exact
      roots, children, visit distributions, actions and values;
  (2) the C++ host ParallelMCTS with a Python subclass of NeuralNetwork -- the reference test
      evaluator HashEvaluator written in Python over state.getHash() / getMoveHistory() -- against
      the REFERENCE's own API golden (tests/golden/ref_api.json.gz case 0) and its 9x9 golden game;
  (3) SelfPlayManager with that Python network and setBatchConfig capping the batch, against the
      CPU restatement."""
import gzip
import json
import os

import numpy as np
import pytest

from test_gpu_search import bits, play_and_compare

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def engine():
    import az_amd
    return az_amd.Engine(0)


def plane_eval(planes):
    """A deterministic function of one state's planes [C][bs][bs] -> (policy [A], value)."""
    x = np.asarray(planes, np.float32)
    A = x.shape[1] * x.shape[2]
    w = (np.arange(A) % 13 + 1).astype(np.float32)
    p = x[0].ravel() * np.float32(0.5) + x[1].ravel() * np.float32(0.25) + np.float32(0.01) * w + \
        x[2].ravel() * np.float32(0.125)
    v = np.float32(np.tanh(np.float32(x[0].sum() - x[1].sum()) * np.float32(0.05) + np.float32(x[3].sum() * 0.01)))
    return p.astype(np.float32), float(v)


@pytest.mark.gpu
def test_gpu_callback_evaluator_matches_oracle(engine):
    import az_amd
    import az_oracle as O
    bs, sims, n = 9, 60, 3
    refs = O.play(seed_stride=1, bs=bs, sims=sims, max_moves=6, eval_kind=O.EVAL_REPLAY, n_games=n,
                  evaluator=lambda g, planes: plane_eval(planes))
    batches = []

    def cb(games, moves, planes):
        batches.append(len(games))
        out = [plane_eval(planes[i]) for i in range(len(games))]
        return np.stack([o[0] for o in out]), np.array([o[1] for o in out], np.float32)

    m = az_amd.ParallelMCTS(engine, n_games=n, board_size=bs, num_simulations=sims, evaluator=az_amd.AZ_EVAL_CALLBACK,
                            callback=cb, noise_seed_stride=1)
    play_and_compare(m, refs, n, max_moves=6)
    assert max(batches) == n                 # the games' leaves arrive in one call per simulation step
    m.close()


def _hash_eval(zhash, hist, A):
    """oracle/ref_harness.cpp hash_eval in numpy (splitmix64 over the Zobrist key and the last six moves)."""
    M = (1 << 64) - 1

    def sm(x):
        x = (x + 0x9E3779B97F4A7C15) & M
        x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & M
        x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & M
        return x ^ (x >> 31)

    key = sm(zhash ^ 0x5A17C0DE)
    for i in range(6):
        mv = hist[len(hist) - 1 - i] if i < len(hist) else -1
        key = sm((key + ((mv + 2) & 0xFFFFFFFF)) & M)
    pol = np.array([sm(key ^ (((a + 1) * 0x9E3779B97F4A7C15) & M)) >> 40 for a in range(A)], np.float32) * \
        np.float32(1.0 / 16777216.0)
    rv = sm(key ^ 0x76A1) >> 40
    v = (np.float32(np.int32(np.uint32(rv))) - np.float32(8388608.0)) * np.float32(1.0 / 8388608.0)
    return pol, float(v)


@pytest.mark.gpu
def test_gpu_host_python_network_matches_reference():
    az = pytest.importorskip("_alphazero_cpp")

    class HashEvaluator(az.NeuralNetwork):
        def __init__(self):
            super().__init__()
            self.calls = 0

        def predict(self, state):
            self.calls += 1
            return _hash_eval(state.getHash(), list(state.getMoveHistory()), state.getActionSpaceSize())

    # (a) the API script: runSingleSimulation / search / releaseMemory / stochastic selection
    case = json.load(gzip.open(os.path.join(GOLD, "ref_api.json.gz"), "rt"))[0]
    bs, sims, script, ev, seed = case["case"]
    net = HashEvaluator()
    cfg = az.MCTSConfig()
    cfg.numSimulations = sims
    m = az.ParallelMCTS(az.GomokuState(bs), cfg, net, az.TranspositionTable(1 << 20))
    m.setDeterministicMode(True)
    last = -1
    for k, op in enumerate(case["ops"]):
        c, arg = op["op"][0], op["op"][1:]
        ret = 0
        if c == "n":
            m.runSingleSimulation()
        elif c == "b":
            m.runBatchedSearch()
        elif c == "s":
            m.search()
        elif c == "r":
            ret = m.releaseMemory(int(arg))
        elif c == "d":
            cfg2 = az.MCTSConfig()
            cfg2.numSimulations = sims
            cfg2.useBatchInference = False
            m.setConfig(cfg2)
        elif c in "ae":
            ret = last = m.selectAction(c == "a", float(arg))
        elif c == "m":
            m.updateWithMove(last)
            ret = last
        elif c == "x":
            m.addDirichletNoise(0.03, 0.25)
        assert ret == op["ret"], (k, op["op"])
        r = m.getRootNode()
        assert [r.visitCount, r.virtualLoss, bits([r.valueSum])[0]] == op["root"], (k, op["op"])
        got = [[a, ch.visitCount, ch.virtualLoss, bits([ch.valueSum])[0], bits([ch.prior])[0]]
               for a, ch in zip(r.actions, r.children)]
        assert got == op["children"], (k, op["op"])
    assert net.calls > 0
    # (b) the 9x9 / 100-sim golden game (playSingleGame loop), first 8 moves
    games = json.load(gzip.open(os.path.join(GOLD, "ref_games.json.gz"), "rt"))
    ref = games[0]
    bs, sims = ref["case"][0], ref["case"][1]
    m = az.ParallelMCTS(az.GomokuState(bs), HashEvaluator(), None, 1, sims, 1.5, 0.0, 3)
    m.setDeterministicMode(True)
    m.addDirichletNoise(0.03, 0.25)
    for ply in range(8):
        m.search()
        T = 1.0 if ply < 30 else 0.0
        probs = m.getActionProbabilities(T)
        act = m.selectAction(True, T)
        r = ref["moves"][ply]
        assert (act, bits(probs), bits([m.getRootValue()])[0]) == (r["action"], r["probs"], r["value"]), ply
        m.updateWithMove(act)
        if ply % 2 == 0:
            m.addDirichletNoise(0.03, 0.25)


@pytest.mark.gpu
def test_gpu_selfplay_manager_python_network_matches_oracle():
    """SelfPlayManager.generateGames with a Python NeuralNetwork subclass (the leaves of every
    simulation step go to its predictBatch as states rebuilt from the moves the engine reports),
    setBatchConfig(2, 5) capping the network batch at two game slots for five games: every record
    equals the CPU restatement with the same evaluator."""
    az = pytest.importorskip("_alphazero_cpp")
    import az_oracle as O

    class HashEvaluator(az.NeuralNetwork):
        def __init__(self):
            super().__init__()
            self.batches = []

        def predict(self, state):
            return _hash_eval(state.getHash(), list(state.getMoveHistory()), state.getActionSpaceSize())

        def predictBatch(self, states):
            self.batches.append(len(states))
            out = [self.predict(s) for s in states]
            return [list(map(float, o[0])) for o in out], [o[1] for o in out]

    total, bs, sims, max_moves = 5, 7, 48, 12
    refs = O.play(seed_stride=1, bs=bs, sims=sims, max_moves=max_moves, eval_kind=O.EVAL_HASH, n_games=total)
    net = HashEvaluator()
    mgr = az.SelfPlayManager(net, total, sims, 4)
    mgr.setBatchConfig(2, 5)
    mgr.setMaxMoves(max_moves)
    mgr.setSeeds(42, 1)
    recs = mgr.generateGames(az.GameType.GOMOKU, bs, False)
    assert len(recs) == total
    for g, (rec, ref) in enumerate(zip(recs, refs)):
        mv = rec.getMoves()
        assert len(mv) == len(ref["moves"]), g
        for ply, (m, r) in enumerate(zip(mv, ref["moves"])):
            assert (m.action, bits(m.policy), bits([m.value])[0]) == (r["action"], r["probs"], r["value"]), (g, ply)
    assert max(net.batches) == 2


@pytest.mark.gpu
def test_gpu_callback_failure_then_retry_matches_oracle(engine):
    """A host evaluator that raises once, in the root expansion of the first addDirichletNoise: the
    call fails with AzError and leaves the roots unexpanded (roots_ready is set only after a root
    step completes), so the retried call expands the roots, then draws and mixes the noise exactly
    as the reference's addDirichletNoise -> expandNode does; the game then matches the oracle bit
    for bit (the failed attempt's TT lookup is not in the oracle's counters, so those are skipped)."""
    import az_amd
    import az_oracle as O
    bs, sims, n = 9, 60, 2
    refs = O.play(seed_stride=1, bs=bs, sims=sims, max_moves=4, eval_kind=O.EVAL_REPLAY, n_games=n,
                  evaluator=lambda g, planes: plane_eval(planes))
    state = {"fail": 1, "calls": 0}

    def cb(games, moves, planes):
        state["calls"] += 1
        if state["fail"]:
            state["fail"] -= 1
            raise RuntimeError("evaluator unavailable (once)")
        out = [plane_eval(planes[i]) for i in range(len(games))]
        return np.stack([o[0] for o in out]), np.array([o[1] for o in out], np.float32)

    m = az_amd.ParallelMCTS(engine, n_games=n, board_size=bs, num_simulations=sims, evaluator=az_amd.AZ_EVAL_CALLBACK,
                            callback=cb, noise_seed_stride=1)
    try:
        m.newGames()
        with pytest.raises(az_amd.AzError):
            m.addDirichletNoise(0.03, 0.25)
        assert state["calls"] == 1
        m.addDirichletNoise(0.03, 0.25)                  # the retry: root expansion, then the noise
        assert state["calls"] == 2
        from test_gpu_search import children_rows
        for g in range(n):
            assert children_rows(m, g) == refs[g]["init_root"], g
        play_and_compare(m, refs, n, max_moves=4, start=False, counters=False)
    finally:
        m.close()
