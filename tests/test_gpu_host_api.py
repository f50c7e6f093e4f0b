"""The C++ host API (_alphazero_cpp) on the GPU: ParallelMCTS / SelfPlayManager /
HipNeuralNetwork reproduce the reference's own golden games and the oracle bit for bit,
through the same classes and methods a reference user calls."""
import gzip
import json
import os

import numpy as np
import pytest

az = pytest.importorskip("_alphazero_cpp", reason="build the host module: make -C alphazero-multi-game_amd")
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def bits(a):
    return np.asarray(a, np.float32).view(np.uint32).tolist()


def host_play(m, moves, n=None):
    """SelfPlayManager::playSingleGame's loop (self_play_manager.cpp:184-215) on a ParallelMCTS, in
    the deterministic mode the reference harness sets (useBatchInference, rng_ seeded 42)."""
    m.setDeterministicMode(True)
    m.addDirichletNoise(0.03, 0.25)
    out = []
    for ply in range(len(moves) if n is None else n):
        m.search()
        T = 1.0 if ply < 30 else 0.0
        probs = m.getActionProbabilities(T)
        act = m.selectAction(True, T)
        val = m.getRootValue()
        out.append((act, bits(probs), bits([val])[0]))
        m.updateWithMove(act)
        if ply % 2 == 0:
            m.addDirichletNoise(0.03, 0.25)
    return out


@pytest.mark.gpu
def test_host_parallel_mcts_random_policy_matches_reference_golden():
    """RandomPolicyNetwork(seed) game of the patched reference (7x7, 200 sims) through
    ParallelMCTS(GomokuState, RandomPolicyNetwork)."""
    games = json.load(gzip.open(os.path.join(GOLD, "ref_games.json.gz"), "rt"))
    ref = next(g for g in games if g["case"][3] == "random")
    bs, sims, _, _, seed, _, cp, fpu = ref["case"]
    net = az.RandomPolicyNetwork(az.GameType.GOMOKU, bs, seed)
    m = az.ParallelMCTS(az.GomokuState(bs), net, None, 1, sims, cp, fpu, 3)
    got = host_play(m, ref["moves"])
    for ply, (g, r) in enumerate(zip(got, ref["moves"])):
        assert g == (r["action"], r["probs"], r["value"]), ply


@pytest.mark.gpu
def test_host_parallel_mcts_without_network_matches_oracle():
    """nn = nullptr: evaluateState's uniform fallback (parallel_mcts.cpp:903-916)."""
    import az_oracle as O
    ref = O.play(bs=9, sims=100, max_moves=12, eval_kind=O.EVAL_UNIFORM)[0]
    cfg = az.MCTSConfig()
    cfg.numSimulations = 100
    tt = az.TranspositionTable(1 << 20)
    m = az.ParallelMCTS(az.GomokuState(9), cfg, None, tt)
    got = host_play(m, ref["moves"])
    for ply, (g, r) in enumerate(zip(got, ref["moves"])):
        assert g == (r["action"], r["probs"], r["value"]), ply
    assert tt.getLookups() == ref["moves"][-1]["tt_lookups"] and tt.getHits() == ref["moves"][-1]["tt_hits"]
    top = m.analyzePosition(3)
    assert len(top) <= 3 and all(len(t) == 4 for t in top)


@pytest.mark.gpu
def test_host_selfplay_manager_matches_oracle(tmp_path):
    """SelfPlayManager.generateGames (device driver, 3 slots for 6 games) == the oracle's
    playSingleGame records; saved files load back identical."""
    import az_oracle as O
    total, bs, sims, max_moves = 6, 7, 64, 30
    refs = O.play(seed_stride=1, bs=bs, sims=sims, max_moves=max_moves, eval_kind=O.EVAL_RANDOM, eval_seed=5,
                  n_games=total)
    net = az.RandomPolicyNetwork(az.GameType.GOMOKU, bs, 5)
    mgr = az.SelfPlayManager(net, total, sims, 4)
    mgr.setConcurrentGames(3)
    mgr.setMaxMoves(max_moves)
    mgr.setSeeds(42, 1)
    mgr.setSaveGames(True, str(tmp_path))
    calls = []
    mgr.setProgressCallback(lambda g, mv, tg, tm: calls.append((g, mv, tg, tm)))
    recs = mgr.generateGames(az.GameType.GOMOKU, bs, False)
    assert len(recs) == total and mgr.getCompletedGamesCount() == total and not mgr.isRunning()
    for g, (rec, ref) in enumerate(zip(recs, refs)):
        mv = rec.getMoves()
        assert len(mv) == len(ref["moves"]), g
        for ply, (m, r) in enumerate(zip(mv, ref["moves"])):
            assert (m.action, bits(m.policy), bits([m.value])[0]) == (r["action"], r["probs"], r["value"]), (g, ply)
        assert int(rec.getResult()) == (ref["result"] if ref["terminal"] else 0)
    assert len(calls) == mgr.getTotalMovesCount() == sum(len(r["moves"]) for r in refs)
    files = sorted(os.listdir(tmp_path))
    assert len(files) == total and files[0].startswith("000_")
    back = az.GameRecord.loadFromFile(str(tmp_path / files[0]))
    assert [m.action for m in back.getMoves()] == [m.action for m in recs[0].getMoves()]


@pytest.mark.gpu
def test_host_selfplay_manager_shard_matches_oracle(tmp_path):
    """SelfPlayManager.setShard (one rank's share of a per-GPU job, shardGames): rank 1 of 2 over 7
    global games plays ids 4..6 -- the oracle's records of those ids (noise / evaluator streams by
    global id), its record files named by the global id."""
    import az_oracle as O
    total, bs, sims, max_moves = 7, 7, 48, 20
    refs = O.play(seed_stride=1, bs=bs, sims=sims, max_moves=max_moves, eval_kind=O.EVAL_RANDOM, eval_seed=5,
                  n_games=total)
    sh = az.shardGames(1, 2, total)
    assert (sh.firstGame, sh.numGames, sh.noiseSeed) == (4, 3, 46)
    mgr = az.SelfPlayManager(az.RandomPolicyNetwork(az.GameType.GOMOKU, bs, 5), 100, sims, 4)
    mgr.setShard(sh)
    mgr.setMaxMoves(max_moves)
    mgr.setSaveGames(True, str(tmp_path))
    recs = mgr.generateGames(az.GameType.GOMOKU, bs, False)
    assert len(recs) == 3 and mgr.getFirstGameId() == 4
    for k, rec in enumerate(recs):
        ref = refs[4 + k]
        got = [(m.action, bits(m.policy), bits([m.value])[0]) for m in rec.getMoves()]
        assert got == [(r["action"], r["probs"], r["value"]) for r in ref["moves"]], 4 + k
    assert sorted(f[:3] for f in os.listdir(tmp_path)) == ["004", "005", "006"]


@pytest.mark.gpu
def test_host_hip_network_predict_batch_matches_torch():
    """HipNeuralNetwork.predictBatch (planes built from GomokuState) == softmax of the fp32
    restatement, <= 1e-4 (north_star tolerance) at f32 precision."""
    import net_oracle
    import az_amd
    net = az.HipNeuralNetwork(boardSize=15, channels=64, blocks=2, precision=0, maxBatch=8)
    desc = az_amd.gomoku_net_desc(board_size=15, channels=64, blocks=2, max_batch=8)
    blob = net_oracle.init_blob(desc, seed=9)
    net.loadWeights(blob)
    states = []
    rng = np.random.default_rng(2)
    for i in range(5):
        s = az.GomokuState(15)
        for _ in range(i * 7):
            s.makeMove(int(rng.choice(s.getLegalMoves())))
        states.append(s)
    pol, val = net.predictBatch(states)
    x = np.stack([np.asarray(s.getEnhancedTensorRepresentation(), np.float32) for s in states])
    rl, rv = net_oracle.forward(desc, blob, x)
    assert np.abs(np.asarray(pol) - net_oracle.softmax_policy(rl)).max() <= 1e-4
    assert np.abs(np.asarray(val) - rv).max() <= 1e-4
    p1, v1 = net.predict(states[3])
    assert np.allclose(p1, pol[3]) and abs(v1 - val[3]) < 1e-6
    assert net.isGpuAvailable() and net.getBatchSize() == 8 and "MI355X" in net.getDeviceInfo()


@pytest.mark.gpu
def test_host_go_parallel_mcts_and_selfplay_match_oracle():
    """Go through the C++ host API: ParallelMCTS(GoState, RandomPolicyNetwork) and
    SelfPlayManager.generateGames(GO) reproduce the oracle's GoState games bit for bit."""
    import az_oracle as O
    bs, sims, mm = 9, 120, 24
    ref = O.play(bs=bs, sims=sims, max_moves=mm, eval_kind=O.EVAL_RANDOM, eval_seed=5, game=O.GAME_GO)[0]
    net = az.RandomPolicyNetwork(az.GameType.GO, bs, 5)
    m = az.ParallelMCTS(az.GoState(bs), net, None, 1, sims, 1.5, 0.0, 3)
    got = host_play(m, ref["moves"])
    for ply, (g, r) in enumerate(zip(got, ref["moves"])):
        assert g == (r["action"], r["probs"], r["value"]), ply
    total = 4
    refs = O.play(seed_stride=1, bs=bs, sims=64, max_moves=mm, eval_kind=O.EVAL_RANDOM, eval_seed=5, n_games=total,
                  game=O.GAME_GO)
    mgr = az.SelfPlayManager(az.RandomPolicyNetwork(az.GameType.GO, bs, 5), total, 64, 4)
    mgr.setConcurrentGames(2)
    mgr.setMaxMoves(mm)
    mgr.setSeeds(42, 1)
    recs = mgr.generateGames(az.GameType.GO, bs, False)
    assert len(recs) == total
    for g, (rec, r) in enumerate(zip(recs, refs)):
        mv = rec.getMoves()
        assert [(x.action, bits(x.policy), bits([x.value])[0]) for x in mv] == \
               [(y["action"], y["probs"], y["value"]) for y in r["moves"]], g
        assert int(rec.getResult()) == (r["result"] if r["terminal"] else 0)


@pytest.mark.gpu
def test_host_dataset_from_selfplay_matches_oracle(tmp_path):
    """Dataset (dataset.cpp) through the host API: generateGames records -> extractExamples
    (device replay + 8-fold augmentation, written into std::shuffle's slots) == the oracle's
    examples permuted by the same libstdc++ shuffle; getBatch / getRandomSubset / shuffle draw
    from the same rng_; save/load round trip."""
    import az_oracle as O
    total, bs, sims = 4, 7, 48
    net = az.RandomPolicyNetwork(az.GameType.GOMOKU, bs, 5)
    mgr = az.SelfPlayManager(net, total, sims, 4)
    mgr.setMaxMoves(24)
    recs = mgr.generateGames(az.GameType.GOMOKU, bs, False)
    ds = az.Dataset()
    ds.setSeed(77)
    for r in recs:
        ds.addGameRecord(r)
    ds.extractExamples(True)
    E = ds.size()
    ref = O.dataset(0, bs, [([m.action for m in r.getMoves()], [m.policy for m in r.getMoves()],
                             int(r.getResult())) for r in recs])
    assert E == len(ref[0]) == 8 * sum(len(r.getMoves()) for r in recs)
    orders = O.shuffle_orders(77, E, 4)
    slot = [x[orders[0]] for x in ref]
    ex = ds.getExamples()
    for i in (0, 1, E // 2, E - 1):
        assert bits(np.asarray(ex[i].state).reshape(-1)) == bits(slot[0][i].reshape(-1))
        assert bits(ex[i].policy) == bits(slot[1][i, :slot[2][i]])
        assert bits([ex[i].value]) == bits([slot[3][i]])
    st, pol, val = ds.getBatch(16)
    idx = orders[1][:16]
    assert bits(np.asarray(st).reshape(-1)) == bits(slot[0][idx].reshape(-1))
    assert bits(val) == bits(slot[3][idx])
    sub = ds.getRandomSubset(3)
    assert [bits([e.value])[0] for e in sub] == bits(slot[3][orders[2][:3]])
    ds.shuffle()
    ex2 = ds.getExamples()
    perm = slot[3][orders[3]]
    assert bits([e.value for e in ex2]) == bits(perm)
    f = str(tmp_path / "d.json")
    assert ds.saveToFile(f)
    ds2 = az.Dataset()
    assert ds2.loadFromFile(f)
    assert ds2.size() == E
    ex3 = ds2.getExamples()
    assert all(bits(np.asarray(a.state).reshape(-1)) == bits(np.asarray(b.state).reshape(-1)) for a, b in zip(ex2[:8], ex3[:8]))
    assert bits([e.value for e in ex3]) == bits(perm)


@pytest.mark.gpu
def test_host_api_script_matches_reference():
    """The host ParallelMCTS runs the reference's API script (tests/golden/ref_api.json.gz case 1,
    RandomPolicyNetwork): noise, search, releaseMemory, stochastic selectAction after
    setConfig(useBatchInference = false) (tree and rng_ kept); root statistics through
    getRootNode() (the MCTSNode snapshot) bit for bit after every operation."""
    case = json.load(gzip.open(os.path.join(GOLD, "ref_api.json.gz"), "rt"))[1]
    bs, sims, script, ev, seed = case["case"]
    assert ev == "random"
    cfg = az.MCTSConfig()
    cfg.numSimulations = sims
    st = az.GomokuState(bs)
    net = az.RandomPolicyNetwork(az.GameType.GOMOKU, bs, seed)
    m = az.ParallelMCTS(st, cfg, net, az.TranspositionTable(1 << 20))
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
        elif c == "d":                                      # setConfig keeps the tree and rng_
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
    assert "Node: V=" in m.getRootNode().toString(1)


@pytest.mark.gpu
def test_host_create_ddw_randwire():
    """createDDWRandWireResNet (TorchNeuralNetwork::createDDWRandWireResNet,
    torch_neural_network.cpp:799-814) through the host module: predictBatch on GomokuStates ==
    softmax of the rand-wire oracle (pinned to the reference C++ module), and ParallelMCTS searches
    with it."""
    import az_amd
    import net_oracle
    import randwire_oracle as RW
    net = az.createDDWRandWireResNet(11, 81, channels=16, num_blocks=2, board_size=9, max_batch=4)
    net.initRandom(5)
    desc = az_amd.randwire_net_desc(9, 16, 2, 11, 4)
    blob = RW.init_blob(desc, RW.load_graphs(), 5)
    states = []
    rng = np.random.default_rng(3)
    for i in range(4):
        s = az.GomokuState(9)
        for _ in range(i * 5):
            s.makeMove(int(rng.choice(s.getLegalMoves())))
        states.append(s)
    pol, val = net.predictBatch(states)
    x = np.stack([np.asarray(s.getEnhancedTensorRepresentation(), np.float32) for s in states])
    rl, rv = RW.forward(desc, RW.load_graphs(), blob, x)
    assert np.abs(np.asarray(pol) - net_oracle.softmax_policy(rl)).max() <= 1e-4
    assert np.abs(np.asarray(val) - rv).max() <= 1e-4
    m = az.ParallelMCTS(az.GomokuState(9), net, None, 1, 64, 1.5, 0.0, 3)
    m.setDeterministicMode(True)
    m.search()
    probs = np.asarray(m.getActionProbabilities(1.0), np.float64)
    assert abs(probs.sum() - 1.0) < 1e-5 and m.selectAction(True, 1.0) in az.GomokuState(9).getLegalMoves()


@pytest.mark.gpu
def test_host_rng_survives_rebuild():
    """setNeuralNetwork / setTranspositionTable rebuild the device handle; rng_ carries over whole
    (az_search_get_rng / az_search_set_rng), as the reference's setters leave rng_ alone: after
    three stochastic draws and a rebuild, the next draws equal those of an object never rebuilt
    (same root, same fresh-evaluator search)."""
    bs, sims = 9, 64
    draws = []
    for rebuild in (False, True):
        cfg = az.MCTSConfig()
        cfg.numSimulations = sims
        net = az.RandomPolicyNetwork(az.GameType.GOMOKU, bs, 7)
        m = az.ParallelMCTS(az.GomokuState(bs), cfg, net, az.TranspositionTable(1 << 16))
        m.setDeterministicMode(True)
        cfg2 = az.MCTSConfig()
        cfg2.numSimulations = sims
        cfg2.useBatchInference = False
        m.setConfig(cfg2)
        first = [m.selectAction(True, 1.0) for _ in range(3)]
        if rebuild:
            m.setNeuralNetwork(net)                   # new handle: tree reset, rng_ kept
            m.setTranspositionTable(az.TranspositionTable(1 << 16))
        draws.append((first, [m.selectAction(True, 1.0) for _ in range(8)]))
    assert draws[0] == draws[1]


@pytest.mark.gpu
def test_host_setters_keep_the_tree():
    """setNeuralNetwork / setTranspositionTable keep the tree, as the reference's setters only
    replace nn_ / tt_ (parallel_mcts.cpp:1190-1222): a device net of the same shape is swapped into
    the handle, a new table of the same size empties the device table; the next search adds its
    simulations to the same root."""
    bs, sims = 9, 48
    a = az.HipNeuralNetwork(boardSize=bs, channels=32, blocks=1, precision=0, maxBatch=4)
    a.initRandom(1)
    b = az.HipNeuralNetwork(boardSize=bs, channels=32, blocks=1, precision=0, maxBatch=4)
    b.initRandom(2)
    cfg = az.MCTSConfig()
    cfg.numSimulations = sims
    m = az.ParallelMCTS(az.GomokuState(bs), cfg, a, az.TranspositionTable(1 << 16))
    m.setDeterministicMode(True)
    m.search()
    n0 = m.getRootNode().visitCount
    kids0 = [c.visitCount for c in m.getRootNode().children]
    m.setNeuralNetwork(b)
    assert m.getRootNode().visitCount == n0 and [c.visitCount for c in m.getRootNode().children] == kids0
    m.setTranspositionTable(az.TranspositionTable(1 << 16))
    assert m.getRootNode().visitCount == n0
    m.search()
    assert m.getRootNode().visitCount == 2 * n0      # the second search adds as many visits as the first
    # another trunk of the same board swaps in too; another evaluator kind needs a new handle
    # (history replayed, fresh tree)
    c = az.HipNeuralNetwork(boardSize=bs, channels=64, blocks=2, precision=0, maxBatch=1)
    c.initRandom(3)
    m.setNeuralNetwork(c)
    assert m.getRootNode().visitCount == 2 * n0
    m.setNeuralNetwork(az.RandomPolicyNetwork(az.GameType.GOMOKU, bs, 3))
    assert m.getRootNode().visitCount == 0


def _opening(bs, k, seed):
    import random
    rng = random.Random(seed)
    s = az.GomokuState(bs)
    for _ in range(k):
        s.makeMove(rng.choice(s.getLegalMoves()))
    return s


def _root_bits(m):
    r = m.getRootNode()
    return (r.visitCount, r.virtualLoss, bits([r.valueSum])[0],
            [(a, c.visitCount, c.virtualLoss, bits([c.valueSum])[0], bits([c.prior])[0]) for a, c in zip(r.actions, r.children)])


def _play(objs, moves, stochastic):
    """Each object: search, record its root, select (stochastic draws on rng_ when asked), move, noise."""
    out = [[] for _ in objs]
    for _ in range(moves):
        for i, m in enumerate(objs):
            m.search()
            out[i].append(_root_bits(m))
            a = m.selectAction(True, 1.0)
            out[i].append(a)
            m.updateWithMove(a)
            m.addDirichletNoise(0.03, 0.25)
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("evaluator", ["random", "net"])
def test_search_group_matches_standalone(evaluator):
    """SearchGroup members (one device handle, a slot per object) play exactly what standalone objects
    play -- root statistics bit for bit after every search, the same actions -- sequentially and with
    one thread per member whose concurrent searches batch into shared device runs."""
    import threading
    bs, sims, n, moves = 9, 48, 6, 3
    cfg = az.MCTSConfig()
    cfg.numSimulations = sims
    if evaluator == "random":
        net = az.RandomPolicyNetwork(az.GameType.GOMOKU, bs, 7)
    else:
        net = az.HipNeuralNetwork(boardSize=bs, channels=32, blocks=1, precision=0, maxBatch=8)
        net.initRandom(4)
    openings = [_opening(bs, k, 100 + k) for k in range(n)]

    def standalone():
        objs = [az.ParallelMCTS(o, cfg, net, az.TranspositionTable(1 << 20)) for o in openings]
        for i, m in enumerate(objs):
            m.setDeterministicMode(True)
            if i % 2:
                c2 = az.MCTSConfig()
                c2.numSimulations = sims
                c2.useBatchInference = False          # stochastic selectAction on rng_
                m.setConfig(c2)
        return objs
    want = _play(standalone(), moves, True)

    group = az.SearchGroup(net, cfg, az.GomokuState(bs), 8)
    members = [az.ParallelMCTS(o, group) for o in openings]
    for i, m in enumerate(members):
        assert m.inGroup()
        m.setDeterministicMode(True)
        if i % 2:
            c2 = az.MCTSConfig()
            c2.numSimulations = sims
            c2.useBatchInference = False              # host-side only: stays in the group
            m.setConfig(c2)
            assert m.inGroup()
    assert group.members() == n
    assert _play(members, moves, True) == want

    # one thread per member: concurrent searches share device runs
    group2 = az.SearchGroup(net, cfg, az.GomokuState(bs), 8)
    group2.setGatherMicros(20000)
    mem2 = [az.ParallelMCTS(o, group2) for o in openings]
    for i, m in enumerate(mem2):
        m.setDeterministicMode(True)
        if i % 2:
            c2 = az.MCTSConfig()
            c2.numSimulations = sims
            c2.useBatchInference = False
            m.setConfig(c2)
    got = [None] * n

    def run(i):
        got[i] = _play([mem2[i]], moves, True)[0]
    th = [threading.Thread(target=run, args=(i,)) for i in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert got == want
    assert group2.searches() == n * moves and group2.deviceRuns() < group2.searches()
    # a member whose search parameters change leaves the group (its history replayed)
    mem2[0].setNumSimulations(sims + 16)
    assert not mem2[0].inGroup() and group2.members() == n - 1
