"""GPU parity of the batched HIP search (through the C-ABI) against
  (1) golden vectors of the patched REFERENCE search (tests/golden/ref_games.json.gz), and
  (2) the CPU restatement (oracle/az_oracle.cpp) for multi-game runs with per-game seeds.
Bit-exact: raw N / VL, fp32 bit patterns of W, P, visit distributions and root values,
chosen actions, TT lookup/hit counters and evaluation counts."""
import gzip
import json
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _games():
    with gzip.open(os.path.join(GOLD, "ref_games.json.gz"), "rt") as f:
        return json.load(f)


GAMES = _games()


def bits(a):
    return np.asarray(a, np.float32).view(np.uint32).tolist()


@pytest.fixture(scope="module")
def engine():
    import az_amd
    return az_amd.Engine(0)


def children_rows(m, g):
    act, N, VL, W, P = m.rootChildren(g)
    return [[int(a), int(n), int(v), w, p] for a, n, v, w, p in zip(act, N, VL, bits(W), bits(P))]


def play_and_compare(m, refs, n_games, max_moves=None, start=True, counters=True):
    """Drive the engine with the playSingleGame loop and compare to per-game reference dicts.
    start=False: the caller already ran newGames + the initial noise; counters=False skips the
    TT lookup / hit / evaluation counters."""
    if start:
        m.newGames()
        m.addDirichletNoise(0.03, 0.25)
    for g in range(n_games):
        assert children_rows(m, g) == refs[g]["init_root"], f"init_root game {g}"
    nmoves = max(len(r["moves"]) for r in refs)
    if max_moves is not None:
        nmoves = min(nmoves, max_moves)
    live = [True] * n_games
    for ply in range(nmoves):
        m.search()
        T = 1.0 if ply < 30 else 0.0
        act, val, probs, cact, nch = m.select(True, T)
        for g in range(n_games):
            if not live[g]:
                continue
            r = refs[g]["moves"][ply]
            N, VL, W = m.rootNode(g)
            assert [N, VL, bits([W])[0]] == r["root"], (g, ply, "root")
            assert children_rows(m, g) == r["children"], (g, ply, "children")
            assert bits(probs[g, :nch[g]]) == r["probs"], (g, ply, "probs")
            assert int(act[g]) == r["action"], (g, ply, "action")
            assert bits([val[g]])[0] == r["value"], (g, ply, "value")
            c = m.counters(g)
            if counters:
                assert (c["tt_lookups"], c["tt_hits"], c["evals"]) == (r["tt_lookups"], r["tt_hits"], r["evals"]), \
                    (g, ply)
        act = np.array([act[g] if live[g] else m.none for g in range(n_games)], np.int32)
        term, res = m.updateWithMove(act)
        for g in range(n_games):
            if live[g] and (term[g] or ply + 1 >= len(refs[g]["moves"])):
                if term[g]:
                    assert int(res[g]) == refs[g]["result"], (g, "result")
                live[g] = False
        if ply % 2 == 0:
            m.addDirichletNoise(0.03, 0.25)


@pytest.mark.gpu
@pytest.mark.parametrize("idx", range(len(GAMES)), ids=[str(g["case"]) for g in GAMES])
def test_gpu_search_matches_reference_golden(engine, idx):
    import az_amd
    ref = GAMES[idx]
    bs, sims, mm, ev, es, nes, cp, fpu = ref["case"]
    m = az_amd.ParallelMCTS(engine, n_games=1, board_size=bs, num_simulations=sims, c_puct=cp, fpu_reduction=fpu,
                            evaluator=az_amd.AZ_EVAL_HASH if ev == "hash" else az_amd.AZ_EVAL_RANDOM, eval_seed=es,
                            use_dirichlet_each_search=bool(nes))
    try:
        play_and_compare(m, [ref], 1)
    finally:
        m.close()


@pytest.mark.gpu
@pytest.mark.parametrize("bs,sims,games,ev", [(9, 64, 16, "hash"), (7, 96, 8, "random"), (15, 128, 6, "hash"),
                                              (9, 100, 4, "uniform")])
def test_gpu_multigame_matches_oracle(engine, bs, sims, games, ev):
    """G independent games with per-game noise seeds (42 + g) and evaluator seeds; "uniform" is
    ParallelMCTS without a network (parallel_mcts.cpp:903-916)."""
    import az_amd
    import az_oracle as O
    kind = {"hash": O.EVAL_HASH, "random": O.EVAL_RANDOM, "uniform": O.EVAL_UNIFORM}[ev]
    dev = {"hash": az_amd.AZ_EVAL_HASH, "random": az_amd.AZ_EVAL_RANDOM, "uniform": az_amd.AZ_EVAL_UNIFORM}[ev]
    max_moves = 40
    refs = O.play(seed_stride=1, bs=bs, sims=sims, max_moves=max_moves, eval_kind=kind, eval_seed=5, n_games=games)
    m = az_amd.ParallelMCTS(engine, n_games=games, board_size=bs, num_simulations=sims, evaluator=dev, eval_seed=5,
                            noise_seed=42, noise_seed_stride=1)
    try:
        play_and_compare(m, refs, games, max_moves)
    finally:
        m.close()


@pytest.mark.gpu
def test_gpu_small_tt_forces_replacement(engine):
    """A 2^6-slot table: collisions and the visits<5 replacement rule on every move."""
    import az_amd
    import az_oracle as O
    refs = O.play(bs=6, sims=300, max_moves=12, eval_kind=O.EVAL_HASH, tt_log2=6)
    m = az_amd.ParallelMCTS(engine, n_games=1, board_size=6, num_simulations=300, evaluator=az_amd.AZ_EVAL_HASH,
                            tt_log2=6)
    try:
        play_and_compare(m, refs, 1, 12)
    finally:
        m.close()


@pytest.mark.gpu
@pytest.mark.parametrize("slots", [3, 8])
def test_gpu_selfplay_run_matches_oracle(engine, slots):
    """az_selfplay_run (the SelfPlayManager::generateGames device driver): 8 games on `slots`
    device slots (finished slots take the next game id) give, game by game, the oracle's
    playSingleGame records -- actions, child-order visit distributions and root values bit for
    bit, results -- independent of the slot count."""
    import az_amd
    import az_oracle as O
    total, bs, sims, max_moves = 8, 7, 64, 30
    refs = O.play(seed_stride=1, bs=bs, sims=sims, max_moves=max_moves, eval_kind=O.EVAL_RANDOM, eval_seed=5,
                  n_games=total)
    mgr = az_amd.SelfPlayManager(engine, numGames=slots, numSimulations=sims, board_size=bs,
                                 evaluator=az_amd.AZ_EVAL_RANDOM, eval_seed=5, noise_seed=42, noise_seed_stride=1)
    seen = []
    mgr.setProgressCallback(lambda gid, mv, tg, tm: seen.append((gid, mv, tg, tm)))
    try:
        recs = mgr.generateGames(totalGames=total, max_moves=max_moves)
    finally:
        mgr.mcts.close()
    assert [r.game_id for r in recs] == list(range(total))
    for g, (rec, ref) in enumerate(zip(recs, refs)):
        assert len(rec.moves) == len(ref["moves"]), g
        for ply, (mv, rm) in enumerate(zip(rec.moves, ref["moves"])):
            assert mv.action == rm["action"], (g, ply)
            assert bits(mv.policy) == rm["probs"], (g, ply)
            assert bits([mv.value])[0] == rm["value"], (g, ply)
            assert len(mv.child_actions) == len(mv.policy)
        assert rec.result == (ref["result"] if ref["terminal"] else 0), g
    assert len(seen) == sum(len(r.moves) for r in recs)
    assert seen[-1][2] == total and seen[-1][3] == len(seen)


@pytest.mark.gpu
def test_gpu_sharded_selfplay_independent_of_rank_count(engine):
    """Two "ranks" (az_amd.dist.shard seeds, 3 games each) play exactly the records a single
    device produces for the same 6 global game ids."""
    import az_amd
    from az_amd import dist as azdist
    bs, sims, max_moves = 7, 48, 20

    def run(n, sh):
        mgr = az_amd.SelfPlayManager(engine, numGames=n, numSimulations=sims, board_size=bs,
                                     evaluator=az_amd.AZ_EVAL_RANDOM, eval_seed=sh["eval_seed"],
                                     noise_seed=sh["noise_seed"], noise_seed_stride=sh["noise_seed_stride"])
        try:
            return mgr.generateGames(totalGames=n, max_moves=max_moves)
        finally:
            mgr.mcts.close()

    one = run(6, azdist.shard(0, 6, eval_seed=5))
    two = run(3, azdist.shard(0, 3, eval_seed=5)) + run(3, azdist.shard(1, 3, eval_seed=5))
    for g, (a, b) in enumerate(zip(one, two)):
        assert [(m.action, bits(m.policy), bits([m.value])[0]) for m in a.moves] == \
               [(m.action, bits(m.policy), bits([m.value])[0]) for m in b.moves], g
        assert a.result == b.result


@pytest.mark.gpu
@pytest.mark.parametrize("ev,slots", [("random", 4), ("hash", 3)])
def test_gpu_selfplay_step_matches_oracle(engine, ev, slots):
    """az_selfplay_step + az_selfplay_step_moves -- the entry point bench.py times -- against the
    oracle's playSingleGame records (self_play_manager.cpp:187-216): `slots` games stepped one move
    at a time for 70 moves with restart_finished (6x6 games end after 25-36 plies, past the T = 0
    drop at 30), every MoveData compared (action, child-order
    visit distribution bits incl. the T = 0 NaNs, root value bits, child actions) with the record
    of the game id its slot plays; a finished slot restarts as the next game id in slot order
    (seeding its noise / evaluator streams by that id), with the noise prefetch on this path."""
    import az_amd
    import az_oracle as O
    bs, sims, steps, total = 6, 48, 70, 24
    kind = O.EVAL_RANDOM if ev == "random" else O.EVAL_HASH
    dev = az_amd.AZ_EVAL_RANDOM if ev == "random" else az_amd.AZ_EVAL_HASH
    refs = O.play(seed_stride=1, bs=bs, sims=sims, eval_kind=kind, eval_seed=5, n_games=total)
    m = az_amd.ParallelMCTS(engine, n_games=slots, board_size=bs, num_simulations=sims, evaluator=dev, eval_seed=5,
                            noise_seed=42, noise_seed_stride=1)
    gid = list(range(slots))            # the game id each slot plays
    ply = [0] * slots
    nxt = slots
    restarts = [0] * slots
    try:
        m.newGames()
        m.addDirichletNoise(0.03, 0.25)
        for step in range(steps):
            mv, _ = m.selfplayStep()
            recs = m.stepMoves(materialize=True)
            assert mv == len(recs) == slots, step            # every slot moves (finished slots restarted)
            assert [s for s, _ in recs] == list(range(slots))
            for s, md in recs:
                assert gid[s] < total, "more games than the oracle played"
                rm = refs[gid[s]]["moves"][ply[s]]
                where = (step, s, gid[s], ply[s])
                assert md.action == rm["action"], where
                assert bits(md.policy) == rm["probs"], where
                assert bits([md.value])[0] == rm["value"], where
                assert list(md.child_actions) == [r[0] for r in rm["children"]], where
                ply[s] += 1
            for s in range(slots):                           # finished: the slot takes the next id
                if ply[s] == len(refs[gid[s]]["moves"]):
                    assert refs[gid[s]]["terminal"], gid[s]
                    gid[s], ply[s], nxt = nxt, 0, nxt + 1
                    restarts[s] += 1
    finally:
        m.close()
    assert min(restarts) >= 1 and sum(restarts) > slots     # every slot restarted, some twice
