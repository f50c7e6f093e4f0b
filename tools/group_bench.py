#!/usr/bin/env python3
"""The reference's object-per-game pattern on the device engine: G host
ParallelMCTS objects, one thread each (as SelfPlayManager's worker threads own one per game,
self_play_manager.cpp:69-89), playing `moves` moves (search, selectAction, updateWithMove, noise):

  group       the G objects are members of one mcts::SearchGroup: concurrent searches batch
  standalone  the G objects each own a single-game handle (capped at --standalone-games objects)
  selfplay    the same G games as ONE multi-game handle stepped by the engine (az_selfplay_step,
              the SelfPlayManager path of bench.py)

Prints positions/s of each and the fractions of the selfplay rate.  Net: 15x15, --channels x
--blocks, fp16 trunk, counter-based random init; --sims simulations per move."""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-multi-game_amd"))
import _alphazero_cpp as az  # noqa: E402
import az_amd  # noqa: E402


def play_threads(objs, moves):
    def run(m):
        for _ in range(moves):
            m.search()
            a = m.selectAction(True, 1.0)
            m.updateWithMove(a)
            m.addDirichletNoise(0.03, 0.25)
    th = [threading.Thread(target=run, args=(m,)) for m in objs]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    return time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--games", type=int, default=64)
    ap.add_argument("--moves", type=int, default=2)
    ap.add_argument("--sims", type=int, default=400)
    ap.add_argument("--channels", type=int, default=64)
    ap.add_argument("--blocks", type=int, default=6)
    ap.add_argument("--standalone-games", type=int, default=8)
    ap.add_argument("--gather-us", type=int, default=2000)
    a = ap.parse_args()
    bs, G = 15, a.games
    cfg = az.MCTSConfig()
    cfg.numSimulations = a.sims
    net = az.HipNeuralNetwork(boardSize=bs, channels=a.channels, blocks=a.blocks, precision=3, maxBatch=G)
    net.initRandom(1234)
    out = {"games": G, "moves": a.moves, "sims": a.sims, "net": f"{a.blocks}b x {a.channels}f fp16, 15x15"}

    group = az.SearchGroup(net, cfg, az.GomokuState(bs), G)
    group.setGatherMicros(a.gather_us)
    members = [az.ParallelMCTS(az.GomokuState(bs), group) for _ in range(G)]
    for m in members:
        m.setDeterministicMode(True)
        m.addDirichletNoise(0.03, 0.25)
    play_threads(members[:1], 1)                       # warm-up (first launches)
    dt = play_threads(members, a.moves)
    out["group"] = {"positions_per_s": (G * a.moves - 0) / dt, "s": dt, "searches": group.searches(),
                    "device_runs": group.deviceRuns()}
    del members

    S = min(a.standalone_games, G)
    solo = [az.ParallelMCTS(az.GomokuState(bs), cfg, net, az.TranspositionTable(1 << 20)) for _ in range(S)]
    for m in solo:
        m.setDeterministicMode(True)
        m.addDirichletNoise(0.03, 0.25)
    dt = play_threads(solo, a.moves)
    out["standalone"] = {"objects": S, "positions_per_s": S * a.moves / dt, "s": dt}
    del solo

    eng = az_amd.Engine(0)
    anet = az_amd.HipNeuralNetwork(eng, az_amd.gomoku_net_desc(board_size=bs, channels=a.channels, blocks=a.blocks,
                                                               precision=az_amd.AZ_PREC_FP16, max_batch=G))
    anet.init_random(1234)
    mc = az_amd.ParallelMCTS(eng, net=anet, n_games=G, board_size=bs, num_simulations=a.sims,
                             evaluator=az_amd.AZ_EVAL_NET, noise_seed=42, noise_seed_stride=1)
    mc.newGames()
    mc.addDirichletNoise(0.03, 0.25)
    mc.selfplayStep()
    t0 = time.perf_counter()
    mv = 0
    for _ in range(a.moves):
        m_, _e = mc.selfplayStep()
        mv += m_
    dt = time.perf_counter() - t0
    out["selfplay"] = {"positions_per_s": mv / dt, "s": dt}
    out["group_fraction_of_selfplay"] = out["group"]["positions_per_s"] / out["selfplay"]["positions_per_s"]
    out["standalone_fraction_of_selfplay"] = out["standalone"]["positions_per_s"] / out["selfplay"]["positions_per_s"]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
