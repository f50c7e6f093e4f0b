#!/usr/bin/env python3
"""How many simulation leaves need the network?  Self-play moves of G Gomoku games (C2 net, random
init) at S sims, then the per-game counters: network evaluations, TT lookups / hits, simulations.
In identity-batch steps every game's leaf is computed; the leaves that do not need the network
(terminal, TT hit) are the work an identity batch wastes.
  python3 tools/tt_probe.py [games] [sims] [moves]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-multi-game_amd"))
import az_amd  # noqa: E402

G = int(sys.argv[1]) if len(sys.argv) > 1 else 256
S = int(sys.argv[2]) if len(sys.argv) > 2 else 800
M = int(sys.argv[3]) if len(sys.argv) > 3 else 12
eng = az_amd.Engine(0)
net = az_amd.HipNeuralNetwork(eng, az_amd.gomoku_net_desc(board_size=15, channels=64, blocks=6,
                                                            precision=az_amd.AZ_PREC_FP16, max_batch=G))
net.init_random(1)
m = az_amd.ParallelMCTS(eng, net=net, n_games=G, board_size=15, num_simulations=S, evaluator=az_amd.AZ_EVAL_NET)
m.newGames()
m.addDirichletNoise(0.03, 0.25)
for mv in range(M):
    m.selfplayStep()
    if mv in (0, M // 2, M - 1):
        c = [m.counters(g) for g in range(G)]
        tot = {k: sum(x[k] for x in c) for k in c[0]}
        print(f"after move {mv + 1}: " + ", ".join(f"{k} {v}" for k, v in tot.items()) +
              f"; evals / sims {tot['evals'] / max(1, tot['sims']):.4f}, tt hits / lookups "
              f"{tot['tt_hits'] / max(1, tot['tt_lookups']):.4f}", flush=True)
