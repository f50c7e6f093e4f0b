#!/usr/bin/env python3
"""Self-play with the DDW-RandWire net in the loop (row f4 inside the hot path): G Gomoku games on
one GPU, every leaf batch evaluated by az_net_create_randwire's net (the reference default 128 ch x
20 blocks unless given), S simulations per move, full playSingleGame semantics (Dirichlet noise,
temperature schedule, TT, subtree reuse) through ParallelMCTS.selfplayStep -- the same driver as
bench.py.  Prints one JSON line: positions/s, NN evals/s, ms per move.  Not a BASELINE.json config
(those name the plain ResNet); a measurement of the f4 net in the self-play loop."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-multi-game_amd"))
import az_amd  # noqa: E402

PREC = {"f32": az_amd.AZ_PREC_F32, "bf16x3": az_amd.AZ_PREC_BF16X3, "fp16": az_amd.AZ_PREC_FP16}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--games", type=int, default=256)
    ap.add_argument("--sims", type=int, default=100)
    ap.add_argument("--channels", type=int, default=128)
    ap.add_argument("--blocks", type=int, default=20)
    ap.add_argument("--precision", default="bf16x3", choices=list(PREC))
    ap.add_argument("--moves", type=int, default=2)
    a = ap.parse_args()
    eng = az_amd.Engine(int(os.environ.get("LOCAL_RANK", 0)))
    d = az_amd.randwire_net_desc(15, a.channels, a.blocks, 11, a.games)
    d.precision = PREC[a.precision]
    net = az_amd.HipNeuralNetwork(eng, d, randwire=True)
    net.init_random(11)
    m = az_amd.ParallelMCTS(eng, net=net, n_games=a.games, board_size=15, num_simulations=a.sims,
                            evaluator=az_amd.AZ_EVAL_NET, noise_seed=42, noise_seed_stride=1)
    m.newGames()
    m.addDirichletNoise(0.03, 0.25)
    m.selfplayStep()                      # warm-up move
    t0 = time.perf_counter()
    moves = evals = 0
    for _ in range(a.moves):
        mv, ev = m.selfplayStep()
        moves += mv
        evals += ev
    dt = time.perf_counter() - t0
    print(json.dumps({"net": f"DDWRandWireResNet(11, 225, {a.channels}, {a.blocks})", "precision": a.precision,
                      "games": a.games, "sims": a.sims, "moves_timed": a.moves,
                      "positions_per_s": round(moves / dt, 2), "nn_evals_per_s": round(evals / dt, 1),
                      "ms_per_move": round(dt * 1e3 / a.moves, 1)}), flush=True)
    m.close()
    net.close()
    eng.close()


if __name__ == "__main__":
    main()
