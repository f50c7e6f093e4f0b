#!/usr/bin/env python3
"""Progress of a search under rocprofv3 --pmc (tools/pmc_hang_probe2.sh): a handle sized for
--cap-sims simulations per move (node pool, prior ring), --games games, the C3 net cut to --blocks
blocks; then --run-sims simulations in chunks of --chunk, a timestamped line after each (flushed),
so a killed pass shows where it stopped.

--mode step replays what bench.py does instead (newGames, noise, optional net/search profiling,
one az_selfplay_step of --cap-sims simulations, the MoveData fetch), one line per phase; every 15 s
the Python stack is dumped to stderr (faulthandler), so a pass that stops names the call it is in."""
import argparse
import faulthandler
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-multi-game_amd"))
import az_amd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--games", type=int, default=256)
ap.add_argument("--cap-sims", type=int, default=800)
ap.add_argument("--run-sims", type=int, default=800)
ap.add_argument("--chunk", type=int, default=50)
ap.add_argument("--blocks", type=int, default=2)
ap.add_argument("--mode", choices=("sims", "step"), default="sims")
ap.add_argument("--profile", type=int, default=1, help="--mode step: net / search profiling on (bench.py's timed step)")
a = ap.parse_args()
faulthandler.dump_traceback_later(15, repeat=True)
t0 = time.perf_counter()


def say(msg):
    print(f"{time.perf_counter() - t0:8.2f} s  {msg}", flush=True)


if os.environ.get("AZ_STEP_TRACE"):          # phase lines of az_selfplay_step on stderr (diag entry point)
    from az_amd import _lib
    _lib.lib().az_diag_set_step_trace(1)
if os.environ.get("AZ_SYNC_EVERY"):          # host sync every n simulation steps (diag entry point)
    from az_amd import _lib
    _lib.lib().az_diag_set_sync_every(int(os.environ["AZ_SYNC_EVERY"]))
eng = az_amd.Engine(0)
net = az_amd.HipNeuralNetwork(eng, az_amd.gomoku_net_desc(board_size=15, channels=256, blocks=a.blocks,
                                                          precision=az_amd.AZ_PREC_FP16, max_batch=a.games))
net.init_random(1234)
m = az_amd.ParallelMCTS(eng, net=net, n_games=a.games, board_size=15, num_simulations=a.cap_sims,
                        evaluator=az_amd.AZ_EVAL_NET, noise_seed=42, noise_seed_stride=1)
m.newGames()
m.addDirichletNoise(0.03, 0.25)
say(f"created ({a.games} games, capacity {a.cap_sims} sims, mode {a.mode})")
if a.mode == "sims":
    done = 0
    while done < a.run_sims:
        k = min(a.chunk, a.run_sims - done)
        m.runSingleSimulation(k)
        done += k
        say(f"{done} sims")
else:
    if a.profile:
        net.profile(True)
        m.profile(True)
        say("profiling on")
    mv, ev = m.selfplayStep()
    say(f"selfplayStep: {mv} moves, {ev} evals")
    recs, _ = m.stepMoves(materialize=False)
    say(f"stepMoves: {0 if recs is None else len(recs)} records")
    if a.profile:
        say(f"net profile {net.profile_read()}, search profile {m.profile_read()}")
faulthandler.cancel_dump_traceback_later()
print("finished", flush=True)
