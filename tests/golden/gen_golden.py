#!/usr/bin/env python3
"""Regenerates the search/rules golden fixtures in tests/golden/ from the patched
REFERENCE build (oracle/_ref/ref_harness, built by oracle/build_ref.sh from the
sources under /root/reference).  Run from the repo root:

    oracle/build_ref.sh && python3 tests/golden/gen_golden.py

Fixtures are data only: the harness' JSON output (inputs = case parameters,
outputs = per-move root statistics as raw fp32 bit patterns).
"""
import gzip
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
OUT = os.path.dirname(os.path.abspath(__file__))

# (bs, sims, max_moves, evaluator, eval_seed, noise_each_search, cpuct, fpu)
GAME_CASES = [
    (9, 100, 1000, "hash", 7, 0, 1.5, 0.0),      # C1-shaped: 9x9, 100 sims, full game
    (5, 300, 1000, "hash", 7, 0, 1.5, 0.0),      # deep trees -> transposition hits
    (6, 400, 1000, "hash", 7, 0, 1.5, 0.0),
    (4, 500, 1000, "hash", 3, 0, 1.5, 0.0),      # draw (board full), many TT hits
    (7, 200, 1000, "random", 11, 0, 1.5, 0.0),   # the reference's RandomPolicyNetwork
    (6, 150, 1000, "hash", 7, 1, 1.5, 0.25),     # useDirichletNoise per search + FPU
    (15, 200, 6, "hash", 7, 0, 2.0, 0.0),        # 15x15 opening
    (15, 800, 2, "hash", 5, 0, 1.5, 0.0),        # C3 shape: 15x15, 800 sims
]


def run(*args):
    r = subprocess.run([HARNESS] + [str(a) for a in args], capture_output=True, text=True, timeout=900)
    if r.returncode != 0:
        sys.exit(f"harness failed: {args}: {r.stderr}")
    return json.loads(r.stdout)


def main():
    if not os.path.exists(HARNESS):
        sys.exit("build oracle/_ref/ref_harness first (oracle/build_ref.sh)")
    games = []
    for c in GAME_CASES:
        d = run("game", *c)
        d["case"] = list(c)
        games.append(d)
        print("game", c, "moves", len(d["moves"]), "result", d["result"])
    with gzip.open(os.path.join(OUT, "ref_games.json.gz"), "wt") as f:
        json.dump(games, f, separators=(",", ":"))
    pos = {str(bs): run("positions", bs, n, seed) for bs, n, seed in [(9, 48, 1), (15, 48, 2), (5, 32, 3)]}
    with gzip.open(os.path.join(OUT, "ref_positions.json.gz"), "wt") as f:
        json.dump(pos, f, separators=(",", ":"))
    gam = run("gamma", 0.03, 225, 6)
    with open(os.path.join(OUT, "ref_gamma.json"), "w") as f:
        json.dump(gam, f, separators=(",", ":"))
    print("wrote", OUT)


if __name__ == "__main__":
    main()
