#!/usr/bin/env python3
"""Regenerates the search/rules golden fixtures in tests/golden/ from the patched
REFERENCE build (oracle/_ref/ref_harness, built by oracle/build_ref.sh from the
sources under /root/reference).  Run from the repo root:

    oracle/build_ref.sh && python3 tests/golden/gen_golden.py [--only go]

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

# GoState (9/13/19, komi 7.5, Chinese area scoring, positional superko), same tuple layout
GO_GAME_CASES = [
    (9, 100, 80, "hash", 3, 0, 1.5, 0.0),       # 75 plies: captures, ko, ends pass / pass (area scoring)
    (9, 150, 40, "hash", 11, 0, 1.5, 0.0),
    (9, 30, 1000, "hash", 7, 0, 1.5, 0.0),      # sims < children: every child once, pass first -> pass / pass
    (9, 60, 30, "hash", 5, 1, 1.5, 0.25),       # useDirichletNoise per search + FPU
    (13, 300, 8, "hash", 7, 0, 1.5, 0.0),
    (19, 500, 2, "hash", 7, 0, 1.5, 0.0),       # C4 board
]

# ParallelMCTS API scripts (ref_harness api): (bs, sims, script, evaluator, eval_seed)
API_CASES = [
    (9, 30, "n,n,n,s,r3,s,d,a1,m,x,s,a1,m,s,e0,m,n,b,r2,s,a0.5,m,s,a0,m", "hash", 7),
    (7, 60, "x,s,d,a1,m,x,s,a1,m,r5,s,a1,m,s,e0,m,s,a0,m,s,a1,m,s,e1,m", "random", 11),
    (9, 40, "b,a1,m,b,e0,m,r1,s,a0,m,n,n,s,d,a0,m,s,e1,m,r4,s,a1,m", "hash", 5),
    (15, 100, "x,s,r2,s,d,a1,m,x,s,a1,m,s,a0,m", "hash", 3),
    (5, 80, "s,r40,s,a1,m,s,r1000,s,a0,m,d,s,a1,m,s,r2,e0,m", "hash", 9),
]


def run(*args):
    r = subprocess.run([HARNESS] + [str(a) for a in args], capture_output=True, text=True, timeout=900)
    if r.returncode != 0:
        sys.exit(f"harness failed: {args}: {r.stderr}")
    return json.loads(r.stdout)


def main():
    if not os.path.exists(HARNESS):
        sys.exit("build oracle/_ref/ref_harness first (oracle/build_ref.sh)")
    api = []
    for c in API_CASES:
        d = run("api", *c)
        d["case"] = list(c)
        api.append(d)
        print("api", c[:2], c[3], "ops", len(d["ops"]))
    with gzip.open(os.path.join(OUT, "ref_api.json.gz"), "wt") as f:
        json.dump(api, f, separators=(",", ":"))
    if sys.argv[1:] == ["--only", "api"]:
        return
    go = []
    for c in GO_GAME_CASES:
        d = run("go_game", *c)
        d["case"] = list(c)
        go.append(d)
        print("go_game", c, "moves", len(d["moves"]), "result", d["result"])
    with gzip.open(os.path.join(OUT, "ref_go_games.json.gz"), "wt") as f:
        json.dump(go, f, separators=(",", ":"))
    gp = {str(bs): run("go_positions", bs, n, seed) for bs, n, seed in [(9, 64, 1), (13, 24, 2), (19, 12, 3)]}
    with gzip.open(os.path.join(OUT, "ref_go_positions.json.gz"), "wt") as f:
        json.dump(gp, f, separators=(",", ":"))
    if sys.argv[1:] == ["--only", "go"]:
        return
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
