#!/usr/bin/env python3
"""Phase stamps of k_select / k_expand_backup for one game (AZ_TREE_STAMPS=<game>) in the C2 workload
(256 games, 400 sims, 6x64 fp16 net) or Go 19x19 (AZ_STAMPS_GO=1: the C4 net shape with 2 blocks -- the
tree phases do not depend on the trunk): the last simulation step of a move, in microseconds and
shader cycles between consecutive stamps.  usage: tree_stamps.py [games] [sims] [moves]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-multi-game_amd"))
import az_amd  # noqa: E402
from az_amd import _lib  # noqa: E402

G = int(sys.argv[1]) if len(sys.argv) > 1 else 256
sims = int(sys.argv[2]) if len(sys.argv) > 2 else 400
moves = int(sys.argv[3]) if len(sys.argv) > 3 else 3
_lib.lib().az_diag_set_tree_stamps(int(os.environ.get("AZ_TREE_STAMPS", "137")))
eng = az_amd.Engine(0)
if os.environ.get("AZ_STAMPS_GO"):
    desc = az_amd.NetDesc(19, 8, 256, 2, 362, 32, 8, 256, 1, 0, az_amd.AZ_PREC_FP16, G)
    net = az_amd.HipNeuralNetwork(eng, desc)
    net.init_random(1)
    m = az_amd.ParallelMCTS(eng, net=net, n_games=G, board_size=19, num_simulations=sims, evaluator=az_amd.AZ_EVAL_NET,
                            game=az_amd.AZ_GAME_GO)
else:
    net = az_amd.HipNeuralNetwork(eng, az_amd.gomoku_net_desc(board_size=15, channels=64, blocks=6, max_batch=G))
    net.init_random(1)
    m = az_amd.ParallelMCTS(eng, net=net, n_games=G, board_size=15, num_simulations=sims, evaluator=az_amd.AZ_EVAL_NET)
m.newGames()
m.addDirichletNoise(0.03, 0.25)
for _ in range(moves):
    m.selfplayStep()
buf = (ctypes.c_ulonglong * 128)()
_lib.lib().az_diag_tree_stamps(buf, 128)
st = list(buf)
names = {0: ["prologue loads issued", "root record", "descent", "leaf board", "terminal test", "TT probe",
             "planes + outputs", "counters / end"],
         1: ["prologue loads issued", "status", "leaf board", "legal moves", "softmax", "prior gather",
             "TT store + children", "backup / end"]}
extra = {1: {8: "  (softmax: logits in, max)", 9: "  (wave max)", 10: "  (exp, stores, barrier)", 11: "  (sequential sum)",
             12: "  (gather, stores, barrier)", 13: "  (sequential sum)"}}
for k, kname in ((0, "k_select"), (1, "k_expand_backup")):
    row = st[64 * k: 64 * k + 64]
    print(kname)
    marks = [(row[i], i, n) for i, n in enumerate(names[k]) if row[i]]
    marks += [(row[i], i, n) for i, n in extra.get(k, {}).items() if row[i]]
    marks.sort()
    prev = None
    for ts, i, n in marks:
        if prev is not None:
            dt = (ts - row[prev]) / 100.0
            cyc = row[32 + i] - row[32 + prev]
            print(f"  {n:28s} {dt:7.2f} us {cyc:7d} cyc")
        prev = i
