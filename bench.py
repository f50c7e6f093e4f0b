#!/usr/bin/env python3
"""bench.py -- self-play positions/s (+ NN evals/s) at 800 sims/move on MI355X.

Workload (BASELINE.json configs[2], "C3"): Gomoku 15x15, 20-block x 256-filter residual
policy/value net, 2048 concurrent games per GPU, 800 simulations per move, the
reference's playSingleGame loop (Dirichlet noise, temperature schedule, subtree
reuse, per-game transposition table).  One step = one committed move of every game
(800 batched simulations: PUCT select -> leaf batch through the ConvNet -> expand /
backup).  Games shard across ranks with no data-path collective (weak scaling:
2048 games per GPU); RCCL only broadcasts the weights and reduces counters.

Synthetic data: games start from the empty board; weights are random-init of the
named architecture (counter-based generator, identical on every rank).

--game go: the C4 workload (BASELINE.json configs[3]) on one GPU per rank: Go 19x19 (GoState:
captures, ko, superko, area scoring on device), 8 input planes, 362-way policy, 1024 games.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.join(ROOT, "alphazero-multi-game_amd"), os.path.join(ROOT, "oracle")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402

METRIC = "self-play positions/sec (+ NN evals/sec) at 800 sims/move, 1/2/4/8 GPU"
PEAK_TFLOPS = {"bf16x3": 2500.0, "bf16": 2500.0, "fp16": 2500.0, "f32": 157.3}   # dense MFMA peaks, MI355X_MICROARCH.md
PREC = {"f32": 0, "bf16x3": 1, "bf16": 2, "fp16": 3}
KERNEL = {"fp16": "conv3x3_v6<2>", "bf16": "conv3x3_v6<1>", "bf16x3": "conv3x3_v4<0>", "f32": "gemm_f32"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--game", default="gomoku", choices=["gomoku", "go"])
    ap.add_argument("--games", type=int, default=None, help="games per GPU (C3: 2048, C4: 1024)")
    ap.add_argument("--sims", type=int, default=800)
    ap.add_argument("--board", type=int, default=None, help="board size (Gomoku 15, Go 19)")
    ap.add_argument("--channels", type=int, default=256)
    ap.add_argument("--blocks", type=int, default=20)
    ap.add_argument("--precision", default="fp16", choices=list(PREC),
                    help="trunk precision: fp16 = the reference useFp16 option (fp16 MFMA operands, fp32 accumulate, "
                         "~2^-20 residual stream; C3 logits within ~6e-5 of fp32), bf16x3 = fp32-faithful")
    ap.add_argument("--cpu-baseline", type=int, default=1, help="time the CPU oracle on rank 0 at N=1")
    ap.add_argument("--cpu-moves", type=int, default=2)   # ~13 s of CPU work at C3
    ap.add_argument("--cpu-sims", type=int, default=None,
                    help="simulations of the CPU sample move (default: --sims for Gomoku, 100 for Go 19x19); a "
                         "shorter sample is scaled to --sims by its evaluations/s")
    ap.add_argument("--seed", type=int, default=1234)
    return ap.parse_args()


def cpu_baseline(desc, blob, board, sims, moves, game="gomoku", sample_sims=None):
    """The CPU restatement (oracle/, Mode S, one game) with the fp32 PyTorch-CPU network
    evaluating one state per call, as the reference's ParallelMCTS::evaluateState does."""
    import torch
    import az_oracle as O
    import net_oracle
    model = net_oracle.Model(desc, blob)
    calls = [0]

    def ev(game, planes):
        calls[0] += 1
        lo, v = model(planes[None])
        return lo[0], float(v[0])

    ev(0, np.zeros((desc.in_planes, board, board), np.float32))   # warm-up
    calls[0] = 0
    ss = sample_sims or sims
    t0 = time.perf_counter()
    O.play(bs=board, sims=ss, max_moves=moves, eval_kind=O.EVAL_NET, evaluator=ev,
           game=O.GAME_GO if game == "go" else O.GAME_GOMOKU)
    dt = time.perf_counter() - t0
    eps = calls[0] / dt
    value = moves / dt if ss == sims else eps / (sims + 1)      # one evaluation per simulation + the root
    return {"value": value, "unit": "positions/s", "cores": torch.get_num_threads(), "kind": "port",
            "evals_per_s": eps,
            "sample": ("" if ss == sims else f"scaled to {sims} sims/move from ") +
                      f"1 game x {moves} move(s) x {ss} sims, {game.capitalize()} {board}x{board}, {desc.blocks}b x "
                      f"{desc.channels}f fp32 net on PyTorch-CPU (B=1 per evaluation), oracle/ Mode S search; "
                      f"{calls[0]} evaluations in {dt:.1f} s"}


def main():
    a = parse()
    go = a.game == "go"
    if a.board is None:
        a.board = 19 if go else 15
    if a.games is None:
        a.games = 1024 if go else 2048
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", init_method="env://")

    import az_amd
    import net_oracle
    eng = az_amd.Engine(local)
    if go:
        desc = az_amd.NetDesc(a.board, 8, a.channels, a.blocks, a.board * a.board + 1, 32, 8, 256, 1, 0,
                              PREC[a.precision], a.games)
    else:
        desc = az_amd.gomoku_net_desc(board_size=a.board, channels=a.channels, blocks=a.blocks,
                                      precision=PREC[a.precision], max_batch=a.games)
    net = az_amd.HipNeuralNetwork(eng, desc)
    from az_amd import dist as azdist
    blob = None
    if dist is None:
        net.init_random(a.seed)
    else:
        blob = net_oracle.init_blob(desc, a.seed) if rank == 0 else None
        blob = azdist.broadcast_weights(dist, blob, net.num_params, f"cuda:{local}")   # RCCL over xGMI, once
        net.load_weights(blob)
    sh = azdist.shard(rank, a.games)       # global game ids / seeds of this rank
    m = az_amd.ParallelMCTS(eng, n_games=a.games, board_size=a.board, num_simulations=a.sims,
                            evaluator=az_amd.AZ_EVAL_NET, net=net, noise_seed=sh["noise_seed"],
                            noise_seed_stride=sh["noise_seed_stride"],
                            game=az_amd.AZ_GAME_GO if go else az_amd.AZ_GAME_GOMOKU)
    m.newGames()
    m.addDirichletNoise(0.03, 0.25)
    for _ in range(a.warmup):
        m.selfplayStep()

    def barrier():
        if dist is not None:
            dist.barrier()
    barrier()
    net.profile(True)
    m.profile(True)
    t0 = time.perf_counter()
    moves = evals = 0
    for _ in range(a.steps):
        mv, ev = m.selfplayStep()
        moves += mv
        evals += ev
    elapsed = time.perf_counter() - t0     # selfplayStep returns after a stream sync
    barrier()
    trunk_ms, launches, forwards = net.profile_read()
    tree = m.profile_read()

    if dist is not None:
        elapsed, (moves, evals) = azdist.reduce_counters(dist, elapsed, [moves, evals], f"cuda:{local}")

    if rank == 0:
        HW = a.board * a.board
        conv_flops_per_eval = 2 * a.blocks * 2.0 * 9 * a.channels * a.channels * HW
        local_evals = evals // max(1, world)
        per_launch_flops = local_evals * conv_flops_per_eval / max(1, launches)
        per_launch_ms = trunk_ms / max(1, launches)
        achieved = per_launch_flops / (per_launch_ms * 1e-3) / 1e12 if launches else 0.0
        peak = PEAK_TFLOPS[a.precision]
        out = {
            "metric": METRIC,
            "value": moves / elapsed,
            "unit": "positions/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": 1e3 * elapsed / a.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": a.precision,
            "data": "synthetic: self-play from empty boards, counter-based random-init weights of the named net",
            "config": {"workload": f"{'C4 Go' if go else 'C3 Gomoku'} {a.board}x{a.board}, {a.blocks}b x "
                                   f"{a.channels}f ResNet, {a.sims} sims/move", "game": a.game,
                       "games_per_gpu": a.games, "global_games": a.games * world,
                       "sims_per_move": a.sims, "board": a.board, "blocks": a.blocks, "channels": a.channels,
                       "parallelism": f"game-shard x{world}"},
            "nn_evals_per_s": evals / elapsed,
            "roofline": {"kernel": f"{KERNEL[a.precision]} ({a.precision} trunk, {a.board}x{a.board})", "bound": "mfma",
                         "achieved": achieved,
                         "peak": peak, "unit": "TFLOP/s", "frac": achieved / peak, "traffic": None,
                         "launches": launches, "avg_launch_ms": per_launch_ms,
                         "flops_per_launch": per_launch_flops},
        }
        steps = max(1, tree["sim_steps"])
        out["tree_kernels"] = {
            name: {"avg_launch_us": 1e3 * tree[f"{k}_ms"] / steps,
                   "bytes_per_launch": tree[f"{k}_bytes"] / steps,
                   "GB_per_s": tree[f"{k}_bytes"] / max(1e-12, 1e-3 * tree[f"{k}_ms"]) / 1e9,
                   "frac_of_hbm_peak": tree[f"{k}_bytes"] / max(1e-12, 1e-3 * tree[f"{k}_ms"]) / 8.0e12}
            for name, k in (("k_select", "select"), ("k_expand_backup", "expand"))}
        out["tree_kernels"]["note"] = ("rank-0 HIP events around each kernel of every simulation step; algorithmic "
                                       "bytes counted by the kernels (child records scanned, path VL/backup "
                                       "read-modify-writes, new nodes, leaf planes); latency-bound (one wave per game, "
                                       "dependent tree levels), peak 8 TB/s; rocprofv3 PMC traffic of the same kernels: "
                                       "profiles/r01e_tree_pmc.json (tools/tree_pmc.sh)")
        tr = pmc_traffic(a, per_launch_flops / (conv_flops_per_eval / (2 * a.blocks)) if launches else 0)
        if tr:
            out["roofline"].update(tr)
        if a.cpu_baseline and world == 1:
            if blob is None:
                blob = net_oracle.init_blob(desc, a.seed)
            out["cpu_baseline"] = cpu_baseline(desc, blob, a.board, a.sims, a.cpu_moves, a.game,
                                               a.cpu_sims or (100 if go else a.sims))
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()


def pmc_traffic(a, boards_per_launch):
    """HBM bytes per trunk launch from the committed rocprofv3 PMC summary of the same kernel
    (profiles/*_trunk_pmc.json: FETCH_SIZE x2 per the gfx950 correction + WRITE_SIZE, measured at
    B boards per launch), scaled to this run's average boards per launch.  None if no summary
    matches the precision / net."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_trunk_pmc.json"))):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if (d.get("precision"), d.get("board"), d.get("channels"), d.get("blocks")) == \
                (a.precision, a.board, a.channels, a.blocks):
            best = (f, d)
    if best is None or boards_per_launch <= 0:
        return None
    f, d = best
    scale = boards_per_launch / d["boards_per_launch"]
    return {"traffic": d["hbm_bytes_per_launch"] * scale, "traffic_unit": "bytes/launch",
            "traffic_source": os.path.relpath(f, ROOT) + f" (PMC at B={d['boards_per_launch']}, scaled x{scale:.4f})"}


if __name__ == "__main__":
    main()
