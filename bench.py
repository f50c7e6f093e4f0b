#!/usr/bin/env python3
"""bench.py -- self-play positions/s (+ NN evals/s) at 800 sims/move on MI355X.

Workload (BASELINE.json configs[2], "C3", the default): Gomoku 15x15, 20-block x 256-filter
residual policy/value net, 2048 concurrent games sharded over the N GPUs (2048/N per GPU,
contiguous global game ids), 800 simulations per move, the reference's playSingleGame loop
(Dirichlet noise, temperature schedule, subtree reuse, per-game transposition table).  One step
= one committed move of every game (800 batched simulations: PUCT select -> leaf batch through
the ConvNet -> expand / backup), with the MoveData records of every move assembled on the host.
Games shard across ranks with no data-path collective; RCCL -- the engine's own communicator
(az_dist_*, csrc/dist.hip) -- only broadcasts rank 0's weights into every rank's device weight
buffers, reduces the counters and runs the timing barriers.  `--scaling weak` keeps 2048 games per GPU instead.

  --config c2   BASELINE.json configs[1]: 15x15, 6b x 64f, 256 games, 400 sims, 1 GPU
  --config c4   BASELINE.json configs[3]: Go 19x19 (GoState on device), 8 planes, 362 actions,
                1024 games sharded over the GPUs

Launch: `python bench.py --gpus N` starts N ranks itself (torch.distributed.run, one process
per GPU, 127.0.0.1 rendezvous) unless WORLD_SIZE is already set by a launcher; it fails loudly
when fewer than N GPUs are visible or WORLD_SIZE != N.

Synthetic data: games start from the empty board; weights are the counter-based random init of
the named architecture (az_net_init_random on rank 0, broadcast to the other ranks).

cpu_baseline (rank 0, N=1): the CPU restatement of the reference search (oracle/, Mode S) with the
fp32 PyTorch-CPU network, one game per worker process, one thread each, on the host's CPU share
(self_play_manager.cpp:69-89), timed over a fixed window.
"""
import argparse
import copy
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "alphazero-multi-game_amd")
if PKG not in sys.path:
    sys.path.insert(0, PKG)

import numpy as np  # noqa: E402

T_START = time.perf_counter()

METRIC = "self-play positions/sec (+ NN evals/sec) at 800 sims/move, 1/2/4/8 GPU"
# Measured error of each trunk precision against the fp32 network (profiles/r04_f16x3_net_parity.log:
# tests/test_gpu_trained_scale.py, a trained-like trunk -- per-channel BN scales a decade apart,
# activations growing to ~64 -- with heads scaled to |logit|max 8, |value| 0.9, at each config's batch)
PREC_NOTE = {
    "fp16": "fp16 MFMA operands, fp32 accumulation (the reference's opt-in useFp16, torch_neural_network.h:29); "
            "trained-like max|dlogit| 4.9e-3 (C3), 4.6e-3 (C4), 7.0e-3 (C5) vs the fp32 net: outside the 1e-4 "
            "parity tolerance, see parity_mode for the fp32-faithful rate",
    "f16x3": "fp32-faithful: fp16 hi + lo operands (weights scaled 2^s per output channel), three MFMAs per "
             "product, fp32 accumulation; trained-like max|dlogit| 1.0e-5 (C3), 1.0e-5 (C4), 1.7e-5 (C5) vs "
             "the fp32 net: within the 1e-4 parity tolerance (activations |x| <= 65504, guarded)",
    "bf16x3": "bf16 hi + lo operands, three MFMAs per product, fp32 accumulation (the full fp32 range); "
              "trained-like max|dlogit| 7.5e-5 (C3), 5.6e-5 (C4), 1.4e-4 (C5) vs the fp32 net",
    "f32": "f32 MFMA (exact fp32 products)",
}
PEAK_TFLOPS = {"f16x3": 2500.0, "bf16x3": 2500.0, "bf16": 2500.0, "fp16": 2500.0, "f32": 157.3}   # dense MFMA peaks, MI355X_MICROARCH.md
PREC = {"f32": 0, "bf16x3": 1, "bf16": 2, "fp16": 3, "f16x3": 4}
PARITY_PREC = "f16x3"    # the parity precision parity_mode times
# f16x3 move time / fp16 move time on C3, measured (profiles/r05_bench_c3_closing.json: 38,640 vs 16,169 ms
# = 2.39), with margin: the parity moves' time estimate against --time-budget
PARITY_RATIO = 2.5
# BASELINE.json configs: game, board, blocks, channels, sims/move, global games
CONFIGS = {
    "c2": dict(game="gomoku", board=15, blocks=6, channels=64, sims=400, games=256,
               name="C2 Gomoku 15x15, 6b x 64f ResNet"),
    "c3": dict(game="gomoku", board=15, blocks=20, channels=256, sims=800, games=2048,
               name="C3 Gomoku 15x15, 20b x 256f ResNet"),
    "c4": dict(game="go", board=19, blocks=20, channels=256, sims=800, games=1024,
               name="C4 Go 19x19, 20b x 256f ResNet"),
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default=None, choices=list(CONFIGS), help="BASELINE.json workload (default c3)")
    ap.add_argument("--game", default=None, choices=["gomoku", "go"], help="go = --config c4")
    ap.add_argument("--global-games", type=int, default=None, help="games over all GPUs (C2 256, C3 2048, C4 1024)")
    ap.add_argument("--games", type=int, default=None, help="games per GPU (implies --scaling weak)")
    ap.add_argument("--scaling", default="strong", choices=["strong", "weak"],
                    help="strong: the global games are sharded over the GPUs (BASELINE 'sharded 1/2/4/8'); "
                         "weak: every GPU plays --global-games games")
    ap.add_argument("--sims", type=int, default=None)
    ap.add_argument("--board", type=int, default=None)
    ap.add_argument("--channels", type=int, default=None)
    ap.add_argument("--blocks", type=int, default=None)
    ap.add_argument("--precision", default="fp16", choices=list(PREC),
                    help="trunk precision: fp16 = the reference useFp16 option (fp16 MFMA operands, fp32 accumulate, "
                         "2^-20 residual stream), f16x3 = fp32-faithful (fp16 hi + lo pieces, three MFMAs per "
                         "product), bf16x3 = bf16 hi + lo pieces (the full fp32 range, ~2^-17)")
    ap.add_argument("--cpu-baseline", type=int, default=1, help="time the CPU restatement on rank 0 at N=1")
    ap.add_argument("--cpu-window", type=float, default=20.0, help="seconds of the CPU baseline's timed window")
    ap.add_argument("--cpu-workers", type=int, default=0, help="CPU baseline processes (0: the host's CPU share, <=16)")
    ap.add_argument("--cpu-beside", type=int, default=0,
                    help="1: run the CPU baseline on its own cores beside the GPU warm-up (saves ~30 s; a GPU "
                         "box's CPU share is a quota, so the baseline then reads 0.74-0.89x its value alone)")
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--conv-flags", default=None,
                    help="diagnostic: conv variant bits (hex) OR'd into the library's default flag set "
                         "(az_conv_flags | bits -> az_diag_set_conv_flags) for same-box A/B runs; the trunk "
                         "kernel the run dispatched is named in roofline.kernel")
    ap.add_argument("--parity-steps", type=int, default=2,
                    help="N=1: after the timed moves, switch the live net to the fp32-faithful f16x3 trunk (the parity "
                         "precision) and time this many more moves of the same games, reported as parity_mode; "
                         "0 disables")
    ap.add_argument("--parity-warmup", type=int, default=0,
                    help="untimed parity-precision moves before parity_mode's timed ones (the piece sets are "
                         "packed at load: none needed)")
    ap.add_argument("--time-budget", type=float, default=560.0,
                    help="seconds: parity_mode is skipped (and says so) when the run so far plus its estimated "
                         "time would exceed this (the driver's run limit is 600 s)")
    ap.add_argument("--kernel-timing", type=int, default=1,
                    help="device clock stamps (s_memrealtime, 100 MHz) around sampled trunk / tree launches (the "
                         "roofline); 0 disables (round 3's HIP-event timing hung under rocprofv3 --pmc; the "
                         "stamps do not)")
    ap.add_argument("--sync-every", type=int, default=0,
                    help="diagnostic: a host synchronisation after every N simulation steps (0: none). "
                         "rocprofv3 --pmc stalls on a selfplay step's unsynchronised queue of dispatches "
                         "(DESIGN.md section 7); tools/tree_pmc.sh passes 100")
    ap.add_argument("--streams", type=int, default=1,
                    help="split each rank's games into this many device handles (own engine / HIP stream / net "
                         "each) stepped concurrently by host threads (StreamWorkload)")
    ap.add_argument("--crash-report", default=None,
                    help="diagnostic: on a fault in any thread, append the thread's name, the fault address, the PC "
                         "and /proc/self/maps to this file (az_diag_crash_report), then the previous handler runs")
    ap.add_argument("--dist-timeout", type=float, default=600.0,
                    help="seconds a rank waits in a collective / barrier before the bench fails (N>1)")
    a = ap.parse_args(argv)
    cfg = a.config or ("c4" if a.game == "go" else "c3")
    c = CONFIGS[cfg]
    a.config = cfg
    a.game = c["game"]
    for k in ("board", "blocks", "channels", "sims"):
        if getattr(a, k) is None:
            setattr(a, k, c[k])
    if a.games is not None:
        a.scaling = "weak"
        a.global_games = a.games
    if a.global_games is None:
        a.global_games = c["games"]
    a.workload_name = c["name"]
    return a


# ------------------------------------------------------------------------------- launching
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(a, argv):
    """--gpus N without a launcher: start N ranks with torch.distributed.run as a child process
    (nothing here has touched the GPU; torch.cuda.device_count() does not initialise it)."""
    import torch
    n = torch.cuda.device_count()
    if n < a.gpus:
        print(f"bench.py: --gpus {a.gpus} requested but only {n} GPU(s) are visible", file=sys.stderr)
        return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + list(argv)
    return subprocess.call(cmd)


# ------------------------------------------------------------------------------- GPU workload
class GpuWorkload:
    """The device self-play handle of one rank: HipNeuralNetwork + ParallelMCTS over `games` slots."""

    def __init__(self, a, local, shard):
        import az_amd
        self.eng = az_amd.Engine(local)
        go = a.game == "go"
        if go:
            desc = az_amd.NetDesc(a.board, 8, a.channels, a.blocks, a.board * a.board + 1, 32, 8, 256, 1, 0,
                                  PREC[a.precision], shard["games"])
        else:
            desc = az_amd.gomoku_net_desc(board_size=a.board, channels=a.channels, blocks=a.blocks,
                                          precision=PREC[a.precision], max_batch=shard["games"])
        self.desc = desc
        self.net = az_amd.HipNeuralNetwork(self.eng, desc)
        self.mcts_args = dict(n_games=shard["games"], board_size=a.board, num_simulations=a.sims,
                              evaluator=az_amd.AZ_EVAL_NET, noise_seed=shard["noise_seed"],
                              noise_seed_stride=shard["noise_seed_stride"],
                              game=az_amd.AZ_GAME_GO if go else az_amd.AZ_GAME_GOMOKU)
        self.mcts = None

    def start(self):
        import az_amd
        self.mcts = az_amd.ParallelMCTS(self.eng, net=self.net, **self.mcts_args)
        self.mcts.newGames()
        self.mcts.addDirichletNoise(0.03, 0.25)

    def step(self):
        mv, ev = self.mcts.selfplayStep()
        # the MoveData records of this move, assembled by the engine in C++ as generateGames keeps
        # them (policy, value, action, child actions per game); fetched without building Python
        # objects (per-record Python lists cost ~1.4 ms per C2 move -- a binding cost, not the path's)
        recs, _ = self.mcts.stepMoves(materialize=False)
        assert recs is None or len(recs) == mv
        return mv, ev

    def sync(self):
        pass                           # selfplayStep returns after a stream synchronize

    def close(self):
        """Free the device search, the net and the engine."""
        if self.mcts is not None:
            self.mcts.close()
            self.mcts = None
        self.net.close()
        self.eng.close()


class _NetGroup:
    """The nets of a StreamWorkload seen as one (rank 0's init on the first, copied to the others)."""

    def __init__(self, nets):
        self.nets = nets
        self.num_params = nets[0].num_params

    def init_random(self, seed):
        self.nets[0].init_random(seed)
        blob = self.nets[0].get_weights()
        for n in self.nets[1:]:
            n.load_weights(blob)

    def get_weights(self):
        return self.nets[0].get_weights()

    def load_weights(self, blob):
        for n in self.nets:
            n.load_weights(blob)

    def set_precision(self, p):
        for n in self.nets:
            n.set_precision(p)

    def profile(self, on):
        for n in self.nets:
            n.profile(on)

    def profile_read(self):
        r = [n.profile_read() for n in self.nets]
        return sum(x[0] for x in r), sum(x[1] for x in r), sum(x[2] for x in r)

    def trunk_kernel(self):
        return self.nets[0].trunk_kernel()


class _MctsGroup:
    def __init__(self, subs):
        self.subs = subs

    def profile(self, on):
        for w in self.subs:
            w.mcts.profile(on)

    def profile_read(self):
        out = {}
        for w in self.subs:
            for k, v in w.mcts.profile_read().items():
                out[k] = out.get(k, 0) + v
        return out

    def tree_evictions(self):
        ev = [getattr(w.mcts, "tree_evictions", None) for w in self.subs]
        return sum(f() for f in ev) if all(ev) else None


class StreamWorkload:
    """`--streams K`: the rank's games split into K independent device handles, each with its
    own engine (HIP stream), net and search, stepped by K host threads at once -- so one handle's
    tree kernels and small launches run beside another's network (the games are independent; each
    keeps its global id's seeds, as a K-way shard).  For latency-bound configs (C2's 256 games, the
    per-rank shards of the 8-GPU configs), where one handle's dependent chain of short launches
    leaves CUs idle."""

    def __init__(self, a, local, shard, k):
        from az_amd import dist as azdist
        self.subs = []
        for i in range(k):
            sub = azdist.shard_range(i, k, shard["games"])
            sh = dict(shard, games=sub["games"], noise_seed=shard["noise_seed"] + sub["first_game"])
            self.subs.append(GpuWorkload(a, local, sh))
        self.eng = self.subs[0].eng
        self.net = _NetGroup([w.net for w in self.subs])
        self.mcts = None
        import concurrent.futures
        self.pool = concurrent.futures.ThreadPoolExecutor(k)

    def start(self):
        for w in self.subs:
            w.start()
        self.mcts = _MctsGroup(self.subs)

    def step(self):
        r = list(self.pool.map(lambda w: w.step(), self.subs))
        return sum(x[0] for x in r), sum(x[1] for x in r)

    def sync(self):
        pass

    def close(self):
        self.pool.shutdown()
        for w in self.subs:
            if hasattr(w, "close"):
                w.close()


def _progress(msg):
    """A progress line on stderr (the JSON line is the only stdout output)."""
    print(f"[bench {time.perf_counter() - T_START:7.1f} s] {msg}", file=sys.stderr, flush=True)


def _timed_moves(a, wl, net, steps, barrier):
    """`steps` self-play moves of the live workload between barriers, with the trunk / tree
    kernel clocks on: the raw counters of one timed region."""
    barrier()
    if a.kernel_timing:
        net.profile(True)
        wl.mcts.profile(True)
    t0 = time.perf_counter()
    moves = evals = 0
    for k in range(steps):
        mv, ev = wl.step()
        moves += mv
        evals += ev
        _progress(f"timed step {k + 1}/{steps}: {mv} moves, {time.perf_counter() - t0:.1f} s")
    wl.sync()
    elapsed = time.perf_counter() - t0
    barrier()
    trunk_ms, launches, forwards = net.profile_read()
    ev = getattr(wl.mcts, "tree_evictions", None)
    return {"elapsed": elapsed, "moves": moves, "evals": evals, "steps": steps, "trunk_ms": trunk_ms,
            "tree_evictions": ev() if ev else None,
            "launches": launches, "forwards": forwards, "tree": wl.mcts.profile_read(),
            "kernel": net.trunk_kernel()}     # the kernel the library dispatches for this net (engine's own choice)


def _roofline(a, m, precision):
    """The dominant kernel's roofline from rank 0's own timed region m: algorithmic conv FLOPs per
    launch / the launch's average device-clock duration, against the precision's dense MFMA peak."""
    HW = a.board * a.board
    conv_flops_per_eval = 2 * a.blocks * 2.0 * 9 * a.channels * a.channels * HW
    launches = m["launches"]
    boards_per_launch = m["evals"] * 2 * a.blocks / max(1, launches)        # rank 0's own launches and boards
    per_launch_flops = boards_per_launch * conv_flops_per_eval / (2 * a.blocks)
    per_launch_ms = m["trunk_ms"] / max(1, launches)
    achieved = per_launch_flops / (per_launch_ms * 1e-3) / 1e12 if launches else 0.0
    peak = PEAK_TFLOPS[precision]
    rf = {"kernel": f"{m['kernel']} ({precision} trunk, {a.board}x{a.board}, {a.channels} ch)",
          "bound": "mfma",
          "achieved": achieved, "peak": peak, "unit": "TFLOP/s", "frac": achieved / peak, "traffic": None,
          "launches": launches, "avg_launch_ms": per_launch_ms, "boards_per_launch": boards_per_launch,
          "flops_per_launch": per_launch_flops,
          # launches are trunk-conv equivalents (2 x blocks per forward); a fused forward (k_smallnet)
          # is one kernel launch per forward, whose rocprofv3 average is avg_forward_ms
          "forwards": m["forwards"], "avg_forward_ms": m["trunk_ms"] / max(1, m["forwards"])}
    if getattr(a, "streams", 1) > 1:
        rf["note"] = (f"{a.streams} streams: the handles' trunk launches overlap in time, so avg_launch_ms includes "
                      "the other streams' share of the CUs and achieved / frac understate the chip's rate")
    b = copy.copy(a)
    b.precision = precision
    tr = pmc_traffic(b, m["kernel"], boards_per_launch if launches else 0)
    if tr:
        rf.update(tr)
    return rf


class EngineColl:
    """The product collectives (N>1): the engine's own RCCL communicator (az_dist_*) over the
    ranks' engines -- rank 0's weights broadcast straight into every rank's device weight buffers,
    device-level barriers, counter reductions.  torch.distributed (gloo) only hands out the id."""

    def __init__(self, engine, rank, world, pg, timeout_s):
        from az_amd import dist as azdist
        box = [azdist.Dist.unique_id() if rank == 0 else None]
        pg.broadcast_object_list(box, src=0)
        self.d = azdist.Dist(engine, rank, world, box[0], timeout_s)
        self.kind = "rccl (engine az_dist_*)"

    def broadcast_weights(self, net):
        nets = getattr(net, "nets", [net])           # a StreamWorkload's nets: into the first, then copied
        self.d.broadcast_weights(nets[0], 0)
        if len(nets) > 1:
            blob = nets[0].get_weights()
            for n in nets[1:]:
                n.load_weights(blob)

    def barrier(self):
        self.d.barrier()

    def reduce(self, elapsed, counters):
        mx = self.d.allreduce([elapsed], "max")[0]
        return mx, [int(round(v)) for v in self.d.allreduce(counters, "sum")]

    def close(self):
        self.d.close()


class TorchColl:
    """The same collectives over a torch.distributed group (gloo on CPU: the rank-logic tests)."""

    def __init__(self, pg, device="cpu"):
        self.pg, self.device = pg, device
        self.kind = f"torch.distributed {pg.get_backend()}"

    def broadcast_weights(self, net):
        from az_amd import dist as azdist
        blob = net.get_weights() if self.pg.get_rank() == 0 else None
        blob = azdist.broadcast_weights(self.pg, blob, net.num_params, self.device)
        if self.pg.get_rank() != 0:
            net.load_weights(blob)

    def barrier(self):
        self.pg.barrier()

    def reduce(self, elapsed, counters):
        from az_amd import dist as azdist
        return azdist.reduce_counters(self.pg, elapsed, counters, self.device)

    def close(self):
        pass


def run_rank(a, rank, world, make_workload, make_coll=None, parity=None, before_timed=None):
    """One rank of the bench: shard, weights (rank 0 init + broadcast), warmup, timed steps between
    barriers, MAX elapsed / SUM counters over ranks.  Returns the JSON dict on rank 0, else None.
    make_coll(workload) (N>1): the collectives (EngineColl on the GPUs, TorchColl in the CPU tests).
    parity (N=1): parity(ms_per_step) -> number of further moves to time with the parity precision
    (the live net switched in place, the same games continued), or a string saying why not."""
    from az_amd import dist as azdist
    sh = azdist.shard_range(rank, world, a.global_games if a.scaling == "strong" else a.global_games * world)
    if sh["games"] < 1:
        raise SystemExit(f"bench.py: rank {rank} got no games ({a.global_games} over {world} ranks)")
    if getattr(a, "crash_report", None):     # diagnostic: symbolisable crash reports (profiler runs)
        from az_amd import _lib
        if _lib.lib().az_diag_crash_report(a.crash_report.encode()) != 0:
            raise RuntimeError("az_diag_crash_report failed")
    if getattr(a, "sync_every", 0):
        from az_amd import _lib
        _lib.lib().az_diag_set_sync_every(int(a.sync_every))
    if os.environ.get("AZ_STEP_TRACE"):      # diagnostic: timestamped phases of every selfplay step on stderr
        from az_amd import _lib
        _lib.lib().az_diag_set_step_trace(1)
    if getattr(a, "conv_flags", None):       # diagnostic: conv variant bits OR'd into the library's defaults
        from az_amd import _lib
        L = _lib.lib()
        L.az_diag_set_conv_flags(L.az_diag_conv_flags() | int(a.conv_flags, 16))
    wl = make_workload(a, int(os.environ.get("LOCAL_RANK", "0")), sh)
    net = wl.net
    coll = make_coll(wl) if world > 1 else None
    try:
        return _run_rank(a, rank, world, sh, wl, net, coll, parity, before_timed)
    finally:
        if coll is not None:
            coll.close()
        if hasattr(wl, "close"):         # the device search, net and engine (after the communicator)
            wl.close()


def _run_rank(a, rank, world, sh, wl, net, coll, parity, before_timed=None):
    if rank == 0:
        net.init_random(a.seed)
    if coll is not None:
        coll.broadcast_weights(net)          # rank 0's weights on every rank, once (RCCL over xGMI)
    wl.start()
    for k in range(a.warmup):
        wl.step()
        _progress(f"warmup step {k + 1}/{a.warmup}")
    if before_timed is not None:
        before_timed()                   # e.g. the CPU baseline that ran beside the setup and warm-up

    def barrier():
        wl.sync()
        if coll is not None:
            coll.barrier()
    m = _timed_moves(a, wl, net, a.steps, barrier)
    pm = None
    if parity is not None and world == 1:
        n_par = parity(1e3 * m["elapsed"] / a.steps)
        if isinstance(n_par, str):
            pm = {"skipped": n_par}
        else:
            # the same live games and weights: only the trunk / FC piece set changes (every piece set
            # is packed at load, az_net_set_precision switches the dispatch)
            net.set_precision(PREC[PARITY_PREC])
            for _ in range(a.parity_warmup):
                wl.step()
            pm = _timed_moves(a, wl, net, n_par, barrier)
    elapsed, tot_moves, tot_evals = m["elapsed"], m["moves"], m["evals"]
    if coll is not None:
        elapsed, (tot_moves, tot_evals) = coll.reduce(elapsed, [m["moves"], m["evals"]])
    if rank != 0:
        return None
    strong = a.scaling == "strong"
    out = {
        "metric": METRIC,
        "value": tot_moves / elapsed,
        "unit": "positions/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": 1e3 * elapsed / a.steps,
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": a.precision,
        "dtype_note": PREC_NOTE.get(a.precision, ""),
        "data": "synthetic: self-play from empty boards, counter-based random-init weights of the named net",
        "config": {"workload": f"{a.workload_name}, {a.global_games if strong else a.global_games * world} games"
                               f"{' sharded' if strong else ''} over {world} GPU(s), {a.sims} sims/move",
                   "baseline_config": a.config, "game": a.game, "global_games": a.global_games if strong else
                   a.global_games * world, "games_per_gpu": sh["games"], "sims_per_move": a.sims, "board": a.board,
                   "blocks": a.blocks, "channels": a.channels, "parallelism": f"game-shard x{world}" +
                   (f", {a.streams} streams" if getattr(a, "streams", 1) > 1 else ""),
                   "collectives": coll.kind if coll is not None else None},
        "nn_evals_per_s": tot_evals / elapsed,
        "evals_per_move": tot_evals / max(1, tot_moves),
        "roofline": _roofline(a, m, a.precision),
    }
    tree = m["tree"]
    steps = max(1, tree["sim_steps"])
    out["tree_kernels"] = {
        name: {"avg_launch_us": 1e3 * tree[f"{k}_ms"] / steps,
               "bytes_per_launch": tree[f"{k}_bytes"] / steps,
               "GB_per_s": tree[f"{k}_bytes"] / max(1e-12, 1e-3 * tree[f"{k}_ms"]) / 1e9,
               "frac_of_hbm_peak": tree[f"{k}_bytes"] / max(1e-12, 1e-3 * tree[f"{k}_ms"]) / 8.0e12}
        for name, k in (("k_select", "select"), ("k_expand_backup", "expand"))}
    if tree.get("fused_launches"):
        # the production tree step: step i's expansion + step i+1's selection in one launch
        fb = (tree["select_bytes"] + tree["expand_bytes"]) / steps
        fus = 1e3 * tree["fused_ms"] / tree["fused_launches"]
        out["tree_kernels"]["k_expand_select"] = {
            "avg_launch_us": fus, "launches": tree["fused_launches"], "bytes_per_launch": fb,
            "GB_per_s": fb / max(1e-12, 1e-6 * fus) / 1e9, "frac_of_hbm_peak": fb / max(1e-12, 1e-6 * fus) / 8.0e12}
    # TreeDev variants re-uploaded over a full slot cache (each a host sync), since the handle was made
    out["tree_kernels"]["tree_dev_evictions"] = m["tree_evictions"]
    out["tree_kernels"]["note"] = ("rank-0 device clock stamps: around each kernel of one simulation step in 16 (those "
                                   "steps run k_select and k_expand_backup as separate launches), and around one "
                                   "launch in 16 of the fused k_expand_select that every other step runs (step i's "
                                   "expansion with step i+1's selection: the production tree step; its bytes are "
                                   "the two kernels' per-step bytes); algorithmic "
                                   "bytes counted by the kernels (child records scanned, path VL/backup "
                                   "read-modify-writes, new nodes, leaf planes); latency-bound (one wave per game, "
                                   "dependent tree levels), peak 8 TB/s; rocprofv3 PMC traffic of the same kernels: "
                                   "profiles/r05_tree_pmc_c3.json (tools/tree_pmc.sh: C3's 2048 games x 800 sims, "
                                   "20-block trunk, --sync-every 10)")
    if pm is not None:
        out["parity_mode"] = pm if "skipped" in pm else parity_line(a, pm, m)
    return out


def pmc_traffic(a, kernel, boards_per_launch):
    """HBM bytes per trunk launch from the committed rocprofv3 PMC summary of the same kernel
    (profiles/*_trunk_pmc.json: FETCH_SIZE x2 per the gfx950 correction + WRITE_SIZE, measured at
    B boards per launch), scaled to this run's average boards per launch.  None if no summary
    matches the kernel (template name) and the precision / net."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_trunk_pmc.json"))):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if (d.get("precision"), d.get("board"), d.get("channels"), d.get("blocks")) == \
                (a.precision, a.board, a.channels, a.blocks) and _same_kernel(d.get("kernel", ""), kernel):
            best = (f, d)
    if best is None or boards_per_launch <= 0:
        return None
    f, d = best
    scale = boards_per_launch / d["boards_per_launch"]
    return {"traffic": d["hbm_bytes_per_launch"] * scale, "traffic_unit": "bytes/launch",
            "traffic_source": os.path.relpath(f, ROOT) + f" (PMC at B={d['boards_per_launch']}, scaled x{scale:.4f})"}


def _same_kernel(profiled, name):
    """rocprof's demangled name ("void conv3x3_v7<2, 15, 1>(ConvBf16Args)", "void
    conv3x3_v7x3<15, 1>(...)") vs the library's label ("conv3x3_v7<2, 15, SLIM>", "conv3x3_v7x3<15,
    SLIM>"): same template and every template argument but the last (the tile geometry, an enum
    that rocprof prints as a number)."""
    import re

    def parts(s):
        m = re.search(r"(conv3x3_v[0-9a-z]+)<([^>]*)>", s)
        if not m:
            return None
        args = [x.strip() for x in m.group(2).split(",")]
        # the split-operand kernels (v7x3 / v9x3: <board, geometry[, variant], piece type> in rocprof,
        # <board, SLIM|DENSE[, f16]> as labelled): the board; the piece type is the precision's.
        # conv3x3_v7: <mode, board, geometry[, tile rows[, ring slots]]> (defaults 256, 4): all but
        # the geometry
        if m.group(1).endswith("x3"):
            return (m.group(1), args[:1])
        if m.group(1) == "conv3x3_v7":
            return (m.group(1), args[:2] + args[3:] + ["256", "4"][len(args[3:]):])
        return (m.group(1), args[:-1])
    p1, p2 = parts(profiled), parts(name)
    return bool(p1 and p2 and p1 == p2)


# ------------------------------------------------------------------------------- CPU baseline
def cpu_share():
    """Host cores this process may use: the affinity mask, capped at 16 (a GPU box's CPU share per GPU;
    nproc there reports the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        n = min(n, int(env))
    return max(1, min(16, n))


def _cpu_worker(i, desc_fields, blob_path, game, board, sims, window, barrier, q, cpu=None):
    """One game on one core: oracle Mode S search, fp32 PyTorch-CPU net at B=1 per evaluation (as
    ParallelMCTS::evaluateState calls NeuralNetwork::predict), evaluations counted in the window."""
    import torch
    if cpu is not None and hasattr(os, "sched_setaffinity"):
        os.sched_setaffinity(0, {cpu})           # its own core, apart from the GPU process's
    torch.set_num_threads(1)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import types
    import az_oracle as O
    import net_oracle
    desc = types.SimpleNamespace(**desc_fields)
    model = net_oracle.Model(desc, np.load(blob_path, mmap_mode="r"))
    model(np.zeros((1, desc.in_planes, board, board), np.float32))          # warm-up evaluation
    st = {"n": 0, "deadline": None}

    def ev(_g, planes):
        if time.perf_counter() >= st["deadline"]:
            raise O.StopPlay()
        lo, v = model(planes[None])
        st["n"] += 1
        return lo[0], float(v[0])

    barrier.wait(timeout=600)
    t0 = time.perf_counter()
    st["deadline"] = t0 + window
    k = 0
    while time.perf_counter() < st["deadline"]:
        O.play(bs=board, sims=sims, eval_kind=O.EVAL_NET, evaluator=ev, noise_seed=42 + i + 1000 * k,
               game=O.GAME_GO if game == "go" else O.GAME_GOMOKU)
        k += 1
    q.put((i, st["n"], time.perf_counter() - t0))


def cpu_baseline(a, workers, window, cpus=None):
    """Raw CPU sample: {evals_per_s, cores, window, workers}; positions/s is derived after the GPU run
    from its measured evaluations per move.  Runs before anything touches the GPU."""
    import multiprocessing as mp
    import tempfile
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import net_oracle
    go = a.game == "go"
    fields = dict(board_size=a.board, in_planes=8 if go else 11, channels=a.channels, blocks=a.blocks,
                  action_size=a.board * a.board + (1 if go else 0), head_channels=32, pool=8, fc_hidden=256,
                  residual=1, conv_bias=0)
    blob = net_oracle.init_blob(__import__("types").SimpleNamespace(**fields), a.seed)   # == az_net_init_random
    fd, path = tempfile.mkstemp(suffix=".npy")
    os.close(fd)
    try:
        np.save(path, blob)
        ctx = mp.get_context("spawn")
        barrier = ctx.Barrier(workers + 1)
        q = ctx.Queue()
        procs = [ctx.Process(target=_cpu_worker, args=(i, fields, path, a.game, a.board, a.sims, window, barrier, q,
                                                         cpus[i] if cpus else None))
                 for i in range(workers)]
        for p in procs:
            p.start()
        barrier.wait(timeout=600)
        res = [q.get(timeout=window + 600) for _ in procs]
        for p in procs:
            p.join(timeout=60)
    finally:
        os.unlink(path)
    evals = sum(r[1] for r in res)
    span = max(r[2] for r in res)
    return {"evals": evals, "evals_per_s": evals / span, "cores": workers, "window_s": span}


def cpu_baseline_line(a, raw, evals_per_move):
    go = a.game == "go"
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None
    return {"value": raw["evals_per_s"] / evals_per_move, "unit": "positions/s", "cores": raw["cores"],
            "cores_from": f"min(16, affinity {aff}, OMP_NUM_THREADS {os.environ.get('OMP_NUM_THREADS')}); "
                          f"nproc {os.cpu_count()}",
            "kind": "port", "evals_per_s": raw["evals_per_s"], "cpus": raw.get("cpus", "alone"),
            "sample": f"{raw['cores']} worker processes x 1 thread, one {'Go' if go else 'Gomoku'} {a.board}x{a.board} "
                      f"game each from the empty board (oracle/ Mode S search, {a.sims} sims/move, fp32 "
                      f"{a.blocks}b x {a.channels}f net on PyTorch-CPU, B=1 per evaluation), {raw['evals']} "
                      f"evaluations in a {raw['window_s']:.1f} s window; positions/s = evaluations/s / "
                      f"{evals_per_move:.1f} evaluations per move (measured on the GPU run of the same workload)" +
                      ("; run on its own cores beside the GPU run's setup and warm-up, joined before its timed moves"
                       if raw.get("cpus", "alone") != "alone" else "; run alone, before the GPU work")}


def parity_line(a, pm, m):
    """parity_mode: the fp32-faithful trunk (f16x3) timed on the same live workload right after the
    headline moves (same games continued, same weights): positions/s and its own roofline."""
    out = {"value": pm["moves"] / pm["elapsed"], "unit": "positions/s", "steps": pm["steps"],
           "warmup": a.parity_warmup, "ms_per_step": 1e3 * pm["elapsed"] / pm["steps"], "dtype": PARITY_PREC,
           "dtype_note": PREC_NOTE[PARITY_PREC], "nn_evals_per_s": pm["evals"] / pm["elapsed"],
           "evals_per_move": pm["evals"] / max(1, pm["moves"]),
           "ratio_to_headline_ms_per_step": (pm["elapsed"] / pm["steps"]) / (m["elapsed"] / m["steps"]),
           "roofline": _roofline(a, pm, PARITY_PREC)}
    rf = out["roofline"]
    rf["mfma_issue_frac"] = 3 * rf["frac"]      # three MFMAs per algorithmic product
    out["note"] = (f"the same {a.global_games} live games continued for {pm['steps']} more moves (moves "
                   f"{a.warmup + a.steps + a.parity_warmup + 1}..{a.warmup + a.steps + a.parity_warmup + pm['steps']} of "
                   "every game) with the net switched in place to the parity precision (az_net_set_precision; every "
                   "piece set is packed at load); roofline FLOPs counted once (algorithmic), so frac <= 1/3 and "
                   "mfma_issue_frac = 3 x frac")
    return out


def parity_budget(a):
    """parity(ms_per_step) for run_rank: the parity moves to time, or why none are -- the run so far
    plus their estimate (PARITY_RATIO x the headline move, measured) must stay inside --time-budget."""
    def decide(ms_per_step):
        n = a.parity_steps + a.parity_warmup
        est = n * ms_per_step / 1e3 * PARITY_RATIO + 5.0
        spent = time.perf_counter() - T_START
        if spent + est <= a.time_budget:
            return a.parity_steps
        return f"time budget: {spent:.0f} s spent + ~{est:.0f} s estimated > {a.time_budget:.0f} s"
    return decide


def split_affinity(local, local_world):
    """Give rank `local` its own slice of the host's CPUs (the engine sizes its host threads from the
    affinity mask), so N ranks do not oversubscribe the CPU share."""
    if not hasattr(os, "sched_getaffinity") or local_world < 2:
        return None
    cpus = sorted(os.sched_getaffinity(0))
    per = len(cpus) // local_world
    if per < 1:
        return None
    mine = cpus[local * per:(local + 1) * per]
    os.sched_setaffinity(0, mine)
    return mine


# ------------------------------------------------------------------------------- main
def main(argv=None, make_workload=None, backend=None):
    """make_workload / backend: test hooks (a stand-in workload over gloo); the product run uses the
    device workload over RCCL."""
    argv = sys.argv[1:] if argv is None else argv
    a = parse(argv)
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        return launch_ranks(a, argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        return 2
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # the CPU baseline (rank 0, N = 1) runs in its own worker processes, alone, before the GPU work.
    # --cpu-beside 1 runs it beside the GPU setup and warm-up instead (joined before the timed moves),
    # but a GPU box's 16-CPU share is a quota that both then draw on: measured 310 evals/s unpinned and
    # 259 pinned to CPUs of their own, against 349 alone (profiles/r06_bench_c3_cpu_pinned.json)
    cpu = {}
    cpu_thread = None
    if a.cpu_baseline and world == 1:
        import threading
        workers = a.cpu_workers or cpu_share()
        mine = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else []
        cpus = None
        if a.cpu_beside and len(mine) >= 4 * workers:
            # a GPU box (256 host CPUs): the workers on the last `workers` CPUs, one each, the GPU process
            # (every thread it starts from here on) on the first quarter -- disjoint cores, SMT siblings
            # included whether they are numbered adjacently or half the machine apart, so neither run
            # takes the other's CPUs (though both draw on the same quota)
            cpus = mine[-workers:]
            os.sched_setaffinity(0, set(mine[:len(mine) // 4]))

        def _cpu():
            try:
                cpu["raw"] = cpu_baseline(a, workers, a.cpu_window, cpus)
                cpu["raw"]["cpus"] = f"{cpus[0]}..{cpus[-1]} (GPU process on {mine[0]}..{mine[len(mine) // 4 - 1]})" \
                    if cpus else "alone"
            except Exception as e:  # noqa: BLE001 -- reported in the line, the GPU run goes on
                cpu["error"] = repr(e)
        cpu_thread = threading.Thread(target=_cpu, name="cpu-baseline")
        cpu_thread.start()
        if cpus is None:
            cpu_thread.join()

    def join_cpu():
        nonlocal cpu_thread
        if cpu_thread is not None:
            cpu_thread.join()
            cpu_thread = None
            if "raw" in cpu:
                _progress(f"cpu baseline: {cpu['raw']['evals_per_s']:.1f} evals/s on {cpu['raw']['cores']} cores")
            else:
                _progress(f"cpu baseline failed: {cpu.get('error')}")
    if make_workload is None and a.streams > 1:
        make_workload = lambda a_, local, shard: StreamWorkload(a_, local, shard, a.streams)   # noqa: E731
    make_workload = make_workload or GpuWorkload
    dist = None
    make_coll = None
    if world > 1:
        import datetime
        import torch
        import torch.distributed as dist
        split_affinity(local, int(os.environ.get("LOCAL_WORLD_SIZE", str(world))))
        if backend is None and torch.cuda.device_count() <= local:
            print(f"bench.py: LOCAL_RANK {local} but {torch.cuda.device_count()} GPU(s) visible", file=sys.stderr)
            return 2
        # one node (the driver runs --nnodes=1): gloo's pairs over loopback, whatever the hostname resolves to
        os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")
        # gloo: the bootstrap group (hands out the engine communicator's id) -- or, with a test
        # backend, the collectives themselves.  A rank that dies leaves the others in a collective:
        # they fail after dist_timeout (gloo's timeout, the engine's RCCL deadline), not hang.
        dist.init_process_group(backend or "gloo", init_method="env://",
                                timeout=datetime.timedelta(seconds=a.dist_timeout))
        if backend is None:
            def make_coll(wl):
                try:
                    return EngineColl(wl.eng, rank, world, dist, a.dist_timeout)
                except Exception as e:  # noqa: BLE001 -- said in the line (config.collectives) and on stderr
                    # every rank fails the same way (the communicator's init is collective, with a
                    # deadline): the run goes on over the gloo group rather than losing the measurement
                    print(f"bench.py: rank {rank}: engine communicator failed ({e}); collectives over gloo",
                          file=sys.stderr, flush=True)
                    c = TorchColl(dist, "cpu")
                    c.kind += f" (engine RCCL init failed: {e})"
                    return c
        else:
            make_coll = lambda wl: TorchColl(dist, "cpu")                                 # noqa: E731
    try:
        parity = None
        if world == 1 and a.parity_steps > 0 and a.precision not in ("f16x3", "bf16x3") and a.channels % 64 == 0:
            parity = parity_budget(a)
        out = run_rank(a, rank, world, make_workload, make_coll, parity=parity, before_timed=join_cpu)
        join_cpu()
        if out is not None:
            if "raw" in cpu:
                out["cpu_baseline"] = cpu_baseline_line(a, cpu["raw"], out["evals_per_move"])
            else:
                out["cpu_baseline"] = {"error": cpu["error"]} if "error" in cpu else None
            print(json.dumps(out), flush=True)
    finally:
        if dist is not None:
            dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
