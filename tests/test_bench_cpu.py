"""bench.py's own rank logic on CPU (no GPU): argument handling and the loud failures of the
launcher, the strong-scaling shard of BASELINE C3 (2048 games sharded over the ranks), rank 0's
weights broadcast into every other rank's load_weights, MAX-elapsed / SUM-counter reduction and
the JSON line -- driven over gloo at world size 2 with a stand-in for the device workload (the
stand-in replaces only the GPU handle; run_rank is bench.py's code).  Also the CPU-baseline leg
(worker processes, fixed window) on a tiny net."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _Net:
    num_params = 777

    def __init__(self):
        self.blob = None
        self.loaded = None
        self.prof = False
        self.precision = None

    def set_precision(self, p):
        self.precision = p

    def init_random(self, seed):
        self.blob = (np.arange(self.num_params, dtype=np.float32) + seed) * 0.25

    def get_weights(self):
        return self.blob.copy()

    def load_weights(self, blob):
        self.loaded = np.asarray(blob, np.float32).copy()
        self.blob = self.loaded

    def profile(self, on):
        self.prof = on

    def profile_read(self):
        return 4.0, 40 * 2, 2      # 4 ms over 80 trunk launches

    def trunk_kernel(self):
        return "conv3x3_v9x3<15, SLIM, f16>" if self.precision == 4 else "conv3x3_v7<2, 15, SLIM>"


class _Mcts:
    def profile(self, on):
        pass

    def profile_read(self):
        return {"select_ms": 1.0, "expand_ms": 0.5, "sim_steps": 10, "select_bytes": 10 ** 6, "expand_bytes": 10 ** 5}


class _Workload:
    def __init__(self, a, local, shard):
        self.shard = shard
        self.net = _Net()
        self.mcts = _Mcts()
        self.steps = 0

    def start(self):
        pass

    def step(self):
        self.steps += 1
        g = self.shard["games"]
        return g, g * 800

    def sync(self):
        pass


def _rank(rank, world, port, q):
    import torch.distributed as dist
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        a = bench.parse(["--gpus", str(world), "--steps", "3", "--warmup", "1"])
        wls = []

        def make(a_, local, shard):
            wls.append(_Workload(a_, local, shard))
            return wls[-1]
        out = bench.run_rank(a, rank, world, make, lambda wl: bench.TorchColl(dist, "cpu"))
        w = wls[0]
        q.put((rank, out, w.shard, None if w.net.loaded is None else float(w.net.loaded.sum()), w.steps))
    finally:
        dist.destroy_process_group()


def test_bench_rank_logic_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=180) for _ in procs), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, out0, sh0, ld0, st0), (_, out1, sh1, ld1, st1) = res
    # C3 default: 2048 games sharded 1024 + 1024, contiguous ids, per-game seeds
    assert (sh0["first_game"], sh0["games"], sh1["first_game"], sh1["games"]) == (0, 1024, 1024, 1024)
    assert sh1["noise_seed"] == 42 + 1024 and sh1["noise_seed_stride"] == 1
    # rank 0 initialised; rank 1 loaded rank 0's blob through the broadcast
    want = float(((np.arange(777, dtype=np.float32) + 1234) * 0.25).sum())
    assert ld0 is None and ld1 == want
    assert st0 == st1 == 4                          # warmup + 3 timed steps
    assert out1 is None
    assert out0["n_gpus"] == 2 and out0["scaling"] == "strong"
    assert out0["config"]["global_games"] == 2048 and out0["config"]["games_per_gpu"] == 1024
    assert out0["steps"] == 3 and out0["warmup"] == 1
    # value = all ranks' moves / slowest rank's elapsed
    moves = 2 * 3 * 1024
    assert abs(out0["value"] - moves / (out0["ms_per_step"] * 3 / 1e3)) < 1e-6 * out0["value"]
    assert abs(out0["nn_evals_per_s"] / out0["value"] - 800) < 1e-6
    # roofline from rank 0's own launches: 3 steps x 1024 boards x 40 convs / 80 launches
    assert out0["roofline"]["boards_per_launch"] == 3 * 1024 * 800 * 40 / 80
    assert out0["roofline"]["bound"] == "mfma" and 0 < out0["roofline"]["frac"]


def test_bench_weak_scaling_and_configs():
    import bench
    a = bench.parse(["--scaling", "weak"])
    assert a.scaling == "weak" and a.global_games == 2048
    a = bench.parse(["--config", "c2"])
    assert (a.board, a.blocks, a.channels, a.sims, a.global_games) == (15, 6, 64, 400, 256)
    a = bench.parse(["--game", "go"])
    assert (a.config, a.board, a.global_games, a.game) == ("c4", 19, 1024, "go")
    a = bench.parse(["--games", "512"])
    assert a.scaling == "weak" and a.global_games == 512
    from az_amd import dist as azdist
    parts = [azdist.shard_range(r, 3, 10) for r in range(3)]
    assert [p["games"] for p in parts] == [4, 3, 3] and [p["first_game"] for p in parts] == [0, 4, 7]


def test_bench_gpus_without_enough_devices_fails_loudly(monkeypatch, capsys):
    import bench
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert bench.main(["--gpus", "2"]) == 2          # this container has no GPU
    assert "only 0 GPU" in capsys.readouterr().err
    monkeypatch.setenv("WORLD_SIZE", "1")
    assert bench.main(["--gpus", "2"]) == 2
    assert "WORLD_SIZE=1" in capsys.readouterr().err


@pytest.mark.timeout(300)
def test_cpu_baseline_workers_window():
    import bench
    a = bench.parse(["--board", "9", "--blocks", "1", "--channels", "16", "--sims", "20"])
    raw = bench.cpu_baseline(a, workers=2, window=2.0)
    assert raw["cores"] == 2 and raw["evals"] > 10 and 1.9 < raw["window_s"] < 10
    line = bench.cpu_baseline_line(a, raw, 20.0)
    assert line["kind"] == "port" and line["cores"] == 2
    assert abs(line["value"] - raw["evals_per_s"] / 20.0) < 1e-9


class _DyingWorkload(_Workload):
    """Rank 1's stand-in dies in its second timed step (a crashed GPU process)."""

    def step(self):
        if self.steps == 2:
            raise RuntimeError("rank 1: simulated device failure")
        return super().step()


def _rank_main(rank, world, port, q):
    import time
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LOCAL_RANK=str(rank), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world))
    t0 = time.time()

    def make(a_, local, shard):
        return (_DyingWorkload if rank == 1 else _Workload)(a_, local, shard)
    try:
        bench.main(["--gpus", str(world), "--steps", "3", "--warmup", "1", "--cpu-baseline", "0",
                    "--dist-timeout", "15"], make_workload=make, backend="gloo")
        q.put((rank, "returned", time.time() - t0))
    except BaseException as e:        # noqa: BLE001 -- reported to the parent, then re-raised
        q.put((rank, type(e).__name__, time.time() - t0))
        raise


@pytest.mark.timeout(240)
def test_bench_rank_death_fails_loudly_gloo_world2():
    """One rank raising mid-run makes bench.py fail on every rank within --dist-timeout (no hang,
    no JSON line from rank 0): the surviving rank's barrier raises, both processes exit non-zero."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=200) for _ in procs), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    assert res[1][1] == "RuntimeError"
    assert res[0][1] != "returned" and res[0][2] < 15 + 60
    assert all(p.exitcode not in (0, None) for p in procs)


def test_pmc_traffic_matches_each_trunk_kernel():
    """roofline.traffic comes from the committed PMC summary of the SAME kernel and precision: the
    fp16 v7 line and parity_mode's bf16x3 v7x3 line each find theirs, and neither takes the other's."""
    import types
    import bench
    assert bench._same_kernel("void conv3x3_v7<2, 15, 1>(ConvBf16Args)", "conv3x3_v7<2, 15, SLIM>")
    assert bench._same_kernel("void conv3x3_v7x3<15, 1>(ConvBf16Args)", "conv3x3_v7x3<15, SLIM>")
    assert not bench._same_kernel("void conv3x3_v7<2, 15, 1>(ConvBf16Args)", "conv3x3_v7x3<15, SLIM>")
    assert not bench._same_kernel("void conv3x3_v6<2, 15, 1>(ConvBf16Args)", "conv3x3_v7<2, 15, SLIM>")
    assert not bench._same_kernel("void conv3x3_v7<1, 15, 1>(ConvBf16Args)", "conv3x3_v7<2, 15, SLIM>")
    assert bench._same_kernel("void conv3x3_v7<2, 8, 2, 64>(ConvBf16Args)", "conv3x3_v7<2, 8, DENSE, 64>")
    assert not bench._same_kernel("void conv3x3_v7<2, 8, 2, 64>(ConvBf16Args)", "conv3x3_v7<2, 8, DENSE, 128>")
    # the ring-slot argument (default 4) and the tile rows (default 256) as rocprof prints them
    assert bench._same_kernel("void conv3x3_v7<2, 15, 1, 256, 4>(ConvBf16Args)", "conv3x3_v7<2, 15, SLIM>")
    assert bench._same_kernel("void conv3x3_v7<2, 19, 2, 128, 3>(ConvBf16Args)", "conv3x3_v7<2, 19, DENSE, 128, 3>")
    assert not bench._same_kernel("void conv3x3_v7<2, 19, 2, 128, 4>(ConvBf16Args)", "conv3x3_v7<2, 19, DENSE, 128, 3>")
    assert bench._same_kernel("void conv3x3_v7<2, 8, 2, 64, 4>(ConvBf16Args)", "conv3x3_v7<2, 8, DENSE, 64>")
    # the split-operand kernels: rocprof <board, geometry, variant, piece type> vs the label
    assert bench._same_kernel("void conv3x3_v9x3<15, 1, 3, 2>(ConvBf16Args)", "conv3x3_v9x3<15, SLIM, f16>")
    assert bench._same_kernel("void conv3x3_v9x3<19, 2, 3, 1>(ConvBf16Args)", "conv3x3_v9x3<19, DENSE>")
    assert not bench._same_kernel("void conv3x3_v9x3<15, 1, 3, 2>(ConvBf16Args)", "conv3x3_v7x3<15, SLIM, f16>")
    assert not bench._same_kernel("void conv3x3_v9x3<15, 1, 3, 2>(ConvBf16Args)", "conv3x3_v9x3<19, DENSE, f16>")
    net = dict(board=15, channels=256, blocks=20)
    fp16 = bench.pmc_traffic(types.SimpleNamespace(precision="fp16", **net), "conv3x3_v7<2, 15, SLIM>", 2048.0)
    x3 = bench.pmc_traffic(types.SimpleNamespace(precision="bf16x3", **net), "conv3x3_v7x3<15, SLIM>", 2048.0)
    assert fp16 and x3 and "v7x3" in x3["traffic_source"] and "v7x3" not in fp16["traffic_source"]
    assert x3["traffic"] > fp16["traffic"] > 0
    half = bench.pmc_traffic(types.SimpleNamespace(precision="fp16", **net), "conv3x3_v7<2, 15, SLIM>", 1024.0)
    assert half["traffic"] == pytest.approx(fp16["traffic"] / 2)


def test_bench_parity_mode_in_place_world1():
    """N=1: after the timed headline moves the live net switches to the parity precision (f16x3) in
    place and the same workload is timed for --parity-steps more moves (no second setup / warm-up);
    the budget rule skips it, and says so, when the estimate would overrun --time-budget."""
    import bench
    a = bench.parse(["--steps", "3", "--warmup", "2", "--parity-steps", "2"])
    wls = []

    def make(a_, local, shard):
        wls.append(_Workload(a_, local, shard))
        return wls[-1]
    out = bench.run_rank(a, 0, 1, make, parity=bench.parity_budget(a))
    w = wls[0]
    assert len(wls) == 1 and w.steps == 2 + 3 + 2          # one workload: warmup, headline, parity moves
    assert w.net.precision == bench.PREC["f16x3"]
    pm = out["parity_mode"]
    assert pm["dtype"] == "f16x3" and pm["steps"] == 2 and pm["value"] > 0
    assert "v9x3" in pm["roofline"]["kernel"] and "v7<" in out["roofline"]["kernel"]
    assert pm["roofline"]["mfma_issue_frac"] == pytest.approx(3 * pm["roofline"]["frac"])
    assert "moves 6..7" in pm["note"]
    # the budget: an estimate past --time-budget skips the parity moves and names the numbers
    b = bench.parse(["--steps", "3", "--warmup", "2", "--parity-steps", "2", "--time-budget", "1"])
    wls.clear()
    out = bench.run_rank(b, 0, 1, make, parity=bench.parity_budget(b))
    assert "skipped" in out["parity_mode"] and "time budget" in out["parity_mode"]["skipped"]
    assert wls[0].steps == 5 and wls[0].net.precision is None


class _FakeDist:
    """Stands in for az_amd.dist.Dist (the engine's RCCL communicator) on CPU: records the id it
    was given; its collectives run over the gloo group so the bench's reductions stay real."""
    made = []

    def __init__(self, engine, rank, world, uid, timeout_s):
        import torch.distributed as dist
        self.rank, self.world, self.uid, self.pg = rank, world, uid, dist
        _FakeDist.made.append(self)

    @staticmethod
    def unique_id():
        return bytes([7]) * 128

    def barrier(self):
        self.pg.barrier()

    def allreduce(self, values, op="sum"):
        import torch
        t = torch.tensor([float(v) for v in values], dtype=torch.float64)
        self.pg.all_reduce(t, op=self.pg.ReduceOp.SUM if op == "sum" else self.pg.ReduceOp.MAX)
        return t.tolist()

    def broadcast_weights(self, net, root=0):
        from az_amd import dist as azdist
        blob = net.get_weights() if self.rank == root else None
        blob = azdist.broadcast_weights(self.pg, blob, net.num_params, "cpu")
        if self.rank != root:
            net.load_weights(blob)

    def close(self):
        pass


class _EngineWorkload(_Workload):
    eng = object()


def _rank_engine(rank, world, port, q):
    import torch.distributed as dist
    import bench
    from az_amd import dist as azdist
    azdist.Dist = _FakeDist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        a = bench.parse(["--gpus", str(world), "--steps", "2", "--warmup", "1"])
        wls = []

        def make(a_, local, shard):
            wls.append(_EngineWorkload(a_, local, shard))
            return wls[-1]
        out = bench.run_rank(a, rank, world, make, lambda wl: bench.EngineColl(wl.eng, rank, world, dist, 30.0))
        d = _FakeDist.made[0]
        q.put((rank, out, d.uid, None if wls[0].net.loaded is None else float(wls[0].net.loaded.sum())))
    finally:
        dist.destroy_process_group()


def test_bench_engine_collectives_bootstrap_gloo_world2():
    """bench.EngineColl (the product's N>1 collectives): rank 0's communicator id reaches every rank
    through the gloo bootstrap group, and the weight broadcast / counter reductions / barriers go
    through the communicator object (a CPU stand-in for az_amd.dist.Dist here)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_engine, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=180) for _ in procs), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, out0, uid0, ld0), (_, out1, uid1, ld1) = res
    assert uid0 == uid1 == bytes([7]) * 128
    assert ld0 is None and ld1 == float(((np.arange(777, dtype=np.float32) + 1234) * 0.25).sum())
    assert out1 is None and out0["config"]["collectives"] == "rccl (engine az_dist_*)"
    assert abs(out0["value"] - 2 * 2 * 1024 / (out0["ms_per_step"] * 2 / 1e3)) < 1e-6 * out0["value"]


def test_bench_stream_workload_splits_games(monkeypatch):
    """--streams K: the rank's games split into K handles with the K-way shard's seeds (game ids and
    noise streams as a K-rank run), rank 0's weights copied into every handle's net, and a step's
    moves / evaluations summed over the handles."""
    import bench
    made = []

    class _W(_Workload):
        def __init__(self, a, local, shard):
            super().__init__(a, local, shard)
            self.eng = object()
            made.append(self)

    monkeypatch.setattr(bench, "GpuWorkload", _W)
    a = bench.parse(["--streams", "3", "--config", "c2"])
    sh = {"first_game": 0, "games": 256, "noise_seed": 42, "noise_seed_stride": 1, "eval_seed": 0}
    wl = bench.StreamWorkload(a, 0, sh, 3)
    assert [w.shard["games"] for w in made] == [86, 85, 85]
    assert [w.shard["noise_seed"] for w in made] == [42, 42 + 86, 42 + 171]
    wl.net.init_random(5)
    assert all(np.array_equal(w.net.loaded, made[0].net.blob) for w in made[1:])
    wl.start()
    assert wl.step() == (256, 256 * 800)
    wl.net.set_precision(4)
    assert all(w.net.precision == 4 for w in made)
    assert wl.net.profile_read() == (12.0, 240, 6)
    wl.pool.shutdown()


def _rank_streams(rank, world, port, q):
    import torch.distributed as dist
    import bench
    from az_amd import dist as azdist
    azdist.Dist = _FakeDist

    class _W(_Workload):
        def __init__(self, a, local, shard):
            super().__init__(a, local, shard)
            self.eng = object()
    bench.GpuWorkload = _W
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        a = bench.parse(["--gpus", str(world), "--steps", "2", "--warmup", "1", "--streams", "2"])
        wls = []

        def make(a_, local, shard):
            wls.append(bench.StreamWorkload(a_, local, shard, 2))
            return wls[-1]
        out = bench.run_rank(a, rank, world, make, lambda wl: bench.EngineColl(wl.eng, rank, world, dist, 30.0))
        nets = wls[0].net.nets
        q.put((rank, out, [None if n.loaded is None else float(n.loaded.sum()) for n in nets],
               [w.shard for w in wls[0].subs]))
    finally:
        dist.destroy_process_group()


def test_bench_streams_at_world2_gloo():
    """--streams 2 on every rank of a 2-rank run: the rank's 1024 games split 512 + 512 with the
    global ids' seeds, rank 0's weights broadcast into rank 1's first net and copied into its second."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_streams, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=180) for _ in procs), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, out0, ld0, sh0), (_, out1, ld1, sh1) = res
    want = float(((np.arange(777, dtype=np.float32) + 1234) * 0.25).sum())
    assert ld1 == [want, want] and ld0[0] is None and ld0[1] == want     # rank 0: init on net 0, copied to net 1
    assert [s["noise_seed"] for s in sh1] == [42 + 1024, 42 + 1024 + 512] and [s["games"] for s in sh0] == [512, 512]
    assert out0["config"]["parallelism"] == "game-shard x2, 2 streams"
