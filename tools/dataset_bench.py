#!/usr/bin/env python3
"""Training-example extraction microbenchmark (row f3, k_dataset_extract): G synthetic game records
of `plies` moves (random distinct cells, random child-order policies of the reference's lengths)
-> extractExamples with the 8-fold augmentation written into a shuffled order.  Prints one JSON
line: kernel time (HIP events on the engine stream), algorithmic bytes (examples written once +
records read once) and GB/s against the 8 TB/s HBM peak.  Also the workload of the rocprofv3
passes for the kernel (tools/r01b_profiles.sh)."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-multi-game_amd"))
import az_amd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--game", default="gomoku", choices=["gomoku", "go"])
    ap.add_argument("--board", type=int, default=None)
    ap.add_argument("--games", type=int, default=2048)
    ap.add_argument("--plies", type=int, default=60)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--augment", type=int, default=1)
    a = ap.parse_args()
    gt = az_amd.GAME_GO if a.game == "go" else az_amd.GAME_GOMOKU
    bs = a.board or (19 if a.game == "go" else 15)
    A = bs * bs
    rng = np.random.default_rng(0)
    G, n = a.games, a.plies
    acts = np.argsort(rng.random((G, A)), axis=1)[:, :n].astype(np.int32)   # distinct cells per game
    nch = np.tile(np.arange(A, A - n, -1, dtype=np.int32), G)                # |legal| shrinks by one per ply
    pol = rng.random(int(nch.sum()), dtype=np.float32)
    res = rng.integers(1, 4, G).astype(np.int32)
    eng = az_amd.Engine(int(os.environ.get("LOCAL_RANK", 0)))
    ds = az_amd.Dataset(eng, gt, bs, seed=1)
    E = G * n * (8 if a.augment else 1)
    order = ds._order(E)
    from az_amd import _fp, _ip, _i64, check, lib
    import ctypes
    ne = ctypes.c_int64()
    times = []
    for _ in range(a.iters):
        t0 = time.perf_counter()
        check(lib().az_dataset_extract(ds.h, G, _ip(np.full(G, n, np.int32)), _ip(acts.reshape(-1)), _ip(nch),
                                       _fp(pol), _ip(res), a.augment, order.ctypes.data_as(_i64), ctypes.byref(ne)))
        times.append(time.perf_counter() - t0)
        ms, by = ds.profile_read()
    out = {"kernel": "k_dataset_extract", "game": a.game, "board": bs, "games": G, "plies": n,
           "examples": int(ne.value), "kernel_ms": ms, "algorithmic_bytes": by, "GB_per_s": by / ms / 1e6,
           "frac_of_hbm_peak": by / ms / 1e6 / 8000.0, "host_call_s": min(times)}
    print(json.dumps(out))
    ds.close()
    eng.close()


if __name__ == "__main__":
    main()
