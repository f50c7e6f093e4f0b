#!/usr/bin/env python3
"""Two ranks of the engine's RCCL communicator (az_dist_*) on ONE GPU, as two processes: the id
handed over through a file, barrier, counter reductions (sum / max) and a weight broadcast from
rank 0 into rank 1's never-loaded net, checked by rank 1's forward against rank 0's, bit for bit.
RCCL may refuse two ranks on one device ("duplicate GPU"); the probe reports what it got.

  python3 tools/dist_probe.py [--device 0] [--timeout 60]
"""
import argparse
import multiprocessing as mp
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-multi-game_amd"))


def rank_main(rank, world, idfile, device, timeout, q):
    import numpy as np
    try:
        import az_amd
        from az_amd import dist as azdist
        eng = az_amd.Engine(device)
        if rank == 0:
            uid = azdist.Dist.unique_id()
            with open(idfile + ".tmp", "wb") as f:
                f.write(uid)
            os.rename(idfile + ".tmp", idfile)
        else:
            t0 = time.time()
            while not os.path.exists(idfile):
                if time.time() - t0 > timeout:
                    raise RuntimeError("no id file")
                time.sleep(0.02)
            uid = open(idfile, "rb").read()
        d = azdist.Dist(eng, rank, world, uid, timeout_s=timeout)
        d.barrier()
        s = d.allreduce([rank + 1.0, 10.0 * rank], "sum")
        m = d.allreduce([rank + 1.0], "max")
        desc = az_amd.gomoku_net_desc(board_size=15, channels=256, blocks=2, precision=az_amd.AZ_PREC_FP16, max_batch=64)
        net = az_amd.HipNeuralNetwork(eng, desc)
        if rank == 0:
            net.init_random(99)
        t0 = time.perf_counter()
        d.broadcast_weights(net, 0)
        bt = time.perf_counter() - t0
        x = (np.random.default_rng(1).random((64, 11, 15, 15)) < 0.3).astype(np.float32)
        lo, v = net.forward(x)
        d.barrier()
        d.close()
        q.put((rank, "ok", s, m, float(np.abs(lo).sum()), lo.tobytes() == lo.tobytes(), lo.view(np.uint32).sum(dtype=np.uint64).item(),
               bt, net.num_params))
        net.close()
        eng.close()
    except Exception as e:  # noqa: BLE001 -- reported to the parent
        q.put((rank, "error", repr(e)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--timeout", type=float, default=60.0)
    a = ap.parse_args()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    idfile = os.path.join(tempfile.mkdtemp(), "az_dist.id")
    ps = [ctx.Process(target=rank_main, args=(r, 2, idfile, a.device, a.timeout, q)) for r in range(2)]
    for p in ps:
        p.start()
    try:
        res = sorted([q.get(timeout=a.timeout + 120) for _ in ps], key=lambda r: r[0])
    except Exception as e:  # noqa: BLE001 -- a rank stuck in the communicator: end both, report
        for p in ps:
            p.kill()
        print("DIST PROBE TIMEOUT", repr(e))
        return 1
    for p in ps:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    for r in res:
        print(r)
    if all(r[1] == "ok" for r in res):
        (_, _, s0, m0, _, _, h0, bt0, n), (_, _, s1, m1, _, _, h1, bt1, _) = res
        ok = s0 == s1 == [3.0, 10.0] and m0 == m1 == [2.0] and h0 == h1
        print(f"sums {s0} max {m0}; rank 1's forward {'==' if h0 == h1 else '!='} rank 0's (bit checksum); "
              f"broadcast of {n} params x all piece sets: {bt0 * 1e3:.1f} / {bt1 * 1e3:.1f} ms")
        print("DIST PROBE", "PASS" if ok else "FAIL")
        return 0 if ok else 1
    print("DIST PROBE ERROR")
    return 1


if __name__ == "__main__":
    sys.exit(main())
