"""Does a net's FIRST forward see all of its weights?  (the unreproduced v7/v6
bf16 mismatch on board 0 of a freshly created net.)

Nets are created, loaded and forwarded right away, many times, while a second thread keeps the
engine's stream busy with forwards of another net -- the situation of a test that follows other GPU
tests in one process.  Creation and weight upload run hipMemset / hipMemcpy on the null stream, the
forwards run on the engine's NON-BLOCKING stream, which does not wait for null-stream work.  Each
first forward is compared bitwise with the result of a forward taken after a device-wide sync.

Usage (on the GPU box): python3 tools/upload_race.py [iterations]; AZ_DIAG_HIP_LIB selects an
in-tree build (e.g. one without the round-5 device synchronisations after creation / upload)."""
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "alphazero-multi-game_amd"), os.path.join(ROOT, "oracle")]
import az_amd            # noqa: E402
import net_oracle        # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    eng = az_amd.Engine(0)
    busy_desc = az_amd.NetDesc(15, 11, 256, 4, 225, 32, 8, 256, 1, 0, az_amd.AZ_PREC_FP16, 512)
    busy = az_amd.HipNeuralNetwork(eng, busy_desc)
    busy.load_weights(net_oracle.init_blob(busy_desc, seed=5))
    xb = (np.random.default_rng(1).random((512, 11, 15, 15)) < 0.2).astype(np.float32)
    stop = threading.Event()

    def spin():
        while not stop.is_set():
            busy.forward(xb)

    cases = [(19, 8, 362, 256, 1, 130, az_amd.AZ_PREC_BF16), (19, 8, 362, 256, 1, 130, az_amd.AZ_PREC_FP16),
             (15, 11, 225, 256, 2, 37, az_amd.AZ_PREC_FP16)]
    refs = {}
    for c in cases:                       # reference outputs: forward after everything settled
        bs, ci, A, ch, blocks, B, prec = c
        d = az_amd.NetDesc(bs, ci, ch, blocks, A, 32, 8, 256, 1, 0, prec, B)
        n = az_amd.HipNeuralNetwork(eng, d)
        n.load_weights(net_oracle.init_blob(d, seed=31))
        time.sleep(0.2)
        x = (np.random.default_rng(bs * 7 + B).random((B, ci, bs, bs)) < 0.25).astype(np.float32)
        refs[c] = (x, n.forward(x))
        n.close()
    th = threading.Thread(target=spin, daemon=True)
    th.start()
    bad = 0
    t0 = time.time()
    for i in range(iters):
        c = cases[i % len(cases)]
        bs, ci, A, ch, blocks, B, prec = c
        d = az_amd.NetDesc(bs, ci, ch, blocks, A, 32, 8, 256, 1, 0, prec, B)
        n = az_amd.HipNeuralNetwork(eng, d)
        n.load_weights(net_oracle.init_blob(d, seed=31))
        x, (lr, vr) = refs[c]
        l1, v1 = n.forward(x)
        l2, v2 = n.forward(x)
        n.close()
        d1 = np.where((l1 != lr).any(axis=1) | (v1 != vr))[0]
        d2 = np.where((l2 != lr).any(axis=1) | (v2 != vr))[0]
        if len(d1) or len(d2):
            bad += 1
        print(f"iter {i} {c[:1] + c[5:]}: first forward boards differing {d1.tolist()[:8]}, second {d2.tolist()[:8]}",
              flush=True)
        if time.time() - t0 > 100:
            break
    stop.set()
    th.join()
    print(f"RESULT {bad} of {i + 1} iterations differ")


if __name__ == "__main__":
    main()
