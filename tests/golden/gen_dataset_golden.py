"""Generates tests/golden/ref_dataset.npz from the REFERENCE Dataset (oracle/_ref/ref_dataset, built by
oracle/build_ref_dataset.sh from src/selfplay/dataset.cpp with only its JSON functions removed).

Inputs are the reference's own self-play games (ref_games.json.gz, grouped by board size: one
Dataset per board, as the device store holds one shape).  Per group and augment in {1, 0}: the
examples_ store after extractExamples (which ends with shuffle() on rng_ seeded 1000 + board).  For
the 9x9 group also the rng sequence getBatch(37) -> getRandomSubset(5) -> shuffle() on seed 1234,
recorded as row indices into the extracted store (identical rows are interchangeable).

Run in this container (the reference is not on the GPU box):  python tests/golden/gen_dataset_golden.py
"""
import os
import struct
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "alphazero-multi-game_amd")]
EXE = os.path.join(ROOT, "oracle", "_ref", "ref_dataset")


def read_store(buf, off):
    E, = struct.unpack_from("<q", buf, off)
    C, H, W, PM = struct.unpack_from("<4i", buf, off + 8)
    off += 24
    st = np.frombuffer(buf, np.float32, E * C * H * W, off).reshape(E, C, H, W)
    off += 4 * E * C * H * W
    pl = np.frombuffer(buf, np.int32, E, off)
    off += 4 * E
    po = np.frombuffer(buf, np.float32, E * PM, off).reshape(E, PM)
    off += 4 * E * PM
    va = np.frombuffer(buf, np.float32, E, off)
    off += 4 * E
    return (st, po, pl, va), off


def run(recs, bs, seed, augment, ops):
    lines = [f"{seed} {int(augment)} {int(ops)} {len(recs)}"]
    for acts, pols, res in recs:
        lines.append(f"{bs} {res} {len(acts)}")
        for a, p in zip(acts, pols):
            b = np.asarray(p, np.float32).view(np.uint32)
            lines.append(f"{a} {len(b)} " + " ".join(str(int(x)) for x in b))
    out = os.path.join("/tmp", f"ref_dataset_{os.getpid()}.bin")
    subprocess.run([EXE, out], input="\n".join(lines) + "\n", text=True, check=True, capture_output=True)
    buf = open(out, "rb").read()
    os.unlink(out)
    stores, off = [], 0
    while off < len(buf):
        s, off = read_store(buf, off)
        stores.append(s)
    return stores


def row_index(store, rows):
    """For each row of `rows`, an index of an equal (bitwise) row of `store`, each used at most once."""
    key = lambda s, i: (s[0][i].tobytes(), s[1][i, :s[2][i]].tobytes(), int(s[2][i]), s[3][i].tobytes())
    free = {}
    for i in range(len(store[0])):
        free.setdefault(key(store, i), []).append(i)
    out = []
    for i in range(len(rows[0])):
        out.append(free[key(rows, i)].pop(0))
    return np.array(out, np.int64)


def main():
    from test_dataset_oracle import GOMOKU, records_of
    by = {}
    for g in GOMOKU:
        by.setdefault(g["bs"], []).append(g)
    data = {}
    for bs, games in sorted(by.items()):
        recs = records_of(games)
        for aug in (1, 0):
            (st, po, pl, va), = run(recs, bs, 1000 + bs, aug, False)
            k = f"b{bs}_a{aug}"
            data[k + "_state"], data[k + "_policy"], data[k + "_plen"], data[k + "_value"] = st, po, pl, va
        if bs == 9:
            s0, batch, sub, s1 = run(recs, bs, 1234, True, True)
            data["ops_batch_idx"] = row_index(s0, batch)
            data["ops_subset_idx"] = row_index(s0, sub)
            data["ops_shuffled_idx"] = row_index(s0, s1)
            k = "ops_s0"
            data[k + "_state"], data[k + "_policy"], data[k + "_plen"], data[k + "_value"] = s0
    np.savez_compressed(os.path.join(HERE, "ref_dataset.npz"), **data)
    print({k: v.shape for k, v in data.items() if k.endswith("_state") or k.endswith("_idx")})


if __name__ == "__main__":
    main()
