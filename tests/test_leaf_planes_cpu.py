"""Leaf records -> feature planes on the CPU (csrc/leaf_planes.h compiled for the host).

The search stores, per leaf that needs the network, a record of the planes' inputs (board, side to
move, last six moves; Go: ko point and min(10, group liberties)), and the network's input stage
(k_smallnet, k_rec_to_g8, k_rec_planes) builds the 16 channels from it with the header's
az_leaf_planes.  Here the same header is compiled with g++ (IEEE division, no FMA contraction) and
fed records built from the reference's own position fixtures (tests/golden/ref_positions.json.gz,
ref_go_positions.json.gz, produced by oracle/ref_harness from the reference's GomokuState / GoState):
every plane must equal the reference's bit for bit.  The GPU tests pin the device side (the planes
the kernels log during self-play equal the oracle's, tests/test_gpu_selfplay_net.py)."""
import ctypes
import gzip
import json
import os
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")


@pytest.fixture(scope="module")
def lib(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("leafplanes") / "libleafplanes.so")
    subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-ffp-contract=off", "-fno-fast-math",
                    "-Wno-unknown-pragmas", os.path.join(HERE, "native", "leaf_planes_host.cpp"), "-o", out],
                   check=True)
    L = ctypes.CDLL(out)
    L.az_rec_planes_host.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    return L


def _load(name):
    with gzip.open(os.path.join(GOLD, name), "rt") as f:
        return json.load(f)


def _ref_planes(p, C, bs):
    flat = np.zeros(C * bs * bs, np.uint32)
    for i, bits in p["planes"]:
        flat[i] = bits
    return flat.reshape(C, bs * bs)


def _synth(lib, rec, go, bs):
    out = np.zeros((bs * bs, 16), np.float32)
    lib.az_rec_planes_host(rec.ctypes.data, go, bs, out.ctypes.data)
    return out.T.copy()          # [16][A]


def _record(lib, board, player, ko=-1, hist6=None, libs=None):
    rec = np.zeros(lib.az_rec_bytes(), np.uint8)
    A = len(board)
    rec[:A] = board
    if libs is not None:
        rec[384:384 + A] = libs
    meta = np.full(8, -1, np.int32)
    meta[0], meta[1] = player, ko
    if hist6 is not None:
        meta[2:8] = hist6
    rec[768:800] = meta.view(np.uint8)
    return rec


@pytest.mark.parametrize("bs", [5, 9, 15])
def test_gomoku_record_planes_match_reference(lib, bs):
    pos = _load("ref_positions.json.gz")[str(bs)]["positions"]
    for k, p in enumerate(pos):
        board = np.zeros(bs * bs, np.uint8)
        for i, a in enumerate(p["moves"]):
            board[a] = 1 if i % 2 == 0 else 2
        hist = list(reversed(p["moves"]))[:6]
        hist += [-1] * (6 - len(hist))
        got = _synth(lib, _record(lib, board, p["player"], hist6=hist), 0, bs)
        ref = _ref_planes(p, p["nplanes"], bs)
        assert np.array_equal(got[:p["nplanes"]].view(np.uint32), ref), (bs, k)
        assert not got[p["nplanes"]:].any()


def _go_libs(board, bs):
    """min(10, liberties of the stone's group) per cell, 0 on empty points."""
    out = np.zeros(bs * bs, np.uint8)
    seen = np.zeros(bs * bs, bool)
    for s in range(bs * bs):
        if board[s] == 0 or seen[s]:
            continue
        group, libs, stack = [], set(), [s]
        seen[s] = True
        while stack:
            c = stack.pop()
            group.append(c)
            y, x = divmod(c, bs)
            for ny, nx in ((y - 1, x), (y + 1, x), (y, x - 1), (y, x + 1)):
                if 0 <= ny < bs and 0 <= nx < bs:
                    n = ny * bs + nx
                    if board[n] == 0:
                        libs.add(n)
                    elif board[n] == board[s] and not seen[n]:
                        seen[n] = True
                        stack.append(n)
        for c in group:
            out[c] = min(10, len(libs))
    return out


@pytest.mark.parametrize("bs", [9, 13, 19])
def test_go_record_planes_match_reference(lib, bs):
    pos = _load("ref_go_positions.json.gz")[str(bs)]["positions"]
    for k, p in enumerate(pos):
        board = np.array(p["board"], np.uint8)
        rec = _record(lib, board, p["player"], ko=p["ko"], libs=_go_libs(board, bs))
        got = _synth(lib, rec, 1, bs)
        ref = _ref_planes(p, p["nplanes"], bs)
        assert np.array_equal(got[:8].view(np.uint32), ref), (bs, k)
        assert not got[8:].any()
