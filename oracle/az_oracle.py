"""oracle/az_oracle.py -- TEST INFRASTRUCTURE ONLY.

ctypes wrapper of oracle/az_oracle.cpp, the CPU restatement of the reference
self-play hot path (Mode S).  Only tests/, bench.py's
cpu_baseline leg and __graft_entry__.smoke() may import this module, and only as
the checker: nothing in the product path (alphazero-multi-game_amd/) imports it.
"""
import ctypes
import json
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")

EVAL_HASH, EVAL_RANDOM, EVAL_NET, EVAL_REPLAY, EVAL_UNIFORM = 0, 1, 2, 3, 4

# int cb(void* user, int game, const float* planes, int n_planes, int A, float* policy, float* value)
EVAL_CB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_float),
                           ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_float),
                           ctypes.POINTER(ctypes.c_float))


class OracleCfg(ctypes.Structure):
    _fields_ = [("bs", ctypes.c_int), ("sims", ctypes.c_int), ("max_moves", ctypes.c_int),
                ("vl", ctypes.c_int), ("noise_each_search", ctypes.c_int), ("temp_drop", ctypes.c_int),
                ("tt_log2", ctypes.c_int), ("eval_kind", ctypes.c_int),
                ("cpuct", ctypes.c_float), ("fpu", ctypes.c_float), ("alpha", ctypes.c_float),
                ("eps", ctypes.c_float), ("t_init", ctypes.c_float), ("t_final", ctypes.c_float),
                ("noise_seed", ctypes.c_uint), ("zobrist_seed", ctypes.c_uint), ("eval_seed", ctypes.c_uint),
                ("n_games", ctypes.c_int), ("game", ctypes.c_int)]

GAME_GOMOKU, GAME_GO = 0, 1


def build():
    """Compile the restatement (make -C oracle)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.az_oracle_play.restype = ctypes.c_void_p
        L.az_oracle_play.argtypes = [ctypes.POINTER(OracleCfg), ctypes.c_int, EVAL_CB, ctypes.c_void_p]
        L.az_oracle_free.argtypes = [ctypes.c_void_p]
        L.az_oracle_position.argtypes = [ctypes.c_int, ctypes.c_uint, ctypes.POINTER(ctypes.c_int), ctypes.c_int,
                                         ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_uint64),
                                         ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                                         ctypes.POINTER(ctypes.c_int)]
        L.az_oracle_go_position.argtypes = [ctypes.c_int, ctypes.c_uint, ctypes.POINTER(ctypes.c_int), ctypes.c_int,
                                            ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_uint64),
                                            ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                                            ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                                            ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_float)]
        L.az_oracle_fresh_order.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
        L.az_oracle_gamma.argtypes = [ctypes.c_uint, ctypes.c_float, ctypes.c_int, ctypes.c_int,
                                      ctypes.POINTER(ctypes.c_float)]
        fp, ip = ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_int)
        L.az_oracle_dataset.restype = ctypes.c_longlong
        L.az_oracle_dataset.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ip, ip, ip, fp, ip, ctypes.c_int,
                                        fp, fp, ctypes.c_int, ip, fp]
        L.az_oracle_shuffle.argtypes = [ctypes.c_uint, ctypes.c_longlong, ctypes.c_int,
                                        ctypes.POINTER(ctypes.c_longlong)]
        _lib = L
    return _lib


def make_cfg(bs=9, sims=100, max_moves=1 << 30, eval_kind=EVAL_HASH, eval_seed=7, n_games=1,
             noise_each_search=0, cpuct=1.5, fpu=0.0, vl=3, alpha=0.03, eps=0.25, temp_drop=30,
             t_init=1.0, t_final=0.0, noise_seed=42, zobrist_seed=12345, tt_log2=20, game=GAME_GOMOKU):
    return OracleCfg(bs, sims, max_moves, vl, noise_each_search, temp_drop, tt_log2, eval_kind,
                     cpuct, fpu, alpha, eps, t_init, t_final, noise_seed, zobrist_seed, eval_seed, n_games, game)


class StopPlay(Exception):
    """Raised by an evaluator to end play() early; play() then returns None."""


def play(seed_stride=0, evaluator=None, **kw):
    """Play games with the restated Mode S loop; returns a list of per-game dicts
    with the same structure as oracle/_ref/ref_harness `game` output.

    evaluator(game, planes[n_planes,bs,bs] float32) -> (policy[A] float32, value float)
    (11 planes / A = bs*bs for Gomoku, 8 planes / A = bs*bs + 1 for Go)
    is used for eval_kind EVAL_NET (raw logits; softmax applied as the reference)
    and EVAL_REPLAY (final policy)."""
    cfg = make_cfg(**kw)

    def _cb(user, game, planes, n_planes, A, pol, val):
        try:
            bs = int(round((A - (1 if cfg.game == GAME_GO else 0)) ** 0.5))
            x = np.ctypeslib.as_array(planes, shape=(n_planes, bs, bs)).copy()
            p, v = evaluator(game, x)
            p = np.asarray(p, dtype=np.float32).reshape(-1)
            ctypes.memmove(pol, p.ctypes.data, 4 * A)
            val[0] = float(v)
            return 0
        except StopPlay:
            return 2
        except Exception as e:  # surfaced as an abort in the oracle
            print("oracle evaluator failed:", repr(e))
            return 1

    cb = EVAL_CB(_cb)
    ptr = lib().az_oracle_play(ctypes.byref(cfg), seed_stride, cb, None)
    if not ptr:
        raise ValueError("az_oracle_play: unsupported configuration")
    try:
        s = ctypes.string_at(ptr).decode()
    finally:
        lib().az_oracle_free(ptr)
    return json.loads(s)


def position(bs, moves, zobrist_seed=12345):
    """(planes[11,bs,bs], zobrist hash, GameResult, legal-move order) after `moves`."""
    A = bs * bs
    mv = (ctypes.c_int * max(1, len(moves)))(*moves)
    planes = np.zeros(11 * A, dtype=np.float32)
    h = ctypes.c_uint64(0)
    res = ctypes.c_int(0)
    legal = (ctypes.c_int * A)()
    nl = ctypes.c_int(0)
    lib().az_oracle_position(bs, zobrist_seed, mv, len(moves),
                             planes.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), ctypes.byref(h),
                             ctypes.byref(res), legal, ctypes.byref(nl))
    return planes.reshape(11, bs, bs), h.value, res.value, list(legal[:nl.value])


def go_position(bs, moves, zobrist_seed=12345):
    """GoState after `moves`: dict of planes[8,bs,bs], hash, result, ko, legal order, board, score."""
    A = bs * bs
    mv = (ctypes.c_int * max(1, len(moves)))(*moves)
    planes = np.zeros(8 * A, dtype=np.float32)
    h = ctypes.c_uint64(0)
    res, ko, nl = ctypes.c_int(0), ctypes.c_int(0), ctypes.c_int(0)
    legal = (ctypes.c_int * (A + 1))()
    board = (ctypes.c_int * A)()
    score = (ctypes.c_float * 2)()
    lib().az_oracle_go_position(bs, zobrist_seed, mv, len(moves),
                                planes.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), ctypes.byref(h),
                                ctypes.byref(res), ctypes.byref(ko), legal, ctypes.byref(nl), board, score)
    return {"planes": planes.reshape(8, bs, bs), "hash": h.value, "result": res.value, "ko": ko.value,
            "legal": list(legal[:nl.value]), "board": list(board), "score": (score[0], score[1])}


def fresh_order(bs):
    out = (ctypes.c_int * (bs * bs))()
    n = lib().az_oracle_fresh_order(bs, out)
    return list(out[:n])


def gamma_draws(seed, alpha, calls, n):
    out = np.zeros(calls * n, dtype=np.float32)
    lib().az_oracle_gamma(seed, alpha, calls, n, out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
    return out.reshape(calls, n)


def dataset(game_type, bs, records, augment=True):
    """Dataset::extractExamples before its shuffle.  records: [(actions, [policy per move], result)].
    Returns states [E][planes][bs][bs], policy [E][stride] (zero past the length), plen [E], value [E]."""
    fp, ip = ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_int)
    A = bs * bs
    planes, stride = (8, A + 1) if game_type == 1 else (11, A)
    n_moves = np.array([len(r[0]) for r in records], np.int32)
    actions = np.array([a for r in records for a in r[0]], np.int32)
    nch = np.array([len(p) for r in records for p in r[1]], np.int32)
    pol = np.array([x for r in records for p in r[1] for x in p], np.float32)
    res = np.array([r[2] for r in records], np.int32)
    E = int(n_moves.sum()) * (8 if augment else 1)
    st = np.zeros((max(E, 1), planes, bs, bs), np.float32)
    po = np.zeros((max(E, 1), stride), np.float32)
    pl = np.zeros(max(E, 1), np.int32)
    va = np.zeros(max(E, 1), np.float32)
    e = lib().az_oracle_dataset(game_type, bs, len(records), n_moves.ctypes.data_as(ip), actions.ctypes.data_as(ip),
                                nch.ctypes.data_as(ip), pol.ctypes.data_as(fp), res.ctypes.data_as(ip), int(augment),
                                st.ctypes.data_as(fp), po.ctypes.data_as(fp), stride, pl.ctypes.data_as(ip),
                                va.ctypes.data_as(fp))
    assert e == E, (e, E)
    return st[:E], po[:E], pl[:E], va[:E]


def shuffle_orders(seed, n, calls=1):
    """std::shuffle of 0..n-1 on std::mt19937(seed), `calls` successive shuffles (Dataset::shuffle)."""
    out = np.zeros((calls, max(n, 1)), np.int64)
    lib().az_oracle_shuffle(seed, n, calls, out.ctypes.data_as(ctypes.POINTER(ctypes.c_longlong)))
    return out[:, :n]
