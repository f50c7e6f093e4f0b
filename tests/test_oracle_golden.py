"""Pins the CPU restatement (oracle/az_oracle.cpp) against golden vectors produced by
the patched REFERENCE build (tests/golden/gen_golden.py -> oracle/_ref/ref_harness).

Everything here is bit-exact: visit counts, virtual loss, W and P as fp32 bit
patterns, visit distributions, chosen actions, root values, TT lookup/hit counts."""
import gzip
import json
import os

import numpy as np
import pytest

import az_oracle as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    p = os.path.join(GOLD, name)
    if name.endswith(".gz"):
        with gzip.open(p, "rt") as f:
            return json.load(f)
    with open(p) as f:
        return json.load(f)


GAMES = _load("ref_games.json.gz")


@pytest.mark.parametrize("idx", range(len(GAMES)), ids=[str(g["case"]) for g in GAMES])
def test_oracle_game_matches_reference(idx):
    ref = GAMES[idx]
    bs, sims, mm, ev, es, nes, cp, fpu = ref["case"]
    got = O.play(bs=bs, sims=sims, max_moves=mm, eval_kind=O.EVAL_HASH if ev == "hash" else O.EVAL_RANDOM,
                 eval_seed=es, noise_each_search=nes, cpuct=cp, fpu=fpu)[0]
    assert got["init_root"] == ref["init_root"]
    assert len(got["moves"]) == len(ref["moves"])
    for a, b in zip(ref["moves"], got["moves"]):
        for k in ("root", "children", "probs", "action", "value", "tt_lookups", "tt_hits", "evals"):
            assert a[k] == b[k], (a["ply"], k)
    assert got["result"] == ref["result"]


def test_golden_covers_transpositions_and_draws():
    hits = [g["moves"][-1]["tt_hits"] for g in GAMES]
    assert max(hits) > 100                      # TT emulation is exercised
    assert any(g["result"] == 1 for g in GAMES)  # a drawn (board-full) game
    assert any(g["result"] == 2 for g in GAMES) and any(g["result"] == 3 for g in GAMES)


@pytest.mark.parametrize("bs", [5, 9, 15])
def test_oracle_positions_match_reference(bs):
    pos = _load("ref_positions.json.gz")[str(bs)]
    for k, p in enumerate(pos["positions"]):
        planes, h, res, legal = O.position(bs, p["moves"])
        assert str(h) == p["hash"]
        assert res == p["result"]
        assert legal == p["legal"]
        flat = planes.reshape(-1)
        ref = np.zeros_like(flat)
        for i, bits in p["planes"]:
            ref[i] = np.array([bits], dtype=np.uint32).view(np.float32)[0]
        assert np.array_equal(flat.view(np.uint32), ref.view(np.uint32)), k
        if k == 0:
            assert O.fresh_order(bs) == p["first_order"]


def test_oracle_gamma_matches_reference():
    g = _load("ref_gamma.json")
    alpha = float(np.array([g["alpha_bits"]], dtype=np.uint32).view(np.float32)[0])
    calls = g["calls"]
    got = O.gamma_draws(42, alpha, len(calls), len(calls[0]))
    assert got.view(np.uint32).tolist() == calls


# ---------------------------------------------------------------- Go
GO_GAMES = _load("ref_go_games.json.gz")


def _f32(b):
    return float(np.array([b], dtype=np.uint32).view(np.float32)[0])


@pytest.mark.parametrize("bs", [9, 13, 19])
def test_oracle_go_positions_match_reference(bs):
    """GoState restatement vs the reference GoState (go_state.cpp / go_rules.cpp): board after
    captures, ko point, Zobrist hash (pieces, side, ko / rules / komi features), legal-move order
    with suicide, ko and positional superko, area score, result and the 8 feature planes."""
    pos = _load("ref_go_positions.json.gz")[str(bs)]
    for k, p in enumerate(pos["positions"]):
        g = O.go_position(bs, p["moves"])
        assert g["board"] == p["board"], k
        assert g["ko"] == p["ko"], k
        assert str(g["hash"]) == p["hash"], k
        assert g["legal"] == p["legal"], k
        assert g["result"] == p["result"], k
        assert [int(np.array([x], np.float32).view(np.uint32)[0]) for x in g["score"]] == p["score"], k
        flat = g["planes"].reshape(-1)
        ref = np.zeros_like(flat)
        for i, bits in p["planes"]:
            ref[i] = _f32(bits)
        assert p["nplanes"] == 8
        assert np.array_equal(flat.view(np.uint32), ref.view(np.uint32)), k


def test_go_golden_covers_captures_ko_and_scoring():
    pos = [p for v in _load("ref_go_positions.json.gz").values() for p in v["positions"]]
    assert any(sum(p["captured"]) > 0 for p in pos)       # captures happened
    assert any(p["ko"] >= 0 for p in pos)                  # a ko point is live
    assert any(p["terminal"] for p in pos)                 # pass / pass, area scoring
    assert any(len(p["legal"]) - 1 < sum(1 for c in p["board"] if c == 0) for p in pos)  # an empty point is illegal


@pytest.mark.parametrize("idx", range(len(GO_GAMES)), ids=[str(g["case"]) for g in GO_GAMES])
def test_oracle_go_game_matches_reference(idx):
    ref = GO_GAMES[idx]
    bs, sims, mm, ev, es, nes, cp, fpu = ref["case"]
    got = O.play(bs=bs, sims=sims, max_moves=mm, eval_kind=O.EVAL_HASH, eval_seed=es, noise_each_search=nes,
                 cpuct=cp, fpu=fpu, game=O.GAME_GO)[0]
    assert got["init_root"] == ref["init_root"]
    assert len(got["moves"]) == len(ref["moves"])
    for a, b in zip(ref["moves"], got["moves"]):
        for k in ("root", "children", "probs", "action", "value", "tt_lookups", "tt_hits", "evals"):
            assert a[k] == b[k], (a["ply"], k)
    assert got["result"] == ref["result"]
