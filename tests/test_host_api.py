"""The C++ host API and the _alphazero_cpp module (alphazero-multi-game_amd/cpp), CPU side:
host Gomoku rules / planes / hash / legal order against the oracle, GameRecord JSON in the
reference's nlohmann::json dump format, and loud failure without a GPU."""
import json
import math
import random

import numpy as np
import pytest

az = pytest.importorskip("_alphazero_cpp", reason="build the host module: make -C alphazero-multi-game_amd")


def test_gomoku_matches_oracle_positions():
    import az_oracle as O
    rng = random.Random(3)
    for bs in (9, 15):
        assert az.GomokuState(bs).getLegalMoves() == O.fresh_order(bs)   # first query
        for _ in range(20):
            s = az.GomokuState(bs)
            s.getLegalMoves()
            moves = []
            for _ in range(rng.randrange(0, bs * bs // 2)):
                if s.isTerminal():
                    break
                a = rng.choice(s.getLegalMoves())
                s.makeMove(a)
                moves.append(a)
            planes, h, res, legal = O.position(bs, moves)
            assert np.array_equal(np.asarray(s.getEnhancedTensorRepresentation(), np.float32), planes)
            assert s.getHash() == h
            assert int(s.getGameResult()) == res
            assert s.getLegalMoves() == (legal if res == 0 else [])


def test_gomoku_rules():
    s = az.GomokuState(9)
    for a, b in zip([0, 1, 2, 3], [9, 10, 11, 12]):   # Black row 0, cols 0..3; White row 1
        s.makeMove(a)
        s.makeMove(b)
    s.makeMove(4)
    assert s.getGameResult() == az.GameResult.WIN_PLAYER1 and s.isTerminal()
    assert s.undoMove() and not s.isTerminal()
    # Black overline (six) is not a win; White's is
    s = az.GomokuState(9)
    for a, b in zip([0, 1, 2, 4, 5], [72, 73, 74, 75, 80]):
        s.makeMove(a)
        s.makeMove(b)
    s.makeMove(3)                                     # black 0..5 = six in a row
    assert s.getGameResult() == az.GameResult.ONGOING
    w = az.GomokuState(9)
    for a, b in zip([80, 60, 42, 24, 78, 66], [9, 10, 11, 13, 14, 12]):
        w.makeMove(a)
        w.makeMove(b)
    assert w.getGameResult() == az.GameResult.WIN_PLAYER2
    with pytest.raises(Exception):
        w.makeMove(0)
    assert s.actionToString(0) == "A9" and s.stringToAction("J1") == 80 and s.stringToAction("I3") is None
    with pytest.raises(Exception):
        az.GomokuState(15, use_renju=True)


def nlohmann_number(v):
    """nlohmann::json number_float dump: shortest round-trip digits (Python repr gives the same
    digits), fixed notation when the decimal point position n is in (-4, 15], else d.ddde+XX."""
    if not math.isfinite(v):
        return "null"
    if v == 0:
        return "-0.0" if math.copysign(1, v) < 0 else "0.0"
    sign = "-" if v < 0 else ""
    m, e = f"{abs(v):.17e}".split("e")
    digits = repr(abs(v))
    # shortest digits from repr
    mant = digits.split("e")[0].replace(".", "").lstrip("0").rstrip("0") or "0"
    if "e" in digits:
        ex = int(digits.split("e")[1])
        lead = digits.split("e")[0].split(".")[0]
        n = ex + len(lead)
    else:
        ip, fp = (digits.split(".") + [""])[:2]
        ip = ip.lstrip("0")
        n = len(ip) if ip else -(len(fp) - len(fp.lstrip("0")))
    k = len(mant)
    if k <= n <= 15:
        return sign + mant + "0" * (n - k) + ".0"
    if 0 < n <= 15:
        return sign + mant[:n] + "." + mant[n:]
    if -4 < n <= 0:
        return sign + "0." + "0" * (-n) + mant
    out = mant[0] + ("." + mant[1:] if k > 1 else "")
    return sign + out + "e" + ("-" if n - 1 < 0 else "+") + f"{abs(n - 1):02d}"


def test_json_number_format_matches_nlohmann_rule():
    rng = np.random.default_rng(0)
    vals = list(rng.random(3000).astype(np.float32).astype(float))
    vals += list((rng.standard_normal(2000) * 10.0 ** rng.integers(-12, 18, 2000)).astype(np.float32).astype(float))
    vals += [0.0, -0.0, 1.0, 0.5, 1e-4, 1e-5, 123456789.0, 1e15, 1e16, float("nan"), float("inf")]
    for v in map(float, vals):
        assert az.jsonNumber(v) == nlohmann_number(v), v


def test_game_record_json_roundtrip(tmp_path):
    r = az.GameRecord(az.GameType.GOMOKU, 15)
    rng = np.random.default_rng(1)
    for i in range(4):
        p = rng.random(7).astype(np.float32)
        p = (p / p.sum()).tolist()
        if i == 3:
            p[2] = float("nan")                          # T = 0 distributions hold NaN
        r.addMove(int(rng.integers(225)), p, float(np.float32(rng.standard_normal())), i)
    r.setResult(az.GameResult.WIN_PLAYER2)
    r.setTimestamp(1700000000)
    text = r.toJson()
    # the nlohmann dump(4) layout: sorted keys, 4-space indent, float32 widened to double
    d = json.loads(text.replace("null", "NaN"))
    assert list(d) == sorted(d) and d["result"] == 3 and d["timestamp"] == "2023-11-14T22:13:20Z"
    assert text.splitlines()[1] == '    "board_size": 15,'
    ref = json.dumps({**d, "moves": [{k: m[k] for k in sorted(m)} for m in d["moves"]]}, indent=4, sort_keys=True)
    ref = ref.replace("NaN", "null")
    assert text == ref
    f = tmp_path / "000_game.json"
    assert r.saveToFile(str(f))
    back = az.GameRecord.loadFromFile(str(f))
    assert back.toJson() == text
    assert back.getResult() == az.GameResult.WIN_PLAYER2 and back.getMetadata() == (az.GameType.GOMOKU, 15, False)
    mv = az.MoveData.fromJson(r.getMoves()[0].toJson())
    assert mv.policy == r.getMoves()[0].policy and mv.action == r.getMoves()[0].action


def test_no_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError):
        az.HipNeuralNetwork(boardSize=9, channels=32, blocks=1)
    with pytest.raises(RuntimeError):
        az.ParallelMCTS(az.GomokuState(9), None)


def test_host_go_state_matches_reference_positions():
    """Host GoState (cpp/src/go_state.cpp) against the reference GoState goldens
    (tests/golden/ref_go_positions.json.gz): board after captures, ko point, hash, legal order
    (suicide / ko / superko), result, area score and the 8 feature planes."""
    import gzip
    import os
    gold = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_go_positions.json.gz")
    with gzip.open(gold, "rt") as f:
        pos = json.load(f)
    for bs, d in pos.items():
        bs = int(bs)
        for k, p in enumerate(d["positions"]):
            s = az.GoState(bs)
            for a in p["moves"]:
                s.makeMove(a)
            assert [s.getStone(a) for a in range(bs * bs)] == p["board"], (bs, k)
            assert s.getKoPoint() == p["ko"] and str(s.getHash()) == p["hash"], (bs, k)
            assert s.getLegalMoves() == p["legal"], (bs, k)
            assert int(s.getGameResult()) == p["result"] and s.isTerminal() == bool(p["terminal"]), (bs, k)
            assert [s.getCapturedStones(1), s.getCapturedStones(2)] == p["captured"], (bs, k)
            sc = np.asarray(s.calculateScore(), np.float32).view(np.uint32).tolist()
            assert sc == p["score"], (bs, k)
            planes = np.asarray(s.getEnhancedTensorRepresentation(), np.float32).reshape(-1)
            ref = np.zeros_like(planes)
            for i, b in p["planes"]:
                ref[i] = np.array([b], np.uint32).view(np.float32)[0]
            assert np.array_equal(planes.view(np.uint32), ref.view(np.uint32)), (bs, k)
            # undo back to the empty board
            for _ in p["moves"]:
                assert s.undoMove()
            assert s.getHash() == az.GoState(bs).getHash() and not s.undoMove()


def test_host_go_rules_and_factory():
    s = az.createGameState(az.GameType.GO, 9)
    assert isinstance(s, az.GoState) and s.getActionSpaceSize() == 82 and s.getLegalMoves()[0] == -1
    assert az.createGameState(az.GameType.GO).getBoardSize() == 19
    assert az.GoState(7).getBoardSize() == 19            # the reference constructor's fallback
    # a few stones, then pass / pass ends the game (area scoring, komi 7.5)
    s = az.GoState(9)
    for a in [1, 2, 9, 12, 19, 20, 11, 10]:
        s.makeMove(a)
    s.makeMove(-1)
    s.makeMove(-1)
    assert s.isTerminal() and s.getGameResult() in (az.GameResult.WIN_PLAYER1, az.GameResult.WIN_PLAYER2)
    with pytest.raises(Exception):
        az.createGameState(az.GameType.CHESS)


def test_training_example_json_matches_python_mirror_and_nlohmann_layout():
    """TrainingExample::toJson (dataset.cpp:16-33): j.dump() -- compact, keys sorted, NaN as null."""
    import az_amd
    e = az.TrainingExample()
    e.state = [[[0.0, 1.0], [0.5, 0.1]], [[1.0, 0.0], [0.0, 0.25]]]
    e.policy = [0.1, float("nan"), 1e-05]
    e.value = -0.0
    txt = e.toJson()
    assert txt == ('{"policy":[0.10000000149011612,null,9.999999747378752e-06],'
                   '"state":[[[0.0,1.0],[0.5,0.10000000149011612]],[[1.0,0.0],[0.0,0.25]]],"value":-0.0}')
    py = az_amd.TrainingExample(np.array(e.state, np.float32), np.array(e.policy, np.float32), e.value)
    assert py.toJson() == txt
    back = az.TrainingExample.fromJson(txt)
    assert back.state == e.state and back.policy[0] == e.policy[0] and math.isnan(back.policy[1])
    assert math.copysign(1.0, back.value) == -1.0


def test_dataset_without_gpu_fails_loudly():
    ds = az.Dataset()
    assert ds.size() == 0
    r = az.GameRecord(az.GameType.GOMOKU, 9)
    r.addMove(40, [1.0], 0.0, 0)
    ds.addGameRecord(r)
    with pytest.raises(RuntimeError, match="HIP|device"):
        ds.extractExamples(True)
    chess = az.Dataset()
    chess.addGameRecord(az.GameRecord(az.GameType.CHESS, 8))
    with pytest.raises(Exception, match="Chess"):
        chess.extractExamples(True)
