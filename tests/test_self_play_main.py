"""The self_play binary (alphazero-multi-game_amd/cpp/tools/self_play_main.cpp; the reference's
src/selfplay/selfplay_main.cpp:156-392) and its run metadata file (row f1: metadata_<ticks>.json,
selfplay_main.cpp:353-389) -- CPU parts: the metadata text (the reference's keys in its order and
its ostream number formatting, then the engine's extension keys), the file name, the game shard
of a per-GPU job, and the binary's help / loud failure without a GPU."""
import glob
import json
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "alphazero-multi-game_amd")
BIN = os.path.join(PKG, "build", "self_play")
sys.path.insert(0, PKG)

# selfplay_main.cpp:357-382, in order
REF_KEYS = ["game", "board_size", "num_games_requested", "num_games_completed", "simulations", "threads",
            "temperature", "temp_drop", "final_temp", "dirichlet_alpha", "dirichlet_epsilon", "variant", "model_path",
            "total_moves", "avg_moves_per_game", "total_time_seconds", "avg_moves_per_second", "use_gpu", "batch_size",
            "batch_timeout", "fp16_used", "c_puct", "fpu_reduction", "virtual_loss", "use_transposition_table",
            "progressive_widening"]
EXT_KEYS = ["rank", "world", "first_game_id", "precision", "device", "job_games_completed", "job_total_moves",
            "job_seconds", "job_moves_per_second"]


def test_run_metadata_text_and_field_set(tmp_path):
    import _alphazero_cpp as A
    m = A.RunMetadata()
    m.game, m.boardSize, m.numGamesRequested, m.numGamesCompleted = "go", 19, 1024, 1000
    m.totalMoves, m.avgMovesPerGame, m.totalTimeSeconds, m.avgMovesPerSecond = 250000, 250.0, 3, 83333.336
    m.modelPath, m.fp16Used, m.precision = 'models/a "b".pt', True, "fp16"
    txt = A.runMetadataJson(m)
    keys = re.findall(r'^  "([a-z_0-9]+)": ', txt, flags=re.M)
    assert keys == REF_KEYS + EXT_KEYS
    j = json.loads(txt)                                  # valid JSON (the path's quotes escaped)
    assert j["model_path"] == 'models/a "b".pt' and j["game"] == "go" and j["fp16_used"] is True
    # the reference's fresh std::ofstream: default 6-significant-digit floats, integers as integers
    assert '"temperature": 1,\n' in txt and '"dirichlet_alpha": 0.03,\n' in txt and '"c_puct": 1.5,\n' in txt
    assert '"avg_moves_per_game": 250,\n' in txt and '"avg_moves_per_second": 83333.3,\n' in txt
    assert '"total_time_seconds": 3,\n' in txt and txt.startswith("{\n") and txt.endswith("\n}\n")
    path = A.writeRunMetadata(m, str(tmp_path))
    assert re.fullmatch(r"metadata_[0-9]+\.json", os.path.basename(path)) and open(path).read() == txt
    assert A.writeRunMetadata(m, str(tmp_path / "missing" / "dir")) == ""


def test_shard_games_matches_bench_shards():
    import _alphazero_cpp as A
    from az_amd import dist as azdist
    for world, total in ((1, 2048), (2, 2048), (8, 2048), (3, 10), (8, 1024), (4, 3)):
        ids = []
        for r in range(world):
            s = A.shardGames(r, world, total)
            py = azdist.shard_range(r, world, total)
            assert (s.firstGame, s.numGames, s.noiseSeed) == (py["first_game"], py["games"], py["noise_seed"])
            ids += list(range(s.firstGame, s.firstGame + s.numGames))
        assert ids == list(range(total))


def test_self_play_binary_help_and_no_gpu():
    if not os.path.exists(BIN):
        pytest.skip("build alphazero-multi-game_amd first")
    r = subprocess.run([BIN, "--help"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "--dist-id-file" in r.stdout and "--num-games" in r.stdout
    r = subprocess.run([BIN, "--no-gpu"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "no CPU path" in r.stderr
    r = subprocess.run([BIN, "--world", "2", "--rank", "1"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "--dist-id-file" in r.stderr
