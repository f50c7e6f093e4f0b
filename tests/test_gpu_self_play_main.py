"""The self_play binary on the GPU (cpp/tools/self_play_main.cpp, the reference's
src/selfplay/selfplay_main.cpp): its records against the oracle's playSingleGame records bit for
bit (RandomPolicyNetwork -> the device random evaluator, the reference main's MCTS settings: fpu
0.1, root noise on every search), its metadata file, and the communicator path (--dist-id-file:
RCCL init, shape + weight broadcast of a random-init 20-block trunk net, the job counters reduced)
on one GPU."""
import glob
import json
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "alphazero-multi-game_amd", "build", "self_play")


def _bits(xs):
    return np.asarray(xs, np.float32).view(np.uint32).tolist()


@pytest.mark.gpu
def test_gpu_self_play_binary_matches_oracle(tmp_path):
    import az_oracle as O
    n, bs, sims = 4, 7, 32
    out = tmp_path / "games"
    r = subprocess.run([BIN, "--game", "gomoku", "--size", str(bs), "--num-games", str(n), "--simulations", str(sims),
                        "--batch-size", str(n), "--output-dir", str(out), "--threads", "4"],
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    refs = O.play(seed_stride=1, bs=bs, sims=sims, eval_kind=O.EVAL_RANDOM, eval_seed=0, n_games=n, fpu=0.1,
                  noise_each_search=1)
    for g in range(n):
        files = glob.glob(str(out / f"{g:03d}_*.json"))
        assert len(files) == 1, g
        rec = json.load(open(files[0]))
        ref = refs[g]
        assert rec["board_size"] == bs and len(rec["moves"]) == len(ref["moves"]), g
        for ply, (mv, rm) in enumerate(zip(rec["moves"], ref["moves"])):
            assert mv["action"] == rm["action"], (g, ply)
            # JSON keeps no NaN payload (null): at T = 0 the reference's NaN entries are compared as NaNs
            rp = np.asarray(rm["probs"], np.uint32).view(np.float32)
            assert len(mv["policy"]) == len(rp) and all((p is None) == bool(np.isnan(r)) for p, r in zip(mv["policy"], rp))
            assert _bits([0.0 if p is None else p for p in mv["policy"]]) == \
                _bits(np.where(np.isnan(rp), np.float32(0.0), rp)), (g, ply)
            assert _bits([mv["value"]])[0] == rm["value"], (g, ply)
        assert rec["result"] == ref["result"], g
    md = [json.load(open(f)) for f in glob.glob(str(out / "metadata_*.json"))]
    assert len(md) == 1
    md = md[0]
    assert (md["game"], md["board_size"], md["num_games_requested"], md["num_games_completed"]) == ("gomoku", bs, n, n)
    assert md["total_moves"] == sum(len(x["moves"]) for x in refs) and md["threads"] == 4
    assert md["world"] == 1 and md["job_total_moves"] == -1


@pytest.mark.gpu
def test_gpu_self_play_binary_dist_path(tmp_path):
    """--dist-id-file on one GPU: rank 0 writes the id, inits a 20 x 256 net, broadcasts shape and
    weights through the engine's communicator, plays, reduces the job counters."""
    out = tmp_path / "games"
    r = subprocess.run([BIN, "--num-games", "8", "--simulations", "16", "--batch-size", "8", "--max-moves", "4",
                        "--net-blocks", "20", "--net-channels", "256", "--precision", "fp16", "--output-dir", str(out),
                        "--world", "1", "--rank", "0", "--dist-id-file", str(tmp_path / "id")],
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    assert os.path.getsize(tmp_path / "id") == 128
    md = json.load(open(glob.glob(str(out / "metadata_*.json"))[0]))
    assert md["precision"] == "fp16" and md["fp16_used"] is True and md["world"] == 1
    assert md["job_total_moves"] == md["total_moves"] == 8 * 4 and md["job_games_completed"] == 8
    assert len(glob.glob(str(out / "0*_*.json"))) == 8
    assert "Job: 8 games, 32 moves" in r.stdout
