"""The ParallelMCTS API beyond the self-play loop, on the device, against the REFERENCE itself:
runSingleSimulation, runBatchedSearch, releaseMemory (tree pruning; an expanded root left with no
children), and selectAction with useBatchInference off (draws on rng_ with libstdc++'s
discrete_distribution / uniform_int_distribution).  The golden scripts (tests/golden/ref_api.json.gz,
tests/golden/gen_golden.py API_CASES, oracle/ref_harness.cpp run_api) record after every operation
the root's raw N / VL / W bits and every child's (action, N, VL, W bits, P bits); each operation is
replayed through the C-ABI and compared bit for bit."""
import gzip
import json
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_api.json.gz")


def _cases():
    with gzip.open(GOLD, "rt") as f:
        return json.load(f)


@pytest.fixture(scope="module")
def engine():
    import az_amd
    return az_amd.Engine(0)


def _bits(x):
    return int(np.float32(x).view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("idx", range(5))
def test_gpu_api_script_matches_reference(engine, idx):
    import az_amd
    import az_oracle as O
    case = _cases()[idx]
    bs, sims, script, ev, seed = case["case"]
    m = az_amd.ParallelMCTS(engine, n_games=1, board_size=bs, num_simulations=sims,
                            evaluator=az_amd.AZ_EVAL_HASH if ev == "hash" else az_amd.AZ_EVAL_RANDOM,
                            eval_seed=seed, noise_seed=42, noise_seed_stride=0)
    m.newGames()
    batch_inference = True
    moves, last = [], -1
    for k, op in enumerate(case["ops"]):
        name = op["op"]
        c, arg = name[0], name[1:]
        ret = 0
        if c == "n":
            m.runSingleSimulation(1)
        elif c == "b":
            m.runBatchedSearch()
        elif c == "s":
            m.search()
        elif c == "r":
            ret = int(m.releaseMemory(int(arg))[0])
        elif c == "d":
            batch_inference = False
        elif c in "ae":
            legal = O.position(bs, moves)[3]
            ret = last = m.selectActionFor(0, c == "a", float(arg), legal, batch_inference)
        elif c == "m":
            m.updateWithMove(np.array([last], np.int32))
            moves.append(last)
            ret = last
        elif c == "x":
            m.addDirichletNoise(0.03, 0.25)
        assert ret == op["ret"], (idx, k, name, ret, op["ret"])
        N, VL, W = m.rootNode(0)
        assert [N, VL, _bits(W)] == op["root"], (idx, k, name, [N, VL, _bits(W)], op["root"])
        act, cN, cVL, cW, cP = m.rootChildren(0)
        got = [[int(a), int(n), int(v), _bits(w), _bits(p)] for a, n, v, w, p in zip(act, cN, cVL, cW, cP)]
        assert got == op["children"], (idx, k, name)
    m.close()
