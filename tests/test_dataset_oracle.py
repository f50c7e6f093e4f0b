"""the CPU restatement of Dataset::extractExamples + augmentExample
(oracle/az_oracle.cpp az_oracle_dataset; src/selfplay/dataset.cpp:60-114,245-436).

Pinning: since round 4 the restatement is pinned against the reference's own Dataset, built with
only its JSON functions removed (oracle/build_ref_dataset.sh, tests/test_dataset_reference.py: every
store bitwise).  Before that, and still checked here, it was pinned by
  * the reference goldens for its inputs: the records are the reference's own self-play games
    (tests/golden/ref_games.json.gz, ref_go_games.json.gz) and the original (s = 0) example of
    every position equals the reference-pinned feature planes of that position;
  * known answers derived by hand from dataset.cpp's index arithmetic (the policy permutation and
    its `oldIdx/newIdx < size` guard on a child-order policy shorter than the board);
  * an independent numpy statement of the eight state transforms.
The shuffle is libstdc++'s std::shuffle on std::mt19937 (third-party, the same library here)."""
import gzip
import json
import os
import struct

import numpy as np
import pytest

import az_oracle as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    with gzip.open(os.path.join(GOLD, name), "rt") as f:
        return json.load(f)


def f32(bits):
    return struct.unpack("<f", struct.pack("<I", bits))[0]


def records_of(games):
    """Golden games -> (actions, child-order policies, result): the playSingleGame records."""
    out = []
    for g in games:
        acts = [m["action"] for m in g["moves"]]
        pols = [[f32(b) for b in m["probs"]] for m in g["moves"]]
        out.append((acts, pols, g["result"]))
    return out


GOMOKU = _load("ref_games.json.gz")
GO = _load("ref_go_games.json.gz")


def sym_states(s):
    """The reference's eight states (dataset.cpp:262-433) with numpy: rot90 maps (i,j)->(j,bs-1-i)."""
    r90 = np.rot90(s, -1, axes=(1, 2))
    r180 = np.rot90(s, 2, axes=(1, 2))
    r270 = np.rot90(s, 1, axes=(1, 2))
    fl = lambda x: x[:, :, ::-1]
    return [s, r90, r180, r270, fl(s), fl(r90), fl(r180), fl(r270)]


def test_policy_guard_known_answer():
    # bs 3, a child-order policy of 4 entries [a,b,c,d] (indices 0..3 of the 9-cell board):
    # rot90 new = j*3 + 2-i: 0->2, 3->1 (1->5, 2->8 skipped)          => [a, d, a, d]
    # rot180 new = (2-i)*3 + 2-j: every target >= 4                    => [a, b, c, d]
    # rot270 new = (2-j)*3 + i: 1->3, 2->0 (0->6, 3->7 skipped)         => [c, b, c, b]
    # flipH new = i*3 + 2-j: 0->2, 1->1, 2->0 (3->5 skipped)            => [c, b, a, d]
    # flipH of rot90 [a,d,a,d] => [a,d,a,d]; of rot180 => [c,b,a,d]; of rot270 [c,b,c,b] => [c,b,c,b]
    a, b, c, d = 0.1, 0.2, 0.3, 0.4
    st, po, pl, va = O.dataset(0, 3, [([4], [[a, b, c, d]], 2)])
    want = [[a, b, c, d], [a, d, a, d], [a, b, c, d], [c, b, c, b], [c, b, a, d], [a, d, a, d], [c, b, a, d],
            [c, b, c, b]]
    assert pl.tolist() == [4] * 8
    np.testing.assert_array_equal(po[:, :4], np.array(want, np.float32))
    assert not po[:, 4:].any()


def test_full_length_policy_is_the_state_permutation():
    # a policy over all A cells permutes exactly like a state plane
    bs = 5
    p = np.arange(25, dtype=np.float32) / 25
    st, po, pl, va = O.dataset(0, bs, [([12], [p.tolist()], 0)])
    for s, want in enumerate(sym_states(p.reshape(1, bs, bs))):
        np.testing.assert_array_equal(po[s], want.reshape(-1))


@pytest.mark.parametrize("game_type,idx", [(0, i) for i in range(len(GOMOKU))] + [(1, i) for i in range(len(GO))])
def test_examples_of_reference_games(game_type, idx):
    g = (GOMOKU if game_type == 0 else GO)[idx]
    bs = g["bs"]
    rec = records_of([g])[0]
    st, po, pl, va = O.dataset(game_type, bs, [rec], augment=True)
    n = len(rec[0])
    assert st.shape[0] == 8 * n
    res = rec[2]
    gv = 1.0 if res == 2 else -1.0 if res == 3 else 0.0
    for i in range(n):
        # original example: the reference-pinned planes of the position before move i
        if game_type == 0:
            planes = O.position(bs, rec[0][:i])[0]
        else:
            planes = O.go_position(bs, rec[0][:i])["planes"]
        np.testing.assert_array_equal(st[8 * i], planes)
        for s, want in enumerate(sym_states(planes)):
            np.testing.assert_array_equal(st[8 * i + s], want)
        # value: game result from the side to move, -gameValue for player 2 (so -0.0 for a draw)
        v = np.float32(-gv if i % 2 == 1 else gv)
        assert va[8 * i:8 * i + 8].view(np.uint32).tolist() == [v.view(np.uint32)] * 8
        assert pl[8 * i] == len(rec[1][i])
        assert po[8 * i, :pl[8 * i]].view(np.uint32).tolist() == np.array(rec[1][i], np.float32).view(np.uint32).tolist()


def test_without_augmentation_is_the_originals():
    recs = records_of(GOMOKU[:3])
    bs = GOMOKU[0]["bs"]
    recs = [r for r, g in zip(recs, GOMOKU[:3]) if g["bs"] == bs]
    a = O.dataset(0, bs, recs, augment=True)
    b = O.dataset(0, bs, recs, augment=False)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x[::8], y)


def test_shuffle_orders_are_libstdcxx_permutations():
    o = O.shuffle_orders(7, 1000, 3)
    for row in o:
        assert sorted(row.tolist()) == list(range(1000))
    assert not (o[0] == o[1]).all()
    np.testing.assert_array_equal(O.shuffle_orders(7, 1000, 3), o)      # seeded: reproducible
    np.testing.assert_array_equal(O.shuffle_orders(7, 1000, 1)[0], o[0])  # successive calls advance rng_
