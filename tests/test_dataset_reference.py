"""Row f3 pinned against the REFERENCE itself: tests/golden/ref_dataset.npz holds what the reference's
own Dataset (src/selfplay/dataset.cpp extractExamples :64-114, augmentExample :245-434, getBatch
:120-145, getRandomSubset :228-243, shuffle :147-149; built by oracle/build_ref_dataset.sh with only
its JSON functions removed, run by tests/golden/gen_dataset_golden.py) produced from the reference's
own self-play games (ref_games.json.gz), one Dataset per board size, rng_ seeded 1000 + board.

CPU: the restatement (oracle/az_oracle.cpp az_oracle_dataset + libstdc++ std::shuffle on mt19937)
reproduces every store bitwise -- states, child-order policies (NaN entries included), their
lengths and the value bits -- and the getBatch / getRandomSubset / shuffle sequence.  The GPU twin
(tests/test_gpu_dataset.py::test_gpu_dataset_matches_reference_build) checks k_dataset_extract
against the same file."""
import os

import numpy as np
import pytest

import az_oracle as O
from test_dataset_oracle import GOMOKU, records_of

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_dataset.npz")
REF = np.load(GOLD)      # allow_pickle=False (numpy's default): plain arrays only


def groups():
    by = {}
    for g in GOMOKU:
        by.setdefault(g["bs"], []).append(g)
    return sorted(by.items())


def store(key):
    return tuple(REF[f"{key}_{f}"] for f in ("state", "policy", "plen", "value"))


def bits(x):
    return np.ascontiguousarray(x, np.float32).view(np.uint32)


def same_rows(a, b, order=None):
    """Bitwise equality of two stores (policies compared over the longer stride, zero-padded)."""
    st, po, pl, va = a
    if order is not None:
        st, po, pl, va = st[order], po[order], pl[order], va[order]
    rst, rpo, rpl, rva = b
    np.testing.assert_array_equal(bits(st), bits(rst))
    np.testing.assert_array_equal(pl, rpl)
    w = max(po.shape[1], rpo.shape[1])
    pad = lambda x: np.pad(x, ((0, 0), (0, w - x.shape[1])))
    np.testing.assert_array_equal(bits(pad(po)), bits(pad(rpo)))
    np.testing.assert_array_equal(bits(va), bits(rva))


@pytest.mark.parametrize("augment", [1, 0])
@pytest.mark.parametrize("bs", [g[0] for g in groups()])
def test_restatement_matches_reference_dataset(bs, augment):
    recs = records_of(dict(groups())[bs])
    ref = store(f"b{bs}_a{augment}")
    mine = O.dataset(0, bs, recs, bool(augment))
    assert len(mine[0]) == len(ref[0]) == sum(len(r[0]) for r in recs) * (8 if augment else 1)
    order = O.shuffle_orders(1000 + bs, len(ref[0]), 1)[0]       # extractExamples ends with shuffle()
    same_rows(mine, ref, order)


def test_restatement_matches_reference_rng_sequence():
    """getBatch(37), getRandomSubset(5), shuffle() after extractExamples on seed 1234 (9x9 games):
    each draws a fresh std::shuffle on the same rng_, in that order."""
    bs = 9
    recs = records_of(dict(groups())[bs])
    s0 = store("ops_s0")
    mine = O.dataset(0, bs, recs, True)
    E = len(s0[0])
    orders = O.shuffle_orders(1234, E, 4)
    same_rows(mine, s0, orders[0])
    slot = tuple(x[orders[0]] for x in mine)
    for name, want in (("ops_batch_idx", orders[1][:37]), ("ops_subset_idx", orders[2][:5]),
                       ("ops_shuffled_idx", orders[3])):
        # the fixture names rows of s0 by content (identical rows are interchangeable)
        same_rows(tuple(x[REF[name]] for x in s0), tuple(x[want] for x in slot))
