"""GPU parity of the device Dataset (Dataset::extractExamples + the 8-fold
augmentExample, getBatch, shuffle, getRandomSubset, save/load; src/selfplay/dataset.cpp) against the
CPU restatement (oracle/az_oracle.cpp az_oracle_dataset, pinned in tests/test_dataset_oracle.py).
Integer/byte work: bit-exact (states, policies including NaN entries, lengths, value bits)."""
import numpy as np
import pytest

from test_dataset_oracle import GO, GOMOKU, records_of


@pytest.fixture(scope="module")
def engine():
    import az_amd
    return az_amd.Engine(0)


def to_records(recs, bs):
    import az_amd
    out = []
    for acts, pols, res in recs:
        r = az_amd.GameRecord(bs, result=res)
        r.moves = [az_amd.MoveData(a, p, 0.0) for a, p in zip(acts, pols)]
        out.append(r)
    return out


def bits(x, nan_sign=True):
    b = np.ascontiguousarray(x, np.float32).view(np.uint32).copy()
    if not nan_sign:                      # JSON stores NaN as null: the sign bit does not survive
        b[np.isnan(np.asarray(x, np.float32))] = 0x7FC00000
    return b


def assert_same(dev, ref, order=None, nan_sign=True):
    st, po, pl, va = dev
    rst, rpo, rpl, rva = ref
    if order is not None:
        rst, rpo, rpl, rva = rst[order], rpo[order], rpl[order], rva[order]
    assert st.shape == rst.shape
    np.testing.assert_array_equal(bits(st), bits(rst))
    np.testing.assert_array_equal(pl, rpl)
    np.testing.assert_array_equal(bits(po, nan_sign), bits(rpo, nan_sign))
    np.testing.assert_array_equal(bits(va), bits(rva))


def groups(games):
    by = {}
    for g in games:
        by.setdefault(g["bs"], []).append(g)
    return sorted(by.items())


@pytest.mark.gpu
@pytest.mark.parametrize("game_type", [0, 1], ids=["gomoku", "go"])
@pytest.mark.parametrize("augment", [True, False])
def test_gpu_extract_matches_oracle_on_reference_games(engine, game_type, augment):
    import az_amd
    import az_oracle as O
    for bs, games in groups(GOMOKU if game_type == 0 else GO):
        recs = records_of(games)
        ds = az_amd.Dataset(engine, game_type, bs, seed=1)
        for r in to_records(recs, bs):
            ds.addGameRecord(r)
        E = ds.extractExamples(augment, shuffle=False)
        ref = O.dataset(game_type, bs, recs, augment)
        assert E == len(ref[0])
        assert_same(ds.gather(np.arange(E)), ref)
        ms, by = ds.profile_read()
        assert ms > 0 and by > 0
        ds.close()


@pytest.mark.gpu
def test_gpu_shuffle_getbatch_subset_follow_the_reference_rng(engine):
    """extractExamples ends with shuffle() (dataset.cpp:112-113); getBatch and getRandomSubset
    each std::shuffle a fresh index list on the same rng_ (:131, :235)."""
    import az_amd
    import az_oracle as O
    bs, games = 9, [g for g in GOMOKU if g["bs"] == 9]
    recs = records_of(games)
    seed = 1234
    ds = az_amd.Dataset(engine, 0, bs, seed=seed)
    for r in to_records(recs, bs):
        ds.addGameRecord(r)
    E = ds.extractExamples(True)
    ref = O.dataset(0, bs, recs, True)
    orders = O.shuffle_orders(seed, E, 4)
    assert_same(ds.gather(np.arange(E)), ref, orders[0])
    slot = [x[orders[0]] for x in ref]          # the shuffled store
    st, pols, va = ds.getBatch(37)
    idx = orders[1][:37]
    np.testing.assert_array_equal(bits(st), bits(slot[0][idx]))
    np.testing.assert_array_equal(bits(va), bits(slot[3][idx]))
    for i, p in enumerate(pols):
        np.testing.assert_array_equal(bits(p), bits(slot[1][idx[i], :slot[2][idx[i]]]))
    sub = ds.getRandomSubset(5)
    idx = orders[2][:5]
    for i, e in enumerate(sub):
        np.testing.assert_array_equal(bits(e.state), bits(slot[0][idx[i]]))
    ds.shuffle()                                 # Dataset::shuffle: permute the store on device
    assert_same(ds.gather(np.arange(E)), slot, orders[3])
    big = ds.getBatch(10 * E)                    # batchSize clamps to size()
    assert len(big[2]) == E
    ds.close()


@pytest.mark.gpu
def test_gpu_selfplay_records_to_examples(engine, tmp_path):
    """Records straight from the device self-play driver (SelfPlayManager.generateGames, NaN entries
    at T = 0 included) -> device examples == oracle examples; save/load round trip."""
    import az_amd
    import az_oracle as O
    bs = 9
    sp = az_amd.SelfPlayManager(engine, numGames=6, numSimulations=64, board_size=bs, evaluator=az_amd.AZ_EVAL_HASH)
    sp.setExplorationParams(0.03, 0.25, 1.0, 4, 0.0)
    recs = sp.generateGames(6, max_moves=40)
    sp.mcts.close()
    assert any(np.isnan(p).any() for r in recs for m in r.moves for p in [np.array(m.policy)])
    ds = az_amd.Dataset(engine, 0, bs, seed=3)
    for r in recs:
        ds.addGameRecord(r)
    E = ds.extractExamples(True, shuffle=False)
    ref = O.dataset(0, bs, [([m.action for m in r.moves], [m.policy for m in r.moves], r.result) for r in recs])
    assert_same(ds.gather(np.arange(E)), ref)
    # save/load (dataset.cpp:151-227) round trip, NaN as null (device self-play NaNs carry the
    # sign bit of inf/inf, 0xFFC00000; null reads back as quiet_NaN, 0x7FC00000)
    f = str(tmp_path / "ds.json")
    assert ds.saveToFile(f)
    ds2 = az_amd.Dataset(engine, 0, bs, seed=3)
    assert ds2.loadFromFile(f)
    assert ds2.size() == E
    assert_same(ds2.gather(np.arange(E)), ref, nan_sign=False)
    ds.close()
    ds2.close()


@pytest.mark.gpu
def test_gpu_extract_at_scale_properties(engine):
    """C3-sized record set (2048 games x 60 plies on 15x15): every example's symmetry group is
    consistent (the 8 states of a position are the numpy transforms of the first) and the
    originals equal the oracle on a sample of games."""
    import az_amd
    import az_oracle as O
    from test_dataset_oracle import sym_states
    bs, G, plies = 15, 2048, 60
    rng = np.random.default_rng(0)
    recs = []
    for g in range(G):
        acts = rng.permutation(bs * bs)[:plies].tolist()
        pols = [rng.random(bs * bs - i).astype(np.float32).tolist() for i in range(plies)]
        recs.append((acts, pols, int(rng.integers(1, 4))))
    ds = az_amd.Dataset(engine, 0, bs, seed=9)
    for r in to_records(recs, bs):
        ds.addGameRecord(r)
    E = ds.extractExamples(True, shuffle=False)
    assert E == G * plies * 8
    ms, by = ds.profile_read()
    print(f"extract {E} examples: {ms:.3f} ms, {by / ms / 1e6:.1f} GB/s algorithmic")
    pick = rng.choice(G * plies, 64, replace=False)
    st, po, pl, va = ds.gather(np.concatenate([np.arange(8) + 8 * p for p in pick]))
    for k in range(64):
        for s, want in enumerate(sym_states(st[8 * k])):
            np.testing.assert_array_equal(st[8 * k + s], want)
    sample = [0, 1, G - 1]
    ref = O.dataset(0, bs, [recs[g] for g in sample], True)
    idx = np.concatenate([np.arange(plies * 8) + g * plies * 8 for g in sample])
    assert_same(ds.gather(idx), ref)
    ds.close()


@pytest.mark.gpu
def test_gpu_bad_records_fail_loudly(engine):
    import az_amd
    ds = az_amd.Dataset(engine, 0, 5, seed=0)
    for acts in ([25], [-1], [3, 3]):
        ds.gameRecords = to_records([(acts, [[1.0]] * len(acts), 2)], 5)
        with pytest.raises(az_amd.AzError, match="out of range|occupied"):
            ds.extractExamples(True)
    ds.gameRecords = to_records([([1], [[0.5] * 26], 2)], 5)
    with pytest.raises(az_amd.AzError, match="policy length"):
        ds.extractExamples(True)
    with pytest.raises(az_amd.AzError, match="game type"):
        az_amd.Dataset(engine, 2, 8)
    ds.close()


@pytest.mark.gpu
@pytest.mark.parametrize("augment", [1, 0])
def test_gpu_dataset_matches_reference_build(engine, augment):
    """k_dataset_extract + the device store against the REFERENCE Dataset's own output
    (tests/golden/ref_dataset.npz from oracle/build_ref_dataset.sh; see test_dataset_reference.py):
    every board group, same rng_ seed, shuffle included -- bitwise; and the getBatch /
    getRandomSubset / shuffle sequence of the 9x9 group."""
    import az_amd
    from test_dataset_reference import REF, groups, same_rows, store
    for bs, games in groups():
        ds = az_amd.Dataset(engine, 0, bs, seed=1000 + bs)
        for r in to_records(records_of(games), bs):
            ds.addGameRecord(r)
        E = ds.extractExamples(bool(augment))
        ref = store(f"b{bs}_a{augment}")
        assert E == len(ref[0])
        same_rows(ds.gather(np.arange(E)), ref)
        ds.close()
    if not augment:
        return
    bs = 9
    ds = az_amd.Dataset(engine, 0, bs, seed=1234)
    for r in to_records(records_of(dict(groups())[bs]), bs):
        ds.addGameRecord(r)
    E = ds.extractExamples(True)
    s0 = store("ops_s0")
    same_rows(ds.gather(np.arange(E)), s0)
    st, pols, va = ds.getBatch(37)
    want = tuple(x[REF["ops_batch_idx"]] for x in s0)
    np.testing.assert_array_equal(bits(st), bits(want[0]))
    np.testing.assert_array_equal(bits(va), bits(want[3]))
    for i, p in enumerate(pols):
        np.testing.assert_array_equal(bits(p), bits(want[1][i, :want[2][i]]))
    sub = ds.getRandomSubset(5)
    for i, e in enumerate(sub):
        np.testing.assert_array_equal(bits(e.state), bits(s0[0][REF["ops_subset_idx"][i]]))
    ds.shuffle()
    same_rows(ds.gather(np.arange(E)), tuple(x[REF["ops_shuffled_idx"]] for x in s0))
    ds.close()
