"""Row f4 (DDW-RandWire, src/nn/ddw_randwire_resnet.cpp) on the CPU, no GPU needed:

* the oracle restatement (oracle/randwire_oracle.py) reproduces the reference C++ module's own
  forward outputs (tests/golden/randwire_golden.npz, from oracle/_ref/ref_randwire: three
  configurations incl. 1-3 blocks, 16/32 channels, 8/9/15 boards);
* the engine's host-side graph builder (az_randwire_graph, csrc/randwire.h) reproduces every
  reference graph of the default 20-block net: nodes() order (= state_dict order), inputs,
  outputs, predecessor lists (router concat order, duplicate edges included), topological order;
* the blob layout is the reference module's state_dict (the generator asserted the names and
  shapes; here its size and the router widths follow the graphs)."""
import os
import types

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden", "randwire_golden.npz")
CASES = ["c16_b1_h9", "c32_b2_h15", "c16_b3_h8"]


def _desc(inp, bs, ch, nb):
    return types.SimpleNamespace(board_size=bs, in_planes=inp, channels=ch, blocks=nb, action_size=bs * bs,
                                 head_channels=32, pool=min(8, bs), fc_hidden=256)


@pytest.mark.parametrize("case", CASES)
def test_randwire_oracle_matches_reference_module(case):
    import randwire_oracle as RW
    g = np.load(GOLD)
    inp, bs, ch, nb, B, seed = (int(v) for v in g[case + "_cfg"])
    d = _desc(inp, bs, ch, nb)
    graphs = RW.load_graphs()
    blob = RW.init_blob(d, graphs, seed)
    lo, v = RW.forward(d, graphs, blob, g[case + "_planes"])
    assert lo.shape == (B, bs * bs)
    np.testing.assert_allclose(lo, g[case + "_logits"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(v, g[case + "_value"], rtol=0, atol=1e-6)


def test_randwire_graphs_match_reference():
    import az_amd
    import randwire_oracle as RW
    graphs = RW.load_graphs()
    assert len(graphs) == 20
    dup = 0
    for i, ref in enumerate(graphs):
        m = az_amd.randwire_graph(i)
        for k in ("nodes", "topo", "input_nodes", "output_nodes"):
            assert m[k] == ref[k], (i, k)
        for v in range(32):
            assert m["preds"][v] == ref["preds"][v], (i, v)
            dup += len(ref["preds"][v]) - len(set(ref["preds"][v]))
        # every edge runs low -> high, so the topological order is a valid compute order
        pos = {v: k for k, v in enumerate(ref["topo"])}
        assert all(pos[a] < pos[b] for a, b in ref["edges"])
        assert sum(len(p) for p in ref["preds"].values()) == len(ref["edges"]) == 64
    assert dup > 0   # the reference keeps duplicate edges (a router then reads one input twice)


def test_randwire_blob_layout():
    import randwire_oracle as RW
    graphs = RW.load_graphs()
    d = _desc(11, 9, 16, 1)
    spec = RW.param_shapes(d, graphs)
    routers = [s for s in spec if ".router_" in s[0] and s[0].endswith(".conv.weight")]
    assert len(routers) == sum(1 for v in graphs[0]["nodes"] if graphs[0]["preds"][v])
    for name, shape, _, _ in routers:
        v = int(name.split("router_")[1].split(".")[0])
        assert shape == (16, 16 * len(graphs[0]["preds"][v]), 1, 1)
    assert sum(int(np.prod(s[1])) for s in spec) == 866722   # the reference module's state size (generator log)


def test_randwire_graph_bad_block():
    import az_amd
    with pytest.raises(az_amd.AzError):
        az_amd.randwire_graph(-1)


def test_randwire_explicit_graph_parsing_errors():
    """az_net_create_randwire_graphs validates the wiring on the host before touching a device:
    a non-permutation order, a bad predecessor, a cycle and trailing ints are refused by name."""
    import ctypes
    import az_amd
    from az_amd import _lib
    L = _lib.lib()
    d = az_amd.randwire_net_desc(9, 16, 1, 11, 4)

    def err(ints):
        arr = (ctypes.c_int * len(ints))(*ints)
        h = ctypes.c_void_p()
        rc = L.az_net_create_randwire_graphs(None, ctypes.byref(d), arr, len(ints), ctypes.byref(h))
        return rc, L.az_last_error().decode()

    ok = [3, 0, 1, 2, 0, 1, 0, 2, 0, 1, 1, 2]   # 0 -> 1, {0, 1} -> 2, sink 2
    rc, msg = err(ok)
    assert rc == -1 and "null argument" in msg          # valid wiring: fails only at the null engine
    assert "permutation" in err([3, 0, 0, 2] + ok[4:])[1]
    assert "predecessor" in err([3, 0, 1, 2, 0, 1, 7, 2, 0, 1, 1, 2])[1]
    assert "cycle" in err([3, 0, 1, 2, 1, 2, 1, 0, 1, 1, 1, 2])[1]
    assert "ints read" in err(ok + [5])[1]
