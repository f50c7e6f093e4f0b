"""Pins the network restatement (oracle/net_oracle.py) and the HIP ConvNet against
golden outputs of the reference's own Python classes (tests/golden/gen_nn_golden.py):
SimplifiedModel (python/simple_export.py) at 8x8 and the exporter fallback stack
(python/scripts/simple_export.py) at 15x15."""
import os

import numpy as np
import pytest

GOLD = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "nn_golden.npz"))
CASES = {"simple8": (8, 16, 2, 64, 1, 1), "fallback15": (15, 16, 2, 225, 0, 0)}


def desc(name, precision=0):
    from az_amd._lib import NetDesc
    bs, ch, blocks, A, res, bias = CASES[name]
    return NetDesc(bs, 11, ch, blocks, A, 32, 8, 256, res, bias, precision, 4)


@pytest.mark.parametrize("name", list(CASES))
def test_net_oracle_matches_reference_classes(name):
    import net_oracle
    d = desc(name)
    blob = net_oracle.init_blob(d, int(GOLD[name + "_seed"]))
    lo, v = net_oracle.forward(d, blob, GOLD[name + "_x"])
    assert np.abs(lo - GOLD[name + "_logits"]).max() <= 1e-6
    assert np.abs(v - GOLD[name + "_value"]).max() <= 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(CASES))
def test_gpu_net_matches_reference_classes(name):
    import az_amd
    import net_oracle
    eng = az_amd.Engine(0)
    d = desc(name)
    net = az_amd.HipNeuralNetwork(eng, d)
    net.load_weights(net_oracle.init_blob(d, int(GOLD[name + "_seed"])))
    lo, v = net.forward(GOLD[name + "_x"])
    assert np.abs(lo - GOLD[name + "_logits"]).max() <= 1e-4
    assert np.abs(v - GOLD[name + "_value"]).max() <= 1e-4
    net.close()
