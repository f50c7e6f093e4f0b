"""The engine's RCCL communicator (include/az_engine.h az_dist_*, csrc/dist.hip) on the GPU box's
one device: a world-1 communicator's barrier, counter reductions and weight broadcast through the
C-ABI, and the non-root side of a broadcast (a never-loaded net's weight buffers allocated, then
filled buffer by buffer from the root's) checked by forward outputs, bit for bit, in every
precision the net runs.  The rank logic at world 2 runs on CPU (tests/test_bench_cpu.py, gloo)."""
import ctypes

import numpy as np
import pytest


@pytest.fixture(scope="module")
def engine():
    import az_amd
    return az_amd.Engine(0)


@pytest.mark.gpu
def test_gpu_dist_world1_collectives(engine):
    import az_amd
    from az_amd import dist as azdist
    uid = azdist.Dist.unique_id()
    assert len(uid) == 128
    d = azdist.Dist(engine, 0, 1, uid, timeout_s=60)
    try:
        d.barrier()
        assert d.allreduce([1.0, 2.5, 3e9], "sum") == [1.0, 2.5, 3e9]
        assert d.allreduce([7.0], "max") == [7.0]
        desc = az_amd.gomoku_net_desc(board_size=15, channels=64, blocks=2, precision=az_amd.AZ_PREC_FP16, max_batch=8)
        net = az_amd.HipNeuralNetwork(engine, desc)
        with pytest.raises(az_amd.AzError):
            d.broadcast_weights(net)                     # the root's net has no weights
        net.init_random(11)
        x = (np.random.default_rng(2).random((8, 11, 15, 15)) < 0.3).astype(np.float32)
        lo0, v0 = net.forward(x)
        w0 = net.get_weights()
        d.broadcast_weights(net)                         # world 1: the root's own buffers, unchanged
        lo1, v1 = net.forward(x)
        assert np.array_equal(lo0, lo1) and np.array_equal(v0, v1)
        assert np.array_equal(net.get_weights(), w0)
        net.close()
    finally:
        d.close()


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(15, 256, 2, 64), (19, 128, 2, 32), (15, 64, 3, 16)],
                         ids=["15x15-256f", "19x19-128f", "15x15-64f"])
def test_gpu_broadcast_receiver_side_matches_root(engine, shape):
    """az_diag_net_copy_weights does to a never-loaded net what az_net_broadcast_weights does on a
    non-root rank; the receiving net must then compute the root's outputs bit for bit in every
    precision (f32, bf16x3, fp16, f16x3) -- the recorded buffer list misses no weight."""
    import az_amd
    from az_amd import _lib
    bs, F, blocks, B = shape
    # created as fp16 nets (the bench's nets): every piece set packed at load, the 64-filter fused
    # kernel's included (an F32-created 64-filter net packs none of them)
    desc = az_amd.gomoku_net_desc(board_size=bs, channels=F, blocks=blocks, precision=az_amd.AZ_PREC_FP16, max_batch=B)
    src = az_amd.HipNeuralNetwork(engine, desc)
    dst = az_amd.HipNeuralNetwork(engine, az_amd.gomoku_net_desc(board_size=bs, channels=F, blocks=blocks,
                                                                  precision=az_amd.AZ_PREC_FP16, max_batch=B))
    try:
        src.init_random(5)
        f = _lib.lib().az_diag_net_copy_weights
        f.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        _lib.check(f(dst.h, src.h))
        assert np.array_equal(dst.get_weights(), src.get_weights())
        x = (np.random.default_rng(3).random((B, 11, bs, bs)) < 0.25).astype(np.float32)
        for prec in (az_amd.AZ_PREC_F32, az_amd.AZ_PREC_BF16X3, az_amd.AZ_PREC_FP16, az_amd.AZ_PREC_F16X3):
            src.set_precision(prec)
            dst.set_precision(prec)
            ls, vs = src.forward(x)
            ld, vd = dst.forward(x)
            assert np.array_equal(ls, ld) and np.array_equal(vs, vd), prec
    finally:
        src.close()
        dst.close()
