"""Row f4: the DDW-RandWire network (src/nn/ddw_randwire_resnet.cpp) on the device engine
(az_net_create_randwire: f32 MFMA GEMMs for the 3x3 convs and routers, k_se_residual for
SE + residual + ReLU), against

* the reference C++ module's own outputs (tests/golden/randwire_golden.npz), tolerance 1e-4
  (BASELINE.json north_star);
* the oracle restatement (pinned to those goldens) at the reference's default width and depth
  (128 channels, 20 rand-wire blocks = 640 SE residual blocks), relative to the output scale;
* itself: a board's outputs do not depend on its batch position or batch size (bitwise);
* the search: a self-play game whose leaves the rand-wire net evaluates replays bit for bit
  through the CPU restatement of the search, and every logged evaluation matches the oracle."""
import types

import numpy as np
import pytest

GOLD_CASES = ["c16_b1_h9", "c32_b2_h15", "c16_b3_h8"]


def _net(eng, bs, ch, nb, B, inp=11):
    import az_amd
    return az_amd.HipNeuralNetwork(eng, az_amd.randwire_net_desc(bs, ch, nb, inp, B), randwire=True)


BF16X3_CAP = 128   # the bf16x3 node convs run on conv3x3_v4 from this capacity up (below: f32 K-split)


@pytest.mark.gpu
@pytest.mark.parametrize("case", GOLD_CASES)
def test_gpu_randwire_matches_reference_module(case):
    import os
    import az_amd
    import randwire_oracle as RW
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "randwire_golden.npz"))
    inp, bs, ch, nb, B, seed = (int(v) for v in g[case + "_cfg"])
    eng = az_amd.Engine(0)
    net = _net(eng, bs, ch, nb, B, inp)
    graphs = RW.load_graphs()
    blob = RW.init_blob(net.desc, graphs, seed)
    assert net.num_params == blob.size
    net.init_random(seed)                      # az_net_init_random over the rand-wire blob order
    assert np.array_equal(net.get_weights().view(np.uint32), blob.view(np.uint32))
    lo, v = net.forward(g[case + "_planes"])
    dl = np.abs(lo - g[case + "_logits"]).max()
    dv = np.abs(v - g[case + "_value"]).max()
    print(f"{case}: max|dlogit| {dl:.3g} max|dvalue| {dv:.3g}")
    assert dl <= 1e-4 and dv <= 1e-4
    p, pv = net.predictBatch(g[case + "_planes"])
    import net_oracle
    assert np.abs(p - net_oracle.softmax_policy(g[case + "_logits"])).max() <= 1e-4
    net.close()
    eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("bs,ch,nb,B", [(15, 128, 20, 2), (15, 128, 2, 24), (9, 64, 3, 7)])
def test_gpu_randwire_matches_oracle(bs, ch, nb, B):
    import az_amd
    import randwire_oracle as RW
    eng = az_amd.Engine(0)
    net = _net(eng, bs, ch, nb, B)
    graphs = RW.load_graphs()
    net.init_random(100 + nb)
    blob = net.get_weights()
    rng = np.random.default_rng(nb)
    planes = (rng.random((B, 11, bs, bs)) < 0.3).astype(np.float32)
    lo, v = net.forward(planes)
    rl, rv = RW.forward(net.desc, graphs, blob, planes)
    scale = max(1.0, float(np.abs(rl).max()))
    dl, dv = np.abs(lo - rl).max(), np.abs(v - rv).max()
    print(f"{bs}x{bs} {ch}ch {nb} blocks B={B}: |logit| max {np.abs(rl).max():.3g}, max|dlogit| {dl:.3g}, "
          f"max|dvalue| {dv:.3g}")
    assert dl <= 1e-4 * scale and dv <= 1e-4
    # batch position / size independence (bitwise)
    sub = [B - 1, 0] if B > 1 else [0]
    lo2, v2 = net.forward(planes[sub])
    assert np.array_equal(lo2.view(np.uint32), lo[sub].view(np.uint32))
    assert np.array_equal(v2.view(np.uint32), v[sub].view(np.uint32))
    net.close()
    eng.close()


@pytest.mark.gpu
def test_gpu_randwire_selfplay_replay():
    import az_amd
    import az_oracle as O
    import net_oracle
    import randwire_oracle as RW
    bs, sims, G, moves, logged = 9, 40, 3, 5, 1
    eng = az_amd.Engine(0)
    net = _net(eng, bs, 16, 1, G)
    net.init_random(5)
    blob = net.get_weights()
    m = az_amd.ParallelMCTS(eng, n_games=G, board_size=bs, num_simulations=sims, evaluator=az_amd.AZ_EVAL_NET,
                            net=net, noise_seed=42, noise_seed_stride=1)
    cap = (sims + 2) * (moves + 1)
    m.enableEvalLog(logged, cap)
    m.newGames()
    m.addDirichletNoise(0.03, 0.25)
    dev = []
    for ply in range(moves):
        m.search()
        act, val, probs, cact, nch = m.select(True, 1.0)
        a, N, VL, W, P = m.rootChildren(logged)
        dev.append(dict(action=int(act[logged]), value=float(val[logged]), N=N.tolist(), W=W.view(np.uint32).tolist(),
                        P=P.view(np.uint32).tolist(), probs=probs[logged, :nch[logged]].view(np.uint32).tolist()))
        term, _ = m.updateWithMove(act)
        if ply % 2 == 0:
            m.addDirichletNoise(0.03, 0.25)
        if term[logged]:
            break
    pol, valv, planes = m.readEvalLog(cap)
    assert len(pol) > sims
    k = [0]

    def replay(game, x):
        i = k[0]
        k[0] += 1
        assert np.array_equal(x, planes[i]), f"feature planes differ at evaluation {i}"
        return pol[i], float(valv[i])

    ref = O.play(bs=bs, sims=sims, max_moves=len(dev), eval_kind=O.EVAL_REPLAY, evaluator=replay,
                 noise_seed=42 + logged)[0]
    assert k[0] == len(pol)
    for ply, (d, r) in enumerate(zip(dev, ref["moves"])):
        kids = r["children"]
        assert d["N"] == [c[1] for c in kids], ply
        assert d["W"] == [c[3] for c in kids] and d["P"] == [c[4] for c in kids], ply
        assert d["probs"] == r["probs"] and d["action"] == r["action"], ply
    rl, rv = RW.forward(net.desc, RW.load_graphs(), blob, planes)
    assert np.abs(valv - rv).max() <= 1e-4
    assert np.abs(pol - net_oracle.softmax_policy(rl)).max() <= 1e-4
    m.close()
    net.close()
    eng.close()


@pytest.mark.gpu
def test_gpu_randwire_rejects_bad_desc():
    import az_amd
    eng = az_amd.Engine(0)
    import randwire_oracle as RW
    graphs = RW.load_graphs()
    for kw in (dict(precision=az_amd.AZ_PREC_FP16), dict(conv_bias=1), dict(channels=24), dict(channels=2048),
               dict(pool=4)):
        d = az_amd.randwire_net_desc(9, 16, 1, 11, 4)
        for k, v in kw.items():
            setattr(d, k, v)
        with pytest.raises(az_amd.AzError):
            az_amd.HipNeuralNetwork(eng, d, randwire=True)
        # the explicit-wiring entry point validates the same desc (k_se_residual's fixed LDS arrays,
        # float4 channel quads; no conv bias; pool min(8, board))
        with pytest.raises(az_amd.AzError):
            az_amd.HipNeuralNetwork(eng, d, graphs=graphs)
    net = _net(eng, 9, 16, 1, 4)
    with pytest.raises(az_amd.AzError):
        net.set_precision(az_amd.AZ_PREC_BF16)
    net.close()
    eng.close()


def _scale_heads(desc, blob, factors):
    """Trained-scale outputs: head FC weights scaled (|logit| ~5-10, value away from 0)."""
    import randwire_oracle as RW
    blob = blob.copy()
    off = 0
    for name, shape, _, _ in RW.param_shapes(desc, RW.load_graphs()):
        n = int(np.prod(shape))
        if name in factors:
            blob[off:off + n] *= np.float32(factors[name])
        off += n
    return blob


@pytest.mark.gpu
@pytest.mark.parametrize("nb,B", [(20, 2), (2, 24)])
def test_gpu_randwire_bf16x3_matches_oracle(nb, B):
    """AZ_PREC_BF16X3: node convs on conv3x3_v4 with fp32-faithful split bf16 operands (three MFMAs
    per product), fp32 routers / SE / residual stream -- the fast parity mode, held to the same
    1e-4 tolerance as the f32 path, batch-position independent bitwise."""
    import az_amd
    import randwire_oracle as RW
    eng = az_amd.Engine(0)
    net = _net(eng, 15, 128, nb, BF16X3_CAP)
    net.set_precision(az_amd.AZ_PREC_BF16X3)
    net.init_random(500 + nb)
    blob = net.get_weights()
    planes = (np.random.default_rng(nb + 1).random((B, 11, 15, 15)) < 0.3).astype(np.float32)
    lo, v = net.forward(planes)
    rl, rv = RW.forward(net.desc, RW.load_graphs(), blob, planes)
    scale = max(1.0, float(np.abs(rl).max()))
    dl, dv = float(np.abs(lo - rl).max()), float(np.abs(v - rv).max())
    print(f"bf16x3 rand-wire 128ch {nb} blocks B={B}: |logit| max {np.abs(rl).max():.3g}, max|dlogit| {dl:.3g}, "
          f"max|dvalue| {dv:.3g}")
    assert dl <= 1e-4 * scale and dv <= 1e-4
    lo2, _ = net.forward(planes[[B - 1, 0]])
    assert np.array_equal(lo2.view(np.uint32), lo[[B - 1, 0]].view(np.uint32))
    net.close()
    eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("prec", ["f32", "bf16x3", "fp16"])
def test_gpu_randwire_trained_scale(prec):
    """Logits of order 5-10 (head FC weights scaled): the fp32 path stays within 1e-4 relative to
    the logit scale; the fp16 throughput mode's error is reported and bounded."""
    import az_amd
    import randwire_oracle as RW
    eng = az_amd.Engine(0)
    B = 8
    net = _net(eng, 15, 128, 3, BF16X3_CAP if prec == "bf16x3" else B)
    if prec != "f32":
        net.set_precision(az_amd.AZ_PREC_FP16 if prec == "fp16" else az_amd.AZ_PREC_BF16X3)
    net.init_random(77)
    blob = _scale_heads(net.desc, net.get_weights(), {"policy_fc.weight": 100.0, "value_fc1.weight": 8.0})
    net.load_weights(blob)
    planes = (np.random.default_rng(77).random((B, 11, 15, 15)) < 0.3).astype(np.float32)
    lo, v = net.forward(planes)
    rl, rv = RW.forward(net.desc, RW.load_graphs(), blob, planes)
    scale = float(np.abs(rl).max())
    dl, dv = float(np.abs(lo - rl).max()), float(np.abs(v - rv).max())
    print(f"trained-scale rand-wire {prec}: |logit| max {scale:.3g}, |value| max {np.abs(rv).max():.3g}, "
          f"max|dlogit| {dl:.3g}, max|dvalue| {dv:.3g}")
    assert scale > 3.0
    if prec != "fp16":
        assert dl <= 1e-4 * scale and dv <= 1e-4
    else:
        assert dl <= 1e-2 * scale and dv <= 1e-2
    net.close()
    eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("nb,B", [(2, 16), (20, 3)])
def test_gpu_randwire_fp16_error(nb, B):
    """AZ_PREC_FP16 rand-wire (node convs on conv3x3_v4, routers on gemm_h16_relu: fp16 operands,
    fp32 accumulation; SE and the residual stream fp32): a throughput mode.  Its error against the
    fp32 reference arithmetic is measured and bounded here; the parity precision is AZ_PREC_F32."""
    import az_amd
    import randwire_oracle as RW
    eng = az_amd.Engine(0)
    net = _net(eng, 15, 128, nb, B)
    net.set_precision(az_amd.AZ_PREC_FP16)
    net.init_random(300 + nb)
    blob = net.get_weights()
    planes = (np.random.default_rng(nb).random((B, 11, 15, 15)) < 0.3).astype(np.float32)
    lo, v = net.forward(planes)
    rl, rv = RW.forward(net.desc, RW.load_graphs(), blob, planes)
    dl, dv = float(np.abs(lo - rl).max()), float(np.abs(v - rv).max())
    print(f"fp16 rand-wire 128ch {nb} blocks B={B}: |logit| max {np.abs(rl).max():.3g}, max|dlogit| {dl:.3g}, "
          f"max|dvalue| {dv:.3g}")
    assert dl <= 1e-2 * max(1.0, float(np.abs(rl).max())) and dv <= 1e-2
    lo2, v2 = net.forward(planes[[B - 1, 0]])
    assert np.array_equal(lo2.view(np.uint32), lo[[B - 1, 0]].view(np.uint32))
    net.close()
    eng.close()


def _custom_graph(n, seed):
    """A Python-DDWRandWireResNet-like wiring (networkx DiGraph semantics: no duplicate edges,
    nodes in edge-insertion order, predecessors in insertion order): edges low -> high id."""
    rng = np.random.default_rng(seed)
    edges = []
    for v in range(1, n):
        for u in rng.choice(v, size=min(v, int(rng.integers(1, 4))), replace=False):
            edges.append((int(u), v))
    rng.shuffle(edges)
    order, preds = [], {v: [] for v in range(n)}
    for u, v in edges:
        for w in (u, v):
            if w not in order:
                order.append(w)
        preds[v].append(u)
    for v in range(n):
        if v not in order:
            order.append(v)
    succ = {v: [] for v in range(n)}
    for u, v in edges:
        succ[u].append(v)
    inputs = [v for v in order if not preds[v]]
    outputs = [v for v in order if not succ[v]]
    indeg = {v: len(preds[v]) for v in range(n)}
    topo = list(inputs)
    for u in topo:
        for w in succ[u]:
            indeg[w] -= 1
            if indeg[w] == 0:
                topo.append(w)
    return {"nodes": order, "preds": preds, "input_nodes": inputs, "output_nodes": outputs, "topo": topo}


@pytest.mark.gpu
def test_gpu_randwire_explicit_graphs():
    """az_net_create_randwire_graphs: the reference wiring passed explicitly reproduces
    az_net_create_randwire bit for bit; a networkx-style custom wiring (12 and 20 nodes, several
    sinks) matches the oracle; a cyclic wiring is refused."""
    import az_amd
    import randwire_oracle as RW
    eng = az_amd.Engine(0)
    B = 5
    planes = (np.random.default_rng(9).random((B, 11, 9, 9)) < 0.3).astype(np.float32)
    ref = _net(eng, 9, 32, 2, B)
    ref.init_random(21)
    lo0, v0 = ref.forward(planes)
    exp = az_amd.HipNeuralNetwork(eng, az_amd.randwire_net_desc(9, 32, 2, 11, B), graphs=RW.load_graphs())
    assert exp.num_params == ref.num_params
    exp.load_weights(ref.get_weights())
    lo1, v1 = exp.forward(planes)
    assert np.array_equal(lo0.view(np.uint32), lo1.view(np.uint32)) and np.array_equal(v0.view(np.uint32), v1.view(np.uint32))
    graphs = [_custom_graph(12, 1), _custom_graph(20, 2)]
    assert all(len(g["output_nodes"]) > 1 for g in graphs)
    d = az_amd.randwire_net_desc(9, 32, 2, 11, B)
    net = az_amd.HipNeuralNetwork(eng, d, graphs=graphs)
    blob = RW.init_blob(d, graphs, 4)
    net.load_weights(blob)
    lo, v = net.forward(planes)
    rl, rv = RW.forward(d, graphs, blob, planes)
    assert np.abs(lo - rl).max() <= 1e-4 and np.abs(v - rv).max() <= 1e-4
    bad = [dict(graphs[0], preds={**graphs[0]["preds"], 0: [graphs[0]["topo"][-1]]}), graphs[1]]
    with pytest.raises(az_amd.AzError):
        az_amd.HipNeuralNetwork(eng, d, graphs=bad)
    for x in (ref, exp, net):
        x.close()
    eng.close()
