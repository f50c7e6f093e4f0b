"""az_amd -- host-side Python mirror of the reference's self-play plugin surface,
over the C-ABI of libaz_hip.so (include/az_engine.h).

Reference surfaces mirrored (paths relative to the reference root):
  HipNeuralNetwork  alphazero::nn::NeuralNetwork  (include/alphazero/nn/neural_network.h:20-132):
                    predict(planes) / predictBatch(planes) with TorchNeuralNetwork::predictBatch
                    semantics (softmax over A, value [B]) (src/nn/torch_neural_network.cpp:224-363)
  ParallelMCTS      alphazero::mcts::ParallelMCTS (include/alphazero/mcts/parallel_mcts.h:131-201),
                    one tree per game, G games per device handle: search(), selectAction(),
                    getActionProbabilities(), getRootValue(), updateWithMove(), addDirichletNoise()
  SelfPlayManager   alphazero::selfplay::SelfPlayManager (src/selfplay/self_play_manager.cpp:47-240):
                    generateGames() with the playSingleGame move loop and temperature schedule.
  Dataset           alphazero::selfplay::Dataset (src/selfplay/dataset.cpp): extractExamples with the
                    8-fold augmentation on device, getBatch, shuffle, getRandomSubset, save/load.
"""
import ctypes
from dataclasses import dataclass, field

import numpy as np

from ._lib import (AZ_EVAL_CALLBACK, AZ_EVAL_HASH, AZ_EVAL_NET, AZ_EVAL_RANDOM, AZ_EVAL_UNIFORM, EVAL_FN, AZ_PREC_BF16, AZ_PREC_BF16X3, AZ_PREC_F16X3, AZ_PREC_F32, AZ_PREC_FP16, AzError,
                   GAME_SINK, PROGRESS_FN, MoveRec as _lib_MoveRec, NetDesc, SearchCfg, SelfPlayCfg, check, lib)

__all__ = ["Engine", "HipNeuralNetwork", "ParallelMCTS", "SelfPlayManager", "GameRecord", "MoveData", "AzError",
           "Dataset", "TrainingExample", "GAME_GOMOKU", "GAME_GO",
           "AZ_PREC_F32", "AZ_PREC_BF16X3", "AZ_PREC_F16X3", "AZ_PREC_BF16", "AZ_PREC_FP16", "AZ_EVAL_NET", "AZ_EVAL_HASH", "AZ_EVAL_RANDOM", "AZ_EVAL_UNIFORM", "AZ_EVAL_CALLBACK",
           "gomoku_net_desc"]

_f = ctypes.POINTER(ctypes.c_float)
_i = ctypes.POINTER(ctypes.c_int)


def _fp(a):
    return a.ctypes.data_as(_f)


def _ip(a):
    return a.ctypes.data_as(_i)


class Engine:
    """One HIP device (az_engine_create).  Raises if no GPU is present."""

    def __init__(self, device=0):
        h = ctypes.c_void_p()
        check(lib().az_engine_create(device, ctypes.byref(h)))
        self.h = h

    @property
    def device_name(self):
        buf = ctypes.create_string_buffer(256)
        check(lib().az_engine_device_name(self.h, buf, 256))
        return buf.value.decode()

    def close(self):
        if self.h:
            lib().az_engine_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def gomoku_net_desc(board_size=15, channels=256, blocks=20, precision=AZ_PREC_F32, max_batch=256, residual=1,
                    conv_bias=0, in_planes=11, head_channels=32, pool=8, fc_hidden=256):
    """Residual policy/value net of BASELINE.json (C2: 6x64, C3: 20x256) for Gomoku."""
    return NetDesc(board_size, in_planes, channels, blocks, board_size * board_size, head_channels, pool, fc_hidden,
                   residual, conv_bias, precision, max_batch)


def randwire_net_desc(board_size=15, channels=128, blocks=20, in_planes=11, max_batch=256, action_size=None):
    """DDWRandWireResNet(in_planes, action_size, channels, blocks) of src/nn/ddw_randwire_resnet.cpp:387-468
    (the reference's defaults: 128 channels, 20 blocks; heads 32 channels, 8x8 pool, 256 hidden)."""
    return NetDesc(board_size, in_planes, channels, blocks, action_size or board_size * board_size, 32,
                   min(8, board_size), 256, 0, 0, AZ_PREC_F32, max_batch)


def createDDWRandWireResNet(engine, input_channels, output_size, channels=128, num_blocks=20, board_size=15,
                            max_batch=256):
    """TorchNeuralNetwork::createDDWRandWireResNet (torch_neural_network.cpp:799-814) on the device engine."""
    d = randwire_net_desc(board_size, channels, num_blocks, input_channels, max_batch, output_size)
    return HipNeuralNetwork(engine, d, randwire=True)


def randwire_graph(block):
    """Host-side wiring of rand-wire block `block` (az_randwire_graph): dict like the reference dump."""
    order, topo, ins, outs = ((ctypes.c_int * 32)() for _ in range(4))
    nin, nout = ctypes.c_int(), ctypes.c_int()
    off = (ctypes.c_int * 33)()
    preds = (ctypes.c_int * 256)()
    check(lib().az_randwire_graph(block, order, topo, ins, ctypes.byref(nin), outs, ctypes.byref(nout), off, preds, 256))
    return {"nodes": list(order), "topo": list(topo), "input_nodes": list(ins)[:nin.value],
            "output_nodes": list(outs)[:nout.value], "preds": {v: list(preds[off[v]:off[v + 1]]) for v in range(32)}}


class HipNeuralNetwork:
    """NeuralNetwork plugin on the MI355X ConvNet kernels."""

    def __init__(self, engine, desc, randwire=False, graphs=None):
        """randwire: the DDW-RandWire net with the reference C++ wiring; graphs: explicit wiring per
        block (dicts with "nodes" (registration order), "preds" {node: [...]}, "output_nodes")."""
        self.engine = engine
        self.desc = desc
        h = ctypes.c_void_p()
        if graphs is not None:
            flat = []
            for g in graphs[:desc.blocks]:
                n = len(g["nodes"])
                flat += [n] + list(g["nodes"])
                for v in range(n):
                    p = list(g["preds"][v])
                    flat += [len(p)] + p
                flat += [len(g["output_nodes"])] + list(g["output_nodes"])
            arr = (ctypes.c_int * max(1, len(flat)))(*flat)
            check(lib().az_net_create_randwire_graphs(engine.h, ctypes.byref(desc), arr, len(flat), ctypes.byref(h)))
        else:
            create = lib().az_net_create_randwire if randwire else lib().az_net_create
            check(create(engine.h, ctypes.byref(desc), ctypes.byref(h)))
        self.h = h
        n = ctypes.c_size_t()
        check(lib().az_net_num_params(self.h, ctypes.byref(n)))
        self.num_params = n.value

    def load_weights(self, blob):
        blob = np.ascontiguousarray(blob, dtype=np.float32).reshape(-1)
        check(lib().az_net_load_weights(self.h, _fp(blob), blob.size))

    def init_random(self, seed):
        check(lib().az_net_init_random(self.h, seed))

    def get_weights(self):
        """The loaded weights as the canonical fp32 blob (az_net_get_weights)."""
        blob = np.empty(self.num_params, np.float32)
        check(lib().az_net_get_weights(self.h, _fp(blob), blob.size))
        return blob

    def set_precision(self, precision):
        check(lib().az_net_set_precision(self.h, precision))
        self.desc.precision = precision

    def forward(self, planes):
        """planes [B, C_in, H, W] fp32 -> (logits [B, A], value [B])."""
        x = np.ascontiguousarray(planes, dtype=np.float32)
        B = x.shape[0]
        A = self.desc.action_size
        lo = np.zeros((B, A), np.float32)
        v = np.zeros(B, np.float32)
        check(lib().az_net_forward(self.h, _fp(x), B, _fp(lo), _fp(v)))
        return lo, v

    def predictBatch(self, planes):
        """TorchNeuralNetwork::predictBatch semantics: (softmax policy [B, A], value [B])."""
        x = np.ascontiguousarray(planes, dtype=np.float32)
        B = x.shape[0]
        A = self.desc.action_size
        p = np.zeros((B, A), np.float32)
        v = np.zeros(B, np.float32)
        check(lib().az_net_predict_batch(self.h, _fp(x), B, _fp(p), _fp(v)))
        return p, v

    def predict(self, planes):
        p, v = self.predictBatch(np.asarray(planes, np.float32)[None])
        return p[0], float(v[0])

    def profile(self, enable=True):
        check(lib().az_net_profile(self.h, int(enable)))

    def profile_read(self):
        """(trunk milliseconds, trunk conv launches, forwards) since profile(True)."""
        ms = ctypes.c_double()
        la = ctypes.c_int64()
        fw = ctypes.c_int64()
        check(lib().az_net_profile_read(self.h, ctypes.byref(ms), ctypes.byref(la), ctypes.byref(fw)))
        return ms.value, la.value, fw.value

    def trunk_kernel(self):
        """Name of the HIP kernel the 3x3 trunk convs dispatch at this net's max_batch."""
        buf = ctypes.create_string_buffer(128)
        check(lib().az_net_trunk_kernel(self.h, buf, 128))
        return buf.value.decode()

    def getBatchSize(self):
        return self.desc.max_batch

    def isGpuAvailable(self):
        return True

    def close(self):
        if self.h:
            lib().az_net_destroy(self.h)
            self.h = None


AZ_GAME_GOMOKU, AZ_GAME_GO, AZ_ACTION_NONE = 0, 1, -2


class ParallelMCTS:
    """G independent ParallelMCTS trees (Mode S semantics, setDeterministicMode) on one device."""

    def __init__(self, engine, n_games=1, board_size=15, num_simulations=800, c_puct=1.5, fpu_reduction=0.0,
                 virtual_loss=3, evaluator=AZ_EVAL_HASH, net=None, eval_seed=7, zobrist_seed=12345, noise_seed=42,
                 noise_seed_stride=0, use_dirichlet_each_search=False, dirichlet_alpha=0.03, dirichlet_eps=0.25,
                 tt_log2=20, node_capacity=0, prior_ring=0, game=0, callback=None):
        """game: AZ_GAME_GOMOKU (0) or AZ_GAME_GO (1) -- GoState(bs 9/13/19, komi 7.5, Chinese rules,
        superko); Go actions are -1 (pass) .. bs*bs-1 and finished games report AZ_ACTION_NONE.
        evaluator=AZ_EVAL_CALLBACK: callback(games [n], moves: per leaf the moves from the empty board,
        planes [n][C][bs][bs]) -> (policy [n][NA] as NeuralNetwork::predict returns it, value [n])."""
        self.G = n_games
        self.bs = board_size
        self.game = game
        self.A = board_size * board_size + (1 if game == AZ_GAME_GO else 0)     # action space
        self.none = AZ_ACTION_NONE if game == AZ_GAME_GO else -1
        cfg = SearchCfg(n_games, board_size, num_simulations, c_puct, fpu_reduction, virtual_loss, evaluator,
                        eval_seed, zobrist_seed, noise_seed, noise_seed_stride, int(use_dirichlet_each_search),
                        dirichlet_alpha, dirichlet_eps, tt_log2, node_capacity, prior_ring, game)
        self.cfg = cfg
        h = ctypes.c_void_p()
        check(lib().az_search_create(engine.h, net.h if net is not None else None, ctypes.byref(cfg), ctypes.byref(h)))
        self.h = h
        self.engine, self.net = engine, net
        self._cb = None
        if evaluator == AZ_EVAL_CALLBACK:
            if callback is None:
                raise ValueError("AZ_EVAL_CALLBACK needs a callback")
            NA = self.A

            def _eval(_user, n, games, plen, moves, max_path, planes, n_planes, pol, val):
                try:
                    g = np.ctypeslib.as_array(games, shape=(n,)).copy()
                    ln = np.ctypeslib.as_array(plen, shape=(n,))
                    mv = np.ctypeslib.as_array(moves, shape=(n, max_path))
                    x = np.ctypeslib.as_array(planes, shape=(n, n_planes, board_size, board_size)).copy()
                    p, v = callback(g, [mv[i, :ln[i]].tolist() for i in range(n)], x)
                    p = np.ascontiguousarray(p, np.float32).reshape(n, NA)
                    v = np.ascontiguousarray(v, np.float32).reshape(n)
                    ctypes.memmove(pol, p.ctypes.data, p.nbytes)
                    ctypes.memmove(val, v.ctypes.data, v.nbytes)
                    return 0
                except Exception as e:  # surfaced as AZ_ERR_STATE
                    print("az_amd evaluator failed:", repr(e))
                    return 1

            self._cb = EVAL_FN(_eval)
            check(lib().az_search_set_evaluator(self.h, self._cb, None))

    def newGames(self, games=None):
        games = np.arange(self.G, dtype=np.int32) if games is None else np.asarray(games, np.int32)
        check(lib().az_search_new_games(self.h, _ip(games), games.size))

    def addDirichletNoise(self, alpha=0.03, epsilon=0.25, mask=None):
        if mask is None:
            check(lib().az_search_add_noise(self.h, alpha, epsilon))
        else:
            m = np.ascontiguousarray(mask, dtype=np.uint8)
            check(lib().az_search_add_noise_masked(self.h, alpha, epsilon,
                                                   m.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))))

    def search(self):
        check(lib().az_search_run(self.h))

    def runSingleSimulation(self, n=1):
        """ParallelMCTS::runSingleSimulation (parallel_mcts.cpp:276-380), n times, every game."""
        check(lib().az_search_simulate(self.h, int(n)))

    def runBatchedSearch(self):
        """ParallelMCTS::runBatchedSearch (parallel_mcts.cpp:1531-1590): numSimulations single simulations."""
        check(lib().az_search_simulate(self.h, self.cfg.num_simulations))

    def releaseMemory(self, visitThreshold=10):
        """ParallelMCTS::releaseMemory (parallel_mcts.cpp:1481-1496): nodes pruned per game."""
        out = np.zeros(self.G, np.int64)
        check(lib().az_search_release(self.h, int(visitThreshold), out.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))))
        return out

    def selectActionFor(self, game, isTraining=False, temperature=1.0, legal=(), useBatchInference=True):
        """ParallelMCTS::selectAction of one game (parallel_mcts.cpp:987-1047); with useBatchInference
        off it draws on the game's rng_ (libstdc++ discrete / uniform_int distributions).  legal: the
        root state's getLegalMoves(), used when the root has no children."""
        lg = np.ascontiguousarray(legal, np.int32)
        a = ctypes.c_int()
        check(lib().az_search_select_action(self.h, int(game), int(bool(isTraining)), float(temperature),
                                            int(bool(useBatchInference)), _ip(lg), int(lg.size), ctypes.byref(a)))
        return a.value

    def select(self, is_training=True, temperature=1.0):
        """(actions [G], root values [G], probs [G][A] child order, child actions [G][A], n_children [G])."""
        G, A = self.G, self.A
        act = np.zeros(G, np.int32)
        val = np.zeros(G, np.float32)
        probs = np.zeros((G, A), np.float32)
        cact = np.zeros((G, A), np.int32)
        nch = np.zeros(G, np.int32)
        check(lib().az_search_select(self.h, int(is_training), temperature, _ip(act), _fp(val), _fp(probs), _ip(cact),
                                     _ip(nch)))
        return act, val, probs, cact, nch

    def selectAction(self, isTraining=False, temperature=1.0):
        return self.select(isTraining, temperature)[0]

    def getActionProbabilities(self, temperature=1.0):
        _, _, probs, _, nch = self.select(True, temperature)
        return [probs[g, :nch[g]].copy() for g in range(self.G)]

    def getRootValue(self):
        return self.select(True, 1.0)[1]

    def updateWithMove(self, actions):
        a = np.ascontiguousarray(actions, dtype=np.int32).reshape(self.G)
        term = np.zeros(self.G, np.int32)
        res = np.zeros(self.G, np.int32)
        check(lib().az_search_apply(self.h, _ip(a), _ip(term), _ip(res)))
        return term, res

    def rootChildren(self, game):
        A = self.A
        act = np.zeros(A, np.int32)
        N = np.zeros(A, np.int32)
        VL = np.zeros(A, np.int32)
        W = np.zeros(A, np.float32)
        Pp = np.zeros(A, np.float32)
        n = ctypes.c_int()
        check(lib().az_search_root_children(self.h, game, _ip(act), _ip(N), _ip(VL), _fp(W), _fp(Pp), ctypes.byref(n)))
        k = n.value
        return act[:k], N[:k], VL[:k], W[:k], Pp[:k]

    def rootNode(self, game):
        N = ctypes.c_int()
        VL = ctypes.c_int()
        W = ctypes.c_float()
        check(lib().az_search_root_node(self.h, game, ctypes.byref(N), ctypes.byref(VL), ctypes.byref(W)))
        return N.value, VL.value, W.value

    def counters(self, game):
        out = (ctypes.c_int64 * 5)()
        check(lib().az_search_counters(self.h, game, out))
        return dict(zip(("evals", "tt_lookups", "tt_hits", "sims", "nodes"), list(out)))

    def enableEvalLog(self, game, capacity):
        check(lib().az_search_enable_eval_log(self.h, game, capacity))

    def readEvalLog(self, capacity):
        A = self.A
        pol = np.zeros((capacity, A), np.float32)
        val = np.zeros(capacity, np.float32)
        planes = np.zeros((capacity, 8 if self.game == AZ_GAME_GO else 11, self.bs, self.bs), np.float32)
        n = ctypes.c_int()
        check(lib().az_search_read_eval_log(self.h, _fp(pol), _fp(val), _fp(planes), ctypes.byref(n)))
        k = n.value
        return pol[:k], val[:k], planes[:k]

    def profile(self, enable=True):
        """Start (reset) / stop tree-kernel timing and byte counting (az_search_profile)."""
        check(lib().az_search_profile(self.h, int(enable)))

    def profile_read(self):
        """dict(select_ms, expand_ms, sim_steps, select_bytes, expand_bytes, fused_ms, fused_launches) since
        profile(True): the split kernels of the sampled steps, the fused k_expand_select of the others."""
        a, b = ctypes.c_double(), ctypes.c_double()
        n, sb, eb = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        check(lib().az_search_profile_read(self.h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(n), ctypes.byref(sb),
                                           ctypes.byref(eb)))
        f, fl = ctypes.c_double(), ctypes.c_int64()
        check(lib().az_search_profile_read_fused(self.h, ctypes.byref(f), ctypes.byref(fl)))
        return {"select_ms": a.value, "expand_ms": b.value, "sim_steps": n.value, "select_bytes": sb.value,
                "expand_bytes": eb.value, "fused_ms": f.value, "fused_launches": fl.value}

    def tree_evictions(self):
        """Diagnostic: TreeDev slot evictions so far (each one a stream synchronisation)."""
        f = lib().az_diag_tree_evictions
        f.restype, f.argtypes = ctypes.c_int64, [ctypes.c_void_p]
        return int(f(self.h))

    def selfplayStep(self, temp_drop_move=30, t_init=1.0, t_final=0.0, restart_finished=True):
        cfg = SelfPlayCfg(temp_drop_move, t_init, t_final, int(restart_finished))
        moves = ctypes.c_int64(0)
        evals = ctypes.c_int64(0)
        check(lib().az_selfplay_step(self.h, ctypes.byref(cfg), ctypes.byref(moves), ctypes.byref(evals)))
        return moves.value, evals.value

    def stepMoves(self, materialize=True):
        """MoveData of the last selfplayStep: [(slot, MoveData)] for every game that moved.
        materialize=False returns the engine's own records as they are (the C++-assembled
        az_move_rec array, as a numpy structured view valid until the next step, and the slots)
        without building Python objects."""
        mv = ctypes.POINTER(_lib_MoveRec)()
        sl = ctypes.POINTER(ctypes.c_int)()
        n = ctypes.c_int()
        check(lib().az_selfplay_step_moves(self.h, ctypes.byref(mv), ctypes.byref(sl), ctypes.byref(n)))
        if not materialize:
            if n.value == 0:
                return None, None
            import numpy as np
            R = _lib_MoveRec
            dt = np.dtype({"names": ["action", "value", "n_children", "policy", "child_actions", "thinking_time_ms"],
                           "formats": ["<i4", "<f4", "<i4", "<u8", "<u8", "<i8"],
                           "offsets": [R.action.offset, R.value.offset, R.n_children.offset, R.policy.offset,
                                       R.child_actions.offset, R.thinking_time_ms.offset],
                           "itemsize": ctypes.sizeof(R)})
            raw = (ctypes.c_char * (n.value * ctypes.sizeof(R))).from_address(ctypes.addressof(mv.contents))
            return np.frombuffer(raw, dtype=dt), np.ctypeslib.as_array(sl, shape=(n.value,))
        out = []
        for i in range(n.value):
            r = mv[i]
            k = r.n_children
            # pointer slices copy the k entries in one C-level call (per-element indexing is ~8 ms/move at C2)
            out.append((int(sl[i]), MoveData(int(r.action), r.policy[:k], float(r.value),
                                             int(r.thinking_time_ms), r.child_actions[:k])))
        return out

    def close(self):
        if self.h:
            lib().az_search_destroy(self.h)
            self.h = None


@dataclass
class MoveData:
    """include/alphazero/selfplay/game_record.h:21-33 (policy in CHILD order, not action-indexed;
    child_actions holds the matching actions, an extension the reference does not record)."""
    action: int
    policy: list
    value: float
    thinking_time_ms: int = 0
    child_actions: list = field(default_factory=list)


@dataclass
class GameRecord:
    board_size: int
    moves: list = field(default_factory=list)
    result: int = 0
    game_id: int = -1


class SelfPlayManager:
    """SelfPlayManager::generateGames over G device-resident games (playSingleGame loop,
    self_play_manager.cpp:151-234): initial noise, search, T = initial until
    temperatureDropMove then final, selectAction(true, T), record, makeMove +
    updateWithMove, noise after every even ply."""

    def __init__(self, engine, net=None, numGames=1, numSimulations=800, board_size=15, evaluator=None, **mcts_kw):
        ev = evaluator if evaluator is not None else (AZ_EVAL_NET if net is not None else AZ_EVAL_HASH)
        self.mcts = ParallelMCTS(engine, n_games=numGames, board_size=board_size, num_simulations=numSimulations,
                                 evaluator=ev, net=net, **mcts_kw)
        self.numGames = numGames
        self.dirichletAlpha, self.dirichletEpsilon = 0.03, 0.25
        self.initialTemperature, self.temperatureDropMove, self.finalTemperature = 1.0, 30, 0.0
        self.progressCallback = None

    def setExplorationParams(self, dirichletAlpha, dirichletEpsilon, initialTemperature, temperatureDropMove,
                             finalTemperature):
        self.dirichletAlpha, self.dirichletEpsilon = dirichletAlpha, dirichletEpsilon
        self.initialTemperature, self.temperatureDropMove = initialTemperature, temperatureDropMove
        self.finalTemperature = finalTemperature

    def setProgressCallback(self, cb):
        self.progressCallback = cb

    def getTemperature(self, moveNum):
        return self.finalTemperature if moveNum >= self.temperatureDropMove else self.initialTemperature

    def generateGames(self, totalGames=None, max_moves=0, abort=None):
        """SelfPlayManager::generateGames through the engine's device driver (az_selfplay_run):
        totalGames games (default numGames) on the handle's slots; returns GameRecords by game id."""
        total = self.numGames if totalGames is None else int(totalGames)
        recs = [None] * total

        def sink(_user, gid, bs, n, moves, result):
            r = GameRecord(bs, result=int(result), game_id=int(gid))
            for i in range(n):
                mv = moves[i]
                k = mv.n_children
                r.moves.append(MoveData(int(mv.action), [float(mv.policy[j]) for j in range(k)], float(mv.value),
                                        int(mv.thinking_time_ms), [int(mv.child_actions[j]) for j in range(k)]))
            recs[gid] = r

        def progress(_user, gid, move, tg, tm):
            if self.progressCallback:
                self.progressCallback(int(gid), int(move), int(tg), int(tm))

        cfg = SelfPlayCfg(self.temperatureDropMove, self.initialTemperature, self.finalTemperature, 0)
        flag = ctypes.c_int(0) if abort is None else abort
        cb_sink, cb_prog = GAME_SINK(sink), PROGRESS_FN(progress)
        check(lib().az_selfplay_run(self.mcts.h, ctypes.byref(cfg), total, int(max_moves), cb_sink, cb_prog, None,
                                    ctypes.byref(flag)))
        return recs

    def generateGamesStepwise(self, max_moves=1 << 30, on_move=None):
        """The playSingleGame loop driven from the host through the per-call C-ABI (search /
        select / apply / noise), all numGames games in lock step -- the cross-check for
        generateGames."""
        m = self.mcts
        G = self.numGames
        m.newGames()
        m.addDirichletNoise(self.dirichletAlpha, self.dirichletEpsilon)
        records = [GameRecord(m.bs) for _ in range(G)]
        live = np.ones(G, bool)
        move = 0
        while live.any() and move < max_moves:
            m.search()
            T = self.getTemperature(move)
            act, val, probs, cact, nch = m.select(True, T)
            if on_move is not None:
                on_move(move, m)
            for g in range(G):
                if live[g]:
                    records[g].moves.append(MoveData(int(act[g]), probs[g, :nch[g]].tolist(), float(val[g]), 0,
                                                     cact[g, :nch[g]].tolist()))
                    if self.progressCallback:
                        self.progressCallback(g, move, G, move * G)
            act = np.where(live, act, -1).astype(np.int32)
            term, res = m.updateWithMove(act)
            for g in range(G):
                if live[g] and term[g]:
                    records[g].result = int(res[g])
                    live[g] = False
            if move % 2 == 0:
                m.addDirichletNoise(self.dirichletAlpha, self.dirichletEpsilon)
            move += 1
        return records


# ---------------------------------------------------------------------------- Dataset (row f3)
GAME_GOMOKU, GAME_GO = 0, 1
_i64 = ctypes.POINTER(ctypes.c_int64)


def _json_number(x):
    """nlohmann::json's text for a float widened to double: shortest round-trip digits, NaN as null."""
    v = float(x)
    if v != v or v in (float("inf"), float("-inf")):
        return "null"
    return repr(v)


@dataclass
class TrainingExample:
    """selfplay::TrainingExample (include/alphazero/selfplay/dataset.h:21-28): state [planes][bs][bs],
    policy (the record's child-order visit distribution), value."""
    state: np.ndarray
    policy: np.ndarray
    value: float

    def toJson(self):
        # TrainingExample::toJson (src/selfplay/dataset.cpp:16-33): j.dump(), keys sorted
        st = "[" + ",".join("[" + ",".join("[" + ",".join(_json_number(v) for v in row) + "]" for row in pl) + "]"
                            for pl in np.asarray(self.state)) + "]"
        pol = "[" + ",".join(_json_number(v) for v in np.asarray(self.policy)) + "]"
        return '{"policy":' + pol + ',"state":' + st + ',"value":' + _json_number(self.value) + "}"

    @staticmethod
    def fromJson(s):
        import json
        j = json.loads(s) if isinstance(s, str) else s
        nan = float("nan")
        state = np.array([[[nan if v is None else v for v in row] for row in pl] for pl in j["state"]], np.float32)
        policy = np.array([nan if v is None else v for v in j["policy"]], np.float32)
        return TrainingExample(state, policy, float(nan if j["value"] is None else j["value"]))


class Dataset:
    """selfplay::Dataset (include/alphazero/selfplay/dataset.h:33-118, src/selfplay/dataset.cpp) over a
    device-resident example store (az_dataset_*): extractExamples replays every record on the GPU and
    writes each position's examples (original + 7 symmetries) straight into their shuffled slots;
    getBatch / getRandomSubset / shuffle are device gathers.  rng_ is the handle's std::mt19937,
    seeded from std::random_device as the reference does unless `seed` is given."""

    def __init__(self, engine, game_type=GAME_GOMOKU, board_size=15, seed=None):
        h = ctypes.c_void_p()
        check(lib().az_dataset_create(engine.h, int(game_type), int(board_size), ctypes.byref(h)))
        self.h = h
        self.engine = engine
        self.game_type, self.bs = int(game_type), int(board_size)
        if seed is not None:
            check(lib().az_dataset_seed(self.h, int(seed) & 0xFFFFFFFF))
        n, c, b, st = ctypes.c_int64(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check(lib().az_dataset_info(self.h, ctypes.byref(n), ctypes.byref(c), ctypes.byref(b), ctypes.byref(st)))
        self.planes, self.policy_stride = c.value, st.value
        self.gameRecords = []

    def addGameRecord(self, record, useEnhancedFeatures=True):
        if record.board_size != self.bs:
            raise ValueError(f"record board {record.board_size} != dataset board {self.bs}")
        self.gameRecords.append(record)

    def _order(self, n):
        out = np.empty(n, np.int64)
        check(lib().az_dataset_shuffle_order(self.h, int(n), out.ctypes.data_as(_i64)))
        return out

    def extractExamples(self, includeAugmentations=True, shuffle=True):
        """Dataset::extractExamples (dataset.cpp:60-114); shuffle=False keeps the pre-shuffle order
        (record order, per position the original then augmentExample's 7)."""
        recs = self.gameRecords
        n_moves = np.array([len(r.moves) for r in recs], np.int32)
        actions = np.array([m.action for r in recs for m in r.moves], np.int32)
        nch = np.array([len(m.policy) for r in recs for m in r.moves], np.int32)
        pols = [np.asarray(m.policy, np.float32) for r in recs for m in r.moves]
        pol = np.concatenate(pols) if pols else np.zeros(0, np.float32)
        res = np.array([r.result for r in recs], np.int32)
        E = int(n_moves.sum()) * (8 if includeAugmentations else 1)
        order = self._order(E) if shuffle else None
        ne = ctypes.c_int64()
        check(lib().az_dataset_extract(self.h, len(recs), _ip(n_moves), _ip(actions), _ip(nch), _fp(pol), _ip(res),
                                       int(bool(includeAugmentations)),
                                       order.ctypes.data_as(_i64) if order is not None else None, ctypes.byref(ne)))
        return ne.value

    def size(self):
        n = ctypes.c_int64()
        check(lib().az_dataset_info(self.h, ctypes.byref(n), None, None, None))
        return n.value

    def gather(self, idx):
        """Examples idx as arrays: states [n][planes][bs][bs], policy [n][stride], policy_len [n], value [n]."""
        idx = np.ascontiguousarray(idx, np.int64)
        n = len(idx)
        st = np.empty((n, self.planes, self.bs, self.bs), np.float32)
        po = np.empty((n, self.policy_stride), np.float32)
        pl = np.empty(n, np.int32)
        va = np.empty(n, np.float32)
        if n:
            check(lib().az_dataset_gather(self.h, idx.ctypes.data_as(_i64), n, _fp(st), _fp(po), _ip(pl), _fp(va)))
        return st, po, pl, va

    def getBatch(self, batchSize):
        """Dataset::getBatch (dataset.cpp:120-145): std::shuffle of all indices, the first batchSize."""
        n = self.size()
        b = min(int(batchSize), n)
        st, po, pl, va = self.gather(self._order(n)[:b])
        return st, [po[i, :pl[i]].copy() for i in range(b)], va

    def shuffle(self):
        n = self.size()
        if n:
            check(lib().az_dataset_permute(self.h, self._order(n).ctypes.data_as(_i64)))

    def getRandomSubset(self, count):
        n = self.size()
        st, po, pl, va = self.gather(self._order(n)[:min(int(count), n)])
        return [TrainingExample(st[i], po[i, :pl[i]].copy(), float(va[i])) for i in range(len(va))]

    def examples(self):
        st, po, pl, va = self.gather(np.arange(self.size()))
        return [TrainingExample(st[i], po[i, :pl[i]].copy(), float(va[i])) for i in range(len(va))]

    def saveToFile(self, filename):
        """Dataset::saveToFile (dataset.cpp:151-186): {"examples":[...]} as j.dump()."""
        try:
            with open(filename, "w") as f:
                f.write('{"examples":[' + ",".join(e.toJson() for e in self.examples()) + "]}")
            return True
        except Exception:
            return False

    def loadFromFile(self, filename):
        """Dataset::loadFromFile (dataset.cpp:188-227); examples go to the device store."""
        import json
        try:
            with open(filename) as f:
                j = json.load(f)
            exs = [TrainingExample.fromJson(e) for e in j["examples"]]
        except Exception:
            return False
        n = len(exs)
        st = np.zeros((n, self.planes, self.bs, self.bs), np.float32)
        po = np.zeros((n, self.policy_stride), np.float32)
        pl = np.zeros(n, np.int32)
        va = np.zeros(n, np.float32)
        for i, e in enumerate(exs):
            st[i] = e.state
            pl[i] = len(e.policy)
            po[i, :pl[i]] = e.policy
            va[i] = e.value
        check(lib().az_dataset_upload(self.h, n, _fp(st), _fp(po), _ip(pl), _fp(va)))
        return True

    def profile_read(self):
        ms, by = ctypes.c_double(), ctypes.c_double()
        check(lib().az_dataset_profile_read(self.h, ctypes.byref(ms), ctypes.byref(by)))
        return ms.value, by.value

    def close(self):
        if self.h:
            lib().az_dataset_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
