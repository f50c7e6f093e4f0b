/*
 * az_engine.h -- C-ABI of the MI355X-native self-play engine (libaz_hip.so).
 *
 * This is the drop-in boundary for the reference's self-play hot path
 * (src/selfplay + src/mcts + src/nn of cosmosapjw-quantum/alphazero-multi-game).
 * Plain pointers and sizes only; no exceptions cross it.  Every entry point
 * returns 0 on success and a negative az_status otherwise; az_last_error()
 * gives a thread-local message.  The caller owns every host buffer (the engine
 * copies in and out); the engine owns all device memory.  Calls on one handle
 * are serialised internally, so the reference's multi-threaded callers stay legal.
 *
 * Reference interfaces replaced (paths relative to the reference root):
 *   az_net_*      alphazero::nn::NeuralNetwork plugin
 *                 (include/alphazero/nn/neural_network.h:20-132),
 *                 TorchNeuralNetwork::predictBatch (src/nn/torch_neural_network.cpp:224-363)
 *   az_search_*   alphazero::mcts::ParallelMCTS, one tree per game, G games per handle
 *                 (include/alphazero/mcts/parallel_mcts.h:131-201)
 *   az_selfplay_* alphazero::selfplay::SelfPlayManager::generateGames / playSingleGame
 *                 (src/selfplay/self_play_manager.cpp:47-234)
 *   az_dist_*     the per-GPU process sharding of python/scripts/orchestrate_selfplay.py:303-311,
 *                 741-749, with RCCL for the weights and the counters
 */
#ifndef AZ_ENGINE_H
#define AZ_ENGINE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum az_status {
    AZ_OK = 0,
    AZ_ERR_ARG = -1,       /* invalid argument / shape */
    AZ_ERR_HIP = -2,       /* HIP runtime error (device missing, launch failure) */
    AZ_ERR_OOM = -3,       /* device allocation failed */
    AZ_ERR_CAPACITY = -4,  /* node pool / prior ring / batch capacity exceeded */
    AZ_ERR_STATE = -5,     /* call not valid in the current state */
    AZ_ERR_RANGE = -6      /* an AZ_PREC_FP16 / F16X3 activation left the fp16 range (|x| > 65504): the
                              outputs of that forward / search are invalid; use AZ_PREC_BF16X3 */
};

typedef struct az_engine az_engine;
typedef struct az_net az_net;
typedef struct az_search az_search;

/* ---------------------------------------------------------------- engine */
const char* az_last_error(void);
int az_engine_create(int device, az_engine** out);   /* hipSetDevice(device); fails loudly without a GPU */
void az_engine_destroy(az_engine* e);
int az_engine_device_name(az_engine* e, char* buf, int len);

/* ------------------------------------------------------- NeuralNetwork */
/* Residual policy/value ConvNet of SURVEY.md CS5 / §8(a) a27:
 *   input 3x3 conv C_in->F (+BN, ReLU); `blocks` x {3x3 conv, BN, ReLU, 3x3 conv, BN,
 *   (+skip if residual), ReLU}; adaptive avg-pool to pool x pool; policy head
 *   1x1 conv F->head_ch + BN + ReLU + FC -> A logits; value head 1x1 conv F->head_ch +
 *   BN + ReLU + FC -> fc_hidden + ReLU + FC -> 1 + tanh.
 *   residual=1,conv_bias=1 : SimplifiedModel (python/simple_export.py:12-66)
 *   residual=0,conv_bias=0 : exporter fallback (python/scripts/simple_export.py:40-96)  */
enum az_precision {
    AZ_PREC_F32 = 0,    /* fp32 operands, f32-input MFMA (exact f32 products)              */
    AZ_PREC_BF16X3 = 1, /* fp32 split into bf16 hi+lo, 3 bf16 MFMAs per product (~2^-17;
                           the full fp32 range)                                            */
    AZ_PREC_BF16 = 2,   /* plain bf16 operands, fp32 accumulate (throughput only)          */
    AZ_PREC_FP16 = 3,   /* fp16 operands, fp32 accumulate: TorchNeuralNetworkConfig::useFp16
                           (include/alphazero/nn/torch_neural_network.h:29); 15x15, F%64==0   */
    AZ_PREC_F16X3 = 4   /* fp32 split into fp16 hi+lo (weights scaled 2^s per output channel),
                           3 fp16 MFMAs per product (~2^-21: the fp32 oracle's own error level);
                           activations must stay within |x| <= 65504 (else AZ_ERR_RANGE; use
                           AZ_PREC_BF16X3); 8/9/13/15/19 boards with channels % 128 == 0, or
                           the 15x15 64-channel net                                        */
};
typedef struct az_net_desc {
    int board_size;     /* H = W */
    int in_planes;      /* 11 for Gomoku (gomoku_state.cpp:207-258) */
    int channels;       /* F */
    int blocks;
    int action_size;    /* A */
    int head_channels;  /* 32 */
    int pool;           /* 8: adaptive_avg_pool2d target */
    int fc_hidden;      /* 256 */
    int residual;       /* 1: relu(x + block(x)) */
    int conv_bias;      /* 1: convolutions carry a bias */
    int precision;      /* az_precision for the 3x3 trunk */
    int max_batch;      /* largest B passed to az_net_* (device buffers sized for it) */
} az_net_desc;

int az_net_create(az_engine* e, const az_net_desc* desc, az_net** out);
/* DDW-RandWire network: DDWRandWireResNet(in_planes, action_size, channels,
 * blocks) of src/nn/ddw_randwire_resnet.cpp:387-468 (TorchNeuralNetwork::createDDWRandWireResNet,
 * torch_neural_network.cpp:799-814).  Each of `blocks` rand-wire blocks is RandWireBlock(channels,
 * 32 nodes, p = 0.75, seed = block index) (:399): 32 SE residual blocks wired by a rewired
 * Watts-Strogatz graph with routers.  desc: conv_bias 0, pool = min(8, board), precision AZ_PREC_F32
 * (the module's arithmetic; parity mode), or on 15x15 with channels % 64 == 0 AZ_PREC_BF16X3
 * (fp32-faithful split-operand node convs from 128 boards of capacity; parity mode) or AZ_PREC_FP16
 * (fp16-operand node convs and routers; throughput mode: node inputs are rounded to fp16 with no
 * range guard, so a net whose trunk activations exceed 65504 overflows to inf -- keep such nets on
 * AZ_PREC_F32 / AZ_PREC_BF16X3) -- SE and the residual stream stay fp32;
 * the reference's heads are
 * head_channels 32, fc_hidden 256; residual is ignored.  The blob is the
 * reference module's state_dict order (num_batches_tracked dropped); every other az_net_* call and
 * the search take the handle as for az_net_create. */
int az_net_create_randwire(az_engine* e, const az_net_desc* desc, az_net** out);
/* The same net with explicit wiring, e.g. the graphs of a Python DDWRandWireResNet
 * (python/alphazero/models/ddw_randwire.py:56-116, networkx Watts-Strogatz + DiGraph): per block
 * n, order[n] (router / block registration order), for node v = 0..n-1: deg_v, preds[deg_v]
 * (concat order), n_out, outputs[n_out] (output-router concat order); n_ints in total.  Inputs
 * are the in-degree-0 nodes in `order`.  AZ_ERR_ARG on a malformed or cyclic wiring. */
int az_net_create_randwire_graphs(az_engine* e, const az_net_desc* desc, const int* graphs, size_t n_ints,
                                  az_net** out);
/* Host only (no device needed): the wiring of rand-wire block `block` (RandWireBlock::_generate_graph,
 * :248-319, with the duplicate-edge test evaluated as written -- DESIGN.md §5c).  order[32] = nodes()
 * order (router / block registration order), topo[32], inputs / outputs (in-/out-degree 0), the
 * predecessors of node v in preds[pred_off[v] .. pred_off[v+1]) (pred_off[33]; preds_cap entries). */
int az_randwire_graph(int block, int* order, int* topo, int* inputs, int* n_inputs, int* outputs, int* n_outputs,
                      int* pred_off, int* preds, int preds_cap);
void az_net_destroy(az_net* n);
/* Number of floats of the canonical parameter blob (torch state_dict order, BN in
 * eval form: weight, bias, running_mean, running_var per BN). */
int az_net_num_params(az_net* n, size_t* count);
int az_net_load_weights(az_net* n, const float* blob, size_t count);
/* Counter-based deterministic init (SplitMix64), identical to tests' generator. */
int az_net_init_random(az_net* n, uint64_t seed);
/* The loaded weights as the canonical blob (count = az_net_num_params): what rank 0 broadcasts
 * to the other ranks; AZ_ERR_STATE before any load/init. */
int az_net_get_weights(az_net* n, float* blob, size_t count);
int az_net_set_precision(az_net* n, int precision);
/* planes: host fp32 NCHW [B][in_planes][H][W].  logits [B][A] raw, value [B] (tanh). */
int az_net_forward(az_net* n, const float* planes, int B, float* logits, float* value);
/* Profiling: HIP events bracket the 3x3 trunk (2*blocks conv launches) of every
 * simulation-batch forward on the engine stream.  read returns the summed trunk time. */
int az_net_profile(az_net* n, int enable);
int az_net_profile_read(az_net* n, double* trunk_ms, int64_t* trunk_launches, int64_t* forwards);
/* The name of the HIP kernel the 3x3 trunk convs of this net dispatch at its max_batch
 * (measurement label, e.g. "conv3x3_v7<2, 15, SLIM>"; "gemm_f32" for the f32 path). */
int az_net_trunk_kernel(az_net* n, char* name, int len);
/* predictBatch semantics: policy = softmax over A (max-subtracted, sequential fp32 sum,
 * torch_neural_network.cpp:296-316), value [B]. */
int az_net_predict_batch(az_net* n, const float* planes, int B, float* policy, float* value);

/* ---------------------------------------------------------------- search */
enum az_eval_kind {
    AZ_EVAL_NET = 0,    /* the ConvNet above (az_search_create's `net`) */
    AZ_EVAL_HASH = 1,   /* HashEvaluator (oracle/ref_harness.cpp hash_eval), tests */
    AZ_EVAL_RANDOM = 2, /* RandomPolicyNetwork(seed + game) semantics (random_policy_network.cpp) */
    AZ_EVAL_UNIFORM = 3,/* no network: ParallelMCTS::evaluateState fallback (parallel_mcts.cpp:903-916) */
    AZ_EVAL_CALLBACK = 4/* a host evaluator (az_search_set_evaluator): any NeuralNetwork subclass's
                           predict / predictBatch (parallel_mcts.cpp:886-901), once per simulation step */
};
typedef struct az_search_cfg {
    int n_games;          /* G: independent games (trees) on this device */
    int board_size;       /* Gomoku bs (standard rules: no Renju/Omok/pro-long) */
    int num_simulations;  /* MCTSConfig::numSimulations */
    float c_puct;         /* 1.5 */
    float fpu_reduction;  /* 0.0 */
    int virtual_loss;     /* 3 */
    int eval_kind;        /* az_eval_kind */
    uint32_t eval_seed;   /* RandomPolicyNetwork seed (game g uses eval_seed + g) */
    uint32_t zobrist_seed;/* ZobristHash seed (reference patch P2 uses 12345) */
    uint32_t noise_seed;  /* ParallelMCTS rng_ seed; setDeterministicMode => 42 */
    int noise_seed_stride;/* game g uses noise_seed + g*stride (0: every game seeded 42) */
    int use_dirichlet_each_search; /* MCTSConfig::useDirichletNoise */
    float dirichlet_alpha;/* 0.03 */
    float dirichlet_eps;  /* 0.25 */
    int tt_log2;          /* TranspositionTable slots = 2^tt_log2 per game (reference: 20) */
    int node_capacity;    /* per-game node pool (0: auto = sims*A + 4*A) */
    int prior_ring;       /* per-game prior ring floats for TT hits (0: auto) */
    int game;             /* AZ_GAME_GOMOKU (0) or AZ_GAME_GO (1): GoState(bs, komi 7.5, Chinese rules,
                             superko), bs 9/13/19, action space bs*bs + 1, pass = action -1.  For Go,
                             az_search_select reports finished games as AZ_ACTION_NONE and
                             az_search_apply skips them (Gomoku: -1, as before). */
} az_search_cfg;

#define AZ_GAME_GOMOKU 0
#define AZ_GAME_GO 1
#define AZ_ACTION_NONE (-2)   /* Go: no move (finished game); -1 is the pass */

int az_search_create(az_engine* e, az_net* net, const az_search_cfg* cfg, az_search** out);
/* AZ_EVAL_CALLBACK: every simulation step hands the n leaves that need an evaluation to the host,
 * in one call on the calling thread: games[i] (the game slot), the path_len[i] moves that lead
 * from the game's initial (empty) state to leaf i -- the moves committed so far, then the search
 * path -- in moves[i * max_path ...], and the leaf's feature planes [n][n_planes][bs][bs]
 * (getEnhancedTensorRepresentation).  The evaluator fills policy [n][NA] -- as
 * NeuralNetwork::predict returns it (post-softmax; used as is by expandNodeWithPolicy) -- and
 * value [n], and returns 0 (nonzero aborts the search with AZ_ERR_STATE). */
typedef int (*az_eval_fn)(void* user, int n, const int* games, const int* path_len, const int* moves, int max_path,
                          const float* planes, int n_planes, float* policy, float* value);
int az_search_set_evaluator(az_search* s, az_eval_fn fn, void* user);
void az_search_destroy(az_search* s);
/* Start fresh games (empty board, new tree and TT) for the listed game slots. */
int az_search_new_games(az_search* s, const int* games, int n);
/* ParallelMCTS::addDirichletNoise(alpha, eps) for every non-terminal game; expands
 * roots first (expandNode semantics).  Gamma draws: host libstdc++ per game. */
int az_search_add_noise(az_search* s, float alpha, float eps);
/* Like az_search_add_noise but only for games with mask[g] != 0. */
int az_search_add_noise_masked(az_search* s, float alpha, float eps, const uint8_t* mask);
/* ParallelMCTS::search() for every active (non-terminal) game. */
int az_search_run(az_search* s);
/* ParallelMCTS::runSingleSimulation() n times for every active game (parallel_mcts.cpp:276-380):
 * no root-expansion step and no noise, unlike az_search_run; an unexpanded root is the first
 * leaf.  runBatchedSearch (:1531-1590, numThreads 1) is n = numSimulations. */
int az_search_simulate(az_search* s, int n);
/* ParallelMCTS::releaseMemory(visitThreshold) (parallel_mcts.cpp:1481-1496, MCTSNode::pruneTree
 * mcts_node.cpp:451-477) for every game: children with visitCount < threshold are removed with
 * their subtrees, recursively from the root (child order kept; a node that loses every child
 * stays expanded).  pruned[g] (optional, G entries) = nodes removed (getTreeSize of each). */
int az_search_release(az_search* s, int threshold, int64_t* pruned);
/* The same for the games with mask[g] != 0 only (G entries); the other games' trees are untouched:
 * the entry points of a handle that several host objects share (mcts::SearchGroup).  The masked
 * search / simulation park the other games for the call (inactive), release copies their trees
 * whole. */
int az_search_run_masked(az_search* s, const uint8_t* mask);
int az_search_simulate_masked(az_search* s, int n, const uint8_t* mask);
int az_search_release_masked(az_search* s, int threshold, int64_t* pruned, const uint8_t* mask);
/* az_search_new_games with each game's stream id for the evaluator / noise seeds given (default:
 * the slot index): id 0 makes a slot's game the one a single-game handle plays. */
int az_search_new_games_ids(az_search* s, const int* games, const int* seed_ids, int n);
/* ParallelMCTS::selectAction(isTraining, T) of one game (parallel_mcts.cpp:987-1047).
 * batch_inference != 0 (MCTSConfig::useBatchInference, forced by setDeterministicMode and
 * SelfPlayManager): the deterministic rules of az_search_select.  Otherwise draws on the game's
 * rng_ (the std::mt19937 of its Dirichlet draws) with libstdc++: discrete_distribution over
 * getActionProbabilities(T) when training with T > 0, else uniform_int_distribution over the
 * most-visited children when they tie.  `legal` (the root state's getLegalMoves()) is used when
 * the root has no children (after releaseMemory): legal[0], or a uniform draw; -1 if empty. */
int az_search_select_action(az_search* s, int game, int training, float temperature, int batch_inference,
                            const int* legal, int n_legal, int* action);
/* getActionProbabilities(T) + selectAction(isTraining, T) + getRootValue() for every
 * game.  probs: [G][NA] in CHILD order (n_children[g] valid entries), children_actions
 * [G][NA] (NA = action space: bs*bs, Go bs*bs + 1); actions[g] = -1 (Go: AZ_ACTION_NONE)
 * for finished games. */
int az_search_select(az_search* s, int training, float temperature, int* actions, float* root_values,
                     float* probs, int* children_actions, int* n_children);
/* state.makeMove(a) + updateWithMove(a) for every game with actions[g] >= 0;
 * terminal[g] / result[g] (GameResult: 0 ongoing, 1 draw, 2 P1 win, 3 P2 win). */
int az_search_apply(az_search* s, const int* actions, int* terminal, int* result);
/* Root children statistics of one game, child order (raw N, VL, W, P). */
int az_search_root_children(az_search* s, int game, int* actions, int* N, int* VL, float* W, float* P,
                            int* n_children);
/* Root node's own N, VL, W. */
int az_search_root_node(az_search* s, int game, int* N, int* VL, float* W);
/* Update the search parameters of a live handle without touching its trees (the reference's
 * setters / setConfig keep the tree, parallel_mcts.h:172-182, parallel_mcts.cpp:1225-1261):
 * num_simulations (up to the node pool sized at creation, else AZ_ERR_CAPACITY), c_puct,
 * fpu_reduction, virtual_loss, the Dirichlet fields and the noise seeds of later new games.
 * Shape, evaluator and table changes need a new handle (AZ_ERR_ARG). */
int az_search_set_params(az_search* s, const az_search_cfg* cfg);
/* Swap the device net of an AZ_EVAL_NET handle in place, trees kept (ParallelMCTS::
 * setNeuralNetwork, parallel_mcts.cpp:1190-1207, only replaces nn_): same engine, board, planes
 * and action space, max_batch >= n_games, weights loaded; else AZ_ERR_ARG / AZ_ERR_STATE. */
int az_search_set_net(az_search* s, az_net* net);
/* Empty every game's transposition table, trees kept (ParallelMCTS::setTranspositionTable with a
 * new table, parallel_mcts.cpp:1209-1222). */
int az_search_clear_tt(az_search* s);
/* Reseed game's rng_ (ParallelMCTS::setDeterministicMode, parallel_mcts.cpp:1263-1274: 42, or
 * std::random_device): the std::mt19937 of the Dirichlet draws and of az_search_select_action. */
int az_search_seed(az_search* s, int game, uint32_t seed);
/* The full state of game's rng_ (std::mt19937: 624 words + the position, 625 uint32), read and
 * restored so that a host object that rebuilds its handle (a new evaluator or table) keeps
 * drawing from the same generator, as the reference's ParallelMCTS keeps rng_ across
 * setNeuralNetwork / setTranspositionTable (parallel_mcts.h:172-182). */
#define AZ_RNG_STATE_WORDS 625
int az_search_get_rng(az_search* s, int game, uint32_t* state);
int az_search_set_rng(az_search* s, int game, const uint32_t* state);
/* Root node flags of one game: 1 expanded (MCTSNode::isExpanded), 2 terminal, bits 2..3 the
 * GameResult of a terminal root. */
#define AZ_NODE_EXPANDED 1
#define AZ_NODE_TERMINAL 2
int az_search_root_flags(az_search* s, int game, int* flags);
/* Counters per game: [0] evals, [1] tt_lookups, [2] tt_hits, [3] simulations, [4] nodes used. */
int az_search_counters(az_search* s, int game, int64_t* out5);
/* Tree-kernel profiling: enable resets; read returns the summed GPU time of K1 (selection +
 * VL + leaf planes) and K3 (expansion + backup) over the simulation steps since enable (HIP
 * events on the engine stream), the number of such steps, and the algorithmic HBM bytes the
 * kernels moved (child records scanned, path updates, new nodes, planes; counted per game). */
int az_search_profile(az_search* s, int enable);
int az_search_profile_read(az_search* s, double* select_ms, double* expand_ms, int64_t* sim_steps,
                           int64_t* select_bytes, int64_t* expand_bytes);
/* The production tree step: simulation steps other than the sampled ones above run step i's
 * expansion and step i+1's selection as ONE launch (k_expand_select); its summed GPU time over those
 * launches since enable (device clock stamps around one launch in AZ_PROF_EVERY, scaled) and their
 * count.  Measurement only, like az_search_profile_read. */
int az_search_profile_read_fused(az_search* s, double* fused_ms, int64_t* fused_launches);
/* Evaluation log (tests): every evaluation of game `game` appends (policy[A] post-softmax,
 * value) in evaluation order; planes too when planes != 0.  Capacity in evaluations. */
int az_search_enable_eval_log(az_search* s, int game, int capacity);
int az_search_read_eval_log(az_search* s, float* policy, float* value, float* planes, int* count);

/* ------------------------------------------------------------- self-play */
/* One SelfPlayManager::playSingleGame move for every active game: search, temperature
 * schedule (T = ply < temp_drop ? t_init : t_final), selectAction(true, T), record,
 * makeMove/updateWithMove, noise after even plies.  Finished games restart when
 * restart != 0, in slot order, as the next game ids (one past the highest id started on the
 * handle; az_search_new_games' slots are ids 0..n-1), each seeding its evaluator / noise streams
 * by its id as az_selfplay_run does.  moves_done/evals_done accumulate the positions and NN
 * evaluations. */
typedef struct az_selfplay_cfg {
    int temp_drop_move;   /* 30 */
    float t_init;         /* 1.0 */
    float t_final;        /* 0.0 */
    int restart_finished; /* throughput mode: start a new game in a finished slot */
} az_selfplay_cfg;
int az_selfplay_step(az_search* s, const az_selfplay_cfg* cfg, int64_t* moves_done, int64_t* evals_done);

/* One committed move of a finished game: selfplay::MoveData (include/alphazero/selfplay/
 * game_record.h:21-33).  policy[] is the visit distribution in CHILD order (as the reference
 * records it, NaN entries at T = 0 included), child_actions[] the matching actions. */
typedef struct az_move_rec {
    int action;
    float value;
    int n_children;
    const float* policy;
    const int* child_actions;
    int64_t thinking_time_ms;
} az_move_rec;

/* The MoveData records az_selfplay_step assembled for its last step (one per game that moved;
 * slots[i] is the device slot of moves[i]); valid until the next call on the handle. */
int az_selfplay_step_moves(az_search* s, const az_move_rec** moves, const int** slots, int* n);

/* Receives every finished game once, on the calling thread between device steps; the arrays
 * are valid only during the call.  result: core::GameResult (0 ONGOING, 1 DRAW, 2 WIN_PLAYER1,
 * 3 WIN_PLAYER2; ONGOING for a game cut at max_moves). */
typedef void (*az_game_sink)(void* user, int game_id, int board_size, int n_moves, const az_move_rec* moves,
                             int result);
/* SelfPlayManager progress callback (gameId, moveNum, totalGames, totalMoves),
 * self_play_manager.cpp:198-203; called once per recorded move. */
typedef void (*az_progress_fn)(void* user, int game_id, int move_num, int total_games, int64_t total_moves);

/* SelfPlayManager::generateGames (self_play_manager.cpp:47-114 + playSingleGame :151-234):
 * plays total_games games, game ids 0..total_games-1, on the handle's n_games device slots
 * (a finished slot takes the next id; each game's evaluator/noise streams are seeded by its id,
 * so records do not depend on n_games).  max_moves <= 0: play to the end.  abort (optional) is
 * polled between moves (setAbort).  Returns 0 or an error code. */
int az_selfplay_run(az_search* s, const az_selfplay_cfg* cfg, int total_games, int max_moves, az_game_sink sink,
                    az_progress_fn progress, void* user, const volatile int* abort_flag);

/* --------------------------------------------------------------- dataset */
/* alphazero::selfplay::Dataset (include/alphazero/selfplay/dataset.h:33-118,
 * src/selfplay/dataset.cpp): device-resident training examples.  Example layout in HBM:
 * states fp32 [E][planes][bs][bs] (TrainingExample::state[plane][row][col]), policy fp32
 * [E][policy_stride] in the record's CHILD order (MoveData::policy, zero past its length),
 * policy length int32 [E], value fp32 [E]. */
typedef struct az_dataset az_dataset;
int az_dataset_create(az_engine* e, int game_type, int board_size, az_dataset** out);   /* AZ_GAME_* */
void az_dataset_destroy(az_dataset* d);
/* Dataset::extractExamples (dataset.cpp:60-114) over n_games records, replacing the examples:
 * game g has n_moves[g] moves; actions[] and n_children[] are concatenated over all moves,
 * policies[] concatenates every move's child-order policy; results[g] is the GameResult.
 * augment != 0: each position yields the original and the 7 augmentExample symmetries
 * (dataset.cpp:245-436) in the reference's order.  order (optional, E entries): slot i receives
 * pre-shuffle example order[i] -- the permutation Dataset::shuffle's std::shuffle applies
 * (dataset.cpp:112-113,147-149); null keeps the pre-shuffle order. */
int az_dataset_extract(az_dataset* d, int n_games, const int* n_moves, const int* actions, const int* n_children,
                       const float* policies, const int* results, int augment, const int64_t* order,
                       int64_t* n_examples);
int az_dataset_info(az_dataset* d, int64_t* n_examples, int* planes, int* board_size, int* policy_stride);
/* The handle's std::mt19937 (Dataset::rng_, dataset.h:115; the reference seeds it from
 * std::random_device, dataset.cpp:57 -- az_dataset_create does the same, az_dataset_seed fixes it). */
int az_dataset_seed(az_dataset* d, uint32_t seed);
/* std::shuffle of 0..n-1 on the handle's engine (libstdc++, as dataset.cpp:113,131,148,235 call it):
 * the order argument of az_dataset_extract / az_dataset_permute, or getBatch's index list. */
int az_dataset_shuffle_order(az_dataset* d, int64_t n, int64_t* order);
/* Replace the examples with n host examples (Dataset::loadFromFile, dataset.cpp:188-227). */
int az_dataset_upload(az_dataset* d, int64_t n, const float* states, const float* policy, const int* policy_len,
                      const float* value);
/* Dataset::shuffle (dataset.cpp:147-149) on device: slot i receives the current example order[i]. */
int az_dataset_permute(az_dataset* d, const int64_t* order);
/* Dataset::getBatch / getRandomSubset (dataset.cpp:120-145,229-243): examples idx[0..n) gathered on
 * the device, then copied to the host buffers (states [n][planes][bs][bs], policy [n][stride]). */
int az_dataset_gather(az_dataset* d, const int64_t* idx, int n, float* states, float* policy, int* policy_len,
                      float* value);
/* Measurement: time (HIP events on the engine stream) and algorithmic HBM bytes of the last
 * extraction kernel. */
int az_dataset_profile_read(az_dataset* d, double* extract_ms, double* bytes);

/* ------------------------------------------------------------ multi-GPU */
/* One process per GPU (the reference's per-GPU self_play processes,
 * python/scripts/orchestrate_selfplay.py:303-311,741-749), games sharded by contiguous global id
 * ranges with no data-path collective; RCCL over xGMI only to broadcast the weights and to reduce
 * the counters.  Rank 0 makes the id (az_dist_unique_id) and hands it to
 * every rank out of band (a file, a launcher's store); each rank calls az_dist_init with its own
 * engine.  Collectives run on the engine's stream and wait with a deadline: after timeout_ms
 * (<= 0: 600 s) without completion -- a rank died or never joined -- the communicator is aborted
 * and the call returns AZ_ERR_STATE, as does every later call on the handle. */
#define AZ_DIST_ID_BYTES 128
typedef struct az_dist az_dist;
enum az_dist_op { AZ_DIST_SUM = 0, AZ_DIST_MAX = 1 };
int az_dist_unique_id(unsigned char* id);   /* id[AZ_DIST_ID_BYTES] */
int az_dist_init(az_engine* e, int rank, int world, const unsigned char* id, int timeout_ms, az_dist** out);
void az_dist_destroy(az_dist* d);
int az_dist_info(az_dist* d, int* rank, int* world);
/* Every rank's engine stream drained and every rank arrived. */
int az_dist_barrier(az_dist* d);
/* out[i] = SUM or MAX over the ranks of in[i], i < count (1..64); host buffers (out may be in). */
int az_counters_allreduce(az_dist* d, const double* in, double* out, int count, int op);
/* Rank root's loaded weights into net n on every rank: ncclBroadcast straight into the net's
 * packed device weight buffers (every precision's piece set) and the canonical fp32 blob
 * (az_net_get_weights); no host hop on the device path.  The nets must share one az_net_desc
 * (checked); a never-loaded net on a non-root rank is allocated first. */
int az_net_broadcast_weights(az_dist* d, az_net* n, int root);

#ifdef __cplusplus
}
#endif
#endif /* AZ_ENGINE_H */
