// ParallelMCTS / TranspositionTable of the host API over az_search_* (one game slot).
#include "alphazero/mcts/parallel_mcts.h"

#include <algorithm>
#include <cmath>
#include <iostream>
#include <random>
#include <sstream>

#include "alphazero/games/go/go_state.h"
#include "alphazero/nn/hip_neural_network.h"
#include "alphazero/nn/random_policy_network.h"

namespace alphazero {
namespace mcts {

static void check(int rc, const char* what) {
    if (rc != 0) throw std::runtime_error(std::string(what) + ": " + az_last_error());
}

TranspositionTable::TranspositionTable(size_t size, size_t numShards) : size_(1), shards_(numShards) { resize(size); }

void TranspositionTable::resize(size_t size) {
    size_ = 1;
    while (size_ < size && size_ < ((size_t)1 << 24)) size_ <<= 1;   // rounded up to 2^k (reference ctor)
    clear();
}

int TranspositionTable::log2Size() const {
    int k = 0;
    while (((size_t)1 << k) < size_) ++k;
    return k;
}

DeviceEvaluator deviceEvaluator(nn::NeuralNetwork* nn) {
    if (!nn) return {AZ_EVAL_UNIFORM, 0u, nullptr, nn::engineForDevice(-1)};
    if (auto* h = dynamic_cast<nn::HipNeuralNetwork*>(nn)) return {AZ_EVAL_NET, 0u, h->handle(), h->engine()};
    if (auto* r = dynamic_cast<nn::RandomPolicyNetwork*>(nn)) return {AZ_EVAL_RANDOM, r->seed(), nullptr, nn::engineForDevice(-1)};
    // any other NeuralNetwork subclass: the device search hands its leaves to the host
    // (AZ_EVAL_CALLBACK, ParallelMCTS::hostEvaluate)
    return {AZ_EVAL_CALLBACK, 0u, nullptr, nn::engineForDevice(-1)};
}

// AZ_EVAL_CALLBACK trampoline: every leaf is the root state plus the moves from the root; one leaf
// goes to nn_->predict as evaluateState calls it (parallel_mcts.cpp:886-901), several to
// predictBatch.  A throwing evaluator gets the reference's fallback: uniform policy, value 0.
int ParallelMCTS::hostEvaluate(void* user, int n, const int* games, const int* pathLen, const int* moves, int maxPath,
                               const float* planes, int nPlanes, float* policy, float* value) {
    auto* self = static_cast<ParallelMCTS*>(user);
    const int A = self->root_->getActionSpaceSize();
    const int h = (int)self->root_->getMoveHistory().size();   // moves[] start from the empty board
    std::vector<std::unique_ptr<core::IGameState>> leaves;
    leaves.reserve(n);
    for (int i = 0; i < n; ++i) {
        auto st = self->root_->clone();
        for (int k = h; k < pathLen[i]; ++k) st->makeMove(moves[(size_t)i * maxPath + k]);
        leaves.push_back(std::move(st));
    }
    auto fallback = [&](int i) {
        for (int a = 0; a < A; ++a) policy[(size_t)i * A + a] = 1.0f / (float)A;
        value[i] = 0.0f;
    };
    auto put = [&](int i, const std::vector<float>& p, float v) {
        for (int a = 0; a < A; ++a) policy[(size_t)i * A + a] = a < (int)p.size() ? p[a] : 0.0f;
        value[i] = v;
    };
    if (n == 1) {
        try {
            auto pv = self->nn_->predict(*leaves[0]);
            put(0, pv.first, pv.second);
        } catch (const std::exception&) { fallback(0); }
        return 0;
    }
    std::vector<std::reference_wrapper<const core::IGameState>> refs;
    for (auto& l : leaves) refs.emplace_back(*l);
    std::vector<std::vector<float>> ps;
    std::vector<float> vs;
    try {
        self->nn_->predictBatch(refs, ps, vs);
        for (int i = 0; i < n; ++i) {
            if (i < (int)ps.size() && i < (int)vs.size()) put(i, ps[i], vs[i]);
            else fallback(i);
        }
    } catch (const std::exception&) {
        for (int i = 0; i < n; ++i) fallback(i);
    }
    return 0;
}

ParallelMCTS::ParallelMCTS(const core::IGameState& root, nn::NeuralNetwork* nn, TranspositionTable* tt, int numThreads,
                           int numSimulations, float cPuct, float fpuReduction, int virtualLoss)
    : nn_(nn), tt_(tt), root_(root.clone()) {
    config_.numThreads = numThreads;
    config_.numSimulations = numSimulations;
    config_.cPuct = cPuct;
    config_.fpuReduction = fpuReduction;
    config_.virtualLoss = virtualLoss;
    rebuild();
}

ParallelMCTS::ParallelMCTS(const core::IGameState& root, const MCTSConfig& config, nn::NeuralNetwork* nn,
                           TranspositionTable* tt)
    : config_(config), nn_(nn), tt_(tt), root_(root.clone()) {
    rebuild();
}

ParallelMCTS::~ParallelMCTS() {
    if (s_) az_search_destroy(s_);
}

az_search_cfg ParallelMCTS::deviceConfig() const {
    const bool go = root_->getGameType() == core::GameType::GO;
    const DeviceEvaluator ev = deviceEvaluator(nn_);
    az_search_cfg c{};
    c.game = go ? AZ_GAME_GO : AZ_GAME_GOMOKU;
    c.n_games = 1;
    c.board_size = root_->getBoardSize();
    c.num_simulations = config_.numSimulations;
    c.c_puct = config_.cPuct;
    c.fpu_reduction = config_.fpuReduction;
    c.virtual_loss = config_.virtualLoss;
    c.eval_kind = ev.kind;
    c.eval_seed = ev.seed;
    c.zobrist_seed = 12345u;
    c.noise_seed = 42u;          // setDeterministicMode's rng seed (parallel_mcts.cpp:1268)
    c.noise_seed_stride = 0;
    c.use_dirichlet_each_search = config_.useDirichletNoise ? 1 : 0;
    c.dirichlet_alpha = config_.dirichletAlpha;
    c.dirichlet_eps = config_.dirichletEpsilon;
    const size_t ttsize = tt_ ? tt_->getSize() : (size_t)config_.transpositionTableSize;
    int k = 0;
    while (((size_t)1 << k) < ttsize && k < 24) ++k;
    c.tt_log2 = k;
    return c;
}

// The reference's setters change config_ and keep the tree (parallel_mcts.h:172-182); the device
// handle takes the new parameters in place when it can, and is rebuilt (history replayed) when the
// evaluator, the table size or a larger node pool is needed.
void ParallelMCTS::applyConfig() {
    const az_search_cfg c = deviceConfig();
    if (s_ && az_search_set_params(s_, &c) == 0) return;
    rebuild();
}

void ParallelMCTS::rebuild() {
    const bool go = root_->getGameType() == core::GameType::GO;
    if (!go && root_->getGameType() != core::GameType::GOMOKU) throw std::invalid_argument("ParallelMCTS: Gomoku or Go");
    if (go) {
        auto* g = dynamic_cast<const go::GoState*>(root_.get());
        if (!g || g->getKomi() != 7.5f || !g->isChineseRules() || !g->isEnforcingSuperko())
            throw std::invalid_argument("ParallelMCTS: the device Go rules are komi 7.5, Chinese rules, superko");
    }
    // rng_ survives the rebuild (the reference's setters leave it alone): carried over whole
    std::vector<uint32_t> rng;
    if (s_) {
        rng.resize(AZ_RNG_STATE_WORDS);
        check(az_search_get_rng(s_, 0, rng.data()), "az_search_get_rng");
        az_search_destroy(s_);
        s_ = nullptr;
    }
    const DeviceEvaluator ev = deviceEvaluator(nn_);
    const az_search_cfg c = deviceConfig();
    check(az_search_create(ev.engine, ev.net, &c, &s_), "az_search_create");
    if (c.eval_kind == AZ_EVAL_CALLBACK) check(az_search_set_evaluator(s_, &ParallelMCTS::hostEvaluate, this), "az_search_set_evaluator");
    const int g0 = 0;
    check(az_search_new_games(s_, &g0, 1), "az_search_new_games");
    // a non-initial root: replay its history (each move a fresh root, as updateWithMove without a search)
    for (int a : root_->getMoveHistory()) {
        int t = 0, r = 0;
        check(az_search_apply(s_, &a, &t, &r), "az_search_apply");
    }
    if (!rng.empty()) check(az_search_set_rng(s_, 0, rng.data()), "az_search_set_rng");
    searched_ = false;
}

void ParallelMCTS::search() {
    if (root_->isTerminal()) return;
    check(az_search_run(s_), "az_search_run");
    searched_ = true;
    int64_t c[5] = {0, 0, 0, 0, 0};
    check(az_search_counters(s_, 0, c), "az_search_counters");
    stats_.evaluationCalls = (size_t)c[0];
    stats_.cacheHits = (size_t)c[2];
    stats_.cacheMisses = (size_t)(c[1] - c[2]);
    stats_.simulationCount = (size_t)c[3];
    stats_.nodesCreated = (size_t)c[4];
    if (tt_) tt_->record((uint64_t)c[1], (uint64_t)c[2], 0);
    if (progress_) progress_(config_.numSimulations, config_.numSimulations);
}

void ParallelMCTS::runSingleSimulation() {
    check(az_search_simulate(s_, 1), "az_search_simulate");
    searched_ = true;
}

void ParallelMCTS::runBatchedSearch() {
    if (config_.numSimulations <= 0) return;
    check(az_search_simulate(s_, config_.numSimulations), "az_search_simulate");
    searched_ = true;
}

size_t ParallelMCTS::releaseMemory(int visitThreshold) {
    int64_t pruned = 0;
    check(az_search_release(s_, visitThreshold, &pruned), "az_search_release");
    return (size_t)pruned;
}

int ParallelMCTS::selectAction(bool isTraining, float temperature) {
    int flags = 0;
    check(az_search_root_flags(s_, 0, &flags), "az_search_root_flags");
    if (!(flags & AZ_NODE_EXPANDED)) search();        // parallel_mcts.cpp:988-991
    const std::vector<int> legal = root_->getLegalMoves();
    int act = -1;
    check(az_search_select_action(s_, 0, isTraining ? 1 : 0, temperature, config_.useBatchInference ? 1 : 0,
                                  legal.data(), (int)legal.size(), &act),
          "az_search_select_action");
    return act;
}

MCTSNode ParallelMCTS::getRootNode() const {
    MCTSNode r;
    int flags = 0;
    check(az_search_root_flags(s_, 0, &flags), "az_search_root_flags");
    check(az_search_root_node(s_, 0, &r.visitCount, &r.virtualLoss, &r.valueSum), "az_search_root_node");
    r.isExpanded = (flags & AZ_NODE_EXPANDED) != 0;
    r.isTerminal = (flags & AZ_NODE_TERMINAL) != 0;
    r.gameResult = r.isTerminal ? (core::GameResult)((flags >> 2) & 3) : root_->getGameResult();
    r.prior = 0.0f;
    const int A = root_->getActionSpaceSize();
    std::vector<int> act(A), N(A), VL(A);
    std::vector<float> W(A), P(A);
    int n = 0;
    check(az_search_root_children(s_, 0, act.data(), N.data(), VL.data(), W.data(), P.data(), &n), "az_search_root_children");
    for (int i = 0; i < n; ++i) {
        auto c = std::make_shared<MCTSNode>();
        c->visitCount = N[i]; c->virtualLoss = VL[i]; c->valueSum = W[i]; c->prior = P[i]; c->action = act[i];
        r.actions.push_back(act[i]);
        r.children.push_back(c);
    }
    return r;
}

std::vector<float> ParallelMCTS::getActionProbabilities(float temperature) const {
    int act = -1, nch = 0;
    float val = 0.0f;
    const int A = root_->getActionSpaceSize();
    std::vector<float> probs(A);
    std::vector<int> cact(A);
    check(az_search_select(s_, 1, temperature, &act, &val, probs.data(), cact.data(), &nch), "az_search_select");
    probs.resize(nch);
    return probs;
}

std::vector<int> ParallelMCTS::getChildActions() const {
    int act = -1, nch = 0;
    float val = 0.0f;
    const int A = root_->getActionSpaceSize();
    std::vector<float> probs(A);
    std::vector<int> cact(A);
    check(az_search_select(s_, 1, 1.0f, &act, &val, probs.data(), cact.data(), &nch), "az_search_select");
    cact.resize(nch);
    return cact;
}

float ParallelMCTS::getRootValue() const {
    int act = -1, nch = 0;
    float val = 0.0f;
    const int A = root_->getActionSpaceSize();
    std::vector<float> probs(A);
    std::vector<int> cact(A);
    check(az_search_select(s_, 1, 1.0f, &act, &val, probs.data(), cact.data(), &nch), "az_search_select");
    return val;
}

void ParallelMCTS::updateWithMove(int action) {
    root_->makeMove(action);
    int t = 0, r = 0;
    check(az_search_apply(s_, &action, &t, &r), "az_search_apply");
    searched_ = false;
}

void ParallelMCTS::addDirichletNoise(float alpha, float epsilon) {
    if (root_->isTerminal()) return;
    check(az_search_add_noise(s_, alpha, epsilon), "az_search_add_noise");
}

void ParallelMCTS::setNumSimulations(int n) { config_.numSimulations = n; applyConfig(); }
void ParallelMCTS::setCPuct(float c) { config_.cPuct = c; applyConfig(); }
void ParallelMCTS::setFpuReduction(float f) { config_.fpuReduction = f; applyConfig(); }
void ParallelMCTS::setVirtualLoss(int v) { config_.virtualLoss = v; applyConfig(); }
// parallel_mcts.cpp:1190-1222: the setters replace nn_ / tt_ and keep the tree.  On the device: a
// device net of the same shape is swapped in place (az_search_set_net), a host evaluator
// (AZ_EVAL_CALLBACK) is read through nn_ at every leaf batch anyway, and a new table of the same
// size empties the device table (az_search_clear_tt); any other change (evaluator kind, random
// network seed, table size) needs a new handle: the history is replayed and the tree rebuilt.
void ParallelMCTS::setNeuralNetwork(nn::NeuralNetwork* nn) {
    const DeviceEvaluator cur = deviceEvaluator(nn_), nxt = deviceEvaluator(nn);
    nn_ = nn;
    if (s_ && cur.kind == AZ_EVAL_NET && nxt.kind == AZ_EVAL_NET && cur.engine == nxt.engine &&
        az_search_set_net(s_, nxt.net) == 0)
        return;
    if (s_ && cur.kind == AZ_EVAL_CALLBACK && nxt.kind == AZ_EVAL_CALLBACK) return;
    rebuild();
}
void ParallelMCTS::setTranspositionTable(TranspositionTable* tt) {
    const az_search_cfg before = deviceConfig();
    TranspositionTable* old = tt_;
    tt_ = tt;
    if (s_ && deviceConfig().tt_log2 == before.tt_log2) {
        if (tt != old) check(az_search_clear_tt(s_), "az_search_clear_tt");
        return;
    }
    rebuild();
}
void ParallelMCTS::setConfig(const MCTSConfig& config) { config_ = config; applyConfig(); }
// parallel_mcts.cpp:1263-1274: useBatchInference = enable; rng_ seeded 42, or from std::random_device
void ParallelMCTS::setDeterministicMode(bool enable) {
    config_.deterministic = enable;
    config_.useBatchInference = enable;
    std::random_device rd;
    check(az_search_seed(s_, 0, enable ? 42u : rd()), "az_search_seed");
}

std::vector<std::tuple<int, int, float, float>> ParallelMCTS::analyzePosition(int topN) const {
    const int A = root_->getActionSpaceSize();
    std::vector<int> act(A), N(A), VL(A);
    std::vector<float> W(A), P(A);
    int n = 0;
    check(az_search_root_children(s_, 0, act.data(), N.data(), VL.data(), W.data(), P.data(), &n),
          "az_search_root_children");
    std::vector<std::tuple<int, int, float, float>> out;
    for (int i = 0; i < n; ++i) out.emplace_back(act[i], N[i], N[i] > 0 ? W[i] / (float)N[i] : 0.0f, P[i]);
    std::stable_sort(out.begin(), out.end(), [](const auto& a, const auto& b) { return std::get<1>(a) > std::get<1>(b); });
    if ((int)out.size() > topN) out.resize(topN);
    return out;
}

std::string ParallelMCTS::getSearchInfo() const {
    int N = 0, VL = 0;
    float W = 0.0f;
    check(az_search_root_node(s_, 0, &N, &VL, &W), "az_search_root_node");
    std::ostringstream o;
    o << "root visits " << N << ", value " << (N ? W / (float)N : 0.0f) << ", simulations "
      << stats_.simulationCount.load() << ", evaluations " << stats_.evaluationCalls.load() << ", TT hits "
      << stats_.cacheHits.load() << "\n";
    for (const auto& [a, n, q, p] : analyzePosition(5))
        o << "  " << root_->actionToString(a) << "  N=" << n << "  Q=" << q << "  P=" << p << "\n";
    return o.str();
}

void ParallelMCTS::printSearchStats() const { std::cout << getSearchInfo(); }

void ParallelMCTS::printSearchPath(int action) const {
    for (const auto& [a, n, q, p] : analyzePosition(root_->getActionSpaceSize()))
        if (a == action) std::cout << root_->actionToString(a) << " N=" << n << " Q=" << q << " P=" << p << "\n";
}

size_t ParallelMCTS::getMemoryUsage() const {
    const size_t A = (size_t)root_->getActionSpaceSize();
    return 2 * (3 * (size_t)std::max(64, config_.numSimulations) * A + 8 * A + 64) * 25 +
           ((size_t)1 << (tt_ ? tt_->log2Size() : 20)) * 24;
}

}  // namespace mcts
}  // namespace alphazero
