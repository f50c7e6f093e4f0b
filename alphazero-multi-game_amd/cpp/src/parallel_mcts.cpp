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

ParallelMCTS::ParallelMCTS(const core::IGameState& root, SearchGroup& group)
    : nn_(group.network()), tt_(nullptr), root_(root.clone()) {
    const az_search_cfg& g = group.deviceConfig();
    config_.numSimulations = g.num_simulations;
    config_.cPuct = g.c_puct;
    config_.fpuReduction = g.fpu_reduction;
    config_.virtualLoss = g.virtual_loss;
    config_.useDirichletNoise = g.use_dirichlet_each_search != 0;
    config_.dirichletAlpha = g.dirichlet_alpha;
    config_.dirichletEpsilon = g.dirichlet_eps;
    config_.transpositionTableSize = 1 << g.tt_log2;
    if (root_->getBoardSize() != g.board_size || (root_->getGameType() == core::GameType::GO) != (g.game == AZ_GAME_GO))
        throw std::invalid_argument("ParallelMCTS: the root's game does not match the group's");
    slot_ = group.acquire(*root_);
    group_ = &group;
    s_ = group.handle();
}

ParallelMCTS::~ParallelMCTS() {
    if (group_) group_->release(slot_);
    else if (s_) az_search_destroy(s_);
}

az_search_cfg makeSearchConfig(const MCTSConfig& config, const core::IGameState& state, nn::NeuralNetwork* nn,
                               const TranspositionTable* tt, int nGames) {
    const bool go = state.getGameType() == core::GameType::GO;
    const DeviceEvaluator ev = deviceEvaluator(nn);
    az_search_cfg c{};
    c.game = go ? AZ_GAME_GO : AZ_GAME_GOMOKU;
    c.n_games = nGames;
    c.board_size = state.getBoardSize();
    c.num_simulations = config.numSimulations;
    c.c_puct = config.cPuct;
    c.fpu_reduction = config.fpuReduction;
    c.virtual_loss = config.virtualLoss;
    c.eval_kind = ev.kind;
    c.eval_seed = ev.seed;
    c.zobrist_seed = 12345u;
    c.noise_seed = 42u;          // setDeterministicMode's rng seed (parallel_mcts.cpp:1268)
    c.noise_seed_stride = 0;
    c.use_dirichlet_each_search = config.useDirichletNoise ? 1 : 0;
    c.dirichlet_alpha = config.dirichletAlpha;
    c.dirichlet_eps = config.dirichletEpsilon;
    const size_t ttsize = tt ? tt->getSize() : (size_t)config.transpositionTableSize;
    int k = 0;
    while (((size_t)1 << k) < ttsize && k < 24) ++k;
    c.tt_log2 = k;
    return c;
}

az_search_cfg ParallelMCTS::deviceConfig() const { return makeSearchConfig(config_, *root_, nn_, tt_, 1); }

std::vector<uint8_t> ParallelMCTS::slotMask() const {
    std::vector<uint8_t> m(group_ ? group_->capacity() : 1, 0);
    m[slot_] = 1;
    return m;
}

static bool sameSearch(const az_search_cfg& a, const az_search_cfg& b) {   // all but n_games
    return a.game == b.game && a.board_size == b.board_size && a.num_simulations == b.num_simulations &&
           a.c_puct == b.c_puct && a.fpu_reduction == b.fpu_reduction && a.virtual_loss == b.virtual_loss &&
           a.eval_kind == b.eval_kind && a.eval_seed == b.eval_seed &&
           a.use_dirichlet_each_search == b.use_dirichlet_each_search && a.dirichlet_alpha == b.dirichlet_alpha &&
           a.dirichlet_eps == b.dirichlet_eps && a.tt_log2 == b.tt_log2;
}

// The reference's setters change config_ and keep the tree (parallel_mcts.h:172-182); the device
// handle takes the new parameters in place when it can, and is rebuilt (history replayed) when the
// evaluator, the table size or a larger node pool is needed.
void ParallelMCTS::applyConfig() {
    const az_search_cfg c = deviceConfig();
    if (group_) {                          // the group's parameters are shared: other ones leave it
        if (!sameSearch(c, group_->deviceConfig())) rebuild();
        return;
    }
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
        check(az_search_get_rng(s_, slot_, rng.data()), "az_search_get_rng");
        if (group_) group_->release(slot_);      // leaves the group: a handle of its own
        else az_search_destroy(s_);
        group_ = nullptr;
        slot_ = 0;
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
    if (group_) group_->search(slot_);
    else check(az_search_run(s_), "az_search_run");
    searched_ = true;
    int64_t c[5] = {0, 0, 0, 0, 0};
    check(az_search_counters(s_, slot_, c), "az_search_counters");
    stats_.evaluationCalls = (size_t)c[0];
    stats_.cacheHits = (size_t)c[2];
    stats_.cacheMisses = (size_t)(c[1] - c[2]);
    stats_.simulationCount = (size_t)c[3];
    stats_.nodesCreated = (size_t)c[4];
    if (tt_) tt_->record((uint64_t)c[1], (uint64_t)c[2], 0);
    if (progress_) progress_(config_.numSimulations, config_.numSimulations);
}

void ParallelMCTS::runSingleSimulation() {
    if (group_) check(az_search_simulate_masked(s_, 1, slotMask().data()), "az_search_simulate_masked");
    else check(az_search_simulate(s_, 1), "az_search_simulate");
    searched_ = true;
}

void ParallelMCTS::runBatchedSearch() {
    if (config_.numSimulations <= 0) return;
    if (group_) check(az_search_simulate_masked(s_, config_.numSimulations, slotMask().data()), "az_search_simulate_masked");
    else check(az_search_simulate(s_, config_.numSimulations), "az_search_simulate");
    searched_ = true;
}

size_t ParallelMCTS::releaseMemory(int visitThreshold) {
    if (group_) {
        std::vector<int64_t> pruned(group_->capacity(), 0);
        check(az_search_release_masked(s_, visitThreshold, pruned.data(), slotMask().data()), "az_search_release_masked");
        return (size_t)pruned[slot_];
    }
    int64_t pruned = 0;
    check(az_search_release(s_, visitThreshold, &pruned), "az_search_release");
    return (size_t)pruned;
}

int ParallelMCTS::selectAction(bool isTraining, float temperature) {
    int flags = 0;
    check(az_search_root_flags(s_, slot_, &flags), "az_search_root_flags");
    if (!(flags & AZ_NODE_EXPANDED)) search();        // parallel_mcts.cpp:988-991
    const std::vector<int> legal = root_->getLegalMoves();
    int act = -1;
    check(az_search_select_action(s_, slot_, isTraining ? 1 : 0, temperature, config_.useBatchInference ? 1 : 0,
                                  legal.data(), (int)legal.size(), &act),
          "az_search_select_action");
    return act;
}

MCTSNode ParallelMCTS::getRootNode() const {
    MCTSNode r;
    int flags = 0;
    check(az_search_root_flags(s_, slot_, &flags), "az_search_root_flags");
    check(az_search_root_node(s_, slot_, &r.visitCount, &r.virtualLoss, &r.valueSum), "az_search_root_node");
    r.isExpanded = (flags & AZ_NODE_EXPANDED) != 0;
    r.isTerminal = (flags & AZ_NODE_TERMINAL) != 0;
    r.gameResult = r.isTerminal ? (core::GameResult)((flags >> 2) & 3) : root_->getGameResult();
    r.prior = 0.0f;
    const int A = root_->getActionSpaceSize();
    std::vector<int> act(A), N(A), VL(A);
    std::vector<float> W(A), P(A);
    int n = 0;
    check(az_search_root_children(s_, slot_, act.data(), N.data(), VL.data(), W.data(), P.data(), &n), "az_search_root_children");
    for (int i = 0; i < n; ++i) {
        auto c = std::make_shared<MCTSNode>();
        c->visitCount = N[i]; c->virtualLoss = VL[i]; c->valueSum = W[i]; c->prior = P[i]; c->action = act[i];
        r.actions.push_back(act[i]);
        r.children.push_back(c);
    }
    return r;
}

// getActionProbabilities(T) + getChildActions + getRootValue of this object's game: az_search_select
// reports every game of the handle (a group's: every slot), this slot's row is taken
ParallelMCTS::RootSelect ParallelMCTS::rootSelect(float temperature) const {
    const int G = group_ ? group_->capacity() : 1;
    const int NA = root_->getActionSpaceSize();
    std::vector<int> act(G), nch(G), cact((size_t)G * NA);
    std::vector<float> val(G), probs((size_t)G * NA);
    check(az_search_select(s_, 1, temperature, act.data(), val.data(), probs.data(), cact.data(), nch.data()),
          "az_search_select");
    RootSelect r;
    const size_t o = (size_t)slot_ * NA;
    r.probs.assign(probs.begin() + o, probs.begin() + o + nch[slot_]);
    r.actions.assign(cact.begin() + o, cact.begin() + o + nch[slot_]);
    r.value = val[slot_];
    return r;
}

std::vector<float> ParallelMCTS::getActionProbabilities(float temperature) const {
    const RootSelect r = rootSelect(temperature);
    return r.probs;
}

std::vector<int> ParallelMCTS::getChildActions() const {
    return rootSelect(1.0f).actions;
}

float ParallelMCTS::getRootValue() const {
    return rootSelect(1.0f).value;
}

void ParallelMCTS::updateWithMove(int action) {
    root_->makeMove(action);
    if (group_) {                          // only this slot moves (the others get no action)
        const int G = group_->capacity();
        std::vector<int> acts(G, AZ_ACTION_NONE), t(G), r(G);
        acts[slot_] = action;
        check(az_search_apply(s_, acts.data(), t.data(), r.data()), "az_search_apply");
    } else {
        int t = 0, r = 0;
        check(az_search_apply(s_, &action, &t, &r), "az_search_apply");
    }
    searched_ = false;
}

void ParallelMCTS::addDirichletNoise(float alpha, float epsilon) {
    if (root_->isTerminal()) return;
    if (group_) check(az_search_add_noise_masked(s_, alpha, epsilon, slotMask().data()), "az_search_add_noise_masked");
    else check(az_search_add_noise(s_, alpha, epsilon), "az_search_add_noise");
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
    if (group_) {                          // the group's evaluator is shared: another one leaves it
        if (nn != nn_) { nn_ = nn; rebuild(); }
        return;
    }
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
    if (group_) {                          // a table of its own: the member leaves the group
        if (tt != old) rebuild();
        return;
    }
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
    check(az_search_seed(s_, slot_, enable ? 42u : rd()), "az_search_seed");
}

std::vector<std::tuple<int, int, float, float>> ParallelMCTS::analyzePosition(int topN) const {
    const int A = root_->getActionSpaceSize();
    std::vector<int> act(A), N(A), VL(A);
    std::vector<float> W(A), P(A);
    int n = 0;
    check(az_search_root_children(s_, slot_, act.data(), N.data(), VL.data(), W.data(), P.data(), &n),
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
    check(az_search_root_node(s_, slot_, &N, &VL, &W), "az_search_root_node");
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
