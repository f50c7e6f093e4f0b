// ParallelMCTS / TranspositionTable of the host API over az_search_* (one game slot).
#include "alphazero/mcts/parallel_mcts.h"

#include <algorithm>
#include <cmath>
#include <iostream>
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
    throw std::invalid_argument("ParallelMCTS: evaluator class has no device implementation "
                                "(use HipNeuralNetwork, RandomPolicyNetwork or nullptr)");
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

void ParallelMCTS::rebuild() {
    const bool go = root_->getGameType() == core::GameType::GO;
    if (!go && root_->getGameType() != core::GameType::GOMOKU) throw std::invalid_argument("ParallelMCTS: Gomoku or Go");
    if (go) {
        auto* g = dynamic_cast<const go::GoState*>(root_.get());
        if (!g || g->getKomi() != 7.5f || !g->isChineseRules() || !g->isEnforcingSuperko())
            throw std::invalid_argument("ParallelMCTS: the device Go rules are komi 7.5, Chinese rules, superko");
    }
    if (s_) { az_search_destroy(s_); s_ = nullptr; }
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
    check(az_search_create(ev.engine, ev.net, &c, &s_), "az_search_create");
    const int g0 = 0;
    check(az_search_new_games(s_, &g0, 1), "az_search_new_games");
    // a non-initial root: replay its history (each move a fresh root, as updateWithMove without a search)
    for (int a : root_->getMoveHistory()) {
        int t = 0, r = 0;
        check(az_search_apply(s_, &a, &t, &r), "az_search_apply");
    }
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

int ParallelMCTS::selectAction(bool isTraining, float temperature) {
    int act = -1, nch = 0;
    float val = 0.0f;
    const int A = root_->getActionSpaceSize();
    std::vector<float> probs(A);
    std::vector<int> cact(A);
    check(az_search_select(s_, isTraining ? 1 : 0, temperature, &act, &val, probs.data(), cact.data(), &nch),
          "az_search_select");
    return act;
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

void ParallelMCTS::setNumSimulations(int n) { config_.numSimulations = n; rebuild(); }
void ParallelMCTS::setCPuct(float c) { config_.cPuct = c; rebuild(); }
void ParallelMCTS::setFpuReduction(float f) { config_.fpuReduction = f; rebuild(); }
void ParallelMCTS::setVirtualLoss(int v) { config_.virtualLoss = v; rebuild(); }
void ParallelMCTS::setNeuralNetwork(nn::NeuralNetwork* nn) { nn_ = nn; rebuild(); }
void ParallelMCTS::setTranspositionTable(TranspositionTable* tt) { tt_ = tt; rebuild(); }
void ParallelMCTS::setConfig(const MCTSConfig& config) { config_ = config; rebuild(); }
void ParallelMCTS::setDeterministicMode(bool enable) {
    config_.deterministic = enable;
    config_.useBatchInference = config_.useBatchInference || enable;   // the device rule is already deterministic
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
