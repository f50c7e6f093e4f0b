// oracle/ref_harness.cpp -- TEST INFRASTRUCTURE ONLY (never shipped, never measured).
//
// Driver that links against a minimally patched build of the REFERENCE search
// (/root/reference/src/{mcts,games/gomoku,nn,core}, compiled into a temp dir by
// oracle/build_ref.sh; patches P1/P2/P5 of SURVEY.md Appendix B, no arithmetic
// change) and dumps golden vectors as JSON:
//
//   game      Mode S self-play: ParallelMCTS with
//             numThreads=1, useBatchedMCTS=false, setDeterministicMode(true),
//             driven by the SelfPlayManager::playSingleGame move loop
//             (src/selfplay/self_play_manager.cpp:175-216).  Per move it records
//             the root children (child order) with raw N / VL / W bits / P bits.
//   positions GomokuState feature planes (gomoku_state.cpp:207-258), Zobrist
//             hash (:620-656), terminal/result (:477-529), legal-move order.
//   gamma     libstdc++ gamma_distribution<float> draws on mt19937(42), as used
//             by ParallelMCTS::addDirichletNoise (parallel_mcts.cpp:1136-1142).
//   api       ParallelMCTS API operations beyond the self-play loop (runSingleSimulation,
//             runBatchedSearch, releaseMemory, stochastic selectAction; see run_api)
//   go_positions / go_game  the same for GoState(bs, komi 7.5, Chinese rules, superko)
//             (src/games/go/go_state.cpp, go_rules.cpp; patch P6 seeds its Zobrist keys).
//
// Evaluators: the reference's own RandomPolicyNetwork(seed) (random_policy_network.cpp)
// and HashEvaluator, a pure function of (Zobrist hash, last 6 moves) that the engine
// and oracle/az_oracle.cpp restate bit-for-bit (see hash_eval below).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <future>
#include <iomanip>
#include <iostream>
#include <limits>
#include <map>
#include <memory>
#include <mutex>
#include <optional>
#include <queue>
#include <random>
#include <set>
#include <sstream>
#include <stack>
#include <string>
#include <thread>
#include <tuple>
#include <unordered_map>
#include <unordered_set>
#include <vector>

// Read access to the tree statistics (rootNode_, children, raw W / VL) without
// editing the reference: the class layout is unchanged by the access keywords.
#define private public
#define protected public
#include "alphazero/mcts/parallel_mcts.h"
#include "alphazero/mcts/transposition_table.h"
#include "alphazero/games/gomoku/gomoku_state.h"
#include "alphazero/games/go/go_state.h"
#include "alphazero/nn/random_policy_network.h"
#undef private
#undef protected

using namespace alphazero;

static uint32_t fbits(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }

static uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

// HashEvaluator: deterministic, history-sensitive evaluator (so transposition-table
// hits are observable: same Zobrist key, different move history => different output).
static void hash_eval(uint64_t zhash, const std::vector<int>& hist, int A,
                      std::vector<float>& policy, float& value) {
    uint64_t key = splitmix64(zhash ^ 0x5A17C0DEULL);
    for (int i = 0; i < 6; ++i) {
        int m = (i < (int)hist.size()) ? hist[hist.size() - 1 - i] : -1;
        key = splitmix64(key + (uint64_t)(uint32_t)(m + 2));
    }
    policy.assign(A, 0.0f);
    for (int a = 0; a < A; ++a) {
        uint64_t r = splitmix64(key ^ ((uint64_t)(a + 1) * 0x9E3779B97F4A7C15ULL));
        policy[a] = (float)(uint32_t)(r >> 40) * (1.0f / 16777216.0f);
    }
    uint64_t rv = splitmix64(key ^ 0x76A1ULL);
    value = ((float)(int32_t)(uint32_t)(rv >> 40) - 8388608.0f) * (1.0f / 8388608.0f);
}

class HashEvaluator : public nn::NeuralNetwork {
public:
    long calls = 0;
    std::pair<std::vector<float>, float> predict(const core::IGameState& s) override {
        ++calls;
        std::vector<float> p; float v;
        hash_eval(s.getHash(), s.getMoveHistory(), s.getActionSpaceSize(), p, v);
        return {p, v};
    }
    void predictBatch(const std::vector<std::reference_wrapper<const core::IGameState>>& states,
                      std::vector<std::vector<float>>& ps, std::vector<float>& vs) override {
        ps.clear(); vs.clear();
        for (auto& r : states) { auto pv = predict(r.get()); ps.push_back(pv.first); vs.push_back(pv.second); }
    }
    std::future<std::pair<std::vector<float>, float>> predictAsync(const core::IGameState& s) override {
        std::promise<std::pair<std::vector<float>, float>> pr; pr.set_value(predict(s)); return pr.get_future();
    }
    bool isGpuAvailable() const override { return false; }
    std::string getDeviceInfo() const override { return "hash"; }
    float getInferenceTimeMs() const override { return 0.f; }
    int getBatchSize() const override { return 1; }
    std::string getModelInfo() const override { return "HashEvaluator"; }
    size_t getModelSizeBytes() const override { return 0; }
    void benchmark(int, int) override {}
    void enableDebugMode(bool) override {}
    void printModelSummary() const override {}
};

// Counts calls into the reference RandomPolicyNetwork (its predict sleeps 1 ms).
class CountingRandom : public nn::RandomPolicyNetwork {
public:
    long calls = 0;
    CountingRandom(int bs, unsigned seed) : nn::RandomPolicyNetwork(core::GameType::GOMOKU, bs, seed) {}
    std::pair<std::vector<float>, float> predict(const core::IGameState& s) override {
        ++calls; return nn::RandomPolicyNetwork::predict(s);
    }
};

static void dump_node_children(std::ostream& o, const mcts::MCTSNode* n) {
    o << "[";
    for (size_t i = 0; i < n->children.size(); ++i) {
        const mcts::MCTSNode* c = n->children[i].get();
        if (i) o << ",";
        o << "[" << n->actions[i] << "," << c->visitCount.load() << "," << c->virtualLoss.load() << ","
          << fbits(c->valueSum.load()) << "," << fbits(c->prior) << "]";
    }
    o << "]";
}

static int run_game(int bs, int sims, int maxMoves, const std::string& evalKind, unsigned evalSeed,
                    int noiseEachSearch, float cpuct, float fpu, bool go = false) {
    std::unique_ptr<core::IGameState> state;
    if (go) state = std::make_unique<go::GoState>(bs, 7.5f, true, true);
    else state = std::make_unique<gomoku::GomokuState>(bs, false, false, 1, false);
    mcts::TranspositionTable tt(1048576);
    mcts::MCTSConfig cfg;
    cfg.numThreads = 1;
    cfg.numSimulations = sims;
    cfg.cPuct = cpuct;
    cfg.fpuReduction = fpu;
    cfg.useBatchInference = false;   // no BatchQueue (Mode S); flipped on by setDeterministicMode
    cfg.useBatchedMCTS = false;
    cfg.useDirichletNoise = noiseEachSearch != 0;
    std::unique_ptr<nn::NeuralNetwork> net;
    HashEvaluator* he = nullptr; CountingRandom* rn = nullptr;
    if (evalKind == "hash") { he = new HashEvaluator(); net.reset(he); }
    else { rn = new CountingRandom(bs, evalSeed); net.reset(rn); }
    mcts::ParallelMCTS m(*state, cfg, net.get(), &tt);
    m.setDeterministicMode(true);
    const float alpha = 0.03f, eps = 0.25f;
    m.addDirichletNoise(alpha, eps);
    std::ostream& o = std::cout;
    o << "{\"mode\":\"" << (go ? "go_game" : "game") << "\",\"bs\":" << bs << ",\"sims\":" << sims << ",\"eval\":\"" << evalKind
      << "\",\"eval_seed\":" << evalSeed << ",\"noise_each_search\":" << noiseEachSearch
      << ",\"cpuct_bits\":" << fbits(cpuct) << ",\"fpu_bits\":" << fbits(fpu)
      << ",\"init_root\":";
    dump_node_children(o, m.rootNode_.get());
    o << ",\"moves\":[";
    int moveNum = 0;
    while (!state->isTerminal() && moveNum < maxMoves) {
        m.search();
        float T = moveNum >= 30 ? 0.0f : 1.0f;
        auto probs = m.getActionProbabilities(T);
        auto* root = m.rootNode_.get();
        std::ostringstream kids; dump_node_children(kids, root);
        int rootN = root->visitCount.load(), rootVL = root->virtualLoss.load();
        uint32_t rootW = fbits(root->valueSum.load());
        int action = m.selectAction(true, T);
        float value = m.getRootValue();
        if (moveNum) o << ",";
        o << "{\"ply\":" << moveNum << ",\"root\":[" << rootN << "," << rootVL << "," << rootW << "],\"children\":"
          << kids.str() << ",\"probs\":[";
        for (size_t i = 0; i < probs.size(); ++i) o << (i ? "," : "") << fbits(probs[i]);
        o << "],\"action\":" << action << ",\"value\":" << fbits(value)
          << ",\"tt_lookups\":" << tt.getLookups() << ",\"tt_hits\":" << tt.getHits()
          << ",\"evals\":" << (he ? he->calls : rn->calls) << "}";
        state->makeMove(action);
        m.updateWithMove(action);
        if (moveNum % 2 == 0) m.addDirichletNoise(alpha, eps);
        ++moveNum;
    }
    o << "],\"terminal\":" << (state->isTerminal() ? 1 : 0) << ",\"result\":" << (int)state->getGameResult()
      << ",\"tt_entries\":" << tt.getEntryCount() << "}\n";
    return 0;
}

static int run_positions(int bs, int count, unsigned seed) {
    std::mt19937 g(seed);
    std::ostream& o = std::cout;
    o << "{\"mode\":\"positions\",\"bs\":" << bs << ",\"positions\":[";
    for (int k = 0; k < count; ++k) {
        gomoku::GomokuState s(bs, false, false, 1, false);
        int target = (int)(g() % (unsigned)(bs * bs + 1));
        std::vector<int> moves;
        // Fresh-state legal order (first query grows the unordered_set from 1 bucket).
        std::vector<int> firstOrder = s.getLegalMoves();
        while ((int)moves.size() < target && !s.isTerminal()) {
            auto legal = s.getLegalMoves();
            int a = legal[g() % legal.size()];
            s.makeMove(a);
            moves.push_back(a);
        }
        auto planes = s.getEnhancedTensorRepresentation();
        if (k) o << ",";
        o << "{\"moves\":[";
        for (size_t i = 0; i < moves.size(); ++i) o << (i ? "," : "") << moves[i];
        o << "],\"hash\":\"" << s.getHash() << "\",\"terminal\":" << (s.isTerminal() ? 1 : 0)
          << ",\"result\":" << (int)s.getGameResult() << ",\"player\":" << s.getCurrentPlayer() << ",\"legal\":[";
        auto legal = s.getLegalMoves();
        for (size_t i = 0; i < legal.size(); ++i) o << (i ? "," : "") << legal[i];
        o << "],\"first_order\":[";
        if (k == 0) for (size_t i = 0; i < firstOrder.size(); ++i) o << (i ? "," : "") << firstOrder[i];
        o << "],\"planes\":[";
        bool first = true;
        for (size_t p = 0; p < planes.size(); ++p)
            for (int x = 0; x < bs; ++x)
                for (int y = 0; y < bs; ++y) {
                    float v = planes[p][x][y];
                    if (v != 0.0f) {
                        o << (first ? "" : ",") << "[" << (p * bs * bs + x * bs + y) << "," << fbits(v) << "]";
                        first = false;
                    }
                }
        o << "],\"nplanes\":" << planes.size() << "}";
    }
    o << "]}\n";
    return 0;
}

// GoState positions: random legal play (passes included, weight 1/16) from the empty board.
static int run_go_positions(int bs, int count, unsigned seed) {
    std::mt19937 g(seed);
    std::ostream& o = std::cout;
    o << "{\"mode\":\"go_positions\",\"bs\":" << bs << ",\"positions\":[";
    for (int k = 0; k < count; ++k) {
        go::GoState s(bs, 7.5f, true, true);
        int target = (int)(g() % (unsigned)(2 * bs * bs));
        std::vector<int> moves;
        while ((int)moves.size() < target && !s.isTerminal()) {
            auto legal = s.getLegalMoves();
            int a = (g() % 16 == 0) ? -1 : legal[1 + g() % (legal.size() - 1 > 0 ? legal.size() - 1 : 1)];
            if (legal.size() == 1) a = -1;
            s.makeMove(a);
            moves.push_back(a);
        }
        auto planes = s.getEnhancedTensorRepresentation();
        auto sc = s.calculateScore();
        if (k) o << ",";
        o << "{\"moves\":[";
        for (size_t i = 0; i < moves.size(); ++i) o << (i ? "," : "") << moves[i];
        o << "],\"hash\":\"" << s.getHash() << "\",\"terminal\":" << (s.isTerminal() ? 1 : 0)
          << ",\"result\":" << (int)s.getGameResult() << ",\"player\":" << s.getCurrentPlayer()
          << ",\"ko\":" << s.getKoPoint() << ",\"captured\":[" << s.getCapturedStones(1) << "," << s.getCapturedStones(2)
          << "],\"score\":[" << fbits(sc.first) << "," << fbits(sc.second) << "],\"legal\":[";
        auto legal = s.getLegalMoves();
        for (size_t i = 0; i < legal.size(); ++i) o << (i ? "," : "") << legal[i];
        o << "],\"board\":[";
        for (int a = 0; a < bs * bs; ++a) o << (a ? "," : "") << s.getStone(a);
        o << "],\"planes\":[";
        bool first = true;
        for (size_t p = 0; p < planes.size(); ++p)
            for (int y = 0; y < bs; ++y)
                for (int x = 0; x < bs; ++x) {
                    float v = planes[p][y][x];
                    if (v != 0.0f) {
                        o << (first ? "" : ",") << "[" << (p * bs * bs + y * bs + x) << "," << fbits(v) << "]";
                        first = false;
                    }
                }
        o << "],\"nplanes\":" << planes.size() << "}";
    }
    o << "]}\n";
    return 0;
}

static int run_gamma(float alpha, int n, int calls) {
    std::mt19937 rng(42);
    std::ostream& o = std::cout;
    o << "{\"mode\":\"gamma\",\"alpha_bits\":" << fbits(alpha) << ",\"calls\":[";
    for (int c = 0; c < calls; ++c) {
        std::gamma_distribution<float> gamma(alpha, 1.0f);   // fresh object per call, as addDirichletNoise
        if (c) o << ",";
        o << "[";
        for (int i = 0; i < n; ++i) o << (i ? "," : "") << fbits(gamma(rng));
        o << "]";
    }
    o << "]}\n";
    return 0;
}

// ParallelMCTS public API beyond the playSingleGame loop (include/alphazero/mcts/parallel_mcts.h:
// 155-159,162-163,198): a script of operations on one tree, with the root statistics after each.
//   n  runSingleSimulation()            b  runBatchedSearch()         s  search()
//   r<k> releaseMemory(k) (returns the pruned node count)
//   d  stochastic selection: setConfig with useBatchInference = false (the rng keeps the state
//      setDeterministicMode(true) seeded, 42), so selectAction samples on rng_
//   a<T> selectAction(true, T)          e<T> selectAction(false, T)
//   m  play the last selected action (state.makeMove + updateWithMove)   x  addDirichletNoise
static int run_api(int bs, int sims, const std::string& script, const std::string& evalKind, unsigned evalSeed) {
    gomoku::GomokuState state(bs, false, false, 1, false);
    mcts::TranspositionTable tt(1048576);
    mcts::MCTSConfig cfg;
    cfg.numThreads = 1;
    cfg.numSimulations = sims;
    cfg.useBatchInference = false;
    cfg.useBatchedMCTS = false;
    std::unique_ptr<nn::NeuralNetwork> net;
    if (evalKind == "hash") net.reset(new HashEvaluator());
    else net.reset(new CountingRandom(bs, evalSeed));
    mcts::ParallelMCTS m(state, cfg, net.get(), &tt);
    m.setDeterministicMode(true);
    std::ostream& o = std::cout;
    o << "{\"mode\":\"api\",\"bs\":" << bs << ",\"sims\":" << sims << ",\"eval\":\"" << evalKind << "\",\"eval_seed\":"
      << evalSeed << ",\"script\":\"" << script << "\",\"ops\":[";
    int last = -1;
    size_t i = 0;
    bool firstOp = true;
    while (i < script.size()) {
        const char op = script[i++];
        std::string arg;
        while (i < script.size() && script[i] != ',') arg += script[i++];
        if (i < script.size()) ++i;
        long long ret = 0;
        if (op == 'n') m.runSingleSimulation();
        else if (op == 'b') m.runBatchedSearch();
        else if (op == 's') m.search();
        else if (op == 'r') ret = (long long)m.releaseMemory(std::atoi(arg.c_str()));
        else if (op == 'd') { mcts::MCTSConfig c = m.config_; c.useBatchInference = false; m.setConfig(c); }
        else if (op == 'a') ret = last = m.selectAction(true, (float)std::atof(arg.c_str()));
        else if (op == 'e') ret = last = m.selectAction(false, (float)std::atof(arg.c_str()));
        else if (op == 'm') { state.makeMove(last); m.updateWithMove(last); ret = last; }
        else if (op == 'x') m.addDirichletNoise(0.03f, 0.25f);
        else { std::fprintf(stderr, "bad op %c\n", op); return 2; }
        auto* root = m.rootNode_.get();
        if (!firstOp) o << ",";
        firstOp = false;
        o << "{\"op\":\"" << op << arg << "\",\"ret\":" << ret << ",\"root\":[" << root->visitCount.load() << ","
          << root->virtualLoss.load() << "," << fbits(root->valueSum.load()) << "],\"children\":";
        dump_node_children(o, root);
        o << "}";
    }
    o << "]}\n";
    o.flush();
    // ~ParallelMCTS deletes a borrowed TT unless useBatchInference: this one is on the stack
    m.config_.useBatchInference = true;
    return 0;
}

int main(int argc, char** argv) {
    if (argc < 2) { std::fprintf(stderr, "usage: ref_harness game|positions|gamma|go_positions|go_game ...\n"); return 2; }
    std::string mode = argv[1];
    auto I = [&](int i, int d) { return argc > i ? std::atoi(argv[i]) : d; };
    auto F = [&](int i, float d) { return argc > i ? (float)std::atof(argv[i]) : d; };
    if (mode == "game")
        return run_game(I(2, 9), I(3, 100), I(4, 1000), argc > 5 ? argv[5] : "hash", (unsigned)I(6, 7), I(7, 0),
                        F(8, 1.5f), F(9, 0.0f));
    if (mode == "positions") return run_positions(I(2, 9), I(3, 16), (unsigned)I(4, 1));
    if (mode == "gamma") return run_gamma(F(2, 0.03f), I(3, 81), I(4, 4));
    if (mode == "go_positions") return run_go_positions(I(2, 9), I(3, 16), (unsigned)I(4, 1));
    if (mode == "api") return run_api(I(2, 9), I(3, 50), argc > 4 ? argv[4] : "s", argc > 5 ? argv[5] : "hash", (unsigned)I(6, 7));
    if (mode == "go_game")
        return run_game(I(2, 9), I(3, 100), I(4, 1000), argc > 5 ? argv[5] : "hash", (unsigned)I(6, 7), I(7, 0),
                        F(8, 1.5f), F(9, 0.0f), true);
    std::fprintf(stderr, "unknown mode\n");
    return 2;
}
