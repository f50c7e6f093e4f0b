// alphazero/mcts/parallel_mcts.h -- ParallelMCTS of the host API on the MI355X engine.
// One tree (one az_search game slot) per object; search() runs the Mode S simulations of
// parallel_mcts.cpp:276-380 on the device, bit-exact with the reference
// for the hash / random / uniform evaluators.  selectAction follows MCTSConfig::useBatchInference
// as the reference does: the deterministic rules (forced by setDeterministicMode and by
// SelfPlayManager) or libstdc++ draws on rng_ (parallel_mcts.cpp:987-1047).  numThreads / batch
// settings are accepted and ignored (the device runs one simulation per game per step, Mode S).
#pragma once
#include <atomic>
#include <functional>
#include <memory>
#include <string>
#include <tuple>
#include <vector>

#include "alphazero/core/igamestate.h"
#include "alphazero/mcts/mcts_node.h"
#include "alphazero/mcts/transposition_table.h"
#include "alphazero/mcts/search_group.h"
#include "alphazero/nn/neural_network.h"
#include "az_engine.h"

namespace alphazero {
namespace mcts {

enum class MCTSNodeSelection { UCB, PUCT, PROGRESSIVE_BIAS, RAVE };
enum class MCTSSearchMode { SERIAL, PARALLEL, BATCHED };

struct MCTSConfig {
    int numThreads = 1;
    int numSimulations = 800;
    float cPuct = 1.5f;
    float fpuReduction = 0.0f;
    int virtualLoss = 3;
    int maxSearchDepth = 1000;
    bool useDirichletNoise = false;
    float dirichletAlpha = 0.03f;
    float dirichletEpsilon = 0.25f;
    bool useBatchInference = false;
    bool useTemporalDifference = false;
    float tdLambda = 0.8f;
    bool useProgressiveWidening = false;
    int minVisitsForWidening = 10;
    float progressiveWideningBase = 2.0f;
    float progressiveWideningExponent = 0.5f;
    MCTSNodeSelection selectionStrategy = MCTSNodeSelection::PUCT;
    int maxRetries = 3;
    int transpositionTableSize = 1048576;
    uint64_t cacheEntryMaxAge = 60000;
    bool useFmapCache = false;
    int batchSize = 16;
    bool useBatchedMCTS = false;
    int batchTimeoutMs = 5;
    MCTSSearchMode searchMode = MCTSSearchMode::PARALLEL;
    bool pinThreads = false;
    bool deterministic = false;
    int cacheSize = 2097152;
};

struct MCTSStats {
    std::atomic<size_t> nodesCreated{0}, nodesExpanded{0}, nodesTotalVisits{0}, simulationCount{0};
    std::atomic<size_t> evaluationCalls{0}, cacheHits{0}, cacheMisses{0}, batchedEvaluations{0}, totalBatches{0};
};

// The device evaluator a NeuralNetwork* maps to: HipNeuralNetwork -> AZ_EVAL_NET,
// RandomPolicyNetwork(seed) -> AZ_EVAL_RANDOM, nullptr -> AZ_EVAL_UNIFORM, any other subclass ->
// AZ_EVAL_CALLBACK (the device search hands each simulation step's leaves to the subclass's
// predict / predictBatch on the calling thread).
struct DeviceEvaluator {
    int kind;
    unsigned seed;
    az_net* net;
    az_engine* engine;
};
DeviceEvaluator deviceEvaluator(nn::NeuralNetwork* nn);

class ParallelMCTS {
 public:
    ParallelMCTS(const core::IGameState& rootState, nn::NeuralNetwork* nn = nullptr, TranspositionTable* tt = nullptr,
                 int numThreads = 1, int numSimulations = 800, float cPuct = 1.5f, float fpuReduction = 0.0f,
                 int virtualLoss = 3);
    ParallelMCTS(const core::IGameState& rootState, const MCTSConfig& config, nn::NeuralNetwork* nn = nullptr,
                 TranspositionTable* tt = nullptr);
    // A member of `group` (alphazero/mcts/search_group.h): plays in a slot of the group's handle
    // with the group's evaluator and configuration; concurrent search() calls of members batch.
    ParallelMCTS(const core::IGameState& rootState, SearchGroup& group);
    ~ParallelMCTS();
    ParallelMCTS(const ParallelMCTS&) = delete;
    ParallelMCTS& operator=(const ParallelMCTS&) = delete;

    void search();
    void runSingleSimulation();                      // parallel_mcts.cpp:276-380
    void runBatchedSearch();                         // :1531-1590 (numSimulations single simulations)
    int selectAction(bool isTraining = false, float temperature = 1.0f);
    std::vector<float> getActionProbabilities(float temperature = 1.0f) const;   // child order
    std::vector<int> getChildActions() const;                                    // matching actions
    float getRootValue() const;
    void updateWithMove(int action);
    void addDirichletNoise(float alpha = 0.03f, float epsilon = 0.25f);

    void setNumThreads(int n) { config_.numThreads = n; }
    void setNumSimulations(int n);
    void setCPuct(float c);
    void setFpuReduction(float f);
    void setVirtualLoss(int v);
    void setNeuralNetwork(nn::NeuralNetwork* nn);
    void setTranspositionTable(TranspositionTable* tt);
    void setSelectionStrategy(MCTSNodeSelection s) { config_.selectionStrategy = s; }
    void setConfig(const MCTSConfig& config);
    void enableBatchedMCTS(bool enable) { config_.useBatchedMCTS = enable; }
    void setBatchSize(int b) { config_.batchSize = b; }
    void setBatchTimeout(int ms) { config_.batchTimeoutMs = ms; }
    void setDeterministicMode(bool enable);
    void setDebugMode(bool enable) { debug_ = enable; }
    void setProgressCallback(std::function<void(int, int)> cb) { progress_ = std::move(cb); }
    void printSearchStats() const;
    std::string getSearchInfo() const;
    void printSearchPath(int action) const;
    size_t getMemoryUsage() const;
    size_t releaseMemory(int visitThreshold = 10);   // :1481-1496 (MCTSNode::pruneTree)
    // Extension: a host snapshot of the root and its children (the reference keeps rootNode_ private)
    MCTSNode getRootNode() const;
    std::vector<std::tuple<int, int, float, float>> analyzePosition(int topN = 10) const;   // (action, N, Q, P)
    const MCTSStats& getStats() const { return stats_; }
    az_search* handle() const { return s_; }
    int slot() const { return slot_; }                       // the game slot of handle()
    bool inGroup() const { return group_ != nullptr; }

 private:
    void rebuild();           // (re)create the device search for the current config / root (leaves a group)
    void applyConfig();       // new parameters in place (tree kept), or rebuild
    static int hostEvaluate(void* user, int n, const int* games, const int* pathLen, const int* moves, int maxPath,
                            const float* planes, int nPlanes, float* policy, float* value);
    az_search_cfg deviceConfig() const;
    MCTSConfig config_;
    nn::NeuralNetwork* nn_;
    TranspositionTable* tt_;
    std::unique_ptr<core::IGameState> root_;
    az_search* s_ = nullptr;
    SearchGroup* group_ = nullptr;   // member of a group: s_ is the group's handle, slot_ the game
    int slot_ = 0;
    std::vector<uint8_t> slotMask() const;
    struct RootSelect {
        std::vector<float> probs;
        std::vector<int> actions;
        float value = 0.0f;
    };
    RootSelect rootSelect(float temperature) const;
    MCTSStats stats_;
    bool debug_ = false;
    bool searched_ = false;
    std::function<void(int, int)> progress_;
};

}  // namespace mcts
}  // namespace alphazero
