// alphazero/selfplay/self_play_manager.h -- SelfPlayManager of the host API.  generateGames
// runs every game on the MI355X engine through az_selfplay_run (many games per device step,
// the playSingleGame loop of self_play_manager.cpp:151-240 per game) instead of a host thread
// pool; records, progress callbacks, saved files and counters keep the reference's meaning.
#pragma once
#include <atomic>
#include <functional>
#include <string>
#include <vector>

#include "alphazero/mcts/parallel_mcts.h"
#include "alphazero/nn/neural_network.h"
#include "alphazero/selfplay/game_record.h"

namespace alphazero {
namespace selfplay {

class Distributed;

// Contiguous global game ids of one rank of a per-GPU job (the first total % world ranks take one
// more) and the noise seed that keeps every game's record independent of the rank count (seed +
// global id): shardGames() in distributed.h, SelfPlayManager::setShard.
struct GameShard {
    int firstGame = 0, numGames = 0;
    unsigned noiseSeed = 42;
};

// Job-wide counters of a sharded run, reduced over the ranks (RCCL) after generateGames.
struct JobStats {
    long long gamesCompleted = 0, totalMoves = 0;
    double seconds = 0.0;          // the slowest rank's generateGames time
};

class SelfPlayManager {
 public:
    // numThreads is kept for the signature; concurrency is the device slot count
    // (setConcurrentGames, default min(numGames, 2048)).  setBatchConfig(batchSize, ...) caps the
    // network batch of a simulation step -- one leaf per game slot -- at batchSize slots (the
    // BatchQueue's batch size, self_play_manager.cpp:133-136, 162-173).
    SelfPlayManager(nn::NeuralNetwork* neuralNetwork, int numGames = 100, int numSimulations = 800,
                    int numThreads = 4);
    ~SelfPlayManager();

    std::vector<GameRecord> generateGames(core::GameType gameType, int boardSize = 0, bool useVariantRules = false);
    void setExplorationParams(float dirichletAlpha = 0.03f, float dirichletEpsilon = 0.25f,
                              float initialTemperature = 1.0f, int temperatureDropMove = 30,
                              float finalTemperature = 0.0f);
    void setProgressCallback(std::function<void(int, int, int, int)> callback) { progress_ = std::move(callback); }
    void setBatchConfig(int batchSize, int batchTimeoutMs) {
        batchSize_ = batchSize; batchTimeoutMs_ = batchTimeoutMs; batchSet_ = true;
    }
    void setSaveGames(bool saveGames, const std::string& outputDir = "games");
    void setAbort(bool abort) { abort_ = abort ? 1 : 0; }
    bool isRunning() const { return running_; }
    void setMctsConfig(const mcts::MCTSConfig& config);
    int getCompletedGamesCount() const { return completed_; }
    int getTotalMovesCount() const { return totalMoves_; }
    float getTemperature(int moveNum) const { return moveNum >= tempDrop_ ? tFinal_ : tInit_; }

    // engine extensions
    // one rank's share of a per-GPU job: its games are the global ids [firstGame, firstGame +
    // numGames) (record file names, noise / evaluator seeds); numGames replaces the constructor's
    void setShard(const GameShard& s) {
        numGames_ = s.numGames; firstGame_ = s.firstGame; noiseSeed_ = s.noiseSeed; noiseStride_ = 1;
    }
    int getFirstGameId() const { return firstGame_; }
    // with a communicator, generateGames ends by reducing the job's counters over the ranks
    // (every rank must call generateGames); getJobStats() then holds them
    void setDistributed(Distributed* d) { dist_ = d; }
    const JobStats& getJobStats() const { return job_; }
    void setConcurrentGames(int n) { slots_ = n; }
    void setMaxMoves(int n) { maxMoves_ = n; }
    void setSeeds(unsigned noiseSeed, int noiseSeedStride) { noiseSeed_ = noiseSeed; noiseStride_ = noiseSeedStride; }
    // Evaluation log (tests: a game replayed through the CPU oracle): every network evaluation of device
    // slot `slot` (the game id while the games fit the slots) -- post-softmax policy [NA], value, feature
    // planes [C][A] -- up to `capacity` evaluations, read after generateGames; capacity 0 turns it off.
    void setEvalLog(int slot, int capacity) { logSlot_ = capacity > 0 ? slot : -1; logCap_ = capacity; }
    struct EvalLog {
        int count = 0, policySize = 0, planes = 0, cells = 0;
        std::vector<float> policy, value, features;   // [count][policySize], [count], [count][planes][cells]
    };
    const EvalLog& getEvalLog() const { return log_; }

 private:
    int runGames(core::GameType type, int bs, bool variant, std::vector<GameRecord>& records, std::vector<char>& done,
                 std::vector<std::string>& written);

    nn::NeuralNetwork* nn_;
    int numGames_, numSimulations_, numThreads_;
    float alpha_ = 0.03f, eps_ = 0.25f, tInit_ = 1.0f, tFinal_ = 0.0f;
    int tempDrop_ = 30;
    int batchSize_ = 16, batchTimeoutMs_ = 5;
    bool save_ = false;
    std::string outDir_ = "games";
    mcts::MCTSConfig mcts_;
    std::function<void(int, int, int, int)> progress_;
    volatile int abort_ = 0;
    std::atomic<bool> running_{false};
    std::atomic<int> completed_{0}, totalMoves_{0};
    int slots_ = 0, maxMoves_ = 0;
    bool batchSet_ = false;
    unsigned noiseSeed_ = 42;
    int noiseStride_ = 1;
    int logSlot_ = -1, logCap_ = 0;
    EvalLog log_;
    int firstGame_ = 0;
    Distributed* dist_ = nullptr;
    JobStats job_;
};

}  // namespace selfplay
}  // namespace alphazero
