// alphazero/nn/random_policy_network.h -- RandomPolicyNetwork (src/nn/random_policy_network.cpp
// semantics): policy 0.001 everywhere, U[0,1) on the legal moves in child order, normalised;
// value U[-0.1, 0.1).  Inside ParallelMCTS / SelfPlayManager it runs on the device
// (AZ_EVAL_RANDOM, one mt19937(seed + game) per game); predict() here is the host version.
#pragma once
#include <random>

#include "alphazero/nn/neural_network.h"

namespace alphazero {
namespace nn {

class RandomPolicyNetwork : public NeuralNetwork {
 public:
    RandomPolicyNetwork(core::GameType gameType, int boardSize = 0, unsigned int seed = 0);
    std::pair<std::vector<float>, float> predict(const core::IGameState& state) override;
    void predictBatch(const std::vector<std::reference_wrapper<const core::IGameState>>& states,
                      std::vector<std::vector<float>>& policies, std::vector<float>& values) override;
    std::future<std::pair<std::vector<float>, float>> predictAsync(const core::IGameState& state) override;
    bool isGpuAvailable() const override { return false; }
    std::string getDeviceInfo() const override { return "device evaluator (AZ_EVAL_RANDOM)"; }
    float getInferenceTimeMs() const override { return 0.0f; }
    int getBatchSize() const override { return 128; }
    std::string getModelInfo() const override { return "Random policy network"; }
    size_t getModelSizeBytes() const override { return 0; }
    void benchmark(int, int) override {}
    void enableDebugMode(bool) override {}
    void printModelSummary() const override {}
    unsigned int seed() const { return seed_; }

 private:
    core::GameType gameType_;
    int boardSize_;
    unsigned int seed_;
    std::mt19937 rng_;
};

}  // namespace nn
}  // namespace alphazero
