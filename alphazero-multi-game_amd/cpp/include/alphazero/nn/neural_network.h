// alphazero/nn/neural_network.h -- the evaluator plugin interface of the host API, with the
// reference's virtuals (include/alphazero/nn/neural_network.h:20-132) so existing callers
// (ParallelMCTS, SelfPlayManager, user code) compile unchanged.
#pragma once
#include <functional>
#include <future>
#include <memory>
#include <string>
#include <vector>

#include "alphazero/core/igamestate.h"

namespace alphazero {
namespace nn {

class NeuralNetwork {
 public:
    virtual ~NeuralNetwork() = default;
    virtual std::pair<std::vector<float>, float> predict(const core::IGameState& state) = 0;
    virtual void predictBatch(const std::vector<std::reference_wrapper<const core::IGameState>>& states,
                              std::vector<std::vector<float>>& policies, std::vector<float>& values) = 0;
    virtual std::future<std::pair<std::vector<float>, float>> predictAsync(const core::IGameState& state) = 0;
    virtual bool isGpuAvailable() const = 0;
    virtual std::string getDeviceInfo() const = 0;
    virtual float getInferenceTimeMs() const = 0;
    virtual int getBatchSize() const = 0;
    virtual std::string getModelInfo() const = 0;
    virtual size_t getModelSizeBytes() const = 0;
    virtual void benchmark(int numIterations = 100, int batchSize = 16) = 0;
    virtual void enableDebugMode(bool enable) = 0;
    virtual void printModelSummary() const = 0;

    // modelPath: an .azw weight file (tools/export_azw.py), or the reference's TorchScript model
    // file of its plain ResNet (read without executing it, HipNeuralNetwork::loadTorchScript) ->
    // HipNeuralNetwork on the MI355X engine; "random" / "" -> RandomPolicyNetwork.  useGpu=false
    // is refused (no CPU path).
    static std::unique_ptr<NeuralNetwork> create(const std::string& modelPath, core::GameType gameType,
                                                 int boardSize = 0, bool useGpu = true);
};

}  // namespace nn
}  // namespace alphazero
