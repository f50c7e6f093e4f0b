// alphazero/nn/hip_neural_network.h -- NeuralNetwork backed by the MI355X ConvNet
// (az_net_* in include/az_engine.h).  predictBatch has TorchNeuralNetwork::predictBatch
// semantics (torch_neural_network.cpp:224-363): policy = softmax over A, value [B].
#pragma once
#include <mutex>

#include "alphazero/nn/neural_network.h"
#include "az_engine.h"

namespace alphazero {
namespace nn {

// One engine per HIP device, shared by every handle of the process (device = LOCAL_RANK or 0
// unless given).
az_engine* engineForDevice(int device = -1);

struct NetShape {
    int boardSize = 15, inPlanes = 11, channels = 256, blocks = 20, actionSize = 225;
    int headChannels = 32, pool = 8, fcHidden = 256, residual = 1, convBias = 0;
    int precision = AZ_PREC_FP16, maxBatch = 2048;
    int randWire = 0;   // 1: DDWRandWireResNet trunk (az_net_create_randwire; not part of the .azw header)
};

class HipNeuralNetwork : public NeuralNetwork {
 public:
    HipNeuralNetwork(const NetShape& shape, int device = -1);
    ~HipNeuralNetwork() override;
    HipNeuralNetwork(const HipNeuralNetwork&) = delete;
    HipNeuralNetwork& operator=(const HipNeuralNetwork&) = delete;

    void loadWeights(const std::vector<float>& blob);   // torch state_dict order, no num_batches_tracked
    void initRandom(uint64_t seed);                      // counter-based init (oracle/net_oracle.init_blob)
    void setPrecision(int precision);
    // .azw file: "AZW1", 12 int32 NetShape fields, uint64 count, float32[count]
    static std::unique_ptr<HipNeuralNetwork> load(const std::string& path, int device = -1);
    // The reference's own model file: a TorchScript archive of its plain ResNet (SimplifiedModel /
    // the exporter fallback; torch_neural_network.cpp:90 loads it with torch::jit::load), read
    // without executing it (alphazero/nn/torchscript_reader.h).  precision: AZ_PREC_* of the trunk
    // (-1: fp32-faithful, the reference's default fp32 inference -- AZ_PREC_F16X3 where its kernels
    // exist, else AZ_PREC_BF16X3 where the trunk has 16-bit kernels, else AZ_PREC_F32);
    // boardSize <= 0: from the policy size.  With precision -1 a net whose activations leave the
    // fp16 range (AZ_ERR_RANGE from an F16X3 forward) is switched to AZ_PREC_BF16X3 (fp32 range) and
    // the forward repeated, so predictBatch never fails on it.
    static std::unique_ptr<HipNeuralNetwork> loadTorchScript(const std::string& path, core::GameType type,
                                                             int boardSize = 0, int precision = -1,
                                                             int maxBatch = 2048, int device = -1);
    // TorchNeuralNetwork::createDDWRandWireResNet (torch_neural_network.cpp:799-814): the
    // DDW-RandWire net (ddw_randwire_resnet.cpp:387-468) on the device engine, fp32 path
    static std::unique_ptr<HipNeuralNetwork> createDDWRandWireResNet(int inputChannels, int outputSize,
                                                                     int channels = 128, int numBlocks = 20,
                                                                     int boardSize = 15, int maxBatch = 256,
                                                                     int device = -1);
    void save(const std::string& path) const;

    std::pair<std::vector<float>, float> predict(const core::IGameState& state) override;
    void predictBatch(const std::vector<std::reference_wrapper<const core::IGameState>>& states,
                      std::vector<std::vector<float>>& policies, std::vector<float>& values) override;
    std::future<std::pair<std::vector<float>, float>> predictAsync(const core::IGameState& state) override;
    bool isGpuAvailable() const override { return true; }
    std::string getDeviceInfo() const override;
    float getInferenceTimeMs() const override { return lastMs_; }
    int getBatchSize() const override { return shape_.maxBatch; }
    std::string getModelInfo() const override;
    size_t getModelSizeBytes() const override { return params_ * sizeof(float); }
    void benchmark(int numIterations = 100, int batchSize = 16) override;
    void enableDebugMode(bool enable) override { debug_ = enable; }
    void printModelSummary() const override;

    // after a weight broadcast into this net (selfplay::Distributed): the host copy of the blob
    void refreshHostWeights();
    // the precision was chosen at load (loadTorchScript, precision -1) and the trunk is F16X3:
    // switch to AZ_PREC_BF16X3 (the fp32 range) and return true -- what predictBatch does on
    // AZ_ERR_RANGE, for callers that run the net inside the engine (SelfPlayManager::generateGames)
    bool fallbackToFp32Range();

    az_net* handle() const { return net_; }
    az_engine* engine() const { return eng_; }
    const NetShape& shape() const { return shape_; }

 private:
    NetShape shape_;
    az_engine* eng_ = nullptr;
    az_net* net_ = nullptr;
    size_t params_ = 0;
    std::vector<float> blob_;
    float lastMs_ = 0.0f;
    bool debug_ = false;
    bool autoPrecision_ = false;   // loadTorchScript chose the precision: F16X3 falls back to BF16X3 on AZ_ERR_RANGE
    std::mutex mu_;
};

}  // namespace nn
}  // namespace alphazero
