// NeuralNetwork plugins of the host API: HipNeuralNetwork (the MI355X ConvNet behind
// az_net_*), RandomPolicyNetwork, the factory, and the per-device engine registry.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <map>
#include <mutex>
#include <sstream>

#include "alphazero/games/go/go_state.h"
#include "alphazero/games/gomoku/gomoku_state.h"
#include "alphazero/nn/hip_neural_network.h"
#include "alphazero/nn/torchscript_reader.h"
#include "alphazero/nn/random_policy_network.h"

namespace alphazero {
namespace nn {

static void check(int rc, const char* what) {
    if (rc != 0) throw std::runtime_error(std::string(what) + ": " + az_last_error());
}

az_engine* engineForDevice(int device) {
    static std::mutex mu;
    static std::map<int, az_engine*> engines;
    if (device < 0) {
        const char* lr = std::getenv("LOCAL_RANK");
        device = lr ? std::atoi(lr) : 0;
    }
    std::lock_guard<std::mutex> lk(mu);
    auto it = engines.find(device);
    if (it != engines.end()) return it->second;
    az_engine* e = nullptr;
    check(az_engine_create(device, &e), "az_engine_create");
    engines[device] = e;   // process lifetime
    return e;
}

static az_net_desc toDesc(const NetShape& s) {
    return az_net_desc{s.boardSize, s.inPlanes, s.channels, s.blocks, s.actionSize, s.headChannels, s.pool,
                       s.fcHidden, s.residual, s.convBias, s.precision, s.maxBatch};
}

HipNeuralNetwork::HipNeuralNetwork(const NetShape& shape, int device) : shape_(shape) {
    eng_ = engineForDevice(device);
    az_net_desc d = toDesc(shape_);
    if (shape_.randWire) check(az_net_create_randwire(eng_, &d, &net_), "az_net_create_randwire");
    else check(az_net_create(eng_, &d, &net_), "az_net_create");
    check(az_net_num_params(net_, &params_), "az_net_num_params");
}

HipNeuralNetwork::~HipNeuralNetwork() {
    if (net_) az_net_destroy(net_);
}

void HipNeuralNetwork::refreshHostWeights() {
    std::lock_guard<std::mutex> lk(mu_);
    blob_.resize(params_);
    check(az_net_get_weights(net_, blob_.data(), blob_.size()), "az_net_get_weights");
}

bool HipNeuralNetwork::fallbackToFp32Range() {
    std::lock_guard<std::mutex> lk(mu_);
    if (!autoPrecision_ || shape_.precision != AZ_PREC_F16X3) return false;
    check(az_net_set_precision(net_, AZ_PREC_BF16X3), "az_net_set_precision");
    shape_.precision = AZ_PREC_BF16X3;
    return true;
}

void HipNeuralNetwork::loadWeights(const std::vector<float>& blob) {
    std::lock_guard<std::mutex> lk(mu_);
    check(az_net_load_weights(net_, blob.data(), blob.size()), "az_net_load_weights");
    blob_ = blob;
}

void HipNeuralNetwork::initRandom(uint64_t seed) {
    std::lock_guard<std::mutex> lk(mu_);
    check(az_net_init_random(net_, seed), "az_net_init_random");
    blob_.clear();
}

void HipNeuralNetwork::setPrecision(int p) {
    std::lock_guard<std::mutex> lk(mu_);
    check(az_net_set_precision(net_, p), "az_net_set_precision");
    shape_.precision = p;
}

static const char kMagic[4] = {'A', 'Z', 'W', '1'};

std::unique_ptr<HipNeuralNetwork> HipNeuralNetwork::load(const std::string& path, int device) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error("cannot open weight file " + path);
    char magic[4];
    int32_t v[12];
    uint64_t count = 0;
    f.read(magic, 4);
    f.read(reinterpret_cast<char*>(v), sizeof v);
    f.read(reinterpret_cast<char*>(&count), 8);
    if (!f || std::memcmp(magic, kMagic, 4) != 0) throw std::runtime_error(path + ": not an AZW1 weight file");
    NetShape s{v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], v[8], v[9], v[10], v[11]};
    std::vector<float> blob(count);
    f.read(reinterpret_cast<char*>(blob.data()), (std::streamsize)(count * 4));
    if (!f) throw std::runtime_error(path + ": truncated weight file");
    auto net = std::make_unique<HipNeuralNetwork>(s, device);
    net->loadWeights(blob);
    return net;
}

std::unique_ptr<HipNeuralNetwork> HipNeuralNetwork::loadTorchScript(const std::string& path, core::GameType type,
                                                                   int boardSize, int precision, int maxBatch, int device) {
    NetShape s;
    s.maxBatch = maxBatch;
    s.precision = precision;
    std::vector<float> blob = torchScriptResNet(path, type, boardSize, s);
    if (precision < 0) {
        // the fp32-faithful trunk: fp16 pieces where their kernels exist (include/az_engine.h
        // AZ_PREC_F16X3: conv3x3_v9x3 / v7x3 boards with channels % 128 == 0, the 15x15 64-channel
        // fused net), else bf16 pieces (channels % 32 == 0), else fp32
        const int b = s.boardSize;
        const bool trunk = (b == 8 || b == 9 || b == 13 || b == 15 || b == 19) && s.channels % 128 == 0 &&
                           (size_t)s.maxBatch * b * b * s.channels * 2 + 524288 < ((size_t)1 << 31);   // check_precision's bound
        const bool small = b == 15 && s.channels == 64 && s.inPlanes <= 16 && s.blocks <= 15 && s.pool <= 8 &&
                           2 * s.headChannels == 64;
        s.precision = (trunk || small) && s.blocks > 0 ? AZ_PREC_F16X3
                      : s.channels % 32 == 0            ? AZ_PREC_BF16X3
                                                        : AZ_PREC_F32;
    }
    auto net = std::make_unique<HipNeuralNetwork>(s, device);
    net->loadWeights(blob);
    net->autoPrecision_ = precision < 0;
    return net;
}

std::unique_ptr<HipNeuralNetwork> HipNeuralNetwork::createDDWRandWireResNet(int inputChannels, int outputSize,
                                                                           int channels, int numBlocks, int boardSize,
                                                                           int maxBatch, int device) {
    NetShape s;
    s.boardSize = boardSize; s.inPlanes = inputChannels; s.channels = channels; s.blocks = numBlocks;
    s.actionSize = outputSize; s.headChannels = 32; s.pool = std::min(8, boardSize); s.fcHidden = 256;
    s.residual = 0; s.convBias = 0; s.precision = AZ_PREC_F32; s.maxBatch = maxBatch; s.randWire = 1;
    return std::make_unique<HipNeuralNetwork>(s, device);
}

void HipNeuralNetwork::save(const std::string& path) const {
    if (shape_.randWire) throw std::runtime_error("save: the .azw header has no rand-wire field; keep the blob");
    if (blob_.empty()) throw std::runtime_error("save: weights were not loaded from a blob");
    std::ofstream f(path, std::ios::binary);
    const NetShape& s = shape_;
    const int32_t v[12] = {s.boardSize, s.inPlanes, s.channels, s.blocks, s.actionSize, s.headChannels,
                           s.pool,      s.fcHidden, s.residual, s.convBias, s.precision, s.maxBatch};
    const uint64_t count = blob_.size();
    f.write(kMagic, 4);
    f.write(reinterpret_cast<const char*>(v), sizeof v);
    f.write(reinterpret_cast<const char*>(&count), 8);
    f.write(reinterpret_cast<const char*>(blob_.data()), (std::streamsize)(count * 4));
    if (!f) throw std::runtime_error("cannot write " + path);
}

static void statePlanes(const core::IGameState& st, float* out) {
    if (auto* g = dynamic_cast<const gomoku::GomokuState*>(&st)) { g->enhancedPlanes(out); return; }
    if (auto* g = dynamic_cast<const go::GoState*>(&st)) { g->enhancedPlanes(out); return; }
    const core::Planes t = st.getEnhancedTensorRepresentation();
    size_t k = 0;
    for (const auto& p : t)
        for (const auto& row : p)
            for (float x : row) out[k++] = x;
}

void HipNeuralNetwork::predictBatch(const std::vector<std::reference_wrapper<const core::IGameState>>& states,
                                    std::vector<std::vector<float>>& policies, std::vector<float>& values) {
    const int B = (int)states.size(), A = shape_.actionSize, P = shape_.inPlanes * A;
    policies.assign(B, std::vector<float>());
    values.assign(B, 0.0f);
    if (B == 0) return;
    std::vector<float> planes((size_t)B * P), pol((size_t)B * A);
    for (int i = 0; i < B; ++i) {
        if (states[i].get().getActionSpaceSize() != A) throw std::invalid_argument("predictBatch: board size mismatch");
        statePlanes(states[i].get(), planes.data() + (size_t)i * P);
    }
    std::lock_guard<std::mutex> lk(mu_);
    const auto t0 = std::chrono::steady_clock::now();
    for (int b0 = 0; b0 < B; b0 += shape_.maxBatch) {
        const int n = std::min(shape_.maxBatch, B - b0);
        auto run = [&]() {
            return az_net_predict_batch(net_, planes.data() + (size_t)b0 * P, n, pol.data() + (size_t)b0 * A,
                                        values.data() + b0);
        };
        int rc = run();
        if (rc == AZ_ERR_RANGE && autoPrecision_ && shape_.precision == AZ_PREC_F16X3 &&
            az_net_set_precision(net_, AZ_PREC_BF16X3) == AZ_OK) {
            // activations beyond fp16's range: the fp32-range split precision from now on
            shape_.precision = AZ_PREC_BF16X3;
            rc = run();
        }
        check(rc, "az_net_predict_batch");
    }
    lastMs_ = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
    for (int i = 0; i < B; ++i) policies[i].assign(pol.begin() + (size_t)i * A, pol.begin() + (size_t)(i + 1) * A);
}

std::pair<std::vector<float>, float> HipNeuralNetwork::predict(const core::IGameState& state) {
    std::vector<std::vector<float>> p;
    std::vector<float> v;
    predictBatch({std::cref(state)}, p, v);
    return {p[0], v[0]};
}

std::future<std::pair<std::vector<float>, float>> HipNeuralNetwork::predictAsync(const core::IGameState& state) {
    std::shared_ptr<core::IGameState> copy(state.clone());
    return std::async(std::launch::async, [this, copy]() { return predict(*copy); });
}

std::string HipNeuralNetwork::getDeviceInfo() const {
    char name[256] = {0};
    az_engine_device_name(eng_, name, sizeof name);
    return std::string("MI355X engine: ") + name;
}

std::string HipNeuralNetwork::getModelInfo() const {
    static const char* prec[] = {"fp32", "bf16x3", "bf16", "fp16", "f16x3"};
    std::ostringstream o;
    o << "ResNet " << shape_.blocks << " blocks x " << shape_.channels << " filters, " << shape_.boardSize << "x"
      << shape_.boardSize << ", " << shape_.inPlanes << " input planes, policy " << shape_.actionSize << ", trunk "
      << (shape_.precision >= 0 && shape_.precision <= 4 ? prec[shape_.precision] : "?");
    return o.str();
}

void HipNeuralNetwork::benchmark(int iters, int batch) {
    gomoku::GomokuState sg(shape_.boardSize >= 5 ? shape_.boardSize : 15);
    go::GoState sgo(shape_.boardSize);
    const core::IGameState& s = shape_.inPlanes == 8 ? (const core::IGameState&)sgo : (const core::IGameState&)sg;
    std::vector<std::reference_wrapper<const core::IGameState>> states(batch, std::cref(s));
    std::vector<std::vector<float>> p;
    std::vector<float> v;
    predictBatch(states, p, v);
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < iters; ++i) predictBatch(states, p, v);
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    std::cout << "HipNeuralNetwork benchmark: batch " << batch << ", " << ms / iters << " ms/batch, "
              << batch * iters * 1000.0 / ms << " evals/s\n";
}

void HipNeuralNetwork::printModelSummary() const {
    std::cout << getModelInfo() << ", " << params_ << " parameters\n";
}

// --------------------------------------------------------------------------
RandomPolicyNetwork::RandomPolicyNetwork(core::GameType t, int bs, unsigned int seed)
    : gameType_(t), boardSize_(bs > 0 ? bs : 15), seed_(seed), rng_(seed) {}

std::pair<std::vector<float>, float> RandomPolicyNetwork::predict(const core::IGameState& state) {
    const int A = state.getActionSpaceSize();
    std::vector<float> p(A, 0.001f);
    std::uniform_real_distribution<float> u(0.0f, 1.0f);
    float sum = 0.0f;
    for (int a : state.getLegalMoves())
        if (a >= 0 && a < A) { p[a] = u(rng_); sum += p[a]; }     // Go's pass (-1) has no entry
    if (sum > 0.0f)
        for (float& x : p) x /= sum;
    std::uniform_real_distribution<float> vd(-0.1f, 0.1f);
    return {p, vd(rng_)};
}

void RandomPolicyNetwork::predictBatch(const std::vector<std::reference_wrapper<const core::IGameState>>& states,
                                       std::vector<std::vector<float>>& policies, std::vector<float>& values) {
    policies.clear();
    values.clear();
    for (const auto& s : states) {
        auto r = predict(s.get());
        policies.push_back(std::move(r.first));
        values.push_back(r.second);
    }
}

std::future<std::pair<std::vector<float>, float>> RandomPolicyNetwork::predictAsync(const core::IGameState& state) {
    std::promise<std::pair<std::vector<float>, float>> pr;
    pr.set_value(predict(state));
    return pr.get_future();
}

// --------------------------------------------------------------------------
std::unique_ptr<NeuralNetwork> NeuralNetwork::create(const std::string& path, core::GameType type, int bs, bool useGpu) {
    if (type == core::GameType::CHESS) throw std::invalid_argument("Chess networks are created from .azw files only");
    if (path.empty() || path == "random") return std::make_unique<RandomPolicyNetwork>(type, bs, 0);
    if (!useGpu) throw std::invalid_argument("the engine has no CPU network path (useGpu=false)");
    if (isZipArchive(path)) return HipNeuralNetwork::loadTorchScript(path, type, bs);   // the reference's .pt
    auto net = HipNeuralNetwork::load(path);
    if (bs > 0 && net->shape().boardSize != bs) throw std::invalid_argument("weight file board size mismatch");
    return net;
}

}  // namespace nn
}  // namespace alphazero
