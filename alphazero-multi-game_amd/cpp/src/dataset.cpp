// Dataset / TrainingExample of the host API (row f3) over az_dataset_* (include/az_engine.h).
// Reference: src/selfplay/dataset.cpp (extractExamples :60-114, getBatch :120-145, shuffle :147-149,
// saveToFile / loadFromFile :151-227, getRandomSubset :229-243, augmentExample :245-436).
#include "alphazero/selfplay/dataset.h"

#include <cmath>
#include <fstream>
#include <random>
#include <sstream>
#include <stdexcept>

#include "alphazero/nn/hip_neural_network.h"
#include "az_engine.h"
#include "json_internal.h"

namespace alphazero {
namespace selfplay {

namespace {

void check(int rc, const char* what) {
    if (rc != 0) throw std::runtime_error(std::string(what) + ": " + az_last_error());
}

int engineGame(core::GameType t) {
    if (t == core::GameType::GOMOKU) return AZ_GAME_GOMOKU;
    if (t == core::GameType::GO) return AZ_GAME_GO;
    throw std::invalid_argument("Dataset: Chess has no rules on this engine");
}

int defaultBoard(core::GameType t, int bs) { return bs > 0 ? bs : (t == core::GameType::GO ? 19 : 15); }

// nlohmann::json::dump() of TrainingExample (dataset.cpp:16-33): compact, keys sorted
void writeExample(std::ostringstream& o, const TrainingExample& e) {
    o << "{\"policy\":[";
    for (size_t i = 0; i < e.policy.size(); ++i) o << (i ? "," : "") << jsonNumber((double)e.policy[i]);
    o << "],\"state\":[";
    for (size_t p = 0; p < e.state.size(); ++p) {
        o << (p ? ",[" : "[");
        for (size_t r = 0; r < e.state[p].size(); ++r) {
            o << (r ? ",[" : "[");
            for (size_t c = 0; c < e.state[p][r].size(); ++c) o << (c ? "," : "") << jsonNumber((double)e.state[p][r][c]);
            o << "]";
        }
        o << "]";
    }
    o << "],\"value\":" << jsonNumber((double)e.value) << "}";
}

float num(const json_internal::Value& v) { return v.kind == json_internal::Value::NUM ? (float)v.num : NAN; }

TrainingExample exampleFrom(const json_internal::Value& j) {
    TrainingExample e;
    for (const auto& pl : j.at("state").arr) {
        e.state.emplace_back();
        for (const auto& row : pl.arr) {
            e.state.back().emplace_back();
            for (const auto& x : row.arr) e.state.back().back().push_back(num(x));
        }
    }
    for (const auto& x : j.at("policy").arr) e.policy.push_back(num(x));
    e.value = num(j.at("value"));
    return e;
}

}  // namespace

std::string TrainingExample::toJson() const {
    std::ostringstream o;
    writeExample(o, *this);
    return o.str();
}

TrainingExample TrainingExample::fromJson(const std::string& json) {
    json_internal::Parser p{json};
    return exampleFrom(p.parse());
}

Dataset::Dataset() : Dataset(-1) {}

Dataset::Dataset(int device) : device_(device), seed_(std::random_device{}()) {}

Dataset::~Dataset() {
    if (h_) az_dataset_destroy(h_);
}

void Dataset::ensureHandle(core::GameType type, int boardSize) const {
    if (h_ && type == type_ && boardSize == boardSize_) return;
    if (h_) {
        az_dataset_destroy(h_);
        h_ = nullptr;
    }
    check(az_dataset_create(nn::engineForDevice(device_), engineGame(type), boardSize, &h_), "az_dataset_create");
    check(az_dataset_seed(h_, seed_), "az_dataset_seed");
    type_ = type;
    boardSize_ = boardSize;
}

void Dataset::setSeed(uint32_t seed) {
    seed_ = seed;
    if (h_) check(az_dataset_seed(h_, seed), "az_dataset_seed");
}

void Dataset::addGameRecord(const GameRecord& record, bool) { gameRecords_.push_back(record); }

void Dataset::extractExamples(bool includeAugmentations) {
    if (gameRecords_.empty()) {
        if (h_) check(az_dataset_extract(h_, 0, nullptr, nullptr, nullptr, nullptr, nullptr, 0, nullptr, nullptr),
                      "az_dataset_extract");
        return;
    }
    auto [t0, bs0, var0] = gameRecords_[0].getMetadata();
    const int bs = defaultBoard(t0, bs0);
    std::vector<int> nMoves, actions, nChildren, results;
    std::vector<float> policies;
    for (const GameRecord& r : gameRecords_) {
        auto [t, b, variant] = r.getMetadata();
        if (t != t0 || defaultBoard(t, b) != bs)
            throw std::invalid_argument("Dataset: records of one dataset must share game type and board size");
        if (variant) throw std::invalid_argument("Dataset: variant rules are not supported on this engine");
        nMoves.push_back((int)r.getMoves().size());
        for (const MoveData& m : r.getMoves()) {
            actions.push_back(m.action);
            nChildren.push_back((int)m.policy.size());
            policies.insert(policies.end(), m.policy.begin(), m.policy.end());
        }
        results.push_back((int)r.getResult());
    }
    ensureHandle(t0, bs);
    // extractExamples ends with shuffle() (dataset.cpp:112-113): draw the permutation first and
    // let the kernel write every example into its shuffled slot
    const int64_t E = (int64_t)actions.size() * (includeAugmentations ? 8 : 1);
    std::vector<int64_t> order = shuffledIndices(E);
    int64_t n = 0;
    check(az_dataset_extract(h_, (int)gameRecords_.size(), nMoves.data(), actions.data(), nChildren.data(),
                             policies.data(), results.data(), includeAugmentations ? 1 : 0, order.data(), &n),
          "az_dataset_extract");
}

size_t Dataset::size() const {
    if (!h_) return 0;
    int64_t n = 0;
    check(az_dataset_info(h_, &n, nullptr, nullptr, nullptr), "az_dataset_info");
    return (size_t)n;
}

std::vector<int64_t> Dataset::shuffledIndices(int64_t n) const {
    std::vector<int64_t> idx((size_t)n);
    if (h_) check(az_dataset_shuffle_order(h_, n, idx.data()), "az_dataset_shuffle_order");
    return idx;
}

std::vector<TrainingExample> Dataset::gather(const std::vector<int64_t>& idx) const {
    std::vector<TrainingExample> out;
    if (idx.empty()) return out;
    int planes = 0, bs = 0, stride = 0;
    check(az_dataset_info(h_, nullptr, &planes, &bs, &stride), "az_dataset_info");
    const size_t n = idx.size(), row = (size_t)planes * bs * bs;
    std::vector<float> st(n * row), po(n * stride), va(n);
    std::vector<int> pl(n);
    check(az_dataset_gather(h_, idx.data(), (int)n, st.data(), po.data(), pl.data(), va.data()), "az_dataset_gather");
    out.resize(n);
    for (size_t i = 0; i < n; ++i) {
        TrainingExample& e = out[i];
        e.state.assign(planes, std::vector<std::vector<float>>(bs, std::vector<float>(bs)));
        const float* s = st.data() + i * row;
        for (int p = 0; p < planes; ++p)
            for (int r = 0; r < bs; ++r)
                for (int c = 0; c < bs; ++c) e.state[p][r][c] = s[((size_t)p * bs + r) * bs + c];
        e.policy.assign(po.begin() + i * stride, po.begin() + i * stride + pl[i]);
        e.value = va[i];
    }
    return out;
}

std::tuple<std::vector<std::vector<std::vector<std::vector<float>>>>, std::vector<std::vector<float>>,
           std::vector<float>>
Dataset::getBatch(size_t batchSize) const {
    const size_t n = size();
    batchSize = std::min(batchSize, n);
    std::vector<int64_t> idx = shuffledIndices((int64_t)n);   // dataset.cpp:129-131
    idx.resize(batchSize);
    std::vector<TrainingExample> ex = gather(idx);
    std::vector<std::vector<std::vector<std::vector<float>>>> states(batchSize);
    std::vector<std::vector<float>> policies(batchSize);
    std::vector<float> values(batchSize);
    for (size_t i = 0; i < batchSize; ++i) {
        states[i] = std::move(ex[i].state);
        policies[i] = std::move(ex[i].policy);
        values[i] = ex[i].value;
    }
    return {states, policies, values};
}

void Dataset::shuffle() {
    const int64_t n = (int64_t)size();
    if (n == 0) return;
    std::vector<int64_t> order = shuffledIndices(n);
    check(az_dataset_permute(h_, order.data()), "az_dataset_permute");
}

std::vector<TrainingExample> Dataset::getRandomSubset(size_t count) const {
    const size_t n = size();
    std::vector<int64_t> idx = shuffledIndices((int64_t)n);   // dataset.cpp:232-235
    idx.resize(std::min(count, n));
    return gather(idx);
}

std::vector<TrainingExample> Dataset::getExamples() const {
    std::vector<int64_t> idx(size());
    for (size_t i = 0; i < idx.size(); ++i) idx[i] = (int64_t)i;
    return gather(idx);
}

double Dataset::lastExtractMs() const {
    double ms = 0.0;
    if (h_) check(az_dataset_profile_read(h_, &ms, nullptr), "az_dataset_profile_read");
    return ms;
}

bool Dataset::saveToFile(const std::string& filename) const {
    try {
        std::ostringstream o;
        o << "{\"examples\":[";
        const std::vector<TrainingExample> ex = getExamples();
        for (size_t i = 0; i < ex.size(); ++i) {
            if (i) o << ",";
            writeExample(o, ex[i]);
        }
        o << "]}";
        std::ofstream f(filename);
        if (!f.is_open()) return false;
        f << o.str();
        return (bool)f;
    } catch (...) {
        return false;
    }
}

bool Dataset::loadFromFile(const std::string& filename) {
    try {
        std::ifstream f(filename);
        if (!f.is_open()) return false;
        std::stringstream b;
        b << f.rdbuf();
        const std::string text = b.str();
        json_internal::Parser p{text};
        const json_internal::Value j = p.parse();
        std::vector<TrainingExample> ex;
        for (const auto& e : j.at("examples").arr) ex.push_back(exampleFrom(e));
        if (ex.empty()) {
            if (h_) check(az_dataset_upload(h_, 0, nullptr, nullptr, nullptr, nullptr), "az_dataset_upload");
            return true;
        }
        // the store's shape from the first example: 11 planes Gomoku, 8 planes Go
        const int planes = (int)ex[0].state.size();
        const int bs = planes ? (int)ex[0].state[0].size() : 0;
        if (planes != 11 && planes != 8) return false;
        ensureHandle(planes == 8 ? core::GameType::GO : core::GameType::GOMOKU, bs);
        int stride = 0;
        check(az_dataset_info(h_, nullptr, nullptr, nullptr, &stride), "az_dataset_info");
        const size_t n = ex.size(), row = (size_t)planes * bs * bs;
        std::vector<float> st(n * row), po(n * stride, 0.0f), va(n);
        std::vector<int> pl(n);
        for (size_t i = 0; i < n; ++i) {
            const TrainingExample& e = ex[i];
            if ((int)e.state.size() != planes || (int)e.policy.size() > stride) return false;
            for (int pi = 0; pi < planes; ++pi) {
                if ((int)e.state[pi].size() != bs) return false;
                for (int r = 0; r < bs; ++r) {
                    if ((int)e.state[pi][r].size() != bs) return false;
                    for (int c = 0; c < bs; ++c) st[i * row + ((size_t)pi * bs + r) * bs + c] = e.state[pi][r][c];
                }
            }
            std::copy(e.policy.begin(), e.policy.end(), po.begin() + i * stride);
            pl[i] = (int)e.policy.size();
            va[i] = e.value;
        }
        check(az_dataset_upload(h_, (int64_t)n, st.data(), po.data(), pl.data(), va.data()), "az_dataset_upload");
        return true;
    } catch (...) {
        return false;
    }
}

}  // namespace selfplay
}  // namespace alphazero
