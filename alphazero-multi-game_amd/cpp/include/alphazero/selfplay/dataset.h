// alphazero/selfplay/dataset.h -- Dataset / TrainingExample of the host API,
// the reference's surface (include/alphazero/selfplay/dataset.h:21-118) over the device example
// store of the C-ABI (az_dataset_*): extractExamples replays every record on the MI355X and writes
// each position's examples (original + the 7 augmentExample symmetries) straight into their
// shuffled slots in HBM; getBatch / getRandomSubset / shuffle are device gathers.
//
// Differences from the reference, all loud: records of one Dataset share one game type and
// board size (the device store has one shape; a mismatch throws), Chess and variant rules throw
// (no device rules for them), and setSeed() fixes rng_ (the reference seeds it from
// std::random_device only).
#pragma once
#include <cstdint>
#include <string>
#include <tuple>
#include <vector>

#include "alphazero/core/igamestate.h"
#include "alphazero/selfplay/game_record.h"

struct az_dataset;

namespace alphazero {
namespace selfplay {

struct TrainingExample {
    std::vector<std::vector<std::vector<float>>> state;   // [plane][row][col]
    std::vector<float> policy;                            // the record's child-order visit distribution
    float value = 0.0f;                                   // game result from the side to move

    std::string toJson() const;
    static TrainingExample fromJson(const std::string& json);
};

class Dataset {
 public:
    Dataset();                        // device: LOCAL_RANK (default 0), rng_ from std::random_device
    explicit Dataset(int device);
    ~Dataset();
    Dataset(const Dataset&) = delete;
    Dataset& operator=(const Dataset&) = delete;

    void addGameRecord(const GameRecord& record, bool useEnhancedFeatures = true);
    void extractExamples(bool includeAugmentations = true);
    size_t size() const;
    std::tuple<std::vector<std::vector<std::vector<std::vector<float>>>>, std::vector<std::vector<float>>,
               std::vector<float>>
    getBatch(size_t batchSize) const;
    void shuffle();
    bool saveToFile(const std::string& filename) const;
    bool loadFromFile(const std::string& filename);
    std::vector<TrainingExample> getRandomSubset(size_t count) const;

    // engine extensions
    void setSeed(uint32_t seed);                            // rng_.seed(seed)
    std::vector<TrainingExample> getExamples() const;       // every example, slot order
    double lastExtractMs() const;                           // HIP-event time of the last extraction

 private:
    void ensureHandle(core::GameType type, int boardSize) const;
    std::vector<TrainingExample> gather(const std::vector<int64_t>& idx) const;
    std::vector<int64_t> shuffledIndices(int64_t n) const;

    int device_;
    std::vector<GameRecord> gameRecords_;
    mutable az_dataset* h_ = nullptr;
    mutable core::GameType type_ = core::GameType::GOMOKU;
    mutable int boardSize_ = 0;
    mutable uint32_t seed_;
};

}  // namespace selfplay
}  // namespace alphazero
