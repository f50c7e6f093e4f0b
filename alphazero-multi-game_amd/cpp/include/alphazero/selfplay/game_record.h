// alphazero/selfplay/game_record.h -- GameRecord / MoveData of the host API with the
// reference's JSON format (src/selfplay/game_record.cpp:17-145: nlohmann::json dump(4) --
// keys sorted, four-space indent, floats as the shortest round-trip text of the float widened
// to double, NaN as null).  SURVEY.md row f1.
#pragma once
#include <chrono>
#include <cstdint>
#include <string>
#include <tuple>
#include <vector>

#include "alphazero/core/igamestate.h"

namespace alphazero {
namespace selfplay {

struct MoveData {
    int action = -1;
    std::vector<float> policy;   // visit distribution in CHILD order (as the reference records it)
    float value = 0.0f;
    int64_t thinking_time_ms = 0;
    std::string toJson() const;
    static MoveData fromJson(const std::string& json);
};

class GameRecord {
 public:
    GameRecord(core::GameType gameType, int boardSize, bool useVariantRules = false);
    void addMove(int action, const std::vector<float>& policy, float value, int64_t thinkingTimeMs);
    void setResult(core::GameResult result) { result_ = result; }
    std::tuple<core::GameType, int, bool> getMetadata() const { return {gameType_, boardSize_, useVariantRules_}; }
    const std::vector<MoveData>& getMoves() const { return moves_; }
    core::GameResult getResult() const { return result_; }
    std::string toJson() const;
    static GameRecord fromJson(const std::string& json);
    bool saveToFile(const std::string& filename) const;
    static GameRecord loadFromFile(const std::string& filename);
    // fixed timestamp (tests / reproducible files); default: construction time
    void setTimestamp(std::chrono::system_clock::time_point t) { timestamp_ = t; }

 private:
    core::GameType gameType_;
    int boardSize_;
    bool useVariantRules_;
    std::vector<MoveData> moves_;
    core::GameResult result_ = core::GameResult::ONGOING;
    std::chrono::system_clock::time_point timestamp_;
};

// nlohmann::json's number_float serialisation of a double (grisu2 shortest digits, fixed
// notation for decimal exponents in (-4, 15], else d.ddde+XX), "null" for NaN / infinity.
std::string jsonNumber(double v);

}  // namespace selfplay
}  // namespace alphazero
