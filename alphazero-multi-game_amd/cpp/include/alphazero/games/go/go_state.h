// alphazero/games/go/go_state.h -- host Go position (include/alphazero/games/go/go_state.h of
// the reference).  Same observable behaviour as the reference GoState and the engine's device
// rules (tree_kernels.hip, Go helpers): Black (1) first; pass = action -1 (action space bs*bs+1);
// captures of libertyless opponent groups, simple ko point (one single-stone capture), suicide
// illegal, positional superko over the positions after every stone move; game over after two
// consecutive passes; area (Chinese) or territory (Japanese) scoring with komi; Zobrist keys of
// ZobristHash(bs, 2, 2, 12345) plus the "ko_point" / "rules" / "komi" features; 8 enhanced
// feature planes.  The device search implements the reference defaults (komi 7.5, Chinese rules,
// superko): ParallelMCTS / SelfPlayManager refuse other settings.
#pragma once
#include <utility>
#include <vector>

#include "alphazero/core/igamestate.h"

namespace alphazero {
namespace go {

class GoState : public core::IGameState {
 public:
    // board sizes other than 9 / 13 / 19 fall back to 19, as the reference constructor does
    GoState(int board_size = 19, float komi = 7.5f, bool chinese_rules = true, bool enforce_superko = true);

    std::vector<int> getLegalMoves() const override;
    bool isLegalMove(int action) const override;
    void makeMove(int action) override;
    bool undoMove() override;
    bool isTerminal() const override { return consecutive_passes_ >= 2; }
    core::GameResult getGameResult() const override;
    int getCurrentPlayer() const override { return current_player_; }
    int getBoardSize() const override { return board_size_; }
    int getActionSpaceSize() const override { return board_size_ * board_size_ + 1; }
    core::Planes getTensorRepresentation() const override;
    core::Planes getEnhancedTensorRepresentation() const override;
    uint64_t getHash() const override;
    std::unique_ptr<core::IGameState> clone() const override;
    std::string actionToString(int action) const override;
    std::optional<int> stringToAction(const std::string& moveStr) const override;
    std::string toString() const override;
    bool equals(const core::IGameState& other) const override;
    std::vector<int> getMoveHistory() const override { return move_history_; }
    bool validate() const override;

    int getStone(int pos) const { return pos >= 0 && pos < board_size_ * board_size_ ? board_[pos] : 0; }
    int getStone(int x, int y) const { return getStone(coordToAction(x, y)); }
    int getCapturedStones(int player) const { return player == 1 || player == 2 ? captured_[player] : 0; }
    float getKomi() const { return komi_; }
    bool isChineseRules() const { return chinese_rules_; }
    bool isEnforcingSuperko() const { return superko_; }
    int getKoPoint() const { return ko_point_; }
    std::pair<int, int> actionToCoord(int action) const;
    int coordToAction(int x, int y) const;
    std::pair<float, float> calculateScore() const;     // (black, white) incl. komi
    // [8][bs*bs] flat planes (NCHW of one sample), the layout az_net_forward takes
    void enhancedPlanes(float* out) const;

 private:
    struct Undo { int action, ko, passes; std::vector<int> captured; };
    int adjacent(int pos, int* out) const;
    bool groupHasLiberty(const std::vector<int8_t>& b, int pos, std::vector<int>& stones, std::vector<char>& seen) const;
    int removeDead(std::vector<int8_t>& b, int color, std::vector<int>* removed, int* groups) const;
    bool suicidal(int pos) const;
    uint64_t hashOf(const std::vector<int8_t>& b, int player, int ko) const;

    int board_size_;
    int current_player_ = 1;
    float komi_;
    bool chinese_rules_, superko_;
    int ko_point_ = -1, consecutive_passes_ = 0;
    int captured_[3] = {0, 0, 0};
    std::vector<int8_t> board_;
    std::vector<int> move_history_;
    std::vector<uint64_t> position_history_;
    std::vector<Undo> undo_;
    std::vector<uint64_t> zpiece_, zko_;
    uint64_t zplayer_[2], zrules_[2], zkomi_[16];
};

}  // namespace go
}  // namespace alphazero
