// alphazero/games/gomoku/gomoku_state.h -- host Gomoku position (standard rules).
// Same observable behaviour as the engine's device rules (tree_kernels.hip K5/K7) and the
// reference GomokuState with its defaults: Black (1) moves first; Black wins with exactly five
// in a row, White with five or more; draw on a full board; Zobrist keys of ZobristHash(bs, 2, 2,
// seed) (12345 unless given); 11 enhanced feature planes; legal-move order of
// SURVEY.md A.6 (a fresh state's first query: libstdc++ unordered_set order; afterwards
// descending cell index).  Renju / Omok / pro-long variants are not supported (throw).
#pragma once
#include <vector>

#include "alphazero/core/igamestate.h"

namespace alphazero {
namespace gomoku {

class GomokuState : public core::IGameState {
 public:
    GomokuState(int board_size = 15, bool use_renju = false, bool use_omok = false, int seed = 0,
                bool use_pro_long_opening = false);

    std::vector<int> getLegalMoves() const override;
    bool isLegalMove(int action) const override;
    void makeMove(int action) override;
    bool undoMove() override;
    bool isTerminal() const override { return getGameResult() != core::GameResult::ONGOING; }
    core::GameResult getGameResult() const override;
    int getCurrentPlayer() const override { return current_player; }
    int getBoardSize() const override { return board_size; }
    int getActionSpaceSize() const override { return board_size * board_size; }
    core::Planes getTensorRepresentation() const override;
    core::Planes getEnhancedTensorRepresentation() const override;
    uint64_t getHash() const override;
    std::unique_ptr<core::IGameState> clone() const override;
    std::string actionToString(int action) const override;
    std::optional<int> stringToAction(const std::string& moveStr) const override;
    std::string toString() const override;
    bool equals(const core::IGameState& other) const override;
    std::vector<int> getMoveHistory() const override { return move_history; }
    bool validate() const override;

    bool is_occupied(int action) const { return cells_[action] != 0; }
    std::vector<std::vector<int>> get_board() const;
    // [11][bs*bs] flat planes (NCHW of one sample), the layout az_net_forward takes
    void enhancedPlanes(float* out) const;

    int board_size;
    int current_player;   // 1 = BLACK, 2 = WHITE
    int action;           // last move or -1
    std::vector<int> move_history;

 private:
    int winnerAfter(int a) const;
    std::vector<uint8_t> cells_;
    std::vector<uint64_t> zkeys_;   // 2*A piece keys, then 2 player keys
    int winner_ = 0;                // 0 none, 1 / 2
    mutable bool queried_ = false;
};

}  // namespace gomoku
}  // namespace alphazero
