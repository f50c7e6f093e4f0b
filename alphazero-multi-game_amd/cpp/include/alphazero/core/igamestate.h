// alphazero/core/igamestate.h -- game-state interface of the host API.
// Mirrors the reference surface (include/alphazero/core/igamestate.h: GameType, GameResult,
// IGameState virtuals, createGameState) so callers compile unchanged; only Gomoku is backed
// by the MI355X engine (SURVEY.md section 8 scope).
#pragma once
#include <cstdint>
#include <memory>
#include <optional>
#include <stdexcept>
#include <string>
#include <vector>

namespace alphazero {
namespace core {

enum class GameType { GOMOKU, CHESS, GO };
enum class GameResult { ONGOING, DRAW, WIN_PLAYER1, WIN_PLAYER2 };

class GameStateException : public std::runtime_error {
 public:
    explicit GameStateException(const std::string& m) : std::runtime_error(m) {}
};
class IllegalMoveException : public GameStateException {
 public:
    IllegalMoveException(const std::string& m, int action) : GameStateException(m), action_(action) {}
    int getAction() const { return action_; }

 private:
    int action_;
};

using Planes = std::vector<std::vector<std::vector<float>>>;

class IGameState {
 public:
    explicit IGameState(GameType type) : type_(type) {}
    virtual ~IGameState() = default;
    virtual std::vector<int> getLegalMoves() const = 0;
    virtual bool isLegalMove(int action) const = 0;
    virtual void makeMove(int action) = 0;
    virtual bool undoMove() = 0;
    virtual bool isTerminal() const = 0;
    virtual GameResult getGameResult() const = 0;
    virtual int getCurrentPlayer() const = 0;
    virtual int getBoardSize() const = 0;
    virtual int getActionSpaceSize() const = 0;
    virtual Planes getTensorRepresentation() const = 0;
    virtual Planes getEnhancedTensorRepresentation() const = 0;
    virtual uint64_t getHash() const = 0;
    virtual std::unique_ptr<IGameState> clone() const = 0;
    virtual std::string actionToString(int action) const = 0;
    virtual std::optional<int> stringToAction(const std::string& moveStr) const = 0;
    virtual std::string toString() const = 0;
    virtual bool equals(const IGameState& other) const = 0;
    virtual std::vector<int> getMoveHistory() const = 0;
    virtual bool validate() const = 0;
    GameType getGameType() const { return type_; }

 private:
    GameType type_;
};

// Gomoku (15x15 default) and Go (19x19, komi 7.5, Chinese rules); Chess throws std::invalid_argument.
std::unique_ptr<IGameState> createGameState(GameType type, int boardSize = 0, bool variantRules = false);

}  // namespace core
}  // namespace alphazero
