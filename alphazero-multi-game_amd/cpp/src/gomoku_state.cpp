// Host Gomoku position for the API surface (createGameState, ParallelMCTS roots, predict).
// The search itself never calls this: the device keeps its own boards (tree_kernels.hip).
#include "alphazero/games/gomoku/gomoku_state.h"
#include "alphazero/games/go/go_state.h"

#include <algorithm>
#include <random>
#include <sstream>
#include <unordered_set>

namespace alphazero {
namespace gomoku {

GomokuState::GomokuState(int bs, bool use_renju, bool use_omok, int seed, bool use_pro_long_opening)
    : core::IGameState(core::GameType::GOMOKU), board_size(bs), current_player(1), action(-1) {
    if (bs < 5 || bs > 19) throw std::invalid_argument("GomokuState: board size must be 5..19");
    if (use_renju || use_omok || use_pro_long_opening)
        throw std::invalid_argument("GomokuState: only standard rules are supported (renju/omok/pro-long off)");
    const int A = bs * bs;
    cells_.assign(A, 0);
    // ZobristHash(bs, 2 pieces, 2 players, seed): mt19937_64 draws, piece keys then player keys
    std::mt19937_64 rng(seed == 0 ? 12345u : (uint64_t)(unsigned)seed);
    zkeys_.resize(2 * A + 2);
    for (auto& k : zkeys_) k = rng();
}

int GomokuState::winnerAfter(int a) const {
    const int bs = board_size, p = cells_[a], x = a / bs, y = a % bs;
    static const int dirs[4][2] = {{0, 1}, {1, 0}, {1, 1}, {1, -1}};
    for (const auto& d : dirs) {
        int run = 1;
        for (int s = -1; s <= 1; s += 2)
            for (int k = 1;; ++k) {
                const int xx = x + s * k * d[0], yy = y + s * k * d[1];
                if (xx < 0 || yy < 0 || xx >= bs || yy >= bs || cells_[xx * bs + yy] != p) break;
                ++run;
            }
        if (p == 1 ? run == 5 : run >= 5) return p;   // Black: exactly five; White: five or more
    }
    return 0;
}

std::vector<int> GomokuState::getLegalMoves() const {
    std::vector<int> out;
    if (isTerminal()) return out;
    const int A = getActionSpaceSize();
    if (!queried_) {
        // first query of this object: the cache set grows from one bucket
        std::unordered_set<int> set;
        for (int a = 0; a < A; ++a)
            if (!cells_[a]) set.insert(a);
        out.assign(set.begin(), set.end());
        queried_ = true;
        return out;
    }
    for (int a = A - 1; a >= 0; --a)
        if (!cells_[a]) out.push_back(a);
    return out;
}

bool GomokuState::isLegalMove(int a) const {
    return a >= 0 && a < getActionSpaceSize() && !cells_[a] && !isTerminal();
}

void GomokuState::makeMove(int a) {
    if (!isLegalMove(a)) throw core::IllegalMoveException("illegal move " + std::to_string(a), a);
    cells_[a] = (uint8_t)current_player;
    move_history.push_back(a);
    action = a;
    if (!winner_) winner_ = winnerAfter(a);
    current_player = 3 - current_player;
}

bool GomokuState::undoMove() {
    if (move_history.empty()) return false;
    const int a = move_history.back();
    move_history.pop_back();
    cells_[a] = 0;
    current_player = 3 - current_player;
    action = move_history.empty() ? -1 : move_history.back();
    winner_ = 0;
    for (int m : move_history)
        if ((winner_ = winnerAfter(m))) break;
    return true;
}

core::GameResult GomokuState::getGameResult() const {
    if (winner_ == 1) return core::GameResult::WIN_PLAYER1;
    if (winner_ == 2) return core::GameResult::WIN_PLAYER2;
    if ((int)move_history.size() >= getActionSpaceSize()) return core::GameResult::DRAW;
    return core::GameResult::ONGOING;
}

void GomokuState::enhancedPlanes(float* out) const {
    const int bs = board_size, A = bs * bs, me = current_player, opp = 3 - current_player;
    std::fill(out, out + 11 * A, 0.0f);
    for (int a = 0; a < A; ++a) {
        if (cells_[a] == me) out[a] = 1.0f;
        else if (cells_[a] == opp) out[A + a] = 1.0f;
        if (me == 1) out[2 * A + a] = 1.0f;
    }
    // planes 3-5 / 6-8: last three moves attributed by the reference's parity rule (A.5)
    const int n = (int)move_history.size();
    for (int pl = 1; pl <= 2; ++pl) {
        int found = 0;
        for (int i = n - 1; i >= 0 && found < 3; --i) {
            const int mover = ((n - i) % 2 == 1) ? me : opp;
            if (mover == pl) out[(pl == 1 ? 3 : 6) * A + found++ * A + move_history[i]] = 1.0f;
        }
    }
    for (int x = 0; x < bs; ++x)
        for (int y = 0; y < bs; ++y) {
            out[9 * A + x * bs + y] = (float)x / (float)(bs - 1);
            out[10 * A + x * bs + y] = (float)y / (float)(bs - 1);
        }
}

static core::Planes unflatten(const std::vector<float>& f, int planes, int bs) {
    core::Planes t(planes, std::vector<std::vector<float>>(bs, std::vector<float>(bs)));
    for (int c = 0; c < planes; ++c)
        for (int x = 0; x < bs; ++x)
            for (int y = 0; y < bs; ++y) t[c][x][y] = f[((size_t)c * bs + x) * bs + y];
    return t;
}

core::Planes GomokuState::getEnhancedTensorRepresentation() const {
    std::vector<float> f((size_t)11 * getActionSpaceSize());
    enhancedPlanes(f.data());
    return unflatten(f, 11, board_size);
}

core::Planes GomokuState::getTensorRepresentation() const {
    std::vector<float> f((size_t)11 * getActionSpaceSize());
    enhancedPlanes(f.data());
    f.resize((size_t)3 * getActionSpaceSize());
    return unflatten(f, 3, board_size);
}

uint64_t GomokuState::getHash() const {
    const int A = getActionSpaceSize();
    uint64_t h = zkeys_[2 * A + current_player - 1];
    for (int a = 0; a < A; ++a)
        if (cells_[a]) h ^= zkeys_[(size_t)(cells_[a] - 1) * A + a];
    return h;
}

std::unique_ptr<core::IGameState> GomokuState::clone() const { return std::make_unique<GomokuState>(*this); }

std::string GomokuState::actionToString(int a) const {
    if (a < 0 || a >= getActionSpaceSize()) return "invalid";
    char col = (char)('A' + a % board_size);
    if (col >= 'I') ++col;   // Go/Gomoku letters skip I
    return std::string(1, col) + std::to_string(board_size - a / board_size);
}

std::optional<int> GomokuState::stringToAction(const std::string& s) const {
    if (s.size() < 2 || s.size() > 3) return std::nullopt;
    char col = s[0];
    if (col >= 'a' && col <= 'z') col = (char)(col - 'a' + 'A');
    if (col < 'A' || col > 'Z' || col == 'I') return std::nullopt;
    if (col > 'I') --col;
    int row = 0;
    for (size_t i = 1; i < s.size(); ++i) {
        if (s[i] < '0' || s[i] > '9') return std::nullopt;
        row = row * 10 + (s[i] - '0');
    }
    const int x = board_size - row, y = col - 'A';
    if (x < 0 || x >= board_size || y < 0 || y >= board_size) return std::nullopt;
    return x * board_size + y;
}

std::string GomokuState::toString() const {
    std::ostringstream o;
    o << "  ";
    for (int y = 0; y < board_size; ++y) {
        char c = (char)('A' + y);
        if (c >= 'I') ++c;
        o << ' ' << c;
    }
    o << '\n';
    for (int x = 0; x < board_size; ++x) {
        const int row = board_size - x;
        o << (row < 10 ? " " : "") << row << ' ';
        for (int y = 0; y < board_size; ++y) o << ".XO"[cells_[x * board_size + y]] << ' ';
        o << row << '\n';
    }
    o << (current_player == 1 ? "Black" : "White") << " to move\n";
    return o.str();
}

bool GomokuState::equals(const core::IGameState& other) const {
    auto* g = dynamic_cast<const GomokuState*>(&other);
    return g && g->board_size == board_size && g->current_player == current_player && g->cells_ == cells_;
}

bool GomokuState::validate() const {
    int b = 0, w = 0;
    for (uint8_t c : cells_) { b += c == 1; w += c == 2; }
    return (b == w || b == w + 1) && current_player == (b == w ? 1 : 2);
}

std::vector<std::vector<int>> GomokuState::get_board() const {
    std::vector<std::vector<int>> b(board_size, std::vector<int>(board_size));
    for (int x = 0; x < board_size; ++x)
        for (int y = 0; y < board_size; ++y) b[x][y] = cells_[x * board_size + y];
    return b;
}

}  // namespace gomoku

namespace core {
std::unique_ptr<IGameState> createGameState(GameType type, int boardSize, bool variantRules) {
    // igamestate.cpp:17-49 / game_factory.cpp:88-115: Gomoku 15x15 standard rules, Go 19x19 komi 7.5
    // Chinese rules; Chess has no rules on this engine (its network shape runs)
    if (type == GameType::GO) return std::make_unique<go::GoState>(boardSize > 0 ? boardSize : 19, 7.5f, true, true);
    if (type != GameType::GOMOKU) throw std::invalid_argument("createGameState: Chess rules are not implemented");
    return std::make_unique<gomoku::GomokuState>(boardSize > 0 ? boardSize : 15, variantRules, false);
}
}  // namespace core
}  // namespace alphazero
