// Host Go position for the API surface (createGameState(GO), ParallelMCTS roots, predict).
// Rules follow the reference src/games/go/go_state.cpp + go_rules.cpp; the device search keeps
// its own boards (tree_kernels.hip) and never calls this.
#include "alphazero/games/go/go_state.h"

#include <algorithm>
#include <functional>
#include <random>
#include <sstream>

namespace alphazero {
namespace go {

GoState::GoState(int bs, float komi, bool chinese, bool superko)
    : core::IGameState(core::GameType::GO), board_size_(bs == 9 || bs == 13 || bs == 19 ? bs : 19), komi_(komi),
      chinese_rules_(chinese), superko_(superko) {
    const int A = board_size_ * board_size_;
    board_.assign(A, 0);
    // ZobristHash(bs, 2, 2, 12345): piece keys, then player keys; features from
    // mt19937_64(std::hash<std::string>(name)) (zobrist_hash.cpp:58-70, go_state.cpp:48-51)
    std::mt19937_64 rng(12345u);
    zpiece_.resize(2 * A);
    for (auto& k : zpiece_) k = rng();
    zplayer_[0] = rng(); zplayer_[1] = rng();
    std::mt19937_64 rk(std::hash<std::string>{}("ko_point"));
    zko_.resize(A + 1);
    for (auto& k : zko_) k = rk();
    std::mt19937_64 rr(std::hash<std::string>{}("rules"));
    for (auto& k : zrules_) k = rr();
    std::mt19937_64 rm(std::hash<std::string>{}("komi"));
    for (auto& k : zkomi_) k = rm();
}

int GoState::adjacent(int pos, int* nb) const {   // up, right, down, left (:800-816)
    const int bs = board_size_, x = pos % bs;
    int n = 0;
    if (pos >= bs) nb[n++] = pos - bs;
    if (x + 1 < bs) nb[n++] = pos + 1;
    if (pos + bs < bs * bs) nb[n++] = pos + bs;
    if (x > 0) nb[n++] = pos - 1;
    return n;
}

bool GoState::groupHasLiberty(const std::vector<int8_t>& b, int pos, std::vector<int>& stones,
                              std::vector<char>& seen) const {
    const int c = b[pos];
    stones.assign(1, pos);
    seen[pos] = 1;
    bool lib = false;
    for (size_t i = 0; i < stones.size(); ++i) {
        int nb[4];
        const int k = adjacent(stones[i], nb);
        for (int j = 0; j < k; ++j) {
            if (b[nb[j]] == 0) lib = true;
            else if (b[nb[j]] == c && !seen[nb[j]]) { seen[nb[j]] = 1; stones.push_back(nb[j]); }
        }
    }
    return lib;
}

// removes every libertyless group of `color`; returns the number of stones removed
int GoState::removeDead(std::vector<int8_t>& b, int color, std::vector<int>* removed, int* groups) const {
    const int A = board_size_ * board_size_;
    std::vector<char> seen(A, 0);
    std::vector<int> st, dead;
    int ng = 0;
    for (int p = 0; p < A; ++p) {
        if (b[p] != color || seen[p]) continue;
        if (!groupHasLiberty(b, p, st, seen)) { dead.insert(dead.end(), st.begin(), st.end()); ++ng; }
    }
    for (int p : dead) b[p] = 0;
    if (removed) *removed = dead;
    if (groups) *groups = ng;
    return (int)dead.size();
}

bool GoState::suicidal(int pos) const {   // GoRules::isSuicidalMove (go_rules.cpp:27-136)
    std::vector<int8_t> b = board_;
    const int p = current_player_;
    b[pos] = (int8_t)p;
    std::vector<char> seen(b.size(), 0);
    std::vector<int> st;
    int nb[4];
    const int k = adjacent(pos, nb);
    for (int j = 0; j < k; ++j)
        if (b[nb[j]] == 3 - p && !seen[nb[j]] && !groupHasLiberty(b, nb[j], st, seen)) return false;
    std::fill(seen.begin(), seen.end(), 0);
    return !groupHasLiberty(b, pos, st, seen);
}

uint64_t GoState::hashOf(const std::vector<int8_t>& b, int player, int ko) const {   // updateHash (:846-877)
    const int A = board_size_ * board_size_;
    uint64_t h = 0;
    for (int a = 0; a < A; ++a)
        if (b[a]) h ^= zpiece_[(size_t)(b[a] - 1) * A + a];
    h ^= zplayer_[player - 1];
    if (ko >= 0) h ^= zko_[ko % (A + 1)];
    h ^= zrules_[chinese_rules_ ? 1 : 0];
    h ^= zkomi_[((int)(komi_ * 2)) & 0xF];
    return h;
}

uint64_t GoState::getHash() const { return hashOf(board_, current_player_, ko_point_); }

std::vector<int> GoState::getLegalMoves() const {   // :116-160
    std::vector<int> out{-1};
    const int A = board_size_ * board_size_;
    for (int a = 0; a < A; ++a) {
        if (board_[a] != 0 || a == ko_point_ || suicidal(a)) continue;
        if (superko_) {
            std::vector<int8_t> b = board_;
            b[a] = (int8_t)current_player_;
            removeDead(b, 3 - current_player_, nullptr, nullptr);
            const uint64_t h = hashOf(b, current_player_, ko_point_);   // side to move and ko point unchanged
            if (std::find(position_history_.begin(), position_history_.end(), h) != position_history_.end()) continue;
        }
        out.push_back(a);
    }
    return out;
}

bool GoState::isLegalMove(int a) const {
    if (a == -1) return true;
    const auto l = getLegalMoves();
    return std::find(l.begin(), l.end(), a) != l.end();
}

void GoState::makeMove(int a) {   // :192-257
    if (!isLegalMove(a)) throw core::IllegalMoveException("GoState: illegal move " + actionToString(a), a);
    Undo u{a, ko_point_, consecutive_passes_, {}};
    if (a == -1) {
        ++consecutive_passes_;
        ko_point_ = -1;
    } else {
        consecutive_passes_ = 0;
        board_[a] = (int8_t)current_player_;
        int groups = 0;
        const int n = removeDead(board_, 3 - current_player_, &u.captured, &groups);
        ko_point_ = (groups == 1 && n == 1) ? u.captured[0] : -1;
        captured_[current_player_] += n;
        position_history_.push_back(getHash());
    }
    move_history_.push_back(a);
    undo_.push_back(std::move(u));
    current_player_ = 3 - current_player_;
}

bool GoState::undoMove() {   // :259-303
    if (undo_.empty()) return false;
    Undo u = std::move(undo_.back());
    undo_.pop_back();
    move_history_.pop_back();
    current_player_ = 3 - current_player_;
    ko_point_ = u.ko;
    consecutive_passes_ = u.passes;
    if (u.action >= 0) {
        position_history_.pop_back();
        board_[u.action] = 0;
        for (int p : u.captured) board_[p] = (int8_t)(3 - current_player_);
        captured_[current_player_] -= (int)u.captured.size();
    }
    return true;
}

std::pair<float, float> GoState::calculateScore() const {   // go_rules.cpp:211-361
    const int A = board_size_ * board_size_;
    std::vector<int> terr(A, 0);
    std::vector<char> seen(A, 0);
    for (int p = 0; p < A; ++p) {
        if (board_[p] != 0 || seen[p]) continue;
        std::vector<int> reg{p};
        seen[p] = 1;
        bool tb = false, tw = false;
        for (size_t i = 0; i < reg.size(); ++i) {
            int nb[4];
            const int k = adjacent(reg[i], nb);
            for (int j = 0; j < k; ++j) {
                const int s = board_[nb[j]];
                if (s == 0) { if (!seen[nb[j]]) { seen[nb[j]] = 1; reg.push_back(nb[j]); } }
                else if (s == 1) tb = true;
                else tw = true;
            }
        }
        const int col = tb && !tw ? 1 : tw && !tb ? 2 : 0;
        for (int r : reg) terr[r] = col;
    }
    if (chinese_rules_)
        for (int p = 0; p < A; ++p) if (board_[p]) terr[p] = board_[p];
    float b = 0.0f, w = 0.0f;
    for (int p = 0; p < A; ++p) {
        if (terr[p] == 1) b += 1.0f;
        else if (terr[p] == 2) w += 1.0f;
    }
    if (!chinese_rules_) { b += (float)captured_[1]; w += (float)captured_[2]; }
    w += komi_;
    return {b, w};
}

core::GameResult GoState::getGameResult() const {
    if (!isTerminal()) return core::GameResult::ONGOING;
    const auto [b, w] = calculateScore();
    if (b > w) return core::GameResult::WIN_PLAYER1;
    if (w > b) return core::GameResult::WIN_PLAYER2;
    return core::GameResult::DRAW;
}

void GoState::enhancedPlanes(float* out) const {   // :338-420
    const int bs = board_size_, A = bs * bs;
    std::fill(out, out + 8 * A, 0.0f);
    for (int a = 0; a < A; ++a) {
        if (board_[a] == 1) out[a] = 1.0f;
        else if (board_[a] == 2) out[A + a] = 1.0f;
        out[2 * A + a] = current_player_ == 1 ? 1.0f : 0.0f;
    }
    std::vector<char> seen(A, 0), lib(A, 0);
    std::vector<int> st;
    for (int p = 0; p < A; ++p) {
        if (!board_[p] || seen[p]) continue;
        groupHasLiberty(board_, p, st, seen);
        int libs = 0;
        std::fill(lib.begin(), lib.end(), 0);
        for (int s : st) {
            int nb[4];
            const int k = adjacent(s, nb);
            for (int j = 0; j < k; ++j) if (board_[nb[j]] == 0 && !lib[nb[j]]) { lib[nb[j]] = 1; ++libs; }
        }
        const float v = std::min(1.0f, (float)libs / 10.0f);
        for (int s : st) out[(board_[p] == 1 ? 3 : 4) * A + s] = v;
    }
    if (ko_point_ >= 0) out[5 * A + ko_point_] = 1.0f;
    for (int y = 0; y < bs; ++y)
        for (int x = 0; x < bs; ++x) {
            out[6 * A + y * bs + x] = (float)std::min(x, bs - 1 - x) / (bs / 2);
            out[7 * A + y * bs + x] = (float)std::min(y, bs - 1 - y) / (bs / 2);
        }
}

static core::Planes toPlanes(const std::vector<float>& flat, int n, int bs) {
    core::Planes t(n, std::vector<std::vector<float>>(bs, std::vector<float>(bs)));
    for (int p = 0; p < n; ++p)
        for (int y = 0; y < bs; ++y)
            for (int x = 0; x < bs; ++x) t[p][y][x] = flat[((size_t)p * bs + y) * bs + x];
    return t;
}

core::Planes GoState::getEnhancedTensorRepresentation() const {
    std::vector<float> f((size_t)8 * board_size_ * board_size_);
    enhancedPlanes(f.data());
    return toPlanes(f, 8, board_size_);
}

core::Planes GoState::getTensorRepresentation() const {
    std::vector<float> f((size_t)8 * board_size_ * board_size_);
    enhancedPlanes(f.data());
    f.resize((size_t)3 * board_size_ * board_size_);
    return toPlanes(f, 3, board_size_);
}

std::unique_ptr<core::IGameState> GoState::clone() const { return std::make_unique<GoState>(*this); }

std::pair<int, int> GoState::actionToCoord(int a) const {
    if (a < 0 || a >= board_size_ * board_size_) return {-1, -1};
    return {a % board_size_, a / board_size_};
}

int GoState::coordToAction(int x, int y) const {
    if (x < 0 || y < 0 || x >= board_size_ || y >= board_size_) return -1;
    return y * board_size_ + x;
}

std::string GoState::actionToString(int a) const {   // A..T without I, rows counted from the bottom
    if (a == -1) return "pass";
    if (a < 0 || a >= board_size_ * board_size_) return "invalid";
    const auto [x, y] = actionToCoord(a);
    char col = (char)('A' + x);
    if (col >= 'I') ++col;
    return std::string(1, col) + std::to_string(board_size_ - y);
}

std::optional<int> GoState::stringToAction(const std::string& s) const {
    if (s == "pass" || s == "PASS" || s == "Pass") return -1;
    if (s.size() < 2) return std::nullopt;
    const char c = (char)std::toupper((unsigned char)s[0]);
    if (c == 'I' || c < 'A' || c > 'Z') return std::nullopt;
    const int x = c >= 'J' ? c - 'A' - 1 : c - 'A';
    int row;
    try { row = std::stoi(s.substr(1)); } catch (...) { return std::nullopt; }
    const int y = board_size_ - row;
    if (x < 0 || x >= board_size_ || y < 0 || y >= board_size_) return std::nullopt;
    return coordToAction(x, y);
}

std::string GoState::toString() const {
    std::ostringstream o;
    for (int y = 0; y < board_size_; ++y) {
        for (int x = 0; x < board_size_; ++x) {
            const int a = y * board_size_ + x;
            o << (board_[a] == 1 ? 'X' : board_[a] == 2 ? 'O' : a == ko_point_ ? 'k' : '.') << ' ';
        }
        o << '\n';
    }
    o << "Current player: " << (current_player_ == 1 ? "Black" : "White") << ", captures B " << captured_[1] << " W "
      << captured_[2] << ", komi " << komi_ << '\n';
    return o.str();
}

bool GoState::equals(const core::IGameState& other) const {
    auto* g = dynamic_cast<const GoState*>(&other);
    return g && g->board_size_ == board_size_ && g->current_player_ == current_player_ && g->ko_point_ == ko_point_ &&
           g->komi_ == komi_ && g->chinese_rules_ == chinese_rules_ && g->consecutive_passes_ == consecutive_passes_ &&
           g->captured_[1] == captured_[1] && g->captured_[2] == captured_[2] && g->board_ == board_;
}

bool GoState::validate() const {
    return (board_size_ == 9 || board_size_ == 13 || board_size_ == 19) && (current_player_ == 1 || current_player_ == 2) &&
           ko_point_ < board_size_ * board_size_;
}

}  // namespace go
}  // namespace alphazero
