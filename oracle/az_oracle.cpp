// oracle/az_oracle.cpp -- TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of the reference self-play hot path in "Mode S" (SURVEY.md
// Appendix A): GomokuState and GoState rules/features/hash, ParallelMCTS sequential simulation
// (numThreads=1, setDeterministicMode(true)), TranspositionTable, Dirichlet noise,
// and the SelfPlayManager::playSingleGame move loop.  Only tests/, bench.py's
// cpu_baseline leg and __graft_entry__.smoke() may load it, and only as the checker.
// It is pinned against golden vectors produced by the patched reference
// (oracle/build_ref.sh -> oracle/_ref/ref_harness -> tests/golden/).
//
// Every function cites the reference lines (paths relative to the reference root)
// it restates.  fp32 arithmetic is written in the reference's evaluation order;
// compile WITHOUT FMA contraction (-ffp-contract=off), as the reference is built.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <random>
#include <sstream>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace {

uint32_t fbits(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }

uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

enum GameResult { ONGOING = 0, DRAW = 1, WIN_P1 = 2, WIN_P2 = 3 };   // igamestate.h:26-31

// ---------------------------------------------------------------------------
// Zobrist keys: ZobristHash(bs, 2 piece types, 2 players, seed)
// (src/core/zobrist_hash.cpp:9-36): mt19937_64(seed); piece[p][pos] then player[p].
struct Zobrist {
    std::vector<uint64_t> piece;   // [2][A]
    uint64_t player[2];
    Zobrist(int A, unsigned seed) : piece(2 * A) {
        std::mt19937_64 rng(seed);
        for (int p = 0; p < 2; ++p)
            for (int a = 0; a < A; ++a) piece[p * A + a] = rng();
        player[0] = rng(); player[1] = rng();
    }
};

// ---------------------------------------------------------------------------
// GomokuState (src/games/gomoku/gomoku_state.cpp), standard rules (no Renju/Omok/pro-long).
struct State {
    static constexpr int NPLANES = 11;
    int bs, A;
    int NA() const { return A; }        // getActionSpaceSize
    std::vector<int8_t> cell;      // 0 empty, 1 black, 2 white
    int player = 1;                // current_player, BLACK=1 moves first (:20)
    std::vector<int> history;      // move_history (:718)
    int stones = 0;
    bool fresh = true;             // unordered_set never grown yet
    const Zobrist* z;
    State(int bs_, const Zobrist* z_) : bs(bs_), A(bs_ * bs_), cell(bs_ * bs_, 0), z(z_) {}

    // count_direction (gomoku_rules.cpp:98-115)
    int count_dir(int x, int y, int dx, int dy, int p) const {
        int c = 0;
        while (x >= 0 && x < bs && y >= 0 && y < bs && cell[x * bs + y] == p) { ++c; x += dx; y += dy; }
        return c;
    }
    // check_line_for_five (gomoku_rules.cpp:62-96): BLACK needs exactly 5, WHITE >= 5.
    bool five_at(int a, int p) const {
        if (cell[a] != p) return false;
        int x = a / bs, y = a % bs;
        static const int D[4][2] = {{0, 1}, {1, 0}, {1, 1}, {1, -1}};
        for (auto& d : D) {
            int len = count_dir(x, y, d[0], d[1], p) + count_dir(x, y, -d[0], -d[1], p) - 1;
            if (p == 1 ? len == 5 : len >= 5) return true;
        }
        return false;
    }
    // refresh_winner_cache (gomoku_state.cpp:477-489): full-board scan, BLACK first.
    int winner() const {
        for (int p : {1, 2})
            for (int a = 0; a < A; ++a)
                if (cell[a] == p && five_at(a, p)) return p;
        return 0;
    }
    // is_terminal (:491-504) / getGameResult (:189-201)
    GameResult result() const {
        int w = winner();
        if (w == 1) return WIN_P1;
        if (w == 2) return WIN_P2;
        if (stones >= A) return DRAW;   // is_stalemate: no empty cell (:506-521)
        return ONGOING;
    }
    bool terminal() const { return result() != ONGOING; }
    // get_valid_moves (:531-578): iteration order of the cached unordered_set<int>.
    // A fresh state's first query grows the set from one bucket (libstdc++ 11
    // prime rehash policy); every later refresh clears and re-inserts ascending into
    // a table with > A buckets, which iterates in strictly descending order.
    std::vector<int> legal() const {
        std::vector<int> out;
        if (fresh) {
            std::unordered_set<int> s;
            for (int a = 0; a < A; ++a) if (!cell[a]) s.insert(a);
            out.assign(s.begin(), s.end());
        } else {
            for (int a = A - 1; a >= 0; --a) if (!cell[a]) out.push_back(a);
        }
        return out;
    }
    // make_move (:681-722)
    void play(int a) {
        cell[a] = (int8_t)player;
        player = 3 - player;
        history.push_back(a);
        ++stones;
        fresh = false;
    }
    // compute_hash_signature (:620-656)
    uint64_t hash() const {
        uint64_t h = 0;
        for (int a = 0; a < A; ++a) {
            if (cell[a] == 1) h ^= z->piece[a];
            else if (cell[a] == 2) h ^= z->piece[A + a];
        }
        return h ^ z->player[player - 1];
    }
    // getEnhancedTensorRepresentation (:207-258, to_tensor :811-840, get_previous_moves :852-869)
    void planes(float* out) const {   // [11][bs][bs]
        std::fill(out, out + 11 * A, 0.0f);
        int me = player, opp = 3 - player;
        for (int a = 0; a < A; ++a) {
            if (cell[a] == me) out[a] = 1.0f;
            else if (cell[a] == opp) out[A + a] = 1.0f;
        }
        if (player == 1) for (int a = 0; a < A; ++a) out[2 * A + a] = 1.0f;
        for (int pl : {1, 2}) {   // BLACK list -> planes 3..5, WHITE list -> 6..8
            int found = 0;
            int n = (int)history.size();
            for (int i = n - 1; i >= 0 && found < 3; --i) {
                int mp = ((n - i) % 2 == 1) ? player : 3 - player;   // reference's parity rule (:860)
                if (mp == pl) { out[(pl == 1 ? 3 : 6) * A + found * A + history[i]] = 1.0f; ++found; }
            }
        }
        for (int x = 0; x < bs; ++x)
            for (int y = 0; y < bs; ++y) {
                out[9 * A + x * bs + y] = (float)x / (bs - 1);
                out[10 * A + x * bs + y] = (float)y / (bs - 1);
            }
    }
};

// ---------------------------------------------------------------------------
// GoState (src/games/go/go_state.cpp, go_rules.cpp) as created by GoState(bs, 7.5, true, true):
// komi 7.5, Chinese (area) scoring, positional superko, pass = -1, action space bs*bs + 1.
struct GoZobrist {
    std::vector<uint64_t> piece;        // [2][A]  ZobristHash(bs, 2, 2, seed) (patch P6)
    uint64_t player[2];
    std::vector<uint64_t> ko;           // addFeature("ko_point", A + 1) (go_state.cpp:49)
    uint64_t rules[2], komi[16];        // addFeature("rules", 2), addFeature("komi", 16)
    GoZobrist(int A, unsigned seed) : piece(2 * A), ko(A + 1) {
        std::mt19937_64 rng(seed);
        for (int p = 0; p < 2; ++p)
            for (int a = 0; a < A; ++a) piece[p * A + a] = rng();
        player[0] = rng(); player[1] = rng();
        // ZobristHash::addFeature (zobrist_hash.cpp:58-70): mt19937_64(std::hash<std::string>(name))
        std::mt19937_64 rk(std::hash<std::string>{}("ko_point"));
        for (int i = 0; i <= A; ++i) ko[i] = rk();
        std::mt19937_64 rr(std::hash<std::string>{}("rules"));
        for (auto& x : rules) x = rr();
        std::mt19937_64 rm(std::hash<std::string>{}("komi"));
        for (auto& x : komi) x = rm();
    }
};

struct GoState {
    static constexpr int NPLANES = 8;
    int bs, A;
    int NA() const { return A + 1; }                 // getActionSpaceSize (:330-332)
    std::vector<int8_t> cell;                        // board_ (0 / 1 black / 2 white), pos = y*bs + x
    int player = 1, ko = -1, passes = 0;
    int captured[3] = {0, 0, 0};
    std::vector<int> history;                        // move_history_ (passes as -1)
    std::vector<uint64_t> poshist;                   // position_history_ (non-pass moves only)
    const GoZobrist* z;
    float komi = 7.5f;
    GoState(int bs_, const GoZobrist* z_) : bs(bs_), A(bs_ * bs_), cell(bs_ * bs_, 0), z(z_) {}

    // getAdjacentPositions (:800-816): up, right, down, left
    int adj(int pos, int* out) const {
        int x = pos % bs, y = pos / bs, n = 0;
        if (y > 0) out[n++] = pos - bs;
        if (x + 1 < bs) out[n++] = pos + 1;
        if (y + 1 < bs) out[n++] = pos + bs;
        if (x > 0) out[n++] = pos - 1;
        return n;
    }
    // the group through `pos` on board b, and whether it has a liberty (go_rules.cpp:150-200)
    bool group(const std::vector<int8_t>& b, int pos, std::vector<int>& stones, std::vector<char>& seen) const {
        const int c = b[pos];
        stones.clear();
        stones.push_back(pos);
        seen[pos] = 1;
        bool lib = false;
        for (size_t i = 0; i < stones.size(); ++i) {
            int nb[4], k = adj(stones[i], nb);
            for (int j = 0; j < k; ++j) {
                if (b[nb[j]] == 0) lib = true;
                else if (b[nb[j]] == c && !seen[nb[j]]) { seen[nb[j]] = 1; stones.push_back(nb[j]); }
            }
        }
        return lib;
    }
    int count_libs(const std::vector<int8_t>& b, const std::vector<int>& stones) const {
        std::vector<char> l(A, 0);
        int n = 0;
        for (int s : stones) {
            int nb[4], k = adj(s, nb);
            for (int j = 0; j < k; ++j) if (b[nb[j]] == 0 && !l[nb[j]]) { l[nb[j]] = 1; ++n; }
        }
        return n;
    }
    // remove every libertyless group of colour c (findGroups + captureGroup); returns the stones
    std::vector<std::vector<int>> capture(std::vector<int8_t>& b, int c) const {
        std::vector<std::vector<int>> caps;
        std::vector<char> seen(A, 0);
        std::vector<int> st;
        for (int p = 0; p < A; ++p) {
            if (b[p] != c || seen[p]) continue;
            if (!group(b, p, st, seen)) caps.push_back(st);
        }
        for (auto& g : caps) for (int s : g) b[s] = 0;
        return caps;
    }
    // GoRules::isSuicidalMove (go_rules.cpp:27-136)
    bool suicidal(int a, int p) const {
        if (cell[a] != 0) return true;
        std::vector<int8_t> b = cell;
        b[a] = (int8_t)p;
        std::vector<char> seen(A, 0);
        std::vector<int> st;
        int nb[4], k = adj(a, nb);
        for (int j = 0; j < k; ++j)
            if (b[nb[j]] == 3 - p && !seen[nb[j]] && !group(b, nb[j], st, seen)) return false;
        std::fill(seen.begin(), seen.end(), 0);
        return !group(b, a, st, seen);
    }
    uint64_t board_hash(const std::vector<int8_t>& b) const {
        uint64_t h = 0;
        for (int a = 0; a < A; ++a) if (b[a]) h ^= z->piece[(b[a] - 1) * A + a];
        return h;
    }
    // updateHash (:846-877): stones ^ player ^ ko feature ^ rules(Chinese = 1) ^ komi(int(komi*2) & 15)
    uint64_t hash_of(const std::vector<int8_t>& b, int pl, int k) const {
        uint64_t h = board_hash(b) ^ z->player[pl - 1];
        if (k >= 0) h ^= z->ko[k % (A + 1)];
        h ^= z->rules[1];
        h ^= z->komi[((int)(komi * 2)) & 0xF];
        return h;
    }
    uint64_t hash() const { return hash_of(cell, player, ko); }
    // getLegalMoves (:116-160): pass first, then every valid point whose resulting position (same
    // side to move, the old ko point) is not in position_history_
    std::vector<int> legal() const {
        std::vector<int> out{-1};
        for (int a = 0; a < A; ++a) {
            if (cell[a] != 0 || a == ko || suicidal(a, player)) continue;
            std::vector<int8_t> b = cell;
            b[a] = (int8_t)player;
            capture(b, 3 - player);
            uint64_t h = hash_of(b, player, ko);
            if (std::find(poshist.begin(), poshist.end(), h) == poshist.end()) out.push_back(a);
        }
        return out;
    }
    // makeMove (:192-257)
    void play(int a) {
        if (a == -1) {
            ++passes;
            ko = -1;
            history.push_back(a);
        } else {
            passes = 0;
            cell[a] = (int8_t)player;
            auto caps = capture(cell, 3 - player);
            int n = 0;
            for (auto& g : caps) n += (int)g.size();
            ko = (caps.size() == 1 && caps[0].size() == 1) ? caps[0][0] : -1;
            captured[player] += n;
            history.push_back(a);
            poshist.push_back(hash());
        }
        player = 3 - player;
    }
    // GoRules::getTerritoryOwnership + calculateScores (go_rules.cpp:211-361), Chinese rules
    std::pair<float, float> score() const {
        std::vector<int> terr(A, 0);
        std::vector<char> vis(A, 0);
        for (int p = 0; p < A; ++p) {
            if (cell[p] != 0 || vis[p]) continue;
            std::vector<int> reg{p};
            vis[p] = 1;
            bool tb = false, tw = false;
            for (size_t i = 0; i < reg.size(); ++i) {
                int nb[4], k = adj(reg[i], nb);
                for (int j = 0; j < k; ++j) {
                    int s = cell[nb[j]];
                    if (s == 0) { if (!vis[nb[j]]) { vis[nb[j]] = 1; reg.push_back(nb[j]); } }
                    else if (s == 1) tb = true;
                    else tw = true;
                }
            }
            int col = (tb && !tw) ? 1 : (tw && !tb) ? 2 : 0;
            for (int r : reg) terr[r] = col;
        }
        for (int p = 0; p < A; ++p) if (cell[p]) terr[p] = cell[p];
        float bsc = 0.0f, wsc = 0.0f;
        for (int p = 0; p < A; ++p) {
            if (terr[p] == 1) bsc += 1.0f;
            else if (terr[p] == 2) wsc += 1.0f;
        }
        wsc += komi;
        return {bsc, wsc};
    }
    GameResult result() const {                     // getGameResult (:295-312)
        if (passes < 2) return ONGOING;
        auto sc = score();
        if (sc.first > sc.second) return WIN_P1;
        if (sc.second > sc.first) return WIN_P2;
        return DRAW;
    }
    bool terminal() const { return passes >= 2; }
    // getEnhancedTensorRepresentation (:338-420): black, white, black-to-move, black / white group
    // liberties min(1, libs/10), ko point, border distances x / y
    void planes(float* out) const {
        std::fill(out, out + 8 * A, 0.0f);
        for (int a = 0; a < A; ++a) {
            if (cell[a] == 1) out[a] = 1.0f;
            else if (cell[a] == 2) out[A + a] = 1.0f;
            out[2 * A + a] = player == 1 ? 1.0f : 0.0f;
        }
        std::vector<char> seen(A, 0);
        std::vector<int> st;
        for (int p = 0; p < A; ++p) {
            if (!cell[p] || seen[p]) continue;
            group(cell, p, st, seen);
            float l = std::min(1.0f, (float)count_libs(cell, st) / 10.0f);
            for (int s : st) out[(cell[p] == 1 ? 3 : 4) * A + s] = l;
        }
        if (ko >= 0) out[5 * A + ko] = 1.0f;
        for (int y = 0; y < bs; ++y)
            for (int x = 0; x < bs; ++x) {
                out[6 * A + y * bs + x] = (float)std::min(x, bs - 1 - x) / (bs / 2);
                out[7 * A + y * bs + x] = (float)std::min(y, bs - 1 - y) / (bs / 2);
            }
    }
};

// ---------------------------------------------------------------------------
// Evaluators
template <class S>
struct Evaluator {
    virtual ~Evaluator() {}
    virtual void eval(int game, const S& s, std::vector<float>& policy, float& value) = 0;
    long calls = 0;
};

// HashEvaluator (same definition as oracle/ref_harness.cpp hash_eval)
template <class S>
struct HashEval : Evaluator<S> {
    void eval(int, const S& s, std::vector<float>& p, float& v) override {
        ++this->calls;
        uint64_t key = splitmix64(s.hash() ^ 0x5A17C0DEULL);
        for (int i = 0; i < 6; ++i) {
            int m = (i < (int)s.history.size()) ? s.history[s.history.size() - 1 - i] : -1;
            key = splitmix64(key + (uint64_t)(uint32_t)(m + 2));
        }
        p.assign(s.NA(), 0.0f);
        for (int a = 0; a < s.NA(); ++a) {
            uint64_t r = splitmix64(key ^ ((uint64_t)(a + 1) * 0x9E3779B97F4A7C15ULL));
            p[a] = (float)(uint32_t)(r >> 40) * (1.0f / 16777216.0f);
        }
        uint64_t rv = splitmix64(key ^ 0x76A1ULL);
        v = ((float)(int32_t)(uint32_t)(rv >> 40) - 8388608.0f) * (1.0f / 8388608.0f);
    }
};

// RandomPolicyNetwork (src/nn/random_policy_network.cpp:9-24,93-138), one instance per game.
template <class State>
struct RandomEval : Evaluator<State> {
    std::vector<std::mt19937> rng;
    RandomEval(int games, unsigned seed) { for (int g = 0; g < games; ++g) rng.emplace_back(seed + g); }
    void eval(int game, const State& s, std::vector<float>& p, float& v) override {
        ++this->calls;
        std::uniform_real_distribution<float> dist(0.0f, 1.0f);
        const int NA = s.NA();
        p.assign(NA, 0.001f);
        float sum = 0.0f;
        auto legal = s.legal();
        for (int m : legal) if (m >= 0 && m < NA) { p[m] = dist(rng[game]); sum += p[m]; }
        if (sum > 0.0f) for (int i = 0; i < NA; ++i) p[i] /= sum;
        else if (!legal.empty()) { float u = 1.0f / (float)legal.size(); for (int m : legal) if (m >= 0) p[m] = u; }
        std::uniform_real_distribution<float> vd(-0.1f, 0.1f);
        v = vd(rng[game]);
    }
};

// No network: ParallelMCTS::evaluateState's fallback (src/mcts/parallel_mcts.cpp:903-916),
// 1/|legal| on the legal actions, value 0.
template <class S>
struct UniformEval : Evaluator<S> {
    void eval(int, const S& s, std::vector<float>& p, float& v) override {
        ++this->calls;
        p.assign(s.NA(), 0.0f);
        auto legal = s.legal();
        if (!legal.empty()) {
            const float u = 1.0f / (float)legal.size();
            for (int m : legal) if (m >= 0 && m < (int)p.size()) p[m] = u;
        }
        v = 0.0f;
    }
};

// Network evaluator through a user callback: planes -> raw logits [A] + value; the
// softmax of TorchNeuralNetwork::predictBatch (torch_neural_network.cpp:296-316) is
// applied here.  Replay evaluator: the callback returns final (post-softmax) policy.
typedef int (*az_eval_cb)(void* user, int game, const float* planes, int n_planes, int A,
                          float* policy_out, float* value_out);
// A callback returning 2 stops the play (bench.py's fixed CPU-baseline window); az_oracle_play
// then returns "null".
struct StopPlay {};
template <class S>
struct CallbackEval : Evaluator<S> {
    az_eval_cb cb; void* user; bool softmax;
    std::vector<float> buf;
    CallbackEval(az_eval_cb c, void* u, bool sm) : cb(c), user(u), softmax(sm) {}
    void eval(int game, const S& s, std::vector<float>& p, float& v) override {
        ++this->calls;
        buf.resize(S::NPLANES * s.A);
        s.planes(buf.data());
        p.assign(s.NA(), 0.0f);
        const int rc = cb(user, game, buf.data(), S::NPLANES, s.NA(), p.data(), &v);
        if (rc == 2) throw StopPlay{};
        if (rc != 0) { std::fprintf(stderr, "eval cb failed\n"); std::abort(); }
        if (softmax) {
            float mx = *std::max_element(p.begin(), p.end());
            float sum = 0.0f;
            for (auto& x : p) { x = std::exp(x - mx); sum += x; }
            if (sum > 0.0f) for (auto& x : p) x /= sum;
        }
    }
};

// ---------------------------------------------------------------------------
// TranspositionTable (src/mcts/transposition_table.cpp:44-191, 405-439) with the
// wall-clock age clause treated as never firing (ages < cacheEntryMaxAge = 60 s):
// replacement of an occupied slot happens iff its visitCount < minVisits (5).
struct TT {
    struct E { uint64_t hash; std::vector<float> policy; float value; int visits; };
    uint64_t mask;
    std::unordered_map<uint64_t, E> slots;
    long lookups = 0, hits = 0;
    explicit TT(int log2) : mask((1ULL << log2) - 1) {}
    bool lookup(uint64_t h, std::vector<float>& p, float& v) {
        ++lookups;
        auto it = slots.find(h & mask);
        if (it != slots.end() && it->second.hash == h) {
            p = it->second.policy; v = it->second.value; ++it->second.visits; ++hits;
            return true;
        }
        return false;
    }
    void store(uint64_t h, const std::vector<float>& p, float v) {
        auto it = slots.find(h & mask);
        if (it != slots.end()) {
            if (it->second.hash == h) { ++it->second.visits; return; }
            if (it->second.visits >= 5) return;   // collision, kept
        }
        E& e = slots[h & mask];
        e.hash = h; e.policy = p; e.value = v; e.visits = 1;
    }
};

// ---------------------------------------------------------------------------
// MCTSNode (include/alphazero/mcts/mcts_node.h:29-275) as a flat arena.
struct Node {
    int N = 0; float W = 0.0f; int VL = 0; float P = 0.0f;
    int action = -1, parent = -1, first = -1, nchild = 0;
    bool expanded = false, terminal = false;
    GameResult result = ONGOING;
};

struct Cfg {
    int bs = 9, sims = 100, max_moves = 1 << 30, vl = 3, noise_each_search = 0, temp_drop = 30;
    float cpuct = 1.5f, fpu = 0.0f, alpha = 0.03f, eps = 0.25f, t_init = 1.0f, t_final = 0.0f;
    unsigned noise_seed = 42, zobrist_seed = 12345;
    int tt_log2 = 20;
};

float convert_value(GameResult r, int player) {   // parallel_mcts.cpp:973-985
    switch (r) {
        case WIN_P1: return player == 1 ? 1.0f : -1.0f;
        case WIN_P2: return player == 2 ? 1.0f : -1.0f;
        default: return 0.0f;
    }
}

template <class State, class Zob>
struct Search {
    const Cfg& cfg;
    int game;
    Evaluator<State>* ev;
    TT tt;
    std::vector<Node> nodes;
    int root = 0;
    State rootState;
    std::mt19937 rng;
    Search(const Cfg& c, int g, Evaluator<State>* e, const Zob* z)
        : cfg(c), game(g), ev(e), tt(c.tt_log2), rootState(c.bs, z), rng(c.noise_seed) {
        nodes.emplace_back();     // root (parallel_mcts.cpp:68), parent = none
        nodes.reserve(1 << 16);
    }

    void add_vl(Node& n) { n.N += cfg.vl; n.VL += cfg.vl; n.W = n.W - (float)cfg.vl; }      // mcts_node.cpp:168-181
    void remove_vl(Node& n) { n.N -= cfg.vl; n.VL -= cfg.vl; n.W = n.W + (float)cfg.vl; }   // mcts_node.cpp:183-196

    // getPuctScore (mcts_node.cpp:61-119); `depth` of the node being selected FROM
    // relative to the current root decides the sign rule (:88-93).
    float puct(const Node& c, const Node& parentNode, int parentDepth, int parentVisits) const {
        int visits = c.N;
        if (visits == 0) return std::numeric_limits<float>::max();
        float q = 0.0f;
        int act = visits - c.VL;
        if (act > 0) q = c.W / (float)act;
        else q = 0.0f;
        if (parentDepth >= 1) {                 // parent && parent->parent
            bool flip = (parentDepth == 1);     // nodePlayer = parent->parent->parent ? cp : 3-cp
            if (flip) q = -q;
        }
        if (parentDepth >= 0 && act <= 0 && cfg.fpu > 0.0f) {   // c has a parent always
            int pa = parentNode.N - parentNode.VL;
            if (pa > 0) q = parentNode.W / (float)pa - cfg.fpu;
            else q = -cfg.fpu;
        }
        float sq = std::sqrt((float)parentVisits);
        float u = cfg.cpuct * c.P * sq / (1.0f + (float)visits);
        float div = 0.0f;
        if (visits < 5) div = 0.05f * (float)(5 - visits);
        return q + u + div;
    }

    // expandNodeWithPolicy (parallel_mcts.cpp:681-745)
    void expand(int ni, const State& s, const std::vector<float>& policy) {
        if (nodes[ni].expanded || nodes[ni].terminal) return;
        std::vector<int> legal = s.legal();
        if (legal.empty()) {
            nodes[ni].terminal = true; nodes[ni].result = s.result(); nodes[ni].expanded = true;
            return;
        }
        float sum = 0.0f;
        std::vector<float> lp(legal.size(), 0.0f);
        for (size_t i = 0; i < legal.size(); ++i) {
            int a = legal[i];
            if (a >= 0 && a < (int)policy.size()) { lp[i] = policy[a]; sum += lp[i]; }
        }
        if (sum > 0.0f) for (auto& x : lp) x /= sum;
        else { float u = 1.0f / (float)legal.size(); for (auto& x : lp) x = u; }
        int first = (int)nodes.size();
        for (size_t i = 0; i < legal.size(); ++i) {
            Node c; c.P = lp[i]; c.action = legal[i]; c.parent = ni;
            nodes.push_back(c);
        }
        nodes[ni].first = first; nodes[ni].nchild = (int)legal.size(); nodes[ni].expanded = true;
    }

    // evaluateState (parallel_mcts.cpp:835-917), direct-NN branch (Mode S)
    void evaluate(const State& s, std::vector<float>& p, float& v) {
        if (s.terminal()) {
            v = convert_value(s.result(), s.player);
            p.assign(s.NA(), 1.0f / (float)s.NA());
            return;
        }
        if (tt.lookup(s.hash(), p, v)) return;
        ev->eval(game, s, p, v);
    }

    // expandNode (parallel_mcts.cpp:636-679)
    void expand_node(int ni, const State& s) {
        if (nodes[ni].expanded || nodes[ni].terminal) return;
        if (s.legal().empty()) {
            nodes[ni].terminal = true; nodes[ni].result = s.result(); nodes[ni].expanded = true;
            return;
        }
        std::vector<float> p; float v;
        if (!tt.lookup(s.hash(), p, v)) { evaluate(s, p, v); tt.store(s.hash(), p, v); }
        expand(ni, s, p);
    }

    // runSingleSimulation (parallel_mcts.cpp:276-380) with selectLeafWithPath (:456-535)
    // and selectChildPuct (:537-563), backpropagate(node, value, path) (:782-833).
    void simulate() {
        State s = rootState;
        std::vector<int> path;
        int ni = root;
        add_vl(nodes[ni]);
        path.push_back(ni);
        int depth = 0;
        while (nodes[ni].expanded && !nodes[ni].terminal && depth < 1000) {
            const Node& n = nodes[ni];
            int pv = n.N;
            float best = -std::numeric_limits<float>::max();
            int bc = -1;
            for (int i = 0; i < n.nchild; ++i) {
                float sc = puct(nodes[n.first + i], n, depth, pv);
                if (sc > best) { best = sc; bc = n.first + i; }
            }
            if (bc < 0) break;
            s.play(nodes[bc].action);
            path.push_back(bc);
            ni = bc;
            ++depth;
        }
        for (int pi : path) add_vl(nodes[pi]);
        float value = 0.0f;
        Node& leaf = nodes[ni];
        if (leaf.terminal) {
            value = convert_value(leaf.result, s.player);
        } else if (s.terminal()) {
            value = convert_value(s.result(), s.player);
            leaf.terminal = true; leaf.result = s.result();
        } else {
            std::vector<float> p;
            if (tt.lookup(s.hash(), p, value)) {
                expand(ni, s, p);
            } else if (nodes[ni].expanded) {
                value = nodes[ni].N == 0 ? 0.0f : nodes[ni].W / (float)nodes[ni].N;
            } else {
                evaluate(s, p, value);
                tt.store(s.hash(), p, value);
                expand(ni, s, p);
            }
        }
        float v = value;
        for (auto it = path.rbegin(); it != path.rend(); ++it) {
            Node& n = nodes[*it];
            remove_vl(n);
            n.N += 1;
            n.W = n.W + v;
            v = -v;
        }
    }

    // addDirichletNoise (parallel_mcts.cpp:1110-1171)
    void add_noise(float alpha, float eps) {
        if (!nodes[root].expanded) expand_node(root, rootState);
        Node& r = nodes[root];
        if (r.nchild == 0) return;
        std::vector<float> noise(r.nchild);
        std::gamma_distribution<float> gamma(alpha, 1.0f);
        float sum = 0.0f;
        for (int i = 0; i < r.nchild; ++i) { noise[i] = std::max(1e-10f, gamma(rng)); sum += noise[i]; }
        if (sum <= 0.0f) { sum = 1.0f; for (auto& x : noise) x = 1.0f / (float)noise.size(); }
        for (auto& x : noise) x /= sum;
        for (int i = 0; i < r.nchild; ++i) {
            Node& c = nodes[r.first + i];
            c.P = (1.0f - eps) * c.P + eps * noise[i];
        }
    }

    // search (parallel_mcts.cpp:142-274), Mode S
    void search() {
        Node& r = nodes[root];
        if (!r.expanded && !rootState.terminal()) {
            std::vector<float> p; float v;
            evaluate(rootState, p, v);
            tt.store(rootState.hash(), p, v);
            expand(root, rootState, p);
        }
        if (cfg.noise_each_search && nodes[root].expanded) add_noise(cfg.alpha, cfg.eps);
        for (int i = 0; i < cfg.sims; ++i) simulate();
    }

    // getVisitCountDistribution (mcts_node.cpp:289-322)
    std::vector<float> probs(float T) const {
        const Node& r = nodes[root];
        std::vector<float> d(r.nchild, 0.0f);
        if (!r.expanded || r.nchild == 0) return {};
        float total = 0.0f;
        std::vector<float> c(r.nchild);
        for (int i = 0; i < r.nchild; ++i) {
            c[i] = std::pow((float)nodes[r.first + i].N, 1.0f / std::max(0.01f, T));
            total += c[i];
        }
        if (total > 0.0f) for (int i = 0; i < r.nchild; ++i) d[i] = c[i] / total;
        else { float u = 1.0f / (float)r.nchild; for (auto& x : d) x = u; }
        return d;
    }

    // selectAction (parallel_mcts.cpp:987-1047) with useBatchInference (deterministic)
    int select_action(bool training, float T) {
        if (!nodes[root].expanded) search();
        const Node& r = nodes[root];
        if (r.terminal || r.nchild == 0) {
            auto l = rootState.legal();
            return l.empty() ? -1 : l[0];
        }
        if (training && T > 0.0f) {
            auto d = probs(T);
            int bi = (int)(std::max_element(d.begin(), d.end()) - d.begin());
            return nodes[r.first + bi].action;
        }
        int mx = 0;
        for (int i = 0; i < r.nchild; ++i) mx = std::max(mx, nodes[r.first + i].N);
        for (int i = 0; i < r.nchild; ++i) if (nodes[r.first + i].N == mx) return nodes[r.first + i].action;
        return -1;
    }

    float root_value() const {   // getRootValue (:1057-1063) -> MCTSNode::getValue (mcts_node.h:80-85)
        const Node& r = nodes[root];
        if (r.nchild == 0) return 0.0f;
        return r.N == 0 ? 0.0f : r.W / (float)r.N;
    }

    // updateWithMove (parallel_mcts.cpp:1065-1108)
    void apply(int action) {
        const Node& r = nodes[root];
        int child = -1;
        for (int i = 0; i < r.nchild; ++i) if (nodes[r.first + i].action == action) { child = r.first + i; break; }
        rootState.play(action);
        if (child >= 0) { root = child; nodes[child].parent = -1; }
        else { nodes.emplace_back(); root = (int)nodes.size() - 1; }
    }

    void dump_children(std::ostringstream& o) const {
        const Node& r = nodes[root];
        o << "[";
        for (int i = 0; i < r.nchild; ++i) {
            const Node& c = nodes[r.first + i];
            o << (i ? "," : "") << "[" << c.action << "," << c.N << "," << c.VL << "," << fbits(c.W) << "," << fbits(c.P) << "]";
        }
        o << "]";
    }
};

char* dup(const std::string& s) {
    char* p = (char*)std::malloc(s.size() + 1);
    std::memcpy(p, s.c_str(), s.size() + 1);
    return p;
}

}  // namespace

extern "C" {

struct az_oracle_cfg {
    int bs, sims, max_moves, vl, noise_each_search, temp_drop, tt_log2, eval_kind;   // eval: 0 hash, 1 random, 2 net cb, 3 replay cb, 4 uniform
    float cpuct, fpu, alpha, eps, t_init, t_final;
    unsigned noise_seed, zobrist_seed, eval_seed;
    int n_games;
    int game;                                                                         // 0 Gomoku, 1 Go
};

void az_oracle_free(char* p) { std::free(p); }

}  // extern "C"

namespace {
template <class S, class Z>
void play_games(const az_oracle_cfg* c, const Cfg& cfg, const Z& z, Evaluator<S>* ev, int seed_stride, std::ostringstream& o) {
    for (int g = 0; g < c->n_games; ++g) {
        Cfg gc = cfg;
        gc.noise_seed = c->noise_seed + (unsigned)(seed_stride * g);
        Search<S, Z> m(gc, g, ev, &z);
        S st(cfg.bs, &z);           // SelfPlayManager's own state (self_play_manager.cpp:157)
        long evals0 = ev->calls;
        m.add_noise(cfg.alpha, cfg.eps);
        if (g) o << ",";
        o << "{\"mode\":\"game\",\"bs\":" << cfg.bs << ",\"sims\":" << cfg.sims << ",\"init_root\":";
        m.dump_children(o);
        o << ",\"moves\":[";
        int move = 0;
        while (!st.terminal() && move < cfg.max_moves) {
            m.search();
            float T = move >= cfg.temp_drop ? cfg.t_final : cfg.t_init;
            auto probs = m.probs(T);
            std::ostringstream kids; m.dump_children(kids);
            const Node& r = m.nodes[m.root];
            int rN = r.N, rVL = r.VL; uint32_t rW = fbits(r.W);
            int action = m.select_action(true, T);
            float value = m.root_value();
            if (move) o << ",";
            o << "{\"ply\":" << move << ",\"root\":[" << rN << "," << rVL << "," << rW << "],\"children\":" << kids.str()
              << ",\"probs\":[";
            for (size_t i = 0; i < probs.size(); ++i) o << (i ? "," : "") << fbits(probs[i]);
            o << "],\"action\":" << action << ",\"value\":" << fbits(value) << ",\"tt_lookups\":" << m.tt.lookups
              << ",\"tt_hits\":" << m.tt.hits << ",\"evals\":" << (ev->calls - evals0) << "}";
            st.play(action);
            m.apply(action);
            if (move % 2 == 0) m.add_noise(cfg.alpha, cfg.eps);
            ++move;
        }
        GameResult res = st.result();
        o << "],\"terminal\":" << (res != ONGOING ? 1 : 0) << ",\"result\":" << (int)res << "}";
    }
}
}  // namespace

extern "C" {

// Plays cfg->n_games independent games (game g uses noise seed noise_seed + g * seed_stride).
// Output: JSON identical in structure to oracle/ref_harness `game` mode, one document per game
// in a JSON array.
char* az_oracle_play(const az_oracle_cfg* c, int seed_stride, az_eval_cb cb, void* user) {
    Cfg cfg;
    cfg.bs = c->bs; cfg.sims = c->sims; cfg.max_moves = c->max_moves; cfg.vl = c->vl;
    cfg.noise_each_search = c->noise_each_search; cfg.temp_drop = c->temp_drop; cfg.tt_log2 = c->tt_log2;
    cfg.cpuct = c->cpuct; cfg.fpu = c->fpu; cfg.alpha = c->alpha; cfg.eps = c->eps;
    cfg.t_init = c->t_init; cfg.t_final = c->t_final;
    cfg.zobrist_seed = c->zobrist_seed;
    std::ostringstream o;
    o << "[";
    if (c->game == 1) {
        GoZobrist z(cfg.bs * cfg.bs, cfg.zobrist_seed);
        HashEval<GoState> he; CallbackEval<GoState> ne(cb, user, c->eval_kind == 2); UniformEval<GoState> ue;
        RandomEval<GoState> re(c->n_games, c->eval_seed);
        Evaluator<GoState>* ev = c->eval_kind == 0 ? (Evaluator<GoState>*)&he : c->eval_kind == 1 ? (Evaluator<GoState>*)&re
                               : c->eval_kind == 4 ? (Evaluator<GoState>*)&ue : (Evaluator<GoState>*)&ne;
        try { play_games<GoState, GoZobrist>(c, cfg, z, ev, seed_stride, o); } catch (const StopPlay&) { return dup("null"); }
    } else {
        Zobrist z(cfg.bs * cfg.bs, cfg.zobrist_seed);
        HashEval<State> he; RandomEval<State> re(c->n_games, c->eval_seed);
        CallbackEval<State> ne(cb, user, c->eval_kind == 2);
        UniformEval<State> ue;
        Evaluator<State>* ev = c->eval_kind == 0 ? (Evaluator<State>*)&he : c->eval_kind == 1 ? (Evaluator<State>*)&re
                             : c->eval_kind == 4 ? (Evaluator<State>*)&ue : (Evaluator<State>*)&ne;
        try { play_games<State, Zobrist>(c, cfg, z, ev, seed_stride, o); } catch (const StopPlay&) { return dup("null"); }
    }
    o << "]";
    return dup(o.str());
}

// Feature planes / hash / terminal / legal order for a move sequence (tests/golden positions).
int az_oracle_position(int bs, unsigned zobrist_seed, const int* moves, int n, float* planes_out,
                       uint64_t* hash_out, int* result_out, int* legal_out, int* n_legal) {
    Zobrist z(bs * bs, zobrist_seed);
    State s(bs, &z);
    for (int i = 0; i < n; ++i) s.play(moves[i]);
    if (planes_out) s.planes(planes_out);
    if (hash_out) *hash_out = s.hash();
    if (result_out) *result_out = (int)s.result();
    if (legal_out) { auto l = s.legal(); std::copy(l.begin(), l.end(), legal_out); *n_legal = (int)l.size(); }
    return 0;
}

// GoState after a move sequence: planes [8][A], hash, result, ko, legal order, board, score bits.
int az_oracle_go_position(int bs, unsigned zobrist_seed, const int* moves, int n, float* planes_out,
                          uint64_t* hash_out, int* result_out, int* ko_out, int* legal_out, int* n_legal,
                          int* board_out, float* score_out) {
    GoZobrist z(bs * bs, zobrist_seed);
    GoState s(bs, &z);
    for (int i = 0; i < n; ++i) s.play(moves[i]);
    if (planes_out) s.planes(planes_out);
    if (hash_out) *hash_out = s.hash();
    if (result_out) *result_out = (int)s.result();
    if (ko_out) *ko_out = s.ko;
    if (legal_out) { auto l = s.legal(); std::copy(l.begin(), l.end(), legal_out); *n_legal = (int)l.size(); }
    if (board_out) for (int a = 0; a < s.A; ++a) board_out[a] = s.cell[a];
    if (score_out) { auto sc = s.score(); score_out[0] = sc.first; score_out[1] = sc.second; }
    return 0;
}

// Initial-root child order of a fresh GomokuState.
int az_oracle_fresh_order(int bs, int* out) {
    std::unordered_set<int> s;
    for (int a = 0; a < bs * bs; ++a) s.insert(a);
    int i = 0;
    for (int a : s) out[i++] = a;
    return i;
}

// libstdc++ gamma_distribution<float>(alpha, 1) draws on mt19937(seed), one fresh
// distribution object per call (parallel_mcts.cpp:1137).
int az_oracle_gamma(unsigned seed, float alpha, int calls, int n, float* out) {
    std::mt19937 rng(seed);
    for (int c = 0; c < calls; ++c) {
        std::gamma_distribution<float> g(alpha, 1.0f);
        for (int i = 0; i < n; ++i) out[c * n + i] = g(rng);
    }
    return 0;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Dataset::extractExamples (src/selfplay/dataset.cpp:60-114) + augmentExample (:245-436), written
// the way the reference writes them (nested vectors, one copy-and-permute loop per transform,
// the policy permuted by board index under the oldIdx/newIdx < size guard), BEFORE the final
// shuffle (:112-113).  Examples are emitted per move: original, then the 7 augmentations.
// Chess is not restated (no rules here); variant rules are not supported.
namespace {
using Planes = std::vector<std::vector<std::vector<float>>>;
struct Example { Planes state; std::vector<float> policy; float value; };

template <class S>
Planes nested_planes(const S& s) {
    std::vector<float> flat((size_t)S::NPLANES * s.A);
    s.planes(flat.data());
    Planes st(S::NPLANES, std::vector<std::vector<float>>(s.bs, std::vector<float>(s.bs)));
    for (int p = 0; p < S::NPLANES; ++p)
        for (int i = 0; i < s.bs; ++i)
            for (int j = 0; j < s.bs; ++j) st[p][i][j] = flat[(size_t)p * s.A + i * s.bs + j];
    return st;
}

enum Tf { ROT90, ROT180, ROT270, FLIPH };
// one transform of augmentExample: state loop + policy loop (e.g. rot90 :262-287)
Example transform(const Example& in, Tf tf) {
    Example out = in;
    const size_t P = in.state.size(), bs = in.state[0].size();
    auto dest = [&](size_t i, size_t j, size_t& r, size_t& c) {
        switch (tf) {
            case ROT90: r = j; c = bs - 1 - i; break;
            case ROT180: r = bs - 1 - i; c = bs - 1 - j; break;
            case ROT270: r = bs - 1 - j; c = i; break;
            default: r = i; c = bs - 1 - j; break;
        }
    };
    for (size_t p = 0; p < P; ++p)
        for (size_t i = 0; i < bs; ++i)
            for (size_t j = 0; j < bs; ++j) { size_t r, c; dest(i, j, r, c); out.state[p][r][c] = in.state[p][i][j]; }
    out.policy.resize(in.policy.size());
    for (size_t i = 0; i < bs; ++i)
        for (size_t j = 0; j < bs; ++j) {
            size_t r, c;
            dest(i, j, r, c);
            const size_t oldIdx = i * bs + j, newIdx = r * bs + c;
            if (oldIdx < in.policy.size() && newIdx < out.policy.size()) out.policy[newIdx] = in.policy[oldIdx];
        }
    return out;
}

template <class S, class Z>
void extract_game(int bs, unsigned zseed, int n, const int* actions, const int* nch, const float* pol, int result,
                  bool augment, std::vector<Example>& ex) {
    Z z(bs * bs, zseed);
    S state(bs, &z);
    for (int i = 0; i < n; ++i) {
        if (i > 0) state.play(actions[i - 1]);
        Example e;
        e.state = nested_planes(state);
        e.policy.assign(pol, pol + nch[i]);
        pol += nch[i];
        float gameValue = 0.0f;
        if (result == WIN_P1) gameValue = 1.0f;
        else if (result == WIN_P2) gameValue = -1.0f;
        if (state.player == 2) gameValue = -gameValue;
        e.value = gameValue;
        ex.push_back(e);
        if (augment) {
            Example r90 = transform(e, ROT90), r180 = transform(e, ROT180), r270 = transform(e, ROT270);
            ex.push_back(r90);
            ex.push_back(r180);
            ex.push_back(r270);
            ex.push_back(transform(e, FLIPH));
            ex.push_back(transform(r90, FLIPH));
            ex.push_back(transform(r180, FLIPH));
            ex.push_back(transform(r270, FLIPH));
        }
    }
}
}  // namespace

extern "C" {
// game_type 0 Gomoku / 1 Go.  Outputs (pre-shuffle order): states [E][planes][bs][bs],
// policy [E][pstride] (zero past the length), plen [E], value [E].  Returns E or -1.
long long az_oracle_dataset(int game_type, int bs, int n_games, const int* n_moves, const int* actions,
                            const int* n_children, const float* policies, const int* results, int augment,
                            float* states_out, float* policy_out, int pstride, int* plen_out, float* value_out) {
    std::vector<Example> ex;
    for (int g = 0; g < n_games; ++g) {
        if (game_type == 1)
            extract_game<GoState, GoZobrist>(bs, 12345u, n_moves[g], actions, n_children, policies, results[g],
                                             augment != 0, ex);
        else if (game_type == 0)
            extract_game<State, Zobrist>(bs, 12345u, n_moves[g], actions, n_children, policies, results[g],
                                         augment != 0, ex);
        else
            return -1;
        for (int i = 0; i < n_moves[g]; ++i) policies += n_children[i];
        actions += n_moves[g];
        n_children += n_moves[g];
    }
    const int A = bs * bs;
    for (size_t e = 0; e < ex.size(); ++e) {
        const Example& x = ex[e];
        const size_t P = x.state.size();
        if (states_out)
            for (size_t p = 0; p < P; ++p)
                for (int i = 0; i < bs; ++i)
                    for (int j = 0; j < bs; ++j) states_out[(e * P + p) * A + i * bs + j] = x.state[p][i][j];
        if (policy_out) {
            for (int k = 0; k < pstride; ++k) policy_out[e * pstride + k] = k < (int)x.policy.size() ? x.policy[k] : 0.0f;
            plen_out[e] = (int)x.policy.size();
        }
        if (value_out) value_out[e] = x.value;
    }
    return (long long)ex.size();
}

// Dataset::shuffle's std::shuffle over n indices with std::mt19937(seed), `calls` times in a row
// on the same engine (dataset.cpp:147-149): out[c][i] = source index of slot i after call c.
int az_oracle_shuffle(unsigned seed, long long n, int calls, long long* out) {
    std::mt19937 rng(seed);
    for (int c = 0; c < calls; ++c) {
        std::vector<long long> idx((size_t)n);
        for (long long i = 0; i < n; ++i) idx[(size_t)i] = i;
        std::shuffle(idx.begin(), idx.end(), rng);
        std::copy(idx.begin(), idx.end(), out + (size_t)c * n);
    }
    return 0;
}
}  // extern "C"
