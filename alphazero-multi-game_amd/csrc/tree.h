// tree.h -- device-side data layout of the batched search (G independent games).
//
// Flat structure-of-arrays node pool per game (two arenas, compacted after every
// committed move), per-game root state, per-step scratch, a direct-mapped
// transposition-table emulation per game and a prior ring that keeps the children
// priors of every TT entry alive for later hits.  See DESIGN.md "Data layout in HBM".
#pragma once
#include <stddef.h>
#include <stdint.h>

#define AZ_MAXA 361          // largest board handled on device (19x19)
#define AZ_MAXNA 362         // largest action space (Go 19x19: 361 points + pass)
#define AZ_DMAX 96           // longest selection path (root + 95 plies); overflow => AZ_ERR_CAPACITY
#define AZ_NCNT 8            // per-game counters
// Go leaf state (k_select -> k_expand_backup): [0, 384) board, [384, 416) int32 {player, ko, passes,
// nph} + u64 stones hash, [416, 416 + 8 * AZ_DMAX) u64 position pushes of the path
#define AZ_GOLEAF_BYTES (416 + 8 * AZ_DMAX)

// ST_EXPANDED: the leaf is already expanded (a childless node after releaseMemory, or the depth
// cap): TT lookup, value = getValue() on a miss; ST_EXPVAL: the same with a TT hit (value cached)
enum { ST_NONE = 0, ST_TERMINAL = 1, ST_TTHIT = 2, ST_EVAL = 3, ST_EXPANDED = 4, ST_EXPVAL = 5 };
enum { MODE_SIM = 0, MODE_ROOT_NOISE = 1, MODE_ROOT_SEARCH = 2 };
enum { FL_EXPANDED = 1, FL_TERMINAL = 2 };   // result (GameResult) in bits 2..3
enum { CNT_EVALS = 0, CNT_LOOKUPS = 1, CNT_HITS = 2, CNT_SIMS = 3, CNT_NODES = 4, CNT_EVALS_TOTAL = 5,
       CNT_BYTES_SEL = 6, CNT_BYTES_EXP = 7 };   // [5..7] survive new games; 6/7: algorithmic HBM bytes of K1 / K3
enum { ERR_NODES = 1, ERR_PATH = 2, ERR_RING = 4, ERR_BATCH = 8, ERR_HIST = 16 };
enum { GAME_GOMOKU = 0, GAME_GO = 1 };

struct Nodes {          // one arena: [G][ncap]
    int* N; float* W; int* VL; float* P; int* first; int16_t* act; int16_t* cnt; uint8_t* flag;
};

struct TreeDev {
    int G, bs, A, ncap;
    int game;                    // GAME_GOMOKU / GAME_GO
    int NA;                      // action space = policy length = max children (A, Go: A + 1 with pass = -1)
    int vl; float cpuct, fpu;
    int eval_kind;
    uint64_t tt_mask; int tt_slots;
    int ring;
    Nodes nd;                    // current arena
    int* atop;                   // [G] next free node in the current arena
    uint8_t* rboard;             // [G][A]   root board, 0 empty 1 black 2 white
    int* rhist;                  // [G][6]   last moves, [0] most recent, -1 none
    int* rplayer; int* rstones; int* rply; uint64_t* rhash; int* rfresh; int* rnode;
    int* active;                 // [G] game searching (not finished)
    // Go root state (GoState): ko point, consecutive passes, position_history_ (hashes of the
    // positions after every stone move, go_state.cpp:250-252); rhash holds the stones-only hash
    int* rko; int* rpass; uint64_t* rposh; int* rnposh; int hmax;
    int pad0 = 0;                // explicit padding (zero): tree_dev() compares TreeDev variants bytewise
    const uint64_t* zko;         // [A + 1] "ko_point" feature keys
    uint64_t zconst;             // "rules"[1] ^ "komi"[int(7.5*2) & 15] (Chinese rules, komi 7.5)
    int* gresult;                // [G] GameResult of the root state
    int* path; int* plen;        // [G][AZ_DMAX], [G]
    int* pact;                   // [G][AZ_DMAX] action of every path node (pact[0] unused)
    int* lstatus; float* lvalue; uint64_t* lhash; int* ttstore; uint64_t* ttref; int* tthslot;
    int4* pstat;                 // [G][AZ_DMAX] path nodes' statistics after k_select's virtual loss {N, VL, W bits, leaf flag}
    int4* rhdr;                  // [G] the root's header {first, cnt, flag} as the last simulation's k_select ended
    int* need_eval; int* eval_slot; int* eval_games; int* n_eval;
    int eval_identity;           // 1: the batch maps are the identity (eval_slot[g] == g): no slot load
    int pad1 = 0;
    uint8_t* leafrec;            // [G][AZ_REC_BYTES] leaf records (leaf_planes.h): the planes' inputs (NET)
    uint8_t* goleaf;             // Go: [G][AZ_GOLEAF_BYTES] the selected leaf's position (board, side to move,
                                 // ko, passes, stones hash, the path's position pushes) for its expansion
    uint64_t* tt_hash; int* tt_visits; float* tt_value; uint64_t* tt_ref;   // [G][slots]
    float* ring_buf; uint64_t* ring_cur;                                     // [G][ring], [G]
    long long* cnt;              // [G][AZ_NCNT]
    const uint64_t* zpiece;      // [2][A]
    const uint64_t* zplayer;     // [2]
    const int* fresh_order;      // [A] first-query legal order of a fresh state
    uint32_t* mt;                // [G][625] mt19937 state + index (RANDOM evaluator)
    int* err;                    // [1] sticky error bits
    const float* net_logits;     // [B][A] (NET) raw policy logits, by eval slot
    const float* net_value;      // [B]
    int log_game, log_cap; float* log_pol; float* log_val; float* log_planes; int* log_n;
    int stamp_game;              // diagnostic: this game's k_select / k_expand_backup write phase stamps (-1 off)
    int pad2 = 0;
};
// no implicit padding: every byte of a TreeDev is a member (tree_dev() finds a variant with memcmp)
static_assert(offsetof(TreeDev, zko) == offsetof(TreeDev, pad0) + sizeof(int), "TreeDev hole after pad0");
static_assert(offsetof(TreeDev, leafrec) == offsetof(TreeDev, pad1) + sizeof(int), "TreeDev hole after pad1");
static_assert(sizeof(TreeDev) == offsetof(TreeDev, pad2) + sizeof(int), "TreeDev tail padding");
static_assert(offsetof(TreeDev, tt_mask) == 10 * sizeof(int), "TreeDev hole before tt_mask");

// Training-example extraction (Dataset::extractExamples + augmentExample).
// Records are flattened: game g owns moves [move_off[g], move_off[g+1]); move m owns policy
// floats [pol_off[m], pol_off[m] + n_children[m]).  Pre-shuffle example e = m * K + s (s = 0
// original, 1..7 the reference's augmentation order); dst[e] is its slot (null: e).
constexpr int AZ_DS_THREADS = 256;   // k_dataset_extract: one 4-wave block per game record (8 waves: no faster, Go slower)
struct DatasetDev {
    int game, bs, A, NA, C, K, n_games;
    const int* move_off;         // [n_games + 1]
    const int* actions;          // [M]
    const long long* pol_off;    // [M]
    const int* n_children;       // [M]
    const float* policies;       // [sum n_children]
    const int* results;          // [n_games] GameResult
    const long long* dst;        // [M * K] or null
    float* states;               // [E][C][A]   (state[plane][row][col], NCHW)
    float* policy;               // [E][NA]     child-order targets, zero past plen
    int* plen;                   // [E]
    float* value;                // [E]
};
