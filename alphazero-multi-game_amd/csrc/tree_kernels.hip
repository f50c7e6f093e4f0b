// tree_kernels.hip -- HIP kernels of the batched PUCT search (gfx950).
//
// One wavefront (64 lanes) per game.  Every fp32 operation that feeds the tree
// statistics is written in the reference's evaluation order and this file is
// compiled with -ffp-contract=off (no FMA contraction) and IEEE division/sqrt, so
// results are bit-identical to the reference CPU search:
//   k_select         ParallelMCTS::selectLeafWithPath + selectChildPuct + VL
//                    (src/mcts/parallel_mcts.cpp:456-563; mcts_node.cpp:61-119,168-196),
//                    leaf state (GomokuState::make_move, gomoku_state.cpp:681-722),
//                    terminal test (gomoku_rules.cpp:39-115), Zobrist hash (:620-656),
//                    TT lookup (transposition_table.cpp:44-84), feature planes (:207-258)
//   k_scan           deterministic compaction of the leaves that need the network
//   k_expand_backup  evaluator output -> softmax (torch_neural_network.cpp:296-316),
//                    TT store (:128-191), expandNodeWithPolicy (parallel_mcts.cpp:681-745),
//                    backpropagate(node, value, path) (:782-833)
//   k_select_action  getVisitCountDistribution (mcts_node.cpp:289-322), selectAction
//                    (parallel_mcts.cpp:987-1047), getRootValue (:1057-1063)
//   k_apply          makeMove + updateWithMove (parallel_mcts.cpp:1065-1108)
//   k_compact        subtree reuse: BFS copy of the new root's subtree into the other arena
//   k_noise          Dirichlet mix of addDirichletNoise (parallel_mcts.cpp:1158-1166)
#include <hip/hip_runtime.h>
#include <float.h>
#include <limits.h>
#include "tree.h"
#include "leaf_planes.h"

namespace {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

// sum_{i < n} x[i] in index order from 0.0f (the reference's sequential float loops) by lane 0,
// 16 values per step read as four ds_read_b128 ahead of their adds; x is 16-B aligned and padded
// with +0.0f to a multiple of 16 entries (adding +0.0f to a non-negative sum changes no bit).
// Returns the sum on lane 0 only.
__device__ __forceinline__ float seq_sum_lds(const float* x, int n) {
    float s = 0.0f;
    const float4* q = reinterpret_cast<const float4*>(x);
    const int nq = (n + 15) / 16;
    if (nq <= 0) return s;
    // the next 16 values are read while the current 16 are added (the add chain, not the LDS
    // latency, is then the critical path)
    float4 a = q[0], b = q[1], c = q[2], d = q[3];
    for (int j = 0; j < nq; ++j) {
        float4 na = a, nb = b, nc = c, nd = d;
        if (j + 1 < nq) { na = q[4 * j + 4]; nb = q[4 * j + 5]; nc = q[4 * j + 6]; nd = q[4 * j + 7]; }
        s += a.x; s += a.y; s += a.z; s += a.w;
        s += b.x; s += b.y; s += b.z; s += b.w;
        s += c.x; s += c.y; s += c.z; s += c.w;
        s += d.x; s += d.y; s += d.z; s += d.w;
        a = na; b = nb; c = nc; d = nd;
    }
    return s;
}

// Cross-lane reductions without the LDS crossbar: DPP moves inside each 16-lane row (xor 1, xor 2,
// half-mirror, mirror: after the four steps every lane of a row holds the row's result), then the
// four rows' results read into scalars.  A __shfl_xor butterfly is six dependent ds_bpermute round
// trips; this is four DPP VALU steps and four v_readlane.  The combine is a total order, so the
// result does not depend on the combining order.
template <int CTRL>
__device__ __forceinline__ int dpp_mov(int v) { return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, false); }
constexpr int DPP_XOR1 = 0xB1, DPP_XOR2 = 0x4E, DPP_HALF_MIRROR = 0x141, DPP_MIRROR = 0x140;

// (r0 + i) mod ring for r0 < ring and i < ring (search creation checks ring >= NA)
__device__ __forceinline__ uint32_t ring_wrap(uint32_t x, int ring) {
    return x >= (uint32_t)ring ? x - (uint32_t)ring : x;
}

__device__ __forceinline__ float wave_max(float v) {
    v = fmaxf(v, __int_as_float(dpp_mov<DPP_XOR1>(__float_as_int(v))));
    v = fmaxf(v, __int_as_float(dpp_mov<DPP_XOR2>(__float_as_int(v))));
    v = fmaxf(v, __int_as_float(dpp_mov<DPP_HALF_MIRROR>(__float_as_int(v))));
    v = fmaxf(v, __int_as_float(dpp_mov<DPP_MIRROR>(__float_as_int(v))));
    const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
    const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
    const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
    const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
    return fmaxf(fmaxf(r0, r1), fmaxf(r2, r3));
}

// first-max argmax over the wave: the largest score, ties to the smallest index (the reference's
// sequential first-max scan); returns wave-uniform (best, index)
__device__ __forceinline__ bool argmax_better(float s, int i, float bs, int bi) {
    return s > bs || (s == bs && i < bi);
}
template <int CTRL>
__device__ __forceinline__ void argmax_step(float& best, int& bi) {
    const float ob = __int_as_float(dpp_mov<CTRL>(__float_as_int(best)));
    const int oi = dpp_mov<CTRL>(bi);
    if (argmax_better(ob, oi, best, bi)) { best = ob; bi = oi; }
}
__device__ __forceinline__ void wave_argmax(float& best, int& bi) {
    argmax_step<DPP_XOR1>(best, bi);
    argmax_step<DPP_XOR2>(best, bi);
    argmax_step<DPP_HALF_MIRROR>(best, bi);
    argmax_step<DPP_MIRROR>(best, bi);
    float b = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(best), 0));
    int i = __builtin_amdgcn_readlane(bi, 0);
#pragma unroll
    for (int r = 1; r < 4; ++r) {
        const float ob = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(best), 16 * r));
        const int oi = __builtin_amdgcn_readlane(bi, 16 * r);
        if (argmax_better(ob, oi, b, i)) { b = ob; i = oi; }
    }
    best = b; bi = i;
}
// v from a wave-uniform lane (v_readlane, no LDS round trip), returned in a VGPR: these values
// live across the descent, where scalar registers are the kernel's tight resource (spills)
__device__ __forceinline__ int lane_bcast(int v, int src) {
    const int x = __builtin_amdgcn_readlane(v, __builtin_amdgcn_readfirstlane(src));
    int r;
    asm("v_mov_b32 %0, %1" : "=v"(r) : "s"(x));
    return r;
}
__device__ __forceinline__ float lane_bcast(float v, int src) {
    return __int_as_float(lane_bcast(__float_as_int(v), src));
}
// lane src's 64-bit value as a wave-uniform (scalar) value; src wave-uniform
__device__ __forceinline__ uint64_t lane_read64(uint64_t v, int src) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, src);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), src);
    return ((uint64_t)hi << 32) | lo;
}

// inclusive prefix sum across the wave
__device__ __forceinline__ int wave_incl_scan(int v, int lane) {
    for (int o = 1; o < 64; o <<= 1) {
        int t = __shfl_up(v, o);
        if (lane >= o) v += t;
    }
    return v;
}

// Diagnostic phase stamps (TreeDev.stamp_game >= 0, env AZ_TREE_STAMPS=<game>): [kernel][i] =
// s_memrealtime (100 MHz) in [0, 32), s_memtime (shader clock) in [32, 64); tools/tree_stamps.py.
__device__ unsigned long long g_tree_stamps[2][64];
__device__ __forceinline__ void tstamp(const TreeDev& t, int g, int k, int i) {
    if (g == t.stamp_game && threadIdx.x == 0) {
        g_tree_stamps[k][i] = __builtin_amdgcn_s_memrealtime();
        g_tree_stamps[k][32 + i] = __builtin_amdgcn_s_memtime();
    }
}

// GameResult (include/alphazero/core/igamestate.h:26-31)
enum { R_ONGOING = 0, R_DRAW = 1, R_WIN1 = 2, R_WIN2 = 3 };

// ParallelMCTS::convertToValue (parallel_mcts.cpp:973-985)
__device__ __forceinline__ float convert_value(int result, int player) {
    if (result == R_WIN1) return player == 1 ? 1.0f : -1.0f;
    if (result == R_WIN2) return player == 2 ? 1.0f : -1.0f;
    return 0.0f;
}

// count_direction / check_line_for_five (gomoku_rules.cpp:62-115): run through cell a.
__device__ int five_at(const uint8_t* board, int bs, int a, int p) {
    int x0 = a / bs, y0 = a % bs;
    const int D[4][2] = {{0, 1}, {1, 0}, {1, 1}, {1, -1}};
    for (int d = 0; d < 4; ++d) {
        int len = -1;
        for (int s = -1; s <= 1; s += 2) {
            int x = x0, y = y0;
            while (x >= 0 && x < bs && y >= 0 && y < bs && board[x * bs + y] == p) {
                ++len; x += s * D[d][0]; y += s * D[d][1];
            }
        }
        if (p == 1 ? len == 5 : len >= 5) return 1;
    }
    return 0;
}

// five_at over the wave: lanes 0..7 walk the 8 rays (4 directions x 2 sides) at once, each capped
// at 5 cells (1 + min(L,5) + min(R,5) is 5 exactly when the run is 5, and >= 5 exactly when it is).
// Every lane of the wave must call it (wave-uniform arguments).
__device__ int five_at_wave(const uint8_t* board, int bs, int a, int p, int lane) {
    const int x0 = a / bs, y0 = a % bs;
    int run = 0;
    if (lane < 8) {
        const int d = lane >> 1, sg = (lane & 1) ? 1 : -1;
        const int dx = d == 0 ? 0 : 1, dy = d == 0 ? 1 : d == 1 ? 0 : d == 2 ? 1 : -1;   // {0,1},{1,0},{1,1},{1,-1}
        int x = x0 + sg * dx, y = y0 + sg * dy;
        while (run < 5 && x >= 0 && x < bs && y >= 0 && y < bs && board[x * bs + y] == p) {
            ++run; x += sg * dx; y += sg * dy;
        }
    }
    const int other = __shfl_xor(run, 1);
    const int len = board[a] == p ? 1 + run + other : -1;
    const bool win = lane < 8 && (lane & 1) == 0 && (p == 1 ? len == 5 : len >= 5);
    return __ballot(win) != 0ULL;
}

// getPuctScore (mcts_node.cpp:61-119).  parentDepth: depth of the node being selected
// FROM (root = 0); the reference negates Q exactly when that node is at depth 1 (:88-93).
__device__ __forceinline__ float puct_score(int visits, float W, int VL, float P, int parentDepth, int pN, int pVL,
                                            float pW, float cpuct, float fpu, float sqrtPV) {
    if (visits == 0) return FLT_MAX;
    float q = 0.0f;
    int act = visits - VL;
    if (act > 0) q = W / (float)act;
    if (parentDepth == 1) q = -q;
    if (act <= 0 && fpu > 0.0f) {
        int pa = pN - pVL;
        q = pa > 0 ? pW / (float)pa - fpu : -fpu;
    }
    float u = cpuct * P * sqrtPV / (1.0f + (float)visits);
    float div = 0.0f;
    if (visits < 5) div = 0.05f * (float)(5 - visits);
    return q + u + div;
}

// HashEvaluator key (oracle/ref_harness.cpp hash_eval)
__device__ uint64_t hash_eval_key(uint64_t zhash, const int* hist6) {
    uint64_t key = splitmix64(zhash ^ 0x5A17C0DEULL);
    for (int i = 0; i < 6; ++i) key = splitmix64(key + (uint64_t)(uint32_t)(hist6[i] + 2));
    return key;
}
__device__ __forceinline__ float hash_eval_p(uint64_t key, int a) {
    uint64_t r = splitmix64(key ^ ((uint64_t)(a + 1) * 0x9E3779B97F4A7C15ULL));
    return (float)(uint32_t)(r >> 40) * (1.0f / 16777216.0f);
}
__device__ __forceinline__ float hash_eval_v(uint64_t key) {
    uint64_t rv = splitmix64(key ^ 0x76A1ULL);
    return ((float)(int32_t)(uint32_t)(rv >> 40) - 8388608.0f) * (1.0f / 8388608.0f);
}

// std::mt19937 (libstdc++ _M_gen_rand / operator()) for RandomPolicyNetwork.
__device__ uint32_t mt_next(uint32_t* st) {
    uint32_t* x = st;
    uint32_t& p = st[624];
    if (p >= 624) {
        const uint32_t up = 0x80000000u, lo = 0x7fffffffu;
        for (int k = 0; k < 624 - 397; ++k) {
            uint32_t y = (x[k] & up) | (x[k + 1] & lo);
            x[k] = x[k + 397] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        }
        for (int k = 624 - 397; k < 623; ++k) {
            uint32_t y = (x[k] & up) | (x[k + 1] & lo);
            x[k] = x[k + (397 - 624)] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        }
        uint32_t y = (x[623] & up) | (x[0] & lo);
        x[623] = x[396] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        p = 0;
    }
    uint32_t z = x[p++];
    z ^= (z >> 11) & 0xffffffffu;
    z ^= (z << 7) & 0x9d2c5680u;
    z ^= (z << 15) & 0xefc60000u;
    z ^= (z >> 18);
    return z;
}
// uniform_real_distribution<float>(a, b) over generate_canonical<float, 24>
__device__ float mt_uniform(uint32_t* st, float a, float b) {
    float c = (float)mt_next(st) / 4294967296.0f;
    if (c >= 1.0f) c = __uint_as_float(0x3F7FFFFFu);   // nextafter(1, 0)
    return (c * (b - a)) + a;
}

struct GamePtrs {
    int* N; float* W; int* VL; float* P; int* first; int16_t* act; int16_t* cnt; uint8_t* flag;
};
__device__ __forceinline__ GamePtrs game_nodes(const Nodes& nd, size_t base) {
    GamePtrs p;
    p.N = nd.N + base; p.W = nd.W + base; p.VL = nd.VL + base; p.P = nd.P + base;
    p.first = nd.first + base; p.act = nd.act + base; p.cnt = nd.cnt + base; p.flag = nd.flag + base;
    return p;
}

// Leaf state = root state + path moves: k_select and k_expand_backup build the Gomoku leaf board
// inline from the root board (loaded up front) and the path actions (sact[i], i = 1..depth):
// path cells are distinct, so the moves go down lane-parallel, and the Zobrist hash is the root
// hash XOR the moves' piece keys XOR the side-to-move keys (gomoku_state.cpp:620-656).

// The leaf record of a Gomoku leaf (leaf_planes.h): board, side to move, last six moves.
__device__ void write_leafrec(const TreeDev& t, int g, int lane, const uint8_t* board, const int* hist6, int player) {
    uint8_t* rec = t.leafrec + (size_t)g * AZ_REC_BYTES;
    for (int a = lane; a < t.A; a += 64) rec[a] = board[a];
    int* meta = reinterpret_cast<int*>(rec + AZ_REC_META);
    if (lane == 0) {
        meta[0] = player; meta[1] = -1;
#pragma unroll
        for (int i = 0; i < 6; ++i) meta[2 + i] = hist6[i];
    }
}

// ---------------------------------------------------------------------------
// Go (GoState as GoState(bs, 7.5, true, true): go_state.cpp / go_rules.cpp).  Rules code runs
// on lane 0 over the game's LDS board (a few hundred LDS operations per move; the network
// forward of the same step is four orders of magnitude longer); per-point work is lane-parallel.
struct GoLds {
    int16_t list[AZ_MAXA];       // BFS list / stack
    int16_t mark[AZ_MAXA];       // visit stamps
    int16_t gid[AZ_MAXA];        // group label of every stone: the group's smallest point (-1 empty)
    int glib[AZ_MAXA];           // distinct liberties of the group labelled l
    uint64_t gxor[AZ_MAXA];      // XOR of the group's piece keys
    uint64_t phist[AZ_DMAX];     // position hashes pushed along the selection path
    uint64_t pkey[AZ_DMAX];      // piece key of the stone path move i places (go_build_leaf prefetch)
    int nph, stamp;
};

__device__ __forceinline__ int go_adj(int pos, int bs, int A, int* nb) {   // getAdjacentPositions (:800-816)
    const int x = pos % bs;
    int n = 0;
    if (pos >= bs) nb[n++] = pos - bs;
    if (x + 1 < bs) nb[n++] = pos + 1;
    if (pos + bs < A) nb[n++] = pos + bs;
    if (x > 0) nb[n++] = pos - 1;
    return n;
}

__device__ void go_clear_marks(GoLds& L, int A, int lane) {
    for (int a = lane; a < A; a += 64) L.mark[a] = -1;
    if (lane == 0) L.stamp = 0;
    __syncthreads();
}

// makeMove (go_state.cpp:192-257) on lane 0: place, remove libertyless opponent groups (only
// groups adjacent to the new stone can have none), ko point, stones hash.  Returns 1 when the
// move pushes a position (stone moves), 0 for a pass.
// key (optional): the placed stone's piece key, already loaded (go_build_leaf prefetches a path's keys)
__device__ int go_play_seq(const TreeDev& t, uint8_t* b, GoLds& L, int a, int p, int& ko, int& passes, uint64_t& bh,
                           const uint64_t* key = nullptr) {
    const int bs = t.bs, A = t.A;
    if (a < 0) { ++passes; ko = -1; return 0; }
    passes = 0;
    b[a] = (uint8_t)p;
    bh ^= key ? *key : t.zpiece[(size_t)(p - 1) * A + a];
    const int opp = 3 - p;
    int ngroups = 0, nstones = 0, last = -1;
    int nb[4];
    const int k = go_adj(a, bs, A, nb);
    const int base = L.stamp;          // stamps of this call are > base
    for (int j = 0; j < k; ++j) {
        const int s0 = nb[j];
        if (b[s0] != opp || L.mark[s0] > base) continue;   // empty / own / group already examined
        const int st = ++L.stamp;
        int n = 0;
        L.list[n++] = (int16_t)s0;
        L.mark[s0] = (int16_t)st;
        bool lib = false;
        for (int i = 0; i < n; ++i) {
            int nb2[4];
            const int k2 = go_adj(L.list[i], bs, A, nb2);
            for (int q = 0; q < k2; ++q) {
                const int c = nb2[q];
                if (b[c] == 0) lib = true;
                else if (b[c] == opp && L.mark[c] != st) { L.mark[c] = (int16_t)st; L.list[n++] = (int16_t)c; }
            }
        }
        if (!lib) {
            for (int i = 0; i < n; ++i) {
                const int c = L.list[i];
                b[c] = 0;
                bh ^= t.zpiece[(size_t)(opp - 1) * A + c];
            }
            ++ngroups;
            nstones += n;
            last = L.list[0];
        }
    }
    ko = (ngroups == 1 && nstones == 1) ? last : -1;
    return 1;
}

// updateHash (go_state.cpp:846-877)
__device__ __forceinline__ uint64_t go_hash(const TreeDev& t, uint64_t bh, int player, int ko) {
    uint64_t h = bh ^ t.zplayer[player - 1];
    if (ko >= 0) h ^= t.zko[ko];
    return h ^ t.zconst;
}

// Piece keys of a wave's points (point a = lane + 64 i): of the stone on it (st) and of a stone of
// `player` on an empty point (pl, the superko candidates) -- all loads issued at once, one L2 round
// trip ahead of go_groups / go_legal, whose per-point loops otherwise waited for one per chunk.
constexpr int GO_PTS = (AZ_MAXA + 63) / 64;
struct GoKeys {
    uint64_t st[GO_PTS], pl[GO_PTS];
};
__device__ __forceinline__ void go_keys(const TreeDev& t, const uint8_t* b, int player, int lane, GoKeys& K) {
    const int A = t.A;
#pragma unroll
    for (int i = 0; i < GO_PTS; ++i) {
        const int a = lane + 64 * i;
        const int c = a < A ? b[a] : 0;
        K.st[i] = c ? t.zpiece[(size_t)(c - 1) * A + a] : 0ULL;
        K.pl[i] = (a < A && !c) ? t.zpiece[(size_t)(player - 1) * A + a] : 0ULL;
    }
}

// Every group of the board (visible to all threads after the call): label gid = the group's
// smallest point index (-1 on empty points), glib[label] its distinct liberties and, with keys (one
// wave: tid = lane, nthr = 64), gxor[label] the XOR of its piece keys.  Thread-parallel over the
// points (tid of nthr): min-label propagation with pointer jumping over same-colour neighbours until
// no label moves, then one liberty per (empty point, adjacent group) pair and one key per stone --
// integers, so the same results as a sequential flood fill (which held the lane-0 chain of dependent
// LDS / L2 accesses here).  The leaf record and the dataset planes need the liberties only.
__device__ void go_groups(const TreeDev& t, const uint8_t* b, GoLds& L, int tid, int nthr, const GoKeys* K = nullptr) {
    const int bs = t.bs, A = t.A;
    for (int a = tid; a < A; a += nthr) {
        L.gid[a] = b[a] ? (int16_t)a : (int16_t)-1;
        L.glib[a] = 0;
        if (K) L.gxor[a] = 0;
    }
    __syncthreads();
    for (;;) {
        bool moved = false;
        for (int a = tid; a < A; a += nthr) {
            const int c = b[a];
            if (!c) continue;
            int m = L.gid[a];
            int nb[4];
            const int k = go_adj(a, bs, A, nb);
            for (int q = 0; q < k; ++q)
                if (b[nb[q]] == c) m = min(m, (int)L.gid[nb[q]]);
            m = min(m, (int)L.gid[m]);                    // jump to the label's own label
            if (m < L.gid[a]) { L.gid[a] = (int16_t)m; moved = true; }
        }
        if (!__syncthreads_or(moved)) break;
    }
    if (K) {
#pragma unroll
        for (int i = 0; i < GO_PTS; ++i) {
            const int a = tid + 64 * i;
            if (a < A && b[a]) atomicXor(reinterpret_cast<unsigned long long*>(&L.gxor[L.gid[a]]), K->st[i]);
        }
    }
    for (int a = tid; a < A; a += nthr) {
        if (b[a]) continue;
        int nb[4], seen[4], ns = 0;
        const int k = go_adj(a, bs, A, nb);
        for (int q = 0; q < k; ++q) {
            if (!b[nb[q]]) continue;
            const int gl = L.gid[nb[q]];
            bool dup = false;
            for (int r = 0; r < ns; ++r) dup |= seen[r] == gl;
            if (!dup) { seen[ns++] = gl; atomicAdd(&L.glib[gl], 1); }
        }
    }
    __syncthreads();
}

// GoRules::getTerritoryOwnership + calculateScores, Chinese rules (go_rules.cpp:211-361) ->
// GameResult of a finished game (go_state.cpp:295-312).  Lane 0.
__device__ int go_result_seq(const TreeDev& t, const uint8_t* b, GoLds& L) {
    const int bs = t.bs, A = t.A;
    float bsc = 0.0f, wsc = 0.0f;
    const int st = ++L.stamp;
    for (int p0 = 0; p0 < A; ++p0) {
        if (b[p0] == 1) { bsc += 1.0f; continue; }
        if (b[p0] == 2) { wsc += 1.0f; continue; }
    }
    for (int p0 = 0; p0 < A; ++p0) {
        if (b[p0] != 0 || L.mark[p0] == st) continue;
        int n = 0;
        bool tb = false, tw = false;
        L.list[n++] = (int16_t)p0;
        L.mark[p0] = (int16_t)st;
        for (int i = 0; i < n; ++i) {
            int nb[4];
            const int k = go_adj(L.list[i], bs, A, nb);
            for (int q = 0; q < k; ++q) {
                const int e = nb[q];
                if (b[e] == 0) { if (L.mark[e] != st) { L.mark[e] = (int16_t)st; L.list[n++] = (int16_t)e; } }
                else if (b[e] == 1) tb = true;
                else tw = true;
            }
        }
        if (tb && !tw) bsc += (float)n;
        else if (tw && !tb) wsc += (float)n;
    }
    wsc += 7.5f;
    if (bsc > wsc) return R_WIN1;
    if (wsc > bsc) return R_WIN2;
    return R_DRAW;
}

// Leaf state of a Go game = root state + path moves (lane 0), with the position hashes the path
// pushes (for positional superko at expansion).
__device__ void go_build_leaf(const TreeDev& t, int g, int lane, const int* sact, int depth,
                              uint8_t* board, GoLds& L, int* hist6, int& player, int& ko, int& passes, uint64_t& bh,
                              uint64_t& hash) {
    const int A = t.A;
    const uint8_t* rb = t.rboard + (size_t)g * A;
    for (int a = lane; a < A; a += 64) board[a] = rb[a];
    go_clear_marks(L, A, lane);
    {   // the piece keys of the stones the path places, loaded lane-parallel ahead of the replay
        const int p0 = t.rplayer[g];
        for (int i = 1 + lane; i <= depth; i += 64) {
            const int a = sact[i];
            const int p = (i & 1) ? p0 : 3 - p0;
            L.pkey[i] = a >= 0 ? t.zpiece[(size_t)(p - 1) * A + a] : 0ULL;
        }
    }
    __syncthreads();
    if (lane == 0) {
        int p = t.rplayer[g], k = t.rko[g], ps = t.rpass[g];
        uint64_t h = t.rhash[g];
        int nph = 0;
        for (int i = 1; i <= depth; ++i) {
            const int a = sact[i];
            if (go_play_seq(t, board, L, a, p, k, ps, h, &L.pkey[i])) L.phist[nph++] = go_hash(t, h, p, k);
            p = 3 - p;
        }
        L.nph = nph;
        L.list[0] = (int16_t)p; L.list[1] = (int16_t)k; L.list[2] = (int16_t)ps;
        L.gxor[0] = h;
    }
    __syncthreads();
    player = L.list[0]; ko = L.list[1]; passes = L.list[2]; bh = L.gxor[0];
    __syncthreads();
    hash = go_hash(t, bh, player, ko);
    for (int i = 0; i < 6; ++i) {
        if (i < depth) hist6[i] = sact[depth - i];
        else hist6[i] = t.rhist[g * 6 + (i - depth)];
    }
}

// The selected Go leaf's position for its expansion (AZ_GOLEAF_BYTES per game): the expansion reads
// it back in one round trip instead of replaying the path's moves, captures and hashes on lane 0 a
// second time.  go_build_leaf must have run (board, L.phist / L.nph in LDS).
__device__ void go_store_leaf(const TreeDev& t, int g, int lane, const uint8_t* board, const GoLds& L, int player,
                              int ko, int passes, uint64_t bh) {
    uint8_t* dst = t.goleaf + (size_t)g * AZ_GOLEAF_BYTES;
    for (int a = lane; a < t.A; a += 64) dst[a] = board[a];
    const int nph = L.nph;
    uint64_t* ph = reinterpret_cast<uint64_t*>(dst + 416);
    for (int r = lane; r < nph; r += 64) ph[r] = L.phist[r];
    if (lane == 0) {
        int* meta = reinterpret_cast<int*>(dst + 384);
        meta[0] = player; meta[1] = ko; meta[2] = passes; meta[3] = nph;
        *reinterpret_cast<uint64_t*>(dst + 400) = bh;
    }
}
// go_build_leaf's results from the stored leaf state (same values: the replay is deterministic)
__device__ void go_load_leaf(const TreeDev& t, int g, int lane, const int* sact, int depth, uint8_t* board, GoLds& L,
                             int* hist6, int& player, int& ko, int& passes, uint64_t& bh, uint64_t& hash) {
    const int A = t.A;
    const uint8_t* src = t.goleaf + (size_t)g * AZ_GOLEAF_BYTES;
    const int* meta = reinterpret_cast<const int*>(src + 384);
    player = meta[0]; ko = meta[1]; passes = meta[2];
    const int nph = meta[3];
    bh = *reinterpret_cast<const uint64_t*>(src + 400);
    for (int a = lane; a < A; a += 64) board[a] = src[a];
    const uint64_t* ph = reinterpret_cast<const uint64_t*>(src + 416);
    for (int r = lane; r < nph; r += 64) L.phist[r] = ph[r];
    go_clear_marks(L, A, lane);
    if (lane == 0) L.nph = nph;
    __syncthreads();
    hash = go_hash(t, bh, player, ko);
    for (int i = 0; i < 6; ++i) {
        if (i < depth) hist6[i] = sact[depth - i];
        else hist6[i] = t.rhist[g * 6 + (i - depth)];
    }
}

// The leaf record of a Go leaf (leaf_planes.h; planes of go_state.cpp:338-420): board, side to
// move, ko point and min(10, group liberties) per stone (go_groups() must have run).
__device__ void go_write_leafrec(const TreeDev& t, int g, int lane, const uint8_t* b, const GoLds& L, int player, int ko) {
    uint8_t* rec = t.leafrec + (size_t)g * AZ_REC_BYTES;
    for (int a = lane; a < t.A; a += 64) {
        rec[a] = b[a];
        rec[AZ_REC_LIBS + a] = b[a] ? (uint8_t)min(10, (int)L.glib[L.gid[a]]) : 0;
    }
    int* meta = reinterpret_cast<int*>(rec + AZ_REC_META);
    if (lane == 0) meta[0] = player;
    if (lane == 1) meta[1] = ko;
    if (lane < 6) meta[2 + lane] = -1;
}

// getLegalMoves (go_state.cpp:116-160): pass, then every empty non-ko point that is not suicide
// (GoRules::isSuicidalMove) and whose resulting position -- same side to move, the old ko point --
// is not in position_history_ (root history + the path's pushes).  Needs go_groups().
__device__ int go_legal(const TreeDev& t, int g, int lane, const uint8_t* b, const GoLds& L, int player, int ko,
                        uint64_t bh, int* legal, const GoKeys& K) {
    const int A = t.A, bs = t.bs;
    const int opp = 3 - player;
    const uint64_t* rh = t.rposh + (size_t)g * t.hmax;
    const int nr = t.rnposh[g];
    const uint64_t tail = t.zplayer[player - 1] ^ (ko >= 0 ? t.zko[ko] : 0ULL) ^ t.zconst;
    if (lane == 0) legal[0] = -1;
    int n = 1;
    const uint64_t hv0 = lane < nr ? rh[lane] : 0ULL;      // the root history's first 64 positions, one per lane
#pragma unroll
    for (int ci = 0; ci < GO_PTS; ++ci) {
        const int c0 = 64 * ci;
        if (c0 >= A) break;
        const int a = c0 + lane;
        bool ok = a < A && b[a] == 0 && a != ko;
        uint64_t hc = 0;                                    // the candidate's resulting position
        if (ok) {
            int nb[4];
            const int k = go_adj(a, bs, A, nb);
            bool alive = false;
            int capg[4], nc = 0;
            uint64_t h = bh ^ K.pl[ci];
            for (int q = 0; q < k; ++q) {
                const int e = nb[q];
                const int v = b[e];
                if (v == 0) { alive = true; continue; }
                const int gi = L.gid[e];
                if (v == player) { if (L.glib[gi] >= 2) alive = true; continue; }
                if (L.glib[gi] == 1) {                // its only liberty is a: captured
                    bool dup = false;
                    for (int r = 0; r < nc; ++r) dup |= capg[r] == gi;
                    if (!dup) { capg[nc++] = gi; h ^= L.gxor[gi]; }
                }
            }
            ok = alive || nc > 0;
            hc = h ^ tail;
        }
        // positional superko, wave-uniform: every candidate against the root history (64 entries per
        // coalesced load, broadcast lane by lane -- not one dependent L2 round trip per entry) and
        // the path's pushes (LDS)
        if (__ballot(ok)) {
            for (int r0 = 0; r0 < nr; r0 += 64) {
                const uint64_t hv = r0 == 0 ? hv0 : (r0 + lane < nr ? rh[r0 + lane] : 0ULL);
                const int m = min(64, nr - r0);
                for (int j = 0; j < m; ++j) ok = ok && lane_read64(hv, j) != hc;
            }
            for (int r = 0; r < L.nph; ++r) ok = ok && L.phist[r] != hc;
        }
        const unsigned long long m = __ballot(ok);
        if (ok) legal[n + __popcll(m & ((1ULL << lane) - 1ULL))] = a;
        n += __popcll(m);
    }
    __syncthreads();
    return n;
}

}  // namespace

// ---------------------------------------------------------------------------
// K1: selection + virtual loss + leaf classification (+ planes for the network).
// K1.  IT = child records per lane per level (IT * 64 >= the action space).  Every level of the
// descent is ONE dependent round trip to memory: each lane loads all IT of its child records in
// full (N, W, VL, P and the child's own header first / cnt / flag / act) before the PUCT scores,
// and the winner's record is broadcast from its lane, so the next level needs no header load.
// What an expansion hands to the selection that follows it in the same wave (k_expand_select):
// the root's statistics after the backup and its header (first child, count, flag: from the
// root-header record k_select keeps, or as the expansion just set them), so the selection starts
// its descent without a round trip for the root.
struct RootHint {
    int valid;                   // the expansion's backup ran: the fields below are current
    int N, VL; float W;
    int first, cnt, flag;
};

// LDS of the selection and of the expansion: separate structs so that the fused k_expand_select
// overlays them (a union: the selection starts after the expansion's last LDS access and a block
// barrier) and shares one GoLds -- 12.3 KB per block instead of 21.1 KB, so 13 blocks fit a CU and
// C3's 2048 one-wave blocks (8 per CU) run in one round instead of two (7 per CU fitted at 21.1 KB)
struct SelLds {
    uint8_t board[AZ_MAXA];
    int spath[AZ_DMAX];
    int sact[AZ_DMAX];
    int sN[AZ_DMAX], sVL[AZ_DMAX];
    float sW[AZ_DMAX];
};
constexpr int EXP_NPAD = ((AZ_MAXNA + 63) / 64) * 64;   // pol / lp padded with +0.0f for seq_sum_lds
struct ExpLds {
    __attribute__((aligned(16))) float pol[EXP_NPAD];
    __attribute__((aligned(16))) float lp[EXP_NPAD];
    uint8_t board[AZ_MAXA];
    int spath[AZ_DMAX];
    int sact[AZ_DMAX];
    int legal[AZ_MAXNA];
    float s_scalar[2];
};

template <int IT>
__device__ __forceinline__ void select_game(const TreeDev& t, int mode, const RootHint* hint, SelLds& SL, GoLds& gl) {
    const int g = blockIdx.x;
    const int lane = threadIdx.x;
    auto& board = SL.board;
    auto& spath = SL.spath;
    auto& sact = SL.sact;
    auto& sN = SL.sN;
    auto& sVL = SL.sVL;
    auto& sW = SL.sW;
    const bool go = t.game == GAME_GO;
    if (g >= t.G) return;
    // per-game inputs that do not depend on the tree, loaded before anything waits
    constexpr int BK = (AZ_MAXA + 63) / 64;
    const int A = t.A;
    const int active = t.active[g];
    const int root = t.rnode[g];
    uint8_t rb[BK];
#pragma unroll
    for (int k = 0; k < BK; ++k) rb[k] = lane + 64 * k < A ? t.rboard[(size_t)g * A + lane + 64 * k] : 0;
    const int p0 = t.rplayer[g], rstones = t.rstones[g], gres = t.gresult[g];
    const uint64_t rhash = t.rhash[g], zpl0 = t.zplayer[0], zpl1 = t.zplayer[1];
    const int rhist = lane < 6 ? t.rhist[g * 6 + lane] : -1;
    long long* cnt = t.cnt + (size_t)g * AZ_NCNT;
    const long long c_look = cnt[CNT_LOOKUPS], c_hits = cnt[CNT_HITS], c_bytes = cnt[CNT_BYTES_SEL];
    tstamp(t, g, 0, 0);
    if (!active) {
        if (lane == 0) { t.lstatus[g] = ST_NONE; t.need_eval[g] = 0; }
        return;
    }
    const size_t base = (size_t)g * t.ncap;
    GamePtrs nd = game_nodes(t.nd, base);
    uint64_t zx = 0;             // XOR of the path moves' piece keys (Gomoku), loaded level by level
    int depth = 0;
    int node = root;
    int status = ST_NONE;
    float value = 0.0f;
    long long scanned = 0;       // child records read by the PUCT scans (25 B each)
    const bool hv = hint && hint->valid;
    int4 rhdr0 = int4{0, 0, 0, 0};
    uint8_t nflag = hv ? (uint8_t)hint->flag : nd.flag[root];   // flag of the current node (the leaf's after the descent)

    if (mode != MODE_SIM) {
        // Root expansion: expandNode (noise) / search() root branch.
        if ((nflag & (FL_EXPANDED | FL_TERMINAL)) || gres != R_ONGOING) {
            if (lane == 0) { t.lstatus[g] = ST_NONE; t.need_eval[g] = 0; }
            return;
        }
        if (lane == 0) spath[0] = root;
    } else {
        // selectLeafWithPath: VL on the root, then PUCT descent.
        int rN = hv ? hint->N : nd.N[root], rVL = hv ? hint->VL : nd.VL[root];
        float rW = hv ? hint->W : nd.W[root];
        int fc = hv ? hint->first : nd.first[root], nc = hv ? hint->cnt : nd.cnt[root];
        rhdr0 = int4{fc, nc, (int)nflag, 0};            // the root's header (its flag as it ends below)
        rN += t.vl; rVL += t.vl; rW = rW - (float)t.vl;           // addVirtualLoss (root, first)
        if (lane == 0) spath[0] = root;
        tstamp(t, g, 0, 1);
        int pN = rN, pVL = rVL;
        float pW = rW;
        while (true) {
            if (!(nflag & FL_EXPANDED) || (nflag & FL_TERMINAL) || depth >= 1000 || nc <= 0) break;
            scanned += nc;
            const float sq = sqrtf((float)pN);
            int cN[IT], cVL[IT], cF[IT], cC[IT], cA[IT], cFl[IT];
            float cW[IT], cP[IT];
#pragma unroll
            for (int k = 0; k < IT; ++k) {                 // all loads of the level before any use
                const int c = fc + min(lane + 64 * k, nc - 1);
                cN[k] = nd.N[c]; cW[k] = nd.W[c]; cVL[k] = nd.VL[c]; cP[k] = nd.P[c];
                cF[k] = nd.first[c]; cC[k] = nd.cnt[c]; cA[k] = nd.act[c]; cFl[k] = nd.flag[c];
            }
            float best = -FLT_MAX;
            int bi = INT_MAX, bk = 0;
#pragma unroll
            for (int k = 0; k < IT; ++k) {
                const int i = lane + 64 * k;
                if (i < nc) {
                    float s = puct_score(cN[k], cW[k], cVL[k], cP[k], depth, pN, pVL, pW, t.cpuct, t.fpu, sq);
                    if (s > best) { best = s; bi = i; bk = k; }
                }
            }
            int bN = cN[0], bVL = cVL[0], bF = cF[0], bC = cC[0], bA = cA[0], bFl = cFl[0];
            float bW = cW[0];
#pragma unroll
            for (int k = 1; k < IT; ++k)
                if (bk == k) { bN = cN[k]; bVL = cVL[k]; bF = cF[k]; bC = cC[k]; bA = cA[k]; bFl = cFl[k]; bW = cW[k]; }
            wave_argmax(best, bi);
            if (bi == INT_MAX) break;
            if (depth + 1 >= AZ_DMAX) { if (lane == 0) atomicOr(t.err, ERR_PATH); break; }
            const int src = bi & 63;
            pN = lane_bcast(bN, src); pVL = lane_bcast(bVL, src); pW = lane_bcast(bW, src);
            nflag = (uint8_t)lane_bcast(bFl, src);
            const int act = lane_bcast(bA, src);
            node = fc + bi;
            fc = lane_bcast(bF, src); nc = lane_bcast(bC, src);
            ++depth;
            // the node's statistics as loaded: its virtual loss below needs no second read
            if (lane == 0) { spath[depth] = node; sact[depth] = act; sN[depth] = pN; sVL[depth] = pVL; sW[depth] = pW; }
            // its piece key lands while the next level's records load (no extra round trip)
            if (!go) zx ^= t.zpiece[(size_t)((depth & 1) ? p0 - 1 : 2 - p0) * A + act];
        }
        tstamp(t, g, 0, 2);
        // addVirtualLoss on every path node, root a second time (parallel_mcts.cpp:293-295), on the
        // statistics the descent loaded (the wave is the tree's only writer); the post-VL values also
        // go to the path record (pstat), which the expansion's backup reads instead of the nodes
        int4* ps = t.pstat + (size_t)g * AZ_DMAX;
        if (lane == 0) {
            rN += t.vl; rVL += t.vl; rW = rW - (float)t.vl;
            nd.N[root] = rN; nd.VL[root] = rVL; nd.W[root] = rW;
            ps[0] = int4{rN, rVL, __float_as_int(rW), depth == 0 ? (int)nflag : 0};
        }
        __syncthreads();
        for (int i = 1 + lane; i <= depth; i += 64) {
            const int n = spath[i];
            const int N = sN[i] + t.vl, VL = sVL[i] + t.vl;
            const float W = sW[i] - (float)t.vl;
            nd.N[n] = N; nd.VL[n] = VL; nd.W[n] = W;
            ps[i] = int4{N, VL, __float_as_int(W), i == depth ? (int)nflag : 0};   // .w: the leaf's flag
        }
    }
    __syncthreads();

    int hist6[6];
    int player, stones = 0;
    uint64_t hash;
    int gko = -1, gpass = 0;
    uint64_t gbh = 0;
    if (go) {
        go_build_leaf(t, g, lane, sact, depth, board, gl, hist6, player, gko, gpass, gbh, hash);
        go_store_leaf(t, g, lane, board, gl, player, gko, gpass, gbh);
    } else {
        // leaf board = root board + path moves (distinct cells, lane-parallel); hash = root hash ^
        // the path's piece keys ^ the side-to-move keys (build_leaf, on registers already loaded)
#pragma unroll
        for (int k = 0; k < BK; ++k) if (lane + 64 * k < A) board[lane + 64 * k] = rb[k];
        __syncthreads();
        for (int i = 1 + lane; i <= depth; i += 64) board[sact[i]] = (uint8_t)((i & 1) ? p0 : 3 - p0);
        player = (depth & 1) ? 3 - p0 : p0;
        stones = rstones + depth;
        hash = rhash ^ zx ^ (p0 == 1 ? zpl0 : zpl1) ^ (player == 1 ? zpl0 : zpl1);
        for (int i = 0; i < 6; ++i) hist6[i] = i < depth ? sact[depth - i] : lane_bcast(rhist, i - depth);
        __syncthreads();
    }
    tstamp(t, g, 0, 3);
    const int leaf = node;
    int store = 0;
    uint64_t ref = 0;
    int hslot = 0;
    long long d_look = 0, d_hits = 0;   // counter increments (written once at the end)

    if (mode == MODE_SIM) {
        const uint8_t f = nflag;
        int result = R_ONGOING;
        if (f & FL_TERMINAL) {
            status = ST_TERMINAL;
            value = convert_value((f >> 2) & 3, player);
        } else {
            if (depth == 0) {
                result = gres;
            } else if (go) {
                // GoState::isTerminal: two consecutive passes; area score (go_state.cpp:291-312)
                if (gpass >= 2) {
                    int r = 0;
                    if (lane == 0) r = go_result_seq(t, board, gl);
                    result = lane_bcast(r, 0);
                }
            } else {
                const int a = sact[depth];
                if (five_at_wave(board, t.bs, a, 3 - player, lane)) result = (3 - player) == 1 ? R_WIN1 : R_WIN2;
                else if (stones >= t.A) result = R_DRAW;
            }
            if (result != R_ONGOING) {
                status = ST_TERMINAL;
                value = convert_value(result, player);
                if (lane == 0) nd.flag[leaf] = (uint8_t)(f | FL_TERMINAL | (result << 2));
                if (depth == 0) rhdr0.z = (int)(uint8_t)(f | FL_TERMINAL | (result << 2));
            } else if (f & FL_EXPANDED) {
                // an expanded leaf: a childless node (releaseMemory pruned its children) or the depth
                // cap.  runSingleSimulation still looks it up in the TT (parallel_mcts.cpp:319-335) and
                // takes the cached value on a hit (no re-expansion), node->getValue() otherwise (:340-344)
                const size_t tb = (size_t)g * t.tt_slots;
                const int hs = (int)(hash & t.tt_mask);
                const int vis = t.tt_visits[tb + hs];
                const uint64_t th = t.tt_hash[tb + hs];
                const float tv = t.tt_value[tb + hs];
                if (vis > 0 && th == hash) {
                    status = ST_EXPVAL;
                    value = tv;
                    if (lane == 0) t.tt_visits[tb + hs] = vis + 1;
                    d_look += 1; d_hits += 1;
                } else {
                    status = ST_EXPANDED;
                    d_look += 1;
                }
            }
        }
    } else if (!go && stones >= t.A) {
        // expandNode: no legal moves -> terminal (parallel_mcts.cpp:646-654); a Go state always
        // has the pass
        if (lane == 0) {
            nd.flag[leaf] = (uint8_t)(nflag | FL_TERMINAL | FL_EXPANDED | (R_DRAW << 2));   // no lookups: counters unchanged
            t.lstatus[g] = ST_NONE; t.need_eval[g] = 0;
        }
        return;
    }

    tstamp(t, g, 0, 4);
    if (status == ST_NONE) {
        // Transposition table (direct-mapped emulation, transposition_table.cpp:44-191)
        const size_t tb = (size_t)g * t.tt_slots;
        hslot = (int)(hash & t.tt_mask);
        const int vis = t.tt_visits[tb + hslot];     // the whole entry in one round trip
        const uint64_t th = t.tt_hash[tb + hslot];
        const float tv = t.tt_value[tb + hslot];
        const uint64_t tr = t.tt_ref[tb + hslot];
        const bool hit = vis > 0 && th == hash;
        if (hit) {
            status = ST_TTHIT;
            value = tv;
            ref = tr;
            if (lane == 0) t.tt_visits[tb + hslot] = vis + (mode == MODE_ROOT_SEARCH ? 2 : 1);
            d_look += 1; d_hits += 1;
        } else {
            status = ST_EVAL;
            store = (vis == 0 || vis < 5) ? 1 : 0;     // empty slot, or shouldReplace (visits < 5)
            d_look += (mode == MODE_ROOT_SEARCH ? 1 : 2);
            tstamp(t, g, 0, 5);
            if (go) {
                go_groups(t, board, gl, lane, 64);
                go_write_leafrec(t, g, lane, board, gl, player, gko);
            } else {
                write_leafrec(t, g, lane, board, hist6, player);
            }
        }
    }
    if (lane == 0) {
        t.lstatus[g] = status;
        t.lvalue[g] = value;
        t.lhash[g] = hash;
        t.ttstore[g] = store;
        t.ttref[g] = ref;
        t.tthslot[g] = hslot;
        t.plen[g] = depth + 1;
        t.need_eval[g] = (status == ST_EVAL && (t.eval_kind == 0 || t.eval_kind == 4)) ? 1 : 0;
        if (mode == MODE_SIM) t.rhdr[g] = rhdr0;        // the root-header record (the next expansion's hint)
    }
    for (int i = lane; i <= depth; i += 64) {
        t.path[(size_t)g * AZ_DMAX + i] = spath[i];
        t.pact[(size_t)g * AZ_DMAX + i] = i ? sact[i] : -1;
    }
    tstamp(t, g, 0, 6);
    if (lane == 0) { cnt[CNT_LOOKUPS] = c_look + d_look; cnt[CNT_HITS] = c_hits + d_hits; }
    if (lane == 0 && mode == MODE_SIM) {
        // algorithmic bytes: child scans (whole 25 B records: N, W, VL, P + the child's header),
        // root header (21 B), VL read-modify-write (12 B + 12 B) and piece key (8 B) per path
        // node, root board, TT probe (12 B, +20 on a hit), the leaf record (A board bytes + 32 B,
        // Go: + A liberty bytes) when the leaf goes to the network, path record (8 B per node)
        long long b = scanned * 25 + 21 + (long long)(depth + 1) * (24 + 8 + 8) + t.A + 12;
        if (status == ST_TTHIT) b += 20;
        if (status == ST_EVAL) b += (go ? 2LL : 1LL) * t.A + 32;
        cnt[CNT_BYTES_SEL] = c_bytes + b;
    }
    tstamp(t, g, 0, 7);
}

template <int IT>
__global__ __launch_bounds__(64) void k_select(const TreeDev* __restrict__ tp, int mode) {
    const TreeDev& t = *tp;                               // device-resident (tree_dev, engine.hip): an 8-byte kernarg
    __shared__ SelLds SL;
    __shared__ GoLds gl;
    select_game<IT>(t, mode, nullptr, SL, gl);
}

extern "C" int az_diag_tree_stamps(unsigned long long* out, int n) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tree_stamps), sizeof(unsigned long long) * (n < 128 ? n : 128)) == hipSuccess ? 0 : -1;
}

void az_launch_select(const TreeDev* t, int NA, int G, int mode, hipStream_t st) {
    if (NA <= 128) hipLaunchKernelGGL(k_select<2>, dim3(G), dim3(64), 0, st, t, mode);
    else if (NA <= 256) hipLaunchKernelGGL(k_select<4>, dim3(G), dim3(64), 0, st, t, mode);
    else hipLaunchKernelGGL(k_select<(AZ_MAXNA + 63) / 64>, dim3(G), dim3(64), 0, st, t, mode);
}

// Host evaluator: the moves from the root to every leaf of the evaluation batch (slot order).
__global__ void k_leaf_moves(TreeDev t, int* moves, int* len) {
    const int i = blockIdx.x;
    if (i >= *t.n_eval) return;
    const int g = t.eval_games[i];
    const int depth = t.plen[g] - 1;
    for (int j = threadIdx.x; j < depth; j += blockDim.x) moves[(size_t)i * AZ_DMAX + j] = t.pact[(size_t)g * AZ_DMAX + j + 1];
    if (threadIdx.x == 0) len[i] = depth;
}

// K2: deterministic compaction of the leaves that need the network (one block).
__global__ __launch_bounds__(1024) void k_scan(const TreeDev* __restrict__ tp) {
    const TreeDev& t = *tp;
    __shared__ int part[1024];
    const int tid = threadIdx.x;
    const int per = (t.G + 1023) / 1024;
    const int b0 = tid * per;
    int s = 0;
    for (int i = 0; i < per; ++i) { int g = b0 + i; if (g < t.G) s += t.need_eval[g]; }
    part[tid] = s;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        int v = tid >= o ? part[tid - o] : 0;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    int off = part[tid] - s;
    for (int i = 0; i < per; ++i) {
        int g = b0 + i;
        if (g < t.G) {
            if (t.need_eval[g]) { t.eval_slot[g] = off; t.eval_games[off] = g; ++off; }
            else t.eval_slot[g] = -1;
        }
    }
    if (tid == 1023) *t.n_eval = part[1023];
}

// K3: evaluator output -> TT store -> expansion -> backup.
// Latency layout: every per-game input (status, path, cached leaf value / hash / batch slot, root
// board, TT / ring / pool cursors, counters) is loaded before anything waits -- one round trip --
// then the leaf's network outputs and the path nodes' statistics -- the second and last one.
// The Gomoku leaf board is the root board plus the path moves (no Zobrist work: k_select stored
// the leaf hash); a Go leaf's position comes back from the state k_select stored (go_load_leaf).
__device__ __forceinline__ void expand_game(const TreeDev& t, int mode, ExpLds& EL, GoLds& gl, RootHint* hint = nullptr) {
    const int g = blockIdx.x;
    const int lane = threadIdx.x;
    if (hint && lane == 0) hint->valid = 0;
    constexpr int NPAD = EXP_NPAD;
    auto& board = EL.board;
    auto& spath = EL.spath;
    auto& sact = EL.sact;
    auto& pol = EL.pol;
    auto& legal = EL.legal;
    auto& lp = EL.lp;
    auto& s_scalar = EL.s_scalar;
    static_assert(AZ_DMAX <= 128, "two path entries per lane");
    constexpr int BK = (AZ_MAXA + 63) / 64, PK = (AZ_MAXNA + 63) / 64;
    const bool go = t.game == GAME_GO;
    if (g >= t.G) return;
    const int A = t.A, NA = t.NA;
    // ---- round trip 1
    const size_t pb = (size_t)g * AZ_DMAX;
    const int status = t.lstatus[g];
    const int plen = t.plen[g];
    const float lvalue = t.lvalue[g];
    const uint64_t lhash = t.lhash[g];
    const int slot = t.eval_identity ? g : t.eval_slot[g];
    const int pth0 = t.path[pb + lane], pac0 = t.pact[pb + lane];
    const int pth1 = lane < AZ_DMAX - 64 ? t.path[pb + 64 + lane] : 0;
    const int pac1 = lane < AZ_DMAX - 64 ? t.pact[pb + 64 + lane] : -1;
    // the path nodes' statistics as k_select left them (pstat; entries past the path are stale and
    // unused) and, with an identity batch, the leaf's network outputs: no second round trip
    const bool sim = mode == MODE_SIM;
    int4 ps0 = int4{0, 0, 0, 0}, ps1 = int4{0, 0, 0, 0};
    if (sim) {
        ps0 = t.pstat[pb + lane];
        if (lane < AZ_DMAX - 64) ps1 = t.pstat[pb + 64 + lane];
    }
    const int4 rh = sim ? t.rhdr[g] : int4{0, 0, 0, 0};   // the root's header as k_select left it
    int rfirst = rh.x, rcnt = rh.y, rflag = rh.z;
    const bool lg_early = t.eval_identity && (t.eval_kind == 0 || t.eval_kind == 4);
    float lg[PK];
    float netv = 0.0f;
    if (lg_early) {
        const float* src = t.net_logits + (size_t)g * NA;
#pragma unroll
        for (int k = 0; k < PK; ++k) lg[k] = lane + 64 * k < NA ? src[lane + 64 * k] : 0.0f;
        netv = t.net_value[g];
    }
    uint8_t rb[BK];
#pragma unroll
    for (int k = 0; k < BK; ++k) rb[k] = lane + 64 * k < A ? t.rboard[(size_t)g * A + lane + 64 * k] : 0;
    const int p0 = t.rplayer[g], rstones = t.rstones[g], rfresh = t.rfresh[g];
    const int atop = t.atop[g], ttstore = t.ttstore[g], tthslot = t.tthslot[g];
    const uint64_t ring_cur = t.ring_cur[g], ttref = t.ttref[g];
    long long* cnt = t.cnt + (size_t)g * AZ_NCNT;
    const long long c_ev = cnt[CNT_EVALS], c_evt = cnt[CNT_EVALS_TOTAL], c_sims = cnt[CNT_SIMS], c_bytes = cnt[CNT_BYTES_EXP];
    tstamp(t, g, 1, 0);
    if (status == ST_NONE) return;
    // the identity batch's logits were loaded in round trip 1: land them in LDS now, so their wait is
    // that round trip's (the compiler would otherwise sink the loads to the softmax)
    if (lg_early && status == ST_EVAL) {
#pragma unroll
        for (int k = 0; k < PK; ++k) if (lane + 64 * k < NA) pol[lane + 64 * k] = lg[k];
    }
    tstamp(t, g, 1, 1);
    const size_t base = (size_t)g * t.ncap;
    GamePtrs nd = game_nodes(t.nd, base);
    const int depth = plen - 1;
    // ---- round trip 2 (batches that are not the identity): the leaf's network outputs
    const bool net_in = status == ST_EVAL && (t.eval_kind == 0 || t.eval_kind == 4);
    if (net_in && !lg_early) {
        const float* src = t.net_logits + (size_t)slot * NA;
#pragma unroll
        for (int k = 0; k < PK; ++k) lg[k] = lane + 64 * k < NA ? src[lane + 64 * k] : 0.0f;
        netv = t.net_value[slot];
    }
    const int bN0 = ps0.x, bVL0 = ps0.y, bN1 = ps1.x, bVL1 = ps1.y;
    const float bW0 = __int_as_float(ps0.z), bW1 = __int_as_float(ps1.z);

    spath[lane] = pth0; sact[lane] = pac0;
    if (lane < AZ_DMAX - 64) { spath[64 + lane] = pth1; sact[64 + lane] = pac1; }
    int hist6[6]; int player; uint64_t hash = lhash;
    int gko = -1, gpass = 0;
    uint64_t gbh = 0;
    if (go) {
        __syncthreads();
        go_load_leaf(t, g, lane, sact, depth, board, gl, hist6, player, gko, gpass, gbh, hash);
    } else {
#pragma unroll
        for (int k = 0; k < BK; ++k) if (lane + 64 * k < A) board[lane + 64 * k] = rb[k];
        __syncthreads();
        if (lane >= 1 && lane <= depth) board[pac0] = (uint8_t)((lane & 1) ? p0 : 3 - p0);
        if (lane + 64 <= depth) board[pac1] = (uint8_t)(((lane + 64) & 1) ? p0 : 3 - p0);
        player = (depth & 1) ? 3 - p0 : p0;
        if (t.eval_kind == 1)
            for (int i = 0; i < 6; ++i) hist6[i] = i < depth ? sact[depth - i] : t.rhist[g * 6 + (i - depth)];
        __syncthreads();
    }
    tstamp(t, g, 1, 2);
    const int leaf = spath[depth];
    float value = lvalue;
    long long ev_add = 0;
    // algorithmic bytes: path (4 + 4 B per level), root board, then below: policy / TT / ring,
    // new child records (25 B), VL-removal + backup read-modify-write (24 B per path node)
    long long kb = (long long)plen * 8 + A;

    if (status == ST_EVAL || status == ST_TTHIT) {
        // legal moves in child order (gomoku_state.cpp:531-578)
        int n = 0;
        const bool fresh = !go && (depth == 0) && rfresh;
        if (go) {
            GoKeys gk;
            go_keys(t, board, player, lane, gk);
            go_groups(t, board, gl, lane, 64, &gk);
            n = go_legal(t, g, lane, board, gl, player, gko, gbh, legal, gk);
        } else if (fresh) {
            for (int i = lane; i < A; i += 64) legal[i] = t.fresh_order[i];
            n = A - rstones;   // fresh root is the empty board
        } else {
            for (int c0 = 0; c0 < A; c0 += 64) {
                const int a = A - 1 - (c0 + lane);
                const bool e = a >= 0 && board[a] == 0;
                const unsigned long long m = __ballot(e);
                const int pos = n + __popcll(m & ((1ULL << lane) - 1ULL));
                if (e) legal[pos] = a;
                n += __popcll(m);
            }
        }
        __syncthreads();
        tstamp(t, g, 1, 3);
        if (status == ST_EVAL || go) {
          if (status == ST_TTHIT) {
            // Go transposition hit: a position's legal set also depends on its history (superko),
            // so the ring keeps the cached policy itself (NA floats) and expandNodeWithPolicy's
            // gather is redone over the current legal set, as the reference does with entry.policy
            if (ring_cur - ttref > (uint64_t)t.ring) { if (lane == 0) atomicOr(t.err, ERR_RING); return; }
            const float* rbuf = t.ring_buf + (size_t)g * t.ring;
            const uint32_t r0 = (uint32_t)(ttref % (uint64_t)t.ring);
            for (int a = lane; a < NA; a += 64) pol[a] = rbuf[ring_wrap(r0 + a, t.ring)];
            __syncthreads();
          } else {
            ev_add = 1;
            if (t.eval_kind == 0) {
                float mx = -FLT_MAX;
#pragma unroll
                for (int k = 0; k < PK; ++k) if (lane + 64 * k < NA) mx = fmaxf(mx, lg[k]);
                tstamp(t, g, 1, 8);
                mx = wave_max(mx);
                tstamp(t, g, 1, 9);
                float e[PK];
#pragma unroll
                for (int k = 0; k < PK; ++k) {
                    e[k] = lane + 64 * k < NA ? expf(lg[k] - mx) : 0.0f;
                    pol[lane + 64 * k] = e[k];                 // +0.0f past NA
                }
                __syncthreads();
                tstamp(t, g, 1, 10);
                if (lane == 0) s_scalar[0] = seq_sum_lds(pol, NA);
                __syncthreads();
                tstamp(t, g, 1, 11);
                const float sum = s_scalar[0];
#pragma unroll
                for (int k = 0; k < PK; ++k)
                    if (lane + 64 * k < NA && sum > 0.0f) pol[lane + 64 * k] = e[k] / sum;
                value = netv;
                tstamp(t, g, 1, 4);
            } else if (t.eval_kind == 4) {
                // host evaluator (az_search_set_evaluator): the policy as NeuralNetwork::predict
                // returns it, used as is by expandNodeWithPolicy (parallel_mcts.cpp:886-901)
#pragma unroll
                for (int k = 0; k < PK; ++k) if (lane + 64 * k < NA) pol[lane + 64 * k] = lg[k];
                value = netv;
            } else if (t.eval_kind == 3) {
                // no network: 1/|legal| on the legal actions, value 0 (parallel_mcts.cpp:903-916)
                const float u = n > 0 ? 1.0f / (float)n : 0.0f;
                for (int a = lane; a < NA; a += 64) pol[a] = 0.0f;
                __syncthreads();
                for (int i = lane; i < n; i += 64) if (legal[i] >= 0) pol[legal[i]] = u;
                value = 0.0f;
            } else if (t.eval_kind == 1) {
                const uint64_t key = hash_eval_key(hash, hist6);
                for (int a = lane; a < NA; a += 64) pol[a] = hash_eval_p(key, a);
                value = hash_eval_v(key);
            } else {
                // RandomPolicyNetwork (random_policy_network.cpp:93-130): draws for legal a >= 0
                uint32_t* st = t.mt + (size_t)g * 625;
                for (int a = lane; a < NA; a += 64) pol[a] = 0.001f;
                __syncthreads();
                if (lane == 0) {
                    float sum = 0.0f;
                    for (int i = 0; i < n; ++i) {
                        if (legal[i] < 0) continue;
                        float u = mt_uniform(st, 0.0f, 1.0f); pol[legal[i]] = u; sum += u;
                    }
                    s_scalar[0] = sum;
                    s_scalar[1] = mt_uniform(st, -0.1f, 0.1f);
                }
                __syncthreads();
                const float sum = s_scalar[0];
                if (sum > 0.0f) for (int a = lane; a < NA; a += 64) pol[a] = pol[a] / sum;
                value = s_scalar[1];
            }
            __syncthreads();
            if (g == t.log_game && t.log_pol) {
                const int k = *t.log_n;
                if (k < t.log_cap) {
                    for (int a = lane; a < NA; a += 64) t.log_pol[(size_t)k * NA + a] = pol[a];
                    if (t.log_planes) {
                        const int npl = go ? 8 : 11;
                        const uint8_t* rec = t.leafrec + (size_t)g * AZ_REC_BYTES;
                        for (int a = lane; a < A; a += 64) {
                            float c[16];
                            az_leaf_planes(rec, go, t.bs, a, c);
#pragma unroll
                            for (int ch = 0; ch < 11; ++ch)
                                if (ch < npl) t.log_planes[((size_t)k * npl + ch) * A + a] = c[ch];
                        }
                    }
                    if (lane == 0) { t.log_val[k] = value; *t.log_n = k + 1; }
                }
            }
          }
            // expandNodeWithPolicy: gather, sequential sum, renormalise (parallel_mcts.cpp:702-724)
            float gv[PK];
#pragma unroll
            for (int k = 0; k < PK; ++k) {
                const int i = lane + 64 * k;
                gv[k] = i < n && legal[i] >= 0 ? pol[legal[i]] : 0.0f;   // pass: no prior
            }
#pragma unroll
            for (int k = 0; k < PK; ++k) lp[lane + 64 * k] = gv[k];   // +0.0f past n
            __syncthreads();
            tstamp(t, g, 1, 12);
            if (lane == 0) s_scalar[0] = seq_sum_lds(lp, n);
            __syncthreads();
            tstamp(t, g, 1, 13);
            const float ps = s_scalar[0];
            const float u = 1.0f / (float)n;
#pragma unroll
            for (int k = 0; k < PK; ++k)
                if (lane + 64 * k < n) lp[lane + 64 * k] = ps > 0.0f ? gv[k] / ps : u;
            tstamp(t, g, 1, 5);
        } else {
            // transposition hit: the stored priors are exactly the renormalised gather of
            // the cached policy over the same legal set (same position => same order).
            if (ring_cur - ttref > (uint64_t)t.ring) { if (lane == 0) atomicOr(t.err, ERR_RING); return; }
            const float* rbuf = t.ring_buf + (size_t)g * t.ring;
            const uint32_t r0 = (uint32_t)(ttref % (uint64_t)t.ring);
            for (int i = lane; i < n; i += 64) lp[i] = rbuf[ring_wrap(r0 + i, t.ring)];
        }
        __syncthreads();
        // TT store (new entry) + prior ring
        if (status == ST_EVAL && ttstore) {
            float* rbuf = t.ring_buf + (size_t)g * t.ring;
            const int len = go ? NA : n;            // Go keeps the policy, Gomoku the children priors
            const float* src = go ? pol : lp;
            const uint32_t r0 = (uint32_t)(ring_cur % (uint64_t)t.ring);
            for (int i = lane; i < len; i += 64) rbuf[ring_wrap(r0 + i, t.ring)] = src[i];
            if (lane == 0) {
                const size_t tb = (size_t)g * t.tt_slots + tthslot;
                t.tt_hash[tb] = hash; t.tt_visits[tb] = 1; t.tt_value[tb] = value; t.tt_ref[tb] = ring_cur;
                t.ring_cur[g] = ring_cur + (uint64_t)len;
            }
        }
        // create children (include/alphazero/mcts/mcts_node.h: N=W=VL=0, prior, action)
        if (atop + n > t.ncap) { if (lane == 0) atomicOr(t.err, ERR_NODES); return; }
        const int first = atop;
#pragma unroll
        for (int k = 0; k < PK; ++k) {                 // unrolled: the LDS reads of every chunk before the stores
            const int i = lane + 64 * k;
            if (i < n) {
                const int c = first + i;
                nd.N[c] = 0; nd.W[c] = 0.0f; nd.VL[c] = 0; nd.P[c] = lp[i];
                nd.first[c] = -1; nd.act[c] = (int16_t)legal[i]; nd.cnt[c] = 0; nd.flag[c] = 0;
            }
        }
        // the leaf's flag: k_select left it in the path record (a simulation step), else from the node
        const int lfw = lane_bcast(depth < 64 ? ps0.w : ps1.w, depth & 63);
        if (lane == 0) {
            t.atop[g] = first + n;
            const uint8_t fl = (uint8_t)((sim ? (uint8_t)lfw : nd.flag[leaf]) | FL_EXPANDED);
            nd.first[leaf] = first; nd.cnt[leaf] = (int16_t)n; nd.flag[leaf] = fl;
            cnt[CNT_NODES] = first + n;
            if (depth == 0) { rfirst = first; rcnt = n; rflag = fl; }   // the root was the leaf
        }
        kb += 25LL * n + 7 + 4LL * n + (status == ST_EVAL ? 4LL * NA + 4 + 24 : 0);
        tstamp(t, g, 1, 6);
    } else if (status == ST_EXPANDED) {
        value = nd.N[leaf] == 0 ? 0.0f : nd.W[leaf] / (float)nd.N[leaf];
    }   // ST_EXPVAL: the TT value k_select cached in lvalue

    if (sim) {
        // backpropagate(node, value, searchPath) (parallel_mcts.cpp:782-833): the reference walks the
        // path leaf -> root negating v at every step, so node i gets (-1)^(depth-i) * value.  Path
        // nodes are distinct and each gets its own unchanged sequence of fp32 operations, so the
        // update runs one lane per node (bit-identical to the sequential walk) on the statistics
        // loaded in round trip 2 (nothing in this kernel writes a path node's N / VL / W before).
        if (lane <= depth) {
            const float v = ((depth - lane) & 1) ? -value : value;
            int N = bN0 - t.vl, VL = bVL0 - t.vl;
            float W = bW0 + (float)t.vl;                   // removeVirtualLoss
            N += 1;
            W = W + v;
            nd.N[pth0] = N; nd.VL[pth0] = VL; nd.W[pth0] = W;
            if (hint && lane == 0) {                    // path[0]: the root
                hint->valid = 1; hint->N = N; hint->VL = VL; hint->W = W;
                hint->first = rfirst; hint->cnt = rcnt; hint->flag = rflag;
            }
        }
        if (lane + 64 <= depth) {
            const float v = ((depth - lane - 64) & 1) ? -value : value;
            int N = bN1 - t.vl, VL = bVL1 - t.vl;
            float W = bW1 + (float)t.vl;
            N += 1;
            W = W + v;
            nd.N[pth1] = N; nd.VL[pth1] = VL; nd.W[pth1] = W;
        }
        kb += 24LL * plen;
    }
    if (lane == 0) {
        if (ev_add) { cnt[CNT_EVALS] = c_ev + 1; cnt[CNT_EVALS_TOTAL] = c_evt + 1; }
        if (sim) { cnt[CNT_SIMS] = c_sims + 1; cnt[CNT_BYTES_EXP] = c_bytes + kb; }
    }
    tstamp(t, g, 1, 7);
}

__global__ __launch_bounds__(64) void k_expand_backup(const TreeDev* __restrict__ tp, int mode) {
    const TreeDev& t = *tp;
    __shared__ ExpLds EL;
    __shared__ GoLds gl;
    expand_game(t, mode, EL, gl);
}

// K3 of simulation step i and K1 of step i+1 in one launch: a game's expansion / backup and its
// next selection are the same wave's consecutive work (no other game is involved), so one
// kernel boundary per step goes (the wave's own global stores are visible to its later loads
// after the block barrier's release / acquire).  te: step i's batch maps, ts: the search's.
// One TreeDev argument (the kernel's scalar registers are the tight resource): the expansion's
// batch map differs from the search's only in eval_slot / eval_identity.
template <int IT>
__global__ __launch_bounds__(64) void k_expand_select(const TreeDev* __restrict__ tsp, const int* eval_slot, int eval_identity) {
    const TreeDev& ts = *tsp;
    __shared__ RootHint hint;
    __shared__ union PhaseLds { SelLds s; ExpLds e; } U;
    __shared__ GoLds gl;
    TreeDev te = ts;
    te.eval_slot = const_cast<int*>(eval_slot);
    te.eval_identity = eval_identity;
    expand_game(te, MODE_SIM, U.e, gl, &hint);
    __syncthreads();                                      // the expansion's LDS is the selection's from here
    select_game<IT>(ts, MODE_SIM, &hint, U.s, gl);
}

void az_launch_expand_select(const TreeDev* ts, const int* eval_slot, int eval_identity, int NA, int G, hipStream_t st) {
    if (NA <= 128) hipLaunchKernelGGL(k_expand_select<2>, dim3(G), dim3(64), 0, st, ts, eval_slot, eval_identity);
    else if (NA <= 256) hipLaunchKernelGGL(k_expand_select<4>, dim3(G), dim3(64), 0, st, ts, eval_slot, eval_identity);
    else hipLaunchKernelGGL(k_expand_select<(AZ_MAXNA + 63) / 64>, dim3(G), dim3(64), 0, st, ts, eval_slot, eval_identity);
}

// K4: visit distribution, action choice and root value per game.
__global__ __launch_bounds__(64) void k_select_action(const TreeDev* __restrict__ tp, int training, float temperature,
                                                      const float* temps, int* actions, float* values, float* probs,
                                                      int* child_actions, int* nchild) {
    const TreeDev& t = *tp;
    const int g = blockIdx.x;
    if (temps && g < t.G) temperature = temps[g];         // per-game schedule (self-play driver)
    const int lane = threadIdx.x;
    __shared__ float c[AZ_MAXNA];
    if (g >= t.G) return;
    const int A = t.A, NA = t.NA;
    const bool go = t.game == GAME_GO;
    if (!t.active[g]) {
        if (lane == 0) { actions[g] = go ? -2 : -1; values[g] = 0.0f; nchild[g] = 0; }
        return;
    }
    GamePtrs nd = game_nodes(t.nd, (size_t)g * t.ncap);
    const int root = t.rnode[g];
    const int fc = nd.first[root], nc = nd.cnt[root];
    const uint8_t f = nd.flag[root];
    if ((f & FL_TERMINAL) || nc == 0) {
        if (lane == 0) {
            // first legal move of the root state (parallel_mcts.cpp:994-1004)
            int a = -1;                                         // Go: the pass leads getLegalMoves
            const uint8_t* rb = t.rboard + (size_t)g * A;
            if (go) a = -1;
            else if (t.rfresh[g]) a = t.fresh_order[0];
            else for (int x = A - 1; x >= 0; --x) if (rb[x] == 0) { a = x; break; }
            actions[g] = a; values[g] = 0.0f; nchild[g] = 0;
        }
        return;
    }
    const float ex = 1.0f / fmaxf(0.01f, temperature);
    for (int i = lane; i < nc; i += 64) {
        const float Nf = (float)nd.N[fc + i];
        float v;
        if (ex == 1.0f) v = Nf;                                // pow(x, 1) == x exactly
        else v = (float)pow((double)Nf, (double)ex);
        c[i] = v;
        child_actions[(size_t)g * NA + i] = nd.act[fc + i];
    }
    __syncthreads();
    if (lane == 0) {
        float total = 0.0f;
        for (int i = 0; i < nc; ++i) total += c[i];
        float* pr = probs + (size_t)g * NA;
        if (total > 0.0f) for (int i = 0; i < nc; ++i) pr[i] = c[i] / total;
        else { const float u = 1.0f / (float)nc; for (int i = 0; i < nc; ++i) pr[i] = u; }
        int bi = 0;
        if (training && temperature > 0.0f) {
            for (int i = 1; i < nc; ++i) if (pr[bi] < pr[i]) bi = i;      // std::max_element
        } else {
            int mx = 0;
            for (int i = 0; i < nc; ++i) mx = max(mx, nd.N[fc + i]);
            for (int i = 0; i < nc; ++i) if (nd.N[fc + i] == mx) { bi = i; break; }
        }
        actions[g] = nd.act[fc + bi];
        const int rN = nd.N[root];
        values[g] = rN == 0 ? 0.0f : nd.W[root] / (float)rN;
        nchild[g] = nc;
    }
}

// updateWithMove's subtree reuse (parallel_mcts.cpp:1065-1108): the child that played `a`
// becomes the root, else a fresh root node.  Lane 0.
// returns the flag of the new root (0 for a fresh node)
__device__ uint8_t reuse_child(const TreeDev& t, int g, const GamePtrs& nd, int a) {
    const int root = t.rnode[g];
    const int fc = nd.first[root], nc = nd.cnt[root];
    int child = -1;
    for (int i = 0; i < nc; ++i) if (nd.act[fc + i] == a) { child = fc + i; break; }
    if (child < 0) {
        child = t.atop[g];
        if (child + 1 > t.ncap) { atomicOr(t.err, ERR_NODES); child = 0; }
        else t.atop[g] = child + 1;
        nd.N[child] = 0; nd.W[child] = 0.0f; nd.VL[child] = 0; nd.P[child] = 0.0f;
        nd.first[child] = -1; nd.act[child] = -1; nd.cnt[child] = 0; nd.flag[child] = 0;
        t.rnode[g] = child;
        return 0;
    }
    t.rnode[g] = child;
    return nd.flag[child];
}

// K5: makeMove + updateWithMove; terminal test of the new root (game loop condition).
// rexp[g] (optional): 1 when the game's root after the move needs no root expansion (expanded or
// terminal, or the game is not playing) -- the host then skips the no-op root steps
__global__ __launch_bounds__(64) void k_apply(TreeDev t, const int* actions, int* terminal, int* result, int* rexp) {
    const int g = blockIdx.x;
    const int lane = threadIdx.x;
    __shared__ uint8_t board[AZ_MAXA];
    __shared__ GoLds gl;
    if (g >= t.G) return;
    const int a = actions[g];
    const int A = t.A;
    const bool go = t.game == GAME_GO;
    if (!t.active[g] || a < (go ? -1 : 0) || a >= A) {          // Go: -1 is the pass
        if (lane == 0) {
            terminal[g] = t.active[g] ? 0 : 1; result[g] = t.gresult[g];
            if (rexp) rexp[g] = t.active[g] ? ((game_nodes(t.nd, (size_t)g * t.ncap).flag[t.rnode[g]] & (FL_EXPANDED | FL_TERMINAL)) != 0) : 1;
        }
        return;
    }
    GamePtrs nd = game_nodes(t.nd, (size_t)g * t.ncap);
    uint8_t* rb = t.rboard + (size_t)g * A;
    const int p = t.rplayer[g];
    for (int i = lane; i < A; i += 64) board[i] = rb[i];
    __syncthreads();
    if (go) {
        // GoState::makeMove (go_state.cpp:192-257)
        go_clear_marks(gl, A, lane);
        if (lane == 0) {
            int pp = p, k = t.rko[g], ps = t.rpass[g];
            uint64_t bh = t.rhash[g];
            if (go_play_seq(t, board, gl, a, pp, k, ps, bh)) {
                const int n = t.rnposh[g];
                if (n >= t.hmax) atomicOr(t.err, ERR_HIST);
                else { t.rposh[(size_t)g * t.hmax + n] = go_hash(t, bh, pp, k); t.rnposh[g] = n + 1; }
            }
            t.rhash[g] = bh; t.rko[g] = k; t.rpass[g] = ps; t.rplayer[g] = 3 - p;
            int* h = t.rhist + g * 6;
            for (int i = 5; i > 0; --i) h[i] = h[i - 1];
            h[0] = a;
            t.rstones[g] += a >= 0 ? 1 : 0;
            t.rply[g] += 1;
            t.rfresh[g] = 0;
            const int res = ps >= 2 ? go_result_seq(t, board, gl) : R_ONGOING;
            t.gresult[g] = res;
            if (res != R_ONGOING) t.active[g] = 0;
            terminal[g] = res != R_ONGOING;
            result[g] = res;
            const uint8_t fl = reuse_child(t, g, nd, a);
            if (rexp) rexp[g] = res != R_ONGOING || (fl & (FL_EXPANDED | FL_TERMINAL)) != 0;
        }
        __syncthreads();
        for (int i = lane; i < A; i += 64) rb[i] = board[i];
        return;
    }
    if (lane == 0) {
        board[a] = (uint8_t)p;
        rb[a] = (uint8_t)p;
        const int np = 3 - p;
        t.rhash[g] = t.rhash[g] ^ t.zpiece[(size_t)(p - 1) * A + a] ^ t.zplayer[p - 1] ^ t.zplayer[np - 1];
        int* h = t.rhist + g * 6;
        for (int i = 5; i > 0; --i) h[i] = h[i - 1];
        h[0] = a;
        t.rplayer[g] = np;
        const int stones = t.rstones[g] + 1;
        t.rstones[g] = stones;
        t.rply[g] += 1;
        t.rfresh[g] = 0;
        int res = R_ONGOING;
        if (five_at(board, t.bs, a, p)) res = p == 1 ? R_WIN1 : R_WIN2;
        else if (stones >= A) res = R_DRAW;
        t.gresult[g] = res;
        if (res != R_ONGOING) t.active[g] = 0;
        terminal[g] = res != R_ONGOING;
        result[g] = res;
        const uint8_t fl = reuse_child(t, g, nd, a);
        if (rexp) rexp[g] = res != R_ONGOING || (fl & (FL_EXPANDED | FL_TERMINAL)) != 0;
    }
}

// K6: copy the subtree of the (new) root into the other arena, breadth first.
// Subtree reuse: BFS copy of the new root's subtree into the other arena (children of a node stay
// contiguous and in order; node k of the copy came from src_of[k]).  One 256-thread block per game
// takes 256 queued nodes per round: a block prefix sum of their child counts places every child,
// and all the round's children are copied in parallel, each thread finding its parent by binary
// search over the prefix (one dependent round of loads per round instead of one per parent).
__global__ __launch_bounds__(256) void k_compact(TreeDev t, Nodes dst, int* src_of) {
    constexpr int NT = 256;
    __shared__ int s_inc[NT];     // inclusive prefix of this round's child counts
    __shared__ int s_fs[NT];      // first child (source arena) of each queued node
    __shared__ int s_wsum[NT / 64];
    const int g = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (g >= t.G) return;
    const size_t base = (size_t)g * t.ncap;
    GamePtrs s = game_nodes(t.nd, base);
    GamePtrs d = game_nodes(dst, base);
    int* so = src_of + base;
    const int root = t.rnode[g];
    if (tid == 0) {
        d.N[0] = s.N[root]; d.W[0] = s.W[root]; d.VL[0] = s.VL[root]; d.P[0] = s.P[root];
        d.act[0] = s.act[root]; d.cnt[0] = s.cnt[root]; d.flag[0] = s.flag[root]; d.first[0] = -1;
        so[0] = root;
    }
    __syncthreads();
    int j = 0, top = 1;
    while (j < top) {
        const int m = min(NT, top - j);
        const int k = j + tid;
        const bool valid = tid < m;
        const int sn = valid ? so[k] : 0;
        const int nc = valid ? (int)s.cnt[sn] : 0;
        const int fs = valid && nc ? s.first[sn] : 0;
        // block inclusive scan of nc
        const int wincl = wave_incl_scan(nc, lane);
        if (lane == 63) s_wsum[wave] = wincl;
        __syncthreads();
        int off = 0;
#pragma unroll
        for (int w = 0; w < NT / 64; ++w) off += w < wave ? s_wsum[w] : 0;
        const int incl = off + wincl;
        s_inc[tid] = incl;
        s_fs[tid] = fs;
        const int tot = s_wsum[0] + s_wsum[1] + s_wsum[2] + s_wsum[3];
        if (valid) d.first[k] = nc ? top + incl - nc : -1;
        __syncthreads();
        if (top + tot > t.ncap) { if (tid == 0) atomicOr(t.err, ERR_NODES); return; }
        for (int c = tid; c < tot; c += NT) {
            int lo = 0, hi = m - 1;                // smallest p with s_inc[p] > c
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (s_inc[mid] > c) hi = mid; else lo = mid + 1;
            }
            const int ex = lo ? s_inc[lo - 1] : 0;
            const int a = s_fs[lo] + (c - ex), b = top + c;
            d.N[b] = s.N[a]; d.W[b] = s.W[a]; d.VL[b] = s.VL[a]; d.P[b] = s.P[a];
            d.act[b] = s.act[a]; d.cnt[b] = s.cnt[a]; d.flag[b] = s.flag[a]; d.first[b] = -1;
            so[b] = a;
        }
        __syncthreads();                           // so[] of this round visible to the next (same CU)
        j += m;
        top += tot;
    }
    if (tid == 0) { t.rnode[g] = 0; t.atop[g] = top; }
}

// releaseMemory(visitThreshold) (parallel_mcts.cpp:1481-1496; MCTSNode::pruneTree mcts_node.cpp:451-477):
// BFS copy of the tree into the other arena keeping, below every node, only the children with
// visitCount >= threshold (in child order; the root itself stays).  A node whose children all go
// stays expanded with none.  pruned[g] = nodes before - nodes after (getTreeSize of every removed
// subtree: the arena holds exactly the tree).
__global__ __launch_bounds__(64) void k_prune(TreeDev t, Nodes dst, int* src_of, int thr_all, const int* thr_g,
                                              long long* pruned) {
    const int g = blockIdx.x;
    const int lane = threadIdx.x;
    if (g >= t.G) return;
    const int thr = thr_g ? thr_g[g] : thr_all;     // per game (0: keep every child, the whole tree)
    const size_t base = (size_t)g * t.ncap;
    GamePtrs s = game_nodes(t.nd, base);
    GamePtrs d = game_nodes(dst, base);
    int* so = src_of + base;
    const int root = t.rnode[g];
    const int before = t.atop[g];
    if (lane == 0) {
        d.N[0] = s.N[root]; d.W[0] = s.W[root]; d.VL[0] = s.VL[root]; d.P[0] = s.P[root];
        d.act[0] = s.act[root]; d.cnt[0] = s.cnt[root]; d.flag[0] = s.flag[root]; d.first[0] = -1;
        so[0] = root;
    }
    __syncthreads();
    int j = 0, top = 1;
    while (j < top) {
        const int k = j + lane;
        const bool valid = k < top;
        const int sn = valid ? so[k] : 0;
        const int fsrc = valid ? s.first[sn] : 0;
        const int ncs = valid ? (int)s.cnt[sn] : 0;
        int nc = 0;                                  // children this node keeps
        for (int i = 0; i < ncs; ++i) nc += s.N[fsrc + i] >= thr ? 1 : 0;
        const int incl = wave_incl_scan(nc, lane);
        const int tot = __shfl(incl, 63);
        const int nf = top + incl - nc;
        if (valid) { d.first[k] = nc ? nf : -1; d.cnt[k] = (int16_t)nc; }
        const int m = min(64, top - j);
        for (int e = 0; e < m; ++e) {
            const int ce = __shfl(ncs, e);
            if (__shfl(nc, e) == 0) continue;
            const int fs = __shfl(fsrc, e);
            int fd = __shfl(nf, e);
            if (fd + __shfl(nc, e) > t.ncap) { if (lane == 0) atomicOr(t.err, ERR_NODES); return; }
            for (int i0 = 0; i0 < ce; i0 += 64) {
                const int i = i0 + lane;
                const int a = fs + i;
                const bool keep = i < ce && s.N[a] >= thr;
                const unsigned long long bm = __ballot(keep);
                if (keep) {
                    const int b = fd + __popcll(bm & ((1ULL << lane) - 1ULL));
                    d.N[b] = s.N[a]; d.W[b] = s.W[a]; d.VL[b] = s.VL[a]; d.P[b] = s.P[a];
                    d.act[b] = s.act[a]; d.cnt[b] = s.cnt[a]; d.flag[b] = s.flag[a]; d.first[b] = -1;
                    so[b] = a;
                }
                fd += __popcll(bm);
            }
        }
        __syncthreads();
        j += m;
        top += tot;
    }
    if (lane == 0) {
        t.rnode[g] = 0; t.atop[g] = top;
        t.cnt[(size_t)g * AZ_NCNT + CNT_NODES] = top;
        pruned[g] = before - top;
    }
}

// K7: Dirichlet mix on the root children (noise already normalised on the host).
__global__ __launch_bounds__(64) void k_noise(TreeDev t, const float* noise, const uint8_t* mask, float eps) {
    const int g = blockIdx.x;
    const int lane = threadIdx.x;
    if (g >= t.G || !mask[g]) return;
    GamePtrs nd = game_nodes(t.nd, (size_t)g * t.ncap);
    const int root = t.rnode[g];
    const int fc = nd.first[root], nc = nd.cnt[root];
    const float* nz = noise + (size_t)g * t.NA;
    for (int i = lane; i < nc; i += 64) {
        const float old = nd.P[fc + i];
        nd.P[fc + i] = (1.0f - eps) * old + eps * nz[i];
    }
}

// K8: fresh games (empty board, new tree; TT visits cleared by the caller).
__global__ __launch_bounds__(64) void k_new_games(TreeDev t, const int* games, const int* seed_ids, int n,
                                                  uint32_t eval_seed) {
    const int idx = blockIdx.x;
    const int lane = threadIdx.x;
    if (idx >= n) return;
    const int g = games[idx];
    uint8_t* rb = t.rboard + (size_t)g * t.A;
    for (int i = lane; i < t.A; i += 64) rb[i] = 0;
    GamePtrs nd = game_nodes(t.nd, (size_t)g * t.ncap);
    long long* cnt = t.cnt + (size_t)g * AZ_NCNT;
    if (lane < CNT_EVALS_TOTAL) cnt[lane] = 0;
    if (lane < 6) t.rhist[g * 6 + lane] = -1;
    if (lane == 0) {
        t.rplayer[g] = 1; t.rstones[g] = 0; t.rply[g] = 0; t.rfresh[g] = 1;
        t.rhash[g] = t.game == GAME_GO ? 0ULL : t.zplayer[0];   // Go: stones-only hash of the empty board
        if (t.game == GAME_GO) { t.rko[g] = -1; t.rpass[g] = 0; t.rnposh[g] = 0; }
        t.rnode[g] = 0; t.atop[g] = 1; t.active[g] = 1; t.gresult[g] = R_ONGOING; t.ring_cur[g] = 0;
        nd.N[0] = 0; nd.W[0] = 0.0f; nd.VL[0] = 0; nd.P[0] = 0.0f; nd.first[0] = -1; nd.act[0] = -1;
        nd.cnt[0] = 0; nd.flag[0] = 0;
        if (t.mt) {
            // std::mt19937(seed + g) seeding (libstdc++ mersenne_twister_engine::seed)
            uint32_t* st = t.mt + (size_t)g * 625;
            st[0] = eval_seed + (uint32_t)(seed_ids ? seed_ids[idx] : g);
            for (int i = 1; i < 624; ++i) st[i] = 1812433253u * (st[i - 1] ^ (st[i - 1] >> 30)) + (uint32_t)i;
            st[624] = 624;
        }
    }
}

// Every slot of a new handle as an idle game: a valid root (node 0 of both arenas, no children),
// inactive.  Kernels that run over every slot (k_apply, k_compact, k_prune copy every game's tree
// when the arenas flip) then never read an uninitialised root index; k_new_games starts a game.
__global__ void k_init_slots(TreeDev t, Nodes other) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= t.G) return;
    t.rnode[g] = 0; t.atop[g] = 1; t.active[g] = 0; t.gresult[g] = R_ONGOING; t.ring_cur[g] = 0;
    t.rplayer[g] = 1; t.rstones[g] = 0; t.rply[g] = 0; t.rfresh[g] = 1; t.rhash[g] = 0;
    const Nodes* ar[2] = {&t.nd, &other};
    for (int k = 0; k < 2; ++k) {
        GamePtrs nd = game_nodes(*ar[k], (size_t)g * t.ncap);
        nd.N[0] = 0; nd.W[0] = 0.0f; nd.VL[0] = 0; nd.P[0] = 0.0f; nd.first[0] = -1; nd.act[0] = -1;
        nd.cnt[0] = 0; nd.flag[0] = 0;
    }
}

// TT clear for the listed games (visits == 0 marks an empty slot).
__global__ void k_tt_clear(TreeDev t, const int* games, int n) {
    const int idx = blockIdx.y;
    if (idx >= n) return;
    int* v = t.tt_visits + (size_t)games[idx] * t.tt_slots;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < t.tt_slots; i += gridDim.x * blockDim.x) v[i] = 0;
}

// Root children readback helper (tests / records).
__global__ void k_root_children(TreeDev t, int g, int* act, int* N, int* VL, float* W, float* P, int* n, int* rootinfo,
                                float* rootW) {
    GamePtrs nd = game_nodes(t.nd, (size_t)g * t.ncap);
    const int root = t.rnode[g];
    const int fc = nd.first[root], nc = nd.cnt[root];
    for (int i = threadIdx.x; i < nc; i += blockDim.x) {
        act[i] = nd.act[fc + i]; N[i] = nd.N[fc + i]; VL[i] = nd.VL[fc + i]; W[i] = nd.W[fc + i]; P[i] = nd.P[fc + i];
    }
    if (threadIdx.x == 0) { *n = nc; rootinfo[0] = nd.N[root]; rootinfo[1] = nd.VL[root]; *rootW = nd.W[root]; }
}

// Root child counts (host-side Dirichlet draws need |children| per game).
__global__ void k_root_nchild(TreeDev t, int* out) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= t.G) return;
    GamePtrs nd = game_nodes(t.nd, (size_t)g * t.ncap);
    const int root = t.rnode[g];
    out[g] = (nd.flag[root] & FL_EXPANDED) ? (int)nd.cnt[root] : 0;
}

// ---------------------------------------------------------------------------
// K-D: training examples (Dataset::extractExamples, src/selfplay/dataset.cpp:60-114, with
// augmentExample :245-436).  One wave per game replays the record (GomokuState / GoState
// makeMove on the LDS board), builds the position's planes in LDS (getEnhancedTensorRepresentation)
// and writes the K = 8 (or 1) examples of every position straight to their shuffled slots:
// no intermediate copy, HBM-bound on the example writes.
//
// Symmetry s maps a state pixel (row, col) to a destination; the kernel runs it backwards
// (src[s][dest]) so the writes are contiguous.  The reference's order: 0 original, 1 rot90
// (i,j)->(j,bs-1-i), 2 rot180, 3 rot270 (i,j)->(bs-1-j,i), 4 flipH (i,j)->(i,bs-1-j),
// 5..7 flipH applied to rot90 / rot180 / rot270 (:372-433).
namespace {
__device__ __forceinline__ int sym_src(int s, int a, int bs) {
    const int r = a / bs, c = a % bs, m = bs - 1;
    switch (s) {
        case 1: return (m - c) * bs + r;
        case 2: return (m - r) * bs + (m - c);
        case 3: return c * bs + (m - r);
        case 4: return r * bs + (m - c);
        case 5: return c * bs + r;
        case 6: return (m - r) * bs + c;
        case 7: return (m - c) * bs + (m - r);
        default: return a;
    }
}
}  // namespace

__global__ __launch_bounds__(AZ_DS_THREADS) void k_dataset_extract(DatasetDev d, TreeDev t) {
    const int g = blockIdx.x;
    const int lane = threadIdx.x;                 // AZ_DS_THREADS threads (4 waves) per game
    if (g >= d.n_games) return;
    const int bs = d.bs, A = d.A, C = d.C, K = d.K, NA = d.NA;
    __shared__ uint8_t board[AZ_MAXA];
    __shared__ float pl[11 * AZ_MAXA];          // planes of the current position, [C][A]
    __shared__ float pin[AZ_MAXNA];             // the move's child-order policy
    __shared__ int16_t src[8][AZ_MAXA];         // sym_src tables
    __shared__ GoLds L;
    __shared__ int hist6[6];
    __shared__ int s_ko;
    for (int a = lane; a < A; a += AZ_DS_THREADS) {
        board[a] = 0;
        for (int s = 0; s < K; ++s) src[s][a] = (int16_t)sym_src(s, a, bs);
    }
    if (lane < 6) hist6[lane] = -1;
    int player = 1, ko = -1, passes = 0;
    uint64_t bh = 0;
    // GameResult -> value of player 1 (:83-89); flipped for player 2 as -gameValue (-0.0f for draws)
    const int res = d.results[g];
    const float gv = res == R_WIN1 ? 1.0f : res == R_WIN2 ? -1.0f : 0.0f;
    const int m0 = d.move_off[g], m1 = d.move_off[g + 1];
    __syncthreads();
    for (int m = m0; m < m1; ++m) {
        // ---- planes of the position before move m
        if (d.game == GAME_GO) {
            go_clear_marks(L, A, lane);
            go_groups(t, board, L, lane, AZ_DS_THREADS);
            const float half = (float)(bs / 2);
            for (int a = lane; a < A; a += AZ_DS_THREADS) {
                const int v = board[a];
                const int x = a % bs, y = a / bs;
                pl[a] = v == 1 ? 1.0f : 0.0f;
                pl[A + a] = v == 2 ? 1.0f : 0.0f;
                pl[2 * A + a] = player == 1 ? 1.0f : 0.0f;
                const float lib = v ? fminf(1.0f, (float)L.glib[L.gid[a]] / 10.0f) : 0.0f;
                pl[3 * A + a] = v == 1 ? lib : 0.0f;
                pl[4 * A + a] = v == 2 ? lib : 0.0f;
                pl[5 * A + a] = a == ko ? 1.0f : 0.0f;
                pl[6 * A + a] = (float)min(x, bs - 1 - x) / half;
                pl[7 * A + a] = (float)min(y, bs - 1 - y) / half;
            }
        } else {
            int hp[6];
            for (int i = 0; i < 6; ++i) hp[i] = (((player == 1) == ((i % 2) == 0)) ? 3 : 6) + i / 2;
            for (int a = lane; a < A; a += AZ_DS_THREADS) {
                float c[11];
                for (int k = 0; k < 11; ++k) c[k] = 0.0f;
                const int v = board[a];
                if (v == player) c[0] = 1.0f;
                else if (v == 3 - player) c[1] = 1.0f;
                if (player == 1) c[2] = 1.0f;
                for (int i = 0; i < 6; ++i)
                    if (hist6[i] == a) c[hp[i]] = 1.0f;
                c[9] = (float)(a / bs) / (float)(bs - 1);
                c[10] = (float)(a % bs) / (float)(bs - 1);
                for (int k = 0; k < 11; ++k) pl[k * A + a] = c[k];
            }
        }
        const int n = d.n_children[m];
        const float* pg = d.policies + d.pol_off[m];
        for (int k = lane; k < n; k += AZ_DS_THREADS) pin[k] = pg[k];
        __syncthreads();
        const float val = player == 2 ? -gv : gv;
        for (int s = 0; s < K; ++s) {
            const long long e = (long long)m * K + s;
            const long long slot = d.dst ? d.dst[e] : e;
            float* o = d.states + slot * (long long)(C * A);
            for (int ca = lane; ca < C * A; ca += AZ_DS_THREADS) {
                const int c = ca / A, a = ca - c * A;
                o[ca] = pl[c * A + src[s][a]];
            }
            // policy: the reference permutes the child-order vector by board index, guarded by
            // oldIdx/newIdx < size; entries it does not overwrite keep the copied value
            float* op = d.policy + slot * (long long)NA;
            for (int k = lane; k < NA; k += AZ_DS_THREADS) {
                float v = 0.0f;
                if (k < n) {
                    if (s == 0) {
                        v = pin[k];
                    } else if (s <= 4) {
                        const int j = k < A ? src[s][k] : n;
                        v = (k < A && j < n) ? pin[j] : pin[k];
                    } else {
                        const int f = k < A ? src[4][k] : n;       // flip source, then the rotation
                        const int q = (k < A && f < n) ? f : k;
                        const int r = q < A ? src[s - 4][q] : n;
                        v = (q < A && r < n) ? pin[r] : pin[q];
                    }
                }
                op[k] = v;
            }
            if (lane == 0) { d.plen[slot] = n; d.value[slot] = val; }
        }
        __syncthreads();
        // ---- makeMove
        const int a = d.actions[m];
        if (d.game == GAME_GO) {
            go_clear_marks(L, A, lane);
            if (lane == 0) go_play_seq(t, board, L, a, player, ko, passes, bh);
        } else if (lane == 0) {
            board[a] = (uint8_t)player;
            for (int i = 5; i > 0; --i) hist6[i] = hist6[i - 1];
            hist6[0] = a;
        }
        player = 3 - player;
        if (lane == 0) s_ko = ko;
        __syncthreads();
        ko = s_ko;
    }
}

// Example gather (getBatch / getRandomSubset / shuffle): destination row i <- source row idx[i];
// one block per row, 16-byte copies when the row length allows.
__global__ __launch_bounds__(256) void k_dataset_gather(const float* states, const float* policy, const int* plen,
                                                        const float* value, int row, int NA, const long long* idx,
                                                        int n, float* ostates, float* opolicy, int* oplen,
                                                        float* ovalue) {
    const int i = blockIdx.x;
    if (i >= n) return;
    const long long j = idx[i];
    const float* s = states + j * row;
    float* o = ostates + (long long)i * row;
    if ((row & 3) == 0) {
        const float4* s4 = reinterpret_cast<const float4*>(s);
        float4* o4 = reinterpret_cast<float4*>(o);
        for (int k = threadIdx.x; k < row / 4; k += 256) o4[k] = s4[k];
    } else {
        for (int k = threadIdx.x; k < row; k += 256) o[k] = s[k];
    }
    for (int k = threadIdx.x; k < NA; k += 256) opolicy[(long long)i * NA + k] = policy[j * NA + k];
    if (threadIdx.x == 0) { oplen[i] = plen[j]; ovalue[i] = value[j]; }
}
