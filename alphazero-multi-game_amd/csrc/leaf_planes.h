// leaf_planes.h -- the leaf record: what k_select stores for a leaf that needs the network, and the
// feature planes every consumer synthesises from it.
//
// A leaf's feature planes (Gomoku getEnhancedTensorRepresentation, gomoku_state.cpp:207-258; Go
// go_state.cpp:338-420) are a function of a few hundred bytes of state: the board, the side to
// move, the last six moves (Gomoku) or the ko point and every stone's group liberties (Go).  The
// search stores that record per game (AZ_REC_BYTES, 0.8 KB instead of A x 16 fp32 = 14.4 KB at
// 15x15) and the network's input stage (k_smallnet, k_rec_to_g8) -- or, for the f32 input path and
// the host evaluator, k_rec_planes -- builds the 16 NHWC channels of every cell on the fly.  Every
// value is produced by the same fp32 expressions as before (0 / 1, x / (bs - 1), min(1, libs / 10),
// min(x, bs - 1 - x) / (bs / 2)), so the planes are bit-identical wherever they are built.
#pragma once
#include <stdint.h>

constexpr int AZ_REC_LIBS = 384;     // Go: min(10, liberties of the cell's group) per cell (u8)
constexpr int AZ_REC_META = 768;     // int32: [0] side to move, [1] ko point (Go, -1 none), [2..7] last six moves
constexpr int AZ_REC_BYTES = 800;    // per game (a multiple of 16)

// The 16 NHWC channels of cell a (channels 11..15 Gomoku / 8..15 Go are zero) from the record's
// values: v = board[a], lib = liberties byte of a (Go), meta = the record's 8 meta ints.
__device__ __forceinline__ void az_leaf_planes_v(int v, int lib8, const int* meta, int go, int bs, int a, float c[16]) {
#pragma clang fp contract(off)
    const int player = meta[0];
#pragma unroll
    for (int k = 0; k < 16; ++k) c[k] = 0.0f;
    if (go) {
        if (v == 1) c[0] = 1.0f;
        else if (v == 2) c[1] = 1.0f;
        c[2] = player == 1 ? 1.0f : 0.0f;
        if (v) {
            const float lib = fminf(1.0f, (float)lib8 / 10.0f);
            if (v == 1) c[3] = lib;
            else c[4] = lib;
        }
        if (a == meta[1]) c[5] = 1.0f;
        const float half = (float)(bs / 2);
        const int x = a % bs, y = a / bs;
        c[6] = (float)min(x, bs - 1 - x) / half;
        c[7] = (float)min(y, bs - 1 - y) / half;
    } else {
        if (v == player) c[0] = 1.0f;
        else if (v == 3 - player) c[1] = 1.0f;
        if (player == 1) c[2] = 1.0f;
        // history slot i: the reference's get_previous_moves parity rule (gomoku_state.cpp:852-869)
        // puts h0, h2, h4 into the "BLACK" planes 3..5 when BLACK is to move, else 6..8
        bool h[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) h[i] = meta[2 + i] == a;
        const bool p1 = player == 1;
        c[3] = (p1 ? h[0] : h[1]) ? 1.0f : 0.0f;
        c[4] = (p1 ? h[2] : h[3]) ? 1.0f : 0.0f;
        c[5] = (p1 ? h[4] : h[5]) ? 1.0f : 0.0f;
        c[6] = (p1 ? h[1] : h[0]) ? 1.0f : 0.0f;
        c[7] = (p1 ? h[3] : h[2]) ? 1.0f : 0.0f;
        c[8] = (p1 ? h[5] : h[4]) ? 1.0f : 0.0f;
        const int x = a / bs, y = a % bs;
        c[9] = (float)x / (float)(bs - 1);
        c[10] = (float)y / (float)(bs - 1);
    }
}

__device__ __forceinline__ void az_leaf_planes(const uint8_t* rec, int go, int bs, int a, float c[16]) {
    az_leaf_planes_v(rec[a], go ? rec[AZ_REC_LIBS + a] : 0, reinterpret_cast<const int*>(rec + AZ_REC_META), go, bs, a, c);
}
