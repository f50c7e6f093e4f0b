// Host build of csrc/leaf_planes.h (the feature planes every network input stage builds from the
// search's leaf records), for tests/test_leaf_planes_cpu.py: the header's own arithmetic, compiled
// for the CPU with IEEE division and no FMA contraction, against the reference's plane fixtures.
#include <algorithm>
#include <cmath>
#include <cstdint>
#define __device__
#define __forceinline__ inline
using std::min;
#include "../../alphazero-multi-game_amd/csrc/leaf_planes.h"

extern "C" int az_rec_bytes() { return AZ_REC_BYTES; }

// planes [A][16] (NHWC16) of every cell of one record
extern "C" void az_rec_planes_host(const uint8_t* rec, int go, int bs, float* out) {
    for (int a = 0; a < bs * bs; ++a) az_leaf_planes(rec, go, bs, a, out + (size_t)a * 16);
}
