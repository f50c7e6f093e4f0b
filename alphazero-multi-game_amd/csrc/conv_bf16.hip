// conv_bf16.hip -- 3x3 trunk convolution on bf16 MFMA (gfx950), implicit GEMM.
//
//   out[m][n] = relu( sum_{tap,c} A[nbr(m,tap)][c] * W[n][tap][c] + bias[n] (+ res[m][n]) )
//   m = pixel (b, y, x) of an NHWC map, K = 9*C, zero padding at the board edge.
//
// AZ_PREC_BF16X3: every fp32 operand x is stored as hi = bf16(x), lo = bf16(x - hi);
// a*b ~= hi*hi + hi*lo + lo*hi (three v_mfma_f32_16x16x32_bf16, fp32 accumulate),
// dropping lo*lo (~2^-16 relative per product).  AZ_PREC_BF16: hi only.
//
// Block tile 128 pixels x 128 channels, BK = 32 (one tap, 32 channels per k-step),
// 256 threads = 2x2 waves of 64x64 (4x4 MFMA 16x16 tiles).  A is gathered row by
// row (64-byte rows) into LDS; rows are XOR-swizzled on their four 16-byte chunks
// (chunk ^ s[(row>>2)&3], s = {0,2,3,1}) so the ds_read_b128 fragment reads of all
// four lane groups hit distinct bank slots.  Double-buffered LDS, register-staged
// loads, one barrier per k-step.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "net.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

namespace {

__device__ __forceinline__ int swz(int row) { return (0x78 >> (2 * ((row >> 2) & 3))) & 3; }

__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }

__device__ __forceinline__ uint16_t f2bf(float f) {   // round to nearest even (finite inputs)
    uint32_t u = __float_as_uint(f);
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

}  // namespace

template <bool SPLIT>
__global__ __launch_bounds__(256, 2) void conv3x3_bf16(ConvBf16Args p) {
    constexpr int BM = 128, BN = 128, BK = 32;
    constexpr int ROWB = BK * 2;                       // 64 bytes per LDS row
    constexpr int TILE = BM * ROWB;                    // 8 KB per operand tile
    constexpr int NOP = SPLIT ? 4 : 2;                 // Ahi, Bhi, (Alo, Blo)
    __shared__ __attribute__((aligned(16))) uint8_t lds[2 * NOP * TILE];

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int nbm = (p.M + BM - 1) / BM;
    const int bm = blockIdx.x % nbm, bn = blockIdx.x / nbm;
    const int m0 = bm * BM, n0 = bn * BN;
    const int Mact = p.m_limit ? min(p.M, *p.m_limit * p.rows_per_sample) : p.M;
    if (m0 >= Mact) return;

    const int C = p.C, H = p.H, W = p.W, HW = H * W;
    const int K = 9 * C;
    const int cpt = C / BK;                             // k-steps per tap
    const int nk = 9 * cpt;

    // loader mapping: row = tid/4 + 64*j, chunk q = tid%4 (16 B = 8 bf16)
    const int q = tid & 3;
    int rb_[2], ry[2], rx[2];
    bool rok[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int m = m0 + (tid >> 2) + 64 * j;
        rok[j] = m < Mact;
        const int b = m / HW, r = m - b * HW;
        rb_[j] = b; ry[j] = r / W; rx[j] = r - (r / W) * W;
    }

    uint4 ra_hi[2], ra_lo[2], rbw_hi[2], rbw_lo[2];
    auto gload = [&](int kt) {
        const int tap = kt / cpt;
        const int c0 = (kt - tap * cpt) * BK + q * 8;
        const int dy = tap / 3 - 1, dx = tap % 3 - 1;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            uint4 vh = make_uint4(0, 0, 0, 0), vl = make_uint4(0, 0, 0, 0);
            const int y = ry[j] + dy, x = rx[j] + dx;
            if (rok[j] && y >= 0 && y < H && x >= 0 && x < W) {
                const size_t off = ((size_t)(rb_[j] * H + y) * W + x) * C + c0;
                vh = *reinterpret_cast<const uint4*>(p.Ahi + off);
                if (SPLIT) vl = *reinterpret_cast<const uint4*>(p.Alo + off);
            }
            ra_hi[j] = vh; ra_lo[j] = vl;
            const int n = n0 + (tid >> 2) + 64 * j;
            uint4 wh = make_uint4(0, 0, 0, 0), wl = make_uint4(0, 0, 0, 0);
            if (n < p.N) {
                const size_t woff = (size_t)n * K + (size_t)kt * BK + q * 8;
                wh = *reinterpret_cast<const uint4*>(p.Bhi + woff);
                if (SPLIT) wl = *reinterpret_cast<const uint4*>(p.Blo + woff);
            }
            rbw_hi[j] = wh; rbw_lo[j] = wl;
        }
    };
    auto lstore = [&](int buf) {
        uint8_t* base = lds + buf * NOP * TILE;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int row = (tid >> 2) + 64 * j;
            const int off = row * ROWB + 16 * (q ^ swz(row));
            *reinterpret_cast<uint4*>(base + 0 * TILE + off) = ra_hi[j];
            *reinterpret_cast<uint4*>(base + 1 * TILE + off) = rbw_hi[j];
            if (SPLIT) {
                *reinterpret_cast<uint4*>(base + 2 * TILE + off) = ra_lo[j];
                *reinterpret_cast<uint4*>(base + 3 * TILE + off) = rbw_lo[j];
            }
        }
    };

    floatx4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

    gload(0);
    lstore(0);
    __syncthreads();
    const int fr = lane & 15, fh = lane >> 4;
    for (int kt = 0; kt < nk; ++kt) {
        const int buf = kt & 1;
        if (kt + 1 < nk) gload(kt + 1);
        const uint8_t* base = lds + buf * NOP * TILE;
        bf16x8 ah[4], bh[4], al[4], bl[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = wm * 64 + i * 16 + fr;
            const int off = row * ROWB + 16 * (fh ^ swz(row));
            ah[i] = *reinterpret_cast<const bf16x8*>(base + 0 * TILE + off);
            if (SPLIT) al[i] = *reinterpret_cast<const bf16x8*>(base + 2 * TILE + off);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int row = wn * 64 + j * 16 + fr;
            const int off = row * ROWB + 16 * (fh ^ swz(row));
            bh[j] = *reinterpret_cast<const bf16x8*>(base + 1 * TILE + off);
            if (SPLIT) bl[j] = *reinterpret_cast<const bf16x8*>(base + 3 * TILE + off);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (SPLIT) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
                }
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
            }
        if (kt + 1 < nk) lstore(buf ^ 1);
        __syncthreads();
    }

    // epilogue: C/D map col = lane&15, row = 4*(lane>>4) + r
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int n = n0 + wn * 64 + j * 16 + fr;
            const bool nok = n < p.N;
            const float bias = nok ? p.bias[n] : 0.0f;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m0 + wm * 64 + i * 16 + 4 * fh + r;
                if (nok && m < Mact) {
                    const size_t o = (size_t)m * p.N + n;
                    float v = acc[i][j][r] + bias;
                    if (p.Rhi) v += bf2f(p.Rhi[o]) + (SPLIT ? bf2f(p.Rlo[o]) : 0.0f);
                    if (p.relu) v = v > 0.0f ? v : 0.0f;
                    const uint16_t hi = f2bf(v);
                    p.Chi[o] = hi;
                    if (SPLIT) p.Clo[o] = f2bf(v - bf2f(hi));
                    if (p.Cf) p.Cf[o] = v;
                }
            }
        }
}

__global__ void k_split_bf16(const float* in, uint16_t* hi, uint16_t* lo, size_t n, const int* m_limit, int rows_per_sample,
                             int C) {
    size_t lim = n;
    if (m_limit) lim = min(n, (size_t)(*m_limit) * rows_per_sample * C);
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < lim; i += (size_t)gridDim.x * blockDim.x) {
        const float v = in[i];
        const uint16_t h = f2bf(v);
        hi[i] = h;
        if (lo) lo[i] = f2bf(v - bf2f(h));
    }
}

void az_conv_bf16_launch(const ConvBf16Args& a, bool split, hipStream_t st) {
    const int nbm = (a.M + 127) / 128, nbn = (a.N + 127) / 128;
    if (split) hipLaunchKernelGGL(conv3x3_bf16<true>, dim3(nbm * nbn), dim3(256), 0, st, a);
    else hipLaunchKernelGGL(conv3x3_bf16<false>, dim3(nbm * nbn), dim3(256), 0, st, a);
}

void az_launch_split_bf16(const float* in, uint16_t* hi, uint16_t* lo, size_t n, const int* m_limit, int rows_per_sample,
                          int C, hipStream_t st) {
    hipLaunchKernelGGL(k_split_bf16, dim3(2048), dim3(256), 0, st, in, hi, lo, n, m_limit, rows_per_sample, C);
}
