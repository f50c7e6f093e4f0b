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
#include <type_traits>
#include "net.h"
#include "leaf_planes.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

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

// ===========================================================================
// v3 (below; its v2 predecessor without fragment double buffering was removed in round 2):
// block tile BM pixels x BN channels, 8 waves (WM x WN), BK = 32.  Operand tiles
// move HBM/L2 -> LDS by global_load_lds_dwordx4 (LDS-DMA, per-lane source address
// = the im2col gather, zero page for the board edge) into a STAGES-deep ring; each
// wave issues its share of the 16-row pieces and retires them with a counted
// s_waitcnt vmcnt before one raw s_barrier per k-step (the loads of k-steps kt+1 ..
// kt+STAGES-1 stay in flight across it).  LDS images are linear rows of 64 B; the
// chunk swizzle is applied to the SOURCE address (glds writes lane-linear).  The
// epilogue stages the fp32 tile through LDS and stores 16-byte vectors.
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void g_void_t;

// ===========================================================================
// v3: v2's glds ring + fragment double buffering.  The wait/barrier that publishes
// k-step kt+1 sits in the MIDDLE of k-step kt's MFMAs; the ds_reads of kt+1's
// fragments (second register set) and the glds issue of k-step kt+3 follow it and
// overlap the second half of kt's MFMAs, so neither LDS latency nor the barrier
// exposes a bubble at the step boundary.
template <bool SPLIT, int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(WM * WN * 64, 1) void conv3x3_v3(ConvBf16Args p) {
    constexpr int STAGES = 3;
    constexpr int NT = WM * WN * 64, NW = WM * WN;
    constexpr int ROWB = 64;
    constexpr int NPL = SPLIT ? 2 : 1;
    constexpr int A_BYTES = BM * ROWB, B_BYTES = BN * ROWB;
    constexpr int STAGE = NPL * (A_BYTES + B_BYTES);
    constexpr int EPI_LD = BN + 4;
    constexpr int EPI = BM * EPI_LD * 4;
    constexpr int LDS = STAGES * STAGE > EPI ? STAGES * STAGE : EPI;
    constexpr int A_INS = BM / 16, B_INS = BN / 16;
    constexpr int INS = NPL * (A_INS + B_INS);
    constexpr int PW = INS / NW;
    static_assert(INS % NW == 0, "pieces must split evenly over waves");
    constexpr int TM = BM / WM, TN = BN / WN;
    constexpr int FM = TM / 16, FN = TN / 16;
    static_assert(FM % 2 == 0, "two MFMA halves");
    __shared__ __attribute__((aligned(16))) uint8_t lds[LDS];

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WN, wn = wave % WN;
    const int nbm = (p.M + BM - 1) / BM;
    const int bm = blockIdx.x % nbm, bn = blockIdx.x / nbm;
    const int m0 = bm * BM, n0 = bn * BN;
    const int Mact = p.m_limit ? min(p.M, *p.m_limit * p.rows_per_sample) : p.M;
    if (m0 >= Mact) return;
    const int C = p.C, H = p.H, W = p.W, HW = H * W, K = 9 * C;
    const int cpt = C / 32, nk = 9 * cpt;

    const uint16_t* src_base[PW];
    int src_y[PW], src_x[PW];
    bool isA[PW];
    int lds_off[PW];
    int chunk[PW];
#pragma unroll
    for (int j = 0; j < PW; ++j) {
        const int q = wave + NW * j;
        const int row_in_piece = lane >> 2, phys = lane & 3;
        if (q < NPL * A_INS) {
            const int plane = q / A_INS, rb = q % A_INS;
            const int row = rb * 16 + row_in_piece;
            const int m = m0 + row;
            isA[j] = true;
            lds_off[j] = plane * A_BYTES + rb * 1024;
            chunk[j] = phys ^ swz(row);
            const uint16_t* base = plane ? p.Alo : p.Ahi;
            if (m < Mact) {
                const int b = m / HW, r = m - b * HW;
                src_base[j] = base + (size_t)b * HW * C;
                src_y[j] = r / W; src_x[j] = r - (r / W) * W;
            } else {
                src_base[j] = base; src_y[j] = -1000; src_x[j] = -1000;
            }
        } else {
            const int qq = q - NPL * A_INS;
            const int plane = qq / B_INS, rb = qq % B_INS;
            const int row = rb * 16 + row_in_piece;
            const int n = n0 + row;
            isA[j] = false;
            lds_off[j] = NPL * A_BYTES + plane * B_BYTES + rb * 1024;
            chunk[j] = phys ^ swz(row);
            const uint16_t* base = plane ? p.Blo : p.Bhi;
            src_base[j] = n < p.N ? base + (size_t)n * K : nullptr;
            src_y[j] = 0; src_x[j] = 0;
        }
    }
    auto issue = [&](int kt) {
        const int tap = kt / cpt;
        const int c0 = (kt - tap * cpt) * 32;
        const int dy = tap / 3 - 1, dx = tap % 3 - 1;
        uint8_t* stage = lds + (kt % STAGES) * STAGE;
#pragma unroll
        for (int j = 0; j < PW; ++j) {
            const uint16_t* src;
            if (isA[j]) {
                const int y = src_y[j] + dy, x = src_x[j] + dx;
                src = (y >= 0 && y < H && x >= 0 && x < W) ? src_base[j] + ((size_t)(y * W + x) * C + c0 + chunk[j] * 8)
                                                           : p.zero + chunk[j] * 8;
            } else {
                src = src_base[j] ? src_base[j] + (size_t)kt * 32 + chunk[j] * 8 : p.zero + chunk[j] * 8;
            }
            __builtin_amdgcn_global_load_lds((g_void_t*)src, (lds_void_t*)(stage + lds_off[j]), 16, 0, 0);
        }
    };
    const int fr = lane & 15, fh = lane >> 4;
    auto read_frags = [&](int kt, bf16x8 (&ah)[FM], bf16x8 (&al)[FM], bf16x8 (&bh)[FN], bf16x8 (&bl)[FN]) {
        const uint8_t* st = lds + (kt % STAGES) * STAGE;
#pragma unroll
        for (int i = 0; i < FM; ++i) {
            const int row = wm * TM + i * 16 + fr;
            const int off = row * ROWB + 16 * (fh ^ swz(row));
            ah[i] = *reinterpret_cast<const bf16x8*>(st + off);
            if (SPLIT) al[i] = *reinterpret_cast<const bf16x8*>(st + A_BYTES + off);
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) {
            const int row = wn * TN + j * 16 + fr;
            const int off = row * ROWB + 16 * (fh ^ swz(row));
            bh[j] = *reinterpret_cast<const bf16x8*>(st + NPL * A_BYTES + off);
            if (SPLIT) bl[j] = *reinterpret_cast<const bf16x8*>(st + NPL * A_BYTES + B_BYTES + off);
        }
    };
    floatx4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    auto mfma_rows = [&](int i0, int i1, const bf16x8 (&ah)[FM], const bf16x8 (&al)[FM], const bf16x8 (&bh)[FN],
                         const bf16x8 (&bl)[FN]) {
#pragma unroll
        for (int i = 0; i < FM; ++i) {
            if (i < i0 || i >= i1) continue;
#pragma unroll
            for (int j = 0; j < FN; ++j) {
                if (SPLIT) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
                }
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
            }
        }
    };
    // one k-step: first half of the MFMAs, publish k+1 (wait + barrier), issue k+3,
    // read k+1's fragments, second half.
    auto step = [&](int kt, const bf16x8 (&ch)[FM], const bf16x8 (&cl)[FM], const bf16x8 (&dh)[FN],
                    const bf16x8 (&dl)[FN], bf16x8 (&nah)[FM], bf16x8 (&nal)[FM], bf16x8 (&nbh)[FN], bf16x8 (&nbl)[FN]) {
        mfma_rows(0, FM / 2, ch, cl, dh, dl);
        if (kt + 1 < nk) {
            if (kt + 2 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PW) : "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_sched_barrier(0);
            if (kt + 3 < nk) issue(kt + 3);
            read_frags(kt + 1, nah, nal, nbh, nbl);
        }
        mfma_rows(FM / 2, FM, ch, cl, dh, dl);
    };

    bf16x8 a0h[FM], a0l[FM], b0h[FN], b0l[FN], a1h[FM], a1l[FM], b1h[FN], b1l[FN];
#pragma unroll
    for (int s = 0; s < STAGES; ++s)
        if (s < nk) issue(s);
    if (nk > 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PW) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    read_frags(0, a0h, a0l, b0h, b0l);
    for (int kt = 0; kt < nk; kt += 2) {
        step(kt, a0h, a0l, b0h, b0l, a1h, a1l, b1h, b1l);
        if (kt + 1 < nk) step(kt + 1, a1h, a1l, b1h, b1l, a0h, a0l, b0h, b0l);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();
    float* ep = reinterpret_cast<float*>(lds);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                ep[(wm * TM + i * 16 + 4 * fh + r) * EPI_LD + wn * TN + j * 16 + fr] = acc[i][j][r];
    __syncthreads();
    constexpr int VPR = BN / 8;
    for (int v = tid; v < BM * VPR; v += NT) {
        const int row = v / VPR, cv = (v % VPR) * 8;
        const int m = m0 + row, n = n0 + cv;
        if (m >= Mact || n >= p.N) continue;
        const float4 x0 = *reinterpret_cast<const float4*>(ep + row * EPI_LD + cv);
        const float4 x1 = *reinterpret_cast<const float4*>(ep + row * EPI_LD + cv + 4);
        float o[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
        const size_t g = (size_t)m * p.N + n;
        const float4 b0 = *reinterpret_cast<const float4*>(p.bias + n);
        const float4 b1 = *reinterpret_cast<const float4*>(p.bias + n + 4);
        const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
        uint16_t rh[8], rl[8];
        if (p.Rhi) {
            *reinterpret_cast<uint4*>(rh) = *reinterpret_cast<const uint4*>(p.Rhi + g);
            if (SPLIT) *reinterpret_cast<uint4*>(rl) = *reinterpret_cast<const uint4*>(p.Rlo + g);
        }
        uint16_t oh[8], ol[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            float val = o[e] + bb[e];
            if (p.Rhi) val += bf2f(rh[e]) + (SPLIT ? bf2f(rl[e]) : 0.0f);
            if (p.relu) val = val > 0.0f ? val : 0.0f;
            o[e] = val;
            oh[e] = f2bf(val);
            if (SPLIT) ol[e] = f2bf(val - bf2f(oh[e]));
        }
        *reinterpret_cast<uint4*>(p.Chi + g) = *reinterpret_cast<const uint4*>(oh);
        if (SPLIT) *reinterpret_cast<uint4*>(p.Clo + g) = *reinterpret_cast<const uint4*>(ol);
        if (p.Cf) {
            *reinterpret_cast<float4*>(p.Cf + g) = make_float4(o[0], o[1], o[2], o[3]);
            *reinterpret_cast<float4*>(p.Cf + g + 4) = make_float4(o[4], o[5], o[6], o[7]);
        }
    }
}

// ===========================================================================
// v4: board-halo implicit GEMM for 15x15 boards (all trunk precisions).
// A block owns TWO boards x BNT output channels.  For every 16-channel chunk the
// zero-padded 17x17 input halo of both boards is DMA'd (global_load_lds) into LDS
// once and read by all nine taps as row-shifted windows: outputs live on a 15x17
// grid (two dead columns) so the tap (dy,dx) operand of 32 consecutive outputs is 32
// consecutive halo rows (shift (dy+1)*17 + (dx+1)).  Activation traffic drops ~9x and
// each weight byte feeds two boards.  LDS images are chunk-major ([16-byte chunk]
// [row]), which keeps every ds_read_b128 lane group on 16 distinct bank slots for ANY
// row shift.  Pipeline: A halo double-buffered per chunk, weights of one tap row
// (3 taps) per step in a 3-slot ring, counted vmcnt + one barrier per step.
//   MODE 0: bf16x3 (hi/lo planes, 3 MFMAs);  1: bf16;  2: fp16 (reference useFp16)
constexpr int V4_HROWS = 320;                 // 17*17 = 289 halo rows, padded to 5 x 64

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void wait_vm(int n) {      // s_waitcnt vmcnt(n), n wave-uniform
    switch (n) {
        case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
        case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
        case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
        case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
        case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
        case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
        case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
        case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
        case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
        case 11: asm volatile("s_waitcnt vmcnt(11)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    }
}

template <int MODE>
__device__ __forceinline__ float v4_load(uint16_t h) {
    if (MODE == 2) { _Float16 x; __builtin_memcpy(&x, &h, 2); return (float)x; }
    return bf2f(h);
}
template <int MODE>
__device__ __forceinline__ uint16_t v4_store(float f) {
    if (MODE == 2) { _Float16 x = (_Float16)f; uint16_t h; __builtin_memcpy(&h, &x, 2); return h; }
    return f2bf(f);
}

#define V4_STAMP(k) do { } while (0)

// BOARDS boards per block of NT threads (default 4 waves per board).  The small-batch bf16x3 layers
// of the 64-channel C2 net launch conv3x3_v4<0, 64, 1, 1, 512>: ONE board per 512-thread block
// (8 waves, two per SIMD, 32 output rows per wave), one block per CU by its LDS -- at 256 boards two
// boards per block would fill only half the CUs, and one board per 256-thread block left a SIMD
// with one wave and nothing to hide its fragment reads behind.  Every output's MFMA chain is the
// same for any BOARDS / NT.
template <int MODE, int BNT, int SCHED, int BOARDS = 2, int NT = 256 * BOARDS>
__global__ __launch_bounds__(NT, 1) void conv3x3_v4(ConvBf16Args p) {
    constexpr bool SPLIT = MODE == 0;
    constexpr int NPL = SPLIT ? 2 : 1;
    constexpr int NW = NT / 64;
    constexpr int A_PLANE = 2 * V4_HROWS * 16;             // one board, one plane, 16 channels: 10 KB
    constexpr int A_BUF = BOARDS * NPL * A_PLANE;
    constexpr int B_TAP = NPL * 2 * BNT * 16;
    constexpr int B_STAGE = 3 * B_TAP;
    constexpr int LDS_MAIN = 2 * A_BUF + 3 * B_STAGE;
    constexpr int EP_LD = BNT + 4;
    constexpr int LDS_EPI = 256 * EP_LD * 4;
    constexpr int LDS = LDS_MAIN > LDS_EPI ? LDS_MAIN : LDS_EPI;
    constexpr int A_INS = BOARDS * NPL * 2 * (V4_HROWS / 64);   // 1 KiB pieces per A chunk
    constexpr int B_INS = 3 * NPL * 2 * (BNT / 64);             // per step
    constexpr int PAX = (A_INS + NW - 1) / NW, PBX = (B_INS + NW - 1) / NW;
    constexpr int WN = BNT >= 128 ? BNT / 64 : 1;
    constexpr int WM = NW / WN;
    constexpr int TM = BOARDS * 256 / WM;              // output rows per wave
    constexpr int FM = TM / 32, FN = BNT / WN / 32;
    typedef typename std::conditional<MODE == 2, f16x8, bf16x8>::type frag;
    __shared__ __attribute__((aligned(16))) uint8_t lds[LDS];

    V4_STAMP(0);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WN, wn = wave % WN;
    const int nsplit = p.N / BNT;
    const int pair = blockIdx.x / nsplit, nb = blockIdx.x % nsplit;
    const int n0 = nb * BNT;
    const int nboards = p.m_limit ? *p.m_limit : p.M / (p.H * p.W);
    const int b0 = pair * BOARDS;
    if (b0 >= nboards) return;
    const int C = p.C, HW = p.H * p.W, K = 9 * C;
    const int NCH = C / 16, NS = NCH * 3;
    const int PA = (A_INS - wave + NW - 1) / NW, PB = (B_INS - wave + NW - 1) / NW;   // this wave's pieces

    const uint16_t* a_src[PAX];
    int a_ch[PAX], a_off[PAX];
#pragma unroll
    for (int j = 0; j < PAX; ++j) {
        const int q = wave + NW * j;
        const int rb = q % 5, ch = (q / 5) % 2, plane = (q / 10) % NPL, bd = q / (10 * NPL);
        const int hr = rb * 64 + lane;
        const int Y = hr / 17, X = hr - Y * 17;
        const int b = b0 + bd;
        const bool ok = q < A_INS && hr < 289 && Y >= 1 && Y <= 15 && X >= 1 && X <= 15 && b < nboards;
        const uint16_t* base = plane ? p.Alo : p.Ahi;
        a_src[j] = ok ? base + ((size_t)b * HW + (Y - 1) * 15 + (X - 1)) * C + ch * 8 : nullptr;
        a_ch[j] = ch;
        a_off[j] = (bd * NPL + plane) * A_PLANE + ch * (V4_HROWS * 16) + rb * 1024;
    }
    const uint16_t* b_src[PBX];
    int b_off[PBX];
#pragma unroll
    for (int j = 0; j < PBX; ++j) {
        const int q = min(wave + NW * j, B_INS - 1);
        constexpr int RB = BNT / 64;
        const int rb = q % RB, ch = (q / RB) % 2, plane = (q / (2 * RB)) % NPL, t = q / (2 * RB * NPL);
        const int n = n0 + rb * 64 + lane;
        const uint16_t* base = plane ? p.Blo : p.Bhi;
        b_src[j] = base + (size_t)n * K + t * C + ch * 8;
        b_off[j] = t * B_TAP + (plane * 2 + ch) * BNT * 16 + rb * 1024;
    }
    uint8_t* abuf = lds;
    uint8_t* bbuf = lds + 2 * A_BUF;
    auto issueA = [&](int c) {
        uint8_t* dst = abuf + (c & 1) * A_BUF;
#pragma unroll
        for (int j = 0; j < PAX; ++j) {
            if (j >= PA) break;
            const uint16_t* src = a_src[j] ? a_src[j] + c * 16 : p.zero + a_ch[j] * 8;
            __builtin_amdgcn_global_load_lds((g_void_t*)src, (lds_void_t*)(dst + a_off[j]), 16, 0, 0);
        }
    };
    auto issueB = [&](int s) {
        const int c = s / 3, r = s - c * 3;
        uint8_t* dst = bbuf + (s % 3) * B_STAGE;
#pragma unroll
        for (int j = 0; j < PBX; ++j) {
            if (j >= PB) break;
            const uint16_t* src = b_src[j] + r * 3 * C + c * 16;
            __builtin_amdgcn_global_load_lds((g_void_t*)src, (lds_void_t*)(dst + b_off[j]), 16, 0, 0);
        }
    };

    floatx16 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;

    issueA(0);
    issueB(0);
    if (NS > 1) issueB(1);
    const int l32 = lane & 31, lh = lane >> 5;
    const int bd_w = (wm * TM) / 256;
    const int q0 = (wm * TM) % 256;
    for (int s = 0; s < NS; ++s) {
        const int c = s / 3, r = s - c * 3;
        // retire B(s) (and A(c) at r == 0); later pieces stay in flight
        wait_vm((s + 1 < NS ? PB : 0) + ((r >= 1 && c + 1 < NCH) ? PA : 0));
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        if (s + 2 < NS) issueB(s + 2);
        if (r == 0 && c + 1 < NCH) issueA(c + 1);
        const uint8_t* ab = abuf + (c & 1) * A_BUF + bd_w * NPL * A_PLANE;
        const uint8_t* bb = bbuf + (s % 3) * B_STAGE;
        // fragments of tap t: A rows shifted by r*17 + t, B tap slot t
        auto load = [&](int t, frag (&ah)[FM], frag (&al)[FM], frag (&bh)[FN], frag (&bl)[FN]) {
            const int shift = r * 17 + t;
#pragma unroll
            for (int i = 0; i < FM; ++i) {
                const int hr = q0 + i * 32 + l32 + shift;
                const int off = lh * (V4_HROWS * 16) + hr * 16;
                ah[i] = *reinterpret_cast<const frag*>(ab + off);
                if (SPLIT) al[i] = *reinterpret_cast<const frag*>(ab + A_PLANE + off);
            }
#pragma unroll
            for (int j = 0; j < FN; ++j) {
                const int n = wn * (BNT / WN) + j * 32 + l32;
                const int off = t * B_TAP + lh * BNT * 16 + n * 16;
                bh[j] = *reinterpret_cast<const frag*>(bb + off);
                if (SPLIT) bl[j] = *reinterpret_cast<const frag*>(bb + 2 * BNT * 16 + off);
            }
        };
        auto mma = [&](frag (&ah)[FM], frag (&al)[FM], frag (&bh)[FN], frag (&bl)[FN]) {
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int j = 0; j < FN; ++j) {
                    if constexpr (MODE == 2) {
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
                    } else {
                        if (SPLIT) {
                            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
                            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
                        }
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
                    }
                }
        };
        if constexpr (SCHED == 0) {
#pragma unroll
            for (int t = 0; t < 3; ++t) {
                frag ah[FM], al[FM], bh[FN], bl[FN];
                load(t, ah, al, bh, bl);
                mma(ah, al, bh, bl);
            }
        } else {
            // register double buffer: tap t+1's fragments are in flight while tap t's MFMAs issue
            frag ah0[FM], al0[FM], bh0[FN], bl0[FN], ah1[FM], al1[FM], bh1[FN], bl1[FN];
            load(0, ah0, al0, bh0, bl0);
            __builtin_amdgcn_sched_barrier(0);
            load(1, ah1, al1, bh1, bl1);
            __builtin_amdgcn_sched_barrier(0);
            mma(ah0, al0, bh0, bl0);
            __builtin_amdgcn_sched_barrier(0);
            load(2, ah0, al0, bh0, bl0);
            __builtin_amdgcn_sched_barrier(0);
            mma(ah1, al1, bh1, bl1);
            __builtin_amdgcn_sched_barrier(0);
            mma(ah0, al0, bh0, bl0);
        }
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();
    V4_STAMP(1);
    float* ep = reinterpret_cast<float*>(lds);
    float vmax = 0.0f;                                 // MODE 2: the largest |output| (the range guard)
    for (int bd = 0; bd < BOARDS; ++bd) {
        if (bd_w == bd) {
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int j = 0; j < FN; ++j)
#pragma unroll
                    for (int e = 0; e < 16; ++e) {
                        const int row = q0 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * lh;
                        ep[row * EP_LD + wn * (BNT / WN) + j * 32 + l32] = acc[i][j][e];
                    }
        }
        __syncthreads();
        const int b = b0 + bd;
        constexpr int VPR = BNT / 8;
        if (b < nboards) {
            for (int v = tid; v < 225 * VPR; v += NT) {
                const int pix = v / VPR, cv = (v % VPR) * 8;
                const int y = pix / 15, x = pix - y * 15;
                const int row = y * 17 + x;
                const float4 x0 = *reinterpret_cast<const float4*>(ep + row * EP_LD + cv);
                const float4 x1 = *reinterpret_cast<const float4*>(ep + row * EP_LD + cv + 4);
                float o[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
                const int n = n0 + cv;
                const size_t g = ((size_t)b * HW + pix) * p.N + n;
                const float4 c0v = *reinterpret_cast<const float4*>(p.bias + n);
                const float4 c1v = *reinterpret_cast<const float4*>(p.bias + n + 4);
                const float bb[8] = {c0v.x, c0v.y, c0v.z, c0v.w, c1v.x, c1v.y, c1v.z, c1v.w};
                uint16_t rh[8], rl[8];
                float rf[8];
                if (p.Rf) {
                    *reinterpret_cast<float4*>(rf) = *reinterpret_cast<const float4*>(p.Rf + g);
                    *reinterpret_cast<float4*>(rf + 4) = *reinterpret_cast<const float4*>(p.Rf + g + 4);
                }
                if (p.Rhi) {
                    *reinterpret_cast<uint4*>(rh) = *reinterpret_cast<const uint4*>(p.Rhi + g);
                    if (SPLIT) *reinterpret_cast<uint4*>(rl) = *reinterpret_cast<const uint4*>(p.Rlo + g);
                }
                uint16_t oh[8], ol[8];
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    float val = o[e] + bb[e];
                    if (p.Rf) val += rf[e];
                    else if (p.Rhi) val += v4_load<MODE>(rh[e]) + (SPLIT ? bf2f(rl[e]) : 0.0f);
                    if (p.relu) val = val > 0.0f ? val : 0.0f;
                    o[e] = val;
                    if constexpr (MODE == 2) vmax = __builtin_fmaxf(vmax, __builtin_fabsf(val));
                    oh[e] = v4_store<MODE>(val);
                    if (SPLIT) ol[e] = f2bf(val - bf2f(oh[e]));
                }
                *reinterpret_cast<uint4*>(p.Chi + g) = *reinterpret_cast<const uint4*>(oh);
                if (SPLIT) *reinterpret_cast<uint4*>(p.Clo + g) = *reinterpret_cast<const uint4*>(ol);
                if (p.Cf) {
                    *reinterpret_cast<float4*>(p.Cf + g) = make_float4(o[0], o[1], o[2], o[3]);
                    *reinterpret_cast<float4*>(p.Cf + g + 4) = make_float4(o[4], o[5], o[6], o[7]);
                }
            }
        }
        __syncthreads();
    }
    if (MODE == 2 && !(vmax <= 65504.0f) && p.ovf) atomicOr(p.ovf, 1);   // fp16 overflow: the engine fails the forward
    V4_STAMP(2);
}

// ===========================================================================
// v5: board-halo implicit GEMM for the single-plane trunk modes (AZ_PREC_FP16, AZ_PREC_BF16).
// Activations live in a channel-blocked layout, [board][C/8][225 pixels][8 channels] 16-bit
// ("g8"), and the weights in [C/16][9 taps][2][N][8]; every LDS-DMA piece (64 lanes x 16 B)
// is then one contiguous KiB.  A block owns two boards x 128 output channels; per 16-channel
// chunk the zero-padded 17x17 halo of both boards and the weights of all nine taps are staged
// (2-deep ring, one barrier per chunk) and the next chunk's pieces are issued one per tap
// between the MFMAs.  Fragment reads run one tap ahead (register double buffer, inline-asm
// ds_read with explicit lgkmcnt: the compiler's own waits drain to zero).
// The residual stream is kept at ~2^-19 relative precision without an fp32 copy: the
// 16-bit value h (the next conv's input) plus an int8 remainder q, x = h + q/254 * ulp(h).
// Blocks b and b+8 of the grid are the two channel halves of one board pair: same XCD
// (round-robin dispatch), so the second half reads the halo from that XCD's L2.
template <int MODE>
struct Half16 {                                         // MODE 2: fp16, MODE 1: bf16
    __device__ static float to_f(uint16_t h) {
        if (MODE == 2) { _Float16 x; __builtin_memcpy(&x, &h, 2); return (float)x; }
        return __uint_as_float((uint32_t)h << 16);
    }
    __device__ static uint16_t from_f(float f) {
        if (MODE == 2) { _Float16 x = (_Float16)f; uint16_t h; __builtin_memcpy(&h, &x, 2); return h; }
        uint32_t u = __float_as_uint(f);
        u += 0x7fffu + ((u >> 16) & 1u);
        return (uint16_t)(u >> 16);
    }
    // x -> (h, q): h = round(x) in 16 bits, q = the next 8 bits of x below h's precision, taken from
    // the fp32 bit patterns: d = bits(x) - bits(float(h)) counts fp32 ulps (x and h share the sign,
    // and the patterns are monotone across binades), q = round(d / 2^SH) clamped to +-127, and
    // x = bits(float(h)) + q * 2^SH reads back to 2^-20 relative (fp16: SH = 5, |d| <= 2^12;
    // bf16: SH = 8, |d| <= 2^15).  Where h is zero or subnormal the clamp bounds the absolute
    // error by the 16-bit subnormal spacing.  Integer adds and shifts: 3 VALU ops to join.
    static constexpr int MANT = MODE == 2 ? 11 : 8;
    static constexpr int SH = 16 - MANT;
    __device__ static void split(float x, uint16_t& h, int8_t& q) {
        h = from_f(x);
        const int d = (int)(__float_as_uint(x) - __float_as_uint(to_f(h)));
        const int r = (d + (1 << (SH - 1))) >> SH;
        q = (int8_t)min(127, max(-127, r));
    }
    __device__ static float join(uint16_t h, int8_t q) {
        return __uint_as_float(__float_as_uint(to_f(h)) + ((uint32_t)(int)q << SH));
    }
};

__device__ __forceinline__ uint32_t lds_addr(const void* p) { return (uint32_t)(uintptr_t)p; }

template <typename F>
__device__ __forceinline__ void ds_rd(F& d, uint32_t addr) {
    asm volatile("ds_read_b128 %0, %1" : "=v"(d) : "v"(addr) : "memory");
}

template <int N, typename F>
__device__ __forceinline__ void lgkm_wait6(F (&a)[4], F (&b)[2]) {
    // the fragments are in-out operands: every MFMA that reads them is ordered after the wait
    asm volatile("s_waitcnt lgkmcnt(%6)"
                 : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(b[0]), "+v"(b[1])
                 : "i"(N));
}

template <int MODE, int DW, int PPT_ = 0>
__global__ __launch_bounds__(512, 1) void conv3x3_v5(ConvBf16Args p) {
    static_assert(MODE == 1 || MODE == 2, "v5: single-plane modes");
    typedef Half16<MODE> H16;
    constexpr int BNT = 128;
    constexpr int BOARDS = 2;
    constexpr int A_PLANE = 2 * V4_HROWS * 16;        // one board, 16 channels: [2 halves][320 rows][16 B]
    constexpr int A_BUF = BOARDS * A_PLANE;            // 20 KB
    constexpr int B_TAP = 2 * BNT * 16;                // [2 halves][BNT][16 B] = 4 KB
    constexpr int B_BUF = 9 * B_TAP;                   // 36 KB
    constexpr int LDS_MAIN = 2 * A_BUF + 2 * B_BUF;    // 112 KB
    constexpr int SC = 64, SLD = SC + 4;               // epilogue: 64 staged columns per pass
    constexpr int LDS_EPI = BOARDS * 256 * SLD * 4;    // 136 KB: [2 boards][256 grid rows][68]
    constexpr int LDS_BIAS = (LDS_MAIN > LDS_EPI ? LDS_MAIN : LDS_EPI);   // + 128 fp32 biases
    constexpr int LDS = LDS_BIAS + BNT * 4;
    constexpr int A_INS = BOARDS * 2 * (V4_HROWS / 64);    // 20 pieces per chunk
    constexpr int B_INS = 9 * 2 * (BNT / 64);              // 36 pieces per chunk
    // DW waves issue the DMA pieces (all 8, or only the first wave of each SIMD pair, which
    // otherwise idles at the chunk barrier); PPT pieces per tap between the MFMAs
    constexpr int PAX = (A_INS + DW - 1) / DW, PBX = (B_INS + DW - 1) / DW;
    constexpr int PPT = PPT_ ? PPT_ : (PAX + PBX + 8) / 9;   // PPT_ = 2 with DW = 8: all pieces in taps 0-3
    static_assert(PPT <= 2, "at most two DMA pieces per tap");
    constexpr int WN = 2, TM = 128;
    constexpr int FM = 4, FN = 2;
    typedef typename std::conditional<MODE == 2, f16x8, bf16x8>::type frag;
    __shared__ __attribute__((aligned(16))) uint8_t lds[LDS];

    V4_STAMP(0);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WN, wn = wave % WN;
    const int nsplit = p.N / BNT;
    const int xcd = blockIdx.x % 8, slot = blockIdx.x / 8;
    const int nb = slot % nsplit, pair = (slot / nsplit) * 8 + xcd;
    const int n0 = nb * BNT;
    const int nboards = p.m_limit ? *p.m_limit : p.M / (p.H * p.W);
    const int b0 = pair * BOARDS;
    if (b0 >= nboards) return;
    float* sbias = reinterpret_cast<float*>(lds + LDS_BIAS);
    if (tid < BNT) sbias[tid] = p.bias[n0 + tid];     // visible after the first chunk barrier
    const int C = p.C, GI = C / 8, GO = p.N / 8;
    const int NCH = C / 16;
    const int PA = wave < DW ? (A_INS - wave + DW - 1) / DW : 0, PB = wave < DW ? (B_INS - wave + DW - 1) / DW : 0;

    // per-piece source element offsets (32-bit: < 2^31 elements) and LDS destinations;
    // a_el < 0 marks a padding row (read from the zero page)
    int a_el[PAX], a_ch[PAX], a_off[PAX];
#pragma unroll
    for (int j = 0; j < PAX; ++j) {
        const int q = wave + DW * j;
        const int rb = q % 5, ch = (q / 5) % 2, bd = q / 10;
        const int hr = rb * 64 + lane;
        const int Y = hr / 17, X = hr - Y * 17;
        const int b = b0 + bd;
        const bool ok = q < A_INS && hr < 289 && Y >= 1 && Y <= 15 && X >= 1 && X <= 15 && b < nboards;
        a_el[j] = ok ? (int)((((size_t)b * GI + ch) * 225 + (Y - 1) * 15 + (X - 1)) * 8) : -1;
        a_ch[j] = ch;
        a_off[j] = bd * A_PLANE + ch * (V4_HROWS * 16) + rb * 1024;
    }
    int b_el[PBX], b_off[PBX];
#pragma unroll
    for (int j = 0; j < PBX; ++j) {
        const int q = min(wave + DW * j, B_INS - 1);
        constexpr int RB = BNT / 64;
        const int rb = q % RB, ch = (q / RB) % 2, t = q / (2 * RB);
        const int n = n0 + rb * 64 + lane;
        b_el[j] = ((t * 2 + ch) * p.N + n) * 8;
        b_off[j] = t * B_TAP + ch * BNT * 16 + rb * 1024;
    }
    uint8_t* abuf = lds;
    uint8_t* bbuf = lds + 2 * A_BUF;
    // one LDS-DMA piece: k < PAX -> activation piece k, else weight piece k - PAX
    auto issue_piece = [&](int k, int c) {
        if (k < PAX) {
            if (k >= PA) return;
            const uint16_t* src = a_el[k] >= 0 ? p.Ahi + a_el[k] + (size_t)c * (2 * 225 * 8) : p.zero + a_ch[k] * 8;
            __builtin_amdgcn_global_load_lds((g_void_t*)src, (lds_void_t*)(abuf + (c & 1) * A_BUF + a_off[k]), 16, 0, 0);
        } else {
            const int j = k - PAX;
            if (j >= PB) return;
            __builtin_amdgcn_global_load_lds((g_void_t*)(p.Bblk + b_el[j] + (size_t)c * 144 * p.N),
                                             (lds_void_t*)(bbuf + (c & 1) * B_BUF + b_off[j]), 16, 0, 0);
        }
    };

    floatx16 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;

#pragma unroll
    for (int k = 0; k < PAX + PBX; ++k) issue_piece(k, 0);
    const int l32 = lane & 31, lh = lane >> 5;
    const int bd_w = (wm * TM) / 256;
    const int q0 = (wm * TM) % 256;
    const uint32_t a_lane = lds_addr(abuf) + bd_w * A_PLANE + lh * (V4_HROWS * 16) + (q0 + l32) * 16;
    const uint32_t b_lane = lds_addr(bbuf) + lh * BNT * 16 + (wn * (BNT / WN) + l32) * 16;
    for (int c = 0; c < NCH; ++c) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        const uint32_t ab = a_lane + (c & 1) * A_BUF;
        const uint32_t bb = b_lane + (c & 1) * B_BUF;
        auto load = [&](int tap, frag (&a)[FM], frag (&b)[FN]) {
            const int shift = (tap / 3) * 17 + (tap % 3);
#pragma unroll
            for (int i = 0; i < FM; ++i) ds_rd(a[i], ab + (i * 32 + shift) * 16);
#pragma unroll
            for (int j = 0; j < FN; ++j) ds_rd(b[j], bb + tap * B_TAP + j * 32 * 16);
        };
        auto mma = [&](frag (&a)[FM], frag (&b)[FN], int tap) {
#pragma unroll
            for (int i = 0; i < FM; ++i) {
                // next chunk's LDS-DMA pieces ride between this chunk's MFMAs, one per tap (two per
                // tap early in the chunk, or staggered between SIMD-mate waves, measured no better)
                const int pk = tap * PPT + (PPT == 1 ? 0 : i / 2);
                if ((PPT == 1 ? i == FM / 2 : (i & 1)) && c + 1 < NCH && pk < PAX + PBX) {
                    __builtin_amdgcn_sched_barrier(0);
                    issue_piece(pk, c + 1);
                    __builtin_amdgcn_sched_barrier(0);
                }
#pragma unroll
                for (int j = 0; j < FN; ++j) {
                    if constexpr (MODE == 2)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[i], b[j], acc[i][j], 0, 0, 0);
                    else
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
                }
            }
        };
        frag a0[FM], b0[FN], a1[FM], b1[FN];
        load(0, a0, b0);
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
            if (tap & 1) {
                if (tap + 1 < 9) { load(tap + 1, a0, b0); lgkm_wait6<6>(a1, b1); }
                else lgkm_wait6<0>(a1, b1);
                mma(a1, b1, tap);
            } else {
                if (tap + 1 < 9) { load(tap + 1, a1, b1); lgkm_wait6<6>(a0, b0); }
                else lgkm_wait6<0>(a0, b0);
                mma(a0, b0, tap);
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();
    V4_STAMP(1);

    // epilogue in two column passes (acc[.][j], j = 0, 1), both boards at once: the staged
    // fp32 tile is [2 boards][225 pixels][64 + 4], so the other pass's accumulators are the only
    // ones live while a pass finishes.  Item v = tid + 512k -> (board, channel group, pixel),
    // pixel fastest: a wave's 16-byte stores cover consecutive pixels of one group (contiguous in g8).
    constexpr int ITEMS = BOARDS * (SC / 8) * 225;     // 3600
    constexpr int ITER = (ITEMS + 511) / 512;          // 8
    float* ep = reinterpret_cast<float*>(lds);
    struct Res { uint4 h; uint2 q; };
    // residual of item v in pass j (zero beyond the items / boards)
    auto fetch = [&](int j, int v) {
        Res r{};
        const int pix = v % 225, t = v / 225, gl = t % 8, bd = t / 8;
        const int b = b0 + bd;
        if (v < ITEMS && b < nboards) {
            const int n = n0 + (gl / 4) * 64 + j * 32 + (gl % 4) * 8;
            const size_t e = (((size_t)b * GO + n / 8) * 225 + pix) * 8;
            r.h = *reinterpret_cast<const uint4*>(p.Rhi + e);
            r.q = *reinterpret_cast<const uint2*>(p.Rq + e);
        }
        return r;
    };
    // residual rows: pass 0's are fetched before its staging, pass 1's right after it, so both
    // latencies hide behind staging / the previous pass's arithmetic
    Res rr[FN][ITER];
    if (p.Rhi) {
#pragma unroll
        for (int k = 0; k < ITER; ++k) rr[0][k] = fetch(0, tid + 512 * k);
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
        Res (&r)[ITER] = rr[j];
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int q = q0 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * lh;   // 15x17 grid row
                ep[(bd_w * 256 + q) * SLD + wn * 32 + l32] = acc[i][j][e];
            }
        __syncthreads();
        if (j + 1 < FN && p.Rhi) {
#pragma unroll
            for (int k = 0; k < ITER; ++k) rr[j + 1][k] = fetch(j + 1, tid + 512 * k);
        }
#pragma unroll
        for (int k = 0; k < ITER; ++k) {
            const int v = tid + 512 * k;
            const int pix = v % 225, t = v / 225, gl = t % 8, bd = t / 8;
            const int b = b0 + bd;
            if (v < ITEMS && b < nboards) {
                const int nl = (gl / 4) * 64 + j * 32 + (gl % 4) * 8, n = n0 + nl;
                const float* src = ep + (bd * 256 + (pix / 15) * 17 + pix % 15) * SLD + gl * 8;
                const float4 x0 = *reinterpret_cast<const float4*>(src);
                const float4 x1 = *reinterpret_cast<const float4*>(src + 4);
                const float4 c0v = *reinterpret_cast<const float4*>(sbias + nl);
                const float4 c1v = *reinterpret_cast<const float4*>(sbias + nl + 4);
                float o[8] = {x0.x + c0v.x, x0.y + c0v.y, x0.z + c0v.z, x0.w + c0v.w,
                              x1.x + c1v.x, x1.y + c1v.y, x1.z + c1v.z, x1.w + c1v.w};
                if (p.Rhi) {
                    uint16_t hh[8];
                    int8_t qq[8];
                    *reinterpret_cast<uint4*>(hh) = r[k].h;
                    *reinterpret_cast<uint2*>(qq) = r[k].q;
#pragma unroll
                    for (int e = 0; e < 8; ++e) o[e] += H16::join(hh[e], qq[e]);
                }
                uint16_t oh[8];
                int8_t oq[8];
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    if (p.relu) o[e] = o[e] > 0.0f ? o[e] : 0.0f;
                    H16::split(o[e], oh[e], oq[e]);
                }
                const size_t e = (((size_t)b * GO + n / 8) * 225 + pix) * 8;
                *reinterpret_cast<uint4*>(p.Chi + e) = *reinterpret_cast<const uint4*>(oh);
                if (p.Cq) *reinterpret_cast<uint2*>(p.Cq + e) = *reinterpret_cast<const uint2*>(oq);
                if (p.Cf) {                            // fp32 NHWC (the trunk output the pool reads)
                    float* cf = p.Cf + ((size_t)b * 225 + pix) * p.N + n;
                    *reinterpret_cast<float4*>(cf) = make_float4(o[0], o[1], o[2], o[3]);
                    *reinterpret_cast<float4*>(cf + 4) = make_float4(o[4], o[5], o[6], o[7]);
                }
            }
        }
        __syncthreads();
    }
    V4_STAMP(2);
}

// ===========================================================================
// v6: the v5 board-halo conv on v_mfma_f32_16x16x32_{f16,bf16}.  The 16x16x32 shape draws less
// power than 32x32x16 for the same FLOPs, and this kernel is power-bound (the chip holds
// ~1.8 GHz under v5; a bare-loop microbenchmark, tools/microbench/mfma_shape.hip, runs
// 16x16x32 at ~2.0 GHz vs ~1.6 GHz).  K = 32 per MFMA = one tap x 32 channels, so a chunk is
// 32 channels: the halo of both boards (40 KB) is double-buffered per chunk and the weights run
// through a 3-deep ring of tap rows (3 taps x 8 KB), one barrier per tap row.  A wave owns 128
// rows x 64 columns as 8 x 4 tiles of 16x16 (128 accumulators).  Fragments of the next tap are
// read while the current tap's MFMAs issue: B(t+1) first, then the low / high halves of A(t+1)
// as soon as the matching half of tap t has issued.  DMA pieces (weights of tap row s+2, and at
// the first row of a chunk the halo of the next chunk) ride between MFMAs.
template <int OFF, typename F>
__device__ __forceinline__ void ds_rd_off(F& d, uint32_t addr) {
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d) : "v"(addr), "i"(OFF) : "memory");
}
template <int I, int N, typename Fn>
__device__ __forceinline__ void static_for(Fn&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<I + 1, N>(f);
    }
}

#define AZ_LGKM_WAIT(N, X)                                                                        \
    asm volatile("s_waitcnt lgkmcnt(" #N ")" : "+v"(X[0]), "+v"(X[1]), "+v"(X[2]), "+v"(X[3]))

// Board geometry of conv3x3_v6 for an HB x HB board: outputs on an HB x (HB+2) grid (two dead
// columns) so tap (dy, dx) of 16 consecutive outputs is 16 consecutive rows of the zero-padded
// (HB+2)^2 halo.
//  * 15x15 (FLAT = false): a board's grid is padded to 256 rows and a 512-row block tile holds two
//    boards (88% live rows).
//  * other boards (FLAT = true): boards are laid end to end, S = (HB+1)(HB+2) grid rows each -- the
//    bottom zero row of the halo of board b is the top zero row of board b+1, so output row Q of
//    the flattened sequence reads halo row Q + dy*WG + dx for every board at once -- and a tile is
//    any 512 consecutive rows, which may span boards (live rows 19x19: 86% instead of 71% with one
//    board per tile; 13x13 80% / 66%; 9x9 74% / 63%; 8x8 71% / 50%).
//  * DENSE (any board): no padding rows or columns at all -- output row Q of a tile is pixel
//    tile*512 + Q of the batch, it reads input pixel Q + (dy-1)*HB + (dx-1), i.e. halo row
//    Q + dy*HB + dx of a halo that starts HB+1 pixels before the tile, and the taps that cross a
//    board edge are zeroed in the A fragments (per-lane masks: x = 0 / HB-1 for dx = 0 / 2,
//    y = 0 / HB-1 for dy = 0 / 2).  Every MFMA row is a live output (100% at every board size,
//    the last tile aside) for 8 v_cndmask per fragment and tap.
template <int HB, bool DENSE_ = false>
struct G8Geom {
    static constexpr bool DENSE = DENSE_;
    static constexpr bool FLAT = DENSE || HB != 15;
    static constexpr int WG = DENSE ? HB : HB + 2;          // grid / halo row width
    static constexpr int HALO = (HB + 2) * (HB + 2);        // halo rows per board (one board per tile)
    static constexpr int S = DENSE ? HB * HB : (HB + 1) * WG;   // FLAT: grid rows per board
    static constexpr int TROWS = 512 + 2 * WG + 2;          // FLAT: halo rows one 512-row tile reads
    static constexpr int HROWS = ((FLAT ? TROWS : HALO) + 63) / 64 * 64;   // whole 1 KiB DMA pieces
    static constexpr int HP = HROWS / 64;                   // pieces per (board, 8-channel group)
    static constexpr int OUTR = HB * WG;                    // grid rows per board
    static constexpr int OUTP = FLAT ? 512 : OUTR <= 128 ? 128 : OUTR <= 256 ? 256 : 512;
    static constexpr int BOARDS = 512 / OUTP;               // FLAT: one flattened tile
    static constexpr int HW = HB * HB;
    static_assert(OUTR <= 512, "board too large for a 512-row tile");
};

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
template <int MODE, int HB = 15, bool DENSE = false>
__global__ __launch_bounds__(512, 1) void conv3x3_v6(ConvBf16Args p) {
    static_assert(MODE == 1 || MODE == 2, "v6: single-plane modes");
    typedef Half16<MODE> H16;
    typedef G8Geom<HB, DENSE> GM;
    constexpr int BNT = 128, BOARDS = GM::BOARDS, KG = 4, WG = GM::WG, HW = GM::HW, OUTP = GM::OUTP;
    constexpr int A_PLANE = KG * GM::HROWS * 16;         // one board, 32 channels: [4 groups][halo rows][16 B]
    constexpr int A_BUF = BOARDS * A_PLANE;              // 40 KB at 15x15
    constexpr int B_TAP = KG * BNT * 16;                 // 8 KB
    constexpr int B_STAGE = 3 * B_TAP;                   // one tap row, 24 KB
    constexpr int LDS_MAIN = 2 * A_BUF + 3 * B_STAGE;    // 152 KB
    constexpr int SC = 64, SLD = SC + 4;
    constexpr int LDS_EPI = BOARDS * OUTP * SLD * 4;     // 136 KB
    constexpr int LDS_BIAS = LDS_MAIN > LDS_EPI ? LDS_MAIN : LDS_EPI;
    constexpr int LDS = LDS_BIAS + BNT * 4;
    constexpr int A_INS = BOARDS * KG * GM::HP;          // 40 pieces per chunk at 15x15
    constexpr int B_INS = 3 * KG * (BNT / 64);           // 24 pieces per tap row
    constexpr int PA = (A_INS + 7) / 8, PB = B_INS / 8;  // 5 / 3 per wave at 15x15
    static_assert(B_INS % 8 == 0 && PA + PB <= 9, "piece schedule");
    constexpr int WN = 2, TM = 128, FM = 8, FN = 4;
    typedef typename std::conditional<MODE == 2, f16x8, bf16x8>::type frag;
    typedef float f32x4v __attribute__((ext_vector_type(4)));
    __shared__ __attribute__((aligned(16))) uint8_t lds[LDS];

    V4_STAMP(0);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: keeps piece offsets in SGPRs
    const int wm = wave / WN, wn = wave % WN;
    const int nsplit = p.N / BNT;
    const int xcd = blockIdx.x % 8, slot = blockIdx.x / 8;
    const int nb = slot % nsplit, pair = (slot / nsplit) * 8 + xcd;
    const int n0 = nb * BNT;
    const int nboards = p.m_limit ? *p.m_limit : p.M / (p.H * p.W);
    const int b0 = pair * BOARDS;                        // FLAT: pair is the tile index
    if (GM::FLAT ? pair * 512 >= nboards * GM::S : b0 >= nboards) return;
    V4_STAMP(3);
    const int C = p.C, GI = C / 8, GO = p.N / 8;
    const int NCH = C / 32, NS = NCH * 3;

    // DMA through buffer descriptors: one 32-bit VGPR offset per piece; padding halo rows use an
    // offset past the end of the activation buffer, which the range check turns into zeros
    // (a range-checked LDS-DMA load is dropped, not zero-filled, so padding rows read the zeroed
    // tail AZ_ACT_TAIL behind the activation buffer; the per-chunk step keeps them inside it)
    // a_bytes: where the zeroed tail starts (the allocation's capacity, not this batch's rows)
    const uint32_t a_bytes = (uint32_t)p.a_tail, b_bytes = (uint32_t)((size_t)9 * C * p.N * 2);
    const __amdgpu_buffer_rsrc_t rsA =
        __builtin_amdgcn_make_buffer_rsrc((void*)p.Ahi, (short)0, (int)(a_bytes + AZ_ACT_TAIL * 2), 0x00020000);
    const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc((void*)p.Bblk, (short)0, (int)b_bytes, 0x00020000);
    const uint32_t PAD = a_bytes;
#define AZ_RSA rsA
#define AZ_RSB rsB
#define AZ_SKIP_A
#define AZ_SKIP_B
    uint32_t a_vo[PA];
    int a_off[PA];
#pragma unroll
    for (int j = 0; j < PA; ++j) {
        const int q = wave + 8 * j;
        const int rb = q % GM::HP, g = (q / GM::HP) % KG, bd = q / (GM::HP * KG);
        const int hr = rb * 64 + lane;
        int Y, X, b;
        bool in;
        if constexpr (GM::DENSE) {                         // halo row -> pixel pair*512 - HB - 1 + hr
            const int gpx = pair * 512 - (HB + 1) + hr;
            b = gpx >= 0 ? gpx / HW : -1;
            const int pix = gpx - b * HW;
            Y = pix / HB + 1; X = pix - (Y - 1) * HB + 1;
            in = hr < GM::TROWS && gpx >= 0;
        } else if constexpr (GM::FLAT) {                   // flattened halo row -> (board, Y, X)
            const int h = pair * 512 + hr;
            b = h / GM::S;
            const int rr = h - b * GM::S;
            Y = rr / WG; X = rr - Y * WG;
            in = hr < GM::TROWS;
        } else {
            Y = hr / WG; X = hr - Y * WG;
            b = b0 + bd;
            in = hr < GM::HALO;
        }
        const bool ok = in && Y >= 1 && Y <= HB && X >= 1 && X <= HB && b < nboards;
        a_vo[j] = ok ? (uint32_t)((((size_t)b * GI + g) * HW + (Y - 1) * HB + (X - 1)) * 16) : PAD;
        a_off[j] = bd * A_PLANE + g * (GM::HROWS * 16) + rb * 1024;
    }
    int b_bo[PB], b_off[PB];   // wave-uniform byte offsets; the lane adds lane * 16
#pragma unroll
    for (int j = 0; j < PB; ++j) {
        const int q = wave + 8 * j;
        const int rb = q % 2, g = (q / 2) % KG, t = q / (2 * KG);
        b_bo[j] = ((((g >> 1) * 9 + t) * 2 + (g & 1)) * p.N + n0 + rb * 64) * 16;
        b_off[j] = t * B_TAP + g * BNT * 16 + rb * 1024;
    }
    const uint32_t lane16 = lane * 16;
    uint8_t* abuf = lds;
    uint8_t* bbuf = lds + 2 * A_BUF;
    auto issueA = [&](int j, int c) {
        if (A_INS % 8 != 0 && wave + 8 * j >= A_INS) return;   // wave-uniform
        AZ_SKIP_A
        __builtin_amdgcn_raw_ptr_buffer_load_lds(AZ_RSA, (lds_void_t*)(abuf + (c & 1) * A_BUF + a_off[j]), 16,
                                                 (int)(a_vo[j] + (uint32_t)c * (KG * HW * 16)), 0, 0, 0);
    };
    auto issueB = [&](int j, int s) {
        const int c = s / 3, r = s - 3 * c;
        AZ_SKIP_B
        __builtin_amdgcn_raw_ptr_buffer_load_lds(AZ_RSB, (lds_void_t*)(bbuf + (s % 3) * B_STAGE + b_off[j]), 16,
                                                 (int)(lane16 + (uint32_t)(b_bo[j] + (36 * c + 6 * r) * p.N * 16)), 0, 0, 0);
    };

    f32x4v acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
            // the bias seeds the accumulators (the lane's column is wn*64 + j*16 + l16), so the
            // epilogue adds nothing for it
            const float bj = p.bias[n0 + wn * 64 + j * 16 + (lane & 15)];
            acc[i][j] = f32x4v{bj, bj, bj, bj};
        }

    // prologue: halo of chunk 0, weights of tap rows 0 and 1
#pragma unroll
    for (int j = 0; j < PA; ++j) issueA(j, 0);
#pragma unroll
    for (int j = 0; j < PB; ++j) issueB(j, 0);
    if (NS > 1) {
#pragma unroll
        for (int j = 0; j < PB; ++j) issueB(j, 1);
    }
    const int bd_w = (wm * TM) / OUTP, q0 = (wm * TM) % OUTP;
    const int l16 = lane & 15, lg = lane >> 4;
    const uint32_t a_lane = lds_addr(abuf) + bd_w * A_PLANE + lg * (GM::HROWS * 16) + (q0 + l16) * 16;
    const uint32_t b_lane = lds_addr(bbuf) + lg * (BNT * 16) + (wn * 64 + l16) * 16;
    // DENSE: board-edge bits of the output row behind each of the lane's 8 A fragments,
    // 4 bits per fragment f: x = 0, x = HB-1, y = 0, y = HB-1
    uint32_t mbits = 0;
    if constexpr (GM::DENSE) {
#pragma unroll
        for (int f = 0; f < 8; ++f) {
            const int gq = pair * 512 + q0 + f * 16 + l16;
            const int pix = gq % HW, y = pix / HB, x = pix - y * HB;
            mbits |= ((x == 0 ? 1u : 0u) | (x == HB - 1 ? 2u : 0u) | (y == 0 ? 4u : 0u) | (y == HB - 1 ? 8u : 0u)) << (4 * f);
        }
    }
    for (int s = 0; s < NS; ++s) {
        const int c = s / 3, r = s - 3 * c;
        // retire B(s) (and A(c) at r == 0): pieces issued after B(s) may stay in flight
        // halo pieces this wave really issues per chunk: issueA skips wave + 8j >= A_INS, so where
        // A_INS is not a multiple of 8 (FLAT / DENSE tiles: 36) waves differ by one, and the vmcnt
        // budget must count exactly or a wave could pass its wait with a weight piece in flight
        const int pa_w = A_INS / 8 + (wave < A_INS % 8 ? 1 : 0);
        auto issued = [&](int u) {          // pieces this wave issued during tap row u
            return (u + 2 < NS ? PB : 0) + ((u % 3) == 0 && u / 3 + 1 < NCH ? pa_w : 0);
        };
        int allow;
        if (s == 0) allow = NS > 1 ? PB : 0;
        else allow = issued(s - 1) + (s >= 2 && ((s - 2) % 3) == 0 && (s - 2) / 3 + 1 < NCH ? pa_w : 0);
        wait_vm(allow);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        const uint32_t ab = a_lane + (c & 1) * A_BUF;
        const uint32_t bb = b_lane + (s % 3) * B_STAGE;
        const int npieces = (s + 2 < NS ? PB : 0) + (r == 0 && c + 1 < NCH ? PA : 0);
        // piece k of this row: weights of row s+2 first, then the next chunk's halo
        auto piece = [&](int k) {
            if (k >= npieces) return;
            if (s + 2 < NS) {
                if (k < PB) { issueB(k, s + 2); return; }
                k -= PB;
            }
            issueA(k, c + 1);
        };
        frag alo[4], ahi[4], bc[4], bn[4];
        const uint32_t abr = ab + r * (WG * 16);       // tap row r: halo rows shifted by WG r
        // DENSE: zero the A rows whose tap (r, t) crosses a board edge
        const uint32_t rtest = r == 0 ? 4u : r == 2 ? 8u : 0u;
        auto maskA = [&](frag (&a)[4], int half, int t) {
            if constexpr (GM::DENSE) {
                const uint32_t test = rtest | (t == 0 ? 1u : t == 2 ? 2u : 0u);
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if (mbits & (test << (4 * (half * 4 + i)))) a[i] = frag{};
            }
        };
        // fragment reads with compile-time LDS offsets (one base VGPR per operand)
        auto loadA = [&](frag (&a)[4], auto tc, auto hc) {
            constexpr int t = decltype(tc)::value, half = decltype(hc)::value;
            static_for<0, 4>([&](auto ic) {
                constexpr int i = decltype(ic)::value;
                ds_rd_off<((half * 4 + i) * 16 + t) * 16>(a[i], abr);
            });
        };
        auto loadB = [&](frag (&b)[4], auto tc) {
            constexpr int t = decltype(tc)::value;
            static_for<0, FN>([&](auto jc) {
                constexpr int j = decltype(jc)::value;
                ds_rd_off<t * B_TAP + j * 16 * 16>(b[j], bb);
            });
        };
        using I0 = std::integral_constant<int, 0>;
        using I1 = std::integral_constant<int, 1>;
        using I2 = std::integral_constant<int, 2>;
        auto mma = [&](const frag (&a)[4], const frag (&b)[4], int half, int t) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                // DMA slots per tap: before rows 0 and 2 of the low half, row 0 of the high half
                if ((half == 0 && (i == 0 || i == 2)) || (half == 1 && i == 0)) {
                    __builtin_amdgcn_sched_barrier(0);
                    piece(t * 3 + (half == 0 ? (i >> 1) : 2));
                    __builtin_amdgcn_sched_barrier(0);
                }
#pragma unroll
                for (int j = 0; j < FN; ++j) {
                    if constexpr (MODE == 2)
                        acc[half * 4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[i], b[j], acc[half * 4 + i][j], 0, 0, 0);
                    else
                        acc[half * 4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[half * 4 + i][j], 0, 0, 0);
                }
            }
        };
        loadA(alo, I0{}, I0{});
        loadA(ahi, I0{}, I1{});
        loadB(bc, I0{});
        // tap 0
        loadB(bn, I1{});
        AZ_LGKM_WAIT(4, alo); AZ_LGKM_WAIT(4, bc);
        maskA(alo, 0, 0);
        mma(alo, bc, 0, 0);
        loadA(alo, I1{}, I0{});
        AZ_LGKM_WAIT(8, ahi);
        maskA(ahi, 1, 0);
        mma(ahi, bc, 1, 0);
        loadA(ahi, I1{}, I1{});
        // tap 1 (bn holds B(1))
        loadB(bc, I2{});
        AZ_LGKM_WAIT(8, alo); AZ_LGKM_WAIT(8, bn);
        maskA(alo, 0, 1);
        mma(alo, bn, 0, 1);
        loadA(alo, I2{}, I0{});
        AZ_LGKM_WAIT(8, ahi);
        maskA(ahi, 1, 1);
        mma(ahi, bn, 1, 1);
        loadA(ahi, I2{}, I1{});
        // tap 2 (bc holds B(2))
        AZ_LGKM_WAIT(4, alo); AZ_LGKM_WAIT(4, bc);
        maskA(alo, 0, 2);
        mma(alo, bc, 0, 2);
        AZ_LGKM_WAIT(0, ahi);
        maskA(ahi, 1, 2);
        mma(ahi, bc, 1, 2);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();
    V4_STAMP(1);

    // epilogue (as v5): two 64-column passes over the block's boards, staged [BOARDS][OUTP][68] fp32
    constexpr int ITEMS = GM::FLAT ? 512 * (SC / 8) : BOARDS * (SC / 8) * HW;
    constexpr int ITER = (ITEMS + 511) / 512;
    float* ep = reinterpret_cast<float*>(lds);
    struct Res { uint4 h; uint2 q; };
    // item v -> (board, pixel, 8-channel group gl, staged row); live: a real output of this tile
    struct Item { int b, pix, gl, srow; bool live; };
    auto item = [&](int v) {
        Item it;
        if constexpr (GM::DENSE) {                         // v = gl * 512 + tile row = pixel pair*512 + row
            const int row = v & 511;
            it.gl = v >> 9;
            const int h = pair * 512 + row;
            it.b = h / HW;
            it.pix = h - it.b * HW;
            it.srow = row;
            it.live = it.b < nboards;
        } else if constexpr (GM::FLAT) {                   // v = gl * 512 + tile row (rows contiguous)
            const int row = v & 511;
            it.gl = v >> 9;
            const int h = pair * 512 + row;
            it.b = h / GM::S;
            const int rr = h - it.b * GM::S, y = rr / WG, x = rr - y * WG;
            it.pix = y * HB + x;
            it.srow = row;
            it.live = y < HB && x < HB && it.b < nboards;
        } else {
            it.pix = v % HW;
            const int t = v / HW, bd = t / 8;
            it.gl = t % 8;
            it.b = b0 + bd;
            it.srow = bd * OUTP + (it.pix / HB) * WG + it.pix % HB;
            it.live = v < ITEMS && it.b < nboards;
        }
        return it;
    };
    constexpr bool d_noload = false, d_nostore = false;
    auto fetch = [&](int pp, int v) {
        Res rr{};
        const Item it = item(v);
        const int pix = it.pix, gl = it.gl, b = it.b;
        if (it.live && !d_noload) {
            const int n = n0 + (gl / 4) * 64 + pp * 32 + (gl % 4) * 8;
            const size_t e = (((size_t)b * GO + n / 8) * HW + pix) * 8;
            // streaming (nt) loads: the residual is read once (-2% trunk time at C3)
            const __amdgpu_buffer_rsrc_t rh = __builtin_amdgcn_make_buffer_rsrc((void*)p.Rhi, (short)0, 0x7fffffff, 0x00020000);
            const __amdgpu_buffer_rsrc_t rqq = __builtin_amdgcn_make_buffer_rsrc((void*)p.Rq, (short)0, 0x7fffffff, 0x00020000);
            const u32x4_t h = __builtin_amdgcn_raw_buffer_load_b128(rh, (int)(e * 2), 0, AZ_RES_AUX);
            const u32x2_t q = __builtin_amdgcn_raw_buffer_load_b64(rqq, (int)e, 0, AZ_RES_AUX);
            __builtin_memcpy(&rr.h, &h, 16);
            __builtin_memcpy(&rr.q, &q, 8);
        }
        return rr;
    };
    Res rq[2][ITER];
    if (p.Rhi) {
#pragma unroll
        for (int k = 0; k < ITER; ++k) rq[0][k] = fetch(0, tid + 512 * k);
    }
    float vmax = 0.0f;                                // fp16: the largest |output| (the range guard)
#pragma unroll
    for (int pp = 0; pp < 2; ++pp) {
        Res (&rres)[ITER] = rq[pp];
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int jj = 0; jj < 2; ++jj)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int row = q0 + i * 16 + lg * 4 + e;            // HB x WG grid row of the board
                    ep[(bd_w * OUTP + row) * SLD + wn * 32 + jj * 16 + l16] = acc[i][2 * pp + jj][e];
                }
        __syncthreads();
        if (pp == 0 && p.Rhi) {
#pragma unroll
            for (int k = 0; k < ITER; ++k) rq[1][k] = fetch(1, tid + 512 * k);
        }
#pragma unroll
        for (int k = 0; k < ITER; ++k) {
            const int v = tid + 512 * k;
            const Item it = item(v);
            const int pix = it.pix, gl = it.gl, b = it.b;
            if (it.live) {
                const int nl = (gl / 4) * 64 + pp * 32 + (gl % 4) * 8, n = n0 + nl;
                const float* src = ep + it.srow * SLD + gl * 8;
                const float4 x0 = *reinterpret_cast<const float4*>(src);
                const float4 x1 = *reinterpret_cast<const float4*>(src + 4);
                float o[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
                if (p.Rhi) {
                    uint16_t hh[8];
                    int8_t qq[8];
                    *reinterpret_cast<uint4*>(hh) = rres[k].h;
                    *reinterpret_cast<uint2*>(qq) = rres[k].q;
#pragma unroll
                    for (int e = 0; e < 8; ++e) o[e] += H16::join(hh[e], qq[e]);
                }
                uint16_t oh[8];
                int8_t oq[8];
#pragma unroll
                for (int e = 0; e < 8; ++e) o[e] = __builtin_amdgcn_fmed3f(o[e], 0.0f, 3.0e38f);   // ReLU: every g8 conv has one
                if constexpr (MODE == 2) {
#pragma unroll
                    for (int e = 0; e < 8; ++e) vmax = __builtin_fmaxf(vmax, o[e]);
                }
                if (p.Cq) {                                // residual-stream output: 16-bit + int8 remainder
#pragma unroll
                    for (int e = 0; e < 8; ++e) H16::split(o[e], oh[e], oq[e]);
                } else {
#pragma unroll
                    for (int e = 0; e < 8; ++e) oh[e] = H16::from_f(o[e]);
                }
                const size_t e = (((size_t)b * GO + n / 8) * HW + pix) * 8;
                if (d_nostore && o[0] != 1234.5f) continue;
                {                                          // streaming (nt) output stores (-1%)
                    u32x4_t h; __builtin_memcpy(&h, oh, 16);
                    asm volatile("global_store_dwordx4 %0, %1, off nt" ::"v"(p.Chi + e), "v"(h) : "memory");
                    if (p.Cq) {
                        u32x2_t q; __builtin_memcpy(&q, oq, 8);
                        asm volatile("global_store_dwordx2 %0, %1, off nt" ::"v"(p.Cq + e), "v"(q) : "memory");
                    }
                }
                if (p.Cf) {
                    float* cf = p.Cf + ((size_t)b * HW + pix) * p.N + n;
                    *reinterpret_cast<float4*>(cf) = make_float4(o[0], o[1], o[2], o[3]);
                    *reinterpret_cast<float4*>(cf + 4) = make_float4(o[4], o[5], o[6], o[7]);
                }
            }
        }
        __syncthreads();
    }
    if (MODE == 2 && !(vmax <= 65504.0f) && p.ovf) atomicOr(p.ovf, 1);   // fp16 overflow: the engine fails the forward
    V4_STAMP(2);
}

#undef AZ_RSA
#undef AZ_RSB
#undef AZ_SKIP_A
#undef AZ_SKIP_B

// fp32 NHWC [B*HW][C] -> g8 16-bit + int8 remainder (the first trunk input and residual)
// Cout >= C (a multiple of 8): groups C/8 .. Cout/8-1 of the output are zero (channel padding)
template <int MODE>
__global__ void k_to_g8(const float* in, uint16_t* hi, int8_t* q, int C, int HW, const int* m_limit, int maxB, int Cout) {
    const int G = Cout / 8, GI = C / 8;
    const int B = m_limit ? min(*m_limit, maxB) : maxB;
    const size_t total = (size_t)B * G * HW;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const int pix = (int)(i % HW);
        const size_t bg = i / HW;
        const int g = (int)(bg % G);
        const size_t b = bg / G;
        float4 v0 = {0.0f, 0.0f, 0.0f, 0.0f}, v1 = v0;
        if (g < GI) {
            const float* src = in + (b * HW + pix) * C + g * 8;
            v0 = *reinterpret_cast<const float4*>(src);
            v1 = *reinterpret_cast<const float4*>(src + 4);
        }
        const float f[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
        uint16_t h[8];
        int8_t r[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) Half16<MODE>::split(f[e], h[e], r[e]);
        *reinterpret_cast<uint4*>(hi + i * 8) = *reinterpret_cast<const uint4*>(h);
        if (q) *reinterpret_cast<uint2*>(q + i * 8) = *reinterpret_cast<const uint2*>(r);
    }
}

// fp32 NHWC [B*HW][C] -> g8 hi + lo planes: PT 1 bf16 pieces (AZ_PREC_BF16X3: hi = bf16(x), lo =
// bf16(x - hi)), PT 2 fp16 pieces (AZ_PREC_F16X3, with the fp16 range guard)
template <int PT>
__global__ void k_to_g8x3(const float* in, uint16_t* hi, uint16_t* lo, int C, int HW, const int* m_limit, int maxB,
                          int* ovf) {
    float vmax = 0.0f;
    const int G = C / 8;
    const int B = m_limit ? min(*m_limit, maxB) : maxB;
    const size_t total = (size_t)B * G * HW;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const int pix = (int)(i % HW);
        const size_t bg = i / HW;
        const int g = (int)(bg % G);
        const size_t b = bg / G;
        const float* src = in + (b * HW + pix) * C + g * 8;
        const float4 v0 = *reinterpret_cast<const float4*>(src);
        const float4 v1 = *reinterpret_cast<const float4*>(src + 4);
        const float f[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
        uint16_t h[8], l[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            h[e] = Half16<PT>::from_f(f[e]);
            l[e] = Half16<PT>::from_f(f[e] - Half16<PT>::to_f(h[e]));
            if (PT == 2) vmax = fmaxf(vmax, fabsf(f[e]));
        }
        *reinterpret_cast<uint4*>(hi + i * 8) = *reinterpret_cast<const uint4*>(h);
        *reinterpret_cast<uint4*>(lo + i * 8) = *reinterpret_cast<const uint4*>(l);
    }
    if (PT == 2 && !(vmax <= 65504.0f) && ovf) atomicOr(ovf, 1);
}

void az_launch_to_g8x3(const float* in, uint16_t* hi, uint16_t* lo, int C, int HW, const int* m_limit, int maxB,
                       hipStream_t st, int pt, int* ovf) {
    if (pt == 2) hipLaunchKernelGGL(k_to_g8x3<2>, dim3(2048), dim3(256), 0, st, in, hi, lo, C, HW, m_limit, maxB, ovf);
    else hipLaunchKernelGGL(k_to_g8x3<1>, dim3(2048), dim3(256), 0, st, in, hi, lo, C, HW, m_limit, maxB, ovf);
}

void az_launch_to_g8(const float* in, uint16_t* hi, int8_t* q, int C, int HW, const int* m_limit, int maxB, int mode,
                     hipStream_t st, int Cout) {
    if (Cout < C) Cout = C;
    if (mode == 2) hipLaunchKernelGGL(k_to_g8<2>, dim3(2048), dim3(256), 0, st, in, hi, q, C, HW, m_limit, maxB, Cout);
    else hipLaunchKernelGGL(k_to_g8<1>, dim3(2048), dim3(256), 0, st, in, hi, q, C, HW, m_limit, maxB, Cout);
}

// The search's leaf records -> the g8 16-bit input of the input conv (16 channels = two groups of 8):
// board b's planes are built from record gidx[b] (leaf_planes.h) and rounded as k_to_g8 rounds them.
// NG 8-channel groups per board: the 16 planes in groups 0-1, zeros in 2..NG-1 (a 32-channel input conv)
template <int MODE>
__global__ void k_rec_to_g8(const uint8_t* rec, const int* gidx, uint16_t* hi, int go, int bs, const int* m_limit,
                            int maxB, int NG) {
    const int HW = bs * bs;
    const int B = m_limit ? min(*m_limit, maxB) : maxB;
    const size_t total = (size_t)B * HW;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const int pix = (int)(i % HW);
        const size_t b = i / HW;
        float c[16];
        az_leaf_planes(rec + (size_t)gidx[b] * AZ_REC_BYTES, go, bs, pix, c);
#pragma unroll
        for (int g = 0; g < 2; ++g) {
            uint16_t h[8];
            int8_t r[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) Half16<MODE>::split(c[8 * g + e], h[e], r[e]);
            *reinterpret_cast<uint4*>(hi + ((b * NG + g) * HW + pix) * 8) = *reinterpret_cast<const uint4*>(h);
        }
        for (int g = 2; g < NG; ++g) *reinterpret_cast<uint4*>(hi + ((b * NG + g) * HW + pix) * 8) = uint4{0, 0, 0, 0};
    }
}

void az_launch_rec_to_g8(const uint8_t* rec, const int* gidx, uint16_t* hi, int go, int bs, const int* m_limit, int maxB,
                         int mode, hipStream_t st, int NG) {
    if (mode == 2) hipLaunchKernelGGL(k_rec_to_g8<2>, dim3(1024), dim3(256), 0, st, rec, gidx, hi, go, bs, m_limit, maxB, NG);
    else hipLaunchKernelGGL(k_rec_to_g8<1>, dim3(1024), dim3(256), 0, st, rec, gidx, hi, go, bs, m_limit, maxB, NG);
}

// adaptive_avg_pool2d(x, (P, P)) of an H x H g8 trunk output (16-bit + int8 remainder) -> fp32 NHWC
// [B][P*P][C]; one thread per (board, 8-channel group, output cell), same summation order as
// k_adaptive_pool (rows, then columns; sum / kh / kw)
// Adaptive average pool of the g8 trunk output (16-bit + int8 remainder) to P x P, fp32
// [B][P*P][C] for the head 1x1 convs.  One block per (board, 32-channel slice): the slice's
// H*W x 32 values are read once, coalesced per 8-channel group, joined to fp32 in LDS (row stride
// 36 floats: conflict-free 16-byte writes; H*W*144 B of dynamic LDS), then every output sums its
// window from LDS in the same order as before (y-major, then x; / kh / kw).
// MODE 0 (AZ_PREC_BF16X3) / 3 (AZ_PREC_F16X3): q is the bf16 / fp16 lo plane (uint16 elements), x = hi + lo.
template <int MODE>
__global__ __launch_bounds__(256) void k_pool_g8(const uint16_t* hi, const int8_t* q, float* out, int C, int H, int P,
                                                 const int* m_limit, int maxB) {
    constexpr int SL = 36;                              // LDS row stride (floats) for 32 channels
    extern __shared__ __attribute__((aligned(16))) float f[];
    const int G = C / 8, HW = H * H, PP = P * P, NS = G / 4;
    const int B = m_limit ? min(*m_limit, maxB) : maxB;
    const int b = blockIdx.x / NS, sl = blockIdx.x - b * NS;
    if (b >= B) return;
    for (int idx = threadIdx.x; idx < 4 * HW; idx += 256) {
        const int gl = idx / HW, pix = idx - gl * HW;
        const size_t e = ((size_t)(b * G + sl * 4 + gl) * HW + pix) * 8;
        uint16_t h[8];
        float v[8];
        *reinterpret_cast<uint4*>(h) = *reinterpret_cast<const uint4*>(hi + e);
        if constexpr (MODE == 0 || MODE == 3) {
            constexpr int PM = MODE == 0 ? 1 : 2;
            uint16_t l[8];
            *reinterpret_cast<uint4*>(l) = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(q) + e);
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = Half16<PM>::to_f(h[k]) + Half16<PM>::to_f(l[k]);
        } else {
            int8_t r[8];
            *reinterpret_cast<uint2*>(r) = *reinterpret_cast<const uint2*>(q + e);
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = Half16<MODE>::join(h[k], r[k]);
        }
        float* d = f + pix * SL + gl * 8;
        *reinterpret_cast<float4*>(d) = make_float4(v[0], v[1], v[2], v[3]);
        *reinterpret_cast<float4*>(d + 4) = make_float4(v[4], v[5], v[6], v[7]);
    }
    __syncthreads();
    const int c8 = (threadIdx.x & 3) * 8;
    for (int o = threadIdx.x >> 2; o < PP; o += 64) {
        const int oy = o / P, ox = o - oy * P;
        const int y0 = (oy * H) / P, y1 = ((oy + 1) * H + P - 1) / P;
        const int x0 = (ox * H) / P, x1 = ((ox + 1) * H + P - 1) / P;
        float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int y = y0; y < y1; ++y)
            for (int x = x0; x < x1; ++x) {
                const float* src = f + (y * H + x) * SL + c8;
                const float4 t0 = *reinterpret_cast<const float4*>(src);
                const float4 t1 = *reinterpret_cast<const float4*>(src + 4);
                s[0] += t0.x; s[1] += t0.y; s[2] += t0.z; s[3] += t0.w;
                s[4] += t1.x; s[5] += t1.y; s[6] += t1.z; s[7] += t1.w;
            }
        const float kh = (float)(y1 - y0), kw = (float)(x1 - x0);
        float* dst = out + ((size_t)b * PP + o) * C + sl * 32 + c8;
        *reinterpret_cast<float4*>(dst) = make_float4(s[0] / kh / kw, s[1] / kh / kw, s[2] / kh / kw, s[3] / kh / kw);
        *reinterpret_cast<float4*>(dst + 4) = make_float4(s[4] / kh / kw, s[5] / kh / kw, s[6] / kh / kw, s[7] / kh / kw);
    }
}

void az_launch_pool_g8(const uint16_t* hi, const int8_t* q, float* out, int B, int C, int H, int P, const int* m_limit,
                       int mode, hipStream_t st) {
    const int grid = B * (C / 32);
    const size_t lds = (size_t)H * H * 36 * sizeof(float);
    if (mode == 2) hipLaunchKernelGGL(k_pool_g8<2>, dim3(grid), dim3(256), lds, st, hi, q, out, C, H, P, m_limit, B);
    else if (mode == 0) hipLaunchKernelGGL(k_pool_g8<0>, dim3(grid), dim3(256), lds, st, hi, q, out, C, H, P, m_limit, B);
    else if (mode == 3) hipLaunchKernelGGL(k_pool_g8<3>, dim3(grid), dim3(256), lds, st, hi, q, out, C, H, P, m_limit, B);
    else hipLaunchKernelGGL(k_pool_g8<1>, dim3(grid), dim3(256), lds, st, hi, q, out, C, H, P, m_limit, B);
}

// The trunk's tail in one launch: adaptive_avg_pool2d of the g8 trunk output to P x P and both head
// 1x1 convs ([policy | value], N = 64 outputs, ReLU) -- what k_pool_g8 + gemm_f32<64> computed with
// an fp32 round trip of the pooled map and a second launch.  One 256-thread block per board walks the
// channels in 32-channel slices: the slice is joined to fp32 in LDS (as k_pool_g8), pooled into
// pooled[cell][k] in the same summation order (rows, then columns; / kh / kw), and multiplied into
// the accumulators with v_mfma_f32_32x32x2_f32 over the slice's k pairs in ascending order -- the
// products, k pairing and order of gemm_f32's chain, so every output is bitwise the same.  The next
// slice's global loads are issued before the current slice is pooled.  Wave w owns the 32 x 32 tile
// (cells 32 (w >> 1).., outputs 32 (w & 1)..).  The slice's weights are prefetched with its
// activations (a weight load per slice on the critical path cost ~1 us each).
template <int MODE>
__global__ __launch_bounds__(256) void k_pool_heads_g8(const uint16_t* hi, const int8_t* q, const float* Wt,
                                                       const float* bias, float* out, int C, int H, int P,
                                                       const int* m_limit, int maxB) {
    constexpr int SL = 36, PL = 33;                     // LDS row strides (floats)
    extern __shared__ __attribute__((aligned(16))) float f[];
    const int G = C / 8, HW = H * H, PP = P * P, NS = G / 4;
    float* pl = f + HW * SL;                            // pooled slice [64 cells][PL]
    float* ws = pl + 64 * PL;                           // weight slice [64 outputs][PL]
    const int B = m_limit ? min(*m_limit, maxB) : maxB;
    const int b = blockIdx.x;
    if (b >= B) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1, kh = lane >> 5, l32 = lane & 31;
    constexpr int MAXI = (4 * 361 + 255) / 256;         // slice items per thread (19x19: 6)
    uint4 rh[MAXI];
    uint4 rl[MAXI];                                     // MODE 0 / 3: the lo plane (16 B); else .x/.y: int8 remainder
    float rw[8];                                        // the slice's weights: 64 outputs x 32 k
    auto load = [&](int sl) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int idx = tid + 256 * i, n = idx >> 5, k = idx & 31;
            rw[i] = Wt[(size_t)n * C + sl * 32 + k];
        }
#pragma unroll
        for (int i = 0; i < MAXI; ++i) {
            const int idx = tid + 256 * i;
            if (idx < 4 * HW) {
                const int gl = idx / HW, pix = idx - gl * HW;
                const size_t e = ((size_t)(b * G + sl * 4 + gl) * HW + pix) * 8;
                rh[i] = *reinterpret_cast<const uint4*>(hi + e);
                if constexpr (MODE == 0 || MODE == 3) rl[i] = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(q) + e);
                else { const uint2 r = *reinterpret_cast<const uint2*>(q + e); rl[i] = make_uint4(r.x, r.y, 0u, 0u); }
            }
        }
    };
    for (int i = tid; i < 64 * PL; i += 256) pl[i] = 0.0f;   // cells >= PP stay zero (their rows are not stored)
    floatx16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
    load(0);
    for (int sl = 0; sl < NS; ++sl) {
        // the slice joined to fp32 (k_pool_g8's values) and its weights [n][32]
#pragma unroll
        for (int i = 0; i < MAXI; ++i) {
            const int idx = tid + 256 * i;
            if (idx < 4 * HW) {
                const int gl = idx / HW, pix = idx - gl * HW;
                uint16_t h[8];
                float v[8];
                *reinterpret_cast<uint4*>(h) = rh[i];
                if constexpr (MODE == 0 || MODE == 3) {
                    constexpr int PM = MODE == 0 ? 1 : 2;
                    uint16_t l[8];
                    *reinterpret_cast<uint4*>(l) = rl[i];
#pragma unroll
                    for (int k = 0; k < 8; ++k) v[k] = Half16<PM>::to_f(h[k]) + Half16<PM>::to_f(l[k]);
                } else {
                    int8_t r[8];
                    *reinterpret_cast<uint2*>(r) = make_uint2(rl[i].x, rl[i].y);
#pragma unroll
                    for (int k = 0; k < 8; ++k) v[k] = Half16<MODE>::join(h[k], r[k]);
                }
                float* d = f + pix * SL + gl * 8;
                *reinterpret_cast<float4*>(d) = make_float4(v[0], v[1], v[2], v[3]);
                *reinterpret_cast<float4*>(d + 4) = make_float4(v[4], v[5], v[6], v[7]);
            }
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int idx = tid + 256 * i, n = idx >> 5, k = idx & 31;
            ws[n * PL + k] = rw[i];
        }
        __syncthreads();
        if (sl + 1 < NS) load(sl + 1);                  // in flight during the pool and the MFMAs
        {
            const int c8 = (tid & 3) * 8, o = tid >> 2;
            if (o < PP) {
                const int oy = o / P, ox = o - oy * P;
                const int y0 = (oy * H) / P, y1 = ((oy + 1) * H + P - 1) / P;
                const int x0 = (ox * H) / P, x1 = ((ox + 1) * H + P - 1) / P;
                float sm[8] = {0, 0, 0, 0, 0, 0, 0, 0};
                for (int y = y0; y < y1; ++y)
                    for (int x = x0; x < x1; ++x) {
                        const float* src = f + (y * H + x) * SL + c8;
                        const float4 t0 = *reinterpret_cast<const float4*>(src);
                        const float4 t1 = *reinterpret_cast<const float4*>(src + 4);
                        sm[0] += t0.x; sm[1] += t0.y; sm[2] += t0.z; sm[3] += t0.w;
                        sm[4] += t1.x; sm[5] += t1.y; sm[6] += t1.z; sm[7] += t1.w;
                    }
                const float kf = (float)(y1 - y0), kw = (float)(x1 - x0);
#pragma unroll
                for (int j = 0; j < 8; ++j) pl[o * PL + c8 + j] = sm[j] / kf / kw;
            }
        }
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < 16; ++kk) {
            const float a = pl[(32 * wm + l32) * PL + 2 * kk + kh];
            const float w = ws[(32 * wn + l32) * PL + 2 * kk + kh];
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, w, acc, 0, 0, 0);
        }
        __syncthreads();                                // f / pl / ws are rewritten by the next slice
    }
    const int n = 32 * wn + l32;
    const float bn = bias ? bias[n] : 0.0f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int m = 32 * wm + (r & 3) + 8 * (r >> 2) + 4 * kh;
        if (m < PP) {
            const float v = acc[r] + bn;
            out[((size_t)b * PP + m) * 64 + n] = v > 0.0f ? v : 0.0f;
        }
    }
}

// true when k_pool_heads_g8 takes this tail: 32-channel slices, at most 64 cells, both heads' 1x1
// convs = 64 outputs, the joined slice within the LDS budget
// k_pool_heads_g8's dynamic LDS: the board's pooled-cell partial sums + two 64 x 33 weight tiles
static size_t pool_heads_lds(int H) { return ((size_t)H * H * 36 + 2 * 64 * 33) * sizeof(float); }
// the device's LDS per workgroup (68.9 KB at 19x19 fits gfx950's 160 KB, not a 64 KB part)
static size_t device_lds_limit() {
    static const size_t lim = [] {
        int dev = 0, v = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) != hipSuccess)
            return (size_t)0;
        return (size_t)v;
    }();
    return lim;
}
bool az_pool_heads_supported(int C, int H, int P, int N) {
    return C % 32 == 0 && P * P <= 64 && N == 64 && H * H <= 361 && pool_heads_lds(H) <= device_lds_limit();
}

int az_launch_pool_heads_g8(const uint16_t* hi, const int8_t* q, const float* Wt, const float* bias, float* out, int B,
                            int C, int H, int P, int N, const int* m_limit, int mode, hipStream_t st) {
    if (!az_pool_heads_supported(C, H, P, N)) return -1;
    const size_t lds = pool_heads_lds(H);
    if (mode == 2) hipLaunchKernelGGL(k_pool_heads_g8<2>, dim3(B), dim3(256), lds, st, hi, q, Wt, bias, out, C, H, P, m_limit, B);
    else if (mode == 0) hipLaunchKernelGGL(k_pool_heads_g8<0>, dim3(B), dim3(256), lds, st, hi, q, Wt, bias, out, C, H, P, m_limit, B);
    else if (mode == 3) hipLaunchKernelGGL(k_pool_heads_g8<3>, dim3(B), dim3(256), lds, st, hi, q, Wt, bias, out, C, H, P, m_limit, B);
    else hipLaunchKernelGGL(k_pool_heads_g8<1>, dim3(B), dim3(256), lds, st, hi, q, Wt, bias, out, C, H, P, m_limit, B);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// true when the g8 trunk (conv3x3_v5 at 15x15 / conv3x3_v6) handles this shape: square boards with a
// G8Geom instantiation, 128-channel output halves, 16-channel chunks (v5, 15x15) or 32 (v6)
static bool g8_board(int H) { return H == 8 || H == 9 || H == 13 || H == 15 || H == 19; }
bool az_conv_g8_supported(int H, int W, int C, int N) {
    if (H != W || !g8_board(H) || N % 128 != 0 || C < 16) return false;
    return H == 15 ? C % 16 == 0 : C % 32 == 0;
}

static int g_conv_flags = 4 | 0x200;   // bit 2: v6 (16x16x32) at 15x15; 0x200: v7 on 15x15 boards only
// Variant bits for A/B measurement inside one process (tools/net_bench.py --flags); none defined now
// (a residual L2 prefetch during the main loop measured 0.6% slower and was removed; a cross-row
// fragment prefetch and a mid-row barrier variant measured 1.5-2% slower)
extern "C" int az_diag_set_conv_flags(int flags) { g_conv_flags = flags; return 0; }
extern "C" int az_diag_conv_flags(void) { return g_conv_flags; }   // the current set (bench.py ORs bits into it)
int az_conv_flags() { return g_conv_flags; }

template <int HB, bool DENSE>
static void v6_launch_g(const ConvBf16Args& a, int mode, hipStream_t st) {
    typedef G8Geom<HB, DENSE> GM;
    const int boards = a.M / GM::HW;
    const int groups = GM::FLAT ? (boards * GM::S + 511) / 512 : (boards + GM::BOARDS - 1) / GM::BOARDS;
    const int grid = (groups + 7) / 8 * 8 * (a.N / 128);   // XCD-aware group/half mapping: whole groups of 8
    if (mode == 2) hipLaunchKernelGGL((conv3x3_v6<2, HB, DENSE>), dim3(grid), dim3(512), 0, st, a);
    else hipLaunchKernelGGL((conv3x3_v6<1, HB, DENSE>), dim3(grid), dim3(512), 0, st, a);
}
// DENSE is the default for every board but 15x15, where two padded boards fill a 512-row tile
// at 88% and B = 2048 comes to exactly 8 rounds of 256 blocks (dense: 1800 blocks, still 8
// rounds, plus the masking).  Measured at B = 2048 (tools/net_bench.py --flags 0x4,0xc): dense
// 19x19 -3.1%, 13x13 -4.0%, 9x9 -14%, 8x8 (C5) -20% trunk time; 15x15 +8.7%.
// Flag 8 forces DENSE, flag 0x4000000 the padded geometry (A/B measurement).
template <int HB>
static void v6_launch(const ConvBf16Args& a, int mode, hipStream_t st) {
    const bool dense = (a.flags & 8) || (HB != 15 && !(a.flags & 0x4000000));
    if (dense) v6_launch_g<HB, true>(a, mode, st);
    else v6_launch_g<HB, false>(a, mode, st);
}

bool az_conv_v7_supported(const ConvBf16Args& a);
int az_conv_v7_launch(const ConvBf16Args& a, int mode, int geo15, hipStream_t st);
int az_conv_v7_tm(const ConvBf16Args& a);
int az_conv_v7_ring(const ConvBf16Args& a);

// Which kernel az_conv_g8_launch takes for a layer (a.flags already set): 0 none (unsupported),
// 1 conv3x3_v7 (*geo = its 15x15 tile geometry), 2 conv3x3_v6 (*geo = 1 when DENSE), 3 conv3x3_v5.
static int g8_choice(const ConvBf16Args& a, int* geo) {
    if (a.H != a.W || !az_conv_g8_supported(a.H, a.W, a.C, a.N)) return 0;
    // conv3x3_v7 (conv_v7.hip, two 256-thread blocks per CU, epilogue from registers) takes every
    // layer it supports (trunk convs: C % 64 == 0) unless flag 0x100 selects v6 (A/B measurement);
    // flag 0x200: v7 only on 15x15 boards; 15x15 tile geometry: SLIM (default), flag 8 DENSE, 0x400 PAD.
    // 15x15 below 1024 boards: a launch is one or two rounds of blocks and v6 is faster (B = 256: 61
    // vs 65 us); the other boards take v7's small DENSE tiles there (next branch).  Flag 0x800 forces
    // v7 at any batch.
    const int boards_g8 = a.M / (a.H * a.W);
    if (!(a.flags & 0x100) && (a.H == 15 || !(a.flags & 0x200)) && (boards_g8 >= 1024 || (a.flags & 0x800)) &&
        az_conv_v7_supported(a)) {
        *geo = (a.flags & 8) ? 2 : (a.flags & 0x400) ? 0 : 1;
        return 1;
    }
    // Small batches on the DENSE boards (the per-rank shards of the 8-GPU C4 / C5 configs): v6's
    // 512-row tiles leave most CUs idle (C5 net, 128 boards: 32 blocks), conv3x3_v7 with 128 / 64-row
    // tiles (az_conv_v7_tm) fills them -- 128 boards of 8x8: 0.0237 vs 0.0644 ms per launch; 19x19 on
    // 128-row tiles with three blocks per CU: 0.0594 vs v6 0.0747 at 128 boards, 0.1106 vs 0.1375 at
    // 256 (profiles/r04_small_batch_tiles_192.txt, r05_small_batch_ring3.txt).  Flag 0x1000 keeps v6.
    if (!(a.flags & (0x100 | 0x1000)) && a.H != 15 && boards_g8 < 1024 && az_conv_v7_supported(a)) {
        *geo = 2;
        return 1;
    }
    const size_t HW = (size_t)a.H * a.W;
    if (a.a_tail < (size_t)a.M * a.C * 2) return 0;
    // v6: the padding offset walks (C/32) chunk steps of 4*HW*16 B into the zeroed tail, and the
    // buffer descriptor's 32-bit range must cover the activations plus that tail
    const bool v6_ok = a.C % 32 == 0 && a.a_tail + AZ_ACT_TAIL * 2 < ((size_t)1 << 31) &&
                       (size_t)(a.C / 32) * 4 * HW * 16 + 16 <= AZ_ACT_TAIL * 2;
    if (a.H != 15 || ((a.flags & 4) && a.C % 32 == 0)) {
        if (!v6_ok || !a.relu) return 0;                 // conv3x3_v6 always applies the ReLU
        *geo = (a.flags & 8) || (a.H != 15 && !(a.flags & 0x4000000));
        return 2;
    }
    return 3;
}

int az_conv_g8_launch(const ConvBf16Args& a_in, int mode, hipStream_t st) {
    ConvBf16Args a = a_in;
    a.flags = g_conv_flags;
    if (a.a_tail == 0) a.a_tail = (size_t)a.M * a.C * 2;
    int geo = 0;
    switch (g8_choice(a, &geo)) {
        case 1: return az_conv_v7_launch(a, mode, geo, st);
        case 2:
            switch (a.H) {
                case 8: v6_launch<8>(a, mode, st); return 0;
                case 9: v6_launch<9>(a, mode, st); return 0;
                case 13: v6_launch<13>(a, mode, st); return 0;
                case 19: v6_launch<19>(a, mode, st); return 0;
                default: v6_launch<15>(a, mode, st); return 0;
            }
        case 3: break;
        default: return -1;
    }
    const int boards = a.M / 225;
    const int pairs = (boards + 1) / 2;
    const int nsplit = a.N / 128;
    const int grid = (pairs + 7) / 8 * 8 * nsplit;     // XCD-aware pair/half mapping needs whole groups of 8
    if (mode == 2) hipLaunchKernelGGL((conv3x3_v5<2, 8>), dim3(grid), dim3(512), 0, st, a);
    else hipLaunchKernelGGL((conv3x3_v5<1, 8>), dim3(grid), dim3(512), 0, st, a);
    return 0;
}

// The name of the kernel az_conv_g8_launch takes for this layer (bench.py's roofline label)
int az_conv_g8_name(const ConvBf16Args& a_in, int mode, char* out, int len) {
    ConvBf16Args a = a_in;
    a.flags = g_conv_flags;
    if (a.a_tail == 0) a.a_tail = (size_t)a.M * a.C * 2;
    int geo = 0;
    static const char* g7[3] = {"PAD", "SLIM", "DENSE"};
    switch (g8_choice(a, &geo)) {
        case 1: {
            const int g = a.H == 15 ? geo : 2, tm = g == 2 ? az_conv_v7_tm(a) : 256;
            const int rg = tm != 256 ? az_conv_v7_ring(a) : 4;
            if (rg != 4) snprintf(out, len, "conv3x3_v7<%d, %d, %s, %d, %d>", mode, a.H, g7[g], tm, rg);
            else if (tm != 256) snprintf(out, len, "conv3x3_v7<%d, %d, %s, %d>", mode, a.H, g7[g], tm);
            else snprintf(out, len, "conv3x3_v7<%d, %d, %s>", mode, a.H, g7[g]);
            return 0;
        }
        case 2: snprintf(out, len, "conv3x3_v6<%d, %d%s>", mode, a.H, geo ? ", DENSE" : ""); return 0;
        case 3: snprintf(out, len, "conv3x3_v5<%d, 8>", mode); return 0;
        default: return -1;
    }
}

// fp32 -> fp16 activations (first trunk input, AZ_PREC_FP16)
__global__ void k_to_f16(const float* in, uint16_t* out, size_t n, const int* m_limit, int rows_per_sample, int C,
                         int* ovf) {
    size_t lim = n;
    if (m_limit) lim = min(n, (size_t)(*m_limit) * rows_per_sample * C);
    float vmax = 0.0f;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < lim; i += (size_t)gridDim.x * blockDim.x) {
        const float v = in[i];
        vmax = __builtin_fmaxf(vmax, __builtin_fabsf(v));
        out[i] = v4_store<2>(v);
    }
    if (!(vmax <= 65504.0f) && ovf) atomicOr(ovf, 1);                // fp16 overflow: the engine fails the forward
}
void az_launch_to_f16(const float* in, uint16_t* out, size_t n, const int* m_limit, int rows_per_sample, int C,
                      hipStream_t st, int* ovf) {
    hipLaunchKernelGGL(k_to_f16, dim3(2048), dim3(256), 0, st, in, out, n, m_limit, rows_per_sample, C, ovf);
}

// true when conv3x3_v4 handles this shape
bool az_conv_v4_supported(int H, int W, int C, int N) { return H == 15 && W == 15 && C % 16 == 0 && N % 64 == 0; }

template <int BNT>
static void v4_launch(const ConvBf16Args& a, int mode, int grid, hipStream_t st) {
    // bf16x3 keeps the single-buffered schedule: the double buffer spills at 256 VGPRs
    if (mode == 0) hipLaunchKernelGGL((conv3x3_v4<0, BNT, 0>), dim3(grid), dim3(512), 0, st, a);
    else if (mode == 1) hipLaunchKernelGGL((conv3x3_v4<1, BNT, 1>), dim3(grid), dim3(512), 0, st, a);
    else hipLaunchKernelGGL((conv3x3_v4<2, BNT, 1>), dim3(grid), dim3(512), 0, st, a);
}

void az_conv_v4_launch(const ConvBf16Args& a, int mode, hipStream_t st) {
    const int boards = a.M / 225;
    const int bnt = a.N % 128 == 0 ? 128 : 64;
    if (mode == 0 && bnt == 64 && boards <= 512) {   // one board per block: fill the CUs at small batches
        hipLaunchKernelGGL((conv3x3_v4<0, 64, 1, 1, 512>), dim3(boards * (a.N / 64)), dim3(512), 0, st, a);
        return;
    }
    const int grid = (boards + 1) / 2 * (a.N / bnt);
    if (bnt == 128) v4_launch<128>(a, mode, grid, st);
    else v4_launch<64>(a, mode, grid, st);
}

// bf16 / bf16x3 trunk conv outside the g8 path: v4 on 15x15 boards, else v3 (N % 256 == 0 or
// N == 64, C % 32 == 0), else v1 (128 x 128 register-staged tiles, any shape)
static int bf16_choice(const ConvBf16Args& a) {
    if (a.rows_per_sample == 225 && az_conv_v4_supported(a.H, a.W, a.C, a.N)) return 4;
    if (a.C % 32 == 0 && (a.N % 256 == 0 || a.N == 64)) return 3;
    return 1;
}

void az_conv_bf16_launch_v(const ConvBf16Args& a, bool split, hipStream_t st) {
    switch (bf16_choice(a)) {
        case 4: az_conv_v4_launch(a, split ? 0 : 1, st); return;
        case 3:
            if (a.N % 256 == 0) {
                const int nbm = (a.M + 127) / 128, nbn = a.N / 256;
                if (split) hipLaunchKernelGGL((conv3x3_v3<true, 128, 256, 2, 4>), dim3(nbm * nbn), dim3(512), 0, st, a);
                else hipLaunchKernelGGL((conv3x3_v3<false, 128, 256, 2, 4>), dim3(nbm * nbn), dim3(512), 0, st, a);
            } else {
                const int nbm = (a.M + 255) / 256;
                if (split) hipLaunchKernelGGL((conv3x3_v3<true, 256, 64, 4, 1>), dim3(nbm), dim3(256), 0, st, a);
                else hipLaunchKernelGGL((conv3x3_v3<false, 256, 64, 4, 1>), dim3(nbm), dim3(256), 0, st, a);
            }
            return;
        default: az_conv_bf16_launch(a, split, st); return;
    }
}

// The name of the kernel az_conv_bf16_launch_v (mode 0 bf16x3 / 1 bf16) or, for fp16 (mode 2),
// az_conv_v4_launch takes for this layer
int az_conv_bf16_name(const ConvBf16Args& a, int mode, char* out, int len) {
    const int c = mode == 2 ? 4 : bf16_choice(a);
    const bool split = mode == 0;
    if (c == 4) snprintf(out, len, "conv3x3_v4<%d, %d>", mode, a.N % 128 == 0 ? 128 : 64);
    else if (c == 3) snprintf(out, len, a.N % 256 == 0 ? "conv3x3_v3<%s, 128, 256>" : "conv3x3_v3<%s, 256, 64>",
                              split ? "split" : "bf16");
    else snprintf(out, len, "conv3x3_bf16<%s>", split ? "split" : "bf16");
    return 0;
}
