// net_kernels.hip -- ConvNet forward for the leaf batch (gfx950).
//
// Every layer of the policy/value net is one implicit
// GEMM  out[m][n] = act( sum_k A(m,k) * Wt[n][k] + bias[n] (+ res[m][n]) )
//   3x3 conv : m = pixel (b, y, x) of an NHWC activation, k = (tap, c), A gathered
//              from the 3x3 neighbourhood (zero padding), BN folded into Wt/bias
//   1x1 conv : taps = 1 over pooled pixels;  FC : taps = 1 over samples.
// Kernels here:
//   gemm_f32   f32-input MFMA (v_mfma_f32_32x32x2_f32): exact f32 products, the
//              AZ_PREC_F32 path and the head layers of every precision.
//   (bf16 MFMA trunk kernels live in conv_bf16.hip.)
#include <hip/hip_runtime.h>
#include <algorithm>
#include <type_traits>
#include <stdint.h>
#include "net.h"
#include "leaf_planes.h"

typedef float floatx16 __attribute__((ext_vector_type(16)));

namespace {

template <int ACT>
__device__ __forceinline__ float activate(float v) {
    if (ACT == ACT_RELU) return v > 0.0f ? v : 0.0f;
    if (ACT == ACT_TANH) return tanhf(v);
    return v;
}

}  // namespace

// Block tile BM x BN (BM = 128), BK = 32, 256 threads = 2x2 waves, wave tile
// (BM/2) x (BN/2) of 32x32 MFMA tiles.  LDS holds A and B transposed ([k][m] with
// row stride BM+1 / BN+1, conflict-free for the transposed writes and for the
// MFMA operand reads), double buffered; global loads are register staged.
template <int BN, int ACT, bool RES>
__global__ __launch_bounds__(256) void gemm_f32(GemmArgs p) {
    constexpr int BM = 128, BK = 32;
    constexpr int LDA = BM + 1, LDB = BN + 1;
    constexpr int TM = BM / 2, TN = BN / 2;
    constexpr int MT = TM / 32, NT = TN / 32;
    constexpr int BROWS = BN / 32;   // B rows loaded per thread (BN*8 float4 / 256 threads)
    __shared__ float As[2][BK * LDA];
    __shared__ float Bs[2][BK * LDB];

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int nbm = (p.M + BM - 1) / BM;
    const int bid = blockIdx.x;
    const int bm = bid % nbm, bn = bid / nbm;
    const int m0 = bm * BM, n0 = bn * BN;
    // device-side leaf batch: rows beyond n_eval * rows_per_sample are skipped
    const int Mact = p.m_limit ? min(p.M, *p.m_limit * p.rows_per_sample) : p.M;
    if (m0 >= Mact) return;

    // Per-thread A rows: m = tid/8 + 32*i, float4 column kq = tid%8.
    const int kq = tid & 7;
    const int r0 = tid >> 3;
    int arow_b[4], arow_y[4], arow_x[4];
    bool arow_ok[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int m = m0 + r0 + 32 * i;
        arow_ok[i] = m < Mact;
        const int pix = p.H * p.W;
        const int b = m / pix, r = m % pix;
        arow_b[i] = b; arow_y[i] = r / p.W; arow_x[i] = r % p.W;
    }
    const int K = p.K;           // taps * C
    const int nk_all = (p.Kpad + BK - 1) / BK;
    // split-K (FC layers at small M): this block accumulates k-tiles [kt0, kt0 + nk)
    const int kper = p.part ? (nk_all + p.splits - 1) / p.splits : nk_all;
    const int kt0 = p.part ? blockIdx.y * kper : 0;
    const int nk = max(0, min(nk_all - kt0, kper));

    float4 ra[4], rb[BROWS];
    auto load_stage = [&](int kt) {
        const int k = kt * BK + kq * 4;
        int tap = 0, c = k;
        if (p.taps == 9) { tap = k / p.Cch; c = k - tap * p.Cch; }
        const int dy = tap / 3 - 1, dx = tap % 3 - 1;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (arow_ok[i] && k < K) {
                const float* src = nullptr;
                if (p.taps == 9) {
                    const int y = arow_y[i] + dy, x = arow_x[i] + dx;
                    if (y >= 0 && y < p.H && x >= 0 && x < p.W)
                        src = p.A + ((size_t)(arow_b[i] * p.H + y) * p.W + x) * p.lda + c;
                } else if (p.Am) {
                    const int j = k / p.Cch;
                    src = p.Am[j] + (size_t)(m0 + r0 + 32 * i) * p.lda + (k - j * p.Cch);
                } else {
                    src = p.A + (size_t)(m0 + r0 + 32 * i) * p.lda + c;
                }
                if (src) v = *reinterpret_cast<const float4*>(src);
            }
            ra[i] = v;
        }
#pragma unroll
        for (int i = 0; i < BROWS; ++i) {
            const int n = n0 + r0 + 32 * i;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (n < p.N && k < K) v = *reinterpret_cast<const float4*>(p.B + (size_t)n * p.ldb + k);
            rb[i] = v;
        }
    };
    auto store_stage = [&](int buf) {
        float* as = As[buf];
        float* bs = Bs[buf];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int m = r0 + 32 * i;
            as[(kq * 4 + 0) * LDA + m] = ra[i].x;
            as[(kq * 4 + 1) * LDA + m] = ra[i].y;
            as[(kq * 4 + 2) * LDA + m] = ra[i].z;
            as[(kq * 4 + 3) * LDA + m] = ra[i].w;
        }
#pragma unroll
        for (int i = 0; i < BROWS; ++i) {
            const int n = r0 + 32 * i;
            bs[(kq * 4 + 0) * LDB + n] = rb[i].x;
            bs[(kq * 4 + 1) * LDB + n] = rb[i].y;
            bs[(kq * 4 + 2) * LDB + n] = rb[i].z;
            bs[(kq * 4 + 3) * LDB + n] = rb[i].w;
        }
    };

    floatx16 acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

    if (nk > 0) load_stage(kt0);
    store_stage(0);
    __syncthreads();
    const int kh = lane >> 5, l32 = lane & 31;
    for (int kt = 0; kt < nk; ++kt) {
        const int buf = kt & 1;
        if (kt + 1 < nk) load_stage(kt0 + kt + 1);
        const float* as = As[buf];
        const float* bs = Bs[buf];
#pragma unroll 4
        for (int kk = 0; kk < BK / 2; ++kk) {
            float a[MT], b[NT];
#pragma unroll
            for (int i = 0; i < MT; ++i) a[i] = as[(kk * 2 + kh) * LDA + wm * TM + i * 32 + l32];
#pragma unroll
            for (int j = 0; j < NT; ++j) b[j] = bs[(kk * 2 + kh) * LDB + wn * TN + j * 32 + l32];
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int j = 0; j < NT; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
        }
        if (kt + 1 < nk) {
            store_stage(buf ^ 1);
        }
        __syncthreads();
    }

    // Epilogue: C/D map col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5).
    if (p.part) {                // raw partial sums; k_splitk_reduce adds bias + activation
        float* part = p.part + (size_t)blockIdx.y * p.M * p.N;
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int j = 0; j < NT; ++j) {
                const int n = n0 + wn * TN + j * 32 + l32;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int m = m0 + wm * TM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * kh;
                    if (n < p.N && m < Mact) part[(size_t)m * p.N + n] = acc[i][j][r];
                }
            }
        return;
    }
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) {
            const int n = n0 + wn * TN + j * 32 + l32;
            const bool nok = n < p.N;
            const float bias = (nok && p.bias) ? p.bias[n] : 0.0f;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + wm * TM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * kh;
                if (nok && m < Mact) {
                    float v = acc[i][j][r] + bias;
                    if (RES) v += p.res[(size_t)m * p.ldc + n];
                    p.C[(size_t)m * p.ldc + n] = activate<ACT>(v);
                }
            }
        }
}

// 1x1-conv GEMM with fp16 operands and fp32 accumulation (v_mfma_f32_32x32x16_f16): the routers of
// an AZ_PREC_FP16 rand-wire net.  out[m][n] = relu(sum_k A(m,k) W[n][k] + bias[n]), taps == 1,
// A from p.Am slices (or p.A), fp32 in memory and rounded to fp16 on the way into LDS, W fp32
// [N][ldb] likewise.  Tile 128 x 128, BK = 32, 2 x 2 waves of 64 x 64 (2 x 2 MFMA tiles); LDS rows
// [m][k] / [n][k] of 32 halves + 8 pad (80 B), each lane's operand (8 consecutive k: A[r][8h + j])
// one ds_read_b128.
typedef _Float16 half4_t __attribute__((ext_vector_type(4)));
typedef _Float16 half8_t __attribute__((ext_vector_type(8)));
__global__ __launch_bounds__(256) void gemm_h16_relu(GemmArgs p) {
    constexpr int BM = 128, BN = 128, BK = 32, LD = BK + 8;
    __shared__ __attribute__((aligned(16))) _Float16 As[2][BM * LD];
    __shared__ __attribute__((aligned(16))) _Float16 Bs[2][BN * LD];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int nbm = (p.M + BM - 1) / BM;
    const int bm = blockIdx.x % nbm, bn = blockIdx.x / nbm;
    const int m0 = bm * BM, n0 = bn * BN;
    const int Mact = p.m_limit ? min(p.M, *p.m_limit * p.rows_per_sample) : p.M;
    if (m0 >= Mact) return;
    const int kq = tid & 7, r0 = tid >> 3;     // float4 column kq of rows r0 + 32 i
    const int nk = (p.Kpad + BK - 1) / BK;
    float4 ra[4], rb[4];
    auto load_stage = [&](int kt) {
        const int k = kt * BK + kq * 4;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int m = m0 + r0 + 32 * i;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (m < Mact && k < p.K) {
                const float* src;
                if (p.Am) { const int j = k / p.Cch; src = p.Am[j] + (size_t)m * p.lda + (k - j * p.Cch); }
                else src = p.A + (size_t)m * p.lda + k;
                v = *reinterpret_cast<const float4*>(src);
            }
            ra[i] = v;
            const int n = n0 + r0 + 32 * i;
            float4 w = make_float4(0.f, 0.f, 0.f, 0.f);
            if (n < p.N && k < p.K) w = *reinterpret_cast<const float4*>(p.B + (size_t)n * p.ldb + k);
            rb[i] = w;
        }
    };
    auto store_stage = [&](int buf) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int r = r0 + 32 * i;
            half4_t a = {(_Float16)ra[i].x, (_Float16)ra[i].y, (_Float16)ra[i].z, (_Float16)ra[i].w};
            half4_t b = {(_Float16)rb[i].x, (_Float16)rb[i].y, (_Float16)rb[i].z, (_Float16)rb[i].w};
            *reinterpret_cast<half4_t*>(&As[buf][r * LD + kq * 4]) = a;
            *reinterpret_cast<half4_t*>(&Bs[buf][r * LD + kq * 4]) = b;
        }
    };
    floatx16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
    load_stage(0);
    store_stage(0);
    __syncthreads();
    const int kh = lane >> 5, l32 = lane & 31;
    for (int kt = 0; kt < nk; ++kt) {
        const int buf = kt & 1;
        if (kt + 1 < nk) load_stage(kt + 1);
        const _Float16* as = As[buf];
        const _Float16* bs = Bs[buf];
#pragma unroll
        for (int kk = 0; kk < BK / 16; ++kk) {
            half8_t a[2], b[2];
#pragma unroll
            for (int i = 0; i < 2; ++i)
                a[i] = *reinterpret_cast<const half8_t*>(&as[(wm * 64 + i * 32 + l32) * LD + kk * 16 + kh * 8]);
#pragma unroll
            for (int j = 0; j < 2; ++j)
                b[j] = *reinterpret_cast<const half8_t*>(&bs[(wn * 64 + j * 32 + l32) * LD + kk * 16 + kh * 8]);
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[i], b[j], acc[i][j], 0, 0, 0);
        }
        if (kt + 1 < nk) store_stage(buf ^ 1);
        __syncthreads();
    }
    // C/D map: col = lane & 31 (n), row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5) (m)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int n = n0 + wn * 64 + j * 32 + l32;
            if (n >= p.N) continue;
            const float bias = p.bias ? p.bias[n] : 0.0f;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * kh;
                if (m < Mact) p.C[(size_t)m * p.ldc + n] = fmaxf(acc[i][j][r] + bias, 0.0f);
            }
        }
}

void az_launch_gemm_h16_relu(const GemmArgs& p, hipStream_t st) {
    const int nbm = (p.M + 127) / 128, nbn = (p.N + 127) / 128;
    hipLaunchKernelGGL(gemm_h16_relu, dim3(nbm * nbn), dim3(256), 0, st, p);
}

// Squeeze-and-excitation + residual + ReLU of a DDW-RandWire node (row f4;
// ddw_randwire_resnet.cpp:10-32 SEBlock, :53-61 ResidualBlock::forward):
//   s = sigmoid(W2 relu(W1 mean_hw(y) + b1) + b2),  out = relu(y * s + x)
// One 256-thread block per board: the per-channel means, the two tiny FCs and the gates stay
// in LDS; y and x are read once more for the scaled residual (both L2-resident right after the
// producing conv).  C <= 1024, R = C / 16.  gridDim.y blocks share a board at small batches: each
// computes the (identical) gates and scales its own slice of the board.
__global__ __launch_bounds__(256) void k_se_residual(const float* y, const float* x, float* out, const float* W1,
                                                     const float* b1, const float* W2, const float* b2, int HW, int C,
                                                     int R, const int* m_limit) {
    __shared__ float mean[1024], hid[64], gate[1024];
    const int b = blockIdx.x;
    if (m_limit && b >= *m_limit) return;
    __shared__ float4 part[256];
    const size_t base = (size_t)b * HW * C;
    const float inv = 1.0f / (float)HW;
    {   // channel quads over 256 / (C/4) pixel groups, then the groups summed in order per channel
        const int C4 = C / 4, G = 256 / C4, t = threadIdx.x;
        const int q = t % C4, g = t / C4;
        float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
        if (g < G) {
            const float4* y4 = reinterpret_cast<const float4*>(y + base) + q;
            for (int p = g; p < HW; p += G) {
                const float4 v = y4[(size_t)p * C4];
                s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
            }
        }
        part[t] = s;
        __syncthreads();
        for (int c = t; c < C; c += 256) {
            const float* pf = reinterpret_cast<const float*>(part);
            float a = 0.0f;
            for (int k = 0; k < G; ++k) a += pf[(k * C4 + c / 4) * 4 + c % 4];
            mean[c] = a * inv;
        }
    }
    __syncthreads();
    for (int r = threadIdx.x; r < R; r += 256) {
        float s = b1[r];
        for (int c = 0; c < C; ++c) s += W1[(size_t)r * C + c] * mean[c];
        hid[r] = s > 0.0f ? s : 0.0f;
    }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += 256) {
        float s = b2[c];
        for (int r = 0; r < R; ++r) s += W2[(size_t)c * R + r] * hid[r];
        gate[c] = 1.0f / (1.0f + expf(-s));
    }
    __syncthreads();
    const int n4 = HW * C / 4;   // C % 16 == 0: float4 items never straddle a pixel
    const float4* y4 = reinterpret_cast<const float4*>(y + base);
    const float4* x4 = reinterpret_cast<const float4*>(x + base);
    float4* o4 = reinterpret_cast<float4*>(out + base);
    for (int i = blockIdx.y * 256 + threadIdx.x; i < n4; i += 256 * gridDim.y) {
        const int c = (i * 4) % C;
        const float4 a = y4[i], r = x4[i];
        float4 o;
        o.x = fmaxf(a.x * gate[c] + r.x, 0.0f);
        o.y = fmaxf(a.y * gate[c + 1] + r.y, 0.0f);
        o.z = fmaxf(a.z * gate[c + 2] + r.z, 0.0f);
        o.w = fmaxf(a.w * gate[c + 3] + r.w, 0.0f);
        o4[i] = o;
    }
}

// adaptive_avg_pool2d(x, (P, P)) on NHWC: out[b][oy][ox][c]
__global__ void k_adaptive_pool(const float* in, float* out, int B, int H, int W, int C, int P, const int* m_limit) {
    const int idx = blockIdx.x;           // b * P*P + oy*P + ox
    const int b = idx / (P * P);
    if (m_limit && b >= *m_limit) return;
    const int o = idx % (P * P);
    const int oy = o / P, ox = o % P;
    const int y0 = (oy * H) / P, y1 = ((oy + 1) * H + P - 1) / P;
    const int x0 = (ox * W) / P, x1 = ((ox + 1) * W + P - 1) / P;
    const float kh = (float)(y1 - y0), kw = (float)(x1 - x0);
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
        float s = 0.0f;
        for (int y = y0; y < y1; ++y)
            for (int x = x0; x < x1; ++x) s += in[((size_t)(b * H + y) * W + x) * C + c];
        out[(size_t)idx * C + c] = s / kh / kw;
    }
}

// NCHW planes [B][Cin][H*W] -> NHWC [B][H*W][Cp] (zero-padded channels)
__global__ void k_pack_input(const float* in, float* out, int B, int Cin, int HW, int Cp) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t total = (size_t)B * HW * Cp;
    if (i >= total) return;
    const int c = (int)(i % Cp);
    const size_t bp = i / Cp;
    const int px = (int)(bp % HW);
    const int b = (int)(bp / HW);
    out[i] = c < Cin ? in[((size_t)b * Cin + c) * HW + px] : 0.0f;
}

// The planes of the leaves that need the network as a dense fp32 NHWC16 batch built from their
// leaf records (leaf_planes.h): dst[s] = planes(rec[eval_games[s]]) (f32 input path, host evaluator).
__global__ void k_rec_planes(const uint8_t* rec, float* dst, const int* eval_games, const int* n_eval, int go, int bs) {
    const int s = blockIdx.y;
    if (s >= *n_eval) return;
    const uint8_t* r = rec + (size_t)eval_games[s] * AZ_REC_BYTES;
    const int A = bs * bs;
    float4* out = reinterpret_cast<float4*>(dst + (size_t)s * A * 16);
    for (int a = blockIdx.x * blockDim.x + threadIdx.x; a < A; a += gridDim.x * blockDim.x) {
        float c[16];
        az_leaf_planes(r, go, bs, a, c);
#pragma unroll
        for (int k = 0; k < 4; ++k) out[(size_t)a * 4 + k] = make_float4(c[4 * k], c[4 * k + 1], c[4 * k + 2], c[4 * k + 3]);
    }
}

void az_launch_rec_planes(const uint8_t* rec, float* dst, const int* eval_games, const int* n_eval, int go, int bs, int maxB,
                          hipStream_t st) {
    hipLaunchKernelGGL(k_rec_planes, dim3(2, maxB), dim3(256), 0, st, rec, dst, eval_games, n_eval, go, bs);
}

// softmax over A per row (predictBatch semantics; host-facing az_net_predict_batch)
__global__ void k_softmax_rows(const float* logits, float* out, int A) {
    const int b = blockIdx.x;
    __shared__ float e[1024];
    __shared__ float s_sum, s_max;
    if (threadIdx.x == 0) {
        float mx = -3.402823466e38f;
        for (int a = 0; a < A; ++a) mx = fmaxf(mx, logits[(size_t)b * A + a]);
        s_max = mx;
    }
    __syncthreads();
    for (int a = threadIdx.x; a < A; a += blockDim.x) e[a] = expf(logits[(size_t)b * A + a] - s_max);
    __syncthreads();
    if (threadIdx.x == 0) {
        float s = 0.0f;
        for (int a = 0; a < A; ++a) s += e[a];
        s_sum = s;
    }
    __syncthreads();
    for (int a = threadIdx.x; a < A; a += blockDim.x) out[(size_t)b * A + a] = s_sum > 0.0f ? e[a] / s_sum : e[a];
}

// split-K reduction: C = act(sum_s part[s] + bias), slices summed in order (deterministic)
template <int ACT>
__global__ void k_splitk_reduce(GemmArgs p) {
    const int Mact = p.m_limit ? min(p.M, *p.m_limit * p.rows_per_sample) : p.M;
    const size_t total = (size_t)Mact * p.N;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const int m = (int)(i / p.N), n = (int)(i % p.N);
        float v = 0.0f;
        for (int s = 0; s < p.splits; ++s) v += p.part[((size_t)s * p.M + m) * p.N + n];
        if (p.bias) v += p.bias[n];
        p.C[(size_t)m * p.ldc + n] = activate<ACT>(v);
    }
}

// ---------------------------------------------------------------------------
template <int BN, int ACT, bool RES>
static void launch_f32(const GemmArgs& p, hipStream_t st) {
    const int nbm = (p.M + 127) / 128, nbn = (p.N + BN - 1) / BN;
    if (p.part && !RES) {
        hipLaunchKernelGGL((gemm_f32<BN, ACT, RES>), dim3(nbm * nbn, p.splits), dim3(256), 0, st, p);
        hipLaunchKernelGGL(k_splitk_reduce<ACT>, dim3(1024), dim3(256), 0, st, p);
        return;
    }
    GemmArgs q = p;
    q.part = nullptr;
    hipLaunchKernelGGL((gemm_f32<BN, ACT, RES>), dim3(nbm * nbn), dim3(256), 0, st, q);
}

// ---------------------------------------------------------------------------
// Both FC heads in two launches: k_fc_heads computes the split-K partials of the policy FC
// (K -> A logits) and the value FC1 (K -> H hidden) as one GEMM over 64-column tiles of
// [policy | value] (f32 MFMA v_mfma_f32_16x16x4_f32: every partial a k-ordered fmaf chain, as
// gemm_f32); k_fc_finish (one 256-thread block per board) sums the slices in order and finishes both heads
// (bias, ReLU, value FC2, tanh).  Deterministic and batch-position independent.
typedef float f32x4n __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_fc_heads(FcHeadArgs p) {
    constexpr int BK = 32;
    __shared__ float As[BK][64 + 1];                   // [k][board]
    __shared__ float Bs[BK][64 + 1];                   // [k][output]
    const int NTP = (p.A + 63) / 64, NTV = (p.H + 63) / 64, NT = NTP + NTV;
    const int mt = blockIdx.x / NT, nt = blockIdx.x - mt * NT, sl = blockIdx.y, S = gridDim.y;
    const int mlim = p.m_limit ? min(p.B, *p.m_limit) : p.B;
    const int m0 = mt * 64;
    if (m0 >= mlim) return;                            // the whole row of tiles is idle (no counter touched)
    const bool pol = nt < NTP;
    const int n0 = pol ? nt * 64 : (nt - NTP) * 64;    // first output of the tile within its head
    const int NO = pol ? p.A : p.H;
    const float* X = pol ? p.pp : p.vp;                // [B][K]
    const float* Wt = pol ? p.Wp : p.Wv1;              // [NO][K]
    const int KS = p.K / S, k0 = sl * KS;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l16 = lane & 15, lg = lane >> 4;
    // staging: thread -> (row r = tid / 4 (+ 64 * second half), float4 column c4 = tid % 4 (+4)) of a 64 x 32 chunk
    f32x4n ra[2], rb[2];
    auto fetch = [&](int kc) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int r = tid >> 2, c4 = (tid & 3) + 4 * h, k = kc + 4 * c4;
            const int m = m0 + r, n = n0 + r;
            // element k of board m's head map: cell k / hc, channel k % hc (cell stride xs)
            const size_t xo = ((size_t)m * (p.K / p.hc) + k / p.hc) * p.xs + k % p.hc;
            ra[h] = m < mlim ? *reinterpret_cast<const f32x4n*>(X + xo) : f32x4n{0.f, 0.f, 0.f, 0.f};
            rb[h] = n < NO ? *reinterpret_cast<const f32x4n*>(Wt + (size_t)n * p.K + k) : f32x4n{0.f, 0.f, 0.f, 0.f};
        }
    };
    auto stash = [&]() {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int r = tid >> 2, c4 = (tid & 3) + 4 * h;
#pragma unroll
            for (int e = 0; e < 4; ++e) { As[4 * c4 + e][r] = ra[h][e]; Bs[4 * c4 + e][r] = rb[h][e]; }
        }
    };
    f32x4n acc[4] = {};
    fetch(k0);
    for (int kc = k0; kc < k0 + KS; kc += BK) {
        __syncthreads();
        stash();
        __syncthreads();
        if (kc + BK < k0 + KS) fetch(kc + BK);
#pragma unroll
        for (int kk = 0; kk < BK / 4; ++kk) {
            const float a = As[4 * kk + lg][16 * wave + l16];
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, Bs[4 * kk + lg][16 * j + l16], acc[j], 0, 0, 0);
        }
    }
    // partial tile: D[board 16 wave + 4 lg + e][output 16 j + l16]
    const int NC = NT * 64, BP = (p.B + 63) / 64 * 64;
    float* part = p.part + (size_t)sl * BP * NC;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) part[(size_t)(m0 + 16 * wave + 4 * lg + e) * NC + nt * 64 + 16 * j + l16] = acc[j][e];
}

// k_fc_heads_x3: the same split-K partials as k_fc_heads in the fp32-faithful bf16x3 arithmetic
// (the FP16 / BF16 / BF16X3 precisions): weights pre-split into bf16 hi / lo rows ([NC][K], policy
// rows padded to 64, then the value rows; p.Wx_hi / p.Wx_lo), activations split on the fly, every
// product hi*hi + lo*hi + hi*lo on v_mfma_f32_16x16x32_bf16 with fp32 accumulation -- 16 x the f32
// MFMA's FLOP per cycle, three MFMAs per product.  256 threads = 4 waves of 32 boards x 32 outputs
// of a 64 x 64 tile; operands go straight from global memory (L2) into registers, one K step of 32
// ahead.  Writes k_fc_finish's partial layout.
typedef __bf16 bf16x8n __attribute__((ext_vector_type(8)));
__device__ __forceinline__ uint32_t fc_bf16_rne(float f) {
    uint32_t u = __float_as_uint(f);
    u += 0x7fffu + ((u >> 16) & 1u);
    return u >> 16;
}
// PT 2 (AZ_PREC_F16X3): fp16 pieces -- the rows pre-scaled by 2^s (k_fc_finish applies p.rs = 2^-s),
// the features split in fp16 with the range guard (p.ovf); v_mfma_f32_16x16x32_f16, same shape.
typedef _Float16 f16x8n __attribute__((ext_vector_type(8)));
template <int PT>
__global__ __launch_bounds__(256) void k_fc_heads_x3(FcHeadArgs p) {
    typedef typename std::conditional<PT == 2, f16x8n, bf16x8n>::type frag;
    const int NTP = (p.A + 63) / 64, NTV = (p.H + 63) / 64, NT = NTP + NTV;
    const int mt = blockIdx.x / NT, nt = blockIdx.x - mt * NT, sl = blockIdx.y, S = gridDim.y;
    const int mlim = p.m_limit ? min(p.B, *p.m_limit) : p.B;
    const int m0 = mt * 64;
    if (m0 >= mlim) return;
    const bool pol = nt < NTP;
    const float* X = pol ? p.pp : p.vp;                // [B][K] (cell stride xs)
    const int K = p.K, KS = K / S, k0 = sl * KS;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave >> 1, wn = wave & 1;
    const int l16 = lane & 15, lg = lane >> 4;
    // weight rows of the lane: output 16 j + l16 of the wave's 32 (rows of the padded [NC][K] matrices)
    const uint16_t* wh[2];
    const uint16_t* wl[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const size_t row = (size_t)nt * 64 + wn * 32 + 16 * j + l16;
        wh[j] = p.Wx_hi + row * K + 8 * lg;
        wl[j] = p.Wx_lo + row * K + 8 * lg;
    }
    // activation rows of the lane: board 16 i + l16 of the wave's 32 (zero past the batch)
    const float* xr[2];
    bool live[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int m = m0 + wm * 32 + 16 * i + l16;
        live[i] = m < mlim;
        xr[i] = X + (size_t)(live[i] ? m : 0) * (K / p.hc) * p.xs;
    }
    // element k of a board's head map: cell k / hc, channel k % hc (cell stride xs); a lane's 8
    // consecutive k never straddle a cell (hc % 8 == 0)
    const int gap = p.xs - p.hc;
    auto xoff = [&](int k) { return (size_t)k + (size_t)(k / p.hc) * gap; };
    typedef float f32x8n __attribute__((ext_vector_type(8)));
    struct Ops { frag wh[2], wl[2]; f32x8n x[2]; };
    auto fetch = [&](Ops& o, int k) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            o.wh[j] = *reinterpret_cast<const frag*>(wh[j] + k);
            o.wl[j] = *reinterpret_cast<const frag*>(wl[j] + k);
        }
        const size_t xo = xoff(k + 8 * lg);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const float4 u = *reinterpret_cast<const float4*>(xr[i] + xo), v = *reinterpret_cast<const float4*>(xr[i] + xo + 4);
            o.x[i] = live[i] ? f32x8n{u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w} : f32x8n{};
        }
    };
    f32x4n acc[2][2] = {};
    float vmax = 0.0f;
    auto mma = [](const frag& w, const frag& x, const f32x4n& c) {
        if constexpr (PT == 2) return __builtin_amdgcn_mfma_f32_16x16x32_f16(w, x, c, 0, 0, 0);
        else return __builtin_amdgcn_mfma_f32_16x16x32_bf16(w, x, c, 0, 0, 0);
    };
    auto step = [&](const Ops& o) {
        frag xh[2], xl[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            if constexpr (PT == 2) {
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const float a = o.x[i][e];
                    vmax = fmaxf(vmax, fabsf(a));
                    xh[i][e] = (_Float16)a;
                    xl[i][e] = (_Float16)(a - (float)xh[i][e]);
                }
            } else {
                uint32_t h[4], l[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float a0 = o.x[i][2 * e], a1 = o.x[i][2 * e + 1];
                    const uint32_t b0 = fc_bf16_rne(a0), b1 = fc_bf16_rne(a1);
                    h[e] = b0 | (b1 << 16);
                    l[e] = fc_bf16_rne(a0 - __uint_as_float(b0 << 16)) | (fc_bf16_rne(a1 - __uint_as_float(b1 << 16)) << 16);
                }
                __builtin_memcpy(&xh[i], h, 16);
                __builtin_memcpy(&xl[i], l, 16);
            }
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[i][j] = mma(o.wh[j], xh[i], acc[i][j]);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[i][j] = mma(o.wl[j], xh[i], acc[i][j]);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[i][j] = mma(o.wh[j], xl[i], acc[i][j]);
    };
    // K steps of 32 in pairs (register double buffer with compile-time roles); KS / 32 is even
    // except for KS = 32 (handled by the tail)
    Ops A, B;
    fetch(A, k0);
    const int steps = KS / 32;
    int st = 0;
    for (; st + 2 <= steps; st += 2) {
        fetch(B, k0 + 32 * (st + 1));
        step(A);
        if (st + 2 < steps) fetch(A, k0 + 32 * (st + 2));
        step(B);
    }
    if (st < steps) step(A);
    if (PT == 2 && !(vmax <= 65504.0f) && p.ovf) atomicOr(p.ovf, 1);
    // acc[i][j][e] = partial of board 16 i + l16, output 16 j + 4 lg + e (of the wave's 32 x 32)
    const int NC = NT * 64, BP = (p.B + 63) / 64 * 64;
    float* part = p.part + (size_t)sl * BP * NC;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
            *reinterpret_cast<f32x4n*>(part + (size_t)(m0 + wm * 32 + 16 * i + l16) * NC + nt * 64 + wn * 32 + 16 * j + 4 * lg) = acc[i][j];
}

// Finish both heads, one 256-thread block per board: K slices summed in slice order (loads
// unrolled), biases, the value hidden layer (ReLU) and value = tanh(hid . w2 + b2), the dot product
// reduced by a fixed xor butterfly per wave and the four wave sums added in wave order
// (deterministic).  (Round 4 tried one wave per board, four boards per block: a quarter of the
// blocks, 11.0 vs 5.2 us at C2.)
__global__ __launch_bounds__(256) void k_fc_finish(FcHeadArgs p) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, tid = threadIdx.x;
    const int b = blockIdx.x;
    const int mlim = p.m_limit ? min(p.B, *p.m_limit) : p.B;
    if (b >= mlim) return;                             // block-uniform
    __shared__ float wsum[4];
    const int NTP = (p.A + 63) / 64, NTV = (p.H + 63) / 64, NC = (NTP + NTV) * 64, BP = (p.B + 63) / 64 * 64, S = p.S;
    const float* row = p.part + (size_t)b * NC;
    const size_t sstride = (size_t)BP * NC;
    auto sum = [&](int col) {
        float v[16];
#pragma unroll
        for (int s = 0; s < 16; ++s) v[s] = s < S ? row[s * sstride + col] : 0.0f;
        float t = 0.0f;
#pragma unroll
        for (int s = 0; s < 16; ++s) if (s < S) t += v[s];
        return t;
    };
    // k_fc_heads_x3<2>: the rows' 2^s scale undone (exact) before the bias
    auto scl = [&](int col) { return p.rs ? p.rs[col] : 1.0f; };
    for (int n = tid; n < p.A; n += 256) p.logits[(size_t)b * p.A + n] = sum(n) * scl(n) + p.bp[n];
    float d = 0.0f;
    for (int h = tid; h < p.H; h += 256) {
        float v = sum(NTP * 64 + h) * scl(NTP * 64 + h) + p.bv1[h];
        v = v > 0.0f ? v : 0.0f;
        p.hid[(size_t)b * p.H + h] = v;
        d = __builtin_fmaf(v, p.wv2[h], d);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) d += __shfl_xor(d, off);
    if (lane == 0) wsum[wave] = d;
    __syncthreads();
    if (tid == 0) p.value[b] = tanhf(((wsum[0] + wsum[1]) + (wsum[2] + wsum[3])) + p.bv2[0]);
}

// k_fc_heads_x3: a block's K steps are a dependent chain of global-load round trips, so slices
// until the blocks cover the CUs once (C2: 32 tiles x 8 slices of 256 K), slices of >= 128 K
int az_fc_heads_splits_x3(int B, int K, int A, int H) {
    const int tiles = (B + 63) / 64 * ((A + 63) / 64 + (H + 63) / 64);
    int s = 1;
    while (s < 16 && tiles * s < 256 && K % (2 * s * 32) == 0 && K / (2 * s) >= 128) s *= 2;
    return s;
}

int az_fc_heads_splits(int B, int K, int A, int H) {
    const int tiles = (B + 63) / 64 * ((A + 63) / 64 + (H + 63) / 64);
    int s = 1;
    while (s < 16 && tiles * s * 2 <= 1024 && K % (2 * s * 32) == 0 && K / (2 * s) >= 128) s *= 2;
    return s;
}

void az_launch_fc_heads(const FcHeadArgs& a, hipStream_t st) {
    const int NT = (a.A + 63) / 64 + (a.H + 63) / 64, MT = (a.B + 63) / 64;
    FcHeadArgs f = a;
    if (a.Wx_hi && a.Wx_lo && a.hc % 8 == 0 && (a.K / a.S) % 32 == 0) {
        if (a.pt == 2) hipLaunchKernelGGL(k_fc_heads_x3<2>, dim3(MT * NT, a.S), dim3(256), 0, st, a);
        else hipLaunchKernelGGL(k_fc_heads_x3<1>, dim3(MT * NT, a.S), dim3(256), 0, st, a);
        if (a.pt != 2) f.rs = nullptr;
    } else {
        hipLaunchKernelGGL(k_fc_heads, dim3(MT * NT, a.S), dim3(256), 0, st, a);
        f.rs = nullptr;                                   // unscaled f32 rows
    }
    hipLaunchKernelGGL(k_fc_finish, dim3(a.B), dim3(256), 0, st, f);
}

// split-K partial sums only (p.part, p.splits): the caller reduces them
void az_launch_gemm_f32_partials(const GemmArgs& p, hipStream_t st) {
    const int nbm = (p.M + 127) / 128;
    if (p.N <= 64) hipLaunchKernelGGL((gemm_f32<64, ACT_NONE, false>), dim3(nbm * ((p.N + 63) / 64), p.splits), dim3(256), 0, st, p);
    else hipLaunchKernelGGL((gemm_f32<128, ACT_NONE, false>), dim3(nbm * ((p.N + 127) / 128), p.splits), dim3(256), 0, st, p);
}

// Value head after FC1's split-K partials, one block per board: h = relu(sum_s part[s][b] + b1)
// (slices summed in order), value = tanh(sum_n h[n] * w2[n] + b2) with a fixed-order block
// reduction.  H <= 1024 hidden units.
__global__ __launch_bounds__(256) void k_value_head(const float* part, int splits, const float* b1, const float* w2,
                                                    const float* b2, float* hid, float* value, int B, int H,
                                                    const int* m_limit) {
    const int b = blockIdx.x;
    if (m_limit && b >= *m_limit) return;
    __shared__ float red[256];
    float acc = 0.0f;
    for (int n = threadIdx.x; n < H; n += 256) {
        float v = 0.0f;
        for (int s = 0; s < splits; ++s) v += part[((size_t)s * B + b) * H + n];
        v += b1[n];
        v = v > 0.0f ? v : 0.0f;
        hid[(size_t)b * H + n] = v;
        acc = __builtin_fmaf(v, w2[n], acc);
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) value[b] = tanhf(red[0] + b2[0]);
}

void az_launch_value_head(const float* part, int splits, const float* b1, const float* w2, const float* b2, float* hid,
                          float* value, int B, int H, const int* m_limit, hipStream_t st) {
    hipLaunchKernelGGL(k_value_head, dim3(B), dim3(256), 0, st, part, splits, b1, w2, b2, hid, value, B, H, m_limit);
}

void az_launch_gemm_f32(const GemmArgs& p, int act, bool res, hipStream_t st) {
    const bool small = p.N <= 64;
    if (small) {
        if (res) { if (act == ACT_RELU) launch_f32<64, ACT_RELU, true>(p, st); else launch_f32<64, ACT_NONE, true>(p, st); }
        else if (act == ACT_RELU) launch_f32<64, ACT_RELU, false>(p, st);
        else if (act == ACT_TANH) launch_f32<64, ACT_TANH, false>(p, st);
        else launch_f32<64, ACT_NONE, false>(p, st);
    } else {
        if (res) { if (act == ACT_RELU) launch_f32<128, ACT_RELU, true>(p, st); else launch_f32<128, ACT_NONE, true>(p, st); }
        else if (act == ACT_RELU) launch_f32<128, ACT_RELU, false>(p, st);
        else if (act == ACT_TANH) launch_f32<128, ACT_TANH, false>(p, st);
        else launch_f32<128, ACT_NONE, false>(p, st);
    }
}

void az_launch_pool(const float* in, float* out, int B, int H, int W, int C, int P, const int* m_limit, hipStream_t st) {
    hipLaunchKernelGGL(k_adaptive_pool, dim3(B * P * P), dim3(C < 256 ? 64 : 256), 0, st, in, out, B, H, W, C, P, m_limit);
}

void az_launch_pack_input(const float* in, float* out, int B, int Cin, int HW, int Cp, hipStream_t st) {
    const size_t total = (size_t)B * HW * Cp;
    hipLaunchKernelGGL(k_pack_input, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, in, out, B, Cin, HW, Cp);
}

void az_launch_softmax_rows(const float* logits, float* out, int B, int A, hipStream_t st) {
    hipLaunchKernelGGL(k_softmax_rows, dim3(B), dim3(256), 0, st, logits, out, A);
}

void az_launch_se_residual(const float* y, const float* x, float* out, const float* W1, const float* b1, const float* W2,
                           const float* b2, int B, int HW, int C, int R, const int* m_limit, hipStream_t st) {
    const int S = B >= 256 ? 1 : std::min(8, 256 / B);   // blocks per board: cover the CUs at small batches
    hipLaunchKernelGGL(k_se_residual, dim3(B, S), dim3(256), 0, st, y, x, out, W1, b1, W2, b2, HW, C, R, m_limit);
}
