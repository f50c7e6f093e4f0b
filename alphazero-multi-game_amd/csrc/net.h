// net.h -- launch interface of the ConvNet kernels (net_kernels.hip, conv_bf16.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

enum { ACT_NONE = 0, ACT_RELU = 1, ACT_TANH = 2 };

// cache-policy bits of the trunk convs' residual-join loads (raw buffer loads of the g8 planes in the
// epilogue; gfx950 CPol: 1 sc0, 2 nt, 16 sc1)
#ifndef AZ_RES_AUX
#define AZ_RES_AUX 2
#endif

// out[m][n] = act( sum_k A(m,k) * B[n][k] + bias[n] (+ res[m][n]) ),  k = tap*C + c
struct GemmArgs {
    const float* A; int lda;        // activations, row-major [rows][lda] (NHWC for convs)
    const float* B; int ldb;        // weights [N][ldb], BN folded
    float* C; int ldc;              // output [rows][ldc]
    const float* bias;              // [N] or null
    const float* res;               // residual [rows][ldc] or null
    int M, N, K, Kpad;              // K = taps*C, Kpad = K rounded up to the k-tile
    int taps, Cch;                  // 9 (3x3, pad 1) or 1; channels per tap
    int H, W;                       // spatial size of one sample (taps == 9)
    const int* m_limit;             // device: active samples (leaf batch) or null
    int rows_per_sample;            // rows of one sample (H*W, P*P or 1)
    float* part;                    // split-K workspace [splits][M][N] (FC layers) or null
    int splits;                     // K slices when part != null
    const float* const* Am;         // taps == 1 only: K spans Cch-wide slices of several inputs,
                                    // slice j from Am[j] (device array; a rand-wire router's concat)
};

// bf16 trunk conv: activations stored as bf16 hi (+ lo) planes, NHWC.
// zeroed tail after every 16-bit activation buffer (elements): the v6 conv's padding source
constexpr size_t AZ_ACT_TAIL = 262144;   // zeroed 16-bit elements behind every g8 activation buffer (512 KB)

struct ConvBf16Args {
    const uint16_t* Ahi; const uint16_t* Alo;   // [rows][C] bf16 (Alo null for plain bf16)
    const uint16_t* Bhi; const uint16_t* Blo;   // [N][9*C] bf16
    const uint16_t* Bblk;                       // chunk-blocked [C/16][9][2][N][8] (v5; same type as Ahi)
    const uint16_t* Bblk_lo;                    // conv3x3_v7x3: the bf16 lo parts of Bblk, same layout
    uint16_t* Chi; uint16_t* Clo;               // outputs (split for the next layer)
    float* Cf;                                  // optional fp32 output [rows][N]
    const float* bias;
    const uint16_t* Rhi; const uint16_t* Rlo;   // residual (split) or null
    const float* Rf;                            // fp32 residual [rows][N] (v4 only)
    const int8_t* Rq; int8_t* Cq;               // v5: int8 remainders of the g8 residual / output
    int M, N, C, H, W;
    size_t a_tail;                              // v6: byte offset of Ahi's zeroed tail (AZ_ACT_TAIL); 0 = M*C*2
    const int* m_limit; int rows_per_sample;
    int relu;
    const uint16_t* zero;                       // >= 64 zero bytes (padding source for glds)
    int stamp;                                  // diagnostic builds: launch slot for phase stamps
    int flags;                                  // kernel variant bits (az_diag_set_conv_flags; A/B tests)
    int* ovf;                                   // fp16 outputs: set to 1 when a value leaves the fp16 range (or null)
    int pt;                                     // x3 kernels (v7x3 / v9x3): pieces 1 = bf16 (0 reads as 1), 2 = fp16
    const float* oscale;                        // pt 2: per-output-channel 2^-s undoing the weights' scale 2^s
    int stagger;                                // conv3x3_v9x3: first-round start offsets spread over this many ns
};

// k_smallnet (smallnet.hip): the whole trunk + pool + head 1x1 convs of a 64-filter net, one board per block
struct SmallNetArgs {
    const float* x0;                // leaf planes [B][H*W][16] fp32 (NHWC16), or null with rec
    const uint8_t* rec;             // or: leaf records (leaf_planes.h, Gomoku), board b = record gidx[b]
    const int* gidx;                // with rec: the batch's games
    int rec_n;                      // with rec: records (games); gidx entries are clamped to it
    int rec_identity;               // with rec: gidx[b] == b (the search's identity batch): gidx not read
    const int* m_limit;             // device: active boards
    const uint16_t* W;              // [2*blocks+1][9][64 n][64 c] fp16, BN folded; layer 0 = input conv (c >= planes zero)
    const uint16_t* Wf;             // the same, fragment-major [layer][tap][kk][J][64 lanes][8] (engine.hip)
    const float* bias;              // [2*blocks+1][64]
    const float* Wpc; const float* bpc;   // policy 1x1 conv [HC][64], [HC] (BN folded)
    const float* Wvc; const float* bvc;   // value 1x1 conv
    float* pp; float* vp;           // head feature maps [B][P*P][HC] fp32
    int H, blocks, residual, HC, P;
    int stamps;                     // diagnostic: block 0 writes phase stamps (az_diag_smallnet_stamps)
    int* ovf;                       // set to 1 when an activation leaves the fp16 range
    const uint16_t* Wxh;            // AZ_PREC_BF16X3 / F16X3 (k_smallnet_x3): hi / lo pieces of the weights,
    const uint16_t* Wxl;            // fragment-major as Wf; null = the fp16 kernel
    int pt;                         // k_smallnet_x3 pieces: 1 bf16, 2 fp16 (weights scaled by 2^s per output channel,
    const float* osc;               // bias = b * 2^s; osc [L][64] = 2^-s)
};
bool az_smallnet_supported(int H, int C, int cin_pad, int pool, int head_channels);
int az_smallnet_max_blocks();
int az_smallnet_launch(const SmallNetArgs& a, int B, hipStream_t st);
int az_smallnet_stamps_mode();        // az_diag_set_smallnet_stamps (0: off)

void az_launch_gemm_f32(const GemmArgs& p, int act, bool res, hipStream_t st);
void az_launch_gemm_f32_partials(const GemmArgs& p, hipStream_t st);

// k_fc_heads + k_fc_finish: policy FC + value FC1/FC2 (split-K partials, then one block per board)
struct FcHeadArgs {
    const float* pp; const float* vp;           // head feature maps [B][K] (K = HC * P * P)
    const float* Wp; const float* bp;           // policy FC [A][K], [A]
    const float* Wv1; const float* bv1;         // value FC1 [H][K], [H]
    const float* wv2; const float* bv2;         // value FC2 [H], [1]
    float* logits; float* hid; float* value;    // [B][A], [B][H], [B]
    float* part;                                // split-K workspace [S][B64][NT * 64]
    const int* m_limit;
    int B, K, A, H, S;
    int hc, xs;                                 // head channels; cell stride of pp / vp (xs == hc: contiguous [B][K])
    const uint16_t* Wx_hi; const uint16_t* Wx_lo;   // bf16x3 (k_fc_heads_x3): [NC][K] hi / lo rows (policy padded
                                                    // to a multiple of 64, then value), or null (f32 k_fc_heads)
    int pt;                                     // k_fc_heads_x3 pieces: 1 bf16, 2 fp16 (rows scaled by 2^s,
    const float* rs;                            // pt 2: [NC] 2^-s, applied by k_fc_finish to the slice sums)
    int* ovf;                                   // pt 2: set to 1 when a head feature leaves the fp16 range
};
int az_fc_heads_splits(int B, int K, int A, int H);
int az_fc_heads_splits_x3(int B, int K, int A, int H);
void az_launch_fc_heads(const FcHeadArgs& a, hipStream_t st);
void az_launch_value_head(const float* part, int splits, const float* b1, const float* w2, const float* b2, float* hid,
                          float* value, int B, int H, const int* m_limit, hipStream_t st);
void az_launch_pool(const float* in, float* out, int B, int H, int W, int C, int P, const int* m_limit, hipStream_t st);
void az_launch_pack_input(const float* in, float* out, int B, int Cin, int HW, int Cp, hipStream_t st);
void az_launch_softmax_rows(const float* logits, float* out, int B, int A, hipStream_t st);

// DDW-RandWire node tail: out = relu(y * SE(y) + x) (k_se_residual; C % 16 == 0, C <= 1024, R = C / 16 <= 64)
void az_launch_se_residual(const float* y, const float* x, float* out, const float* W1, const float* b1, const float* W2,
                           const float* b2, int B, int HW, int C, int R, const int* m_limit, hipStream_t st);
// 1x1 GEMM with fp16 operands (rounded from fp32 on load), fp32 accumulation, bias + ReLU
// (gemm_h16_relu: the fp16 rand-wire routers; taps == 1, K % 4 == 0, Am slices or A)
void az_launch_gemm_h16_relu(const GemmArgs& p, hipStream_t st);
