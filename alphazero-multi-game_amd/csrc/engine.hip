// engine.hip -- host runtime behind include/az_engine.h (libaz_hip.so).
//
// Owns device memory, streams and launches; no exceptions cross the C-ABI.
// The product path never falls back to the CPU: without a HIP device every entry
// point fails with AZ_ERR_HIP.
#include <hip/hip_runtime.h>
#include <pthread.h>
#include <sched.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <future>
#include <mutex>
#include <sstream>
#include <chrono>
#include <random>
#include <string>
#include <thread>
#include <unordered_set>
#include <vector>

#include "../../include/az_engine.h"
#include "engine_internal.h"
#include "net.h"
#include "tree.h"
#include "leaf_planes.h"
#include "randwire.h"

// kernels (tree_kernels.hip)
void az_launch_select(const TreeDev* t, int NA, int G, int mode, hipStream_t st);
void az_launch_expand_select(const TreeDev* ts, const int* eval_slot, int eval_identity, int NA, int G, hipStream_t st);
__global__ void k_scan(const TreeDev* __restrict__ tp);
__global__ void k_expand_backup(const TreeDev* __restrict__ tp, int mode);
__global__ void k_select_action(const TreeDev* __restrict__ tp, int training, float temperature, const float* temps, int* actions, float* values, float* probs,
                                int* child_actions, int* nchild);
__global__ void k_apply(TreeDev t, const int* actions, int* terminal, int* result, int* rexp);
__global__ void k_compact(TreeDev t, Nodes dst, int* src_of);
__global__ void k_leaf_moves(TreeDev t, int* moves, int* len);
__global__ void k_prune(TreeDev t, Nodes dst, int* src_of, int thr_all, const int* thr_g, long long* pruned);
__global__ void k_noise(TreeDev t, const float* noise, const uint8_t* mask, float eps);
__global__ void k_new_games(TreeDev t, const int* games, const int* seed_ids, int n, uint32_t eval_seed);
__global__ void k_init_slots(TreeDev t, Nodes other);
__global__ void k_tt_clear(TreeDev t, const int* games, int n);
__global__ void k_root_nchild(TreeDev t, int* out);
__global__ void k_root_children(TreeDev t, int g, int* act, int* N, int* VL, float* W, float* P, int* n, int* rootinfo,
                                float* rootW);
void az_conv_bf16_launch_v(const ConvBf16Args& a, bool split, hipStream_t st);
bool az_conv_v4_supported(int H, int W, int C, int N);
void az_conv_v4_launch(const ConvBf16Args& a, int mode, hipStream_t st);
int az_conv_bf16_name(const ConvBf16Args& a, int mode, char* out, int len);
int az_conv_g8_name(const ConvBf16Args& a, int mode, char* out, int len);
extern "C" int az_diag_set_conv_flags(int flags);
bool az_conv_g8_supported(int H, int W, int C, int N);
int az_conv_g8_launch(const ConvBf16Args& a, int mode, hipStream_t st);
void az_launch_to_g8(const float* in, uint16_t* hi, int8_t* q, int C, int HW, const int* m_limit, int maxB, int mode,
                     hipStream_t st, int Cout = 0);
void az_launch_rec_to_g8(const uint8_t* rec, const int* gidx, uint16_t* hi, int go, int bs, const int* m_limit, int maxB,
                         int mode, hipStream_t st, int NG = 2);
void az_launch_rec_planes(const uint8_t* rec, float* dst, const int* eval_games, const int* n_eval, int go, int bs, int maxB,
                          hipStream_t st);
void az_launch_pool_g8(const uint16_t* hi, const int8_t* q, float* out, int B, int C, int H, int P, const int* m_limit,
                       int mode, hipStream_t st);
bool az_pool_heads_supported(int C, int H, int P, int N);
int az_launch_pool_heads_g8(const uint16_t* hi, const int8_t* q, const float* Wt, const float* bias, float* out, int B,
                            int C, int H, int P, int N, const int* m_limit, int mode, hipStream_t st);
void az_launch_to_g8x3(const float* in, uint16_t* hi, uint16_t* lo, int C, int HW, const int* m_limit, int maxB,
                       hipStream_t st, int pt, int* ovf);
bool az_conv_v7x3_supported(const ConvBf16Args& a);
int az_conv_v7x3_launch(const ConvBf16Args& a, hipStream_t st);
int az_conv_x3_name(const ConvBf16Args& a, char* out, int len);
int az_conv_flags();
void az_launch_to_f16(const float* in, uint16_t* out, size_t n, const int* m_limit, int rows_per_sample, int C,
                      hipStream_t st, int* ovf);
void az_launch_split_bf16(const float* in, uint16_t* hi, uint16_t* lo, size_t n, const int* m_limit, int rows_per_sample,
                          int C, hipStream_t st);

namespace {
thread_local std::string g_err;
}  // namespace

int az_fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

namespace {


uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

}  // namespace


struct Layer {            // one implicit-GEMM layer, BN folded
    float* W = nullptr;   // [N][K] fp32
    uint16_t* Whi = nullptr; uint16_t* Wlo = nullptr;   // bf16 split copies (3x3 trunk)
    uint16_t* Wh16 = nullptr;                           // fp16 copy (3x3 trunk, AZ_PREC_FP16)
    uint16_t* Wbk_bf = nullptr; uint16_t* Wbk_h = nullptr;  // chunk-blocked bf16 / fp16 copies (v5 conv)
    uint16_t* Wbk_lo = nullptr;                         // chunk-blocked bf16 lo parts (conv3x3_v7x3, AZ_PREC_BF16X3)
    // AZ_PREC_F16X3: the weights of output channel o scaled by 2^s_o (max |W[o]| in [2^13, 2^14)) and
    // split into chunk-blocked fp16 hi / lo pieces; bx = b * 2^s (the accumulators' start), sx = 2^-s
    uint16_t* Wbk_fh = nullptr; uint16_t* Wbk_fl = nullptr;
    float* bx = nullptr; float* sx = nullptr;
    float* b = nullptr;   // [N]
    int N = 0, K = 0, Kpad = 0, taps = 1, C = 0;
};

// One DDW-RandWire node (row f4): its router (only used with >1 predecessors), the residual
// block's two 3x3 convs (BN folded) and the SE block's two linear layers.
struct RwNode {
    Layer router, c1, c2;
    const float** ins = nullptr;   // device: the predecessors' output buffers (the router's concat)
    float *w1 = nullptr, *b1 = nullptr, *w2 = nullptr, *b2 = nullptr;   // SE: [R][C], [R], [C][R], [C]
};
struct RwBlock {
    azrw::Plan plan;
    std::vector<RwNode> node;   // by node id
    Layer out_router;           // when the block has more than one sink
    const float** outs = nullptr;   // device: the sinks' output buffers
};

// Sampled kernel timing (az_net_profile / az_search_profile, bench.py's roofline and tree-kernel
// times): a one-wave kernel on the engine stream writes the 100 MHz device clock (s_memrealtime)
// into the next slot of a device buffer; a timed interval is the difference of two stamps around
// the kernels it brackets (same-stream order: each stamp runs after the previous kernel completes).
// HIP events, used before round 4, never completed under rocprofv3 --pmc counter collection once a
// selfplay step had recorded them (profiles/r03e_pmc_hang_probe.txt); stamps are ordinary dispatches.
__global__ void k_clock_stamp(unsigned long long* out) {
    if (threadIdx.x == 0) out[threadIdx.x] = __builtin_amdgcn_s_memrealtime();   // vector store (lane-indexed)
}
struct ProfClock {
    static constexpr size_t CAP = 1 << 16;      // stamps per profiling session (bench: a few thousand)
    unsigned long long* d = nullptr;
    size_t used = 0;
    bool room(size_t k) const { return d && used + k <= CAP; }
    void stamp(hipStream_t st) { hipLaunchKernelGGL(k_clock_stamp, dim3(1), dim3(64), 0, st, d + used); ++used; }
    // the stamps [0, used) on the host, in milliseconds (10 ns ticks)
    std::vector<double> read_ms() const {
        std::vector<unsigned long long> h(used);
        if (used && hipMemcpy(h.data(), d, used * 8, hipMemcpyDeviceToHost) != hipSuccess) h.assign(used, 0);
        std::vector<double> out(used);
        for (size_t i = 0; i < used; ++i) out[i] = (double)h[i] * 1e-5;
        return out;
    }
    void release() { if (d) (void)hipFree(d); d = nullptr; used = 0; }
};

struct az_net {
    az_engine* e = nullptr;
    az_net_desc d{};
    int cin_pad = 16;
    int HW = 0, P2 = 0;
    size_t act_elems = 0;   // elements of every 16-bit activation buffer before its zeroed tail
    size_t nparams = 0;
    Layer in, pconv, vconv, pfc, vfc1, vfc2;
    // the input conv with its 16 input channels zero-padded to 32 (16-bit chunk-blocked copies only
    // used): boards other than 15x15 take it on conv3x3_v6 (32-channel chunks) instead of the f32
    // GEMM + fp32 -> g8 conversion (C4 Go, 128-board shard: ~98 -> ~15 us per forward)
    Layer in32;
    Layer hconv;              // [pconv; vconv] as one 1x1 conv (2 HC outputs): both heads in one GEMM
    float* hpv = nullptr;     // its output [B * P * P][2 HC] (policy channels, then value)
    std::vector<Layer> blk;   // 2 per block
    // activations (max_batch samples)
    float *x0 = nullptr, *h0 = nullptr, *h1 = nullptr, *t = nullptr, *pool = nullptr;
    uint16_t *hh[2] = {nullptr, nullptr}, *hl[2] = {nullptr, nullptr}, *th = nullptr, *tl = nullptr;
    float *pp = nullptr, *vp = nullptr, *v1 = nullptr, *logits = nullptr, *value = nullptr, *soft = nullptr;
    float* ws = nullptr;                                // split-K workspace of the FC layers
    float* in_nchw = nullptr;
    int* d_nb = nullptr;
    int* ovf = nullptr;         // set by the fp16 kernels when an activation leaves the fp16 range (sticky until read)
    uint16_t* zero = nullptr;   // 256 zero bytes: glds source for the board edge
    // k_smallnet (64-filter fp16 nets): [2*blocks+1][9][64][64] fp16 trunk weights incl. the input conv, biases
    uint16_t* sm_W = nullptr;
    uint16_t* sm_Wf = nullptr;                  // the same weights fragment-major (k_smallnet's register path)
    uint16_t* sm_Wfh = nullptr; uint16_t* sm_Wfl = nullptr;   // scaled fp16 pieces (k_smallnet_x3<.., 2>, AZ_PREC_F16X3)
    float* sm_bx = nullptr; float* sm_sx = nullptr;           // their biases * 2^s and scales 2^-s, [L][64]
    uint16_t* sm_Wxh = nullptr;                 // bf16 hi / lo parts, fragment-major (k_smallnet_x3, AZ_PREC_BF16X3)
    uint16_t* sm_Wxl = nullptr;
    uint16_t* fcx_hi = nullptr;                 // both FC layers' bf16 hi / lo rows (k_fc_heads_x3)
    uint16_t* fcx_lo = nullptr;
    uint16_t* fcf_hi = nullptr;                 // the same rows scaled by 2^s, fp16 hi / lo (k_fc_heads_x3<2>, F16X3)
    uint16_t* fcf_lo = nullptr;
    float* fcf_rs = nullptr;                    // [NC] 2^-s
    float* sm_b = nullptr;
    // DDW-RandWire trunk (az_net_create_randwire): d.blocks rand-wire blocks of 32 nodes
    bool rw = false;
    std::vector<RwBlock> rwb;
    std::vector<float*> rw_out;       // node outputs [B*HW][F], by node id
    float *rw_t2 = nullptr, *rw_in = nullptr;   // conv2 output, router output
    int rw_splits = 1;                // K slices of the node convs (from the capacity: batch-size independent)
    float* rw_ws = nullptr;           // their split-K partials [rw_splits][rows][F]
    bool loaded = false;
    std::vector<float> host_blob;   // canonical blob of the loaded weights (az_net_get_weights)
    // the device buffers of the loaded weights, in allocation order (recorded at the first load;
    // later loads rewrite the same buffers): what az_net_broadcast_weights sends
    std::vector<std::pair<void*, size_t>> wbufs;
    // every activation / workspace buffer (pointer, bytes before any zeroed tail): the poison
    // diagnostic (az_diag_set_poison) overwrites them before each forward
    std::vector<std::pair<void*, size_t>> scratch;
    // profiling: HIP events bracketing the 3x3 trunk of every forward (on the launch stream)
    bool prof = false;
    ProfClock pc;                 // sampled trunk timing (az_net_profile)
    long long prof_launches = 0, prof_forwards = 0;
    long long prof_tick = 0, prof_sampled = 0;    // events on every prof_every()-th forward only
    std::mutex mu;
};

// diagnostic: the game whose k_select / k_expand_backup write phase stamps (tools/tree_stamps.py),
// read at search creation; -1 off
static int g_tree_stamp_game = -1;
extern "C" int az_diag_set_tree_stamps(int game) {
    g_tree_stamp_game = game;
    return 0;
}

// Profiling stamps (ProfClock) are recorded on one simulation step / forward in AZ_PROF_EVERY
// (default 16): every marker on the queue leaves a gap of a few us (round 2 measured ~6 us per HIP
// event), which at C2 (a ~140 us simulation step) would otherwise inflate the timed loop.  Reads
// scale the sampled times to all steps.
static int prof_every() {
    static const int p = getenv("AZ_PROF_EVERY") ? std::max(1, atoi(getenv("AZ_PROF_EVERY"))) : 16;
    return p;
}

// ---------------------------------------------------------------- network
namespace {

struct ParamCursor {
    const float* p; size_t off = 0;
    const float* take(size_t n) { const float* r = p + off; off += n; return r; }
};

size_t count_params(const az_net_desc& d) {
    const size_t F = d.channels, Ci = d.in_planes, HC = d.head_channels, PP = (size_t)d.pool * d.pool;
    size_t n = 0;
    auto conv = [&](size_t co, size_t ci, size_t k) { n += co * ci * k * k + (d.conv_bias ? co : 0) + 4 * co; };
    conv(F, Ci, 3);
    for (int i = 0; i < d.blocks; ++i) { conv(F, F, 3); conv(F, F, 3); }
    conv(HC, F, 1);
    n += (size_t)d.action_size * HC * PP + d.action_size;
    conv(HC, F, 1);
    n += (size_t)d.fc_hidden * HC * PP + d.fc_hidden;
    n += (size_t)d.fc_hidden + 1;
    return n;
}

// Blob layout of a rand-wire net: (count, init kind, fan_in) per state entry in the reference's
// state_dict order (oracle/randwire_oracle.param_shapes; kinds as az_net_init_random).
struct PSpec { size_t n; int kind; int fan_in; };
std::vector<PSpec> rw_spec(const az_net_desc& d, const std::vector<RwBlock>& rwb) {
    const int C = d.channels, R = C / 16, HC = d.head_channels, PP = d.pool * d.pool;
    std::vector<PSpec> s;
    auto conv = [&](int co, int ci, int k) { s.push_back({(size_t)co * ci * k * k, 0, ci * k * k}); };
    auto bn = [&](int co) { for (int kd = 2; kd <= 5; ++kd) s.push_back({(size_t)co, kd, 1}); };
    auto lin = [&](int o, int i) { s.push_back({(size_t)o * i, 0, i}); s.push_back({(size_t)o, 1, i}); };
    conv(C, d.in_planes, 3); bn(C);
    for (const RwBlock& b : rwb) {
        for (int v : b.plan.order)
            if (!b.plan.preds[v].empty()) { conv(C, (int)b.plan.preds[v].size() * C, 1); bn(C); }
        for (size_t k = 0; k < b.plan.order.size(); ++k) {
            conv(C, C, 3); bn(C); conv(C, C, 3); bn(C);
            lin(R, C); lin(C, R);
        }
        if (b.plan.outputs.size() > 1) { conv(C, (int)b.plan.outputs.size() * C, 1); bn(C); }
    }
    conv(HC, C, 1); bn(HC); lin(d.action_size, HC * PP);
    conv(HC, C, 1); bn(HC); lin(d.fc_hidden, HC * PP); lin(1, d.fc_hidden);
    return s;
}

uint16_t f2bf(float f) {   // round to nearest even
    uint32_t u; std::memcpy(&u, &f, 4);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}
float bf2f(uint16_t h) { uint32_t u = (uint32_t)h << 16; float f; std::memcpy(&f, &u, 4); return f; }

// conv + BN (eval) -> folded [co][tap*cpad + c] weights and bias
void fold_conv(ParamCursor& pc, int co, int ci, int k, int cpad, bool has_bias, std::vector<float>& W, std::vector<float>& b) {
    const float* w = pc.take((size_t)co * ci * k * k);
    const float* cb = has_bias ? pc.take(co) : nullptr;
    const float* g = pc.take(co);
    const float* be = pc.take(co);
    const float* mu = pc.take(co);
    const float* var = pc.take(co);
    const int taps = k * k;
    W.assign((size_t)co * taps * cpad, 0.0f);
    b.assign(co, 0.0f);
    for (int o = 0; o < co; ++o) {
        const float scale = g[o] / std::sqrt(var[o] + 1e-5f);
        b[o] = ((cb ? cb[o] : 0.0f) - mu[o]) * scale + be[o];
        for (int c = 0; c < ci; ++c)
            for (int t = 0; t < taps; ++t) W[((size_t)o * taps + t) * cpad + c] = w[((size_t)o * ci + c) * taps + t] * scale;
    }
}

int upload_layer(Layer& L, const std::vector<float>& W, const std::vector<float>& b, int N, int K, int taps, int C,
                 bool split) {
    L.N = N; L.K = K; L.Kpad = (K + 31) / 32 * 32; L.taps = taps; L.C = C;
    if (!L.W) { DALLOC(L.W, W.size()); DALLOC(L.b, b.size()); }
    HIPCHK(hipMemcpy(L.W, W.data(), W.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(L.b, b.data(), b.size() * 4, hipMemcpyHostToDevice));
    if (split) {
        std::vector<uint16_t> hi(W.size()), lo(W.size());
        for (size_t i = 0; i < W.size(); ++i) { hi[i] = f2bf(W[i]); lo[i] = f2bf(W[i] - bf2f(hi[i])); }
        if (!L.Whi) { DALLOC(L.Whi, W.size()); DALLOC(L.Wlo, W.size()); }
        HIPCHK(hipMemcpy(L.Whi, hi.data(), hi.size() * 2, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(L.Wlo, lo.data(), lo.size() * 2, hipMemcpyHostToDevice));
        std::vector<uint16_t> h16(W.size());
        for (size_t i = 0; i < W.size(); ++i) { _Float16 h = (_Float16)W[i]; std::memcpy(&h16[i], &h, 2); }
        if (!L.Wh16) DALLOC(L.Wh16, W.size());
        HIPCHK(hipMemcpy(L.Wh16, h16.data(), h16.size() * 2, hipMemcpyHostToDevice));
        if (taps == 9 && C % 16 == 0) {
            // [N][9][C] -> [C/16][9][2][N][8]: one 64-row piece of a chunk/tap/half is 1 KiB contiguous
            std::vector<uint16_t> bb(W.size()), bh(W.size()), bl(W.size()), fh(W.size()), fl(W.size());
            std::vector<float> bx(N), sx(N);
            for (int o = 0; o < N; ++o) {
                float m = 0.0f;
                for (size_t k = 0; k < (size_t)9 * C; ++k) m = std::max(m, std::fabs(W[(size_t)o * 9 * C + k]));
                // max |W[o]| * 2^s in [2^13, 2^14); s capped at 60 so that a near-zero channel (max |w| below
                // 2^-47) cannot overflow 2^s or bias * 2^s (its tiny weights keep only fp16's subnormal precision)
                const int s = m > 0.0f ? std::min(60, 13 - std::ilogb(m)) : 0;
                const float up = std::ldexp(1.0f, s);
                bx[o] = b[o] * up;
                sx[o] = std::ldexp(1.0f, -s);
                for (int t = 0; t < 9; ++t)
                    for (int c = 0; c < C; ++c) {
                        const size_t src = ((size_t)o * 9 + t) * C + c;
                        const size_t dst = ((((size_t)(c / 16) * 9 + t) * 2 + (c / 8) % 2) * N + o) * 8 + c % 8;
                        bb[dst] = hi[src]; bh[dst] = h16[src]; bl[dst] = lo[src];
                        const float ws = W[src] * up;                     // exact: a power of two
                        const _Float16 ph = (_Float16)ws;
                        const _Float16 pl = (_Float16)(ws - (float)ph);
                        std::memcpy(&fh[dst], &ph, 2);
                        std::memcpy(&fl[dst], &pl, 2);
                    }
            }
            if (!L.Wbk_bf) {
                DALLOC(L.Wbk_bf, W.size()); DALLOC(L.Wbk_h, W.size()); DALLOC(L.Wbk_lo, W.size());
                DALLOC(L.Wbk_fh, W.size()); DALLOC(L.Wbk_fl, W.size()); DALLOC(L.bx, N); DALLOC(L.sx, N);
            }
            HIPCHK(hipMemcpy(L.Wbk_bf, bb.data(), bb.size() * 2, hipMemcpyHostToDevice));
            HIPCHK(hipMemcpy(L.Wbk_h, bh.data(), bh.size() * 2, hipMemcpyHostToDevice));
            HIPCHK(hipMemcpy(L.Wbk_lo, bl.data(), bl.size() * 2, hipMemcpyHostToDevice));
            HIPCHK(hipMemcpy(L.Wbk_fh, fh.data(), fh.size() * 2, hipMemcpyHostToDevice));
            HIPCHK(hipMemcpy(L.Wbk_fl, fl.data(), fl.size() * 2, hipMemcpyHostToDevice));
            HIPCHK(hipMemcpy(L.bx, bx.data(), N * 4, hipMemcpyHostToDevice));
            HIPCHK(hipMemcpy(L.sx, sx.data(), N * 4, hipMemcpyHostToDevice));
        }
    }
    return 0;
}

int load_heads(az_net* n, ParamCursor& pc);

int net_load(az_net* n, const float* blob) {
    const az_net_desc& d = n->d;
    ParamCursor pc{blob};
    const int F = d.channels, HC = d.head_channels, PP = d.pool * d.pool;
    std::vector<float> W, b;
    const bool split = F % 32 == 0;
    // k_smallnet weights: every 3x3 layer as [tap][n][c] over 64 channels (input conv zero-padded):
    // fp16 for k_smallnet_g, bf16 hi / lo parts for k_smallnet_x3 (AZ_PREC_BF16X3), scaled fp16 hi / lo
    // pieces for k_smallnet_x3<.., 2> (AZ_PREC_F16X3)
    const bool sm = (d.precision == AZ_PREC_FP16 || d.precision == AZ_PREC_BF16X3 || d.precision == AZ_PREC_F16X3) &&
                    az_smallnet_supported(d.board_size, F, n->cin_pad, d.pool, HC) && d.blocks <= az_smallnet_max_blocks();
    std::vector<float> smf;
    std::vector<float> smb;
    auto sm_add = [&](const std::vector<float>& Wl, const std::vector<float>& bl, int cl) {
        const size_t o = smf.size();
        smf.resize(o + (size_t)9 * F * F, 0.0f);
        for (int t = 0; t < 9; ++t)
            for (int nn = 0; nn < F; ++nn)
                for (int c = 0; c < cl; ++c) smf[o + ((size_t)t * F + nn) * F + c] = Wl[((size_t)nn * 9 + t) * cl + c];
        smb.insert(smb.end(), bl.begin(), bl.end());
    };
    fold_conv(pc, F, d.in_planes, 3, n->cin_pad, d.conv_bias, W, b);
    if (int r = upload_layer(n->in, W, b, F, 9 * n->cin_pad, 9, n->cin_pad, F % 32 == 0)) return r;  // 16-bit copies: g8 input conv
    if (n->cin_pad == 16 && d.board_size != 15 && az_conv_g8_supported(d.board_size, d.board_size, F, F) &&
        az_conv_g8_supported(d.board_size, d.board_size, 32, F)) {
        std::vector<float> W32((size_t)F * 9 * 32, 0.0f);   // [F][9][32]: channels 16..31 zero
        for (size_t ot = 0; ot < (size_t)F * 9; ++ot) std::copy(&W[ot * 16], &W[ot * 16] + 16, &W32[ot * 32]);
        if (int r = upload_layer(n->in32, W32, b, F, 9 * 32, 9, 32, true)) return r;
    }
    if (sm) sm_add(W, b, n->cin_pad);
    n->blk.resize(2 * d.blocks);
    for (int i = 0; i < 2 * d.blocks; ++i) {
        fold_conv(pc, F, F, 3, F, d.conv_bias, W, b);
        if (int r = upload_layer(n->blk[i], W, b, F, 9 * F, 9, F, split)) return r;
        if (sm) sm_add(W, b, F);
    }
    if (sm) {
        const size_t ne = smf.size();
        std::vector<uint16_t> smw(ne), smh(ne), sml(ne), sfh(ne), sfl(ne);
        for (size_t i = 0; i < ne; ++i) {
            _Float16 h = (_Float16)smf[i];
            std::memcpy(&smw[i], &h, 2);
            smh[i] = f2bf(smf[i]);
            sml[i] = f2bf(smf[i] - bf2f(smh[i]));
        }
        // fp16 pieces: output channel nn of layer l scaled by 2^s (max |W| in [2^13, 2^14)), as upload_layer
        const size_t nl = ne / ((size_t)9 * F * F);
        std::vector<float> sbx(smb.size()), ssx(smb.size());
        for (size_t l = 0; l < nl; ++l)
            for (int nn = 0; nn < F; ++nn) {
                float m = 0.0f;
                for (int t = 0; t < 9; ++t)
                    for (int c = 0; c < F; ++c) m = std::max(m, std::fabs(smf[((l * 9 + t) * F + nn) * F + c]));
                const int sc = m > 0.0f ? std::min(60, 13 - std::ilogb(m)) : 0;   // capped as in upload_layer
                const float up = std::ldexp(1.0f, sc);
                sbx[l * F + nn] = smb[l * F + nn] * up;
                ssx[l * F + nn] = std::ldexp(1.0f, -sc);
                for (int t = 0; t < 9; ++t)
                    for (int c = 0; c < F; ++c) {
                        const size_t i = ((l * 9 + t) * F + nn) * F + c;
                        const float ws = smf[i] * up;
                        const _Float16 ph = (_Float16)ws, pl = (_Float16)(ws - (float)ph);
                        std::memcpy(&sfh[i], &ph, 2);
                        std::memcpy(&sfl[i], &pl, 2);
                    }
            }
        if (!n->sm_W) {
            DALLOC(n->sm_W, ne); DALLOC(n->sm_Wf, ne); DALLOC(n->sm_Wxh, ne); DALLOC(n->sm_Wxl, ne); DALLOC(n->sm_b, smb.size());
            DALLOC(n->sm_Wfh, ne); DALLOC(n->sm_Wfl, ne); DALLOC(n->sm_bx, smb.size()); DALLOC(n->sm_sx, smb.size());
        }
        HIPCHK(hipMemcpy(n->sm_W, smw.data(), ne * 2, hipMemcpyHostToDevice));
        // fragment-major: [layer][tap][32-channel chunk kk][16-channel block J][lane][8] -- one MFMA
        // A operand (rows 16 J + lane % 16, channels 32 kk + 8 (lane / 16) ..) is 1 KB contiguous
        auto frag_major = [&](const std::vector<uint16_t>& src) {
            std::vector<uint16_t> out(ne);
            const size_t nl = ne / ((size_t)9 * F * F);
            for (size_t l = 0; l < nl; ++l)
                for (int t = 0; t < 9; ++t)
                    for (int kk = 0; kk < F / 32; ++kk)
                        for (int J = 0; J < F / 16; ++J)
                            for (int ln = 0; ln < 64; ++ln)
                                for (int e = 0; e < 8; ++e) {
                                    const int nn = 16 * J + (ln & 15), c = 32 * kk + 8 * (ln >> 4) + e;
                                    out[((((l * 9 + t) * (F / 32) + kk) * (F / 16) + J) * 64 + ln) * 8 + e] =
                                        src[((l * 9 + t) * F + nn) * F + c];
                                }
            return out;
        };
        HIPCHK(hipMemcpy(n->sm_Wf, frag_major(smw).data(), ne * 2, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(n->sm_Wxh, frag_major(smh).data(), ne * 2, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(n->sm_Wxl, frag_major(sml).data(), ne * 2, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(n->sm_Wfh, frag_major(sfh).data(), ne * 2, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(n->sm_Wfl, frag_major(sfl).data(), ne * 2, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(n->sm_bx, sbx.data(), sbx.size() * 4, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(n->sm_sx, ssx.data(), ssx.size() * 4, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(n->sm_b, smb.data(), smb.size() * 4, hipMemcpyHostToDevice));
    }
    if (int r = load_heads(n, pc)) return r;
    if (pc.off != n->nparams) return az_fail(AZ_ERR_ARG, "parameter blob size mismatch (%zu vs %zu)", pc.off, n->nparams);
    n->loaded = true;
    return 0;
}

// policy head: 1x1 conv + BN, FC over the flattened (c, y, x) pooled map; value head likewise
int load_heads(az_net* n, ParamCursor& pc) {
    const az_net_desc& d = n->d;
    const int F = d.channels, HC = d.head_channels, PP = d.pool * d.pool;
    std::vector<float> W, b;
    fold_conv(pc, HC, F, 1, F, d.conv_bias, W, b);
    if (int r = upload_layer(n->pconv, W, b, HC, F, 1, F, false)) return r;
    std::vector<float> hW = W, hb = b;                 // the combined head conv, policy rows first
    auto fc_perm = [&](int out, int hc, int pp, std::vector<float>& Wt, std::vector<float>& bt) {
        // torch flattens NCHW (index c*pp + px); our pooled head map is [px][c].
        const float* w = pc.take((size_t)out * hc * pp);
        const float* bb = pc.take(out);
        Wt.assign((size_t)out * hc * pp, 0.0f);
        for (int o = 0; o < out; ++o)
            for (int c = 0; c < hc; ++c)
                for (int px = 0; px < pp; ++px) Wt[((size_t)o * pp + px) * hc + c] = w[((size_t)o * hc + c) * pp + px];
        bt.assign(bb, bb + out);
    };
    fc_perm(d.action_size, HC, PP, W, b);
    if (int r = upload_layer(n->pfc, W, b, d.action_size, HC * PP, 1, HC * PP, false)) return r;
    fold_conv(pc, HC, F, 1, F, d.conv_bias, W, b);
    if (int r = upload_layer(n->vconv, W, b, HC, F, 1, F, false)) return r;
    hW.insert(hW.end(), W.begin(), W.end());
    hb.insert(hb.end(), b.begin(), b.end());
    if (int r = upload_layer(n->hconv, hW, hb, 2 * HC, F, 1, F, false)) return r;
    fc_perm(d.fc_hidden, HC, PP, W, b);
    if (int r = upload_layer(n->vfc1, W, b, d.fc_hidden, HC * PP, 1, HC * PP, false)) return r;
    {
        const float* w = pc.take(d.fc_hidden);
        const float* bb = pc.take(1);
        W.assign(w, w + d.fc_hidden);
        b.assign(bb, bb + 1);
        if (int r = upload_layer(n->vfc2, W, b, 1, d.fc_hidden, 1, d.fc_hidden, false)) return r;
    }
    // both FC layers as one bf16 hi / lo matrix [NC][K] for k_fc_heads_x3: policy rows padded to a
    // multiple of 64, then the value rows (the partial-column layout of k_fc_finish)
    {
        const int K = HC * PP, A = d.action_size, H = d.fc_hidden;
        const int NTP = (A + 63) / 64, NTV = (H + 63) / 64, NC = (NTP + NTV) * 64;
        std::vector<float> Wp((size_t)A * K), Wv((size_t)H * K);
        HIPCHK(hipMemcpy(Wp.data(), n->pfc.W, Wp.size() * 4, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(Wv.data(), n->vfc1.W, Wv.size() * 4, hipMemcpyDeviceToHost));
        std::vector<uint16_t> hi((size_t)NC * K, 0), lo((size_t)NC * K, 0), fh((size_t)NC * K, 0), fl((size_t)NC * K, 0);
        std::vector<float> rs(NC, 1.0f);
        auto put = [&](const std::vector<float>& Wm, int rows, int r0) {
            for (int r = 0; r < rows; ++r) {
                float m = 0.0f;
                for (int k = 0; k < K; ++k) m = std::max(m, std::fabs(Wm[(size_t)r * K + k]));
                const int s = m > 0.0f ? std::min(60, 13 - std::ilogb(m)) : 0;   // max |row| * 2^s in [2^13, 2^14); capped
                const float up = std::ldexp(1.0f, s);
                rs[r0 + r] = std::ldexp(1.0f, -s);
                for (int k = 0; k < K; ++k) {
                    const float w = Wm[(size_t)r * K + k];
                    const uint16_t h = f2bf(w);
                    hi[(size_t)(r0 + r) * K + k] = h;
                    lo[(size_t)(r0 + r) * K + k] = f2bf(w - bf2f(h));
                    const float ws = w * up;
                    const _Float16 ph = (_Float16)ws, pl = (_Float16)(ws - (float)ph);
                    std::memcpy(&fh[(size_t)(r0 + r) * K + k], &ph, 2);
                    std::memcpy(&fl[(size_t)(r0 + r) * K + k], &pl, 2);
                }
            }
        };
        put(Wp, A, 0);
        put(Wv, H, NTP * 64);
        if (!n->fcx_hi) {
            DALLOC(n->fcx_hi, hi.size()); DALLOC(n->fcx_lo, lo.size());
            DALLOC(n->fcf_hi, fh.size()); DALLOC(n->fcf_lo, fl.size()); DALLOC(n->fcf_rs, rs.size());
        }
        HIPCHK(hipMemcpy(n->fcx_hi, hi.data(), hi.size() * 2, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(n->fcx_lo, lo.data(), lo.size() * 2, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(n->fcf_hi, fh.data(), fh.size() * 2, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(n->fcf_lo, fl.data(), fl.size() * 2, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(n->fcf_rs, rs.data(), rs.size() * 4, hipMemcpyHostToDevice));
    }
    return 0;
}

// DDW-RandWire blob (rw_spec order): input conv, per block the routers (nodes() order, in-degree
// > 0), the nodes' residual blocks incl. SE, the output router; then the heads.
int net_load_rw(az_net* n, const float* blob) {
    const az_net_desc& d = n->d;
    const int F = d.channels, R = F / 16;
    ParamCursor pc{blob};
    std::vector<float> W, b;
    fold_conv(pc, F, d.in_planes, 3, n->cin_pad, false, W, b);
    if (int r = upload_layer(n->in, W, b, F, 9 * n->cin_pad, 9, n->cin_pad, false)) return r;
    auto raw = [&](float** dst, size_t cnt) -> int {
        if (!*dst) DALLOC(*dst, cnt);
        HIPCHK(hipMemcpy(*dst, pc.take(cnt), cnt * 4, hipMemcpyHostToDevice));
        return 0;
    };
    for (RwBlock& blk : n->rwb) {
        const azrw::Plan& pl = blk.plan;
        for (int v : pl.order) {
            const int deg = (int)pl.preds[v].size();
            if (!deg) continue;
            fold_conv(pc, F, deg * F, 1, deg * F, false, W, b);
            if (int r = upload_layer(blk.node[v].router, W, b, F, deg * F, 1, deg * F, false)) return r;
        }
        for (int v : pl.order) {
            RwNode& nd = blk.node[v];
            const bool h16 = F % 32 == 0;   // 16-bit weight copies: the fp16 node convs (conv3x3_v4)
            fold_conv(pc, F, F, 3, F, false, W, b);
            if (int r = upload_layer(nd.c1, W, b, F, 9 * F, 9, F, h16)) return r;
            fold_conv(pc, F, F, 3, F, false, W, b);
            if (int r = upload_layer(nd.c2, W, b, F, 9 * F, 9, F, h16)) return r;
            if (int r = raw(&nd.w1, (size_t)R * F)) return r;
            if (int r = raw(&nd.b1, R)) return r;
            if (int r = raw(&nd.w2, (size_t)F * R)) return r;
            if (int r = raw(&nd.b2, F)) return r;
        }
        const int no = (int)pl.outputs.size();
        if (no > 1) {
            fold_conv(pc, F, no * F, 1, no * F, false, W, b);
            if (int r = upload_layer(blk.out_router, W, b, F, no * F, 1, no * F, false)) return r;
        }
    }
    if (int r = load_heads(n, pc)) return r;
    if (pc.off != n->nparams) return az_fail(AZ_ERR_ARG, "parameter blob size mismatch (%zu vs %zu)", pc.off, n->nparams);
    n->loaded = true;
    return 0;
}

GemmArgs gemm_args(const Layer& L, const float* A, int lda, float* C, int ldc, const float* res, int M, int H, int W,
                   const int* m_limit, int rows_per_sample) {
    GemmArgs p{};
    p.A = A; p.lda = lda; p.B = L.W; p.ldb = L.K; p.C = C; p.ldc = ldc; p.bias = L.b; p.res = res;
    p.M = M; p.N = L.N; p.K = L.K; p.Kpad = L.Kpad; p.taps = L.taps; p.Cch = L.C; p.H = H; p.W = W;
    p.m_limit = m_limit; p.rows_per_sample = rows_per_sample;
    return p;
}

// K slices for an FC layer of B rows: enough blocks to cover the chip (a 128 x 128 f32 tile is
// bound by the CU's f32 MFMA rate), slices of >= 64 K
constexpr int FC_MAX_SPLITS = 64;
static int fc_splits(int B, int K) {
    const int tiles = (B + 127) / 128 * 2;
    int s = 1;
    while (s < FC_MAX_SPLITS && tiles * s < 512 && K / (2 * s) >= 64) s *= 2;
    return s;
}

int net_heads_fc(az_net* n, int B, const int* nb, float* logits, float* value, hipStream_t st,
                 const float* pp = nullptr, const float* vp = nullptr, int xs = 0);

// Trunk conv i (0: first conv of a block, 1: second) of an AZ_PREC_BF16X3 / AZ_PREC_F16X3 net on the
// g8 hi / lo planes (conv3x3_v9x3 / v7x3): input / output / residual plane pairs by ping-pong index `cur`.
ConvBf16Args x3_conv_args(const az_net* n, const Layer& L, int second, int cur, int B, const int* nb) {
    const az_net_desc& d = n->d;
    ConvBf16Args a{};
    a.Ahi = second ? n->th : n->hh[cur]; a.Alo = second ? n->tl : n->hl[cur];
    a.Bblk = L.Wbk_bf; a.Bblk_lo = L.Wbk_lo;
    a.pt = d.precision == AZ_PREC_F16X3 ? 2 : 1;
    if (a.pt == 2) { a.Bblk = L.Wbk_fh; a.Bblk_lo = L.Wbk_fl; a.oscale = L.sx; }
    a.Chi = second ? n->hh[cur ^ 1] : n->th; a.Clo = second ? n->hl[cur ^ 1] : n->tl;
    if (second && d.residual) { a.Rhi = n->hh[cur]; a.Rlo = n->hl[cur]; }
    a.bias = a.pt == 2 ? L.bx : L.b;
    a.M = B * n->HW; a.N = d.channels; a.C = d.channels; a.H = d.board_size; a.W = d.board_size;
    a.m_limit = nb; a.rows_per_sample = n->HW; a.relu = 1;
    a.a_tail = n->act_elems * 2;
    a.zero = n->zero; a.ovf = n->ovf;
    a.stamp = -1;
    return a;
}
// true when an AZ_PREC_BF16X3 net runs its trunk on conv3x3_v7x3 (else the NHWC split path,
// conv3x3_v4<0>): decided by the shapes alone (the chunk-blocked hi / lo weights exist for every
// 3x3 layer of a net with channels % 32 == 0 once it is loaded)
bool x3_trunk(const az_net* n) {
    const az_net_desc& d = n->d;
    if (n->rw || (d.precision != AZ_PREC_BF16X3 && d.precision != AZ_PREC_F16X3) || d.blocks < 1 || !n->hh[0] ||
        d.channels % 32)
        return false;
    Layer probe;
    probe.Wbk_bf = probe.Wbk_lo = probe.Wbk_fh = probe.Wbk_fl = n->zero;   // stand-ins for the shape check
    probe.sx = reinterpret_cast<float*>(n->zero);
    return az_conv_v7x3_supported(x3_conv_args(n, probe, 1, 0, d.max_batch, nullptr));
}

// How the forward reads its input planes: NET_IN_SMALL (k_smallnet), NET_IN_G8 (k_to_g8 + the
// g8 input conv) -- both can build board b's planes from the search's leaf record gidx[b]
// (leaf_planes.h), so the search hands its leaves over without a plane batch -- or NET_IN_GEMM
// (f32 input conv on x0).
enum { NET_IN_GEMM = 0, NET_IN_SMALL = 1, NET_IN_G8 = 2 };
int net_input_path(const az_net* n) {
    const az_net_desc& d = n->d;
    const int H = d.board_size, F = d.channels, prec = d.precision;
    if (n->rw) return NET_IN_GEMM;   // rand-wire: f32 input conv on x0
    if (n->sm_W && (prec == AZ_PREC_FP16 || prec == AZ_PREC_BF16X3 || prec == AZ_PREC_F16X3) && d.blocks > 0)
        return NET_IN_SMALL;
    const bool bf = (prec == AZ_PREC_BF16 || prec == AZ_PREC_FP16) && F % 32 == 0;
    if (bf && az_conv_g8_supported(H, H, F, F) &&
        ((n->in.Wbk_h != nullptr && az_conv_g8_supported(H, H, n->cin_pad, F)) || n->in32.Wbk_h != nullptr))
        return NET_IN_G8;
    return NET_IN_GEMM;
}

struct LeafRecs {                 // the search's leaf records: sample b = record gidx[b] (n records)
    const uint8_t* rec; const int* gidx; int go; int n;
    int identity;                 // gidx[b] == b (the identity batch): the fused forward skips that load
};

// Router of a rand-wire node: relu(BN(conv1x1(concat(ins)))) as ONE GEMM over K = deg F whose
// k-slice j is read straight from input j's buffer (the device table `dins`, same k order as the
// reference's torch::cat); BN folded into the weights and bias.
void rw_router(const az_net* n, const Layer& L, const float* const* dins, float* out, int rows, const int* nb,
               hipStream_t st) {
    const int F = n->d.channels, H = n->d.board_size;
    GemmArgs p{};
    p.Am = dins; p.lda = F; p.B = L.W; p.ldb = L.K; p.C = out; p.ldc = F; p.bias = L.b;
    p.M = rows; p.N = F; p.K = L.K; p.Kpad = L.Kpad; p.taps = 1; p.Cch = F; p.H = H; p.W = H;
    p.m_limit = nb; p.rows_per_sample = n->HW;
    if (n->d.precision == AZ_PREC_FP16) az_launch_gemm_h16_relu(p, st);   // fp16 operands, fp32 accumulation
    else az_launch_gemm_f32(p, ACT_RELU, false, st);
}

// DDW-RandWire trunk (ddw_randwire_resnet.cpp:321-384 per block): input nodes on the block input,
// the others in topological order on their router's output (or their single predecessor's
// output), the block output (output router or the single sink) into the h0 / h1 ping-pong.
float* rw_trunk(az_net* n, int B, const int* nb, hipStream_t st) {
    const az_net_desc& d = n->d;
    const int F = d.channels, H = d.board_size, HW = n->HW, rows = B * HW, R = F / 16;
    float* x = n->h0;
    for (const RwBlock& blk : n->rwb) {
        const azrw::Plan& pl = blk.plan;
        auto node = [&](int v, const float* in) {
            const RwNode& nd = blk.node[v];
            if (d.precision == AZ_PREC_FP16) {
                // fp16 operands, fp32 accumulation (conv3x3_v4): conv1 -> fp16 t, conv2 -> fp32 y;
                // the residual stream, routers and SE stay fp32
                az_launch_to_f16(in, n->hh[0], (size_t)rows * F, nb, HW, F, st, n->ovf);
                ConvBf16Args a{};
                a.Ahi = n->hh[0]; a.Bhi = nd.c1.Wh16; a.Bblk = nd.c1.Wbk_h; a.Chi = n->th; a.bias = nd.c1.b;
                a.M = rows; a.N = F; a.C = F; a.H = H; a.W = H; a.m_limit = nb; a.rows_per_sample = HW; a.relu = 1;
                a.zero = n->zero; a.ovf = n->ovf; a.stamp = -1;
                az_conv_v4_launch(a, 2, st);
                ConvBf16Args c = a;
                c.Ahi = n->th; c.Bhi = nd.c2.Wh16; c.Bblk = nd.c2.Wbk_h; c.Chi = n->hh[1]; c.Cf = n->rw_t2; c.bias = nd.c2.b;
                c.relu = 0;
                az_conv_v4_launch(c, 2, st);
                az_launch_se_residual(n->rw_t2, in, n->rw_out[v], nd.w1, nd.b1, nd.w2, nd.b2, B, HW, F, R, nb, st);
                return;
            }
            if (d.precision == AZ_PREC_BF16X3 && d.max_batch >= 128) {
                // fp32-faithful: operands split into bf16 hi + lo, three MFMAs per product, fp32
                // accumulation (conv3x3_v4 mode 0); conv1 -> split t, conv2 -> fp32 y.  Below 128
                // boards of capacity v4 has too few tiles (one per two boards) and the K-split f32
                // GEMM below is faster (chosen by capacity: batch-size independent)
                az_launch_split_bf16(in, n->hh[0], n->hl[0], (size_t)rows * F, nb, HW, F, st);
                ConvBf16Args a{};
                a.Ahi = n->hh[0]; a.Alo = n->hl[0]; a.Bhi = nd.c1.Whi; a.Blo = nd.c1.Wlo; a.Bblk = nd.c1.Wbk_bf;
                a.Chi = n->th; a.Clo = n->tl; a.bias = nd.c1.b;
                a.M = rows; a.N = F; a.C = F; a.H = H; a.W = H; a.m_limit = nb; a.rows_per_sample = HW; a.relu = 1;
                a.zero = n->zero; a.ovf = n->ovf; a.stamp = -1;
                az_conv_v4_launch(a, 0, st);
                ConvBf16Args c = a;
                c.Ahi = n->th; c.Alo = n->tl; c.Bhi = nd.c2.Whi; c.Blo = nd.c2.Wlo; c.Bblk = nd.c2.Wbk_bf;
                c.Chi = n->hh[1]; c.Clo = n->hl[1]; c.Cf = n->rw_t2; c.bias = nd.c2.b; c.relu = 0;
                az_conv_v4_launch(c, 0, st);
                az_launch_se_residual(n->rw_t2, in, n->rw_out[v], nd.w1, nd.b1, nd.w2, nd.b2, B, HW, F, R, nb, st);
                return;
            }
            GemmArgs g1 = gemm_args(nd.c1, in, F, n->t, F, nullptr, rows, H, H, nb, HW);
            GemmArgs g2 = gemm_args(nd.c2, n->t, F, n->rw_t2, F, nullptr, rows, H, H, nb, HW);
            if (n->rw_ws) { g1.part = g2.part = n->rw_ws; g1.splits = g2.splits = n->rw_splits; }
            az_launch_gemm_f32(g1, ACT_RELU, false, st);
            az_launch_gemm_f32(g2, ACT_NONE, false, st);
            az_launch_se_residual(n->rw_t2, in, n->rw_out[v], nd.w1, nd.b1, nd.w2, nd.b2, B, HW, F, R, nb, st);
        };
        for (int v : pl.inputs) node(v, x);
        for (int v : pl.topo) {
            const auto& pr = pl.preds[v];
            if (pr.empty() || std::find(pl.inputs.begin(), pl.inputs.end(), v) != pl.inputs.end()) continue;
            if (pr.size() == 1) { node(v, n->rw_out[pr[0]]); continue; }
            rw_router(n, blk.node[v].router, blk.node[v].ins, n->rw_in, rows, nb, st);
            node(v, n->rw_in);
        }
        float* y = x == n->h0 ? n->h1 : n->h0;
        if (pl.outputs.size() > 1) {
            rw_router(n, blk.out_router, blk.outs, y, rows, nb, st);
        } else {
            (void)hipMemcpyAsync(y, n->rw_out[pl.outputs[0]], (size_t)rows * F * 4, hipMemcpyDeviceToDevice, st);
        }
        x = y;
    }
    return x;
}

// Diagnostic (az_diag_set_poison): with a byte value >= 0, every activation / workspace buffer of a
// net (not the zeroed tails, not the weights) is filled with that byte before each forward, so a
// kernel that reads memory its forward never wrote gives a result that depends on the byte
// (0xff: NaN in every float format) -- the tests compare forwards under two poisons bitwise
static int g_poison = -1;
extern "C" int az_diag_set_poison(int byte) { g_poison = byte < 0 ? -1 : (byte & 0xff); return 0; }
static int poison_net(az_net* n, hipStream_t st, bool inputs) {
    if (g_poison < 0) return 0;
    for (const auto& b : n->scratch) {
        const bool in = b.first == (void*)n->x0 || b.first == (void*)n->in_nchw;
        if (in == inputs) HIPCHK(hipMemsetAsync(b.first, g_poison, b.second, st));
    }
    return 0;
}

// Forward of B samples (B = capacity; *nb = active samples, device side) from the
// NHWC16 input x0 -> logits [B][A], value [B].  lr (optional; only where
// net_input_path != NET_IN_GEMM): the planes come from leaf records instead of x0.
int net_forward(az_net* n, const float* x0, int B, const int* nb, float* logits, float* value, hipStream_t st,
                const LeafRecs* lr = nullptr) {
    const az_net_desc& d = n->d;
    const int H = d.board_size, W = d.board_size, HW = n->HW, F = d.channels, P = d.pool, PP = n->P2;
    const int rows = B * HW;
    const int prec = d.precision;
    const bool bf = (prec == AZ_PREC_BF16X3 || prec == AZ_PREC_F16X3 || prec == AZ_PREC_BF16 || prec == AZ_PREC_FP16) &&
                    F % 32 == 0;
    const bool f16 = prec == AZ_PREC_FP16;
    const bool x3 = prec == AZ_PREC_BF16X3 || prec == AZ_PREC_F16X3;
    // g8 path (v5 / v6 conv, fp16/bf16): input conv, trunk and pool all on 16-bit channel-blocked rows
    const bool g8 = !n->rw && bf && !x3 && az_conv_g8_supported(H, W, F, F);
    const bool g8x3 = x3_trunk(n);   // AZ_PREC_BF16X3 / F16X3 on the g8 hi / lo planes
    const int mode = f16 ? 2 : 1;
    int8_t* hq[2] = {reinterpret_cast<int8_t*>(n->hl[0]), reinterpret_cast<int8_t*>(n->hl[1])};
    const int inpath = net_input_path(n);
    // the trunk's tail -- pool and both head 1x1 convs -- in one launch on the g8 paths
    // (k_pool_heads_g8, bitwise what k_pool_g8 + gemm_f32 give; conv flag 0x400000 keeps those for A/B)
    const bool tail_fused = (g8 || g8x3) && n->hpv && (d.head_channels * PP) % 32 == 0 &&
                            az_pool_heads_supported(F, H, P, 2 * d.head_channels) && !(az_conv_flags() & 0x400000);
    if (lr && inpath == NET_IN_GEMM) return az_fail(AZ_ERR_ARG, "net_forward: this net cannot read leaf records");
    if (int r = poison_net(n, st, false)) return r;
    if (prec == AZ_PREC_F16X3 && !g8x3 && inpath != NET_IN_SMALL)
        return az_fail(AZ_ERR_ARG, "AZ_PREC_F16X3: no fp16-piece trunk for this shape");
    if (inpath == NET_IN_SMALL) {
        // one launch: input conv, trunk, pool and the two head 1x1 convs (smallnet.hip)
        bool sampled = false;
        if (n->prof) {
            n->prof_launches += 2 * d.blocks;    // counted in trunk-conv equivalents (bench.py's per-conv rate)
            n->prof_forwards += 1;
        }
        if (n->prof && n->prof_tick++ % prof_every() == 0 && n->pc.room(2)) {
            n->prof_sampled += 1;
            sampled = true;
            n->pc.stamp(st);
        }
        SmallNetArgs sa{};
        sa.x0 = x0; sa.m_limit = nb; sa.ovf = n->ovf;
        if (lr) {
            if (lr->go) return az_fail(AZ_ERR_ARG, "smallnet: Gomoku leaf records only");
            sa.x0 = nullptr; sa.rec = lr->rec; sa.gidx = lr->gidx; sa.rec_n = lr->n; sa.rec_identity = lr->identity;
        } sa.W = n->sm_W; sa.Wf = n->sm_Wf; sa.bias = n->sm_b;
        if (prec == AZ_PREC_BF16X3) { sa.Wxh = n->sm_Wxh; sa.Wxl = n->sm_Wxl; sa.pt = 1; }   // k_smallnet_x3
        if (prec == AZ_PREC_F16X3) {
            sa.Wxh = n->sm_Wfh; sa.Wxl = n->sm_Wfl; sa.pt = 2; sa.bias = n->sm_bx; sa.osc = n->sm_sx;
        }
        sa.Wpc = n->pconv.W; sa.bpc = n->pconv.b; sa.Wvc = n->vconv.W; sa.bvc = n->vconv.b;
        sa.pp = n->pp; sa.vp = n->vp;
        sa.H = H; sa.blocks = d.blocks; sa.residual = d.residual; sa.HC = d.head_channels; sa.P = P;
        sa.stamps = az_smallnet_stamps_mode();   // diagnostic phase stamps (az_diag_set_smallnet_stamps)
        if (az_smallnet_launch(sa, B, st)) return az_fail(AZ_ERR_ARG, "smallnet: unsupported shape");
        if (sampled) n->pc.stamp(st);
        return net_heads_fc(n, B, nb, logits, value, st);
    }
    if (inpath == NET_IN_G8) {
        // input planes -> g8 16-bit (0/1 planes are exact), then the input conv on the g8 kernel; 16
        // planes on a board whose g8 conv needs 32-channel chunks: zero groups 2-3 and in32
        // (15x15 keeps 16 channels on conv3x3_v5: 126 us per 2048-board launch against 146 us for
        // conv3x3_v6 on the zero-padded 32, profiles/r05_fused_tail_ab.txt)
        const bool i32 = !az_conv_g8_supported(H, W, n->cin_pad, F);
        const Layer& IN = i32 ? n->in32 : n->in;
        const int cin = i32 ? 32 : n->cin_pad;
        if (lr) {
            if (n->cin_pad != 16) return az_fail(AZ_ERR_ARG, "leaf records carry 16 planes");
            az_launch_rec_to_g8(lr->rec, lr->gidx, n->th, lr->go, H, nb, B, mode, st, cin / 8);
        } else {
            az_launch_to_g8(x0, n->th, nullptr, n->cin_pad, HW, nb, B, mode, st, cin);
        }
        ConvBf16Args a{};
        a.Ahi = n->th;
        a.Bblk = f16 ? IN.Wbk_h : IN.Wbk_bf;
        a.Chi = n->hh[0]; a.Cq = hq[0];
        a.bias = IN.b;
        a.M = rows; a.N = F; a.C = cin; a.H = H; a.W = W; a.m_limit = nb; a.rows_per_sample = HW; a.relu = 1;
        a.a_tail = n->act_elems * 2;          // th's zeroed tail sits behind its full capacity
        a.zero = n->zero; a.ovf = n->ovf;
        a.stamp = -1;
        if (az_conv_g8_launch(a, mode, st)) return az_fail(AZ_ERR_ARG, "g8 input conv: unsupported shape");
    } else if (g8) {
        // few input planes on a board v6 cannot take at 16 channels: f32 input conv, then to g8
        az_launch_gemm_f32(gemm_args(n->in, x0, n->cin_pad, n->h0, F, nullptr, rows, H, W, nb, HW), ACT_RELU, false, st);
        az_launch_to_g8(n->h0, n->hh[0], hq[0], F, HW, nb, B, mode, st);
    } else {
        az_launch_gemm_f32(gemm_args(n->in, x0, n->cin_pad, n->h0, F, nullptr, rows, H, W, nb, HW), ACT_RELU, false, st);
    }
    float* h = n->h0;
    float* other = n->h1;
    bool ev1 = false;                    // a sampled forward: the trunk's closing stamp is pending
    if (n->prof && d.blocks > 0) {
        n->prof_launches += 2 * d.blocks;
        n->prof_forwards += 1;
    }
    if (n->prof && d.blocks > 0 && n->prof_tick++ % prof_every() == 0 && n->pc.room(2)) {
        n->prof_sampled += 1;
        ev1 = true;
        n->pc.stamp(st);
    }
    if (n->rw) {
        h = rw_trunk(n, B, nb, st);
    } else if (!bf) {
        for (int i = 0; i < d.blocks; ++i) {
            az_launch_gemm_f32(gemm_args(n->blk[2 * i], h, F, n->t, F, nullptr, rows, H, W, nb, HW), ACT_RELU, false, st);
            az_launch_gemm_f32(gemm_args(n->blk[2 * i + 1], n->t, F, other, F, d.residual ? h : nullptr, rows, H, W, nb, HW),
                               ACT_RELU, d.residual != 0, st);
            std::swap(h, other);
        }
    } else if (g8x3) {
        // fp32-faithful trunk: every activation as g8 hi + lo planes (bf16 or fp16 pieces), three MFMAs
        // per product
        const int pt = prec == AZ_PREC_F16X3 ? 2 : 1;
        az_launch_to_g8x3(h, n->hh[0], n->hl[0], F, HW, nb, B, st, pt, n->ovf);
        int cur = 0;
        for (int i = 0; i < d.blocks; ++i) {
            ConvBf16Args a = x3_conv_args(n, n->blk[2 * i], 0, cur, B, nb);
            a.stamp = 2 * i;
            if (az_conv_v7x3_launch(a, st)) return az_fail(AZ_ERR_ARG, "bf16x3 trunk conv: unsupported shape");
            ConvBf16Args b2 = x3_conv_args(n, n->blk[2 * i + 1], 1, cur, B, nb);
            b2.stamp = 2 * i + 1;
            if (az_conv_v7x3_launch(b2, st)) return az_fail(AZ_ERR_ARG, "bf16x3 trunk conv: unsupported shape");
            cur ^= 1;
        }
        if (ev1) n->pc.stamp(st);
        ev1 = false;
        if (tail_fused) {
            if (az_launch_pool_heads_g8(n->hh[cur], reinterpret_cast<const int8_t*>(n->hl[cur]), n->hconv.W, n->hconv.b,
                                        n->hpv, B, F, H, P, 2 * d.head_channels, nb, pt == 2 ? 3 : 0, st))
                return az_fail(AZ_ERR_HIP, "k_pool_heads_g8 launch failed");
        } else {
            az_launch_pool_g8(n->hh[cur], reinterpret_cast<const int8_t*>(n->hl[cur]), n->pool, B, F, H, P, nb,
                              pt == 2 ? 3 : 0, st);
        }
    } else {
        const bool split = prec == AZ_PREC_BF16X3;
        if (g8) {
            // g8 layout, v5 conv; the int8 remainder planes live in the (otherwise idle) bf16 lo buffers
            int cur = 0;
            for (int i = 0; i < d.blocks; ++i) {
                const Layer& L1 = n->blk[2 * i];
                const Layer& L2 = n->blk[2 * i + 1];
                ConvBf16Args a{};
                a.Ahi = n->hh[cur];
                a.Bblk = f16 ? L1.Wbk_h : L1.Wbk_bf;
                a.Chi = n->th;
                a.bias = L1.b;
                a.M = rows; a.N = F; a.C = F; a.H = H; a.W = W; a.m_limit = nb; a.rows_per_sample = HW; a.relu = 1;
                a.a_tail = n->act_elems * 2;
                a.zero = n->zero; a.ovf = n->ovf;
                a.stamp = 2 * i;
                if (az_conv_g8_launch(a, mode, st)) return az_fail(AZ_ERR_ARG, "g8 trunk conv: unsupported shape");
                ConvBf16Args b2 = a;
                b2.stamp = 2 * i + 1;
                b2.Ahi = n->th;
                b2.Bblk = f16 ? L2.Wbk_h : L2.Wbk_bf;
                b2.Chi = n->hh[cur ^ 1]; b2.Cq = hq[cur ^ 1];
                b2.bias = L2.b;
                if (d.residual) { b2.Rhi = n->hh[cur]; b2.Rq = hq[cur]; }
                if (az_conv_g8_launch(b2, mode, st)) return az_fail(AZ_ERR_ARG, "g8 trunk conv: unsupported shape");
                cur ^= 1;
            }
            if (ev1) n->pc.stamp(st);
            ev1 = false;
            if (tail_fused) {
                if (az_launch_pool_heads_g8(n->hh[cur], hq[cur], n->hconv.W, n->hconv.b, n->hpv, B, F, H, P,
                                            2 * d.head_channels, nb, mode, st))
                    return az_fail(AZ_ERR_HIP, "k_pool_heads_g8 launch failed");
            } else {
                az_launch_pool_g8(n->hh[cur], hq[cur], n->pool, B, F, H, P, nb, mode, st);
            }
        } else {
        if (f16) az_launch_to_f16(h, n->hh[0], (size_t)rows * F, nb, HW, F, st, n->ovf);
        else az_launch_split_bf16(h, n->hh[0], split ? n->hl[0] : nullptr, (size_t)rows * F, nb, HW, F, st);
        int cur = 0;
        for (int i = 0; i < d.blocks; ++i) {
            const Layer& L1 = n->blk[2 * i];
            const Layer& L2 = n->blk[2 * i + 1];
            ConvBf16Args a{};
            a.Ahi = n->hh[cur]; a.Alo = split ? n->hl[cur] : nullptr;
            a.Bhi = L1.Whi; a.Blo = split ? L1.Wlo : nullptr;
            a.Chi = n->th; a.Clo = split ? n->tl : nullptr; a.Cf = nullptr;
            a.bias = L1.b; a.Rhi = nullptr; a.Rlo = nullptr;
            a.M = rows; a.N = F; a.C = F; a.H = H; a.W = W; a.m_limit = nb; a.rows_per_sample = HW; a.relu = 1;
            a.zero = n->zero; a.ovf = n->ovf;
            a.stamp = 2 * i;
            a.Bblk = f16 ? L1.Wbk_h : L1.Wbk_bf;
            if (f16) a.Bhi = L1.Wh16;
            if (f16) az_conv_v4_launch(a, 2, st);
            else az_conv_bf16_launch_v(a, split, st);
            ConvBf16Args b2 = a;
            b2.Ahi = n->th; b2.Alo = split ? n->tl : nullptr;
            b2.Bhi = L2.Whi; b2.Blo = split ? L2.Wlo : nullptr;
            b2.Chi = n->hh[cur ^ 1]; b2.Clo = split ? n->hl[cur ^ 1] : nullptr;
            b2.bias = L2.b;
            b2.stamp = 2 * i + 1;
            b2.Bblk = f16 ? L2.Wbk_h : L2.Wbk_bf;
            b2.Rhi = d.residual ? n->hh[cur] : nullptr; b2.Rlo = d.residual && split ? n->hl[cur] : nullptr;
            b2.Cf = (i == d.blocks - 1) ? other : nullptr;
            if (f16) {
                // fp16 conv operands, fp32 residual stream (an fp16 stream doubles the logit error)
                b2.Bhi = L2.Wh16;
                b2.Rhi = nullptr;
                b2.Rf = d.residual ? h : nullptr;
                b2.Cf = other;
                az_conv_v4_launch(b2, 2, st);
                std::swap(h, other);
            } else {
                az_conv_bf16_launch_v(b2, split, st);
            }
            cur ^= 1;
        }
        if (d.blocks > 0 && !f16) h = other;
        }
    }
    if (ev1) n->pc.stamp(st);
    if (!g8 && !g8x3) az_launch_pool(h, n->pool, B, H, W, F, P, nb, st);
    const int HC = d.head_channels, HK = HC * PP;
    if (tail_fused) return net_heads_fc(n, B, nb, logits, value, st, n->hpv, n->hpv + HC, 2 * HC);
    if (HK % 32 == 0 && n->hpv) {
        // both head 1x1 convs as one GEMM (2 HC outputs; every output is the same k-ordered fp32
        // chain as in two launches), read by the FC heads with a 2 HC cell stride
        az_launch_gemm_f32(gemm_args(n->hconv, n->pool, F, n->hpv, 2 * HC, nullptr, B * PP, 1, 1, nb, PP), ACT_RELU, false, st);
        return net_heads_fc(n, B, nb, logits, value, st, n->hpv, n->hpv + HC, 2 * HC);
    }
    az_launch_gemm_f32(gemm_args(n->pconv, n->pool, F, n->pp, HC, nullptr, B * PP, 1, 1, nb, PP), ACT_RELU, false, st);
    az_launch_gemm_f32(gemm_args(n->vconv, n->pool, F, n->vp, HC, nullptr, B * PP, 1, 1, nb, PP), ACT_RELU, false, st);
    return net_heads_fc(n, B, nb, logits, value, st);
}

// The FC layers of both heads from the head feature maps pp / vp ([B][P*P][HC]; cell stride xs,
// default HC: pp / vp may be the two halves of the combined head-conv output).
int net_heads_fc(az_net* n, int B, const int* nb, float* logits, float* value, hipStream_t st, const float* pp,
                 const float* vp, int xs) {
    const az_net_desc& d = n->d;
    const int PP = n->P2;
    const int HK = d.head_channels * PP;
    if (!pp) { pp = n->pp; vp = n->vp; xs = d.head_channels; }
    // Both FC heads: k_fc_heads (split-K partials of both FCs in one GEMM) + k_fc_finish (per board)
    if (HK % 32 == 0 && HK % 4 == 0) {
        FcHeadArgs fa{};
        fa.pp = pp; fa.vp = vp; fa.hc = d.head_channels; fa.xs = xs;
        fa.Wp = n->pfc.W; fa.bp = n->pfc.b; fa.Wv1 = n->vfc1.W; fa.bv1 = n->vfc1.b; fa.wv2 = n->vfc2.W; fa.bv2 = n->vfc2.b;
        fa.logits = logits; fa.hid = n->v1; fa.value = value;
        fa.part = n->ws; fa.m_limit = nb;
        fa.B = B; fa.K = HK; fa.A = d.action_size; fa.H = d.fc_hidden;
        fa.S = az_fc_heads_splits(d.max_batch, HK, d.action_size, d.fc_hidden);   // from the capacity: batch-size independent
        // split-operand FC products at 5x the f32 MFMA rate: the throughput precisions (fp16 / bf16
        // trunk) in bf16 pieces (~2^-16 per product; their trunk error is 30x larger), AZ_PREC_F16X3 in
        // scaled fp16 pieces (~2^-21, as its trunk).  AZ_PREC_BF16X3 and F32 keep exact f32 products
        // (bf16 pieces would add ~2.5e-5 at trained-scale logits).  Conv flag 0x08000000 keeps the f32
        // k_fc_heads (A/B, diagnosis).
        // Below 512 boards of capacity the f32 pair is the faster one (C2, 256 boards: k_fc_heads 10.6 us
        // vs k_fc_heads_x3 12.0 -- both latency-bound chains of L2 round trips at 0.5 GFLOP).
        const bool fx = !(az_conv_flags() & 0x08000000) && n->fcx_hi && d.max_batch >= 512;
        if (fx && (d.precision == AZ_PREC_FP16 || d.precision == AZ_PREC_BF16)) {
            fa.Wx_hi = n->fcx_hi; fa.Wx_lo = n->fcx_lo; fa.pt = 1;
            fa.S = az_fc_heads_splits_x3(d.max_batch, HK, d.action_size, d.fc_hidden);
        } else if (fx && d.precision == AZ_PREC_F16X3) {
            fa.Wx_hi = n->fcf_hi; fa.Wx_lo = n->fcf_lo; fa.pt = 2; fa.rs = n->fcf_rs; fa.ovf = n->ovf;
            fa.S = az_fc_heads_splits_x3(d.max_batch, HK, d.action_size, d.fc_hidden);
        }
        az_launch_fc_heads(fa, st);
        HIPCHK(hipGetLastError());
        return 0;
    }
    // generic shapes: split-K partials (deterministic reductions); the value head's FC1 partials
    // are reduced, ReLU'd and dotted with FC2 by one kernel per board
    if (xs != d.head_channels) return az_fail(AZ_ERR_ARG, "net_heads_fc: strided head maps need k_fc_heads");
    GemmArgs pf = gemm_args(n->pfc, n->pp, HK, logits, d.action_size, nullptr, B, 1, 1, nb, 1);
    GemmArgs v1 = gemm_args(n->vfc1, n->vp, HK, n->v1, d.fc_hidden, nullptr, B, 1, 1, nb, 1);
    const int splits = fc_splits(d.max_batch, HK);
    pf.part = n->ws; pf.splits = splits;
    v1.part = n->ws + (size_t)B * d.action_size * splits; v1.splits = splits;
    if (splits > 1) az_launch_gemm_f32(pf, ACT_NONE, false, st);
    else { pf.part = nullptr; az_launch_gemm_f32(pf, ACT_NONE, false, st); }
    az_launch_gemm_f32_partials(v1, st);
    az_launch_value_head(v1.part, splits, n->vfc1.b, n->vfc2.W, n->vfc2.b, n->v1, value, B, d.fc_hidden, nb, st);
    HIPCHK(hipGetLastError());
    return 0;
}

}  // namespace

// ===========================================================================
// A page-locked host buffer: per-move copies to / from it run at DMA speed (a pageable host side
// goes through the runtime's staging buffer).  get(k) grows it to k elements (null on failure).
template <class T>
struct Pinned {
    T* p = nullptr;
    size_t n = 0;
    T* get(size_t k) {
        if (k > n) {
            if (p) (void)hipHostFree(p);
            p = nullptr; n = 0;
            if (hipHostMalloc((void**)&p, k * sizeof(T), hipHostMallocDefault) != hipSuccess) p = nullptr;
            else n = k;
        }
        return p;
    }
    T* data() { return p; }
    ~Pinned() { if (p) (void)hipHostFree(p); }
};

struct az_search {
    az_engine* e = nullptr;
    az_net* net = nullptr;
    az_search_cfg c{};
    TreeDev t{};
    Nodes arena[2]{};
    int cur = 0;
    int* d_src_of = nullptr;
    float* d_batch = nullptr;       // gathered NHWC16 planes [G][A][16]
    int* d_id = nullptr;            // AZ_EVAL_NET: [G + 1] = 0, 1, ..., G-1, G (identity batch map + its count)
    // AZ_EVAL_CALLBACK: host evaluator, leaf moves / lengths and host staging
    az_eval_fn eval_fn = nullptr; void* eval_user = nullptr;
    int* d_lmoves = nullptr; int* d_llen = nullptr;
    std::vector<float> h_planes, h_nchw, h_pol, h_val;
    std::vector<int> h_games, h_lmoves, h_llen, h_full;
    std::vector<std::vector<int>> hist;    // per slot: the moves committed since the game started
    float* d_logits = nullptr; float* d_value = nullptr;
    float* d_noise = nullptr; uint8_t* d_mask = nullptr;
    int* d_actions = nullptr; float* d_values = nullptr; float* d_probs = nullptr; int* d_cact = nullptr; int* d_nch = nullptr;
    int* d_term = nullptr; int* d_res = nullptr; int* d_games = nullptr; int* d_seed_ids = nullptr;
    int* d_rexp = nullptr;          // k_apply: per game, its new root needs no root expansion
    // every playing game's root is expanded (or terminal): the root steps (MODE_ROOT_SEARCH /
    // MODE_ROOT_NOISE) would select nothing, evaluate nothing and expand nothing -- skipped
    bool roots_ready = false;
    // scratch allocated once: one game's root-children readback, per-game prune thresholds / counts
    int* d_rc = nullptr; float* d_rcf = nullptr; int* d_thr = nullptr; long long* d_pruned = nullptr;
    float* d_temps = nullptr;
    // host mirrors
    std::vector<int> stones, active, fresh, ply, expanded;
    // az_search_profile
    bool prof = false;
    ProfClock pc;                 // sampled tree-kernel timing (az_search_profile)
    int64_t prof_steps = 0, prof_sampled = 0;
    ProfClock pcf;                // sampled timing of the fused k_expand_select (the production tree step)
    int64_t prof_fused = 0, prof_fused_launches = 0;
    std::vector<long long> prof_cnt0;
    std::vector<std::mt19937> rng;
    Pinned<float> h_noise; std::vector<uint8_t> h_mask;   // [G][NA] Dirichlet noise (page-locked: its H2D per move)
    // az_selfplay_step's MoveData records of the last step (az_selfplay_step_moves)
    // page-locked (Pinned): the per-move D2H of every game's visit distribution and child actions
    Pinned<float> sp_probs, sp_values;
    Pinned<int> sp_cact, sp_nch;
    std::vector<int> sp_slots;
    std::vector<az_move_rec> sp_moves;
    int sp_next_id = 0;             // one past the highest game id started on the handle (az_selfplay_step restarts)
    // device-resident copies of the TreeDev variants the per-step kernels take (tree_dev()): those
    // kernels get one 8-byte pointer instead of the ~550-byte struct by value, on ~38k dispatches per
    // C3 move.  Slot i's host shadow (pinned, the source of its async upload) is h_tree[i].
    TreeDev* d_tree = nullptr;
    TreeDev* h_tree = nullptr;
    int n_tree = 0, next_tree = 0;
    int64_t tree_evictions = 0;     // slot reuses (each a stream synchronisation): az_diag_tree_evictions
    // Dirichlet draws of the NEXT move, made on a host thread while the device searches this one
    // (prefetch_noise; Gomoku self-play): per game the child count they were drawn for (-1: none)
    // and the generator state after them, taken over only when the next noise call asks for exactly
    // that count; otherwise discarded (the game's own rng was never touched) and drawn inline.
    struct NoisePrefetch {
        std::future<void> job;
        bool on = false;
        float alpha = 0.0f;
        std::vector<int> nc;
        std::vector<std::mt19937> rng;
        std::vector<float> noise;
    } pf;
    std::mutex mu;
};

namespace {

constexpr int AZ_TREE_SLOTS = 16;
// The device copy of TreeDev t (a variant with another arena or batch map is another slot).  A new
// variant is uploaded on the engine stream, so kernels queued before it still read their slot's old
// contents; a slot is reused only after a stream synchronisation (no queued kernel reads it then).
// Variants repeat (2 arenas x {search, identity batch}), so uploads happen at the first moves only.
const TreeDev* tree_dev(az_search* s, const TreeDev& t) {
    for (int i = 0; i < s->n_tree; ++i)
        if (std::memcmp(&s->h_tree[i], &t, sizeof(TreeDev)) == 0) return s->d_tree + i;
    int k;
    if (s->n_tree < AZ_TREE_SLOTS) {
        k = s->n_tree++;
    } else {
        if (hipStreamSynchronize(s->e->stream) != hipSuccess) return nullptr;
        ++s->tree_evictions;
        k = s->next_tree;
        s->next_tree = (k + 1) % AZ_TREE_SLOTS;
    }
    std::memcpy(&s->h_tree[k], &t, sizeof(TreeDev));
    if (hipMemcpyAsync(s->d_tree + k, &s->h_tree[k], sizeof(TreeDev), hipMemcpyHostToDevice, s->e->stream) != hipSuccess)
        return nullptr;
    return s->d_tree + k;
}
#define TREE_DEV(var, s, t)                                                       \
    const TreeDev* var = tree_dev(s, t);                                          \
    if (!var) return az_fail(AZ_ERR_HIP, "TreeDev upload failed")

// The fp16 range guard's flag of a net (sticky on the device until read here): AZ_ERR_RANGE once set.
int check_ovf(az_net* n, int ovf) {
    if (!ovf) return 0;
    HIPCHK(hipMemsetAsync(n->ovf, 0, 4, n->e->stream));
    HIPCHK(hipStreamSynchronize(n->e->stream));
    return az_fail(AZ_ERR_RANGE, "fp16 activation overflow (|x| > 65504) in the network forward: its outputs are invalid; "
                                 "use AZ_PREC_BF16X3 for nets with activations of this magnitude");
}

int check_err(az_search* s) {
    int err = 0, ovf = 0;
    HIPCHK(hipMemcpyAsync(&err, s->t.err, 4, hipMemcpyDeviceToHost, s->e->stream));
    if (s->net && s->c.eval_kind == AZ_EVAL_NET) HIPCHK(hipMemcpyAsync(&ovf, s->net->ovf, 4, hipMemcpyDeviceToHost, s->e->stream));
    HIPCHK(hipStreamSynchronize(s->e->stream));
    if (err) return az_fail(AZ_ERR_CAPACITY, "device capacity exceeded (flags 0x%x: 1 node pool, 2 path, 4 prior ring)", err);
    if (int r = check_ovf(s->net, ovf)) return r;
    return 0;
}

// One batched step over all games: select -> (network) -> expand/backup.
// tree-kernel timing (az_search_profile): events around K1 and K3 of simulation steps
// (clock stamps, ProfClock: four per sampled step -- before / after the selection and the expansion)

// AZ_EVAL_CALLBACK: the leaves that need an evaluation go to the host evaluator as (game, moves
// from the root, NCHW feature planes); its policies / values come back for k_expand_backup.
int host_evaluate(az_search* s) {
    hipStream_t st = s->e->stream;
    const int G = s->c.n_games, A = s->t.A, NA = s->t.NA, C = s->t.game == GAME_GO ? 8 : 11;
    TREE_DEV(dt, s, s->t);
    hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, st, dt);
    int n = 0;
    HIPCHK(hipMemcpyAsync(&n, s->t.n_eval, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (n == 0) return 0;
    if (!s->eval_fn) return az_fail(AZ_ERR_STATE, "AZ_EVAL_CALLBACK search without az_search_set_evaluator");
    az_launch_rec_planes(s->t.leafrec, s->d_batch, s->t.eval_games, s->t.n_eval, s->t.game == GAME_GO, s->t.bs, G, st);
    hipLaunchKernelGGL(k_leaf_moves, dim3(G), dim3(64), 0, st, s->t, s->d_lmoves, s->d_llen);
    s->h_planes.resize((size_t)n * A * 16); s->h_games.resize(n); s->h_lmoves.resize((size_t)n * AZ_DMAX); s->h_llen.resize(n);
    HIPCHK(hipMemcpyAsync(s->h_planes.data(), s->d_batch, (size_t)n * A * 16 * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(s->h_games.data(), s->t.eval_games, (size_t)n * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(s->h_lmoves.data(), s->d_lmoves, (size_t)n * AZ_DMAX * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(s->h_llen.data(), s->d_llen, (size_t)n * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    s->h_nchw.resize((size_t)n * C * A);
    for (int i = 0; i < n; ++i)
        for (int c = 0; c < C; ++c)
            for (int a = 0; a < A; ++a) s->h_nchw[((size_t)i * C + c) * A + a] = s->h_planes[((size_t)i * A + a) * 16 + c];
    s->h_pol.assign((size_t)n * NA, 0.0f);
    s->h_val.assign(n, 0.0f);
    // moves from the game's initial state: the slot's committed moves, then the path
    size_t mx = 1;
    for (int i = 0; i < n; ++i) mx = std::max(mx, s->hist[s->h_games[i]].size() + (size_t)s->h_llen[i]);
    s->h_full.assign((size_t)n * mx, 0);
    std::vector<int> len(n);
    for (int i = 0; i < n; ++i) {
        const std::vector<int>& h = s->hist[s->h_games[i]];
        int* dst = s->h_full.data() + (size_t)i * mx;
        std::copy(h.begin(), h.end(), dst);
        std::copy(s->h_lmoves.begin() + (size_t)i * AZ_DMAX, s->h_lmoves.begin() + (size_t)i * AZ_DMAX + s->h_llen[i],
                  dst + h.size());
        len[i] = (int)h.size() + s->h_llen[i];
    }
    if (s->eval_fn(s->eval_user, n, s->h_games.data(), len.data(), s->h_full.data(), (int)mx, s->h_nchw.data(), C,
                   s->h_pol.data(), s->h_val.data()) != 0)
        return az_fail(AZ_ERR_STATE, "host evaluator failed");
    HIPCHK(hipMemcpyAsync(s->d_logits, s->h_pol.data(), (size_t)n * NA * 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(s->d_value, s->h_val.data(), (size_t)n * 4, hipMemcpyHostToDevice, st));
    return 0;
}

// pre: this step's selection was already issued (fused into the previous step's expansion);
// fuse_next: issue this step's expansion fused with the next simulation step's selection.
int search_step(az_search* s, int mode, bool pre = false, bool fuse_next = false) {
    hipStream_t st = s->e->stream;
    const int G = s->c.n_games;
    if (mode != MODE_SIM && s->roots_ready) return 0;   // every playing root expanded: a no-op step
    // a root step that fails part-way (TreeDev upload, the host evaluator, the net forward) leaves
    // the roots unexpanded: roots_ready is set only once the step is fully issued (below)
    if (mode != MODE_SIM) s->roots_ready = false;
    s->t.nd = s->arena[s->cur];
    const int64_t sidx = s->prof_steps;   // this simulation step's index while profiling
    const bool prof = s->prof && mode == MODE_SIM && s->prof_steps++ % prof_every() == 0 && s->pc.room(4);
    if (prof) s->pc.stamp(st);
    TREE_DEV(dts, s, s->t);
    if (!pre) az_launch_select(dts, s->t.NA, s->t.G, mode, st);
    if (prof) s->pc.stamp(st);
    if (s->c.eval_kind == AZ_EVAL_CALLBACK) {
        if (int r = host_evaluate(s)) return r;
    }
    TreeDev tt = s->t;
    if (s->c.eval_kind == AZ_EVAL_NET) {
        // The batch: in a simulation step with every game active, every game has a leaf and nearly
        // all of them need the network (C3: 800 evaluations per 800-sim move), so the batch is the
        // identity (slot = game; the few terminal / TT-hit leaves are computed and ignored: the
        // net's outputs are batch-position independent) and k_scan's compaction is skipped.
        // Otherwise (root steps, finished slots) k_scan compacts the leaves that need it.
        bool identity = mode == MODE_SIM && s->d_id != nullptr;
        for (int g = 0; identity && g < G; ++g) identity = s->active[g] != 0;
        if (identity) {
            tt.eval_slot = s->d_id; tt.eval_games = s->d_id; tt.n_eval = s->d_id + G; tt.eval_identity = 1;
        } else {
            hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, st, dts);
        }
        // the net's input stage builds the leaves' planes from their records (record eval_games[b])
        // where it can; otherwise a dense fp32 plane batch is built first
        const bool in_place = net_input_path(s->net) != NET_IN_GEMM;
        const LeafRecs lr{tt.leafrec, tt.eval_games, tt.game == GAME_GO, G, identity ? 1 : 0};
        if (!in_place) az_launch_rec_planes(tt.leafrec, s->d_batch, tt.eval_games, tt.n_eval, lr.go, tt.bs, G, st);
        const bool prof = s->net->prof;
        if (mode != MODE_SIM) s->net->prof = false;   // time only the simulation batches
        int r = in_place ? net_forward(s->net, nullptr, G, tt.n_eval, s->d_logits, s->d_value, st, &lr)
                         : net_forward(s->net, s->d_batch, G, tt.n_eval, s->d_logits, s->d_value, st);
        s->net->prof = prof;
        if (r) return r;
    }
    if (prof) s->pc.stamp(st);
    if (fuse_next) {
        // the fused launch is timed on its own cadence, half-way between the split sampled steps
        const bool fs = s->prof && mode == MODE_SIM && sidx % prof_every() == prof_every() / 2 && s->pcf.room(2);
        if (s->prof && mode == MODE_SIM) ++s->prof_fused_launches;
        if (fs) s->pcf.stamp(st);
        az_launch_expand_select(dts, tt.eval_slot, tt.eval_identity, s->t.NA, G, st);
        if (fs) { s->pcf.stamp(st); ++s->prof_fused; }
    } else {
        TREE_DEV(dte, s, tt);
        hipLaunchKernelGGL(k_expand_backup, dim3(G), dim3(64), 0, st, dte, mode);
    }
    if (prof) { s->pc.stamp(st); s->prof_sampled += 1; }
    HIPCHK(hipGetLastError());
    if (mode != MODE_SIM) s->roots_ready = true;         // after it every playing root is (expanded or terminal)
    return 0;
}

// diagnostic phase trace of az_selfplay_step on stderr (az_diag_set_step_trace; tools/pmc_progress.py):
// names the host call a step is blocked in when a profiler stalls it
static int g_step_trace = 0;
extern "C" int az_diag_set_step_trace(int on) { g_step_trace = on; return 0; }
// diagnostic: a host synchronisation after every n simulation steps (0: none, the product default) --
// bounds the dispatches queued on the engine stream (rocprofv3 --pmc probe)
static int g_sync_every = 0;
extern "C" int az_diag_set_sync_every(int n) { g_sync_every = n; return 0; }
// each line carries the host's wall clock (ms, steady_clock) so the phases of a move can be timed
#define STEP_TRACE(...)                                                                               \
    do {                                                                                              \
        if (g_step_trace) {                                                                           \
            fprintf(stderr, "[step %.3f] ", std::chrono::duration<double, std::milli>(                \
                                                std::chrono::steady_clock::now().time_since_epoch()).count()); \
            fprintf(stderr, __VA_ARGS__); fputc('\n', stderr); fflush(stderr);                        \
        }                                                                                             \
    } while (0)

// n simulation steps.  Step i's expansion and step i+1's selection share one launch
// (k_expand_select) except around the profiled steps (their kernels are timed separately) and
// with the host evaluator (which runs between the two).
int search_sims(az_search* s, int n) {
    const bool can_fuse = s->c.eval_kind != AZ_EVAL_CALLBACK;
    bool pre = false;
    for (int i = 0; i < n; ++i) {
        const bool sampled = s->prof && s->prof_steps % prof_every() == 0;
        const bool next_sampled = s->prof && (s->prof_steps + 1) % prof_every() == 0;
        const bool fuse = can_fuse && i + 1 < n && !sampled && !next_sampled;
        if (int r = search_step(s, MODE_SIM, pre, fuse)) return r;
        pre = fuse;
        if ((i + 1) % 100 == 0) STEP_TRACE("%d sims issued", i + 1);
        if (g_sync_every > 0 && (i + 1) % g_sync_every == 0) HIPCHK(hipStreamSynchronize(s->e->stream));
    }
    return 0;
}

// Host worker threads for per-game host work: the process's CPU share -- its affinity mask (a
// multi-GPU bench rank runs on its own slice of the host, bench.py), capped by OMP_NUM_THREADS
// where set (the GPU boxes, where hardware_concurrency reports the whole machine) and by 16.
int host_threads() {
    static const int n = [] {
        int h = (int)std::thread::hardware_concurrency();
        cpu_set_t cs;
        if (sched_getaffinity(0, sizeof(cs), &cs) == 0 && CPU_COUNT(&cs) > 0) h = std::min(h, (int)CPU_COUNT(&cs));
        if (const char* e = getenv("OMP_NUM_THREADS")) if (atoi(e) > 0) h = std::min(h, atoi(e));
        return std::max(1, std::min(16, h));
    }();
    return n;
}

// addDirichletNoise's draws for one game (parallel_mcts.cpp:1136-1156): nc gammas of a fresh
// libstdc++ gamma_distribution<float>(alpha) on the game's mt19937, floored and normalised
void draw_dirichlet(std::mt19937& rng, float alpha, int nc, float* nz) {
    std::gamma_distribution<float> gamma(alpha, 1.0f);
    float sum = 0.0f;
    for (int i = 0; i < nc; ++i) { nz[i] = std::max(1e-10f, gamma(rng)); sum += nz[i]; }
    if (sum <= 0.0f) { sum = 1.0f; for (int i = 0; i < nc; ++i) nz[i] = 1.0f / (float)nc; }
    for (int i = 0; i < nc; ++i) nz[i] /= sum;
}

// the prefetch job done (every accessor of s->rng / s->pf calls this first)
void pf_wait(az_search* s) {
    if (s->pf.job.valid()) s->pf.job.get();
}
// game g's generator changes outside the noise path (reseed, set, stochastic selectAction): its
// prefetched draws no longer follow from it
void pf_drop(az_search* s, int g) {
    pf_wait(s);
    if (s->pf.on && g >= 0 && g < (int)s->pf.nc.size()) s->pf.nc[g] = -1;
}

// Start drawing the next move's noise for the games in `want` on a host thread (Gomoku: a root
// after one more stone has A - stones - 1 legal children).  The draws use copies of the games'
// generators; search_noise adopts a game's copy only when it asks for that very draw.
void prefetch_noise(az_search* s, float alpha, const std::vector<uint8_t>& want) {
    pf_wait(s);
    auto& P = s->pf;
    const int G = s->c.n_games, A = s->t.A, NA = s->t.NA;
    P.on = false;
    if (s->t.game != GAME_GOMOKU) return;
    P.nc.assign(G, -1);
    P.rng.resize(G);
    P.noise.resize((size_t)G * NA);
    bool any = false;
    for (int g = 0; g < G; ++g)
        if (want[g] && s->active[g] && A - s->stones[g] - 1 > 0) { P.nc[g] = A - s->stones[g] - 1; any = true; }
    if (!any) return;
    P.on = true;
    P.alpha = alpha;
    P.job = std::async(std::launch::async, [s, alpha, G, NA] {
        pthread_setname_np(pthread_self(), "az-noise-pf");   // named in crash reports (az_diag_crash_report)
        auto& Q = s->pf;
        for (int g = 0; g < G; ++g) {
            if (Q.nc[g] < 0) continue;
            Q.rng[g] = s->rng[g];
            draw_dirichlet(Q.rng[g], alpha, Q.nc[g], Q.noise.data() + (size_t)g * NA);
        }
    });
}

int search_noise(az_search* s, float alpha, float eps, const uint8_t* mask) {
    const int G = s->c.n_games, A = s->t.A, NA = s->t.NA;
    if (int r = search_step(s, MODE_ROOT_NOISE)) return r;
    pf_wait(s);
    STEP_TRACE("noise: root step issued");
    std::vector<int> nroot;
    if (s->t.game == GAME_GO) {        // |children| of each root (legal moves incl. pass and superko)
        nroot.resize(G);
        s->t.nd = s->arena[s->cur];
        hipLaunchKernelGGL(k_root_nchild, dim3((G + 255) / 256), dim3(256), 0, s->e->stream, s->t, s->d_nch);
        HIPCHK(hipMemcpyAsync(nroot.data(), s->d_nch, G * 4, hipMemcpyDeviceToHost, s->e->stream));
        HIPCHK(hipStreamSynchronize(s->e->stream));
    }
    // addDirichletNoise draws (parallel_mcts.cpp:1136-1156): libstdc++ gamma on the host,
    // one fresh gamma_distribution per call on the game's mt19937.
    // Every game draws from its own mt19937, so the games split over host threads without changing
    // a single draw (a C2 move's 128 x 225 draws take ~6 ms on one core).
    auto& P = s->pf;
    const bool pfo = P.on && P.alpha == alpha;
    int inline_games = 0;
    for (int g = 0; g < G; ++g) {
        if (!s->active[g] || (mask && !mask[g])) continue;
        const int nc = !nroot.empty() ? nroot[g] : s->fresh[g] ? A : A - s->stones[g];
        inline_games += !(pfo && nc > 0 && P.nc[g] == nc);
    }
    auto draw = [&](int g0, int g1) {
        if (g0 > 0) pthread_setname_np(pthread_self(), "az-gamma");   // the workers (g0 = 0: the caller)
        for (int g = g0; g < g1; ++g) {
            s->h_mask[g] = 0;
            if (!s->active[g] || (mask && !mask[g])) continue;
            const int nc = !nroot.empty() ? nroot[g] : s->fresh[g] ? A : A - s->stones[g];
            if (nc <= 0) continue;
            float* nz = s->h_noise.data() + (size_t)g * NA;
            if (pfo && P.nc[g] == nc) {               // drawn ahead from a copy of this very generator state
                std::copy(P.noise.begin() + (size_t)g * NA, P.noise.begin() + (size_t)g * NA + nc, nz);
                s->rng[g] = P.rng[g];
            } else {
                draw_dirichlet(s->rng[g], alpha, nc, nz);
            }
            s->h_mask[g] = 1;
        }
    };
    // host threads only for the draws still to be made (none when the prefetch covered the move)
    const int nt = std::max(1, std::min({host_threads(), inline_games / 16}));
    if (nt == 1) {
        draw(0, G);
    } else {
        std::vector<std::thread> th;
        for (int t = 1; t < nt; ++t) th.emplace_back(draw, (int)((long)G * t / nt), (int)((long)G * (t + 1) / nt));
        draw(0, (int)((long)G / nt));
        for (auto& x : th) x.join();
    }
    P.on = false;                                       // consumed (or superseded): each prefetch serves one call
    STEP_TRACE("noise: gamma draws done (%d inline)", inline_games);
    bool any = false;
    for (int g = 0; g < G && !any; ++g) any = s->h_mask[g] != 0;
    if (!any) return 0;
    hipStream_t st = s->e->stream;
    HIPCHK(hipMemcpyAsync(s->d_noise, s->h_noise.data(), (size_t)G * NA * 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(s->d_mask, s->h_mask.data(), G, hipMemcpyHostToDevice, st));
    s->t.nd = s->arena[s->cur];
    hipLaunchKernelGGL(k_noise, dim3(G), dim3(64), 0, st, s->t, s->d_noise, s->d_mask, eps);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(st));
    return 0;
}

int search_run(az_search* s) {
    STEP_TRACE("search_run: root step");
    if (int r = search_step(s, MODE_ROOT_SEARCH)) return r;
    if (s->c.use_dirichlet_each_search)
        if (int r = search_noise(s, s->c.dirichlet_alpha, s->c.dirichlet_eps, nullptr)) return r;
    STEP_TRACE("search_run: sims");
    if (int r = search_sims(s, s->c.num_simulations)) return r;
    STEP_TRACE("search_run: check_err");
    const int r = check_err(s);
    STEP_TRACE("search_run: done");
    return r;
}

// (Re)start the listed slots with fresh games.  seed_ids (optional) give each game its own
// stream id for the evaluator / noise seeds (default: the slot index), so a game's record
// does not depend on which slot plays it.
int search_new_games(az_search* s, const int* games, int n, const int* seed_ids = nullptr) {
    if (n <= 0) return 0;
    hipStream_t st = s->e->stream;
    for (int i = 0; i < n; ++i)
        if (games[i] < 0 || games[i] >= s->c.n_games) return az_fail(AZ_ERR_ARG, "game index %d out of range", games[i]);
    HIPCHK(hipMemcpyAsync(s->d_games, games, n * 4, hipMemcpyHostToDevice, st));
    if (seed_ids) HIPCHK(hipMemcpyAsync(s->d_seed_ids, seed_ids, n * 4, hipMemcpyHostToDevice, st));
    s->t.nd = s->arena[s->cur];
    hipLaunchKernelGGL(k_new_games, dim3(n), dim3(64), 0, st, s->t, s->d_games, seed_ids ? s->d_seed_ids : nullptr, n,
                       s->c.eval_seed);
    hipLaunchKernelGGL(k_tt_clear, dim3(64, n), dim3(256), 0, st, s->t, s->d_games, n);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(st));
    for (int i = 0; i < n; ++i) {
        const int g = games[i];
        s->stones[g] = 0; s->active[g] = 1; s->fresh[g] = 1; s->ply[g] = 0;
        s->hist[g].clear();
        s->roots_ready = false;                          // a fresh root: unexpanded
        const int id = seed_ids ? seed_ids[i] : g;
        s->sp_next_id = std::max(s->sp_next_id, id + 1);
        pf_drop(s, g);
        s->rng[g].seed(s->c.noise_seed + (uint32_t)(s->c.noise_seed_stride * id));
    }
    return 0;
}

int search_select(az_search* s, int training, const float* temps_host, float T, int* actions, float* values, float* probs,
                  int* cact, int* nch) {
    hipStream_t st = s->e->stream;
    const int G = s->c.n_games, A = s->t.NA;     // child-order arrays are [G][NA]
    s->t.nd = s->arena[s->cur];
    if (temps_host) HIPCHK(hipMemcpyAsync(s->d_temps, temps_host, G * 4, hipMemcpyHostToDevice, st));
    TREE_DEV(dt, s, s->t);
    hipLaunchKernelGGL(k_select_action, dim3(G), dim3(64), 0, st, dt, training, T, temps_host ? s->d_temps : nullptr,
                       s->d_actions, s->d_values, s->d_probs, s->d_cact, s->d_nch);
    HIPCHK(hipGetLastError());
    if (actions) HIPCHK(hipMemcpyAsync(actions, s->d_actions, G * 4, hipMemcpyDeviceToHost, st));
    if (values) HIPCHK(hipMemcpyAsync(values, s->d_values, G * 4, hipMemcpyDeviceToHost, st));
    if (probs) HIPCHK(hipMemcpyAsync(probs, s->d_probs, (size_t)G * A * 4, hipMemcpyDeviceToHost, st));
    if (cact) HIPCHK(hipMemcpyAsync(cact, s->d_cact, (size_t)G * A * 4, hipMemcpyDeviceToHost, st));
    if (nch) HIPCHK(hipMemcpyAsync(nch, s->d_nch, G * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    return 0;
}

// makeMove + updateWithMove (device), then subtree compaction into the other arena.
int search_apply_dev(az_search* s, int* terminal, int* result) {
    hipStream_t st = s->e->stream;
    const int G = s->c.n_games;
    s->t.nd = s->arena[s->cur];
    std::vector<int> acts(G);
    HIPCHK(hipMemcpyAsync(acts.data(), s->d_actions, G * 4, hipMemcpyDeviceToHost, st));
    hipLaunchKernelGGL(k_apply, dim3(G), dim3(64), 0, st, s->t, s->d_actions, s->d_term, s->d_res, s->d_rexp);
    hipLaunchKernelGGL(k_compact, dim3(G), dim3(256), 0, st, s->t, s->arena[s->cur ^ 1], s->d_src_of);
    HIPCHK(hipGetLastError());
    s->cur ^= 1;
    s->t.nd = s->arena[s->cur];
    std::vector<int> term(G), res(G);
    HIPCHK(hipMemcpyAsync(term.data(), s->d_term, G * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(res.data(), s->d_res, G * 4, hipMemcpyDeviceToHost, st));
    std::vector<int> rexp(G);
    HIPCHK(hipMemcpyAsync(rexp.data(), s->d_rexp, G * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    bool ready = true;
    for (int g = 0; g < G; ++g) {
        if (s->active[g] && acts[g] >= (s->t.game == GAME_GO ? -1 : 0)) {
            s->hist[g].push_back(acts[g]);
            s->stones[g] += 1; s->ply[g] += 1; s->fresh[g] = 0;
            if (term[g]) s->active[g] = 0;
        }
        ready = ready && rexp[g] != 0;
    }
    s->roots_ready = ready;
    if (terminal) std::copy(term.begin(), term.end(), terminal);
    if (result) std::copy(res.begin(), res.end(), result);
    return check_err(s);
}

}  // namespace

// ===========================================================================
extern "C" {

const char* az_last_error(void) { return g_err.c_str(); }

int az_engine_create(int device, az_engine** out) {
    if (!out) return az_fail(AZ_ERR_ARG, "null out");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n <= 0) return az_fail(AZ_ERR_HIP, "no HIP device available (hipGetDeviceCount: %s)", hipGetErrorString(e));
    if (device < 0 || device >= n) return az_fail(AZ_ERR_ARG, "device %d out of range (%d devices)", device, n);
    auto* en = new az_engine();
    en->device = device;
    hipError_t r = hipSetDevice(device);
    if (r == hipSuccess) r = hipGetDeviceProperties(&en->prop, device);
    if (r == hipSuccess) r = hipStreamCreateWithFlags(&en->stream, hipStreamNonBlocking);
    if (r != hipSuccess) { delete en; return az_fail(AZ_ERR_HIP, "device init: %s", hipGetErrorString(r)); }
    *out = en;
    return 0;
}

void az_engine_destroy(az_engine* e) {
    if (!e) return;
    (void)hipSetDevice(e->device);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    delete e;
}

int az_engine_device_name(az_engine* e, char* buf, int len) {
    if (!e || !buf || len <= 0) return az_fail(AZ_ERR_ARG, "bad args");
    snprintf(buf, len, "%s (%s)", e->prop.name, e->prop.gcnArchName);
    return 0;
}

// ------------------------------------------------------------------ net
static int check_precision(const az_net_desc& d, int precision) {
    if (precision < 0 || precision > 4) return az_fail(AZ_ERR_ARG, "bad precision %d", precision);
    if (precision == AZ_PREC_F16X3) {
        // the fp16-piece kernels: conv3x3_v9x3 / v7x3 (8/9/13/15/19 boards, channels % 128 == 0) or
        // k_smallnet_x3 (15x15, 64 channels)
        const int H = d.board_size;
        // (the shape test of az_conv_v7x3_supported at the capacity, as x3_trunk applies it: the 32-bit
        // buffer ranges of the activations + their zeroed tail and of the weights)
        const size_t act_bytes = (size_t)d.max_batch * H * H * d.channels * 2;
        const bool trunk = (H == 8 || H == 9 || H == 13 || H == 15 || H == 19) && d.channels % 128 == 0 &&
                           act_bytes + AZ_ACT_TAIL * 2 < ((size_t)1 << 31) &&
                           (size_t)9 * d.channels * d.channels * 2 < ((size_t)1 << 31);
        const bool small = az_smallnet_supported(H, d.channels, (d.in_planes + 15) / 16 * 16, d.pool, d.head_channels) &&
                           d.blocks <= az_smallnet_max_blocks();
        if (!trunk && !small && d.blocks > 0)
            return az_fail(AZ_ERR_ARG, "AZ_PREC_F16X3 needs an 8/9/13/15/19 board with channels %% 128 == 0 (and under 2 GiB "
                                    "per activation buffer), or the 15x15 64-channel net; use AZ_PREC_BF16X3 or AZ_PREC_F32");
    }
    if (precision != AZ_PREC_F32 && d.channels % 32) return az_fail(AZ_ERR_ARG, "bf16/fp16 trunk needs channels %% 32 == 0");
    if (precision == AZ_PREC_FP16 && !az_conv_v4_supported(d.board_size, d.board_size, d.channels, d.channels) &&
        !az_conv_g8_supported(d.board_size, d.board_size, d.channels, d.channels))
        return az_fail(AZ_ERR_ARG, "AZ_PREC_FP16 trunk needs 15x15 boards and channels %% 64 == 0, or an 8/9/13/15/19 board "
                                "and channels %% 128 == 0");
    return 0;
}

static int net_create(az_engine* e, const az_net_desc* d, az_net** out, bool rw,
                      const std::vector<azrw::Plan>* plans = nullptr) {
    if (!e || !d || !out) return az_fail(AZ_ERR_ARG, "null argument");
    if (d->board_size < 2 || d->board_size * d->board_size > AZ_MAXA || d->in_planes < 1 || d->in_planes > 128 ||
        d->channels < 4 || d->channels % 4 || d->blocks < 0 || d->action_size < 1 || d->action_size > 8192 ||
        d->head_channels < 1 || d->head_channels % 4 || d->pool < 1 || d->fc_hidden < 1 || d->fc_hidden % 4 ||
        d->max_batch < 1)
        return az_fail(AZ_ERR_ARG, "unsupported network description");
    if (int r = check_precision(*d, d->precision)) return r;
    std::lock_guard<std::mutex> lk(e->mu);
    HIPCHK(hipSetDevice(e->device));
    auto* n = new az_net();
    n->e = e;
    n->d = *d;
    n->HW = d->board_size * d->board_size;
    n->P2 = d->pool * d->pool;
    // input channels padded to 16 (the search's plane records); more than 16 planes on a g8 board
    // pad to 32 so the v6 conv takes the input layer as whole 32-channel chunks
    n->cin_pad = (d->in_planes + 15) / 16 * 16;
    if (n->cin_pad > 16 && d->channels % 128 == 0) n->cin_pad = (d->in_planes + 31) / 32 * 32;
    n->rw = rw;
    if (rw) {
        n->rwb.resize(d->blocks);
        for (int i = 0; i < d->blocks; ++i) {
            n->rwb[i].plan = plans ? (*plans)[i] : azrw::plan(i);
            n->rwb[i].node.resize(n->rwb[i].plan.preds.size());
        }
        n->nparams = 0;
        for (const PSpec& ps : rw_spec(*d, n->rwb)) n->nparams += ps.n;
    } else {
        n->nparams = count_params(*d);
    }
    const size_t B = d->max_batch, rows = B * n->HW, F = d->channels;
    n->act_elems = rows * F;
    int r = 0;
    auto A_ = [&](float** p, size_t cnt) {
        if (!r) r = dalloc(p, cnt);
        if (!r) n->scratch.emplace_back((void*)*p, cnt * 4);
    };
    // 16-bit activation planes carry a zeroed tail (AZ_ACT_TAIL elements): the v6 conv points the
    // DMA of halo padding rows there
    auto H_ = [&](uint16_t** p, size_t cnt) {
        if (!r) r = dalloc(p, cnt + AZ_ACT_TAIL);
        if (!r && hipMemset(*p + cnt, 0, AZ_ACT_TAIL * 2) != hipSuccess) r = az_fail(AZ_ERR_HIP, "hipMemset");
        if (!r) n->scratch.emplace_back((void*)*p, cnt * 2);
    };
    A_(&n->x0, rows * n->cin_pad);
    A_(&n->h0, rows * F); A_(&n->h1, rows * F); A_(&n->t, rows * F);
    if (F % 32 == 0) {
        H_(&n->hh[0], rows * F); H_(&n->hh[1], rows * F); H_(&n->hl[0], rows * F); H_(&n->hl[1], rows * F);
        H_(&n->th, rows * F); H_(&n->tl, rows * F);
    }
    A_(&n->pool, B * n->P2 * F);
    A_(&n->pp, B * n->P2 * d->head_channels); A_(&n->vp, B * n->P2 * d->head_channels);
    A_(&n->hpv, B * n->P2 * 2 * d->head_channels);
    A_(&n->v1, B * d->fc_hidden);
    {   // split-K workspace: gemm_f32 partials, or k_fc_heads' [<= 16 slices][B padded to 64][64-column tiles]
        const size_t nc = (size_t)((d->action_size + 63) / 64 + (d->fc_hidden + 63) / 64) * 64;
        A_(&n->ws, std::max((size_t)B * (d->action_size + d->fc_hidden) * FC_MAX_SPLITS, 16 * ((size_t)B + 63) / 64 * 64 * nc));
    }
    A_(&n->logits, B * d->action_size); A_(&n->value, B); A_(&n->soft, B * d->action_size);
    A_(&n->in_nchw, B * d->in_planes * n->HW);
    if (rw) {
        size_t nodes = 0;
        for (const RwBlock& blk : n->rwb) nodes = std::max(nodes, blk.node.size());
        n->rw_out.assign(nodes, nullptr);
        for (float*& p : n->rw_out) A_(&p, rows * F);
        A_(&n->rw_t2, rows * F); A_(&n->rw_in, rows * F);
        // Small capacities leave most CUs idle (one 128 x 128 f32 tile of a K = 9F conv is ~60 us
        // of one CU): split K so the node convs cover the chip.  Chosen from max_batch, so a
        // board's summation order never depends on the batch it arrives in.
        {
            const int bn = F <= 64 ? 64 : 128, nk = (int)((9 * F + 31) / 32);
            const long tiles = (long)((rows + 127) / 128) * (long)((F + bn - 1) / bn);
            while (n->rw_splits < 8 && tiles * n->rw_splits < 256 && nk / (2 * n->rw_splits) >= 4) n->rw_splits *= 2;
            if (n->rw_splits > 1) A_(&n->rw_ws, (size_t)n->rw_splits * rows * F);
        }
        // routers read their inputs straight from the node buffers: per router a device table
        auto table = [&](const std::vector<int>& ids, const float*** dst) {
            if (r || ids.size() < 2) return;
            std::vector<const float*> t;
            for (int u : ids) t.push_back(n->rw_out[u]);
            if (hipMalloc((void**)dst, t.size() * sizeof(float*)) != hipSuccess ||
                hipMemcpy((void*)*dst, t.data(), t.size() * sizeof(float*), hipMemcpyHostToDevice) != hipSuccess)
                r = az_fail(AZ_ERR_OOM, "router input table");
        };
        for (RwBlock& blk : n->rwb) {
            for (size_t v = 0; v < blk.node.size(); ++v) table(blk.plan.preds[v], &blk.node[v].ins);
            table(blk.plan.outputs, &blk.outs);
        }
    }
    if (!r) r = dalloc(&n->d_nb, 1);
    if (!r) r = dalloc(&n->ovf, 1);
    if (!r && hipMemset(n->ovf, 0, 4) != hipSuccess) r = az_fail(AZ_ERR_HIP, "memset");
    if (!r) r = dalloc(&n->zero, 128);
    if (!r && hipMemset(n->zero, 0, 256) != hipSuccess) r = az_fail(AZ_ERR_HIP, "memset");
    // the memsets above run on the null stream, the forwards on the engine's non-blocking stream,
    // which does not wait for it: finish them here
    if (!r && hipDeviceSynchronize() != hipSuccess) r = az_fail(AZ_ERR_HIP, "hipDeviceSynchronize");
    if (r) { az_net_destroy(n); return r; }
    *out = n;
    return 0;
}

int az_net_create(az_engine* e, const az_net_desc* d, az_net** out) { return net_create(e, d, out, false); }

// Rand-wire precisions: AZ_PREC_F32 (the reference module's arithmetic, any shape), or on 15x15
// with channels % 64 == 0 the conv3x3_v4 node convs: AZ_PREC_BF16X3 (fp32-faithful split operands,
// fp32 routers) or AZ_PREC_FP16 (fp16 operands, fp16-operand routers); SE and the residual stream
// stay fp32 in every mode.
static int check_rw_precision(const az_net_desc& d, int precision) {
    if (precision == AZ_PREC_F32) return 0;
    if ((precision == AZ_PREC_FP16 || precision == AZ_PREC_BF16X3) &&
        az_conv_v4_supported(d.board_size, d.board_size, d.channels, d.channels))
        return 0;
    return az_fail(AZ_ERR_ARG, "rand-wire nets: AZ_PREC_F32, or AZ_PREC_BF16X3 / AZ_PREC_FP16 on 15x15 with channels %% 64 == 0");
}

// Every rand-wire create path: the precision, then the shapes the node kernels assume
// (k_se_residual: C % 16 == 0 for its float4 channel quads, C <= 1024 and R = C / 16 <= 64 for
// its fixed LDS arrays; no conv bias; the reference's adaptive pool to min(8, board)).
static int check_rw_desc(const az_net_desc& d) {
    if (int r = check_rw_precision(d, d.precision)) return r;
    if (d.conv_bias) return az_fail(AZ_ERR_ARG, "rand-wire convolutions carry no bias (conv_bias = 0)");
    if (d.channels < 16 || d.channels % 16 || d.channels > 1024)
        return az_fail(AZ_ERR_ARG, "rand-wire channels: a multiple of 16 in [16, 1024]");
    if (d.pool != std::min(8, d.board_size)) return az_fail(AZ_ERR_ARG, "rand-wire heads pool to min(8, board)");
    return 0;
}

int az_net_create_randwire(az_engine* e, const az_net_desc* d, az_net** out) {
    if (!d) return az_fail(AZ_ERR_ARG, "null argument");
    if (int r = check_rw_desc(*d)) return r;
    return net_create(e, d, out, true);
}

// Explicit wiring (e.g. the Python DDWRandWireResNet's networkx graphs, python/alphazero/models/
// ddw_randwire.py:56-116): per block  n, order[n], then for node v = 0..n-1: deg_v, preds[deg_v],
// then n_out, outputs[n_out].  Inputs are the in-degree-0 nodes in `order`; the compute order is
// any topological order (a node's output depends only on its inputs).
int az_net_create_randwire_graphs(az_engine* e, const az_net_desc* d, const int* g, size_t n_ints, az_net** out) {
    if (!d || !g) return az_fail(AZ_ERR_ARG, "null argument");
    if (int r = check_rw_desc(*d)) return r;
    std::vector<azrw::Plan> plans(std::max(0, d->blocks));
    size_t k = 0;
    auto next = [&](int& v) { if (k >= n_ints) return false; v = g[k++]; return true; };
    for (int b = 0; b < d->blocks; ++b) {
        azrw::Plan& pl = plans[b];
        int n = 0;
        if (!next(n) || n < 1 || n > 1024) return az_fail(AZ_ERR_ARG, "block %d: bad node count", b);
        pl.order.resize(n);
        std::vector<char> seen(n, 0);
        for (int& v : pl.order) {
            if (!next(v) || v < 0 || v >= n || seen[v]) return az_fail(AZ_ERR_ARG, "block %d: order is not a permutation", b);
            seen[v] = 1;
        }
        pl.preds.assign(n, {});
        std::vector<int> indeg(n, 0);
        std::vector<std::vector<int>> succ(n);
        for (int v = 0; v < n; ++v) {
            int deg = 0;
            if (!next(deg) || deg < 0 || deg > 64) return az_fail(AZ_ERR_ARG, "block %d node %d: bad degree", b, v);
            for (int j = 0; j < deg; ++j) {
                int u = 0;
                if (!next(u) || u < 0 || u >= n) return az_fail(AZ_ERR_ARG, "block %d node %d: bad predecessor", b, v);
                pl.preds[v].push_back(u);
                succ[u].push_back(v);
            }
            indeg[v] = deg;
        }
        int no = 0;
        if (!next(no) || no < 1 || no > n) return az_fail(AZ_ERR_ARG, "block %d: bad output count", b);
        pl.outputs.resize(no);
        for (int& v : pl.outputs)
            if (!next(v) || v < 0 || v >= n) return az_fail(AZ_ERR_ARG, "block %d: bad output node", b);
        for (int v : pl.order)
            if (pl.preds[v].empty()) pl.inputs.push_back(v);
        std::vector<int> q = pl.inputs;   // Kahn over `order`
        for (size_t h = 0; h < q.size(); ++h)
            for (int w : succ[q[h]])
                if (--indeg[w] == 0) q.push_back(w);
        if ((int)q.size() != n) return az_fail(AZ_ERR_ARG, "block %d: the wiring has a cycle", b);
        pl.topo = q;
    }
    if (k != n_ints) return az_fail(AZ_ERR_ARG, "graph description: %zu ints read, %zu given", k, n_ints);
    return net_create(e, d, out, true, &plans);
}

int az_randwire_graph(int block, int* order, int* topo, int* inputs, int* n_inputs, int* outputs, int* n_outputs,
                      int* pred_off, int* preds, int preds_cap) {
    if (block < 0 || !order || !topo || !inputs || !n_inputs || !outputs || !n_outputs || !pred_off || !preds)
        return az_fail(AZ_ERR_ARG, "null argument / negative block");
    const azrw::Plan pl = azrw::plan(block);
    const int nn = (int)pl.order.size();
    std::copy(pl.order.begin(), pl.order.end(), order);
    std::copy(pl.topo.begin(), pl.topo.end(), topo);
    std::copy(pl.inputs.begin(), pl.inputs.end(), inputs);
    std::copy(pl.outputs.begin(), pl.outputs.end(), outputs);
    *n_inputs = (int)pl.inputs.size();
    *n_outputs = (int)pl.outputs.size();
    int k = 0;
    for (int v = 0; v < nn; ++v) {
        pred_off[v] = k;
        for (int u : pl.preds[v]) {
            if (k >= preds_cap) return az_fail(AZ_ERR_CAPACITY, "preds_cap %d too small", preds_cap);
            preds[k++] = u;
        }
    }
    pred_off[nn] = k;
    return 0;
}

void az_net_destroy(az_net* n) {
    if (!n) return;
    (void)hipSetDevice(n->e->device);
    auto F = [](void* p) { if (p) (void)hipFree(p); };
    std::vector<Layer*> ls = {&n->in, &n->in32, &n->pconv, &n->vconv, &n->hconv, &n->pfc, &n->vfc1, &n->vfc2};
    for (auto& l : n->blk) ls.push_back(&l);
    for (auto& blk : n->rwb) {
        ls.push_back(&blk.out_router);
        F((void*)blk.outs);
        for (auto& nd : blk.node) {
            ls.push_back(&nd.router); ls.push_back(&nd.c1); ls.push_back(&nd.c2);
            F(nd.w1); F(nd.b1); F(nd.w2); F(nd.b2); F((void*)nd.ins);
        }
    }
    for (float* p : n->rw_out) F(p);
    F(n->rw_t2); F(n->rw_in); F(n->rw_ws);
    for (Layer* l : ls) { F(l->W); F(l->b); F(l->Whi); F(l->Wlo); F(l->Wh16); F(l->Wbk_bf); F(l->Wbk_h); F(l->Wbk_lo);
                          F(l->Wbk_fh); F(l->Wbk_fl); F(l->bx); F(l->sx); }
    for (void* p : {(void*)n->x0, (void*)n->h0, (void*)n->h1, (void*)n->t, (void*)n->pool, (void*)n->pp, (void*)n->vp, (void*)n->hpv,
                    (void*)n->v1, (void*)n->ws, (void*)n->logits, (void*)n->value, (void*)n->soft, (void*)n->in_nchw, (void*)n->d_nb, (void*)n->ovf,
                    (void*)n->hh[0], (void*)n->hh[1], (void*)n->hl[0], (void*)n->hl[1], (void*)n->th, (void*)n->tl,
                    (void*)n->zero, (void*)n->sm_W, (void*)n->sm_Wf, (void*)n->sm_Wxh, (void*)n->sm_Wxl, (void*)n->sm_b, (void*)n->fcx_hi, (void*)n->fcx_lo, (void*)n->fcf_hi, (void*)n->fcf_lo, (void*)n->fcf_rs,
                    (void*)n->sm_Wfh, (void*)n->sm_Wfl, (void*)n->sm_bx, (void*)n->sm_sx})
        F(p);
    n->pc.release();
    delete n;
}

int az_net_num_params(az_net* n, size_t* count) {
    if (!n || !count) return az_fail(AZ_ERR_ARG, "null argument");
    *count = n->nparams;
    return 0;
}

int az_net_load_weights(az_net* n, const float* blob, size_t count) {
    if (!n || !blob) return az_fail(AZ_ERR_ARG, "null argument");
    if (count != n->nparams) return az_fail(AZ_ERR_ARG, "expected %zu parameters, got %zu", n->nparams, count);
    std::lock_guard<std::mutex> lk(n->mu);
    HIPCHK(hipSetDevice(n->e->device));
    {
        // the first load allocates the weight buffers: record them (net_weight_buffers)
        WeightRegistry reg(n->wbufs.empty() ? &n->wbufs : nullptr);
        if (int r = n->rw ? net_load_rw(n, blob) : net_load(n, blob)) return r;
    }
    HIPCHK(hipDeviceSynchronize());   // null-stream uploads done before the non-blocking stream reads them
    n->host_blob.assign(blob, blob + count);
    return 0;
}

}  // extern "C"
// ---- net internals for dist.hip (engine_internal.h), C++ linkage
int net_weight_buffers(az_net* n, std::vector<std::pair<void*, size_t>>& out) {
    if (n->wbufs.empty()) {
        // never loaded: a load of zero weights allocates (and records) every weight buffer, which a
        // broadcast then overwrites (host work once per net, no device traffic beyond the uploads)
        std::vector<float> zero(n->nparams, 0.0f);
        WeightRegistry reg(&n->wbufs);
        if (int r = n->rw ? net_load_rw(n, zero.data()) : net_load(n, zero.data())) return r;
        HIPCHK(hipDeviceSynchronize());
        n->loaded = false;
    }
    out = n->wbufs;
    return 0;
}
const std::vector<float>& net_host_blob(az_net* n) { return n->host_blob; }
size_t net_param_count(az_net* n) { return n->nparams; }
az_engine* net_engine(az_net* n) { return n->e; }
std::mutex& net_mutex(az_net* n) { return n->mu; }
void net_adopt_blob(az_net* n, const float* blob) {
    n->host_blob.assign(blob, blob + n->nparams);
    n->loaded = true;
}
extern "C" {

int az_net_get_weights(az_net* n, float* blob, size_t count) {
    if (!n || !blob) return az_fail(AZ_ERR_ARG, "null argument");
    std::lock_guard<std::mutex> lk(n->mu);
    if (!n->loaded) return az_fail(AZ_ERR_STATE, "weights not loaded");
    if (count != n->nparams) return az_fail(AZ_ERR_ARG, "expected %zu parameters, got %zu", n->nparams, count);
    std::copy(n->host_blob.begin(), n->host_blob.end(), blob);
    return 0;
}

// Counter-based init; tests/nn_weights.py restates it in numpy (same fp32 ops).
int az_net_init_random(az_net* n, uint64_t seed) {
    if (!n) return az_fail(AZ_ERR_ARG, "null net");
    const az_net_desc& d = n->d;
    std::vector<float> blob(n->nparams);
    size_t off = 0;
    int tensor = 0;
    auto fill = [&](size_t cnt, int kind, int fan_in) {
        // kind: 0 weight U(-1,1)/sqrt(fan_in); 1 bias U(-1,1)/sqrt(fan_in); 2 bn gamma 1+0.1u;
        //       3 bn beta 0.1u; 4 bn mean 0.1u; 5 bn var 1+0.25(u+1)
        const float bound = 1.0f / std::sqrt((float)fan_in);
        for (size_t i = 0; i < cnt; ++i) {
            const uint64_t r = splitmix64(seed ^ ((uint64_t)tensor << 40) ^ (uint64_t)i);
            const float u = (float)(int32_t)(r >> 40) * (1.0f / 8388608.0f) - 1.0f;
            float v;
            switch (kind) {
                case 0: case 1: v = u * bound; break;
                case 2: v = 1.0f + 0.1f * u; break;
                case 3: case 4: v = 0.1f * u; break;
                default: v = 1.0f + 0.25f * (u + 1.0f); break;
            }
            blob[off + i] = v;
        }
        off += cnt;
        ++tensor;
    };
    if (n->rw) {
        for (const PSpec& ps : rw_spec(d, n->rwb)) fill(ps.n, ps.kind, ps.fan_in);
        if (off != n->nparams) return az_fail(AZ_ERR_STATE, "init size mismatch");
        return az_net_load_weights(n, blob.data(), blob.size());
    }
    const int F = d.channels, HC = d.head_channels, PP = d.pool * d.pool;
    auto conv = [&](int co, int ci, int k) {
        fill((size_t)co * ci * k * k, 0, ci * k * k);
        if (d.conv_bias) fill(co, 1, ci * k * k);
        fill(co, 2, 1); fill(co, 3, 1); fill(co, 4, 1); fill(co, 5, 1);
    };
    conv(F, d.in_planes, 3);
    for (int i = 0; i < d.blocks; ++i) { conv(F, F, 3); conv(F, F, 3); }
    conv(HC, F, 1);
    fill((size_t)d.action_size * HC * PP, 0, HC * PP); fill(d.action_size, 1, HC * PP);
    conv(HC, F, 1);
    fill((size_t)d.fc_hidden * HC * PP, 0, HC * PP); fill(d.fc_hidden, 1, HC * PP);
    fill(d.fc_hidden, 0, d.fc_hidden); fill(1, 1, d.fc_hidden);
    if (off != n->nparams) return az_fail(AZ_ERR_STATE, "init size mismatch");
    return az_net_load_weights(n, blob.data(), blob.size());
}

int az_net_set_precision(az_net* n, int precision) {
    if (!n) return az_fail(AZ_ERR_ARG, "null net");
    if (n->rw && check_rw_precision(n->d, precision)) return AZ_ERR_ARG;
    if (int r = check_precision(n->d, precision)) return r;
    n->d.precision = precision;
    return 0;
}

static int net_host_forward(az_net* n, const float* planes, int B, float* logits, float* value, bool soft) {
    if (!n || !planes || B < 1 || B > n->d.max_batch) return az_fail(AZ_ERR_ARG, "bad batch (1..%d)", n ? n->d.max_batch : 0);
    if (!n->loaded) return az_fail(AZ_ERR_STATE, "weights not loaded");
    std::lock_guard<std::mutex> lk(n->mu);
    HIPCHK(hipSetDevice(n->e->device));
    hipStream_t st = n->e->stream;
    const int A = n->d.action_size;
    if (int r = poison_net(n, st, true)) return r;
    HIPCHK(hipMemcpyAsync(n->in_nchw, planes, (size_t)B * n->d.in_planes * n->HW * 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(n->d_nb, &B, 4, hipMemcpyHostToDevice, st));
    az_launch_pack_input(n->in_nchw, n->x0, B, n->d.in_planes, n->HW, n->cin_pad, st);
    if (int r = net_forward(n, n->x0, B, n->d_nb, n->logits, n->value, st)) return r;
    const float* pol = n->logits;
    if (soft) { az_launch_softmax_rows(n->logits, n->soft, B, A, st); pol = n->soft; }
    HIPCHK(hipGetLastError());
    if (logits) HIPCHK(hipMemcpyAsync(logits, pol, (size_t)B * A * 4, hipMemcpyDeviceToHost, st));
    if (value) HIPCHK(hipMemcpyAsync(value, n->value, (size_t)B * 4, hipMemcpyDeviceToHost, st));
    int ovf = 0;
    HIPCHK(hipMemcpyAsync(&ovf, n->ovf, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    return check_ovf(n, ovf);
}

int az_net_trunk_kernel(az_net* n, char* name, int len) {
    if (!n || !name || len < 1) return az_fail(AZ_ERR_ARG, "null net / name");
    const az_net_desc& d = n->d;
    const int prec = d.precision, F = d.channels, H = d.board_size;
    const bool bf = (prec == AZ_PREC_BF16X3 || prec == AZ_PREC_F16X3 || prec == AZ_PREC_BF16 || prec == AZ_PREC_FP16) &&
                    F % 32 == 0;
    const bool f16 = prec == AZ_PREC_FP16;
    if (n->rw) {
        const bool v4x3 = prec == AZ_PREC_BF16X3 && d.max_batch >= 128;   // as rw_trunk dispatches
        snprintf(name, len, f16 ? "conv3x3_v4<2, 128, 1>" : v4x3 ? "conv3x3_v4<0, 128, 0>" : "gemm_f32");
        return 0;
    }
    if (!bf || d.blocks < 1) { snprintf(name, len, "gemm_f32"); return 0; }
    if ((f16 || prec == AZ_PREC_BF16X3 || prec == AZ_PREC_F16X3) && az_smallnet_supported(H, F, n->cin_pad, d.pool, d.head_channels) &&
        d.blocks <= az_smallnet_max_blocks()) {
        if (f16) snprintf(name, len, "k_smallnet_g<%d, 8, %s>", H, d.residual ? "true" : "false");   // as rocprofv3 names it
        else snprintf(name, len, "k_smallnet_x3<%d, 8, %s, %d>", H, d.residual ? "true" : "false", prec == AZ_PREC_F16X3 ? 2 : 1);
        return 0;
    }
    // the trunk's second conv of a block, as net_forward builds it at the net's capacity
    ConvBf16Args a{};
    a.M = d.max_batch * n->HW; a.N = F; a.C = F; a.H = H; a.W = H; a.rows_per_sample = n->HW; a.relu = 1;
    a.a_tail = n->act_elems * 2;
    if (x3_trunk(n)) {
        Layer probe;
        probe.Wbk_bf = probe.Wbk_lo = probe.Wbk_fh = probe.Wbk_fl = n->zero;
        probe.sx = reinterpret_cast<float*>(n->zero);
        return az_conv_x3_name(x3_conv_args(n, probe, 1, 0, d.max_batch, nullptr), name, len) ? az_fail(AZ_ERR_ARG, "x3 name") : 0;
    }
    if (prec == AZ_PREC_F16X3) return az_fail(AZ_ERR_ARG, "AZ_PREC_F16X3: no fp16-piece trunk for this net");
    const bool g8 = prec != AZ_PREC_BF16X3 && az_conv_g8_supported(H, H, F, F);
    const int r = g8 ? az_conv_g8_name(a, f16 ? 2 : 1, name, len)
                     : az_conv_bf16_name(a, f16 ? 2 : prec == AZ_PREC_BF16X3 ? 0 : 1, name, len);
    return r ? az_fail(AZ_ERR_ARG, "no trunk kernel for this net") : 0;
}

int az_net_profile(az_net* n, int enable) {
    if (!n) return az_fail(AZ_ERR_ARG, "null net");
    std::lock_guard<std::mutex> lk(n->mu);
    n->prof = enable != 0;
    if (n->prof && !n->pc.d) {
        HIPCHK(hipSetDevice(n->e->device));
        if (hipMalloc((void**)&n->pc.d, ProfClock::CAP * 8) != hipSuccess) { n->pc.d = nullptr; return az_fail(AZ_ERR_OOM, "profile clock buffer"); }
    }
    n->pc.used = 0; n->prof_launches = 0; n->prof_forwards = 0; n->prof_tick = 0; n->prof_sampled = 0;
    return 0;
}

int az_net_profile_read(az_net* n, double* trunk_ms, int64_t* trunk_launches, int64_t* forwards) {
    if (!n) return az_fail(AZ_ERR_ARG, "null net");
    std::lock_guard<std::mutex> lk(n->mu);
    HIPCHK(hipSetDevice(n->e->device));
    HIPCHK(hipStreamSynchronize(n->e->stream));
    double ms = 0.0;
    const std::vector<double> t = n->pc.read_ms();
    for (size_t i = 0; i + 1 < t.size(); i += 2) ms += t[i + 1] - t[i];
    // the sampled forwards' trunk time scaled to every profiled forward
    if (trunk_ms) *trunk_ms = n->prof_sampled ? ms * (double)n->prof_forwards / (double)n->prof_sampled : 0.0;
    if (trunk_launches) *trunk_launches = n->prof_launches;
    if (forwards) *forwards = n->prof_forwards;
    return 0;
}

int az_net_forward(az_net* n, const float* planes, int B, float* logits, float* value) {
    return net_host_forward(n, planes, B, logits, value, false);
}

int az_net_predict_batch(az_net* n, const float* planes, int B, float* policy, float* value) {
    return net_host_forward(n, planes, B, policy, value, true);
}

// ------------------------------------------------------------------ search
int az_search_create(az_engine* e, az_net* net, const az_search_cfg* c, az_search** out) {
    if (!e || !c || !out) return az_fail(AZ_ERR_ARG, "null argument");
    const int bs = c->board_size, A = bs * bs, G = c->n_games;
    const bool go = c->game == AZ_GAME_GO;
    const int NA = go ? A + 1 : A;
    if (bs < 3 || A > AZ_MAXA || G < 1 || c->num_simulations < 0 || c->virtual_loss < 0 || c->tt_log2 < 4 ||
        c->tt_log2 > 24 || c->eval_kind < 0 || c->eval_kind > 4 || (c->game != AZ_GAME_GOMOKU && !go))
        return az_fail(AZ_ERR_ARG, "unsupported search configuration");
    if (go && bs != 9 && bs != 13 && bs != 19)
        return az_fail(AZ_ERR_ARG, "Go board %d: GoState supports 9, 13 and 19 (go_state.cpp:24-26)", bs);
    if (c->eval_kind == AZ_EVAL_NET) {
        if (!net) return az_fail(AZ_ERR_ARG, "AZ_EVAL_NET needs a network");
        if (net->d.board_size != bs || net->d.action_size != NA || net->d.in_planes != (go ? 8 : 11))
            return az_fail(AZ_ERR_ARG, "network shape does not match the board");
        if (net->d.max_batch < G) return az_fail(AZ_ERR_ARG, "network max_batch %d < n_games %d", net->d.max_batch, G);
        if (!net->loaded) return az_fail(AZ_ERR_STATE, "network weights not loaded");
    }
    if (c->prior_ring > 0 && c->prior_ring < NA)
        return az_fail(AZ_ERR_ARG, "prior_ring %d is smaller than one policy (%d entries)", c->prior_ring, NA);
    std::lock_guard<std::mutex> lk(e->mu);
    HIPCHK(hipSetDevice(e->device));
    auto* s = new az_search();
    s->e = e; s->net = net; s->c = *c;
    const int ncap = c->node_capacity > 0 ? c->node_capacity : 3 * std::max(64, c->num_simulations) * NA + 8 * NA + 64;
    const int ring = c->prior_ring > 0 ? c->prior_ring : std::max(1 << 16, 12 * std::max(64, c->num_simulations) * NA);
    s->c.node_capacity = ncap; s->c.prior_ring = ring;
    TreeDev& t = s->t;
    t.G = G; t.bs = bs; t.A = A; t.ncap = ncap; t.game = go ? GAME_GO : GAME_GOMOKU; t.NA = NA;
    t.hmax = go ? 2048 : 0; t.vl = c->virtual_loss; t.cpuct = c->c_puct; t.fpu = c->fpu_reduction;
    t.eval_kind = c->eval_kind; t.tt_slots = 1 << c->tt_log2; t.tt_mask = (uint64_t)t.tt_slots - 1; t.ring = ring;
    t.log_game = -1; t.log_cap = 0;
    t.stamp_game = g_tree_stamp_game;   // diagnostic phase stamps (az_diag_set_tree_stamps)
    const size_t NG = (size_t)G * ncap;
    int r = 0;
#define SA(p, n) do { if (!r) r = dalloc(&(p), (size_t)(n)); } while (0)
    for (int k = 0; k < 2; ++k) {
        Nodes& nd = s->arena[k];
        SA(nd.N, NG); SA(nd.W, NG); SA(nd.VL, NG); SA(nd.P, NG); SA(nd.first, NG); SA(nd.act, NG); SA(nd.cnt, NG);
        SA(nd.flag, NG);
    }
    SA(t.atop, G); SA(t.rboard, (size_t)G * A); SA(t.rhist, G * 6); SA(t.rplayer, G); SA(t.rstones, G); SA(t.rply, G);
    SA(t.rhash, G); SA(t.rfresh, G); SA(t.rnode, G); SA(t.active, G); SA(t.gresult, G);
    uint64_t* zko = nullptr;
    if (go) { SA(t.rko, G); SA(t.rpass, G); SA(t.rposh, (size_t)G * t.hmax); SA(t.rnposh, G); SA(zko, A + 1); }
    SA(t.path, (size_t)G * AZ_DMAX); SA(t.pact, (size_t)G * AZ_DMAX); SA(t.pstat, (size_t)G * AZ_DMAX); SA(t.rhdr, G); SA(t.plen, G); SA(t.lstatus, G); SA(t.lvalue, G); SA(t.lhash, G); SA(t.ttstore, G);
    SA(t.ttref, G); SA(t.tthslot, G); SA(t.need_eval, G); SA(t.eval_slot, G); SA(t.eval_games, G); SA(t.n_eval, 1);
    SA(t.leafrec, (size_t)G * AZ_REC_BYTES);
    if (t.game == GAME_GO) SA(t.goleaf, (size_t)G * AZ_GOLEAF_BYTES);
    SA(t.tt_hash, (size_t)G * t.tt_slots); SA(t.tt_visits, (size_t)G * t.tt_slots); SA(t.tt_value, (size_t)G * t.tt_slots);
    SA(t.tt_ref, (size_t)G * t.tt_slots);
    SA(t.ring_buf, (size_t)G * ring); SA(t.ring_cur, G); SA(t.cnt, (size_t)G * AZ_NCNT);
    if (!r) r = hipMemset(t.cnt, 0, (size_t)G * AZ_NCNT * 8) == hipSuccess ? 0 : az_fail(AZ_ERR_HIP, "memset");
    uint64_t* zp = nullptr; uint64_t* zpl = nullptr; int* fo = nullptr;
    SA(zp, 2 * A); SA(zpl, 2); SA(fo, A);
    if (c->eval_kind == AZ_EVAL_RANDOM) SA(t.mt, (size_t)G * 625);
    SA(t.err, 1);
    SA(s->d_src_of, NG);
    if (c->eval_kind == AZ_EVAL_NET || c->eval_kind == AZ_EVAL_CALLBACK) {
        SA(s->d_batch, (size_t)G * A * 16); SA(s->d_logits, (size_t)G * NA); SA(s->d_value, G);
    }
    if (c->eval_kind == AZ_EVAL_NET) SA(s->d_id, G + 1);
    if (c->eval_kind == AZ_EVAL_CALLBACK) { SA(s->d_lmoves, (size_t)G * AZ_DMAX); SA(s->d_llen, G); }
    SA(s->d_noise, (size_t)G * NA); SA(s->d_mask, G); SA(s->d_actions, G); SA(s->d_values, G); SA(s->d_probs, (size_t)G * NA);
    SA(s->d_cact, (size_t)G * NA); SA(s->d_nch, G); SA(s->d_term, G); SA(s->d_res, G); SA(s->d_rexp, G); SA(s->d_games, G); SA(s->d_seed_ids, G); SA(s->d_temps, G);
    SA(s->d_rc, 4 * (size_t)NA + 8); SA(s->d_rcf, 2 * (size_t)NA + 4); SA(s->d_thr, G); SA(s->d_pruned, G);
#undef SA
    if (r) { az_search_destroy(s); return r; }
    t.zpiece = zp; t.zplayer = zpl; t.fresh_order = fo; t.zko = zko;
    if (s->d_id) {
        std::vector<int> id(G + 1);
        for (int i = 0; i <= G; ++i) id[i] = i;
        HIPCHK(hipMemcpy(s->d_id, id.data(), (G + 1) * 4, hipMemcpyHostToDevice));
    }
    if (go) {
        // GoState Zobrist features (go_state.cpp:48-51; ZobristHash::addFeature, zobrist_hash.cpp:58-70):
        // mt19937_64 seeded with std::hash<std::string> of the feature name
        std::mt19937_64 rk(std::hash<std::string>{}("ko_point"));
        std::vector<uint64_t> ko(A + 1);
        for (auto& k : ko) k = rk();
        HIPCHK(hipMemcpy(zko, ko.data(), (A + 1) * 8, hipMemcpyHostToDevice));
        std::mt19937_64 rr(std::hash<std::string>{}("rules"));
        uint64_t rules[2] = {rr(), rr()};
        std::mt19937_64 rm(std::hash<std::string>{}("komi"));
        uint64_t komi[16];
        for (auto& k : komi) k = rm();
        t.zconst = rules[1] ^ komi[((int)(7.5f * 2)) & 0xF];   // Chinese rules, komi 7.5
    }
    t.net_logits = s->d_logits; t.net_value = s->d_value;
    // Zobrist keys: ZobristHash(bs, 2, 2, seed) (src/core/zobrist_hash.cpp:9-36)
    {
        std::mt19937_64 rng(c->zobrist_seed);
        std::vector<uint64_t> keys(2 * A + 2);
        for (auto& k : keys) k = rng();
        HIPCHK(hipMemcpy(zp, keys.data(), 2 * A * 8, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(zpl, keys.data() + 2 * A, 16, hipMemcpyHostToDevice));
    }
    // First-query legal order of a fresh GomokuState: libstdc++ unordered_set growth
    {
        std::unordered_set<int> set;
        for (int a = 0; a < A; ++a) set.insert(a);
        std::vector<int> order(set.begin(), set.end());
        HIPCHK(hipMemcpy(fo, order.data(), A * 4, hipMemcpyHostToDevice));
    }
    HIPCHK(hipMemset(t.err, 0, 4));
    if (hipMalloc((void**)&s->d_tree, AZ_TREE_SLOTS * sizeof(TreeDev)) != hipSuccess ||
        hipHostMalloc((void**)&s->h_tree, AZ_TREE_SLOTS * sizeof(TreeDev), hipHostMallocDefault) != hipSuccess) {
        az_search_destroy(s);
        return az_fail(AZ_ERR_OOM, "TreeDev slots");
    }
    HIPCHK(hipDeviceSynchronize());   // the null-stream copies / memsets above, before the engine stream runs
    // every slot an idle game with a valid root until k_new_games starts it
    t.nd = s->arena[0];
    hipLaunchKernelGGL(k_init_slots, dim3((G + 255) / 256), dim3(256), 0, e->stream, t, s->arena[1]);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(e->stream));
    s->stones.assign(G, 0); s->active.assign(G, 0); s->fresh.assign(G, 1); s->ply.assign(G, 0); s->expanded.assign(G, 0);
    s->rng.resize(G);
    s->hist.assign(G, {});
    if (!s->h_noise.get((size_t)G * NA)) { az_search_destroy(s); return az_fail(AZ_ERR_OOM, "hipHostMalloc (noise)"); }
    std::fill(s->h_noise.p, s->h_noise.p + (size_t)G * NA, 0.0f);
    s->h_mask.assign(G, 0);
    *out = s;
    return 0;
}

void az_search_destroy(az_search* s) {
    if (s) { pf_wait(s); s->pc.release(); s->pcf.release(); }
    if (!s) return;
    (void)hipSetDevice(s->e->device);
    auto F = [](const void* p) { if (p) (void)hipFree((void*)p); };
    for (auto& nd : s->arena) { F(nd.N); F(nd.W); F(nd.VL); F(nd.P); F(nd.first); F(nd.act); F(nd.cnt); F(nd.flag); }
    TreeDev& t = s->t;
    for (const void* p : {(const void*)t.atop, (const void*)t.rboard, (const void*)t.rhist, (const void*)t.rplayer,
                          (const void*)t.rstones, (const void*)t.rply, (const void*)t.rhash, (const void*)t.rfresh,
                          (const void*)t.rnode, (const void*)t.active, (const void*)t.gresult, (const void*)t.path, (const void*)t.pact,
                          (const void*)t.pstat, (const void*)t.rhdr,
                          (const void*)t.plen, (const void*)t.lstatus, (const void*)t.lvalue, (const void*)t.lhash,
                          (const void*)t.ttstore, (const void*)t.ttref, (const void*)t.tthslot, (const void*)t.need_eval,
                          (const void*)t.eval_slot, (const void*)t.eval_games, (const void*)t.n_eval, (const void*)t.leafrec, (const void*)t.goleaf,
                          (const void*)t.tt_hash, (const void*)t.tt_visits, (const void*)t.tt_value, (const void*)t.tt_ref,
                          (const void*)t.ring_buf, (const void*)t.ring_cur, (const void*)t.cnt, (const void*)t.zpiece,
                          (const void*)t.zplayer, (const void*)t.fresh_order, (const void*)t.mt, (const void*)t.err,
                          (const void*)t.rko, (const void*)t.rpass, (const void*)t.rposh, (const void*)t.rnposh,
                          (const void*)t.zko, (const void*)s->d_lmoves, (const void*)s->d_llen,
                          (const void*)t.log_pol, (const void*)t.log_val, (const void*)t.log_planes, (const void*)t.log_n,
                          (const void*)s->d_src_of, (const void*)s->d_batch, (const void*)s->d_id, (const void*)s->d_logits,
                          (const void*)s->d_value, (const void*)s->d_noise, (const void*)s->d_mask, (const void*)s->d_actions,
                          (const void*)s->d_values, (const void*)s->d_probs, (const void*)s->d_cact, (const void*)s->d_nch,
                          (const void*)s->d_term, (const void*)s->d_res, (const void*)s->d_rexp, (const void*)s->d_games, (const void*)s->d_seed_ids, (const void*)s->d_temps,
                          (const void*)s->d_rc, (const void*)s->d_rcf, (const void*)s->d_thr, (const void*)s->d_pruned,
                          (const void*)s->d_tree})
        F(p);
    if (s->h_tree) (void)hipHostFree(s->h_tree);
    delete s;
}

int az_search_new_games(az_search* s, const int* games, int n) {
    if (!s || (!games && n)) return az_fail(AZ_ERR_ARG, "null argument");
    std::lock_guard<std::mutex> lk(s->mu);
    HIPCHK(hipSetDevice(s->e->device));
    return search_new_games(s, games, n);
}

int az_search_add_noise(az_search* s, float alpha, float eps) {
    if (!s) return az_fail(AZ_ERR_ARG, "null search");
    std::lock_guard<std::mutex> lk(s->mu);
    HIPCHK(hipSetDevice(s->e->device));
    return search_noise(s, alpha, eps, nullptr);
}

int az_search_add_noise_masked(az_search* s, float alpha, float eps, const uint8_t* mask) {
    if (!s || !mask) return az_fail(AZ_ERR_ARG, "null argument");
    std::lock_guard<std::mutex> lk(s->mu);
    HIPCHK(hipSetDevice(s->e->device));
    return search_noise(s, alpha, eps, mask);
}

int az_search_run(az_search* s) {
    if (!s) return az_fail(AZ_ERR_ARG, "null search");
    std::lock_guard<std::mutex> lk(s->mu);
    HIPCHK(hipSetDevice(s->e->device));
    return search_run(s);
}

int az_search_select(az_search* s, int training, float temperature, int* actions, float* root_values, float* probs,
                     int* children_actions, int* n_children) {
    if (!s) return az_fail(AZ_ERR_ARG, "null search");
    std::lock_guard<std::mutex> lk(s->mu);
    HIPCHK(hipSetDevice(s->e->device));
    return search_select(s, training, nullptr, temperature, actions, root_values, probs, children_actions, n_children);
}

int az_search_simulate(az_search* s, int n) {
    if (!s || n < 0) return az_fail(AZ_ERR_ARG, "bad argument");
    std::lock_guard<std::mutex> lk(s->mu);
    HIPCHK(hipSetDevice(s->e->device));
    if (int r = search_sims(s, n)) return r;
    return check_err(s);
}

static int search_release(az_search* s, int threshold, int64_t* pruned, const uint8_t* mask) {
    HIPCHK(hipSetDevice(s->e->device));
    hipStream_t st = s->e->stream;
    const int G = s->c.n_games;
    long long* d_pr = s->d_pruned;
    int* d_thr = nullptr;
    if (mask) {   // games outside the mask keep every child (the whole tree is copied as it is)
        std::vector<int> thr(G);
        for (int g = 0; g < G; ++g) thr[g] = mask[g] ? threshold : 0;
        d_thr = s->d_thr;
        HIPCHK(hipMemcpy(d_thr, thr.data(), (size_t)G * 4, hipMemcpyHostToDevice));
    }
    s->t.nd = s->arena[s->cur];
    hipLaunchKernelGGL(k_prune, dim3(G), dim3(64), 0, st, s->t, s->arena[s->cur ^ 1], s->d_src_of, threshold, d_thr, d_pr);
    s->cur ^= 1;
    s->t.nd = s->arena[s->cur];
    std::vector<long long> pr(G);
    hipError_t e1 = hipGetLastError();
    hipError_t e2 = hipMemcpyAsync(pr.data(), d_pr, (size_t)G * 8, hipMemcpyDeviceToHost, st);
    hipError_t e3 = hipStreamSynchronize(st);
    if (e1 != hipSuccess || e2 != hipSuccess || e3 != hipSuccess)
        return az_fail(AZ_ERR_HIP, "az_search_release: %s", hipGetErrorString(e1 != hipSuccess ? e1 : e2 != hipSuccess ? e2 : e3));
    if (pruned) for (int g = 0; g < G; ++g) pruned[g] = pr[g];
    return check_err(s);
}

int az_search_release(az_search* s, int threshold, int64_t* pruned) {
    if (!s) return az_fail(AZ_ERR_ARG, "null search");
    std::lock_guard<std::mutex> lk(s->mu);
    return search_release(s, threshold, pruned, nullptr);
}

int az_search_release_masked(az_search* s, int threshold, int64_t* pruned, const uint8_t* mask) {
    if (!s || !mask) return az_fail(AZ_ERR_ARG, "null argument");
    std::lock_guard<std::mutex> lk(s->mu);
    return search_release(s, threshold, pruned, mask);
}

// Park every game outside `mask` (inactive on the host and the device) around fn, then give the
// parked games their flags back: the masked entry points run the search of some games of a handle
// that several host objects share (mcts::SearchGroup), leaving the others' trees untouched.
static int with_masked(az_search* s, const uint8_t* mask, const std::function<int()>& fn) {
    const int G = s->c.n_games;
    const std::vector<int> saved = s->active;
    std::vector<int> now(G);
    bool parked = false;
    for (int g = 0; g < G; ++g) {
        now[g] = saved[g] && mask[g];
        parked |= now[g] != saved[g];
    }
    // roots_ready speaks for the games playing when it was set: parked games may have unexpanded roots
    s->roots_ready = false;
    if (parked) {
        s->active = now;
        HIPCHK(hipStreamSynchronize(s->e->stream));   // no queued kernel may still read the old flags
        HIPCHK(hipMemcpy(s->t.active, now.data(), (size_t)G * 4, hipMemcpyHostToDevice));
    }
    const int r = fn();
    if (parked) {
        HIPCHK(hipStreamSynchronize(s->e->stream));
        std::vector<int> back(G);
        for (int g = 0; g < G; ++g) back[g] = mask[g] ? s->active[g] : saved[g];
        s->active = back;
        HIPCHK(hipMemcpy(s->t.active, back.data(), (size_t)G * 4, hipMemcpyHostToDevice));
        s->roots_ready = false;
    }
    return r;
}

int az_search_run_masked(az_search* s, const uint8_t* mask) {
    if (!s || !mask) return az_fail(AZ_ERR_ARG, "null argument");
    std::lock_guard<std::mutex> lk(s->mu);
    HIPCHK(hipSetDevice(s->e->device));
    return with_masked(s, mask, [&] { return search_run(s); });
}

int az_search_simulate_masked(az_search* s, int n, const uint8_t* mask) {
    if (!s || !mask || n < 0) return az_fail(AZ_ERR_ARG, "bad argument");
    std::lock_guard<std::mutex> lk(s->mu);
    HIPCHK(hipSetDevice(s->e->device));
    return with_masked(s, mask, [&] {
        if (int r = search_sims(s, n)) return r;
        return check_err(s);
    });
}

int az_search_new_games_ids(az_search* s, const int* games, const int* seed_ids, int n) {
    if (!s || (!games && n) || (!seed_ids && n)) return az_fail(AZ_ERR_ARG, "null argument");
    std::lock_guard<std::mutex> lk(s->mu);
    HIPCHK(hipSetDevice(s->e->device));
    return search_new_games(s, games, n, seed_ids);
}

int az_search_select_action(az_search* s, int game, int training, float temperature, int batch_inference,
                            const int* legal, int n_legal, int* action) {
    if (!s || !action || game < 0 || game >= s->c.n_games || n_legal < 0 || (n_legal > 0 && !legal))
        return az_fail(AZ_ERR_ARG, "bad argument");
    std::lock_guard<std::mutex> lk(s->mu);
    HIPCHK(hipSetDevice(s->e->device));
    const int G = s->c.n_games, NA = s->t.NA;
    std::vector<int> acts(G), cact((size_t)G * NA), nch(G);
    std::vector<float> vals(G), probs((size_t)G * NA);
    const bool stoch = training && temperature > 0.0f;
    if (int r = search_select(s, training ? 1 : 0, nullptr, temperature, acts.data(), vals.data(), probs.data(), cact.data(),
                              nch.data()))
        return r;
    pf_drop(s, game);                                // this draw moves the game's generator
    std::mt19937& rng = s->rng[game];
    const int nc = nch[game];
    if (nc == 0) {                                   // no children: a legal move (parallel_mcts.cpp:994-1010)
        if (n_legal == 0) { *action = -1; return 0; }
        if (batch_inference) { *action = legal[0]; return 0; }
        std::uniform_int_distribution<size_t> dist(0, (size_t)n_legal - 1);
        *action = legal[dist(rng)];
        return 0;
    }
    const int* ca = cact.data() + (size_t)game * NA;
    if (batch_inference) { *action = acts[game]; return 0; }   // k_select_action: the deterministic rules
    if (stoch) {                                     // sample the visit distribution (:1013-1027)
        const float* pd = probs.data() + (size_t)game * NA;
        std::discrete_distribution<int> dist(pd, pd + nc);
        *action = ca[dist(rng)];
        return 0;
    }
    // evaluation or T = 0: the most visited children, one at random when tied (:1028-1046)
    std::vector<int> N(NA), act(NA), VL(NA);
    std::vector<float> W(NA), P(NA);
    int n = 0;
    s->t.nd = s->arena[s->cur];
    int* d_tmp = s->d_rc;
    float* d_f = s->d_rcf;
    hipStream_t st = s->e->stream;
    hipLaunchKernelGGL(k_root_children, dim3(1), dim3(64), 0, st, s->t, game, d_tmp, d_tmp + NA, d_tmp + 2 * NA, d_f,
                       d_f + NA, d_tmp + 3 * NA, d_tmp + 3 * NA + 1, d_f + 2 * NA);
    hipError_t e1 = hipMemcpyAsync(act.data(), d_tmp, NA * 4, hipMemcpyDeviceToHost, st);
    hipError_t e2 = hipMemcpyAsync(N.data(), d_tmp + NA, NA * 4, hipMemcpyDeviceToHost, st);
    hipError_t e3 = hipMemcpyAsync(&n, d_tmp + 3 * NA, 4, hipMemcpyDeviceToHost, st);
    hipError_t e4 = hipStreamSynchronize(st);
    if (e1 != hipSuccess || e2 != hipSuccess || e3 != hipSuccess || e4 != hipSuccess)
        return az_fail(AZ_ERR_HIP, "az_search_sample_action: root children readback failed");
    int mx = 0;
    for (int i = 0; i < n; ++i) mx = std::max(mx, N[i]);
    std::vector<int> best;
    for (int i = 0; i < n; ++i) if (N[i] == mx) best.push_back(act[i]);
    if (best.empty()) { *action = -1; return 0; }
    if (best.size() == 1) { *action = best[0]; return 0; }
    std::uniform_int_distribution<size_t> dist(0, best.size() - 1);
    *action = best[dist(rng)];
    return 0;
}

int az_search_apply(az_search* s, const int* actions, int* terminal, int* result) {
    if (!s || !actions) return az_fail(AZ_ERR_ARG, "null argument");
    std::lock_guard<std::mutex> lk(s->mu);
    HIPCHK(hipSetDevice(s->e->device));
    const int G = s->c.n_games, A = s->t.A;
    for (int g = 0; g < G; ++g)
        if (actions[g] >= A || (s->t.game == GAME_GO && actions[g] < AZ_ACTION_NONE))
            return az_fail(AZ_ERR_ARG, "action %d out of range for game %d", actions[g], g);
    HIPCHK(hipMemcpyAsync(s->d_actions, actions, G * 4, hipMemcpyHostToDevice, s->e->stream));
    return search_apply_dev(s, terminal, result);
}

int az_search_root_children(az_search* s, int game, int* actions, int* N, int* VL, float* W, float* P, int* n_children) {
    if (!s || game < 0 || game >= s->c.n_games || !n_children) return az_fail(AZ_ERR_ARG, "bad argument");
    std::lock_guard<std::mutex> lk(s->mu);
    HIPCHK(hipSetDevice(s->e->device));
    hipStream_t st = s->e->stream;
    const int A = s->t.NA;
    int *da, *dN, *dVL, *dn, *dri; float *dW, *dP, *drw;
    DALLOC(da, A); DALLOC(dN, A); DALLOC(dVL, A); DALLOC(dn, 1); DALLOC(dri, 2); DALLOC(dW, A); DALLOC(dP, A); DALLOC(drw, 1);
    s->t.nd = s->arena[s->cur];
    hipLaunchKernelGGL(k_root_children, dim3(1), dim3(256), 0, st, s->t, game, da, dN, dVL, dW, dP, dn, dri, drw);
    int n = 0;
    HIPCHK(hipMemcpyAsync(&n, dn, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (actions) HIPCHK(hipMemcpy(actions, da, n * 4, hipMemcpyDeviceToHost));
    if (N) HIPCHK(hipMemcpy(N, dN, n * 4, hipMemcpyDeviceToHost));
    if (VL) HIPCHK(hipMemcpy(VL, dVL, n * 4, hipMemcpyDeviceToHost));
    if (W) HIPCHK(hipMemcpy(W, dW, n * 4, hipMemcpyDeviceToHost));
    if (P) HIPCHK(hipMemcpy(P, dP, n * 4, hipMemcpyDeviceToHost));
    *n_children = n;
    for (void* p : {(void*)da, (void*)dN, (void*)dVL, (void*)dn, (void*)dri, (void*)dW, (void*)dP, (void*)drw}) (void)hipFree(p);
    return 0;
}

int az_search_set_evaluator(az_search* s, az_eval_fn fn, void* user) {
    if (!s) return az_fail(AZ_ERR_ARG, "null search");
    if (s->c.eval_kind != AZ_EVAL_CALLBACK) return az_fail(AZ_ERR_STATE, "the handle was not created with AZ_EVAL_CALLBACK");
    std::lock_guard<std::mutex> lk(s->mu);
    s->eval_fn = fn; s->eval_user = user;
    return 0;
}

// A new device net for a handle created with AZ_EVAL_NET, the tree kept (ParallelMCTS::
// setNeuralNetwork only swaps nn_, parallel_mcts.cpp:1190-1207): same engine, board, planes and
// action space, a batch capacity covering the handle's games, weights loaded.
int az_search_set_net(az_search* s, az_net* net) {
    if (!s || !net) return az_fail(AZ_ERR_ARG, "null argument");
    if (s->c.eval_kind != AZ_EVAL_NET) return az_fail(AZ_ERR_STATE, "the handle was not created with AZ_EVAL_NET");
    if (net->e != s->e) return az_fail(AZ_ERR_ARG, "the network lives on another engine");
    const int bs = s->c.board_size, NA = s->t.NA;
    const bool go = s->c.game == AZ_GAME_GO;
    if (net->d.board_size != bs || net->d.action_size != NA || net->d.in_planes != (go ? 8 : 11))
        return az_fail(AZ_ERR_ARG, "network shape does not match the board");
    if (net->d.max_batch < s->c.n_games) return az_fail(AZ_ERR_ARG, "network max_batch < n_games");
    if (!net->loaded) return az_fail(AZ_ERR_STATE, "network weights not loaded");
    std::lock_guard<std::mutex> lk(s->mu);
    s->net = net;
    return 0;
}

// Empty every game's transposition table (a new TranspositionTable object: ParallelMCTS::
// setTranspositionTable, parallel_mcts.cpp:1209-1222); trees and counters kept.
int az_search_clear_tt(az_search* s) {
    if (!s) return az_fail(AZ_ERR_ARG, "null search");
    std::lock_guard<std::mutex> lk(s->mu);
    HIPCHK(hipSetDevice(s->e->device));
    const int G = s->c.n_games;
    std::vector<int> g(G);
    for (int i = 0; i < G; ++i) g[i] = i;
    hipStream_t st = s->e->stream;
    HIPCHK(hipMemcpyAsync(s->d_games, g.data(), (size_t)G * 4, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_tt_clear, dim3(64, G), dim3(256), 0, st, s->t, s->d_games, G);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(st));
    return 0;
}

int az_search_set_params(az_search* s, const az_search_cfg* c) {
    if (!s || !c) return az_fail(AZ_ERR_ARG, "null argument");
    std::lock_guard<std::mutex> lk(s->mu);
    const az_search_cfg& o = s->c;
    if (c->n_games != o.n_games || c->board_size != o.board_size || c->eval_kind != o.eval_kind ||
        c->eval_seed != o.eval_seed || c->zobrist_seed != o.zobrist_seed || c->tt_log2 != o.tt_log2 ||
        c->game != o.game || (c->node_capacity > 0 && c->node_capacity != o.node_capacity) ||
        (c->prior_ring > 0 && c->prior_ring != o.prior_ring) || c->num_simulations < 0 || c->virtual_loss < 0)
        return az_fail(AZ_ERR_ARG, "az_search_set_params: shape / evaluator / table changes need a new handle");
    // the node pool and prior ring were sized for the creation's simulations per search
    const int NA = s->t.NA;
    if (3 * std::max(64, c->num_simulations) * NA + 8 * NA + 64 > o.node_capacity ||
        12 * std::max(64, c->num_simulations) * NA > o.prior_ring)
        return az_fail(AZ_ERR_CAPACITY, "az_search_set_params: %d simulations exceed the node pool sized at creation",
                       c->num_simulations);
    s->c.num_simulations = c->num_simulations;
    s->c.c_puct = c->c_puct; s->c.fpu_reduction = c->fpu_reduction; s->c.virtual_loss = c->virtual_loss;
    s->c.use_dirichlet_each_search = c->use_dirichlet_each_search;
    s->c.dirichlet_alpha = c->dirichlet_alpha; s->c.dirichlet_eps = c->dirichlet_eps;
    s->c.noise_seed = c->noise_seed; s->c.noise_seed_stride = c->noise_seed_stride;
    s->t.cpuct = c->c_puct; s->t.fpu = c->fpu_reduction; s->t.vl = c->virtual_loss;
    return 0;
}

int az_search_seed(az_search* s, int game, uint32_t seed) {
    if (!s || game < 0 || game >= s->c.n_games) return az_fail(AZ_ERR_ARG, "bad argument");
    std::lock_guard<std::mutex> lk(s->mu);
    pf_drop(s, game);
    s->rng[game].seed(seed);
    return 0;
}

// std::mt19937's state through its stream operators (libstdc++: the 624 state words, then the
// position), as 625 uint32
int az_search_get_rng(az_search* s, int game, uint32_t* state) {
    if (!s || !state || game < 0 || game >= s->c.n_games) return az_fail(AZ_ERR_ARG, "bad argument");
    std::lock_guard<std::mutex> lk(s->mu);
    pf_wait(s);
    std::ostringstream os;
    os << s->rng[game];
    std::istringstream is(os.str());
    for (int i = 0; i < AZ_RNG_STATE_WORDS; ++i)
        if (!(is >> state[i])) return az_fail(AZ_ERR_ARG, "rng state: unexpected serialisation");
    return 0;
}

int az_search_set_rng(az_search* s, int game, const uint32_t* state) {
    if (!s || !state || game < 0 || game >= s->c.n_games) return az_fail(AZ_ERR_ARG, "bad argument");
    std::lock_guard<std::mutex> lk(s->mu);
    std::ostringstream os;
    for (int i = 0; i < AZ_RNG_STATE_WORDS; ++i) os << state[i] << (i + 1 < AZ_RNG_STATE_WORDS ? " " : "");
    std::istringstream is(os.str());
    std::mt19937 r;
    if (!(is >> r) || state[AZ_RNG_STATE_WORDS - 1] > 624) return az_fail(AZ_ERR_ARG, "rng state: not an mt19937 state");
    pf_drop(s, game);
    s->rng[game] = r;
    return 0;
}

int az_search_root_flags(az_search* s, int game, int* flags) {
    if (!s || !flags || game < 0 || game >= s->c.n_games) return az_fail(AZ_ERR_ARG, "bad argument");
    std::lock_guard<std::mutex> lk(s->mu);
    HIPCHK(hipSetDevice(s->e->device));
    HIPCHK(hipStreamSynchronize(s->e->stream));   // its queued kernels first: the reads below are null-stream copies
    int root = 0;
    uint8_t f = 0;
    HIPCHK(hipMemcpy(&root, s->t.rnode + game, 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(&f, s->arena[s->cur].flag + (size_t)game * s->t.ncap + root, 1, hipMemcpyDeviceToHost));
    *flags = f;
    return 0;
}

int az_search_root_node(az_search* s, int game, int* N, int* VL, float* W) {
    if (!s || game < 0 || game >= s->c.n_games) return az_fail(AZ_ERR_ARG, "bad argument");
    std::lock_guard<std::mutex> lk(s->mu);
    HIPCHK(hipSetDevice(s->e->device));
    HIPCHK(hipStreamSynchronize(s->e->stream));   // its queued kernels first: the reads below are null-stream copies
    int root = 0;
    HIPCHK(hipMemcpy(&root, s->t.rnode + game, 4, hipMemcpyDeviceToHost));
    const size_t off = (size_t)game * s->t.ncap + root;
    const Nodes& nd = s->arena[s->cur];
    if (N) HIPCHK(hipMemcpy(N, nd.N + off, 4, hipMemcpyDeviceToHost));
    if (VL) HIPCHK(hipMemcpy(VL, nd.VL + off, 4, hipMemcpyDeviceToHost));
    if (W) HIPCHK(hipMemcpy(W, nd.W + off, 4, hipMemcpyDeviceToHost));
    return 0;
}

int az_search_counters(az_search* s, int game, int64_t* out5) {
    if (!s || game < 0 || game >= s->c.n_games || !out5) return az_fail(AZ_ERR_ARG, "bad argument");
    std::lock_guard<std::mutex> lk(s->mu);
    HIPCHK(hipSetDevice(s->e->device));
    HIPCHK(hipStreamSynchronize(s->e->stream));   // its queued kernels first: the reads below are null-stream copies
    long long c[AZ_NCNT];
    HIPCHK(hipMemcpy(c, s->t.cnt + (size_t)game * AZ_NCNT, sizeof c, hipMemcpyDeviceToHost));
    for (int i = 0; i < 5; ++i) out5[i] = c[i];
    return 0;
}

int az_search_enable_eval_log(az_search* s, int game, int capacity) {
    if (!s || game < 0 || game >= s->c.n_games || capacity < 1) return az_fail(AZ_ERR_ARG, "bad argument");
    std::lock_guard<std::mutex> lk(s->mu);
    HIPCHK(hipSetDevice(s->e->device));
    TreeDev& t = s->t;
    if (t.log_pol) { (void)hipFree(t.log_pol); (void)hipFree(t.log_val); (void)hipFree(t.log_planes); (void)hipFree(t.log_n); }
    t.log_pol = nullptr; t.log_val = nullptr; t.log_planes = nullptr; t.log_n = nullptr;
    const int npl = t.game == GAME_GO ? 8 : 11;
    DALLOC(t.log_pol, (size_t)capacity * t.NA); DALLOC(t.log_val, capacity); DALLOC(t.log_planes, (size_t)capacity * npl * t.A);
    DALLOC(t.log_n, 1);
    HIPCHK(hipMemset(t.log_n, 0, 4));
    t.log_game = game; t.log_cap = capacity;
    return 0;
}

int az_search_read_eval_log(az_search* s, float* policy, float* value, float* planes, int* count) {
    if (!s || !count) return az_fail(AZ_ERR_ARG, "bad argument");
    std::lock_guard<std::mutex> lk(s->mu);
    HIPCHK(hipSetDevice(s->e->device));
    HIPCHK(hipStreamSynchronize(s->e->stream));   // its queued kernels first: the reads below are null-stream copies
    TreeDev& t = s->t;
    if (!t.log_pol) { *count = 0; return 0; }
    int n = 0;
    HIPCHK(hipMemcpy(&n, t.log_n, 4, hipMemcpyDeviceToHost));
    if (policy) HIPCHK(hipMemcpy(policy, t.log_pol, (size_t)n * t.NA * 4, hipMemcpyDeviceToHost));
    if (value) HIPCHK(hipMemcpy(value, t.log_val, (size_t)n * 4, hipMemcpyDeviceToHost));
    if (planes) HIPCHK(hipMemcpy(planes, t.log_planes, (size_t)n * (t.game == GAME_GO ? 8 : 11) * t.A * 4,
                                 hipMemcpyDeviceToHost));
    *count = n;
    return 0;
}

// One playSingleGame move for every active game (self_play_manager.cpp:187-216).
int az_selfplay_step(az_search* s, const az_selfplay_cfg* cfg, int64_t* moves_done, int64_t* evals_done) {
    if (!s || !cfg) return az_fail(AZ_ERR_ARG, "null argument");
    std::lock_guard<std::mutex> lk(s->mu);
    HIPCHK(hipSetDevice(s->e->device));
    const int G = s->c.n_games;
    std::vector<long long> c0((size_t)G * AZ_NCNT), c1((size_t)G * AZ_NCNT);
    hipStream_t st = s->e->stream;
    // the counters on the engine stream (a null-stream copy would not wait for its queued kernels)
    if (evals_done) {
        HIPCHK(hipMemcpyAsync(c0.data(), s->t.cnt, c0.size() * 8, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
    }
    const auto t0 = std::chrono::steady_clock::now();
    STEP_TRACE("step start");
    if (int r = search_run(s)) return r;
    std::vector<float> temps(G);
    std::vector<int> was_active = s->active;
    std::vector<int> ply0 = s->ply;
    for (int g = 0; g < G; ++g) temps[g] = s->ply[g] >= cfg->temp_drop_move ? cfg->t_final : cfg->t_init;
    std::vector<int> actions(G);
    // the same D2H and MoveData assembly as az_selfplay_run (getActionProbabilities + getRootValue
    // per game, self_play_manager.cpp:187-203); read back with az_selfplay_step_moves
    const int NA = s->t.NA;
    float* probs = s->sp_probs.get((size_t)G * NA);
    int* cact = s->sp_cact.get((size_t)G * NA);
    float* vals = s->sp_values.get(G);
    int* nch = s->sp_nch.get(G);
    if (!probs || !cact || !vals || !nch) return az_fail(AZ_ERR_OOM, "hipHostMalloc (move records)");
    STEP_TRACE("select");
    if (int r = search_select(s, 1, temps.data(), 0.0f, actions.data(), vals, probs, cact, nch))
        return r;
    STEP_TRACE("apply");
    const int64_t ms = std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count();
    std::vector<int> term(G), res(G);
    if (int r = search_apply_dev(s, term.data(), res.data())) return r;
    int64_t moves = 0;
    std::vector<uint8_t> noise_mask(G, 0);
    const int none = s->t.game == GAME_GO ? AZ_ACTION_NONE : -1;
    s->sp_moves.clear(); s->sp_slots.clear();
    for (int g = 0; g < G; ++g) {
        if (!was_active[g] || actions[g] == none) continue;
        ++moves;
        if (ply0[g] % 2 == 0) noise_mask[g] = 1;
        s->sp_moves.push_back(az_move_rec{actions[g], vals[g], nch[g], probs + (size_t)g * NA, cact + (size_t)g * NA, ms});
        s->sp_slots.push_back(g);
    }
    STEP_TRACE("noise");
    if (int r = search_noise(s, s->c.dirichlet_alpha, s->c.dirichlet_eps, noise_mask.data())) return r;
    STEP_TRACE("restart / counters");
    if (cfg->restart_finished) {
        std::vector<int> fin;
        for (int g = 0; g < G; ++g) if (!s->active[g]) fin.push_back(g);
        if (!fin.empty()) {
            // a restarted slot plays the next game id (slot order), whose evaluator / noise streams
            // it seeds -- as az_selfplay_run hands out ids -- rather than replaying its slot's seed
            std::vector<int> ids(fin.size());
            for (size_t i = 0; i < fin.size(); ++i) ids[i] = s->sp_next_id + (int)i;
            if (int r = search_new_games(s, fin.data(), (int)fin.size(), ids.data())) return r;
            std::vector<uint8_t> m(G, 0);
            for (int g : fin) m[g] = 1;
            if (int r = search_noise(s, s->c.dirichlet_alpha, s->c.dirichlet_eps, m.data())) return r;
        }
    }
    if (s->t.game == GAME_GOMOKU && !s->c.use_dirichlet_each_search) {
        // the next move's noise (games whose next ply is even, self_play_manager.cpp:209-211) is drawn
        // on a host thread while the device searches
        std::vector<uint8_t> want(G, 0);
        for (int g = 0; g < G; ++g) want[g] = s->active[g] && s->ply[g] % 2 == 0;
        prefetch_noise(s, s->c.dirichlet_alpha, want);
    }
    if (moves_done) *moves_done += moves;
    if (evals_done) {
        HIPCHK(hipMemcpyAsync(c1.data(), s->t.cnt, c1.size() * 8, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        long long ev = 0;
        for (int g = 0; g < G; ++g) ev += c1[(size_t)g * AZ_NCNT + CNT_EVALS_TOTAL] - c0[(size_t)g * AZ_NCNT + CNT_EVALS_TOTAL];
        *evals_done += ev;
    }
    STEP_TRACE("step done");
    return 0;
}

int az_selfplay_step_moves(az_search* s, const az_move_rec** moves, const int** slots, int* n) {
    if (!s || !moves || !n) return az_fail(AZ_ERR_ARG, "null argument");
    std::lock_guard<std::mutex> lk(s->mu);
    *moves = s->sp_moves.data();
    if (slots) *slots = s->sp_slots.data();
    *n = (int)s->sp_moves.size();
    return 0;
}

int az_selfplay_run(az_search* s, const az_selfplay_cfg* cfg, int total_games, int max_moves, az_game_sink sink,
                    az_progress_fn progress, void* user, const volatile int* abort_flag) {
    if (!s || !cfg || total_games < 0) return az_fail(AZ_ERR_ARG, "bad argument");
    std::lock_guard<std::mutex> lk(s->mu);
    HIPCHK(hipSetDevice(s->e->device));
    hipStream_t st = s->e->stream;
    const int G = s->c.n_games, A = s->t.NA;     // child-order records: up to NA children
    const int none = s->t.game == GAME_GO ? AZ_ACTION_NONE : -1;
    struct Rec {
        std::vector<az_move_rec> moves;
        std::vector<std::vector<float>> pol;
        std::vector<std::vector<int>> cact;
    };
    std::vector<Rec> rec(G);
    std::vector<int> game_of(G, -1);
    int next = 0;
    int64_t total_moves = 0;
    // every slot idle, then the first min(G, total) games
    std::fill(s->active.begin(), s->active.end(), 0);
    HIPCHK(hipMemsetAsync(s->t.active, 0, (size_t)G * sizeof(int), st));
    auto start = [&](const std::vector<int>& slots) -> int {
        if (slots.empty()) return 0;
        std::vector<int> ids(slots.size());
        std::vector<uint8_t> mask(G, 0);
        for (size_t i = 0; i < slots.size(); ++i) {
            ids[i] = next++;
            game_of[slots[i]] = ids[i];
            rec[slots[i]] = Rec{};
            mask[slots[i]] = 1;
        }
        if (int r = search_new_games(s, slots.data(), (int)slots.size(), ids.data())) return r;
        return search_noise(s, s->c.dirichlet_alpha, s->c.dirichlet_eps, mask.data());   // :184
    };
    std::vector<int> first;
    for (int g = 0; g < G && g < total_games; ++g) first.push_back(g);
    if (int r = start(first)) return r;
    std::vector<float> temps(G), values(G), probs((size_t)G * A);
    std::vector<int> actions(G), cact((size_t)G * A), nch(G), term(G), res(G);
    for (;;) {
        bool any = false;
        for (int g = 0; g < G; ++g) any |= s->active[g] != 0;
        if (!any || (abort_flag && *abort_flag)) break;
        const auto t0 = std::chrono::steady_clock::now();
        if (int r = search_run(s)) return r;
        for (int g = 0; g < G; ++g) temps[g] = s->ply[g] >= cfg->temp_drop_move ? cfg->t_final : cfg->t_init;  // :236-240
        if (int r = search_select(s, 1, temps.data(), 0.0f, actions.data(), values.data(), probs.data(), cact.data(),
                                  nch.data()))
            return r;
        const int64_t ms = std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count();
        std::vector<int> was_active = s->active, ply0 = s->ply;
        for (int g = 0; g < G; ++g) {
            if (!was_active[g] || actions[g] == none) continue;
            Rec& R = rec[g];
            R.pol.emplace_back(probs.begin() + (size_t)g * A, probs.begin() + (size_t)g * A + nch[g]);
            R.cact.emplace_back(cact.begin() + (size_t)g * A, cact.begin() + (size_t)g * A + nch[g]);
            R.moves.push_back(az_move_rec{actions[g], values[g], nch[g], nullptr, nullptr, ms});
            ++total_moves;
            if (progress) progress(user, game_of[g], ply0[g], total_games, total_moves);
        }
        if (int r = search_apply_dev(s, term.data(), res.data())) return r;
        std::vector<uint8_t> noise(G, 0);
        std::vector<int> done, restart;
        for (int g = 0; g < G; ++g) {
            if (!was_active[g]) continue;
            const bool fin = !s->active[g] || (max_moves > 0 && s->ply[g] >= max_moves);
            if (!fin) {
                if (ply0[g] % 2 == 0) noise[g] = 1;                                            // :209-211
                continue;
            }
            done.push_back(g);
        }
        if (int r = search_noise(s, s->c.dirichlet_alpha, s->c.dirichlet_eps, noise.data())) return r;
        for (int g : done) {
            Rec& R = rec[g];
            for (size_t i = 0; i < R.moves.size(); ++i) { R.moves[i].policy = R.pol[i].data(); R.moves[i].child_actions = R.cact[i].data(); }
            const int result = s->active[g] ? 0 : res[g];
            if (s->active[g]) {                     // cut at max_moves: park the slot
                s->active[g] = 0;
                HIPCHK(hipMemsetAsync(s->t.active + g, 0, sizeof(int), st));
            }
            if (sink) sink(user, game_of[g], s->c.board_size, (int)R.moves.size(), R.moves.data(), result);
            rec[g] = Rec{};
            game_of[g] = -1;
            if (next + (int)restart.size() < total_games) restart.push_back(g);
        }
        if (int r = start(restart)) return r;
        if (s->t.game == GAME_GOMOKU && !s->c.use_dirichlet_each_search) {   // as az_selfplay_step
            std::vector<uint8_t> want(G, 0);
            for (int g = 0; g < G; ++g) want[g] = s->active[g] && s->ply[g] % 2 == 0;
            prefetch_noise(s, s->c.dirichlet_alpha, want);
        }
    }
    pf_wait(s);
    HIPCHK(hipStreamSynchronize(st));
    return 0;
}

// diagnostic: TreeDev slot evictions so far (bench.py reports it: a steady-state step should have none)
int64_t az_diag_tree_evictions(az_search* s) { return s ? s->tree_evictions : -1; }

int az_search_profile(az_search* s, int enable) {
    if (!s) return az_fail(AZ_ERR_ARG, "null search");
    std::lock_guard<std::mutex> lk(s->mu);
    HIPCHK(hipSetDevice(s->e->device));
    HIPCHK(hipStreamSynchronize(s->e->stream));
    s->prof = enable != 0;
    for (ProfClock* pc : {&s->pc, &s->pcf})
        if (s->prof && !pc->d && hipMalloc((void**)&pc->d, ProfClock::CAP * 8) != hipSuccess) {
            pc->d = nullptr;
            return az_fail(AZ_ERR_OOM, "profile clock buffer");
        }
    s->pc.used = 0; s->pcf.used = 0;
    s->prof_steps = 0; s->prof_sampled = 0; s->prof_fused = 0; s->prof_fused_launches = 0;
    s->prof_cnt0.assign((size_t)s->c.n_games * AZ_NCNT, 0);
    HIPCHK(hipMemcpy(s->prof_cnt0.data(), s->t.cnt, s->prof_cnt0.size() * 8, hipMemcpyDeviceToHost));
    return 0;
}

int az_search_profile_read(az_search* s, double* select_ms, double* expand_ms, int64_t* sim_steps,
                           int64_t* select_bytes, int64_t* expand_bytes) {
    if (!s) return az_fail(AZ_ERR_ARG, "null search");
    std::lock_guard<std::mutex> lk(s->mu);
    HIPCHK(hipSetDevice(s->e->device));
    HIPCHK(hipStreamSynchronize(s->e->stream));
    double sel = 0.0, exp = 0.0;
    const std::vector<double> t = s->pc.read_ms();
    for (size_t i = 0; i + 3 < t.size(); i += 4) {
        sel += t[i + 1] - t[i];
        exp += t[i + 3] - t[i + 2];
    }
    std::vector<long long> c((size_t)s->c.n_games * AZ_NCNT);
    HIPCHK(hipMemcpy(c.data(), s->t.cnt, c.size() * 8, hipMemcpyDeviceToHost));
    long long bs = 0, be = 0;
    for (int g = 0; g < s->c.n_games; ++g) {
        const size_t o = (size_t)g * AZ_NCNT;
        const long long* c0 = s->prof_cnt0.empty() ? nullptr : s->prof_cnt0.data() + o;
        bs += c[o + CNT_BYTES_SEL] - (c0 ? c0[CNT_BYTES_SEL] : 0);
        be += c[o + CNT_BYTES_EXP] - (c0 ? c0[CNT_BYTES_EXP] : 0);
    }
    // sampled steps' kernel times scaled to every simulation step
    const double k = s->prof_sampled ? (double)s->prof_steps / (double)s->prof_sampled : 0.0;
    if (select_ms) *select_ms = sel * k;
    if (expand_ms) *expand_ms = exp * k;
    if (sim_steps) *sim_steps = s->prof_steps;
    if (select_bytes) *select_bytes = bs;
    if (expand_bytes) *expand_bytes = be;
    return 0;
}

int az_search_profile_read_fused(az_search* s, double* fused_ms, int64_t* fused_launches) {
    if (!s) return az_fail(AZ_ERR_ARG, "null search");
    std::lock_guard<std::mutex> lk(s->mu);
    HIPCHK(hipSetDevice(s->e->device));
    HIPCHK(hipStreamSynchronize(s->e->stream));
    double f = 0.0;
    const std::vector<double> t = s->pcf.read_ms();
    for (size_t i = 0; i + 1 < t.size(); i += 2) f += t[i + 1] - t[i];
    // sampled fused launches' time scaled to every fused launch
    if (fused_ms) *fused_ms = s->prof_fused ? f * (double)s->prof_fused_launches / (double)s->prof_fused : 0.0;
    if (fused_launches) *fused_launches = s->prof_fused_launches;
    return 0;
}

}  // extern "C"
