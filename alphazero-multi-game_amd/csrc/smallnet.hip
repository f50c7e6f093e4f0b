// smallnet.hip -- the whole ConvNet trunk of a small net in ONE launch, one board per block
// (fp16 MFMA operands, fp32 accumulation, fp32 residual stream).
//
// For 64-filter nets (BASELINE.json C2: 15x15, 6 blocks x 64 filters, 256 games) a trunk conv is
// 4.2 GFLOP at 256 boards: one launch per layer is latency-bound (a 2-board v4 tile gives 128
// blocks for 256 CUs) and the activations make an HBM round trip per layer.  A board's
// activations are small (225 px x 64 ch: 57.6 KB fp32, 28.8 KB fp16), so one 256-thread block
// keeps them in LDS through every layer:
//
//   input planes -> input conv -> 2*blocks residual convs -> adaptive pool -> policy / value 1x1 convs
//
// and writes only the two head feature maps (pp / vp, [board][P*P][HC] fp32, the layout the FC
// layers read).  Weights stream per tap from L2 (every block reads the same 74 KB per layer) into a
// ring of LDS tiles with global_load_lds; one barrier per tap.
//
// The fp32 residual stream stays in REGISTERS: a lane owns the same (pixel, 4 channels) outputs in
// every layer, so the second conv of a block adds its own values (64 VGPRs per lane).
// LDS (15x15): two zero-padded halo images X and Y fp16 [IR][64] (2 x 37.4 KB), a ring of 8 weight
// tiles [64 n][64 c] fp16 (8 x 8 KB, loaded 6 taps ahead so the L2 latency is hidden), the biases.
// Every tap ends with a barrier that certifies the weight tile two taps ahead, so the fragments of
// the next (tap, chunk) step are read while the current step's 16 MFMAs run.
// Rows of 64 fp16 channels
// are 8 chunks of 16 B stored at chunk ^ (row & 7): conflict-free ds_read_b128 for every tap shift.
// Outputs live on the HB x (HB+2) grid (two dead columns per row): tap (dy, dx) of output grid row q
// is halo row q + dy*(HB+2) + dx, so an operand fragment is 16 consecutive halo rows.
//
// MFMA v_mfma_f32_16x16x32_f16 with the weights as the 16-row operand and the activations as the
// 16-column one: a lane's accumulator holds 4 consecutive output channels of one pixel, so the
// epilogue (bias already in the accumulator, residual join, ReLU) writes xs and the next image from
// registers.  Layer roles: 0 = input conv (reads Y = planes, writes xs + X), odd = first conv of a
// residual block (reads X, writes Y), even >= 2 = second conv (reads Y, adds xs, writes xs + X).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <type_traits>

#include "net.h"
#include "leaf_planes.h"

namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;

constexpr int SF = 64;           // filters (channels) of the fused trunk

template <int HB, int NW = 4>
struct SmGeom {
    static constexpr int WG = HB + 2;                    // grid / halo row width
    static constexpr int HW = HB * HB;
    static constexpr int GRID = HB * WG;                 // output grid rows
    static constexpr int NFRAG = (GRID + 15) / 16;       // 16-row pixel fragments
    static constexpr int FPW = (NFRAG + 3) / 4;          // fragments per pixel-wave (4 pixel groups)
    static constexpr int JN = 4 * 4 / NW;                // 16-channel output blocks per wave (NW = 4: all 4, 8: 2)
    static constexpr int IR = NFRAG * 16 + 2 * WG + 2;   // halo rows the last fragment's taps read
    static constexpr int IMG = IR * SF * 2;              // bytes of one halo image
    static constexpr int XS = HW * SF * 4;               // fp32 stream at the end (over the two images)
    static constexpr int WT = SF * SF * 2;               // bytes of one tap's weight tile
    static constexpr int NSLOT = 8, DIST = 6;            // weight ring: tiles DIST taps ahead
    static constexpr int MAXL = 32;                      // layers (biases staged in LDS)
    static constexpr int LDS = 2 * IMG + NSLOT * WT + MAXL * SF * 4;
    static_assert(LDS <= 160 * 1024, "board does not fit the CU's LDS");
    static_assert(XS <= 2 * IMG, "fp32 stream does not fit over the images");
};

__device__ __forceinline__ uint32_t img_off(int row, int chunk) {   // byte offset of (row, 16-B chunk)
    return (uint32_t)(row * 128 + ((chunk ^ (row & 7)) << 4));
}
__device__ __forceinline__ uint32_t xs_off(int p, int chunk4) {     // fp32 stream: 16 chunks of 4 channels
    return (uint32_t)(p * 256 + ((chunk4 ^ (p & 15)) << 4));
}

template <int I, int N, typename Fn>
__device__ __forceinline__ void static_for(Fn&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<I + 1, N>(f);
    }
}

// diagnostic phase stamps of block 0 (s_memrealtime, 100 MHz): SmallNetArgs.stamps != 0
__device__ unsigned long long g_sm_stamps[128];      // [0, 64): s_memrealtime, [64, 128): s_memtime (shader clock)
__device__ __forceinline__ void sm_stamp(const SmallNetArgs& p, int i) {
    if (p.stamps && blockIdx.x == 0 && threadIdx.x == 0 && i < 64) {
        g_sm_stamps[i] = __builtin_amdgcn_s_memrealtime();
        g_sm_stamps[64 + i] = __builtin_amdgcn_s_memtime();
    }
}

// s_waitcnt lgkmcnt(N), then every fragment of a and b tied to that point (empty asm rewriting
// them), so no MFMA that reads them is scheduled above the wait
template <int N, int JA, int JB, typename F>
__device__ __forceinline__ void certify_frags(F (&a)[JA], F (&b)[JB]) {
    asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(N) : "memory");
#pragma unroll
    for (int j = 0; j < JA; ++j) asm volatile("" : "+v"(a[j]));
#pragma unroll
    for (int i = 0; i < JB; ++i) asm volatile("" : "+v"(b[i]));
}

}  // namespace

// measurement only (tools/sm_check.sh, tools/net_bench.py): 4 = one wave per SIMD instead of the
// default 8-wave block of the round-2 kernel.  Kernel 0 (default) = k_smallnet_g (weights streamed
// into registers), 1 = the round-2 kernel (k_smallnet_r2: A/B and the bitwise-equality test)
static int g_sm_waves = 8;
static int g_sm_kernel = 0;
static int g_sm_stamp_mode = 0;
int az_smallnet_stamps_mode() { return g_sm_stamp_mode; }
// phase stamps of block 0 (tools/sm_stamps.py): nonzero = on
extern "C" int az_diag_set_smallnet_stamps(int mode) {
    g_sm_stamp_mode = mode;
    return 0;
}
extern "C" int az_diag_set_smallnet_waves(int nw) {
    g_sm_waves = nw == 4 ? 4 : 8;
    return 0;
}
extern "C" int az_diag_set_smallnet_kernel(int k) {
    g_sm_kernel = k == 1 ? 1 : 0;
    return 0;
}

extern "C" int az_diag_smallnet_stamps(unsigned long long* out, int n) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sm_stamps), sizeof(unsigned long long) * (n < 128 ? n : 128)) == hipSuccess ? 0 : -1;
}

// The round-2 kernel (A/B and the bitwise-equality test of k_smallnet_g; its timing-only
// variants are gone, their measurements are in profiles/r03e_smallnet_diag_variants.txt).
// NW = 4: one wave per SIMD, each wave all 64 output channels of its 4 pixel fragments.  NW = 8
// (default; AZ_SM_WAVES=4 selects the other): two waves per SIMD, wave w owns the pixel fragments
// of group w & 3 and output channels 32 (w >> 2) .. +31.  Measured (phase stamps, 256 boards): the
// layers take the same 11.3k cycles either way -- every layer ends in a block-wide epilogue and
// barrier that no MFMA can overlap, one board per CU -- while the prologue, pool and head convs
// are 2.4 us shorter with 8 waves.
template <int HB, int NW = 4>
__global__ __launch_bounds__(64 * NW, 1) void k_smallnet_r2(SmallNetArgs p) {
    typedef SmGeom<HB, NW> GM;
    constexpr int NT = 64 * NW;                          // threads
    constexpr int WG = GM::WG, HW = GM::HW, NFRAG = GM::NFRAG, FPW = GM::FPW, NSLOT = GM::NSLOT, DIST = GM::DIST;
    constexpr int JN = GM::JN;
    __shared__ __attribute__((aligned(16))) uint8_t lds[GM::LDS];
    uint8_t* imgX = lds;
    uint8_t* imgY = lds + GM::IMG;
    uint8_t* wbuf = lds + 2 * GM::IMG;
    float* bsm = reinterpret_cast<float*>(wbuf + NSLOT * GM::WT);   // [L][64] biases

    const int b = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63;
    // the leaf record's bytes of this thread's pixel and its meta ints, fetched first: the batch
    // index loads beside m_limit (clamped: entries past the active boards are stale), the record
    // right after it
    int rv = 0;
    int meta[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (p.rec) {
        const int gi = p.rec_identity ? min(b, p.rec_n - 1) : min(max(p.gidx[b], 0), p.rec_n - 1);
        const uint8_t* rec = p.rec + (size_t)gi * AZ_REC_BYTES;
        rv = tid < HW ? rec[tid] : 0;
        const int4 m0 = *reinterpret_cast<const int4*>(rec + AZ_REC_META);
        const int4 m1 = *reinterpret_cast<const int4*>(rec + AZ_REC_META + 16);
        meta[0] = m0.x; meta[1] = m0.y; meta[2] = m0.z; meta[3] = m0.w;
        meta[4] = m1.x; meta[5] = m1.y; meta[6] = m1.z; meta[7] = m1.w;
    }
    if (p.m_limit && b >= *p.m_limit) return;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wp = wave & 3;                             // pixel group: fragments wp + 4 i
    const int j0 = (wave >> 2) * JN;                     // first 16-channel output block of this wave
    const int L = 2 * p.blocks + 1;
    const int S = 9 * L;                                 // weight tiles streamed: (layer, tap)
    sm_stamp(p, 0);

    // weight tile s -> ring slot s % NSLOT: 512 pieces of 16 B, two per thread; LDS position (row n,
    // physical chunk pc) holds logical chunk pc ^ (n & 7) (the swizzle applied at the source).
    // Past the last tile the last tile is reloaded into the free slot, so every tap issues the
    // same two loads and the vmcnt budget is a constant.
    constexpr int WPT = 512 / NT;                        // weight pieces per thread per tile
    auto issue_w = [&](int s) {
        uint8_t* dst = wbuf + (s % NSLOT) * GM::WT;
        const int sl = s < S ? s : S - 1;
#pragma unroll
        for (int j = 0; j < WPT; ++j) {
            const int P = j * NT + tid, n = P >> 3, pc = P & 7, k = pc ^ (n & 7);
            const uint16_t* src = p.W + ((size_t)sl * SF + n) * SF + 8 * k;
            __builtin_amdgcn_global_load_lds((const void*)src, (lds_void_t*)(dst + (j * NT + wave * 64) * 16), 16, 0, 0);
        }
    };
    for (int s = 0; s < DIST; ++s) issue_w(s);

    // zero both halo images (borders and dead columns stay zero), the input planes into Y, biases
    for (int i = tid; i < 2 * GM::IMG / 16; i += NT) *reinterpret_cast<uint4*>(imgX + i * 16) = uint4{0, 0, 0, 0};
    for (int i = tid; i < L * SF; i += NT) bsm[i] = p.bias[i];
    __syncthreads();
    // the head 1x1 conv weights, transposed to [c][o], fetched now (written to LDS after the trunk)
    constexpr int HWT = SF * SF / NT;                    // weights per thread (2 * HC == SF outputs)
    float wpre[HWT];
    auto head_w = [&]() {
#pragma unroll
        for (int k = 0; k < HWT; ++k) {
            const int i = tid + NT * k, o = i / SF, c = i - o * SF;
            wpre[k] = o < p.HC ? p.Wpc[o * SF + c] : p.Wvc[(o - p.HC) * SF + c];
        }
    };
    if constexpr (NW == 4) head_w();                     // NW = 8: after the trunk (registers)
    if (p.rec) {
        // the search's leaf record: the 16 planes of this thread's cell built here (leaf_planes.h)
        static_assert(HW <= 256, "one cell per thread");
        if (tid < HW) {
            const int px = tid;
            float c[16];
            az_leaf_planes_v(rv, 0, meta, 0, HB, px, c);
            const int y = px / HB, x = px - y * HB;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                f16x8 o = {(_Float16)c[8 * h], (_Float16)c[8 * h + 1], (_Float16)c[8 * h + 2], (_Float16)c[8 * h + 3],
                           (_Float16)c[8 * h + 4], (_Float16)c[8 * h + 5], (_Float16)c[8 * h + 6], (_Float16)c[8 * h + 7]};
                *reinterpret_cast<f16x8*>(imgY + img_off((y + 1) * WG + x + 1, h)) = o;
            }
        }
    } else {
        const float* x0 = p.x0 + (size_t)b * HW * 16;
        for (int i = tid; i < HW * 2; i += NT) {           // (pixel, 8-channel half) of the 16 input channels
            const int px = i >> 1, h = i & 1;
            const float4 u = *reinterpret_cast<const float4*>(x0 + px * 16 + 8 * h);
            const float4 v = *reinterpret_cast<const float4*>(x0 + px * 16 + 8 * h + 4);
            f16x8 o = {(_Float16)u.x, (_Float16)u.y, (_Float16)u.z, (_Float16)u.w,
                       (_Float16)v.x, (_Float16)v.y, (_Float16)v.z, (_Float16)v.w};
            const int y = px / HB, x = px - y * HB;
            *reinterpret_cast<f16x8*>(imgY + img_off((y + 1) * WG + x + 1, h)) = o;
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    sm_stamp(p, 1);

    const int l16 = lane & 15, lg = lane >> 4;
    f32x4v acc[FPW][JN];
    f32x4v xr[FPW][JN];                                  // the lane's residual-stream values (fp32), kept in registers
    f16x8 fa[3][JN], fb[3][FPW];                         // operand fragments, three buffers: reads run 2 steps ahead

    // one (tap, 32-channel chunk) step: fragments into buffer `r` / MFMAs from buffer `r`
    // fragment reads as inline-asm ds_read_b128 with explicit lgkmcnt waits: the compiler's own
    // waits drained to lgkmcnt(0) before every other step's MFMAs, i.e. the next step's reads had to
    // land before this step's MFMAs could issue (no prefetch distance for half the steps)
    auto rd = [&](f16x8& d, const uint8_t* ptr) {
        asm volatile("ds_read_b128 %0, %1" : "=v"(d) : "v"((uint32_t)(uintptr_t)ptr) : "memory");
    };
    auto load = [&](int r, const uint8_t* src, int s, auto tc, auto kc) {
        constexpr int t = decltype(tc)::value, kk = decltype(kc)::value;
        constexpr int sh = (t / 3) * WG + (t % 3);
        const uint8_t* wt = wbuf + (s % NSLOT) * GM::WT;
        // NW = 8: recompute the lane's fragment addresses at every step (an opaque copy of the lane
        // id): hoisted out of the layer loop, the 18 steps' addresses alone would spill the
        // 256-register budget of two waves per SIMD
        int ln = lane;
        if constexpr (NW == 8) asm volatile("" : "+v"(ln));
        const int l16 = ln & 15, lg = ln >> 4;
        static_for<0, JN>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            rd(fa[r][j], wt + img_off(16 * (j0 + j) + l16, 4 * kk + lg));
        });
        static_for<0, FPW>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            const int f = wp + 4 * i;
            if (NFRAG % 4 == 0 || f < NFRAG)
                rd(fb[r][i], src + img_off(16 * f + l16 + sh, 4 * kk + lg));
        });
    };
    // wait until at most N fragment reads are outstanding (the next step's), then tie buffer r's
    // fragments to that point so no MFMA reading them is scheduled above the wait
    auto certify = [&](auto rc, auto nc) {
        constexpr int R = decltype(rc)::value, N = decltype(nc)::value;
        certify_frags<N>(fa[R], fb[R]);
    };
    static_assert(NFRAG % 4 == 0, "every pixel-wave loads FPW fragments (the certify counts)");
    auto mma = [&](int r) {
        static_for<0, FPW>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            if (NFRAG % 4 == 0 || wp + 4 * i < NFRAG)
                static_for<0, JN>([&](auto jc) {
                    constexpr int j = decltype(jc)::value;
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[r][j], fb[r][i], acc[i][j], 0, 0, 0);
                });
        });
    };
    // epilogue: lane holds channels 16j + 4lg + e of output grid row q
    auto epilogue = [&](int layer, uint8_t* dst) {
        const bool odd = layer & 1;
        static_for<0, FPW>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            const int f = wp + 4 * i;
            const int q = 16 * f + l16, y = q / WG, x = q - y * WG;
            const bool live = f < NFRAG && y < HB && x < HB;
            const int row = (y + 1) * WG + x + 1;
            static_for<0, JN>([&](auto jc) {
                constexpr int j = decltype(jc)::value;
                const int c0 = 16 * (j0 + j) + 4 * lg;
                f32x4v v = acc[i][j];
                if (layer > 0 && !odd && p.residual) v += xr[i][j];
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.0f);
                if (!odd) xr[i][j] = v;
                typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
                const f16x4 h = {(_Float16)v[0], (_Float16)v[1], (_Float16)v[2], (_Float16)v[3]};
                if (live) *reinterpret_cast<f16x4*>(dst + img_off(row, c0 >> 3) + (c0 & 7) * 2) = h;
            });
        });
    };
    // One layer: 9 taps x NCH chunks.  The weight tile of tap s+1 is certified (landed + barrier)
    // before tap s starts, so the last step of a tap prefetches the next tap's fragments.
    auto run_layer = [&](int layer, auto nchc) {
        constexpr int NCH = decltype(nchc)::value;
        const bool odd = layer & 1;
        const uint8_t* src = odd ? imgX : imgY;
        uint8_t* dst = odd ? imgY : imgX;
        static_for<0, JN>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            const f32x4v bv = *reinterpret_cast<const f32x4v*>(bsm + layer * SF + 16 * (j0 + j) + 4 * lg);
            static_for<0, FPW>([&](auto ic) { acc[decltype(ic)::value][j] = bv; });
        });
        const int s0 = layer * 9;
        // step x's fragments are read at step x - 2 (buffer x % 3); the two steps of a layer's first
        // tap before the loop.  A step's reads are certified once at most the younger batches are
        // outstanding.  Tile (tap) t+1 is certified before tap t starts, so reads one tap ahead are legal.
        constexpr int NSTEP = 9 * NCH;
        auto LD = [](int x) constexpr { return x < NSTEP; };
        load(0, src, s0, std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{});
        if constexpr (LD(1))
            load(1, src, s0 + 1 / NCH, std::integral_constant<int, 1 / NCH>{}, std::integral_constant<int, 1 % NCH>{});
        static_for<0, NSTEP>([&](auto qc) {
            constexpr int q = decltype(qc)::value, t = q / NCH, kk = q % NCH, r = q % 3;
            if constexpr (kk == 0) issue_w(s0 + t + DIST);   // its slot was last read at tap s - 3
            if constexpr (LD(q + 2))
                load((q + 2) % 3, src, s0 + (q + 2) / NCH, std::integral_constant<int, (q + 2) / NCH>{},
                     std::integral_constant<int, (q + 2) % NCH>{});
            constexpr int younger = ((LD(q + 1) ? 1 : 0) + (LD(q + 2) ? 1 : 0)) * (JN + FPW);
            certify(std::integral_constant<int, r>{}, std::integral_constant<int, (younger > 15 ? 15 : younger)>{});   // lgkmcnt <= 15
            // pin the order: the next steps' reads are in flight while this step's MFMAs issue
            __builtin_amdgcn_sched_barrier(0);
            mma(r);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (kk == NCH - 1) {
                // tile s+2 landed (s+3..s+DIST stay in flight: no __syncthreads, whose vmcnt(0) would
                // drain them); the epilogue's image writes are complete before the barrier
                // (DIST - 2) tiles of WPT loads each stay in flight
                if constexpr (t == 8) {
                    if (layer == 5) sm_stamp(p, 52);             // diagnostic: MFMAs of the layer issued
                    epilogue(layer, dst);
                    if (layer == 5) sm_stamp(p, 53);             // epilogue issued
                    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"i"((DIST - 2) * WPT) : "memory");
                } else {
                    if (layer == 5) sm_stamp(p, 43 + t);         // tap t's MFMAs issued (before the wait)
                    asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"i"((DIST - 2) * WPT) : "memory");
                }
            }
        });
    };
    run_layer(0, std::integral_constant<int, 1>{});
    sm_stamp(p, 2);
    for (int layer = 1; layer < L; ++layer) {
        run_layer(layer, std::integral_constant<int, 2>{});
        sm_stamp(p, 2 + layer);
    }
    __syncthreads();                                     // every wave's reload DMAs into the ring landed

    // the fp32 stream to LDS (over the two images), adaptive average pool to P x P cells (torch
    // adaptive_avg_pool2d bins), then the policy / value 1x1 convs (BN folded, k-ordered fp32 FMA
    // chain + bias, ReLU); the 1x1 weights are staged transposed ([c][o]) in the ring
    if constexpr (NW == 8) head_w();
    uint8_t* xs = lds;
    static_for<0, FPW>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        const int f = wp + 4 * i;
        const int q = 16 * f + l16, y = q / WG, x = q - y * WG;
        if (f < NFRAG && y < HB && x < HB)
            static_for<0, JN>([&](auto jc) {
                constexpr int j = decltype(jc)::value;
                *reinterpret_cast<f32x4v*>(xs + xs_off(y * HB + x, (16 * (j0 + j) + 4 * lg) >> 2)) = xr[i][j];
            });
    });
    const int P = p.P, PP = P * P, HC = p.HC;
    constexpr int HO = SF;                               // 2 * HC head outputs
    float* pooled = reinterpret_cast<float*>(wbuf);      // [64 c][64 cells] (cells >= PP zero)
    float* wt = pooled + SF * 64;                        // [64 c][HO o] (policy outputs, then value)
#pragma unroll
    for (int k = 0; k < HWT; ++k) {
        const int i = tid + NT * k, o = i / SF, c = i - o * SF;
        wt[c * HO + o] = wpre[k];
    }
    for (int i = tid; i < SF * 64; i += NT) pooled[i] = 0.0f;
    __syncthreads();
    sm_stamp(p, 40);
    for (int i = tid; i < PP * (SF / 4); i += NT) {
        const int cell = i / (SF / 4), c4 = i - cell * (SF / 4), oy = cell / P, ox = cell - oy * P;
        const int y0 = (oy * HB) / P, y1 = ((oy + 1) * HB + P - 1) / P;
        const int xa = (ox * HB) / P, xb = ((ox + 1) * HB + P - 1) / P;
        f32x4v sum = {0.0f, 0.0f, 0.0f, 0.0f};
        for (int y = y0; y < y1; ++y)
            for (int x = xa; x < xb; ++x) sum += *reinterpret_cast<const f32x4v*>(xs + xs_off(y * HB + x, c4));
        const float cnt = (float)((y1 - y0) * (xb - xa));
#pragma unroll
        for (int e = 0; e < 4; ++e) pooled[(4 * c4 + e) * 64 + cell] = sum[e] / cnt;
    }
    __syncthreads();
    sm_stamp(p, 41);
    // head 1x1 convs on the f32 MFMA (v_mfma_f32_16x16x4_f32: an exact k-ordered fmaf chain, as
    // gemm_f32): D[o][cell] = sum_c W[o][c] pooled[cell][c]; wave w owns cells 16w..16w+15
    {
        const int cell = 16 * wp + l16;                  // wave w: cells 16 (w & 3) .., outputs 16 (j0 + j) ..
        f32x4v hacc[JN] = {};
        for (int kb = 0; kb < SF / 4; ++kb) {
            const int c = 4 * kb + lg;
            const float bv = pooled[c * 64 + cell];
#pragma unroll
            for (int j = 0; j < JN; ++j)
                hacc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(wt[c * HO + 16 * (j0 + j) + l16], bv, hacc[j], 0, 0, 0);
        }
        if (cell < PP) {
#pragma unroll
            for (int j = 0; j < JN; ++j) {
                const int o = 16 * (j0 + j) + 4 * lg;       // 4 consecutive outputs, all policy or all value
                const bool pol = o < HC;
                const int oc = pol ? o : o - HC;
                const float* bias = (pol ? p.bpc : p.bvc) + oc;
                f32x4v v;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float t = hacc[j][e] + bias[e];
                    v[e] = t > 0.0f ? t : 0.0f;
                }
                *reinterpret_cast<f32x4v*>((pol ? p.pp : p.vp) + ((size_t)b * PP + cell) * HC + oc) = v;
            }
        }
    }
    sm_stamp(p, 42);
}

namespace {
// ------------------------------------------------------------------------------------------------
// k_smallnet_g (round 3, the shipped kernel): the same fused forward, rebuilt around what the
// round-2 kernel's phase stamps measured (profiles/r03e_smallnet_diag_variants.txt, r03f_*): its 18
// steps of a layer ran at ~2x the MFMA time, and each layer paid ~2.4k cycles of epilogue on top.
//  * operand addresses are a per-lane base plus a compile-time offset (ds_read_b128 offset:imm), so
//    a step issues its fragment reads and 8 MFMAs with no address VALU (the round-2 kernel
//    recomputed 6 XOR-swizzled addresses per step: ~40 VALU, more issue cycles than its MFMAs at
//    two waves per SIMD).  Activation rows are padded to RS = 160 B instead of swizzled: every tap
//    shift of a fragment is then a constant offset, and the 16-lane groups of ds_read_b128 still
//    hit 16 distinct 16-B bank slots (10 r + c mod 16 over a group's rows r and chunks c; 128, 144
//    and 192 B strides conflict);
//  * the weights stream from L1 / L2 straight into registers (below), so the LDS carries only
//    activations and a layer has one barrier (a variant with an LDS weight ring and compile-time
//    slots over layer pairs measured 57.9 vs 55.7 us per forward, profiles/r03f_smallnet_ab.txt);
//  * layers run in pairs (first / second conv of a residual block) with the role compile-time: no
//    runtime selects in the epilogue, which is one v_med3 per value (ReLU and the dead-row mask in
//    one: med3(v, 0, +inf) on live rows, med3(v, 0, 0) = 0 on the grid's dead columns, which land
//    on the halo's zero padding) plus the fp16 pack and one ds_write_b64;
//  * the prologue zeroes only the halo rows no epilogue writes; the adaptive pool issues all its
//    loads before the y-major sums.
// Arithmetic is the round-2 kernel's: the same MFMAs in the same order (tap-major, 32-channel
// chunk minor), fp32 residual stream in registers, fp16 activations rounded to nearest even
// (tests/test_gpu_net.py::test_gpu_smallnet_matches_round2_kernel: bitwise equal).
constexpr int RS = 160;          // activation row stride, bytes (64 fp16 channels + 32 B pad)

template <int HB, int NW>
struct Sm2 {                                             // the board's geometry in k_smallnet_g
    static constexpr int WG = HB + 2, HW = HB * HB, GRID = HB * WG;
    static constexpr int NFRAG = (GRID + 15) / 16;       // 16-row pixel fragments (wave wp: wp + 4 i)
    static constexpr int FPW = NFRAG / 4;
    static constexpr int JN = 16 / NW;                   // 16-channel output blocks per wave
    static constexpr int NT = 64 * NW;
    static constexpr int IR = NFRAG * 16 + 2 * WG + 2;   // halo rows the last fragment's taps read
    static constexpr int IMG = IR * RS;
    static constexpr int MAXL = 32;                      // bias rows (L <= 31: the epilogue reads row L)
    static_assert(NFRAG % 4 == 0, "four pixel groups of FPW fragments");
    static_assert(HW * SF * 4 <= 2 * IMG, "fp32 stream does not fit over the images");
    static_assert(64 * RS * (FPW - 1) + RS * (2 * WG + 2) + 64 < 65536, "activation offsets fit offset:imm");
};

template <int OFF, typename T>
__device__ __forceinline__ void ds_rd(T& d, uint32_t base) {
    static_assert(sizeof(T) == 16, "b128");
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d) : "v"(base), "i"(OFF) : "memory");
}
template <int OFF>
__device__ __forceinline__ void ds_wr64(uint32_t base, uint32_t lo, uint32_t hi) {
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    const u32x2 v = {lo, hi};
    asm volatile("ds_write_b64 %0, %1 offset:%2" ::"v"(base), "v"(v), "i"(OFF) : "memory");
}
__device__ __forceinline__ uint32_t pack_f16(float a, float b) {
    typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
    const f16x2 h = {(_Float16)a, (_Float16)b};
    return __builtin_bit_cast(uint32_t, h);
}
// two fp32 -> bf16, round to nearest even (finite inputs), low half = a
__device__ __forceinline__ uint32_t pack_bf16(float a, float b) {
    auto r = [](float f) {
        uint32_t u = __float_as_uint(f);
        u += 0x7fffu + ((u >> 16) & 1u);
        return u >> 16;
    };
    return r(a) | (r(b) << 16);
}

template <int PT, typename F>
__device__ __forceinline__ f32x4v x3_mma(const F& w, const F& a, const f32x4v& c) {
    if constexpr (PT == 2) return __builtin_amdgcn_mfma_f32_16x16x32_f16(w, a, c, 0, 0, 0);
    else return __builtin_amdgcn_mfma_f32_16x16x32_bf16(w, a, c, 0, 0, 0);
}
// two fp32 -> a hi pair and a lo pair (x - hi) of 16-bit pieces: PT 1 bf16, PT 2 fp16
template <int PT>
__device__ __forceinline__ void split_pair(float a, float b, uint32_t& h, uint32_t& l) {
    if constexpr (PT == 1) {
        h = pack_bf16(a, b);
        l = pack_bf16(a - __uint_as_float(h << 16), b - __uint_as_float(h & 0xffff0000u));
    } else {
        typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
        const f16x2 x = {(_Float16)a, (_Float16)b};
        h = __builtin_bit_cast(uint32_t, x);
        l = pack_f16(a - (float)x[0], b - (float)x[1]);
    }
}

template <int V> using IC = std::integral_constant<int, V>;
enum { ROLE_IN = 0, ROLE_ODD = 1, ROLE_EVEN = 2 };

// adaptive average pool of the fp32 stream xs ([HW][64], xs_off layout) to P x P cells (torch
// adaptive_avg_pool2d bins, y-major sums from 0, / count): item i = (c4 = i / PP, cell = i % PP), so
// consecutive lanes write consecutive cells of pooled [64 c][64 cells].  PC = P at compile time (the
// bins become constants) or 0 (runtime P); bins of at most 3 x 3 issue every load before the sums.
template <int HB, int PC, int NT>
__device__ __forceinline__ void pool_cells(const uint8_t* xs, float* pooled, int tid, int Prt = 0) {
    if constexpr (PC > 0 && (HB + PC - 1) / PC + 1 <= 3) {
        // compile-time bins of at most 3 x 3: the loads of all the thread's items are issued before
        // any sum or store (the stores to pooled would otherwise fence the next item's loads)
        constexpr int PP = PC * PC, NI = (PP * (SF / 4) + NT - 1) / NT;
        f32x4v v[NI][3][3];
#pragma unroll
        for (int k = 0; k < NI; ++k) {
            const int i = tid + NT * k, ii = i < PP * (SF / 4) ? i : 0;
            const int c4 = ii / PP, cell = ii - c4 * PP, oy = cell / PC, ox = cell - oy * PC;
            const int y0 = (oy * HB) / PC, xa = (ox * HB) / PC;
#pragma unroll
            for (int dy = 0; dy < 3; ++dy)
#pragma unroll
                for (int dx = 0; dx < 3; ++dx) {
                    const int y = min(y0 + dy, HB - 1), x = min(xa + dx, HB - 1);
                    v[k][dy][dx] = *reinterpret_cast<const f32x4v*>(xs + xs_off(y * HB + x, c4));
                }
        }
#pragma unroll
        for (int k = 0; k < NI; ++k) {
            const int i = tid + NT * k;
            if (i >= PP * (SF / 4)) break;
            const int c4 = i / PP, cell = i - c4 * PP, oy = cell / PC, ox = cell - oy * PC;
            const int y0 = (oy * HB) / PC, y1 = ((oy + 1) * HB + PC - 1) / PC;
            const int xa = (ox * HB) / PC, xb = ((ox + 1) * HB + PC - 1) / PC;
            f32x4v sum = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
            for (int dy = 0; dy < 3; ++dy)
#pragma unroll
                for (int dx = 0; dx < 3; ++dx)
                    if (y0 + dy < y1 && xa + dx < xb) sum += v[k][dy][dx];
            const float cnt = (float)((y1 - y0) * (xb - xa));
#pragma unroll
            for (int e = 0; e < 4; ++e) pooled[(4 * c4 + e) * 64 + cell] = sum[e] / cnt;
        }
        return;
    }
    const int P = PC ? PC : Prt, PP = P * P;
    for (int i = tid; i < PP * (SF / 4); i += NT) {
        const int c4 = i / PP, cell = i - c4 * PP, oy = cell / P, ox = cell - oy * P;
        const int y0 = (oy * HB) / P, y1 = ((oy + 1) * HB + P - 1) / P;
        const int xa = (ox * HB) / P, xb = ((ox + 1) * HB + P - 1) / P;
        f32x4v sum = {0.0f, 0.0f, 0.0f, 0.0f};
        if (y1 - y0 <= 3 && xb - xa <= 3) {
            f32x4v v[3][3];
#pragma unroll
            for (int dy = 0; dy < 3; ++dy)
#pragma unroll
                for (int dx = 0; dx < 3; ++dx) {
                    const int y = min(y0 + dy, HB - 1), x = min(xa + dx, HB - 1);
                    v[dy][dx] = *reinterpret_cast<const f32x4v*>(xs + xs_off(y * HB + x, c4));
                }
#pragma unroll
            for (int dy = 0; dy < 3; ++dy)
#pragma unroll
                for (int dx = 0; dx < 3; ++dx)
                    if (y0 + dy < y1 && xa + dx < xb) sum += v[dy][dx];
        } else {
            for (int y = y0; y < y1; ++y)
                for (int x = xa; x < xb; ++x) sum += *reinterpret_cast<const f32x4v*>(xs + xs_off(y * HB + x, c4));
        }
        const float cnt = (float)((y1 - y0) * (xb - xa));
#pragma unroll
        for (int e = 0; e < 4; ++e) pooled[(4 * c4 + e) * 64 + cell] = sum[e] / cnt;
    }
}

}  // namespace

namespace {
// k_smallnet_g: k_smallnet with the weights streamed from L1 / L2 straight into registers instead of
// through an LDS ring.  Per 32-channel step a wave loads its JN weight fragments (1 KB each,
// fragment-major Wf: one coalesced global_load_dwordx4 per lane) PW = 6 steps ahead into a 6-deep
// register ring whose slot is the step's global index mod 6 (compile-time: layer 0 has 9 steps, a
// trunk layer 18, so every trunk layer starts at slot 3).  The LDS then carries only activation
// fragments (4 ds_read_b128 per step instead of 6, and no 8 KB tile DMA per tap), and a layer has
// one barrier, at its end.  Waves of a pixel group share their weight fragments through the CU's
// L1.  Arithmetic identical to k_smallnet (same MFMA order, epilogue).
template <int HB, int NW>
struct SmG {
    typedef Sm2<HB, NW> B;
    static constexpr int PW = 6;                         // weight prefetch distance = ring depth (steps)
    static constexpr int OX = 0, OY = B::IMG, OB = 2 * B::IMG;
    static constexpr int OS = OB;                        // pool / head staging (after the trunk, over the biases)
    static constexpr int LDS = OB + 2 * SF * SF * 4 > OB + B::MAXL * SF * 4 ? OB + 2 * SF * SF * 4 : OB + B::MAXL * SF * 4;
    static_assert(LDS <= 160 * 1024, "");
    static_assert(9 % 3 == 0 && 18 % PW == 0 && 9 % PW == 3, "trunk layers start at ring slot 3");
};

}  // namespace


// The fused forward's tail, shared by k_smallnet_g and k_smallnet_x3: the fp32 residual stream
// (registers xr) staged in LDS, the adaptive pool, and the two head 1x1 convs (f32 MFMA, exact f32
// products) with bias + ReLU into pp / vp.  wpre: the transposed head weights prefetched at start.
template <int HB, int NW, int FPW, int JN, int HWT>
__device__ __forceinline__ void smallnet_tail(const SmallNetArgs& p, uint8_t* lds, int OS, const f32x4v (&xr)[FPW][JN],
                                              const float (&wpre)[HWT], int b, int tid, int wp, int l16, int lg, int J0) {
    typedef Sm2<HB, NW> G;
    constexpr int NT = G::NT, WG = G::WG;
    uint8_t* xs = lds;
    static_for<0, FPW>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        const int q = 16 * (wp + 4 * i) + l16, y = q / WG, x = q - y * WG;
        if (y < HB && x < HB)
            static_for<0, JN>([&](auto jc) {
                constexpr int j = decltype(jc)::value;
                *reinterpret_cast<f32x4v*>(xs + xs_off(y * HB + x, (16 * (J0 + j) + 4 * lg) >> 2)) = xr[i][j];
            });
    });
    const int P = p.P, PP = P * P, HC = p.HC;
    constexpr int HO = SF;
    // the head biases (global loads) in flight during the staging and the pool
    const int cell = 16 * wp + l16;
    f32x4v hbias[JN];
#pragma unroll
    for (int j = 0; j < JN; ++j) {
        const int o = 16 * (J0 + j) + 4 * lg;
        const float* bias = o < HC ? p.bpc + o : p.bvc + (o - HC);
#pragma unroll
        for (int e = 0; e < 4; ++e) hbias[j][e] = bias[e];
    }
    float* pooled = reinterpret_cast<float*>(lds + OS);
    float* wt = pooled + SF * 64;
#pragma unroll
    for (int k = 0; k < HWT; ++k) wt[tid + NT * k] = wpre[k];
    for (int i = tid; i < SF * (64 - PP); i += NT) {
        const int c = i / (64 - PP), cell = PP + (i - c * (64 - PP));
        pooled[c * 64 + cell] = 0.0f;
    }
    sm_stamp(p, 56);
    __syncthreads();
    sm_stamp(p, 40);
    if (P == 8) pool_cells<HB, 8, NT>(xs, pooled, tid);
    else pool_cells<HB, 0, NT>(xs, pooled, tid, P);
    sm_stamp(p, 57);
    __syncthreads();
    sm_stamp(p, 41);
    {
        // every operand read before the first MFMA (one LDS round trip), then the k-ordered chain
        f32x4v hacc[JN] = {};
        float pv[SF / 4], wv[SF / 4][JN];
#pragma unroll
        for (int kb = 0; kb < SF / 4; ++kb) {
            const int c = 4 * kb + lg;
            pv[kb] = pooled[c * 64 + cell];
#pragma unroll
            for (int j = 0; j < JN; ++j) wv[kb][j] = wt[c * HO + 16 * (J0 + j) + l16];
        }
#pragma unroll
        for (int kb = 0; kb < SF / 4; ++kb)
#pragma unroll
            for (int j = 0; j < JN; ++j) hacc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv[kb][j], pv[kb], hacc[j], 0, 0, 0);
        sm_stamp(p, 58);
        if (cell < PP) {
#pragma unroll
            for (int j = 0; j < JN; ++j) {
                const int o = 16 * (J0 + j) + 4 * lg;
                const bool pol = o < HC;
                const int oc = pol ? o : o - HC;
                f32x4v v;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float t = hacc[j][e] + hbias[j][e];
                    v[e] = t > 0.0f ? t : 0.0f;
                }
                *reinterpret_cast<f32x4v*>((pol ? p.pp : p.vp) + ((size_t)b * PP + cell) * HC + oc) = v;
            }
        }
    }
}

template <int HB, int NW, bool RES>
__global__ __launch_bounds__(64 * NW, 1) void k_smallnet_g(SmallNetArgs p) {
    typedef Sm2<HB, NW> G;
    typedef SmG<HB, NW> H;
    constexpr int NT = G::NT, WG = G::WG, HW = G::HW, FPW = G::FPW, JN = G::JN, PW = H::PW;
    __shared__ __attribute__((aligned(16))) uint8_t lds[H::LDS];
    const uint32_t L0 = (uint32_t)(uintptr_t)lds;
    const int b = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63;
    const int gq = tid, gy = gq / WG, gx = gq - gy * WG;
    const bool glive = gq < G::NFRAG * 16 && gy < HB && gx < HB;
    float vmax = 0.0f;                             // largest fp16 activation written (the range guard)
    int rv = 0;
    int meta[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (p.rec) {
        const int gi = p.rec_identity ? min(b, p.rec_n - 1) : min(max(p.gidx[b], 0), p.rec_n - 1);
        const uint8_t* rec = p.rec + (size_t)gi * AZ_REC_BYTES;
        rv = glive ? rec[gy * HB + gx] : 0;
        const int4 m0 = *reinterpret_cast<const int4*>(rec + AZ_REC_META);
        const int4 m1 = *reinterpret_cast<const int4*>(rec + AZ_REC_META + 16);
        meta[0] = m0.x; meta[1] = m0.y; meta[2] = m0.z; meta[3] = m0.w;
        meta[4] = m1.x; meta[5] = m1.y; meta[6] = m1.z; meta[7] = m1.w;
    }
    if (p.m_limit && b >= *p.m_limit) return;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wp = wave & 3;
    const int J0 = (wave >> 2) * JN;
    const int l16 = lane & 15, lg = lane >> 4;
    const int L = 2 * p.blocks + 1;
    const int NFR = L * 18;                              // weight fragment groups (layer, tap, kk)
    sm_stamp(p, 0);

    constexpr int HWT = SF * SF / NT;
    float wpre[HWT];
#pragma unroll
    for (int k = 0; k < HWT; ++k) {
        const int i = tid + NT * k, c = i / SF, o = i - c * SF;
        wpre[k] = o < p.HC ? p.Wpc[o * SF + c] : p.Wvc[(o - p.HC) * SF + c];
    }
    constexpr int BPT = (G::MAXL * SF + NT - 1) / NT;
    float bpre[BPT];
#pragma unroll
    for (int k = 0; k < BPT; ++k) {
        const int i = tid + NT * k;
        bpre[k] = i < L * SF ? p.bias[i] : 0.0f;
    }
    // weight register ring: fw[slot][j] = fragment group fg's block J0 + j
    f16x8 fw[PW][JN];
    const f16x8* wsrc = reinterpret_cast<const f16x8*>(p.Wf) + J0 * 64 + lane;
    auto wload = [&](auto slotc, int fg) {
        constexpr int slot = decltype(slotc)::value;
        const f16x8* src = wsrc + (size_t)min(fg, NFR - 1) * (4 * 64);
        static_for<0, JN>([&](auto jc) { fw[slot][decltype(jc)::value] = src[64 * decltype(jc)::value]; });
    };
    // layer 0 reads chunk kk = 0 of each tap: fragment group 2 t
    static_for<0, PW>([&](auto xc) { wload(xc, 2 * decltype(xc)::value); });

    {
        constexpr int TOP = WG + 1, BOT0 = G::NFRAG * 16 + WG + 1, NPAD = TOP + (G::IR - BOT0);
        for (int i = tid; i < 2 * NPAD * 8; i += NT) {
            const int img = i / (NPAD * 8), k = i - img * NPAD * 8, r = k >> 3, c = k & 7;
            const int row = r < TOP ? r : BOT0 + (r - TOP);
            *reinterpret_cast<uint4*>(lds + (img ? H::OY : H::OX) + row * RS + c * 16) = uint4{0, 0, 0, 0};
        }
        if (tid < G::NFRAG * 16) {
            float c[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) c[k] = 0.0f;
            if (glive) {
                const int px = gy * HB + gx;
                if (p.rec) {
                    az_leaf_planes_v(rv, 0, meta, 0, HB, px, c);
                } else {
                    const float* x0 = p.x0 + ((size_t)b * HW + px) * 16;
#pragma unroll
                    for (int k = 0; k < 16; k += 4) {
                        const float4 u = *reinterpret_cast<const float4*>(x0 + k);
                        c[k] = u.x; c[k + 1] = u.y; c[k + 2] = u.z; c[k + 3] = u.w;
                    }
                }
            }
            uint8_t* dst = lds + H::OY + (gq + WG + 1) * RS;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const uint4 v = {pack_f16(c[8 * h], c[8 * h + 1]), pack_f16(c[8 * h + 2], c[8 * h + 3]),
                                 pack_f16(c[8 * h + 4], c[8 * h + 5]), pack_f16(c[8 * h + 6], c[8 * h + 7])};
                *reinterpret_cast<uint4*>(dst + 16 * h) = v;
                *reinterpret_cast<uint4*>(dst + 32 + 16 * h) = uint4{0, 0, 0, 0};
            }
        }
        float* bsm = reinterpret_cast<float*>(lds + H::OB);
#pragma unroll
        for (int k = 0; k < BPT; ++k) {
            const int i = tid + NT * k;
            if (i < L * SF) bsm[i] = bpre[k];
        }
    }
    __syncthreads();
    sm_stamp(p, 1);

    const uint32_t aX = L0 + H::OX + (16 * wp + l16) * RS + 16 * lg, aY = aX + H::OY;
    const uint32_t eX = L0 + H::OX + (16 * wp + l16 + WG + 1) * RS + 32 * J0 + 8 * lg, eY = eX + H::OY;
    const uint32_t bb = L0 + H::OB + (16 * J0 + 4 * lg) * 4;
    float mlive[FPW];
#pragma unroll
    for (int i = 0; i < FPW; ++i) {
        const int q = 16 * (wp + 4 * i) + l16, y = q / WG, x = q - y * WG;
        mlive[i] = (y < HB && x < HB) ? __builtin_inff() : 0.0f;
    }

    f32x4v acc[FPW][JN];
    f32x4v xr[FPW][JN];
    f32x4v bn[JN];
    f16x8 fb[3][FPW];                                    // activation fragments (reads PF steps ahead)
    auto read_bias = [&](int layer) {
        const uint32_t a = bb + layer * (SF * 4);
        static_for<0, JN>([&](auto jc) { ds_rd<64 * decltype(jc)::value>(bn[decltype(jc)::value], a); });
    };
    read_bias(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");

    // ROLE, NCH chunks per tap, R0 = ring slot of the layer's step 0 (0 for layer 0, 3 otherwise);
    // NNCH = chunks per tap of the next layer (its fragment groups are prefetched here)
    auto run_layer = [&](int layer, auto rolec, auto nchc, auto r0c) {
        constexpr int ROLE = decltype(rolec)::value, NCH = decltype(nchc)::value, R0 = decltype(r0c)::value;
        constexpr int NSTEP = 9 * NCH, PF = NCH == 1 ? 1 : 2, NB = PF + 1;
        const uint32_t src = ROLE == ROLE_ODD ? aX : aY;
        const uint32_t dst = ROLE == ROLE_ODD ? eY : eX;
        const int fg0 = layer * 18;                      // this layer's first fragment group
        auto aload = [&](auto bufc, auto xc) {
            constexpr int buf = decltype(bufc)::value, x = decltype(xc)::value;
            constexpr int t = x / NCH, kk = x % NCH, sh = (t / 3) * WG + (t % 3);
            static_for<0, FPW>([&](auto ic) {
                constexpr int i = decltype(ic)::value;
                ds_rd<64 * RS * i + RS * sh + 64 * kk>(fb[buf][i], src);
            });
        };
        static_for<0, PF>([&](auto xc) { aload(IC<decltype(xc)::value % NB>{}, xc); });
        static_for<0, NSTEP>([&](auto qc) {
            constexpr int q = decltype(qc)::value, t = q / NCH, kk = q % NCH, r = q % NB, ws = (R0 + q) % PW;
            if constexpr (q + PF < NSTEP) aload(IC<(q + PF) % NB>{}, IC<q + PF>{});
            // the next layer's biases, mid-layer: bn's last reads (step 0's MFMAs) are long done,
            // and the reads land long before the epilogue's wait (the certify waits below count
            // them as younger reads: at most a wait for more than needed)
            if constexpr (q == NSTEP / 2) read_bias(layer + 1);
            constexpr int ahead = (NSTEP - 1 - q) < PF ? (NSTEP - 1 - q) : PF;
            certify_frags<(ahead * FPW > 15 ? 15 : ahead * FPW)>(fw[ws], fb[r]);
            __builtin_amdgcn_sched_barrier(0);
            static_for<0, FPW>([&](auto ic) {
                static_for<0, JN>([&](auto jc) {
                    constexpr int i = decltype(ic)::value, j = decltype(jc)::value;
                    // step 0 accumulates onto the bias registers (no copies into the accumulators)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fw[ws][j], fb[r][i], q == 0 ? bn[j] : acc[i][j], 0, 0, 0);
                });
            });
            // the MFMAs are left free to interleave with the ring refill (global loads) and, in the
            // last step, with the epilogue's VALU
            // the ring slot just consumed takes the fragment group PW steps ahead (possibly the next
            // layer's: 2 chunks per tap from layer 1 on)
            {
                constexpr int ahead_step = q + PW;
                if constexpr (ahead_step < NSTEP) {
                    wload(IC<ws>{}, fg0 + (ahead_step / NCH) * 2 + ahead_step % NCH);
                } else {
                    wload(IC<ws>{}, fg0 + 18 + (ahead_step - NSTEP));   // next layer: 2 chunks per tap
                }
            }
            if constexpr (kk == NCH - 1) {
                if constexpr (t < 8) if (layer == 5) sm_stamp(p, 43 + t);
                if constexpr (t == 8) {
                    static_for<0, FPW>([&](auto ic) {
                        static_for<0, JN>([&](auto jc) {
                            constexpr int i = decltype(ic)::value, j = decltype(jc)::value;
                            f32x4v v = acc[i][j];
                            if constexpr (ROLE == ROLE_EVEN && RES) v += xr[i][j];
#pragma unroll
                            for (int e = 0; e < 4; ++e) v[e] = __builtin_amdgcn_fmed3f(v[e], 0.0f, mlive[i]);
#pragma unroll
                            for (int e = 0; e < 4; ++e) vmax = __builtin_fmaxf(vmax, v[e]);
                            if constexpr (ROLE != ROLE_ODD) xr[i][j] = v;
                            ds_wr64<64 * RS * i + 32 * j>(dst, pack_f16(v[0], v[1]), pack_f16(v[2], v[3]));
                        });
                    });
                    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
                }
            }
        });
    };
    run_layer(0, IC<ROLE_IN>{}, IC<1>{}, IC<0>{});
    sm_stamp(p, 2);
    for (int layer = 1; layer < L; layer += 2) {
        run_layer(layer, IC<ROLE_ODD>{}, IC<2>{}, IC<3>{});
        sm_stamp(p, 2 + layer);
        run_layer(layer + 1, IC<ROLE_EVEN>{}, IC<2>{}, IC<3>{});
        sm_stamp(p, 3 + layer);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // the ring's trailing (clamped) loads
    if (!(vmax <= 65504.0f) && p.ovf) atomicOr(p.ovf, 1);   // fp16 overflow: the engine fails the forward
    sm_stamp(p, 54);
    __syncthreads();
    sm_stamp(p, 55);

    smallnet_tail<HB, NW>(p, lds, H::OS, xr, wpre, b, tid, wp, l16, lg, J0);
    sm_stamp(p, 42);
}

// ------------------------------------------------------------------------------------------------
// k_smallnet_x3: the fused forward in the fp32-faithful parity precisions (PT 1: AZ_PREC_BF16X3,
// PT 2: AZ_PREC_F16X3).  Every activation is carried as two 16-bit planes, hi = p(x) and lo =
// p(x - hi) for the piece type p (bf16 or fp16), and every weight likewise (fragment-major Wxh / Wxl;
// fp16 pieces of weights scaled by 2^s per output channel, the accumulators start at bias * 2^s and
// the epilogue multiplies by p.osc = 2^-s); a product is hi*hi + lo*hi + hi*lo -- three MFMAs
// (v_mfma_f32_16x16x32_bf16 / _f16) per 32-channel step, fp32 accumulation (the arithmetic of
// conv3x3_v9x3 / v7x3).  The fp32 residual stream stays in registers as in k_smallnet_g, and the
// tail (pool, head convs) is the same code.  What differs:
//  * ONE activation image per plane (hi, lo: 2 x 46.7 KB), updated IN PLACE: a layer's outputs stay
//    in the accumulators until every wave has read its last input fragment (barrier A), then the
//    epilogue writes them over the input and barrier B certifies them for the next layer -- two
//    images per plane (k_smallnet_g's X / Y) would need 187 KB;
//  * per step a wave reads 2 x FPW activation fragments (hi, lo) one step ahead and holds a 3-step
//    register ring of 2 x JN weight fragments (hi, lo; a step is 3x the MFMAs of the fp16 kernel,
//    so three steps cover the L2 latency): 24 MFMAs per step in three sweeps (Wh*Ah, Wl*Ah, Wh*Al),
//    so an accumulator is reused every JN * FPW = 8 MFMAs;
//  * layer 0 reads the input planes split the same way (hi + lo) and runs the same three sweeps.
template <int HB, int NW, bool RES, int PT>
__global__ __launch_bounds__(64 * NW, 1) void k_smallnet_x3(SmallNetArgs p) {
    typedef Sm2<HB, NW> G;
    constexpr int NT = G::NT, WG = G::WG, HW = G::HW, FPW = G::FPW, JN = G::JN;
    constexpr int PW = 3;                                // weight ring depth (steps): 9 and 18 are multiples
    constexpr int OH = 0, OL = G::IMG, OB = 2 * G::IMG, OS = OB;
    constexpr int OSC = OB + G::MAXL * SF * 4;           // PT 2: the per-channel scales [L][64] behind the biases
    constexpr int LDS = OB + 2 * SF * SF * 4 > OB + 2 * G::MAXL * SF * 4 ? OB + 2 * SF * SF * 4 : OB + 2 * G::MAXL * SF * 4;
    static_assert(LDS <= 160 * 1024, "");
    typedef typename std::conditional<PT == 2, _Float16, __bf16>::type piece_t;
    typedef piece_t bf16x8 __attribute__((ext_vector_type(8)));
    __shared__ __attribute__((aligned(16))) uint8_t lds[LDS];
    const uint32_t L0 = (uint32_t)(uintptr_t)lds;
    const int b = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63;
    const int gq = tid, gy = gq / WG, gx = gq - gy * WG;
    const bool glive = gq < G::NFRAG * 16 && gy < HB && gx < HB;
    int rv = 0;
    int meta[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (p.rec) {
        const int gi = p.rec_identity ? min(b, p.rec_n - 1) : min(max(p.gidx[b], 0), p.rec_n - 1);
        const uint8_t* rec = p.rec + (size_t)gi * AZ_REC_BYTES;
        rv = glive ? rec[gy * HB + gx] : 0;
        const int4 m0 = *reinterpret_cast<const int4*>(rec + AZ_REC_META);
        const int4 m1 = *reinterpret_cast<const int4*>(rec + AZ_REC_META + 16);
        meta[0] = m0.x; meta[1] = m0.y; meta[2] = m0.z; meta[3] = m0.w;
        meta[4] = m1.x; meta[5] = m1.y; meta[6] = m1.z; meta[7] = m1.w;
    }
    if (p.m_limit && b >= *p.m_limit) return;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wp = wave & 3;
    const int J0 = (wave >> 2) * JN;
    const int l16 = lane & 15, lg = lane >> 4;
    const int L = 2 * p.blocks + 1;
    const int NFR = L * 18;                              // weight fragment groups (layer, tap, kk)

    constexpr int HWT = SF * SF / NT;
    float wpre[HWT];
#pragma unroll
    for (int k = 0; k < HWT; ++k) {
        const int i = tid + NT * k, c = i / SF, o = i - c * SF;
        wpre[k] = o < p.HC ? p.Wpc[o * SF + c] : p.Wvc[(o - p.HC) * SF + c];
    }
    constexpr int BPT = (G::MAXL * SF + NT - 1) / NT;
    float bpre[BPT];
#pragma unroll
    for (int k = 0; k < BPT; ++k) {
        const int i = tid + NT * k;
        bpre[k] = i < L * SF ? p.bias[i] : 0.0f;
    }
    if constexpr (PT == 2) {
        float* ssm = reinterpret_cast<float*>(lds + OSC);
        for (int i = tid; i < L * SF; i += NT) ssm[i] = p.osc[i];
    }
    // weight register ring: fwh / fwl[slot][j] = fragment group fg's block J0 + j, hi / lo
    bf16x8 fwh[PW][JN], fwl[PW][JN];
    const bf16x8* wsh = reinterpret_cast<const bf16x8*>(p.Wxh) + J0 * 64 + lane;
    const bf16x8* wsl = reinterpret_cast<const bf16x8*>(p.Wxl) + J0 * 64 + lane;
    auto wload = [&](auto slotc, int fg) {
        constexpr int slot = decltype(slotc)::value;
        const size_t o = (size_t)min(fg, NFR - 1) * (4 * 64);
        static_for<0, JN>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            fwh[slot][j] = wsh[o + 64 * j];
            fwl[slot][j] = wsl[o + 64 * j];
        });
    };
    static_for<0, PW>([&](auto xc) { wload(xc, 2 * decltype(xc)::value); });   // layer 0: chunk 0 of taps 0..2

    {
        // zero the halo rows no epilogue writes (both planes) and write the input planes, split into
        // hi + lo like every other operand (the coordinate planes are not exact in 16 bits), into the
        // first 32 channels of both planes
        constexpr int TOP = WG + 1, BOT0 = G::NFRAG * 16 + WG + 1, NPAD = TOP + (G::IR - BOT0);
        for (int i = tid; i < 2 * NPAD * 8; i += NT) {
            const int pl = i / (NPAD * 8), k = i - pl * NPAD * 8, r = k >> 3, c = k & 7;
            const int row = r < TOP ? r : BOT0 + (r - TOP);
            *reinterpret_cast<uint4*>(lds + (pl ? OL : OH) + row * RS + c * 16) = uint4{0, 0, 0, 0};
        }
        if (tid < G::NFRAG * 16) {
            float c[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) c[k] = 0.0f;
            if (glive) {
                const int px = gy * HB + gx;
                if (p.rec) {
                    az_leaf_planes_v(rv, 0, meta, 0, HB, px, c);
                } else {
                    const float* x0 = p.x0 + ((size_t)b * HW + px) * 16;
#pragma unroll
                    for (int k = 0; k < 16; k += 4) {
                        const float4 u = *reinterpret_cast<const float4*>(x0 + k);
                        c[k] = u.x; c[k + 1] = u.y; c[k + 2] = u.z; c[k + 3] = u.w;
                    }
                }
            }
            const int row = gq + WG + 1;
            uint8_t* dh = lds + OH + row * RS;
            uint8_t* dl = lds + OL + row * RS;
            uint32_t hp[8], lp[8];                       // hi / lo pairs
#pragma unroll
            for (int k = 0; k < 8; ++k) split_pair<PT>(c[2 * k], c[2 * k + 1], hp[k], lp[k]);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const uint4 v = {hp[4 * h], hp[4 * h + 1], hp[4 * h + 2], hp[4 * h + 3]};
                const uint4 w = {lp[4 * h], lp[4 * h + 1], lp[4 * h + 2], lp[4 * h + 3]};
                *reinterpret_cast<uint4*>(dh + 16 * h) = v;
                *reinterpret_cast<uint4*>(dh + 32 + 16 * h) = uint4{0, 0, 0, 0};
                *reinterpret_cast<uint4*>(dl + 16 * h) = w;
                *reinterpret_cast<uint4*>(dl + 32 + 16 * h) = uint4{0, 0, 0, 0};
            }
        }
        float* bsm = reinterpret_cast<float*>(lds + OB);
#pragma unroll
        for (int k = 0; k < BPT; ++k) {
            const int i = tid + NT * k;
            if (i < L * SF) bsm[i] = bpre[k];
        }
    }
    __syncthreads();

    // fragment reads and epilogue writes through ordinary LDS pointers (compile-time offsets), so the
    // compiler orders every read before its MFMA and every write before the barriers itself
    const uint8_t* aH = lds + OH + (16 * wp + l16) * RS + 16 * lg;
    const uint8_t* aL = aH + OL;
    uint8_t* eH = lds + OH + (16 * wp + l16 + WG + 1) * RS + 32 * J0 + 8 * lg;
    uint8_t* eL = eH + OL;
    const float* bb = reinterpret_cast<const float*>(lds + OB) + 16 * J0 + 4 * lg;
    const float* sb = reinterpret_cast<const float*>(lds + OSC) + 16 * J0 + 4 * lg;
    float vmax = 0.0f;                                   // PT 2: the fp16 range guard
    float mlive[FPW];
#pragma unroll
    for (int i = 0; i < FPW; ++i) {
        const int q = 16 * (wp + 4 * i) + l16, y = q / WG, x = q - y * WG;
        mlive[i] = (y < HB && x < HB) ? __builtin_inff() : 0.0f;
    }

    f32x4v acc[FPW][JN];
    f32x4v xr[FPW][JN];
    f32x4v bn[JN];
    bf16x8 fbh[2][FPW], fbl[2][FPW];                     // activation fragments (read one step ahead)
    auto read_bias = [&](int layer) {
        static_for<0, JN>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            bn[j] = *reinterpret_cast<const f32x4v*>(bb + layer * SF + 16 * j);
        });
    };
    read_bias(0);

    auto run_layer = [&](int layer, auto rolec, auto nchc) {
        constexpr int ROLE = decltype(rolec)::value, NCH = decltype(nchc)::value;
        constexpr int NSTEP = 9 * NCH;
        const int fg0 = layer * 18;
        auto aload = [&](auto bufc, auto xc) {           // activation fragments of step x, both planes
            constexpr int buf = decltype(bufc)::value, x = decltype(xc)::value;
            constexpr int t = x / NCH, kk = x % NCH, sh = (t / 3) * WG + (t % 3);
            static_for<0, FPW>([&](auto ic) {
                constexpr int i = decltype(ic)::value, off = 64 * RS * i + RS * sh + 64 * kk;
                fbh[buf][i] = *reinterpret_cast<const bf16x8*>(aH + off);
                fbl[buf][i] = *reinterpret_cast<const bf16x8*>(aL + off);
            });
        };
        // sched_barriers keep every load where it is issued (one step ahead for the activation
        // fragments, PW steps ahead for the weight ring): left alone, the scheduler sinks each load
        // next to its first MFMA and every step waits out an L2 / LDS round trip
        aload(IC<0>{}, IC<0>{});
        static_for<0, NSTEP>([&](auto qc) {
            constexpr int q = decltype(qc)::value, r = q % 2, ws = q % PW;
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (q + 1 < NSTEP) aload(IC<(q + 1) % 2>{}, IC<q + 1>{});
            if constexpr (q == NSTEP / 2) read_bias(layer + 1);
            __builtin_amdgcn_sched_barrier(0);
            static_for<0, FPW>([&](auto ic) {
                static_for<0, JN>([&](auto jc) {
                    constexpr int i = decltype(ic)::value, j = decltype(jc)::value;
                    acc[i][j] = x3_mma<PT>(fwh[ws][j], fbh[r][i], q == 0 ? bn[j] : acc[i][j]);
                });
            });
            static_for<0, FPW>([&](auto ic) {
                static_for<0, JN>([&](auto jc) {
                    constexpr int i = decltype(ic)::value, j = decltype(jc)::value;
                    acc[i][j] = x3_mma<PT>(fwl[ws][j], fbh[r][i], acc[i][j]);
                });
            });
            static_for<0, FPW>([&](auto ic) {
                static_for<0, JN>([&](auto jc) {
                    constexpr int i = decltype(ic)::value, j = decltype(jc)::value;
                    acc[i][j] = x3_mma<PT>(fwh[ws][j], fbl[r][i], acc[i][j]);
                });
            });
            __builtin_amdgcn_sched_barrier(0);
            {
                constexpr int ahead_step = q + PW;
                if constexpr (ahead_step < NSTEP) wload(IC<ws>{}, fg0 + (ahead_step / NCH) * 2 + ahead_step % NCH);
                else wload(IC<ws>{}, fg0 + 18 + (ahead_step - NSTEP));   // next layer: 2 chunks per tap
            }
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (q == NSTEP - 1) {
                // barrier A: every wave has read its last input fragment; the outputs go in place
                __syncthreads();
                static_for<0, FPW>([&](auto ic) {
                    static_for<0, JN>([&](auto jc) {
                        constexpr int i = decltype(ic)::value, j = decltype(jc)::value;
                        f32x4v v = acc[i][j];
                        if constexpr (PT == 2) v *= *reinterpret_cast<const f32x4v*>(sb + layer * SF + 16 * j);
                        if constexpr (ROLE == ROLE_EVEN && RES) v += xr[i][j];
#pragma unroll
                        for (int e = 0; e < 4; ++e) v[e] = __builtin_amdgcn_fmed3f(v[e], 0.0f, mlive[i]);
                        if constexpr (PT == 2) {
#pragma unroll
                            for (int e = 0; e < 4; ++e) vmax = __builtin_fmaxf(vmax, v[e]);
                        }
                        if constexpr (ROLE != ROLE_ODD) xr[i][j] = v;
                        uint32_t h[2], l[2];
#pragma unroll
                        for (int e = 0; e < 2; ++e) split_pair<PT>(v[2 * e], v[2 * e + 1], h[e], l[e]);
                        constexpr int off = 64 * RS * i + 32 * j;
                        *reinterpret_cast<uint2*>(eH + off) = uint2{h[0], h[1]};
                        *reinterpret_cast<uint2*>(eL + off) = uint2{l[0], l[1]};
                    });
                });
                __syncthreads();                         // barrier B: the layer's outputs are in place
            }
        });
    };
    run_layer(0, IC<ROLE_IN>{}, IC<1>{});
    for (int layer = 1; layer < L; layer += 2) {
        run_layer(layer, IC<ROLE_ODD>{}, IC<2>{});
        run_layer(layer + 1, IC<ROLE_EVEN>{}, IC<2>{});
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // the ring's trailing (clamped) loads
    if (PT == 2 && !(vmax <= 65504.0f) && p.ovf) atomicOr(p.ovf, 1);   // fp16 pieces: the engine fails the forward
    __syncthreads();
    smallnet_tail<HB, NW>(p, lds, OS, xr, wpre, b, tid, wp, l16, lg, J0);
}

bool az_smallnet_supported(int H, int C, int cin_pad, int pool, int head_channels) {
    return H == 15 && C == SF && cin_pad == 16 && pool >= 1 && pool <= 8 && 2 * head_channels == SF && head_channels % 4 == 0;
}
// layers (2 * blocks + 1) whose biases fit the kernel's LDS
int az_smallnet_max_blocks() { return (SmGeom<15>::MAXL - 1) / 2; }

int az_smallnet_launch(const SmallNetArgs& a, int B, hipStream_t st) {
    if (!az_smallnet_supported(a.H, SF, 16, a.P, a.HC)) return -1;
    if (g_sm_kernel == 1) {                              // A/B only: the round-2 kernel
        if (g_sm_waves == 4) hipLaunchKernelGGL((k_smallnet_r2<15, 4>), dim3(B), dim3(256), 0, st, a);
        else hipLaunchKernelGGL((k_smallnet_r2<15, 8>), dim3(B), dim3(512), 0, st, a);
        return 0;
    }
    if (a.Wxh) {                                         // AZ_PREC_BF16X3 (pt 1) / AZ_PREC_F16X3 (pt 2)
        if (!a.Wxl || (a.pt == 2 && !a.osc)) return -1;
        if (a.pt == 2) {
            if (a.residual) hipLaunchKernelGGL((k_smallnet_x3<15, 8, true, 2>), dim3(B), dim3(512), 0, st, a);
            else hipLaunchKernelGGL((k_smallnet_x3<15, 8, false, 2>), dim3(B), dim3(512), 0, st, a);
            return 0;
        }
        if (a.residual) hipLaunchKernelGGL((k_smallnet_x3<15, 8, true, 1>), dim3(B), dim3(512), 0, st, a);
        else hipLaunchKernelGGL((k_smallnet_x3<15, 8, false, 1>), dim3(B), dim3(512), 0, st, a);
        return 0;
    }
    if (a.residual) hipLaunchKernelGGL((k_smallnet_g<15, 8, true>), dim3(B), dim3(512), 0, st, a);
    else hipLaunchKernelGGL((k_smallnet_g<15, 8, false>), dim3(B), dim3(512), 0, st, a);
    return 0;
}
