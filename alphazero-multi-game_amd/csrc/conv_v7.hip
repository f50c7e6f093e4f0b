// conv_v7.hip -- 3x3 trunk convolution of the g8 residual stream (fp16 / bf16 MFMA, gfx950).
//
//   out[b][n][pix] = relu( sum_{tap,c} A[b][c][pix + tap] * W[n][tap][c] + bias[n] (+ res) )
//
// Same data formats as conv3x3_v6 (conv_bf16.hip): activations in the g8 layout
// [board][C/8][pixel][8] 16-bit with an int8 remainder plane of the residual stream, weights
// chunk-blocked [C/16][9][2][N][8], zero padding read from the zeroed tail behind every
// activation buffer (AZ_ACT_TAIL).  What changes is the shape of the work:
//
//  * a 256-thread block (4 waves) owns a 256-row output tile x 128 channels and needs 72 KB of
//    LDS (halo of one 32-channel chunk double-buffered, 2 x 20 KB; a 4-slot ring of per-tap
//    weight tiles, 4 x 8 KB), so TWO blocks share a CU.  The scheduler interleaves them: while one
//    block sits in a barrier or in its epilogue, the other block's waves keep the SIMD's matrix
//    pipe busy (v6 runs one 512-thread block per CU and its epilogue leaves the pipes idle);
//  * the MFMA operands are swapped (weights as the 16-row operand, activations as the 16-column
//    one), so a lane's accumulator holds 4 consecutive output CHANNELS of one pixel: the epilogue
//    joins the residual, applies the ReLU, splits the result into 16 bits + int8 remainder and
//    stores straight from registers -- no LDS staging, no block barrier, each wave on its own;
//  * one barrier per tap.  Weight tiles land 4 taps ahead; each barrier certifies the NEXT tap's
//    tile, so every fragment of tap s+1 is read during tap s's MFMAs (no read latency after a
//    barrier).  The halo of chunk c+1 is fetched during taps 0..4 of chunk c.
//
// Tile geometry (as v6): 15x15 boards use the padded grid (outputs on a 15x17 grid, one board per
// 256-row tile, 225 of 256 rows live) or DENSE tiles; every other board uses DENSE tiles (256
// consecutive pixels of the batch; taps that leave the board are zeroed in the fragments).
// The result is bit-identical to conv3x3_v6 (same products, same accumulation order).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <type_traits>

#include "net.h"

// conv3x3_v7's output stores: streaming (nt) by default; AZ_V7_ST_PLAIN=1 builds plain stores (A/B of
// the row-boundary partial writes)
#if defined(AZ_V7_ST_PLAIN) && AZ_V7_ST_PLAIN
#define AZ_V7_ST ""
#else
#define AZ_V7_ST " nt"
#endif

namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void lds_void_t;

template <int MODE>
struct H16 {                                           // MODE 2: fp16, MODE 1: bf16 (as Half16, conv_bf16.hip)
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
    static constexpr int SH = 16 - (MODE == 2 ? 11 : 8);
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

// The split-operand (x3) kernels' piece type: PT 1 = bf16 pieces (AZ_PREC_BF16X3), PT 2 = fp16 pieces
// (AZ_PREC_F16X3; weights per-output-channel power-of-2 scaled, undone in the epilogue by oscale)
template <int PT> struct X3T;
template <> struct X3T<1> {
    typedef bf16x8 frag;
    __device__ static f32x4v mma(const frag& b, const frag& a, const f32x4v& c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(b, a, c, 0, 0, 0);
    }
};
template <> struct X3T<2> {
    typedef f16x8 frag;
    __device__ static f32x4v mma(const frag& b, const frag& a, const f32x4v& c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(b, a, c, 0, 0, 0);
    }
};

__device__ __forceinline__ uint32_t lds_addr(const void* p) { return (uint32_t)(uintptr_t)p; }

#ifdef AZ_V9_STAMPS
// Diagnostic builds only (make EXTRA=-DAZ_V9_STAMPS OUT=build_stamps): wave 0 of every block of the
// selected conv3x3_v9x3 launch (ConvBf16Args::stamp == g_v9_sel) records s_memrealtime (100 MHz) at
// its start, after the prologue barrier, after the main loop, after the epilogue's stores issue and
// after they complete, plus HW_ID / XCC_ID (tools/v9_stamps.py)
constexpr int V9_MAXB = 8192;
__device__ int g_v9_sel = -1;
__device__ unsigned long long g_v9_st[V9_MAXB][5];
__device__ unsigned g_v9_hw[V9_MAXB][2];
#define V9_STAMP(k)                                                                                 \
    do {                                                                                            \
        if (p.stamp == g_v9_sel && tid == 0 && blockIdx.x < V9_MAXB) {                              \
            g_v9_st[blockIdx.x][k] = __builtin_amdgcn_s_memrealtime();                              \
            if (k == 0) {                                                                           \
                g_v9_hw[blockIdx.x][0] = __builtin_amdgcn_s_getreg((31 << 11) | 4);                 \
                g_v9_hw[blockIdx.x][1] = __builtin_amdgcn_s_getreg((31 << 11) | 20);                \
            }                                                                                       \
        }                                                                                           \
    } while (0)
#else
#define V9_STAMP(k) do { } while (0)
#endif

template <int OFF, typename F>
__device__ __forceinline__ void ds_rd(F& d, uint32_t addr) {
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d) : "v"(addr), "i"(OFF) : "memory");
}
// s_waitcnt lgkmcnt(N) with the fragments it certifies as in-out operands, so every MFMA that
// reads them is ordered after the wait (the ds_reads are inline asm the compiler does not track)
template <int N, typename F>
__device__ __forceinline__ void lgkm(F (&x)[4]) {
    asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "i"(N) : "memory");
}

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

template <int I, int N, typename Fn>
__device__ __forceinline__ void static_for(Fn&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<I + 1, N>(f);
    }
}

// Tile geometries (one board per tile unless DENSE):
//  GEO_PAD   outputs on an HB x (HB+2) grid: tap (dy, dx) of output row q is halo row q + dy*WG + dx
//            of the zero-padded (HB+2)^2 halo (two dead columns per grid row; 15x15: 225 of 256 rows live)
//  GEO_SLIM  outputs on an HB x (HB+1) grid over a halo of HB+2 rows of HB+1 columns whose column 0
//            is zero: the one zero column is the right neighbour of x = HB-1 (the next grid row's
//            column 0) and the left neighbour of x = 0, so no tap needs masking; one dead column per
//            grid row (15x15: 240 rows = 15 fragments of 16; the 16th fragment of the tile reads the
//            halo's all-zero rows >= 256 instead, so its MFMAs run on zero operands, which cost the
//            power-limited chip little -- a branch around them would route every accumulator
//            through phi copies and spill)
//  GEO_DENSE 256 consecutive pixels of the batch, taps that leave the board zeroed in the fragments
//  TM        DENSE only: output rows per tile (256; 128 / 64 for small batches, conv3x3_v7 only)
enum { GEO_PAD = 0, GEO_SLIM = 1, GEO_DENSE = 2 };
template <int HB, int GEO, int TM = 256>
struct Geom7 {
    static constexpr bool DENSE = GEO == GEO_DENSE, SLIM = GEO == GEO_SLIM;
    static constexpr int WG = DENSE ? HB : SLIM ? HB + 1 : HB + 2;   // grid / halo row width
    static constexpr int HW = HB * HB;
    static constexpr int GRID = DENSE ? TM : HB * WG;                // output grid rows of a tile
    static constexpr int NFRAG = (GRID + 15) / 16;                   // 16-row fragments with live rows
    static constexpr int TROWS = DENSE ? TM + 2 * HB + 2 : SLIM ? NFRAG * 16 + 2 * WG + 2 : (HB + 2) * (HB + 2);
    // DMA pieces of 64 rows per 8-channel group: 5 (320 rows) for 256-row tiles
    static constexpr int HROWS = (DENSE && TM < 256) ? (TROWS + 63) / 64 * 64 : 320;
    static constexpr int NRB = HROWS / 64;
    static_assert(TROWS <= HROWS, "halo does not fit");
    static_assert(DENSE ? (TM == 256 || TM == 192 || TM == 128 || TM == 64) : (TM == 256 && GRID <= 256 && NFRAG > 8),
                  "tile geometry");
};

}  // namespace

// MODE 2: fp16 operands, MODE 1: bf16.  Requires C % 64 == 0 (an even number of 32-channel
// chunks), N % 128 == 0, a ReLU (every g8 conv has one), no fp32 output.
// TM < 256 (DENSE, small batches): each wave owns TM / 2 rows = NI fragments (6, 4 or 2) x 64
// channels in one or two A register sets of NA fragments; the halo is NRB pieces per group.
// RG: weight-tile ring slots (4: tiles land 4 taps ahead, two blocks per CU; 3: 3 taps ahead, and
// with TM <= 128 (LDS 48 KB, <= 168 VGPRs) THREE blocks per CU -- small batches, more resident waves
// to hide the per-tap barrier and fragment latencies)
template <int MODE, int HB, int GEO, int TM = 256, int RG = 4>
__global__ __launch_bounds__(256, RG == 3 ? 3 : 2) void conv3x3_v7(ConvBf16Args p) {
    typedef H16<MODE> H;
    typedef Geom7<HB, GEO, TM> GM;
    constexpr bool DENSE = GM::DENSE, SLIM = GM::SLIM;
    typedef typename std::conditional<MODE == 2, f16x8, bf16x8>::type frag;
    constexpr int BNT = 128, WG = GM::WG, HW = GM::HW, HROWS = GM::HROWS, NRB = GM::NRB;
    constexpr int NI = TM / 32, NA = NI <= 4 ? NI : NI / 2, HALVES = NI / NA;   // fragments per wave / per A set
#ifdef AZ_V7_NOSKIP
    constexpr bool SKIP = false;
#else
    constexpr bool SKIP = SLIM && HALVES == 2;            // waves wm = 1 skip the SLIM tile's dead 16th fragment
#endif
    static_assert(NA * HALVES == NI && NA <= 4, "fragment split");
    static_assert(RG == 4 || (RG == 3 && TM <= 128), "ring");
    constexpr int WR = TM / 2;                            // rows per wave
    constexpr int A_BUF = 4 * HROWS * 16;                 // one chunk: [4 groups][320 rows][16 B] = 20 KB
    constexpr int B_TAP = 4 * BNT * 16;                   // one tap: [4 groups][128 ch][16 B] = 8 KB
    constexpr int LDS = 2 * A_BUF + RG * B_TAP;           // 72 KB (RG 4, TM 256); 48 KB (RG 3, TM 128)
    __shared__ __attribute__((aligned(16))) uint8_t lds[LDS];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 1, wn = wave & 1;             // 128 pixels x 64 channels per wave
    const int nsplit = p.N / BNT;
    const int xcd = blockIdx.x % 8, slot = blockIdx.x / 8;
    const int nb = slot % nsplit, tile = (slot / nsplit) * 8 + xcd;   // a tile's channel halves share an XCD
    const int n0 = nb * BNT;
    const int nboards = p.m_limit ? *p.m_limit : p.M / HW;
    if (DENSE ? tile * TM >= nboards * HW : tile >= nboards) return;
    const int C = p.C, GI = C / 8, GO = p.N / 8;
    const int NCH = C / 32, NS = 9 * NCH;

    const uint32_t a_bytes = (uint32_t)p.a_tail, b_bytes = (uint32_t)((size_t)9 * C * p.N * 2);
    const __amdgpu_buffer_rsrc_t rsA =
        __builtin_amdgcn_make_buffer_rsrc((void*)p.Ahi, (short)0, (int)(a_bytes + AZ_ACT_TAIL * 2), 0x00020000);
    const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc((void*)p.Bblk, (short)0, (int)b_bytes, 0x00020000);
    const uint32_t PAD = a_bytes;                         // zeroed tail: padding rows

    // halo piece j of this wave: q = wave + 4j -> (8-channel group g, 64-row block rb); the lane's
    // source offset is recomputed at every issue (a handful of VALU; keeping five offsets live
    // across the main loop would spill)
    auto a_src = [&](int j, int ln) -> uint32_t {
        const int q = wave + 4 * j, rb = q % NRB, g = q / NRB;
        const int hr = rb * 64 + ln;
        int Y, X, b;
        bool in;
        if constexpr (DENSE) {                            // halo row -> pixel tile*TM - HB - 1 + hr
            const int gpx = tile * TM - (HB + 1) + hr;
            b = gpx >= 0 ? gpx / HW : -1;
            const int pix = gpx - b * HW;
            Y = pix / HB + 1; X = pix - (Y - 1) * HB + 1;
            in = hr < GM::TROWS && gpx >= 0;
        } else {
            Y = hr / WG; X = hr - Y * WG;
            b = tile;
            in = hr < GM::TROWS;
        }
        const bool ok = in && Y >= 1 && Y <= HB && X >= 1 && X <= HB && b < nboards;   // SLIM: X = 0 is the zero column
        return ok ? (uint32_t)((((size_t)b * GI + g) * HW + (Y - 1) * HB + (X - 1)) * 16) : PAD;
    };
    // weight pieces: q = wave + 4j (j = 0, 1) -> (group g = q / 2, 64-channel block rb = q % 2)
    int b_src[2], b_dst[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int q = wave + 4 * j, rb = q & 1, g = q >> 1;
        b_src[j] = (((g >> 1) * 18 + (g & 1)) * p.N + n0 + rb * 64) * 16;
        b_dst[j] = g * (BNT * 16) + rb * 1024;
    }
    const uint32_t lane16 = lane * 16;
    uint8_t* abuf = lds;
    uint8_t* bbuf = lds + 2 * A_BUF;
    // voffset = the lane's part (VGPR), soffset = the wave-uniform part (SGPR): keeps the per-tap
    // offsets out of vector registers
    auto issueA = [&](int j, int c, int buf) {            // piece j of chunk c's halo into A buffer `buf`
        const int q = wave + 4 * j, rb = q % NRB, g = q / NRB;
        int ln = lane;
        asm volatile("" : "+v"(ln));                      // recompute here, do not hoist
        const uint32_t vo = a_src(j, ln);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_void_t*)(abuf + buf * A_BUF + g * (HROWS * 16) + rb * 1024),
                                                 16, (int)vo, __builtin_amdgcn_readfirstlane(c * (4 * HW * 16)), 0, 0);
    };
    auto issueB = [&](int s, int slot) {                  // the wave's two pieces of tap s's weights
        const int c = s / 9, t = s - 9 * c;
        const int so = __builtin_amdgcn_readfirstlane((36 * c + 2 * t) * p.N * 16);
#pragma unroll
        for (int j = 0; j < 2; ++j)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, (lds_void_t*)(bbuf + slot * B_TAP + b_dst[j]), 16,
                                                     (int)lane16, so + b_src[j], 0, 0);
    };

    f32x4v acc[NI][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {                         // the bias seeds the accumulators
        const float4 bv = *reinterpret_cast<const float4*>(p.bias + n0 + wn * 64 + j * 16 + 4 * (lane >> 4));
#pragma unroll
        for (int i = 0; i < NI; ++i) acc[i][j] = f32x4v{bv.x, bv.y, bv.z, bv.w};
    }

    // fragment addresses: activations (MFMA column operand) at halo row wm*WR + 16i + l16 + tap
    // shift, group l >> 4; weights (row operand) at channel wn*64 + 16j + l16, group l >> 4
    const int l16 = lane & 15, lg = lane >> 4;
    const uint32_t a_lane = lds_addr(abuf) + lg * (HROWS * 16) + (wm * WR + l16) * 16;
    const uint32_t b_lane = lds_addr(bbuf) + lg * (BNT * 16) + (wn * 64 + l16) * 16;
    uint32_t mbits = 0;                                   // DENSE: board-edge bits of the lane's NI pixels
    if constexpr (DENSE) {
#pragma unroll
        for (int f = 0; f < NI; ++f) {
            const int gq = tile * TM + wm * WR + f * 16 + l16;
            const int pix = gq % HW, y = pix / HB, x = pix - y * HB;
            mbits |= ((x == 0 ? 1u : 0u) | (x == HB - 1 ? 2u : 0u) | (y == 0 ? 4u : 0u) | (y == HB - 1 ? 8u : 0u)) << (4 * f);
        }
    }

    // prologue: halo of chunk 0, weights of taps 0..RG-1
#pragma unroll
    for (int j = 0; j < NRB; ++j) issueA(j, 0, 0);
#pragma unroll
    for (int s = 0; s < RG; ++s) issueB(s, s);
    wait_vm(2 * (RG - 1));                                // A(0), B(0) landed; B(1..RG-1) may fly
    __builtin_amdgcn_s_barrier();

    auto maskA = [&](frag (&a)[4], int half, int dy, int dx) {
        if constexpr (DENSE) {
            const uint32_t test = (dy == 0 ? 4u : dy == 2 ? 8u : 0u) | (dx == 0 ? 1u : dx == 2 ? 2u : 0u);
            if (test) {
#pragma unroll
                for (int i = 0; i < NA; ++i)
                    if (mbits & (test << (4 * (half * NA + i)))) a[i] = frag{};
            }
        }
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    // The main loop, compiled once per row half of the tile (WMC = wm, a wave-uniform branch): on the
    // SLIM grid the second half's 16th fragment (grid rows 240..255) holds no live output, so with
    // SKIP waves wm = 1 neither read nor multiply it -- 1/16 of the tile's MFMAs and fragment reads
    // (as conv3x3_v9x3's SKIP variant).  -DAZ_V7_NOSKIP builds the round-5 kernel (A/B measurement),
    // where those MFMAs run on all-zero halo rows.
    auto main_loop = [&](auto wmc) {
        constexpr int WMC = decltype(wmc)::value;
        constexpr int NI1 = (SKIP && WMC == 1) ? NA - 1 : NA;   // fragments of the second A set this wave computes
        frag alo[4], ahi[4], bw[2][4];
        // fragments of tap t (compile time) of the chunk in A buffer `ab`, weights in slot `bs`
        // SLIM without SKIP: the 16th fragment (rows 240..255, no live outputs) of the second row half
        // reads 16 rows further on, where every halo row of every tap is zero (rows >= 256: halo row Y >= 16)
        const uint32_t z16 = (SLIM && wm == 1) ? 16 * 16 : 0;
        auto loadA = [&](frag (&a)[4], uint32_t ab, auto tc, auto hc) {
            constexpr int t = decltype(tc)::value, half = decltype(hc)::value;
            constexpr int sh = (t / 3) * WG + (t % 3);
            static_for<0, NA>([&](auto ic) {
                constexpr int i = decltype(ic)::value;
                if constexpr (half == 1 && i >= NI1) return;
                else if constexpr (SLIM && half == 1 && i == 3) ds_rd<((half * NA + i) * 16 + sh) * 16>(a[i], ab + z16);
                else ds_rd<((half * NA + i) * 16 + sh) * 16>(a[i], ab);
            });
        };
        auto loadB = [&](frag (&b)[4], uint32_t bs) {
            static_for<0, 4>([&](auto jc) {
                constexpr int j = decltype(jc)::value;
                ds_rd<j * 256>(b[j], bs);
            });
        };
        auto mma = [&](const frag (&a)[4], const frag (&b)[4], auto hc) {
            constexpr int half = decltype(hc)::value, NIH = half == 1 ? NI1 : NA;
#pragma unroll
            for (int i = 0; i < NIH; ++i) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    if constexpr (MODE == 2)
                        acc[half * NA + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(b[j], a[i], acc[half * NA + i][j], 0, 0, 0);
                    else
                        acc[half * NA + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[half * NA + i][j], 0, 0, 0);
                }
            }
        };
        // tap 0 of chunk 0
        loadB(bw[0], b_lane);
        loadA(alo, a_lane, I0{}, I0{});
        if constexpr (HALVES == 2) loadA(ahi, a_lane, I0{}, I1{});

        // Two chunks per iteration: 18 taps, the weight registers alternate by tap parity.  Every tap
        // issues the same DMA pieces (a halo piece at taps 0..4, two weight pieces), past the end as
        // harmless reloads into free buffers, so the vmcnt budget is a compile-time constant: the
        // weights of tap s+1 were issued in tap s-RG+1 (the prologue for s < RG-1), followed by the
        // pieces of the RG-2 taps after it.  Fragments are read one tap ahead, past the end from free buffers.
        for (int c2 = 0; c2 < NCH; c2 += 2) {
            static_for<0, 18>([&](auto tc18) {
                constexpr int T = decltype(tc18)::value;      // tap of the chunk pair
                constexpr int t = T % 9, cur = T & 1, nxt = cur ^ 1;
                constexpr int allow = RG == 4 ? (t >= 2 && t - 2 < NRB ? 1 : 0) + (t >= 1 && t - 1 < NRB ? 1 : 0) + 4
                                              : (t >= 1 && t - 1 < NRB ? 1 : 0) + 2;
                constexpr int NAF = NA + (HALVES - 1) * NI1;  // activation fragment reads per tap
                const int c = c2 + T / 9;
                const int s = 9 * c + t;
                if constexpr (DENSE) asm volatile("" : "+v"(mbits));   // keep the edge masks inside the loop (no SGPR hoisting)
                // the NAF youngest LDS reads are this tap's activation fragments: the weights of tap s
                // (read one tap ago) are in registers -- required before the barrier frees their slot
                lgkm<NAF>(bw[cur]);
                wait_vm(allow);                               // weights of tap s+1 (and at t == 8 the next halo) landed
                __builtin_amdgcn_s_barrier();
                __builtin_amdgcn_sched_barrier(0);
                // DMA for later taps: a halo piece of chunk c+1 at taps 0..NRB-1 (the last chunk reloads
                // itself into the free buffer), then the weights of tap s+RG (clamped to the last tap)
                if constexpr (t < NRB) issueA(t, c + 1 < NCH ? c + 1 : c, (c + 1) & 1);
                issueB(s + RG < NS ? s + RG : NS - 1, (s + RG) % RG);
                // weights of tap s+1 (certified by the barrier above)
                loadB(bw[nxt], b_lane + ((s + 1) % RG) * B_TAP);
                __builtin_amdgcn_sched_barrier(0);
                lgkm<(HALVES - 1) * NI1 + 4>(alo);            // activations of tap s, low half
                maskA(alo, 0, t / 3, t % 3);
                mma(alo, bw[cur], I0{});
                __builtin_amdgcn_sched_barrier(0);
                const uint32_t an = a_lane + ((t == 8 ? c + 1 : c) & 1) * A_BUF;
                constexpr int tn = (t + 1) % 9;
                loadA(alo, an, std::integral_constant<int, tn>{}, I0{});
                if constexpr (HALVES == 2) {
                    lgkm<4 + NA>(ahi);                        // activations of tap s, high half
                    maskA(ahi, 1, t / 3, t % 3);
                    __builtin_amdgcn_sched_barrier(0);
                    mma(ahi, bw[cur], I1{});
                    __builtin_amdgcn_sched_barrier(0);
                    loadA(ahi, an, std::integral_constant<int, tn>{}, I1{});
                }
                __builtin_amdgcn_sched_barrier(0);
            });
        }
        // drain: the last tap's fragment reads (past the end) may still be in flight.  The compiler does
        // not see them, so without the fragments as operands of the wait it reuses their registers in
        // the epilogue, and a late LDS return overwrites a live value (seen as wrong outputs under LDS
        // contention: three blocks per CU, tools/lds_hazards.py)
        lgkm<0>(alo);
        if constexpr (HALVES == 2) lgkm<0>(ahi);
        lgkm<0>(bw[0]);
        lgkm<0>(bw[1]);
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    };
    if constexpr (SKIP) {
        if (wm == 0) main_loop(I0{});
        else main_loop(I1{});
    } else {
        main_loop(I0{});
    }

    // epilogue, straight from the accumulators: lane holds channels 4*(l >> 4) + e of pixel l16
    // of every 16 x 16 tile; residual join, ReLU, 16-bit + int8 split, streaming stores
    const __amdgpu_buffer_rsrc_t rh = __builtin_amdgcn_make_buffer_rsrc((void*)p.Rhi, (short)0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc((void*)p.Rq, (short)0, 0x7fffffff, 0x00020000);
    const int chl = n0 + wn * 64 + 4 * lg;                // first channel of the lane in tile j = 0
    float vmax = 0.0f;                                    // fp16: the largest output (the range guard)
    auto locate = [&](int i, int& b, int& pix) -> bool {  // fragment row i of the lane: board, pixel, live
        const int q = wm * WR + i * 16 + l16;             // output grid row of the tile
        if constexpr (DENSE) {
            const int gq = tile * TM + q;
            b = gq / HW;
            pix = gq - b * HW;
            return b < nboards;
        } else {
            const int y = q / WG, x = q - y * WG;
            b = tile;
            pix = y * HB + x;
            return y < HB && x < HB;
        }
    };
    // The residual join's loads go out EB fragment rows at a time (one memory round trip per burst,
    // two per wave at NI = 8), not one round trip per row: each row's loads would otherwise wait
    // behind the previous row's stores (the asm stores are memory barriers to the compiler), and a
    // 2nd conv's epilogue was eight serial HBM round trips per wave (conv2 498 us vs conv1 423 us per
    // C3 launch under PMC, profiles/r06_c3_fp16_pmc_calib.json).  <= 48 VGPRs per burst; the
    // arithmetic and the stored values are unchanged.
    constexpr int EB = NI <= 4 ? NI : NI % 4 == 0 ? 4 : NI % 3 == 0 ? 3 : NI % 2 == 0 ? 2 : 1;
    static_assert(NI % EB == 0, "bursts");
#pragma unroll
    for (int i0 = 0; i0 < NI; i0 += EB) {
    u32x2_t hv[EB][4];
    uint32_t qv[EB][4];
    if (p.Rhi) {
#pragma unroll
        for (int ii = 0; ii < EB; ++ii) {
            int b, pix;
            if (!locate(i0 + ii, b, pix)) continue;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int ch = chl + j * 16;
                const size_t e = (((size_t)b * GO + (ch >> 3)) * HW + pix) * 8 + (ch & 7);
                hv[ii][j] = __builtin_amdgcn_raw_buffer_load_b64(rh, (int)(e * 2), 0, AZ_RES_AUX);
                qv[ii][j] = __builtin_amdgcn_raw_buffer_load_b32(rq, (int)e, 0, AZ_RES_AUX);
            }
        }
    }
#pragma unroll
    for (int ii = 0; ii < EB; ++ii) {
        const int i = i0 + ii;
        int b, pix;
        if (!locate(i, b, pix)) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int ch = chl + j * 16;
            const size_t e = (((size_t)b * GO + (ch >> 3)) * HW + pix) * 8 + (ch & 7);
            float o[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
            if (p.Rhi) {
                uint16_t hh[4];
                int8_t qq[4];
                __builtin_memcpy(hh, &hv[ii][j], 8);
                __builtin_memcpy(qq, &qv[ii][j], 4);
#pragma unroll
                for (int k = 0; k < 4; ++k) o[k] += H::join(hh[k], qq[k]);
            }
            uint16_t oh[4];
            int8_t oq[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                o[k] = __builtin_amdgcn_fmed3f(o[k], 0.0f, 3.0e38f);   // ReLU
                if constexpr (MODE == 2) vmax = __builtin_fmaxf(vmax, o[k]);
                if (p.Cq) H::split(o[k], oh[k], oq[k]);
                else oh[k] = H::from_f(o[k]);
            }
            u32x2_t hs;
            __builtin_memcpy(&hs, oh, 8);
            asm volatile("global_store_dwordx2 %0, %1, off" AZ_V7_ST ::"v"(p.Chi + e), "v"(hs) : "memory");
            if (p.Cq) {
                uint32_t qs;
                __builtin_memcpy(&qs, oq, 4);
                asm volatile("global_store_dword %0, %1, off" AZ_V7_ST ::"v"(p.Cq + e), "v"(qs) : "memory");
            }
        }
    }
    }
    if (MODE == 2 && !(vmax <= 65504.0f) && p.ovf) atomicOr(p.ovf, 1);   // fp16 overflow: the engine fails the forward
}

// conv3x3_v7x3: the fp32-faithful trunk conv (AZ_PREC_BF16X3) on the v7 tile.
//
// Every fp32 operand x is carried as two bf16 planes, hi = bf16(x) and lo = bf16(x - hi), each
// in the g8 layout (activations) or the chunk-blocked layout (weights), and a product is
// hi*hi + lo*hi + hi*lo: three v_mfma_f32_16x16x32_bf16 with fp32 accumulation (lo*lo, ~2^-18
// of the product, is dropped) -- the arithmetic of conv3x3_v4<0>, on v7's geometry:
//
//  * tile 256 output rows x 128 channels per 256-thread block, wave tile 128 x 64 (as v7);
//  * LDS 144 KB: the halo of a 32-channel chunk, hi and lo planes, double-buffered (2 x 40 KB),
//    and a 4-slot ring of per-tap weight tiles, hi and lo (4 x 16 KB) -- one block per CU.
//    A tap is 96 MFMAs per wave (3x v7's), so one wave per SIMD keeps the matrix pipe fed, and
//    every fragment of tap s+1 (24 ds_read_b128: weights hi/lo, both row halves hi/lo) is read
//    into a second register set during tap s's MFMAs, in three batches of 8 (each batch waits
//    for the previous one, which is long done by then: never more than 8 LDS reads in flight);
//  * MFMAs in six units of 16 (Bh*Ah, Bl*Ah, Bh*Al per row half): consecutive MFMAs never
//    share an accumulator, so no unit waits on the previous one's result;
//  * epilogue from registers: residual hi + lo joined in fp32, ReLU, re-split into hi / lo,
//    streaming stores.
// Input: p.Ahi / p.Alo (g8 hi / lo, both with zeroed tails at p.a_tail), p.Bblk / p.Bblk_lo,
// residual p.Rhi / p.Rlo (optional), output p.Chi / p.Clo.
template <int HB, int GEO, int PT>
__global__ __launch_bounds__(256, 1) void conv3x3_v7x3(ConvBf16Args p) {
    typedef Geom7<HB, GEO> GM;
    typedef H16<PT> H;
    constexpr bool DENSE = GM::DENSE, SLIM = GM::SLIM;
    typedef typename X3T<PT>::frag frag;
    constexpr int BNT = 128, WG = GM::WG, HW = GM::HW, HROWS = GM::HROWS;
    constexpr int A_PL = 4 * HROWS * 16;                  // one plane of a chunk's halo: 20 KB
    constexpr int A_BUF = 2 * A_PL;                       // hi + lo: 40 KB
    constexpr int B_PL = 4 * BNT * 16;                    // one plane of a tap's weights: 8 KB
    constexpr int B_TAP = 2 * B_PL;                       // hi + lo: 16 KB
    constexpr int LDS = 2 * A_BUF + 4 * B_TAP;            // 144 KB
    __shared__ __attribute__((aligned(16))) uint8_t lds[LDS];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    const int nsplit = p.N / BNT;
    const int xcd = blockIdx.x % 8, slot = blockIdx.x / 8;
    const int nb = slot % nsplit, tile = (slot / nsplit) * 8 + xcd;   // a tile's channel halves share an XCD
    const int n0 = nb * BNT;
    const int nboards = p.m_limit ? *p.m_limit : p.M / HW;
    if (DENSE ? tile * 256 >= nboards * HW : tile >= nboards) return;
    const int C = p.C, GI = C / 8, GO = p.N / 8;
    const int NCH = C / 32, NS = 9 * NCH;

    const uint32_t a_bytes = (uint32_t)p.a_tail, b_bytes = (uint32_t)((size_t)9 * C * p.N * 2);
    const __amdgpu_buffer_rsrc_t rsA =
        __builtin_amdgcn_make_buffer_rsrc((void*)p.Ahi, (short)0, (int)(a_bytes + AZ_ACT_TAIL * 2), 0x00020000);
    const __amdgpu_buffer_rsrc_t rsAl =
        __builtin_amdgcn_make_buffer_rsrc((void*)p.Alo, (short)0, (int)(a_bytes + AZ_ACT_TAIL * 2), 0x00020000);
    const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc((void*)p.Bblk, (short)0, (int)b_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsBl =
        __builtin_amdgcn_make_buffer_rsrc((void*)p.Bblk_lo, (short)0, (int)b_bytes, 0x00020000);
    const uint32_t PAD = a_bytes;                         // zeroed tails: padding rows

    auto a_src = [&](int j, int ln) -> uint32_t {         // as conv3x3_v7: halo piece j of this wave
        const int q = wave + 4 * j, rb = q % 5, g = q / 5;
        const int hr = rb * 64 + ln;
        int Y, X, b;
        bool in;
        if constexpr (DENSE) {
            const int gpx = tile * 256 - (HB + 1) + hr;
            b = gpx >= 0 ? gpx / HW : -1;
            const int pix = gpx - b * HW;
            Y = pix / HB + 1; X = pix - (Y - 1) * HB + 1;
            in = hr < GM::TROWS && gpx >= 0;
        } else {
            Y = hr / WG; X = hr - Y * WG;
            b = tile;
            in = hr < GM::TROWS;
        }
        const bool ok = in && Y >= 1 && Y <= HB && X >= 1 && X <= HB && b < nboards;
        return ok ? (uint32_t)((((size_t)b * GI + g) * HW + (Y - 1) * HB + (X - 1)) * 16) : PAD;
    };
    int b_src[2], b_dst[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int q = wave + 4 * j, rb = q & 1, g = q >> 1;
        b_src[j] = (((g >> 1) * 18 + (g & 1)) * p.N + n0 + rb * 64) * 16;
        b_dst[j] = g * (BNT * 16) + rb * 1024;
    }
    const uint32_t lane16 = lane * 16;
    uint8_t* abuf = lds;
    uint8_t* bbuf = lds + 2 * A_BUF;
    auto issueA = [&](int j, int c, int buf) {            // piece j of chunk c's halo, hi and lo planes
        const int q = wave + 4 * j, rb = q % 5, g = q / 5;
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const uint32_t vo = a_src(j, ln);
        const int so = __builtin_amdgcn_readfirstlane(c * (4 * HW * 16));
        uint8_t* dst = abuf + buf * A_BUF + g * (HROWS * 16) + rb * 1024;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_void_t*)dst, 16, (int)vo, so, 0, 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsAl, (lds_void_t*)(dst + A_PL), 16, (int)vo, so, 0, 0);
    };
    auto issueB = [&](int s, int slot) {                  // the wave's four pieces of tap s's weights
        const int c = s / 9, t = s - 9 * c;
        const int so = __builtin_amdgcn_readfirstlane((36 * c + 2 * t) * p.N * 16);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            uint8_t* dst = bbuf + slot * B_TAP + b_dst[j];
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, (lds_void_t*)dst, 16, (int)lane16, so + b_src[j], 0, 0);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsBl, (lds_void_t*)(dst + B_PL), 16, (int)lane16, so + b_src[j], 0, 0);
        }
    };

    f32x4v acc[8][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const float4 bv = *reinterpret_cast<const float4*>(p.bias + n0 + wn * 64 + j * 16 + 4 * (lane >> 4));
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i][j] = f32x4v{bv.x, bv.y, bv.z, bv.w};
    }

    const int l16 = lane & 15, lg = lane >> 4;
    const uint32_t a_lane = lds_addr(abuf) + lg * (HROWS * 16) + (wm * 128 + l16) * 16;
    const uint32_t b_lane = lds_addr(bbuf) + lg * (BNT * 16) + (wn * 64 + l16) * 16;
    uint32_t mbits = 0;
    if constexpr (DENSE) {
#pragma unroll
        for (int f = 0; f < 8; ++f) {
            const int gq = tile * 256 + wm * 128 + f * 16 + l16;
            const int pix = gq % HW, y = pix / HB, x = pix - y * HB;
            mbits |= ((x == 0 ? 1u : 0u) | (x == HB - 1 ? 2u : 0u) | (y == 0 ? 4u : 0u) | (y == HB - 1 ? 8u : 0u)) << (4 * f);
        }
    }

    // prologue: halo of chunk 0 (hi + lo), weights of taps 0..3
#pragma unroll
    for (int j = 0; j < 5; ++j) issueA(j, 0, 0);
#pragma unroll
    for (int s = 0; s < 4; ++s) issueB(s, s);
    wait_vm(12);                                          // A(0), B(0) landed; B(1..3) may fly
    __builtin_amdgcn_s_barrier();

    // fragment registers, double-buffered by tap parity: a[buf][row half][plane][i], bw[buf][plane][j]
    frag a[2][2][2][4], bw[2][2][4];
    auto maskA = [&](frag (&x)[4], int half, int dy, int dx) {
        if constexpr (DENSE) {
            const uint32_t test = (dy == 0 ? 4u : dy == 2 ? 8u : 0u) | (dx == 0 ? 1u : dx == 2 ? 2u : 0u);
            if (test) {
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if (mbits & (test << (4 * (half * 4 + i)))) x[i] = frag{};
            }
        }
    };
    const uint32_t z16 = (SLIM && wm == 1) ? 16 * 16 : 0;  // SLIM: 16th fragment reads all-zero halo rows
    auto loadA = [&](frag (&x)[4], uint32_t ab, auto tc, auto hc, auto pc) {
        constexpr int t = decltype(tc)::value, half = decltype(hc)::value, pl = decltype(pc)::value;
        constexpr int sh = (t / 3) * WG + (t % 3);
        static_for<0, 4>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            if constexpr (SLIM && half == 1 && i == 3) ds_rd<pl * A_PL + ((half * 4 + i) * 16 + sh) * 16>(x[i], ab + z16);
            else ds_rd<pl * A_PL + ((half * 4 + i) * 16 + sh) * 16>(x[i], ab);
        });
    };
    auto loadB = [&](frag (&x)[4], uint32_t bs, auto pc) {
        constexpr int pl = decltype(pc)::value;
        static_for<0, 4>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            ds_rd<pl * B_PL + j * 256>(x[j], bs);
        });
    };
    auto mma = [&](const frag (&x)[4], const frag (&b)[4], int half) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                acc[half * 4 + i][j] = X3T<PT>::mma(b[j], x[i], acc[half * 4 + i][j]);
        }
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    // fragments of tap 0 of chunk 0, in batches of 8 LDS reads
    loadB(bw[0][0], b_lane, I0{});
    loadB(bw[0][1], b_lane, I1{});
    lgkm<0>(bw[0][0]);
    loadA(a[0][0][0], a_lane, I0{}, I0{}, I0{});
    loadA(a[0][0][1], a_lane, I0{}, I0{}, I1{});
    lgkm<0>(a[0][0][0]);
    loadA(a[0][1][0], a_lane, I0{}, I1{}, I0{});
    loadA(a[0][1][1], a_lane, I0{}, I1{}, I1{});

    // Two chunks per iteration (18 taps, register sets alternate by tap parity).  DMA as conv3x3_v7
    // with twice the pieces: a halo piece pair at taps 0..4, four weight pieces per tap; the weights
    // of tap s+1 were issued in tap s-3, followed by the pieces of taps s-2 and s-1.
    for (int c2 = 0; c2 < NCH; c2 += 2) {
        static_for<0, 18>([&](auto tc18) {
            constexpr int T = decltype(tc18)::value;
            constexpr int t = T % 9, cur = T & 1, nxt = cur ^ 1;
            constexpr int allow = 2 * (t >= 2 && t - 2 < 5 ? 1 : 0) + 2 * (t >= 1 && t - 1 < 5 ? 1 : 0) + 8;
            constexpr int tn = (t + 1) % 9;
            using TN = std::integral_constant<int, tn>;
            const int c = c2 + T / 9;
            const int s = 9 * c + t;
            if constexpr (DENSE) asm volatile("" : "+v"(mbits));
            // every fragment of tap s is in registers (the last batch was read before the previous
            // tap's last MFMA units): required before the barrier frees tap s's weight slot
            lgkm<0>(a[cur][1][0]);
            lgkm<0>(a[cur][1][1]);
            wait_vm(allow);                               // weights of tap s+1 (and at t == 8 the next halo) landed
            __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (t < 5) issueA(t, c + 1 < NCH ? c + 1 : c, (c + 1) & 1);
            issueB(s + 4 < NS ? s + 4 : NS - 1, (s + 4) & 3);
            // batch 1: the weights of tap s+1 (certified by the barrier above)
            const uint32_t bn = b_lane + ((s + 1) & 3) * B_TAP;
            loadB(bw[nxt][0], bn, I0{});
            loadB(bw[nxt][1], bn, I1{});
            __builtin_amdgcn_sched_barrier(0);
            maskA(a[cur][0][0], 0, t / 3, t % 3);
            maskA(a[cur][0][1], 0, t / 3, t % 3);
            mma(a[cur][0][0], bw[cur][0], 0);             // hi x hi, row half 0
            __builtin_amdgcn_sched_barrier(0);
            lgkm<0>(bw[nxt][0]);
            lgkm<0>(bw[nxt][1]);
            // batch 2: row half 0 of tap s+1
            const uint32_t an = a_lane + ((t == 8 ? c + 1 : c) & 1) * A_BUF;
            loadA(a[nxt][0][0], an, TN{}, I0{}, I0{});
            loadA(a[nxt][0][1], an, TN{}, I0{}, I1{});
            __builtin_amdgcn_sched_barrier(0);
            mma(a[cur][0][0], bw[cur][1], 0);             // hi(act) x lo(weights)
            __builtin_amdgcn_sched_barrier(0);
            mma(a[cur][0][1], bw[cur][0], 0);             // lo(act) x hi(weights)
            __builtin_amdgcn_sched_barrier(0);
            lgkm<0>(a[nxt][0][0]);
            lgkm<0>(a[nxt][0][1]);
            // batch 3: row half 1 of tap s+1
            loadA(a[nxt][1][0], an, TN{}, I1{}, I0{});
            loadA(a[nxt][1][1], an, TN{}, I1{}, I1{});
            __builtin_amdgcn_sched_barrier(0);
            maskA(a[cur][1][0], 1, t / 3, t % 3);
            maskA(a[cur][1][1], 1, t / 3, t % 3);
            mma(a[cur][1][0], bw[cur][0], 1);
            __builtin_amdgcn_sched_barrier(0);
            mma(a[cur][1][0], bw[cur][1], 1);
            __builtin_amdgcn_sched_barrier(0);
            mma(a[cur][1][1], bw[cur][0], 1);
            __builtin_amdgcn_sched_barrier(0);
        });
    }
    // drain with every fragment register as an operand (see conv3x3_v7)
#pragma unroll
    for (int k = 0; k < 8; ++k) lgkm<0>(a[k >> 2][(k >> 1) & 1][k & 1]);
#pragma unroll
    for (int k = 0; k < 4; ++k) lgkm<0>(bw[k >> 1][k & 1]);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");

    // epilogue from the accumulators: residual hi + lo joined in fp32, ReLU, split, streaming stores
    const __amdgpu_buffer_rsrc_t rh = __builtin_amdgcn_make_buffer_rsrc((void*)p.Rhi, (short)0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rl = __builtin_amdgcn_make_buffer_rsrc((void*)p.Rlo, (short)0, 0x7fffffff, 0x00020000);
    const int chl = n0 + wn * 64 + 4 * lg;
    float4 osc[4];                                        // PT 2: the weights' per-channel scale, undone
    if constexpr (PT == 2) {
#pragma unroll
        for (int j = 0; j < 4; ++j) osc[j] = *reinterpret_cast<const float4*>(p.oscale + chl + j * 16);
    }
    float vmax = 0.0f;                                    // PT 2: fp16 range guard
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int q = wm * 128 + i * 16 + l16;
        int b, pix;
        bool live;
        if constexpr (DENSE) {
            const int gq = tile * 256 + q;
            b = gq / HW;
            pix = gq - b * HW;
            live = b < nboards;
        } else {
            const int y = q / WG, x = q - y * WG;
            b = tile;
            pix = y * HB + x;
            live = y < HB && x < HB;
        }
        if (!live) continue;
        u32x2_t hv[4], lv[4];
        if (p.Rhi) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int ch = chl + j * 16;
                const size_t e = (((size_t)b * GO + (ch >> 3)) * HW + pix) * 8 + (ch & 7);
                hv[j] = __builtin_amdgcn_raw_buffer_load_b64(rh, (int)(e * 2), 0, AZ_RES_AUX);
                lv[j] = __builtin_amdgcn_raw_buffer_load_b64(rl, (int)(e * 2), 0, AZ_RES_AUX);
            }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int ch = chl + j * 16;
            const size_t e = (((size_t)b * GO + (ch >> 3)) * HW + pix) * 8 + (ch & 7);
            float o[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
            if constexpr (PT == 2) {
                o[0] *= osc[j].x; o[1] *= osc[j].y; o[2] *= osc[j].z; o[3] *= osc[j].w;
            }
            if (p.Rhi) {
                uint16_t hh[4], ll[4];
                __builtin_memcpy(hh, &hv[j], 8);
                __builtin_memcpy(ll, &lv[j], 8);
#pragma unroll
                for (int k = 0; k < 4; ++k) o[k] += H::to_f(hh[k]) + H::to_f(ll[k]);
            }
            uint16_t oh[4], ol[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                o[k] = __builtin_amdgcn_fmed3f(o[k], 0.0f, 3.0e38f);   // ReLU
                if constexpr (PT == 2) vmax = fmaxf(vmax, o[k]);
                oh[k] = H::from_f(o[k]);
                ol[k] = H::from_f(o[k] - H::to_f(oh[k]));
            }
            u32x2_t hs, ls;
            __builtin_memcpy(&hs, oh, 8);
            __builtin_memcpy(&ls, ol, 8);
            asm volatile("global_store_dwordx2 %0, %1, off nt" ::"v"(p.Chi + e), "v"(hs) : "memory");
            asm volatile("global_store_dwordx2 %0, %1, off nt" ::"v"(p.Clo + e), "v"(ls) : "memory");
        }
    }
    if (PT == 2 && !(vmax <= 65504.0f) && p.ovf) atomicOr(p.ovf, 1);    // fp16 pieces: the engine fails the forward
}

// conv3x3_v9x3: the fp32-faithful trunk conv on a full-width tile (the default for AZ_PREC_BF16X3
// at N % 256 == 0; conv3x3_v7x3 above is the A/B reference).
//
// Same operands and arithmetic as conv3x3_v7x3 -- every accumulator receives, per tap, Bh*Ah,
// then Bl*Ah, then Bh*Al, so the two kernels are bitwise equal -- on a different shape of work:
//
//  * ONE 512-thread block per CU (8 waves, two per SIMD: waves w and w + 4 share one) owns a
//    256-row tile x ALL 256 output channels (wave tile 128 rows x 64 channels, as v7x3).  The halo
//    is fetched once per tile, not once per channel half (v7x3 reads it twice: 1.36x algorithmic
//    HBM), and a SIMD's two waves hide each other's LDS-DMA issue (~60 cycles a piece), fragment
//    reads and barrier skew -- with v7x3's one wave per SIMD the matrix pipe idles through them;
//  * LDS 144 KB: the 32-channel halo chunk, hi + lo, double-buffered (2 x 40 KB) and a 2-slot
//    ring of per-tap weight tiles, hi + lo for 256 channels (2 x 32 KB).  Tap s's barrier certifies
//    tap s+1's weights (issued one tap earlier) and frees tap s's slot for tap s+2;
//  * a tap is four MFMA units per wave -- U0 Ah(rows 0-63 of the wave) x {Bh, Bl}, U1 Al x Bh,
//    U2 Ah(rows 64-127) x {Bh, Bl}, U3 Al x Bh -- over two 4-fragment activation register sets:
//    the next unit's fragments are read during the current one, and the next tap's weights are
//    read fragment by fragment as U2 / U3 release them (64 fragment VGPRs + 128 accumulators:
//    two waves per SIMD fit the register file);
//  * epilogue from registers as v7x3.
template <int HB, int GEO, int VAR, int PT>
__global__ __launch_bounds__(512, 1) void conv3x3_v9x3(ConvBf16Args p) {
    constexpr bool MID = VAR & 1;                         // the tap barrier after unit U0 (else at the tap start)
    constexpr bool SKIP = (VAR & 2) && GEO == GEO_SLIM;   // waves 4-7 skip the SLIM tile's dead 16th fragment
    typedef Geom7<HB, GEO> GM;
    typedef H16<PT> H;
    constexpr bool DENSE = GM::DENSE, SLIM = GM::SLIM;
    typedef typename X3T<PT>::frag frag;
    constexpr int BNT = 256, WG = GM::WG, HW = GM::HW, HROWS = GM::HROWS;
    constexpr int A_PL = 4 * HROWS * 16;                  // one plane of a chunk's halo: 20 KB
    constexpr int A_BUF = 2 * A_PL;                       // hi + lo: 40 KB
    constexpr int B_PL = 4 * BNT * 16;                    // one plane of a tap's weights: 16 KB
    constexpr int B_TAP = 2 * B_PL;                       // hi + lo: 32 KB
    constexpr int LDS = 2 * A_BUF + 2 * B_TAP;            // 144 KB
    __shared__ __attribute__((aligned(16))) uint8_t lds[LDS];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 2, wn = wave & 3;             // 128 pixels x 64 channels per wave
    const int nsplit = p.N / BNT;
    const int nb = blockIdx.x % nsplit, tile = blockIdx.x / nsplit;
    const int n0 = nb * BNT;
    const int nboards = p.m_limit ? *p.m_limit : p.M / HW;
    if (DENSE ? tile * 256 >= nboards * HW : tile >= nboards) return;
    // First-round stagger: the blocks of a launch run in lockstep rounds (one per CU, identical
    // work), so every CU reaches its epilogue at once and the epilogues' stores (and the second
    // conv's residual reads) saturate HBM together (tools/v9_stamps.py: 22 us of a 148 us block).
    // Offsetting the first round's starts over p.stagger ns keeps the CUs out of phase for the
    // whole launch, and each epilogue overlaps other CUs' main loops.
    if (p.stagger > 0 && blockIdx.x < 256) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        const uint64_t wait = (uint64_t)(((blockIdx.x * 37u) & 63u) * (uint32_t)p.stagger) / 640u;   // 10 ns ticks
        while (__builtin_amdgcn_s_memrealtime() - t0 < wait) __builtin_amdgcn_s_sleep(4);
    }
    V9_STAMP(0);
    const int C = p.C, GI = C / 8, GO = p.N / 8;
    const int NCH = C / 32, NS = 9 * NCH;

    const uint32_t a_bytes = (uint32_t)p.a_tail, b_bytes = (uint32_t)((size_t)9 * C * p.N * 2);
    const __amdgpu_buffer_rsrc_t rsA =
        __builtin_amdgcn_make_buffer_rsrc((void*)p.Ahi, (short)0, (int)(a_bytes + AZ_ACT_TAIL * 2), 0x00020000);
    const __amdgpu_buffer_rsrc_t rsAl =
        __builtin_amdgcn_make_buffer_rsrc((void*)p.Alo, (short)0, (int)(a_bytes + AZ_ACT_TAIL * 2), 0x00020000);
    const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc((void*)p.Bblk, (short)0, (int)b_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsBl =
        __builtin_amdgcn_make_buffer_rsrc((void*)p.Bblk_lo, (short)0, (int)b_bytes, 0x00020000);
    const uint32_t PAD = a_bytes;                         // zeroed tails: padding rows

    // halo piece pair q (hi + lo) = (8-channel group g = q / 5, 64-row block rb = q % 5): 20 pairs
    // per chunk, pair q = wave + 8j issued at tap j of the previous chunk (j = 0..2, q < 20)
    auto a_src = [&](int q, int ln) -> uint32_t {
        const int rb = q % 5, g = q / 5;
        const int hr = rb * 64 + ln;
        int Y, X, b;
        bool in;
        if constexpr (DENSE) {
            const int gpx = tile * 256 - (HB + 1) + hr;
            b = gpx >= 0 ? gpx / HW : -1;
            const int pix = gpx - b * HW;
            Y = pix / HB + 1; X = pix - (Y - 1) * HB + 1;
            in = hr < GM::TROWS && gpx >= 0;
        } else {
            Y = hr / WG; X = hr - Y * WG;
            b = tile;
            in = hr < GM::TROWS;
        }
        const bool ok = in && Y >= 1 && Y <= HB && X >= 1 && X <= HB && b < nboards;
        return ok ? (uint32_t)((((size_t)b * GI + g) * HW + (Y - 1) * HB + (X - 1)) * 16) : PAD;
    };
    // weight pieces of a tap, per plane 16 (group g = q >> 2, 64-channel block rb = q & 3): q = wave + 8j
    int b_src[2], b_dst[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int q = wave + 8 * j, rb = q & 3, g = q >> 2;
        b_src[j] = (((g >> 1) * 18 + (g & 1)) * p.N + n0 + rb * 64) * 16;
        b_dst[j] = g * (BNT * 16) + rb * 1024;
    }
    const uint32_t lane16 = lane * 16;
    uint8_t* abuf = lds;
    uint8_t* bbuf = lds + 2 * A_BUF;
    auto issueA = [&](int j, int c, int buf) {            // pair j of this wave for chunk c's halo
        const int q = wave + 8 * j;
        if (q >= 20) return;                              // wave-uniform
        const int rb = q % 5, g = q / 5;
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const uint32_t vo = a_src(q, ln);
        const int so = __builtin_amdgcn_readfirstlane(c * (4 * HW * 16));
        uint8_t* dst = abuf + buf * A_BUF + g * (HROWS * 16) + rb * 1024;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_void_t*)dst, 16, (int)vo, so, 0, 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsAl, (lds_void_t*)(dst + A_PL), 16, (int)vo, so, 0, 0);
    };
    auto issueB = [&](int s, int slot) {                  // the wave's four pieces of tap s's weights
        const int c = s / 9, t = s - 9 * c;
        const int so = __builtin_amdgcn_readfirstlane((36 * c + 2 * t) * p.N * 16);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            uint8_t* dst = bbuf + slot * B_TAP + b_dst[j];
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, (lds_void_t*)dst, 16, (int)lane16, so + b_src[j], 0, 0);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsBl, (lds_void_t*)(dst + B_PL), 16, (int)lane16, so + b_src[j], 0, 0);
        }
    };

    f32x4v acc[8][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const float4 bv = *reinterpret_cast<const float4*>(p.bias + n0 + wn * 64 + j * 16 + 4 * (lane >> 4));
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i][j] = f32x4v{bv.x, bv.y, bv.z, bv.w};
    }

    const int l16 = lane & 15, lg = lane >> 4;
    const uint32_t a_lane = lds_addr(abuf) + lg * (HROWS * 16) + (wm * 128 + l16) * 16;
    const uint32_t b_lane = lds_addr(bbuf) + lg * (BNT * 16) + (wn * 64 + l16) * 16;
    uint32_t mbits = 0;
    if constexpr (DENSE) {
#pragma unroll
        for (int f = 0; f < 8; ++f) {
            const int gq = tile * 256 + wm * 128 + f * 16 + l16;
            const int pix = gq % HW, y = pix / HB, x = pix - y * HB;
            mbits |= ((x == 0 ? 1u : 0u) | (x == HB - 1 ? 2u : 0u) | (y == 0 ? 4u : 0u) | (y == HB - 1 ? 8u : 0u)) << (4 * f);
        }
    }

    // prologue: halo of chunk 0 (hi + lo), weights of taps 0 and 1
#pragma unroll
    for (int j = 0; j < 3; ++j) issueA(j, 0, 0);
    issueB(0, 0);
    issueB(1, 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    V9_STAMP(1);

    frag aX[4], aY[4], bh[4], bl[4];
    auto maskA = [&](frag (&x)[4], int half, int dy, int dx) {
        if constexpr (DENSE) {
            const uint32_t test = (dy == 0 ? 4u : dy == 2 ? 8u : 0u) | (dx == 0 ? 1u : dx == 2 ? 2u : 0u);
            if (test) {
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if (mbits & (test << (4 * (half * 4 + i)))) x[i] = frag{};
            }
        }
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    // The main loop, compiled once per row half of the tile (WMC = wm): with SKIP the second half
    // (waves 4-7) neither reads nor multiplies its 16th fragment, whose rows hold no live outputs
    // on the SLIM grid -- 1/16 of a SIMD's MFMAs saved without a branch inside the loop.
    auto main_loop = [&](auto wmc) {
        constexpr int WMC = decltype(wmc)::value;
        constexpr int NI1 = (SKIP && WMC == 1) ? 3 : 4;  // fragments of row half 1 this wave computes
        const uint32_t z16 = (SLIM && wm == 1) ? 16 * 16 : 0;    // SLIM: 16th fragment reads all-zero halo rows
        auto loadA = [&](frag (&x)[4], uint32_t ab, auto tc, auto hc, auto pc) {
            constexpr int t = decltype(tc)::value, half = decltype(hc)::value, pl = decltype(pc)::value;
            constexpr int sh = (t / 3) * WG + (t % 3);
            static_for<0, 4>([&](auto ic) {
                constexpr int i = decltype(ic)::value;
                if constexpr (half == 1 && i >= NI1) return;
                else if constexpr (SLIM && half == 1 && i == 3) ds_rd<pl * A_PL + ((half * 4 + i) * 16 + sh) * 16>(x[i], ab + z16);
                else ds_rd<pl * A_PL + ((half * 4 + i) * 16 + sh) * 16>(x[i], ab);
            });
        };
        auto loadB = [&](frag (&x)[4], uint32_t bs, auto pc) {
            constexpr int pl = decltype(pc)::value;
            static_for<0, 4>([&](auto jc) {
                constexpr int j = decltype(jc)::value;
                ds_rd<pl * B_PL + j * 256>(x[j], bs);
            });
        };
        auto mma = [&](const frag (&x)[4], const frag (&b)[4], auto hc) {
            constexpr int half = decltype(hc)::value, NI = half == 1 ? NI1 : 4;
#pragma unroll
            for (int i = 0; i < NI; ++i) {
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[half * 4 + i][j] = X3T<PT>::mma(b[j], x[i], acc[half * 4 + i][j]);
            }
        };
        // row half 1 with the weights b, j-major: after fragment j's MFMAs, b[j] is reloaded with
        // plane pl of the next tap's weights (at bn)
        auto mma_reload = [&](const frag (&x)[4], frag (&b)[4], uint32_t bn, auto pc) {
            constexpr int pl = decltype(pc)::value;
            static_for<0, 4>([&](auto jc) {
                constexpr int j = decltype(jc)::value;
#pragma unroll
                for (int i = 0; i < NI1; ++i)
                    acc[4 + i][j] = X3T<PT>::mma(b[j], x[i], acc[4 + i][j]);
                __builtin_amdgcn_sched_barrier(0);
                ds_rd<pl * B_PL + j * 256>(b[j], bn);
                __builtin_amdgcn_sched_barrier(0);
            });
        };
        // the tap's DMA: a halo piece pair of chunk c+1 at t < 3 (the last chunk reloads itself into
        // the free buffer) and the weights of tap s+2 (clamped) into tap s's slot
        auto dma = [&](int t, int c, int s) {
            if (t < 3) issueA(t, c + 1 < NCH ? c + 1 : c, (c + 1) & 1);
            issueB(s + 2 < NS ? s + 2 : NS - 1, s & 1);
        };
        loadB(bh, b_lane, I0{});
        loadB(bl, b_lane, I1{});
        loadA(aX, a_lane, I0{}, I0{}, I0{});

        for (int c2 = 0; c2 < NCH; c2 += 2) {
            static_for<0, 18>([&](auto tc18) {
                constexpr int T = decltype(tc18)::value;
                constexpr int t = T % 9, tn = (t + 1) % 9;
                using TC = std::integral_constant<int, t>;
                using TN = std::integral_constant<int, tn>;
                const int c = c2 + T / 9;
                const int s = 9 * c + t;
                if constexpr (DENSE) asm volatile("" : "+v"(mbits));
                // tap s's weights and U0's fragments are in registers
                lgkm<0>(aX);
                lgkm<0>(bh);
                lgkm<0>(bl);
                if constexpr (!MID) {
                    // barrier at the tap start: tap s's weight reads are done (its slot may take tap
                    // s+2), tap s+1's weights (and at t == 8 the next halo) landed in every wave
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    __builtin_amdgcn_s_barrier();
                    __builtin_amdgcn_sched_barrier(0);
                    dma(t, c, s);
                }
                const uint32_t ac = a_lane + (c & 1) * A_BUF;
                loadA(aY, ac, TC{}, I0{}, I1{});          // U1: lo, row half 0
                __builtin_amdgcn_sched_barrier(0);
                maskA(aX, 0, t / 3, t % 3);
                mma(aX, bh, I0{});                        // U0: hi x hi, hi(act) x lo(weights)
                __builtin_amdgcn_sched_barrier(0);
                mma(aX, bl, I0{});
                __builtin_amdgcn_sched_barrier(0);
                lgkm<0>(aY);
                if constexpr (MID) {
                    // barrier after U0: every wave's reads of tap s's weights (issued at the end of
                    // tap s-1) have completed behind U0's MFMAs, so tap s's slot may take tap s+2;
                    // tap s+1's weights (and at t == 8 the next halo) landed in every wave
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    __builtin_amdgcn_s_barrier();
                    __builtin_amdgcn_sched_barrier(0);
                    dma(t, c, s);
                }
                loadA(aX, ac, TC{}, I1{}, I0{});          // U2: hi, row half 1
                __builtin_amdgcn_sched_barrier(0);
                maskA(aY, 0, t / 3, t % 3);
                mma(aY, bh, I0{});                        // U1: lo(act) x hi(weights)
                __builtin_amdgcn_sched_barrier(0);
                lgkm<0>(aX);
                loadA(aY, ac, TC{}, I1{}, I1{});          // U3: lo, row half 1
                __builtin_amdgcn_sched_barrier(0);
                maskA(aX, 1, t / 3, t % 3);
                mma(aX, bh, I1{});                        // U2
                __builtin_amdgcn_sched_barrier(0);
                const uint32_t bn = b_lane + ((s + 1) & 1) * B_TAP;
                mma_reload(aX, bl, bn, I1{});             // U2, releasing bl to tap s+1
                if constexpr (NI1 == 4) lgkm<4>(aY);      // U3's fragments (the 4 weight reads may fly)
                else asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(aY[0]), "+v"(aY[1]), "+v"(aY[2]) :: "memory");
                const uint32_t an = a_lane + ((t == 8 ? c + 1 : c) & 1) * A_BUF;
                loadA(aX, an, TN{}, I0{}, I0{});          // next tap's U0
                __builtin_amdgcn_sched_barrier(0);
                maskA(aY, 1, t / 3, t % 3);
                mma_reload(aY, bh, bn, I0{});             // U3, releasing bh to tap s+1
            });
        }
        // drain with every fragment register as an operand (see conv3x3_v7): the next tap's reads
        // past the end are in flight, and the two row-half branches' registers merge after this
        lgkm<0>(aX);
        lgkm<0>(aY);
        lgkm<0>(bh);
        lgkm<0>(bl);
    };
    if (SKIP && wm == 1) main_loop(I1{});
    else main_loop(I0{});
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    V9_STAMP(2);

    // epilogue from the accumulators: residual hi + lo joined in fp32, ReLU, split, streaming stores.
    // The residual of row fragments 0-3 is loaded in one burst, then 4-7 once 0-3 are stored (their
    // accumulators and residual registers free): two memory round trips per wave, not eight.
    const __amdgpu_buffer_rsrc_t rh = __builtin_amdgcn_make_buffer_rsrc((void*)p.Rhi, (short)0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rl = __builtin_amdgcn_make_buffer_rsrc((void*)p.Rlo, (short)0, 0x7fffffff, 0x00020000);
    const int chl = n0 + wn * 64 + 4 * lg;
    float4 osc[4];                                        // PT 2: the weights' per-channel scale, undone
    if constexpr (PT == 2) {
#pragma unroll
        for (int j = 0; j < 4; ++j) osc[j] = *reinterpret_cast<const float4*>(p.oscale + chl + j * 16);
    }
    float vmax = 0.0f;                                    // PT 2: fp16 range guard
    auto row_of = [&](int i, int& b, int& pix) -> bool {  // output row of fragment i of this lane
        const int q = wm * 128 + i * 16 + l16;
        if constexpr (DENSE) {
            const int gq = tile * 256 + q;
            b = gq / HW;
            pix = gq - b * HW;
            return b < nboards;
        } else {
            const int y = q / WG, x = q - y * WG;
            b = tile;
            pix = y * HB + x;
            return y < HB && x < HB;
        }
    };
    u32x2_t hv[4][4], lv[4][4];
    auto load_res = [&](auto i0c) {
        constexpr int i0 = decltype(i0c)::value;
#pragma unroll
        for (int ii = 0; ii < 4; ++ii) {
            int b, pix;
            if (!row_of(i0 + ii, b, pix)) continue;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int ch = chl + j * 16;
                const size_t e = (((size_t)b * GO + (ch >> 3)) * HW + pix) * 8 + (ch & 7);
                hv[ii][j] = __builtin_amdgcn_raw_buffer_load_b64(rh, (int)(e * 2), 0, AZ_RES_AUX);
                lv[ii][j] = __builtin_amdgcn_raw_buffer_load_b64(rl, (int)(e * 2), 0, AZ_RES_AUX);
            }
        }
    };
    auto finish = [&](auto i0c) {
        constexpr int i0 = decltype(i0c)::value;
#pragma unroll
        for (int ii = 0; ii < 4; ++ii) {
            const int i = i0 + ii;
            int b, pix;
            if (!row_of(i, b, pix)) continue;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int ch = chl + j * 16;
                const size_t e = (((size_t)b * GO + (ch >> 3)) * HW + pix) * 8 + (ch & 7);
                float o[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
                if constexpr (PT == 2) {
                    o[0] *= osc[j].x; o[1] *= osc[j].y; o[2] *= osc[j].z; o[3] *= osc[j].w;
                }
                if (p.Rhi) {
                    uint16_t hh[4], ll[4];
                    __builtin_memcpy(hh, &hv[ii][j], 8);
                    __builtin_memcpy(ll, &lv[ii][j], 8);
#pragma unroll
                    for (int k = 0; k < 4; ++k) o[k] += H::to_f(hh[k]) + H::to_f(ll[k]);
                }
                uint16_t oh[4], ol[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    o[k] = __builtin_amdgcn_fmed3f(o[k], 0.0f, 3.0e38f);   // ReLU
                    if constexpr (PT == 2) vmax = fmaxf(vmax, o[k]);
                    oh[k] = H::from_f(o[k]);
                    ol[k] = H::from_f(o[k] - H::to_f(oh[k]));
                }
                u32x2_t hs, ls;
                __builtin_memcpy(&hs, oh, 8);
                __builtin_memcpy(&ls, ol, 8);
                asm volatile("global_store_dwordx2 %0, %1, off nt" ::"v"(p.Chi + e), "v"(hs) : "memory");
                asm volatile("global_store_dwordx2 %0, %1, off nt" ::"v"(p.Clo + e), "v"(ls) : "memory");
            }
        }
    };
    using I4 = std::integral_constant<int, 4>;
    if (p.Rhi) load_res(I0{});
    finish(I0{});
    if (p.Rhi) load_res(I4{});
    finish(I4{});
#ifdef AZ_V9_STAMPS
    V9_STAMP(3);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    V9_STAMP(4);
#endif
    if (PT == 2 && !(vmax <= 65504.0f) && p.ovf) atomicOr(p.ovf, 1);    // fp16 pieces: the engine fails the forward
}

// Host side ----------------------------------------------------------------------------------
// diagnostic: select the stamped conv3x3_v9x3 launch / read its stamps (AZ_V9_STAMPS builds; else -1)
extern "C" int az_diag_v9_stamps(int sel, unsigned long long* st, unsigned* hw, int n) {
#ifdef AZ_V9_STAMPS
    if (sel >= -1) {
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_v9_sel), &sel, sizeof(int)) != hipSuccess) return -2;
        static unsigned long long zero[V9_MAXB][5];
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_v9_st), zero, sizeof(zero)) != hipSuccess) return -2;
    }
    if (st && n > 0) {
        n = n < V9_MAXB ? n : V9_MAXB;
        if (hipDeviceSynchronize() != hipSuccess) return -2;
        if (hipMemcpyFromSymbol(st, HIP_SYMBOL(g_v9_st), (size_t)n * 5 * 8) != hipSuccess) return -2;
        if (hw && hipMemcpyFromSymbol(hw, HIP_SYMBOL(g_v9_hw), (size_t)n * 2 * 4) != hipSuccess) return -2;
    }
    return 0;
#else
    (void)sel; (void)st; (void)hw; (void)n;
    return -1;
#endif
}

template <int HB, int GEO, int TM = 256, int RG = 4>
static void v7_launch_g(const ConvBf16Args& a, int mode, hipStream_t st) {
    const int boards = a.M / (HB * HB);
    const int tiles = GEO == GEO_DENSE ? (boards * HB * HB + TM - 1) / TM : boards;
    const int grid = (tiles + 7) / 8 * 8 * (a.N / 128);   // XCD-aware tile/half mapping: whole groups of 8
    // diagnostic conv flag 0x100000: 64 KB of unused dynamic LDS per block (fewer blocks per CU)
    const unsigned dyn = (a.flags & 0x100000) ? 65536u : 0u;
    if (mode == 2) hipLaunchKernelGGL((conv3x3_v7<2, HB, GEO, TM, RG>), dim3(grid), dim3(256), dyn, st, a);
    else hipLaunchKernelGGL((conv3x3_v7<1, HB, GEO, TM, RG>), dim3(grid), dim3(256), dyn, st, a);
}
// DENSE boards: the tile rows (256 / 128 / 64) for this launch -- small batches take smaller tiles
// so one round of blocks covers the CUs (az_conv_v7_tm; flag bits 0x70000 force 256 / 128 / 64 / 192)
int az_conv_v7_tm(const ConvBf16Args& a);
int az_conv_v7_ring(const ConvBf16Args& a);
template <int HB>
static void v7_launch_dense(const ConvBf16Args& a, int mode, hipStream_t st) {
    const bool r3 = az_conv_v7_ring(a) == 3;
    switch (az_conv_v7_tm(a)) {
        case 64: if (r3) v7_launch_g<HB, GEO_DENSE, 64, 3>(a, mode, st); else v7_launch_g<HB, GEO_DENSE, 64>(a, mode, st); break;
        case 128: if (r3) v7_launch_g<HB, GEO_DENSE, 128, 3>(a, mode, st); else v7_launch_g<HB, GEO_DENSE, 128>(a, mode, st); break;
        case 192: v7_launch_g<HB, GEO_DENSE, 192>(a, mode, st); break;
        default: v7_launch_g<HB, GEO_DENSE, 256>(a, mode, st); break;
    }
}

// The DENSE tile rows of a conv3x3_v7 launch: 256 unless the launch is under two rounds of blocks
// (two blocks per CU), where 192 / 128 / 64-row tiles spread the work over more CUs.  Conv flag bits
// 0x70000 force 256 (1) / 128 (2) / 64 (3) / 192 (4) for A/B measurement.
int az_conv_v7_tm(const ConvBf16Args& a) {
    const int force = (a.flags >> 16) & 7;
    if (force) return force == 1 ? 256 : force == 2 ? 128 : force == 3 ? 64 : 192;
    const long rows = (long)a.M;
    const int halves = a.N / 128;
    const long boards = rows / ((long)a.H * a.W);
    auto blocks = [&](int tm) { return ((rows + tm - 1) / tm + 7) / 8 * 8 * halves; };
    // below 1024 boards (g8_choice's small-batch branch) 19x19 -- and 13x13 once 128-row tiles fill
    // the CUs -- take 128-row tiles on the 3-slot ring (az_conv_v7_ring) at every size, including
    // those whose 256-row tiles would make 1024 blocks: 19x19 128 boards 0.0594 ms (192-row: 0.0620),
    // 256: 0.1106 (0.1160), 384: 0.1645 (256-row: 0.1887), 512: 0.2111 (0.2268; v6 0.2107), 768:
    // 0.3085 (0.3392) (profiles/r05_small_batch_ring3.txt)
    if (boards < 1024 && (a.H == 19 || (a.H == 13 && blocks(128) >= 512))) return 128;
    if (blocks(256) >= 1024) return 256;
    if (blocks(128) >= 512) return 128;
    return 64;
}

// Weight-ring slots of a DENSE conv3x3_v7 launch with tiles under 256 rows: 3 (three blocks per CU)
// for the automatic 128-row tiles or with conv flag 0x80000, else 4 (two blocks per CU).  128-row
// tiles, 4 -> 3 slots: 19x19 128 boards 0.0620 (192-row) -> 0.0594 ms, 13x13 256 0.0709 -> 0.0592,
// 13x13 512 0.1230 -> 0.1092, 9x9 512 0.0700 -> 0.0578, 8x8 512 0.0444 -> 0.0436; the 64-row tiles
// measured within +-2 % (8x8 128 0.0217 vs 0.0221, 9x9 256 0.0360 vs 0.0353) and keep 4
// (profiles/r05_small_batch_ring3.txt)
int az_conv_v7_ring(const ConvBf16Args& a) {
    const int tm = az_conv_v7_tm(a);
    if (tm > 128) return 4;
    if (a.flags & 0x80000) return 3;
    return (tm == 128 && !((a.flags >> 16) & 7)) ? 3 : 4;
}

// true when conv3x3_v7 takes this layer
bool az_conv_v7_supported(const ConvBf16Args& a) {
    if (a.H != a.W || a.C % 64 || a.N % 128 || !a.relu || a.Cf || a.Clo) return false;
    const int HB = a.H;
    if (HB != 8 && HB != 9 && HB != 13 && HB != 15 && HB != 19) return false;
    const size_t HW = (size_t)HB * HB;
    // the padding offset walks C/32 chunk steps into the zeroed tail; 32-bit buffer ranges
    return a.a_tail + AZ_ACT_TAIL * 2 < ((size_t)1 << 31) && (size_t)(a.C / 32) * 4 * HW * 16 + 16 <= AZ_ACT_TAIL * 2 &&
           (size_t)9 * a.C * a.N * 2 < ((size_t)1 << 31);
}

// conv3x3_v7x3 (AZ_PREC_BF16X3 on the g8 hi / lo planes): same shapes as conv3x3_v7, plus the lo
// planes of the input and the weights and both output planes; a residual needs both of its planes
bool az_conv_v7x3_supported(const ConvBf16Args& a) {
    if (a.H != a.W || a.C % 64 || a.N % 128 || !a.relu || a.Cf || a.Cq || a.Rq) return false;
    if (!a.Ahi || !a.Alo || !a.Bblk || !a.Bblk_lo || !a.Chi || !a.Clo || (!a.Rhi) != (!a.Rlo)) return false;
    if (a.pt == 2 && !a.oscale) return false;             // fp16 pieces: the weights' per-channel scale
    const int HB = a.H;
    if (HB != 8 && HB != 9 && HB != 13 && HB != 15 && HB != 19) return false;
    const size_t HW = (size_t)HB * HB;
    return a.a_tail >= (size_t)a.M * a.C * 2 && a.a_tail + AZ_ACT_TAIL * 2 < ((size_t)1 << 31) &&
           (size_t)(a.C / 32) * 4 * HW * 16 + 16 <= AZ_ACT_TAIL * 2 && (size_t)9 * a.C * a.N * 2 < ((size_t)1 << 31);
}

template <int HB, int GEO>
static void v7x3_launch_g(const ConvBf16Args& a, hipStream_t st) {
    const int boards = a.M / (HB * HB);
    const int tiles = GEO == GEO_DENSE ? (boards * HB * HB + 255) / 256 : boards;
    const int grid = (tiles + 7) / 8 * 8 * (a.N / 128);
    if (a.pt == 2) hipLaunchKernelGGL((conv3x3_v7x3<HB, GEO, 2>), dim3(grid), dim3(256), 0, st, a);
    else hipLaunchKernelGGL((conv3x3_v7x3<HB, GEO, 1>), dim3(grid), dim3(256), 0, st, a);
}

int az_conv_flags();
// first-round stagger (ns; az_diag_set_v9_stagger): 32 us measured best of 0 / 8 / 16 / 32 / 64 us,
// -0.8 % per C3 launch, -0.7 % C4 (profiles/r04_v9x3_stagger.txt); only on launches of >= 1024 blocks
// (several rounds), where a one-off delay of the last-started CU is amortised
static int g_v9_stagger = 32000;
extern "C" int az_diag_set_v9_stagger(int ns) { g_v9_stagger = ns; return 0; }
// conv3x3_v9x3 variants (A/B measurement, bf16 pieces): flag 0x20000000 puts the tap barrier at the
// tap start instead of after unit U0, 0x40000000 keeps the SLIM tile's dead 16th fragment in waves
// 4-7.  fp16 pieces (AZ_PREC_F16X3) run the default variant only.
template <int HB, int GEO>
static void v9x3_launch_g(const ConvBf16Args& a, hipStream_t st) {
    const int boards = a.M / (HB * HB);
    const int tiles = GEO == GEO_DENSE ? (boards * HB * HB + 255) / 256 : boards;
    const int f = az_conv_flags(), var = ((f & 0x20000000) ? 0 : 1) | ((f & 0x40000000) ? 0 : 2);
    const dim3 grid(tiles * (a.N / 256)), block(512);
    ConvBf16Args b = a;
    b.stagger = tiles * (a.N / 256) >= 1024 ? g_v9_stagger : 0;
    if (a.pt == 2) {
        hipLaunchKernelGGL((conv3x3_v9x3<HB, GEO, 3, 2>), grid, block, 0, st, b);
        return;
    }
    switch (var) {
        case 0: hipLaunchKernelGGL((conv3x3_v9x3<HB, GEO, 0, 1>), grid, block, 0, st, b); break;
        case 1: hipLaunchKernelGGL((conv3x3_v9x3<HB, GEO, 1, 1>), grid, block, 0, st, b); break;
        case 2: hipLaunchKernelGGL((conv3x3_v9x3<HB, GEO, 2, 1>), grid, block, 0, st, b); break;
        default: hipLaunchKernelGGL((conv3x3_v9x3<HB, GEO, 3, 1>), grid, block, 0, st, b); break;
    }
}

// conv3x3_v9x3 takes every bf16x3 trunk layer with N % 256 == 0 unless conv flag 0x10000000
// selects conv3x3_v7x3 (A/B measurement)
static bool x3_wide(const ConvBf16Args& a) { return a.N % 256 == 0 && !(az_conv_flags() & 0x10000000); }

// the kernel az_conv_v7x3_launch takes (bench.py's roofline label)
int az_conv_x3_name(const ConvBf16Args& a, char* out, int len) {
    if (!az_conv_v7x3_supported(a)) return -1;
    snprintf(out, len, "%s<%d, %s%s>", x3_wide(a) ? "conv3x3_v9x3" : "conv3x3_v7x3", a.H, a.H == 15 ? "SLIM" : "DENSE",
             a.pt == 2 ? ", f16" : "");
    return 0;
}

// 15x15 boards on the SLIM tile, every other board DENSE (as conv3x3_v7's defaults)
int az_conv_v7x3_launch(const ConvBf16Args& a, hipStream_t st) {
    if (!az_conv_v7x3_supported(a)) return -1;
    if (x3_wide(a)) {
        switch (a.H) {
            case 8: v9x3_launch_g<8, GEO_DENSE>(a, st); return 0;
            case 9: v9x3_launch_g<9, GEO_DENSE>(a, st); return 0;
            case 13: v9x3_launch_g<13, GEO_DENSE>(a, st); return 0;
            case 19: v9x3_launch_g<19, GEO_DENSE>(a, st); return 0;
            default: v9x3_launch_g<15, GEO_SLIM>(a, st); return 0;
        }
    }
    switch (a.H) {
        case 8: v7x3_launch_g<8, GEO_DENSE>(a, st); return 0;
        case 9: v7x3_launch_g<9, GEO_DENSE>(a, st); return 0;
        case 13: v7x3_launch_g<13, GEO_DENSE>(a, st); return 0;
        case 19: v7x3_launch_g<19, GEO_DENSE>(a, st); return 0;
        default: v7x3_launch_g<15, GEO_SLIM>(a, st); return 0;
    }
}

// geo15: the 15x15 tile geometry (GEO_PAD / GEO_SLIM / GEO_DENSE); other boards are DENSE
int az_conv_v7_launch(const ConvBf16Args& a, int mode, int geo15, hipStream_t st) {
    if (!az_conv_v7_supported(a)) return -1;
    switch (a.H) {
        case 8: v7_launch_dense<8>(a, mode, st); return 0;
        case 9: v7_launch_dense<9>(a, mode, st); return 0;
        case 13: v7_launch_dense<13>(a, mode, st); return 0;
        case 19: v7_launch_dense<19>(a, mode, st); return 0;
        default:
            if (geo15 == GEO_DENSE) v7_launch_dense<15>(a, mode, st);
            else if (geo15 == GEO_PAD) v7_launch_g<15, GEO_PAD>(a, mode, st);
            else v7_launch_g<15, GEO_SLIM>(a, mode, st);
            return 0;
    }
}
