// Bare MFMA loop: 32x32x16 f16 vs 16x16x32 f16 at full occupancy (2 waves/SIMD, all CUs),
// random operands, same FLOPs per iteration; reports TFLOP/s and the in-kernel clock.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int SHAPE>
__global__ __launch_bounds__(512, 1) void k(const f16x8* in, float* out, int iters, unsigned long long* clk) {
    const int lane = threadIdx.x & 63;
    f16x8 a[4], b[2];
    for (int i = 0; i < 4; ++i) a[i] = in[(blockIdx.x * 8 + i) * 64 + lane];
    for (int j = 0; j < 2; ++j) b[j] = in[(blockIdx.x * 8 + 4 + j) * 64 + lane];
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    float s = 0.0f;
    if constexpr (SHAPE == 32) {
        f32x16 acc[4][2] = {};
        for (int it = 0; it < iters; ++it)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[i], b[j], acc[i][j], 0, 0, 0);
        for (int i = 0; i < 4; ++i) for (int j = 0; j < 2; ++j) for (int e = 0; e < 16; ++e) s += acc[i][j][e];
    } else {
        // same FLOPs: 8 x (32x32x16) = 32 x (16x16x32)
        f32x4 acc[8][4] = {};
        for (int it = 0; it < iters; ++it)
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[i & 3], b[j & 1], acc[i][j], 0, 0, 0);
        for (int i = 0; i < 8; ++i) for (int j = 0; j < 4; ++j) for (int e = 0; e < 4; ++e) s += acc[i][j][e];
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * 512 + threadIdx.x] = s;
    if (threadIdx.x == 0) { clk[blockIdx.x * 2] = t1 - t0; clk[blockIdx.x * 2 + 1] = r1 - r0; }
}

int main() {
    const int blocks = 256 * 4, iters = 20000;
    f16x8* in; float* out; unsigned long long* clk;
    hipMalloc(&in, (size_t)blocks * 8 * 64 * 16);
    hipMalloc(&out, (size_t)blocks * 512 * 4);
    hipMalloc(&clk, (size_t)blocks * 16);
    std::vector<_Float16> h((size_t)blocks * 8 * 64 * 8);
    unsigned x = 1;
    for (auto& v : h) { x = x * 1664525u + 1013904223u; v = (_Float16)(((x >> 9) & 0xffff) / 65536.0f - 0.5f); }
    hipMemcpy(in, h.data(), h.size() * 2, hipMemcpyHostToDevice);
    for (int rep = 0; rep < 2; ++rep)
        for (int shape : {32, 16}) {
            hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
            hipEventRecord(e0);
            if (shape == 32) hipLaunchKernelGGL(k<32>, dim3(blocks), dim3(512), 0, 0, in, out, iters, clk);
            else hipLaunchKernelGGL(k<16>, dim3(blocks), dim3(512), 0, 0, in, out, iters, clk);
            hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1);
            std::vector<unsigned long long> c((size_t)blocks * 2);
            hipMemcpy(c.data(), clk, c.size() * 8, hipMemcpyDeviceToHost);
            double ghz = 0; for (int b = 0; b < blocks; ++b) ghz += (double)c[2 * b] / (double)c[2 * b + 1] * 0.1; ghz /= blocks;
            const double flops = (double)blocks * 8 * iters * 8 * 2.0 * 32 * 32 * 16;
            printf("shape %dx%d: %.3f ms  %.0f TFLOP/s  clock %.2f GHz\n", shape, shape, ms, flops / ms / 1e9, ghz);
        }
    return 0;
}
