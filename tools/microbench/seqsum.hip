// Sequential fp32 sum of 240 values (the tree kernel's softmax normaliser, bit-exact order) on one
// wave: (A) the shipped seq_sum_lds loop, (C) a chain of v_mfma_f32_16x16x4_f32 with B = 1.0
// (4 ordered fma(1, x, s) per MFMA, operands read beforehand).  Prints cycles (s_memtime) and
// whether C equals A bitwise over many vectors, with and without denormal inputs.
// Measured (round 3): A 2172 cycles (9 per dependent v_add_f32), C 1940 (32 per dependent MFMA =
// 8 per add), bitwise equal on all 400 vectors incl. 79 with denormal inputs: not worth a change.   hipcc --offload-arch=gfx950 -O3 seqsum.hip -o seqsum && ./seqsum
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <cmath>
#include <vector>
#include <random>

typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int N = 240;

__device__ __forceinline__ float seq_sum_lds(const float* x, int n) {
    float s = 0.0f;
    const float4* q = reinterpret_cast<const float4*>(x);
    const int nq = (n + 15) / 16;
    float4 a = q[0], b = q[1], c = q[2], d = q[3];
    for (int j = 0; j < nq; ++j) {
        float4 na = a, nb = b, nc = c, nd = d;
        if (j + 1 < nq) { na = q[4 * j + 4]; nb = q[4 * j + 5]; nc = q[4 * j + 6]; nd = q[4 * j + 7]; }
        s += a.x; s += a.y; s += a.z; s += a.w;
        s += b.x; s += b.y; s += b.z; s += b.w;
        s += c.x; s += c.y; s += c.z; s += c.w;
        s += d.x; s += d.y; s += d.z; s += d.w;
        a = na; b = nb; c = nc; d = nd;
    }
    return s;
}

__device__ __forceinline__ long long mtime() {
    long long t;
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
    return t;
}

__global__ void k_sum(const float* in, float* out, long long* cyc, int nvec) {
    __shared__ __attribute__((aligned(16))) float x[256];
    const int lane = threadIdx.x;
    for (int v = 0; v < nvec; ++v) {
        for (int i = lane; i < 256; i += 64) x[i] = i < N ? in[(size_t)v * N + i] : 0.0f;
        __syncthreads();
        long long t0 = mtime();
        float sa = seq_sum_lds(x, N);
        asm volatile("" : "+v"(sa));
        long long t1 = mtime();
        long long t2 = 0, t3 = 0;
        const float sb = sa;
        // (C) MFMA chain: A[row][k] = x[4m + k] (lane 16 k + row), B = 1, C = running sum
        float am[N / 4];
#pragma unroll
        for (int m = 0; m < N / 4; ++m) am[m] = x[4 * m + (lane >> 4)];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        long long t4 = mtime();
#pragma unroll
        for (int m = 0; m < N / 4; ++m) asm volatile("" : "+v"(am[m]));
        f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int m = 0; m < N / 4; ++m) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(am[m], 1.0f, acc, 0, 0, 0);
        float sc = acc[0];
        asm volatile("" : "+v"(sc));
        long long t5 = mtime();
        if (lane == 0) {
            out[3 * v] = sa; out[3 * v + 1] = sb; out[3 * v + 2] = sc;
            cyc[3 * v] = t1 - t0; cyc[3 * v + 1] = t3 - t2; cyc[3 * v + 2] = t5 - t4;
        }
        __syncthreads();
    }
}

int main() {
    const int nvec = 400;
    std::vector<float> h((size_t)nvec * N);
    std::mt19937 g(5);
    for (int v = 0; v < nvec; ++v) {
        // logits of spread S: softmax numerators exp(l - max); the last 100 vectors have spreads up
        // to 200 (denormal numerators) 
        const float S = v < 300 ? 2.0f + 0.05f * v : 60.0f + 1.4f * (v - 300);
        std::uniform_real_distribution<float> U(-S, 0.0f);
        float mx = -1e30f;
        std::vector<float> l(N);
        for (int i = 0; i < N; ++i) { l[i] = U(g); mx = std::max(mx, l[i]); }
        for (int i = 0; i < N; ++i) h[(size_t)v * N + i] = (i < 225) ? expf(l[i] - mx) : 0.0f;
    }
    float *din, *dout; long long* dc;
    hipMalloc(&din, h.size() * 4); hipMalloc(&dout, nvec * 3 * 4); hipMalloc(&dc, nvec * 3 * 8);
    hipMemcpy(din, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_sum, dim3(1), dim3(64), 0, 0, din, dout, dc, nvec);
    std::vector<float> o(nvec * 3); std::vector<long long> c(nvec * 3);
    hipMemcpy(o.data(), dout, o.size() * 4, hipMemcpyDeviceToHost);
    hipMemcpy(c.data(), dc, c.size() * 8, hipMemcpyDeviceToHost);
    int eqb = 0, eqc = 0, eqc_norm = 0, n_norm = 0;
    long long ca = 0, cb = 0, cc = 0;
    for (int v = 0; v < nvec; ++v) {
        uint32_t a, b, cc_;
        memcpy(&a, &o[3 * v], 4); memcpy(&b, &o[3 * v + 1], 4); memcpy(&cc_, &o[3 * v + 2], 4);
        eqb += a == b; eqc += a == cc_;
        bool denorm = false;
        for (int i = 0; i < 225; ++i) { const float x = h[(size_t)v * N + i]; if (x != 0.0f && fabsf(x) < 1.17549435e-38f) denorm = true; }
        if (!denorm) { ++n_norm; eqc_norm += a == cc_; }
        if (v >= 10) { ca += c[3 * v]; cb += c[3 * v + 1]; cc += c[3 * v + 2]; }
    }
    printf("cycles per 240-value sum: A seq_sum_lds %.0f, C MFMA chain %.0f\n", ca / double(nvec - 10),
           cc / double(nvec - 10));
    printf("bitwise equal to A: C %d / %d (vectors without denormal inputs: %d / %d)\n", eqc, nvec, eqc_norm, n_norm);
    return 0;
}
