// Checks the assumed operand / result lane maps of v_mfma_f32_16x16x32_f16 with exact integers:
// lane l holds A[l&15][8(l>>4)+j], B[8(l>>4)+j][l&15]; result reg e of lane l = C[(l>>4)*4+e][l&15].
#include <hip/hip_runtime.h>
#include <cstdio>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
__global__ void k(const float* A, const float* B, float* C) {
    const int l = threadIdx.x;
    f16x8 a, b;
    for (int j = 0; j < 8; ++j) {
        a[j] = (_Float16)A[(l & 15) * 32 + 8 * (l >> 4) + j];
        b[j] = (_Float16)B[(8 * (l >> 4) + j) * 16 + (l & 15)];
    }
    f32x4 c = {0, 0, 0, 0};
    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
    for (int e = 0; e < 4; ++e) C[((l >> 4) * 4 + e) * 16 + (l & 15)] = c[e];
}
int main() {
    float hA[16 * 32], hB[32 * 16], hC[256], ref[256];
    for (int i = 0; i < 512; ++i) { hA[i] = (float)((i * 7) % 5 - 2); hB[i] = (float)((i * 11) % 7 - 3); }
    for (int r = 0; r < 16; ++r) for (int c = 0; c < 16; ++c) { float s = 0; for (int k = 0; k < 32; ++k) s += hA[r * 32 + k] * hB[k * 16 + c]; ref[r * 16 + c] = s; }
    float *dA, *dB, *dC;
    hipMalloc(&dA, sizeof hA); hipMalloc(&dB, sizeof hB); hipMalloc(&dC, sizeof hC);
    hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice); hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dC);
    hipMemcpy(hC, dC, sizeof hC, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 256; ++i) bad += hC[i] != ref[i];
    printf("16x16x32 f16 layout: %d / 256 mismatches (C[0]=%g ref %g, C[17]=%g ref %g)\n", bad, hC[0], ref[0], hC[17], ref[17]);
    return bad != 0;
}
