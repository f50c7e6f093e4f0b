// buffer_load_dwordx4 ... lds: where does each lane's 16 B land in LDS?
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((address_space(3))) void lds_void_t;
__global__ void k(const unsigned* src, unsigned* out) {
    __shared__ __attribute__((aligned(16))) unsigned lds[1024];
    for (int i = threadIdx.x; i < 1024; i += 64) lds[i] = 0xdeadbeef;
    __syncthreads();
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, 16384, 0x00020000);
    const int lane = threadIdx.x;
    // lane l reads bytes [1024 + 32 l, +16) (a strided source) into LDS at byte 256
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)((unsigned char*)lds + 256), 16, 1024 + 32 * lane, 0, 0, 0);
    __builtin_amdgcn_s_waitcnt(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = threadIdx.x; i < 1024; i += 64) out[i] = lds[i];
}
int main() {
    unsigned h[4096], o[1024];
    for (int i = 0; i < 4096; ++i) h[i] = i;
    unsigned *d, *dout;
    hipMalloc(&d, sizeof h); hipMalloc(&dout, sizeof o);
    hipMemcpy(d, h, sizeof h, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, dout);
    hipMemcpy(o, dout, sizeof o, hipMemcpyDeviceToHost);
    // expected: lds word 64 + 4 l + w == (1024 + 32 l) / 4 + w
    int bad = 0;
    for (int l = 0; l < 64; ++l) for (int w = 0; w < 4; ++w) bad += o[64 + 4 * l + w] != (unsigned)((1024 + 32 * l) / 4 + w);
    printf("lane-linear 16 B per lane: %d mismatches; lds[64..72) = %x %x %x %x %x %x %x %x\n", bad, o[64], o[65], o[66], o[67], o[68], o[69], o[70], o[71]);
    return 0;
}
