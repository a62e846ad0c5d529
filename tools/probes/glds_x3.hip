// Probe: LDS layout of __builtin_amdgcn_global_load_lds with 12-byte (dwordx3) and 16-byte pieces on
// gfx950.  One wave; lane i reads 12 (16) bytes at src + 12 i (16 i); LDS dumped.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define PROBE(NAME, SZ)                                                                                         \
__global__ void NAME(const uint32_t* src, uint32_t* out)                                                          \
{                                                                                                                 \
    __shared__ uint32_t s[512];                                                                                   \
    for (int i = threadIdx.x; i < 512; i += 64) s[i] = 0xFFFFFFFFu;                                               \
    __syncthreads();                                                                                              \
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + (SZ / 4) * threadIdx.x), \
                                     (__attribute__((address_space(3))) void*)s, SZ, 0, 0);                       \
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                                                             \
    __syncthreads();                                                                                              \
    for (int i = threadIdx.x; i < 512; i += 64) out[i] = s[i];                                                    \
}
PROBE(k12, 12)
PROBE(k16, 16)
template <int SZ>
__global__ void k_unused(const uint32_t* src, uint32_t* out)
{
}
int main()
{
    uint32_t h[1024];
    for (int i = 0; i < 1024; ++i) h[i] = i;
    uint32_t *d, *o;
    hipMalloc(&d, sizeof(h));
    hipMalloc(&o, 512 * 4);
    hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
    uint32_t r[512];
    hipLaunchKernelGGL(k12, dim3(1), dim3(64), 0, 0, d, o);
    hipMemcpy(r, o, sizeof(r), hipMemcpyDeviceToHost);
    printf("x3:");
    for (int i = 0; i < 200; ++i) printf(" %d", (int)r[i]);
    printf("\n");
    hipLaunchKernelGGL(k16, dim3(1), dim3(64), 0, 0, d, o);
    hipMemcpy(r, o, sizeof(r), hipMemcpyDeviceToHost);
    printf("x4:");
    for (int i = 0; i < 260; ++i) printf(" %d", (int)r[i]);
    printf("\n");
    return 0;
}
