// Achievable-HBM-bandwidth probe for bench.py's roofline denominator: a 16-byte-per-lane
// streaming copy, the shape MI355X_MICROARCH.md quotes 6.29 TB/s for.  Not part of liborbx.so.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o tools/probes/libhbm_copy.so tools/probes/hbm_copy.hip
// hbm_copy(dst, src, n16, blocks, unroll, nt, stream): n16 uint4 elements; each thread copies `unroll`
// consecutive-by-stride elements per trip of a grid-stride loop; nt = 1 uses non-temporal loads and stores.
#include <hip/hip_runtime.h>
#include <cstdint>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void k_copy(u32x4* __restrict__ dst, const u32x4* __restrict__ src, size_t n)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + (U - 1) * stride < n; i += U * stride) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = NT ? __builtin_nontemporal_load(src + i + u * stride) : src[i + u * stride];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (NT) __builtin_nontemporal_store(v[u], dst + i + u * stride);
            else dst[i + u * stride] = v[u];
        }
    }
    for (; i < n; i += stride) dst[i] = src[i];
}

extern "C" int hbm_copy(void* dst, const void* src, size_t n16, int blocks, int unroll, int nt, void* stream)
{
    hipStream_t s = (hipStream_t)stream;
    u32x4* d = (u32x4*)dst;
    const u32x4* a = (const u32x4*)src;
    dim3 g(blocks), b(256);
    if (unroll == 1 && !nt) hipLaunchKernelGGL((k_copy<1, false>), g, b, 0, s, d, a, n16);
    else if (unroll == 1) hipLaunchKernelGGL((k_copy<1, true>), g, b, 0, s, d, a, n16);
    else if (unroll == 4 && !nt) hipLaunchKernelGGL((k_copy<4, false>), g, b, 0, s, d, a, n16);
    else if (unroll == 4) hipLaunchKernelGGL((k_copy<4, true>), g, b, 0, s, d, a, n16);
    else if (unroll == 8 && !nt) hipLaunchKernelGGL((k_copy<8, false>), g, b, 0, s, d, a, n16);
    else if (unroll == 8) hipLaunchKernelGGL((k_copy<8, true>), g, b, 0, s, d, a, n16);
    else return -1;
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
