// Achievable-HBM-bandwidth probe for bench.py's roofline denominator: a 16-byte-per-lane
// streaming copy, the shape MI355X_MICROARCH.md quotes 6.29 TB/s for.  Not part of liborbx.so.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o tools/probes/libhbm_copy.so tools/probes/hbm_copy.hip
// hbm_copy(dst, src, n16, blocks, unroll, nt, stream): n16 uint4 elements.
//   blocks > 0: grid-stride loop; each thread copies `unroll` elements one grid apart per trip.
//   blocks = 0: one workgroup per contiguous chunk of 256 * unroll elements (grid = n16 / chunk), no loop.
// nt = 1 uses non-temporal loads and stores.
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

template <int U, bool NT>
__global__ __launch_bounds__(256) void k_copy_chunk(u32x4* __restrict__ dst, const u32x4* __restrict__ src, size_t n)
{
    const size_t base = (size_t)blockIdx.x * (256 * U) + threadIdx.x;
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (base + u * 256 < n) v[u] = NT ? __builtin_nontemporal_load(src + base + u * 256) : src[base + u * 256];
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (base + u * 256 < n) {
            if (NT) __builtin_nontemporal_store(v[u], dst + base + u * 256);
            else dst[base + u * 256] = v[u];
        }
}

template <int U, bool NT>
static void launch(int blocks, u32x4* d, const u32x4* a, size_t n, hipStream_t s)
{
    if (blocks > 0) hipLaunchKernelGGL((k_copy<U, NT>), dim3(blocks), dim3(256), 0, s, d, a, n);
    else hipLaunchKernelGGL((k_copy_chunk<U, NT>), dim3((unsigned)((n + 256 * U - 1) / (256 * U))), dim3(256), 0, s,
                            d, a, n);
}

extern "C" int hbm_copy(void* dst, const void* src, size_t n16, int blocks, int unroll, int nt, void* stream)
{
    hipStream_t s = (hipStream_t)stream;
    u32x4* d = (u32x4*)dst;
    const u32x4* a = (const u32x4*)src;
    if (blocks < 0) return -1;
    switch (unroll * 2 + (nt ? 1 : 0)) {
    case 2: launch<1, false>(blocks, d, a, n16, s); break;
    case 3: launch<1, true>(blocks, d, a, n16, s); break;
    case 4: launch<2, false>(blocks, d, a, n16, s); break;
    case 5: launch<2, true>(blocks, d, a, n16, s); break;
    case 8: launch<4, false>(blocks, d, a, n16, s); break;
    case 9: launch<4, true>(blocks, d, a, n16, s); break;
    case 16: launch<8, false>(blocks, d, a, n16, s); break;
    case 17: launch<8, true>(blocks, d, a, n16, s); break;
    default: return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
