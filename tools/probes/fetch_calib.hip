// Probe: what rocprofv3 FETCH_SIZE counts on gfx950 for the access shapes of this library's kernels, against
// a known byte count (MI355X_MICROARCH.md: FETCH_SIZE reads half the bytes of a wide 16-B/lane streaming read;
// "other access widths are uncalibrated").  Each kernel reads a 256 MiB buffer (past the 256 MiB Infinity
// Cache) once:
//   k_dense16   16 B per lane, coalesced
//   k_dense4    4 B per lane, coalesced (the quadtree gather, k_si_* loads)
//   k_seg       60-byte runs at a 256-byte stride, 4 B per lane (k_quadtree's per-cell candidate slots:
//               a cell's candidates are contiguous, cells sit slot_cap apart)
// Run: rocprofv3 --pmc FETCH_SIZE -- ./fetch_calib ; the program prints each kernel's requested bytes.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

constexpr size_t kBytes = 256ull << 20;

__global__ void k_dense16(const uint4* __restrict__ p, size_t n, uint32_t* out)
{
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_dense4(const uint32_t* __restrict__ p, size_t n, uint32_t* out)
{
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        acc ^= p[i];
    if (acc == 0x12345678u) out[0] = acc;
}

// segment s (256 B apart) holds 15 dwords; thread t of the grid reads dword t % 16 of segment t / 16 (lane 15 of
// each group of 16 idle)
__global__ void k_seg(const uint32_t* __restrict__ p, size_t nseg, uint32_t* out)
{
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nseg * 16; i += (size_t)gridDim.x * blockDim.x) {
        const size_t s = i >> 4, j = i & 15;
        if (j < 15) acc ^= p[s * 64 + j];
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main()
{
    void* buf;
    uint32_t* out;
    hipMalloc(&buf, kBytes);
    hipMalloc(&out, 64);
    hipMemset(buf, 1, kBytes);
    hipDeviceSynchronize();
    const dim3 grid(256 * 32), block(256);
    hipLaunchKernelGGL(k_dense16, grid, block, 0, 0, (const uint4*)buf, kBytes / 16, out);
    hipLaunchKernelGGL(k_dense4, grid, block, 0, 0, (const uint32_t*)buf, kBytes / 4, out);
    hipLaunchKernelGGL(k_seg, grid, block, 0, 0, (const uint32_t*)buf, kBytes / 256, out);
    hipDeviceSynchronize();
    printf("requested bytes: k_dense16 %zu, k_dense4 %zu, k_seg %zu (60 of every 256; lines touched: %zu)\n", kBytes,
           kBytes, kBytes / 256 * 60, kBytes / 2);
    return 0;
}
