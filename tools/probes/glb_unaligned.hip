// Probe: global dword loads at byte-misaligned addresses on gfx950 -- exact against a byte model, and the
// cost against aligned loads in FAST's staging shape (each lane one dword of a 44-byte row segment, rows
// 1241 bytes apart, many waves).  Build: hipcc --offload-arch=gfx950 -O3 -o glb_unaligned glb_unaligned.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef const __attribute__((address_space(1))) uint8_t gbyte;

__global__ void k_check(const uint8_t* src, uint32_t* out)
{
    // lane l reads the dword at byte 7 * l + (l & 3) from the start
    const uint32_t o = 7u * threadIdx.x + (threadIdx.x & 3u);
    out[threadIdx.x] = *(const __attribute__((address_space(1))) uint32_t*)((gbyte*)src + o);
}

// FAST-like staging: wave w reads a 44 x 40 byte ROI at (row0, col0) of a 1241-pitch image, one dword per
// lane per pass (11 dwords per row, 5 rows per pass, 8 passes); kMis = 0: the ROI origin rounded down to a
// multiple of 4 (aligned loads, what the kernel does before realigning), 1: the exact origin
template <int kMis>
__global__ void k_time(const uint8_t* img, uint32_t* out, int iters)
{
    const int lane = threadIdx.x & 63, rl = lane / 11, kl = lane - 11 * (lane / 11);
    uint32_t acc = 0;
    uint32_t x = blockIdx.x * 2654435761u + threadIdx.x / 64 * 40503u;
    for (int it = 0; it < iters; ++it) {
        x = x * 1664525u + 1013904223u;
        const uint32_t row0 = (x >> 8) % 320u, col0 = (x >> 4) % 1180u;
        uint32_t org = row0 * 1241u + col0;
        if (!kMis) org &= ~3u;
        if (rl < 5) {
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const uint32_t o = org + (uint32_t)(u * 5 + rl) * 1241u + 4u * kl;
                acc += *(const __attribute__((address_space(1))) uint32_t*)((gbyte*)img + (kMis ? o : (o & ~3u)));
            }
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main()
{
    const size_t n = 1241 * 400 + 4096;
    std::vector<uint8_t> h(n);
    for (size_t i = 0; i < n; ++i) h[i] = (uint8_t)(i * 131 + (i >> 8) * 7);
    uint8_t* d;
    uint32_t* o;
    hipMalloc(&d, n);
    hipMalloc(&o, 1 << 24);
    hipMemcpy(d, h.data(), n, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_check, dim3(1), dim3(64), 0, 0, d, o);
    uint32_t r[64];
    hipMemcpy(r, o, sizeof(r), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; ++l) {
        const uint32_t a = 7u * l + (l & 3u);
        const uint32_t want = h[a] | (h[a + 1] << 8) | (h[a + 2] << 16) | ((uint32_t)h[a + 3] << 24);
        if (r[l] != want) {
            if (bad < 4) printf("lane %d: got %08x want %08x (byte %u)\n", l, r[l], want, a);
            ++bad;
        }
    }
    printf("misaligned global dword loads: %s (%d mismatches)\n", bad ? "WRONG" : "exact", bad);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 256, blocks = 256 * 24;
    for (int mis = 0; mis < 2; ++mis)
        for (int rep = 0; rep < 3; ++rep) {
            hipEventRecord(e0);
            if (mis) hipLaunchKernelGGL(k_time<1>, dim3(blocks), dim3(64), 0, 0, d, o, iters);
            else hipLaunchKernelGGL(k_time<0>, dim3(blocks), dim3(64), 0, 0, d, o, iters);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            if (rep) printf("%s: %.3f ms (%.1f G ROI passes/s)\n", mis ? "misaligned" : "aligned   ", ms,
                            (double)blocks * iters * 8 / ms / 1e6);
        }
    return bad != 0;
}
