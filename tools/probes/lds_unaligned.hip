// Probe: LDS reads at 2-byte-misaligned addresses on gfx950 (correctness against a byte model, and the
// cost of random gathers of four dwords at aligned vs misaligned addresses, the shape of k_describe's
// BRIEF samples).  Build: hipcc --offload-arch=gfx950 -O3 -o lds_unaligned lds_unaligned.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

constexpr int kWords = 1024;   // 4 KB table per workgroup

// lane reads 4 dwords from byte address 2 * (u16 index) (misaligned when the index is odd)
__global__ void k_check(const uint32_t* idx, uint32_t* out)
{
    __shared__ __attribute__((aligned(16))) uint32_t s[kWords + 8];
    for (int i = threadIdx.x; i < kWords + 8; i += 64) s[i] = 0x01000100u * (uint32_t)(2 * i) + 0x00010001u * (uint32_t)i;
    __syncthreads();
    const uint32_t u16i = idx[threadIdx.x];
    const uint32_t addr = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t*)s + 2u * u16i;
    const __attribute__((address_space(3))) uint32_t* p = (const __attribute__((address_space(3))) uint32_t*)(uintptr_t)addr;
    out[4 * threadIdx.x + 0] = p[0];
    out[4 * threadIdx.x + 1] = p[1];
    out[4 * threadIdx.x + 2] = p[2];
    out[4 * threadIdx.x + 3] = p[3];
}

// timing: every lane gathers 4 dwords at a pseudo-random u16 index per iteration; kMis = 0 rounds the index
// down to even (aligned), 1 keeps it (half the reads misaligned)
template <int kMis>
__global__ void k_time(uint32_t* out, int iters)
{
    __shared__ __attribute__((aligned(16))) uint32_t s[kWords + 8];
    for (int i = threadIdx.x; i < kWords + 8; i += blockDim.x) s[i] = (uint32_t)i * 2654435761u;
    __syncthreads();
    const uint32_t base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t*)s;
    uint32_t x = threadIdx.x * 977u + blockIdx.x * 131u, acc = 0;
    for (int it = 0; it < iters; ++it) {
        x = x * 1664525u + 1013904223u;
        uint32_t u = (x >> 8) % (2 * kWords - 8);
        if (!kMis) u &= ~1u;
        const __attribute__((address_space(3))) uint32_t* p =
            (const __attribute__((address_space(3))) uint32_t*)(uintptr_t)(base + 2u * u);
        acc += p[0] ^ p[1] ^ p[2] ^ p[3];
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main()
{
    uint32_t hidx[64];
    for (int i = 0; i < 64; ++i) hidx[i] = (uint32_t)(i * 37 + (i & 1)) % (2 * kWords);
    uint32_t *didx, *dout;
    hipMalloc(&didx, sizeof(hidx));
    hipMalloc(&dout, 1 << 24);
    hipMemcpy(didx, hidx, sizeof(hidx), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_check, dim3(1), dim3(64), 0, 0, didx, dout);
    uint32_t hout[256];
    hipMemcpy(hout, dout, sizeof(hout), hipMemcpyDeviceToHost);
    // byte model of the table
    static uint8_t bytes[4 * (kWords + 8)];
    for (int i = 0; i < kWords + 8; ++i) {
        const uint32_t v = 0x01000100u * (uint32_t)(2 * i) + 0x00010001u * (uint32_t)i;
        for (int b = 0; b < 4; ++b) bytes[4 * i + b] = (uint8_t)(v >> (8 * b));
    }
    int bad = 0;
    for (int l = 0; l < 64; ++l)
        for (int k = 0; k < 4; ++k) {
            const uint32_t a = 2 * hidx[l] + 4 * k;
            const uint32_t want = bytes[a] | (bytes[a + 1] << 8) | (bytes[a + 2] << 16) | ((uint32_t)bytes[a + 3] << 24);
            if (hout[4 * l + k] != want) {
                if (bad < 4) printf("lane %d dword %d: got %08x want %08x (u16 index %u)\n", l, k, hout[4 * l + k], want, hidx[l]);
                ++bad;
            }
        }
    printf("misaligned LDS reads: %s (%d mismatches)\n", bad ? "WRONG" : "exact", bad);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 4096, blocks = 256 * 28;
    for (int mis = 0; mis < 2; ++mis) {
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(e0);
            if (mis) hipLaunchKernelGGL(k_time<1>, dim3(blocks), dim3(64), 0, 0, dout, iters);
            else hipLaunchKernelGGL(k_time<0>, dim3(blocks), dim3(64), 0, 0, dout, iters);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            if (rep) printf("%s: %.3f ms (%.1f G gathers/s)\n", mis ? "misaligned" : "aligned   ", ms,
                            (double)blocks * 64 * iters / ms / 1e6);
        }
    }
    return bad != 0;
}
