// Probe: operand / result layout of v_mfma_i32_16x16x64_i8 on gfx950.
// Assumed: lane l (r = l&15, h = l>>4) holds A[r][16h + j] and B[16h + j][r] (j = 0..15),
// C[4h + g][r] in accumulator register g.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef int v4i __attribute__((ext_vector_type(4)));
__global__ void k(const signed char* A, const signed char* B, int* C)
{
    const int l = threadIdx.x, r = l & 15, h = l >> 4;
    signed char a[16], b[16];
    for (int j = 0; j < 16; ++j) { a[j] = A[r * 64 + 16 * h + j]; b[j] = B[(16 * h + j) * 16 + r]; }
    v4i av, bv;
    __builtin_memcpy(&av, a, 16);
    __builtin_memcpy(&bv, b, 16);
    v4i c = {0, 0, 0, 0};
    c = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bv, c, 0, 0, 0);
    for (int g = 0; g < 4; ++g) C[(4 * h + g) * 16 + r] = c[g];
}
int main()
{
    signed char hA[1024], hB[1024];
    int hC[256], ref[256];
    srand(2);
    for (int i = 0; i < 1024; ++i) { hA[i] = (signed char)(rand() % 256 - 128); hB[i] = (signed char)(rand() % 256 - 128); }
    for (int m = 0; m < 16; ++m)
        for (int n = 0; n < 16; ++n) {
            int s = 0;
            for (int q = 0; q < 64; ++q) s += hA[m * 64 + q] * hB[q * 16 + n];
            ref[m * 16 + n] = s;
        }
    signed char *dA, *dB;
    int* dC;
    (void)hipMalloc(&dA, 1024); (void)hipMalloc(&dB, 1024); (void)hipMalloc(&dC, 1024);
    (void)hipMemcpy(dA, hA, 1024, hipMemcpyHostToDevice);
    (void)hipMemcpy(dB, hB, 1024, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dC);
    (void)hipMemcpy(hC, dC, 1024, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 256; ++i) bad += hC[i] != ref[i];
    printf("mfma_i32_16x16x64_i8 layout mismatches: %d / 256 (C[0]=%d ref=%d)\n", bad, hC[0], ref[0]);
    return bad != 0;
}
