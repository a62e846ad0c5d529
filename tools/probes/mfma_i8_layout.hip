// Probe: operand / result layout of v_mfma_i32_32x32x32_i8 on gfx950.
// A[m][k], B[k][n] random int8 (row-major in global), C = A*B; lane l (r = l&31, h = l>>5)
// is assumed to hold A[r][16h + j] and B[16h + j][r] (j = 0..15), C rows (reg&3)+8*(reg>>2)+4h.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
__global__ void k(const signed char* A, const signed char* B, int* C)
{
    const int l = threadIdx.x, r = l & 31, h = l >> 5;
    signed char a[16], b[16];
    for (int j = 0; j < 16; ++j) { a[j] = A[r * 32 + 16 * h + j]; b[j] = B[(16 * h + j) * 32 + r]; }
    v4i av, bv;
    __builtin_memcpy(&av, a, 16);
    __builtin_memcpy(&bv, b, 16);
    v16i c = {0};
    c = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bv, c, 0, 0, 0);
    for (int g = 0; g < 16; ++g) C[((g & 3) + 8 * (g >> 2) + 4 * h) * 32 + r] = c[g];
}
int main()
{
    signed char hA[1024], hB[1024];
    int hC[1024], ref[1024];
    srand(1);
    for (int i = 0; i < 1024; ++i) { hA[i] = (signed char)(rand() % 256 - 128); hB[i] = (signed char)(rand() % 256 - 128); }
    for (int m = 0; m < 32; ++m)
        for (int n = 0; n < 32; ++n) {
            int s = 0;
            for (int q = 0; q < 32; ++q) s += hA[m * 32 + q] * hB[q * 32 + n];
            ref[m * 32 + n] = s;
        }
    signed char *dA, *dB;
    int* dC;
    hipMalloc(&dA, 1024); hipMalloc(&dB, 1024); hipMalloc(&dC, 4096);
    hipMemcpy(dA, hA, 1024, hipMemcpyHostToDevice);
    hipMemcpy(dB, hB, 1024, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dC);
    hipMemcpy(hC, dC, 4096, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 1024; ++i) bad += hC[i] != ref[i];
    printf("mfma_i32_32x32x32_i8 layout mismatches: %d / 1024 (C[0]=%d ref=%d)\n", bad, hC[0], ref[0]);
    return bad != 0;
}
