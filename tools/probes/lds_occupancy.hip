// LDS allocation granule on this GPU: the runtime's occupancy answer for one-wave workgroups of a given dynamic
// LDS size.  Build: hipcc --offload-arch=gfx950 -O2 -o tools/probes/ldsocc tools/probes/lds_occupancy.hip
// Measured (MI355X, ROCm 7.2): floor(163,840 / bytes) at this resolution -- 5,120 B 32, 5,121 B 31, 5,461 B 30,
// 5,462 B 29, 5,792 B (k_describe) 28, 6,720 B (k_fast_cells at KITTI) 24, 6,848 B 23: no coarse granule.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ __launch_bounds__(64) void k_lds(int* out)
{
    extern __shared__ int s[];
    s[threadIdx.x] = threadIdx.x;
    __syncthreads();
    if (out) out[threadIdx.x] = s[63 - threadIdx.x];
}
int main()
{
    const int sizes[] = {4096, 5120, 5121, 5248, 5376, 5461, 5462, 5632, 5633, 5792, 6144, 6145, 6400, 6720, 6784, 6848, 6912, 7168};
    for (int b : sizes) {
        int n = 0;
        if (hipFuncSetAttribute((const void*)k_lds, hipFuncAttributeMaxDynamicSharedMemorySize, 65536) != hipSuccess)
            return 1;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_lds, 64, b) != hipSuccess) return 1;
        printf("lds %5d B -> %2d one-wave workgroups per CU\n", b, n);
    }
    return 0;
}
