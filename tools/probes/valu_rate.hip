// VALU issue-rate probe for the instructions that dominate the extractor kernels (k_fast_cells:
// v_pk_maximum3_f16 / v_pk_minimum3_f16, v_perm_b32, v_xor_b32; k_describe: v_dot4_u32_u8,
// v_alignbyte_b32, v_fma_f32; the matchers: v_bcnt_u32_b32).  Each lane runs 8 independent chains of
// one instruction (inline asm: exactly the instruction named), 32 per loop trip, over the whole chip
// at 1, 2, 4 and 8 waves per SIMD.  Prints wave-instructions per second per instruction and
// occupancy: the measured VALU peak that bench.py's roofline.valu divides by.
//   hipcc --offload-arch=gfx950 -O3 -o valu_rate tools/probes/valu_rate.hip && ./valu_rate
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                          \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                                 \
        }                                                                                 \
    } while (0)

constexpr int kIter = 4096;   // loop trips; 32 instructions per trip per wave

#define OP3(ins) asm volatile(ins " %0, %0, %1, %2" : "+v"(r) : "v"(b), "v"(c))
#define OP2(ins) asm volatile(ins " %0, %0, %1" : "+v"(r) : "v"(b))

template <int K>
__device__ __forceinline__ void op(uint32_t& r, uint32_t b, uint32_t c)
{
    if constexpr (K == 0) OP3("v_pk_maximum3_f16");
    else if constexpr (K == 1) OP3("v_perm_b32");
    else if constexpr (K == 2) OP2("v_xor_b32");
    else if constexpr (K == 3) OP2("v_bcnt_u32_b32");
    else if constexpr (K == 4) OP3("v_dot4_u32_u8");
    else if constexpr (K == 5) OP3("v_alignbyte_b32");
    else if constexpr (K == 6) OP3("v_fma_f32");
    else if constexpr (K == 7) OP3("v_pk_minimum3_f16");
    else if constexpr (K == 8) OP2("v_pk_max_f16");
    else if constexpr (K == 9) OP2("v_pk_add_u16");
    else if constexpr (K == 10) OP3("v_max3_u32");
    else if constexpr (K == 11) OP2("v_max_u32");
    else if constexpr (K == 12) OP3("v_dot2_u32_u16");
    else if constexpr (K == 13) OP3("v_lshl_or_b32");
    else if constexpr (K == 14) OP3("v_add3_u32");
    else if constexpr (K == 15) OP2("v_mul_lo_u32");
    else if constexpr (K == 16) OP3("v_mad_u32_u24");
    else if constexpr (K == 17) OP3("v_sad_u32");
    else if constexpr (K == 18) OP3("v_bfi_b32");
    else if constexpr (K == 19) OP2("v_pk_sub_u16");
}

template <int K>
__global__ __launch_bounds__(256) void k_rate(uint32_t* out, uint32_t seed)
{
    uint32_t r[8];
    const uint32_t b = seed ^ threadIdx.x, c = seed * 3u + blockIdx.x;
#pragma unroll
    for (int i = 0; i < 8; ++i) r[i] = seed + i * 0x01010101u + threadIdx.x;
    for (int it = 0; it < kIter; ++it) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
#pragma unroll
            for (int i = 0; i < 8; ++i) op<K>(r[i], b, c);
        }
    }
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) x ^= r[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;   // vector store keeps the chains live
}

template <int K>
double run(int waves_per_simd, int cus, uint32_t* out)
{
    const int blocks = cus * waves_per_simd;   // 256 threads = 4 waves = one per SIMD
    hipEvent_t a, z;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&z));
    hipLaunchKernelGGL(k_rate<K>, dim3(blocks), dim3(256), 0, 0, out, 7u);   // warm up
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a, 0));
    hipLaunchKernelGGL(k_rate<K>, dim3(blocks), dim3(256), 0, 0, out, 9u);
    CHECK(hipEventRecord(z, 0));
    CHECK(hipEventSynchronize(z));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, a, z));
    CHECK(hipEventDestroy(a));
    CHECK(hipEventDestroy(z));
    const double insts = (double)blocks * 4 * kIter * 32;   // wave-instructions
    return insts / (ms * 1e-3) / 1e9;                     // G wave-instr/s
}

int main()
{
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    uint32_t* out = nullptr;
    CHECK(hipMalloc(&out, sizeof(uint32_t) * 256 * cus * 8));
    constexpr int kOps = 20;
    const char* names[kOps] = {"v_pk_maximum3_f16", "v_perm_b32", "v_xor_b32", "v_bcnt_u32_b32", "v_dot4_u32_u8",
                               "v_alignbyte_b32", "v_fma_f32", "v_pk_minimum3_f16", "v_pk_max_f16", "v_pk_add_u16",
                               "v_max3_u32", "v_max_u32", "v_dot2_u32_u16", "v_lshl_or_b32", "v_add3_u32",
                               "v_mul_lo_u32", "v_mad_u32_u24", "v_sad_u32", "v_bfi_b32", "v_pk_sub_u16"};
    const double clk = p.clockRate * 1e3;   // Hz
    std::printf("{\"cus\": %d, \"clock_mhz\": %.0f, \"issue_peak_2cyc\": %.1f, \"rates\": {", cus, clk / 1e6,
                cus * 4 * clk / 2 / 1e9);
    const int occ[4] = {1, 2, 4, 8};
    for (int k = 0; k < kOps; ++k) {
        std::printf("%s\"%s\": [", k ? ", " : "", names[k]);
        for (int o = 0; o < 4; ++o) {
            double g = 0;
            switch (k) {
                case 0: g = run<0>(occ[o], cus, out); break;
                case 1: g = run<1>(occ[o], cus, out); break;
                case 2: g = run<2>(occ[o], cus, out); break;
                case 3: g = run<3>(occ[o], cus, out); break;
                case 4: g = run<4>(occ[o], cus, out); break;
                case 5: g = run<5>(occ[o], cus, out); break;
                case 6: g = run<6>(occ[o], cus, out); break;
                case 7: g = run<7>(occ[o], cus, out); break;
                case 8: g = run<8>(occ[o], cus, out); break;
                case 9: g = run<9>(occ[o], cus, out); break;
                case 10: g = run<10>(occ[o], cus, out); break;
                case 11: g = run<11>(occ[o], cus, out); break;
                case 12: g = run<12>(occ[o], cus, out); break;
                case 13: g = run<13>(occ[o], cus, out); break;
                case 14: g = run<14>(occ[o], cus, out); break;
                case 15: g = run<15>(occ[o], cus, out); break;
                case 16: g = run<16>(occ[o], cus, out); break;
                case 17: g = run<17>(occ[o], cus, out); break;
                case 18: g = run<18>(occ[o], cus, out); break;
                case 19: g = run<19>(occ[o], cus, out); break;
            }
            std::printf("%s%.1f", o ? ", " : "", g);
        }
        std::printf("]");
    }
    std::printf("}, \"waves_per_simd\": [1, 2, 4, 8], \"unit\": \"G wave-instr/s\"}\n");
    CHECK(hipFree(out));
    return 0;
}
