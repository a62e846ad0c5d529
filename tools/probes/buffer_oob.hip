// Does a raw buffer load's range check (offset vs the descriptor's num_records) include the scalar offset
// (soffset)?  A 64-byte descriptor over a 4 KiB buffer of nonzero words; each lane loads its dword at
// voffset = 4 lane with soffset 0, 64 and 256.  Zeros past byte 64 in every row mean the check covers the
// sum; data means soffset bypasses it.  k_fast_cells' first staging passes (fast_issue0,
// orb-slam-_amd/csrc/orbx_extract.hip) rely on the first answer: tests/test_gpu_edges.py runs this probe
// through liboob_probe.so (built by __graft_entry__.build()) on every GPU test pass.
//   hipcc --offload-arch=gfx950 -O2 -o /tmp/buffer_oob tools/probes/buffer_oob.hip && /tmp/buffer_oob
//   hipcc --offload-arch=gfx950 -O2 -shared -fPIC -DOOB_PROBE_LIB -o tools/probes/liboob_probe.so tools/probes/buffer_oob.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void k_probe(const uint32_t* src, uint32_t* out)
{
    const int lane = threadIdx.x;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, 64, 0x00020000);
    const int soff[3] = {0, 64, 256};
#pragma unroll
    for (int k = 0; k < 3; ++k) out[k * 64 + lane] = __builtin_amdgcn_raw_buffer_load_b32(rs, 4u * lane, soff[k], 0);
}

// r[3 * 64]: the 64 lanes' loads at soffset 0, 64, 256 over h[i] = 0x1000 + i.  Returns 0 on success.
extern "C" int oob_probe_run(uint32_t* r)
{
    uint32_t h[1024];
    for (int i = 0; i < 1024; ++i) h[i] = 0x1000u + i;
    uint32_t *d = nullptr, *o = nullptr;
    int rc = 1;
    if (hipMalloc(&d, sizeof(h)) == hipSuccess && hipMalloc(&o, 3 * 64 * 4) == hipSuccess &&
        hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice) == hipSuccess) {
        hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, d, o);
        if (hipGetLastError() == hipSuccess && hipMemcpy(r, o, 3 * 64 * 4, hipMemcpyDeviceToHost) == hipSuccess) rc = 0;
    }
    if (d) (void)hipFree(d);
    if (o) (void)hipFree(o);
    return rc;
}

#ifndef OOB_PROBE_LIB
int main()
{
    uint32_t r[3 * 64];
    if (oob_probe_run(r) != 0) return 1;
    for (int k = 0; k < 3; ++k) {
        int nz = 0, first_zero = -1;
        for (int l = 0; l < 64; ++l) {
            if (r[k * 64 + l]) ++nz;
            else if (first_zero < 0) first_zero = l;
        }
        printf("soffset %3d: %2d nonzero lanes, first zero lane %d, lane0 %#x lane15 %#x lane16 %#x\n", k == 0 ? 0 : k == 1 ? 64 : 256,
               nz, first_zero, r[k * 64], r[k * 64 + 15], r[k * 64 + 16]);
    }
    return 0;
}
#endif
