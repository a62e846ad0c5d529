// gfx950 kernels of the ORBmatcher Hamming searches (include/ORBmatcher.h:37-102).
//
//   M3 k_allpairs_top2 / k_allpairs_full   brute-force 256-bit Hamming (config 5)
//   M1 k_search_init                        SearchForInitialization, src/ORBmatcher.cc:417-588
//
// Distance = popcount(a ^ b) over four little-endian u64 words, identical to
// the reference's 8 x u32 SWAR DescriptorDistance (src/ORBmatcher.cc:1728-1744).
#include <hip/hip_runtime.h>
#include <limits.h>

#include "orbx_kernels.hpp"

namespace orbx {

__device__ __forceinline__ int ham256(const ulonglong2& a0, const ulonglong2& a1, const ulonglong2& b0,
                                      const ulonglong2& b1)
{
    return __popcll(a0.x ^ b0.x) + __popcll(a0.y ^ b0.y) + __popcll(a1.x ^ b1.x) + __popcll(a1.y ^ b1.y);
}

// ---------------------------------------------------------------------------
// M3 TOP2: each thread owns one query; targets stream through LDS in tiles of
// 256 and are read by broadcast.  Targets are split over blockIdx.y so the
// 10k x 10k case fills all 256 CUs; partial (best, second, idx) triples are
// merged in target order, which keeps the reference's first-min tie rule.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_allpairs_top2(const ulonglong2* __restrict__ q, int nq,
                                                       const ulonglong2* __restrict__ t, int nt, int chunk,
                                                       int* __restrict__ part)
{
    __shared__ ulonglong2 st[256 * 2];
    const int tid = threadIdx.x;
    const int qi = blockIdx.x * 256 + tid;
    const int t0 = blockIdx.y * chunk, t1 = min(nt, t0 + chunk);
    ulonglong2 a0 = make_ulonglong2(0, 0), a1 = a0;
    if (qi < nq) {
        a0 = q[2 * (size_t)qi];
        a1 = q[2 * (size_t)qi + 1];
    }
    int b1 = 256, b2 = 256, bi = -1;
    for (int base = t0; base < t1; base += 256) {
        const int n = min(256, t1 - base);
        __syncthreads();
        if (tid < n) {
            st[2 * tid] = t[2 * (size_t)(base + tid)];
            st[2 * tid + 1] = t[2 * (size_t)(base + tid) + 1];
        }
        __syncthreads();
        for (int j = 0; j < n; ++j) {
            const int d = ham256(a0, a1, st[2 * j], st[2 * j + 1]);
            if (d < b1) {
                b2 = b1;
                b1 = d;
                bi = base + j;
            } else if (d < b2) {
                b2 = d;
            }
        }
    }
    if (qi < nq) {
        int* o = part + 3 * ((size_t)blockIdx.y * nq + qi);
        o[0] = b1;
        o[1] = b2;
        o[2] = bi;
    }
}

__global__ void k_allpairs_merge(const int* __restrict__ part, int nq, int nsplit, int* __restrict__ bi_out,
                                 int* __restrict__ b1_out, int* __restrict__ b2_out)
{
    const int qi = blockIdx.x * blockDim.x + threadIdx.x;
    if (qi >= nq) return;
    int B1 = 256, B2 = 256, BI = -1;
    for (int s = 0; s < nsplit; ++s) {
        const int* p = part + 3 * ((size_t)s * nq + qi);
        const int y1 = p[0], y2 = p[1], yi = p[2];
        if (y1 < B1) {
            B2 = min(B1, y2);
            B1 = y1;
            BI = yi;
        } else {
            B2 = min(B2, y1);
        }
    }
    bi_out[qi] = BI;
    b1_out[qi] = B1;
    b2_out[qi] = B2;
}

void launch_allpairs_top2(const uint8_t* q, int nq, const uint8_t* t, int nt, int* bi, int* b1, int* b2,
                          int* part, int nsplit, hipStream_t s)
{
    int chunk = (nt + nsplit - 1) / nsplit;
    chunk = (chunk + 255) / 256 * 256;
    const int used = chunk > 0 ? (nt + chunk - 1) / chunk : 1;
    dim3 grid((nq + 255) / 256, used > 0 ? used : 1);
    hipLaunchKernelGGL(k_allpairs_top2, grid, dim3(256), 0, s, (const ulonglong2*)q, nq, (const ulonglong2*)t,
                       nt, chunk, part);
    hipLaunchKernelGGL(k_allpairs_merge, dim3((nq + 255) / 256), dim3(256), 0, s, part, nq, (int)grid.y, bi, b1,
                       b2);
}

// ---------------------------------------------------------------------------
// M3 FULL_U16: the nq x nt distance matrix.  A thread keeps 4 consecutive
// targets in registers; a block stages 64 queries in LDS and writes one
// 8-byte (4 x u16) store per lane per query: 512 contiguous bytes per wave.
// HBM-write bound (2 bytes per pair).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_allpairs_full(const ulonglong2* __restrict__ q, int nq,
                                                       const ulonglong2* __restrict__ t, int nt,
                                                       uint16_t* __restrict__ out)
{
    __shared__ ulonglong2 sq[64 * 2];
    const int tid = threadIdx.x;
    const int tb = (blockIdx.x * 256 + tid) * 4;
    const int q0 = blockIdx.y * 64;
    const int nqb = min(64, nq - q0);
    if (tid < 2 * nqb) sq[tid] = q[2 * (size_t)q0 + tid];
    ulonglong2 r[4][2];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int ti = tb + k;
        if (ti < nt) {
            r[k][0] = t[2 * (size_t)ti];
            r[k][1] = t[2 * (size_t)ti + 1];
        } else {
            r[k][0] = r[k][1] = make_ulonglong2(0, 0);
        }
    }
    __syncthreads();
    if (tb >= nt) return;
    const bool full = tb + 4 <= nt && (nt & 3) == 0;
    for (int i = 0; i < nqb; ++i) {
        const ulonglong2 a0 = sq[2 * i], a1 = sq[2 * i + 1];
        uint16_t d[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) d[k] = (uint16_t)ham256(a0, a1, r[k][0], r[k][1]);
        uint16_t* o = out + (size_t)(q0 + i) * nt + tb;
        if (full) {
            const unsigned long long v = (unsigned long long)d[0] | ((unsigned long long)d[1] << 16) |
                                         ((unsigned long long)d[2] << 32) | ((unsigned long long)d[3] << 48);
            *reinterpret_cast<unsigned long long*>(o) = v;
        } else {
            for (int k = 0; k < 4 && tb + k < nt; ++k) o[k] = d[k];
        }
    }
}

void launch_allpairs_full(const uint8_t* q, int nq, const uint8_t* t, int nt, uint16_t* out, hipStream_t s)
{
    dim3 grid((nt + 1023) / 1024, (nq + 63) / 64);
    hipLaunchKernelGGL(k_allpairs_full, grid, dim3(256), 0, s, (const ulonglong2*)q, nq, (const ulonglong2*)t, nt,
                       out);
}

// ---------------------------------------------------------------------------
// M1: SearchForInitialization for one frame pair per workgroup (512 threads).
//   1. F2's level-0 keypoints are sorted the way Frame::GetFeaturesInArea
//      visits them: grid cell (ix outer, iy inner, Frame::PosInGrid rounding),
//      then index (AssignFeaturesToGrid insertion order), src/Frame.cc:292-518.
//      Keys and positions stay in LDS.
//   2. Every wave takes level-0 queries; a query's window columns are one
//      contiguous key range (binary search), filtered by row and |dx|,|dy| < r.
//      Candidate lists (i2, Hamming) are written in visit order, CSR, in LDS
//      (global scratch only if a pair overflows the LDS budget).
//   3. One wave replays the greedy pass in query order (vMatchedDistance skip,
//      best/second, ratio test, eviction), then the rotation-histogram filter
//      (ComputeThreeMaxima, src/ORBmatcher.cc:1679-1723).
// ---------------------------------------------------------------------------
constexpr int kGridCols = 64, kGridRows = 48;
constexpr int SI_NT = 512, SI_NW = SI_NT / 64;

__device__ __forceinline__ void bitonic_asc(uint32_t* k, int p2)
{
    for (int size = 2; size <= p2; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int i = threadIdx.x; i < (p2 >> 1); i += blockDim.x) {
                const int lo = 2 * i - (i & (stride - 1));
                const int hi = lo + stride;
                const bool asc = (lo & size) == 0;
                const uint32_t a = k[lo], b = k[hi];
                if ((a > b) == asc) {
                    k[lo] = b;
                    k[hi] = a;
                }
            }
            __syncthreads();
        }
    }
}

__device__ __forceinline__ int lower_bound_u32(const uint32_t* a, int n, uint32_t v)
{
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (a[mid] < v) lo = mid + 1; else hi = mid;
    }
    return lo;
}

struct SiLayout {
    size_t keys, gxy, off, mdist, m21, m12, bin, cand, total;
};

__host__ __device__ inline SiLayout si_layout(int cap, int cand_lds)
{
    SiLayout L;
    int p2 = 1;
    while (p2 < cap) p2 <<= 1;
    size_t o = 0;
    auto take = [&](size_t b) {
        const size_t r = o;
        o += (b + 15) & ~(size_t)15;
        return r;
    };
    L.keys = take(4 * (size_t)p2);
    L.gxy = take(8 * (size_t)cap);
    L.off = take(4 * ((size_t)cap + 1));
    L.mdist = take(2 * (size_t)cap);
    L.m21 = take(2 * (size_t)cap);
    L.m12 = take(2 * (size_t)cap);
    L.bin = take((size_t)cap);
    L.cand = take(4 * (size_t)cand_lds);
    L.total = o;
    return L;
}

__global__ __launch_bounds__(SI_NT) void k_search_init(const orbx_keypoint* __restrict__ kps,
                                                       const uint8_t* __restrict__ desc,
                                                       const int* __restrict__ counts, int cap,
                                                       const int* __restrict__ pa, const int* __restrict__ pb,
                                                       int rows, int cols, int window, float nnratio, int check_ori,
                                                       uint32_t* __restrict__ cand_g, int cand_per_pair, int cand_lds,
                                                       int* __restrict__ m12_out, int* __restrict__ nm_out)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const SiLayout Ly = si_layout(cap, cand_lds);
    uint32_t* keys = (uint32_t*)(smem + Ly.keys);
    float2* gxy = (float2*)(smem + Ly.gxy);
    uint32_t* off = (uint32_t*)(smem + Ly.off);
    uint16_t* mdist = (uint16_t*)(smem + Ly.mdist);
    int16_t* m21 = (int16_t*)(smem + Ly.m21);
    int16_t* m12 = (int16_t*)(smem + Ly.m12);
    int8_t* bin = (int8_t*)(smem + Ly.bin);
    uint32_t* cand_l = (uint32_t*)(smem + Ly.cand);
    __shared__ int s_n[4];
    __shared__ int s_hist[32];

    const int pair = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int fa = pa[pair], fb = pb[pair];
    const orbx_keypoint* k1 = kps + (size_t)fa * cap;
    const orbx_keypoint* k2 = kps + (size_t)fb * cap;
    const uint8_t* d1 = desc + (size_t)fa * cap * 32;
    const uint8_t* d2 = desc + (size_t)fb * cap * 32;
    const int n1 = min(counts[fa], cap), n2 = min(counts[fb], cap);
    if (tid < 4) s_n[tid] = 0;
    __syncthreads();
    // level-0 keypoints come first (src/ORBextractor.cc:1290-1333)
    int c1 = 0, c2 = 0;
    for (int i = tid; i < n1; i += SI_NT) c1 += k1[i].octave == 0;
    for (int i = tid; i < n2; i += SI_NT) c2 += k2[i].octave == 0;
    if (c1) atomicAdd(&s_n[0], c1);
    if (c2) atomicAdd(&s_n[1], c2);
    __syncthreads();
    const int n10 = s_n[0], n20 = s_n[1];
    int p2 = 1;
    while (p2 < n20) p2 <<= 1;

    const float invW = (float)kGridCols / ((float)cols - 0.0f);
    const float invH = (float)kGridRows / ((float)rows - 0.0f);
    for (int i = tid; i < p2; i += SI_NT) {
        uint32_t key = 0xFFFFFFFFu;
        if (i < n20) {
            const int px = (int)roundf((k2[i].x - 0.0f) * invW);
            const int py = (int)roundf((k2[i].y - 0.0f) * invH);
            if (px >= 0 && px < kGridCols && py >= 0 && py < kGridRows) {
                key = ((uint32_t)(px * kGridRows + py) << 16) | (uint32_t)i;
                atomicAdd(&s_n[2], 1);
            }
        }
        keys[i] = key;
    }
    __syncthreads();
    bitonic_asc(keys, p2);   // invalid keys (outside the grid, PosInGrid false) sort last
    const int ng_ = s_n[2];
    for (int g = tid; g < ng_; g += SI_NT) {
        const int i2 = (int)(keys[g] & 0xFFFF);
        gxy[g] = make_float2(k2[i2].x, k2[i2].y);
    }
    __syncthreads();
    const int ng = ng_;

    const float r = (float)window;
    uint32_t* pc = cand_l;
    for (int pass = 0; pass < 2; ++pass) {
        for (int i1 = wave; i1 < n10; i1 += SI_NW) {
            const float x = k1[i1].x, y = k1[i1].y;
            // Frame::GetFeaturesInArea(x, y, r, 0, 0) cell range, src/Frame.cc:421-440
            const int cx0 = max(0, (int)floorf((x - 0.0f - r) * invW));
            const int cx1 = min(kGridCols - 1, (int)ceilf((x - 0.0f + r) * invW));
            const int cy0 = max(0, (int)floorf((y - 0.0f - r) * invH));
            const int cy1 = min(kGridRows - 1, (int)ceilf((y - 0.0f + r) * invH));
            int base = pass ? (int)off[i1] : 0;
            if (cx0 < kGridCols && cx1 >= 0 && cy0 < kGridRows && cy1 >= 0) {
                const int lo = lower_bound_u32(keys, ng, (uint32_t)(cx0 * kGridRows) << 16);
                const int hi = lower_bound_u32(keys, ng, (uint32_t)((cx1 + 1) * kGridRows) << 16);
                ulonglong2 a0 = make_ulonglong2(0, 0), a1 = a0;
                if (pass) {
                    const ulonglong2* a = (const ulonglong2*)(d1 + (size_t)i1 * 32);
                    a0 = a[0];
                    a1 = a[1];
                }
                for (int g0 = lo; g0 < hi; g0 += 64) {
                    const int g = g0 + lane;
                    bool in = false;
                    int i2 = 0;
                    if (g < hi) {
                        const uint32_t key = keys[g];
                        const int iy = (int)(key >> 16) % kGridRows;
                        if (iy >= cy0 && iy <= cy1) {
                            const float2 p = gxy[g];
                            in = fabsf(p.x - x) < r && fabsf(p.y - y) < r;
                            i2 = (int)(key & 0xFFFF);
                        }
                    }
                    const unsigned long long m = __ballot(in);
                    if (pass && in) {
                        const ulonglong2* b = (const ulonglong2*)(d2 + (size_t)i2 * 32);
                        const int d = ham256(a0, a1, b[0], b[1]);
                        const int idx = base + (int)__builtin_amdgcn_mbcnt_hi(
                                                   (uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                        pc[idx] = (uint32_t)i2 | ((uint32_t)d << 16);
                    }
                    base += __popcll(m);
                }
            }
            if (!pass && lane == 0) off[i1] = (uint32_t)base;
        }
        __syncthreads();
        if (!pass) {
            // exclusive scan of off[0..n10) (one wave; n10 is a few hundred)
            if (wave == 0) {
                uint32_t run = 0;
                for (int b0 = 0; b0 < n10; b0 += 64) {
                    const int i = b0 + lane;
                    const uint32_t v = i < n10 ? off[i] : 0u;
                    uint32_t inc = v;
                    for (int o = 1; o < 64; o <<= 1) {
                        const uint32_t y = __shfl_up(inc, o);
                        if (lane >= o) inc += y;
                    }
                    if (i < n10) off[i] = run + inc - v;
                    run += __shfl(inc, 63);
                }
                if (lane == 0) {
                    off[n10] = run;
                    s_n[3] = (int)run;
                }
            }
            __syncthreads();
            const int total = s_n[3];
            if (total > cand_lds) {
                if (total > cand_per_pair) {   // cannot hold the lists: report, do nothing
                    for (int i = tid; i < cap; i += SI_NT) m12_out[(size_t)pair * cap + i] = -1;
                    if (tid == 0) nm_out[pair] = -1;
                    return;
                }
                pc = cand_g + (size_t)pair * cand_per_pair;
            }
        }
    }

    if (wave != 0) return;
    // pass B: the reference's sequential greedy loop
    for (int i = lane; i < n2; i += 64) {
        mdist[i] = 0xFFFF;   // INT_MAX: larger than any distance
        m21[i] = -1;
    }
    for (int i = lane; i < n1; i += 64) {
        m12[i] = -1;
        bin[i] = -1;
    }
    if (lane < 32) s_hist[lane] = 0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    int nmatches = 0;
    const float factor = 1.0f / 30;
    for (int i1 = 0; i1 < n10; ++i1) {
        const int o0 = (int)off[i1], o1 = (int)off[i1 + 1];
        if (o1 == o0) continue;   // vIndices2.empty()
        int b1 = INT_MAX, b2 = INT_MAX, bp = INT_MAX;
        for (int j = o0 + lane; j < o1; j += 64) {
            const uint32_t e = pc[j];
            const int i2 = (int)(e & 0xFFFF), d = (int)(e >> 16);
            if ((int)mdist[i2] <= d) continue;
            if (d < b1) {
                b2 = b1;
                b1 = d;
                bp = j;
            } else if (d < b2) {
                b2 = d;
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const int y1 = __shfl_xor(b1, o), yp = __shfl_xor(bp, o), y2 = __shfl_xor(b2, o);
            if (y1 < b1 || (y1 == b1 && yp < bp)) {
                b2 = min(b1, y2);
                b1 = y1;
                bp = yp;
            } else {
                b2 = min(b2, y1);
            }
        }
        if (b1 <= 50 && (float)b1 < (float)b2 * nnratio) {
            const int bi = (int)(pc[bp] & 0xFFFF);
            if (lane == 0) {
                if (m21[bi] >= 0) {
                    m12[m21[bi]] = -1;
                    --nmatches;
                }
                m12[i1] = (int16_t)bi;
                m21[bi] = (int16_t)i1;
                mdist[bi] = (uint16_t)b1;
                ++nmatches;
                if (check_ori) {
                    float rot = k1[i1].angle - k2[bi].angle;
                    if (rot < 0.0f) rot += 360.0f;
                    int bb = (int)roundf(rot * factor);
                    if (bb == 30) bb = 0;
                    bin[i1] = (int8_t)bb;
                    s_hist[bb] += 1;
                }
            }
            nmatches = __shfl(nmatches, 0);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
    }
    if (check_ori) {
        int ind1 = -1, ind2 = -1, ind3 = -1, max1 = 0, max2 = 0, max3 = 0;
        for (int i = 0; i < 30; ++i) {
            const int s = s_hist[i];
            if (s > max1) { max3 = max2; max2 = max1; max1 = s; ind3 = ind2; ind2 = ind1; ind1 = i; }
            else if (s > max2) { max3 = max2; max2 = s; ind3 = ind2; ind2 = i; }
            else if (s > max3) { max3 = s; ind3 = i; }
        }
        if ((float)max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
        else if ((float)max3 < 0.1f * (float)max1) { ind3 = -1; }
        int removed = 0;
        for (int i = lane; i < n10; i += 64) {
            const int bb = bin[i];
            if (bb < 0 || bb == ind1 || bb == ind2 || bb == ind3) continue;
            if (m12[i] >= 0) {
                m12[i] = -1;
                ++removed;
            }
        }
        for (int o = 32; o > 0; o >>= 1) removed += __shfl_xor(removed, o);
        nmatches -= removed;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    int* out = m12_out + (size_t)pair * cap;
    for (int i = lane; i < cap; i += 64) out[i] = i < n1 ? (int)m12[i] : -1;
    if (lane == 0) nm_out[pair] = nmatches;
}

int search_init_cand_lds(int cap)
{
    // LDS left for candidate lists after the per-pair arrays (160 KiB per CU, one pair per workgroup)
    const size_t fixed = si_layout(cap, 0).total + 256;
    const long left = (long)(160 * 1024) - (long)fixed;
    return left > 0 ? (int)(left / 4) : 0;
}

void launch_search_init(const orbx_keypoint* kps, const uint8_t* desc, const int* counts, int cap, const int* pa,
                        const int* pb, int npairs, int rows, int cols, int window, float nnratio, int check_ori,
                        uint32_t* cand, int cand_per_pair, int* m12, int* nm, hipStream_t s)
{
    const int cand_lds = search_init_cand_lds(cap);
    const size_t smem = si_layout(cap, cand_lds).total;
    hipFuncSetAttribute((const void*)k_search_init, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    hipLaunchKernelGGL(k_search_init, dim3(npairs), dim3(SI_NT), smem, s, kps, desc, counts, cap, pa, pb, rows, cols,
                       window, nnratio, check_ori, cand, cand_per_pair, cand_lds, m12, nm);
}

}  // namespace orbx
