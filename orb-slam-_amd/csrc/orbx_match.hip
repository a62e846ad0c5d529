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
// M1: SearchForInitialization for one frame pair per workgroup.
//   1. F2's level-0 keypoints are ordered like Frame::GetFeaturesInArea visits
//      them: grid cell (ix outer, iy inner, Frame::PosInGrid rounding), then
//      index (AssignFeaturesToGrid insertion order), src/Frame.cc:292-518.
//   2. All waves build every level-0 query's candidate list (window test and
//      Hamming distance) in that order: CSR in global scratch.
//   3. One wave replays the greedy pass in query order (vMatchedDistance skip,
//      best/second, ratio test, eviction), then the rotation-histogram filter
//      (ComputeThreeMaxima, src/ORBmatcher.cc:1679-1723).
// ---------------------------------------------------------------------------
constexpr int kGridCols = 64, kGridRows = 48;

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

struct Window {
    int cx0, cx1, cy0, cy1;
    bool empty;
};

// Frame::GetFeaturesInArea cell range, src/Frame.cc:421-440 (float arithmetic as written)
__device__ __forceinline__ Window window_cells(float x, float y, float r, float invW, float invH)
{
    Window w;
    const float minX = 0.0f, minY = 0.0f;
    w.cx0 = max(0, (int)floorf((x - minX - r) * invW));
    w.cx1 = min(kGridCols - 1, (int)ceilf((x - minX + r) * invW));
    w.cy0 = max(0, (int)floorf((y - minY - r) * invH));
    w.cy1 = min(kGridRows - 1, (int)ceilf((y - minY + r) * invH));
    w.empty = w.cx0 >= kGridCols || w.cx1 < 0 || w.cy0 >= kGridRows || w.cy1 < 0;
    return w;
}

__global__ __launch_bounds__(256) void k_search_init(const orbx_keypoint* __restrict__ kps,
                                                     const uint8_t* __restrict__ desc,
                                                     const int* __restrict__ counts, int cap,
                                                     const int* __restrict__ pa, const int* __restrict__ pb,
                                                     int rows, int cols, int window, float nnratio, int check_ori,
                                                     uint32_t* __restrict__ cand, int cand_per_pair,
                                                     int* __restrict__ m12_out, int* __restrict__ nm_out)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    int p2 = 1;
    while (p2 < cap) p2 <<= 1;
    uint32_t* keys = (uint32_t*)smem;                 // [p2]
    uint32_t* off = keys + p2;                        // [cap + 1]
    int* mdist = (int*)(off + cap + 1);               // [cap]
    int* m21 = mdist + cap;                           // [cap]
    int* m12 = m21 + cap;                             // [cap]
    int* bin = m12 + cap;                             // [cap]
    __shared__ int s_n[4];
    __shared__ int s_hist[32];
    __shared__ uint32_t s_wsum[5];

    const int pair = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int fa = pa[pair], fb = pb[pair];
    const orbx_keypoint* k1 = kps + (size_t)fa * cap;
    const orbx_keypoint* k2 = kps + (size_t)fb * cap;
    const uint8_t* d1 = desc + (size_t)fa * cap * 32;
    const uint8_t* d2 = desc + (size_t)fb * cap * 32;
    const int n1 = min(counts[fa], cap), n2 = min(counts[fb], cap);
    if (tid == 0) { s_n[0] = 0; s_n[1] = 0; }
    __syncthreads();
    // level-0 keypoints come first (src/ORBextractor.cc:1290-1333)
    int c1 = 0, c2 = 0;
    for (int i = tid; i < n1; i += 256) c1 += k1[i].octave == 0;
    for (int i = tid; i < n2; i += 256) c2 += k2[i].octave == 0;
    atomicAdd(&s_n[0], c1);
    atomicAdd(&s_n[1], c2);
    __syncthreads();
    const int n10 = s_n[0], n20 = s_n[1];

    const float invW = (float)kGridCols / ((float)cols - 0.0f);
    const float invH = (float)kGridRows / ((float)rows - 0.0f);
    for (int i = tid; i < p2; i += 256) {
        uint32_t key = 0xFFFFFFFFu;
        if (i < n20) {
            const int px = (int)roundf((k2[i].x - 0.0f) * invW);
            const int py = (int)roundf((k2[i].y - 0.0f) * invH);
            if (px >= 0 && px < kGridCols && py >= 0 && py < kGridRows)
                key = ((uint32_t)(px * kGridRows + py) << 16) | (uint32_t)i;
        }
        keys[i] = key;
    }
    __syncthreads();
    bitonic_asc(keys, p2);
    int ng = 0;
    for (int i = 0; i < n20; ++i) ng += keys[i] != 0xFFFFFFFFu;   // uniform, cheap (n20 small)

    const float r = (float)window;
    uint32_t* pc = cand + (size_t)pair * cand_per_pair;
    // pass A1/A2: count then write candidate lists (one wave per query)
    for (int pass = 0; pass < 2; ++pass) {
        for (int i1 = wave; i1 < n10; i1 += 4) {
            const float x = k1[i1].x, y = k1[i1].y;
            const Window W = window_cells(x, y, r, invW, invH);
            int base = pass ? (int)off[i1] : 0;
            const int limit = pass ? (int)off[i1 + 1] : 0;
            const ulonglong2* a = (const ulonglong2*)(d1 + (size_t)i1 * 32);
            const ulonglong2 a0 = a[0], a1 = a[1];
            for (int g0 = 0; g0 < ng; g0 += 64) {
                const int g = g0 + lane;
                bool in = false;
                int i2 = 0;
                if (!W.empty && g < ng) {
                    const uint32_t key = keys[g];
                    const int cell = (int)(key >> 16);
                    const int ix = cell / kGridRows, iy = cell - ix * kGridRows;
                    i2 = (int)(key & 0xFFFF);
                    if (ix >= W.cx0 && ix <= W.cx1 && iy >= W.cy0 && iy <= W.cy1) {
                        const float dx = k2[i2].x - x, dy = k2[i2].y - y;
                        in = fabsf(dx) < r && fabsf(dy) < r;
                    }
                }
                const unsigned long long m = __ballot(in);
                if (pass && in) {
                    const ulonglong2* b = (const ulonglong2*)(d2 + (size_t)i2 * 32);
                    const int d = ham256(a0, a1, b[0], b[1]);
                    const int idx = base + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                    __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                    if (idx < limit) pc[idx] = (uint32_t)i2 | ((uint32_t)d << 16);
                }
                base += __popcll(m);
            }
            if (!pass && lane == 0) off[i1] = (uint32_t)base;
        }
        __syncthreads();
        if (!pass) {
            // exclusive scan of off[0..n10) (single wave; n10 is a few hundred)
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
                    s_n[2] = (int)run > cand_per_pair ? 1 : 0;
                }
            }
            __syncthreads();
            if (s_n[2]) {   // scratch too small: clamp lists (reported through nmatches = -1)
                for (int i = tid; i <= n10; i += 256) off[i] = min(off[i], (uint32_t)cand_per_pair);
                __syncthreads();
            }
        }
    }
    (void)s_wsum;

    if (wave != 0) return;
    // pass B: the reference's sequential greedy loop
    for (int i = lane; i < n2; i += 64) {
        mdist[i] = INT_MAX;
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
            if (mdist[i2] <= d) continue;
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
                m12[i1] = bi;
                m21[bi] = i1;
                mdist[bi] = b1;
                ++nmatches;
                if (check_ori) {
                    float rot = k1[i1].angle - k2[bi].angle;
                    if (rot < 0.0f) rot += 360.0f;
                    int bb = (int)roundf(rot * factor);
                    if (bb == 30) bb = 0;
                    bin[i1] = bb;
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
    for (int i = lane; i < cap; i += 64) out[i] = i < n1 ? m12[i] : -1;
    if (lane == 0) nm_out[pair] = s_n[2] ? -1 : nmatches;
}

void launch_search_init(const orbx_keypoint* kps, const uint8_t* desc, const int* counts, int cap, const int* pa,
                        const int* pb, int npairs, int rows, int cols, int window, float nnratio, int check_ori,
                        uint32_t* cand, int cand_per_pair, int* m12, int* nm, hipStream_t s)
{
    int p2 = 1;
    while (p2 < cap) p2 <<= 1;
    const size_t smem = sizeof(uint32_t) * (p2 + cap + 1) + sizeof(int) * 4 * cap;
    hipLaunchKernelGGL(k_search_init, dim3(npairs), dim3(256), smem, s, kps, desc, counts, cap, pa, pb, rows, cols,
                       window, nnratio, check_ori, cand, cand_per_pair, m12, nm);
}

}  // namespace orbx
