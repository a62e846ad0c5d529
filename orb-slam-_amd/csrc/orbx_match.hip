// gfx950 kernels of the ORBmatcher Hamming searches (include/ORBmatcher.h:37-102).
//
//   M3 k_allpairs_top2 / k_allpairs_full   brute-force 256-bit Hamming (config 5)
//   M1 k_search_init                        SearchForInitialization, src/ORBmatcher.cc:417-588
//
// Distance = popcount(a ^ b) over four little-endian u64 words, identical to
// the reference's 8 x u32 SWAR DescriptorDistance (src/ORBmatcher.cc:1728-1744).
#include <hip/hip_runtime.h>
#include <limits.h>

#include <algorithm>

#include <type_traits>
#include <cstdlib>

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

// ---------------------------------------------------------------------------
// orbm_best2_csr: one lane per query walks its candidate list in order (the reference's
// sequential loop); lists are a few to a few hundred entries.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_best2_csr(const uint4* __restrict__ q, int nq, const uint4* __restrict__ t,
                                                   const int* __restrict__ ptr, const int* __restrict__ idx,
                                                   int tie_last, int* __restrict__ bi, int* __restrict__ b1,
                                                   int* __restrict__ b2)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= nq) return;
    const uint4 q0 = q[2 * i], q1 = q[2 * i + 1];
    int best = 256, second = 256, bidx = -1;
    const int e = ptr[i + 1];
    for (int c = ptr[i]; c < e; ++c) {
        const int j = idx[c];
        const uint4 t0 = t[2 * j], t1 = t[2 * j + 1];
        const int d = __popc(q0.x ^ t0.x) + __popc(q0.y ^ t0.y) + __popc(q0.z ^ t0.z) + __popc(q0.w ^ t0.w) +
                      __popc(q1.x ^ t1.x) + __popc(q1.y ^ t1.y) + __popc(q1.z ^ t1.z) + __popc(q1.w ^ t1.w);
        if (d < best) {
            second = best;
            best = d;
            bidx = j;
        } else {
            if (tie_last && d == best) bidx = j;   // the candidate replaces the best, the second is unchanged
            if (d < second) second = d;
        }
    }
    bi[i] = bidx;
    b1[i] = best;
    b2[i] = second;
}

void launch_best2_csr(const uint8_t* q, int nq, const uint8_t* t, const int* ptr, const int* idx, int tie_last,
                      int* bi, int* b1, int* b2, hipStream_t s)
{
    hipLaunchKernelGGL(k_best2_csr, dim3((nq + 255) / 256), dim3(256), 0, s, (const uint4*)q, nq, (const uint4*)t, ptr,
                       idx, tie_last, bi, b1, b2);
}

void launch_allpairs_full(const uint8_t* q, int nq, const uint8_t* t, int nt, uint16_t* out, hipStream_t s)
{
    dim3 grid((nt + 1023) / 1024, (nq + 63) / 64);
    hipLaunchKernelGGL(k_allpairs_full, grid, dim3(256), 0, s, (const ulonglong2*)q, nq, (const ulonglong2*)t, nt,
                       out);
}

// ---------------------------------------------------------------------------
// M1: SearchForInitialization (src/ORBmatcher.cc:417-588) for a batch of
// frame pairs, in three launches:
//   k_si_grid   one workgroup per frame: its level-0 keypoints ranked the way
//               Frame::GetFeaturesInArea visits them — grid cell (ix outer,
//               iy inner, Frame::PosInGrid rounding), then index
//               (AssignFeaturesToGrid insertion order), src/Frame.cc:292-518.
//   k_si_build  (pair, query-slice) workgroups, four lanes per query: the
//               window's columns are one contiguous key range (a column-start
//               table in LDS), filtered by row and |dx|,|dy| < r.  The quad keeps
//               the 4 smallest (Hamming, visit position) candidates and the count.
//   k_si_greedy one workgroup per pair: one wave replays the order-dependent
//               greedy pass (vMatchedDistance skip, best/second, ratio test,
//               eviction) and the rotation-histogram filter
//               (ComputeThreeMaxima, :1679-1723).  best/second are the first
//               two candidates in (Hamming, position) order that the skip
//               does not drop, so a step needs only the query's top-4; a
//               candidate outside it has Hamming >= the 4th, which settles
//               the step unless the best is within the ratio of it — then the
//               wave re-enumerates the window (k_si_build's walk) and scans.
// ---------------------------------------------------------------------------
constexpr int kGridCols = 64, kGridRows = 48;
constexpr int SI_BUILD_NT = 256;
constexpr int SI_TOPK = 4;
constexpr int kSiCells = kGridCols * kGridRows;
constexpr int kSiRankMax = 4096;   // k_si_grid: rank sort up to this many level-0 keypoints, counting sort above

__host__ __device__ inline size_t si_grid_smem(int cap)
{
    return (size_t)((cap + 3) & ~3) * 4 + (cap > kSiRankMax ? (size_t)(kSiCells + 4) * 4 : 0);
}

// min over the 64 lanes with DPP row permutations + 4 readlanes (all lanes active)
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v)
{
    v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true));    // quad_perm [1,0,3,2]
    v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, true));    // quad_perm [2,3,0,1]
    v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, true));   // row_half_mirror
    v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, true));   // row_mirror
    const uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)v, 0);
    const uint32_t b = (uint32_t)__builtin_amdgcn_readlane((int)v, 16);
    const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)v, 32);
    const uint32_t d = (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
    return min(min(a, b), min(c, d));
}

// orders this wave's LDS accesses (a wave-level barrier for data exchanged through LDS)
__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int lanes_below_u64(unsigned long long m)
{
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
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

__global__ __launch_bounds__(256) void k_si_grid(const orbx_keypoint* __restrict__ kps, const int* __restrict__ counts,
                                                 int cap, orbm_grid G, uint32_t* __restrict__ gkeys,
                                                 float2* __restrict__ gxy, int* __restrict__ gn)
{
    // Keys (cell << 16 | index) are unique, so a key's place in the sorted order is the number of smaller
    // keys: every thread ranks its keys against the whole array by broadcast 16-byte LDS reads, one
    // barrier, and scatters (round 2: a bitonic network, log2(n)^2 / 2 barrier-separated stages).
    extern __shared__ __attribute__((aligned(16))) uint32_t keys[];
    __shared__ int s_ng, s_n0;
    const int f = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
    const orbx_keypoint* k = kps + (size_t)f * cap;
    const int n = min(counts[f], cap);
    if (tid == 0) s_ng = s_n0 = 0;
    __syncthreads();
    // one pass over the keypoints: the level-0 count is the number of octave-0 keypoints (they come first,
    // src/ORBextractor.cc:1290-1333), the grid count the number of valid keys; both by wave ballots, one
    // LDS atomic per wave (per-key atomics on one word, or a binary search of dependent global loads,
    // serialised)
    for (int i = tid; i < ((n + 3) & ~3); i += 256) {
        uint32_t key = 0xFFFFFFFFu;   // another octave, outside the grid, or padding: above every key
        bool l0 = false;
        if (i < n && k[i].octave == 0) {
            l0 = true;
            const int px = (int)roundf((k[i].x - G.min_x) * G.grid_w_inv);
            const int py = (int)roundf((k[i].y - G.min_y) * G.grid_h_inv);
            if (px >= 0 && px < kGridCols && py >= 0 && py < kGridRows)   // PosInGrid
                key = ((uint32_t)(px * kGridRows + py) << 16) | (uint32_t)i;
        }
        keys[i] = key;
        const unsigned long long b0 = __ballot(l0), bg = __ballot(key != 0xFFFFFFFFu);
        if (lane == 0) {
            atomicAdd(&s_n0, __popcll(b0));
            atomicAdd(&s_ng, __popcll(bg));
        }
    }
    __syncthreads();
    const int n0 = s_n0;
    if (n0 > kSiRankMax) {
        // large frames: a stable counting sort over the 3072 cells, O(n) instead of the rank's O(n^2)
        // LDS reads.  Per-cell counts by LDS atomics (arrival slots unordered), an exclusive scan, a
        // scatter of the indices into their cell segments, then each key's stable place = the number
        // of lower indices in its own segment (a few entries).  gxy holds the scratch words until the
        // last step: even word i = key i's arrival slot, then its sorted position; odd word p = the
        // index scattered to position p.
        uint32_t* start = keys + ((cap + 3) & ~3);   // [kSiCells + 1]
        uint32_t* tmp = (uint32_t*)(gxy + (size_t)f * cap);
        for (int c = tid; c <= kSiCells; c += 256) start[c] = 0u;
        __syncthreads();
        for (int i = tid; i < n0; i += 256) {
            const uint32_t key = keys[i];
            if (key != 0xFFFFFFFFu) tmp[2 * i] = atomicAdd(&start[key >> 16], 1u);
        }
        __syncthreads();
        if (tid < 64) {   // exclusive scan of the 3072 counts by one wave, 48 per lane
            constexpr int kPer = kSiCells / 64;
            uint32_t sum = 0;
            for (int j = 0; j < kPer; ++j) sum += start[lane * kPer + j];
            uint32_t incl = sum;
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(incl, o);
                if (lane >= o) incl += y;
            }
            uint32_t base = incl - sum;
            for (int j = 0; j < kPer; ++j) {
                const uint32_t c = start[lane * kPer + j];
                start[lane * kPer + j] = base;
                base += c;
            }
            if (lane == 63) start[kSiCells] = base;
        }
        __syncthreads();
        for (int i = tid; i < n0; i += 256) {
            const uint32_t key = keys[i];
            if (key != 0xFFFFFFFFu) tmp[2 * (start[key >> 16] + tmp[2 * i]) + 1] = (uint32_t)i;
        }
        __syncthreads();
        for (int i = tid; i < n0; i += 256) {
            const uint32_t key = keys[i];
            if (key == 0xFFFFFFFFu) continue;
            const int s0 = (int)start[key >> 16], s1 = (int)start[(key >> 16) + 1];
            int r = 0;
            for (int j = s0; j < s1; ++j) r += tmp[2 * j + 1] < (uint32_t)i;
            gkeys[(size_t)f * cap + s0 + r] = key;
            keys[i] = (uint32_t)(s0 + r);   // read only by this thread below
        }
        __syncthreads();
        for (int i = tid; i < n0; i += 256) {
            const uint32_t pos = keys[i];
            if (pos < (uint32_t)cap) gxy[(size_t)f * cap + pos] = make_float2(k[i].x, k[i].y);
        }
    } else {
        const int n4 = (n0 + 3) >> 2;
        const uint4* k4 = (const uint4*)keys;
        for (int i = tid; i < n0; i += 256) {
            const uint32_t key = keys[i];
            if (key == 0xFFFFFFFFu) continue;
            int r = 0;
            for (int j4 = 0; j4 < n4; ++j4) {
                const uint4 v = k4[j4];
                r += (int)(v.x < key) + (int)(v.y < key) + (int)(v.z < key) + (int)(v.w < key);
            }
            gkeys[(size_t)f * cap + r] = key;
            gxy[(size_t)f * cap + r] = make_float2(k[i].x, k[i].y);
        }
    }
    if (tid == 0) {
        gn[2 * f] = n0;
        gn[2 * f + 1] = s_ng;
    }
}

// query window of GetFeaturesInArea(x, y, r, 0, 0) (src/Frame.cc:410-440) over the sorted
// grid keys: the cells' columns are one key range [lo, hi), rows are filtered per key
struct SiWindow {
    int lo, hi, cy0, cy1;
    float x, y, r;
};

// first key of every grid column (keys are sorted by column-major cell): colstart[c] for c = 0..64
__device__ __forceinline__ void si_colstart(const uint32_t* keys, int ng, int* colstart, int tid, int nt)
{
    for (int g = tid; g <= ng; g += nt) {
        const int cp = g > 0 ? (int)(keys[g - 1] >> 16) / kGridRows : -1;
        const int cc = g < ng ? (int)(keys[g] >> 16) / kGridRows : kGridCols;
        for (int c = cp + 1; c <= cc; ++c) colstart[c] = g;
    }
}

__device__ __forceinline__ SiWindow si_window(const uint32_t* keys, int ng, float2 c, float r, const orbm_grid& G,
                                              const int* colstart = nullptr)
{
    SiWindow w;
    const float x = c.x, y = c.y;
    w.x = x;
    w.y = y;
    w.r = r;
    const int cx0 = max(0, (int)floorf((x - G.min_x - r) * G.grid_w_inv));
    const int cx1 = min(kGridCols - 1, (int)ceilf((x - G.min_x + r) * G.grid_w_inv));
    w.cy0 = max(0, (int)floorf((y - G.min_y - r) * G.grid_h_inv));
    w.cy1 = min(kGridRows - 1, (int)ceilf((y - G.min_y + r) * G.grid_h_inv));
    w.lo = w.hi = 0;
    if (cx0 < kGridCols && cx1 >= 0 && w.cy0 < kGridRows && w.cy1 >= 0) {
        if (colstart) {   // two independent table reads instead of two binary searches
            w.lo = colstart[cx0];
            w.hi = colstart[cx1 + 1];
        } else {
            w.lo = lower_bound_u32(keys, ng, (uint32_t)(cx0 * kGridRows) << 16);
            w.hi = lower_bound_u32(keys, ng, (uint32_t)((cx1 + 1) * kGridRows) << 16);
        }
    }
    return w;
}

__device__ __forceinline__ bool si_in_window(const uint32_t* keys, const float2* xy, const SiWindow& w, int g,
                                             int& i2)
{
    if (g >= w.hi) return false;
    const uint32_t key = keys[g];
    const int iy = (int)(key >> 16) % kGridRows;
    if (iy < w.cy0 || iy > w.cy1) return false;
    const float2 p = xy[g];
    i2 = (int)(key & 0xFFFF);
    return fabsf(p.x - w.x) < w.r && fabsf(p.y - w.y) < w.r;
}

// F2 level-0 keypoints whose grid keys, positions and descriptors k_si_build stages in LDS (22 KB per
// workgroup); a pair with more reads them from global memory instead
constexpr int kSiBuildLds = 512;

__host__ __device__ inline size_t si_build_xy_off() { return ((size_t)kSiBuildLds * 4 + 15) & ~(size_t)15; }
__host__ __device__ inline size_t si_build_desc_off() { return si_build_xy_off() + (size_t)kSiBuildLds * 8; }
size_t si_build_smem_bytes() { return si_build_desc_off() + (size_t)kSiBuildLds * 32; }

__global__ __launch_bounds__(SI_BUILD_NT) void k_si_build(const orbx_keypoint* __restrict__ kps,
                                                          const uint8_t* __restrict__ desc, int cap,
                                                          const int* __restrict__ pa, const int* __restrict__ pb,
                                                          orbm_grid G, int window, const float2* __restrict__ prev,
                                                          const uint32_t* __restrict__ gkeys,
                                                          const float2* __restrict__ gxy, const int* __restrict__ gn,
                                                          int* __restrict__ qcnt, uint4* __restrict__ qtop)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int pair = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave: uniform
    const int fa = pa[pair], fb = pb[pair];
    const int n10 = gn[2 * fa], ng = gn[2 * fb + 1];
    const uint8_t* d2 = desc + (size_t)fb * cap * 32;
    __shared__ int colstart[kGridCols + 1];
    // the window scans read F2's grid keys, positions and descriptors once per candidate per query: in LDS
    // when they fit (one L2 round trip per candidate otherwise dominated the kernel)
    const bool staged = ng <= kSiBuildLds;   // block-uniform
    uint32_t* skeys = (uint32_t*)smem;
    float2* sxy = (float2*)(smem + si_build_xy_off());
    ulonglong2* sdesc = (ulonglong2*)(smem + si_build_desc_off());
    if (staged) {
        for (int g = tid; g < ng; g += SI_BUILD_NT) {
            const uint32_t key = gkeys[(size_t)fb * cap + g];
            skeys[g] = key;
            sxy[g] = gxy[(size_t)fb * cap + g];
            const ulonglong2* b = (const ulonglong2*)(d2 + (size_t)(key & 0xFFFF) * 32);
            sdesc[2 * g] = b[0];
            sdesc[2 * g + 1] = b[1];
        }
        __syncthreads();
    }
    // global and LDS sources kept apart (a pointer that may be either compiles to flat loads, which wait on both
    // counters)
    const uint32_t* keys = gkeys + (size_t)fb * cap;
    const float2* xy = gxy + (size_t)fb * cap;
    if (staged) si_colstart((const uint32_t*)skeys, ng, colstart, tid, SI_BUILD_NT);
    else si_colstart(keys, ng, colstart, tid, SI_BUILD_NT);
    __syncthreads();
    const orbx_keypoint* k1 = kps + (size_t)fa * cap;
    const uint8_t* d1 = desc + (size_t)fa * cap * 32;
    const float2* pv = prev ? prev + (size_t)pair * cap : nullptr;
    const int nwaves = gridDim.y * (SI_BUILD_NT / 64);
    // Four lanes per query (a quad), 16 queries per wave: the quad's lanes take the window's key range
    // round-robin, each keeping its 4 smallest (Hamming << 16 | visit position), and two quad-DPP steps per
    // output merge them.  A candidate's visit position is the quad's in-window count before it in key
    // order (the quad's ballot bits).  (Round 2: a wave per query, whose 64-lane merge of the top-4 was
    // most of the kernel's instructions for ~74 keys per window.)
    auto quad_min = [](uint32_t v) {
        v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true));   // quad_perm [1,0,3,2]
        return min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, true));  // quad_perm [2,3,0,1]
    };
    auto quad_or = [](uint32_t v) {
        v |= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true);
        return v | (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, true);
    };
    const int sub = lane & 3, qbase = lane & ~3;
    auto scan_queries = [&](auto staged_tag) {
        constexpr bool kStaged = decltype(staged_tag)::value;
        const uint32_t* K = kStaged ? (const uint32_t*)skeys : keys;
        const float2* XY = kStaged ? (const float2*)sxy : xy;
        const int wg = blockIdx.y * (SI_BUILD_NT / 64) + wave;
        for (int r0 = wg * 16; r0 < n10; r0 += nwaves * 16) {   // wave-uniform
            const int q = r0 + (lane >> 2);
            SiWindow w;
            ulonglong2 a0 = make_ulonglong2(0, 0), a1 = make_ulonglong2(0, 0);
            w.lo = w.hi = 0;
            if (q < n10) {
                const ulonglong2* a = (const ulonglong2*)(d1 + (size_t)q * 32);
                a0 = a[0];
                a1 = a[1];
                // window centre vbPrevMatched[q] (src/ORBmatcher.cc:456-460); F1's own keypoint when not given
                const float2 c = pv ? pv[q] : make_float2(k1[q].x, k1[q].y);
                w = si_window(K, ng, c, (float)window, G, colstart);
            }
            uint32_t hk[SI_TOPK], hi2[SI_TOPK];
#pragma unroll
            for (int t = 0; t < SI_TOPK; ++t) hk[t] = hi2[t] = 0xFFFFFFFFu;
            int count = 0;
            for (int g0 = w.lo; g0 < w.hi; g0 += 4) {   // quad-uniform trip count
                int i2 = 0;
                const int g = g0 + sub;
                const bool in = si_in_window(K, XY, w, g, i2);
                const uint32_t qb = (uint32_t)(__ballot(in) >> qbase) & 0xFu;
                if (in) {
                    int d;
                    if constexpr (kStaged) {
                        d = ham256(a0, a1, sdesc[2 * g], sdesc[2 * g + 1]);
                    } else {
                        const ulonglong2* b = (const ulonglong2*)(d2 + (size_t)i2 * 32);
                        d = ham256(a0, a1, b[0], b[1]);
                    }
                    const int pos = count + __builtin_popcount(qb & ((1u << sub) - 1u));
                    uint32_t k = ((uint32_t)d << 16) | (uint32_t)pos, v = (uint32_t)i2;
#pragma unroll
                    for (int t = 0; t < SI_TOPK; ++t) {   // sorted insert
                        if (k < hk[t]) {
                            const uint32_t tk = hk[t], tv = hi2[t];
                            hk[t] = k;
                            hi2[t] = v;
                            k = tk;
                            v = tv;
                        }
                    }
                }
                count += __builtin_popcount(qb);
            }
            // quad merge: keys are unique (visit positions), so one lane pops per round
            uint32_t top[SI_TOPK];
#pragma unroll
            for (int t = 0; t < SI_TOPK; ++t) {
                const uint32_t kmin = quad_min(hk[0]);
                const bool own = kmin != 0xFFFFFFFFu && hk[0] == kmin;
                const uint32_t i2 = quad_or(own ? hi2[0] : 0u);
                top[t] = kmin == 0xFFFFFFFFu ? 0xFFFFFFFFu : ((kmin & 0xFFFF0000u) | i2);
                if (own) {
#pragma unroll
                    for (int u = 0; u + 1 < SI_TOPK; ++u) {
                        hk[u] = hk[u + 1];
                        hi2[u] = hi2[u + 1];
                    }
                    hk[SI_TOPK - 1] = hi2[SI_TOPK - 1] = 0xFFFFFFFFu;
                }
            }
            if (sub == 0 && q < n10) {
                const size_t at = (size_t)pair * cap + q;
                qtop[at] = make_uint4(top[0], top[1], top[2], top[3]);
                qcnt[at] = count;
            }
        }
    };
    if (staged)
        scan_queries(std::true_type{});
    else
        scan_queries(std::false_type{});
}

// level-0 keypoints per frame the SearchForInitialization greedy pass keeps in LDS in its common launch:
// 1792 keeps the workgroup under 80 KB (two per CU; the extractor's levels hold at most ~1,700)
constexpr int kSiLdsCap = 1792;
constexpr int kSiGreedySmall = 512;   // the common tier: KITTI / EuRoC / TUM frames keep <= ~440 level-0 keypoints

struct SgLayout {
    size_t top, cnt, ang1, ang2, mdist, m21, m12, bin, wmax, wmin, total;
};

__host__ __device__ inline SgLayout sg_layout(int cap)
{
    SgLayout L;
    size_t o = 0;
    auto take = [&](size_t b) {
        const size_t r = o;
        o += (b + 15) & ~(size_t)15;
        return r;
    };
    L.top = take(16 * ((size_t)cap + 2));   // padded with 2 empty entries past n10
    L.cnt = take(4 * ((size_t)cap + 2));
    L.ang1 = take(4 * (size_t)cap);
    L.ang2 = take(4 * (size_t)cap);
    L.mdist = take(2 * (size_t)cap);
    L.m21 = take(2 * (size_t)cap);
    L.m12 = take(2 * (size_t)cap);
    L.bin = take((size_t)cap);
    L.wmax = take(4 * (size_t)cap);
    L.wmin = take(4 * (size_t)cap);
    L.total = o;
    return L;
}

// kG: the per-pair arrays live in a global region (gbuf, sg_stride bytes per pair) instead of LDS, for frames
// with more level-0 keypoints than a workgroup's LDS holds (about 3,800; e.g. Tracking's 2 * nFeatures
// initialisation extractor at 1080p and beyond).  Same algorithm; the histogram stays in LDS.
template <bool kG>
__global__ __launch_bounds__(256) void k_si_greedy(const orbx_keypoint* __restrict__ kps,
                                                   const uint8_t* __restrict__ desc, const int* __restrict__ counts,
                                                   int cap, const int* __restrict__ pa, const int* __restrict__ pb,
                                                   orbm_grid G, int window, float nnratio, int check_ori,
                                                   float2* __restrict__ prev,
                                                   const uint32_t* __restrict__ gkeys,
                                                   const float2* __restrict__ gxy, const int* __restrict__ gn,
                                                   const int* __restrict__ qcnt, const uint4* __restrict__ qtop,
                                                   int* __restrict__ m12_out, int* __restrict__ nm_out, int lcap,
                                                   int tier_lo, uint8_t* __restrict__ gbuf, size_t sg_stride)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_lds[];
#ifdef ORBX_SI_PROF
    const long long pt0 = clock64();
#endif
    // The LDS arrays hold level-0 keypoints only (queries of F1, candidates of F2), sized lcap.  Pairs are
    // tiered by their larger level-0 count: this launch takes the pairs in (tier_lo, lcap], launches sized
    // for the larger tiers take the rest (launch_search_init), so the common launch's workgroups stay small
    // (22 KB for up to 512 level-0 keypoints) and find room beside the extractor's under the pipeline.
    {
        const int n0 = max(gn[2 * pa[blockIdx.x]], gn[2 * pb[blockIdx.x]]);
        if (n0 <= tier_lo || n0 > lcap) return;
    }
    const SgLayout Ly = sg_layout(lcap);
    uint8_t* smem = smem_lds;
    if constexpr (kG) smem = gbuf + (size_t)blockIdx.x * sg_stride;
    uint4* top = (uint4*)(smem + Ly.top);
    int* cnt = (int*)(smem + Ly.cnt);
    float* ang1 = (float*)(smem + Ly.ang1);
    float* ang2 = (float*)(smem + Ly.ang2);
    uint16_t* mdist = (uint16_t*)(smem + Ly.mdist);
    int16_t* m21 = (int16_t*)(smem + Ly.m21);
    int16_t* m12 = (int16_t*)(smem + Ly.m12);
    int8_t* bin = (int8_t*)(smem + Ly.bin);
    uint32_t* wmax = (uint32_t*)(smem + Ly.wmax);
    uint32_t* wmin = (uint32_t*)(smem + Ly.wmin);
    __shared__ int s_hist[32];
    const int pair = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
    const int fa = pa[pair], fb = pb[pair];
    const int n10 = gn[2 * fa], ng = gn[2 * fb + 1], n20 = gn[2 * fb];   // level-0 counts
    int* out = m12_out + (size_t)pair * cap;
    const orbx_keypoint* k1 = kps + (size_t)fa * cap;
    const orbx_keypoint* k2 = kps + (size_t)fb * cap;
    for (int i = tid; i < n10; i += 256) {
        cnt[i] = qcnt[(size_t)pair * cap + i];
        top[i] = qtop[(size_t)pair * cap + i];
        ang1[i] = k1[i].angle;
    }
    if (tid < 2) {
        cnt[n10 + tid] = 0;
        top[n10 + tid] = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
    }
    for (int i = tid; i < n20; i += 256) {   // candidates are F2's level-0 keypoints
        mdist[i] = 0xFFFF;   // INT_MAX: larger than any distance
        m21[i] = -1;
        wmax[i] = wmin[i] = 0;
        ang2[i] = k2[i].angle;
    }
    for (int i = tid; i < n10; i += 256) {
        m12[i] = -1;
        bin[i] = -1;
    }
    if (tid < 32) s_hist[tid] = 0;
    __syncthreads();
    if (tid >= 64) {
        // vnMatches12 past the level-0 queries is -1: written by the idle waves while wave 0 runs the
        // greedy pass (one wave writing all cap entries at the end was a third of the kernel's time)
        for (int i = n10 + tid - 64; i < cap; i += 192) out[i] = -1;
        return;
    }
#ifdef ORBX_SI_PROF
    const long long pt1 = clock64();
#endif

    // Greedy pass, 64 steps at a time (lane = step).  m12 holds each query's tentative
    // match (kept even if a later query evicts it: the reference's rotHist keeps evicted
    // entries too, :506-536); the final vnMatches12 is m12[i1] where m21 still points back.
    //
    // A step's outcome is a function of mdist over its top-4 targets, which earlier steps
    // change only by their own matches.  Each lane decides from the mdist of the chunk's
    // start patched with the previous round's decisions of the lanes before it; a round
    // publishes every lane's match (target, lane, distance) in LDS tables stamped with the
    // round, so a lane finds the last earlier writer of each of its targets with two reads.
    // The rounds reach the fixed point where every lane's decision follows from the ones
    // before it, which is the sequential result.  A step that needs a full scan ends the
    // chunk's exact prefix: it is replayed on its own with the wave.
    const int n2c = max(n20 - 1, 0);
    float2* pv = prev ? prev + (size_t)pair * cap : nullptr;
    auto decide = [&](const uint32_t (&e)[SI_TOPK], const uint32_t (&md)[SI_TOPK], int c, int& bi, int& bd,
                      bool& scan) -> bool {
        bool ok[SI_TOPK];
        int d[SI_TOPK];
#pragma unroll
        for (int q = 0; q < SI_TOPK; ++q) {
            d[q] = (int)(e[q] >> 16);
            ok[q] = e[q] != 0xFFFFFFFFu && md[q] > (uint32_t)d[q];   // vMatchedDistance[i2] <= dist: skip
        }
        const int nf = (int)ok[0] + (int)ok[1] + (int)ok[2] + (int)ok[3];
        // best = first survivor, second = the next one (entries are in (dist, position) order)
        int bd2 = INT_MAX;
        bd = INT_MAX;
        bi = -1;
        if (ok[0]) {
            bd = d[0];
            bi = (int)(e[0] & 0xFFFF);
            bd2 = ok[1] ? d[1] : ok[2] ? d[2] : ok[3] ? d[3] : INT_MAX;
        } else if (ok[1]) {
            bd = d[1];
            bi = (int)(e[1] & 0xFFFF);
            bd2 = ok[2] ? d[2] : ok[3] ? d[3] : INT_MAX;
        } else if (ok[2]) {
            bd = d[2];
            bi = (int)(e[2] & 0xFFFF);
            bd2 = ok[3] ? d[3] : INT_MAX;
        } else if (ok[3]) {
            bd = d[3];
            bi = (int)(e[3] & 0xFFFF);
        }
        // Candidates past the top-4 have Hamming >= d[3], so when fewer than two of the
        // top-4 survive, d[3] usually settles the step without the rest:
        //   none survive  -> best >= d[3]: no match if d[3] > TH_LOW;
        //   one survives  -> second >= d[3]: the ratio test holds if best < d[3] * r.
        scan = false;
        if (c > SI_TOPK && nf < 2) {
            if (nf == 0)
                scan = d[3] <= 50;
            else if (bd <= 50 && (float)bd < (float)d[3] * nnratio)
                bd2 = d[3];   // stands in for the exact second: both pass the test
            else
                scan = bd <= 50;
        }
        return !scan && bd <= 50 && (float)bd < (float)bd2 * nnratio;   // TH_LOW, mfNNratio
    };
#ifdef ORBX_SI_PROF
    int prof_chunks = 0, prof_scans = 0;   // exact-prefix chunks and full-window scans of the greedy pass
#endif
    uint32_t stamp = 0;   // round stamp of the writer tables (tables start at 0)
    int base = 0;
    while (base < n10) {
        const int i1 = base + lane;
        const bool act = i1 < n10;
        const int ii = min(i1, n10);   // top[n10] is an empty entry
        const uint4 tv = top[ii];
        const int c = act ? cnt[ii] : 0;
        const uint32_t e[SI_TOPK] = {tv.x, tv.y, tv.z, tv.w};
        uint32_t md0[SI_TOPK], md[SI_TOPK];
#pragma unroll
        for (int q = 0; q < SI_TOPK; ++q) {
            const uint32_t v = mdist[min((int)(e[q] & 0xFFFF), n2c)];
            md0[q] = md[q] = e[q] == 0xFFFFFFFFu ? 0u : v;
        }
        int bi, bd;
        bool scan;
        bool mt = decide(e, md, c, bi, bd, scan);
        for (;;) {
            ++stamp;
            if (mt) {
                atomicMax(&wmax[bi], (stamp << 12) | ((uint32_t)lane << 6) | (uint32_t)bd);
                atomicMax(&wmin[bi], (stamp << 12) | ((uint32_t)(63 - lane) << 6) | (uint32_t)bd);
            }
            wave_lds_sync();
            bool amb = false;
#pragma unroll
            for (int q = 0; q < SI_TOPK; ++q) {
                const int i2 = min((int)(e[q] & 0xFFFF), n2c);
                const uint32_t a = wmax[i2], b = wmin[i2];
                md[q] = md0[q];
                if (e[q] != 0xFFFFFFFFu && (a >> 12) == stamp) {
                    const int hi = (int)((a >> 6) & 63), lo = 63 - (int)((b >> 6) & 63);
                    if (hi < lane)
                        md[q] = a & 63;   // the last writer before this lane
                    else if (lo < lane)
                        amb = true;       // writers on both sides: resolved below
                }
            }
            if (__ballot(amb)) {
                // exact last-earlier-writer by broadcasting every lane's decision
#pragma unroll
                for (int q = 0; q < SI_TOPK; ++q) md[q] = md0[q];
                for (int j = 0; j < 64; ++j) {
                    if (!__builtin_amdgcn_readlane((int)mt, j)) continue;
                    const int bij = __builtin_amdgcn_readlane(bi, j), bdj = __builtin_amdgcn_readlane(bd, j);
#pragma unroll
                    for (int q = 0; q < SI_TOPK; ++q)
                        if (j < lane && e[q] != 0xFFFFFFFFu && (int)(e[q] & 0xFFFF) == bij) md[q] = (uint32_t)bdj;
                }
            }
            int nbi, nbd;
            bool nscan;
            const bool nmt = decide(e, md, c, nbi, nbd, nscan);
            const bool ch = nmt != mt || nbi != bi || nbd != bd || nscan != scan;
            mt = nmt;
            bi = nbi;
            bd = nbd;
            scan = nscan;
            if (!__ballot(ch)) break;
        }
        // the first step that needs a scan bounds the exact prefix
        const unsigned long long sm = __ballot(act && scan);
        const int lim = sm ? (int)__builtin_ctzll(sm) : min(64, n10 - base);
        // commit: tentative m12 for every match; the last writer of a target owns m21/mdist
        ++stamp;
        const bool cm = mt && lane < lim;
        if (cm) atomicMax(&wmax[bi], (stamp << 12) | ((uint32_t)lane << 6) | (uint32_t)bd);
        wave_lds_sync();
        if (cm) {
            m12[i1] = (int16_t)bi;
            if ((int)((wmax[bi] >> 6) & 63) == lane) {
                m21[bi] = (int16_t)i1;   // evicts the previous owner (:513-517)
                mdist[bi] = (uint16_t)bd;
            }
        }
        wave_lds_sync();
        base += lim;
#ifdef ORBX_SI_PROF
        prof_chunks += 1;
        prof_scans += sm ? 1 : 0;
#endif
        if (sm) {
            // step `base`: re-enumerate its window (global grid of frame fb) and scan it with
            // the current mdist: lane-local best (first min) and second, best = min (dist,
            // position) over lanes, second = min over lanes of (winner ? its b2 : b1)
            const int q1 = base;
            const uint32_t* keys = gkeys + (size_t)fb * cap;
            const float2* xy = gxy + (size_t)fb * cap;
            const ulonglong2* a = (const ulonglong2*)(desc + ((size_t)fa * cap + q1) * 32);
            const ulonglong2 a0 = a[0], a1 = a[1];
            const float2 c = pv ? pv[q1] : make_float2(k1[q1].x, k1[q1].y);
            const SiWindow w = si_window(keys, ng, c, (float)window, G);
            uint32_t b1 = 0x1FF, b2 = 0x1FF, bp = 0xFFFF, bx = 0;
            int count = 0;
            for (int g0 = w.lo; g0 < w.hi; g0 += 64) {
                int i2 = 0;
                const bool in = si_in_window(keys, xy, w, g0 + lane, i2);
                const unsigned long long m = __ballot(in);
                if (in) {
                    const ulonglong2* b = (const ulonglong2*)(desc + ((size_t)fb * cap + i2) * 32);
                    const uint32_t d = (uint32_t)ham256(a0, a1, b[0], b[1]);
                    if ((uint32_t)mdist[i2] > d) {
                        if (d < b1) {
                            b2 = b1;
                            b1 = d;
                            bp = (uint32_t)(count + lanes_below_u64(m));
                            bx = (uint32_t)i2;
                        } else if (d < b2) {
                            b2 = d;
                        }
                    }
                }
                count += __popcll(m);
            }
            const uint32_t key = (b1 << 16) | bp;
            const uint32_t kmin = wave_min_u32(key);
            const uint32_t sec = wave_min_u32(key == kmin ? b2 : b1);
            const unsigned long long wm = __ballot(key == kmin);
            const int wl = wm ? (int)__builtin_ctzll(wm) : 0;
            const int sbd = kmin >> 16 >= 0x1FF ? INT_MAX : (int)(kmin >> 16);
            const int sbd2 = sec >= 0x1FF ? INT_MAX : (int)sec;
            if (sbd <= 50 && (float)sbd < (float)sbd2 * nnratio) {
                const int sbi = __builtin_amdgcn_readlane((int)bx, wl);
                if (lane == 0) {
                    m12[q1] = (int16_t)sbi;
                    m21[sbi] = (int16_t)q1;
                    mdist[sbi] = (uint16_t)sbd;
                }
            }
            wave_lds_sync();
            base += 1;
        }
    }
#ifdef ORBX_SI_PROF
    const long long pt2 = clock64();
#endif
    // rotation bins of every match made (evicted ones included), final vnMatches12
    const float factor = 1.0f / 30;
    for (int i = lane; i < n10; i += 64) {
        const int b = m12[i];
        if (b < 0) continue;
        if (check_ori) {
            float rot = ang1[i] - ang2[b];
            if (rot < 0.0f) rot += 360.0f;
            int bb = (int)roundf(rot * factor);
            if (bb == 30) bb = 0;
            bin[i] = (int8_t)bb;
            atomicAdd(&s_hist[bb], 1);
        }
        if (m21[b] != i) m12[i] = -1;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (check_ori) {   // ComputeThreeMaxima + removal, src/ORBmatcher.cc:562-580
        // the 30 bins in one LDS read (lane = bin), then three wave maxima of (count, 31 - bin): the
        // sequential scan's first-max-wins order is the smallest bin among equal counts
        const int hv = lane < 30 ? s_hist[lane] : 0;
        uint32_t key = lane < 30 && hv > 0 ? ((uint32_t)hv << 5) | (uint32_t)(31 - lane) : 0u;
        int ind[3] = {-1, -1, -1}, mx[3] = {0, 0, 0};
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            uint32_t m = key;
            m = max(m, (uint32_t)__builtin_amdgcn_mov_dpp((int)m, 0xB1, 0xF, 0xF, true));
            m = max(m, (uint32_t)__builtin_amdgcn_mov_dpp((int)m, 0x4E, 0xF, 0xF, true));
            m = max(m, (uint32_t)__builtin_amdgcn_mov_dpp((int)m, 0x141, 0xF, 0xF, true));
            m = max(m, (uint32_t)__builtin_amdgcn_mov_dpp((int)m, 0x140, 0xF, 0xF, true));
            m = max(max((uint32_t)__builtin_amdgcn_readlane((int)m, 0), (uint32_t)__builtin_amdgcn_readlane((int)m, 16)),
                    max((uint32_t)__builtin_amdgcn_readlane((int)m, 32), (uint32_t)__builtin_amdgcn_readlane((int)m, 48)));
            if (m) {
                ind[r] = 31 - (int)(m & 31u);
                mx[r] = (int)(m >> 5);
                if (key == m) key = 0u;
            }
        }
        int ind1 = ind[0], ind2 = ind[1], ind3 = ind[2];
        const int max1 = mx[0], max2 = mx[1], max3 = mx[2];
        if ((float)max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
        else if ((float)max3 < 0.1f * (float)max1) { ind3 = -1; }
        for (int i = lane; i < n10; i += 64) {
            const int bb = bin[i];
            if (bb < 0 || bb == ind1 || bb == ind2 || bb == ind3) continue;
            m12[i] = -1;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    int nmatches = 0;   // wave-uniform: ballot counts
    for (int i0 = 0; i0 < n10; i0 += 256) {   // four rows of 64 at a time: their k2 loads in flight together
        int v[4];
        float2 kp[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = i0 + 64 * u + lane;
            v[u] = i < n10 ? (int)m12[i] : -1;
            if (pv && v[u] >= 0) kp[u] = make_float2(k2[v[u]].x, k2[v[u]].y);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = i0 + 64 * u + lane;
            if (i < n10) {
                out[i] = v[u];
                if (pv && v[u] >= 0) pv[i] = kp[u];   // update vbPrevMatched (:580-584)
            }
            nmatches += __popcll(__ballot(v[u] >= 0));
        }
    }
    if (lane == 0) nm_out[pair] = nmatches;
#ifdef ORBX_SI_PROF
    const long long pt3 = clock64();
    if (lane == 0) {   // phase cycles (staging, greedy loop, bins+filter+output) over the unused tail
        out[cap - 6] = prof_chunks;
        out[cap - 5] = prof_scans;
        out[cap - 4] = (int)(pt1 - pt0);
        out[cap - 3] = (int)(pt2 - pt1);
        out[cap - 2] = (int)(pt3 - pt2);
        out[cap - 1] = n10;
    }
#endif
}

// largest level-0 count whose greedy-pass arrays fit a workgroup's 160 KiB of LDS; larger frames take the
// global-array launch (k_si_greedy<true>)
static int si_lds_max_cap()
{
    static const int c = [] {
        int v = 32767;
        while (v > 1 && sg_layout(v).total > 160 * 1024 - 256) v -= 16;   // + the static histogram
        return v;
    }();
    return c;
}

static size_t si_global_stride(int cap) { return (sg_layout(cap).total + 255) & ~(size_t)255; }

size_t search_init_scratch_bytes(int nframes, int npairs, int cap)
{
    size_t b = (size_t)nframes * cap * (4 + 8) + (size_t)nframes * 2 * 4 + (size_t)npairs * cap * (4 + 16) + 64 * 7;
    if (cap > si_lds_max_cap()) b += (size_t)npairs * si_global_stride(cap);
    return b;
}

void launch_search_init(const orbx_keypoint* kps, const uint8_t* desc, const int* counts, int nframes, int cap,
                        const int* pa, const int* pb, int npairs, const orbm_grid& G, int window, float nnratio,
                        int check_ori, float* prev, void* scratch, int* m12, int* nm, hipStream_t s)
{
    uint8_t* p = (uint8_t*)scratch;
    auto carve = [&](size_t bytes) {
        uint8_t* r = p;
        p += (bytes + 63) & ~(size_t)63;
        return r;
    };
    uint32_t* gkeys = (uint32_t*)carve((size_t)nframes * cap * 4);
    float2* gxy = (float2*)carve((size_t)nframes * cap * 8);
    int* gn = (int*)carve((size_t)nframes * 2 * 4);
    int* qcnt = (int*)carve((size_t)npairs * cap * 4);
    uint4* qtop = (uint4*)carve((size_t)npairs * cap * 16);
    hipFuncSetAttribute((const void*)k_si_grid, hipFuncAttributeMaxDynamicSharedMemorySize, (int)si_grid_smem(cap));
    hipLaunchKernelGGL(k_si_grid, dim3(nframes), dim3(256), si_grid_smem(cap), s, kps, counts, cap, G, gkeys, gxy, gn);
    const size_t bsmem = si_build_smem_bytes();
    // query slices per pair: about 8 waves per SIMD over the chip, at least 4 queries per wave
    const int qsplit = std::max(1, std::min((2048 + npairs - 1) / npairs, (cap + 15) / 16));
    hipLaunchKernelGGL(k_si_build, dim3(npairs, qsplit), dim3(SI_BUILD_NT), bsmem, s, kps, desc, cap, pa, pb, G,
                       window, (const float2*)prev, gkeys, gxy, gn, qcnt, qtop);
    const int ldscap = std::min(cap, si_lds_max_cap());
    hipFuncSetAttribute((const void*)k_si_greedy<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        (int)sg_layout(ldscap).total);
    // tiers by level-0 count: up to 512 (22 KB per workgroup), up to kSiLdsCap (two workgroups per CU), the
    // LDS maximum, then cap from global memory; a launch whose tier holds no pair costs a few microseconds
    // (its workgroups return at once)
    const int tiers[3] = {std::min(cap, kSiGreedySmall), std::min(cap, kSiLdsCap), ldscap};
    int lo = -1;
    for (int t = 0; t < 3; ++t) {
        if (tiers[t] <= lo) continue;
        hipLaunchKernelGGL(k_si_greedy<false>, dim3(npairs), dim3(256), sg_layout(tiers[t]).total, s, kps, desc,
                           counts, cap, pa, pb, G, window, nnratio, check_ori, (float2*)prev, gkeys, gxy, gn, qcnt,
                           qtop, m12, nm, tiers[t], lo, (uint8_t*)nullptr, (size_t)0);
        lo = tiers[t];
    }
    if (cap > lo) {
        uint8_t* gbuf = carve((size_t)npairs * si_global_stride(cap));
        hipLaunchKernelGGL(k_si_greedy<true>, dim3(npairs), dim3(256), 0, s, kps, desc, counts, cap, pa, pb, G, window,
                           nnratio, check_ori, (float2*)prev, gkeys, gxy, gn, qcnt, qtop, m12, nm, cap, lo, gbuf,
                           si_global_stride(cap));
    }
}

}  // namespace orbx
