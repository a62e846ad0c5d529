// gfx950 kernels of Frame::ComputeStereoMatches (src/Frame.cc:630-872) on the
// device pyramid of a rectified stereo pair.  Integer work (Hamming + SAD) with
// the reference's float geometry restated operation by operation
// (-ffp-contract=off, like the reference's GCC build: SURVEY.md F6).
//
//   S1 k_stereo_match  one lane per left keypoint: row-band coarse search
//                      (first min of (Hamming, iR), :645-757) + 11x11 SAD over 11
//                      shifts + parabola (:759-853), on the pyramid level `octave`
//   S2 k_stereo_cut    one workgroup per pair: median of the accepted SADs and
//                      the 2.1 x median outlier cut (:857-871)
#include <hip/hip_runtime.h>
#include <limits.h>

#include "orbx_kernels.hpp"

namespace orbx {

constexpr int kStNT = 256;

__device__ __forceinline__ const uint8_t* st_level(const FramePtrs& P, const Geometry* G, int f, int l, int& pitch)
{
    if (l == 0) {
        pitch = P.in_pitch;
        return P.in + (size_t)f * P.in_fstride;
    }
    pitch = G->lv[l].pitch;
    return P.pyr + (size_t)f * P.pyr_fstride + G->lv[l].pyr_off;
}

// BORDER_REFLECT_101 index inside the 19-px pad of a level (ComputePyramid :1350-1373)
__device__ __forceinline__ int st_reflect(int p, int len)
{
    if (len == 1) return 0;
    while (p < 0 || p >= len) p = p < 0 ? -p : 2 * len - 2 - p;
    return p;
}

__device__ __forceinline__ int ham256(const uint4& a0, const uint4& a1, const uint4& b0, const uint4& b1)
{
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

struct StereoLds {
    int* off;          // [rows + 1] bucket offsets (bucket = floor(kpY))
    uint16_t* list;    // [cap] right keypoints grouped by bucket
    float* rx;         // [cap] right kp x
    float* ry;         // [cap] right kp y
    int8_t* ro;        // [cap] right kp octave
};

__host__ __device__ inline size_t stereo_lds_bytes(int rows, int cap)
{
    return (size_t)4 * (rows + 2) + (size_t)cap * (2 + 4 + 4 + 1) + 64;
}

// right keypoints -> row buckets (vRowIndices, :645-673): keypoints grouped by floor(kpY), clamped
// to [0, rows); off[b] ends as the end of bucket b (= the start of bucket b + 1)
__device__ __forceinline__ void st_buckets(StereoLds& S, const orbx_keypoint* __restrict__ KR, int nR, int rows,
                                           int tid)
{
    for (int r = tid; r <= rows; r += kStNT) S.off[r] = 0;
    __syncthreads();
    for (int i = tid; i < nR; i += kStNT) {
        const orbx_keypoint k = KR[i];
        S.rx[i] = k.x;
        S.ry[i] = k.y;
        S.ro[i] = (int8_t)k.octave;
        const int b = min(max((int)floorf(k.y), 0), rows - 1);
        atomicAdd(&S.off[b + 1], 1);
    }
    __syncthreads();
    if (tid < 64) {   // inclusive scan of rows+1 counts by one wave
        int run = 0;
        for (int base = 0; base <= rows; base += 64) {
            const int i = base + tid;
            int v = i <= rows ? S.off[i] : 0;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int y = __shfl_up(v, o);
                if (tid >= o) v += y;
            }
            if (i <= rows) S.off[i] = run + v;
            run += __shfl(v, 63);
        }
    }
    __syncthreads();
    for (int i = tid; i < nR; i += kStNT) {
        const int b = min(max((int)floorf(S.ry[i]), 0), rows - 1);
        const int slot = atomicAdd(&S.off[b], 1);   // off[b] walks to the bucket end
        S.list[slot] = (uint16_t)i;
    }
    __syncthreads();
}

// the coarse search of one left keypoint (:699-757): right keypoints whose band
// [floor(kpY - r), ceil(kpY + r)], r = 2 * scale[octave], holds the left row, octave within
// levelL +- 1, uR in [minU, maxU]; first min of Hamming in increasing iR = min of (dist << 16 | iR).
// Returns (bestDist << 16 | bestIdxR), 100 << 16 when nothing beats TH_HIGH.
template <class ScaleOf>
__device__ __forceinline__ int st_coarse(const StereoLds& S, int rows, int rband, ScaleOf scale_of, int row, int levelL,
                                         float minU, float maxU, const uint4& a0, const uint4& a1,
                                         const uint8_t* __restrict__ descR)
{
    int bestKey = 100 << 16;   // (bestDist = TH_HIGH, bestIdxR = 0)
    const int b0 = max(row - rband - 1, 0), b1 = min(row + rband + 1, rows - 1);
    for (int j = b0 == 0 ? 0 : S.off[b0 - 1]; j < S.off[b1]; ++j) {
        const int iR = S.list[j];
        const float kpY = S.ry[iR];
        const int oR = S.ro[iR];
        const float r = 2.0f * scale_of(oR);   // :662
        const int maxr = (int)ceilf(kpY + r), minr = (int)floorf(kpY - r);
        if (row < minr || row > maxr) continue;
        if (oR < levelL - 1 || oR > levelL + 1) continue;   // :729-730
        const float uR = S.rx[iR];
        if (uR >= minU && uR <= maxU) {
            const uint4* dr = reinterpret_cast<const uint4*>(descR + (size_t)iR * 32);
            bestKey = min(bestKey, (ham256(a0, a1, dr[0], dr[1]) << 16) | iR);
        }
    }
    return bestKey;
}

__global__ __launch_bounds__(kStNT) void k_stereo_match(const Geometry* __restrict__ G, FramePtrs PL, FramePtrs PR,
                                                        const orbx_keypoint* __restrict__ kps,
                                                        const uint8_t* __restrict__ desc,
                                                        const int* __restrict__ counts, int cap,
                                                        const int* __restrict__ fleft, const int* __restrict__ fright,
                                                        float bf, float maxD, int rband,
                                                        float* __restrict__ uright, float* __restrict__ depth,
                                                        int* __restrict__ sad)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t s_st[];
    const int p = blockIdx.y, tid = threadIdx.x;
    const int fl = fleft[p], fr = fright[p];
    const int nL = min(counts[fl], cap), nR = min(counts[fr], cap);
    const int rows = G->rows;
    StereoLds S;
    S.off = (int*)s_st;
    S.rx = (float*)(s_st + (((size_t)4 * (rows + 2) + 15) & ~(size_t)15));
    S.ry = S.rx + cap;
    S.list = (uint16_t*)(S.ry + cap);
    S.ro = (int8_t*)(S.list + cap);
    const orbx_keypoint* KR = kps + (size_t)fr * cap;
    const orbx_keypoint* KL = kps + (size_t)fl * cap;

    st_buckets(S, KR, nR, rows, tid);

    const int iL = blockIdx.x * kStNT + tid;
    if (iL >= nL) return;
    const size_t o = (size_t)p * cap + iL;
    float outU = -1.0f, outD = -1.0f;
    int outS = -1;
    const orbx_keypoint kpL = KL[iL];
    const int levelL = kpL.octave;
    const float vL = kpL.y, uL = kpL.x;
    const float minD = 0.0f;
    bool ok = vL >= 0.0f && levelL >= 0 && levelL < G->nlevels;
    const int row = ok ? (int)vL : 0;   // vRowIndices[vL]: float -> index truncation (:699)
    ok = ok && row < rows;
    const float minU = uL - maxD, maxU = uL - minD;   // :707-708
    ok = ok && !(maxU < 0);
    int bestKey = 100 << 16;
    if (ok) {
        const uint4* dl = reinterpret_cast<const uint4*>(desc + ((size_t)fl * cap + iL) * 32);
        bestKey = st_coarse(S, rows, rband, [&](int oR) { return G->lv[oR].scale; }, row, levelL, minU, maxU, dl[0],
                            dl[1], desc + (size_t)fr * cap * 32);
    }
    const int bestDist = bestKey >> 16, bestIdxR = bestKey & 0xFFFF;
    if (ok && bestDist < 75) {   // thOrbDist = (TH_HIGH + TH_LOW) / 2, :762
        const LevelGeom& LG = G->lv[levelL];
        const float uR0 = S.rx[bestIdxR];
        const float scaleFactor = LG.inv_scale;
        const float scaleduL = roundf(kpL.x * scaleFactor);
        const float scaledvL = roundf(kpL.y * scaleFactor);
        const float scaleduR0 = roundf(uR0 * scaleFactor);
        const int w = 5, L = 5;
        const float iniu = scaleduR0 + L - w;   // the reference's +L (quirk kept), :795
        const float endu = scaleduR0 + L + w + 1;
        const int W = LG.w, H = LG.h;
        const int vy = (int)scaledvL, ux = (int)scaleduL, ur = (int)scaleduR0;
        bool go = !(iniu < 0 || endu >= W);
        // windows inside the level's 19-px reflect-101 padding; beyond it the reference is UB
        go = go && vy - w >= -kEdge && vy + w < H + kEdge && ux - w >= -kEdge && ux + w < W + kEdge &&
             ur - L - w >= -kEdge;
        if (go) {
            int pl, pr;
            const uint8_t* IL = st_level(PL, G, fl, levelL, pl);
            const uint8_t* IR = st_level(PR, G, fr, levelL, pr);
            const bool inner = vy - w >= 0 && vy + w < H && ux - w >= 0 && ux + w < W && ur - L - w >= 0 &&
                               ur + L + w < W;
            auto px = [&](const uint8_t* I, int pitch, int x, int y) -> int {
                if (!inner) {
                    x = st_reflect(x, W);
                    y = st_reflect(y, H);
                }
                return I[(size_t)y * pitch + x];
            };
            const int cL = px(IL, pl, ux, vy);
            int cR[11], acc[11];
#pragma unroll
            for (int s = 0; s < 11; ++s) {
                cR[s] = px(IR, pr, ur + s - L, vy);
                acc[s] = 0;
            }
            // |(IL - cL) - (IR - cR)| = |(IL + cR) - (IR + cL)|: both sides are non-negative
            // and < 2^16, so two columns go through one v_sad_u16 (packed u16 halves)
            for (int y = -w; y <= w; ++y) {
                uint32_t lp[6], rr[22];
#pragma unroll
                for (int k = 0; k < 6; ++k) {
                    const int x0 = 2 * k, x1 = 2 * k + 1;
                    lp[k] = (uint32_t)px(IL, pl, ux - w + x0, vy + y) |
                            (x1 < 11 ? (uint32_t)px(IL, pl, ux - w + x1, vy + y) << 16 : 0u);
                }
#pragma unroll
                for (int x = 0; x < 21; ++x) rr[x] = (uint32_t)(px(IR, pr, ur - L - w + x, vy + y) + cL);
                rr[21] = 0;
#pragma unroll
                for (int s = 0; s < 11; ++s) {
                    const uint32_t cc = (uint32_t)cR[s] * 0x10001u;
                    uint32_t a = (uint32_t)acc[s];
#pragma unroll
                    for (int k = 0; k < 6; ++k) {
                        const uint32_t lo = rr[s + 2 * k];
                        const uint32_t hi = 2 * k + 1 < 11 ? rr[s + 2 * k + 1] : 0u;
                        // the unused high half of the last pair: left 0 + cc vs right 0 -> mask it out
                        const uint32_t lv = 2 * k + 1 < 11 ? lp[k] + cc : lp[k] + (uint32_t)cR[s];
                        a = __builtin_amdgcn_sad_u16(lv, lo | (hi << 16), a);
                    }
                    acc[s] = (int)a;
                }
            }
            int best = INT_MAX, bestinc = 0;   // first strict minimum (:803-808)
            float vD[11];
#pragma unroll
            for (int s = 0; s < 11; ++s) {
                vD[s] = (float)acc[s];
                if (acc[s] < best) {
                    best = acc[s];
                    bestinc = s - L;
                }
            }
            if (bestinc != -L && bestinc != L) {   // :816-817
                const float dist1 = vD[L + bestinc - 1], dist2 = vD[L + bestinc], dist3 = vD[L + bestinc + 1];
                const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
                if (!(deltaR < -1 || deltaR > 1)) {
                    float bestuR = LG.scale * ((float)scaleduR0 + (float)bestinc + deltaR);   // :834
                    float disparity = (uL - bestuR);
                    if (disparity >= minD && disparity < maxD) {
                        if (disparity <= 0) {
                            disparity = (float)0.01;
                            bestuR = (float)((double)uL - 0.01);
                        }
                        outD = bf / disparity;
                        outU = bestuR;
                        outS = best;
                    }
                }
            }
        }
    }
    uright[o] = outU;
    depth[o] = outD;
    sad[o] = outS;
}

// S2: vDistIdx sorted, median = element size/2, cut every pair with dist >= 2.1 x median
// (:857-871).  Only the k-th smallest distance is needed: bitonic sort of the accepted
// SADs in LDS.
__global__ __launch_bounds__(1024) void k_stereo_cut(const int* __restrict__ counts, int cap,
                                                     const int* __restrict__ fleft, float* __restrict__ uright,
                                                     float* __restrict__ depth, const int* __restrict__ sad,
                                                     int* __restrict__ ngood)
{
    extern __shared__ uint32_t s_key[];
    __shared__ int s_n, s_good;
    const int p = blockIdx.x, tid = threadIdx.x;
    const int nL = min(counts[fleft[p]], cap);
    const size_t base = (size_t)p * cap;
    if (tid == 0) {
        s_n = 0;
        s_good = 0;
    }
    __syncthreads();
    for (int i = tid; i < nL; i += 1024) {
        const int d = sad[base + i];
        if (d >= 0) s_key[atomicAdd(&s_n, 1)] = (uint32_t)d;
    }
    __syncthreads();
    const int n = s_n;
    if (n == 0) {   // an empty vDistIdx is UB in the reference: nothing to cut
        if (tid == 0) ngood[p] = 0;
        return;
    }
    int p2 = 1;
    while (p2 < n) p2 <<= 1;
    for (int i = n + tid; i < p2; i += 1024) s_key[i] = 0xFFFFFFFFu;
    __syncthreads();
    for (int size = 2; size <= p2; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int i = tid; i < (p2 >> 1); i += 1024) {
                const int lo = 2 * i - (i & (stride - 1)), hi = lo + stride;
                const bool up = (lo & size) == 0;
                const uint32_t a = s_key[lo], b = s_key[hi];
                if ((a > b) == up) {
                    s_key[lo] = b;
                    s_key[hi] = a;
                }
            }
            __syncthreads();
        }
    }
    const float median = (float)(int)s_key[n / 2];
    const float thDist = 1.5f * 1.4f * median;
    int good = 0;
    for (int i = tid; i < nL; i += 1024) {
        const int d = sad[base + i];
        if (d < 0) continue;
        if ((float)d < thDist) {
            ++good;
        } else {
            uright[base + i] = -1.0f;
            depth[base + i] = -1.0f;
        }
    }
    atomicAdd(&s_good, good);
    __syncthreads();
    if (tid == 0) ngood[p] = s_good;
}

// S3 k_stereo_band: the coarse stage alone (orbm_stereo_band), for callers that keep their own SAD
// stage.  Same buckets and search as S1; the scale table comes by value and is staged in LDS.
__global__ __launch_bounds__(kStNT) void k_stereo_band(StBandArgs A, const orbx_keypoint* __restrict__ kps,
                                                       const uint8_t* __restrict__ desc,
                                                       const int* __restrict__ counts, int cap,
                                                       const int* __restrict__ fleft, const int* __restrict__ fright,
                                                       int* __restrict__ best_idx, int* __restrict__ best_dist)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t s_st[];
    __shared__ float s_scale[kStMaxLevels];
    const int p = blockIdx.y, tid = threadIdx.x;
    const int fl = fleft[p], fr = fright[p];
    const int nL = min(counts[fl], cap), nR = min(counts[fr], cap);
    const int rows = A.rows;
    if (tid < kStMaxLevels) s_scale[tid] = A.scale[tid];
    StereoLds S;
    S.off = (int*)s_st;
    S.rx = (float*)(s_st + (((size_t)4 * (rows + 2) + 15) & ~(size_t)15));
    S.ry = S.rx + cap;
    S.list = (uint16_t*)(S.ry + cap);
    S.ro = (int8_t*)(S.list + cap);
    st_buckets(S, kps + (size_t)fr * cap, nR, rows, tid);   // its barriers also cover s_scale

    const int iL = blockIdx.x * kStNT + tid;
    if (iL >= nL) return;
    const orbx_keypoint kpL = kps[(size_t)fl * cap + iL];
    const int row = (int)kpL.y;   // vRowIndices[vL] (:699)
    const float minU = kpL.x - A.maxD, maxU = kpL.x - A.minD;   // :707-708
    int bestKey = 100 << 16;
    if (kpL.y >= 0.0f && row < rows && !(maxU < 0)) {
        const uint4* dl = reinterpret_cast<const uint4*>(desc + ((size_t)fl * cap + iL) * 32);
        const int nlv = A.nlevels;
        bestKey = st_coarse(S, rows, A.rband, [&](int oR) { return s_scale[min(max(oR, 0), nlv - 1)]; }, row,
                            kpL.octave, minU, maxU, dl[0], dl[1], desc + (size_t)fr * cap * 32);
    }
    const size_t o = (size_t)p * cap + iL;
    const int bd = bestKey >> 16;
    best_dist[o] = bd;
    best_idx[o] = bd < 100 ? (bestKey & 0xFFFF) : -1;
}

size_t stereo_match_smem(const Geometry& g, int cap) { return stereo_lds_bytes(g.rows, cap); }

size_t stereo_band_smem(int rows, int cap) { return stereo_lds_bytes(rows, cap); }

void launch_stereo_band(const StBandArgs& a, const orbx_keypoint* kps, const uint8_t* desc, const int* counts, int cap,
                        const int* fl, const int* fr, int npairs, int* best_idx, int* best_dist, hipStream_t s)
{
    const size_t sm = stereo_lds_bytes(a.rows, cap);
    hipFuncSetAttribute((const void*)k_stereo_band, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
    hipLaunchKernelGGL(k_stereo_band, dim3((cap + kStNT - 1) / kStNT, npairs), dim3(kStNT), sm, s, a, kps, desc,
                       counts, cap, fl, fr, best_idx, best_dist);
}

void launch_stereo(const Geometry& g, const Geometry* d_geom, const FramePtrs& PL, const FramePtrs& PR,
                   const orbx_keypoint* kps, const uint8_t* desc, const int* counts, int cap, const int* fl,
                   const int* fr, int npairs, float bf, float maxD, int rband, float* uright, float* depth, int* sad,
                   int* ngood, hipStream_t s)
{
    const size_t sm = stereo_lds_bytes(g.rows, cap);
    hipFuncSetAttribute((const void*)k_stereo_match, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
    hipLaunchKernelGGL(k_stereo_match, dim3((cap + kStNT - 1) / kStNT, npairs), dim3(kStNT), sm, s, d_geom, PL, PR,
                       kps, desc, counts, cap, fl, fr, bf, maxD, rband, uright, depth, sad);
    int p2 = 1;
    while (p2 < cap) p2 <<= 1;
    hipFuncSetAttribute((const void*)k_stereo_cut, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(4 * p2));
    hipLaunchKernelGGL(k_stereo_cut, dim3(npairs), dim3(1024), (size_t)4 * p2, s, counts, cap, fl, uright, depth,
                       sad, ngood);
}

}  // namespace orbx
