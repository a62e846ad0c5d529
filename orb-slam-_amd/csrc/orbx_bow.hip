// gfx950 kernels of the vocabulary-node Hamming searches of ORBmatcher
// (SURVEY.md §8a rows a12/a13):
//   SearchByBoW(KeyFrame*, Frame&)         src/ORBmatcher.cc:159-288
//   SearchByBoW(KeyFrame*, KeyFrame*)      src/ORBmatcher.cc:590-723
//   SearchForTriangulation + CheckDistEpipolarLine   :725-891, :140-157
//
// B1 k_bow_nodes  one wave per node of view1's FeatureVector.  The node is looked
//                 up in view2's (the merge-join of :175-257 visits exactly the shared
//                 ids), then the node's view1 features are replayed in order: each is
//                 one wave-wide search over the node's view2 features (64 per pass),
//                 reduced to (best, first index) and the multiset second best; the
//                 greedy "already matched" state is a per-wave LDS bitmap because
//                 nodes own disjoint feature sets.
// B2 k_bow_rot    one workgroup per pair: rotation histogram, ComputeThreeMaxima
//                 (:1679-1723) and removal, nmatches.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "orbx_kernels.hpp"

namespace orbx {

constexpr int kBowMaxCand = ORBM_MAX_FEATURES;     // view2 features per node (LDS bitmap per wave, 2 KiB)
constexpr int kBowWords = kBowMaxCand / 32;
constexpr int kTH_LOW = 50, kHisto = 30;

__device__ __forceinline__ void bow_wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o));
    return v;
}

// the same over a fully active wave with DPP row reductions and four readlanes (no LDS round trips)
__device__ __forceinline__ uint32_t wave_min_dpp(uint32_t v)
{
    auto dpp_min = [](uint32_t x, auto ctrl) {
        return min(x, (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, decltype(ctrl)::value, 0xF, 0xF, false));
    };
    v = dpp_min(v, std::integral_constant<int, 0xB1>{});    // quad_perm [1,0,3,2]
    v = dpp_min(v, std::integral_constant<int, 0x4E>{});    // quad_perm [2,3,0,1]
    v = dpp_min(v, std::integral_constant<int, 0x141>{});   // row_half_mirror
    v = dpp_min(v, std::integral_constant<int, 0x140>{});   // row_mirror
    const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)v, 0), r1 = (uint32_t)__builtin_amdgcn_readlane((int)v, 16);
    const uint32_t r2 = (uint32_t)__builtin_amdgcn_readlane((int)v, 32), r3 = (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
    return min(min(r0, r1), min(r2, r3));
}

__device__ __forceinline__ int bow_rot_bin(float a1, float a2)
{
    const float factor = 1.0f / kHisto;   // the reference's 1/HISTO_LENGTH (bins 0..12 used)
    float rot = a1 - a2;
    if (rot < 0.0f) rot += 360.0f;
    int bin = (int)roundf(rot * factor);
    if (bin == kHisto) bin = 0;
    return bin;
}

// CheckDistEpipolarLine with the FMAs GCC 11 -O3 -march=native forms
__device__ __forceinline__ bool bow_epipolar(float x1, float y1, float x2, float y2, int oct2,
                                             const orbm_triang_params& T)
{
    const float* F = T.F12;
    const float a = __builtin_fmaf(x1, F[0], y1 * F[3]) + F[6];
    const float b = __builtin_fmaf(x1, F[1], y1 * F[4]) + F[7];
    const float c = __builtin_fmaf(y1, F[5], x1 * F[2]) + F[8];
    const float num = __builtin_fmaf(b, y2, a * x2) + c;
    const float den = __builtin_fmaf(a, a, b * b);
    if (den == 0) return false;
    const float dsqr = num * num / den;
    return (double)dsqr < 3.84 * (double)T.sigma2_2[oct2];
}

__device__ __forceinline__ int ham_u4(const uint4& a0, const uint4& a1, const uint4& b0, const uint4& b1)
{
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

// A view with its arrays as global pointers: the struct's pointers are loaded from memory, where the compiler no
// longer knows they are global, and reads through them would be flat loads (which wait on both counters).
#define ORBX_G1 __attribute__((address_space(1)))
struct GView {
    const ORBX_G1 orbx_keypoint* kps;
    const ORBX_G1 uint8_t* desc;
    const ORBX_G1 uint8_t* has_mp;
    const ORBX_G1 float* u_right;
    const ORBX_G1 int32_t* fv_node;
    const ORBX_G1 int32_t* fv_ptr;
    const ORBX_G1 int32_t* fv_idx;
    int32_t n, fv_nnodes;
};
__device__ __forceinline__ orbx_keypoint kp_at(const ORBX_G1 orbx_keypoint* k, int i)
{
    const ORBX_G1 orbx_keypoint& q = k[i];
    orbx_keypoint r;
    r.x = q.x;
    r.y = q.y;
    r.size = q.size;
    r.angle = q.angle;
    r.response = q.response;
    r.octave = q.octave;
    r.class_id = q.class_id;
    return r;
}
// descriptor i's 32 bytes as two uint4
__device__ __forceinline__ void desc_at(const ORBX_G1 uint8_t* d, int i, uint4& a, uint4& b)
{
    const ORBX_G1 uint32_t* q = (const ORBX_G1 uint32_t*)(d + (size_t)i * 32);
    a = make_uint4(q[0], q[1], q[2], q[3]);
    b = make_uint4(q[4], q[5], q[6], q[7]);
}
__device__ __forceinline__ GView gview(const orbm_bow_view& v)
{
    return GView{(const ORBX_G1 orbx_keypoint*)v.kps, (const ORBX_G1 uint8_t*)v.desc,
                 (const ORBX_G1 uint8_t*)v.has_mp, (const ORBX_G1 float*)v.u_right,
                 (const ORBX_G1 int32_t*)v.fv_node, (const ORBX_G1 int32_t*)v.fv_ptr,
                 (const ORBX_G1 int32_t*)v.fv_idx, v.n, v.fv_nnodes};
}

__global__ __launch_bounds__(256) void k_bow_nodes(int mode, const orbm_bow_view* __restrict__ V1,
                                                   const orbm_bow_view* __restrict__ V2,
                                                   const orbm_triang_params* __restrict__ TP, float nnratio,
                                                   int check_ori, int* __restrict__ match, int* __restrict__ bins,
                                                   int stride)
{
    __shared__ uint32_t s_done[4][kBowWords];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;   // uniform
    const int p = blockIdx.y;
    const GView A = gview(V1[p]), B = gview(V2[p]);
    const int k = blockIdx.x * 4 + wave;
    if (k >= A.fv_nnodes) return;   // wave-uniform; no block barriers below
    const int node = A.fv_node[k];
    int lo = 0, hi = B.fv_nnodes;   // lower_bound of the node id in view2 (:249-256)
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (B.fv_node[mid] < node) lo = mid + 1; else hi = mid;
    }
    if (lo >= B.fv_nnodes || B.fv_node[lo] != node) return;
    const int a0 = A.fv_ptr[k], a1 = A.fv_ptr[k + 1];
    const int b0 = B.fv_ptr[lo];
    const int nb = min(B.fv_ptr[lo + 1] - b0, kBowMaxCand);
    int* M = match + (size_t)p * stride;
    int* BN = bins + (size_t)p * stride;
    uint32_t* done = s_done[wave];
    for (int i = lane; i < (nb + 31) / 32; i += 64) done[i] = 0;
    bow_wave_sync();
    const bool tri = mode == ORBM_TRIANGULATION;
    orbm_triang_params T;
    if (tri) T = TP[p];

    // The node's first 64 view2 features stay in registers for all of its view1 features, and the
    // view1 features are loaded 64 at a time (lane j = feature j) and broadcast by readlane: the
    // serial replay below touches global memory only for nodes with more than 64 view2 features.
    int c_idx2 = 0;
    bool c_mp2 = false, c_st2 = false;
    uint4 c_e0 = make_uint4(0, 0, 0, 0), c_e1 = c_e0;
    orbx_keypoint c_kp2{};
    if (lane < nb) {
        c_idx2 = B.fv_idx[b0 + lane];
        c_mp2 = B.has_mp ? B.has_mp[c_idx2] != 0 : false;
        desc_at(B.desc, c_idx2, c_e0, c_e1);
        if (tri) {
            c_st2 = B.u_right ? B.u_right[c_idx2] >= 0 : false;
            c_kp2 = kp_at(B.kps, c_idx2);
        }
    }
    const int n1 = a1 - a0;
    for (int abase = 0; abase < n1; abase += 64) {
        int l_idx1 = 0, l_flags = 0;
        uint4 l_q0 = make_uint4(0, 0, 0, 0), l_q1 = l_q0;
        float l_x = 0.f, l_y = 0.f, l_ang = 0.f;
        if (abase + lane < n1) {
            l_idx1 = A.fv_idx[a0 + abase + lane];
            const bool mp = A.has_mp ? A.has_mp[l_idx1] != 0 : false;
            const bool st = tri && A.u_right ? A.u_right[l_idx1] >= 0 : false;
            l_flags = (mp ? 1 : 0) | (st ? 2 : 0);
            desc_at(A.desc, l_idx1, l_q0, l_q1);
            const orbx_keypoint kp = kp_at(A.kps, l_idx1);
            l_x = kp.x;
            l_y = kp.y;
            l_ang = kp.angle;
        }
        const int cnt = min(64, n1 - abase);
        for (int j = 0; j < cnt; ++j) {
            auto bc = [&](uint32_t v) { return (uint32_t)__builtin_amdgcn_readlane((int)v, j); };
            auto bcf = [&](float v) { return __builtin_bit_cast(float, bc(__builtin_bit_cast(uint32_t, v))); };
            const int idx1 = (int)bc((uint32_t)l_idx1);
            const int flags1 = (int)bc((uint32_t)l_flags);
            const bool mp1 = flags1 & 1;
            bool stereo1 = false;
            if (tri) {
                if (mp1) continue;   // "If there is already a MapPoint skip" (:775-776)
                stereo1 = (flags1 & 2) != 0;
                if (T.only_stereo && !stereo1) continue;
            } else if (!mp1) {
                continue;            // !pMP || pMP->isBad()
            }
            const uint4 q0 = make_uint4(bc(l_q0.x), bc(l_q0.y), bc(l_q0.z), bc(l_q0.w));
            const uint4 q1 = make_uint4(bc(l_q1.x), bc(l_q1.y), bc(l_q1.z), bc(l_q1.w));
            const float x1 = bcf(l_x), y1 = bcf(l_y), ang1 = bcf(l_ang);
            uint32_t best = 0xFFFFFFFFu;   // greedy: (dist << 16 | pos) first min; triangulation: (dist, last pos)
            int second = 256;              // this lane's second smallest distance (multiset)
            for (int c = 0; c < nb; c += 64) {
                const int pos = c + lane;
                if (pos >= nb) break;
                int idx2 = c_idx2;
                bool mp2 = c_mp2;
                uint4 e0 = c_e0, e1 = c_e1;
                if (c > 0) {
                    idx2 = B.fv_idx[b0 + pos];
                    mp2 = B.has_mp ? B.has_mp[idx2] != 0 : false;
                    desc_at(B.desc, idx2, e0, e1);
                }
                bool ok;
                if (tri) {
                    ok = !mp2;
                } else {
                    ok = !((done[pos >> 5] >> (pos & 31)) & 1u);
                    if (mode == ORBM_BOW_KF_KF) ok = ok && mp2;
                }
                if (!ok) continue;
                const int dist = ham_u4(q0, q1, e0, e1);
                if (tri) {
                    const bool stereo2 = c > 0 ? (B.u_right ? B.u_right[idx2] >= 0 : false) : c_st2;
                    if (T.only_stereo && !stereo2) continue;
                    if (dist > kTH_LOW) continue;
                    const orbx_keypoint kp2 = c > 0 ? kp_at(B.kps, idx2) : c_kp2;
                    if (!stereo1 && !stereo2) {   // :800-806
                        const float distex = T.ex - kp2.x, distey = T.ey - kp2.y;
                        if (__builtin_fmaf(distex, distex, distey * distey) < 100 * T.scale2[kp2.octave]) continue;
                    }
                    if (!bow_epipolar(x1, y1, kp2.x, kp2.y, kp2.octave, T)) continue;
                    // the sequential `dist > bestDist -> skip, else take` keeps the LAST minimum
                    best = min(best, ((uint32_t)dist << 16) | (uint32_t)(0xFFFF - pos));
                } else {
                    const uint32_t key = ((uint32_t)dist << 16) | (uint32_t)pos;
                    if (key < best) {
                        second = min(second, (int)(best >> 16));
                        best = key;
                    } else {
                        second = min(second, dist);
                    }
                }
            }
            const uint32_t wbest = wave_min_dpp(best);
            if (wbest == 0xFFFFFFFFu) continue;
            const int bdist = (int)(wbest >> 16);
            if (tri) {
                const int pos = 0xFFFF - (int)(wbest & 0xFFFF);
                if (lane == 0) {
                    const int idx2 = B.fv_idx[b0 + pos];
                    M[idx1] = idx2;
                    if (check_ori) BN[idx1] = bow_rot_bin(ang1, B.kps[idx2].angle);
                }
                continue;
            }
            // second best of the whole node = min(the winner lane's second, every other lane's best)
            const int mine = best == wbest ? second : (int)min(best >> 16, 256u);
            const int bsecond = (int)wave_min_dpp((uint32_t)mine);
            const bool accept = (mode == ORBM_BOW_KF_F ? bdist <= kTH_LOW : bdist < kTH_LOW) &&
                                (float)bdist < nnratio * (float)bsecond;
            if (accept) {
                const int pos = (int)(wbest & 0xFFFF);
                if (lane == 0) {
                    const int idx2 = B.fv_idx[b0 + pos];
                    done[pos >> 5] |= 1u << (pos & 31);
                    if (mode == ORBM_BOW_KF_F) {
                        M[idx2] = idx1;
                        if (check_ori) BN[idx2] = bow_rot_bin(ang1, B.kps[idx2].angle);
                    } else {
                        M[idx1] = idx2;
                        if (check_ori) BN[idx1] = bow_rot_bin(ang1, B.kps[idx2].angle);
                    }
                }
                bow_wave_sync();
            }
        }
    }
}

__global__ __launch_bounds__(256) void k_bow_rot(int mode, const orbm_bow_view* __restrict__ V1,
                                                 const orbm_bow_view* __restrict__ V2, int check_ori,
                                                 int* __restrict__ match, const int* __restrict__ bins, int stride,
                                                 int* __restrict__ nmatches)
{
    __shared__ int s_hist[kHisto];
    __shared__ int s_ind[3];
    __shared__ int s_n;
    const int p = blockIdx.x, tid = threadIdx.x;
    const int n = min(mode == ORBM_BOW_KF_F ? V2[p].n : V1[p].n, stride);
    int* M = match + (size_t)p * stride;
    const int* BN = bins + (size_t)p * stride;
    if (tid < kHisto) s_hist[tid] = 0;
    if (tid == 0) s_n = 0;
    __syncthreads();
    if (check_ori) {
        for (int i = tid; i < n; i += 256)
            if (BN[i] >= 0) atomicAdd(&s_hist[BN[i]], 1);
        __syncthreads();
        if (tid == 0) {   // ComputeThreeMaxima, src/ORBmatcher.cc:1679-1723
            int ind1 = -1, ind2 = -1, ind3 = -1, max1 = 0, max2 = 0, max3 = 0;
            for (int i = 0; i < kHisto; ++i) {
                const int s = s_hist[i];
                if (s > max1) { max3 = max2; max2 = max1; max1 = s; ind3 = ind2; ind2 = ind1; ind1 = i; }
                else if (s > max2) { max3 = max2; max2 = s; ind3 = ind2; ind2 = i; }
                else if (s > max3) { max3 = s; ind3 = i; }
            }
            if ((float)max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
            else if ((float)max3 < 0.1f * (float)max1) { ind3 = -1; }
            s_ind[0] = ind1;
            s_ind[1] = ind2;
            s_ind[2] = ind3;
        }
        __syncthreads();
    }
    int cnt = 0;
    for (int i = tid; i < n; i += 256) {
        if (M[i] < 0) continue;
        if (check_ori) {
            const int b = BN[i];
            if (b >= 0 && b != s_ind[0] && b != s_ind[1] && b != s_ind[2]) {
                M[i] = -1;
                continue;
            }
        }
        ++cnt;
    }
    atomicAdd(&s_n, cnt);
    __syncthreads();
    if (tid == 0) nmatches[p] = s_n;
}

void launch_bow(int mode, const orbm_bow_view* v1, const orbm_bow_view* v2, const orbm_triang_params* tp,
                int npairs, int max_nodes1, float nnratio, int check_ori, int* match, int* bins, int stride,
                int* nmatches, hipStream_t s)
{
    hipMemsetAsync(match, 0xFF, sizeof(int) * (size_t)npairs * stride, s);   // -1
    hipMemsetAsync(bins, 0xFF, sizeof(int) * (size_t)npairs * stride, s);
    if (max_nodes1 > 0)
        hipLaunchKernelGGL(k_bow_nodes, dim3((max_nodes1 + 3) / 4, npairs), dim3(256), 0, s, mode, v1, v2, tp,
                           nnratio, check_ori, match, bins, stride);
    hipLaunchKernelGGL(k_bow_rot, dim3(npairs), dim3(256), 0, s, mode, v1, v2, check_ori, match, bins, stride,
                       nmatches);
}

}  // namespace orbx
