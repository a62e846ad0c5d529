// gfx950 kernels of ORBmatcher::SearchByProjection(Frame&, vector<MapPoint*>, th)
// (src/ORBmatcher.cc:45-129), the local-map search of Tracking::SearchLocalPoints,
// over Frame::GetFeaturesInArea (src/Frame.cc:410-495).  SURVEY.md §8f row 3.
//
// J1 k_pj_grid     one workgroup per frame: (cell, feature) keys of AssignFeaturesToGrid
//                  sorted in LDS, so a window's columns are one key range and the keys
//                  run in GetFeaturesInArea's visiting order (ix, then iy, then insertion)
// J2 k_pj_points   one lane per MapPoint: the reference's sequential scan over its window,
//                  against the frame's claims on entry, kept as the first kTop candidates in
//                  (distance, visiting position) order -- best and second are the first two
// J3 k_pj_resolve  one wave per frame replays the MapPoints in order, 64 at a time
//                  (replay_chunks): each takes the first unclaimed entries of its list; the
//                  lanes before the first collision with an earlier lane's claim commit
//                  together; a MapPoint whose list ran out searches its window again.
//                  Assignments and claims live in LDS.
#include <hip/hip_runtime.h>

#include "orbx_kernels.hpp"

namespace orbx {

constexpr int kPjCols = 64, kPjRows = 48;   // FRAME_GRID_COLS / ROWS (include/Frame.h:37-38)

__device__ __forceinline__ int pj_ham(const uint4& a0, const uint4& a1, const uint4& b0, const uint4& b1)
{
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

// J1 as a stable counting sort over the 3072 cells: per-cell counts by LDS atomics (the
// arrival slot is unordered), an exclusive scan, a scatter, then each feature's stable rank
// = the number of lower indices in its own cell segment (a few entries).  Keys are
// cell << 16 | index in ascending order, i.e. (cell, insertion) order.
constexpr int kPjCells = kPjCols * kPjRows;

// per frame: cap keys, then the kPjCells + 1 cell offsets (cell c = keys [off[c], off[c + 1]))
__host__ __device__ inline size_t pj_grid_stride(int cap) { return (size_t)cap + kPjCells + 4; }

__host__ __device__ inline size_t pj_grid_smem(int cap) { return (size_t)4 * (kPjCells + 4) + (size_t)6 * cap + 16; }

__global__ __launch_bounds__(256) void k_pj_grid(const orbx_keypoint* __restrict__ kps, const int* __restrict__ counts,
                                                 int cap, float min_x, float min_y, float grid_w_inv,
                                                 float grid_h_inv, uint32_t* __restrict__ gkeys, int* __restrict__ gn)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t s_grid[];
    __shared__ uint32_t s_wsum[4];
    uint32_t* start = s_grid;                                   // [kPjCells + 1] counts, then offsets
    uint16_t* code = (uint16_t*)(s_grid + kPjCells + 4);        // [cap] cell, 0xFFFF = outside the grid
    uint16_t* pos = code + cap;                                 // [cap] arrival slot within the cell
    uint16_t* tmp = pos + cap;                                  // [cap] features grouped by cell
    const int f = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int n = min(counts[f], cap);
    for (int c = tid; c <= kPjCells; c += 256) start[c] = 0u;
    __syncthreads();
    const orbx_keypoint* k = kps + (size_t)f * cap;
    for (int i = tid; i < n; i += 256) {   // PosInGrid, src/Frame.cc:504-518
        const int px = (int)roundf((k[i].x - min_x) * grid_w_inv);
        const int py = (int)roundf((k[i].y - min_y) * grid_h_inv);
        uint16_t cc = 0xFFFF;
        if (px >= 0 && px < kPjCols && py >= 0 && py < kPjRows) {
            cc = (uint16_t)(px * kPjRows + py);
            pos[i] = (uint16_t)atomicAdd(&start[cc], 1u);
        }
        code[i] = cc;
    }
    __syncthreads();
    constexpr int kPer = kPjCells / 256;   // 12 consecutive cells per thread
    uint32_t loc[kPer], sum = 0;
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
        loc[j] = start[tid * kPer + j];
        sum += loc[j];
    }
    uint32_t incl = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
    }
    if (lane == 63) s_wsum[wave] = incl;
    __syncthreads();
    uint32_t base = incl - sum;
    for (int w = 0; w < wave; ++w) base += s_wsum[w];
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
        start[tid * kPer + j] = base;
        base += loc[j];
    }
    if (tid == 255) start[kPjCells] = base;
    __syncthreads();
    for (int i = tid; i < n; i += 256)
        if (code[i] != 0xFFFF) tmp[start[code[i]] + pos[i]] = (uint16_t)i;
    __syncthreads();
    uint32_t* out = gkeys + (size_t)f * pj_grid_stride(cap);
    for (int c = tid; c <= kPjCells; c += 256) out[cap + c] = start[c];   // cell -> first key position
    for (int i = tid; i < n; i += 256) {
        const int cc = code[i];
        if (cc == 0xFFFF) continue;
        const int s0 = (int)start[cc], s1 = (int)start[cc + 1];
        int r = 0;
        for (int j = s0; j < s1; ++j) r += tmp[j] < i;
        out[s0 + r] = (uint32_t)cc << 16 | (uint32_t)i;
    }
    if (tid == 0) gn[f] = (int)start[kPjCells];
}

void launch_pj_grid(const orbx_keypoint* kps, const int* counts, int nframes, int cap, float min_x, float min_y,
                    float grid_w_inv, float grid_h_inv, uint32_t* gkeys, int* gn, hipStream_t s)
{
    const size_t sm = pj_grid_smem(cap);
    hipFuncSetAttribute((const void*)k_pj_grid, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
    hipLaunchKernelGGL(k_pj_grid, dim3(nframes), dim3(256), sm, s, kps, counts, cap, min_x, min_y, grid_w_inv,
                       grid_h_inv, gkeys, gn);
}

// GetFeaturesInArea(x, y, r * scale[level], level - 1, level) window of one MapPoint
struct PjWindow {
    int lo, hi, cx0, cx1, cy0, cy1, minLevel, maxLevel;
    float x, y, rr, rs;   // rr = window radius; rs = r * scale[level] for the stereo test
    bool ok;
};

__device__ __forceinline__ PjWindow pj_window(const orbm_proj_point& M, const orbm_proj_params& P,
                                              const uint32_t* keys, int cap)
{
    PjWindow w;
    w.ok = false;
    w.lo = w.hi = 0;
    const int level = M.level;
    if (level < 0 || level >= 16) return w;       // outside mvScaleFactors: UB in the reference
    float r = M.view_cos > 0.998 ? 2.5f : 4.0f;   // RadiusByViewingCos, src/ORBmatcher.cc:130-136
    if (P.th != 1.0f) r *= P.th;
    w.rr = r * P.scale[level];
    w.rs = r * P.scale[level];
    w.x = M.proj_x;
    w.y = M.proj_y;
    w.minLevel = level - 1;
    w.maxLevel = level;
    const int cx0 = max(0, (int)floorf((w.x - P.min_x - w.rr) * P.grid_w_inv));
    if (cx0 >= kPjCols) return w;
    const int cx1 = min(kPjCols - 1, (int)ceilf((w.x - P.min_x + w.rr) * P.grid_w_inv));
    if (cx1 < 0) return w;
    w.cy0 = max(0, (int)floorf((w.y - P.min_y - w.rr) * P.grid_h_inv));
    if (w.cy0 >= kPjRows) return w;
    w.cy1 = min(kPjRows - 1, (int)ceilf((w.y - P.min_y + w.rr) * P.grid_h_inv));
    if (w.cy1 < 0) return w;
    w.cx0 = cx0;
    w.cx1 = cx1;
    w.lo = (int)keys[cap + cx0 * kPjRows];
    w.hi = (int)keys[cap + (cx1 + 1) * kPjRows];
    w.ok = true;
    return w;
}

// candidate at key position p: the feature index if it is in the window (and not claimed,
// and passes the stereo test), else -1
__device__ __forceinline__ int pj_candidate(const PjWindow& w, const orbm_proj_point& M, const uint32_t* keys,
                                            int p, const orbx_keypoint* kps, const float* uright)
{
    const uint32_t key = keys[p];
    const int iy = (int)(key >> 16) % kPjRows;
    if (iy < w.cy0 || iy > w.cy1) return -1;
    const int idx = (int)(key & 0xFFFF);
    const orbx_keypoint kp = kps[idx];
    if (kp.octave < w.minLevel) return -1;   // bCheckLevels is true for level >= 0
    if (w.maxLevel >= 0 && kp.octave > w.maxLevel) return -1;
    const float distx = kp.x - w.x, disty = kp.y - w.y;
    if (!(fabsf(distx) < w.rr && fabsf(disty) < w.rr)) return -1;
    if (uright[idx] > 0) {   // src/ORBmatcher.cc:86-91
        const float er = fabsf(M.proj_xr - uright[idx]);
        if (er > w.rs) return -1;
    }
    return idx;
}

// The first kTop candidates of a window in (distance, visiting position) order -- the order in which
// the reference's sequential strict-< scan ranks them -- packed as dist:9 | bin:5 | octave:4 | idx:14
// (frames of up to ORBM_MAX_FEATURES = 16384 features; a distance is at most 256, 9 bits).
// A claim made later in the call only removes candidates, so the replay takes the first unclaimed
// entries of this list and scans the window again only when more than kTop were taken.
constexpr int kTop = 8;
struct TopK {
    uint32_t e[kTop];
    int n;   // candidates seen (saturating at 255)
};

__device__ __forceinline__ uint32_t top_entry(int dist, int bin, int oct, int idx)
{
    return (uint32_t)dist << 23 | (uint32_t)bin << 18 | (uint32_t)(oct & 15) << 14 | (uint32_t)idx;
}
static_assert(ORBM_MAX_FEATURES <= (1 << 14), "top_entry packs a feature index in 14 bits");
__device__ __forceinline__ int top_idx(uint32_t e) { return (int)(e & 0x3FFF); }
__device__ __forceinline__ int top_oct(uint32_t e) { return (int)((e >> 14) & 15); }
__device__ __forceinline__ int top_bin(uint32_t e) { return (int)((e >> 18) & 31); }
__device__ __forceinline__ int top_dist(uint32_t e) { return (int)(e >> 23); }

__device__ __forceinline__ void top_insert(TopK& t, uint32_t entry)
{
    const uint32_t dnew = entry >> 23;
    uint32_t carry = entry;
    bool shifting = false;   // stable: after the entries of equal distance, then everything moves down
#pragma unroll
    for (int k = 0; k < kTop; ++k) {
        const bool take = shifting || k >= t.n || (t.e[k] >> 23) > dnew;
        if (take) {
            const uint32_t x = t.e[k];
            t.e[k] = carry;
            carry = x;
            shifting = true;
        }
    }
    t.n = min(t.n + 1, 255);
}

// J2 / P1 give a MapPoint kSub adjacent lanes: sub-lane s scans window positions lo + s, lo + s +
// kSub, ...  Each keeps its own first kTop as 64-bit keys dist:9 | position:16 | entry low 23 bits
// (bin, octave, index), i.e. in (distance, visiting position) order, and the group merges its
// lists by kTop rounds of a min over the group's heads.  Same list as one sequential scan.
constexpr int kSub = 4;
struct TopK64 {
    unsigned long long e[kTop];
    int n;   // candidates this sub-lane saw (saturating)
};

__device__ __forceinline__ unsigned long long top_key(uint32_t entry, int p)
{
    return (unsigned long long)(entry >> 23) << 39 | (unsigned long long)p << 23 | (entry & 0x7FFFFFu);
}

__device__ __forceinline__ void top64_insert(TopK64& t, unsigned long long key)
{
    unsigned long long carry = key;
    bool shifting = false;   // positions only grow within a sub-lane: equal distances stay in visiting order
#pragma unroll
    for (int k = 0; k < kTop; ++k) {
        const bool take = shifting || k >= t.n || t.e[k] > key;
        if (take) {
            const unsigned long long x = t.e[k];
            t.e[k] = carry;
            carry = x;
            shifting = true;
        }
    }
    t.n = min(t.n + 1, 255);
}

__device__ __forceinline__ unsigned long long sub_min_u64(unsigned long long v)
{
#pragma unroll
    for (int o = 1; o < kSub; o <<= 1) {
        const unsigned long long y = __shfl_xor(v, o);
        v = y < v ? y : v;
    }
    return v;
}

// every lane of the group returns the merged list (entries as top_entry packs them)
__device__ __forceinline__ TopK top_merge(TopK64& t)
{
    int total = t.n;
#pragma unroll
    for (int o = 1; o < kSub; o <<= 1) total += __shfl_xor(total, o);
    TopK out;
    out.n = min(total, 255);
    int have = min(t.n, kTop);
#pragma unroll
    for (int r = 0; r < kTop; ++r) {
        const unsigned long long h = have > 0 ? t.e[0] : ~0ull;
        const unsigned long long m = sub_min_u64(h);
        if (have > 0 && h == m) {   // keys are unique (positions): only the owner pops
#pragma unroll
            for (int k = 0; k + 1 < kTop; ++k) t.e[k] = t.e[k + 1];
            --have;
        }
        out.e[r] = m == ~0ull ? 0u : (uint32_t)((m >> 39) << 23 | (m & 0x7FFFFFu));
    }
    return out;
}

// J2 result per MapPoint: the top-kTop list and the accept decision of its first entries
struct TopResult {
    uint32_t e[kTop];
    int n;        // candidates in the window (not claimed on entry), saturating
    int accept;   // the reference's accept test on the J2 best (and second)
};
using PjResult = TopResult;

__device__ __forceinline__ bool pj_accept(int bestDist, int bestLevel, int bestDist2, int bestLevel2, float nnratio)
{
    if (!(bestDist <= 100)) return false;   // TH_HIGH
    if (bestLevel == bestLevel2 && (float)bestDist > nnratio * (float)bestDist2) return false;
    return true;
}

__global__ __launch_bounds__(256) void k_pj_points(const orbx_keypoint* __restrict__ kps,
                                                   const uint8_t* __restrict__ desc, const float* __restrict__ uright,
                                                   const uint8_t* __restrict__ claimed, int cap,
                                                   const orbm_proj_point* __restrict__ pts,
                                                   const uint8_t* __restrict__ pdesc, const int* __restrict__ npts,
                                                   int pcap, orbm_proj_params P, const uint32_t* __restrict__ gkeys,
                                                   const int* __restrict__ gn, PjResult* __restrict__ res)
{
    const int f = blockIdx.y, m = blockIdx.x * (256 / kSub) + threadIdx.x / kSub, sub = threadIdx.x % kSub;
    if (m >= min(npts[f], pcap)) return;   // uniform over the kSub lanes of a MapPoint
    const size_t mo = (size_t)f * pcap + m;
    TopK64 T64;
    T64.n = 0;
#pragma unroll
    for (int k = 0; k < kTop; ++k) T64.e[k] = 0ull;
    int accept = 0;
    const orbm_proj_point M = pts[mo];
    bool scanned = false;
    if (M.flags & 1) {
        const uint32_t* keys = gkeys + (size_t)f * pj_grid_stride(cap);
        const PjWindow w = pj_window(M, P, keys, cap);
        if (w.ok) {
            scanned = true;
            const orbx_keypoint* K = kps + (size_t)f * cap;
            const float* U = uright + (size_t)f * cap;
            const uint8_t* C = claimed + (size_t)f * cap;
            const uint4* qd = reinterpret_cast<const uint4*>(pdesc + mo * 32);
            const uint4 q0 = qd[0], q1 = qd[1];
            for (int cx = w.cx0; cx <= w.cx1; ++cx) {   // src/ORBmatcher.cc:78-113, visiting order
                const int a = (int)keys[cap + cx * kPjRows + w.cy0], b = (int)keys[cap + cx * kPjRows + w.cy1 + 1];
                for (int p = a + sub; p < b; p += kSub) {
                    const int idx = pj_candidate(w, M, keys, p, K, U);
                    if (idx < 0 || C[idx]) continue;
                    const uint4* d = reinterpret_cast<const uint4*>(desc + ((size_t)f * cap + idx) * 32);
                    top64_insert(T64, top_key(top_entry(pj_ham(q0, q1, d[0], d[1]), 0, K[idx].octave, idx), p));
                }
            }
        }
    }
    const TopK T = top_merge(T64);   // whole group: `scanned` is uniform over it
    if (sub != 0) return;
    // the scan's best / second are the first two entries (multiset top two, first wins ties)
    if (scanned && T.n > 0)
        accept = pj_accept(top_dist(T.e[0]), top_oct(T.e[0]), T.n > 1 ? top_dist(T.e[1]) : 256,
                           T.n > 1 ? top_oct(T.e[1]) : -1, P.nnratio);
    PjResult R;
#pragma unroll
    for (int k = 0; k < kTop; ++k) R.e[k] = T.e[k];
    R.n = T.n;
    R.accept = accept;
    res[mo] = R;
}

__device__ __forceinline__ unsigned long long pj_wave_min_u64(unsigned long long v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long y = __shfl_xor(v, o);
        v = y < v ? y : v;
    }
    return v;
}

// ---- chunk-parallel, in-order replay of the reference's greedy loop (both searches) ----
// A claim made earlier in the call only removes candidates, so each MapPoint's result is a function
// of its J2 list and of the claims of the MapPoints before it.  A chunk of 64 MapPoints settles in
// rounds: every pending lane takes the first unclaimed entries of its list; the first lane whose
// choice collides with a claim of an earlier pending lane, or whose list ran out, stops the round;
// the lanes before it are final and commit together (last writer = the largest MapPoint index,
// claims, rotation bins); the next round starts at that lane, which now sees every claim before it.
// A lane whose list ran out searches its window again, wave-parallel, against the claims.
struct ReplayLds {
    int* mo;          // [cap] MapPoint assigned to the feature (last writer), -1
    uint32_t* bins;   // [cap] rotation bins of the matches that assigned the feature
    int* first;       // [cap] smallest pending lane claiming the feature in this round (64 = none)
    uint8_t* taken;   // [cap] claimed earlier in this call
    int* hist;        // [32] rotHist sizes
};

// kBig (frames of more than kReplayLdsCap features): `mo` is the frame's output row in global memory (the
// last-writer atomics go to it directly, and the final copy is in place), the rest stays in LDS: 9 bytes per
// feature instead of 13, so up to kProjMaxFeatures features fit a workgroup's 160 KiB.
constexpr int kReplayLdsCap = 8192;
template <bool kBig>
__device__ __forceinline__ ReplayLds replay_lds(int cap, int* mo_global)
{
    extern __shared__ int s_replay[];
    ReplayLds S;
    if constexpr (kBig) {
        S.mo = mo_global;
        S.bins = reinterpret_cast<uint32_t*>(s_replay);
        S.first = s_replay + cap;
        S.hist = s_replay + 2 * cap;
        S.taken = reinterpret_cast<uint8_t*>(s_replay + 2 * cap + 32);
    } else {
        S.mo = s_replay;
        S.bins = reinterpret_cast<uint32_t*>(s_replay + cap);
        S.first = s_replay + 2 * cap;
        S.hist = s_replay + 3 * cap;
        S.taken = reinterpret_cast<uint8_t*>(s_replay + 3 * cap + 32);
    }
    return S;
}

inline size_t replay_lds_bytes(int cap) { return cap > kReplayLdsCap ? (size_t)9 * cap + 128 : (size_t)13 * cap + 128; }

struct ReplayPick {
    int g, accept, bin;
};

template <bool kSecond, bool kRot, class ObsFn, class AcceptFn, class RescanFn>
__device__ __forceinline__ int replay_chunks(int n, int np, const TopResult* __restrict__ R, const ReplayLds& S,
                                             ObsFn obs_of, AcceptFn accept_of, RescanFn rescan)
{
    const int lane = threadIdx.x;
    for (int i = lane; i < n; i += 64) {
        S.mo[i] = -1;
        S.bins[i] = 0u;
        S.first[i] = 64;
        S.taken[i] = 0;
    }
    if (lane < 32) S.hist[lane] = 0;
    __syncthreads();
    int count = 0;
    for (int base = 0; base < np; base += 64) {
        const int m = base + lane;
        TopResult r{{0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u}, 0, 0};
        int obs = 0;
        if (m < np) {
            r = R[m];
            obs = obs_of(m);
        }
        // no candidate, or (single-best searches) a J2 best over the threshold: final, no match
        bool pending = r.n > 0 && (kSecond || r.accept);
        unsigned long long pend = __ballot(pending);
        while (pend) {
            int k1 = -1, k2 = -1;
            uint32_t c1 = 0u, c2 = 0u;
            bool out_of_list = false;
            if (pending) {
                const int lim = min(r.n, kTop);
#pragma unroll
                for (int k = 0; k < kTop; ++k) {
                    if (k < lim && (kSecond ? k2 < 0 : k1 < 0) && !S.taken[top_idx(r.e[k])]) {
                        if (k1 < 0) {
                            k1 = k;
                            c1 = r.e[k];
                        } else {
                            k2 = k;
                            c2 = r.e[k];
                        }
                    }
                }
                out_of_list = (kSecond ? k2 < 0 : k1 < 0) && r.n > kTop;
            }
            const bool acc = pending && !out_of_list && k1 >= 0 && accept_of(c1, k2 >= 0, c2);
            const bool claim = acc && obs;
            if (claim) atomicMin(&S.first[top_idx(c1)], lane);
            __syncthreads();
            bool stop = pending && out_of_list;
            if (pending && !out_of_list && k1 >= 0)
                stop = S.first[top_idx(c1)] < lane || (kSecond && k2 >= 0 && S.first[top_idx(c2)] < lane);
            __syncthreads();
            if (claim) S.first[top_idx(c1)] = 64;
            const unsigned long long stops = __ballot(stop);
            const int j0 = stops ? __builtin_ctzll(stops) : 64;
            const bool commit = pending && lane < j0;
            if (commit && acc) {
                const int g = top_idx(c1);
                atomicMax(&S.mo[g], m);   // F.mvpMapPoints[bestIdx] = pMP, in MapPoint order
                if (kRot) {
                    atomicOr(&S.bins[g], 1u << top_bin(c1));
                    atomicAdd(&S.hist[top_bin(c1)], 1);
                }
                if (obs) S.taken[g] = 1;
            }
            count += __popcll(__ballot(commit && acc));
            if (commit) pending = false;
            __syncthreads();
            if (j0 < 64 && __builtin_amdgcn_readlane((int)out_of_list, j0)) {   // wave-uniform
                const ReplayPick pk = rescan(base + j0, S.taken);
                if (pk.accept) {
                    if (lane == 0) {
                        atomicMax(&S.mo[pk.g], base + j0);
                        if (kRot) {
                            atomicOr(&S.bins[pk.g], 1u << pk.bin);
                            atomicAdd(&S.hist[pk.bin], 1);
                        }
                        if (__builtin_amdgcn_readlane(obs, j0)) S.taken[pk.g] = 1;
                    }
                    ++count;
                }
                if (lane == j0) pending = false;
                __syncthreads();
            }
            pend = __ballot(pending);
        }
    }
    __syncthreads();
    return count;
}

template <bool kBig>
__global__ __launch_bounds__(64) void k_pj_resolve(const orbx_keypoint* __restrict__ kps,
                                                   const uint8_t* __restrict__ desc, const float* __restrict__ uright,
                                                   const uint8_t* __restrict__ claimed, const int* __restrict__ counts,
                                                   int cap, const orbm_proj_point* __restrict__ pts,
                                                   const uint8_t* __restrict__ pdesc, const int* __restrict__ npts,
                                                   int pcap, orbm_proj_params P, const uint32_t* __restrict__ gkeys,
                                                   const int* __restrict__ gn, const PjResult* __restrict__ res,
                                                   int* __restrict__ match, int* __restrict__ nmatches)
{
    const int f = blockIdx.x, lane = threadIdx.x;
    const int n = min(counts[f], cap), np = min(npts[f], pcap);
    int* Mo = match + (size_t)f * cap;
    const ReplayLds S = replay_lds<kBig>(cap, Mo);
    const uint32_t* keys = gkeys + (size_t)f * pj_grid_stride(cap);
    const orbx_keypoint* K = kps + (size_t)f * cap;
    const float* U = uright + (size_t)f * cap;
    const uint8_t* C = claimed + (size_t)f * cap;
    const orbm_proj_point* Pf = pts + (size_t)f * pcap;
    auto obs_of = [&](int m) { return (Pf[m].flags & 2) ? 1 : 0; };
    auto accept_of = [&](uint32_t c1, bool has2, uint32_t c2) {
        return pj_accept(top_dist(c1), top_oct(c1), has2 ? top_dist(c2) : 256, has2 ? top_oct(c2) : -1, P.nnratio);
    };
    // search again against the current claims: best = first min of (dist, position), second = first
    // min of the rest (the sequential scan's result)
    auto rescan = [&](int m, const uint8_t* taken) {
        const orbm_proj_point Mp = Pf[m];
        const PjWindow w = pj_window(Mp, P, keys, cap);
        const uint4* qd = reinterpret_cast<const uint4*>(pdesc + ((size_t)f * pcap + m) * 32);
        const uint4 q0 = qd[0], q1 = qd[1];
        unsigned long long b1 = ~0ull, b2 = ~0ull;
        for (int p0 = w.lo; p0 < w.hi; p0 += 64) {
            const int p = p0 + lane;
            unsigned long long key = ~0ull;
            if (p < w.hi) {
                const int idx = pj_candidate(w, Mp, keys, p, K, U);
                if (idx >= 0 && !C[idx] && !taken[idx]) {
                    const uint4* d = reinterpret_cast<const uint4*>(desc + ((size_t)f * cap + idx) * 32);
                    key = ((unsigned long long)pj_ham(q0, q1, d[0], d[1]) << 32) | ((unsigned long long)p << 16) |
                          (unsigned)idx;
                }
            }
            const unsigned long long c1 = pj_wave_min_u64(key);
            const unsigned long long c2 = pj_wave_min_u64(key == c1 ? ~0ull : key);
            if (c1 < b1) {   // merge: the multiset top two by (dist, position)
                b2 = min(b1, c2);
                b1 = c1;
            } else {
                b2 = min(b2, c1);
            }
        }
        ReplayPick pk{-1, 0, 0};
        if (b1 != ~0ull) {
            pk.g = (int)(b1 & 0xFFFF);
            const int bd2 = b2 == ~0ull ? 256 : (int)(b2 >> 32);
            const int bl2 = b2 == ~0ull ? -1 : K[(int)(b2 & 0xFFFF)].octave;
            pk.accept = pj_accept((int)(b1 >> 32), K[pk.g].octave, bd2, bl2, P.nnratio);
        }
        return pk;
    };
    const int count = replay_chunks<true, false>(n, np, res + (size_t)f * pcap, S, obs_of, accept_of, rescan);
    if constexpr (!kBig)
        for (int i = lane; i < n; i += 64) Mo[i] = S.mo[i];
    if (lane == 0) nmatches[f] = count;
}

size_t proj_scratch_bytes(int nframes, int cap, int pcap)
{
    return (size_t)nframes * pj_grid_stride(cap) * 4 + (size_t)nframes * 4 + (size_t)nframes * pcap * sizeof(PjResult) + 256;
}

void launch_proj(const orbx_keypoint* kps, const uint8_t* desc, const float* uright, const uint8_t* claimed,
                 const int* counts, int nframes, int cap, const orbm_proj_point* pts, const uint8_t* pdesc,
                 const int* npts, int pcap, const orbm_proj_params& P, void* scratch, int* match, int* nmatches,
                 hipStream_t s)
{
    uint32_t* gkeys = (uint32_t*)scratch;
    int* gn = (int*)(gkeys + (size_t)nframes * pj_grid_stride(cap));
    PjResult* res = (PjResult*)(((uintptr_t)(gn + nframes) + 15) & ~(uintptr_t)15);
    launch_pj_grid(kps, counts, nframes, cap, P.min_x, P.min_y, P.grid_w_inv, P.grid_h_inv, gkeys, gn, s);
    hipLaunchKernelGGL(k_pj_points, dim3((pcap + 256 / kSub - 1) / (256 / kSub), nframes), dim3(256), 0, s, kps, desc,
                       uright, claimed, cap, pts, pdesc, npts, pcap, P, gkeys, gn, res);
    auto resolve = [&](auto kern) {
        hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)replay_lds_bytes(cap));
        hipLaunchKernelGGL(kern, dim3(nframes), dim3(64), replay_lds_bytes(cap), s, kps, desc, uright, claimed, counts,
                           cap, pts, pdesc, npts, pcap, P, gkeys, gn, res, match, nmatches);
    };
    if (cap > kReplayLdsCap) resolve(k_pj_resolve<true>);
    else resolve(k_pj_resolve<false>);
}

// =====================================================================================
// Pose-projection searches: SearchByProjection(CurrentFrame, LastFrame) (:1396-1538),
// SearchByProjection(CurrentFrame, pKF, sAlreadyFound) (:1540-1667), SearchByProjection(pKF,
// Scw, ...) (:290-403), Fuse(pKF, ...) (:893-1043), Fuse(pKF, Scw, ...) (:1045-1168).
//
// J1 k_pj_grid     as above
// J2 k_ps_points   one lane per MapPoint: project with the frame pose, scan the window in
//                  GetFeaturesInArea order against the claims on entry (first minimum).
//                  The Fuse overloads claim nothing during the search: they finish here.
// J3 k_ps_resolve  one wave per frame replays the three searches in MapPoint order with
//                  replay_chunks (above), then the rotation histogram from per-feature bin
//                  masks in LDS.
// Float arithmetic is oracle/orbref.c proj_* operation for operation (no contraction in this
// file; the reference's GCC -march=native FMAs are explicit).
// =====================================================================================

__device__ __forceinline__ int ps_x86_int(double v)   // cvttsd2si: NaN / out of range -> INT_MIN
{
    return (v >= -2147483648.0 && v < 2147483648.0) ? (int)v : (-2147483647 - 1);
}

__device__ __forceinline__ float ps_row(const float* r, int stride, float x, float y, float z)
{
    return (r[0] * x + r[stride] * y) + r[2 * stride] * z;   // OpenCV 3.x gemm small-matrix order
}

struct PsCam {
    float R[9], t[3], Ow[3];
    int fwd, bwd;
};

__device__ __forceinline__ PsCam ps_camera(int mode, const float* __restrict__ pose, const orbm_pose_params& P)
{
    PsCam c;
    if (mode == ORBM_PROJ_SIM3 || mode == ORBM_FUSE_SIM3) {   // Decompose Scw (:298-303)
        double d = 0.0;
        for (int k = 0; k < 3; ++k) d += (double)pose[k] * (double)pose[k];
        const float scw = (float)__builtin_sqrt(d);
        const float s = (float)(1.0 / (double)scw);
        for (int r = 0; r < 3; ++r) {
            for (int k = 0; k < 3; ++k) c.R[3 * r + k] = pose[4 * r + k] * s + 0.0f;
            c.t[r] = pose[4 * r + 3] * s + 0.0f;
        }
    } else {
        for (int r = 0; r < 3; ++r) {
            for (int k = 0; k < 3; ++k) c.R[3 * r + k] = pose[4 * r + k];
            c.t[r] = pose[4 * r + 3];
        }
    }
    for (int r = 0; r < 3; ++r) c.Ow[r] = -ps_row(c.R + r, 3, c.t[0], c.t[1], c.t[2]);   // -Rcw.t()*tcw
    c.fwd = c.bwd = 0;
    if (mode == ORBM_PROJ_LAST_FRAME) {   // tlc = Rlw*twc+tlw (:1409-1417)
        const float tlc2 = ps_row(pose + 20, 1, c.Ow[0], c.Ow[1], c.Ow[2]) + pose[23];
        c.fwd = tlc2 > P.b && !P.mono;
        c.bwd = -tlc2 > P.b && !P.mono;
    }
    return c;
}

struct PsWin {
    float u, v, r, ur;
    int minLevel, maxLevel, cx0, cx1, cy0, cy1, lo, hi;
};

// MapPoint::PredictScale (src/MapPoint.cc:385-417)
__device__ __forceinline__ int ps_predict_scale(float max_dist, float dist, const orbm_pose_params& P)
{
    const float ratio = max_dist / dist;
    int n = ps_x86_int(__builtin_ceil(log((double)ratio) / (double)P.log_scale));
    if (n < 0) n = 0;
    else if (n >= P.nlevels) n = P.nlevels - 1;
    return n;
}

// the per-MapPoint part before GetFeaturesInArea; false where the reference `continue`s
template <int MODE>
__device__ __forceinline__ bool ps_project(const PsCam& c, const orbm_map_point& M, const orbm_pose_params& P,
                                           PsWin& w)
{
    const float X = M.x, Y = M.y, Z = M.z;
    const float xc = ps_row(c.R, 1, X, Y, Z) + c.t[0];
    const float yc = ps_row(c.R + 3, 1, X, Y, Z) + c.t[1];
    const float zc = ps_row(c.R + 6, 1, X, Y, Z) + c.t[2];
    w.ur = 0.0f;
    if (MODE == ORBM_PROJ_LAST_FRAME || MODE == ORBM_PROJ_KEYFRAME) {
        const float invzc = (float)(1.0 / (double)zc);
        if (MODE == ORBM_PROJ_LAST_FRAME && invzc < 0) return false;
        const float u = __builtin_fmaf(P.fx * xc, invzc, P.cx);   // fx*xc*invzc+cx
        const float v = __builtin_fmaf(P.fy * yc, invzc, P.cy);
        if (u < P.min_x || u > P.max_x) return false;
        if (v < P.min_y || v > P.max_y) return false;
        w.u = u;
        w.v = v;
        if (MODE == ORBM_PROJ_LAST_FRAME) {   // :1446-1458
            const int L = M.octave & 15;
            w.r = P.th * P.scale[L];
            if (c.fwd) { w.minLevel = L; w.maxLevel = -1; }
            else if (c.bwd) { w.minLevel = 0; w.maxLevel = L; }
            else { w.minLevel = L - 1; w.maxLevel = L + 1; }
            w.ur = __builtin_fmaf(-P.bf, invzc, u);   // u - mbf*invzc
            return true;
        }
    } else {
        if (zc < 0.0f) return false;
        const float invz = MODE == ORBM_FUSE_SIM3 ? (float)(1.0 / (double)zc) : 1.0f / zc;
        const float x = xc * invz, y = yc * invz;
        const float u = __builtin_fmaf(P.fx, x, P.cx);
        const float v = __builtin_fmaf(P.fy, y, P.cy);
        if (!(u >= P.min_x && u < P.max_x && v >= P.min_y && v < P.max_y)) return false;   // IsInImage
        w.u = u;
        w.v = v;
        if (MODE == ORBM_FUSE) w.ur = __builtin_fmaf(-P.bf, invz, u);
    }
    const float maxD = 1.2f * M.max_dist, minD = 0.8f * M.min_dist;
    const float PO0 = X - c.Ow[0], PO1 = Y - c.Ow[1], PO2 = Z - c.Ow[2];
    double s = 0.0;
    s += (double)PO0 * (double)PO0;
    s += (double)PO1 * (double)PO1;
    s += (double)PO2 * (double)PO2;
    const float dist = (float)__builtin_sqrt(s);   // cv::norm(PO)
    if (dist < minD || dist > maxD) return false;
    if (MODE != ORBM_PROJ_KEYFRAME) {   // PO.dot(Pn) < 0.5*dist
        double dot = 0.0;
        dot += (double)PO0 * (double)M.nx;
        dot += (double)PO1 * (double)M.ny;
        dot += (double)PO2 * (double)M.nz;
        if (dot < 0.5 * (double)dist) return false;
    }
    const int L = ps_predict_scale(M.max_dist, dist, P);
    w.r = P.th * P.scale[L & 15];
    w.minLevel = L - 1;
    w.maxLevel = MODE == ORBM_PROJ_KEYFRAME ? L + 1 : L;
    return true;
}

__device__ __forceinline__ bool ps_window(PsWin& w, const orbm_pose_params& P, const uint32_t* keys, int cap)
{
    const int cx0 = max(0, ps_x86_int(floorf((w.u - P.min_x - w.r) * P.grid_w_inv)));
    if (cx0 >= kPjCols) return false;
    const int cx1 = min(kPjCols - 1, ps_x86_int(ceilf((w.u - P.min_x + w.r) * P.grid_w_inv)));
    if (cx1 < 0) return false;
    w.cy0 = max(0, ps_x86_int(floorf((w.v - P.min_y - w.r) * P.grid_h_inv)));
    if (w.cy0 >= kPjRows) return false;
    w.cy1 = min(kPjRows - 1, ps_x86_int(ceilf((w.v - P.min_y + w.r) * P.grid_h_inv)));
    if (w.cy1 < 0) return false;
    w.cx0 = cx0;
    w.cx1 = cx1;
    w.lo = (int)keys[cap + cx0 * kPjRows];
    w.hi = (int)keys[cap + (cx1 + 1) * kPjRows];
    return true;
}

// feature index at key position p if it passes the mode's window / level / stereo tests
template <int MODE>
__device__ __forceinline__ int ps_candidate(const PsWin& w, const uint32_t* keys, int p, const orbx_keypoint* K,
                                            const float* U, const orbm_pose_params& P)
{
    const uint32_t key = keys[p];
    const int iy = (int)(key >> 16) % kPjRows;
    if (iy < w.cy0 || iy > w.cy1) return -1;
    const int idx = (int)(key & 0xFFFF);
    const orbx_keypoint kp = K[idx];
    if (kp.octave < w.minLevel) return -1;
    if (w.maxLevel >= 0 && kp.octave > w.maxLevel) return -1;
    const float distx = kp.x - w.u, disty = kp.y - w.v;
    if (!(fabsf(distx) < w.r && fabsf(disty) < w.r)) return -1;
    if (MODE == ORBM_PROJ_LAST_FRAME) {   // :1475-1481
        const float ur = U[idx];
        if (ur > 0 && fabsf(w.ur - ur) > w.r) return -1;
    }
    if (MODE == ORBM_FUSE) {   // :982-1006
        const float ur = U[idx];
        const float ex = w.u - kp.x, ey = w.v - kp.y;
        const float is2 = P.inv_sigma2[kp.octave & 15];
        if (ur >= 0) {
            const float er = w.ur - ur;
            const float e2 = __builtin_fmaf(er, er, __builtin_fmaf(ex, ex, ey * ey));
            if ((double)(e2 * is2) > 7.8) return -1;
        } else {
            const float e2 = __builtin_fmaf(ex, ex, ey * ey);
            if ((double)(e2 * is2) > 5.99) return -1;
        }
    }
    return idx;
}

template <int MODE>
__device__ __forceinline__ int ps_threshold(const orbm_pose_params& P)
{
    return MODE == ORBM_PROJ_LAST_FRAME ? 100 : (MODE == ORBM_PROJ_KEYFRAME ? P.orb_dist : 50);   // TH_HIGH / TH_LOW
}

__device__ __forceinline__ int ps_rot_bin(float a1, float a2)
{
    const float factor = 1.0f / 30;   // 1/HISTO_LENGTH
    float rot = a1 - a2;
    if (rot < 0.0f) rot += 360.0f;
    int bin = (int)roundf(rot * factor);
    if (bin == 30) bin = 0;
    return bin;
}

using PsResult = TopResult;   // bins filled for the rotation-checked searches

template <int MODE>
__global__ __launch_bounds__(256) void k_ps_points(const orbx_keypoint* __restrict__ kps,
                                                   const uint8_t* __restrict__ desc, const float* __restrict__ uright,
                                                   const uint8_t* __restrict__ claimed, int cap,
                                                   const float* __restrict__ pose, const orbm_map_point* __restrict__ pts,
                                                   const uint8_t* __restrict__ pdesc, const int* __restrict__ npts,
                                                   int pcap, orbm_pose_params P, const uint32_t* __restrict__ gkeys,
                                                   const int* __restrict__ gn, PsResult* __restrict__ res,
                                                   int* __restrict__ match, int* __restrict__ nmatches)
{
    constexpr bool kSearch = MODE <= ORBM_PROJ_SIM3;
    const int f = blockIdx.y, m = blockIdx.x * (256 / kSub) + threadIdx.x / kSub, sub = threadIdx.x % kSub;
    if (m >= min(npts[f], pcap)) return;   // uniform over the kSub lanes of a MapPoint
    const size_t mo = (size_t)f * pcap + m;
    int bestIdx = -1, accept = 0;
    TopK64 T64;
    T64.n = 0;
#pragma unroll
    for (int k = 0; k < kTop; ++k) T64.e[k] = 0ull;
    unsigned long long best = ~0ull;   // Fuse: first minimum as (dist, position, index)
    const orbm_map_point M = pts[mo];
    bool scanned = false;
    if (M.flags & 1) {
        const PsCam c = ps_camera(MODE, pose + (size_t)f * 24, P);
        const uint32_t* keys = gkeys + (size_t)f * pj_grid_stride(cap);
        PsWin w;
        if (ps_project<MODE>(c, M, P, w) && ps_window(w, P, keys, cap)) {
            scanned = true;
            const orbx_keypoint* K = kps + (size_t)f * cap;
            const float* U = uright + (size_t)f * cap;
            const uint8_t* C = claimed + (size_t)f * cap;
            const uint4* qd = reinterpret_cast<const uint4*>(pdesc + mo * 32);
            const uint4 q0 = qd[0], q1 = qd[1];
            const bool bins = kSearch && (MODE == ORBM_PROJ_LAST_FRAME || MODE == ORBM_PROJ_KEYFRAME) && P.check_ori;
            for (int cx = w.cx0; cx <= w.cx1; ++cx) {   // GetFeaturesInArea order, rows cy0..cy1 only
                const int a = (int)keys[cap + cx * kPjRows + w.cy0], b = (int)keys[cap + cx * kPjRows + w.cy1 + 1];
                for (int p = a + sub; p < b; p += kSub) {
                    const int idx = ps_candidate<MODE>(w, keys, p, K, U, P);
                    if (idx < 0 || (kSearch && C[idx])) continue;
                    const uint4* d = reinterpret_cast<const uint4*>(desc + ((size_t)f * cap + idx) * 32);
                    const int dist = pj_ham(q0, q1, d[0], d[1]);
                    if (kSearch) {
                        top64_insert(T64, top_key(top_entry(dist, bins ? ps_rot_bin(M.angle, K[idx].angle) : 0, 0,
                                                            idx),
                                                  p));
                    } else {
                        const unsigned long long key =
                            (unsigned long long)dist << 32 | (unsigned long long)p << 16 | (unsigned)idx;
                        best = key < best ? key : best;
                    }
                }
            }
        }
    }
    TopK T;
    if (kSearch) {
        T = top_merge(T64);   // whole group: `scanned` is uniform over it
        if (scanned && T.n > 0) {
            bestIdx = top_idx(T.e[0]);
            accept = top_dist(T.e[0]) <= ps_threshold<MODE>(P);
        }
    } else {
        best = sub_min_u64(best);
        if (best != ~0ull) {
            bestIdx = (int)(best & 0xFFFF);
            accept = (int)(best >> 32) <= ps_threshold<MODE>(P);
        }
    }
    if (sub != 0) return;
    if (kSearch) {
        PsResult R;
#pragma unroll
        for (int k = 0; k < kTop; ++k) R.e[k] = T.e[k];
        R.n = T.n;
        R.accept = accept;
        res[mo] = R;
    } else {
        match[mo] = accept ? bestIdx : -1;
        if (accept) atomicAdd(&nmatches[f], 1);
    }
}

template <int MODE, bool kBig>
__global__ __launch_bounds__(64) void k_ps_resolve(const orbx_keypoint* __restrict__ kps,
                                                   const uint8_t* __restrict__ desc, const float* __restrict__ uright,
                                                   const uint8_t* __restrict__ claimed, const int* __restrict__ counts,
                                                   int cap, const float* __restrict__ pose,
                                                   const orbm_map_point* __restrict__ pts,
                                                   const uint8_t* __restrict__ pdesc, const int* __restrict__ npts,
                                                   int pcap, orbm_pose_params P, const uint32_t* __restrict__ gkeys,
                                                   const int* __restrict__ gn, const PsResult* __restrict__ res,
                                                   int* __restrict__ match, int* __restrict__ nmatches)
{
    constexpr bool kRotMode = MODE == ORBM_PROJ_LAST_FRAME || MODE == ORBM_PROJ_KEYFRAME;
    const int f = blockIdx.x, lane = threadIdx.x;
    const int n = min(counts[f], cap), np = min(npts[f], pcap);
    int* Mo = match + (size_t)f * cap;
    const ReplayLds S = replay_lds<kBig>(cap, Mo);
    const uint32_t* keys = gkeys + (size_t)f * pj_grid_stride(cap);
    const orbx_keypoint* K = kps + (size_t)f * cap;
    const float* U = uright + (size_t)f * cap;
    const uint8_t* C = claimed + (size_t)f * cap;
    const orbm_map_point* Pf = pts + (size_t)f * pcap;
    const PsCam cam = ps_camera(MODE, pose + (size_t)f * 24, P);
    const bool rot = kRotMode && P.check_ori;
    const int thr = ps_threshold<MODE>(P);
    // LAST_FRAME claims a feature only for a MapPoint with Observations() > 0 (:1471-1473); the
    // other searches skip every feature already assigned (:1609-1610, :375-376)
    auto obs_of = [&](int m) { return MODE != ORBM_PROJ_LAST_FRAME || (Pf[m].flags & 2) ? 1 : 0; };
    auto accept_of = [&](uint32_t c1, bool, uint32_t) { return top_dist(c1) <= thr; };
    auto rescan = [&](int m, const uint8_t* taken) {
        const orbm_map_point Mp = Pf[m];
        PsWin w;
        ps_project<MODE>(cam, Mp, P, w);   // true and non-empty: J2 found candidates in it
        ps_window(w, P, keys, cap);
        const uint4* qd = reinterpret_cast<const uint4*>(pdesc + ((size_t)f * pcap + m) * 32);
        const uint4 q0 = qd[0], q1 = qd[1];
        unsigned long long b1 = ~0ull;
        for (int p0 = w.lo; p0 < w.hi; p0 += 64) {
            const int p = p0 + lane;
            unsigned long long key = ~0ull;
            if (p < w.hi) {
                const int idx = ps_candidate<MODE>(w, keys, p, K, U, P);
                if (idx >= 0 && !C[idx] && !taken[idx]) {
                    const uint4* d = reinterpret_cast<const uint4*>(desc + ((size_t)f * cap + idx) * 32);
                    key = ((unsigned long long)pj_ham(q0, q1, d[0], d[1]) << 32) | ((unsigned long long)p << 16) |
                          (unsigned)idx;
                }
            }
            const unsigned long long c1 = pj_wave_min_u64(key);
            b1 = c1 < b1 ? c1 : b1;
        }
        ReplayPick pk{-1, 0, 0};
        if (b1 != ~0ull) {
            pk.g = (int)(b1 & 0xFFFF);
            pk.accept = (int)(b1 >> 32) <= thr;
            if (rot) pk.bin = ps_rot_bin(Mp.angle, K[pk.g].angle);
        }
        return pk;
    };
    int count = rot ? replay_chunks<false, true>(n, np, res + (size_t)f * pcap, S, obs_of, accept_of, rescan)
                    : replay_chunks<false, false>(n, np, res + (size_t)f * pcap, S, obs_of, accept_of, rescan);
    uint32_t drop = 0u;   // the bins outside the three maxima
    if (rot) {            // ComputeThreeMaxima (:1679-1723); every match in another bin is undone
        int ind1 = -1, ind2 = -1, ind3 = -1, max1 = 0, max2 = 0, max3 = 0;
        for (int i = 0; i < 30; ++i) {
            const int h = S.hist[i];
            if (h > max1) { max3 = max2; max2 = max1; max1 = h; ind3 = ind2; ind2 = ind1; ind1 = i; }
            else if (h > max2) { max3 = max2; max2 = h; ind3 = ind2; ind2 = i; }
            else if (h > max3) { max3 = h; ind3 = i; }
        }
        if ((float)max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
        else if ((float)max3 < 0.1f * (float)max1) { ind3 = -1; }
        drop = 0x3FFFFFFFu;
        if (ind1 >= 0) drop &= ~(1u << ind1);
        if (ind2 >= 0) drop &= ~(1u << ind2);
        if (ind3 >= 0) drop &= ~(1u << ind3);
        for (int i = 0; i < 30; ++i)
            if ((drop >> i) & 1u) count -= S.hist[i];
    }
    for (int i = lane; i < n; i += 64) Mo[i] = (S.bins[i] & drop) ? -2 : S.mo[i];   // NULL-ed by the filter (in place when kBig)
    if (lane == 0) nmatches[f] = count;
}

size_t pose_scratch_bytes(int nframes, int cap, int pcap)
{
    return (size_t)nframes * pj_grid_stride(cap) * 4 + (size_t)nframes * 4 + (size_t)nframes * pcap * sizeof(PsResult) + 256;
}

template <int MODE>
static void ps_launch(const orbx_keypoint* kps, const uint8_t* desc, const float* uright, const uint8_t* claimed,
                      const int* counts, int nframes, int cap, const float* pose, const orbm_map_point* pts,
                      const uint8_t* pdesc, const int* npts, int pcap, const orbm_pose_params& P,
                      const uint32_t* gkeys, const int* gn, PsResult* res, int* match, int* nmatches,
                      hipStream_t s)
{
    if (MODE >= ORBM_FUSE) hipMemsetAsync(nmatches, 0, sizeof(int) * (size_t)nframes, s);
    hipLaunchKernelGGL(k_ps_points<MODE>, dim3((pcap + 256 / kSub - 1) / (256 / kSub), nframes), dim3(256), 0, s,
                       kps, desc, uright,
                       claimed, cap, pose, pts, pdesc, npts, pcap, P, gkeys, gn, res, match, nmatches);
    if (MODE <= ORBM_PROJ_SIM3) {
        auto resolve = [&](auto kern) {
            hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)replay_lds_bytes(cap));
            hipLaunchKernelGGL(kern, dim3(nframes), dim3(64), replay_lds_bytes(cap), s, kps, desc, uright, claimed,
                               counts, cap, pose, pts, pdesc, npts, pcap, P, gkeys, gn, res, match, nmatches);
        };
        if (cap > kReplayLdsCap) resolve(k_ps_resolve<MODE, true>);
        else resolve(k_ps_resolve<MODE, false>);
    }
}

void launch_pose_search(int mode, const orbx_keypoint* kps, const uint8_t* desc, const float* uright,
                        const uint8_t* claimed, const int* counts, int nframes, int cap, const float* pose,
                        const orbm_map_point* pts, const uint8_t* pdesc, const int* npts, int pcap,
                        const orbm_pose_params& P, void* scratch, int* match, int* nmatches, hipStream_t s)
{
    uint32_t* gkeys = (uint32_t*)scratch;
    int* gn = (int*)(gkeys + (size_t)nframes * pj_grid_stride(cap));
    PsResult* res = (PsResult*)(((uintptr_t)(gn + nframes) + 15) & ~(uintptr_t)15);
    launch_pj_grid(kps, counts, nframes, cap, P.min_x, P.min_y, P.grid_w_inv, P.grid_h_inv, gkeys, gn, s);
    switch (mode) {
    case ORBM_PROJ_LAST_FRAME:
        ps_launch<ORBM_PROJ_LAST_FRAME>(kps, desc, uright, claimed, counts, nframes, cap, pose, pts, pdesc, npts, pcap,
                                        P, gkeys, gn, res, match, nmatches, s);
        break;
    case ORBM_PROJ_KEYFRAME:
        ps_launch<ORBM_PROJ_KEYFRAME>(kps, desc, uright, claimed, counts, nframes, cap, pose, pts, pdesc, npts, pcap,
                                      P, gkeys, gn, res, match, nmatches, s);
        break;
    case ORBM_PROJ_SIM3:
        ps_launch<ORBM_PROJ_SIM3>(kps, desc, uright, claimed, counts, nframes, cap, pose, pts, pdesc, npts, pcap, P,
                                  gkeys, gn, res, match, nmatches, s);
        break;
    case ORBM_FUSE:
        ps_launch<ORBM_FUSE>(kps, desc, uright, claimed, counts, nframes, cap, pose, pts, pdesc, npts, pcap, P, gkeys,
                             gn, res, match, nmatches, s);
        break;
    default:
        ps_launch<ORBM_FUSE_SIM3>(kps, desc, uright, claimed, counts, nframes, cap, pose, pts, pdesc, npts, pcap, P,
                                  gkeys, gn, res, match, nmatches, s);
        break;
    }
}

}  // namespace orbx
