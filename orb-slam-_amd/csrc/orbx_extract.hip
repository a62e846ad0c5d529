// gfx950 kernels of the ORB extractor (ORB_SLAM2::ORBextractor::operator(),
// src/ORBextractor.cc:1248-1334).  Integer/bitwise path: no MFMA.
//
//   K1 k_pyramid_level  ComputePyramid, src/ORBextractor.cc:1342-1377
//   K2 k_fast_cells     per-cell FAST-9 + NMS + threshold retry, :952-1000
//   K3 k_quadtree       DistributeOctTree, :644-907 (one workgroup per frame x level)
//   K4 k_describe       IC_Angle + GaussianBlur + rBRIEF + scale/pack,
//                       :84-128, :1300-1332, :141-192
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "orbx_kernels.hpp"
#include "orbx_math.hpp"

namespace orbx {

__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The dynamic LDS of a kernel without static LDS, as the constant address 0.  An extern __shared__ array's
// address is a symbol the compiler adds to every LDS address it forms from a runtime offset (one v_add of 0
// each, and registers to hold the sums: k_quadtree<256,4> and <512,16> spilled 16 and 8 bytes per lane to
// scratch with it).  The backend lowers __builtin_amdgcn_groupstaticsize (the static LDS size) to a
// constant, so base plus offset folds into the instructions; the check below costs one scalar compare of
// two constants per wave.
__device__ __forceinline__ uint8_t* dyn_lds()
{
    const uint32_t base = __builtin_amdgcn_groupstaticsize();
    if (base != 0u) __builtin_trap();   // a kernel with static LDS would need the rounded offset and a larger launch size
    return (uint8_t*)(__attribute__((address_space(3))) uint8_t*)(uintptr_t)base;
}

__device__ __forceinline__ int lanes_below(unsigned long long mask)
{
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                          __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

__device__ __forceinline__ const uint8_t* level_base(const FramePtrs& P, const Geometry* G, int f, int l,
                                                     int& pitch)
{
    if (l == 0) {
        pitch = P.in_pitch;
        return P.in + (size_t)f * P.in_fstride;
    }
    pitch = G->lv[l].pitch;
    return P.pyr + (size_t)f * P.pyr_fstride + G->lv[l].pyr_off;
}

typedef unsigned short ushort2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ ushort2_t as_us2(uint32_t v)
{
    ushort2_t r;
    r.x = (unsigned short)(v & 0xFFFF);
    r.y = (unsigned short)(v >> 16);
    return r;
}

// ---------------------------------------------------------------------------
// K1: level l from level l-1, cv::resize INTER_LINEAR u8 fixed point
// (11-bit coefficients, 22-bit vertical rounding) — SURVEY.md A.2.
// Coefficient tables are built on the host exactly like OpenCV builds them.
// ---------------------------------------------------------------------------
#ifndef ORBX_PYR_ROWS
#define ORBX_PYR_ROWS 12   // output rows per block (round 4, 768-frame steps: 12 -> 267.8k / 267.9k against 8 ->
                           // 265.6k / 266.1k frames/s on one box, launches within 2 us of each other; 16 -> 267.0k)
#endif
#ifndef ORBX_PYR_NT
#define ORBX_PYR_NT 256
#endif
constexpr int kPyrRows = ORBX_PYR_ROWS;
constexpr int kPyrNT = ORBX_PYR_NT;   // threads per pyramid workgroup

// SURVEY.md A.2's SSE2 vertical pass (ORBX_RESIZE_SSE2): VResizeLinearVec_32s8u's
// ((mulhi16(h0 >> 4, b0) + mulhi16(h1 >> 4, b1) + 2) >> 2) of the horizontal sums h0, h1 (h >> 4 <= 32640 and
// b <= 2048 are non-negative: mulhi16 is the plain (x * b) >> 16, every product a 24 x 24-bit multiply)
__device__ __forceinline__ uint32_t rz_sse2(uint32_t h0, uint32_t h1, uint32_t b0, uint32_t b1)
{
    const uint32_t v = ((__umul24(h0 >> 4, b0) >> 16) + (__umul24(h1 >> 4, b1) >> 16) + 2u) >> 2;
    return min(v, 255u);
}

// kA: every staged source row starts 4-byte aligned in LDS (source pitch and base multiples of 4, always
// so for levels >= 1), so a lane's realignment shift is the same on every row.  kRM: ORBX_RESIZE_* (columns
// [0, rz_simd_end) of an ORBX_RESIZE_SSE2 level take rz_sse2; rz_simd_end is a multiple of 4, so a 4-column
// group takes one form)
template <bool kWin, bool kA, int kRM>
__global__ __launch_bounds__(kPyrNT) void k_pyramid_level(const Geometry* __restrict__ G, FramePtrs P, int l,
                                                       const int2* __restrict__ xtab,
                                                       const int2* __restrict__ ytab, int lp)
{
    // A block makes kPyrRows output rows of one frame.  The source rows they need arrive in LDS by
    // LDS-DMA (global_load_lds_dwordx4): row r is the 16-byte aligned run of lp bytes that holds it,
    // at LDS byte r * lp, so its pixel x sits at r * lp + sh_r + x with sh_r = its start address & 15
    // (0 on every row of levels >= 1, whose pitch is a multiple of 64).  A chunk is fetched only if it
    // holds a byte of its row: it then lies in the row's own 16-byte aligned span, which cannot cross a
    // page boundary, so no read leaves the caller's allocation.  (Round 2: aligned dword loads realigned
    // by alignbyte and stored to LDS, about 14 VALU per staged dword.)
    extern __shared__ __attribute__((aligned(16))) uint32_t s_src[];
    const int lb = xcd_block(blockIdx.y + blockIdx.z * gridDim.y, gridDim.y * gridDim.z);
    const int f = lb / gridDim.y, dy0 = (lb - f * gridDim.y) * kPyrRows;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const LevelGeom& D = G->lv[l];
    const int sw = G->lv[l - 1].w;
    const int dyn = min(kPyrRows, D.h - dy0);
    int spitch;
    const uint8_t* src = level_base(P, G, f, l - 1, spitch);
    const int sy0 = ytab[D.ytab_off + dy0].x & 0xFFFF;
    const int sy1 = (int)((uint32_t)ytab[D.ytab_off + dy0 + dyn - 1].x >> 16);
    const int nrows = sy1 - sy0 + 1;
    const int nc = lp >> 4;   // 16-byte chunks per staged row
    const uintptr_t ra = (uintptr_t)src + (size_t)sy0 * spitch;
    const uint8_t* gb = (const uint8_t*)(ra & ~(uintptr_t)15);
    const uint32_t sh0 = (uint32_t)(ra & 15);
    // row r's offset from gb: sh0 + r * spitch; the chunk split uses the float reciprocal of nc
    // ((i + 0.5) / nc sits 0.5 / nc from any integer: exact for i < 2^22)
    const int total = nrows * nc;
    const float inv_nc = 1.0f / (float)nc;
    const int nt = blockDim.x;
    for (int i0 = wave * 64; i0 < total; i0 += nt) {
        const int i = i0 + lane;
        const int r = (int)(((float)i + 0.5f) * inv_nc), c = i - __mul24(r, nc);
        const uint32_t ro = sh0 + __umul24((uint32_t)r, (uint32_t)spitch);
        const uint32_t co = (ro & ~15u) + 16u * (uint32_t)c;
        if (i < total && co < ro + (uint32_t)sw)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(gb + co),
                                             (__attribute__((address_space(3))) void*)(s_src + 4 * i0), 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const uint8_t* S = (const uint8_t*)s_src;
    // LDS byte of staged row r's pixel 0 (block-uniform)
    auto rowb = [&](int r) -> uint32_t { return (uint32_t)(r * lp) + ((sh0 + (uint32_t)r * (uint32_t)spitch) & 15u); };
    // a thread owns a group of 4 output columns: their coefficients are loaded once and
    // reused for the block's rows
    const int q = (D.w + 3) >> 2;
    uint8_t* drow0 = P.pyr + (size_t)f * P.pyr_fstride + D.pyr_off + (size_t)dy0 * D.pitch;
    for (int g = threadIdx.x; g < q; g += nt) {
        const int dx0 = g * 4;
        // every product fits a 24 x 24 -> 32-bit multiply (v_mul_u32_u24, full rate; the compiler
        // otherwise emits the quarter-rate v_mul_lo_u32 for h * b).  The two taps keep separate
        // addresses: byte reads at x0 and x0 + 1 merge into an unaligned ds_read_u16, which
        // measured 3.5x slower for the whole kernel.
        int x0[4], x1[4];
        uint32_t a0[4], a1[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int2 xt = xtab[D.xtab_off + min(dx0 + k, D.w - 1)];
            x0[k] = xt.x & 0xFFFF;
            x1[k] = (int)((uint32_t)xt.x >> 16);
            a0[k] = (uint32_t)xt.y & 0xFFFFu;
            a1[k] = (uint32_t)xt.y >> 16;
        }
        if constexpr (kWin) {
            // The group's 8 taps lie in the 8 bytes from x0[0] (LevelGeom::pyr_win, checked on the host):
            // per source row three dword reads, realigned to x0[0] by two alignbytes; each column's tap
            // pair is one v_perm into a u16 pair and one v_dot2_u32_u16 with (a0, a1)
            uint32_t sel[4], ak[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                sel[k] = (uint32_t)(x0[k] - x0[0]) | 0x0C00u | ((uint32_t)(x1[k] - x0[0]) << 16) | 0x0C000000u;
                ak[k] = a0[k] | (a1[k] << 16);
            }
            const uint32_t xo = (uint32_t)x0[0] & ~3u, xw = (uint32_t)x0[0] & 3u;
            auto hrow = [&](int r, uint32_t h[4]) {
                uint32_t A, wo;
                if constexpr (kA) {   // one add per row: the row offset is block-uniform, the shift per lane
                    A = rowb(r) + xo;
                    wo = xw;
                } else {
                    A = rowb(r) + (uint32_t)x0[0];
                    wo = A & 3u;
                    A &= ~3u;
                }
                const uint32_t* qd = (const uint32_t*)(S + A);
                const uint32_t d0 = qd[0], d1 = qd[1], d2 = qd[2];
                const uint32_t e0 = __builtin_amdgcn_alignbyte(d1, d0, wo), e1 = __builtin_amdgcn_alignbyte(d2, d1, wo);
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    h[k] = __builtin_amdgcn_udot2(as_us2(__builtin_amdgcn_perm(e1, e0, sel[k])), as_us2(ak[k]), 0u,
                                                  false);
            };
            // Output rows in order; consecutive rows share a source row (lo(y + 1) == hi(y)) at scale
            // factors up to 2, and that row's horizontal sums are kept instead of recomputed.  The
            // vertical sum is taken x4, (4 (h0 b0 + h1 b1) + 2^23) >> 24 = (h0 b0 + h1 b1 + 2^21) >> 22,
            // so each result is byte 3 of its sum and two v_perm pack four of them; the host checks that
            // the coefficient sums keep 4 * 255 * sum(a) * sum(b) + 2^23 below 2^32, which also makes
            // every result <= 255 (no saturation).
            int cr = -1;
            uint32_t hc[4] = {0u, 0u, 0u, 0u};
#pragma unroll
            for (int rr = 0; rr < kPyrRows; ++rr) {
                if (rr >= dyn) break;
                const int2 yt = ytab[D.ytab_off + dy0 + rr];
                const int lo = (yt.x & 0xFFFF) - sy0, hi = (int)((uint32_t)yt.x >> 16) - sy0;
                const uint32_t b0 = ((uint32_t)yt.y & 0xFFFFu) << 2, b1 = ((uint32_t)yt.y >> 16) << 2;
                uint32_t h0[4], h1[4];
                if (lo == cr) {
#pragma unroll
                    for (int k = 0; k < 4; ++k) h0[k] = hc[k];
                } else {
                    hrow(lo, h0);
                }
                if (hi == lo) {
#pragma unroll
                    for (int k = 0; k < 4; ++k) h1[k] = h0[k];
                } else {
                    hrow(hi, h1);
                }
                uint32_t acc[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    // two v_mad_u32_u24 (the compiler's form is two multiplies and an add3)
                    uint32_t t;
                    asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(t) : "v"(h0[k]), "s"(b0), "v"(1u << 23));
                    asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(acc[k]) : "v"(h1[k]), "s"(b1), "v"(t));
                }
                uint32_t packed = __builtin_amdgcn_perm(acc[1], acc[0], 0x0C0C0703u) |
                                  __builtin_amdgcn_perm(acc[3], acc[2], 0x07030C0Cu);
                if constexpr (kRM == 1) {
                    if (dx0 < D.rz_simd_end) {
                        packed = 0u;
#pragma unroll
                        for (int k = 0; k < 4; ++k) packed |= rz_sse2(h0[k], h1[k], b0 >> 2, b1 >> 2) << (8 * k);
                    }
                }
                *reinterpret_cast<uint32_t*>(drow0 + (size_t)rr * D.pitch + dx0) = packed;
                cr = hi;
#pragma unroll
                for (int k = 0; k < 4; ++k) hc[k] = h1[k];
            }
            continue;
        }
        for (int rr = 0; rr < dyn; ++rr) {
            const int2 yt = ytab[D.ytab_off + dy0 + rr];
            const uint8_t* r0 = S + rowb((yt.x & 0xFFFF) - sy0);
            const uint8_t* r1 = S + rowb((int)((uint32_t)yt.x >> 16) - sy0);
            const uint32_t b0 = (uint32_t)yt.y & 0xFFFFu, b1 = (uint32_t)yt.y >> 16;
            uint32_t packed = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t h0 = __umul24(r0[x0[k]], a0[k]) + __umul24(r0[x1[k]], a1[k]);
                const uint32_t h1 = __umul24(r1[x0[k]], a0[k]) + __umul24(r1[x1[k]], a1[k]);
                const uint32_t v = (kRM == 1 && dx0 < D.rz_simd_end) ? rz_sse2(h0, h1, b0, b1)
                                                                    : (__umul24(h0, b0) + __umul24(h1, b1) + (1u << 21)) >> 22;
                packed |= min(v, 255u) << (8 * k);
            }
            // columns past the level width land in the row's pitch padding (pitch = align64(w))
            *reinterpret_cast<uint32_t*>(drow0 + (size_t)rr * D.pitch + dx0) = packed;
        }
    }
}

// ---------------------------------------------------------------------------
// K1 for small batches (the per-frame host path, batch <= kLatencyMaxBatch): levels s+1..s+n from level s
// in one launch, so a single frame's pyramid is one or two launches instead of a chain of seven (each
// ~4.6 us of launch latency for a 640x480 frame).  Large batches keep one launch per level: there the
// kernel is VALU-bound and the bands' halo rows would add work.
// ---------------------------------------------------------------------------
constexpr int kPyrMaxNT = 512;

constexpr int kPyrChunk = 8;   // output rows per work item (unrolled; their row-table entries loaded up front)

// Rows [e.x, e.y] of level D from the source rows held in LDS (row r of the source level at LDS byte
// (r - sfirst) * slp + ((ssh0 + (r - sfirst) * ssp) & 15)), into LDS (dst, pitch dlp, from row e.x; unless
// `last`) and, for the rows this block owns ([e.z, e.w]), into the level's global image.
__device__ __forceinline__ void pyr_rows(const LevelGeom& Dg, const int2* __restrict__ xtab,
                                         const int2* __restrict__ ytab, const uint8_t* S, int slp, int sfirst,
                                         uint32_t ssh0, uint32_t ssp, uint8_t* dst, int dlp, int4 e, bool last,
                                         uint8_t* gimg, int nt, int split, int wave, int lane, int rm)
{
    // the level's fields in registers: the stores below could alias the geometry as far as the compiler
    // knows, which would reload them after every store
    const int w = Dg.w, pitch = Dg.pitch, xoff = Dg.xtab_off, yoff = Dg.ytab_off, win = Dg.pyr_win;
    const int xs = rm == 1 ? Dg.rz_simd_end : 0;   // ORBX_RESIZE_SSE2 columns (a multiple of 4)
    auto rowb = [&](int r) -> uint32_t {
        const int k = r - sfirst;
        return (uint32_t)(k * slp) + ((ssh0 + (uint32_t)k * ssp) & 15u);
    };
    // work items: (chunk of up to kPyrChunk rows, 4-column group), a wave's 64 groups in one chunk, so
    // every wave walks its rows in lock-step (row tables by scalar loads); on narrow levels the threads
    // beyond the first chunk take further chunks instead of idling
    const int q = (w + 3) >> 2, qp = (q + 63) & ~63;
    const int nrows = e.y - e.x + 1;
    const int nch = max((nrows + kPyrChunk - 1) / kPyrChunk, split ? min(nrows, nt / qp) : 1);
    const int rpc = (nrows + nch - 1) / nch;   // <= kPyrChunk
    const int items = qp * nch;
    for (int w0 = wave * 64; w0 < items; w0 += nt) {
        const int c = w0 / qp;
        const int g = w0 - c * qp + lane;
        const int r0 = e.x + c * rpc, nr = min(e.y - r0 + 1, rpc);
        if (g >= q || nr <= 0) continue;
        const int dx0 = g * 4;
        int2 yt[kPyrChunk];
#pragma unroll
        for (int k = 0; k < kPyrChunk; ++k) yt[k] = ytab[yoff + r0 + min(k, nr - 1)];
        // every product fits a 24 x 24 -> 32-bit multiply (v_mul_u32_u24, full rate; the compiler
        // otherwise emits the quarter-rate v_mul_lo_u32 for h * b).  The two taps keep separate
        // addresses: byte reads at x0 and x0 + 1 merge into an unaligned ds_read_u16, which
        // measured 3.5x slower for the whole kernel.
        int x0[4], x1[4];
        uint32_t a0[4], a1[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int2 xt = xtab[xoff + min(dx0 + k, w - 1)];
            x0[k] = xt.x & 0xFFFF;
            x1[k] = (int)((uint32_t)xt.x >> 16);
            a0[k] = (uint32_t)xt.y & 0xFFFFu;
            a1[k] = (uint32_t)xt.y >> 16;
        }
        auto put = [&](int rr, uint32_t packed) {
            if (!last) *reinterpret_cast<uint32_t*>(dst + (rr - e.x) * dlp + dx0) = packed;
            // columns past the level width land in the row's pitch padding (pitch = align64(w))
            if (rr >= e.z && rr <= e.w) *reinterpret_cast<uint32_t*>(gimg + (size_t)rr * pitch + dx0) = packed;
        };
        if (win) {   // block-uniform
            // The group's 8 taps lie in the 8 bytes from x0[0] (LevelGeom::pyr_win, checked on the host):
            // per source row three dword reads, realigned to x0[0] by two alignbytes; each column's tap
            // pair is one v_perm into a u16 pair and one v_dot2_u32_u16 with (a0, a1)
            uint32_t sel[4], ak[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                sel[k] = (uint32_t)(x0[k] - x0[0]) | 0x0C00u | ((uint32_t)(x1[k] - x0[0]) << 16) | 0x0C000000u;
                ak[k] = a0[k] | (a1[k] << 16);
            }
            auto hrow = [&](int r, uint32_t h[4]) {
                const uint32_t A = rowb(r) + (uint32_t)x0[0];
                const uint32_t* qd = (const uint32_t*)(S + (A & ~3u));
                const uint32_t d0 = qd[0], d1 = qd[1], d2 = qd[2], wo = A & 3u;
                const uint32_t e0 = __builtin_amdgcn_alignbyte(d1, d0, wo), e1 = __builtin_amdgcn_alignbyte(d2, d1, wo);
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    h[k] = __builtin_amdgcn_udot2(as_us2(__builtin_amdgcn_perm(e1, e0, sel[k])), as_us2(ak[k]), 0u,
                                                  false);
            };
            // Output rows in order; consecutive rows share a source row (lo(y + 1) == hi(y)) at scale
            // factors up to 2, and that row's horizontal sums are kept instead of recomputed.  The
            // vertical sum is taken x4, (4 (h0 b0 + h1 b1) + 2^23) >> 24 = (h0 b0 + h1 b1 + 2^21) >> 22,
            // so each result is byte 3 of its sum and two v_perm pack four of them; the host checks that
            // the coefficient sums keep 4 * 255 * sum(a) * sum(b) + 2^23 below 2^32, which also makes
            // every result <= 255 (no saturation).
            int cr = -1;
            uint32_t hc[4] = {0u, 0u, 0u, 0u};
#pragma unroll
            for (int k = 0; k < kPyrChunk; ++k) {
                if (k >= nr) break;
                const int lo = yt[k].x & 0xFFFF, hi = (int)((uint32_t)yt[k].x >> 16);
                const uint32_t b0 = ((uint32_t)yt[k].y & 0xFFFFu) << 2, b1 = ((uint32_t)yt[k].y >> 16) << 2;
                uint32_t h0[4], h1[4];
                if (lo == cr) {
#pragma unroll
                    for (int t = 0; t < 4; ++t) h0[t] = hc[t];
                } else {
                    hrow(lo, h0);
                }
                if (hi == lo) {
#pragma unroll
                    for (int t = 0; t < 4; ++t) h1[t] = h0[t];
                } else {
                    hrow(hi, h1);
                }
                uint32_t acc[4];
#pragma unroll
                for (int t = 0; t < 4; ++t) acc[t] = __umul24(h1[t], b1) + (__umul24(h0[t], b0) + (1u << 23));
                uint32_t packed = __builtin_amdgcn_perm(acc[1], acc[0], 0x0C0C0703u) |
                                  __builtin_amdgcn_perm(acc[3], acc[2], 0x07030C0Cu);
                if (dx0 < xs) {
                    packed = 0u;
#pragma unroll
                    for (int t = 0; t < 4; ++t) packed |= rz_sse2(h0[t], h1[t], b0 >> 2, b1 >> 2) << (8 * t);
                }
                put(r0 + k, packed);
                cr = hi;
#pragma unroll
                for (int t = 0; t < 4; ++t) hc[t] = h1[t];
            }
        } else {
#pragma unroll
            for (int k = 0; k < kPyrChunk; ++k) {
                if (k >= nr) break;
                const uint8_t* p0 = S + rowb(yt[k].x & 0xFFFF);
                const uint8_t* p1 = S + rowb((int)((uint32_t)yt[k].x >> 16));
                const uint32_t b0 = (uint32_t)yt[k].y & 0xFFFFu, b1 = (uint32_t)yt[k].y >> 16;
                uint32_t packed = 0;
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const uint32_t h0 = __umul24(p0[x0[t]], a0[t]) + __umul24(p0[x1[t]], a1[t]);
                    const uint32_t h1 = __umul24(p1[x0[t]], a0[t]) + __umul24(p1[x1[t]], a1[t]);
                    const uint32_t v = dx0 < xs ? rz_sse2(h0, h1, b0, b1) : (__umul24(h0, b0) + __umul24(h1, b1) + (1u << 21)) >> 22;
                    packed |= min(v, 255u) << (8 * t);
                }
                put(r0 + k, packed);
            }
        }
    }
}

// One block per (frame, band): a band is `rows` rows of the group's last level; its band-table entries
// (Geometry::pg, pyr_plan) name the rows of every level of the group it computes and the rows it owns.
// Level s's rows arrive in LDS by LDS-DMA (global_load_lds_dwordx4 of the 16-byte chunks that hold each
// row, so row r sits at LDS byte r * lp + sh_r with sh_r = its start address & 15; 0 for levels >= 1,
// whose pitch is a multiple of 64).  A chunk is fetched only if it holds a byte of its row: it then lies
// in the row's own 16-byte aligned span, which cannot cross a page boundary, so no read leaves the
// caller's allocation.  Levels s+1 .. s+n-1 stay in LDS (two row buffers) for the next level, and each
// block writes the rows it owns to the pyramid.  Blocks recompute the few rows their neighbours share
// (about one per level at each band edge) instead of synchronising.
__global__ __launch_bounds__(kPyrMaxNT) void k_pyramid_fused(const Geometry* __restrict__ G, FramePtrs P, int gi,
                                                    const int2* __restrict__ xtab, const int2* __restrict__ ytab,
                                                    const int4* __restrict__ bands, int rm)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t s_src[];
    const PyrGroup& PG = G->pg[gi];
    const int nt = blockDim.x;
    const int lb = xcd_block(blockIdx.y + blockIdx.z * gridDim.y, gridDim.y * gridDim.z);
    const int f = lb / gridDim.y, band = lb - f * gridDim.y;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int s = PG.s, n = PG.n;
    const int4* B = bands + PG.bt_off + (size_t)band * (n + 1);
    const int4 e0 = B[0];
    const int sw = G->lv[s].w;
    int spitch;
    const uint8_t* src = level_base(P, G, f, s, spitch);
    const int lp0 = ((sw + 30) >> 4) << 4;   // the 16-byte chunks spanning a row at any start alignment
    const int nc = lp0 >> 4;
    const uintptr_t ra = (uintptr_t)src + (size_t)e0.x * spitch;
    const uint8_t* gb = (const uint8_t*)(ra & ~(uintptr_t)15);
    const uint32_t sh0 = (uint32_t)(ra & 15);
    // row r's offset from gb: sh0 + r * spitch; the chunk split uses the float reciprocal of nc
    // ((i + 0.5) / nc sits 0.5 / nc from any integer: exact for i < 2^22)
    const int total = (e0.y - e0.x + 1) * nc;
    const float inv_nc = 1.0f / (float)nc;
    for (int i0 = wave * 64; i0 < total; i0 += nt) {
        const int i = i0 + lane;
        const int r = (int)(((float)i + 0.5f) * inv_nc), c = i - __mul24(r, nc);
        const uint32_t ro = sh0 + __umul24((uint32_t)r, (uint32_t)spitch);
        const uint32_t co = (ro & ~15u) + 16u * (uint32_t)c;
        if (i < total && co < ro + (uint32_t)sw)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(gb + co),
                                             (__attribute__((address_space(3))) void*)(s_src + 4 * i0), 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    uint8_t* X = (uint8_t*)s_src;
    uint8_t* Y = X + PG.lds_x;
    const uint8_t* S = X;
    int slp = lp0, sfirst = e0.x;
    uint32_t ssh0 = sh0, ssp = (uint32_t)spitch;
    for (int i = 1; i <= n; ++i) {
        const LevelGeom& D = G->lv[s + i];
        const int4 e = B[i];
        const bool last = i == n;
        uint8_t* dst = (i & 1) ? Y : X;
        const int dlp = ((D.w + 15) >> 4) << 4;
        uint8_t* gimg = P.pyr + (size_t)f * P.pyr_fstride + D.pyr_off;
        pyr_rows(D, xtab, ytab, S, slp, sfirst, ssh0, ssp, dst, dlp, e, last, gimg, nt, PG.split, wave, lane, rm);
        if (last) break;
        __syncthreads();   // level s+i is whole in LDS; the buffer it was made from is free
        S = dst;
        slp = dlp;
        sfirst = e.x;
        ssh0 = 0;
        ssp = 0;
    }
}

bool pyr_plan(Geometry& g, const int2* yt, std::vector<int4>& bands)
{
    bands.clear();
    g.pyr_ngroups = 0;
    if (g.nlevels < 2) return true;
    // ORBX_PYR_FUSED=0: per-level launches for every batch (tested against the oracle,
    // tests/test_gpu_parity.py test_pyramid_per_level_launches_small_batch)
    if (const char* v = getenv("ORBX_PYR_FUSED"))
        if (atoi(v) == 0) return true;
    // group starts (first computed level of each launch): levels 1-3 from level 0, 4-7 from level 3 (640x480
    // host path: 0.147 against 0.150-0.156 ms for 1 or 3 launches); bands of 4 rows of a group's last level
    std::vector<int> st = {1};
    if (4 < g.nlevels) st.push_back(4);
    const int R = 4;
    auto lo = [&](int j, int y) { return yt[g.lv[j].ytab_off + y].x & 0xFFFF; };
    auto hi = [&](int j, int y) { return (int)((uint32_t)yt[g.lv[j].ytab_off + y].x >> 16); };
    auto lds_pitch = [&](int j, bool staged) { return staged ? ((g.lv[j].w + 30) >> 4) << 4 : ((g.lv[j].w + 15) >> 4) << 4; };
    for (size_t gi = 0; gi < st.size(); ++gi) {
        const int s = st[gi] - 1, b = gi + 1 < st.size() ? st[gi + 1] - 1 : g.nlevels - 1, n = b - s;
        const int K = (g.lv[b].h + R - 1) / R;
        // start[j - s][k]: first row of level j owned by band k (k = K: the level height)
        std::vector<std::vector<int>> start(n + 1, std::vector<int>(K + 1));
        for (int k = 0; k <= K; ++k) start[n][k] = std::min(k * R, g.lv[b].h);
        for (int j = b - 1; j > s; --j) {
            start[j - s][0] = 0;
            start[j - s][K] = g.lv[j].h;
            for (int k = 1; k < K; ++k) start[j - s][k] = std::max(start[j - s][k - 1], lo(j + 1, start[j + 1 - s][k]));
        }
        PyrGroup& P = g.pg[g.pyr_ngroups];
        P.s = s;
        P.n = n;
        P.rows = R;
        P.nbands = K;
        P.bt_off = (int)bands.size();
        P.lds_x = P.lds_y = 0;
        int qmax = 0;
        for (int j = s + 1; j <= b; ++j) qmax = std::max(qmax, (g.lv[j].w + 3) >> 2);
        P.nt = qmax > 256 ? std::min(kPyrMaxNT, (qmax + 63) & ~63) : 256;
        P.split = 1;
        std::vector<int4> e(n + 1);
        for (int k = 0; k < K; ++k) {
            e[n] = make_int4(start[n][k], start[n][k + 1] - 1, start[n][k], start[n][k + 1] - 1);
            for (int j = b - 1; j > s; --j) {
                const int of = start[j - s][k], ol = start[j - s][k + 1] - 1;
                int f0 = lo(j + 1, e[j + 1 - s].x), l0 = hi(j + 1, e[j + 1 - s].y);
                if (of <= ol) {
                    f0 = std::min(f0, of);
                    l0 = std::max(l0, ol);
                }
                e[j - s] = make_int4(f0, l0, of, ol);
            }
            e[0] = make_int4(lo(s + 1, e[1].x), hi(s + 1, e[1].y), 0, -1);
            for (int i = 0; i <= n; ++i) {
                if (e[i].y < e[i].x) {   // (cannot happen for a shrinking pyramid) per-level launches
                    g.pyr_ngroups = 0;
                    bands.clear();
                    return true;
                }
                const int bytes = (e[i].y - e[i].x + 1) * lds_pitch(s + i, i == 0);
                if (i % 2 == 0) P.lds_x = std::max(P.lds_x, bytes);
                else if (i < n) P.lds_y = std::max(P.lds_y, bytes);
            }
            bands.insert(bands.end(), e.begin(), e.end());
        }
        // + 16 bytes: the window path's third dword of a group at the end of the last row; a group whose rows
        // outgrow a workgroup's LDS (very wide images) leaves the small-batch path on the per-level launches
        if (P.lds_x + P.lds_y + 16 > 160 * 1024) {
            g.pyr_ngroups = 0;
            bands.clear();
            return true;
        }
        ++g.pyr_ngroups;
    }
    return true;
}

size_t pyr_level_lds(const Geometry& g, int l)
{
    // source rows per block: kPyrRows * (src/dst scale) + 2, bounded by the level ratio; an LDS row is the
    // 16-byte chunks spanning a source row at any start alignment; + 16 bytes: the window path's third dword
    // of a group at the end of the last row
    const int srows = (kPyrRows * g.lv[l - 1].h + g.lv[l].h - 1) / g.lv[l].h + 2;
    const int lp = ((g.lv[l - 1].w + 15 + 15) >> 4) << 4;
    return (size_t)srows * lp + 16;
}

void launch_pyramid(const Geometry& g, const ExtractBufs& b, const FramePtrs& p, int batch, hipStream_t s)
{
    if (batch <= kLatencyMaxBatch && g.pyr_ngroups > 0) {
        for (int i = 0; i < g.pyr_ngroups; ++i) {
            const PyrGroup& P = g.pg[i];
            const size_t smem = (size_t)P.lds_x + P.lds_y + 16;
            if (smem > 64 * 1024)
                hipFuncSetAttribute((const void*)k_pyramid_fused, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
            hipLaunchKernelGGL(k_pyramid_fused, dim3(1, P.nbands, batch), dim3(P.nt), smem, s, b.geom, p, i, b.xtab,
                               b.ytab, b.pyr_bands, b.resize_mode);
        }
        return;
    }
    for (int l = 1; l < g.nlevels; ++l) {
        const int h = g.lv[l].h;
        // source rows per block: kPyrRows * (src/dst scale) + 2, bounded by the level ratio
        const int srows = (kPyrRows * g.lv[l - 1].h + g.lv[l].h - 1) / g.lv[l].h + 2;
        // LDS row: the 16-byte chunks spanning a row at any start alignment; + 16 bytes: the window
        // path's third dword of a group at the end of the last row
        const int lp = ((g.lv[l - 1].w + 15 + 15) >> 4) << 4;
        const size_t smem = (size_t)srows * lp + 16;
        dim3 grid(1, (h + kPyrRows - 1) / kPyrRows, batch);
        // a thread per 4-column group: narrow levels take fewer waves per block
        const int q = (g.lv[l].w + 3) >> 2;
        const int nt = std::min(kPyrNT, (q + 63) & ~63);
        const bool al = l >= 2 || (((uintptr_t)p.in | (uintptr_t)p.in_pitch | (uintptr_t)p.in_fstride) & 3) == 0;
        // (levels of images wider than about 4,000 px stage more than the default 64 KiB; ensure_geometry
        // rejects any above the workgroup's 160 KiB, pyr_level_lds)
        auto launch = [&](auto kern) {
            if (smem > 64 * 1024)
                hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
            hipLaunchKernelGGL(kern, grid, dim3(nt), smem, s, b.geom, p, l, b.xtab, b.ytab, lp);
        };
        auto go = [&](auto rm_tag) {
            constexpr int RM = decltype(rm_tag)::value;
            if (g.lv[l].pyr_win && al) launch(k_pyramid_level<true, true, RM>);
            else if (g.lv[l].pyr_win) launch(k_pyramid_level<true, false, RM>);
            else launch(k_pyramid_level<false, false, RM>);
        };
        if (b.resize_mode == ORBX_RESIZE_SSE2) go(std::integral_constant<int, 1>{});
        else go(std::integral_constant<int, 0>{});
    }
}

// ---------------------------------------------------------------------------
// K2: FAST-9/16 on one cell ROI per wave (cv::FAST(roi, kps, th, true)).
// s = max(A, -B) with A = max over 9-arcs of min(v - ring), B = min of max:
// a pixel is a corner at t iff s > t, and cornerScore = s - 1.
// NMS is evaluated inside the cell with scores masked by the cell threshold;
// the cell falls back to minThFAST iff NMS at iniThFAST keeps nothing
// (src/ORBextractor.cc:982-987).  Survivors are emitted row-major, i.e. in
// OpenCV's emission order.
// ---------------------------------------------------------------------------
// The ROI tile holds the pixel bytes x, one byte per pixel.  A byte read into the low half of a VGPR
// (ds_read_u8_d16) is the f16 bit pattern of the denormal x * 2^-24: denormals are exact fixed-point
// values (the kernels run with f16 denormals preserved, .amdhsa_float_denorm_mode_16_64 3), so f16
// max/min/sub/compare on them are exact integer operations, and a non-negative result's bit pattern is
// its integer value.  Each ring value enters the arithmetic as the packed pair (h, -h): the compiler
// folds that into the first packed instruction's source modifiers (op_sel_hi = 0, neg_hi), so it costs
// nothing, and packed f16 max/min/sub work on both polarities at once.  (Round 2 stored 0x6400 | x, the
// normal f16 1024 + x, 2 bytes per pixel: the byte tile halves the tile's LDS and its commit is one
// alignbyte and one 4-byte store per pass.)  gfx950's v_pk_maximum3_f16 / v_pk_minimum3_f16 take three
// operands: a 9-arc max of the pairs is the "brighter" arc value and, in the other half, minus the 9-arc
// min ("darker").
typedef _Float16 fh2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ fh2 as_fh2(uint32_t u) { return __builtin_bit_cast(fh2, u); }
__device__ __forceinline__ fh2 pmax2(fh2 a, fh2 b) { return __builtin_elementwise_maximum(a, b); }
__device__ __forceinline__ fh2 pmin2(fh2 a, fh2 b) { return __builtin_elementwise_minimum(a, b); }
__device__ __forceinline__ fh2 pmax3(fh2 a, fh2 b, fh2 c) { return pmax2(pmax2(a, b), c); }
__device__ __forceinline__ fh2 pmin3(fh2 a, fh2 b, fh2 c) { return pmin2(pmin2(a, b), c); }
// pixel byte as the f16 denormal x * 2^-24; an integer threshold likewise
__device__ __forceinline__ _Float16 px16(const uint8_t* p) { return __builtin_bit_cast(_Float16, (uint16_t)*p); }
__device__ __forceinline__ _Float16 int16_as_f16(int t) { return __builtin_bit_cast(_Float16, (uint16_t)t); }
__device__ __forceinline__ fh2 dup_neg(_Float16 h)
{
    fh2 r;
    r.x = h;
    r.y = -h;
    return r;
}

// Tile row pitch in dwords (pixels): a compile-time constant per kernel instantiation, so every ring
// and neighbour access is one base register plus an immediate LDS offset (no per-access address
// arithmetic).  40 covers the ROIs of every BASELINE configuration (37-38 px); 68 the 66-px cap.
__host__ __device__ constexpr int fast_tile_pitch(int max_roi_w) { return max_roi_w <= 40 ? 40 : 68; }
// per-wave LDS: ROI tile [rh][TP] bytes, zero-bordered strength map [rh - 4][TP] bytes (the
// detection window plus a one-pixel frame, at the tile's pitch so a map index is a tile index minus a
// constant), and the candidate list (u16 tile indices) of the largest window, filled from both ends
__host__ __device__ inline size_t fast_map_bytes(int rw, int rh)
{
    return ((size_t)(rh - 4) * fast_tile_pitch(rw) + 3) & ~(size_t)3;
}
__host__ __device__ inline int fast_list_cap(int rw, int rh) { return (rh - 6) * (rw - 6); }
// Output buffer (packed candidates) of the wave's cells, written to HBM once after its last cell: a global
// store inside the cell loop would make the next cell's wait for its prefetched ROI (vmcnt counts loads
// and stores, completed in issue order) wait for the store's round trip as well.
#ifndef ORBX_FAST_OBCAP
#define ORBX_FAST_OBCAP 128
#endif
constexpr int kFastObCap = ORBX_FAST_OBCAP;
constexpr int kFastScratch = 128;   // a u16 per lane after obuf (the masked-off lanes' list and map writes)
__host__ __device__ inline size_t fast_list_bytes(int rw, int rh) { return (2 * (size_t)fast_list_cap(rw, rh) + 3) & ~(size_t)3; }
__host__ __device__ inline size_t fast_wave_bytes(int rw, int rh)
{
    const size_t tile = (size_t)rh * fast_tile_pitch(rw);
    return (tile + fast_map_bytes(rw, rh) + fast_list_bytes(rw, rh) + 4 * kFastObCap + kFastScratch + 15) & ~(size_t)15;
}

// max(v - minMax, maxMin - v) over the 16 cyclic 9-arcs of the Bresenham ring of the
// pixel at tile byte c[0]
template <int TP>
__device__ __forceinline__ int fast_strength(const uint8_t* c)
{
    fh2 x[16];
    x[0] = dup_neg(px16(c + 3 * TP));
    x[1] = dup_neg(px16(c + 3 * TP + 1));
    x[2] = dup_neg(px16(c + 2 * TP + 2));
    x[3] = dup_neg(px16(c + TP + 3));
    x[4] = dup_neg(px16(c + 3));
    x[5] = dup_neg(px16(c - TP + 3));
    x[6] = dup_neg(px16(c - 2 * TP + 2));
    x[7] = dup_neg(px16(c - 3 * TP + 1));
    x[8] = dup_neg(px16(c - 3 * TP));
    x[9] = dup_neg(px16(c - 3 * TP - 1));
    x[10] = dup_neg(px16(c - 2 * TP - 2));
    x[11] = dup_neg(px16(c - TP - 3));
    x[12] = dup_neg(px16(c - 3));
    x[13] = dup_neg(px16(c + TP - 3));
    x[14] = dup_neg(px16(c + 2 * TP - 2));
    x[15] = dup_neg(px16(c + 3 * TP - 1));
    fh2 m3[16], a[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) m3[k] = pmax3(x[k], x[(k + 1) & 15], x[(k + 2) & 15]);
#pragma unroll
    for (int k = 0; k < 16; ++k) a[k] = pmax3(m3[k], m3[(k + 3) & 15], m3[(k + 6) & 15]);
    const fh2 b0 = pmin3(a[0], a[1], a[2]), b1 = pmin3(a[3], a[4], a[5]), b2 = pmin3(a[6], a[7], a[8]);
    const fh2 b3 = pmin3(a[9], a[10], a[11]), b4 = pmin3(a[12], a[13], a[14]);
    const fh2 mm = pmin3(pmin3(b0, b1, b2), pmin2(b3, b4), a[15]);   // (minMax, -maxMin)
    const fh2 d = dup_neg(px16(c)) - mm;   // (v - minMax, maxMin - v)
    // the integer value of a non-negative result; a negative one reads as a negative int16 (not a corner)
    return (int)__builtin_bit_cast(int16_t, __builtin_fmaxf16(d.x, d.y));
}

// Compass value q of the pixel at c[0]: a 9-arc holds two consecutive compass points (ring positions
// 0, 4, 8, 12), so s > t needs some consecutive pair brighter than v + t or darker than v - t, i.e.
// q = max(max pair-min - v, v - min pair-max) > t.  An integer-valued f16.  Over the 4-cycle
// (N, E, S, W) the largest pair minimum is min(max(N, S), max(E, W)): each consecutive pair holds one of
// {N, S} and one of {E, W}, and the larger of N, S forms a pair with each of E, W.  Three packed ops.
template <int TP>
__device__ __forceinline__ _Float16 fast_compass_q(const uint8_t* c)
{
    const fh2 a = dup_neg(px16(c + 3 * TP)), b = dup_neg(px16(c + 3)), d = dup_neg(px16(c - 3 * TP)),
              e = dup_neg(px16(c - 3));
    const fh2 m = pmin2(pmax2(a, d), pmax2(b, e));   // (br, -dk)
    const fh2 q = m - dup_neg(px16(c));              // (br - v, v - dk)
    return __builtin_fmaxf16(q.x, q.y);   // one v_max_f16 (SDWA high-half operand)
}

// strict 3x3 non-maximum suppression on the strength map at threshold t (m[0]: the pixel).  cv::FAST keeps
// a corner whose score s - 1 beats every neighbour's score, a neighbour that is no corner at t scoring 0:
//   s > t and, for each neighbour n, (n > t ? s > n : s > 1),
// and since s > t already beats every n <= t, that is s > max(t, 1, n_0 .. n_7): four max3, one compare.
// (t1 = max(t, 1), wave-uniform)
__device__ __forceinline__ uint32_t umax3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_elementwise_max(__builtin_elementwise_max(a, b), c); }
template <int TP>
__device__ __forceinline__ bool nms_keep(const uint8_t* m, uint32_t t1)
{
    const uint32_t a = umax3(m[-TP - 1], m[-TP], m[-TP + 1]);
    const uint32_t b = umax3(m[-1], m[1], m[TP - 1]);
    const uint32_t c = umax3(m[TP], m[TP + 1], t1);
    return (uint32_t)m[0] > umax3(a, b, c);
}

// ROI bytes of one cell staged in registers, in passes of rpp whole rows: lane = rl * nd + kl loads
// dword kl of row u * rpp + rl (nd = dwords per ROI row) at its exact byte, so a pass costs one register.
// LD passes are prefetched (the launch's largest ROI: 8 for
// 38 x 39, 10 for 38 x 46 ROIs); bigger ROIs load their remainder synchronously.
// kCellsPerWave (orbx_kernels.hpp) cells per wave: the next cell's ROI loads fly under this one's passes

template <int LD>
struct FastPrefetch {
    uint32_t w[LD];
};

struct FastCellSrc {
    const uint8_t* src;   // ROI origin
    int pitch, nd, rh;    // dwords per row ceil(roi_w / 4), rows
};

// The lane map of the tile pitch's widest row (TP / 4 dwords + the extra one): rows per pass and the
// lane's (row in pass, dword) are compile-time / per-kernel constants, so every pass's offsets are
// immediates; a narrower cell leaves its lanes past its own dwords idle.
// Each lane loads its dword at the exact (unaligned) ROI byte, which gfx950 serves exactly
// (tools/probes/glb_unaligned.hip), so the commit is a plain store: TP / 4 lanes per row.
__host__ __device__ constexpr int fast_lanes_per_row(int tp) { return tp / 4; }
template <int TP>
struct FastLaneMap {
    static constexpr int kND1 = fast_lanes_per_row(TP), kRPP = 64 / kND1;
    int rl, kl;
    __device__ explicit FastLaneMap(int lane) : rl(lane / kND1), kl(lane - (lane / kND1) * kND1) {}
};

template <int TP, int LD>
__device__ __forceinline__ void fast_issue(const FastCellSrc& S, const FastLaneMap<TP>& M, int u0, FastPrefetch<LD>& F)
{
    // branch-free: every lane loads, its row clamped to the ROI's last and its dword to the row's last (the
    // lanes past a row's dwords and past a pass's rows repeat a neighbour's load, which the commit stores to
    // the same place): no exec save / branch / restore per pass
    // (an empty cell -- the level padding's -- loads nothing: its clamps would go negative)
    if (S.rh <= 0 || S.nd <= 0) return;   // wave-uniform
    const __attribute__((address_space(1))) uint8_t* base = (const __attribute__((address_space(1))) uint8_t*)S.src;
    const uint32_t kb = 4u * (uint32_t)min(M.kl, S.nd - 1);
#pragma unroll
    for (int u = 0; u < LD; ++u) {
        const uint32_t row = (uint32_t)min((u0 + u) * FastLaneMap<TP>::kRPP + M.rl, S.rh - 1);
        F.w[u] = *(const __attribute__((address_space(1))) uint32_t*)(base + (__umul24(row, (uint32_t)S.pitch) + kb));
    }
}

// The first LD passes of a cell (u0 = 0) without per-pass address arithmetic or tests: every pass loads, from
// a scalar row offset plus the lane's fixed one, through a buffer descriptor whose size ends at the ROI's last
// byte, so the rows past the ROI read zeros (gfx950's range check covers soffset too,
// tools/probes/buffer_oob.hip) instead of each pass taking a scalar compare and branch.  The commit stores the
// passes holding ROI rows at immediate LDS offsets (a partial pass's rows past the ROI land in the map,
// cleared after the commit).  No VALU per pass; the general form below clamps every lane's row (3 VALU per pass).
template <int TP, int LD>
__device__ __forceinline__ void fast_issue0(const FastCellSrc& S, const FastLaneMap<TP>& M, FastPrefetch<LD>& F)
{
    constexpr int kRPP = FastLaneMap<TP>::kRPP;
    if (S.rh <= 0 || S.nd <= 0) return;   // wave-uniform
    const uint32_t lo = __umul24((uint32_t)M.rl, (uint32_t)S.pitch) + 4u * (uint32_t)min(M.kl, S.nd - 1);
    // the pass's row offset goes in the scalar offset (buffer_load ... offen with soffset), the lane's in the
    // vector one
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)S.src, (short)0,
                                                                         (S.rh - 1) * S.pitch + 4 * S.nd, 0x00020000);
#pragma unroll
    for (int u = 0; u < LD; ++u) F.w[u] = __builtin_amdgcn_raw_buffer_load_b32(rs, lo, u * kRPP * S.pitch, 0);
}
template <int TP, int LD>
__device__ __forceinline__ void fast_commit0(const FastPrefetch<LD>& F, const FastCellSrc& S, const FastLaneMap<TP>& M,
                                             uint8_t* tile)
{
    constexpr int kRPP = FastLaneMap<TP>::kRPP;
    if (S.rh > 0 && S.nd > 0) {   // wave-uniform (empty cells store nothing)
        const uint32_t a = __umul24((uint32_t)M.rl, (uint32_t)TP) + 4u * (uint32_t)min(M.kl, S.nd - 1) +
                           (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)tile;
#pragma unroll
        for (int u = 0; u < LD; ++u)
            if (u * kRPP < S.rh)   // wave-uniform; an immediate offset
                *(__attribute__((address_space(3))) uint32_t*)(uintptr_t)(a + (uint32_t)(u * kRPP * TP)) = F.w[u];
    }
}

// 4 pixels of ROI row r from column 4 kl: the lane's dword and its neighbour's realigned by the row's
// byte shift (v_alignbyte uses the shift's low two bits, so the shift of pass u is the lane's first one
// plus a uniform step), one 4-byte LDS store at an immediate offset per pass
template <int TP, int LD>
__device__ __forceinline__ void fast_commit(const FastPrefetch<LD>& F, const FastCellSrc& S,
                                            const FastLaneMap<TP>& M, int u0, uint8_t* tile)
{
    constexpr int kRPP = FastLaneMap<TP>::kRPP;
    if (S.rh > 0 && S.nd > 0) {   // wave-uniform (empty cells store nothing)
        // 32-bit LDS byte addresses (a pointer offset compiles to a 64-bit multiply-add)
        const uint32_t dst = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)tile +
                             4u * (uint32_t)min(M.kl, S.nd - 1);
#pragma unroll
        for (int u = 0; u < LD; ++u) {
            const uint32_t row = (uint32_t)min(u0 * kRPP + u * kRPP + M.rl, S.rh - 1);
            *(__attribute__((address_space(3))) uint32_t*)(uintptr_t)(__umul24(row, (uint32_t)TP) + dst) = F.w[u];
        }
    }
}

#ifdef ORBX_FAST_PROF
// per-phase cycle sums of all FAST waves: staging commit, map clear, pass 1, pass 2, NMS, output, cells
__device__ unsigned long long g_fast_prof[8];
#define FP_STAMP(k)                          \
    do {                                     \
        const long long t1_ = clock64();     \
        fp_acc[k] += t1_ - fp_t;             \
        fp_t = t1_;                          \
    } while (0)
#else
#define FP_STAMP(k) ((void)0)
#endif

__device__ __forceinline__ unsigned long long ballot64(bool p) { return __builtin_amdgcn_ballot_w64(p); }
// (a + b) << 1 in one v_add_lshl_u32
__device__ __forceinline__ uint32_t add_lshl1(uint32_t a, uint32_t b)
{
    uint32_t r;
    asm("v_add_lshl_u32 %0, %1, %2, 1" : "=v"(r) : "v"(a), "s"(b));
    return r;
}
__device__ __forceinline__ uint16_t* lds_u16(uint32_t a) { return (uint16_t*)(__attribute__((address_space(3))) uint16_t*)(uintptr_t)a; }
// per lane: a if the lane's bit of the scalar mask m is set, else b -- one v_cndmask on the mask, with every
// lane active (the compiler's form of the select is an exec-masked region)
__device__ __forceinline__ uint16_t* lds_select(unsigned long long m, uint16_t* a, uint16_t* b)
{
    const uint32_t ua = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint16_t*)a;
    const uint32_t ub = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint16_t*)b;
    uint32_t r;
    asm volatile("v_cndmask_b32 %0, %1, %2, %3" : "=v"(r) : "v"(ub), "v"(ua), "s"(m));
    return (uint16_t*)(__attribute__((address_space(3))) uint16_t*)(uintptr_t)r;
}

// K2: one wave per workgroup (LDS is granted per wave), cpw consecutive cells per wave.  Per cell
// (src/ORBextractor.cc:952-1000, cv::FAST on the cell ROI with nonmax suppression, retried at
// minThFAST when iniThFAST keeps nothing):
//   pass 1   compass value q of every window pixel; q > iniThFAST lists the pixel at the list's front,
//            minThFAST < q <= iniThFAST at its back (q <= t implies strength <= t)
//   pass 2a  exact strength of the front entries into the map (kept if above the lower threshold)
//   NMS      at iniThFAST over the front entries
//   pass 2b  only when it kept nothing: strengths of the back entries, then NMS at minThFAST over both
//   output   kept pixels marked in a per-row bitmask, emitted in row-major order (cv::FAST's order)
// On the synthetic KITTI sequence about 45% of cells fall back, and the front holds about 2% of the
// pixels against 26% for both ends, so the fallback-free cells skip most strength evaluations.
#ifndef ORBX_FAST_WPE
#define ORBX_FAST_WPE 1
#endif
#ifndef ORBX_FAST_WPE10
#define ORBX_FAST_WPE10 1   // 6 (80 VGPRs, 6 dwords spilled) measured 200.9 against 183.3 us
#endif
// A wave's candidates go to HBM as one run from its first cell's slot region, which starts on a 128-byte line
// (the slot regions of a wave's cells are consecutive, so the run fits).  (Measured and removed in round 4:
// the run taken from a per-(frame, level) fill counter by one atomic after the wave's last cell, which makes
// each level's candidates dense -- quadtree fetch 1.05x algorithmic -- but makes every wave wait on the
// atomic's round trip: FAST +13-19 us per 384 frames, -0.8% frames/s)
// Row-validity masks of pass 1: 0 = a ballot of one compare per row step; 1 = scalar arithmetic per trip
// (697.6 against 641.5 us: FAST is sensitive to its scalar instruction count), 2 = the last trip's masks
// hoisted out of the loop, a select per trip (657.7 us)
template <int TP, int LD>
__global__ __launch_bounds__(64, LD >= 10 ? ORBX_FAST_WPE10 : ORBX_FAST_WPE) void k_fast_cells(const Geometry* __restrict__ G, FramePtrs P,
                                                   const Cell* __restrict__ cells, uint32_t* __restrict__ slots,
                                                   int* __restrict__ cell_counts, int cb, int ce, int rw, int rh,
                                                   int cpw)
{
    // cells [cb, ce); LDS sized from the group's largest cell ROI (rw x rh)
    const int lane = threadIdx.x;
    const int lb = xcd_block(blockIdx.x + blockIdx.y * gridDim.x, gridDim.x * gridDim.y);
    const int f = lb / gridDim.x;
    const int c0 = cb + (lb - f * gridDim.x) * cpw;
    const int c1 = min(c0 + cpw, ce);
    if (c0 >= c1) return;   // wave-uniform; no block barriers below
    uint8_t* tile = dyn_lds();
    uint8_t* map = tile + (size_t)rh * TP;
    uint16_t* list = (uint16_t*)(map + fast_map_bytes(rw, rh));
    uint32_t* obuf = (uint32_t*)((uint8_t*)list + fast_list_bytes(rw, rh));
    const int lcap = fast_list_cap(rw, rh);
    uint16_t* const bscratch = (uint16_t*)(obuf + kFastObCap) + lane;
    uint32_t* fslots = slots + (size_t)f * G->slots_per_frame;
    // lane i: the wave's cell c0 + i -- its candidate count, obuf offset (buffered cells) and the slot its
    // candidates start at.  The wave's cells (one level: the cell lists are padded to whole waves) are
    // buffered in obuf and go to HBM together after its last cell, as one run from a 128-byte line, so the
    // quadtree's gather reads few partial lines.  A cell that does not fit obuf, and the wave's cells after
    // it, write to their own slot regions (flagged kCellDirect in cell_counts).
    int cnt_all = 0, c_off = -1;   // c_off >= 0: the lane's cell is buffered
    int obn = 0;
    bool direct = false;   // wave-uniform
    // kept-pixel bitmask, one u64 per window row: aliases the tile, which is dead once every strength
    // of the cell is known
    unsigned long long* kept = (unsigned long long*)tile;
    const int t_ini = G->ini_th, t_min = G->min_th;
    const int t_lo = min(t_ini, t_min);
    const _Float16 f_hi = int16_as_f16(t_ini), f_lo = int16_as_f16(t_lo);   // thresholds as denormals
#ifdef ORBX_FAST_PROF
    long long fp_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    long long fp_t = clock64();
#endif

    // ROI -> LDS: aligned dword loads (alignbyte realigns rows of any pitch; the ROI ends >= 16
    // px before the level's right edge, so the 8-byte read stays in the row), 4 packed pixels
    // per 16-byte LDS store.  The next cell's loads are issued before this cell's passes.
    auto cell_src = [&](const Cell& C) {
        FastCellSrc S;
        int pitch;
        const uint8_t* img = level_base(P, G, f, C.level, pitch);
        S.src = img + (size_t)C.roi_y0 * pitch + C.roi_x0;
        S.pitch = pitch;
        S.nd = (C.roi_w + 3) >> 2;
        S.rh = C.roi_h;
        return S;
    };
    // the cell descriptor as whole dwords: scalar loads (a 16-bit field read is a vector load, whose
    // vmcnt wait would also drain every store still in flight)
    auto load_cell = [&](int ci) {
        const uint32_t* w = (const uint32_t*)(cells + ci);
        const uint32_t w0 = w[0], w1 = w[1];
        Cell r;
        r.level = (int16_t)(w0 & 0xFFFF);
        r.roi_w = (int16_t)(w0 >> 16);
        r.roi_h = (int16_t)(w1 & 0xFFFF);
        r.pad = 0;
        r.roi_x0 = (int32_t)w[2];
        r.roi_y0 = (int32_t)w[3];
        r.slot_base = (int32_t)w[4];
        r.slot_cap = (int32_t)w[5];
        return r;
    };
    Cell C = load_cell(c0);
    FastCellSrc S = cell_src(C);
    const FastLaneMap<TP> M(lane);
    FastPrefetch<LD> F;
    fast_issue0(S, M, F);

#pragma unroll 1
    for (int c = c0; c < c1; ++c) {
        const int dw = C.roi_w - 6, dh = C.roi_h - 6;
        const Cell Cc = C;
        FP_STAMP(7);
        fast_commit0(F, S, M, tile);
        for (int u0 = LD; u0 * FastLaneMap<TP>::kRPP < S.rh; u0 += LD) {   // ROIs beyond LD passes
            FastPrefetch<LD> R;
            fast_issue(S, M, u0, R);
            fast_commit(R, S, M, u0, tile);
        }
        const int mapn = (dh + 2) * TP;
        FP_STAMP(0);
        if constexpr (TP % 8 == 0) {   // the map (at rh * TP) and mapn are whole 8-byte words: half the stores
            for (int i = lane; i < mapn >> 3; i += 64) ((uint2*)map)[i] = make_uint2(0u, 0u);
        } else {
            for (int i = lane; i < (mapn + 3) >> 2; i += 64) ((uint32_t*)map)[i] = 0u;
        }
        wave_lds_sync();
        FP_STAMP(1);
        if (c + 1 < c1) {   // prefetch the next cell (registers only; lands under the passes below)
            C = load_cell(c + 1);
            S = cell_src(C);
            fast_issue0(S, M, F);
        }
        if (dw <= 0 || dh <= 0) {
            wave_lds_sync();
            continue;
        }

        // ---- pass 1: a pass covers 64 / cw rows of cw = 32 or 64 columns (row-major lanes); two row
        // steps per trip.  Lanes outside the window read in-bounds LDS (the tile's slack rows, the map)
        // and are masked out.  Pixels are named by their window index m = i * TP + j: the pixel's tile
        // value is tile[m + 3 * TP + 3] and its map byte map[m + TP + 1], so every ring, compass and
        // neighbour access is (tile or map) + m plus a non-negative immediate offset.
        int nf = 0, nb = 0;   // front / back entries
        // Exec for the list writes comes straight from the scalar masks (inverse ballot: no per-lane flag
        // in a VGPR, no VALU compare to rebuild it).  The order of entries inside a list does not matter
        // (survivors are emitted through the row bitmask), so a trip's back entries take
        // [lcap - nb - count, lcap - nb) in lane order.  The loop is compiled once per column width
        // (cw = 32 or 64), so the second row step's offset is an immediate.
        auto pass1 = [&](auto cw_tag) {
            constexpr int kCwShift = decltype(cw_tag)::value;
            const int cw_shift = kCwShift > 0 ? kCwShift : (dw <= 32 ? 5 : 6);
            const int col = lane & ((1 << cw_shift) - 1);
            const int rstep = 64 >> cw_shift;
            const int rlane = lane >> cw_shift;
            int t = rlane * TP + col;   // the lane's window index m in the trip's first row step
            // LDS address of list[lcap - nb] in u16 entries: a back write's byte address is one v_add_lshl from
            // it, and its update one scalar subtract of the count
            const uint32_t bend = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint16_t*)(list + lcap);
            uint32_t bptr = bend >> 1;
            const int rlane_b = rlane + rstep;
            // Thresholds per lane: +inf in the lanes past the window's columns, so a full trip's compares need no
            // column mask (two scalar ANDs per row step fewer).  The last, partial trip also takes its row masks
            // (the loop body is a lambda of the two masks, inlined twice).
            const _Float16 inf16 = __builtin_bit_cast(_Float16, (uint16_t)0x7C00);
            const _Float16 th_hi = col < dw ? f_hi : inf16, th_lo = col < dw ? f_lo : inf16;
            int rem = dh;
            auto trip = [&](auto full_tag, const unsigned long long va, const unsigned long long vb) {
                constexpr bool kFull = decltype(full_tag)::value;
                const _Float16 qa = fast_compass_q<TP>(tile + t + (3 * TP + 3));
                const _Float16 qb = fast_compass_q<TP>(tile + t + (rstep * TP + 3 * TP + 3));
                const unsigned long long hqa = ballot64(qa > th_hi), hqb = ballot64(qb > th_hi);
                const unsigned long long lqa = ballot64(qa > th_lo) & ~hqa, lqb = ballot64(qb > th_lo) & ~hqb;
                const unsigned long long mfa = kFull ? hqa : hqa & va, mba = kFull ? lqa : lqa & va;
                const unsigned long long mfb = kFull ? hqb : hqb & vb, mbb = kFull ? lqb : lqb & vb;
                // front entries are rare (about 2% of the pixels): one scalar test per trip skips both writes'
                // exec save / restore and the count updates (s_or sets SCC)
                if (mfa | mfb) {
                    if (__builtin_amdgcn_inverse_ballot_w64(mfa)) list[nf + lanes_below(mfa)] = (uint16_t)t;
                    nf += __popcll(mfa);
                    if (__builtin_amdgcn_inverse_ballot_w64(mfb)) list[nf + lanes_below(mfb)] = (uint16_t)(t + rstep * TP);
                    nf += __popcll(mfb);
                }
                // back entries (a quarter of the pixels: the mask is rarely empty) written by every lane, the
                // lanes outside the mask into their own scratch dword: an address select instead of the exec
                // save / branch / restore (FAST's time follows its scalar instruction count)
                bptr -= (uint32_t)__popcll(mba);
                *lds_select(mba, lds_u16(add_lshl1((uint32_t)lanes_below(mba), bptr)), bscratch) = (uint16_t)t;
                bptr -= (uint32_t)__popcll(mbb);
                *lds_select(mbb, lds_u16(add_lshl1((uint32_t)lanes_below(mbb), bptr)), bscratch) = (uint16_t)(t + rstep * TP);
                t += 2 * rstep * TP;
            };
            // a bottom-tested count of full trips: one scalar decrement, compare and branch per trip
            const int nfull = rem / (2 * rstep);
            if (nfull > 0) {
                int k = nfull;
                do trip(std::true_type{}, 0ull, 0ull);
                while (--k > 0);
            }
            rem -= nfull * 2 * rstep;
            if (rem > 0) trip(std::false_type{}, ballot64(rlane < rem), ballot64(rlane_b < rem));
            nb = (int)((bend >> 1) - bptr);
        };
        if constexpr (LD < 10) {   // (the 10-register prefetch kernels: 76 VGPRs, 6 waves per SIMD)
            if (dw <= 32) pass1(std::integral_constant<int, 5>{});
            else pass1(std::integral_constant<int, 6>{});
        } else {
            pass1(std::integral_constant<int, 0>{});
        }
        wave_lds_sync();
        FP_STAMP(2);

        // ---- pass 2: exact strengths of list entries [j0, j1) (front: ascending positions, back:
        // descending from lcap - 1) into the map; the entries above the lower threshold are compacted in
        // place (a trip writes at or before what it has read).  Returns the compacted count.
        auto strengths = [&](int n, bool back) {
            int n2 = 0;
            // one entry per lane per trip: the strength's 16 ring values and their arc maxima are the
            // kernel's register peak, and only ~15% of the window gets here
            // full trips (64 entries) without the tail clamp and its mask; the last, partial trip peeled (the
            // 8-register prefetch only: 67 VGPRs; the 10-register ones would drop to 6 waves per SIMD)
            if constexpr (LD < 10) {
            auto trip = [&](const int j0, auto full_tag) {
                constexpr bool kFull = decltype(full_tag)::value;
                const int ja = j0 + lane;
                const int jc = kFull ? ja : min(ja, n - 1);   // lanes past the list re-test its last entry
                const int ka = list[back ? lcap - 1 - jc : jc];
                const int sa = fast_strength<TP>(tile + ka + (3 * TP + 3));
                const unsigned long long ma = kFull ? ballot64(sa > t_lo) : ballot64(ja < n) & ballot64(sa > t_lo);
                *(uint8_t*)lds_select(ma, (uint16_t*)(map + ka + (TP + 1)), bscratch) = (uint8_t)sa;
                wave_lds_sync();   // the entries are read before the compaction overwrites the list
                *lds_select(ma, &list[back ? lcap - 1 - (n2 + lanes_below(ma)) : n2 + lanes_below(ma)], bscratch) = (uint16_t)ka;
                n2 += __popcll(ma);
            };
            int j0 = 0;
            for (; j0 + 64 <= n; j0 += 64) trip(j0, std::true_type{});
            if (j0 < n) trip(j0, std::false_type{});
            } else
            for (int j0 = 0; j0 < n; j0 += 64) {
                const int ja = j0 + lane;
                // lanes past the list re-test its last entry, masked out below
                const int pa = back ? lcap - 1 - min(ja, n - 1) : min(ja, n - 1);
                const int ka = list[pa];
                const int sa = fast_strength<TP>(tile + ka + (3 * TP + 3));
                // mask before any branch (an i1 live across a divergent branch is materialised in a VGPR)
                const unsigned long long ma = ballot64(ja < n) & ballot64(sa > t_lo);
                // both stores by every lane through address selects (the masked-off lanes into scratch)
                *(uint8_t*)lds_select(ma, (uint16_t*)(map + ka + (TP + 1)), bscratch) = (uint8_t)sa;
                wave_lds_sync();   // the entries are read before the compaction overwrites the list
                *lds_select(ma, &list[back ? lcap - 1 - (n2 + lanes_below(ma)) : n2 + lanes_below(ma)], bscratch) = (uint16_t)ka;
                n2 += __popcll(ma);
            }
            wave_lds_sync();
            return n2;
        };
        const int nf2 = strengths(nf, false);
        FP_STAMP(3);

        // ---- NMS: rounds of 64 entries over the front [0, nf2) then the back; survivors remembered
        // per round (at most 2 * 57 rounds for the 66 x 66 cap: two masks)
        auto nms = [&](int nfr, int nbk, int th, unsigned long long (&keepm)[2]) {
            const int rounds = (nfr + nbk + 63) >> 6;
            int kept_n = 0;
            keepm[0] = keepm[1] = 0;
            auto round = [&](int r, unsigned long long& km) {
                const int j = lane + (r << 6);
                // branch-free: lanes past the entries re-test the last one, masked out of the ballot
                const int jc = min(j, nfr + nbk - 1);
                const int k = list[jc < nfr ? jc : lcap - 1 - (jc - nfr)];
                const bool keep = (j < nfr + nbk) & nms_keep<TP>(map + k + (TP + 1), (uint32_t)max(th, 1));
                km |= (unsigned long long)keep << (r & 63);
                kept_n += __popcll(ballot64(keep));
            };
            // one loop per mask word, so that the word is not selected by the round at run time
            const int r1 = min(rounds, 64);
            for (int r = 0; r < r1; ++r) round(r, keepm[0]);
            for (int r = 64; r < rounds; ++r) round(r, keepm[1]);
            return kept_n;
        };
        unsigned long long keepm[2];
        int nbk = 0;
        int kept_n = nms(nf2, 0, t_ini, keepm);
        if (kept_n == 0) {   // src/ORBextractor.cc:982-987: retry the cell at minThFAST
            if (t_min < t_ini) nbk = strengths(nb, true);
            kept_n = nms(nf2, nbk, t_min, keepm);
        }
        FP_STAMP(4);

        // ---- output, row-major (cv::FAST's order) into the wave's output buffer, or straight to HBM for a
        // cell with more than the buffer holds.  Survivors of the front list alone (no fallback: about 55% of
        // KITTI cells) are already in row-major order -- pass 1 appends a trip's front entries in lane order,
        // trips in row order, and the strength pass compacts in place -- so they go out by one ballot per NMS
        // round.  A fallback cell merges front and back survivors through a per-row bitmask (the tile is dead
        // now): one bit per kept pixel, then lane i emits window row i.
        if (kept_n > 0) {
            const int xr0 = Cc.roi_x0 + 3 - kMinBorder, yr0 = Cc.roi_y0 + 3 - kMinBorder;
            const uint32_t kxb = (uint32_t)G->kp_xbits;   // packed keypoint x width (pack_kp)
            const int ci = c - c0;
            const bool buffered = !direct && obn + kept_n <= kFastObCap;   // wave-uniform
            const int rounds = (nf2 + nbk + 63) >> 6;
            // (one copy of the emission per destination, so that each store's address space is known: a pointer
            // that may be either compiles to flat stores, which wait on both counters)
            auto emit = [&](uint32_t* dst) {
                if (nbk == 0) {
                    int idx = 0;
                    auto round = [&](int r, unsigned long long kw) {
                        const bool keep = (kw >> (r & 63)) & 1ull;
                        const unsigned long long km = ballot64(keep);
                        if (km == 0ull) return;   // wave-uniform
                        if (keep) {
                            const int m = list[lane + (r << 6)];   // window (i, j) at m = i * TP + j
                            const int wi = m / TP, wj = m - wi * TP;
                            const int sc = map[m + TP + 1];
                            dst[idx + lanes_below(km)] = pack_kp((uint32_t)(xr0 + wj), (uint32_t)(yr0 + wi), (uint32_t)(sc - 1), kxb);
                        }
                        idx += __popcll(km);
                    };
                    for (int r = 0; r < min(rounds, 64); ++r) round(r, keepm[0]);
                    for (int r = 64; r < rounds; ++r) round(r, keepm[1]);
                } else {
                    for (int i = lane; i < dh; i += 64) kept[i] = 0ull;
                    wave_lds_sync();
                    auto mark = [&](int r, unsigned long long kw) {
                        if (!((kw >> (r & 63)) & 1ull)) return;
                        const int j = lane + (r << 6);
                        const int m = list[j < nf2 ? j : lcap - 1 - (j - nf2)];
                        const int wi = m / TP;
                        atomicOr(&kept[wi], 1ull << (m - wi * TP));
                    };
                    for (int r = 0; r < min(rounds, 64); ++r) mark(r, keepm[0]);
                    for (int r = 64; r < rounds; ++r) mark(r, keepm[1]);
                    wave_lds_sync();
                    // lane i emits window row i (rows <= 60): prefix sum of the row counts gives its first slot
                    const unsigned long long rowbits = lane < dh ? kept[lane] : 0ull;
                    const int cnt = __popcll(rowbits);
                    int base = 0;
                    {
                        int v = cnt;
                        // inclusive wave scan of the counts
#pragma unroll
                        for (int o = 1; o < 64; o <<= 1) {
                            const int u = __shfl_up(v, o);
                            if (lane >= o) v += u;
                        }
                        base = v - cnt;
                    }
                    unsigned long long bits = rowbits;
                    int idx = base;
                    while (bits) {
                        const int jj = __builtin_ctzll(bits);
                        bits &= bits - 1;
                        const int sc = map[(lane + 1) * TP + jj + 1];
                        dst[idx++] = pack_kp((uint32_t)(xr0 + jj), (uint32_t)(yr0 + lane), (uint32_t)(sc - 1), kxb);
                    }
                }
            };
            if (buffered) {
                if (lane == ci) c_off = obn;
                emit(obuf + obn);
                obn += kept_n;
            } else {   // rare: more than obuf holds
                direct = true;
                emit(fslots + Cc.slot_base);
            }
        }
        if (lane == c - c0) cnt_all = kept_n;
        wave_lds_sync();   // tile, map and list are rewritten by the next cell
        FP_STAMP(5);
#ifdef ORBX_FAST_PROF
        fp_acc[6] += 1;
#endif
    }
    if (obn > 0) {   // the buffered cells: one run from the wave's first cell's slot base (128-byte aligned)
        uint32_t* out = fslots + cells[c0].slot_base;
        if (lane < obn) out[lane] = obuf[lane];
        if (kFastObCap > 64 && lane + 64 < obn) out[lane + 64] = obuf[lane + 64];
        static_assert(kFastObCap <= 128, "two stores per lane");
    }
    // a cell written straight to its own slots is flagged; the buffered ones' slots follow from the counts
    if (lane < c1 - c0)
        cell_counts[(size_t)f * G->ncells + c0 + lane] = (int)((uint32_t)cnt_all | (c_off < 0 && cnt_all > 0 ? kCellDirect : 0u));
#ifdef ORBX_FAST_PROF
    if (lane == 0)
        for (int k = 0; k < 8; ++k) atomicAdd(&g_fast_prof[k], (unsigned long long)fp_acc[k]);
#endif
}
#ifdef ORBX_FAST_PROF
}  // namespace orbx
extern "C" int orbx_debug_fast_prof(unsigned long long* out, int reset)
{
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(orbx::g_fast_prof), sizeof(orbx::g_fast_prof)) != hipSuccess) return -1;
    if (reset) {
        static unsigned long long zero[8];
        if (hipMemcpyToSymbol(HIP_SYMBOL(orbx::g_fast_prof), zero, sizeof(zero)) != hipSuccess) return -1;
    }
    return 0;
}
namespace orbx {
#endif

// LDS per CU on gfx950: the occupancy a FAST launch's per-wave tiles allow, up to what the kernel's
// registers allow (<40, 8>: 71 VGPRs, 7 waves per SIMD, 28 one-wave workgroups per CU; round 3's
// realigning staging: 80 VGPRs, 24)
#ifndef ORBX_FAST_OCC
#define ORBX_FAST_OCC 28
#endif
constexpr size_t kLdsPerCu = 160 * 1024;
constexpr int kFastVgprWavesPerCu = ORBX_FAST_OCC;
static int fast_blocks_per_cu(int w, int h)
{
    return std::min((int)(kLdsPerCu / fast_wave_bytes(w, h)), kFastVgprWavesPerCu);
}

void fast_groups(Geometry& g)
{
    // The longest prefix of levels whose largest ROI keeps level 0's occupancy is launch 0; the
    // remaining levels are launch 1.  Cells are stored level by level, so each launch is a contiguous
    // range.  With the byte tile every KITTI level's ROI (up to 38x46) fits the register-limited 6 waves
    // per SIMD, so KITTI runs one launch.
    int w = g.lv[0].roi_mw, h = g.lv[0].roi_mh, split = g.nlevels;
    const int occ0 = fast_blocks_per_cu(std::max(w, 8), std::max(h, 8));
    for (int l = 1; l < g.nlevels; ++l) {
        const int nw = std::max(w, g.lv[l].roi_mw), nh = std::max(h, g.lv[l].roi_mh);
        if (fast_blocks_per_cu(nw, nh) < occ0) {
            split = l;
            break;
        }
        w = nw;
        h = nh;
    }
    g.fast_cb[0] = 0;
    g.fast_rw[0] = std::max(w, 8);
    g.fast_rh[0] = std::max(h, 8);
    if (split == g.nlevels) {
        g.fast_groups = 1;
        g.fast_cb[1] = g.ncells;
        return;
    }
    int w1 = 8, h1 = 8;
    for (int l = split; l < g.nlevels; ++l) {
        w1 = std::max(w1, g.lv[l].roi_mw);
        h1 = std::max(h1, g.lv[l].roi_mh);
    }
    g.fast_groups = 2;
    g.fast_cb[1] = g.lv[split].cell_begin;
    g.fast_cb[2] = g.ncells;
    g.fast_rw[1] = w1;
    g.fast_rh[1] = h1;
}

template <int TP, int LD>
static void fast_launch(const ExtractBufs& b, const FramePtrs& p, int cb, int ce, int rw, int rh, int cpw,
                        int batch, hipStream_t s)
{
    dim3 grid((ce - cb + cpw - 1) / cpw, batch);
    const size_t smem = fast_wave_bytes(rw, rh);
    hipFuncSetAttribute((const void*)k_fast_cells<TP, LD>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    hipLaunchKernelGGL((k_fast_cells<TP, LD>), grid, dim3(64), smem, s, b.geom, p, b.cells, b.slots, b.cell_counts,
                       cb, ce, rw, rh, cpw);
}

void launch_fast(const Geometry& g, const ExtractBufs& b, const FramePtrs& p, int batch, hipStream_t s)
{
    // small batches (the per-frame host path) are latency-bound: one cell per wave, 3x the waves
    const int cpw = fast_cells_per_wave(batch);
    // small batches: every cell in one launch sized for the largest ROI (one launch latency fewer; the
    // occupancy split only pays when the chip is full)
    if (batch <= kLatencyMaxBatch && g.fast_groups > 1) {
        const int rw = std::max(g.fast_rw[0], g.fast_rw[1]), rh = std::max(g.fast_rh[0], g.fast_rh[1]);
        const int rpp = 64 / fast_lanes_per_row(fast_tile_pitch(rw)), ld = (rh + rpp - 1) / rpp;
        if (fast_tile_pitch(rw) == 40) {
            if (ld <= 8) fast_launch<40, 8>(b, p, 0, g.ncells, rw, rh, cpw, batch, s);
            else fast_launch<40, 10>(b, p, 0, g.ncells, rw, rh, cpw, batch, s);
        } else {
            fast_launch<68, 10>(b, p, 0, g.ncells, rw, rh, cpw, batch, s);
        }
        return;
    }
    for (int i = 0; i < g.fast_groups; ++i) {
        const int cb = g.fast_cb[i], ce = g.fast_cb[i + 1];
        if (ce <= cb) continue;
        const int rw = g.fast_rw[i], rh = g.fast_rh[i];
        // register prefetch passes: the group's largest ROI in passes of whole rows (FastLaneMap)
        const int rpp = 64 / fast_lanes_per_row(fast_tile_pitch(rw)), ld = (rh + rpp - 1) / rpp;
        if (fast_tile_pitch(rw) == 40) {
            if (ld <= 8) fast_launch<40, 8>(b, p, cb, ce, rw, rh, cpw, batch, s);
            else fast_launch<40, 10>(b, p, cb, ce, rw, rh, cpw, batch, s);
        } else {
            fast_launch<68, 10>(b, p, cb, ce, rw, rh, cpw, batch, s);
        }
    }
}

// ---------------------------------------------------------------------------
// K3: DistributeOctTree (src/ORBextractor.cc:644-907), one workgroup per
// (frame, level).  Keypoints stay in registers (KPT per thread, overflow in a
// global spill array) and carry the list position of their node; nodes live in
// LDS arrays indexed by list position and are renumbered every round, so the
// std::list push_front/erase order is reproduced with prefix sums:
//   after a round the list is [children of the last split node (n4..n1), ...,
//   children of the first split node, surviving nodes in their old order].
// The phase-2 size sort breaks ties by creation order (canonical; the
// reference uses heap addresses).
// ---------------------------------------------------------------------------
constexpr int QT_NT = 512;
constexpr int QT_NW = QT_NT / 64;
#ifdef ORBX_QT_PROF
// per-level phase cycle sums (thread 0 of each workgroup): gather, init, phase-1 rounds, phase-2
// rounds, phase-2 sorts, retain, #phase-1 rounds, #phase-2 rounds, #workgroups
__device__ unsigned long long g_qt_prof[16][16];
// stamps accumulate in registers and are flushed once at the end: a global atomic per stamp would hold
// every later barrier (__syncthreads waits for the wave's outstanding memory operations)
#define QT_STAMP(slot, t0)                                                            \
    do {                                                                              \
        const long long t1_ = clock64();                                              \
        qt_acc[slot] += (unsigned long long)(t1_ - (t0));                             \
        t0 = t1_;                                                                     \
    } while (0)
#else
#define QT_STAMP(slot, t0) ((void)0)
#endif

// Inclusive wave64 prefix sum with DPP: row shifts within each 16-lane row, then row broadcasts
// (lane 15 into row 1 and 3, lane 31 into rows 2 and 3).  Six dependent VALU steps of a few cycles
// each, where a __shfl_up ladder is six ds_bpermute round trips through the LDS crossbar.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v)
{
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true);   // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true);   // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true);   // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, true);   // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return v;
}

// Exclusive scan of a[0..n) in LDS by the whole block; returns the total.  Each thread scans a
// contiguous run of per = ceil(n / NT) entries; wave totals meet in wsum, which every thread then
// reads whole (QT_NW broadcast reads) instead of waiting on one thread's serial pass.
template <int QT_NT>
__device__ uint32_t block_scan_excl(uint32_t* a, int n, uint32_t* wsum)
{
    constexpr int QT_NW = QT_NT / 64;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int per = (n + QT_NT - 1) / QT_NT;
    const int b = tid * per, e = min(n, b + per);
    uint32_t local = 0;
    for (int i = b; i < e; ++i) local += a[i];
    const uint32_t inc = wave_incl_scan(local);
    if (lane == 63) wsum[wid] = inc;
    __syncthreads();
    uint32_t before = 0, total = 0;
#pragma unroll
    for (int w = 0; w < QT_NW; ++w) {
        const uint32_t t = wsum[w];
        before += w < wid ? t : 0u;
        total += t;
    }
    uint32_t run = before + inc - local;
    for (int i = b; i < e; ++i) {
        const uint32_t t = a[i];
        a[i] = run;
        run += t;
    }
    __syncthreads();
    return total;
}

// Exclusive scan of v(0..n) into a[]; returns the total.  v is evaluated (twice) by the thread whose run
// holds the element, so a scan whose terms come from LDS already in place needs no barrier before it.
template <int QT_NT, class F>
__device__ uint32_t block_scan_fn(uint32_t* a, int n, uint32_t* wsum, F&& v)
{
    constexpr int QT_NW = QT_NT / 64;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int per = (n + QT_NT - 1) / QT_NT;
    const int b = tid * per, e = min(n, b + per);
    uint32_t local = 0;
    for (int i = b; i < e; ++i) local += v(i);
    const uint32_t inc = wave_incl_scan(local);
    if (lane == 63) wsum[wid] = inc;
    __syncthreads();
    uint32_t before = 0, total = 0;
#pragma unroll
    for (int w = 0; w < QT_NW; ++w) {
        const uint32_t t = wsum[w];
        before += w < wid ? t : 0u;
        total += t;
    }
    uint32_t run = before + inc - local;
    for (int i = b; i < e; ++i) {
        const uint32_t t = v(i);
        a[i] = run;
        run += t;
    }
    __syncthreads();
    return total;
}

__device__ __forceinline__ int next_pow2(int v)
{
    int p = 1;
    while (p < v) p <<= 1;
    return p;
}

// The slot of cell c's first candidate, in two steps around the level's exclusive count scan: before it, the
// word cell_slot_word (the cell's own slot base | kCellDirect for a directly written cell, else its wave's first
// cell's slot base), after it cell_slot_fix (the run offset: the counts of the wave's cells before c).  cpw:
// FAST's cells per wave for this batch (fast_cells_per_wave); level cell lists start at multiples of it.
static_assert(offsetof(Cell, slot_base) == 16 && alignof(Cell) >= 4 && sizeof(Cell) % 4 == 0,
              "cell_slot_base reads Cell::slot_base as dword 4");
__device__ __forceinline__ uint32_t cell_slot_base(const Cell* cells, int c)
{
    return ((const uint32_t*)(cells + c))[4];   // Cell::slot_base (a whole-dword scalar-friendly load)
}
__device__ __forceinline__ uint32_t cell_slot_word(const Cell* cells, int cb, int c, uint32_t raw, int cpw)
{
    return (raw & kCellDirect) ? (cell_slot_base(cells, cb + c) | kCellDirect) : cell_slot_base(cells, cb + c - c % cpw);
}
__device__ __forceinline__ uint32_t cell_slot_fix(uint32_t w, const uint32_t* scan, int c, int cpw)
{
    return (w & kCellDirect) ? (w & ~kCellDirect) : w + scan[c] - scan[c - c % cpw];
}

struct QtLayout {
    size_t scan, rect, cnt, srank, npos, snode, sinfo, ccnt, cpos, vprev, vnew, skey, best, wsum, sh, kpa, total;
};

// Keypoints held in LDS instead of registers (kpa, one dword per register slot) by the wide LDS-node
// templates (16+ keypoints per thread): their 32 register arrays under the 128-VGPR budget spilled to
// scratch.  Slot r of thread t is kpa[t + r * NT], so a wave's accesses are conflict-free.
__host__ __device__ constexpr int qt_kpn(int nt, int kpt, int glob) { return (!glob && kpt >= 16) ? nt * kpt : 0; }

// ixb: bytes per node index (2 with the node arrays in LDS, 4 in global memory); kpn: LDS keypoint slots
__host__ __device__ inline QtLayout qt_layout(int lcap, int cellcap, int ixb = 2, int kpn = 0)
{
    QtLayout L;
    size_t o = 0;
    auto take = [&](size_t bytes) {
        const size_t r = o;
        o += (bytes + 15) & ~(size_t)15;
        return r;
    };
    // scans: the cells' counts (cellcap), a round's split ranks (<= lcap) and phase 2's non-split flags from
    // lcap + 1 (scan2), so 2 lcap + 2 entries cover the rounds
    const int scan_n = (2 * lcap + 2 > cellcap ? 2 * lcap + 2 : cellcap) + 1;
    L.scan = take(sizeof(uint32_t) * scan_n);
    L.rect = take(sizeof(int16_t) * 4 * 2 * lcap);   // [2 buffers][4 coords][lcap]
    L.cnt = take(sizeof(uint32_t) * 2 * lcap);
    L.srank = take((size_t)ixb * lcap);
    L.npos = take((size_t)ixb * lcap);
    L.snode = take((size_t)ixb * lcap);
    L.sinfo = take(sizeof(uint32_t) * lcap);
    L.ccnt = take(sizeof(uint32_t) * 4 * lcap);
    L.cpos = take((size_t)ixb * 4 * lcap);
    L.vprev = take((size_t)ixb * lcap);
    L.vnew = take((size_t)ixb * lcap);
    L.skey = take(sizeof(uint32_t) * (lcap + 4));   // + padding to whole 16-byte groups (rank sort)
    // the retain step's per-node best keys reuse the node rectangles (dead once the rounds end: 16 bytes per
    // node against 8), which takes 8 bytes per node off the workgroup's LDS
    L.best = L.rect;
    L.wsum = take(sizeof(uint32_t) * (QT_NW + 1));
    L.sh = take(sizeof(int) * 16);
    L.kpa = take(sizeof(uint32_t) * kpn);
    L.total = o;
    return L;
}

// LDS of a global-node workgroup: the wave totals and the shared scalars only
constexpr size_t kQtGlobWsum = 0, kQtGlobSh = 64, kQtGlobSmem = 128;
// Largest LDS node layout a workgroup takes (the CU's 160 KiB); larger lists run from global memory.
// The LDS form packs a keypoint's child slot (4 * lcap) beside its node index in one 32-bit word.
constexpr size_t kQtLdsMax = 160 * 1024;
constexpr int kQtLdsMaxList = 16383;

// shared scalar slots
// SH_BIG: some phase-2 node holds more than 0xFFFF keys, so the packed (size, creation) sort key overflows
enum { SH_N = 0, SH_L, SH_PHASE, SH_M, SH_DONE, SH_KK, SH_ERR, SH_S, SH_C, SH_NEWL, SH_BIG };

// ctr[key] += 1 for every lane with key >= 0, one LDS atomic per run of equal keys in consecutive
// lanes.  Lanes hold consecutive candidates (cell order), which are spatial neighbours and mostly fall
// into the same node and quadrant: in the first split rounds thousands of keypoints meet at a handful
// of counters, and one atomic per lane serialises on them.  Called by whole waves (uniform control).
__device__ __forceinline__ void wave_run_add(uint32_t* ctr, int key)
{
    const int lane = threadIdx.x & 63;
    const int prev = __builtin_amdgcn_update_dpp(-2, key, 0x138, 0xF, 0xF, false);   // wave_shr:1, lane 0 <- -2
    const unsigned long long heads = __ballot(key != prev);
    if (key >= 0 && key != prev) {
        const unsigned long long later = lane == 63 ? 0ull : heads >> (lane + 1);
        const int len = later ? (int)__builtin_ctzll(later) + 1 : 64 - lane;
        atomicAdd(&ctr[key], (uint32_t)len);
    }
}

#ifndef ORBX_QT0_WPE
#define ORBX_QT0_WPE 4
#endif
#ifndef ORBX_QT1_WPE
#define ORBX_QT1_WPE 4
#endif
#ifndef ORBX_QT2_WPE
#define ORBX_QT2_WPE 6
#endif
// Minimum waves per SIMD (HIP's second __launch_bounds__ argument), i.e. a VGPR budget per template:
//   <512,16> (level 0) 4: 128 VGPRs (7 dwords spilled) instead of the compiler's 172, so two workgroups
//            share a CU and a 384-frame launch runs every frame at once: 106 -> 68 us;
//   <512,8>  (level 1) 5: 96 VGPRs (5 spilled) instead of 128: 43.8 -> 42.5 us;
//   <256,4>  (levels 2-7) 6: 80 VGPRs (3 spilled) instead of 100: 88 -> 70 us.
// Smaller workgroups also find room beside describe's sooner under the pipeline (+1.5% frames/s together).
// Round 3: levels 1 and 2-7 at 128 / 96 VGPRs (4 / 5 waves per SIMD, no spill): their occupancy is set by
// LDS and workgroup waves anyway (2 and 5 workgroups per CU), quadtree 0.165 -> 0.164 ms.
// FAST at 5 (94 VGPRs, no spill) measured slower (485 -> 495 us) and keeps the compiler's choice.
// Round 5: <256,4> at 6 (80 VGPRs, 5 dwords spilled) once its LDS fits six workgroups per CU (the retain
// step's keys over the node rectangles, the scan array at 2 lcap + 3 entries instead of 4 lcap + 1, the rank
// sort's keys at lcap + 4 instead of the next power of two: 28.7 -> 23.0 KB at KITTI): 135 -> 120 us per
// 1,024 frames; at 7 (72 VGPRs, 12 dwords spilled) 123 us.  With the dynamic LDS at a constant base (dyn_lds)
// none of the three spills at these budgets; <256,4> at 7 then spills 5 dwords (112 against 117 us, the
// pipelined rate unchanged).
#define ORBX_QT_WPE(NT, KPT, G) ((G) ? 1                                          \
                                 : ((NT) == 512 && (KPT) == 16) ? ORBX_QT0_WPE  \
                                 : ((NT) == 512 && (KPT) == 8) ? ORBX_QT1_WPE   \
                                 : ((NT) == 256) ? ORBX_QT2_WPE : 1)
//
// The node-list form of DistributeOctTree, one workgroup per (frame, level).
// kG: the node arrays live in the level's global region (LevelGeom::qtg_off) instead of LDS, with 32-bit
// node indices, for budgets whose node list outgrows a workgroup's LDS (e.g. Tracking's
// 2 * nFeatures initialisation extractor, src/Tracking.cc:133, at 4000 features).  The algorithm and its
// order of operations are the same; only the wave totals and the shared scalars stay in LDS.
// kWide: images wider or taller than 4096 px, whose packed keypoints split x / y at Geometry::kp_xbits; the
// standard form keeps the 12-bit split as a constant (a runtime split costs <256,4> a spilled register)
template <int QT_NT, int QT_KPT, bool kG, bool kWide>
__device__ __forceinline__ void qt_nodes(const int l, const int f, const Geometry* __restrict__ G,
                                         const Cell* __restrict__ cells, const uint32_t* __restrict__ slots,
                                         const int* __restrict__ cell_counts,
                                         uint32_t* __restrict__ spill,
                                         uint32_t* __restrict__ spill_node, uint8_t* __restrict__ gnodes,
                                         uint32_t* __restrict__ qt_out, int* __restrict__ qt_cnt,
                                         int* __restrict__ frame_counts, int* __restrict__ status, int lcap,
                                         int cellcap)
{
    // node index type; kNoneI marks "no node" (and compares above every valid rank)
    using Ix = typename std::conditional<kG, uint32_t, uint16_t>::type;
    constexpr Ix kNoneI = (Ix)~(Ix)0;
    constexpr uint32_t kPosMask = kG ? 0xFFFFFFFFu : 0xFFFFu;   // node position bits of a keypoint's node word
    uint8_t* const smem = dyn_lds();   // the dynamic LDS (no static LDS in this kernel)
    const int tid = threadIdx.x;
#ifdef ORBX_QT_PROF
    const long long qt_t0 = clock64();
    unsigned long long qt_acc[16] = {};
#endif
    const LevelGeom& LG = G->lv[l];
    const uint32_t xb = kWide ? (uint32_t)__builtin_amdgcn_readfirstlane(G->kp_xbits) : 12u;   // packed keypoint x width
    // lcap / cellcap: node-list and cell capacity of this launch's levels (qt_launch)
    constexpr bool kKpL = qt_kpn(QT_NT, QT_KPT, kG) > 0;
    const QtLayout Ly = qt_layout(lcap, cellcap, (int)sizeof(Ix), qt_kpn(QT_NT, QT_KPT, kG));
    uint32_t* kpa = (uint32_t*)(smem + Ly.kpa);
    uint8_t* nb = smem;
    if constexpr (kG) nb = gnodes + (size_t)f * G->qtg_per_frame + LG.qtg_off;
    uint32_t* scan = (uint32_t*)(nb + Ly.scan);
    int16_t* rect = (int16_t*)(nb + Ly.rect);
    uint32_t* cntb = (uint32_t*)(nb + Ly.cnt);
    Ix* srank = (Ix*)(nb + Ly.srank);
    Ix* npos = (Ix*)(nb + Ly.npos);
    Ix* snode = (Ix*)(nb + Ly.snode);
    uint32_t* sinfo = (uint32_t*)(nb + Ly.sinfo);   // per list position: split candidate flag | midlines
    uint32_t* ccnt = (uint32_t*)(nb + Ly.ccnt);
    Ix* cpos = (Ix*)(nb + Ly.cpos);
    Ix* vprev = (Ix*)(nb + Ly.vprev);
    Ix* vnew = (Ix*)(nb + Ly.vnew);
    uint32_t* skey = (uint32_t*)(nb + Ly.skey);
    unsigned long long* best = (unsigned long long*)(nb + Ly.best);
    uint32_t* wsum = (uint32_t*)(smem + (kG ? kQtGlobWsum : Ly.wsum));
    int* sh = (int*)(smem + (kG ? kQtGlobSh : Ly.sh));
    // rect buffers: [buf][coord][lcap], coord 0..3 = x0, x1, y0, y1
    auto R = [&](int buf, int coord) { return rect + (size_t)(buf * 4 + coord) * lcap; };

    // ---- 1. gather this level's FAST candidates in reference order ----------
    const int ncl = LG.ncells, cb = LG.cell_begin;
    const uint32_t* fslots = slots + (size_t)f * G->slots_per_frame;
    // LDS node arrays (rect .. wsum) are free until the candidates are in registers: the cells' slot bases
    // load there beside the counts (both in flight together), and after the scan a per-candidate owner
    // map (u16 cell index) lets every candidate's slot load go out at once, with no per-candidate binary
    // search and no dependent cell-table load.
    uint32_t* gbase = (uint32_t*)(nb + Ly.rect);
    uint16_t* owner = (uint16_t*)(gbase + ncl);
    const size_t gregion = kG ? 0 : Ly.wsum - Ly.rect;
    const bool gb_ok = !kG && ncl <= 65536 && (size_t)4 * ncl <= gregion;   // block-uniform
    const int cpw = fast_cells_per_wave(gridDim.y);   // gridDim.y = the batch FAST ran on
    for (int c = tid; c < ncl; c += QT_NT) {
        const uint32_t raw = (uint32_t)cell_counts[(size_t)f * G->ncells + cb + c];
        scan[c] = raw & ~kCellDirect;
        if (gb_ok) gbase[c] = cell_slot_word(cells, cb, c, raw, cpw);
    }
    __syncthreads();
    const int n = (int)block_scan_excl<QT_NT>(scan, ncl, wsum);
    // the slot of cell c's first candidate without the per-cell table (the search and staged forms)
    auto caddr = [&](int c) -> uint32_t {
        const uint32_t raw = (uint32_t)cell_counts[(size_t)f * G->ncells + cb + c];
        return cell_slot_fix(cell_slot_word(cells, cb, c, raw, cpw), scan, c, cpw);
    };
#ifdef ORBX_QT_PROF
    long long qt_g = qt_t0;
    QT_STAMP(4, qt_g);
#endif
    const bool omap = gb_ok && (size_t)4 * ncl + 2 * (size_t)n <= gregion;
    if (omap) {
        for (int c = tid; c < ncl; c += QT_NT) {
            const int base = (int)scan[c], cnt = (c + 1 < ncl ? (int)scan[c + 1] : n) - base;
            gbase[c] = cell_slot_fix(gbase[c], scan, c, cpw);
            for (int j = 0; j < cnt; ++j) owner[base + j] = (uint16_t)c;
        }
        __syncthreads();
    }
#ifdef ORBX_QT_PROF
    QT_STAMP(14, qt_g);
#endif
    uint32_t* fspill = spill + (size_t)f * G->spill_per_frame + (LG.slot_begin > 0 ? 0 : 0);
    uint32_t* fspill_node = spill_node + (size_t)f * G->spill_per_frame;
    // spill region of this level: levels share the frame's spill array in level order
    {
        int off = 0;
        for (int q = 0; q < l; ++q) {
            const int extra = G->lv[q].slot_cap - qt_regcap(*G, q);
            off += extra > 0 ? extra : 0;
        }
        fspill += off;
        fspill_node += off;
    }
    auto fetch = [&](int i) -> uint32_t {
        if (omap) {
            const int c = owner[i];
            return fslots[gbase[c] + (uint32_t)(i - (int)scan[c])];
        }
        int lo = 0, hi = ncl - 1;   // last cell with scan[c] <= i
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if ((int)scan[mid] <= i) lo = mid; else hi = mid - 1;
        }
        return fslots[caddr(lo) + (i - (int)scan[lo])];
    };
    uint32_t kp[kKpL ? 1 : QT_KPT], nd[QT_KPT];
    // register slot r's keypoint (candidate tid + r * QT_NT)
    auto kpr = [&](int r) -> uint32_t {
        if constexpr (kKpL) return kpa[tid + r * QT_NT];
        else return kp[r];
    };
    // kG: the level's global region is sized to stage every candidate slot (qt_prepare); every thread
    // copies whole cells into it (a cell's candidates are contiguous in its slots) and then reads its own
    // indices
    uint32_t* stage = (uint32_t*)(nb + Ly.rect);
    const bool staged = kG && (long long)n * 4 <= LG.qtg_bytes - (long long)Ly.rect;   // block-uniform
    if (staged) {
        for (int c = tid; c < ncl; c += QT_NT) {
            const int base = (int)scan[c], cnt = (c + 1 < ncl ? (int)scan[c + 1] : n) - base;
            const uint32_t* src = fslots + caddr(c);
            // 8 loads in flight per batch instead of one dependent HBM round trip per candidate
            for (int j0 = 0; j0 < cnt; j0 += 8) {
                uint32_t v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) v[u] = j0 + u < cnt ? src[j0 + u] : 0u;
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    if (j0 + u < cnt) stage[base + j0 + u] = v[u];
            }
        }
        __syncthreads();
    }
    // register slot r of thread t is candidate t + r * QT_NT (a wave's lanes hold consecutive candidates:
    // coalesced loads, conflict-free LDS slots, runs of equal nodes for wave_run_add).  The owner-map and
    // staged forms are branch-free (indices clamped, the loads of every slot in flight together); the
    // search form branches.
    if (n > 0 && (omap || staged)) {   // block-uniform
        // every slot's load in flight before the first LDS store: an LDS store waiting for its global load
        // holds the LDS reads queued behind it (the next slot's owner lookups), which serialised the slots'
        // HBM round trips (level 0: 17.9k of the workgroup's 130k cycles)
        uint32_t v[QT_KPT];
#pragma unroll
        for (int r = 0; r < QT_KPT; ++r) {
            const int ii = min(tid + r * QT_NT, n - 1);
            if (omap) {
                const int c = owner[ii];
                v[r] = fslots[gbase[c] + (uint32_t)(ii - (int)scan[c])];
            } else {
                v[r] = stage[ii];
            }
        }
#pragma unroll
        for (int r = 0; r < QT_KPT; ++r) {
            const int i = tid + r * QT_NT;
            if constexpr (kKpL) kpa[i] = i < n ? v[r] : 0u;
            else kp[r] = i < n ? v[r] : 0u;
            nd[r] = 0;
        }
    } else {
#pragma unroll
        for (int r = 0; r < QT_KPT; ++r) {
            const int i = tid + r * QT_NT;
            if constexpr (kKpL) kpa[i] = i < n ? fetch(i) : 0u;
            else kp[r] = i < n ? fetch(i) : 0u;
            nd[r] = 0;
        }
    }
    for (int i = QT_NT * QT_KPT + tid; i < n; i += QT_NT) fspill[i - QT_NT * QT_KPT] = staged ? stage[i] : fetch(i);
#ifdef ORBX_QT_PROF
    QT_STAMP(15, qt_g);
#endif
    __syncthreads();   // the staging area becomes the node arrays
#ifdef ORBX_QT_PROF
    QT_STAMP(13, qt_g);
#endif

    // visit every keypoint (register part unrolled, spill part in a loop)
    auto visit = [&](auto&& fn) {
#pragma unroll
        for (int r = 0; r < QT_KPT; ++r) {
            const int i = tid + r * QT_NT;
            if (i < n) {
                uint32_t k = kpr(r);
                fn(k, nd[r], i);
            }
        }
        for (int i = QT_NT * QT_KPT + tid; i < n; i += QT_NT) {
            uint32_t k = fspill[i - QT_NT * QT_KPT];
            uint32_t d = fspill_node[i - QT_NT * QT_KPT];
            fn(k, d, i);
            fspill_node[i - QT_NT * QT_KPT] = d;
        }
    };

#ifdef ORBX_QT_PROF
    __syncthreads();
    long long qt_t = qt_t0;
    QT_STAMP(0, qt_t);
#endif
    // ---- 2. initial nodes, src/ORBextractor.cc:650-699 ------------------------
    const int nIni = LG.nIni;
    const float hX = LG.hX;
    const int N = LG.nfeat;
    for (int i = tid; i < nIni; i += QT_NT) ccnt[i] = 0;
    __syncthreads();
    auto root_of = [&](uint32_t k) {
        int r = (int)((float)(int)kp_x(k, xb) / hX);
        return r >= nIni ? nIni - 1 : r;
    };
    const int wave_i0 = tid - (tid & 63);   // this wave's first candidate index in register slot 0
#pragma unroll
    for (int r = 0; r < QT_KPT; ++r) {
        if (wave_i0 + r * QT_NT >= n) break;   // wave-uniform
        const int i = tid + r * QT_NT;
        int key = -1;
        if (i < n) {
            key = root_of(kpr(r));
            nd[r] = (uint32_t)key;
        }
        wave_run_add(ccnt, key);
    }
    for (int i = QT_NT * QT_KPT + tid; i < n; i += QT_NT) {   // spilled candidates
        const int key = root_of(fspill[i - QT_NT * QT_KPT]);
        fspill_node[i - QT_NT * QT_KPT] = (uint32_t)key;
        atomicAdd(&ccnt[key], 1u);
    }
    __syncthreads();
    if (tid == 0) {
        int L = 0;
        for (int i = 0; i < nIni; ++i) {
            npos[i] = kNoneI;
            if (ccnt[i] > 0) {
                if (L < lcap) {
                    R(0, 0)[L] = (int16_t)(int)(hX * (float)i);
                    R(0, 1)[L] = (int16_t)(int)(hX * (float)(i + 1));
                    R(0, 2)[L] = 0;
                    R(0, 3)[L] = (int16_t)LG.qh;
                    cntb[L] = ccnt[i];
                }
                npos[i] = (Ix)L;
                ++L;
            }
        }
        sh[SH_N] = n;
        sh[SH_L] = L;
        sh[SH_PHASE] = 1;
        sh[SH_DONE] = 0;
        sh[SH_BIG] = 0;
        sh[SH_ERR] = L > lcap ? kStatusListOverflow : 0;
        if (L > lcap) sh[SH_DONE] = 1;
    }
    __syncthreads();
    visit([&](uint32_t&, uint32_t& d, int) { d = npos[d]; });

    int cur = 0;
#ifdef ORBX_QT_PROF
    __syncthreads();
    QT_STAMP(1, qt_t);
    const long long qt_r0 = qt_t;
#endif
    // A round is five barrier-separated steps (phase 1: 8 barriers, was 15):
    //   A  split set: phase 1 every node with more than one key, ranked in list order (a scan);
    //      phase 2 vPrev ranked by (size, creation) descending.  The ranking thread also writes the
    //      node's midlines (ExtractorNode::DivideNode, :572-573) and clears its four child counters.
    //   B  count pass: every keypoint's child slot (4 * split rank + quadrant) and the child counts.
    //   C  one scan of (children, expandable children) per split node, packed in 16-bit halves;
    //      phase 2 then finds how many candidates are split (kk) and the non-split ranks.
    //   D  the new list: children of split rank s at Ctot - prefix(s) - children(s) (later splits in
    //      front, n4..n1), the rest after them in order; expandable children in creation order.
    //   E  relabel every keypoint with its new list position.
    // The scans evaluate their terms from LDS already in place (block_scan_fn), so no barrier precedes them.
    uint32_t* scan2 = scan + lcap + 1;   // phase 2's non-split flags (scan[0..S] holds step C's prefixes)
    while (true) {
        __syncthreads();
        if (sh[SH_DONE]) break;
#ifdef ORBX_QT_PROF
        if (sh[SH_PHASE] == 1) qt_acc[6] += 1;
        else qt_acc[7] += 1;
#endif
        const int L = sh[SH_L];
        const int phase = sh[SH_PHASE];
        uint32_t* cntc = cntb + (size_t)cur * lcap;
        uint32_t* cntn = cntb + (size_t)(cur ^ 1) * lcap;
        int16_t *cx0 = R(cur, 0), *cx1 = R(cur, 1), *cy0 = R(cur, 2), *cy1 = R(cur, 3);
        int16_t *nx0 = R(cur ^ 1, 0), *nx1 = R(cur ^ 1, 1), *ny0 = R(cur ^ 1, 2), *ny1 = R(cur ^ 1, 3);
        const Ix* vin = cur ? vnew : vprev;   // this round's vPrev (the previous round's expandable children)
        Ix* vout = cur ? vprev : vnew;
        auto set_split = [&](int s, int p) {
            srank[p] = (Ix)s;
            snode[s] = (Ix)p;
            const int hx = (int)ceilf((float)(cx1[p] - cx0[p]) / 2);
            const int hy = (int)ceilf((float)(cy1[p] - cy0[p]) / 2);
            sinfo[p] = 0x80000000u | (uint32_t)(cx0[p] + hx) | ((uint32_t)(cy0[p] + hy) << xb);
            ccnt[4 * p] = ccnt[4 * p + 1] = ccnt[4 * p + 2] = ccnt[4 * p + 3] = 0;
        };

        // ---- A ----
        int S;   // number of candidate (split) nodes this round
        if (phase == 1) {
            S = (int)block_scan_fn<QT_NT>(scan, L, wsum, [&](int p) { return cntc[p] > 1 ? 1u : 0u; });
            for (int p = tid; p < L; p += QT_NT) {
                const int sp = (int)scan[p];
                if (cntc[p] > 1) {
                    set_split(sp, p);
                } else {
                    srank[p] = kNoneI;
                    sinfo[p] = 0u;
                }
                npos[p] = (Ix)(p - sp);   // rank among non-split nodes
            }
        } else {
            // phase 2: sort vPrev by (size, creation) descending and split from the front.  The keys
            // are unique (creation index in the low bits), so an element's place is the number of
            // larger keys: every thread ranks its elements against the whole key array by broadcast
            // 16-byte reads, with one barrier in place of a bitonic network's log2(m)^2 / 2 stages.
            const int m = sh[SH_M];
            const int m4 = (m + 3) >> 2;
            for (int k = tid; k < 4 * m4; k += QT_NT) {
                uint32_t key = 0u;   // 0: below every key
                if (k < m) {
                    const uint32_t c = cntc[vin[k]];
                    key = (c << 16) | (uint32_t)k;
                    if (c > 0xFFFFu) sh[SH_BIG] = 1;   // the packed key would wrap (reset at the round's end)
                }
                skey[k] = key;
            }
            for (int p = tid; p < L; p += QT_NT) {
                srank[p] = kNoneI;
                sinfo[p] = 0u;
            }
            __syncthreads();
            if (sh[SH_BIG] == 0 && m <= 0x10000) {   // block-uniform
                const uint4* k4 = (const uint4*)skey;
                for (int k = tid; k < m; k += QT_NT) {
                    const uint32_t key = skey[k];
                    int j = 0;
                    for (int i4 = 0; i4 < m4; ++i4) {
                        const uint4 v = k4[i4];
                        j += (int)(v.x > key) + (int)(v.y > key) + (int)(v.z > key) + (int)(v.w > key);
                    }
                    set_split(j, (int)vin[k]);
                }
            } else {
                // a node of more than 0xFFFF keys (huge levels with small budgets) or more than 2^16
                // candidates: the same order, compared as (size, creation) pairs
                for (int k = tid; k < m; k += QT_NT) {
                    const uint32_t c = cntc[vin[k]];
                    int j = 0;
                    for (int k2 = 0; k2 < m; ++k2) {
                        const uint32_t c2 = cntc[vin[k2]];
                        j += (int)(c2 > c || (c2 == c && k2 > k));
                    }
                    set_split(j, (int)vin[k]);
                }
            }
            S = m;
        }
        __syncthreads();
        QT_STAMP(3, qt_t);

        // ---- B: a keypoint's child slot is 4 * (its node's list position) + quadrant; the candidate flag
        // and quadrant are kept in its node word beside the position for the relabel (bit 18, bits 16-17).
        // kG: node words hold the full position, and the relabel recomputes the child slot (sinfo is
        // unchanged until then).
        auto child_key = [&](uint32_t k, uint32_t d) {
            const uint32_t p = d & kPosMask;
            const uint32_t w = sinfo[p];
            if (!(w & 0x80000000u)) return -1;
            return (int)(4 * p + (kp_x(k, xb) >= kp_x(w, xb) ? 1u : 0u) + (kp_y(k, xb) >= kp_y(w, xb) ? 2u : 0u));
        };
        if constexpr (!kG) {
            // keys first, branch-free (every slot's node and keypoint LDS reads in flight together; a slot
            // past n has node 0, a valid index, and is masked), then the counts: interleaved, each slot's
            // loads would wait behind the previous slot's atomics
            uint32_t wv[QT_KPT], kv[QT_KPT];
#pragma unroll
            for (int r = 0; r < QT_KPT; ++r) wv[r] = sinfo[nd[r] & 0xFFFFu];
#pragma unroll
            for (int r = 0; r < QT_KPT; ++r) kv[r] = kpr(r);
#pragma unroll
            for (int r = 0; r < QT_KPT; ++r) {
                const int i = tid + r * QT_NT;
                const uint32_t w = wv[r], k = kv[r];
                const bool cand = i < n && (w & 0x80000000u);
                const uint32_t qd = (kp_x(k, xb) >= kp_x(w, xb) ? 1u : 0u) + (kp_y(k, xb) >= kp_y(w, xb) ? 2u : 0u);
                nd[r] = (nd[r] & 0xFFFFu) | (cand ? 0x40000u | (qd << 16) : 0u);
            }
#pragma unroll
            for (int r = 0; r < QT_KPT; ++r) {
                if (wave_i0 + r * QT_NT >= n) break;   // wave-uniform
                wave_run_add(ccnt, (nd[r] & 0x40000u) ? (int)(4 * (nd[r] & 0xFFFFu) + ((nd[r] >> 16) & 3u)) : -1);
            }
        } else {
#pragma unroll
            for (int r = 0; r < QT_KPT; ++r) {
                if (wave_i0 + r * QT_NT >= n) break;   // wave-uniform
                const int i = tid + r * QT_NT;
                wave_run_add(ccnt, i < n ? child_key(kpr(r), nd[r]) : -1);
            }
        }
        for (int i = QT_NT * QT_KPT + tid; i < n; i += QT_NT) {
            uint32_t& d = fspill_node[i - QT_NT * QT_KPT];
            const int key = child_key(fspill[i - QT_NT * QT_KPT], d);
            if constexpr (!kG) d = (d & 0xFFFFu) | (key >= 0 ? 0x40000u | ((uint32_t)(key & 3) << 16) : 0u);
            if (key >= 0) atomicAdd(&ccnt[key], 1u);
        }
        if (tid == 0) sh[SH_KK] = S;   // phase 2: lowered in step C by the split that reaches N
        __syncthreads();
        QT_STAMP(9, qt_t);

        // ---- C: children (low half) and expandable children (high half) per split rank ----
        auto kids = [&](int s) -> uint32_t {
            const int p = snode[s];
            uint32_t v = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t c = ccnt[4 * p + q];
                v += (c > 0 ? 1u : 0u) + (c > 1 ? 0x10000u : 0u);
            }
            return v;
        };
        const uint32_t T = block_scan_fn<QT_NT>(scan, S, wsum, kids);
        int kk = S;
        uint32_t pre = T;   // prefix at kk
        if (phase == 2) {
            // how many candidates are actually split: the size after splitting j grows with j (a split
            // node leaves >= 1 child), so the one j that crosses N writes
            for (int j = tid; j < S; j += QT_NT) {
                const int cs = (int)(kids(j) & 0xFFFFu), sj = (int)(scan[j] & 0xFFFFu);
                if (L + sj + cs - (j + 1) >= N && L + sj - j < N) sh[SH_KK] = j + 1;
            }
            __syncthreads();
            kk = sh[SH_KK];
            if (kk < S) pre = scan[kk];
            block_scan_fn<QT_NT>(scan2, L, wsum, [&](int p) {
                return (srank[p] != kNoneI && (int)srank[p] < kk) ? 1u : 0u;
            });
        }
        QT_STAMP(10, qt_t);
        const int Ctot = (int)(pre & 0xFFFFu), nexp = (int)(pre >> 16);
        const int newL = Ctot + (L - kk);
        if (newL > lcap) {
            if (tid == 0) {
                sh[SH_ERR] |= kStatusListOverflow;
                sh[SH_DONE] = 1;
            }
            continue;
        }

        // ---- D ----
        for (int s = tid; s < kk; s += QT_NT) {
            const int p = snode[s];
            const uint32_t ps = scan[s];
            uint32_t c4[4];
            int cs = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                c4[q] = ccnt[4 * p + q];
                cs += c4[q] > 0;
            }
            const int pos0 = Ctot - (int)(ps & 0xFFFFu) - cs;   // later splits are pushed in front
            int e = (int)(ps >> 16);
            const uint32_t w = sinfo[p];
            const int mx = (int)kp_x(w, xb), my = (int)kp_y(w, xb);
            const int x0 = cx0[p], x1 = cx1[p], y0 = cy0[p], y1 = cy1[p];
            int np = pos0 + cs;   // n1 lands last (it was pushed first)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t c = c4[q];
                if (c == 0) continue;   // (no keypoint looks its slot up)
                --np;
                cpos[4 * p + q] = (Ix)np;
                nx0[np] = (int16_t)((q & 1) ? mx : x0);
                nx1[np] = (int16_t)((q & 1) ? x1 : mx);
                ny0[np] = (int16_t)((q & 2) ? my : y0);
                ny1[np] = (int16_t)((q & 2) ? y1 : my);
                cntn[np] = c;
                if (c > 1) vout[e++] = (Ix)np;   // creation order: split rank, then n1..n4
            }
        }
        for (int p = tid; p < L; p += QT_NT) {
            const bool split = srank[p] != kNoneI && (int)srank[p] < kk;
            if (!split) {
                const int np = Ctot + (phase == 1 ? (int)npos[p] : p - (int)scan2[p]);
                npos[p] = (Ix)np;
                nx0[np] = cx0[p];
                nx1[np] = cx1[p];
                ny0[np] = cy0[p];
                ny1[np] = cy1[p];
                cntn[np] = cntc[p];
                // a phase-2 candidate past kk keeps its keypoints: its child slots all lead to its new place
                if (srank[p] != kNoneI) cpos[4 * p] = cpos[4 * p + 1] = cpos[4 * p + 2] = cpos[4 * p + 3] = (Ix)np;
            }
        }
        if (tid == 0) {
            // src/ORBextractor.cc:793-803 and :871-872 (read at the next round's start)
            sh[SH_L] = newL;
            if (newL >= N || newL == L) {
                sh[SH_DONE] = 1;
            } else if (phase == 1) {
                if (newL + 3 * nexp > N) sh[SH_PHASE] = 2;
            }
            sh[SH_M] = nexp;
            sh[SH_BIG] = 0;
        }
        __syncthreads();
        QT_STAMP(11, qt_t);

        // ---- E: relabel keypoints with their new list position ----
        if constexpr (!kG) {
            // register slots branch-free: one LDS read per slot from the child or the node table, every
            // slot's read in flight together; slots past n keep node 0
            uint32_t v[QT_KPT];
#pragma unroll
            for (int r = 0; r < QT_KPT; ++r) {
                const uint32_t d = nd[r];
                const Ix* src = (d & 0x40000u) ? cpos + (4 * (d & 0xFFFFu) + ((d >> 16) & 3u)) : npos + (d & 0xFFFFu);
                v[r] = (uint32_t)*src;
            }
#pragma unroll
            for (int r = 0; r < QT_KPT; ++r) nd[r] = tid + r * QT_NT < n ? v[r] : 0u;
            for (int i = QT_NT * QT_KPT + tid; i < n; i += QT_NT) {   // spilled keypoints
                uint32_t& d = fspill_node[i - QT_NT * QT_KPT];
                const int ck = (d & 0x40000u) ? (int)(4 * (d & 0xFFFFu) + ((d >> 16) & 3u)) : -1;
                d = ck >= 0 ? (uint32_t)cpos[ck] : (uint32_t)npos[d & kPosMask];
            }
        } else {
            visit([&](uint32_t& k, uint32_t& d, int) {
                // child slot from the count pass, -1 if the node was not a candidate
                const int ck = child_key(k, d);
                d = ck >= 0 ? (uint32_t)cpos[ck] : (uint32_t)npos[d & kPosMask];
            });
        }
        QT_STAMP(12, qt_t);
        cur ^= 1;
    }

#ifdef ORBX_QT_PROF
    // (the round loop's time: stamped at each round's end below would need the phase; charge the
    // whole loop to slot 2 and let the caller split it with the sort and round counts)
    qt_acc[2] += (unsigned long long)(clock64() - qt_r0);
    qt_t = clock64();
#endif
    // ---- 4. retain the best keypoint per node (first max wins), :882-906 -----
    const int L = sh[SH_L];
    const bool ok = sh[SH_ERR] == 0;
    for (int p = tid; p < L && ok; p += QT_NT) best[p] = 0ull;
    __syncthreads();
    if (ok) {
        visit([&](uint32_t& k, uint32_t& d, int i) {
            const unsigned long long key = ((unsigned long long)(k >> 24) << 56) |
                                           ((unsigned long long)(0xFFFFFFu - (uint32_t)i) << 32) |
                                           (unsigned long long)(k & 0xFFFFFFu);
            atomicMax(&best[d], key);
        });
    }
    __syncthreads();
    const int outn = ok ? (L < LG.cap ? L : LG.cap) : 0;
    uint32_t* out = qt_out + (size_t)f * G->out_per_frame + LG.out_off;
    for (int p = tid; p < outn; p += QT_NT) {
        const unsigned long long key = best[p];
        const uint32_t x = kp_x((uint32_t)key, xb) + kMinBorder;
        const uint32_t y = kp_y((uint32_t)key, xb) + kMinBorder;
        out[p] = pack_kp(x, y, (uint32_t)(key >> 56), xb);
    }
    if (tid == 0) {
        qt_cnt[(size_t)f * G->nlevels + l] = outn;
#ifdef ORBX_QT_PROF
        QT_STAMP(5, qt_t);
        qt_acc[8] = 1;
        for (int k = 0; k < 16; ++k) atomicAdd(&g_qt_prof[l][k], qt_acc[k]);
#endif
        atomicAdd(&frame_counts[f], outn);
        int err = sh[SH_ERR];
        if (ok && L > LG.cap) err |= kStatusOutOverflow;
        if (err) atomicOr(status, err);
    }
}

template <int QT_NT, int QT_KPT, bool kG, bool kWide>
__global__ __launch_bounds__(QT_NT, ORBX_QT_WPE(QT_NT, QT_KPT, kG)) void k_quadtree(
    int level0, const Geometry* __restrict__ G, const Cell* __restrict__ cells, const uint32_t* __restrict__ slots,
    const int* __restrict__ cell_counts, uint32_t* __restrict__ spill,
    uint32_t* __restrict__ spill_node, uint8_t* __restrict__ gnodes, uint32_t* __restrict__ qt_out,
    int* __restrict__ qt_cnt, int* __restrict__ frame_counts, int* __restrict__ status, int lcap, int cellcap)
{
    qt_nodes<QT_NT, QT_KPT, kG, kWide>(level0 + blockIdx.x, blockIdx.y, G, cells, slots, cell_counts, spill,
                                spill_node, gnodes, qt_out, qt_cnt, frame_counts, status, lcap, cellcap);
}

template <int NT, int KPT, bool kG>
static void qt_launch(const Geometry& g, const ExtractBufs& b, int* frame_counts, const QtGroup& q, int batch,
                      hipStream_t s)
{
    const size_t smem = kG ? kQtGlobSmem : qt_layout(q.lcap, q.cellcap, 2, qt_kpn(NT, KPT, 0)).total;
    auto launch = [&](auto kern) {
        hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
        hipLaunchKernelGGL(kern, dim3(q.nl, batch), dim3(NT), smem, s, q.l0, b.geom, b.cells, b.slots, b.cell_counts,
                           b.spill, b.spill_node, b.qt_nodes, b.qt_out, b.qt_cnt, frame_counts, b.status, q.lcap,
                           q.cellcap);
    };
    if (g.kp_xbits == 12) launch(k_quadtree<NT, KPT, kG, false>);
    else launch(k_quadtree<NT, KPT, kG, true>);
}

// Launch groups.  A group's node capacity is the largest cap + 4 of its levels: a level's list never holds
// more than cap + 3 nodes (phase 1 stops before L + 3 * expandable exceeds N, phase 2 once L >= N;
// cap >= max(N + 2, 4 * nIni)), so the coarse levels' workgroups take less LDS than level 0's and more of
// them fit on a CU.
int qt_plan(const Geometry& g, int batch, QtGroup* out)
{
    auto caps = [&](QtGroup& q) {
        q.lcap = 8;
        q.cellcap = 1;
        for (int l = q.l0; l < q.l0 + q.nl; ++l) {
            q.lcap = std::max(q.lcap, g.lv[l].cap + 4);
            q.cellcap = std::max(q.cellcap, g.lv[l].ncells);
        }
    };
    bool anyg = false;
    for (int l = 0; l < g.nlevels; ++l) anyg |= g.lv[l].qt_glob != 0;
    // Small batches (the per-frame host path): one launch of the level-0 kernel over every level, so
    // the levels run concurrently instead of as dependent launches (latency, not throughput).
    // A level run with more register capacity than qt_regcap(g, l) spills less than its region holds.
    if (batch <= kQtMergedMaxBatch && !anyg) {
        QtGroup q{0, g.nlevels, 512, g.qt_kpt0, 0, 0, 0};
        caps(q);
        if (qt_layout(q.lcap, q.cellcap, 2, qt_kpn(q.nt, q.kpt, 0)).total <= kQtLdsMax) {
            out[0] = q;
            return 1;
        }
    }
    // one launch per run of consecutive levels with the same configuration; the launched template is
    // exactly qt_nt / qt_kpt, which size the spill regions
    int n = 0;
    for (int l0 = 0; l0 < g.nlevels;) {
        const int nt = qt_nt(g, l0), kpt = qt_kpt(g, l0), gl = g.lv[l0].qt_glob;
        int l1 = l0 + 1;
        while (l1 < g.nlevels && qt_nt(g, l1) == nt && qt_kpt(g, l1) == kpt && g.lv[l1].qt_glob == gl) ++l1;
        QtGroup q{l0, l1 - l0, nt, kpt, gl, 0, 0};
        caps(q);
        out[n++] = q;
        l0 = l1;
    }
    return n;
}

bool qt_prepare(Geometry& g)
{
    // a level's own node list decides; a group whose shared capacity outgrows LDS moves to global too
    for (int l = 0; l < g.nlevels; ++l) {
        const int lc = g.lv[l].cap + 4;
        const int kpn = qt_kpn(l == 0 ? 512 : 256, l == 0 ? g.qt_kpt0 : 4, 0);
        g.lv[l].qt_glob = lc > kQtLdsMaxList || qt_layout(lc, g.lv[l].ncells, 2, kpn).total > kQtLdsMax;
        g.lv[l].qtg_off = g.lv[l].qtg_bytes = 0;
    }
    QtGroup grp[kQtMaxGroups];
    for (;;) {
        const int ng = qt_plan(g, 1 << 30, grp);
        bool moved = false;
        for (int i = 0; i < ng; ++i) {
            if (grp[i].glob || qt_layout(grp[i].lcap, grp[i].cellcap, 2, qt_kpn(grp[i].nt, grp[i].kpt, 0)).total <= kQtLdsMax)
                continue;
            for (int l = grp[i].l0; l < grp[i].l0 + grp[i].nl; ++l) g.lv[l].qt_glob = 1;
            moved = true;
        }
        if (moved) continue;
        // global regions: the group's node layout with 32-bit indices, or room to stage every candidate
        // slot of the level (the gather reads them in index order from there), whichever is larger
        long long off = 0;
        for (int i = 0; i < ng; ++i) {
            if (!grp[i].glob) continue;
            const QtLayout Ly = qt_layout(grp[i].lcap, grp[i].cellcap, 4);
            for (int l = grp[i].l0; l < grp[i].l0 + grp[i].nl; ++l) {
                long long bytes = std::max((long long)Ly.total, (long long)Ly.rect + 4LL * g.lv[l].slot_cap);
                bytes = (bytes + 255) & ~255LL;
                g.lv[l].qtg_off = off;
                g.lv[l].qtg_bytes = bytes;
                off += bytes;
            }
        }
        g.qtg_per_frame = off;
        return true;
    }
}

#ifdef ORBX_QT_PROF
}  // namespace orbx
extern "C" int orbx_debug_qt_prof(unsigned long long* out, int reset)
{
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(orbx::g_qt_prof), sizeof(orbx::g_qt_prof)) != hipSuccess) return -1;
    if (reset) {
        static unsigned long long zero[16][16];
        if (hipMemcpyToSymbol(HIP_SYMBOL(orbx::g_qt_prof), zero, sizeof(zero)) != hipSuccess) return -1;
    }
    return 0;
}
namespace orbx {
#endif

void launch_quadtree(const Geometry& g, const ExtractBufs& b, int* frame_counts, int batch, hipStream_t s)
{
    QtGroup grp[kQtMaxGroups];
    const int ng = qt_plan(g, batch, grp);
    for (int i = 0; i < ng; ++i) {
        const QtGroup& q = grp[i];
        if (q.glob) qt_launch<kQtGlobNT, kQtGlobKPT, true>(g, b, frame_counts, q, batch, s);
        else if (q.nt == 512 && q.kpt == 24) qt_launch<512, 24, false>(g, b, frame_counts, q, batch, s);
        else if (q.nt == 512 && q.kpt == 16) qt_launch<512, 16, false>(g, b, frame_counts, q, batch, s);
        else if (q.nt == 512) qt_launch<512, 8, false>(g, b, frame_counts, q, batch, s);
        else qt_launch<256, 4, false>(g, b, frame_counts, q, batch, s);
    }
}

// ---------------------------------------------------------------------------
// K4: a wave describes kDescPerWave consecutive retained keypoints.
//   raw   the 43-row neighbourhood of the keypoint in LDS, 48 B per row.
//         Interior keypoints arrive by LDS-DMA (global_load_lds_dwordx4: three
//         instructions of 16-byte pieces, three per row, so row r starts at
//         byte sh_r = (src + r*pitch) & 3 of its LDS row);
//         border keypoints are filled with reflect-101 bytes at shift 0.  The next keypoint's DMA is issued as soon as the
//         current one's raw reads are done, so it lands under the BRIEF work.
//   angle IC_Angle: u*I and v*I over the 749-pixel disc as per-lane column
//         sums (lane = disc column, half-wave = upper/lower rows), wave
//         reduction, then cv::fastAtan2 (src/ORBextractor.cc:84-128).
//   blur  GaussianBlur 7x7 integer kernel [18 34 49 55 49 34 18], >>16
//         (SURVEY.md A.3): the horizontal pass is v_dot4_u32_u8 on 4 output
//         columns x 2 rows per lane, stored transposed as u16 row pairs; the
//         vertical pass is evaluated only at the 512 BRIEF sample points with
//         four v_dot2_u32_u16 each.
//   BRIEF fmaf sample coordinates, 256 tests -> four __ballot
//         words = the descriptor's little-endian u64 words (:141-192).
// ---------------------------------------------------------------------------
constexpr int kRawP = 48;                             // LDS row pitch (bytes): the 43 columns + shift slack
constexpr int kRawRows = 44;                          // 43 rows used (row 43 repeats row 42)
constexpr int kRawSlots = kRawRows * kRawP / 4;
// row-blurred, transposed: [col][row pairs], 23 dwords per column (22 hold the 44 rows; the odd pitch spreads
// the horizontal pass's column stores over the banks: 48 LDS-array cycles per keypoint against 68 at 22, and
// 98 against 108 for the blur reads of tools/gen/brief_slots.py's slots)
constexpr int kTCols = 40, kTP = 23;
#ifndef ORBX_DESC_KPW
#define ORBX_DESC_KPW 4
#endif
constexpr int kDescPerWave = ORBX_DESC_KPW;           // keypoints per wave (lane state set up once per wave)
#ifndef ORBX_DESC_WAVES
#define ORBX_DESC_WAVES 1
#endif
// waves per describe workgroup: one, so a workgroup's LDS (6.3 KB) frees as soon as its own keypoints are done
// and no wave waits on slower siblings (4 waves: 863 us per 384 frames, 2: 815, 1: 768; pipelined 169.1k ->
// 176.4k frames/s)
constexpr int kDescWaves = ORBX_DESC_WAVES;

// Horizontal-pass items (row pair rp << 8 | column group cg) that BRIEF can read: a sample
// (18 + xx, 18 + yy) has |(x, y)| <= 18.39 before rounding (the pattern's largest radius), so a
// column group needs only the row pairs its disc chord reaches, plus the 7-tap reach of
// blur_acc.  189 of the 22 x 10 items: three per lane, row-pair major so that the lanes of a
// load read neighbouring raw dwords (distinct LDS banks).
__constant__ uint16_t c_blur_items[192] = {2,3,4,5,6,257,258,259,260,261,262,263,513,514,515,516,517,518,519,768,769,770,771,772,773,774,775,776,1024,1025,1026,1027,1028,1029,1030,1031,1032,1280,1281,1282,1283,1284,1285,1286,1287,1288,1536,1537,1538,1539,1540,1541,1542,1543,1544,1545,1792,1793,1794,1795,1796,1797,1798,1799,1800,1801,2048,2049,2050,2051,2052,2053,2054,2055,2056,2057,2304,2305,2306,2307,2308,2309,2310,2311,2312,2313,2560,2561,2562,2563,2564,2565,2566,2567,2568,2569,2816,2817,2818,2819,2820,2821,2822,2823,2824,2825,3072,3073,3074,3075,3076,3077,3078,3079,3080,3081,3328,3329,3330,3331,3332,3333,3334,3335,3336,3337,3584,3585,3586,3587,3588,3589,3590,3591,3592,3593,3840,3841,3842,3843,3844,3845,3846,3847,3848,3849,4096,4097,4098,4099,4100,4101,4102,4103,4104,4352,4353,4354,4355,4356,4357,4358,4359,4360,4609,4610,4611,4612,4613,4614,4615,4616,4865,4866,4867,4868,4869,4870,4871,5122,5123,5124,5125,5126,5127,5379,5380,5381,5382,65535,65535,65535};
constexpr int kUmax[16] = {15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3};
// GaussianBlur(7x7, sigma 2)'s integer taps per ORBX_BLUR_* mode: OpenCV <= 3.4.1 (scalar and
// SSE2 column passes) converts getGaussianKernel's floats at x256, [18 34 49 55 49 34 18] (sum 257); 3.4.6+ / 4.x's
// bit-exact GaussianBlur carries the rounding error inwards and closes the sum at 256, [18 34 48 56 48 34 18]
__host__ __device__ constexpr uint32_t blur_tap(int bm, int t)
{
    return t == 2 || t == 4 ? (bm == ORBX_BLUR_BITEXACT ? 48u : 49u)
                            : t == 3 ? (bm == ORBX_BLUR_BITEXACT ? 56u : 55u) : (t == 1 || t == 5 ? 34u : 18u);
}
// GaussianBlur's 7 taps starting at byte `off` of four consecutive raw dwords: the weight bytes of dword d
__host__ __device__ constexpr uint32_t blur_wshift(int off, int d, int bm = ORBX_BLUR_SCALAR)
{
    uint32_t w = 0;
    for (int b = 0; b < 4; ++b) {
        const int t = 4 * d + b - off;
        if (t >= 0 && t < 7) w |= blur_tap(bm, t) << (8 * b);
    }
    return w;
}
constexpr int kPattern[1024] = {
#include "orb_pattern.inc"
};
#include "orb_slots.inc"

// Keypoint-independent lane state of k_describe, a function of the lane alone, built at compile time
// (the kernel loads it instead of computing ~235 VALU instructions per wave).
//   IC_Angle: lane 2i + h owns disc row v = i - 15 (i < 31), half h: u = -15..0 or 1..15, as 4
//   realigned dwords of the raw row dotted (v_dot4_u32_u8) with per-lane weights that are zero
//   outside |u| <= umax[|v|]: w1 = (u + 16) for m10 (minus 16 * sum I), w0 = 1 for sum I.
//   rBRIEF: the pattern's 512 points hold 375 distinct ones.  Each is blurred once, in slot 64 q + lane (lane,
//   round q < 6) of a u16 table; test m = 64 wd + lane (wd = q >> 1) reads its two samples (e = q & 1) from
//   slot byte offsets rd[q].  Which point sits in which slot (orb_slots.inc, tools/gen/brief_slots.py) keeps
//   each half-round's 32 points a compact cluster of the pattern, so their blur reads share LDS addresses
//   and spread over the banks at any keypoint angle (98 LDS-array cycles per keypoint against 156 for the
//   points in order of first use, 212 for the 512 points of round 4), and orders lanes inside each
//   half-round for the table reads' banks.
constexpr int kDescSlots = 6;   // distinct sample points per lane (384 slots >= 375)
struct DescLane {
    uint32_t w1[4], w0[4];
    float upx[kDescSlots], upy[kDescSlots];
    uint32_t rd[8];
};
struct DescLaneTable {
    DescLane l[64];
};
constexpr DescLaneTable make_desc_lanes()
{
    DescLaneTable t{};
    for (int lane = 0; lane < 64; ++lane) {
        const int icv = lane >> 1, ich = lane & 1, vrow = icv - 15;
        const int rmax = icv < 31 ? kUmax[vrow < 0 ? -vrow : vrow] : -1;
        for (int k = 0; k < 4; ++k)
            for (int b = 0; b < 4; ++b) {
                const int uu = (ich ? 1 : -15) + 4 * k + b;
                if (uu <= (ich ? 15 : 0) && (uu < 0 ? -uu : uu) <= rmax) {
                    t.l[lane].w1[k] |= (uint32_t)(uu + 16) << (8 * b);
                    t.l[lane].w0[k] |= 1u << (8 * b);
                }
            }
    }
    for (int lane = 0; lane < 64; ++lane) {
        for (int q = 0; q < kDescSlots; ++q) {
            const int i = kSlotPt[64 * q + lane];
            t.l[lane].upx[q] = (float)kPattern[2 * i];
            t.l[lane].upy[q] = (float)kPattern[2 * i + 1];
        }
        for (int q = 0; q < 8; ++q) {
            const int m = (q >> 1) * 64 + lane, e = q & 1;
            t.l[lane].rd[q] = 2u * (uint32_t)kPtSlot[2 * m + e];
        }
    }
    return t;
}
// every pattern point's slot holds that point
constexpr bool desc_slots_ok()
{
    for (int i = 0; i < 512; ++i) {
        const int s = kPtSlot[i];
        if (s < 0 || s >= 64 * kDescSlots) return false;
        const int j = kSlotPt[s];
        if (kPattern[2 * j] != kPattern[2 * i] || kPattern[2 * j + 1] != kPattern[2 * i + 1]) return false;
    }
    return true;
}
static_assert(desc_slots_ok(), "orb_slots.inc does not match orb_pattern.inc");
__constant__ DescLaneTable c_desc_lanes = make_desc_lanes();

__device__ __forceinline__ int reflect101(int p, int len)
{
    if (len == 1) return 0;
    while (p < 0 || p >= len) p = p < 0 ? -p : 2 * len - 2 - p;
    return p;
}

// wave sum: row (16-lane) sums with DPP, then the four rows by readlane (all lanes active)
__device__ __forceinline__ int wave_sum(int v)
{
    v += __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, true);    // quad_perm [1,0,3,2]
    v += __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, true);    // quad_perm [2,3,0,1]
    v += __builtin_amdgcn_mov_dpp(v, 0x141, 0xF, 0xF, true);   // row_half_mirror
    v += __builtin_amdgcn_mov_dpp(v, 0x140, 0xF, 0xF, true);   // row_mirror
    return __builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16) +
           __builtin_amdgcn_readlane(v, 32) + __builtin_amdgcn_readlane(v, 48);
}

// Sample coordinates as float bits: fl + 1.5 * 2^23 rounds fl to the nearest integer, ties to even
// (one f32 addition into [2^23, 2^24), whose ulp is 1; the magic number is even, so the tie parity
// is fl's), exactly __float2int_rn for |fl| < 2^22, and leaves that integer in the low mantissa
// bits: bits = 0x4B400000 + round(fl).  The blur lookup indexes with these bits directly.
constexpr float kRoundMagic = 12582912.0f;
constexpr uint32_t kRoundBits = 0x4B400000u;

// blurred value at patch row 18 + yy, column 18 + xx (|xx|, |yy| <= 19, given as kRoundMagic
// bits by, bx): sum_t k[t] * rowblur[y+t][x], + 2^15 (the >> 16 rounding) folded into the sum.
// The dword index is (18 + xx) * kTP + ((18 + yy) >> 1), in wrapping u32 arithmetic on the bits of
// bx (its low 24 bits are 0x400000 + xx) and by (bits 1..23: 0x200000 + ((18 + yy) >> 1) - 9).
// The LDS byte address in three VALU: bfe of by's bits 1..23 (0x200000 + (yy >> 1)), shifted and added to
// mad24(bx, 4 kTP, C) with C = rowT + 4 (9 - 0x200000 + (18 - 0x400000) kTP) (mod 2^32); the compiler's
// form of (by >> 1) + bx * kTP + rowT took five.
constexpr uint32_t kBlurByte0 = 4u * (9u - 0x200000u + (18u - 0x400000u) * (uint32_t)kTP);
template <int kBM>
__device__ __forceinline__ uint32_t blur_acc(uint32_t C, uint32_t by, uint32_t bx)
{
    const uint32_t t = __umul24(bx, 4u * (uint32_t)kTP) + C, f = __builtin_amdgcn_ubfe(by, 1, 23);
    uint32_t a;
    // one v_lshl_add_u32 (the compiler rewrites (f << 2) + t as (by << 1) & mask plus an add)
    asm("v_lshl_add_u32 %0, %1, 2, %2" : "=v"(a) : "v"(f), "v"(t));
    const __attribute__((address_space(3))) uint32_t* col = (const __attribute__((address_space(3))) uint32_t*)(uintptr_t)a;
    const uint32_t d0 = col[0], d1 = col[1], d2 = col[2], d3 = col[3];
    // rows y..y+6 are (d0.lo d0.hi d1.lo d1.hi d2.lo d2.hi d3.lo) for even y and (d0.hi .. d3.hi) for odd y:
    // shifting the dword chain right by 16 bits for odd y (v_alignbit uses its shift's low five bits, so
    // by << 4 is that shift) leaves the same weights for both parities -- in SGPRs, where the per-lane
    // selection of round 4 (four v_cndmask, a test) held both weight sets in VGPRs
    const uint32_t sh = by << 4;
    const uint32_t e0 = __builtin_amdgcn_alignbit(d1, d0, sh), e1 = __builtin_amdgcn_alignbit(d2, d1, sh);
    const uint32_t e2 = __builtin_amdgcn_alignbit(d3, d2, sh), e3 = d3 >> (sh & 31u);
    constexpr unsigned short k1 = (unsigned short)blur_tap(kBM, 2), k3 = (unsigned short)blur_tap(kBM, 3);
    uint32_t acc = __builtin_amdgcn_udot2(as_us2(e0), ushort2_t{18, 34}, 1u << 15, false);
    acc = __builtin_amdgcn_udot2(as_us2(e1), ushort2_t{k1, k3}, acc, false);
    acc = __builtin_amdgcn_udot2(as_us2(e2), ushort2_t{k1, 34}, acc, false);
    return __builtin_amdgcn_udot2(as_us2(e3), ushort2_t{18, 0}, acc, false);
}
#ifndef ORBX_DESC_WPE
#define ORBX_DESC_WPE 1
#endif
// kBM: ORBX_BLUR_* (the kernel taps; ORBX_BLUR_SSE2 also rounds the column pass half to even on the level's
// columns below w & ~3, as SymmColumnVec_32s8u does)
template <int kBM>
__global__ __launch_bounds__(64 * kDescWaves, ORBX_DESC_WPE) void k_describe(const Geometry* __restrict__ G, FramePtrs P,
                                               const uint32_t* __restrict__ qt_out,
                                               const int* __restrict__ qt_cnt,
                                               orbx_keypoint* __restrict__ kps, uint8_t* __restrict__ desc,
                                               int cap, int* __restrict__ status, int kpw)
{
    __shared__ __attribute__((aligned(16))) uint32_t s_raw[kDescWaves][kRawSlots];
    __shared__ __attribute__((aligned(16))) uint32_t s_rowT[kDescWaves][kTCols * kTP];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;   // wave: uniform (SGPR)
    const int lb = xcd_block(blockIdx.x + blockIdx.y * gridDim.x, gridDim.x * gridDim.y);
    const int f = lb / gridDim.x, bx = lb - f * gridDim.x;
    const int L = G->nlevels;
    const uint32_t kxb = (uint32_t)__builtin_amdgcn_readfirstlane(G->kp_xbits);   // packed keypoint x width
    const int* cnts = qt_cnt + (size_t)f * L;
    uint32_t* raw32 = s_raw[wave];
    uint8_t* raw = (uint8_t*)raw32;
    uint32_t* rowT = s_rowT[wave];
    const int g0 = (bx * kDescWaves + wave) * kpw;

    // ---- keypoint-independent lane state (c_desc_lanes), loaded once for the wave's keypoints ----
    const int icv = lane >> 1, ich = lane & 1;
    const int vrow = icv - 15;
    const DescLane& DL = c_desc_lanes.l[lane];
    uint32_t W1[4], W0[4];
    float ppx[kDescSlots], ppy[kDescSlots];
    uint32_t rdo[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        W1[k] = DL.w1[k];
        W0[k] = DL.w0[k];
    }
#pragma unroll
    for (int q = 0; q < kDescSlots; ++q) {
        ppx[q] = DL.upx[q];
        ppy[q] = DL.upy[q];
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) rdo[q] = DL.rd[q];
    const int ic_row = 21 + vrow, ic_col = ich ? 22 : 6;   // raw row, patch column of the first pixel
    int bitem[3];
#pragma unroll
    for (int it = 0; it < 3; ++it) bitem[it] = c_blur_items[lane + 64 * it];

    // output index g (level-major, as the reference concatenates levels) -> level, keypoint: lane j < kpw
    // looks up the wave's keypoint j once, up front, so no keypoint waits for its packed entry's global load
    // before its patch DMA can go out.  The wave's indices are consecutive, so past the frame's total (or
    // the output capacity) the rest are too, and the valid lanes are a prefix.
    int my_l = 0;
    uint32_t my_pk = 0;
    bool my_ok = false;
    if (lane < kpw) {
        const int g = g0 + lane;
        int base = 0, l = 0;
        for (; l < L; ++l) {
            if (g < base + cnts[l]) break;
            base += cnts[l];
        }
        if (l < L) {
            if (g >= cap) {
                atomicOr(status, (int)kStatusCapOverflow);
            } else {
                my_ok = true;
                my_l = l;
                my_pk = qt_out[(size_t)f * G->out_per_frame + G->lv[l].out_off + (g - base)];
            }
        }
    }
    const int nkp = __builtin_popcountll(__ballot(my_ok));
    auto lookup = [&](int jj, int& l, uint32_t& pk) -> bool {
        if (jj >= nkp) return false;
        l = __builtin_amdgcn_readlane(my_l, jj);
        pk = (uint32_t)__builtin_amdgcn_readlane((int)my_pk, jj);
        return true;
    };
    // raw patch rows cy-21..cy+21 from column cx-21 (48 bytes used per row); sets the
    // wave-uniform row-shift state: row r starts at byte (sb + r*sp) & 3 of its LDS row
    // the DMA's address registers kept live until the loop-top wait for it, so no later write to them makes
    // the compiler wait for the DMA (a write-after-read on a VMEM source register) before BRIEF
    uint32_t dma_va[3] = {0u, 0u, 0u};
    auto fill = [&](int l, uint32_t pk, int& sb, int& sp) {
        const int cx = (int)kp_x(pk, kxb), cy = (int)kp_y(pk, kxb);
        const int w = G->lv[l].w, h = G->lv[l].h;
        int pitch;
        const uint8_t* img = level_base(P, G, f, l, pitch);
        // Interior keypoints, and right-border ones whose 43 columns are all inside the level (cx + 21 < w):
        // those read up to 9 bytes past the row end, which land in the next row of the same level (cy + 22 < h)
        // and only feed blurred columns BRIEF never samples (|x| <= 18 + the 3-tap reach).  About 2/3 of the
        // 6.5% of KITTI keypoints the reflect-101 byte path took before (13% of the describe launch).
        if (cx >= 21 && cy >= 21 && cy + 21 < h && (cx + 31 <= w || (cx + 21 < w && cy + 22 < h))) {
            // 16-byte piece c = 64 t + lane of DMA instruction t (global_load_lds_dwordx4: lane L's 16 bytes
            // land at byte 16 L of the instruction's 1 KiB) is piece c % 3 of row c / 3, so three instructions
            // fill rows 0..43 (the third with lanes 0..3 only; row 43 repeats row 42).  Each row's aligned
            // bytes start at or after the 4-byte aligned allocation; a row reads 48 bytes from its aligned
            // start, at most cx + 26 (inside the level row, or in the next row of the same level for the
            // right-border case).  (Round 2: eleven 4-row global_load_lds_dword instructions into 64-byte
            // rows, 2816 B; the 48-byte rows take the wave to 5.6 KB of LDS, 7 waves per SIMD.)
            const uintptr_t s0 = (uintptr_t)(img + (size_t)(cy - 21) * pitch + (cx - 21));
            const uint8_t* ub = (const uint8_t*)(s0 & ~(uintptr_t)3);   // wave-uniform, aligned
            sb = (int)(s0 & 3);
            sp = pitch & 3;
#pragma unroll
            for (int t = 0; t < 3; ++t) {
                const int c = 64 * t + lane, row = c / 3, k = c - 3 * row;
                if (t < 2 || lane < 4) {
                    const uint32_t o = (uint32_t)((sb + min(row, 42) * pitch) & ~3) + 16u * (uint32_t)k;
                    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(ub + o),
                                                     (__attribute__((address_space(3))) void*)(raw32 + 256 * t), 16, 0, 0);
                    dma_va[t] = o;
                }
            }
        } else if (l > 0 && pitch - w >= 16) {
            // Border keypoints of levels >= 1 (about 5% of KITTI's keypoints, 12% at level 7): the same DMA,
            // through a buffer descriptor over the level's rows (pitch x h bytes of the handle's pyramid block),
            // so that the patch bytes outside the level read as zeros instead of touching memory (the range check
            // covers the whole offset: tests/test_gpu_edges.py test_buffer_range_check_covers_soffset); the
            // reflect-101 bytes are copied in from inside the patch at the loop top (desc_border_fixup).  Offsets
            // of rows above the level wrap to large unsigned values, also out of range.  A 16-byte chunk can straddle
            // the descriptor's end only within the level's last 16 bytes, which pitch - w >= 16 makes row padding,
            // so whether the range check drops such a chunk whole or by dwords, no pixel is lost (a level with
            // less padding, e.g. 444 px in a 448-byte pitch, takes the byte path below).
            const long long s0 = (long long)(cy - 21) * pitch + (cx - 21);
            const uint32_t a0 = (uint32_t)(s0 & ~3ll);
            sb = (int)(s0 & 3);
            sp = pitch & 3;   // 0: pitch = align64(w)
            const __amdgpu_buffer_rsrc_t rs =
                __builtin_amdgcn_make_buffer_rsrc((void*)img, (short)0, pitch * h, 0x00020000);
#pragma unroll
            for (int t = 0; t < 3; ++t) {
                const int c = 64 * t + lane, row = c / 3, k = c - 3 * row;
                if (t < 2 || lane < 4) {
                    const uint32_t o = a0 + (uint32_t)((sb + min(row, 42) * pitch) & ~3) + 16u * (uint32_t)k;
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(raw32 + 256 * t), 16,
                                                         o, 0, 0, 0);
                    dma_va[t] = o;
                }
            }
        } else {
            sb = 0;
            sp = 0;
            // level-0 border keypoints (the caller's image: no room around it to read past) and those of levels
            // with under 16 bytes of row padding: reflect-101 bytes,
            // lane = column (43 of the 48 per row), the column reflection once per lane,
            // the row's per row (wave-uniform), and 11 rows' loads in flight before their LDS stores
            static_assert(kRawRows >= 44, "rows 0..43 filled");
            const uint8_t* col = img + reflect101(cx - 21 + min(lane, 42), w);
            for (int s0 = 0; s0 < 44; s0 += 11) {
                uint8_t v[11];
#pragma unroll
                for (int u = 0; u < 11; ++u) v[u] = col[(size_t)reflect101(cy - 21 + min(s0 + u, 42), h) * pitch];   // row 43 repeats row 42
                if (lane < kRawP) {
#pragma unroll
                    for (int u = 0; u < 11; ++u) raw[(s0 + u) * kRawP + lane] = v[u];
                }
            }
            // (no-op at run time: every byte load above is consumed; it tells the compiler's wait-count pass so,
            // which otherwise waits for the DMA path's loads before BRIEF reuses these registers)
            __builtin_amdgcn_s_waitcnt(0x0F70);
        }
    };

    int nl = 0, sb = 0, sp = 0;
    uint32_t npk = 0;
    bool nvalid = lookup(0, nl, npk);
    if (nvalid) fill(nl, npk, sb, sp);
    // IC_Angle (src/ORBextractor.cc:84-128) of the wave's keypoints up front, from the level images in
    // global memory: a keypoint lies >= 19 px inside its level (FAST's cell windows), so its radius-15 disc
    // never leaves it (lanes 62-63 read row 16 with zero weights).  cv::fastAtan2 and sincosf then run
    // once per wave with lane j on keypoint j, instead of once per keypoint on every lane (the angle was
    // 17% of the launch).  Loads of every keypoint first, then the sums.
    float kp_ang = 0.f, kp_cos = 1.f, kp_sin = 0.f;
    int ic_m10 = 0, ic_m01 = 0;   // lane j: keypoint j's moments
    // (keypoints in groups of 4: one group's 20 row dwords in registers at a time)
    constexpr int kIcGroup = kDescPerWave < 4 ? kDescPerWave : 4;
#pragma unroll 1
    for (int j0 = 0; j0 < kDescPerWave && j0 < nkp; j0 += kIcGroup) {
        uint32_t q[kIcGroup][5], qs[kIcGroup];
#pragma unroll
        for (int ji = 0; ji < kIcGroup; ++ji) {
            const int jj = j0 + ji;
            const int jc = jj < nkp ? jj : nkp - 1;   // wave-uniform
            const int l = __builtin_amdgcn_readlane(my_l, jc);
            const uint32_t pk = (uint32_t)__builtin_amdgcn_readlane((int)my_pk, jc);
            const int cx = (int)kp_x(pk, kxb), cy = (int)kp_y(pk, kxb);
            int pitch;
            const uint8_t* img = level_base(P, G, f, l, pitch);
            const uintptr_t a = (uintptr_t)(img + (size_t)(cy + vrow) * pitch + (cx - 15 + 16 * ich));
            // (as a global pointer: an integer cast loses the address space, and flat loads count against both
            // wait counters)
            const __attribute__((address_space(1))) uint32_t* src =
                (const __attribute__((address_space(1))) uint32_t*)(a & ~(uintptr_t)3);
            qs[ji] = (uint32_t)(a & 3);
#pragma unroll
            for (int k = 0; k < 5; ++k) q[ji][k] = src[k];
        }
        int pv[kIcGroup][2];   // the lane's partial moments of the group's keypoints: (m10, m01)
#pragma unroll
        for (int ji = 0; ji < kIcGroup; ++ji) {
            uint32_t s1 = 0u, s0 = 0u;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t w = __builtin_amdgcn_alignbyte(q[ji][k + 1], q[ji][k], qs[ji]);
                s1 = __builtin_amdgcn_udot4(w, W1[k], s1, false);
                s0 = __builtin_amdgcn_udot4(w, W0[k], s0, false);
            }
            pv[ji][0] = (int)s1 - 16 * (int)s0;
            pv[ji][1] = vrow * (int)s0;
        }
        if constexpr (kIcGroup == 4) {
            // the eight wave sums as one reduce-scatter: v_permlane32_swap and v_permlane16_swap exchange half /
            // quarter waves, so each swap-and-add halves the lanes of two sums at once and packs them into one
            // register; the last 16-lane step is the DPP butterfly of wave_sum.  28 VALU for the group instead of
            // eight wave_sum (64).  Quarters of Q0: (m10 k0, m10 k1, m01 k0, m01 k1); of Q1 the same for k2, k3.
            auto swap_add = [](int a, int b, bool sixteen) {
                const auto r = sixteen ? __builtin_amdgcn_permlane16_swap(a, b, false, false)
                                       : __builtin_amdgcn_permlane32_swap(a, b, false, false);
                return (int)r[0] + (int)r[1];
            };
            auto row_sum = [](int v) {
                v += __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, true);    // quad_perm [1,0,3,2]
                v += __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, true);    // quad_perm [2,3,0,1]
                v += __builtin_amdgcn_mov_dpp(v, 0x141, 0xF, 0xF, true);   // row_half_mirror
                return v + __builtin_amdgcn_mov_dpp(v, 0x140, 0xF, 0xF, true);   // row_mirror
            };
            const int r0 = swap_add(pv[0][0], pv[0][1], false), r1 = swap_add(pv[1][0], pv[1][1], false);
            const int r2 = swap_add(pv[2][0], pv[2][1], false), r3 = swap_add(pv[3][0], pv[3][1], false);
            const int q0 = row_sum(swap_add(r0, r1, true)), q1 = row_sum(swap_add(r2, r3, true));
            const int m10[4] = {__builtin_amdgcn_readlane(q0, 0), __builtin_amdgcn_readlane(q0, 16),
                                __builtin_amdgcn_readlane(q1, 0), __builtin_amdgcn_readlane(q1, 16)};
            const int m01[4] = {__builtin_amdgcn_readlane(q0, 32), __builtin_amdgcn_readlane(q0, 48),
                                __builtin_amdgcn_readlane(q1, 32), __builtin_amdgcn_readlane(q1, 48)};
#pragma unroll
            for (int ji = 0; ji < 4; ++ji)
                if (lane == j0 + ji) {
                    ic_m10 = m10[ji];
                    ic_m01 = m01[ji];
                }
        } else {
#pragma unroll
            for (int ji = 0; ji < kIcGroup; ++ji) {
                const int x10 = wave_sum(pv[ji][0]), x01 = wave_sum(pv[ji][1]);
                if (lane == j0 + ji) {
                    ic_m10 = x10;
                    ic_m01 = x01;
                }
            }
        }
    }
    if (nkp > 0) {
        kp_ang = fast_atan2_deg((float)ic_m01, (float)ic_m10);
        glibc_sincosf_pair(kp_ang * kFactorPI, &kp_sin, &kp_cos);   // (src/ORBextractor.cc:148)
    }
#pragma unroll 1
    for (int jj = 0; jj < kpw && nvalid; ++jj) {
        const int oidx = g0 + jj, l = nl;
        const uint32_t pk = npk;
        const int csb = sb, csp = sp;
        const LevelGeom& LG = G->lv[l];
        const int cx = (int)kp_x(pk, kxb), cy = (int)kp_y(pk, kxb), score = (int)(pk >> 24);
        // this keypoint's DMA has landed.  vmcnt counts loads and stores and retires them in issue order, and
        // the previous keypoint's three output stores (desc dwordx2, cv::KeyPoint dwordx4 + dwordx3) were issued
        // after this DMA: waiting down to 3 leaves their round trip in flight
        // (the builtin, not inline asm: the compiler's wait-count pass sees it, and does not wait again for
        // loads it already covers -- an inline-asm wait is opaque to it; gfx9 simm16: vmcnt[3:0], expcnt[6:4]
        // = 7, lgkmcnt[11:8] = 15, vmcnt[5:4] at [15:14])
        // (also right for jj = 0: the IC_Angle loads issued after the first keypoint's DMA were waited for)
        __builtin_amdgcn_s_waitcnt(0x0F73);   // vmcnt(3)
        asm volatile("" ::"v"(dma_va[0]), "v"(dma_va[1]), "v"(dma_va[2]));
        wave_lds_sync();
        // a level >= 1 border keypoint's patch: reflect-101 (copyMakeBorder's BORDER_REFLECT_101, which
        // GaussianBlur applies at the level's edges) from the bytes inside it, columns first (lane = row), then
        // whole rows (lane = column), so the corners reflect in both directions.  The patch spans level columns
        // cx - 21 .. cx + 21 and rows cy - 21 .. cy + 21 (patch row 43 repeats row 42), and a keypoint lies >= 19 px
        // inside its level, so one reflection reaches every byte.
        if (l > 0 && LG.pitch - LG.w >= 16 &&
            !(cx >= 21 && cy >= 21 && cy + 21 < LG.h && (cx + 31 <= LG.w || (cx + 21 < LG.w && cy + 22 < LG.h)))) {
            const int w = LG.w, h = LG.h, x0 = cx - 21, y0 = cy - 21;
            auto at = [&](int r, int c) { return raw + r * kRawP + ((csb + r * csp) & 3) + c; };
            if (x0 < 0 || x0 + 42 >= w) {   // wave-uniform
                if (lane < kRawRows) {
#pragma unroll
                    for (int c = 0; c < 2; ++c)
                        if (x0 + c < 0) *at(lane, c) = *at(lane, -(x0 + c) - x0);
#pragma unroll
                    for (int c = 40; c <= 42; ++c)
                        if (x0 + c >= w) *at(lane, c) = *at(lane, 2 * w - 2 - (x0 + c) - x0);
                }
                wave_lds_sync();
            }
            if (y0 < 0 || y0 + 42 >= h) {   // wave-uniform
                // (cy in [19, h - 20]: only patch rows 0, 1 (above) and 41, 42, 43 (below) can leave the level)
                constexpr int kEdgeRows[5] = {0, 1, 41, 42, 43};
#pragma unroll
                for (int i = 0; i < 5; ++i) {
                    const int r = kEdgeRows[i], Y = y0 + min(r, 42);
                    if (Y >= 0 && Y < h) continue;   // wave-uniform
                    const int rr = (Y < 0 ? -Y : 2 * h - 2 - Y) - y0;
                    if (lane <= 42) *at(r, lane) = *at(rr, lane);
                }
                wave_lds_sync();
            }
        }

        // horizontal 7-tap pass: lane item = (row pair rp, column group cg) -> 2 rows x 4 columns.
        // Output column j of the realigned bytes R0 | R1 | R2 is sum_t w[t] * byte[j + t]: a dot4 of each
        // dword with the kernel shifted by j (zero outside the 7 taps), 10 dot4 per row instead of 8
        // byte-realignments and 8 dot4.
        // (kW[j][d] = blur_wshift(j, d): for the default kernel {18 | 34 << 8 | 49 << 16 | 55 << 24, 49 | 34 << 8 |
        // 18 << 16, 0} for j = 0, and so on)
        constexpr uint32_t kW[4][3] = {
            {blur_wshift(0, 0, kBM), blur_wshift(0, 1, kBM), blur_wshift(0, 2, kBM)},
            {blur_wshift(1, 0, kBM), blur_wshift(1, 1, kBM), blur_wshift(1, 2, kBM)},
            {blur_wshift(2, 0, kBM), blur_wshift(2, 1, kBM), blur_wshift(2, 2, kBM)},
            {blur_wshift(3, 0, kBM), blur_wshift(3, 1, kBM), blur_wshift(3, 2, kBM)}};
        static_assert(kBM != ORBX_BLUR_SCALAR || (kW[0][0] == (18u | 34u << 8 | 49u << 16 | 55u << 24) &&
                                                  kW[3][2] == (34u | 18u << 8)), "row-pass weights");
        // Rows that all start at the same byte shift S (csp == 0: the level pitch is a multiple of 4, or the
        // reflect-101 byte path) skip the realignment: output column j is a dot4 of each raw dword with the
        // kernel shifted by S + j bytes, still 10 dot4 per row (2 or 3 per column) and no alignbyte.
        auto hpass = [&](auto s_tag) {
            constexpr int S = decltype(s_tag)::value;   // -1: per-row shifts
#pragma unroll
            for (int it = 0; it < 3; ++it) {
                if (bitem[it] == 0xFFFF) break;
                const int rp = bitem[it] >> 8, cg = bitem[it] & 0xFF;
                uint32_t o[2][4];
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    const int r = 2 * rp + e;
                    const uint32_t* rr = raw32 + r * (kRawP / 4) + cg;
                    const uint32_t W[4] = {rr[0], rr[1], rr[2], rr[3]};
                    if constexpr (S < 0) {
                        const uint32_t sh = ((uint32_t)csb + __umul24((uint32_t)r, (uint32_t)csp)) & 3u;
                        const uint32_t R[3] = {__builtin_amdgcn_alignbyte(W[1], W[0], sh),
                                               __builtin_amdgcn_alignbyte(W[2], W[1], sh),
                                               __builtin_amdgcn_alignbyte(W[3], W[2], sh)};
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            uint32_t acc = __builtin_amdgcn_udot4(R[0], kW[j][0], 0u, false);
                            acc = __builtin_amdgcn_udot4(R[1], kW[j][1], acc, false);
                            if (j >= 2) acc = __builtin_amdgcn_udot4(R[2], kW[j][2], acc, false);
                            o[e][j] = acc;
                        }
                    } else {
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            uint32_t acc = 0u;
#pragma unroll
                            for (int d = 0; d < 4; ++d) {
                                const uint32_t w = blur_wshift(S + j, d, kBM);   // folds to a constant
                                if (w) acc = __builtin_amdgcn_udot4(W[d], w, acc, false);
                            }
                            o[e][j] = acc;
                        }
                    }
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    rowT[(4 * cg + j) * kTP + rp] = o[0][j] | (o[1][j] << 16);
                }
            }
        };
        if (csp != 0) hpass(std::integral_constant<int, -1>{});
        else if (csb == 0) hpass(std::integral_constant<int, 0>{});
        else if (csb == 1) hpass(std::integral_constant<int, 1>{});
        else if (csb == 2) hpass(std::integral_constant<int, 2>{});
        else hpass(std::integral_constant<int, 3>{});
        wave_lds_sync();   // raw is free: start the next keypoint's patch, it lands under BRIEF
        nvalid = lookup(jj + 1, nl, npk);
        if (nvalid) fill(nl, npk, sb, sp);

        // rBRIEF with the reference's contracted FMAs; blur evaluated at each sample point
        const float angle = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, kp_ang), jj));
        const float a = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, kp_cos), jj));
        const float b = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, kp_sin), jj));
        // GaussianBlur's u8 saturation: min(t0, 255) < min(t1, 255) iff t0 < min(t1, 255)
        const uint32_t cblur = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t*)rowT + kBlurByte0;
        // the lane's distinct sample points blurred, two per packed coordinate evaluation, then written to
        // the u16 sample table over rowT's first 768 bytes (one wave: its LDS reads and writes complete in
        // issue order, so every sample's rowT reads precede the table writes)
        typedef float f2v __attribute__((ext_vector_type(2)));
        // (the magic pair through an opaque scalar move: as a literal the compiler splits BX's packed add into two
        // v_add_f32, VOP3P having no literal operand)
        float mgs = kRoundMagic;
        asm("" : "+s"(mgs));
        const f2v va = {a, a}, vb = {b, b}, mg = {mgs, mgs};
        uint32_t tv[kDescSlots];
#pragma unroll
        for (int q = 0; q < kDescSlots; q += 2) {
            // (v_pk_mul / v_pk_fma / v_pk_add: the same roundings as the scalar statements, two samples per
            // instruction)
            const f2v PX = {ppx[q], ppx[q + 1]}, PY = {ppy[q], ppy[q + 1]};
            const f2v BY = __builtin_elementwise_fma(PX, vb, PY * va) + mg;
            const f2v BX = __builtin_elementwise_fma(PX, va, -(PY * vb)) + mg;
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                uint32_t t = blur_acc<kBM>(cblur, __float_as_uint(BY[e]), __float_as_uint(BX[e]));
                if constexpr (kBM == ORBX_BLUR_SSE2) {
                    // SymmColumnVec_32s8u: _mm_cvtps_epi32 of the exact sum T / 2^16 rounds half to even, so a
                    // tie (T % 2^16 == 2^15, here t = T + 2^15 with t % 2^16 == 0) above an even T >> 16 (t's bit
                    // 16 set) rounds down, on every level column below w & ~3
                    const int xl = cx + (int)(__float_as_uint(BX[e]) - kRoundBits);
                    if ((t & 0x1FFFFu) == 0x10000u && xl < (LG.w & ~3)) t -= 0x10000u;
                }
                tv[q + e] = t;
            }
        }
        uint16_t* const stab = (uint16_t*)rowT;
#pragma unroll
        for (int q = 0; q < kDescSlots; ++q) stab[64 * q + lane] = (uint16_t)(tv[q] >> 16);
        wave_lds_sync();
        unsigned long long words[4];
#pragma unroll
        for (int wd = 0; wd < 4; ++wd) {
            const uint32_t t0 = *(const uint16_t*)((const uint8_t*)stab + rdo[2 * wd]);
            const uint32_t t1 = *(const uint16_t*)((const uint8_t*)stab + rdo[2 * wd + 1]);
            words[wd] = __ballot(t0 < (t1 < 255u ? t1 : 255u));
        }
        {   // A/B knob: per-keypoint stores (round 2)
            const size_t o = (size_t)f * cap + oidx;
            if (lane < 4) reinterpret_cast<unsigned long long*>(desc + o * 32)[lane] = words[lane];
            if (lane == 0) {
                float x = (float)cx, y = (float)cy;
                if (l != 0) {
                    x *= LG.scale;
                    y *= LG.scale;
                }
                orbx_keypoint k;
                k.x = x;
                k.y = y;
                k.size = LG.patch_size;
                k.angle = angle;
                k.response = (float)score;
                k.octave = l;
                k.class_id = -1;
                kps[o] = k;
            }
        }
        wave_lds_sync();   // rowT is rewritten by the next keypoint
    }
}

void launch_describe(const Geometry& g, const ExtractBufs& b, const FramePtrs& p, orbx_keypoint* kps,
                     uint8_t* desc, int cap, int batch, hipStream_t s)
{
    // small batches (the per-frame host path) are latency-bound: one keypoint per wave
    const int kpw = batch <= kLatencyMaxBatch ? 1 : kDescPerWave;
    dim3 grid((g.out_per_frame + kDescWaves * kpw - 1) / (kDescWaves * kpw), batch);
    if (b.blur_mode == ORBX_BLUR_SSE2)
        hipLaunchKernelGGL(k_describe<ORBX_BLUR_SSE2>, grid, dim3(64 * kDescWaves), 0, s, b.geom, p, b.qt_out, b.qt_cnt,
                           kps, desc, cap, b.status, kpw);
    else if (b.blur_mode == ORBX_BLUR_BITEXACT)
        hipLaunchKernelGGL(k_describe<ORBX_BLUR_BITEXACT>, grid, dim3(64 * kDescWaves), 0, s, b.geom, p, b.qt_out,
                           b.qt_cnt, kps, desc, cap, b.status, kpw);
    else
        hipLaunchKernelGGL(k_describe<ORBX_BLUR_SCALAR>, grid, dim3(64 * kDescWaves), 0, s, b.geom, p, b.qt_out,
                           b.qt_cnt, kps, desc, cap, b.status, kpw);
}

}  // namespace orbx
