// gfx950 image ingest, SURVEY.md §8f row 4: the per-frame input preparation in front of
// ORBextractor::operator().
//
// I1 k_ingest  cv::remap(src, dst, M1, M2, INTER_LINEAR) with CV_32F maps and the default
//              BORDER_CONSTANT 0 (Examples/Stereo/stereo_euroc.cc:136-137), per channel, then
//              cvtColor {RGB,BGR,RGBA,BGRA}2GRAY (Tracking::GrabImage*, src/Tracking.cc:185-210).
//              One lane produces 4 adjacent output pixels (one dword store).  The maps are shared
//              by every frame of a batch (nmaps pairs, frame f uses f % nmaps), so after the first
//              frame they are served from L2 / MALL; HBM traffic is src + dst.
// I2 k_depth   GrabImageRGBD's imDepth.convertTo(CV_32F, mDepthMapFactor) (src/Tracking.cc:234-235).
//
// Arithmetic is OpenCV 3.x's fixed-point path (oracle/orbref.c orbref_ingest): coordinates
// cvRound(m * 32) split into an integer part (saturated to short) and 5-bit fractions, weights
// (32-fx)(32-fy)*32 ..., (sum + 2^14) >> 15; gray = (w0*c0 + 9617*c1 + w2*c2 + 2^13) >> 14.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "orbx_kernels.hpp"

namespace orbx {

__device__ __forceinline__ int ig_round_x86(float v)   // cvRound (cvtss2si): NaN / out of range -> INT_MIN
{
    return (v >= -2147483648.0f && v < 2147483648.0f) ? __float2int_rn(v) : (-2147483647 - 1);
}

// the two horizontal taps (sx, sx+1) of one source row, all channels: one aligned 8- or 12-byte load
// and a funnel shift when the window lies inside the row, byte loads with the border value 0 otherwise
template <int CH>
__device__ __forceinline__ void ig_taps(const uint8_t* __restrict__ row, int sx, int cols, bool rowin, int t0[3],
                                        int t1[3])
{
    constexpr int C3 = CH > 1 ? 3 : 1;
#pragma unroll
    for (int k = 0; k < C3; ++k) t0[k] = t1[k] = 0;
    if (!rowin) return;
    const uintptr_t a = (uintptr_t)(row + (ptrdiff_t)sx * CH), a4 = a & ~(uintptr_t)3;
    constexpr int kWords = CH == 1 ? 2 : 3;   // bytes [sh/8, sh/8 + 2*CH) of the aligned window
    if (sx >= 0 && sx + 1 < cols && a4 >= (uintptr_t)row && a4 + 4 * kWords <= (uintptr_t)(row + (size_t)cols * CH)) {
        const int sh = (int)(a - a4) * 8;
        unsigned long long v;
        if (kWords == 2) {
            // (through a global pointer: an integer cast loses the address space, and flat loads count against both
            // wait counters)
            const __attribute__((address_space(1))) uint32_t* q = (const __attribute__((address_space(1))) uint32_t*)a4;
            const uint2 w = make_uint2(q[0], q[1]);
            v = ((unsigned long long)w.y << 32 | w.x) >> sh;
        } else {
            const __attribute__((address_space(1))) uint32_t* q = (const __attribute__((address_space(1))) uint32_t*)a4;
            const uint3 w = make_uint3(q[0], q[1], q[2]);
            const unsigned long long lo = (unsigned long long)w.y << 32 | w.x;
            v = sh ? (lo >> sh) | ((unsigned long long)w.z << (64 - sh)) : lo;
        }
#pragma unroll
        for (int k = 0; k < C3; ++k) {
            t0[k] = (int)((v >> (8 * k)) & 255);
            t1[k] = (int)((v >> (8 * (k + CH))) & 255);
        }
        return;
    }
    const bool x0 = (unsigned)sx < (unsigned)cols, x1 = (unsigned)(sx + 1) < (unsigned)cols;
#pragma unroll
    for (int k = 0; k < C3; ++k) {
        if (x0) t0[k] = row[(size_t)sx * CH + k];
        if (x1) t1[k] = row[(size_t)(sx + 1) * CH + k];
    }
}

template <int CH>
__device__ __forceinline__ uint32_t ig_gray(const int v[3], int w0, int w2)
{
    if (CH == 1) return (uint32_t)v[0];
    return (uint32_t)((v[0] * w0 + v[1] * 9617 + v[2 < CH ? 2 : 0] * w2 + (1 << 13)) >> 14);
}

// Interior pixels (all four taps inside, rows 4-byte aligned): one aligned 8/12-byte load per
// source row, realigned by alignbyte; per channel the two taps of a row are gathered by one v_perm
// and blended horizontally by one v_dot4_u32_u8 with (32 - fx, fx).  OpenCV's sum
// (a0 (32-fx)(32-fy) 32 + ... + 2^14) >> 15 is 32 X with X = (32-fy) h_a + fy h_b, so it equals
// (X + 512) >> 10 exactly.
template <int CH>
__device__ __forceinline__ uint32_t ig_remap_pixel(const uint8_t* __restrict__ S, int rows, int cols, size_t sstep,
                                                   int xlim, float mxv, float myv, int w0, int w2)
{
    constexpr int C3 = CH > 1 ? 3 : 1;
    const int sx32 = ig_round_x86(mxv * 32.0f);
    const int sy32 = ig_round_x86(myv * 32.0f);
    const int fx = sx32 & 31, fy = sy32 & 31;
    const int sx = min(max(sx32 >> 5, -32768), 32767), sy = min(max(sy32 >> 5, -32768), 32767);
    if ((unsigned)sx < (unsigned)xlim && (unsigned)sy < (unsigned)(rows - 1)) {   // xlim = 0: never
        const uint8_t* pa = S + (size_t)sy * sstep + sx * CH;
        const uint32_t sh = (uint32_t)((uintptr_t)pa & 3);
        const uint8_t* a4 = pa - sh;
        uint32_t la, ha, lb, hb;
        if (CH == 1) {
            const uint2 A = *reinterpret_cast<const uint2*>(a4);
            const uint2 B = *reinterpret_cast<const uint2*>(a4 + sstep);
            la = __builtin_amdgcn_alignbyte(A.y, A.x, sh);
            lb = __builtin_amdgcn_alignbyte(B.y, B.x, sh);
            ha = hb = 0u;
        } else {
            const uint3 A = *reinterpret_cast<const uint3*>(a4);
            const uint3 B = *reinterpret_cast<const uint3*>(a4 + sstep);
            la = __builtin_amdgcn_alignbyte(A.y, A.x, sh);
            ha = __builtin_amdgcn_alignbyte(A.z, A.y, sh);
            lb = __builtin_amdgcn_alignbyte(B.y, B.x, sh);
            hb = __builtin_amdgcn_alignbyte(B.z, B.y, sh);
        }
        const uint32_t wx = (uint32_t)(32 - fx) | (uint32_t)fx << 8;
        const uint32_t wy0 = (uint32_t)(32 - fy), wy1 = (uint32_t)fy;
        int val[3];
#pragma unroll
        for (int k = 0; k < C3; ++k) {
            const uint32_t sel = (uint32_t)k | (uint32_t)(k + CH) << 8 | 0x0C0C0000u;   // (tap x, tap x+1, 0, 0)
            const uint32_t hA = __builtin_amdgcn_udot4(__builtin_amdgcn_perm(ha, la, sel), wx, 0u, false);
            const uint32_t hB = __builtin_amdgcn_udot4(__builtin_amdgcn_perm(hb, lb, sel), wx, 0u, false);
            val[k] = (int)((hA * wy0 + hB * wy1 + 512u) >> 10);
        }
        return ig_gray<CH>(val, w0, w2);
    }
    const int w00 = (32 - fx) * (32 - fy) * 32, w01 = fx * (32 - fy) * 32;
    const int w10 = (32 - fx) * fy * 32, w11 = fx * fy * 32;
    const bool y0 = (unsigned)sy < (unsigned)rows, y1 = (unsigned)(sy + 1) < (unsigned)rows;
    int a0[3], a1[3], b0[3], b1[3], val[3];
    ig_taps<CH>(S + (size_t)(y0 ? sy : 0) * sstep, sx, cols, y0, a0, a1);
    ig_taps<CH>(S + (size_t)(y1 ? sy + 1 : 0) * sstep, sx, cols, y1, b0, b1);
#pragma unroll
    for (int k = 0; k < C3; ++k) val[k] = (a0[k] * w00 + a1[k] * w01 + b0[k] * w10 + b1[k] * w11 + (1 << 14)) >> 15;
    return ig_gray<CH>(val, w0, w2);
}

template <int CH>
__global__ __launch_bounds__(256) void k_ingest(const uint8_t* __restrict__ src, int rows, int cols, int rgb,
                                                size_t sstep, size_t sfs, const float* __restrict__ mx,
                                                const float* __restrict__ my, int nmaps, int drows, int dcols,
                                                uint8_t* __restrict__ dst, size_t dstep, size_t dfs, int gpr,
                                                int xlim)
{
    constexpr int C3 = CH > 1 ? 3 : 1;
    const int f = blockIdx.y;
    const int g = blockIdx.x * 256 + threadIdx.x;
    const int y = g / gpr, x0 = (g - y * gpr) * 4;
    if (y >= drows) return;
    const uint8_t* S = src + (size_t)f * sfs;
    const int w0 = rgb ? 4899 : 1868, w2 = rgb ? 1868 : 4899;   // RGB2Gray<uchar> coefficient order
    uint8_t* D = dst + (size_t)f * dfs + (size_t)y * dstep;
    const int n = min(4, dcols - x0);
    uint32_t packed = 0;
    if (mx) {
        const size_t mo = (size_t)(f % nmaps) * drows * dcols + (size_t)y * dcols + x0;
        float4 vx, vy;
        if (n == 4 && (((uintptr_t)(mx + mo) | (uintptr_t)(my + mo)) & 15) == 0) {
            vx = *reinterpret_cast<const float4*>(mx + mo);
            vy = *reinterpret_cast<const float4*>(my + mo);
        } else {
            vx.x = mx[mo]; vy.x = my[mo];
            vx.y = n > 1 ? mx[mo + 1] : 0.f; vy.y = n > 1 ? my[mo + 1] : 0.f;
            vx.z = n > 2 ? mx[mo + 2] : 0.f; vy.z = n > 2 ? my[mo + 2] : 0.f;
            vx.w = n > 3 ? mx[mo + 3] : 0.f; vy.w = n > 3 ? my[mo + 3] : 0.f;
        }
        const float xs[4] = {vx.x, vx.y, vx.z, vx.w}, ys[4] = {vy.x, vy.y, vy.z, vy.w};
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (k < n) packed |= ig_remap_pixel<CH>(S, rows, cols, sstep, xlim, xs[k], ys[k], w0, w2) << (8 * k);
    } else {
        const uint8_t* p = S + (size_t)y * sstep + (size_t)x0 * CH;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (k < n) {
                int v[3];
#pragma unroll
                for (int c = 0; c < C3; ++c) v[c] = p[k * CH + c];
                packed |= ig_gray<CH>(v, w0, w2) << (8 * k);
            }
        }
    }
    if (n == 4 && ((uintptr_t)(D + x0) & 3) == 0) {
        *reinterpret_cast<uint32_t*>(D + x0) = packed;
    } else {
        for (int k = 0; k < n; ++k) D[x0 + k] = (uint8_t)(packed >> (8 * k));
    }
}

__global__ __launch_bounds__(256) void k_depth(const uint8_t* __restrict__ src, int depth_type, int rows, int cols,
                                               size_t sstep, size_t sfs, float factor, float* __restrict__ dst,
                                               size_t dstep, size_t dfs)
{
    const int f = blockIdx.y;
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (size_t)rows * cols) return;
    const int y = (int)(i / cols), x = (int)(i - (size_t)y * cols);
    const uint8_t* row = src + (size_t)f * sfs + (size_t)y * sstep;
    const float v = depth_type == 0 ? (float)reinterpret_cast<const uint16_t*>(row)[x] : reinterpret_cast<const float*>(row)[x];
    reinterpret_cast<float*>(reinterpret_cast<uint8_t*>(dst) + (size_t)f * dfs + (size_t)y * dstep)[x] = v * factor + 0.0f;
}

void launch_ingest(const uint8_t* src, int batch, int rows, int cols, int channels, int rgb, size_t sstep,
                   size_t sfs, const float* mx, const float* my, int nmaps, int drows, int dcols, uint8_t* dst,
                   size_t dstep, size_t dfs, hipStream_t s)
{
    const int gpr = (dcols + 3) / 4;
    const dim3 grid((unsigned)(((size_t)gpr * drows + 255) / 256), batch);
    // interior fast path bound (ig_remap_pixel): x + 1 < cols and the aligned 8/12-byte window inside
    // the row; it needs 4-byte aligned rows, otherwise every pixel takes the checked path
    const int kw = channels == 1 ? 8 : 12;
    int xlim = std::min(cols - 2, (cols * channels - kw) / channels) + 1;   // fast iff 0 <= x < xlim
    if ((((uintptr_t)src | sstep | sfs) & 3) || cols * channels < kw || xlim < 0) xlim = 0;
    switch (channels) {
    case 1:
        hipLaunchKernelGGL(k_ingest<1>, grid, dim3(256), 0, s, src, rows, cols, rgb, sstep, sfs, mx, my, nmaps, drows,
                           dcols, dst, dstep, dfs, gpr, xlim);
        break;
    case 3:
        hipLaunchKernelGGL(k_ingest<3>, grid, dim3(256), 0, s, src, rows, cols, rgb, sstep, sfs, mx, my, nmaps, drows,
                           dcols, dst, dstep, dfs, gpr, xlim);
        break;
    default:
        hipLaunchKernelGGL(k_ingest<4>, grid, dim3(256), 0, s, src, rows, cols, rgb, sstep, sfs, mx, my, nmaps, drows,
                           dcols, dst, dstep, dfs, gpr, xlim);
        break;
    }
}

void launch_depth(const void* src, int depth_type, int batch, int rows, int cols, size_t sstep, size_t sfs,
                  float factor, float* dst, size_t dstep, size_t dfs, hipStream_t s)
{
    const dim3 grid((unsigned)(((size_t)rows * cols + 255) / 256), batch);
    hipLaunchKernelGGL(k_depth, grid, dim3(256), 0, s, (const uint8_t*)src, depth_type, rows, cols, sstep, sfs, factor,
                       dst, dstep, dfs);
}

}  // namespace orbx
