// Arithmetic helpers shared by the gfx950 kernels and the host.
//
// Everything here must round exactly like the reference's CPU code:
//   * cv::fastAtan2        (OpenCV 3.x atan_f32, float, no FMA)   SURVEY.md A.4
//   * glibc 2.35 cosf/sinf (sysdeps/ieee754/flt-32 sincosf.h; double
//     evaluation, table of the x86-64 libm — constants read back from the
//     host libm, algorithm verified equal to libm on every float in
//     [0, 2*pi] by tests/test_host_math.py)                          SURVEY.md A.5 / F7
// The library is compiled with -ffp-contract=off; the FMAs below are the ones
// glibc's x86-64 FMA variant forms and are written out explicitly.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define ORBX_HD __host__ __device__ __forceinline__
#else
#define ORBX_HD inline
#endif

namespace orbx {

// __sincosf_table[0] (glibc sincosf_data.c, x86-64 build without TOINT intrinsics).
// __sincosf_table[1] is the same table with the cosine coefficients c0..c4 negated, so a
// cosine polynomial evaluated through it is exactly the negation of the one below
// (negating every fma operand negates the correctly rounded result).
constexpr double kSC_hpi_inv = 0x1.45f306dc9c883p+23, kSC_hpi = 0x1.921fb54442d18p+0;
constexpr double kSC_c0 = 0x1p0, kSC_c1 = -0x1.ffffffd0c621cp-2, kSC_c2 = 0x1.55553e1068f19p-5,
                 kSC_c3 = -0x1.6c087e89a359dp-10, kSC_c4 = 0x1.99343027bf8c3p-16;
constexpr double kSC_s1 = -0x1.555545995a603p-3, kSC_s2 = 0x1.1107605230bc4p-7, kSC_s3 = -0x1.994eb3774cf24p-13;

ORBX_HD uint32_t f32_bits(float f) { union { float f; uint32_t u; } c; c.f = f; return c.u; }
ORBX_HD uint32_t abstop12(float x) { return (f32_bits(x) >> 20) & 0x7ff; }

ORBX_HD double fma_d(double a, double b, double c) { return __builtin_fma(a, b, c); }

// sinf_poly (table 0): sine polynomial
ORBX_HD float sin_poly(double x, double x2)
{
    const double x3 = x * x2;
    const double s1 = fma_d(x2, kSC_s3, kSC_s2);
    const double x7 = x3 * x2;
    const double s = fma_d(x3, kSC_s1, x);
    return (float)fma_d(x7, s1, s);
}

// sinf_poly (table 0): cosine polynomial
ORBX_HD float cos_poly(double x2)
{
    const double x4 = x2 * x2;
    const double c2 = fma_d(x2, kSC_c4, kSC_c3);
    const double c1 = fma_d(x2, kSC_c1, kSC_c0);
    const double x6 = x4 * x2;
    const double c = fma_d(x4, kSC_c2, c1);
    return (float)fma_d(x6, c2, c);
}

// glibc sinf and cosf of one argument, |y| < 120 (every BRIEF angle is in [0, 2*pi)).
// glibc's sinf(y) = sinf_poly(x*s, x*x, p, n) and cosf(y) = sinf_poly(x*s, x*x, p, n^1)
// with p = table (n & 2); the reduction is shared.
ORBX_HD void glibc_sincosf_pair(float y, float* sinv, float* cosv)
{
    const float pio4f = 0x1.921FB6p-1f;
    double x = y;
    if (abstop12(y) < abstop12(pio4f)) {
        const double x2 = x * x;
        if (abstop12(y) < abstop12(0x1p-12f)) {
            *sinv = y;
            *cosv = 1.0f;
            return;
        }
        *sinv = sin_poly(x, x2);
        *cosv = cos_poly(x2);
        return;
    }
    const double r = x * kSC_hpi_inv;
    const int n = ((int32_t)r + 0x800000) >> 24;
    x = fma_d(-(double)n, kSC_hpi, x);
    const double xs = ((n + 1) & 2) ? -x : x;   // sign[n & 3] = {1, -1, -1, 1}
    const double x2 = x * x;
    const float sp = sin_poly(xs, x2);
    const float cp = (n & 2) ? -cos_poly(x2) : cos_poly(x2);
    // n even: sinf = sine poly, cosf = cosine poly; n odd: swapped
    *sinv = (n & 1) ? cp : sp;
    *cosv = (n & 1) ? sp : cp;
}

// which = 0 -> sinf(y), 1 -> cosf(y)
ORBX_HD float glibc_sincosf(float y, int which)
{
    float s, c;
    glibc_sincosf_pair(y, &s, &c);
    return which ? c : s;
}

// cv::fastAtan2 (OpenCV 3.x), degrees in [0, 360)
ORBX_HD float fast_atan2_deg(float y, float x)
{
    const float k180pi = (float)(180 / 3.1415926535897932384626433832795);
    const float p1 = 0.9997878412794807f * k180pi;
    const float p3 = -0.3258083974640975f * k180pi;
    const float p5 = 0.1555786518463281f * k180pi;
    const float p7 = -0.04432655554792128f * k180pi;
    const float ax = x < 0 ? -x : x, ay = y < 0 ? -y : y;
    const float eps = (float)2.2204460492503131e-16;   // (float)DBL_EPSILON
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + eps);
        c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = ax / (ay + eps);
        c2 = c * c;
        a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

// (float)(CV_PI/180.f), src/ORBextractor.cc:131
constexpr float kFactorPI = (float)(3.1415926535897932384626433832795 / 180.f);

}  // namespace orbx
