// ndt_libm.h — the glibc libm functions the reference's f32 arithmetic calls, restated from glibc's published
// algorithms (sysdeps/ieee754/flt-32: e_expf.c, s_sinf.c, s_cosf.c, sincosf.h / sincosf_data.c), evaluated as the x86-64
// FMA build of glibc evaluates them (every multiply-add fused), so that host and device produce glibc's bits:
//   exp_f   — std::exp(float) in updateDerivatives (ndt_omp_impl.hpp:507);
//   sinf_r, cosf_r — std::sin / std::cos on float in Eigen::AngleAxisf::toRotationMatrix, i.e. convertTransform
//             (ndt_omp.h:210-229) for every pass's transform.
// Checked bit for bit against the host's glibc (exhaustively once; strided samples in tests/native/libm_check.cpp).
// Host and device code.
#pragma once
#include <math.h>

#if defined(__HIPCC__)
#define NDT_LIBM_FN __host__ __device__ __attribute__((always_inline)) inline
#else
#define NDT_LIBM_FN __attribute__((always_inline)) inline
#endif

namespace ndt {

// expf as the reference evaluates it: std::exp(float) at ndt_omp_impl.hpp:507 is glibc's expf, whose published algorithm
// (sysdeps/ieee754/flt-32/e_expf.c, the x86-64 build selects its FMA variant) is restated here: x N / ln2 = k + r (N = 32,
// k rounded to nearest by the 1.5 * 2^52 shift), 2^(k/N) from a 32-entry table of 2^(i/N) bit patterns with the exponent
// added as an integer, 2^(r/N) by a cubic in r, every multiply-add fused, the f64 result rounded to f32 once.  Equal bit
// for bit to the host's glibc expf on all 4,278,190,082 non-NaN f32 inputs (checked exhaustively; tests/native/
// expf_check.cpp re-checks a strided sample), where the correctly rounded (float)exp((double)x) differs on 170,648.
// tab: kExp2fTab (host) or its LDS copy (device: a per-lane lookup).
#define NDT_EXP2F_TAB                                                                                                  \
    0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull, 0x3fef72b83c7d517bull, \
        0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull, 0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, \
        0x3feedea64c123422ull, 0x3feece086061892dull, 0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, \
        0x3feea47eb03a5585ull, 0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull, \
        0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull, 0x3feee89f995ad3adull, \
        0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull, 0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, \
        0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull
constexpr int kExp2fTabLen = 32;

NDT_LIBM_FN unsigned long long bits_d(double d) {
    unsigned long long u;
    __builtin_memcpy(&u, &d, 8);
    return u;
}
NDT_LIBM_FN double from_bits_d(unsigned long long u) {
    double d;
    __builtin_memcpy(&d, &u, 8);
    return d;
}

NDT_LIBM_FN float exp_f(float x, const unsigned long long* tab) {
    constexpr double kN = 32.0, kInvLn2N = 0x1.71547652b82fep+0 * kN, kShift = 0x1.8p+52;
    constexpr double kC0 = 0x1.c6af84b912394p-5 / kN / kN / kN, kC1 = 0x1.ebfce50fac4f3p-3 / kN / kN,
                     kC2 = 0x1.62e42ff0c52d6p-1 / kN;
    unsigned ux;
    __builtin_memcpy(&ux, &x, 4);
    const unsigned abstop = (ux >> 20) & 0x7ffu;
    const double xd = (double)x;
    double kd = fma(kInvLn2N, xd, kShift);
    const unsigned long long ki = bits_d(kd);
    kd -= kShift;
    const double r = fma(kInvLn2N, xd, -kd);
    const double s = from_bits_d(tab[ki % 32] + (ki << 47));
    const double z = fma(kC0, r, kC1);
    const double r2 = r * r;
    double y = fma(kC2, r, 1.0);
    y = fma(z, r2, y);
    y = y * s;
    const float out = (float)y;
    // |x| >= 88 or NaN (glibc's slow path, selected branch-free): -inf -> 0, NaN / +inf -> x + x, overflow -> inf,
    // underflow -> 0
    const float slow = ux == 0xff800000u        ? 0.f
                       : abstop >= 0x7f8u        ? x + x
                       : x > 0x1.62e42ep6f       ? __builtin_inff()
                       : x < -0x1.9fe368p6f      ? 0.f
                                                 : out;
    return abstop >= (0x42b00000u >> 20) ? slow : out;
}


// sinf / cosf (glibc, |x| < 120): |x| < pi/4 evaluates the odd (sine) or even (cosine) polynomial in double on x; else x
// is reduced by n * pi/2 (n from x * 2^24 * 2/pi truncated, rounded by the 2^23 bias) and quadrant n picks the polynomial
// and the sign; the f64 result is rounded to f32 once.  |x| < 2^-12 returns x (sine) or 1 (cosine).  For |x| >= 120 or a
// non-finite x (glibc: Payne-Hanek reduction / NaN) the correctly rounded double value is returned instead — angles of a
// pose parameter never come near 120 rad (parity unpinned there).
struct SinCosPoly {
    double c0, c1, c2, c3, c4, s1, s2, s3;
};
// glibc's two coefficient sets: quadrants 0-1 and 2-3 (the latter with the cosine polynomial negated)
NDT_LIBM_FN SinCosPoly sincosf_poly_coeffs(bool upper) {
    const double g = upper ? -1.0 : 1.0;
    return SinCosPoly{g * 0x1p0, g * -0x1.ffffffd0c621cp-2, g * 0x1.55553e1068f19p-5, g * -0x1.6c087e89a359dp-10,
                      g * 0x1.99343027bf8c3p-16, -0x1.555545995a603p-3, 0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13};
}
// sinf_poly: the sine polynomial for even n, the cosine polynomial for odd n
NDT_LIBM_FN float sincosf_eval(double x, double x2, const SinCosPoly& p, int n) {
    if ((n & 1) == 0) {
        const double x3 = x * x2;
        const double s1 = fma(x2, p.s3, p.s2);
        const double x7 = x3 * x2;
        const double s = fma(x3, p.s1, x);
        return (float)fma(x7, s1, s);
    }
    const double x4 = x2 * x2;
    const double c2 = fma(x2, p.c4, p.c3);
    const double c1 = fma(x2, p.c1, p.c0);
    const double x6 = x4 * x2;
    const double c = fma(x4, p.c2, c1);
    return (float)fma(x6, c2, c);
}
NDT_LIBM_FN unsigned abstop12_f(float x) {
    unsigned u;
    __builtin_memcpy(&u, &x, 4);
    return (u >> 20) & 0x7ffu;
}
// cos = 0: sinf, 1: cosf
NDT_LIBM_FN float sincosf_r(float y, int cos) {
    const double x = (double)y;
    if (abstop12_f(y) < abstop12_f(0x1.921fb6p-1f)) {  // |y| < pi/4
        if (abstop12_f(y) < abstop12_f(0x1p-12f)) return cos ? 1.0f : y;
        return sincosf_eval(x, x * x, sincosf_poly_coeffs(false), cos);
    }
    if (abstop12_f(y) < abstop12_f(120.0f)) {
        const double r = x * 0x1.45f306dc9c883p+23;  // x * 2/pi * 2^24
        const int n = ((int)r + 0x800000) >> 24;
        const double xr = fma(-(double)n, 0x1.921fb54442d18p0, x);
        const double sgn = (n & 3) == 1 || (n & 3) == 2 ? -1.0 : 1.0;
        return sincosf_eval(xr * sgn, xr * xr, sincosf_poly_coeffs((n & 2) != 0), n + cos);
    }
    return cos ? (float)::cos(x) : (float)::sin(x);
}
NDT_LIBM_FN float sinf_r(float x) { return sincosf_r(x, 0); }
NDT_LIBM_FN float cosf_r(float x) { return sincosf_r(x, 1); }

}  // namespace ndt
