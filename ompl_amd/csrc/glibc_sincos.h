// glibc_sincos.h — restatement of the sin / cos / sincos the reference's arithmetic actually
// calls, for host and device, so the device's KinematicChain geometry (demos/KinematicChain.h:105-124
// distance, :200-226 isValid) and SO3 interpolation (SO3StateSpace.cpp:289-318) reproduce the
// reference's bit for bit.
//
// Third-party algorithm: GNU C Library 2.35 (the image's libm, Ubuntu GLIBC 2.35-0ubuntu3),
// sysdeps/ieee754/dbl-64/s_sin.c (__sin / __cos) and s_sincos.c (__sincos) — the IBM Accurate
// Mathematical Library algorithm as simplified in glibc 2.28:
//   |x| < 2^-26 (sin) / 2^-27 (cos)   x / 1
//   |x| < 0.855469                     do_sin(x, 0) / do_cos(x, 0)
//   |x| < 2.426265                     pi/2 - |x| as a double-double, then do_cos / do_sin
//   |x| < 105414350                    reduce_sincos (Cody-Waite, pi/2 = mp1 + mp2 + pp3 + pp4,
//                                      136 bits), do_sin / do_cos by quadrant
//   do_sin: |x| < 0.126 -> TAYLOR_SIN (degree 11 + the (1 - x^2) dx / 2 correction); else the
//           table point X = round(128 |x|) / 128, sin(X + d) = sn + ssn + s ccs - sn c + cs s with
//           s = sin(d) - ..., c = 1 - cos(d) from short polynomials; do_cos the mirror image
//   table   sin / cos of k / 128, k = 0..109, as double-doubles (tools/gen_glibc_sincos.py)
// Which build the reference gets (both measured, tools/glibc_fit.cpp):
//   * sin and cos are x86-64 multiarch functions: __sin_fma / __cos_fma (the same C compiled with
//     -mfma -mavx2, chosen at run time on every CPU with FMA), so every multiply-add GCC contracts
//     is fused — FMA = true below;
//   * sincos has no FMA variant: the generic build, no fused operation — FMA = false.  GCC turns a
//     cos(t) and a sin(t) of the same argument into one sincos(t) call (its sincos CSE at -O1 and
//     above), which is what the reference's KinematicChain distance / isValid / horn environment
//     and every host feature row (host_features.cpp) get: glibc_sincos below.
// Arguments >= 105414350 (never on the hot path: cumulative chain angles stay below 32 pi) take
// the math library's functions.
// Pinned: tools/glibc_fit.cpp / tools/glibc_sincos_check.cpp compare this arithmetic with the
// host's glibc — 0 differences in 6 x 10^8 sin / cos and 4 x 10^7 sincos evaluations over
// |x| <= 100, arguments within 1e-6 .. 1e-15 of multiples of pi/2 and tiny arguments;
// tools/libm_probe.py runs the device form (0 differences in 4 x 10^6); tests/test_gpu_chain_boundary.py
// checks the chain's knife edges against the oracle (glibc).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cmath>

#include "sincos_tables.h"

namespace ompl_amd {
namespace gsc {

constexpr double kBig = 0x1.8p45;                    // 52776558133248: rounds |x| to a multiple of 1/128
constexpr double kHp0 = 0x1.921fb54442d18p0;         // pi/2 (hi)
constexpr double kHp1 = 0x1.1a62633145c07p-54;       // pi/2 (lo)
constexpr double kMp1 = 0x1.921fb58p0;               // pi/2 = mp1 + mp2 + pp3 + pp4 (136 bits)
constexpr double kMp2 = -0x1.dde973cp-27;
constexpr double kPp3 = -0x1.cb3b398p-55;
constexpr double kPp4 = -0x1.d747f23e32ed7p-83;
constexpr double kHpInv = 0x1.45f306dc9c883p-1;      // 2/pi
constexpr double kToInt = 0x1.8p52;
constexpr double kSn3 = -1.66666666666664880952546298448555E-01, kSn5 = 8.33333214285722277379541354343671E-03,
                 kCs2 = 4.99999999999999999999950396842453E-01, kCs4 = -4.16666666666664434524222570944589E-02,
                 kCs6 = 1.38888874007937613028114285595617E-03;
constexpr double kS1 = -0x1.5555555555555p-3, kS2 = 0x1.1111111110ecep-7, kS3 = -0x1.a01a019db08b8p-13,
                 kS4 = 0x1.71de27b9a7ed9p-19, kS5 = -0x1.addffc2fcdf59p-26;

__host__ __device__ __forceinline__ uint64_t bits(double x) {
    uint64_t u;
    __builtin_memcpy(&u, &x, sizeof u);
    return u;
}

// a * b + c: fused in the FMA build, two roundings in the generic one (-ffp-contract=off)
template <bool FMA>
__host__ __device__ __forceinline__ double mad(double a, double b, double c) {
    if constexpr (FMA) return fma(a, b, c);
    else return a * b + c;
}

// TAYLOR_SIN(xx, a, da): a - a^3/3! + ... + (1 - a^2) da / 2
template <bool FMA>
__host__ __device__ __forceinline__ double taylor_sin(double xx, double a, double da) {
    const double p = mad<FMA>(mad<FMA>(mad<FMA>(mad<FMA>(kS5, xx, kS4), xx, kS3), xx, kS2), xx, kS1);
    const double t = mad<FMA>(FMA ? fma(p, a, -(0.5 * da)) : p * a - 0.5 * da, xx, da);
    return a + t;
}

template <bool FMA>
__host__ __device__ __forceinline__ double do_cos(double x, double dx, const double *tab = kSinCosTab) {
    if (x < 0) dx = -dx;
    const double u = kBig + fabs(x);
    x = fabs(x) - (u - kBig) + dx;
    const double xx = x * x;
    const double s = mad<FMA>(x * xx, mad<FMA>(xx, kSn5, kSn3), x);
    const double c = xx * mad<FMA>(xx, mad<FMA>(xx, kCs6, kCs4), kCs2);
    const int k = (int)(uint32_t)bits(u) << 2;
    const double sn = tab[k], ssn = tab[k + 1], cs = tab[k + 2], ccs = tab[k + 3];
    const double cor = mad<FMA>(-sn, s, mad<FMA>(-cs, c, mad<FMA>(-s, ssn, ccs)));
    return cs + cor;
}

template <bool FMA>
__host__ __device__ __forceinline__ double do_sin(double x, double dx, const double *tab = kSinCosTab) {
    const double xold = x;
    if (fabs(x) < 0.126) return taylor_sin<FMA>(x * x, x, dx);
    if (x <= 0) dx = -dx;
    const double u = kBig + fabs(x);
    x = fabs(x) - (u - kBig);
    const double xx = x * x;
    const double s = x + mad<FMA>(x * xx, mad<FMA>(xx, kSn5, kSn3), dx);
    const double r = mad<FMA>(xx, mad<FMA>(xx, kCs6, kCs4), kCs2);
    const double c = FMA ? fma(x, dx, xx * r) : x * dx + xx * r;
    const int k = (int)(uint32_t)bits(u) << 2;
    const double sn = tab[k], ssn = tab[k + 1], cs = tab[k + 2], ccs = tab[k + 3];
    const double cor = mad<FMA>(cs, s, mad<FMA>(-sn, c, mad<FMA>(s, ccs, ssn)));
    return copysign(sn + cor, xold);
}

// reduce_sincos: x - n pi/2 = a + da, returns n mod 4
template <bool FMA>
__host__ __device__ __forceinline__ int reduce(double x, double &a, double &da) {
    const double t = mad<FMA>(x, kHpInv, kToInt);
    const double xn = t - kToInt;
    const double y = mad<FMA>(-xn, kMp2, mad<FMA>(-xn, kMp1, x));
    const int n = (int)((uint32_t)bits(t) & 3u);
    double t1 = xn * kPp3;
    const double t2 = y - t1;
    double db = (y - t2) - t1;
    t1 = xn * kPp4;
    const double b = t2 - t1;
    db += (t2 - b) - t1;
    a = b;
    da = db;
    return n;
}

template <bool FMA>
__host__ __device__ __forceinline__ double quadrant(double a, double da, int n) {
    const double r = (n & 1) ? do_cos<FMA>(a, da) : do_sin<FMA>(a, da);
    return (n & 2) ? -r : r;
}

}  // namespace gsc

// sin(x) as glibc's __sin_fma (s_sin.c)
__host__ __device__ __forceinline__ double glibc_sin(double x) {
    const uint32_t k = (uint32_t)(gsc::bits(x) >> 32) & 0x7fffffffu;
    if (k < 0x3e500000u) return x;
    if (k < 0x3feb6000u) return gsc::do_sin<true>(x, 0.0);
    if (k < 0x400368fdu) return copysign(gsc::do_cos<true>(gsc::kHp0 - fabs(x), gsc::kHp1), x);
    if (k < 0x419921fbu) {
        double a, da;
        const int n = gsc::reduce<true>(x, a, da);
        return gsc::quadrant<true>(a, da, n);
    }
    return sin(x);  // |x| >= 105414350, inf, NaN: outside the hot path
}

// cos(x) as glibc's __cos_fma (s_sin.c)
__host__ __device__ __forceinline__ double glibc_cos(double x) {
    const uint32_t k = (uint32_t)(gsc::bits(x) >> 32) & 0x7fffffffu;
    if (k < 0x3e400000u) return 1.0;
    if (k < 0x3feb6000u) return gsc::do_cos<true>(x, 0.0);
    if (k < 0x400368fdu) {
        const double y = gsc::kHp0 - fabs(x);
        const double a = y + gsc::kHp1;
        const double da = (y - a) + gsc::kHp1;
        return gsc::do_sin<true>(a, da);
    }
    if (k < 0x419921fbu) {
        double a, da;
        const int n = gsc::reduce<true>(x, a, da);
        return gsc::quadrant<true>(a, da, n + 1);
    }
    return cos(x);
}

// sincos(x, &s, &c) as glibc's generic __sincos (s_sincos.c).  Every branch ends in one do_sin and
// one do_cos evaluation of branch-dependent arguments, so the pair is computed with exactly one of
// each and no divergent paths apart from do_sin's Taylor / table split — what a wavefront of lanes
// at different angles wants:
//   |x| < 0.855469   s = do_sin(x, 0)                    c = do_cos(x, 0)
//   |x| < 2.426265   (a, da) = pi/2 - |x|:  s = copysign(do_cos(a, da), x)   c = do_sin(a, da)
//   else (n = quadrant)  {do_sin, do_cos}(a, da) assigned to s / c by n, signed by n & 2
// tab: the table (a kernel may pass its LDS copy of gsc::kSinCosTab)
__host__ __device__ __forceinline__ void glibc_sincos(double x, double &s, double &c, const double *tab = gsc::kSinCosTab) {
    const uint32_t k = (uint32_t)(gsc::bits(x) >> 32) & 0x7fffffffu;
    if (!(k < 0x419921fbu)) {  // outside the hot path (and inf / NaN)
        s = sin(x);
        c = cos(x);
        return;
    }
    double a = x, da = 0.0;
    int n = 0;
    const bool mid = k >= 0x3feb6000u && k < 0x400368fdu, big = k >= 0x400368fdu;
    if (mid) {
        const double y = gsc::kHp0 - fabs(x);
        a = y + gsc::kHp1;
        da = (y - a) + gsc::kHp1;
    } else if (big) {
        n = gsc::reduce<false>(x, a, da);
    }
    const double P = gsc::do_sin<false>(a, da, tab), Q = gsc::do_cos<false>(a, da, tab);
    if (mid) {
        s = copysign(Q, x);
        c = P;
    } else if (big) {
        const double ev = (n & 2) ? -P : P, od = (n & 2) ? -Q : Q;  // n even: sin = +-P, cos = +-Q
        const double ev1 = ((n + 1) & 2) ? -P : P, od1 = ((n + 1) & 2) ? -Q : Q;
        s = (n & 1) ? od : ev;
        c = (n & 1) ? ev1 : od1;
    } else {
        s = k < 0x3e400000u ? x : P;
        c = k < 0x3e400000u ? 1.0 : Q;
    }
}

}  // namespace ompl_amd
