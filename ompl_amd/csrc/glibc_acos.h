// glibc_acos.h — restatement of the acos the reference's SO3StateSpace::distance calls
// (SO3StateSpace.cpp:254-262 arcLength, via :289-318 interpolate too), for host and device, so
// SO3 / SE3 distances, segment counts and slerped states reproduce the reference's bit for bit.
//
// Third-party algorithm: GNU C Library 2.35 (the image's libm, Ubuntu GLIBC 2.35-0ubuntu3),
// sysdeps/ieee754/dbl-64/e_asin.c __ieee754_acos (the IBM Accurate Mathematical Library algorithm,
// slow paths removed in glibc 2.34), (C) IBM Corporation 2001 / Free Software Foundation,
// LGPL-2.1-or-later.  x86-64 builds it as a multiarch function: __ieee754_acos_fma (the same C with
// -mfma -mavx2, chosen at run time on every CPU with FMA and AVX2 — the reference's hosts and the
// GPU boxes' hosts) — so every multiply-add GCC contracted there is an fma() below and nothing
// else is fused (this file is compiled -ffp-contract=off).  By |x| (k = the high word of |x|):
//   |x| < 2^-54               pi/2
//   |x| < 0.125               pi/2 - x - x^3 P(x^2) with the hp1 correction (f1..f6)
//   0.125 <= |x| < 0.96875    table point x0 of |x|'s interval (6 interval sets, 11-15 entries per
//                             point): t = c1 xx + (xx^2 P(xx) + lo), acos = (pi/2 -+ asin(x0)) -+ t
//   0.96875 <= |x| < 1        z = (1 -+ x) / 2, sqrt(z) as y + cc (an inverse-root table guess,
//                             a polynomial and a Newton step, y its 26-bit head), acos =
//                             2 (y + cc + p (y + cc)) for x > 0, 2 (pi/2 - y + hp1 - cc - p (y + cc))
//   |x| == 1                  0 or pi;  |x| > 1 or NaN: NaN
// The tables (acos_tables.h) are the library's own data, read from that libm by
// tools/gen_glibc_acos.py.  Pinned: tools/glibc_acos_check.cpp compares this arithmetic with the
// host's glibc acos (0 differences: see the header of that file); tools/libm_probe.py runs the
// device form.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cmath>

#include "acos_tables.h"

namespace ompl_amd {
namespace gac {

constexpr double kHp0 = 0x1.921fb54442d18p+0;  // pi/2 (hi)
constexpr double kHp1 = 0x1.1a62633145c07p-54; // pi/2 (lo)
constexpr double kPi = 0x1.921fb54442d18p+1;
constexpr double kF1 = 0x1.55555555554f9p-3, kF2 = 0x1.333333336127dp-4, kF3 = 0x1.6db6dae42c0e4p-5,
                 kF4 = 0x1.f1c7e04f4ad99p-6, kF5 = 0x1.6e442c822d419p-6, kF6 = 0x1.292d80f453c72p-6;
constexpr double kRt0 = 0x1.fffffffecc1ddp-1, kRt1 = 0x1.fffffff757304p-2, kRt2 = 0x1.800496769c91ap-2,
                 kRt3 = 0x1.4006318d1dab9p-2;
constexpr double kT27 = 0x1.0p+27;

__host__ __device__ __forceinline__ uint64_t bits(double x) {
    uint64_t u;
    __builtin_memcpy(&u, &x, sizeof u);
    return u;
}

// f1 + f2 z + ... + f6 z^5, Horner with every step fused
__host__ __device__ __forceinline__ double fpoly(double z) {
    return fma(z, fma(z, fma(z, fma(z, fma(z, kF6, kF5), kF4), kF3), kF2), kF1);
}

// the table intervals: n = the interval's first entry, m = its polynomial's top entry (n + m);
// t = xx c1 + (xx^2 (c2 + xx (c3 + ...)) + lo), returns t and the interval's asin(x0) in y
__host__ __device__ __forceinline__ double table_t(double ax, int n, int m, double &y, const double *T) {
    const double xx = ax - T[n];
    double p = T[n + m];
    p = fma(xx, p, T[n + m - 1]);
    const double xx2 = xx * xx;
    for (int j = m - 2; j >= 2; --j) p = fma(xx, p, T[n + j]);
    p = fma(xx2, p, T[n + m + 1]);
    y = T[n + m + 2];
    return fma(xx, T[n + 1], p);
}

}  // namespace gac

// acos(x) as glibc 2.35's __ieee754_acos_fma (e_asin.c).  T: the __asncs table (a kernel may pass
// an LDS copy of gac::kAsnCs).
__host__ __device__ __forceinline__ double glibc_acos(double x, const double *T = gac::kAsnCs) {
    using namespace gac;
    const uint64_t u = bits(x);
    const int32_t m = (int32_t)(u >> 32);
    const int32_t k = m & 0x7fffffff;
    if (k < 0x3c880000) return kHp0;
    if (k < 0x3fc00000) {  // |x| < 0.125
        const double x2 = x * x;
        const double p = fpoly(x2);
        const double r = kHp0 - x;
        const double cor = fma(-p, x * x2, ((kHp0 - r) - x) + kHp1);
        return r + cor;
    }
    if (k < 0x3fef0000) {  // 0.125 <= |x| < 0.96875: a table interval
        int n, top;
        if (k < 0x3fd00000) {
            n = 11 * ((k >> 15) & 0x1f), top = 6;
        } else if (k < 0x3fe00000) {
            n = 11 * ((k >> 14) & 0x3f) + 352, top = 6;
        } else if (k < 0x3fe80000) {
            n = 12 * ((k >> 13) & 0x7f) + 1056, top = 7;
        } else if (k < 0x3fed8000) {
            n = 13 * ((k >> 13) & 0x7f) + 992, top = 8;
        } else if (k < 0x3fee8000) {
            n = 14 * ((k >> 13) & 0x7f) + 884, top = 9;
        } else {
            n = 15 * ((k >> 13) & 0x7f) + 768, top = 10;
        }
        double y;
        const double t = table_t(m > 0 ? x : -x, n, top, y, T);
        if (m > 0) return (kHp1 - t) + (kHp0 - y);
        return (t + kHp1) + (y + kHp0);
    }
    if (k < 0x3ff00000) {  // 0.96875 <= |x| < 1
        const double z = (m > 0 ? 1.0 - x : x + 1.0) * 0.5;
        const uint64_t zb = bits(z);
        const int hi21 = (int)((int64_t)zb >> 53), hi14 = (int)(((int64_t)zb >> 46) & 0x7f);
        double t = kInRoot[hi14] * kPowTwo[511 - hi21];
        const double r = fma(-(t * t), z, 1.0);
        t = fma(r, fma(r, fma(r, kRt3, kRt2), kRt1), kRt0) * t;
        const double c = z * t;
        const double s = fma(-c, t * 0.5, 1.5);
        const double y = fma(-kT27, c, fma(c, kT27, c));
        const double den = fma(s, c, y);
        const double cc = fma(-y, y, z) / den;
        const double p = fpoly(z) * z;
        const double q = p * (y + cc);
        if (m < 0) {
            const double res = ((kHp1 - cc) - q) + (kHp0 - y);
            return res + res;
        }
        const double res = (cc + q) + y;
        return res + res;
    }
    if (k == 0x3ff00000 && (uint32_t)u == 0u) return m > 0 ? 0.0 : kPi;
    if (k > 0x7ff00000 || (k == 0x7ff00000 && (uint32_t)u != 0u)) return x + x;
    return (x - x) / (x - x);
}

}  // namespace ompl_amd
