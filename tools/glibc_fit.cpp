// glibc_fit.cpp — measurement tool (not product): which fused-multiply-add contraction of glibc's
// dbl-64 sin / cos (the x86-64 __sin_fma / __cos_fma variants, the same C compiled with -mfma)
// reproduces the host's results.  Each ambiguous expression is a template switch.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "../ompl_amd/csrc/sincos_tables.h"

using ompl_amd::gsc::kSinCosTab;

static inline double hx(uint64_t u) { double d; std::memcpy(&d, &u, 8); return d; }
static const double big = hx(0x42C8000000000000ull), hp0 = hx(0x3FF921FB54442D18ull), hp1 = hx(0x3C91A62633145C07ull),
                    mp1 = hx(0x3FF921FB58000000ull), mp2 = hx(0xBE4DDE973C000000ull), pp3 = hx(0xBC8CB3B398000000ull),
                    pp4 = hx(0xBACD747F23E32ED7ull), hpinv = hx(0x3FE45F306DC9C883ull), toint = hx(0x4338000000000000ull);
static const double sn3 = -1.66666666666664880952546298448555E-01, sn5 = 8.33333214285722277379541354343671E-03,
                    cs2 = 4.99999999999999999999950396842453E-01, cs4 = -4.16666666666664434524222570944589E-02,
                    cs6 = 1.38888874007937613028114285595617E-03;
static const double s1 = -0x1.5555555555555p-3, s2 = 0x1.1111111110ECEp-7, s3 = -0x1.A01A019DB08B8p-13,
                    s4 = 0x1.71DE27B9A7ED9p-19, s5 = -0x1.ADDFFC2FCDF59p-26;

// V bits: 1 = FMA build at all; 2 = do_sin's c: fma(xx, R, x*dx) (else fma(x, dx, xx*R));
//         4 = TAYLOR's P*a - 0.5*da: fma(-0.5, da, P*a) (else fma(P, a, -0.5*da));
//         8 = reduce: the twice-used products fused at both uses (else computed once, not fused)
template <int V>
struct G {
    static constexpr bool F = V & 1;
    static inline double mad(double a, double b, double c) { return F ? std::fma(a, b, c) : a * b + c; }
    static inline int idx(double u) { uint64_t b; std::memcpy(&b, &u, 8); return (int)(uint32_t)b; }
    static double taylor(double xx, double a, double da) {
        double p2 = mad(mad(mad(s5, xx, s4), xx, s3), xx, s2);
        double P = F ? std::fma(p2, xx, s1) : p2 * xx + s1;
        double t0;
        if (!F) t0 = P * a - 0.5 * da;
        else if (V & 4) t0 = std::fma(-0.5, da, P * a);
        else t0 = std::fma(P, a, -(0.5 * da));
        double t = mad(t0, xx, da);
        return a + t;
    }
    static double do_cos(double x, double dx) {
        if (x < 0) dx = -dx;
        double u = big + std::fabs(x);
        x = std::fabs(x) - (u - big) + dx;
        double xx = x * x;
        double s = F ? std::fma(x * xx, std::fma(xx, sn5, sn3), x) : x + x * xx * (sn3 + xx * sn5);
        double c = F ? xx * std::fma(xx, std::fma(xx, cs6, cs4), cs2) : xx * (cs2 + xx * (cs4 + xx * cs6));
        int k = idx(u) << 2;
        double sn = kSinCosTab[k], ssn = kSinCosTab[k + 1], cs = kSinCosTab[k + 2], ccs = kSinCosTab[k + 3];
        double cor = F ? std::fma(-sn, s, std::fma(-cs, c, std::fma(-s, ssn, ccs))) : (ccs - s * ssn - cs * c) - sn * s;
        return cs + cor;
    }
    static double do_sin(double x, double dx) {
        double xold = x;
        if (std::fabs(x) < 0.126) return taylor(x * x, x, dx);
        if (x <= 0) dx = -dx;
        double u = big + std::fabs(x);
        x = std::fabs(x) - (u - big);
        double xx = x * x;
        double s = F ? x + std::fma(x * xx, std::fma(xx, sn5, sn3), dx) : x + (dx + x * xx * (sn3 + xx * sn5));
        double R = F ? std::fma(xx, std::fma(xx, cs6, cs4), cs2) : (cs2 + xx * (cs4 + xx * cs6));
        double c;
        if (!F) c = x * dx + xx * R;
        else if (V & 2) c = std::fma(xx, R, x * dx);
        else c = std::fma(x, dx, xx * R);
        int k = idx(u) << 2;
        double sn = kSinCosTab[k], ssn = kSinCosTab[k + 1], cs = kSinCosTab[k + 2], ccs = kSinCosTab[k + 3];
        double cor = F ? std::fma(cs, s, std::fma(-sn, c, std::fma(s, ccs, ssn))) : (ssn + s * ccs - sn * c) + cs * s;
        return std::copysign(sn + cor, xold);
    }
    static int reduce(double x, double *a, double *da) {
        double t = F ? std::fma(x, hpinv, toint) : x * hpinv + toint;
        double xn = t - toint;
        double y = F ? std::fma(-xn, mp2, std::fma(-xn, mp1, x)) : (x - xn * mp1) - xn * mp2;
        int n = idx(t) & 3;
        double t1, t2, db, b;
        if (F && (V & 8)) {
            t2 = std::fma(-xn, pp3, y);
            db = std::fma(-xn, pp3, y - t2);
            b = std::fma(-xn, pp4, t2);
            db += std::fma(-xn, pp4, t2 - b);
        } else {
            t1 = xn * pp3;
            t2 = y - t1;
            db = (y - t2) - t1;
            t1 = xn * pp4;
            b = t2 - t1;
            db += (t2 - b) - t1;
        }
        *a = b;
        *da = db;
        return n;
    }
    static double sincos_q(double a, double da, int n) {
        double r = (n & 1) ? do_cos(a, da) : do_sin(a, da);
        return (n & 2) ? -r : r;
    }
    static double sin(double x) {
        uint64_t b; std::memcpy(&b, &x, 8);
        uint32_t k = (uint32_t)(b >> 32) & 0x7fffffffu;
        if (k < 0x3e500000u) return x;
        if (k < 0x3feb6000u) return do_sin(x, 0);
        if (k < 0x400368fdu) { double t = hp0 - std::fabs(x); return std::copysign(do_cos(t, hp1), x); }
        double a, da; int n = reduce(x, &a, &da); return sincos_q(a, da, n);
    }
    static double cos(double x) {
        uint64_t b; std::memcpy(&b, &x, 8);
        uint32_t k = (uint32_t)(b >> 32) & 0x7fffffffu;
        if (k < 0x3e400000u) return 1.0;
        if (k < 0x3feb6000u) return do_cos(x, 0);
        if (k < 0x400368fdu) { double y = hp0 - std::fabs(x); double a = y + hp1; double da = (y - a) + hp1; return do_sin(a, da); }
        double a, da; int n = reduce(x, &a, &da); return sincos_q(a, da, n + 1);
    }
};

template <int V>
static void test(const std::vector<double> &xs) {
    uint64_t bs = 0, bc = 0; double fs = 0, fc = 0;
    for (double x : xs) {
        if (G<V>::sin(x) != std::sin(x)) { if (!bs) fs = x; ++bs; }
        if (G<V>::cos(x) != std::cos(x)) { if (!bc) fc = x; ++bc; }
    }
    std::printf("V=%2d sin_differ=%llu cos_differ=%llu  first %.17g %.17g\n", V, (unsigned long long)bs,
                (unsigned long long)bc, fs, fc);
}

int diag(size_t);
int main(int argc, char **argv) {
    if (argc > 2) return diag(std::strtoull(argv[1], nullptr, 10));
    size_t n = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 2000000;
    std::mt19937_64 g(7);
    std::uniform_real_distribution<double> u(-40.0, 40.0), v(-1.0, 1.0);
    std::vector<double> xs;
    for (size_t i = 0; i < n; ++i) xs.push_back(u(g));
    for (size_t i = 0; i < n / 4; ++i) xs.push_back(v(g) * std::ldexp(1.0, -(int)(g() % 30)));
    test<0>(xs); test<1>(xs); test<3>(xs); test<5>(xs); test<7>(xs); test<9>(xs); test<11>(xs); test<13>(xs); test<15>(xs);
}
// (diagnostic) branch of each mismatch
int diag(size_t n) {
    std::mt19937_64 g(7);
    std::uniform_real_distribution<double> u(-40.0, 40.0);
    int cnt[2][4] = {};
    for (size_t i = 0; i < n; ++i) {
        double x = u(g);
        for (int w = 0; w < 2; ++w) {
            double mine = w ? G<1>::cos(x) : G<1>::sin(x), ref = w ? std::cos(x) : std::sin(x);
            if (mine == ref) continue;
            double ax = std::fabs(x), a = 0, da = 0; int br;
            if (ax < 0.855469) { a = x; br = 0; }
            else if (ax < 2.426265) { double y = hp0 - ax; a = y + hp1; da = (y - a) + hp1; br = 1; }
            else { int q = G<1>::reduce(x, &a, &da); br = 2; bool c = ((q + w) & 1); if (c) br = 3; }
            cnt[w][br]++;
            if (cnt[w][br] <= 3) std::printf("w=%d br=%d x=%.17g a=%.17g da=%.3g taylor=%d mine=%a ref=%a\n", w, br, x, a, da,
                                            std::fabs(a) < 0.126, mine, ref);
        }
    }
    std::printf("sin: %d %d %d %d  cos: %d %d %d %d\n", cnt[0][0], cnt[0][1], cnt[0][2], cnt[0][3], cnt[1][0], cnt[1][1],
                cnt[1][2], cnt[1][3]);
    return 0;
}
