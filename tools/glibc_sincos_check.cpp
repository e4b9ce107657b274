// glibc_sincos_check.cpp — measurement tool (not product): the product header
// ompl_amd/csrc/glibc_sincos.h (host form, hipcc, -ffp-contract=off as the library) against the
// host's glibc sin, cos and sincos on 8 threads.  hipcc -O2 -ffp-contract=off -o tools/bin/glibc_sincos_check
// tools/glibc_sincos_check.cpp -lpthread;  tools/bin/glibc_sincos_check [n per set]
#include <math.h>

#include <cmath>
#include <cstdio>
#include <random>
#include <thread>
#include <vector>

#include "../ompl_amd/csrc/glibc_sincos.h"

// the host's glibc through function pointers, so no compiler folds a sin / cos pair into sincos
static double (*volatile g_sin)(double) = ::sin;
static double (*volatile g_cos)(double) = ::cos;
static void (*volatile g_sincos)(double, double *, double *) = ::sincos;

static void run(int kind, uint64_t seed, uint64_t n, uint64_t *bad) {
    std::mt19937_64 g(seed);
    std::uniform_real_distribution<double> u(-100.0, 100.0), v(-1.0, 1.0);
    uint64_t b = 0;
    for (uint64_t i = 0; i < n; ++i) {
        double x;
        if (kind == 0) x = u(g);
        else if (kind == 1) x = (int)(g() % 121 - 60) * 1.5707963267948966 + v(g) * std::pow(10.0, -6.0 - (double)(g() % 10));
        else x = v(g) * std::ldexp(1.0, -(int)(g() % 40));
        double s, c, gs, gc;
        ompl_amd::glibc_sincos(x, s, c);
        g_sincos(x, &gs, &gc);
        b += (s != gs) + (c != gc) + (ompl_amd::glibc_sin(x) != g_sin(x)) + (ompl_amd::glibc_cos(x) != g_cos(x));
    }
    *bad = b;
}

int main(int argc, char **argv) {
    const uint64_t n = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 8000000ull;
    int rc = 0;
    for (int kind = 0; kind < 3; ++kind) {
        uint64_t bad[8];
        std::vector<std::thread> th;
        for (int t = 0; t < 8; ++t) th.emplace_back(run, kind, (uint64_t)(977 * kind + t), n / 8, &bad[t]);
        for (auto &t : th) t.join();
        uint64_t tot = 0;
        for (uint64_t b : bad) tot += b;
        std::printf("{\"set\": %d, \"arguments\": %llu, \"differences\": %llu}\n", kind, (unsigned long long)n,
                    (unsigned long long)tot);
        rc |= tot != 0;
    }
    return rc;
}
