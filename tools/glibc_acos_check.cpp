// glibc_acos_check.cpp — measurement tool (not product): the product header
// ompl_amd/csrc/glibc_acos.h (host form, hipcc, -ffp-contract=off as the library) against the host's
// glibc acos on 8 threads, over every branch of e_asin.c's __ieee754_acos: uniform |x| in each
// branch's range (both signs), |x| within 2^-60 .. 2^-20 of 1, of the branch and table-interval
// boundaries, and the dot products SO3 distances take (|q1.q2| of uniform quaternions).
//   hipcc -O2 -ffp-contract=off -o tools/bin/glibc_acos_check tools/glibc_acos_check.cpp -lpthread
//   tools/bin/glibc_acos_check [n per set]
#include <math.h>

#include <cmath>
#include <cstdio>
#include <random>
#include <thread>
#include <vector>

#include "../ompl_amd/csrc/glibc_acos.h"

static double (*volatile g_acos)(double) = ::acos;

static const double kEdges[] = {0x1p-54, 0.125, 0.25, 0.5, 0.75, 0.921875, 0.953125, 0.96875, 1.0};

static double draw(int set, std::mt19937_64 &g) {
    std::uniform_real_distribution<double> u(0.0, 1.0);
    const double sgn = (g() & 1) ? -1.0 : 1.0;
    switch (set) {
    case 0: {  // uniform in one branch's range
        const int b = (int)(g() % 8);
        return sgn * (kEdges[b] + (kEdges[b + 1] - kEdges[b]) * u(g));
    }
    case 1:  // near 1
        return sgn * (1.0 - std::ldexp(u(g), -(int)(20 + g() % 41)));
    case 2: {  // near a branch edge or a table-interval edge (multiples of 2^-10 .. 2^-7 of the mantissa)
        double e = (g() & 1) ? kEdges[g() % 9] : std::ldexp(std::floor(u(g) * 1024.0), -10);
        return sgn * std::nextafter(e, (g() & 1) ? 2.0 : -2.0) * (1.0 + (double)((int)(g() % 7) - 3) * 0x1p-52);
    }
    case 3: {  // tiny
        return sgn * std::ldexp(u(g), -(int)(g() % 70));
    }
    default: {  // |q1.q2| of two uniform unit quaternions (the SO3 distance's argument)
        double q[8], n1 = 0, n2 = 0;
        std::normal_distribution<double> nd;
        for (int i = 0; i < 8; ++i) q[i] = nd(g);
        for (int i = 0; i < 4; ++i) n1 += q[i] * q[i], n2 += q[4 + i] * q[4 + i];
        const double dq = std::fabs((q[0] * q[4] + q[1] * q[5] + q[2] * q[6] + q[3] * q[7]) / std::sqrt(n1 * n2));
        return dq > 1.0 ? 1.0 : dq;
    }
    }
}

static void run(int set, uint64_t seed, uint64_t n, uint64_t *bad) {
    std::mt19937_64 g(seed);
    uint64_t b = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const double x = draw(set, g);
        const double r = ompl_amd::glibc_acos(x), e = g_acos(x);
        if (std::isnan(e) ? !std::isnan(r) : (r != e || std::signbit(r) != std::signbit(e))) {
            if (b < 5) std::printf("  x = %a: restatement %a, glibc %a\n", x, r, e);
            ++b;
        }
    }
    *bad = b;
}

int main(int argc, char **argv) {
    const uint64_t n = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 8000000ull;
    int rc = 0;
    const double special[] = {0.0, -0.0, 1.0, -1.0, 1.0000000000000002, -1.5, INFINITY, -INFINITY, NAN, 0x1p-1074};
    for (double x : special) {
        const double r = ompl_amd::glibc_acos(x), e = g_acos(x);
        if (!(r == e || (std::isnan(r) && std::isnan(e)))) {
            std::printf("special x = %a: restatement %a, glibc %a\n", x, r, e);
            rc = 1;
        }
    }
    for (int set = 0; set < 5; ++set) {
        uint64_t bad[8];
        std::vector<std::thread> th;
        for (int t = 0; t < 8; ++t) th.emplace_back(run, set, (uint64_t)(7919 * set + t), n / 8, &bad[t]);
        for (auto &t : th) t.join();
        uint64_t tot = 0;
        for (uint64_t b : bad) tot += b;
        std::printf("{\"set\": %d, \"arguments\": %llu, \"differences\": %llu}\n", set, (unsigned long long)n,
                    (unsigned long long)tot);
        rc |= tot != 0;
    }
    return rc;
}
