// ompl_surface_rng.h — ompl::RNG, the reference's random-number source (util/RandomNumbers.h:56-197,
// util/src/RandomNumbers.cpp:53-279), for the plugin surface.
//
// With OMPL_AMD_WITH_OMPL the genuine <ompl/util/RandomNumbers.h> is used.  Without it the same
// class is declared here, behaviour for behaviour, because seed-stream alignment is part of the
// drop-in contract: every RNG() draws the next seed from one process-wide seed generator
// (std::ranlux24_base + std::uniform_int_distribution<>(1, 1e9), RandomNumbers.cpp:53-113), so a
// nearest-neighbour structure that constructs a different number of RNGs than the reference's
// (GNAT owns one, GreedyKCenters.h:127) shifts the streams of every sampler built after it.
// The generators and distributions are the C++ standard library's, exactly as the reference uses
// them, so the streams are the reference's on the same standard library.
//
// Not restated: uniformNormalVector / uniformInBall / the prolate-hyperspheroid samplers (they
// use boost::uniform_on_sphere and are off the hot path).
#pragma once

// (the genuine header needs the generated ompl/config.h of an installed OMPL; a bare source tree
// such as the reference's falls back to the declaration below)
#if defined(OMPL_AMD_WITH_OMPL) && __has_include(<ompl/config.h>)
#include <ompl/util/RandomNumbers.h>
#else
#include <algorithm>
#include <cassert>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <mutex>
#include <random>

namespace ompl {

namespace rng_detail {
// RandomNumbers.cpp:53-113
class SeedGenerator {
public:
    SeedGenerator()
      : firstSeed_(std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::system_clock::now() -
                                                                         std::chrono::system_clock::time_point::min())
                       .count()),
        sGen_(firstSeed_), sDist_(1, 1000000000) {}
    std::uint_fast32_t firstSeed() {
        std::lock_guard<std::mutex> lk(mu_);
        return firstSeed_;
    }
    void setSeed(std::uint_fast32_t seed) {
        std::lock_guard<std::mutex> lk(mu_);
        if (seed > 0) {
            if (someSeedsGenerated_)
                std::fprintf(stderr, "Error: Random number generation already started. Changing seed now will not "
                                     "lead to deterministic sampling.\n");
            else
                firstSeed_ = seed;
        } else {
            if (someSeedsGenerated_) {
                std::fprintf(stderr, "Warning: Random generator seed cannot be 0. Ignoring seed.\n");
                return;
            }
            std::fprintf(stderr, "Warning: Random generator seed cannot be 0. Using 1 instead.\n");
            seed = 1;
        }
        sGen_.seed(seed);  // as the reference: reseeds after the error too (RandomNumbers.cpp:71-97)
    }
    std::uint_fast32_t nextSeed() {
        std::lock_guard<std::mutex> lk(mu_);
        someSeedsGenerated_ = true;
        ++drawn_;
        return sDist_(sGen_);
    }
    // seeds handed out so far (not in the reference: lets tests observe seed consumption)
    std::uint64_t drawn() {
        std::lock_guard<std::mutex> lk(mu_);
        return drawn_;
    }

private:
    bool someSeedsGenerated_{false};
    std::uint_fast32_t firstSeed_;
    std::mutex mu_;
    std::ranlux24_base sGen_;
    std::uniform_int_distribution<> sDist_;
    std::uint64_t drawn_{0};
};

// one generator per process, created on first use (RandomNumbers.cpp:115-127)
inline SeedGenerator &seedGenerator() {
    static SeedGenerator g;
    return g;
}
}  // namespace rng_detail

class RNG {
public:
    RNG() : localSeed_(rng_detail::seedGenerator().nextSeed()), generator_(localSeed_) {}  // :218-223
    explicit RNG(std::uint_fast32_t localSeed) : localSeed_(localSeed), generator_(localSeed_) {}

    double uniform01() { return uniDist_(generator_); }
    double uniformReal(double lower_bound, double upper_bound) {
        assert(lower_bound <= upper_bound);
        return (upper_bound - lower_bound) * uniDist_(generator_) + lower_bound;
    }
    int uniformInt(int lower_bound, int upper_bound) {
        auto r = (int)std::floor(uniformReal((double)lower_bound, (double)(upper_bound) + 1.0));
        return (r > upper_bound) ? upper_bound : r;
    }
    bool uniformBool() { return uniDist_(generator_) <= 0.5; }
    double gaussian01() { return normalDist_(generator_); }
    double gaussian(double mean, double stddev) { return normalDist_(generator_) * stddev + mean; }
    double halfNormalReal(double r_min, double r_max, double focus = 3.0) {  // :244-255
        assert(r_min <= r_max);
        const double mean = r_max - r_min;
        double v = gaussian(mean, mean / focus);
        if (v > mean) v = 2.0 * mean - v;
        double r = v >= 0.0 ? v + r_min : r_min;
        return r > r_max ? r_max : r;
    }
    int halfNormalInt(int r_min, int r_max, double focus = 3.0) {  // :257-261
        auto r = (int)std::floor(halfNormalReal((double)r_min, (double)(r_max) + 1.0, focus));
        return (r > r_max) ? r_max : r;
    }
    // Shoemake, "Uniform Random Rotations" (:263-277); order x, y, z, w
    void quaternion(double value[4]) {
        constexpr double pi = 3.141592653589793238462643383279502884;
        double x0 = uniDist_(generator_);
        double r1 = std::sqrt(1.0 - x0), r2 = std::sqrt(x0);
        double t1 = 2.0 * pi * uniDist_(generator_), t2 = 2.0 * pi * uniDist_(generator_);
        double c1 = std::cos(t1), s1 = std::sin(t1);
        double c2 = std::cos(t2), s2 = std::sin(t2);
        value[0] = s1 * r1;
        value[1] = c1 * r1;
        value[2] = s2 * r2;
        value[3] = c2 * r2;
    }
    void eulerRPY(double value[3]) {  // :280-285
        constexpr double pi = 3.141592653589793238462643383279502884;
        value[0] = pi * (-2.0 * uniDist_(generator_) + 1.0);
        value[1] = std::acos(1.0 - 2.0 * uniDist_(generator_)) - pi / 2.0;
        value[2] = pi * (-2.0 * uniDist_(generator_) + 1.0);
    }
    static void setSeed(std::uint_fast32_t seed) { rng_detail::seedGenerator().setSeed(seed); }
    static std::uint_fast32_t getSeed() { return rng_detail::seedGenerator().firstSeed(); }
    void setLocalSeed(std::uint_fast32_t localSeed) {  // :230-242
        localSeed_ = localSeed;
        generator_.seed(localSeed_);
        uniDist_.reset();
        normalDist_.reset();
    }
    std::uint_fast32_t getLocalSeed() const { return localSeed_; }
    template <class RandomAccessIterator>
    void shuffle(RandomAccessIterator first, RandomAccessIterator last) {
        std::shuffle(first, last, generator_);
    }

private:
    std::uint_fast32_t localSeed_;
    std::mt19937 generator_;
    std::uniform_real_distribution<> uniDist_{0, 1};
    std::normal_distribution<> normalDist_{0, 1};
};

}  // namespace ompl
#endif
