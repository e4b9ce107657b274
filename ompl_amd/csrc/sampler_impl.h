// sampler_impl.h — the sampler handle behind include/ompl_gpu.h's ompl_gpu_sampler, shared by
// sampler.cpp (its C ABI) and capi.hip (BIT*'s batch sampler, which needs to rewind a stream to
// the exact try the reference loop stops at).
#pragma once
#include <cstddef>
#include <memory>
#include <vector>

#include "../../include/ompl_amd/ompl_surface_rng.h"

struct ompl_gpu_sampler {
    int kind = 0, dim = 0, nrn = 0;  // nrn: reals of the R^n part (SE3: 3; SO3: 0)
    std::vector<double> low, high;
    // construction order of the reference: [compound], R^n / SO3 component samplers
    std::unique_ptr<ompl::RNG> compound, rn, so3;

    // n successive sampleUniform calls (StateSampler.cpp:47-52, RealVectorStateSpace.cpp:45-53,
    // SO3StateSpace.cpp:99-102), AoS rows; defined in sampler.cpp (g++ and glibc libm, like the
    // reference build)
    void sample(size_t n, double *out);
};

namespace ompl_amd {
// a copy of the sampler's engine states (the compound RNG draws nothing while sampling)
struct SamplerMark {
    std::unique_ptr<ompl::RNG> rn, so3;
    explicit SamplerMark(const ompl_gpu_sampler &s)
        : rn(s.rn ? new ompl::RNG(*s.rn) : nullptr), so3(s.so3 ? new ompl::RNG(*s.so3) : nullptr) {}
    void rewind(ompl_gpu_sampler &s) const {
        if (rn) *s.rn = *rn;
        if (so3) *s.so3 = *so3;
    }
};
}  // namespace ompl_amd
