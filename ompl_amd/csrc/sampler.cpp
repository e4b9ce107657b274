// sampler.cpp — the reference's input streams: RNG seed generator + uniform state samplers, as
// C-ABI entry points (include/ompl_gpu.h "reference RNG streams").  Host code: the samplers are
// sequential std::mt19937 streams (util/src/RandomNumbers.cpp), produced here once and uploaded;
// they are what planners feed the hot path, not part of it.
//
//   RNG::setSeed / getSeed                    util/src/RandomNumbers.cpp:208-216
//   StateSpace::allocStateSampler             base/src/StateSpace.cpp:800-806
//   CompoundStateSpace::allocDefaultStateSampler (one RNG for the compound sampler, then one per
//                                             component, in component order) StateSpace.cpp:1118-1128
//   CompoundStateSampler::sampleUniform       base/src/StateSampler.cpp:47-52
//   RealVectorStateSampler::sampleUniform     base/spaces/src/RealVectorStateSpace.cpp:45-53
//   SO3StateSampler::sampleUniform            base/spaces/src/SO3StateSpace.cpp:99-102 -> RNG::quaternion
//   KinematicChainSpace (RealVectorStateSpace(n) with bounds [-pi, pi])  demos/KinematicChain.h:87-100
#include <cstring>
#include <new>

#include "../../include/ompl_gpu.h"
#include "sampler_impl.h"

void ompl_gpu_sampler::sample(size_t n, double *out) {
    for (size_t i = 0; i < n; ++i) {
        double *o = out + i * dim;
        for (int c = 0; c < nrn; ++c) o[c] = rn->uniformReal(low[c], high[c]);
        if (so3) so3->quaternion(o + nrn);
    }
}

namespace ompl_amd {
void set_last_error(const char *msg);  // capi.hip
}

extern "C" {

void ompl_gpu_rng_set_seed(uint32_t seed) { ompl::RNG::setSeed(seed); }

uint32_t ompl_gpu_rng_get_seed(void) { return (uint32_t)ompl::RNG::getSeed(); }

uint64_t ompl_gpu_rng_seeds_drawn(void) { return ompl::rng_detail::seedGenerator().drawn(); }

uint32_t ompl_gpu_rng_next_seed(void) { return (uint32_t)ompl::rng_detail::seedGenerator().nextSeed(); }

ompl_gpu_status ompl_gpu_rng_uniform_real(uint32_t local_seed, size_t n, double low, double high, double *out) {
    if (n && !out) {
        ompl_amd::set_last_error("NULL argument");
        return OMPL_GPU_ERR_INVALID_ARG;
    }
    ompl::RNG rng(local_seed);  // RandomNumbers.cpp:225-228: no seed drawn from the generator
    for (size_t i = 0; i < n; ++i) out[i] = rng.uniformReal(low, high);
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_sampler_create(ompl_gpu_sampler **out, const ompl_gpu_space *space, const double *low,
                                        const double *high) {
    if (!out || !space) {
        ompl_amd::set_last_error("NULL argument");
        return OMPL_GPU_ERR_INVALID_ARG;
    }
    *out = nullptr;
    const int kind = space->kind, dim = space->dim;
    int nrn = 0;
    double dlo = 0.0, dhi = 1.0;
    switch (kind) {
    case OMPL_GPU_SPACE_REALVECTOR: nrn = dim; break;
    case OMPL_GPU_SPACE_SE3: nrn = 3; break;
    case OMPL_GPU_SPACE_SO3: nrn = 0; break;
    case OMPL_GPU_SPACE_KCHAIN:
        nrn = dim;
        dlo = -3.141592653589793238462643383279502884;  // KinematicChain.h: bounds.setLow(-M_PI)
        dhi = 3.141592653589793238462643383279502884;
        break;
    default: ompl_amd::set_last_error("unsupported state space"); return OMPL_GPU_ERR_UNSUPPORTED;
    }
    if (dim < 1 || (kind == OMPL_GPU_SPACE_SE3 && dim != 7) || (kind == OMPL_GPU_SPACE_SO3 && dim != 4)) {
        ompl_amd::set_last_error("state dimension does not match the space");
        return OMPL_GPU_ERR_INVALID_ARG;
    }
    auto *s = new (std::nothrow) ompl_gpu_sampler();
    if (!s) return OMPL_GPU_ERR_OOM;
    s->kind = kind;
    s->dim = dim;
    s->nrn = nrn;
    s->low.assign(nrn, dlo);
    s->high.assign(nrn, dhi);
    for (int i = 0; i < nrn; ++i) {
        if (low) s->low[i] = low[i];
        if (high) s->high[i] = high[i];
    }
    if (kind == OMPL_GPU_SPACE_SE3) {  // CompoundStateSampler, then R^3, then SO3
        s->compound.reset(new ompl::RNG());
        s->rn.reset(new ompl::RNG());
        s->so3.reset(new ompl::RNG());
    } else if (kind == OMPL_GPU_SPACE_SO3) {
        s->so3.reset(new ompl::RNG());
    } else {
        s->rn.reset(new ompl::RNG());
    }
    *out = s;
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_sampler_destroy(ompl_gpu_sampler *s) {
    delete s;
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_sampler_sample_uniform(ompl_gpu_sampler *s, size_t n, double *out) {
    if (!s || (n && !out)) {
        ompl_amd::set_last_error("NULL argument");
        return OMPL_GPU_ERR_INVALID_ARG;
    }
    s->sample(n, out);
    return OMPL_GPU_OK;
}

ompl_gpu_status ompl_gpu_sampler_local_seeds(const ompl_gpu_sampler *s, uint32_t *seeds, int *count) {
    if (!s || !seeds || !count) {
        ompl_amd::set_last_error("NULL argument");
        return OMPL_GPU_ERR_INVALID_ARG;
    }
    int c = 0;
    for (const auto *r : {s->compound.get(), s->rn.get(), s->so3.get()})
        if (r) seeds[c++] = (uint32_t)r->getLocalSeed();
    *count = c;
    return OMPL_GPU_OK;
}

}  // extern "C"
