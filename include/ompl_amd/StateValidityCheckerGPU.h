// StateValidityCheckerGPU.h — drop-in for ompl::base::StateValidityChecker
// (base/StateValidityChecker.h:85-161) for the closed set of device predicates of
// include/ompl_gpu.h (AllValid, HypercubeBenchmark, spheres, Circles2D, KinematicChain).
// A planner's SpaceInformation takes it through setStateValidityChecker
// (SpaceInformation.h:146-157):
//
//     auto svc = std::make_shared<ompl_amd::StateValidityCheckerGPU>(si.get(), space, checker, 0,
//         [&](const ompl::base::State *s, double *out) { /* StateSpace::copyToReals */ });
//     si->setStateValidityChecker(svc);
//
// isValid(state) — the single-state call planners make (si_->isValid, e.g. BIT*'s sample filter
// ImplicitGraph.cpp:981, PRM's growRoadmap) — runs on the host CPU the same predicate source the
// device kernel runs (ompl_gpu_svc_check_host; device_space.h is __host__ __device__): one state
// is cheaper to test in place than to send to the GPU.  The result is bit-identical to the device
// predicate for every checker without libm calls (all but KinematicChain, whose cos / sin are
// glibc's on the host, exactly the reference's).  isValid(states, out) is the batched extension:
// one device launch for many states.  clearance() keeps the reference default (0, no
// clearance computation, specs_ NONE).  Thread safe: the host path is reentrant, the batched
// path is serialised on the handle's mutex (StateValidityChecker.h:87-89).
#pragma once

#include <cstdint>
#include <functional>
#include <string>
#include <utility>
#include <vector>

#include "../ompl_gpu.h"
#include "ompl_surface_base.h"

namespace ompl_amd {

class StateValidityCheckerGPU : public ompl::base::StateValidityChecker {
public:
    using StateRealPacker = std::function<void(const ompl::base::State *, double *)>;

    StateValidityCheckerGPU(ompl::base::SpaceInformation *si, const ompl_gpu_space &space,
                            const ompl_gpu_checker &checker, int device, StateRealPacker packer)
      : ompl::base::StateValidityChecker(si), dim_(space.dim), packer_(std::move(packer)) {
        if (!packer_) throw ompl::Exception("StateValidityCheckerGPU: a state packer is required");
        const ompl_gpu_status st = ompl_gpu_mv_create(&h_, &space, &checker, device);
        if (st != OMPL_GPU_OK) raise(st, "create");
    }
    ~StateValidityCheckerGPU() override {
        if (h_) ompl_gpu_mv_destroy(h_);
    }
    StateValidityCheckerGPU(const StateValidityCheckerGPU &) = delete;
    StateValidityCheckerGPU &operator=(const StateValidityCheckerGPU &) = delete;

    // StateValidityChecker.h:111 — host evaluation of the device predicate
    bool isValid(const ompl::base::State *state) const override {
        double buf[64];
        std::vector<double> big;
        double *x = buf;
        if (dim_ > 64) {
            big.resize(dim_);
            x = big.data();
        }
        packer_(state, x);
        uint8_t v = 0;
        const ompl_gpu_status st = ompl_gpu_svc_check_host(h_, x, 1, &v);
        if (st != OMPL_GPU_OK) raise(st, "isValid");
        return v != 0;
    }

    // Batched extension: out[i] = isValid(states[i]), one device launch.
    void isValid(const std::vector<const ompl::base::State *> &states, std::vector<uint8_t> &out) const {
        out.assign(states.size(), 0);
        if (states.empty()) return;
        std::vector<double> x(states.size() * dim_);
        for (std::size_t i = 0; i < states.size(); ++i) packer_(states[i], x.data() + i * dim_);
        isValidReals(x.data(), states.size(), out.data());
    }
    // the same on packed reals (AoS rows of the space's dimension)
    void isValidReals(const double *reals, std::size_t m, uint8_t *out) const {
        const ompl_gpu_status st = ompl_gpu_svc_check(h_, reals, m, out);
        if (st != OMPL_GPU_OK) raise(st, "isValid (batched)");
    }

    ompl_gpu_mv *handle() const { return h_; }

private:
    [[noreturn]] static void raise(ompl_gpu_status st, const char *what) {
        throw ompl::Exception(std::string("StateValidityCheckerGPU: ") + what + " failed (status " +
                              std::to_string((int)st) + "): " + ompl_gpu_last_error());
    }

    ompl_gpu_mv *h_ = nullptr;
    int dim_ = 0;
    StateRealPacker packer_;
};

}  // namespace ompl_amd
