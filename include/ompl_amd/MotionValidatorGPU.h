// MotionValidatorGPU.h — drop-in MI355X replacement for ompl::base::DiscreteMotionValidator
// (base/src/DiscreteMotionValidator.cpp:48-145) behind the unchanged ompl::base::MotionValidator
// interface (base/MotionValidator.h:64-140).  A planner's SpaceInformation takes it through
// setMotionValidator (SpaceInformation.h:168-172):
//
//     auto mv = std::make_shared<ompl_amd::MotionValidatorGPU>(si.get(), space, checker, 0,
//         [&](const ompl::base::State *s, double *out) { /* StateSpace::copyToReals */ },
//         [&](const ompl::base::State *a, const ompl::base::State *b, double t, ompl::base::State *o) {
//             si->getStateSpace()->interpolate(a, b, t, o); });
//     si->setMotionValidator(mv);
//
// The device evaluates the closed set of validity checkers of include/ompl_gpu.h (the
// predicate is data, not code), so arbitrary user isValid code stays with the reference's
// validator.  The packer hands the device a state's reals in copyToReals order
// (StateSpace.h:404).  The lastValid overload asks the device for the first invalid sample of
// the linear sweep and, like the reference (:66-68, :79-81), interpolates lastValid.first on
// the host.  checkMotions() is the batched extension: many edges per launch.  The counters
// are the base class's valid_ / invalid_ (MotionValidator.h:136-139).  Calls are serialised
// on the handle's mutex, so the validator is thread safe as the interface requires
// (MotionValidator.h:60-63).
#pragma once

#include <cstdint>
#include <functional>
#include <string>
#include <utility>
#include <vector>

#include "../ompl_gpu.h"
#include "ompl_surface_base.h"

namespace ompl_amd {

class MotionValidatorGPU : public ompl::base::MotionValidator {
public:
    using StateRealPacker = std::function<void(const ompl::base::State *, double *)>;
    using Interpolator =
        std::function<void(const ompl::base::State *, const ompl::base::State *, double, ompl::base::State *)>;

    MotionValidatorGPU(ompl::base::SpaceInformation *si, const ompl_gpu_space &space, const ompl_gpu_checker &checker,
                       int device, StateRealPacker packer, Interpolator interpolate = nullptr)
      : ompl::base::MotionValidator(si), dim_(space.dim), packer_(std::move(packer)),
        interp_(std::move(interpolate)) {
        if (!packer_) throw ompl::Exception("MotionValidatorGPU: a state packer is required");
        const ompl_gpu_status st = ompl_gpu_mv_create(&h_, &space, &checker, device);
        if (st != OMPL_GPU_OK) raise(st, "create");
    }
    ~MotionValidatorGPU() override {
        if (h_) ompl_gpu_mv_destroy(h_);
    }
    MotionValidatorGPU(const MotionValidatorGPU &) = delete;
    MotionValidatorGPU &operator=(const MotionValidatorGPU &) = delete;

    // DiscreteMotionValidator.cpp:93-145: s2 first, then the bisection samples; s1 assumed valid
    bool checkMotion(const ompl::base::State *s1, const ompl::base::State *s2) const override {
        uint8_t v = 0;
        run(&s1, &s2, 1, &v, nullptr, nullptr);
        count(v != 0);
        return v != 0;
    }

    // DiscreteMotionValidator.cpp:48-91: linear sweep; on failure lastValid.second = (j - 1) / nd
    // of the first invalid sample j (nd when only s2 fails) and lastValid.first is interpolated there
    bool checkMotion(const ompl::base::State *s1, const ompl::base::State *s2,
                     std::pair<ompl::base::State *, double> &lastValid) const override {
        uint8_t v = 0;
        int32_t nd = 0, fi = -1;
        run(&s1, &s2, 1, &v, &nd, &fi);
        count(v != 0);
        if (!v) {
            lastValid.second = (double)(fi - 1) / (double)nd;
            if (lastValid.first != nullptr) {
                if (!interp_) throw ompl::Exception("MotionValidatorGPU: lastValid.first needs an interpolator");
                interp_(s1, s2, lastValid.second, lastValid.first);
            }
        }
        return v != 0;
    }

    // Batched extension: valid[i] = checkMotion(edges[i].first, edges[i].second), one launch.
    void checkMotions(const std::vector<std::pair<const ompl::base::State *, const ompl::base::State *>> &edges,
                      std::vector<uint8_t> &valid) const {
        std::vector<const ompl::base::State *> a(edges.size()), b(edges.size());
        for (std::size_t i = 0; i < edges.size(); ++i) {
            a[i] = edges[i].first;
            b[i] = edges[i].second;
        }
        valid.assign(edges.size(), 0);
        if (edges.empty()) return;
        run(a.data(), b.data(), edges.size(), valid.data(), nullptr, nullptr);
        for (uint8_t v : valid) count(v != 0);
    }

private:
    [[noreturn]] static void raise(ompl_gpu_status st, const char *what) {
        throw ompl::Exception(std::string("MotionValidatorGPU: ") + what + " failed (status " + std::to_string((int)st) +
                              "): " + ompl_gpu_last_error());
    }
    void count(bool v) const {
        if (v)
            ++valid_;
        else
            ++invalid_;
    }
    void run(const ompl::base::State *const *s1, const ompl::base::State *const *s2, std::size_t m, uint8_t *valid,
             int32_t *nd, int32_t *fi) const {
        std::vector<double> a(m * dim_), b(m * dim_);
        for (std::size_t i = 0; i < m; ++i) {
            packer_(s1[i], a.data() + i * dim_);
            packer_(s2[i], b.data() + i * dim_);
        }
        const ompl_gpu_status st = ompl_gpu_mv_check(h_, a.data(), b.data(), m, valid, nd, fi);
        if (st != OMPL_GPU_OK) raise(st, "checkMotion");
    }

    ompl_gpu_mv *h_ = nullptr;
    int dim_ = 0;
    StateRealPacker packer_;
    Interpolator interp_;
};

}  // namespace ompl_amd
