// ompl_surface_base.h — the slice of OMPL's base plugin surface MotionValidatorGPU and
// StateValidityCheckerGPU implement: ompl::base::State, SpaceInformation (opaque),
// MotionValidator and StateValidityChecker.
//
// With a real OMPL installation define OMPL_AMD_WITH_OMPL and the genuine headers are used:
//     <ompl/base/MotionValidator.h>              (base/MotionValidator.h:64-140)
//     <ompl/base/StateValidityChecker.h>         (base/StateValidityChecker.h:57-185)
// Without it the same abstract interface is declared here, member for member.  (The
// reference's base/State.h needs Boost, absent from this image, so only the standalone
// form is compiled by the tests.)
#pragma once

#include "ompl_surface.h"

#ifdef OMPL_AMD_WITH_OMPL
#include <ompl/base/MotionValidator.h>
#include <ompl/base/StateValidityChecker.h>
#else
#include <memory>
#include <utility>

namespace ompl {
namespace base {

// base/State.h:52-84: an opaque, space-specific state
class State {
protected:
    State() = default;
    virtual ~State() = default;
};

class SpaceInformation;

// base/MotionValidator.h:64-140
class MotionValidator {
public:
    MotionValidator(SpaceInformation *si) : si_(si), valid_(0), invalid_(0) {}
    virtual ~MotionValidator() = default;
    virtual bool checkMotion(const State *s1, const State *s2) const = 0;
    virtual bool checkMotion(const State *s1, const State *s2, std::pair<State *, double> &lastValid) const = 0;
    unsigned int getValidMotionCount() const { return valid_; }
    unsigned int getInvalidMotionCount() const { return invalid_; }
    unsigned int getCheckedMotionCount() const { return valid_ + invalid_; }
    double getValidMotionFraction() const {
        return valid_ == 0 ? 0.0 : (double)valid_ / (double)(invalid_ + valid_);
    }
    void resetMotionCounter() { valid_ = invalid_ = 0; }

protected:
    SpaceInformation *si_;
    mutable unsigned int valid_;
    mutable unsigned int invalid_;
};

using MotionValidatorPtr = std::shared_ptr<MotionValidator>;

// base/StateValidityChecker.h:57-80
struct StateValidityCheckerSpecs {
    enum ClearanceComputationType { NONE = 0, EXACT, APPROXIMATE, BOUNDED_APPROXIMATE };
    StateValidityCheckerSpecs() = default;
    ClearanceComputationType clearanceComputationType{NONE};
    bool hasValidDirectionComputation{false};
};

// base/StateValidityChecker.h:85-161
class StateValidityChecker {
public:
    StateValidityChecker(SpaceInformation *si) : si_(si) {}
    virtual ~StateValidityChecker() = default;
    virtual bool isValid(const State *state) const = 0;
    virtual bool isValid(const State *state, double &dist) const {
        dist = clearance(state);
        return isValid(state);
    }
    virtual bool isValid(const State *state, double &dist, State *validState, bool &validStateAvailable) const {
        dist = clearance(state, validState, validStateAvailable);
        return isValid(state);
    }
    virtual double clearance(const State * /*state*/) const { return 0.0; }
    virtual double clearance(const State *state, State * /*validState*/, bool &validStateAvailable) const {
        validStateAvailable = false;
        return clearance(state);
    }
    const StateValidityCheckerSpecs &getSpecs() const { return specs_; }

protected:
    SpaceInformation *si_;
    StateValidityCheckerSpecs specs_;
};

using StateValidityCheckerPtr = std::shared_ptr<StateValidityChecker>;

}  // namespace base
}  // namespace ompl
#endif
