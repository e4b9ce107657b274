// ompl_surface_base.h — the slice of OMPL's base plugin surface MotionValidatorGPU implements:
// ompl::base::State, SpaceInformation (opaque) and MotionValidator.
//
// With a real OMPL installation define OMPL_AMD_WITH_OMPL and the genuine header is used:
//     <ompl/base/MotionValidator.h>              (base/MotionValidator.h:64-140)
// Without it the same abstract interface is declared here, member for member.  (The
// reference's base/State.h needs Boost, absent from this image, so only the standalone
// form is compiled by the tests.)
#pragma once

#include "ompl_surface.h"

#ifdef OMPL_AMD_WITH_OMPL
#include <ompl/base/MotionValidator.h>
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

}  // namespace base
}  // namespace ompl
#endif
