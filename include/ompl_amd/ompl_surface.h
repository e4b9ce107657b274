// ompl_surface.h — the slice of the OMPL plugin surface the GPU backend implements.
//
// With a real OMPL installation (or the reference tree on the include path) define
// OMPL_AMD_WITH_OMPL and the genuine headers are used:
//     <ompl/datastructures/NearestNeighbors.h>   (NearestNeighbors.h:46-115)
//     <ompl/util/Exception.h>
// Without it (standalone builds of this repo) the same abstract interface is declared
// here, signature for signature, so the plugin compiles and runs on its own.
#pragma once

#include "ompl_surface_rng.h"  // ompl::RNG (one per NN instance, as GNAT's GreedyKCenters::rng_)

#ifdef OMPL_AMD_WITH_OMPL
#include <ompl/datastructures/NearestNeighbors.h>
#include <ompl/util/Exception.h>
#else
#include <cstddef>
#include <functional>
#include <stdexcept>
#include <string>
#include <vector>

namespace ompl {

// ompl::Exception (util/Exception.h): a std::runtime_error
class Exception : public std::runtime_error {
public:
    explicit Exception(const std::string &what) : std::runtime_error(what) {}
    Exception(const std::string &prefix, const std::string &what) : std::runtime_error(prefix + ": " + what) {}
};

// ompl::NearestNeighbors<_T> — the abstract container planners hold as nn_
template <typename _T>
class NearestNeighbors {
public:
    using DistanceFunction = std::function<double(const _T &, const _T &)>;
    NearestNeighbors() = default;
    virtual ~NearestNeighbors() = default;
    virtual void setDistanceFunction(const DistanceFunction &distFun) { distFun_ = distFun; }
    const DistanceFunction &getDistanceFunction() const { return distFun_; }
    virtual bool reportsSortedResults() const = 0;
    virtual void clear() = 0;
    virtual void add(const _T &data) = 0;
    virtual void add(const std::vector<_T> &data) {
        for (const auto &d : data) add(d);
    }
    virtual bool remove(const _T &data) = 0;
    virtual _T nearest(const _T &data) const = 0;
    virtual void nearestK(const _T &data, std::size_t k, std::vector<_T> &nbh) const = 0;
    virtual void nearestR(const _T &data, double radius, std::vector<_T> &nbh) const = 0;
    virtual std::size_t size() const = 0;
    virtual void list(std::vector<_T> &data) const = 0;

protected:
    DistanceFunction distFun_;
};

}  // namespace ompl
#endif
