// SelfConfigGPU.h — default-selection hook for the GPU nearest-neighbour structure, the
// counterpart of tools::SelfConfig::getDefaultNearestNeighbors (tools/config/SelfConfig.h:106-117),
// which every planner's setup() calls when no structure was set (RRT.cpp:77-79,
// RRTstar.cpp:104-106, PRM.cpp:158-163, ImplicitGraph.cpp:110-119).
//
// The reference picks GNAT / GNAT-NoThreadSafety for metric spaces and SqrtApprox otherwise.
// getDefaultNearestNeighbors<_T>() below returns a NearestNeighborsGPU<_T> for a metric space
// when the GPU structure was requested — OMPL_AMD_NN=gpu in the environment, or
// setGpuNearestNeighborsDefault(true) — and a GPU space was configured (setDefaultGpuSpace);
// otherwise nullptr, and the caller keeps the reference's choice.  INTEGRATION.md shows the
// one-line SelfConfig.h patch that consults it; with it, OMPL_AMD_NN=gpu switches every planner.
#pragma once

#include <cstdlib>
#include <cstring>

#include "NearestNeighborsGPU.h"

namespace ompl_amd {

// -1: follow the environment; 0 / 1: set by the program
inline int &gpuDefaultOverride() {
    static int v = -1;
    return v;
}
inline void setGpuNearestNeighborsDefault(bool on) { gpuDefaultOverride() = on ? 1 : 0; }

inline bool gpuNearestNeighborsRequested() {
    if (gpuDefaultOverride() >= 0) return gpuDefaultOverride() == 1;
    const char *e = std::getenv("OMPL_AMD_NN");
    return e && (std::strcmp(e, "gpu") == 0 || std::strcmp(e, "GPU") == 0);
}

// metricSpace: StateSpace::isMetricSpace() of the planner's space (SelfConfig.h:110)
template <typename _T>
ompl::NearestNeighbors<_T> *getDefaultNearestNeighbors(bool metricSpace) {
    if (!metricSpace || !gpuNearestNeighborsRequested() || !gpuDefaults().configured) return nullptr;
    return new NearestNeighborsGPU<_T>();
}

}  // namespace ompl_amd
