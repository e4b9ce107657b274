// feat_dist.h — exact fp64 distance on feature rows (device), shared by the kNN kernels.
#pragma once
#include "device_space.h"

namespace ompl_amd {

// ---------------------------------------------------------------------------------
// distance on features (element first, query second: NearestNeighborsLinear.h:104)
template <int SP, int F, int NMAX>
__device__ __forceinline__ double feat_dist(const double *s, const double *q, const DevSpace &sp) {
    if constexpr (SP == OMPL_GPU_SPACE_REALVECTOR) {
        double acc = 0.0;
#pragma unroll
        for (int f = 0; f < F; ++f) {
            double diff = s[f] - q[f];
            acc += diff * diff;
        }
        return sqrt(acc);
    } else if constexpr (SP == OMPL_GPU_SPACE_SO3) {
        return so3_arc(s, q);
    } else if constexpr (SP == OMPL_GPU_SPACE_SE3) {
        return se3_dist(s, q, sp.w0, sp.w1);
    } else {
        return chain_dist_feat<NMAX>(s, q, sp.dim, sp.link);
    }
}

template <int F>
struct LdsStride {
    static constexpr int value = (F + 1) & ~1;  // even -> 16-byte aligned rows for ds_read_b128
};

}  // namespace ompl_amd
