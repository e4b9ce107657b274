// knn_fast_so3.hip — SO(3) instantiation of the fp32 screen + fp64 certificate (knn_fast_impl.h).
// SO3 has no sorted store (no culling): the chunked brute-force screen serves it.
#include "knn_fast_impl.h"

namespace ompl_amd {

hipError_t fast_so3(const DevSpace &sp, const FeatGeom &g, const double *feat64, const float *feat32, uint64_t cap,
                    uint64_t n_end, const SortedStore *, const double *qfeat64, uint32_t nq, uint32_t k,
                    const FastBounds &b, double *out_d, uint32_t *out_i, void *ws, size_t ws_bytes, int num_cus,
                    hipStream_t st, uint32_t **fail_count, uint32_t **fail_list) {
    return fast_entry<OMPL_GPU_SPACE_SO3, 4>(sp, g, feat64, feat32, cap, n_end, nullptr, qfeat64, nq, k, b, out_d,
                                             out_i, ws, ws_bytes, num_cus, st, fail_count, fail_list);
}

hipError_t fast_so3_build(const FeatGeom &, const float *, uint64_t, uint32_t, const FastBounds &, SortedStore *,
                          hipStream_t) {
    return hipErrorInvalidValue;
}

hipError_t fast_so3_radius(const DevSpace &, const FeatGeom &, const double *, uint64_t, const SortedStore *,
                           const double *, uint32_t, double, const FastBounds &, void *, size_t, int, uint64_t **,
                           uint32_t *, double *, hipStream_t) {
    return hipErrorInvalidValue;  // no sorted store for SO3: nearestR runs the exact scan
}

}  // namespace ompl_amd
