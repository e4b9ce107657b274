// knn_fast_se3.hip — SE(3) instantiation of the fp32 screen + fp64 certificate (knn_fast_impl.h).
#include "knn_fast_impl.h"

namespace ompl_amd {

hipError_t fast_se3(const DevSpace &sp, const FeatGeom &g, const double *feat64, const float *feat32, uint64_t cap,
                    uint64_t n_end, const SortedStore *sorted, const double *qfeat64, uint32_t nq, uint32_t k,
                    const FastBounds &b, double *out_d, uint32_t *out_i, void *ws, size_t ws_bytes, int num_cus,
                    hipStream_t st, uint32_t **fail_count, uint32_t **fail_list) {
    return fast_entry<OMPL_GPU_SPACE_SE3, 7>(sp, g, feat64, feat32, cap, n_end, sorted, qfeat64, nq, k, b, out_d,
                                             out_i, ws, ws_bytes, num_cus, st, fail_count, fail_list);
}

hipError_t fast_se3_build(const FeatGeom &, const float *feat32, const double *feat64, uint64_t cap, uint64_t n_total,
                          uint32_t n_live, const uint8_t *live, SortedStore *s, hipStream_t st) {
    return build_sorted<OMPL_GPU_SPACE_SE3, 7>(feat32, feat64, cap, n_total, n_live, live, s, st);
}

hipError_t fast_se3_append(const FeatGeom &, const float *feat32, const double *feat64, uint64_t cap, uint64_t n_total,
                           const FastBounds &b, SortedStore *s, hipStream_t st, bool *fits) {
    return append_sorted<OMPL_GPU_SPACE_SE3, 7>(feat32, feat64, cap, n_total, b, s, st, fits);
}

hipError_t fast_se3_radius(const DevSpace &sp, const FeatGeom &g, const double *feat64, uint64_t cap,
                           const SortedStore *sorted, const double *qfeat64, uint32_t nq, double r, const FastBounds &b,
                           void *ws, size_t ws_bytes, int phase, uint64_t **d_offsets, uint32_t *out_i, double *out_d,
                           hipStream_t st) {
    return fast_radius_entry<OMPL_GPU_SPACE_SE3, 7>(sp, g, feat64, cap, sorted, qfeat64, nq, r, b, ws, ws_bytes, phase,
                                                    d_offsets, out_i, out_d, st);
}

}  // namespace ompl_amd
