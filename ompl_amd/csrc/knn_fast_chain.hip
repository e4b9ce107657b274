// knn_fast_chain.hip — KinematicChain instantiations (4 / 8 / 12 / 16 link buckets) of the fp32
// screen + fp64 certificate (knn_fast_impl.h): the screen scans joint positions, the
// certificate recomputes the reference's chain distance (demos/KinematicChain.h:105-124) from
// the cumulative cos / sin features.  No sorted store: the chunked brute-force screen serves it.
#include "knn_fast_impl.h"

namespace ompl_amd {

hipError_t fast_chain(const DevSpace &sp, const FeatGeom &g, const double *feat64, const float *feat32, uint64_t cap,
                      uint64_t n_end, const SortedStore *sorted, const double *qfeat64, uint32_t nq, uint32_t k,
                      const FastBounds &b, double *out_d, uint32_t *out_i, void *ws, size_t ws_bytes, int num_cus,
                      hipStream_t st, uint32_t **fail_count, uint32_t **fail_list) {
#define OMPL_AMD_CHAIN(FF)                                                                                      \
    return fast_entry<OMPL_GPU_SPACE_KCHAIN, FF>(sp, g, feat64, feat32, cap, n_end, sorted, qfeat64, nq, k, b,  \
                                                 out_d, out_i, ws, ws_bytes, num_cus, st, fail_count, fail_list)
    if (g.F == 8) OMPL_AMD_CHAIN(8);
    if (g.F == 16) OMPL_AMD_CHAIN(16);
    if (g.F == 24) OMPL_AMD_CHAIN(24);
    OMPL_AMD_CHAIN(32);
#undef OMPL_AMD_CHAIN
}

// k-d sorted store of the joint positions (the culled chain scan, knn32_chain_cull_kernel)
hipError_t fast_chain_build(const FeatGeom &g, const float *feat32, const double *feat64, uint64_t cap,
                            uint64_t n_total, uint32_t n_live, const uint8_t *live, SortedStore *s, hipStream_t st) {
#define OMPL_AMD_CHAIN_B(FF) \
    return build_sorted<OMPL_GPU_SPACE_KCHAIN, FF>(feat32, feat64, cap, n_total, n_live, live, s, st)
    if (g.F == 8) OMPL_AMD_CHAIN_B(8);
    if (g.F == 16) OMPL_AMD_CHAIN_B(16);
    if (g.F == 24) OMPL_AMD_CHAIN_B(24);
    OMPL_AMD_CHAIN_B(32);
#undef OMPL_AMD_CHAIN_B
}

hipError_t fast_chain_append(const FeatGeom &g, const float *feat32, const double *feat64, uint64_t cap,
                             uint64_t n_total, const FastBounds &b, SortedStore *s, hipStream_t st, bool *fits) {
#define OMPL_AMD_CHAIN_A(FF) \
    return append_sorted<OMPL_GPU_SPACE_KCHAIN, FF>(feat32, feat64, cap, n_total, b, s, st, fits)
    if (g.F == 8) OMPL_AMD_CHAIN_A(8);
    if (g.F == 16) OMPL_AMD_CHAIN_A(16);
    if (g.F == 24) OMPL_AMD_CHAIN_A(24);
    OMPL_AMD_CHAIN_A(32);
#undef OMPL_AMD_CHAIN_A
}

hipError_t fast_chain_radius(const DevSpace &, const FeatGeom &, const double *, uint64_t, const SortedStore *,
                             const double *, uint32_t, double, const FastBounds &, void *, size_t, int, uint64_t **,
                             uint32_t *, double *, hipStream_t) {
    return hipErrorInvalidValue;  // no sorted store for the chain metric: nearestR runs the exact scan
}

namespace {
__global__ void chain_rows32_kernel(const double *__restrict__ feat, uint64_t cap, int nmax, uint64_t first,
                                    uint64_t n, float *__restrict__ f32) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const uint64_t i = first + t;
    double cx = 0.0, cy = 0.0;
    for (int j = 0; j < nmax; ++j) {
        cx += feat[(uint64_t)j * cap + i];
        cy += feat[(uint64_t)(nmax + j) * cap + i];
        f32[(uint64_t)j * cap + i] = (float)cx;
        f32[(uint64_t)(nmax + j) * cap + i] = (float)cy;
    }
}
}  // namespace

hipError_t launch_chain_rows32(const double *feat64, uint64_t cap, int nmax, uint64_t first, uint64_t n, float *feat32,
                               hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(chain_rows32_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, feat64, cap, nmax,
                       first, n, feat32);
    return hipGetLastError();
}

}  // namespace ompl_amd
