// rrt.hip — sequential RRT growth on device (RRT.cpp:128-192, without the goal test).
//
// RRT's iterations are strictly dependent: sample i's nearest neighbour is searched among
// every state the samples before it added.  On the host each iteration is a query, a copy
// back and a decision; here all iterations are queued on one stream with no host round
// trip, because the store's live size lives in device memory:
//   rrt_scan_kernel   streaming scan for the sample's nearest stored state (RRT.cpp:137);
//                     the grid covers the largest size the store can have reached by this
//                     iteration, waves past the current size exit at once;
//   rrt_step_kernel   one block: merge the per-block minima, steer to max_distance
//                     (RRT.cpp:141-146), check the motion with the whole block — the bit of
//                     DiscreteMotionValidator::checkMotion (DiscreteMotionValidator.cpp:93-145)
//                     is the AND over s2 and the samples j/nd, whatever order they are tested
//                     in — and append the steered state (RRT.cpp:170-173).
// Spaces whose stored features are their coordinates (R^n, SO3, SE3): an appended state's
// features are then its reals, exactly as ompl_gpu_nn_add would store them.
#include <hip/hip_runtime.h>

#include "feat_dist.h"
#include "kernels.h"
#include "topk.h"

namespace ompl_amd {

namespace {

constexpr int kRrtItems = 4;                      // states per lane of the scan
constexpr int kRrtBlockStates = 256 * kRrtItems;  // states per scan block

template <int SP, int F>
__global__ __launch_bounds__(256) void rrt_scan_kernel(const double *__restrict__ feat, uint64_t cap,
                                                       const uint64_t *__restrict__ n_dev,
                                                       const double *__restrict__ sample, DevSpace sp,
                                                       double *__restrict__ part_d, uint32_t *__restrict__ part_i) {
    __shared__ double lds_d[4];
    __shared__ uint32_t lds_i[4];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t n = *n_dev;
    double qf[F];
#pragma unroll
    for (int f = 0; f < F; ++f) qf[f] = f < sp.dim ? sample[f] : 0.0;
    TopK<1> top;
    top.init();
    const uint64_t wbase = ((uint64_t)blockIdx.x * 4 + wave) * (64 * kRrtItems);
    if (wbase < n) {
        double sf[kRrtItems][F];
#pragma unroll
        for (int it = 0; it < kRrtItems; ++it) {
            const uint64_t id = wbase + (uint64_t)it * 64 + lane;
#pragma unroll
            for (int f = 0; f < F; ++f) sf[it][f] = id < n ? feat[(uint64_t)f * cap + id] : __builtin_nan("");
        }
#pragma unroll
        for (int it = 0; it < kRrtItems; ++it)
            top.offer(feat_dist<SP, F, 0>(sf[it], qf, sp), (uint32_t)(wbase + (uint64_t)it * 64 + lane));
    }
    double rd;
    uint32_t ri;
    block_select<1>(top, lds_d, lds_i, rd, ri);
    if (threadIdx.x == 0) {
        part_d[blockIdx.x] = rd;
        part_i[blockIdx.x] = ri;
    }
}

template <int F>
__global__ __launch_bounds__(256) void rrt_step_kernel(double *__restrict__ feat, float *__restrict__ feat32,
                                                       int rows32, uint64_t cap, uint64_t *__restrict__ n_dev,
                                                       const double *__restrict__ sample,
                                                       const double *__restrict__ part_d,
                                                       const uint32_t *__restrict__ part_i, uint32_t nparts,
                                                       DevSpace sp, DevSpace msp, DevChecker ck, double maxd,
                                                       uint32_t *__restrict__ nearest_out,
                                                       uint32_t *__restrict__ added_out,
                                                       unsigned long long *__restrict__ counters) {
    __shared__ double lds_d[4];
    __shared__ uint32_t lds_i[4];
    __shared__ double s1[kChainMaxLinks], s2[kChainMaxLinks];
    __shared__ int sh_nd, sh_bad, sh_ok;
    TopK<1> top;
    top.init();
    for (uint32_t j = threadIdx.x; j < nparts; j += blockDim.x) top.offer(part_d[j], part_i[j]);
    double rd;
    uint32_t ri;
    block_select<1>(top, lds_d, lds_i, rd, ri);
    const int dim = sp.dim;
    if (threadIdx.x == 0) {
        sh_ok = ri != kNoId;
        sh_bad = 0;
        sh_nd = 0;
        *nearest_out = ri;
        if (sh_ok) {
            double a[kChainMaxLinks], b[kChainMaxLinks], o[kChainMaxLinks];
            for (int c = 0; c < dim; ++c) {
                a[c] = feat[(uint64_t)c * cap + ri];
                b[c] = sample[c];
            }
            const double d = raw_distance(sp, a, b);  // si_->distance(nmotion->state, rstate)  RRT.cpp:141
            if (d > maxd) {
                interpolate(sp, a, b, maxd / d, o);   // RRT.cpp:142-145
            } else {
                for (int c = 0; c < dim; ++c) o[c] = b[c];
            }
            for (int c = 0; c < dim; ++c) {
                s1[c] = a[c];
                s2[c] = o[c];
            }
            sh_nd = (int)valid_segment_count(msp, a, o);
        }
    }
    __syncthreads();
    if (sh_ok) {
        // sample 0 stands for s2 (DiscreteMotionValidator.cpp:96), samples j in [1, nd-1] for j/nd
        const int nd = sh_nd;
        const int ns = nd > 1 ? nd : 1;
        for (int j = threadIdx.x; j < ns; j += blockDim.x) {
            double t[kChainMaxLinks];
            if (j == 0) {
                for (int c = 0; c < dim; ++c) t[c] = s2[c];
            } else {
                interpolate(msp, s1, s2, (double)j / (double)nd, t);
            }
            if (!is_valid(msp, ck, t)) sh_bad = 1;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t added = kNoId;
        const uint64_t n = *n_dev;
        if (sh_ok && !sh_bad && n < cap) {
            for (int f = 0; f < F; ++f) feat[(uint64_t)f * cap + n] = f < dim ? s2[f] : 0.0;
            for (int r = 0; r < rows32; ++r) feat32[(uint64_t)r * cap + n] = (float)(r < dim ? s2[r] : 0.0);
            *n_dev = n + 1;
            added = (uint32_t)n;
        }
        *added_out = added;
        if (counters && sh_ok) atomicAdd(&counters[sh_bad ? 1 : 0], 1ull);  // valid_ / invalid_
    }
}

template <int SP, int F>
hipError_t run_rrt(const DevSpace &sp, const DevSpace &msp, const DevChecker &ck, double *feat, float *feat32,
                   int rows32, uint64_t cap, uint64_t n0, uint64_t *n_dev, const double *samples, uint32_t ns,
                   double maxd, double *part_d, uint32_t *part_i, uint32_t *nearest, uint32_t *added,
                   unsigned long long *counters, hipStream_t st) {
    const int dim = sp.dim;
    for (uint32_t i = 0; i < ns; ++i) {
        // before sample i the store holds at most n0 + i states
        const uint64_t nmax = n0 + i;
        const uint32_t blocks = (uint32_t)((nmax + kRrtBlockStates - 1) / kRrtBlockStates);
        const double *s = samples + (size_t)i * dim;
        hipLaunchKernelGGL((rrt_scan_kernel<SP, F>), dim3(blocks), dim3(256), 0, st, feat, cap, n_dev, s, sp, part_d,
                           part_i);
        hipLaunchKernelGGL((rrt_step_kernel<F>), dim3(1), dim3(256), 0, st, feat, feat32, rows32, cap, n_dev, s,
                           part_d, part_i, blocks, sp, msp, ck, maxd, nearest + i, added + i, counters);
    }
    return hipGetLastError();
}

}  // namespace

size_t rrt_part_entries(uint64_t n_max) { return (size_t)((n_max + kRrtBlockStates - 1) / kRrtBlockStates); }

hipError_t launch_rrt_grow(const DevSpace &sp, const DevSpace &msp, const DevChecker &ck, const FeatGeom &g,
                           double *feat, float *feat32, int rows32, uint64_t cap, uint64_t n0, uint64_t *n_dev,
                           const double *samples, uint32_t ns, double maxd, double *part_d, uint32_t *part_i,
                           uint32_t *nearest, uint32_t *added, unsigned long long *counters, hipStream_t st) {
    if (ns == 0) return hipSuccess;
    switch (sp.kind) {
    case OMPL_GPU_SPACE_SE3:
        return run_rrt<OMPL_GPU_SPACE_SE3, 7>(sp, msp, ck, feat, feat32, rows32, cap, n0, n_dev, samples, ns, maxd,
                                              part_d, part_i, nearest, added, counters, st);
    case OMPL_GPU_SPACE_SO3:
        return run_rrt<OMPL_GPU_SPACE_SO3, 4>(sp, msp, ck, feat, feat32, rows32, cap, n0, n_dev, samples, ns, maxd,
                                              part_d, part_i, nearest, added, counters, st);
    case OMPL_GPU_SPACE_REALVECTOR:
        if (g.F == 4)
            return run_rrt<OMPL_GPU_SPACE_REALVECTOR, 4>(sp, msp, ck, feat, feat32, rows32, cap, n0, n_dev, samples,
                                                         ns, maxd, part_d, part_i, nearest, added, counters, st);
        if (g.F == 8)
            return run_rrt<OMPL_GPU_SPACE_REALVECTOR, 8>(sp, msp, ck, feat, feat32, rows32, cap, n0, n_dev, samples,
                                                         ns, maxd, part_d, part_i, nearest, added, counters, st);
        return run_rrt<OMPL_GPU_SPACE_REALVECTOR, 16>(sp, msp, ck, feat, feat32, rows32, cap, n0, n_dev, samples, ns,
                                                      maxd, part_d, part_i, nearest, added, counters, st);
    }
    return hipErrorInvalidValue;
}

}  // namespace ompl_amd
