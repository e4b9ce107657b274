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

#include <algorithm>

#include "knn_fast_impl.h"  // state_dist32 / screen_error of the fp32 screen

namespace ompl_amd {

namespace {

constexpr int kRrtItems = 4;                      // states per lane of the scan
constexpr int kRrtBlockStates = 256 * kRrtItems;  // states per scan block

template <int SP, int F>
__global__ __launch_bounds__(256) void rrt_scan_kernel(const double *__restrict__ feat, uint64_t cap,
                                                       const uint64_t *__restrict__ n_dev,
                                                       const double *__restrict__ sample, DevSpace sp,
                                                       double *__restrict__ part_d, uint32_t *__restrict__ part_i,
                                                       const uint64_t *__restrict__ done) {
    __shared__ double lds_d[4];
    __shared__ uint32_t lds_i[4];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t n = *n_dev;
    if (done && *done != ~0ull) return;  // solved earlier in the run: nothing left to do
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

// sample's nearest stored state ri (kNoId: none): steer to max_distance (RRT.cpp:141-146) and
// check the motion with the whole block — the bit of DiscreteMotionValidator::checkMotion
// (DiscreteMotionValidator.cpp:93-145) is the AND over s2 and the samples j / nd, whatever order
// they are tested in.  Leaves s1 / s2 (the motion), *sh_ok (a neighbour exists) and *sh_bad (some
// sample invalid) in LDS for every thread.
template <class RowOf>
__device__ void rrt_decide(RowOf row_of, const double *__restrict__ sample, uint32_t ri, const DevSpace &sp,
                           const DevSpace &msp, const DevChecker &ck, double maxd, double *s1, double *s2, int *sh_nd,
                           int *sh_bad, int *sh_ok) {
    const int dim = sp.dim;
    if (threadIdx.x == 0) {
        *sh_ok = ri != kNoId;
        *sh_bad = 0;
        *sh_nd = 0;
        if (ri != kNoId) {
            double a[kChainMaxLinks], b[kChainMaxLinks], o[kChainMaxLinks];
            for (int c = 0; c < dim; ++c) {
                a[c] = row_of(c);
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
            *sh_nd = (int)valid_segment_count(msp, a, o);
        }
    }
    __syncthreads();
    if (*sh_ok) {
        // sample 0 stands for s2 (DiscreteMotionValidator.cpp:96), samples j in [1, nd-1] for j/nd
        const int nd = *sh_nd;
        const int ns = nd > 1 ? nd : 1;
        for (int j = threadIdx.x; j < ns; j += blockDim.x) {
            double t[kChainMaxLinks];
            if (j == 0) {
                for (int c = 0; c < dim; ++c) t[c] = s2[c];
            } else {
                interpolate(msp, s1, s2, (double)j / (double)nd, t);
            }
            if (!is_valid(msp, ck, t)) *sh_bad = 1;
        }
    }
    __syncthreads();
}

// Goal test of RRT.cpp:175-187 after each added state: GoalRegion::isSatisfied (distance to the
// goal < threshold, GoalRegion.cpp:52-58) ends the run at that iteration; otherwise the state
// becomes the approximate solution when strictly closer than every earlier one.
struct RrtGoal {
    const double *goal;  // device, dim reals; nullptr: no goal test (the growth form)
    double threshold;
};
// device record of the run (rrt_goal_words 64-bit words): [0] iteration that solved
// (~0: none), [1] approximate-solution distance bits (+inf initially), [2] its id
constexpr int kGoalWords = 3;

__device__ __forceinline__ bool rrt_goal_test(const RrtGoal &gl, const DevSpace &sp, const double *x, uint32_t id,
                                              uint32_t iter, uint64_t *rec) {
    if (!gl.goal) return false;
    double g[kChainMaxLinks];
    for (int c = 0; c < sp.dim; ++c) g[c] = gl.goal[c];
    const double d = raw_distance(sp, x, g);  // goal->isSatisfied(nmotion->state, &dist)  RRT.cpp:175
    if (d < gl.threshold) {
        rec[0] = iter;
        return true;
    }
    if (d < __longlong_as_double((long long)rec[1])) {  // RRT.cpp:183-187
        rec[1] = (uint64_t)__double_as_longlong(d);
        rec[2] = id;
    }
    return false;
}

// append s2 at position n (its features are its reals: R^n, SO3, SE3) — one thread
template <int F>
__device__ __forceinline__ void rrt_append(double *__restrict__ feat, float *__restrict__ feat32, int rows32,
                                           uint64_t cap, uint64_t n, const double *s2, int dim) {
    for (int f = 0; f < F; ++f) feat[(uint64_t)f * cap + n] = f < dim ? s2[f] : 0.0;
    for (int r = 0; r < rows32; ++r) feat32[(uint64_t)r * cap + n] = (float)(r < dim ? s2[r] : 0.0);
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
                                                       unsigned long long *__restrict__ counters, RrtGoal gl,
                                                       uint64_t *__restrict__ grec, uint32_t iter) {
    if (gl.goal && grec[0] != ~0ull) return;  // solved earlier: the host marks the rest
    __shared__ double lds_d[4];
    __shared__ uint32_t lds_i[4];
    __shared__ double s1[kChainMaxLinks], s2[kChainMaxLinks];
    __shared__ int sh_nd, sh_bad, sh_ok;
    __shared__ uint32_t sh_ri;
    TopK<1> top;
    top.init();
    for (uint32_t j = threadIdx.x; j < nparts; j += blockDim.x) top.offer(part_d[j], part_i[j]);
    double rd;
    uint32_t ri;
    block_select<1>(top, lds_d, lds_i, rd, ri);
    if (threadIdx.x == 0) sh_ri = ri;
    __syncthreads();
    ri = sh_ri;
    rrt_decide([&](int c) { return feat[(uint64_t)c * cap + ri]; }, sample, ri, sp, msp, ck, maxd, s1, s2, &sh_nd,
               &sh_bad, &sh_ok);
    if (threadIdx.x == 0) {
        *nearest_out = ri;
        uint32_t added = kNoId;
        const uint64_t n = *n_dev;
        if (sh_ok && !sh_bad && n < cap) {
            rrt_append<F>(feat, feat32, rows32, cap, n, s2, sp.dim);
            *n_dev = n + 1;
            added = (uint32_t)n;
            rrt_goal_test(gl, sp, s2, added, iter, grec);
        }
        *added_out = added;
        if (counters && sh_ok) atomicAdd(&counters[sh_bad ? 1 : 0], 1ull);  // valid_ / invalid_
    }
}


// ---- persistent form: one cooperative launch for all iterations --------------------------
// One block per CU; block b owns the store positions [b * slice, (b + 1) * slice) for the whole
// run, so its slice of the fp32 rows (28 B per SE3 state; 10^6 states = 3.5 MB per XCD) stays in
// its XCD's L2 from one iteration to the next.  Iteration i:
//   1. every block screens its slice in fp32 for sample i (per thread the two smallest d32),
//      refines the candidates within the screen's error bound of the block's fp32 minimum in
//      fp64 (the reference's operation order) and so finds the slice's exact nearest (d, id):
//      a state with d32 > thr = (m + E)(1 + 32u) has d64 > m + E/2 >= d64 of the block's fp32
//      argmin (the knn_stream32.hip argument with K = 1); a thread whose second smallest d32 is
//      within thr rescans its own positions;
//   2. it publishes (d, id, fp64 row) in its own record and raises its own arrival flag (no
//      shared counter: a same-address atomic per block per iteration serialises in memory);
//   3. block 0 — the decider — polls the nb flags with nb threads, merges the records, steers,
//      checks the motion with the whole block (rrt_decide), runs the goal test, and publishes the
//      decision and the next generation; the other blocks poll the generation word;
//   4. the block owning the new position appends the row (fp64 + fp32): it is the only block that
//      reads that position later, so the store needs no cross-XCD coherence.
// All cross-block words live in an UNCACHED device buffer (hipDeviceMallocUncached): every access
// goes to memory, so blocks on different XCDs (each with its own L2) see each other's writes
// without L2 write-back / invalidate.  A writer waits for its stores to complete (s_waitcnt) before
// the word that announces them; a reader issues its loads after the announcing load returned.  A
// waiting block gives up after kSpinLimit polls and raises the abort word, which every waiter polls
// too, so a grid that cannot make progress drains instead of hanging (the host reports it).
// The screen's error bound needs B >= every |coordinate| and (SE3) eta >= every |q|^2 - 1 of the
// store and the query: the host passes them for the initial store, the decider extends them with
// each appended state, every block with each sample.
constexpr uint32_t kSpinLimit = 1u << 22;  // ~0.1 s of s_sleep(1) polls per wait
constexpr uint32_t kRrtMaxCoopBlocks = 256;  // <= blockDim: the decider polls one flag per thread

// the uncached synchronisation record (rrt_sync_bytes): 64-bit words
//   [1] generation  [2] abort  [3] size  [4] neighbour  [5] added  [6] solved  [7] B  [28] eta
//   [8 .. 8+16)  the new state      [24 .. 27) the goal record (RrtGoal), read and written by the
//   decider        [32 ..) per block: arrival flag (nb), distance (nb), id (nb), row (nb x 16)
constexpr int kSyncState = 8, kSyncGoal = 24, kSyncB = 7, kSyncEta = 28, kSyncParts = 32, kSyncRow = 16;

__device__ __forceinline__ void stores_done() { __builtin_amdgcn_s_waitcnt(0); }  // vmcnt = expcnt = lgkmcnt = 0
__device__ __forceinline__ uint64_t ld_sync(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sync(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t dbits(double v) { return (uint64_t)__double_as_longlong(v); }
__device__ __forceinline__ double bitsd(uint64_t v) { return __longlong_as_double((long long)v); }

// block-wide argmin of (d, i) by (distance, id); every thread returns the result
__device__ __forceinline__ void block_argmin(double &d, uint32_t &i, double *lds_d, uint32_t *lds_i) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    wave_argmin(d, i);
    if (lane == 0) {
        lds_d[wave] = d;
        lds_i[wave] = i;
    }
    __syncthreads();
#pragma unroll
    for (int w = 0; w < 4; ++w)
        if (lex_less(lds_d[w], lds_i[w], d, i)) {
            d = lds_d[w];
            i = lds_i[w];
        }
    __syncthreads();
}

__device__ __forceinline__ float block_minf(float v, float *lds) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = fminf(v, __shfl_xor(v, off, 64));
    if (lane == 0) lds[wave] = v;
    __syncthreads();
    v = fminf(fminf(lds[0], lds[1]), fminf(lds[2], lds[3]));
    __syncthreads();
    return v;
}

// max |coordinate| (the screen's B: SE3 translation, R^n every coordinate) and SE3 |q|^2 - 1
template <int SP, int F>
__device__ __forceinline__ double coord_absmax(const double *x) {
    const int nc = SP == OMPL_GPU_SPACE_SE3 ? 3 : F;
    double m = 0.0;
    for (int c = 0; c < nc; ++c) m = fmax(m, fabs(x[c]));
    return m;
}

template <int SP, int F>
__global__ __launch_bounds__(256) void rrt_persistent_kernel(
    double *__restrict__ feat, float *__restrict__ feat32, int rows32, uint64_t cap, uint64_t n0,
    uint64_t *__restrict__ n_dev, const double *__restrict__ samples, uint32_t ns, uint64_t slice, DevSpace sp,
    DevSpace msp, DevChecker ck, double maxd, uint64_t *__restrict__ sync, uint32_t *__restrict__ nearest_out,
    uint32_t *__restrict__ added_out, unsigned long long *__restrict__ counters, RrtGoal gl,
    uint64_t *__restrict__ grec) {
    constexpr int FS = Geo<SP, F>::FS;
    __shared__ double lds_d[4];
    __shared__ uint32_t lds_i[4];
    __shared__ float lds_f[4];
    __shared__ double s1[kChainMaxLinks], s2[kChainMaxLinks];
    __shared__ int sh_nd, sh_bad, sh_ok, sh_run, sh_stop;
    __shared__ uint64_t sh_n, sh_added;
    __shared__ double sh_row[F], sh_B, sh_eta;
    const uint32_t nb = gridDim.x, b = blockIdx.x;
    const int dim = sp.dim;
    const uint64_t lo = (uint64_t)b * slice, hi = lo + slice;
    uint64_t *flag = sync + kSyncParts, *pd = flag + nb, *pi = pd + nb, *prow = pi + nb;
    uint64_t n = n0;
    double Bst = bitsd(ld_sync(&sync[kSyncB])), eta_st = bitsd(ld_sync(&sync[kSyncEta]));
    const float w0 = (float)sp.w0, w1 = (float)sp.w1;
    for (uint32_t i = 0; i < ns; ++i) {
        const double *s = samples + (size_t)i * dim;
        double qv[F];
#pragma unroll
        for (int f = 0; f < F; ++f) qv[f] = f < dim ? s[f] : 0.0;
        float q32[FS];
        if constexpr (SP == OMPL_GPU_SPACE_SE3) {
#pragma unroll
            for (int c = 0; c < 3; ++c) q32[c] = (float)qv[c];
            q32[3] = 0.f;
#pragma unroll
            for (int c = 0; c < 4; ++c) q32[4 + c] = (float)qv[3 + c];
        } else {
#pragma unroll
            for (int f = 0; f < F; ++f) q32[f] = (float)qv[f];
        }
        // 1. this block's slice (RRT.cpp:137): fp32 screen, two smallest per thread
        const uint64_t end = hi < n ? hi : n;
        float c0 = __builtin_inff(), c1 = __builtin_inff();
        uint32_t i0 = kNoId;
        const float nanf_ = __builtin_nanf("");
#pragma unroll 2
        for (uint64_t p = lo + 4 * threadIdx.x; p < end; p += 1024) {
            float4 x[F];
#pragma unroll
            for (int f = 0; f < F; ++f) x[f] = *reinterpret_cast<const float4 *>(feat32 + (uint64_t)f * cap + p);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                float v[F];
#pragma unroll
                for (int f = 0; f < F; ++f) v[f] = u == 0 ? x[f].x : u == 1 ? x[f].y : u == 2 ? x[f].z : x[f].w;
                float d = state_dist32<SP, F>(v, q32, w0, w1);
                if (p + u >= end) d = nanf_;
                if (d < c1) {  // NaN never passes; positions ascend, so ties keep the smaller id first
                    if (d < c0) {
                        c1 = c0;
                        c0 = d;
                        i0 = (uint32_t)(p + u);
                    } else {
                        c1 = d;
                    }
                }
            }
        }
        const float m = block_minf(c0, lds_f);
        double bd = __builtin_inf();
        uint32_t bi = kNoId;
        double brow[F];
        if (m == m && m < __builtin_inff()) {
            const double B = fmax(Bst, coord_absmax<SP, F>(qv));
            const double E = screen_error<SP>(sp, B, (double)m, eta_st + query_eta<SP>(qv));
            const double thr = ((double)m + E) * (1.0 + 32.0 * kU);
            auto refine = [&](uint32_t id) {
                double sv[F];
#pragma unroll
                for (int f = 0; f < F; ++f) sv[f] = feat[(uint64_t)f * cap + id];
                const double d = feat_dist<SP, F, 0>(sv, qv, sp);
                if (lex_less(d, id, bd, bi)) {
                    bd = d;
                    bi = id;
#pragma unroll
                    for (int f = 0; f < F; ++f) brow[f] = sv[f];
                }
            };
            if ((double)c1 <= thr) {  // maybe more than two of this thread's states qualify: rescan them
                for (uint64_t p = lo + 4 * threadIdx.x; p < end; p += 1024)
                    for (int u = 0; u < 4 && p + u < end; ++u) {
                        float v[F];
#pragma unroll
                        for (int f = 0; f < F; ++f) v[f] = feat32[(uint64_t)f * cap + p + u];
                        if ((double)state_dist32<SP, F>(v, q32, w0, w1) <= thr) refine((uint32_t)(p + u));
                    }
            } else if ((double)c0 <= thr) {
                refine(i0);
            }
        }
        double wd = bd;
        uint32_t wi = bi;
        block_argmin(wd, wi, lds_d, lds_i);
        if (wi != kNoId && bi == wi) {  // the winning thread (ids are unique)
#pragma unroll
            for (int f = 0; f < F; ++f) sh_row[f] = brow[f];
        }
        __syncthreads();
        // 2. publish: record, then the arrival flag
        if (threadIdx.x == 0) {
            st_sync(&pd[b], dbits(wd));
            st_sync(&pi[b], wi);
            if (wi != kNoId)
                for (int f = 0; f < F; ++f) st_sync(&prow[(size_t)b * kSyncRow + f], dbits(sh_row[f]));
            stores_done();
            st_sync(&flag[b], (uint64_t)i + 1);
        }
        if (b == 0) {
            // 3. the decider: wait for every block's flag, merge, decide
            int ok = 1;
            if (threadIdx.x < nb) {
                uint32_t spins = 0;
                while (ld_sync(&flag[threadIdx.x]) <= (uint64_t)i) {
                    __builtin_amdgcn_s_sleep(1);
                    if (++spins > kSpinLimit || ld_sync(&sync[2])) {
                        ok = 0;
                        break;
                    }
                }
            }
            if (!__syncthreads_and(ok)) {
                if (threadIdx.x == 0) st_sync(&sync[2], 1);
                return;  // aborted: the host sees the abort word and fails the call
            }
            double gd = __builtin_inf();
            uint32_t gi = kNoId;
            if (threadIdx.x < nb) {
                gd = bitsd(ld_sync(&pd[threadIdx.x]));
                gi = (uint32_t)ld_sync(&pi[threadIdx.x]);
            }
            block_argmin(gd, gi, lds_d, lds_i);
            const uint32_t ri = gi;
            const uint64_t *wrow = prow + (size_t)(ri != kNoId ? ri / slice : 0) * kSyncRow;  // the winner's block
            rrt_decide([&](int c) { return bitsd(ld_sync(&wrow[c])); }, s, ri, sp, msp, ck, maxd, s1, s2, &sh_nd,
                       &sh_bad, &sh_ok);
            if (threadIdx.x == 0) {
                uint32_t added = kNoId;
                bool solved = false;
                if (sh_ok && !sh_bad && n < cap) {
                    added = (uint32_t)n;
                    double x[F];
                    for (int f = 0; f < F; ++f) x[f] = f < dim ? s2[f] : 0.0;
                    for (int f = 0; f < F; ++f) st_sync(&sync[kSyncState + f], dbits(x[f]));
                    Bst = fmax(Bst, coord_absmax<SP, F>(x));
                    eta_st = fmax(eta_st, query_eta<SP>(x));
                    st_sync(&sync[kSyncB], dbits(Bst));
                    st_sync(&sync[kSyncEta], dbits(eta_st));
                    solved = rrt_goal_test(gl, sp, x, added, i, sync + kSyncGoal);
                }
                st_sync(&sync[6], solved);
                nearest_out[i] = ri;
                added_out[i] = added;
                if (counters && sh_ok) atomicAdd(&counters[sh_bad ? 1 : 0], 1ull);  // valid_ / invalid_
                st_sync(&sync[3], added != kNoId ? n + 1 : n);
                st_sync(&sync[5], added);
                stores_done();
                st_sync(&sync[1], (uint64_t)i + 1);  // release the others
            }
            __syncthreads();
        } else if (threadIdx.x == 0) {
            bool ok = true;
            uint32_t spins = 0;
            while (ld_sync(&sync[1]) <= (uint64_t)i) {
                __builtin_amdgcn_s_sleep(1);
                if (++spins > kSpinLimit || ld_sync(&sync[2])) {
                    ok = false;
                    break;
                }
            }
            if (!ok) st_sync(&sync[2], 1);
            sh_run = ok;
        }
        if (b != 0) {
            __syncthreads();
            if (!sh_run) return;  // aborted: the host sees the abort word and fails the call
        }
        // 4. the decision, and the append by the block that owns the new position
        if (threadIdx.x == 0) {
            sh_n = ld_sync(&sync[3]);
            sh_added = ld_sync(&sync[5]);
            sh_stop = (int)ld_sync(&sync[6]);  // solved: every block stops after this iteration
            sh_B = bitsd(ld_sync(&sync[kSyncB]));
            sh_eta = bitsd(ld_sync(&sync[kSyncEta]));
        }
        __syncthreads();
        const uint64_t added = sh_added;
        Bst = sh_B;
        eta_st = sh_eta;
        if (added != kNoId && added >= lo && added < hi) {
            if (threadIdx.x < F) sh_row[threadIdx.x] = bitsd(ld_sync(&sync[kSyncState + threadIdx.x]));
            __syncthreads();
            if (threadIdx.x == 0) rrt_append<F>(feat, feat32, rows32, cap, added, sh_row, dim);
            // this CU's L1 may hold the line of the new row as loaded before the append: drop it
            // before the next scan reads the row (one block per iteration pays the invalidate)
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "agent");
        }
        n = sh_n;
        const bool stop = sh_stop != 0;
        __syncthreads();  // shared words are rewritten in the next iteration
        if (stop) break;
    }
    if (b == 0 && threadIdx.x == 0) {
        *n_dev = n;
        for (int w = 0; w < kGoalWords; ++w) grec[w] = ld_sync(&sync[kSyncGoal + w]);
    }
}

template <int SP, int F>
hipError_t run_rrt(const DevSpace &sp, const DevSpace &msp, const DevChecker &ck, double *feat, float *feat32,
                   int rows32, uint64_t cap, uint64_t n0, uint64_t *n_dev, const double *samples, uint32_t ns,
                   double maxd, double *part_d, uint32_t *part_i, uint32_t *nearest, uint32_t *added,
                   unsigned long long *counters, uint64_t *sync, uint32_t coop_blocks, RrtGoal gl, uint64_t *grec,
                   hipStream_t st) {
    const int dim = sp.dim;
    if constexpr (SP == OMPL_GPU_SPACE_SE3 || SP == OMPL_GPU_SPACE_REALVECTOR) {
        if (coop_blocks > 0 && sync) {
            // slices of whole block-steps (1,024 positions), covering the largest size of the run
            const uint64_t nmax = n0 + ns;
            uint64_t slice = (nmax + coop_blocks - 1) / coop_blocks;
            slice = (slice + 1023) & ~(uint64_t)1023;
            const uint32_t nb = (uint32_t)((nmax + slice - 1) / slice);
            void *args[] = {&feat, &feat32, &rows32, &cap, &n0, &n_dev, &samples, &ns, &slice, (void *)&sp,
                            (void *)&msp, (void *)&ck, &maxd, &sync, &nearest, &added, &counters, &gl, &grec};
            return hipLaunchCooperativeKernel((const void *)rrt_persistent_kernel<SP, F>, dim3(nb), dim3(256), args,
                                              0, st);
        }
    }
    for (uint32_t i = 0; i < ns; ++i) {
        // before sample i the store holds at most n0 + i states
        const uint64_t nmax = n0 + i;
        const uint32_t blocks = (uint32_t)((nmax + kRrtBlockStates - 1) / kRrtBlockStates);
        const double *s = samples + (size_t)i * dim;
        hipLaunchKernelGGL((rrt_scan_kernel<SP, F>), dim3(blocks), dim3(256), 0, st, feat, cap, n_dev, s, sp, part_d,
                           part_i, gl.goal ? grec : nullptr);
        hipLaunchKernelGGL((rrt_step_kernel<F>), dim3(1), dim3(256), 0, st, feat, feat32, rows32, cap, n_dev, s,
                           part_d, part_i, blocks, sp, msp, ck, maxd, nearest + i, added + i, counters, gl, grec, i);
    }
    return hipGetLastError();
}

}  // namespace

uint32_t rrt_coop_blocks(int device, const DevSpace &sp, const FeatGeom &g) {
#if defined(OMPL_AMD_VARIANT) && OMPL_AMD_VARIANT == 3
    return 0;  // A/B build: the two-launch form
#endif
    int coop = 0, cus = 0;
    if (hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, device) != hipSuccess || !coop) return 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0) return 0;
    const void *fn = nullptr;
    switch (sp.kind) {
    case OMPL_GPU_SPACE_SE3: fn = (const void *)rrt_persistent_kernel<OMPL_GPU_SPACE_SE3, 7>; break;
    case OMPL_GPU_SPACE_REALVECTOR:
        fn = g.F == 4 ? (const void *)rrt_persistent_kernel<OMPL_GPU_SPACE_REALVECTOR, 4>
             : g.F == 8 ? (const void *)rrt_persistent_kernel<OMPL_GPU_SPACE_REALVECTOR, 8>
                        : (const void *)rrt_persistent_kernel<OMPL_GPU_SPACE_REALVECTOR, 16>;
        break;
    default: return 0;
    }
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 256, 0) != hipSuccess || per_cu <= 0) return 0;
    return (uint32_t)std::min<int64_t>(cus, kRrtMaxCoopBlocks);  // one block per CU
}

size_t rrt_part_entries(uint64_t n_max) { return (size_t)((n_max + kRrtBlockStates - 1) / kRrtBlockStates); }

size_t rrt_goal_words() { return kGoalWords; }

size_t rrt_sync_bytes() { return sizeof(uint64_t) * (kSyncParts + (3 + kSyncRow) * kRrtMaxCoopBlocks); }

hipError_t launch_rrt_grow(const DevSpace &sp, const DevSpace &msp, const DevChecker &ck, const FeatGeom &g,
                           double *feat, float *feat32, int rows32, uint64_t cap, uint64_t n0, uint64_t *n_dev,
                           const double *samples, uint32_t ns, double maxd, double *part_d, uint32_t *part_i,
                           uint32_t *nearest, uint32_t *added, unsigned long long *counters, uint64_t *sync,
                           uint32_t coop_blocks, const double *goal, double goal_threshold, uint64_t *grec,
                           hipStream_t st) {
    const RrtGoal gl{goal, goal_threshold};
    if (ns == 0) return hipSuccess;
    coop_blocks = std::min<uint32_t>(coop_blocks, kRrtMaxCoopBlocks);
#define OMPL_AMD_RRT(SPK, FK)                                                                                      \
    return run_rrt<SPK, FK>(sp, msp, ck, feat, feat32, rows32, cap, n0, n_dev, samples, ns, maxd, part_d, part_i, \
                            nearest, added, counters, sync, coop_blocks, gl, grec, st)
    switch (sp.kind) {
    case OMPL_GPU_SPACE_SE3:
        OMPL_AMD_RRT(OMPL_GPU_SPACE_SE3, 7);
    case OMPL_GPU_SPACE_SO3:
        OMPL_AMD_RRT(OMPL_GPU_SPACE_SO3, 4);
    case OMPL_GPU_SPACE_REALVECTOR:
        if (g.F == 4) OMPL_AMD_RRT(OMPL_GPU_SPACE_REALVECTOR, 4);
        if (g.F == 8) OMPL_AMD_RRT(OMPL_GPU_SPACE_REALVECTOR, 8);
        OMPL_AMD_RRT(OMPL_GPU_SPACE_REALVECTOR, 16);
    }
#undef OMPL_AMD_RRT
    return hipErrorInvalidValue;
}

}  // namespace ompl_amd
