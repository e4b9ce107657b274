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
// fixed width of the persistent kernel's decider: SE3 states are 7 reals (the checkers allowed
// with SE3 — mv_create — all have fixed forms); other spaces keep the runtime width
template <int SP>
constexpr int kRrtWidth = SP == OMPL_GPU_SPACE_SE3 ? 7 : 0;

// SP / W: fixed-width form (device_space.h fixed_space; W = 0: runtime width)
template <int SP, int W, class RowOf>
__device__ void rrt_decide(RowOf row_of, const double *__restrict__ sample, uint32_t ri, const DevSpace &sp_in,
                           const DevSpace &msp_in, const DevChecker &ck, double maxd, double *s1, double *s2, int *sh_nd,
                           int *sh_bad, int *sh_ok) {
    const DevSpace sp = fixed_space<SP, W>(sp_in), msp = fixed_space<SP, W>(msp_in);
    const int dim = sp.dim;
    if (threadIdx.x == 0) {
        *sh_ok = ri != kNoId;
        *sh_bad = 0;
        *sh_nd = 0;
        if (ri != kNoId) {
            double a[Width<W>::N], b[Width<W>::N], o[Width<W>::N];
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
            double t[Width<W>::N];
            if (j == 0) {
                for (int c = 0; c < dim; ++c) t[c] = s2[c];
            } else if constexpr (W > 0) {
                double u[W], v[W];  // the motion's ends from LDS into registers
                for (int c = 0; c < W; ++c) {
                    u[c] = s1[c];
                    v[c] = s2[c];
                }
                interpolate(msp, u, v, (double)j / (double)nd, t);
            } else {
                interpolate(msp, s1, s2, (double)j / (double)nd, t);
            }
            if (!valid_t<W>(msp, ck, t)) *sh_bad = 1;
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

template <int SP, int W>
__device__ __forceinline__ bool rrt_goal_test(const RrtGoal &gl, const DevSpace &sp_in, const double *x, uint32_t id,
                                              uint32_t iter, uint64_t *rec) {
    if (!gl.goal) return false;
    const DevSpace sp = fixed_space<SP, W>(sp_in);
    double g[Width<W>::N];
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
    rrt_decide<0, 0>([&](int c) { return feat[(uint64_t)c * cap + ri]; }, sample, ri, sp, msp, ck, maxd, s1, s2, &sh_nd,
               &sh_bad, &sh_ok);
    if (threadIdx.x == 0) {
        *nearest_out = ri;
        uint32_t added = kNoId;
        const uint64_t n = *n_dev;
        if (sh_ok && !sh_bad && n < cap) {
            rrt_append<F>(feat, feat32, rows32, cap, n, s2, sp.dim);
            *n_dev = n + 1;
            added = (uint32_t)n;
            rrt_goal_test<0, 0>(gl, sp, s2, added, iter, grec);
        }
        *added_out = added;
        if (counters && sh_ok) atomicAdd(&counters[sh_bad ? 1 : 0], 1ull);  // valid_ / invalid_
    }
}


// ---- persistent form: one cooperative launch for all iterations --------------------------
// Scanning blocks (one per CU) each own the store positions [b * slice, (b + 1) * slice) for the
// whole run, so their slice of the fp32 rows (28 B per SE3 state; 10^6 states = 3.5 MB per XCD)
// stays in their XCD's L2.  One more block, the decider, owns no slice.
//
// Scanning runs AHEAD of the decisions by L samples: a block answers sample s over the positions
// below n_{s-L} (the store size before decision s - L; n0 for s < L), which needs only the decisions
// up to s - L - 1, and publishes the slice's exact nearest (d, id, fp64 row) in its record ring; the
// decider answers sample j from the records of all slices plus the states that decisions
// j - L .. j - 1 appended (positions [n_{j-L}, n_j), at most L, kept in its LDS), steers, checks the
// motion, runs the goal test and publishes decision j.  The scan is off the critical path: an
// iteration costs the decider's own round trips (flags, records, decision) and its arithmetic.
//
// A slice's exact nearest: the fp32 screen keeps each thread's two smallest d32; candidates within
// the screen's error bound of the block's fp32 minimum m are refined in fp64 (reference operation
// order): a state with d32 > thr = (m + E)(1 + 32u) has d64 > m + E/2 >= d64 of the block's fp32
// argmin (knn_stream32.hip's argument with K = 1); a thread whose second smallest d32 is within thr
// rescans its own positions.  E needs B >= every |coordinate| and (SE3) eta >= every |q|^2 - 1 of
// the store and the query: the host passes them for the initial store, each decision extends them.
//
// The block owning an appended position writes its row (fp64 + fp32) when it processes that
// decision, before it next scans: it is the only block that reads that position, so the store needs
// no cross-XCD coherence.  All cross-block words live in an UNCACHED buffer (hipDeviceMallocUncached):
// every access goes to memory, so blocks on different XCDs see each other's writes without L2
// write-back / invalidate.  A writer waits for its stores (s_waitcnt) before the word announcing them;
// a reader loads after the announcing load returned.  Rings of depth R = L + 2 (records, decisions):
// slot s mod R is rewritten only after every reader is done with it (a block publishes record s + R
// after decision s + R - L - 1 > s, which the decider made after reading record s; the decider makes
// decision j + R after record j + R of every block, which each block wrote after reading decision j).
// The decision's generation word is written in 8 copies 512 B apart, block b polling copy b % 8, so
// the pollers spread over memory channels.  A waiting block gives up after kSpinLimit polls and
// raises the abort word, which every waiter polls too: a grid that cannot progress drains (the host
// reports it).
constexpr uint32_t kSpinLimit = 1u << 22;    // ~0.1 s of s_sleep(1) polls per wait
constexpr uint32_t kRrtMaxCoopBlocks = 256;  // scanning blocks + the decider; the decider polls one flag per thread
constexpr int kLook = 2;                     // samples the scans run ahead of the decisions
constexpr int kRing = kLook + 2;             // record / decision ring depth

// the uncached synchronisation record (rrt_sync_bytes), 64-bit words:
//   [2] abort  [4] spin limit override (0: kSpinLimit)  [7] B of the initial store  [24 .. 27) goal record  [28] eta of the initial store
//   [64 + 64 c] (c < 8) generation copies: index + 1 of the latest decision
//   [kSyncDec + kDecWords r]  decision slot r: [1] added  [2] solved  [3] B  [4] eta  [8 .. 8+F) row
//   [kSyncFlags + b]  block b's published records: index + 1 of the latest sample
//   [kSyncRec + kRecWords (r nb + b)]  block b's record slot r: [0] distance  [1] id  [2 .. 2+F) row
constexpr int kSyncB = 7, kSyncGoal = 24, kSyncEta = 28, kSyncGen = 64, kGenCopies = 8, kGenStride = 64;
constexpr int kSyncDec = kSyncGen + kGenCopies * kGenStride, kDecWords = 32;
constexpr int kSyncFlags = kSyncDec + kRing * kDecWords, kSyncRec = kSyncFlags + (int)kRrtMaxCoopBlocks;
constexpr int kRecWords = 18;  // distance, id, F <= 16 reals

__device__ __forceinline__ void stores_done() { __builtin_amdgcn_s_waitcnt(0); }  // vmcnt = expcnt = lgkmcnt = 0
__device__ __forceinline__ uint64_t ld_sync(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sync(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t dbits(double v) { return (uint64_t)__double_as_longlong(v); }
__device__ __forceinline__ double bitsd(uint64_t v) { return __longlong_as_double((long long)v); }

// poll *p until it reaches `want` (false: the spin limit passed or some block aborted)
// (word [4] of the record, when non-zero, replaces kSpinLimit: the tests force an abort with it)
__device__ __forceinline__ bool wait_for(const uint64_t *p, uint64_t want, uint64_t *abort_word) {
    uint32_t spins = 0;
    const uint64_t lim = ld_sync(abort_word + 2);
    const uint32_t limit = lim ? (uint32_t)lim : kSpinLimit;
    while (ld_sync(p) < want) {
        __builtin_amdgcn_s_sleep(2);
        if (++spins > limit || ld_sync(abort_word)) return false;
    }
    return true;
}

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

// max |coordinate| (the screen's B: SE3 translation, R^n every coordinate)
template <int SP, int F>
__device__ __forceinline__ double coord_absmax(const double *x) {
    const int nc = SP == OMPL_GPU_SPACE_SE3 ? 3 : F;
    double m = 0.0;
    for (int c = 0; c < nc; ++c) m = fmax(m, fabs(x[c]));
    return m;
}

template <int SP, int F>
__device__ __forceinline__ void load_sample(const double *s, int dim, double *qv) {
#pragma unroll
    for (int f = 0; f < F; ++f) qv[f] = f < dim ? s[f] : 0.0;
}

// exact nearest of sample qv among positions [lo, end) of the store (see the header); every
// thread returns (d, id), and row = its fp64 row in LDS (valid when id != kNoId)
template <int SP, int F>
__device__ void slice_nearest(const double *__restrict__ feat, const float *__restrict__ feat32, uint64_t cap,
                              uint64_t lo, uint64_t end, const double *qv, const DevSpace &sp, double Bst, double eta_st,
                              double &wd, uint32_t &wi, double *row, double *lds_d, uint32_t *lds_i, float *lds_f) {
    constexpr int FS = Geo<SP, F>::FS;
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
    const float w0 = (float)sp.w0, w1 = (float)sp.w1;
    float c0 = __builtin_inff(), c1 = __builtin_inff();
    uint32_t i0 = kNoId;
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
            if (p + u >= end) d = __builtin_nanf("");
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
    wd = bd;
    wi = bi;
    block_argmin(wd, wi, lds_d, lds_i);
    if (wi != kNoId && bi == wi) {  // the winning thread (ids are unique)
#pragma unroll
        for (int f = 0; f < F; ++f) row[f] = brow[f];
    }
    __syncthreads();
}

template <int SP, int F>
__global__ __launch_bounds__(256) void rrt_persistent_kernel(
    double *__restrict__ feat, float *__restrict__ feat32, int rows32, uint64_t cap, uint64_t n0,
    uint64_t *__restrict__ n_dev, const double *__restrict__ samples, uint32_t ns, uint64_t slice, DevSpace sp,
    DevSpace msp, DevChecker ck, double maxd, uint64_t *__restrict__ sync, uint32_t *__restrict__ nearest_out,
    uint32_t *__restrict__ added_out, unsigned long long *__restrict__ counters, RrtGoal gl,
    uint64_t *__restrict__ grec) {
    __shared__ double lds_d[4];
    __shared__ uint32_t lds_i[4];
    __shared__ float lds_f[4];
    __shared__ double s1[kChainMaxLinks], s2[kChainMaxLinks], sh_q[F];
    __shared__ int sh_nd, sh_bad, sh_ok, sh_go, sh_stop;
    __shared__ uint64_t sh_added;
    __shared__ double sh_row[F];
    const uint32_t nsb = gridDim.x - 1, b = blockIdx.x;  // block nsb decides
    const int dim = sp.dim;
    uint64_t *abort_word = sync + 2, *flag = sync + kSyncFlags, *rec = sync + kSyncRec;
    double Bst = bitsd(ld_sync(&sync[kSyncB])), eta_st = bitsd(ld_sync(&sync[kSyncEta]));
    if (b < nsb) {
        // ---- a scanning block
        const uint64_t lo = (uint64_t)b * slice, hi = lo + slice;
        const uint64_t *gen = sync + kSyncGen + (b % kGenCopies) * kGenStride;
        uint64_t n = n0;       // n_{s-L}: the store size the scan of sample s sees
        uint32_t next_dec = 0;  // decisions processed so far
        // decision j: the new size, the appended row (this block's slice), the bounds; false = stop
        auto process = [&](uint32_t j) -> bool {
            const uint64_t *dec = sync + kSyncDec + (j % kRing) * kDecWords;
            if (threadIdx.x == 0) {
                sh_go = wait_for(gen, (uint64_t)j + 1, abort_word);
                if (!sh_go) st_sync(abort_word, 1);
                sh_added = ld_sync(&dec[1]);
                sh_stop = (int)ld_sync(&dec[2]);
                lds_d[0] = bitsd(ld_sync(&dec[3]));
                lds_d[1] = bitsd(ld_sync(&dec[4]));
            }
            __syncthreads();
            if (!sh_go) return false;
            const uint64_t added = sh_added;
            Bst = lds_d[0];
            eta_st = lds_d[1];
            const bool stop = sh_stop != 0;
            if (added != kNoId) {
                n = added + 1;
                if (added >= lo && added < hi) {
                    if (threadIdx.x < F) sh_row[threadIdx.x] = bitsd(ld_sync(&dec[8 + threadIdx.x]));
                    __syncthreads();
                    if (threadIdx.x == 0) rrt_append<F>(feat, feat32, rows32, cap, added, sh_row, dim);
                    // this CU's L1 may hold the line of the new row as loaded before the append: drop
                    // it before the next scan reads the row
                    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "agent");
                }
            }
            next_dec = j + 1;
            __syncthreads();  // shared words are rewritten by the next call
            return !stop;
        };
        for (uint32_t s = 0; s < ns; ++s) {
            if (s >= (uint32_t)kLook + 1 && !process(s - kLook - 1)) return;
            double qv[F];
            load_sample<SP, F>(samples + (size_t)s * dim, dim, qv);
            double wd;
            uint32_t wi;
            slice_nearest<SP, F>(feat, feat32, cap, lo, hi < n ? hi : n, qv, sp, Bst, eta_st, wd, wi, sh_row, lds_d,
                                 lds_i, lds_f);
            if (threadIdx.x == 0) {  // record slot s mod R, then the flag
                uint64_t *r = rec + ((size_t)(s % kRing) * nsb + b) * kRecWords;
                st_sync(&r[0], dbits(wd));
                st_sync(&r[1], wi);
                if (wi != kNoId)
                    for (int f = 0; f < F; ++f) st_sync(&r[2 + f], dbits(sh_row[f]));
                stores_done();
                st_sync(&flag[b], (uint64_t)s + 1);
            }
        }
        // the decisions not processed yet: their rows still go into the store
        for (uint32_t j = next_dec; j < ns;)
            if (!process(j++)) break;
        return;
    }
    // ---- the decider
    __shared__ double xrow[kLook][F];     // rows appended by the last L decisions, slot = decision % L
    __shared__ uint32_t xid[kLook], xdec[kLook];
    if (threadIdx.x < kLook) {
        xid[threadIdx.x] = kNoId;
        xdec[threadIdx.x] = 0;
    }
    uint64_t n = n0;
    uint32_t j = 0;
    for (; j < ns; ++j) {
        const double *s = samples + (size_t)j * dim;
        if (threadIdx.x < F) sh_q[threadIdx.x] = threadIdx.x < (uint32_t)dim ? s[threadIdx.x] : 0.0;
        // 1. every slice's record of sample j
        int ok = 1;
        if (threadIdx.x < nsb) ok = wait_for(&flag[threadIdx.x], (uint64_t)j + 1, abort_word);
        if (!__syncthreads_and(ok)) {
            if (threadIdx.x == 0) st_sync(abort_word, 1);
            return;  // aborted: the host sees the abort word and fails the call
        }
        double gd = __builtin_inf();
        uint32_t gi = kNoId;
        double row[F];
        if (threadIdx.x < nsb) {
            const uint64_t *r = rec + ((size_t)(j % kRing) * nsb + threadIdx.x) * kRecWords;
            gd = bitsd(ld_sync(&r[0]));
            gi = (uint32_t)ld_sync(&r[1]);
#pragma unroll
            for (int f = 0; f < F; ++f) row[f] = bitsd(ld_sync(&r[2 + f]));
        } else if (threadIdx.x >= 256 - kLook) {
            // 2. the states appended by decisions j - L .. j - 1, which no scan of sample j saw
            const int e = 255 - threadIdx.x;
            if (xid[e] != kNoId && xdec[e] + kLook >= j) {
                double qv[F];
#pragma unroll
                for (int f = 0; f < F; ++f) {
                    row[f] = xrow[e][f];
                    qv[f] = sh_q[f];
                }
                gd = feat_dist<SP, F, 0>(row, qv, sp);
                gi = xid[e];
            }
        }
        const uint32_t mine = gi;
        block_argmin(gd, gi, lds_d, lds_i);
        if (gi != kNoId && mine == gi) {
#pragma unroll
            for (int f = 0; f < F; ++f) sh_row[f] = row[f];
        }
        __syncthreads();
        // 3. steer, check the motion, goal test (RRT.cpp:137-187)
        const uint32_t ri = gi;
        rrt_decide<SP, kRrtWidth<SP>>([&](int c) { return sh_row[c]; }, sh_q, ri, sp, msp, ck, maxd, s1, s2, &sh_nd,
                                      &sh_bad, &sh_ok);
        if (threadIdx.x == 0) {
            uint64_t *dec = sync + kSyncDec + (j % kRing) * kDecWords;
            uint32_t added = kNoId;
            bool solved = false;
            if (sh_ok && !sh_bad && n < cap) {
                added = (uint32_t)n;
                double x[F];
                for (int f = 0; f < F; ++f) x[f] = f < dim ? s2[f] : 0.0;
                for (int f = 0; f < F; ++f) st_sync(&dec[8 + f], dbits(x[f]));
                Bst = fmax(Bst, coord_absmax<SP, F>(x));
                eta_st = fmax(eta_st, query_eta<SP>(x));
                solved = rrt_goal_test<SP, kRrtWidth<SP>>(gl, sp, x, added, j, sync + kSyncGoal);
                const int e = j % kLook;
                for (int f = 0; f < F; ++f) xrow[e][f] = x[f];
                xid[e] = added;
                xdec[e] = j;
                n += 1;
            }
            st_sync(&dec[1], added == kNoId ? (uint64_t)kNoId : (uint64_t)added);
            st_sync(&dec[2], solved);
            st_sync(&dec[3], dbits(Bst));
            st_sync(&dec[4], dbits(eta_st));
            nearest_out[j] = ri;
            added_out[j] = added;
            if (counters && sh_ok) atomicAdd(&counters[sh_bad ? 1 : 0], 1ull);  // valid_ / invalid_
            stores_done();
            for (int c = 0; c < kGenCopies; ++c) st_sync(&sync[kSyncGen + c * kGenStride], (uint64_t)j + 1);
            sh_go = !solved;
        }
        __syncthreads();
        if (!sh_go) break;
    }
    if (threadIdx.x == 0) {
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
            const uint32_t nscan = coop_blocks - 1;  // one block decides
            uint64_t slice = (nmax + nscan - 1) / nscan;
            slice = (slice + 1023) & ~(uint64_t)1023;
            const uint32_t nb = (uint32_t)((nmax + slice - 1) / slice) + 1;
            // one 256-thread block per CU: the grid is co-resident on any device that runs it at all
            // (a CU holds 8 such blocks), so an ordinary launch; a wait that outlives kSpinLimit
            // (the device shared with a long kernel) aborts the grid and the caller re-runs the batch
            // in the two-launch form.  (hipLaunchCooperativeKernel's queue made the HIP runtime's
            // exit-time teardown fault under rocprofv3: profiles/r3_extras.)
            hipLaunchKernelGGL((rrt_persistent_kernel<SP, F>), dim3(nb), dim3(256), 0, st, feat, feat32, rows32, cap,
                               n0, n_dev, samples, ns, slice, sp, msp, ck, maxd, sync, nearest, added, counters, gl,
                               grec);
            return hipGetLastError();
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
    int cus = 0;
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
    if (cus < 2) return 0;
    // one block per CU, one of them decides; the decider's last kLook threads fold in the states
    // of the last decisions, the others read one slice's record each
    return (uint32_t)std::min<int64_t>(cus, kRrtMaxCoopBlocks - kLook);
}

size_t rrt_part_entries(uint64_t n_max) { return (size_t)((n_max + kRrtBlockStates - 1) / kRrtBlockStates); }

size_t rrt_goal_words() { return kGoalWords; }

size_t rrt_sync_bytes() { return sizeof(uint64_t) * (kSyncRec + (size_t)kRing * kRrtMaxCoopBlocks * kRecWords); }

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
