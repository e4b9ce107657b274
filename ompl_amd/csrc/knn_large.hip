// knn_large.hip — exact kNN for large k (k > 32), e.g. RRT*'s k = ceil(k_rrt log(n+1))
// ≈ 6,169 at n = 10^6 (RRTstar.cpp:603-618, :1147-1159).  Register top-K lists do not
// scale to thousands, so the selection is done by distance thresholds:
//
//   1. histogram (fp32 screen): per query, 64 distance bins of width w over [0, 64 w);
//      bin counts accumulate in LDS (each thread owns a padded row) then global;
//   2. threshold: the first bin where the cumulative count reaches k gives r_hi with
//      #{d32 <= r_hi} >= k, hence the exact k-th distance d*_k <= r_hi + e and every
//      true top-k element has d32 <= r_hi + 2e (e = the fp32 error bound of
//      knn_fast.hip); r = r_hi + 2e;
//   3. count + fill (fp32 screen, exact fp64 distance for survivors): candidates
//      d32 <= r are written per (query, chunk) in ascending id order;
//   4. stable segmented radix sort by fp64 distance -> (distance, id) order; the first k
//      of each query's segment are the answer (exact, as the reference's ascending list).
#include <hip/hip_runtime.h>
#include <cstring>  // (rocPRIM block primitives need memset declared)
#include <rocprim/rocprim.hpp>

#include <algorithm>
#include <cmath>
#include <vector>

#include "feat_dist.h"
#include "kernels.h"
#include "topk.h"

namespace ompl_amd {

namespace {

constexpr int kBins = 64;
constexpr int kBinStride = kBins + 1;  // padded LDS rows: bank = (tid + bin) mod 32
constexpr double kU = 5.9604644775390625e-08;

template <int SP, int F>
struct Row {
    static constexpr int FS = SP == OMPL_GPU_SPACE_SE3 ? 8 : F;
};

__device__ __forceinline__ float abs1(float x) {
    float a = fabsf(x);
    return a > 1.f ? 1.f : a;
}

// fp32 screening distance (element row s, query row q); KinematicChain: rows are the joint
// positions (knn_fast.hip chain rows), w0 = the link length, nl = the number of links
template <int SP, int FS>
__device__ __forceinline__ float d32(const float *s, const float *q, float w0, float w1, int nl) {
    if constexpr (SP == OMPL_GPU_SPACE_KCHAIN) {
        constexpr int NM = FS / 2;
        float acc = 0.f;
#pragma unroll
        for (int i = 0; i < NM; ++i) {
            if (i < nl) {
                const float dx = s[i] - q[i], dy = s[NM + i] - q[NM + i];
                acc += __builtin_amdgcn_sqrtf(fmaf(dy, dy, dx * dx));
            }
        }
        return acc * w0;
    } else if constexpr (SP == OMPL_GPU_SPACE_SE3) {
        const float dx = s[0] - q[0], dy = s[1] - q[1], dz = s[2] - q[2];
        float t = dx * dx;
        t = fmaf(dy, dy, t);
        t = fmaf(dz, dz, t);
        // rotation by the chord, as the culled walks (knn_fast_impl.h header: error bound)
        return fmaf(w1, chord_angle(s + 4, q + 4), w0 * __builtin_amdgcn_sqrtf(t));
    } else if constexpr (SP == OMPL_GPU_SPACE_SO3) {
        float dot = s[0] * q[0];
        dot = fmaf(s[1], q[1], dot);
        dot = fmaf(s[2], q[2], dot);
        dot = fmaf(s[3], q[3], dot);
        return acosf(abs1(dot));
    } else {
        float acc = 0.f;
#pragma unroll
        for (int f = 0; f < FS; ++f) {
            const float diff = s[f] - q[f];
            acc = fmaf(diff, diff, acc);
        }
        return sqrtf(acc);
    }
}

template <int SP, int FS>
__device__ __forceinline__ void stage_tile(float *tile, const float *__restrict__ f32, uint64_t cap, uint64_t g) {
    if constexpr (SP == OMPL_GPU_SPACE_SE3) {
        float4 a, r;
        a.x = f32[g]; a.y = f32[cap + g]; a.z = f32[2 * cap + g]; a.w = 0.f;
        r.x = f32[3 * cap + g]; r.y = f32[4 * cap + g]; r.z = f32[5 * cap + g]; r.w = f32[6 * cap + g];
        reinterpret_cast<float4 *>(tile)[threadIdx.x * 2] = a;
        reinterpret_cast<float4 *>(tile)[threadIdx.x * 2 + 1] = r;
    } else {
#pragma unroll
        for (int f = 0; f < FS; ++f) tile[threadIdx.x * FS + f] = f32[(uint64_t)f * cap + g];
    }
}

template <int SP, int F>
__global__ void rows32_kernel(const double *__restrict__ qf, uint32_t nq, float *__restrict__ q32) {
    constexpr int FS = Row<SP, F>::FS;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nq) return;
    const double *s = qf + (size_t)i * F;
    float *o = q32 + (size_t)i * FS;
    if constexpr (SP == OMPL_GPU_SPACE_SE3) {
        o[0] = (float)s[0]; o[1] = (float)s[1]; o[2] = (float)s[2]; o[3] = 0.f;
        o[4] = (float)s[3]; o[5] = (float)s[4]; o[6] = (float)s[5]; o[7] = (float)s[6];
    } else if constexpr (SP == OMPL_GPU_SPACE_KCHAIN) {
        // joint positions: prefix sums of the cumulative cos / sin features in fp64, then
        // rounded (the stored rows' recipe)
        constexpr int NM = F / 2;
        double cx = 0.0, cy = 0.0;
        for (int i = 0; i < NM; ++i) {
            cx += s[i];
            cy += s[NM + i];
            o[i] = (float)cx;
            o[NM + i] = (float)cy;
        }
    } else {
        for (int f = 0; f < FS; ++f) o[f] = (float)s[f];
    }
}

template <int SP, int F>
__global__ __launch_bounds__(256) void hist_kernel(const float *__restrict__ f32, uint64_t cap, uint64_t n_end,
                                                   const float *__restrict__ q32, uint32_t nq, uint32_t chunk_len,
                                                   float w0, float w1, int nl, float inv_bin,
                                                   unsigned int *__restrict__ hist) {
    constexpr int FS = Row<SP, F>::FS;
    __shared__ __attribute__((aligned(16))) float tile[kTile * FS];
    __shared__ unsigned int h[kTile * kBinStride];
    for (int b = 0; b < kBins; ++b) h[threadIdx.x * kBinStride + b] = 0;
    const uint32_t q = blockIdx.x * kTile + threadIdx.x;
    float qf[FS];
#pragma unroll
    for (int f = 0; f < FS; ++f) qf[f] = q < nq ? q32[(size_t)q * FS + f] : __builtin_nanf("");
    const uint64_t c0 = (uint64_t)blockIdx.y * chunk_len, c1 = min(c0 + chunk_len, n_end);
    for (uint64_t base = c0; base < c1; base += kTile) {
        stage_tile<SP, FS>(tile, f32, cap, base + threadIdx.x);
        __syncthreads();
        for (int s = 0; s < kTile; ++s) {
            const float d = d32<SP, FS>(&tile[s * FS], qf, w0, w1, nl);
            if (d == d) {  // NaN (removed / padding / idle thread) is not counted
                const float x = d * inv_bin;
                const int b = x < (float)(kBins - 1) ? (int)x : kBins - 1;
                h[threadIdx.x * kBinStride + b] += 1u;
            }
        }
        __syncthreads();
    }
    if (q >= nq) return;
    for (int b = 0; b < kBins; ++b) {
        const unsigned int c = h[threadIdx.x * kBinStride + b];
        if (c) atomicAdd(&hist[(size_t)q * kBins + b], c);
    }
}

// eta (SE3): the store's largest |norm^2 - 1| of a quaternion + the query's (the chord bound,
// knn_fast_impl.h screen_error<SE3>)
template <int SP>
__device__ __forceinline__ double query_eta(const double *qv) {  // |norm^2 - 1| of an SE3 query's quaternion
    if constexpr (SP == OMPL_GPU_SPACE_SE3) {
        const double n = qv[3] * qv[3] + qv[4] * qv[4] + qv[5] * qv[5] + qv[6] * qv[6];
        return fabs(n - 1.0);
    }
    return 0.0;
}

template <int SP>
__device__ __forceinline__ double screen_err(const DevSpace &sp, double B, double L, double eta) {
    double e;
    if constexpr (SP == OMPL_GPU_SPACE_SE3)
        e = sp.w0 * (6.0 * 1.7320508075688772 * kU * B) + 6.0 * kU * L +
            sp.w1 * (2.25 * sqrt(0.5 * eta + 1e-15) + 2e-6 + 4.5e-5) + sp.w0 * sqrt(3.0 * 1.1754943508222875e-38);
    else if constexpr (SP == OMPL_GPU_SPACE_SO3)
        e = 1.1 * sqrt(12.0 * kU) + 1e-6 + 4.5e-5;
    else if constexpr (SP == OMPL_GPU_SPACE_KCHAIN) {  // knn_fast_impl.h screen_error<KCHAIN>
        const double n = (double)sp.dim;
        e = sp.link * 8.0 * kU * n * (n + 1.0) + (n + 2.0) * kU * L + sp.link * n * sqrt(2.0 * 1.1754943508222875e-38);
        return 2.0 * e;
    } else
        e = 6.0 * sqrt((double)sp.dim) * kU * B + 6.0 * kU * L;
    e += sqrt(16.0 * 1.1754943508222875e-38);  // underflow of the squares (knn_fast_impl.h screen_error)
    return 2.0 * e;
}

template <int SP, int F>
__global__ void threshold_kernel(const unsigned int *__restrict__ hist, const double *__restrict__ qf64, uint32_t nq,
                                 uint32_t k, float bin_w, float absmax, float seta, DevSpace sp,
                                 float *__restrict__ radius) {
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nq) return;
    unsigned long long cum = 0;
    int b = 0;
    for (; b < kBins; ++b) {
        cum += hist[(size_t)q * kBins + b];
        if (cum >= k) break;
    }
    if (b >= kBins - 1) {  // k-th lies in the overflow bin, or fewer than k live elements
        radius[q] = __builtin_inff();
        return;
    }
    const double r_hi = (double)(b + 1) * bin_w * (1.0 + 1e-5);  // slack for the float bin index
    double B = absmax;
    const int nc = SP == OMPL_GPU_SPACE_SE3 ? 3 : (SP == OMPL_GPU_SPACE_REALVECTOR ? F : 0);
    for (int c = 0; c < nc; ++c) B = fmax(B, fabs(qf64[(size_t)q * F + c]));
    const double e = screen_err<SP>(sp, B, r_hi + 1.0, (double)seta + query_eta<SP>(qf64 + (size_t)q * F));
    radius[q] = (float)((r_hi + 2.0 * e) * (1.0 + 16.0 * kU));
}

// FILL=false: counts[q][chunk]; FILL=true: write (d64, id) from offsets[q][chunk]
template <int SP, int F, bool FILL>
__global__ __launch_bounds__(256) void select_kernel(const float *__restrict__ f32, const double *__restrict__ f64,
                                                     uint64_t cap, uint64_t n_end, const float *__restrict__ q32,
                                                     const double *__restrict__ qf64, uint32_t q0, uint32_t q1,
                                                     uint32_t chunk_len, uint32_t chunks, DevSpace sp,
                                                     const float *__restrict__ radius, uint32_t *__restrict__ counts,
                                                     const uint64_t *__restrict__ offsets, double *__restrict__ od,
                                                     uint32_t *__restrict__ oi) {
    constexpr int FS = Row<SP, F>::FS;
    __shared__ __attribute__((aligned(16))) float tile[kTile * FS];
    const uint32_t q = q0 + blockIdx.x * kTile + threadIdx.x;
    const bool live = q < q1;
    float qf[FS];
#pragma unroll
    for (int f = 0; f < FS; ++f) qf[f] = live ? q32[(size_t)q * FS + f] : __builtin_nanf("");
    double qv[F];
    if (FILL) {
#pragma unroll
        for (int f = 0; f < F; ++f) qv[f] = live ? qf64[(size_t)q * F + f] : 0.0;
    }
    const float r = live ? radius[q] : -1.f;
    const uint64_t c0 = (uint64_t)blockIdx.y * chunk_len, c1 = min(c0 + chunk_len, n_end);
    uint32_t cnt = 0;
    uint64_t out = (FILL && live) ? offsets[(size_t)(q - q0) * chunks + blockIdx.y] : 0;
    for (uint64_t base = c0; base < c1; base += kTile) {
        stage_tile<SP, FS>(tile, f32, cap, base + threadIdx.x);
        __syncthreads();
        for (int s = 0; s < kTile; ++s) {
            const float d = SP == OMPL_GPU_SPACE_KCHAIN ? d32<SP, FS>(&tile[s * FS], qf, (float)sp.link, 0.f, sp.dim)
                                                        : d32<SP, FS>(&tile[s * FS], qf, (float)sp.w0, (float)sp.w1, 0);
            if (d <= r) {
                if (FILL) {
                    const uint32_t id = (uint32_t)(base + s);
                    double sv[F];
#pragma unroll
                    for (int f = 0; f < F; ++f) sv[f] = f64[(uint64_t)f * cap + id];
                    od[out] = feat_dist<SP, F, SP == OMPL_GPU_SPACE_KCHAIN ? F / 2 : 0>(sv, qv, sp);
                    oi[out] = id;
                    ++out;
                } else {
                    ++cnt;
                }
            }
        }
        __syncthreads();
    }
    if (!FILL && live) counts[(size_t)q * chunks + blockIdx.y] = cnt;
}

__global__ void take_first_k_kernel(const double *__restrict__ sd, const uint32_t *__restrict__ si,
                                    const uint64_t *__restrict__ seg, uint32_t q0, uint32_t nqb, uint32_t k,
                                    double *__restrict__ out_d, uint32_t *__restrict__ out_i) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (uint64_t)nqb * k) return;
    const uint32_t ql = (uint32_t)(t / k), j = (uint32_t)(t % k);
    const uint64_t b = seg[ql], e = seg[ql + 1];
    const size_t o = (size_t)(q0 + ql) * k + j;
    if (b + j < e) {
        out_d[o] = sd[b + j];
        out_i[o] = si[b + j];
    } else {
        out_d[o] = __builtin_inf();
        out_i[o] = kNoId;
    }
}

struct Plan {
    uint32_t chunks, chunk_len;
};

Plan plan(uint32_t nq, uint64_t n_end, int num_cus) {
    const uint64_t tiles = std::max<uint64_t>(n_end / kTile, 1);
    const uint64_t qblocks = (nq + kTile - 1) / kTile;
    const uint64_t target = (uint64_t)num_cus * 4;
    uint64_t S = std::max<uint64_t>(1, std::min<uint64_t>((target + qblocks - 1) / qblocks, tiles));
    const uint64_t per = (tiles + S - 1) / S;
    Plan p;
    p.chunk_len = (uint32_t)(per * kTile);
    p.chunks = (uint32_t)((n_end + p.chunk_len - 1) / p.chunk_len);
    return p;
}

template <int SP, int F>
hipError_t run_large(const DevSpace &sp, const double *f64, const float *f32, uint64_t cap, uint64_t n_end,
                     const double *qf64, uint32_t nq, uint32_t k, float absmax, float seta, float dmax,
                     double *out_d, uint32_t *out_i, size_t mem_budget, int num_cus, hipStream_t st) {
    constexpr int FS = Row<SP, F>::FS;
    const Plan p = plan(nq, n_end, num_cus);
    const float bin_w = dmax / (float)(kBins - 1);
    float *q32 = nullptr, *radius = nullptr;
    unsigned int *hist = nullptr;
    uint32_t *counts = nullptr;
    hipError_t e;
    auto cleanup = [&]() {
        if (q32) (void)hipFree(q32);
        if (radius) (void)hipFree(radius);
        if (hist) (void)hipFree(hist);
        if (counts) (void)hipFree(counts);
    };
#define TRYL(x)                    \
    if ((e = (x)) != hipSuccess) { \
        cleanup();                 \
        return e;                  \
    }
    TRYL(hipMalloc(&q32, sizeof(float) * nq * FS));
    TRYL(hipMalloc(&radius, sizeof(float) * nq));
    TRYL(hipMalloc(&hist, sizeof(unsigned int) * nq * kBins));
    TRYL(hipMalloc(&counts, sizeof(uint32_t) * (size_t)nq * p.chunks));
    TRYL(hipMemsetAsync(hist, 0, sizeof(unsigned int) * nq * kBins, st));
    hipLaunchKernelGGL((rows32_kernel<SP, F>), dim3((nq + 255) / 256), dim3(256), 0, st, qf64, nq, q32);
    const dim3 grid((nq + kTile - 1) / kTile, p.chunks);
    timer_begin(st, "hist_kernel");
    const float w0 = SP == OMPL_GPU_SPACE_KCHAIN ? (float)sp.link : (float)sp.w0;
    hipLaunchKernelGGL((hist_kernel<SP, F>), grid, dim3(kTile), 0, st, f32, cap, n_end, q32, nq, p.chunk_len, w0,
                       (float)sp.w1, sp.dim, 1.0f / bin_w, hist);
    timer_end(st);
    hipLaunchKernelGGL((threshold_kernel<SP, F>), dim3((nq + 255) / 256), dim3(256), 0, st, hist, qf64, nq, k, bin_w,
                       absmax, seta, sp, radius);
    hipLaunchKernelGGL((select_kernel<SP, F, false>), grid, dim3(kTile), 0, st, f32, f64, cap, n_end, q32, qf64, 0u,
                       nq, p.chunk_len, p.chunks, sp, radius, counts, nullptr, nullptr, nullptr);
    std::vector<uint32_t> hc((size_t)nq * p.chunks);
    TRYL(hipMemcpyAsync(hc.data(), counts, sizeof(uint32_t) * hc.size(), hipMemcpyDeviceToHost, st));
    TRYL(hipStreamSynchronize(st));
    // sub-batches of queries whose candidates fit the memory budget
    const size_t per_cand = sizeof(double) * 2 + sizeof(uint32_t) * 2;
    const uint64_t budget = std::max<uint64_t>(mem_budget / per_cand, (uint64_t)k * 2);
    uint32_t q0 = 0;
    while (q0 < nq) {
        uint64_t tot = 0;
        uint32_t q1 = q0;
        while (q1 < nq) {
            uint64_t c = 0;
            for (uint32_t j = 0; j < p.chunks; ++j) c += hc[(size_t)q1 * p.chunks + j];
            if (q1 > q0 && tot + c > budget) break;
            tot += c;
            ++q1;
        }
        const uint32_t nqb = q1 - q0;
        if (tot > 0x7FFFFFF0ull) {
            cleanup();
            return hipErrorOutOfMemory;  // one query's candidates beyond a radix-sort segment
        }
        std::vector<uint64_t> off((size_t)nqb * p.chunks), seg(nqb + 1);
        uint64_t run = 0;
        for (uint32_t ql = 0; ql < nqb; ++ql) {
            seg[ql] = run;
            for (uint32_t j = 0; j < p.chunks; ++j) {
                off[(size_t)ql * p.chunks + j] = run;
                run += hc[(size_t)(q0 + ql) * p.chunks + j];
            }
        }
        seg[nqb] = run;
        uint64_t *d_off = nullptr, *d_seg = nullptr;
        double *cd = nullptr, *sd = nullptr;
        uint32_t *ci = nullptr, *si = nullptr;
        void *tmp = nullptr;
        auto free_batch = [&]() {
            for (void *x : {(void *)d_off, (void *)d_seg, (void *)cd, (void *)sd, (void *)ci, (void *)si, tmp})
                if (x) (void)hipFree(x);
        };
#define TRYB(x)                    \
    if ((e = (x)) != hipSuccess) { \
        free_batch();              \
        cleanup();                 \
        return e;                  \
    }
        const size_t ncand = std::max<uint64_t>(run, 1);
        TRYB(hipMalloc(&d_off, sizeof(uint64_t) * off.size()));
        TRYB(hipMalloc(&d_seg, sizeof(uint64_t) * seg.size()));
        TRYB(hipMalloc(&cd, sizeof(double) * ncand));
        TRYB(hipMalloc(&sd, sizeof(double) * ncand));
        TRYB(hipMalloc(&ci, sizeof(uint32_t) * ncand));
        TRYB(hipMalloc(&si, sizeof(uint32_t) * ncand));
        TRYB(hipMemcpyAsync(d_off, off.data(), sizeof(uint64_t) * off.size(), hipMemcpyHostToDevice, st));
        TRYB(hipMemcpyAsync(d_seg, seg.data(), sizeof(uint64_t) * seg.size(), hipMemcpyHostToDevice, st));
        const dim3 gb((nqb + kTile - 1) / kTile, p.chunks);
        hipLaunchKernelGGL((select_kernel<SP, F, true>), gb, dim3(kTile), 0, st, f32, f64, cap, n_end, q32, qf64, q0,
                           q1, p.chunk_len, p.chunks, sp, radius, nullptr, d_off, cd, ci);
        uint64_t longest = 0;
        for (uint32_t ql = 0; ql < nqb; ++ql) longest = std::max<uint64_t>(longest, seg[ql + 1] - seg[ql]);
        TRYB(hipMalloc(&tmp, segment_sort_workspace(run)));
        int second = 0;  // (distance, id) order: the candidates' ties by id
        TRYB(launch_segment_sort(d_seg, nqb, run, longest, ci, cd, si, sd, tmp, st, &second));
        const uint64_t nout = (uint64_t)nqb * k;
        hipLaunchKernelGGL(take_first_k_kernel, dim3((unsigned)((nout + 255) / 256)), dim3(256), 0, st,
                           second ? sd : cd, second ? si : ci, d_seg, q0, nqb, k, out_d, out_i);
        TRYB(hipStreamSynchronize(st));
        free_batch();
#undef TRYB
        q0 = q1;
    }
    cleanup();
#undef TRYL
    return hipGetLastError();
}

// ---- device-decided select (k <= kLargeSelMaxK): no host round trip -------------------------
// 1. two sampled histograms of the fp32 screen (every kSampleA-th / kSampleB-th 256-state tile):
//    A over [0, dmax) sets each query's range, B over that range (64 bins) gives a radius r whose
//    estimated population is k plus six standard deviations of the sampling error;
// 2. one pass over the store: every state with d32 <= r + 2e gets its exact fp64 distance and is
//    written to the query's slab for that chunk (fixed capacity, in id order), and the states with
//    d32 <= r are counted — at least k of them prove that the exact k-th distance is <= r + e, so
//    every true neighbour (d32 <= d64 + e) is a candidate;
// 3. a block per query radix-selects the k-th smallest (distance, id) among its candidates, packs the
//    k selected in id order into LDS and block-radix-sorts them by distance (stable: (distance, id));
// 4. a query whose slab overflowed or whose count fell short (sampling outlier, heavy ties) is
//    answered by the exact fallback: a block per query, the same select over every stored state.
constexpr uint32_t kSampleA = 64, kSampleB = 8;
constexpr uint32_t kLargeSelMaxK = 8192;  // selected entries sorted in LDS
constexpr int kSelBlock = 1024, kSelItems = kLargeSelMaxK / kSelBlock;

template <int SP, int F>
__global__ __launch_bounds__(256) void hist_sample_kernel(const float *__restrict__ f32, uint64_t cap,
                                                          uint64_t n_end, const float *__restrict__ q32, uint32_t nq,
                                                          uint32_t chunk_len, uint32_t stride, float w0, float w1,
                                                          int nl, const float *__restrict__ inv_bin_q,
                                                          float inv_bin, unsigned int *__restrict__ hist) {
    constexpr int FS = Row<SP, F>::FS;
    __shared__ __attribute__((aligned(16))) float tile[kTile * FS];
    __shared__ unsigned int h[kTile * kBinStride];
    for (int b = 0; b < kBins; ++b) h[threadIdx.x * kBinStride + b] = 0;
    const uint32_t q = blockIdx.x * kTile + threadIdx.x;
    float qf[FS];
#pragma unroll
    for (int f = 0; f < FS; ++f) qf[f] = q < nq ? q32[(size_t)q * FS + f] : __builtin_nanf("");
    const float ib = inv_bin_q ? (q < nq ? inv_bin_q[q] : 0.f) : inv_bin;
    const uint64_t c0 = (uint64_t)blockIdx.y * chunk_len, c1 = min(c0 + chunk_len, n_end);
    // the sample is every stride-th 256-state tile of the whole store (global tile index), so the
    // sampled fraction is 1 / stride whatever the chunk length (chunks start on tile boundaries)
    const uint64_t t0 = (c0 / kTile + stride - 1) / stride * stride;
    for (uint64_t base = t0 * kTile; base < c1; base += (uint64_t)kTile * stride) {
        stage_tile<SP, FS>(tile, f32, cap, base + threadIdx.x);
        __syncthreads();
        for (int s = 0; s < kTile; ++s) {
            const float d = d32<SP, FS>(&tile[s * FS], qf, w0, w1, nl);
            const float x = d * ib;
            if (x < (float)kBins) h[threadIdx.x * kBinStride + (int)x] += 1u;  // NaN / beyond the range: not counted
        }
        __syncthreads();
    }
    if (q >= nq) return;
    for (int b = 0; b < kBins; ++b) {
        const unsigned int c = h[threadIdx.x * kBinStride + b];
        if (c) atomicAdd(&hist[(size_t)q * kBins + b], c);
    }
}

// from sampled histogram A (over [0, dmax)): each query's range for B — the first bin whose
// scaled count passes 1.5 k + 64 (or dmax) — as 64 / range
__global__ void sel_range_kernel(const unsigned int *__restrict__ hist, uint32_t nq, uint32_t k, float bin_w,
                                 float *__restrict__ inv_bin_q) {
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nq) return;
    const double need = (1.5 * k + 64.0) / kSampleA;
    double cum = 0;
    int b = 0;
    for (; b < kBins; ++b) {
        cum += hist[(size_t)q * kBins + b];
        if (cum >= need) break;
    }
    const float range = (float)(b + 1) * bin_w * 1.0001f;
    inv_bin_q[q] = (float)kBins / range;
}

// from sampled histogram B: r (the counting radius) and r + 2e (the collecting radius)
template <int SP, int F>
__global__ void sel_radius_kernel(const unsigned int *__restrict__ hist, const float *__restrict__ inv_bin_q,
                                  const double *__restrict__ qf64, uint32_t nq, uint32_t k, float absmax, float seta,
                                  DevSpace sp, float *__restrict__ r_count, float *__restrict__ r_fill) {
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nq) return;
    const double need = ((double)k + 6.0 * sqrt((double)kSampleB * k) + 2.0 * kSampleB) / kSampleB;
    double cum = 0;
    int b = 0;
    for (; b < kBins - 1; ++b) {
        cum += hist[(size_t)q * kBins + b];
        if (cum >= need) break;
    }
    const double r = (double)(b + 1) / (double)inv_bin_q[q] * (1.0 + 1e-5);
    double B = absmax;
    const int nc = SP == OMPL_GPU_SPACE_SE3 ? 3 : (SP == OMPL_GPU_SPACE_REALVECTOR ? F : 0);
    for (int c = 0; c < nc; ++c) B = fmax(B, fabs(qf64[(size_t)q * F + c]));
    const double e = screen_err<SP>(sp, B, r + 1.0, (double)seta + query_eta<SP>(qf64 + (size_t)q * F));
    r_count[q] = (float)r;
    r_fill[q] = (float)((r + 2.0 * e) * (1.0 + 16.0 * kU));
}

// one pass: candidates d32 <= r_fill of (query, chunk) into that slab (ascending id), exact fp64
// distance; counts of d32 <= r_count per query.  slab_cnt may exceed `slab` (overflow).
template <int SP, int F>
__global__ __launch_bounds__(256) void sel_fill_kernel(const float *__restrict__ f32, const double *__restrict__ f64,
                                                       uint64_t cap, uint64_t n_end, const float *__restrict__ q32,
                                                       const double *__restrict__ qf64, uint32_t nq,
                                                       uint32_t chunk_len, uint32_t chunks, DevSpace sp,
                                                       const float *__restrict__ r_count,
                                                       const float *__restrict__ r_fill, uint32_t slab,
                                                       uint32_t ovcap, uint32_t *__restrict__ ci,
                                                       uint32_t *__restrict__ ov, uint32_t *__restrict__ ov_cnt,
                                                       uint32_t *__restrict__ slab_cnt,
                                                       unsigned int *__restrict__ count_r) {
    constexpr int FS = Row<SP, F>::FS;
    __shared__ __attribute__((aligned(16))) float tile[kTile * FS];
    const uint32_t q = blockIdx.x * kTile + threadIdx.x;
    const bool live = q < nq;
    float qf[FS];
#pragma unroll
    for (int f = 0; f < FS; ++f) qf[f] = live ? q32[(size_t)q * FS + f] : __builtin_nanf("");
    const float rc = live ? r_count[q] : -1.f, rf = live ? r_fill[q] : -1.f;
    const uint64_t c0 = (uint64_t)blockIdx.y * chunk_len, c1 = min(c0 + chunk_len, n_end);
    const size_t sbase = ((size_t)q * chunks + blockIdx.y) * slab;
    uint32_t cnt = 0, cr = 0;
    for (uint64_t base = c0; base < c1; base += kTile) {
        stage_tile<SP, FS>(tile, f32, cap, base + threadIdx.x);
        __syncthreads();
        for (int s = 0; s < kTile; ++s) {
            const float d = SP == OMPL_GPU_SPACE_KCHAIN ? d32<SP, FS>(&tile[s * FS], qf, (float)sp.link, 0.f, sp.dim)
                                                        : d32<SP, FS>(&tile[s * FS], qf, (float)sp.w0, (float)sp.w1, 0);
            cr += d <= rc ? 1u : 0u;
            if (d <= rf) {  // the exact distance comes later, densely (sel_sort_kernel): here it
                            // would run for the whole wave whenever one lane has a candidate
                if (cnt < slab) {
                    ci[sbase + cnt] = (uint32_t)(base + s);
                } else {  // a full slab spills to the query's pool (the ids whose chunk is dense:
                          // a store whose id order follows space puts a query's whole
                          // neighbourhood in a few chunks)
                    const uint32_t p = atomicAdd(&ov_cnt[q], 1u);
                    if (p < ovcap) ov[(size_t)q * ovcap + p] = (uint32_t)(base + s);
                }
                ++cnt;
            }
        }
        __syncthreads();
    }
    if (!live) return;
    slab_cnt[(size_t)q * chunks + blockIdx.y] = cnt;
    if (cr) atomicAdd(&count_r[q], cr);
}

// (distance, id) as a 96-bit key, ordered: distances are >= 0 so their bits order as integers
struct SelKey {
    uint64_t d;
    uint32_t i;
};
__device__ __forceinline__ bool sel_le(uint64_t d, uint32_t i, uint64_t Td, uint32_t Ti) {
    return d < Td || (d == Td && i <= Ti);
}

// Block-wide selection over a candidate source: `count` candidates indexed 0..count-1 in id
// order, get(e, d_bits, id) fetching one (valid == false: skip).  Finds the k-th smallest
// (distance, id) by radix select (8-bit digits: 64 bits of the distance, then 32 of the id),
// packs the k selected (id order) into LDS, sorts them stably by distance and writes row q.
// id_sort: the source is not in id order (slab spills): the k selected are sorted by id first, so
// that the stable distance sort still orders equal distances by id.
// A digit whose boundary bin is taken whole (its count equals what is still needed) ends the
// select early: every key with that prefix is selected, whatever its lower bits — usually after
// 3-4 of the 9 digits.
template <class Get>
__device__ void block_select_sort(Get get, uint32_t count, uint32_t k, uint32_t q, double *__restrict__ out_d,
                                  uint32_t *__restrict__ out_i, bool id_sort = false) {
    using BlockSort = rocprim::block_radix_sort<uint64_t, kSelBlock, kSelItems, uint32_t>;
    using IdSort = rocprim::block_radix_sort<uint32_t, kSelBlock, kSelItems, uint64_t>;
    using BlockScan = rocprim::block_scan<uint32_t, kSelBlock>;
    constexpr int kDigit = 11, kRadix = 1 << kDigit;
    __shared__ union {
        struct {
            uint64_t d[kLargeSelMaxK];
            uint32_t i[kLargeSelMaxK];
        } stage;
        typename BlockSort::storage_type sort;
        typename IdSort::storage_type id_sort;
    } sh;
    __shared__ typename BlockScan::storage_type scan_storage;
    __shared__ uint32_t hist[kRadix];
    __shared__ uint32_t sh_digit, sh_need, sh_full;
    const uint32_t tid = threadIdx.x;
    const int lane = threadIdx.x & 63;
    // radix select of the k-th smallest (distance bits, id): 11-bit digits, most significant
    // first — 64 distance bits in 6 digits (11, 11, 11, 11, 11, 9), then 32 id bits in 3
    constexpr int kShift[9] = {53, 42, 31, 20, 9, 0, 21, 10, 0};
    constexpr int kBits[9] = {11, 11, 11, 11, 11, 9, 11, 11, 10};
    uint64_t Td = 0;
    uint32_t Ti = 0;
    uint32_t need = min(k, count);
    for (int dg = 0; dg < 9; ++dg) {
        const bool on_d = dg < 6;
        const int shift = kShift[dg], bits = kBits[dg];
        const uint32_t dmask = (1u << bits) - 1u;
        for (uint32_t b = tid; b < kRadix; b += kSelBlock) hist[b] = 0;
        if (tid == 0) {  // defaults: nothing left to select (need == 0) takes the whole digit range
            sh_digit = dmask;
            sh_need = 0;
            sh_full = 1;
        }
        __syncthreads();
        for (uint32_t e0 = 0; e0 < count; e0 += kSelBlock) {  // uniform trip count: the ballots below
            const uint32_t e = e0 + tid;
            uint64_t d = 0;
            uint32_t i = 0;
            bool part = e < count && get(e, d, i);
            uint32_t digit;
            if (on_d) {
                part = part && (dg == 0 || (d >> (shift + bits)) == (Td >> (shift + bits)));
                digit = (uint32_t)(d >> shift) & dmask;
            } else {
                part = part && d == Td && (dg == 6 || (i >> (shift + bits)) == (Ti >> (shift + bits)));
                digit = (i >> shift) & dmask;
            }
            // the leading digits are mostly equal across a wave (the distances' exponent): one
            // atomic with the wave's count then, instead of 64 serialised on one LDS address
            const uint64_t pm = __ballot(part);
            if (pm) {
                const int leader = __builtin_ctzll(pm);
                const uint32_t ld = (uint32_t)__shfl((int)digit, leader);
                if (__ballot(part && digit == ld) == pm) {
                    if (lane == leader) atomicAdd(&hist[ld], (uint32_t)__popcll(pm));
                } else if (part) {
                    atomicAdd(&hist[digit], 1u);
                }
            }
        }
        __syncthreads();
        // the digit where the running count reaches `need`: block scan of the 2,048 counts
        uint32_t c0 = hist[2 * tid], c1 = hist[2 * tid + 1], pre = 0, tot = 0;
        BlockScan().exclusive_scan(c0 + c1, pre, 0u, tot, scan_storage);
        if (pre < need && pre + c0 >= need) {
            sh_digit = 2 * tid;
            sh_need = need - pre;
            sh_full = pre + c0 == need ? 1u : 0u;
        } else if (pre + c0 < need && pre + c0 + c1 >= need) {
            sh_digit = 2 * tid + 1;
            sh_need = need - pre - c0;
            sh_full = pre + c0 + c1 == need ? 1u : 0u;
        }
        __syncthreads();  // (fewer candidates than k: the defaults take them all)
        if (on_d)
            Td |= (uint64_t)sh_digit << shift;
        else
            Ti |= sh_digit << shift;
        need = sh_need;
        const bool full = sh_full != 0;
        __syncthreads();
        if (full) {  // the boundary bin is taken whole: every lower bit (and id) passes
            if (on_d) {
                Td |= shift ? ((1ull << shift) - 1ull) : 0ull;
                Ti = 0xFFFFFFFFu;
            } else {
                Ti |= shift ? ((1u << shift) - 1u) : 0u;
            }
            break;
        }
    }
    // pack the selected keys (<= (Td, Ti)) in source order (id order): block prefix sums
    uint32_t base = 0;
    for (uint32_t e0 = 0; e0 < count; e0 += kSelBlock) {
        const uint32_t e = e0 + tid;
        uint64_t d = 0;
        uint32_t i = 0;
        const bool take = e < count && get(e, d, i) && sel_le(d, i, Td, Ti);
        uint32_t pos = 0, tot = 0;
        BlockScan().exclusive_scan(take ? 1u : 0u, pos, 0u, tot, scan_storage);
        if (take && base + pos < kLargeSelMaxK) {
            sh.stage.d[base + pos] = d;
            sh.stage.i[base + pos] = i;
        }
        base += tot;
        __syncthreads();
    }
    const uint32_t sel = min(min(base, k), kLargeSelMaxK);  // k, or every live state when fewer
    for (uint32_t e = sel + tid; e < kLargeSelMaxK; e += kSelBlock) {
        sh.stage.d[e] = ~0ull;
        sh.stage.i[e] = kNoId;
    }
    __syncthreads();
    uint64_t kd[kSelItems];
    uint32_t ki[kSelItems];
#pragma unroll
    for (int j = 0; j < kSelItems; ++j) {
        kd[j] = sh.stage.d[tid * kSelItems + j];
        ki[j] = sh.stage.i[tid * kSelItems + j];
    }
    __syncthreads();
    if (id_sort) {  // block-uniform
        IdSort().sort(ki, kd, sh.id_sort);
        __syncthreads();
    }
    BlockSort().sort(kd, ki, sh.sort);  // stable: equal distances keep id order
#pragma unroll
    for (int j = 0; j < kSelItems; ++j) {
        const uint32_t r = tid * kSelItems + j;
        if (r < k) {
            out_d[(size_t)q * k + r] = r < sel ? __longlong_as_double((long long)kd[j]) : __builtin_inf();
            out_i[(size_t)q * k + r] = r < sel ? ki[j] : kNoId;
        }
    }
}

// a block per query: its candidates' exact fp64 distances computed densely (id order: chunk
// by chunk, slot by slot) into dd / di, then the select + sort over them; or, on a slab
// overflow or a short count, the query goes to the fallback list
template <int SP, int F>
__global__ __launch_bounds__(kSelBlock) void sel_sort_kernel(const double *__restrict__ f64, uint64_t cap,
                                                             const double *__restrict__ aos, int da,
                                                             const double *__restrict__ qf64, DevSpace sp,
                                                             const uint32_t *__restrict__ ci,
                                                             const uint32_t *__restrict__ ov,
                                                             const uint32_t *__restrict__ ov_cnt, uint32_t ovcap,
                                                             const uint32_t *__restrict__ slab_cnt,
                                                             const unsigned int *__restrict__ count_r, uint32_t nq,
                                                             uint32_t chunks, uint32_t slab, uint32_t k,
                                                             double *__restrict__ dd, uint32_t *__restrict__ di,
                                                             double *__restrict__ out_d, uint32_t *__restrict__ out_i,
                                                             uint32_t *__restrict__ fb_count,
                                                             uint32_t *__restrict__ fb_list,
                                                             unsigned long long *__restrict__ stats) {
    using BlockScan = rocprim::block_scan<uint32_t, kSelBlock>;
    __shared__ typename BlockScan::storage_type scan_storage;
    __shared__ uint32_t coff[kSelBlock + 1];  // chunk offsets of the dense order (chunks <= kSelBlock)
    __shared__ uint32_t sh_bad;
    const uint32_t q = blockIdx.x;
    if (q >= nq) return;
    const uint32_t tid = threadIdx.x;
    const uint32_t *cnt = slab_cnt + (size_t)q * chunks;
    const uint32_t c = tid < chunks ? min(cnt[tid], slab) : 0u;  // a slab's overflow is in the pool
    uint32_t pre = 0, tot = 0;
    BlockScan().exclusive_scan(c, pre, 0u, tot, scan_storage);
    const uint32_t nov = ov_cnt[q];
    if (tid == 0) sh_bad = (count_r[q] < k || nov > ovcap) ? 1u : 0u;
    __syncthreads();
    if (tid < chunks) coff[tid] = pre;
    if (tid == 0) coff[chunks] = tot;
    __syncthreads();
    if (stats && tid == 0 && (sh_bad || nov > 0)) atomicAdd(&stats[sh_bad ? 1 : 0], 1ull);
    if (sh_bad) {
        if (tid == 0) fb_list[atomicAdd(fb_count, 1u)] = q;
        return;
    }
    double qv[F];
#pragma unroll
    for (int f = 0; f < F; ++f) qv[f] = qf64[(size_t)q * F + f];
    const size_t sbase = (size_t)q * chunks * slab;
    const size_t dbase = (size_t)q * ((size_t)chunks * slab + ovcap);
    double *qd = dd + dbase;
    uint32_t *qi = di + dbase;
    const uint32_t all = tot + nov;  // dense order: the slabs chunk by chunk (id order), then the pool
    for (uint32_t e = tid; e < all; e += kSelBlock) {
        uint32_t id;
        if (e < tot) {
            uint32_t lo = 0, hi = chunks;  // the chunk holding dense position e: coff[lo] <= e < coff[lo + 1]
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (coff[mid] <= e)
                    lo = mid;
                else
                    hi = mid;
            }
            id = ci[sbase + (size_t)lo * slab + (e - coff[lo])];
        } else {
            id = ov[(size_t)q * ovcap + (e - tot)];
        }
        double sv[F];
        if (aos) {  // one contiguous row per candidate (the raw AoS copy; features = raw coordinates)
#pragma unroll
            for (int f = 0; f < F; ++f) sv[f] = f < sp.dim ? aos[(size_t)id * da + f] : 0.0;
        } else {
#pragma unroll
            for (int f = 0; f < F; ++f) sv[f] = f64[(uint64_t)f * cap + id];
        }
        qd[e] = feat_dist<SP, F, SP == OMPL_GPU_SPACE_KCHAIN ? F / 2 : 0>(sv, qv, sp);
        qi[e] = id;
    }
    __syncthreads();
    auto get = [&](uint32_t e, uint64_t &d, uint32_t &i) -> bool {
        d = (uint64_t)__double_as_longlong(qd[e]);
        i = qi[e];
        return true;
    };
    block_select_sort(get, all, k, q, out_d, out_i, nov > 0);
}

// exact fallback: a block per listed query, the same select over every stored state (each
// radix pass recomputes the exact distances) — slow, for sampling outliers and heavy ties
template <int SP, int F>
__global__ __launch_bounds__(kSelBlock) void sel_fallback_kernel(const double *__restrict__ f64, uint64_t cap,
                                                                 uint64_t n_end, const double *__restrict__ qf64,
                                                                 DevSpace sp, uint32_t k,
                                                                 const uint32_t *__restrict__ fb_count,
                                                                 const uint32_t *__restrict__ fb_list,
                                                                 double *__restrict__ out_d,
                                                                 uint32_t *__restrict__ out_i) {
    const uint32_t n_fb = *fb_count;
    for (uint32_t f = blockIdx.x; f < n_fb; f += gridDim.x) {
        const uint32_t q = fb_list[f];
        double qv[F];
#pragma unroll
        for (int c = 0; c < F; ++c) qv[c] = qf64[(size_t)q * F + c];
        auto get = [&](uint32_t e, uint64_t &d, uint32_t &i) -> bool {
            double sv[F];
#pragma unroll
            for (int c = 0; c < F; ++c) sv[c] = f64[(uint64_t)c * cap + e];
            const double x = feat_dist<SP, F, SP == OMPL_GPU_SPACE_KCHAIN ? F / 2 : 0>(sv, qv, sp);
            if (!(x == x)) return false;  // unused / removed slot
            d = (uint64_t)__double_as_longlong(x);
            i = e;
            return true;
        };
        // live states only: count them once (NaN slots are skipped by get)
        block_select_sort(get, (uint32_t)n_end, k, q, out_d, out_i);
        __syncthreads();
    }
}

struct SelLayout {
    size_t q32, hist, inv, rc, rf, cntr, scnt, fb, ovc, cd, ci, ov, di, total;
    uint32_t chunks, chunk_len, slab, ovcap, qb;
};

inline size_t sel_align(size_t x) { return (x + 255) & ~(size_t)255; }

// queries per batch and slab capacity: the slabs of a batch hold about 1.25 (k + 8 sqrt(8k) +
// 1024) candidates per query spread over the chunks, plus slack for the spread between chunks;
// what a chunk holds beyond its slab goes to the query's pool (as many slots as the estimate)
SelLayout sel_layout(int FS, uint32_t nq, uint32_t k, uint64_t n_end, int num_cus) {
    SelLayout L{};
    Plan p = plan(std::min<uint32_t>(nq, 4096u), n_end, num_cus);
    if (p.chunks > (uint32_t)kSelBlock) {  // sel_sort_kernel scans one chunk count per thread
        const uint64_t tiles = (n_end + kTile - 1) / kTile, per = (tiles + kSelBlock - 1) / kSelBlock;
        p.chunk_len = (uint32_t)(per * kTile);
        p.chunks = (uint32_t)((n_end + p.chunk_len - 1) / p.chunk_len);
    }
    L.chunks = p.chunks;
    L.chunk_len = p.chunk_len;
    const double est = (double)k + 8.0 * std::sqrt(8.0 * k) + 1024.0;
    const double per = 1.25 * est / L.chunks;
    L.slab = (uint32_t)std::ceil(per + 3.0 * std::sqrt(per) + 8.0);
    L.ovcap = (uint32_t)std::ceil(est);
    L.qb = std::min<uint32_t>(nq, 4096u);
    size_t off = 0;
    auto take = [&](size_t b) {
        const size_t o = off;
        off += sel_align(b);
        return o;
    };
    L.q32 = take(4ull * nq * FS);
    L.hist = take(4ull * L.qb * kBins);
    L.inv = take(4ull * L.qb);
    L.rc = take(4ull * L.qb);
    L.rf = take(4ull * L.qb);
    L.cntr = take(4ull * L.qb);
    L.scnt = take(4ull * L.qb * L.chunks);
    L.fb = take(4ull * (L.qb + 1));
    L.ovc = take(4ull * L.qb);
    const size_t dense = (size_t)L.qb * ((size_t)L.chunks * L.slab + L.ovcap);
    L.cd = take(8ull * dense);
    L.ci = take(4ull * L.qb * L.chunks * L.slab);
    L.ov = take(4ull * L.qb * L.ovcap);
    L.di = take(4ull * dense);
    L.total = off;
    return L;
}

template <int SP, int F>
hipError_t run_large_select(const DevSpace &sp, const double *f64, const float *f32, uint64_t cap, uint64_t n_end,
                            const double *aos, int da, const double *qf64, uint32_t nq, uint32_t k, float absmax,
                            float seta, float dmax, double *out_d, uint32_t *out_i, void *ws, size_t ws_bytes,
                            int num_cus, hipStream_t st, unsigned long long *stats) {
    constexpr int FS = Row<SP, F>::FS;
    const SelLayout L = sel_layout(FS, nq, k, n_end, num_cus);
    if (ws_bytes < L.total) return hipErrorInvalidValue;
    char *w = (char *)ws;
    float *q32 = (float *)(w + L.q32), *inv = (float *)(w + L.inv), *rc = (float *)(w + L.rc), *rf = (float *)(w + L.rf);
    unsigned int *hist = (unsigned int *)(w + L.hist), *cntr = (unsigned int *)(w + L.cntr);
    uint32_t *scnt = (uint32_t *)(w + L.scnt), *fb = (uint32_t *)(w + L.fb), *ovc = (uint32_t *)(w + L.ovc);
    uint32_t *ov = (uint32_t *)(w + L.ov);
    double *cd = (double *)(w + L.cd);  // the dense exact distances of each query's candidates
    uint32_t *ci = (uint32_t *)(w + L.ci), *di = (uint32_t *)(w + L.di);
    const float w0 = SP == OMPL_GPU_SPACE_KCHAIN ? (float)sp.link : (float)sp.w0;
    const float bin_a = dmax / (float)kBins;
    hipLaunchKernelGGL((rows32_kernel<SP, F>), dim3((nq + 255) / 256), dim3(256), 0, st, qf64, nq, q32);
    hipError_t e;
    for (uint32_t q0 = 0; q0 < nq; q0 += L.qb) {
        const uint32_t nb = std::min(L.qb, nq - q0);
        const float *bq32 = q32 + (size_t)q0 * FS;
        const double *bqf = qf64 + (size_t)q0 * F;
        const dim3 grid((nb + kTile - 1) / kTile, L.chunks);
        if ((e = hipMemsetAsync(hist, 0, 4ull * nb * kBins, st)) != hipSuccess) return e;
        hipLaunchKernelGGL((hist_sample_kernel<SP, F>), grid, dim3(kTile), 0, st, f32, cap, n_end, bq32, nb,
                           L.chunk_len, kSampleA, w0, (float)sp.w1, sp.dim, (const float *)nullptr, 1.f / bin_a, hist);
        hipLaunchKernelGGL(sel_range_kernel, dim3((nb + 255) / 256), dim3(256), 0, st, hist, nb, k, bin_a, inv);
        if ((e = hipMemsetAsync(hist, 0, 4ull * nb * kBins, st)) != hipSuccess) return e;
        hipLaunchKernelGGL((hist_sample_kernel<SP, F>), grid, dim3(kTile), 0, st, f32, cap, n_end, bq32, nb,
                           L.chunk_len, kSampleB, w0, (float)sp.w1, sp.dim, (const float *)inv, 0.f, hist);
        hipLaunchKernelGGL((sel_radius_kernel<SP, F>), dim3((nb + 255) / 256), dim3(256), 0, st, hist, inv, bqf, nb, k,
                           absmax, seta, sp, rc, rf);
        if ((e = hipMemsetAsync(cntr, 0, 4ull * nb, st)) != hipSuccess) return e;
        if ((e = hipMemsetAsync(ovc, 0, 4ull * nb, st)) != hipSuccess) return e;
        if ((e = hipMemsetAsync(fb, 0, 4, st)) != hipSuccess) return e;
        if (q0 == 0) timer_begin(st, "sel_fill_kernel");
        hipLaunchKernelGGL((sel_fill_kernel<SP, F>), grid, dim3(kTile), 0, st, f32, f64, cap, n_end, bq32, bqf, nb,
                           L.chunk_len, L.chunks, sp, rc, rf, L.slab, L.ovcap, ci, ov, ovc, scnt, cntr);
        if (q0 == 0) timer_end(st);
        hipLaunchKernelGGL((sel_sort_kernel<SP, F>), dim3(nb), dim3(kSelBlock), 0, st, f64, cap, aos, da, bqf, sp, ci,
                           ov, ovc, L.ovcap, scnt, cntr, nb, L.chunks, L.slab, k, cd, di, out_d + (size_t)q0 * k,
                           out_i + (size_t)q0 * k, fb, fb + 1, stats);
        hipLaunchKernelGGL((sel_fallback_kernel<SP, F>), dim3((unsigned)std::max(num_cus, 1)), dim3(kSelBlock), 0, st,
                           f64, cap, n_end, bqf, sp, k, fb, fb + 1, out_d + (size_t)q0 * k, out_i + (size_t)q0 * k);
    }
    return hipGetLastError();
}

}  // namespace

bool large_k_supported(const DevSpace &sp) {
    return sp.kind == OMPL_GPU_SPACE_SE3 || sp.kind == OMPL_GPU_SPACE_SO3 || sp.kind == OMPL_GPU_SPACE_REALVECTOR ||
           sp.kind == OMPL_GPU_SPACE_KCHAIN;
}

size_t knn_large_workspace_bytes(const DevSpace &sp, const FeatGeom &g, uint32_t nq, uint32_t k, uint64_t n_end,
                                 int num_cus) {
    if (nq == 0 || k == 0 || k > kLargeSelMaxK) return 0;
    const int FS = sp.kind == OMPL_GPU_SPACE_SE3 ? 8 : g.F;
    return sel_layout(FS, nq, k, n_end, num_cus).total;
}

hipError_t launch_knn_large(const DevSpace &sp, const FeatGeom &g, const double *feat64, const float *feat32,
                            uint64_t cap, uint64_t n_end, const double *aos, int da, const double *qfeat64, uint32_t nq,
                            uint32_t k, float absmax, float seta, float dmax, double *out_d, uint32_t *out_i,
                            size_t mem_budget, int num_cus, hipStream_t st, void *ws, size_t ws_bytes,
                            unsigned long long *stats) {
    if (nq == 0 || k == 0) return hipSuccess;
    // k <= kLargeSelMaxK: the device-decided select (asynchronous); larger k: count, host offsets, fill
    const bool sel = k <= kLargeSelMaxK && ws && ws_bytes >= knn_large_workspace_bytes(sp, g, nq, k, n_end, num_cus);
#define OMPL_AMD_LARGE(SPK, FK)                                                                                    \
    return sel ? run_large_select<SPK, FK>(sp, feat64, feat32, cap, n_end, SPK == OMPL_GPU_SPACE_KCHAIN ? nullptr \
                                           : aos, da, qfeat64, nq, k, absmax, seta, dmax, out_d, out_i, ws,        \
                                           ws_bytes, num_cus, st, stats)                                           \
               : run_large<SPK, FK>(sp, feat64, feat32, cap, n_end, qfeat64, nq, k, absmax, seta, dmax, out_d,     \
                                    out_i, mem_budget, num_cus, st)
    switch (sp.kind) {
    case OMPL_GPU_SPACE_SE3:
        OMPL_AMD_LARGE(OMPL_GPU_SPACE_SE3, 7);
    case OMPL_GPU_SPACE_SO3:
        OMPL_AMD_LARGE(OMPL_GPU_SPACE_SO3, 4);
    case OMPL_GPU_SPACE_REALVECTOR:
        if (g.F == 4) OMPL_AMD_LARGE(OMPL_GPU_SPACE_REALVECTOR, 4);
        if (g.F == 8) OMPL_AMD_LARGE(OMPL_GPU_SPACE_REALVECTOR, 8);
        OMPL_AMD_LARGE(OMPL_GPU_SPACE_REALVECTOR, 16);
    case OMPL_GPU_SPACE_KCHAIN:  // features: cos / sin of the cumulative angles, nmax links each
        if (g.nmax == 4) OMPL_AMD_LARGE(OMPL_GPU_SPACE_KCHAIN, 8);
        if (g.nmax == 8) OMPL_AMD_LARGE(OMPL_GPU_SPACE_KCHAIN, 16);
        if (g.nmax == 12) OMPL_AMD_LARGE(OMPL_GPU_SPACE_KCHAIN, 24);
        if (g.nmax == 16) OMPL_AMD_LARGE(OMPL_GPU_SPACE_KCHAIN, 32);
        return hipErrorInvalidValue;
    }
#undef OMPL_AMD_LARGE
    return hipErrorInvalidValue;
}

}  // namespace ompl_amd
