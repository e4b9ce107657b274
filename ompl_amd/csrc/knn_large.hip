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
#include <hipcub/hipcub.hpp>

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
        float dot = s[4] * q[4];
        dot = fmaf(s[5], q[5], dot);
        dot = fmaf(s[6], q[6], dot);
        dot = fmaf(s[7], q[7], dot);
        return w0 * sqrtf(t) + w1 * acosf(abs1(dot));
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

template <int SP>
__device__ __forceinline__ double screen_err(const DevSpace &sp, double B, double L) {
    double e;
    if constexpr (SP == OMPL_GPU_SPACE_SE3)
        e = sp.w0 * (6.0 * 1.7320508075688772 * kU * B) + 6.0 * kU * L + sp.w1 * (1.1 * sqrt(12.0 * kU) + 1e-6 + 4.5e-5);
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
                                 uint32_t k, float bin_w, float absmax, DevSpace sp, float *__restrict__ radius) {
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
    const double e = screen_err<SP>(sp, B, r_hi + 1.0);
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
                     const double *qf64, uint32_t nq, uint32_t k, float absmax, float dmax, double *out_d,
                     uint32_t *out_i, size_t mem_budget, int num_cus, hipStream_t st) {
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
                       absmax, sp, radius);
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
        size_t tb = 0;
        TRYB(hipcub::DeviceSegmentedRadixSort::SortPairs(nullptr, tb, cd, sd, ci, si, (int)run, (int)nqb, d_seg,
                                                          d_seg + 1, 0, 64, st));
        TRYB(hipMalloc(&tmp, std::max<size_t>(tb, 1)));
        TRYB(hipcub::DeviceSegmentedRadixSort::SortPairs(tmp, tb, cd, sd, ci, si, (int)run, (int)nqb, d_seg,
                                                          d_seg + 1, 0, 64, st));
        const uint64_t nout = (uint64_t)nqb * k;
        hipLaunchKernelGGL(take_first_k_kernel, dim3((unsigned)((nout + 255) / 256)), dim3(256), 0, st, sd, si, d_seg,
                           q0, nqb, k, out_d, out_i);
        TRYB(hipStreamSynchronize(st));
        free_batch();
#undef TRYB
        q0 = q1;
    }
    cleanup();
#undef TRYL
    return hipGetLastError();
}

}  // namespace

bool large_k_supported(const DevSpace &sp) {
    return sp.kind == OMPL_GPU_SPACE_SE3 || sp.kind == OMPL_GPU_SPACE_SO3 || sp.kind == OMPL_GPU_SPACE_REALVECTOR ||
           sp.kind == OMPL_GPU_SPACE_KCHAIN;
}

hipError_t launch_knn_large(const DevSpace &sp, const FeatGeom &g, const double *feat64, const float *feat32,
                            uint64_t cap, uint64_t n_end, const double *qfeat64, uint32_t nq, uint32_t k, float absmax,
                            float dmax, double *out_d, uint32_t *out_i, size_t mem_budget, int num_cus,
                            hipStream_t st) {
    if (nq == 0 || k == 0) return hipSuccess;
    switch (sp.kind) {
    case OMPL_GPU_SPACE_SE3:
        return run_large<OMPL_GPU_SPACE_SE3, 7>(sp, feat64, feat32, cap, n_end, qfeat64, nq, k, absmax, dmax, out_d,
                                                 out_i, mem_budget, num_cus, st);
    case OMPL_GPU_SPACE_SO3:
        return run_large<OMPL_GPU_SPACE_SO3, 4>(sp, feat64, feat32, cap, n_end, qfeat64, nq, k, absmax, dmax, out_d,
                                                 out_i, mem_budget, num_cus, st);
    case OMPL_GPU_SPACE_REALVECTOR:
        if (g.F == 4)
            return run_large<OMPL_GPU_SPACE_REALVECTOR, 4>(sp, feat64, feat32, cap, n_end, qfeat64, nq, k, absmax,
                                                            dmax, out_d, out_i, mem_budget, num_cus, st);
        if (g.F == 8)
            return run_large<OMPL_GPU_SPACE_REALVECTOR, 8>(sp, feat64, feat32, cap, n_end, qfeat64, nq, k, absmax,
                                                            dmax, out_d, out_i, mem_budget, num_cus, st);
        return run_large<OMPL_GPU_SPACE_REALVECTOR, 16>(sp, feat64, feat32, cap, n_end, qfeat64, nq, k, absmax, dmax,
                                                         out_d, out_i, mem_budget, num_cus, st);
    case OMPL_GPU_SPACE_KCHAIN:  // features: cos / sin of the cumulative angles, nmax links each
#define OMPL_AMD_LARGE_CHAIN(NMX)                                                                                  \
    if (g.nmax == NMX)                                                                                             \
        return run_large<OMPL_GPU_SPACE_KCHAIN, 2 * NMX>(sp, feat64, feat32, cap, n_end, qfeat64, nq, k, absmax, dmax, \
                                                         out_d, out_i, mem_budget, num_cus, st);
        OMPL_AMD_LARGE_CHAIN(4)
        OMPL_AMD_LARGE_CHAIN(8)
        OMPL_AMD_LARGE_CHAIN(12)
        OMPL_AMD_LARGE_CHAIN(16)
#undef OMPL_AMD_LARGE_CHAIN
        return hipErrorInvalidValue;
    }
    return hipErrorInvalidValue;
}

}  // namespace ompl_amd
