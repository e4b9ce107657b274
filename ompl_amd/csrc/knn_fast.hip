// knn_fast.hip — exact batched kNN via an fp32 screen and an fp64 certificate (gfx950).
//
// The reference ranks in fp64 (NearestNeighborsGNAT.h:544-558 on
// StateSpace::distance).  fp64 VALU issues at half the fp32 rate on CDNA4 and the fp64
// sqrt / acos expansions are long, so the scan runs in fp32 and fp64 is spent only on a
// short candidate list:
//
//   1. queries are ordered along a Morton curve of their first three coordinates (for SE3
//      the translation), so the 64 queries of a wave are spatial neighbours;
//   2. screen (fp32): one thread per query, 256-state LDS tiles read by broadcast, a
//      register list of the K2 > k smallest fp32 distances; for SE3 the translation part
//      is computed first and the rotation (acos) only where sqrt(t) can still beat the
//      list's K2-th distance — with spatially ordered queries that branch is coherent
//      across the wave, so most (wave, state) pairs cost 3 sub + 3 fma + 1 compare;
//   3. certify (fp64): merge the chunk lists, recompute the K2 candidates exactly in the
//      reference's operation order, keep the k best by (distance, id), and prove that no
//      element outside the list can enter: |d32 - d64| <= e for every element, so if the
//      exact k-th distance + e < the list's K2-th fp32 distance L the answer is exact.
//      Queries that fail the proof are appended to a list the caller re-runs on the exact
//      fp64 path (knn.hip), so results are always identical to the exact path.
//
// Error bound e (u = 2^-24, B = max |coordinate|, D = dims, L as above), doubled for slack:
//   translation / R^n : 6 sqrt(D) u B + 6 u L   (fp32 conversion + sum of squares + sqrt)
//   rotation          : 1.1 sqrt(2 * 6u) + 1e-6 + 4.5e-5
//                       (|dot32 - dot| <= 6u; acos is 1/2-Hoelder near 1; the reference
//                        returns 0 for dot > 1 - 1e-9, SO3StateSpace.cpp:258-260)
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>

#include "feat_dist.h"
#include "kernels.h"
#include "topk.h"

namespace ompl_amd {

namespace {

constexpr double kU = 5.9604644775390625e-08;  // 2^-24

template <int SP, int F>
struct Screen {  // fp32 row width in LDS / query rows
    static constexpr int FS = SP == OMPL_GPU_SPACE_SE3 ? 8 : F;
};

__device__ __forceinline__ uint32_t spread3(uint32_t x) {
    x &= 0x3ffu;
    x = (x | (x << 16)) & 0x030000FFu;
    x = (x | (x << 8)) & 0x0300F00Fu;
    x = (x | (x << 4)) & 0x030C30C3u;
    x = (x | (x << 2)) & 0x09249249u;
    return x;
}

__global__ void morton_kernel(const double *__restrict__ qf, int F, int ncoord, uint32_t nq, FastBounds b,
                              uint32_t *__restrict__ keys, uint32_t *__restrict__ idx) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nq) return;
    uint32_t key = 0;
    for (int c = 0; c < ncoord; ++c) {
        float t = ((float)qf[(size_t)i * F + c] - b.lo[c]) * b.inv[c];
        t = t > 0.f ? (t < 1023.f ? t : 1023.f) : 0.f;  // NaN -> 0
        key |= spread3((uint32_t)t) << c;
    }
    keys[i] = key;
    idx[i] = i;
}

template <int SP, int F>
__global__ void query32_kernel(const double *__restrict__ qf, const uint32_t *__restrict__ perm, uint32_t nq,
                               float *__restrict__ q32) {
    constexpr int FS = Screen<SP, F>::FS;
    const uint32_t qs = blockIdx.x * blockDim.x + threadIdx.x;
    if (qs >= nq) return;
    const double *s = qf + (size_t)perm[qs] * F;
    float *o = q32 + (size_t)qs * FS;
    if constexpr (SP == OMPL_GPU_SPACE_SE3) {
        o[0] = (float)s[0]; o[1] = (float)s[1]; o[2] = (float)s[2]; o[3] = 0.f;
        o[4] = (float)s[3]; o[5] = (float)s[4]; o[6] = (float)s[5]; o[7] = (float)s[6];
    } else {
        for (int f = 0; f < FS; ++f) o[f] = (float)s[f];
    }
}

__device__ __forceinline__ float clamp_abs1(float x) {  // |x| clamped to 1; NaN stays NaN
    float a = fabsf(x);
    return a > 1.f ? 1.f : a;
}

template <int SP, int F, int K2>
__global__ __launch_bounds__(256) void knn32_screen_kernel(const float *__restrict__ f32, uint64_t cap,
                                                           uint64_t n_end, const float *__restrict__ q32,
                                                           uint32_t nq, uint32_t chunk_len, float w0, float w1,
                                                           float *__restrict__ pd, uint32_t *__restrict__ pi) {
    constexpr int FS = Screen<SP, F>::FS;
    __shared__ __attribute__((aligned(16))) float tile[kTile * FS];
    const uint32_t qs = blockIdx.x * kTile + threadIdx.x;
    float qf[FS];
#pragma unroll
    for (int f = 0; f < FS; ++f) qf[f] = qs < nq ? q32[(size_t)qs * FS + f] : __builtin_nanf("");
    const float w0sq = w0 * w0;
    TopK32<K2> top;
    top.init();
    const uint64_t c0 = (uint64_t)blockIdx.y * chunk_len;
    const uint64_t c1 = min(c0 + chunk_len, n_end);
    for (uint64_t base = c0; base < c1; base += kTile) {
        const uint64_t g = base + threadIdx.x;
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
        __syncthreads();
#pragma unroll 4
        for (int s = 0; s < kTile; ++s) {
            const uint32_t id = (uint32_t)(base + s);
            if constexpr (SP == OMPL_GPU_SPACE_SE3) {
                const float4 a = reinterpret_cast<const float4 *>(tile)[s * 2];
                const float dx = a.x - qf[0], dy = a.y - qf[1], dz = a.z - qf[2];
                float t = dx * dx;
                t = fmaf(dy, dy, t);
                t = fmaf(dz, dz, t);
                if (t * w0sq < top.tau2) {
                    const float4 r = reinterpret_cast<const float4 *>(tile)[s * 2 + 1];
                    float dot = r.x * qf[4];
                    dot = fmaf(r.y, qf[5], dot);
                    dot = fmaf(r.z, qf[6], dot);
                    dot = fmaf(r.w, qf[7], dot);
                    const float d = w0 * sqrtf(t) + w1 * acosf(clamp_abs1(dot));
                    if (top.admits(d, id)) top.push(d, id);
                }
            } else if constexpr (SP == OMPL_GPU_SPACE_SO3) {
                const float4 r = reinterpret_cast<const float4 *>(tile)[s];
                float dot = r.x * qf[0];
                dot = fmaf(r.y, qf[1], dot);
                dot = fmaf(r.z, qf[2], dot);
                dot = fmaf(r.w, qf[3], dot);
                const float d = acosf(clamp_abs1(dot));
                if (top.admits(d, id)) top.push(d, id);
            } else {
                float acc = 0.f;
#pragma unroll
                for (int f = 0; f < FS; ++f) {
                    const float diff = tile[s * FS + f] - qf[f];
                    acc = fmaf(diff, diff, acc);
                }
                if (acc < top.tau2) {
                    const float d = sqrtf(acc);
                    if (top.admits(d, id)) top.push(d, id);
                }
            }
        }
        __syncthreads();
    }
    if (qs >= nq) return;
    const size_t o = ((size_t)blockIdx.y * nq + qs) * K2;
#pragma unroll
    for (int j = 0; j < K2; ++j) {
        pd[o + j] = top.d[j];
        pi[o + j] = top.i[j];
    }
}

template <int SP>
__device__ __forceinline__ double screen_error(const DevSpace &sp, double B, double L) {
    double e = 0.0;
    if constexpr (SP == OMPL_GPU_SPACE_SE3) {
        e = sp.w0 * (6.0 * 1.7320508075688772 * kU * B) + 6.0 * kU * L +
            sp.w1 * (1.1 * sqrt(12.0 * kU) + 1e-6 + 4.5e-5);
    } else if constexpr (SP == OMPL_GPU_SPACE_SO3) {
        e = 1.1 * sqrt(12.0 * kU) + 1e-6 + 4.5e-5;
    } else {
        e = 6.0 * sqrt((double)sp.dim) * kU * B + 6.0 * kU * L;
    }
    return 2.0 * e;
}

template <int SP, int F, int K2, int K>
__global__ __launch_bounds__(256) void knn_certify_kernel(const float *__restrict__ pd, const uint32_t *__restrict__ pi,
                                                          uint32_t S, uint32_t nq, const uint32_t *__restrict__ perm,
                                                          const double *__restrict__ feat64, uint64_t cap,
                                                          const double *__restrict__ qf64, DevSpace sp,
                                                          float absmax, double *__restrict__ out_d,
                                                          uint32_t *__restrict__ out_i, uint32_t out_k,
                                                          uint32_t *__restrict__ fail_count,
                                                          uint32_t *__restrict__ fail_list) {
    const uint32_t qs = blockIdx.x * blockDim.x + threadIdx.x;
    if (qs >= nq) return;
    TopK32<K2> t;
    t.init();
    for (uint32_t s = 0; s < S; ++s) {
        const size_t o = ((size_t)s * nq + qs) * K2;
        for (int j = 0; j < K2; ++j) {
            const float d = pd[o + j];
            const uint32_t id = pi[o + j];
            if (!t.admits(d, id)) break;  // chunk lists are sorted
            t.push(d, id);
        }
    }
    const uint32_t q = perm[qs];
    double qv[F];
#pragma unroll
    for (int f = 0; f < F; ++f) qv[f] = qf64[(size_t)q * F + f];
    TopK<K> ex;
    ex.init();
#pragma unroll
    for (int j = 0; j < K2; ++j) {
        const uint32_t id = t.i[j];
        if (id != kNoId) {
            double sv[F];
#pragma unroll
            for (int f = 0; f < F; ++f) sv[f] = feat64[(uint64_t)f * cap + id];
            ex.offer(feat_dist<SP, F, 0>(sv, qv, sp), id);  // reference formula, fp64
        }
    }
    bool ok = true;
    if (t.i[K2 - 1] != kNoId) {  // the list is full: elements were excluded, prove none can enter
        double B = absmax;
        const int nc = SP == OMPL_GPU_SPACE_SE3 ? 3 : (SP == OMPL_GPU_SPACE_SO3 ? 0 : F);
        for (int c = 0; c < nc; ++c) B = fmax(B, fabs(qv[c]));
        const double L = (double)t.d[K2 - 1];
        double dk = ex.d[K - 1];
#pragma unroll
        for (int j = 0; j < K; ++j)
            if (j == (int)out_k - 1) dk = ex.d[j];
        ok = dk + screen_error<SP>(sp, B, L) < L * (1.0 - 8.0 * kU);
    }
#pragma unroll
    for (int j = 0; j < K; ++j)
        if (j < (int)out_k) {
            out_d[(size_t)q * out_k + j] = ex.d[j];
            out_i[(size_t)q * out_k + j] = ex.i[j];
        }
    if (!ok) fail_list[atomicAdd(fail_count, 1u)] = q;
}

__global__ void to_fp32_kernel(const double *__restrict__ f64, uint64_t cap, int rows, uint64_t first, uint64_t n,
                               float *__restrict__ f32) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * rows) return;
    const uint64_t r = t / n, i = first + t % n;
    f32[r * cap + i] = (float)f64[r * cap + i];
}

__global__ void gather_rows_kernel(const double *__restrict__ src, int F, const uint32_t *__restrict__ list,
                                   uint32_t n, double *__restrict__ dst) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * (uint32_t)F) return;
    const uint32_t i = t / F, f = t % F;
    dst[t] = src[(size_t)list[i] * F + f];
}

__global__ void scatter_results_kernel(const double *__restrict__ d, const uint32_t *__restrict__ ids, uint32_t k,
                                       const uint32_t *__restrict__ list, uint32_t n, double *__restrict__ out_d,
                                       uint32_t *__restrict__ out_i) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * k) return;
    const uint32_t i = t / k, j = t % k;
    out_d[(size_t)list[i] * k + j] = d[t];
    out_i[(size_t)list[i] * k + j] = ids[t];
}

struct FastPlan {
    int K2, K;
    uint32_t chunks, chunk_len;
};

FastPlan fast_plan(const DevSpace &sp, uint32_t nq, uint32_t k, uint64_t n_end, int num_cus) {
    FastPlan p{};
    p.K2 = fast_k2(sp, k, nq);
    p.K = k_bucket(k);
    const uint64_t tiles = std::max<uint64_t>(n_end / kTile, 1);
    const uint64_t qblocks = (nq + kTile - 1) / kTile;
    const uint64_t target = (uint64_t)num_cus * 8;
    uint64_t S = std::max<uint64_t>(1, std::min<uint64_t>((target + qblocks - 1) / qblocks, tiles));
    const uint64_t per = (tiles + S - 1) / S;
    p.chunk_len = (uint32_t)(per * kTile);
    p.chunks = (uint32_t)((n_end + p.chunk_len - 1) / p.chunk_len);
    return p;
}

inline size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

struct FastLayout {
    size_t keys, keys2, idx, perm, cub, q32, pd, pi, fail, total;
    size_t cub_bytes;
};

FastLayout fast_layout(const DevSpace &sp, const FeatGeom &g, const FastPlan &p, uint32_t nq) {
    FastLayout L{};
    size_t off = 0;
    auto take = [&](size_t b) {
        size_t o = off;
        off += align_up(b);
        return o;
    };
    L.keys = take(4ull * nq);
    L.keys2 = take(4ull * nq);
    L.idx = take(4ull * nq);
    L.perm = take(4ull * nq);
    size_t cb = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, cb, (uint32_t *)nullptr, (uint32_t *)nullptr,
                                             (uint32_t *)nullptr, (uint32_t *)nullptr, (int)nq, 0, 30);
    L.cub_bytes = cb;
    L.cub = take(cb);
    const int FS = sp.kind == OMPL_GPU_SPACE_SE3 ? 8 : g.F;
    L.q32 = take(4ull * nq * FS);
    L.pd = take(4ull * p.chunks * nq * p.K2);
    L.pi = take(4ull * p.chunks * nq * p.K2);
    L.fail = take(4ull * (nq + 1));
    L.total = off;
    return L;
}

template <int SP, int F, int K2, int K>
hipError_t run_fast(const DevSpace &sp, const FastPlan &p, const FastLayout &L, char *ws, const float *f32,
                    const double *f64, uint64_t cap, uint64_t n_end, const double *qf64, uint32_t nq, uint32_t k,
                    const FastBounds &b, double *od, uint32_t *oi, hipStream_t st) {
    uint32_t *keys = (uint32_t *)(ws + L.keys), *keys2 = (uint32_t *)(ws + L.keys2);
    uint32_t *idx = (uint32_t *)(ws + L.idx), *perm = (uint32_t *)(ws + L.perm);
    float *q32 = (float *)(ws + L.q32);
    float *pd = (float *)(ws + L.pd);
    uint32_t *pi = (uint32_t *)(ws + L.pi);
    uint32_t *fail = (uint32_t *)(ws + L.fail);
    const int ncoord = SP == OMPL_GPU_SPACE_SO3 ? 0 : std::min(F, 3);
    const dim3 b256(256);
    hipLaunchKernelGGL(morton_kernel, dim3((nq + 255) / 256), b256, 0, st, qf64, F, ncoord, nq, b, keys, idx);
    size_t cb = L.cub_bytes;
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(ws + L.cub, cb, keys, keys2, idx, perm, (int)nq, 0, 30, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((query32_kernel<SP, F>), dim3((nq + 255) / 256), b256, 0, st, qf64, perm, nq, q32);
    e = hipMemsetAsync(fail, 0, 4, st);
    if (e != hipSuccess) return e;
    const dim3 grid((nq + kTile - 1) / kTile, p.chunks);
    timer_begin(st, "knn32_screen_kernel");
    hipLaunchKernelGGL((knn32_screen_kernel<SP, F, K2>), grid, dim3(kTile), 0, st, f32, cap, n_end, q32, nq,
                       p.chunk_len, (float)sp.w0, (float)sp.w1, pd, pi);
    timer_end(st);
    hipLaunchKernelGGL((knn_certify_kernel<SP, F, K2, K>), dim3((nq + 255) / 256), b256, 0, st, pd, pi, p.chunks, nq,
                       perm, f64, cap, qf64, sp, b.absmax, od, oi, k, fail, fail + 1);
    return hipGetLastError();
}

template <int SP, int F, int K2>
hipError_t run_fast_k(const DevSpace &sp, const FastPlan &p, const FastLayout &L, char *ws, const float *f32,
                      const double *f64, uint64_t cap, uint64_t n_end, const double *qf64, uint32_t nq, uint32_t k,
                      const FastBounds &b, double *od, uint32_t *oi, hipStream_t st) {
    switch (p.K) {
    case 1: return run_fast<SP, F, K2, 1>(sp, p, L, ws, f32, f64, cap, n_end, qf64, nq, k, b, od, oi, st);
    case 4: return run_fast<SP, F, K2, 4>(sp, p, L, ws, f32, f64, cap, n_end, qf64, nq, k, b, od, oi, st);
    case 16: return run_fast<SP, F, K2, 16>(sp, p, L, ws, f32, f64, cap, n_end, qf64, nq, k, b, od, oi, st);
    case 32:
        if constexpr (K2 >= 32) return run_fast<SP, F, K2, 32>(sp, p, L, ws, f32, f64, cap, n_end, qf64, nq, k, b, od, oi, st);
    }
    return hipErrorInvalidValue;
}

template <int SP, int F>
hipError_t run_fast_space(const DevSpace &sp, const FastPlan &p, const FastLayout &L, char *ws, const float *f32,
                          const double *f64, uint64_t cap, uint64_t n_end, const double *qf64, uint32_t nq,
                          uint32_t k, const FastBounds &b, double *od, uint32_t *oi, hipStream_t st) {
    switch (p.K2) {
    case 16: return run_fast_k<SP, F, 16>(sp, p, L, ws, f32, f64, cap, n_end, qf64, nq, k, b, od, oi, st);
    case 32: return run_fast_k<SP, F, 32>(sp, p, L, ws, f32, f64, cap, n_end, qf64, nq, k, b, od, oi, st);
    case 64: return run_fast_k<SP, F, 64>(sp, p, L, ws, f32, f64, cap, n_end, qf64, nq, k, b, od, oi, st);
    }
    return hipErrorInvalidValue;
}

}  // namespace

// K2: the smallest list bucket >= max(k + 6, 16); the certify kernel's K bucket fits inside it.
int fast_k2(const DevSpace &sp, uint32_t k, uint32_t nq) {
    if (sp.kind == OMPL_GPU_SPACE_KCHAIN || nq < kStreamMaxQ || k == 0) return 0;
    const int K = k_bucket(k);
    if (K == 0 || K > 32) return 0;  // the exact path serves k > 32
    int K2 = k_bucket(k + 6);
    if (K2 < 16) K2 = 16;
    if (K2 == 0 || K2 < K) return 0;
    return K2;
}

int fp32_rows(const DevSpace &sp, const FeatGeom &g) { return sp.kind == OMPL_GPU_SPACE_KCHAIN ? 0 : g.F; }

size_t knn_fast_workspace_bytes(const DevSpace &sp, const FeatGeom &g, uint32_t nq, uint32_t k, uint64_t n_end,
                                int num_cus) {
    const FastPlan p = fast_plan(sp, nq, k, n_end, num_cus);
    if (p.K2 == 0) return 0;
    return fast_layout(sp, g, p, nq).total;
}

hipError_t launch_knn_fast(const DevSpace &sp, const FeatGeom &g, const double *feat64, const float *feat32,
                           uint64_t cap, uint64_t n_end, const double *qfeat64, uint32_t nq, uint32_t k,
                           const FastBounds &b, double *out_d, uint32_t *out_i, void *ws, size_t ws_bytes,
                           int num_cus, hipStream_t st, uint32_t **fail_count, uint32_t **fail_list) {
    const FastPlan p = fast_plan(sp, nq, k, n_end, num_cus);
    if (p.K2 == 0) return hipErrorInvalidValue;
    const FastLayout L = fast_layout(sp, g, p, nq);
    if (L.total > ws_bytes) return hipErrorInvalidValue;
    char *w = (char *)ws;
    *fail_count = (uint32_t *)(w + L.fail);
    *fail_list = *fail_count + 1;
    switch (sp.kind) {
    case OMPL_GPU_SPACE_SE3:
        return run_fast_space<OMPL_GPU_SPACE_SE3, 7>(sp, p, L, w, feat32, feat64, cap, n_end, qfeat64, nq, k, b,
                                                      out_d, out_i, st);
    case OMPL_GPU_SPACE_SO3:
        return run_fast_space<OMPL_GPU_SPACE_SO3, 4>(sp, p, L, w, feat32, feat64, cap, n_end, qfeat64, nq, k, b,
                                                      out_d, out_i, st);
    case OMPL_GPU_SPACE_REALVECTOR:
        if (g.F == 4)
            return run_fast_space<OMPL_GPU_SPACE_REALVECTOR, 4>(sp, p, L, w, feat32, feat64, cap, n_end, qfeat64, nq,
                                                                 k, b, out_d, out_i, st);
        if (g.F == 8)
            return run_fast_space<OMPL_GPU_SPACE_REALVECTOR, 8>(sp, p, L, w, feat32, feat64, cap, n_end, qfeat64, nq,
                                                                 k, b, out_d, out_i, st);
        return run_fast_space<OMPL_GPU_SPACE_REALVECTOR, 16>(sp, p, L, w, feat32, feat64, cap, n_end, qfeat64, nq, k,
                                                              b, out_d, out_i, st);
    }
    return hipErrorInvalidValue;
}

hipError_t launch_to_fp32(const double *feat64, uint64_t cap, int rows, uint64_t first, uint64_t n, float *feat32,
                          hipStream_t st) {
    if (n == 0 || rows == 0) return hipSuccess;
    const uint64_t t = n * rows;
    hipLaunchKernelGGL(to_fp32_kernel, dim3((unsigned)((t + 255) / 256)), dim3(256), 0, st, feat64, cap, rows, first,
                       n, feat32);
    return hipGetLastError();
}

hipError_t launch_gather_rows(const double *src, int F, const uint32_t *list, uint32_t n, double *dst, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(gather_rows_kernel, dim3((n * F + 255) / 256), dim3(256), 0, st, src, F, list, n, dst);
    return hipGetLastError();
}

hipError_t launch_scatter_results(const double *d, const uint32_t *ids, uint32_t k, const uint32_t *list, uint32_t n,
                                  double *out_d, uint32_t *out_i, hipStream_t st) {
    if (n == 0 || k == 0) return hipSuccess;
    hipLaunchKernelGGL(scatter_results_kernel, dim3((n * k + 255) / 256), dim3(256), 0, st, d, ids, k, list, n, out_d,
                       out_i);
    return hipGetLastError();
}

}  // namespace ompl_amd
