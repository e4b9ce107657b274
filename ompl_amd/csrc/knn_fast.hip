// knn_fast.hip — exact batched kNN via an fp32 screen and an fp64 certificate (gfx950).
//
// The reference ranks in fp64 (NearestNeighborsGNAT.h:544-558 on StateSpace::distance).
// fp64 VALU issues at half the fp32 rate on CDNA4 and the fp64 sqrt / acos expansions
// are long, so the scan runs in fp32 and fp64 is spent only on a short candidate list:
//
//   1. queries are ordered along a Morton curve (SE3: translation; R^n: first <= 6 dims)
//      so the 64 queries of a wave are spatial neighbours;
//   2. screen (fp32), one thread per query, register list of the K2 > k smallest fp32
//      distances.  Two variants:
//        culled (SE3, R^n): the store is kept in a Morton-sorted copy with 64-state tiles
//          and 2048-state super-tiles carrying boxes of the Euclidean part of the metric;
//          a wave walks super-tiles outward from its own position on the curve and skips
//          every (super-)tile whose box is farther than each lane's current K2-th
//          distance (a lower bound: the SO3 part of an SE3 distance is >= 0);
//        chunked (SO3): the whole store, split in chunks along grid.y.
//      Inside a tile, for SE3 the translation part is computed first and the rotation
//      (acos) only where sqrt(t) can still beat the K2-th distance: with spatially
//      ordered queries that branch is coherent across the wave.
//   3. certify (fp64): merge the lists, recompute the K2 candidates exactly in the
//      reference's operation order, keep the k best by (distance, id), and prove that no
//      element outside the list can enter: |d32 - d64| <= e for every element, so if the
//      exact k-th distance + e < the list's K2-th fp32 distance L the answer is exact.
//      Queries that fail the proof are listed; the caller re-runs them on the exact fp64
//      path (knn.hip), so the results always equal the exact path's.
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
struct Geo {
    static constexpr int FS = SP == OMPL_GPU_SPACE_SE3 ? 8 : F;  // fp32 row width (LDS / queries)
    static constexpr int NB = SP == OMPL_GPU_SPACE_SE3 ? 3 : F;  // box dims (Euclidean part)
    static constexpr int R = SP == OMPL_GPU_SPACE_SE3 ? 7 : F;   // rows of the fp32 SoA store
};

__device__ __forceinline__ float abs1(float x) {  // |x| clamped to 1; NaN stays NaN
    float a = fabsf(x);
    return a > 1.f ? 1.f : a;
}

// 30-bit Morton key of a fp32 row (SE3 row layout x y z . qx qy qz qw); NaN -> max key
__device__ __forceinline__ uint32_t morton_key(const float *c, const FastBounds &b) {
    if (!(c[0] == c[0])) return 0xFFFFFFFFu;
    const int D = b.nkey;
    if (D <= 0) return 0u;
    const int bits = 30 / D;
    const float scale = (float)((1u << bits) - 1u);
    uint32_t v[kKeyDims];
    for (int d = 0; d < D; ++d) {
        float t = (c[d] - b.lo[d]) * b.inv[d] * scale;
        t = t > 0.f ? (t < scale ? t : scale) : 0.f;
        v[d] = (uint32_t)t;
    }
    uint32_t key = 0;
    for (int bit = bits - 1; bit >= 0; --bit)
        for (int d = 0; d < D; ++d) key = (key << 1) | ((v[d] >> bit) & 1u);
    return key;
}

// ---- queries: fp32 rows, keys, order ---------------------------------------------------
template <int SP, int F>
__global__ void query_rows_kernel(const double *__restrict__ qf, uint32_t nq, FastBounds b, float *__restrict__ q32u,
                                  uint32_t *__restrict__ keys, uint32_t *__restrict__ idx) {
    constexpr int FS = Geo<SP, F>::FS;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nq) return;
    const double *s = qf + (size_t)i * F;
    float o[FS];
    if constexpr (SP == OMPL_GPU_SPACE_SE3) {
        o[0] = (float)s[0]; o[1] = (float)s[1]; o[2] = (float)s[2]; o[3] = 0.f;
        o[4] = (float)s[3]; o[5] = (float)s[4]; o[6] = (float)s[5]; o[7] = (float)s[6];
    } else {
        for (int f = 0; f < FS; ++f) o[f] = (float)s[f];
    }
    for (int f = 0; f < FS; ++f) q32u[(size_t)i * FS + f] = o[f];
    keys[i] = morton_key(o, b);
    idx[i] = i;
}

template <int FS>
__global__ void query_gather_kernel(const float *__restrict__ q32u, const uint32_t *__restrict__ perm, uint32_t nq,
                                    float *__restrict__ q32) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nq * (uint32_t)FS) return;
    const uint32_t qs = t / FS, f = t % FS;
    q32[t] = q32u[(size_t)perm[qs] * FS + f];
}

// ---- sorted store (culled screen) ----------------------------------------------------------
template <int SP, int F>
__global__ void tree_key_kernel(const float *__restrict__ f32, uint64_t cap, uint32_t n, FastBounds b,
                                uint32_t *__restrict__ keys, uint32_t *__restrict__ ids) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float c[kKeyDims];
    const int D = b.nkey;
    for (int d = 0; d < D; ++d) c[d] = f32[(uint64_t)d * cap + i];
    keys[i] = D > 0 ? morton_key(c, b) : (c[0] == c[0] ? 0u : 0xFFFFFFFFu);
    ids[i] = i;
}

template <int SP, int F>
__global__ void tree_gather_kernel(const float *__restrict__ f32, uint64_t cap, const uint32_t *__restrict__ ids_sorted,
                                   uint32_t n, uint32_t n_pad, float *__restrict__ rows, uint32_t *__restrict__ ids) {
    constexpr int R = Geo<SP, F>::R;
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n_pad) return;
    if (p < n) {
        const uint32_t id = ids_sorted[p];
        for (int r = 0; r < R; ++r) rows[(size_t)r * n_pad + p] = f32[(uint64_t)r * cap + id];
        ids[p] = id;
    } else {
        for (int r = 0; r < R; ++r) rows[(size_t)r * n_pad + p] = __builtin_nanf("");
        ids[p] = kNoId;
    }
}

template <int SP, int F>
__global__ void tile_box_kernel(const float *__restrict__ rows, uint32_t n_pad, uint32_t ntiles,
                                const uint32_t *__restrict__ keys_sorted, uint32_t n, float *__restrict__ tbox,
                                uint32_t *__restrict__ tkey0) {
    constexpr int NB = Geo<SP, F>::NB;
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntiles) return;
    float lo[NB], hi[NB];
    for (int c = 0; c < NB; ++c) {
        lo[c] = __builtin_inff();
        hi[c] = -__builtin_inff();
    }
    for (int j = 0; j < kCullTile; ++j) {
        const uint32_t p = t * kCullTile + j;
        for (int c = 0; c < NB; ++c) {
            const float v = rows[(size_t)c * n_pad + p];
            if (v == v) {
                lo[c] = fminf(lo[c], v);
                hi[c] = fmaxf(hi[c], v);
            }
        }
    }
    for (int c = 0; c < NB; ++c) {
        tbox[(size_t)t * 2 * NB + c] = lo[c];
        tbox[(size_t)t * 2 * NB + NB + c] = hi[c];
    }
    tkey0[t] = t * kCullTile < n ? keys_sorted[t * kCullTile] : 0xFFFFFFFFu;
}

__global__ void super_box_kernel(const float *__restrict__ tbox, uint32_t ntiles, int NB, uint32_t nsuper,
                                 float *__restrict__ sbox) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nsuper) return;
    for (int c = 0; c < NB; ++c) {
        float lo = __builtin_inff(), hi = -__builtin_inff();
        for (uint32_t t = s * kSuperTiles; t < min((s + 1) * kSuperTiles, ntiles); ++t) {
            lo = fminf(lo, tbox[(size_t)t * 2 * NB + c]);
            hi = fmaxf(hi, tbox[(size_t)t * 2 * NB + NB + c]);
        }
        sbox[(size_t)s * 2 * NB + c] = lo;
        sbox[(size_t)s * 2 * NB + NB + c] = hi;
    }
}

// ---- screening --------------------------------------------------------------------------
// acos on [0, 1] (Abramowitz & Stegun 4.4.46, |error| <= 2e-8; fp32 evaluation adds
// < 1e-6, inside the screen's error bound).  NaN propagates.
__device__ __forceinline__ float acos01(float x) {
    float p = -0.0012624911f;
    p = fmaf(p, x, 0.0066700901f);
    p = fmaf(p, x, -0.0170881256f);
    p = fmaf(p, x, 0.0308918810f);
    p = fmaf(p, x, -0.0501743046f);
    p = fmaf(p, x, 0.0889789874f);
    p = fmaf(p, x, -0.2145988016f);
    p = fmaf(p, x, 1.5707963050f);
    return __builtin_amdgcn_sqrtf(1.f - x) * p;
}

// Rotation pre-reject threshold: an element with |dot| <= cos(tau/w1 + 1e-5) has
// acos(|dot|) > tau/w1 even after every fp32 error, hence distance > tau: skip it without
// the square root and the arc cosine.  ctau < 0 rejects nothing.
__device__ __forceinline__ float rot_threshold(float tau, float w1) {
    const float x = tau / w1 + 1e-5f;
    return x < 1.5707963f ? cosf(x) : -1.f;
}

// fp32 distance of LDS state j to the lane's query, with the SE3 translation pre-reject
// and the rotation pre-reject
template <int SP, int FS, int K2>
__device__ __forceinline__ void screen_pair(const float *tile, int j, const float *qf, float w0, float w0sq, float w1,
                                            uint32_t id, TopK32<K2> &top, float &ctau) {
    if constexpr (SP == OMPL_GPU_SPACE_SE3) {
        const float4 a = reinterpret_cast<const float4 *>(tile)[j * 2];
        const float dx = a.x - qf[0], dy = a.y - qf[1], dz = a.z - qf[2];
        float t = dx * dx;
        t = fmaf(dy, dy, t);
        t = fmaf(dz, dz, t);
        if (t * w0sq < top.tau2) {
            const float4 r = reinterpret_cast<const float4 *>(tile)[j * 2 + 1];
            float dot = r.x * qf[4];
            dot = fmaf(r.y, qf[5], dot);
            dot = fmaf(r.z, qf[6], dot);
            dot = fmaf(r.w, qf[7], dot);
            const float c = abs1(dot);
            if (c > ctau) {
                const float d = w0 * __builtin_amdgcn_sqrtf(t) + w1 * acos01(c);
                if (top.admits(d, id)) {
                    top.push(d, id);
                    ctau = rot_threshold(top.d[K2 - 1], w1);
                }
            }
        }
    } else if constexpr (SP == OMPL_GPU_SPACE_SO3) {
        const float4 r = reinterpret_cast<const float4 *>(tile)[j];
        float dot = r.x * qf[0];
        dot = fmaf(r.y, qf[1], dot);
        dot = fmaf(r.z, qf[2], dot);
        dot = fmaf(r.w, qf[3], dot);
        const float c = abs1(dot);
        if (c > ctau) {
            const float d = acos01(c);
            if (top.admits(d, id)) {
                top.push(d, id);
                ctau = rot_threshold(top.d[K2 - 1], 1.f);
            }
        }
    } else {
        float acc = 0.f;
#pragma unroll
        for (int f = 0; f < FS; ++f) {
            const float diff = tile[j * FS + f] - qf[f];
            acc = fmaf(diff, diff, acc);
        }
        if (acc < top.tau2) {
            const float d = __builtin_amdgcn_sqrtf(acc);
            if (top.admits(d, id)) top.push(d, id);
        }
    }
}

template <int SP, int FS>
__device__ __forceinline__ void stage_row(float *tile, int slot, const float *__restrict__ src, uint64_t stride,
                                          uint64_t g) {
    if constexpr (SP == OMPL_GPU_SPACE_SE3) {
        float4 a, r;
        a.x = src[g]; a.y = src[stride + g]; a.z = src[2 * stride + g]; a.w = 0.f;
        r.x = src[3 * stride + g]; r.y = src[4 * stride + g]; r.z = src[5 * stride + g]; r.w = src[6 * stride + g];
        reinterpret_cast<float4 *>(tile)[slot * 2] = a;
        reinterpret_cast<float4 *>(tile)[slot * 2 + 1] = r;
    } else {
#pragma unroll
        for (int f = 0; f < FS; ++f) tile[slot * FS + f] = src[(uint64_t)f * stride + g];
    }
}

// chunked brute-force screen (SO3, or when no sorted copy exists)
template <int SP, int F, int K2>
__global__ __launch_bounds__(256) void knn32_screen_kernel(const float *__restrict__ f32, uint64_t cap,
                                                           uint64_t n_end, const float *__restrict__ q32,
                                                           uint32_t nq, uint32_t chunk_len, float w0, float w1,
                                                           float *__restrict__ pd, uint32_t *__restrict__ pi) {
    constexpr int FS = Geo<SP, F>::FS;
    __shared__ __attribute__((aligned(16))) float tile[kTile * FS];
    const uint32_t qs = blockIdx.x * kTile + threadIdx.x;
    float qf[FS];
#pragma unroll
    for (int f = 0; f < FS; ++f) qf[f] = qs < nq ? q32[(size_t)qs * FS + f] : __builtin_nanf("");
    const float w0sq = w0 * w0;
    TopK32<K2> top;
    top.init();
    float ctau = -1.f;
    const uint64_t c0 = (uint64_t)blockIdx.y * chunk_len;
    const uint64_t c1 = min(c0 + chunk_len, n_end);
    for (uint64_t base = c0; base < c1; base += kTile) {
        stage_row<SP, FS>(tile, threadIdx.x, f32, cap, base + threadIdx.x);
        __syncthreads();
#pragma unroll 4
        for (int s = 0; s < kTile; ++s)
            screen_pair<SP, FS, K2>(tile, s, qf, w0, w0sq, w1, (uint32_t)(base + s), top, ctau);
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

// culled screen: one wave = 64 spatially adjacent queries, nearest-first walk over
// super-tiles with box culling (the Euclidean part is a lower bound of the distance)
template <int SP, int F, int K2>
__global__ __launch_bounds__(64) void knn32_cull_kernel(
    const float *__restrict__ rows, uint32_t n_pad, const uint32_t *__restrict__ ids, uint32_t ntiles,
    const float *__restrict__ tbox, const float *__restrict__ sbox, uint32_t nsuper,
    const uint32_t *__restrict__ tkey0, const float *__restrict__ q32, const uint32_t *__restrict__ qkeys,
    uint32_t nq, float w0, float w1, float *__restrict__ pd, uint32_t *__restrict__ pi,
    unsigned long long *__restrict__ counters) {
    constexpr int FS = Geo<SP, F>::FS;
    constexpr int NB = Geo<SP, F>::NB;
    __shared__ __attribute__((aligned(16))) float tile[kCullTile * FS];
    __shared__ uint32_t tid[kCullTile];
    const int lane = threadIdx.x;
    const uint32_t qs = blockIdx.x * kCullTile + lane;
    const bool active = qs < nq;
    float qf[FS];
#pragma unroll
    for (int f = 0; f < FS; ++f) qf[f] = active ? q32[(size_t)qs * FS + f] : __builtin_nanf("");
    const float w0sq = w0 * w0;
    TopK32<K2> top;
    top.init();
    float ctau = -1.f;
    uint32_t visited = 0;
    // start at the tile holding this wave's middle query on the Morton curve
    const uint32_t key = qkeys[min(blockIdx.x * kCullTile + kCullTile / 2, nq - 1)];
    uint32_t lo = 0, hi = ntiles;  // first tile with tkey0 > key
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (tkey0[mid] <= key)
            lo = mid + 1;
        else
            hi = mid;
    }
    const int s0 = (int)((lo > 0 ? lo - 1 : 0) / kSuperTiles);
    auto culled = [&](const float *box) {
        float lb2 = 0.f;
#pragma unroll
        for (int c = 0; c < NB; ++c) {
            const float g = fmaxf(fmaxf(box[c] - qf[c], qf[c] - box[NB + c]), 0.f);
            lb2 = fmaf(g, g, lb2);
        }
        return __all(!active || lb2 * w0sq >= top.tau2);
    };
    for (int step = 0; step < 2 * (int)nsuper; ++step) {
        const int s = (step & 1) ? s0 + (step + 1) / 2 : s0 - step / 2;  // s0, s0+1, s0-1, s0+2, ...
        if (s < 0 || s >= (int)nsuper) continue;
        if (culled(sbox + (size_t)s * 2 * NB)) continue;
        const uint32_t t_end = min((uint32_t)(s + 1) * kSuperTiles, ntiles);
        for (uint32_t t = (uint32_t)s * kSuperTiles; t < t_end; ++t) {
            if (culled(tbox + (size_t)t * 2 * NB)) continue;
            const uint64_t p = (uint64_t)t * kCullTile + lane;
            stage_row<SP, FS>(tile, lane, rows, n_pad, p);
            tid[lane] = ids[p];
            __syncthreads();
#pragma unroll 4
            for (int j = 0; j < kCullTile; ++j)
                screen_pair<SP, FS, K2>(tile, j, qf, w0, w0sq, w1, tid[j], top, ctau);
            ++visited;
            __syncthreads();
        }
    }
    if (counters && lane == 0) atomicAdd(counters, (unsigned long long)visited);  // tiles scanned
    if (!active) return;
    const size_t o = (size_t)qs * K2;
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
            sp.w1 * (1.1 * sqrt(12.0 * kU) + 2e-6 + 4.5e-5);
    } else if constexpr (SP == OMPL_GPU_SPACE_SO3) {
        e = 1.1 * sqrt(12.0 * kU) + 2e-6 + 4.5e-5;
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
            if (!t.admits(d, id)) break;  // lists are sorted
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
            ex.offer(feat_dist<SP, F, 0>(sv, qv, sp), id);  // the reference formula, fp64
        }
    }
    bool ok = true;
    if (t.i[K2 - 1] != kNoId) {  // the list is full: prove that no excluded element can enter
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

// ---- host orchestration -----------------------------------------------------------------
struct FastPlan {
    int K2, K;
    bool cull;
    uint32_t chunks, chunk_len;
};

FastPlan fast_plan(const DevSpace &sp, uint32_t nq, uint32_t k, uint64_t n_end, int num_cus, bool cull) {
    FastPlan p{};
    p.K2 = fast_k2(sp, k, nq);
    p.K = k_bucket(k);
    p.cull = cull;
    if (cull) {
        p.chunks = 1;
        p.chunk_len = 0;
        return p;
    }
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
    size_t keys, keys2, idx, perm, cub, q32u, q32, pd, pi, fail, total;
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
                                             (uint32_t *)nullptr, (uint32_t *)nullptr, (int)nq, 0, 32);
    L.cub_bytes = cb;
    L.cub = take(cb);
    const int FS = sp.kind == OMPL_GPU_SPACE_SE3 ? 8 : g.F;
    L.q32u = take(4ull * nq * FS);
    L.q32 = take(4ull * nq * FS);
    L.pd = take(4ull * p.chunks * nq * p.K2);
    L.pi = take(4ull * p.chunks * nq * p.K2);
    L.fail = take(4ull * (nq + 1));
    L.total = off;
    return L;
}

template <int SP, int F, int K2, int K>
hipError_t run_fast(const DevSpace &sp, const FastPlan &p, const FastLayout &L, char *ws, const float *f32,
                    const double *f64, uint64_t cap, uint64_t n_end, const SortedStore *ss, const double *qf64,
                    uint32_t nq, uint32_t k, const FastBounds &b, double *od, uint32_t *oi, hipStream_t st) {
    constexpr int FS = Geo<SP, F>::FS;
    uint32_t *keys = (uint32_t *)(ws + L.keys), *keys2 = (uint32_t *)(ws + L.keys2);
    uint32_t *idx = (uint32_t *)(ws + L.idx), *perm = (uint32_t *)(ws + L.perm);
    float *q32u = (float *)(ws + L.q32u), *q32 = (float *)(ws + L.q32);
    float *pd = (float *)(ws + L.pd);
    uint32_t *pi = (uint32_t *)(ws + L.pi);
    uint32_t *fail = (uint32_t *)(ws + L.fail);
    const dim3 b256(256);
    hipLaunchKernelGGL((query_rows_kernel<SP, F>), dim3((nq + 255) / 256), b256, 0, st, qf64, nq, b, q32u, keys, idx);
    size_t cb = L.cub_bytes;
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(ws + L.cub, cb, keys, keys2, idx, perm, (int)nq, 0, 32, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((query_gather_kernel<FS>), dim3((nq * FS + 255) / 256), b256, 0, st, q32u, perm, nq, q32);
    e = hipMemsetAsync(fail, 0, 4, st);
    if (e != hipSuccess) return e;
    if (p.cull) {
        timer_begin(st, "knn32_cull_kernel");
        hipLaunchKernelGGL((knn32_cull_kernel<SP, F, K2>), dim3((nq + kCullTile - 1) / kCullTile), dim3(kCullTile), 0,
                           st, ss->rows, ss->n_pad, ss->ids, ss->ntiles, ss->tbox, ss->sbox, ss->nsuper, ss->tkey0,
                           q32, keys2, nq, (float)sp.w0, (float)sp.w1, pd, pi, ss->counters);
        timer_end(st);
    } else {
        timer_begin(st, "knn32_screen_kernel");
        hipLaunchKernelGGL((knn32_screen_kernel<SP, F, K2>), dim3((nq + kTile - 1) / kTile, p.chunks), dim3(kTile), 0,
                           st, f32, cap, n_end, q32, nq, p.chunk_len, (float)sp.w0, (float)sp.w1, pd, pi);
        timer_end(st);
    }
    hipLaunchKernelGGL((knn_certify_kernel<SP, F, K2, K>), dim3((nq + 255) / 256), b256, 0, st, pd, pi, p.chunks, nq,
                       perm, f64, cap, qf64, sp, b.absmax, od, oi, k, fail, fail + 1);
    return hipGetLastError();
}

template <int SP, int F, int K2>
hipError_t run_fast_k(const DevSpace &sp, const FastPlan &p, const FastLayout &L, char *ws, const float *f32,
                      const double *f64, uint64_t cap, uint64_t n_end, const SortedStore *ss, const double *qf64,
                      uint32_t nq, uint32_t k, const FastBounds &b, double *od, uint32_t *oi, hipStream_t st) {
    switch (p.K) {
    case 1: return run_fast<SP, F, K2, 1>(sp, p, L, ws, f32, f64, cap, n_end, ss, qf64, nq, k, b, od, oi, st);
    case 4: return run_fast<SP, F, K2, 4>(sp, p, L, ws, f32, f64, cap, n_end, ss, qf64, nq, k, b, od, oi, st);
    case 16: return run_fast<SP, F, K2, 16>(sp, p, L, ws, f32, f64, cap, n_end, ss, qf64, nq, k, b, od, oi, st);
    case 32:
        if constexpr (K2 >= 32)
            return run_fast<SP, F, K2, 32>(sp, p, L, ws, f32, f64, cap, n_end, ss, qf64, nq, k, b, od, oi, st);
    }
    return hipErrorInvalidValue;
}

template <int SP, int F>
hipError_t run_fast_space(const DevSpace &sp, const FastPlan &p, const FastLayout &L, char *ws, const float *f32,
                          const double *f64, uint64_t cap, uint64_t n_end, const SortedStore *ss, const double *qf64,
                          uint32_t nq, uint32_t k, const FastBounds &b, double *od, uint32_t *oi, hipStream_t st) {
    switch (p.K2) {
    case 16: return run_fast_k<SP, F, 16>(sp, p, L, ws, f32, f64, cap, n_end, ss, qf64, nq, k, b, od, oi, st);
    case 32: return run_fast_k<SP, F, 32>(sp, p, L, ws, f32, f64, cap, n_end, ss, qf64, nq, k, b, od, oi, st);
    case 64: return run_fast_k<SP, F, 64>(sp, p, L, ws, f32, f64, cap, n_end, ss, qf64, nq, k, b, od, oi, st);
    }
    return hipErrorInvalidValue;
}

template <int SP, int F>
hipError_t build_sorted(const float *f32, uint64_t cap, uint32_t n, const FastBounds &b, SortedStore *s,
                        hipStream_t st) {
    constexpr int R = Geo<SP, F>::R, NB = Geo<SP, F>::NB;
    free_sorted_store(s);
    s->n = n;
    s->ntiles = std::max<uint32_t>(1, (n + kCullTile - 1) / kCullTile);
    s->n_pad = s->ntiles * kCullTile;
    s->nsuper = (s->ntiles + kSuperTiles - 1) / kSuperTiles;
    uint32_t *keys = nullptr, *ids0 = nullptr, *keys_s = nullptr, *ids_s = nullptr;
    void *tmp = nullptr;
    size_t tb = 0;
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(nullptr, tb, keys, keys_s, ids0, ids_s, (int)n, 0, 32, st);
    auto done = [&](hipError_t r) {
        for (void *x : {(void *)keys, (void *)ids0, (void *)keys_s, (void *)ids_s, tmp})
            if (x) (void)hipFree(x);
        if (r != hipSuccess) free_sorted_store(s);
        return r;
    };
    if (e != hipSuccess) return done(e);
    if ((e = hipMalloc(&keys, 4ull * std::max<uint32_t>(n, 1))) != hipSuccess) return done(e);
    if ((e = hipMalloc(&ids0, 4ull * std::max<uint32_t>(n, 1))) != hipSuccess) return done(e);
    if ((e = hipMalloc(&keys_s, 4ull * std::max<uint32_t>(n, 1))) != hipSuccess) return done(e);
    if ((e = hipMalloc(&ids_s, 4ull * std::max<uint32_t>(n, 1))) != hipSuccess) return done(e);
    if ((e = hipMalloc(&tmp, std::max<size_t>(tb, 1))) != hipSuccess) return done(e);
    if ((e = hipMalloc(&s->rows, 4ull * R * s->n_pad)) != hipSuccess) return done(e);
    if ((e = hipMalloc(&s->ids, 4ull * s->n_pad)) != hipSuccess) return done(e);
    if ((e = hipMalloc(&s->tbox, 8ull * NB * s->ntiles)) != hipSuccess) return done(e);
    if ((e = hipMalloc(&s->sbox, 8ull * NB * s->nsuper)) != hipSuccess) return done(e);
    if ((e = hipMalloc(&s->tkey0, 4ull * s->ntiles)) != hipSuccess) return done(e);
    s->bytes = 4ull * R * s->n_pad + 4ull * s->n_pad + 8ull * NB * (s->ntiles + s->nsuper) + 4ull * s->ntiles;
    if (n) {
        hipLaunchKernelGGL((tree_key_kernel<SP, F>), dim3((n + 255) / 256), dim3(256), 0, st, f32, cap, n, b, keys,
                           ids0);
        if ((e = hipcub::DeviceRadixSort::SortPairs(tmp, tb, keys, keys_s, ids0, ids_s, (int)n, 0, 32, st)) !=
            hipSuccess)
            return done(e);
    }
    hipLaunchKernelGGL((tree_gather_kernel<SP, F>), dim3((s->n_pad + 255) / 256), dim3(256), 0, st, f32, cap, ids_s,
                       n, s->n_pad, s->rows, s->ids);
    hipLaunchKernelGGL((tile_box_kernel<SP, F>), dim3((s->ntiles + 255) / 256), dim3(256), 0, st, s->rows, s->n_pad,
                       s->ntiles, keys_s, n, s->tbox, s->tkey0);
    hipLaunchKernelGGL(super_box_kernel, dim3((s->nsuper + 255) / 256), dim3(256), 0, st, s->tbox, s->ntiles, NB,
                       s->nsuper, s->sbox);
    if ((e = hipGetLastError()) != hipSuccess) return done(e);
    if ((e = hipStreamSynchronize(st)) != hipSuccess) return done(e);  // temporaries freed below
    return done(hipSuccess);
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

bool cull_supported(const DevSpace &sp) {
    return sp.kind == OMPL_GPU_SPACE_SE3 || sp.kind == OMPL_GPU_SPACE_REALVECTOR;
}

void free_sorted_store(SortedStore *s) {
    for (void *x : {(void *)s->rows, (void *)s->ids, (void *)s->tbox, (void *)s->sbox, (void *)s->tkey0})
        if (x) (void)hipFree(x);
    *s = SortedStore{};
}

hipError_t build_sorted_store(const DevSpace &sp, const FeatGeom &g, const float *feat32, uint64_t cap, uint32_t n,
                              const FastBounds &b, SortedStore *s, hipStream_t st) {
    switch (sp.kind) {
    case OMPL_GPU_SPACE_SE3: return build_sorted<OMPL_GPU_SPACE_SE3, 7>(feat32, cap, n, b, s, st);
    case OMPL_GPU_SPACE_REALVECTOR:
        if (g.F == 4) return build_sorted<OMPL_GPU_SPACE_REALVECTOR, 4>(feat32, cap, n, b, s, st);
        if (g.F == 8) return build_sorted<OMPL_GPU_SPACE_REALVECTOR, 8>(feat32, cap, n, b, s, st);
        return build_sorted<OMPL_GPU_SPACE_REALVECTOR, 16>(feat32, cap, n, b, s, st);
    }
    return hipErrorInvalidValue;
}

size_t knn_fast_workspace_bytes(const DevSpace &sp, const FeatGeom &g, uint32_t nq, uint32_t k, uint64_t n_end,
                                int num_cus, bool cull) {
    const FastPlan p = fast_plan(sp, nq, k, n_end, num_cus, cull);
    if (p.K2 == 0) return 0;
    return fast_layout(sp, g, p, nq).total;
}

hipError_t launch_knn_fast(const DevSpace &sp, const FeatGeom &g, const double *feat64, const float *feat32,
                           uint64_t cap, uint64_t n_end, const SortedStore *sorted, const double *qfeat64, uint32_t nq,
                           uint32_t k, const FastBounds &b, double *out_d, uint32_t *out_i, void *ws, size_t ws_bytes,
                           int num_cus, hipStream_t st, uint32_t **fail_count, uint32_t **fail_list) {
    const FastPlan p = fast_plan(sp, nq, k, n_end, num_cus, sorted != nullptr);
    if (p.K2 == 0) return hipErrorInvalidValue;
    const FastLayout L = fast_layout(sp, g, p, nq);
    if (L.total > ws_bytes) return hipErrorInvalidValue;
    char *w = (char *)ws;
    *fail_count = (uint32_t *)(w + L.fail);
    *fail_list = *fail_count + 1;
    switch (sp.kind) {
    case OMPL_GPU_SPACE_SE3:
        return run_fast_space<OMPL_GPU_SPACE_SE3, 7>(sp, p, L, w, feat32, feat64, cap, n_end, sorted, qfeat64, nq, k,
                                                      b, out_d, out_i, st);
    case OMPL_GPU_SPACE_SO3:
        return run_fast_space<OMPL_GPU_SPACE_SO3, 4>(sp, p, L, w, feat32, feat64, cap, n_end, nullptr, qfeat64, nq,
                                                      k, b, out_d, out_i, st);
    case OMPL_GPU_SPACE_REALVECTOR:
        if (g.F == 4)
            return run_fast_space<OMPL_GPU_SPACE_REALVECTOR, 4>(sp, p, L, w, feat32, feat64, cap, n_end, sorted,
                                                                 qfeat64, nq, k, b, out_d, out_i, st);
        if (g.F == 8)
            return run_fast_space<OMPL_GPU_SPACE_REALVECTOR, 8>(sp, p, L, w, feat32, feat64, cap, n_end, sorted,
                                                                 qfeat64, nq, k, b, out_d, out_i, st);
        return run_fast_space<OMPL_GPU_SPACE_REALVECTOR, 16>(sp, p, L, w, feat32, feat64, cap, n_end, sorted,
                                                              qfeat64, nq, k, b, out_d, out_i, st);
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
