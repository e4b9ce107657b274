// knn.hip — nearest-neighbour kernels for gfx950 (MI355X / CDNA4).
//
// Replaces the reference's per-query tree walk (NearestNeighborsGNAT.h:335-356,
// :565-662) with exact brute-force scans over a structure-of-arrays state store in
// HBM.  Two mappings:
//   * tiled   (batched queries, nq >= kStreamMaxQ): one thread = one query; a 256-
//             state tile of the store is staged through LDS and read by broadcast;
//             the store is split into chunks along grid.y so the grid fills 256 CUs;
//             per-thread register top-K; per-chunk lists merged by knn_merge.
//   * stream  (small nq, the RRT one-query-per-iteration case): one wave = 64*ITEMS
//             consecutive states, coalesced SoA loads, per-lane top-K, wave/block
//             selection by shuffles; partial lists merged per query.
// Distances are fp64 in the reference's operation order (device_space.h); results
// are ordered by (distance, id), which is the reference's ascending order with ties
// resolved by insertion id.
#include <hip/hip_runtime.h>
#include <math.h>

#include <algorithm>

#include "kernels.h"
#include "feat_dist.h"
#include "topk.h"

namespace ompl_amd {

constexpr int kStreamItems = 16;      // states per lane in the stream radius mapping


// ---------------------------------------------------------------------------------
// tiled batched kNN
template <int SP, int F, int NMAX, int K>
__global__ __launch_bounds__(256) void knn_tiled_kernel(const double *__restrict__ feat, uint64_t cap,
                                                        uint64_t n_end, const double *__restrict__ qfeat,
                                                        uint32_t nq, uint32_t chunk_len, DevSpace sp,
                                                        double *__restrict__ out_d, uint32_t *__restrict__ out_i,
                                                        uint32_t out_k) {
    constexpr int FP = LdsStride<F>::value;
    __shared__ __attribute__((aligned(16))) double tile[kTile * FP];
    const uint32_t q = blockIdx.x * kTile + threadIdx.x;
    double qf[F];
#pragma unroll
    for (int f = 0; f < F; ++f) qf[f] = q < nq ? qfeat[(size_t)q * F + f] : __builtin_nan("");
    TopK<K> top;
    top.init();
    const uint64_t c0 = (uint64_t)blockIdx.y * chunk_len;
    const uint64_t c1 = min(c0 + chunk_len, n_end);
    for (uint64_t base = c0; base < c1; base += kTile) {
#pragma unroll
        for (int f = 0; f < F; ++f) tile[threadIdx.x * FP + f] = feat[(uint64_t)f * cap + base + threadIdx.x];
        __syncthreads();
#pragma unroll 2
        for (int s = 0; s < kTile; ++s) {
            double sf[F];
#pragma unroll
            for (int f = 0; f < F; ++f) sf[f] = tile[s * FP + f];
            const double d = feat_dist<SP, F, NMAX>(sf, qf, sp);
            const uint32_t id = (uint32_t)(base + s);
            if (top.admits(d, id)) top.push(d, id);
        }
        __syncthreads();
    }
    if (q >= nq) return;
    // out layout: [blockIdx.y][nq][out_k]
    const size_t o = ((size_t)blockIdx.y * nq + q) * out_k;
#pragma unroll
    for (int j = 0; j < K; ++j)
        if (j < (int)out_k) {
            out_d[o + j] = top.d[j];
            out_i[o + j] = top.i[j];
        }
}

// thread per query: merge S sorted partial lists of K
template <int K>
__global__ __launch_bounds__(256) void knn_merge_kernel(const double *__restrict__ pd, const uint32_t *__restrict__ pi,
                                                        uint32_t S, uint32_t nq, double *__restrict__ out_d,
                                                        uint32_t *__restrict__ out_i, uint32_t out_k) {
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nq) return;
    TopK<K> top;
    top.init();
    for (uint32_t s = 0; s < S; ++s) {
        const size_t o = ((size_t)s * nq + q) * K;
        for (int j = 0; j < K; ++j) {
            const double d = pd[o + j];
            const uint32_t id = pi[o + j];
            if (!top.admits(d, id)) break;  // lists are sorted
            top.push(d, id);
        }
    }
#pragma unroll
    for (int j = 0; j < K; ++j)
        if (j < (int)out_k) {
            out_d[(size_t)q * out_k + j] = top.d[j];
            out_i[(size_t)q * out_k + j] = top.i[j];
        }
}

// ---------------------------------------------------------------------------------
// stream kNN (small nq): grid (blocks, nq); wave gw scans [gw*64*ITEMS, (gw+1)*64*ITEMS).
// HBM/MALL-bound: every wave issues all of its ITEMS x F row loads before the first
// distance, and the grid has ~4 waves per SIMD, so the whole store is in flight at once
// instead of a few serial load rounds per wave.  n_end is a multiple of kTile = 64*ITEMS,
// so a wave is either wholly inside the store or wholly past it (wave-uniform guard).
constexpr int kScanItems = 4;
static_assert(64 * kScanItems == kTile, "stream waves must tile n_end exactly");

template <int SP, int F, int NMAX, int K>
__global__ __launch_bounds__(256) void knn_stream_kernel(const double *__restrict__ feat, uint64_t cap,
                                                         uint64_t n_end, const double *__restrict__ qfeat,
                                                         DevSpace sp, double *__restrict__ part_d,
                                                         uint32_t *__restrict__ part_i) {
    __shared__ double lds_d[4 * K];
    __shared__ uint32_t lds_i[4 * K];
    const uint32_t q = blockIdx.y;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    double qf[F];
#pragma unroll
    for (int f = 0; f < F; ++f) qf[f] = qfeat[(size_t)q * F + f];
    TopK<K> top;
    top.init();
    const uint64_t wbase = ((uint64_t)blockIdx.x * 4 + wave) * (64 * kScanItems);
    if (wbase < n_end) {
        double sf[kScanItems][F];
#pragma unroll
        for (int it = 0; it < kScanItems; ++it)
#pragma unroll
            for (int f = 0; f < F; ++f) sf[it][f] = feat[(uint64_t)f * cap + wbase + (uint64_t)it * 64 + lane];
#pragma unroll
        for (int it = 0; it < kScanItems; ++it) {
            const uint32_t id = (uint32_t)(wbase + (uint64_t)it * 64 + lane);
            if constexpr (SP == OMPL_GPU_SPACE_SE3) {
                // se3_dist is (0 + w0 * |dt|) + w1 * arc with arc >= 0, so in fp64 it is >= the
                // first term computed by the same operations: a state whose translation term
                // alone exceeds the current K-th distance cannot enter, and its acos is skipped
                const double a = sp.w0 * l2_dist(sf[it], qf, 3);
                if (!(a > top.d[K - 1])) {
                    double d = 0.0;
                    d += a;
                    d += sp.w1 * so3_arc(sf[it] + 3, qf + 3);
                    top.offer(d, id);
                }
            } else {
                top.offer(feat_dist<SP, F, NMAX>(sf[it], qf, sp), id);
            }
        }
    }
    double rd;
    uint32_t ri;
    block_select<K>(top, lds_d, lds_i, rd, ri);
    if (wave == 0 && lane < K) {
        const size_t o = ((size_t)q * gridDim.x + blockIdx.x) * K + lane;
        part_d[o] = rd;
        part_i[o] = ri;
    }
}

// block per query: merge P lists of K
template <int K>
__global__ __launch_bounds__(256) void knn_stream_merge_kernel(const double *__restrict__ pd,
                                                               const uint32_t *__restrict__ pi, uint32_t P,
                                                               double *__restrict__ out_d,
                                                               uint32_t *__restrict__ out_i, uint32_t out_k) {
    __shared__ double lds_d[4 * K];
    __shared__ uint32_t lds_i[4 * K];
    const uint32_t q = blockIdx.x;
    TopK<K> top;
    top.init();
    const size_t base = (size_t)q * P * K;
    for (size_t j = threadIdx.x; j < (size_t)P * K; j += blockDim.x) top.offer(pd[base + j], pi[base + j]);
    double rd;
    uint32_t ri;
    block_select<K>(top, lds_d, lds_i, rd, ri);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (wave == 0 && lane < (int)out_k) {
        out_d[(size_t)q * out_k + lane] = rd;
        out_i[(size_t)q * out_k + lane] = ri;
    }
}

// ---------------------------------------------------------------------------------
// bounded exact re-run of the fast path's uncertified queries.  The certificate already
// wrote, for query q, the exact k-th distance b_q among its screened candidates; those k
// candidates are stored states, so the true k nearest all have d <= b_q.  One pass over
// the store therefore keeps every state with exact d <= b_q (few per query) and a rank
// sort of that set yields the exact (distance, id) top-k — the same answer as the full
// stream re-run, at one read of the store for all failed queries together instead of one
// per query.  A query with more than kBoundedCap such states overflows to the full scan.
//
// One persistent launch (a block per CU) runs the three phases — the bounded pass, the
// per-query rank select, the full scans of the overflow list — separated by grid-wide
// barriers.  The failed-query count is read on the device (no host round trip): when nothing
// failed, every block returns at once, so the common batch pays one small launch instead of
// three (two of them store-sized grids).  All blocks are co-resident (one per CU, whatever
// else runs beside them eventually drains), so the barriers cannot deadlock.

// grid-wide barrier: each thread releases its phase's writes at agent scope (the L2s of the
// XCDs are not coherent with each other), thread 0 of each block counts in and waits for the
// target on the monotone counter, and every thread acquires before the next phase
__device__ __forceinline__ void rerun_grid_sync(uint32_t *ctr, uint32_t target) {
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        while (__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) __builtin_amdgcn_s_sleep(4);
    }
    __syncthreads();
    __threadfence();
}

template <int SP, int F, int NMAX, int ITEMS, int K>
__global__ __launch_bounds__(256) void knn_rerun_kernel(const double *__restrict__ feat, uint64_t cap, uint64_t n_end,
                                                        const double *__restrict__ qfeat,
                                                        const uint32_t *__restrict__ list,
                                                        const uint32_t *__restrict__ nlist_ptr, DevSpace sp,
                                                        uint32_t out_k, double *__restrict__ out_d,
                                                        uint32_t *__restrict__ out_i, uint32_t *__restrict__ counts,
                                                        double *__restrict__ cand_d, uint32_t *__restrict__ cand_i,
                                                        unsigned long long *__restrict__ stats) {
    const uint32_t total = *nlist_ptr;
    if (total == 0) return;  // the common batch: every query certified
    const uint32_t nlist = min(total, kBoundedMaxQ);
    uint32_t *ov_count = counts + kBoundedMaxQ, *bar = counts + kBoundedMaxQ + 1, *ov_list = counts + kBoundedMaxQ + 2;

    // phase 1: the bounded pass — chunks of 256 * ITEMS states, block-strided
    const uint64_t nchunk = (n_end + 256 * ITEMS - 1) / (256 * ITEMS);
    for (uint64_t c = blockIdx.x; c < nchunk; c += gridDim.x) {
        const uint64_t base = c * (256 * ITEMS) + threadIdx.x;
        double sf[ITEMS][F];
#pragma unroll
        for (int it = 0; it < ITEMS; ++it) {
            const uint64_t g = base + (uint64_t)it * 256;
#pragma unroll
            for (int f = 0; f < F; ++f) sf[it][f] = g < n_end ? feat[(uint64_t)f * cap + g] : __builtin_nan("");
        }
        for (uint32_t j = 0; j < nlist; ++j) {
            const uint32_t q = list[j];
            const double b = out_d[(size_t)q * out_k + out_k - 1];
            double qv[F];
#pragma unroll
            for (int f = 0; f < F; ++f) qv[f] = qfeat[(size_t)q * F + f];
#pragma unroll
            for (int it = 0; it < ITEMS; ++it) {
                double d;
                if constexpr (SP == OMPL_GPU_SPACE_SE3) {
                    // as knn_stream_kernel: the translation term alone bounds the distance below
                    const double a = sp.w0 * l2_dist(sf[it], qv, 3);
                    if (!(a <= b)) continue;
                    d = 0.0;
                    d += a;
                    d += sp.w1 * so3_arc(sf[it] + 3, qv + 3);
                } else {
                    d = feat_dist<SP, F, NMAX>(sf[it], qv, sp);
                }
                if (d <= b) {  // NaN (unused / removed slot) never passes
                    const uint32_t slot = atomicAdd(&counts[j], 1u);
                    if (slot < kBoundedCap) {
                        cand_d[(size_t)j * kBoundedCap + slot] = d;
                        cand_i[(size_t)j * kBoundedCap + slot] = (uint32_t)(base + (uint64_t)it * 256);
                    }
                }
            }
        }
    }
    rerun_grid_sync(bar, gridDim.x);

    // phase 2: entry j < nlist rank-sorts its candidates by (distance, id) in LDS and writes the
    // first out_k into its output row; too many (or, impossibly, too few) candidates put the
    // query on the overflow list.  Entry kBoundedMaxQ moves list entries beyond kBoundedMaxQ
    // (not re-run by the bounded pass) to the overflow list.
    {
        __shared__ double sd[kBoundedCap];
        __shared__ uint32_t si[kBoundedCap];
        for (uint32_t j = blockIdx.x; j <= kBoundedMaxQ; j += gridDim.x) {
            if (j == kBoundedMaxQ) {
                for (uint32_t e = kBoundedMaxQ + threadIdx.x; e < total; e += blockDim.x)
                    ov_list[atomicAdd(ov_count, 1u)] = list[e];
            } else if (j < nlist) {
                const uint32_t q = list[j];
                const uint32_t c = counts[j];
                if (c > kBoundedCap || c < out_k) {
                    if (threadIdx.x == 0) ov_list[atomicAdd(ov_count, 1u)] = q;
                } else {
                    for (uint32_t e = threadIdx.x; e < c; e += blockDim.x) {
                        sd[e] = cand_d[(size_t)j * kBoundedCap + e];
                        si[e] = cand_i[(size_t)j * kBoundedCap + e];
                    }
                    __syncthreads();
                    for (uint32_t e = threadIdx.x; e < c; e += blockDim.x) {
                        const double d = sd[e];
                        const uint32_t id = si[e];
                        uint32_t rank = 0;
                        for (uint32_t m = 0; m < c; ++m) rank += (sd[m] < d || (sd[m] == d && si[m] < id)) ? 1u : 0u;
                        if (rank < out_k) {
                            out_d[(size_t)q * out_k + rank] = d;
                            out_i[(size_t)q * out_k + rank] = id;
                        }
                    }
                }
            }
            __syncthreads();  // LDS reuse by the block's next entry
        }
    }
    rerun_grid_sync(bar, 2 * gridDim.x);

    // phase 3: full exact scan of the overflow list, block b answering entries b, b + gridDim.x,
    // ... (per-thread register top-K, block selection) — the rare path
    __shared__ double lds_d[4 * K];
    __shared__ uint32_t lds_i[4 * K];
    const uint32_t count = *ov_count;
    if (stats && blockIdx.x == 0 && threadIdx.x == 0) {  // the re-run statistics (ompl_gpu_nn_stats)
        stats[0] += total;
        stats[1] += count;
    }
    for (uint32_t e = blockIdx.x; e < count; e += gridDim.x) {
        const uint32_t q = ov_list[e];
        double qf[F];
#pragma unroll
        for (int f = 0; f < F; ++f) qf[f] = qfeat[(size_t)q * F + f];
        TopK<K> top;
        top.init();
        for (uint64_t i = threadIdx.x; i < n_end; i += blockDim.x) {
            double sf[F];
#pragma unroll
            for (int f = 0; f < F; ++f) sf[f] = feat[(uint64_t)f * cap + i];
            top.offer(feat_dist<SP, F, NMAX>(sf, qf, sp), (uint32_t)i);
        }
        double rd;
        uint32_t ri;
        block_select<K>(top, lds_d, lds_i, rd, ri);
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
        if (wave == 0 && lane < (int)out_k) {
            out_d[(size_t)q * out_k + lane] = rd;
            out_i[(size_t)q * out_k + lane] = ri;
        }
        __syncthreads();  // lds reuse by the next entry
    }
}

template <int SP, int F, int NMAX>
hipError_t run_knn_bounded(const DevSpace &sp, const double *feat, uint64_t cap, uint64_t n_end, const double *qf,
                           const uint32_t *list, const uint32_t *d_nlist, uint32_t k, double *od, uint32_t *oi,
                           uint32_t *counts, double *cand_d, uint32_t *cand_i, int num_cus, hipStream_t st,
                           unsigned long long *stats) {
    constexpr int ITEMS = F <= 8 ? 4 : 1;
    const dim3 grid((unsigned)std::max(num_cus, 1));  // one block per CU: co-resident (the barriers)
    switch (k_bucket(k)) {
#define OMPL_AMD_RERUN(KK)                                                                                          \
    case KK:                                                                                                       \
        hipLaunchKernelGGL((knn_rerun_kernel<SP, F, NMAX, ITEMS, KK>), grid, dim3(256), 0, st, feat, cap, n_end, qf, \
                           list, d_nlist, sp, k, od, oi, counts, cand_d, cand_i, stats);                           \
        break;
        OMPL_AMD_RERUN(1)
        OMPL_AMD_RERUN(4)
        OMPL_AMD_RERUN(16)
        OMPL_AMD_RERUN(32)
        OMPL_AMD_RERUN(64)
#undef OMPL_AMD_RERUN
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------
// radius search.  Hits are written per (query, chunk) segment in ascending id order
// so that a stable sort by distance yields (distance, id) order.
template <int SP, int F, int NMAX, bool FILL>
__global__ __launch_bounds__(256) void radius_tiled_kernel(const double *__restrict__ feat, uint64_t cap,
                                                           uint64_t n_end, const double *__restrict__ qfeat,
                                                           uint32_t nq, uint32_t chunk_len, uint32_t chunks,
                                                           DevSpace sp, double r, uint32_t *__restrict__ counts,
                                                           const uint64_t *__restrict__ offsets,
                                                           uint32_t *__restrict__ ids, double *__restrict__ dists) {
    constexpr int FP = LdsStride<F>::value;
    __shared__ __attribute__((aligned(16))) double tile[kTile * FP];
    const uint32_t q = blockIdx.x * kTile + threadIdx.x;
    double qf[F];
#pragma unroll
    for (int f = 0; f < F; ++f) qf[f] = q < nq ? qfeat[(size_t)q * F + f] : __builtin_nan("");
    const uint64_t c0 = (uint64_t)blockIdx.y * chunk_len;
    const uint64_t c1 = min(c0 + chunk_len, n_end);
    uint32_t cnt = 0;
    uint64_t out = FILL && q < nq ? offsets[(size_t)q * chunks + blockIdx.y] : 0;
    for (uint64_t base = c0; base < c1; base += kTile) {
#pragma unroll
        for (int f = 0; f < F; ++f) tile[threadIdx.x * FP + f] = feat[(uint64_t)f * cap + base + threadIdx.x];
        __syncthreads();
#pragma unroll 2
        for (int s = 0; s < kTile; ++s) {
            double sf[F];
#pragma unroll
            for (int f = 0; f < F; ++f) sf[f] = tile[s * FP + f];
            const double d = feat_dist<SP, F, NMAX>(sf, qf, sp);
            if (d <= r) {
                if (FILL) {
                    ids[out] = (uint32_t)(base + s);
                    dists[out] = d;
                    ++out;
                } else {
                    ++cnt;
                }
            }
        }
        __syncthreads();
    }
    if (!FILL && q < nq) counts[(size_t)q * chunks + blockIdx.y] = cnt;
}

// stream radius: chunk = one wave's 64*ITEMS consecutive states; ballot-ordered writes
template <int SP, int F, int NMAX, bool FILL>
__global__ __launch_bounds__(256) void radius_stream_kernel(const double *__restrict__ feat, uint64_t cap,
                                                            uint64_t n_end, const double *__restrict__ qfeat,
                                                            uint32_t chunks, DevSpace sp, double r,
                                                            uint32_t *__restrict__ counts,
                                                            const uint64_t *__restrict__ offsets,
                                                            uint32_t *__restrict__ ids, double *__restrict__ dists) {
    const uint32_t q = blockIdx.y;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t chunk = blockIdx.x * 4 + wave;
    if (chunk >= chunks) return;
    double qf[F];
#pragma unroll
    for (int f = 0; f < F; ++f) qf[f] = qfeat[(size_t)q * F + f];
    const uint64_t wbase = (uint64_t)chunk * (64 * kStreamItems);
    uint64_t cursor = FILL ? offsets[(size_t)q * chunks + chunk] : 0;
    uint32_t cnt = 0;
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    for (int it = 0; it < kStreamItems; ++it) {
        const uint64_t id = wbase + (uint64_t)it * 64 + lane;
        bool hit = false;
        double d = 0.0;
        if (id < n_end) {
            double sf[F];
#pragma unroll
            for (int f = 0; f < F; ++f) sf[f] = feat[(uint64_t)f * cap + id];
            d = feat_dist<SP, F, NMAX>(sf, qf, sp);
            hit = d <= r;
        }
        const uint64_t bal = __ballot(hit);
        if (FILL && hit) {
            const uint64_t pos = cursor + __popcll(bal & lt_mask);
            ids[pos] = (uint32_t)id;
            dists[pos] = d;
        }
        cursor += __popcll(bal);
        cnt += (uint32_t)__popcll(bal);
    }
    if (!FILL && lane == 0) counts[(size_t)q * chunks + chunk] = cnt;
}

// ---------------------------------------------------------------------------------
// helpers: features, SoA scatter, steer
__global__ void features_kernel(DevSpace sp, FeatGeom g, const double *__restrict__ raw, uint32_t n,
                                double *__restrict__ feat) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double *s = raw + (size_t)i * sp.dim;
    double *o = feat + (size_t)i * g.F;
    if (sp.kind == OMPL_GPU_SPACE_KCHAIN) {
        double th = 0.;
        for (int j = 0; j < g.nmax; ++j) {
            if (j < sp.dim) {
                th += s[j];
                glibc_sincos(th, o[g.nmax + j], o[j]);  // glibc's cos / sin, as the host's features
            } else {
                o[j] = 0.;
                o[g.nmax + j] = 0.;
            }
        }
    } else {
        for (int j = 0; j < g.F; ++j) o[j] = j < sp.dim ? s[j] : 0.0;
    }
}

__global__ void store_soa_kernel(const double *__restrict__ aos, uint32_t n, int width, double *__restrict__ soa,
                                 uint64_t cap, uint64_t first) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (uint64_t)n * width) return;
    const uint64_t i = t / width, c = t % width;
    soa[c * cap + first + i] = aos[t];
}

// SP / W: fixed-width form (device_space.h; W = 0: runtime width, states in scratch)
template <int SP, int W>
__global__ void steer_kernel(DevSpace sp_in, const double *__restrict__ raw, uint64_t cap, const double *__restrict__ q,
                             uint32_t nq, const uint32_t *__restrict__ nearest, uint32_t stride, double maxd,
                             double *__restrict__ from, double *__restrict__ to) {
    const DevSpace sp = fixed_space<SP, W>(sp_in);
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nq) return;
    const int dim = sp.dim;
    double a[Width<W>::N], b[Width<W>::N], o[Width<W>::N];
    const uint32_t nid = nearest[(size_t)i * stride];
    for (int c = 0; c < dim; ++c) {
        b[c] = q[(size_t)i * dim + c];
        a[c] = nid < cap ? raw[(uint64_t)c * cap + nid] : b[c];  // a missing id (kNoId): from = to = q
    }
    const double d = raw_distance(sp, a, b);  // si_->distance(nmotion->state, rstate)  RRT.cpp:141
    if (d > maxd) {
        interpolate(sp, a, b, maxd / d, o);  // RRT.cpp:142-145
    } else {
        for (int c = 0; c < dim; ++c) o[c] = b[c];
    }
    for (int c = 0; c < dim; ++c) {
        from[(size_t)i * dim + c] = a[c];
        to[(size_t)i * dim + c] = o[c];
    }
}

// Sort each CSR segment by (distance, id) by rank placement: one wave per segment stages
// it in LDS and every element's rank is the number of elements ordered before it, so it
// goes to offsets[q] + rank (ids are unique inside a segment: the ranks are a permutation).
__global__ __launch_bounds__(64) void segment_rank_sort_kernel(const uint64_t *__restrict__ off,
                                                               const uint32_t *__restrict__ in_i,
                                                               const double *__restrict__ in_d,
                                                               uint32_t *__restrict__ out_i,
                                                               double *__restrict__ out_d, uint32_t in_stride) {
    __shared__ double sd[kRankSortMax];
    __shared__ uint32_t si[kRankSortMax];
    const uint32_t q = blockIdx.x;
    const uint64_t b = off[q];
    const uint32_t L = (uint32_t)(off[q + 1] - b);
    if (L > kRankSortMax) return;  // the caller sorts with radix passes instead
    const uint64_t ib = in_stride ? (uint64_t)q * in_stride : b;
    for (uint32_t j = threadIdx.x; j < L; j += blockDim.x) {
        sd[j] = in_d[ib + j];
        si[j] = in_i[ib + j];
    }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < L; j += blockDim.x) {
        const double dj = sd[j];
        const uint32_t ij = si[j];
        uint32_t rank = 0;
        for (uint32_t t = 0; t < L; ++t) rank += lex_less(sd[t], si[t], dj, ij) ? 1u : 0u;
        out_d[b + rank] = dj;
        out_i[b + rank] = ij;
    }
}

// Motion endpoints of a batch of neighbour results, the edges the planners check after a
// neighbour query: PRM checkMotion(state[n], state[m]) (PRM.cpp:577-582, from_query = 0),
// BIT* checkMotion(vertex, sample) (BITstar.cpp:815, from_query = 1).  Edge e pairs query q
// with stored state ids[e]; a missing id (fewer stored states than k) pairs q with itself.
__global__ void edges_kernel(DevSpace sp, const double *__restrict__ raw, uint64_t cap, const double *__restrict__ q,
                             uint32_t nq, const uint64_t *__restrict__ off, const uint32_t *__restrict__ ids,
                             uint32_t stride, uint64_t m, int from_query, double *__restrict__ from,
                             double *__restrict__ to, const double *__restrict__ aos, int da) {
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= m) return;
    uint32_t qi;
    if (off) {  // the segment holding e: off[qi] <= e < off[qi + 1]
        uint32_t lo = 0, hi = nq;
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (off[mid] <= e)
                lo = mid;
            else
                hi = mid;
        }
        qi = lo;
    } else {
        qi = (uint32_t)(e / stride);
    }
    const int dim = sp.dim;
    const uint32_t id = ids[e];
    double *qd = (from_query ? from : to) + e * dim;
    double *nd = (from_query ? to : from) + e * dim;
    for (int c = 0; c < dim; ++c) {
        const double qv = q[(size_t)qi * dim + c];
        qd[c] = qv;
        nd[c] = id == kNoId ? qv : (aos ? aos[(uint64_t)id * da + c] : raw[(uint64_t)c * cap + id]);
    }
}

// ---------------------------------------------------------------------------------
// host side

bool feature_geometry(const DevSpace &sp, FeatGeom *g) {
    g->nmax = 0;
    switch (sp.kind) {
    case OMPL_GPU_SPACE_REALVECTOR:
        if (sp.dim < 1 || sp.dim > 16) return false;
        g->F = sp.dim <= 4 ? 4 : sp.dim <= 8 ? 8 : 16;
        return true;
    case OMPL_GPU_SPACE_SO3:
        if (sp.dim != 4) return false;
        g->F = 4;
        return true;
    case OMPL_GPU_SPACE_SE3:
        if (sp.dim != 7) return false;
        g->F = 7;
        return true;
    case OMPL_GPU_SPACE_KCHAIN:
        if (sp.dim < 1 || sp.dim > 16) return false;
        g->nmax = sp.dim <= 4 ? 4 : sp.dim <= 8 ? 8 : sp.dim <= 12 ? 12 : 16;
        g->F = 2 * g->nmax;
        return true;
    }
    return false;
}

int k_bucket(uint32_t k) {
    if (k <= 1) return 1;
    if (k <= 4) return 4;
    if (k <= 16) return 16;
    if (k <= 32) return 32;
    if (k <= 64) return 64;
    return 0;
}

namespace {

struct KnnPlan {
    bool stream;
    uint32_t chunks;      // tiled: grid.y ; stream: blocks per query
    uint32_t chunk_len;   // tiled only
    int K;
};

KnnPlan knn_plan(uint32_t nq, uint32_t k, uint64_t n_end, int num_cus) {
    KnnPlan p{};
    p.K = k_bucket(k);
    const uint64_t tiles = n_end / kTile;
    if (nq < kStreamMaxQ) {
        p.stream = true;
        p.chunks = (uint32_t)((n_end + 256 * kScanItems - 1) / (256 * kScanItems));
        if (p.chunks == 0) p.chunks = 1;
        return p;
    }
    p.stream = false;
    const uint64_t qblocks = (nq + kTile - 1) / kTile;
    const uint64_t target = (uint64_t)num_cus * 8;  // ~8 resident blocks per CU
    uint64_t S = (target + qblocks - 1) / qblocks;
    S = std::max<uint64_t>(1, std::min<uint64_t>(S, std::max<uint64_t>(tiles, 1)));
    const uint64_t tiles_per_chunk = (tiles + S - 1) / S;
    p.chunk_len = (uint32_t)(std::max<uint64_t>(tiles_per_chunk, 1) * kTile);
    p.chunks = (uint32_t)((n_end + p.chunk_len - 1) / p.chunk_len);
    if (p.chunks == 0) p.chunks = 1;
    return p;
}

// ---- dispatch over (space, feature bucket) then K -------------------------------
template <int SP, int F, int NMAX, int K>
hipError_t run_knn_k(const DevSpace &sp, const KnnPlan &p, const double *feat, uint64_t cap, uint64_t n_end,
                     const double *qf, uint32_t nq, uint32_t k, double *od, uint32_t *oi, void *ws,
                     hipStream_t st) {
    double *pd = (double *)ws;
    if (p.stream) {
        const size_t np = (size_t)nq * p.chunks * K;
        uint32_t *pi = (uint32_t *)(pd + np);
        timer_begin(st, "knn_stream_kernel");
        hipLaunchKernelGGL((knn_stream_kernel<SP, F, NMAX, K>), dim3(p.chunks, nq), dim3(256), 0, st, feat, cap,
                           n_end, qf, sp, pd, pi);
        timer_end(st);
        hipLaunchKernelGGL((knn_stream_merge_kernel<K>), dim3(nq), dim3(256), 0, st, pd, pi, p.chunks, od, oi, k);
        return hipGetLastError();
    }
    const dim3 grid((nq + kTile - 1) / kTile, p.chunks);
    if (p.chunks == 1) {
        timer_begin(st, "knn_tiled_kernel");
        hipLaunchKernelGGL((knn_tiled_kernel<SP, F, NMAX, K>), grid, dim3(kTile), 0, st, feat, cap, n_end, qf, nq,
                           p.chunk_len, sp, od, oi, k);
        timer_end(st);
        return hipGetLastError();
    }
    const size_t np = (size_t)nq * p.chunks * K;
    uint32_t *pi = (uint32_t *)(pd + np);
    timer_begin(st, "knn_tiled_kernel");
    hipLaunchKernelGGL((knn_tiled_kernel<SP, F, NMAX, K>), grid, dim3(kTile), 0, st, feat, cap, n_end, qf, nq,
                       p.chunk_len, sp, pd, pi, (uint32_t)K);
    timer_end(st);
    hipLaunchKernelGGL((knn_merge_kernel<K>), dim3((nq + 255) / 256), dim3(256), 0, st, pd, pi, p.chunks, nq, od,
                       oi, k);
    return hipGetLastError();
}

template <int SP, int F, int NMAX>
hipError_t run_knn(const DevSpace &sp, const KnnPlan &p, const double *feat, uint64_t cap, uint64_t n_end,
                   const double *qf, uint32_t nq, uint32_t k, double *od, uint32_t *oi, void *ws, hipStream_t st) {
    switch (p.K) {
    case 1: return run_knn_k<SP, F, NMAX, 1>(sp, p, feat, cap, n_end, qf, nq, k, od, oi, ws, st);
    case 4: return run_knn_k<SP, F, NMAX, 4>(sp, p, feat, cap, n_end, qf, nq, k, od, oi, ws, st);
    case 16: return run_knn_k<SP, F, NMAX, 16>(sp, p, feat, cap, n_end, qf, nq, k, od, oi, ws, st);
    case 32: return run_knn_k<SP, F, NMAX, 32>(sp, p, feat, cap, n_end, qf, nq, k, od, oi, ws, st);
    case 64: return run_knn_k<SP, F, NMAX, 64>(sp, p, feat, cap, n_end, qf, nq, k, od, oi, ws, st);
    }
    return hipErrorInvalidValue;
}

#define OMPL_AMD_SPACE_DISPATCH(FN, ...)                                                              \
    switch (sp.kind) {                                                                               \
    case OMPL_GPU_SPACE_REALVECTOR:                                                                  \
        if (g.F == 4) return FN<OMPL_GPU_SPACE_REALVECTOR, 4, 0>(__VA_ARGS__);                       \
        if (g.F == 8) return FN<OMPL_GPU_SPACE_REALVECTOR, 8, 0>(__VA_ARGS__);                       \
        return FN<OMPL_GPU_SPACE_REALVECTOR, 16, 0>(__VA_ARGS__);                                    \
    case OMPL_GPU_SPACE_SO3: return FN<OMPL_GPU_SPACE_SO3, 4, 0>(__VA_ARGS__);                       \
    case OMPL_GPU_SPACE_SE3: return FN<OMPL_GPU_SPACE_SE3, 7, 0>(__VA_ARGS__);                       \
    case OMPL_GPU_SPACE_KCHAIN:                                                                      \
        if (g.nmax == 4) return FN<OMPL_GPU_SPACE_KCHAIN, 8, 4>(__VA_ARGS__);                        \
        if (g.nmax == 8) return FN<OMPL_GPU_SPACE_KCHAIN, 16, 8>(__VA_ARGS__);                       \
        if (g.nmax == 12) return FN<OMPL_GPU_SPACE_KCHAIN, 24, 12>(__VA_ARGS__);                     \
        return FN<OMPL_GPU_SPACE_KCHAIN, 32, 16>(__VA_ARGS__);                                       \
    }                                                                                                \
    return hipErrorInvalidValue;

template <int SP, int F, int NMAX>
hipError_t run_radius_count(const DevSpace &sp, const RadiusPlan &p, const double *feat, uint64_t cap,
                            uint64_t n_end, const double *qf, uint32_t nq, double r, uint32_t *counts,
                            hipStream_t st) {
    if (p.stream) {
        hipLaunchKernelGGL((radius_stream_kernel<SP, F, NMAX, false>), dim3((p.chunks + 3) / 4, nq), dim3(256), 0,
                           st, feat, cap, n_end, qf, p.chunks, sp, r, counts, nullptr, nullptr, nullptr);
    } else {
        hipLaunchKernelGGL((radius_tiled_kernel<SP, F, NMAX, false>), dim3((nq + kTile - 1) / kTile, p.chunks),
                           dim3(kTile), 0, st, feat, cap, n_end, qf, nq, p.chunk_len, p.chunks, sp, r, counts,
                           nullptr, nullptr, nullptr);
    }
    return hipGetLastError();
}

template <int SP, int F, int NMAX>
hipError_t run_radius_fill(const DevSpace &sp, const RadiusPlan &p, const double *feat, uint64_t cap,
                           uint64_t n_end, const double *qf, uint32_t nq, double r, const uint64_t *offsets,
                           uint32_t *ids, double *dists, hipStream_t st) {
    if (p.stream) {
        hipLaunchKernelGGL((radius_stream_kernel<SP, F, NMAX, true>), dim3((p.chunks + 3) / 4, nq), dim3(256), 0,
                           st, feat, cap, n_end, qf, p.chunks, sp, r, nullptr, offsets, ids, dists);
    } else {
        hipLaunchKernelGGL((radius_tiled_kernel<SP, F, NMAX, true>), dim3((nq + kTile - 1) / kTile, p.chunks),
                           dim3(kTile), 0, st, feat, cap, n_end, qf, nq, p.chunk_len, p.chunks, sp, r, nullptr,
                           offsets, ids, dists);
    }
    return hipGetLastError();
}

}  // namespace

size_t knn_workspace_bytes(const DevSpace &sp, const FeatGeom &g, uint32_t nq, uint32_t k, uint64_t n_end,
                           int num_cus) {
    (void)sp;
    (void)g;
    const KnnPlan p = knn_plan(nq, k, n_end, num_cus);
    if (!p.stream && p.chunks == 1) return 0;
    return (size_t)nq * p.chunks * p.K * (sizeof(double) + sizeof(uint32_t));
}

hipError_t launch_knn(const DevSpace &sp, const FeatGeom &g, const double *feat, uint64_t cap, uint64_t n_end,
                      const double *qf, uint32_t nq, uint32_t k, double *od, uint32_t *oi, void *ws, size_t ws_bytes,
                      int num_cus, hipStream_t st) {
    if (nq == 0 || k == 0) return hipSuccess;
    const KnnPlan p = knn_plan(nq, k, n_end, num_cus);
    if (p.K == 0) return hipErrorInvalidValue;
    if (knn_workspace_bytes(sp, g, nq, k, n_end, num_cus) > ws_bytes) return hipErrorInvalidValue;
    OMPL_AMD_SPACE_DISPATCH(run_knn, sp, p, feat, cap, n_end, qf, nq, k, od, oi, ws, st)
}

hipError_t launch_knn_bounded(const DevSpace &sp, const FeatGeom &g, const double *feat, uint64_t cap,
                              uint64_t n_end, const double *qf, const uint32_t *list, const uint32_t *d_nlist,
                              uint32_t k, double *od, uint32_t *oi, uint32_t *counts, double *cand_d,
                              uint32_t *cand_i, int num_cus, hipStream_t st, unsigned long long *stats) {
    if (k == 0) return hipSuccess;
    OMPL_AMD_SPACE_DISPATCH(run_knn_bounded, sp, feat, cap, n_end, qf, list, d_nlist, k, od, oi, counts, cand_d, cand_i,
                            num_cus, st, stats)
}

RadiusPlan radius_plan(uint32_t nq, uint64_t n_end, int num_cus) {
    RadiusPlan p{};
    if (nq < kStreamMaxQ) {
        p.stream = true;
        p.chunk_len = 64 * kStreamItems;
        p.chunks = (uint32_t)std::max<uint64_t>(1, (n_end + p.chunk_len - 1) / p.chunk_len);
        return p;
    }
    const KnnPlan kp = knn_plan(nq, 1, n_end, num_cus);
    p.stream = false;
    p.chunk_len = kp.chunk_len;
    p.chunks = kp.chunks;
    return p;
}

hipError_t launch_radius_count(const DevSpace &sp, const FeatGeom &g, const RadiusPlan &p, const double *feat,
                               uint64_t cap, uint64_t n_end, const double *qf, uint32_t nq, double r,
                               uint32_t *counts, hipStream_t st) {
    OMPL_AMD_SPACE_DISPATCH(run_radius_count, sp, p, feat, cap, n_end, qf, nq, r, counts, st)
}

hipError_t launch_radius_fill(const DevSpace &sp, const FeatGeom &g, const RadiusPlan &p, const double *feat,
                              uint64_t cap, uint64_t n_end, const double *qf, uint32_t nq, double r,
                              const uint64_t *offsets, uint32_t *ids, double *dists, hipStream_t st) {
    OMPL_AMD_SPACE_DISPATCH(run_radius_fill, sp, p, feat, cap, n_end, qf, nq, r, offsets, ids, dists, st)
}

hipError_t launch_features(const DevSpace &sp, const FeatGeom &g, const double *raw, uint32_t n, double *feat,
                           hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(features_kernel, dim3((n + 255) / 256), dim3(256), 0, st, sp, g, raw, n, feat);
    return hipGetLastError();
}

hipError_t launch_store_soa(const double *aos, uint32_t n, int width, double *soa, uint64_t cap, uint64_t first,
                            hipStream_t st) {
    if (n == 0) return hipSuccess;
    const uint64_t t = (uint64_t)n * width;
    hipLaunchKernelGGL(store_soa_kernel, dim3((unsigned)((t + 255) / 256)), dim3(256), 0, st, aos, n, width, soa, cap,
                       first);
    return hipGetLastError();
}

hipError_t launch_segment_rank_sort(const uint64_t *offsets, const uint32_t *in_i, const double *in_d, uint32_t nq,
                                    uint32_t *out_i, double *out_d, hipStream_t st, uint32_t in_stride) {
    if (nq == 0) return hipSuccess;
    hipLaunchKernelGGL(segment_rank_sort_kernel, dim3(nq), dim3(64), 0, st, offsets, in_i, in_d, out_i, out_d,
                       in_stride);
    return hipGetLastError();
}

// CSR segment of every edge: qidx[e] = q for off[q] <= e < min(off[q + 1], m); edges past
// off[nq] get kNoId (left unwritten by edges_copy_kernel).  A wave per segment (grid-stride),
// so a query with 10^5 neighbours is written 64 entries per step, not by one lane.
__global__ void edge_query_kernel(const uint64_t *__restrict__ off, uint32_t nq, uint64_t m,
                                  uint32_t *__restrict__ qidx) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nw = (gridDim.x * blockDim.x) >> 6;
    for (uint32_t q = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; q <= nq; q += nw) {
        const uint64_t e0 = off[q], e1 = q < nq ? min(off[q + 1], m) : m;
        const uint32_t v = q < nq ? q : kNoId;
        for (uint64_t e = e0 + lane; e < e1; e += 64) qidx[e] = v;
    }
}

// thread per (edge, coordinate): consecutive threads write consecutive reals of the AoS
// endpoint rows (edges_kernel's per-edge threads wrote 56-B strided rows and binary-searched
// the CSR per edge)
__global__ void edges_copy_kernel(const double *__restrict__ raw, uint64_t cap, int dim, const double *__restrict__ q,
                                  const uint32_t *__restrict__ qidx, const uint32_t *__restrict__ ids,
                                  uint32_t stride, uint64_t m, int from_query, double *__restrict__ from,
                                  double *__restrict__ to, const double *__restrict__ aos, int da) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= m * (uint64_t)dim) return;
    const uint64_t e = t / (uint64_t)dim;
    const int c = (int)(t - e * (uint64_t)dim);
    const uint32_t qi = qidx ? qidx[e] : (uint32_t)(e / stride);
    if (qi == kNoId) return;  // past the CSR's last segment
    const uint32_t id = ids[e];
    const double qv = q[(size_t)qi * dim + c];
    (from_query ? from : to)[t] = qv;
    (from_query ? to : from)[t] = id == kNoId ? qv : (aos ? aos[(uint64_t)id * da + c] : raw[(uint64_t)c * cap + id]);
}

hipError_t launch_edge_query(const uint64_t *offsets, uint32_t nq, uint64_t m, uint32_t *qidx, hipStream_t st) {
    if (m == 0) return hipSuccess;
    hipLaunchKernelGGL(edge_query_kernel, dim3(std::min<uint32_t>(nq / 4 + 1, 8192)), dim3(256), 0, st, offsets, nq, m,
                       qidx);
    return hipGetLastError();
}

hipError_t launch_edges(const DevSpace &sp, const double *raw, uint64_t cap, const double *q, uint32_t nq,
                        const uint64_t *offsets, const uint32_t *ids, uint32_t stride, uint64_t m, int from_query,
                        double *from, double *to, hipStream_t st, const double *aos, int da, uint32_t *qidx) {
    if (m == 0) return hipSuccess;
    if (offsets && !qidx) {  // no scratch: the per-edge search form
        hipLaunchKernelGGL(edges_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, st, sp, raw, cap, q, nq,
                           offsets, ids, stride, m, from_query, from, to, aos, da);
        return hipGetLastError();
    }
    if (offsets)
        hipLaunchKernelGGL(edge_query_kernel, dim3(std::min<uint32_t>(nq / 4 + 1, 8192)), dim3(256), 0, st, offsets, nq,
                           (uint64_t)m, qidx);
    const uint64_t n = m * (uint64_t)sp.dim;
    hipLaunchKernelGGL(edges_copy_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, raw, cap, sp.dim, q,
                       offsets ? qidx : nullptr, ids, stride, m, from_query, from, to, aos, da);
    return hipGetLastError();
}

__global__ void aos_rows_kernel(const double *__restrict__ soa, uint64_t cap, int dim, int da, uint64_t first,
                                uint64_t n, double *__restrict__ aos) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;  // one thread per (state, column)
    if (t >= n * da) return;
    const uint64_t i = first + t / da;
    const int c = (int)(t % da);
    aos[i * da + c] = c < dim ? soa[(uint64_t)c * cap + i] : 0.0;
}

hipError_t launch_aos_rows(const double *soa, uint64_t cap, int dim, int da, uint64_t first, uint64_t n, double *aos,
                           hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(aos_rows_kernel, dim3((unsigned)((n * da + 255) / 256)), dim3(256), 0, st, soa, cap, dim, da,
                       first, n, aos);
    return hipGetLastError();
}

// tree-sharded kNN / nearestR: per-shard results of the same queries merged by rank placement
// (merge path): every element's place in the merged order is its index in its own sorted list
// plus, for every other list, the number of that list's elements ordered before it (a binary
// search) — no per-thread list heads, no data-dependent loop over the lists.  Keys are (distance,
// id), ids are global and distinct across shards, so the places are a permutation.
__device__ __forceinline__ uint32_t count_before(const double *__restrict__ d, const uint32_t *__restrict__ ids,
                                                 uint64_t b, uint32_t L, double x, uint32_t xi) {
    uint32_t lo = 0, hi = L;  // first position whose key is not below (x, xi)
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (lex_less(d[b + mid], ids[b + mid], x, xi))
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}

// lists x nq x k, each sorted by (distance, id), missing = (+inf, kNoId) at the end: thread per
// (query, list, entry)
__global__ __launch_bounds__(256) void topk_merge_kernel(const double *__restrict__ d, const uint32_t *__restrict__ ids,
                                                         uint32_t lists, uint32_t nq, uint32_t k,
                                                         double *__restrict__ od, uint32_t *__restrict__ oi) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (uint64_t)nq * lists * k) return;
    const uint32_t j = (uint32_t)(t % k), w = (uint32_t)((t / k) % lists), q = (uint32_t)(t / ((uint64_t)k * lists));
    auto base = [&](uint32_t l) { return ((uint64_t)l * nq + q) * k; };
    const double x = d[base(w) + j];
    const uint32_t xi = ids[base(w) + j];
    if (xi != kNoId) {
        uint32_t rank = j;
        for (uint32_t l = 0; l < lists; ++l)
            if (l != w) rank += count_before(d, ids, base(l), k, x, xi);
        if (rank < k) {
            od[(size_t)q * k + rank] = x;
            oi[(size_t)q * k + rank] = xi;
        }
    }
    if (w == 0) {  // the entries past every list's valid ones are missing
        uint32_t valid = 0;
        for (uint32_t l = 0; l < lists; ++l) valid += count_before(d, ids, base(l), k, __builtin_inf(), kNoId);
        if (j >= valid) {
            od[(size_t)q * k + j] = __builtin_inf();
            oi[(size_t)q * k + j] = kNoId;
        }
    }
}

hipError_t launch_topk_merge(const double *d, const uint32_t *ids, uint32_t lists, uint32_t nq, uint32_t k, double *od,
                             uint32_t *oi, hipStream_t st) {
    if (nq == 0 || k == 0) return hipSuccess;
    if (lists == 0 || lists > 64) return hipErrorInvalidValue;
    const uint64_t n = (uint64_t)nq * lists * k;
    hipLaunchKernelGGL(topk_merge_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, d, ids, lists, nq, k, od,
                       oi);
    return hipGetLastError();
}

// lists CSR results of the same nq queries (list l: offsets offs[l][0..nq], payload ids / d at
// l * stride, each segment sorted by (distance, id)) -> one CSR: out_off[q] = sum_l offs[l][q]
// (the offsets are exclusive prefix sums), segment q holding the union in (distance, id) order.
// Block per query.
__global__ __launch_bounds__(64) void csr_merge_kernel(const uint64_t *__restrict__ offs, uint32_t lists, uint32_t nq,
                                                       const uint32_t *__restrict__ ids, const double *__restrict__ d,
                                                       uint64_t stride, uint64_t *__restrict__ out_off,
                                                       uint32_t *__restrict__ out_i, double *__restrict__ out_d) {
    const uint32_t q = blockIdx.x;
    uint64_t ob = 0;
    for (uint32_t l = 0; l < lists; ++l) ob += offs[(uint64_t)l * (nq + 1) + q];
    if (threadIdx.x == 0) {
        out_off[q] = ob;
        if (q + 1 == nq) {
            uint64_t e = 0;
            for (uint32_t l = 0; l < lists; ++l) e += offs[(uint64_t)l * (nq + 1) + nq];
            out_off[nq] = e;
        }
    }
    for (uint32_t w = 0; w < lists; ++w) {
        const uint64_t bw = offs[(uint64_t)w * (nq + 1) + q];
        const uint32_t Lw = (uint32_t)(offs[(uint64_t)w * (nq + 1) + q + 1] - bw);
        for (uint32_t j = threadIdx.x; j < Lw; j += blockDim.x) {
            const double x = d[(uint64_t)w * stride + bw + j];
            const uint32_t xi = ids[(uint64_t)w * stride + bw + j];
            uint64_t rank = j;
            for (uint32_t l = 0; l < lists; ++l) {
                if (l == w) continue;
                const uint64_t bl = offs[(uint64_t)l * (nq + 1) + q];
                const uint32_t Ll = (uint32_t)(offs[(uint64_t)l * (nq + 1) + q + 1] - bl);
                rank += count_before(d, ids, (uint64_t)l * stride + bl, Ll, x, xi);
            }
            out_d[ob + rank] = x;
            out_i[ob + rank] = xi;
        }
    }
}

hipError_t launch_csr_merge(const uint64_t *offs, uint32_t lists, uint32_t nq, const uint32_t *ids, const double *d,
                            uint64_t stride, uint64_t *out_off, uint32_t *out_i, double *out_d, hipStream_t st) {
    if (nq == 0) return hipMemsetAsync(out_off, 0, sizeof(uint64_t), st);  // out_off[0]: no entries
    hipLaunchKernelGGL(csr_merge_kernel, dim3(nq), dim3(64), 0, st, offs, lists, nq, ids, d, stride, out_off, out_i,
                       out_d);
    return hipGetLastError();
}

hipError_t launch_steer(const DevSpace &sp, const double *raw, uint64_t cap, const double *q, uint32_t nq,
                        const uint32_t *nearest, uint32_t stride, double maxd, double *from, double *to,
                        hipStream_t st) {
    if (nq == 0) return hipSuccess;
    if (sp.kind == OMPL_GPU_SPACE_SE3 && sp.dim == 7)
        hipLaunchKernelGGL((steer_kernel<OMPL_GPU_SPACE_SE3, 7>), dim3((nq + 255) / 256), dim3(256), 0, st, sp, raw, cap,
                           q, nq, nearest, stride, maxd, from, to);
    else
        hipLaunchKernelGGL((steer_kernel<0, 0>), dim3((nq + 255) / 256), dim3(256), 0, st, sp, raw, cap, q, nq, nearest,
                           stride, maxd, from, to);
    return hipGetLastError();
}

}  // namespace ompl_amd
