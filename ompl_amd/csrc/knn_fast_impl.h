// knn_fast_impl.h — exact batched kNN via an fp32 screen and an fp64 certificate (gfx950).
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
//      Inside a tile, for SE3 the chord bound fma(w1, c, w0 |t|) (c <= theta) is tested
//      first and the angle polynomial evaluated only when some lane of the wave can still
//      beat the K2-th distance.
//   3. certify (fp64): merge the lists, recompute the K2 candidates exactly in the
//      reference's operation order, keep the k best by (distance, id), and prove that no
//      element outside the list can enter: |d32 - d64| <= e for every element, so if the
//      exact k-th distance + e < the list's K2-th fp32 distance L the answer is exact.
//      Queries that fail the proof are listed; the caller re-runs them on the exact fp64
//      path (knn.hip), so the results always equal the exact path's.
//
// Error bound e (u = 2^-24, B = max |coordinate|, D = dims, L as above), doubled for slack:
//   translation / R^n : 6 sqrt(D) u B + 6 u L   (fp32 conversion + sum of squares + sqrt)
//   SE3 rotation      : the screen measures the rotation by the chord, theta = 2 asin(c / 2),
//                       c = min(|p - q|, |p + q|), which is well conditioned near theta = 0
//                       (acos(|p.q|) in fp32 is not: its error there is sqrt(12 u) ~ 1e-3).  For
//                       unit quaternions 2 asin(c / 2) = acos(|p.q|) exactly; with norms
//                       |p|^2 = 1 + eta_p, |q|^2 = 1 + eta_q the two differ by at most
//                       2.25 sqrt(|eta_p + eta_q| / 2) (acos is 1/2-Hoelder with constant pi/sqrt 2);
//                       + 4.5e-5 (the reference returns 0 for |dot| > 1 - 1e-9,
//                       SO3StateSpace.cpp:258-260) + 2e-6 (fp32 evaluation; chord_theta's
//                       polynomial <= 1.1e-7, with its fp32 evaluation <= 1.8e-7)
//   SO3 rotation      : 1.1 sqrt(2 * 6u) + 1e-6 + 4.5e-5 (the chunked screen keeps acos(|dot|))
#pragma once
// Included by one translation unit per space (knn_fast_{se3,so3,rv}.hip) so that the
// template instantiations compile in parallel; knn_fast.hip holds the dispatch.
#include <hip/hip_runtime.h>
#include <cstring>  // (rocPRIM block primitives need memset declared)
#include <rocprim/rocprim.hpp>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <type_traits>

#include "feat_dist.h"
#include "kernels.h"
#include "topk.h"

namespace ompl_amd {

namespace {

constexpr double kU = 5.9604644775390625e-08;  // 2^-24

template <int SP, int F>
struct Geo {
    static constexpr int FS = SP == OMPL_GPU_SPACE_SE3 ? 8 : F;  // fp32 row width (LDS / queries)
    static constexpr int NB = SP == OMPL_GPU_SPACE_SE3 ? 7 : F;  // box dims (every stored coordinate)
    static constexpr int R = SP == OMPL_GPU_SPACE_SE3 ? 7 : F;   // rows of the fp32 SoA store
    // box record: lo[NB], hi[NB]; SE3 adds eta (largest |q|^2 - 1 >= 0 of the quaternions) + pad
    static constexpr int BW = SP == OMPL_GPU_SPACE_SE3 ? 16 : 2 * F;
};

// one tile's R rows for this lane (position 64 t + lane) from the tile-blocked store (kernels.h
// blk_index): a 16-byte load per full segment of 4 rows, one 4 / 8 / 12-byte load for the rest
template <int R, typename T>
__device__ __forceinline__ void load_blk(const T *__restrict__ rows, uint32_t t, int lane, T (&x)[R]) {
    static_assert(sizeof(T) == 4, "32-bit rows");
    const T *b = rows + (uint64_t)t * (64 * R);
#pragma unroll
    for (int s = 0; s < R / 4; ++s) {
        const uint4 v = *reinterpret_cast<const uint4 *>(b + s * 256 + lane * 4);
        x[4 * s] = __builtin_bit_cast(T, v.x);
        x[4 * s + 1] = __builtin_bit_cast(T, v.y);
        x[4 * s + 2] = __builtin_bit_cast(T, v.z);
        x[4 * s + 3] = __builtin_bit_cast(T, v.w);
    }
    constexpr int Q = R % 4, S = R / 4;
    if constexpr (Q == 1) {
        x[R - 1] = b[S * 256 + lane];
    } else if constexpr (Q == 2) {
        const uint2 v = *reinterpret_cast<const uint2 *>(b + S * 256 + lane * 2);
        x[R - 2] = __builtin_bit_cast(T, v.x);
        x[R - 1] = __builtin_bit_cast(T, v.y);
    } else if constexpr (Q == 3) {
        const T *q = b + S * 256 + lane * 3;
        x[R - 3] = q[0];
        x[R - 2] = q[1];
        x[R - 1] = q[2];
    }
}

__device__ __forceinline__ float abs1(float x) {  // |x| clamped to 1; NaN stays NaN
    float a = fabsf(x);
    return a > 1.f ? 1.f : a;
}

// 30-bit Morton key of the key coordinates c[0..nkey); NaN -> max key
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

// key coordinates of a state given as its R stored coordinates (SE3: x y z qx qy qz qw):
// SE3 keys on the translation and the vector part of the sign-canonical (w >= 0)
// quaternion, so that tiles are compact in rotation too; R^n on its first coordinates.
template <int SP>
__device__ __forceinline__ void key_coords(const float *x, float *c, int nkey) {
    if constexpr (SP == OMPL_GPU_SPACE_SE3) {
        const float sg = x[6] < 0.f ? -1.f : 1.f;
        c[0] = x[0]; c[1] = x[1]; c[2] = x[2];
        c[3] = sg * x[3]; c[4] = sg * x[4]; c[5] = sg * x[5];
    } else {
        for (int d = 0; d < nkey; ++d) c[d] = x[d];
    }
}

// KinematicChain screening rows: the joint positions P_i = (sum_{j<=i} cos t_j, sum_{j<=i} sin t_j)
// from the cumulative cos / sin features (summed in fp64, then rounded), so that the chain
// distance (demos/KinematicChain.h:105-124) becomes link * sum_i |P_i(a) - P_i(b)|
template <int NM>
__device__ __forceinline__ void chain_positions(const double *feat, float *o) {
    double cx = 0.0, cy = 0.0;
#pragma unroll
    for (int i = 0; i < NM; ++i) {
        cx += feat[i];
        cy += feat[NM + i];
        o[i] = (float)cx;
        o[NM + i] = (float)cy;
    }
}

// ---- queries: fp32 rows, keys, order ---------------------------------------------------
// home leaf of coordinates c (the box coordinates of Geo::NB) in the k-d tree of the sorted store
__device__ __forceinline__ uint32_t kd_home_tile(const float *c, const KdNode *__restrict__ nodes, uint32_t ntiles) {
    uint32_t node = 0, t0 = 0, tiles = ntiles;
    for (int depth = 0; tiles > 1 && depth < 40; ++depth) {
        const KdNode nd = nodes[node];
        if (c[nd.dim] < nd.split) {
            tiles = nd.left_tiles;
            node = node + 1;
        } else {
            t0 += nd.left_tiles;
            tiles -= nd.left_tiles;
            node = nd.right;
        }
    }
    return t0;
}

template <int SP, int F>
__global__ void query_rows_kernel(const double *__restrict__ qf, uint32_t nq, FastBounds b, float *__restrict__ q32u,
                                  uint32_t *__restrict__ keys, uint32_t *__restrict__ idx,
                                  const KdNode *__restrict__ nodes, uint32_t ntiles, uint32_t *__restrict__ qcnt = nullptr,
                                  uint32_t *__restrict__ slot = nullptr) {
    constexpr int FS = Geo<SP, F>::FS;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
#pragma unroll
    for (int r = 0; r < 3; ++r)
        if (b.zero[r])
            for (uint32_t t = i; t < b.nzero[r]; t += gridDim.x * blockDim.x) b.zero[r][t] = 0u;
    if (i >= nq) return;
    const double *s = qf + (size_t)i * F;
    float o[FS];
    float x[kKeyDims + 1];
    if constexpr (SP == OMPL_GPU_SPACE_SE3) {
        o[0] = (float)s[0]; o[1] = (float)s[1]; o[2] = (float)s[2];
        o[4] = (float)s[3]; o[5] = (float)s[4]; o[6] = (float)s[5]; o[7] = (float)s[6];
        // slot 3: the quaternion's norm excess max(|q|^2 - 1, 0), used by the box bound
        float n2 = o[4] * o[4];
        n2 = fmaf(o[5], o[5], n2);
        n2 = fmaf(o[6], o[6], n2);
        n2 = fmaf(o[7], o[7], n2);
        o[3] = fmaxf(n2 - 1.f, 0.f) * 1.00001f;
        x[0] = o[0]; x[1] = o[1]; x[2] = o[2]; x[3] = o[4]; x[4] = o[5]; x[5] = o[6]; x[6] = o[7];
    } else if constexpr (SP == OMPL_GPU_SPACE_KCHAIN) {
        chain_positions<FS / 2>(s, o);
    } else {
        for (int f = 0; f < FS; ++f) o[f] = (float)s[f];
        for (int d = 0; d < b.nkey; ++d) x[d] = o[d];
    }
    for (int f = 0; f < FS; ++f) q32u[(size_t)i * FS + f] = o[f];
    if (SP == OMPL_GPU_SPACE_KCHAIN && !(nodes && ntiles > 1)) {
        keys[i] = 0u;  // no sorted store: the brute-force wave scan needs no order
    } else if (nodes && ntiles > 1) {
        // order by home leaf: the box coordinates, quaternion sign-canonical as in the store
        float c[Geo<SP, F>::NB];
        if constexpr (SP == OMPL_GPU_SPACE_SE3) {
            const float sg = x[6] < 0.f ? -1.f : 1.f;
            c[0] = x[0]; c[1] = x[1]; c[2] = x[2];
            c[3] = sg * x[3]; c[4] = sg * x[4]; c[5] = sg * x[5]; c[6] = sg * x[6];
        } else {
            for (int d = 0; d < Geo<SP, F>::NB; ++d) c[d] = o[d];
        }
        const uint32_t k = kd_home_tile(c, nodes, ntiles);
        keys[i] = k;
        if (qcnt) slot[i] = atomicAdd(&qcnt[k], 1u);  // the counting sort's count (home_place_kernel)
    } else {
        float c[kKeyDims];
        key_coords<SP>(x, c, b.nkey);
        keys[i] = morton_key(c, b);
    }
    idx[i] = i;
}

// queries sorted by home tile.  Home-tile keys (< bins = the k-d tiles) take a counting sort over
// the whole grid — a count kernel whose atomicAdd also hands each query its slot inside its tile,
// a one-block exclusive scan of the bins, a scatter: three launches; queries of one tile land in
// any order, which only changes how the walk's groups are formed, never a result.  Wider keys
// (32-bit Morton codes when there is no k-d tree; the tail's Morton / home keys) are counted by
// their top 16 bits (key >> shift): 65,536 cells of the Morton curve, order inside a cell
// arbitrary — a coarser curve, still exact (tile order never changes a result).  (Measured and
// rejected in round 3: a one-block LDS counting sort, one CU doing every atomic and write: nn
// phase 1.41 -> 1.48 ms.)
__global__ void home_count_kernel(const uint32_t *__restrict__ keys, uint32_t nq, uint32_t *__restrict__ cnt,
                                  uint32_t *__restrict__ slot, int shift) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nq) slot[i] = atomicAdd(&cnt[keys[i] >> shift], 1u);
}
// exclusive scan of the bin counts in two levels: each block of 1,024 bins in place (coalesced,
// one block scan) with its total to bsum, then the block totals by one block; the scatter adds
// both.  (A single block looping over the 156 k bins of a 10^7-state store took 257 us.)
__global__ __launch_bounds__(1024) void home_scan_kernel(uint32_t *__restrict__ cnt, uint32_t bins,
                                                         uint32_t *__restrict__ bsum) {
    using BlockScan = rocprim::block_scan<uint32_t, 1024>;
    __shared__ typename BlockScan::storage_type sh;
    const uint32_t b = blockIdx.x * 1024 + threadIdx.x;
    const uint32_t c = b < bins ? cnt[b] : 0u;
    uint32_t pre = 0, tot = 0;
    BlockScan().exclusive_scan(c, pre, 0u, tot, sh);
    if (b < bins) cnt[b] = pre;
    if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}
__global__ __launch_bounds__(1024) void home_scan_blocks_kernel(uint32_t *__restrict__ bsum, uint32_t nb) {
    using BlockScan = rocprim::block_scan<uint32_t, 1024>;
    __shared__ typename BlockScan::storage_type sh;
    uint32_t run = 0;
    for (uint32_t b0 = 0; b0 < nb; b0 += 1024) {  // uniform trip count
        const uint32_t b = b0 + threadIdx.x;
        const uint32_t c = b < nb ? bsum[b] : 0u;
        uint32_t pre = 0, tot = 0;
        BlockScan().exclusive_scan(c, pre, 0u, tot, sh);
        __syncthreads();
        if (b < nb) bsum[b] = run + pre;
        run += tot;
    }
}
__global__ void home_scatter_kernel(const uint32_t *__restrict__ keys, const uint32_t *__restrict__ idx,
                                    const uint32_t *__restrict__ slot, uint32_t nq, const uint32_t *__restrict__ start,
                                    const uint32_t *__restrict__ bsum, uint32_t *__restrict__ keys2,
                                    uint32_t *__restrict__ perm, int shift) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nq) return;
    const uint32_t k = keys[i], c = k >> shift, p = bsum[c >> 10] + start[c] + slot[i];
    keys2[p] = k;
    perm[p] = idx[i];
}
inline size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }
// The home-key sort over the store's persistent bins (SortedStore::qcount: counts | start | block
// sums), which stay zero between calls — zeroed once when allocated, and by home_bins_scan_kernel
// as it reads them: query_rows_kernel counts (slot = its atomicAdd), the scan turns each block of
// 1,024 counts into exclusive prefixes in start[] with the block's total in bsum, and
// home_place_kernel puts each query at (prefix of the block totals) + start + slot, writing its
// key and its fp32 row in sorted order.  Three launches instead of six (count, two scans, scatter,
// row gather, and the zeroing of the bins).
__global__ __launch_bounds__(1024) void home_bins_scan_kernel(uint32_t *__restrict__ cnt, uint32_t bins,
                                                              uint32_t *__restrict__ start,
                                                              uint32_t *__restrict__ bsum) {
    using BlockScan = rocprim::block_scan<uint32_t, 1024>;
    __shared__ typename BlockScan::storage_type sh;
    const uint32_t b = blockIdx.x * 1024 + threadIdx.x;
    const uint32_t c = b < bins ? cnt[b] : 0u;
    uint32_t pre = 0, tot = 0;
    BlockScan().exclusive_scan(c, pre, 0u, tot, sh);
    if (b < bins) {
        start[b] = pre;
        cnt[b] = 0u;  // ready for the next call
    }
    if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}
template <int FS>
__global__ __launch_bounds__(256) void home_place_kernel(const uint32_t *__restrict__ keys,
                                                         const uint32_t *__restrict__ slot, uint32_t nq,
                                                         const uint32_t *__restrict__ start,
                                                         const uint32_t *__restrict__ bsum, uint32_t nb,
                                                         const float *__restrict__ q32u, uint32_t *__restrict__ keys2,
                                                         uint32_t *__restrict__ perm, float *__restrict__ q32) {
    __shared__ uint32_t boff[1024];  // exclusive prefix of the block totals, 1,024 at a time
    __shared__ uint32_t carry;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t k = i < nq ? keys[i] : 0u, kb = k >> 10;
    uint32_t off = 0;
    if (threadIdx.x == 0) carry = 0;
    for (uint32_t c0 = 0; c0 < nb; c0 += 1024) {  // uniform trip count
        __syncthreads();
        for (uint32_t t = threadIdx.x; t < 1024; t += blockDim.x) boff[t] = c0 + t < nb ? bsum[c0 + t] : 0u;
        __syncthreads();
        if (threadIdx.x == 0) {  // serial scan of <= 1,024 block totals (153 at 10^7 states)
            uint32_t run = carry;
            const uint32_t m = nb - c0 < 1024 ? nb - c0 : 1024;
            for (uint32_t t = 0; t < m; ++t) {
                const uint32_t v = boff[t];
                boff[t] = run;
                run += v;
            }
            carry = run;
        }
        __syncthreads();
        if (i < nq && kb >= c0 && kb < c0 + 1024) off = boff[kb - c0];
    }
    if (i >= nq) return;
    const uint32_t p = off + start[k] + slot[i];
    keys2[p] = k;
    perm[p] = i;
#pragma unroll
    for (int f = 0; f < FS; ++f) q32[(size_t)p * FS + f] = q32u[(size_t)i * FS + f];
}
// words of SortedStore::qcount for `tiles` bins: counts and start padded to 1,024, the block sums
inline size_t home_bins_words(uint32_t tiles) {
    const size_t nb = ((size_t)tiles + 1023) / 1024;
    return 2 * nb * 1024 + nb + 1;
}
constexpr int kCountBitsMax = 16;  // counting-sort cells of a wide key: its top 16 bits
// scratch of sort_home_keys without a caller's bin array: the slots, then 2^16 bins padded to
// 1,024 and their block sums
inline size_t home_sort_bytes(uint32_t n) {
    return align_up(4ull * std::max<uint32_t>(n, 1)) + 4ull * ((1u << kCountBitsMax) / 1024 * 1025 + 1);
}
// (keys, idx) -> (keys2, perm) ordered by key >> shift; shift = 0 with a caller's bin array
// (qcount, bins > every key: the k-d home tiles), else the key's top kCountBitsMax of key_bits
inline hipError_t sort_home_keys(char *ws, size_t ws_bytes, const uint32_t *keys, uint32_t *keys2,
                                 const uint32_t *idx, uint32_t *perm, uint32_t nq, int key_bits, hipStream_t st,
                                 uint32_t *qcount = nullptr, uint32_t bins = 0, bool zeroed = false) {
    // the counting sort (measured 0.081-0.083 ms against 0.113-0.115 ms for a radix sort of the
    // nn phase outside the walk on cfg3)
    if (nq == 0) return hipSuccess;
    if (ws_bytes < 4ull * nq) return hipErrorInvalidValue;
    uint32_t *slot = (uint32_t *)ws;
    int shift = 0;
    if (!(qcount && bins)) {  // own bins after the slots: the key's top bits
        if (ws_bytes < home_sort_bytes(nq)) return hipErrorInvalidValue;
        shift = std::max(0, key_bits - kCountBitsMax);
        bins = (uint32_t)((((uint64_t)1 << key_bits) - 1) >> shift) + 1;
        qcount = (uint32_t *)(ws + align_up(4ull * nq));
        zeroed = false;
    }
    if (!zeroed) {  // (query_rows_kernel zeroes the bins when the caller listed them)
        const hipError_t e = hipMemsetAsync(qcount, 0, 4ull * bins, st);
        if (e != hipSuccess) return e;
    }
    const uint32_t nb = (bins + 1023) / 1024;
    uint32_t *bsum = qcount + nb * 1024;  // qcount holds the bins padded to 1,024, then the block sums
    hipLaunchKernelGGL(home_count_kernel, dim3((nq + 255) / 256), dim3(256), 0, st, keys, nq, qcount, slot, shift);
    hipLaunchKernelGGL(home_scan_kernel, dim3(nb), dim3(1024), 0, st, qcount, bins, bsum);
    hipLaunchKernelGGL(home_scan_blocks_kernel, dim3(1), dim3(1024), 0, st, bsum, nb);
    hipLaunchKernelGGL(home_scatter_kernel, dim3((nq + 255) / 256), dim3(256), 0, st, keys, idx, slot, nq, qcount,
                       bsum, keys2, perm, shift);
    return hipGetLastError();
}

template <int FS>
__global__ void query_gather_kernel(const float *__restrict__ q32u, const uint32_t *__restrict__ perm, uint32_t nq,
                                    float *__restrict__ q32) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nq * (uint32_t)FS) return;
    const uint32_t qs = t / FS, f = t % FS;
    q32[t] = q32u[(size_t)perm[qs] * FS + f];
}

// queries ordered by key for the walks: the home-key sort when the store has a k-d tree
// (home_keys), else the counting sort on the Morton key's top bits + a row gather
template <int SP, int F>
hipError_t sort_queries(const double *qf64, uint32_t nq, const FastBounds &b, const SortedStore *ss, bool home_keys,
                        char *ws, size_t ws_bytes, float *q32u, uint32_t *keys, uint32_t *keys2, uint32_t *idx,
                        uint32_t *perm, float *q32, hipStream_t st, const KdNode *nodes, uint32_t ntiles) {
    constexpr int FS = Geo<SP, F>::FS;
    const dim3 b256(256);
    if (home_keys) {
        const uint32_t bins = ss->kd_tiles, nb = (bins + 1023) / 1024;
        uint32_t *cnt = ss->qcount, *start = cnt + (size_t)nb * 1024, *bsum = start + (size_t)nb * 1024;
        uint32_t *slot = (uint32_t *)ws;
        if (ws_bytes < 4ull * nq) return hipErrorInvalidValue;
        hipLaunchKernelGGL((query_rows_kernel<SP, F>), dim3((nq + 255) / 256), b256, 0, st, qf64, nq, b, q32u, keys, idx,
                           nodes, ntiles, cnt, slot);
        hipLaunchKernelGGL(home_bins_scan_kernel, dim3(nb), dim3(1024), 0, st, cnt, bins, start, bsum);
        hipLaunchKernelGGL((home_place_kernel<FS>), dim3((nq + 255) / 256), b256, 0, st, keys, slot, nq, start, bsum,
                           nb, q32u, keys2, perm, q32);
        return hipGetLastError();
    }
    hipLaunchKernelGGL((query_rows_kernel<SP, F>), dim3((nq + 255) / 256), b256, 0, st, qf64, nq, b, q32u, keys, idx,
                       nodes, ntiles, nullptr, nullptr);
    const hipError_t e = sort_home_keys(ws, ws_bytes, keys, keys2, idx, perm, nq, 32, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((query_gather_kernel<FS>), dim3((nq * FS + 255) / 256), b256, 0, st, q32u, perm, nq, q32);
    return hipGetLastError();
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

// fp32 screen of NS LDS states against the lane's query, in batches of kBatch: the cheap
// part (SE3 translation, SO3 dot, R^n squared distance) of a whole batch is computed from
// back-to-back LDS reads before any data-dependent branch, so one LDS latency is paid per
// batch, not per state.  Pre-rejects: SE3 translation vs tau, rotation |dot| vs ctau.
constexpr int kBatch = 8;

template <int SP, int FS, int K2, int NS, class IdOf>
__device__ __forceinline__ void screen_tile(const float *tile, const float *qf, float w0, float w0sq, float w1,
                                            int nlinks, IdOf id_of, TopK32<K2> &top, float &ctau) {
    const float4 *t4 = reinterpret_cast<const float4 *>(tile);
#pragma unroll 2
    for (int j0 = 0; j0 < NS; j0 += kBatch) {
        float v[kBatch];
        if constexpr (SP == OMPL_GPU_SPACE_SE3) {
#pragma unroll
            for (int u = 0; u < kBatch; ++u) {
                const float4 a = t4[(j0 + u) * 2];
                const float dx = a.x - qf[0], dy = a.y - qf[1], dz = a.z - qf[2];
                float t = dx * dx;
                t = fmaf(dy, dy, t);
                v[u] = fmaf(dz, dz, t);
            }
#pragma unroll
            for (int u = 0; u < kBatch; ++u) {
                if (v[u] * w0sq < top.tau2) {  // the translation term alone loses: skip the rotation
                    const float4 r = t4[(j0 + u) * 2 + 1];
                    const float p[4] = {r.x, r.y, r.z, r.w};
                    const float d = fmaf(w1, chord_angle(p, qf + 4), w0 * __builtin_amdgcn_sqrtf(v[u]));
                    const uint32_t id = id_of(j0 + u);
                    if (top.admits(d, id)) top.push(d, id);
                }
            }
        } else if constexpr (SP == OMPL_GPU_SPACE_SO3) {
#pragma unroll
            for (int u = 0; u < kBatch; ++u) {
                const float4 r = t4[j0 + u];
                float dot = r.x * qf[0];
                dot = fmaf(r.y, qf[1], dot);
                dot = fmaf(r.z, qf[2], dot);
                dot = fmaf(r.w, qf[3], dot);
                v[u] = abs1(dot);
            }
#pragma unroll
            for (int u = 0; u < kBatch; ++u) {
                if (v[u] > ctau) {
                    const float d = acos01(v[u]);
                    const uint32_t id = id_of(j0 + u);
                    if (top.admits(d, id)) {
                        top.push(d, id);
                        ctau = rot_threshold(top.d[K2 - 1], 1.f);
                    }
                }
            }
        } else if constexpr (SP == OMPL_GPU_SPACE_KCHAIN) {
            // w0 = link length; rows are joint positions (chain_positions)
            constexpr int NM = FS / 2;
#pragma unroll
            for (int u = 0; u < kBatch; ++u) {
                const float *t = tile + (j0 + u) * FS;
                float acc = 0.f;
#pragma unroll
                for (int i = 0; i < NM; ++i) {
                    if (i < nlinks) {
                        const float dx = t[i] - qf[i], dy = t[NM + i] - qf[NM + i];
                        acc += __builtin_amdgcn_sqrtf(fmaf(dy, dy, dx * dx));
                    }
                }
                v[u] = acc * w0;
            }
#pragma unroll
            for (int u = 0; u < kBatch; ++u) {
                const uint32_t id = id_of(j0 + u);
                if (top.admits(v[u], id)) top.push(v[u], id);
            }
        } else {
#pragma unroll
            for (int u = 0; u < kBatch; ++u) {
                float acc = 0.f;
#pragma unroll
                for (int f = 0; f < FS; ++f) {
                    const float diff = tile[(j0 + u) * FS + f] - qf[f];
                    acc = fmaf(diff, diff, acc);
                }
                v[u] = acc;
            }
#pragma unroll
            for (int u = 0; u < kBatch; ++u) {
                if (v[u] < top.tau2) {
                    const float d = __builtin_amdgcn_sqrtf(v[u]);
                    const uint32_t id = id_of(j0 + u);
                    if (top.admits(d, id)) top.push(d, id);
                }
            }
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
                                                           int nlinks, float *__restrict__ pd,
                                                           uint32_t *__restrict__ pi) {
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
        screen_tile<SP, FS, K2, kTile>(tile, qf, w0, w0sq, w1, nlinks, [&](int j) { return (uint32_t)(base + j); },
                                       top, ctau);
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

// ---- group walk (SE3, R^n) ----------------------------------------------------------------
// One wave serves G queries that are neighbours on the Morton curve.  Lanes hold the states
// of a 64-state tile (registers), the G queries are broadcast from LDS, and every query keeps
// its K2-list spread over the wave (lane j holds entry j, sorted by (distance, id)), so an
// insertion is one shift by a lane.  Tiles and super-tiles whose box is farther than every
// query's current K2-th distance are skipped; the box bound covers the whole metric.

// lower bound of the fp32 distance from query row q (FS layout) to any state inside box bx.
// (A packed-fp32 form of the gaps — v_pk_add pairs — measured no faster for the kNN walk and
// 20% slower for the radius walk, whose register allocation it upsets.)
__device__ __forceinline__ float gap(float a, float b) { return fmaxf(fmaxf(a, b), 0.f); }

// SCHED: translation and rotation gaps as two scheduling regions (fewer live temporaries: the
// kNN walk's pipelined loop stays at 7 waves per SIMD; the radius walk is faster without)
template <int SP, int F, bool SCHED = false>
__device__ __forceinline__ float box_lb(const float *bx, const float *q, float w0, float w1) {
    constexpr int NB = Geo<SP, F>::NB;
    if constexpr (SP == OMPL_GPU_SPACE_SE3) {
        float tg = 0.f;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const float g = gap(bx[c] - q[c], q[c] - bx[NB + c]);
            tg = fmaf(g, g, tg);
        }
        if constexpr (SCHED) __builtin_amdgcn_sched_barrier(0);
        // rotation: the screened 2 asin(c / 2) >= c = min(|p - q|, |p + q|) >= the distance
        // from q or from -q to the box (state_dist32)
        float rp = 0.f, rm = 0.f;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const float lo = bx[3 + c], hi = bx[NB + 3 + c], v = q[4 + c];
            const float gp = gap(lo - v, v - hi);
            const float gm = gap(lo + v, -v - hi);
            rp = fmaf(gp, gp, rp);
            rm = fmaf(gm, gm, rm);
        }
        return w0 * __builtin_amdgcn_sqrtf(tg) + w1 * __builtin_amdgcn_sqrtf(fminf(rp, rm));
    } else {
        float acc = 0.f;
#pragma unroll
        for (int c = 0; c < F; ++c) {
            const float g = gap(bx[c] - q[c], q[c] - bx[F + c]);
            acc = fmaf(g, g, acc);
        }
        return __builtin_amdgcn_sqrtf(acc);
    }
}

// fp32 screened distance of a lane's state x (R stored coordinates) to query row q.  SE3:
// translation as the reference, rotation by the chord (error bound in the header):
// theta = 2 asin(c / 2) = pi - 2 acos(c / 2), c^2 = min(|p - q|^2, |p + q|^2), both sums on
// packed fp32 (one v_pk_add / v_pk_fma per component gives both)
template <int SP, int F>
__device__ __forceinline__ float state_dist32(const float *x, const float *q, float w0, float w1) {
    if constexpr (SP == OMPL_GPU_SPACE_SE3) {
        const float dx = x[0] - q[0], dy = x[1] - q[1], dz = x[2] - q[2];
        float t = dx * dx;
        t = fmaf(dy, dy, t);
        t = fmaf(dz, dz, t);
        return fmaf(w1, chord_angle(x + 3, q + 4), w0 * __builtin_amdgcn_sqrtf(t));
    } else {
        float acc = 0.f;
#pragma unroll
        for (int f = 0; f < F; ++f) {
            const float diff = x[f] - q[f];
            acc = fmaf(diff, diff, acc);
        }
        return __builtin_amdgcn_sqrtf(acc);
    }
}

__device__ __forceinline__ float readlane_f(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ uint32_t readlane_u(uint32_t v, int l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}
// value of lane - 1 (wave-wide DPP shift); lane 0 receives `first`
__device__ __forceinline__ float shr1_f(float v, float first) {
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(first), __float_as_int(v), 0x138, 0xF, 0xF, false));
}
__device__ __forceinline__ uint32_t shr1_u(uint32_t v, uint32_t first) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)first, (int)v, 0x138, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t fold_tiles(uint64_t m) {  // lanes t and t+32 describe tile t
    return (uint32_t)(m | (m >> 32));
}

// (distance, id) order of the wave lists
__device__ __forceinline__ bool lex_less32(float a, uint32_t ia, float b, uint32_t ib) {
    return a < b || (a == b && ia < ib);
}
// one compare-exchange stage of a wave-wide bitonic network: partner lane ^ j, this lane
// keeps the smaller pair iff `keep_min`
__device__ __forceinline__ void bitonic_step(float &d, uint32_t &i, int j, bool keep_min) {
    const float od = __shfl_xor(d, j);
    const uint32_t oi = (uint32_t)__shfl_xor((int)i, j);
    const bool other_less = lex_less32(od, oi, d, i);
    if (other_less == keep_min) {
        d = od;
        i = oi;
    }
}
// Merge the wave's candidates (d, i) (non-candidates hold (+inf, kNoId)) into the sorted
// 64-entry list (Ld, Li) (lane j = entry j): sort the candidates ascending (bitonic, 21
// stages), reverse them against the list, keep the lane-wise minimum — the 64 smallest of
// the union, as a bitonic sequence — and sort that (6 stages).  Costs ~27 shuffle stages,
// against one list shift per candidate for the one-by-one insertion; used when many lanes
// pass at once (the first tiles of a walk).
__device__ __forceinline__ void wave_merge_sorted(float &Ld, uint32_t &Li, float d, uint32_t i, int lane) {
#pragma unroll
    for (int k = 2; k <= 64; k <<= 1)
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) bitonic_step(d, i, j, ((lane & j) == 0) == ((lane & k) == 0));
    const float rd = __shfl(d, 63 - lane);
    const uint32_t ri = (uint32_t)__shfl((int)i, 63 - lane);
    if (lex_less32(rd, ri, Ld, Li)) {
        Ld = rd;
        Li = ri;
    }
#pragma unroll
    for (int j = 32; j > 0; j >>= 1) bitonic_step(Ld, Li, j, (lane & j) == 0);
}
// (distance, id) as one 64-bit key: the walk's distances are >= 0 (or +inf / NaN), so their
// IEEE bits (sign cleared) order as unsigned integers and the key orders (distance, id)
// lexicographically — one 64-bit compare instead of the lex_less32 pair of compares and the
// SALU mask logic around it
__device__ __forceinline__ uint64_t kpack(float d, uint32_t id) {
    return ((uint64_t)(__float_as_uint(d) & 0x7FFFFFFFu) << 32) | id;
}
__device__ __forceinline__ float kdist(uint64_t k) { return __uint_as_float((uint32_t)(k >> 32)); }
constexpr uint64_t kMaxKey = (0x7F800000ull << 32) | 0xFFFFFFFFull;  // (+inf, kNoId)
__device__ __forceinline__ uint64_t readlane_k(uint64_t v, int l) {
    return ((uint64_t)readlane_u((uint32_t)(v >> 32), l) << 32) | readlane_u((uint32_t)v, l);
}
__device__ __forceinline__ uint64_t shr1_k(uint64_t v, uint64_t first) {
    return ((uint64_t)shr1_u((uint32_t)(v >> 32), (uint32_t)(first >> 32)) << 32) | shr1_u((uint32_t)v, (uint32_t)first);
}
__device__ __forceinline__ uint64_t shfl_k(uint64_t v, int src) {
    return ((uint64_t)(uint32_t)__shfl((int)(v >> 32), src) << 32) | (uint32_t)__shfl((int)v, src);
}
__device__ __forceinline__ uint64_t shfl_xor_k(uint64_t v, int j) {
    return ((uint64_t)(uint32_t)__shfl_xor((int)(v >> 32), j) << 32) | (uint32_t)__shfl_xor((int)v, j);
}
// the value of lane ^ j without the LDS crossbar (ds_bpermute waits on lgkmcnt at every stage of
// a serial network): DPP inside a row of 16 — quad_perm for j = 1, 2, row_shl / row_shr by 4 for
// j = 4, row_ror:8 for j = 8 — and gfx950's permlane swaps across rows (permlane16_swap trades the
// odd rows of its first operand with the even rows of its second, permlane32_swap the upper half
// of the first with the lower half of the second; with both operands v, lane l finds its partner
// in the first result iff bit j of l is set).  j is a compile-time constant after unrolling.
__device__ __forceinline__ uint32_t xor_lane_u(uint32_t v, int j, int lane) {
    switch (j) {
    case 1: return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0xB1, 0xF, 0xF, false);  // [1,0,3,2]
    case 2: return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x4E, 0xF, 0xF, false);  // [2,3,0,1]
    case 4: {
        const uint32_t up = (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x104, 0xF, 0xF, false);  // row_shl:4
        const uint32_t dn = (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x114, 0xF, 0xF, false);  // row_shr:4
        return (lane & 4) ? dn : up;
    }
    case 8: return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x128, 0xF, 0xF, false);  // row_ror:8
    case 16: {
        const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        return (lane & 16) ? r[0] : r[1];
    }
    default: {
        const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        return (lane & 32) ? r[0] : r[1];
    }
    }
}
__device__ __forceinline__ uint64_t xor_lane_k(uint64_t v, int j, int lane) {
    return ((uint64_t)xor_lane_u((uint32_t)(v >> 32), j, lane) << 32) | xor_lane_u((uint32_t)v, j, lane);
}
// the value of lane 63 - lane = lane ^ 63: row_mirror (lane ^ 15 inside each row), then ^ 16, ^ 32
__device__ __forceinline__ uint64_t reverse_lanes_k(uint64_t v, int lane) {
    auto mirror = [](uint32_t x) { return (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x140, 0xF, 0xF, false); };
    const uint64_t m = ((uint64_t)mirror((uint32_t)(v >> 32)) << 32) | mirror((uint32_t)v);
    return xor_lane_k(xor_lane_k(m, 16, lane), 32, lane);
}
__device__ __forceinline__ void bitonic_step_k(uint64_t &k, int j, bool keep_min, int lane) {
    const uint64_t o = xor_lane_k(k, j, lane);
    if ((o < k) == keep_min) k = o;
}
// wave_merge_sorted on packed keys: candidates c (non-candidates kMaxKey) into the sorted list L
__device__ __forceinline__ void wave_merge_sorted_k(uint64_t &L, uint64_t c, int lane) {
#pragma unroll
    for (int k = 2; k <= 64; k <<= 1)
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) bitonic_step_k(c, j, ((lane & j) == 0) == ((lane & k) == 0), lane);
    const uint64_t r = reverse_lanes_k(c, lane);
    if (r < L) L = r;
#pragma unroll
    for (int j = 32; j > 0; j >>= 1) bitonic_step_k(L, j, (lane & j) == 0, lane);
}
// candidates in one ballot above which the bulk merge is used.  Measured (G = 4): SE3 1.58 /
// 1.42 / 1.41 ms at 64 / 8 / 32; R^6 1.60 / 1.12 / 1.13 / 1.21 ms at 64 / 8 / 16 / 32
// At G = 2 (round 4): 4 / 8 / 16 / 32 / 64 -> cfg3 1.17-1.24 / 1.22-1.23 / 1.18-1.23 / 1.20-1.21 /
// 1.29-1.30 ms, cfg5k 4.06 / 4.10 / 3.93-3.97 / 4.03 / 4.29 ms, cfg2 flat (profiles/r4_ab)
constexpr int kBulkThreshold = 16;

// LDS-DMA bookkeeping.  The compiler does not order an LDS read after the global_load_lds that
// fills it (ROCm 7.2 emits no vmcnt for it), so the waits are explicit: vmcnt(0) before reading a
// filled slot (at that point the DMA is the only vector memory op the walk has in flight),
// lgkmcnt(0) before the slot is refilled (its reads have returned).  s_waitcnt simm16 on gfx9:
// vmcnt[3:0] | expcnt << 4 | lgkmcnt << 8 | vmcnt[5:4] << 14.
__device__ __forceinline__ void lds_dma_wait_all() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    asm volatile("" ::: "memory");
}
__device__ __forceinline__ void lds_reads_done() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    asm volatile("" ::: "memory");
}

// translation part of box_lb<SE3>: the squared gap of query row q to box bx
__device__ __forceinline__ float box_tgap2(const float *bx, const float *q, int NB) {
    float tg = 0.f;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const float g = gap(bx[c] - q[c], q[c] - bx[NB + c]);
        tg = fmaf(g, g, tg);
    }
    return tg;
}

// K2: lanes per query in the output (16 / 32 / 64); k2 <= K2: the list length the walk keeps
// (the certificate's margin: k + 3 for the culled spaces, whose screen error is small).
// (Measured and rejected, DESIGN §8: tile bounds only for the queries whose super-tile bound
// passes; square-root-free rejects before the chord; a translation-only first mask pass; tiles
// from a 16-bit copy.)
template <int SP, int F, int K2, int G, bool QS>
// (amdgpu_waves_per_eu(8), lists of up to 32 lanes: with the next super-tile's boxes in LDS the
// walk fits 64 VGPRs and, with the scalar registers it then spills to VGPR lanes, 8 waves per SIMD
// instead of 7 — cfg3's walk 1.022-1.028 against 1.046-1.049 ms isolated on one box, cfg2
// unchanged; the boxes in LDS at 7 waves were slower, 8 waves with the boxes in registers spill to
// scratch.  BIT*'s 64-lane lists keep the boxes in registers at 7 waves: 8 waves were no faster
// (3.22-3.25 against 3.20-3.22 ms) and read 8 % more bytes, the LDS boxes at 7 waves were slower.)
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(K2 == 64 ? 7 : 8))) void knn32_group_kernel(
    const float *__restrict__ rows, uint32_t n_pad, const uint32_t *__restrict__ ids, uint32_t ntiles,
    const float *__restrict__ tbox, const float *__restrict__ sbox, uint32_t nsuper, const float *__restrict__ mbox,
    uint32_t nmega, const uint32_t *__restrict__ tkey0, const float *__restrict__ q32, const uint32_t *__restrict__ qkeys,
    uint32_t nq, float w0, float w1, float *__restrict__ pd, uint32_t *__restrict__ pi,
    unsigned long long *__restrict__ counters, int k2, float pmin) {
    constexpr int FS = Geo<SP, F>::FS, R = Geo<SP, F>::R, BW = Geo<SP, F>::BW;
    constexpr int GH = G / 2;
    // PK (SE3, two queries): a tile is screened for both queries at once on packed fp32, the
    // rotation first by a certified lower bound from the quaternion dot products (below)
    constexpr bool PK = SP == OMPL_GPU_SPACE_SE3 && G == 2;
    static_assert(G % 2 == 0 && K2 <= 64 && kMegaSupers == 64, "group walk shape");
    __shared__ __attribute__((aligned(16))) float qrow[G * FS];
    __shared__ __attribute__((aligned(16))) float qpair[PK ? 2 * FS : 2];  // (query 0, query 1) per coordinate
    const int lane = threadIdx.x;
    const int half = lane >> 5;
    // XCD-aware group order: blocks b and b + 8 share an XCD (and its L2), so each XCD gets
    // one contiguous stretch of the Morton-ordered groups; neighbouring groups walk mostly
    // the same tiles, which then hit in that XCD's L2 instead of crossing the fabric
    const uint32_t nb = gridDim.x, xq = nb / 8, xr = nb % 8, xb = blockIdx.x % 8;
    const uint32_t blk = (xb < xr ? xb * (xq + 1) : xr * (xq + 1) + (xb - xr) * xq) + blockIdx.x / 8;
    const uint32_t g0 = blk * G;
    for (int t = lane; t < G * FS; t += 64) {
        const uint32_t qi = g0 + t / FS;
        const float v = qi < nq ? q32[(size_t)qi * FS + t % FS] : __builtin_nanf("");
        qrow[t] = v;
        if constexpr (PK) qpair[2 * (t % FS) + t / FS] = v;
    }
    __syncthreads();
    // PK's rotation bound.  For the fp32 rows p (state) and q (query), the screened chord is
    // c2 = min(|p - q|^2, |p + q|^2) in fp32 (chord2), and exactly |p|^2 + |q|^2 - 2 |p.q| >=
    // pmin + |q|^2 - 2 |p.q| (pmin <= every stored |p|^2: the store's norm excess qeta and the
    // fp32 rounding, from the host).  With the fp32 dot product (error <= 2.5e-7), |q|^2 from
    // its fp32 sum (relative error <= 5e-7), the fp32 chord's own relative error (<= 4e-7 of at
    // most 4) and the square roots' ulps, c2lb = pmin + |q|^2 (1 - 6e-7) - 8e-6 - 2 |dot| gives
    // sqrt(max(c2lb, 0)) <= the screened chord c, so fma(w1, that, w0 |t|) <= the chord bound
    // fma(w1, c, w0 |t|) <= the screened distance: no lane it rejects could have been offered.
    float kq[2] = {0.f, 0.f};
    if constexpr (PK) {
#pragma unroll
        for (int g = 0; g < 2; ++g) {
            const float *qq = &qrow[g * FS + 4];
            float n2 = qq[0] * qq[0];
            n2 = fmaf(qq[1], qq[1], n2);
            n2 = fmaf(qq[2], qq[2], n2);
            n2 = fmaf(qq[3], qq[3], n2);
            kq[g] = pmin + n2 * (1.f - 6e-7f) - 8e-6f;
        }
    }
    // QS: re-read the wave-uniform query rows from LDS (broadcast reads) at every tile
    // through an offset the compiler cannot see through, instead of letting it hoist all
    // G x FS values into vector registers for the whole walk (which caps occupancy)
    uint32_t qoff = 0;
    auto relaunder = [&]() {
        if constexpr (QS) asm volatile("" : "+s"(qoff));
    };
    auto qscan = [&](int g) -> const float * { return &qrow[qoff + g * FS]; };
    // the lists (lane j = entry j) and their K2-th entries (wave-uniform); a padding query
    // gets threshold -inf so that it admits nothing and needs no tile
    uint64_t Lk[G];  // packed (distance, id) list entries (kpack)
    float td[G];     // the K2-th distance (box and ballot tests)
    uint64_t tk[G];  // the K2-th entry: a candidate enters iff its key is below it
#pragma unroll
    for (int g = 0; g < G; ++g) {
        Lk[g] = kMaxKey;
        td[g] = g0 + g < nq ? __builtin_inff() : -__builtin_inff();
        tk[g] = g0 + g < nq ? kMaxKey : 0ull;
    }
    uint32_t visited = 0, qscans = 0;  // tiles fetched; (tile, query) scans
#ifdef OMPL_AMD_PROBE
    uint32_t pr_offers = 0, pr_bulk = 0, pr_ins = 0, pr_supers = 0, pr_rounds = 0, pr_empty = 0, pr_skip = 0;
    // probe timers (shader clock, per wave): the masks of popped super-tiles, the wait for a fetched
    // tile, its scan, next_super (its mega / super rounds' box loads and bounds), the whole walk
    uint64_t pt_mask = 0, pt_wait = 0, pt_scan = 0, pt_next = 0, pt_pro = 0, pt_issue = 0, pt_tail = 0, pt_offer = 0, pt_cwait = 0, pt_dummy = 0;
    const uint64_t pt_start = __builtin_amdgcn_s_memtime();
#define OMPL_PT(acc, ...)                                          \
    do {                                                            \
        __builtin_amdgcn_sched_barrier(0);                          \
        const uint64_t pt_a = __builtin_amdgcn_s_memtime();         \
        __builtin_amdgcn_sched_barrier(0);                          \
        __VA_ARGS__;                                                \
        __builtin_amdgcn_sched_barrier(0);                          \
        acc += __builtin_amdgcn_s_memtime() - pt_a;                 \
        __builtin_amdgcn_sched_barrier(0);                          \
    } while (0)
#else
#define OMPL_PT(acc, ...) do { __VA_ARGS__; } while (0)
#endif

    // tiles of super-tile s some query may still need; lb[j]: this lane's bound for tile
    // (lane & 31) and query half * GH + j
    // this lane's row of super-tile s's tile boxes (tile s * 32 + (lane & 31)); rows past
    // the last tile read as empty boxes (lo = +inf, hi = -inf), whose bound is +inf, so no
    // tile past the end is ever fetched (a NaN box would not do: fmaxf drops NaN)
    auto load_tbox_regs = [&](uint32_t s, float (&bx)[BW]) {
        const uint32_t t = s * kSuperTiles + (lane & 31);
        if (t < ntiles) {
            const float4 *b4 = reinterpret_cast<const float4 *>(tbox + (size_t)t * BW);
#pragma unroll
            for (int c = 0; c < BW / 4; ++c) {
                const float4 v = b4[c];
                bx[4 * c] = v.x; bx[4 * c + 1] = v.y; bx[4 * c + 2] = v.z; bx[4 * c + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int c = 0; c < BW; ++c) bx[c] = c < Geo<SP, F>::NB ? __builtin_inff() : -__builtin_inff();
            if constexpr (SP == OMPL_GPU_SPACE_SE3) bx[2 * Geo<SP, F>::NB] = bx[2 * Geo<SP, F>::NB + 1] = 0.f;
        }
    };
    // tiles of the super-tile whose boxes are in bx that some query may still need;
    // lb[j]: this lane's bound for its tile and query half * GH + j
    auto tile_mask = [&](const float (&bx)[BW], float (&lb)[GH]) -> uint32_t {
        relaunder();
#ifdef OMPL_AMD_PROBE
        ++pr_supers;
#endif
        bool need = false;
#pragma unroll
        for (int j = 0; j < GH; ++j) {
            lb[j] = box_lb<SP, F, true>(bx, &qrow[qoff + (half * GH + j) * FS], w0, w1);
            need |= lb[j] < (half ? td[GH + j] : td[j]);
            __builtin_amdgcn_sched_barrier(0);  // one bound at a time (temporaries)
        }
        return fold_tiles(__ballot(need));
    };
    auto load_state = [&](uint32_t t, float (&x)[R], uint32_t &id) {
        const uint64_t p = (uint64_t)t * kCullTile + lane;
        load_blk<R>(rows, t, lane, x);
        id = (uint32_t)p;  // lists hold sorted positions; the certificate maps them to ids
        (void)ids;
        (void)n_pad;
    };
    // scan tile tin (index inside its super-tile) against every query whose own box bound
    // lb (held by lane tin + 32 * (g / GH)) is still below its threshold: the tile was
    // fetched for the group, but each query skips it on a wave-uniform branch when its own
    // bound already excludes it
    // offer this lane's distance d to query g's list.  Only d < td[g] is offered: an element
    // tied with the K2-th entry stays out, which the certificate allows (every excluded
    // element still has a screened distance >= the final K2-th distance)
    auto offer = [&](int g, float d, uint32_t id) {
#ifdef OMPL_AMD_PROBE
            const uint64_t pt_o = __builtin_amdgcn_s_memtime();
            struct PtO { uint64_t &acc; uint64_t t0; __device__ ~PtO() { acc += __builtin_amdgcn_s_memtime() - t0; } } pt_od{pt_offer, pt_o};
#endif
            uint64_t bm = __ballot(d < td[g]);
#ifdef OMPL_AMD_PROBE
            ++pr_offers;
#endif
            if (__popcll(bm) > kBulkThreshold) {  // many at once: sort-merge (same top K2)
#ifdef OMPL_AMD_PROBE
                ++pr_bulk;
#endif
                wave_merge_sorted_k(Lk[g], d < td[g] ? kpack(d, id) : kMaxKey, lane);
                tk[g] = readlane_k(Lk[g], k2 - 1);
                td[g] = kdist(tk[g]);
                return;
            }
            // every lane that passed the offer's threshold is shifted into the 64-lane list in
            // turn, with no re-test against the threshold its predecessors tightened: a candidate
            // above the new k2-th entry lands at a position >= k2 (or falls off the end), so the
            // first k2 entries — all the walk and its output read — are those of the one-by-one
            // insertion with a test each, and the k2-th entry is read once, after the loop (the
            // serial readlane -> 64-bit compare -> branch chain per candidate is gone)
            const uint64_t mk = kpack(d, id);
            while (bm) {
                const int l = __builtin_ctzll(bm);
                bm &= bm - 1;
                const uint64_t ck = readlane_k(mk, l);
#ifdef OMPL_AMD_PROBE
                ++pr_ins;
#endif
                const uint64_t pv = shr1_k(Lk[g], 0ull);
                const bool lt_prev = lane > 0 && ck < pv;
                Lk[g] = lt_prev ? pv : (ck < Lk[g] ? ck : Lk[g]);
            }
            tk[g] = readlane_k(Lk[g], k2 - 1);
            td[g] = kdist(tk[g]);
    };
    auto scan_state = [&](const float (&x)[R], uint32_t id, int tin, const float (&lb)[GH]) {
        relaunder();
        if constexpr (PK) {
            // both queries' translation terms and rotation lower bounds in one packed pass (the
            // translation in scan order: the same fp32 bits as the one-query form)
            bool on[2];
            on[0] = readlane_f(lb[0], tin) < td[0];
            on[1] = readlane_f(lb[0], tin + 32) < td[1];
            const f2 *qp = reinterpret_cast<const f2 *>(&qpair[qoff]);
            f2 a = f2{x[0], x[0]} - qp[0];
            f2 t2 = a * a;
            a = f2{x[1], x[1]} - qp[1];
            t2 = pk_fma(a, a, t2);
            a = f2{x[2], x[2]} - qp[2];
            t2 = pk_fma(a, a, t2);
            f2 dt = f2{x[3], x[3]} * qp[4];
            dt = pk_fma(f2{x[4], x[4]}, qp[5], dt);
            dt = pk_fma(f2{x[5], x[5]}, qp[6], dt);
            dt = pk_fma(f2{x[6], x[6]}, qp[7], dt);
            const float wt[2] = {w0 * __builtin_amdgcn_sqrtf(t2.x), w0 * __builtin_amdgcn_sqrtf(t2.y)};
            const float dd[2] = {dt.x, dt.y};
#pragma unroll
            for (int g = 0; g < 2; ++g) {
                if (!on[g]) continue;
                ++qscans;
                const float clb = __builtin_amdgcn_sqrtf(fmaxf(fmaf(-2.f, fabsf(dd[g]), kq[g]), 0.f));
                if (!__ballot(fmaf(w1, clb, wt[g]) < td[g])) continue;
                const float c2 = chord2(x + 3, qscan(g) + 4);
                const float c = __builtin_amdgcn_sqrtf(c2);
                if (!__ballot(fmaf(w1, c, wt[g]) < td[g])) continue;
                offer(g, fmaf(w1, chord_theta(c, c2), wt[g]), id);
            }
            return;
        }
#pragma unroll
        for (int g = 0; g < G; ++g) {
            if (!(readlane_f(lb[g % GH], tin + (g < GH ? 0 : 32)) < td[g])) continue;
            ++qscans;
            if constexpr (SP == OMPL_GPU_SPACE_SE3) {
                // screened d = fma(w1, theta, w0 |t|) with theta >= c: when no lane's chord
                // bound fma(w1, c, w0 |t|) is below the threshold, no lane's d is either, and
                // the angle polynomial is skipped for the whole wave
                const float *qq = qscan(g);
                const float dx = x[0] - qq[0], dy = x[1] - qq[1], dz = x[2] - qq[2];
                float t = dx * dx;
                t = fmaf(dy, dy, t);
                t = fmaf(dz, dz, t);
                const float c2 = chord2(x + 3, qq + 4);
                const float c = __builtin_amdgcn_sqrtf(c2), wt = w0 * __builtin_amdgcn_sqrtf(t);
                if (!__ballot(fmaf(w1, c, wt) < td[g])) continue;
                offer(g, fmaf(w1, chord_theta(c, c2), wt), id);
            } else {
                offer(g, state_dist32<SP, F>(x, qscan(g), w0, w1), id);
            }
        }
    };
    // start at the super-tile holding the group's middle query's home tile.  The store's tile
    // keys are the tile indices (SortedStore::tkey0 = iota) and a query's key is its home tile,
    // so the last tile whose key is <= the query's is min(key, ntiles - 1): no search (the binary
    // search over tkey0 it replaces was a chain of 14 dependent loads at the start of every wave)
    (void)tkey0;
    const uint32_t key = qkeys[min(g0 + G / 2, nq - 1)];
    const uint32_t th = min(key, ntiles - 1);
    const uint32_t s0 = th / kSuperTiles;
    // scan the middle query's home tile (its k-d leaf) first, for every query of the group:
    // the thresholds start near the final K2-th distances, so the box tests that follow
    // exclude more tiles; the home tile is then dropped from its super-tile's mask
    {
        float x[R];
        uint32_t id;
        load_state(th, x, id);
        float lbh[GH];
#pragma unroll
        for (int j = 0; j < GH; ++j) lbh[j] = -__builtin_inff();
        scan_state(x, id, 0, lbh);
        ++visited;
    }
    // visit order: s0 - 1, s0, s0 + 1 (the group's neighbourhood, which sets the thresholds),
    // then every other super-tile in curve order whose box passes, 64 box tests at a time
    uint32_t base = s0 > 0 ? s0 - 1 : 0;
    uint64_t sm = (s0 > 0 ? 7ull : 3ull) & ((nsuper - base >= 64) ? ~0ull : ((1ull << (nsuper - base)) - 1));
    uint32_t sb = 0;
    // the round's super-tile bounds (slb[g][l]: super-tile base + l, query g): a super-tile
    // popped later is skipped when the thresholds have tightened past all of its bounds since
    // its round, before its 32 tile boxes are loaded and tested.  Kept in LDS, not VGPRs: G
    // values live across the whole walk cost 29 VGPRs (69 -> 98, 7 -> 5 waves per SIMD)
    __shared__ float slb[G][64];
    bool first_round = true;  // the neighbourhood's three are always visited
    // mega-tiles (kMegaSupers super-tiles each): a round tests 64 mega boxes; a super-tile round
    // then covers the 64 super-tiles of one passing mega.  A popped mega is re-checked against the
    // tightened thresholds by its round bounds (mlb, LDS) like a popped super-tile.
    __shared__ float mlb[G][64];
    uint32_t mb = 0, mbase = 0;
    uint64_t mm = 0;
    auto next_mega = [&]() -> int {
        for (;;) {
            if (mm) {
                bool keep = false;
#pragma unroll
                for (int g = 0; g < G; ++g) keep |= mlb[g][lane] < td[g];
                mm &= __ballot(keep);
            }
            if (mm) {
                const int l = __builtin_ctzll(mm);
                mm &= mm - 1;
                return (int)(mbase + l);
            }
            if (mb >= nmega) return -1;
            relaunder();
            const uint32_t mi = mb + lane;
            bool need = false;
            float lbm[G];
#pragma unroll
            for (int g = 0; g < G; ++g) lbm[g] = __builtin_inff();
            if (mi < nmega) {
                float bx[BW];
                const float4 *b4 = reinterpret_cast<const float4 *>(mbox + (size_t)mi * BW);
#pragma unroll
                for (int c = 0; c < BW / 4; ++c) {
                    const float4 v = b4[c];
                    bx[4 * c] = v.x; bx[4 * c + 1] = v.y; bx[4 * c + 2] = v.z; bx[4 * c + 3] = v.w;
                }
#pragma unroll
                for (int g = 0; g < G; ++g) {
                    lbm[g] = box_lb<SP, F, true>(bx, &qrow[qoff + g * FS], w0, w1);
                    need |= lbm[g] < td[g];
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
#pragma unroll
            for (int g = 0; g < G; ++g) mlb[g][lane] = lbm[g];
            __builtin_amdgcn_wave_barrier();
            mm = __ballot(need);
            mbase = mb;
            mb += 64;
        }
    };
    auto next_super = [&]() -> int {  // next super-tile to visit, -1 when done
        for (;;) {
            if (sm && !first_round) {  // drop what the tightened thresholds exclude
                bool keep = false;
#pragma unroll
                for (int g = 0; g < G; ++g) keep |= slb[g][lane] < td[g];
#ifdef OMPL_AMD_PROBE
                pr_skip += __popcll(sm & ~__ballot(keep));
#endif
                sm &= __ballot(keep);
            }
            if (sm) {
                const int l = __builtin_ctzll(sm);
                sm &= sm - 1;
                return (int)(base + l);
            }
            const int mg = next_mega();
            if (mg < 0) return -1;
            sb = (uint32_t)mg * kMegaSupers;
            relaunder();
#ifdef OMPL_AMD_PROBE
            ++pr_rounds;
#endif
            const uint32_t s = sb + lane;
            bool need = false;
            float lbs[G];
#pragma unroll
            for (int g = 0; g < G; ++g) lbs[g] = __builtin_inff();
            if (s < nsuper && (s + 1 < s0 || s > s0 + 1)) {
                float bx[BW];
                const float4 *b4 = reinterpret_cast<const float4 *>(sbox + (size_t)s * BW);
#pragma unroll
                for (int c = 0; c < BW / 4; ++c) {
                    const float4 v = b4[c];
                    bx[4 * c] = v.x; bx[4 * c + 1] = v.y; bx[4 * c + 2] = v.z; bx[4 * c + 3] = v.w;
                }
#pragma unroll
                for (int g = 0; g < G; ++g) {
                    lbs[g] = box_lb<SP, F, true>(bx, &qrow[qoff + g * FS], w0, w1);
                    need |= lbs[g] < td[g];
                    // one query's bound at a time: interleaving the G bounds needs ~40 temporaries
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
#pragma unroll
            for (int g = 0; g < G; ++g) slb[g][lane] = lbs[g];
            __builtin_amdgcn_wave_barrier();  // one wave: its LDS ops complete in order
            first_round = false;
            sm = __ballot(need);
            base = sb;
        }
    };
    // Software pipeline: the tile boxes of the next super-tile sn are loaded while the tiles
    // of s are scanned, and the next tile is always fetched before the current one is scanned
    // — within s, and across the boundary: on the last tile of s, sn's mask is computed (its
    // boxes arrived meanwhile) and its first tile fetched, so no tile fetch waits behind a box
    // bound; the super-tile after sn is popped (a round's box loads included) only after that
    // scan.  Masks use the thresholds of their moment; every tile is re-checked against the
    // current thresholds before it is scanned.  (Measured: 1.27-1.29 -> 1.25-1.26 ms on cfg3.)
    // the next super-tile's 32 tile boxes: staged in LDS by LDS-DMA (BW / 8 loads of 1 KB, no
    // registers held across the scans) when the record width allows, else in registers
    constexpr bool kLdsBox = BW % 8 == 0 && K2 < 64;
    __shared__ __attribute__((aligned(16))) float tbs[kLdsBox ? kSuperTiles * BW : 4];
    float bx[kLdsBox ? 1 : BW];
    auto load_tbox = [&](uint32_t sv) {
        if constexpr (kLdsBox) {
            lds_reads_done();  // the previous boxes were read out of the slot
            const char *blk = reinterpret_cast<const char *>(tbox + (size_t)sv * kSuperTiles * BW);
#pragma unroll
            for (int j = 0; j < BW / 8; ++j) {
                // this lane's 16 bytes of piece j; a piece past the last tile reads the first box
                // instead (never used: mask_of gives tiles past the end empty boxes)
                const uint32_t off = (uint32_t)j * 1024u + (uint32_t)lane * 16u;
                const bool in = sv * kSuperTiles + off / (BW * 4) < ntiles;
                __builtin_amdgcn_global_load_lds((const void *)(in ? blk + off : reinterpret_cast<const char *>(tbox)),
                                                 (void *)(tbs + j * 256), 16, 0, 0);
            }
        } else {
            load_tbox_regs(sv, bx);
        }
    };
    const uint32_t home_s = th / kSuperTiles;
    auto mask_of = [&](int sv, float (&l)[GH]) -> uint32_t {
        uint32_t mm;
        if constexpr (kLdsBox) {
            float bl[BW];
            lds_dma_wait_all();  // the boxes' DMA (and nothing later is in flight here)
            const uint32_t t = (uint32_t)sv * kSuperTiles + (lane & 31);
            if (t < ntiles) {
                const float4 *b4 = reinterpret_cast<const float4 *>(tbs + (lane & 31) * BW);
#pragma unroll
                for (int c = 0; c < BW / 4; ++c) {
                    const float4 v = b4[c];
                    bl[4 * c] = v.x; bl[4 * c + 1] = v.y; bl[4 * c + 2] = v.z; bl[4 * c + 3] = v.w;
                }
            } else {
#pragma unroll
                for (int c = 0; c < BW; ++c) bl[c] = c < Geo<SP, F>::NB ? __builtin_inff() : -__builtin_inff();
                if constexpr (SP == OMPL_GPU_SPACE_SE3) bl[2 * Geo<SP, F>::NB] = bl[2 * Geo<SP, F>::NB + 1] = 0.f;
            }
            mm = tile_mask(bl, l);
        } else {
            mm = tile_mask(bx, l);
        }
        if ((uint32_t)sv == home_s) mm &= ~(1u << (th % kSuperTiles));  // scanned first
#ifdef OMPL_AMD_PROBE
        if (!mm) ++pr_empty;
#endif
        return mm;
    };
    float lb[GH];
    float x[R], xn[R];
    uint32_t idn = kNoId, m = 0;  // (the scan recomputes the position ids)
    int t = 0, tn = 0, s = -1;
    bool have = false;  // x holds a fetched tile of s
    int sn = next_super();
    if (sn >= 0) load_tbox((uint32_t)sn);
#ifdef OMPL_AMD_PROBE
    __builtin_amdgcn_sched_barrier(0);
    pt_pro = __builtin_amdgcn_s_memtime() - pt_start;
    __builtin_amdgcn_sched_barrier(0);
#endif
    // one site each for the mask, the fetch, the scan and next_super (every inlined copy of
    // next_super's round adds its box-bound temporaries to the live set of its site)
    for (;;) {
        // fetch the next tile (xn) while x is scanned: the next of s, or else the first tile of
        // sn (bx holds its boxes) when its mask is not empty
        bool got = false, cross = false, consumed = false;
        uint32_t mn = 0;
        float lbn[GH];
#ifdef OMPL_AMD_PROBE
        OMPL_PT(pt_dummy, (void)0);  // the timer's own cost
#endif
        if (!m && sn >= 0) {
            OMPL_PT(pt_mask, mn = mask_of(sn, lbn));
            consumed = true;
            cross = mn != 0;
        }
        uint32_t &mf = cross ? mn : m;
        OMPL_PT(pt_issue, if (mf) {
            tn = __builtin_ctz(mf);
            mf &= mf - 1;
            load_state((uint32_t)(cross ? sn : s) * kSuperTiles + tn, xn, idn);
            got = true;
        });
        if (have) {  // the list ids are sorted positions: recomputed, not carried in a VGPR
            const uint32_t pid = ((uint32_t)s * kSuperTiles + (uint32_t)t) * kCullTile + (uint32_t)lane;
#ifdef OMPL_AMD_PROBE
            OMPL_PT(pt_wait, asm volatile("" ::"v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3]), "v"(x[4]), "v"(x[5]),
                                          "v"(x[R - 1])));
#endif
            OMPL_PT(pt_scan, scan_state(x, pid, t, lb));
            ++visited;
        }
        if (cross) {
            s = sn;
            m = mn;
#pragma unroll
            for (int j = 0; j < GH; ++j) lb[j] = lbn[j];
        }
        if (consumed) {  // after the scan: a round's box loads wait behind it, not before
            OMPL_PT(pt_next, sn = next_super());
            if (sn >= 0) load_tbox((uint32_t)sn);
        }
#ifdef OMPL_AMD_PROBE
        __builtin_amdgcn_sched_barrier(0);
        const uint64_t pt_t = __builtin_amdgcn_s_memtime();
        __builtin_amdgcn_sched_barrier(0);
#endif
        bool still = false;  // drop the tiles of s that the tightened thresholds exclude
#pragma unroll
        for (int j = 0; j < GH; ++j) still |= lb[j] < (half ? td[GH + j] : td[j]);
        m &= fold_tiles(__ballot(still));
        have = got;
#ifdef OMPL_AMD_PROBE
        __builtin_amdgcn_sched_barrier(0);
        pt_tail += __builtin_amdgcn_s_memtime() - pt_t;
        __builtin_amdgcn_sched_barrier(0);
#endif
        if (got) {
#ifdef OMPL_AMD_PROBE
            OMPL_PT(pt_cwait, asm volatile("" ::"v"(xn[0]), "v"(xn[1]), "v"(xn[2]), "v"(xn[3]), "v"(xn[4]), "v"(xn[5]),
                                           "v"(xn[R - 1])));
#endif
#pragma unroll
            for (int r = 0; r < R; ++r) x[r] = xn[r];
            t = tn;
        } else if (sn < 0 && !m) {
            break;
        }
    }
    // every staged box DMA was consumed by a mask before the loop could end; wait anyway, so that no
    // LDS-DMA can land in LDS the next workgroup on this CU already owns
    if constexpr (kLdsBox) lds_dma_wait_all();
    if (counters && lane == 0) {
        unsigned long long *cs = counters + (blockIdx.x % kCounterSlots) * kCounterStride;
        atomicAdd(&cs[0], (unsigned long long)visited);  // tiles scanned
        atomicAdd(&cs[1], (unsigned long long)ntiles);   // tiles of a brute-force walk
        atomicAdd(&cs[2], (unsigned long long)qscans);   // (tile, query) pairs scanned
#ifdef OMPL_AMD_PROBE
        atomicAdd(&cs[5], (unsigned long long)pr_offers);
        atomicAdd(&cs[6], (unsigned long long)pr_bulk);
        atomicAdd(&cs[7], (unsigned long long)pr_ins);
        atomicAdd(&cs[8], (unsigned long long)pr_supers);
        atomicAdd(&cs[9], (unsigned long long)pr_rounds);
        atomicAdd(&cs[10], (unsigned long long)pr_empty);
        atomicAdd(&cs[11], (unsigned long long)pr_skip);
        atomicAdd(&cs[12], (unsigned long long)(__builtin_amdgcn_s_memtime() - pt_start));
        atomicAdd(&cs[13], (unsigned long long)pt_pro);
        atomicAdd(&cs[14], (unsigned long long)pt_mask);
        atomicAdd(&cs[15], (unsigned long long)pt_issue);
        atomicAdd(&cs[16], (unsigned long long)pt_wait);
        atomicAdd(&cs[17], (unsigned long long)pt_scan);
        atomicAdd(&cs[18], (unsigned long long)pt_offer);
        atomicAdd(&cs[19], (unsigned long long)pt_next);
        atomicAdd(&cs[20], (unsigned long long)pt_tail);
        atomicAdd(&cs[21], (unsigned long long)pt_cwait);
        atomicAdd(&cs[22], (unsigned long long)pt_dummy);
#endif
    }
#undef OMPL_PT
#pragma unroll
    for (int g = 0; g < G; ++g)
        if (g0 + g < nq && lane < K2) {
            const size_t o = (size_t)(g0 + g) * K2 + lane;
            pd[o] = lane < k2 ? kdist(Lk[g]) : __builtin_inff();
            pi[o] = lane < k2 ? (uint32_t)Lk[g] : kNoId;
        }
}

// ---- wave scan (KinematicChain) --------------------------------------------------------------
// The chain metric has no box bound worth culling with, so every (query, state) pair is
// evaluated; a thread-per-query list of PRM*'s k = 41 (ConnectionStrategy.h:147) plus margin
// does not fit in registers, so the layout of the group walk is used instead: a wave serves
// kWaveGroup consecutive queries, lane l holds state l of the current 64-state tile (joint
// positions, chain_positions), and query g's K2-list lives across the wave (lane j = entry j).
// The store is split in chunks along grid.y; the certificate merges the chunk lists.
constexpr int kWaveGroup = 8;
// queries per wave of the culled chain scan: 4 (57 VGPRs, 8 waves per SIMD) — measured on cfg4 step
// 7.58-7.65 against 7.90-7.92 ms at 8 (73 VGPRs) and a 5.55-5.60 ms kernel at 2 (against 4.50-4.53)
constexpr int kChainCullG = 4;

// ORD 0: links in the reference's order, the wave-wide exit tested after links 4 and 8; ORD 1:
// outermost links first (|P_i(a) - P_i(b)| grows with i, so the partial sum nears the distance
// sooner) and the exit tested after every pair.  Summing in another order is inside the screen's
// error bound (screen_error<KCHAIN>: (n + 1) u of the sum covers any order of n non-negative
// terms); the certificate recomputes every candidate in the reference's order.
// WPB waves per block share every tile: the block stages it once in LDS (double-buffered, the
// next tile's global loads in flight while the current one is scanned), so the store is read
// once per WPB * G queries instead of once per G (measured: 8 queries per read moved ~98 GB per
// 8,192-milestone batch).
template <int F, int K2, int G, int ORD, int WPB>
__global__ __launch_bounds__(64 * WPB) void knn32_wave_scan_kernel(const float *__restrict__ f32, uint64_t cap,
                                                                   uint64_t n_end, const float *__restrict__ q32,
                                                                   uint32_t nq, uint32_t chunk_len, float link,
                                                                   int nlinks, float *__restrict__ pd,
                                                                   uint32_t *__restrict__ pi) {
    constexpr int NM = F / 2;
    constexpr int NT = 64 * WPB;                 // threads
    constexpr int PER = (F * 64 + NT - 1) / NT;  // tile floats staged per thread
    static_assert(K2 <= 64, "lists are spread over one wave");
    __shared__ __attribute__((aligned(16))) float qrow[WPB][G * F];
    __shared__ float tile[2][F][64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t g0 = (blockIdx.x * WPB + wv) * G;
    for (int t = lane; t < G * F; t += 64) {
        const uint32_t qi = g0 + t / F;
        qrow[wv][t] = qi < nq ? q32[(size_t)qi * F + t % F] : __builtin_nanf("");
    }
    uint32_t qoff = 0;  // re-read the wave-uniform query rows from LDS per tile (see knn32_group_kernel)
    uint64_t Lk[G];     // packed (distance, id) entries, as knn32_group_kernel
    float td[G];
    uint64_t tk[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        Lk[g] = kMaxKey;
        td[g] = g0 + g < nq ? __builtin_inff() : -__builtin_inff();
        tk[g] = g0 + g < nq ? kMaxKey : 0ull;
    }
    auto offer = [&](int g, float d, uint32_t id) {
        uint64_t bm = __ballot(d < td[g]);
        const uint64_t mk = kpack(d, id);
        while (bm) {
            const int l = __builtin_ctzll(bm);
            bm &= bm - 1;
            const uint64_t ck = readlane_k(mk, l);
            if (ck < tk[g]) {
                const uint64_t pv = shr1_k(Lk[g], 0ull);
                const bool lt_prev = lane > 0 && ck < pv;
                Lk[g] = lt_prev ? pv : (ck < Lk[g] ? ck : Lk[g]);
                tk[g] = readlane_k(Lk[g], K2 - 1);
                td[g] = kdist(tk[g]);
            }
        }
    };
    const uint64_t c0 = (uint64_t)blockIdx.y * chunk_len;
    const uint64_t c1 = min(c0 + chunk_len, n_end);
    // staging: thread t moves floats t, t + NT, ... of the F x 64 tile (row f = index / 64)
    float pre[PER];
    auto fetch = [&](uint64_t base) {
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int v = (int)threadIdx.x + u * NT;
            if (v < F * 64) pre[u] = f32[(uint64_t)(v >> 6) * cap + base + (v & 63)];
        }
    };
    auto stage = [&](int b) {
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int v = (int)threadIdx.x + u * NT;
            if (v < F * 64) tile[b][v >> 6][v & 63] = pre[u];
        }
    };
    int cur = 0;
    if (c0 < c1) {
        fetch(c0);
        stage(0);
    }
    __syncthreads();
    for (uint64_t base = c0; base < c1; base += 64) {
        const bool more = base + 64 < c1;
        if (more) fetch(base + 64);  // in flight while this tile is scanned
        float x[F];
#pragma unroll
        for (int f = 0; f < F; ++f) x[f] = tile[cur][f][lane];
        const uint32_t id = (uint32_t)(base + lane);
        asm volatile("" : "+s"(qoff));
#pragma unroll
        for (int g = 0; g < G; ++g) {
            // link * sum_i |P_i(a) - P_i(b)| (joint positions) with a wave-wide early exit: the
            // partial sums only grow (fp32 addition of non-negative terms is monotone, so is the
            // final * link), so once no lane's partial distance is below the threshold no lane's
            // full distance is either, and the query's list could not change.  Two links per step
            // on packed fp32 (v_pk_add / v_pk_mul / v_pk_fma).
            const float *qq = &qrow[wv][qoff + g * F];
            float acc = 0.f;
            bool alive = true;
            static_assert(NM % 2 == 0, "joint positions come in link pairs");
#pragma unroll
            for (int s = 0; s < NM; s += 2) {
                const int i = ORD ? NM - 2 - s : s;
                if (i < nlinks) {
                    const f2 dx = f2{x[i], x[i + 1]} - f2{qq[i], qq[i + 1]};
                    const f2 dy = f2{x[NM + i], x[NM + i + 1]} - f2{qq[NM + i], qq[NM + i + 1]};
                    const f2 s2 = pk_fma(dy, dy, dx * dx);
                    acc += __builtin_amdgcn_sqrtf(s2.x);
                    if (i + 1 < nlinks) acc += __builtin_amdgcn_sqrtf(s2.y);
                }
                const bool check = ORD ? (s + 2 < NM) : ((i & 3) == 2 && i + 2 < NM && i + 2 < nlinks);
                if (check && !__ballot(acc * link < td[g])) {
                    alive = false;
                    break;
                }
            }
            if (alive) offer(g, acc * link, id);
        }
        if (more) stage(cur ^ 1);  // the other buffer: every wave left it at the last barrier
        __syncthreads();
        cur ^= 1;
    }
#pragma unroll
    for (int g = 0; g < G; ++g)
        if (g0 + g < nq && lane < K2) {
            const size_t o = ((size_t)blockIdx.y * nq + g0 + g) * K2 + lane;
            pd[o] = kdist(Lk[g]);
            pi[o] = (uint32_t)Lk[g];
        }
}

// Underflow: a square below FLT_MIN (flushed or subnormal) is off by at most FLT_MIN in
// absolute terms, so a screened distance sqrt(sum of D squares) is off by at most
// sqrt(D * FLT_MIN) ~ 1e-19 — negligible at any usual scale, but the relative terms above
// vanish for stores whose coordinates are all tiny.
constexpr double kFltMin = 1.1754943508222875e-38;

// eta: |norm^2 - 1| of the stored quaternions (largest) plus the query's (SE3)
// Merge of the S chunk lists of a query (each sorted, K2 <= 64 entries) into one list of the
// K2 best by (distance, id), written over chunk 0's slots: a wave per query, one bitonic merge
// per further chunk (wave_merge_sorted_k).  The culled chain scan's lists then take the wave
// certificate (a lane per candidate) instead of the thread-per-query one.
template <int K2>
__global__ __launch_bounds__(256) void knn_chunk_merge_kernel(float *__restrict__ pd, uint32_t *__restrict__ pi,
                                                              uint32_t S, uint32_t nq) {
    const uint32_t qs = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (qs >= nq) return;  // uniform over the wave
    auto entry = [&](uint32_t c) -> uint64_t {
        if (lane >= K2) return kMaxKey;
        const size_t o = ((size_t)c * nq + qs) * K2 + lane;
        const uint32_t id = pi[o];
        return id == kNoId ? kMaxKey : kpack(pd[o], id);
    };
    uint64_t L = entry(0);
    for (uint32_t c = 1; c < S; ++c) {
        const uint64_t e = entry(c);
        // a chunk list whose smallest key is not below the merged K2-th cannot change the merge
        // (with shared thresholds most chunks hold only keys above it)
        if (readlane_k(e, 0) >= readlane_k(L, K2 - 1)) continue;
        wave_merge_sorted_k(L, e, lane);
    }
    if (lane < K2) {
        const size_t o = (size_t)qs * K2 + lane;
        pd[o] = L == kMaxKey ? __builtin_inff() : kdist(L);
        pi[o] = L == kMaxKey ? kNoId : (uint32_t)L;
    }
}

// ---- culled KinematicChain scan --------------------------------------------------------------
// PRM*'s kNN on the chain metric (demos/KinematicChain.h:105-124 = link * sum_i |P_i(a) - P_i(b)|
// over the joint positions P_i; ConnectionStrategy.h:145-149 sets k) over the k-d sorted store of
// joint positions (the same device build as SE3 / R^n, boxes over all 2 NM position
// coordinates).  A tile's box bounds the distance of each of its states from below by
// link * sum_i dist(P_i(q), box_i) (each term is >= the distance from P_i(q) to the 2-D box of
// the P_i), so a tile whose bound is not below a query's threshold cannot change its list.
// One wave serves G queries adjacent in k-d order (sorted by home tile) over one chunk of tiles
// (grid.y; the certificate merges the chunk lists, as for the brute-force wave scan):
//   1. threshold: the G queries scan the 4 tiles around the middle query's home tile; each
//      query's tau = the K2-th smallest screened distance there.  At least K2 stored states
//      have d32 <= tau, so the K2 best of all stored states have d32 <= tau: every chunk keeps
//      only keys <= (tau, max id) and the merged lists are still the exact K2 best (those home
//      tiles belong to some chunk, so the merge is full).  The lists are then emptied.
//   2. the chunk's tiles in blocks of 64 (lane = tile): box bounds of the G queries, one ballot
//      per query; the passing tiles are fetched (lane = state) and scanned for every query whose
//      own bound is still below its threshold, with the wave scan's outer-links-first partial
//      sums and wave-wide early exit.
// Lists hold sorted positions (round 4; were original ids): the certificate reads each
// candidate's fp64 features as one contiguous AoS row (SortedStore::rows64, 192 B for 12 links)
// instead of 24 gathers by id, and maps positions to ids (SortedStore::ids).  Keys (distance,
// position) are a total order as (distance, id) was, which is all the thresholds' argument needs;
// the certificate ranks by (exact distance, id).
//
// MODE 0: as above.  MODE 1 / 2 (the default, two launches): the thresholds are shared across the
// chunks.  Each chunk only sees 1/S of the store, so its own list converges to its chunk's K2-th
// distance — for a chunk far from the query that is far above the store's — and culls little.
// But the store's K2 best have keys <= every chunk's K2-th key (a chunk's K2-th key has K2 stored
// states at or below it), so any chunk may drop what is above the smallest of them:
//   MODE 1 (one wave per group, no chunks): phase 1 over kChainTauTiles tiles around the home
//     tile; key[q] = (tau, max id) to global memory;
//   MODE 2 (the chunk pass): starts from key[q], and after every 64-tile block publishes its own
//     K2-th key (atomicMin, device scope) and takes the smallest published one — the chunk holding
//     the query's neighbourhood tightens everybody's threshold.  The chunk's blocks are visited
//     from the one holding the home tile on (wrapping), so that chunk publishes early.
// The merge stays exact: a store state among the K2 best has a key <= every published key, and
// fewer than K2 states of its own chunk are below it, so it is in its chunk's list.
//
// Q16 (the default): the tiles are read from the 16-bit fixed-point copy (SortedStore::rows16,
// half the bytes of the fp32 rows) and the screen works in quanta: term i = step_i *
// |code_i(s) - (P_i(q) + i + 1) S_i|, step_i = 1 / S_i.  Every quantity that decides what a list
// keeps is this d16; the tile bounds stay on the fp32 boxes and are lowered by qerr
// (chain_q16_error, >= |d16 - d32|), and the certificate's screen error grows by the same qerr.
constexpr int kChainTauTiles = 16;
// MODE 1 is the pre-pass (the home window's thresholds, published by atomicMin), MODE 2 the chunk
// pass.  (Measured and rejected, DESIGN §8: each chunk on its own thresholds; the next tile in
// flight; pre-pass windows of 8 / 32 tiles and pre-passes split in parts.)
template <int F, int K2, int G, int MODE, bool Q16>
__global__ __launch_bounds__(64) void knn32_chain_cull_kernel(
    const float *__restrict__ rows, const uint32_t *__restrict__ rows16, uint32_t n_pad,
    const uint32_t *__restrict__ ids, uint32_t ntiles, const float *__restrict__ tbox, const float *__restrict__ q32,
    const uint32_t *__restrict__ qkeys, uint32_t nq, uint32_t chunk_tiles, float link, int nlinks, float qerr,
    float *__restrict__ pd, uint32_t *__restrict__ pi, unsigned long long *__restrict__ counters,
    unsigned long long *__restrict__ shared_key) {
    constexpr int NM = F / 2;
    static_assert(K2 <= 64 && NM % 2 == 0 && (MODE == 1 || MODE == 2), "chain cull shape");
    __shared__ __attribute__((aligned(16))) float qrow[G * F];
    __shared__ __attribute__((aligned(16))) float qcode[Q16 ? G * F : 1];  // the queries in quanta
    const int lane = threadIdx.x;
    const uint32_t g0 = blockIdx.x * G;
    for (int t = lane; t < G * F; t += 64) {
        const uint32_t qi = g0 + t / F;
        const float v = qi < nq ? q32[(size_t)qi * F + t % F] : __builtin_nanf("");
        qrow[t] = v;
        if constexpr (Q16) {
            const int f = t % F, li = f < NM ? f : f - NM;
            qcode[t] = (v + (float)(li + 1)) * (kChainQ16 / (float)(2 * (li + 1)));
        }
    }
    __syncthreads();
    uint32_t qoff = 0;  // re-read the wave-uniform query rows from LDS (see knn32_group_kernel)
    uint64_t Lk[G];
    float td[G];
    uint64_t tk[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        Lk[g] = kMaxKey;
        td[g] = g0 + g < nq ? __builtin_inff() : -__builtin_inff();
        tk[g] = g0 + g < nq ? kMaxKey : 0ull;
    }
    uint64_t tauk[G];  // the chunk-independent key bound (phase 1)
    auto offer = [&](int g, float d, uint32_t id) {
        uint64_t bm = __ballot(d < td[g]);
        const uint64_t mk = kpack(d, id);
        while (bm) {
            const int l = __builtin_ctzll(bm);
            bm &= bm - 1;
            const uint64_t ck = readlane_k(mk, l);
            if (ck < tk[g]) {
                const uint64_t pv = shr1_k(Lk[g], 0ull);
                const bool lt_prev = lane > 0 && ck < pv;
                Lk[g] = lt_prev ? pv : (ck < Lk[g] ? ck : Lk[g]);
                const uint64_t lk = readlane_k(Lk[g], K2 - 1);
                if (lk < tk[g]) {
                    tk[g] = lk;
                    td[g] = kdist(lk);
                }
            }
        }
    };
    uint32_t visited = 0, qscans = 0;
    auto load_raw = [&](uint32_t t, uint32_t (&w)[NM]) { load_blk<NM>(rows16, t, lane, w); };
    auto decode = [&](const uint32_t (&w)[NM], float (&x)[F]) {
#pragma unroll
        for (int j = 0; j < NM; ++j) {
            x[2 * j] = (float)(w[j] & 0xFFFFu);
            x[2 * j + 1] = (float)(w[j] >> 16);
        }
        if ((w[0] & 0xFFFFu) == 0xFFFFu) x[0] = __builtin_nanf("");  // padding / removed
    };
    auto load_tile = [&](uint32_t t, float (&x)[F]) {
        if constexpr (Q16) {
            uint32_t w[NM];
            load_raw(t, w);
            decode(w, x);
        } else {
            load_blk<F>(rows, t, lane, x);
        }
    };
    // query g against the lane's state x, outermost links first (|P_i(a) - P_i(b)| grows with
    // i), the wave leaving as soon as no lane's partial sum is below the threshold
    auto scan = [&](int g, const float (&x)[F], uint32_t id) {
        ++qscans;
        const float *qq = Q16 ? &qcode[qoff + g * F] : &qrow[qoff + g * F];
        float acc = 0.f;
#pragma unroll
        for (int s = 0; s < NM; s += 2) {
            const int i = NM - 2 - s;
            if (i < nlinks) {
                const f2 dx = f2{x[i], x[i + 1]} - f2{qq[i], qq[i + 1]};
                const f2 dy = f2{x[NM + i], x[NM + i + 1]} - f2{qq[NM + i], qq[NM + i + 1]};
                const f2 s2 = pk_fma(dy, dy, dx * dx);
                if constexpr (Q16) {  // back from quanta: step_i = 2 (i + 1) / kChainQ16 (immediates)
                    acc = fmaf(__builtin_amdgcn_sqrtf(s2.x), (float)(2 * (i + 1)) / kChainQ16, acc);
                    if (i + 1 < nlinks) acc = fmaf(__builtin_amdgcn_sqrtf(s2.y), (float)(2 * (i + 2)) / kChainQ16, acc);
                } else {
                    acc += __builtin_amdgcn_sqrtf(s2.x);
                    if (i + 1 < nlinks) acc += __builtin_amdgcn_sqrtf(s2.y);
                }
            }
            if (s + 2 < NM && !__ballot(acc * link < td[g])) return;
        }
        offer(g, acc * link, id);
    };
    // 1. thresholds from the home neighbourhood
    const uint32_t home = min(qkeys[min(g0 + G / 2, nq - 1)], ntiles - 1);
    auto up_of = [](float tau) {  // the next float above tau (>= 0 or +inf): a distance equal to tau still passes
        return tau < __builtin_inff() ? __uint_as_float(__float_as_uint(tau) + 1u) : tau;
    };
    if constexpr (MODE == 2) {  // the pre-pass's keys
        uint64_t v = kMaxKey;
        if (lane < G && g0 + lane < nq)
            v = __hip_atomic_load(&shared_key[g0 + lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int g = 0; g < G; ++g) {
            tk[g] = g0 + g < nq ? readlane_k(v, g) : 0ull;
            td[g] = g0 + g < nq ? up_of(kdist(tk[g])) : -__builtin_inff();
        }
    } else {  // the pre-pass: the kChainTauTiles tiles around the home tile
        const uint32_t h = home, span = (uint32_t)kChainTauTiles;
        const uint32_t t0 = min(h >= span / 2 ? h - span / 2 : 0u, ntiles), t1 = min(t0 + span, ntiles);
        for (uint32_t t = t0; t < t1; ++t) {
            float x[F];
            load_tile(t, x);
            const uint32_t id = t * kCullTile + (uint32_t)lane;  // sorted position
            asm volatile("" : "+s"(qoff));
#pragma unroll
            for (int g = 0; g < G; ++g) scan(g, x, id);
        }
#pragma unroll
        for (int g = 0; g < G; ++g) {
            // tau = the K2-th screened distance (+inf when fewer live states): keys <= (tau, max)
            const float tau = kdist(readlane_k(Lk[g], K2 - 1));
            tauk[g] = g0 + g < nq ? kpack(tau, 0xFFFFFFFFu) : 0ull;
            Lk[g] = kMaxKey;
            tk[g] = tauk[g];
            td[g] = g0 + g < nq ? up_of(tau) : -__builtin_inff();
        }
        // the window's K2-th key bounds the store's: publish it (keep the smallest)
#pragma unroll
        for (int g = 0; g < G; ++g)
            if (lane == g && g0 + g < nq)
                (void)__hip_atomic_fetch_min(&shared_key[g0 + g], tauk[g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    // 2. the chunk's tiles (MODE 2: from the home tile's block on, wrapping)
    const uint32_t c0 = blockIdx.y * chunk_tiles, c1 = min(c0 + chunk_tiles, ntiles);
    const uint32_t nblk = c1 > c0 ? (c1 - c0 + 63) / 64 : 0u;
    const uint32_t sblk = (home >= c0 && home < c1) ? (home - c0) / 64 : 0u;
    // blocks nearest the home tile in k-d order first: a chunk below the home tile walks its
    // blocks backwards, one above it forwards, the home chunk from the home block on (wrapping) —
    // each chunk's own list then tightens on its nearest tiles first (measured: 4.75-4.82 against
    // 4.84-4.85 ms on cfg4)
    const bool backwards = c1 <= home;
    for (uint32_t bi = 0; bi < nblk; ++bi) {
        const uint32_t tb = c0 + (backwards ? nblk - 1 - bi : (sblk + bi) % nblk) * 64;
        {  // share the thresholds: publish this chunk's K2-th keys, take the smallest
            if (bi) {
                uint64_t mine = kMaxKey;
#pragma unroll
                for (int g = 0; g < G; ++g) mine = lane == g ? tk[g] : mine;
                uint64_t best = kMaxKey;
                if (lane < G && g0 + lane < nq)
                    best = __hip_atomic_fetch_min(&shared_key[g0 + lane], mine, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
                for (int g = 0; g < G; ++g) {
                    const uint64_t o = readlane_k(best, g);
                    if (g0 + g < nq && o < tk[g]) {
                        tk[g] = o;
                        td[g] = up_of(kdist(o));
                    }
                }
            }
        }
        const uint32_t t = tb + lane;
        float lb[G];
#pragma unroll
        for (int g = 0; g < G; ++g) lb[g] = t < c1 ? 0.f : __builtin_inff();
        asm volatile("" : "+s"(qoff));
        if (t < c1) {
            const float *bx = tbox + (size_t)t * (2 * F);
#pragma unroll
            for (int i = 0; i < NM; i += 2) {
                if (i < nlinks) {
                    const float2 lx = *reinterpret_cast<const float2 *>(bx + i);
                    const float2 ly = *reinterpret_cast<const float2 *>(bx + NM + i);
                    const float2 hx = *reinterpret_cast<const float2 *>(bx + F + i);
                    const float2 hy = *reinterpret_cast<const float2 *>(bx + F + NM + i);
#pragma unroll
                    for (int g = 0; g < G; ++g) {
                        const float *qq = &qrow[qoff + g * F];
                        const float ax = gap(lx.x - qq[i], qq[i] - hx.x), ay = gap(ly.x - qq[NM + i], qq[NM + i] - hy.x);
                        lb[g] += __builtin_amdgcn_sqrtf(fmaf(ay, ay, ax * ax));
                        if (i + 1 < nlinks) {
                            const float bx2 = gap(lx.y - qq[i + 1], qq[i + 1] - hx.y);
                            const float by2 = gap(ly.y - qq[NM + i + 1], qq[NM + i + 1] - hy.y);
                            lb[g] += __builtin_amdgcn_sqrtf(fmaf(by2, by2, bx2 * bx2));
                        }
                    }
                }
            }
            // the sum of the per-link bounds rounds like the distance's own sum (monotone in its
            // terms): shave (n + 2) u off so that the bound stays below every screened distance
#pragma unroll
            for (int g = 0; g < G; ++g) lb[g] = lb[g] * link * (1.f - 4e-6f) - qerr;
        }
        uint64_t need = 0;
#pragma unroll
        for (int g = 0; g < G; ++g) need |= __ballot(lb[g] < td[g]);
        while (need) {
            const int l = __builtin_ctzll(need);
            need &= need - 1;
            float x[F];
            load_tile(tb + (uint32_t)l, x);
            const uint32_t id = (tb + (uint32_t)l) * kCullTile + (uint32_t)lane;
            ++visited;
            asm volatile("" : "+s"(qoff));
#pragma unroll
            for (int g = 0; g < G; ++g)
                if (readlane_f(lb[g], l) < td[g]) scan(g, x, id);
            uint64_t still = 0;  // drop the tiles the tightened thresholds now exclude
#pragma unroll
            for (int g = 0; g < G; ++g) still |= __ballot(lb[g] < td[g]);
            need &= still;
        }
    }
    if (counters && lane == 0) {
        unsigned long long *cs = counters + (blockIdx.x % kCounterSlots) * kCounterStride;
        atomicAdd(&cs[0], (unsigned long long)visited);
        atomicAdd(&cs[1], (unsigned long long)(c1 > c0 ? c1 - c0 : 0));
        atomicAdd(&cs[2], (unsigned long long)qscans);
    }
#pragma unroll
    for (int g = 0; g < G; ++g)
        if (g0 + g < nq && lane < K2) {
            const size_t o = ((size_t)blockIdx.y * nq + g0 + g) * K2 + lane;
            pd[o] = kdist(Lk[g]);
            pi[o] = (uint32_t)Lk[g];
        }
}

template <int SP>
__device__ __forceinline__ double screen_error(const DevSpace &sp, double B, double L, double eta = 0.0) {
    double e = 0.0;
    if constexpr (SP == OMPL_GPU_SPACE_SE3) {
        e = sp.w0 * (6.0 * 1.7320508075688772 * kU * B) + 6.0 * kU * L +
            sp.w1 * (2.25 * sqrt(0.5 * eta + 1e-15) + 2e-6 + 4.5e-5);
    } else if constexpr (SP == OMPL_GPU_SPACE_SO3) {
        e = 1.1 * sqrt(12.0 * kU) + 2e-6 + 4.5e-5;
    } else if constexpr (SP == OMPL_GPU_SPACE_KCHAIN) {
        // |P_i| <= i: rounding the positions and differencing them costs <= 4 u i per
        // coordinate, each term <= 14.2 u i, so the terms together <= 7.1 u n (n + 1); the n
        // additions and the final link product cost <= (n + 1) u of the sum
        const double n = (double)sp.dim;
        // eta: the 16-bit screen's quantisation bound (chain_q16_error) when it ran, else 0
        e = sp.link * 8.0 * kU * n * (n + 1.0) + (n + 2.0) * kU * L + sp.link * n * sqrt(2.0 * kFltMin) + eta;
    } else {
        e = 6.0 * sqrt((double)sp.dim) * kU * B + 6.0 * kU * L;
    }
    if constexpr (SP == OMPL_GPU_SPACE_SE3) e += sp.w0 * sqrt(3.0 * kFltMin);
    if constexpr (SP == OMPL_GPU_SPACE_REALVECTOR) e += sqrt(16.0 * kFltMin);
    return 2.0 * e;
}

// |norm^2 - 1| of an SE3 query's quaternion (fp64), for screen_error
template <int SP>
__device__ __forceinline__ double query_eta(const double *qv) {
    if constexpr (SP == OMPL_GPU_SPACE_SE3) {
        const double n = qv[3] * qv[3] + qv[4] * qv[4] + qv[5] * qv[5] + qv[6] * qv[6];
        return fabs(n - 1.0);
    }
    return 0.0;
}

template <int SP, int F, int K2, int K>
__global__ __launch_bounds__(256) void knn_certify_kernel(const float *__restrict__ pd, const uint32_t *__restrict__ pi,
                                                          uint32_t S, uint32_t nq, const uint32_t *__restrict__ perm,
                                                          const double *__restrict__ feat64, uint64_t cap,
                                                          const double *__restrict__ qf64, DevSpace sp,
                                                          float absmax, float qeta, uint32_t n_live,
                                                          double *__restrict__ out_d,
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
            ex.offer(feat_dist<SP, F, SP == OMPL_GPU_SPACE_KCHAIN ? F / 2 : 0>(sv, qv, sp), id);  // fp64, reference order
        }
    }
    bool ok = true;
    if (t.i[K2 - 1] != kNoId) {  // the list is full: prove that no excluded element can enter
        double B = absmax;
        const int nc = SP == OMPL_GPU_SPACE_SE3 ? 3 : (SP == OMPL_GPU_SPACE_REALVECTOR ? F : 0);
        for (int c = 0; c < nc; ++c) B = fmax(B, fabs(qv[c]));
        const double L = (double)t.d[K2 - 1];
        double dk = ex.d[K - 1];
#pragma unroll
        for (int j = 0; j < K; ++j)
            if (j == (int)out_k - 1) dk = ex.d[j];
        ok = dk + screen_error<SP>(sp, B, L, (double)qeta + query_eta<SP>(qv)) < L * (1.0 - 8.0 * kU);
    } else {  // a list that is not full must hold every live state (an overflowed d32 is never admitted)
        uint32_t held = 0;
#pragma unroll
        for (int j = 0; j < K2; ++j) held += t.i[j] != kNoId ? 1u : 0u;
        ok = held >= n_live;
    }
#pragma unroll
    for (int j = 0; j < K; ++j)
        if (j < (int)out_k) {
            out_d[(size_t)q * out_k + j] = ex.d[j];
            out_i[(size_t)q * out_k + j] = ex.i[j];
        }
    if (!ok) fail_list[atomicAdd(fail_count, 1u)] = q;
}

// The same certificate with one lane per candidate (single screening list per query, the
// group walk's output): K2 lanes of a wave serve one query, each recomputes its candidate's
// exact distance (the K2 gathers of a query are in flight together instead of one thread
// issuing them in turn), ranks it by (distance, id) against its K2 - 1 neighbours with
// cross-lane reads, and writes itself at its rank if the rank is below out_k.  The proof
// is the same expression as knn_certify_kernel's on the same values.
template <int SP, int F, int K2>
__global__ __launch_bounds__(256) void knn_certify_wave_kernel(const float *__restrict__ pd,
                                                               const uint32_t *__restrict__ pi, uint32_t nq,
                                                               const uint32_t *__restrict__ perm,
                                                               const double *__restrict__ feat64, uint64_t cap,
                                                               const uint32_t *__restrict__ pos_ids,
                                                               const double *__restrict__ rows64,
                                                               const double *__restrict__ qf64, DevSpace sp,
                                                               float absmax, float qeta, uint32_t n_live,
                                                               uint32_t k2, double *__restrict__ out_d,
                                                               uint32_t *__restrict__ out_i, uint32_t out_k,
                                                               uint32_t *__restrict__ fail_count,
                                                               uint32_t *__restrict__ fail_list,
                                                               float xerr = 0.f) {
    static_assert(K2 == 16 || K2 == 32 || K2 == 64, "lanes per query");
    constexpr int QPB = 256 / K2;
    const uint32_t qs = blockIdx.x * QPB + threadIdx.x / K2;
    const int j = (int)(threadIdx.x % K2);
    const int gbase = (int)(threadIdx.x & 63) - j;  // wave lane of this query's entry 0
    const bool live = qs < nq;                      // uniform over the query's lanes
    const float d32 = live ? pd[(size_t)qs * K2 + j] : __builtin_inff();
    const uint32_t e = live ? pi[(size_t)qs * K2 + j] : kNoId;  // id, or sorted position (rows64)
    const uint32_t q = live ? perm[qs] : 0u;
    double qv[F];
#pragma unroll
    for (int f = 0; f < F; ++f) qv[f] = live ? qf64[(size_t)q * F + f] : 0.0;
    double d = __builtin_inf();
    uint32_t id = kNoId;
    if (e != kNoId) {
        double sv[F];
        if (rows64) {  // the group walk's lists: one contiguous fp64 row per candidate
            constexpr int FA = (F + 3) & ~3;
            id = pos_ids[e];
            const double2 *r2 = reinterpret_cast<const double2 *>(rows64 + (size_t)e * FA);
#pragma unroll
            for (int c = 0; c < FA / 2; ++c) {
                const double2 v = r2[c];
                if (2 * c < F) sv[2 * c] = v.x;
                if (2 * c + 1 < F) sv[2 * c + 1] = v.y;
            }
        } else {
            id = e;
#pragma unroll
            for (int f = 0; f < F; ++f) sv[f] = feat64[(uint64_t)f * cap + id];
        }
        d = feat_dist<SP, F, SP == OMPL_GPU_SPACE_KCHAIN ? F / 2 : 0>(sv, qv, sp);  // fp64, reference order
    }
    uint32_t rank = 0;
#pragma unroll 4
    for (int m = 0; m < K2; ++m) {
        const double dm = __shfl(d, gbase + m);
        const uint32_t im = (uint32_t)__shfl((int)id, gbase + m);
        rank += (dm < d || (dm == d && (im < id || (im == id && m < j)))) ? 1u : 0u;
    }
    // exact k-th distance = the largest of the first out_k ranks
    double dk = rank < out_k ? d : -__builtin_inf();
#pragma unroll
    for (int o = K2 / 2; o > 0; o >>= 1) dk = fmax(dk, __shfl_xor(dk, o));
    // the walk's list holds k2 <= K2 entries (the rest of the K2 lanes are empty)
    const bool full = (uint32_t)__shfl((int)id, gbase + (int)k2 - 1) != kNoId;
    const float L32 = __shfl(d32, gbase + (int)k2 - 1);
    // entries this query's list holds (its K2 lanes of the wave)
    uint64_t gmask = ~0ull;
    if constexpr (K2 < 64) gmask = ((1ull << K2) - 1ull) << gbase;
    const uint32_t held = (uint32_t)__popcll(__ballot(id != kNoId) & gmask);
    bool ok = full || held >= n_live;  // not full: it must hold every live state
    if (full) {  // prove that no element outside the list can enter (knn_certify_kernel)
        double B = absmax;
        const int nc = SP == OMPL_GPU_SPACE_SE3 ? 3 : (SP == OMPL_GPU_SPACE_REALVECTOR ? F : 0);
        for (int c = 0; c < nc; ++c) B = fmax(B, fabs(qv[c]));
        const double L = (double)L32;
        // xerr: a 16-bit screen's coding bound, on both sides like the screen error (x 2)
        ok = dk + screen_error<SP>(sp, B, L, (double)qeta + query_eta<SP>(qv)) + 2.0 * (double)xerr <
             L * (1.0 - 8.0 * kU);
    }
    if (!live) return;
    if (rank < out_k) {
        out_d[(size_t)q * out_k + rank] = d;
        out_i[(size_t)q * out_k + rank] = id;
    }
    if (j == 0 && !ok) fail_list[atomicAdd(fail_count, 1u)] = q;
}

// ---- culled radius search (SE3, R^n) ------------------------------------------------------
// nearestR (NearestNeighborsGNAT.h:236-245; Linear :135-142: d <= r inclusive, ascending).
// The bound is fixed, so no step of the walk waits on an earlier result: a wave serves G
// Morton-adjacent queries, tests 64 super-tile boxes per ballot and the 32 tile boxes of a
// passing super-tile at once, and scans a tile only for the queries whose own box bound
// comes within their inflated radius.  The fp32 screen keeps d32 <= r + e (e = the screen's
// error bound, the same as the kNN certificate's, so no element with d <= r is lost); every
// kept element is then decided by its exact fp64 distance in the reference's operation
// order.  FILL = false counts the hits of each query, FILL = true writes (id, d) into the
// query's CSR segment in tile order; the caller sorts each segment by (distance, id).
// MODE 2 (SLAB) counts like MODE 0 and also writes the first `slab` hits of each query to its
// fixed-size slab, so that one walk suffices when no query has more hits than that.
// (Measured and rejected: 7 / 8 waves per SIMD from the compiler — 72 / 64 VGPRs with 24 / 68 B
// of scratch spills — against the default's 80 VGPRs, 6 waves; round 6: the next super-tile's
// boxes staged in LDS by LDS-DMA, 69 VGPRs at 7 waves / 64 at 8 without scratch — 1.24-1.26 /
// 1.27-1.28 against 1.19-1.22 ms.)
#define OMPL_RADIUS_LB __launch_bounds__(64)
// Q16 (SE3, MODE 2; Q16 = false reads the fp32 rows): the tiles come from the 16-bit copy
// (SortedStore::rows16, 16 B per state against 28), decoded to fp32 once per tile; every
// threshold grows by qerr >= |d16 - d32| (se3_q16_error), so no state with d32 <= r + e is lost
// and the box bounds (over the fp32 rows) stay valid.
template <int SP, int F, int G, int MODE, bool Q16 = false>
__global__ OMPL_RADIUS_LB void radius32_group_kernel(
    const float *__restrict__ rows, uint32_t n_pad, const uint32_t *__restrict__ ids, uint32_t ntiles,
    const float *__restrict__ tbox, const float *__restrict__ sbox, uint32_t nsuper, const float *__restrict__ mbox,
    uint32_t nmega, const float *__restrict__ q32, const uint32_t *__restrict__ perm, uint32_t nq, const double *__restrict__ rows64,
    const double *__restrict__ qf64, DevSpace sp, float absmax, float qeta, double r, uint64_t *__restrict__ counts,
    const uint64_t *__restrict__ offsets, uint32_t *__restrict__ out_i, double *__restrict__ out_d,
    unsigned long long *__restrict__ counters, uint32_t slab, const uint32_t *__restrict__ rows16 = nullptr,
    Q16Geo qg = Q16Geo{}, double qerr = 0.0) {
    static_assert(!Q16 || SP == OMPL_GPU_SPACE_SE3, "16-bit rows: SE3");
    constexpr int FS = Geo<SP, F>::FS, R = Geo<SP, F>::R, BW = Geo<SP, F>::BW;
    constexpr int GH = G / 2;
    constexpr bool FILL = MODE == 1, SLAB = MODE == 2;
    static_assert(G % 2 == 0, "radius walk shape");
    __shared__ __attribute__((aligned(16))) float qrow[G * FS];
    const int lane = threadIdx.x;
    const int half = lane >> 5;
    const float w0 = (float)sp.w0, w1 = (float)sp.w1;
    // XCD-aware group order, as in knn32_group_kernel
    const uint32_t nb = gridDim.x, xq = nb / 8, xr = nb % 8, xb = blockIdx.x % 8;
    const uint32_t blk = (xb < xr ? xb * (xq + 1) : xr * (xq + 1) + (xb - xr) * xq) + blockIdx.x / 8;
    const uint32_t g0 = blk * G;
    for (int t = lane; t < G * FS; t += 64) {
        const uint32_t qi = g0 + t / FS;
        qrow[t] = qi < nq ? q32[(size_t)qi * FS + t % FS] : __builtin_nanf("");
    }
    __syncthreads();
    // the exact query rows live in LDS (read on a hit, a broadcast): G x F doubles held in
    // VGPRs for the whole walk cost 2 G F registers (56 for SE3, G = 4)
    __shared__ double qv[G][F];
    uint32_t qo[G];
    float thr[G];
    uint64_t cur[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const bool live = g0 + g < nq;
        qo[g] = live ? perm[g0 + g] : 0u;
        double qd[F];
#pragma unroll
        for (int f = 0; f < F; ++f) qd[f] = live ? qf64[(size_t)qo[g] * F + f] : 0.0;
        if (lane < F) qv[g][lane] = qd[lane < F ? lane : 0];
        double B = absmax;
        const int nc = SP == OMPL_GPU_SPACE_SE3 ? 3 : F;
        for (int c = 0; c < nc; ++c) B = fmax(B, fabs(qd[c]));
        // every element with d <= r has d32 <= r + e; rounding to fp32 is covered by the 16 u
        const double t = (r + screen_error<SP>(sp, B, r, (double)qeta + query_eta<SP>(qd)) + (Q16 ? qerr : 0.0)) *
                         (1.0 + 16.0 * kU);
        thr[g] = live ? (float)t : -__builtin_inff();
        cur[g] = (FILL && live) ? offsets[qo[g]] : 0ull;
    }
    __syncthreads();
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    uint64_t cnt[G];
#pragma unroll
    for (int g = 0; g < G; ++g) cnt[g] = 0;
    uint32_t visited = 0, qscans = 0;
    // re-read the wave-uniform query rows from LDS at every use through an offset the compiler
    // cannot see through, instead of letting it hoist them into VGPRs for the whole walk
    uint32_t qoff = 0;
    // super-tiles whose box comes within some query's bound, 64 box tests per round.  (Measured
    // and rejected, DESIGN §8: tile bounds only for the queries a super-tile passes, paired onto
    // the half-waves; a translation-only pre-test before the chord bound.)
    uint32_t sb = 0, base = 0;
    uint64_t sm = 0;
    // mega-tiles first (64 mega boxes per round), then the super-tiles of each passing mega
    uint32_t mb = 0, mbase = 0;
    uint64_t mm = 0;
    auto next_mega = [&]() -> int {
        while (!mm) {
            if (mb >= nmega) return -1;
            asm volatile("" : "+s"(qoff));
            const uint32_t mi = mb + lane;
            bool need = false;
            if (mi < nmega) {
                float bx[BW];
                const float4 *b4 = reinterpret_cast<const float4 *>(mbox + (size_t)mi * BW);
#pragma unroll
                for (int c = 0; c < BW / 4; ++c) {
                    const float4 v = b4[c];
                    bx[4 * c] = v.x; bx[4 * c + 1] = v.y; bx[4 * c + 2] = v.z; bx[4 * c + 3] = v.w;
                }
#pragma unroll
                for (int g = 0; g < G; ++g) {
                    need |= box_lb<SP, F>(bx, &qrow[qoff + g * FS], w0, w1) <= thr[g];
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
            mm = __ballot(need);
            mbase = mb;
            mb += 64;
        }
        const int l = __builtin_ctzll(mm);
        mm &= mm - 1;
        return (int)(mbase + l);
    };
    auto next_super = [&]() -> int {
        while (!sm) {
            const int mg = next_mega();
            if (mg < 0) return -1;
            sb = (uint32_t)mg * kMegaSupers;
            asm volatile("" : "+s"(qoff));
            const uint32_t s = sb + lane;
            bool need = false;
            if (s < nsuper) {
                float bx[BW];
                const float4 *b4 = reinterpret_cast<const float4 *>(sbox + (size_t)s * BW);
#pragma unroll
                for (int c = 0; c < BW / 4; ++c) {
                    const float4 v = b4[c];
                    bx[4 * c] = v.x; bx[4 * c + 1] = v.y; bx[4 * c + 2] = v.z; bx[4 * c + 3] = v.w;
                }
#pragma unroll
                for (int g = 0; g < G; ++g) {
                    need |= box_lb<SP, F>(bx, &qrow[qoff + g * FS], w0, w1) <= thr[g];
                    __builtin_amdgcn_sched_barrier(0);  // one bound at a time (temporaries)
                }
            }
            sm = __ballot(need);
            base = sb;
        }
        const int l = __builtin_ctzll(sm);
        sm &= sm - 1;
        return (int)(base + l);
    };
    // this lane's row of super-tile ss's tile boxes (tile ss * 32 + (lane & 31)); rows past the
    // last tile read as empty boxes (bound +inf)
    auto load_tbox = [&](uint32_t ss, float (&bx)[BW]) {
        const uint32_t tt = ss * kSuperTiles + (lane & 31);
        if (tt < ntiles) {
            const float4 *b4 = reinterpret_cast<const float4 *>(tbox + (size_t)tt * BW);
#pragma unroll
            for (int c = 0; c < BW / 4; ++c) {
                const float4 v = b4[c];
                bx[4 * c] = v.x; bx[4 * c + 1] = v.y; bx[4 * c + 2] = v.z; bx[4 * c + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int c = 0; c < BW; ++c) bx[c] = c < Geo<SP, F>::NB ? __builtin_inff() : -__builtin_inff();
            if constexpr (SP == OMPL_GPU_SPACE_SE3) bx[2 * Geo<SP, F>::NB] = bx[2 * Geo<SP, F>::NB + 1] = 0.f;
        }
    };
    auto load_tile = [&](uint32_t ss, int t, float (&x)[R], uint32_t &id) {
        const uint64_t p = (uint64_t)(ss * kSuperTiles + t) * kCullTile + lane;
        load_blk<R>(rows, ss * kSuperTiles + t, lane, x);
        id = ids[p];
    };
    // Q16: a tile in flight stays raw (4 words per lane) and is decoded when it is scanned, so
    // the next tile's loads overlap the current scan
    auto load_raw = [&](uint32_t ss, int t, uint32_t (&w)[4], uint32_t &id) {
        const uint64_t p = (uint64_t)(ss * kSuperTiles + t) * kCullTile + lane;
        load_blk<4>(rows16, ss * kSuperTiles + t, lane, w);
        id = ids[p];
    };
    auto decode = [&](const uint32_t (&w)[4], float (&v)[R]) {
#pragma unroll
        for (int rr = 0; rr < R; ++rr) {
            const uint32_t c = (rr & 1) ? (w[rr >> 1] >> 16) : (w[rr >> 1] & 0xFFFFu);
            v[rr] = fmaf((float)c, qg.step[rr], qg.lo[rr]);
            if (rr == 0 && c == 0xFFFFu) v[0] = __builtin_nanf("");  // padding / removed
        }
    };
    auto scan_tile = [&](uint32_t ss, int t, const float (&x)[R], uint32_t id, const float (&lb)[GH]) {
        asm volatile("" : "+s"(qoff));
        const uint64_t p = (uint64_t)(ss * kSuperTiles + t) * kCullTile + lane;
        ++visited;
#pragma unroll
        for (int g = 0; g < G; ++g) {
            if (!(readlane_f(lb[g % GH], t + (g < GH ? 0 : 32)) <= thr[g])) continue;
            ++qscans;
            bool hit;  // NaN never hits
            if constexpr (SP == OMPL_GPU_SPACE_SE3) {  // chord bound first, as in the kNN walk
                const float *qq = &qrow[qoff + g * FS];
                const float dx = x[0] - qq[0], dy = x[1] - qq[1], dz = x[2] - qq[2];
                float tt = dx * dx;
                tt = fmaf(dy, dy, tt);
                tt = fmaf(dz, dz, tt);
                const float c2 = chord2(x + 3, qq + 4);
                const float c = __builtin_amdgcn_sqrtf(c2), wt = w0 * __builtin_amdgcn_sqrtf(tt);
                hit = __ballot(fmaf(w1, c, wt) <= thr[g]) && fmaf(w1, chord_theta(c, c2), wt) <= thr[g];
            } else {
                hit = state_dist32<SP, F>(x, &qrow[qoff + g * FS], w0, w1) <= thr[g];
            }
            if constexpr (SLAB) {
                // the screen's candidates go to the slab as sorted positions; their exact fp64
                // decisions run afterwards (radius_slab_exact_kernel), off the walk: no fp64
                // registers or dependent row loads here
                const uint64_t bm = __ballot(hit);
                if (hit) {
                    const uint64_t j = cnt[g] + (uint64_t)__popcll(bm & lt);
                    if (j < slab) out_i[(uint64_t)qo[g] * slab + j] = (uint32_t)p;
                }
                cnt[g] += (uint64_t)__popcll(bm);
                continue;
            }
            double dd = 0.0;
            if (hit) {  // exact decision from the sorted fp64 row (coalesced over the tile)
                constexpr int FA = (F + 3) & ~3;
                double sv[F];
                const double2 *r2 = reinterpret_cast<const double2 *>(rows64 + p * FA);
#pragma unroll
                for (int c = 0; c < FA / 2; ++c) {
                    const double2 v = r2[c];
                    if (2 * c < F) sv[2 * c] = v.x;
                    if (2 * c + 1 < F) sv[2 * c + 1] = v.y;
                }
                double qd[F];
#pragma unroll
                for (int f = 0; f < F; ++f) qd[f] = (&qv[0][0])[qoff + g * F + f];
                dd = feat_dist<SP, F, 0>(sv, qd, sp);
                hit = dd <= r;
            }
            const uint64_t bm = __ballot(hit);
            if (FILL && hit) {
                const uint64_t pos = cur[g] + (uint64_t)__popcll(bm & lt);
                out_i[pos] = id;
                out_d[pos] = dd;
            }
            cur[g] += (uint64_t)__popcll(bm);
            cnt[g] += (uint64_t)__popcll(bm);
        }
    };
    // Software pipeline (the bound is fixed, so nothing waits on a result): the next tile is
    // fetched while the current one is scanned, and the next super-tile's tile boxes while the
    // current super-tile's tiles are; tiles are visited in the same order as before, so FILL
    // writes each CSR segment in tile order.
    float bx[BW];
    int ss = next_super();
    if (ss >= 0) load_tbox((uint32_t)ss, bx);
    while (ss >= 0) {
        float lb[GH];
        bool tneed = false;
        asm volatile("" : "+s"(qoff));
#pragma unroll
        for (int j = 0; j < GH; ++j) {
            lb[j] = box_lb<SP, F>(bx, &qrow[qoff + (half * GH + j) * FS], w0, w1);
            tneed |= lb[j] <= (half ? thr[GH + j] : thr[j]);
            __builtin_amdgcn_sched_barrier(0);
        }
        uint32_t m = fold_tiles(__ballot(tneed));
        uint32_t id = 0, idn = 0;
        int t = 0, tn = 0;
        const bool have = m != 0;
        if constexpr (Q16) {
            uint32_t x[4], xn[4];
            if (have) {
                t = __builtin_ctz(m);
                m &= m - 1;
                load_raw((uint32_t)ss, t, x, id);
            }
            const int ssn = next_super();
            if (ssn >= 0) load_tbox((uint32_t)ssn, bx);
            while (have) {
                const bool more = m != 0;
                if (more) {
                    tn = __builtin_ctz(m);
                    m &= m - 1;
                    load_raw((uint32_t)ss, tn, xn, idn);
                }
                float xd[R];
                decode(x, xd);
                scan_tile((uint32_t)ss, t, xd, id, lb);
                if (!more) break;
#pragma unroll
                for (int j = 0; j < 4; ++j) x[j] = xn[j];
                id = idn;
                t = tn;
            }
            ss = ssn;
            continue;
        }
        float x[R], xn[R];
        if (have) {
            t = __builtin_ctz(m);
            m &= m - 1;
            load_tile((uint32_t)ss, t, x, id);
        }
        const int ssn = next_super();
        if (ssn >= 0) load_tbox((uint32_t)ssn, bx);
        while (have) {
            const bool more = m != 0;
            if (more) {
                tn = __builtin_ctz(m);
                m &= m - 1;
                load_tile((uint32_t)ss, tn, xn, idn);
            }
            scan_tile((uint32_t)ss, t, x, id, lb);
            if (!more) break;
#pragma unroll
            for (int rr = 0; rr < R; ++rr) x[rr] = xn[rr];
            id = idn;
            t = tn;
        }
        ss = ssn;
    }
    if (lane == 0) {
        if (!FILL) {
#pragma unroll
            for (int g = 0; g < G; ++g)
                if (g0 + g < nq) counts[qo[g]] = cnt[g];
        }
        if (MODE != 0 && counters) {
            unsigned long long *cs = counters + (blockIdx.x % kCounterSlots) * kCounterStride;
            atomicAdd(&cs[3], (unsigned long long)visited);  // tiles fetched by the radius walk
            atomicAdd(&cs[4], (unsigned long long)qscans);   // (tile, query) pairs scanned
        }
    }
}

// Exact decisions of the one-walk radius pass (MODE 2): query q's slab holds the sorted positions
// of its screen candidates (d32 <= r + e, counts[q] of them); a wave per query recomputes each
// candidate's fp64 distance from the sorted fp64 rows in the reference's operation order, keeps
// d <= r (Linear :135-142, inclusive) and compacts the hits in place as (id, d), in candidate
// order.  counts[q] becomes the hit count; a query whose candidates overflowed its slab keeps its
// candidate count (> slab), which sends the call to the two-walk path (exact counts, then fill).
template <int SP, int F>
__global__ __launch_bounds__(64) void radius_slab_exact_kernel(const double *__restrict__ rows64,
                                                               const uint32_t *__restrict__ ids,
                                                               const double *__restrict__ qf64, DevSpace sp, double r,
                                                               uint32_t slab, uint64_t *__restrict__ counts,
                                                               uint32_t *__restrict__ slab_i,
                                                               double *__restrict__ slab_d) {
    constexpr int FA = (F + 3) & ~3;
    const uint32_t q = blockIdx.x, lane = threadIdx.x;
    const uint64_t c = counts[q];
    if (c > slab) return;
    double qv[F];
#pragma unroll
    for (int f = 0; f < F; ++f) qv[f] = qf64[(size_t)q * F + f];
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    const size_t base = (size_t)q * slab;
    uint32_t hits = 0;
    for (uint32_t j0 = 0; j0 < (uint32_t)c; j0 += 64) {
        const uint32_t j = j0 + lane;
        bool hit = false;
        double d = 0.0;
        uint32_t id = kNoId;
        if (j < c) {
            const uint32_t p = slab_i[base + j];
            double sv[F];
            const double2 *r2 = reinterpret_cast<const double2 *>(rows64 + (size_t)p * FA);
#pragma unroll
            for (int cc = 0; cc < FA / 2; ++cc) {
                const double2 v = r2[cc];
                if (2 * cc < F) sv[2 * cc] = v.x;
                if (2 * cc + 1 < F) sv[2 * cc + 1] = v.y;
            }
            d = feat_dist<SP, F, 0>(sv, qv, sp);
            hit = d <= r;
            id = ids[p];
        }
        // every lane has read its entry (the ballot depends on it) before any write below;
        // writes land at or below the positions read
        const uint64_t bm = __ballot(hit);
        if (hit) {
            const uint32_t o = hits + (uint32_t)__popcll(bm & lt);
            slab_i[base + o] = id;
            slab_d[base + o] = d;
        }
        hits += (uint32_t)__popcll(bm);
    }
    if (lane == 0) counts[q] = hits;
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
    int K2, K;   // K2: lanes / slots per query list (16 / 32 / 64); K: the certificate's k bucket
    int k2;      // entries the walk keeps (<= K2): k + 3 for the culled walks, K2 otherwise
    bool cull;
    uint32_t chunks, chunk_len;
};

FastPlan fast_plan(const DevSpace &sp, uint32_t nq, uint32_t k, uint64_t n_end, int num_cus, bool cull) {
    FastPlan p{};
    p.K2 = fast_k2(sp, k, nq, cull);
    p.K = k_bucket(k);
    p.k2 = p.K2;
    p.cull = cull;
    if (cull && sp.kind == OMPL_GPU_SPACE_KCHAIN) {
        // culled chain scan: full K2 lists per chunk (the chunked certificate's proof takes the
        // merged list's K2-th entry), chunks along grid.y for ~24 waves per CU
        p.K2 = k_bucket(k + 6) < 16 ? 16 : k_bucket(k + 6);
        p.k2 = p.K2;
        const uint64_t ntile = std::max<uint64_t>(1, (n_end + kCullTile - 1) / kCullTile);
        const uint64_t groups = (nq + kChainCullG - 1) / kChainCullG;
        // waves per CU the chunks aim at and the chunk cap.  With the thresholds shared across
        // chunks (MODE 2) more chunks only add parallelism: measured on cfg4 (8,192 milestones,
        // 1,024 groups) 24 / 48 / 96 / 192 / 384 waves per CU -> 8.14 / 6.79 / 5.59 / 4.88 / 4.67 ms
        // (384 reaches the 64-chunk cap; 128 / 256 chunks: the merge eats the gain)
        constexpr uint64_t wpc = 384, smax = 64;
        const uint64_t S = std::max<uint64_t>(1, std::min<uint64_t>(((uint64_t)num_cus * wpc + groups - 1) / groups, smax));
        const uint64_t per = (ntile + S - 1) / S;
        p.chunk_len = (uint32_t)per;  // tiles per chunk
        p.chunks = (uint32_t)((ntile + per - 1) / per);
        return p;
    }
    if (cull) {  // group walk: one list per query, k + 3 entries in the smallest slot bucket
        // k + 3: measured on cfg3 (SE3 10^6, k = 10, 10^5 queries), k + 2 left 250 of 10^5
        // queries uncertified (a 90 us bounded re-run), k + 3 none, for +0.01 ms of walk
        p.k2 = (int)k + 3;
        int lanes = k_bucket(k + 3);
        if (lanes < 16) lanes = 16;
        if (p.K2 > 0 && lanes <= p.K2) p.K2 = lanes;
        // the 64-lane lists (BIT*'s k = 57) keep all 64 entries: with k + 3, 66 of 10^5 queries
        // per cfg5k batch failed the proof (the 57th-60th distances within the screen error) and
        // their bounded re-run — a pass over the 10^7 fp64 rows — took 1.67 ms of a 7.9 ms step
        if (p.K2 == 64) p.k2 = 64;
        p.chunks = 1;
        p.chunk_len = 0;
        return p;
    }
    const uint64_t tiles = std::max<uint64_t>(n_end / kTile, 1);
    if (sp.kind == OMPL_GPU_SPACE_KCHAIN) {  // wave scan: ~8 waves per SIMD
        const uint64_t groups = (nq + 4 * kWaveGroup - 1) / (4 * kWaveGroup);  // blocks of 4 waves
        const uint64_t target = (uint64_t)num_cus * 8;
        const uint64_t S = std::max<uint64_t>(1, std::min<uint64_t>((target + groups - 1) / groups, tiles));
        const uint64_t per = (tiles + S - 1) / S;
        p.chunk_len = (uint32_t)(per * kTile);
        p.chunks = (uint32_t)((n_end + p.chunk_len - 1) / p.chunk_len);
        return p;
    }
    const uint64_t qblocks = (nq + kTile - 1) / kTile;
    const uint64_t target = (uint64_t)num_cus * 8;
    uint64_t S = std::max<uint64_t>(1, std::min<uint64_t>((target + qblocks - 1) / qblocks, tiles));
    const uint64_t per = (tiles + S - 1) / S;
    p.chunk_len = (uint32_t)(per * kTile);
    p.chunks = (uint32_t)((n_end + p.chunk_len - 1) / p.chunk_len);
    return p;
}


struct FastLayout {
    size_t keys, keys2, idx, perm, cub, q32u, q32, pd, pi, fail, tau, total;
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
    L.cub_bytes = home_sort_bytes(nq);  // the counting sort's per-query slots (+ its bins for wide keys)
    L.cub = take(L.cub_bytes);
    const int FS = sp.kind == OMPL_GPU_SPACE_SE3 ? 8 : g.F;
    L.q32u = take(4ull * nq * FS);
    L.q32 = take(4ull * nq * FS);
    L.pd = take(4ull * p.chunks * nq * p.K2);
    L.pi = take(4ull * p.chunks * nq * p.K2);
    L.fail = take(4ull * (nq + 1));
    L.tau = take(8ull * nq);  // the chain cull's shared threshold keys
    L.total = off;
    return L;
}

template <int SP, int F, int K2, int K>
hipError_t run_fast(const DevSpace &sp, const FastPlan &p, const FastLayout &L, char *ws, const float *f32,
                    const double *f64, uint64_t cap, uint64_t n_end, const SortedStore *ss, const double *qf64,
                    uint32_t nq, uint32_t k, const FastBounds &b, double *od, uint32_t *oi, hipStream_t st) {
    uint32_t *keys = (uint32_t *)(ws + L.keys), *keys2 = (uint32_t *)(ws + L.keys2);
    uint32_t *idx = (uint32_t *)(ws + L.idx), *perm = (uint32_t *)(ws + L.perm);
    float *q32u = (float *)(ws + L.q32u), *q32 = (float *)(ws + L.q32);
    float *pd = (float *)(ws + L.pd);
    uint32_t *pi = (uint32_t *)(ws + L.pi);
    uint32_t *fail = (uint32_t *)(ws + L.fail);
    const dim3 b256(256);
    // home-tile keys (a k-d tree): the fused counting sort over the store's bins; else Morton keys
    const bool home_keys = p.cull && ss && ss->nodes && ss->kd_tiles > 1;
    FastBounds bz = b;  // + the fail count, zeroed by query_rows_kernel
    bz.zero[2] = fail;
    bz.nzero[2] = 1u;
    hipError_t e = sort_queries<SP, F>(qf64, nq, bz, ss, home_keys, ws + L.cub, L.cub_bytes, q32u, keys, keys2, idx,
                                       perm, q32, st, (p.cull && ss) ? ss->nodes : nullptr,
                                       (p.cull && ss) ? ss->kd_tiles : 0u);
    if (e != hipSuccess) return e;
    bool walked = false;
    float chain_qerr = 0.f;  // the culled chain scan's 16-bit screen error (certificate)
    if constexpr (SP == OMPL_GPU_SPACE_SE3 || SP == OMPL_GPU_SPACE_REALVECTOR) {  // cull_supported
        if (p.cull) {
            timer_begin(st, "knn32_group_kernel");
            // (BIT*'s 64-lane lists too: cfg5k G = 2 4.08-4.14 ms, 4 4.24-4.35, 8 5.07-5.09)
            constexpr int G = group_queries<SP>();
            hipLaunchKernelGGL((knn32_group_kernel<SP, F, K2, G, true>), dim3((nq + G - 1) / G), dim3(64), 0, st,
                               ss->rows, ss->n_pad, ss->ids, ss->ntiles, ss->tbox, ss->sbox, ss->nsuper, ss->mbox, ss->nmega, ss->tkey0, q32,
                               keys2, nq, (float)sp.w0, (float)sp.w1, pd, pi, ss->counters, p.k2,
                               (float)((1.0 - (double)b.qeta) * (1.0 - 4e-7)));
            timer_end(st);
            walked = true;
        }
    }
    if constexpr (SP == OMPL_GPU_SPACE_KCHAIN) {
        if (p.cull) {
            if (!ss || !ss->built) return hipErrorInvalidValue;
            // the plan's chunk count sized the lists; the store's tiles (main + tail) set their length
            const uint32_t per = (ss->ntiles + p.chunks - 1) / p.chunks;
            // thresholds shared across the chunks: the pre-pass (MODE 1) publishes each query's
            // window bound, the chunk pass (MODE 2) tightens them by device-scope atomicMin
            unsigned long long *skey = (unsigned long long *)(ws + L.tau);
            const uint32_t ng = (nq + kChainCullG - 1) / kChainCullG;
            // the 16-bit rows when the store's copy is current (refresh_chain_rows16)
            const bool q16 = ss->rows16 && ss->gen16 == ss->gen;
            const float qerr = q16 ? (float)(chain_q16_error(sp) * (1.0 + 1e-5)) : 0.f;
#define OMPL_AMD_CHAIN_CULL(MODE, Q, GY, CNT)                                                                   \
    hipLaunchKernelGGL((knn32_chain_cull_kernel<F, K2, kChainCullG, MODE, Q>), dim3(ng, GY), dim3(64), 0, st,   \
                       ss->rows, ss->rows16, ss->n_pad, ss->ids, ss->ntiles, ss->tbox, q32, keys2, nq, per,     \
                       (float)sp.link, sp.dim, qerr, pd, pi, CNT, skey)
            hipError_t me = hipMemsetAsync(skey, 0xFF, 8ull * nq, st);  // above every key
            if (me != hipSuccess) return me;
            if (q16) {
                OMPL_AMD_CHAIN_CULL(1, true, 1, nullptr);
                timer_begin(st, "knn32_chain_cull_kernel");
                OMPL_AMD_CHAIN_CULL(2, true, p.chunks, ss->counters);
            } else {
                OMPL_AMD_CHAIN_CULL(1, false, 1, nullptr);
                timer_begin(st, "knn32_chain_cull_kernel");
                OMPL_AMD_CHAIN_CULL(2, false, p.chunks, ss->counters);
            }
#undef OMPL_AMD_CHAIN_CULL
            timer_end(st);
            chain_qerr = qerr;
            walked = true;
        }
    }
    if (p.cull && !walked) return hipErrorInvalidValue;
    if constexpr (SP == OMPL_GPU_SPACE_KCHAIN) if (!p.cull) {
        timer_begin(st, "knn32_wave_scan_kernel");
        // outer links first, four waves sharing each staged tile (measured against the reference
        // link order with two exit tests and one wave per block)
        const uint32_t qpb = (uint32_t)(kWaveGroup * 4);
        const dim3 grid((nq + qpb - 1) / qpb, p.chunks);
        hipLaunchKernelGGL((knn32_wave_scan_kernel<F, K2, kWaveGroup, 1, 4>), grid, dim3(256), 0, st, f32, cap, n_end,
                           q32, nq, p.chunk_len, (float)sp.link, sp.dim, pd, pi);
        timer_end(st);
        walked = true;
    }
    if (!walked) {
        timer_begin(st, "knn32_screen_kernel");
        const float w0 = SP == OMPL_GPU_SPACE_KCHAIN ? (float)sp.link : (float)sp.w0;
        hipLaunchKernelGGL((knn32_screen_kernel<SP, F, K2>), dim3((nq + kTile - 1) / kTile, p.chunks), dim3(kTile), 0,
                           st, f32, cap, n_end, q32, nq, p.chunk_len, w0, (float)sp.w1, sp.dim, pd, pi);
        timer_end(st);
    }
    if (SP == OMPL_GPU_SPACE_KCHAIN && p.cull) {
        // the culled chain scan: merge its chunk lists, then the wave certificate (ids, SoA rows)
        if (p.chunks > 1)
            hipLaunchKernelGGL((knn_chunk_merge_kernel<K2>), dim3((nq + 3) / 4), b256, 0, st, pd, pi, p.chunks, nq);
        constexpr uint32_t QPB = 256 / K2;
        if (!ss->rows64) return hipErrorInvalidValue;
        hipLaunchKernelGGL((knn_certify_wave_kernel<SP, F, K2>), dim3((nq + QPB - 1) / QPB), b256, 0, st, pd, pi, nq,
                           perm, f64, cap, ss->ids, ss->rows64, qf64, sp, b.absmax, b.qeta + chain_qerr, b.n_live,
                           (uint32_t)K2, od, oi, k, fail, fail + 1);
    } else if (p.chunks == 1) {
        constexpr uint32_t QPB = 256 / K2;
        // the group walk's lists hold positions in the sorted store (rows64 / ids map them)
        const bool pos = walked && p.cull;
        if (pos && !ss->rows64) return hipErrorInvalidValue;
        hipLaunchKernelGGL((knn_certify_wave_kernel<SP, F, K2>), dim3((nq + QPB - 1) / QPB), b256, 0, st, pd, pi, nq,
                           perm, f64, cap, pos ? ss->ids : nullptr, pos ? ss->rows64 : nullptr, qf64, sp, b.absmax,
                           b.qeta, b.n_live, (uint32_t)p.k2, od, oi, k, fail, fail + 1, 0.f);
    } else {
        if (p.cull) return hipErrorInvalidValue;  // position lists need the wave certificate
        if constexpr (K == 64 && SP != OMPL_GPU_SPACE_KCHAIN) {
            return hipErrorInvalidValue;  // culled walk only
        } else {
            hipLaunchKernelGGL((knn_certify_kernel<SP, F, K2, K>), dim3((nq + 255) / 256), b256, 0, st, pd, pi, p.chunks,
                               nq, perm, f64, cap, qf64, sp, b.absmax, b.qeta, b.n_live, od, oi, k, fail, fail + 1);
        }
    }
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
        break;
    case 64:
        // PRM* k = 41 on the chain (ConnectionStrategy.h:147); BIT* k = 57 on the culled walk
        if constexpr (K2 >= 64)
            if (SP == OMPL_GPU_SPACE_KCHAIN || p.cull)
                return run_fast<SP, F, K2, 64>(sp, p, L, ws, f32, f64, cap, n_end, ss, qf64, nq, k, b, od, oi, st);
        break;
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

// radius workspace: query order + fp32 rows (as the kNN walk), per-query counts (nq + 1,
// the last one zero) and the offsets their exclusive scan gives (nq + 2: [nq] = total,
// [nq + 1] = longest segment)
constexpr int kRadiusGroup = 4;  // 10^7-state radius pass: G=2 2.37 ms, G=4 2.27 ms (tiles shared by more queries)
// the one-walk (slab) pass holds no fp64 state, so a group could be wider (each fetched tile
// serving more queries): 8 measured no faster
constexpr int kRadiusSlabGroup = 4;

struct RadiusLayout {
    size_t keys, keys2, idx, perm, cub, q32u, q32, counts, off, scan, total;
    size_t cub_bytes;
};

RadiusLayout radius_layout(const DevSpace &sp, const FeatGeom &g, uint32_t nq) {
    RadiusLayout L{};
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
    L.cub_bytes = home_sort_bytes(nq);  // the counting sort's per-query slots (+ its bins for wide keys)
    L.cub = take(L.cub_bytes);
    const int FS = sp.kind == OMPL_GPU_SPACE_SE3 ? 8 : g.F;
    L.q32u = take(4ull * nq * FS);
    L.q32 = take(4ull * nq * FS);
    L.counts = take(8ull * (nq + 1));
    L.off = take(8ull * (nq + 2));
    L.scan = take(exclusive_scan_u64_workspace((uint64_t)nq + 1));
    L.total = off;
    return L;
}

template <int SP, int F>
hipError_t run_radius_fast(const DevSpace &sp, const RadiusLayout &L, char *ws, const double *f64, uint64_t cap,
                           const SortedStore *ss, const double *qf64, uint32_t nq, double r, const FastBounds &b,
                           int phase, uint32_t *out_i, double *out_d, hipStream_t st) {
    uint32_t *keys = (uint32_t *)(ws + L.keys), *keys2 = (uint32_t *)(ws + L.keys2);
    uint32_t *idx = (uint32_t *)(ws + L.idx), *perm = (uint32_t *)(ws + L.perm);
    float *q32u = (float *)(ws + L.q32u), *q32 = (float *)(ws + L.q32);
    uint64_t *counts = (uint64_t *)(ws + L.counts), *offs = (uint64_t *)(ws + L.off);
    const dim3 grid((nq + kRadiusGroup - 1) / kRadiusGroup), b64(64);
    if (!ss->rows64) return hipErrorInvalidValue;
    (void)f64;
    (void)cap;
    hipError_t e;
    if (phase == 2 && (b.slab == 0 || !out_i || !out_d)) return hipErrorInvalidValue;
    if (phase == 0 || phase == 2) {
        const bool home_keys = ss->nodes && ss->kd_tiles > 1;
        FastBounds bz = b;  // + the walk's candidate total, zeroed by query_rows_kernel
        bz.zero[2] = (uint32_t *)(counts + nq);
        bz.nzero[2] = 2u;
        if ((e = sort_queries<SP, F>(qf64, nq, bz, ss, home_keys, ws + L.cub, L.cub_bytes, q32u, keys, keys2, idx, perm,
                                     q32, st, ss->nodes, ss->kd_tiles)) != hipSuccess)
            return e;
        if (phase == 2) {
            timer_begin(st, "radius32_group_kernel");
            const dim3 gs((nq + kRadiusSlabGroup - 1) / kRadiusSlabGroup);
            bool q16 = false;
            if constexpr (SP == OMPL_GPU_SPACE_SE3) {
                if (ss->rows16 && ss->gen16 == ss->gen) {
                    q16 = true;
                    hipLaunchKernelGGL((radius32_group_kernel<SP, F, kRadiusSlabGroup, 2, true>), gs, b64, 0, st,
                                       ss->rows, ss->n_pad, ss->ids, ss->ntiles, ss->tbox, ss->sbox, ss->nsuper, ss->mbox, ss->nmega, q32,
                                       perm, nq, ss->rows64, qf64, sp, b.absmax, b.qeta, r, counts, nullptr, out_i,
                                       out_d, ss->counters, b.slab, ss->rows16, ss->q16, se3_q16_error(sp, ss->q16));
                }
            }
            if (!q16)
                hipLaunchKernelGGL((radius32_group_kernel<SP, F, kRadiusSlabGroup, 2>), gs, b64, 0, st, ss->rows,
                                   ss->n_pad, ss->ids, ss->ntiles, ss->tbox, ss->sbox, ss->nsuper, ss->mbox, ss->nmega, q32, perm, nq,
                                   ss->rows64, qf64, sp, b.absmax, b.qeta, r, counts, nullptr, out_i, out_d,
                                   ss->counters, b.slab);
            timer_end(st);
            hipLaunchKernelGGL((radius_slab_exact_kernel<SP, F>), dim3(nq), b64, 0, st, ss->rows64, ss->ids, qf64, sp,
                               r, b.slab, counts, out_i, out_d);
        } else {
            hipLaunchKernelGGL((radius32_group_kernel<SP, F, kRadiusGroup, 0>), grid, b64, 0, st, ss->rows, ss->n_pad,
                               ss->ids, ss->ntiles, ss->tbox, ss->sbox, ss->nsuper, ss->mbox, ss->nmega, q32, perm, nq, ss->rows64, qf64,
                               sp, b.absmax, b.qeta, r, counts, nullptr, nullptr, nullptr, nullptr, 0u);
        }
        // offsets (offs[nq] = the total) and the longest segment (offs[nq + 1])
        return launch_exclusive_scan_u64(counts, (uint64_t)nq, offs, ws + L.scan, st, offs + nq + 1);
    }
    timer_begin(st, "radius32_group_kernel");
    hipLaunchKernelGGL((radius32_group_kernel<SP, F, kRadiusGroup, 1>), grid, b64, 0, st, ss->rows, ss->n_pad,
                       ss->ids, ss->ntiles, ss->tbox, ss->sbox, ss->nsuper, ss->mbox, ss->nmega, q32, perm, nq, ss->rows64, qf64, sp,
                       b.absmax, b.qeta, r, nullptr, offs, out_i, out_d, ss->counters, 0u);
    timer_end(st);
    return hipGetLastError();
}

// ---- device k-d build of the sorted store (no host round trip) -------------------------------
// The tree shape depends only on the number of live states: a node of T tiles splits into
// floor(T/2) (left) and T - floor(T/2) tiles, down to one-tile leaves (the left part holds
// exactly floor(T/2) full tiles, so only the last leaf is partial).  A node is identified at
// level L by the L bits of its path; its tile range follows from the path, its pre-order index
// too (left child = index + 1, right child = index + floor(T/2)).  Per level, every node picks
// the widest coordinate of its box and its states are sorted by (node, coordinate) — one radix
// sort of (path << 16 | coordinate quantised over the node's extent) keys, L + 16 bits, for all
// nodes of the level — which puts the floor(T/2) * 64 smallest on the left: the host median
// split (std::nth_element) of round 1, as one sort per level on the device.
struct KdNodeRef {
    uint32_t t0, T, pidx;
    bool valid;
};

__device__ __forceinline__ KdNodeRef kd_node_at(uint32_t ntiles, int level, uint32_t path) {
    KdNodeRef r{0u, ntiles, 0u, true};
    for (int b = level - 1; b >= 0; --b) {
        if (r.T <= 1) {
            r.valid = false;
            return r;
        }
        const uint32_t tl = r.T >> 1;
        if ((path >> b) & 1u) {
            r.pidx += tl;
            r.t0 += tl;
            r.T -= tl;
        } else {
            r.pidx += 1;
            r.T = tl;
        }
    }
    return r;
}

__global__ void kd_live_flags_kernel(const uint8_t *__restrict__ live, uint64_t n, uint8_t *__restrict__ flags) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) flags[i] = live[i];
}

// rows / ids of positions [p0, p1): ids from src (index p - p0) for p - p0 < cnt, else padding
template <int SP, int F>
__global__ void sorted_gather_kernel(const float *__restrict__ f32, uint64_t cap, const uint32_t *__restrict__ src,
                                     uint32_t cnt, uint32_t p0, uint32_t p1, uint32_t n_pad, float *__restrict__ rows,
                                     uint32_t *__restrict__ ids, uint32_t *__restrict__ inv) {
    constexpr int R = Geo<SP, F>::R;
    const uint32_t p = p0 + blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= p1) return;
    if (p - p0 < cnt) {
        const uint32_t id = src[p - p0];
        float x[R];
#pragma unroll
        for (int r = 0; r < R; ++r) x[r] = f32[(uint64_t)r * cap + id];
        if constexpr (SP == OMPL_GPU_SPACE_SE3) {  // |dot| is sign-invariant: store w >= 0
            if (x[6] < 0.f)
#pragma unroll
                for (int r = 3; r < 7; ++r) x[r] = -x[r];
        }
#pragma unroll
        for (int r = 0; r < R; ++r) rows[blk_index(p, r, R)] = x[r];
        ids[p] = id;
        inv[id] = p;
    } else {
#pragma unroll
        for (int r = 0; r < R; ++r) rows[blk_index(p, r, R)] = __builtin_nanf("");
        ids[p] = kNoId;
    }
}

template <int SP, int F>
__global__ void tail_keys_kernel(const float *__restrict__ f32, uint64_t cap, uint64_t first, uint32_t n, FastBounds b,
                                 const KdNode *__restrict__ nodes, uint32_t kd_tiles, uint32_t *__restrict__ keys,
                                 uint32_t *__restrict__ idx) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t id = (uint32_t)(first + i);
    constexpr int R = Geo<SP, F>::R;
    float x[R > kKeyDims + 1 ? R : kKeyDims + 1];
#pragma unroll
    for (int r = 0; r < R; ++r) x[r] = f32[(uint64_t)r * cap + id];
    if constexpr (SP == OMPL_GPU_SPACE_KCHAIN) {
        // the chain's 2 NM position coordinates have no Morton order worth the name: order the
        // tail by the k-d home tile of the main part, so that tail tiles are compact too
        keys[i] = (nodes && kd_tiles > 1) ? kd_home_tile(x, nodes, kd_tiles) : 0u;
    } else {
        float c[kKeyDims];
        key_coords<SP>(x, c, b.nkey);
        keys[i] = morton_key(c, b);
    }
    idx[i] = id;
}

__global__ void iota_kernel(uint32_t *__restrict__ a, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) a[i] = i;
}

__global__ void rows64_range_kernel(const double *__restrict__ f64, uint64_t cap, int F, int FA,
                                    const uint32_t *__restrict__ ids, uint32_t p0, uint32_t p1,
                                    double *__restrict__ rows64) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;  // (slot, column)
    const uint64_t p = p0 + t / FA;
    if (p >= p1) return;
    const int f = (int)(t % FA);
    const uint32_t id = ids[p];
    rows64[p * FA + f] = f >= F ? 0.0 : (id == kNoId ? __builtin_nan("") : f64[(uint64_t)f * cap + id]);
}

template <int SP, int F>
__global__ void tile_box_range_kernel(const float *__restrict__ rows, uint32_t n_pad, uint32_t t0, uint32_t t1,
                                      float *__restrict__ tbox) {
    constexpr int NB = Geo<SP, F>::NB, BW = Geo<SP, F>::BW;
    const uint32_t t = t0 + blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (t >= t1) return;
    float xr[Geo<SP, F>::R];
    load_blk<Geo<SP, F>::R>(rows, t, lane, xr);
    (void)n_pad;
    float x[NB];
#pragma unroll
    for (int c = 0; c < NB; ++c) x[c] = xr[c];
    const bool ok = x[0] == x[0];  // padding / removed
    float eta = 0.f;
    if constexpr (SP == OMPL_GPU_SPACE_SE3) {
        if (ok) {
            float n2 = x[3] * x[3];
            n2 = fmaf(x[4], x[4], n2);
            n2 = fmaf(x[5], x[5], n2);
            n2 = fmaf(x[6], x[6], n2);
            eta = fmaxf(n2 - 1.f, 0.f);
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) eta = fmaxf(eta, __shfl_xor(eta, o));
    }
    float *o = tbox + (size_t)t * BW;
#pragma unroll
    for (int c = 0; c < NB; ++c) {
        float lo = ok ? x[c] : __builtin_inff(), hi = ok ? x[c] : -__builtin_inff();
#pragma unroll
        for (int s = 32; s > 0; s >>= 1) {
            lo = fminf(lo, __shfl_xor(lo, s));
            hi = fmaxf(hi, __shfl_xor(hi, s));
        }
        if (lane == 0) {
            o[c] = lo;
            o[NB + c] = hi;
        }
    }
    if constexpr (SP == OMPL_GPU_SPACE_SE3) {
        if (lane == 0) {
            o[2 * NB] = eta * 1.00001f;
            o[2 * NB + 1] = 0.f;
        }
    }
}

// boxes of groups of `group` (<= 64) consecutive input boxes (tile boxes -> super-tiles, super-tile
// boxes -> mega-tiles): output box sI covers inputs [sI * group, min((sI + 1) * group, n_in)).  A
// wave per output box, a lane per input box, wave reductions per coordinate (a thread per output
// box looping over 64 inputs x 48 coordinates took 0.11 ms for the KinematicChain tail).
template <int SP, int F>
__global__ __launch_bounds__(256) void super_box_range_kernel(const float *__restrict__ tbox, uint32_t n_in,
                                                              uint32_t group, uint32_t s0, uint32_t s1,
                                                              float *__restrict__ sbox) {
    constexpr int NB = Geo<SP, F>::NB, BW = Geo<SP, F>::BW;
    const uint32_t sI = s0 + blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (sI >= s1) return;
    const uint32_t t = sI * group + (uint32_t)lane;
    const bool in = (uint32_t)lane < group && t < n_in;
    const float *b = tbox + (size_t)(in ? t : 0) * BW;
    float *o = sbox + (size_t)sI * BW;
    for (int c = 0; c < NB; ++c) {
        float lo = in ? b[c] : __builtin_inff(), hi = in ? b[NB + c] : -__builtin_inff();
#pragma unroll
        for (int m = 32; m > 0; m >>= 1) {
            lo = fminf(lo, __shfl_xor(lo, m));
            hi = fmaxf(hi, __shfl_xor(hi, m));
        }
        if (lane == 0) {
            o[c] = lo;
            o[NB + c] = hi;
        }
    }
    if constexpr (SP == OMPL_GPU_SPACE_SE3) {
        float eta = in ? b[2 * NB] : 0.f;
#pragma unroll
        for (int m = 32; m > 0; m >>= 1) eta = fmaxf(eta, __shfl_xor(eta, m));
        if (lane == 0) {
            o[2 * NB] = eta;
            o[2 * NB + 1] = 0.f;
        }
    }
}

// ---- build over physically permuted rows ---------------------------------------------------
// The level loop keeps the states' box coordinates in a working array of AoS rows in the current
// order (KdRow: the NB box coordinates — SE3 quaternion sign-canonical — and the id's bits,
// padded to a multiple of 4 floats: 32 B per SE3 state), so every per-level pass (tile boxes,
// sort keys) reads contiguous rows, and one gather of whole rows per level follows the sort.
// (Round 2 gathered each of the 8 coordinates by id in two passes per level: 8 cache lines per
// state, 1.5 ms per level at 10^7 states.)
constexpr int kKdQBits = 12;                       // split-coordinate quantisation of the build's sort keys
constexpr uint32_t kKdQ = (1u << kKdQBits) - 1u;

template <int SP, int F>
struct KdRow {
    static constexpr int NB = Geo<SP, F>::NB;
    static constexpr int W = (NB + 1 + 3) & ~3;  // floats per row (last used slot: the id)
};

template <int SP, int F>
__global__ void kd_rows_init_kernel(const float *__restrict__ f32, uint64_t cap, const uint32_t *__restrict__ sel,
                                    uint32_t n, float *__restrict__ W) {
    constexpr int NB = KdRow<SP, F>::NB, RW = KdRow<SP, F>::W;
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const uint32_t id = sel[p];
    float r[RW];
#pragma unroll
    for (int d = 0; d < RW; ++d) r[d] = 0.f;
#pragma unroll
    for (int d = 0; d < NB; ++d) r[d] = f32[(uint64_t)d * cap + id];
    if constexpr (SP == OMPL_GPU_SPACE_SE3) {
        if (r[6] < 0.f)
#pragma unroll
            for (int d = 3; d < 7; ++d) r[d] = -r[d];
    }
    r[NB] = __uint_as_float(id);
    float4 *o = reinterpret_cast<float4 *>(W + (size_t)p * RW);
#pragma unroll
    for (int c = 0; c < RW / 4; ++c) o[c] = make_float4(r[4 * c], r[4 * c + 1], r[4 * c + 2], r[4 * c + 3]);
}

// boxes of the 64-row tiles of the current order (a wave per tile, contiguous rows)
template <int SP, int F>
__global__ void kd_row_tile_boxes_kernel(const float *__restrict__ W, uint32_t n, uint32_t ntiles,
                                         float *__restrict__ tb) {
    constexpr int NB = KdRow<SP, F>::NB, RW = KdRow<SP, F>::W;
    const uint32_t t = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (t >= ntiles) return;
    const uint32_t p = t * kCullTile + lane;
    float r[RW];
    if (p < n) {
        const float4 *w4 = reinterpret_cast<const float4 *>(W + (size_t)p * RW);
#pragma unroll
        for (int c = 0; c < RW / 4; ++c) {
            const float4 v = w4[c];
            r[4 * c] = v.x; r[4 * c + 1] = v.y; r[4 * c + 2] = v.z; r[4 * c + 3] = v.w;
        }
    }
#pragma unroll
    for (int d = 0; d < NB; ++d) {
        float lo = p < n ? r[d] : __builtin_inff();
        float hi = p < n ? r[d] : -__builtin_inff();
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            lo = fminf(lo, __shfl_xor(lo, o));
            hi = fmaxf(hi, __shfl_xor(hi, o));
        }
        if (lane == 0) {
            tb[(size_t)t * 2 * NB + d] = lo;
            tb[(size_t)t * 2 * NB + NB + d] = hi;
        }
    }
}

// one block per node of the level: widest box coordinate -> nsplit[path] = {dim, lo, kKdQ / extent}
template <int SP, int F, int BS>
__global__ __launch_bounds__(BS) void kd_node_split_dim_kernel(const float *__restrict__ tb, uint32_t ntiles,
                                                                int level, float4 *__restrict__ nsplit) {
    constexpr int NB = Geo<SP, F>::NB;
    __shared__ float slo[NB][BS], shi[NB][BS];
    const KdNodeRef nd = kd_node_at(ntiles, level, blockIdx.x);
    if (!nd.valid || nd.T <= 1) return;
    float lo[NB], hi[NB];
#pragma unroll
    for (int d = 0; d < NB; ++d) {
        lo[d] = __builtin_inff();
        hi[d] = -__builtin_inff();
    }
    for (uint32_t t = nd.t0 + threadIdx.x; t < nd.t0 + nd.T; t += blockDim.x)
#pragma unroll
        for (int d = 0; d < NB; ++d) {
            lo[d] = fminf(lo[d], tb[(size_t)t * 2 * NB + d]);
            hi[d] = fmaxf(hi[d], tb[(size_t)t * 2 * NB + NB + d]);
        }
    if (nd.T <= 64) {  // small node: one wave reduces (the other waves hold empty boxes)
        if (threadIdx.x >= 64) return;
#pragma unroll
        for (int d = 0; d < NB; ++d)
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                lo[d] = fminf(lo[d], __shfl_xor(lo[d], o));
                hi[d] = fmaxf(hi[d], __shfl_xor(hi[d], o));
            }
    } else {
#pragma unroll
        for (int d = 0; d < NB; ++d) {
            slo[d][threadIdx.x] = lo[d];
            shi[d][threadIdx.x] = hi[d];
        }
        __syncthreads();
        for (int w = BS / 2; w > 0; w >>= 1) {
            if ((int)threadIdx.x < w)
#pragma unroll
                for (int d = 0; d < NB; ++d) {
                    slo[d][threadIdx.x] = fminf(slo[d][threadIdx.x], slo[d][threadIdx.x + w]);
                    shi[d][threadIdx.x] = fmaxf(shi[d][threadIdx.x], shi[d][threadIdx.x + w]);
                }
            __syncthreads();
        }
#pragma unroll
        for (int d = 0; d < NB; ++d) {
            lo[d] = slo[d][0];
            hi[d] = shi[d][0];
        }
    }
    if (threadIdx.x == 0) {
        int bd = 0;
        float be = -1.f;
#pragma unroll
        for (int d = 0; d < NB; ++d) {
            const float e = hi[d] - lo[d];
            if (e > be) {  // first widest, as the host build
                be = e;
                bd = d;
            }
        }
        const float inv = be > 0.f ? (float)kKdQ / be : 0.f;
        nsplit[blockIdx.x] = make_float4(__uint_as_float((uint32_t)bd), lo[bd], inv, 0.f);
    }
}

// a split coordinate quantised to kKdQBits bits over the node's extent.  Quantisation only
// decides how states with nearly equal coordinates straddle the split: the left part still gets
// exactly floor(T/2) tiles, and every tile / super-tile box is computed from the states it holds,
// so the walks' bounds do not depend on it.
__device__ __forceinline__ uint32_t kd_quant(float v, float4 ns) {
    const float x = (v - ns.y) * ns.z;
    return x > 0.f ? (x < (float)kKdQ ? (uint32_t)x : kKdQ) : 0u;
}

// ---- global levels as a median partition (no sort) -----------------------------------------
// A level only has to put the floor(T/2) * 64 states with the smallest quantised split coordinate
// of every node on its left; their order inside each child is free.  So instead of a radix sort of
// (path, q) keys (2-3 digit passes over keys and values, then a row gather) a level is: a
// histogram of q per node (kd_part_hist_kernel, which keeps q), the median bin b* and how many of
// its states go left (kd_part_select_kernel, which also writes the node record), per-chunk counts
// of q < b* / q == b* (kd_part_count_kernel), and one stable scatter of the rows
// (kd_part_scatter_kernel: q < b* left, q > b* right, the first `need` states of bin b* in the
// current order left) that also reduces both children's boxes, from which the next level's split
// coordinates follow (kd_part_split_dim_kernel) without a tile-box pass.  Deterministic (the
// histogram's atomics only count); every tile / super-tile box is still computed from the states
// it ends up holding.
constexpr uint32_t kPartChunk = 4096;  // states per block of the per-level passes (64 tiles)
constexpr uint32_t kPartBins = kKdQ + 1;

struct KdPartRange {
    uint32_t P0, c0, c1, L;
    bool ok;
};
__device__ __forceinline__ KdPartRange kd_part_range(const KdNodeRef &nd, uint32_t n, uint32_t chunk) {
    KdPartRange r{nd.t0 * kCullTile, 0u, 0u, (nd.T >> 1) * kCullTile, false};
    const uint32_t pend = min((nd.t0 + nd.T) * kCullTile, n);
    r.c0 = r.P0 + chunk * kPartChunk;
    r.c1 = min(r.c0 + kPartChunk, pend);
    r.ok = nd.valid && nd.T > 1 && r.c0 < pend;
    return r;
}

template <int SP, int F>
__global__ __launch_bounds__(256) void kd_part_hist_kernel(const float *__restrict__ W, uint32_t n, uint32_t ntiles,
                                                           int level, const float4 *__restrict__ nsplit,
                                                           uint16_t *__restrict__ Q, uint32_t *__restrict__ H) {
    constexpr int RW = KdRow<SP, F>::W;
    __shared__ uint32_t h[kPartBins];
    const uint32_t node = blockIdx.y;
    const KdPartRange r = kd_part_range(kd_node_at(ntiles, level, node), n, blockIdx.x);
    if (!r.ok) return;
    for (uint32_t b = threadIdx.x; b < kPartBins; b += 256) h[b] = 0;
    __syncthreads();
    const float4 ns = nsplit[node];
    const int d = (int)__float_as_uint(ns.x);
    for (uint32_t p = r.c0 + threadIdx.x; p < r.c1; p += 256) {
        const uint32_t q = kd_quant(W[(size_t)p * RW + d], ns);
        Q[p] = (uint16_t)q;
        atomicAdd(&h[q], 1u);
    }
    __syncthreads();
    uint32_t *hn = H + (size_t)node * kPartBins;
    for (uint32_t b = threadIdx.x; b < kPartBins; b += 256)
        if (h[b]) atomicAdd(&hn[b], h[b]);
}

// block-wide exclusive scan of one flag per thread (256 threads); returns the prefix, `total` the sum
__device__ __forceinline__ uint32_t block_flag_scan(bool f, uint32_t *wsum, uint32_t &total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t m = __ballot(f);
    const uint32_t pre = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) wsum[wave] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t before = 0;
    total = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const uint32_t v = wsum[w];
        before += w < wave ? v : 0u;
        total += v;
    }
    __syncthreads();
    return pre + before;
}

// one block per node: the median bin b* (the first whose cumulative count reaches L) and the
// number of its states that go left; the node record (split: the lower edge of bin b*, which
// routes the home-tile descent of a query — only a heuristic, never a bound)
template <int SP, int F>
__global__ __launch_bounds__(256) void kd_part_select_kernel(const uint32_t *__restrict__ H, uint32_t n,
                                                             uint32_t ntiles, int level,
                                                             const float4 *__restrict__ nsplit,
                                                             uint2 *__restrict__ sel, KdNode *__restrict__ nodes) {
    constexpr uint32_t PER = (kPartBins + 255) / 256;
    __shared__ uint32_t part[256];
    const uint32_t node = blockIdx.x;
    const KdNodeRef nd = kd_node_at(ntiles, level, node);
    const KdPartRange r = kd_part_range(nd, n, 0);
    if (!r.ok) return;
    const uint32_t *hn = H + (size_t)node * kPartBins;
    const uint32_t b0 = threadIdx.x * PER;
    uint32_t sum = 0;
    for (uint32_t i = 0; i < PER; ++i)
        if (b0 + i < kPartBins) sum += hn[b0 + i];
    part[threadIdx.x] = sum;
    __syncthreads();
    for (uint32_t o = 1; o < 256; o <<= 1) {  // inclusive Hillis-Steele scan
        const uint32_t v = threadIdx.x >= o ? part[threadIdx.x - o] : 0u;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    const uint32_t incl = part[threadIdx.x], excl = incl - sum;
    if (excl < r.L && r.L <= incl) {  // exactly one thread: L >= 1 and the total covers L
        uint32_t c = excl, b = b0;
        for (uint32_t i = 0; i < PER && b0 + i < kPartBins; ++i) {
            const uint32_t v = hn[b0 + i];
            if (c + v >= r.L) {
                b = b0 + i;
                break;
            }
            c += v;
        }
        sel[node] = make_uint2(b, r.L - c);
        const float4 ns = nsplit[node];
        const uint32_t tl = nd.T >> 1;
        const float split = ns.z > 0.f ? ns.y + (float)b / ns.z : ns.y;
        nodes[nd.pidx] = KdNode{__float_as_uint(ns.x), split, tl, nd.pidx + tl};
    }
}

// per (node, chunk): states with q < b* and with q == b*
__global__ __launch_bounds__(256) void kd_part_count_kernel(const uint16_t *__restrict__ Q, uint32_t n,
                                                            uint32_t ntiles, int level,
                                                            const uint2 *__restrict__ sel, uint32_t cpn,
                                                            uint2 *__restrict__ cnt) {
    __shared__ uint32_t wsum[4];
    const uint32_t node = blockIdx.y;
    const KdPartRange r = kd_part_range(kd_node_at(ntiles, level, node), n, blockIdx.x);
    if (!r.ok) return;
    const uint32_t b = sel[node].x;
    uint32_t lt = 0, eq = 0;
    for (uint32_t p = r.c0 + threadIdx.x; p < r.c1; p += 256) {
        const uint32_t q = Q[p];
        lt += q < b ? 1u : 0u;
        eq += q == b ? 1u : 0u;
    }
    for (int o = 32; o > 0; o >>= 1) {
        lt += (uint32_t)__shfl_xor((int)lt, o);
        eq += (uint32_t)__shfl_xor((int)eq, o);
    }
    __shared__ uint32_t esum[4];
    if ((threadIdx.x & 63) == 0) {
        wsum[threadIdx.x >> 6] = lt;
        esum[threadIdx.x >> 6] = eq;
    }
    __syncthreads();
    if (threadIdx.x == 0)
        cnt[(size_t)node * cpn + blockIdx.x] =
            make_uint2(wsum[0] + wsum[1] + wsum[2] + wsum[3], esum[0] + esum[1] + esum[2] + esum[3]);
}

// ordered-integer image of a float (min of images = image of the min), for the box atomics
__device__ __forceinline__ uint32_t kd_fenc(float f) {
    const uint32_t b = __float_as_uint(f);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float kd_fdec(uint32_t e) {
    return __uint_as_float((e & 0x80000000u) ? (e & 0x7FFFFFFFu) : ~e);
}

// the stable scatter of one chunk; cbox[child path][2 NB]: images of min v and of min -v
// (both minima, so one 0xFF fill initialises them)
template <int SP, int F>
__global__ __launch_bounds__(256) void kd_part_scatter_kernel(const float *__restrict__ W, float *__restrict__ W2,
                                                              uint32_t n, uint32_t ntiles, int level,
                                                              const uint16_t *__restrict__ Q,
                                                              const uint2 *__restrict__ sel,
                                                              const uint2 *__restrict__ cnt, uint32_t cpn,
                                                              uint32_t *__restrict__ cbox) {
    constexpr int NB = KdRow<SP, F>::NB, RW = KdRow<SP, F>::W;
    __shared__ uint32_t wsum[4], red[2][2 * NB];
    const uint32_t node = blockIdx.y;
    const KdPartRange r = kd_part_range(kd_node_at(ntiles, level, node), n, blockIdx.x);
    if (!r.ok) return;
    const uint2 sv = sel[node];
    const uint32_t b = sv.x, need = sv.y;
    // states of this node before the chunk: q < b* and q == b* (the chunks' counts)
    uint32_t lt = 0, eq = 0;
    for (uint32_t c = threadIdx.x; c < blockIdx.x; c += 256) {
        const uint2 v = cnt[(size_t)node * cpn + c];
        lt += v.x;
        eq += v.y;
    }
    for (int o = 32; o > 0; o >>= 1) {
        lt += (uint32_t)__shfl_xor((int)lt, o);
        eq += (uint32_t)__shfl_xor((int)eq, o);
    }
    for (uint32_t i = threadIdx.x; i < 2 * 2 * NB; i += 256) (&red[0][0])[i] = 0xFFFFFFFFu;
    __shared__ uint32_t lts[4], eqs[4];
    if ((threadIdx.x & 63) == 0) {
        lts[threadIdx.x >> 6] = lt;
        eqs[threadIdx.x >> 6] = eq;
    }
    __syncthreads();
    uint32_t eq_before = eqs[0] + eqs[1] + eqs[2] + eqs[3];
    uint32_t left_before = lts[0] + lts[1] + lts[2] + lts[3] + min(eq_before, need);
    uint32_t right_before = (r.c0 - r.P0) - left_before;
    float lo[2][NB], nhi[2][NB];  // per side: min v, min -v
#pragma unroll
    for (int sd = 0; sd < 2; ++sd)
#pragma unroll
        for (int d = 0; d < NB; ++d) lo[sd][d] = nhi[sd][d] = __builtin_inff();
    for (uint32_t base = r.c0; base < r.c1; base += 256) {
        const uint32_t p = base + threadIdx.x;
        const bool in = p < r.c1;
        const uint32_t q = in ? (uint32_t)Q[p] : 0xFFFFFFFFu;
        uint32_t te, tl;
        const uint32_t er = block_flag_scan(in && q == b, wsum, te);
        const bool take = in && (q < b || (q == b && eq_before + er < need));
        const uint32_t lr = block_flag_scan(take, wsum, tl);
        if (in) {
            const uint32_t dst = take ? r.P0 + left_before + lr : r.P0 + r.L + right_before + (threadIdx.x - lr);
            const float4 *src4 = reinterpret_cast<const float4 *>(W + (size_t)p * RW);
            float4 *dst4 = reinterpret_cast<float4 *>(W2 + (size_t)dst * RW);
            float row[RW];
#pragma unroll
            for (int c = 0; c < RW / 4; ++c) {
                const float4 v = src4[c];
                dst4[c] = v;
                row[4 * c] = v.x; row[4 * c + 1] = v.y; row[4 * c + 2] = v.z; row[4 * c + 3] = v.w;
            }
            const int sd = take ? 0 : 1;
#pragma unroll
            for (int d = 0; d < NB; ++d) {
                if (sd == 0) {
                    lo[0][d] = fminf(lo[0][d], row[d]);
                    nhi[0][d] = fminf(nhi[0][d], -row[d]);
                } else {
                    lo[1][d] = fminf(lo[1][d], row[d]);
                    nhi[1][d] = fminf(nhi[1][d], -row[d]);
                }
            }
        }
        const uint32_t cnt_step = min(256u, r.c1 - base);
        eq_before += te;
        left_before += tl;
        right_before += cnt_step - tl;
    }
    // children's boxes: wave minima, then LDS atomics, then one global atomic per value
#pragma unroll
    for (int sd = 0; sd < 2; ++sd)
#pragma unroll
        for (int d = 0; d < NB; ++d) {
            float a = lo[sd][d], c = nhi[sd][d];
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                a = fminf(a, __shfl_xor(a, o));
                c = fminf(c, __shfl_xor(c, o));
            }
            if ((threadIdx.x & 63) == 0) {
                if (a < __builtin_inff()) atomicMin(&red[sd][d], kd_fenc(a));
                if (c < __builtin_inff()) atomicMin(&red[sd][NB + d], kd_fenc(c));
            }
        }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < 2 * 2 * NB; i += 256) {
        const uint32_t sd = i / (2 * NB), j = i % (2 * NB);
        const uint32_t v = red[sd][j];
        if (v != 0xFFFFFFFFu) atomicMin(&cbox[(size_t)(2 * node + sd) * 2 * NB + j], v);
    }
}

// split coordinates of the nodes of `level` (>= 1) from the boxes the previous scatter reduced
template <int SP, int F>
__global__ void kd_part_split_dim_kernel(const uint32_t *__restrict__ cbox, uint32_t ntiles, int level,
                                         float4 *__restrict__ nsplit) {
    constexpr int NB = KdRow<SP, F>::NB;
    const uint32_t path = blockIdx.x * blockDim.x + threadIdx.x;
    if (path >= (1u << level)) return;
    const KdNodeRef nd = kd_node_at(ntiles, level, path);
    if (!nd.valid || nd.T <= 1) return;
    const uint32_t *cb = cbox + (size_t)path * 2 * NB;
    int bd = 0;
    float be = -1.f, blo = 0.f;
    for (int d = 0; d < NB; ++d) {
        const float lo = kd_fdec(cb[d]), hi = -kd_fdec(cb[NB + d]);
        const float e = hi - lo;
        if (e > be) {  // first widest, as kd_node_split_dim_kernel
            be = e;
            bd = d;
            blo = lo;
        }
    }
    nsplit[path] = make_float4(__uint_as_float((uint32_t)bd), blo, be > 0.f ? (float)kKdQ / be : 0.f, 0.f);
}

// The deep levels in LDS: one block per node of level L0 (at most kd_lds_tiles<SP, F>() tiles,
// so its rows fit in LDS) splits its whole subtree there — per sub-level the same steps as the
// global loop (tile boxes of the current order, the widest coordinate of every splitting
// sub-node, (sub-path, quantised coordinate) keys), the sort being rocPRIM's block radix sort of
// packed (key << 11 | row index) words in LDS instead of a device-wide one; then it writes the
// node records and its rows in leaf order.  Padding slots (past the last state) get the largest
// key and stay last.
template <int SP, int F>
constexpr uint32_t kd_lds_tiles() {
    constexpr int RW = KdRow<SP, F>::W;
    return RW <= 8 ? 32u : (RW <= 12 ? 16u : 8u);  // <= 64 KiB of rows
}
template <int SP, int F>
constexpr uint32_t kd_lds_block() {
    constexpr uint32_t rows = kd_lds_tiles<SP, F>() * kCullTile;
    return (rows < 1024u) ? rows : 1024u;
}
constexpr int kKdIdxBits = 11;  // row index inside the node (<= 2,048 rows)

template <int SP, int F>
__global__ __launch_bounds__(1024) void kd_lds_finish_kernel(
    const float *__restrict__ W, float *__restrict__ Wout, uint32_t n, uint32_t ntiles, int L0, int depth,
    KdNode *__restrict__ nodes) {
    constexpr int NB = KdRow<SP, F>::NB, RW = KdRow<SP, F>::W;
    constexpr uint32_t LT = kd_lds_tiles<SP, F>(), NMAX = LT * kCullTile, BS = kd_lds_block<SP, F>();
    constexpr uint32_t IPT = NMAX / BS;
    static_assert(NMAX <= (1u << kKdIdxBits), "row index bits");
    using BlockSort = rocprim::block_radix_sort<uint32_t, BS, IPT>;
    __shared__ __attribute__((aligned(16))) float rows[NMAX * RW];
    __shared__ uint16_t ord[NMAX];
    __shared__ float tbs[LT][2 * NB];
    __shared__ float4 nsp[LT];
    __shared__ typename BlockSort::storage_type sort_storage;
    const KdNodeRef nd = kd_node_at(ntiles, L0, blockIdx.x);
    if (!nd.valid) return;
    const uint32_t P0 = nd.t0 * kCullTile, T = nd.T;
    const uint32_t cnt = min(T * kCullTile, n > P0 ? n - P0 : 0u);
    const uint32_t tid = threadIdx.x;
    for (uint32_t e = tid; e < cnt * (RW / 4); e += BS)
        reinterpret_cast<float4 *>(rows)[e] = reinterpret_cast<const float4 *>(W + (size_t)P0 * RW)[e];
    for (uint32_t e = tid; e < NMAX; e += BS) ord[e] = (uint16_t)e;
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int l = 0; L0 + l < depth && T > 1; ++l) {
        // 1. tile boxes of the current order (a wave per tile)
        for (uint32_t t = wave; t < T; t += BS / 64) {
            const uint32_t e = t * kCullTile + lane;
            const bool in = e < cnt;
            const float *r = rows + (size_t)ord[in ? e : 0] * RW;
#pragma unroll
            for (int d = 0; d < NB; ++d) {
                float lo = in ? r[d] : __builtin_inff(), hi = in ? r[d] : -__builtin_inff();
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) {
                    lo = fminf(lo, __shfl_xor(lo, o));
                    hi = fmaxf(hi, __shfl_xor(hi, o));
                }
                if (lane == 0) {
                    tbs[t][d] = lo;
                    tbs[t][NB + d] = hi;
                }
            }
        }
        __syncthreads();
        // 2. widest coordinate of every sub-node that splits at this sub-level: a wave per
        //    sub-node, a lane per tile (<= LT <= 32 tiles), the box extents by wave min / max
        //    reductions (exact, so the same split as a serial scan; round 3 had one thread loop
        //    over the node's tiles x coordinates, ~10 us of serial LDS reads at the top sub-level)
        const uint32_t nsub = 1u << l;
        for (uint32_t sp = (uint32_t)wave; sp < nsub; sp += BS / 64) {
            const KdNodeRef sn = kd_node_at(T, l, sp);
            if (!sn.valid || sn.T <= 1) continue;  // wave-uniform
            const bool in = (uint32_t)lane < sn.T;
            int bd = 0;
            float be = -1.f, blo = 0.f;
#pragma unroll
            for (int d = 0; d < NB; ++d) {
                float lo = in ? tbs[sn.t0 + lane][d] : __builtin_inff();
                float hi = in ? tbs[sn.t0 + lane][NB + d] : -__builtin_inff();
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) {
                    lo = fminf(lo, __shfl_xor(lo, o));
                    hi = fmaxf(hi, __shfl_xor(hi, o));
                }
                if (hi - lo > be) {  // first widest, as the global levels
                    be = hi - lo;
                    bd = d;
                    blo = lo;
                }
            }
            if (lane == 0)
                nsp[sp] = make_float4(__uint_as_float((uint32_t)bd), blo, be > 0.f ? (float)kKdQ / be : 0.f, 0.f);
        }
        __syncthreads();
        // 3. packed keys of the current order (blocked: thread tid holds positions tid * IPT + i)
        uint32_t kw[IPT];
#pragma unroll
        for (uint32_t i = 0; i < IPT; ++i) {
            const uint32_t e = tid * IPT + i;
            uint32_t kk = 1u << (kKdQBits + l);  // padding: above every (l-bit path, q) key
            if (e < cnt) {
                const uint32_t t = e / kCullTile;
                uint32_t t0 = 0, TT = T, path = 0;
                int ll = 0;
                for (; ll < l && TT > 1; ++ll) {
                    const uint32_t tl = TT >> 1;
                    const uint32_t right = t >= t0 + tl ? 1u : 0u;
                    path = (path << 1) | right;
                    if (right) {
                        t0 += tl;
                        TT -= tl;
                    } else {
                        TT = tl;
                    }
                }
                uint32_t q = 0;
                if (ll == l && TT > 1) {
                    const float4 ns = nsp[path];
                    q = kd_quant(rows[(size_t)ord[e] * RW + (int)__float_as_uint(ns.x)], ns);
                } else {
                    path <<= (l - ll);
                }
                kk = (path << kKdQBits) | q;
            }
            kw[i] = (kk << kKdIdxBits) | (e < NMAX ? (uint32_t)ord[e] : 0u);
        }
        // 4. block radix sort on the key bits only: l path bits + 12 coordinate bits + the padding
        //    bit (13 + l <= 17 bits instead of all 21 above the row index: fewer digit passes)
        BlockSort().sort(kw, sort_storage, kKdIdxBits, kKdIdxBits + kKdQBits + l + 1);
        __syncthreads();
#pragma unroll
        for (uint32_t i = 0; i < IPT; ++i) ord[tid * IPT + i] = (uint16_t)(kw[i] & ((1u << kKdIdxBits) - 1u));
        __syncthreads();
        // 5. node records of the sub-level (pre-order index = the node's + the relative one)
        for (uint32_t sp = tid; sp < nsub; sp += BS) {
            const KdNodeRef sn = kd_node_at(T, l, sp);
            if (!sn.valid || sn.T <= 1) continue;
            const uint32_t tl = sn.T >> 1, e = (sn.t0 + tl) * kCullTile;
            const int d = (int)__float_as_uint(nsp[sp].x);
            const float split = e < cnt ? rows[(size_t)ord[e] * RW + d] : __builtin_inff();
            const uint32_t pidx = nd.pidx + sn.pidx;
            nodes[pidx] = KdNode{(uint32_t)d, split, tl, pidx + tl};
        }
        __syncthreads();
    }
    for (uint32_t e = tid; e < cnt; e += BS) {
        const float4 *src = reinterpret_cast<const float4 *>(rows + (size_t)ord[e] * RW);
        float4 *dst = reinterpret_cast<float4 *>(Wout + (size_t)(P0 + e) * RW);
#pragma unroll
        for (int c = 0; c < RW / 4; ++c) dst[c] = src[c];
    }
}

// the sorted fp32 rows / ids / inverse map from the final working rows (positions [0, p_end);
// rows past n are padding)
template <int SP, int F>
__global__ void kd_rows_store_kernel(const float *__restrict__ W, uint32_t n, uint32_t p_end, uint32_t n_pad,
                                     float *__restrict__ rows, uint32_t *__restrict__ ids,
                                     uint32_t *__restrict__ inv) {
    constexpr int R = Geo<SP, F>::R, RW = KdRow<SP, F>::W, NB = KdRow<SP, F>::NB;
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= p_end) return;
    if (p < n) {
        float r[RW];
        const float4 *w4 = reinterpret_cast<const float4 *>(W + (size_t)p * RW);
#pragma unroll
        for (int c = 0; c < RW / 4; ++c) {
            const float4 v = w4[c];
            r[4 * c] = v.x; r[4 * c + 1] = v.y; r[4 * c + 2] = v.z; r[4 * c + 3] = v.w;
        }
        const uint32_t id = __float_as_uint(r[NB]);
#pragma unroll
        for (int c = 0; c < R; ++c) rows[blk_index(p, c, R)] = r[c];
        ids[p] = id;
        inv[id] = p;
    } else {
#pragma unroll
        for (int c = 0; c < R; ++c) rows[blk_index(p, c, R)] = __builtin_nanf("");
        ids[p] = kNoId;
    }
}

// fp64 features by id, AoS (fa per row, zero padded): the transpose of the SoA store, a thread per
// id (coalesced column reads, one contiguous row written), so that the sorted fp64 rows are then
// gathered one contiguous row per state
__global__ void feat_aos_kernel(const double *__restrict__ f64, uint64_t cap, int F, int fa, uint64_t n,
                                double *__restrict__ aos) {
    const uint64_t id = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= n) return;
    double2 *o = reinterpret_cast<double2 *>(aos + id * fa);
    for (int c = 0; c < fa; c += 2) {
        double2 v;
        v.x = c < F ? f64[(uint64_t)c * cap + id] : 0.0;
        v.y = c + 1 < F ? f64[(uint64_t)(c + 1) * cap + id] : 0.0;
        o[c / 2] = v;
    }
}

__global__ void rows64_gather_kernel(const double *__restrict__ aos, int F, int fa, const uint32_t *__restrict__ ids,
                                     uint32_t p_end, double *__restrict__ rows64) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;  // (slot, double2 column)
    const int h = fa / 2;
    if (t >= (uint64_t)p_end * h) return;
    const uint64_t p = t / h;
    const int c = (int)(t % h);
    const uint32_t id = ids[p];
    double2 v;
    if (id == kNoId) {  // padding: NaN features, zero pad columns
        v.x = 2 * c < F ? __builtin_nan("") : 0.0;
        v.y = 2 * c + 1 < F ? __builtin_nan("") : 0.0;
    } else {
        v = reinterpret_cast<const double2 *>(aos)[(uint64_t)id * h + c];
    }
    reinterpret_cast<double2 *>(rows64)[t] = v;
}

inline hipError_t scratch_ensure(SortedStore *s, size_t bytes) {
    if (bytes <= s->scratch_bytes) return hipSuccess;
    if (s->scratch) (void)hipFree(s->scratch);
    s->scratch = nullptr;
    s->scratch_bytes = 0;
    const size_t nb = std::max(bytes, (size_t)1 << 20);
    hipError_t e = hipMalloc(&s->scratch, nb);
    if (e == hipSuccess) s->scratch_bytes = nb;
    return e;
}

template <typename T>
inline hipError_t grow_array(T **p, size_t &have, size_t need) {
    if (need <= have && *p) return hipSuccess;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    have = 0;
    hipError_t e = hipMalloc((void **)p, sizeof(T) * std::max<size_t>(need, 1));
    if (e == hipSuccess) have = need;
    return e;
}

// (re)allocate the store's arrays for `pad_tiles` tiles (grow-only: no free / realloc in the
// steady state, so builds and tail appends stay asynchronous)
template <int SP, int F>
hipError_t sorted_alloc(SortedStore *s, uint32_t pad_tiles, uint32_t max_nodes, uint64_t inv_cap, int fa,
                        hipStream_t st) {
    constexpr int R = Geo<SP, F>::R, BW = Geo<SP, F>::BW;
    const size_t n_pad = (size_t)pad_tiles * kCullTile;
    const uint32_t nsup = (pad_tiles + kSuperTiles - 1) / kSuperTiles;
    hipError_t e;
    s->rw = R;
    if (n_pad > s->cap_pos) {  // reallocate all per-position arrays together
        size_t dummy = 0;
        if ((e = grow_array(&s->rows, dummy, (size_t)R * n_pad)) != hipSuccess) return e;
        dummy = 0;
        if ((e = grow_array(&s->ids, dummy, n_pad)) != hipSuccess) return e;
        dummy = 0;
        if ((e = grow_array(&s->rows64, dummy, n_pad * (size_t)fa)) != hipSuccess) return e;
        dummy = 0;
        if ((e = grow_array(&s->tbox, dummy, (size_t)pad_tiles * BW)) != hipSuccess) return e;
        dummy = 0;
        if ((e = grow_array(&s->sbox, dummy, (size_t)nsup * BW)) != hipSuccess) return e;
        dummy = 0;
        if ((e = grow_array(&s->mbox, dummy, (size_t)((nsup + kMegaSupers - 1) / kMegaSupers) * BW)) != hipSuccess)
            return e;
        dummy = 0;
        if ((e = grow_array(&s->tkey0, dummy, (size_t)pad_tiles)) != hipSuccess) return e;
        dummy = 0;
        if ((e = grow_array(&s->qcount, dummy, home_bins_words(pad_tiles))) != hipSuccess) return e;
        // the home-key bins are zero between calls (home_bins_scan_kernel re-zeroes what it reads)
        if ((e = hipMemsetAsync(s->qcount, 0, 4 * home_bins_words(pad_tiles), st)) != hipSuccess) return e;
        s->cap_pos = n_pad;
        hipLaunchKernelGGL(iota_kernel, dim3((pad_tiles + 255) / 256), dim3(256), 0, st, s->tkey0, pad_tiles);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    s->n_pad = (uint32_t)s->cap_pos;
    s->fa = fa;
    if ((e = grow_array(&s->nodes, s->cap_nodes, std::max<uint32_t>(max_nodes, 1))) != hipSuccess) return e;
    if ((e = grow_array(&s->inv, s->cap_inv, inv_cap)) != hipSuccess) return e;
    s->bytes = s->cap_pos * (4ull * R + 4 + 8ull * fa) + (s->cap_pos / kCullTile) * (4ull * BW + 4) +
               ((s->cap_pos / kCullTile + kSuperTiles - 1) / kSuperTiles) * 4ull * BW * (kMegaSupers + 1) / kMegaSupers +
               s->cap_nodes * sizeof(KdNode) +
               s->cap_inv * 4ull;
    return hipSuccess;
}

// Full build over ids [0, n_total) whose live flag is set (n_live of them), on `st`, no sync.
template <int SP, int F>
hipError_t build_sorted(const float *f32, const double *f64, uint64_t cap, uint64_t n_total, uint32_t n_live,
                        const uint8_t *live, SortedStore *s, hipStream_t st) {
    constexpr int NB = Geo<SP, F>::NB;
    const int fa = (F + 3) & ~3;
    const uint32_t main_tiles = std::max<uint32_t>(1, (n_live + kCullTile - 1) / kCullTile);
    const uint32_t main_sup_tiles = (main_tiles + kSuperTiles - 1) / kSuperTiles * kSuperTiles;
    const uint32_t tail_tiles = (std::max<uint32_t>(64, main_tiles / 8) + kSuperTiles - 1) / kSuperTiles * kSuperTiles;
    hipError_t e;
    if ((e = sorted_alloc<SP, F>(s, main_sup_tiles + tail_tiles, main_tiles, std::max<uint64_t>(cap, n_total), fa,
                                 st)) != hipSuccess)
        return e;
    // scratch: flags | selected ids | quantised coordinates | rows x2 | tile boxes | node splits |
    // selected count | rocPRIM temp.  The two row buffers are adjacent: after the level
    // loop they hold the fp64 features by id (feat_aos_kernel) for the rows64 gather.
    const size_t n = std::max<uint64_t>(n_total, 1);
    const uint32_t nl = std::max<uint32_t>(n_live, 1);
    constexpr int RW = KdRow<SP, F>::W;
    int depth = 0;
    while ((1u << depth) < main_tiles) ++depth;
    // global levels while some node holds more tiles than one block's LDS: level Lg is the first
    // whose nodes (ceil(main_tiles / 2^L) tiles at most) fit; kd_lds_finish_kernel does the rest
    int Lg = 0;
    while (Lg < depth && ((main_tiles + (1u << Lg) - 1) >> Lg) > kd_lds_tiles<SP, F>()) ++Lg;
    size_t tmp_sel = 0;
    rocprim::counting_iterator<uint32_t> count_it(0);
    if ((e = rocprim::select(nullptr, tmp_sel, count_it, (const uint8_t *)nullptr, (uint32_t *)nullptr,
                             (uint32_t *)nullptr, n, st)) != hipSuccess)
        return e;
    const size_t row_bytes = std::max<size_t>(4ull * RW * nl, 4ull * fa * n);  // each half of the pair
    size_t off = 0;
    auto take = [&](size_t b) {
        const size_t o = off;
        off += align_up(b);
        return o;
    };
    const size_t o_flags = take(n), o_sel = take(4 * n), o_k0 = take(4ull * nl), o_w = take(2 * row_bytes),
                 o_tb = take(4ull * main_tiles * 2 * NB), o_ns = take(16ull * main_tiles + 16), o_cnt = take(8),
                 o_tmp = take(tmp_sel);
    // median partition: bin counts per node of the deepest global level, children's boxes,
    // per-node selections, per-chunk counts
    const size_t nodes_max = Lg > 0 ? (size_t)1 << (Lg - 1) : 1;
    const size_t o_h = take(4ull * kPartBins * nodes_max), o_cb = take(4ull * 2 * NB * 2 * nodes_max),
                 o_ps = take(8ull * nodes_max), o_pc = take(8ull * (nodes_max + main_tiles / (kPartChunk / kCullTile) + 2));
    if ((e = scratch_ensure(s, off)) != hipSuccess) return e;
    char *w = (char *)s->scratch;
    uint8_t *flags = (uint8_t *)(w + o_flags);
    uint32_t *sel = (uint32_t *)(w + o_sel), *nsel = (uint32_t *)(w + o_cnt);
    uint16_t *Qp = (uint16_t *)(w + o_k0);
    float *W0 = (float *)(w + o_w), *W1 = (float *)(w + o_w + row_bytes);
    float *tb = (float *)(w + o_tb);
    float4 *nsplit = (float4 *)(w + o_ns);
    uint32_t *H = (uint32_t *)(w + o_h), *cbox = (uint32_t *)(w + o_cb);
    uint2 *psel = (uint2 *)(w + o_ps), *pcnt = (uint2 *)(w + o_pc);
    const dim3 b256(256);
    if (n_total)
        hipLaunchKernelGGL(kd_live_flags_kernel, dim3((unsigned)((n_total + 255) / 256)), b256, 0, st, live, n_total,
                           flags);
    size_t tb_bytes = tmp_sel;
    if ((e = rocprim::select(w + o_tmp, tb_bytes, count_it, flags, sel, nsel, (size_t)n_total, st)) != hipSuccess)
        return e;
    hipLaunchKernelGGL((kd_rows_init_kernel<SP, F>), dim3((nl + 255) / 256), b256, 0, st, f32, cap, sel, n_live, W0);
    if (Lg > 0)
        hipLaunchKernelGGL((kd_row_tile_boxes_kernel<SP, F>), dim3((main_tiles + 3) / 4), b256, 0, st, W0, n_live,
                           main_tiles, tb);
    for (int level = 0; level < Lg; ++level) {  // the global levels: median partitions
        constexpr int BSL = NB * 8 * 1024 <= 150 * 1024 ? 1024 : 256;
        if (level == 0) {
            if ((main_tiles >> level) > 4096u && BSL == 1024)
                hipLaunchKernelGGL((kd_node_split_dim_kernel<SP, F, BSL>), dim3(1), dim3(BSL), 0, st, tb, main_tiles,
                                   0, nsplit);
            else
                hipLaunchKernelGGL((kd_node_split_dim_kernel<SP, F, 256>), dim3(1), b256, 0, st, tb, main_tiles, 0,
                                   nsplit);
        } else {
            hipLaunchKernelGGL((kd_part_split_dim_kernel<SP, F>), dim3(((1u << level) + 255) / 256), b256, 0, st, cbox,
                               main_tiles, level, nsplit);
        }
        const uint32_t nodes_l = 1u << level;
        const uint32_t tmax = (main_tiles + nodes_l - 1) >> level;
        const uint32_t cpn = (tmax * kCullTile + kPartChunk - 1) / kPartChunk;
        const dim3 grid(cpn, nodes_l);
        if ((e = hipMemsetAsync(H, 0, 4ull * kPartBins * nodes_l, st)) != hipSuccess) return e;
        hipLaunchKernelGGL((kd_part_hist_kernel<SP, F>), grid, b256, 0, st, W0, n_live, main_tiles, level, nsplit, Qp, H);
        hipLaunchKernelGGL((kd_part_select_kernel<SP, F>), dim3(nodes_l), b256, 0, st, H, n_live, main_tiles, level,
                           nsplit, psel, s->nodes);
        hipLaunchKernelGGL(kd_part_count_kernel, grid, b256, 0, st, Qp, n_live, main_tiles, level, psel, cpn, pcnt);
        if ((e = hipMemsetAsync(cbox, 0xFF, 4ull * 2 * NB * 2 * nodes_l, st)) != hipSuccess) return e;
        hipLaunchKernelGGL((kd_part_scatter_kernel<SP, F>), grid, b256, 0, st, W0, W1, n_live, main_tiles, level, Qp,
                           psel, pcnt, cpn, cbox);
        std::swap(W0, W1);
    }
    if (Lg < depth) {  // every node of level Lg finishes its subtree in LDS
        hipLaunchKernelGGL((kd_lds_finish_kernel<SP, F>), dim3(1u << Lg), dim3(kd_lds_block<SP, F>()), 0, st, W0, W1,
                           n_live, main_tiles, Lg, depth, s->nodes);
        std::swap(W0, W1);
    }
    if ((e = hipMemsetAsync(s->inv, 0xFF, 4ull * s->cap_inv, st)) != hipSuccess) return e;
    const uint32_t p_end = (main_sup_tiles + tail_tiles) * kCullTile;  // padding: gap and tail region NaN
    hipLaunchKernelGGL((kd_rows_store_kernel<SP, F>), dim3((p_end + 255) / 256), b256, 0, st, W0, n_live, p_end,
                       s->n_pad, s->rows, s->ids, s->inv);
    hipLaunchKernelGGL((tile_box_range_kernel<SP, F>), dim3((main_sup_tiles + 3) / 4), b256, 0, st, s->rows, s->n_pad,
                       0u, main_sup_tiles, s->tbox);
    const uint32_t nsup = main_sup_tiles / kSuperTiles;
    hipLaunchKernelGGL((super_box_range_kernel<SP, F>), dim3((nsup + 3) / 4), b256, 0, st, s->tbox, main_sup_tiles,
                       (uint32_t)kSuperTiles, 0u, nsup, s->sbox);
    const uint32_t nmeg = (nsup + kMegaSupers - 1) / kMegaSupers;
    hipLaunchKernelGGL((super_box_range_kernel<SP, F>), dim3((nmeg + 3) / 4), b256, 0, st, s->sbox, nsup,
                       (uint32_t)kMegaSupers, 0u, nmeg, s->mbox);
    // fp64 rows in sorted order: transpose the SoA features by id into the (now free) row
    // buffers, then one contiguous row per slot
    double *aos = (double *)(w + o_w);
    if (n_total)
        hipLaunchKernelGGL(feat_aos_kernel, dim3((unsigned)((n_total + 255) / 256)), b256, 0, st, f64, cap, F, fa,
                           (uint64_t)n_total, aos);
    const uint32_t p64 = main_sup_tiles * kCullTile;
    const uint64_t c64 = (uint64_t)p64 * (fa / 2);
    hipLaunchKernelGGL(rows64_gather_kernel, dim3((unsigned)((c64 + 255) / 256)), b256, 0, st, aos, F, fa, s->ids, p64,
                       s->rows64);
    s->kd_tiles = main_tiles;
    s->nnodes = main_tiles - 1;
    s->main_live = n_live;
    s->tail_t0 = main_sup_tiles;
    s->tail_cap_tiles = tail_tiles;
    s->ntiles = main_sup_tiles;
    s->nsuper = nsup;
    s->nmega = nmeg;
    s->n = n_live;
    s->covered = n_total;
    s->main_covered = n_total;
    s->removed = 0;
    s->built = true;
    return hipGetLastError();
}

// Tail append: ids [main_covered, n_total) (states added since the build) re-tiled along the
// Morton curve in the tail region (tiles from tail_t0, a super-tile boundary), with their
// boxes; false in *fits when they exceed the tail region (the caller rebuilds).
template <int SP, int F>
hipError_t append_sorted(const float *f32, const double *f64, uint64_t cap, uint64_t n_total, const FastBounds &b,
                         SortedStore *s, hipStream_t st, bool *fits) {
    const uint64_t n_tail64 = n_total - s->main_covered;
    *fits = s->built && n_tail64 <= (uint64_t)s->tail_cap_tiles * kCullTile;
    if (!*fits) return hipSuccess;
    hipError_t e;
    if (n_total > s->cap_inv) {  // the store grew past the id map: grow it, keeping the placed ids
        uint32_t *ninv = nullptr;
        const size_t ncap = std::max<size_t>(2 * s->cap_inv, n_total);
        if ((e = hipMalloc(&ninv, 4ull * ncap)) != hipSuccess) return e;
        if ((e = hipMemsetAsync(ninv, 0xFF, 4ull * ncap, st)) != hipSuccess) return e;
        if ((e = hipMemcpyAsync(ninv, s->inv, 4ull * s->cap_inv, hipMemcpyDeviceToDevice, st)) != hipSuccess) return e;
        if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;  // before the old map is freed
        (void)hipFree(s->inv);
        s->inv = ninv;
        s->cap_inv = ncap;
    }
    const uint32_t n_tail = (uint32_t)n_tail64;
    if (n_tail == 0) return hipSuccess;
    const size_t cub = home_sort_bytes(n_tail);
    size_t off = 0;
    auto take = [&](size_t bb) {
        const size_t o = off;
        off += align_up(bb);
        return o;
    };
    const size_t o_k0 = take(4ull * n_tail), o_k1 = take(4ull * n_tail), o_i0 = take(4ull * n_tail),
                 o_i1 = take(4ull * n_tail), o_cub = take(cub);
    if ((e = scratch_ensure(s, off)) != hipSuccess) return e;
    char *w = (char *)s->scratch;
    uint32_t *k0 = (uint32_t *)(w + o_k0), *k1 = (uint32_t *)(w + o_k1);
    uint32_t *i0 = (uint32_t *)(w + o_i0), *i1 = (uint32_t *)(w + o_i1);
    const dim3 b256(256);
    hipLaunchKernelGGL((tail_keys_kernel<SP, F>), dim3((n_tail + 255) / 256), b256, 0, st, f32, cap, s->main_covered,
                       n_tail, b, s->nodes, s->kd_tiles, k0, i0);
    // Morton keys: 32 bits; the chain's home tiles: below kd_tiles
    const int key_bits = SP == OMPL_GPU_SPACE_KCHAIN ? (s->kd_tiles > 1 ? 32 - __builtin_clz(s->kd_tiles - 1) : 1) : 32;
    if ((e = sort_home_keys(w + o_cub, cub, k0, k1, i0, i1, n_tail, key_bits, st)) != hipSuccess) return e;
    const uint32_t tiles = (n_tail + kCullTile - 1) / kCullTile;
    const uint32_t p0 = s->tail_t0 * kCullTile, p1 = p0 + tiles * kCullTile;
    hipLaunchKernelGGL((sorted_gather_kernel<SP, F>), dim3((p1 - p0 + 255) / 256), b256, 0, st, f32, cap, i1, n_tail,
                       p0, p1, s->n_pad, s->rows, s->ids, s->inv);
    const uint32_t t1 = s->tail_t0 + tiles;
    hipLaunchKernelGGL((tile_box_range_kernel<SP, F>), dim3((tiles + 3) / 4), b256, 0, st, s->rows, s->n_pad,
                       s->tail_t0, t1, s->tbox);
    const uint32_t s0 = s->tail_t0 / kSuperTiles, s1 = (t1 + kSuperTiles - 1) / kSuperTiles;
    hipLaunchKernelGGL((super_box_range_kernel<SP, F>), dim3((s1 - s0 + 3) / 4), b256, 0, st, s->tbox, t1,
                       (uint32_t)kSuperTiles, s0, s1, s->sbox);
    // the megas over the re-boxed super-tiles (the first may also hold main super-tiles: a union)
    const uint32_t m0 = s0 / kMegaSupers, m1 = (s1 + kMegaSupers - 1) / kMegaSupers;
    hipLaunchKernelGGL((super_box_range_kernel<SP, F>), dim3((m1 - m0 + 3) / 4), b256, 0, st, s->sbox, s1,
                       (uint32_t)kMegaSupers, m0, m1, s->mbox);
    const uint64_t c64 = (uint64_t)(p1 - p0) * s->fa;
    hipLaunchKernelGGL(rows64_range_kernel, dim3((unsigned)((c64 + 255) / 256)), b256, 0, st, f64, cap, F, s->fa,
                       s->ids, p0, p1, s->rows64);
    s->ntiles = t1;
    s->nsuper = s1;
    s->nmega = m1;
    s->n = p1;
    s->covered = n_total;
    return hipGetLastError();
}

}  // namespace

// per-space entry points (one translation unit each)
#define OMPL_AMD_FAST_DECL(NAME)                                                                             \
    hipError_t NAME(const DevSpace &sp, const FeatGeom &g, const double *feat64, const float *feat32,          \
                    uint64_t cap, uint64_t n_end, const SortedStore *sorted, const double *qfeat64, uint32_t nq, \
                    uint32_t k, const FastBounds &b, double *out_d, uint32_t *out_i, void *ws, size_t ws_bytes,  \
                    int num_cus, hipStream_t st, uint32_t **fail_count, uint32_t **fail_list);                  \
    hipError_t NAME##_build(const FeatGeom &g, const float *feat32, const double *feat64, uint64_t cap,          \
                            uint64_t n_total, uint32_t n_live, const uint8_t *live, SortedStore *s, hipStream_t st); \
    hipError_t NAME##_append(const FeatGeom &g, const float *feat32, const double *feat64, uint64_t cap,         \
                             uint64_t n_total, const FastBounds &b, SortedStore *s, hipStream_t st, bool *fits);  \
    hipError_t NAME##_radius(const DevSpace &sp, const FeatGeom &g, const double *feat64, uint64_t cap,          \
                             const SortedStore *sorted, const double *qfeat64, uint32_t nq, double r,          \
                             const FastBounds &b, void *ws, size_t ws_bytes, int phase, uint64_t **d_offsets,  \
                             uint32_t *out_i, double *out_d, hipStream_t st);
OMPL_AMD_FAST_DECL(fast_se3)
OMPL_AMD_FAST_DECL(fast_so3)
OMPL_AMD_FAST_DECL(fast_rv)
OMPL_AMD_FAST_DECL(fast_chain)

// common body of the per-space entry points
template <int SP, int F>
hipError_t fast_entry(const DevSpace &sp, const FeatGeom &g, const double *feat64, const float *feat32, uint64_t cap,
                      uint64_t n_end, const SortedStore *sorted, const double *qfeat64, uint32_t nq, uint32_t k,
                      const FastBounds &b, double *out_d, uint32_t *out_i, void *ws, size_t ws_bytes, int num_cus,
                      hipStream_t st, uint32_t **fail_count, uint32_t **fail_list) {
    const FastPlan p = fast_plan(sp, nq, k, n_end, num_cus, sorted != nullptr);
    if (p.K2 == 0) return hipErrorInvalidValue;
    const FastLayout L = fast_layout(sp, g, p, nq);
    if (L.total > ws_bytes) return hipErrorInvalidValue;
    char *w = (char *)ws;
    *fail_count = (uint32_t *)(w + L.fail);
    *fail_list = *fail_count + 1;
    return run_fast_space<SP, F>(sp, p, L, w, feat32, feat64, cap, n_end, sorted, qfeat64, nq, k, b, out_d, out_i,
                                 st);
}

template <int SP, int F>
hipError_t fast_radius_entry(const DevSpace &sp, const FeatGeom &g, const double *feat64, uint64_t cap,
                             const SortedStore *sorted, const double *qfeat64, uint32_t nq, double r,
                             const FastBounds &b, void *ws, size_t ws_bytes, int phase, uint64_t **d_offsets,
                             uint32_t *out_i, double *out_d, hipStream_t st) {
    if (!sorted || nq == 0) return hipErrorInvalidValue;
    const RadiusLayout L = radius_layout(sp, g, nq);
    if (L.total > ws_bytes) return hipErrorInvalidValue;
    char *w = (char *)ws;
    *d_offsets = (uint64_t *)(w + L.off);
    return run_radius_fast<SP, F>(sp, L, w, feat64, cap, sorted, qfeat64, nq, r, b, phase, out_i, out_d, st);
}

}  // namespace ompl_amd
