// rrtstar.hip — RRT*'s iteration batch on the device (the RRT* half).
//
// RRTstar::solve (geometric/planners/rrt/src/RRTstar.cpp:247-542) with its defaults — k-nearest
// neighbourhoods (useKNearest_, RRTstar.h:445), delayed collision checks (delayCC_, :458), no
// new-state rejection, no tree pruning — does per sample s_i, in order:
//   nmotion = nearest(s_i)                                         :266
//   x_i = s_i, or interpolate(nmotion, s_i, maxDistance / d)       :271-279
//   if checkMotion(nmotion, x_i):                                  :282
//     nbh = nearestK(x_i, k_i), k_i = ceil(k_rrt ln(size + 1))     :292, getNeighbors :603-618
//     parent = first in cost order with d < maxDistance and checkMotion(nbh, x_i)   :319-357
//     add x_i                                                      :410
//     rewire every nbh whose cost improves through x_i, checkMotion(x_i, nbh)       :414-457
// The geometric part — nearest, steer, the motion bit, which states join the tree, every
// neighbourhood, and both motion bits of every (neighbour, x_i) pair — does not depend on the
// costs, so the device computes it for a whole batch; the planner's cost logic (parent choice in
// cost order, rewiring, child-cost propagation) then needs only lookups (ompl_amd/rrtstar.py).
//
// The batch is exact for the sequential loop, in which sample i sees the states of samples < i:
//   1. every sample's nearest stored state (the batched kNN), steer, checkMotion;
//   2. fixed point over the batch: sample i's nearest is the smaller (distance, id) of its stored
//      nearest and the nearest earlier added state x_j (a wave per sample over the compacted list
//      of added states; added ids are n0 + rank); steer and check again; repeat until no state
//      and no bit changes.  Sample i depends only on samples < i, so each round fixes at least
//      one more leading sample and the loop ends (in practice after 1-2 rounds);
//   3. neighbourhoods of the added states: the stored part by the batched kNN (large-k path), the
//      in-batch part by PRM*'s causal scan (prm.hip: earlier added states within the stored
//      list's k_i-th distance), merged per segment in (distance, id) order and cut at k_i;
//   4. checkMotion(nbh, x_i) and checkMotion(x_i, nbh) for every neighbourhood entry;
//   5. the added states join the store.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "kernels.h"
#include "topk.h"

namespace ompl_amd {

namespace {

constexpr uint32_t kInBatch = kRrtStarInBatch;  // nearest source: bit 31 = sample j of the batch

// state of a nearest source: a stored id (raw SoA) or an earlier sample's steered state
template <int W>
__device__ __forceinline__ void source_state(uint32_t src, const double *__restrict__ raw, uint64_t cap,
                                             const double *__restrict__ x, int dim, double *o) {
    if (src & kInBatch) {
        const double *p = x + (size_t)(src & ~kInBatch) * dim;
        for (int c = 0; c < dim; ++c) o[c] = p[c];
    } else {
        for (int c = 0; c < dim; ++c) o[c] = raw[(uint64_t)c * cap + src];
    }
}

// RRT.cpp:141-146 / RRTstar.cpp:271-279 from each sample's current nearest source: from, to
// (= the new state x_i) and inc = distance(nmotion, x_i) (the motion's incCost, RRTstar.cpp:288)
template <int SP, int W>
__global__ void rrtstar_steer_kernel(DevSpace sp_in, const double *__restrict__ raw, uint64_t cap,
                                     const double *__restrict__ samples, uint32_t ns, const uint32_t *__restrict__ src,
                                     const double *__restrict__ x_prev, double maxd, double *__restrict__ from,
                                     double *__restrict__ to, double *__restrict__ inc) {
    const DevSpace sp = fixed_space<SP, W>(sp_in);
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= ns) return;
    const int dim = sp.dim;
    double a[Width<W>::N], b[Width<W>::N], o[Width<W>::N];
    source_state<W>(src[i], raw, cap, x_prev, dim, a);
    for (int c = 0; c < dim; ++c) b[c] = samples[(size_t)i * dim + c];
    const double d = raw_distance(sp, a, b);
    if (d > maxd) {
        interpolate(sp, a, b, maxd / d, o);
        inc[i] = raw_distance(sp, a, o);
    } else {
        for (int c = 0; c < dim; ++c) o[c] = b[c];
        inc[i] = d;
    }
    for (int c = 0; c < dim; ++c) {
        from[(size_t)i * dim + c] = a[c];
        to[(size_t)i * dim + c] = o[c];
    }
}

// exclusive ranks of the added samples (valid[i] != 0) and their compacted list, one block of
// 1,024 threads: rank[i], list[rank] = i, rank[ns] = the count
__global__ __launch_bounds__(1024) void rrtstar_rank_kernel(const uint8_t *__restrict__ valid, uint32_t ns,
                                                            uint32_t *__restrict__ rank, uint32_t *__restrict__ list) {
    __shared__ uint32_t wsum[16];
    const uint32_t t = threadIdx.x, per = (ns + 1023) / 1024;
    const uint32_t b = t * per, e = min(ns, b + per);
    uint32_t c = 0;
    for (uint32_t i = b; i < e; ++i) c += valid[i] ? 1u : 0u;
    // block exclusive scan of c: wave inclusive scans, then the wave totals
    const int lane = t & 63, w = t >> 6;
    uint32_t inc = c;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t v = __shfl_up(inc, o, 64);
        if (lane >= o) inc += v;
    }
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    if (t == 0) {
        uint32_t s = 0;
        for (int i = 0; i < 16; ++i) {
            const uint32_t v = wsum[i];
            wsum[i] = s;
            s += v;
        }
    }
    __syncthreads();
    uint32_t r = wsum[w] + inc - c;
    for (uint32_t i = b; i < e; ++i) {
        rank[i] = r;
        if (valid[i]) list[r++] = i;
    }
    if (t == 1023) rank[ns] = r;
}

// one wave per sample i: the nearest earlier added state, (distance, index) smallest, against the
// stored nearest (near_d, near_id); src[i] = the winner (stored wins a tie: its id is smaller)
template <int SP, int W>
__global__ __launch_bounds__(256) void rrtstar_causal_kernel(DevSpace sp_in, const double *__restrict__ samples,
                                                            uint32_t ns, const double *__restrict__ x,
                                                            const uint32_t *__restrict__ rank,
                                                            const uint32_t *__restrict__ list,
                                                            const uint32_t *__restrict__ near_id,
                                                            const double *__restrict__ near_d,
                                                            uint32_t *__restrict__ src) {
    const DevSpace sp = fixed_space<SP, W>(sp_in);
    const uint32_t i = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (i >= ns) return;
    const int dim = sp.dim;
    double q[Width<W>::N], s[Width<W>::N];
    for (int c = 0; c < dim; ++c) q[c] = samples[(size_t)i * dim + c];
    const uint32_t before = rank[i];  // added samples j < i
    double bd = __builtin_inf();
    uint32_t bt = 0xFFFFFFFFu;
    for (uint32_t t = lane; t < before; t += 64) {
        const uint32_t j = list[t];
        for (int c = 0; c < dim; ++c) s[c] = x[(size_t)j * dim + c];
        const double d = raw_distance(sp, s, q);  // element first, query second
        if (d < bd) {  // t increases: the first minimum is the smallest id
            bd = d;
            bt = t;
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        const double od = __shfl_xor(bd, o, 64);
        const uint32_t ot = __shfl_xor(bt, o, 64);
        if (od < bd || (od == bd && ot < bt)) {
            bd = od;
            bt = ot;
        }
    }
    if (lane == 0) {
        const double sd = near_d[i];
        src[i] = (bt != 0xFFFFFFFFu && bd < sd) ? (kInBatch | list[bt]) : near_id[i];
    }
}

// changed += the samples whose new state or motion bit differs from the previous round's
__global__ void rrtstar_diff_kernel(const double *__restrict__ xa, const double *__restrict__ xb,
                                    const uint8_t *__restrict__ va, const uint8_t *__restrict__ vb, uint32_t ns, int dim,
                                    uint32_t *__restrict__ changed) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    bool d = false;
    if (i < ns) {
        d = va[i] != vb[i];
        for (int c = 0; c < dim && !d; ++c) {
            const double a = xa[(size_t)i * dim + c], b = xb[(size_t)i * dim + c];
            d = __double_as_longlong(a) != __double_as_longlong(b);
        }
    }
    const uint64_t m = __ballot(d);
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(changed, (uint32_t)__popcll(m));
}

// per sample: the nearest id (in-batch sources -> n0 + rank), the added id, and the compacted
// rows of the added states (xa) in rank order
__global__ void rrtstar_finish_kernel(const uint32_t *__restrict__ src, const uint8_t *__restrict__ valid,
                                      const uint32_t *__restrict__ rank, const double *__restrict__ x, uint32_t ns,
                                      int dim, uint32_t n0, uint32_t *__restrict__ nearest, uint32_t *__restrict__ added,
                                      double *__restrict__ xa) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= ns) return;
    const uint32_t s = src[i];
    nearest[i] = (s & kInBatch) ? n0 + rank[s & ~kInBatch] : s;
    const bool v = valid[i] != 0;
    added[i] = v ? n0 + rank[i] : kNoId;
    if (v)
        for (int c = 0; c < dim; ++c) xa[(size_t)rank[i] * dim + c] = x[(size_t)i * dim + c];
}

// a segment's candidates (the unsorted tail after its st stored entries) sorted in LDS by
// (distance, id), then merged with the sorted stored entries by rank: entry at merged rank r < k
// goes to out + r.  One block of 256 per segment; segments with more than kMergeCands candidates
// are left to the caller (flag).
constexpr uint32_t kMergeCands = kRrtStarMergeCands;
__global__ __launch_bounds__(256) void rrtstar_merge_kernel(const uint64_t *__restrict__ seg_off,
                                                            const uint32_t *__restrict__ stored_cnt,
                                                            const uint32_t *__restrict__ kj,
                                                            const uint32_t *__restrict__ in_i,
                                                            const double *__restrict__ in_d,
                                                            const uint64_t *__restrict__ out_off,
                                                            uint32_t *__restrict__ out_i, double *__restrict__ out_d,
                                                            uint32_t *__restrict__ out_seg, uint32_t rows,
                                                            uint32_t *__restrict__ overflow) {
    __shared__ double cd[kMergeCands];
    __shared__ uint32_t ci[kMergeCands];
    __shared__ double sd2[kMergeCands];
    __shared__ uint32_t si2[kMergeCands];
    const uint32_t j = blockIdx.x;
    if (j >= rows) return;
    const uint64_t b = seg_off[j], len = seg_off[j + 1] - b;
    const uint32_t st = stored_cnt[j];
    const uint32_t nc = (uint32_t)(len - st);
    const uint64_t ob = out_off[j];
    const uint32_t k = (uint32_t)(out_off[j + 1] - ob);  // min(k_j, len)
    (void)kj;
    if (nc > kMergeCands) {
        if (threadIdx.x == 0) atomicAdd(overflow, 1u);
        return;
    }
    for (uint32_t t = threadIdx.x; t < nc; t += blockDim.x) {
        cd[t] = in_d[b + st + t];
        ci[t] = in_i[b + st + t];
    }
    __syncthreads();
    // candidates ranked among themselves (ids unique), placed sorted
    for (uint32_t t = threadIdx.x; t < nc; t += blockDim.x) {
        const double d = cd[t];
        const uint32_t id = ci[t];
        uint32_t r = 0;
        for (uint32_t u = 0; u < nc; ++u) r += (cd[u] < d || (cd[u] == d && ci[u] < id)) ? 1u : 0u;
        sd2[r] = d;
        si2[r] = id;
    }
    __syncthreads();
    // stored entry r: merged rank r + #candidates ordered before it
    for (uint32_t r = threadIdx.x; r < st; r += blockDim.x) {
        const double d = in_d[b + r];
        const uint32_t id = in_i[b + r];
        uint32_t lo = 0, hi = nc;  // first candidate not before (d, id)
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (sd2[mid] < d || (sd2[mid] == d && si2[mid] < id))
                lo = mid + 1;
            else
                hi = mid;
        }
        const uint32_t pos = r + lo;
        if (pos < k) {
            out_i[ob + pos] = id;
            out_d[ob + pos] = d;
            out_seg[ob + pos] = j;
        }
    }
    // candidate c: merged rank c + #stored entries ordered before it
    for (uint32_t c = threadIdx.x; c < nc; c += blockDim.x) {
        const double d = sd2[c];
        const uint32_t id = si2[c];
        uint32_t lo = 0, hi = st;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            const double md = in_d[b + mid];
            const uint32_t mi = in_i[b + mid];
            if (md < d || (md == d && mi < id))
                lo = mid + 1;
            else
                hi = mid;
        }
        const uint32_t pos = c + lo;
        if (pos < k) {
            out_i[ob + pos] = id;
            out_d[ob + pos] = d;
            out_seg[ob + pos] = j;
        }
    }
}

// fully sorted segments (the radix fallback): the first out counts of each
__global__ void rrtstar_take_kernel(const uint64_t *__restrict__ seg_off, const uint32_t *__restrict__ in_i,
                                    const double *__restrict__ in_d, const uint64_t *__restrict__ out_off, uint32_t rows,
                                    uint32_t *__restrict__ out_i, double *__restrict__ out_d, uint32_t *__restrict__ out_seg) {
    const uint32_t j = blockIdx.x;
    if (j >= rows) return;
    const uint64_t b = seg_off[j], ob = out_off[j], k = out_off[j + 1] - ob;
    for (uint64_t r = threadIdx.x; r < k; r += blockDim.x) {
        out_i[ob + r] = in_i[b + r];
        out_d[ob + r] = in_d[b + r];
        out_seg[ob + r] = j;
    }
}

// stored entries kept per segment (those of the first min(k_j, kq) that exist) and the output
// count min(k_j, segment length)
// a block per row: the row's stored entries (of its first min(k_j, kq)) counted over the block,
// coalesced (a thread per row read its kq-long row serially: ~1 ms per 10^4-sample batch)
__global__ __launch_bounds__(256) void rrtstar_counts_kernel(const uint32_t *__restrict__ si, uint32_t kq,
                                                             const uint32_t *__restrict__ kj,
                                                             const uint64_t *__restrict__ seg_off, uint32_t rows,
                                                             uint32_t *__restrict__ stored_cnt,
                                                             uint64_t *__restrict__ out_cnt) {
    const uint32_t j = blockIdx.x;
    const uint32_t lim = min(kj[j], kq);
    uint32_t c = 0;
    for (uint32_t r = threadIdx.x; r < lim; r += blockDim.x) c += si[(size_t)j * kq + r] != kNoId ? 1u : 0u;
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    __shared__ uint32_t part[4];
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        stored_cnt[j] = part[0] + part[1] + part[2] + part[3];
        out_cnt[j] = min((uint64_t)kj[j], seg_off[j + 1] - seg_off[j]);
    }
}

// edge e of the merged neighbourhoods: s1 = the neighbour's state, s2 = the segment's new state
__global__ void rrtstar_edges_kernel(const uint32_t *__restrict__ ids, const uint32_t *__restrict__ seg, uint64_t E,
                                     uint32_t n0, int dim, const double *__restrict__ aos, int da,
                                     const double *__restrict__ xa, double *__restrict__ s1, double *__restrict__ s2) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= E * (uint64_t)dim) return;
    const uint64_t e = t / dim;
    const int c = (int)(t % dim);
    const uint32_t id = ids[e];
    s1[t] = id < n0 ? aos[(size_t)id * da + c] : xa[(size_t)(id - n0) * dim + c];
    s2[t] = xa[(size_t)seg[e] * dim + c];
}

__global__ void rrtstar_bits_kernel(const uint8_t *__restrict__ fwd, const uint8_t *__restrict__ bwd, uint64_t E,
                                    uint8_t *__restrict__ bits) {
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e < E) bits[e] = (uint8_t)((fwd[e] ? 1u : 0u) | (bwd[e] ? 2u : 0u));
}

// per-sample CSR offsets of the neighbourhoods: segment of sample i = segment rank[i] of the
// added states when sample i was added, else empty
__global__ void rrtstar_sample_offsets_kernel(const uint8_t *__restrict__ valid, const uint32_t *__restrict__ rank,
                                              const uint64_t *__restrict__ out_off, uint32_t ns,
                                              uint64_t *__restrict__ off) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i > ns) return;
    off[i] = out_off[rank[i]];  // rank[ns] = m: the total
    (void)valid;
}

template <class F>
hipError_t with_width(const DevSpace &sp, F &&f) {
    if (sp.kind == OMPL_GPU_SPACE_SE3 && sp.dim == 7) return f(std::integral_constant<int, OMPL_GPU_SPACE_SE3>{}, std::integral_constant<int, 7>{});
    if (sp.kind == OMPL_GPU_SPACE_REALVECTOR && sp.dim == 6)
        return f(std::integral_constant<int, OMPL_GPU_SPACE_REALVECTOR>{}, std::integral_constant<int, 6>{});
    return f(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{});
}

}  // namespace

hipError_t launch_rrtstar_steer(const DevSpace &sp, const double *raw, uint64_t cap, const double *samples, uint32_t ns,
                                const uint32_t *src, const double *x_prev, double maxd, double *from, double *to,
                                double *inc, hipStream_t st) {
    if (ns == 0) return hipSuccess;
    return with_width(sp, [&](auto S, auto W) {
        hipLaunchKernelGGL((rrtstar_steer_kernel<decltype(S)::value, decltype(W)::value>), dim3((ns + 255) / 256),
                           dim3(256), 0, st, sp, raw, cap, samples, ns, src, x_prev, maxd, from, to, inc);
        return hipGetLastError();
    });
}

hipError_t launch_rrtstar_rank(const uint8_t *valid, uint32_t ns, uint32_t *rank, uint32_t *list, hipStream_t st) {
    hipLaunchKernelGGL(rrtstar_rank_kernel, dim3(1), dim3(1024), 0, st, valid, ns, rank, list);
    return hipGetLastError();
}

hipError_t launch_rrtstar_causal(const DevSpace &sp, const double *samples, uint32_t ns, const double *x,
                                 const uint32_t *rank, const uint32_t *list, const uint32_t *near_id,
                                 const double *near_d, uint32_t *src, hipStream_t st) {
    if (ns == 0) return hipSuccess;
    return with_width(sp, [&](auto S, auto W) {
        hipLaunchKernelGGL((rrtstar_causal_kernel<decltype(S)::value, decltype(W)::value>), dim3((ns + 3) / 4),
                           dim3(256), 0, st, sp, samples, ns, x, rank, list, near_id, near_d, src);
        return hipGetLastError();
    });
}

hipError_t launch_rrtstar_diff(const double *xa, const double *xb, const uint8_t *va, const uint8_t *vb, uint32_t ns,
                               int dim, uint32_t *changed, hipStream_t st) {
    if (ns == 0) return hipSuccess;
    hipLaunchKernelGGL(rrtstar_diff_kernel, dim3((ns + 255) / 256), dim3(256), 0, st, xa, xb, va, vb, ns, dim, changed);
    return hipGetLastError();
}

hipError_t launch_rrtstar_finish(const uint32_t *src, const uint8_t *valid, const uint32_t *rank, const double *x,
                                 uint32_t ns, int dim, uint32_t n0, uint32_t *nearest, uint32_t *added, double *xa,
                                 hipStream_t st) {
    if (ns == 0) return hipSuccess;
    hipLaunchKernelGGL(rrtstar_finish_kernel, dim3((ns + 255) / 256), dim3(256), 0, st, src, valid, rank, x, ns, dim, n0,
                       nearest, added, xa);
    return hipGetLastError();
}

hipError_t launch_rrtstar_counts(const uint32_t *si, uint32_t kq, const uint32_t *kj, const uint64_t *seg_off,
                                 uint32_t rows, uint32_t *stored_cnt, uint64_t *out_cnt, hipStream_t st) {
    if (rows == 0) return hipSuccess;
    hipLaunchKernelGGL(rrtstar_counts_kernel, dim3(rows), dim3(256), 0, st, si, kq, kj, seg_off, rows, stored_cnt,
                       out_cnt);
    return hipGetLastError();
}

hipError_t launch_rrtstar_merge(const uint64_t *seg_off, const uint32_t *stored_cnt, const uint32_t *kj,
                                const uint32_t *in_i, const double *in_d, const uint64_t *out_off, uint32_t *out_i,
                                double *out_d, uint32_t *out_seg, uint32_t rows, uint32_t *overflow, hipStream_t st) {
    if (rows == 0) return hipSuccess;
    hipLaunchKernelGGL(rrtstar_merge_kernel, dim3(rows), dim3(256), 0, st, seg_off, stored_cnt, kj, in_i, in_d, out_off,
                       out_i, out_d, out_seg, rows, overflow);
    return hipGetLastError();
}

hipError_t launch_rrtstar_take(const uint64_t *seg_off, const uint32_t *in_i, const double *in_d, const uint64_t *out_off,
                               uint32_t rows, uint32_t *out_i, double *out_d, uint32_t *out_seg, hipStream_t st) {
    if (rows == 0) return hipSuccess;
    hipLaunchKernelGGL(rrtstar_take_kernel, dim3(rows), dim3(256), 0, st, seg_off, in_i, in_d, out_off, rows, out_i,
                       out_d, out_seg);
    return hipGetLastError();
}

hipError_t launch_rrtstar_edges(const uint32_t *ids, const uint32_t *seg, uint64_t E, uint32_t n0, int dim,
                                const double *aos, int da, const double *xa, double *s1, double *s2, hipStream_t st) {
    const uint64_t n = E * (uint64_t)dim;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(rrtstar_edges_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, ids, seg, E, n0, dim,
                       aos, da, xa, s1, s2);
    return hipGetLastError();
}

hipError_t launch_rrtstar_bits(const uint8_t *fwd, const uint8_t *bwd, uint64_t E, uint8_t *bits, hipStream_t st) {
    if (E == 0) return hipSuccess;
    hipLaunchKernelGGL(rrtstar_bits_kernel, dim3((unsigned)((E + 255) / 256)), dim3(256), 0, st, fwd, bwd, E, bits);
    return hipGetLastError();
}

hipError_t launch_rrtstar_sample_offsets(const uint8_t *valid, const uint32_t *rank, const uint64_t *out_off,
                                         uint32_t ns, uint64_t *off, hipStream_t st) {
    hipLaunchKernelGGL(rrtstar_sample_offsets_kernel, dim3((ns + 1 + 255) / 256), dim3(256), 0, st, valid, rank, out_off,
                       ns, off);
    return hipGetLastError();
}

}  // namespace ompl_amd
