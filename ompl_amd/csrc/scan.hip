// scan.hip — exclusive prefix sums of 64-bit counts on the device (CSR offsets of the radius,
// PRM* and RRT* paths): out[i] = in[0] + ... + in[i - 1] for i in [0, n], so out[n] is the total,
// and optionally the largest element (the radius path's longest segment).  Three launches, no host
// round trip: per-1,024-element block totals (and maxima), one block scanning the totals, then
// every block's local scan plus its offset.  Wave scans by shuffles.
//
// Also the segmented sort by (distance, id) for segments too long for a wave's LDS rank sort
// (knn.hip segment_rank_sort_kernel, <= kRankSortMax): bottom-up merge passes, each element placing
// itself by a binary search in its partner run (merge path), ping-pong buffers.
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace ompl_amd {

namespace {

constexpr uint32_t kScanBlock = 1024;  // elements per block (256 threads x 4)

__device__ __forceinline__ uint64_t wave_inclusive(uint64_t v) {
    const int lane = threadIdx.x & 63;
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t u = (uint64_t)__shfl_up((long long)v, o, 64);
        if (lane >= o) v += u;
    }
    return v;
}

// block exclusive scan of one value per thread (256 threads); *total = the block's sum
__device__ __forceinline__ uint64_t block_exclusive(uint64_t v, uint64_t *total) {
    __shared__ uint64_t ws[4];
    const uint64_t inc = wave_inclusive(v);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 63) ws[w] = inc;
    __syncthreads();
    uint64_t off = 0, tot = 0;
    for (int i = 0; i < 4; ++i) {
        if (i < w) off += ws[i];
        tot += ws[i];
    }
    __syncthreads();
    *total = tot;
    return off + inc - v;
}

// block maximum of one value per thread (256 threads), valid in every thread
__device__ __forceinline__ uint64_t block_max(uint64_t v) {
    __shared__ uint64_t wm[4];
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t u = (uint64_t)__shfl_xor((long long)v, o, 64);
        v = u > v ? u : v;
    }
    if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = v;
    __syncthreads();
    uint64_t m = wm[0];
    for (int i = 1; i < 4; ++i) m = wm[i] > m ? wm[i] : m;
    __syncthreads();
    return m;
}

// part[b] = block b's total; with MAX, part[nb + b] = its largest element
template <bool MAX>
__global__ __launch_bounds__(256) void scan_totals_kernel(const uint64_t *__restrict__ in, uint64_t n,
                                                          uint64_t *__restrict__ part) {
    const uint64_t b = (uint64_t)blockIdx.x * kScanBlock + threadIdx.x * 4;
    uint64_t s = 0, m = 0;
    for (int k = 0; k < 4; ++k) {
        const uint64_t v = b + k < n ? in[b + k] : 0;
        s += v;
        m = v > m ? v : m;
    }
    uint64_t tot;
    block_exclusive(s, &tot);
    if (threadIdx.x == 0) part[blockIdx.x] = tot;
    if constexpr (MAX) {
        m = block_max(m);
        if (threadIdx.x == 0) part[gridDim.x + blockIdx.x] = m;
    }
}

// one block: exclusive scan of nb block totals in place, chunk by chunk; with MAX the largest of
// the block maxima goes to *max_out
template <bool MAX>
__global__ __launch_bounds__(256) void scan_parts_kernel(uint64_t *__restrict__ part, uint32_t nb,
                                                         uint64_t *__restrict__ max_out) {
    __shared__ uint64_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    uint64_t m = 0;
    for (uint32_t c = 0; c < nb; c += 256) {
        const uint32_t i = c + threadIdx.x;
        const uint64_t v = i < nb ? part[i] : 0;
        if (MAX && i < nb) m = part[nb + i] > m ? part[nb + i] : m;
        uint64_t tot;
        const uint64_t ex = block_exclusive(v, &tot);
        const uint64_t base = carry;
        if (i < nb) part[i] = base + ex;
        __syncthreads();
        if (threadIdx.x == 0) carry = base + tot;
        __syncthreads();
    }
    if constexpr (MAX) {
        m = block_max(m);
        if (threadIdx.x == 0) *max_out = m;
    }
}

__global__ __launch_bounds__(256) void scan_apply_kernel(const uint64_t *__restrict__ in, uint64_t n,
                                                         const uint64_t *__restrict__ part, uint64_t *__restrict__ out) {
    const uint64_t b = (uint64_t)blockIdx.x * kScanBlock + threadIdx.x * 4;
    uint64_t v[4], s = 0;
    for (int k = 0; k < 4; ++k) {
        v[k] = b + k < n ? in[b + k] : 0;
        s += v[k];
    }
    uint64_t tot;
    uint64_t run = part[blockIdx.x] + block_exclusive(s, &tot);
    for (int k = 0; k < 4; ++k) {
        if (b + k < n) out[b + k] = run;
        run += v[k];
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 255) out[n] = part[blockIdx.x] + tot;
}

// (distance, id) as one total order: the distance's bits made monotone (NaN above +inf)
__device__ __forceinline__ uint64_t dist_order(double d) {
    const uint64_t u = (uint64_t)__double_as_longlong(d);
    return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}

__global__ void segment_of_kernel(const uint64_t *__restrict__ off, uint32_t nseg, uint64_t n,
                                  uint32_t *__restrict__ seg) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    uint32_t lo = 0, hi = nseg;  // the last segment whose start is <= t
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (off[mid] <= t) lo = mid; else hi = mid;
    }
    seg[t] = lo;
}

// one pass: runs of w elements of a segment merged pairwise; an element of the left run counts the
// partner's elements ordered before it, one of the right run those ordered before or equal
__global__ void merge_pass_kernel(const uint64_t *__restrict__ off, const uint32_t *__restrict__ seg, uint64_t n,
                                  uint64_t w, const uint32_t *__restrict__ in_i, const double *__restrict__ in_d,
                                  uint32_t *__restrict__ out_i, double *__restrict__ out_d) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const uint32_t s = seg[t];
    const uint64_t a = off[s], b = off[s + 1], p = t - a, r = p / w;
    const uint64_t pa = a + (r ^ 1) * w, pb = pa + w < b ? pa + w : b;
    const uint32_t id = in_i[t];
    const double d = in_d[t];
    if (pa >= b) {  // the segment's last run has no partner this pass
        out_i[t] = id;
        out_d[t] = d;
        return;
    }
    const uint64_t key = dist_order(d);
    const bool left = (r & 1) == 0;
    uint64_t lo = pa, hi = pb;  // first partner element not ordered before this one
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        const uint64_t km = dist_order(in_d[mid]);
        const uint32_t im = in_i[mid];
        const bool before = left ? (km < key || (km == key && im < id)) : (km < key || (km == key && im <= id));
        if (before) lo = mid + 1; else hi = mid;
    }
    const uint64_t pos = a + (r & ~1ull) * w + (p - r * w) + (lo - pa);
    out_i[pos] = id;
    out_d[pos] = d;
}

}  // namespace

size_t segment_sort_workspace(uint64_t n) { return sizeof(uint32_t) * (n ? n : 1); }

hipError_t launch_segment_sort(const uint64_t *off, uint32_t nseg, uint64_t n, uint64_t max_len, uint32_t *i0,
                               double *d0, uint32_t *i1, double *d1, void *ws, hipStream_t st, int *in_second) {
    *in_second = 0;
    if (n == 0 || nseg == 0 || max_len < 2) return hipSuccess;
    uint32_t *seg = (uint32_t *)ws;
    const unsigned blocks = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(segment_of_kernel, dim3(blocks), dim3(256), 0, st, off, nseg, n, seg);
    int cur = 0;
    for (uint64_t w = 1; w < max_len; w <<= 1) {
        hipLaunchKernelGGL(merge_pass_kernel, dim3(blocks), dim3(256), 0, st, off, seg, n, w, cur ? i1 : i0,
                           cur ? d1 : d0, cur ? i0 : i1, cur ? d0 : d1);
        cur ^= 1;
    }
    *in_second = cur;
    return hipGetLastError();
}

size_t exclusive_scan_u64_workspace(uint64_t n) {
    return sizeof(uint64_t) * (2 * ((n + kScanBlock - 1) / kScanBlock) + 1);
}

hipError_t launch_exclusive_scan_u64(const uint64_t *in, uint64_t n, uint64_t *out, void *ws, hipStream_t st,
                                     uint64_t *max_out) {
    if (n == 0) {
        if (max_out) {
            const hipError_t e = hipMemsetAsync(max_out, 0, sizeof(uint64_t), st);
            if (e != hipSuccess) return e;
        }
        return hipMemsetAsync(out, 0, sizeof(uint64_t), st);
    }
    const uint32_t nb = (uint32_t)((n + kScanBlock - 1) / kScanBlock);
    uint64_t *part = (uint64_t *)ws;
    if (max_out) {
        hipLaunchKernelGGL(scan_totals_kernel<true>, dim3(nb), dim3(256), 0, st, in, n, part);
        hipLaunchKernelGGL(scan_parts_kernel<true>, dim3(1), dim3(256), 0, st, part, nb, max_out);
    } else {
        hipLaunchKernelGGL(scan_totals_kernel<false>, dim3(nb), dim3(256), 0, st, in, n, part);
        hipLaunchKernelGGL(scan_parts_kernel<false>, dim3(1), dim3(256), 0, st, part, nb, nullptr);
    }
    hipLaunchKernelGGL(scan_apply_kernel, dim3(nb), dim3(256), 0, st, in, n, part, out);
    return hipGetLastError();
}

}  // namespace ompl_amd
