// prm.hip — PRM*'s causal milestone insertion on the device.
//
// PRM::addMilestone (geometric/planners/prm/src/PRM.cpp:562-596) with KStarStrategy
// (ConnectionStrategy.h:124-156): milestone i is connected to its k_i = ceil((e + e/d) ln(i + 1))
// nearest among the vertices added before it — the stored states AND the milestones of the same
// batch that precede it — and every edge is checked with checkMotion(state[n], state[m]).  A batch
// is answered exactly in three parts: the stored part by the batched kNN (certified fp32 screen),
// the in-batch part by a causal scan (milestone j against milestones j' < j, fp64 in the
// reference's operation order, keeping only those within the stored list's k_j-th distance), and
// a segmented sort by (distance, id) of the union, whose first k_j entries are the answer.
#include <hip/hip_runtime.h>

#include "feat_dist.h"
#include "kernels.h"
#include "topk.h"

namespace ompl_amd {

namespace {

// stored-list bound of milestone j: its k_j-th stored neighbour's distance (+inf when the stored
// list has fewer than k_j entries)
__device__ __forceinline__ double stored_bound(const double *sd, const uint32_t *si, uint32_t kq, uint32_t kj,
                                               uint32_t j) {
    if (kj == 0) return -1.0;  // k_0 = 0: no neighbour at all (PRM.cpp:566, log(1) = 0)
    if (kj > kq) return __builtin_inf();
    const size_t o = (size_t)j * kq + kj - 1;
    return si[o] == kNoId ? __builtin_inf() : sd[o];
}

// the stored entries among row j's first min(k_j, kq): one lane (short rows: PRM*'s k <= 41) ...
__device__ __forceinline__ uint32_t stored_take_lane(const uint32_t *si, uint32_t kq, uint32_t kj, uint32_t j) {
    uint32_t c = 0;
    const uint32_t lim = kj < kq ? kj : kq;
    for (uint32_t r = 0; r < lim; ++r) c += si[(size_t)j * kq + r] != kNoId ? 1u : 0u;
    return c;
}
// ... or counted over the whole wave, every lane active (every lane gets the count; a lane walking
// RRT*'s 6,169-entry rows alone took ~0.3 ms per batch)
__device__ __forceinline__ uint32_t stored_take(const uint32_t *si, uint32_t kq, uint32_t kj, uint32_t j) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t lim = kj < kq ? kj : kq;
    uint32_t c = 0;
    for (uint32_t r = lane; r < lim; r += 64) c += si[(size_t)j * kq + r] != kNoId ? 1u : 0u;
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    return c;
}

// KinematicChain joint positions of the batch rows in fp32 (knn_fast_impl.h chain_positions: fp64
// prefix sums of the cumulative cos / sin features, then rounded), for the causal screen
template <int F>
__global__ void prm_positions_kernel(const double *__restrict__ bf, uint32_t m, float *__restrict__ p32) {
    constexpr int NM = F / 2;
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m) return;
    double cx = 0.0, cy = 0.0;
#pragma unroll
    for (int i = 0; i < NM; ++i) {
        cx += bf[(size_t)j * F + i];
        cy += bf[(size_t)j * F + NM + i];
        p32[(size_t)j * F + i] = (float)cx;
        p32[(size_t)j * F + NM + i] = (float)cy;
    }
}

// one wave per milestone j: FILL = false counts the in-batch candidates j' < j with
// d(j', j) <= bound; FILL = true writes the segment [stored entries | candidates in j' order].
// KinematicChain with p32: each pair is screened first by the fp32 joint-position distance
// link * sum_i |P_i(j') - P_i(j)| against bound + e (e: the chain screen's rounding bound,
// knn_fast_impl.h screen_error<KCHAIN>), and only the survivors — a few per milestone, against
// every earlier milestone of the batch before — take the exact fp64 distance with its 12 fp64
// square roots.  The decision is still the exact d <= bound, so the segments are unchanged.
template <int SP, int F, int NMAX, bool FILL>
__global__ __launch_bounds__(256) void prm_causal_kernel(const double *__restrict__ bf, uint32_t j0, uint32_t rows,
                                                         uint32_t n0, DevSpace sp, const uint32_t *__restrict__ kj_arr,
                                                         const double *__restrict__ sd, const uint32_t *__restrict__ si,
                                                         uint32_t kq, uint64_t *__restrict__ seg_len,
                                                         const uint64_t *__restrict__ seg_off,
                                                         double *__restrict__ out_d, uint32_t *__restrict__ out_i,
                                                         const float *__restrict__ p32,
                                                         unsigned long long *__restrict__ seg_max) {
    const uint32_t row = blockIdx.x * 4 + (threadIdx.x >> 6), j = j0 + row;  // row of this rank's slice
    const int lane = threadIdx.x & 63;
    if (row >= rows) return;
    const uint32_t kj = kj_arr[j];
    const double bound = stored_bound(sd, si, kq, kj, row);
    double qv[F];
#pragma unroll
    for (int f = 0; f < F; ++f) qv[f] = bf[(size_t)j * F + f];
    constexpr int NM = F / 2;
    float qp[SP == OMPL_GPU_SPACE_KCHAIN ? F : 1];
    float thr32 = __builtin_inff();
    if constexpr (SP == OMPL_GPU_SPACE_KCHAIN) {
        if (p32) {
#pragma unroll
            for (int f = 0; f < F; ++f) qp[f] = p32[(size_t)j * F + f];
            constexpr double u = 5.9604644775390625e-08, fmin = 1.1754943508222875e-38;
            const double n = (double)sp.dim;
            const double e = 2.0 * (sp.link * 8.0 * u * n * (n + 1.0) + (n + 2.0) * u * bound + sp.link * n * sqrt(2.0 * fmin));
            thr32 = bound < __builtin_inf() ? (float)((bound + e) * (1.0 + 16.0 * u)) : __builtin_inff();
        }
    }
    uint64_t pos = 0;
    if (FILL) {
        pos = seg_off[row];
        const uint32_t st = stored_take(si, kq, kj, row);
        for (uint32_t r = lane; r < st; r += 64) {  // stored entries first: (distance, id) sorted already
            out_d[pos + r] = sd[(size_t)row * kq + r];
            out_i[pos + r] = si[(size_t)row * kq + r];
        }
        pos += st;
    }
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    uint64_t cnt = 0;
    for (uint32_t b = 0; b < j; b += 64) {
        const uint32_t jp = b + lane;
        bool hit = false;
        double d = 0.0;
        bool cand = jp < j && bound >= 0.0;
        if constexpr (SP == OMPL_GPU_SPACE_KCHAIN) {
            if (p32 && cand) {  // fp32 screen (see above); NaN never passes
                float acc = 0.f;
#pragma unroll
                for (int i = 0; i < NM; ++i) {
                    if (i < sp.dim) {
                        const float dx = p32[(size_t)jp * F + i] - qp[i], dy = p32[(size_t)jp * F + NM + i] - qp[NM + i];
                        acc += __builtin_amdgcn_sqrtf(fmaf(dy, dy, dx * dx));
                    }
                }
                cand = acc * (float)sp.link <= thr32;
            }
        }
        if (cand) {
            double sv[F];
#pragma unroll
            for (int f = 0; f < F; ++f) sv[f] = bf[(size_t)jp * F + f];
            d = feat_dist<SP, F, NMAX>(sv, qv, sp);  // fp64, the reference's operation order
            hit = d <= bound;
        }
        const uint64_t bm = __ballot(hit);
        if (FILL && hit) {
            const uint64_t p = pos + cnt + (uint64_t)__popcll(bm & lt);
            out_d[p] = d;
            out_i[p] = n0 + jp;
        }
        cnt += (uint64_t)__popcll(bm);
    }
    if (!FILL) {
        const uint64_t len = stored_take(si, kq, kj, row) + cnt;  // wave-wide: every lane takes part
        if (lane == 0) {
            seg_len[row] = len;
            if (seg_max) atomicMax(seg_max, (unsigned long long)len);
        }
    }
}

// The KinematicChain form of the causal scan, tiled: a wave serves kCausalGroup consecutive
// milestones of the slice over one chunk of kCausalChunk earlier batch rows (grid.y), lanes
// hold 64 rows j' at a time (their fp32 joint positions, read once per tile for the whole
// group); each milestone screens the tile by the fp32 chain distance against its stored bound +
// the chain screen error, and only the survivors take the exact fp64 distance.  Counts add into
// seg_len (zeroed by the caller, the stored entries counted by chunk 0); the fill appends each
// chunk's hits at an atomic cursor per milestone, so a segment's candidates are in no particular
// order — the caller sorts every segment by (distance, id), which is the order the stable sort
// of [stored | candidates in id order] gives.  (Round 4 measured: one wave per milestone with
// the screen 1.5 ms per pass over 8,192 milestones; a wave per 4 milestones over every earlier
// row 0.55 ms, its longest waves 128 dependent tile loads; the unscreened fp64 form 0.6 ms.)
constexpr int kCausalGroup = 4;
constexpr uint32_t kCausalChunk = 1024;
template <int F, int NMAX, bool FILL>
__global__ __launch_bounds__(64) void prm_causal_tile_kernel(const double *__restrict__ bf,
                                                             const float *__restrict__ p32, uint32_t j0,
                                                             uint32_t rows, uint32_t n0, DevSpace sp,
                                                             const uint32_t *__restrict__ kj_arr,
                                                             const double *__restrict__ sd,
                                                             const uint32_t *__restrict__ si, uint32_t kq,
                                                             uint64_t *__restrict__ seg_len,
                                                             const uint64_t *__restrict__ seg_off,
                                                             double *__restrict__ out_d, uint32_t *__restrict__ out_i,
                                                             unsigned long long *__restrict__ cursor) {
    constexpr int NM = F / 2, GJ = kCausalGroup;
    static_assert(F % 4 == 0, "float4 rows");
    // the group's rows and per-milestone state live in LDS (one wave: its LDS operations complete
    // in order), read at each use: held in VGPRs for every milestone they cost ~390 registers
    __shared__ __attribute__((aligned(16))) float qp[GJ][F];
    __shared__ double qv[GJ][F];
    __shared__ double s_bound[GJ];
    __shared__ float s_thr[GJ];
    __shared__ unsigned long long s_cnt[GJ], s_pos[GJ];
    __shared__ uint32_t s_stored[GJ];
    const int lane = threadIdx.x;
    const uint32_t r0 = blockIdx.x * GJ;
    const uint32_t cb = blockIdx.y * kCausalChunk;  // this wave's rows j' in [cb, cb + kCausalChunk)
    if (r0 >= rows || cb >= j0 + min(r0 + GJ, rows) - 1 + (blockIdx.y == 0 ? 1u : 0u)) return;  // no earlier row here
    for (int t = lane; t < GJ * F; t += 64) {
        const uint32_t row = r0 + t / F;
        const bool ok = row < rows;
        qp[t / F][t % F] = ok ? p32[(size_t)(j0 + row) * F + t % F] : __builtin_nanf("");
        qv[t / F][t % F] = ok ? bf[(size_t)(j0 + row) * F + t % F] : 0.0;
    }
    if (lane < GJ) {
        const uint32_t row = r0 + lane;
        const bool ok = row < rows;
        const uint32_t kj = ok ? kj_arr[j0 + row] : 0u;
        const double bound = ok ? stored_bound(sd, si, kq, kj, row) : -1.0;
        constexpr double u = 5.9604644775390625e-08, fmin = 1.1754943508222875e-38;
        const double n = (double)sp.dim;
        const double e = 2.0 * (sp.link * 8.0 * u * n * (n + 1.0) + (n + 2.0) * u * bound + sp.link * n * sqrt(2.0 * fmin));
        s_bound[lane] = bound;
        s_thr[lane] = bound < __builtin_inf() ? (float)((bound + e) * (1.0 + 16.0 * u)) : __builtin_inff();
        s_stored[lane] = ok ? stored_take_lane(si, kq, kj, row) : 0u;
        s_cnt[lane] = 0;
        s_pos[lane] = (FILL && ok) ? seg_off[row] + s_stored[lane] : 0ull;
    }
    __syncthreads();
    if (FILL && blockIdx.y == 0) {
        for (int g = 0; g < GJ; ++g) {  // stored entries first: (distance, id) sorted already
            const uint32_t row = r0 + g;
            if (row >= rows) break;
            const uint64_t p0 = seg_off[row];
            for (uint32_t r = lane; r < s_stored[g]; r += 64) {
                out_d[p0 + r] = sd[(size_t)row * kq + r];
                out_i[p0 + r] = si[(size_t)row * kq + r];
            }
        }
    }
    const uint32_t last = min(r0 + GJ, rows);
    const uint32_t jend = min(j0 + last - 1, cb + kCausalChunk);  // rows j' < jend can precede the group
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    const float link = (float)sp.link;
    uint32_t off = 0;  // LDS row offset the compiler cannot see through (no hoisting into VGPRs)
    for (uint32_t b = cb; b < jend; b += 64) {
        const uint32_t jp = b + lane;
        float x[F];
        if (jp < jend) {
            const float4 *r4 = reinterpret_cast<const float4 *>(p32 + (size_t)jp * F);
#pragma unroll
            for (int c = 0; c < F / 4; ++c) {
                const float4 v = r4[c];
                x[4 * c] = v.x; x[4 * c + 1] = v.y; x[4 * c + 2] = v.z; x[4 * c + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int c = 0; c < F; ++c) x[c] = __builtin_nanf("");
        }
#pragma unroll 1
        for (int g = 0; g < GJ; ++g) {
            const uint32_t j = j0 + r0 + g;
            asm volatile("" : "+s"(off));
            const double bound = s_bound[g];
            if (r0 + g >= rows || b >= j || !(bound >= 0.0)) continue;  // wave-uniform
            const float *q = &qp[0][0] + off + g * F;
            float acc = 0.f;
#pragma unroll
            for (int i = 0; i < NM; ++i) {
                if (i < sp.dim) {
                    const float dx = x[i] - q[i], dy = x[NM + i] - q[NM + i];
                    acc += __builtin_amdgcn_sqrtf(fmaf(dy, dy, dx * dx));
                }
            }
            const bool cand = jp < j && acc * link <= s_thr[g];  // NaN never passes
            bool hit = false;
            double d = 0.0;
            if (__ballot(cand)) {
                if (cand) {
                    double sv[F];
#pragma unroll
                    for (int f = 0; f < F; ++f) sv[f] = bf[(size_t)jp * F + f];
                    d = feat_dist<OMPL_GPU_SPACE_KCHAIN, F, NMAX>(sv, &qv[0][0] + off + g * F, sp);  // reference order
                    hit = d <= bound;
                }
            }
            const uint64_t bm = __ballot(hit);
            if (bm) {
                if (FILL) {  // this tile's hits at the milestone's cursor (chunks append concurrently)
                    unsigned long long c = 0;
                    if (lane == 0) c = atomicAdd(&cursor[r0 + g], (unsigned long long)__popcll(bm));
                    c = (unsigned long long)__shfl((long long)c, 0);
                    if (hit) {
                        const uint64_t p = s_pos[g] + c + (uint64_t)__popcll(bm & lt);
                        out_d[p] = d;
                        out_i[p] = n0 + jp;
                    }
                } else {
                    const unsigned long long c = s_cnt[g];
                    __builtin_amdgcn_wave_barrier();
                    if (lane == 0) s_cnt[g] = c + (unsigned long long)__popcll(bm);
                    __builtin_amdgcn_wave_barrier();
                }
            }
        }
    }
    __syncthreads();
    if (!FILL && lane < GJ && r0 + lane < rows) {
        const uint64_t add = (blockIdx.y == 0 ? s_stored[lane] : 0u) + s_cnt[lane];
        if (add) atomicAdd((unsigned long long *)&seg_len[r0 + lane], (unsigned long long)add);
    }
}

// the longest segment (the sort's choice): wave max, one atomic per wave
__global__ void seg_max_kernel(const uint64_t *__restrict__ len, uint32_t rows, unsigned long long *__restrict__ mx) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long v = i < rows ? len[i] : 0ull;
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long w = (unsigned long long)__shfl_xor((long long)v, o);
        v = w > v ? w : v;
    }
    if ((threadIdx.x & 63) == 0 && v) atomicMax(mx, v);
}

// thread per (milestone, rank): the first min(k_j, segment) sorted entries
__global__ void prm_take_kernel(const uint32_t *__restrict__ sorted_i, const double *__restrict__ sorted_d,
                                const uint64_t *__restrict__ seg_off, const uint32_t *__restrict__ kj_arr, uint32_t m,
                                uint32_t k_cap, uint32_t *__restrict__ nbr, uint32_t *__restrict__ cnt,
                                double *__restrict__ dist) {  // kj_arr: this slice; dist may be NULL
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (uint64_t)m * k_cap) return;
    const uint32_t j = (uint32_t)(t / k_cap), r = (uint32_t)(t % k_cap);
    const uint64_t len = seg_off[j + 1] - seg_off[j];
    const uint32_t c = (uint32_t)min((uint64_t)kj_arr[j], len);
    nbr[t] = r < c ? sorted_i[seg_off[j] + r] : kNoId;
    if (dist) dist[t] = r < c ? sorted_d[seg_off[j] + r] : __builtin_inf();
    if (r == 0) cnt[j] = c;
}

// edge e = eoff[j] + r: checkMotion(state[nbr], state[milestone j]) (PRM.cpp:582)
__global__ void prm_edges_kernel(const uint32_t *__restrict__ nbr, const uint32_t *__restrict__ cnt,
                                 const uint64_t *__restrict__ eoff, uint32_t m, uint32_t j0, uint32_t k_cap, uint32_t n0,
                                 int dim,
                                 const double *__restrict__ stored_aos, int da, const double *__restrict__ braw,
                                 double *__restrict__ s1, double *__restrict__ s2) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (uint64_t)m * k_cap) return;
    const uint32_t j = (uint32_t)(t / k_cap), r = (uint32_t)(t % k_cap);
    if (r >= cnt[j]) return;
    const uint64_t e = eoff[j] + r;
    const uint32_t id = nbr[t];
    const double *a = id < n0 ? stored_aos + (size_t)id * da : braw + (size_t)(id - n0) * dim;
    const double *b = braw + (size_t)(j0 + j) * dim;
    for (int c = 0; c < dim; ++c) {
        s1[e * dim + c] = a[c];
        s2[e * dim + c] = b[c];
    }
}

__global__ void prm_scatter_valid_kernel(const uint8_t *__restrict__ vc, const uint32_t *__restrict__ cnt,
                                         const uint64_t *__restrict__ eoff, uint32_t m, uint32_t k_cap,
                                         uint8_t *__restrict__ valid) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (uint64_t)m * k_cap) return;
    const uint32_t j = (uint32_t)(t / k_cap), r = (uint32_t)(t % k_cap);
    valid[t] = r < cnt[j] ? vc[eoff[j] + r] : 0;
}

template <int SP, int F, int NMAX>
hipError_t run_prm_causal(const DevSpace &sp, bool fill, const double *bf, uint32_t j0, uint32_t rows, uint32_t n0,
                          const uint32_t *kj, const double *sd, const uint32_t *si, uint32_t kq, uint64_t *seg_len,
                          const uint64_t *seg_off, double *out_d, uint32_t *out_i, float *p32, uint32_t m,
                          unsigned long long *seg_max, hipStream_t st) {
    const dim3 grid((rows + 3) / 4), block(256);
    if constexpr (SP != OMPL_GPU_SPACE_KCHAIN) p32 = nullptr;
    if (p32 && !fill)  // the positions of every batch row (earlier milestones of other slices too)
        hipLaunchKernelGGL((prm_positions_kernel<F>), dim3((m + 255) / 256), dim3(256), 0, st, bf, m, p32);
    if constexpr (SP == OMPL_GPU_SPACE_KCHAIN) {
        if (p32) {
            // chunks of earlier rows: the last milestone of the slice has j0 + rows - 1 of them
            const uint32_t nc = (j0 + rows - 1 + kCausalChunk) / kCausalChunk;
            const dim3 gt((rows + kCausalGroup - 1) / kCausalGroup, nc), b64(64);
            hipError_t e;
            if (fill) {
                // the cursors live past the counts' slots: seg_max[1 .. rows] (zeroed here)
                if ((e = hipMemsetAsync(seg_max + 1, 0, sizeof(unsigned long long) * rows, st)) != hipSuccess) return e;
                hipLaunchKernelGGL((prm_causal_tile_kernel<F, NMAX, true>), gt, b64, 0, st, bf, p32, j0, rows, n0, sp,
                                   kj, sd, si, kq, seg_len, seg_off, out_d, out_i, seg_max + 1);
            } else {
                if ((e = hipMemsetAsync(seg_len, 0, sizeof(uint64_t) * rows, st)) != hipSuccess) return e;
                hipLaunchKernelGGL((prm_causal_tile_kernel<F, NMAX, false>), gt, b64, 0, st, bf, p32, j0, rows, n0, sp,
                                   kj, sd, si, kq, seg_len, seg_off, out_d, out_i, nullptr);
                hipLaunchKernelGGL(seg_max_kernel, dim3((rows + 255) / 256), dim3(256), 0, st, seg_len, rows, seg_max);
            }
            return hipGetLastError();
        }
    }
    if (fill)
        hipLaunchKernelGGL((prm_causal_kernel<SP, F, NMAX, true>), grid, block, 0, st, bf, j0, rows, n0, sp, kj, sd, si,
                           kq, seg_len, seg_off, out_d, out_i, p32, nullptr);
    else
        hipLaunchKernelGGL((prm_causal_kernel<SP, F, NMAX, false>), grid, block, 0, st, bf, j0, rows, n0, sp, kj, sd,
                           si, kq, seg_len, seg_off, out_d, out_i, p32, seg_max);
    return hipGetLastError();
}

}  // namespace

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

hipError_t launch_prm_causal(const DevSpace &sp, const FeatGeom &g, bool fill, const double *bf, uint32_t j0,
                             uint32_t rows, uint32_t n0, const uint32_t *kj, const double *sd, const uint32_t *si,
                             uint32_t kq, uint64_t *seg_len, const uint64_t *seg_off, double *out_d, uint32_t *out_i,
                             float *p32, uint32_t m, unsigned long long *seg_max, hipStream_t st) {
    if (rows == 0) return hipSuccess;
    OMPL_AMD_SPACE_DISPATCH(run_prm_causal, sp, fill, bf, j0, rows, n0, kj, sd, si, kq, seg_len, seg_off, out_d, out_i,
                            p32, m, seg_max, st)
}

hipError_t launch_prm_take(const uint32_t *sorted_i, const double *sorted_d, const uint64_t *seg_off,
                           const uint32_t *kj, uint32_t m, uint32_t k_cap, uint32_t *nbr, uint32_t *cnt, double *dist,
                           hipStream_t st) {
    const uint64_t n = (uint64_t)m * k_cap;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(prm_take_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, sorted_i, sorted_d, seg_off,
                       kj, m, k_cap, nbr, cnt, dist);
    return hipGetLastError();
}

hipError_t launch_prm_edges(const uint32_t *nbr, const uint32_t *cnt, const uint64_t *eoff, uint32_t m, uint32_t j0,
                            uint32_t k_cap, uint32_t n0, int dim, const double *stored_aos, int da, const double *braw,
                            double *s1, double *s2, hipStream_t st) {
    const uint64_t n = (uint64_t)m * k_cap;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(prm_edges_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, nbr, cnt, eoff, m, j0,
                       k_cap, n0, dim, stored_aos, da, braw, s1, s2);
    return hipGetLastError();
}

namespace {
__global__ void widen_kernel(const uint32_t *__restrict__ a, uint32_t n, uint64_t *__restrict__ b) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) b[i] = a[i];
}
}  // namespace

hipError_t launch_widen_u32(const uint32_t *a, uint32_t n, uint64_t *b, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(widen_kernel, dim3((n + 255) / 256), dim3(256), 0, st, a, n, b);
    return hipGetLastError();
}

hipError_t launch_prm_scatter_valid(const uint8_t *vc, const uint32_t *cnt, const uint64_t *eoff, uint32_t m,
                                    uint32_t k_cap, uint8_t *valid, hipStream_t st) {
    const uint64_t n = (uint64_t)m * k_cap;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(prm_scatter_valid_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, vc, cnt, eoff, m,
                       k_cap, valid);
    return hipGetLastError();
}

}  // namespace ompl_amd
