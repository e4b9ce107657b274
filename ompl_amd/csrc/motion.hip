// motion.hip — discrete motion validation and state validity for gfx950.
//
// DiscreteMotionValidator::checkMotion(s1, s2) (DiscreteMotionValidator.cpp:93-145)
// checks s2, then the interior samples j/nd, j in [1, nd-1], in FIFO-bisection order
// with early exit; s1 is assumed valid.  The result bit does not depend on the order,
// but the work does, so each thread walks the same order without a queue: the FIFO
// visits the implicit interval tree level by level, left to right, so level L is
// enumerated by the 2^L root-to-node paths and empty intervals are skipped.  The
// number of isValid() calls therefore equals the reference's exactly (counters[2]).
//
// The lastValid variant (DiscreteMotionValidator.cpp:48-91, linear sweep) is served
// by first_invalid: the first failing j in linear order, nd when only s2 fails.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <type_traits>

#include "feat_dist.h"
#include "kernels.h"
#include "topk.h"

namespace ompl_amd {

// Kernels are specialised on the space kind SP and a compile-time state width DIM (DIM = 0:
// the runtime width, up to kChainMaxLinks): device_space.h Width / fixed_space / valid_t.

template <int SP, int DIM>
__device__ __forceinline__ void motion_body(DevSpace sp_in, DevChecker ck, const double *__restrict__ s1,
                                            const double *__restrict__ s2, uint32_t m, uint8_t *__restrict__ valid,
                                            int32_t *__restrict__ nd_out, int32_t *__restrict__ fi_out,
                                            unsigned long long *__restrict__ counters, int rot) {
    const DevSpace sp = fixed_space<SP, DIM>(sp_in);
    const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
    // the runtime-width form serves the KinematicChain: its sin / cos table (glibc's, 3.5 KB) in
    // LDS, read 4 words per sin-cos pair at lane-dependent points
    constexpr bool kTab = DIM == 0;
    __shared__ double stab[kTab ? 440 : 1];
    if constexpr (kTab) {
        for (int i = threadIdx.x; i < 440; i += blockDim.x) stab[i] = gsc::kSinCosTab[i];
        __syncthreads();
    }
    const double *tab = kTab ? stab : gsc::kSinCosTab;
    bool result = true;
    uint32_t checks = 0;
    if (e < m) {
        const int dim = sp.dim;
        double a[Width<DIM>::N], b[Width<DIM>::N], t[Width<DIM>::N];
        load_state<DIM>(s1 + (size_t)e * dim, dim, a);
        load_state<DIM>(s2 + (size_t)e * dim, dim, b);
        ++checks;
        result = valid_sp<SP, DIM>(sp, ck, b, tab);  // :96 — s2 first, as the reference
        // the segment count (an arc cosine for SE3) only when something reads it: the sweep of a
        // motion whose s2 is valid, the lastValid sweep, or the caller
        const int nd = (result || nd_out || fi_out) ? (int)valid_segment_count(sp, a, b, tab) : 0;
        if (nd_out) nd_out[e] = nd;
        if (result && nd >= 2) {
            // level-order walk of the FIFO bisection :104-134
            bool any = true;
            for (int L = 0; any && result && L < 32; ++L) {
                any = false;
                const uint32_t np = 1u << L;
                for (uint32_t p = 0; p < np && result; ++p) {
                    int lo = 1, hi = nd - 1;
                    bool empty = false;
                    for (int bit = L - 1; bit >= 0; --bit) {
                        const int mid = (lo + hi) / 2;
                        if ((p >> bit) & 1u)
                            lo = mid + 1;
                        else
                            hi = mid - 1;
                        if (lo > hi) {
                            empty = true;
                            break;
                        }
                    }
                    if (empty) continue;
                    any = true;
                    const int mid = (lo + hi) / 2;
                    interpolate(sp, a, b, (double)mid / (double)nd, t, rot != 0);
                    ++checks;
                    if (!valid_sp<SP, DIM>(sp, ck, t, tab)) result = false;
                }
            }
        }
        if (valid) valid[e] = result ? 1 : 0;
        if (fi_out) {
            int fi = -1;
            if (!result) {
                // linear sweep :57-69, then s2 :73-79
                for (int j = 1; j < nd; ++j) {
                    interpolate(sp, a, b, (double)j / (double)nd, t, rot != 0);
                    if (!valid_sp<SP, DIM>(sp, ck, t, tab)) {
                        fi = j;
                        break;
                    }
                }
                if (fi < 0) fi = nd;
            }
            fi_out[e] = fi;
        }
    }
    if (counters) {
        // wave-aggregated counter updates: valid_, invalid_ (MotionValidator.h:136-139), isValid calls
        unsigned long long nv = (e < m && result) ? 1ull : 0ull;
        unsigned long long ni = (e < m && !result) ? 1ull : 0ull;
        unsigned long long nc = checks;
        for (int off = 32; off > 0; off >>= 1) {
            nv += __shfl_xor(nv, off, 64);
            ni += __shfl_xor(ni, off, 64);
            nc += __shfl_xor(nc, off, 64);
        }
        // then block-aggregated: one atomic per counter per block — same-address atomics from
        // every wave of the grid serialise at the L2 and cost more than the checks themselves
        __shared__ unsigned long long part[3][4];
        const int w = threadIdx.x >> 6;
        if ((threadIdx.x & 63) == 0) {
            part[0][w] = nv;
            part[1][w] = ni;
            part[2][w] = nc;
        }
        __syncthreads();
        if (threadIdx.x < 3) {
            unsigned long long v = 0;
            for (int i = 0; i < (int)(blockDim.x >> 6); ++i) v += part[threadIdx.x][i];
            if (v) atomicAdd(&counters[threadIdx.x], v);
        }
    }
}

// ---- sample-parallel form (the fixed-width spaces) ---------------------------------------------
// The thread-per-edge walk costs a wave the LONGEST of its 64 edges (nd varies along a vertex's
// neighbour list), and the sphere field's loop waits on a scalar load per obstacle.  Here a wave
// takes 64 edges, checks every s2 and nd lane-per-edge, then lays the interior samples of its edges
// end to end (a wave prefix sum of nd - 1) and checks them 64 at a time, lane-per-sample: the
// wave's cost is the MEAN segment count.  Every interior sample of an edge whose s2 is valid is
// checked (no early exit inside an edge), so the result bit is the reference's (valid iff s2 and
// every sample is), and the two orders of the reference are recovered exactly from the failing
// samples: the FIFO bisection (:104-134) stops at the failing sample of smallest FIFO rank — the
// isValid count is 1 + that rank + 1 (fifo_rank below) — and the linear lastValid sweep (:57-69)
// at the failing sample of smallest index.

// Number of non-empty intervals `d` levels below an interval of s indices in the FIFO bisection
// (the queue holds only non-empty intervals: `x.first < mid`, `x.second > mid`, :130-133).  An
// interval of s >= 1 indices has children of floor((s - 1) / 2) and ceil((s - 1) / 2); the sizes of
// one level take at most two consecutive values, so a level is (v, count of v, count of v + 1).
__device__ __forceinline__ uint32_t fifo_level_count(uint32_t s, int d) {
    uint32_t v = s, a = 1, b = 0;
    for (int i = 0; i < d; ++i) {
        // children: a intervals of v -> (v - 1) >> 1 and the rest; b of v + 1 -> v >> 1 and the rest
        const bool ha = v >= 1 && a, hb = b != 0;
        if (!ha && !hb) return 0;
        const uint32_t l1 = ha ? (v - 1) >> 1 : 0, h1 = ha ? v - 1 - l1 : 0;
        const uint32_t l2 = v >> 1, h2 = v - l2;
        const uint32_t nv = ha ? l1 : l2;  // l1 <= l2: the level's smaller size
        uint32_t na = 0, nb = 0;
        if (ha) {
            na += a;                                  // l1 == nv
            (h1 == nv ? na : nb) += a;
        }
        if (hb) {
            (l2 == nv ? na : nb) += b;
            (h2 == nv ? na : nb) += b;
        }
        v = nv;
        a = na;
        b = nb;
    }
    return (v >= 1 ? a : 0) + b;
}

// 0-based position of interior sample j (1 <= j <= nd - 1) in the reference's FIFO order: every
// non-empty interval of the levels above j's, plus the non-empty intervals of j's level to the left
// of it (those below the left siblings of j's right turns)
__device__ inline uint32_t fifo_rank(int j, int nd) {
    int lo = 1, hi = nd - 1, L = 0;
    for (int mid = (lo + hi) / 2; j != mid; mid = (lo + hi) / 2, ++L) {  // j's level
        if (j > mid) lo = mid + 1;
        else hi = mid - 1;
    }
    uint32_t r = 0;
    for (int d = 0; d < L; ++d) r += fifo_level_count((uint32_t)(nd - 1), d);
    lo = 1;
    hi = nd - 1;
    for (int d = 0; d < L; ++d) {  // again, adding the left siblings' intervals at j's level
        const int mid = (lo + hi) / 2;
        if (j > mid) {
            r += fifo_level_count((uint32_t)(mid - lo), L - d - 1);
            lo = mid + 1;
        } else {
            hi = mid - 1;
        }
    }
    return r;
}

// Sphere field on packed fp32, certified.  The reference test is fp64: dx*dx + dy*dy + dz*dz < r^2
// with dx = c_x - s_x (device_space.h spheres_valid).  Here a pair of spheres is screened per packed
// instruction from fp32 copies in LDS: c32 = fl32(c), r_hi = fl32(r^2 (1 + 2^-21)) >= r^2, s32 =
// fl32(s).  With u = 2^-24 and B >= |c_i| + |s_i| for every coordinate, each fp32 difference is
// within 2.01 u B of the exact one, so the fp32 sum of squares (one rounded product, two fmas) is
// within 3.01 u 3 B^2 + 3 (2 B 2.01 u B + (2.01 u B)^2) <= 21.2 u B^2 of the exact sum, which the
// fp64 sum matches to 4e-16 relative: g = fl32(D32 - r_hi) > E = 48 u B^2 proves D64 >= r^2 — the
// sphere does not contain s.  When every sphere's g clears E the state is valid; otherwise (a
// state inside or within E of a sphere) the exact fp64 test decides.  NaN / huge states fail the
// screen (NaN or infinite E) and take the fp64 test too.
constexpr int kLdsSpheres = 128;  // spheres staged in LDS (more: the fp64 test alone)
struct SphereScreen {
    float4 c[kLdsSpheres / 2][2];  // pair p: {cx_0, cx_1, cy_0, cy_1}, {cz_0, cz_1, rhi_0, rhi_1}
    float mc;                      // >= every |centre coordinate| (rounded up)
};

__device__ __forceinline__ void stage_spheres(SphereScreen &ss, const double *__restrict__ c, int count) {
    unsigned int *mcb = reinterpret_cast<unsigned int *>(&ss.mc);
    if (threadIdx.x == 0) *mcb = 0u;
    __syncthreads();
    float mloc = 0.f;
    for (int i = threadIdx.x; i < kLdsSpheres; i += blockDim.x) {
        float x = 0.f, y = 0.f, z = 0.f, rh = -__builtin_inff();  // padding: never contains a state
        if (i < count) {
            x = (float)c[4 * i];
            y = (float)c[4 * i + 1];
            z = (float)c[4 * i + 2];
            rh = (float)(c[4 * i + 3] * (1.0 + 0x1p-21));
            mloc = fmaxf(mloc, fmaxf(fabsf(x), fmaxf(fabsf(y), fabsf(z))));
        }
        float *q = reinterpret_cast<float *>(&ss.c[i >> 1][0]);
        const int h = i & 1;
        q[0 + h] = x;
        q[2 + h] = y;
        q[4 + h] = z;
        q[6 + h] = rh;
    }
    // |c| <= fl32(|c|) (1 + u): round the bound up by 2^-20 (non-negative floats order as integers)
    atomicMax(mcb, __float_as_uint(mloc * (1.f + 0x1p-20f)));
    __syncthreads();
}

// false: some sphere may contain s (the caller runs the exact test); true: no sphere contains s
__device__ __forceinline__ bool spheres_clear32(const double *s, const SphereScreen &ss, int count) {
    const float x = (float)s[0], y = (float)s[1], z = (float)s[2];
    const float b = (ss.mc + fmaxf(fabsf(x), fmaxf(fabsf(y), fabsf(z)))) * (1.f + 0x1p-20f);
    const float E = 48.f * 0x1p-24f * b * b;
    const f2 nx = f2{-x, -x}, ny = f2{-y, -y}, nz = f2{-z, -z};
    float gmin = __builtin_inff();
#pragma unroll 2
    for (int p = 0; p < (count + 1) >> 1; ++p) {
        const float4 a = ss.c[p][0], q = ss.c[p][1];
        const f2 dx = f2{a.x, a.y} + nx, dy = f2{a.z, a.w} + ny, dz = f2{q.x, q.y} + nz;
        f2 d2 = dx * dx;
        d2 = pk_fma(dy, dy, d2);
        d2 = pk_fma(dz, dz, d2);
        const f2 g = d2 - f2{q.z, q.w};
        gmin = fminf(gmin, fminf(g.x, g.y));  // (a NaN g is dropped: the fp64 test of a NaN state passes too)
    }
    return gmin > E;
}

// Endpoint sources of the sample-parallel kernel.  PairSrc: the caller's rows s1[e], s2[e]
// (ompl_gpu_mv_check_device).  EdgeSrc: the edges of a neighbour query read where they live —
// the query row and the stored state's AoS row by id (ompl_gpu_mv_check_edges_device), the pairs
// edges_copy_kernel would have materialised: a missing neighbour (kNoId) is the zero-length motion
// from the query to itself; an edge past the last CSR segment does not exist.
struct PairSrc {
    const double *s1, *s2;
    template <int DIM>
    __device__ __forceinline__ bool load(uint32_t e, double (&a)[DIM], double (&b)[DIM]) const {
        load_state<DIM>(s1 + (size_t)e * DIM, DIM, a);
        load_state<DIM>(s2 + (size_t)e * DIM, DIM, b);
        return true;
    }
};
struct EdgeSrc {
    const double *q;       // [nq][DIM] query rows
    const uint32_t *qidx;  // CSR: the query of each edge (kNoId past the last segment); null: e / stride
    const uint32_t *ids;   // [m] neighbour ids (kNoId: none)
    uint32_t stride;
    int from_query;        // 1: checkMotion(query, neighbour), 0: checkMotion(neighbour, query)
    const double *aos;     // stored states by id, rows of da reals
    int da;
    template <int DIM>
    __device__ __forceinline__ bool load(uint32_t e, double (&a)[DIM], double (&b)[DIM]) const {
        const uint32_t qi = qidx ? qidx[e] : e / stride;
        if (qi == kNoId) return false;
        const uint32_t id = ids[e];
        const double *qr = q + (size_t)qi * DIM, *sr = id == kNoId ? qr : aos + (size_t)id * da;
        load_state<DIM>(from_query ? qr : sr, DIM, a);
        load_state<DIM>(from_query ? sr : qr, DIM, b);
        return true;
    }
};

// ROT: the interpolation's SO3 part (false when the checker reads only the SE3 translation)
template <int SP, int DIM, bool ROT, class Src>
__global__ __launch_bounds__(256) __attribute__((flatten)) void motion_kernel(
    DevSpace sp_in, DevChecker ck, Src src, uint32_t m, uint8_t *__restrict__ valid, int32_t *__restrict__ nd_out,
    int32_t *__restrict__ fi_out, unsigned long long *__restrict__ counters) {
    static_assert(DIM > 0, "the sample-parallel form holds states in registers");
    const DevSpace sp = fixed_space<SP, DIM>(sp_in);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t wbase = blockIdx.x * blockDim.x + (uint32_t)w * 64, e = wbase + lane;
    __shared__ int s_off[4][64], s_nd[4][64], s_fj[4][64], s_fr[4][64];
    // the sphere field's screen (the SE3 translation / the first three reals)
    constexpr bool kSph = (SP == OMPL_GPU_SPACE_SE3 || SP == OMPL_GPU_SPACE_REALVECTOR) && DIM >= 3;
    __shared__ SphereScreen ss;
    const bool sph = kSph && ck.kind == OMPL_GPU_CHECK_SPHERES && ck.count <= kLdsSpheres;
    if (sph) stage_spheres(ss, ck.data, ck.count);
    bool s2ok = false, has = false;
    int nd = 0;
    double a[DIM], b[DIM];
    if (e < m) has = src.template load<DIM>(e, a, b);
    if (has) {
        s2ok = valid_sp<SP, DIM>(sp, ck, b);  // :96 — s2 first, as the reference
        nd = (s2ok || nd_out || fi_out) ? (int)valid_segment_count(sp, a, b, gsc::kSinCosTab) : 0;
        if (nd_out) nd_out[e] = nd;
    }
    // the coordinates the samples need (the SE3 translation alone when the checker reads only it),
    // kept per wave in LDS: the sample lanes read their edge's endpoints from there, not again from
    // the rows (for EdgeSrc, a query row and a stored row by id)
    constexpr int NL = (SP == OMPL_GPU_SPACE_SE3 && !ROT) ? 3 : DIM;
    __shared__ double s_ab[4][2][NL][64];
#pragma unroll
    for (int c = 0; c < NL; ++c) {
        s_ab[w][0][c][lane] = a[c];
        s_ab[w][1][c][lane] = b[c];
    }
    // interior samples this edge contributes: the FIFO walk's (s2 valid), or the lastValid sweep's
    const int cnt = (has && nd >= 2 && (s2ok || fi_out)) ? nd - 1 : 0;
    int inc = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(inc, o, 64);
        if (lane >= o) inc += v;
    }
    const int total = __shfl(inc, 63, 64);
    s_off[w][lane] = inc - cnt;
    s_nd[w][lane] = nd;
    s_fj[w][lane] = 0x7FFFFFFF;
    s_fr[w][lane] = 0x7FFFFFFF;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    for (int k0 = 0; k0 < total; k0 += 64) {
        const int k = k0 + lane;
        if (k < total) {
            int i = 0;  // the last edge whose samples start at or before k (edges with none share it)
#pragma unroll
            for (int step = 32; step; step >>= 1)
                if (s_off[w][i + step] <= k) i += step;
            const int ndi = s_nd[w][i], j = k - s_off[w][i] + 1;
            double a[DIM], b[DIM], t[DIM];
#pragma unroll
            for (int c = 0; c < NL; ++c) {
                a[c] = s_ab[w][0][c][i];
                b[c] = s_ab[w][1][c][i];
            }
            interpolate(sp, a, b, (double)j / (double)ndi, t, ROT);  // (reads coordinates < NL only)
            if (!(sph && spheres_clear32(t, ss, ck.count)) && !valid_sp<SP, DIM>(sp, ck, t)) {
                atomicMin(&s_fj[w][i], j);
                if (counters) atomicMin(&s_fr[w][i], (int)fifo_rank(j, ndi));
            }
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const int fj = s_fj[w][lane], fr = s_fr[w][lane];
    const bool result = s2ok && fj == 0x7FFFFFFF;
    if (e < m) {  // (an edge that does not exist reports invalid and is not counted)
        if (valid) valid[e] = result ? 1 : 0;
        if (fi_out) fi_out[e] = result ? -1 : (fj != 0x7FFFFFFF ? fj : nd);
    }
    if (counters) {
        unsigned long long nv = (has && result) ? 1ull : 0ull;
        unsigned long long ni = (has && !result) ? 1ull : 0ull;
        // isValid calls of the FIFO form: s2, then every interior sample, or up to the failing one
        unsigned long long nc = has ? 1ull + (s2ok ? (fj == 0x7FFFFFFF ? (unsigned)cnt : (unsigned)fr + 1u) : 0u) : 0ull;
        for (int off = 32; off > 0; off >>= 1) {
            nv += __shfl_xor(nv, off, 64);
            ni += __shfl_xor(ni, off, 64);
            nc += __shfl_xor(nc, off, 64);
        }
        __shared__ unsigned long long part[3][4];
        if (lane == 0) {
            part[0][w] = nv;
            part[1][w] = ni;
            part[2][w] = nc;
        }
        __syncthreads();
        if (threadIdx.x < 3) {
            unsigned long long v = 0;
            for (int q = 0; q < (int)(blockDim.x >> 6); ++q) v += part[threadIdx.x][q];
            if (v) atomicAdd(&counters[threadIdx.x], v);
        }
    }
}

// the runtime-width form (the KinematicChain's): held to 64 VGPRs for 8 waves per SIMD — its fp64
// sin / cos chains and segment tests wait on their own latencies at the 2 waves its natural 194
// VGPRs allow (measured per cfg4 batch of motion checks: 2 / 4 / 5 / 6 / 8 waves 1.55 / 1.18 /
// 1.17 / 1.09 / 1.07 ms; the scratch it spills to stays in the L1 / L2)
__global__ __launch_bounds__(256) __attribute__((flatten, amdgpu_waves_per_eu(8, 8))) void motion_rt_kernel(
    DevSpace sp_in, DevChecker ck, const double *__restrict__ s1, const double *__restrict__ s2, uint32_t m,
    uint8_t *__restrict__ valid, int32_t *__restrict__ nd_out, int32_t *__restrict__ fi_out,
    unsigned long long *__restrict__ counters, int rot) {
    motion_body<0, 0>(sp_in, ck, s1, s2, m, valid, nd_out, fi_out, counters, rot);
}

// KinematicChain space + KinematicChain checker (the PRM* workload): motion_body's walk with the
// link endpoints in registers (chain_valid_np, NP >= dim + 2 points) and no state arrays — the
// endpoints are read from the edge's rows and every sample's angles are interpolated on the fly in
// chain_interp's arithmetic.  Same order of checks, same counts, same results as motion_body.
// held to 4 waves per SIMD (128 VGPRs, 64 B of spills); measured per cfg4 batch of motion checks:
// 2 / 4 / 5 waves 0.80 / 0.63 / 1.37 ms (the runtime form: 1.06 ms; with the side pre-test 1.08 —
// its state arrays in scratch were the cost); one check site instead of three: 0.70 ms
template <int NP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 4))) void motion_chain_kernel(DevSpace sp, DevChecker ck, const double *__restrict__ s1,
                                                           const double *__restrict__ s2, uint32_t m,
                                                           uint8_t *__restrict__ valid, int32_t *__restrict__ nd_out,
                                                           int32_t *__restrict__ fi_out,
                                                           unsigned long long *__restrict__ counters) {
    const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
    __shared__ double tab[440];  // glibc's sin / cos table, read at lane-dependent points
    for (int i = threadIdx.x; i < 440; i += blockDim.x) tab[i] = gsc::kSinCosTab[i];
    __syncthreads();
    bool result = true;
    uint32_t checks = 0;
    if (e < m) {
        const int n = sp.dim;
        const double *a = s1 + (size_t)e * n, *b = s2 + (size_t)e * n;
        ++checks;
        result = chain_valid_np<NP>([&](int i) { return b[i]; }, n, sp.link, ck.data, ck.count, ck.slack, tab);
        const int nd = (result || nd_out || fi_out)
                           ? (int)seg_count(chain_dist_raw(a, b, n, sp.link, tab), sp.lvs0, sp.f0)
                           : 0;
        if (nd_out) nd_out[e] = nd;
        auto sample_valid = [&](int j) {
            const double t = (double)j / (double)nd;
            return chain_valid_np<NP>([&](int i) { return chain_interp1(a[i], b[i], t); }, n, sp.link, ck.data,
                                      ck.count, ck.slack, tab);
        };
        if (result && nd >= 2) {  // level-order walk of the FIFO bisection (motion_body)
            bool any = true;
            for (int L = 0; any && result && L < 32; ++L) {
                any = false;
                const uint32_t np = 1u << L;
                for (uint32_t p = 0; p < np && result; ++p) {
                    int lo = 1, hi = nd - 1;
                    bool empty = false;
                    for (int bit = L - 1; bit >= 0; --bit) {
                        const int mid = (lo + hi) / 2;
                        if ((p >> bit) & 1u)
                            lo = mid + 1;
                        else
                            hi = mid - 1;
                        if (lo > hi) {
                            empty = true;
                            break;
                        }
                    }
                    if (empty) continue;
                    any = true;
                    ++checks;
                    if (!sample_valid((lo + hi) / 2)) result = false;
                }
            }
        }
        if (valid) valid[e] = result ? 1 : 0;
        if (fi_out) {
            int fi = -1;
            if (!result) {
                for (int j = 1; j < nd; ++j)
                    if (!sample_valid(j)) {
                        fi = j;
                        break;
                    }
                if (fi < 0) fi = nd;
            }
            fi_out[e] = fi;
        }
    }
    if (counters) {
        unsigned long long nv = (e < m && result) ? 1ull : 0ull;
        unsigned long long ni = (e < m && !result) ? 1ull : 0ull;
        unsigned long long nc = checks;
        for (int off = 32; off > 0; off >>= 1) {
            nv += __shfl_xor(nv, off, 64);
            ni += __shfl_xor(ni, off, 64);
            nc += __shfl_xor(nc, off, 64);
        }
        __shared__ unsigned long long part[3][4];
        const int w = threadIdx.x >> 6;
        if ((threadIdx.x & 63) == 0) {
            part[0][w] = nv;
            part[1][w] = ni;
            part[2][w] = nc;
        }
        __syncthreads();
        if (threadIdx.x < 3) {
            unsigned long long v = 0;
            for (int i = 0; i < (int)(blockDim.x >> 6); ++i) v += part[threadIdx.x][i];
            if (v) atomicAdd(&counters[threadIdx.x], v);
        }
    }
}

// (Measured and rejected: the KinematicChain motion as a compacted FIFO walk — a wave handing its
// lanes the next pending (FIFO rank, edge) samples of its 64 edges, every rank below an edge's first
// failure checked first, so bits and counts stay exact — 862 us per cfg4 batch against 622 us for
// motion_chain_kernel: about half of PRM*'s edges fail early, which the thread-per-edge walk leaves
// at once, and the rank-to-sample mapping and extra in-round checks cost more than the balance gains.)

template <int NP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 4))) void state_chain_kernel(DevSpace sp, DevChecker ck, const double *__restrict__ s,
                                                          uint32_t m, uint8_t *__restrict__ valid) {
    __shared__ double tab[440];
    for (int i = threadIdx.x; i < 440; i += blockDim.x) tab[i] = gsc::kSinCosTab[i];
    __syncthreads();
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const double *x = s + (size_t)i * sp.dim;
    valid[i] = chain_valid_np<NP>([&](int j) { return x[j]; }, sp.dim, sp.link, ck.data, ck.count, ck.slack, tab)
                   ? 1
                   : 0;
}

// the register forms' point counts: 14 (up to 12 links, the PRM* benchmark's chain) and 18 (16)
static int chain_np(const DevSpace &sp, const DevChecker &ck) {
    if (sp.kind != OMPL_GPU_SPACE_KCHAIN || ck.kind != OMPL_GPU_CHECK_KCHAIN) return 0;
    return sp.dim <= 12 ? 14 : (sp.dim <= 16 ? 18 : 0);
}

template <int SP, int DIM>
__global__ __launch_bounds__(256) __attribute__((flatten)) void state_valid_kernel(
    DevSpace sp_in, DevChecker ck, const double *__restrict__ s, uint32_t m, uint8_t *__restrict__ valid) {
    const DevSpace sp = fixed_space<SP, DIM>(sp_in);
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    double a[Width<DIM>::N];
    load_state<DIM>(s + (size_t)i * sp.dim, sp.dim, a);
    valid[i] = valid_sp<SP, DIM>(sp, ck, a) ? 1 : 0;
}

// the specialisations: SE3 (7 reals), SO3 (4), R^2 / R^3 / R^6 (the closed checker set's
// spaces); everything else (other R^n, KinematicChain) takes the runtime-width form.  A
// hypercube over more coordinates than the fixed width, and the KinematicChain checker, never
// take a fixed form.
template <class F>
static hipError_t dispatch_width(const DevSpace &sp, const DevChecker &ck, F &&launch) {
    const bool fixed_ok = (ck.kind == OMPL_GPU_CHECK_ALL_VALID || ck.kind == OMPL_GPU_CHECK_SPHERES ||
                           ck.kind == OMPL_GPU_CHECK_CIRCLES2D ||
                           (ck.kind == OMPL_GPU_CHECK_HYPERCUBE && ck.ndim <= sp.dim));
    // the KinematicChain checker takes the runtime-width form (motion_rt_kernel).  (Measured and
    // rejected for the 12-link chain, DESIGN §8: the pair loops fully unrolled — 290 VGPRs, 2.49 ms
    // per cfg4 batch of motion checks; the positions in VGPRs indexed by the loop counters — 189
    // VGPRs, 1.27 ms at 2 waves per SIMD, 1.04 at 4, 3.39 at 6 (spills); edges walked in order of
    // their segment counts — 0.95 ms for the walk but the ordering's atomics cost more; against
    // the runtime form's 1.06 ms at 8 waves.)
    if (fixed_ok) {
        if (sp.kind == OMPL_GPU_SPACE_SE3 && sp.dim == 7) return launch(std::integral_constant<int, OMPL_GPU_SPACE_SE3>{}, std::integral_constant<int, 7>{});
        if (sp.kind == OMPL_GPU_SPACE_SO3 && sp.dim == 4) return launch(std::integral_constant<int, OMPL_GPU_SPACE_SO3>{}, std::integral_constant<int, 4>{});
        if (sp.kind == OMPL_GPU_SPACE_REALVECTOR) {
            switch (sp.dim) {
            case 2: return launch(std::integral_constant<int, OMPL_GPU_SPACE_REALVECTOR>{}, std::integral_constant<int, 2>{});
            case 3: return launch(std::integral_constant<int, OMPL_GPU_SPACE_REALVECTOR>{}, std::integral_constant<int, 3>{});
            case 6: return launch(std::integral_constant<int, OMPL_GPU_SPACE_REALVECTOR>{}, std::integral_constant<int, 6>{});
            default: break;
            }
        }
    }
    return launch(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{});
}

// (Measured and rejected, DESIGN §8: a wave per chain state check — lane per link, positions in
// LDS, the segment tests over the lanes — 1.88 ms per cfg4 batch of motion checks against 1.17 ms
// for the thread-per-edge form, which leaves at its first intersection.)

static bool needs_rotation(const DevSpace &sp, const DevChecker &ck) {
    if (sp.kind != OMPL_GPU_SPACE_SE3) return true;
    switch (ck.kind) {
    case OMPL_GPU_CHECK_ALL_VALID: return false;
    case OMPL_GPU_CHECK_HYPERCUBE: return ck.ndim > 3;
    case OMPL_GPU_CHECK_SPHERES: return false;
    case OMPL_GPU_CHECK_CIRCLES2D: return false;
    default: return true;
    }
}

hipError_t launch_motion(const DevSpace &sp, const DevChecker &ck, const double *s1, const double *s2, uint32_t m,
                         uint8_t *valid, int32_t *nd, int32_t *first_invalid, unsigned long long *counters,
                         hipStream_t st) {
    if (m == 0) return hipSuccess;
    switch (chain_np(sp, ck)) {
    case 14:
        hipLaunchKernelGGL(motion_chain_kernel<14>, dim3((m + 255) / 256), dim3(256), 0, st, sp, ck, s1, s2, m, valid,
                           nd, first_invalid, counters);
        return hipGetLastError();
    case 18:
        hipLaunchKernelGGL(motion_chain_kernel<18>, dim3((m + 255) / 256), dim3(256), 0, st, sp, ck, s1, s2, m, valid,
                           nd, first_invalid, counters);
        return hipGetLastError();
    default: break;
    }
    const int rot = needs_rotation(sp, ck) ? 1 : 0;
    return dispatch_width(sp, ck, [&](auto kind, auto width) {
        if constexpr (decltype(width)::value == 0)
            hipLaunchKernelGGL(motion_rt_kernel, dim3((m + 255) / 256), dim3(256), 0, st, sp, ck, s1, s2, m, valid, nd,
                               first_invalid, counters, rot);
        else if (rot)
            hipLaunchKernelGGL((motion_kernel<decltype(kind)::value, decltype(width)::value, true, PairSrc>),
                               dim3((m + 255) / 256), dim3(256), 0, st, sp, ck, PairSrc{s1, s2}, m, valid, nd,
                               first_invalid, counters);
        else
            hipLaunchKernelGGL((motion_kernel<decltype(kind)::value, decltype(width)::value, false, PairSrc>),
                               dim3((m + 255) / 256), dim3(256), 0, st, sp, ck, PairSrc{s1, s2}, m, valid, nd,
                               first_invalid, counters);
        return hipGetLastError();
    });
}

// the edges of a neighbour query checked in place (EdgeSrc); hipErrorNotSupported when the space /
// checker has no fixed-width form (the caller materialises the pairs and calls launch_motion)
hipError_t launch_motion_edges(const DevSpace &sp, const DevChecker &ck, const double *q, const uint32_t *qidx,
                               const uint32_t *ids, uint32_t stride, int from_query, const double *aos, int da,
                               uint32_t m, uint8_t *valid, unsigned long long *counters, hipStream_t st) {
    if (m == 0) return hipSuccess;
    if (chain_np(sp, ck)) return hipErrorNotSupported;
    const EdgeSrc src{q, qidx, ids, stride, from_query, aos, da};
    const int rot = needs_rotation(sp, ck) ? 1 : 0;
    return dispatch_width(sp, ck, [&](auto kind, auto width) {
        if constexpr (decltype(width)::value == 0) {
            return hipErrorNotSupported;
        } else {
            if (rot)
                hipLaunchKernelGGL((motion_kernel<decltype(kind)::value, decltype(width)::value, true, EdgeSrc>),
                                   dim3((m + 255) / 256), dim3(256), 0, st, sp, ck, src, m, valid, nullptr, nullptr,
                                   counters);
            else
                hipLaunchKernelGGL((motion_kernel<decltype(kind)::value, decltype(width)::value, false, EdgeSrc>),
                                   dim3((m + 255) / 256), dim3(256), 0, st, sp, ck, src, m, valid, nullptr, nullptr,
                                   counters);
            return hipGetLastError();
        }
    });
}

// SpaceInformation::getMotionStates (SpaceInformation.cpp:201-275, alloc = true): thread per
// (motion, output slot); slot k of a motion is s1 (k = 0 with endpoints), s2 (last slot with
// endpoints), else the interior sample j = k (+1 without endpoints) at t = j / (count + 1)
__global__ __launch_bounds__(256) void motion_states_kernel(DevSpace sp, const double *__restrict__ s1,
                                                            const double *__restrict__ s2, uint32_t m, uint32_t count,
                                                            int endpoints, uint32_t per, double *__restrict__ out) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (uint64_t)m * per) return;
    const uint32_t e = (uint32_t)(t / per), k = (uint32_t)(t % per);
    const int dim = sp.dim;
    double *o = out + t * dim;
    const double *a = s1 + (size_t)e * dim, *b = s2 + (size_t)e * dim;
    if (endpoints && k == 0) {
        for (int c = 0; c < dim; ++c) o[c] = a[c];
        return;
    }
    if (endpoints && k == per - 1) {
        for (int c = 0; c < dim; ++c) o[c] = b[c];
        return;
    }
    const uint32_t j = endpoints ? k : k + 1;
    double x[kChainMaxLinks], y[kChainMaxLinks], r[kChainMaxLinks];
    load_state<0>(a, dim, x);
    load_state<0>(b, dim, y);
    interpolate(sp, x, y, (double)j / (double)(count + 1), r);
    for (int c = 0; c < dim; ++c) o[c] = r[c];
}

hipError_t launch_motion_states(const DevSpace &sp, const double *s1, const double *s2, uint32_t m, uint32_t count,
                                int endpoints, double *out, hipStream_t st) {
    const uint32_t per = (uint32_t)motion_states_per(count, endpoints);  // count <= UINT32_MAX - 2 (capi)
    const uint64_t n = (uint64_t)m * per;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(motion_states_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, sp, s1, s2, m, count,
                       endpoints, per, out);
    return hipGetLastError();
}

// StateSpace::distance / StateSpace::interpolate per pair (the reference's virtuals:
// RealVectorStateSpace.cpp:230-265, SO3StateSpace.cpp:254-318, StateSpace.cpp:1068-1116,
// KinematicChain.h:105-175) with the device fp64 code the kernels use: thread per pair; t per pair
// (interpolate) or NULL (distance -> out[m]).  Not a hot path: the state-space known-answer tests
// (tests/base/StateSpaceTest.h) and planners that need single distances on device data.
__global__ __launch_bounds__(256) void space_pairs_kernel(DevSpace sp, const double *__restrict__ a,
                                                          const double *__restrict__ b, const double *__restrict__ t,
                                                          uint32_t m, double *__restrict__ out) {
    const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= m) return;
    const int dim = sp.dim;
    double x[kChainMaxLinks], y[kChainMaxLinks], r[kChainMaxLinks];
    load_state<0>(a + (size_t)e * dim, dim, x);
    load_state<0>(b + (size_t)e * dim, dim, y);
    if (!t) {
        out[e] = raw_distance(sp, x, y);
        return;
    }
    interpolate(sp, x, y, t[e], r);
    for (int c = 0; c < dim; ++c) out[(size_t)e * dim + c] = r[c];
}

hipError_t launch_space_pairs(const DevSpace &sp, const double *a, const double *b, const double *t, uint32_t m,
                              double *out, hipStream_t st) {
    if (m == 0) return hipSuccess;
    hipLaunchKernelGGL(space_pairs_kernel, dim3((m + 255) / 256), dim3(256), 0, st, sp, a, b, t, m, out);
    return hipGetLastError();
}

hipError_t launch_state_valid(const DevSpace &sp, const DevChecker &ck, const double *s, uint32_t m, uint8_t *valid,
                              hipStream_t st) {
    if (m == 0) return hipSuccess;
    switch (chain_np(sp, ck)) {
    case 14:
        hipLaunchKernelGGL(state_chain_kernel<14>, dim3((m + 255) / 256), dim3(256), 0, st, sp, ck, s, m, valid);
        return hipGetLastError();
    case 18:
        hipLaunchKernelGGL(state_chain_kernel<18>, dim3((m + 255) / 256), dim3(256), 0, st, sp, ck, s, m, valid);
        return hipGetLastError();
    default: break;
    }
    return dispatch_width(sp, ck, [&](auto kind, auto width) {
        hipLaunchKernelGGL((state_valid_kernel<decltype(kind)::value, decltype(width)::value>), dim3((m + 255) / 256),
                           dim3(256), 0, st, sp, ck, s, m, valid);
        return hipGetLastError();
    });
}

}  // namespace ompl_amd
