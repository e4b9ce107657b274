// knn_stream32.hip — exact small-batch kNN (nq < kStreamMaxQ: RRT's one nearest() per
// iteration, RRT.cpp:137 / NearestNeighborsGNAT.h:209-219) streaming the fp32 SoA rows.
//
// The fp64 stream (knn.hip knn_stream_kernel) reads 56 B per SE(3) state; this one reads the
// fp32 screening rows, 28 B per state, which is what bounds a scan of 10^7 states (280 MB,
// larger than the 256 MB Infinity Cache): HBM.  Two kernels, exact without a certificate round
// trip: the streaming kernel only screens (fp32, error bound screen_error: |d32 - d64| <= E/2) and
// writes each chunk's short candidate list; a refine block per query takes the global threshold
// and evaluates the exact fp64 distances (reference operation order, feat_dist) of the survivors.
// (Measured and rejected, DESIGN §8: refining inside the chunk before the block retires, and a
// persistent k = 1 block per range — 14.3 against 9.1 us at 10^6, 54.5 against 49 us at 10^7.)
#include "knn_fast_impl.h"

namespace ompl_amd {

namespace {

constexpr int kS32Threads = 256;
constexpr int kS32Items = 4;  // measured: 1,024 states per block (8 waves / SIMD) streams ~10 % faster at 10^7

__device__ __forceinline__ float4 load_row4(const float *p) { return *reinterpret_cast<const float4 *>(p); }

// ---- the stream kernel only screens -------------------------------------------------------
// (A block that refined its chunk in fp64 before it retired held its slot through a dependent HBM
// read of a few scattered rows with no row loads in flight.)  Per chunk of 256 * ITEMS states the
// streaming kernel writes the
// positions with d32 <= thr_c = (t_c + E(t_c))(1 + 32u) (t_c = the chunk's K-th d32; at most
// CandCap of them, a longer list is marked by its count) and records t_c (one word per chunk);
// the refine kernel reduces T = min_c t_c and takes Gthr = (T + E(T))(1 + 32u):
// T >= the store's K-th d32 (chunk c alone has K states <= t_c), so the K best exact states have
// d32 <= Gthr (the in-chunk argument, globally), and T <= t_c for every chunk, so Gthr <= thr_c
// and every state with d32 <= Gthr is in its chunk's list (an overflowed list is rescanned from
// the fp32 rows).  Exact fp64 distances of those, per refine block a top-K.
template <int K>
struct CandCap {
    static constexpr int value = 2 * K + 6;
};

template <int SP, int F, int K, int ITEMS>
__global__ __launch_bounds__(kS32Threads) void knn_stream32_screen_kernel(
    const float *__restrict__ feat32, uint64_t cap, uint64_t n_end, const double *__restrict__ qfeat, DevSpace sp,
    float absmax, float qeta, uint32_t *__restrict__ cand, float *__restrict__ cd32, uint32_t *__restrict__ ccount,
    uint32_t *__restrict__ tmin, uint32_t *__restrict__ mmin) {
    static_assert(ITEMS % 4 == 0, "float4 loads");
    constexpr int FS = Geo<SP, F>::FS;
    constexpr int NV = ITEMS / 4;
    constexpr int C = CandCap<K>::value;
    __shared__ double lds_d[4 * K];
    __shared__ uint32_t lds_i[4 * K];
    __shared__ float sh_thr;
    __shared__ uint32_t sh_n;
    const uint32_t q = blockIdx.y, P = gridDim.x;
    double qv[F];
#pragma unroll
    for (int f = 0; f < F; ++f) qv[f] = qfeat[(size_t)q * F + f];
    float q32[FS];
    if constexpr (SP == OMPL_GPU_SPACE_SE3) {
#pragma unroll
        for (int c = 0; c < 3; ++c) q32[c] = (float)qv[c];
        q32[3] = 0.f;
#pragma unroll
        for (int c = 0; c < 4; ++c) q32[4 + c] = (float)qv[3 + c];
    } else {
#pragma unroll
        for (int f = 0; f < F; ++f) q32[f] = (float)qv[f];
    }
    const float w0 = (float)sp.w0, w1 = (float)sp.w1;
    const uint64_t base = (uint64_t)blockIdx.x * (kS32Threads * ITEMS) + 4 * threadIdx.x;
    const float nan4 = __builtin_nanf("");
    float4 x[NV][F];
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const uint64_t p = base + (uint64_t)j * (4 * kS32Threads);
#pragma unroll
        for (int f = 0; f < F; ++f)
            x[j][f] = p < n_end ? load_row4(feat32 + (uint64_t)f * cap + p) : make_float4(nan4, nan4, nan4, nan4);
    }
    float d32[ITEMS];
    TopK<K> top;
    top.init();
#pragma unroll
    for (int j = 0; j < NV; ++j) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            float sv[F];
#pragma unroll
            for (int f = 0; f < F; ++f) sv[f] = u == 0 ? x[j][f].x : u == 1 ? x[j][f].y : u == 2 ? x[j][f].z : x[j][f].w;
            const float d = state_dist32<SP, F>(sv, q32, w0, w1);
            d32[j * 4 + u] = d;
            const uint32_t id = (uint32_t)(base + (uint64_t)j * (4 * kS32Threads) + u);
            if (top.admits((double)d, id)) top.push((double)d, id);
        }
    }
    double rd;
    uint32_t ri;
    block_select<K>(top, lds_d, lds_i, rd, ri);
    const uint32_t Pp = (P + 3) & ~3u;  // row stride of the per-chunk arrays
    if (threadIdx.x == 0) mmin[(size_t)q * Pp + blockIdx.x] = __float_as_uint((float)rd);  // the chunk's smallest d32
    if (threadIdx.x == K - 1) {
        const double t = rd;  // +inf: fewer than K live states, every one of them is a candidate
        double B = absmax;
        const int nc = SP == OMPL_GPU_SPACE_SE3 ? 3 : F;
        for (int c = 0; c < nc; ++c) B = fmax(B, fabs(qv[c]));
        const double E = screen_error<SP>(sp, B, t, (double)qeta + query_eta<SP>(qv));
        sh_thr = (float)((t + E) * (1.0 + 32.0 * kU) * (1.0 + 4.0 * kU));  // rounded up to fp32
        sh_n = 0;
        // t is a d32 value (exact in fp32); one word per chunk: a same-address atomicMin from
        // every block of the grid serialises at the L2 (measured 130 us against 55 us)
        tmin[(size_t)q * Pp + blockIdx.x] = __float_as_uint((float)t);
    }
    __syncthreads();
    const float thr = sh_thr;
    const size_t cb = ((size_t)q * Pp + blockIdx.x) * C;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (d32[j * 4 + u] <= thr) {  // NaN never passes
                const uint32_t slot = atomicAdd(&sh_n, 1u);
                if (slot < (uint32_t)C) {
                    cand[cb + slot] = (uint32_t)(base + (uint64_t)j * (4 * kS32Threads) + u);
                    cd32[cb + slot] = d32[j * 4 + u];
                }
            }
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) ccount[(size_t)q * Pp + blockIdx.x] = sh_n;
}

// block per query: T = min_c t_c, Gthr; only chunks whose smallest d32 is <= Gthr can hold a
// state with d32 <= Gthr (a handful of the P chunks), so the block reads 2 P words and the
// candidate slots of those chunks, refines them in fp64 and writes the query's k results
template <int SP, int F, int K, int ITEMS>
__global__ __launch_bounds__(kS32Threads) void knn_stream32_refine_kernel(
    const float *__restrict__ feat32, const double *__restrict__ feat64, uint64_t cap, uint64_t n_end,
    const double *__restrict__ qfeat, DevSpace sp, float absmax, float qeta, uint32_t P,
    const uint32_t *__restrict__ cand, const float *__restrict__ cd32, const uint32_t *__restrict__ ccount,
    const uint32_t *__restrict__ tmin, const uint32_t *__restrict__ mmin, double *__restrict__ out_d,
    uint32_t *__restrict__ out_i, uint32_t out_k) {
    constexpr int FS = Geo<SP, F>::FS;
    constexpr int C = CandCap<K>::value;
    constexpr int kMaxOver = 64;  // overflowed chunks rescanned by the whole block
    __shared__ double lds_d[4 * K];
    __shared__ uint32_t lds_i[4 * K];
    __shared__ uint32_t sh_t[kS32Threads / 64];
    __shared__ uint32_t over[kMaxOver];
    __shared__ uint32_t n_over;
    const uint32_t q = blockIdx.x;
    double qv[F];
#pragma unroll
    for (int f = 0; f < F; ++f) qv[f] = qfeat[(size_t)q * F + f];
    float q32[FS];
    if constexpr (SP == OMPL_GPU_SPACE_SE3) {
#pragma unroll
        for (int c = 0; c < 3; ++c) q32[c] = (float)qv[c];
        q32[3] = 0.f;
#pragma unroll
        for (int c = 0; c < 4; ++c) q32[4 + c] = (float)qv[3 + c];
    } else {
#pragma unroll
        for (int f = 0; f < F; ++f) q32[f] = (float)qv[f];
    }
    const float w0 = (float)sp.w0, w1 = (float)sp.w1;
    if (threadIdx.x == 0) n_over = 0;
    // T = min over the chunks' K-th screened distances (non-negative floats order as their bits);
    // the per-chunk words are read 4 at a time with the loads of several steps in flight (a
    // scalar strided loop over 10^4 words took ~25 us of one CU's load latency)
    const uint32_t Pp = (P + 3) & ~3u;  // row stride of the per-chunk arrays (16-byte aligned rows)
    const uint32_t P4 = P / 4;
    uint32_t tb = 0xFFFFFFFFu;
    {
        const uint4 *t4 = reinterpret_cast<const uint4 *>(tmin + (size_t)q * Pp);
#pragma unroll 4
        for (uint32_t i = threadIdx.x; i < P4; i += blockDim.x) {
            const uint4 v = t4[i];
            tb = min(tb, min(min(v.x, v.y), min(v.z, v.w)));
        }
        for (uint32_t c = P4 * 4 + threadIdx.x; c < P; c += blockDim.x) tb = min(tb, tmin[(size_t)q * Pp + c]);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) tb = min(tb, (uint32_t)__shfl_xor((int)tb, o));
    if ((threadIdx.x & 63) == 0) sh_t[threadIdx.x >> 6] = tb;
    __syncthreads();
    tb = sh_t[0];
#pragma unroll
    for (int w = 1; w < kS32Threads / 64; ++w) tb = min(tb, sh_t[w]);
    const double T = (double)__uint_as_float(tb);
    double B = absmax;
    const int nc = SP == OMPL_GPU_SPACE_SE3 ? 3 : F;
    for (int c = 0; c < nc; ++c) B = fmax(B, fabs(qv[c]));
    const double gthr = (T + screen_error<SP>(sp, B, T, (double)qeta + query_eta<SP>(qv))) * (1.0 + 32.0 * kU);
    TopK<K> top;
    top.init();
    auto refine = [&](uint32_t id) {
        double sv[F];
#pragma unroll
        for (int f = 0; f < F; ++f) sv[f] = feat64[(uint64_t)f * cap + id];
        top.offer(feat_dist<SP, F, 0>(sv, qv, sp), id);
    };
    auto visit = [&](uint32_t c) {  // chunk c holds a state with d32 <= Gthr
        const size_t qc = (size_t)q * Pp + c;
        const uint32_t n = ccount[qc];
        if (n > (uint32_t)C) {  // overflowed list: the block rescans the chunk below
            const uint32_t o = atomicAdd(&n_over, 1u);
            if (o < (uint32_t)kMaxOver) over[o] = c;
            return;
        }
        for (uint32_t j = 0; j < n; ++j)
            if ((double)cd32[qc * C + j] <= gthr) refine(cand[qc * C + j]);
    };
    __syncthreads();  // n_over
    {
        const uint4 *m4 = reinterpret_cast<const uint4 *>(mmin + (size_t)q * Pp);
#pragma unroll 4
        for (uint32_t i = threadIdx.x; i < P4; i += blockDim.x) {
            const uint4 v = m4[i];  // (an empty chunk: +inf, never <= Gthr)
            if ((double)__uint_as_float(v.x) <= gthr) visit(4 * i);
            if ((double)__uint_as_float(v.y) <= gthr) visit(4 * i + 1);
            if ((double)__uint_as_float(v.z) <= gthr) visit(4 * i + 2);
            if ((double)__uint_as_float(v.w) <= gthr) visit(4 * i + 3);
        }
        for (uint32_t c = P4 * 4 + threadIdx.x; c < P; c += blockDim.x)
            if ((double)__uint_as_float(mmin[(size_t)q * Pp + c]) <= gthr) visit(c);
    }
    __syncthreads();
    const uint32_t no = n_over;
    auto dist32 = [&](uint64_t p) -> float {
        float sv[F];
#pragma unroll
        for (int f = 0; f < F; ++f) sv[f] = feat32[(uint64_t)f * cap + p];
        return state_dist32<SP, F>(sv, q32, w0, w1);
    };
    if (no <= (uint32_t)kMaxOver) {
        for (uint32_t i = 0; i < no; ++i) {
            const uint64_t b0 = (uint64_t)over[i] * (kS32Threads * ITEMS), b1 = min(b0 + kS32Threads * ITEMS, n_end);
            for (uint64_t p = b0 + threadIdx.x; p < b1; p += blockDim.x)
                if ((double)dist32(p) <= gthr) refine((uint32_t)p);  // NaN never passes
        }
    } else {  // more overflowed chunks than the list holds: every chunk under Gthr is rescanned
        top.init();
        for (uint32_t c = 0; c < P; ++c) {
            if (!((double)__uint_as_float(mmin[(size_t)q * Pp + c]) <= gthr)) continue;
            const uint64_t b0 = (uint64_t)c * (kS32Threads * ITEMS), b1 = min(b0 + kS32Threads * ITEMS, n_end);
            for (uint64_t p = b0 + threadIdx.x; p < b1; p += blockDim.x)
                if ((double)dist32(p) <= gthr) refine((uint32_t)p);
        }
    }
    double rd;
    uint32_t ri;
    block_select<K>(top, lds_d, lds_i, rd, ri);
    if (threadIdx.x < out_k) {
        out_d[(size_t)q * out_k + threadIdx.x] = rd;
        out_i[(size_t)q * out_k + threadIdx.x] = ri;
    }
}




// screen + refine (HBM-sized stores); workspace: split_bytes
inline size_t split_bytes(uint32_t nq, uint32_t P, int K) {
    const size_t C = (size_t)(2 * K + 6), Pp = (P + 3) & ~3u;
    return 2 * (((size_t)nq * Pp * C * 4 + 255) / 256 * 256) + 3 * (((size_t)nq * Pp * 4 + 255) / 256 * 256);
}

template <int SP, int F, int K, int ITEMS>
hipError_t run_stream32_split(const DevSpace &sp, const float *feat32, const double *feat64, uint64_t cap,
                              uint64_t n_end, const double *qfeat, uint32_t nq, uint32_t k, float absmax, float qeta,
                              double *out_d, uint32_t *out_i, void *ws, size_t ws_bytes, hipStream_t st) {
    constexpr int C = CandCap<K>::value;
    const uint32_t P = (uint32_t)((n_end + kS32Threads * ITEMS - 1) / (kS32Threads * ITEMS));
    if (ws_bytes < split_bytes(nq, P, K)) return hipErrorInvalidValue;
    char *w = (char *)ws;
    const uint32_t Pp = (P + 3) & ~3u;
    const size_t cb = ((size_t)nq * Pp * C * 4 + 255) / 256 * 256, pb = ((size_t)nq * Pp * 4 + 255) / 256 * 256;
    uint32_t *cand = (uint32_t *)w;
    float *cd32 = (float *)(w + cb);
    uint32_t *ccount = (uint32_t *)(w + 2 * cb);
    uint32_t *tmin = (uint32_t *)(w + 2 * cb + pb);  // per (query, chunk): the chunk's K-th d32 (float bits)
    uint32_t *mmin = (uint32_t *)(w + 2 * cb + 2 * pb);  // and its smallest
    timer_begin(st, "knn_stream32_screen_kernel");
    hipLaunchKernelGGL((knn_stream32_screen_kernel<SP, F, K, ITEMS>), dim3(P, nq), dim3(kS32Threads), 0, st, feat32,
                       cap, n_end, qfeat, sp, absmax, qeta, cand, cd32, ccount, tmin, mmin);
    timer_end(st);
    hipLaunchKernelGGL((knn_stream32_refine_kernel<SP, F, K, ITEMS>), dim3(nq), dim3(kS32Threads), 0, st, feat32,
                       feat64, cap, n_end, qfeat, sp, absmax, qeta, P, cand, cd32, ccount, tmin, mmin, out_d, out_i, k);
    return hipGetLastError();
}

template <int SP, int F>
hipError_t stream32_k(const DevSpace &sp, const float *feat32, const double *feat64, uint64_t cap, uint64_t n_end,
                      const double *qfeat, uint32_t nq, uint32_t k, float absmax, float qeta, double *out_d,
                      uint32_t *out_i, void *ws, size_t ws_bytes, hipStream_t st) {
    if (k <= 1)
        return run_stream32_split<SP, F, 1, kS32Items>(sp, feat32, feat64, cap, n_end, qfeat, nq, k, absmax, qeta,
                                                        out_d, out_i, ws, ws_bytes, st);
    if (k <= 4)
        return run_stream32_split<SP, F, 4, kS32Items>(sp, feat32, feat64, cap, n_end, qfeat, nq, k, absmax, qeta,
                                                        out_d, out_i, ws, ws_bytes, st);
    return run_stream32_split<SP, F, 16, kS32Items>(sp, feat32, feat64, cap, n_end, qfeat, nq, k, absmax, qeta,
                                                     out_d, out_i, ws, ws_bytes, st);
}

}  // namespace

bool stream32_supported(const DevSpace &sp, const FeatGeom &g, uint32_t nq, uint32_t k) {
    if (nq == 0 || nq >= kStreamMaxQ || k == 0 || k > kStream32MaxK) return false;
    if (sp.kind == OMPL_GPU_SPACE_SE3) return g.F == 7;
    if (sp.kind == OMPL_GPU_SPACE_REALVECTOR) return g.F == 4 || g.F == 8 || g.F == 16;
    return false;
}

size_t stream32_workspace_bytes(uint32_t nq, uint64_t n_end) {
    const uint32_t P = (uint32_t)((n_end + kS32Threads * kS32Items - 1) / (kS32Threads * kS32Items));
    return split_bytes(nq, P, 16);
}

hipError_t launch_knn_stream32(const DevSpace &sp, const FeatGeom &g, const float *feat32, const double *feat64,
                               uint64_t cap, uint64_t n_end, const double *qfeat, uint32_t nq, uint32_t k, float absmax,
                               float qeta, double *out_d, uint32_t *out_i, void *ws, size_t ws_bytes, hipStream_t st) {
    if (!stream32_supported(sp, g, nq, k) || (cap & 3) || n_end > cap) return hipErrorInvalidValue;
    if (sp.kind == OMPL_GPU_SPACE_SE3)
        return stream32_k<OMPL_GPU_SPACE_SE3, 7>(sp, feat32, feat64, cap, n_end, qfeat, nq, k, absmax, qeta, out_d,
                                                 out_i, ws, ws_bytes, st);
    if (g.F == 4)
        return stream32_k<OMPL_GPU_SPACE_REALVECTOR, 4>(sp, feat32, feat64, cap, n_end, qfeat, nq, k, absmax, qeta,
                                                        out_d, out_i, ws, ws_bytes, st);
    if (g.F == 8)
        return stream32_k<OMPL_GPU_SPACE_REALVECTOR, 8>(sp, feat32, feat64, cap, n_end, qfeat, nq, k, absmax, qeta,
                                                        out_d, out_i, ws, ws_bytes, st);
    return stream32_k<OMPL_GPU_SPACE_REALVECTOR, 16>(sp, feat32, feat64, cap, n_end, qfeat, nq, k, absmax, qeta, out_d,
                                                     out_i, ws, ws_bytes, st);
}

}  // namespace ompl_amd
