// knn_stream32.hip — exact small-batch kNN (nq < kStreamMaxQ: RRT's one nearest() per
// iteration, RRT.cpp:137 / NearestNeighborsGNAT.h:209-219) streaming the fp32 SoA rows.
//
// The fp64 stream (knn.hip knn_stream_kernel) reads 56 B per SE(3) state; this one reads the
// fp32 screening rows, 28 B per state, which is what bounds a scan of 10^7 states (280 MB,
// larger than the 256 MB Infinity Cache): HBM.  Exactness without a certificate round trip:
// a block owns a contiguous chunk of 256 * ITEMS states; it
//   1. screens the chunk in fp32 (state_dist32, error bound screen_error: |d32 - d64| <= E/2),
//      keeping the distances in registers, and finds t = the chunk's K-th smallest d32;
//   2. evaluates the exact fp64 distance (reference operation order, feat_dist) of every state
//      of the chunk with d32 <= thr = (t + E)(1 + 32u), reading its fp64 row (a handful per
//      chunk), and keeps the chunk's exact top-K by (distance, id).
// A state with d32 > thr has d64 > t + E/2 >= the d64 of each of the K states with d32 <= t,
// so it is not among the chunk's K best: the chunk's list is exact, and the merge of all
// chunks' lists (knn_stream32_merge_kernel) is the exact top-K of the store.
#include "knn_fast_impl.h"

namespace ompl_amd {

namespace {

constexpr int kS32Threads = 256;
// knn_stream1_kernel blocks over the batch; OMPL_GPU_S1_BLOCKS overrides (A/B), 0 selects the
// chunked form for k = 1 too
// the split (screen-only stream + refine) form from 4 M states up; OMPL_GPU_STREAM_SPLIT=0: the
// in-chunk refinement form (A/B)
inline bool stream_split() {
    static const bool b = [] {
        const char *v = std::getenv("OMPL_GPU_STREAM_SPLIT");
        return v ? std::atoi(v) != 0 : true;
    }();
    return b;
}
// smallest store the split form serves (OMPL_GPU_SPLIT_MIN overrides).  Measured at 10^6 (k = 1,
// Infinity-Cache resident): split 9.1 us / 5.6e4 queries/s against the persistent
// knn_stream1_kernel's 14.3 us / 4.7e4; at 10^7 49 us / 1.6e4 against 54.5 us / 1.37e4
inline uint64_t stream_split_min() {
    static const uint64_t m = [] {
        const char *v = std::getenv("OMPL_GPU_SPLIT_MIN");
        return v ? (uint64_t)std::atoll(v) : 0ull;
    }();
    return m;
}
inline uint32_t stream1_blocks() {
    static const uint32_t b = [] {
        const char *v = std::getenv("OMPL_GPU_S1_BLOCKS");
        return v ? (uint32_t)std::atoi(v) : 2048u;
    }();
    return b;
}

#if defined(OMPL_AMD_VARIANT) && (OMPL_AMD_VARIANT == 1 || OMPL_AMD_VARIANT == 3)
__device__ __forceinline__ float4 load_row4(const float *p) {  // A/B build: non-temporal stream
    typedef float f4 __attribute__((ext_vector_type(4)));
    const f4 v = __builtin_nontemporal_load(reinterpret_cast<const f4 *>(p));
    return make_float4(v.x, v.y, v.z, v.w);
}
#else
__device__ __forceinline__ float4 load_row4(const float *p) { return *reinterpret_cast<const float4 *>(p); }
#endif
#if defined(OMPL_AMD_VARIANT) && (OMPL_AMD_VARIANT == 2 || OMPL_AMD_VARIANT == 3)
constexpr int kS32LargeItems = 8;  // A/B build: 2,048 states per block from 4 M states up
#else
constexpr int kS32LargeItems = 4;  // measured: 1,024 states per block (8 waves / SIMD) streams ~10 % faster at 10^7
#endif

// one block = one chunk of 256 * ITEMS consecutive store positions of query blockIdx.y.  Lane
// loads are float4 (4 consecutive states of a row): load j of thread t covers positions
// base + j * 1024 + 4 t .. + 3, so a wave reads 1 KB per row per load instruction.
template <int SP, int F, int K, int ITEMS>
__global__ __launch_bounds__(kS32Threads) void knn_stream32_kernel(const float *__restrict__ feat32,
                                                                   const double *__restrict__ feat64, uint64_t cap,
                                                                   uint64_t n_end, const double *__restrict__ qfeat,
                                                                   DevSpace sp, float absmax, float qeta,
                                                                   double *__restrict__ part_d,
                                                                   uint32_t *__restrict__ part_i) {
    static_assert(ITEMS % 4 == 0, "float4 loads");
    constexpr int FS = Geo<SP, F>::FS;
    constexpr int NV = ITEMS / 4;
    __shared__ double lds_d[4 * K];
    __shared__ uint32_t lds_i[4 * K];
    __shared__ double sh_thr;
    const uint32_t q = blockIdx.y;
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
    // 1. fp32 screen: every row load of the chunk issued before the first distance
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
            float s[F];
#pragma unroll
            for (int f = 0; f < F; ++f) s[f] = u == 0 ? x[j][f].x : u == 1 ? x[j][f].y : u == 2 ? x[j][f].z : x[j][f].w;
            const float d = state_dist32<SP, F>(s, q32, w0, w1);  // NaN row 0: unused / removed slot
            d32[j * 4 + u] = d;
            const uint32_t id = (uint32_t)(base + (uint64_t)j * (4 * kS32Threads) + u);
            if (top.admits((double)d, id)) top.push((double)d, id);
        }
    }
    double rd;
    uint32_t ri;
    block_select<K>(top, lds_d, lds_i, rd, ri);
    if (threadIdx.x == K - 1) {
        // t = the chunk's K-th fp32 distance (+inf: fewer than K live states, all refined)
        const double t = rd;
        double B = absmax;
        const int nc = SP == OMPL_GPU_SPACE_SE3 ? 3 : F;
        for (int c = 0; c < nc; ++c) B = fmax(B, fabs(qv[c]));
        const double E = screen_error<SP>(sp, B, t, (double)qeta + query_eta<SP>(qv));
        sh_thr = (t + E) * (1.0 + 32.0 * kU);
    }
    __syncthreads();
    const double thr = sh_thr;
    // 2. exact fp64 distance of the chunk's candidates (reference order)
    top.init();
#pragma unroll
    for (int j = 0; j < NV; ++j) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if ((double)d32[j * 4 + u] <= thr) {  // NaN never passes
                const uint64_t id = base + (uint64_t)j * (4 * kS32Threads) + u;
                double sv[F];
#pragma unroll
                for (int f = 0; f < F; ++f) sv[f] = feat64[(uint64_t)f * cap + id];
                top.offer(feat_dist<SP, F, 0>(sv, qv, sp), (uint32_t)id);
            }
        }
    }
    __syncthreads();  // lds_d / lds_i are reused
    block_select<K>(top, lds_d, lds_i, rd, ri);
    if (threadIdx.x < K) {
        const size_t o = ((size_t)q * gridDim.x + blockIdx.x) * K + threadIdx.x;
        part_d[o] = rd;
        part_i[o] = ri;
    }
}

// ---- HBM-sized stores (>= 4 M states): the stream kernel only screens ---------------------
// knn_stream32_kernel refines its chunk's candidates in fp64 before it retires, so every block
// holds its slot through a dependent HBM read of a few scattered fp64 rows while no row loads are
// in flight.  From 4 M states up the streaming kernel only screens: per chunk it writes the
// positions with d32 <= thr_c = (t_c + E(t_c))(1 + 32u) (t_c = the chunk's K-th d32; at most
// CandCap of them, a longer list is marked by its count) and records t_c (one word per chunk);
// the refine kernel reduces T = min_c t_c and takes Gthr = (T + E(T))(1 + 32u):
// T >= the store's K-th d32 (chunk c alone has K states <= t_c), so the K best exact states have
// d32 <= Gthr (the in-chunk argument, globally), and T <= t_c for every chunk, so Gthr <= thr_c
// and every state with d32 <= Gthr is in its chunk's list (an overflowed list is rescanned from
// the fp32 rows).  Exact fp64 distances of those, per refine block a top-K, merged as before.
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


// block per query: the exact top-out_k of its P chunk lists
template <int K>
__global__ __launch_bounds__(256) void knn_stream32_merge_kernel(const double *__restrict__ pd,
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
    if (threadIdx.x < out_k) {
        out_d[(size_t)q * out_k + threadIdx.x] = rd;
        out_i[(size_t)q * out_k + threadIdx.x] = ri;
    }
}

// k = 1 (RRT's nearest, RRT.cpp:137): a persistent form.  Each block streams one long
// contiguous range (n / P states, P ~ 4 blocks per CU over the batch), its row loads two float4
// groups ahead of the arithmetic, and every thread keeps only its two smallest d32.  Then, as
// above with K = 1, thr = (m + E)(1 + 32u) from the block's fp32 minimum m: the block's exact
// nearest has d32 <= thr; a thread's smallest is refined in fp64 when <= thr, and a thread whose
// second smallest is <= thr too rescans its positions (rare).  One selection per range instead
// of two per 1,024 states, so the loads keep streaming.

template <int SP, int F>
__global__ __launch_bounds__(kS32Threads) void knn_stream1_kernel(const float *__restrict__ feat32,
                                                                  const double *__restrict__ feat64, uint64_t cap,
                                                                  uint64_t n_end, uint64_t range,
                                                                  const double *__restrict__ qfeat, DevSpace sp,
                                                                  float absmax, float qeta,
                                                                  double *__restrict__ part_d,
                                                                  uint32_t *__restrict__ part_i) {
    constexpr int FS = Geo<SP, F>::FS;
    __shared__ double lds_d[4];
    __shared__ uint32_t lds_i[4];
    __shared__ float lds_f[4];
    const uint32_t q = blockIdx.y;
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
    // grid-stride over 1,024-state groups (group g = blockIdx.x + j gridDim.x): at any moment the
    // blocks stream neighbouring groups of every row, as a one-shot grid would (a contiguous range
    // per block streamed 5-10 % slower at 10^7 states)
    (void)range;
    const uint64_t gstride = (uint64_t)gridDim.x * 4 * kS32Threads;
    const uint64_t b0 = (uint64_t)blockIdx.x * 4 * kS32Threads, b1 = n_end;
    const float nan4 = __builtin_nanf("");
    float m1 = __builtin_inff(), m2 = __builtin_inff();
    uint32_t i1 = kNoId;
    auto screen = [&](const float4 (&x)[F], uint64_t p) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            float s[F];
#pragma unroll
            for (int f = 0; f < F; ++f) s[f] = u == 0 ? x[f].x : u == 1 ? x[f].y : u == 2 ? x[f].z : x[f].w;
            const float d = state_dist32<SP, F>(s, q32, w0, w1);  // NaN: unused / removed slot
            if (d < m1) {
                m2 = m1;
                m1 = d;
                i1 = (uint32_t)(p + u);
            } else if (d < m2) {
                m2 = d;
            }
        }
    };
    auto load = [&](float4 (&x)[F], uint64_t p) {
#pragma unroll
        for (int f = 0; f < F; ++f)
            x[f] = p < b1 ? load_row4(feat32 + (uint64_t)f * cap + p) : make_float4(nan4, nan4, nan4, nan4);
    };
    // thread t covers positions b0 + 4t + 1024 j (a wave reads 1 KB per row per load)
    float4 xa[F], xb[F];
    uint64_t p = b0 + 4 * threadIdx.x;
    load(xa, p);
    load(xb, p + gstride);
    for (; p < b1; p += 2 * gstride) {
        screen(xa, p);
        load(xa, p + 2 * gstride);
        screen(xb, p + gstride);
        load(xb, p + 3 * gstride);
    }
    // the block's fp32 minimum and the refinement threshold
    float m = m1;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fminf(m, __shfl_xor(m, o));
    if ((threadIdx.x & 63) == 0) lds_f[threadIdx.x >> 6] = m;
    __syncthreads();
    m = fminf(fminf(lds_f[0], lds_f[1]), fminf(lds_f[2], lds_f[3]));
    double B = absmax;
    const int nc = SP == OMPL_GPU_SPACE_SE3 ? 3 : F;
    for (int c = 0; c < nc; ++c) B = fmax(B, fabs(qv[c]));
    const double t = (double)m;  // +inf: no live state in the range (nothing passes below)
    const double thr = (t + screen_error<SP>(sp, B, t, (double)qeta + query_eta<SP>(qv))) * (1.0 + 32.0 * kU);
    // exact fp64 distances of this thread's candidates (reference operation order)
    double bd = __builtin_inf();
    uint32_t bi = kNoId;
    auto refine = [&](uint64_t id) {
        double sv[F];
#pragma unroll
        for (int f = 0; f < F; ++f) sv[f] = feat64[(uint64_t)f * cap + id];
        const double x = feat_dist<SP, F, 0>(sv, qv, sp);
        if (lex_less(x, (uint32_t)id, bd, bi)) {
            bd = x;
            bi = (uint32_t)id;
        }
    };
    if ((double)m2 <= thr) {  // two or more candidates here: rescan this thread's positions
        for (uint64_t pp = b0 + 4 * threadIdx.x; pp < b1; pp += gstride) {
            float4 x[F];
            load(x, pp);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                float s[F];
#pragma unroll
                for (int f = 0; f < F; ++f) s[f] = u == 0 ? x[f].x : u == 1 ? x[f].y : u == 2 ? x[f].z : x[f].w;
                if ((double)state_dist32<SP, F>(s, q32, w0, w1) <= thr) refine(pp + u);
            }
        }
    } else if ((double)m1 <= thr) {
        refine(i1);
    }
    wave_argmin(bd, bi);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) {
        lds_d[threadIdx.x >> 6] = bd;
        lds_i[threadIdx.x >> 6] = bi;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 4; ++w)
            if (lex_less(lds_d[w], lds_i[w], bd, bi)) {
                bd = lds_d[w];
                bi = lds_i[w];
            }
        part_d[(size_t)q * gridDim.x + blockIdx.x] = bd;
        part_i[(size_t)q * gridDim.x + blockIdx.x] = bi;
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

template <int SP, int F, int K, int ITEMS>
hipError_t run_stream32(const DevSpace &sp, const float *feat32, const double *feat64, uint64_t cap, uint64_t n_end,
                        const double *qfeat, uint32_t nq, uint32_t k, float absmax, float qeta, double *out_d,
                        uint32_t *out_i, void *ws, size_t ws_bytes, hipStream_t st) {
    const uint32_t P = (uint32_t)((n_end + kS32Threads * ITEMS - 1) / (kS32Threads * ITEMS));
    const size_t need = (size_t)nq * P * K * (sizeof(double) + sizeof(uint32_t));
    if (ws_bytes < need) return hipErrorInvalidValue;
    double *pd = (double *)ws;
    uint32_t *pi = (uint32_t *)(pd + (size_t)nq * P * K);
    timer_begin(st, "knn_stream32_kernel");
    hipLaunchKernelGGL((knn_stream32_kernel<SP, F, K, ITEMS>), dim3(P, nq), dim3(kS32Threads), 0, st, feat32, feat64,
                       cap, n_end, qfeat, sp, absmax, qeta, pd, pi);
    timer_end(st);
    hipLaunchKernelGGL((knn_stream32_merge_kernel<K>), dim3(nq), dim3(256), 0, st, pd, pi, P, out_d, out_i, k);
    return hipGetLastError();
}

// states per block: 1,024 (kS32LargeItems from 4 M states up; the A/B build tries 2,048 there)
template <int SP, int F, int K>
hipError_t stream32_items(const DevSpace &sp, const float *feat32, const double *feat64, uint64_t cap, uint64_t n_end,
                          const double *qfeat, uint32_t nq, uint32_t k, float absmax, float qeta, double *out_d,
                          uint32_t *out_i, void *ws, size_t ws_bytes, hipStream_t st) {
    if (stream_split() && n_end >= stream_split_min())
        return run_stream32_split<SP, F, K, kS32LargeItems>(sp, feat32, feat64, cap, n_end, qfeat, nq, k, absmax,
                                                            qeta, out_d, out_i, ws, ws_bytes, st);
    if (n_end >= (4ull << 20))
        return run_stream32<SP, F, K, kS32LargeItems>(sp, feat32, feat64, cap, n_end, qfeat, nq, k, absmax, qeta, out_d, out_i, ws,
                                         ws_bytes, st);
    return run_stream32<SP, F, K, 4>(sp, feat32, feat64, cap, n_end, qfeat, nq, k, absmax, qeta, out_d, out_i, ws,
                                     ws_bytes, st);
}

template <int SP, int F>
hipError_t stream32_k(const DevSpace &sp, const float *feat32, const double *feat64, uint64_t cap, uint64_t n_end,
                      const double *qfeat, uint32_t nq, uint32_t k, float absmax, float qeta, double *out_d,
                      uint32_t *out_i, void *ws, size_t ws_bytes, hipStream_t st) {
    // Default dispatch: every k, every store size takes the split form (stream32_items: the
    // streaming kernel screens, one refine block per query decides; OMPL_GPU_SPLIT_MIN = 0).  The
    // persistent k = 1 form below is kept only behind the A/B switches (OMPL_GPU_STREAM_SPLIT=0 or
    // OMPL_GPU_SPLIT_MIN above the store size): measured at 10^6 it took 14.3 us against the split
    // form's 9.1 us, at 10^7 54.5 against 49 us
    if (k <= 1 && (n_end >= (4ull << 20) || stream1_blocks() == 0 || (stream_split() && n_end >= stream_split_min())))
        return stream32_items<SP, F, 1>(sp, feat32, feat64, cap, n_end, qfeat, nq, k, absmax, qeta, out_d, out_i, ws,
                                        ws_bytes, st);
    if (k <= 1) {  // the persistent form: ~8 blocks per CU over the batch
        const uint64_t groups = (n_end + 1023) / 1024;  // 1,024-state steps (a block's stride)
        const uint64_t P = std::max<uint64_t>(1, std::min<uint64_t>(groups, (uint64_t)stream1_blocks() / nq + 1));
        const uint64_t range = (groups + P - 1) / P * 1024;
        const uint32_t Pb = (uint32_t)((n_end + range - 1) / range);
        const size_t need = (size_t)nq * Pb * (sizeof(double) + sizeof(uint32_t));
        if (ws_bytes < need) return hipErrorInvalidValue;
        double *pd = (double *)ws;
        uint32_t *pi = (uint32_t *)(pd + (size_t)nq * Pb);
        timer_begin(st, "knn_stream1_kernel");
        hipLaunchKernelGGL((knn_stream1_kernel<SP, F>), dim3(Pb, nq), dim3(kS32Threads), 0, st, feat32, feat64, cap,
                           n_end, range, qfeat, sp, absmax, qeta, pd, pi);
        timer_end(st);
        hipLaunchKernelGGL((knn_stream32_merge_kernel<1>), dim3(nq), dim3(256), 0, st, pd, pi, Pb, out_d, out_i, k);
        return hipGetLastError();
    }
    if (k <= 4)
        return stream32_items<SP, F, 4>(sp, feat32, feat64, cap, n_end, qfeat, nq, k, absmax, qeta, out_d, out_i, ws,
                                        ws_bytes, st);
    return stream32_items<SP, F, 16>(sp, feat32, feat64, cap, n_end, qfeat, nq, k, absmax, qeta, out_d, out_i, ws,
                                     ws_bytes, st);
}

}  // namespace

bool stream32_supported(const DevSpace &sp, const FeatGeom &g, uint32_t nq, uint32_t k) {
    if (nq == 0 || nq >= kStreamMaxQ || k == 0 || k > kStream32MaxK) return false;
    if (sp.kind == OMPL_GPU_SPACE_SE3) return g.F == 7;
    if (sp.kind == OMPL_GPU_SPACE_REALVECTOR) return g.F == 4 || g.F == 8 || g.F == 16;
    return false;
}

size_t stream32_workspace_bytes(uint32_t nq, uint64_t n_end) {
    const uint64_t P = (n_end + kS32Threads * 4 - 1) / (kS32Threads * 4);
    const size_t chunked = (size_t)nq * P * 16 * (sizeof(double) + sizeof(uint32_t));
    const uint32_t PL = (uint32_t)((n_end + kS32Threads * kS32LargeItems - 1) / (kS32Threads * kS32LargeItems));
    return std::max(chunked, split_bytes(nq, PL, 16));
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
