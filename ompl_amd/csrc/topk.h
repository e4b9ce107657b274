// topk.h — register top-K lists and wave/block selection for the NN kernels.
//
// Order: lexicographic on (distance, id).  That makes every kernel's result
// independent of traversal order and equal to NearestNeighborsLinear's
// ascending output (NearestNeighborsLinear.h:119-131) with ties resolved by id;
// the reference leaves tie order unspecified (partial_sort / GNAT heap order).
// NaN distances (removed entries, padding) are never admitted.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ompl_amd {

constexpr uint32_t kNoId = 0xFFFFFFFFu;

__device__ __forceinline__ bool lex_less(double a, uint32_t ia, double b, uint32_t ib) {
    return a < b || (a == b && ia < ib);
}

template <int K>
struct TopK {
    double d[K];
    uint32_t i[K];

    __device__ __forceinline__ void init() {
#pragma unroll
        for (int j = 0; j < K; ++j) {
            d[j] = __builtin_inf();
            i[j] = kNoId;
        }
    }
    __device__ __forceinline__ bool admits(double cd, uint32_t ci) const { return lex_less(cd, ci, d[K - 1], i[K - 1]); }
    // sorted insert by a fully unrolled compare-exchange sweep (static register indices)
    __device__ __forceinline__ void push(double cd, uint32_t ci) {
#pragma unroll
        for (int j = 0; j < K; ++j) {
            bool sw = lex_less(cd, ci, d[j], i[j]);
            double td = d[j];
            uint32_t ti = i[j];
            d[j] = sw ? cd : td;
            i[j] = sw ? ci : ti;
            cd = sw ? td : cd;
            ci = sw ? ti : ci;
        }
    }
    __device__ __forceinline__ void offer(double cd, uint32_t ci) {
        if (admits(cd, ci)) push(cd, ci);
    }
    __device__ __forceinline__ void pop_front() {
#pragma unroll
        for (int j = 0; j + 1 < K; ++j) {
            d[j] = d[j + 1];
            i[j] = i[j + 1];
        }
        d[K - 1] = __builtin_inf();
        i[K - 1] = kNoId;
    }
};

// fp32 screening list: same (distance, id) order, plus the squared admission radius used
// by the cheap translation pre-reject (inflated by 2^-19 so rounding never rejects an
// element whose fp32 distance would still be admitted).
template <int K>
struct TopK32 {
    float d[K];
    uint32_t i[K];
    float tau2;

    __device__ __forceinline__ void init() {
#pragma unroll
        for (int j = 0; j < K; ++j) {
            d[j] = __builtin_inff();
            i[j] = kNoId;
        }
        tau2 = __builtin_inff();
    }
    __device__ __forceinline__ bool admits(float cd, uint32_t ci) const {
        return cd < d[K - 1] || (cd == d[K - 1] && ci < i[K - 1]);
    }
    __device__ __forceinline__ void push(float cd, uint32_t ci) {
#pragma unroll
        for (int j = 0; j < K; ++j) {
            bool sw = cd < d[j] || (cd == d[j] && ci < i[j]);
            float td = d[j];
            uint32_t ti = i[j];
            d[j] = sw ? cd : td;
            i[j] = sw ? ci : ti;
            cd = sw ? td : cd;
            ci = sw ? ti : ci;
        }
        const float w = d[K - 1];
        tau2 = w * w * 1.0000020f;
    }
};

__device__ __forceinline__ void wave_argmin(double &d, uint32_t &i) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        double od = __shfl_xor(d, off, 64);
        uint32_t oi = __shfl_xor(i, off, 64);
        bool take = lex_less(od, oi, d, i);
        d = take ? od : d;
        i = take ? oi : i;
    }
}

// K rounds of wave argmin over the lanes' sorted lists: lane r (r < K) ends with
// the r-th smallest (d, id) of the union.  K <= 64.
template <int K>
__device__ __forceinline__ void wave_select(TopK<K> &t, double &rd, uint32_t &ri) {
    const int lane = threadIdx.x & 63;
    rd = __builtin_inf();
    ri = kNoId;
#pragma unroll 1
    for (int r = 0; r < K; ++r) {
        double md = t.d[0];
        uint32_t mi = t.i[0];
        wave_argmin(md, mi);
        if (lane == r) {
            rd = md;
            ri = mi;
        }
        if (t.i[0] == mi && t.d[0] == md) t.pop_front();
    }
}

// Block (blockDim.x == 256, 4 waves) top-K of all threads' lists; lanes 0..K-1 of
// wave 0 return the result (others return inf/kNoId).  Uses 4*K*(8+4) bytes of LDS.
template <int K>
__device__ __forceinline__ void block_select(TopK<K> &t, double *lds_d, uint32_t *lds_i, double &rd, uint32_t &ri) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    double wd;
    uint32_t wi;
    wave_select<K>(t, wd, wi);
    if (lane < K) {
        lds_d[wave * K + lane] = wd;
        lds_i[wave * K + lane] = wi;
    }
    __syncthreads();
    rd = __builtin_inf();
    ri = kNoId;
    if (wave == 0) {
        TopK<K> u;
        u.init();
        for (int j = lane; j < 4 * K; j += 64) u.offer(lds_d[j], lds_i[j]);
        wave_select<K>(u, rd, ri);
    }
}

}  // namespace ompl_amd
