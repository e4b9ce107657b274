// feat_dist.h — exact fp64 distance on feature rows (device), shared by the kNN kernels.
#pragma once
#include "device_space.h"

namespace ompl_amd {

// ---------------------------------------------------------------------------------
// distance on features (element first, query second: NearestNeighborsLinear.h:104)
template <int SP, int F, int NMAX>
__device__ __forceinline__ double feat_dist(const double *s, const double *q, const DevSpace &sp) {
    if constexpr (SP == OMPL_GPU_SPACE_REALVECTOR) {
        double acc = 0.0;
#pragma unroll
        for (int f = 0; f < F; ++f) {
            double diff = s[f] - q[f];
            acc += diff * diff;
        }
        return sqrt(acc);
    } else if constexpr (SP == OMPL_GPU_SPACE_SO3) {
        return so3_arc(s, q);
    } else if constexpr (SP == OMPL_GPU_SPACE_SE3) {
        return se3_dist(s, q, sp.w0, sp.w1);
    } else {
        return chain_dist_feat<NMAX>(s, q, sp.dim, sp.link);
    }
}

// ---------------------------------------------------------------------------------
// fp32 screen of the SO3 angle by the chord (knn_fast_impl.h header: error bound); shared by
// the culled walks and the large-k select
typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f2 pk_fma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }

// squared chord c^2 = min(|p - q|^2, |p + q|^2) of two quaternions, both sums on packed fp32
// (one v_pk_add / v_pk_fma per component gives both)
__device__ __forceinline__ float chord2(const float *p, const float *q) {
    f2 a = f2{p[0], p[0]} + f2{-q[0], q[0]};
    f2 c2 = a * a;
    a = f2{p[1], p[1]} + f2{-q[1], q[1]};
    c2 = pk_fma(a, a, c2);
    a = f2{p[2], p[2]} + f2{-q[2], q[2]};
    c2 = pk_fma(a, a, c2);
    a = f2{p[3], p[3]} + f2{-q[3], q[3]};
    c2 = pk_fma(a, a, c2);
    return fminf(c2.x, c2.y);
}

// theta = 2 asin(c / 2) from the chord c and c^2: theta = c (1 + x R(x)), x = c^2 / 4 in
// [0, 0.5], R a degree-5 fit of (asin(h) / h - 1) / h^2 (|error on theta| <= 1.1e-7, fp32
// evaluation <= 1.8e-7 over the whole range; tools/fit_asin.py).  x R(x) >= 0, so the fp32
// result is never below c: c is a lower bound of the screened angle, bit for bit.
__device__ __forceinline__ float chord_theta(float c, float c2) {
    const float x = 0.25f * c2;
    float r = 0.11142297f;
    r = fmaf(r, x, -0.07120271f);
    r = fmaf(r, x, 0.070305005f);
    r = fmaf(r, x, 0.036311187f);
    r = fmaf(r, x, 0.07580938f);
    r = fmaf(r, x, 0.16663891f);
    return fmaf(c, x * r, c);
}

__device__ __forceinline__ float chord_angle(const float *p, const float *q) {
    const float c2 = chord2(p, q);
    return chord_theta(__builtin_amdgcn_sqrtf(c2), c2);
}

template <int F>
struct LdsStride {
    static constexpr int value = (F + 1) & ~1;  // even -> 16-byte aligned rows for ds_read_b128
};

}  // namespace ompl_amd
