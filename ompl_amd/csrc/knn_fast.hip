// knn_fast.hip — dispatch of the exact batched kNN (fp32 screen + fp64 certificate).
// The kernels and their host orchestration live in knn_fast_impl.h, instantiated per
// space in knn_fast_se3.hip / knn_fast_so3.hip / knn_fast_rv.hip.
#include "knn_fast_impl.h"

namespace ompl_amd {
// K2: the smallest list bucket >= max(k + 6, 16); the certify kernel's K bucket fits inside it.
// The culled group walk (SE3, R^n) keeps k + 3 entries spread over the wave (one per lane), so
// it serves every k <= 61 — BIT*'s default nearestK at 10^7 samples is k = 57
// (bitstar/src/ImplicitGraph.cpp:313-316, 1383-1387).  The chunked thread-per-query screens
// hold their lists in registers and stop at k <= 32 (the chain's wave scan at k <= 58).
int fast_k2(const DevSpace &sp, uint32_t k, uint32_t nq, bool cull) {
    if (nq < kStreamMaxQ || k == 0) return 0;
    const int K = k_bucket(k);
    if (cull && cull_supported(sp) && sp.kind != OMPL_GPU_SPACE_KCHAIN) {
        if (K == 0 || k + 3 > 64) return 0;
        const int K2 = k_bucket(k + 3);
        return K2 < 16 ? 16 : K2;
    }
    if (K == 0 || (K > 32 && sp.kind != OMPL_GPU_SPACE_KCHAIN)) return 0;
    int K2 = k_bucket(k + 6);
    if (K2 < 16) K2 = 16;
    if (K2 == 0 || K2 < K) return 0;
    return K2;
}

// fp32 screening rows: the features (R^n, SO3, SE3) or the joint positions (KCHAIN)
int fp32_rows(const DevSpace &sp, const FeatGeom &g) { (void)sp; return g.F; }

hipError_t launch_rows32(const DevSpace &sp, const FeatGeom &g, const double *feat64, uint64_t cap, uint64_t first,
                         uint64_t n, float *feat32, hipStream_t st) {
    if (sp.kind == OMPL_GPU_SPACE_KCHAIN) return launch_chain_rows32(feat64, cap, g.nmax, first, n, feat32, st);
    return launch_to_fp32(feat64, cap, g.F, first, n, feat32, st);
}

// spaces with a k-d sorted store: the SE3 / R^n group walks (kNN and radius) and the
// KinematicChain culled scan (kNN only: radius_cull_supported)
bool cull_supported(const DevSpace &sp) {
    return sp.kind == OMPL_GPU_SPACE_SE3 || sp.kind == OMPL_GPU_SPACE_REALVECTOR || sp.kind == OMPL_GPU_SPACE_KCHAIN;
}
bool radius_cull_supported(const DevSpace &sp) {
    return sp.kind == OMPL_GPU_SPACE_SE3 || sp.kind == OMPL_GPU_SPACE_REALVECTOR;
}

void free_sorted_store(SortedStore *s) {
    for (void *x : {(void *)s->rows, (void *)s->ids, (void *)s->tbox, (void *)s->sbox, (void *)s->mbox, (void *)s->tkey0, (void *)s->nodes,
                    (void *)s->rows64, (void *)s->inv, (void *)s->qcount, (void *)s->rows16, s->scratch})
        if (x) (void)hipFree(x);
    *s = SortedStore{};
}

namespace {
__global__ void tombstone_kernel(const uint32_t *__restrict__ inv, uint64_t id, float *__restrict__ rows, int rw,
                                 uint32_t *__restrict__ rows16, int w16) {
    const uint32_t p = inv[id];
    if (p == kNoId) return;
    rows[blk_index(p, 0, rw)] = __builtin_nanf("");  // row 0 of the fp32 copy: every distance is NaN
    if (rows16) rows16[blk_index(p, 0, w16)] |= 0xFFFFu;  // the 16-bit copy's NaN marker (coordinate 0)
}
// thread = sorted position: the F = 2 nm fp32 coordinates to nm words (both tile-blocked)
__global__ void chain_rows16_kernel(const float *__restrict__ rows, uint32_t n_pad, uint32_t n, int nm,
                                    uint32_t *__restrict__ r16) {
    (void)n_pad;
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    bool dead = false;
    uint32_t w0 = 0;
    for (int w = 0; w < nm; ++w) {
        uint32_t c[2];
        for (int h = 0; h < 2; ++h) {
            const int f = 2 * w + h, li = f < nm ? f : f - nm;
            const float v = rows[blk_index(p, f, 2 * nm)];
            dead |= !(v == v);
            const float t = rintf((v + (float)(li + 1)) * (kChainQ16 / (float)(2 * (li + 1))));
            c[h] = (uint32_t)fminf(fmaxf(t, 0.f), kChainQ16);
        }
        const uint32_t word = c[0] | (c[1] << 16);
        if (w == 0) w0 = word;
        else r16[blk_index(p, w, nm)] = word;
    }
    r16[blk_index(p, 0, nm)] = dead ? (w0 | 0xFFFFu) : w0;
}
// thread = sorted position: the 7 SE3 coordinates to 4 words (the last half unused)
__global__ void se3_rows16_kernel(const float *__restrict__ rows, uint32_t n_pad, uint32_t n, Q16Geo q,
                                  uint32_t *__restrict__ r16) {
    (void)n_pad;
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    bool dead = false;
    uint32_t c[8];
#pragma unroll
    for (int f = 0; f < 7; ++f) {
        const float v = rows[blk_index(p, f, 7)];
        dead |= !(v == v);
        const float t = rintf((v - q.lo[f]) * q.inv[f]);
        c[f] = (uint32_t)fminf(fmaxf(t, 0.f), kQ16Max);
    }
    c[7] = 0u;
    if (dead) c[0] = 0xFFFFu;
#pragma unroll
    for (int w = 0; w < 4; ++w) r16[blk_index(p, w, 4)] = c[2 * w] | (c[2 * w + 1] << 16);
}
}  // namespace

hipError_t refresh_se3_rows16(const double *lo, const double *hi, SortedStore *s, hipStream_t st) {
    if (!s->built || !s->rows || s->ntiles == 0) return hipSuccess;
    if (s->rows16 && s->gen16 == s->gen) return hipSuccess;
    Q16Geo q{};
    for (int f = 0; f < 8; ++f) {
        // quaternion components: |q_i| <= sqrt(1 + eta) < 1.001 (screen_safe: eta <= 1e-4)
        const double l = f < 3 ? lo[f] : -1.001, ext = f < 3 ? hi[f] - lo[f] : 2.002;
        q.lo[f] = (float)l;
        q.step[f] = ext > 0.0 ? (float)(ext / (double)kQ16Max) : 0.f;
        q.inv[f] = ext > 0.0 ? (float)((double)kQ16Max / ext) : 0.f;
    }
    hipError_t e = grow_array(&s->rows16, s->cap16, (size_t)4 * s->n_pad);
    if (e != hipSuccess) return e;
    const uint32_t n = s->ntiles * kCullTile;
    hipLaunchKernelGGL(se3_rows16_kernel, dim3((n + 255) / 256), dim3(256), 0, st, s->rows, s->n_pad, n, q, s->rows16);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    s->w16 = 4;
    s->q16 = q;
    s->gen16 = s->gen;
    return hipSuccess;
}

// per coordinate the decoded value lo + code * step is within 0.52 step of the fp32 row (no
// clamping: the ranges hold every stored value; 0.5 for the rounding of the code, the rest the
// fp32 scaling) plus the rounding of that fp32 fmaf itself, half an ulp of the largest decoded
// magnitude (max(|lo|, |lo + ext|)): a box far from the origin with a narrow extent has steps near
// that ulp.  The translation gap moves by <= sqrt(3) of the per-coordinate error, the
// chord by <= |dq| <= 2 of the quaternion's, and theta(c) = 2 asin(c / 2) by <= 1.415 |dc| on
// c <= sqrt(2) (+ 5 %)
double se3_q16_error(const DevSpace &sp, const Q16Geo &q) {
    auto half_ulp = [](double m) {
        const float f = (float)m;
        return 0.5 * ((double)std::nextafter(f, __builtin_inff()) - (double)f);
    };
    double st = 0.0, ut = 0.0;
    for (int c = 0; c < 3; ++c) {
        st = std::max(st, (double)q.step[c]);
        const double top = (double)q.lo[c] + (double)q.step[c] * (double)kQ16Max;
        ut = std::max(ut, half_ulp(std::max(std::fabs((double)q.lo[c]), std::fabs(top))));
    }
    const double uq = half_ulp(1.001);
    return sp.w0 * 1.7320508075688772 * (0.52 * st + ut) * 1.01 +
           sp.w1 * 1.415 * 2.0 * (0.52 * (double)q.step[3] + uq) * 1.05 + 1e-7;
}

double chain_q16_error(const DevSpace &sp) {
    const double n = (double)sp.dim;
    return sp.link * 1.4142135623730951 * 0.6 * n * (n + 1.0) / (double)kChainQ16;
}

hipError_t refresh_chain_rows16(const FeatGeom &g, SortedStore *s, hipStream_t st) {
    if (!s->built || !s->rows || s->ntiles == 0) return hipSuccess;
    if (s->rows16 && s->gen16 == s->gen) return hipSuccess;
    const int nm = g.F / 2;
    hipError_t e = grow_array(&s->rows16, s->cap16, (size_t)nm * s->n_pad);
    if (e != hipSuccess) return e;
    const uint32_t n = s->ntiles * kCullTile;
    hipLaunchKernelGGL(chain_rows16_kernel, dim3((n + 255) / 256), dim3(256), 0, st, s->rows, s->n_pad, n, nm,
                       s->rows16);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    s->w16 = nm;
    s->gen16 = s->gen;
    return hipSuccess;
}

hipError_t tombstone_sorted_store(SortedStore *s, uint64_t id, hipStream_t st) {
    if (!s->built || id >= s->covered || id >= s->cap_inv) return hipSuccess;
    // a current 16-bit copy is patched in place and stays current
    const bool q16 = s->rows16 && s->gen16 == s->gen;
    hipLaunchKernelGGL(tombstone_kernel, dim3(1), dim3(1), 0, st, s->inv, id, s->rows, s->rw, q16 ? s->rows16 : nullptr,
                       s->w16);
    s->removed += 1;
    s->gen += 1;
    if (q16) s->gen16 = s->gen;
    return hipGetLastError();
}

hipError_t build_sorted_store(const DevSpace &sp, const FeatGeom &g, const float *feat32, const double *feat64,
                              uint64_t cap, uint64_t n_total, uint32_t n_live, const uint8_t *live, SortedStore *s,
                              hipStream_t st) {
    s->gen += 1;
    switch (sp.kind) {
    case OMPL_GPU_SPACE_SE3: return fast_se3_build(g, feat32, feat64, cap, n_total, n_live, live, s, st);
    case OMPL_GPU_SPACE_REALVECTOR: return fast_rv_build(g, feat32, feat64, cap, n_total, n_live, live, s, st);
    case OMPL_GPU_SPACE_KCHAIN: return fast_chain_build(g, feat32, feat64, cap, n_total, n_live, live, s, st);
    }
    return hipErrorInvalidValue;
}

hipError_t append_sorted_store(const DevSpace &sp, const FeatGeom &g, const float *feat32, const double *feat64,
                               uint64_t cap, uint64_t n_total, const FastBounds &b, SortedStore *s, hipStream_t st,
                               bool *fits) {
    s->gen += 1;
    switch (sp.kind) {
    case OMPL_GPU_SPACE_SE3: return fast_se3_append(g, feat32, feat64, cap, n_total, b, s, st, fits);
    case OMPL_GPU_SPACE_REALVECTOR: return fast_rv_append(g, feat32, feat64, cap, n_total, b, s, st, fits);
    case OMPL_GPU_SPACE_KCHAIN: return fast_chain_append(g, feat32, feat64, cap, n_total, b, s, st, fits);
    }
    *fits = false;
    return hipErrorInvalidValue;
}

size_t knn_fast_workspace_bytes(const DevSpace &sp, const FeatGeom &g, uint32_t nq, uint32_t k, uint64_t n_end,
                                int num_cus, bool cull) {
    const FastPlan p = fast_plan(sp, nq, k, n_end, num_cus, cull);
    if (p.K2 == 0) return 0;
    return fast_layout(sp, g, p, nq).total;
}

hipError_t launch_knn_fast(const DevSpace &sp, const FeatGeom &g, const double *feat64, const float *feat32,
                           uint64_t cap, uint64_t n_end, const SortedStore *sorted, const double *qfeat64, uint32_t nq,
                           uint32_t k, const FastBounds &b, double *out_d, uint32_t *out_i, void *ws, size_t ws_bytes,
                           int num_cus, hipStream_t st, uint32_t **fail_count, uint32_t **fail_list) {
    switch (sp.kind) {
    case OMPL_GPU_SPACE_SE3:
        return fast_se3(sp, g, feat64, feat32, cap, n_end, sorted, qfeat64, nq, k, b, out_d, out_i, ws, ws_bytes,
                        num_cus, st, fail_count, fail_list);
    case OMPL_GPU_SPACE_SO3:
        return fast_so3(sp, g, feat64, feat32, cap, n_end, nullptr, qfeat64, nq, k, b, out_d, out_i, ws, ws_bytes,
                        num_cus, st, fail_count, fail_list);
    case OMPL_GPU_SPACE_REALVECTOR:
        return fast_rv(sp, g, feat64, feat32, cap, n_end, sorted, qfeat64, nq, k, b, out_d, out_i, ws, ws_bytes,
                       num_cus, st, fail_count, fail_list);
    case OMPL_GPU_SPACE_KCHAIN:
        return fast_chain(sp, g, feat64, feat32, cap, n_end, sorted, qfeat64, nq, k, b, out_d, out_i, ws, ws_bytes,
                          num_cus, st, fail_count, fail_list);
    }
    return hipErrorInvalidValue;
}

size_t radius_fast_workspace_bytes(const DevSpace &sp, const FeatGeom &g, uint32_t nq) {
    return radius_layout(sp, g, nq).total;
}

hipError_t launch_radius_fast(const DevSpace &sp, const FeatGeom &g, const double *feat64, uint64_t cap,
                              const SortedStore *sorted, const double *qfeat64, uint32_t nq, double r,
                              const FastBounds &b, void *ws, size_t ws_bytes, int phase, uint64_t **d_offsets,
                              uint32_t *out_i, double *out_d, hipStream_t st) {
    switch (sp.kind) {
    case OMPL_GPU_SPACE_SE3:
        return fast_se3_radius(sp, g, feat64, cap, sorted, qfeat64, nq, r, b, ws, ws_bytes, phase, d_offsets, out_i,
                               out_d, st);
    case OMPL_GPU_SPACE_REALVECTOR:
        return fast_rv_radius(sp, g, feat64, cap, sorted, qfeat64, nq, r, b, ws, ws_bytes, phase, d_offsets, out_i,
                              out_d, st);
    }
    return hipErrorInvalidValue;
}

hipError_t launch_to_fp32(const double *feat64, uint64_t cap, int rows, uint64_t first, uint64_t n, float *feat32,
                          hipStream_t st) {
    if (n == 0 || rows == 0) return hipSuccess;
    const uint64_t t = n * rows;
    hipLaunchKernelGGL(to_fp32_kernel, dim3((unsigned)((t + 255) / 256)), dim3(256), 0, st, feat64, cap, rows, first,
                       n, feat32);
    return hipGetLastError();
}

hipError_t launch_gather_rows(const double *src, int F, const uint32_t *list, uint32_t n, double *dst, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(gather_rows_kernel, dim3((n * F + 255) / 256), dim3(256), 0, st, src, F, list, n, dst);
    return hipGetLastError();
}

hipError_t launch_scatter_results(const double *d, const uint32_t *ids, uint32_t k, const uint32_t *list, uint32_t n,
                                  double *out_d, uint32_t *out_i, hipStream_t st) {
    if (n == 0 || k == 0) return hipSuccess;
    hipLaunchKernelGGL(scatter_results_kernel, dim3((n * k + 255) / 256), dim3(256), 0, st, d, ids, k, list, n, out_d,
                       out_i);
    return hipGetLastError();
}

}  // namespace ompl_amd
