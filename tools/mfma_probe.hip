// mfma_probe.hip — measurement probe (not the product): the brute-force fp32 MFMA distance
// matrix that configs[4] names, timed on MI355X against the culled radius walk the product uses.
//
// What it computes: for every (query, state) pair the squared translation distance
//   d^2 = |q|^2 + |s|^2 - 2 q.s
// as a K = 4 contraction on v_mfma_f32_32x32x2_f32 (A row = [-2qx, -2qy, -2qz, 1],
// B column = [sx, sy, sz, |s|^2], threshold r^2 - |q|^2 per row), and counts the pairs with
// d^2 <= r^2.  This is the cheapest possible MFMA prefilter for BIT*'s nearestR on SE(3): the
// translation term alone (d_SE3 >= d_R3), one compare per pair, no hit list written, no rotation
// term, no exact re-check — a lower bound on any brute-force MFMA radius search.
//
// Tiling: one wave = 64 queries (two 32-row groups) x one 32-state tile per step; 4 waves per
// block stride over the block's state range; blockIdx.x = query block, so the blocks resident
// together share one state range in L2.  Counts: per wave, one atomic at the end.
//
// usage: mfma_probe [n_states=10000000] [n_queries=8192] [radius=0.1528]
//   prints a JSON line: kernel ms (HIP events, median of 5), pairs/s, TFLOP/s (8 flop per pair:
//   2 MFMA k-steps x 2 x 2 — the contraction only), and the count checked against a CPU fp64
//   count on a subsample.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x16 __attribute__((ext_vector_type(16)));

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

constexpr int kWaves = 4;

__global__ __launch_bounds__(256) void mfma_radius_count(const float4 *__restrict__ S, uint32_t n_tiles,
                                                         const float4 *__restrict__ Q, uint32_t tiles_per_block,
                                                         float r2, unsigned long long *hits) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int row = lane & 31, kh = lane >> 5;  // A[i=row][k=kh], B[k=kh][j=row]
    const uint32_t q0 = blockIdx.x * 64;
    float a1[2], a2[2], thr[2][16];
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        const float4 q = Q[q0 + 32 * g + row];
        a1[g] = kh ? -2.f * q.y : -2.f * q.x;  // k = 0, 1
        a2[g] = kh ? 1.f : -2.f * q.z;          // k = 2, 3
#pragma unroll
        for (int i = 0; i < 16; ++i) {  // D row of register i: (i & 3) + 8 (i >> 2) + 4 (lane >> 5)
            const float4 qi = Q[q0 + 32 * g + (i & 3) + 8 * (i >> 2) + 4 * kh];
            thr[g][i] = r2 - qi.w;
        }
    }
    const uint32_t t0 = blockIdx.y * tiles_per_block;
    const uint32_t t1 = min(n_tiles, t0 + tiles_per_block);
    uint32_t cnt = 0;
    const f32x16 zero = {0};
    for (uint32_t t = t0 + wave; t < t1; t += kWaves) {
        const float4 s = S[(size_t)t * 32 + row];
        const float b1 = kh ? s.y : s.x, b2 = kh ? s.w : s.z;
#pragma unroll
        for (int g = 0; g < 2; ++g) {
            f32x16 acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[g], b1, zero, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a2[g], b2, acc, 0, 0, 0);
#pragma unroll
            for (int i = 0; i < 16; ++i) cnt += acc[i] <= thr[g][i] ? 1u : 0u;
        }
    }
    // wave sum, one atomic per wave
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
    if (lane == 0 && cnt) atomicAdd(hits, (unsigned long long)cnt);
}

static uint64_t lcg(uint64_t &s) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    return s >> 11;
}

int main(int argc, char **argv) {
    const size_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 10000000;
    const size_t nq = argc > 2 ? strtoull(argv[2], nullptr, 10) : 8192;
    const double r = argc > 3 ? atof(argv[3]) : 0.1528;
    if (nq % 64 || nq == 0 || n == 0) {
        fprintf(stderr, "n_queries must be a positive multiple of 64\n");
        return 2;
    }
    const size_t n_tiles = (n + 31) / 32, n_pad = n_tiles * 32;
    std::vector<float4> hs(n_pad), hq(nq);
    std::vector<double> ds(3 * n), dq(3 * nq);
    uint64_t seed = 42;
    auto u = [&]() { return (double)lcg(seed) * (1.0 / 9007199254740992.0); };
    for (size_t i = 0; i < n; ++i) {
        double x = u(), y = u(), z = u();
        ds[3 * i] = x, ds[3 * i + 1] = y, ds[3 * i + 2] = z;
        float fx = (float)x, fy = (float)y, fz = (float)z;
        hs[i] = make_float4(fx, fy, fz, fx * fx + fy * fy + fz * fz);
    }
    for (size_t i = n; i < n_pad; ++i) hs[i] = make_float4(0.f, 0.f, 0.f, 1e30f);  // padding never counts
    for (size_t i = 0; i < nq; ++i) {
        double x = u(), y = u(), z = u();
        dq[3 * i] = x, dq[3 * i + 1] = y, dq[3 * i + 2] = z;
        float fx = (float)x, fy = (float)y, fz = (float)z;
        hq[i] = make_float4(fx, fy, fz, fx * fx + fy * fy + fz * fz);
    }
    float4 *dS, *dQ;
    unsigned long long *dH;
    CK(hipMalloc(&dS, sizeof(float4) * n_pad));
    CK(hipMalloc(&dQ, sizeof(float4) * nq));
    CK(hipMalloc(&dH, sizeof(unsigned long long)));
    CK(hipMemcpy(dS, hs.data(), sizeof(float4) * n_pad, hipMemcpyHostToDevice));
    CK(hipMemcpy(dQ, hq.data(), sizeof(float4) * nq, hipMemcpyHostToDevice));
    const uint32_t splits = 64;
    const uint32_t tpb = (uint32_t)((n_tiles + splits - 1) / splits);
    dim3 grid((unsigned)(nq / 64), splits);
    const float r2 = (float)(r * r);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> ms;
    unsigned long long hits = 0;
    for (int rep = 0; rep < 6; ++rep) {
        CK(hipMemset(dH, 0, sizeof(unsigned long long)));
        CK(hipEventRecord(e0));
        mfma_radius_count<<<grid, 256>>>(dS, (uint32_t)n_tiles, dQ, tpb, r2, dH);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float t;
        CK(hipEventElapsedTime(&t, e0, e1));
        if (rep) ms.push_back(t);  // first launch is warm-up
        CK(hipMemcpy(&hits, dH, sizeof(hits), hipMemcpyDeviceToHost));
    }
    std::sort(ms.begin(), ms.end());
    const double kms = ms[ms.size() / 2];
    // CPU fp64 count on the first 64 queries over all states, scaled check against a GPU run on
    // those 64 queries alone
    CK(hipMemset(dH, 0, sizeof(unsigned long long)));
    mfma_radius_count<<<dim3(1, splits), 256>>>(dS, (uint32_t)n_tiles, dQ, tpb, r2, dH);
    unsigned long long gpu64 = 0;
    CK(hipMemcpy(&gpu64, dH, sizeof(gpu64), hipMemcpyDeviceToHost));
    unsigned long long cpu64 = 0;
    for (size_t q = 0; q < 64; ++q)
        for (size_t i = 0; i < n; ++i) {
            const double dx = dq[3 * q] - ds[3 * i], dy = dq[3 * q + 1] - ds[3 * i + 1], dz = dq[3 * q + 2] - ds[3 * i + 2];
            cpu64 += dx * dx + dy * dy + dz * dz <= r * r;
        }
    const double pairs = (double)n * (double)nq;
    printf("{\"probe\": \"mfma_radius_count\", \"states\": %zu, \"queries\": %zu, \"radius\": %.6g, \"kernel_ms\": %.4f, "
           "\"pairs_per_s\": %.4e, \"tflops_contraction\": %.2f, \"hits\": %llu, \"hit_fraction\": %.5f, "
           "\"check_64_queries\": {\"gpu\": %llu, \"cpu_fp64\": %llu}, "
           "\"ms_per_1e5_queries\": %.3f}\n",
           n, nq, r, kms, pairs / (kms * 1e-3), pairs * 8.0 / (kms * 1e-3) / 1e12, hits, hits / pairs, gpu64, cpu64,
           kms * 1e5 / (double)nq);
    return 0;
}
