// fetch_calib.hip — measurement tool (not product): calibrates rocprofv3's FETCH_SIZE on gfx950 for
// the walks' access width.  MI355X_MICROARCH.md (HBM) calibrates wide 16-B-per-lane streaming reads
// (FETCH_SIZE = 1/2 of the bytes) and calls other widths uncalibrated; the culled walks read tiles
// as R rows of 64 lanes x 4 B (one float per lane, 256 B per wave instruction, rows n_pad apart).
// Each kernel reads a 512 MiB buffer (twice the Infinity Cache) exactly once: (a) 4 B per lane in
// the walks' tile layout (7 rows of 256 B per 64-state tile), (b) 16 B per lane; the profiled
// FETCH_SIZE per dispatch divided by 512 MiB is the factor to apply.
//   hipcc -O3 --offload-arch=gfx950 -o tools/bin/fetch_calib tools/fetch_calib.hip
//   rocprofv3 --pmc FETCH_SIZE -d gpurun_out/calib -o fetch --output-format csv -- tools/bin/fetch_calib
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr size_t kBytes = 512ull << 20;
constexpr int kRows = 7;

// (a) tiles of 64 states, kRows rows n_pad floats apart: wave w reads tile w, lane l its state
__global__ void read4_tiles(const float *__restrict__ rows, size_t n_pad, float *__restrict__ out) {
    const size_t tile = (size_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    const size_t p = tile * 64 + (threadIdx.x & 63);
    if (p >= n_pad) return;
    float s = 0.f;
#pragma unroll
    for (int r = 0; r < kRows; ++r) s += rows[(size_t)r * n_pad + p];
    if (s == 12345.f) out[0] = s;  // keeps the loads
}

// (b) 16 B per lane, contiguous
__global__ void read16(const float4 *__restrict__ a, size_t n, float *__restrict__ out) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float4 v = a[i];
    if (v.x + v.y + v.z + v.w == 12345.f) out[0] = v.x;
}

int main() {
    float *buf = nullptr, *out = nullptr;
    if (hipMalloc(&buf, kBytes) != hipSuccess || hipMalloc(&out, 16) != hipSuccess) return 2;
    if (hipMemset(buf, 0, kBytes) != hipSuccess) return 2;
    const size_t n_pad = kBytes / 4 / kRows / 64 * 64;
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(read4_tiles, dim3((unsigned)(n_pad / 256)), dim3(256), 0, 0, buf, n_pad, out);
        hipLaunchKernelGGL(read16, dim3((unsigned)(kBytes / 16 / 256)), dim3(256), 0, 0, (const float4 *)buf,
                           kBytes / 16, out);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 3;
    std::printf("{\"read4_tiles_bytes\": %zu, \"read16_bytes\": %zu}\n", n_pad * 4 * kRows, kBytes);
    (void)hipFree(buf);
    (void)hipFree(out);
    return 0;
}
