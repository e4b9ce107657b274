// libm_probe.hip — measurement tool (not product): the device math library's sin / cos / acos
// against the host's, on the argument ranges the hot path uses (cumulative KinematicChain angles
// |theta| <= 12 pi; SO3 |q1 . q2| in [0, 1]).  Reads n doubles from argv[1], writes
// sin, cos, acos of each and the glibc restatements' sin, cos, sincos, acos (ompl_amd/csrc/glibc_sincos.h, glibc_acos.h) to
// argv[2] (8 n doubles: sin, cos, acos, glibc sin, cos, sincos (2), acos); tools/libm_probe.py compares with glibc.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>

#include "../ompl_amd/csrc/glibc_acos.h"
#include "../ompl_amd/csrc/glibc_sincos.h"

__global__ void probe(const double *x, size_t n, double *o) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double v = x[i];
    o[i] = sin(v);
    o[n + i] = cos(v);
    o[2 * n + i] = acos(fabs(v) <= 1.0 ? v : 0.5);
    o[3 * n + i] = ompl_amd::glibc_sin(v);
    o[4 * n + i] = ompl_amd::glibc_cos(v);
    ompl_amd::glibc_sincos(v, o[5 * n + i], o[6 * n + i]);
    o[7 * n + i] = ompl_amd::glibc_acos(fabs(v) <= 1.0 ? v : 0.5);
}

int main(int argc, char **argv) {
    if (argc < 3) return 2;
    FILE *f = fopen(argv[1], "rb");
    if (!f) return 2;
    std::vector<double> x;
    double b[4096];
    size_t r;
    while ((r = fread(b, sizeof(double), 4096, f)) > 0) x.insert(x.end(), b, b + r);
    fclose(f);
    const size_t n = x.size();
    double *dx, *dout;
    if (hipMalloc(&dx, n * sizeof(double)) != hipSuccess || hipMalloc(&dout, 8 * n * sizeof(double)) != hipSuccess)
        return 3;
    hipMemcpy(dx, x.data(), n * sizeof(double), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, dx, n, dout);
    std::vector<double> out(8 * n);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(out.data(), dout, 8 * n * sizeof(double), hipMemcpyDeviceToHost);
    if (e != hipSuccess) {
        fprintf(stderr, "libm_probe: %s\n", hipGetErrorString(e));
        return 4;
    }
    hipFree(dx);
    hipFree(dout);
    FILE *g = fopen(argv[2], "wb");
    fwrite(out.data(), sizeof(double), out.size(), g);
    fclose(g);
    return 0;
}
