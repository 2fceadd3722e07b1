// Issue-rate probe (gfx950): cycles per v_fma_f64 for one wave with 8 / 16 independent chains,
// and cycles per exp_rbf evaluation (8 independent), one wave per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probe_issue tools/probe_issue.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../gp-mpc_amd/csrc/gpmpc_common.h"

template <int C>
__global__ __launch_bounds__(64) void fma_chains(double* out, long long* cyc, int iters) {
    double a[C];
    for (int c = 0; c < C; ++c) a[c] = threadIdx.x * 1e-3 + c;
    const double m = 0.999999, b = 1e-7;
    long long t0 = clock64();
    for (int i = 0; i < iters; ++i)
#pragma unroll
        for (int c = 0; c < C; ++c) a[c] = fma(a[c], m, b);
    long long t1 = clock64();
    double s = 0;
    for (int c = 0; c < C; ++c) s += a[c];
    out[blockIdx.x * 64 + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ __launch_bounds__(64) void exp_chains(double* out, long long* cyc, int iters) {
    double a[8], acc[8];
    for (int c = 0; c < 8; ++c) { a[c] = -0.01 * (threadIdx.x + c); acc[c] = 0; }
    long long t0 = clock64();
    for (int i = 0; i < iters; ++i)
#pragma unroll
        for (int c = 0; c < 8; ++c) { acc[c] += gpmpc::exp_rbf(a[c]); a[c] -= 1e-6; }
    long long t1 = clock64();
    double s = 0;
    for (int c = 0; c < 8; ++c) s += acc[c];
    out[blockIdx.x * 64 + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    double* out; long long* cyc;
    hipMalloc(&out, 1 << 20); hipMalloc(&cyc, 1 << 16);
    long long h[2048];
    const int iters = 4096;
    auto report = [&](const char* name, int blocks, double per) {
        hipMemcpy(h, cyc, blocks * sizeof(long long), hipMemcpyDeviceToHost);
        double m = 0; for (int i = 0; i < blocks; ++i) m += h[i]; m /= blocks;
        printf("%-28s blocks %5d: %.2f clock64 ticks per %s\n", name, blocks, m / (iters * per), per == 8 ? "exp (8 chains)" : "instr");
    };
    for (int blocks : {1024, 2048}) {
        fma_chains<8><<<blocks, 64>>>(out, cyc, iters); hipDeviceSynchronize();
        fma_chains<8><<<blocks, 64>>>(out, cyc, iters); hipDeviceSynchronize(); report("fma f64, 8 chains", blocks, 8);
        fma_chains<16><<<blocks, 64>>>(out, cyc, iters); hipDeviceSynchronize(); report("fma f64, 16 chains", blocks, 16);
        exp_chains<<<blocks, 64>>>(out, cyc, iters); hipDeviceSynchronize(); report("exp_rbf, 8 chains", blocks, 8);
    }
    return 0;
}
