// Throughput probe (gfx950): back-to-back v_mfma_f64_16x16x4_f64 and v_mfma_f64_4x4x4_4b_f64 on
// independent accumulators, whole chip (blocks x waves), to calibrate the FP64 matrix peak the
// rooflines quote.  Prints TFLOP/s from HIP events and cycles per MFMA from clock64.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probe_mfma_rate tools/probe_mfma_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

typedef double f64x4 __attribute__((ext_vector_type(4)));

template <int U>
__global__ __launch_bounds__(256) void mfma16(double* out, long long* cyc, int iters) {
    f64x4 c[U];
    for (int u = 0; u < U; ++u) c[u] = f64x4{0, 0, 0, 0};
    const double a = 1e-3 * (threadIdx.x & 63), b = 0.5;
    const long long t0 = clock64();
    for (int i = 0; i < iters; ++i)
#pragma unroll
        for (int u = 0; u < U; ++u) c[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[u], 0, 0, 0);
    const long long t1 = clock64();
    double s = 0;
    for (int u = 0; u < U; ++u) s += c[u][0] + c[u][1] + c[u][2] + c[u][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int U>
__global__ __launch_bounds__(256) void mfma4(double* out, long long* cyc, int iters) {
    double c[U];
    for (int u = 0; u < U; ++u) c[u] = 0;
    const double a = 1e-3 * (threadIdx.x & 63), b = 0.5;
    const long long t0 = clock64();
    for (int i = 0; i < iters; ++i)
#pragma unroll
        for (int u = 0; u < U; ++u) c[u] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c[u], 0, 0, 0);
    const long long t1 = clock64();
    double s = 0;
    for (int u = 0; u < U; ++u) s += c[u];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <typename K>
void run(const char* name, K kern, int wps, double flop_per_mfma, int U) {
    const int blocks = 256 * 4, threads = 64 * wps, iters = 4000;   // 4 blocks per CU -> wps waves per SIMD
    double* out;
    long long* cyc;
    CK(hipMalloc(&out, (size_t)blocks * threads * sizeof(double)));
    CK(hipMalloc(&cyc, blocks * sizeof(long long)));
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, out, cyc, 10);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, out, cyc, iters);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    long long c0;
    CK(hipMemcpy(&c0, cyc, sizeof(c0), hipMemcpyDeviceToHost));
    const double flops = (double)blocks * wps * iters * U * flop_per_mfma;
    printf("%-22s U=%2d waves/SIMD %d: %.2f TFLOP/s, %.1f clock64 ticks per MFMA per wave\n", name, U, wps,
           flops / ms * 1e-9, (double)c0 / (iters * U));
    CK(hipFree(out));
    CK(hipFree(cyc));
}

int main() {
    run("mfma_f64_16x16x4", mfma16<8>, 1, 16 * 16 * 4 * 2.0, 8);
    run("mfma_f64_16x16x4", mfma16<8>, 2, 16 * 16 * 4 * 2.0, 8);
    run("mfma_f64_16x16x4", mfma16<4>, 2, 16 * 16 * 4 * 2.0, 4);
    run("mfma_f64_4x4x4_4b", mfma4<8>, 1, 4 * 4 * 4 * 4 * 2.0, 8);
    run("mfma_f64_4x4x4_4b", mfma4<8>, 2, 4 * 4 * 4 * 4 * 2.0, 8);
    return 0;
}
