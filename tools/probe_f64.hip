// f64 VALU issue/latency probes for one wave per SIMD (gfx950), loop overhead amortised over
// 64 unrolled instructions:
//   dependent v_fma_f64 chain; 2 / 4 / 8 independent chains interleaved; exp_rbf serial vs
//   8 interleaved exps; the same with 2 waves on one SIMD (block of 128 threads on a 1-CU
//   grid is placed over SIMDs by the hardware, so the 2-wave rows use blocks of 64 and 2 blocks
//   per CU are not guaranteed on one SIMD: read them as "two waves in the CU").
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probe_f64 tools/probe_f64.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#include "../gp-mpc_amd/csrc/gpmpc_common.h"

template <int C>
__device__ __forceinline__ void chains(double (&x)[C], int reps) {
    for (int i = 0; i < reps; ++i) {
#pragma unroll
        for (int u = 0; u < 64 / C; ++u)
#pragma unroll
            for (int c = 0; c < C; ++c) x[c] = fma(x[c], 0.999, 1e-3);
    }
}

template <int C>
__global__ void k_chain(double* out, long long* cyc, int reps) {
    double x[C];
#pragma unroll
    for (int c = 0; c < C; ++c) x[c] = 1.0 + threadIdx.x * 1e-3 + c;
    const long long t0 = clock64();
    chains<C>(x, reps);
    const long long t1 = clock64();
    double s = 0;
#pragma unroll
    for (int c = 0; c < C; ++c) s += x[c];
    out[threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int C>
__global__ void k_exp(double* out, long long* cyc, int reps) {
    double x[C];
#pragma unroll
    for (int c = 0; c < C; ++c) x[c] = -0.5 - threadIdx.x * 1e-3 - c * 0.1;
    double acc = 0.0;
    const long long t0 = clock64();
    for (int i = 0; i < reps; ++i) {
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const double e = gpmpc::exp_rbf(x[c]);
            acc += e;
            x[c] = x[c] - 1e-9 * e;
        }
    }
    const long long t1 = clock64();
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int C>
__global__ void k_expn(double* out, long long* cyc, int reps) {
    double x[C];
#pragma unroll
    for (int c = 0; c < C; ++c) x[c] = -0.5 - threadIdx.x * 1e-3 - c * 0.1;
    double acc = 0.0;
    const long long t0 = clock64();
    for (int i = 0; i < reps; ++i) {
        double e[C];
#pragma unroll
        for (int c = 0; c < C; ++c) e[c] = x[c];
        gpmpc::exp_rbf_n<C>(e);
#pragma unroll
        for (int c = 0; c < C; ++c) {
            acc += e[c];
            x[c] = x[c] - 1e-9 * e[c];
        }
    }
    const long long t1 = clock64();
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <class K>
static void run(const char* name, K kern, int blocks, int reps, double per) {
    double* out;
    long long* cyc;
    (void)hipMalloc(&out, 64 * 8);
    (void)hipMalloc(&cyc, 4096 * 8);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), 0, 0, out, cyc, 4);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), 0, 0, out, cyc, reps);
    static long long h[4096];
    (void)hipMemcpy(h, cyc, blocks * 8, hipMemcpyDeviceToHost);
    double m = 0;
    for (int b = 0; b < blocks; ++b) m += h[b];
    m /= blocks;
    printf("%-36s blocks %4d  %.2f cycles per %s\n", name, blocks, m / (reps * per), per == 64 ? "fma" : "exp");
    (void)hipFree(out);
    (void)hipFree(cyc);
}

int main() {
    const int reps = 200;
    for (int blocks : {1, 1024, 2048, 4096}) {
        run("dep fma chain", k_chain<1>, blocks, reps, 64);
        run("2 chains", k_chain<2>, blocks, reps, 64);
        run("4 chains", k_chain<4>, blocks, reps, 64);
        run("8 chains", k_chain<8>, blocks, reps, 64);
        run("exp serial (1)", k_exp<1>, blocks, reps, 1);
        run("exp x4", k_exp<4>, blocks, reps, 4);
        run("exp x8", k_exp<8>, blocks, reps, 8);
        run("exp_rbf_n<8>", k_expn<8>, blocks, reps, 8);
        run("exp_rbf_n<16>", k_expn<16>, blocks, reps, 16);
    }
    return 0;
}
