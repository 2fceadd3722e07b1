// Design probes for the GP-MPC solve path on gfx950 (MI355X).
//  1. v_mfma_f64_16x16x4_f64 operand / accumulator lane map (exact integer data, asymmetric B).
//  2. fp64 exp throughput (ocml exp vs FMA) with one wave per SIMD and with 4 waves per SIMD.
//  3. intra-wave LDS round-trip latency (ds_write_b64 -> ds_read_b64 chain).
// Build: hipcc --offload-arch=gfx950 -O3 -o probe tools/probe_gfx950.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

typedef double f64x4 __attribute__((ext_vector_type(4)));

// A is 16x4 (row-major), B is 4x16, C = A*B 16x16.
// Guide: A/B as the f32 16x16x4 form (lane l: A[l&15][k=l>>4], B[k=l>>4][l&15]);
// C/D: col = lane&15, row = (lane>>4) + 4*reg.
__global__ void mfma_f64_map(const double* A, const double* B, double* C) {
    int l = threadIdx.x;
    double a = A[(l & 15) * 4 + (l >> 4)];
    double b = B[(l >> 4) * 16 + (l & 15)];
    f64x4 acc = {0, 0, 0, 0};
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
    for (int r = 0; r < 4; ++r) C[((l >> 4) + 4 * r) * 16 + (l & 15)] = acc[r];
}

__global__ void exp_tput(const double* in, double* out, int iters) {
    double x = in[blockIdx.x * blockDim.x + threadIdx.x];
    double s0 = 0, s1 = 0, s2 = 0, s3 = 0;
    for (int i = 0; i < iters; ++i) {
        s0 += exp(-x * (1.0 + 1e-3 * i));
        s1 += exp(-x * (1.1 + 1e-3 * i));
        s2 += exp(-x * (1.2 + 1e-3 * i));
        s3 += exp(-x * (1.3 + 1e-3 * i));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = s0 + s1 + s2 + s3;
}

__global__ void fma_tput(const double* in, double* out, int iters) {
    double x = in[blockIdx.x * blockDim.x + threadIdx.x];
    double s0 = x, s1 = x + 1, s2 = x + 2, s3 = x + 3, s4 = x + 4, s5 = x + 5, s6 = x + 6, s7 = x + 7;
    for (int i = 0; i < iters; ++i) {
        s0 = fma(s0, 0.999, 1e-3); s1 = fma(s1, 0.999, 1e-3); s2 = fma(s2, 0.999, 1e-3); s3 = fma(s3, 0.999, 1e-3);
        s4 = fma(s4, 0.999, 1e-3); s5 = fma(s5, 0.999, 1e-3); s6 = fma(s6, 0.999, 1e-3); s7 = fma(s7, 0.999, 1e-3);
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = s0 + s1 + s2 + s3 + s4 + s5 + s6 + s7;
}

__global__ void lds_roundtrip(double* out, long long* cyc, int iters) {
    __shared__ double buf[128];
    int l = threadIdx.x;
    double v = l;
    buf[l] = v;
    __builtin_amdgcn_wave_barrier();
    long long t0 = clock64();
    for (int i = 0; i < iters; ++i) {
        double r = buf[(l + 1 + i) & 63];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        buf[l] = r * 0.5 + 1.0;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
    long long t1 = clock64();
    out[l] = buf[l];
    if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    // 1. MFMA map
    std::vector<double> A(64), B(64), C(256), R(256, 0);
    for (int i = 0; i < 16; ++i) for (int k = 0; k < 4; ++k) A[i * 4 + k] = i * 4 + k + 1;
    for (int k = 0; k < 4; ++k) for (int j = 0; j < 16; ++j) B[k * 16 + j] = (k + 1) * 100 + j * j;
    for (int i = 0; i < 16; ++i) for (int j = 0; j < 16; ++j) for (int k = 0; k < 4; ++k) R[i * 16 + j] += A[i * 4 + k] * B[k * 16 + j];
    double *dA, *dB, *dC;
    CK(hipMalloc(&dA, 64 * 8)); CK(hipMalloc(&dB, 64 * 8)); CK(hipMalloc(&dC, 256 * 8));
    CK(hipMemcpy(dA, A.data(), 64 * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, B.data(), 64 * 8, hipMemcpyHostToDevice));
    mfma_f64_map<<<1, 64>>>(dA, dB, dC);
    CK(hipMemcpy(C.data(), dC, 256 * 8, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int i = 0; i < 256; ++i) bad += (C[i] != R[i]);
    printf("mfma_f64_16x16x4 map: %s (%d mismatches)\n", bad ? "FAIL" : "OK", bad);

    // 2. exp / fma throughput
    const int nthreads = 256 * 4 * 64 * 4;  // 4 waves per SIMD over 256 CUs
    double *din, *dout;
    CK(hipMalloc(&din, nthreads * 8)); CK(hipMalloc(&dout, nthreads * 8));
    std::vector<double> h(nthreads);
    for (int i = 0; i < nthreads; ++i) h[i] = 0.1 + (i % 97) * 0.01;
    CK(hipMemcpy(din, h.data(), nthreads * 8, hipMemcpyHostToDevice));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int wps : {1, 4}) {
        int blocks = 256 * wps;  // 256-thread blocks: 4 waves = 1 per SIMD
        int iters = 2000;
        exp_tput<<<blocks, 256>>>(din, dout, 10);
        CK(hipEventRecord(e0));
        exp_tput<<<blocks, 256>>>(din, dout, iters);
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        double nexp = (double)blocks * 256 * iters * 4;
        printf("exp f64: %d wave/SIMD: %.3f ms, %.2f Gexp/s\n", wps, ms, nexp / ms * 1e-6);
        fma_tput<<<blocks, 256>>>(din, dout, 10);
        CK(hipEventRecord(e0));
        fma_tput<<<blocks, 256>>>(din, dout, iters * 4);
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        double nf = (double)blocks * 256 * iters * 4 * 8 * 2;
        printf("fma f64: %d wave/SIMD: %.3f ms, %.2f TFLOP/s\n", wps, ms, nf / ms * 1e-9);
    }
    // 3. LDS round trip
    long long* dcyc; CK(hipMalloc(&dcyc, 8 * 8));
    lds_roundtrip<<<1, 64>>>(dout, dcyc, 10);
    lds_roundtrip<<<1, 64>>>(dout, dcyc, 1000);
    long long cyc; CK(hipMemcpy(&cyc, dcyc, 8, hipMemcpyDeviceToHost));
    printf("lds round trip (read->write): %.1f cycles/iter\n", cyc / 1000.0);
    return 0;
}
