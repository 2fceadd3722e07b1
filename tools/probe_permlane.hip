// gfx950 cross-lane probes (diagnostic only): semantics of v_permlane16/32_swap with
// vdst == src0 (expected: lane l receives lane l^16 / l^32), DPP row_ror / quad_perm moves,
// and dependent-chain latencies of each, plus a 6x6 matvec recurrence with v_readlane
// broadcast (the shape of the Riccati vector sweeps).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probe_permlane tools/probe_permlane.hip
#include <hip/hip_runtime.h>

#include <cstdio>

__device__ __forceinline__ int xor32_i(int v) {
    auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return r[0];
}
__device__ __forceinline__ int xor16_i(int v) {
    auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return r[0];
}

__global__ void sem(int* out) {
    const int l = threadIdx.x;
    auto a = __builtin_amdgcn_permlane32_swap(l, l + 100, false, false);
    auto b = __builtin_amdgcn_permlane16_swap(l, l + 100, false, false);
    out[l * 8 + 0] = a[0];
    out[l * 8 + 1] = a[1];
    out[l * 8 + 2] = b[0];
    out[l * 8 + 3] = b[1];
    out[l * 8 + 4] = __builtin_amdgcn_update_dpp(-1, l, 0x128, 0xf, 0xf, false);  // row_ror:8
    out[l * 8 + 5] = __builtin_amdgcn_update_dpp(-1, l, 0x124, 0xf, 0xf, false);  // row_ror:4
    out[l * 8 + 6] = __builtin_amdgcn_update_dpp(-1, l, 0x4E, 0xf, 0xf, false);   // quad_perm [2,3,0,1]
    out[l * 8 + 7] = __builtin_amdgcn_update_dpp(-1, l, 0xB1, 0xf, 0xf, false);   // quad_perm [1,0,3,2]
}

__global__ void lat(double* sink, long long* cyc, int iters, const double* A) {
    const int l = threadIdx.x;
    int v = l;
    long long t0 = clock64();
    for (int i = 0; i < iters; ++i) v = xor32_i(v) + 1;
    long long t1 = clock64();
    int w = l;
    for (int i = 0; i < iters; ++i) w = xor16_i(w) + 1;
    long long t2 = clock64();
    int d = l;
    for (int i = 0; i < iters; ++i) d = __builtin_amdgcn_update_dpp(0, d, 0x128, 0xf, 0xf, false) + 1;
    long long t3 = clock64();
    int s = l;
    for (int i = 0; i < iters; ++i) s = __shfl_xor(s, 32) + 1;
    long long t4 = clock64();
    // 6-dim recurrence x <- A x + b, lane i < 6 owns x[i], broadcast by readlane
    double a[6];
    for (int j = 0; j < 6; ++j) a[j] = A[(l % 6) * 6 + j];
    double x = 0.01 * l;
    long long t5 = clock64();
    for (int i = 0; i < iters; ++i) {
        double acc = 0.001;
#pragma unroll
        for (int j = 0; j < 6; ++j) {
            const long long bits = __double_as_longlong(x);
            const int lo = __builtin_amdgcn_readlane((int)bits, j);
            const int hi = __builtin_amdgcn_readlane((int)(bits >> 32), j);
            acc = fma(a[j], __longlong_as_double(((long long)hi << 32) | (unsigned)lo), acc);
        }
        x = acc;
    }
    long long t6 = clock64();
    double y = 1.0 + l;
    for (int i = 0; i < iters; ++i) y = fma(y, 0.999, 1e-3);
    long long t7 = clock64();
    sink[l] = v + w + d + s + x + y;
    if (l == 0) {
        cyc[0] = t1 - t0; cyc[1] = t2 - t1; cyc[2] = t3 - t2; cyc[3] = t4 - t3; cyc[4] = t6 - t5; cyc[5] = t7 - t6;
    }
}

int main() {
    int* d_o;
    (void)hipMalloc(&d_o, 64 * 8 * sizeof(int));
    sem<<<1, 64>>>(d_o);
    int h[64 * 8];
    (void)hipMemcpy(h, d_o, sizeof(h), hipMemcpyDeviceToHost);
    const char* names[8] = {"p32swap[0]", "p32swap[1]", "p16swap[0]", "p16swap[1]", "ror8", "ror4", "qp2301", "qp1032"};
    for (int q = 0; q < 8; ++q) {
        printf("%-11s", names[q]);
        for (int l = 0; l < 64; ++l) printf(" %d", h[l * 8 + q]);
        printf("\n");
    }
    double *sink, *A;
    long long* cyc;
    (void)hipMalloc(&sink, 64 * sizeof(double));
    (void)hipMalloc(&A, 36 * sizeof(double));
    double hA[36];
    for (int i = 0; i < 36; ++i) hA[i] = (i % 7 == 0) ? 0.9 : 0.01;
    (void)hipMemcpy(A, hA, sizeof(hA), hipMemcpyHostToDevice);
    (void)hipMalloc(&cyc, 8 * sizeof(long long));
    const int iters = 1000;
    lat<<<1, 64>>>(sink, cyc, iters, A);
    lat<<<1, 64>>>(sink, cyc, iters, A);
    long long c[8];
    (void)hipMemcpy(c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    const char* ln[6] = {"permlane32 dep", "permlane16 dep", "dpp ror8 dep", "shfl_xor32 dep", "6-dim readlane matvec", "fma f64 dep"};
    for (int q = 0; q < 6; ++q) printf("%-24s %8.1f cycles/iter\n", ln[q], (double)c[q] / iters);
    return 0;
}
