// gfx950 dependent-chain latencies, 16 links unrolled per loop trip (diagnostic only).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probe_chain tools/probe_chain.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double f64x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ double rl(double v, int l) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, l);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xf, 0xf, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

#define U 16
__global__ void chains(double* sink, long long* cyc, int iters, double* lds_init) {
    __shared__ double sh[64 * 4];
    const int l = threadIdx.x;
    long long t[16];
    int n = 0;
    double x = 1.0 + 1e-3 * l, acc = 0.0;
    t[n++] = clock64();
    for (int i = 0; i < iters; ++i) {   // 0 empty loop (loop overhead baseline)
        __asm__ volatile("" : "+v"(x));
    }
    t[n++] = clock64();
    for (int i = 0; i < iters; ++i) {   // 1 fma dependent
#pragma unroll
        for (int u = 0; u < U; ++u) x = fma(x, 0.999, 1e-3);
    }
    t[n++] = clock64();
    double y0 = x, y1 = x + 1, y2 = x + 2, y3 = x + 3;
    for (int i = 0; i < iters; ++i) {   // 2 fma 4 independent chains (per link = 4 fmas)
#pragma unroll
        for (int u = 0; u < U; ++u) {
            y0 = fma(y0, 0.999, 1e-3); y1 = fma(y1, 0.999, 1e-3); y2 = fma(y2, 0.999, 1e-3); y3 = fma(y3, 0.999, 1e-3);
        }
    }
    t[n++] = clock64();
    acc += y0 + y1 + y2 + y3;
    for (int i = 0; i < iters; ++i) {   // 3 readlane -> fma
#pragma unroll
        for (int u = 0; u < U; ++u) x = fma(rl(x, u & 7), 0.999, 1e-3 * l);
    }
    t[n++] = clock64();
    for (int i = 0; i < iters; ++i) {   // 4 dpp row_ror:8 (f64 = 2 movs) -> add
#pragma unroll
        for (int u = 0; u < U; ++u) x = dpp_d<0x128>(x) + 1e-3;
    }
    t[n++] = clock64();
    for (int i = 0; i < iters; ++i) {   // 5 ds_write -> ds_read round trip
#pragma unroll
        for (int u = 0; u < U; ++u) {
            sh[l] = x;
            __builtin_amdgcn_s_waitcnt(0xc07f);
            x = sh[(l + 1) & 63] + 1e-3;
        }
    }
    t[n++] = clock64();
    for (int i = 0; i < iters; ++i) {   // 6 shfl (ds_bpermute) -> add
#pragma unroll
        for (int u = 0; u < U; ++u) x = __shfl(x, (l + 1) & 63) + 1e-3;
    }
    t[n++] = clock64();
    f64x4 c = {x, x, x, x};
    for (int i = 0; i < iters; ++i) {   // 7 mfma C-chain
#pragma unroll
        for (int u = 0; u < U; ++u) c = __builtin_amdgcn_mfma_f64_16x16x4f64(x, 0.5, c, 0, 0, 0);
    }
    t[n++] = clock64();
    double a = x;
    for (int i = 0; i < iters; ++i) {   // 8 mfma out -> A operand
#pragma unroll
        for (int u = 0; u < U; ++u) {
            f64x4 d = __builtin_amdgcn_mfma_f64_16x16x4f64(a, 0.5, f64x4{0, 0, 0, 0}, 0, 0, 0);
            a = d[0];
        }
    }
    t[n++] = clock64();
    double v = x;
    for (int i = 0; i < iters; ++i) {   // 9 mfma out -> valu fma -> mfma
#pragma unroll
        for (int u = 0; u < U; ++u) {
            f64x4 d = __builtin_amdgcn_mfma_f64_16x16x4f64(v, 0.5, f64x4{0, 0, 0, 0}, 0, 0, 0);
            v = fma(d[0], 0.5, 1e-3);
        }
    }
    t[n++] = clock64();
    double r = x;
    for (int i = 0; i < iters; ++i) {   // 10 v_rcp_f64 -> fma
#pragma unroll
        for (int u = 0; u < U; ++u) r = fma(__builtin_amdgcn_rcp(r), 0.5, 1.0);
    }
    t[n++] = clock64();
    double bb = x;
    for (int i = 0; i < iters; ++i) {   // 11 mfma out -> B operand
#pragma unroll
        for (int u = 0; u < U; ++u) {
            f64x4 d = __builtin_amdgcn_mfma_f64_16x16x4f64(0.5, bb, f64x4{0, 0, 0, 0}, 0, 0, 0);
            bb = d[0];
        }
    }
    t[n++] = clock64();
    double bv = x;
    for (int i = 0; i < iters; ++i) {   // 12 two independent mfma -> v_add -> B operand of both
#pragma unroll
        for (int u = 0; u < U; ++u) {
            f64x4 d0 = __builtin_amdgcn_mfma_f64_16x16x4f64(0.5, bv, f64x4{0, 0, 0, 0}, 0, 0, 0);
            f64x4 d1 = __builtin_amdgcn_mfma_f64_16x16x4f64(0.25, bv, f64x4{0, 0, 0, 0}, 0, 0, 0);
            bv = d0[0] + d1[1];
        }
    }
    t[n++] = clock64();
    double b4 = x;
    for (int i = 0; i < iters; ++i) {   // 13 4x4x4_4b out -> B operand
#pragma unroll
        for (int u = 0; u < U; ++u) b4 = __builtin_amdgcn_mfma_f64_4x4x4f64(0.5, b4, 0.0, 0, 0, 0);
    }
    t[n++] = clock64();
    sink[l] = x + acc + c[0] + c[1] + a + v + r + bb + bv + b4;
    if (l == 0)
        for (int q = 0; q + 1 < n; ++q) cyc[q] = t[q + 1] - t[q];
}

int main() {
    double *sink, *li;
    long long* cyc;
    (void)hipMalloc(&sink, 64 * sizeof(double));
    (void)hipMalloc(&li, 64 * sizeof(double));
    (void)hipMalloc(&cyc, 16 * sizeof(long long));
    const int iters = 200;
    chains<<<1, 64>>>(sink, cyc, iters, li);
    chains<<<1, 64>>>(sink, cyc, iters, li);
    long long c[16] = {};
    (void)hipMemcpy(c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    const char* names[] = {"loop overhead / trip", "fma f64 dep", "fma f64 x4 indep (per 4)", "readlane->fma",
                           "dpp f64 -> add", "lds write->read", "shfl -> add", "mfma C chain",
                           "mfma out -> A", "mfma out -> fma -> mfma", "rcp -> fma", "mfma out -> B",
                           "2 indep mfma -> add -> B", "4x4x4_4b out -> B"};
    printf("%-28s %10.1f cycles\n", names[0], (double)c[0] / iters);
    for (int q = 1; q < 14; ++q) printf("%-28s %10.1f cycles/link\n", names[q], (double)c[q] / iters / U);
    return 0;
}
