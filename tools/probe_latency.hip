// Latency probes for the register-resident Riccati design (gfx950):
//   dependent v_mfma_f64_16x16x4_f64 chain, dependent v_fma_f64 chain, __shfl (ds_bpermute)
//   round trip, LDS write->read round trip, v_readlane -> VALU.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probe_latency tools/probe_latency.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double f64x4 __attribute__((ext_vector_type(4)));

__global__ void probes(double* out, long long* cyc, int iters) {
    const int l = threadIdx.x;
    double a = 1.0 + l * 1e-3, b = 0.5 - l * 1e-4;
    f64x4 acc = {0.1, 0.2, 0.3, 0.4};
    // 1. dependent MFMA chain (acc -> acc)
    long long t0 = clock64();
    for (int i = 0; i < iters; ++i) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
    long long t1 = clock64();
    // 2. MFMA chain where the output feeds the B operand of the next (acc[0] -> b)
    f64x4 acc2 = {0.0, 0.0, 0.0, 0.0};
    double bb = b;
    long long t2 = clock64();
    for (int i = 0; i < iters; ++i) {
        acc2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bb, f64x4{0.0, 0.0, 0.0, 0.0}, 0, 0, 0);
        bb = acc2[0] * 1e-3 + 0.5;
    }
    long long t3 = clock64();
    // 3. dependent f64 FMA chain
    double x = a;
    long long t4 = clock64();
    for (int i = 0; i < iters; ++i) x = fma(x, 0.999, 1e-3);
    long long t5 = clock64();
    // 4. shfl round trip (dependent)
    double y = b;
    long long t6 = clock64();
    for (int i = 0; i < iters; ++i) y = __shfl(y, (l + 1) & 63) * 0.999 + 1e-3;
    long long t7 = clock64();
    // 5. readlane -> valu dependent
    double z = a;
    long long t8 = clock64();
    for (int i = 0; i < iters; ++i) {
        const int lo = __builtin_amdgcn_readfirstlane(__double2loint(z));
        const int hi = __builtin_amdgcn_readfirstlane(__double2hiint(z));
        z = __hiloint2double(hi, lo) * 0.999 + 1e-3 + l * 1e-9;
    }
    long long t9 = clock64();
    // 5b. dependent v_mfma_f64_4x4x4_4b chain (acc -> acc) and output -> B operand
    double q = 0.1 + l * 1e-3;
    long long tc = clock64();
    for (int i = 0; i < iters; ++i) q = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, q, 0, 0, 0);
    long long td = clock64();
    double qb = b;
    long long te = clock64();
    for (int i = 0; i < iters; ++i) qb = __builtin_amdgcn_mfma_f64_4x4x4f64(a, qb, 0.0, 0, 0, 0) * 1e-3 + 0.5;
    long long tf = clock64();
    // 6. independent MFMAs (4 accumulators)
    f64x4 c0 = acc, c1 = acc, c2 = acc, c3 = acc;
    long long ta = clock64();
    for (int i = 0; i < iters; ++i) {
        c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
    }
    long long tb = clock64();
    out[l] = acc[0] + acc2[1] + x + y + z + c0[0] + c1[1] + c2[2] + c3[3] + q + qb;
    if (l == 0) {
        cyc[0] = t1 - t0; cyc[1] = t3 - t2; cyc[2] = t5 - t4; cyc[3] = t7 - t6; cyc[4] = t9 - t8; cyc[5] = tb - ta; cyc[6] = td - tc; cyc[7] = tf - te;
    }
}

int main() {
    double* out;
    long long* cyc;
    (void)hipMalloc(&out, 64 * 8);
    (void)hipMalloc(&cyc, 8 * 8);
    const int iters = 1000;
    probes<<<1, 64>>>(out, cyc, 10);
    probes<<<1, 64>>>(out, cyc, iters);
    long long h[8];
    (void)hipMemcpy(h, cyc, 8 * 8, hipMemcpyDeviceToHost);
    const char* names[] = {"mfma f64 dep (acc)", "mfma f64 out->B operand", "fma f64 dep", "shfl dep",
                           "readfirstlane dep", "mfma f64 indep x4 (per 4)", "mfma f64 4x4x4 dep (acc)",
                           "mfma f64 4x4x4 out->B"};
    for (int i = 0; i < 8; ++i) printf("%-28s %.1f cycles/iter\n", names[i], (double)h[i] / iters);
    return 0;
}
