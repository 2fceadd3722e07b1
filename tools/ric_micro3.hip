// quad3d (NX = 12, NU = 4) Riccati factorisation: the MFMA version (mfma_backward_big) against the
// VALU one (riccati_factor) on synthetic stage data -- agreement of P', K', Ru^-1 and cycles/stage.
// Diagnostic only.  Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I gp-mpc_amd/csrc
//                          -mllvm -amdgpu-mfma-vgpr-form=1 -o tools/ric_micro3 tools/ric_micro3.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "sqp_kernel.hip"

using namespace gpmpc;
using K3 = SqpKernel<kQuad3D>;

__device__ void init3(const K3::Lds& L, int H, int lane) {
    constexpr int NX = K3::NX, NB = K3::NB, GS = K3::GS;
    if (lane < 8) L.zero[lane] = (lane == 7) ? 1.0 : 0.0;
    for (int e = lane; e < H * NX * GS; e += 64) {
        const int j = e % GS, i = (e / GS) % NX;
        const double r = 0.5 - 0.37 * ((e * 7919) % 101) / 101.0;
        L.G[e] = (j < NX) ? ((i == j) ? 1.0 : 0.0) + 0.02 * r : (j < NB ? 0.1 * r : 0.01 + 0.02 * r);
    }
    for (int e = lane; e < (H + 1) * NB; e += 64) {
        L.hq[e] = 1.0 + 0.1 * ((e * 31) % 17);
        L.gq[e] = 0.01 * ((e * 13) % 7) - 0.03;
    }
    __syncthreads();
}

template <int V>
__global__ __launch_bounds__(64) void bench3(int H, int reps, unsigned long long* out, double* sink) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const auto L = K3::carve(smem, H);
    const int lane = threadIdx.x;
    init3(L, H, lane);
    const auto E = K3::decode(lane);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; ++r) {
        if constexpr (V == 0) K3::riccati_factor(L, H, lane, E);
        else K3::mfma_backward_big(L, H, lane);
        __syncthreads();
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[blockIdx.x] = t1 - t0;
    sink[blockIdx.x * 64 + lane] = L.P[lane] + L.K[lane] + L.Rui[lane & 15];
}

__global__ __launch_bounds__(64) void cmp3(int H, double* out) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const auto L = K3::carve(smem, H);
    const int lane = threadIdx.x;
    constexpr int NU = K3::NU, PS = K3::PS, PP = K3::PP;
    const int np = (H + 1) * PP, nk = H * NU * PS, nr = H * NU * NU;
    init3(L, H, lane);
    const bool ok0 = K3::riccati_factor(L, H, lane, K3::decode(lane));
    __syncthreads();
    double pa[64], ka[12], ra[12];
    for (int q = 0; q < 64; ++q) { const int e = lane + 64 * q; pa[q] = e < np ? L.P[e] : 0.0; }
    for (int q = 0; q < 12; ++q) { const int e = lane + 64 * q; ka[q] = e < nk ? L.K[e] : 0.0; }
    for (int q = 0; q < 12; ++q) { const int e = lane + 64 * q; ra[q] = e < nr ? L.Rui[e] : 0.0; }
    __syncthreads();
    init3(L, H, lane);
    const bool ok1 = K3::mfma_backward_big(L, H, lane);
    __syncthreads();
    double ep = 0, mp = 0, ek = 0, mk = 0, er = 0, mr = 0;
    for (int q = 0; q < 64; ++q) {
        const int e = lane + 64 * q;
        if (e >= PP && e < np) { ep = fmax(ep, fabs(L.P[e] - pa[q])); mp = fmax(mp, fabs(pa[q])); }
    }
    for (int q = 0; q < 12; ++q) {
        const int e = lane + 64 * q;
        if (e < nk) { ek = fmax(ek, fabs(L.K[e] - ka[q])); mk = fmax(mk, fabs(ka[q])); }
        if (e < nr) { er = fmax(er, fabs(L.Rui[e] - ra[q])); mr = fmax(mr, fabs(ra[q])); }
    }
    ep = wave_max(ep); mp = wave_max(mp); ek = wave_max(ek); mk = wave_max(mk); er = wave_max(er); mr = wave_max(mr);
    if (lane == 0) {
        out[0] = ep; out[1] = mp; out[2] = ek; out[3] = mk; out[4] = er; out[5] = mr;
        out[6] = ok0; out[7] = ok1;
    }
}

int main() {
    const int H = 40, B = 512, reps = 10;
    const size_t lds = K3::lds_doubles(H) * sizeof(double);
    (void)hipFuncSetAttribute((const void*)cmp3, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    (void)hipFuncSetAttribute((const void*)bench3<0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    (void)hipFuncSetAttribute((const void*)bench3<1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    double* d;
    (void)hipMalloc(&d, 8 * sizeof(double));
    cmp3<<<1, 64, lds>>>(H, d);
    double h[8];
    (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("quad3d H=%d: MFMA vs VALU factor: P' %.3e (max %.3e)  K' %.3e (max %.3e)  Ru^-1 %.3e (max %.3e)  ok %g %g\n",
           H, h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7]);
    unsigned long long* d_out;
    double* sink;
    (void)hipMalloc(&d_out, B * sizeof(unsigned long long));
    (void)hipMalloc(&sink, B * 64 * sizeof(double));
    for (int v = 0; v < 2; ++v) {
        if (v == 0) bench3<0><<<B, 64, lds>>>(H, reps, d_out, sink);
        else bench3<1><<<B, 64, lds>>>(H, reps, d_out, sink);
        (void)hipDeviceSynchronize();
        std::vector<unsigned long long> o(B);
        (void)hipMemcpy(o.data(), d_out, B * sizeof(unsigned long long), hipMemcpyDeviceToHost);
        double m = 0;
        for (auto x : o) m += (double)x;
        m /= B;
        printf("%-14s %9.0f cycles/factor  %7.1f cycles/stage\n", v ? "MFMA factor" : "VALU factor", m / reps, m / reps / H);
    }
    return 0;
}
