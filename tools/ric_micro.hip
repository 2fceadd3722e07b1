// Micro-benchmark of the Riccati factorisation of SqpKernel<quad2d> / <cartpole> in isolation
// (diagnostic only): the production device function mfma_backward_h in its two forms -- M' and the
// Schur product on v_mfma_f64_16x16x4 (HY = false) or v_mfma_f64_4x4x4_4b (HY = true) -- on
// synthetic stage data in LDS, one wave per instance, 1024 instances, plus an agreement check of
// every output (packed P', K', Ru^-1) between the two forms.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form=1 \
//        -I gp-mpc_amd/csrc -o tools/ric_micro tools/ric_micro.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "sqp_kernel.hip"

using namespace gpmpc;

template <int ID>
__device__ void init_stage_data(const typename SqpKernel<ID>::Lds& L, int H, int lane, int salt) {
    using K = SqpKernel<ID>;
    constexpr int NX = K::NX, NB = K::NB, GS = K::GS;
    if (lane < 8) L.zero[lane] = (lane == 7) ? 1.0 : 0.0;
    // synthetic, well-conditioned stage data: G' = [I + 0.01 R | 0.1 R | c], hq >= 1
    for (int e = lane; e < H * NX * GS; e += 64) {
        const int j = e % GS, i = (e / GS) % NX;
        const double r = 0.5 - 0.37 * ((e * (7919 + salt)) % 101) / 101.0;
        L.G[e] = (j < NX) ? ((i == j) ? 1.0 : 0.0) + 0.01 * r : (j < NB ? 0.1 * r : 0.01 + 0.02 * r);
    }
    for (int e = lane; e < (H + 1) * NB; e += 64) {
        L.hq[e] = 1.0 + 0.1 * ((e * (31 + salt)) % 17);
        L.gq[e] = 0.01 * ((e * (13 + salt)) % 7) - 0.03;
    }
    __syncthreads();
}

template <int ID, bool HY>
__global__ __launch_bounds__(64) void micro(int H, int reps, unsigned long long* out, double* sink) {
    using K = SqpKernel<ID>;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const auto L = K::carve(smem, H);
    const int lane = threadIdx.x;
    init_stage_data<ID>(L, H, lane, blockIdx.x & 7);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    bool ok = true;
    for (int r = 0; r < reps; ++r) {
        ok = K::template mfma_backward_h<HY>(L, H, lane) && ok;
        __syncthreads();
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[blockIdx.x] = t1 - t0;
    if (lane < K::NX) sink[blockIdx.x * 8 + lane] = L.P[lane] + L.K[lane] + (ok ? 0.0 : 1.0);
}

// both forms on the same data: max |difference| of P' (every stage), K', Ru^-1 and the magnitudes
template <int ID>
__global__ __launch_bounds__(64) void cmp(int H, double* out) {
    using K = SqpKernel<ID>;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const auto L = K::carve(smem, H);
    const int lane = threadIdx.x;
    const int np = (H + 1) * K::PP, nk = H * K::NU * K::PS, nr = H * K::NU * K::NU;
    init_stage_data<ID>(L, H, lane, 5);
    K::template mfma_backward_h<false>(L, H, lane);
    __syncthreads();
    constexpr int CAP = 24;
    double a[CAP], b[CAP], c[CAP];
    for (int q = 0; q < CAP; ++q) {
        const int e = lane + 64 * q;
        a[q] = e < np ? L.P[e] : 0.0;
        b[q] = e < nk ? L.K[e] : 0.0;
        c[q] = e < nr ? L.Rui[e] : 0.0;
    }
    __syncthreads();
    init_stage_data<ID>(L, H, lane, 5);
    K::template mfma_backward_h<true>(L, H, lane);
    __syncthreads();
    double ep = 0.0, ek = 0.0, er = 0.0, mp = 0.0, mk = 0.0;
    for (int q = 0; q < CAP; ++q) {
        const int e = lane + 64 * q;
        if (e >= K::PP && e < np) { ep = fmax(ep, fabs(L.P[e] - a[q])); mp = fmax(mp, fabs(a[q])); }
        if (e < nk) { ek = fmax(ek, fabs(L.K[e] - b[q])); mk = fmax(mk, fabs(b[q])); }
        if (e < nr) er = fmax(er, fabs(L.Rui[e] - c[q]));
    }
    ep = wave_max(ep); ek = wave_max(ek); er = wave_max(er); mp = wave_max(mp); mk = wave_max(mk);
    if (lane == 0) { out[0] = ep; out[1] = mp; out[2] = ek; out[3] = mk; out[4] = er; }
}

template <int ID, bool HY>
static double run(const char* name, int H, int B, int reps, unsigned long long* d_out, double* d_sink) {
    const size_t lds = SqpKernel<ID>::lds_doubles(H) * sizeof(double);
    micro<ID, HY><<<B, 64, lds>>>(H, reps, d_out, d_sink);
    (void)hipDeviceSynchronize();
    micro<ID, HY><<<B, 64, lds>>>(H, reps, d_out, d_sink);
    (void)hipDeviceSynchronize();
    std::vector<unsigned long long> h(B);
    (void)hipMemcpy(h.data(), d_out, B * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    double mean = 0.0;
    for (auto v : h) mean += (double)v;
    mean /= B;
    const double per = mean / reps;
    printf("%-34s H=%d: %9.0f cycles/factorisation  %7.1f cycles/stage\n", name, H, per, per / H);
    return per;
}

template <int ID>
static void check(const char* name, int H) {
    double* d;
    (void)hipMalloc(&d, 8 * sizeof(double));
    cmp<ID><<<1, 64, SqpKernel<ID>::lds_doubles(H) * sizeof(double)>>>(H, d);
    double h[8];
    (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("check %s H=%d hybrid vs 16x16x4: P' %.3e (max %.3e)  K' %.3e (max %.3e)  Ru^-1 %.3e\n", name, H, h[0], h[1],
           h[2], h[3], h[4]);
    (void)hipFree(d);
}

int main() {
    const int B = 1024, reps = 50;
    unsigned long long* d_out;
    double* d_sink;
    (void)hipMalloc(&d_out, B * sizeof(unsigned long long));
    (void)hipMalloc(&d_sink, B * 8 * sizeof(double));
    run<kQuad2D, false>("quad2d factor, 16x16x4", 30, B, reps, d_out, d_sink);
    run<kQuad2D, true>("quad2d factor, hybrid 4x4x4_4b", 30, B, reps, d_out, d_sink);
    run<kCartpole, false>("cartpole factor, 16x16x4", 20, B, reps, d_out, d_sink);
    run<kCartpole, true>("cartpole factor, hybrid 4x4x4_4b", 20, B, reps, d_out, d_sink);
    check<kQuad2D>("quad2d", 30);
    check<kCartpole>("cartpole", 20);
    return 0;
}
