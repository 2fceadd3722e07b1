// Micro-benchmark of the Riccati sweeps of SqpKernel<quad2d> in isolation (diagnostic only).
// Times the production device functions (mfma_backward, valu_vector_backward, acl_phase,
// valu_forward, and the MFMA forward for comparison) on synthetic stage data in LDS, one wave per instance, 1024 instances.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I gp-mpc_amd/csrc -o tools/ric_micro tools/ric_micro.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "sqp_kernel.hip"

using namespace gpmpc;
using KQ = SqpKernel<kQuad2D>;

template <int V>
__global__ __launch_bounds__(64) void micro(int H, int reps, unsigned long long* out, double* sink) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const auto L = KQ::carve(smem, H);
    const int lane = threadIdx.x;
    constexpr int NX = KQ::NX, NB = KQ::NB, GS = KQ::GS, PS = KQ::PS;
    if (lane < 8) L.zero[lane] = 0.0;
    // synthetic, well-conditioned stage data: G' = [I + 0.01 R | 0.1 R | 0.01], hq >= 1
    for (int e = lane; e < H * NX * GS; e += 64) {
        const int j = e % GS, i = (e / GS) % NX;
        const double r = 0.5 - 0.37 * ((e * 7919) % 101) / 101.0;
        L.G[e] = (j < NX) ? ((i == j) ? 1.0 : 0.0) + 0.01 * r : (j < NB ? 0.1 * r : 0.01);
    }
    for (int e = lane; e < (H + 1) * NB; e += 64) {
        L.hq[e] = 1.0 + 0.1 * ((e * 31) % 17);
        L.gq[e] = 0.01 * ((e * 13) % 7) - 0.03;
    }
    WSYNC();
    KQ::mfma_backward(L, H, lane);
    WSYNC();
    KQ::template acl_phase<true>(L, H, lane);
    WSYNC();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; ++r) {
        if constexpr (V == 0) KQ::mfma_backward(L, H, lane);
        if constexpr (V == 1) KQ::valu_vector_backward(L, H, lane);
        if constexpr (V == 2) KQ::template acl_phase<true>(L, H, lane);
        if constexpr (V == 3) KQ::mfma_forward(L, H, lane);
        if constexpr (V == 4) KQ::valu_forward(L, H, lane);
        if constexpr (V == 5) { double v = (double)r; for (int q = 0; q < H; ++q) v = wave_sum(v) * 1e-3; L.dummy[lane] = v; }
        WSYNC();
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[blockIdx.x] = t1 - t0;
    if (lane < NX) sink[blockIdx.x * 8 + lane] = L.P[lane] + L.dxv[H * NX + lane] + L.K[lane];
    (void)PS;
}

template <int V>
static double run(const char* name, int H, int B, int reps, unsigned long long* d_out, double* d_sink) {
    const size_t lds = KQ::lds_doubles(H) * sizeof(double);
    micro<V><<<B, 64, lds>>>(H, reps, d_out, d_sink);
    (void)hipDeviceSynchronize();
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a);
    micro<V><<<B, 64, lds>>>(H, reps, d_out, d_sink);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, a, b);
    std::vector<unsigned long long> h(B);
    (void)hipMemcpy(h.data(), d_out, B * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    double mean = 0.0;
    for (auto v : h) mean += (double)v;
    mean /= B;
    const double per = mean / reps;
    printf("%-22s H=%d: %9.0f cycles/sweep  %7.1f cycles/stage   (kernel %.3f ms)\n", name, H, per, per / H, ms);
    return per;
}

int main() {
    const int H = 30, B = 1024, reps = 50;
    unsigned long long* d_out;
    double* d_sink;
    (void)hipMalloc(&d_out, B * sizeof(unsigned long long));
    (void)hipMalloc(&d_sink, B * 8 * sizeof(double));
    run<0>("backward (factor)", H, B, reps, d_out, d_sink);
    run<1>("backward (vector)", H, B, reps, d_out, d_sink);
    run<2>("closed-loop maps", H, B, reps, d_out, d_sink);
    run<3>("forward (mfma)", H, B, reps, d_out, d_sink);
    run<4>("forward (valu)", H, B, reps, d_out, d_sink);
    run<5>("wave_sum x H", H, B, reps, d_out, d_sink);
    return 0;
}
