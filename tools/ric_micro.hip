// Micro-benchmark of the Newton-system recursions of SqpKernel<quad2d> / <cartpole> in isolation
// (diagnostic only): the production device functions mfma_backward_h (factorisation),
// mfma4_forward (forward sweep) and mfma4_vector_backward (corrector) on synthetic stage data in
// LDS, one wave per instance, 1024 instances.  Round 4 also timed with it the hybrid factorisation
// (tools/hybrid_riccati_overlap.patch; profiles/r4/ab_hybrid_overlap/ric_micro.txt) and the sweeps
// with their stage operands two stages ahead instead of one (profiles/r4/ab_pf/ric_micro.txt), and the
// segmented forward sweep on the helper waves (tools/segmented_forward_sweep.patch, which also adds
// its timing here; profiles/r4/ab_seg/ric_micro.txt): all slower in the kernel and not kept.
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
        const int j = e % GS, i = (e / GS) % NX, k = e / (NX * GS);
        const double r = 0.5 - 0.37 * ((e * (7919 + salt)) % 101) / 101.0;
        L.G[(size_t)k * NX * GS + i * GS + j] = (j < NX) ? ((i == j) ? 1.0 : 0.0) + 0.01 * r : (j < NB ? 0.1 * r : 0.01 + 0.02 * r);
    }
    for (int e = lane; e < (H + 1) * NB; e += 64) {
        const int kk = e / NB, v = e - kk * NB;
        L.hq[kk * K::NBS + v] = 1.0 + 0.1 * ((e * (31 + salt)) % 17);
        L.gq[kk * K::NBS + v] = 0.01 * ((e * (13 + salt)) % 7) - 0.03;
    }
    __syncthreads();
    K::mfma_backward_h(L, H, lane);
    __syncthreads();
    K::template acl_phase<true>(L, H, lane);
    __syncthreads();
}

// V: 0 factorisation, 1 forward sweep, 2 corrector (vector backward)
template <int ID, int V>
__global__ __launch_bounds__(64) void micro(int H, int reps, unsigned long long* out, double* sink) {
    using K = SqpKernel<ID>;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const auto L = K::carve(smem, H);
    const int lane = threadIdx.x;
    init_stage_data<ID>(L, H, lane, blockIdx.x & 7);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    bool ok = true;
    for (int r = 0; r < reps; ++r) {
        if constexpr (V == 0) ok = K::mfma_backward_h(L, H, lane) && ok;
        if constexpr (V == 1) K::mfma4_forward(L, H, lane);
        if constexpr (V == 2) K::mfma4_vector_backward(L, H, lane);
        __syncthreads();
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[blockIdx.x] = t1 - t0;
    if (lane < K::NX) sink[blockIdx.x * 8 + lane] = L.P[lane] + L.K[lane] + L.dxv[lane] + (ok ? 0.0 : 1.0);
}

template <int ID, int V>
static double run(const char* name, int H, int B, int reps, unsigned long long* d_out, double* d_sink) {
    const size_t lds = SqpKernel<ID>::lds_doubles(H) * sizeof(double);
    micro<ID, V><<<B, 64, lds>>>(H, reps, d_out, d_sink);
    (void)hipDeviceSynchronize();
    micro<ID, V><<<B, 64, lds>>>(H, reps, d_out, d_sink);
    (void)hipDeviceSynchronize();
    std::vector<unsigned long long> h(B);
    (void)hipMemcpy(h.data(), d_out, B * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    double mean = 0.0;
    for (auto v : h) mean += (double)v;
    mean /= B;
    const double per = mean / reps;
    printf("%-34s H=%d: %9.0f cycles/recursion  %7.1f cycles/stage\n", name, H, per, per / H);
    return per;
}

int main() {
    const int B = 1024, reps = 50;
    unsigned long long* d_out;
    double* d_sink;
    (void)hipMalloc(&d_out, B * sizeof(unsigned long long));
    (void)hipMalloc(&d_sink, B * 8 * sizeof(double));
    run<kQuad2D, 0>("quad2d factorisation", 30, B, reps, d_out, d_sink);
    run<kQuad2D, 1>("quad2d forward sweep", 30, B, reps, d_out, d_sink);
    run<kQuad2D, 2>("quad2d corrector", 30, B, reps, d_out, d_sink);
    run<kCartpole, 0>("cartpole factorisation", 20, B, reps, d_out, d_sink);
    run<kCartpole, 1>("cartpole forward sweep", 20, B, reps, d_out, d_sink);
    run<kCartpole, 2>("cartpole corrector", 20, B, reps, d_out, d_sink);
    return 0;
}
