// Micro-benchmark of the segment-parallel Newton solve's pieces (SqpKernel<ID, 4, true>: three segments, diagnostic only):
// each production device function timed alone on wave 0 of a 4-wave workgroup, on synthetic stage
// data in LDS (tools/ric_micro.hip's), 256 instances (one per CU).  Cycles per call (s_memtime).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form=1 \
//        -I gp-mpc_amd/csrc -o tools/seg_micro tools/seg_micro.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "sqp_kernel.hip"

using namespace gpmpc;

template <int ID>
using KS = SqpKernel<ID, 4, true>;

template <int ID>
__device__ void init_data(const typename KS<ID>::Lds& L, int H, int lane, int salt) {
    using K = KS<ID>;
    constexpr int NX = K::NX, NB = K::NB, GS = K::GS;
    if (lane < 8) L.zero[lane] = (lane == 7) ? 1.0 : 0.0;
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
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    for (int w = K::NSEG - 1; w >= 0; --w) {
        const int k0 = K::seg_start(w, H), k1 = K::seg_start(w + 1, H);
        if (w == K::NSEG - 1) K::template seg_factor<false>(L, H, lane, k0, k1, nullptr);
        else K::template seg_factor<true>(L, H, lane, k0, k1, L.sb + K::SB_V + 256 * w);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        K::template seg_acl<true>(L, lane, k0, k1);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    K::seg_chain_full(L, H, lane);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// V: 0 factor A, 1 factor B, 2 boundary (predictor), 3 fold + forward A, 4 forward B,
//    5 vector backward A (+ V_l1), 6 vector backward B, 7 boundary (corrector), 8 acl<true> A
template <int ID, int V>
__global__ __launch_bounds__(256) void micro(int H, int reps, unsigned long long* out, double* sink) {
    using K = KS<ID>;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const auto L = K::carve(smem, H);
    if (threadIdx.x >= 64) return;   // wave 0 only
    const int lane = threadIdx.x;
    init_data<ID>(L, H, lane, blockIdx.x & 7);
    const int S1 = K::seg_start(1, H), SL = K::seg_start(K::NSEG - 1, H);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    bool ok = true;
    for (int r = 0; r < reps; ++r) {
        if constexpr (V == 0) ok = K::template seg_factor<true>(L, H, lane, 0, S1, L.sb + K::SB_V) && ok;
        if constexpr (V == 1) ok = K::template seg_factor<false>(L, H, lane, SL, H, nullptr) && ok;
        if constexpr (V == 2) K::seg_chain_full(L, H, lane);
        if constexpr (V == 3) {
            K::seg_fold(L, lane, 0, S1, L.sb + K::SB_LAM);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            K::seg_forward(L, lane, 0, S1, nullptr, false);
        }
        if constexpr (V == 4) K::seg_forward(L, lane, SL, H, L.sb + K::SB_XM + 8 * (K::NSEG - 1), true);
        if constexpr (V == 5) K::seg_vector_backward(L, H, lane, 0, S1, false, L.sb + K::SB_VL1);
        if constexpr (V == 6) K::seg_vector_backward(L, H, lane, SL, H, true, nullptr);
        if constexpr (V == 7) K::seg_chain_vec(L, H, lane);
        if constexpr (V == 8) K::template seg_acl<true>(L, lane, 0, S1);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[blockIdx.x] = t1 - t0;
    if (lane < K::NX) sink[blockIdx.x * 8 + lane] = L.P[lane] + L.K[lane] + L.dxv[lane] + L.sb[lane] + (ok ? 0.0 : 1.0);
}

template <int ID, int V>
static void run(const char* name, int H, int B, int reps, unsigned long long* d_out, double* d_sink) {
    const size_t lds = KS<ID>::lds_doubles(H) * sizeof(double);
    (void)hipFuncSetAttribute((const void*)micro<ID, V>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    micro<ID, V><<<B, 256, lds>>>(H, reps, d_out, d_sink);
    (void)hipDeviceSynchronize();
    micro<ID, V><<<B, 256, lds>>>(H, reps, d_out, d_sink);
    (void)hipDeviceSynchronize();
    std::vector<unsigned long long> h(B);
    (void)hipMemcpy(h.data(), d_out, B * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    double mean = 0.0;
    for (auto v : h) mean += (double)v;
    printf("%-40s H=%d: %9.0f cycles/call\n", name, H, mean / B / reps);
}

int main() {
    const int B = 256, reps = 50;
    unsigned long long* d_out;
    double* d_sink;
    (void)hipMalloc(&d_out, B * sizeof(unsigned long long));
    (void)hipMalloc(&d_sink, B * 8 * sizeof(double));
    for (int H : {30}) {
        run<kQuad2D, 0>("quad2d factor first segment (lambda)", H, B, reps, d_out, d_sink);
        run<kQuad2D, 1>("quad2d factor last segment", H, B, reps, d_out, d_sink);
        run<kQuad2D, 8>("quad2d acl<true> first segment", H, B, reps, d_out, d_sink);
        run<kQuad2D, 2>("quad2d boundary chain (predictor)", H, B, reps, d_out, d_sink);
        run<kQuad2D, 3>("quad2d fold + forward first segment", H, B, reps, d_out, d_sink);
        run<kQuad2D, 4>("quad2d forward last segment", H, B, reps, d_out, d_sink);
        run<kQuad2D, 5>("quad2d vector backward first (+ V_l1)", H, B, reps, d_out, d_sink);
        run<kQuad2D, 6>("quad2d vector backward last", H, B, reps, d_out, d_sink);
        run<kQuad2D, 7>("quad2d boundary chain (corrector)", H, B, reps, d_out, d_sink);
    }
    return 0;
}
