// Micro-benchmark of the Riccati sweeps of SqpKernel<quad2d> in isolation (diagnostic only).
// Times the production device functions (mfma_backward, valu_vector_backward, acl_phase,
// valu_forward, and the MFMA forward for comparison) on synthetic stage data in LDS, one wave per instance, 1024 instances.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I gp-mpc_amd/csrc -o tools/ric_micro tools/ric_micro.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "sqp_kernel.hip"

#undef WSYNC
#define WSYNC() __syncthreads()   // the micro-benchmark kernels are one wave per block

using namespace gpmpc;
using KQ = SqpKernel<kQuad2D>;

template <int V>
__global__ __launch_bounds__(64) void micro(int H, int reps, unsigned long long* out, double* sink) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const auto L = KQ::carve(smem, H);
    const int lane = threadIdx.x;
    constexpr int NX = KQ::NX, NB = KQ::NB, GS = KQ::GS, PS = KQ::PS;
    if (lane < 8) L.zero[lane] = (lane == 7) ? 1.0 : 0.0;
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
        if constexpr (V == 7) KQ::mfma_backward<true>(L, H, lane);
        if constexpr (V == 9) KQ::mfma_backward<false, 1>(L, H, lane);
        if constexpr (V == 10) KQ::mfma_backward<false, 3>(L, H, lane);
        if constexpr (V == 11) KQ::mfma_backward<false, 4>(L, H, lane);
        if constexpr (V == 12) KQ::mfma_backward_h(L, H, lane);
        if constexpr (V == 13) KQ::mfma_backward_h<1>(L, H, lane);
        if constexpr (V == 14) KQ::mfma4_forward2(L, H, lane);
        if constexpr (V == 8) KQ::mfma4_forward<1>(L, H, lane);
        if constexpr (V == 1) KQ::valu_vector_backward<0>(L, H, lane);
        if constexpr (V == 2) KQ::template acl_phase<true>(L, H, lane);
        if constexpr (V == 3) KQ::mfma4_forward(L, H, lane);
        if constexpr (V == 4) KQ::valu_forward(L, H, lane);
        if constexpr (V == 6) KQ::valu_vector_backward<1>(L, H, lane);
        if constexpr (V == 15) KQ::valu_vector_backward<2>(L, H, lane);
        if constexpr (V == 16) KQ::mfma_backward_h<8>(L, H, lane);
        if constexpr (V == 17) KQ::mfma_backward_h<16>(L, H, lane);
        if constexpr (V == 18) KQ::mfma_backward_h<32>(L, H, lane);
        if constexpr (V == 19) KQ::mfma_backward_h<48>(L, H, lane);
        if constexpr (V == 5) { double v = (double)r; for (int q = 0; q < H; ++q) v = wave_sum(v) * 1e-3; L.dummy[lane] = v; }
        WSYNC();
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[blockIdx.x] = t1 - t0;
    if (lane < NX) sink[blockIdx.x * 8 + lane] = L.P[lane] + L.dxv[H * NX + lane] + L.K[lane];
    (void)PS;
}

// correctness: the MFMA4 sweeps against the VALU sweeps on the same stage data
__device__ void init_stage_data(const KQ::Lds& L, int H, int lane, int salt) {
    constexpr int NX = KQ::NX, NB = KQ::NB, GS = KQ::GS;
    if (lane < 8) L.zero[lane] = (lane == 7) ? 1.0 : 0.0;
    for (int e = lane; e < H * NX * GS; e += 64) {
        const int j = e % GS, i = (e / GS) % NX;
        const double r = 0.5 - 0.37 * ((e * 7919) % 101) / 101.0;
        L.G[e] = (j < NX) ? ((i == j) ? 1.0 : 0.0) + 0.01 * r : (j < NB ? 0.1 * r : 0.01 + 0.02 * r);
    }
    for (int e = lane; e < (H + 1) * NB; e += 64) {
        L.hq[e] = 1.0 + 0.1 * ((e * 31) % 17);
        L.gq[e] = 0.01 * ((e * (13 + salt)) % 7) - 0.03;
    }
    WSYNC();
    KQ::mfma_backward(L, H, lane);
    WSYNC();
    KQ::template acl_phase<true>(L, H, lane);
    WSYNC();
}

__global__ __launch_bounds__(64) void cmp(int H, double* out) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const auto L = KQ::carve(smem, H);
    const int lane = threadIdx.x;
    constexpr int NX = KQ::NX, NU = KQ::NU, PS = KQ::PS, PP = KQ::PP, PO = KQ::PO;
    const int nd = (H + 1) * NX, nk = H * NU;
    auto pval = [&](int e) { return L.P[(e / NX) * PP + PO + e % NX]; };
    auto kval = [&](int e) { return L.K[(e / NU) * NU * PS + (e % NU) * PS + NX]; };
    init_stage_data(L, H, lane, 0);
    KQ::valu_forward(L, H, lane);
    WSYNC();
    double a[8];
    for (int q = 0; q < 8; ++q) { const int e = lane + 64 * q; a[q] = e < nd ? L.dxv[e] : 0.0; }
    WSYNC();
    KQ::mfma4_forward(L, H, lane);
    WSYNC();
    double err = 0.0, mag = 0.0;
    for (int q = 0; q < 8; ++q) { const int e = lane + 64 * q; if (e < nd) { err = fmax(err, fabs(L.dxv[e] - a[q])); mag = fmax(mag, fabs(a[q])); } }
    WSYNC();
    KQ::mfma4_forward<1>(L, H, lane);
    WSYNC();
    for (int q = 0; q < 8; ++q) { const int e = lane + 64 * q; if (e < nd) err = fmax(err, fabs(L.dxv[e] - a[q])); }
    WSYNC();
    // factorisation with the N-form Schur step against the MFMA Schur step: P', K', Ru^-1
    {
        constexpr int PPn = KQ::PP;
        init_stage_data(L, H, lane, 5);
        double pa[16], ka[8];
        for (int q = 0; q < 16; ++q) { const int e = lane + 64 * q; pa[q] = e < (H + 1) * PPn ? L.P[e] : 0.0; }
        for (int q = 0; q < 8; ++q) { const int e = lane + 64 * q; ka[q] = e < H * KQ::NU * KQ::PS ? L.K[e] : 0.0; }
        WSYNC();
        init_stage_data(L, H, lane, 5);
        if (out[6] > 1.5) KQ::mfma_backward_h(L, H, lane);
        else if (out[6] > 0.5) KQ::mfma_backward<false, 4>(L, H, lane);
        else KQ::mfma_backward<true>(L, H, lane);
        WSYNC();
        double ef = 0.0, mf = 0.0;
        for (int q = 0; q < 16; ++q) { const int e = lane + 64 * q; if (e >= PPn && e < (H + 1) * PPn) { ef = fmax(ef, fabs(L.P[e] - pa[q])); mf = fmax(mf, fabs(pa[q])); } }
        for (int q = 0; q < 8; ++q) { const int e = lane + 64 * q; if (e < H * KQ::NU * KQ::PS) { ef = fmax(ef, fabs(L.K[e] - ka[q])); mf = fmax(mf, fabs(ka[q])); } }
        ef = wave_max(ef); mf = wave_max(mf);
        if (lane == 0) { out[4] = ef; out[5] = mf; }
    }
    WSYNC();
    init_stage_data(L, H, lane, 3);
    KQ::valu_vector_backward<0>(L, H, lane);
    double p1[8], k1[4];
    for (int q = 0; q < 8; ++q) { const int e = lane + 64 * q; p1[q] = e < nd ? pval(e) : 0.0; }
    for (int q = 0; q < 4; ++q) { const int e = lane + 64 * q; k1[q] = e < nk ? kval(e) : 0.0; }
    WSYNC();
    init_stage_data(L, H, lane, 3);
    KQ::valu_vector_backward<1>(L, H, lane);
    double errp = 0.0, magp = 0.0;
    for (int q = 0; q < 8; ++q) { const int e = lane + 64 * q; if (e < nd) { errp = fmax(errp, fabs(pval(e) - p1[q])); magp = fmax(magp, fabs(p1[q])); } }
    for (int q = 0; q < 4; ++q) { const int e = lane + 64 * q; if (e < nk) { errp = fmax(errp, fabs(kval(e) - k1[q])); magp = fmax(magp, fabs(k1[q])); } }
    {   // DPP-free corrector sweep against the VALU one (p1, k1)
        WSYNC();
        init_stage_data(L, H, lane, 3);
        KQ::valu_vector_backward<2>(L, H, lane);
        double e3 = 0.0;
        for (int q = 0; q < 8; ++q) { const int e = lane + 64 * q; if (e < nd) e3 = fmax(e3, fabs(pval(e) - p1[q])); }
        for (int q = 0; q < 4; ++q) { const int e = lane + 64 * q; if (e < nk) e3 = fmax(e3, fabs(kval(e) - k1[q])); }
        e3 = wave_max(e3);
        if (lane == 0) out[8] = e3;
        WSYNC();
        init_stage_data(L, H, lane, 0);
        KQ::valu_forward(L, H, lane);
        WSYNC();
        for (int q = 0; q < 8; ++q) { const int e = lane + 64 * q; a[q] = e < nd ? L.dxv[e] : 0.0; }
        WSYNC();
    }
    {   // DPP-free forward sweep against the stored result of the VALU sweep (a[])
        KQ::mfma4_forward2(L, H, lane);
        WSYNC();
        double e2 = 0.0;
        for (int q = 0; q < 8; ++q) { const int e = lane + 64 * q; if (e < nd) e2 = fmax(e2, fabs(L.dxv[e] - a[q])); }
        e2 = wave_max(e2);
        if (lane == 0) out[7] = e2;
        WSYNC();
    }
    err = wave_max(err); mag = wave_max(mag); errp = wave_max(errp); magp = wave_max(magp);
    if (lane == 0) { out[0] = err; out[1] = mag; out[2] = errp; out[3] = magp; }
}

static void check(int H) {
    double* d;
    (void)hipMalloc(&d, 9 * sizeof(double));
    for (int variant = 0; variant < 3; ++variant) {
        const double flag = variant;
        (void)hipMemcpy(d + 6, &flag, sizeof(double), hipMemcpyHostToDevice);
        cmp<<<1, 64, KQ::lds_doubles(H) * sizeof(double)>>>(H, d);
        double h[9];
        (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
        printf("check forward mfma4 (both) vs valu: max |diff| %.3e (max |dx| %.3e); vector backward: %.3e (max %.3e); "
               "factor %s vs MFMA Schur: %.3e (max %.3e)\n", h[0], h[1], h[2], h[3],
               variant == 2 ? "homogeneous" : (variant ? "deferred-store" : "N-form"), h[4], h[5]);
        printf("  DPP-free forward vs VALU forward: max |diff| %.3e; DPP-free corrector vs VALU: %.3e\n", h[7], h[8]);
    }
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
    run<3>("forward (mfma4)", H, B, reps, d_out, d_sink);
    run<4>("forward (valu)", H, B, reps, d_out, d_sink);
    run<6>("backward (vec mfma4)", H, B, reps, d_out, d_sink);
    run<7>("backward (factor, N)", H, B, reps, d_out, d_sink);
    run<8>("forward (mfma4 2x)", H, B, reps, d_out, d_sink);
    run<5>("wave_sum x H", H, B, reps, d_out, d_sink);
    run<9>("factor, no stores", H, B, reps, d_out, d_sink);
    run<10>("factor, MFMA chain", H, B, reps, d_out, d_sink);
    run<11>("factor, deferred st", H, B, reps, d_out, d_sink);
    run<12>("factor, homogeneous", H, B, reps, d_out, d_sink);
    run<13>("factor, homog no st", H, B, reps, d_out, d_sink);
    run<14>("forward (4-chain)", H, B, reps, d_out, d_sink);
    run<15>("backward (vec 4-chain)", H, B, reps, d_out, d_sink);
    run<16>("factor h, no P' st", H, B, reps, d_out, d_sink);
    run<17>("factor h, no sched_b", H, B, reps, d_out, d_sink);
    run<18>("factor h, st after M", H, B, reps, d_out, d_sink);
    run<19>("factor h, after M nsb", H, B, reps, d_out, d_sink);
    check(H);
    return 0;
}
