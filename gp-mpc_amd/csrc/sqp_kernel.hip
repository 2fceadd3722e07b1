// Batched GP-MPC control step on CDNA4 (gfx950): one 64-lane wavefront per MPC instance.
//
// One launch = one call of GPMPC.select_action for B instances (gpmpc/gpmpc.py:334-368):
//   1. constraint tightening from the previous solution      (gpmpc/gpmpc.py:425-498)
//      -- the GP variances come from gp_var_tri_kernel / gp_post_kernel (gp_kernels.hip); the
//         H-step covariance recursion is evaluated as a convolution of the per-stage GP noise
//         with a host-built gain table (ProblemDev::tgain), every stage in parallel
//   2. acados-style SQP, Gauss-Newton Hessian, full steps,   (gpmpc/gpmpc.py:257-264)
//      status codes 0/1/2/4 (gpmpc/gpmpc.py:365)
//      a. linearisation: RK4 of prior + GP residual, exact tangent map (gpmpc/gpmpc.py:166-221)
//         -- GP mean + input-gradient sums over the training set as MFMA tile contractions
//            (gp_tiles: exponents on v_mfma_f64_16x16x4, sums on v_mfma_f64_4x4x4_4b)
//      b. NLP residuals (stat / eq / ineq / comp) with the previous multipliers
//      c. box-constrained LQ sub-problem: Mehrotra primal-dual IPM whose Newton systems
//         are solved by a Riccati recursion over the horizon (the HPIPM structure): the
//         factorisation on MFMA (mfma_backward) when a stage fits a 16x16 tile, the VALU
//         otherwise; forward and corrector sweeps on the VALU with readlane broadcasts
//   3. u0, the new iterate (= x_prev/u_prev for the next step) and the multipliers.
//
// Lane layout: lane k (0..H) owns stage k for the SQP-level work: w_k = [x_k; u_k] (x_0 fixed to
// obs, u_H absent), its bounds and the dynamics multiplier pi_k.  The IPM state of a stage is
// split over lanes k and k + 32 when H + 1 <= 32 (SPL).  The Riccati recursion is sequential
// over stages and parallel over matrix entries.  DESIGN.md §2.1 has the layouts and timings.
#include <algorithm>
#include <type_traits>

#include "gpmpc_common.h"
#include "models.h"

#ifndef GPMPC_SEG_FALLBACK   // 1: boundary-chain pivot check and one-segment fallback (A/B variants: 0)
#define GPMPC_SEG_FALLBACK 1
#endif
#ifndef GPMPC_SOLVE_STAMP    // 1: per-instance solve time in stats slots 10-11 (A/B variants: 0)
#define GPMPC_SOLVE_STAMP 1
#endif
#ifndef GPMPC_PHASE_LANE   // (round-6 A/B of phase_lane: 0 off, 1 one-wave and quad3d kernels, 2 every kernel)
#define GPMPC_PHASE_LANE 1
#endif

namespace gpmpc {

// Orders the LDS traffic of the (main) wave.  One wave per block: __syncthreads.  With GP helper
// waves (SqpKernel::NWAVES > 1) only the tile passes synchronise the block (B1/B2 in eval_gps and
// helper_loop); everywhere else the main wave orders its own LDS traffic: a wave's LDS operations
// execute in issue order, so a wavefront-scope fence (compiler ordering + lgkmcnt wait) suffices.
template <int NW>
__device__ __forceinline__ void wave_sync() {
    if constexpr (NW == 1) {
        __syncthreads();
    } else {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
}
#define WSYNC() wave_sync<NWAVES>()

// Diagnostic phase timing (build with -DGPMPC_TIMING): shader-clock cycles per phase,
// accumulated by the wave and stored per instance.  Phases (kPhases): 0 tightening, 1 linearise,
// 2 residuals/QP setup, 3 IPM vector work, 4 Riccati factor, 5 Riccati vector, 6 forward sweeps,
// 7 other, 8 closed-loop maps, 9 step recovery, 10 IPM residuals/Newton data.
#ifdef GPMPC_TIMING
#define TPHASE(id)                                                   \
    do {                                                             \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();  \
        tacc[tcur] += t_ - tlast;                                    \
        tlast = t_;                                                  \
        tcur = (id);                                                 \
    } while (0)
#else
#define TPHASE(id) do { } while (0)
#endif

// ------------------------------------------------------------------ cross-lane moves (gfx950)
// Butterfly partners without the LDS crossbar: DPP row rotations / quad permutes inside a
// 16-lane row, v_permlane16_swap / v_permlane32_swap across rows.  With vdst == src0 the swap
// instructions return the partner lane l^16 (l^32) in one of their two results.
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xf, 0xf, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
// Lanes in the banks (quads of a 16-lane row) selected by BANK receive v's DPP-moved value, the
// others keep `old` (the update_dpp old-value semantics).
template <int CTRL, int BANK>
__device__ __forceinline__ double dpp_merge(double old, double v) {
    const long long o = __double_as_longlong(old), b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp((int)o, (int)b, CTRL, 0xf, BANK, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(o >> 32), (int)(b >> 32), CTRL, 0xf, BANK, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ double xor16_d(double v) {   // value of lane l ^ 16
    const long long b = __double_as_longlong(v);
    const auto lo = __builtin_amdgcn_permlane16_swap((int)b, (int)b, false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap((int)(b >> 32), (int)(b >> 32), false, false);
    const bool odd = threadIdx.x & 16;
    const unsigned int rl = odd ? lo[0] : lo[1], rh = odd ? hi[0] : hi[1];
    return __longlong_as_double(((long long)rh << 32) | rl);
}
__device__ __forceinline__ double xor32_d(double v) {   // value of lane l ^ 32
    const long long b = __double_as_longlong(v);
    const auto lo = __builtin_amdgcn_permlane32_swap((int)b, (int)b, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((int)(b >> 32), (int)(b >> 32), false, false);
    const bool up = threadIdx.x & 32;
    const unsigned int rl = up ? lo[0] : lo[1], rh = up ? hi[0] : hi[1];
    return __longlong_as_double(((long long)rh << 32) | rl);
}
// Whole-wave reductions (all 64 lanes active).  Every lane ends with the bitwise-same value:
// each step combines a lane with a partner holding the mirrored partial (commutative ops).
template <class Op>
__device__ __forceinline__ double wave_reduce(double v, Op op) {
    v = op(v, dpp_d<0x128>(v));   // row_ror:8
    v = op(v, dpp_d<0x124>(v));   // row_ror:4
    v = op(v, dpp_d<0x4E>(v));    // quad_perm [2,3,0,1]
    v = op(v, dpp_d<0xB1>(v));    // quad_perm [1,0,3,2]
    v = op(v, xor16_d(v));
    return op(v, xor32_d(v));
}
__device__ __forceinline__ double wave_max(double v) {
    return wave_reduce(v, [](double a, double b) { return fmax(a, b); });
}
__device__ __forceinline__ double wave_min(double v) {
    return wave_reduce(v, [](double a, double b) { return fmin(a, b); });
}
__device__ __forceinline__ double wave_sum(double v) {
    return wave_reduce(v, [](double a, double b) { return a + b; });
}

typedef double f64x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ double readlane_d(double v, int l) {
    const long long bits = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)bits, l);
    const int hi = __builtin_amdgcn_readlane((int)(bits >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// Branch-free per-lane select (v_bfi_b32 on both halves): m all ones -> a, zero -> b.  A ternary on
// values computed only for the selecting lanes lets the compiler sink their computation into exec-
// masked branches; the bit select needs both values on every lane.
__device__ __forceinline__ double bsel(unsigned m, double a, double b) {
    const unsigned long long ia = __double_as_longlong(a), ib = __double_as_longlong(b);
    const unsigned lo = ((unsigned)ia & m) | ((unsigned)ib & ~m);
    const unsigned hi = ((unsigned)(ia >> 32) & m) | ((unsigned)(ib >> 32) & ~m);
    return __longlong_as_double(((long long)hi << 32) | lo);
}

__device__ __forceinline__ f64x4 mfma64(double a, double b, f64x4 c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// 1/x to full double precision (no IEEE div sequence): the v_rcp_f64 estimate r0 = (1 - eps)/x,
// |eps| <= 2^-23, refined by one cubic step r0 (1 + e + e^2), e = 1 - x r0, whose error is eps^3.
// Three dependent f64 ops after the estimate instead of four for two Newton steps (a dependent
// f64 VALU op waits ~7.3 cycles on gfx950, tools/probe_f64.hip).
// |x| ordering key: the high word with the sign cleared (exponent and 20 mantissa bits)
__device__ __forceinline__ unsigned hi_abs(double x) {
    return (unsigned)((unsigned long long)__double_as_longlong(x) >> 32) & 0x7fffffffu;
}

__device__ __forceinline__ double fast_rcp(double x) {
    const double r = __builtin_amdgcn_rcp(x);
    const double e = fma(-x, r, 1.0);
    return fma(r, fma(e, e, e), r);
}

// GP mean + input gradient at up to 16*NE evaluation points on the f64 matrix cores
// (gpmpc/gp.py:12-14 covSE, :84-85 mean k(z,X) K^-1 y with alpha = K^-1 y precomputed).
// Per 16-row training tile t (GPDev::tX / tW, centred on xbar) and 16-point evaluation tile:
//   A  = X'_t Z'^T + c|z|^2           1 v_mfma_f64_16x16x4_f64: X' rows [(x - xbar)/ell^2, c|x - xbar|^2],
//                                     Z' columns [z - xbar, 1], C-init c|z - xbar|^2 (c = -1/(2 ell^2)),
//                                     so A is the exponent c|z - x|^2 itself
//   E  = exp(A)                       4 exps per lane; register r of lane l holds
//                                     E[x = (l>>4) + 4r][z = l&15] (C/D layout)
//   S += W_t^T E                      4 v_mfma_f64_4x4x4_4b_f64 (K-steps r = 0..3), W = [alpha,
//                                     alpha (x - xbar)]: block b = z/4 of that instruction takes
//                                     A[b][j][k] from lane 16k + 4b + j and B[b][k][n] from lane
//                                     16k + 4b + n (layout probed by tools/probe_mfma4x4.hip), so
//                                     the exps are its B operand as they lie, and D[b][j][n] lands
//                                     in lane 16j + 4b + n: every output is a wanted S entry, a
//                                     quarter of the 16x16x4 contraction's matrix-core cycles
// so lane (j, z) ends with S[j][z], j < 4: {sum alpha E, sum alpha (x_d - xbar_d) E}.
// zb: [16*NE][4] {z - xbar, 1}; czz: [16*NE] c|z - xbar|^2; out: [16*NE][4].
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, int bytes) {
    const unsigned long long a = (unsigned long long)p;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a), hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
    void* u = (void*)(((unsigned long long)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(u, 0, __builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// TS > 1: this wave takes the tiles t0, t0 + TS, t0 + 2 TS, ... (the GP helper waves of a
// multi-wave instance, SqpKernel::NWAVES); its partial sums go to `out`.
template <int NE, int TS = 1>
__device__ __forceinline__ void gp_tiles(const double* tX, const double* tW, int nt, const double* zb,
                                         const double* czzb, double* out, int lane, int t0 = 0) {
    const int lr = lane >> 4, lc = lane & 15;
    double zo[NE], czz[NE];
#pragma unroll
    for (int e = 0; e < NE; ++e) {
        zo[e] = zb[(16 * e + lc) * 4 + lr];
        czz[e] = czzb[16 * e + lc];
    }
    double acc[NE];   // S[j = lr][z = 16 e + lc]
#pragma unroll
    for (int e = 0; e < NE; ++e) acc[e] = 0.0;
    // Tile operands through buffer loads (SGPR resource, per-lane byte offsets): the loads are
    // intrinsics, so the two-tile prefetch below survives the IR optimiser (plain loads through
    // a phi get folded back to the use), and reads past the pack return 0.
    const __amdgpu_buffer_rsrc_t rx = make_rsrc(tX, nt * 64 * 8);
    const __amdgpu_buffer_rsrc_t rw = make_rsrc(tW, nt * 64 * 8);
    const int ox = (lc * 4 + lr) * 8, ow = (lr * 4 + (lc & 3)) * 32;
    // i-th tile of this wave: t0 + i TS (reads past the pack return zeros)
    auto ldx = [&](int i) { return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rx, ox + (t0 + i * TS) * 512, 0, 0)); };
    auto ldw = [&](int i, int h) { return __builtin_amdgcn_raw_buffer_load_b128(rw, ow + (t0 + i * TS) * 512 + 16 * h, 0, 0); };
    struct Wops { decltype(ldw(0, 0)) a, b; };
    auto loadw = [&](int t, Wops& w) { w.a = ldw(t, 0); w.b = ldw(t, 1); };
    // exponent tile of training tile t (one MFMA per evaluation tile)
    auto dist = [&](double x, f64x4 (&a)[NE]) {
#pragma unroll
        for (int e = 0; e < NE; ++e) a[e] = mfma64(x, zo[e], f64x4{czz[e], czz[e], czz[e], czz[e]});
    };
    // exps + contraction of one training tile
    auto finish = [&](const f64x4 (&a)[NE], const Wops& w) {
        auto d = [](unsigned lo, unsigned hi) { return __builtin_bit_cast(double, (unsigned long long)lo | ((unsigned long long)hi << 32)); };
        const double wr[4] = {d(w.a[0], w.a[1]), d(w.a[2], w.a[3]), d(w.b[0], w.b[1]), d(w.b[2], w.b[3])};
        double ex[NE * 4];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int e = 0; e < NE; ++e) ex[e * 4 + r] = a[e][r];
        exp_rbf_n<NE * 4>(ex);   // all exps of the tile interleaved (issue-bound, not chain-bound)
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int e = 0; e < NE; ++e) acc[e] = __builtin_amdgcn_mfma_f64_4x4x4f64(wr[r], ex[e * 4 + r], acc[e], 0, 0, 0);
    };
    // Software pipeline, two tiles per iteration (ping-pong names, no register copies on the
    // back edge): tile t+1's exponent MFMAs are issued before tile t's exps and contraction, so
    // they run under that VALU work; X operands are fetched two tiles ahead, W one tile ahead.
    // The loop body is one basic block: tiles past nt read zeros (buffer range), whose exponent
    // is finite and whose weights contribute nothing.
    nt = TS == 1 ? nt : (nt - t0 + TS - 1) / TS;   // tiles of this wave
    double x0 = ldx(0), x1 = ldx(1);
    Wops w0, w1;
    loadw(0, w0);
    f64x4 a0[NE], a1[NE];
    dist(x0, a0);
    x0 = ldx(2);
    int t = 0;
    for (; t + 1 < nt; t += 2) {
        dist(x1, a1);            // tile t+1
        x1 = ldx(t + 3);
        loadw(t + 1, w1);
        finish(a0, w0);          // tile t
        dist(x0, a0);            // tile t+2
        x0 = ldx(t + 4);
        loadw(t + 2, w0);
        finish(a1, w1);          // tile t+1
    }
    if (t < nt) finish(a0, w0);  // odd tile count: the last tile
#pragma unroll
    for (int e = 0; e < NE; ++e) out[(16 * e + lc) * 4 + lr] = acc[e];   // S[lr][z]
}

template <int N, class F, int I = 0>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<N, F, I + 1>(static_cast<F&&>(f));
    }
}

// One copy of the tile loop per evaluation-tile count, shared by every call site (noinline).
// Three or four evaluation tiles (H > 32) run as two passes to bound the register footprint.
template <int TS = 1>
__device__ __attribute__((noinline)) void gp_tiles_dispatch(const double* tX, const double* tW, int ntile,
                                                          const double* zb, const double* czz, double* out,
                                                          int lane, int ne, int t0 = 0) {
    switch (ne) {
        case 1: gp_tiles<1, TS>(tX, tW, ntile, zb, czz, out, lane, t0); break;
        case 2: gp_tiles<2, TS>(tX, tW, ntile, zb, czz, out, lane, t0); break;
        case 3:
            gp_tiles<2, TS>(tX, tW, ntile, zb, czz, out, lane, t0);
            gp_tiles<1, TS>(tX, tW, ntile, zb + 32 * 4, czz + 32, out + 32 * 4, lane, t0);
            break;
        default:
            gp_tiles<2, TS>(tX, tW, ntile, zb, czz, out, lane, t0);
            gp_tiles<2, TS>(tX, tW, ntile, zb + 32 * 4, czz + 32, out + 32 * 4, lane, t0);
            break;
    }
}

// Waves per instance: the wide model (quad3d) always runs four (its LDS allows one instance per CU);
// the single-tile models run one, or two / four when the batch leaves SIMDs idle (launch_sqp_step).
template <int ID>
constexpr int kDefaultWaves = (Model<ID>::NB + 1 > 16) ? 4 : 1;

template <int ID, int NW = kDefaultWaves<ID>, bool SEG = false>
struct SqpKernel {
    using M = Model<ID>;
    static constexpr int NX = M::NX, NU = M::NU, NB = M::NB, NGP = M::NGP, NUNC = M::NUNC;
    static constexpr int GS = NB + 1;   // row stride of G'_k = [A_k | B_k | c_k]
    // cost of a solve for the dispatch order (StateDev::cost) in half IPM iterations: an SQP
    // iteration's linearisation costs ~1.4 IPM iterations on the single-tile models and ~2.6 on
    // quad3d (FITC tile sums over M = 2000; phase tables of DESIGN §2.1 / §4)
    static constexpr int kCostLin = (NB + 1 > 16) ? 5 : 3;
    static constexpr int PS = NX + 1;   // row stride of P'_k = [P_k | p_k] and K'_k = [K_k | kff_k]
    // stage stride of hq / gq: odd, so the IPM's one-stage-per-lane accesses (lanes k, k + 1, ..) hit
    // distinct LDS banks (NB = 8 made every ds_read_b64 / ds_write_b64 of them an 8-way conflict)
    static constexpr int NBS = NB | 1;
    static constexpr int CB = 4;        // tangent column block
    static constexpr int NCB = (NB + CB - 1) / CB;

    // Riccati on v_mfma_f64_16x16x4 when every stage product fits one 16x16 tile
    // (G' has NB+1 <= 16 columns, the forward state [dx; 1] has NX+1 <= 8 rows).
    static constexpr bool kMfma = (NB + 1 <= 16) && (NX + 1 <= 8);
    // multipliers kept in LDS during the step when the layout has room for them (single-tile models on
    // four waves: one instance per CU); otherwise they stay in global memory (rows read / written per
    // SQP iteration).  quad3d keeps them global: its LDS copy measured 4.6 % slower at config 5 (the
    // 14 KB push its 140 KB layout further and the copies sit on the step's critical path).
    static constexpr bool lds_mult = NW > 1 && kMfma;
    // Waves per instance.  The wide model (quad3d) needs more LDS than two instances per CU can
    // have, so its CU's other SIMDs would idle: three GP helper waves take a share of every GP
    // tile pass (gp_tiles over tiles w, w + 4, ...) and of the IPM's elementwise work (WSPL), the
    // main wave runs the recursions.  The single-tile models use the same protocol when the batch
    // is small enough for every instance to have a CU (B <= CUs): the idle SIMDs then do that work.
    static constexpr int NWAVES = NW;
    static_assert(NW == 1 || NW == 4 || (NW == 2 && kMfma), "one wave per instance, two (single-tile models) or four: one per SIMD");
    static constexpr int PP = NX * (NX + 1) / 2 + NX;   // packed P (upper triangle) + p
    static constexpr int PO = NX * (NX + 1) / 2;        // offset of p in a packed P' block
    // Segment-parallel Newton solves (kSeg): the horizon splits into NSEG segments
    // (three on four waves, two on two), factorised and swept at the same time on different waves;
    // every segment but the last runs over z = [x; 1; lambda] from the terminal cost lambda' x_b (lambda
    // the unknown costate of its end state x_b, solved for by the boundary chain), the last from the
    // true P'_H.  lambda takes tile slots LI .. LI + NX - 1; a P' block then also carries P_x,lambda
    // (NX x NX at PXL) and K'_k = [K | kff | K_lambda] (row stride KST).
    static constexpr bool kSeg = SEG;
    static_assert(!SEG || (NW >= 2 && NB + 1 <= 16 && NX + 1 <= 8), "segment-parallel solve: single-tile models on >= 2 waves");
    static constexpr int LI = 8 + NU;
    static_assert(!SEG || LI + NX <= 16, "lambda slots in the 16-wide tile");
    static constexpr int KST = SEG ? 2 * NX + 1 : PS;          // K' row stride
    static constexpr int PPB = SEG ? PP + NX * NX : PP;        // P' block stride
    static constexpr int PXL = PP;                             // offset of P_x,lambda in a P' block
    static constexpr int NSEG = NW >= 4 ? 3 : 2;   // segments: waves 1, 2, 3 (four waves) or 1, 0 (two)
    static constexpr int NBD = NSEG - 1;            // boundaries
    // segment boundary data (doubles): per boundary b (segment b's end) the factorised tile of the
    // segment's first stage (16 x 16, row-major), lambda_b, the segment's V_lambda,1 of the corrector,
    // T_b^-1, Y_b, y_b and the true cost-to-go at s_{b+1} when the chain computed it (packed P, p);
    // per segment its start state x_w
    static constexpr int SB_V = 0, SB_LAM = SB_V + 256 * NBD, SB_XM = SB_LAM + 8 * NBD, SB_VL1 = SB_XM + 8 * NSEG,
                         SB_TI = SB_VL1 + 8 * NBD, SB_Y = SB_TI + NX * NX * NBD, SB_YV = SB_Y + NX * NX * NBD,
                         SB_PH = SB_YV + 8 * NBD, SB = SEG ? (SB_PH + PP * NBD + 7) / 8 * 8 : 0;
    // (SB rounds up to 64 bytes: the regions carved after it keep the 16-byte alignment their wide
    // LDS accesses assume)

    // LDS carve (doubles), sized by H at launch.
    struct Lds {
        double *G, *P, *K, *Rui, *hq, *gq, *dxv, *cd, *Acl, *dummy, *zero, *gz, *gc, *gs, *gsh;
        double* sb;                  // kSeg: segment boundary data (SB doubles)
        double *Dq, *xs;             // WSPL: step-vector exchange, reduction slots
        double *lam, *pim;           // the instance's multipliers during the step (acados memory):
                                     // bounds [H+1][2 NB], dynamics [H][NX]
        int* ctrl;   // GP helper command (NWAVES > 1): GP index of the next tile pass, -1 = exit
    };
    // tightening: per-stage noise terms cd_k of the covariance convolution
    __host__ __device__ static size_t tight_scratch(int H) { return (size_t)H * NUNC; }
    // GP evaluation scratch of the linearisation: points [NGP][16*NE][4], c|z|^2 [NGP][16*NE], sums
    // [NGP][16*NE][4].  It aliases
    // the P' region, which is dead between the QP solves.
    __host__ __device__ static size_t gp_scratch(int H) {
        // + the helper waves' partial sums [NWAVES-1][16*NE][4]
        return (size_t)9 * NGP * 16 * ((H + 15) / 16) + (size_t)(NWAVES - 1) * 64 * ((H + 15) / 16);
    }
    // P'_k of every stage boundary | GP scratch
    __host__ __device__ static size_t p_region(int H) {
        const size_t pp = (size_t)(H + 1) * PPB;
        return pp > gp_scratch(H) ? pp : gp_scratch(H);
    }
    __host__ __device__ static size_t lds_doubles(int H) {
        const size_t common = (size_t)64                     // dummy store slots (branch-free stores)
                              + (size_t)8                    // zero slots (branch-free masked loads)
                              + (size_t)8                    // GP helper command slot
                              + (lds_mult ? (size_t)(H + 1) * 2 * NB + (size_t)H * NX : 0)   // multipliers
                              + (size_t)SB                   // segment boundary data (kSeg)
                              + (size_t)H * NX * GS            // G'_k
                              + (size_t)H * NU * KST         // K'_k
                              + (size_t)H * NU * NU          // Ru_k^-1
                              + (size_t)(H + 1) * NBS * 2    // hq, gq (stage stride NBS)
                              + (size_t)(H + 1) * NX;        // dx (forward sweep; WSPL: the published residual)
        if (kMfma) {
            // closed-loop A'_k; the tightening scratch and (WSPL) the step-vector exchange Dq alias it
            const size_t acl = (size_t)H * NX * PS;
            return common + p_region(H) + (acl > tight_scratch(H) ? acl : tight_scratch(H))
                   + (NWAVES > 1 ? 64 : 0);   // WSPL: xs
        }
        return common + p_region(H)                             // P'_k (packed) | GP scratch
               + tight_scratch(H)
               + (NWAVES > 1 ? (size_t)(H + 1) * NB + 64 : 0);  // WSPL exchange (Dq, xs)
    }
    __device__ static Lds carve(double* s, int H) {
        Lds L{};
        L.dummy = s; s += 64;
        L.zero = s;  s += 8;
        L.ctrl = reinterpret_cast<int*>(s);  s += 8;
        if constexpr (lds_mult) {
            L.lam = s; s += (size_t)(H + 1) * 2 * NB;
            L.pim = s; s += (size_t)H * NX;
        }
        L.sb = s;  s += SB;
        L.G = s;   s += (size_t)H * NX * GS;
        L.K = s;   s += (size_t)H * NU * KST;
        L.Rui = s; s += (size_t)H * NU * NU;
        L.hq = s;  s += (size_t)(H + 1) * NBS;
        L.gq = s;  s += (size_t)(H + 1) * NBS;
        L.dxv = s; s += (size_t)(H + 1) * NX;
        L.gz = s;
        L.gc = s + (size_t)NGP * 16 * ((H + 15) / 16) * 4;
        L.gs = L.gc + (size_t)NGP * 16 * ((H + 15) / 16);
        L.gsh = L.gs + (size_t)NGP * 16 * ((H + 15) / 16) * 4;
        if (kMfma) {
            L.P = s;   s += p_region(H);
            L.Acl = s;
            L.cd = s;
            if constexpr (NWAVES > 1) {   // Dq: live only inside an IPM iteration's residual phase
                L.Dq = s;
                const size_t acl = (size_t)H * NX * PS;
                s += acl > tight_scratch(H) ? acl : tight_scratch(H);
                L.xs = s;
            }
        } else {
            L.P = s;   s += p_region(H);
            L.cd = s;  s += tight_scratch(H);
            if constexpr (NWAVES > 1) {
                L.Dq = s;  s += (size_t)(H + 1) * NB;
                L.xs = s;
            }
        }
        return L;
    }

    // ------------------------------------------------------------------ GP sums on MFMA
    // One pass evaluates every GP of one kind (u-only or state-dependent) at all H stage points:
    // the stage lanes write their centred points to LDS, the whole wave runs the MFMA tile sums
    // (gp_tiles), and every lane reads the sums of its stage back.
    template <int G>
    __device__ static void gp_input(const double* x, const double* u, double* z) {
#pragma unroll
        for (int d = 0; d < M::gp_dim[G]; ++d) {
            const int s = M::gp_src[G][d];
            z[d] = s < NX ? x[s] : u[s - NX];
        }
    }

    template <int G>
    __device__ static void gp_centred(const GPDev& g, const double* x, const double* u, double (&zc)[3]) {
        double z[3];
        gp_input<G>(x, u, z);
#pragma unroll
        for (int d = 0; d < 3; ++d) zc[d] = d < M::gp_dim[G] ? z[d] - g.xbar[d] : 0.0;
    }

    __device__ static void eval_gps(const ProblemDev& P, const Lds& L, bool state_pass, const double* x,
                                    const double* u, int stage, int lane, int H, double* gm, double (*gg)[3]) {
        if (!P.use_gp) {
            if (!state_pass)
                for (int g = 0; g < NGP; ++g) { gm[g] = 0.0; gg[g][0] = gg[g][1] = gg[g][2] = 0.0; }
            return;
        }
        const int ne = (H + 15) >> 4, np = 16 * ne;
        // 1. points {z - xbar, c |z - xbar|^2}; padding points are zero
        static_for<NGP>([&](auto gi) {
            constexpr int G = decltype(gi)::value;
            if (M::gp_state_dep[G] != state_pass || lane >= np) return;
            double zc[3];
            gp_centred<G>(P.gp[G], x, u, zc);
            const double sq = fma(zc[0], zc[0], fma(zc[1], zc[1], zc[2] * zc[2]));
            const bool on = lane < H;
            double* dst = L.gz + ((size_t)G * np + lane) * 4;
            dst[0] = on ? zc[0] : 0.0;
            dst[1] = on ? zc[1] : 0.0;
            dst[2] = on ? zc[2] : 0.0;
            dst[3] = 1.0;
            L.gc[G * np + lane] = on ? -0.5 * P.gp[G].inv_ell2 * sq : 0.0;
        });
        WSYNC();
        // 2. MFMA tile sums
        static_for<NGP>([&](auto gi) {
            constexpr int G = decltype(gi)::value;
            if (M::gp_state_dep[G] != state_pass) return;
            const GPDev& g = P.gp[G];
            double* zb = L.gz + (size_t)G * np * 4;
            double* cz = L.gc + G * np;
            double* so = L.gs + (size_t)G * np * 4;
            if constexpr (NWAVES == 1) {
                gp_tiles_dispatch(g.tX, g.tW, g.ntile, zb, cz, so, lane, ne);
            } else {
                // the helper waves take tiles 1, 2, 3 (mod 4) of this pass (helper_loop)
                if (lane == 0) L.ctrl[0] = G;
                __syncthreads();   // B1: points and command visible to every wave
                gp_tiles_dispatch<NWAVES>(g.tX, g.tW, g.ntile, zb, cz, so, lane, ne, 0);
                __syncthreads();   // B2: partial sums of every wave written
                for (int e = lane; e < np * 4; e += 64) {
                    double part[NWAVES];   // every load before the sum (scheduling barrier)
                    part[0] = so[e];
#pragma unroll
                    for (int w = 1; w < NWAVES; ++w) part[w] = L.gsh[(size_t)(w - 1) * np * 4 + e];
                    __builtin_amdgcn_sched_barrier(0);
                    double v = part[0];
#pragma unroll
                    for (int w = 1; w < NWAVES; ++w) v += part[w];
                    so[e] = v;
                }
            }
        });
        WSYNC();
        // 3. mean sf2 S0 and input gradient sf2/ell^2 (S_{1+d} - (z_d - xbar_d) S0) of this lane's stage
        static_for<NGP>([&](auto gi) {
            constexpr int G = decltype(gi)::value;
            if (M::gp_state_dep[G] != state_pass) return;
            const GPDev& g = P.gp[G];
            const double* o = L.gs + ((size_t)G * np + stage) * 4;
            const double s0 = o[0], s1 = o[1], s2 = o[2], s3 = o[3];
            double zc[3];
            gp_centred<G>(g, x, u, zc);
            const double gs = g.sf2 * g.inv_ell2;
            gm[G] = g.sf2 * s0;
            gg[G][0] = gs * fma(-zc[0], s0, s1);
            gg[G][1] = M::gp_dim[G] > 1 ? gs * fma(-zc[1], s0, s2) : 0.0;
            gg[G][2] = M::gp_dim[G] > 2 ? gs * fma(-zc[2], s0, s3) : 0.0;
        });
    }

    // ------------------------------------------------------------------ linearisation
    // Every lane computes RK4 for stage s = lane % H (its chunk of the GP sums); chunk-c lanes
    // then build tangent column blocks jb with jb % C == c.  Lane s (chunk 0) returns F_s and
    // G'_s[:, 0:NB] = [A_s B_s] lands in LDS.
    __device__ static void linearize(const ProblemDev& P, const Lds& L, int H, int lane, const double (&w)[NB],
                                     double (&F)[NX], unsigned long long* tgp) {
        const int C = max(1, 64 / H);
        const int stage = lane % H;
        const int chunk = lane < C * H ? lane / H : C;  // chunk C: empty training range
        double x[NX], u[NU];
#pragma unroll
        for (int i = 0; i < NX; ++i) x[i] = __shfl(w[i], stage);
#pragma unroll
        for (int a = 0; a < NU; ++a) u[a] = __shfl(w[NX + a], stage);

        const double h = P.dt;
        double xs[4][NX], gm[4][NGP], gg[4][NGP][3];
        double gm0[NGP], gg0[NGP][3];
#ifdef GPMPC_TIMING
        unsigned long long tg0 = __builtin_amdgcn_s_memtime();
#endif
        eval_gps(P, L, false, x, u, stage, lane, H, gm0, gg0);  // GPs of u only: once per stage
#ifdef GPMPC_TIMING
        *tgp += __builtin_amdgcn_s_memtime() - tg0;
#endif
        double kprev[NX], acc[NX];
        const double cs[4] = {0.0, 0.5, 0.5, 1.0}, ws[4] = {1.0, 2.0, 2.0, 1.0};
#pragma unroll
        for (int s = 0; s < 4; ++s) {
#pragma unroll
            for (int i = 0; i < NX; ++i) xs[s][i] = (s == 0) ? x[i] : fma(cs[s] * h, kprev[i], x[i]);
#pragma unroll
            for (int g = 0; g < NGP; ++g) {
                gm[s][g] = gm0[g];
                gg[s][g][0] = gg0[g][0]; gg[s][g][1] = gg0[g][1]; gg[s][g][2] = gg0[g][2];
            }
#ifdef GPMPC_TIMING
            tg0 = __builtin_amdgcn_s_memtime();
#endif
            eval_gps(P, L, true, xs[s], u, stage, lane, H, gm[s], gg[s]);
#ifdef GPMPC_TIMING
            *tgp += __builtin_amdgcn_s_memtime() - tg0;
#endif
            M::f(P.params, xs[s], u, gm[s], kprev);
#pragma unroll
            for (int i = 0; i < NX; ++i) acc[i] = (s == 0) ? kprev[i] : fma(ws[s], kprev[i], acc[i]);
        }
#pragma unroll
        for (int i = 0; i < NX; ++i) F[i] = fma(h / 6.0, acc[i], x[i]);

        // tangent map of the RK4 step, column block by column block
        for (int jb = 0; jb < NCB; ++jb) {
            if (jb % C != (chunk < C ? chunk : -1)) continue;
            const int j0 = jb * CB;
            double V[NX][CB], dk[NX][CB], dF[NX][CB];
#pragma unroll
            for (int i = 0; i < NX; ++i)
#pragma unroll
                for (int j = 0; j < CB; ++j) { V[i][j] = (i == j0 + j) ? 1.0 : 0.0; dF[i][j] = V[i][j]; }
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                M::template tangent<CB>(P.params, xs[s], u, gm[s], gg[s], V, j0, dk);
                const double cn = (s < 3) ? cs[s + 1] * h : 0.0;
#pragma unroll
                for (int i = 0; i < NX; ++i)
#pragma unroll
                    for (int j = 0; j < CB; ++j) {
                        dF[i][j] = fma(h / 6.0 * ws[s], dk[i][j], dF[i][j]);
                        V[i][j] = fma(cn, dk[i][j], (i == j0 + j) ? 1.0 : 0.0);
                    }
            }
            if (chunk < C) {
                double* Gs = L.G + (size_t)stage * NX * GS;
#pragma unroll
                for (int i = 0; i < NX; ++i)
#pragma unroll
                    for (int j = 0; j < CB; ++j)
                        if (j0 + j < NB) Gs[i * GS + j0 + j] = dF[i][j];
            }
        }
    }

    // ------------------------------------------------------------------ Riccati recursion
    // Newton system of the IPM (HPIPM's backward/forward Riccati structure):
    //   min sum_k 1/2 w_k' diag(hq_k) w_k + gq_k' w_k   s.t.  dx_{k+1} = A_k dx_k + B_k du_k + c_k, dx_0 = 0
    // with w_k = [dx_k; du_k], G'_k = [A_k B_k c_k].  Sequential over stages, parallel over the
    // entries of each stage's small dense products: mfma_backward_h (one 16x16 tile per stage) or
    // mfma_backward_big (two column tiles, quad3d) below; the sweeps with the stored factorisation
    // on the 4-block MFMA (single tile) or the VALU with readlane broadcasts (wide stages).

    // ------------------------------------------------------------------ VALU sweeps in registers (wide stages)
    // Forward sweep dx_0 = 0, du_k = K'_k [dx_k; 1], dx_{k+1} = G'_k [dx_k; du_k; 1] with the state in
    // registers (lane i < NX: dx[i]) and broadcast by v_readlane: every lane forms the x-part of its
    // G' row and lanes NX..NB-1 (a = lane - NX) the input du_a from their K' row, then du is broadcast
    // the same way.  The stage operands (one G' row, one K' row per lane) are loaded a stage ahead.
    // Output: dxv.
    __device__ static void valu_forward_big(const Lds& L, int H, int lane) {
        lane = phase_lane(lane);
        const int row = lane < NX ? lane : 0;
        const int a = (lane >= NX && lane < NB) ? lane - NX : 0;
        const double* gp = L.G + (size_t)row * GS;
        const double* kp = L.K + (size_t)a * PS;
        struct St { double g[GS], kr[PS]; };
        auto load = [&](int k, St& st) {
#pragma unroll
            for (int j = 0; j < GS; ++j) st.g[j] = gp[(size_t)k * NX * GS + j];
#pragma unroll
            for (int j = 0; j < PS; ++j) st.kr[j] = kp[(size_t)k * NU * PS + j];
        };
        if (lane < NX) L.dxv[lane] = 0.0;
        double* out = (lane < NX) ? L.dxv + NX + lane : L.dummy;
        const int ost = (lane < NX) ? NX : 0;
        double x = 0.0;
        auto step = [&](const St& st) {
            double xs[NX];
#pragma unroll
            for (int j = 0; j < NX; ++j) xs[j] = readlane_d(x, j);
            double du0 = st.kr[NX], du1 = 0.0, ax0 = st.g[NB], ax1 = 0.0;
#pragma unroll
            for (int j = 0; j < NX; ++j) {
                if (j & 1) {
                    du1 = fma(st.kr[j], xs[j], du1);
                    ax1 = fma(st.g[j], xs[j], ax1);
                } else {
                    du0 = fma(st.kr[j], xs[j], du0);
                    ax0 = fma(st.g[j], xs[j], ax0);
                }
            }
            const double du = du0 + du1;
            double acc = ax0 + ax1;
#pragma unroll
            for (int b2 = 0; b2 < NU; ++b2) acc = fma(st.g[NX + b2], readlane_d(du, NX + b2), acc);
            x = acc;
            *out = acc;
            out += ost;
        };
        St s0, s1;
        load(0, s0);
        int k = 0;
        for (; k + 1 < H; k += 2) {
            load(k + 1, s1);
            step(s0);
            if (k + 2 < H) load(k + 2, s0);
            step(s1);
        }
        if (k < H) step(s0);
        WSYNC();
    }

    // Corrector vector sweep (HPIPM's solve with the stored factorisation), state in registers:
    //   pv = t_k + p_{k+1} (t_k = P_{k+1} c_k for all stages in parallel first),
    //   lane j < NB: s_j = gq_kj + sum_l G'_k[l][j] pv_l   (x-part of p_k for j < NX, gu_a for j = NX + a),
    //   p_k = s_x + K_k' gu (lanes < NX),  kff_k = -Ru_k^-1 gu (lanes NX..NB-1),
    // with pv and gu broadcast by v_readlane.  Outputs: p in P', kff in K'.
    // Scratch: t aliases hq (rewritten before the next factorisation).
    __device__ static void valu_vector_big(const Lds& L, int H, int lane) {
        lane = phase_lane(lane);
        double* T = L.hq;
        const int n = H * NX;
        auto t_entry = [&](int e) {
            const int k = e / NX, i = e - k * NX;
            const double* Pn = L.P + (size_t)(k + 1) * PP;
            const double* G = L.G + (size_t)k * NX * GS;
            double acc = 0.0;
#pragma unroll
            for (int l = 0; l < NX; ++l) acc = fma(Pn[i <= l ? pidx(i, l) : pidx(l, i)], G[l * GS + NB], acc);
            return acc;
        };
        for (int e0 = lane; e0 < n; e0 += 128) {
            const int e1 = e0 + 64;
            const bool has1 = e1 < n;
            const double a0 = t_entry(e0), a1 = t_entry(has1 ? e1 : e0);
            T[e0] = a0;
            if (has1) T[e1] = a1;
        }
        WSYNC();
        const int col = lane < NB ? lane : 0;
        const int row = lane < NX ? lane : 0;
        const int a = (lane >= NX && lane < NB) ? lane - NX : 0;
        struct St { double g[NX], kc[NU], ri[NU], gq, t; };
        auto load = [&](int k, St& st) {
            const double* G = L.G + (size_t)k * NX * GS + col;
#pragma unroll
            for (int l = 0; l < NX; ++l) st.g[l] = G[l * GS];
#pragma unroll
            for (int b2 = 0; b2 < NU; ++b2) {
                st.kc[b2] = L.K[(size_t)k * NU * PS + b2 * PS + row];
                st.ri[b2] = L.Rui[(size_t)k * NU * NU + a * NU + b2];
            }
            st.gq = L.gq[k * NBS + col];
            st.t = T[k * NX + row];
        };
        double p = (lane < NX) ? L.gq[H * NBS + lane] : 0.0;
        if (lane < NX) L.P[(size_t)H * PP + PO + lane] = p;
        double* pout = (lane < NX) ? L.P + (size_t)(H - 1) * PP + PO + lane : L.dummy;
        const int pst = (lane < NX) ? PP : 0;
        double* kout = (lane >= NX && lane < NB) ? L.K + (size_t)(H - 1) * NU * PS + a * PS + NX : L.dummy;
        const int kst = (lane >= NX && lane < NB) ? NU * PS : 0;
        auto step = [&](int k, const St& st) {
            const double pv = st.t + p;
            double s0 = st.gq, s1 = 0.0;
#pragma unroll
            for (int l = 0; l < NX; ++l) {
                const double pl = readlane_d(pv, l);
                if (l & 1) s1 = fma(st.g[l], pl, s1);
                else s0 = fma(st.g[l], pl, s0);
            }
            const double sj = s0 + s1;
            double pn = sj, kf = 0.0;
#pragma unroll
            for (int b2 = 0; b2 < NU; ++b2) {
                const double gu = readlane_d(sj, NX + b2);
                pn = fma(st.kc[b2], gu, pn);
                kf = fma(st.ri[b2], gu, kf);
            }
            p = pn;
            if (k >= 1) *pout = pn;   // p_0 is not needed
            pout -= pst;
            *kout = -kf;
            kout -= kst;
        };
        St s0, s1;
        load(H - 1, s0);
        int k = H - 1;
        for (; k >= 1; k -= 2) {
            load(k - 1, s1);
            step(k, s0);
            if (k >= 2) load(k - 2, s0);
            step(k - 1, s1);
        }
        if (k == 0) step(0, s0);
        WSYNC();
    }

    // Per-lane step of stage k from the Riccati solution: dd = [dx_k; du_k] and dpi_k.
    __device__ static void recover_step(const Lds& L, int H, int lane, double (&dd)[NB], double (&dpi)[NX]) {
        lane = phase_lane(lane);
        const bool on = lane <= H;
        double dx[NX], dxn[NX];
#pragma unroll
        for (int i = 0; i < NX; ++i) {
            dx[i] = (on && lane >= 1) ? L.dxv[(size_t)lane * NX + i] : 0.0;
            dxn[i] = (lane < H) ? L.dxv[(size_t)(lane + 1) * NX + i] : 0.0;
        }
#pragma unroll
        for (int i = 0; i < NX; ++i) dd[i] = dx[i];
        const int kk = min(lane, H - 1);
#pragma unroll
        for (int a = 0; a < NU; ++a) {
            double kr[PS];
#pragma unroll
            for (int j = 0; j < PS; ++j) kr[j] = L.K[(size_t)kk * NU * PS + a * PS + j];
            double du = kr[NX];
#pragma unroll
            for (int j = 0; j < NX; ++j) du = fma(kr[j], dx[j], du);
            dd[NX + a] = (lane < H) ? du : 0.0;
        }
        const double* Pn = L.P + (size_t)(kk + 1) * PP;
#pragma unroll
        for (int i = 0; i < NX; ++i) {
            double pr[PS];
#pragma unroll
            for (int j = 0; j < NX; ++j) pr[j] = Pn[i <= j ? pidx(i, j) : pidx(j, i)];
            pr[NX] = Pn[PO + i];
            double acc = pr[NX];
#pragma unroll
            for (int j = 0; j < NX; ++j) acc = fma(pr[j], dxn[j], acc);
            dpi[i] = (lane < H) ? -acc : 0.0;
        }
    }

    // ------------------------------------------------------------------ Riccati on MFMA (NB+1 <= 16)
    // Tile conventions of v_mfma_f64_16x16x4_f64 (lane l, lr = l>>4, lc = l&15):
    //   A operand of K-step s: A[lc][4s+lr];  B operand: B[4s+lr][lc];  C/D register r: D[lr+4r][lc].
    // A matrix held in C layout is therefore directly the B operand of the next product, and
    // a SYMMETRIC matrix in C layout is also its own A operand.  P (symmetric) stays in
    // registers from stage to stage; per stage:
    //   W = P G' (+ p on column NB)      2 MFMAs, B = G' rows (LDS)
    //   M = G'^T W + [diag(hq) | gq]     2 MFMAs, A = the same G' registers, B = W registers
    //   Schur onto the state block       Ru by readlane, row/column slices by lane shuffles
    __device__ static int pidx(int i, int j) { return i * NX - (i * (i - 1)) / 2 + (j - i); }  // i <= j < NX

    // Riccati factorisation on v_mfma_f64_16x16x4 in the homogeneous tile layout: tile index t of
    // the 16-wide operands is x_t for t < NX, the affine "1" at CI = NX, u_a at UI + a (UI = 8),
    // zero elsewhere.  The affine column c of G'_k becomes row/column CI of [G'_k; e_CI]
    // (G'' row CI = e_CI, the one slot of the LDS zero block), so W' = P'_{k+1} G'' needs no
    // C-init from P' (p_{k+1} rides in row CI of P', inside the K range 0..7 of the two MFMAs),
    // and M' = G''^T W' + D (D: diag(hq), gq in row and column CI) keeps P'_k = Schur(M')
    // symmetric, so the Schur MFMA's output registers are the next stage's A operand as they
    // stand: no select or copy between the Schur product and the next W' on the recursion.
    // The u rows sit at 8..8+NU-1 = lane groups 0..NU-1 of element 2: the Schur A operand needs no
    // lane move.  Stores of stage k are issued after stage k-1's W' products (sched_barrier), off
    // the chain.  Outputs: packed P', K' = [K | kff], Ru^-1 per stage.
    __device__ static bool mfma_backward_h(const Lds& L, int H, int lane) {
        lane = phase_lane(lane);
        const int lr = lane >> 4, lc = lane & 15;
        constexpr int CI = NX, UI = 8;
        static_assert(NX + 1 <= 8 && NU <= 2 && UI + NU <= 16, "homogeneous tile layout");
        // tile index -> G' column (-1: structurally zero) and stage variable (-1: none)
        auto gcol = [](int t) { return t < NX ? t : (t == CI ? NB : ((t >= UI && t < UI + NU) ? NX + t - UI : -1)); };
        auto svar = [](int t) { return t < NX ? t : ((t >= UI && t < UI + NU) ? NX + t - UI : -1); };
        const int gc_lc = gcol(lc), sv_lc = svar(lc);
        double pn[2];
#pragma unroll
        for (int r = 0; r < 2; ++r) {   // P'_H: diag(hq_H[x]), gq_H[x] in row and column CI
            const int t = lr + 4 * r;
            double v = 0.0;
            if (t < NX && lc < NX) v = (t == lc) ? L.hq[H * NBS + t] : 0.0;
            else if (t < NX && lc == CI) v = L.gq[H * NBS + t];
            else if (t == CI && lc < NX) v = L.gq[H * NBS + lc];
            pn[r] = v;
        }
        {   // P'_H (packed) for the multiplier recovery of stage H-1
            double* PH = L.P + (size_t)H * PP;
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                const int t = lr + 4 * r;
                if (t < NX) {
                    if (lc == CI) PH[PO + t] = pn[r];
                    else if (lc < NX && t <= lc) PH[pidx(t, lc)] = pn[r];
                }
            }
        }
        bool ok = true;
        // G'' rows 4s + lr (K index), column lc: per-lane (base, stride) streams
        const double* pg[2];
        int gst[2];
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
            const int t = lr + 4 * s2;
            const bool ld = t < NX && gc_lc >= 0;
            const bool one = t == CI && lc == CI;
            pg[s2] = ld ? L.G + (size_t)(H - 1) * NX * GS + t * GS + gc_lc : L.zero + (one ? 7 : 0);
            gst[s2] = ld ? NX * GS : 0;
        }
        // C-init of M' (rows lr + 4r, r = 0..2): hq on the diagonal, gq in row and column CI
        const double* pd[3];
        int dst[3];
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            const int t = lr + 4 * r, sv_t = svar(t);
            const double* base = L.zero;
            bool on = false;
            if (sv_t >= 0 && t == lc) { base = L.hq + sv_t; on = true; }
            else if (sv_t >= 0 && lc == CI) { base = L.gq + sv_t; on = true; }
            else if (t == CI && sv_lc >= 0) { base = L.gq + sv_lc; on = true; }
            pd[r] = on ? base + (size_t)(H - 1) * NBS : L.zero;
            dst[r] = on ? NBS : 0;
        }
        struct Stage { double g[2], d[3]; };
        auto load_stage = [&](Stage& st) {
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                st.g[q] = *pg[q];
                pg[q] -= gst[q];
            }
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                st.d[q] = *pd[q];
                pd[q] -= dst[q];
            }
        };
        // store streams (stages H-1 .. 0), dummy slot with stride 0 for entries not stored
        double* sp[2];
        int sp_st[2];
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const int t = lr + 4 * r;
            const bool st = t < NX && ((lc == CI) || (lc < NX && t <= lc));
            const int idx = (lc == CI) ? PO + t : pidx(t < lc ? t : lc, t < lc ? lc : t);
            sp[r] = st ? L.P + (size_t)(H - 1) * PP + idx : L.dummy;
            sp_st[r] = st ? PP : 0;
        }
        const bool kst = lr < NU && (lc < NX || lc == CI);
        double* sk = kst ? L.K + (size_t)(H - 1) * NU * PS + lr * PS + (lc == CI ? NX : lc) : L.dummy;
        const int sk_st = kst ? NU * PS : 0;
        const bool rst = lane < NU * NU;
        double* srui = rst ? L.Rui + (size_t)(H - 1) * NU * NU + lane : L.dummy;
        const int srui_st = rst ? NU * NU : 0;
        double pend_p[2] = {0.0, 0.0}, pend_k = 0.0, pend_r = 0.0;
        auto flush = [&]() {
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                *sp[r] = pend_p[r];
                sp[r] -= sp_st[r];
            }
            *sk = pend_k;
            sk -= sk_st;
            *srui = pend_r;
            srui -= srui_st;
        };
        // fl: the previous stage's stores are pending (every stage but the first, which is peeled off the
        // loop: no branch inside the stage); issued after this stage's W' products, off the chain
        auto stage = [&](const Stage& sd, auto fl) {
            f64x4 w = mfma64(pn[0], sd.g[0], f64x4{0.0, 0.0, 0.0, 0.0});
            w = mfma64(pn[1], sd.g[1], w);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (decltype(fl)::value) flush();
            __builtin_amdgcn_sched_barrier(0);
            f64x4 m = mfma64(sd.g[0], w[0], f64x4{sd.d[0], sd.d[1], sd.d[2], 0.0});
            m = mfma64(sd.g[1], w[1], m);
            double Ru[NU][NU];
#pragma unroll
            for (int a = 0; a < NU; ++a)
#pragma unroll
                for (int b2 = a; b2 < NU; ++b2) {
                    Ru[a][b2] = readlane_d(m[2], (a << 4) | (UI + b2));
                    Ru[b2][a] = Ru[a][b2];
                }
            const double mu = m[2];   // lane (a, c) <- M'[UI + a][c]
            double kb, Ri[NU][NU];
            if constexpr (NU == 1) {
                ok = ok && (Ru[0][0] > 0.0);
                const double id = fast_rcp(Ru[0][0]);
                Ri[0][0] = id;
                kb = -id * mu;
            } else {
                const double det = Ru[0][0] * Ru[1][1] - Ru[0][1] * Ru[0][1];
                ok = ok && (Ru[0][0] > 0.0) && (det > 0.0);
                const double mo = xor16_d(mu);
                const double num = fma((lr & 1) ? Ru[0][0] : Ru[1][1], mu, -Ru[0][1] * mo);   // adj(Ru) M'_u
                // id = r (1 + e + e^2): kb = t + t (e + e^2) with t = -num r formed beside e
                const double r0 = __builtin_amdgcn_rcp(det);
                const double e = fma(-det, r0, 1.0);
                const double ee = fma(e, e, e);
                const double t = num * -r0;
                const double id = fma(r0, ee, r0);
                kb = fma(t, ee, t);
                Ri[0][0] = Ru[1][1] * id;
                Ri[1][1] = Ru[0][0] * id;
                Ri[0][1] = Ri[1][0] = -Ru[0][1] * id;
            }
            const f64x4 pk = mfma64(lr < NU ? mu : 0.0, kb, m);   // P'_k = M' + M'_{.u} K'
            double rv = Ri[0][0];
            if constexpr (NU == 2) rv = (lane == 0) ? Ri[0][0] : ((lane == 3) ? Ri[1][1] : Ri[0][1]);
            pend_p[0] = pk[0];
            pend_p[1] = pk[1];
            pend_k = kb;
            pend_r = rv;
            pn[0] = pk[0];
            pn[1] = pk[1];
        };
        Stage s0, s1;
        load_stage(s0);
        load_stage(s1);
        stage(s0, std::false_type{});
        int k = H - 2;
        for (; k >= 1; k -= 2) {
            load_stage(s0);
            stage(s1, std::true_type{});
            load_stage(s1);   // (past stage 0 on the last pass: the zero / previous slots, never used)
            stage(s0, std::true_type{});
        }
        if (k == 0) stage(s1, std::true_type{});
        flush();
        return ok;
    }

    // ------------------------------------------------------------------ Riccati on MFMA, NX <= 12, NU <= 4
    // For stages wider than one 16x16 tile (quad3d: NX = 12, NU = 4, NB + 1 = 17) the products are
    // split over two column tiles of v_mfma_f64_16x16x4_f64: T1 = [x | c] (c at tile column NX) and
    // T2 = u.  With P' = [P | p] in the C layout (rows 0..NX-1 in elements 0..KS-1, p in column NX):
    //   W1 = P' [G'_x | c] + p e_NX      W2 = P' G'_u                       (KS chained MFMAs each)
    //   M11 = T1^T W1 + [diag(hq_x) | gq_x]   M21 = T2^T W1 + [0 | gq_u]   M22 = T2^T W2 + diag(hq_u)
    //   Ru = M22 (readlane), Ru^-1 by 2x2 blocks (two reciprocals), K' = -Ru^-1 M21 per lane from the
    //   four u rows of its column (permlane16/32 swaps), P'_k = M11 + M21^T K' (one MFMA).
    // M21's element 0 (lane (a, j) = M21[a][j]) is both the Schur product's A operand and the
    // right-hand side of K'.  Outputs as mfma_backward_h (packed P', K', Ru^-1).
    static constexpr bool kMfmaBig = !kMfma && NX <= 12 && NX + 1 <= 16 && NU == 4;
    __device__ static bool mfma_backward_big(const Lds& L, int H, int lane) {
        lane = phase_lane(lane);
        if constexpr (!kMfmaBig) {
            return false;
        } else {
        const int lr = lane >> 4, lc = lane & 15;
        constexpr int KS = (NX + 3) / 4;   // K steps over the state rows
        double pn[KS];
#pragma unroll
        for (int r = 0; r < KS; ++r) {   // P'_H = [diag(hq_H[x]) | gq_H[x]]
            const int t = lr + 4 * r;
            double v = 0.0;
            if (t < NX && lc < NX) v = (t == lc) ? L.hq[H * NBS + t] : 0.0;
            else if (t < NX && lc == NX) v = L.gq[H * NBS + t];
            pn[r] = v;
        }
        {
            double* PH = L.P + (size_t)H * PP;
#pragma unroll
            for (int r = 0; r < KS; ++r) {
                const int t = lr + 4 * r;
                if (t < NX) {
                    if (lc == NX) PH[PO + t] = pn[r];
                    else if (lc < NX && t <= lc) PH[pidx(t, lc)] = pn[r];
                }
            }
        }
        bool ok = true;
        // stage operand streams (stages H-1 .. 0)
        const double* pa[KS];   // T1 = [G'_x | c]: row 4s + lr, tile column lc
        const double* pb[KS];   // T2 = G'_u
        int ast[KS], bst[KS];
#pragma unroll
        for (int s2 = 0; s2 < KS; ++s2) {
            const int t = lr + 4 * s2;
            const bool la = t < NX && lc <= NX;
            const bool lb = t < NX && lc < NU;
            pa[s2] = la ? L.G + (size_t)(H - 1) * NX * GS + t * GS + (lc < NX ? lc : NB) : L.zero;
            pb[s2] = lb ? L.G + (size_t)(H - 1) * NX * GS + t * GS + NX + lc : L.zero;
            ast[s2] = la ? NX * GS : 0;
            bst[s2] = lb ? NX * GS : 0;
        }
        const double* pd11[KS];   // M11 C-init: hq_x on the diagonal, gq_x in column NX
        int d11st[KS];
#pragma unroll
        for (int r = 0; r < KS; ++r) {
            const int t = lr + 4 * r;
            const bool dg = t < NX && t == lc, gc = t < NX && lc == NX;
            pd11[r] = dg ? L.hq + (size_t)(H - 1) * NBS + t : (gc ? L.gq + (size_t)(H - 1) * NBS + t : L.zero);
            d11st[r] = (dg || gc) ? NBS : 0;
        }
        const bool g21 = lr < NU && lc == NX, d22 = lr < NU && lc == lr;
        const double* pd21 = g21 ? L.gq + (size_t)(H - 1) * NBS + NX + lr : L.zero;
        const double* pd22 = d22 ? L.hq + (size_t)(H - 1) * NBS + NX + lr : L.zero;
        const int d21st = g21 ? NBS : 0, d22st = d22 ? NBS : 0;
        struct Stage { double a[KS], b[KS], d11[KS], d21, d22; };
        auto load_stage = [&](Stage& st) {
#pragma unroll
            for (int q = 0; q < KS; ++q) {
                st.a[q] = *pa[q];
                pa[q] -= ast[q];
                st.b[q] = *pb[q];
                pb[q] -= bst[q];
                st.d11[q] = *pd11[q];
                pd11[q] -= d11st[q];
            }
            st.d21 = *pd21;
            pd21 -= d21st;
            st.d22 = *pd22;
            pd22 -= d22st;
        };
        // store streams
        double* sp[KS];
        int sp_st[KS];
#pragma unroll
        for (int r = 0; r < KS; ++r) {
            const int t = lr + 4 * r;
            const bool st = t < NX && ((lc == NX) || (lc < NX && t <= lc));
            const int idx = (lc == NX) ? PO + t : pidx(t < lc ? t : lc, t < lc ? lc : t);
            sp[r] = st ? L.P + (size_t)(H - 1) * PP + idx : L.dummy;
            sp_st[r] = st ? PP : 0;
        }
        const bool kst = lr < NU && lc <= NX;
        double* sk = kst ? L.K + (size_t)(H - 1) * NU * PS + lr * PS + lc : L.dummy;
        const int sk_st = kst ? NU * PS : 0;
        const bool rst = lr < NU && lc < NU;
        double* srui = rst ? L.Rui + (size_t)(H - 1) * NU * NU + lr * NU + lc : L.dummy;
        const int srui_st = rst ? NU * NU : 0;
        const unsigned ma0 = lr == 0 ? ~0u : 0u, ma1 = lr == 1 ? ~0u : 0u, ma2 = lr == 2 ? ~0u : 0u;
        const unsigned mb1 = (lr & 2) ? ~0u : 0u, mb2 = (lr & 1) ? ~0u : 0u, mb3 = ((lr ^ (lr >> 1)) & 1) ? ~0u : 0u;
        const int tsel = lc ^ lr;
        const unsigned mt0 = tsel == 0 ? ~0u : 0u, mt1 = tsel == 1 ? ~0u : 0u, mt2 = tsel == 2 ? ~0u : 0u;
        auto stage = [&](const Stage& sd) {
            f64x4 w1 = {0.0, 0.0, 0.0, 0.0}, w2 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int r = 0; r < KS; ++r) w1[r] = (lc == NX) ? pn[r] : 0.0;
#pragma unroll
            for (int s2 = 0; s2 < KS; ++s2) {
                w1 = mfma64(pn[s2], sd.a[s2], w1);
                w2 = mfma64(pn[s2], sd.b[s2], w2);
            }
            f64x4 m22 = {sd.d22, 0.0, 0.0, 0.0}, m21 = {sd.d21, 0.0, 0.0, 0.0}, m11 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int r = 0; r < KS; ++r) m11[r] = sd.d11[r];
#pragma unroll
            for (int s2 = 0; s2 < KS; ++s2) {
                m22 = mfma64(sd.b[s2], w2[s2], m22);
                m21 = mfma64(sd.b[s2], w1[s2], m21);
                m11 = mfma64(sd.a[s2], w1[s2], m11);
            }
            // Ru = M22[0..3][0..3] and its inverse by 2x2 blocks [[A, B], [B^T, C]]
            const double mz = m22[0];
            const double a00 = readlane_d(mz, 0), a01 = readlane_d(mz, 1), a11 = readlane_d(mz, 16 + 1);
            const double b00 = readlane_d(mz, 2), b01 = readlane_d(mz, 3), b10 = readlane_d(mz, 16 + 2),
                         b11 = readlane_d(mz, 16 + 3);
            const double c00 = readlane_d(mz, 32 + 2), c01 = readlane_d(mz, 32 + 3), c11 = readlane_d(mz, 48 + 3);
            const double dA = fma(a00, a11, -a01 * a01);
            const double iA = fast_rcp(dA);
            const double A00 = a11 * iA, A01 = -a01 * iA, A11 = a00 * iA;
            const double X00 = fma(A00, b00, A01 * b10), X01 = fma(A00, b01, A01 * b11);
            const double X10 = fma(A01, b00, A11 * b10), X11 = fma(A01, b01, A11 * b11);
            const double S00 = c00 - fma(b00, X00, b10 * X10), S01 = c01 - fma(b00, X01, b10 * X11);
            const double S11 = c11 - fma(b01, X01, b11 * X11);
            const double dS = fma(S00, S11, -S01 * S01);
            ok = ok && (a00 > 0.0) && (dA > 0.0) && (dS > 0.0);
            const double iS = fast_rcp(dS);
            const double C00 = S11 * iS, C01 = -S01 * iS, C11 = S00 * iS;
            const double Y00 = fma(X00, C00, X01 * C01), Y01 = fma(X00, C01, X01 * C11);
            const double Y10 = fma(X10, C00, X11 * C01), Y11 = fma(X10, C01, X11 * C11);
            const double Z00 = A00 + fma(Y00, X00, Y01 * X01), Z01 = A01 + fma(Y00, X10, Y01 * X11);
            const double Z11 = A11 + fma(Y10, X10, Y11 * X11);
            // Ru^-1 = [[Z, -Y], [-Y^T, C]]; row a, column a ^ t, for lane group a (branch-free selects)
            const double c0 = bsel(ma0, Z00, bsel(ma1, Z11, bsel(ma2, C00, C11)));
            const double c1 = bsel(mb1, C01, Z01);
            const double c2 = bsel(mb2, -Y11, -Y00);                  // (0,2) = -Y00, (1,3) = -Y11
            const double c3 = bsel(mb3, -Y10, -Y01);                  // (0,3) = -Y01, (1,2) = -Y10
            // the four u rows of this lane's column of M21 (lane group b holds row b)
            const double v0 = m21[0], v1 = xor16_d(v0), v2 = xor32_d(v0), v3 = xor32_d(v1);
            const double kb = -fma(c0, v0, fma(c1, v1, fma(c2, v2, c3 * v3)));
            const f64x4 pk = mfma64(lr < NU ? v0 : 0.0, kb, m11);   // P'_k = M11 + M21^T K'
            // stores: P' (packed), K' (feedback + kff), Ru^-1 (lane (a, c): column c = a ^ t)
            const double rv = bsel(mt0, c0, bsel(mt1, c1, bsel(mt2, c2, c3)));
#pragma unroll
            for (int r = 0; r < KS; ++r) {
                *sp[r] = pk[r];
                sp[r] -= sp_st[r];
                pn[r] = pk[r];
            }
            *sk = kb;
            sk -= sk_st;
            *srui = rv;
            srui -= srui_st;
        };
        Stage s0, s1;
        load_stage(s0);
        int k = H - 1;
        for (; k >= 1; k -= 2) {
            load_stage(s1);
            stage(s0);
            if (k >= 2) load_stage(s0);
            stage(s1);
        }
        if (k == 0) stage(s0);
        return ok;
        }
    }

    // Closed-loop stage maps A'_k = [A + B K | B kff + c] (all stages in parallel); only the
    // affine column when the factorisation is unchanged (corrector).
    template <bool full>
    __device__ static void acl_phase(const Lds& L, int H, int lane) {
        lane = phase_lane(lane);
        if constexpr (full) {
            // one row (k, i) of A'_k per lane and pass: the G'_k row and K'_k are contiguous reads,
            // the PS outputs one contiguous store
            for (int e = lane; e < H * NX; e += 64) {
                const int k = e / NX, i = e - k * NX;
                const double* G = L.G + (size_t)k * NX * GS + i * GS;
                const double* Kk = L.K + (size_t)k * NU * PS;
                double g[GS], kr[NU][PS];
#pragma unroll
                for (int j = 0; j < GS; ++j) g[j] = G[j];
#pragma unroll
                for (int a = 0; a < NU; ++a)
#pragma unroll
                    for (int j = 0; j < PS; ++j) kr[a][j] = Kk[a * PS + j];
                double* out = L.Acl + (size_t)k * NX * PS + i * PS;
#pragma unroll
                for (int j = 0; j < PS; ++j) {
                    double acc = (j < NX) ? g[j] : g[NB];
#pragma unroll
                    for (int a = 0; a < NU; ++a) acc = fma(g[NX + a], kr[a][j], acc);
                    out[j] = acc;
                }
            }
        } else {
            // three entries per pass, all computed before any is stored (the stores to A' would
            // otherwise order the next entry's reads behind them)
            const int n = H * NX;
            for (int e0 = lane; e0 < n; e0 += 192) {
                double acc[3];
#pragma unroll
                for (int r = 0; r < 3; ++r) {
                    const int e = min(e0 + 64 * r, n - 1);
                    const int k = e / NX, i = e - k * NX;
                    const double* G = L.G + (size_t)k * NX * GS + i * GS;
                    const double* Kk = L.K + (size_t)k * NU * PS;
                    acc[r] = G[NB];
#pragma unroll
                    for (int a = 0; a < NU; ++a) acc[r] = fma(G[NX + a], Kk[a * PS + NX], acc[r]);
                }
#pragma unroll
                for (int r = 0; r < 3; ++r) {
                    const int e = e0 + 64 * r;
                    if (e < n) {
                        const int k = e / NX, i = e - k * NX;
                        L.Acl[(size_t)k * NX * PS + i * PS + NX] = acc[r];
                    }
                }
            }
        }
    }

    // ------------------------------------------------------------------ sweeps on v_mfma_f64_4x4x4_4b
    // An affine recurrence y_{k+1} = M_k y_k over the homogeneous 8-vector y = [v (NX); 1; 0] (4 <= NX <= 6)
    // as ONE 4-block MFMA per stage.  Lane l = 16r + 4b + c: the instruction's block b takes A_b[m][k]
    // from lane (k, b, m) and B_b[k][n] from lane (k, b, n) and writes D_b[m][n] to lane (m, b, n)
    // (tools/probe_mfma4x4.hip), so D lands in the B layout of the next stage.  Blocks:
    //   b = 0: M_ll y_lo   b = 1: M_lh y_hi   b = 2: M_hh y_hi   b = 3: M_hl y_lo
    // (lo/hi = rows or columns 0..3 / 4..7), every column n carrying the same vector.  Then
    //   S = D + (D of the next quad)          quad 0: y'_lo, quad 2: y'_hi   (DPP row_ror:12 + one add)
    //   B' = S, quads 1 and 3 <- next quad     quads (lo, hi, hi, lo)         (one bank-masked DPP move)
    // so a stage is MFMA -> DPP -> add -> DPP on the chain instead of a 6-term dot product behind
    // v_readlane broadcasts.  The stage operands M_k are loaded one stage ahead (one LDS read per lane).
    struct Mfma4Lane {
        int r, b, c, row, col;
    };
    __device__ static Mfma4Lane mfma4_lane(int lane) {
        Mfma4Lane q;
        q.r = lane >> 4;
        q.b = (lane >> 2) & 3;
        q.c = lane & 3;
        q.row = ((q.b >> 1) ? 4 : 0) + q.c;                    // row of M_k this lane supplies (A_b[m = c])
        q.col = ((q.b == 1 || q.b == 2) ? 4 : 0) + q.r;        // column (A_b[k = r])
        return q;
    }
    // y (B layout) of the homogeneous vector [v; 1; 0] with v[i] = vget(i)
    template <class F>
    __device__ static double mfma4_vec(const Mfma4Lane& q, F&& vget) {
        const int idx = ((q.b == 1 || q.b == 2) ? 4 : 0) + q.r;
        return idx < NX ? vget(idx) : (idx == NX ? 1.0 : 0.0);
    }
    // One stage: D = M_k y; returns y_{k+1} in the B layout and the stage output in `s`
    // (lanes (r, 0, c): v'[r], lanes (r, 2, c): v'[4 + r]).
    __device__ static double mfma4_stage(double a, double y, double& s) {
        const double d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, y, 0.0, 0, 0, 0);
        s = d + dpp_d<0x12C>(d);                  // row_ror:12: lane i <- lane (i + 4) mod 16
        return dpp_merge<0x12C, 0xA>(s, s);       // quads 1, 3 <- quads 2, 0
    }

    // Forward sweep: dx_0 = 0, dx_{k+1} = A'_k [dx_k; 1]  (M_k = [A'_k; e_NX]).  Masked lanes read the
    // LDS zero slot (stride 0) and the homogeneous corner the one slot, so the stage operand is one
    // unconditional load issued a stage ahead.
    __device__ static void mfma4_forward(const Lds& L, int H, int lane) {
        lane = phase_lane(lane);
        static_assert(NX >= 4 && NX + 1 <= 8, "homogeneous 8-vector");
        {
            const Mfma4Lane q = mfma4_lane(lane);
            const bool ld = q.row < NX && q.col <= NX;
            const double* src = ld ? L.Acl + q.row * PS + q.col : L.zero + ((q.row == NX && q.col == NX) ? 7 : 0);
            const int st = ld ? NX * PS : 0;
            const bool stlo = q.b == 0 && q.c == 0 && q.r < NX;
            const bool sthi = q.b == 2 && q.c == 0 && 4 + q.r < NX;
            double* out = stlo ? L.dxv + NX + q.r : (sthi ? L.dxv + NX + 4 + q.r : L.dummy);
            const int ost = (stlo || sthi) ? NX : 0;
            if (lane < NX) L.dxv[lane] = 0.0;
            double y = mfma4_vec(q, [](int) { return 0.0; });
            double an = *src;
            for (int k = 0; k < H; ++k) {
                const double a = an;
                src += (k + 1 < H) ? st : 0;
                an = *src;
                double s;
                y = mfma4_stage(a, y, s);
                *out = s;
                out += ost;
            }
        }
    }

    // Corrector right-hand side with the factorisation unchanged (the Riccati "solve" of HPIPM):
    //   p_k = vt_k + A_cl,k^T p_{k+1},  vt_k = q_k + K_k^T r_k + A_cl,k^T P_{k+1} c_k,  p_H = q_H,
    //   kff_k = -Ru_k^-1 (r_k + B_k^T (P_{k+1} c_k + p_{k+1})),
    // with [q; r] = gq.  Only the p recurrence is sequential (one v_mfma_f64_4x4x4_4b + DPP merge per
    // stage, mfma4_stage); t_k = P_{k+1} c_k and vt_k are built for all stages in parallel.
    // Scratch: t aliases hq (rewritten before the next factorisation), vt aliases dxv.
    __device__ static void mfma4_vector_backward(const Lds& L, int H, int lane) {
        lane = phase_lane(lane);
        double* T = L.hq;
        double* VT = L.dxv;
        // entries (k, i) two per pass, both computed before either is stored (T and VT alias other
        // LDS buffers, so a store would otherwise order the next entry's reads behind it)
        // (each pass issues every load of its entries before a scheduling barrier: loads interleaved
        // with their uses issue a few at a time)
        const int n = H * NX;
        struct TOps { double pr[NX], gc[NX]; };
        auto t_load = [&](int e, TOps& o) {
            const int k = e / NX, i = e - k * NX;
            const double* Pn = L.P + (size_t)(k + 1) * PP;
            const double* G = L.G + (size_t)k * NX * GS;
#pragma unroll
            for (int l = 0; l < NX; ++l) {
                o.pr[l] = Pn[i <= l ? pidx(i, l) : pidx(l, i)];
                o.gc[l] = G[l * GS + NB];
            }
        };
        auto t_dot = [](const TOps& o) {
            double acc = 0.0;
#pragma unroll
            for (int l = 0; l < NX; ++l) acc = fma(o.pr[l], o.gc[l], acc);
            return acc;
        };
        for (int e0 = lane; e0 < n; e0 += 128) {
            const int e1 = e0 + 64;
            const bool has1 = e1 < n;
            TOps o0, o1;
            t_load(e0, o0);
            t_load(has1 ? e1 : e0, o1);
            __builtin_amdgcn_sched_barrier(0);
            const double a0 = t_dot(o0), a1 = t_dot(o1);
            T[e0] = a0;
            if (has1) T[e1] = a1;
        }
        WSYNC();
        struct VOps { double g0, gu[NU], kc[NU], ac[NX], tk[NX]; };
        auto vt_load = [&](int e, VOps& o) {
            const int k = e / NX, i = e - k * NX;
            const double* A = L.Acl + (size_t)k * NX * PS;
            const double* Kk = L.K + (size_t)k * NU * PS;
            o.g0 = L.gq[k * NBS + i];
#pragma unroll
            for (int a = 0; a < NU; ++a) {
                o.kc[a] = Kk[a * PS + i];
                o.gu[a] = L.gq[k * NBS + NX + a];
            }
#pragma unroll
            for (int l = 0; l < NX; ++l) {
                o.ac[l] = A[l * PS + i];
                o.tk[l] = T[k * NX + l];
            }
        };
        auto vt_dot = [](const VOps& o) {
            double acc = o.g0;
#pragma unroll
            for (int a = 0; a < NU; ++a) acc = fma(o.kc[a], o.gu[a], acc);
#pragma unroll
            for (int l = 0; l < NX; ++l) acc = fma(o.ac[l], o.tk[l], acc);
            return acc;
        };
        for (int e0 = lane; e0 < n; e0 += 128) {
            const int e1 = e0 + 64;
            const bool has1 = e1 < n;
            VOps o0, o1;
            vt_load(e0, o0);
            vt_load(has1 ? e1 : e0, o1);
            __builtin_amdgcn_sched_barrier(0);
            const double a0 = vt_dot(o0), a1 = vt_dot(o1);
            VT[e0] = a0;
            if (has1) VT[e1] = a1;
        }
        WSYNC();
        {
            // p_k = vt_k + A'_k^T p_{k+1} as the homogeneous recurrence [p_k; 1] = M_k [p_{k+1}; 1],
            // M_k = [[A'_k[:, :NX]^T, vt_k], [0, 1]] (mfma4_stage), stages H-1 .. 0
            const Mfma4Lane q = mfma4_lane(lane);
            const bool lda = q.row < NX && q.col < NX, ldv = q.row < NX && q.col == NX;
            const double* src = lda ? L.Acl + (size_t)(H - 1) * NX * PS + q.col * PS + q.row
                                    : (ldv ? VT + (size_t)(H - 1) * NX + q.row
                                           : L.zero + ((q.row == NX && q.col == NX) ? 7 : 0));
            const int st = lda ? NX * PS : (ldv ? NX : 0);
            if (lane < NX) L.P[(size_t)H * PP + PO + lane] = L.gq[H * NBS + lane];
            double y = mfma4_vec(q, [&](int i) { return L.gq[H * NBS + i]; });
            const bool stlo = q.b == 0 && q.c == 0 && q.r < NX;
            const bool sthi = q.b == 2 && q.c == 0 && 4 + q.r < NX;
            double* out = stlo ? L.P + (size_t)(H - 1) * PP + PO + q.r
                               : (sthi ? L.P + (size_t)(H - 1) * PP + PO + 4 + q.r : L.dummy);
            const int ost = (stlo || sthi) ? PP : 0;
            double an = *src;
            for (int k = H - 1; k >= 0; --k) {
                const double a = an;
                src -= (k >= 1) ? st : 0;
                an = *src;
                double sv;
                y = mfma4_stage(a, y, sv);
                *out = sv;
                out -= ost;
            }
        }
        WSYNC();
        for (int e = lane; e < H * NU; e += 64) {
            const int k = e / NU, a = e - k * NU;
            const double* G = L.G + (size_t)k * NX * GS;
            const double* pn = L.P + (size_t)(k + 1) * PP + PO;
            double gb[NU][NX], tp[NX], gqv[NU], rui[NU];
#pragma unroll
            for (int b2 = 0; b2 < NU; ++b2) {
                gqv[b2] = L.gq[k * NBS + NX + b2];
                rui[b2] = L.Rui[(size_t)k * NU * NU + a * NU + b2];
#pragma unroll
                for (int l = 0; l < NX; ++l) gb[b2][l] = G[l * GS + NX + b2];
            }
#pragma unroll
            for (int l = 0; l < NX; ++l) tp[l] = T[k * NX + l] + pn[l];
            __builtin_amdgcn_sched_barrier(0);
            double kf = 0.0;
#pragma unroll
            for (int b2 = 0; b2 < NU; ++b2) {
                double acc = gqv[b2];
#pragma unroll
                for (int l = 0; l < NX; ++l) acc = fma(gb[b2][l], tp[l], acc);
                kf = fma(rui[b2], acc, kf);
            }
            L.K[(size_t)k * NU * PS + a * PS + NX] = -kf;
        }
        WSYNC();
    }

    // Per-lane step from the MFMA Riccati solution (packed P').
    __device__ static void recover_step_mfma(const Lds& L, int H, int lane, double (&dd)[NB], double (&dpi)[NX]) {
        lane = phase_lane(lane);
        const bool on = lane <= H;
        const int kk = min(lane, H - 1);
        double dx[NX], dxn[NX];
#pragma unroll
        for (int i = 0; i < NX; ++i) {
            dx[i] = (on && lane >= 1) ? L.dxv[(size_t)lane * NX + i] : 0.0;
            dxn[i] = L.dxv[(size_t)(kk + 1) * NX + i];
        }
#pragma unroll
        for (int i = 0; i < NX; ++i) dd[i] = dx[i];
#pragma unroll
        for (int a = 0; a < NU; ++a) {
            double kr[PS];
#pragma unroll
            for (int j = 0; j < PS; ++j) kr[j] = L.K[(size_t)kk * NU * PS + a * PS + j];
            double du = kr[NX];
#pragma unroll
            for (int j = 0; j < NX; ++j) du = fma(kr[j], dx[j], du);
            dd[NX + a] = (lane < H) ? du : 0.0;
        }
        const double* Pn = L.P + (size_t)(kk + 1) * PP;
        double pp[PP];
#pragma unroll
        for (int q = 0; q < PP; ++q) pp[q] = Pn[q];
#pragma unroll
        for (int i = 0; i < NX; ++i) {
            double acc = pp[NX * (NX + 1) / 2 + i];
#pragma unroll
            for (int j = 0; j < NX; ++j) acc = fma(pp[i <= j ? pidx(i, j) : pidx(j, i)], dxn[j], acc);
            dpi[i] = (lane < H) ? -acc : 0.0;
        }
    }

    // ------------------------------------------------------------------ segment-parallel Newton solve (kSeg)
    // Segment w = stages seg_start(w) .. seg_start(w + 1) - 1 on wave seg_wave(w) (tools/seg2_proto.py
    // is the numpy model of the two-segment form, tests/test_segment_model_cpu.py of any count, against
    // the dense KKT solve).
    __host__ __device__ static int seg_start(int w, int H) { return (w * H) / NSEG; }
    __device__ static int lam_of(int t) { return (t >= LI && t < LI + NX) ? t - LI : -1; }
    // Every Newton-solve phase starts from an opaque copy of its lane index, so the lane-derived LDS
    // addresses of the phase are recomputed there (a few VALU operations) instead of hoisted out of the
    // SQP loop, held across the IPM and spilled to AGPRs / scratch (reloaded with a memory latency per
    // phase).  Round 6: the quad2d / cartpole kernels' scratch 112-208 B/lane -> 0.
    __device__ static int phase_lane(int lane) {
        if constexpr (GPMPC_PHASE_LANE == 2 || (GPMPC_PHASE_LANE == 1 && (NWAVES == 1 || !kMfma)))
            asm volatile("" : "+v"(lane));
        return lane;
    }
    // P_x,lambda of stage k of a lambda segment (in its P' block)
    __device__ static double* pxl_at(const Lds& L, int k) { return L.P + (size_t)k * PPB + PXL; }

    template <bool AUG>
    struct Fac {
        static constexpr int CI = NX, UI = 8, NR = AUG ? 4 : 2;
        static_assert(NX + 1 <= 8 && NU <= 2 && UI + NU <= 16, "homogeneous tile layout");
        struct Stage { double g[2], d[3]; };
        double pn[NR];
        // G'' rows 4s + lr, column lc: LDS streams (masked lanes read the zero / one slots, stride 0)
        const double* pg[2];
        int gst[2];
        const double* pd[3];
        int dst[3];
        double* sp[2];
        int sp_st[2];
        double* sk;
        int sk_st;
        double* srui;
        int srui_st;
        bool lamc, lam2, lam3;
        double pend_p[2], pend_k, pend_r;   // the last stage's stores, issued during the next stage
        bool ok;
        int lr, lc, lane;

        __device__ static int gcol(int t) { return t < NX ? t : (t == CI ? NB : ((t >= UI && t < UI + NU) ? NX + t - UI : -1)); }
        __device__ static int svar(int t) { return t < NX ? t : ((t >= UI && t < UI + NU) ? NX + t - UI : -1); }

        // stages k0 .. k1-1, backward; AUG: from lambda' x_k1, else from the true P'_H (k1 = H)
        __device__ void init(const Lds& L, int H, int ln, int k0, int k1) {
            (void)k0;
            lane = phase_lane(ln);
            lr = lane >> 4;
            lc = lane & 15;
            const int gc_lc = gcol(lc), sv_lc = svar(lc), lm_lc = AUG ? lam_of(lc) : -1;
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                const int t = lr + 4 * r;
                double v = 0.0;
                if constexpr (AUG) {   // lambda' x_k1: P'[x_i][lambda_i] = P'[lambda_i][x_i] = 1
                    v = ((t < NX && lm_lc == t) || (lam_of(t) >= 0 && lam_of(t) == lc)) ? 1.0 : 0.0;
                } else {               // P'_H: diag(hq_H[x]), gq_H[x] in row and column CI
                    if (t < NX && lc < NX) v = (t == lc) ? L.hq[H * NBS + t] : 0.0;
                    else if (t < NX && lc == CI) v = L.gq[H * NBS + t];
                    else if (t == CI && lc < NX) v = L.gq[H * NBS + lc];
                }
                pn[r] = v;
            }
            if constexpr (!AUG) {   // P'_H (packed) for the multiplier recovery of stage H-1
                double* PH = L.P + (size_t)H * PPB;
#pragma unroll
                for (int r = 0; r < 2; ++r) {
                    const int t = lr + 4 * r;
                    if (t < NX) {
                        if (lc == CI) PH[PO + t] = pn[r];
                        else if (lc < NX && t <= lc) PH[pidx(t, lc)] = pn[r];
                    }
                }
            }
            ok = true;
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                const int t = lr + 4 * s2;
                const bool ld = t < NX && gc_lc >= 0;
                const bool one = t == CI && lc == CI;
                pg[s2] = ld ? L.G + (size_t)(k1 - 1) * NX * GS + t * GS + gc_lc : L.zero + (one ? 7 : 0);
                gst[s2] = ld ? NX * GS : 0;
            }
#pragma unroll
            for (int r = 0; r < 3; ++r) {
                const int t = lr + 4 * r, sv_t = svar(t);
                const double* base = L.zero;
                bool on = false;
                if (sv_t >= 0 && t == lc) { base = L.hq + sv_t; on = true; }
                else if (sv_t >= 0 && lc == CI) { base = L.gq + sv_t; on = true; }
                else if (t == CI && sv_lc >= 0) { base = L.gq + sv_lc; on = true; }
                pd[r] = on ? base + (size_t)(k1 - 1) * NBS : L.zero;
                dst[r] = on ? NBS : 0;
            }
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                const int t = lr + 4 * r;
                const bool st = t < NX && ((lc == CI) || (lc < NX && t <= lc) || lm_lc >= 0);
                const int idx = (lc == CI) ? PO + t
                                           : (lm_lc >= 0 ? PXL + t * NX + lm_lc : pidx(t < lc ? t : lc, t < lc ? lc : t));
                sp[r] = st ? L.P + (size_t)(k1 - 1) * PPB + idx : L.dummy;
                sp_st[r] = st ? PPB : 0;
            }
            const int kcol = lc < NX ? lc : (lc == CI ? NX : (lm_lc >= 0 ? NX + 1 + lm_lc : -1));
            const bool kst = lr < NU && kcol >= 0;
            sk = kst ? L.K + (size_t)(k1 - 1) * NU * KST + lr * KST + kcol : L.dummy;
            sk_st = kst ? NU * KST : 0;
            const bool rst = lane < NU * NU;
            srui = rst ? L.Rui + (size_t)(k1 - 1) * NU * NU + lane : L.dummy;
            srui_st = rst ? NU * NU : 0;
            // C-init masks of the lambda blocks: columns (W') and rows of elements 2, 3 (M')
            lamc = lm_lc >= 0;
            lam2 = AUG && lam_of(lr + 8) >= 0;
            lam3 = AUG && lam_of(lr + 12) >= 0;
            pend_p[0] = pend_p[1] = pend_k = pend_r = 0.0;
        }
        __device__ void load(const Lds& L, Stage& st) {
            (void)L;
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                st.g[q] = *pg[q];
                pg[q] -= gst[q];
            }
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                st.d[q] = *pd[q];
                pd[q] -= dst[q];
            }
        }
        __device__ void flush() {   // the previous stage's stores
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                *sp[r] = pend_p[r];
                sp[r] -= sp_st[r];
            }
            *sk = pend_k;
            sk -= sk_st;
            *srui = pend_r;
            srui -= srui_st;
        }
        // W' = P' G'' (2 chained MFMAs; AUG: P's lambda columns as the C-init)
        __device__ f64x4 wprod(const Stage& sd) const {
            f64x4 cw = {0.0, 0.0, 0.0, 0.0};
            if constexpr (AUG) {
#pragma unroll
                for (int r = 0; r < 4; ++r) cw[r] = lamc ? pn[r] : 0.0;
            }
            f64x4 w = mfma64(pn[0], sd.g[0], cw);
            return mfma64(pn[1], sd.g[1], w);
        }
        // C-init of M' = G''^T W' + D (AUG: W's lambda rows)
        __device__ f64x4 mcinit(const Stage& sd, const f64x4& w) const {
            f64x4 cm = {sd.d[0], sd.d[1], sd.d[2], 0.0};
            if constexpr (AUG) {
                cm[2] = lam2 ? w[2] : sd.d[2];
                cm[3] = lam3 ? w[3] : 0.0;
            }
            return cm;
        }
        // Ru = M'_uu (readlane), K' = -Ru^-1 M'_u. (adjugate / cubic reciprocal), Schur MFMA P'_k = M' + M'_.u K'
        __device__ void finish(const f64x4& m) {
            double Ru[NU][NU];
#pragma unroll
            for (int a = 0; a < NU; ++a)
#pragma unroll
                for (int b2 = a; b2 < NU; ++b2) {
                    Ru[a][b2] = readlane_d(m[2], (a << 4) | (UI + b2));
                    Ru[b2][a] = Ru[a][b2];
                }
            const double mu = m[2];
            double kb, Ri[NU][NU];
            if constexpr (NU == 1) {
                ok = ok && (Ru[0][0] > 0.0);
                const double id = fast_rcp(Ru[0][0]);
                Ri[0][0] = id;
                kb = -id * mu;
            } else {
                const double det = Ru[0][0] * Ru[1][1] - Ru[0][1] * Ru[0][1];
                ok = ok && (Ru[0][0] > 0.0) && (det > 0.0);
                const double mo = xor16_d(mu);
                const double num = fma((lr & 1) ? Ru[0][0] : Ru[1][1], mu, -Ru[0][1] * mo);
                const double r0 = __builtin_amdgcn_rcp(det);
                const double e = fma(-det, r0, 1.0);
                const double ee = fma(e, e, e);
                const double t = num * -r0;
                const double id = fma(r0, ee, r0);
                kb = fma(t, ee, t);
                Ri[0][0] = Ru[1][1] * id;
                Ri[1][1] = Ru[0][0] * id;
                Ri[0][1] = Ri[1][0] = -Ru[0][1] * id;
            }
            const f64x4 pk = mfma64(lr < NU ? mu : 0.0, kb, m);   // P'_k = M' + M'_{.u} K'
            double rv = Ri[0][0];
            if constexpr (NU == 2) rv = (lane == 0) ? Ri[0][0] : ((lane == 3) ? Ri[1][1] : Ri[0][1]);
            pend_p[0] = pk[0];
            pend_p[1] = pk[1];
            pend_k = kb;
            pend_r = rv;
#pragma unroll
            for (int r = 0; r < NR; ++r) pn[r] = pk[r];
        }
        // one stage; the previous stage's stores (FL: there is one) issued after this stage's W' products,
        // off the chain
        template <bool FL>
        __device__ void stage(const Stage& sd) {
            const f64x4 w = wprod(sd);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (FL) flush();
            __builtin_amdgcn_sched_barrier(0);
            f64x4 m = mfma64(sd.g[0], w[0], mcinit(sd, w));
            m = mfma64(sd.g[1], w[1], m);
            finish(m);
        }
        // AUG: the stage-k0 tile V (row-major 16 x 16) into the boundary data
        __device__ void store_tile(double* vtile) const {
            if constexpr (AUG) {
#pragma unroll
                for (int r = 0; r < 4; ++r) vtile[(lr + 4 * r) * 16 + lc] = pn[r];
            }
        }
    };

    // Riccati factorisation of stages k0 .. k1-1, mfma_backward_h's stage.  AUG (segment A): over
    // z = [x; 1; lambda] from the terminal cost lambda' x_k1; else (segment B, k1 = H) from the true P'_H.
    // The lambda blocks add no MFMA to the stage: the lambda rows of G'' are the identity, so
    //   W' = P' G''          = P'[:, 0..7] G''[0..7, :] + (P' on the lambda columns)   C-init of W's first MFMA
    //   M' = G''^T W' + D    = G''[0..7, :]^T W'[0..7, :] + (W' on the lambda rows, D elsewhere)
    // and the Schur MFMA P'_k = M' + M'_{.u} K' covers all 16 columns (K_lambda rides in K').  Stores per
    // stage: packed P and p (AUG: + P_x,lambda at PXL), K' = [K | kff (| K_lambda)],
    // Ru^-1; AUG: the stage-k0 tile V (row-major 16 x 16) into the boundary data.
    template <bool AUG>
    __device__ static bool seg_factor(const Lds& L, int H, int lane, int k0, int k1, double* vtile) {
        Fac<AUG> f;
        f.init(L, H, lane, k0, k1);
        typename Fac<AUG>::Stage s0, s1;
        f.load(L, s0);
        f.load(L, s1);
        f.template stage<false>(s0);   // (the first stage has no stores pending)
        int k = k1 - 2;
        for (; k >= k0 + 1; k -= 2) {
            f.load(L, s0);
            f.template stage<true>(s1);
            f.load(L, s1);   // (past stage k0 on the last pass: loaded, never used)
            f.template stage<true>(s0);
        }
        if (k == k0) f.template stage<true>(s1);
        f.flush();
        f.store_tile(vtile);
        return f.ok;
    }

    // Closed-loop stage maps A'_k = [A + B K | B kff + c] of stages k0 .. k1-1 (acl_phase over a range,
    // K' row stride KST); only the affine column when the feedback is unchanged.
    template <bool full>
    __device__ static void seg_acl(const Lds& L, int lane, int k0, int k1) {
        lane = phase_lane(lane);
        if constexpr (full) {
            for (int e = k0 * NX + lane; e < k1 * NX; e += 64) {
                const int k = e / NX, i = e - k * NX;
                const double* G = L.G + (size_t)k * NX * GS + i * GS;
                const double* Kk = L.K + (size_t)k * NU * KST;
                double g[GS], kr[NU][PS];
#pragma unroll
                for (int j = 0; j < GS; ++j) g[j] = G[j];
#pragma unroll
                for (int a = 0; a < NU; ++a)
#pragma unroll
                    for (int j = 0; j < PS; ++j) kr[a][j] = Kk[a * KST + j];
                double* out = L.Acl + (size_t)k * NX * PS + i * PS;
#pragma unroll
                for (int j = 0; j < PS; ++j) {
                    double acc = (j < NX) ? g[j] : g[NB];
#pragma unroll
                    for (int a = 0; a < NU; ++a) acc = fma(g[NX + a], kr[a][j], acc);
                    out[j] = acc;
                }
            }
        } else {
            const int n = k1 * NX;
            for (int e0 = k0 * NX + lane; e0 < n; e0 += 192) {
                double acc[3];
#pragma unroll
                for (int r = 0; r < 3; ++r) {
                    const int e = min(e0 + 64 * r, n - 1);
                    const int k = e / NX, i = e - k * NX;
                    const double* G = L.G + (size_t)k * NX * GS + i * GS;
                    const double* Kk = L.K + (size_t)k * NU * KST;
                    acc[r] = G[NB];
#pragma unroll
                    for (int a = 0; a < NU; ++a) acc[r] = fma(G[NX + a], Kk[a * KST + NX], acc[r]);
                }
#pragma unroll
                for (int r = 0; r < 3; ++r) {
                    const int e = e0 + 64 * r;
                    if (e < n) {
                        const int k = e / NX, i = e - k * NX;
                        L.Acl[(size_t)k * NX * PS + i * PS + NX] = acc[r];
                    }
                }
            }
        }
    }

    // Forward sweep of stages k0 .. k1-1 from dx_k0 = xs (NULL: 0), mfma4_forward over a range; dx_k0 is
    // stored, dx_k1 only when store_end (segment A leaves x_SM to segment B, which starts from it).
    __device__ static void seg_forward(const Lds& L, int lane, int k0, int k1, const double* xs, bool store_end) {
        lane = phase_lane(lane);
        const Mfma4Lane q = mfma4_lane(lane);
        const bool ld = q.row < NX && q.col <= NX;
        const double* src = ld ? L.Acl + (size_t)k0 * NX * PS + q.row * PS + q.col
                               : L.zero + ((q.row == NX && q.col == NX) ? 7 : 0);
        const int st = ld ? NX * PS : 0;
        const bool stlo = q.b == 0 && q.c == 0 && q.r < NX;
        const bool sthi = q.b == 2 && q.c == 0 && 4 + q.r < NX;
        double* dx0 = L.dxv + (size_t)k0 * NX;
        double* out = stlo ? dx0 + NX + q.r : (sthi ? dx0 + NX + 4 + q.r : L.dummy);
        const int ost = (stlo || sthi) ? NX : 0;
        if (lane < NX) dx0[lane] = xs ? xs[lane] : 0.0;
        double y = xs ? mfma4_vec(q, [&](int i) { return xs[i]; }) : mfma4_vec(q, [](int) { return 0.0; });
        const int n = k1 - k0;
        double an = *src;
        for (int k = 0; k < n; ++k) {
            const double a = an;
            src += (k + 1 < n) ? st : 0;
            an = *src;
            double sv;
            y = mfma4_stage(a, y, sv);
            if (store_end || k + 1 < n) *out = sv;
            out += ost;
        }
    }

    // Corrector right-hand side over stages k0 .. k1-1 (mfma4_vector_backward over a range): last
    // (segment B): from the true p_H; else (segment A) from the zero terminal P_k1 = 0, p_k1 = 0, plus
    // V_lambda,1 = sum_k P_lambda,x,k+1 (c_k + B_k kff_k) (P_lambda,x,k1 = I) into the boundary data.
    __device__ static void seg_vector_backward(const Lds& L, int H, int lane, int k0, int k1, bool last, double* vl1) {
        lane = phase_lane(lane);
        double* T = L.hq;
        double* VT = L.dxv;
        const int n = k1 * NX;
        // (each pass issues every load of its entries before a scheduling barrier)
        struct TOps { double pr[NX], gc[NX]; };
        auto t_load = [&](int e, TOps& o) {
            const int k = e / NX, i = e - k * NX;
            const double* Pn = L.P + (size_t)(k + 1) * PPB;
            const double* G = L.G + (size_t)k * NX * GS;
#pragma unroll
            for (int l = 0; l < NX; ++l) {
                o.pr[l] = Pn[i <= l ? pidx(i, l) : pidx(l, i)];
                o.gc[l] = G[l * GS + NB];
            }
        };
        auto t_dot = [&](int e, const TOps& o) {
            double acc = 0.0;
#pragma unroll
            for (int l = 0; l < NX; ++l) acc = fma(o.pr[l], o.gc[l], acc);
            return (last || e / NX + 1 < k1) ? acc : 0.0;
        };
        for (int e0 = k0 * NX + lane; e0 < n; e0 += 128) {
            const int e1 = e0 + 64;
            const bool has1 = e1 < n;
            TOps o0, o1;
            t_load(e0, o0);
            t_load(has1 ? e1 : e0, o1);
            __builtin_amdgcn_sched_barrier(0);
            const double a0 = t_dot(e0, o0), a1 = t_dot(has1 ? e1 : e0, o1);
            T[e0] = a0;
            if (has1) T[e1] = a1;
        }
        WSYNC();
        struct VOps { double g0, gu[NU], kc[NU], ac[NX], tk[NX]; };
        auto vt_load = [&](int e, VOps& o) {
            const int k = e / NX, i = e - k * NX;
            const double* A = L.Acl + (size_t)k * NX * PS;
            const double* Kk = L.K + (size_t)k * NU * KST;
            o.g0 = L.gq[k * NBS + i];
#pragma unroll
            for (int a = 0; a < NU; ++a) {
                o.kc[a] = Kk[a * KST + i];
                o.gu[a] = L.gq[k * NBS + NX + a];
            }
#pragma unroll
            for (int l = 0; l < NX; ++l) {
                o.ac[l] = A[l * PS + i];
                o.tk[l] = T[k * NX + l];
            }
        };
        auto vt_dot = [](const VOps& o) {
            double acc = o.g0;
#pragma unroll
            for (int a = 0; a < NU; ++a) acc = fma(o.kc[a], o.gu[a], acc);
#pragma unroll
            for (int l = 0; l < NX; ++l) acc = fma(o.ac[l], o.tk[l], acc);
            return acc;
        };
        for (int e0 = k0 * NX + lane; e0 < n; e0 += 128) {
            const int e1 = e0 + 64;
            const bool has1 = e1 < n;
            VOps o0, o1;
            vt_load(e0, o0);
            vt_load(has1 ? e1 : e0, o1);
            __builtin_amdgcn_sched_barrier(0);
            const double a0 = vt_dot(o0), a1 = vt_dot(o1);
            VT[e0] = a0;
            if (has1) VT[e1] = a1;
        }
        WSYNC();
        {
            const Mfma4Lane q = mfma4_lane(lane);
            const bool lda = q.row < NX && q.col < NX, ldv = q.row < NX && q.col == NX;
            const double* src = lda ? L.Acl + (size_t)(k1 - 1) * NX * PS + q.col * PS + q.row
                                    : (ldv ? VT + (size_t)(k1 - 1) * NX + q.row
                                           : L.zero + ((q.row == NX && q.col == NX) ? 7 : 0));
            const int st = lda ? NX * PS : (ldv ? NX : 0);
            if (last && lane < NX) L.P[(size_t)H * PPB + PO + lane] = L.gq[H * NBS + lane];
            double y = last ? mfma4_vec(q, [&](int i) { return L.gq[H * NBS + i]; }) : mfma4_vec(q, [](int) { return 0.0; });
            const bool stlo = q.b == 0 && q.c == 0 && q.r < NX;
            const bool sthi = q.b == 2 && q.c == 0 && 4 + q.r < NX;
            double* out = stlo ? L.P + (size_t)(k1 - 1) * PPB + PO + q.r
                               : (sthi ? L.P + (size_t)(k1 - 1) * PPB + PO + 4 + q.r : L.dummy);
            const int ost = (stlo || sthi) ? PPB : 0;
            double an = *src;
            for (int k = k1 - 1; k >= k0; --k) {
                const double a = an;
                src -= (k >= k0 + 1) ? st : 0;
                an = *src;
                double sv;
                y = mfma4_stage(a, y, sv);
                *out = sv;
                out -= ost;
            }
        }
        WSYNC();
        for (int e = k0 * NU + lane; e < k1 * NU; e += 64) {
            const int k = e / NU, a = e - k * NU;
            const double* G = L.G + (size_t)k * NX * GS;
            const unsigned mz = (!last && k + 1 == k1) ? 0xffffffffu : 0u;   // segment end: p_k1 = 0
            const double* pn = L.P + (size_t)(k + 1) * PPB + PO;
            // every load first (before a scheduling barrier), the p_k1 = 0 select branch-free
            double gb[NU][NX], tk[NX], pv[NX], gqv[NU], rui[NU];
#pragma unroll
            for (int b2 = 0; b2 < NU; ++b2) {
                gqv[b2] = L.gq[k * NBS + NX + b2];
                rui[b2] = L.Rui[(size_t)k * NU * NU + a * NU + b2];
#pragma unroll
                for (int l = 0; l < NX; ++l) gb[b2][l] = G[l * GS + NX + b2];
            }
#pragma unroll
            for (int l = 0; l < NX; ++l) {
                tk[l] = T[k * NX + l];
                pv[l] = pn[l];
            }
            __builtin_amdgcn_sched_barrier(0);
            double kf = 0.0;
#pragma unroll
            for (int b2 = 0; b2 < NU; ++b2) {
                double acc = gqv[b2];
#pragma unroll
                for (int l = 0; l < NX; ++l) acc = fma(gb[b2][l], tk[l] + bsel(mz, 0.0, pv[l]), acc);
                kf = fma(rui[b2], acc, kf);
            }
            L.K[(size_t)k * NU * KST + a * KST + NX] = -kf;
        }
        WSYNC();
        if (!last) seg_vl1(L, lane, k0, k1, vl1);
    }

    // V_lambda,1 = sum_k P_lambda,x,k+1 z_k of a lambda segment k0 .. k1-1 (its corrector pass), into vl1
    __device__ static void seg_vl1(const Lds& L, int lane, int k0, int k1, double* vl1) {
        lane = phase_lane(lane);
        double* VT = L.dxv;
        const int n = k1 * NX;
        // V_lambda,1 = sum_k P_lambda,x,k+1 z_k with z_k = c_k + B_k kff_k (this pass's kff, formed
        // here: the closed-loop maps' affine columns follow during the chain, seg_part): lane (k, j)
        // forms term j of stage k into VT (its p-recurrence input is consumed), then lanes j < NX add
        // the terms
        for (int e = k0 * NX + lane; e < n; e += 64) {
            const int k = e / NX, j = e - k * NX;
            const double* G = L.G + (size_t)k * NX * GS;
            const double* Kk = L.K + (size_t)k * NU * KST + NX;
            const double* Pl = pxl_at(L, k + 1);
            // every load first (before a scheduling barrier); P_lambda,x,k1 = I at the segment end, the
            // P' load unconditional (bsel: a ternary would sink it into a branch with a wait per term)
            double kf[NU], gc[NX], gu[NX][NU], pl[NX];
#pragma unroll
            for (int a = 0; a < NU; ++a) kf[a] = Kk[a * KST];
#pragma unroll
            for (int t = 0; t < NX; ++t) {
                gc[t] = G[t * GS + NB];
                pl[t] = Pl[t * NX + j];
#pragma unroll
                for (int a = 0; a < NU; ++a) gu[t][a] = G[t * GS + NX + a];
            }
            __builtin_amdgcn_sched_barrier(0);
            const unsigned mend = (k + 1 == k1) ? 0xffffffffu : 0u;
            double acc = 0.0;
#pragma unroll
            for (int t = 0; t < NX; ++t) {
                double z = gc[t];
#pragma unroll
                for (int a = 0; a < NU; ++a) z = fma(gu[t][a], kf[a], z);
                acc = fma(bsel(mend, t == j ? 1.0 : 0.0, pl[t]), z, acc);
            }
            VT[e] = acc;
        }
        WSYNC();
        if (lane < NX) {
            double acc = 0.0;
            for (int k = k0; k < k1; ++k) acc += VT[k * NX + lane];
            vl1[lane] = acc;
        }
        WSYNC();
    }

    // Boundary chain of the predictor (wave 1, after every segment's factorisation).  Backward over the
    // boundaries b = NSEG-2 .. 0; boundary b joins segment b (tile V: its first stage's P'_aug) to the
    // true cost-to-go Ph, ph at s_{b+1} (the last segment's P' there, or the previous boundary's result):
    //   T_b = I - Ph V_ll,   [Y_b | y_b] = T_b^-1 [Ph V_lx | Ph V_l1 + ph],
    //   Ph <- V_xx + V_xl Y_b,  ph <- V_x1 + V_xl y_b          (the cost-to-go at s_b, for boundary b - 1)
    // (lambda_b = Ph x_{b+1} + ph and x_{b+1} = V_lx x_b + V_l1 + V_ll lambda_b).  T_b is not symmetric,
    // but with W = -V_ll (negative semidefinite: the segment's value is concave in its terminal costate)
    //   T_b^-1 = Ph M^-1,   M = Ph + Ph W Ph   (symmetric positive definite: Ph > 0, W >= 0),
    // so Gauss-Jordan runs on M without pivoting (no pivot search or row swaps on the chain's critical
    // path), lane c holding column c of [M | Ph V_lx | Ph V_l1 + ph | I] (rows in registers, the pivot
    // column read by v_readlane), and [Y_b | y_b | T_b^-1] = Ph x (the eliminated right-hand sides).
    // Then seg_chain_forward.  T_b^-1, Y_b and the computed cost-to-go matrices stay in the boundary
    // data for the corrector.
    // M is positive definite only while Ph is: a state direction that no cost, bound barrier or
    // coupling reaches (q_i = 0 on an unbounded or barely bounded state) leaves Ph singular and a
    // pivot at rounding level.  Every pivot is checked against the largest diagonal entry of Ph
    // (ProblemDev::seg_piv_rel, 1e-10 by default; M = Ph (I + W Ph) with W >= 0 has no smaller
    // diagonal, and Ph is in every lane's
    // registers already, so the check adds no cross-lane move to the chain): the return value false
    // sends the solve to the one-segment recursion (seg_part's fallback), which never inverts Ph.
    __device__ static bool seg_chain_full(const Lds& L, int H, int lane, double P_piv_rel) {
        lane = phase_lane(lane);
        constexpr int CI = NX;
        const int c = min(lane, 3 * NX);
        const int cm = min(c, NX - 1);
        const unsigned mcol = c < NX ? 0xffffffffu : 0u;
        bool piv_ok = true;
        for (int b = NSEG - 2; b >= 0; --b) {
            const double* V = L.sb + SB_V + b * 256;
            const double* Pm = (b == NSEG - 2) ? L.P + (size_t)seg_start(NSEG - 1, H) * PPB : L.sb + SB_PH + b * PP;
            // every load first and unconditional (a load under a lane condition becomes a branch with its
            // own wait; loads interleaved with their uses issue a few at a time): Ph, column cm of Ph, the
            // uniform V_ll and the lane's right-hand side column of the tile
            const int bc = (c >= NX && c < 2 * NX) ? c - NX : CI;
            const double bs = (c >= NX && c <= 2 * NX) ? 1.0 : 0.0;
            double pk[PP], phc[NX], vll[NX][NX], vr[NX];
#pragma unroll
            for (int q = 0; q < PP; ++q) pk[q] = Pm[q];
#pragma unroll
            for (int m = 0; m < NX; ++m) phc[m] = Pm[m <= cm ? pidx(m, cm) : pidx(cm, m)];
#pragma unroll
            for (int l = 0; l < NX; ++l) {
                vr[l] = V[(LI + l) * 16 + bc];
#pragma unroll
                for (int m = 0; m < NX; ++m) vll[l][m] = V[(LI + l) * 16 + LI + m];
            }
            __builtin_amdgcn_sched_barrier(0);   // keeps the scheduler from sinking the loads into their uses
            double bv[NX];
#pragma unroll
            for (int l = 0; l < NX; ++l) {
                double w = (l == cm) ? 1.0 : 0.0;   // (e_c + W Ph e_c)_l
#pragma unroll
                for (int m = 0; m < NX; ++m) w = fma(-vll[l][m], phc[m], w);
                bv[l] = bsel(mcol, w, bs * vr[l]);
            }
            double col[NX];
#pragma unroll
            for (int i = 0; i < NX; ++i) {
                double acc = c == 2 * NX ? pk[PO + i] : (c > 2 * NX ? (i == c - 2 * NX - 1 ? 1.0 : 0.0) : 0.0);
#pragma unroll
                for (int l = 0; l < NX; ++l) acc = fma(pk[i <= l ? pidx(i, l) : pidx(l, i)], bv[l], acc);
                col[i] = acc;
            }
            double dmx = 0.0;   // largest diagonal entry of Ph
#pragma unroll
            for (int i = 0; i < NX; ++i) dmx = fmax(dmx, pk[pidx(i, i)]);
            const double pmin = P_piv_rel * dmx;
#pragma unroll
            for (int p = 0; p < NX; ++p) {
                double cp[NX];
#pragma unroll
                for (int i = 0; i < NX; ++i) cp[i] = readlane_d(col[i], p);
                piv_ok = piv_ok && (cp[p] > pmin);   // (false for a NaN pivot too)
                const double inv = fast_rcp(cp[p]);
                col[p] *= inv;
#pragma unroll
                for (int i = 0; i < NX; ++i)
                    if (i != p) col[i] = fma(-cp[i], col[p], col[i]);
            }
            // [Y_b | y_b | T_b^-1] = Ph M^-1 [...]
#pragma unroll
            for (int i = 0; i < NX; ++i) {
                double acc = 0.0;
#pragma unroll
                for (int l = 0; l < NX; ++l) acc = fma(pk[i <= l ? pidx(i, l) : pidx(l, i)], col[l], acc);
                bv[i] = acc;
            }
#pragma unroll
            for (int i = 0; i < NX; ++i) col[i] = bv[i];
            // branch-free stores: Y_b columns (b >= 1), y_b, T_b^-1 columns; other lanes into the dummy slots
            {
                const bool sy = b >= 1 && lane >= NX && lane < 2 * NX, syv = lane == 2 * NX,
                           sti = lane > 2 * NX && lane <= 3 * NX;
                double* dst = sy ? L.sb + SB_Y + b * NX * NX + (lane - NX)
                                 : (syv ? L.sb + SB_YV + 8 * b
                                        : (sti ? L.sb + SB_TI + b * NX * NX + (lane - 2 * NX - 1) : L.dummy + lane));
                const int ds = (sy || sti) ? NX : (syv ? 1 : 0);
#pragma unroll
                for (int i = 0; i < NX; ++i) dst[i * ds] = col[i];
            }
            if (b >= 1) {
                // cost-to-go at s_b, packed, one entry per lane: lane (i, j) = i (NX + 1) + j forms row i of
                // column j of V_xx + V_xl Y_b (j < NX) or of the vector V_x1 + V_xl y_b (j = NX), from the
                // Y_b / y_b just stored (one load round trip, stores branch-free)
                WSYNC();
                const int e = min(lane, NX * (NX + 1) - 1), i = e / (NX + 1), j = e - i * (NX + 1);
                const double* yc = j < NX ? L.sb + SB_Y + b * NX * NX + j : L.sb + SB_YV + 8 * b;
                const int ys = j < NX ? NX : 1;
                double acc = V[i * 16 + (j < NX ? j : CI)], vxl[NX], yl[NX];
#pragma unroll
                for (int l = 0; l < NX; ++l) {
                    vxl[l] = V[i * 16 + LI + l];
                    yl[l] = yc[l * ys];
                }
                __builtin_amdgcn_sched_barrier(0);   // loads first
#pragma unroll
                for (int l = 0; l < NX; ++l) acc = fma(vxl[l], yl[l], acc);
                const bool st = lane < NX * (NX + 1) && (j == NX || i <= j);
                *(st ? L.sb + SB_PH + (b - 1) * PP + (j == NX ? PO + i : pidx(min(i, j), max(i, j))) : L.dummy + lane) = acc;
                WSYNC();
            }
        }
        WSYNC();   // y_b, Y_b of every boundary before the forward pass reads them on other lanes
        seg_chain_forward(L, lane, false);
        return piv_ok;
    }

    // Forward over the boundaries from x_0 = 0: lambda_b = Y_b x_b + y_b (boundary 0: y_0),
    // x_{b+1} = V_lx x_b + V_l1 + V_ll lambda_b; lambda_b and the segment start states x_w into the
    // boundary data.  V_l1 is the tile's affine column after a factorisation, the corrector's vector
    // pass result (SB_VL1) after a vector pass (vec).
    __device__ static void seg_chain_forward(const Lds& L, int lane, bool vec) {
        lane = phase_lane(lane);
        constexpr int CI = NX;
        const int i = min(lane, NX - 1);
        double xh[NX];
#pragma unroll
        for (int l = 0; l < NX; ++l) xh[l] = 0.0;
        // every load first (before a scheduling barrier), the stores after the recursion
        double yv0[NBD], yr[NBD][NX], v1[NBD], vx[NBD][NX], vl[NBD][NX];
#pragma unroll
        for (int b = 0; b < NBD; ++b) {
            const double* V = L.sb + SB_V + b * 256;
            yv0[b] = L.sb[SB_YV + 8 * b + i];
            v1[b] = vec ? L.sb[SB_VL1 + 8 * b + i] : V[(LI + i) * 16 + CI];
#pragma unroll
            for (int l = 0; l < NX; ++l) {
                yr[b][l] = b >= 1 ? L.sb[SB_Y + b * NX * NX + i * NX + l] : 0.0;
                vx[b][l] = V[(LI + i) * 16 + l];
                vl[b][l] = V[(LI + i) * 16 + LI + l];
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        double lvs[NBD], xns[NBD];
#pragma unroll
        for (int b = 0; b < NBD; ++b) {
            double lv = yv0[b];
            if (b >= 1) {
#pragma unroll
                for (int l = 0; l < NX; ++l) lv = fma(yr[b][l], xh[l], lv);
            }
            double lam[NX];
#pragma unroll
            for (int j = 0; j < NX; ++j) lam[j] = readlane_d(lv, j);
            double xn = v1[b];
#pragma unroll
            for (int l = 0; l < NX; ++l) xn = fma(vx[b][l], xh[l], xn);
#pragma unroll
            for (int j = 0; j < NX; ++j) xn = fma(vl[b][j], lam[j], xn);
            lvs[b] = lv;
            xns[b] = xn;
            if (b + 1 < NBD) {
#pragma unroll
                for (int l = 0; l < NX; ++l) xh[l] = readlane_d(xn, l);
            }
        }
        const bool st = lane < NX;
#pragma unroll
        for (int b = 0; b < NBD; ++b) {
            *(st ? L.sb + SB_LAM + 8 * b + lane : L.dummy + lane) = lvs[b];
            *(st ? L.sb + SB_XM + 8 * (b + 1) + lane : L.dummy + lane) = xns[b];
        }
        WSYNC();
    }

    // Boundary chain of the corrector (wave 1): the factorisation, hence T_b^-1, Y_b and the cost-to-go
    // matrices, is unchanged; new vectors only: ph at s_{NSEG-1} from the last segment's vector pass,
    // V_l1 and V_x1 (the segment's zero-terminal p at its start) from the others':
    //   y_b = T_b^-1 (Ph V_l1 + ph),  ph <- V_x1 + V_xl y_b,  then seg_chain_forward.
    __device__ static void seg_chain_vec(const Lds& L, int H, int lane) {
        lane = phase_lane(lane);
        const int i = min(lane, NX - 1);
        // every load first (before a scheduling barrier), the stores after the recursion
        double phv = L.P[(size_t)seg_start(NSEG - 1, H) * PPB + PO + i];
        double prow[NBD][NX], vl1[NBD][NX], ti[NBD][NX], p1s[NBD], vxl[NBD][NX];
#pragma unroll
        for (int b = NBD - 1; b >= 0; --b) {
            const double* Pm = (b == NBD - 1) ? L.P + (size_t)seg_start(NSEG - 1, H) * PPB : L.sb + SB_PH + b * PP;
            const double* V = L.sb + SB_V + b * 256;
            p1s[b] = b >= 1 ? L.P[(size_t)seg_start(b, H) * PPB + PO + i] : 0.0;
#pragma unroll
            for (int l = 0; l < NX; ++l) {
                prow[b][l] = Pm[i <= l ? pidx(i, l) : pidx(l, i)];
                vl1[b][l] = L.sb[SB_VL1 + 8 * b + l];
                ti[b][l] = L.sb[SB_TI + b * NX * NX + i * NX + l];
                vxl[b][l] = b >= 1 ? V[i * 16 + LI + l] : 0.0;
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        double yvs[NBD];
#pragma unroll
        for (int b = NBD - 1; b >= 0; --b) {
            double r = phv;
#pragma unroll
            for (int l = 0; l < NX; ++l) r = fma(prow[b][l], vl1[b][l], r);
            double rv[NX];
#pragma unroll
            for (int j = 0; j < NX; ++j) rv[j] = readlane_d(r, j);
            double yv = 0.0;
#pragma unroll
            for (int j = 0; j < NX; ++j) yv = fma(ti[b][j], rv[j], yv);
            yvs[b] = yv;
            if (b >= 1) {
                double yu[NX];
#pragma unroll
                for (int j = 0; j < NX; ++j) yu[j] = readlane_d(yv, j);
                double p1 = p1s[b];
#pragma unroll
                for (int l = 0; l < NX; ++l) p1 = fma(vxl[b][l], yu[l], p1);
                phv = p1;
            }
        }
#pragma unroll
        for (int b = 0; b < NBD; ++b) *(lane < NX ? L.sb + SB_YV + 8 * b + lane : L.dummy + lane) = yvs[b];
        WSYNC();
        seg_chain_forward(L, lane, true);
    }

    // A segment with its solved terminal costate lambda: the feedforward kff_k += K_lambda,k lambda and
    // the costate vectors p_k += P_x,lambda,k lambda (k0 <= k < k1, k >= 1), so the sweep and the
    // multiplier recovery read an ordinary factorisation (the next factorisation or corrector pass
    // rewrites both); the closed-loop affine column A'_k[:, CI] = c_k + B_k kff_k follows in the same
    // pass (+ B_k K_lambda,k lambda), so no closed-loop pass runs between the fold and the sweep.
    __device__ static void seg_fold(const Lds& L, int lane, int k0, int k1, const double* lamp) {
        lane = phase_lane(lane);
        double lam[NX];
#pragma unroll
        for (int j = 0; j < NX; ++j) lam[j] = lamp[j];
        for (int e = k0 * NX + lane; e < k1 * NX; e += 64) {
            const int k = e / NX, i = e - k * NX;
            const double* Kk = L.K + (size_t)k * NU * KST;
            const double* G = L.G + (size_t)k * NX * GS + i * GS;
            double* Pk = L.P + (size_t)k * PPB;
            double* kp = i < NU ? L.K + (size_t)k * NU * KST + min(i, NU - 1) * KST + NX : L.dummy + lane;
            // every load first (before a scheduling barrier), stores branch-free (dummy slots for the
            // other lanes)
            double kl[NU][NX], gb[NU], pxl[NX];
#pragma unroll
            for (int a = 0; a < NU; ++a) {
                gb[a] = G[NX + a];
#pragma unroll
                for (int j = 0; j < NX; ++j) kl[a][j] = Kk[a * KST + NX + 1 + j];
            }
#pragma unroll
            for (int j = 0; j < NX; ++j) pxl[j] = pxl_at(L, k)[i * NX + j];
            double ac = L.Acl[(size_t)k * NX * PS + i * PS + NX];
            double pv = Pk[PO + i];
            const double kv = *kp;
            __builtin_amdgcn_sched_barrier(0);
            double dk[NU];   // K_lambda,k lambda
#pragma unroll
            for (int a = 0; a < NU; ++a) {
                double acc = 0.0;
#pragma unroll
                for (int j = 0; j < NX; ++j) acc = fma(kl[a][j], lam[j], acc);
                dk[a] = acc;
            }
#pragma unroll
            for (int a = 0; a < NU; ++a) ac = fma(gb[a], dk[a], ac);
#pragma unroll
            for (int j = 0; j < NX; ++j) pv = fma(pxl[j], lam[j], pv);
            L.Acl[(size_t)k * NX * PS + i * PS + NX] = ac;
            *(k >= 1 ? Pk + PO + i : L.dummy + lane) = pv;
            *kp = kv + dk[i < NU ? i : 0];
        }
    }

    // Per-lane step from the segment-parallel solution: recover_step_mfma with the KST / PPB strides (the
    // boundary costate is already folded into segment A's kff and p, seg_fold).
    __device__ static void recover_step_seg(const Lds& L, int H, int lane, double (&dd)[NB], double (&dpi)[NX]) {
        lane = phase_lane(lane);
        const bool on = lane <= H;
        const int kk = min(lane, H - 1);
        double dx[NX], dxn[NX];
#pragma unroll
        for (int i = 0; i < NX; ++i) {
            dx[i] = (on && lane >= 1) ? L.dxv[(size_t)lane * NX + i] : 0.0;
            dxn[i] = L.dxv[(size_t)(kk + 1) * NX + i];
        }
#pragma unroll
        for (int i = 0; i < NX; ++i) dd[i] = dx[i];
#pragma unroll
        for (int a = 0; a < NU; ++a) {
            double kr[PS];
#pragma unroll
            for (int j = 0; j < PS; ++j) kr[j] = L.K[(size_t)kk * NU * KST + a * KST + j];
            double du = kr[NX];
#pragma unroll
            for (int j = 0; j < NX; ++j) du = fma(kr[j], dx[j], du);
            dd[NX + a] = (lane < H) ? du : 0.0;
        }
        const double* Pn = L.P + (size_t)(kk + 1) * PPB;
        double pp[PP];
#pragma unroll
        for (int q = 0; q < PP; ++q) pp[q] = Pn[q];
#pragma unroll
        for (int i = 0; i < NX; ++i) {
            double acc = pp[PO + i];
#pragma unroll
            for (int j = 0; j < NX; ++j) acc = fma(pp[i <= j ? pidx(i, j) : pidx(j, i)], dxn[j], acc);
            dpi[i] = (lane < H) ? -acc : 0.0;
        }
    }

    // The segment-parallel solves, posted by wave 0 to the helper waves (helper_loop).  Segment w runs
    // on wave seg_wave(w): waves 1, 2, 3 with four waves, so wave 0 -- whose registers hold the IPM state
    // -- only posts and waits; waves 1 and 0 with two (wave 0 then runs the last segment, an ordinary
    // recursion over a range: no more registers than the one-segment kernel's).  Wave 1 also runs the
    // boundary chain.
    //   kCmdSegFactor (predictor): B1 | factorisations | Bm1 | wave 1: chain, others: closed-loop maps |
    //                 Bm2 | forward sweeps (after the fold of each segment's lambda) | B2
    //   kCmdSegVector (corrector): B1 | vector passes | Bm1 | wave 1: chain, others: affine columns |
    //                 Bm2 | forward | B2
    // Factorisation statuses in ctrl[8 + w].  Fallback: when the boundary chain meets a pivot it cannot
    // trust (seg_chain_full), it sets ctrl[kFb]; the segments' fold and sweep run regardless, and wave 0
    // (which reads the flag after Bm2, where it has slack) then posts a fallback command after B2: the
    // chain wave runs the one-segment recursion over the whole horizon in the same layout
    // (seg_fallback: factorisation into ctrl[kFb + 1], closed-loop maps, forward sweep from dx_0 = 0),
    // overwriting what the segments wrote; the corrector of the same IPM iteration likewise.  The helper
    // waves never read the flag (a flag tested by every wave before the sweeps cost the 4- and 8-GPU
    // shards 3 %, one tested after B2 1.5 %, profiles/r6/ab_fallback/).
    static constexpr int kCmdSegFactor = -3, kCmdSegVector = -4, kCmdSegFbFactor = -5, kCmdSegFbVector = -6;
    static constexpr int kFb = 12;   // ctrl slots: fallback flag, fallback factorisation status
    static constexpr int kTs = 14;   // ctrl slots 14-15: the instance's start time stamp (stats slot 10)
    __host__ __device__ static constexpr int seg_of_wave(int w) { return NSEG == 3 ? w - 1 : (w == 1 ? 0 : (w == 0 ? 1 : -1)); }
    // KIND 0: no segment on this wave; 1: segment sg < NSEG - 1 (lambda recursion); 2: the last segment
    // The closed-loop maps A'_k (seg_acl) are formed between Bm1 and Bm2, while wave 1 runs the boundary
    // chain, by the waves free then: with three segments wave 2 those of segments 0 and 1 and wave 3 the
    // last segment's (wave 0, holding the IPM state, takes none); with two, wave 0 all of them.
    __device__ static void acl_range(int w, int H, int& a0, int& a1) {
        if constexpr (NSEG == 3) {
            a0 = w == 3 ? seg_start(2, H) : 0;
            a1 = w == 2 ? seg_start(2, H) : (w == 3 ? H : 0);
        } else {
            a0 = 0;
            a1 = w == 0 ? H : 0;
        }
    }
    template <int KIND>
    __device__ static bool seg_part(const Lds& L, int H, int lane, int w, int sg, bool chain, int cmd, double piv_rel,
                                    int* fb = nullptr) {
        const int k0 = seg_start(sg, H), k1 = seg_start(sg + 1, H);
        double* xs = L.sb + SB_XM + 8 * sg;
        int a0, a1;
        acl_range(w, H, a0, a1);
        bool ok = true;
        if (cmd == kCmdSegFactor) {
            if constexpr (KIND == 1) {
                const bool fok = seg_factor<true>(L, H, lane, k0, k1, L.sb + SB_V + sg * 256);
                if (lane == 0) L.ctrl[8 + sg] = fok ? 1 : 0;
            } else if constexpr (KIND == 2) {
                const bool fok = seg_factor<false>(L, H, lane, k0, H, nullptr);
                if (lane == 0) L.ctrl[8 + sg] = fok ? 1 : 0;
            }
            __syncthreads();   // Bm1
            {   // every segment's status flag loaded at once (a short-circuit && loads them one by one)
                int f[NSEG];
#pragma unroll
                for (int q = 0; q < NSEG; ++q) f[q] = L.ctrl[8 + q];
                int all = 1;
#pragma unroll
                for (int q = 0; q < NSEG; ++q) all &= (f[q] != 0) ? 1 : 0;
                ok = all != 0;
            }
            if (chain && ok) {
                const bool cok = seg_chain_full(L, H, lane, piv_rel);
                if constexpr (GPMPC_SEG_FALLBACK) {
                    if (lane == 0) L.ctrl[kFb] = cok ? 0 : 1;
                }
            }
            if (a1 > a0) seg_acl<true>(L, lane, a0, a1);
            __syncthreads();   // Bm2: lambda_b, x_w, A'_k
            if (fb != nullptr) *fb = L.ctrl[kFb];   // (wave 0: read here, used after B2 by seg_run)
            if (ok) {
                if constexpr (KIND == 1) {
                    seg_fold(L, lane, k0, k1, L.sb + SB_LAM + 8 * sg);
                    WSYNC();
                    seg_forward(L, lane, k0, k1, sg ? xs : nullptr, false);
                } else if constexpr (KIND == 2) {
                    seg_forward(L, lane, k0, H, xs, true);
                }
            }
            __syncthreads();   // B2
        } else {
            if (fb != nullptr) *fb = L.ctrl[kFb];   // (this IPM iteration's predictor set it)
            if constexpr (KIND == 1) seg_vector_backward(L, H, lane, k0, k1, false, L.sb + SB_VL1 + 8 * sg);
            if constexpr (KIND == 2) seg_vector_backward(L, H, lane, k0, H, true, nullptr);
            __syncthreads();   // Bm1
            if (chain) seg_chain_vec(L, H, lane);
            if (a1 > a0) seg_acl<false>(L, lane, a0, a1);
            __syncthreads();   // Bm2: lambda_b, x_w, A'_k[:, CI]
            if constexpr (KIND == 1) {
                seg_fold(L, lane, k0, k1, L.sb + SB_LAM + 8 * sg);
                WSYNC();
                seg_forward(L, lane, k0, k1, sg ? xs : nullptr, false);
            } else if constexpr (KIND == 2) {
                seg_forward(L, lane, k0, H, xs, true);
            }
            __syncthreads();   // B2
        }
        return ok;
    }
    // The chain wave's one-segment recursion over the whole horizon in the segment layout (the fallback
    // commands): predictor -- factorisation (status into ctrl[kFb + 1]), closed-loop maps, forward sweep
    // from dx_0 = 0; corrector -- vector pass, affine columns, forward sweep.  It overwrites everything
    // the segments' fold and sweep wrote.
    __device__ static void seg_fallback(const Lds& L, int H, int lane, int cmd) {
        if (cmd == kCmdSegFbFactor) {
            const bool fok = seg_factor<false>(L, H, lane, 0, H, nullptr);
            if (lane == 0) L.ctrl[kFb + 1] = fok ? 1 : 0;
            WSYNC();
            if (fok) {
                seg_acl<true>(L, lane, 0, H);
                WSYNC();
                seg_forward(L, lane, 0, H, nullptr, true);
            }
        } else {
            seg_vector_backward(L, H, lane, 0, H, true, nullptr);
            seg_acl<false>(L, lane, 0, H);
            WSYNC();
            seg_forward(L, lane, 0, H, nullptr, true);
        }
    }
    // wave 0 (inside qp_ipm): post the command, then its own part; when the chain refused a pivot, one
    // more command has the chain wave redo the solve as the one-segment recursion (B1 | recursion | B2),
    // so the helper waves never wait on the flag
    __device__ static bool seg_run(const Lds& L, int H, int lane, int cmd) {
        if (lane == 0) L.ctrl[0] = cmd;
        __syncthreads();   // B1
        constexpr int sg0 = seg_of_wave(0);
        int fbv = 0;
        bool ok = seg_part<sg0 < 0 ? 0 : (sg0 == NSEG - 1 ? 2 : 1)>(L, H, lane, 0, sg0 < 0 ? 0 : sg0, false, cmd, 0.0, &fbv);
        if constexpr (GPMPC_SEG_FALLBACK) {
            if (ok && fbv != 0) {
                const bool pred = cmd == kCmdSegFactor;
                if (lane == 0) L.ctrl[0] = pred ? kCmdSegFbFactor : kCmdSegFbVector;
                __syncthreads();   // B1
                __syncthreads();   // B2 (the chain wave's recursion)
                if (pred) ok = L.ctrl[kFb + 1] != 0;
            }
        }
        return ok;
    }
    // helper wave w's part of a segment command (after B1)
    __device__ static void seg_helper(const Lds& L, int H, int lane, int w, int cmd, double piv_rel) {
        const int sg = seg_of_wave(w);
        if (sg == NSEG - 1) (void)seg_part<2>(L, H, lane, w, sg, w == 1, cmd, piv_rel);
        else if (sg >= 0) (void)seg_part<1>(L, H, lane, w, sg, w == 1, cmd, piv_rel);
        else (void)seg_part<0>(L, H, lane, w, 0, false, cmd, piv_rel);
    }

    // C' pi restricted to stage k variables: x_k: pi_{k-1} - A_k' pi_k ; u_k: -B_k' pi_k.
    __device__ static void ctpi(const Lds& L, int H, int lane, const double (&pi)[NX], double (&out)[NB]) {
        double pim1[NX];
#pragma unroll
        for (int i = 0; i < NX; ++i) pim1[i] = dpp_d<0x138>(pi[i]);   // wave_shr:1, lane - 1 (lane 0: unused)
        const double* G = L.G + (size_t)min(lane, H - 1) * NX * GS;
        double g[NX][NB];
#pragma unroll
        for (int l = 0; l < NX; ++l)
#pragma unroll
            for (int j = 0; j < NB; ++j) g[l][j] = G[l * GS + j];
#pragma unroll
        for (int j = 0; j < NB; ++j) {
            double acc = 0.0;
#pragma unroll
            for (int l = 0; l < NX; ++l) acc = fma(g[l][j], pi[l], acc);
            out[j] = ((lane < H) ? -acc : 0.0) + ((j < NX && lane >= 1 && lane <= H) ? pim1[j] : 0.0);
        }
    }

    // ------------------------------------------------------------------ IPM-layout helpers
    // (lane holds stage kq's variables vb .. vb + NV - 1; SPL: halves in lanes kq and kq + 32)
    // C' pi restricted to this lane's variables: x_k: pi_{k-1} - A_k' pi_k ; u_k: -B_k' pi_k.
    template <bool SPL, int NV>
    __device__ static void ctpi_q(const Lds& L, int H, int kq, int vb, const double (&pi)[NX], double (&out)[NV]) {
        double pim1[NX];   // pi of stage kq - 1: the previous lane of the same half
#pragma unroll
        for (int i = 0; i < NX; ++i) pim1[i] = dpp_d<0x138>(pi[i]);   // wave_shr:1, lane - 1 (lane 0: unused)
        const double* G = L.G + (size_t)min(kq, H - 1) * NX * GS + vb;
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const int v = vb + j;
            double acc = 0.0;
#pragma unroll
            for (int l = 0; l < NX; ++l) acc = fma(G[l * GS + j], pi[l], acc);
            double pm = (j < NX) ? pim1[j < NX ? j : 0] : 0.0;
            if constexpr (SPL) {
                const double ph = (NV + j < NX) ? pim1[NV + j < NX ? NV + j : 0] : 0.0;
                pm = vb ? ph : pm;
            }
            if constexpr (WSPL) {   // variable vb + j, vb = w NV uniform over the wave
#pragma unroll
                for (int q = 1; q < NWAVES; ++q) {
                    const int vq = q * NV + j;
                    if (vb == q * NV) pm = (vq < NX) ? pim1[vq < NX ? vq : 0] : 0.0;
                }
            }
            out[j] = (v < NB) ? (((kq < H) ? -acc : 0.0) + ((v < NX && kq >= 1 && kq <= H) ? pm : 0.0)) : 0.0;
        }
    }

    // dyn residual of stage kq (kq < H): y_{k+1} - A_k y_k - B_k v_k - c_k for stage vectors y = [x; u]
    template <bool SPL, int NV>
    __device__ static void dyn_residual_q(const Lds& L, int H, int kq, const double (&d)[NV], const double (&c)[NX],
                                          double (&r)[NX]) {
        const int lane = threadIdx.x & 63;
        // full stage vectors of stages kq and kq + 1, by lane moves without the LDS crossbar: the
        // other half of the stage is lane ^ 32 (permlane32 swap), the next stage is lane + 1 of the
        // same half (DPP wave_shl:1; lanes whose source is past the end are unused stages)
        double df[NB], xn[NX];
        const int h = lane >> 5;
        double dother[NV];
#pragma unroll
        for (int j = 0; j < NV; ++j) dother[j] = SPL ? xor32_d(d[j]) : d[j];
#pragma unroll
        for (int v = 0; v < NB; ++v) df[v] = (!SPL || v / NV == h) ? d[v % NV] : dother[v % NV];
#pragma unroll
        for (int i = 0; i < NX; ++i) xn[i] = dpp_d<0x130>((!SPL || i / NV == h) ? d[i % NV] : dother[i % NV]);
        const double* G = L.G + (size_t)min(kq, H - 1) * NX * GS;
#pragma unroll
        for (int i = 0; i < NX; ++i) {
            double gr[NB];
#pragma unroll
            for (int j = 0; j < NB; ++j) gr[j] = G[i * GS + j];
            double acc = xn[i] - c[i];
#pragma unroll
            for (int j = 0; j < NB; ++j) acc = fma(-gr[j], df[j], acc);
            r[i] = (kq < H) ? acc : 0.0;
        }
    }

    // Step of stage kq from the Riccati solution, restricted to this lane's variables, and dpi_kq.
    template <int NV>
    __device__ static void recover_q(const Lds& L, int H, int kq, int vb, double (&dd)[NV], double (&dp)[NX]) {
        double ddf[NB];
        if constexpr (kSeg) recover_step_seg(L, H, kq, ddf, dp);
        else if constexpr (kMfma) recover_step_mfma(L, H, kq, ddf, dp);
        else recover_step(L, H, kq, ddf, dp);
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const double lo = ddf[j < NB ? j : 0];
            if constexpr (WSPL) {   // vb = w NV, uniform over the wave
                double v = lo;
#pragma unroll
                for (int q = 1; q < NWAVES; ++q)
                    if (vb == q * NV) v = ddf[q * NV + j < NB ? q * NV + j : 0];
                dd[j] = v;
            } else {
                const double up = (NV + j < NB) ? ddf[NV + j < NB ? NV + j : 0] : 0.0;
                dd[j] = vb ? up : lo;
            }
        }
    }

    // ------------------------------------------------------------------ the QP (HPIPM's role), Mehrotra IPM
    // IPM layout: lane l holds stage kq's variables v = vb + j (j < NV).  SPL: the stage vectors are
    // split over lanes kq and kq + 32 (NV = NB/2), halving the per-lane IPM state and the elementwise
    // work.  WSPL (NWAVES > 1, quad3d): split over the instance's waves, wave w holding variables
    // w NV .. (w + 1) NV - 1 of every stage (lane = stage, NV = NB / NWAVES): the GP helper waves, idle
    // outside the tile passes, take their share of the elementwise work, and no lane holds more than
    // NV variables' IPM state (the unsplit layout spilled 3.5 KB per lane to scratch at H = 40).  The
    // full step vector for the dynamics residual, the reductions and the Riccati status cross the
    // waves through LDS at block barriers; the Riccati recursion runs on wave 0.
    // (the single-tile models keep their two-lanes-per-stage split on wave 0 when they run four waves:
    // their helpers take the GP tile passes and the segment solves -- sharing the IPM's elementwise work
    // costs more in cross-wave reductions than it saves at NB <= 8, round 3; with the segment solve, where
    // every wave then runs its part of the solve from inside the IPM, the kernel spilled 400 B/lane and
    // the 8-GPU shard's SQP kernel took 0.544 instead of 0.366 ms, round 6: tools/wspl_seg.patch)
    static constexpr bool WSPL = NWAVES > 1 && !kMfma;
    // (WSPL: NWAVES NV may exceed NB -- cartpole's 5 variables in slots of 2 -- and the slots past NB
    // are inactive: never stored, never published)
    template <bool SPL>
    __host__ __device__ static constexpr int nv_of() { return WSPL ? (NB + NWAVES - 1) / NWAVES : (SPL ? (NB + 1) / 2 : NB); }
    struct Tm {   // phase-timing state (GPMPC_TIMING)
        unsigned long long acc[kPhases];
        unsigned long long last;
        int cur;
    };
    __device__ static void XSYNC() {
        if constexpr (WSPL) __syncthreads();
        else wave_sync<NWAVES>();
    }
    // reductions over the instance (WSPL: wave reduction, one LDS exchange with a block barrier;
    // the two slot sets alternate, so one barrier per exchange suffices)
    __device__ static void xred2(const Lds& L, int lane, int wv, int& par, double vmax, double vsum, double& omax,
                                 double& osum) {
        vmax = wave_max(vmax);
        vsum = wave_sum(vsum);
        if constexpr (WSPL) {
            double* sl = L.xs + par * 2 * NWAVES;
            if (lane == 0) {
                sl[wv] = vmax;
                sl[NWAVES + wv] = vsum;
            }
            __syncthreads();
            vmax = sl[0];
            vsum = sl[NWAVES];
#pragma unroll
            for (int q = 1; q < NWAVES; ++q) {
                vmax = fmax(vmax, sl[q]);
                vsum += sl[NWAVES + q];
            }
            par ^= 1;
        }
        omax = vmax;
        osum = vsum;
    }
    __device__ static double xmax(const Lds& L, int lane, int wv, int& par, double v) {
        double m, s;
        xred2(L, lane, wv, par, v, 0.0, m, s);
        return m;
    }
    __device__ static double xsum(const Lds& L, int lane, int wv, int& par, double v) {
        double m, s;
        xred2(L, lane, wv, par, 0.0, v, m, s);
        return s;
    }
    __device__ static bool xall(const Lds& L, int lane, int wv, int& par, bool ok) {
        return xmax(L, lane, wv, par, ok ? 0.0 : 1.0) == 0.0;
    }
    // WSPL: wave owning row i of the dynamics residual
    __host__ __device__ static constexpr int xrow_of(int i) { return i / ((NX + NWAVES - 1) / NWAVES); }
    // dynamics residual of stage kq; WSPL: the waves exchange their parts of the step vector in LDS
    // and each computes its rows (its share of the max norm and of column NB of G')
    template <bool SPL, int NV>
    __device__ static void dyn_residual_x(const Lds& L, int H, int kq, int vb, const double (&d)[NV],
                                          const double (&c)[NX], double (&r)[NX]) {
        if constexpr (WSPL) {
            if (kq <= H) {
#pragma unroll
                for (int j = 0; j < NV; ++j)
                    if (vb + j < NB) L.Dq[(size_t)kq * NB + vb + j] = d[j];
            }
            __syncthreads();
            const double* dk = L.Dq + (size_t)min(kq, H) * NB;
            const double* dn = L.Dq + (size_t)min(kq + 1, H) * NB;
            const double* G = L.G + (size_t)min(kq, H - 1) * NX * GS;
            const int wv = threadIdx.x >> 6;
            double df[NB];
#pragma unroll
            for (int v = 0; v < NB; ++v) df[v] = dk[v];
#pragma unroll
            for (int i = 0; i < NX; ++i) {   // this wave's rows (xrow_of); the others are 0 here
                if (xrow_of(i) != wv) {
                    r[i] = 0.0;
                    continue;
                }
                double acc = dn[i] - c[i];
#pragma unroll
                for (int j = 0; j < NB; ++j) acc = fma(-G[i * GS + j], df[j], acc);
                r[i] = (kq < H) ? acc : 0.0;
            }
        } else {
            dyn_residual_q<SPL, NV>(L, H, kq, d, c, r);
        }
    }

    // WSPL: this wave's QP data from what wave 0 published (hq: lower bound distances, gq: upper,
    // Dq: cost gradient, dxv: dynamics residual, xs + 4 NWAVES: dx_0), then a barrier so that no wave
    // overwrites the buffers before every wave has read them.
    template <int NV>
    __device__ static void qp_setup_pub(const ProblemDev& P, const Lds& L, int H, int lane, int wv, double (&blo)[NV],
                                        double (&bup)[NV], double (&gv)[NV], double (&hd)[NV], double (&d)[NV],
                                        double (&cqq)[NX]) {
        const int kk = min(lane, H), vb = wv * NV;
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const int v = vb + j < NB ? vb + j : NB - 1;   // (slots past NB: inactive, any finite value)
            blo[j] = L.hq[(size_t)kk * NBS + v];
            bup[j] = L.gq[(size_t)kk * NBS + v];
            gv[j] = L.Dq[(size_t)kk * NB + v];
            hd[j] = hdiag(P, v, lane, H);
            d[j] = (lane == 0 && v < NX) ? L.xs[4 * NWAVES + (v < NX ? v : 0)] : 0.0;
        }
#pragma unroll
        for (int i = 0; i < NX; ++i) cqq[i] = L.dxv[(size_t)kk * NX + i];
        __syncthreads();
    }
    // WSPL: every wave's part of the QP step into Dq; the barrier is B2 of the helper command
    template <int NV>
    __device__ static void qp_publish_step(const Lds& L, int H, int lane, int wv, const double (&d)[NV]) {
        if (lane <= H) {
#pragma unroll
            for (int j = 0; j < NV; ++j)
                if (wv * NV + j < NB) L.Dq[(size_t)lane * NB + wv * NV + j] = d[j];
        }
        __syncthreads();
    }

    // One QP of the SQP iteration: blo/bup/gv/hd/d (this lane's variables) and cqq (the stage's
    // dynamics residual) in, the step d, the bound multipliers and piq (dynamics multipliers of
    // stage kq) out.  Every wave of the instance calls it (WSPL) with the same control flow.
    template <bool SPL, int NV>
    __device__ static bool qp_ipm(const ProblemDev& P, const Lds& L, int H, int lane, int wv,
                                  const double (&blo)[NV], const double (&bup)[NV], const double (&gv)[NV],
                                  const double (&hd)[NV], double (&d)[NV], const double (&cqq)[NX], double (&ll)[NV],
                                  double (&lu)[NV], double (&piq)[NX], int& qit_out, Tm& tm) {
        const bool hi_half = SPL && lane >= 32;
        const int kq = SPL ? (lane & 31) : lane;
        const int vb = WSPL ? wv * NV : (hi_half ? NV : 0);
        const bool on_q = kq <= H;
        const bool actx_q = on_q && kq >= 1;
        const bool actu_q = kq < H;
        const int k_q = min(kq, H);
        auto avq = [&](int j) { const int v = vb + j; return v < NX ? actx_q : (v < NB && actu_q); };
        const double nc = 2.0 * (double)H * (double)NB;
#ifdef GPMPC_TIMING
        unsigned long long(&tacc)[kPhases] = tm.acc;
        unsigned long long& tlast = tm.last;
        int& tcur = tm.cur;
#else
        (void)tm;
#endif
        double sl[NV], su[NV];
        // cold start (acados / HPIPM default): slacks at the bound distances floored at 1e-2,
        // multipliers mu0 / s, dynamics multipliers 0
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const bool av = avq(j);
            sl[j] = av ? fmax(-blo[j], 1e-2) : 1.0;
            su[j] = av ? fmax(bup[j], 1e-2) : 1.0;
            ll[j] = av ? P.qp_mu0 * fast_rcp(sl[j]) : 0.0;
            lu[j] = av ? P.qp_mu0 * fast_rcp(su[j]) : 0.0;
        }
#pragma unroll
        for (int i = 0; i < NX; ++i) piq[i] = 0.0;
        bool qp_ok = true;
        int qit = 0, par = 0;
        TPHASE(3);
        for (qit = 0; qit < P.qp_max_iter; ++qit) {
            double rp[NX];
            TPHASE(10);
            // slack reciprocals, once per IPM iteration: every later 1/s of this iteration
            // and the ratio-test step lengths (1 / max(-ds/s)) reuse them
            double isl[NV], isu[NV];
#pragma unroll
            for (int j = 0; j < NV; ++j) {
                isl[j] = fast_rcp(sl[j]);
                isu[j] = fast_rcp(su[j]);
            }
            {
                double ctq[NV];
                ctpi_q<SPL, NV>(L, H, kq, vb, piq, ctq);
                dyn_residual_x<SPL, NV>(L, H, kq, vb, d, cqq, rp);
                double m_rd = 0.0, m_rb = 0.0, m_lu = 0.0, mu_l = 0.0;
#pragma unroll
                for (int j = 0; j < NV; ++j) {
                    const bool av = avq(j);
                    const double rd = av ? fma(hd[j], d[j], gv[j]) - ll[j] + lu[j] + ctq[j] : 0.0;
                    const double rl = av ? d[j] - blo[j] - sl[j] : 0.0;
                    const double ru = av ? bup[j] - d[j] - su[j] : 0.0;
                    m_rd = fmax(m_rd, fabs(rd));
                    m_lu = fmax(m_lu, fmax(fabs(rl), fabs(ru)));
                    mu_l += av ? ll[j] * sl[j] + lu[j] * su[j] : 0.0;
                    if (on_q && vb + j < NB) {
                        // Riccati data: hq = H + Sigma; predictor gq with r_ml = ll sl, r_mu = lu su
                        const double hv = hd[j] + (av ? ll[j] * isl[j] + lu[j] * isu[j] : 0.0);
                        const double gqv = av ? rd + ll[j] + ll[j] * rl * isl[j] - lu[j] - lu[j] * ru * isu[j] : 0.0;
                        L.hq[k_q * NBS + vb + j] = hv;
                        L.gq[k_q * NBS + vb + j] = gqv;
                    }
                }
#pragma unroll
                for (int i = 0; i < NX; ++i) m_rb = fmax(m_rb, fabs(rp[i]));
                // the stopping test only needs the largest of the three residual norms: one reduction
                double mu, m_res;
                xred2(L, lane, wv, par, fmax(m_rd, fmax(m_rb, m_lu)), mu_l, m_res, mu);
                mu /= nc;
                if (!(mu == mu) || !(m_res == m_res)) { qp_ok = false; break; }
                if (m_res <= P.qp_tol && mu <= P.qp_tol) break;
                if (actu_q && !hi_half) {
#pragma unroll
                    for (int i = 0; i < NX; ++i)
                        if (!WSPL || xrow_of(i) == wv) L.G[(size_t)kq * NX * GS + i * GS + NB] = -rp[i];
                }
                XSYNC();
                TPHASE(4);
                double dd[NV], dp[NX];
                if constexpr (kSeg) {
                    // segment-parallel solve on the helper waves (seg_run)
                    const bool rok = seg_run(L, H, lane, kCmdSegFactor);
                    if (!rok) { qp_ok = false; break; }
                    TPHASE(9);
                    recover_q<NV>(L, H, kq, vb, dd, dp);
                    TPHASE(3);
                } else if constexpr (kMfma) {
                    bool rok = true;
                    if (wv == 0) {   // (WSPL: the other waves wait at the status exchange)
                        rok = mfma_backward_h(L, H, lane);
                        WSYNC();
                        TPHASE(8);
                        if (rok) acl_phase<true>(L, H, lane);
                        WSYNC();
                        TPHASE(6);
                        if (rok) mfma4_forward(L, H, lane);
                        WSYNC();
                    }
                    if constexpr (WSPL) rok = xall(L, lane, wv, par, rok);
                    if (!rok) { qp_ok = false; break; }
                    TPHASE(9);
                    recover_q<NV>(L, H, kq, vb, dd, dp);
                    TPHASE(3);
                } else {
                    // the recursion on wave 0 (WSPL: the other waves wait at the status exchange)
                    static_assert(kMfmaBig, "stage products must fit one (mfma_backward_h) or two (mfma_backward_big) tiles");
                    bool rok = true;
                    if (wv == 0) {
                        rok = mfma_backward_big(L, H, lane);
                        WSYNC();
                        TPHASE(6);
                        if (rok) valu_forward_big(L, H, lane);
                    }
                    if constexpr (WSPL) rok = xall(L, lane, wv, par, rok);
                    if (!rok) { qp_ok = false; break; }
                    TPHASE(3);
                    recover_q<NV>(L, H, kq, vb, dd, dp);
                }
                // affine step: ds/s = q, dl/l = -1 - q (predictor r_m = l s); ratio test
                // alpha_max = 1 / max(1, max_i -dv_i / v_i)
                double rmax = 1.0, mua_l = 0.0;
#pragma unroll
                for (int j = 0; j < NV; ++j) {
                    if (avq(j)) {
                        const double rl = d[j] - blo[j] - sl[j];
                        const double ru = bup[j] - d[j] - su[j];
                        const double ql = (dd[j] + rl) * isl[j], qu = (-dd[j] + ru) * isu[j];
                        rmax = fmax(rmax, fmax(fmax(-ql, -qu), fmax(1.0 + ql, 1.0 + qu)));
                    }
                }
                const double a_aff = fast_rcp(xmax(L, lane, wv, par, rmax));
#pragma unroll
                for (int j = 0; j < NV; ++j) {
                    if (avq(j)) {
                        const double rl = d[j] - blo[j] - sl[j];
                        const double ru = bup[j] - d[j] - su[j];
                        const double dsl = dd[j] + rl, dsu = -dd[j] + ru;
                        const double ql = dsl * isl[j], qu = dsu * isu[j];
                        mua_l += ll[j] * fma(-a_aff, 1.0 + ql, 1.0) * fma(a_aff, dsl, sl[j]) +
                                 lu[j] * fma(-a_aff, 1.0 + qu, 1.0) * fma(a_aff, dsu, su[j]);
                    }
                }
                const double mu_aff = xsum(L, lane, wv, par, mua_l) / nc;
                const double sr = mu_aff / mu;
                const double smu = sr * sr * sr * mu;
                // corrector: r_ml = ll sl + dll_aff dsl_aff - sigma mu  ->  gq += (dll dsl - smu)/sl - (dlu dsu - smu)/su
                double dda[NV];
#pragma unroll
                for (int j = 0; j < NV; ++j) {
                    dda[j] = dd[j];
                    if (on_q && avq(j)) {
                        const double rl = d[j] - blo[j] - sl[j];
                        const double ru = bup[j] - d[j] - su[j];
                        const double dsl = dd[j] + rl, dsu = -dd[j] + ru;
                        const double dll = -ll[j] * fma(dsl, isl[j], 1.0);
                        const double dlu = -lu[j] * fma(dsu, isu[j], 1.0);
                        L.gq[k_q * NBS + vb + j] += (dll * dsl - smu) * isl[j] - (dlu * dsu - smu) * isu[j];
                    }
                }
                XSYNC();
                TPHASE(5);
                if constexpr (kSeg) {
                    (void)seg_run(L, H, lane, kCmdSegVector);
                    TPHASE(9);
                    recover_q<NV>(L, H, kq, vb, dd, dp);
                    TPHASE(3);
                } else if constexpr (kMfma) {
                    if (wv == 0) {
                        mfma4_vector_backward(L, H, lane);
                        TPHASE(8);
                        acl_phase<false>(L, H, lane);
                        WSYNC();
                        TPHASE(6);
                        mfma4_forward(L, H, lane);
                        WSYNC();
                    }
                    XSYNC();
                    TPHASE(9);
                    recover_q<NV>(L, H, kq, vb, dd, dp);
                    TPHASE(3);
                } else {
                    if (wv == 0) {
                        valu_vector_big(L, H, lane);
                        TPHASE(6);
                        valu_forward_big(L, H, lane);
                    }
                    XSYNC();
                    TPHASE(3);
                    recover_q<NV>(L, H, kq, vb, dd, dp);
                }
                rmax = 1.0;
                double dsl[NV], dsu[NV], dll[NV], dlu[NV];
#pragma unroll
                for (int j = 0; j < NV; ++j) {
                    dsl[j] = dsu[j] = dll[j] = dlu[j] = 0.0;
                    if (avq(j)) {
                        const double rl = d[j] - blo[j] - sl[j];
                        const double ru = bup[j] - d[j] - su[j];
                        const double dsla = dda[j] + rl, dsua = -dda[j] + ru;
                        const double dlla = -ll[j] * fma(dsla, isl[j], 1.0);
                        const double dlua = -lu[j] * fma(dsua, isu[j], 1.0);
                        const double rml = ll[j] * sl[j] + dlla * dsla - smu;
                        const double rmu = lu[j] * su[j] + dlua * dsua - smu;
                        dsl[j] = dd[j] + rl;
                        dsu[j] = -dd[j] + ru;
                        dll[j] = (-rml - ll[j] * dsl[j]) * isl[j];
                        dlu[j] = (-rmu - lu[j] * dsu[j]) * isu[j];
                        const double ill = fast_rcp(ll[j]), ilu = fast_rcp(lu[j]);
                        rmax = fmax(rmax, fmax(fmax(-dsl[j] * isl[j], -dsu[j] * isu[j]),
                                               fmax(-dll[j] * ill, -dlu[j] * ilu)));
                    }
                }
                const double alpha = fmin(1.0, 0.995 * fast_rcp(xmax(L, lane, wv, par, rmax)));
#pragma unroll
                for (int j = 0; j < NV; ++j) {
                    if (avq(j)) {
                        d[j] = fma(alpha, dd[j], d[j]);
                        sl[j] = fma(alpha, dsl[j], sl[j]);
                        su[j] = fma(alpha, dsu[j], su[j]);
                        ll[j] = fma(alpha, dll[j], ll[j]);
                        lu[j] = fma(alpha, dlu[j], lu[j]);
                    }
                }
                if (actu_q) {
#pragma unroll
                    for (int i = 0; i < NX; ++i) piq[i] = fma(alpha, dp[i], piq[i]);
                }
            }
        }
        qit_out = qit;
        return qp_ok;
    }

    // cost Hessian diagonal of stage variable v on lane k (acados cost_scaling: dt on stages, 1 terminal)
    __device__ static double hdiag(const ProblemDev& P, int v, int lane, int H) {
        if (v < NX) return (lane >= 1 && lane <= H) ? ((lane < H) ? P.cost_scale : 1.0) * P.q[v] : 1.0;
        return (lane < H) ? P.cost_scale * P.r[v - NX] : 1.0;
    }

    // GP helper wave w (1..NWAVES-1): waits for the main wave's tile passes (B1), runs its share
    // of the pass's tiles into its partial buffer, and meets the main wave again (B2); the main wave
    // ends the loop with command -1 at the end of the kernel (one more B1).
    // Command -2 (WSPL): the wave takes its variables' share of the QP (qp_ipm) and publishes its
    // part of the step at B2.
    __device__ static void helper_loop(const ProblemDev& P, const StateDev& S, const Lds& L, int w, int lane, int b) {
        const int H = P.H;
        const int ne = (H + 15) >> 4, np = 16 * ne;
        for (;;) {
            __syncthreads();   // B1
            const int G = L.ctrl[0];
            if (G == -1) break;
            if constexpr (kSeg) {   // a segment-parallel Newton solve (seg_run)
                if (G == kCmdSegFactor || G == kCmdSegVector) {
                    seg_helper(L, H, lane, w, G, P.seg_piv_rel);
                    continue;
                }
                if (G == kCmdSegFbFactor || G == kCmdSegFbVector) {   // (the chain wave: w = 1)
                    if (w == 1) seg_fallback(L, H, lane, G);
                    __syncthreads();   // B2
                    continue;
                }
            }
            if constexpr (WSPL) {
                if (G == -2) {
                    constexpr int NV = nv_of<false>();
                    double blo[NV], bup[NV], gv[NV], hd[NV], d[NV], ll[NV], lu[NV], piq[NX], cqq[NX];
                    qp_setup_pub<NV>(P, L, H, lane, w, blo, bup, gv, hd, d, cqq);
                    Tm tm{};
                    int qit = 0;
                    const bool ok = qp_ipm<false, NV>(P, L, H, lane, w, blo, bup, gv, hd, d, cqq, ll, lu, piq, qit, tm);
                    if (ok && lane <= H) {   // this wave's bound multipliers (acados memory)
                        double* lam_q = lds_mult ? L.lam + (size_t)lane * 2 * NB
                                                     : S.lam + ((size_t)b * (H + 1) + lane) * 2 * NB;
#pragma unroll
                        for (int j = 0; j < NV; ++j) {
                            const int v = w * NV + j;
                            const bool ab = v < NX ? (lane >= 1) : (lane < H);
                            if (v < NB) {
                                lam_q[v] = ab ? ll[j] : 0.0;
                                lam_q[NB + v] = ab ? lu[j] : 0.0;
                            }
                        }
                    }
                    qp_publish_step<NV>(L, H, lane, w, d);   // B2
                    continue;
                }
            }
            static_for<NGP>([&](auto gi) {   // static index into the kernel-argument GP array
                constexpr int GG = decltype(gi)::value;
                if (GG != G) return;
                const GPDev& g = P.gp[GG];
                gp_tiles_dispatch<NWAVES>(g.tX, g.tW, g.ntile, L.gz + (size_t)GG * np * 4, L.gc + (size_t)GG * np,
                                          L.gsh + (size_t)(w - 1) * np * 4, lane, ne, w);
            });
            __syncthreads();   // B2
        }
    }

    // ------------------------------------------------------------------ the kernel body
    // SPL: the QP's per-variable state is split over two lanes per stage (needs H + 1 <= 32)
    template <bool SPL>
    __device__ static void run(const ProblemDev& P, const StateDev& S, const StepIO& io) {
        const int H = P.H;
        const int lane = threadIdx.x & 63;
        const int b = S.order ? __builtin_amdgcn_readfirstlane(S.order[S.first + blockIdx.x]) : (int)blockIdx.x;
        extern __shared__ __attribute__((aligned(16))) double smem[];
        const Lds L = carve(smem, H);
        if constexpr (NWAVES > 1) {
            if (threadIdx.x >= 64) {   // GP helper wave
                helper_loop(P, S, L, threadIdx.x >> 6, lane, b);
                return;
            }
        }
        if (lane < 8) L.zero[lane] = (lane == 7) ? 1.0 : 0.0;   // read by the masked stage-operand streams (7: one)
        const bool on = lane <= H;
        const bool act_x = on && lane >= 1;
        const bool act_u = lane < H;
        const int k = min(lane, H);
        // IPM lane layout (see the QP below): stage kq, variables vb .. vb + NV - 1
        static_assert(!(WSPL && SPL), "one IPM split at a time");
        constexpr int NV = nv_of<SPL>();
        const bool hi_half = SPL && lane >= 32;
        const int kq = SPL ? (lane & 31) : lane;
        const int vb = hi_half ? NV : 0;   // (WSPL: wave 0 holds variables 0 .. NV - 1)
        const bool on_q = kq <= H;
        const bool actx_q = on_q && kq >= 1;
        const bool actu_q = kq < H;
        const int k_q = min(kq, H);
        auto avq = [&](int j) { const int v = vb + j; return v < NX ? actx_q : (v < NB && actu_q); };
        Tm tm{};
#ifdef GPMPC_TIMING
        unsigned long long(&tacc)[kPhases] = tm.acc;
        unsigned long long& tlast = tm.last;
        int& tcur = tm.cur;
        tlast = __builtin_amdgcn_s_memtime();
        tcur = 7;
#endif
        // ---------------- load instance state (acados memory: iterate + multipliers)
        // The multipliers are read once per SQP iteration for the residuals and written after each
        // QP, so they hold no registers through the QP (the register file is the binding resource of
        // this kernel): they live in LDS during the step (this lane's rows of L.lam / L.pim) and go
        // to global memory (S.lam / S.pi) once, at the end of the step, when the layout has room
        // (lds_mult); otherwise every SQP iteration reads and writes the global rows.
        constexpr bool kLM = lds_mult;
        double w[NB];
        const double* xg = S.x + (size_t)b * (H + 1) * NX;
        const double* ug = S.u + (size_t)b * H * NU;
        double* lam_g = S.lam + ((size_t)b * (H + 1) + k) * 2 * NB;
        double* pi_g = S.pi + ((size_t)b * H + (act_u ? k : 0)) * NX;
        double* lam_l = kLM ? L.lam + (size_t)k * 2 * NB : lam_g;          // this lane's stage
        double* pi_l = kLM ? L.pim + (size_t)(act_u ? k : 0) * NX : pi_g;
        double* lam_q = kLM ? L.lam + (size_t)k_q * 2 * NB                  // this lane's stage in the IPM layout
                            : S.lam + ((size_t)b * (H + 1) + k_q) * 2 * NB;
        if constexpr (kLM) {
            if (on) {
#pragma unroll
                for (int v = 0; v < 2 * NB; ++v) lam_l[v] = lam_g[v];
            }
            if (act_u) {
#pragma unroll
                for (int i = 0; i < NX; ++i) pi_l[i] = pi_g[i];
            }
        }
#pragma unroll
        for (int i = 0; i < NX; ++i) w[i] = on ? xg[k * NX + i] : 0.0;
#pragma unroll
        for (int a = 0; a < NU; ++a) w[NX + a] = act_u ? ug[k * NU + a] : 0.0;
        double x0[NX];
#pragma unroll
        for (int i = 0; i < NX; ++i) x0[i] = io.x0[(size_t)b * NX + i];
        const int tref = (io.tstep[b] + k) % P.traj_len;
        // instance solve time (stats slots 10-11), stamped once the instance state is loaded: the stamp
        // waits in an LDS slot (taken at the kernel's first instruction, or held in registers, it cost the
        // one-wave kernel 48 B/lane of scratch)
        if constexpr (GPMPC_SOLVE_STAMP) {
            if (threadIdx.x == 0) *reinterpret_cast<unsigned long long*>(L.ctrl + kTs) = __builtin_amdgcn_s_memrealtime();
        }

        TPHASE(0);
        // ---------------- constraint tightening from the previous solution (gpmpc.py:425-498)
        double tsd[NB];  // icdf * sqrt(variance) per stage variable
#pragma unroll
        for (int v = 0; v < NB; ++v) tsd[v] = 0.0;
        if (P.tighten && S.has_prev[b]) {
            if (lane < H) {
                double Wt[NUNC][NGP];
                M::var_weights(w, w + NX, Wt);
                const double dt2 = P.dt * P.dt;
#pragma unroll
                for (int j = 0; j < NUNC; ++j) {
                    double acc = 0.0;
#pragma unroll
                    for (int g = 0; g < NGP; ++g)
                        acc = fma(Wt[j][g], S.var[((size_t)b * H + lane) * NGP + g] + P.gp[g].sn2, acc);
                    L.cd[lane * NUNC + j] = acc * dt2;
                }
            }
            WSYNC();
            // diag Sigma_k = sum_{m<k} sum_q tgain[m][.][q] cd_{k-1-m}[q]: the H-step covariance
            // recursion of gpmpc.py:478-495 with Sigma_0 = 0 and diagonal noise, restated as a
            // convolution so every stage (lane k) accumulates in parallel; tgain[m] is uniform
            // across the wave (scalar loads), cd_{k-1-m} is the lane's LDS read.
            double sv[NB];
#pragma unroll
            for (int v = 0; v < NB; ++v) sv[v] = 0.0;
            constexpr int NG = NB * NUNC;
            // k >> 8 is 0 (H < 256) but not provably uniform, so the table rows are vector loads
            // that can be issued one term ahead (scalar loads of uniform rows were serialised by
            // SGPR pressure); the rows come from L1.
            const double* gbase = P.tgain + (k >> 8);
            auto load_g = [&](int m, double (&g)[NG]) {
#pragma unroll
                for (int e = 0; e < NG; ++e) g[e] = gbase[(size_t)m * NG + e];
            };
            auto term = [&](int m, const double (&g)[NG]) {
                const bool act = m < k && on;
                const double* cdk = L.cd + (act ? (k - 1 - m) * NUNC : 0);   // unmasked read, masked value
                double cdv[NUNC];
#pragma unroll
                for (int q = 0; q < NUNC; ++q) {
                    const double cv = cdk[q];
                    cdv[q] = act ? cv : 0.0;
                }
#pragma unroll
                for (int v = 0; v < NB; ++v)
#pragma unroll
                    for (int q = 0; q < NUNC; ++q) sv[v] = fma(g[v * NUNC + q], cdv[q], sv[v]);
            };
            double g0[NG], g1[NG];
            load_g(0, g0);
            int m = 0;
            for (; m + 1 < H; m += 2) {
                load_g(m + 1, g1);
                term(m, g0);
                if (m + 2 < H) load_g(m + 2, g0);
                term(m + 1, g1);
            }
            if (m < H) term(m, g0);
#pragma unroll
            for (int v = 0; v < NB; ++v) tsd[v] = on ? P.icdf * sqrt(fmax(sv[v], 0.0)) : 0.0;
        }
        if (S.tight != nullptr && on) {
#pragma unroll
            for (int v = 0; v < NB; ++v) S.tight[((size_t)b * (H + 1) + k) * NB + v] = tsd[v];
        }
        // tightened boxes lo + t - uh <= w <= hi - t + uh   (gpmpc.py:296-314)
        auto lbv = [&](int v) { return (v < NX ? P.x_lo[v] : P.u_lo[v - NX]) + tsd[v] - P.uh; };
        auto ubv = [&](int v) { return (v < NX ? P.x_hi[v] : P.u_hi[v - NX]) - tsd[v] + P.uh; };

        // ---------------- stage-0 state rows (gpmpc.py:288,296,309-310; mpc.py:141,145,157-158)
        // x_0 is pinned to obs (lbx = ubx = obs, gpmpc.py:339-340), so these rows only decide
        // feasibility: an obs outside the stage-0 box by more than the inequality tolerance makes
        // every QP infeasible, which acados reports as a QP failure (status 4; the reference then
        // asserts, gpmpc.py:365).  Within the tolerance the rows enter the NLP residual only.
        double v0 = 0.0;   // largest stage-0 state-row violation of x0 (NaN-propagating)
#pragma unroll
        for (int i = 0; i < NX; ++i) {
            const double e = fmax(P.x_lo[i] - P.uh - x0[i], x0[i] - P.x_hi[i] - P.uh);
            v0 = (e == e && v0 == v0) ? fmax(v0, e) : __builtin_nan("");
        }
        const bool x0_ok = v0 <= P.tol_ineq;   // uniform: x0 and the bounds are the same on every lane
        // linearisation cache: the rows of the stored iterate's linearisation (StateDev::lin) are
        // valid when the step that stored the iterate also stored them and no host call since has
        // changed the iterate, the GPs or the model (lin_tag == lin_gen)
        double* lin_b = S.lin ? S.lin + (size_t)b * H * NX * GS : nullptr;
        const bool lin_hit = lin_b != nullptr && P.lin_gen != 0 &&
                             __builtin_amdgcn_readfirstlane(S.lin_tag[b]) == P.lin_gen;
        // store this step's final linearisation (and F of this lane's stage) before a good exit
        // (F goes into the c column of G' first, dead at this point, so the rows leave in one
        // coalesced pass)
        auto lin_store = [&](const double (&Fs)[NX]) {
            if (lin_b == nullptr) return;
            if (lane < H) {
#pragma unroll
                for (int i = 0; i < NX; ++i) L.G[(size_t)lane * NX * GS + i * GS + NB] = Fs[i];
            }
            WSYNC();
            for (int e = lane; e < H * NX * GS; e += 64) lin_b[e] = L.G[e];
        };
        // ---------------- SQP-GN, full steps (gpmpc.py:257-264, 364)
        int status = kMaxIter, it = 0, qp_total = 0;
        double res[4] = {0, 0, 0, 0};
        if (!x0_ok) status = kQPFailure;
        for (it = 0; x0_ok; ++it) {
            double lamL[NB], lamU[NB], pi[NX];
#pragma unroll
            for (int v = 0; v < NB; ++v) {
                const bool av = v < NX ? act_x : act_u;
                lamL[v] = av ? lam_l[v] : 0.0;
                lamU[v] = av ? lam_l[NB + v] : 0.0;
            }
#pragma unroll
            for (int i = 0; i < NX; ++i) pi[i] = act_u ? pi_l[i] : 0.0;
            double F[NX];
            TPHASE(1);
#ifdef GPMPC_TIMING
            unsigned long long* tgp = &tacc[11];
#else
            unsigned long long* tgp = nullptr;
#endif
            if (it == 0 && lin_hit) {
                // the first SQP iteration linearises at the stored iterate: identical rows
                for (int e = lane; e < H * NX * GS; e += 64) L.G[e] = lin_b[e];
#pragma unroll
                for (int i = 0; i < NX; ++i) F[i] = (lane < H) ? lin_b[(size_t)lane * NX * GS + i * GS + NB] : 0.0;
            } else {
                linearize(P, L, H, lane, w, F, tgp);
            }
            WSYNC();
            TPHASE(2);
            // stage reference (gpmpc.py:356-361)
            double yr[NB];
#pragma unroll
            for (int i = 0; i < NX; ++i) yr[i] = P.traj[(size_t)tref * NX + i];
#pragma unroll
            for (int a = 0; a < NU; ++a) yr[NX + a] = P.u_eq[a];
            // NLP residuals with the current multipliers
            double ct[NB];
            ctpi(L, H, lane, pi, ct);
            double xn[NX];
#pragma unroll
            for (int i = 0; i < NX; ++i) xn[i] = dpp_d<0x130>(w[i]);   // wave_shl:1, stage k + 1 (lane 63 unused)
            double r_stat = 0.0, r_eq = 0.0, r_ineq = 0.0, r_comp = 0.0;
            double g[NB];
#pragma unroll
            for (int v = 0; v < NB; ++v) {
                const bool av = v < NX ? act_x : act_u;
                g[v] = av ? hdiag(P, v, lane, H) * (w[v] - yr[v]) : 0.0;
                if (av) {
                    const double lb = lbv(v), ub = ubv(v);
                    r_stat = fmax(r_stat, fabs(g[v] - lamL[v] + lamU[v] + ct[v]));
                    r_ineq = fmax(r_ineq, fmax(lb - w[v], w[v] - ub));
                    r_comp = fmax(r_comp, fmax(fabs(lamL[v] * (w[v] - lb)), fabs(lamU[v] * (ub - w[v]))));
                }
            }
            double cq[NX];
#pragma unroll
            for (int i = 0; i < NX; ++i) {
                cq[i] = act_u ? F[i] - xn[i] : 0.0;
                r_eq = fmax(r_eq, fabs(cq[i]));
            }
            if (lane == 0) {
#pragma unroll
                for (int i = 0; i < NX; ++i) {
                    r_ineq = fmax(r_ineq, fabs(x0[i] - w[i]));  // lbx = ubx = obs
                    // stage-0 state rows on the iterate's x_0 (= obs after the first step)
                    r_ineq = fmax(r_ineq, fmax(P.x_lo[i] - P.uh - w[i], w[i] - P.x_hi[i] - P.uh));
                }
            }
            res[0] = wave_max(r_stat);
            res[1] = wave_max(r_eq);
            res[2] = wave_max(r_ineq);
            res[3] = wave_max(r_comp);
            if (!(res[0] == res[0] && res[1] == res[1] && res[2] == res[2] && res[3] == res[3])) { status = kNaN; break; }
            if (res[0] <= P.tol_stat && res[1] <= P.tol_eq && res[2] <= P.tol_ineq && res[3] <= P.tol_comp) {
                status = kSuccess;
                lin_store(F);
                break;
            }
            if (it == P.max_iter) { status = kMaxIter; lin_store(F); break; }

            // ---------------- QP in the step variables (HPIPM's role): qp_ipm
            // qv(): variable vb + j of stage kq from a stage vector held in the lane = stage layout.
            auto qv = [&](const double (&full)[NB], int j) {
                const double lo = (j < NB) ? full[j < NB ? j : 0] : 0.0;
                if constexpr (!SPL) return lo;
                const double up = xor32_d((NV + j < NB) ? full[NV + j < NB ? NV + j : 0] : 0.0);   // lane kq
                return hi_half ? up : lo;
            };
            double blo[NV], bup[NV], gv[NV], hd[NV], d[NV], ll[NV], lu[NV], piq[NX], cqq[NX];
            if constexpr (WSPL) {
                // publish the stage data for the helper waves (LDS buffers free at this point:
                // hq <- lower bound distances, gq <- upper, Dq <- cost gradient, dxv <- dynamics
                // residual, xs + 16 <- dx_0) and wake them for the QP (command -2)
                if (on) {
#pragma unroll
                    for (int v = 0; v < NB; ++v) {
                        L.hq[(size_t)k * NBS + v] = lbv(v) - w[v];
                        L.gq[(size_t)k * NBS + v] = ubv(v) - w[v];
                        L.Dq[(size_t)k * NB + v] = g[v];
                    }
#pragma unroll
                    for (int i = 0; i < NX; ++i) L.dxv[(size_t)k * NX + i] = cq[i];
                }
                if (lane == 0) {
#pragma unroll
                    for (int i = 0; i < NX; ++i) L.xs[4 * NWAVES + i] = x0[i] - w[i];
                    L.ctrl[0] = -2;
                }
                __syncthreads();   // B1
                qp_setup_pub<NV>(P, L, H, lane, 0, blo, bup, gv, hd, d, cqq);
            } else {
                double lbm[NB], ubm[NB], hdf[NB], d0[NB];
#pragma unroll
                for (int v = 0; v < NB; ++v) {
                    lbm[v] = lbv(v) - w[v];
                    ubm[v] = ubv(v) - w[v];
                    hdf[v] = hdiag(P, v, lane, H);
                    d0[v] = (lane == 0 && v < NX) ? x0[v] - w[v] : 0.0;   // dx_0 = e0 fixed
                }
#pragma unroll
                for (int j = 0; j < NV; ++j) {
                    blo[j] = qv(lbm, j);
                    bup[j] = qv(ubm, j);
                    gv[j] = qv(g, j);
                    hd[j] = qv(hdf, j);
                    d[j] = qv(d0, j);
                }
#pragma unroll
                for (int i = 0; i < NX; ++i) {
                    if constexpr (SPL) {
                        const double o = xor32_d(cq[i]);   // lane kq for the upper half
                        cqq[i] = hi_half ? o : cq[i];
                    } else {
                        cqq[i] = cq[i];
                    }
                }
            }
            int qit = 0;
            const bool qp_ok = qp_ipm<SPL, NV>(P, L, H, lane, 0, blo, bup, gv, hd, d, cqq, ll, lu, piq, qit, tm);
            if constexpr (WSPL) qp_publish_step<NV>(L, H, lane, 0, d);   // B2: the full step in Dq
            qp_total += qit;
            TPHASE(2);
            if (!qp_ok) { status = kQPFailure; break; }
            // full SQP step: w += d, multipliers <- QP multipliers
            if (on_q) {
#pragma unroll
                for (int j = 0; j < NV; ++j) {
                    if (vb + j < NB) {
                        const bool ab = avq(j);
                        lam_q[vb + j] = ab ? ll[j] : 0.0;
                        lam_q[NB + vb + j] = ab ? lu[j] : 0.0;
                    }
                }
            }
            bool fin = true;
#pragma unroll
            for (int v = 0; v < NB; ++v) {
                // d of variable v of this lane's stage (lane = stage layout: lanes 0..31)
                double dv = (v < NV) ? d[v < NV ? v : 0] : 0.0;
                if constexpr (WSPL) dv = L.Dq[(size_t)k * NB + v];
                if constexpr (SPL) {
                    const double up = xor32_d(d[v >= NV ? v - NV : 0]);   // lane + 32 (upper lanes: unused)
                    dv = (v >= NV) ? up : dv;
                }
                const bool av = v < NX ? (act_x || lane == 0) : act_u;
                if (av) w[v] += dv;
                fin = fin && (w[v] == w[v]);
            }
            if (act_u) {
#pragma unroll
                for (int i = 0; i < NX; ++i) pi_l[i] = piq[i];
            }
            if (lane == 0) {
#pragma unroll
                for (int i = 0; i < NX; ++i) w[i] = x0[i];
            }
            if (wave_min(fin ? 1.0 : 0.0) < 0.5) { status = kNaN; break; }
        }
        TPHASE(7);
#ifdef GPMPC_TIMING
        if (lane == 0 && io.timing != nullptr)
            for (int q = 0; q < kPhases; ++q) io.timing[(size_t)b * kPhases + q] = tacc[q];
#endif
        // ---------------- write back (acados memory + x_prev/u_prev, gpmpc.py:366-368)
        double* xo = S.x + (size_t)b * (H + 1) * NX;
        double* uo = S.u + (size_t)b * H * NU;
        // A failed solve (status 1 or 4; the reference asserts on it, gpmpc.py:365) must not poison
        // the instance's next step: the iterate keeps the previous solution, the multipliers
        // restart from zero, u0 is the previous solution's first input and the next step runs
        // untightened (as after a reset).
        const bool good = (status == kSuccess) || (status == kMaxIter);
        if constexpr (kLM) WSYNC();   // the last QP's multiplier rows (both lanes of a split stage) are in LDS
        if (good) {
            if (on) {
#pragma unroll
                for (int i = 0; i < NX; ++i) xo[k * NX + i] = w[i];
                if constexpr (kLM) {
#pragma unroll
                    for (int v = 0; v < 2 * NB; ++v) lam_g[v] = lam_l[v];
                }
            }
            if (act_u) {
#pragma unroll
                for (int a = 0; a < NU; ++a) uo[k * NU + a] = w[NX + a];
                if constexpr (kLM) {
#pragma unroll
                    for (int i = 0; i < NX; ++i) pi_g[i] = pi_l[i];
                }
            }
        } else {
            if (on) {
#pragma unroll
                for (int v = 0; v < 2 * NB; ++v) lam_g[v] = 0.0;
            }
            if (act_u) {
#pragma unroll
                for (int i = 0; i < NX; ++i) pi_g[i] = 0.0;
            }
        }
        if constexpr (NWAVES > 1) {   // release the GP helper waves
            if (lane == 0) L.ctrl[0] = -1;
            __syncthreads();   // B1
        }
        if (lane == 0) {
#pragma unroll
            for (int a = 0; a < NU; ++a) io.u0[(size_t)b * NU + a] = good ? w[NX + a] : uo[a];
            io.status[b] = status;
            io.sqp_iter[b] = it;
            io.qp_iter[b] = qp_total;
#pragma unroll
            for (int q = 0; q < 4; ++q) io.res[(size_t)b * 4 + q] = res[q];
            S.has_prev[b] = good ? 1 : 0;
            if (lin_b != nullptr) S.lin_tag[b] = good ? P.lin_gen : 0;
            if (S.cost != nullptr)   // this solve's work, for the next launch's dispatch order
                S.cost[b] = (uint32_t)(kCostLin * it + 2 * qp_total);
            if (io.stats != nullptr) {
                long long* st = io.stats + (size_t)b * kStatsSlots;
                st[0] += it;
                st[1] += qp_total;
                if (status >= 0 && status <= 4) st[2 + status] += 1;
                st[7] = max(st[7], (long long)it);
                st[8] = max(st[8], (long long)qp_total);
                st[9] += x0_ok ? it + 1 - (lin_hit ? 1 : 0) : 0;   // linearisations computed
                if constexpr (GPMPC_SOLVE_STAMP) {
                    const long long dt = (long long)(__builtin_amdgcn_s_memrealtime() -
                                                     *reinterpret_cast<const unsigned long long*>(L.ctrl + kTs));   // 100 MHz ticks
                    st[10] += dt;
                    st[11] = dt;
                }
            }
        }
    }
};

}  // namespace gpmpc

namespace gpmpc {

// GP mean + input gradient of the linearisation (gp_tiles) for arbitrary points: one wavefront
// per 64 points.  Z [P][d] -> mean [P] = sf2 S0, grad [P][d] = sf2/ell^2 (S_{1+k} - (z_k - xbar_k) S0).
__global__ __launch_bounds__(64) void gp_mean_grad_kernel(GPDev g, const double* Z, int P, double* mean, double* grad) {
    __shared__ double zb[64 * 4], czz[64], out[64 * 4];
    const int lane = threadIdx.x, p = blockIdx.x * 64 + lane;
    double zc[3] = {0.0, 0.0, 0.0};
    if (p < P)
        for (int k = 0; k < g.d; ++k) zc[k] = Z[(size_t)p * g.d + k] - g.xbar[k];
    zb[lane * 4 + 0] = zc[0];
    zb[lane * 4 + 1] = zc[1];
    zb[lane * 4 + 2] = zc[2];
    zb[lane * 4 + 3] = 1.0;
    czz[lane] = -0.5 * g.inv_ell2 * fma(zc[0], zc[0], fma(zc[1], zc[1], zc[2] * zc[2]));
    __syncthreads();
    gp_tiles_dispatch(g.tX, g.tW, g.ntile, zb, czz, out, lane, 4);
    __syncthreads();
    if (p < P) {
        const double s0 = out[lane * 4];
        if (mean) mean[p] = g.sf2 * s0;
        if (grad)
            for (int k = 0; k < g.d; ++k) grad[(size_t)p * g.d + k] = g.sf2 * g.inv_ell2 * fma(-zc[k], s0, out[lane * 4 + 1 + k]);
    }
}

hipError_t launch_gp_mean_grad(const GPDev& g, const double* Z, int P, double* mean, double* grad, hipStream_t stream) {
    hipLaunchKernelGGL(gp_mean_grad_kernel, dim3((P + 63) / 64), dim3(64), 0, stream, g, Z, P, mean, grad);
    return hipGetLastError();
}

// LINEAR_LS stage costs of the stored solution (gpmpc_set_cost_buffer), one thread per (instance,
// stage), queued right behind the SQP launch: cost[b][k] = 1/2 ||y_k - y_ref,k||^2_W, y = [x; u],
// W = dt blkdiag(Q, R) on stages 0..H-1 and Q on stage H (gpmpc.py:231-239, mpc.py:101-102, acados
// cost_scaling); NaN for an instance whose solve failed (status 1 / 4: x, u hold the previous
// solution).  A separate kernel so that the SQP kernel's register allocation does not change.
template <int ID>
__global__ __launch_bounds__(256) void stage_cost_kernel(ProblemDev P, const double* __restrict__ x,
                                                         const double* __restrict__ u, const int32_t* __restrict__ tstep,
                                                         const int32_t* __restrict__ status, double* __restrict__ cost,
                                                         int B) {
    using M = Model<ID>;
    constexpr int NX = M::NX, NU = M::NU;
    const int H = P.H;
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= B * (H + 1)) return;
    const int b = e / (H + 1), k = e - b * (H + 1);
    const int tref = (tstep[b] + k) % P.traj_len;
    const double ws = k < H ? P.cost_scale : 1.0;
    double c = 0.0;
#pragma unroll
    for (int i = 0; i < NX; ++i) {
        const double d = x[((size_t)b * (H + 1) + k) * NX + i] - P.traj[(size_t)tref * NX + i];
        c = fma(0.5 * ws * P.q[i] * d, d, c);
    }
    if (k < H) {
#pragma unroll
        for (int a = 0; a < NU; ++a) {
            const double d = u[((size_t)b * H + k) * NU + a] - P.u_eq[a];
            c = fma(0.5 * P.cost_scale * P.r[a] * d, d, c);
        }
    }
    const int st = status[b];
    cost[e] = (st == kSuccess || st == kMaxIter) ? c : __builtin_nan("");
}

hipError_t launch_stage_cost(const ProblemDev& P, const double* x, const double* u, const int32_t* tstep,
                             const int32_t* status, double* cost, int B, hipStream_t stream) {
    const int n = B * (P.H + 1), blocks = (n + 255) / 256;
    switch (P.model) {
        case kQuad2D: hipLaunchKernelGGL(stage_cost_kernel<kQuad2D>, dim3(blocks), dim3(256), 0, stream, P, x, u, tstep, status, cost, B); break;
        case kQuad3D: hipLaunchKernelGGL(stage_cost_kernel<kQuad3D>, dim3(blocks), dim3(256), 0, stream, P, x, u, tstep, status, cost, B); break;
        case kCartpole: hipLaunchKernelGGL(stage_cost_kernel<kCartpole>, dim3(blocks), dim3(256), 0, stream, P, x, u, tstep, status, cost, B); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// order[r] = the instance of rank r by decreasing cost (ties by instance id: a permutation);
// one thread per instance counts the instances ranked before it.  Used only for multi-round
// launches (a few hundred to a few thousand instances: O(B^2 / threads) broadcast LDS reads).
__global__ __launch_bounds__(256) void order_by_cost_kernel(const uint32_t* __restrict__ cost, int B,
                                                            int32_t* __restrict__ order) {
    __shared__ uint32_t cs[2048];
    const int i = blockIdx.x * 256 + threadIdx.x;
    const uint32_t ci = i < B ? cost[i] : 0u;
    int rank = 0;
    for (int j0 = 0; j0 < B; j0 += 2048) {
        const int n = min(2048, B - j0);
        __syncthreads();
        for (int j = threadIdx.x; j < n; j += 256) cs[j] = cost[j0 + j];
        __syncthreads();
        for (int j = 0; j < n; ++j) {
            const uint32_t cj = cs[j];
            rank += (cj > ci || (cj == ci && j0 + j < i)) ? 1 : 0;
        }
    }
    if (i < B) order[rank] = i;
}

// One wave per SIMD: every wave of an instance owns a SIMD's register file.
template <int ID, int NW, bool SPL, bool SEG = false>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(1, 1))) void sqp_step_kernel(ProblemDev P, StateDev S, StepIO io) {
    SqpKernel<ID, NW, SEG>::template run<SPL>(P, S, io);
}
// count < 0: the whole batch (ordered by cost here when it needs more than one round of workgroups);
// count >= 0: ranks first .. first + count - 1 of an order[] launch_sqp_order already filled
template <int ID, int NW, bool SPL, bool SEG = false>
hipError_t launch_sqp_variant(const ProblemDev& P, const StateDev& S, const StepIO& io, int batch, hipStream_t stream,
                              int first, int count) {
    const size_t lds = SqpKernel<ID, NW, SEG>::lds_doubles(P.H) * sizeof(double);
    if (lds > 64 * 1024) {
        const hipError_t e = hipFuncSetAttribute((const void*)sqp_step_kernel<ID, NW, SPL, SEG>,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    // instances resident at once: one wave per SIMD (4 / NW per CU), bounded by the CU's 160 KB LDS
    const int per_cu = std::max(1, std::min(4 / NW, (int)((160 * 1024) / lds)));
    StateDev Sl = S;
    Sl.first = 0;
    if (count >= 0) {   // a chunk of ranks of the order already computed
        if (count == 0) return hipSuccess;
        Sl.first = first;
        hipLaunchKernelGGL((sqp_step_kernel<ID, NW, SPL, SEG>), dim3(count), dim3(64 * NW), lds, stream, P, Sl, io);
        return hipGetLastError();
    }
    // (rank by counting: O(B^2) comparisons, a few microseconds up to ~16 k instances; larger
    // launches keep instance order rather than pay for it)
    if (S.order != nullptr && S.cost != nullptr && P.order_dispatch && P.n_cu > 0 &&
        (batch > P.n_cu * per_cu || P.order_dispatch == 2) && batch <= 16384) {
        hipLaunchKernelGGL(order_by_cost_kernel, dim3((batch + 255) / 256), dim3(256), 0, stream, S.cost, batch,
                           const_cast<int32_t*>(S.order));
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    } else {
        Sl.order = nullptr;
    }
    hipLaunchKernelGGL((sqp_step_kernel<ID, NW, SPL, SEG>), dim3(batch), dim3(64 * NW), lds, stream, P, Sl, io);
    return hipGetLastError();
}

// waves per instance for this launch: the model's default, or (single-tile models) as many as the
// batch leaves SIMDs for -- four when every instance can have a CU of its own (batch <= CUs), two
// when two instances share a CU (batch <= 2 CUs), else one -- unless the request fixes it (P.waves:
// 0 = auto)
template <int ID>
int sqp_waves(const ProblemDev& P, int batch) {
    if constexpr (kDefaultWaves<ID> > 1) {
        return kDefaultWaves<ID>;
    } else {
        if (P.waves == 1 || P.waves == 2 || P.waves == 4) return P.waves;
        if (P.n_cu <= 0) return 1;
        return batch <= P.n_cu ? 4 : (batch <= 2 * P.n_cu ? 2 : 1);
    }
}

// segment-parallel Newton solves (SqpKernel::kSeg): the single-tile models on two or four waves per
// instance, when the option allows it (P.seg) and the horizon has at least four stages (segments of one
// stage or more).  (One wave running both segments' recursions interleaved was built and measured in
// round 6 and does not pay: tools/one_wave_segments.patch)
template <int ID>
static bool sqp_seg_of(const ProblemDev& P, int nw) { return P.seg != 0 && nw >= 2 && P.H >= 4; }

template <int ID>
hipError_t launch_sqp_step(const ProblemDev& P, const StateDev& S, const StepIO& io, int batch, hipStream_t stream,
                           int first, int count) {
    if constexpr (kDefaultWaves<ID> == 1) {
        // stage vectors split over two lanes when the H + 1 stages fit in half a wavefront
        const bool spl = P.H + 1 <= 32;
        const int nw = sqp_waves<ID>(P, batch);   // from the whole batch, also for a chunk of it
        const bool seg = sqp_seg_of<ID>(P, nw);
        if (nw == 4) {
            if (seg)
                return spl ? launch_sqp_variant<ID, 4, true, true>(P, S, io, batch, stream, first, count)
                           : launch_sqp_variant<ID, 4, false, true>(P, S, io, batch, stream, first, count);
            return spl ? launch_sqp_variant<ID, 4, true>(P, S, io, batch, stream, first, count)
                       : launch_sqp_variant<ID, 4, false>(P, S, io, batch, stream, first, count);
        }
        if (nw == 2) {
            if (seg)
                return spl ? launch_sqp_variant<ID, 2, true, true>(P, S, io, batch, stream, first, count)
                           : launch_sqp_variant<ID, 2, false, true>(P, S, io, batch, stream, first, count);
            return spl ? launch_sqp_variant<ID, 2, true>(P, S, io, batch, stream, first, count)
                       : launch_sqp_variant<ID, 2, false>(P, S, io, batch, stream, first, count);
        }
        return spl ? launch_sqp_variant<ID, 1, true>(P, S, io, batch, stream, first, count)
                   : launch_sqp_variant<ID, 1, false>(P, S, io, batch, stream, first, count);
    } else {
        // multi-wave models split the IPM state over their waves instead (WSPL)
        return launch_sqp_variant<ID, kDefaultWaves<ID>, false>(P, S, io, batch, stream, first, count);
    }
}

// Whether a step of `batch` instances runs as two overlapped halves (gpmpc_solve): when its SQP
// launch needs more than one round of workgroups (config 5: 512 quad3d instances, one per CU).
// A launch that fits the device at once runs its instances side by side, and there the halves were
// measured slower (profiles/r4/ab_overlap/: config 3 0.609 -> 0.933 ms per step, config 4 1.155 ->
// 1.706): the costlier half then shares its CUs' LDS and instruction traffic with other costly
// instances for the whole step instead of with instances that finish early.
template <int ID>
static bool overlap_ok_of(const ProblemDev& P, int batch) {
    if (P.n_cu <= 0) return false;
    const int nw = sqp_waves<ID>(P, batch);
    size_t lds = SqpKernel<ID>::lds_doubles(P.H);
    if constexpr (kDefaultWaves<ID> == 1) {
        const bool seg = sqp_seg_of<ID>(P, nw);
        if (nw == 4) lds = seg ? SqpKernel<ID, 4, true>::lds_doubles(P.H) : SqpKernel<ID, 4>::lds_doubles(P.H);
        if (nw == 2) lds = seg ? SqpKernel<ID, 2, true>::lds_doubles(P.H) : SqpKernel<ID, 2>::lds_doubles(P.H);
    }
    const int per_cu = std::max(1, std::min(4 / nw, (int)((160 * 1024) / (lds * sizeof(double)))));
    return batch > P.n_cu * per_cu;
}
bool sqp_overlap_ok(const ProblemDev& P, int batch) {
    switch (P.model) {
        case kQuad2D: return overlap_ok_of<kQuad2D>(P, batch);
        case kQuad3D: return overlap_ok_of<kQuad3D>(P, batch);
        case kCartpole: return overlap_ok_of<kCartpole>(P, batch);
    }
    return false;
}
// Whether a step may run the tail boost (gpmpc_solve, GPMPC_TUNE_TAIL): a single-tile model whose
// automatic launch gives every instance one wave in one round of workgroups, segment solves on.
template <int ID>
static bool tail_ok_of(const ProblemDev& P, int batch) {
    if constexpr (kDefaultWaves<ID> == 1) {
        return P.waves == 0 && P.n_cu > 0 && batch >= 2 && sqp_waves<ID>(P, batch) == 1 &&
               sqp_seg_of<ID>(P, 2) && !overlap_ok_of<ID>(P, batch);
    }
    return false;
}
bool sqp_tail_ok(const ProblemDev& P, int batch) {
    switch (P.model) {
        case kQuad2D: return tail_ok_of<kQuad2D>(P, batch);
        case kQuad3D: return tail_ok_of<kQuad3D>(P, batch);
        case kCartpole: return tail_ok_of<kCartpole>(P, batch);
    }
    return false;
}
// The SIMDs a one-wave, one-round launch of `batch` instances leaves free (0 when the tail boost
// does not apply): the automatic K of GPMPC_TUNE_TAIL, one extra wave per boosted instance.
template <int ID>
static int tail_spare_of(const ProblemDev& P, int batch) {
    if (!tail_ok_of<ID>(P, batch)) return 0;
    const size_t lds = SqpKernel<ID>::lds_doubles(P.H) * sizeof(double);
    const int per_cu = std::max(1, std::min(4, (int)((160 * 1024) / lds)));
    return std::max(0, std::min(P.n_cu * per_cu - batch, batch - 1));
}
int sqp_tail_spare(const ProblemDev& P, int batch) {
    switch (P.model) {
        case kQuad2D: return tail_spare_of<kQuad2D>(P, batch);
        case kQuad3D: return tail_spare_of<kQuad3D>(P, batch);
        case kCartpole: return tail_spare_of<kCartpole>(P, batch);
    }
    return 0;
}
int sqp_launch_waves(const ProblemDev& P, int batch) {
    switch (P.model) {
        case kQuad2D: return sqp_waves<kQuad2D>(P, batch);
        case kQuad3D: return sqp_waves<kQuad3D>(P, batch);
        case kCartpole: return sqp_waves<kCartpole>(P, batch);
    }
    return 0;
}
template <int ID>
static int segments_of(const ProblemDev& P, int batch) {
    if constexpr (kDefaultWaves<ID> == 1) {
        const int nw = sqp_waves<ID>(P, batch);
        if (!sqp_seg_of<ID>(P, nw)) return 1;
        return nw == 4 ? SqpKernel<ID, 4, true>::NSEG : SqpKernel<ID, 2, true>::NSEG;
    }
    return 1;
}
int sqp_launch_segments(const ProblemDev& P, int batch) {
    switch (P.model) {
        case kQuad2D: return segments_of<kQuad2D>(P, batch);
        case kQuad3D: return segments_of<kQuad3D>(P, batch);
        case kCartpole: return segments_of<kCartpole>(P, batch);
    }
    return 0;
}

// order[] = the instances by decreasing cost of their last solve
hipError_t launch_sqp_order(const StateDev& S, int batch, hipStream_t stream) {
    if (batch > 16384) return hipErrorInvalidValue;
    hipLaunchKernelGGL(order_by_cost_kernel, dim3((batch + 255) / 256), dim3(256), 0, stream, S.cost, batch,
                       const_cast<int32_t*>(S.order));
    return hipGetLastError();
}

template <int ID>
static int unc_dims_of(int32_t* unc) {
    for (int q = 0; q < Model<ID>::NUNC; ++q) unc[q] = Model<ID>::unc[q];
    return Model<ID>::NUNC;
}

int model_unc_dims(int model, int32_t* unc) {
    switch (model) {
        case kQuad2D: return unc_dims_of<kQuad2D>(unc);
        case kQuad3D: return unc_dims_of<kQuad3D>(unc);
        case kCartpole: return unc_dims_of<kCartpole>(unc);
    }
    return 0;
}

template <int ID>
static size_t lds_bytes_of(int H) {   // the larger of the default-wave layouts a launch may pick
    return SqpKernel<ID>::lds_doubles(H) * sizeof(double);
}

size_t sqp_lds_bytes(int model, int H) {
    switch (model) {
        case kQuad2D: return lds_bytes_of<kQuad2D>(H);
        case kQuad3D: return lds_bytes_of<kQuad3D>(H);
        case kCartpole: return lds_bytes_of<kCartpole>(H);
    }
    return 0;
}

hipError_t launch_sqp(const ProblemDev& P, const StateDev& S, const StepIO& io, int batch, hipStream_t stream,
                      int first, int count) {
    switch (P.model) {
        case kQuad2D: return launch_sqp_step<kQuad2D>(P, S, io, batch, stream, first, count);
        case kQuad3D: return launch_sqp_step<kQuad3D>(P, S, io, batch, stream, first, count);
        case kCartpole: return launch_sqp_step<kCartpole>(P, S, io, batch, stream, first, count);
    }
    return hipErrorInvalidValue;
}

}  // namespace gpmpc
