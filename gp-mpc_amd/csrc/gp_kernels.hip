// GP posterior kernels on CDNA4 (gfx950):
//
//   gp_post_kernel: mean m(z) = sf2 * sum_i alpha_i e_i (over vrows, i.e. an exact GP) and exact variance
//                   var(z) = sf2 - || L^-1 k(z, X) ||^2 (+ sn2)        (gpmpc/gpmpc.py:441-445)
//   The variance is the dense contraction of the path: V = K_ZX (P x N) * L^-T (N x N,
//   upper triangular) on v_mfma_f64_16x16x4_f64, A-operand tiles generated on the fly
//   (one exp per lane per K-step), triangular K-steps skipped, and the squared row norms
//   reduced in registers.  One wavefront = 16 points; 4 wavefronts per workgroup.
//
//   plant_step_kernel: one RK4 step of the prior-only dynamics with the "true" parameters --
//   the synthetic closed-loop plant that replaces crazyflow's env.step (scripts/run_gp_mpc.py:59).
#include "gpmpc_common.h"
#include "models.h"

namespace gpmpc {

typedef double f64x4 __attribute__((ext_vector_type(4)));


template <bool FROM_STATE>
__device__ __forceinline__ void load_point(const PostArgs& a, int p, double (&z)[3]) {
    if (FROM_STATE) {
        const int b = p / a.H, k = p % a.H;
#pragma unroll
        for (int dd = 0; dd < 3; ++dd) {
            const int s = a.src[dd];
            z[dd] = (dd < a.d) ? (s < a.nx ? a.sx[((size_t)b * (a.H + 1) + k) * a.nx + s]
                                           : a.su[((size_t)b * a.H + k) * a.nu + (s - a.nx)])
                               : 0.0;
        }
    } else {
#pragma unroll
        for (int dd = 0; dd < 3; ++dd) z[dd] = (dd < a.d) ? a.Z[(size_t)p * a.ldz + dd] : 0.0;
    }
}

constexpr int kColTiles = 8;  // 128 output columns per pass over K

template <bool FROM_STATE>
__global__ __launch_bounds__(256) void gp_post_kernel(GPDev g, int npad, PostArgs a) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int p0 = (blockIdx.x * 4 + wave) * 16;
    if (p0 >= a.P) return;
    const int prow = lane & 15;   // A-operand row (point) of this lane
    const int kq = lane >> 4;     // A-operand k / B-operand k of this lane
    const int p = p0 + prow;
    const bool pvalid = p < a.P;
    double z[3];
    load_point<FROM_STATE>(a, pvalid ? p : p0, z);
    const double c = -0.5 * g.inv_ell2;
    const double4* rows = reinterpret_cast<const double4*>(g.vrows);
    const int nsteps = npad / 4;
    double msum = 0.0;
    double sq[4] = {0.0, 0.0, 0.0, 0.0};
    const bool want_var = (a.var != nullptr) && (g.linvT != nullptr);
    const int ngroups = want_var ? (npad + 16 * kColTiles - 1) / (16 * kColTiles) : 1;
    for (int grp = 0; grp < ngroups; ++grp) {
        const int c0 = grp * 16 * kColTiles;
        f64x4 acc[kColTiles];
#pragma unroll
        for (int t = 0; t < kColTiles; ++t) acc[t] = f64x4{0.0, 0.0, 0.0, 0.0};
        // K-steps needed by this column group: i <= last column (L^-T upper triangular)
        const int last_col = min(npad, c0 + 16 * kColTiles) - 1;
        const int s_end = want_var ? min(nsteps, last_col / 4 + 1) : nsteps;
        for (int s = 0; s < s_end; ++s) {
            const int i = 4 * s + kq;
            double kv = 0.0;
            if (i < g.nv && pvalid) {
                const double4 r = rows[i];
                const double xr[3] = {r.x, r.y, r.z};
                double q = 0.0;
#pragma unroll
                for (int dd = 0; dd < 3; ++dd) {
                    const double df = (dd < g.d) ? xr[dd] - z[dd] : 0.0;
                    q = fma(df, df, q);
                }
                kv = g.sf2 * exp(c * q);
                if (grp == ngroups - 1) msum = fma(kv, r.w, msum);  // the last group spans every K-step
            }
            if (want_var) {
                const double* brow = g.linvT + (size_t)i * npad + c0 + (lane & 15);
#pragma unroll
                for (int t = 0; t < kColTiles; ++t) {
                    const int col0 = c0 + 16 * t;
                    if (col0 < npad && 4 * s <= col0 + 15) {   // wave-uniform: skip zero triangle
                        const double bv = brow[16 * t];
                        acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(kv, bv, acc[t], 0, 0, 0);
                    }
                }
            }
        }
        if (want_var) {
            // acc[t][r] = V[row = kq + 4r][col = c0 + 16t + (lane&15)]
#pragma unroll
            for (int t = 0; t < kColTiles; ++t)
#pragma unroll
                for (int r = 0; r < 4; ++r) sq[r] = fma(acc[t][r], acc[t][r], sq[r]);
        }
    }
    // mean: reduce the 4 k-lanes of each point (lanes prow, prow+16, prow+32, prow+48)
    msum += __shfl_xor(msum, 16);
    msum += __shfl_xor(msum, 32);
    if (a.mean != nullptr && kq == 0 && pvalid) a.mean[p] = msum;
    if (want_var) {
        // reduce squared norms over the 16 column lanes sharing kq
#pragma unroll
        for (int r = 0; r < 4; ++r) {
#pragma unroll
            for (int o = 1; o < 16; o <<= 1) sq[r] += __shfl_xor(sq[r], o);
        }
        if ((lane & 15) == 0) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int pr = p0 + kq + 4 * r;
                if (pr < a.P) {
                    const double v = g.sf2 - sq[r] + (a.with_noise ? g.sn2 : 0.0);
                    a.var[(size_t)pr * a.var_stride + a.var_off] = v;
                }
            }
        }
    }
}

hipError_t launch_gp_post(const GPDev& g, int npad, const PostArgs& a, bool from_state, hipStream_t stream) {
    const int waves = (a.P + 15) / 16;
    const int blocks = (waves + 3) / 4;
    if (blocks == 0) return hipSuccess;
    if (from_state)
        hipLaunchKernelGGL(gp_post_kernel<true>, dim3(blocks), dim3(256), 0, stream, g, npad, a);
    else
        hipLaunchKernelGGL(gp_post_kernel<false>, dim3(blocks), dim3(256), 0, stream, g, npad, a);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------- plant
template <int ID>
__global__ void plant_step_kernel(const double* __restrict__ params, double dt, const double* __restrict__ x,
                                  const double* __restrict__ u, double* __restrict__ xn, int32_t* tstep, int B) {
    using M = Model<ID>;
    constexpr int NX = M::NX, NU = M::NU;
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    double p[kMaxParams];
#pragma unroll
    for (int i = 0; i < kMaxParams; ++i) p[i] = params[i];
    double xs[NX], us[NU], k[NX], acc[NX], xi[NX];
    const double gm[kMaxGP] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int i = 0; i < NX; ++i) xs[i] = x[(size_t)b * NX + i];
#pragma unroll
    for (int a = 0; a < NU; ++a) us[a] = u[(size_t)b * NU + a];
    const double cs[4] = {0.0, 0.5, 0.5, 1.0}, ws[4] = {1.0, 2.0, 2.0, 1.0};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
#pragma unroll
        for (int i = 0; i < NX; ++i) xi[i] = (s == 0) ? xs[i] : fma(cs[s] * dt, k[i], xs[i]);
        M::f(p, xi, us, gm, k);
#pragma unroll
        for (int i = 0; i < NX; ++i) acc[i] = (s == 0) ? k[i] : fma(ws[s], k[i], acc[i]);
    }
#pragma unroll
    for (int i = 0; i < NX; ++i) xn[(size_t)b * NX + i] = fma(dt / 6.0, acc[i], xs[i]);
    if (tstep != nullptr) tstep[b] += 1;
}

hipError_t launch_plant(int model, const double* params, double dt, const double* x, const double* u, double* xn,
                        int32_t* tstep, int B, hipStream_t stream) {
    const int blocks = (B + 63) / 64;
    switch (model) {
        case kQuad2D: hipLaunchKernelGGL(plant_step_kernel<kQuad2D>, dim3(blocks), dim3(64), 0, stream, params, dt, x, u, xn, tstep, B); break;
        case kQuad3D: hipLaunchKernelGGL(plant_step_kernel<kQuad3D>, dim3(blocks), dim3(64), 0, stream, params, dt, x, u, xn, tstep, B); break;
        case kCartpole: hipLaunchKernelGGL(plant_step_kernel<kCartpole>, dim3(blocks), dim3(64), 0, stream, params, dt, x, u, xn, tstep, B); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace gpmpc
