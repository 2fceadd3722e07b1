// GP posterior kernels on CDNA4 (gfx950):
//
//   gp_post_kernel: mean m(z) = sf2 * sum_i alpha_i e_i (over vrows, i.e. an exact GP) and exact variance
//                   var(z) = sf2 - || L^-1 k(z, X) ||^2 (+ sn2)        (gpmpc/gpmpc.py:441-445)
//   The variance is the dense contraction of the path: V = K_ZX (P x N) * L^-T (N x N,
//   upper triangular) on v_mfma_f64_16x16x4_f64, A-operand tiles generated on the fly
//   (one exp per lane per K-step), B panels staged in LDS and shared by the workgroup,
//   the zero triangle skipped, squared row norms reduced in registers.  One wavefront =
//   16 points; 8 wavefronts per workgroup; all GPs of a step in one launch (grid.y).
//
//   plant_step_kernel: one RK4 step of the prior-only dynamics with the "true" parameters --
//   the synthetic closed-loop plant that replaces crazyflow's env.step (scripts/run_gp_mpc.py:59).
#include "gpmpc_common.h"
#include "models.h"

#include <algorithm>
#include <atomic>
#include <type_traits>

namespace gpmpc {

typedef double f64x4 __attribute__((ext_vector_type(4)));


template <bool FROM_STATE>
__device__ __forceinline__ void load_point(const PostArgs& a, int p, double (&z)[3]) {
    if (FROM_STATE) {
        const int r = p / a.H, k = p - r * a.H;
        const int b = a.order ? a.order[a.first + r] : r;
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

// ---------------------------------------------------------------------------- posterior
// Workgroup = 8 wavefronts = 128 points.  (L^-1)^T streams through LDS in 16-row panels
// (double-buffered, register-staged global loads), shared by the 8 waves: each panel row
// feeds 8 x 16 points.  Column tiles of one pass stay in accumulators (<= kMaxCT tiles =
// 256 columns; larger N loops over column groups and regenerates the kernel values).
// Only the upper triangle is loaded and multiplied.  The LDS row stride is an odd number of
// 16-column tiles so the four k-rows of a B fragment hit disjoint bank halves.
constexpr int kPostWaves = 8;
constexpr int kMaxCT = 16;

__device__ __forceinline__ double dpp_row_sum(double v) {
    auto mv = [](double x, auto ctrl) {
        const long long b = __double_as_longlong(x);
        const int lo = __builtin_amdgcn_update_dpp(0, (int)b, decltype(ctrl)::value, 0xf, 0xf, false);
        const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), decltype(ctrl)::value, 0xf, 0xf, false);
        return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
    };
    v += mv(v, std::integral_constant<int, 0x128>{});   // row_ror:8
    v += mv(v, std::integral_constant<int, 0x124>{});   // row_ror:4
    v += mv(v, std::integral_constant<int, 0x4E>{});    // quad_perm [2,3,0,1]
    v += mv(v, std::integral_constant<int, 0xB1>{});    // quad_perm [1,0,3,2]
    return v;
}

__host__ __device__ inline int post_ct(int npad) { return npad / 16 < kMaxCT ? npad / 16 : kMaxCT; }
__host__ __device__ inline int post_stride(int ct) { return 16 * (ct | 1); }

// FULL: every column group of the launch has kMaxCT tiles (npad >= 256 for L^-T, >= 256 root
// columns): each panel is staged whole, with zeros for the skipped triangle and past the last
// column, so the K loop runs every tile unconditionally (no scalar branch per MFMA; the few zero
// tiles of each group's diagonal block cost less than the branches did).
template <bool FROM_STATE, bool FULL>
__global__ __launch_bounds__(64 * kPostWaves) void gp_post_kernel(PostBatch pb) {
    extern __shared__ __attribute__((aligned(16))) double panel[];
    const GPDev& g = pb.g[blockIdx.y];
    const PostArgs& a = pb.a[blockIdx.y];
    const int npad = pb.npad[blockIdx.y];
    if ((int)blockIdx.x * kPostWaves * 16 >= a.P) return;   // whole workgroup past the end (uniform)
    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int lc = lane & 15;   // A-operand row (point) / B-operand column of this lane
    const int kq = lane >> 4;   // k index within a K-step
    const int p0 = (blockIdx.x * kPostWaves + wave) * 16;
    const int p = p0 + lc;
    const bool pvalid = p < a.P;
    double z[3];
    load_point<FROM_STATE>(a, pvalid ? p : a.P - 1, z);
    const double c = -0.5 * g.inv_ell2;
    const double4* rows = reinterpret_cast<const double4*>(g.vrows);
    double msum = 0.0;
    auto kval = [&](int i, bool acc_mean) {
        double kv = 0.0;
        if (i < g.nv) {
            const double4 r = rows[i];
            const double xr[3] = {r.x, r.y, r.z};
            double q = 0.0;
#pragma unroll
            for (int dd = 0; dd < 3; ++dd) {
                const double df = (dd < g.d) ? xr[dd] - z[dd] : 0.0;
                q = fma(df, df, q);
            }
            kv = g.sf2 * exp_rbf(c * q);
            if (acc_mean) msum = fma(kv, r.w, msum);
        }
        return kv;
    };
    const bool want_var = (a.var != nullptr) && (g.linvT != nullptr || g.vroot != nullptr);
    double sq[4] = {0.0, 0.0, 0.0, 0.0};
    if (!want_var) {
        for (int s = 0; s < npad / 4; ++s) (void)kval(4 * s + kq, true);
    } else {
        // B = (L^-1)^T (npad x npad, upper triangular: the zero triangle is skipped) or the LOVE
        // root R (npad x vroot_cols, dense: every K row against every column)
        const bool tri = g.vroot == nullptr;
        const double* Bm = tri ? g.linvT : g.vroot;
        const int ncols = tri ? npad : g.vroot_cols;
        const int ntile = ncols / 16;
        const int ct = post_ct(ncols);
        const int Wp = post_stride(ct);
        const int ngroups = (ntile + ct - 1) / ct;
        for (int grp = 0; grp < ngroups; ++grp) {
            const int t0 = grp * ct;
            const int tn = min(ct, ntile - t0);
            const int npan = tri ? t0 + tn : npad / 16;     // K rows < 16 (t0 + tn): upper triangle
            const bool last = grp == ngroups - 1;           // the last group visits every K row
            // staged copy of panel `pan` (columns of tiles >= max(pan, t0) of this group)
            double2 stage[4];
            auto fetch = [&](int pan) {
                if constexpr (FULL) {
                    // the whole 16 x 256 panel: zeros below the diagonal (tiles < pan) and past ncols
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int e = 2 * (tid + j * 64 * kPostWaves);
                        const int row = e >> 8, col = e & 255, gc = 16 * t0 + col;
                        const bool nz = gc < ncols && !(tri && gc < 16 * pan);
                        stage[j] = nz ? *reinterpret_cast<const double2*>(Bm + (size_t)(16 * pan + row) * ncols + gc)
                                      : double2{0.0, 0.0};
                    }
                } else {
                    const int lt0 = tri ? max(pan - t0, 0) : 0, w = 16 * (tn - lt0);
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int e = 2 * (tid + j * 64 * kPostWaves);
                        const int row = e / w, col = e - row * w;
                        stage[j] = (row < 16)
                                       ? *reinterpret_cast<const double2*>(Bm + (size_t)(16 * pan + row) * ncols +
                                                                           16 * (t0 + lt0) + col)
                                       : double2{0.0, 0.0};
                    }
                }
            };
            auto deposit = [&](int pan, double* buf) {
                if constexpr (FULL) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int e = 2 * (tid + j * 64 * kPostWaves);
                        *reinterpret_cast<double2*>(buf + (e >> 8) * Wp + (e & 255)) = stage[j];
                    }
                } else {
                    const int lt0 = tri ? max(pan - t0, 0) : 0, w = 16 * (tn - lt0);
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int e = 2 * (tid + j * 64 * kPostWaves);
                        const int row = e / w, col = e - row * w;
                        if (row < 16) *reinterpret_cast<double2*>(buf + row * Wp + 16 * lt0 + col) = stage[j];
                    }
                }
            };
            f64x4 acc[kMaxCT];
#pragma unroll
            for (int t = 0; t < kMaxCT; ++t) acc[t] = f64x4{0.0, 0.0, 0.0, 0.0};
            fetch(0);
            deposit(0, panel);
            __syncthreads();
            for (int pan = 0; pan < npan; ++pan) {
                const double* buf = panel + (pan & 1) * 16 * Wp;
                if (pan + 1 < npan) fetch(pan + 1);
                const int lt0 = tri ? max(pan - t0, 0) : 0;
                double kvs[4];   // the panel's four kernel values first: independent exps (ILP)
#pragma unroll
                for (int ks = 0; ks < 4; ++ks) kvs[ks] = kval(16 * pan + 4 * ks + kq, last);
#pragma unroll
                for (int ks = 0; ks < 4; ++ks) {
                    const double kv = kvs[ks];
                    const double* brow = buf + (4 * ks + kq) * Wp + lc;
#pragma unroll
                    for (int t = 0; t < kMaxCT; ++t)
                        if (FULL || (t >= lt0 && t < tn))
                            acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(kv, brow[16 * t], acc[t], 0, 0, 0);
                }
                if (pan + 1 < npan) deposit(pan + 1, panel + ((pan + 1) & 1) * 16 * Wp);
                __syncthreads();
            }
            // acc[t][r] = V[point kq + 4r][column 16 (t0 + t) + lc]
#pragma unroll
            for (int t = 0; t < kMaxCT; ++t)
#pragma unroll
                for (int r = 0; r < 4; ++r) sq[r] = (t < tn) ? fma(acc[t][r], acc[t][r], sq[r]) : sq[r];
        }
    }
    // mean: reduce the 4 k-lanes of each point (lanes lc, lc+16, lc+32, lc+48)
    msum += __shfl_xor(msum, 16);
    msum += __shfl_xor(msum, 32);
    if (a.mean != nullptr && kq == 0 && pvalid) a.mean[p] = msum;
    if (want_var) {
#pragma unroll
        for (int r = 0; r < 4; ++r) sq[r] = dpp_row_sum(sq[r]);   // over the 16 column lanes
        if (lc == 0) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int pr = p0 + kq + 4 * r;
                if (pr < a.P) {
                    const double v = g.sf2 - sq[r] + (a.with_noise ? g.sn2 : 0.0);
                    a.var[post_row(a, pr) * a.var_stride + a.var_off] = v;
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------- variance, N <= 256
// The variance-only launch for small training sets (npad <= 256, i.e. NT <= 16 column tiles:
// config 2/3 and the per-step tightening) with every loop bound known at compile time: the
// panel loop is unrolled, so the triangle skip costs no branches and the compiler can hoist
// the B-fragment LDS reads and the next panel's training rows over the MFMAs.  Same math and
// layout as gp_post_kernel: 8 wavefronts x 16 points, (L^-1)^T panels double-buffered in LDS.
template <int NT, bool FROM_STATE>
__global__ __launch_bounds__(64 * kPostWaves) void gp_var_tri_kernel(PostBatch pb) {
    extern __shared__ __attribute__((aligned(16))) double panel[];
    constexpr int W = 16 * (NT | 1);   // odd number of 16-column tiles: conflict-free B fragments
    const GPDev& g = pb.g[blockIdx.y];
    const PostArgs& a = pb.a[blockIdx.y];
    if ((int)blockIdx.x * kPostWaves * 16 >= a.P) return;   // uniform
    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int lc = lane & 15, kq = lane >> 4;
    const int p0 = (blockIdx.x * kPostWaves + wave) * 16;
    const int p = p0 + lc;
    double z[3];
    load_point<FROM_STATE>(a, p < a.P ? p : a.P - 1, z);
    const double c = -0.5 * g.inv_ell2, sf2 = g.sf2;
    const int npad = 16 * NT;
    const double4* rows = reinterpret_cast<const double4*>(g.vrows);
    // staged copy of panel q (rows 16q.., columns >= 16q)
    double2 stage[4];
    auto fetch = [&](int q) {
        const int w = 16 * (NT - q);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int e = 2 * (tid + j * 64 * kPostWaves);
            const int row = e / w, col = e - row * w;
            stage[j] = (row < 16) ? *reinterpret_cast<const double2*>(g.linvT + (size_t)(16 * q + row) * npad + 16 * q + col)
                                  : double2{0.0, 0.0};
        }
    };
    auto deposit = [&](int q, double* buf) {
        const int w = 16 * (NT - q);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int e = 2 * (tid + j * 64 * kPostWaves);
            const int row = e / w, col = e - row * w;
            if (row < 16) *reinterpret_cast<double2*>(buf + row * W + 16 * q + col) = stage[j];
        }
    };
    double4 rw[4];
    auto load_rows = [&](int q) {
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) rw[ks] = rows[16 * q + 4 * ks + kq];
    };
    f64x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f64x4{0.0, 0.0, 0.0, 0.0};
    fetch(0);
    load_rows(0);
    deposit(0, panel);
    __syncthreads();
#pragma unroll
    for (int q = 0; q < NT; ++q) {
        const double* buf = panel + (q & 1) * 16 * W;
        double kv[4];   // k(z_point, x_row) for the four K-steps of the panel (independent exps)
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            const double d0 = rw[ks].x - z[0], d1 = rw[ks].y - z[1], d2 = rw[ks].z - z[2];
            kv[ks] = sf2 * exp_rbf(c * fma(d0, d0, fma(d1, d1, d2 * d2)));
        }
        if (q + 1 < NT) {
            fetch(q + 1);
            load_rows(q + 1);
        }
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            const double* brow = buf + (4 * ks + kq) * W + lc;
#pragma unroll
            for (int t = q; t < NT; ++t) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(kv[ks], brow[16 * t], acc[t], 0, 0, 0);
        }
        if (q + 1 < NT) deposit(q + 1, panel + ((q + 1) & 1) * 16 * W);
        __syncthreads();
    }
    // acc[t][r] = V[point kq + 4r][column 16 t + lc]
    double sq[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) sq[r] = fma(acc[t][r], acc[t][r], sq[r]);
#pragma unroll
    for (int r = 0; r < 4; ++r) sq[r] = dpp_row_sum(sq[r]);
    if (lc == 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int pr = p0 + kq + 4 * r;
            if (pr < a.P) a.var[post_row(a, pr) * a.var_stride + a.var_off] = sf2 - sq[r] + (a.with_noise ? g.sn2 : 0.0);
        }
    }
}

// ---------------------------------------------------------------------------- variance, N <= 256, few points
// The same variance when the launch has too few points to fill the device (the tightening of the
// strong-scaled shards: 128-256 instances, 30-60 workgroups of 128 points per GP): a wave of
// gp_var_tri_kernel owns 16 points against every column tile of the triangle (364 dependent-free
// but serially issued MFMAs at NT = 13), so a sparse launch lasts one wave's MFMA stream.  Here the
// column tiles of a 16-point tile are split over S waves (snake order over the triangle's per-tile
// work: 24 / 23 / 22 / 22 panels at NT = 13, S = 4), the workgroup's 8 waves covering 8/S point tiles:
// S times the waves, each with 1/S of the MFMAs.  The kernel values are computed once per point
// tile (wave cg takes K-steps cg, cg + S, ..) and exchanged through LDS one panel ahead, behind the
// panel barrier the L^-T staging already has.  Each wave reduces its tiles' squared norms; the
// S partial norms of a point are added in wave order (deterministic) by the tile's first wave.
__host__ __device__ constexpr int split_owner(int t, int nt, int s) {
    const int i = nt - 1 - t;   // position in descending per-tile work (tile t: t + 1 panels)
    const int r = i / s, j = i % s;
    return (r & 1) ? s - 1 - j : j;
}

template <int NT, bool FROM_STATE, int S, int CG>
__device__ __forceinline__ void var_split_body(const GPDev& g, const PostArgs& a, double* panel, double* kvb,
                                               double* red, int pt) {
    constexpr int PT = kPostWaves / S;   // point tiles per workgroup
    constexpr int W = 16 * (NT | 1);
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int lc = lane & 15, kq = lane >> 4;
    const int p0 = (blockIdx.x * PT + pt) * 16;
    const int p = p0 + lc;
    double z[3];
    load_point<FROM_STATE>(a, p < a.P ? p : a.P - 1, z);
    const double c = -0.5 * g.inv_ell2, sf2 = g.sf2;
    constexpr int npad = 16 * NT;
    const double4* rows = reinterpret_cast<const double4*>(g.vrows);
    double2 stage[4];
    auto fetch = [&](int q) {
        const int w = 16 * (NT - q);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int e = 2 * (tid + j * 64 * kPostWaves);
            const int row = e / w, col = e - row * w;
            stage[j] = (row < 16) ? *reinterpret_cast<const double2*>(g.linvT + (size_t)(16 * q + row) * npad + 16 * q + col)
                                  : double2{0.0, 0.0};
        }
    };
    auto deposit = [&](int q, double* buf) {
        const int w = 16 * (NT - q);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int e = 2 * (tid + j * 64 * kPostWaves);
            const int row = e / w, col = e - row * w;
            if (row < 16) *reinterpret_cast<double2*>(buf + row * W + 16 * q + col) = stage[j];
        }
    };
    // this wave's K-steps of panel q: exps into kvb[q & 1][pt][ks][lane]
    auto kvals = [&](int q) {
        double* dst = kvb + ((size_t)(q & 1) * PT + pt) * 4 * 64 + lane;
#pragma unroll
        for (int ks = CG; ks < 4; ks += S) {
            const double4 rw = rows[16 * q + 4 * ks + kq];
            const double d0 = rw.x - z[0], d1 = rw.y - z[1], d2 = rw.z - z[2];
            dst[ks * 64] = sf2 * exp_rbf(c * fma(d0, d0, fma(d1, d1, d2 * d2)));
        }
    };
    f64x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f64x4{0.0, 0.0, 0.0, 0.0};
    fetch(0);
    kvals(0);
    deposit(0, panel);
    __syncthreads();
#pragma unroll
    for (int q = 0; q < NT; ++q) {
        const double* buf = panel + (q & 1) * 16 * W;
        double kv[4];
        const double* src = kvb + ((size_t)(q & 1) * PT + pt) * 4 * 64 + lane;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) kv[ks] = src[ks * 64];
        if (q + 1 < NT) {
            fetch(q + 1);
            kvals(q + 1);
        }
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            const double* brow = buf + (4 * ks + kq) * W + lc;
#pragma unroll
            for (int t = q; t < NT; ++t)   // (unrolled: the ownership test folds)
                if (split_owner(t, NT, S) == CG)
                    acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(kv[ks], brow[16 * t], acc[t], 0, 0, 0);
        }
        if (q + 1 < NT) deposit(q + 1, panel + ((q + 1) & 1) * 16 * W);
        __syncthreads();
    }
    double sq[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int t = 0; t < NT; ++t)
        if (split_owner(t, NT, S) == CG) {
#pragma unroll
            for (int r = 0; r < 4; ++r) sq[r] = fma(acc[t][r], acc[t][r], sq[r]);
        }
#pragma unroll
    for (int r = 0; r < 4; ++r) sq[r] = dpp_row_sum(sq[r]);
    if (lc == 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) red[((size_t)pt * S + CG) * 16 + kq + 4 * r] = sq[r];
    }
    __syncthreads();
    if (CG == 0 && lane < 16) {
        double v = 0.0;
#pragma unroll
        for (int w = 0; w < S; ++w) v += red[((size_t)pt * S + w) * 16 + lane];
        const int pr = p0 + lane;
        if (pr < a.P) a.var[post_row(a, pr) * a.var_stride + a.var_off] = sf2 - v + (a.with_noise ? g.sn2 : 0.0);
    }
}

template <int NT, bool FROM_STATE, int S>
__global__ __launch_bounds__(64 * kPostWaves) void gp_var_split_kernel(PostBatch pb) {
    extern __shared__ __attribute__((aligned(16))) double panel[];
    constexpr int PT = kPostWaves / S;
    constexpr int W = 16 * (NT | 1);
    const GPDev& g = pb.g[blockIdx.y];
    const PostArgs& a = pb.a[blockIdx.y];
    if ((int)blockIdx.x * PT * 16 >= a.P) return;   // uniform
    double* kvb = panel + 2 * 16 * W;                // [2][PT][4][64]
    double* red = kvb + 2 * PT * 4 * 64;             // [PT][S][16]
    const int wave = threadIdx.x >> 6;
    const int pt = wave / S, cg = wave % S;
    static_assert(S == 4, "four column groups (the shipped split; two measured slower)");
    switch (cg) {   // wave-uniform: the column ownership is compile-time inside each body
        case 0: var_split_body<NT, FROM_STATE, S, 0>(g, a, panel, kvb, red, pt); break;
        case 1: var_split_body<NT, FROM_STATE, S, 1>(g, a, panel, kvb, red, pt); break;
        case 2: var_split_body<NT, FROM_STATE, S, 2>(g, a, panel, kvb, red, pt); break;
        default: var_split_body<NT, FROM_STATE, S, 3>(g, a, panel, kvb, red, pt); break;
    }
}
__host__ __device__ constexpr int var_split_lds(int nt, int s) {
    return (2 * 16 * 16 * (nt | 1) + 2 * (kPostWaves / s) * 4 * 64 + kPostWaves * 16) * (int)sizeof(double);
}

// ---------------------------------------------------------------------------- variance, LOVE root
// var(z) = sf2 - ||R^T k(z, X)||^2 (+ sn2) with the dense LOVE root R [npad][rank, padded to 16]
// (gpytorch fast_pred_var, rank <= 100 for configs 4/5).  No LDS and no barriers: one wavefront =
// 16 points, K-steps of four training rows (lane (kq, lc): point lc, row 4s + kq), four K-steps per
// round, the next K-step's exp computed behind the current K-step's MFMAs, and the next round's
// training rows and root entries loaded a round ahead (the blocks of one GP run together, so its
// root, 3.6 MB at N = 4000 and 112
// columns, streams through L2 once per wave generation).  Per GP (love_tiles) the root's columns
// go to nf full 16-column tiles on v_mfma_f64_16x16x4_f64 (accumulators acc[t]) and, when at most
// 8 columns remain, nq <= 2 four-column quads on v_mfma_f64_4x4x4_4b_f64, whose A operand is the
// same register (block b takes A_b[m][k] from lane 16k + 4b + m = point 4b + m, row k) and whose B
// operand is the quad's four columns replicated over the blocks: D_b[m][n] (lane 16m + 4b + n) is
// point 4b + m against column n, a quarter of a 16-column tile's matrix-core cycles for the last
// 4 of a rank-100 root's columns (the tile would be 12/16 padding).  Each GP of the launch does
// only its own tiles (the 12-column thrust root of config 4 one tile, not the pitch root's 7).
// The two round buffers take the kernel past 256 VGPRs, one wave per SIMD (two measured slower).
// sf2 is applied to the squared norm (sf2^2), not to every kernel value.
constexpr int kLoveWaves = 4;
constexpr int kLoveMaxTiles = 8;
__host__ __device__ inline void love_tiles(int rank, int& nf, int& nq) {
    nf = rank >> 4;
    const int rem = rank & 15;
    nq = (rem + 3) >> 2;
    if (nq > 2) { nf += 1; nq = 0; }
}
// One wave's 16 points against one GP's root with NF full tiles and NQ quads, both compile-time
// (love_dispatch picks the instantiation per block): with runtime tile counts every MFMA and every
// root load of the K loop sat behind its own scalar branch, and the loop body was ~40 basic blocks
// the scheduler could not work across.  Round 3: config 4 LOVE 0.339 -> 0.227 ms, config 5
// 1.50 -> 1.06 ms (profiles/r3/ab_love_pipe/).  Each K-step's MFMAs are followed by the next
// K-step's kernel value (one exp per lane), which runs while the matrix core works; pinning an
// MFMA / 4-VALU interleave with sched_group_barrier measured slower (0.257 ms).
template <int NF, int NQ, bool FROM_STATE>
__device__ __forceinline__ void love_points(const GPDev& g, const PostArgs& a, int npad, int p0, int lane) {
    constexpr int NFa = NF > 0 ? NF : 1, NQa = NQ > 0 ? NQ : 1;
    const int lc = lane & 15, kq = lane >> 4;
    const int p = p0 + lc;
    double z[3];
    load_point<FROM_STATE>(a, p < a.P ? p : a.P - 1, z);
    const double c = -0.5 * g.inv_ell2;
    const double4* rows = reinterpret_cast<const double4*>(g.vrows);
    const int NC = g.vroot_cols;   // row stride of the padded root
    const double* Rl = g.vroot + kq * NC + lc;                        // R[16 s4 + 4 ks + kq][16 t + lc]
    const double* Rq = g.vroot + kq * NC + 16 * NF + (lc & 3);        // R[..][16 NF + 4 q + n]
    const int nv = g.nv, nround = npad / 16;
    struct Round { double4 x[4]; double b[4][NFa]; double bq[4][NQa]; };
    auto load = [&](int s4, Round& rd) {
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            const int i = 16 * s4 + 4 * ks + kq;
            rd.x[ks] = rows[i < nv ? i : 0];
            const size_t ro = (size_t)(16 * s4 + 4 * ks) * NC;
#pragma unroll
            for (int t = 0; t < NF; ++t) rd.b[ks][t] = Rl[ro + 16 * t];
#pragma unroll
            for (int q = 0; q < NQ; ++q) rd.bq[ks][q] = Rq[ro + 4 * q];
        }
    };
    // kernel value of K-step ks of round s4 (row 16 s4 + 4 ks + kq, point lc); rows past the
    // training set, and the round after the last (its rows stale), give 0
    auto kval = [&](const Round& rd, int s4, int ks) {
        const double4 r = rd.x[ks];
        const double d0 = r.x - z[0], d1 = r.y - z[1], d2 = r.z - z[2];
        const double e = exp_rbf(c * fma(d0, d0, fma(d1, d1, d2 * d2)));   // unused dims are zero on both sides
        return (16 * s4 + 4 * ks + kq < nv) ? e : 0.0;
    };
    f64x4 acc[NFa];
#pragma unroll
    for (int t = 0; t < NFa; ++t) acc[t] = f64x4{0.0, 0.0, 0.0, 0.0};
    double accq[NQa];
#pragma unroll
    for (int q = 0; q < NQa; ++q) accq[q] = 0.0;
    // the round's four K-steps; kv holds the current K-step's kernel value and leaves with the
    // next round's first one (rows of `nx`, loaded one round ahead)
    auto round = [&](const Round& rd, int s4, double& kv, const Round& nx) {
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
#pragma unroll
            for (int t = 0; t < NF; ++t) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(kv, rd.b[ks][t], acc[t], 0, 0, 0);
#pragma unroll
            for (int q = 0; q < NQ; ++q) accq[q] = __builtin_amdgcn_mfma_f64_4x4x4f64(kv, rd.bq[ks][q], accq[q], 0, 0, 0);
            kv = (ks < 3) ? kval(rd, s4, ks + 1) : kval(nx, s4 + 1, 0);
        }
    };
    Round r0, r1;
    load(0, r0);
    double kv = kval(r0, 0, 0);
    int s4 = 0;
    for (; s4 + 1 < nround; s4 += 2) {
        load(s4 + 1, r1);
        round(r0, s4, kv, r1);
        if (s4 + 2 < nround) load(s4 + 2, r0);
        round(r1, s4 + 1, kv, r0);
    }
    if (s4 < nround) round(r0, s4, kv, r1);
    // acc[t][r]: point kq + 4r, column 16 t + lc; accq[q] (lane 16 m + 4 b + n): point 4 b + m,
    // column 16 NF + 4 q + n, i.e. row kq's point kq + 4r sits in the lanes of quad r
    double tq = 0.0;
#pragma unroll
    for (int q = 0; q < NQ; ++q) tq = fma(accq[q], accq[q], tq);
    double sq[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) sq[r] = ((lc >> 2) == r) ? tq : 0.0;
#pragma unroll
    for (int t = 0; t < NF; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) sq[r] = fma(acc[t][r], acc[t][r], sq[r]);
#pragma unroll
    for (int r = 0; r < 4; ++r) sq[r] = dpp_row_sum(sq[r]);   // over the 16 column lanes
    if (lc == 0) {
        const double sf2sq = g.sf2 * g.sf2;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int pr = p0 + kq + 4 * r;
            if (pr < a.P) a.var[post_row(a, pr) * a.var_stride + a.var_off] = g.sf2 - sf2sq * sq[r] + (a.with_noise ? g.sn2 : 0.0);
        }
    }
}

// (NF, NQ) of the block's GP -> its instantiation (key 3 NF + NQ, NF <= kLoveMaxTiles, NQ <= 2)
template <int K, bool FROM_STATE>
__device__ __forceinline__ void love_dispatch(int key, const GPDev& g, const PostArgs& a, int npad, int p0, int lane) {
    if (key == K) {
        love_points<K / 3, K % 3, FROM_STATE>(g, a, npad, p0, lane);
        return;
    }
    if constexpr (K + 1 < 3 * (kLoveMaxTiles + 1)) love_dispatch<K + 1, FROM_STATE>(key, g, a, npad, p0, lane);
}

template <bool FROM_STATE>
__global__ __launch_bounds__(64 * kLoveWaves) void gp_love_kernel(PostBatch pb) {
    // by-value copies: the dynamically indexed kernel-argument arrays otherwise go to scratch
    // when referenced from the dispatched bodies
    const GPDev g = pb.g[blockIdx.y];
    const PostArgs a = pb.a[blockIdx.y];
    const int npad = pb.npad[blockIdx.y];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int p0 = (blockIdx.x * kLoveWaves + wave) * 16;
    if (p0 >= a.P) return;   // wave-uniform
    int nf, nq;              // this GP's full tiles and four-column quads
    love_tiles(g.vroot_rank, nf, nq);
    love_dispatch<1, FROM_STATE>(3 * nf + nq, g, a, npad, p0, lane);
}

template <bool FROM_STATE>
hipError_t launch_love(const PostBatch& pb, hipStream_t stream) {
    int blocks = 0;
    for (int q = 0; q < pb.n; ++q) blocks = max(blocks, (pb.a[q].P + 16 * kLoveWaves - 1) / (16 * kLoveWaves));
    hipLaunchKernelGGL((gp_love_kernel<FROM_STATE>), dim3(blocks, pb.n), dim3(64 * kLoveWaves), 0, stream, pb);
    return hipGetLastError();
}

template <bool FROM_STATE, int NT = 1>
hipError_t launch_var_tri(const PostBatch& pb, int ntile, int blocks, int split, hipStream_t stream) {
    if constexpr (NT <= kMaxCT) {
        if (ntile == NT) {
            if (split == 4) {   // few points: column tiles over four waves per point tile
                static bool sattr = false;
                const int lds = var_split_lds(NT, split);
                auto* k = gp_var_split_kernel<NT, FROM_STATE, 4>;
                if (!sattr) {
                    const hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
                    if (e != hipSuccess) return e;
                    sattr = true;
                }
                const int pts = 16 * (kPostWaves / split);
                int sblocks = 0;
                for (int q = 0; q < pb.n; ++q) sblocks = std::max(sblocks, (pb.a[q].P + pts - 1) / pts);
                hipLaunchKernelGGL(k, dim3(sblocks, pb.n), dim3(64 * kPostWaves), lds, stream, pb);
                return hipGetLastError();
            }
            static bool attr = false;
            const int lds = 2 * 16 * 16 * (NT | 1) * (int)sizeof(double);
            if (!attr) {
                const hipError_t e = hipFuncSetAttribute((const void*)gp_var_tri_kernel<NT, FROM_STATE>,
                                                         hipFuncAttributeMaxDynamicSharedMemorySize, lds);
                if (e != hipSuccess) return e;
                attr = true;
            }
            hipLaunchKernelGGL((gp_var_tri_kernel<NT, FROM_STATE>), dim3(blocks, pb.n), dim3(64 * kPostWaves), lds,
                               stream, pb);
            return hipGetLastError();
        }
        return launch_var_tri<FROM_STATE, NT + 1>(pb, ntile, blocks, split, stream);
    }
    return hipErrorInvalidValue;
}

hipError_t launch_gp_post_batch(const PostBatch& pb, bool from_state, hipStream_t stream) {
    int blocks = 0;
    size_t lds = 0;
    for (int q = 0; q < pb.n; ++q) {
        blocks = max(blocks, (pb.a[q].P + 16 * kPostWaves - 1) / (16 * kPostWaves));
        if (pb.a[q].var != nullptr && (pb.g[q].linvT != nullptr || pb.g[q].vroot != nullptr)) {
            const int ncols = pb.g[q].vroot ? pb.g[q].vroot_cols : pb.npad[q];
            lds = std::max(lds, (size_t)2 * 16 * post_stride(post_ct(ncols)) * sizeof(double));
        }
    }
    if (blocks == 0 || pb.n == 0) return hipSuccess;
    bool love = true;   // every entry variance-only with a LOVE root of <= 128 columns
    for (int q = 0; q < pb.n; ++q) {
        love = love && pb.a[q].mean == nullptr && pb.a[q].var != nullptr && pb.g[q].vroot != nullptr &&
               pb.g[q].vroot_cols % 16 == 0 && pb.g[q].vroot_cols <= 16 * kLoveMaxTiles &&
               pb.g[q].vroot_rank >= 1 && pb.g[q].vroot_rank <= pb.g[q].vroot_cols;
    }
    if (love)
        return from_state ? launch_love<true>(pb, stream) : launch_love<false>(pb, stream);
    bool tri = true;   // every entry variance-only with the same npad <= 256
    for (int q = 0; q < pb.n; ++q)
        tri = tri && pb.a[q].mean == nullptr && pb.a[q].var != nullptr && pb.g[q].linvT != nullptr &&
              pb.g[q].vroot == nullptr && pb.npad[q] == pb.npad[0] && pb.npad[q] <= 16 * kMaxCT;
    if (tri) {
        // column split over four waves when the 128-point workgroups would fill at most half the CUs
        // (measured, profiles/r4/ab_varsplit/: 128 quad2d instances 35.9 -> 19.7 us, 256: 36.5 -> 28.5 us,
        // cartpole 256: 10.1 -> 9.0 us; at 512 and 1024 instances the split is slower: 38 -> 42 / 51 us,
        // 71 -> 77 us; two waves per point tile measured between the two, eight: 128 instances 19 us,
        // 256: 33 us, ab_varsplit8/).  PostBatch::var_split = 1 / 4 forces a choice (GPMPC_TUNE_VAR_SPLIT).
        static const int ncu = [] {   // (thread-safe one-time initialisation)
            int dev = 0, n = 0;
            if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
                n = 256;
            return n;
        }();
        const int step_blocks = pb.step_points > 0 ? (pb.step_points + 16 * kPostWaves - 1) / (16 * kPostWaves) : blocks;
        const int wgs = step_blocks * pb.n;   // the split choice follows the whole step (bit-identical halves)
        int split = 2 * wgs <= ncu ? 4 : 1;
        if (pb.var_split == 1 || pb.var_split == 4) split = pb.var_split;
        return from_state ? launch_var_tri<true>(pb, pb.npad[0] / 16, blocks, split, stream)
                          : launch_var_tri<false>(pb, pb.npad[0] / 16, blocks, split, stream);
    }
    // dynamic-LDS limit of the post kernels, raised once per process; the latch is atomic because
    // handles on different host threads may launch concurrently (a race sets the same attribute
    // twice, which is harmless), and it stays clear when a call fails so the next launch retries
    static std::atomic<bool> attr{false};
    if (!attr.load(std::memory_order_acquire)) {
        const int mx = 2 * 16 * post_stride(kMaxCT) * (int)sizeof(double);
        for (const void* k : {(const void*)gp_post_kernel<true, false>, (const void*)gp_post_kernel<false, false>,
                              (const void*)gp_post_kernel<true, true>, (const void*)gp_post_kernel<false, true>}) {
            const hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, mx);
            if (e != hipSuccess) return e;
        }
        attr.store(true, std::memory_order_release);
    }
    bool full = true;   // every variance entry's column groups have kMaxCT tiles
    for (int q = 0; q < pb.n; ++q) {
        const bool var = pb.a[q].var != nullptr && (pb.g[q].linvT != nullptr || pb.g[q].vroot != nullptr);
        const int ncols = pb.g[q].vroot ? pb.g[q].vroot_cols : pb.npad[q];
        full = full && (!var || post_ct(ncols) == kMaxCT);
    }
    auto* k = from_state ? (full ? gp_post_kernel<true, true> : gp_post_kernel<true, false>)
                         : (full ? gp_post_kernel<false, true> : gp_post_kernel<false, false>);
    hipLaunchKernelGGL(k, dim3(blocks, pb.n), dim3(64 * kPostWaves), lds, stream, pb);
    return hipGetLastError();
}

hipError_t launch_gp_post(const GPDev& g, int npad, const PostArgs& a, bool from_state, hipStream_t stream) {
    PostBatch pb{};
    pb.g[0] = g;
    pb.a[0] = a;
    pb.npad[0] = npad;
    pb.n = 1;
    return launch_gp_post_batch(pb, from_state, stream);
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
