// Shared host/device definitions for the MI355X GP-MPC solve path.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace gpmpc {

constexpr int kMaxGP = 4;       // GPs per model (quad3d: 3)
constexpr int kMaxGPDim = 3;    // inputs per GP (packed rows are 4 doubles: x0,x1,x2,alpha)
constexpr int kMaxNX = 12;
constexpr int kMaxNU = 4;
constexpr int kMaxH = 63;       // one lane per stage 0..H (64-lane wavefront)
constexpr int kPhases = 12;  // diagnostic phase slots (GPMPC_TIMING builds)
constexpr int kMaxParams = 16;
constexpr int kStatsSlots = 12;  // per-instance solver statistics (gpmpc_set_stats_buffer, = GPMPC_STATS_SLOTS)

enum ModelId : int32_t { kQuad2D = 0, kQuad3D = 1, kCartpole = 2 };

// acados status codes (acados_c/ocp_nlp_interface.h) -- gpmpc/gpmpc.py:365
enum SolveStatus : int32_t { kSuccess = 0, kNaN = 1, kMaxIter = 2, kMinStep = 3, kQPFailure = 4 };

// One GP replica in device memory.
struct GPDev {
    const double* rows;   // [n][4]: mean inputs (d <= 3, zero padded) + weight alpha = K^-1 y (gpmpc/gp.py:84-85)
                          //         (FITC: inducing inputs + posterior weights, gpmpc/gpmpc.py:377-400)
    const double* vrows;  // [nv][4]: training inputs of the variance GP (== rows for an exact GP)
    const double* linvT;  // [npad][npad] row-major (L^-1)^T, L = chol(K); NULL -> no variance
    // MFMA tile pack of the mean rows (the SQP linearisation's GP sums, sqp_kernel.hip gp_tiles):
    //   tX[t][16][4]     rows [(x_i - xbar)/ell^2 (zero padded to 3 dims), c|x_i - xbar|^2],
    //                    c = -1/(2 ell^2); rows past n are zero
    //   tW[t][4][4][4]   for lane group g and output column j: {W[i][j], i = 16t+g+4r, r = 0..3},
    //                    W[i] = [alpha_i, alpha_i (x_i - xbar)]
    const double* tX;
    const double* tW;
    int32_t ntile;
    double xbar[3];       // centre of the mean rows (the RBF kernel is shift invariant)
    int32_t n;
    int32_t nv;
    int32_t d;
    // LOVE root (gpytorch fast_pred_var, gpmpc/gpmpc.py:442-444): [npad][vroot_cols] row-major,
    // R R^T ~ (K + sn2 I)^-1; when set, the variance is sf2 - ||R^T k||^2 instead of the exact
    // triangular form (set only in the tightening's variance launch).  NULL: exact.
    const double* vroot;
    int32_t vroot_cols;   // padded to 16
    int32_t vroot_rank;   // the root's columns before padding
    double inv_ell2;      // 1 / lengthscale^2 (isotropic RBF, gpmpc/gp.py:34)
    double sf2;           // outputscale
    double sn2;           // likelihood noise (gpmpc/gp.py:31)
};

// Everything the per-step kernels need, passed by value.
struct ProblemDev {
    int32_t model;
    int32_t nx, nu, H;
    int32_t n_gp;
    int32_t use_gp;           // 0: nominal MPC (gpmpc/mpc.py)
    double dt;
    double cost_scale;        // acados cost_scaling for stages 0..H-1 (time step), 1 for terminal
    double uh;                // h <= uh: -1e-8 GPMPC (gpmpc.py:309-314), +1e-8 MPC (mpc.py:157-162)
    double params[kMaxParams];
    double x_lo[kMaxNX], x_hi[kMaxNX], u_lo[kMaxNU], u_hi[kMaxNU];
    double q[kMaxNX], r[kMaxNU], u_eq[kMaxNU];
    // reference trajectory (nx, L) column-major by time: traj[t * nx + i]   (gpmpc.py:509-514)
    const double* traj;
    int32_t traj_len;
    // tightening (gpmpc.py:425-498)
    int32_t tighten;
    double icdf;
    double Acl[kMaxNX * kMaxNX];   // A_d + B_d K_lqr (the four-term update of gpmpc.py:489-495)
    double K[kMaxNU * kMaxNX];     // K_lqr
    // diag of Sigma_k and K Sigma_k K^T as a convolution of the per-stage GP noise (Sigma_0 = 0,
    // Sigma_{k+1} = Acl Sigma_k Acl^T + Bd D_k Bd^T with D_k diagonal):
    //   tgain[m][v][q] = (Acl^m Bd)_{vq}^2 (v < nx),  (K Acl^m Bd)_{v-nx,q}^2 (v >= nx),  m = 0..H-1
    const double* tgain;
    // SQP / QP options (gpmpc.py:257-263; acados default tolerances)
    int32_t max_iter, qp_max_iter;
    double tol_stat, tol_eq, tol_ineq, tol_comp, qp_tol, qp_mu0;
    // linearisation cache generation: bumped by every host call that changes what the
    // linearisation depends on (iterate, GPs, model parameters, GP switch); 0 disables the cache
    int32_t lin_gen;
    // launch shape of the SQP kernel: waves per instance (0: auto -- four when batch <= n_cu for the
    // single-tile models, sqp_kernel.hip sqp_waves)
    int32_t waves;
    int32_t n_cu;             // compute units of the device (set by gpmpc_create)
    // cost-ordered dispatch (StateDev::order): on when a launch has more instances than the
    // device holds at once (gpmpc_set_tuning GPMPC_TUNE_ORDER: 0 off, 2 ranks every launch)
    int32_t order_dispatch;
    // segment-parallel Newton solves when the launch runs two or four waves per instance (single-tile
    // models; gpmpc_set_tuning GPMPC_TUNE_SEG)
    int32_t seg;
    // the boundary chain's pivot threshold relative to Ph's largest diagonal entry (gpmpc_set_tuning
    // GPMPC_TUNE_SEG_PIVOT): below it the solve falls back to the one-segment recursion
    double seg_piv_rel;
    GPDev gp[kMaxGP];
};

// Per-instance state owned by the handle (acados keeps the same in its memory).
struct StateDev {
    double* x;        // [B][H+1][nx] iterate / previous solution (x_prev)
    double* u;        // [B][H][nu]
    double* pi;       // [B][H][nx]  dynamics multipliers
    double* lam;      // [B][H+1][2*nb] bound multipliers (lower | upper), nb = nx+nu
    int32_t* has_prev;   // [B] previous solution valid -> tighten (gpmpc.py:432-433)
    const double* var;   // [B][H][n_gp] GP variances at the previous solution (incl. noise)
    double* tight;       // [B][H+1][2*nb] tightening values (state lo|hi, input lo|hi), optional
    // Linearisation of the stored iterate (x, u above): [B][H][nx][nb+1], per stage the rows of
    // [A_k B_k | F_k] with F_k = RK4(x_k, u_k), written by the step that produced the iterate.
    // The next step's first SQP iteration linearises at exactly that iterate (acados keeps it as
    // the initial guess), so it reads the rows instead of recomputing them when lin_tag[b] equals
    // ProblemDev::lin_gen.  Optional (NULL: always recompute).
    double* lin;
    int32_t* lin_tag;    // [B]
    // Cost-ordered dispatch.  cost[b]: the work of instance b's last solve, SQP iterations and IPM
    // iterations weighted by their measured cycle ratio (written by every SQP launch, optional;
    // in-kernel timestamps cost the single-wave kernel 48 B/lane of scratch).  order[blockIdx.x] = instance: when a launch needs more than one
    // round of workgroups (config 5: 512 instances, one per CU), launch_sqp fills order[] with the
    // instances by decreasing previous cost, so the dispatcher starts the slowest instances first
    // and the fast ones fill in behind them (longest-processing-time-first; an instance's cost
    // barely changes from one control step to the next).  NULL: identity.
    const int32_t* order;
    uint32_t* cost;      // [B]
    // rank of this launch's first workgroup in order[] (a launch over ranks first .. first + grid - 1:
    // the two halves of an overlapped step, capi.hip gpmpc_solve); 0 otherwise
    int32_t first;
};

struct StepIO {
    const double* x0;        // [B][nx]
    const int32_t* tstep;    // [B] reference index
    double* u0;              // [B][nu] out
    int32_t* status;         // [B] out
    int32_t* sqp_iter;       // [B] out
    int32_t* qp_iter;        // [B] out, total IPM iterations
    double* res;             // [B][4] out, final NLP residuals (stat, eq, ineq, comp)
    unsigned long long* timing;  // [B][kPhases] phase cycles (GPMPC_TIMING builds only), may be null
    long long* stats;            // [B][kStatsSlots] sqp iters, qp iters (sums), status 0..4 counts,
                                 // max sqp iters, max qp iters per solve, linearisations
                                 // computed, the instance's solve time in s_memrealtime ticks
                                 // (sum; the last solve's); may be null
};

// Arguments of the GP posterior kernel (gp_kernels.hip).
struct PostArgs {
    // points: either dense Z[P][ldz] (first d columns), or gathered from the solver state
    const double* Z;
    int32_t ldz;
    const double* sx;     // state x [B][H+1][nx]
    const double* su;     // state u [B][H][nu]
    int32_t H, nx, nu, ngp, gp_index;
    int32_t src[3];       // var input map into z = [x; u] (gpmpc.py:437-444)
    int32_t P;            // number of points
    int32_t d;
    int32_t with_noise;
    double* mean;         // [P] or null
    double* var;          // var[p * var_stride + var_off] or null
    int32_t var_stride, var_off;
    // gathered points only: point p is stage p % H of the instance of rank first + p / H in order[]
    // (var row: that instance's), or of instance p / H when order is null
    const int32_t* order;
    int32_t first;
};

// var row of point p (see PostArgs::order)
__device__ __forceinline__ size_t post_row(const PostArgs& a, int p) {
    if (a.order == nullptr) return (size_t)p;
    const int r = p / a.H;
    return (size_t)a.order[a.first + r] * a.H + (p - r * a.H);
}

// exp(x) for the RBF kernel, x <= 0 and finite: Cody-Waite reduction x = n ln2 + r, |r| <= ln2/2,
// degree-11 Chebyshev fit of exp on [-ln2/2, ln2/2] (mpmath chebyfit, fit error 3.2e-18; max
// relative error of this f64 evaluation 1 ulp on a 2e5-point grid), scale by 2^n.  n comes from
// the magic-number rounding t = x log2(e) + 1.5 2^52 (one fma; the low word of t is n in two's
// complement) and 2^n is applied by an integer add to the exponent field of p, so the f64 work
// is 15 operations instead of 17 (rint, cvt and ldexp gone).  n is clamped at -1022 for the
// scaling: below exp(-708) the result is p 2^-1022 (< 3e-308) instead of a denormal or 0.
// No overflow/NaN guards: the argument is -0.5 q/ell^2.
__device__ __forceinline__ double exp_rbf(double x) {
    constexpr double kMagic = 6755399441055744.0;   // 1.5 * 2^52
    const double t = fma(x, 1.4426950408889634, kMagic);
    const double n = t - kMagic;
    double r = fma(n, -6.93147180369123816490e-01, x);
    r = fma(n, -1.90821492927058770002e-10, r);
    double p = 2.5110037605963777e-08;
    p = fma(p, r, 2.763263963904103e-07);
    p = fma(p, r, 2.755724091857897e-06);
    p = fma(p, r, 2.4801485482328494e-05);
    p = fma(p, r, 0.00019841269890047113);
    p = fma(p, r, 0.0013888888952314775);
    p = fma(p, r, 0.008333333333319601);
    p = fma(p, r, 0.0416666666664881);
    p = fma(p, r, 0.1666666666666668);
    p = fma(p, r, 0.5000000000000019);
    p = fma(p, r, 1.0);
    p = fma(p, r, 1.0);
    const int ni = max(__double2loint(t), -1022);
    return __hiloint2double(__double2hiint(p) + (ni << 20), __double2loint(p));
}

// exp_rbf of K independent arguments, written step by step across the K values.  One wave
// issues an f64 VALU operation every ~5.5 cycles whether or not it depends on the previous one,
// but a dependent one waits ~7.3 (tools/probe_f64.hip): the compiler schedules back-to-back
// exp_rbf calls as K serial 15-deep chains (124 cycles per exp), the interleaved form runs at
// the issue rate (94 cycles per exp with K = 8).  Same operations, same results as exp_rbf.
template <int K>
__device__ __forceinline__ void exp_rbf_n(double (&x)[K]) {
    constexpr double kMagic = 6755399441055744.0;   // 1.5 * 2^52
    constexpr double c[12] = {2.5110037605963777e-08, 2.763263963904103e-07, 2.755724091857897e-06,
                              2.4801485482328494e-05, 0.00019841269890047113, 0.0013888888952314775,
                              0.008333333333319601, 0.0416666666664881, 0.1666666666666668,
                              0.5000000000000019, 1.0, 1.0};
    double t[K], r[K], p[K];
#pragma unroll
    for (int k = 0; k < K; ++k) t[k] = fma(x[k], 1.4426950408889634, kMagic);
#pragma unroll
    for (int k = 0; k < K; ++k) r[k] = fma(t[k] - kMagic, -6.93147180369123816490e-01, x[k]);
#pragma unroll
    for (int k = 0; k < K; ++k) r[k] = fma(t[k] - kMagic, -1.90821492927058770002e-10, r[k]);
#pragma unroll
    for (int k = 0; k < K; ++k) p[k] = fma(c[0], r[k], c[1]);
#pragma unroll
    for (int i = 2; i < 12; ++i)
#pragma unroll
        for (int k = 0; k < K; ++k) p[k] = fma(p[k], r[k], c[i]);
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int ni = max(__double2loint(t[k]), -1022);
        x[k] = __hiloint2double(__double2hiint(p[k]) + (ni << 20), __double2loint(p[k]));
    }
}

// Up to kMaxGP posterior evaluations in one launch (grid.y = GP).
struct PostBatch {
    GPDev g[kMaxGP];
    PostArgs a[kMaxGP];
    int32_t npad[kMaxGP];
    int32_t n;
    // points of the whole step when this launch is one part of it (the overlapped halves): the
    // kernel choice follows the step, so both halves use the kernel a single launch would (0: P)
    int32_t step_points;
    // triangular variance kernel's column split (GPMPC_TUNE_VAR_SPLIT): 0 automatic, 1 or 4 forced
    int32_t var_split;
};

// Launchers (sqp_kernel.hip, gp_kernels.hip).
// count < 0: the whole batch; else ranks first .. first + count - 1 of order[] (launch_sqp_order)
hipError_t launch_sqp(const ProblemDev& P, const StateDev& S, const StepIO& io, int batch, hipStream_t stream,
                      int first = 0, int count = -1);
hipError_t launch_sqp_order(const StateDev& S, int batch, hipStream_t stream);
bool sqp_overlap_ok(const ProblemDev& P, int batch);
bool sqp_tail_ok(const ProblemDev& P, int batch);   // GPMPC_TUNE_TAIL applies (gpmpc_solve)
int sqp_tail_spare(const ProblemDev& P, int batch);  // its automatic K: SIMDs the one-wave launch leaves free
int sqp_launch_waves(const ProblemDev& P, int batch);   // waves per instance launch_sqp would use
int sqp_launch_segments(const ProblemDev& P, int batch);   // horizon segments of its Newton solves
size_t sqp_lds_bytes(int model, int H);
int model_unc_dims(int model, int32_t* unc);   // the model's uncertain state dims (Bd columns), returns their count
hipError_t launch_stage_cost(const ProblemDev& P, const double* x, const double* u, const int32_t* tstep,
                             const int32_t* status, double* cost, int B, hipStream_t stream);
hipError_t launch_gp_mean_grad(const GPDev& g, const double* Z, int P, double* mean, double* grad, hipStream_t stream);
hipError_t launch_gp_post(const GPDev& g, int npad, const PostArgs& a, bool from_state, hipStream_t stream);
hipError_t launch_gp_post_batch(const PostBatch& pb, bool from_state, hipStream_t stream);
hipError_t launch_plant(int model, const double* params, double dt, const double* x, const double* u, double* xn,
                        int32_t* tstep, int B, hipStream_t stream);

}  // namespace gpmpc
