/* C ABI of the MI355X-native GP-MPC solve path (gfx950).
 *
 * This is the drop-in boundary for the reference's hot path.  Each entry point names the
 * reference interface it replaces (file:line in amacati/gp-mpc).  All device pointers are
 * plain HIP device allocations (e.g. torch tensors' data_ptr()); host pointers are noted.
 * Calls are asynchronous on the given stream (NULL = default stream) unless noted.
 * No C++ exceptions cross this boundary; every call returns a gpmpc_status and
 * gpmpc_last_error() describes the last failure of the calling thread.
 *
 * Threading: one handle per GPU/process, driven by one host thread at a time
 * (the reference drives one acados solver from one Python thread, gpmpc/gpmpc.py:105-107).
 * Streams: every call queues its work on its stream argument.  The handle's device state is
 * shared by all of them, so each call that touches it ends by recording a handle-owned event on
 * its stream, and a call on a different stream first makes its stream wait for that event
 * (hipStreamWaitEvent: no host synchronisation, and the previous stream may already be gone).
 * The library reads no environment variables: every option is an explicit call.
 */
#ifndef GPMPC_MI355X_H
#define GPMPC_MI355X_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct gpmpc_handle gpmpc_handle;

typedef enum {
    GPMPC_OK = 0,
    GPMPC_ERR_ARG = -1,     /* invalid argument / shape */
    GPMPC_ERR_HIP = -2,     /* HIP runtime error (message in gpmpc_last_error) */
    GPMPC_ERR_STATE = -3,   /* call out of order (e.g. solve before set_model) */
    GPMPC_ERR_NOMEM = -4
} gpmpc_status;

/* Model ids (gpmpc/models.py MODEL_*). */
enum { GPMPC_MODEL_QUAD2D = 0, GPMPC_MODEL_QUAD3D = 1, GPMPC_MODEL_CARTPOLE = 2 };

/* Per-instance solver status codes, identical to acados (asserted in {0,2} at
 * gpmpc/gpmpc.py:365 and gpmpc/mpc.py:185).  An obs outside the stage-0 state box
 * (gpmpc/gpmpc.py:288,296,309-310; gpmpc/mpc.py:141,145,157-158) by more than the inequality
 * tolerance makes the QP infeasible: GPMPC_QP_FAILURE, as acados reports it.  After a failed
 * solve (NAN or QP_FAILURE) the instance keeps its previous iterate, its multipliers restart
 * from zero and its next solve runs untightened (no poisoning of later steps). */
enum { GPMPC_SUCCESS = 0, GPMPC_NAN = 1, GPMPC_MAXITER = 2, GPMPC_MINSTEP = 3, GPMPC_QP_FAILURE = 4 };

/* Create a solver for `max_batch` independent instances of model `model_id` with horizon
 * `horizon` on HIP device `device`.
 * Replaces: AcadosOcpSolver(ocp, json) construction at gpmpc/gpmpc.py:105-107 and
 * gpmpc/mpc.py:58 (code generation + compile there; nothing to compile here). */
gpmpc_status gpmpc_create(int32_t model_id, int32_t horizon, int32_t max_batch, int32_t device, gpmpc_handle** out);
void gpmpc_destroy(gpmpc_handle* h);
const char* gpmpc_last_error(void);

/* OCP definition (host arrays, float64).
 * Replaces: setup_acados_model / setup_acados_optimizer / setup_acados_constraints,
 * gpmpc/gpmpc.py:166-320 (and gpmpc/mpc.py:65-163).
 *   params      prior parameters in the model's order (gpmpc/models.py param_vector)
 *   x_lo..u_hi  box bounds (gpmpc/gpmpc.py:242-246)
 *   q_diag, r_diag  LINEAR_LS weights W = blkdiag(Q,R), W_e = Q (gpmpc/gpmpc.py:233-234)
 *   u_eq        input reference (ref_action, gpmpc/gpmpc.py:54)
 *   uh          upper bound of h = A[x;u] - b - t: -1e-8 GPMPC (gpmpc.py:309-314), +1e-8 MPC
 *   cost_scaling 1: stage costs scaled by dt, terminal by 1 (acados time-step scaling) */
gpmpc_status gpmpc_set_model(gpmpc_handle* h, const double* params, int32_t n_params, double dt,
                             const double* x_lo, const double* x_hi, const double* u_lo, const double* u_hi,
                             const double* q_diag, const double* r_diag, const double* u_eq, double uh,
                             int32_t cost_scaling);

/* Periodic reference trajectory (host, shape (nx, L) row-major like the reference's
 * traj array).  Replaces: GPMPC.reference_trajectory, gpmpc/gpmpc.py:509-514. */
gpmpc_status gpmpc_set_reference(gpmpc_handle* h, const double* traj_nx_by_L, int32_t L);

/* SQP / QP options.  Reference: nlp_solver_max_iter = 25 (gpmpc/gpmpc.py:262); acados
 * default NLP tolerances 1e-6.  The QP options belong to the batched IPM: qp_max_iter 50
 * (acados qp_solver_iter_max), qp_tol 1e-6 by default -- the OCP leaves the QP tolerances unset,
 * and acados' SQP then passes its NLP tolerances on to the QP solver. */
gpmpc_status gpmpc_set_options(gpmpc_handle* h, int32_t max_iter, double tol_stat, double tol_eq,
                               double tol_ineq, double tol_comp, int32_t qp_max_iter, double qp_tol, double qp_mu0);

/* Load GP `gp_id` (host arrays).
 *   Mean:      inputs X [n][d] (d <= 3) and weights alpha [n]: m(z) = sf2 sum_i alpha_i e(z, X_i).
 *              Exact GP: alpha = K^-1 y (gpytorch_predict2casadi, gpmpc/gp.py:72-85).
 *              FITC: X = inducing inputs, alpha = posterior weights (gpmpc/gpmpc.py:175-187,377-400).
 *   Variance:  training inputs Xv [nv][d] (NULL -> Xv = X, nv = n) and Linv = inverse Cholesky
 *              factor of K(Xv,Xv) + noise I [nv][nv] (row-major lower; NULL -> no variance).
 *              The reference takes the variance from the exact GP even in FITC mode
 *              (gpmpc/gpmpc.py:441-445).
 *   lengthscale (isotropic), outputscale, noise: ScaleKernel(RBFKernel()) + Gaussian likelihood. */
gpmpc_status gpmpc_set_gp(gpmpc_handle* h, int32_t gp_id, int32_t n, int32_t d, const double* X,
                          const double* alpha, int32_t nv, const double* Xv, const double* Linv,
                          double lengthscale, double outputscale, double noise);

/* LOVE variance for the constraint tightening (replaces GaussianProcess predictive variance
 * under gpytorch.settings.fast_pred_var, gpmpc/gpmpc.py:442-444): R [n][r] row-major with
 * R R^T ~ (K(Xv,Xv) + noise I)^-1 (a rank-r Lanczos root, gpmpc/gp.py love_root); the tightening
 * variance becomes outputscale - ||R^T k(z, Xv)||^2 + noise.  n must equal the GP's nv,
 * 1 <= r <= 256.  R = NULL restores the exact variance; gpmpc_set_gp clears the root.
 * gpmpc_gp_predict / gpmpc_gp_posterior stay exact. */
gpmpc_status gpmpc_set_gp_variance_root(gpmpc_handle* h, int32_t gp_id, int32_t n, int32_t r, const double* R);

/* Enable (1) / disable (0) the GP residual in the dynamics: 0 = nominal MPC
 * (gpmpc/mpc.py, prior dynamics only). */
gpmpc_status gpmpc_use_gp(gpmpc_handle* h, int32_t enabled);

/* Constraint tightening (gpmpc/gpmpc.py:425-498): inverse_cdf (gpmpc.py:63-65) and the
 * prior LQR closed loop: Ad [nx][nx], Bd [nx][nu], K [nu][nx] (gpmpc.py:500-507).
 * enabled = 0 disables tightening (nominal MPC).  Builds the H-term gain table of the covariance
 * recursion on the host and copies it to the device (synchronous; a setup call). */
gpmpc_status gpmpc_set_tightening(gpmpc_handle* h, int32_t enabled, double inverse_cdf, const double* Ad,
                                  const double* Bd, const double* K);

/* Input map of GP gp_id's tightening variance: indices src[0..d) into z = [x; u] (d = the
 * GP's input dimension).  The default is the reference's map, which evaluates GP g at
 * z[:, gp_idx[g]] with gp_idx indexing the GP-input space (gpmpc/gpmpc.py:59 vs 437-444,
 * reproduced for quad3d); passing the GP's own dynamics inputs (gpmpc/gpmpc.py:173)
 * evaluates the variance where the mean is evaluated. */
gpmpc_status gpmpc_set_var_inputs(gpmpc_handle* h, int32_t gp_id, const int32_t* src, int32_t d);

/* Forget the previous solution for instances [0, batch): the next solve runs without
 * tightening (GPMPC.reset, gpmpc/gpmpc.py:109-111).  reset_iterate = 1 also zeroes the
 * warm-start iterate and multipliers (acados_solver.reset(), gpmpc/mpc.py:62; and the fresh
 * AcadosOcpSolver GPMPC.reset builds after new GPs, gpmpc/gpmpc.py:97-108). */
gpmpc_status gpmpc_reset(gpmpc_handle* h, int32_t batch, int32_t reset_iterate, void* stream);

/* Set the warm-start iterate (device arrays x [B][H+1][nx], u [B][H][nu]); multipliers zeroed. */
gpmpc_status gpmpc_set_iterate(gpmpc_handle* h, int32_t batch, const double* x_dev, const double* u_dev, void* stream);

/* One batched control step: GPMPC.select_action(obs) for every instance
 * (gpmpc/gpmpc.py:334-368): tightening from the stored previous solution, SQP to
 * convergence warm-started from it, store the new solution.
 *   x0      [B][nx]  initial states (obs)                                   (device)
 *   tstep   [B]      reference index per instance (traj_step)               (device)
 *   u0      [B][nu]  first input (return value of select_action)            (device, out)
 *   status  [B]      acados status code                                     (device, out)
 *   sqp_iter, qp_iter [B]  SQP iterations / total IPM iterations            (device, out, may be NULL)
 *   res     [B][4]   final NLP residuals stat, eq, ineq, comp               (device, out, may be NULL)
 * When the SQP launch needs more than one round of workgroups (more instances than the device
 * holds at once) and the step has a variance launch, half of the step's work runs on a handle-owned
 * side stream forked from and joined back into `stream` (results bit-identical;
 * gpmpc_set_tuning(GPMPC_TUNE_OVERLAP, 0) turns it off): work queued on `stream` after the call
 * still sees the whole step complete. */
gpmpc_status gpmpc_solve(gpmpc_handle* h, int32_t batch, const double* x0, const int32_t* tstep, double* u0,
                         int32_t* status, int32_t* sqp_iter, int32_t* qp_iter, double* res, void* stream);

/* Copy the current solution (x_prev / u_prev, gpmpc/gpmpc.py:366-367) into device arrays
 * x [B][H+1][nx], u [B][H][nu]; tight [B][H+1][nx+nu] receives the last tightening
 * magnitudes (icdf*sqrt(var)) if non-NULL. */
gpmpc_status gpmpc_get_solution(gpmpc_handle* h, int32_t batch, double* x_dev, double* u_dev, double* tight_dev,
                                void* stream);

/* Copy the GP variances the last tightening used (the variance kernel's output at the previous
 * solution, likelihood noise included, gpmpc/gpmpc.py:437-445) into var [B][H][n_gp] (device).
 * Diagnostic / parity surface: the values the constraint tightening consumed.  GPMPC_ERR_STATE
 * when the last gpmpc_solve ran no variance launch (first step after a reset, tightening or GPs
 * off): there are no such values; GPMPC_ERR_ARG when batch exceeds that launch's batch. */
gpmpc_status gpmpc_get_variance(gpmpc_handle* h, int32_t batch, double* var_dev, void* stream);

/* GP posterior at P points Z [P][d] (device): mean [P] and/or variance [P] (either may be
 * NULL; variance needs Linv).  with_noise = 1 adds the likelihood noise
 * (gp.likelihood(gp(z)), gpmpc/gpmpc.py:444).  GaussianProcess.predict() of the build. */
gpmpc_status gpmpc_gp_predict(gpmpc_handle* h, int32_t gp_id, const double* Z, int32_t P, double* mean,
                              double* var, int32_t with_noise, void* stream);

/* GP mean and its input gradient at P points Z [P][d] (device): mean [P], grad [P][d] (either
 * may be NULL), through the MFMA tile sums the SQP linearisation uses (sqp_kernel.hip
 * gp_tiles).  Replaces the casadi mean export gpytorch_predict2casadi (gpmpc/gp.py:72-85) and
 * the CasADi AD of it inside setup_acados_model (gpmpc/gpmpc.py:189-209). */
gpmpc_status gpmpc_gp_mean_grad(gpmpc_handle* h, int32_t gp_id, const double* Z, int32_t P, double* mean,
                                double* grad, void* stream);

/* Handle-free GP posterior (GaussianProcess.predict() of the build): GP data already on the
 * device in the kernel layout -- rows [npad][4] = (x0, x1, x2 zero padded, alpha) and
 * linvT [npad][npad] = (L^-1)^T zero padded (NULL -> mean only), npad = n rounded up to 16.
 * Replaces the gpytorch posterior of gpmpc/gpmpc.py:441-445 and the casadi mean export
 * gpmpc/gp.py:72-85. */
gpmpc_status gpmpc_gp_posterior(int32_t n, int32_t d, int32_t npad, const double* rows, const double* linvT,
                                double lengthscale, double outputscale, double noise, const double* Z, int32_t P,
                                double* mean, double* var, int32_t with_noise, void* stream);

/* Synthetic plant: x_next = RK4(prior-form dynamics with `params`, no GP) for B instances,
 * tstep += 1 if tstep != NULL (crazyflow env.step replacement, scripts/run_gp_mpc.py:59). */
gpmpc_status gpmpc_plant_step(gpmpc_handle* h, int32_t batch, const double* params, const double* x,
                              const double* u, double* x_next, int32_t* tstep, void* stream);

/* Launch shape of the SQP kernel (no reference counterpart: the reference solves one instance).
 *   waves     0 = auto: one wavefront per instance, or -- for the models whose stage fits one MFMA
 *             tile (quad2d, cartpole) -- four per instance when batch <= the device's compute units
 *             and two when batch <= twice that, so the SIMDs that would idle take the GP tile sums;
 *             1 / 2 / 4 force a count for quad2d / cartpole.  quad3d always runs four: it accepts
 *             0 or 4 and rejects any other count (GPMPC_ERR_ARG), so a setting never silently
 *             does nothing.
 * Results are identical up to floating-point rounding; a performance option. */
gpmpc_status gpmpc_set_launch(gpmpc_handle* h, int32_t waves);

/* What gpmpc_solve would run for `batch` instances with the current options (host, no device
 * work): waves per instance of the SQP launch, and overlapped = 1 when a step with a variance
 * launch runs as two overlapped halves (see gpmpc_solve).  With overlapped = 1 the profiling
 * events of gpmpc_kernel_times bracket the costlier half's variance launch ("variance") and the
 * span from its end to the join of both halves' SQP launches ("SQP", which also contains the
 * cheaper half's variance launch): spans of the step, not per-kernel durations.  overlapped = 2:
 * the tail boost of GPMPC_TUNE_TAIL applies (two SQP launches side by side, the "SQP" events
 * bracketing both; `waves` is then the other instances' one). */
gpmpc_status gpmpc_get_launch_info(gpmpc_handle* h, int32_t batch, int32_t* waves, int32_t* overlapped);

/* Horizon segments of the Newton solves gpmpc_solve would run for `batch` instances (host, no
 * device work): 1 = one wave runs each recursion over the whole horizon; 2 or 3 = the
 * segment-parallel solve of GPMPC_TUNE_SEG (two segments on two waves per instance, three on four). */
gpmpc_status gpmpc_get_launch_segments(gpmpc_handle* h, int32_t batch, int32_t* segments);

/* Performance switches (no reference counterpart; every output is bit-identical or identical up
 * to rounding whichever value is set -- A/B measurement knobs, all on their default after
 * gpmpc_create).  gpmpc_set_tuning(h, option, value):
 *   GPMPC_TUNE_LIN_CACHE   1 (default): the first SQP iteration of a step reads the stored
 *                          iterate's linearisation; 0: recompute it (bit-identical)
 *   GPMPC_TUNE_ORDER       1 (default): a launch needing more than one round of workgroups runs
 *                          its instances by decreasing previous cost; 0: instance order; 2: rank
 *                          every launch (bit-identical)
 *   GPMPC_TUNE_OVERLAP     1 (default): overlapped halves for multi-round steps; 0: sequential
 *   GPMPC_TUNE_VAR_SPLIT   0 (default): automatic; 1: one wave per 16-point tile of the
 *                          triangular variance kernel; 4: its four-wave column split
 *   GPMPC_TUNE_EVENT_FENCE 0 (default): profiling events without the system-scope fence;
 *                          1: default (fenced) events
 *   GPMPC_TUNE_SEG         1 (default): segment-parallel Newton solves when a launch runs two or
 *                          four waves per instance (quad2d, cartpole): the horizon's two (two
 *                          waves) or three (four waves) segments are factorised and swept on
 *                          different waves at once and joined by a chain over the boundaries;
 *                          0: one wave runs the whole recursion; identical up to rounding
 *   GPMPC_TUNE_TAIL        -1 (default): automatic, K = the SIMDs the launch leaves free (4 x CUs - B,
 *                          so 0 at B = 4 x CUs); 0: off; K > 0: fixed.  A step whose SQP launch gives
 *                          every instance one wave in one round of workgroups (quad2d, cartpole; batch
 *                          between 2 and 4 x CUs, waves automatic, segments on) runs its K costliest
 *                          instances (by the cost of their previous solve) as two-wave segment solves
 *                          on the caller's stream, beside the other instances' one-wave launch on a
 *                          second stream; identical up to rounding (each instance's arithmetic is that of
 *                          its launch shape).  The SQP profiling events then bracket both launches
 *   GPMPC_TUNE_SEG_PIVOT   10 (default): the segment solve's boundary chain refuses a pivot below
 *                          10^-value x Ph's largest diagonal entry and redoes that Newton solve as
 *                          the one-segment recursion; -1: refuses every pivot (every segment solve
 *                          takes that fallback: a test of it) */
enum {
    GPMPC_TUNE_LIN_CACHE = 0,
    GPMPC_TUNE_ORDER = 1,
    GPMPC_TUNE_OVERLAP = 2,
    GPMPC_TUNE_VAR_SPLIT = 3,
    GPMPC_TUNE_EVENT_FENCE = 4,
    GPMPC_TUNE_SEG = 5,
    GPMPC_TUNE_TAIL = 6,
    GPMPC_TUNE_SEG_PIVOT = 7
};
gpmpc_status gpmpc_set_tuning(gpmpc_handle* h, int32_t option, int32_t value);

/* Optional device buffer [max_batch][H+1] (float64) receiving, on every gpmpc_solve, the stage
 * costs of each instance's new solution: the acados LINEAR_LS cost 1/2 ||y_k - y_ref,k||^2_W with
 * W = blkdiag(Q, R) scaled by dt on stages 0..H-1 and W_e = Q unscaled on stage H
 * (gpmpc/gpmpc.py:231-239, gpmpc/mpc.py:101-102, acados cost_scaling), y_k = [x_k; u_k],
 * y_ref,k = [reference window; u_eq].  Their sum is the objective value acados reports ("cost").
 * A solve that ends with any status other than 0 or 2 (a failed solve: its x, u hold the previous
 * solution) writes NaN.  NULL disables (default). */
gpmpc_status gpmpc_set_cost_buffer(gpmpc_handle* h, void* cost_dev);

/* Kernel timing with HIP events recorded on the solve stream around the variance kernel
 * and the SQP kernel of every gpmpc_solve while enabled.  gpmpc_kernel_times synchronises
 * on the recorded events, returns the summed milliseconds and launch counts, and clears them.
 * gpmpc_kernel_time_list returns the per-launch milliseconds instead (host arrays of capacity
 * `cap`; n_var / n_sqp receive the counts, at most cap are written) and clears them.
 * Replaces the perf_counter around select_action, scripts/run_gp_mpc.py:55-57. */
gpmpc_status gpmpc_set_profiling(gpmpc_handle* h, int32_t enabled);
gpmpc_status gpmpc_kernel_times(gpmpc_handle* h, double* var_ms, int32_t* n_var, double* sqp_ms, int32_t* n_sqp);
gpmpc_status gpmpc_kernel_time_list(gpmpc_handle* h, int32_t cap, double* var_ms, int32_t* n_var, double* sqp_ms,
                                    int32_t* n_sqp);

/* Diagnostic builds (-DGPMPC_TIMING) only: device buffer [max_batch][12] (uint64) receiving
 * per-phase shader-clock cycles of each instance's last solve; NULL disables. */
gpmpc_status gpmpc_set_timing_buffer(gpmpc_handle* h, void* timing_dev);

/* Optional device buffer [max_batch][GPMPC_STATS_SLOTS] (int64) of running solver statistics,
 * accumulated by the SQP kernel on every gpmpc_solve: [0] SQP iterations, [1] QP (IPM) iterations, [2 + s] number
 * of solves that ended with status s (0..4), [7] largest SQP iteration count of one solve,
 * [8] largest QP iteration total of one solve, [9] linearisations computed (the first SQP
 * iteration of a step reads the stored iterate's linearisation when it is valid), [10] the
 * instance's solve time inside the SQP kernel in s_memrealtime ticks (the 100 MHz constant clock:
 * 10 ns; from the instance's first to its last instruction, summed over solves), [11] the last
 * solve's time in ticks (the slot holds the start stamp while the solve runs).  The slowest instance's time against the kernel's duration is the
 * latency-bound figure of bench.py's roofline block.  The caller
 * zeroes it; NULL disables (default).  `slots` is the caller's row stride in int64: it must
 * equal GPMPC_STATS_SLOTS (a buffer laid out for another slot count is rejected, not
 * overrun).
 * Replaces reading acados' per-solve "sqp_iter" / "qp_iter" / status stats in a host loop. */
enum { GPMPC_STATS_SLOTS = 12 };
gpmpc_status gpmpc_set_stats_buffer(gpmpc_handle* h, void* stats_dev, int32_t slots);

/* LDS bytes one instance's workgroup needs (capacity planning / tests). */
int64_t gpmpc_lds_bytes(int32_t model_id, int32_t horizon);

/* Build provenance (host, static string): "src=<sha256 of the library's sources, 16 hex digits>
 * git=<commit at build time>[+dirty] kind=<product|timing>".  The Python binding recomputes the
 * source hash from the tree and refuses an in-tree library built from other sources. */
const char* gpmpc_build_id(void);

#ifdef __cplusplus
}
#endif
#endif
