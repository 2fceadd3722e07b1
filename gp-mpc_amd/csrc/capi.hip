// C ABI (include/gpmpc_mi355x.h): handle management, GP upload, batched control step.
#include "../../include/gpmpc_mi355x.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "gpmpc_common.h"

using namespace gpmpc;

static_assert(GPMPC_STATS_SLOTS == kStatsSlots, "public stats-slot count must match the kernel's");

namespace {
thread_local std::string g_err;

gpmpc_status fail(gpmpc_status s, const std::string& msg) {
    g_err = msg;
    return s;
}

#define HIPCHK(expr)                                                                        \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess)                                                               \
            return fail(GPMPC_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));   \
    } while (0)

struct ModelDims {
    int nx, nu, ngp, nparams;
    int gp_dim[kMaxGP];
    int var_src[kMaxGP][3];
};

bool model_dims(int id, ModelDims& m) {
    switch (id) {
        case kQuad2D:
            m = ModelDims{6, 2, 2, 6, {1, 3, 0, 0}, {{6, 0, 0}, {4, 5, 7}, {0, 0, 0}, {0, 0, 0}}};
            return true;
        case kQuad3D:
            m = ModelDims{12, 4, 3, 9, {1, 3, 3, 0}, {{0, 0, 0}, {1, 2, 3}, {4, 5, 6}, {0, 0, 0}}};
            return true;
        case kCartpole:
            m = ModelDims{4, 1, 2, 4, {3, 3, 0, 0}, {{2, 3, 4}, {2, 3, 4}, {0, 0, 0}, {0, 0, 0}}};
            return true;
    }
    return false;
}
}  // namespace

struct gpmpc_handle {
    int device = 0;
    int model = 0;
    int H = 0;
    int max_batch = 0;
    ModelDims md{};
    int nb = 0;
    bool model_set = false, ref_set = false;
    bool gp_set[kMaxGP] = {false, false, false, false};
    bool any_prev = false;
    ProblemDev P{};
    // device state
    double *x = nullptr, *u = nullptr, *pi = nullptr, *lam = nullptr, *var = nullptr, *tight = nullptr;
    int32_t* has_prev = nullptr;
    double* lin = nullptr;          // linearisation cache of the stored iterate (StateDev::lin)
    int32_t* lin_tag = nullptr;
    bool lin_cache = true;          // GPMPC_TUNE_LIN_CACHE
    int32_t* order = nullptr;       // cost-ordered dispatch (StateDev::order / cost)
    uint32_t* cost = nullptr;
    double* traj = nullptr;
    double* plant_params = nullptr;
    double* tgain = nullptr;        // [H][nb][n_unc] tightening gain table (ProblemDev::tgain)
    double plant_params_host[kMaxParams] = {0};
    bool plant_params_valid = false;
    double* gp_rows[kMaxGP] = {nullptr, nullptr, nullptr, nullptr};
    double* gp_vrows[kMaxGP] = {nullptr, nullptr, nullptr, nullptr};
    double* gp_linvT[kMaxGP] = {nullptr, nullptr, nullptr, nullptr};
    double* gp_tiles[kMaxGP] = {nullptr, nullptr, nullptr, nullptr};   // tX | tW (MFMA tile pack)
    int gp_npad[kMaxGP] = {0, 0, 0, 0};
    double* gp_vroot[kMaxGP] = {nullptr, nullptr, nullptr, nullptr};   // LOVE roots (tightening only)
    int gp_vroot_cols[kMaxGP] = {0, 0, 0, 0};
    int gp_vroot_rank[kMaxGP] = {0, 0, 0, 0};
    // optional per-kernel HIP-event timing (bench.py's roofline leg)
    bool profiling = false;
    std::vector<hipEvent_t> ev_pool;
    // whether each profiling event was created fenced (GPMPC_TUNE_EVENT_FENCE at its creation): events
    // still in ev_var / ev_sqp when the option changes return to the pool later and are dropped there
    std::unordered_map<hipEvent_t, bool> ev_fenced;
    // (start, end) per launch; a variance launch's end event is also the following SQP launch's
    // start (one event between the two kernels), so the SQP list owns it
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_var, ev_sqp;
    // end events of ev_var pairs that no SQP pair took over (the SQP launch failed or got no
    // end event): the variance list returns these to the pool itself
    std::vector<hipEvent_t> ev_var_owned;
    unsigned long long* timing = nullptr;  // diagnostic phase cycles (GPMPC_TIMING builds)
    long long* stats = nullptr;            // optional per-instance solver statistics accumulators
    int32_t* scratch_i = nullptr;   // [2][max_batch]
    double* scratch_d = nullptr;    // [max_batch][4]
    // the batch whose tightening variances the last solve's variance launch wrote into `var`
    // (0: the last solve ran none, var is stale or unset)
    int var_batch = 0;
    // stream of the last call that queued work on the handle's device state and an event recorded
    // on it when that call returned: a call on another stream first waits for the event
    // (order_after_last / StreamMark), so consecutive calls never overlap
    hipStream_t last_stream = nullptr;
    hipEvent_t ev_last = nullptr;
    bool ev_last_valid = false;
    // overlapped steps (gpmpc_solve): the second half's variance and SQP launches run on `side`,
    // forked from and joined back into the caller's stream by two events
    bool overlap = true;            // GPMPC_TUNE_OVERLAP
    int var_split = 0;              // GPMPC_TUNE_VAR_SPLIT
    bool event_fence = false;       // GPMPC_TUNE_EVENT_FENCE
    double* stage_cost = nullptr;   // caller's [max_batch][H+1] stage-cost buffer (StepIO::stage_cost)
    hipStream_t side = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    // tail boost (GPMPC_TUNE_TAIL): the costliest `tail` instances of a one-wave, one-round step run
    // as two-wave segment solves on the caller's stream, the others' one-wave launch on `side`
    // (-1: as many as the launch leaves SIMDs free, sqp_tail_spare)
    int tail = -1;
};

// The handle's device state (iterate, multipliers, variances, dispatch order) is read and written
// by every queued call, so calls on different streams must not overlap.  Each such call ends by
// recording the handle's event on its stream (StreamMark); a call on another stream first makes
// its stream wait for that event.  No host synchronisation, and a destroyed previous stream leaves
// nothing dangling (the event outlives it).
static hipError_t order_after_last(gpmpc_handle* h, hipStream_t s) {
    if (!h->ev_last) {
        const hipError_t e = hipEventCreateWithFlags(&h->ev_last, hipEventDisableTiming);
        if (e != hipSuccess) {
            h->ev_last = nullptr;
            return e;
        }
    }
    if (h->ev_last_valid && h->last_stream != s) return hipStreamWaitEvent(s, h->ev_last, 0);
    return hipSuccess;
}
// Records the handle's event on the call's stream when the call returns, whatever it queued.  If
// the record fails the stream is drained on the host instead, so the next call needs no wait.
struct StreamMark {
    gpmpc_handle* h;
    hipStream_t s;
    ~StreamMark() {
        if (h->ev_last && hipEventRecord(h->ev_last, s) == hipSuccess) {
            h->ev_last_valid = true;
        } else {
            (void)hipStreamSynchronize(s);
            h->ev_last_valid = false;
        }
        h->last_stream = s;
    }
};

// The second stream of overlapped and tail-boosted steps and its fork / join events (lowest
// priority), created together on first use or not at all.
static hipError_t ensure_side(gpmpc_handle* h) {
    if (h->side) return hipSuccess;
    int lo = 0, hi = 0;
    if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) lo = hi = 0;
    hipStream_t side = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;
    hipError_t ce = hipStreamCreateWithPriority(&side, hipStreamNonBlocking, lo);   // lowest priority
    if (ce == hipSuccess) ce = hipEventCreateWithFlags(&fork, hipEventDisableTiming);
    if (ce == hipSuccess) ce = hipEventCreateWithFlags(&join, hipEventDisableTiming);
    if (ce != hipSuccess) {
        if (join) (void)hipEventDestroy(join);
        if (fork) (void)hipEventDestroy(fork);
        if (side) (void)hipStreamDestroy(side);
        return ce;
    }
    h->side = side;
    h->ev_fork = fork;
    h->ev_join = join;
    return hipSuccess;
}

// Instances the tail boost runs on two waves for this step (0: none, the ordinary launch)
static int tail_count(const gpmpc_handle* h, const ProblemDev& P, int batch) {
    if (h->tail == 0 || !sqp_tail_ok(P, batch)) return 0;
    return h->tail < 0 ? sqp_tail_spare(P, batch) : std::min(h->tail, batch - 1);
}

static hipEvent_t take_event(gpmpc_handle* h) {
    while (!h->ev_pool.empty()) {
        hipEvent_t e = h->ev_pool.back();
        h->ev_pool.pop_back();
        const auto it = h->ev_fenced.find(e);
        if (it != h->ev_fenced.end() && it->second == h->event_fence) return e;
        // created under the other GPMPC_TUNE_EVENT_FENCE setting: an A/B run must not mix them
        if (it != h->ev_fenced.end()) h->ev_fenced.erase(it);
        (void)hipEventDestroy(e);
    }
    hipEvent_t e = nullptr;
    // timing-only events: no system-scope fence (cache writeback / invalidate) when recorded,
    // which otherwise adds ~5 us of dispatch gap around every kernel it brackets
    const unsigned flags = h->event_fence ? hipEventDefault : hipEventDisableSystemFence;
    if (hipEventCreateWithFlags(&e, flags) != hipSuccess) return nullptr;
    h->ev_fenced[e] = h->event_fence;
    return e;
}

// Invalidate every instance's linearisation cache (StateDev::lin): the iterate, the GPs or the
// model changed.  Tags written by earlier launches no longer match the new generation.
static void bump_lin(gpmpc_handle* h) {
    if (++h->P.lin_gen <= 0) h->P.lin_gen = 1;
}

static void free_handle(gpmpc_handle* h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    for (auto& pr : h->ev_var) h->ev_pool.push_back(pr.first);
    for (hipEvent_t e : h->ev_var_owned) h->ev_pool.push_back(e);
    for (auto& pr : h->ev_sqp) { h->ev_pool.push_back(pr.first); h->ev_pool.push_back(pr.second); }
    for (hipEvent_t e : h->ev_pool) (void)hipEventDestroy(e);
    if (h->ev_fork) (void)hipEventDestroy(h->ev_fork);
    if (h->ev_join) (void)hipEventDestroy(h->ev_join);
    if (h->ev_last) (void)hipEventDestroy(h->ev_last);
    if (h->side) (void)hipStreamDestroy(h->side);
    for (double* p : {h->x, h->u, h->pi, h->lam, h->var, h->tight, h->traj, h->plant_params, h->tgain, h->lin})
        if (p) (void)hipFree(p);
    if (h->has_prev) (void)hipFree(h->has_prev);
    if (h->lin_tag) (void)hipFree(h->lin_tag);
    if (h->order) (void)hipFree(h->order);
    if (h->cost) (void)hipFree(h->cost);
    if (h->scratch_i) (void)hipFree(h->scratch_i);
    if (h->scratch_d) (void)hipFree(h->scratch_d);
    for (int g = 0; g < kMaxGP; ++g) {
        if (h->gp_rows[g]) (void)hipFree(h->gp_rows[g]);
        if (h->gp_vrows[g]) (void)hipFree(h->gp_vrows[g]);
        if (h->gp_linvT[g]) (void)hipFree(h->gp_linvT[g]);
        if (h->gp_tiles[g]) (void)hipFree(h->gp_tiles[g]);
        if (h->gp_vroot[g]) (void)hipFree(h->gp_vroot[g]);
    }
    delete h;
}

extern "C" {

const char* gpmpc_last_error(void) { return g_err.c_str(); }

int64_t gpmpc_lds_bytes(int32_t model_id, int32_t horizon) {
    return (int64_t)sqp_lds_bytes(model_id, horizon);
}

gpmpc_status gpmpc_create(int32_t model_id, int32_t horizon, int32_t max_batch, int32_t device, gpmpc_handle** out) {
    if (!out) return fail(GPMPC_ERR_ARG, "out is NULL");
    *out = nullptr;
    ModelDims md;
    if (!model_dims(model_id, md)) return fail(GPMPC_ERR_ARG, "unknown model id " + std::to_string(model_id));
    if (horizon < 1 || horizon > kMaxH) return fail(GPMPC_ERR_ARG, "horizon must be in [1, 63]");
    if (max_batch < 1) return fail(GPMPC_ERR_ARG, "max_batch must be >= 1");
    auto* h = new gpmpc_handle();
    h->device = device;
    h->model = model_id;
    h->H = horizon;
    h->max_batch = max_batch;
    h->md = md;
    h->nb = md.nx + md.nu;
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) {
        delete h;
        return fail(GPMPC_ERR_HIP, std::string("hipSetDevice: ") + hipGetErrorString(e));
    }
    const size_t B = max_batch, H = horizon;
    struct A { void** p; size_t bytes; } allocs[] = {
        {(void**)&h->x, B * (H + 1) * md.nx * sizeof(double)},
        {(void**)&h->u, B * H * md.nu * sizeof(double)},
        {(void**)&h->pi, B * H * md.nx * sizeof(double)},
        {(void**)&h->lam, B * (H + 1) * 2 * h->nb * sizeof(double)},
        {(void**)&h->var, B * H * md.ngp * sizeof(double)},
        {(void**)&h->tight, B * (H + 1) * h->nb * sizeof(double)},
        {(void**)&h->has_prev, B * sizeof(int32_t)},
        {(void**)&h->lin, B * H * md.nx * (h->nb + 1) * sizeof(double)},
        {(void**)&h->lin_tag, B * sizeof(int32_t)},
        {(void**)&h->order, B * sizeof(int32_t)},
        {(void**)&h->cost, B * sizeof(uint32_t)},
        {(void**)&h->plant_params, kMaxParams * sizeof(double)},
        {(void**)&h->scratch_i, 2 * B * sizeof(int32_t)},
        {(void**)&h->scratch_d, 4 * B * sizeof(double)},
    };
    for (auto& a : allocs) {
        e = hipMalloc(a.p, a.bytes);
        if (e == hipSuccess) e = hipMemset(*a.p, 0, a.bytes);
        if (e != hipSuccess) {
            free_handle(h);
            return fail(GPMPC_ERR_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
        }
    }
    ProblemDev& P = h->P;
    P.model = model_id;
    P.nx = md.nx;
    P.nu = md.nu;
    P.H = horizon;
    P.n_gp = md.ngp;
    P.use_gp = 0;
    P.cost_scale = 1.0;
    P.uh = -1e-8;
    P.tighten = 0;
    P.max_iter = 25;          // gpmpc.py:262
    P.tol_stat = P.tol_eq = P.tol_ineq = P.tol_comp = 1e-6;  // acados defaults
    P.qp_max_iter = 50;   // acados qp_solver_iter_max default
    // QP tolerances = the NLP tolerances: gpmpc.py:257-263 leaves qp_solver_tol_* unset, and acados'
    // SQP passes each NLP tolerance it is given (tol_stat/eq/ineq/comp, 1e-6 by default) on to the QP
    // solver as that solver's tolerance (ocp_nlp_sqp_opts_set -> qp_solver opts_set "tol_stat", ...)
    P.qp_tol = 1e-6;
    P.qp_mu0 = 1.0;
    P.lin_gen = 1;   // tags start at 0: nothing cached
    P.waves = 0;            // automatic launch shape (gpmpc_set_launch)
    P.order_dispatch = 1;   // cost-ordered dispatch of multi-round launches (GPMPC_TUNE_ORDER)
    P.seg = 1;              // segment-parallel Newton solves (GPMPC_TUNE_SEG)
    P.seg_piv_rel = 1e-10;  // their boundary chain's pivot threshold (GPMPC_TUNE_SEG_PIVOT)
    {
        int ncu = 0;
        if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) ncu = 0;
        P.n_cu = ncu;
    }
    const size_t lds = sqp_lds_bytes(model_id, horizon);
    if (lds > 160 * 1024) {
        free_handle(h);
        return fail(GPMPC_ERR_ARG, "horizon too long for the LDS budget (" + std::to_string(lds) + " bytes)");
    }
    *out = h;
    return GPMPC_OK;
}

void gpmpc_destroy(gpmpc_handle* h) { free_handle(h); }

gpmpc_status gpmpc_set_model(gpmpc_handle* h, const double* params, int32_t n_params, double dt, const double* x_lo,
                             const double* x_hi, const double* u_lo, const double* u_hi, const double* q_diag,
                             const double* r_diag, const double* u_eq, double uh, int32_t cost_scaling) {
    if (!h) return fail(GPMPC_ERR_ARG, "null handle");
    if (!params || !x_lo || !x_hi || !u_lo || !u_hi || !q_diag || !r_diag || !u_eq)
        return fail(GPMPC_ERR_ARG, "null array");
    if (n_params != h->md.nparams)
        return fail(GPMPC_ERR_ARG, "model expects " + std::to_string(h->md.nparams) + " parameters");
    if (!(dt > 0.0)) return fail(GPMPC_ERR_ARG, "dt must be > 0");
    ProblemDev& P = h->P;
    std::memset(P.params, 0, sizeof(P.params));
    for (int i = 0; i < n_params; ++i) P.params[i] = params[i];
    P.dt = dt;
    for (int i = 0; i < h->md.nx; ++i) {
        P.x_lo[i] = x_lo[i];
        P.x_hi[i] = x_hi[i];
        P.q[i] = q_diag[i];
        if (!(q_diag[i] >= 0.0)) return fail(GPMPC_ERR_ARG, "q_diag must be >= 0");
    }
    for (int a = 0; a < h->md.nu; ++a) {
        P.u_lo[a] = u_lo[a];
        P.u_hi[a] = u_hi[a];
        P.r[a] = r_diag[a];
        P.u_eq[a] = u_eq[a];
        if (!(r_diag[a] > 0.0)) return fail(GPMPC_ERR_ARG, "r_diag must be > 0 (GN Hessian)");
    }
    P.uh = uh;
    P.cost_scale = cost_scaling ? dt : 1.0;
    bump_lin(h);
    h->model_set = true;
    return GPMPC_OK;
}

gpmpc_status gpmpc_set_reference(gpmpc_handle* h, const double* traj, int32_t L) {
    if (!h || !traj || L < 1) return fail(GPMPC_ERR_ARG, "bad reference");
    (void)hipSetDevice(h->device);
    const int nx = h->md.nx;
    std::vector<double> tm((size_t)L * nx);
    for (int t = 0; t < L; ++t)
        for (int i = 0; i < nx; ++i) tm[(size_t)t * nx + i] = traj[(size_t)i * L + t];
    if (h->traj) HIPCHK(hipFree(h->traj));
    h->traj = nullptr;
    HIPCHK(hipMalloc(&h->traj, tm.size() * sizeof(double)));
    HIPCHK(hipMemcpy(h->traj, tm.data(), tm.size() * sizeof(double), hipMemcpyHostToDevice));
    h->P.traj = h->traj;
    h->P.traj_len = L;
    h->ref_set = true;
    return GPMPC_OK;
}

gpmpc_status gpmpc_set_options(gpmpc_handle* h, int32_t max_iter, double tol_stat, double tol_eq, double tol_ineq,
                               double tol_comp, int32_t qp_max_iter, double qp_tol, double qp_mu0) {
    if (!h) return fail(GPMPC_ERR_ARG, "null handle");
    if (max_iter < 0 || qp_max_iter < 1 || !(qp_mu0 > 0.0)) return fail(GPMPC_ERR_ARG, "bad options");
    ProblemDev& P = h->P;
    P.max_iter = max_iter;
    P.tol_stat = tol_stat;
    P.tol_eq = tol_eq;
    P.tol_ineq = tol_ineq;
    P.tol_comp = tol_comp;
    P.qp_max_iter = qp_max_iter;
    P.qp_tol = qp_tol;
    P.qp_mu0 = qp_mu0;
    return GPMPC_OK;
}

gpmpc_status gpmpc_set_gp(gpmpc_handle* h, int32_t gp_id, int32_t n, int32_t d, const double* X, const double* alpha,
                          int32_t nv, const double* Xv, const double* Linv, double lengthscale, double outputscale,
                          double noise) {
    if (!h) return fail(GPMPC_ERR_ARG, "null handle");
    if (gp_id < 0 || gp_id >= h->md.ngp) return fail(GPMPC_ERR_ARG, "gp_id out of range");
    if (d != h->md.gp_dim[gp_id])
        return fail(GPMPC_ERR_ARG, "GP " + std::to_string(gp_id) + " expects input dimension " +
                                       std::to_string(h->md.gp_dim[gp_id]));
    if (n < 1 || !X || !alpha) return fail(GPMPC_ERR_ARG, "empty GP");
    if (!(lengthscale > 0.0) || !(outputscale > 0.0) || !(noise >= 0.0)) return fail(GPMPC_ERR_ARG, "bad hyperparameters");
    if (!Xv) { Xv = X; nv = n; }
    if (nv < 1) return fail(GPMPC_ERR_ARG, "empty variance GP");
    (void)hipSetDevice(h->device);
    auto pack = [&](const double* Xs, const double* w, int m, std::vector<double>& out) {
        const int mp = (m + 15) / 16 * 16;
        out.assign((size_t)mp * 4, 0.0);
        for (int i = 0; i < m; ++i) {
            for (int k = 0; k < d; ++k) out[(size_t)i * 4 + k] = Xs[(size_t)i * d + k];
            out[(size_t)i * 4 + 3] = w ? w[i] : 0.0;
        }
    };
    std::vector<double> rows, vrows;
    pack(X, alpha, n, rows);
    const bool exact = (Xv == X);
    if (!exact) pack(Xv, nullptr, nv, vrows);
    const int npad = (nv + 15) / 16 * 16;
    // MFMA tile pack of the mean rows, centred on their mean (sqp_kernel.hip gp_tiles)
    const double c = -0.5 / (lengthscale * lengthscale);
    double xbar[3] = {0.0, 0.0, 0.0};
    for (int i = 0; i < n; ++i)
        for (int k = 0; k < d; ++k) xbar[k] += X[(size_t)i * d + k] / n;
    const int ntile = (n + 15) / 16;
    std::vector<double> tiles((size_t)ntile * (64 + 64), 0.0);
    double* tX = tiles.data();
    double* tW = tiles.data() + (size_t)ntile * 64;
    const double m2c = 1.0 / (lengthscale * lengthscale);
    for (int i = 0; i < n; ++i) {
        // MFMA C/D rows: register q of lane group grp holds row grp + 4q
        const int t = i / 16, r = i % 16, grp = r % 4, q = r / 4;
        double xc[3] = {0.0, 0.0, 0.0}, sq = 0.0;
        for (int k = 0; k < d; ++k) {
            xc[k] = X[(size_t)i * d + k] - xbar[k];
            sq += xc[k] * xc[k];
            tX[(size_t)t * 64 + r * 4 + k] = m2c * xc[k];
        }
        tX[(size_t)t * 64 + r * 4 + 3] = c * sq;
        const double wv[4] = {alpha[i], alpha[i] * xc[0], alpha[i] * xc[1], alpha[i] * xc[2]};
        for (int j = 0; j < 4; ++j) tW[(size_t)t * 64 + (grp * 4 + j) * 4 + q] = wv[j];
    }
    for (double** p : {&h->gp_rows[gp_id], &h->gp_vrows[gp_id], &h->gp_linvT[gp_id], &h->gp_tiles[gp_id],
                       &h->gp_vroot[gp_id]}) {   // (a LOVE root belongs to the previous training set)
        if (*p) HIPCHK(hipFree(*p));
        *p = nullptr;
    }
    h->gp_vroot_cols[gp_id] = 0;
    h->gp_vroot_rank[gp_id] = 0;
    HIPCHK(hipMalloc(&h->gp_rows[gp_id], rows.size() * sizeof(double)));
    HIPCHK(hipMemcpy(h->gp_rows[gp_id], rows.data(), rows.size() * sizeof(double), hipMemcpyHostToDevice));
    HIPCHK(hipMalloc(&h->gp_tiles[gp_id], tiles.size() * sizeof(double)));
    HIPCHK(hipMemcpy(h->gp_tiles[gp_id], tiles.data(), tiles.size() * sizeof(double), hipMemcpyHostToDevice));
    if (!exact) {
        HIPCHK(hipMalloc(&h->gp_vrows[gp_id], vrows.size() * sizeof(double)));
        HIPCHK(hipMemcpy(h->gp_vrows[gp_id], vrows.data(), vrows.size() * sizeof(double), hipMemcpyHostToDevice));
    }
    if (Linv) {
        std::vector<double> lt((size_t)npad * npad, 0.0);
        for (int i = 0; i < nv; ++i)
            for (int j = 0; j <= i; ++j) lt[(size_t)j * npad + i] = Linv[(size_t)i * nv + j];  // (L^-1)^T
        HIPCHK(hipMalloc(&h->gp_linvT[gp_id], lt.size() * sizeof(double)));
        HIPCHK(hipMemcpy(h->gp_linvT[gp_id], lt.data(), lt.size() * sizeof(double), hipMemcpyHostToDevice));
    }
    GPDev& g = h->P.gp[gp_id];
    g.rows = h->gp_rows[gp_id];
    g.vrows = exact ? h->gp_rows[gp_id] : h->gp_vrows[gp_id];
    g.linvT = h->gp_linvT[gp_id];
    g.tX = h->gp_tiles[gp_id];
    g.tW = h->gp_tiles[gp_id] + (size_t)ntile * 64;
    g.ntile = ntile;
    for (int k = 0; k < 3; ++k) g.xbar[k] = xbar[k];
    g.n = n;
    g.nv = nv;
    g.d = d;
    g.inv_ell2 = 1.0 / (lengthscale * lengthscale);
    g.sf2 = outputscale;
    g.sn2 = noise;
    h->gp_npad[gp_id] = npad;
    h->gp_set[gp_id] = true;
    bump_lin(h);
    return GPMPC_OK;
}

gpmpc_status gpmpc_set_var_inputs(gpmpc_handle* h, int32_t gp_id, const int32_t* src, int32_t d) {
    if (!h) return fail(GPMPC_ERR_ARG, "null handle");
    if (gp_id < 0 || gp_id >= h->md.ngp) return fail(GPMPC_ERR_ARG, "gp_id out of range");
    if (!src || d != h->md.gp_dim[gp_id]) return fail(GPMPC_ERR_ARG, "variance input map must have the GP's dimension");
    for (int k = 0; k < d; ++k)
        if (src[k] < 0 || src[k] >= h->md.nx + h->md.nu) return fail(GPMPC_ERR_ARG, "variance input index out of range");
    for (int k = 0; k < 3; ++k) h->md.var_src[gp_id][k] = k < d ? src[k] : 0;
    return GPMPC_OK;
}

gpmpc_status gpmpc_set_gp_variance_root(gpmpc_handle* h, int32_t gp_id, int32_t n, int32_t r, const double* R) {
    if (!h) return fail(GPMPC_ERR_ARG, "null handle");
    if (gp_id < 0 || gp_id >= h->md.ngp) return fail(GPMPC_ERR_ARG, "gp_id out of range");
    (void)hipSetDevice(h->device);
    auto drop = [&]() {   // back to the exact variance: root, columns and rank together
        if (h->gp_vroot[gp_id]) (void)hipFree(h->gp_vroot[gp_id]);
        h->gp_vroot[gp_id] = nullptr;
        h->gp_vroot_cols[gp_id] = 0;
        h->gp_vroot_rank[gp_id] = 0;
    };
    if (!R) {
        drop();
        return GPMPC_OK;
    }
    if (h->gp_npad[gp_id] == 0) return fail(GPMPC_ERR_STATE, "gpmpc_set_gp first");
    if (n != h->P.gp[gp_id].nv) return fail(GPMPC_ERR_ARG, "root rows must equal the variance GP's training rows");
    if (r < 1 || r > 16 * 16) return fail(GPMPC_ERR_ARG, "root rank must be 1..256");
    const int npad = h->gp_npad[gp_id], rpad = (r + 15) / 16 * 16;
    std::vector<double> rp((size_t)npad * rpad, 0.0);
    for (int i = 0; i < n; ++i)
        for (int c = 0; c < r; ++c) rp[(size_t)i * rpad + c] = R[(size_t)i * r + c];
    // staged in a local buffer: the handle's root, columns and rank change together, on success only
    double* buf = nullptr;
    hipError_t e = hipMalloc(&buf, rp.size() * sizeof(double));
    if (e == hipSuccess) e = hipMemcpy(buf, rp.data(), rp.size() * sizeof(double), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        if (buf) (void)hipFree(buf);
        return fail(GPMPC_ERR_HIP, std::string("LOVE root upload: ") + hipGetErrorString(e));
    }
    drop();
    h->gp_vroot[gp_id] = buf;
    h->gp_vroot_cols[gp_id] = rpad;
    h->gp_vroot_rank[gp_id] = r;
    return GPMPC_OK;
}

gpmpc_status gpmpc_use_gp(gpmpc_handle* h, int32_t enabled) {
    if (!h) return fail(GPMPC_ERR_ARG, "null handle");
    if (enabled)
        for (int g = 0; g < h->md.ngp; ++g)
            if (!h->gp_set[g]) return fail(GPMPC_ERR_STATE, "GP " + std::to_string(g) + " not set");
    if (h->P.use_gp != (enabled ? 1 : 0)) bump_lin(h);
    h->P.use_gp = enabled ? 1 : 0;
    return GPMPC_OK;
}

gpmpc_status gpmpc_set_tightening(gpmpc_handle* h, int32_t enabled, double inverse_cdf, const double* Ad,
                                  const double* Bd, const double* K) {
    if (!h) return fail(GPMPC_ERR_ARG, "null handle");
    ProblemDev& P = h->P;
    P.tighten = enabled ? 1 : 0;
    if (!enabled) return GPMPC_OK;
    if (!Ad || !Bd || !K) return fail(GPMPC_ERR_ARG, "null tightening matrices");
    const int nx = h->md.nx, nu = h->md.nu;
    P.icdf = inverse_cdf;
    for (int i = 0; i < nx; ++i)
        for (int j = 0; j < nx; ++j) {
            double acc = Ad[i * nx + j];
            for (int a = 0; a < nu; ++a) acc += Bd[i * nu + a] * K[a * nx + j];
            P.Acl[i * nx + j] = acc;
        }
    for (int a = 0; a < nu * nx; ++a) P.K[a] = K[a];
    // Gain table of the covariance convolution: column q of Acl^m Bd is column unc[q] of Acl^m
    // (Bd selects the uncertain state dims, gpmpc.py:68-69), squared entrywise, and likewise
    // for K Acl^m.  m = 0..H-1.
    int32_t unc[kMaxNX];
    const int nunc = model_unc_dims(h->model, unc);
    const int H = h->H, nb = nx + nu;
    std::vector<double> tab((size_t)H * nb * nunc), Am((size_t)nx * nx, 0.0), tmp((size_t)nx * nx);
    for (int i = 0; i < nx; ++i) Am[i * nx + i] = 1.0;
    for (int m = 0; m < H; ++m) {
        double* t = tab.data() + (size_t)m * nb * nunc;
        for (int q = 0; q < nunc; ++q) {
            for (int i = 0; i < nx; ++i) {
                const double a = Am[i * nx + unc[q]];
                t[i * nunc + q] = a * a;
            }
            for (int a = 0; a < nu; ++a) {
                double acc = 0.0;
                for (int j = 0; j < nx; ++j) acc += K[a * nx + j] * Am[j * nx + unc[q]];
                t[(nx + a) * nunc + q] = acc * acc;
            }
        }
        for (int i = 0; i < nx; ++i)   // Am <- Acl Am
            for (int j = 0; j < nx; ++j) {
                double acc = 0.0;
                for (int l = 0; l < nx; ++l) acc += P.Acl[i * nx + l] * Am[l * nx + j];
                tmp[i * nx + j] = acc;
            }
        Am.swap(tmp);
    }
    (void)hipSetDevice(h->device);
    if (!h->tgain) {
        const hipError_t e = hipMalloc(&h->tgain, tab.size() * sizeof(double));
        if (e != hipSuccess) {
            h->tgain = nullptr;
            P.tighten = 0;
            return fail(GPMPC_ERR_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
        }
    }
    HIPCHK(hipMemcpy(h->tgain, tab.data(), tab.size() * sizeof(double), hipMemcpyHostToDevice));
    P.tgain = h->tgain;
    return GPMPC_OK;
}

gpmpc_status gpmpc_reset(gpmpc_handle* h, int32_t batch, int32_t reset_iterate, void* stream) {
    if (!h) return fail(GPMPC_ERR_ARG, "null handle");
    if (batch < 1 || batch > h->max_batch) return fail(GPMPC_ERR_ARG, "batch out of range");
    (void)hipSetDevice(h->device);
    hipStream_t s = (hipStream_t)stream;
    const size_t B = batch, H = h->H;
    HIPCHK(order_after_last(h, s));
    StreamMark mark{h, s};
    HIPCHK(hipMemsetAsync(h->has_prev, 0, B * sizeof(int32_t), s));
    bump_lin(h);
    if (reset_iterate) {
        HIPCHK(hipMemsetAsync(h->x, 0, B * (H + 1) * h->md.nx * sizeof(double), s));
        HIPCHK(hipMemsetAsync(h->u, 0, B * H * h->md.nu * sizeof(double), s));
        HIPCHK(hipMemsetAsync(h->pi, 0, B * H * h->md.nx * sizeof(double), s));
        HIPCHK(hipMemsetAsync(h->lam, 0, B * (H + 1) * 2 * h->nb * sizeof(double), s));
    }
    if (batch == h->max_batch) h->any_prev = false;
    h->var_batch = 0;
    return GPMPC_OK;
}

gpmpc_status gpmpc_set_iterate(gpmpc_handle* h, int32_t batch, const double* x_dev, const double* u_dev, void* stream) {
    if (!h || !x_dev || !u_dev) return fail(GPMPC_ERR_ARG, "null argument");
    if (batch < 1 || batch > h->max_batch) return fail(GPMPC_ERR_ARG, "batch out of range");
    (void)hipSetDevice(h->device);
    hipStream_t s = (hipStream_t)stream;
    const size_t B = batch, H = h->H;
    HIPCHK(order_after_last(h, s));
    StreamMark mark{h, s};
    HIPCHK(hipMemcpyAsync(h->x, x_dev, B * (H + 1) * h->md.nx * sizeof(double), hipMemcpyDeviceToDevice, s));
    HIPCHK(hipMemcpyAsync(h->u, u_dev, B * H * h->md.nu * sizeof(double), hipMemcpyDeviceToDevice, s));
    bump_lin(h);
    HIPCHK(hipMemsetAsync(h->pi, 0, B * H * h->md.nx * sizeof(double), s));
    HIPCHK(hipMemsetAsync(h->lam, 0, B * (H + 1) * 2 * h->nb * sizeof(double), s));
    return GPMPC_OK;
}

gpmpc_status gpmpc_solve(gpmpc_handle* h, int32_t batch, const double* x0, const int32_t* tstep, double* u0,
                         int32_t* status, int32_t* sqp_iter, int32_t* qp_iter, double* res, void* stream) {
    if (!h) return fail(GPMPC_ERR_ARG, "null handle");
    if (!h->model_set) return fail(GPMPC_ERR_STATE, "gpmpc_set_model not called");
    if (!h->ref_set) return fail(GPMPC_ERR_STATE, "gpmpc_set_reference not called");
    if (batch < 1 || batch > h->max_batch) return fail(GPMPC_ERR_ARG, "batch out of range");
    if (!x0 || !tstep || !u0 || !status) return fail(GPMPC_ERR_ARG, "null output/input");
    if (h->P.tighten && h->P.use_gp)
        for (int g = 0; g < h->md.ngp; ++g)
            if (!h->gp_linvT[g]) return fail(GPMPC_ERR_STATE, "tightening needs Linv for every GP");
    (void)hipSetDevice(h->device);
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(order_after_last(h, s));
    StreamMark mark{h, s};
    ProblemDev P = h->P;
    P.tighten = (h->P.tighten && h->P.use_gp) ? 1 : 0;
    // Profiling events are best effort: a failed record drops that launch's timing (the events go
    // back to the pool), never the solve.  Every early return below recycles what it took.
    auto give_back = [&](hipEvent_t& e) {
        if (e) h->ev_pool.push_back(e);
        e = nullptr;
    };
    // GP variances at the previous solution (the MFMA contraction) of the instances of ranks
    // first .. first + count - 1 in `order` (null: instances first .. first + count - 1)
    auto launch_var = [&](int first, int count, const int32_t* order, hipStream_t st) -> hipError_t {
        PostBatch pb{};
        pb.n = h->md.ngp;
        pb.step_points = batch * h->H;
        pb.var_split = h->var_split;
        for (int g = 0; g < h->md.ngp; ++g) {
            PostArgs& a = pb.a[g];
            a.sx = h->x;
            a.su = h->u;
            a.H = h->H;
            a.nx = h->md.nx;
            a.nu = h->md.nu;
            a.ngp = h->md.ngp;
            a.gp_index = g;
            for (int k = 0; k < 3; ++k) a.src[k] = h->md.var_src[g][k];
            a.P = count * h->H;
            a.d = h->md.gp_dim[g];
            a.with_noise = 1;   // gp.likelihood(gp(z)) (gpmpc.py:444)
            a.mean = nullptr;
            a.var = h->var;
            a.var_stride = h->md.ngp;
            a.var_off = g;
            a.order = order;
            a.first = first;
            pb.g[g] = P.gp[g];
            pb.g[g].vroot = h->gp_vroot[g];   // LOVE (fast_pred_var) when a root is set
            pb.g[g].vroot_cols = h->gp_vroot_cols[g];
            pb.g[g].vroot_rank = h->gp_vroot_rank[g];
            pb.npad[g] = h->gp_npad[g];
        }
        return launch_gp_post_batch(pb, true, st);
    };
    StateDev S{h->x, h->u, h->pi, h->lam, h->has_prev, h->var, h->tight, h->lin_cache ? h->lin : nullptr, h->lin_tag,
               h->order, h->cost, 0};
    StepIO io{x0, tstep, u0, status, sqp_iter, qp_iter, res, h->timing, h->stats};
    // optional outputs go to handle-owned scratch when NULL
    if (!io.sqp_iter) io.sqp_iter = h->scratch_i;
    if (!io.qp_iter) io.qp_iter = h->scratch_i + h->max_batch;
    if (!io.res) io.res = h->scratch_d;
    hipEvent_t e0 = nullptr, e1 = nullptr, mid = nullptr;
    const bool var_launch = P.tighten && h->any_prev;

    // Overlapped step: when the variance launch precedes an SQP launch that fills the device with one
    // wave per instance (or needs more than one round of workgroups), the instances are ranked by
    // the cost of their last solve and split in two halves.  The costlier half's variances run
    // first and its SQP launch starts right after them; the cheaper half's variances and SQP launch
    // run on a second stream beside it, so the step waits only for the first half's variances before
    // the solves that set its length begin.  Each instance's arithmetic is unchanged (same kernels,
    // same per-instance data), so the results are bit-identical to the sequential order.
    if (var_launch && h->overlap && batch >= 2 && batch <= 16384 && sqp_overlap_ok(P, batch)) {
        if (const hipError_t ce = ensure_side(h); ce != hipSuccess)
            return fail(GPMPC_ERR_HIP, std::string("side stream: ") + hipGetErrorString(ce));
        const int b1 = (batch + 1) / 2, b2 = batch - b1;
        HIPCHK(launch_sqp_order(S, batch, s));
        if (h->profiling) {
            e0 = take_event(h);
            e1 = take_event(h);
            if (e0 && hipEventRecord(e0, s) != hipSuccess) give_back(e0);
        }
        hipError_t ve = launch_var(0, b1, h->order, s);
        if (ve == hipSuccess && e0 && e1 && hipEventRecord(e1, s) == hipSuccess) {
            h->ev_var.push_back({e0, e1});
            mid = e1;
        } else {
            give_back(e0);
            give_back(e1);
        }
        if (ve == hipSuccess) ve = hipEventRecord(h->ev_fork, s);
        if (ve == hipSuccess) ve = hipStreamWaitEvent(h->side, h->ev_fork, 0);
        if (ve != hipSuccess) {
            h->var_batch = 0;
            if (mid) h->ev_var_owned.push_back(mid);
            return fail(GPMPC_ERR_HIP, std::string("variance launch: ") + hipGetErrorString(ve));
        }
        // var rows are valid only for what is queued: the costlier half now (ranked instances, so
        // no prefix of the batch is complete: none), the whole batch once the second half's
        // variance launch is queued too
        h->var_batch = 0;
        hipEvent_t e2 = h->profiling && mid ? take_event(h) : nullptr;
        hipError_t le = launch_sqp(P, S, io, batch, s, 0, b1);
        // once an SQP launch is queued it will update the iterate: the host state follows it
        if (le == hipSuccess) h->any_prev = true;
        if (le == hipSuccess) le = launch_var(b1, b2, h->order, h->side);
        if (le == hipSuccess) h->var_batch = batch;
        if (le == hipSuccess) le = launch_sqp(P, S, io, batch, h->side, b1, b2);
        // the join is recorded whatever happened above, so the caller's stream never runs ahead of
        // work already queued on the side stream
        const hipError_t je = hipEventRecord(h->ev_join, h->side);
        const hipError_t we = je == hipSuccess ? hipStreamWaitEvent(s, h->ev_join, 0) : je;
        if (le == hipSuccess) le = we;
        if (le != hipSuccess) {
            if (mid) h->ev_var_owned.push_back(mid);
            give_back(e2);
            return fail(GPMPC_ERR_HIP, std::string("launch_sqp: ") + hipGetErrorString(le));
        }
        if (mid && e2 && hipEventRecord(e2, s) == hipSuccess) {
            h->ev_sqp.push_back({mid, e2});
        } else {
            if (mid) h->ev_var_owned.push_back(mid);
            give_back(e2);
        }
        if (h->stage_cost) HIPCHK(launch_stage_cost(P, h->x, h->u, tstep, status, h->stage_cost, batch, s));
        return GPMPC_OK;
    }

    // 1. GP variances at the previous solution, only when needed
    if (var_launch) {
        if (h->profiling) {
            e0 = take_event(h);
            e1 = take_event(h);
            if (e0 && hipEventRecord(e0, s) != hipSuccess) give_back(e0);
        }
        const hipError_t ve = launch_var(0, batch, nullptr, s);
        if (ve != hipSuccess) {
            give_back(e0);
            give_back(e1);
            h->var_batch = 0;
            return fail(GPMPC_ERR_HIP, std::string("launch_gp_post_batch: ") + hipGetErrorString(ve));
        }
        if (e0 && e1 && hipEventRecord(e1, s) == hipSuccess) {
            h->ev_var.push_back({e0, e1});
            mid = e1;   // also the SQP launch's start
        } else {
            give_back(e0);
            give_back(e1);
        }
    }
    h->var_batch = var_launch ? batch : 0;
    // 2. the SQP step
    e0 = e1 = nullptr;
    if (h->profiling) {
        e0 = mid;
        if (!e0) {
            e0 = take_event(h);
            if (e0 && hipEventRecord(e0, s) != hipSuccess) give_back(e0);
        }
        e1 = take_event(h);
        if (!e0) give_back(e1);
    }
    // events not handed to ev_sqp: the shared `mid` stays in use as ev_var's end event (the
    // variance list takes ownership of it), the others go back to the pool, on every exit path
    auto recycle = [&]() {
        if (e0 && e0 == mid) h->ev_var_owned.push_back(e0);
        else if (e0) h->ev_pool.push_back(e0);
        if (e1) h->ev_pool.push_back(e1);
    };
    // Tail boost (GPMPC_TUNE_TAIL = K > 0): a launch that gives every instance one wave in one round
    // of workgroups (the metric's 1024 quad2d instances on one MI355X) lasts as long as its slowest
    // instance, and the costliest instances stay costly from step to step (StateDev::cost).  The
    // instances are ranked by the cost of their previous solve; the K costliest run as two-wave
    // segment solves (their recursions split over two waves) on the caller's stream, right behind the
    // ranking kernel, and the others as one-wave instances on the side stream, released by the same
    // ranking kernel (the side stream's wait resolves after the caller's next packet is dispatched, so
    // the two-wave instances take their SIMDs first).  With one SIMD per wave the K extra waves make
    // the K cheapest instances (dispatched last) wait for the SIMDs of the first instances to finish.
    // Each instance's arithmetic is its launch shape's, identical up to rounding to the one-wave
    // solve (the parity tests cover both shapes).
    bool tail_queued = false;
    auto launch_step = [&]() -> hipError_t {
        const int K = tail_count(h, P, batch);
        if (K <= 0) return launch_sqp(P, S, io, batch, s);
        hipError_t e = ensure_side(h);
        if (e == hipSuccess) e = launch_sqp_order(S, batch, s);
        if (e == hipSuccess) e = hipEventRecord(h->ev_fork, s);
        if (e == hipSuccess) e = hipStreamWaitEvent(h->side, h->ev_fork, 0);
        if (e != hipSuccess) return e;
        ProblemDev P2 = P, P1 = P;
        P2.waves = 2;   // (sqp_tail_ok: segment solves on two waves)
        P1.waves = 1;
        e = launch_sqp(P2, S, io, batch, s, 0, K);
        if (e == hipSuccess) tail_queued = true;
        if (e == hipSuccess) e = launch_sqp(P1, S, io, batch, h->side, K, batch - K);
        // the join is recorded whatever happened above, so the caller's stream never runs ahead of
        // work already queued on the side stream
        const hipError_t je = hipEventRecord(h->ev_join, h->side);
        const hipError_t we = je == hipSuccess ? hipStreamWaitEvent(s, h->ev_join, 0) : je;
        return e == hipSuccess ? we : e;
    };
    const hipError_t le = launch_step();
    if (le != hipSuccess) {
        if (tail_queued) h->any_prev = true;   // part of the batch's iterate is being updated
        recycle();
        return fail(GPMPC_ERR_HIP, std::string("launch_sqp: ") + hipGetErrorString(le));
    }
    // the SQP kernel is queued and will update the iterate: from here on the host state follows it
    h->any_prev = true;
    if (e0 && e1 && hipEventRecord(e1, s) == hipSuccess) h->ev_sqp.push_back({e0, e1});
    else recycle();   // lost profiling data only
    // stage costs of the stored solution, behind the SQP launch (and outside its timing events)
    if (h->stage_cost) HIPCHK(launch_stage_cost(P, h->x, h->u, tstep, status, h->stage_cost, batch, s));
    return GPMPC_OK;
}

gpmpc_status gpmpc_get_variance(gpmpc_handle* h, int32_t batch, double* var_dev, void* stream) {
    if (!h || !var_dev) return fail(GPMPC_ERR_ARG, "null argument");
    if (batch < 1 || batch > h->max_batch) return fail(GPMPC_ERR_ARG, "batch out of range");
    if (h->var_batch == 0)
        return fail(GPMPC_ERR_STATE, "the last solve ran no variance launch (first step, tightening or GPs off)");
    if (batch > h->var_batch)
        return fail(GPMPC_ERR_ARG, "the last variance launch covered " + std::to_string(h->var_batch) + " instances");
    (void)hipSetDevice(h->device);
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(order_after_last(h, s));
    StreamMark mark{h, s};
    const size_t B = batch, H = h->H;
    HIPCHK(hipMemcpyAsync(var_dev, h->var, B * H * h->md.ngp * sizeof(double), hipMemcpyDeviceToDevice, s));
    return GPMPC_OK;
}

gpmpc_status gpmpc_set_launch(gpmpc_handle* h, int32_t waves) {
    if (!h) return fail(GPMPC_ERR_ARG, "null handle");
    if (waves != 0 && waves != 1 && waves != 2 && waves != 4) return fail(GPMPC_ERR_ARG, "waves must be 0 (auto), 1, 2 or 4");
    if (h->model == kQuad3D && waves != 0 && waves != 4)
        return fail(GPMPC_ERR_ARG, "quad3d runs four waves per instance (waves must be 0 or 4)");
    h->P.waves = waves;
    return GPMPC_OK;
}

gpmpc_status gpmpc_get_launch_info(gpmpc_handle* h, int32_t batch, int32_t* waves, int32_t* overlapped) {
    if (!h) return fail(GPMPC_ERR_ARG, "null handle");
    if (batch < 1 || batch > h->max_batch) return fail(GPMPC_ERR_ARG, "batch out of range");
    if (waves) *waves = sqp_launch_waves(h->P, batch);
    // the overlap needs a variance launch (tightening with GPs) besides the shape
    if (overlapped) {
        *overlapped = (h->overlap && h->P.tighten && h->P.use_gp && batch >= 2 && batch <= 16384 &&
                       sqp_overlap_ok(h->P, batch)) ? 1 : 0;
        if (*overlapped == 0 && tail_count(h, h->P, batch) > 0) *overlapped = 2;   // tail boost
    }
    return GPMPC_OK;
}

gpmpc_status gpmpc_get_launch_segments(gpmpc_handle* h, int32_t batch, int32_t* segments) {
    if (!h) return fail(GPMPC_ERR_ARG, "null handle");
    if (batch < 1 || batch > h->max_batch) return fail(GPMPC_ERR_ARG, "batch out of range");
    if (!segments) return fail(GPMPC_ERR_ARG, "null output");
    *segments = sqp_launch_segments(h->P, batch);
    return GPMPC_OK;
}

gpmpc_status gpmpc_set_tuning(gpmpc_handle* h, int32_t option, int32_t value) {
    if (!h) return fail(GPMPC_ERR_ARG, "null handle");
    switch (option) {
        case GPMPC_TUNE_LIN_CACHE:
            if (value != 0 && value != 1) break;
            if (h->lin_cache != (value == 1)) bump_lin(h);   // tags written under the other setting are stale
            h->lin_cache = value == 1;
            return GPMPC_OK;
        case GPMPC_TUNE_ORDER:
            if (value < 0 || value > 2) break;
            h->P.order_dispatch = value;
            return GPMPC_OK;
        case GPMPC_TUNE_OVERLAP:
            if (value != 0 && value != 1) break;
            h->overlap = value == 1;
            return GPMPC_OK;
        case GPMPC_TUNE_VAR_SPLIT:
            if (value != 0 && value != 1 && value != 4) break;
            h->var_split = value;
            return GPMPC_OK;
        case GPMPC_TUNE_SEG:
            if (value != 0 && value != 1) break;
            h->P.seg = value;
            return GPMPC_OK;
        case GPMPC_TUNE_SEG_PIVOT:
            // threshold 10^-value; -1: every pivot refused (every solve takes the fallback, a test of it)
            if (value < -1 || value > 300) break;
            h->P.seg_piv_rel = value < 0 ? HUGE_VAL : std::pow(10.0, -value);
            return GPMPC_OK;
        case GPMPC_TUNE_TAIL:
            if (value < -1 || value > 16384) break;
            h->tail = value;
            return GPMPC_OK;
        case GPMPC_TUNE_EVENT_FENCE:
            if (value != 0 && value != 1) break;
            if (h->event_fence != (value == 1)) {   // pooled events carry the old flags (the ones still in
                for (hipEvent_t e : h->ev_pool) {     // use are dropped when they come back: take_event)
                    h->ev_fenced.erase(e);
                    (void)hipEventDestroy(e);
                }
                h->ev_pool.clear();
            }
            h->event_fence = value == 1;
            return GPMPC_OK;
        default:
            return fail(GPMPC_ERR_ARG, "unknown tuning option " + std::to_string(option));
    }
    return fail(GPMPC_ERR_ARG, "bad value " + std::to_string(value) + " for tuning option " + std::to_string(option));
}

gpmpc_status gpmpc_set_cost_buffer(gpmpc_handle* h, void* cost_dev) {
    if (!h) return fail(GPMPC_ERR_ARG, "null handle");
    h->stage_cost = (double*)cost_dev;
    return GPMPC_OK;
}

gpmpc_status gpmpc_set_profiling(gpmpc_handle* h, int32_t enabled) {
    if (!h) return fail(GPMPC_ERR_ARG, "null handle");
    h->profiling = enabled != 0;
    return GPMPC_OK;
}

// true (and forgotten) if `e` is an ev_var end event that the variance list owns
static bool release_owned(gpmpc_handle* h, hipEvent_t e) {
    for (size_t i = 0; i < h->ev_var_owned.size(); ++i)
        if (h->ev_var_owned[i] == e) {
            h->ev_var_owned.erase(h->ev_var_owned.begin() + i);
            return true;
        }
    return false;
}

gpmpc_status gpmpc_kernel_times(gpmpc_handle* h, double* var_ms, int32_t* n_var, double* sqp_ms, int32_t* n_sqp) {
    if (!h) return fail(GPMPC_ERR_ARG, "null handle");
    (void)hipSetDevice(h->device);
    // (the variance list's end events belong to the SQP list, which returns them to the pool)
    auto sum = [&](std::vector<std::pair<hipEvent_t, hipEvent_t>>& v, double* ms, int32_t* n) -> gpmpc_status {
        const bool sqp_list = &v == &h->ev_sqp;
        double acc = 0.0;
        for (auto& pr : v) {
            HIPCHK(hipEventSynchronize(pr.second));
            float t = 0.0f;
            HIPCHK(hipEventElapsedTime(&t, pr.first, pr.second));
            acc += t;
            h->ev_pool.push_back(pr.first);
            if (sqp_list || release_owned(h, pr.second)) h->ev_pool.push_back(pr.second);
        }
        if (ms) *ms = acc;
        if (n) *n = (int32_t)v.size();
        v.clear();
        return GPMPC_OK;
    };
    gpmpc_status st = sum(h->ev_var, var_ms, n_var);
    if (st != GPMPC_OK) return st;
    return sum(h->ev_sqp, sqp_ms, n_sqp);
}

gpmpc_status gpmpc_kernel_time_list(gpmpc_handle* h, int32_t cap, double* var_ms, int32_t* n_var, double* sqp_ms,
                                    int32_t* n_sqp) {
    if (!h) return fail(GPMPC_ERR_ARG, "null handle");
    if (cap < 0) return fail(GPMPC_ERR_ARG, "negative capacity");
    (void)hipSetDevice(h->device);
    // (the variance list's end events belong to the SQP list, which returns them to the pool)
    auto take = [&](std::vector<std::pair<hipEvent_t, hipEvent_t>>& v, double* ms, int32_t* n) -> gpmpc_status {
        const bool sqp_list = &v == &h->ev_sqp;
        int32_t i = 0;
        for (auto& pr : v) {
            HIPCHK(hipEventSynchronize(pr.second));
            float t = 0.0f;
            HIPCHK(hipEventElapsedTime(&t, pr.first, pr.second));
            if (ms && i < cap) ms[i] = t;
            ++i;
            h->ev_pool.push_back(pr.first);
            if (sqp_list || release_owned(h, pr.second)) h->ev_pool.push_back(pr.second);
        }
        if (n) *n = i;
        v.clear();
        return GPMPC_OK;
    };
    gpmpc_status st = take(h->ev_var, var_ms, n_var);
    if (st != GPMPC_OK) return st;
    return take(h->ev_sqp, sqp_ms, n_sqp);
}

gpmpc_status gpmpc_set_timing_buffer(gpmpc_handle* h, void* timing_dev) {
    if (!h) return fail(GPMPC_ERR_ARG, "null handle");
    h->timing = (unsigned long long*)timing_dev;
    return GPMPC_OK;
}

gpmpc_status gpmpc_set_stats_buffer(gpmpc_handle* h, void* stats_dev, int32_t slots) {
    if (!h) return fail(GPMPC_ERR_ARG, "null handle");
    if (stats_dev && slots < kStatsSlots)
        return fail(GPMPC_ERR_ARG, "stats buffer needs GPMPC_STATS_SLOTS = " + std::to_string(kStatsSlots) +
                                       " int64 slots per instance, got " + std::to_string(slots));
    if (stats_dev && slots != kStatsSlots)
        return fail(GPMPC_ERR_ARG, "stats buffer row stride must be GPMPC_STATS_SLOTS = " + std::to_string(kStatsSlots));
    h->stats = (long long*)stats_dev;
    return GPMPC_OK;
}

gpmpc_status gpmpc_get_solution(gpmpc_handle* h, int32_t batch, double* x_dev, double* u_dev, double* tight_dev,
                                void* stream) {
    if (!h) return fail(GPMPC_ERR_ARG, "null handle");
    if (batch < 1 || batch > h->max_batch) return fail(GPMPC_ERR_ARG, "batch out of range");
    (void)hipSetDevice(h->device);
    hipStream_t s = (hipStream_t)stream;
    const size_t B = batch, H = h->H;
    HIPCHK(order_after_last(h, s));
    StreamMark mark{h, s};
    if (x_dev) HIPCHK(hipMemcpyAsync(x_dev, h->x, B * (H + 1) * h->md.nx * sizeof(double), hipMemcpyDeviceToDevice, s));
    if (u_dev) HIPCHK(hipMemcpyAsync(u_dev, h->u, B * H * h->md.nu * sizeof(double), hipMemcpyDeviceToDevice, s));
    if (tight_dev)
        HIPCHK(hipMemcpyAsync(tight_dev, h->tight, B * (H + 1) * h->nb * sizeof(double), hipMemcpyDeviceToDevice, s));
    return GPMPC_OK;
}

gpmpc_status gpmpc_gp_predict(gpmpc_handle* h, int32_t gp_id, const double* Z, int32_t P, double* mean, double* var,
                              int32_t with_noise, void* stream) {
    if (!h) return fail(GPMPC_ERR_ARG, "null handle");
    if (gp_id < 0 || gp_id >= h->md.ngp || !h->gp_set[gp_id]) return fail(GPMPC_ERR_STATE, "GP not set");
    if (P < 0 || (P > 0 && !Z)) return fail(GPMPC_ERR_ARG, "bad points");
    if (var && !h->gp_linvT[gp_id]) return fail(GPMPC_ERR_STATE, "variance needs Linv");
    if (P == 0) return GPMPC_OK;
    (void)hipSetDevice(h->device);
    const GPDev& g = h->P.gp[gp_id];
    PostArgs a{};
    a.Z = Z;
    a.ldz = h->md.gp_dim[gp_id];
    a.P = P;
    a.d = h->md.gp_dim[gp_id];
    a.with_noise = with_noise;
    a.var_stride = 1;
    a.var_off = 0;
    if (mean) {  // mean over the mean set (exact: training set; FITC: inducing set)
        GPDev gm = g;
        gm.vrows = g.rows;
        gm.nv = g.n;
        gm.linvT = nullptr;
        a.mean = mean;
        a.var = nullptr;
        HIPCHK(launch_gp_post(gm, (g.n + 15) / 16 * 16, a, false, (hipStream_t)stream));
    }
    if (var) {
        a.mean = nullptr;
        a.var = var;
        HIPCHK(launch_gp_post(g, h->gp_npad[gp_id], a, false, (hipStream_t)stream));
    }
    return GPMPC_OK;
}

gpmpc_status gpmpc_gp_mean_grad(gpmpc_handle* h, int32_t gp_id, const double* Z, int32_t P, double* mean,
                                double* grad, void* stream) {
    if (!h) return fail(GPMPC_ERR_ARG, "null handle");
    if (gp_id < 0 || gp_id >= h->md.ngp || !h->gp_set[gp_id]) return fail(GPMPC_ERR_STATE, "GP not set");
    if (P < 0 || (P > 0 && !Z)) return fail(GPMPC_ERR_ARG, "bad points");
    if (P == 0) return GPMPC_OK;
    (void)hipSetDevice(h->device);
    HIPCHK(launch_gp_mean_grad(h->P.gp[gp_id], Z, P, mean, grad, (hipStream_t)stream));
    return GPMPC_OK;
}

gpmpc_status gpmpc_gp_posterior(int32_t n, int32_t d, int32_t npad, const double* rows, const double* linvT,
                                double lengthscale, double outputscale, double noise, const double* Z, int32_t P,
                                double* mean, double* var, int32_t with_noise, void* stream) {
    if (n < 1 || d < 1 || d > kMaxGPDim || npad < n || npad % 16 != 0 || !rows)
        return fail(GPMPC_ERR_ARG, "bad GP layout (need 1 <= d <= 3, npad = 16-multiple >= n)");
    if (P < 0 || (P > 0 && !Z)) return fail(GPMPC_ERR_ARG, "bad points");
    if (var && !linvT) return fail(GPMPC_ERR_ARG, "variance needs linvT");
    if (!(lengthscale > 0.0) || !(outputscale > 0.0) || !(noise >= 0.0)) return fail(GPMPC_ERR_ARG, "bad hyperparameters");
    if (P == 0) return GPMPC_OK;
    GPDev g{};
    g.rows = rows;
    g.vrows = rows;
    g.linvT = linvT;
    g.n = g.nv = n;
    g.d = d;
    g.inv_ell2 = 1.0 / (lengthscale * lengthscale);
    g.sf2 = outputscale;
    g.sn2 = noise;
    PostArgs a{};
    a.Z = Z;
    a.ldz = d;
    a.P = P;
    a.d = d;
    a.with_noise = with_noise;
    a.mean = mean;
    a.var = var;
    a.var_stride = 1;
    a.var_off = 0;
    HIPCHK(launch_gp_post(g, npad, a, false, (hipStream_t)stream));
    return GPMPC_OK;
}

gpmpc_status gpmpc_plant_step(gpmpc_handle* h, int32_t batch, const double* params, const double* x, const double* u,
                              double* x_next, int32_t* tstep, void* stream) {
    if (!h || !params || !x || !u || !x_next) return fail(GPMPC_ERR_ARG, "null argument");
    if (batch < 1) return fail(GPMPC_ERR_ARG, "batch out of range");
    (void)hipSetDevice(h->device);
    hipStream_t s = (hipStream_t)stream;
    bool same = h->plant_params_valid;
    for (int i = 0; i < h->md.nparams; ++i) same = same && (h->plant_params_host[i] == params[i]);
    if (!same) {  // synchronous upload of a 16-double table, only when the parameters change
        for (int i = 0; i < kMaxParams; ++i) h->plant_params_host[i] = i < h->md.nparams ? params[i] : 0.0;
        HIPCHK(hipStreamSynchronize(s));
        HIPCHK(hipMemcpy(h->plant_params, h->plant_params_host, sizeof(h->plant_params_host), hipMemcpyHostToDevice));
        h->plant_params_valid = true;
    }
    HIPCHK(launch_plant(h->model, h->plant_params, h->P.dt, x, u, x_next, tstep, batch, s));
    return GPMPC_OK;
}

}  // extern "C"
