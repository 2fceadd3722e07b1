// CPU restatement of the GP-MPC control step in C++ -- TEST / BASELINE INFRASTRUCTURE ONLY.
//
// Only tests/ and bench.py's cpu_baseline leg load this library (oracle/lib/libcpuref.so,
// built by oracle/Makefile); the product path (gp-mpc_amd/) never does.  It is the
// "acados CPU path" stand-in of SURVEY.md §8(d): acados/HPIPM/CasADi are not installable
// here, so this is the same algorithm as oracle/gpmpc_oracle.py written the way those
// libraries run it -- compiled double-precision code, one instance per thread, the QP's
// Newton systems solved by a Riccati recursion over the horizon (HPIPM's structure)
// instead of the numpy oracle's dense KKT factorisation.
//
// Restated reference functions (file:line in amacati/gp-mpc):
//   covSE / GP mean k(z,X) K^-1 y and its input gradient   gpmpc/gp.py:12-21, 72-85
//   exact posterior variance + likelihood noise             gpmpc/gpmpc.py:441-445
//   GP-augmented dynamics + RK4 + exact tangent map         gpmpc/gpmpc.py:166-221, gpmpc/mpc.py:65-88
//   constraint tightening (covariance recursion)            gpmpc/gpmpc.py:425-498
//   tightened box constraints (uh = -1e-8 / +1e-8)           gpmpc/gpmpc.py:275-332, gpmpc/mpc.py:125-170
//   SQP-GN, full steps, acados status codes                 gpmpc/gpmpc.py:257-264, 334-368
//   reference window                                        gpmpc/gpmpc.py:509-514
// Conventions (variable layout d = [u_0, x_1, u_1, ..., x_T], the Mehrotra IPM, residual
// definitions, warm start) follow oracle/gpmpc_oracle.py line for line, so the two CPU
// restatements agree to rounding (tests/test_cpu_ref.py).
#include <omp.h>

#include <cstdio>
#include <cstdlib>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace {

constexpr int MX = 12, MU = 4, MB = MX + MU, MG = 4;
enum { kQuad2D = 0, kQuad3D = 1, kCartpole = 2 };
enum { kSuccess = 0, kNaN = 1, kMaxIter = 2, kQPFailure = 4 };

struct GP {
    int n = 0, d = 0, nv = 0;
    std::vector<double> X, alpha, L;   // X [n][d], L lower Cholesky of K(Xv, Xv) [nv][nv] (may be empty)
    std::vector<double> Xv;            // variance rows [nv][d]; empty: Xv = X (exact GP).  FITC:
                                       // mean over inducing rows X, variance over the training set
    std::vector<double> R;             // LOVE root [m][r] of the variance rows (empty: exact variance)
    int rr = 0;
    double ell = 1, sf2 = 1, sn2 = 0;
    int in_idx[3] = {0, 0, 0}, var_idx[3] = {0, 0, 0};

    // m(z) and dm/dz  (gpmpc/gp.py:12-14, 84-85 with alpha = K^-1 y)
    double mean_grad(const double* z, double* g) const {
        const double c = -0.5 / (ell * ell);
        double m = 0.0, gs[3] = {0.0, 0.0, 0.0};
        for (int i = 0; i < n; ++i) {
            const double* x = &X[(size_t)i * d];
            double q = 0.0, df[3];
            for (int k = 0; k < d; ++k) {
                df[k] = x[k] - z[k];
                q += df[k] * df[k];
            }
            const double w = alpha[i] * sf2 * std::exp(c * q);
            m += w;
            for (int k = 0; k < d; ++k) gs[k] += w * df[k];
        }
        for (int k = 0; k < d; ++k) g[k] = gs[k] / (ell * ell);
        return m;
    }
    // sf2 - |L^-1 k|^2 + sn2  (exact posterior variance with the likelihood noise), or with a LOVE
    // root R (R R^T ~ K^-1, gpytorch fast_pred_var, gpmpc/gpmpc.py:442-444) sf2 - |R^T k|^2 + sn2
    double var(const double* z, std::vector<double>& v) const {
        const double c = -0.5 / (ell * ell);
        const bool own = !Xv.empty();
        const int m = own ? nv : n;
        if (rr > 0) {
            v.assign(rr, 0.0);
            for (int i = 0; i < m; ++i) {
                const double* x = own ? &Xv[(size_t)i * d] : &X[(size_t)i * d];
                double q = 0.0;
                for (int k = 0; k < d; ++k) q += (x[k] - z[k]) * (x[k] - z[k]);
                const double s = sf2 * std::exp(c * q);
                const double* Ri = &R[(size_t)i * rr];
                for (int j = 0; j < rr; ++j) v[j] += s * Ri[j];
            }
            double acc = 0.0;
            for (int j = 0; j < rr; ++j) acc += v[j] * v[j];
            return sf2 - acc + sn2;
        }
        v.resize(m);
        double acc = 0.0;
        for (int i = 0; i < m; ++i) {
            const double* x = own ? &Xv[(size_t)i * d] : &X[(size_t)i * d];
            double q = 0.0;
            for (int k = 0; k < d; ++k) q += (x[k] - z[k]) * (x[k] - z[k]);
            double s = sf2 * std::exp(c * q);
            const double* Li = &L[(size_t)i * m];
            for (int j = 0; j < i; ++j) s -= Li[j] * v[j];
            v[i] = s / Li[i];
            acc += v[i] * v[i];
        }
        return sf2 - acc + sn2;
    }
};

struct Problem {
    int model = 0, H = 0, nx = 0, nu = 0, ngp = 0;
    double p[16] = {0}, dt = 0.02, uh = -1e-8;
    double xlo[MX], xhi[MX], ulo[MU], uhi[MU], q[MX], r[MU], ueq[MU];
    bool cost_scaling = true, use_gp = false;
    int max_iter = 25, qp_max_iter = 50;
    double tol = 1e-6, qp_tol = 1e-6;   // acados: the QP solves to the NLP tolerances
    GP gp[MG];
    std::vector<double> traj;   // [L][nx]
    int traj_len = 0;
    bool tighten = false;
    double icdf = 0.0, Ad[MX * MX], Bd[MX * MU], K[MU * MX];
    int unc[MX], n_unc = 0;
};

// ------------------------------------------------------------------------------ models
// f(x, u) and J = [df/dx, df/du] (nx x (nx+nu)), GP means gm and input gradients gg
// (oracle/gpmpc_oracle.py _quad2d_f / _quad3d_f / _cartpole_f).
void f_jac(const Problem& P, const double* x, const double* u, const double* gm, const double (*gg)[3], double* f,
           double* J) {
    const int nx = P.nx, nb = P.nx + P.nu;
    std::fill(J, J + nx * nb, 0.0);
    const double* p = P.p;
    auto Jr = [&](int i, int j) -> double& { return J[i * nb + j]; };
    if (P.model == kQuad2D) {   // p = [a, b, f, h, l, g]
        const double th = x[4], s = std::sin(th), c = std::cos(th);
        const double acc = p[0] * u[0] + p[1] + gm[0], dacc = p[0] + gg[0][0];
        f[0] = x[1]; f[1] = acc * s; f[2] = x[3]; f[3] = acc * c - p[5]; f[4] = x[5];
        f[5] = p[2] * th + p[3] * x[5] + p[4] * u[1] + gm[1];
        Jr(0, 1) = 1.0; Jr(1, 4) = acc * c; Jr(1, 6) = dacc * s; Jr(2, 3) = 1.0;
        Jr(3, 4) = -acc * s; Jr(3, 6) = dacc * c; Jr(4, 5) = 1.0;
        Jr(5, 4) = p[2] + gg[1][0]; Jr(5, 5) = p[3] + gg[1][1]; Jr(5, 7) = p[4] + gg[1][2];
    } else if (P.model == kQuad3D) {   // p = [a, b, c, d, e, f, h, l, g]
        const double phi = x[6], th = x[7], psi = x[8];
        const double cf = std::cos(phi), sf = std::sin(phi), ct = std::cos(th), st = std::sin(th);
        const double cp = std::cos(psi), sp = std::sin(psi);
        const double A = p[0] * u[0] + p[1], mT = gm[0], g = p[8];
        const double gx = cf * st * cp + sf * sp, gy = cf * st * sp - sf * cp, gz = cf * ct;
        f[0] = x[1]; f[1] = A * gx + mT * cf * st; f[2] = x[3]; f[3] = A * gy - mT * sf; f[4] = x[5];
        f[5] = A * gz - g + mT * cf * ct; f[6] = x[9]; f[7] = x[10]; f[8] = x[11];
        f[9] = p[2] * phi + p[3] * x[9] + p[4] * u[1] + gm[1];
        f[10] = p[5] * th + p[6] * x[10] + p[7] * u[2] + gm[2];
        f[11] = p[2] * psi + p[3] * x[11] + p[4] * u[3];
        const double dA = p[0], dmT = gg[0][0];
        Jr(0, 1) = Jr(2, 3) = Jr(4, 5) = 1.0;
        Jr(1, 6) = A * (-sf * st * cp + cf * sp) + mT * (-sf * st);
        Jr(1, 7) = A * (cf * ct * cp) + mT * (cf * ct);
        Jr(1, 8) = A * (-cf * st * sp + sf * cp);
        Jr(1, 12) = dA * gx + dmT * cf * st;
        Jr(3, 6) = A * (-sf * st * sp - cf * cp) - mT * cf;
        Jr(3, 7) = A * (cf * ct * sp);
        Jr(3, 8) = A * (cf * st * cp + sf * sp);
        Jr(3, 12) = dA * gy - dmT * sf;
        Jr(5, 6) = A * (-sf * ct) + mT * (-sf * ct);
        Jr(5, 7) = A * (-cf * st) + mT * (-cf * st);
        Jr(5, 12) = dA * gz + dmT * cf * ct;
        Jr(6, 9) = Jr(7, 10) = Jr(8, 11) = 1.0;
        Jr(9, 6) = p[2] + gg[1][0]; Jr(9, 9) = p[3] + gg[1][1]; Jr(9, 13) = p[4] + gg[1][2];
        Jr(10, 7) = p[5] + gg[2][0]; Jr(10, 10) = p[6] + gg[2][1]; Jr(10, 14) = p[7] + gg[2][2];
        Jr(11, 8) = p[2]; Jr(11, 11) = p[3]; Jr(11, 15) = p[4];
    } else {   // cartpole, p = [m_c, m_p, l, g]
        const double mc = p[0], mp = p[1], l = p[2], g = p[3], M = mc + mp;
        const double th = x[2], w = x[3], F = u[0], s = std::sin(th), c = std::cos(th);
        const double tmp = (F + mp * l * w * w * s) / M;
        const double den = l * (4.0 / 3.0 - mp * c * c / M);
        const double num = g * s - c * tmp;
        const double tha = num / den, k = mp * l / M, xa = tmp - k * tha * c;
        const double dtmp[3] = {mp * l * w * w * c / M, 2 * mp * l * w * s / M, 1.0 / M};
        const double dden[3] = {l * 2 * mp * c * s / M, 0.0, 0.0};
        const double dnum[3] = {g * c + s * tmp - c * dtmp[0], -c * dtmp[1], -c * dtmp[2]};
        f[0] = x[1]; f[1] = xa + gm[0]; f[2] = w; f[3] = tha + gm[1];
        Jr(0, 1) = 1.0; Jr(2, 3) = 1.0;
        for (int j = 0; j < 3; ++j) {
            const double dtha = (dnum[j] * den - num * dden[j]) / (den * den);
            const double dxa = dtmp[j] - k * (dtha * c - (j == 0 ? tha * s : 0.0));
            Jr(1, 2 + j) = dxa + gg[0][j];
            Jr(3, 2 + j) = dtha + gg[1][j];
        }
    }
}

// GP means/gradients of the GPs whose inputs are all controls are constant over the RK4 stages of
// one step and are evaluated once (u_only = true pass); the state-dependent ones at every stage.
bool u_only(const Problem& P, int g) {
    for (int k = 0; k < P.gp[g].d; ++k)
        if (P.gp[g].in_idx[k] < P.nx) return false;
    return true;
}

void gp_eval(const Problem& P, const double* x, const double* u, bool u_pass, double* gm, double (*gg)[3]) {
    if (!P.use_gp) return;
    double z[MB];
    std::copy(x, x + P.nx, z);
    std::copy(u, u + P.nu, z + P.nx);
    for (int g = 0; g < P.ngp; ++g) {
        if (u_only(P, g) != u_pass) continue;
        double zi[3];
        for (int k = 0; k < P.gp[g].d; ++k) zi[k] = z[P.gp[g].in_idx[k]];
        gm[g] = P.gp[g].mean_grad(zi, gg[g]);
    }
}

// x+ = RK4(x, u) and [dx+/dx | dx+/du]  (Dynamics.rk4)
void rk4(const Problem& P, const double* x, const double* u, double* xn, double* Jn) {
    const int nx = P.nx, nb = P.nx + P.nu;
    const double h = P.dt;
    double k[4][MX], dk[4][MX * MB], J[MX * MB], xs[MX];
    const double cs[4] = {0.0, 0.5, 0.5, 1.0};
    double gm[MG] = {0, 0, 0, 0}, gg[MG][3] = {};
    gp_eval(P, x, u, true, gm, gg);
    for (int s = 0; s < 4; ++s) {
        for (int i = 0; i < nx; ++i) xs[i] = s == 0 ? x[i] : x[i] + cs[s] * h * k[s - 1][i];
        gp_eval(P, xs, u, false, gm, gg);
        f_jac(P, xs, u, gm, gg, k[s], J);
        // dk_s = J_x (E + c h dk_{s-1}) + [0 | J_u]
        for (int i = 0; i < nx; ++i)
            for (int j = 0; j < nb; ++j) {
                double acc = j >= nx ? J[i * nb + j] : 0.0;
                for (int m = 0; m < nx; ++m) {
                    const double e = (m == j ? 1.0 : 0.0) + (s == 0 ? 0.0 : cs[s] * h * dk[s - 1][m * nb + j]);
                    acc += J[i * nb + m] * e;
                }
                dk[s][i * nb + j] = acc;
            }
    }
    for (int i = 0; i < nx; ++i) {
        xn[i] = x[i] + h / 6.0 * (k[0][i] + 2 * k[1][i] + 2 * k[2][i] + k[3][i]);
        for (int j = 0; j < nb; ++j)
            Jn[i * nb + j] = (i == j ? 1.0 : 0.0) +
                             h / 6.0 * (dk[0][i * nb + j] + 2 * dk[1][i * nb + j] + 2 * dk[2][i * nb + j] + dk[3][i * nb + j]);
    }
}

// per-point tightening weights W[j][g]: cov_d[j] = sum_g W[j][g] var_g  (variance_weights)
void var_weights(const Problem& P, const double* x, double (*W)[MG]) {
    for (int j = 0; j < MX; ++j)
        for (int g = 0; g < MG; ++g) W[j][g] = 0.0;
    if (P.model == kQuad3D) {
        const double phi = x[6], th = x[7];
        W[0][0] = std::cos(phi) * std::sin(th) * std::sin(th);   // gpmpc.py:449 (cos not squared)
        W[1][0] = std::sin(phi) * std::sin(phi);
        W[2][0] = std::cos(phi) * std::cos(th) * std::cos(phi) * std::cos(th);
        W[3][1] = 1.0;
        W[4][2] = 1.0;
    } else if (P.model == kQuad2D) {
        const double th = x[4];
        W[0][0] = std::sin(th) * std::sin(th);
        W[1][0] = std::cos(th) * std::cos(th);
        W[2][1] = 1.0;
    } else {
        W[0][0] = 1.0;
        W[1][1] = 1.0;
    }
}

// ------------------------------------------------------------------------------ small dense helpers
void matmul(const double* A, const double* B, double* C, int n, int k, int m) {   // C = A B
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < m; ++j) {
            double s = 0.0;
            for (int l = 0; l < k; ++l) s += A[i * k + l] * B[l * m + j];
            C[i * m + j] = s;
        }
}
bool spd_inverse(double* A, double* Ai, int n) {   // Gauss-Jordan, SPD (no pivoting)
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) Ai[i * n + j] = i == j ? 1.0 : 0.0;
    for (int c = 0; c < n; ++c) {
        const double piv = A[c * n + c];
        if (!(piv > 0.0)) return false;
        const double rp = 1.0 / piv;
        for (int j = 0; j < n; ++j) { A[c * n + j] *= rp; Ai[c * n + j] *= rp; }
        for (int i = 0; i < n; ++i) {
            if (i == c) continue;
            const double f = A[i * n + c];
            for (int j = 0; j < n; ++j) { A[i * n + j] -= f * A[c * n + j]; Ai[i * n + j] -= f * Ai[c * n + j]; }
        }
    }
    return true;
}

// ------------------------------------------------------------------------------ one instance
struct Instance {
    const Problem& P;
    int H, nx, nu, nb, n;
    std::vector<double> x, u, pi, ll, lu;   // acados memory: iterate + multipliers
    std::vector<double> A, B, F;            // linearisation
    std::vector<double> hd, g, yref, lbw, ubw, w;
    std::vector<double> Pm, pv, Km, kv, tmp;
    int qp_iters = 0;

    explicit Instance(const Problem& p) : P(p), H(p.H), nx(p.nx), nu(p.nu), nb(p.nx + p.nu), n(p.H * (p.nx + p.nu)) {
        A.resize((size_t)H * nx * nx);
        B.resize((size_t)H * nx * nu);
        F.resize((size_t)H * nx);
        hd.resize(n); g.resize(n); yref.resize(n); lbw.resize(n); ubw.resize(n); w.resize(n);
        Pm.resize((size_t)(H + 1) * nx * nx); pv.resize((size_t)(H + 1) * nx);
        Km.resize((size_t)H * nu * nx); kv.resize((size_t)H * nu);
        const double sc = P.cost_scaling ? P.dt : 1.0;
        for (int k = 0; k < H; ++k) {
            for (int a = 0; a < nu; ++a) hd[k * nb + a] = sc * P.r[a];
            for (int i = 0; i < nx; ++i) hd[k * nb + nu + i] = (k == H - 1 ? 1.0 : sc) * P.q[i];
        }
    }
    int ui(int k) const { return k * nb; }            // u_k
    int xi(int k) const { return (k - 1) * nb + nu; } // x_k, k >= 1

    void pack(const double* xs, const double* us, double* out) const {
        for (int k = 0; k < H; ++k) {
            for (int a = 0; a < nu; ++a) out[ui(k) + a] = us[k * nu + a];
            for (int i = 0; i < nx; ++i) out[xi(k + 1) + i] = xs[(k + 1) * nx + i];
        }
    }

    void linearize(const double* xs, const double* us) {
        std::vector<double> J((size_t)nx * nb);
        for (int k = 0; k < H; ++k) {
            rk4(P, &xs[k * nx], &us[k * nu], &F[k * nx], J.data());
            for (int i = 0; i < nx; ++i) {
                for (int j = 0; j < nx; ++j) A[(size_t)k * nx * nx + i * nx + j] = J[i * nb + j];
                for (int a = 0; a < nu; ++a) B[(size_t)k * nx * nu + i * nu + a] = J[i * nb + nx + a];
            }
        }
    }

    // Newton system of the IPM by Riccati: min 1/2 d'(Hd+Sig)d + rhs'd  s.t.
    // dx_{k+1} = A_k dx_k + B_k du_k + c_k, dx_0 = 0.  Returns dd and the dynamics multipliers dp.
    bool riccati(const double* Hs, const double* rhs, const double* c, double* dd, double* dp) {
        double* Pn = &Pm[(size_t)H * nx * nx];
        double* pn = &pv[(size_t)H * nx];
        for (int i = 0; i < nx; ++i) {
            for (int j = 0; j < nx; ++j) Pn[i * nx + j] = i == j ? Hs[xi(H) + i] : 0.0;
            pn[i] = rhs[xi(H) + i];
        }
        double PA[MX * MX], PB[MX * MU], t[MX], Huu[MU * MU], Hui[MU * MU], Hux[MU * MX], hu[MU];
        for (int k = H - 1; k >= 0; --k) {
            const double* Ak = &A[(size_t)k * nx * nx];
            const double* Bk = &B[(size_t)k * nx * nu];
            const double* P1 = &Pm[(size_t)(k + 1) * nx * nx];
            const double* p1 = &pv[(size_t)(k + 1) * nx];
            matmul(P1, Ak, PA, nx, nx, nx);
            matmul(P1, Bk, PB, nx, nx, nu);
            for (int i = 0; i < nx; ++i) {   // t = P c + p
                double s = p1[i];
                for (int j = 0; j < nx; ++j) s += P1[i * nx + j] * c[k * nx + j];
                t[i] = s;
            }
            for (int a = 0; a < nu; ++a) {
                for (int b = 0; b < nu; ++b) {
                    double s = a == b ? Hs[ui(k) + a] : 0.0;
                    for (int i = 0; i < nx; ++i) s += Bk[i * nu + a] * PB[i * nu + b];
                    Huu[a * nu + b] = s;
                }
                for (int j = 0; j < nx; ++j) {
                    double s = 0.0;
                    for (int i = 0; i < nx; ++i) s += Bk[i * nu + a] * PA[i * nx + j];
                    Hux[a * nx + j] = s;
                }
                double s = rhs[ui(k) + a];
                for (int i = 0; i < nx; ++i) s += Bk[i * nu + a] * t[i];
                hu[a] = s;
            }
            if (!spd_inverse(Huu, Hui, nu)) return false;
            double* Kk = &Km[(size_t)k * nu * nx];
            double* kk = &kv[(size_t)k * nu];
            for (int a = 0; a < nu; ++a) {
                for (int j = 0; j < nx; ++j) {
                    double s = 0.0;
                    for (int b = 0; b < nu; ++b) s -= Hui[a * nu + b] * Hux[b * nx + j];
                    Kk[a * nx + j] = s;
                }
                double s = 0.0;
                for (int b = 0; b < nu; ++b) s -= Hui[a * nu + b] * hu[b];
                kk[a] = s;
            }
            if (k == 0) break;   // P_0 is not needed (dx_0 = 0)
            double* P0 = &Pm[(size_t)k * nx * nx];
            double* p0 = &pv[(size_t)k * nx];
            for (int i = 0; i < nx; ++i) {
                for (int j = 0; j < nx; ++j) {
                    double s = i == j ? Hs[xi(k) + i] : 0.0;
                    for (int l = 0; l < nx; ++l) s += Ak[l * nx + i] * PA[l * nx + j];
                    for (int a = 0; a < nu; ++a) s += Hux[a * nx + i] * Kk[a * nx + j];
                    P0[i * nx + j] = s;
                }
                double s = rhs[xi(k) + i];
                for (int l = 0; l < nx; ++l) s += Ak[l * nx + i] * t[l];
                for (int a = 0; a < nu; ++a) s += Hux[a * nx + i] * kk[a];
                p0[i] = s;
            }
        }
        double dx[MX], dxn[MX];
        std::fill(dx, dx + nx, 0.0);
        for (int k = 0; k < H; ++k) {
            const double* Ak = &A[(size_t)k * nx * nx];
            const double* Bk = &B[(size_t)k * nx * nu];
            double du[MU];
            for (int a = 0; a < nu; ++a) {
                double s = kv[(size_t)k * nu + a];
                for (int j = 0; j < nx; ++j) s += Km[(size_t)k * nu * nx + a * nx + j] * dx[j];
                du[a] = s;
                dd[ui(k) + a] = s;
            }
            for (int i = 0; i < nx; ++i) {
                double s = c[k * nx + i];
                for (int j = 0; j < nx; ++j) s += Ak[i * nx + j] * dx[j];
                for (int a = 0; a < nu; ++a) s += Bk[i * nu + a] * du[a];
                dxn[i] = s;
                dd[xi(k + 1) + i] = s;
            }
            const double* P1 = &Pm[(size_t)(k + 1) * nx * nx];
            const double* p1 = &pv[(size_t)(k + 1) * nx];
            for (int i = 0; i < nx; ++i) {   // pi_k = -(P_{k+1} dx_{k+1} + p_{k+1})
                double s = p1[i];
                for (int j = 0; j < nx; ++j) s += P1[i * nx + j] * dxn[j];
                dp[k * nx + i] = -s;
            }
            std::copy(dxn, dxn + nx, dx);
        }
        return true;
    }

    // C d - r and C' pi in the d layout (DenseQP.build: rows x_{k+1} - A_k x_k - B_k u_k)
    void cmul(const double* d, const double* r, double* out) const {
        for (int k = 0; k < H; ++k)
            for (int i = 0; i < nx; ++i) {
                double s = d[xi(k + 1) + i] - r[k * nx + i];
                for (int a = 0; a < nu; ++a) s -= B[(size_t)k * nx * nu + i * nu + a] * d[ui(k) + a];
                if (k > 0)
                    for (int j = 0; j < nx; ++j) s -= A[(size_t)k * nx * nx + i * nx + j] * d[xi(k) + j];
                out[k * nx + i] = s;
            }
    }
    void ctmul(const double* p, double* out) const {
        std::fill(out, out + n, 0.0);
        for (int k = 0; k < H; ++k)
            for (int i = 0; i < nx; ++i) {
                const double v = p[k * nx + i];
                out[xi(k + 1) + i] += v;
                for (int a = 0; a < nu; ++a) out[ui(k) + a] -= B[(size_t)k * nx * nu + i * nu + a] * v;
                if (k > 0)
                    for (int j = 0; j < nx; ++j) out[xi(k) + j] -= A[(size_t)k * nx * nx + i * nx + j] * v;
            }
    }

    // Mehrotra predictor-corrector primal-dual IPM (DenseQP.solve), Newton steps by Riccati
    int qp(const double* r, const double* cr, const double* lb, const double* ub, std::vector<double>& d,
           std::vector<double>& pq, std::vector<double>& sl, std::vector<double>& su, std::vector<double>& l1,
           std::vector<double>& l2) {
        const int m = H * nx;
        d.assign(n, 0.0);
        pq.assign(m, 0.0);
        sl.resize(n); su.resize(n); l1.resize(n); l2.resize(n);
        for (int i = 0; i < n; ++i) {
            sl[i] = std::max(d[i] - lb[i], 1e-2);
            su[i] = std::max(ub[i] - d[i], 1e-2);
            l1[i] = 1.0 / sl[i];
            l2[i] = 1.0 / su[i];
        }
        const double nc = 2.0 * n;
        std::vector<double> rd(n), rp(m), rl(n), ru(n), ctp(n), Hs(n), rhs(n), cc(m), dd(n), dp(m);
        std::vector<double> dsl(n), dsu(n), dll(n), dlu(n), rml(n), rmu(n);
        for (int it = 0; it < P.qp_max_iter; ++it) {
            qp_iters = it;
            ctmul(pq.data(), ctp.data());
            cmul(d.data(), r, rp.data());
            double mrd = 0, mrp = 0, mlu = 0, mu = 0;
            for (int i = 0; i < n; ++i) {
                rd[i] = hd[i] * d[i] + g[i] + ctp[i] - l1[i] + l2[i];
                rl[i] = d[i] - lb[i] - sl[i];
                ru[i] = ub[i] - d[i] - su[i];
                mu += l1[i] * sl[i] + l2[i] * su[i];
                mrd = std::max(mrd, std::fabs(rd[i]));
                mlu = std::max(mlu, std::max(std::fabs(rl[i]), std::fabs(ru[i])));
            }
            for (int i = 0; i < m; ++i) mrp = std::max(mrp, std::fabs(rp[i]));
            mu /= nc;
            if (!(mu == mu)) return 1;
            if (mrd <= P.qp_tol && mrp <= P.qp_tol && mlu <= P.qp_tol && mu <= P.qp_tol) return 0;
            for (int i = 0; i < n; ++i) Hs[i] = hd[i] + l1[i] / sl[i] + l2[i] / su[i];
            for (int i = 0; i < m; ++i) cc[i] = -rp[i];
            auto newton = [&](const double* rml, const double* rmu) {
                for (int i = 0; i < n; ++i) rhs[i] = rd[i] + (rml[i] + l1[i] * rl[i]) / sl[i] - (rmu[i] + l2[i] * ru[i]) / su[i];
                if (!riccati(Hs.data(), rhs.data(), cc.data(), dd.data(), dp.data())) return false;
                for (int i = 0; i < n; ++i) {
                    dsl[i] = dd[i] + rl[i];
                    dsu[i] = -dd[i] + ru[i];
                    dll[i] = (-rml[i] - l1[i] * dsl[i]) / sl[i];
                    dlu[i] = (-rmu[i] - l2[i] * dsu[i]) / su[i];
                }
                return true;
            };
            auto step_len = [&]() {
                double a = 1.0;
                for (int i = 0; i < n; ++i) {
                    if (dsl[i] < 0) a = std::min(a, -sl[i] / dsl[i]);
                    if (dsu[i] < 0) a = std::min(a, -su[i] / dsu[i]);
                    if (dll[i] < 0) a = std::min(a, -l1[i] / dll[i]);
                    if (dlu[i] < 0) a = std::min(a, -l2[i] / dlu[i]);
                }
                return a;
            };
            for (int i = 0; i < n; ++i) { rml[i] = l1[i] * sl[i]; rmu[i] = l2[i] * su[i]; }
            if (!newton(rml.data(), rmu.data())) return 1;
            const double aa = step_len();
            double mua = 0.0;
            for (int i = 0; i < n; ++i)
                mua += (l1[i] + aa * dll[i]) * (sl[i] + aa * dsl[i]) + (l2[i] + aa * dlu[i]) * (su[i] + aa * dsu[i]);
            mua /= nc;
            const double sig = std::pow(mua / mu, 3);
            for (int i = 0; i < n; ++i) {
                rml[i] = l1[i] * sl[i] + dll[i] * dsl[i] - sig * mu;
                rmu[i] = l2[i] * su[i] + dlu[i] * dsu[i] - sig * mu;
            }
            if (!newton(rml.data(), rmu.data())) return 1;
            const double a = std::min(1.0, 0.995 * step_len());
            for (int i = 0; i < n; ++i) {
                d[i] += a * dd[i]; sl[i] += a * dsl[i]; su[i] += a * dsu[i]; l1[i] += a * dll[i]; l2[i] += a * dlu[i];
            }
            for (int i = 0; i < m; ++i) pq[i] += a * dp[i];
            for (int i = 0; i < n; ++i)
                if (!std::isfinite(d[i])) return 1;
        }
        qp_iters = P.qp_max_iter;
        return 2;
    }

    // tightening from the previous solution (gpmpc/gpmpc.py:425-498): t (H+1) x nb
    void tightening(const double* xs, const double* us, double* t) const {
        std::fill(t, t + (size_t)(H + 1) * nb, 0.0);
        double cov[MX * MX] = {0}, T1[MX * MX], cu[MU * MX];
        std::vector<double> scratch;
        auto record = [&](int k) {
            for (int i = 0; i < nx; ++i) t[(size_t)k * nb + i] = P.icdf * std::sqrt(std::max(cov[i * nx + i], 0.0));
            if (k == H) return;
            for (int a = 0; a < nu; ++a) {   // sqrt(diag K cov K')
                double s = 0.0;
                for (int i = 0; i < nx; ++i)
                    for (int j = 0; j < nx; ++j) s += P.K[a * nx + i] * cov[i * nx + j] * P.K[a * nx + j];
                t[(size_t)k * nb + nx + a] = P.icdf * std::sqrt(std::max(s, 0.0));
            }
        };
        double Acl[MX * MX];   // A_d + B_d K (the four-term update of gpmpc.py:489-495)
        for (int i = 0; i < nx; ++i)
            for (int j = 0; j < nx; ++j) {
                double s = P.Ad[i * nx + j];
                for (int a = 0; a < nu; ++a) s += P.Bd[i * nu + a] * P.K[a * nx + j];
                Acl[i * nx + j] = s;
            }
        (void)cu;
        for (int k = 0; k < H; ++k) {
            record(k);
            double z[MB], vg[MG] = {0, 0, 0, 0}, W[MX][MG];
            std::copy(&xs[k * nx], &xs[k * nx] + nx, z);
            std::copy(&us[k * nu], &us[k * nu] + nu, z + nx);
            for (int g = 0; g < P.ngp; ++g) {
                double zi[3];
                for (int q = 0; q < P.gp[g].d; ++q) zi[q] = z[P.gp[g].var_idx[q]];
                vg[g] = P.gp[g].var(zi, scratch);
            }
            var_weights(P, &xs[k * nx], W);
            matmul(Acl, cov, T1, nx, nx, nx);
            for (int i = 0; i < nx; ++i)
                for (int j = 0; j < nx; ++j) {
                    double s = 0.0;
                    for (int l = 0; l < nx; ++l) s += T1[i * nx + l] * Acl[j * nx + l];
                    cov[i * nx + j] = s;
                }
            for (int q = 0; q < P.n_unc; ++q) {   // Bd cov_d Bd', cov_d = W (var + noise) dt^2
                double s = 0.0;
                for (int g = 0; g < P.ngp; ++g) s += W[q][g] * (vg[g] + P.gp[g].sn2);
                cov[P.unc[q] * nx + P.unc[q]] += s * P.dt * P.dt;
            }
        }
        record(H);
    }

    bool trace = false;   // diagnostic: per-iteration NLP residuals to stderr

    int step(const double* x0, int tstep, bool has_prev, double* u0, int& sqp_iter, int& qp_total) {
        std::vector<double> t((size_t)(H + 1) * nb, 0.0);
        if (P.tighten && has_prev) tightening(x.data(), u.data(), t.data());
        // bounds and reference in the d layout
        for (int k = 0; k < H; ++k) {
            for (int a = 0; a < nu; ++a) {
                lbw[ui(k) + a] = P.ulo[a] + t[(size_t)k * nb + nx + a] - P.uh;
                ubw[ui(k) + a] = P.uhi[a] - t[(size_t)k * nb + nx + a] + P.uh;
                yref[ui(k) + a] = P.ueq[a];
            }
            const int tr = (tstep + k + 1) % P.traj_len;
            for (int i = 0; i < nx; ++i) {
                lbw[xi(k + 1) + i] = P.xlo[i] + t[(size_t)(k + 1) * nb + i] - P.uh;
                ubw[xi(k + 1) + i] = P.xhi[i] - t[(size_t)(k + 1) * nb + i] + P.uh;
                yref[xi(k + 1) + i] = P.traj[(size_t)tr * nx + i];
            }
        }
        std::vector<double> xs = x, us = u, r((size_t)H * nx), cr((size_t)H * nx), lb(n), ub(n), ctp(n);
        std::vector<double> d, pq, sl, su, l1, l2;
        int status = kMaxIter, it = 0;
        qp_total = 0;
        // stage-0 state rows (gpmpc/gpmpc.py:288,296,309-310; gpmpc/mpc.py:141,145,157-158): x_0 is
        // pinned to obs, so they only decide feasibility; an obs outside the box by more than the
        // inequality tolerance is an infeasible QP (acados status 4)
        double v0 = 0.0;
        for (int i = 0; i < nx; ++i) {
            const double e = std::max(P.xlo[i] - P.uh - x0[i], x0[i] - P.xhi[i] - P.uh);
            v0 = (e == e && v0 == v0) ? std::max(v0, e) : NAN;
        }
        const bool x0_ok = v0 <= P.tol;
        if (!x0_ok) status = kQPFailure;
        for (it = 0; x0_ok && it <= P.max_iter; ++it) {
            linearize(xs.data(), us.data());
            pack(xs.data(), us.data(), w.data());
            for (int i = 0; i < n; ++i) g[i] = hd[i] * (w[i] - yref[i]);
            ctmul(pi.data(), ctp.data());
            double rs = 0, re = 0, ri = 0, rc = 0;
            for (int i = 0; i < n; ++i) {
                rs = std::max(rs, std::fabs(g[i] + ctp[i] - ll[i] + lu[i]));
                ri = std::max(ri, std::max(std::max(lbw[i] - w[i], w[i] - ubw[i]), 0.0));
                rc = std::max(rc, std::max(std::fabs(ll[i] * (w[i] - lbw[i])), std::fabs(lu[i] * (ubw[i] - w[i]))));
            }
            for (int k = 0; k < H; ++k)
                for (int i = 0; i < nx; ++i) re = std::max(re, std::fabs(F[k * nx + i] - xs[(k + 1) * nx + i]));
            for (int i = 0; i < nx; ++i) {
                ri = std::max(ri, std::fabs(x0[i] - xs[i]));
                ri = std::max(ri, std::max(P.xlo[i] - P.uh - xs[i], xs[i] - P.xhi[i] - P.uh));
            }
            if (trace) std::fprintf(stderr, "  sqp %d: stat %.3e eq %.3e ineq %.3e comp %.3e (qp iters so far %d)\n", it, rs, re, ri, rc, qp_total);
            if (!(rs == rs && re == re && ri == ri && rc == rc)) { status = kNaN; break; }
            if (rs <= P.tol && re <= P.tol && ri <= P.tol && rc <= P.tol) { status = kSuccess; break; }
            if (it == P.max_iter) { status = kMaxIter; break; }
            // QP in the step: r_0 = c_0 + A_0 e0, r_k = c_k
            for (int k = 0; k < H; ++k)
                for (int i = 0; i < nx; ++i) {
                    double s = F[k * nx + i] - xs[(k + 1) * nx + i];
                    if (k == 0)
                        for (int j = 0; j < nx; ++j) s += A[i * nx + j] * (x0[j] - xs[j]);
                    r[k * nx + i] = s;
                }
            for (int i = 0; i < n; ++i) { lb[i] = lbw[i] - w[i]; ub[i] = ubw[i] - w[i]; }
            const int qst = qp(r.data(), cr.data(), lb.data(), ub.data(), d, pq, sl, su, l1, l2);
            qp_total += qp_iters;
            if (qst == 1) { status = kQPFailure; break; }
            for (int i = 0; i < nx; ++i) xs[i] = x0[i];
            for (int k = 0; k < H; ++k) {
                for (int a = 0; a < nu; ++a) us[k * nu + a] += d[ui(k) + a];
                for (int i = 0; i < nx; ++i) xs[(k + 1) * nx + i] += d[xi(k + 1) + i];
            }
            pi = pq;
            ll = l1;
            lu = l2;
            bool fin = true;
            for (double v : xs) fin = fin && std::isfinite(v);
            for (double v : us) fin = fin && std::isfinite(v);
            if (!fin) { status = kNaN; break; }
        }
        const bool good = status == kSuccess || status == kMaxIter;
        if (good) {
            x = xs;
            u = us;
        } else {   // a failed solve keeps the previous iterate and restarts the multipliers
            std::fill(pi.begin(), pi.end(), 0.0);
            std::fill(ll.begin(), ll.end(), 0.0);
            std::fill(lu.begin(), lu.end(), 0.0);
        }
        sqp_iter = it;
        for (int a = 0; a < nu; ++a) u0[a] = u[a];
        return status;
    }
};

struct Handle {
    Problem P;
};

}  // namespace

extern "C" {

void* cpuref_create(int model, int H, const double* params, int n_params, double dt, const double* x_lo,
                    const double* x_hi, const double* u_lo, const double* u_hi, const double* q, const double* r,
                    const double* u_eq, double uh, int cost_scaling) {
    if (model < 0 || model > 2 || H < 1) return nullptr;
    auto* h = new Handle();
    Problem& P = h->P;
    P.model = model;
    P.H = H;
    P.nx = model == kQuad2D ? 6 : model == kQuad3D ? 12 : 4;
    P.nu = model == kQuad2D ? 2 : model == kQuad3D ? 4 : 1;
    P.ngp = model == kQuad3D ? 3 : 2;
    for (int i = 0; i < n_params && i < 16; ++i) P.p[i] = params[i];
    P.dt = dt;
    P.uh = uh;
    P.cost_scaling = cost_scaling != 0;
    for (int i = 0; i < P.nx; ++i) { P.xlo[i] = x_lo[i]; P.xhi[i] = x_hi[i]; P.q[i] = q[i]; }
    for (int a = 0; a < P.nu; ++a) { P.ulo[a] = u_lo[a]; P.uhi[a] = u_hi[a]; P.r[a] = r[a]; P.ueq[a] = u_eq[a]; }
    return h;
}

void cpuref_destroy(void* h) { delete static_cast<Handle*>(h); }

void cpuref_set_options(void* h, int max_iter, double tol, int qp_max_iter, double qp_tol) {
    Problem& P = static_cast<Handle*>(h)->P;
    P.max_iter = max_iter;
    P.tol = tol;
    P.qp_max_iter = qp_max_iter;
    P.qp_tol = qp_tol;
}

// X [n][d], alpha [n], L lower Cholesky of K [n][n] (NULL: no variance); in_idx / var_idx: the
// GP's input columns of z = [x; u] for the dynamics and for the tightening variance.
int cpuref_set_gp(void* h, int g, int n, int d, const double* X, const double* alpha, const double* L, double ell,
                  double sf2, double sn2, const int* in_idx, const int* var_idx) {
    Problem& P = static_cast<Handle*>(h)->P;
    if (g < 0 || g >= P.ngp || d < 1 || d > 3 || n < 1) return -1;
    GP& G = P.gp[g];
    G.n = n;
    G.d = d;
    G.nv = 0;
    G.Xv.clear();
    G.X.assign(X, X + (size_t)n * d);
    G.alpha.assign(alpha, alpha + n);
    if (L) G.L.assign(L, L + (size_t)n * n); else G.L.clear();
    G.ell = ell;
    G.sf2 = sf2;
    G.sn2 = sn2;
    for (int k = 0; k < d; ++k) { G.in_idx[k] = in_idx[k]; G.var_idx[k] = var_idx[k]; }
    return 0;
}

// FITC: the variance of GP g runs over its own rows Xv [nv][d] (the training set) with L the
// Cholesky factor of K(Xv, Xv) [nv][nv], while cpuref_set_gp's X / alpha are the inducing rows and
// weights of the mean (gpmpc/gpmpc.py:175-187 mean, :441-445 exact variance).
int cpuref_set_gp_var(void* h, int g, int nv, const double* Xv, const double* L) {
    Problem& P = static_cast<Handle*>(h)->P;
    if (g < 0 || g >= P.ngp || nv < 1 || !Xv || !L) return -1;
    GP& G = P.gp[g];
    if (G.d < 1) return -1;
    G.nv = nv;
    G.Xv.assign(Xv, Xv + (size_t)nv * G.d);
    G.L.assign(L, L + (size_t)nv * nv);
    return 0;
}

// LOVE variance of GP g: R [m][r] row-major over the variance rows (m = nv, or n for an exact GP),
// R R^T ~ (K + sn2 I)^-1 (gpmpc/gp.py love_root); R = NULL restores the exact variance.
int cpuref_set_gp_var_root(void* h, int g, int m, int r, const double* R) {
    Problem& P = static_cast<Handle*>(h)->P;
    if (g < 0 || g >= P.ngp) return -1;
    GP& G = P.gp[g];
    if (!R) {
        G.R.clear();
        G.rr = 0;
        return 0;
    }
    if (m != (G.Xv.empty() ? G.n : G.nv) || r < 1) return -1;
    G.R.assign(R, R + (size_t)m * r);
    G.rr = r;
    return 0;
}

// Tightening variance of GP g (likelihood noise included) at P points Z [P][d] -> out [P].
int cpuref_gp_var(void* h, int g, int P, const double* Z, double* out) {
    const Problem& Pr = static_cast<Handle*>(h)->P;
    if (g < 0 || g >= Pr.ngp || P < 0) return -1;
    const GP& G = Pr.gp[g];
    if (G.L.empty() && G.rr == 0) return -1;
    std::vector<double> v;
    for (int p = 0; p < P; ++p) out[p] = G.var(Z + (size_t)p * G.d, v);
    return 0;
}

void cpuref_use_gp(void* h, int on) { static_cast<Handle*>(h)->P.use_gp = on != 0; }

void cpuref_set_tightening(void* h, int on, double icdf, const double* Ad, const double* Bd, const double* K,
                           const int* unc, int n_unc) {
    Problem& P = static_cast<Handle*>(h)->P;
    P.tighten = on != 0;
    if (!on) return;
    P.icdf = icdf;
    std::copy(Ad, Ad + P.nx * P.nx, P.Ad);
    std::copy(Bd, Bd + P.nx * P.nu, P.Bd);
    std::copy(K, K + P.nu * P.nx, P.K);
    P.n_unc = n_unc;
    std::copy(unc, unc + n_unc, P.unc);
}

// traj: [L][nx] (time-major)
void cpuref_set_reference(void* h, const double* traj, int L) {
    Problem& P = static_cast<Handle*>(h)->P;
    P.traj.assign(traj, traj + (size_t)L * P.nx);
    P.traj_len = L;
}

// One closed-loop control step for B instances (OpenMP, one instance per thread).  State per
// instance (acados memory, updated in place): x [H+1][nx], u [H][nu], pi [H][nx], ll/lu [H*(nx+nu)]
// in the d layout, has_prev.  Outputs u0 [B][nu], status, sqp_iter, qp_iter [B].
int cpuref_step(void* h, int B, const double* x0, const int* tstep, double* xs, double* us, double* pi, double* ll,
                double* lu, int* has_prev, double* u0, int* status, int* sqp_iter, int* qp_iter, int threads) {
    const Problem& P = static_cast<Handle*>(h)->P;
    const int H = P.H, nx = P.nx, nu = P.nu, n = H * (nx + nu);
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel
    {
        Instance I(P);
#pragma omp for schedule(dynamic, 1)
        for (int b = 0; b < B; ++b) {
            I.x.assign(xs + (size_t)b * (H + 1) * nx, xs + (size_t)(b + 1) * (H + 1) * nx);
            I.u.assign(us + (size_t)b * H * nu, us + (size_t)(b + 1) * H * nu);
            I.pi.assign(pi + (size_t)b * H * nx, pi + (size_t)(b + 1) * H * nx);
            I.ll.assign(ll + (size_t)b * n, ll + (size_t)(b + 1) * n);
            I.lu.assign(lu + (size_t)b * n, lu + (size_t)(b + 1) * n);
            int si = 0, qi = 0;
            const char* tr = std::getenv("CPUREF_TRACE");   // instance index to trace
            I.trace = tr != nullptr && std::atoi(tr) == b;
            status[b] = I.step(x0 + (size_t)b * nx, tstep[b], has_prev[b] != 0, u0 + (size_t)b * nu, si, qi);
            sqp_iter[b] = si;
            qp_iter[b] = qi;
            has_prev[b] = (status[b] == kSuccess || status[b] == kMaxIter) ? 1 : 0;
            std::copy(I.x.begin(), I.x.end(), xs + (size_t)b * (H + 1) * nx);
            std::copy(I.u.begin(), I.u.end(), us + (size_t)b * H * nu);
            std::copy(I.pi.begin(), I.pi.end(), pi + (size_t)b * H * nx);
            std::copy(I.ll.begin(), I.ll.end(), ll + (size_t)b * n);
            std::copy(I.lu.begin(), I.lu.end(), lu + (size_t)b * n);
        }
    }
    return 0;
}

}  // extern "C"
