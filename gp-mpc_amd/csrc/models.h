// Device-side model definitions: GP-augmented continuous dynamics f(x,u) and its
// tangent map (forward-mode derivative), the GP input maps, and the tightening weights.
//
// Reference: f = f_prior(x,u) + res_dyn(GP means)  gpmpc/gpmpc.py:171-199 (quad3d);
// tightening weights gpmpc/gpmpc.py:447-469; Bd gpmpc/gpmpc.py:68-69.
// Prior parameter vectors: see gpmpc/models.py ModelSpec.param_vector.
#pragma once
#include "gpmpc_common.h"

namespace gpmpc {

template <int ID> struct Model;

// ---------------------------------------------------------------------------- quad2d
// x = [px, vx, pz, vz, th, w], u = [T, P]; p = [a, b, f, h, l, g]
template <> struct Model<kQuad2D> {
    static constexpr int NX = 6, NU = 2, NB = 8, NGP = 2, NUNC = 3;
    static constexpr int gp_dim[NGP] = {1, 3};
    static constexpr int gp_src[NGP][3] = {{NX + 0, 0, 0}, {4, 5, NX + 1}};
    static constexpr int var_src[NGP][3] = {{NX + 0, 0, 0}, {4, 5, NX + 1}};
    static constexpr bool gp_state_dep[NGP] = {false, true};
    static constexpr int unc[NUNC] = {1, 3, 5};

    __device__ static void f(const double* p, const double* x, const double* u, const double* gm, double* o) {
        double s, c;
        sincos(x[4], &s, &c);
        const double acc = p[0] * u[0] + p[1] + gm[0];
        o[0] = x[1];
        o[1] = acc * s;
        o[2] = x[3];
        o[3] = acc * c - p[5];
        o[4] = x[5];
        o[5] = p[2] * x[4] + p[3] * x[5] + p[4] * u[1] + gm[1];
    }

    // dk = df/dw for CB columns j0.. of the stage variables, given V = dx/dw on those
    // columns, the GP means gm and the GP input-gradients gg.
    template <int CB>
    __device__ static void tangent(const double* p, const double* x, const double* u, const double* gm,
                                   const double (*gg)[3], const double (&V)[NX][CB], int j0, double (&dk)[NX][CB]) {
        double s, c;
        sincos(x[4], &s, &c);
        const double acc = p[0] * u[0] + p[1] + gm[0];
#pragma unroll
        for (int j = 0; j < CB; ++j) {
            const int col = j0 + j;
            const double dmT = gg[0][0] * (col == NX + 0 ? 1.0 : 0.0);
            const double dmP = gg[1][0] * V[4][j] + gg[1][1] * V[5][j] + gg[1][2] * (col == NX + 1 ? 1.0 : 0.0);
            const double dacc = p[0] * (col == NX + 0 ? 1.0 : 0.0) + dmT;
            dk[0][j] = V[1][j];
            dk[1][j] = dacc * s + acc * c * V[4][j];
            dk[2][j] = V[3][j];
            dk[3][j] = dacc * c - acc * s * V[4][j];
            dk[4][j] = V[5][j];
            dk[5][j] = p[2] * V[4][j] + p[3] * V[5][j] + p[4] * (col == NX + 1 ? 1.0 : 0.0) + dmP;
        }
    }

    // cov_d[j] = sum_g W[j][g] * var_g   (quad2d analogue of gpmpc.py:447-457)
    __device__ static void var_weights(const double* x, const double* u, double (*W)[NGP]) {
        double s, c;
        sincos(x[4], &s, &c);
        W[0][0] = s * s; W[0][1] = 0.0;
        W[1][0] = c * c; W[1][1] = 0.0;
        W[2][0] = 0.0;   W[2][1] = 1.0;
    }
};

// ---------------------------------------------------------------------------- quad3d
// x = [px,vx,py,vy,pz,vz,phi,th,psi,dphi,dth,dpsi], u = [T,R,P,Y]; p = [a,b,c,d,e,f,h,l,g]
template <> struct Model<kQuad3D> {
    static constexpr int NX = 12, NU = 4, NB = 16, NGP = 3, NUNC = 5;
    static constexpr int gp_dim[NGP] = {1, 3, 3};
    static constexpr int gp_src[NGP][3] = {{NX + 0, 0, 0}, {6, 9, NX + 1}, {7, 10, NX + 2}};  // gpmpc.py:173
    // gpmpc.py:437-444 evaluates the variance at z[:, gp_idx] with gp_idx = [[0],[1,2,3],[4,5,6]]
    static constexpr int var_src[NGP][3] = {{0, 0, 0}, {1, 2, 3}, {4, 5, 6}};
    static constexpr bool gp_state_dep[NGP] = {false, true, true};
    static constexpr int unc[NUNC] = {1, 3, 5, 9, 10};  // gpmpc.py:68

    __device__ static void f(const double* p, const double* x, const double* u, const double* gm, double* o) {
        double sf, cf, st, ct, sp, cp;
        sincos(x[6], &sf, &cf);
        sincos(x[7], &st, &ct);
        sincos(x[8], &sp, &cp);
        const double A = p[0] * u[0] + p[1];
        const double mT = gm[0];
        o[0] = x[1];
        o[1] = A * (cf * st * cp + sf * sp) + mT * cf * st;
        o[2] = x[3];
        o[3] = A * (cf * st * sp - sf * cp) - mT * sf;
        o[4] = x[5];
        o[5] = A * cf * ct - p[8] + mT * cf * ct;
        o[6] = x[9];
        o[7] = x[10];
        o[8] = x[11];
        o[9] = p[2] * x[6] + p[3] * x[9] + p[4] * u[1] + gm[1];
        o[10] = p[5] * x[7] + p[6] * x[10] + p[7] * u[2] + gm[2];
        o[11] = p[2] * x[8] + p[3] * x[11] + p[4] * u[3];
    }

    template <int CB>
    __device__ static void tangent(const double* p, const double* x, const double* u, const double* gm,
                                   const double (*gg)[3], const double (&V)[NX][CB], int j0, double (&dk)[NX][CB]) {
        double sf, cf, st, ct, sp, cp;
        sincos(x[6], &sf, &cf);
        sincos(x[7], &st, &ct);
        sincos(x[8], &sp, &cp);
        const double A = p[0] * u[0] + p[1];
        const double mT = gm[0];
        const double gx = cf * st * cp + sf * sp, gy = cf * st * sp - sf * cp, gz = cf * ct;
        const double gx_f = -sf * st * cp + cf * sp, gx_t = cf * ct * cp, gx_p = -cf * st * sp + sf * cp;
        const double gy_f = -sf * st * sp - cf * cp, gy_t = cf * ct * sp, gy_p = cf * st * cp + sf * sp;
        const double gz_f = -sf * ct, gz_t = -cf * st;
#pragma unroll
        for (int j = 0; j < CB; ++j) {
            const int col = j0 + j;
            const double e12 = col == NX + 0 ? 1.0 : 0.0, e13 = col == NX + 1 ? 1.0 : 0.0;
            const double e14 = col == NX + 2 ? 1.0 : 0.0, e15 = col == NX + 3 ? 1.0 : 0.0;
            const double df = V[6][j], dt = V[7][j], dp = V[8][j];
            const double dA = p[0] * e12;
            const double dmT = gg[0][0] * e12;
            const double dmR = gg[1][0] * V[6][j] + gg[1][1] * V[9][j] + gg[1][2] * e13;
            const double dmP = gg[2][0] * V[7][j] + gg[2][1] * V[10][j] + gg[2][2] * e14;
            dk[0][j] = V[1][j];
            dk[1][j] = dA * gx + A * (gx_f * df + gx_t * dt + gx_p * dp) + dmT * cf * st + mT * (-sf * st * df + cf * ct * dt);
            dk[2][j] = V[3][j];
            dk[3][j] = dA * gy + A * (gy_f * df + gy_t * dt + gy_p * dp) - dmT * sf - mT * cf * df;
            dk[4][j] = V[5][j];
            dk[5][j] = (dA + dmT) * gz + (A + mT) * (gz_f * df + gz_t * dt);
            dk[6][j] = V[9][j];
            dk[7][j] = V[10][j];
            dk[8][j] = V[11][j];
            dk[9][j] = p[2] * V[6][j] + p[3] * V[9][j] + p[4] * e13 + dmR;
            dk[10][j] = p[5] * V[7][j] + p[6] * V[10][j] + p[7] * e14 + dmP;
            dk[11][j] = p[2] * V[8][j] + p[3] * V[11][j] + p[4] * e15;
        }
    }

    // gpmpc.py:447-457, including cos(phi) * sin(theta)^2 on the first row (cos not squared)
    __device__ static void var_weights(const double* x, const double* u, double (*W)[NGP]) {
        double sf, cf, st, ct;
        sincos(x[6], &sf, &cf);
        sincos(x[7], &st, &ct);
#pragma unroll
        for (int j = 0; j < NUNC; ++j)
#pragma unroll
            for (int g = 0; g < NGP; ++g) W[j][g] = 0.0;
        W[0][0] = cf * st * st;
        W[1][0] = sf * sf;
        W[2][0] = (cf * ct) * (cf * ct);
        W[3][1] = 1.0;
        W[4][2] = 1.0;
    }
};

// ---------------------------------------------------------------------------- cartpole
// x = [px, vx, th, w], u = [F]; p = [m_c, m_p, l, g]  (gym cart-pole, l = half length)
template <> struct Model<kCartpole> {
    static constexpr int NX = 4, NU = 1, NB = 5, NGP = 2, NUNC = 2;
    static constexpr int gp_dim[NGP] = {3, 3};
    static constexpr int gp_src[NGP][3] = {{2, 3, NX}, {2, 3, NX}};
    static constexpr int var_src[NGP][3] = {{2, 3, NX}, {2, 3, NX}};
    static constexpr bool gp_state_dep[NGP] = {true, true};
    static constexpr int unc[NUNC] = {1, 3};

    struct Acc { double xa, tha, dxa[3], dtha[3]; };

    __device__ static Acc acc(const double* p, double th, double w, double F) {
        const double mc = p[0], mp = p[1], l = p[2], g = p[3];
        const double M = mc + mp;
        double s, c;
        sincos(th, &s, &c);
        const double tmp = (F + mp * l * w * w * s) / M;
        const double den = l * (4.0 / 3.0 - mp * c * c / M);
        const double num = g * s - c * tmp;
        Acc a;
        a.tha = num / den;
        const double k = mp * l / M;
        a.xa = tmp - k * a.tha * c;
        const double dtmp[3] = {mp * l * w * w * c / M, 2.0 * mp * l * w * s / M, 1.0 / M};
        const double dden[3] = {l * 2.0 * mp * c * s / M, 0.0, 0.0};
        const double dnum[3] = {g * c + s * tmp - c * dtmp[0], -c * dtmp[1], -c * dtmp[2]};
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            a.dtha[i] = (dnum[i] * den - num * dden[i]) / (den * den);
            a.dxa[i] = dtmp[i] - k * (a.dtha[i] * c - (i == 0 ? a.tha * s : 0.0));
        }
        return a;
    }

    __device__ static void f(const double* p, const double* x, const double* u, const double* gm, double* o) {
        const Acc a = acc(p, x[2], x[3], u[0]);
        o[0] = x[1];
        o[1] = a.xa + gm[0];
        o[2] = x[3];
        o[3] = a.tha + gm[1];
    }

    template <int CB>
    __device__ static void tangent(const double* p, const double* x, const double* u, const double* gm,
                                   const double (*gg)[3], const double (&V)[NX][CB], int j0, double (&dk)[NX][CB]) {
        const Acc a = acc(p, x[2], x[3], u[0]);
#pragma unroll
        for (int j = 0; j < CB; ++j) {
            const double e4 = (j0 + j) == NX ? 1.0 : 0.0;
            const double d0 = V[2][j], d1 = V[3][j];
            dk[0][j] = V[1][j];
            dk[1][j] = (a.dxa[0] + gg[0][0]) * d0 + (a.dxa[1] + gg[0][1]) * d1 + (a.dxa[2] + gg[0][2]) * e4;
            dk[2][j] = V[3][j];
            dk[3][j] = (a.dtha[0] + gg[1][0]) * d0 + (a.dtha[1] + gg[1][1]) * d1 + (a.dtha[2] + gg[1][2]) * e4;
        }
    }

    __device__ static void var_weights(const double* x, const double* u, double (*W)[NGP]) {
        W[0][0] = 1.0; W[0][1] = 0.0;
        W[1][0] = 0.0; W[1][1] = 1.0;
    }
};

}  // namespace gpmpc
