// hvp_admm.h -- the local MIQP of the naive-ADMM platoon controller (fleet_naive_admm.py:24-253).
//
// LocalMpcADMM differs from the decentralised LocalMpcMld in one respect: the neighbours'
// trajectories are not fixed predictions but COPY variables x_front, x_back (2, N+1) of the
// local problem (:84-102), priced by the tracking terms (:110-133), the ADMM terms
//     y_k' (c_k - z_k) + rho/2 |c_k - z_k|^2                      (:172-198)
// and the soft safe-distance rows  p_k - s_f <= e_f,k - d_safe,  p_k + s_b >= e_b,k + d_safe
// (:217-236) with slack cost w s (:164-169), e = position component of the copy.
//
// Given the own trajectory x_k the copy at step k enters only its own terms, so it is
// eliminated in closed form (per step, per side):
//     f(c; x) = 1/2 c'Ac - b(x)'c + (x-quadratic) + w max(0, sa * c_0 + h(x))
//     min_c f = [quadratic envelope q(x)] + Hub(u*(x)),   u*(x) = sa * [A^-1 b(x)]_0 + h(x)
//     Hub(u) = 0 (u <= 0),  u^2 / (2 kappa) (0 <= u <= w kappa),  w u - w^2 kappa / 2 (u >= w kappa)
// with kappa = [A^-1]_00: the hinge in the copy becomes a convex C^1 Huber-type function of the
// violation u* of the unconstrained copy.  Both q and the active piece of Hub are quadratic
// forms in (p_k, v_k), i.e. exactly the per-step terms setup_lane already assembles, so the
// local problem is the same velocity-space QP with one extra discrete state per hinge
// (inactive / quadratic / saturated).  solve_admm_lane iterates: assemble with the current
// hinge states, solve (hvp_gi.h), reclassify every hinge at the solution; at a consistent
// fixed point the QP's KKT conditions are those of the piecewise-quadratic problem (pieces
// agree in value and gradient at their breakpoints), so the point is its exact optimum.
//
// Parameter block (hvp_params_stride_admm(N) doubles):
//   [x0 (2) | y_front | z_front | y_back | z_back | leader_x], each (2, N+1) row-major.
#pragma once

#include "hvp_gi.h"
#include "hvp_ipm.h"

namespace hvp {

enum { HUB_OFF = 0, HUB_QUAD = 1, HUB_SAT = 2 };

// Closed-form elimination of one copy (side 0: front, 1: back) at one step.
struct CopyTerm {
    double Wpp, Wpv, Wvv, lp, lv, cc;  // envelope x'Wx + 2 l'x + cc
    double gp, gv, g0, kappa;          // u*(x) = gp p + gv v + g0
    double Ai00, Ai01, Ai11;           // A^-1 (symmetric)
    double B00, B01, B10, B11, b0, b1; // b(x) = B x + b
    double sa;                         // sign of the copy position in the hinge
};

HVP_HD inline void admm_copy(const Consts& C, bool track, int side, double y0, double y1, double z0, double z1,
                             CopyTerm& T) {
    const double rho = C.rho;
    const double qpp = track ? C.Qpp : 0.0, qpv = track ? C.Qpv : 0.0, qvv = track ? C.Qvv : 0.0;
    const double t0 = C.t0, d0 = C.d0;
    // S = M = [[1, t0], [0, 1]]
    // front: r = S x + (d0, 0);   back: residual = M c + (d0, 0) - x
    // M'QM (= S'QS)
    const double mqm00 = qpp, mqm01 = qpp * t0 + qpv, mqm11 = t0 * (qpp * t0 + qpv) + qpv * t0 + qvv;
    double A00, A01, A11;
    if (side == 0) {
        A00 = 2.0 * qpp + rho;
        A01 = 2.0 * qpv;
        A11 = 2.0 * qvv + rho;
    } else {
        A00 = 2.0 * mqm00 + rho;
        A01 = 2.0 * mqm01;
        A11 = 2.0 * mqm11 + rho;
    }
    const double det = A00 * A11 - A01 * A01;
    const double id = 1.0 / det;
    T.Ai00 = A11 * id;
    T.Ai01 = -A01 * id;
    T.Ai11 = A00 * id;
    double Wpp, Wpv, Wvv, lp, lv, cc;
    if (side == 0) {
        // B = 2 Q S,  b = 2 Q s0 + rho z - y,  s0 = (d0, 0)
        T.B00 = 2.0 * qpp;
        T.B01 = 2.0 * (qpp * t0 + qpv);
        T.B10 = 2.0 * qpv;
        T.B11 = 2.0 * (qpv * t0 + qvv);
        T.b0 = 2.0 * qpp * d0 + rho * z0 - y0;
        T.b1 = 2.0 * qpv * d0 + rho * z1 - y1;
        // S'QS and S'Q s0
        Wpp = mqm00;
        Wpv = mqm01;
        Wvv = mqm11;
        lp = qpp * d0;
        lv = (t0 * qpp + qpv) * d0;
        cc = qpp * d0 * d0;
    } else {
        // B = 2 M'Q,  b = -2 M'Q m + rho z - y,  m = (d0, 0)
        T.B00 = 2.0 * qpp;
        T.B01 = 2.0 * qpv;
        T.B10 = 2.0 * (t0 * qpp + qpv);
        T.B11 = 2.0 * (t0 * qpv + qvv);
        T.b0 = -2.0 * qpp * d0 + rho * z0 - y0;
        T.b1 = -2.0 * (t0 * qpp + qpv) * d0 + rho * z1 - y1;
        // (m - x)'Q(m - x) = x'Qx - 2 m'Q x + m'Q m
        Wpp = qpp;
        Wpv = qpv;
        Wvv = qvv;
        lp = -qpp * d0;
        lv = -qpv * d0;
        cc = qpp * d0 * d0;
    }
    cc += 0.5 * rho * (z0 * z0 + z1 * z1) - (y0 * z0 + y1 * z1);
    // - 1/2 (Bx + b)' A^-1 (Bx + b)
    const double K00 = T.Ai00 * T.B00 + T.Ai01 * T.B10, K01 = T.Ai00 * T.B01 + T.Ai01 * T.B11;  // A^-1 B
    const double K10 = T.Ai01 * T.B00 + T.Ai11 * T.B10, K11 = T.Ai01 * T.B01 + T.Ai11 * T.B11;
    const double k0 = T.Ai00 * T.b0 + T.Ai01 * T.b1, k1 = T.Ai01 * T.b0 + T.Ai11 * T.b1;          // A^-1 b
    Wpp -= 0.5 * (T.B00 * K00 + T.B10 * K10);
    Wpv -= 0.5 * (T.B00 * K01 + T.B10 * K11);
    Wvv -= 0.5 * (T.B01 * K01 + T.B11 * K11);
    lp -= 0.5 * (T.B00 * k0 + T.B10 * k1);
    lv -= 0.5 * (T.B01 * k0 + T.B11 * k1);
    cc -= 0.5 * (T.b0 * k0 + T.b1 * k1);
    T.Wpp = Wpp;
    T.Wpv = Wpv;
    T.Wvv = Wvv;
    T.lp = lp;
    T.lv = lv;
    T.cc = cc;
    // hinge: front  u = p - e + d_safe,  back  u = e + d_safe - p
    T.sa = side == 0 ? -1.0 : 1.0;
    T.gp = T.sa * K00 - T.sa;
    T.gv = T.sa * K01;
    T.g0 = T.sa * k0 + C.d_safe;
    T.kappa = T.Ai00;
}

// multiplier of the hinge at the optimum of the copy, given the unconstrained violation
HVP_HD inline int hub_state(double u, double w, double kappa) {
    return u <= 0.0 ? HUB_OFF : (u < w * kappa ? HUB_QUAD : HUB_SAT);
}

// adds the active Huber piece to an envelope
HVP_HD inline void hub_add(const CopyTerm& T, int st, double w, double& Wpp, double& Wpv, double& Wvv, double& lp,
                           double& lv, double& cc) {
    if (st == HUB_QUAD) {
        const double s = 0.5 / T.kappa;
        Wpp += s * T.gp * T.gp;
        Wpv += s * T.gp * T.gv;
        Wvv += s * T.gv * T.gv;
        lp += s * T.g0 * T.gp;
        lv += s * T.g0 * T.gv;
        cc += s * T.g0 * T.g0;
    } else if (st == HUB_SAT) {
        lp += 0.5 * w * T.gp;
        lv += 0.5 * w * T.gv;
        cc += w * T.g0 - 0.5 * w * w * T.kappa;
    }
}

// hinge-state bits: 2 per (step k = 1..N, side): index 2 (k - 1) + side
HVP_HD inline int hub_get(uint64_t hs, int k, int side) { return (int)((hs >> (2 * (2 * (k - 1) + side))) & 3u); }
HVP_HD inline uint64_t hub_set(uint64_t hs, int k, int side, int st) {
    const int sh = 2 * (2 * (k - 1) + side);
    return (hs & ~(3ull << sh)) | ((uint64_t)st << sh);
}

// copy blocks of the ADMM parameter layout
HVP_HD inline const double* admm_y(const double* prm, int side, int N) { return prm + 2 + (2 * side) * 2 * (N + 1); }
HVP_HD inline const double* admm_z(const double* prm, int side, int N) { return prm + 2 + (2 * side + 1) * 2 * (N + 1); }
HVP_HD inline const double* admm_leader(const double* prm, int N) { return prm + 2 + 8 * (N + 1); }

// ---------------------------------------------------------------- switching ADMM (HVP_FORM_GADMM)
// fleet_g_admm.LocalMpc (:22-205) for a GIVEN region sequence.  Same velocity-space problem as
// the naive-ADMM local problem with two differences: the vehicle's OWN trajectory is part of
// the augmented state (MpcAdmm [EXT]: y_own'(x_k - z_own,k) + rho/2 |x_k - z_own,k|^2 for
// k = 0..N), and the copy of the vehicle behind (HVP_ROLE_BACK_COPY) carries its ADMM term only
// (the cost tracks the front copy only, :136-158; safety only w.r.t. it, :98-109), so it
// decouples: c_b = z_b - y_b / rho with value -|y_b|^2 / (2 rho) per step.
// Parameter block (hvp_params_stride_gadmm(N)): the ADMM block followed by y_own | z_own.
HVP_HD inline const double* gadmm_yo(const double* prm, int N) { return prm + 2 + 10 * (N + 1); }
HVP_HD inline const double* gadmm_zo(const double* prm, int N) { return prm + 2 + 12 * (N + 1); }

// own-state ADMM term at step k as a form x'Wx + 2 l'x + cc
HVP_HD inline void gadmm_own_add(const Consts& C, const double* prm, int N, int k, double& Wpp, double& Wvv,
                                 double& lp, double& lv, double& cc) {
    const int K1 = N + 1;
    const double* yo = gadmm_yo(prm, N);
    const double* zo = gadmm_zo(prm, N);
    const double y0 = yo[k], y1 = yo[K1 + k], z0 = zo[k], z1 = zo[K1 + k];
    Wpp += 0.5 * C.rho;
    Wvv += 0.5 * C.rho;
    lp += 0.5 * (y0 - C.rho * z0);
    lv += 0.5 * (y1 - C.rho * z1);
    cc += 0.5 * C.rho * (z0 * z0 + z1 * z1) - (y0 * z0 + y1 * z1);
}

// own-state ADMM term of state k and the back-copy term, evaluated directly
HVP_HD inline double gadmm_state_terms(const Consts& C, int role, const double* prm, int N, int k, double p,
                                       double v) {
    const int K1 = N + 1;
    const double* yo = gadmm_yo(prm, N);
    const double* zo = gadmm_zo(prm, N);
    const double dp = p - zo[k], dv = v - zo[K1 + k];
    double J = yo[k] * dp + yo[K1 + k] * dv + 0.5 * C.rho * (dp * dp + dv * dv);
    if (role & HVP_ROLE_BACK_COPY) {
        const double* yb = admm_y(prm, 1, N);
        J -= (yb[k] * yb[k] + yb[K1 + k] * yb[K1 + k]) / (2.0 * C.rho);
    }
    return J;
}

// Velocity-space QP of the ADMM local problem for region code (first K steps fixed) and the
// hinge states hs.  Same row set and input-cost terms as setup_lane; the safe-distance rows are
// inert (the safety lives in the copies' hinges).
template <int N, class M>
HVP_HD inline bool setup_lane_admm(LaneQp<N, M>& q, const hvp_system& S, const Consts& C, int role,
                                   const double* prm, uint64_t code, int K, uint64_t hs) {
    const double p0 = prm[0], v0 = prm[1];
    const double* xl = admm_leader(prm, N);
    const double ts = S.ts;
    q.v0 = v0;
    q.ts = ts;
    q.P1 = p0 + ts * v0;
    q.pmin = S.pmin;
    q.pmax = S.pmax;
    q.has_sf = false;
    q.has_sb = false;
    double a[N], b[N], c[N];
#pragma unroll
    for (int k = 0; k < N; ++k) {
        const int r = code_region(code, k);
        const bool fixed = k < K;
        a[k] = fixed ? S.a[r] : 1.0;
        b[k] = fixed ? S.b[r] : 1.0;
        c[k] = fixed ? S.c[r] : 0.0;
        q.mem.set(F_AM, k, a[k]);
        q.mem.set(F_ULO, k, fixed ? c[k] + b[k] * S.umin : -1e30);
        q.mem.set(F_UHI, k, fixed ? c[k] + b[k] * S.umax : 1e30);
        if (k + 1 < K) {
            const int r1 = code_region(code, k + 1);
            q.mem.set(F_VLO, k, fmax(S.vmin, S.vlo[r1]));
            q.mem.set(F_VHI, k, fmin(S.vmax, S.vhi[r1]));
        } else {
            q.mem.set(F_VLO, k, S.vmin);
            q.mem.set(F_VHI, k, S.vmax);
        }
    }
#pragma unroll
    for (int j = 0; j < N - 1; ++j) {
        const double reach = ts * (j + 1);
        q.mem.set(F_HF, j, q.P1 + reach * S.vmax + 100.0);
        q.mem.set(F_HB, j, q.P1 + reach * S.vmin - 100.0);
    }
#pragma unroll
    for (int i = 0; i < LaneQp<N, M>::NT; ++i) q.H[i] = 0.0;
#pragma unroll
    for (int i = 0; i < N; ++i) q.f[i] = 0.0;
    double C0 = 0.0;
    const bool hf = (role & HVP_ROLE_SAFE_FRONT) != 0, hb = (role & HVP_ROLE_SAFE_BACK) != 0;
    const bool tf = (role & HVP_ROLE_TRACK_FRONT) != 0, tb = (role & HVP_ROLE_TRACK_BACK) != 0;
    const bool tl = (role & HVP_ROLE_TRACK_LEADER) != 0;
    const double* yf = admm_y(prm, 0, N);
    const double* zf = admm_z(prm, 0, N);
    const double* yb = admm_y(prm, 1, N);
    const double* zb = admm_z(prm, 1, N);
    const int K1 = N + 1;
#pragma unroll
    for (int k = 1; k <= N; ++k) {
        double Wpp = 0, Wpv = 0, Wvv = 0, lp = 0, lv = 0, cc = 0;
        if (tl) {  // |x_k - leader_x_k|^2_Q (fleet_naive_admm.py:134-141)
            const double r0 = -xl[k], r1 = -xl[K1 + k];
            Wpp += C.Qpp;
            Wpv += C.Qpv;
            Wvv += C.Qvv;
            lp += C.Qpp * r0 + C.Qpv * r1;
            lv += C.Qpv * r0 + C.Qvv * r1;
            cc += r0 * (C.Qpp * r0 + C.Qpv * r1) + r1 * (C.Qpv * r0 + C.Qvv * r1);
        }
        for (int side = 0; side < 2; ++side) {
            if (!(side == 0 ? hf : hb)) continue;
            const double* yy = side == 0 ? yf : yb;
            const double* zz = side == 0 ? zf : zb;
            CopyTerm T;
            admm_copy(C, side == 0 ? tf : tb, side, yy[k], yy[K1 + k], zz[k], zz[K1 + k], T);
            Wpp += T.Wpp;
            Wpv += T.Wpv;
            Wvv += T.Wvv;
            lp += T.lp;
            lv += T.lv;
            cc += T.cc;
            hub_add(T, hub_get(hs, k, side), C.w, Wpp, Wpv, Wvv, lp, lv, cc);
        }
        if (C.form == HVP_FORM_GADMM) gadmm_own_add(C, prm, N, k, Wpp, Wvv, lp, lv, cc);
        // x_k = xbar + Gamma y : p = P1 + ts prefix(0..k-2), v = e_{k-1}
        const double pbar = q.P1;
        const double gp = 2.0 * (Wpp * pbar + lp);
        const double gv = 2.0 * (Wpv * pbar + lv);
        C0 += Wpp * pbar * pbar + 2.0 * lp * pbar + cc;
        const int jv = k - 1;
        q.H[tri(jv, jv)] += 2.0 * Wvv;
        q.f[jv] += gv;
#pragma unroll
        for (int i = 0; i < N; ++i) {
            if (i > k - 2) break;
            q.f[i] += ts * gp;
#pragma unroll
            for (int i2 = 0; i2 <= i; ++i2) q.H[tri(i, i2)] += 2.0 * Wpp * ts * ts;
            q.H[tri(jv, i)] += 2.0 * Wpv * ts;
        }
    }
    // control effort / variation on the first K steps (as setup_lane)
    double ubar[N], gk[N], gkm[N];
#pragma unroll
    for (int k = 0; k < N; ++k) {
        const double ib = 1.0 / b[k];
        ubar[k] = k == 0 ? -(a[0] * v0 + c[0]) * ib : -c[k] * ib;
        gk[k] = ib;
        gkm[k] = k == 0 ? 0.0 : -a[k] * ib;
        const double w2 = k < K ? 2.0 * C.Qu : 0.0;
        q.H[tri(k, k)] += w2 * gk[k] * gk[k];
        q.f[k] += w2 * ubar[k] * gk[k];
        if (k >= 1) {
            q.H[tri(k - 1, k - 1)] += w2 * gkm[k] * gkm[k];
            q.H[tri(k, k - 1)] += w2 * gk[k] * gkm[k];
            q.f[k - 1] += w2 * ubar[k] * gkm[k];
        }
        C0 += k < K ? C.Qu * ubar[k] * ubar[k] : 0.0;
    }
    if (C.Qdu != 0.0) {
#pragma unroll
        for (int k = 0; k + 1 < N; ++k) {
            double g[N];
#pragma unroll
            for (int i = 0; i < N; ++i) g[i] = 0.0;
            g[k + 1] += gk[k + 1];
            g[k] += gkm[k + 1] - gk[k];
            if (k >= 1) g[k - 1] -= gkm[k];
            const double eb = ubar[k + 1] - ubar[k];
            const double w2 = k + 1 < K ? 2.0 * C.Qdu : 0.0;
#pragma unroll
            for (int i = 0; i < N; ++i) {
                q.f[i] += w2 * eb * g[i];
#pragma unroll
                for (int i2 = 0; i2 <= i; ++i2) q.H[tri(i, i2)] += w2 * g[i] * g[i2];
            }
            C0 += k + 1 < K ? C.Qdu * eb * eb : 0.0;
        }
    }
    q.C0 = C0;
    return q.P1 >= S.pmin - 1e-9 * (1.0 + fabs(S.pmin)) && q.P1 <= S.pmax + 1e-9 * (1.0 + fabs(S.pmax));
}

// Hinge states consistent with the trajectory y (k = 1..N): the new state word.
template <int N>
HVP_HD inline uint64_t admm_classify(const Consts& C, int role, const double* prm, double P1, double ts,
                                     const double* y, uint64_t hs, bool* consistent) {
    const bool hf = (role & HVP_ROLE_SAFE_FRONT) != 0, hb = (role & HVP_ROLE_SAFE_BACK) != 0;
    const bool tf = (role & HVP_ROLE_TRACK_FRONT) != 0, tb = (role & HVP_ROLE_TRACK_BACK) != 0;
    const int K1 = N + 1;
    uint64_t out = 0;
    bool same = true;
    double p = P1, cum = 0.0;
#pragma unroll
    for (int k = 1; k <= N; ++k) {
        if (k >= 2) {
            cum += y[k - 2];
            p = P1 + ts * cum;
        }
        const double v = y[k - 1];
        for (int side = 0; side < 2; ++side) {
            if (!(side == 0 ? hf : hb)) continue;
            const double* yy = admm_y(prm, side, N);
            const double* zz = admm_z(prm, side, N);
            CopyTerm T;
            admm_copy(C, side == 0 ? tf : tb, side, yy[k], yy[K1 + k], zz[k], zz[K1 + k], T);
            const double u = T.gp * p + T.gv * v + T.g0;
            const int old = hub_get(hs, k, side);
            int st = hub_state(u, C.w, T.kappa);
            // at a breakpoint the two pieces agree to first order: keep the current state
            const double tol = 1e-10 * (1.0 + fabs(u) + fabs(p));
            if (st != old) {
                const double lo = old == HUB_OFF ? -1e300 : (old == HUB_QUAD ? 0.0 : C.w * T.kappa);
                const double hi = old == HUB_OFF ? 0.0 : (old == HUB_QUAD ? C.w * T.kappa : 1e300);
                if (u >= lo - tol && u <= hi + tol) st = old;
            }
            if (st != old) same = false;
            out = hub_set(out, k, side, st);
        }
    }
    *consistent = same;
    return out;
}

// Optimal copy of one side at step k for the own state (p, v), its slack and its term of the
// objective (tracking + ADMM + w * slack), as the reference's Gurobi model evaluates them.
HVP_HD inline double admm_copy_value(const Consts& C, bool track, int side, double y0, double y1, double z0, double z1,
                                     double p, double v, double* c0_out, double* c1_out) {
    CopyTerm T;
    admm_copy(C, track, side, y0, y1, z0, z1, T);
    const double u = T.gp * p + T.gv * v + T.g0;
    const int st = hub_state(u, C.w, T.kappa);
    const double mu = st == HUB_OFF ? 0.0 : (st == HUB_QUAD ? u / T.kappa : C.w);
    // c = A^-1 (B x + b - mu sa e_0)
    const double r0 = T.B00 * p + T.B01 * v + T.b0 - mu * T.sa, r1 = T.B10 * p + T.B11 * v + T.b1;
    const double e = T.Ai00 * r0 + T.Ai01 * r1, g = T.Ai01 * r0 + T.Ai11 * r1;
    const double s = fmax(0.0, T.sa * e + (side == 0 ? p : -p) + C.d_safe);
    double J = C.w * s;
    if (track) {
        double ep, ev;
        if (side == 0) { ep = p + C.t0 * v + C.d0 - e; ev = v - g; }
        else { ep = e + C.t0 * g + C.d0 - p; ev = g - v; }
        J += C.Qpp * ep * ep + 2.0 * C.Qpv * ep * ev + C.Qvv * ev * ev;
    }
    J += y0 * (e - z0) + y1 * (g - z1) + 0.5 * C.rho * ((e - z0) * (e - z0) + (g - z1) * (g - z1));
    if (c0_out) *c0_out = e;
    if (c1_out) *c1_out = g;
    return J;
}

// Objective of the ADMM local problem at the trajectory y (first K steps with their regions'
// input terms), evaluated term by term (fleet_naive_admm.py:107-198).
template <int N, class M>
HVP_HD inline double admm_direct_cost(const LaneQp<N, M>& q, const hvp_system& S_in, const Consts& C, int role,
                                      const double* prm_in, uint64_t code, int K) {
    const double* prm = opaque_ptr(prm_in);
    const hvp_system& S = *opaque_ptr(&S_in);
    const double* xl = admm_leader(prm, N);
    const bool hf = (role & HVP_ROLE_SAFE_FRONT) != 0, hb = (role & HVP_ROLE_SAFE_BACK) != 0;
    const bool tf = (role & HVP_ROLE_TRACK_FRONT) != 0, tb = (role & HVP_ROLE_TRACK_BACK) != 0;
    const bool tl = (role & HVP_ROLE_TRACK_LEADER) != 0;
    const int K1 = N + 1;
    double J = 0.0, p = prm[0], v = prm[1], uprev = 0.0;
    for (int k = 0; k <= N; ++k) {
        if (tl) {
            const double ep = p - xl[k], ev = v - xl[K1 + k];
            J += C.Qpp * ep * ep + 2.0 * C.Qpv * ep * ev + C.Qvv * ev * ev;
        }
        if (hf)
            J += admm_copy_value(C, tf, 0, admm_y(prm, 0, N)[k], admm_y(prm, 0, N)[K1 + k], admm_z(prm, 0, N)[k],
                                 admm_z(prm, 0, N)[K1 + k], p, v, nullptr, nullptr);
        if (hb)
            J += admm_copy_value(C, tb, 1, admm_y(prm, 1, N)[k], admm_y(prm, 1, N)[K1 + k], admm_z(prm, 1, N)[k],
                                 admm_z(prm, 1, N)[K1 + k], p, v, nullptr, nullptr);
        if (C.form == HVP_FORM_GADMM) J += gadmm_state_terms(C, role, prm, N, k, p, v);
        if (k < N) {
            const int r = code_region(code, k);
            const double vn = q.y[k];
            const double u = (vn - S.a[r] * v - S.c[r]) / S.b[r];
            if (k < K) J += C.Qu * u * u;
            if (k >= 1 && k < K) J += C.Qdu * (u - uprev) * (u - uprev);
            uprev = u;
            p = p + S.ts * v;
            v = vn;
        }
    }
    return J;
}

// The ADMM local QP for one region code: hinge-state iteration around the active-set solve.
// Returns GI_OK with the optimum in q.y, or a GI_FAIL_* code (GI_FAIL_ITER also when the hinge
// states do not settle within kHubRounds).
constexpr int kHubRounds = 12;
constexpr uint64_t kHubNone = ~0ull;  // no starting hinge states given (two bits per hinge use 0..2)
template <int N, class M>
HVP_HD inline int solve_admm_lane(LaneQp<N, M>& q, const hvp_system& S, const Consts& C, int role, const double* prm,
                                  uint64_t code, int K, int max_iter, int& iters, uint32_t* edge = nullptr,
                                  uint64_t* hs_io = nullptr, int* rounds = nullptr) {
    uint64_t hs = 0;
    iters = 0;
    if (hs_io && *hs_io != kHubNone) {
        hs = *hs_io;  // warm: the caller's starting states (a parent's, another iteration's)
    } else {
        // initial states: those of the unconstrained copies at the constant-velocity trajectory
        double y[N];
#pragma unroll
        for (int k = 0; k < N; ++k) y[k] = prm[1];
        bool c;
        hs = admm_classify<N>(C, role, prm, prm[0] + S.ts * prm[1], S.ts, y, 0, &c);
    }
    for (int round = 0; round < kHubRounds; ++round) {
        setup_lane_admm<N>(q, S, C, role, prm, code, K, hs);
        int it = 0;
        const int st = solve_gi<N>(q, C, max_iter, it, edge);
        iters += it;
        if (rounds) *rounds = round + 1;
        if (st != GI_OK) return st;
        bool consistent;
        hs = admm_classify<N>(C, role, prm, q.P1, q.ts, q.y, hs, &consistent);
        if (consistent) {
            if (hs_io) *hs_io = hs;
            return GI_OK;
        }
    }
    return GI_FAIL_ITER;
}

// The interior-point fallback of the ADMM local QP (naive ADMM leaves, switching-ADMM local QPs):
// the hinge-state iteration of solve_admm_lane with the Mehrotra interior point (hvp_ipm.h Solver)
// in place of the active-set method, for the QPs the active-set method fails on (degenerate
// vertices, its iteration cap).  The row set is setup_lane_admm's, so the optimum is the same QP's
// -- what fleet_naive_admm.py:407-419 (Gurobi) and fleet_g_admm.py:162,195-205 (qpOASES) return for
// it.  edge: the switching rule's bits (V rows active with multiplier > kEdgeMultTol, as
// GiLane::verify reports them), from the interior point's multipliers.
template <int N, class M>
HVP_HD HVP_FORCEINLINE inline int solve_admm_ipm(LaneQp<N, M>& q, const hvp_system& S, const Consts& C, int role, const double* prm,
                                 uint64_t code, int K, int& iters, uint32_t* edge = nullptr) {
    uint64_t hs = 0;
    iters = 0;
    {
        double y[N];
#pragma unroll
        for (int k = 0; k < N; ++k) y[k] = prm[1];
        bool c;
        hs = admm_classify<N>(C, role, prm, prm[0] + S.ts * prm[1], S.ts, y, 0, &c);
    }
    for (int round = 0; round < kHubRounds; ++round) {
        setup_lane_admm<N>(q, S, C, role, prm, code, K, hs);
        const QpOut o = Solver<N, true, M>::solve(q, C);
        iters += o.iters;
        // the interior point's own answer, kept for a polish that fails
        double yi[N];
        uint32_t mi = 0;
#pragma unroll
        for (int j = 0; j < N; ++j) {
            yi[j] = q.y[j];
            if (q.llo[3 * j] > kEdgeMultTol) mi |= 1u << (2 * j);
            if (q.lhi[3 * j] > kEdgeMultTol) mi |= 1u << (2 * j + 1);
        }
        // exact optimum and multipliers from the interior point's active set (hvp_gi.h gi_polish;
        // tried from a non-converged iterate too: its active set may still be the right one)
        int pit = 0;
        uint32_t mp = 0;
        const int pst = gi_polish<N>(q, C, 8 * GiConstraintSet<N>::NC, pit, &mp);
        iters += pit;
        if (pst != GI_OK) {
            if (o.status != 0) return GI_FAIL_ITER;
#pragma unroll
            for (int j = 0; j < N; ++j) q.y[j] = yi[j];
        }
        bool consistent;
        hs = admm_classify<N>(C, role, prm, q.P1, q.ts, q.y, hs, &consistent);
        if (consistent) {
            if (edge) *edge = pst == GI_OK ? mp : mi;
            return GI_OK;
        }
    }
    return GI_FAIL_ITER;
}

}  // namespace hvp
