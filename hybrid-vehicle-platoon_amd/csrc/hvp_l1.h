// hvp_l1.h -- fixed-sequence LP of the min_1_norm local MPC (the L1 / MILP variant).
//
// LocalMpcMld.setup_cost_and_constraints(quadratic_cost=False) (fleet_decent_mld.py:73-76)
// prices every term of the objective with min_1_norm [EXT dmpcpwa]: sum_i Q_ii |e_i| of the
// tracking errors (:110-153), Q_u |u_k| (:155), Q_du |u_{k+1} - u_k| (:157-162), plus the
// linear slack cost w (s_f + s_b) (:164-169).  With the region sequence sigma fixed the MLD
// MILP is an LP; its optimum over sigma is the MILP optimum (same search and tie rule as the
// quadratic path: hvp_lane.h k_enum / k_select).
//
// Formulation (velocity space, as hvp_ipm.h): y = (v_1 .. v_N), p_k = P1 + ts (y_0 + .. + y_{k-2}),
// u_k = (y_k - a_k y_{k-1} - c_k) / b_k.
//   hard rows  g.y <= h : V (region sigma_{k+1} and the state box), U (input box), A (accel
//              rows with tightening), P (position box)                       8N - 2 rows
//   pairs      w |g.y + e0|        (alpha = 1: tracking errors, u, du)   or
//              w max(0, g.y + e0)  (alpha = 0: the soft safe-distance rows, slack eliminated)
//              each with its epigraph variable t:  g.y - t <= -e0,  -alpha g.y - t <= alpha e0,
//              cost w t.
// Variable-free terms (k = 0, the p_1 errors, the k = 0, 1 slacks) are constants: they enter the
// cost (l1_direct_cost) but not the LP.
//
// Solver: Mehrotra predictor-corrector primal-dual interior point in (y, t), every epigraph
// variable eliminated analytically from its two rows (Schur complement per pair:
// D1 D2 (1 + alpha)^2 / (D1 + D2) g g'), so the Newton system is N x N whatever the number of
// terms.  The interior point converges to a point of the optimal face; the objective -- what
// the sequence search compares -- is evaluated term by term on it (l1_direct_cost).  Before it
// runs, l1_infeasible decides the hard rows exactly (velocity lattice + position extremes); an LP
// it cannot solve is L1_FAIL (unresolved), never silently dropped.  Search: enumeration (N <= 8)
// or branch and bound with the node LPs relaxed after K steps (l1_steps, the quadratic path's
// tail relaxation).
//
// No HIP dependency: hvp_lane.h compiles it for gfx950, the test-only host build
// (hvp_hostref.cpp) with g++.
#pragma once

#include "hvp_ipm.h"

namespace hvp {

constexpr int kL1MaxIter = 120;  // interior-point iteration cap (hvp_problem.max_iter > 0 overrides it)
#ifndef HVP_L1_SHORT
#define HVP_L1_SHORT 0.1
#endif
#ifndef HVP_L1_CENTRE
#define HVP_L1_CENTRE 0.5
#endif
constexpr double kL1Short = HVP_L1_SHORT;    // corrector steps shorter than this fall back to centring
constexpr double kL1Centre = HVP_L1_CENTRE;  // sigma of that centring step

// LP status: converged / proven infeasible (a Farkas certificate of the hard rows, l1_farkas) /
// unresolved (iteration cap or a numerical failure without a certificate: the search reports
// HVP_MAXITER for an instance where such an LP may hold the optimum, never a worse sequence).
enum { L1_OK = 0, L1_INFEASIBLE = 1, L1_FAIL = 2 };

// Infeasibility certificate of the hard rows G y <= h from nonnegative multipliers lam: every
// feasible y lies in the velocity box [ylo, yhi]^N (the V rows), so lam'G y >= sum_a min(r_a ylo,
// r_a yhi) with r = G' lam; if that exceeds lam'h (with a relative margin), no y satisfies the
// rows.  On a primal-infeasible LP the interior point's hard-row multipliers grow along such a
// ray.  r (N) and hl = lam'h are the sums over the rows; scale = sum |lam_i h_i|.
template <int N>
HVP_HD inline bool l1_farkas(const double* r, double hl, double scale, double ylo, double yhi) {
    double lower = 0.0, mag = scale;
    for (int a = 0; a < N; ++a) {
        lower += fmin(r[a] * ylo, r[a] * yhi);
        mag += fabs(r[a]) * fmax(fabs(ylo), fabs(yhi));
    }
    return mag > 0.0 && mag < 1e250 && lower > hl + 1e-9 * mag;
}

template <int N>
struct L1Lp {
    static constexpr int MH = 8 * N - 2;
    static constexpr int MP = 10 * N;
    static constexpr int NT = N * (N + 1) / 2;
    int mh, mp;
    double gh[MH][N], h[MH];
    double gp[MP][N], e0[MP], wp[MP], al[MP];
    // iterate
    double y[N], t[MP];
    double sh[MH], lh[MH];
    double s1[MP], s2[MP], l1[MP], l2[MP];
    // affine (predictor) directions of s and l, for the corrector's second-order term
    double dsh[MH], dlh[MH], ds1[MP], dl1[MP], ds2[MP], dl2[MP];
};

// Cholesky factorisation of the LP's Newton matrix (inverse diagonal stored, as hvp_ipm.h cholesky)
// with the "Cholesky infinity" rule of LP interior points: near a degenerate vertex the matrix
// sum_r D_r g_r g_r' spans scalings 1e-12 .. 1e12 and a pivot can lose all its digits; such a pivot
// (<= 1e-13 of its diagonal before elimination) is taken as infinite, i.e. the direction leaves
// that component where it is.  The iteration continues instead of stopping at a converged-but-
// degenerate point (the oracle solves those LPs; without the rule they ended unresolved).
template <int N>
HVP_HD inline void cholesky_l1(double* K) {
#pragma unroll
    for (int j = 0; j < N; ++j) {
        const double d = K[tri(j, j)];
        double s = d;
#pragma unroll
        for (int k = 0; k < j; ++k) s -= K[tri(j, k)] * K[tri(j, k)];
        const double il = s > 1e-13 * d ? frcp(sqrt(s)) : 0.0;
        K[tri(j, j)] = il;
#pragma unroll
        for (int i = j + 1; i < N; ++i) {
            double v = K[tri(i, j)];
#pragma unroll
            for (int k = 0; k < j; ++k) v -= K[tri(i, k)] * K[tri(j, k)];
            K[tri(i, j)] = v * il;
        }
    }
}

template <int N>
HVP_HD inline double l1_dot(const double* g, const double* y) {
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < N; ++i) s += g[i] * y[i];
    return s;
}

// Per-step data of a (node) LP: the dynamics (a, b, c) of every step, which steps carry their
// input rows and |u| cost (bit k of `on`), and the bounds of v_{k+1}.  Steps k < K take the
// regions of `code`; steps k >= K are RELAXED exactly as the quadratic bound (hvp_ipm.h
// setup_input / relax_step): from the exact interval [rlo, rhi] of v_K each undecided v_{k+1} keeps
// its reachable interval and, where the regions step k may take share (a, c), the step takes the
// virtual region (a, b_max, c) with its input rows and cost (Q_u |s| <= Q_u |u| for s = u b_r / b_max);
// otherwise the step's input rows and cost are dropped.  rlo > rhi (the default) = no relaxation
// information (K = N leaves, enumeration candidates).
HVP_HD inline void l1_steps_rt(const hvp_system& S, const Consts& C, uint64_t code, int K, double rlo, double rhi, int N,
                               double* a, double* b, double* c, unsigned& on, double* vlo, double* vhi) {
    bool relax = rlo <= rhi;
    on = 0;
    for (int k = 0; k < N; ++k) {
        const bool fixed = k < K;
        int vr = -1;
        double bm = 1.0, nlo = S.vmin, nhi = S.vmax;
        if (!fixed && relax) {
            bool dead;
            vr = relax_step(S, C, k, rlo, rhi, nlo, nhi, bm, dead);
            relax = !dead;
            rlo = nlo;
            rhi = nhi;
        }
        const bool st_on = fixed || vr >= 0;
        const int r = fixed ? code_region(code, k) : (vr >= 0 ? vr : 0);
        a[k] = st_on ? S.a[r] : 1.0;
        b[k] = fixed ? S.b[r] : (vr >= 0 ? bm : 1.0);
        c[k] = st_on ? S.c[r] : 0.0;
        on |= st_on ? 1u << k : 0u;
        if (k + 1 < K) {  // v_{k+1} in region sigma_{k+1} and the state box
            const int r1 = code_region(code, k + 1);
            vlo[k] = fmax(S.vmin, S.vlo[r1]);
            vhi[k] = fmin(S.vmax, S.vhi[r1]);
        } else if (!fixed && relax) {  // a relaxed v_{k+1}: its reachable interval
            vlo[k] = fmax(S.vmin, nlo);
            vhi[k] = fmin(S.vmax, nhi);
        } else {
            vlo[k] = S.vmin;
            vhi[k] = S.vmax;
        }
    }
}

template <int N>
HVP_HD inline void l1_steps(const hvp_system& S, const Consts& C, uint64_t code, int K, double rlo, double rhi,
                            double* a, double* b, double* c, unsigned& on, double* vlo, double* vhi) {
    l1_steps_rt(S, C, code, K, rlo, rhi, N, a, b, c, on, vlo, vhi);
}

// Rows of the fixed-sequence LP of instance params prm (x0, x_front, x_back, leader_x) and
// region code -- or, with K < N, of the branch-and-bound relaxation of the prefix code[0..K-1]
// (l1_steps) -- in a fixed order: hard(idx, g, sgn, h) for the row sgn*g.y <= h and
// pair(idx, g, e0, w, alpha) for every term with a variable part (zero-weight and constant terms
// are skipped, so the indices are dense).  Both callbacks see every row in the same order on
// every lane: the per-lane host solver stores them all (l1_setup), the wave-cooperative kernels
// (hvp_lane.h) keep the rows whose index maps to their lane.  Returns (mh, mp) through the
// counters and false when the constant row p_1 in [pmin, pmax] is violated.
// xl_blk: the leader window's offset in the params row in units of N + 1 (4: HVP_FORM_DECENT; the
// naive-ADMM form's own rows (l1_admm_*) pass 8 with every role bit but HVP_ROLE_TRACK_LEADER
// cleared, so xf / xb are never read).
template <int N, class FH, class FP>
HVP_HD inline bool l1_rows(const hvp_system& S, const Consts& C, int role, const double* prm, uint64_t code, int K,
                           double rlo, double rhi, int& mh, int& mp, FH&& hard_cb, FP&& pair_cb, int xl_blk = 4) {
    const double p0 = prm[0], v0 = prm[1];
    const double* xf = prm + 2;
    const double* xb = prm + 2 + 2 * (N + 1);
    const double* xl = prm + 2 + xl_blk * (N + 1);
    const int K1 = N + 1;
    const double ts = S.ts, P1 = p0 + ts * v0;
    mh = 0;
    mp = 0;
    auto hard = [&](const double* g, double sgn, double hh) {
        hard_cb(mh, g, sgn, hh);
        ++mh;
    };
    auto pair = [&](const double* g, double e0, double w, double alpha) {
        bool any = false;
        for (int i = 0; i < N; ++i) any = any || g[i] != 0.0;
        if (!(w > 0.0) || !any) return;  // zero weight, or a constant term (in the direct cost)
        pair_cb(mp, g, e0, w, alpha);
        ++mp;
    };
    double a[N], b[N], c[N], vlo[N], vhi[N];
    unsigned on;
    l1_steps<N>(S, C, code, K, rlo, rhi, a, b, c, on, vlo, vhi);
    double g[N];
    auto zero = [&]() {
        for (int i = 0; i < N; ++i) g[i] = 0.0;
    };
    // ---- hard rows
    for (int j = 0; j < N; ++j) {
        // V: v_{j+1} in region sigma_{j+1} (k < N) and the state box (relaxed: reachable interval)
        zero();
        g[j] = 1.0;
        hard(g, 1.0, vhi[j]);
        hard(g, -1.0, -vlo[j]);
        // U: c + b umin <= v_{j+1} - a v_j <= c + b umax   (F u <= G); dropped on a relaxed step
        // without a virtual region
        if ((on >> j) & 1u) {
            const double cu = j == 0 ? a[0] * v0 : 0.0;
            zero();
            g[j] = 1.0;
            if (j) g[j - 1] = -a[j];
            hard(g, 1.0, c[j] + b[j] * S.umax + cu);
            hard(g, -1.0, -(c[j] + b[j] * S.umin + cu));
        }
        // A: dec_j <= v_{j+1} - v_j <= acc_j   (fleet_decent_mld.py:172-188)
        const double ca = j == 0 ? v0 : 0.0;
        zero();
        g[j] = 1.0;
        if (j) g[j - 1] = -1.0;
        hard(g, 1.0, C.acc[j] + ca);
        hard(g, -1.0, -(C.dec[j] + ca));
    }
    for (int m = 0; m + 2 <= N; ++m) {  // P: pmin <= p_{m+2} <= pmax
        for (int i = 0; i < N; ++i) g[i] = i <= m ? ts : 0.0;
        hard(g, 1.0, S.pmax - P1);
        hard(g, -1.0, P1 - S.pmin);
    }
    // ---- L1 terms and soft rows
    const bool tf = (role & HVP_ROLE_TRACK_FRONT) != 0, tb = (role & HVP_ROLE_TRACK_BACK) != 0;
    const bool tl = (role & HVP_ROLE_TRACK_LEADER) != 0, lsp = (role & HVP_ROLE_LEADER_SPACING) != 0;
    const bool sf = (role & HVP_ROLE_SAFE_FRONT) != 0, sb = (role & HVP_ROLE_SAFE_BACK) != 0;
    const double t0 = C.t0, d0 = C.d0;
    for (int k = 1; k <= N; ++k) {
        double gpre[N], gv[N], tmp[N];
        for (int i = 0; i < N; ++i) {
            gpre[i] = i <= k - 2 ? ts : 0.0;  // p_k = P1 + gpre.y
            gv[i] = i == k - 1 ? 1.0 : 0.0;   // v_k = gv.y
        }
        if (tf) {  // x_k - xf_k - spacing(x_k)   (:110-121)
            for (int i = 0; i < N; ++i) tmp[i] = gpre[i] + t0 * gv[i];
            pair(tmp, P1 + d0 - xf[k], C.Qpp, 1.0);
            pair(gv, -xf[K1 + k], C.Qvv, 1.0);
        }
        if (tb) {  // xb_k - x_k - spacing(xb_k)   (:122-133)
            for (int i = 0; i < N; ++i) tmp[i] = -gpre[i];
            pair(tmp, xb[k] + t0 * xb[K1 + k] + d0 - P1, C.Qpp, 1.0);
            for (int i = 0; i < N; ++i) tmp[i] = -gv[i];
            pair(tmp, xb[K1 + k], C.Qvv, 1.0);
        }
        if (tl) {  // x_k - leader_x_k (- spacing(x_k) with real_vehicle_as_reference)   (:134-153)
            for (int i = 0; i < N; ++i) tmp[i] = gpre[i] + (lsp ? t0 * gv[i] : 0.0);
            pair(tmp, P1 - xl[k] + (lsp ? d0 : 0.0), C.Qpp, 1.0);
            pair(gv, -xl[K1 + k], C.Qvv, 1.0);
        }
        if (k >= 2 && sf) pair(gpre, P1 - xf[k] + C.d_safe, C.w, 0.0);  // w max(0, p_k - pf_k + d_safe)
        if (k >= 2 && sb) {                                                // w max(0, pb_k + d_safe - p_k)
            for (int i = 0; i < N; ++i) tmp[i] = -gpre[i];
            pair(tmp, xb[k] + C.d_safe - P1, C.w, 0.0);
        }
    }
    // inputs u_k = ubar_k + gu_k.y ; Q_u |u_k| (steps carrying their input) and Q_du |u_{k+1} - u_k|
    // (both steps decided)
    double gprev[N], uprev = 0.0;
    for (int k = 0; k < N; ++k) {
        double gu[N];
        const double ib = 1.0 / b[k];
        for (int i = 0; i < N; ++i) gu[i] = i == k ? ib : (i + 1 == k ? -a[k] * ib : 0.0);
        const double ubar = k == 0 ? -(a[0] * v0 + c[0]) * ib : -c[k] * ib;
        if ((on >> k) & 1u) pair(gu, ubar, C.Qu, 1.0);
        if (k >= 1 && k < K) {
            double gd[N];
            for (int i = 0; i < N; ++i) gd[i] = gu[i] - gprev[i];
            pair(gd, ubar - uprev, C.Qdu, 1.0);
        }
        for (int i = 0; i < N; ++i) gprev[i] = gu[i];
        uprev = ubar;
    }
    return P1 >= S.pmin - 1e-9 * (1.0 + fabs(S.pmin)) && P1 <= S.pmax + 1e-9 * (1.0 + fabs(S.pmax));
}

// Exact infeasibility test of the hard rows (V, U, A, P of l1_rows with the same relaxation),
// run before the interior point: with v_{k+1} in [L_k(v_k), U_k(v_k)] and L_k, U_k nondecreasing
// (a > 0), the velocity-feasible trajectories form a lattice, so the interval of each v_k over all
// of them is the forward-reachable interval intersected with the backward-feasible one, and the
// componentwise lowest / highest trajectories are feasible.  They give every prefix sum its exact
// minimum / maximum, so
//   * an empty interval, or
//   * a position row p_m <= pmax violated by the lowest trajectory (or p_m >= pmin by the highest)
// proves the LP infeasible (margin 1e-9 relative).  The one case it cannot decide -- rows on both
// sides of the position box binding within one horizon -- is reported feasible: the interior point
// then runs and, if it does not converge, the LP stays unresolved (L1_FAIL), never "infeasible".
HVP_HD inline bool l1_infeasible_rt(const hvp_system& S, const Consts& C, double p0, double v0, uint64_t code, int K,
                                    double rlo, double rhi, int N) {
    double a[HVP_MAX_N], b[HVP_MAX_N], c[HVP_MAX_N], vlo[HVP_MAX_N], vhi[HVP_MAX_N];
    unsigned on;
    l1_steps_rt(S, C, code, K, rlo, rhi, N, a, b, c, on, vlo, vhi);
    const double P1 = p0 + S.ts * v0;
    auto tol = [](double x) { return 1e-9 * (1.0 + fabs(x)); };
    // the v_j for which step j admits some v_{j+1}: L_j(v) <= U_j(v)
    auto step_ok = [&](int j, double& lo, double& hi) {
        if ((on >> j) & 1u) {
            if (!(a[j] > 0.0)) return false;
            const double cl = c[j] + b[j] * S.umin, cu = c[j] + b[j] * S.umax, oma = 1.0 - a[j];
            if (cu < cl - tol(cl)) return false;
            if (oma > 0.0) {
                lo = fmax(lo, -(C.acc[j] - cl) / oma);
                hi = fmin(hi, (cu - C.dec[j]) / oma);
            } else if (oma < 0.0) {
                hi = fmin(hi, (C.acc[j] - cl) / (-oma));
                lo = fmax(lo, (cu - C.dec[j]) / oma);
            } else if (C.acc[j] - cl < -tol(cl) || cu - C.dec[j] < -tol(cu)) {
                return false;
            }
        }
        return C.acc[j] >= C.dec[j] - tol(C.dec[j]);
    };
    auto Lmap = [&](int j, double v) {
        return ((on >> j) & 1u) ? fmax(a[j] * v + c[j] + b[j] * S.umin, v + C.dec[j]) : v + C.dec[j];
    };
    auto Umap = [&](int j, double v) {
        return ((on >> j) & 1u) ? fmin(a[j] * v + c[j] + b[j] * S.umax, v + C.acc[j]) : v + C.acc[j];
    };
    double flo[HVP_MAX_N + 1], fhi[HVP_MAX_N + 1];
    flo[0] = fhi[0] = v0;
    for (int j = 0; j < N; ++j) {  // forward: v_{j+1} reachable
        double lo = flo[j], hi = fhi[j];
        if (!step_ok(j, lo, hi) || lo > hi + tol(hi)) return true;
        if (lo > hi) lo = hi = 0.5 * (lo + hi);
        flo[j + 1] = fmax(vlo[j], Lmap(j, lo));
        fhi[j + 1] = fmin(vhi[j], Umap(j, hi));
        if (flo[j + 1] > fhi[j + 1] + tol(fhi[j + 1])) return true;
        if (flo[j + 1] > fhi[j + 1]) flo[j + 1] = fhi[j + 1] = 0.5 * (flo[j + 1] + fhi[j + 1]);
    }
    for (int j = N - 1; j >= 1; --j) {  // backward: v_j with a continuation (flo/fhi = projection)
        double lo = flo[j], hi = fhi[j];
        if (!step_ok(j, lo, hi)) return true;
        const double B = fhi[j + 1], A = flo[j + 1];
        hi = fmin(hi, B - C.dec[j]);  // L_j(v) <= B
        lo = fmax(lo, A - C.acc[j]);  // U_j(v) >= A
        if ((on >> j) & 1u) {
            hi = fmin(hi, (B - c[j] - b[j] * S.umin) / a[j]);
            lo = fmax(lo, (A - c[j] - b[j] * S.umax) / a[j]);
        }
        if (lo > hi + tol(hi)) return true;
        if (lo > hi) lo = hi = 0.5 * (lo + hi);
        flo[j] = lo;
        fhi[j] = hi;
    }
    // position rows p_{m+2} = P1 + ts (v_1 + .. + v_{m+1}) on the lowest / highest trajectories
    double smin = 0.0, smax = 0.0;
    for (int m = 0; m + 2 <= N; ++m) {
        smin += flo[m + 1];
        smax += fhi[m + 1];
        const double pl = P1 + S.ts * smin, ph = P1 + S.ts * smax;
        if (pl > S.pmax + tol(S.pmax) || ph < S.pmin - tol(S.pmin)) return true;
    }
    return false;
}

template <int N>
HVP_HD inline bool l1_infeasible(const hvp_system& S, const Consts& C, const double* prm, uint64_t code, int K,
                                 double rlo, double rhi) {
    return l1_infeasible_rt(S, C, prm[0], prm[1], code, K, rlo, rhi, N);
}

// All rows into the lane's arrays (host build and per-lane use).
template <int N>
HVP_HD inline bool l1_setup(L1Lp<N>& L, const hvp_system& S, const Consts& C, int role, const double* prm,
                            uint64_t code, int K = N, double rlo = 0.0, double rhi = -1.0) {
    return l1_rows<N>(
        S, C, role, prm, code, K, rlo, rhi, L.mh, L.mp,
        [&](int i, const double* g, double sgn, double hh) {
            for (int a = 0; a < N; ++a) L.gh[i][a] = sgn * g[a];
            L.h[i] = hh;
        },
        [&](int j, const double* g, double e0, double w, double alpha) {
            for (int a = 0; a < N; ++a) L.gp[j][a] = g[a];
            L.e0[j] = e0;
            L.wp[j] = w;
            L.al[j] = alpha;
        });
}

// Newton direction for the complementarity targets rc_i = s_i l_i - sigmu (predictor: sigmu = 0;
// centring: sigmu > 0) or s_i l_i + ds_i dl_i - sigmu (corr: the corrector, with the predictor's
// directions held in L); the
// residuals of the current iterate are recomputed here.  Returns false if the N x N Schur
// complement is not positive definite.
template <int N>
HVP_HD inline bool l1_direction(L1Lp<N>& L, double sigmu, bool corr, double* dy, double* dt, double* dsh, double* dlh,
                                double* ds1, double* dl1, double* ds2, double* dl2) {
    const int mh = L.mh, mp = L.mp;
    double K[L1Lp<N>::NT], rhs[N];
    for (int i = 0; i < L1Lp<N>::NT; ++i) K[i] = 0.0;
    for (int i = 0; i < N; ++i) rhs[i] = 0.0;
    // rd_y = sum_h l g + sum_p (l1 - alpha l2) g   (accumulated into rhs with a minus sign)
    for (int i = 0; i < mh; ++i) {
        const double* g = L.gh[i];
        const double gy = l1_dot<N>(g, L.y);
        const double rp = gy + L.sh[i] - L.h[i];
        const double D = L.lh[i] / L.sh[i];
        const double rc = L.sh[i] * L.lh[i] + (corr ? L.dsh[i] * L.dlh[i] : 0.0) - sigmu;
        const double rho = (L.lh[i] * rp - rc) / L.sh[i];
        const double coef = -(L.lh[i] + rho);
        for (int a = 0; a < N; ++a) {
            rhs[a] += coef * g[a];
            for (int b = 0; b <= a; ++b) K[tri(a, b)] += D * g[a] * g[b];
        }
    }
    for (int j = 0; j < mp; ++j) {
        const double* g = L.gp[j];
        const double al = L.al[j];
        const double gy = l1_dot<N>(g, L.y);
        const double rp1 = gy - L.t[j] + L.s1[j] + L.e0[j];
        const double rp2 = -al * gy - L.t[j] + L.s2[j] - al * L.e0[j];
        const double D1 = L.l1[j] / L.s1[j], D2 = L.l2[j] / L.s2[j];
        const double rc1 = L.s1[j] * L.l1[j] + (corr ? L.ds1[j] * L.dl1[j] : 0.0) - sigmu;
        const double rc2 = L.s2[j] * L.l2[j] + (corr ? L.ds2[j] * L.dl2[j] : 0.0) - sigmu;
        const double rho1 = (L.l1[j] * rp1 - rc1) / L.s1[j], rho2 = (L.l2[j] * rp2 - rc2) / L.s2[j];
        const double rdt = L.wp[j] - L.l1[j] - L.l2[j];
        const double rhst = -rdt + rho1 + rho2;
        const double mt = D1 + D2, m = al * D2 - D1;
        const double ce = D1 * D2 * (1.0 + al) * (1.0 + al) / mt;
        // rhs_y -= (l1 - al l2) g + (rho1 - al rho2) g + m g rhs_t / Mtt
        const double coef = -(L.l1[j] - al * L.l2[j]) - (rho1 - al * rho2) - m * rhst / mt;
        for (int a = 0; a < N; ++a) {
            rhs[a] += coef * g[a];
            for (int b = 0; b <= a; ++b) K[tri(a, b)] += ce * g[a] * g[b];
        }
    }
    cholesky_l1<N>(K);
    chol_solve<N>(K, rhs, dy);
    for (int i = 0; i < mh; ++i) {
        const double* g = L.gh[i];
        const double gy = l1_dot<N>(g, L.y), gd = l1_dot<N>(g, dy);
        const double rp = gy + L.sh[i] - L.h[i];
        const double D = L.lh[i] / L.sh[i];
        const double rc = L.sh[i] * L.lh[i] + (corr ? L.dsh[i] * L.dlh[i] : 0.0) - sigmu;
        const double rho = (L.lh[i] * rp - rc) / L.sh[i];
        dsh[i] = -rp - gd;
        dlh[i] = D * gd + rho;
    }
    for (int j = 0; j < mp; ++j) {
        const double* g = L.gp[j];
        const double al = L.al[j];
        const double gy = l1_dot<N>(g, L.y), gd = l1_dot<N>(g, dy);
        const double rp1 = gy - L.t[j] + L.s1[j] + L.e0[j];
        const double rp2 = -al * gy - L.t[j] + L.s2[j] - al * L.e0[j];
        const double D1 = L.l1[j] / L.s1[j], D2 = L.l2[j] / L.s2[j];
        const double rc1 = L.s1[j] * L.l1[j] + (corr ? L.ds1[j] * L.dl1[j] : 0.0) - sigmu;
        const double rc2 = L.s2[j] * L.l2[j] + (corr ? L.ds2[j] * L.dl2[j] : 0.0) - sigmu;
        const double rho1 = (L.l1[j] * rp1 - rc1) / L.s1[j], rho2 = (L.l2[j] * rp2 - rc2) / L.s2[j];
        const double rdt = L.wp[j] - L.l1[j] - L.l2[j];
        const double rhst = -rdt + rho1 + rho2;
        const double mt = D1 + D2, m = al * D2 - D1;
        dt[j] = (rhst - m * gd) / mt;
        const double a1 = gd - dt[j], a2 = -al * gd - dt[j];
        ds1[j] = -rp1 - a1;
        ds2[j] = -rp2 - a2;
        // the multiplier of the side with the smaller scaling from its complementarity row, the
        // other from the t row dl1 + dl2 = w - l1 - l2 exactly: D a of the side with D ~ 1e10
        // carries the cancellation of a = gd - dt (the t row's residual grew iterate by iterate)
        if (D1 >= D2) {
            dl2[j] = D2 * a2 + rho2;
            dl1[j] = rdt - dl2[j];
        } else {
            dl1[j] = D1 * a1 + rho1;
            dl2[j] = rdt - dl1[j];
        }
    }
    return true;
}

HVP_HD inline void l1_ratio(double& a, double v, double dv) {
    if (dv < 0.0) a = fmin(a, -v / dv);
}

// Interior point on the rows of l1_setup.  Returns L1_OK, L1_INFEASIBLE (certificate, l1_farkas,
// velocity box [ylo, yhi]) or L1_FAIL; the iterate is left in L.y.
template <int N>
HVP_HD inline int l1_cert(const L1Lp<N>& L, double ylo, double yhi) {
    double r[N], hl = 0.0, sc = 0.0;
    for (int a = 0; a < N; ++a) r[a] = 0.0;
    for (int i = 0; i < L.mh; ++i) {
        for (int a = 0; a < N; ++a) r[a] += L.lh[i] * L.gh[i][a];
        hl += L.lh[i] * L.h[i];
        sc += fabs(L.lh[i] * L.h[i]);
    }
    return l1_farkas<N>(r, hl, sc, ylo, yhi) ? L1_INFEASIBLE : L1_FAIL;
}

template <int N>
HVP_HD inline int l1_solve(L1Lp<N>& L, double v0, int max_iter, int& iters, double ylo = -1e300, double yhi = 1e300) {
    const int mh = L.mh, mp = L.mp;
    const int mtot = mh + 2 * mp;
    double hscale = 1.0, wmax = 1.0;
    for (int i = 0; i < N; ++i) L.y[i] = v0;
    for (int i = 0; i < mh; ++i) {
        L.sh[i] = fmax(L.h[i] - l1_dot<N>(L.gh[i], L.y), 1.0);
        L.lh[i] = 1.0;
        hscale = fmax(hscale, fabs(L.h[i]));
    }
    for (int j = 0; j < mp; ++j) {
        const double e = l1_dot<N>(L.gp[j], L.y) + L.e0[j];
        L.t[j] = (L.al[j] > 0.0 ? fabs(e) : fmax(e, 0.0)) + 1.0;
        L.s1[j] = L.t[j] - e;
        L.s2[j] = L.t[j] + L.al[j] * e;
        L.l1[j] = 0.5 * L.wp[j];
        L.l2[j] = 0.5 * L.wp[j];
        wmax = fmax(wmax, L.wp[j]);
        hscale = fmax(hscale, fabs(L.e0[j]));
    }
    // the corrector overwrites the predictor's directions in place (row i reads its own
    // predictor ds_i dl_i before writing them), which keeps the lane's private segment small
    double dy[N], dt[L1Lp<N>::MP];
    double *dsh = L.dsh, *dlh = L.dlh, *ds1 = L.ds1, *dl1 = L.dl1, *ds2 = L.ds2, *dl2 = L.dl2;
    for (iters = 0; iters < max_iter; ++iters) {
        // residuals and the duality measure
        double gap = 0.0, obj = 0.0, rpmax = 0.0, rdmax = 0.0;
        double rdy[N];
        for (int a = 0; a < N; ++a) rdy[a] = 0.0;
        for (int i = 0; i < mh; ++i) {
            gap += L.sh[i] * L.lh[i];
            rpmax = fmax(rpmax, fabs(l1_dot<N>(L.gh[i], L.y) + L.sh[i] - L.h[i]));
            for (int a = 0; a < N; ++a) rdy[a] += L.lh[i] * L.gh[i][a];
        }
        for (int j = 0; j < mp; ++j) {
            const double gy = l1_dot<N>(L.gp[j], L.y), al = L.al[j];
            gap += L.s1[j] * L.l1[j] + L.s2[j] * L.l2[j];
            obj += L.wp[j] * L.t[j];
            rpmax = fmax(rpmax, fabs(gy - L.t[j] + L.s1[j] + L.e0[j]));
            rpmax = fmax(rpmax, fabs(-al * gy - L.t[j] + L.s2[j] - al * L.e0[j]));
            rdmax = fmax(rdmax, fabs(L.wp[j] - L.l1[j] - L.l2[j]));
            for (int a = 0; a < N; ++a) rdy[a] += (L.l1[j] - al * L.l2[j]) * L.gp[j][a];
        }
        for (int a = 0; a < N; ++a) rdmax = fmax(rdmax, fabs(rdy[a]));
        if (rpmax <= 1e-10 * hscale && rdmax <= 1e-10 * wmax && gap <= 1e-12 * fmax(1.0, fabs(obj))) return L1_OK;
        const double mu = gap / mtot;
        // predictor
        if (!l1_direction<N>(L, 0.0, false, dy, dt, L.dsh, L.dlh, L.ds1, L.dl1, L.ds2, L.dl2)) return l1_cert<N>(L, ylo, yhi);
        double ap = 1.0, ad = 1.0;
        for (int i = 0; i < mh; ++i) {
            l1_ratio(ap, L.sh[i], L.dsh[i]);
            l1_ratio(ad, L.lh[i], L.dlh[i]);
        }
        for (int j = 0; j < mp; ++j) {
            l1_ratio(ap, L.s1[j], L.ds1[j]);
            l1_ratio(ap, L.s2[j], L.ds2[j]);
            l1_ratio(ad, L.l1[j], L.dl1[j]);
            l1_ratio(ad, L.l2[j], L.dl2[j]);
        }
        double gaff = 0.0;
        for (int i = 0; i < mh; ++i) gaff += (L.sh[i] + ap * L.dsh[i]) * (L.lh[i] + ad * L.dlh[i]);
        for (int j = 0; j < mp; ++j)
            gaff += (L.s1[j] + ap * L.ds1[j]) * (L.l1[j] + ad * L.dl1[j]) +
                    (L.s2[j] + ap * L.ds2[j]) * (L.l2[j] + ad * L.dl2[j]);
        const double ratio = gaff / gap;
        const double sigma = ratio * ratio * ratio;
        // corrector (centring + second-order term); a corrector step shorter than kL1Short is
        // replaced by a pure centring step (the second-order term can lock the iterate into a cycle
        // of short steps near a degenerate optimum)
        for (int pass = 0; pass < 2; ++pass) {
            if (!l1_direction<N>(L, pass ? kL1Centre * mu : sigma * mu, pass == 0, dy, dt, dsh, dlh, ds1, dl1, ds2,
                                 dl2))
                return l1_cert<N>(L, ylo, yhi);
            ap = 1.0 / 0.995;
            ad = 1.0 / 0.995;
            for (int i = 0; i < mh; ++i) {
                l1_ratio(ap, L.sh[i], dsh[i]);
                l1_ratio(ad, L.lh[i], dlh[i]);
            }
            for (int j = 0; j < mp; ++j) {
                l1_ratio(ap, L.s1[j], ds1[j]);
                l1_ratio(ap, L.s2[j], ds2[j]);
                l1_ratio(ad, L.l1[j], dl1[j]);
                l1_ratio(ad, L.l2[j], dl2[j]);
            }
            if (fmin(ap, ad) >= kL1Short) break;
        }
        ap *= 0.995;
        ad *= 0.995;
        for (int a = 0; a < N; ++a) L.y[a] += ap * dy[a];
        for (int i = 0; i < mh; ++i) {
            L.sh[i] += ap * dsh[i];
            L.lh[i] += ad * dlh[i];
        }
        for (int j = 0; j < mp; ++j) {
            L.t[j] += ap * dt[j];
            L.s1[j] += ap * ds1[j];
            L.s2[j] += ap * ds2[j];
            L.l1[j] += ad * dl1[j];
            L.l2[j] += ad * dl2[j];
        }
    }
    return l1_cert<N>(L, ylo, yhi);
}

// Objective of a trajectory (y = v_1 .. v_N under region code), term by term as the reference
// writes it with min_1_norm (fleet_decent_mld.py:107-169): Q_ii |e_i| of the tracking errors,
// Q_u |u|, Q_du |du| and w * max(0, .) slacks, constants included.  K < N: the objective of the
// relaxation of the prefix (l1_steps: virtual-region inputs priced, dropped ones not, Q_du only
// between decided steps) -- the branch-and-bound bound.
template <int N>
HVP_HD inline double l1_direct_cost(const double* y, const hvp_system& S, const Consts& C, int role, const double* prm,
                                    uint64_t code, int K = N, double rlo = 0.0, double rhi = -1.0, int xl_blk = 4) {
    const double* xf = prm + 2;
    const double* xb = prm + 2 + 2 * (N + 1);
    const double* xl = prm + 2 + xl_blk * (N + 1);
    const int K1 = N + 1;
    const bool tf = (role & HVP_ROLE_TRACK_FRONT) != 0, tb = (role & HVP_ROLE_TRACK_BACK) != 0;
    const bool tl = (role & HVP_ROLE_TRACK_LEADER) != 0, lsp = (role & HVP_ROLE_LEADER_SPACING) != 0;
    const bool sf = (role & HVP_ROLE_SAFE_FRONT) != 0, sb = (role & HVP_ROLE_SAFE_BACK) != 0;
    double a[N], b[N], c[N], vlo[N], vhi[N];
    unsigned on;
    l1_steps<N>(S, C, code, K, rlo, rhi, a, b, c, on, vlo, vhi);
    double J = 0.0, p = prm[0], v = prm[1], uprev = 0.0;
    for (int k = 0; k <= N; ++k) {
        auto nrm = [&](double ep, double ev) { return C.Qpp * fabs(ep) + C.Qvv * fabs(ev); };
        if (tf) J += nrm(p + C.t0 * v + C.d0 - xf[k], v - xf[K1 + k]);
        if (tb) J += nrm(xb[k] + C.t0 * xb[K1 + k] + C.d0 - p, xb[K1 + k] - v);
        if (tl) J += nrm(p - xl[k] + (lsp ? C.t0 * v + C.d0 : 0.0), v - xl[K1 + k]);
        if (sf) J += C.w * fmax(0.0, p - xf[k] + C.d_safe);
        if (sb) J += C.w * fmax(0.0, xb[k] + C.d_safe - p);
        if (k < N) {
            const double u = (y[k] - a[k] * v - c[k]) / b[k];
            if ((on >> k) & 1u) J += C.Qu * fabs(u);
            if (k >= 1 && k < K) J += C.Qdu * fabs(u - uprev);
            uprev = u;
            p = p + S.ts * v;
            v = y[k];
        }
    }
    return J;
}

// ---- naive ADMM with min_1_norm: the exact copies of a trajectory
// A copy group (side, step k) of LocalMpcADMM(quadratic_cost=False) (fleet_naive_admm.py:74-77)
// given the own state (p_k, v_k): c = (c_p, c_v) minimises rho/2 |c - m|^2 (the ADMM terms,
// :172-198, m = z - y / rho) + sum_j w+_j max(e_j, 0) + w-_j max(-e_j, 0), e_j = a_j . c + b_j (the
// copy's L1 tracking terms, :110-133, and its soft safe row, :205-236).  The interior point leaves c
// ~1e-9 off the safe row's kink, where w = 1e4 turns that into ~1e-5 of objective; the exact
// minimiser is the stationary point of one kink pattern (each term > 0, < 0 or at its kink), so the
// patterns' points are compared by the objective and the best taken.  l1_admm_node_lp prices the
// trajectory and returns the copies with it.
struct CopyTerms {
    int nt;
    double a[3][2], b[3], wp[3], wn[3];
};

HVP_HD inline double copy_objective(const CopyTerms& T, double rho, const double* m, double c0, double c1) {
    double f = 0.5 * rho * ((c0 - m[0]) * (c0 - m[0]) + (c1 - m[1]) * (c1 - m[1]));
    for (int j = 0; j < T.nt; ++j) {
        const double e = T.a[j][0] * c0 + T.a[j][1] * c1 + T.b[j];
        f += e > 0.0 ? T.wp[j] * e : -T.wn[j] * e;
    }
    return f;
}

HVP_HD inline void copy_exact(const CopyTerms& T, double rho, const double* m, double* c) {
    double best = 1e308;
    c[0] = m[0];
    c[1] = m[1];
    int npat = 1;
    for (int j = 0; j < T.nt; ++j) npat *= 3;
    for (int pat = 0; pat < npat; ++pat) {
        int kink[2] = {-1, -1}, nk = 0, r = pat;
        double g0 = 0.0, g1 = 0.0;
        for (int j = 0; j < T.nt; ++j, r /= 3) {
            const int s = r % 3;  // 0 kink, 1 e > 0, 2 e < 0
            if (s == 0) {
                if (nk < 2) kink[nk] = j;
                ++nk;
            } else {
                const double sl = s == 1 ? T.wp[j] : -T.wn[j];
                g0 += sl * T.a[j][0];
                g1 += sl * T.a[j][1];
            }
        }
        if (nk > 2) continue;
        const double f0 = m[0] - g0 / rho, f1 = m[1] - g1 / rho;
        double x0 = f0, x1 = f1;
        if (nk == 1) {
            const double* a = T.a[kink[0]];
            const double aa = a[0] * a[0] + a[1] * a[1];
            if (!(aa > 0.0)) continue;
            const double mu = (a[0] * f0 + a[1] * f1 + T.b[kink[0]]) / aa;  // lambda / rho
            x0 = f0 - a[0] * mu;
            x1 = f1 - a[1] * mu;
        } else if (nk == 2) {
            const double *a = T.a[kink[0]], *d = T.a[kink[1]];
            const double m00 = a[0] * a[0] + a[1] * a[1], m01 = a[0] * d[0] + a[1] * d[1], m11 = d[0] * d[0] + d[1] * d[1];
            const double det = m00 * m11 - m01 * m01;
            if (!(fabs(det) > 1e-12 * (m00 * m11 + 1e-300))) continue;
            const double r0 = a[0] * f0 + a[1] * f1 + T.b[kink[0]], r1 = d[0] * f0 + d[1] * f1 + T.b[kink[1]];
            const double u0 = (m11 * r0 - m01 * r1) / det, u1 = (m00 * r1 - m01 * r0) / det;
            x0 = f0 - a[0] * u0 - d[0] * u1;
            x1 = f1 - a[1] * u0 - d[1] * u1;
        }
        const double f = copy_objective(T, rho, m, x0, x1);
        if (f < best) {
            best = f;
            c[0] = x0;
            c[1] = x1;
        }
    }
}

// the terms of copy group (side, k) at own state (p, v) (roles: HVP_ROLE_SAFE_* = the copy exists,
// HVP_ROLE_TRACK_* = its tracking terms)
HVP_HD inline CopyTerms copy_terms(const Consts& C, int role, int side, double p, double v) {
    CopyTerms T;
    T.nt = 0;
    const bool tr = (role & (side == 0 ? HVP_ROLE_TRACK_FRONT : HVP_ROLE_TRACK_BACK)) != 0;
    auto add = [&](double a0, double a1, double b, double wp, double wn) {
        T.a[T.nt][0] = a0;
        T.a[T.nt][1] = a1;
        T.b[T.nt] = b;
        T.wp[T.nt] = wp;
        T.wn[T.nt] = wn;
        ++T.nt;
    };
    if (tr && side == 0) {  // p + t0 v + d0 - c_p ; v - c_v
        add(-1.0, 0.0, p + C.t0 * v + C.d0, C.Qpp, C.Qpp);
        add(0.0, -1.0, v, C.Qvv, C.Qvv);
    } else if (tr) {  // c_p + t0 c_v + d0 - p ; c_v - v
        add(1.0, C.t0, C.d0 - p, C.Qpp, C.Qpp);
        add(0.0, 1.0, -v, C.Qvv, C.Qvv);
    }
    if (side == 0) add(-1.0, 0.0, p + C.d_safe, C.w, 0.0);  // w max(0, p - c_p + d_safe)
    else add(1.0, 0.0, C.d_safe - p, C.w, 0.0);            // w max(0, c_p + d_safe - p)
    return T;
}

}  // namespace hvp
