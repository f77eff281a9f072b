// hvp_lp.h -- the fixed-sequence LP of the min_1_norm local MPC by a per-lane simplex method.
//
// Same LP as hvp_l1.h (LocalMpcMld.setup_cost_and_constraints(quadratic_cost=False),
// fleet_decent_mld.py:73-76 and :107-208; rows and terms exactly those of l1_rows): in velocity
// space y = (v_1 .. v_N) minimise
//     F(y) = sum_h  s+_h max(0, z_h(y)) + s-_h max(0, -z_h(y)),     z_h(y) = a_h . y + b_h,
// a convex piecewise-linear function of N <= 8 variables.  Every term is one hyperplane z_h = 0:
//   * the L1 terms Q |e| (s+ = s- = Q) and the soft safe rows w max(0, .) (s+ = w, s- = 0);
//   * the hard rows (V, U, A, P) as walls with an exact penalty M on the violating side
//     (s+ = M, s- = 0 for g.y <= h; M > every multiplier of the LP, so the minimiser is the LP's
//     optimum -- checked at the end: a violated hard row leaves the LP unresolved, L1_FAIL).
// Every normal is structured: cp ts (e_0 + .. + e_m) + c0 e_j + c1 e_{j-1} + c2 e_{j-2} (a prefix
// for positions, at most three consecutive velocities for v, u, du and the accel rows), so a term's
// value at y or along a direction d is O(1) from the prefix sums of y / d; no per-term state is kept.
//
// Method: the primal simplex on F (Barrodale-Roberts style long steps).  A vertex is N basic
// hyperplanes (A_B y = -b_B, A_B's inverse kept explicitly, N x N).  Edge (k, side): leave basic
// hyperplane k to one side, along d = +-A_B^-1 e_k; its directional derivative is
// +-(A_B^-T g)_k + s_k(side) with g the gradient of the nonbasic terms.  The most negative edge is
// followed through the breakpoints of the nonbasic terms (the derivative grows by (s+ + s-)|a_h.d|
// at each) until it turns non-negative; that hyperplane enters the basis.  At an optimal vertex
// every edge derivative is >= 0 (the basic multipliers lie in their [-s-, s+] boxes: the LP's dual
// certificate).  Degenerate (zero-length) pivots switch to Bland's rule with single steps, which
// cannot cycle.  Start: the vertex of the V rows nearest v0 (A_B = I).
//
// Per lane the state is y, A_B^-1 and the basis ids -- what the Goldfarb-Idnani lane solver of the
// quadratic path keeps -- so one LP runs per LANE (64 per wavefront), where the interior point of
// hvp_l1.h needs a wavefront per LP.  The cost the search compares is l1_direct_cost of the vertex.
#pragma once

#include "hvp_l1.h"

namespace hvp {

// Term ids (Bland's rule and the basis refer to them):
//   6 j + {0 V_lo, 1 V_hi, 2 U_lo, 3 U_hi, 4 A_lo, 5 A_hi}               hard, step j = 0..N-1
//   6 N + 2 m + {0 P_lo, 1 P_hi}                                          hard, p_{m+2}, m = 0..N-2
//   8 N - 2 + 8 j + {0 F_p, 1 F_v, 2 B_p, 3 B_v, 4 L_p, 5 L_v, 6 SF, 7 SB}  state k = j + 1
//   16 N - 2 + 2 j + {0 U, 1 DU}                                          inputs of step j
template <int N>
constexpr int kLpTerms = 18 * N - 2;

enum { LP_OK = 0, LP_FAIL = 2 };

// one hyperplane: z = cp (y_0 + .. + y_m) + c0 y_j + c1 y_{j-1} + c2 y_{j-2} + b  (m < 0: no
// prefix part; cp includes ts), cost sp max(0, z) + sm max(0, -z)
struct LpHyp {
    int m, j;
    double cp, c0, c1, c2, b, sp, sm;
};

// per-step fields of an LP (a lane's row of per-step data; the device keeps them in LDS, where a
// lane reads them at a data-dependent step without spilling, hvp_lane.h LpLdsMem)
enum { LF_A = 0, LF_B, LF_IB, LF_C, LF_VLO, LF_VHI, LF_DEC, LF_ACC, LF_COUNT };

template <int N>
struct LpArrayMem {
    double v[LF_COUNT * N];
    HVP_HD double get(int f, int j) const { return v[f * N + j]; }
    HVP_HD void set(int f, int j, double x) { v[f * N + j] = x; }
};

// The per-lane data of one (node) LP: the instance (prm, role), the step data of l1_steps and the
// exact penalty of the hard rows.
template <int N, class MEM = LpArrayMem<N>>
struct LpData {
    const double* prm;
    int role, K;
    unsigned on;
    double v0, P1, ts, pmin, pmax, umin, umax, M;
    MEM mem;
};

template <int N, class MEM>
HVP_HD inline void lp_data(LpData<N, MEM>& D, const hvp_system& S, const Consts& C, int role, const double* prm,
                           uint64_t code, int K, double rlo, double rhi) {
    double a[N], b[N], c[N], vlo[N], vhi[N];
    l1_steps<N>(S, C, code, K, rlo, rhi, a, b, c, D.on, vlo, vhi);
#pragma unroll
    for (int k = 0; k < N; ++k) {
        D.mem.set(LF_A, k, a[k]);
        D.mem.set(LF_B, k, b[k]);
        D.mem.set(LF_IB, k, 1.0 / b[k]);
        D.mem.set(LF_C, k, c[k]);
        D.mem.set(LF_VLO, k, vlo[k]);
        D.mem.set(LF_VHI, k, vhi[k]);
        D.mem.set(LF_DEC, k, C.dec[k]);
        D.mem.set(LF_ACC, k, C.acc[k]);
    }
    D.prm = prm;
    D.role = role;
    D.K = K;
    D.v0 = prm[1];
    D.ts = S.ts;
    D.P1 = prm[0] + S.ts * prm[1];
    D.pmin = S.pmin;
    D.pmax = S.pmax;
    D.umin = S.umin;
    D.umax = S.umax;
    // exact penalty: above any multiplier of the hard rows (bounded by the weights times the
    // basis condition of these bidiagonal / prefix rows, a few N)
    D.M = 1e4 * (C.Qpp + C.Qvv + C.Qu + C.Qdu + C.w + 1.0);
}

// Hyperplane `id` of the LP (false: the term is absent -- its role bit is off, its weight zero, its
// step relaxed without an input, or its normal vanishes (a constant term, priced by the direct
// cost only)).  Mirrors l1_rows term by term.
template <int N, class MEM>
HVP_HD inline bool lp_hyp(const LpData<N, MEM>& D, const Consts& C, int id, LpHyp& h) {
    h.m = -1;
    h.j = 0;
    h.cp = h.c0 = h.c1 = h.c2 = 0.0;
    h.sp = h.sm = 0.0;
    h.b = 0.0;
    const double M = D.M;
    if (id < 6 * N) {  // V, U, A of step j
        const int j = id / 6, r = id % 6;
        const bool hi = r & 1;
        h.j = j;
        h.c0 = 1.0;
        h.sp = hi ? M : 0.0;
        h.sm = hi ? 0.0 : M;
        if (r < 2) {
            h.b = -D.mem.get(hi ? LF_VHI : LF_VLO, j);
            return true;
        }
        if (r < 4) {
            if (!((D.on >> j) & 1u)) return false;
            const double aj = D.mem.get(LF_A, j);
            const double cu = j == 0 ? aj * D.v0 : 0.0;
            h.c1 = j ? -aj : 0.0;
            h.b = -(D.mem.get(LF_C, j) + D.mem.get(LF_B, j) * (hi ? D.umax : D.umin) + cu);
            return true;
        }
        const double ca = j == 0 ? D.v0 : 0.0;
        h.c1 = j ? -1.0 : 0.0;
        h.b = -(D.mem.get(hi ? LF_ACC : LF_DEC, j) + ca);
        return true;
    }
    if (id < 8 * N - 2) {  // P: pmin <= p_{m+2} <= pmax
        const int m = (id - 6 * N) / 2;
        const bool hi = (id - 6 * N) & 1;
        h.m = m;
        h.cp = D.ts;
        h.b = hi ? D.P1 - D.pmax : D.P1 - D.pmin;
        h.sp = hi ? M : 0.0;
        h.sm = hi ? 0.0 : M;
        return true;
    }
    const int K1 = N + 1;
    const double* xf = D.prm + 2;
    const double* xb = D.prm + 2 + 2 * K1;
    const double* xl = D.prm + 2 + 4 * K1;
    if (id < 16 * N - 2) {
        const int j = (id - (8 * N - 2)) / 8, r = (id - (8 * N - 2)) % 8;
        const int k = j + 1;  // state k: p_k = P1 + ts (y_0 + .. + y_{k-2}), v_k = y_{k-1} = y_j
        const int role = D.role;
        const bool pos = (r & 1) == 0;
        double w = 0.0;
        h.j = j;
        if (r < 6) {
            const int side = r / 2;  // 0 front, 1 back, 2 leader
            const int bit = side == 0 ? HVP_ROLE_TRACK_FRONT : (side == 1 ? HVP_ROLE_TRACK_BACK : HVP_ROLE_TRACK_LEADER);
            if (!(role & bit)) return false;
            w = pos ? C.Qpp : C.Qvv;
            if (pos) {
                const bool lsp = (role & HVP_ROLE_LEADER_SPACING) != 0;
                const double sg = side == 1 ? -1.0 : 1.0;
                h.m = k - 2;
                h.cp = sg * D.ts;
                h.c0 = side == 0 ? C.t0 : (side == 2 && lsp ? C.t0 : 0.0);
                if (side == 0) h.b = D.P1 + C.d0 - xf[k];
                else if (side == 1) h.b = xb[k] + C.t0 * xb[K1 + k] + C.d0 - D.P1;
                else h.b = D.P1 - xl[k] + (lsp ? C.d0 : 0.0);
            } else {
                h.c0 = side == 1 ? -1.0 : 1.0;
                h.b = side == 0 ? -xf[K1 + k] : (side == 1 ? xb[K1 + k] : -xl[K1 + k]);
            }
            h.sp = h.sm = w;
        } else {
            if (k < 2) return false;
            const bool front = r == 6;
            if (!(role & (front ? HVP_ROLE_SAFE_FRONT : HVP_ROLE_SAFE_BACK))) return false;
            w = C.w;
            h.m = k - 2;
            h.cp = front ? D.ts : -D.ts;
            h.b = front ? D.P1 - xf[k] + C.d_safe : xb[k] + C.d_safe - D.P1;
            h.sp = w;
            h.sm = 0.0;
        }
        if (!(w > 0.0)) return false;
        return h.m >= 0 ? true : h.c0 != 0.0;  // m < 0 and c0 = 0: a constant term
    }
    // inputs: u_j = ubar_j + ib_j y_j - a_j ib_j y_{j-1}; du_j = u_j - u_{j-1}
    const int j = (id - (16 * N - 2)) / 2;
    const bool du = ((id - (16 * N - 2)) & 1) != 0;
    h.j = j;
    const double aj = D.mem.get(LF_A, j), ibj = D.mem.get(LF_IB, j);
    const double ubar = j == 0 ? -(aj * D.v0 + D.mem.get(LF_C, 0)) * ibj : -D.mem.get(LF_C, j) * ibj;
    if (!du) {
        if (!((D.on >> j) & 1u) || !(C.Qu > 0.0)) return false;
        h.c0 = ibj;
        h.c1 = j ? -aj * ibj : 0.0;
        h.b = ubar;
        h.sp = h.sm = C.Qu;
        return true;
    }
    if (j < 1 || j >= D.K || !(C.Qdu > 0.0)) return false;
    const double ap = D.mem.get(LF_A, j - 1), ibp = D.mem.get(LF_IB, j - 1);
    const double ubp = j - 1 == 0 ? -(ap * D.v0 + D.mem.get(LF_C, 0)) * ibp : -D.mem.get(LF_C, j - 1) * ibp;
    h.c0 = ibj;
    h.c1 = -aj * ibj - ibp;
    h.c2 = j >= 2 ? ap * ibp : 0.0;
    h.b = ubar - ubp;
    h.sp = h.sm = C.Qdu;
    return true;
}

// a . x from x and its prefix sums X (X[m] = x_0 + .. + x_m); h.j, h.m are compile-time constants
// where the caller unrolls its loop over the term ids (no dynamic register indexing)
template <int N>
HVP_HD inline double lp_dot(const LpHyp& h, const double* x, const double* X) {
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        s += i == h.j ? h.c0 * x[i] : 0.0;
        s += i + 1 == h.j ? h.c1 * x[i] : 0.0;
        s += i + 2 == h.j ? h.c2 * x[i] : 0.0;
        s += i == h.m ? h.cp * X[i] : 0.0;
    }
    return s;
}

template <int N>
HVP_HD inline void lp_prefix(const double* x, double* X) {
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        s += x[i];
        X[i] = s;
    }
}

// dense normal of hyperplane h
template <int N>
HVP_HD inline void lp_normal(const LpHyp& h, double* a) {
#pragma unroll
    for (int i = 0; i < N; ++i)
        a[i] = (i <= h.m ? h.cp : 0.0) + (i == h.j ? h.c0 : 0.0) + (i + 1 == h.j ? h.c1 : 0.0) + (i + 2 == h.j ? h.c2 : 0.0);
}

// ---- the scans over the terms, step by step.  Every term of step j (its V, U, A rows, the P rows
// of p_{j+1}, the tracking / safe terms of state j + 1, the input terms of step j: 18 per step, 16
// at j = 0) is z = cp X_{j-1} + c0 x_j + c1 x_{j-1} + c2 x_{j-2} + b with coefficients whose
// STRUCTURE is fixed per term type (lp_hyp's, term for term); a scan loops over the steps (uniform
// j, rolled) and visits the 18 terms with that structure known at compile time -- a handful of
// FMAs per term from four primitives of y (and of the direction), where a lookup by term id
// (lp_hyp) costs a run-time decode and selects per term.  lp_hyp stays for the basis lookups.
struct LpPrim {
    double x0, x1, x2, p1;  // x_j, x_{j-1}, x_{j-2}, X_{j-1} (0 where the index is < 0)
};
template <int N>
HVP_HD inline LpPrim lp_prim(const double* x, const double* X, int j) {
    LpPrim r{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int i = 0; i < N; ++i) {
        r.x0 = i == j ? x[i] : r.x0;
        r.x1 = i + 1 == j ? x[i] : r.x1;
        r.x2 = i + 2 == j ? x[i] : r.x2;
        r.p1 = i + 1 == j ? X[i] : r.p1;
    }
    return r;
}
struct LpTerm {
    int id;
    bool ok;  // present (lp_hyp's true)
    double cp, c0, c1, c2, b, sp, sm;
};
// a . x in lp_dot's summation order (c2, c1, cp, c0)
HVP_HD inline double lp_val(const LpTerm& t, const LpPrim& p) {
    double s = t.c2 * p.x2;
    s += t.c1 * p.x1;
    s += t.cp * p.p1;
    s += t.c0 * p.x0;
    return s;
}
template <int N, class MEM, class F>
HVP_HD inline void lp_step_terms(const LpData<N, MEM>& D, const Consts& C, int j, F&& f) {
    const int k = j + 1, K1 = N + 1;
    const double M = D.M;
    const double aj = D.mem.get(LF_A, j), bj = D.mem.get(LF_B, j), ibj = D.mem.get(LF_IB, j);
    const double cj = D.mem.get(LF_C, j);
    const bool on = ((D.on >> j) & 1u) != 0;
    // V, U, A rows of step j (hard)
    f(LpTerm{6 * j + 0, true, 0.0, 1.0, 0.0, 0.0, -D.mem.get(LF_VLO, j), 0.0, M});
    f(LpTerm{6 * j + 1, true, 0.0, 1.0, 0.0, 0.0, -D.mem.get(LF_VHI, j), M, 0.0});
    const double cu = j == 0 ? aj * D.v0 : 0.0;
    const double c1u = j ? -aj : 0.0;
    f(LpTerm{6 * j + 2, on, 0.0, 1.0, c1u, 0.0, -(cj + bj * D.umin + cu), 0.0, M});
    f(LpTerm{6 * j + 3, on, 0.0, 1.0, c1u, 0.0, -(cj + bj * D.umax + cu), M, 0.0});
    const double ca = j == 0 ? D.v0 : 0.0;
    const double c1a = j ? -1.0 : 0.0;
    f(LpTerm{6 * j + 4, true, 0.0, 1.0, c1a, 0.0, -(D.mem.get(LF_DEC, j) + ca), 0.0, M});
    f(LpTerm{6 * j + 5, true, 0.0, 1.0, c1a, 0.0, -(D.mem.get(LF_ACC, j) + ca), M, 0.0});
    // P rows of p_{j+1} (prefix m = j - 1; none at j = 0)
    const double cpj = j >= 1 ? D.ts : 0.0;
    f(LpTerm{6 * N + 2 * (j - 1), j >= 1, cpj, 0.0, 0.0, 0.0, D.P1 - D.pmin, 0.0, M});
    f(LpTerm{6 * N + 2 * (j - 1) + 1, j >= 1, cpj, 0.0, 0.0, 0.0, D.P1 - D.pmax, M, 0.0});
    // tracking and safe terms of state k = j + 1
    const double* xf = D.prm + 2;
    const double* xb = D.prm + 2 + 2 * K1;
    const double* xl = D.prm + 2 + 4 * K1;
    const int role = D.role;
    const bool tf = (role & HVP_ROLE_TRACK_FRONT) != 0, tb = (role & HVP_ROLE_TRACK_BACK) != 0;
    const bool tl = (role & HVP_ROLE_TRACK_LEADER) != 0, lsp = (role & HVP_ROLE_LEADER_SPACING) != 0;
    const bool qp = C.Qpp > 0.0, qv = C.Qvv > 0.0;
    const double xfk = xf[k], xfv = xf[K1 + k], xbk = xb[k], xbv = xb[K1 + k], xlk = xl[k], xlv = xl[K1 + k];
    const int base = 8 * N - 2 + 8 * j;
    f(LpTerm{base + 0, tf && qp && (j >= 1 || C.t0 != 0.0), cpj, C.t0, 0.0, 0.0, D.P1 + C.d0 - xfk, C.Qpp, C.Qpp});
    f(LpTerm{base + 1, tf && qv, 0.0, 1.0, 0.0, 0.0, -xfv, C.Qvv, C.Qvv});
    f(LpTerm{base + 2, tb && qp && j >= 1, -cpj, 0.0, 0.0, 0.0, xbk + C.t0 * xbv + C.d0 - D.P1, C.Qpp, C.Qpp});
    f(LpTerm{base + 3, tb && qv, 0.0, -1.0, 0.0, 0.0, xbv, C.Qvv, C.Qvv});
    const double c0l = lsp ? C.t0 : 0.0;
    f(LpTerm{base + 4, tl && qp && (j >= 1 || c0l != 0.0), cpj, c0l, 0.0, 0.0, D.P1 - xlk + (lsp ? C.d0 : 0.0),
             C.Qpp, C.Qpp});
    f(LpTerm{base + 5, tl && qv, 0.0, 1.0, 0.0, 0.0, -xlv, C.Qvv, C.Qvv});
    const bool qw = C.w > 0.0;
    f(LpTerm{base + 6, j >= 1 && qw && (role & HVP_ROLE_SAFE_FRONT) != 0, cpj, 0.0, 0.0, 0.0, D.P1 - xfk + C.d_safe,
             C.w, 0.0});
    f(LpTerm{base + 7, j >= 1 && qw && (role & HVP_ROLE_SAFE_BACK) != 0, -cpj, 0.0, 0.0, 0.0, xbk + C.d_safe - D.P1,
             C.w, 0.0});
    // input terms of step j: Q_u |u_j|, Q_du |u_j - u_{j-1}| (u_j = ubar_j + ib_j y_j - a_j ib_j y_{j-1})
    const double ubar = -(cu + cj) * ibj;
    f(LpTerm{16 * N - 2 + 2 * j, on && C.Qu > 0.0, 0.0, ibj, j ? -aj * ibj : 0.0, 0.0, ubar, C.Qu, C.Qu});
    const int jp = j >= 1 ? j - 1 : 0;
    const double ap = D.mem.get(LF_A, jp), ibp = D.mem.get(LF_IB, jp);
    const double ubp = jp == 0 ? -(ap * D.v0 + D.mem.get(LF_C, 0)) * ibp : -D.mem.get(LF_C, jp) * ibp;
    f(LpTerm{16 * N - 2 + 2 * j + 1, j >= 1 && j < D.K && C.Qdu > 0.0, 0.0, ibj, -aj * ibj - ibp,
             j >= 2 ? ap * ibp : 0.0, ubar - ubp, C.Qdu, C.Qdu});
}

// inverse of the basis matrix (rows = basic normals) by Gauss-Jordan with partial pivoting, all
// indices static (the pivot row is swapped in by selects); false if singular
template <int N, class MEM>
HVP_HD inline bool lp_invert(const LpData<N, MEM>& D, const Consts& C, const int* basis, double (*Bi)[N]) {
    double A[N][N];
#pragma unroll
    for (int r = 0; r < N; ++r) {
        LpHyp h;
        lp_hyp<N>(D, C, basis[r], h);
        lp_normal<N>(h, A[r]);
#pragma unroll
        for (int c = 0; c < N; ++c) Bi[r][c] = r == c ? 1.0 : 0.0;
    }
    bool ok = true;
#pragma unroll
    for (int col = 0; col < N; ++col) {
        int piv = col;
        double best = fabs(A[col][col]);
#pragma unroll
        for (int r = col + 1; r < N; ++r) {
            const bool bt = fabs(A[r][col]) > best;
            best = bt ? fabs(A[r][col]) : best;
            piv = bt ? r : piv;
        }
        ok = ok && best > 1e-14;
        // swap rows col and piv
#pragma unroll
        for (int r = col + 1; r < N; ++r) {
            const bool sw = r == piv;
#pragma unroll
            for (int c = 0; c < N; ++c) {
                const double a0 = A[col][c], a1 = A[r][c], b0 = Bi[col][c], b1 = Bi[r][c];
                A[col][c] = sw ? a1 : a0;
                A[r][c] = sw ? a0 : a1;
                Bi[col][c] = sw ? b1 : b0;
                Bi[r][c] = sw ? b0 : b1;
            }
        }
        const double ip = best > 1e-14 ? 1.0 / A[col][col] : 0.0;
#pragma unroll
        for (int c = 0; c < N; ++c) {
            A[col][c] *= ip;
            Bi[col][c] *= ip;
        }
#pragma unroll
        for (int r = 0; r < N; ++r) {
            if (r == col) continue;
            const double f = A[r][col];
#pragma unroll
            for (int c = 0; c < N; ++c) {
                A[r][c] -= f * A[col][c];
                Bi[r][c] -= f * Bi[col][c];
            }
        }
    }
    return ok;
}

// The LP by the simplex method.  On LP_OK y holds an optimal vertex.  iters: pivots.
#ifndef HVP_LP_WHY
#define HVP_LP_WHY(code) (void)0
#endif
#ifndef HVP_LP_TRACE
#define HVP_LP_TRACE(...) (void)0
#endif
#ifndef HVP_LP_PASS
#define HVP_LP_PASS() (void)0
#endif
// The simplex state of one LP (per lane): basis, A_B^-1 and the basic terms' data, the recorded
// sides of the kink terms, counters, and the phase of the current pivot.  init() sets the start
// vertex; every trip() runs ONE scan over the terms -- the gradient at the vertex (GRAD), one pass
// of the ratio test along the chosen edge (RATIO), or the final check of the hard rows (CHECK) --
// so that the lanes of a wavefront, whatever phase of whatever LP they are in, execute the same
// scan together (one pivot used to be a gradient scan plus 1 to N+ ratio passes, and a wave ran as
// many passes as its slowest lane: lane utilisation 0.22, profiles/r04k_decent_n10_N5_l1_*).  The
// rebuild of A_B^-1 (every kLpRefresh pivots, and to confirm an optimum on an exact inverse) is a
// phase of its own (INV), run when the caller says so (`do_inv`: the refill kernel batches the
// lanes that wait for it, a rebuild costs about one scan; lp_simplex always).  Returns LP_RUN until
// the LP ends (LP_OK with the vertex in y, or LP_FAIL).  The arithmetic and its order are the
// one-pivot-per-call version's, so pivots, vertices and iteration counts are unchanged.
enum { LP_RUN = 1 };
enum { LPH_GRAD = 0, LPH_RATIO = 1, LPH_CHECK = 2, LPH_INV = 3 };
template <int N>
struct LpLane {
    static constexpr int NT = kLpTerms<N>;
    static constexpr int NW = (NT + 63) / 64;
    static constexpr int kLpRefresh = 12;  // pivots between rebuilds of A_B^-1 (rank-1 updates between)
    int basis[N];
    double Bi[N][N];  // A_B^-1 (A_B y = -b_B)
    // the basic terms' offsets and slopes (updated at each pivot: no lookup of basic terms per
    // iteration)
    double bB[N], spB[N], smB[N];
    // side of every nonbasic term that sits on its kink (|z| <= its tolerance): bit set = the '-'
    // side.  A term keeps the side it was left on (a basic term leaving to one side, a breakpoint
    // crossed), so a degenerate vertex is priced consistently from pivot to pivot -- what makes
    // Bland's rule terminate.  Initially the cheaper side.  (Words selected by static index.)
    uint64_t neg[NW];
    int since, iters;
    bool bland;
    // the pivot in progress: phase, the edge (basic position ek left to side esd, derivative eD),
    // its direction d, and the ratio test's running slope / last breakpoint / passes
    int phase, ek, esd, idprev, passes;
    double eD, slope, tprev, dmax;
    double d[N];

    HVP_HD bool neg_bit(int id) const {
        uint64_t wd = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) wd = (id >> 6) == w ? neg[w] : wd;
        return ((wd >> (id & 63)) & 1ull) != 0;
    }
    HVP_HD void set_side(int id, int side) {
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            const uint64_t bit = (id >> 6) == w ? 1ull << (id & 63) : 0ull;
            neg[w] = side < 0 ? (neg[w] | bit) : (neg[w] & ~bit);
        }
    }
    HVP_HD bool is_basic(int id) const {
        bool b = false;
#pragma unroll
        for (int r = 0; r < N; ++r) b = b || basis[r] == id;
        return b;
    }

    // start: the V rows nearest v0 (A_B = I)
    template <class MEM>
    HVP_HD HVP_FORCEINLINE void init(const LpData<N, MEM>& D, const Consts& C) {
        since = 0;
        iters = 0;
        bland = false;
        phase = LPH_GRAD;
#pragma unroll
        for (int j = 0; j < N; ++j) d[j] = 0.0;
        dmax = 0.0;
#pragma unroll
        for (int j = 0; j < N; ++j) {
            const double vlo = D.mem.get(LF_VLO, j), vhi = D.mem.get(LF_VHI, j);
            const bool up = fabs(vhi - D.v0) < fabs(D.v0 - vlo);
            basis[j] = 6 * j + (up ? 1 : 0);
            bB[j] = -(up ? vhi : vlo);
            spB[j] = up ? D.M : 0.0;
            smB[j] = up ? 0.0 : D.M;
#pragma unroll
            for (int c = 0; c < N; ++c) Bi[j][c] = j == c ? 1.0 : 0.0;
        }
#pragma unroll
        for (int w = 0; w < NW; ++w) neg[w] = 0ull;
#pragma unroll 1
        for (int j = 0; j < N; ++j)
            lp_step_terms<N>(D, C, j, [&](const LpTerm& t) {
                if (!(t.ok && t.sp > t.sm)) return;
#pragma unroll
                for (int w = 0; w < NW; ++w) neg[w] |= (t.id >> 6) == w ? 1ull << (t.id & 63) : 0ull;
            });
    }

    // the LP is waiting for a rebuild of A_B^-1 (the caller's do_inv batches these)
    HVP_HD bool wants_inv() const { return phase == LPH_INV; }

    template <class MEM>
    HVP_HD HVP_FORCEINLINE int trip(const LpData<N, MEM>& D, const Consts& C, int max_iter, double* y,
                                    bool do_inv = true) {
        const double wmax = fmax(fmax(C.Qpp, C.Qvv), fmax(fmax(C.Qu, C.Qdu), fmax(C.w, 1e-300)));
        const double dtol = 1e-11 * wmax;  // edge derivatives within -dtol of zero count as >= 0
        if (phase == LPH_INV) {
            if (!do_inv) return LP_RUN;  // waits for the wave's batch
            if (!lp_invert<N>(D, C, basis, Bi)) {
                HVP_LP_WHY(4);
                return LP_FAIL;
            }
            since = 0;
            phase = LPH_GRAD;
        }
        if (phase == LPH_GRAD) {
            // vertex: y = A_B^-1 (-b_B)
#pragma unroll
            for (int i = 0; i < N; ++i) {
                double s = 0.0;
#pragma unroll
                for (int r = 0; r < N; ++r) s -= Bi[i][r] * bB[r];
                y[i] = s;
            }
        }
        double Y[N], Dd[N];
        lp_prefix<N>(y, Y);
        lp_prefix<N>(d, Dd);
        // ---- the scan: every term once, in the mode of the lane's phase
        //   GRAD:  gradient of the nonbasic terms (a term on its kink takes its recorded side)
        //   RATIO: the next breakpoint along d after (tprev, idprev) (a term whose value hardly moves
        //          along d -- |a.d| at rounding level of |a| |d| -- is parallel to the edge)
        //   CHECK: the hard rows (V, U, A, P) at the optimal vertex
        const int ph = phase;
        double g[N], gpre[N];
#pragma unroll
        for (int i = 0; i < N; ++i) g[i] = gpre[i] = 0.0;
        double tb = 1e300, jump = 0.0;
        int ib = -1, ibside = 1;
        bool viol = false;
        if (ph == LPH_RATIO) HVP_LP_PASS();
#pragma unroll 1
        for (int j = 0; j < N; ++j) {
            const LpPrim py = lp_prim<N>(y, Y, j), pd = lp_prim<N>(d, Dd, j);
            double g0 = 0.0, g1 = 0.0, g2 = 0.0, gp = 0.0;
            lp_step_terms<N>(D, C, j, [&](const LpTerm& t) {
                if (!t.ok) return;
                const int id = t.id;
                const double z = lp_val(t, py) + t.b;
                if (ph == LPH_CHECK) {
                    if (id >= 8 * N - 2) return;
                    const double tol = 1e-9 * (1.0 + fabs(t.b));
                    viol = viol || (t.sp > 0.0 && z > tol) || (t.sm > 0.0 && z < -tol);
                    return;
                }
                if (is_basic(id)) return;
                const double zt = 1e-12 * (1.0 + fabs(t.b));
                const bool pos = z > zt || (!(z < -zt) && !neg_bit(id));
                if (ph == LPH_GRAD) {
                    const double sl = pos ? t.sp : -t.sm;
                    g0 += sl * t.c0;
                    g1 += sl * t.c1;
                    g2 += sl * t.c2;
                    gp += sl * t.cp;
                    return;
                }
                const double rd = lp_val(t, pd);
                const double an = fabs(t.cp) * j + fabs(t.c0) + fabs(t.c1) + fabs(t.c2);
                if (!(fabs(rd) > 1e-10 * an * dmax)) return;
                if (pos == (rd > 0.0)) return;  // moving away from its kink
                const double tt = fmax(0.0, -z / rd);
                const bool after = tt > tprev || (tt == tprev && id > idprev);
                const bool better = after && (tt < tb || (tt == tb && id < ib));
                tb = better ? tt : tb;
                ib = better ? id : ib;
                ibside = better ? (pos ? -1 : 1) : ibside;
                jump = better ? (t.sp + t.sm) * fabs(rd) : jump;
            });
#pragma unroll
            for (int i = 0; i < N; ++i) {
                g[i] += i == j ? g0 : 0.0;
                g[i] += i + 1 == j ? g1 : 0.0;
                g[i] += i + 2 == j ? g2 : 0.0;
                gpre[i] += i + 1 == j ? gp : 0.0;
            }
        }
        if (ph == LPH_CHECK) {  // optimal: every edge non-decreasing; the hard rows must hold
            if (viol) HVP_LP_WHY(2);
            return viol ? LP_FAIL : LP_OK;
        }
        if (ph == LPH_GRAD) {
            {
                double acc = 0.0;
#pragma unroll
                for (int i = N - 1; i >= 0; --i) {
                    acc += gpre[i];
                    g[i] += acc;
                }
            }
            // edge derivatives: +-pi_k + s_k(side), pi = A_B^-T g
            int k_ = -1, sd_ = 0, eid = 0;
            double dv_ = -dtol;
#pragma unroll
            for (int k = 0; k < N; ++k) {
                double pk = 0.0;
#pragma unroll
                for (int i = 0; i < N; ++i) pk += Bi[i][k] * g[i];
#pragma unroll
                for (int sd = 0; sd < 2; ++sd) {
                    const double dv = sd == 0 ? pk + spB[k] : -pk + smB[k];
                    const bool cand = dv < -dtol;
                    const bool take = cand && (bland ? (k_ < 0 || basis[k] < eid) : dv < dv_);
                    k_ = take ? k : k_;
                    sd_ = take ? sd : sd_;
                    eid = take ? basis[k] : eid;
                    dv_ = take ? dv : dv_;
                }
            }
            if (k_ < 0) {
                // optimal: confirm on a freshly built A_B^-1 (exact vertex), then the hard rows
                phase = since > 0 ? LPH_INV : LPH_CHECK;
                return LP_RUN;
            }
            if (iters == max_iter) {
                HVP_LP_WHY(1);
                return LP_FAIL;
            }
            ek = k_;
            esd = sd_;
            eD = dv_;
            // direction d = +-A_B^-1 e_k (column ek selected by static index)
            const double sg = esd == 0 ? 1.0 : -1.0;
            dmax = 0.0;
#pragma unroll
            for (int i = 0; i < N; ++i) {
                double v = 0.0;
#pragma unroll
                for (int k = 0; k < N; ++k) v = k == ek ? Bi[i][k] : v;
                d[i] = sg * v;
                dmax = fmax(dmax, fabs(v));
            }
            slope = eD;
            tprev = 0.0;
            idprev = -1;
            passes = 0;
            phase = LPH_RATIO;
            return LP_RUN;
        }
        // ---- RATIO: one pass of the ratio test through the breakpoints in (t, id) order
        if (ib < 0) {  // no breakpoint left: unbounded (cannot happen with the V walls)
            HVP_LP_WHY(3);
            return LP_FAIL;
        }
        slope += jump;
        tprev = tb;
        idprev = ib;
        if (!(slope > -dtol || bland)) {  // still decreasing: crossed, now on its far side
            set_side(ib, ibside);
            if (++passes >= NT) {
                HVP_LP_WHY(3);
                return LP_FAIL;
            }
            return LP_RUN;
        }
        // the function stops decreasing here (Bland: first breakpoint): the term enters
        const int enter = ib;
        const double tstep = tb;
        // the entering term (one lookup) replaces basic position ek
        LpHyp he;
        lp_hyp<N>(D, C, enter, he);
        double ae[N];
        lp_normal<N>(he, ae);
        int old = 0;
#pragma unroll
        for (int k = 0; k < N; ++k) {
            const bool at = k == ek;
            old = at ? basis[k] : old;
            basis[k] = at ? enter : basis[k];
            bB[k] = at ? he.b : bB[k];
            spB[k] = at ? he.sp : spB[k];
            smB[k] = at ? he.sm : smB[k];
        }
        set_side(old, esd == 0 ? 1 : -1);  // the leaving term is on the side the edge took it to
        // A_B^-1 with row ek replaced by a_e (Sherman-Morrison): with c = A_B^-1 e_ek (the edge's
        // column) and w = a_e' A_B^-1, the new inverse is A_B^-1 - c (w - e_ek') / (a_e . c)
        double cc[N], w[N];
        double piv = 0.0;
#pragma unroll
        for (int i = 0; i < N; ++i) {
            double v = 0.0;
#pragma unroll
            for (int k = 0; k < N; ++k) v = k == ek ? Bi[i][k] : v;
            cc[i] = v;
            piv += ae[i] * v;
        }
#pragma unroll
        for (int c = 0; c < N; ++c) {
            double v = 0.0;
#pragma unroll
            for (int i = 0; i < N; ++i) v += ae[i] * Bi[i][c];
            w[c] = v - (c == ek ? 1.0 : 0.0);
        }
        if (++since >= kLpRefresh || !(fabs(piv) > 1e-11)) {
            phase = LPH_INV;  // rebuilt from the new basis before the next gradient
        } else {
            const double ip = 1.0 / piv;
#pragma unroll
            for (int i = 0; i < N; ++i)
#pragma unroll
                for (int c = 0; c < N; ++c) Bi[i][c] -= cc[i] * w[c] * ip;
            phase = LPH_GRAD;
        }
        HVP_LP_TRACE(iters, old, esd, eD, enter, tstep, bland, y);
        if (!(tstep > 1e-13)) bland = true;  // a degenerate pivot: Bland's rule from here on
        ++iters;
        return LP_RUN;
    }
};

template <int N, class MEM>
HVP_HD inline int lp_simplex(const LpData<N, MEM>& D, const Consts& C, int max_iter, double* y, int& iters) {
    LpLane<N> L;
    L.init(D, C);
    int st;
    do {
        st = L.trip(D, C, max_iter, y);
    } while (st == LP_RUN);
    iters = L.iters;
    return st;
}

// The node LP (relaxed after K steps) or leaf LP (K = N) of l1_rows by the simplex: L1_OK with the
// vertex in y, L1_INFEASIBLE (the exact hard-row test l1_infeasible), or L1_FAIL (unresolved).
template <int N, class MEM = LpArrayMem<N>>
HVP_HD inline int lp_solve_l1(LpData<N, MEM>& D, const hvp_system& S, const Consts& C, int role, const double* prm,
                              uint64_t code, int K, double rlo, double rhi, int max_iter, double* y, int& iters) {
    iters = 0;
    if (l1_infeasible<N>(S, C, prm, code, K, rlo, rhi)) return L1_INFEASIBLE;
    lp_data<N>(D, S, C, role, prm, code, K, rlo, rhi);
    return lp_simplex<N>(D, C, max_iter, y, iters) == LP_OK ? L1_OK : L1_FAIL;
}

}  // namespace hvp
