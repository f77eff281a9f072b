// hvp_gi.h -- Goldfarb-Idnani dual active-set solver of the fixed-sequence QP (fast path).
//
// Same QP as hvp_ipm.h, written as an exact-penalty problem in velocity space:
//     min  1/2 y'Hy + f'y + w sum_soft max(0, c_i.y - d_i)   s.t.  c_i.y <= d_i  (hard rows)
// The soft rows are the safe-distance rows (fleet_decent_mld.py:190-208) with their slack
// variables eliminated: a slack s >= 0 with cost w s is exactly the penalty w max(0, .), i.e.
// a constraint whose multiplier is bounded above by w.
//
// Goldfarb & Idnani (1983): start from the unconstrained minimiser, repeatedly add the most
// violated row, keep the current point optimal for the active rows (J = L^-T Q, R from the QR
// of L^-1 N_A), drop rows whose multipliers would turn negative.  Extension for the soft rows:
// when a soft row's multiplier reaches w during a step it is SATURATED -- removed from the
// active set and moved into the objective as the linear term w c_i (stationarity is preserved
// exactly, since its multiplier equals w at that point).
//
// State per lane: y, J (N x N), R (N x N upper), the active multipliers and ids -- a few dozen
// doubles instead of the IPM's per-row slacks and multipliers.  All loops run over the static
// bound N with predication so every array stays in registers.
//
// The result is verified (primal feasibility, multiplier signs and bounds, consistency of the
// saturated rows); a lane that fails verification or the iteration cap reports GI_FAIL and is
// re-solved by the interior-point path (hvp_ipm.h).
#pragma once

#include "hvp_ipm.h"

namespace hvp {

// GI_OK, or why the lane is handed to the interior-point fallback
enum { GI_OK = 0, GI_FAIL_CHOL = 5, GI_FAIL_ITER = 6, GI_FAIL_DUAL = 7, GI_FAIL_VERIFY = 8 };

template <int N>
struct GiConstraintSet {
    static constexpr int NV = 6 * N;            // V/U/A rows, 6 per step
    static constexpr int NPRE = 4 * (N - 1);    // P_lo, P_hi, SF (soft), SB (soft) per step >= 2
    static constexpr int NC = NV + NPRE;
};

// Row ids: V/U/A rows 6j + {0 V_lo, 1 V_hi, 2 U_lo, 3 U_hi, 4 A_lo, 5 A_hi} (step k = j + 1),
// prefix rows 6N + 4m + {0 P_lo, 1 P_hi, 2 SF, 3 SB} (step k = m + 2).  GI_REV marks the
// reversed copy of a saturated soft row (see solve_gi).
constexpr int GI_REV = 256;

template <int N>
HVP_HD constexpr bool gi_soft(int id) {
    return (id & (GI_REV - 1)) >= 6 * N && (((id & (GI_REV - 1)) - 6 * N) & 2) != 0;
}

// Normal (in <= form, c.y <= d) of row id, densely in c[], and its bound d.
template <int N, class M>
HVP_HD inline void gi_row(const LaneQp<N, M>& q, const Consts& C, int id_in, double* c, double& d) {
    const int id = id_in & (GI_REV - 1);
    if (id < 6 * N) {
        const int j = id / 6, r = id % 6;
        const int pair = r / 2;                   // 0 V, 1 U, 2 A
        const double sgn = (r & 1) ? 1.0 : -1.0;  // lo rows are negated
        const double a = pair == 1 ? q.am(j) : (pair == 2 ? 1.0 : 0.0);
        double lo, hi;
        if (pair == 0) { lo = q.vlo(j); hi = q.vhi(j); }
        else if (pair == 1) { lo = q.ulo(j); hi = q.uhi(j); }
        else { lo = C.dec[j]; hi = C.acc[j]; }
        // row value g.y (+ const for j = 0): V: y_j ; U: y_j - a y_{j-1} ; A: y_j - y_{j-1}
        const double cst = j == 0 ? -a * q.v0 : 0.0;
#pragma unroll
        for (int i = 0; i < N; ++i) c[i] = (i == j ? sgn : 0.0) + (i + 1 == j ? -sgn * a : 0.0);
        d = (r & 1) ? hi - cst : -(lo - cst);
    } else {
        const int m = (id - 6 * N) / 4, r = (id - 6 * N) % 4;
        const double sgn = (r == 1 || r == 2) ? 1.0 : -1.0;  // P_hi, SF: +prefix ; P_lo, SB: -prefix
#pragma unroll
        for (int i = 0; i < N; ++i) c[i] = i <= m ? sgn * q.ts : 0.0;
        if (r == 0) d = q.P1 - q.pmin;
        else if (r == 1) d = q.pmax - q.P1;
        else if (r == 2) d = q.hf(m) - q.P1;
        else d = q.P1 - q.hb(m);
    }
    if (id_in & GI_REV) {
#pragma unroll
        for (int i = 0; i < N; ++i) c[i] = -c[i];
        d = -d;
    }
}

// Row mask: 128 bits cover N <= 8 (at most 76 rows); longer horizons use the generic form.
template <int N, bool WIDE = (GiConstraintSet<N>::NC > 128)>
struct GiMask {
    uint64_t lo = 0, hi = 0;
    HVP_HD bool get(int id) const { return id < 64 ? ((lo >> id) & 1ull) != 0 : ((hi >> (id - 64)) & 1ull) != 0; }
    HVP_HD void set(int id, bool on) {
        if (id < 64) lo = on ? (lo | (1ull << id)) : (lo & ~(1ull << id));
        else hi = on ? (hi | (1ull << (id - 64))) : (hi & ~(1ull << (id - 64)));
    }
};
template <int N>
struct GiMask<N, true> {
    static constexpr int W = (GiConstraintSet<N>::NC + 63) / 64;
    uint64_t w[W] = {};
    HVP_HD bool get(int id) const { return ((w[id >> 6] >> (id & 63)) & 1ull) != 0; }
    HVP_HD void set(int id, bool on) {
        if (on) w[id >> 6] |= 1ull << (id & 63);
        else w[id >> 6] &= ~(1ull << (id & 63));
    }
};

// Slack d - c.y of every row (structured: O(1) per row) and the most violated one (largest
// violation relative to |c|).  Active rows are skipped; a saturated soft row is represented by
// its reversed copy (violated when the row is satisfied strictly).
template <int N, class M>
HVP_HD inline int gi_most_violated(const LaneQp<N, M>& q, const Consts& C, const double* y, const GiMask<N>& act,
                                   uint32_t sat, double tol, double& s_out) {
    int best = -1;
    double best_v2 = 0.0, best_nn = 1.0, best_s = 0.0;
    auto consider = [&](int id, double slack, double nn, double scale) {
        if (act.get(id & (GI_REV - 1)) || !(slack < -tol * scale)) return;
        // maximise slack^2 / |c|^2 among violated rows
        const double v2 = slack * slack;
        if (best < 0 || v2 * best_nn > best_v2 * nn) {
            best = id;
            best_v2 = v2;
            best_nn = nn;
            best_s = slack;
        }
    };
    double yprev = q.v0, cum = 0.0;
#pragma unroll
    for (int k = 1; k <= N; ++k) {
        const int j = k - 1;
        const double yk = y[j];
        const double a = q.am(j);
        const double gv = yk, gu = yk - a * yprev, ga = yk - yprev;
        const double nu = j ? 1.0 + a * a : 1.0, na = j ? 2.0 : 1.0;
        const double vl = q.vlo(j), vh = q.vhi(j), ul = q.ulo(j), uh = q.uhi(j), al = C.dec[j], ah = C.acc[j];
        consider(6 * j + 0, gv - vl, 1.0, 1.0 + fabs(vl));
        consider(6 * j + 1, vh - gv, 1.0, 1.0 + fabs(vh));
        consider(6 * j + 2, gu - ul, nu, 1.0 + fabs(ul) + fabs(a * yprev));
        consider(6 * j + 3, uh - gu, nu, 1.0 + fabs(uh) + fabs(a * yprev));
        consider(6 * j + 4, ga - al, na, 1.0 + fabs(yprev));
        consider(6 * j + 5, ah - ga, na, 1.0 + fabs(yprev));
        if (k >= 2) {
            const int m = k - 2;
            cum += y[m];
            const double p = q.P1 + q.ts * cum, nn = q.ts * q.ts * (m + 1);
            const double sc = 1.0 + fabs(p);
            const int b = 6 * N + 4 * m;
            consider(b + 0, p - q.pmin, nn, sc);
            consider(b + 1, q.pmax - p, nn, sc);
            const double sfw = q.hf(m) - p, sbw = p - q.hb(m);
            const bool satf = (sat >> (2 * m)) & 1u, satb = (sat >> (2 * m + 1)) & 1u;
            consider(satf ? (b + 2) | GI_REV : b + 2, satf ? -sfw : sfw, nn, sc);
            consider(satb ? (b + 3) | GI_REV : b + 3, satb ? -sbw : sbw, nn, sc);
        }
        yprev = yk;
    }
    s_out = best_s;
    return best;
}

HVP_HD inline void givens(double a, double b, double& c, double& s) {
    // rotation [c s; -s c] with  c a + s b = r,  -s a + c b = 0
    const double h = sqrt(a * a + b * b);
    if (h == 0.0) { c = 1.0; s = 0.0; return; }
    const double ih = frcp(h);
    c = a * ih;
    s = b * ih;
}

// Goldfarb-Idnani with soft rows.  Invariant: y minimises
//     1/2 y'Hy + f'y + w sum_{i in S} (c_i.y - d_i)   subject to the active rows at equality,
// where S is the saturated set (soft rows whose multiplier reached w).  A saturated row whose
// penalty term turns inactive again (c_i.y < d_i) shows up as a violated REVERSED soft row
// -c_i.y <= -d_i; saturating that reversed row (multiplier w) cancels the linear term, i.e. the
// row leaves S.  Returns GI_OK with the optimum in q.y, or a GI_FAIL_* reason.
// Multiplier above which an active velocity row counts for the switching rule (hvp_gadmm.h).
constexpr double kEdgeMultTol = 1e-6;

// edge (optional): bit 2 j + 0 / + 1 set when the V_lo / V_hi row of y_j (= v_{j+1}) is active
// at the optimum with multiplier > kEdgeMultTol.
template <int N, class M>
HVP_HD inline int solve_gi(LaneQp<N, M>& q, const Consts& C, int max_iter, int& iters, uint32_t* edge = nullptr) {
    iters = 0;
    // ---- unconstrained minimiser and J = L^-T
    double L[N * (N + 1) / 2];
#pragma unroll
    for (int i = 0; i < N * (N + 1) / 2; ++i) L[i] = q.H[i];
    if (!cholesky<N>(L)) return GI_FAIL_CHOL;  // stores the inverse diagonal
    double negf[N];
#pragma unroll
    for (int i = 0; i < N; ++i) negf[i] = -q.f[i];
    chol_solve<N>(L, negf, q.y);
    double J[N][N];  // J[row][col]
    // L^-1 (lower) by forward substitution of the identity; J = (L^-1)^T
#pragma unroll
    for (int col = 0; col < N; ++col) {
        double x[N];
#pragma unroll
        for (int i = 0; i < N; ++i) {
            double v = i == col ? 1.0 : 0.0;
#pragma unroll
            for (int k = 0; k < i; ++k) v -= L[tri(i, k)] * x[k];
            x[i] = v * L[tri(i, i)];
        }
#pragma unroll
        for (int i = 0; i < N; ++i) J[col][i] = x[i];
    }
    double R[N][N];
#pragma unroll
    for (int i = 0; i < N; ++i)
#pragma unroll
        for (int j = 0; j < N; ++j) R[i][j] = 0.0;
    double u[N];
    int ids[N];
#pragma unroll
    for (int i = 0; i < N; ++i) { u[i] = 0.0; ids[i] = -1; }
    int nact = 0;
    GiMask<N> act;
    uint32_t sat = 0;  // bit 2m: SF of step m + 2 saturated, bit 2m + 1: SB
    const double w = C.w;
    const double tol = 1e-11;
    // saturate (on) / unsaturate soft row id; a reversed row flips the meaning
    auto saturate = [&](int id) {
        const int base = id & (GI_REV - 1);
        const uint32_t bit = 1u << (base - 6 * N - 2 - 2 * ((base - 6 * N) / 4));
        if (id & GI_REV) sat &= ~bit;
        else sat |= bit;
    };

    int iter = 0;
    for (;;) {
        // ---------------- step 1: most violated row
        q.mem.refresh();
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
        for (int i = 0; i < N; ++i) {
            asm volatile("" : "+v"(q.y[i]), "+v"(u[i]));
#pragma unroll
            for (int j = 0; j < N; ++j) asm volatile("" : "+v"(J[i][j]), "+v"(R[i][j]));
        }
#endif
        double sp;
        const int p = gi_most_violated(q, C, q.y, act, sat, tol, sp);
        if (p < 0) break;
        double np[N], dp;
        gi_row(q, C, p, np, dp);
        const bool psoft = gi_soft<N>(p);
#pragma unroll
        for (int i = 0; i < N; ++i) np[i] = -np[i];  // >= form: n = -c, b = -d ; slack s = n.y - b
        double unew = 0.0;
        for (;;) {
            if (++iter > max_iter) { iters = iter; return GI_FAIL_ITER; }
            // ---------------- step 2: directions
            double dv[N];
#pragma unroll
            for (int col = 0; col < N; ++col) {
                double s = 0.0;
#pragma unroll
                for (int i = 0; i < N; ++i) s += J[i][col] * np[i];
                dv[col] = s;
            }
            double z[N];
            double d2n = 0.0, dn = 0.0;
#pragma unroll
            for (int col = 0; col < N; ++col) {
                dn += dv[col] * dv[col];
                if (col >= nact) d2n += dv[col] * dv[col];
            }
#pragma unroll
            for (int i = 0; i < N; ++i) {
                double s = 0.0;
#pragma unroll
                for (int col = 0; col < N; ++col) s += col >= nact ? J[i][col] * dv[col] : 0.0;
                z[i] = s;
            }
            double r[N];
#pragma unroll
            for (int i = N - 1; i >= 0; --i) {
                double v = dv[i];
#pragma unroll
                for (int j = i + 1; j < N; ++j) v -= (j < nact) ? R[i][j] * r[j] : 0.0;
                r[i] = (i < nact) ? v / R[i][i] : 0.0;
            }
            // partial step: an active multiplier reaches zero
            double t1 = 1e300;
            int k1 = -1;
#pragma unroll
            for (int j = 0; j < N; ++j) {
                if (j < nact && r[j] > 0.0) {
                    const double tj = u[j] / r[j];
                    if (tj < t1) { t1 = tj; k1 = j; }
                }
            }
            // soft bound: a multiplier reaches w (active soft rows with r < 0, or the new row)
            double t3 = psoft ? w - unew : 1e300;
            int k3 = psoft ? N : -1;  // N denotes the new row p
#pragma unroll
            for (int j = 0; j < N; ++j) {
                if (j < nact && gi_soft<N>(ids[j]) && r[j] < 0.0) {
                    const double tj = (w - u[j]) / (-r[j]);
                    if (tj < t3) { t3 = tj; k3 = j; }
                }
            }
            // full step: the new row becomes active
            const bool zstep = d2n > 1e-14 * dn;
            double zn = 0.0;
#pragma unroll
            for (int i = 0; i < N; ++i) zn += z[i] * np[i];
            double sp_now = dp;
#pragma unroll
            for (int i = 0; i < N; ++i) sp_now += np[i] * q.y[i];  // current slack n.y - b
            const double t2 = zstep && zn > 0.0 ? fmax(-sp_now, 0.0) / zn : 1e300;
            const double t = fmin(t1, fmin(t2, t3));
            if (!(t < 1e299)) { iters = iter; return GI_FAIL_DUAL; }  // dual unbounded: infeasible QP
            if (t2 < 1e299) {
#pragma unroll
                for (int i = 0; i < N; ++i) q.y[i] += t * z[i];
            }
#pragma unroll
            for (int j = 0; j < N; ++j)
                if (j < nact) u[j] -= t * r[j];
            unew += t;
            if (t2 <= t1 && t2 <= t3) {
                // ---- add p: Givens rotations zero dv[nact+1..N-1], rotating J's columns
#pragma unroll
                for (int i = N - 1; i >= 1; --i) {
                    if (i > nact) {
                        double gc, gs;
                        givens(dv[i - 1], dv[i], gc, gs);
                        dv[i - 1] = gc * dv[i - 1] + gs * dv[i];
                        dv[i] = 0.0;
#pragma unroll
                        for (int row = 0; row < N; ++row) {
                            const double a0 = J[row][i - 1], a1 = J[row][i];
                            J[row][i - 1] = gc * a0 + gs * a1;
                            J[row][i] = -gs * a0 + gc * a1;
                        }
                    }
                }
#pragma unroll
                for (int i = 0; i < N; ++i)
#pragma unroll
                    for (int col = 0; col < N; ++col)
                        if (col == nact && i <= nact) R[i][col] = dv[i];
#pragma unroll
                for (int j = 0; j < N; ++j)
                    if (j == nact) { u[j] = unew; ids[j] = p; }
                act.set(p & (GI_REV - 1), true);
                ++nact;
                break;
            }
            // ---- a row leaves the active set: the zero-multiplier one (t1) or a saturating soft one (t3)
            int drop;
            if (t3 <= t1) {
                if (k3 == N) {
                    // the new soft row saturates: it joins the objective, no constraint is added
                    saturate(p);
                    break;
                }
                drop = k3;
            } else {
                drop = k1;
            }
            int dropped_id = -1;
#pragma unroll
            for (int j = 0; j < N; ++j)
                if (j == drop) dropped_id = ids[j];
            if (t3 <= t1) saturate(dropped_id);
            act.set(dropped_id & (GI_REV - 1), false);
            // remove the active row at position `drop`: shift columns of R, u, ids; re-triangularise
#pragma unroll
            for (int j = 0; j < N - 1; ++j) {
                if (j >= drop && j < nact - 1) {
                    u[j] = u[j + 1];
                    ids[j] = ids[j + 1];
#pragma unroll
                    for (int i = 0; i < N; ++i) R[i][j] = R[i][j + 1];
                }
            }
#pragma unroll
            for (int i = 0; i < N; ++i)
#pragma unroll
                for (int j = 0; j < N; ++j)
                    if (j == nact - 1) R[i][j] = 0.0;
            // R is now upper Hessenberg in columns drop..nact-2: rotate rows (i, i+1)
#pragma unroll
            for (int i = 0; i < N - 1; ++i) {
                if (i >= drop && i < nact - 1) {
                    double gc, gs;
                    givens(R[i][i], R[i + 1][i], gc, gs);
#pragma unroll
                    for (int col = 0; col < N; ++col) {
                        if (col >= i && col < nact - 1) {
                            const double a0 = R[i][col], a1 = R[i + 1][col];
                            R[i][col] = gc * a0 + gs * a1;
                            R[i + 1][col] = -gs * a0 + gc * a1;
                        }
                    }
#pragma unroll
                    for (int row = 0; row < N; ++row) {
                        const double a0 = J[row][i], a1 = J[row][i + 1];
                        J[row][i] = gc * a0 + gs * a1;
                        J[row][i + 1] = -gs * a0 + gc * a1;
                    }
                }
            }
#pragma unroll
            for (int j = 0; j < N; ++j)
                if (j == nact - 1) { u[j] = 0.0; ids[j] = -1; }
            --nact;
            // continue with the same p (step 2)
        }
    }
    iters = iter;

    // ---------------- verification: multipliers of the active rows within [0, w] (soft) or >= 0
    bool ok = true;
#pragma unroll
    for (int j = 0; j < N; ++j) {
        if (j < nact) {
            if (u[j] < -1e-9 * w) ok = false;
            if (gi_soft<N>(ids[j]) && u[j] > w * (1.0 + 1e-9)) ok = false;
        }
    }
    // primal feasibility and the saturated rows' sides hold by the exit condition of step 1
    if (edge) {
        uint32_t m = 0;
#pragma unroll
        for (int j = 0; j < N; ++j) {
            if (j < nact && ids[j] >= 0 && ids[j] < 6 * N && ids[j] % 6 < 2 && u[j] > kEdgeMultTol)
                m |= 1u << (2 * (ids[j] / 6) + ids[j] % 6);
        }
        *edge = m;
    }
    return ok ? GI_OK : GI_FAIL_VERIFY;
}

}  // namespace hvp
