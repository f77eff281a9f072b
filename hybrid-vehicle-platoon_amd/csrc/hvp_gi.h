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
enum { GI_OK = 0, GI_FAIL_CHOL = 5, GI_FAIL_ITER = 6, GI_FAIL_DUAL = 7, GI_FAIL_VERIFY = 8,
       GI_WARM_LOST = 9 /* hvp_coop.h warm_start: set the QP up again, then solve cold */ };

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
// its reversed copy (violated when the row is satisfied strictly).  The chosen row's bound d
// and U-row coefficient a are returned with it (d_out, a_out), so that the active-set steps
// build the row from registers (gi_normal) without indexing the per-lane rows dynamically.
template <int N, class M>
HVP_HD inline int gi_most_violated(const LaneQp<N, M>& q, const Consts& C, const double* y, const GiMask<N>& act,
                                   uint32_t sat, double tol, double& d_out, double& a_out) {
    int best = -1;
    double best_v2 = 0.0, best_nn = 1.0, best_d = 0.0, best_a = 0.0;
    auto consider = [&](int id, double slack, double nn, double scale, double d, double a) {
        if (act.get(id & (GI_REV - 1)) || !(slack < -tol * scale)) return;
        // maximise slack^2 / |c|^2 among violated rows
        const double v2 = slack * slack;
        if (best < 0 || v2 * best_nn > best_v2 * nn) {
            best = id;
            best_v2 = v2;
            best_nn = nn;
            best_d = d;
            best_a = a;
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
        // row bounds in <= form (gi_row): the step-1 rows carry the constant -a v0 / -v0
        const double cu = j == 0 ? -a * q.v0 : 0.0, ca = j == 0 ? -q.v0 : 0.0;
        consider(6 * j + 0, gv - vl, 1.0, 1.0 + fabs(vl), -vl, a);
        consider(6 * j + 1, vh - gv, 1.0, 1.0 + fabs(vh), vh, a);
        consider(6 * j + 2, gu - ul, nu, 1.0 + fabs(ul) + fabs(a * yprev), cu - ul, a);
        consider(6 * j + 3, uh - gu, nu, 1.0 + fabs(uh) + fabs(a * yprev), uh - cu, a);
        consider(6 * j + 4, ga - al, na, 1.0 + fabs(yprev), ca - al, a);
        consider(6 * j + 5, ah - ga, na, 1.0 + fabs(yprev), ah - ca, a);
        if (k >= 2) {
            const int m = k - 2;
            cum += y[m];
            const double p = q.P1 + q.ts * cum, nn = q.ts * q.ts * (m + 1);
            const double sc = 1.0 + fabs(p);
            const int b = 6 * N + 4 * m;
            consider(b + 0, p - q.pmin, nn, sc, q.P1 - q.pmin, a);
            consider(b + 1, q.pmax - p, nn, sc, q.pmax - q.P1, a);
            const double hf = q.hf(m), hb = q.hb(m);
            const double sfw = hf - p, sbw = p - hb;
            const bool satf = (sat >> (2 * m)) & 1u, satb = (sat >> (2 * m + 1)) & 1u;
            consider(satf ? (b + 2) | GI_REV : b + 2, satf ? -sfw : sfw, nn, sc, satf ? q.P1 - hf : hf - q.P1, a);
            consider(satb ? (b + 3) | GI_REV : b + 3, satb ? -sbw : sbw, nn, sc, satb ? hb - q.P1 : q.P1 - hb, a);
        }
        yprev = yk;
    }
    d_out = best_d;
    a_out = best_a;
    return best;
}

// Normal c (<= form) of row id from its U-row coefficient a (see gi_row): branch-free over N.
template <int N>
HVP_HD inline void gi_normal(int id_in, double a_u, double ts, double* c) {
    const int id = id_in & (GI_REV - 1);
    const double neg = (id_in & GI_REV) ? -1.0 : 1.0;
    if (id < 6 * N) {
        const int j = id / 6, r = id % 6;
        const int pair = r / 2;                         // 0 V, 1 U, 2 A
        const double sgn = ((r & 1) ? 1.0 : -1.0) * neg;  // lo rows are negated
        const double a = pair == 1 ? a_u : (pair == 2 ? 1.0 : 0.0);
#pragma unroll
        for (int i = 0; i < N; ++i) c[i] = (i == j ? sgn : 0.0) + (i + 1 == j ? -sgn * a : 0.0);
    } else {
        const int m = (id - 6 * N) / 4, r = (id - 6 * N) % 4;
        const double sgn = ((r == 1 || r == 2) ? 1.0 : -1.0) * neg;  // P_hi, SF: +prefix ; P_lo, SB: -prefix
#pragma unroll
        for (int i = 0; i < N; ++i) c[i] = i <= m ? sgn * ts : 0.0;
    }
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
// row leaves S.
//
// Register discipline (gfx950: the lane kernels must fit 256 VGPRs for 2 waves per SIMD): the
// state is J (N x N), R as a packed upper triangle, the active multipliers and ids; every
// update is branch-free over the static bound N -- the add step is ONE Householder reflection
// of J's trailing columns (no sequence of Givens rotations under lane-dependent predicates),
// the drop step rotates with the identity (c = 1, s = 0) where a rotation does not apply, and
// R entries beyond the active set are kept at zero so that back substitution needs no masks.
// The solver is a small state machine (init / scan / step / verify) so that a kernel can run
// lanes at different stages of different QPs (hvp_lane.h: k_bnb_bound refills idle lanes).
// Multiplier above which an active velocity row counts for the switching rule (hvp_gadmm.h).
constexpr double kEdgeMultTol = 1e-6;

// R(i, j), i <= j, column-major packed upper triangle
HVP_HD constexpr int rix(int i, int j) { return j * (j + 1) / 2 + i; }

enum { GI_STEP_MORE = 0, GI_STEP_NEXT = 1 };

template <int N>
struct GiLane {
    static constexpr int NT = N * (N + 1) / 2;
    double J[N][N];  // J[row][col]
    double R[NT];
    double u[N];
    int ids[N];
    GiMask<N> act;
    uint32_t sat;    // bit 2m: SF of step m + 2 saturated, bit 2m + 1: SB
    int nact, p, iter;
    double unew;
    double pd, pa;   // bound (<= form) and U-row coefficient of row p (from scan)

    // pins the iterate to registers at a stage boundary (stops GVN from keeping copies alive)
    // and makes the lane's scalars opaque, so that loop-invariant code motion cannot hoist
    // values derived from them (ts^2 multiples, 1 + |v0|, ...) and keep them live across the
    // whole solve
    template <class M>
    HVP_HD void fence(LaneQp<N, M>& q) {
        fence(q.y);
#if defined(__HIP_DEVICE_COMPILE__)
        asm volatile("" : "+v"(q.ts), "+v"(q.v0), "+v"(q.P1), "+v"(q.pmin), "+v"(q.pmax));
#endif
    }
    HVP_HD void fence(double* y) {
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
        for (int i = 0; i < N; ++i) {
            asm volatile("" : "+v"(y[i]), "+v"(u[i]));
#pragma unroll
            for (int j = 0; j < N; ++j) asm volatile("" : "+v"(J[i][j]));
        }
#pragma unroll
        for (int i = 0; i < NT; ++i) asm volatile("" : "+v"(R[i]));
#else
        (void)y;
#endif
    }

    // unconstrained minimiser y = -H^-1 f and J = L^-T; GI_OK or GI_FAIL_CHOL
    template <class M>
    HVP_HD int init(LaneQp<N, M>& q) {
        iter = 0;
        nact = 0;
        p = -1;
        sat = 0;
        unew = 0.0;
        act = GiMask<N>();
        double L[NT];
#pragma unroll
        for (int i = 0; i < NT; ++i) L[i] = q.H[i];
        const bool ok = cholesky<N>(L);  // stores the inverse diagonal
        double negf[N];
#pragma unroll
        for (int i = 0; i < N; ++i) negf[i] = -q.f[i];
        chol_solve<N>(L, negf, q.y);
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
#pragma unroll
        for (int i = 0; i < NT; ++i) R[i] = 0.0;
#pragma unroll
        for (int i = 0; i < N; ++i) {
            u[i] = 0.0;
            ids[i] = -1;
        }
        return ok ? GI_OK : GI_FAIL_CHOL;
    }

    // step 1: the most violated row becomes p; false when the point is feasible (optimal)
    template <class M>
    HVP_HD bool scan(const LaneQp<N, M>& q, const Consts& C) {
        p = gi_most_violated(q, C, q.y, act, sat, 1e-11, pd, pa);
        unew = 0.0;
        return p >= 0;
    }

    HVP_HD void saturate(int id) {
        const int base = id & (GI_REV - 1);
        const uint32_t bit = 1u << (base - 6 * N - 2 - 2 * ((base - 6 * N) / 4));
        if (id & GI_REV) sat &= ~bit;
        else sat |= bit;
    }

    // step 2 for row p: one partial or full step.  GI_STEP_NEXT: p was added (or saturated) --
    // scan next; GI_STEP_MORE: a row left the active set, step again with the same p;
    // GI_FAIL_ITER / GI_FAIL_DUAL (dual unbounded: infeasible QP).
    template <class M>
    HVP_HD int step(LaneQp<N, M>& q, const Consts& C, int max_iter) {
        if (++iter > max_iter) return GI_FAIL_ITER;
        const double w = C.w;
        double c[N];
        gi_normal<N>(p, pa, q.ts, c);  // c.y <= pd ; the >= form has n = -c, slack s = pd - c.y
        const double dp = pd;
        // d = J'n, v = its part beyond the active set, z = J v (primal direction)
        double d[N];
        double dn = 0.0, d2n = 0.0;
#pragma unroll
        for (int col = 0; col < N; ++col) {
            double s = 0.0;
#pragma unroll
            for (int i = 0; i < N; ++i) s -= J[i][col] * c[i];
            d[col] = s;
            dn += s * s;
            d2n += col >= nact ? s * s : 0.0;
        }
        double z[N];
        double zn = 0.0, slack = dp;
#pragma unroll
        for (int i = 0; i < N; ++i) {
            double s = 0.0;
#pragma unroll
            for (int col = 0; col < N; ++col) s += col >= nact ? J[i][col] * d[col] : 0.0;
            z[i] = s;
            zn -= s * c[i];
            slack -= c[i] * q.y[i];
        }
        // r = R^-1 d1 (entries of R beyond the active set are zero)
        double r[N];
#pragma unroll
        for (int i = N - 1; i >= 0; --i) {
            double s = d[i];
#pragma unroll
            for (int j = i + 1; j < N; ++j) s -= R[rix(i, j)] * r[j];
            r[i] = i < nact ? s * frcp(R[rix(i, i)]) : 0.0;
        }
        // partial step: an active multiplier reaches zero (t1) or a soft one reaches w (t3)
        double t1 = 1e300, t3 = 1e300;
        int k1 = -1, k3 = -1;
        const bool psoft = gi_soft<N>(p);
        if (psoft) {
            t3 = w - unew;
            k3 = N;  // N denotes the new row p
        }
#pragma unroll
        for (int j = 0; j < N; ++j) {
            const double rj = r[j], ir = frcp(rj);
            const double tj1 = u[j] * ir;
            if (j < nact && rj > 0.0 && tj1 < t1) {
                t1 = tj1;
                k1 = j;
            }
            const double tj3 = (u[j] - w) * ir;
            if (j < nact && rj < 0.0 && gi_soft<N>(ids[j]) && tj3 < t3) {
                t3 = tj3;
                k3 = j;
            }
        }
        // full step: the new row becomes active
        const bool zstep = d2n > 1e-14 * dn;
        const double t2 = zstep && zn > 0.0 ? fmax(-slack, 0.0) / zn : 1e300;
        const double t = fmin(t1, fmin(t2, t3));
        if (!(t < 1e299)) return GI_FAIL_DUAL;
        const double ty = t2 < 1e299 ? t : 0.0;
#pragma unroll
        for (int i = 0; i < N; ++i) {
            q.y[i] += ty * z[i];
            u[i] -= t * r[i];  // r = 0 beyond the active set
        }
        unew += t;
        // the add and the drop below run on different lanes: the fences keep the compiler from
        // interleaving (if-converting) the two and holding both sets of temporaries at once
        fence(q.y);
        if (t2 <= t1 && t2 <= t3) {
            add(d, d2n);
            return GI_STEP_NEXT;
        }
        fence(q.y);
        int drop;
        if (t3 <= t1) {
            if (k3 == N) {  // the new soft row saturates: it joins the objective, nothing is added
                saturate(p);
                return GI_STEP_NEXT;
            }
            drop = k3;
        } else {
            drop = k1;
        }
        int dropped = -1;
#pragma unroll
        for (int j = 0; j < N; ++j) dropped = j == drop ? ids[j] : dropped;
        if (t3 <= t1) saturate(dropped);
        act.set(dropped & (GI_REV - 1), false);
        remove(drop);
        return GI_STEP_MORE;
    }

    // add p: Householder reflection of J's columns nact.. mapping v to alpha e_nact; R gets the
    // column (d_0 .. d_{nact-1}, alpha)
    HVP_HD void add(const double* d, double d2n) {
        double vk = 0.0, v[N];
#pragma unroll
        for (int col = 0; col < N; ++col) {
            v[col] = col >= nact ? d[col] : 0.0;
            vk = col == nact ? d[col] : vk;
        }
        const double sigma = sqrt(d2n);
        const double alpha = vk >= 0.0 ? -sigma : sigma;
        const double beta = frcp(sigma * (sigma + fabs(vk)));  // 2 / |v - alpha e|^2
#pragma unroll
        for (int col = 0; col < N; ++col) v[col] = col == nact ? vk - alpha : v[col];
#pragma unroll
        for (int row = 0; row < N; ++row) {
            double s = 0.0;
#pragma unroll
            for (int col = 0; col < N; ++col) s += J[row][col] * v[col];
            s *= beta;
#pragma unroll
            for (int col = 0; col < N; ++col) J[row][col] -= s * v[col];
        }
#pragma unroll
        for (int j = 0; j < N; ++j) {
#pragma unroll
            for (int i = 0; i <= j; ++i) {
                const double val = i < j ? d[i] : alpha;
                R[rix(i, j)] = j == nact ? val : R[rix(i, j)];
            }
        }
#pragma unroll
        for (int j = 0; j < N; ++j) {
            u[j] = j == nact ? unew : u[j];
            ids[j] = j == nact ? p : ids[j];
        }
        act.set(p & (GI_REV - 1), true);
        ++nact;
    }

    // remove the active row at position `drop`: shift u, ids and R's columns left, rotate the
    // resulting upper Hessenberg R back to triangular (rows i, i + 1 for i = drop .. nact - 2),
    // rotating J's columns alike
    HVP_HD void remove(int drop) {
        double sub[N > 1 ? N - 1 : 1];
#pragma unroll
        for (int j = 0; j < N - 1; ++j) {
            const bool sh = j >= drop && j < nact - 1;
            u[j] = sh ? u[j + 1] : u[j];
            ids[j] = sh ? ids[j + 1] : ids[j];
#pragma unroll
            for (int i = 0; i <= j; ++i) R[rix(i, j)] = sh ? R[rix(i, j + 1)] : R[rix(i, j)];
            sub[j] = sh ? R[rix(j + 1, j + 1)] : 0.0;
        }
#pragma unroll
        for (int j = 0; j < N; ++j) {
            const bool last = j == nact - 1;
            u[j] = last ? 0.0 : u[j];
            ids[j] = last ? -1 : ids[j];
#pragma unroll
            for (int i = 0; i <= j; ++i) R[rix(i, j)] = last ? 0.0 : R[rix(i, j)];
        }
#pragma unroll
        for (int i = 0; i < N - 1; ++i) {
            const bool on = i >= drop && i < nact - 1;
            const double a = R[rix(i, i)], b = sub[i];
            const double h = sqrt(a * a + b * b);
            const bool rot = on && h > 0.0;
            const double ih = frcp(h);
            const double gc = rot ? a * ih : 1.0, gs = rot ? b * ih : 0.0;
            R[rix(i, i)] = rot ? h : a;
#pragma unroll
            for (int j = i + 1; j < N; ++j) {
                const double a0 = R[rix(i, j)], a1 = R[rix(i + 1, j)];
                R[rix(i, j)] = gc * a0 + gs * a1;
                R[rix(i + 1, j)] = -gs * a0 + gc * a1;
            }
#pragma unroll
            for (int row = 0; row < N; ++row) {
                const double a0 = J[row][i], a1 = J[row][i + 1];
                J[row][i] = gc * a0 + gs * a1;
                J[row][i + 1] = -gs * a0 + gc * a1;
            }
        }
        --nact;
    }

    // multipliers of the active rows within [0, w] (soft) or >= 0; primal feasibility and the
    // saturated rows' sides hold by the exit condition of scan().  edge (optional): bit
    // 2 j + 0 / + 1 set when the V_lo / V_hi row of y_j (= v_{j+1}) is active at the optimum
    // with multiplier > kEdgeMultTol.
    HVP_HD int verify(const Consts& C, uint32_t* edge) const {
        const double w = C.w;
        bool ok = true;
#pragma unroll
        for (int j = 0; j < N; ++j) {
            if (j < nact) {
                if (u[j] < -1e-9 * w) ok = false;
                if (gi_soft<N>(ids[j]) && u[j] > w * (1.0 + 1e-9)) ok = false;
            }
        }
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
};

// The scan / step loop of Goldfarb-Idnani from the lane's current state to the verified optimum.
template <int N, class M>
HVP_HD HVP_FORCEINLINE inline int gi_run(GiLane<N>& g, LaneQp<N, M>& q, const Consts& C, int max_iter, int& iters, uint32_t* edge) {
    for (;;) {
        q.mem.refresh();
        g.fence(q);
        if (!g.scan(q, C)) break;
        int r;
        do {
            r = g.step(q, C, max_iter);
        } while (r == GI_STEP_MORE);
        if (r != GI_STEP_NEXT) {
            iters = g.iter;
            return r;
        }
    }
    iters = g.iter;
    return g.verify(C, edge);
}

// One QP from start to finish.  Returns GI_OK with the optimum in q.y, or a GI_FAIL_* reason.
template <int N, class M>
HVP_HD inline int solve_gi(LaneQp<N, M>& q, const Consts& C, int max_iter, int& iters, uint32_t* edge = nullptr) {
    GiLane<N> g;
    int st = g.init(q);
    iters = 0;
    if (st != GI_OK) return st;
    return gi_run<N>(g, q, C, max_iter, iters, edge);
}

// Row `id` made active as an EQUALITY whatever its slack (the polish below): the step of
// GiLane::step with the signed full length t = -slack / |v|^2 and no ratio test, so the
// invariant (y optimal for the active rows at equality, u their multipliers, of any sign)
// holds after it.  false (nothing changed) when the row depends on the active ones.
template <int N, class M>
HVP_HD HVP_FORCEINLINE inline bool gi_force_add(GiLane<N>& g, LaneQp<N, M>& q, const Consts& C, int id) {
    double c[N], dp;
    gi_row<N>(q, C, id, c, dp);
    double d[N];
    double dn = 0.0, d2n = 0.0;
#pragma unroll
    for (int col = 0; col < N; ++col) {
        double s = 0.0;
#pragma unroll
        for (int i = 0; i < N; ++i) s -= g.J[i][col] * c[i];
        d[col] = s;
        dn += s * s;
        d2n += col >= g.nact ? s * s : 0.0;
    }
    if (!(d2n > 1e-14 * dn) || g.nact >= N) return false;
    double z[N], slack = dp;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        double s = 0.0;
#pragma unroll
        for (int col = 0; col < N; ++col) s += col >= g.nact ? g.J[i][col] * d[col] : 0.0;
        z[i] = s;
        slack -= c[i] * q.y[i];
    }
    double r[N];
#pragma unroll
    for (int i = N - 1; i >= 0; --i) {
        double s = d[i];
#pragma unroll
        for (int j = i + 1; j < N; ++j) s -= g.R[rix(i, j)] * r[j];
        r[i] = i < g.nact ? s * frcp(g.R[rix(i, i)]) : 0.0;
    }
    const double t = -slack / d2n;  // z.n = |v|^2
#pragma unroll
    for (int i = 0; i < N; ++i) {
        q.y[i] += t * z[i];
        g.u[i] -= t * r[i];
    }
    g.unew = t;
    g.p = id;
    g.add(d, d2n);
    return true;
}

// Active-set polish of an interior-point solution (the ADMM forms' fallback, hvp_admm.h
// solve_admm_ipm).  The rows the interior point holds active (multiplier above slack: l t = mu
// separates them from the inactive ones) are added as equalities from the unconstrained
// minimiser, which gives the equality-constrained optimum on that set with its exact
// multipliers; a row whose multiplier comes out negative leaves the set and the adds start over
// (at most 4 times); from that dual-feasible state Goldfarb-Idnani runs to its verified optimum,
// adding what the set missed.  So the answer, its multipliers and the switching rule's edge bits
// are the active-set method's, not the interior point's approximations of them.  Only QPs
// without soft rows (the ADMM forms: the safety lives in the copies' hinges); GI_OK with the
// optimum in q.y, else a GI_FAIL_* code and q.y undefined.
template <int N, class M>
HVP_HD HVP_FORCEINLINE inline int gi_polish(LaneQp<N, M>& q, const Consts& C, int max_iter, int& iters, uint32_t* edge) {
    iters = 0;
    if (q.has_sf || q.has_sb) return GI_FAIL_VERIFY;
    GiMask<N> cand;
#pragma unroll
    for (int p = 0; p < LaneQp<N, M>::NPAIR; ++p) {
        const int id = p < 3 * N ? 6 * (p / 3) + 2 * (p % 3) : 6 * N + 4 * (p - 3 * N);
        if (q.llo[p] > q.tlo[p]) cand.set(id, true);
        if (q.lhi[p] > q.thi[p]) cand.set(id + 1, true);
    }
    GiLane<N> g;
    bool dual_ok = false;
    for (int attempt = 0; attempt < 4 && !dual_ok; ++attempt) {
        if (g.init(q) != GI_OK) return GI_FAIL_CHOL;
#pragma unroll 1
        for (int id = 0; id < GiConstraintSet<N>::NC; ++id)
            if (cand.get(id)) gi_force_add<N>(g, q, C, id);
        dual_ok = true;
#pragma unroll
        for (int j = 0; j < N; ++j) {
            if (j < g.nact && g.u[j] < -1e-9 * C.w) {
                cand.set(g.ids[j] & (GI_REV - 1), false);
                dual_ok = false;
            }
        }
    }
    if (!dual_ok) return GI_FAIL_DUAL;
    return gi_run<N>(g, q, C, max_iter, iters, edge);
}

}  // namespace hvp
