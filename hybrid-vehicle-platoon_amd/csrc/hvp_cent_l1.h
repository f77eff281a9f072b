// hvp_cent_l1.h -- the centralised platoon LP of the min_1_norm cost (MpcMldCent with
// quadratic_cost=False, mpcs/cent_mld.py:58-61) for a GIVEN (possibly partial) region assignment,
// solved by ONE 64-lane wavefront.  The reference's MILP-vs-MIQP study drives exactly this
// controller (fleet_cent_mld.py:137-175 with sim.quadratic_cost, results_analysis/
// analyse_results_MILP_MIQP.py).
//
// With the regions fixed the MILP is an LP in the n N velocities y_{i,a} = v_{i,a+1}: every term of
// cent_mld.py:83-140 priced as sum_i Q_ii |e_i| (leader tracking, chain spacing, Q_u |u|, Q_du |du|)
// plus w max(0, p_i - p_{i-1} + d_safe) for the eliminated slacks, under the hard rows of each
// vehicle (V, U, A, P: hvp_cent.h setup, the quadratic QP's rows and tail relaxation).
//
// Lane t = i N + a owns variable y_{i,a} and the rows of state a + 1 of vehicle i: 8 hard rows and
// up to 7 L1 terms (hvp_l1.h's epigraph pairs).  Every row's normal is
//     g = cp * [own prefix b < a] + cq * [vehicle i-1's prefix b < a] + c0 e_t + c1 e_{t-1}
//         + c2 e_{t-2} + d0 e_{t-N},
// so g.y is a handful of cross-lane values (the vehicle prefix sums and three shifted lanes).
// Solver: the Mehrotra predictor-corrector of hvp_l1.h (epigraph variables eliminated per pair,
// the accurate multiplier directions, the centring fallback, Cholesky with the infinity rule); the
// V x V Newton matrix is assembled in LDS column by column: the rows go through a 64-row descriptor
// buffer one slot at a time, lane s adds the products of every row touching variable s to column s
// (deterministic, no atomics), then a wave Cholesky (hvp_cent.h's) factors it.
#pragma once

#include "hvp_cent.h"
#include "hvp_l1.h"

namespace hvp {
namespace cent {

constexpr int kLpHard = 8;   // V lo/hi, U lo/hi, A lo/hi, P lo/hi
constexpr int kLpPair = 7;   // leader p, v; chain p, v; u; du; safe hinge
constexpr int kLpDesc = 10;  // descriptor doubles per row in the LDS buffer
// Stopping rule.  The platoon LP's Newton matrix (n N up to 64 variables) reaches condition
// numbers past 1e25 once mu < 1e-12: an iteration or two beyond a relative gap of ~1e-11 the solve
// error feeds the dual residual and the iterate wanders off (traces of HVP_CENT_DEBUG=4).  A
// relative gap of 1e-11 with dual residuals below 1e-9 of the largest weight prices the LP within
// ~1e-11 of its optimum (the tie window is 1e-9, the prune margin 1e-7).  Should the iteration
// wander off first, the best iterate seen within kLpRescueGap (primal feasible, dual residual
// within 1e-8) is returned: the LP's value is the primal objective at y, so a feasible y with a
// small gap prices it as well as the last iterate would.
constexpr double kLpGapTol = 1e-11;
constexpr double kLpDualTol = 1e-9;
constexpr double kLpRescueGap = 1e-9;

struct LpG {
    double cp, cq, c0, c1, c2, d0;
};

// per-lane neighbour data of the LP (fixed for one LP)
struct LpCtx {
    double P1m;            // P1 of vehicle i-1
    double amm, ubm, ucm;  // input map of step a-1 (same vehicle)
    int Ki;                // fixed steps of the lane's vehicle
};

// cross-lane values of a vector (y or dy) that every row dot product needs
struct LpVals {
    double pre, prem, v, vm1, vm2, vmN;
};

__device__ inline LpVals lp_vals(double v, int N, bool on) {
    const int t = lane();
    LpVals o;
    const double vv = on ? v : 0.0;
    o.v = vv;
    o.pre = vehicle_prefix(vv, N);
    o.prem = __shfl(o.pre, t >= N ? t - N : t, W);
    o.vm1 = shift_up1(vv);
    o.vm2 = shift_up1(o.vm1);
    o.vmN = __shfl(vv, t >= N ? t - N : t, W);
    return o;
}

__device__ inline double lp_dot(const LpG& g, const LpVals& x) {
    return g.cp * x.pre + g.cq * x.prem + g.c0 * x.v + g.c1 * x.vm1 + g.c2 * x.vm2 + g.d0 * x.vmN;
}

// hard row r (0..7) of the lane: g.y <= h; false if absent
__device__ inline bool lp_hard(int r, const Lane& L, const Inst& I, LpG& g, double& h) {
    g = LpG{0, 0, 0, 0, 0, 0};
    h = 0.0;
    if (!L.on) return false;
    const int a = L.a;
    switch (r) {
        case 0: g.c0 = 1.0; h = L.vhi; return true;
        case 1: g.c0 = -1.0; h = -L.vlo; return true;
        case 2:
        case 3: {
            if (!(L.ulo > -1e29)) return false;  // a relaxed step without a virtual region
            const double cst = a == 0 ? L.am * L.v0 : 0.0;
            const double sg = r == 2 ? 1.0 : -1.0;
            g.c0 = sg;
            g.c1 = a >= 1 ? -sg * L.am : 0.0;
            h = r == 2 ? L.uhi + cst : -(L.ulo + cst);
            return true;
        }
        case 4:
        case 5: {
            const double cst = a == 0 ? L.v0 : 0.0;
            const double sg = r == 4 ? 1.0 : -1.0;
            g.c0 = sg;
            g.c1 = a >= 1 ? -sg : 0.0;
            h = r == 4 ? L.acc + cst : -(L.dec + cst);
            return true;
        }
        case 6:
        case 7:
            if (a < 1) return false;  // p_1 is a constant (checked by setup)
            g.cp = r == 6 ? L.ts : -L.ts;
            h = r == 6 ? L.pmax - L.P1 : L.P1 - L.pmin;
            return true;
    }
    (void)I;
    return false;
}

// L1 term r (0..6) of the lane: w |g.y + e0| (al = 1) or w max(0, g.y + e0) (al = 0); false if
// absent or constant (constants are priced by lp_direct_cost only)
__device__ inline bool lp_pair(int r, const Lane& L, const Consts& C, const Inst& I, const LpCtx& X, LpG& g,
                               double& e0, double& w, double& al) {
    g = LpG{0, 0, 0, 0, 0, 0};
    e0 = 0.0;
    w = 0.0;
    al = 1.0;
    if (!L.on) return false;
    const int i = L.i, a = L.a, k = a + 1, N = I.N;
    switch (r) {
        case 0:  // leader tracking, position (cent_mld.py:85-105)
            if (i != I.L) return false;
            g.cp = a >= 1 ? L.ts : 0.0;
            g.c0 = I.lsp ? C.t0 : 0.0;
            e0 = L.P1 - I.xl[k] + (I.lsp ? C.d0 : 0.0);
            w = C.Qpp;
            break;
        case 1:  // leader tracking, velocity
            if (i != I.L) return false;
            g.c0 = 1.0;
            e0 = -I.xl[N + 1 + k];
            w = C.Qvv;
            break;
        case 2:  // chain spacing, position (:106-117): p_i + t0 v_i + d0 - p_{i-1}
            if (i < 1) return false;
            g.cp = a >= 1 ? L.ts : 0.0;
            g.cq = a >= 1 ? -L.ts : 0.0;
            g.c0 = C.t0;
            e0 = L.P1 - X.P1m + C.d0;
            w = C.Qpp;
            break;
        case 3:  // chain spacing, velocity
            if (i < 1) return false;
            g.c0 = 1.0;
            g.d0 = -1.0;
            w = C.Qvv;
            break;
        case 4: {  // Q_u |u_{i,a}| (fixed steps and relaxed steps in a virtual region)
            if (!L.ucost) return false;
            const double ib = 1.0 / L.ub;
            g.c0 = ib;
            g.c1 = a >= 1 ? -L.am * ib : 0.0;
            e0 = -(L.uc + (a == 0 ? L.am * L.v0 : 0.0)) * ib;
            w = C.Qu;
            break;
        }
        case 5: {  // Q_du |u_{i,a} - u_{i,a-1}| between decided steps
            if (a < 1 || a >= X.Ki) return false;
            const double ib = 1.0 / L.ub, ibm = 1.0 / X.ubm;
            g.c0 = ib;
            g.c1 = -L.am * ib - ibm;
            g.c2 = a >= 2 ? X.amm * ibm : 0.0;
            e0 = -L.uc * ib + (X.ucm + (a == 1 ? X.amm * L.v0 : 0.0)) * ibm;
            w = C.Qdu;
            break;
        }
        case 6:  // w max(0, p_i - p_{i-1} + d_safe) (:170-177; the leader's w.r.t. x_ref, :164-169)
            if (a < 1 || L.sf == 0) return false;
            g.cp = L.ts;
            g.cq = L.sf == 1 ? -L.ts : 0.0;
            e0 = L.sf == 1 ? L.P1 - X.P1m + C.d_safe : L.P1 - I.xl[k] + C.d_safe;
            w = C.w;
            al = 0.0;
            break;
    }
    const bool any = g.cp != 0.0 || g.cq != 0.0 || g.c0 != 0.0 || g.c1 != 0.0 || g.c2 != 0.0 || g.d0 != 0.0;
    return w > 0.0 && any;
}

// entry s of the normal of the row owned by lane l (vehicle il = l / N, step al = l % N)
__device__ inline double lp_gs(const LpG& g, int l, int s, int N) {
    const int s0 = l - l % N;
    double v = 0.0;
    if (s >= s0 && s < l) v += g.cp;
    if (s >= s0 - N && s < l - N) v += g.cq;
    if (s == l) v += g.c0;
    if (s == l - 1) v += g.c1;
    if (s == l - 2) v += g.c2;
    if (s == l - N) v += g.d0;
    return v;
}

// Assembly of one slot of rows (every lane's row of that slot) into the Newton system: lane s
// adds sum_l coef_l g_l[s] to rhs and lam_l g_l[s] to rdy, and (withK) D_l g_l[s] g_l[s'] to the
// lower column s of K (LDS, row stride LD) for s' >= s in the row's support.
__device__ inline void lp_assemble_slot(const Lds& S, int V, int N, bool on, const LpG& g, double D, double coef,
                                        double lam, bool withK, double& rhs, double& rdy) {
    const int t = lane();
    double* dsc = S.desc;
    dsc[t * kLpDesc + 0] = on ? D : 0.0;
    dsc[t * kLpDesc + 1] = on ? coef : 0.0;
    dsc[t * kLpDesc + 2] = on ? lam : 0.0;
    dsc[t * kLpDesc + 3] = g.cp;
    dsc[t * kLpDesc + 4] = g.cq;
    dsc[t * kLpDesc + 5] = g.c0;
    dsc[t * kLpDesc + 6] = g.c1;
    dsc[t * kLpDesc + 7] = g.c2;
    dsc[t * kLpDesc + 8] = g.d0;
    dsc[t * kLpDesc + 9] = on ? 1.0 : 0.0;
    wsync();
    if (t < V) {
        const int s = t;
        for (int l = 0; l < V; ++l) {
            const double* q = dsc + l * kLpDesc;
            if (q[9] == 0.0) continue;  // wave-uniform (broadcast read)
            const LpG gl{q[3], q[4], q[5], q[6], q[7], q[8]};
            const double gsv = lp_gs(gl, l, s, N);
            if (gsv == 0.0) continue;
            rhs += q[1] * gsv;
            rdy += q[2] * gsv;
            if (!withK) continue;
            const double f = q[0] * gsv;
            // support of row l at indices >= s: its own-vehicle prefix [s0, l) (which holds the
            // band points l-1, l-2 whenever c1, c2 are set: they need a >= 1, 2), the previous
            // vehicle's prefix [s0 - N, l - N), and the points l (c0) and l - N (d0)
            const int s0 = l - l % N;
            double* col = S.J + s;
            for (int sp = s0 > s ? s0 : s; sp < l; ++sp) col[sp * S.LD] += f * lp_gs(gl, l, sp, N);
            for (int sp = s0 - N > s ? s0 - N : s; sp < l - N; ++sp) col[sp * S.LD] += f * lp_gs(gl, l, sp, N);
            if (l >= s) col[l * S.LD] += f * gl.c0;
            if (l - N >= s && gl.d0 != 0.0) col[(l - N) * S.LD] += f * gl.d0;
        }
    }
    wsync();
}

// Cholesky K = R R' of the assembled lower triangle (J) into R with hvp_l1.h's infinity rule (a
// pivot that lost its digits, <= 1e-13 of its diagonal, is infinite: its inverse is 0)
__device__ inline void lp_cholesky(const Lds& S, int V) {
    const int t = lane(), LD = S.LD;
    double* J = S.J;
    double* R = S.R;
    for (int j = 0; j < V; ++j) {
        if (t == j) {
            const double d = J[j * LD + j];
            double s = d;
            for (int k = 0; k < j; ++k) s -= R[j * LD + k] * R[j * LD + k];
            R[j * LD + j] = s > 1e-13 * d ? sqrt(s) : 0.0;
        }
        wsync();
        const double dj = R[j * LD + j];
        const double dinv = dj > 0.0 ? 1.0 / dj : 0.0;
        if (t > j && t < V) {
            double v = J[t * LD + j];
            for (int k = 0; k < j; ++k) v -= R[t * LD + k] * R[j * LD + k];
            R[t * LD + j] = v * dinv;
        }
        wsync();
    }
}

// R R' x = b (lane t holds b_t and receives x_t)
__device__ inline double lp_solve_rr(const Lds& S, int V, double b) {
    const int t = lane(), LD = S.LD;
    const double* R = S.R;
    const double rd = t < V ? R[t * LD + t] : 0.0;
    const double ldinv = rd > 0.0 ? 1.0 / rd : 0.0;
    double acc = t < V ? b : 0.0, w = 0.0;
    for (int i = 0; i < V; ++i) {
        const double wi = bcu(acc * ldinv, i);
        if (t == i) w = wi;
        if (t > i && t < V) acc -= R[t * LD + i] * wi;
    }
    double acc2 = w, x = 0.0;
    for (int i = V - 1; i >= 0; --i) {
        const double xi = bcu(acc2 * ldinv, i);
        if (t == i) x = xi;
        if (t < i) acc2 -= R[i * LD + t] * xi;
    }
    return x;
}

// iterate and directions of the lane's rows
struct LpState {
    double hs[kLpHard], hl[kLpHard], hds[kLpHard], hdl[kLpHard];
    double pt[kLpPair], ps1[kLpPair], ps2[kLpPair], pl1[kLpPair], pl2[kLpPair];
    double pds1[kLpPair], pdl1[kLpPair], pds2[kLpPair], pdl2[kLpPair], pdt[kLpPair];
};

// Newton system of the targets rc = s l + (corr ? ds dl : 0) - sigmu: rows slot by slot into
// K (withK) and the lane's rhs; residuals into gap / obj / rpm / rdm when res.
__device__ inline void lp_system(const LpState& Q, const Lane& L, const Consts& C, const Inst& I, const LpCtx& X,
                                 const Lds& S, const LpVals& Y, bool corr, double sigmu, bool withK, double& rhs,
                                 double& rdy, double& gap, double& obj, double& rpm, double& rdm) {
    const int t = lane(), V = I.V, N = I.N, LD = S.LD;
    if (withK && t < V)
        for (int r = t; r < V; ++r) S.J[r * LD + t] = 0.0;
    rhs = 0.0;
    rdy = 0.0;
#pragma unroll
    for (int r = 0; r < kLpHard; ++r) {
        LpG g;
        double h;
        const bool on = lp_hard(r, L, I, g, h);
        double D = 0.0, coef = 0.0, lam = 0.0;
        if (on) {
            const double rp = lp_dot(g, Y) + Q.hs[r] - h;
            D = Q.hl[r] / Q.hs[r];
            const double rc = Q.hs[r] * Q.hl[r] + (corr ? Q.hds[r] * Q.hdl[r] : 0.0) - sigmu;
            const double rho = (Q.hl[r] * rp - rc) / Q.hs[r];
            coef = -(Q.hl[r] + rho);
            lam = Q.hl[r];
            gap += Q.hs[r] * Q.hl[r];
            rpm = fmax(rpm, fabs(rp));
        }
        lp_assemble_slot(S, V, N, on, g, D, coef, lam, withK, rhs, rdy);
    }
#pragma unroll
    for (int r = 0; r < kLpPair; ++r) {
        LpG g;
        double e0, w, al;
        const bool on = lp_pair(r, L, C, I, X, g, e0, w, al);
        double D = 0.0, coef = 0.0, lam = 0.0;
        if (on) {
            const double gy = lp_dot(g, Y);
            const double rp1 = gy - Q.pt[r] + Q.ps1[r] + e0;
            const double rp2 = -al * gy - Q.pt[r] + Q.ps2[r] - al * e0;
            const double D1 = Q.pl1[r] / Q.ps1[r], D2 = Q.pl2[r] / Q.ps2[r];
            const double rc1 = Q.ps1[r] * Q.pl1[r] + (corr ? Q.pds1[r] * Q.pdl1[r] : 0.0) - sigmu;
            const double rc2 = Q.ps2[r] * Q.pl2[r] + (corr ? Q.pds2[r] * Q.pdl2[r] : 0.0) - sigmu;
            const double rho1 = (Q.pl1[r] * rp1 - rc1) / Q.ps1[r], rho2 = (Q.pl2[r] * rp2 - rc2) / Q.ps2[r];
            const double rdt = w - Q.pl1[r] - Q.pl2[r];
            const double rhst = -rdt + rho1 + rho2;
            const double mt = D1 + D2, m = al * D2 - D1;
            D = D1 * D2 * (1.0 + al) * (1.0 + al) / mt;
            coef = -(Q.pl1[r] - al * Q.pl2[r]) - (rho1 - al * rho2) - m * rhst / mt;
            lam = Q.pl1[r] - al * Q.pl2[r];
            gap += Q.ps1[r] * Q.pl1[r] + Q.ps2[r] * Q.pl2[r];
            obj += w * Q.pt[r];
            rpm = fmax(rpm, fmax(fabs(rp1), fabs(rp2)));
            rdm = fmax(rdm, fabs(rdt));
        }
        lp_assemble_slot(S, V, N, on, g, D, coef, lam, withK, rhs, rdy);
    }
}

// directions of the lane's rows for dy (same targets as lp_system), written over the stored ones
// (each row reads its predictor ds dl first); the local step limits into ap / ad
__device__ inline void lp_directions(LpState& Q, const Lane& L, const Consts& C, const Inst& I, const LpCtx& X,
                                     const LpVals& Y, const LpVals& DY, bool corr, double sigmu, double& ap,
                                     double& ad) {
#pragma unroll
    for (int r = 0; r < kLpHard; ++r) {
        LpG g;
        double h;
        if (!lp_hard(r, L, I, g, h)) continue;
        const double gd = lp_dot(g, DY);
        const double rp = lp_dot(g, Y) + Q.hs[r] - h, D = Q.hl[r] / Q.hs[r];
        const double rc = Q.hs[r] * Q.hl[r] + (corr ? Q.hds[r] * Q.hdl[r] : 0.0) - sigmu;
        const double rho = (Q.hl[r] * rp - rc) / Q.hs[r];
        Q.hds[r] = -rp - gd;
        Q.hdl[r] = D * gd + rho;
        l1_ratio(ap, Q.hs[r], Q.hds[r]);
        l1_ratio(ad, Q.hl[r], Q.hdl[r]);
    }
#pragma unroll
    for (int r = 0; r < kLpPair; ++r) {
        LpG g;
        double e0, w, al;
        if (!lp_pair(r, L, C, I, X, g, e0, w, al)) continue;
        const double gy = lp_dot(g, Y), gd = lp_dot(g, DY);
        const double rp1 = gy - Q.pt[r] + Q.ps1[r] + e0;
        const double rp2 = -al * gy - Q.pt[r] + Q.ps2[r] - al * e0;
        const double D1 = Q.pl1[r] / Q.ps1[r], D2 = Q.pl2[r] / Q.ps2[r];
        const double rc1 = Q.ps1[r] * Q.pl1[r] + (corr ? Q.pds1[r] * Q.pdl1[r] : 0.0) - sigmu;
        const double rc2 = Q.ps2[r] * Q.pl2[r] + (corr ? Q.pds2[r] * Q.pdl2[r] : 0.0) - sigmu;
        const double rho1 = (Q.pl1[r] * rp1 - rc1) / Q.ps1[r], rho2 = (Q.pl2[r] * rp2 - rc2) / Q.ps2[r];
        const double rdt = w - Q.pl1[r] - Q.pl2[r];
        const double rhst = -rdt + rho1 + rho2;
        const double mt = D1 + D2, m = al * D2 - D1;
        Q.pdt[r] = (rhst - m * gd) / mt;
        const double a1 = gd - Q.pdt[r], a2 = -al * gd - Q.pdt[r];
        Q.pds1[r] = -rp1 - a1;
        Q.pds2[r] = -rp2 - a2;
        const bool big1 = D1 >= D2;  // the larger-scaled side's multiplier from the t row (hvp_l1.h)
        const double dls = big1 ? D2 * a2 + rho2 : D1 * a1 + rho1;
        Q.pdl1[r] = big1 ? rdt - dls : dls;
        Q.pdl2[r] = big1 ? dls : rdt - dls;
        l1_ratio(ap, Q.ps1[r], Q.pds1[r]);
        l1_ratio(ap, Q.ps2[r], Q.pds2[r]);
        l1_ratio(ad, Q.pl1[r], Q.pdl1[r]);
        l1_ratio(ad, Q.pl2[r], Q.pdl2[r]);
    }
}

__device__ inline double wmin(double x) { return -wmax(-x); }

// The platoon LP of lane data L (hvp_cent.h setup): L1_OK / L1_FAIL (hard-row infeasibility is
// decided before, by platoon_lp).  L.y receives the iterate.
__device__ inline int lp_solve(Lane& L, const Lds& S, const Consts& C, const Inst& I, const LpCtx& X, int max_iter,
                               int& iters) {
    const int N = I.N, V = I.V;
    LpState Q;
    L.y = L.on ? L.v0 : 0.0;
    double hsc = 1.0, wmx = 1.0, cnt = 0.0;
    {
        const LpVals Y = lp_vals(L.y, N, L.on);
#pragma unroll
        for (int r = 0; r < kLpHard; ++r) {
            LpG g;
            double h;
            Q.hds[r] = Q.hdl[r] = 0.0;
            Q.hs[r] = 1.0;
            Q.hl[r] = 0.0;
            if (!lp_hard(r, L, I, g, h)) continue;
            Q.hs[r] = fmax(h - lp_dot(g, Y), 1.0);
            Q.hl[r] = 1.0;
            hsc = fmax(hsc, fabs(h));
            cnt += 1.0;
        }
#pragma unroll
        for (int r = 0; r < kLpPair; ++r) {
            LpG g;
            double e0, w, al;
            Q.pds1[r] = Q.pdl1[r] = Q.pds2[r] = Q.pdl2[r] = Q.pdt[r] = 0.0;
            Q.pt[r] = 0.0;
            Q.ps1[r] = Q.ps2[r] = 1.0;
            Q.pl1[r] = Q.pl2[r] = 0.0;
            if (!lp_pair(r, L, C, I, X, g, e0, w, al)) continue;
            const double e = lp_dot(g, Y) + e0;
            Q.pt[r] = (al > 0.0 ? fabs(e) : fmax(e, 0.0)) + 1.0;
            Q.ps1[r] = Q.pt[r] - e;
            Q.ps2[r] = Q.pt[r] + al * e;
            Q.pl1[r] = 0.5 * w;
            Q.pl2[r] = 0.5 * w;
            wmx = fmax(wmx, w);
            hsc = fmax(hsc, fabs(e0));
            cnt += 2.0;
        }
    }
    hsc = wmax(hsc);
    wmx = wmax(wmx);
    const double mtot = fmax(wsum(cnt), 1.0);
    double ybest = L.y, best = __builtin_inf();  // best iterate (relative gap) for the rescue
    if (I.debug == 5) {  // diagnostics: every lane's rows (g, h / e0, w, al) at the start
#pragma unroll
        for (int r = 0; r < kLpHard; ++r) {
            LpG g;
            double h;
            if (lp_hard(r, L, I, g, h))
                printf("[lp] hard lane %d r %d g %.17g %.17g %.17g %.17g %.17g %.17g h %.17g\n", lane(), r, g.cp,
                       g.cq, g.c0, g.c1, g.c2, g.d0, h);
        }
#pragma unroll
        for (int r = 0; r < kLpPair; ++r) {
            LpG g;
            double e0, w, al;
            if (lp_pair(r, L, C, I, X, g, e0, w, al))
                printf("[lp] pair lane %d r %d g %.17g %.17g %.17g %.17g %.17g %.17g e0 %.17g w %.17g al %g\n", lane(),
                       r, g.cp, g.cq, g.c0, g.c1, g.c2, g.d0, e0, w, al);
        }
    }
    for (iters = 0; iters < max_iter; ++iters) {
        const LpVals Y = lp_vals(L.y, N, L.on);
        double rhs, rdy, gap = 0.0, obj = 0.0, rpm = 0.0, rdm = 0.0;
        lp_system(Q, L, C, I, X, S, Y, false, 0.0, true, rhs, rdy, gap, obj, rpm, rdm);
        gap = wsum(gap);
        obj = wsum(obj);
        rpm = wmax(rpm);
        rdm = fmax(wmax(rdm), wmax(L.on ? fabs(rdy) : 0.0));
        if ((I.debug == 4 || I.debug == 5) && lane() == 0)
            printf("[lp] it %d rpm %.3e/%.3e rdm %.3e/%.3e gap %.3e obj %.9e\n", iters, rpm, 1e-10 * hsc, rdm,
                   1e-10 * wmx, gap, obj);
        const double rgap = gap / fmax(1.0, fabs(obj));
        if (rpm <= 1e-10 * hsc && rdm <= kLpDualTol * wmx && rgap <= kLpGapTol) return L1_OK;
        if (rpm <= 1e-10 * hsc && rdm <= 1e-8 * wmx && rgap < best) {  // wave-uniform
            best = rgap;
            ybest = L.y;
        }
        const double mu = gap / mtot;
        lp_cholesky(S, V);
        double dy = lp_solve_rr(S, V, rhs);
        double ap = 1.0, ad = 1.0;
        LpVals DY = lp_vals(dy, N, L.on);
        lp_directions(Q, L, C, I, X, Y, DY, false, 0.0, ap, ad);
        ap = wmin(ap);
        ad = wmin(ad);
        double gaff = 0.0;
#pragma unroll
        for (int r = 0; r < kLpHard; ++r) {
            LpG g;
            double h;
            if (lp_hard(r, L, I, g, h)) gaff += (Q.hs[r] + ap * Q.hds[r]) * (Q.hl[r] + ad * Q.hdl[r]);
        }
#pragma unroll
        for (int r = 0; r < kLpPair; ++r) {
            LpG g;
            double e0, w, al;
            if (lp_pair(r, L, C, I, X, g, e0, w, al))
                gaff += (Q.ps1[r] + ap * Q.pds1[r]) * (Q.pl1[r] + ad * Q.pdl1[r]) +
                        (Q.ps2[r] + ap * Q.pds2[r]) * (Q.pl2[r] + ad * Q.pdl2[r]);
        }
        gaff = wsum(gaff);
        const double ratio = gaff / gap;
        const double sigmu = ratio * ratio * ratio * mu;
        // corrector (same K, new right-hand side); a short step falls back to pure centring
        for (int pass = 0; pass < 2; ++pass) {
            const bool corr = pass == 0;
            const double sm = corr ? sigmu : kL1Centre * mu;
            double rhs2, rdy2, g2 = 0.0, o2 = 0.0, r2 = 0.0, d2 = 0.0;
            lp_system(Q, L, C, I, X, S, Y, corr, sm, false, rhs2, rdy2, g2, o2, r2, d2);
            dy = lp_solve_rr(S, V, rhs2);
            DY = lp_vals(dy, N, L.on);
            ap = 1.0 / 0.995;
            ad = 1.0 / 0.995;
            lp_directions(Q, L, C, I, X, Y, DY, corr, sm, ap, ad);
            ap = wmin(ap);
            ad = wmin(ad);
            if (fmin(ap, ad) >= kL1Short) break;
        }
        ap *= 0.995;
        ad *= 0.995;
        if (I.debug == 4 || I.debug == 5) {
            const double rdiag = lane() < V ? S.R[lane() * S.LD + lane()] : 1.0;
            const double rmin = wmin(lane() < V ? rdiag : 1e300), rmax = wmax(lane() < V ? rdiag : 0.0);
            const double dyn = wmax(L.on ? fabs(dy) : 0.0);
            if (lane() == 0)
                printf("[lp]    mu %.3e sigmu %.3e ap %.3e ad %.3e |dy| %.3e R diag %.3e..%.3e\n", mu, sigmu, ap, ad,
                       dyn, rmin, rmax);
        }
        if (L.on) L.y += ap * dy;
#pragma unroll
        for (int r = 0; r < kLpHard; ++r) {
            Q.hs[r] += ap * Q.hds[r];
            Q.hl[r] += ad * Q.hdl[r];
        }
#pragma unroll
        for (int r = 0; r < kLpPair; ++r) {
            Q.pt[r] += ap * Q.pdt[r];
            Q.ps1[r] += ap * Q.pds1[r];
            Q.ps2[r] += ap * Q.pds2[r];
            Q.pl1[r] += ad * Q.pdl1[r];
            Q.pl2[r] += ad * Q.pdl2[r];
        }
    }
    if (best <= kLpRescueGap) {
        L.y = ybest;
        return L1_OK;
    }
    return L1_FAIL;
}

// min_1_norm objective of the platoon trajectory, term by term (cent_mld.py:83-140 with
// min_1_norm; relaxed steps a >= K_i priced only in a virtual region, Q_du between decided steps).
// u_lane (optional) receives the lane's input u_{i,a}.
__device__ inline double lp_direct_cost(const Lane& L, const Consts& C, const Inst& I, int Ki, double* u_lane = nullptr) {
    const int t = lane();
    const int N = I.N;
    const double yv = L.on ? L.y : 0.0;
    double vp = shift_up1(yv);
    if (L.a == 0) vp = L.v0;
    const double cum = vehicle_prefix(yv, N);
    const double pn = L.P1 + L.ts * cum, vn = yv;        // state a + 1
    const double pnm = __shfl(pn, t >= N ? t - N : t, W);  // vehicle i-1, same step
    const double vnm = __shfl(vn, t >= N ? t - N : t, W);
    const double p0 = L.on ? I.x0[2 * L.i] : 0.0, v0 = L.v0;
    const double p0m = L.on && L.i >= 1 ? I.x0[2 * (L.i - 1)] : 0.0, v0m = L.on && L.i >= 1 ? I.x0[2 * L.i - 1] : 0.0;
    auto nrm = [&](double ep, double ev) { return C.Qpp * fabs(ep) + C.Qvv * fabs(ev); };
    auto state_terms = [&](int k, double p, double v, double pm, double vm) {
        double Jt = 0.0;
        if (L.i == I.L) Jt += nrm(p - I.xl[k] + (I.lsp ? C.t0 * v + C.d0 : 0.0), v - I.xl[N + 1 + k]);
        if (L.i >= 1) {
            Jt += nrm(p + C.t0 * v + C.d0 - pm, v - vm);
            Jt += C.w * fmax(0.0, p - pm + C.d_safe);
        } else if (I.lsp && I.L == 0) {
            Jt += C.w * fmax(0.0, p - I.xl[k] + C.d_safe);
        }
        return Jt;
    };
    double Jt = 0.0, u = 0.0;
    if (L.on) {
        Jt += state_terms(L.a + 1, pn, vn, pnm, vnm);
        u = (vn - L.am * vp - L.uc) / L.ub;
        if (L.ucost) Jt += C.Qu * fabs(u);
        if (L.a == 0) Jt += state_terms(0, p0, v0, p0m, v0m);
    }
    const double uprev = shift_up1(u);
    if (L.on && L.a >= 1 && L.a < Ki) Jt += C.Qdu * fabs(u - uprev);
    if (u_lane) *u_lane = u;
    return wsum(Jt);
}

}  // namespace cent
}  // namespace hvp
