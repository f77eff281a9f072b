// hvp_coop.h -- the fixed-sequence QP solved by a GROUP of 16 lanes (long horizons, N <= 16).
//
// The lane-per-QP solver (hvp_gi.h) keeps J (N x N) and R (N x N) of the Goldfarb-Idnani method
// in registers: fine up to N ~ 8, but at N = 10 / 15 (C3, C5) it needs 200 / 450 doubles per
// lane and the kernel lives in scratch.  Here one QP is owned by a 16-lane DPP row of the
// wavefront (4 QPs per wave):
//
//   lane t      owns variable y_t = v_{t+1}, the rows of step t+1 (V/U/A) and the position /
//               safe-distance rows of step t+1 (prefix rows of m = t - 1), their active and
//               saturation bits, the multiplier and row id of active position t, and row t of
//               the Hessian during setup;
//   LDS         the group's J (row t of J is lane t's) and R (upper triangular), row stride
//               17 doubles (bank-conflict-free column walks), plus two scratch vectors;
//   shuffles    sums / argmax / scans within the 16-lane group (__shfl*, width 16).
//
// Same algorithm as hvp_gi.h (most violated row, dual step, soft rows with saturation and the
// reversed rows that unsaturate them, the same verification), same velocity-space QP as
// setup_lane / setup_lane_admm (the Hessian rows are assembled in closed form from the per-step
// quadratic forms), so the results agree with the lane solver to rounding.
#pragma once

#include <hip/hip_runtime.h>

#include "hvp_admm.h"
#include "hvp_gi.h"
#include "hvp_ipm.h"

namespace hvp {
namespace coop {

constexpr int G = 16;
constexpr int LD = 17;  // padded LDS row stride (doubles)

struct GroupLds {
    double J[G * LD];
    double R[G * LD];
    double v[G];  // broadcast vector (dv, y*, ...)
    double pad[G];
};

__device__ inline int lane16() { return (int)(threadIdx.x & (G - 1)); }
__device__ inline void gsync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}
__device__ inline double gsum(double x) {
    x += __shfl_xor(x, 8, G);
    x += __shfl_xor(x, 4, G);
    x += __shfl_xor(x, 2, G);
    x += __shfl_xor(x, 1, G);
    return x;
}
__device__ inline int gor(int x) {
    x |= __shfl_xor(x, 8, G);
    x |= __shfl_xor(x, 4, G);
    x |= __shfl_xor(x, 2, G);
    x |= __shfl_xor(x, 1, G);
    return x;
}
__device__ inline unsigned long long gor64(unsigned long long x) {
    x |= __shfl_xor(x, 8, G);
    x |= __shfl_xor(x, 4, G);
    x |= __shfl_xor(x, 2, G);
    x |= __shfl_xor(x, 1, G);
    return x;
}
template <class T>
__device__ inline T bcast(T x, int src) { return __shfl(x, src, G); }
// inclusive prefix sum over the group
__device__ inline double gscan(double x) {
    const int t = lane16();
#pragma unroll
    for (int d = 1; d < G; d <<= 1) {
        const double o = __shfl_up(x, d, G);
        if (t >= d) x += o;
    }
    return x;
}
// group argmin of (key, lane) -> (key, lane); ties to the lower lane
__device__ inline void gargmin(double& key, int& who) {
#pragma unroll
    for (int d = G / 2; d > 0; d >>= 1) {
        const double ok = __shfl_xor(key, d, G);
        const int ow = __shfl_xor(who, d, G);
        if (ok < key || (ok == key && ow < who)) { key = ok; who = ow; }
    }
}
// select x[t] of a register array with a lane-dependent index (predicated, no scratch)
template <int N>
__device__ inline double pick(const double* x, int t) {
    double r = 0.0;
#pragma unroll
    for (int i = 0; i < N; ++i) r = i == t ? x[i] : r;
    return r;
}

// ------------------------------------------------------------------ per-lane problem data
template <int N>
struct Lane {
    // uniform
    double v0, P1, ts, pmin, pmax;
    bool has_sf, has_sb;
    // step t = lane (valid if t < N)
    double am, vlo, vhi, ulo, uhi, dec, acc;
    double ub, uc;  // input map of step t: u = (v_{t+1} - am v_t - uc) / ub
    bool ucost;     // step t carries its input cost (fixed, or relaxed in a virtual region)
    double hf, hb;  // prefix rows of m = t - 1 (t >= 1)
    double y;       // y_t
    double f;       // linear term f_t
};

// Per-step quadratic form of the tracking / copy terms at step k = 1..N (setup_lane's
// Wpp, Wpv, Wvv, lp, lv with the constant folded at pbar = P1).
struct StepForm {
    double Wpp, Wpv, Wvv, lp, lv;
};

template <int N>
__device__ inline StepForm decent_form(const Consts& C, int role, const double* prm, int k) {
    const double* xf = prm + 2;
    const double* xb = prm + 2 + 2 * (N + 1);
    const double* xl = prm + 2 + 4 * (N + 1);
    const bool tf = (role & HVP_ROLE_TRACK_FRONT) != 0, tb = (role & HVP_ROLE_TRACK_BACK) != 0;
    const bool tl = (role & HVP_ROLE_TRACK_LEADER) != 0, lsp = (role & HVP_ROLE_LEADER_SPACING) != 0;
    const double Qpp = C.Qpp, Qpv = C.Qpv, Qvv = C.Qvv, t0 = C.t0, d0 = C.d0;
    StepForm F{0, 0, 0, 0, 0};
    auto add = [&](double m00, double m01, double m11, double r0, double r1) {
        const double qa = Qpp * m00;
        const double qc = Qpp * m01 + Qpv * m11, qd = Qpv * m01 + Qvv * m11;
        F.Wpp += m00 * qa;
        F.Wpv += m00 * qc;
        F.Wvv += m01 * qc + m11 * qd;
        const double Qr0 = Qpp * r0 + Qpv * r1, Qr1 = Qpv * r0 + Qvv * r1;
        F.lp += m00 * Qr0;
        F.lv += m01 * Qr0 + m11 * Qr1;
    };
    const int K1 = N + 1;
    if (tf) add(1.0, t0, 1.0, d0 - xf[k], -xf[K1 + k]);
    if (tb) add(-1.0, 0.0, -1.0, xb[k] + t0 * xb[K1 + k] + d0, xb[K1 + k]);
    if (tl) {
        if (lsp) add(1.0, t0, 1.0, d0 - xl[k], -xl[K1 + k]);
        else add(1.0, 0.0, 1.0, -xl[k], -xl[K1 + k]);
    }
    return F;
}

template <int N>
__device__ inline StepForm admm_form(const Consts& C, int role, const double* prm, int k, uint64_t hs) {
    const double* xl = admm_leader(prm, N);
    const bool hf = (role & HVP_ROLE_SAFE_FRONT) != 0, hb = (role & HVP_ROLE_SAFE_BACK) != 0;
    const bool tf = (role & HVP_ROLE_TRACK_FRONT) != 0, tb = (role & HVP_ROLE_TRACK_BACK) != 0;
    const bool tl = (role & HVP_ROLE_TRACK_LEADER) != 0;
    const int K1 = N + 1;
    double Wpp = 0, Wpv = 0, Wvv = 0, lp = 0, lv = 0, cc = 0;
    if (tl) {
        const double r0 = -xl[k], r1 = -xl[K1 + k];
        Wpp += C.Qpp;
        Wpv += C.Qpv;
        Wvv += C.Qvv;
        lp += C.Qpp * r0 + C.Qpv * r1;
        lv += C.Qpv * r0 + C.Qvv * r1;
    }
    for (int side = 0; side < 2; ++side) {
        if (!(side == 0 ? hf : hb)) continue;
        const double* yy = admm_y(prm, side, N);
        const double* zz = admm_z(prm, side, N);
        CopyTerm T;
        admm_copy(C, side == 0 ? tf : tb, side, yy[k], yy[K1 + k], zz[k], zz[K1 + k], T);
        Wpp += T.Wpp;
        Wpv += T.Wpv;
        Wvv += T.Wvv;
        lp += T.lp;
        lv += T.lv;
        hub_add(T, hub_get(hs, k, side), C.w, Wpp, Wpv, Wvv, lp, lv, cc);
    }
    if (C.form == HVP_FORM_GADMM) gadmm_own_add(C, prm, N, k, Wpp, Wvv, lp, lv, cc);
    return StepForm{Wpp, Wpv, Wvv, lp, lv};
}

// Lane data + this lane's Hessian row (into LDS J area, row t) for region code / relaxation K;
// [lo, hi] (lo <= hi) = exact interval of v_K: the decentralised tail relaxation of
// hvp_ipm.h:relax_step (as setup_lane), each lane propagating it up to its own step.
// need_h = false (group-uniform): the lane data and f only -- a warm start takes the factors of
// the Hessian from its record (warm_start), so H is not assembled.
template <int N>
__device__ inline bool setup(Lane<N>& L, GroupLds& S_lds, const hvp_system& S, const Consts& C, int role,
                             const double* prm, uint64_t code, int K, uint64_t hs, double lo = 0.0,
                             double hi = -1.0, bool need_h = true) {
    const int t = lane16();
    const bool admm = C.form == HVP_FORM_ADMM || C.form == HVP_FORM_GADMM;
    const double p0 = prm[0], v0 = prm[1], ts = S.ts;
    L.v0 = v0;
    L.ts = ts;
    L.P1 = p0 + ts * v0;
    L.pmin = S.pmin;
    L.pmax = S.pmax;
    L.has_sf = !admm && (role & HVP_ROLE_SAFE_FRONT) != 0;
    L.has_sb = !admm && (role & HVP_ROLE_SAFE_BACK) != 0;
    const int tt = t < N ? t : N - 1;
    // relaxed steps tt, tt + 1: virtual regions and the reachable interval of v_{tt+1}
    const bool relax = !admm && lo <= hi;
    int virt0 = -1, virt1 = -1;
    double bm0 = 1.0, bm1 = 1.0, rlo = S.vmin, rhi = S.vmax;
    if (relax && tt + 1 >= K) {
        const int kend = tt + 1 < N ? tt + 1 : N - 1;
        for (int k = K; k <= kend; ++k) {
            double nlo, nhi, bm;
            bool dead;
            const int vr = relax_step(S, C, k, lo, hi, nlo, nhi, bm, dead);
            if (dead) break;
            if (k == tt) {
                virt0 = vr;
                bm0 = bm;
                rlo = nlo;
                rhi = nhi;
            } else {
                virt1 = vr;
                bm1 = bm;
            }
            lo = nlo;
            hi = nhi;
        }
    }
    // dynamics of step k in {tt, tt + 1} (t - 1 .. t + 1 when fixed; relaxed beyond K)
    auto dyn = [&](int k, double& a, double& b, double& c) {
        const int vr = k == tt ? virt0 : (k == tt + 1 ? virt1 : -1);
        const bool fx = k < K;
        const int r = fx ? code_region(code, k) : (vr >= 0 ? vr : 0);
        const bool on = fx || vr >= 0;
        a = on ? S.a[r] : 1.0;
        b = fx ? S.b[r] : (vr >= 0 ? (k == tt ? bm0 : bm1) : 1.0);
        c = on ? S.c[r] : 0.0;
    };
    {
        double a, b, c;
        dyn(tt, a, b, c);
        const bool on = tt < K || virt0 >= 0;
        L.am = a;
        L.ub = b;
        L.uc = c;
        L.ucost = on;
        L.ulo = on ? c + b * S.umin : -1e30;
        L.uhi = on ? c + b * S.umax : 1e30;
        if (tt + 1 < K) {
            const int r1 = code_region(code, tt + 1);
            L.vlo = fmax(S.vmin, S.vlo[r1]);
            L.vhi = fmin(S.vmax, S.vhi[r1]);
        } else if (relax && tt >= K) {  // relaxed v_{tt+1}: its reachable interval
            L.vlo = fmax(S.vmin, rlo);
            L.vhi = fmin(S.vmax, rhi);
        } else {
            L.vlo = S.vmin;
            L.vhi = S.vmax;
        }
        L.dec = C.dec[tt];
        L.acc = C.acc[tt];
        // prefix rows of m = t - 1: safe rows at step k = t + 1 (inert when absent)
        const double* xf = prm + 2;
        const double* xb = prm + 2 + 2 * (N + 1);
        const int m = tt >= 1 ? tt - 1 : 0;
        const double reach = ts * (m + 1);
        L.hf = L.has_sf ? xf[m + 2] - C.d_safe : L.P1 + reach * S.vmax + 100.0;
        L.hb = L.has_sb ? xb[m + 2] + C.d_safe : L.P1 + reach * S.vmin - 100.0;
    }
    // ---- Hessian row t and f_t from the per-step forms: lane t evaluates the form of ITS step
    // k = t + 1 only; the suffix sums over k (Spp(m) = sum_{k >= m} 2 Wpp_k ts^2, likewise the
    // prefix gradient) are group scans, and the entries right of the diagonal come from the
    // column owner's lane:
    //   H[t][c] = Spp(max(t, c) + 2) + 2 Wpv_{max(t,c)+1} ts (c != t),  H[t][t] = 2 Wvv_{t+1} + Spp(t + 2)
    //   f_t = 2 (Wpv_{t+1} P1 + lv_{t+1}) + sum_{k >= t+2} ts 2 (Wpp_k P1 + lp_k)
    double* Hrow = S_lds.J + (t < N ? t : 0) * LD;  // row t (lanes >= N never store)
    const double P1 = L.P1;
    StepForm F{0, 0, 0, 0, 0};
    if (t < N) F = admm ? admm_form<N>(C, role, prm, t + 1, hs) : decent_form<N>(C, role, prm, t + 1);
    const double wgp = t < N ? ts * 2.0 * (F.Wpp * P1 + F.lp) : 0.0;
    // suffix sums: total - inclusive prefix + own
    const double pre_gp = gscan(wgp);
    const double tot_gp = bcast(pre_gp, G - 1);
    const double suf_gp = tot_gp - pre_gp + wgp;
    const double sgp_next = __shfl_down(suf_gp, 1, G);
    const double sgp2 = t + 1 < N ? sgp_next : 0.0;
    if (need_h) {
        const double wpp = t < N ? 2.0 * F.Wpp * ts * ts : 0.0;
        const double pre_pp = gscan(wpp);
        const double tot_pp = bcast(pre_pp, G - 1);
        const double suf_pp = tot_pp - pre_pp + wpp;  // Spp(t + 1) at lane t
        const double spp_next = __shfl_down(suf_pp, 1, G);  // Spp(t + 2)
        const double spp2 = t + 1 < N ? spp_next : 0.0;
        const double wpv2 = 2.0 * F.Wpv * ts;
        const double colv = spp2 + wpv2;  // value of column t in the rows above it
#pragma unroll
        for (int c = 0; c < N; ++c) {
            const double cv = bcast(colv, c);
            if (t < N) Hrow[c] = c < t ? spp2 + wpv2 : (c > t ? cv : 2.0 * F.Wvv + spp2);
        }
    }
    double f = 2.0 * (F.Wpv * P1 + F.lv) + sgp2;
    // input cost Qu u_k^2 (k < K) and variation Qdu (u_{k+1} - u_k)^2 (k + 1 < K)
    auto ucoef = [&](int k, double& ub, double& gk, double& gkm) {
        double a, b, c;
        dyn(k, a, b, c);
        const double ib = 1.0 / b;
        ub = k == 0 ? -(a * v0 + c) * ib : -c * ib;
        gk = ib;
        gkm = k == 0 ? 0.0 : -a * ib;
    };
    const double w2 = 2.0 * C.Qu;
    if (t < N) {
        double ub, gk, gkm;
        ucoef(t, ub, gk, gkm);
        if (L.ucost) {
            if (need_h) Hrow[t] += w2 * gk * gk;
            f += w2 * ub * gk;
            if (need_h && t >= 1) Hrow[t - 1] += w2 * gk * gkm;
        }
        if (t + 1 < N && (t + 1 < K || virt1 >= 0)) {
            double ub1, gk1, gkm1;
            ucoef(t + 1, ub1, gk1, gkm1);
            if (need_h) Hrow[t] += w2 * gkm1 * gkm1;
            f += w2 * ub1 * gkm1;
            if (need_h) Hrow[t + 1] += w2 * gk1 * gkm1;
        }
        if (C.Qdu != 0.0) {
            const double wd = 2.0 * C.Qdu;
            for (int k = t - 1; k <= t + 1; ++k) {
                if (k < 0 || k + 1 >= N || !(k + 1 < K)) continue;
                double ubk, gkk, gkmk, ubk1, gkk1, gkmk1;
                ucoef(k, ubk, gkk, gkmk);
                ucoef(k + 1, ubk1, gkk1, gkmk1);
                // e = u_{k+1} - u_k: entries k+1: gk_{k+1}; k: gkm_{k+1} - gk_k; k-1: -gkm_k
                const double g_kp = gkk1, g_k = gkmk1 - gkk, g_km = k >= 1 ? -gkmk : 0.0;
                const double eb = ubk1 - ubk;
                const double gt = t == k + 1 ? g_kp : (t == k ? g_k : (t == k - 1 ? g_km : 0.0));
                if (gt == 0.0) continue;
                f += wd * eb * gt;
                if (need_h) {
                    Hrow[k + 1] += wd * gt * g_kp;
                    Hrow[k] += wd * gt * g_k;
                    if (k >= 1) Hrow[k - 1] += wd * gt * g_km;
                }
            }
        }
    }
    L.f = t < N ? f : 0.0;
    return L.P1 >= S.pmin - 1e-9 * (1.0 + fabs(S.pmin)) && L.P1 <= S.pmax + 1e-9 * (1.0 + fabs(S.pmax));
}

// Row-local constraint evaluation: the rows lane t owns, in the order of hvp_gi.h.
// id < 6N: 6t + {V_lo, V_hi, U_lo, U_hi, A_lo, A_hi}; prefix rows 6N + 4(t-1) + {P_lo, P_hi, SF, SB}.
template <int N>
__device__ inline void most_violated_lane(const Lane<N>& L, const Consts& C, double y, double yprev, double cum,
                                          unsigned act, unsigned sat, double tol, double& best_score, int& best_id,
                                          double& best_slack) {
    const int t = lane16();
    best_score = -1.0;
    best_id = -1;
    best_slack = 0.0;
    if (t >= N) return;
    double best_v2 = 0.0, best_nn = 1.0;
    auto consider = [&](int local, int id, double slack, double nn, double scale) {
        if (((act >> local) & 1u) || !(slack < -tol * scale)) return;
        const double v2 = slack * slack;
        if (best_id < 0 || v2 * best_nn > best_v2 * nn) {
            best_id = id;
            best_v2 = v2;
            best_nn = nn;
            best_slack = slack;
        }
    };
    const int j = t;
    const double a = L.am;
    const double gv = y, gu = y - a * yprev, ga = y - yprev;
    const double nu = j ? 1.0 + a * a : 1.0, na = j ? 2.0 : 1.0;
    consider(0, 6 * j + 0, gv - L.vlo, 1.0, 1.0 + fabs(L.vlo));
    consider(1, 6 * j + 1, L.vhi - gv, 1.0, 1.0 + fabs(L.vhi));
    consider(2, 6 * j + 2, gu - L.ulo, nu, 1.0 + fabs(L.ulo) + fabs(a * yprev));
    consider(3, 6 * j + 3, L.uhi - gu, nu, 1.0 + fabs(L.uhi) + fabs(a * yprev));
    consider(4, 6 * j + 4, ga - L.dec, na, 1.0 + fabs(yprev));
    consider(5, 6 * j + 5, L.acc - ga, na, 1.0 + fabs(yprev));
    if (t >= 1) {
        const int m = t - 1;
        const double p = L.P1 + L.ts * cum;  // cum = y_0 + .. + y_m
        const double nn = L.ts * L.ts * (m + 1);
        const double sc = 1.0 + fabs(p);
        const int b = 6 * N + 4 * m;
        consider(6, b + 0, p - L.pmin, nn, sc);
        consider(7, b + 1, L.pmax - p, nn, sc);
        const double sfw = L.hf - p, sbw = p - L.hb;
        const bool satf = sat & 1u, satb = (sat >> 1) & 1u;
        consider(8, satf ? (b + 2) | GI_REV : b + 2, satf ? -sfw : sfw, nn, sc);
        consider(9, satb ? (b + 3) | GI_REV : b + 3, satb ? -sbw : sbw, nn, sc);
    }
    if (best_id >= 0) best_score = best_v2 / best_nn;
}

// owner lane and local bit of a row id
template <int N>
__device__ inline void row_owner(int id_in, int& lane, int& bit) {
    const int id = id_in & (GI_REV - 1);
    if (id < 6 * N) {
        lane = id / 6;
        bit = id % 6;
    } else {
        const int m = (id - 6 * N) / 4;
        lane = m + 1;
        bit = 6 + (id - 6 * N) % 4;
    }
}

// Final state of one QP's active-set solve, kept in HBM between the ADMM iterations of the
// switching ADMM (one record per local QP): the region code and hinge states it was solved for,
// the active rows in position order and the factors J (= L^-T Q, rows) and R (upper, rows) of
// that active set.  Next iteration the QP differs only in its linear term and row bounds (the
// ADMM y, z terms), so with the same code and hinge states the Hessian -- and J, R -- are the
// same, and the equality-constrained optimum on the old active set is two triangular solves and
// two N x N products away (warm_start below).  `key` names the rest of what the Hessian depends
// on (system index, role bits): a record written for another QP -- a handle called again with a
// different batch -- never starts this one.  RS: the row stride of the factors (G for the
// switching ADMM's per-QP records; N for the naive ADMM's node records, hvp_lane.h node_index,
// which are kept per tree node and so are many).
template <int RS_>
struct WarmRec {
    static constexpr int RS = RS_;
    uint64_t code, hs, key;
    int32_t nact, valid;
    int32_t ids[RS_];
    double J[RS_ * RS_];
    double R[RS_ * RS_];
};
using WarmQp = WarmRec<G>;

// right-hand side dd of row p in the group's >= form (n = -c, slack dd + n.y): every lane
// calls it with the same p; the owner lane computes the bound, the group receives it
template <int N>
__device__ inline double row_dd(const Lane<N>& L, int p) {
    const int t = lane16();
    const int base = p & (GI_REV - 1);
    const bool rev = (p & GI_REV) != 0;
    double dloc = 0.0;
    int ol, ob;
    row_owner<N>(p, ol, ob);
    if (base < 6 * N) {
        const int rj = base / 6, r = base % 6, pair = r / 2;
        if (t == rj) {
            const double a = pair == 1 ? L.am : (pair == 2 ? 1.0 : 0.0);
            double lo, hi;
            if (pair == 0) { lo = L.vlo; hi = L.vhi; }
            else if (pair == 1) { lo = L.ulo; hi = L.uhi; }
            else { lo = L.dec; hi = L.acc; }
            const double cst = rj == 0 ? -a * L.v0 : 0.0;
            dloc = (r & 1) ? hi - cst : -(lo - cst);
        }
    } else {
        const int rm = (base - 6 * N) / 4, r = (base - 6 * N) % 4;
        if (t == rm + 1) {
            if (r == 0) dloc = L.P1 - L.pmin;
            else if (r == 1) dloc = L.pmax - L.P1;
            else if (r == 2) dloc = L.hf - L.P1;
            else dloc = L.P1 - L.hb;
        }
    }
    return (rev ? -1.0 : 1.0) * bcast(dloc, ol);
}

// row_dd of every lane's own row p (lanes with p < 0 get 0): the owner lanes' bounds gathered all
// at once (independent cross-lane reads) where row_dd takes two dependent broadcasts per row
template <int N>
__device__ inline double own_row_dd(const Lane<N>& L, int p) {
    const int t = lane16();
    int ol = t, ob = 0;
    if (p >= 0) row_owner<N>(p, ol, ob);
    const double am = __shfl(L.am, ol, G), vlo = __shfl(L.vlo, ol, G), vhi = __shfl(L.vhi, ol, G);
    const double ulo = __shfl(L.ulo, ol, G), uhi = __shfl(L.uhi, ol, G);
    const double dec = __shfl(L.dec, ol, G), acc = __shfl(L.acc, ol, G);
    const double hf = __shfl(L.hf, ol, G), hb = __shfl(L.hb, ol, G);
    if (p < 0) return 0.0;
    const int base = p & (GI_REV - 1);
    const bool rev = (p & GI_REV) != 0;
    double dloc;
    if (base < 6 * N) {
        const int rj = base / 6, r = base % 6, pair = r / 2;
        const double a = pair == 1 ? am : (pair == 2 ? 1.0 : 0.0);
        const double lo = pair == 0 ? vlo : (pair == 1 ? ulo : dec);
        const double hi = pair == 0 ? vhi : (pair == 1 ? uhi : acc);
        const double cst = rj == 0 ? -a * L.v0 : 0.0;
        dloc = (r & 1) ? hi - cst : -(lo - cst);
    } else {
        const int r = (base - 6 * N) % 4;
        if (r == 0) dloc = L.P1 - L.pmin;
        else if (r == 1) dloc = L.pmax - L.P1;
        else if (r == 2) dloc = hf - L.P1;
        else dloc = L.P1 - hb;
    }
    return (rev ? -1.0 : 1.0) * dloc;
}

// w (lane t: w1 = R^-T b at the active positions t < na, -s beyond) and u = R^-1 (w1 + s1) of the
// active rows ids (lane j: row of position j) with the factors J, R at (Jp, Rp), row stride rs;
// s = J' f, b_j = -dd of row j.  Every lane of the group calls it.
template <int N>
__device__ inline void warm_solve(const Lane<N>& L, GroupLds& Sg, const double* Jp, const double* Rp, int rs, int na,
                                  int myid, double& w, double& uu) {
    const int t = lane16();
    const double b = -own_row_dd<N>(L, t < na ? myid : -1);
    double* v = Sg.v;
    gsync();
    v[t] = t < N ? L.f : 0.0;
    gsync();
    double s = 0.0;
    if (t < N) {
#pragma unroll
        for (int i = 0; i < N; ++i) s += Jp[i * rs + t] * v[i];
    }
    w = t < N && t >= na ? -s : 0.0;
    {
        double acc = t < na ? b : 0.0;
        for (int j = 0; j < na; ++j) {
            double wj = 0.0;
            if (t == j) wj = acc / Rp[j * rs + j];
            wj = bcast(wj, j);
            if (t == j) w = wj;
            if (t > j && t < na) acc -= Rp[j * rs + t] * wj;
        }
    }
    uu = 0.0;
    {
        double acc = t < na ? w + s : 0.0;
        for (int j = na - 1; j >= 0; --j) {
            double uj = 0.0;
            if (t == j) uj = acc / Rp[j * rs + j];
            uj = bcast(uj, j);
            if (t == j) uu = uj;
            if (t < j) acc -= Rp[t * rs + j] * uj;
        }
    }
}

enum { WARM_COLD = 0, WARM_OK = 1, WARM_LOST = 2, WARM_DROPPED = 3 };
constexpr int kWarmDrops = 4;

// The equality-constrained optimum on the active set of the last solve (WarmQp), made dual
// feasible: y = J1 R^-T b - J2 J2' f, u = R^-1 (R^-T b + J1' f) with b_j = -dd of active row j
// (n_j.y = b_j).  When a multiplier is negative (the new linear term or bounds moved the optimum
// off a row), the most negative row leaves the set -- a column of R out,
// Givens rotations back to triangular, J's columns rotated alike, as Goldfarb-Idnani's own drop --
// up to kWarmDrops times (a row left out is added back by the loop if the new point violates it).
// The record's factors are read into LDS first (over H: independent loads, where the substitutions
// would otherwise wait on global loads one after another).  WARM_OK: J, R in LDS, L.y, u, id, act,
// nact set, and Goldfarb-Idnani continues from there (WARM_DROPPED: the same after drops, so the
// factors in LDS no longer equal the record's).  WARM_COLD: an unusable record, nothing
// touched.  WARM_LOST: still infeasible after the drops -- the Hessian in LDS is overwritten, and
// the caller sets the QP up again for a cold start.
// Multipliers down to -1e-9 w count as zero (clamped).
template <int N, class W>
__device__ inline int warm_start(Lane<N>& L, GroupLds& Sg, const Consts& C, const W* wq, double& u, int& id,
                                 unsigned& act, int& nact) {
    constexpr int RS = W::RS;
    static_assert(RS >= N, "record rows shorter than the horizon");
    const int t = lane16();
    int na = wq->nact;
    if (na < 0 || na > N) return WARM_COLD;
    int myid = t < na ? wq->ids[t] : -1;
    // the factors into LDS (over H): independent loads, one row per lane
    double* J = Sg.J;
    double* R = Sg.R;
    if (t < N) {  // (lane t's own rows: nobody reads H in between)
#pragma unroll
        for (int c = 0; c < N; ++c) {
            J[t * LD + c] = wq->J[t * RS + c];
            R[t * LD + c] = wq->R[t * RS + c];
        }
    }
    gsync();
    const double wgt = C.w;
    double w, uu;
    warm_solve<N>(L, Sg, J, R, LD, na, myid, w, uu);
    auto verdict = [&]() {  // 0 dual feasible, 1 a negative multiplier, 2 a soft row above w
        int neg = 0, over = 0;
        if (t < na) {
            if (!(uu >= -1e-9 * wgt)) neg = 1;  // NaN-safe
            if (gi_soft<N>(myid) && uu > wgt) over = 1;
        }
        return gor(over) ? 2 : (gor(neg) ? 1 : 0);
    };
    int vd = verdict();
    // drop the most negative multiplier's row until the rest is dual feasible
    int drop_n = 0;
    for (; vd == 1; ++drop_n) {
        if (drop_n == kWarmDrops || na == 0) return WARM_LOST;
        // NaN-safe key: a NaN multiplier (flagged negative by verdict) is the most negative, so
        // the xor butterfly compares ordered values only and every lane agrees on `drop`
        double key = t < na ? (uu == uu ? uu : -1e300) : 1e300;
        int drop = t;
        gargmin(key, drop);
        const int id_n = __shfl_down(myid, 1, G);
        if (t >= drop && t < na - 1) myid = id_n;
        if (t == na - 1) myid = -1;
        if (t < N) {
#pragma unroll
            for (int j = 0; j < N - 1; ++j)
                if (j >= drop && j < na - 1) R[t * LD + j] = R[t * LD + j + 1];
#pragma unroll
            for (int j = 0; j < N; ++j)
                if (j == na - 1) R[t * LD + j] = 0.0;
        }
        gsync();
#pragma unroll
        for (int i = 0; i < N - 1; ++i) {
            if (i >= drop && i < na - 1) {
                double gc, gs;
                givens(R[i * LD + i], R[(i + 1) * LD + i], gc, gs);
                gsync();
                if (t >= i && t < na - 1) {
                    const double a0 = R[i * LD + t], a1 = R[(i + 1) * LD + t];
                    R[i * LD + t] = gc * a0 + gs * a1;
                    R[(i + 1) * LD + t] = -gs * a0 + gc * a1;
                }
                if (t < N) {
                    const double a0 = J[t * LD + i], a1 = J[t * LD + i + 1];
                    J[t * LD + i] = gc * a0 + gs * a1;
                    J[t * LD + i + 1] = -gs * a0 + gc * a1;
                }
                gsync();
            }
        }
        --na;
        warm_solve<N>(L, Sg, J, R, LD, na, myid, w, uu);
        vd = verdict();
    }
    if (vd == 2) return WARM_LOST;
    // y_t = sum_c J[t][c] w_c
    double* v = Sg.v;
    gsync();
    v[t] = w;
    gsync();
    double y = 0.0;
    if (t < N) {
#pragma unroll
        for (int c = 0; c < N; ++c) y += J[t * LD + c] * v[c];
        L.y = y;
    }
    u = t < na ? fmax(uu, 0.0) : 0.0;
    id = myid;
    act = 0;
    for (int j = 0; j < na; ++j) {
        int ol, ob;
        row_owner<N>(bcast(myid, j), ol, ob);
        if (t == ol) act |= 1u << ob;
    }
    nact = na;
    gsync();
    return drop_n ? WARM_DROPPED : WARM_OK;
}

// Cooperative Goldfarb-Idnani.  On GI_OK lane t < N holds y_t in L.y.
// wq (optional): the QP's WarmQp record -- tried as the starting active set when it was written
// for the same code and hinge states (wcode, whs) and wtry is set; rewritten on success.
// no_h: the caller did not assemble H (setup need_h = false) -- any start but the record's is lost.
template <int N, class W = WarmQp>
__device__ inline int solve(Lane<N>& L, GroupLds& Sg, const Consts& C, int max_iter, int& iters,
                            unsigned* edge = nullptr, W* wq = nullptr, uint64_t wcode = 0, uint64_t whs = 0,
                            bool wtry = false, uint64_t wkey = 0, bool no_h = false) {
    constexpr int RS = W::RS;
    const int t = lane16();
    iters = 0;
    double* J = Sg.J;  // holds H on entry (row t written by lane t)
    double* R = Sg.R;
    double u = 0.0;  // multiplier of active position t
    int id = -1;     // row id of active position t
    int nact = 0;
    unsigned act = 0;  // active bits of the rows lane t owns
    gsync();
    int warmed = WARM_COLD;
    if (wq && wtry && wq->valid && wq->code == wcode && wq->hs == whs && wq->key == wkey)  // group-uniform
        warmed = warm_start<N, W>(L, Sg, C, wq, u, id, act, nact);
    const bool warm_ok = warmed == WARM_OK || warmed == WARM_DROPPED;
    if (warmed == WARM_LOST || (no_h && !warm_ok)) {
        iters = 0;
        return GI_WARM_LOST;
    }
    if (warmed == WARM_COLD) {
    // ---- Cholesky H = L L' into R area (lower, row-major), column by column
#pragma unroll
    for (int j = 0; j < N; ++j) {
        // diagonal (lane j)
        if (t == j) {
            double s = J[j * LD + j];
            for (int k = 0; k < j; ++k) s -= R[j * LD + k] * R[j * LD + k];
            R[j * LD + j] = s > 0.0 ? sqrt(s) : -1.0;
        }
        gsync();
        const double d = R[j * LD + j];
        if (!(d > 0.0)) return GI_FAIL_CHOL;
        if (t > j && t < N) {
            double v = J[t * LD + j];
            for (int k = 0; k < j; ++k) v -= R[t * LD + k] * R[j * LD + k];
            R[t * LD + j] = v / d;
        }
        gsync();
    }
    // ---- unconstrained minimiser: L w = -f, L' y = w
    double w = 0.0;  // w_t at lane t
    {
        double acc = -L.f;
#pragma unroll
        for (int i = 0; i < N; ++i) {
            double wi = 0.0;
            if (t == i) wi = acc / R[i * LD + i];
            wi = bcast(wi, i);
            if (t == i) w = wi;
            if (t > i && t < N) acc -= R[t * LD + i] * wi;
        }
        // back substitution: y_i = (w_i - sum_{k>i} L[k][i] y_k) / L[i][i]
        double acc2 = w;
        L.y = 0.0;
#pragma unroll
        for (int i = N - 1; i >= 0; --i) {
            double yi = 0.0;
            if (t == i) yi = acc2 / R[i * LD + i];
            yi = bcast(yi, i);
            if (t == i) L.y = yi;
            // lanes k < i need L[i][k] (row i, column k): read from LDS
            if (t < i) acc2 -= R[i * LD + t] * yi;
        }
    }
    // ---- J = L^-T: row t of J = column t of L^-1 (forward substitution of e_t, all lanes)
    {
        // row t of J is column t of L^-1: forward substitution written in place (H is dead)
        gsync();
        if (t < N) {
            for (int i = 0; i < N; ++i) {
                double v = i == t ? 1.0 : 0.0;
                for (int k = 0; k < i; ++k) v -= R[i * LD + k] * J[t * LD + k];
                J[t * LD + i] = v / R[i * LD + i];
            }
        }
        gsync();
        // R starts empty
        if (t < N)
            for (int c = 0; c < N; ++c) R[t * LD + c] = 0.0;
        gsync();
    }
    }  // cold start
    unsigned sat = 0;  // saturation bits (SF = 1, SB = 2) of lane t's prefix rows
    const double wgt = C.w;
    const double tol = 1e-11;
    int iter = 0;
    for (;;) {
        // ---------------- most violated row
        const double yv = t < N ? L.y : 0.0;
        double yprev = __shfl_up(yv, 1, G);
        if (t == 0) yprev = L.v0;
        const double cum = gscan(yv) - yv;  // y_0 + .. + y_{t-1}
        double score;
        int bid;
        double bsl;
        most_violated_lane<N>(L, C, yv, yprev, cum, act, sat, tol, score, bid, bsl);
        double key = -score;
        int who = t;
        gargmin(key, who);
        if (!(key < 0.0)) break;  // no violated row
        const int p = bcast(bid, who);
        const bool psoft = gi_soft<N>(p);
        // row normal: np_i = -c_i (>= form), rhs dp = -d
        const int base = p & (GI_REV - 1);
        const bool rev = (p & GI_REV) != 0;
        int rj = 0, rtype = 0, rm = 0;
        double rsgn = 1.0, ra = 0.0, d = 0.0;
        // bound d computed by the owner lane
        double dloc = 0.0;
        {
            int ol, ob;
            row_owner<N>(p, ol, ob);
            if (base < 6 * N) {
                rj = base / 6;
                const int r = base % 6, pair = r / 2;
                rtype = 0;
                rsgn = (r & 1) ? 1.0 : -1.0;
                if (t == rj) {
                    const double a = pair == 1 ? L.am : (pair == 2 ? 1.0 : 0.0);
                    double lo, hi;
                    if (pair == 0) { lo = L.vlo; hi = L.vhi; }
                    else if (pair == 1) { lo = L.ulo; hi = L.uhi; }
                    else { lo = L.dec; hi = L.acc; }
                    const double cst = rj == 0 ? -a * L.v0 : 0.0;
                    dloc = (r & 1) ? hi - cst : -(lo - cst);
                }
                ra = bcast(pair == 1 ? L.am : (pair == 2 ? 1.0 : 0.0), rj);
            } else {
                rm = (base - 6 * N) / 4;
                const int r = (base - 6 * N) % 4;
                rtype = 1;
                rsgn = (r == 1 || r == 2) ? 1.0 : -1.0;
                if (t == rm + 1) {
                    if (r == 0) dloc = L.P1 - L.pmin;
                    else if (r == 1) dloc = L.pmax - L.P1;
                    else if (r == 2) dloc = L.hf - L.P1;
                    else dloc = L.P1 - L.hb;
                }
            }
            d = bcast(dloc, ol);
        }
        const double flip = rev ? -1.0 : 1.0;
        // c_i of row p for index i (uniform across lanes)
        auto cof = [&](int i) -> double {
            double c;
            if (rtype == 0) c = (i == rj ? rsgn : 0.0) + (i + 1 == rj ? -rsgn * ra : 0.0);
            else c = i <= rm ? rsgn * L.ts : 0.0;
            return flip * c;
        };
        const double dd = flip * d;
        const double np_t = t < N ? -cof(t) : 0.0;
        const double dp = dd;  // slack of row p at y: n.y + dp = d - c.y
        double unew = 0.0;
        for (;;) {
            if (++iter > max_iter) { iters = iter; return GI_FAIL_ITER; }
            // ---- dv_c = sum_i J[i][c] np_i  (lane c)
            double dv = 0.0;
            if (t < N) {
#pragma unroll
                for (int i = 0; i < N; ++i) {
                    const double ni = -cof(i);
                    if (ni != 0.0) dv += J[i * LD + t] * ni;
                }
            }
            double* dvr = Sg.v;  // dv, shared by the group
            dvr[t] = dv;
            gsync();
            const double dn = gsum(dv * dv);
            const double d2n = gsum(t >= nact ? dv * dv : 0.0);
            // ---- z_t = sum_{c >= nact} J[t][c] dv_c
            double z = 0.0;
            if (t < N) {
                for (int c = nact; c < N; ++c) z += J[t * LD + c] * dvr[c];
            }
            // ---- r = R^-1 dv (active part), column-oriented back substitution
            double r = 0.0;
            {
                double accr = t < nact ? dv : 0.0;
#pragma unroll
                for (int j = N - 1; j >= 0; --j) {
                    if (j >= nact) continue;
                    double rj_ = 0.0;
                    if (t == j) rj_ = accr / R[j * LD + j];
                    rj_ = bcast(rj_, j);
                    if (t == j) r = rj_;
                    if (t < j) accr -= R[t * LD + j] * rj_;
                }
            }
            // ---- step lengths
            double k1key = 1e300;
            int k1 = t;
            if (t < nact && r > 0.0) k1key = u / r;
            gargmin(k1key, k1);
            const double t1 = k1key;
            double k3key = 1e300;
            int k3 = t;
            if (t < nact && gi_soft<N>(id) && r < 0.0) k3key = (wgt - u) / (-r);
            gargmin(k3key, k3);
            double t3 = k3key;
            bool new_sat = false;
            if (psoft && wgt - unew <= t3) {
                t3 = wgt - unew;
                new_sat = true;
            }
            const bool zstep = d2n > 1e-14 * dn;
            const double zn = d2n;
            const double sp_now = dp + gsum(np_t * (t < N ? L.y : 0.0));
            const double t2 = zstep && zn > 0.0 ? fmax(-sp_now, 0.0) / zn : 1e300;
            const double tstep = fmin(t1, fmin(t2, t3));
            if (!(tstep < 1e299)) { iters = iter; return GI_FAIL_DUAL; }
            if (t2 < 1e299 && t < N) L.y += tstep * z;
            if (t < nact) u -= tstep * r;
            unew += tstep;
            if (t2 <= t1 && t2 <= t3) {
                // ---- add p: Givens zeroing dv[nact+1 .. N-1] bottom-up, rotating J's columns
                // (every lane runs the same rotation sequence on its register copy of the pair)
                double carry = N - 1 > nact ? dvr[N - 1] : 0.0;
                for (int i = N - 1; i > nact; --i) {
                    const double lo = dvr[i - 1];
                    double gc, gs;
                    givens(lo, carry, gc, gs);
                    carry = gc * lo + gs * carry;
                    if (t < N) {
                        const double a0 = J[t * LD + i - 1], a1 = J[t * LD + i];
                        J[t * LD + i - 1] = gc * a0 + gs * a1;
                        J[t * LD + i] = -gs * a0 + gc * a1;
                    }
                }
                // after the sweep dv[nact] = carry, dv[0..nact-1] unchanged
                if (t < nact) R[t * LD + nact] = dv;
                if (t == nact) R[t * LD + nact] = N - 1 > nact ? carry : dv;
                if (t == nact) { u = unew; id = p; }
                {
                    int ol, ob;
                    row_owner<N>(p, ol, ob);
                    if (t == ol) act |= 1u << ob;
                }
                ++nact;
                gsync();
                break;
            }
            // ---- a row leaves the active set
            int drop;
            const bool by_sat = t3 <= t1;
            if (by_sat) {
                if (new_sat) {
                    // the new soft row saturates: it joins the objective
                    int ol, ob;
                    row_owner<N>(p, ol, ob);
                    if (t == ol) sat ^= 1u << (ob - 8);  // SF -> bit 0, SB -> bit 1 (GI_REV toggles back)
                    gsync();
                    break;
                }
                drop = k3;
            } else {
                drop = k1;
            }
            const int dropped = bcast(id, drop);
            {
                int ol, ob;
                row_owner<N>(dropped, ol, ob);
                if (t == ol) {
                    act &= ~(1u << ob);
                    if (by_sat) sat ^= 1u << (ob - 8);
                }
            }
            // shift positions drop.. nact-2 (u, id, R columns)
            const double u_n = __shfl_down(u, 1, G);
            const int id_n = __shfl_down(id, 1, G);
            if (t >= drop && t < nact - 1) { u = u_n; id = id_n; }
            if (t == nact - 1) { u = 0.0; id = -1; }
            if (t < N) {
#pragma unroll
                for (int j = 0; j < N - 1; ++j)
                    if (j >= drop && j < nact - 1) R[t * LD + j] = R[t * LD + j + 1];
#pragma unroll
                for (int j = 0; j < N; ++j)
                    if (j == nact - 1) R[t * LD + j] = 0.0;
            }
            gsync();
            // re-triangularise: rotations of rows (i, i+1), i = drop .. nact-2
#pragma unroll
            for (int i = 0; i < N - 1; ++i) {
                if (i >= drop && i < nact - 1) {
                    double gc, gs;
                    givens(R[i * LD + i], R[(i + 1) * LD + i], gc, gs);
                    gsync();
                    if (t >= i && t < nact - 1) {
                        const double a0 = R[i * LD + t], a1 = R[(i + 1) * LD + t];
                        R[i * LD + t] = gc * a0 + gs * a1;
                        R[(i + 1) * LD + t] = -gs * a0 + gc * a1;
                    }
                    if (t < N) {
                        const double a0 = J[t * LD + i], a1 = J[t * LD + i + 1];
                        J[t * LD + i] = gc * a0 + gs * a1;
                        J[t * LD + i + 1] = -gs * a0 + gc * a1;
                    }
                    gsync();
                }
            }
            --nact;
        }
    }
    iters = iter;
    // ---- verification: multipliers in [0, w] (soft) or >= 0
    int bad = 0;
    if (t < nact) {
        if (u < -1e-9 * wgt) bad = 1;
        if (gi_soft<N>(id) && u > wgt * (1.0 + 1e-9)) bad = 1;
    }
    if (edge) {
        int bit = 0;
        if (t < nact && id >= 0 && id < 6 * N && id % 6 < 2 && u > kEdgeMultTol) bit = 1 << (2 * (id / 6) + id % 6);
        *edge = (unsigned)gor(bit);
    }
    const bool ok = gor(bad) == 0;
    if (wq) {  // the final active set and factors for the next ADMM iteration
        const bool keep = ok && gor((int)sat) == 0;  // saturated soft rows: not warm-startable
        // started from this very record (same code, hinge states and key, no drop) and no add or
        // drop since: active set and factors are the record's, so only a lost `valid` is written
        const bool same = warmed == WARM_OK && iter == 0;
        if (!same) {
            if (t < N) {
                for (int c = 0; c < N; ++c) {
                    wq->J[t * RS + c] = J[t * LD + c];
                    wq->R[t * RS + c] = R[t * LD + c];
                }
                wq->ids[t] = t < nact ? id : -1;
            }
            if (t == 0) {
                wq->code = wcode;
                wq->hs = whs;
                wq->key = wkey;
                wq->nact = nact;
                wq->valid = keep ? 1 : 0;
            }
        } else if (!keep && t == 0) {
            wq->valid = 0;
        }
        if (!same || !keep) {
            // the record may be read again by this wave before the kernel ends (the next hinge
            // round, the hint leaf after the dive leaf on one slot): its stores must be complete and
            // seen by every lane first, not a mix of old and new rows
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            gsync();
        }
    }
    return ok ? GI_OK : GI_FAIL_VERIFY;
}

// ------------------------------------------------------------------ trajectory helpers
// lane t: v_t (velocity entering step t), p_{t+1}, v_{t+1} of the group's trajectory y.
template <int N>
__device__ inline void lane_state(const Lane<N>& L, double& v_prev, double& p_next, double& v_next) {
    const int t = lane16();
    const double yv = t < N ? L.y : 0.0;
    double vp = __shfl_up(yv, 1, G);
    if (t == 0) vp = L.v0;
    const double excl = gscan(yv) - yv;
    v_prev = vp;
    p_next = L.P1 + L.ts * excl;  // p_{t+1} = P1 + ts (y_0 + .. + y_{t-1})
    v_next = yv;
}

// Objective (direct, term by term) of the decentralised local problem: lane t adds the terms
// of state k = t + 1 and of input step t; lane 0 also those of x_0 (as direct_cost).
template <int N>
__device__ inline double direct_cost_decent(const Lane<N>& L, const hvp_system& S, const Consts& C, int role,
                                            const double* prm, uint64_t code, int K) {
    const int t = lane16();
    const double* xf = prm + 2;
    const double* xb = prm + 2 + 2 * (N + 1);
    const double* xl = prm + 2 + 4 * (N + 1);
    const bool tf = (role & HVP_ROLE_TRACK_FRONT) != 0, tb = (role & HVP_ROLE_TRACK_BACK) != 0;
    const bool tl = (role & HVP_ROLE_TRACK_LEADER) != 0, lsp = (role & HVP_ROLE_LEADER_SPACING) != 0;
    const bool sf = (role & HVP_ROLE_SAFE_FRONT) != 0, sb = (role & HVP_ROLE_SAFE_BACK) != 0;
    const double Qpv2 = 2.0 * C.Qpv;
    auto quad = [&](double ep, double ev) { return C.Qpp * ep * ep + Qpv2 * ep * ev + C.Qvv * ev * ev; };
    auto state_terms = [&](int k, double p, double v) {
        double J = 0.0;
        if (tf) J += quad(p + C.t0 * v + C.d0 - xf[k], v - xf[N + 1 + k]);
        if (tb) J += quad(xb[k] + C.t0 * xb[N + 1 + k] + C.d0 - p, xb[N + 1 + k] - v);
        if (tl) J += quad(p - xl[k] + (lsp ? C.t0 * v + C.d0 : 0.0), v - xl[N + 1 + k]);
        if (sf) J += C.w * fmax(0.0, p - xf[k] + C.d_safe);
        if (sb) J += C.w * fmax(0.0, xb[k] + C.d_safe - p);
        return J;
    };
    double vprev, pn, vn;
    lane_state<N>(L, vprev, pn, vn);
    double J = 0.0, u = 0.0;
    if (t < N) {
        J += state_terms(t + 1, pn, vn);
        u = (vn - L.am * vprev - L.uc) / L.ub;
        if (L.ucost) J += C.Qu * u * u;
    }
    const double uprev = __shfl_up(u, 1, G);
    if (t >= 1 && t < N && t < K) J += C.Qdu * (u - uprev) * (u - uprev);
    if (t == 0) J += state_terms(0, prm[0], prm[1]);
    return gsum(J);
}

template <int N>
__device__ inline double direct_cost_admm(const Lane<N>& L, const hvp_system& S, const Consts& C, int role,
                                          const double* prm, uint64_t code, int K) {
    const int t = lane16();
    const double* xl = admm_leader(prm, N);
    const bool hf = (role & HVP_ROLE_SAFE_FRONT) != 0, hb = (role & HVP_ROLE_SAFE_BACK) != 0;
    const bool tf = (role & HVP_ROLE_TRACK_FRONT) != 0, tb = (role & HVP_ROLE_TRACK_BACK) != 0;
    const bool tl = (role & HVP_ROLE_TRACK_LEADER) != 0;
    const int K1 = N + 1;
    auto state_terms = [&](int k, double p, double v) {
        double J = 0.0;
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
        return J;
    };
    double vprev, pn, vn;
    lane_state<N>(L, vprev, pn, vn);
    double J = 0.0, u = 0.0;
    if (t < N) {
        J += state_terms(t + 1, pn, vn);
        const int r = code_region(code, t);
        u = (vn - S.a[r] * vprev - S.c[r]) / S.b[r];
        if (t < K) J += C.Qu * u * u;
    }
    const double uprev = __shfl_up(u, 1, G);
    if (t >= 1 && t < N && t < K) J += C.Qdu * (u - uprev) * (u - uprev);
    if (t == 0) J += state_terms(0, prm[0], prm[1]);
    return gsum(J);
}

// ADMM hinge states at the group's trajectory (k = t + 1 per lane); *consistent = no change
template <int N>
__device__ inline uint64_t admm_classify_group(const Lane<N>& L, const Consts& C, int role, const double* prm,
                                               uint64_t hs, bool* consistent) {
    const int t = lane16();
    const bool hf = (role & HVP_ROLE_SAFE_FRONT) != 0, hb = (role & HVP_ROLE_SAFE_BACK) != 0;
    const bool tf = (role & HVP_ROLE_TRACK_FRONT) != 0, tb = (role & HVP_ROLE_TRACK_BACK) != 0;
    const int K1 = N + 1;
    double vprev, p, v;
    lane_state<N>(L, vprev, p, v);
    unsigned long long mine = 0;
    int changed = 0;
    if (t < N) {
        const int k = t + 1;
        for (int side = 0; side < 2; ++side) {
            if (!(side == 0 ? hf : hb)) continue;
            const double* yy = admm_y(prm, side, N);
            const double* zz = admm_z(prm, side, N);
            CopyTerm T;
            admm_copy(C, side == 0 ? tf : tb, side, yy[k], yy[K1 + k], zz[k], zz[K1 + k], T);
            const double uu = T.gp * p + T.gv * v + T.g0;
            const int old = hub_get(hs, k, side);
            int st = hub_state(uu, C.w, T.kappa);
            const double tol = 1e-10 * (1.0 + fabs(uu) + fabs(p));
            if (st != old) {
                const double lo = old == HUB_OFF ? -1e300 : (old == HUB_QUAD ? 0.0 : C.w * T.kappa);
                const double hi = old == HUB_OFF ? 0.0 : (old == HUB_QUAD ? C.w * T.kappa : 1e300);
                if (uu >= lo - tol && uu <= hi + tol) st = old;
            }
            if (st != old) changed = 1;
            mine = hub_set(mine, k, side, st);
        }
    }
    *consistent = gor(changed) == 0;
    return gor64(mine);
}

// initial hinge states: those at the constant-velocity trajectory (as solve_admm_lane)
template <int N>
__device__ inline uint64_t admm_initial_states(Lane<N>& L, const Consts& C, int role, const double* prm) {
    const double ysave = L.y;
    L.y = prm[1];
    bool c;
    const uint64_t hs = admm_classify_group<N>(L, C, role, prm, 0, &c);
    L.y = ysave;
    return hs;
}

// One fixed-sequence (relaxed beyond K) QP of either formulation, solved by the group.
// Returns GI_OK with y in L.y (lane t < N) and the direct objective in *cost.
//
// wq (ADMM forms, optional): this QP's WarmQp record.  With warm set its hinge states replace
// the constant-velocity guess as the starting states (the iterates change little from one ADMM
// iteration to the next, so the first solve is usually consistent) and its active set / factors
// start the active-set method (solve); every solve writes the record back.  The fixed point
// reached is the QP's optimum either way (the Huber pieces are convex and C1, so the states only
// decide which solve certifies it).  Should the warm-started run not settle (a solve fails, or the
// hinge states still change after kHubRounds), the QP is solved once more from the cold start
// (constant-velocity states, Cholesky of H), so a warm start never fails a QP the cold start solves.
// wkey: the record's owner key (system index, role bits; WarmQp).
template <int N, class W = WarmQp>
__device__ inline int solve_qp(Lane<N>& L, GroupLds& Sg, const hvp_system& S, const Consts& C, int role,
                               const double* prm, uint64_t code, int K, int max_iter, int& iters, double* cost,
                               unsigned* edge = nullptr, double lo = 0.0, double hi = -1.0,
                               W* wq = nullptr, bool warm = false, uint64_t wkey = 0) {
    iters = 0;
    if (C.form == HVP_FORM_ADMM || C.form == HVP_FORM_GADMM) {
        // group-uniform (one address per group).  A node record (RS < G: one table slot shared by
        // the nodes that hash to it) starts only the node it was written for; the switching ADMM's
        // per-QP record also lends its hinge states to the QP's next region sequence
        bool w = wq && warm && wq->valid && wq->key == wkey && (W::RS == G || wq->code == code);
        int st = GI_FAIL_ITER;
        for (int attempt = 0; attempt < 2; ++attempt) {
            uint64_t hs;
            if (w) {
                hs = wq->hs;
            } else {
                // the lane data the classification reads (lane_state: v0, ts, P1 as setup sets them)
                Lane<N> L0;
                L0.v0 = prm[1];
                L0.ts = S.ts;
                L0.P1 = prm[0] + S.ts * prm[1];
                hs = admm_initial_states<N>(L0, C, role, prm);
            }
            st = GI_FAIL_ITER;
            for (int round = 0; round < kHubRounds; ++round) {
                gsync();
                // the record will start this round (solve's test): no Hessian to assemble
                const bool from_rec = w && wq->code == code && wq->hs == hs && wq->key == wkey;
                setup<N>(L, Sg, S, C, role, prm, code, K, hs, 0.0, -1.0, !from_rec);
                int it = 0;
                st = solve<N, W>(L, Sg, C, max_iter, it, edge, wq, code, hs, w, wkey, from_rec);
                if (st == GI_WARM_LOST) {  // the warm start overwrote the Hessian and failed: cold
                    gsync();
                    setup<N>(L, Sg, S, C, role, prm, code, K, hs);
                    st = solve<N, W>(L, Sg, C, max_iter, it, edge, wq, code, hs, false, wkey);
                }
                iters += it;
                if (st != GI_OK) break;
                bool consistent;
                hs = admm_classify_group<N>(L, C, role, prm, hs, &consistent);
                if (consistent) {
                    *cost = direct_cost_admm<N>(L, S, C, role, prm, code, K);
                    return GI_OK;
                }
                st = GI_FAIL_ITER;
            }
            if (!w) break;  // the cold start was the last resort
            w = false;
        }
        return st;
    }
    gsync();
    setup<N>(L, Sg, S, C, role, prm, code, K, 0, lo, hi);
    const int st = solve<N>(L, Sg, C, max_iter, iters);
    if (st != GI_OK) return st;
    *cost = direct_cost_decent<N>(L, S, C, role, prm, code, K);
    return GI_OK;
}

}  // namespace coop
}  // namespace hvp
