// hvp_ipm.h -- per-lane fixed-region-sequence QP solver of the local hybrid MPC.
//
// One lane owns one (instance, region sequence sigma) pair: the local MIQP of
// LocalMpcMld (fleet_decent_mld.py:61-208 on top of MpcMld [EXT dmpcpwa]) with the binaries
// fixed to sigma is a convex QP; the MIQP optimum is the minimum of these QPs over sigma.
//
// Formulation (velocity space).  With x = (p, v) and the velocity-partitioned PWA model
//     p_{k+1} = p_k + ts v_k,     v_{k+1} = a_k v_k + b_k u_k + c_k     (a_k,b_k,c_k from sigma_k)
// the decision variables are y = (v_1 .. v_N) plus the safe-distance slacks s_f,k / s_b,k for
// k = 2..N (p_1 = p_0 + ts v_0 is fixed, so the k = 0, 1 slacks are constants).  Then
//     u_k = (v_{k+1} - a_k v_k - c_k) / b_k          (bidiagonal in y)
//     p_k = p_1 + ts * (v_1 + .. + v_{k-1})          (prefix sums of y, sigma-independent)
// and every constraint row of the MLD model with sigma fixed is one of
//     V  vlo_k <= v_k <= vhi_k          region sigma_k (k < N) intersected with the state box
//     U  c + b umin <= v_k - a v_{k-1} <= c + b umax        (F u <= G, k = 1..N)
//     A  dec <= v_k - v_{k-1} <= acc                         (accel rows, fleet_decent_mld.py:172-188)
//     P  pmin <= p_k <= pmax                                 (D x <= E position rows)
//     SF p_k - s_f <= pf_k - d_safe,  s_f >= 0               (fleet_decent_mld.py:191-199)
//     SB -p_k - s_b <= -(pb_k + d_safe), s_b >= 0            (fleet_decent_mld.py:200-208)
// so the Newton matrix is  H + diag + bidiagonal + sum of prefix outer products : assembled
// in O(N^2) (not O(m N^2)), with the slacks eliminated analytically (2x2 per row pair).
//
// Solver: Mehrotra predictor-corrector primal-dual IPM, CVXOPT-style initial point, dense
// N x N Cholesky (N <= 8, all in registers), lambda/t of every row kept in registers.
//
// This header has no HIP dependency: hvp_kernels.hip compiles it for gfx950, and the
// test-only host build (hvp_hostref.cpp) compiles it with g++ to debug the algorithm on a
// machine without a GPU.  The product library never runs it on the CPU.
#pragma once

#include <math.h>
#include <stdint.h>

#include "hvp.h"

#ifndef HVP_HD
#define HVP_HD
#endif

namespace hvp {

// Uniform (per handle) constants in the form the lanes use.
struct Consts {
    double Qpp, Qpv, Qvv;    // symmetric Qx
    double Qu, Qdu, w;
    double d_safe, d0, t0;
    double dec[HVP_MAX_N];   // accel lower bound of step k (a_dec*ts + k*tight)
    double acc[HVP_MAX_N];   // accel upper bound of step k (a_acc*ts - k*tight)
    double tol;
    int max_iter;
    int N;
};

struct QpOut {
    double cost;
    int status;  // 0 converged, 2 not converged
    int iters;
};

// packed lower-triangular index
HVP_HD constexpr int tri(int i, int j) { return i * (i + 1) / 2 + j; }

template <int N>
struct LaneQp {
    static constexpr int NP = N - 1;        // position-type rows exist for k = 2..N
    static constexpr int NT = N * (N + 1) / 2;
    static constexpr int RV = 6 * N;        // V/U/A rows: 6 per k = 1..N
    static constexpr int R = RV + 6 * NP;   // + P/SF/SB rows: 6 per k = 2..N

    // ---------------- problem data
    double v0, P1, ts;
    double am[N];             // a_{k-1} (coefficient of v_{k-1} in the U row of step k)
    double vlo[N], vhi[N];    // bounds on v_k
    double ulo[N], uhi[N];    // bounds on v_k - a v_{k-1}
    double pmin, pmax;
    double hf[NP > 0 ? NP : 1], hb[NP > 0 ? NP : 1];  // pf_k - d_safe, pb_k + d_safe (k = 2..N)
    bool has_sf, has_sb;
    double H[NT], f[N], C0;

    // ---------------- iterate
    double y[N], sf[NP > 0 ? NP : 1], sb[NP > 0 ? NP : 1];
    double lam[R], t[R];
};

// Row layout: for k = 1..N  base 6(k-1): Vlo Vhi Ulo Uhi Alo Ahi
//             for k = 2..N  base 6N + 6(k-2): Plo Phi SF SF0 SB SB0
enum { VLO = 0, VHI, ULO, UHI, ALO, AHI };
enum { PLO = 0, PHI, SFR, SF0, SBR, SB0 };

template <int N>
HVP_HD inline bool row_active(const LaneQp<N>& q, int i) {
    if (i < LaneQp<N>::RV) return true;
    int r = (i - LaneQp<N>::RV) % 6;
    if (r == SFR || r == SF0) return q.has_sf;
    if (r == SBR || r == SB0) return q.has_sb;
    return true;
}

// Affine row values G z (+ constants when with_const) for z = (y, sf, sb).
// Calls emit(i, value) for every row.  v_prev of step 1 is the constant v0 (0 for directions),
// p_k = P1 + ts * cum (P1 -> 0 for directions).
template <int N, class F>
HVP_HD inline void for_rows(const LaneQp<N>& q, const double* y, const double* sf, const double* sb, bool with_const,
                            F&& emit) {
    double vprev = with_const ? q.v0 : 0.0;
    double cum = 0.0;
    const double p1 = with_const ? q.P1 : 0.0;
#pragma unroll
    for (int k = 1; k <= N; ++k) {
        const double vk = y[k - 1];
        const int b = 6 * (k - 1);
        const double du = vk - q.am[k - 1] * vprev;
        const double da = vk - vprev;
        emit(b + VLO, -vk);
        emit(b + VHI, vk);
        emit(b + ULO, -du);
        emit(b + UHI, du);
        emit(b + ALO, -da);
        emit(b + AHI, da);
        if (k >= 2) {
            cum += y[k - 2];
            const double pk = p1 + q.ts * cum;
            const int c = LaneQp<N>::RV + 6 * (k - 2);
            emit(c + PLO, -pk);
            emit(c + PHI, pk);
            emit(c + SFR, pk - sf[k - 2]);
            emit(c + SF0, -sf[k - 2]);
            emit(c + SBR, -pk - sb[k - 2]);
            emit(c + SB0, -sb[k - 2]);
        }
        vprev = vk;
    }
}

template <int N>
HVP_HD inline double row_h(const LaneQp<N>& q, const Consts& C, int i) {
    if (i < LaneQp<N>::RV) {
        const int k = i / 6, r = i % 6;  // step k+1
        switch (r) {
            case VLO: return -q.vlo[k];
            case VHI: return q.vhi[k];
            case ULO: return -q.ulo[k];
            case UHI: return q.uhi[k];
            case ALO: return -C.dec[k];
            default: return C.acc[k];
        }
    }
    const int k = (i - LaneQp<N>::RV) / 6, r = (i - LaneQp<N>::RV) % 6;  // step k+2
    switch (r) {
        case PLO: return -q.pmin;
        case PHI: return q.pmax;
        case SFR: return q.hf[k];
        case SBR: return -q.hb[k];
        default: return 0.0;
    }
}

// Newton direction of the reduced (y-space) system.
//   d[i]   : row scaling lambda_i / t_i
//   rt[i]  : r~_i = r_p,i - r_c,i / lambda_i
//   rd[N]  : dual residual of y, rsf/rsb: dual residuals of the slacks
// Outputs dy, dsf, dsb.  K is factorised here (Cholesky, packed).
template <int N>
HVP_HD inline bool reduced_solve(const LaneQp<N>& q, const double* d, const double* rt, const double* rd,
                                 const double* rsf, const double* rsb, double* dy, double* dsf, double* dsb) {
    constexpr int NT = LaneQp<N>::NT;
    constexpr int RV = LaneQp<N>::RV;
    double K[NT];
    double rhs[N];
#pragma unroll
    for (int i = 0; i < NT; ++i) K[i] = q.H[i];
#pragma unroll
    for (int j = 0; j < N; ++j) rhs[j] = -rd[j];
    // V / U / A rows of step k (variable j = k-1)
#pragma unroll
    for (int j = 0; j < N; ++j) {
        const int b = 6 * j;
        const double DV = d[b + VLO] + d[b + VHI];
        const double rV = -d[b + VLO] * rt[b + VLO] + d[b + VHI] * rt[b + VHI];
        const double DU = d[b + ULO] + d[b + UHI];
        const double rU = -d[b + ULO] * rt[b + ULO] + d[b + UHI] * rt[b + UHI];
        const double DA = d[b + ALO] + d[b + AHI];
        const double rA = -d[b + ALO] * rt[b + ALO] + d[b + AHI] * rt[b + AHI];
        K[tri(j, j)] += DV + DU + DA;
        rhs[j] -= rV + rU + rA;
        if (j >= 1) {
            const double a = q.am[j];
            K[tri(j - 1, j - 1)] += DU * a * a + DA;
            K[tri(j, j - 1)] -= DU * a + DA;
            rhs[j - 1] += a * rU + rA;
        }
    }
    // position-type rows of step k = j+2 act on y[0..j] through ts * prefix
    if (N >= 2) {
        double beta[N > 1 ? N - 1 : 1], rho[N > 1 ? N - 1 : 1];
#pragma unroll
        for (int j = 0; j < N - 1; ++j) {
            const int c = RV + 6 * j;
            double B = d[c + PLO] + d[c + PHI];
            double r = -d[c + PLO] * rt[c + PLO] + d[c + PHI] * rt[c + PHI];
            if (q.has_sf) {
                const double d1 = d[c + SFR], d2 = d[c + SF0], inv = 1.0 / (d1 + d2);
                B += d1 * d2 * inv;
                r += (d1 * d2 * (rt[c + SFR] - rt[c + SF0]) + d1 * rsf[j]) * inv;
            }
            if (q.has_sb) {
                const double d1 = d[c + SBR], d2 = d[c + SB0], inv = 1.0 / (d1 + d2);
                B += d1 * d2 * inv;
                r -= (d1 * d2 * (rt[c + SBR] - rt[c + SB0]) + d1 * rsb[j]) * inv;
            }
            beta[j] = B * q.ts * q.ts;
            rho[j] = r * q.ts;
        }
        // suffix sums: entry (i1, i2) receives beta of every step whose prefix covers max(i1, i2)
        double sb_ = 0.0, sr = 0.0;
#pragma unroll
        for (int m = N - 2; m >= 0; --m) {
            sb_ += beta[m];
            sr += rho[m];
            rhs[m] -= sr;
#pragma unroll
            for (int i2 = 0; i2 <= m; ++i2) K[tri(m, i2)] += sb_;
        }
    }
    // Cholesky K = L L^T (in place, packed)
#pragma unroll
    for (int j = 0; j < N; ++j) {
        double s = K[tri(j, j)];
#pragma unroll
        for (int k = 0; k < j; ++k) s -= K[tri(j, k)] * K[tri(j, k)];
        if (!(s > 0.0)) return false;
        const double l = sqrt(s), il = 1.0 / l;
        K[tri(j, j)] = l;
#pragma unroll
        for (int i = j + 1; i < N; ++i) {
            double v = K[tri(i, j)];
#pragma unroll
            for (int k = 0; k < j; ++k) v -= K[tri(i, k)] * K[tri(j, k)];
            K[tri(i, j)] = v * il;
        }
    }
#pragma unroll
    for (int i = 0; i < N; ++i) {
        double v = rhs[i];
#pragma unroll
        for (int k = 0; k < i; ++k) v -= K[tri(i, k)] * dy[k];
        dy[i] = v / K[tri(i, i)];
    }
#pragma unroll
    for (int i = N - 1; i >= 0; --i) {
        double v = dy[i];
#pragma unroll
        for (int k = i + 1; k < N; ++k) v -= K[tri(k, i)] * dy[k];
        dy[i] = v / K[tri(i, i)];
    }
    // slack directions (eliminated 2x2 blocks)
    double cum = 0.0;
#pragma unroll
    for (int j = 0; j < N - 1; ++j) {
        cum += dy[j];
        const int c = RV + 6 * j;
        const double gdy = q.ts * cum;
        if (q.has_sf) {
            const double d1 = d[c + SFR], d2 = d[c + SF0];
            dsf[j] = (d1 * gdy + d1 * rt[c + SFR] + d2 * rt[c + SF0] - rsf[j]) / (d1 + d2);
        } else {
            dsf[j] = 0.0;
        }
        if (q.has_sb) {
            const double d1 = d[c + SBR], d2 = d[c + SB0];
            dsb[j] = (-d1 * gdy + d1 * rt[c + SBR] + d2 * rt[c + SB0] - rsb[j]) / (d1 + d2);
        } else {
            dsb[j] = 0.0;
        }
    }
    return true;
}

// Dual residuals r_d = H y + f + G_y' lam and r_s = w - lam_row - lam_nonneg.
template <int N>
HVP_HD inline void dual_residual(const LaneQp<N>& q, const Consts& C, const double* y, const double* lam, double* rd,
                                 double* rsf, double* rsb) {
    constexpr int RV = LaneQp<N>::RV;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        double s = q.f[i];
#pragma unroll
        for (int j = 0; j < N; ++j) s += q.H[i >= j ? tri(i, j) : tri(j, i)] * y[j];
        rd[i] = s;
    }
#pragma unroll
    for (int j = 0; j < N; ++j) {
        const int b = 6 * j;
        const double lU = lam[b + UHI] - lam[b + ULO];
        rd[j] += lam[b + VHI] - lam[b + VLO] + lU + lam[b + AHI] - lam[b + ALO];
        if (j >= 1) rd[j - 1] -= q.am[j] * lU + (lam[b + AHI] - lam[b + ALO]);
    }
    double s = 0.0;
#pragma unroll
    for (int m = N - 2; m >= 0; --m) {
        const int c = RV + 6 * m;
        double g = lam[c + PHI] - lam[c + PLO];
        if (q.has_sf) g += lam[c + SFR];
        if (q.has_sb) g -= lam[c + SBR];
        s += g;
        rd[m] += q.ts * s;
        rsf[m] = q.has_sf ? C.w - lam[c + SFR] - lam[c + SF0] : 0.0;
        rsb[m] = q.has_sb ? C.w - lam[c + SBR] - lam[c + SB0] : 0.0;
    }
}

template <int N>
HVP_HD inline double objective(const LaneQp<N>& q, const Consts& C, const double* y) {
    double J = q.C0;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        double hy = 0.0;
#pragma unroll
        for (int j = 0; j < N; ++j) hy += q.H[i >= j ? tri(i, j) : tri(j, i)] * y[j];
        J += (0.5 * hy + q.f[i]) * y[i];
    }
    // exact penalty of the safe rows at y (= w * optimal slack)
    double cum = 0.0;
#pragma unroll
    for (int j = 0; j < N - 1; ++j) {
        cum += y[j];
        const double pk = q.P1 + q.ts * cum;
        if (q.has_sf) J += C.w * fmax(0.0, pk - q.hf[j]);
        if (q.has_sb) J += C.w * fmax(0.0, q.hb[j] - pk);
    }
    return J;
}

template <int N>
HVP_HD inline double max_step(const double* v, const double* dv, const LaneQp<N>& q) {
    double a = 1.0;
#pragma unroll
    for (int i = 0; i < LaneQp<N>::R; ++i)
        if (row_active(q, i) && dv[i] < 0.0) a = fmin(a, -v[i] / dv[i]);
    return a;
}

// Mehrotra predictor-corrector.  Returns objective (exact penalty form) and status.
template <int N>
HVP_HD inline QpOut solve_lane(LaneQp<N>& q, const Consts& C) {
    constexpr int R = LaneQp<N>::R;
    constexpr int NP1 = N > 1 ? N - 1 : 1;
    double h[R];
    int m = 0;
#pragma unroll
    for (int i = 0; i < R; ++i) {
        h[i] = row_h(q, C, i);
        m += row_active(q, i) ? 1 : 0;
    }
    double val[R], rp[R], d[R], rt[R], dl[R], dt[R];
    double rd[N], rsf[NP1], rsb[NP1], dy[N], dsf[NP1], dsb[NP1];
    QpOut out{0.0, 2, 0};

    // ---- initial point: one reduced solve with unit scaling from (y, s, t, lam) = 0
    {
        const double zero[N > 0 ? N : 1] = {};
        const double zs[NP1] = {};
        for_rows(q, zero, zs, zs, true, [&](int i, double v) { val[i] = v; });
#pragma unroll
        for (int i = 0; i < R; ++i) {
            d[i] = row_active(q, i) ? 1.0 : 0.0;
            rt[i] = val[i] - h[i];
        }
#pragma unroll
        for (int i = 0; i < N; ++i) rd[i] = q.f[i];
#pragma unroll
        for (int j = 0; j < NP1; ++j) { rsf[j] = q.has_sf ? C.w : 0.0; rsb[j] = q.has_sb ? C.w : 0.0; }
        // masked rows: d = 0 would make the slack blocks singular; give them unit weight there
        if (!q.has_sf)
#pragma unroll
            for (int j = 0; j < N - 1; ++j) { d[LaneQp<N>::RV + 6 * j + SFR] = 1.0; d[LaneQp<N>::RV + 6 * j + SF0] = 1.0; }
        if (!q.has_sb)
#pragma unroll
            for (int j = 0; j < N - 1; ++j) { d[LaneQp<N>::RV + 6 * j + SBR] = 1.0; d[LaneQp<N>::RV + 6 * j + SB0] = 1.0; }
        if (!reduced_solve(q, d, rt, rd, rsf, rsb, q.y, q.sf, q.sb)) return out;
        for_rows(q, q.y, q.sf, q.sb, true, [&](int i, double v) { val[i] = v; });
        double tmin = 1e300, lmin = 1e300;
#pragma unroll
        for (int i = 0; i < R; ++i) {
            q.t[i] = h[i] - val[i];
            q.lam[i] = -q.t[i];
            if (row_active(q, i)) { tmin = fmin(tmin, q.t[i]); lmin = fmin(lmin, q.lam[i]); }
        }
        const double st = fmax(-1.5 * tmin, 0.0), sl = fmax(-1.5 * lmin, 0.0);
        double tl = 0.0, ssum = 0.0, lsum = 0.0;
#pragma unroll
        for (int i = 0; i < R; ++i) {
            q.t[i] += st;
            q.lam[i] += sl;
            if (row_active(q, i)) { tl += q.t[i] * q.lam[i]; ssum += q.t[i]; lsum += q.lam[i]; }
        }
        const double dt0 = lsum > 0 ? 0.5 * tl / lsum : 1.0, dl0 = ssum > 0 ? 0.5 * tl / ssum : 1.0;
#pragma unroll
        for (int i = 0; i < R; ++i) {
            q.t[i] += dt0;
            q.lam[i] += dl0;
            if (!(q.t[i] > 0.0)) q.t[i] = 1.0;
            if (!(q.lam[i] > 0.0)) q.lam[i] = 1.0;
            if (!row_active(q, i)) { q.t[i] = 1.0; q.lam[i] = 0.0; }
        }
    }

    double sq = fmax(1.0, C.w);
#pragma unroll
    for (int i = 0; i < N; ++i) sq = fmax(sq, fabs(q.f[i]));
    double sh = 1.0;
#pragma unroll
    for (int i = 0; i < R; ++i)
        if (row_active(q, i)) sh = fmax(sh, fabs(h[i]));

    const int maxit = C.max_iter;
    for (int it = 0; it <= maxit; ++it) {
        // ---- residuals
        for_rows(q, q.y, q.sf, q.sb, true, [&](int i, double v) { val[i] = v; });
        double gap = 0.0, rpmax = 0.0;
#pragma unroll
        for (int i = 0; i < R; ++i) {
            rp[i] = val[i] + q.t[i] - h[i];
            if (row_active(q, i)) {
                gap += q.lam[i] * q.t[i];
                rpmax = fmax(rpmax, fabs(rp[i]));
            }
        }
        dual_residual(q, C, q.y, q.lam, rd, rsf, rsb);
        double rdmax = 0.0;
#pragma unroll
        for (int i = 0; i < N; ++i) rdmax = fmax(rdmax, fabs(rd[i]));
#pragma unroll
        for (int j = 0; j < N - 1; ++j) rdmax = fmax(rdmax, fmax(fabs(rsf[j]), fabs(rsb[j])));
        const double J = objective(q, C, q.y);
        out.iters = it;
        if (rdmax <= C.tol * sq && rpmax <= C.tol * sh && gap <= 0.1 * C.tol * fmax(1.0, fabs(J))) {
            out.status = 0;
            out.cost = J;
            return out;
        }
        if (it == maxit) break;
        const double mu = gap / m;
#pragma unroll
        for (int i = 0; i < R; ++i) {
            if (row_active(q, i)) {
                d[i] = q.lam[i] / q.t[i];
                rt[i] = rp[i] - q.t[i];  // predictor: r_c = lam * t
            } else {
                d[i] = 1.0;
                rt[i] = 0.0;
            }
        }
        // ---- predictor
        double dya[N], dsfa[NP1], dsba[NP1];
        if (!reduced_solve(q, d, rt, rd, rsf, rsb, dya, dsfa, dsba)) break;
        for_rows(q, dya, dsfa, dsba, false, [&](int i, double v) { val[i] = v; });
#pragma unroll
        for (int i = 0; i < R; ++i) {
            dl[i] = d[i] * (val[i] + rt[i]);
            dt[i] = -rp[i] - val[i];
        }
        const double aa = fmin(max_step(q.t, dt, q), max_step(q.lam, dl, q));
        double mua = 0.0;
#pragma unroll
        for (int i = 0; i < R; ++i)
            if (row_active(q, i)) mua += (q.lam[i] + aa * dl[i]) * (q.t[i] + aa * dt[i]);
        mua /= m;
        const double sr = mua / mu;
        const double sig = sr * sr * sr;
        // ---- corrector: r_c = lam t + dlam_a dt_a - sig mu
#pragma unroll
        for (int i = 0; i < R; ++i)
            if (row_active(q, i)) rt[i] = rp[i] - q.t[i] - (dl[i] * dt[i] - sig * mu) / q.lam[i];
        if (!reduced_solve(q, d, rt, rd, rsf, rsb, dy, dsf, dsb)) break;
        for_rows(q, dy, dsf, dsb, false, [&](int i, double v) { val[i] = v; });
#pragma unroll
        for (int i = 0; i < R; ++i) {
            dl[i] = d[i] * (val[i] + rt[i]);
            dt[i] = -rp[i] - val[i];
        }
        const double amax = fmin(max_step(q.t, dt, q), max_step(q.lam, dl, q));
        const double alpha = fmin(1.0, 0.99 * amax);
#pragma unroll
        for (int i = 0; i < N; ++i) q.y[i] += alpha * dy[i];
#pragma unroll
        for (int j = 0; j < N - 1; ++j) {
            q.sf[j] += alpha * dsf[j];
            q.sb[j] += alpha * dsb[j];
        }
#pragma unroll
        for (int i = 0; i < R; ++i)
            if (row_active(q, i)) {
                q.lam[i] += alpha * dl[i];
                q.t[i] += alpha * dt[i];
            }
    }
    out.status = 2;
    out.cost = objective(q, C, q.y);
    return out;
}

// ------------------------------------------------------------------ problem setup
// Builds the lane QP for instance params (x0, x_front, x_back, leader_x) and region code.
// Returns false when a sigma-independent constant row (p_1 box) is violated.
template <int N>
HVP_HD inline bool setup_lane(LaneQp<N>& q, const hvp_system& S, const Consts& C, int role, const double* prm,
                              uint32_t code) {
    const double p0 = prm[0], v0 = prm[1];
    const double* xf = prm + 2;
    const double* xb = prm + 2 + 2 * (N + 1);
    const double* xl = prm + 2 + 4 * (N + 1);
    const double ts = S.ts;
    q.v0 = v0;
    q.ts = ts;
    q.P1 = p0 + ts * v0;
    q.pmin = S.pmin;
    q.pmax = S.pmax;
    q.has_sf = (role & HVP_ROLE_SAFE_FRONT) != 0;
    q.has_sb = (role & HVP_ROLE_SAFE_BACK) != 0;
    double a[N], b[N], c[N];
#pragma unroll
    for (int k = 0; k < N; ++k) {
        const int r = (code >> (3 * k)) & 7;
        a[k] = S.a[r];
        b[k] = S.b[r];
        c[k] = S.c[r];
        q.am[k] = a[k];
        q.ulo[k] = c[k] + b[k] * S.umin;
        q.uhi[k] = c[k] + b[k] * S.umax;
        // bounds on v_{k+1}: region sigma_{k+1} (if any) intersected with the state box
        if (k + 1 < N) {
            const int r1 = (code >> (3 * (k + 1))) & 7;
            q.vlo[k] = fmax(S.vmin, S.vlo[r1]);
            q.vhi[k] = fmin(S.vmax, S.vhi[r1]);
        } else {
            q.vlo[k] = S.vmin;
            q.vhi[k] = S.vmax;
        }
    }
    // step-1 rows carry the constant v0 on the left: U: v1 - a0 v0, A: v1 - v0 (handled in for_rows)
#pragma unroll
    for (int j = 0; j < N - 1; ++j) {
        q.hf[j] = xf[j + 2] - C.d_safe;
        q.hb[j] = xb[j + 2] + C.d_safe;
    }

    // ---- cost: 1/2 y'Hy + f'y + C0
#pragma unroll
    for (int i = 0; i < LaneQp<N>::NT; ++i) q.H[i] = 0.0;
#pragma unroll
    for (int i = 0; i < N; ++i) q.f[i] = 0.0;
    double C0 = 0.0;
    // quadratic form  x'Wx + 2 l'x + c0  of the tracking terms at step k, x = (p, v)
    const bool tf = (role & HVP_ROLE_TRACK_FRONT) != 0, tb = (role & HVP_ROLE_TRACK_BACK) != 0;
    const bool tl = (role & HVP_ROLE_TRACK_LEADER) != 0, lsp = (role & HVP_ROLE_LEADER_SPACING) != 0;
    const double Qpp = C.Qpp, Qpv = C.Qpv, Qvv = C.Qvv, t0 = C.t0, d0 = C.d0;
#pragma unroll
    for (int k = 0; k <= N; ++k) {
        double Wpp = 0, Wpv = 0, Wvv = 0, lp = 0, lv = 0, cc = 0;
        // e = M x + r ; adds M'QM, M'Q r, r'Q r
        auto add = [&](double m00, double m01, double m11, double r0, double r1) {
            // M = [[m00, m01], [0, m11]]
            const double qa = Qpp * m00, qb = Qpv * m00;               // (QM)[0][0], (QM)[1][0]
            const double qc = Qpp * m01 + Qpv * m11, qd = Qpv * m01 + Qvv * m11;  // (QM)[0][1], (QM)[1][1]
            Wpp += m00 * qa;
            Wpv += m00 * qc;
            Wvv += m01 * qc + m11 * qd;
            const double Qr0 = Qpp * r0 + Qpv * r1, Qr1 = Qpv * r0 + Qvv * r1;
            lp += m00 * Qr0;
            lv += m01 * Qr0 + m11 * Qr1;
            cc += r0 * Qr0 + r1 * Qr1;
            (void)qb;
        };
        const int K1 = N + 1;
        if (tf) add(1.0, t0, 1.0, d0 - xf[k], -xf[K1 + k]);
        if (tb) add(-1.0, 0.0, -1.0, xb[k] + t0 * xb[K1 + k] + d0, xb[K1 + k]);
        if (tl) {
            if (lsp) add(1.0, t0, 1.0, d0 - xl[k], -xl[K1 + k]);
            else add(1.0, 0.0, 1.0, -xl[k], -xl[K1 + k]);
        }
        // x_k = xbar + Gamma y : p = pbar + ts*prefix(0..k-2), v = vbar + e_{k-1}
        const double pbar = k == 0 ? p0 : q.P1;
        const double vbar = k == 0 ? v0 : 0.0;
        // gradient of the quadratic form at xbar
        const double gp = 2.0 * (Wpp * pbar + Wpv * vbar + lp);
        const double gv = 2.0 * (Wpv * pbar + Wvv * vbar + lv);
        C0 += Wpp * pbar * pbar + 2.0 * Wpv * pbar * vbar + Wvv * vbar * vbar + 2.0 * (lp * pbar + lv * vbar) + cc;
        if (k >= 1) {
            const int jv = k - 1;  // v_k = y[jv]
            q.H[tri(jv, jv)] += 2.0 * Wvv;
            q.f[jv] += gv;
            // prefix part (indices 0..k-2) with weight ts
#pragma unroll
            for (int i = 0; i < N; ++i) {
                if (i > k - 2) break;
                q.f[i] += ts * gp;
#pragma unroll
                for (int i2 = 0; i2 <= i; ++i2) q.H[tri(i, i2)] += 2.0 * Wpp * ts * ts;
                // cross p-v: 2 * Wpv * (ts e_i)(e_jv)' symmetric ; jv > i always
                q.H[tri(jv, i)] += 2.0 * Wpv * ts;
            }
        }
    }
    // control effort  Qu u_k^2 and variation Qdu (u_{k+1} - u_k)^2, u_k = ubar_k + gu_k . y
    // gu_k has entries at k (1/b_k) and k-1 (-a_k/b_k)
    double ubar[N], gk[N], gkm[N];
#pragma unroll
    for (int k = 0; k < N; ++k) {
        const double ib = 1.0 / b[k];
        ubar[k] = k == 0 ? -(a[0] * v0 + c[0]) * ib : -c[k] * ib;
        gk[k] = ib;
        gkm[k] = k == 0 ? 0.0 : -a[k] * ib;
        const double w2 = 2.0 * C.Qu;
        q.H[tri(k, k)] += w2 * gk[k] * gk[k];
        q.f[k] += w2 * ubar[k] * gk[k];
        if (k >= 1) {
            q.H[tri(k - 1, k - 1)] += w2 * gkm[k] * gkm[k];
            q.H[tri(k, k - 1)] += w2 * gk[k] * gkm[k];
            q.f[k - 1] += w2 * ubar[k] * gkm[k];
        }
        C0 += C.Qu * ubar[k] * ubar[k];
    }
    if (C.Qdu != 0.0) {
#pragma unroll
        for (int k = 0; k + 1 < N; ++k) {
            // e = u_{k+1} - u_k : entries  k+1: gk[k+1]; k: gkm[k+1] - gk[k]; k-1: -gkm[k]
            double g[N];
#pragma unroll
            for (int i = 0; i < N; ++i) g[i] = 0.0;
            g[k + 1] += gk[k + 1];
            g[k] += gkm[k + 1] - gk[k];
            if (k >= 1) g[k - 1] -= gkm[k];
            const double eb = ubar[k + 1] - ubar[k];
            const double w2 = 2.0 * C.Qdu;
#pragma unroll
            for (int i = 0; i < N; ++i) {
                q.f[i] += w2 * eb * g[i];
#pragma unroll
                for (int i2 = 0; i2 <= i; ++i2) q.H[tri(i, i2)] += w2 * g[i] * g[i2];
            }
            C0 += C.Qdu * eb * eb;
        }
    }
    // constant slacks of k = 0, 1 (p_0, p_1 fixed)
    if (q.has_sf) C0 += C.w * (fmax(0.0, p0 - xf[0] + C.d_safe) + fmax(0.0, q.P1 - xf[1] + C.d_safe));
    if (q.has_sb) C0 += C.w * (fmax(0.0, xb[0] + C.d_safe - p0) + fmax(0.0, xb[1] + C.d_safe - q.P1));
    q.C0 = C0;
    return q.P1 >= S.pmin - 1e-9 * (1.0 + fabs(S.pmin)) && q.P1 <= S.pmax + 1e-9 * (1.0 + fabs(S.pmax));
}

// Objective of the lane's solution evaluated term by term on the trajectory, as the reference
// writes it (fleet_decent_mld.py:107-169): squared tracking errors, Q_u u^2, Q_du du^2 and
// w * max(0, .) slacks.  Avoids the cancellation of C0 + 1/2 y'Hy + f'y (positions ~3e3), so
// the costs the argmin compares carry relative error ~1e-15 instead of ~1e-9.
template <int N>
HVP_HD inline double direct_cost(const LaneQp<N>& q, const hvp_system& S, const Consts& C, int role,
                                 const double* prm, uint32_t code) {
    const double* xf = prm + 2;
    const double* xb = prm + 2 + 2 * (N + 1);
    const double* xl = prm + 2 + 4 * (N + 1);
    const bool tf = (role & HVP_ROLE_TRACK_FRONT) != 0, tb = (role & HVP_ROLE_TRACK_BACK) != 0;
    const bool tl = (role & HVP_ROLE_TRACK_LEADER) != 0, lsp = (role & HVP_ROLE_LEADER_SPACING) != 0;
    const double Qpv2 = 2.0 * C.Qpv;
    double J = 0.0, p = prm[0], v = prm[1], uprev = 0.0;
#pragma unroll
    for (int k = 0; k <= N; ++k) {
        auto quad = [&](double ep, double ev) { return C.Qpp * ep * ep + Qpv2 * ep * ev + C.Qvv * ev * ev; };
        if (tf) J += quad(p + C.t0 * v + C.d0 - xf[k], v - xf[N + 1 + k]);
        if (tb) J += quad(xb[k] + C.t0 * xb[N + 1 + k] + C.d0 - p, xb[N + 1 + k] - v);
        if (tl) J += quad(p - xl[k] + (lsp ? C.t0 * v + C.d0 : 0.0), v - xl[N + 1 + k]);
        if (q.has_sf) J += C.w * fmax(0.0, p - xf[k] + C.d_safe);
        if (q.has_sb) J += C.w * fmax(0.0, xb[k] + C.d_safe - p);
        if (k < N) {
            const int r = (code >> (3 * k)) & 7;
            const double vn = q.y[k];
            const double u = (vn - S.a[r] * v - S.c[r]) / S.b[r];
            J += C.Qu * u * u;
            if (k >= 1) J += C.Qdu * (u - uprev) * (u - uprev);
            uprev = u;
            p = p + S.ts * v;
            v = vn;
        }
    }
    return J;
}

// ------------------------------------------------------------------ sigma enumeration
// Velocity reachability of one step: v in [lo, hi] (already inside region sigma_k), inputs
// u in [umin, umax], accel v' - v in [dec, acc], state box v' in [vmin, vmax].  The set of
// reachable v' is [L(lo'), U(hi')] where [lo', hi'] = {v in [lo,hi] : L(v) <= U(v)},
// L(v) = max(a v + c + b umin, v + dec), U(v) = min(a v + c + b umax, v + acc)
// (both nondecreasing, L - U convex -> the feasible v form an interval).
HVP_HD inline bool reach_step(double lo, double hi, double a, double b, double c, double umin, double umax,
                              double dec, double acc, double vmin, double vmax, double* nlo, double* nhi) {
    const double cl = c + b * umin, cu = c + b * umax;
    // (a - 1) v <= acc - cl   and   (1 - a) v <= cu - dec
    const double oma = 1.0 - a;
    if (oma > 0.0) {
        lo = fmax(lo, -(acc - cl) / oma);
        hi = fmin(hi, (cu - dec) / oma);
    } else if (oma < 0.0) {
        hi = fmin(hi, (acc - cl) / (-oma));
        lo = fmax(lo, (cu - dec) / oma);
    } else if (acc - cl < 0.0 || cu - dec < 0.0) {
        return false;
    }
    if (cu < cl || acc < dec) return false;
    const double tol = 1e-9 * (1.0 + fabs(hi));
    if (lo > hi + tol) return false;
    if (lo > hi) lo = hi = 0.5 * (lo + hi);
    double L = fmax(a * lo + cl, lo + dec);
    double U = fmin(a * hi + cu, hi + acc);
    L = fmax(L, vmin);
    U = fmin(U, vmax);
    if (L > U + 1e-9 * (1.0 + fabs(U))) return false;
    if (L > U) L = U = 0.5 * (L + U);
    *nlo = L;
    *nhi = U;
    return true;
}

// Depth-first enumeration of every feasible region sequence in lexicographic order.
// visit(code) is called for each; returns the count.  Iterative (explicit stack).
template <class F>
HVP_HD inline int enumerate_sequences(const hvp_system& S, const Consts& C, double v0, F&& visit) {
    const int N = C.N;
    int reg[HVP_MAX_N];
    double lo[HVP_MAX_N + 1], hi[HVP_MAX_N + 1];
    lo[0] = v0;
    hi[0] = v0;
    int k = 0;
    reg[0] = -1;
    int count = 0;
    uint32_t code = 0;
    while (k >= 0) {
        int r = reg[k] + 1;
        bool advanced = false;
        for (; r < S.n_regions; ++r) {
            const double tol = 1e-9 * (1.0 + fabs(fmin(hi[k], S.vhi[r])));
            double ilo = fmax(lo[k], S.vlo[r]), ihi = fmin(hi[k], S.vhi[r]);
            if (ilo > ihi + tol) continue;
            if (ilo > ihi) ilo = ihi = 0.5 * (ilo + ihi);
            double nlo, nhi;
            if (!reach_step(ilo, ihi, S.a[r], S.b[r], S.c[r], S.umin, S.umax, C.dec[k], C.acc[k], S.vmin, S.vmax,
                            &nlo, &nhi))
                continue;
            reg[k] = r;
            code = (code & ~(7u << (3 * k))) | ((uint32_t)r << (3 * k));
            lo[k + 1] = nlo;
            hi[k + 1] = nhi;
            advanced = true;
            break;
        }
        if (!advanced) {
            --k;
            continue;
        }
        if (k + 1 == N) {
            visit(code, count);
            ++count;
            // stay at this depth, try the next region
        } else {
            ++k;
            reg[k] = -1;
        }
    }
    return count;
}

}  // namespace hvp
