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
// The solvers are inlined into every kernel that calls them.  Left to the compiler, a solver called
// from several kernels of one unit becomes a real function (Solver<10>::solve, 204 KB, from the
// three interior-point fallback kernels of N = 10), and that build's k_bnb_ipm<10> did not return
// on MI355X (r04e/r04g: the same source inlined, commit 8abfabc, finishes the solve in 8 ms).
#ifndef HVP_FORCEINLINE
#define HVP_FORCEINLINE __attribute__((always_inline))
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
    int form;      // HVP_FORM_*
    int stride;    // parameter block stride (doubles)
    double rho;    // ADMM penalty
    int l1;        // 1: min_1_norm cost (hvp_l1.h), 0: min_2_norm
    int leaf_cap;  // > 0: active-set cap of the long-horizon leaf QPs (HVP_LEAF_GI_CAP, tests of
                   // the interior-point leaf fallback); 0: the solver's own cap
    int cent_cut;  // 1: the centralised search stops a QP once its dual bound passes the incumbent
                   // (hvp_cent.h solve; HVP_CENT_CUT=0 turns it off)
};

struct QpOut {
    double cost;
    int status;  // 0 converged, 2 not converged
    int iters;
};

// packed lower-triangular index
HVP_HD constexpr int tri(int i, int j) { return i * (i + 1) / 2 + j; }

// Region sequence codes: 4 bits per step (HVP_MAX_REGIONS = 16 modes), step k at bits 4k.
constexpr int kCodeBits = 4;
constexpr uint32_t kCodeMask = (1u << kCodeBits) - 1u;
HVP_HD constexpr int code_region(uint64_t code, int k) { return (int)((code >> (kCodeBits * k)) & kCodeMask); }
HVP_HD constexpr uint64_t code_with(uint64_t code, int k, int r) {
    return (code & ~((uint64_t)kCodeMask << (kCodeBits * k))) | ((uint64_t)r << (kCodeBits * k));
}

// Refined hardware reciprocal: v_rcp_f64 estimate + two Newton steps (full double accuracy
// in 1 + 4 FMA instead of the ~12-instruction IEEE division sequence).
HVP_HD inline double frcp(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
    double r = __builtin_amdgcn_rcp(x);
    r = fma(r, fma(-x, r, 1.0), r);
    r = fma(r, fma(-x, r, 1.0), r);
    return r;
#else
    return 1.0 / x;
#endif
}

// Per-lane constant row data (sigma- and instance-dependent bounds).  The host build keeps it
// in the lane's own array; the gfx950 kernel keeps it in LDS (LdsMem in hvp_kernels.hip) so the
// register file holds only the IPM iterate.
enum { F_AM = 0, F_VLO, F_VHI, F_ULO, F_UHI, F_HF, F_HB, F_COUNT };

template <int N>
struct ArrayMem {
    double v[F_COUNT * N];
    HVP_HD double get(int f, int j) const { return v[f * N + j]; }
    HVP_HD void set(int f, int j, double x) { v[f * N + j] = x; }
    HVP_HD void refresh() {}
};

template <int N, class M = ArrayMem<N>>
struct LaneQp {
    static constexpr int NP = N - 1;              // position-type groups exist for k = 2..N
    static constexpr int NPX = N > 1 ? N - 1 : 1;
    static constexpr int NT = N * (N + 1) / 2;
    static constexpr int NPAIR = 3 * N + NP;      // two-sided rows: V,U,A (k = 1..N), P (k = 2..N)

    // ---------------- problem data
    double v0, P1, ts;
    double pmin, pmax;
    bool has_sf, has_sb;
    double H[NT], f[N], C0;
    M mem;                    // a_{k-1}, bounds of v_k, of v_k - a v_{k-1}, pf_k - d_safe, pb_k + d_safe
    HVP_HD double am(int j) const { return mem.get(F_AM, j); }
    HVP_HD double vlo(int j) const { return mem.get(F_VLO, j); }
    HVP_HD double vhi(int j) const { return mem.get(F_VHI, j); }
    HVP_HD double ulo(int j) const { return mem.get(F_ULO, j); }
    HVP_HD double uhi(int j) const { return mem.get(F_UHI, j); }
    HVP_HD double hf(int j) const { return mem.get(F_HF, j); }
    HVP_HD double hb(int j) const { return mem.get(F_HB, j); }

    // ---------------- iterate: slack t and multiplier l of both sides of every two-sided row;
    // for a safe row pair {sgn*p_k - s <= h, -s <= 0} the slack variable s (which is also the
    // second row's t), the first row's t and both multipliers.
    double y[N];
    double tlo[NPAIR], thi[NPAIR], llo[NPAIR], lhi[NPAIR];
    double sf[NPX], tf[NPX], lf[NPX], lf2[NPX];
    double sb[NPX], tb[NPX], lb[NPX], lb2[NPX];

    // Start of a sweep: make the iterate opaque to the compiler.  Every sweep recomputes its
    // per-row quantities (scalings, residuals, directions) from the iterate instead of storing
    // them; without this fence GVN merges the identical expressions of different sweeps and
    // keeps them live across the whole iteration, which spills the register file.
    HVP_HD void fence() {
        mem.refresh();
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
        for (int i = 0; i < N; ++i) asm volatile("" : "+v"(y[i]));
#pragma unroll
        for (int i = 0; i < NPAIR; ++i) {
            asm volatile("" : "+v"(tlo[i]), "+v"(thi[i]), "+v"(llo[i]), "+v"(lhi[i]));
        }
#pragma unroll
        for (int i = 0; i < NPX; ++i) {
            asm volatile("" : "+v"(sf[i]), "+v"(tf[i]), "+v"(lf[i]), "+v"(lf2[i]));
            asm volatile("" : "+v"(sb[i]), "+v"(tb[i]), "+v"(lb[i]), "+v"(lb2[i]));
        }
#endif
    }
};

// bounds of pair p (V,U,A of step k = p/3 + 1; P of step k = p - 3N + 2)
template <int N, class M>
HVP_HD inline void pair_bounds(const LaneQp<N, M>& q, const Consts& C, int p, double& lo, double& hi) {
    if (p < 3 * N) {
        const int j = p / 3, r = p % 3;
        if (r == 0) { lo = q.vlo(j); hi = q.vhi(j); }
        else if (r == 1) { lo = q.ulo(j); hi = q.uhi(j); }
        else { lo = C.dec[j]; hi = C.acc[j]; }
    } else {
        lo = q.pmin;
        hi = q.pmax;
    }
}

// Row-group traversal over three vectors at once: y (with the constants v0 / P1), a and b
// (directions, no constants).  emit_pair(p, g.y, g.a, g.b); emit_safe(j, p_k(y), g.a, g.b)
// with g the prefix gradient ts * (e_0 + .. + e_j) of p_{j+2}.
template <int N, class M, class FP, class FS>
HVP_HD inline void for_groups3(const LaneQp<N, M>& q, const double* y, const double* a, const double* b, FP&& emit_pair,
                               FS&& emit_safe) {
    double yp = q.v0, ap = 0.0, bp = 0.0;
    double cy = 0.0, ca = 0.0, cb = 0.0;
#pragma unroll
    for (int k = 1; k <= N; ++k) {
        const double yk = y[k - 1], ak = a[k - 1], bk = b[k - 1], am = q.am(k - 1);
        emit_pair(3 * (k - 1) + 0, yk, ak, bk);
        emit_pair(3 * (k - 1) + 1, yk - am * yp, ak - am * ap, bk - am * bp);
        emit_pair(3 * (k - 1) + 2, yk - yp, ak - ap, bk - bp);
        if (k >= 2) {
            cy += y[k - 2];
            ca += a[k - 2];
            cb += b[k - 2];
            const double py = q.P1 + q.ts * cy, pa = q.ts * ca, pb = q.ts * cb;
            emit_pair(3 * N + (k - 2), py, pa, pb);
            emit_safe(k - 2, py, pa, pb);
        }
        yp = yk;
        ap = ak;
        bp = bk;
    }
}

// K += D g g', rhs -= rho g for the gradient shape of pair p (diag / bidiagonal / prefix).
template <int N, class M>
HVP_HD inline void scatter_pair(const LaneQp<N, M>& q, int p, double D, double rho, double* K, double* rhs, double* beta,
                                double* rpre) {
    if (p < 3 * N) {
        const int j = p / 3, r = p % 3;
        K[tri(j, j)] += D;
        rhs[j] -= rho;
        if (r != 0 && j >= 1) {
            const double a = r == 1 ? q.am(j) : 1.0;
            K[tri(j - 1, j - 1)] += D * a * a;
            K[tri(j, j - 1)] -= D * a;
            rhs[j - 1] += a * rho;
        }
    } else {
        beta[p - 3 * N] += D;
        rpre[p - 3 * N] += rho;
    }
}

// rhs -= rho g only (corrector: the factorised K is reused).
template <int N, class M>
HVP_HD inline void scatter_rhs(const LaneQp<N, M>& q, int p, double rho, double* rhs, double* rpre) {
    if (p < 3 * N) {
        const int j = p / 3, r = p % 3;
        rhs[j] -= rho;
        if (r != 0 && j >= 1) rhs[j - 1] += (r == 1 ? q.am(j) : 1.0) * rho;
    } else {
        rpre[p - 3 * N] += rho;
    }
}

// prefix groups: entry (i1, i2) of K receives ts^2 beta of every step whose prefix covers
// max(i1, i2); rhs[i] -= ts * rho of every step covering i.
template <int N, class M>
HVP_HD inline void expand_prefix(const LaneQp<N, M>& q, const double* beta, const double* rpre, double* K, double* rhs) {
    double sb_ = 0.0, sr = 0.0;
    const double ts = q.ts;
#pragma unroll
    for (int m = N - 2; m >= 0; --m) {
        sb_ += beta[m];
        sr += rpre[m];
        rhs[m] -= ts * sr;
        if (K) {
#pragma unroll
            for (int i2 = 0; i2 <= m; ++i2) K[tri(m, i2)] += ts * ts * sb_;
        }
    }
}

template <int N>
HVP_HD inline bool cholesky(double* K) {
#pragma unroll
    for (int j = 0; j < N; ++j) {
        double s = K[tri(j, j)];
#pragma unroll
        for (int k = 0; k < j; ++k) s -= K[tri(j, k)] * K[tri(j, k)];
        if (!(s > 0.0)) return false;
        const double il = frcp(sqrt(s));
        K[tri(j, j)] = il;  // the inverse diagonal is stored
#pragma unroll
        for (int i = j + 1; i < N; ++i) {
            double v = K[tri(i, j)];
#pragma unroll
            for (int k = 0; k < j; ++k) v -= K[tri(i, k)] * K[tri(j, k)];
            K[tri(i, j)] = v * il;
        }
    }
    return true;
}

template <int N>
HVP_HD inline void chol_solve(const double* L, const double* rhs, double* x) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
        double v = rhs[i];
#pragma unroll
        for (int k = 0; k < i; ++k) v -= L[tri(i, k)] * x[k];
        x[i] = v * L[tri(i, i)];
    }
#pragma unroll
    for (int i = N - 1; i >= 0; --i) {
        double v = x[i];
#pragma unroll
        for (int k = i + 1; k < N; ++k) v -= L[tri(k, i)] * x[k];
        x[i] = v * L[tri(i, i)];
    }
}

// ---------------------------------------------------------------- row algebra
// Generic row  val(z) <= h  with slack t, multiplier l, primal residual r = val + t - h,
// scaling d = l / t and  rt = r - rc / l :
//   dl = d (g.dz + rt),   dt = -r - g.dz,   predictor rc = l t,   corrector rc = l t + dl_a dt_a - s mu
//
// Two-sided pair lo <= g.y <= hi (rows -g.y <= -lo and g.y <= hi):
struct PairRow {
    double rlo, rhi, dlo, dhi;
    HVP_HD PairRow(double gy, double lo, double hi, double tlo, double thi, double llo, double lhi) {
        rlo = -gy + tlo + lo;
        rhi = gy + thi - hi;
        dlo = llo * frcp(tlo);
        dhi = lhi * frcp(thi);
    }
    // direction for g.dy = gd and scaled residuals rtlo / rthi
    HVP_HD void dir(double gd, double rtlo, double rthi, double& dtlo, double& dthi, double& dllo, double& dlhi) const {
        dtlo = -rlo + gd;
        dthi = -rhi - gd;
        dllo = dlo * (rtlo - gd);
        dlhi = dhi * (rthi + gd);
    }
};

// Safe pair: row 1  sgn * p_k - s <= h1 (t1, l1), row 2  -s <= 0 (t2 == s, l2); the slack s
// is eliminated with its dual residual r_s = w - l1 - l2 (K gets e g g', rhs gets c g).
struct SafeRow {
    double r1, d1, d2, ie, rs;
    HVP_HD SafeRow(double sgn_pk, double h1, double s, double t1, double l1, double l2, double w) {
        r1 = sgn_pk - s + t1 - h1;
        d1 = l1 * frcp(t1);
        d2 = l2 * frcp(s);
        ie = frcp(d1 + d2);
        rs = w - l1 - l2;
    }
    HVP_HD double e() const { return d1 * d2 * ie; }
    HVP_HD double c(double rt1, double rt2) const { return (d1 * d2 * (rt1 - rt2) + d1 * rs) * ie; }
    // gd = sgn * (prefix gradient . dy)
    HVP_HD void dir(double gd, double rt1, double rt2, double& ds, double& dt1, double& dl1, double& dl2) const {
        ds = (d1 * (gd + rt1) + d2 * rt2 - rs) * ie;
        dl1 = d1 * (gd - ds + rt1);
        dl2 = d2 * (rt2 - ds);
        dt1 = -r1 - gd + ds;
    }
};

// Ratio test with the raw hardware reciprocal: the step is scaled by 0.99 afterwards, so a
// relative error of ~1e-8 in the limit is harmless and saves the Newton refinement.
HVP_HD inline double rcp_approx(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_rcp(x);
#else
    return 1.0 / x;
#endif
}
HVP_HD inline void ratio_test(double& a, double v, double dv) {
    const double r = -v * rcp_approx(dv);
    a = dv < 0.0 ? fmin(a, r) : a;
}

// Accumulators of one assembly of the reduced system.
template <int N>
struct Assembly {
    static constexpr int NPX = N > 1 ? N - 1 : 1;
    double K[N * (N + 1) / 2];
    double rhs[N];            // - sum_rows d rt g   (the -rd part is added at the end)
    double beta[NPX], rpre[NPX];
    double lam_pre[NPX];      // prefix part of sum lam g
    double rd[N];             // non-prefix part of sum lam g
    double gap, rpmax, rsmax;
};

// Row set: two-sided pairs V, U, A for every step (and P when PBOX), safe pairs for k >= 2.
// PBOX = false drops the position-box rows 0 <= p_k <= 10000 (never active for a platoon:
// the caller verifies the solution and re-solves the rare violator with PBOX = true, which is
// exact: a relaxed optimum that satisfies the dropped rows is the optimum).
template <int N, bool PBOX, class M = ArrayMem<N>>
struct Solver {
    static constexpr int NP = N - 1;
    static constexpr int NPX = N > 1 ? N - 1 : 1;
    static constexpr int NT = N * (N + 1) / 2;
    static constexpr int NPAIR_ACTIVE = 3 * N + (PBOX ? NP : 0);

    // traversal over (y, a, b) skipping the P pairs when !PBOX
    template <class FP, class FS>
    HVP_HD static void groups(const LaneQp<N, M>& q, const double* y, const double* a, const double* b, FP&& fp,
                              FS&& fs) {
        for_groups3(
            q, y, a, b,
            [&](int p, double gy, double ga, double gb) {
                if (PBOX || p < 3 * N) fp(p, gy, ga, gb);
            },
            fs);
    }

    // contributions of the state (tlo, thi, llo, lhi / s, t1, l1, l2) at row values gy / pk
    HVP_HD static void assemble_pair(const LaneQp<N, M>& q, const Consts& C, Assembly<N>& A, int p, double gy) {
        double lo, hi;
        pair_bounds(q, C, p, lo, hi);
        const double tl = q.tlo[p], th = q.thi[p], ll = q.llo[p], lh = q.lhi[p];
        const PairRow R(gy, lo, hi, tl, th, ll, lh);
        A.gap += ll * tl + lh * th;
        A.rpmax = fmax(A.rpmax, fmax(fabs(R.rlo), fabs(R.rhi)));
        // predictor rt = r - t ; rho = -dlo rtlo + dhi rthi ; dual part (lhi - llo) g
        const double rho = -R.dlo * (R.rlo - tl) + R.dhi * (R.rhi - th);
        double Kd[1];
        (void)Kd;
        if (p < 3 * N) {
            const int j = p / 3, r = p % 3;
            const double D = R.dlo + R.dhi, lg = lh - ll;
            A.K[tri(j, j)] += D;
            A.rhs[j] -= rho;
            A.rd[j] += lg;
            if (r != 0 && j >= 1) {
                const double am = r == 1 ? q.am(j) : 1.0;
                A.K[tri(j - 1, j - 1)] += D * am * am;
                A.K[tri(j, j - 1)] -= D * am;
                A.rhs[j - 1] += am * rho;
                A.rd[j - 1] -= am * lg;
            }
        } else {
            const int j = p - 3 * N;
            A.beta[j] += R.dlo + R.dhi;
            A.rpre[j] += rho;
            A.lam_pre[j] += lh - ll;
        }
    }
    HVP_HD static void assemble_safe(const LaneQp<N, M>& q, Assembly<N>& A, int j, double sgn, double sgnpk, double h1,
                                     double s, double t1, double l1, double l2, double w) {
        const SafeRow R(sgnpk, h1, s, t1, l1, l2, w);
        A.gap += l1 * t1 + l2 * s;
        A.rpmax = fmax(A.rpmax, fabs(R.r1));
        A.rsmax = fmax(A.rsmax, fabs(R.rs));
        A.beta[j] += R.e();
        A.rpre[j] += sgn * R.c(R.r1 - t1, -s);
        A.lam_pre[j] += sgn * l1;
    }

    HVP_HD static void assemble_begin(const LaneQp<N, M>& q, Assembly<N>& A) {
#pragma unroll
        for (int i = 0; i < NT; ++i) A.K[i] = q.H[i];
#pragma unroll
        for (int i = 0; i < N; ++i) { A.rhs[i] = 0.0; A.rd[i] = 0.0; }
#pragma unroll
        for (int i = 0; i < NPX; ++i) { A.beta[i] = 0.0; A.rpre[i] = 0.0; A.lam_pre[i] = 0.0; }
        A.gap = 0.0;
        A.rpmax = 0.0;
        A.rsmax = 0.0;
    }
    // finish: rd = H y + f + G'lam ; rhs = -rd - sum d rt g ; K prefix expansion
    HVP_HD static void assemble_end(const LaneQp<N, M>& q, Assembly<N>& A, const double* y) {
        double sb_ = 0.0, sr = 0.0, sl = 0.0;
        const double ts = q.ts;
#pragma unroll
        for (int m = N - 2; m >= 0; --m) {
            sb_ += A.beta[m];
            sr += A.rpre[m];
            sl += A.lam_pre[m];
            A.rhs[m] -= ts * sr;
            A.rd[m] += ts * sl;
#pragma unroll
            for (int i2 = 0; i2 <= m; ++i2) A.K[tri(m, i2)] += ts * ts * sb_;
        }
#pragma unroll
        for (int i = 0; i < N; ++i) {
            double s = q.f[i];
#pragma unroll
            for (int j = 0; j < N; ++j) s += q.H[i >= j ? tri(i, j) : tri(j, i)] * y[j];
            A.rd[i] += s;
            A.rhs[i] -= A.rd[i];
        }
    }

    HVP_HD HVP_FORCEINLINE static QpOut solve(LaneQp<N, M>& q, const Consts& C) {
        QpOut out{0.0, 2, 0};
        const double w = C.w;
        const int m = 2 * NPAIR_ACTIVE + (true ? 2 * NP : 0) + (true ? 2 * NP : 0);
        const double zero[N] = {};

        // =============== initial point (CVXOPT / Mehrotra): minimise 1/2 y'Hy + f'y + w 1's
        // + 1/2 |h - Gz|^2 (one unit-scaled reduced solve from z = t = lam = 0), then
        // t = h - Gz, lam = -t, both shifted into the interior and centred.
        {
            double K[NT], rhs[N], beta[NPX], rpre[NPX];
#pragma unroll
            for (int i = 0; i < NT; ++i) K[i] = q.H[i];
#pragma unroll
            for (int i = 0; i < N; ++i) rhs[i] = -q.f[i];
#pragma unroll
            for (int i = 0; i < NPX; ++i) { beta[i] = 0.0; rpre[i] = 0.0; }
            groups(q, zero, zero, zero,
                   [&](int p, double gy, double, double) {
                       double lo, hi;
                       pair_bounds(q, C, p, lo, hi);
                       scatter_pair(q, p, 2.0, -(-gy + lo) + (gy - hi), K, rhs, beta, rpre);
                   },
                   [&](int j, double pk, double, double) {
                       if (true) { beta[j] += 0.5; rpre[j] += 0.5 * ((pk - q.hf(j)) + w); }
                       if (true) { beta[j] += 0.5; rpre[j] -= 0.5 * ((-pk + q.hb(j)) + w); }
                   });
            expand_prefix<N>(q, beta, rpre, K, rhs);
            if (!cholesky<N>(K)) return out;
            chol_solve<N>(K, rhs, q.y);
            double tmin = 1e300, tmax = -1e300;
            groups(q, q.y, zero, zero,
                   [&](int p, double gy, double, double) {
                       double lo, hi;
                       pair_bounds(q, C, p, lo, hi);
                       q.tlo[p] = gy - lo;
                       q.thi[p] = hi - gy;
                       tmin = fmin(tmin, fmin(q.tlo[p], q.thi[p]));
                       tmax = fmax(tmax, fmax(q.tlo[p], q.thi[p]));
                   },
                   [&](int j, double pk, double, double) {
                       // slack of the unit solve: s = (g.y + rt1 - r_s) / 2 = (sgn p_k - h - w) / 2
                       if (true) {
                           const double s = 0.5 * (pk - q.hf(j) - w);
                           q.sf[j] = s;
                           q.tf[j] = q.hf(j) - (pk - s);
                           tmin = fmin(tmin, fmin(q.tf[j], s));
                           tmax = fmax(tmax, fmax(q.tf[j], s));
                       }
                       if (true) {
                           const double s = 0.5 * (-pk + q.hb(j) - w);
                           q.sb[j] = s;
                           q.tb[j] = -q.hb(j) - (-pk - s);
                           tmin = fmin(tmin, fmin(q.tb[j], s));
                           tmax = fmax(tmax, fmax(q.tb[j], s));
                       }
                   });
            const double st = fmax(-1.5 * tmin, 0.0), sl = fmax(1.5 * tmax, 0.0);  // lam = -t
            double tl = 0.0, tsum = 0.0, lsum = 0.0;
            auto acc = [&](double t) {
                const double tt = t + st, ll = -t + sl;
                tl += tt * ll;
                tsum += tt;
                lsum += ll;
            };
            groups(q, zero, zero, zero, [&](int p, double, double, double) { acc(q.tlo[p]); acc(q.thi[p]); },
                   [&](int j, double, double, double) {
                       if (true) { acc(q.tf[j]); acc(q.sf[j]); }
                       if (true) { acc(q.tb[j]); acc(q.sb[j]); }
                   });
            const double dt0 = lsum > 0 ? 0.5 * tl / lsum : 1.0, dl0 = tsum > 0 ? 0.5 * tl / tsum : 1.0;
            auto fix = [&](double& t, double& l) {
                const double t0v = t;
                t = t0v + st + dt0;
                l = -t0v + sl + dl0;
                t = t > 0.0 ? t : 1.0;
                l = l > 0.0 ? l : 1.0;
            };
            groups(q, zero, zero, zero,
                   [&](int p, double, double, double) { fix(q.tlo[p], q.llo[p]); fix(q.thi[p], q.lhi[p]); },
                   [&](int j, double, double, double) {
                       if (true) { fix(q.tf[j], q.lf[j]); fix(q.sf[j], q.lf2[j]); }
                       if (true) { fix(q.tb[j], q.lb[j]); fix(q.sb[j], q.lb2[j]); }
                   });
        }

        double sq = fmax(1.0, w);
#pragma unroll
        for (int i = 0; i < N; ++i) sq = fmax(sq, fabs(q.f[i]));
        const double sh = fmax(fmax(1.0, fabs(q.pmax)), fmax(fabs(q.pmin), fmax(fabs(q.P1), 1e4)));

        // =============== assembly at the initial point
        Assembly<N> A;
        assemble_begin(q, A);
        groups(q, q.y, zero, zero, [&](int p, double gy, double, double) { assemble_pair(q, C, A, p, gy); },
               [&](int j, double pk, double, double) {
                   if (true) assemble_safe(q, A, j, 1.0, pk, q.hf(j), q.sf[j], q.tf[j], q.lf[j], q.lf2[j], w);
                   if (true) assemble_safe(q, A, j, -1.0, -pk, -q.hb(j), q.sb[j], q.tb[j], q.lb[j], q.lb2[j], w);
               });
        assemble_end(q, A, q.y);

        const int maxit = C.max_iter;
        double dya[N], dy[N];
        double last_step = 1e300;  // max |alpha dy| of the previous iteration: u / x accuracy
        for (int it = 0; it <= maxit; ++it) {
            // ------------------------------------------------ convergence
            double rdmax = A.rsmax;
#pragma unroll
            for (int i = 0; i < N; ++i) rdmax = fmax(rdmax, fabs(A.rd[i]));
            double J = q.C0;
#pragma unroll
            for (int i = 0; i < N; ++i) {
                double hy = 0.0;
#pragma unroll
                for (int j = 0; j < N; ++j) hy += q.H[i >= j ? tri(i, j) : tri(j, i)] * q.y[j];
                J += (0.5 * hy + q.f[i]) * q.y[i];
            }
            out.iters = it;
            if (rdmax <= C.tol * sq && A.rpmax <= C.tol * sh && A.gap <= 0.1 * C.tol * fmax(1.0, fabs(J)) &&
                last_step <= 1e-9) {
                out.status = 0;
                return out;
            }
            // fp64 floor: at the iteration cap, or where the Newton matrix no longer factors (its
            // condition grows as mu -> 0; the ADMM forms' Huber pieces reach that point first), accept
            // an iterate that meets a 1e3-looser tolerance
            const bool loose = rdmax <= 1e3 * C.tol * sq && A.rpmax <= 1e3 * C.tol * sh &&
                               A.gap <= 1e2 * C.tol * fmax(1.0, fabs(J));
            if (it == maxit) {
                if (loose) out.status = 0;
                return out;
            }
            if (!cholesky<N>(A.K)) {
                if (loose) out.status = 0;
                return out;
            }
            chol_solve<N>(A.K, A.rhs, dya);
            const double mu = A.gap / m;

            q.fence();
            // ------------------------------------------------ pass X: affine step, centring and the
            // corrector rhs split as  rhsA + sigma mu * rhsB  (linear in sigma mu)
            double amax_a = 1.0, S1 = 0.0, S2 = 0.0;
            double rA[N], rB[N], pA[NPX], pB[NPX];
#pragma unroll
            for (int i = 0; i < N; ++i) { rA[i] = 0.0; rB[i] = 0.0; }
#pragma unroll
            for (int i = 0; i < NPX; ++i) { pA[i] = 0.0; pB[i] = 0.0; }
            groups(q, q.y, dya, zero,
                   [&](int p, double gy, double ga, double) {
                       double lo, hi;
                       pair_bounds(q, C, p, lo, hi);
                       const double tl = q.tlo[p], th = q.thi[p], ll = q.llo[p], lh = q.lhi[p];
                       const PairRow R(gy, lo, hi, tl, th, ll, lh);
                       double dtl, dth, dll, dlh;
                       R.dir(ga, R.rlo - tl, R.rhi - th, dtl, dth, dll, dlh);
                       ratio_test(amax_a, tl, dtl);
                       ratio_test(amax_a, th, dth);
                       ratio_test(amax_a, ll, dll);
                       ratio_test(amax_a, lh, dlh);
                       S1 += ll * dtl + tl * dll + lh * dth + th * dlh;
                       S2 += dll * dtl + dlh * dth;
                       // rt_c = r - t - (dl_a dt_a)/l + sigma mu / l ; d / l = 1 / t
                       const double rtlA = R.rlo - tl - dll * dtl * frcp(ll);
                       const double rthA = R.rhi - th - dlh * dth * frcp(lh);
                       const double rhoA = -R.dlo * rtlA + R.dhi * rthA;
                       const double rhoB = -frcp(tl) + frcp(th);
                       scatter_rhs(q, p, rhoA, rA, pA);
                       scatter_rhs(q, p, rhoB, rB, pB);
                   },
                   [&](int j, double pk, double ga, double) {
                       auto safe = [&](double sgn, double h1, double s, double t1, double l1, double l2) {
                           const SafeRow R(sgn * pk, h1, s, t1, l1, l2, w);
                           double ds, dt1, dl1, dl2;
                           R.dir(sgn * ga, R.r1 - t1, -s, ds, dt1, dl1, dl2);
                           ratio_test(amax_a, s, ds);
                           ratio_test(amax_a, t1, dt1);
                           ratio_test(amax_a, l1, dl1);
                           ratio_test(amax_a, l2, dl2);
                           S1 += l1 * dt1 + t1 * dl1 + l2 * ds + s * dl2;
                           S2 += dl1 * dt1 + dl2 * ds;
                           const double rt1A = R.r1 - t1 - dl1 * dt1 * frcp(l1);
                           const double rt2A = -s - dl2 * ds * frcp(l2);
                           pA[j] += sgn * R.c(rt1A, rt2A);
                           pB[j] += sgn * R.d1 * R.d2 * R.ie * (frcp(l1) - frcp(l2));
                       };
                       if (true) safe(1.0, q.hf(j), q.sf[j], q.tf[j], q.lf[j], q.lf2[j]);
                       if (true) safe(-1.0, -q.hb(j), q.sb[j], q.tb[j], q.lb[j], q.lb2[j]);
                   });
            const double mua = (A.gap + amax_a * S1 + amax_a * amax_a * S2) / m;
            const double sr = fmax(mua, 0.0) / mu;
            const double smu = sr * sr * sr * mu;
            {
                double rhs[N];
                double sa = 0.0, sb_ = 0.0;
#pragma unroll
                for (int mm = N - 2; mm >= 0; --mm) {
                    sa += pA[mm];
                    sb_ += pB[mm];
                    rA[mm] -= q.ts * sa;
                    rB[mm] -= q.ts * sb_;
                }
                // rA / rB hold -sum rho g (scatter_rhs subtracts)
#pragma unroll
                for (int i = 0; i < N; ++i) rhs[i] = -A.rd[i] + rA[i] + smu * rB[i];
                chol_solve<N>(A.K, rhs, dy);
            }

            // ------------------------------------------------ pass Y: corrector step length
            // corrector scaled residuals of a row from its affine direction
            auto pair_dirs = [&](const PairRow& R, double ga, double gd, double tl, double th, double ll, double lh,
                                 double& dtl, double& dth, double& dll, double& dlh) {
                double atl, ath, all_, alh;
                R.dir(ga, R.rlo - tl, R.rhi - th, atl, ath, all_, alh);
                const double rtl = R.rlo - tl - (all_ * atl - smu) * frcp(ll);
                const double rth = R.rhi - th - (alh * ath - smu) * frcp(lh);
                R.dir(gd, rtl, rth, dtl, dth, dll, dlh);
            };
            auto safe_dirs = [&](const SafeRow& R, double ga, double gd, double s, double t1, double l1, double l2,
                                 double& ds, double& dt1, double& dl1, double& dl2) {
                double as, at1, al1, al2;
                R.dir(ga, R.r1 - t1, -s, as, at1, al1, al2);
                const double rt1 = R.r1 - t1 - (al1 * at1 - smu) * frcp(l1);
                const double rt2 = -s - (al2 * as - smu) * frcp(l2);
                R.dir(gd, rt1, rt2, ds, dt1, dl1, dl2);
            };
            double amax = 1.0;
            q.fence();
            groups(q, q.y, dya, dy,
                   [&](int p, double gy, double ga, double gd) {
                       double lo, hi;
                       pair_bounds(q, C, p, lo, hi);
                       const double tl = q.tlo[p], th = q.thi[p], ll = q.llo[p], lh = q.lhi[p];
                       const PairRow R(gy, lo, hi, tl, th, ll, lh);
                       double dtl, dth, dll, dlh;
                       pair_dirs(R, ga, gd, tl, th, ll, lh, dtl, dth, dll, dlh);
                       ratio_test(amax, tl, dtl);
                       ratio_test(amax, th, dth);
                       ratio_test(amax, ll, dll);
                       ratio_test(amax, lh, dlh);
                   },
                   [&](int j, double pk, double ga, double gd) {
                       auto safe = [&](double sgn, double h1, double s, double t1, double l1, double l2) {
                           const SafeRow R(sgn * pk, h1, s, t1, l1, l2, w);
                           double ds, dt1, dl1, dl2;
                           safe_dirs(R, sgn * ga, sgn * gd, s, t1, l1, l2, ds, dt1, dl1, dl2);
                           ratio_test(amax, s, ds);
                           ratio_test(amax, t1, dt1);
                           ratio_test(amax, l1, dl1);
                           ratio_test(amax, l2, dl2);
                       };
                       if (true) safe(1.0, q.hf(j), q.sf[j], q.tf[j], q.lf[j], q.lf2[j]);
                       if (true) safe(-1.0, -q.hb(j), q.sb[j], q.tb[j], q.lb[j], q.lb2[j]);
                   });
            const double alpha = fmin(1.0, 0.99 * amax);

            // ------------------------------------------------ pass Z: update + next assembly
            double ynew[N];
#pragma unroll
            for (int i = 0; i < N; ++i) ynew[i] = q.y[i] + alpha * dy[i];
            assemble_begin(q, A);
            q.fence();
            groups(q, q.y, dya, dy,
                   [&](int p, double gy, double ga, double gd) {
                       double lo, hi;
                       pair_bounds(q, C, p, lo, hi);
                       const double tl = q.tlo[p], th = q.thi[p], ll = q.llo[p], lh = q.lhi[p];
                       const PairRow R(gy, lo, hi, tl, th, ll, lh);
                       double dtl, dth, dll, dlh;
                       pair_dirs(R, ga, gd, tl, th, ll, lh, dtl, dth, dll, dlh);
                       q.tlo[p] = tl + alpha * dtl;
                       q.thi[p] = th + alpha * dth;
                       q.llo[p] = ll + alpha * dll;
                       q.lhi[p] = lh + alpha * dlh;
                       assemble_pair(q, C, A, p, gy + alpha * gd);
                   },
                   [&](int j, double pk, double ga, double gd) {
                       auto safe = [&](double sgn, double h1, double& s, double& t1, double& l1, double& l2) {
                           const SafeRow R(sgn * pk, h1, s, t1, l1, l2, w);
                           double ds, dt1, dl1, dl2;
                           safe_dirs(R, sgn * ga, sgn * gd, s, t1, l1, l2, ds, dt1, dl1, dl2);
                           s += alpha * ds;
                           t1 += alpha * dt1;
                           l1 += alpha * dl1;
                           l2 += alpha * dl2;
                           assemble_safe(q, A, j, sgn, sgn * (pk + alpha * gd), h1, s, t1, l1, l2, w);
                       };
                       if (true) safe(1.0, q.hf(j), q.sf[j], q.tf[j], q.lf[j], q.lf2[j]);
                       if (true) safe(-1.0, -q.hb(j), q.sb[j], q.tb[j], q.lb[j], q.lb2[j]);
                   });
            last_step = 0.0;
#pragma unroll
            for (int i = 0; i < N; ++i) {
                last_step = fmax(last_step, fabs(ynew[i] - q.y[i]));
                q.y[i] = ynew[i];
            }
            assemble_end(q, A, q.y);
        }
        out.status = 2;
        return out;
    }
};

template <int N, class M>
HVP_HD inline QpOut solve_lane(LaneQp<N, M>& q, const Consts& C) {
    return Solver<N, true, M>::solve(q, C);
}

// Position-box check of a relaxed (PBOX = false) solution: p_k in [pmin, pmax] for k = 2..N.
template <int N, class M>
HVP_HD inline bool pbox_ok(const LaneQp<N, M>& q) {
    double cum = 0.0;
    const double tol = 1e-9 * (1.0 + fmax(fabs(q.pmin), fabs(q.pmax)));
#pragma unroll
    for (int j = 0; j < N - 1; ++j) {
        cum += q.y[j];
        const double pk = q.P1 + q.ts * cum;
        if (pk < q.pmin - tol || pk > q.pmax + tol) return false;
    }
    return true;
}

// tail relaxation of one undecided step (defined below with reach_step)
HVP_HD inline int relax_step(const hvp_system& S, const Consts& C, int k, double lo, double hi, double& nlo,
                             double& nhi, double& bmax, bool& dead);

// ------------------------------------------------------------------ problem setup
// The lane QP of (instance params (x0, x_front, x_back, leader_x), region code) is assembled in
// two parts:
//   setup_track  sigma-independent: the tracking terms (H, f, C0), the safe-distance bounds
//                (hf, hb) and the constant k = 0, 1 slacks -- the same for every node of an
//                instance, so the branch-and-bound kernels compute it once per instance
//                (hvp_lane.h: K_inst_prep) and the node kernels only load it;
//   setup_input  per region sequence / node: dynamics a, b, c of every step (tail relaxed from
//                v_K in [rlo, rhi] for branch-and-bound bounds), the input and accel bounds, the
//                velocity bounds, and the input cost Q_u u^2 + Q_du du^2 added to (H, f, C0).
// setup_lane = both, in this order (H and f accumulate exactly as one pass would).

// tracking part: H (packed lower, NT), f (N), C0, hf / hb (N - 1): bounds of the safe rows of
// steps 2..N (an absent neighbour gets an INERT row: its bound lies beyond any position
// reachable under the velocity box, so the row can never be active and every lane runs the same
// branch-free code).  Returns P1 = p_0 + ts v_0.
template <int N>
HVP_HD inline double setup_track(const hvp_system& S, const Consts& C, int role, const double* prm, double* H,
                                 double* f, double& C0_out, double* hf, double* hb) {
    const double p0 = prm[0], v0 = prm[1];
    const double* xf = prm + 2;
    const double* xb = prm + 2 + 2 * (N + 1);
    const double* xl = prm + 2 + 4 * (N + 1);
    const double ts = S.ts;
    const double P1 = p0 + ts * v0;
    const bool has_sf = (role & HVP_ROLE_SAFE_FRONT) != 0, has_sb = (role & HVP_ROLE_SAFE_BACK) != 0;
#pragma unroll
    for (int j = 0; j < N - 1; ++j) {
        const double reach = ts * (j + 1);
        hf[j] = has_sf ? xf[j + 2] - C.d_safe : P1 + reach * S.vmax + 100.0;
        hb[j] = has_sb ? xb[j + 2] + C.d_safe : P1 + reach * S.vmin - 100.0;
    }
#pragma unroll
    for (int i = 0; i < N * (N + 1) / 2; ++i) H[i] = 0.0;
#pragma unroll
    for (int i = 0; i < N; ++i) f[i] = 0.0;
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
            const double qa = Qpp * m00;                                           // (QM)[0][0]
            const double qc = Qpp * m01 + Qpv * m11, qd = Qpv * m01 + Qvv * m11;  // (QM)[0][1], (QM)[1][1]
            Wpp += m00 * qa;
            Wpv += m00 * qc;
            Wvv += m01 * qc + m11 * qd;
            const double Qr0 = Qpp * r0 + Qpv * r1, Qr1 = Qpv * r0 + Qvv * r1;
            lp += m00 * Qr0;
            lv += m01 * Qr0 + m11 * Qr1;
            cc += r0 * Qr0 + r1 * Qr1;
        };
        const int K1 = N + 1;
        if (tf) add(1.0, t0, 1.0, d0 - xf[k], -xf[K1 + k]);
        if (tb) add(-1.0, 0.0, -1.0, xb[k] + t0 * xb[K1 + k] + d0, xb[K1 + k]);
        if (tl) {
            if (lsp) add(1.0, t0, 1.0, d0 - xl[k], -xl[K1 + k]);
            else add(1.0, 0.0, 1.0, -xl[k], -xl[K1 + k]);
        }
        // x_k = xbar + Gamma y : p = pbar + ts*prefix(0..k-2), v = vbar + e_{k-1}
        const double pbar = k == 0 ? p0 : P1;
        const double vbar = k == 0 ? v0 : 0.0;
        // gradient of the quadratic form at xbar
        const double gp = 2.0 * (Wpp * pbar + Wpv * vbar + lp);
        const double gv = 2.0 * (Wpv * pbar + Wvv * vbar + lv);
        C0 += Wpp * pbar * pbar + 2.0 * Wpv * pbar * vbar + Wvv * vbar * vbar + 2.0 * (lp * pbar + lv * vbar) + cc;
        if (k >= 1) {
            const int jv = k - 1;  // v_k = y[jv]
            H[tri(jv, jv)] += 2.0 * Wvv;
            f[jv] += gv;
            // prefix part (indices 0..k-2) with weight ts
#pragma unroll
            for (int i = 0; i < N; ++i) {
                if (i > k - 2) break;
                f[i] += ts * gp;
#pragma unroll
                for (int i2 = 0; i2 <= i; ++i2) H[tri(i, i2)] += 2.0 * Wpp * ts * ts;
                // cross p-v: 2 * Wpv * (ts e_i)(e_jv)' symmetric ; jv > i always
                H[tri(jv, i)] += 2.0 * Wpv * ts;
            }
        }
    }
    // constant slacks of k = 0, 1 (p_0, p_1 fixed)
    if (has_sf) C0 += C.w * (fmax(0.0, p0 - xf[0] + C.d_safe) + fmax(0.0, P1 - xf[1] + C.d_safe));
    if (has_sb) C0 += C.w * (fmax(0.0, xb[0] + C.d_safe - p0) + fmax(0.0, xb[1] + C.d_safe - P1));
    C0_out = C0;
    return P1;
}

// lane scalars of the instance (the p_1 row is sigma-independent).  Returns false when the
// constant row p_1 in [pmin, pmax] is violated.
template <int N, class M>
HVP_HD inline bool setup_scalars(LaneQp<N, M>& q, const hvp_system& S, int role, double p0, double v0) {
    q.v0 = v0;
    q.ts = S.ts;
    q.P1 = p0 + S.ts * v0;
    q.pmin = S.pmin;
    q.pmax = S.pmax;
    q.has_sf = (role & HVP_ROLE_SAFE_FRONT) != 0;
    q.has_sb = (role & HVP_ROLE_SAFE_BACK) != 0;
    return q.P1 >= S.pmin - 1e-9 * (1.0 + fabs(S.pmin)) && q.P1 <= S.pmax + 1e-9 * (1.0 + fabs(S.pmax));
}

// per-node part (see above); q.H, q.f, q.C0 hold the tracking part on entry
template <int N, class M>
HVP_HD inline void setup_input(LaneQp<N, M>& q, const hvp_system& S, const Consts& C, uint64_t code, int K = N,
                               double rlo = 0.0, double rhi = -1.0) {
    const double v0 = q.v0;
    double a[N], b[N], c[N];
    unsigned ucost = 0;      // steps carrying their input cost
    bool relax = rlo <= rhi;  // [rlo, rhi] = exact interval of v_K (branch and bound)
#pragma unroll
    for (int k = 0; k < N; ++k) {
        // steps k >= K are RELAXED (branch-and-bound bound problem, hvp_ipm.h:relax_step): v_{k+1}
        // keeps the interval reachable from v_K and, when the regions step k may take share
        // (a, c), the step takes the virtual region (a, b_max, c) with its input rows and cost;
        // otherwise the input rows and input cost are dropped.  What remains is a valid lower
        // bound of every completion of the fixed prefix.
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
        const bool on = fixed || vr >= 0;
        const int r = fixed ? code_region(code, k) : (vr >= 0 ? vr : 0);
        a[k] = on ? S.a[r] : 1.0;
        b[k] = fixed ? S.b[r] : (vr >= 0 ? bm : 1.0);
        c[k] = on ? S.c[r] : 0.0;
        ucost |= on ? 1u << k : 0u;
        q.mem.set(F_AM, k, a[k]);
        q.mem.set(F_ULO, k, on ? c[k] + b[k] * S.umin : -1e30);
        q.mem.set(F_UHI, k, on ? c[k] + b[k] * S.umax : 1e30);
        // bounds on v_{k+1}: region sigma_{k+1} (if fixed) intersected with the state box; a
        // relaxed v_{k+1} its reachable interval (v_K's own is implied by the prefix)
        if (k + 1 < K) {
            const int r1 = code_region(code, k + 1);
            q.mem.set(F_VLO, k, fmax(S.vmin, S.vlo[r1]));
            q.mem.set(F_VHI, k, fmin(S.vmax, S.vhi[r1]));
        } else if (!fixed && relax) {
            q.mem.set(F_VLO, k, fmax(S.vmin, nlo));
            q.mem.set(F_VHI, k, fmin(S.vmax, nhi));
        } else {
            q.mem.set(F_VLO, k, S.vmin);
            q.mem.set(F_VHI, k, S.vmax);
        }
    }
    // control effort  Qu u_k^2 and variation Qdu (u_{k+1} - u_k)^2, u_k = ubar_k + gu_k . y
    // gu_k has entries at k (1/b_k) and k-1 (-a_k/b_k)
    double ubar[N], gk[N], gkm[N];
    double C0 = q.C0;
#pragma unroll
    for (int k = 0; k < N; ++k) {
        const double ib = 1.0 / b[k];
        ubar[k] = k == 0 ? -(a[0] * v0 + c[0]) * ib : -c[k] * ib;
        gk[k] = ib;
        gkm[k] = k == 0 ? 0.0 : -a[k] * ib;
        const bool uk = (ucost >> k) & 1u;
        const double w2 = uk ? 2.0 * C.Qu : 0.0;
        q.H[tri(k, k)] += w2 * gk[k] * gk[k];
        q.f[k] += w2 * ubar[k] * gk[k];
        if (k >= 1) {
            q.H[tri(k - 1, k - 1)] += w2 * gkm[k] * gkm[k];
            q.H[tri(k, k - 1)] += w2 * gk[k] * gkm[k];
            q.f[k - 1] += w2 * ubar[k] * gkm[k];
        }
        C0 += uk ? C.Qu * ubar[k] * ubar[k] : 0.0;
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
}

// Builds the lane QP for instance params (x0, x_front, x_back, leader_x) and region code.
// Returns false when a sigma-independent constant row (p_1 box) is violated.
template <int N, class M>
HVP_HD inline bool setup_lane(LaneQp<N, M>& q, const hvp_system& S, const Consts& C, int role, const double* prm,
                              uint64_t code, int K = N, double rlo = 0.0, double rhi = -1.0) {
    const bool ok = setup_scalars<N>(q, S, role, prm[0], prm[1]);
    double hf[N > 1 ? N - 1 : 1], hb[N > 1 ? N - 1 : 1];
    setup_track<N>(S, C, role, prm, q.H, q.f, q.C0, hf, hb);
#pragma unroll
    for (int j = 0; j < N - 1; ++j) {
        q.mem.set(F_HF, j, hf[j]);
        q.mem.set(F_HB, j, hb[j]);
    }
    setup_input<N>(q, S, C, code, K, rlo, rhi);
    return ok;
}

// Objective of the lane's solution evaluated term by term on the trajectory, as the reference
// writes it (fleet_decent_mld.py:107-169): squared tracking errors, Q_u u^2, Q_du du^2 and
// w * max(0, .) slacks.  Avoids the cancellation of C0 + 1/2 y'Hy + f'y (positions ~3e3), so
// the costs the argmin compares carry relative error ~1e-15 instead of ~1e-9.
// Launders a pointer on the device so that loads through it are not merged with loads made
// before a solve (which would keep those values live in registers across the whole IPM).
template <class T>
HVP_HD inline T* opaque_ptr(T* p) {
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+v"(p));
#endif
    return p;
}

template <int N, class M>
HVP_HD inline double direct_cost(const LaneQp<N, M>& q, const hvp_system& S_in, const Consts& C, int role,
                                 const double* prm_in, uint64_t code, int K = N) {
    const double* prm = opaque_ptr(prm_in);
    const hvp_system& S = *opaque_ptr(&S_in);
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
            const int r = code_region(code, k);
            const double vn = q.y[k];
            double u = (vn - S.a[r] * v - S.c[r]) / S.b[r];
            if (k < K) {
                J += C.Qu * u * u;
            } else if (q.ulo(k) > -1e29) {  // relaxed step in a virtual region (setup_lane)
                const double bv = (q.mem.get(F_UHI, k) - q.ulo(k)) / (S.umax - S.umin);
                const double cv = q.ulo(k) - bv * S.umin;
                const double uv = (vn - q.am(k) * v - cv) / bv;
                J += C.Qu * uv * uv;
            }
            if (k >= 1 && k < K) J += C.Qdu * (u - uprev) * (u - uprev);
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

// Child of a node at depth k (prefix of k steps, v_k in [lo, hi]) taking region r at step k:
// false if r is not reachable (band disjoint from [lo, hi] or no admissible input / accel).
HVP_HD inline bool bnb_child(const hvp_system& S, const Consts& C, int k, double lo, double hi, int r, double* nlo,
                             double* nhi) {
    const double tol = 1e-9 * (1.0 + fabs(fmin(hi, S.vhi[r])));
    double ilo = fmax(lo, S.vlo[r]), ihi = fmin(hi, S.vhi[r]);
    if (ilo > ihi + tol) return false;
    if (ilo > ihi) ilo = ihi = 0.5 * (ilo + ihi);
    return reach_step(ilo, ihi, S.a[r], S.b[r], S.c[r], S.umin, S.umax, C.dec[k], C.acc[k], S.vmin, S.vmax, nlo, nhi);
}

// Tail relaxation, one undecided step k (oracle: hvp_oracle.c:relax_tail).  From the interval
// [lo, hi] of v_k: the hull [nlo, nhi] of v_{k+1} over every region step k may still take and,
// when all of them share the velocity dynamics (a, c) with b > 0 (and umin <= 0 <= umax), the
// VIRTUAL region of the step: dynamics (a, bmax, c) with the input box and cost on
// s = u b_r / bmax, a valid relaxation of every region's input (|s| <= |u|).  Returns the first
// such region (virt) or -1; dead = no region is reachable (the relaxation stops there).
HVP_HD inline int relax_step(const hvp_system& S, const Consts& C, int k, double lo, double hi, double& nlo,
                             double& nhi, double& bmax, bool& dead) {
    nlo = 1e300;
    nhi = -1e300;
    bmax = 0.0;
    int first = -1;
    bool shared = S.umin <= 0.0 && S.umax >= 0.0 && S.umax > S.umin;
    for (int r = 0; r < S.n_regions; ++r) {
        double a, b;
        if (!bnb_child(S, C, k, lo, hi, r, &a, &b)) continue;
        nlo = fmin(nlo, a);
        nhi = fmax(nhi, b);
        if (first < 0) first = r;
        else if (S.a[r] != S.a[first] || S.c[r] != S.c[first]) shared = false;
        if (!(S.b[r] > 0.0)) shared = false;
        bmax = fmax(bmax, S.b[r]);
    }
    dead = first < 0;
    return shared && !dead ? first : -1;
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
            code = (uint32_t)code_with(code, k, r);
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
