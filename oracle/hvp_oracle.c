/*
 * hvp_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's local hybrid-MPC solve, used as the parity checker for
 * libhvpsolve.so (tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg are the
 * only code allowed to load it).  It is never part of the product path.
 *
 * What it restates (reference file:line; [EXT] = dmpcpwa/gurobipy, absent from the container,
 * behaviour inferred from the call sites -- see DESIGN.md "Oracle"):
 *   - MLD model of MpcMld [EXT] as used by LocalMpcMld (fleet_decent_mld.py:46-48,
 *     constrain_first_state=False): x(2,N+1), u(1,N); D x_k <= E for k = 1..N; F u_k <= G for
 *     k = 0..N-1; one region per step with S_r x_k + R_r u_k <= T_r (closed regions, exact MLD,
 *     i.e. no strictness epsilon) and x_{k+1} = A_r x_k + B_r u_k + c_r; x_0 = state (IC).
 *   - cost / constraints of LocalMpcMld.setup_cost_and_constraints (fleet_decent_mld.py:61-208):
 *     front/back/leader tracking with the spacing policy (misc/spacing_policy.py:14-37),
 *     Q_u u^2, Q_du (du)^2, w (s_f + s_b); accel rows with tightening (:172-188); soft safe
 *     distance rows (:190-208); s >= 0 and s == 0 for the front / trailer vehicle (:100-105).
 *     min_2_norm (x' Q x) or min_1_norm (sum_i Q_ii |x_i|, diagonal Q) [EXT].
 *   - MpcMld.solve_mpc -> Gurobi MIQP optimum [EXT]: restated as  min over region sequences
 *     sigma of the convex QP with sigma fixed (exact: the MLD big-M model with delta fixed IS
 *     that QP).  Sequences are enumerated depth-first in lexicographic order; a sequence is
 *     kept when the velocity constraints admit a trajectory, decided per step by an exact 2-D
 *     vertex enumeration of the (v_k, v_{k+1}) polygon.  Ties (costs within 1e-9 relative)
 *     go to the lexicographically smallest sequence.
 *
 * Independent of the product kernel on purpose: the QP here is posed in the full (x, u, s)
 * space with the dynamics as equality constraints and assembled term by term from the
 * reference's expressions; it is solved by a dense Mehrotra primal-dual interior point method
 * with LU-factored KKT systems, then polished on the identified active set and certified by
 * its KKT conditions.  The product condenses to velocity space and runs a structured IPM.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define OR_MAX_N 16
#define OR_MAX_REG 16
#define OR_MAX_NZ 264
#define OR_MAX_EQ 128
#define OR_MAX_M 760
#define OR_MAX_KKT (OR_MAX_NZ + OR_MAX_EQ + OR_MAX_M)
#define OR_BIG 1e6

/* ------------------------------------------------------------------ model description */
typedef struct {
    int nreg, nsr, nd, nf;
    double S[OR_MAX_REG][4][2], R[OR_MAX_REG][4], T[OR_MAX_REG][4];
    double A[OR_MAX_REG][2][2], B[OR_MAX_REG][2], c[OR_MAX_REG][2];
    double D[8][2], E[8], F[4], G[4];
} or_model;

typedef struct {
    int N;
    int quadratic;
    double Qx[2][2], Qu, Qdu, w, a_acc, a_dec, ts, d_safe, tight, d0, t0;
    int role; /* HVP_ROLE_* bits, see include/hvp.h */
    /* naive ADMM local problem (fleet_naive_admm.py:24-253): the neighbour trajectories are
     * decision variables (copies) with ADMM terms; y/z blocks (2, N+1) replace xf / xb */
    int admm;
    double rho;
    const double *yf, *zf, *yb, *zb;
    /* switching-ADMM local problem of fleet_g_admm.LocalMpc (fleet_g_admm.py:22-205): on top of
     * the copies, the OWN state enters the augmented Lagrangian (MpcAdmm augmented state [EXT]:
     * y_own'(x - z_own) + rho/2 |x - z_own|^2, k = 0..N); the back copy is priced by its ADMM
     * term only (the cost tracks the front copy only, :136-158; safety only w.r.t. the front
     * copy, :98-109). */
    int gadmm, back_copy;
    const double *yo, *zo;
} or_cfg;

enum { R_SF = 1, R_SB = 2, R_TF = 4, R_TB = 8, R_TL = 16, R_LSP = 32 };

/* ------------------------------------------------------------------ linear expressions */
typedef struct {
    int n;
    int idx[8];
    double cf[8];
    double cst;
} lin;

static lin lin_const(double c) { lin e; e.n = 0; e.cst = c; return e; }
static void lin_add(lin* e, int idx, double cf) {
    if (cf == 0.0) return;
    for (int i = 0; i < e->n; ++i)
        if (e->idx[i] == idx) { e->cf[i] += cf; return; }
    e->idx[e->n] = idx; e->cf[e->n] = cf; e->n++;
}
static lin lin_axpy(double a, const lin* x, const lin* y) { /* a*x + y */
    lin r = *y;
    for (int i = 0; i < x->n; ++i) lin_add(&r, x->idx[i], a * x->cf[i]);
    r.cst += a * x->cst;
    return r;
}

/* ------------------------------------------------------------------ QP container */
typedef struct {
    int nz, neq, m;
    double P[OR_MAX_NZ][OR_MAX_NZ];
    double q[OR_MAX_NZ];
    double r0;
    double Aeq[OR_MAX_EQ][OR_MAX_NZ], beq[OR_MAX_EQ];
    double G[OR_MAX_M][OR_MAX_NZ], h[OR_MAX_M];
    int infeasible_const; /* a variable-free row was violated */
    int reg_row[OR_MAX_N][4]; /* inequality index of region row (k, row), -1 if variable-free */
} or_qp;

static void qp_add_prod(or_qp* qp, double wgt, const lin* a, const lin* b) { /* wgt * a * b */
    for (int i = 0; i < a->n; ++i)
        for (int j = 0; j < b->n; ++j) {
            double v = wgt * a->cf[i] * b->cf[j];
            qp->P[a->idx[i]][b->idx[j]] += v;
            qp->P[b->idx[j]][a->idx[i]] += v;
        }
    for (int i = 0; i < a->n; ++i) qp->q[a->idx[i]] += wgt * a->cf[i] * b->cst;
    for (int j = 0; j < b->n; ++j) qp->q[b->idx[j]] += wgt * b->cf[j] * a->cst;
    qp->r0 += wgt * a->cst * b->cst;
}
static void qp_add_lin(or_qp* qp, const lin* a) {
    for (int i = 0; i < a->n; ++i) qp->q[a->idx[i]] += a->cf[i];
    qp->r0 += a->cst;
}
static void qp_add_le(or_qp* qp, const lin* e, double rhs) { /* e <= rhs */
    if (e->n == 0) {
        if (e->cst > rhs + 1e-9 * (1.0 + fabs(rhs))) qp->infeasible_const = 1;
        return;
    }
    int r = qp->m++;
    memset(qp->G[r], 0, sizeof(double) * OR_MAX_NZ);
    for (int i = 0; i < e->n; ++i) qp->G[r][e->idx[i]] += e->cf[i];
    qp->h[r] = rhs - e->cst;
}
static void qp_add_eq(or_qp* qp, const lin* e, double rhs) { /* e == rhs */
    int r = qp->neq++;
    memset(qp->Aeq[r], 0, sizeof(double) * OR_MAX_NZ);
    for (int i = 0; i < e->n; ++i) qp->Aeq[r][e->idx[i]] += e->cf[i];
    qp->beq[r] = rhs - e->cst;
}

/* ------------------------------------------------------------------ problem assembly */
typedef struct {
    int N, nx_idx, nu_idx, nsf_idx, nsb_idx, naux;
    const double *x0, *xf, *xb, *xl; /* (2, N+1) row-major */
} or_layout;

/* state component i of x_k as an expression (x_0 is the fixed initial state) */
static lin X(const or_layout* L, int k, int i) {
    if (k == 0) return lin_const(L->x0[i]);
    lin e = lin_const(0.0);
    lin_add(&e, L->nx_idx + 2 * (k - 1) + i, 1.0);
    return e;
}
static lin U(const or_layout* L, int k) {
    lin e = lin_const(0.0);
    lin_add(&e, L->nu_idx + k, 1.0);
    return e;
}
static double par(const double* M, int N, int i, int k) { return M[i * (N + 1) + k]; }

/* sum_ij Q_ij e_i e_j  (min_2_norm)  or  sum_i Q_ii |e_i|  (min_1_norm, via aux >= +-Q_ii e_i) */
static void add_norm(or_qp* qp, or_layout* L, const or_cfg* cf, const lin e[2], const double Q[2][2],
                     int dim) {
    if (cf->quadratic) {
        for (int i = 0; i < dim; ++i)
            for (int j = 0; j < dim; ++j)
                if (Q[i][j] != 0.0) qp_add_prod(qp, Q[i][j], &e[i], &e[j]);
        return;
    }
    for (int i = 0; i < dim; ++i) {
        int a = L->nsb_idx + L->naux++;
        lin y = lin_const(0.0);
        lin_add(&y, a, 1.0);
        lin pos = lin_axpy(Q[i][i], &e[i], &(lin){.n = 0, .cst = 0.0}); /* Q_ii e_i */
        lin t1 = lin_axpy(-1.0, &y, &pos);                          /* Q e - y <= 0 */
        qp_add_le(qp, &t1, 0.0);
        lin neg = lin_axpy(-1.0, &pos, &(lin){.n = 0, .cst = 0.0});
        lin t2 = lin_axpy(-1.0, &y, &neg); /* -Q e - y <= 0 */
        qp_add_le(qp, &t2, 0.0);
        qp_add_lin(qp, &y);
    }
}

/* Builds the fixed-sigma QP. Returns number of variables (0 on layout overflow).
 * K < N builds the branch-and-bound RELAXATION of the prefix sigma_0..sigma_{K-1}: for steps
 * k >= K the region is free, so the region-dependent rows are dropped -- the velocity row of the
 * dynamics, the region rows S x_k + R u_k <= T and the input cost -- while the position row of
 * the dynamics (identical in every region, checked by oracle_bnb_ok), the state box, the
 * acceleration rows and all tracking / slack terms stay.  Its optimum bounds every completion of
 * the prefix from below. */
static int build_qp_k(or_qp* qp, const or_model* md, const or_cfg* cf, const int* sigma, int K, const double* x0,
                      const double* xf, const double* xb, const double* xl);
static int build_qp(or_qp* qp, const or_model* md, const or_cfg* cf, const int* sigma, const double* x0,
                    const double* xf, const double* xb, const double* xl) {
    return build_qp_k(qp, md, cf, sigma, cf->N, x0, xf, xb, xl);
}
static int build_qp_k(or_qp* qp, const or_model* md, const or_cfg* cf, const int* sigma, int K, const double* x0,
                      const double* xf, const double* xb, const double* xl) {
    const int N = cf->N;
    or_layout L;
    L.N = N; L.x0 = x0; L.xf = xf; L.xb = xb; L.xl = xl;
    L.nx_idx = 0;
    L.nu_idx = 2 * N;
    int nz = 3 * N;
    L.nsf_idx = nz;
    if (cf->role & R_SF) nz += N + 1;
    int sb0 = nz;
    if (cf->role & R_SB) nz += N + 1;
    int cf_idx = -1, cb_idx = -1; /* ADMM copies x_front, x_back (2, N+1), fleet_naive_admm.py:84-102 */
    if (cf->admm) {
        if (cf->role & R_SF) { cf_idx = nz; nz += 2 * (N + 1); }
        if ((cf->role & R_SB) || cf->back_copy) { cb_idx = nz; nz += 2 * (N + 1); }
    }
    L.nsb_idx = nz; /* aux (L1) variables are appended after the slacks (and copies) */
    L.naux = 0;
    int aux_needed = cf->quadratic ? 0 : (N + 1) * 2 * 3 + N * 2;
    if (nz + aux_needed > OR_MAX_NZ) return 0;
    memset(qp->P, 0, sizeof(qp->P));
    memset(qp->q, 0, sizeof(qp->q));
    qp->r0 = 0.0; qp->neq = 0; qp->m = 0; qp->infeasible_const = 0;

    /* dynamics of the selected region (MLD with delta fixed) */
    for (int k = 0; k < N; ++k) {
        int r = k < K ? sigma[k] : 0;
        for (int i = 0; i < (k < K ? 2 : 1); ++i) {
            lin e = X(&L, k + 1, i);
            for (int j = 0; j < 2; ++j) { lin xj = X(&L, k, j); e = lin_axpy(-md->A[r][i][j], &xj, &e); }
            lin uk = U(&L, k);
            e = lin_axpy(-md->B[r][i], &uk, &e);
            qp_add_eq(qp, &e, md->c[r][i]);
        }
    }
    /* region rows S x_k + R u_k <= T (k = 0..N-1) */
    for (int k = 0; k < OR_MAX_N; ++k)
        for (int row = 0; row < 4; ++row) qp->reg_row[k][row] = -1;
    for (int k = 0; k < K; ++k) {
        int r = sigma[k];
        for (int row = 0; row < md->nsr; ++row) {
            lin e = lin_const(0.0);
            for (int j = 0; j < 2; ++j) { lin xj = X(&L, k, j); e = lin_axpy(md->S[r][row][j], &xj, &e); }
            lin uk = U(&L, k);
            e = lin_axpy(md->R[r][row], &uk, &e);
            const int m0 = qp->m;
            qp_add_le(qp, &e, md->T[r][row]);
            if (qp->m > m0) qp->reg_row[k][row] = m0;
        }
    }
    /* state box k = 1..N, input box k = 0..N-1 */
    for (int k = 1; k <= N; ++k)
        for (int row = 0; row < md->nd; ++row) {
            lin e = lin_const(0.0);
            for (int j = 0; j < 2; ++j) { lin xj = X(&L, k, j); e = lin_axpy(md->D[row][j], &xj, &e); }
            qp_add_le(qp, &e, md->E[row]);
        }
    for (int k = 0; k < N; ++k)
        for (int row = 0; row < md->nf; ++row) {
            lin uk = U(&L, k);
            lin e = lin_axpy(md->F[row], &uk, &(lin){.n = 0, .cst = 0.0});
            qp_add_le(qp, &e, md->G[row]);
        }
    /* acceleration rows: a_dec*ts <= v_{k+1}-v_k - k*tight ; v_{k+1}-v_k <= a_acc*ts - k*tight */
    for (int k = 0; k < N; ++k) {
        lin v1 = X(&L, k + 1, 1), v0 = X(&L, k, 1);
        lin dv = lin_axpy(-1.0, &v0, &v1);
        lin ndv = lin_axpy(-1.0, &dv, &(lin){.n = 0, .cst = 0.0});
        qp_add_le(qp, &ndv, -(cf->a_dec * cf->ts) - k * cf->tight);
        qp_add_le(qp, &dv, cf->a_acc * cf->ts - k * cf->tight);
    }
    /* slacks: s >= 0 and the soft safe-distance rows */
    for (int k = 0; k <= N; ++k) {
        lin pk = X(&L, k, 0);
        if (cf->role & R_SF) {
            lin s = lin_const(0.0);
            lin_add(&s, L.nsf_idx + k, 1.0);
            lin ns = lin_axpy(-1.0, &s, &(lin){.n = 0, .cst = 0.0});
            qp_add_le(qp, &ns, 0.0);
            lin e = lin_axpy(-1.0, &s, &pk); /* p_k - s_f <= pf_k - d_safe */
            if (cf->admm) { /* pf_k is the copy's position (fleet_naive_admm.py:217-226) */
                lin_add(&e, cf_idx + k, -1.0);
                qp_add_le(qp, &e, -cf->d_safe);
            } else
            qp_add_le(qp, &e, par(xf, N, 0, k) - cf->d_safe);
            lin ws = lin_axpy(cf->w, &s, &(lin){.n = 0, .cst = 0.0});
            qp_add_lin(qp, &ws);
        }
        if (cf->role & R_SB) {
            lin s = lin_const(0.0);
            lin_add(&s, sb0 + k, 1.0);
            lin ns = lin_axpy(-1.0, &s, &(lin){.n = 0, .cst = 0.0});
            qp_add_le(qp, &ns, 0.0);
            lin e = lin_axpy(-1.0, &pk, &ns); /* -p_k - s_b <= -(pb_k + d_safe) */
            if (cf->admm) { /* (:227-236) */
                lin_add(&e, cb_idx + k, 1.0);
                qp_add_le(qp, &e, -cf->d_safe);
            } else
            qp_add_le(qp, &e, -(par(xb, N, 0, k) + cf->d_safe));
            lin ws = lin_axpy(cf->w, &s, &(lin){.n = 0, .cst = 0.0});
            qp_add_lin(qp, &ws);
        }
    }
    /* tracking costs, k = 0..N */
    for (int k = 0; k <= N; ++k) {
        lin p = X(&L, k, 0), v = X(&L, k, 1);
        lin e[2];
        if (cf->role & R_TF) { /* x_k - xf_k - spacing(x_k) ; spacing(x) = [-d0 - t0 v, 0] */
            e[0] = lin_axpy(cf->t0, &v, &p);
            e[0].cst += cf->d0;
            e[1] = v;
            if (cf->admm) { lin_add(&e[0], cf_idx + k, -1.0); lin_add(&e[1], cf_idx + N + 1 + k, -1.0); }
            else { e[0].cst -= par(xf, N, 0, k); e[1].cst -= par(xf, N, 1, k); }
            add_norm(qp, &L, cf, e, cf->Qx, 2);
        }
        if (cf->role & R_TB) { /* xb_k - x_k - spacing(xb_k) */
            if (cf->admm) {
                e[0] = lin_axpy(-1.0, &p, &(lin){.n = 0, .cst = cf->d0});
                lin_add(&e[0], cb_idx + k, 1.0);
                lin_add(&e[0], cb_idx + N + 1 + k, cf->t0);
                e[1] = lin_axpy(-1.0, &v, &(lin){.n = 0, .cst = 0.0});
                lin_add(&e[1], cb_idx + N + 1 + k, 1.0);
            } else {
                double pb = par(xb, N, 0, k), vb = par(xb, N, 1, k);
                e[0] = lin_axpy(-1.0, &p, &(lin){.n = 0, .cst = pb + cf->d0 + cf->t0 * vb});
                e[1] = lin_axpy(-1.0, &v, &(lin){.n = 0, .cst = vb});
            }
            add_norm(qp, &L, cf, e, cf->Qx, 2);
        }
        if (cf->admm) { /* y'(c - z) + rho/2 |c - z|^2 per copy (fleet_naive_admm.py:172-198) */
            const int idx[2] = {cf_idx, cb_idx};
            const double* yy[2] = {cf->yf, cf->yb};
            const double* zz[2] = {cf->zf, cf->zb};
            for (int side = 0; side < 2; ++side) {
                if (idx[side] < 0) continue;
                for (int i = 0; i < 2; ++i) {
                    lin d = lin_const(-par(zz[side], N, i, k));
                    lin_add(&d, idx[side] + i * (N + 1) + k, 1.0);
                    qp_add_prod(qp, 0.5 * cf->rho, &d, &d);
                    lin yd = lin_axpy(par(yy[side], N, i, k), &d, &(lin){.n = 0, .cst = 0.0});
                    qp_add_lin(qp, &yd);
                }
            }
        }
        if (cf->gadmm) { /* own state in the augmented Lagrangian: y_own'(x_k - z_k) + rho/2 |x_k - z_k|^2 */
            lin xs[2] = {p, v};
            for (int i = 0; i < 2; ++i) {
                lin d = xs[i];
                d.cst -= par(cf->zo, N, i, k);
                qp_add_prod(qp, 0.5 * cf->rho, &d, &d);
                lin yd = lin_axpy(par(cf->yo, N, i, k), &d, &(lin){.n = 0, .cst = 0.0});
                qp_add_lin(qp, &yd);
            }
        }
        if (cf->role & R_TL) { /* x_k - xl_k (- spacing(x_k) for real_vehicle_as_reference) */
            if (cf->role & R_LSP) { e[0] = lin_axpy(cf->t0, &v, &p); e[0].cst += cf->d0; }
            else e[0] = p;
            e[0].cst -= par(xl, N, 0, k);
            e[1] = v; e[1].cst -= par(xl, N, 1, k);
            add_norm(qp, &L, cf, e, cf->Qx, 2);
        }
    }
    /* control effort and variation */
    double Qu[2][2] = {{cf->Qu, 0}, {0, 0}}, Qdu[2][2] = {{cf->Qdu, 0}, {0, 0}};
    for (int k = 0; k < K; ++k) {
        lin e[2]; e[0] = U(&L, k); e[1] = lin_const(0.0);
        add_norm(qp, &L, cf, e, Qu, 1);
    }
    for (int k = 0; k + 1 < K; ++k) {
        lin e[2];
        lin a = U(&L, k + 1), b = U(&L, k);
        e[0] = lin_axpy(-1.0, &b, &a); e[1] = lin_const(0.0);
        if (cf->Qdu != 0.0) add_norm(qp, &L, cf, e, Qdu, 1);
    }
    qp->nz = L.nsb_idx + L.naux;
    return qp->nz;
}

/* ------------------------------------------------------------------ dense LU */
static int lu_factor(int n, double* M, int ld, int* piv) {
    double big = 0.0;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) big = fmax(big, fabs(M[i * ld + j]));
    if (big == 0.0) return -1;
    for (int k = 0; k < n; ++k) {
        int p = k;
        double mx = fabs(M[k * ld + k]);
        for (int i = k + 1; i < n; ++i)
            if (fabs(M[i * ld + k]) > mx) { mx = fabs(M[i * ld + k]); p = i; }
        piv[k] = p;
        if (mx <= 1e-300 * big || !isfinite(mx)) return -1;
        if (p != k)
            for (int j = 0; j < n; ++j) { double t = M[k * ld + j]; M[k * ld + j] = M[p * ld + j]; M[p * ld + j] = t; }
        double inv = 1.0 / M[k * ld + k];
        for (int i = k + 1; i < n; ++i) {
            double f = M[i * ld + k] * inv;
            M[i * ld + k] = f;
            if (f != 0.0)
                for (int j = k + 1; j < n; ++j) M[i * ld + j] -= f * M[k * ld + j];
        }
    }
    return 0;
}
static void lu_solve(int n, const double* M, int ld, const int* piv, double* x) {
    for (int k = 0; k < n; ++k)
        if (piv[k] != k) { double t = x[k]; x[k] = x[piv[k]]; x[piv[k]] = t; }
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < i; ++j) x[i] -= M[i * ld + j] * x[j];
    for (int i = n - 1; i >= 0; --i) {
        for (int j = i + 1; j < n; ++j) x[i] -= M[i * ld + j] * x[j];
        x[i] /= M[i * ld + i];
    }
}

/* ------------------------------------------------------------------ IPM */
typedef struct {
    double z[OR_MAX_NZ], nu[OR_MAX_EQ], lam[OR_MAX_M], t[OR_MAX_M];
    double K[OR_MAX_KKT * OR_MAX_KKT];
    int piv[OR_MAX_KKT];
    double rhs[OR_MAX_KKT];
} or_work;

static double vmaxabs(const double* v, int n) {
    double m = 0.0;
    for (int i = 0; i < n; ++i) m = fmax(m, fabs(v[i]));
    return m;
}
static double objective(const or_qp* qp, const double* z) {
    double f = qp->r0;
    for (int i = 0; i < qp->nz; ++i) {
        double pz = 0.0;
        for (int j = 0; j < qp->nz; ++j) pz += qp->P[i][j] * z[j];
        f += 0.5 * z[i] * pz + qp->q[i] * z[i];
    }
    return f;
}

/* Solves the KKT system [[P + G'DG, A'], [A, 0]] [dz; dnu] = rhs ; factorises once per call. */
static int ipm_factor(const or_qp* qp, or_work* w, const double* d) {
    const int nz = qp->nz, ne = qp->neq, n = nz + ne, ld = n;
    for (int i = 0; i < nz; ++i)
        for (int j = 0; j < nz; ++j) w->K[i * ld + j] = qp->P[i][j];
    for (int r = 0; r < qp->m; ++r) {
        const double* g = qp->G[r];
        for (int i = 0; i < nz; ++i) {
            if (g[i] == 0.0) continue;
            double gi = d[r] * g[i];
            for (int j = 0; j < nz; ++j) w->K[i * ld + j] += gi * g[j];
        }
    }
    for (int e = 0; e < ne; ++e)
        for (int j = 0; j < nz; ++j) { w->K[(nz + e) * ld + j] = qp->Aeq[e][j]; w->K[j * ld + nz + e] = qp->Aeq[e][j]; }
    for (int e = 0; e < ne; ++e)
        for (int f = 0; f < ne; ++f) w->K[(nz + e) * ld + nz + f] = 0.0;
    return lu_factor(n, w->K, ld, w->piv);
}

/* Newton direction for residuals (rd, re, rp, rc). Outputs dz, dnu, dlam, dt. */
static void ipm_direction(const or_qp* qp, or_work* w, const double* d, const double* rd, const double* re,
                          const double* rp, const double* rc, double* dz, double* dnu, double* dl, double* dt) {
    const int nz = qp->nz, ne = qp->neq, m = qp->m;
    double tmp[OR_MAX_M];
    for (int i = 0; i < m; ++i) tmp[i] = d[i] * rp[i] - rc[i] / w->t[i];
    for (int j = 0; j < nz; ++j) {
        double s = -rd[j];
        for (int i = 0; i < m; ++i) s -= qp->G[i][j] * tmp[i];
        w->rhs[j] = s;
    }
    for (int e = 0; e < ne; ++e) w->rhs[nz + e] = -re[e];
    lu_solve(nz + ne, w->K, nz + ne, w->piv, w->rhs);
    for (int j = 0; j < nz; ++j) dz[j] = w->rhs[j];
    for (int e = 0; e < ne; ++e) dnu[e] = w->rhs[nz + e];
    for (int i = 0; i < m; ++i) {
        double gdz = 0.0;
        for (int j = 0; j < nz; ++j) gdz += qp->G[i][j] * dz[j];
        dl[i] = d[i] * (gdz + rp[i]) - rc[i] / w->t[i];
        dt[i] = -rp[i] - gdz;
    }
}

static double max_step(const double* v, const double* dv, int n) {
    double a = 1.0;
    for (int i = 0; i < n; ++i)
        if (dv[i] < 0.0) a = fmin(a, -v[i] / dv[i]);
    return a;
}

typedef struct {
    int converged, certified, iters;
    double obj;
} or_result;

static void residuals(const or_qp* qp, const or_work* w, double* rd, double* re, double* rp) {
    for (int j = 0; j < qp->nz; ++j) {
        double s = qp->q[j];
        for (int k = 0; k < qp->nz; ++k) s += qp->P[j][k] * w->z[k];
        for (int e = 0; e < qp->neq; ++e) s += qp->Aeq[e][j] * w->nu[e];
        for (int i = 0; i < qp->m; ++i) s += qp->G[i][j] * w->lam[i];
        rd[j] = s;
    }
    for (int e = 0; e < qp->neq; ++e) {
        double s = -qp->beq[e];
        for (int j = 0; j < qp->nz; ++j) s += qp->Aeq[e][j] * w->z[j];
        re[e] = s;
    }
    for (int i = 0; i < qp->m; ++i) {
        double s = w->t[i] - qp->h[i];
        for (int j = 0; j < qp->nz; ++j) s += qp->G[i][j] * w->z[j];
        rp[i] = s;
    }
}

/* Active-set polish: solve the equality QP on a guessed active set (rows with lam > t), then
 * correct the guess -- drop the row with the most negative multiplier, or add the most
 * violated inactive row -- until the solution is primal and dual feasible.  It then satisfies
 * the KKT conditions exactly (certificate of global optimality for the convex QP).  Degenerate
 * vertices (dependent active rows, weakly active rows) are what the correction steps are for. */
static int polish(const or_qp* qp, or_work* w) {
    const int nz = qp->nz, ne = qp->neq, m = qp->m;
    int inA[OR_MAX_M];
    for (int i = 0; i < m; ++i) inA[i] = w->lam[i] > w->t[i];
    const double scale_h = 1.0 + vmaxabs(qp->h, m), scale_l = 1.0 + vmaxabs(w->lam, m);
    for (int round = 0; round < 3 * OR_MAX_N + 10; ++round) {
        int act[OR_MAX_M], na = 0;
        for (int i = 0; i < m; ++i)
            if (inA[i]) act[na++] = i;
        const int n = nz + ne + na, ld = n;
        if (n > OR_MAX_KKT) return 0;
        /* quasi-definite regularisation (+delta on the primal block, -delta on the multiplier
         * rows) keeps the factorisation defined for dependent active rows; iterative refinement
         * against the unregularised system then converges to an exact solution when the system
         * is consistent (degenerate vertex) */
        const double delta = 1e-10;
        double* K = w->K;
        memset(K, 0, sizeof(double) * (size_t)n * (size_t)n);
        for (int i = 0; i < nz; ++i)
            for (int j = 0; j < nz; ++j) K[i * ld + j] = qp->P[i][j] + (i == j ? delta : 0.0);
        for (int e = 0; e < ne; ++e)
            for (int j = 0; j < nz; ++j) { K[(nz + e) * ld + j] = qp->Aeq[e][j]; K[j * ld + nz + e] = qp->Aeq[e][j]; }
        for (int a = 0; a < na; ++a)
            for (int j = 0; j < nz; ++j) {
                K[(nz + ne + a) * ld + j] = qp->G[act[a]][j];
                K[j * ld + nz + ne + a] = qp->G[act[a]][j];
            }
        for (int i = nz; i < n; ++i) K[i * ld + i] = -delta;
        if (lu_factor(n, K, ld, w->piv) != 0) return 0;
        double x[OR_MAX_KKT], r[OR_MAX_KKT];
        for (int i = 0; i < n; ++i) x[i] = 0.0;
        for (int ref = 0; ref < 60; ++ref) {
            /* r = rhs - K0 x with K0 the unregularised KKT matrix */
            double rn = 0.0;
            for (int j = 0; j < nz; ++j) {
                double s = -qp->q[j];
                for (int k = 0; k < nz; ++k) s -= qp->P[j][k] * x[k];
                for (int e = 0; e < ne; ++e) s -= qp->Aeq[e][j] * x[nz + e];
                for (int a = 0; a < na; ++a) s -= qp->G[act[a]][j] * x[nz + ne + a];
                r[j] = s;
                rn = fmax(rn, fabs(s));
            }
            for (int e = 0; e < ne; ++e) {
                double s = qp->beq[e];
                for (int j = 0; j < nz; ++j) s -= qp->Aeq[e][j] * x[j];
                r[nz + e] = s;
                rn = fmax(rn, fabs(s));
            }
            for (int a = 0; a < na; ++a) {
                double s = qp->h[act[a]];
                for (int j = 0; j < nz; ++j) s -= qp->G[act[a]][j] * x[j];
                r[nz + ne + a] = s;
                rn = fmax(rn, fabs(s));
            }
            if (rn <= 1e-15 * scale_h) break;
            lu_solve(n, K, ld, w->piv, r);
            for (int i = 0; i < n; ++i) x[i] += r[i];
        }
        /* the certificate checks the computed KKT residuals, not the solve: stationarity,
         * equality rows and active rows at equality (a near-singular system fails here) */
        double kkt = 0.0, sq = 1.0 + vmaxabs(qp->q, nz);
        for (int j = 0; j < nz; ++j) {
            double s = qp->q[j];
            for (int k = 0; k < nz; ++k) s += qp->P[j][k] * x[k];
            for (int e = 0; e < ne; ++e) s += qp->Aeq[e][j] * x[nz + e];
            for (int a = 0; a < na; ++a) s += qp->G[act[a]][j] * x[nz + ne + a];
            kkt = fmax(kkt, fabs(s) / sq);
        }
        for (int e = 0; e < ne; ++e) {
            double s = -qp->beq[e];
            for (int j = 0; j < nz; ++j) s += qp->Aeq[e][j] * x[j];
            kkt = fmax(kkt, fabs(s) / scale_h);
        }
        for (int a = 0; a < na; ++a) {
            double s = -qp->h[act[a]];
            for (int j = 0; j < nz; ++j) s += qp->G[act[a]][j] * x[j];
            kkt = fmax(kkt, fabs(s) / scale_h);
        }
        if (!(kkt <= 1e-9)) {
            int worst = -1;
            for (int a = 0; a < na; ++a)
                if (worst < 0 || w->lam[act[a]] < w->lam[act[worst]]) worst = a;
            if (worst < 0) return 0;
            inA[act[worst]] = 0;
            continue;
        }
        int neg = -1;
        double negv = -1e-9 * scale_l;
        for (int a = 0; a < na; ++a)
            if (x[nz + ne + a] < negv) { negv = x[nz + ne + a]; neg = a; }
        if (neg >= 0) {
            inA[act[neg]] = 0;
            continue;
        }
        int vio = -1;
        double viov = 1e-9 * scale_h;
        for (int i = 0; i < m; ++i) {
            if (inA[i]) continue;
            double g = -qp->h[i];
            for (int j = 0; j < nz; ++j) g += qp->G[i][j] * x[j];
            if (g > viov) { viov = g; vio = i; }
        }
        if (vio >= 0) {
            inA[vio] = 1;
            continue;
        }
        for (int j = 0; j < nz; ++j) w->z[j] = x[j];
        for (int i = 0; i < m; ++i) w->lam[i] = 0.0; /* multipliers of the certified active set */
        for (int a = 0; a < na; ++a) w->lam[act[a]] = x[nz + ne + a];
        return 1;
    }
    return 0;
}

static or_result ipm_solve(const or_qp* qp, or_work* w, int maxit) {
    const int nz = qp->nz, ne = qp->neq, m = qp->m;
    double rd[OR_MAX_NZ], re[OR_MAX_EQ], rp[OR_MAX_M], rc[OR_MAX_M], d[OR_MAX_M];
    double dz[OR_MAX_NZ], dnu[OR_MAX_EQ], dl[OR_MAX_M], dt[OR_MAX_M];
    double dza[OR_MAX_NZ], dnua[OR_MAX_EQ], dla[OR_MAX_M], dta[OR_MAX_M];
    or_result res = {0, 0, 0, 0.0};
    /* initial point (CVXOPT-style): minimise 1/2 z'Pz + q'z + 1/2 |h - Gz|^2 s.t. Az = b, then
     * t = h - Gz, lam = -t, both shifted into the interior (Mehrotra's heuristic). */
    for (int i = 0; i < m; ++i) d[i] = 1.0;
    if (ipm_factor(qp, w, d) != 0) return res;
    for (int j = 0; j < nz; ++j) {
        double s = -qp->q[j];
        for (int i = 0; i < m; ++i) s += qp->G[i][j] * qp->h[i];
        w->rhs[j] = s;
    }
    for (int e = 0; e < ne; ++e) w->rhs[nz + e] = qp->beq[e];
    lu_solve(nz + ne, w->K, nz + ne, w->piv, w->rhs);
    for (int j = 0; j < nz; ++j) w->z[j] = w->rhs[j];
    for (int e = 0; e < ne; ++e) w->nu[e] = w->rhs[nz + e];
    {
        double tmin = INFINITY, lmin = INFINITY;
        for (int i = 0; i < m; ++i) {
            double g = 0.0;
            for (int j = 0; j < nz; ++j) g += qp->G[i][j] * w->z[j];
            w->t[i] = qp->h[i] - g;
            w->lam[i] = -w->t[i];
            tmin = fmin(tmin, w->t[i]);
            lmin = fmin(lmin, w->lam[i]);
        }
        double st = fmax(-1.5 * tmin, 0.0), sl = fmax(-1.5 * lmin, 0.0), tl = 0.0, ssum = 0.0, lsum = 0.0;
        for (int i = 0; i < m; ++i) { w->t[i] += st; w->lam[i] += sl; }
        for (int i = 0; i < m; ++i) { tl += w->t[i] * w->lam[i]; ssum += w->t[i]; lsum += w->lam[i]; }
        double dt0 = lsum > 0 ? 0.5 * tl / lsum : 1.0, dl0 = ssum > 0 ? 0.5 * tl / ssum : 1.0;
        for (int i = 0; i < m; ++i) {
            w->t[i] += dt0; w->lam[i] += dl0;
            if (!(w->t[i] > 0)) w->t[i] = 1.0;
            if (!(w->lam[i] > 0)) w->lam[i] = 1.0;
        }
    }
    double sq = 1.0 + vmaxabs(qp->q, nz), sb = 1.0 + vmaxabs(qp->beq, ne), sh = 1.0 + vmaxabs(qp->h, m);
    for (int it = 0; it < maxit; ++it) {
        residuals(qp, w, rd, re, rp);
        double mu = 0.0;
        for (int i = 0; i < m; ++i) mu += w->lam[i] * w->t[i];
        double gap = mu;
        mu /= (m > 0 ? m : 1);
        double obj = objective(qp, w->z);
        res.iters = it;
        const double rdn = vmaxabs(rd, nz), ren = vmaxabs(re, ne), rpn = vmaxabs(rp, m);
        if (rdn <= 1e-10 * sq && ren <= 1e-10 * sb && rpn <= 1e-10 * sh && gap <= 1e-11 * fmax(1.0, fabs(obj))) {
            res.converged = 1;
            break;
        }
        /* Degenerate vertices (a row with t -> 0 and lam -> 0 together) make P + G'DG singular as
         * mu -> 0 and the residuals blow up again.  Near the optimum, try the active-set polish:
         * when it certifies the KKT conditions the solution is exact, whatever the IPM does next. */
        if (rdn <= 1e-7 * sq && ren <= 1e-7 * sb && rpn <= 1e-7 * sh && gap <= 1e-5 * fmax(1.0, fabs(obj))) {
            double zs[OR_MAX_NZ];
            memcpy(zs, w->z, sizeof(double) * nz);
            if (polish(qp, w)) {
                res.converged = 1;
                res.certified = 1;
                res.iters = it;
                res.obj = objective(qp, w->z);
                return res;
            }
            memcpy(w->z, zs, sizeof(double) * nz);
        }
        for (int i = 0; i < m; ++i) d[i] = w->lam[i] / w->t[i];
        if (ipm_factor(qp, w, d) != 0) break;
        /* predictor */
        for (int i = 0; i < m; ++i) rc[i] = w->lam[i] * w->t[i];
        ipm_direction(qp, w, d, rd, re, rp, rc, dza, dnua, dla, dta);
        double ap = max_step(w->t, dta, m), ad = max_step(w->lam, dla, m);
        double alpha = fmin(ap, ad);
        double mua = 0.0;
        for (int i = 0; i < m; ++i) mua += (w->lam[i] + alpha * dla[i]) * (w->t[i] + alpha * dta[i]);
        mua /= (m > 0 ? m : 1);
        double sigma = mu > 0 ? pow(mua / mu, 3.0) : 0.0;
        /* corrector */
        for (int i = 0; i < m; ++i) rc[i] = w->lam[i] * w->t[i] + dla[i] * dta[i] - sigma * mu;
        ipm_direction(qp, w, d, rd, re, rp, rc, dz, dnu, dl, dt);
        ap = max_step(w->t, dt, m);
        ad = max_step(w->lam, dl, m);
        alpha = fmin(1.0, 0.99 * fmin(ap, ad));
        for (int j = 0; j < nz; ++j) w->z[j] += alpha * dz[j];
        for (int e = 0; e < ne; ++e) w->nu[e] += alpha * dnu[e];
        for (int i = 0; i < m; ++i) { w->lam[i] += alpha * dl[i]; w->t[i] += alpha * dt[i]; }
        res.iters = it + 1;
    }
    if (res.converged) {
        res.certified = polish(qp, w);
    } else if (polish(qp, w)) {
        res.converged = 1;  /* certified by the KKT check even though the IPM stalled */
        res.certified = 1;
    }
    res.obj = objective(qp, w->z);
    return res;
}

/* Exact copies of the min_1_norm naive-ADMM local problem for a given own trajectory (TEST
 * INFRASTRUCTURE restatement).  Each (side, step) copy c = (c_p, c_v) minimises
 *   rho/2 |c - m|^2 + sum_j phi_j(a_j . c + b_j),  m = z - y/rho  (y'(c - z) + rho/2 |c - z|^2, :172-198),
 * phi_j(e) = wp_j max(e, 0) + wn_j max(-e, 0): the L1 tracking terms Q_ii |e_i| of the copy
 * (:110-133) and the soft safe row w max(0, .) on its position (:205-236).  The interior point's copy
 * stops ~1e-9 away from a kink of the w = 1e4 safe row, which moves the priced objective by ~1e-5;
 * the exact minimiser is one of the stationary points of the 3^3 kink patterns (each term strictly
 * positive, strictly negative or at its kink), so every pattern's point is evaluated and the best
 * kept.  Used for the objective and the returned copies of the L1 form only. */
static double prox_obj(double rho, const double* m, int nt, const double (*a)[2], const double* b, const double* wp,
                       const double* wn, const double* c) {
    double f = 0.5 * rho * ((c[0] - m[0]) * (c[0] - m[0]) + (c[1] - m[1]) * (c[1] - m[1]));
    for (int j = 0; j < nt; ++j) {
        double e = a[j][0] * c[0] + a[j][1] * c[1] + b[j];
        f += e > 0.0 ? wp[j] * e : -wn[j] * e;
    }
    return f;
}

static void copy_prox(double rho, const double* m, int nt, const double (*a)[2], const double* b, const double* wp,
                      const double* wn, double* c) {
    int npat = 1;
    for (int j = 0; j < nt; ++j) npat *= 3;
    double best = INFINITY;
    c[0] = m[0]; c[1] = m[1];
    for (int pat = 0; pat < npat; ++pat) {
        int st[3], zs[3], nz = 0, q = pat;
        double g[2] = {0.0, 0.0};
        for (int j = 0; j < nt; ++j) {
            st[j] = q % 3; q /= 3; /* 0: at the kink, 1: e > 0, 2: e < 0 */
            if (st[j] == 0) zs[nz++] = j;
            else { double s = st[j] == 1 ? wp[j] : -wn[j]; g[0] += s * a[j][0]; g[1] += s * a[j][1]; }
        }
        if (nz > 2) continue;
        double c0[2] = {m[0] - g[0] / rho, m[1] - g[1] / rho}, cc[2] = {c0[0], c0[1]};
        if (nz == 1) {
            const double* aj = a[zs[0]];
            double aa = aj[0] * aj[0] + aj[1] * aj[1];
            if (!(aa > 0.0)) continue;
            double lam = rho * (aj[0] * c0[0] + aj[1] * c0[1] + b[zs[0]]) / aa;
            cc[0] = c0[0] - aj[0] * lam / rho; cc[1] = c0[1] - aj[1] * lam / rho;
        } else if (nz == 2) {
            const double *aj = a[zs[0]], *ak = a[zs[1]];
            double A00 = aj[0] * aj[0] + aj[1] * aj[1], A01 = aj[0] * ak[0] + aj[1] * ak[1];
            double A11 = ak[0] * ak[0] + ak[1] * ak[1], det = A00 * A11 - A01 * A01;
            if (!(fabs(det) > 1e-12 * (A00 * A11 + 1e-300))) continue;
            double r0 = rho * (aj[0] * c0[0] + aj[1] * c0[1] + b[zs[0]]), r1 = rho * (ak[0] * c0[0] + ak[1] * c0[1] + b[zs[1]]);
            double l0 = (A11 * r0 - A01 * r1) / det, l1 = (A00 * r1 - A01 * r0) / det;
            cc[0] = c0[0] - (aj[0] * l0 + ak[0] * l1) / rho; cc[1] = c0[1] - (aj[1] * l0 + ak[1] * l1) / rho;
        }
        double f = prox_obj(rho, m, nt, a, b, wp, wn, cc);
        if (f < best) { best = f; c[0] = cc[0]; c[1] = cc[1]; }
    }
}

/* overwrite the copies of the solution z (layout of build_qp_k) by their exact minimisers given
 * the own trajectory in z (naive ADMM, min_1_norm) */
static void admm_l1_exact_copies(const or_cfg* cf, const double* x0, double* z) {
    const int N = cf->N;
    int idx = 3 * N + ((cf->role & R_SF) ? N + 1 : 0) + ((cf->role & R_SB) ? N + 1 : 0);
    const double rho = cf->rho;
    for (int side = 0; side < 2; ++side) {
        if (!(cf->role & (side == 0 ? R_SF : R_SB))) continue;
        const int tr = (cf->role & (side == 0 ? R_TF : R_TB)) != 0;
        const double* yy = side == 0 ? cf->yf : cf->yb;
        const double* zz = side == 0 ? cf->zf : cf->zb;
        for (int k = 0; k <= N; ++k) {
            double p = k == 0 ? x0[0] : z[2 * (k - 1)], v = k == 0 ? x0[1] : z[2 * (k - 1) + 1];
            double a[3][2], b[3], wp[3], wn[3];
            int nt = 0;
            if (tr) {
                if (side == 0) { /* p + t0 v + d0 - c_p, v - c_v */
                    a[nt][0] = -1.0; a[nt][1] = 0.0; b[nt] = p + cf->t0 * v + cf->d0; wp[nt] = wn[nt] = fabs(cf->Qx[0][0]); nt++;
                    a[nt][0] = 0.0; a[nt][1] = -1.0; b[nt] = v; wp[nt] = wn[nt] = fabs(cf->Qx[1][1]); nt++;
                } else { /* c_p + t0 c_v + d0 - p, c_v - v */
                    a[nt][0] = 1.0; a[nt][1] = cf->t0; b[nt] = cf->d0 - p; wp[nt] = wn[nt] = fabs(cf->Qx[0][0]); nt++;
                    a[nt][0] = 0.0; a[nt][1] = 1.0; b[nt] = -v; wp[nt] = wn[nt] = fabs(cf->Qx[1][1]); nt++;
                }
            }
            /* w max(0, p - c_p + d_safe) (front) / w max(0, c_p + d_safe - p) (back) */
            a[nt][0] = side == 0 ? -1.0 : 1.0; a[nt][1] = 0.0; b[nt] = side == 0 ? p + cf->d_safe : cf->d_safe - p;
            wp[nt] = cf->w; wn[nt] = 0.0; nt++;
            double m[2] = {par(zz, N, 0, k) - par(yy, N, 0, k) / rho, par(zz, N, 1, k) - par(yy, N, 1, k) / rho}, c[2];
            copy_prox(rho, m, nt, (const double(*)[2])a, b, wp, wn, c);
            z[idx + k] = c[0];
            z[idx + N + 1 + k] = c[1];
        }
        idx += 2 * (N + 1);
    }
}

/* Objective evaluated term by term on the trajectory (the form of fleet_decent_mld.py:107-169):
 * sums of squared tracking errors, control terms and w * slack with the slacks at their optimal
 * value max(0, .).  Avoids the cancellation of 1/2 z'Pz + q'z + r0 (positions ~3e3). */
static double direct_objective_k(const or_cfg* cf, const double* x0, const double* xf, const double* xb,
                                 const double* xl, const double* z, int K);
static double direct_objective(const or_cfg* cf, const double* x0, const double* xf, const double* xb,
                               const double* xl, const double* z) {
    return direct_objective_k(cf, x0, xf, xb, xl, z, cf->N);
}
/* K < N: objective of the relaxation built by build_qp_k (no input terms for k >= K) */
static double direct_objective_k(const or_cfg* cf, const double* x0, const double* xf, const double* xb,
                                 const double* xl, const double* z, int K) {
    const int N = cf->N;
    double J = 0.0;
    if (cf->admm) { /* the copies are part of the solution; price their ADMM terms */
        int idx = 3 * N + ((cf->role & R_SF) ? N + 1 : 0) + ((cf->role & R_SB) ? N + 1 : 0);
        const int has_b = (cf->role & R_SB) || cf->back_copy;
        if (cf->role & R_SF) { xf = z + idx; idx += 2 * (N + 1); }
        if (has_b) xb = z + idx;
        const double* cc[2] = {(cf->role & R_SF) ? xf : NULL, has_b ? xb : NULL};
        const double* yy[2] = {cf->yf, cf->yb};
        const double* zz[2] = {cf->zf, cf->zb};
        for (int side = 0; side < 2; ++side) {
            if (!cc[side]) continue;
            for (int k = 0; k <= N; ++k)
                for (int i = 0; i < 2; ++i) {
                    double d = par(cc[side], N, i, k) - par(zz[side], N, i, k);
                    J += par(yy[side], N, i, k) * d + 0.5 * cf->rho * d * d;
                }
        }
    }
    if (cf->gadmm)
        for (int k = 0; k <= N; ++k)
            for (int i = 0; i < 2; ++i) {
                double xi = k == 0 ? x0[i] : z[2 * (k - 1) + i];
                double d = xi - par(cf->zo, N, i, k);
                J += par(cf->yo, N, i, k) * d + 0.5 * cf->rho * d * d;
            }
    for (int k = 0; k <= N; ++k) {
        double p = k == 0 ? x0[0] : z[2 * (k - 1)], v = k == 0 ? x0[1] : z[2 * (k - 1) + 1];
        double e[3][2];
        int ne = 0;
        if (cf->role & R_TF) { e[ne][0] = p + cf->t0 * v + cf->d0 - par(xf, N, 0, k); e[ne][1] = v - par(xf, N, 1, k); ne++; }
        if (cf->role & R_TB) {
            double pb = par(xb, N, 0, k), vb = par(xb, N, 1, k);
            e[ne][0] = pb + cf->t0 * vb + cf->d0 - p; e[ne][1] = vb - v; ne++;
        }
        if (cf->role & R_TL) {
            e[ne][0] = p - par(xl, N, 0, k) + ((cf->role & R_LSP) ? cf->t0 * v + cf->d0 : 0.0);
            e[ne][1] = v - par(xl, N, 1, k); ne++;
        }
        for (int t = 0; t < ne; ++t) {
            if (cf->quadratic)
                J += cf->Qx[0][0] * e[t][0] * e[t][0] + (cf->Qx[0][1] + cf->Qx[1][0]) * e[t][0] * e[t][1] +
                     cf->Qx[1][1] * e[t][1] * e[t][1];
            else
                J += fabs(cf->Qx[0][0] * e[t][0]) + fabs(cf->Qx[1][1] * e[t][1]);
        }
        if (cf->role & R_SF) J += cf->w * fmax(0.0, p - par(xf, N, 0, k) + cf->d_safe);
        if (cf->role & R_SB) J += cf->w * fmax(0.0, par(xb, N, 0, k) + cf->d_safe - p);
    }
    for (int k = 0; k < K; ++k) {
        double u = z[2 * N + k];
        J += cf->quadratic ? cf->Qu * u * u : fabs(cf->Qu * u);
        if (k + 1 < K) {
            double du = z[2 * N + k + 1] - u;
            J += cf->quadratic ? cf->Qdu * du * du : fabs(cf->Qdu * du);
        }
    }
    return J;
}

/* ------------------------------------------------------------------ sigma enumeration */
/* velocity interval of a region / the state box from rows acting on v only */
static int v_interval(const double (*S)[2], const double* T, int nrows, double* lo, double* hi) {
    *lo = -OR_BIG; *hi = OR_BIG;
    for (int r = 0; r < nrows; ++r) {
        if (S[r][0] != 0.0) continue; /* position rows are handled by the QP */
        double s = S[r][1];
        if (s > 0) *hi = fmin(*hi, T[r] / s);
        else if (s < 0) *lo = fmax(*lo, T[r] / s);
        else if (T[r] < 0) return 0;
    }
    return *lo <= *hi;
}

/* Exact projection onto v' of the polygon {(v, v'): lo<=v<=hi, v' = a v + b u + c for some
 * u in [ul, uh], dec <= v'-v <= acc, blo <= v' <= bhi} by vertex enumeration. */
static int next_interval(double lo, double hi, double a, double b, double c, double ul, double uh, double dec,
                         double acc, double blo, double bhi, double* nlo, double* nhi) {
    /* half-planes  n0*v + n1*v' <= r */
    double H[8][3];
    int nh = 0;
    double bl = fmin(b * ul, b * uh), bu = fmax(b * ul, b * uh);
    H[nh][0] = -1; H[nh][1] = 0; H[nh++][2] = -lo;
    H[nh][0] = 1; H[nh][1] = 0; H[nh++][2] = hi;
    H[nh][0] = a; H[nh][1] = -1; H[nh++][2] = -(c + bl);  /* v' >= a v + c + bl */
    H[nh][0] = -a; H[nh][1] = 1; H[nh++][2] = c + bu;     /* v' <= a v + c + bu */
    H[nh][0] = 1; H[nh][1] = -1; H[nh++][2] = -dec;       /* v' - v >= dec */
    H[nh][0] = -1; H[nh][1] = 1; H[nh++][2] = acc;        /* v' - v <= acc */
    H[nh][0] = 0; H[nh][1] = -1; H[nh++][2] = -blo;
    H[nh][0] = 0; H[nh][1] = 1; H[nh++][2] = bhi;
    int found = 0;
    double mn = OR_BIG, mx = -OR_BIG;
    for (int i = 0; i < nh; ++i)
        for (int j = i + 1; j < nh; ++j) {
            double det = H[i][0] * H[j][1] - H[i][1] * H[j][0];
            if (fabs(det) < 1e-14) continue;
            double v = (H[i][2] * H[j][1] - H[i][1] * H[j][2]) / det;
            double vp = (H[i][0] * H[j][2] - H[i][2] * H[j][0]) / det;
            int ok = 1;
            for (int k = 0; k < nh && ok; ++k) {
                double tol = 1e-9 * (1.0 + fabs(H[k][2]));
                if (H[k][0] * v + H[k][1] * vp > H[k][2] + tol) ok = 0;
            }
            if (ok) { found = 1; mn = fmin(mn, vp); mx = fmax(mx, vp); }
        }
    if (!found) return 0;
    *nlo = mn; *nhi = mx;
    return 1;
}

typedef struct {
    double a[OR_MAX_REG], b[OR_MAX_REG], c[OR_MAX_REG], rlo[OR_MAX_REG], rhi[OR_MAX_REG];
    int rok[OR_MAX_REG];
    double blo, bhi, ul, uh;
} or_vmodel;

static int make_vmodel(const or_model* md, or_vmodel* vm) {
    for (int r = 0; r < md->nreg; ++r) {
        if (md->A[r][1][0] != 0.0) return -1; /* velocity dynamics must not depend on p */
        for (int row = 0; row < md->nsr; ++row)
            if (md->S[r][row][0] != 0.0 || md->R[r][row] != 0.0) return -1;
        vm->a[r] = md->A[r][1][1]; vm->b[r] = md->B[r][1]; vm->c[r] = md->c[r][1];
        vm->rok[r] = v_interval((const double(*)[2])md->S[r], md->T[r], md->nsr, &vm->rlo[r], &vm->rhi[r]);
    }
    if (!v_interval((const double(*)[2])md->D, md->E, md->nd, &vm->blo, &vm->bhi)) return -1;
    vm->ul = -OR_BIG; vm->uh = OR_BIG;
    for (int row = 0; row < md->nf; ++row) {
        if (md->F[row] > 0) vm->uh = fmin(vm->uh, md->G[row] / md->F[row]);
        else if (md->F[row] < 0) vm->ul = fmax(vm->ul, md->G[row] / md->F[row]);
    }
    return 0;
}

/* Tail relaxation of one vehicle's undecided steps k >= K (centralised branch and bound):
 *  - v_k stays in the interval reachable from [lo, hi] = the exact interval of v_K, propagated as
 *    the hull over the regions step k may still take (the regions whose band meets the interval);
 *  - when all those regions share the velocity dynamics (a, c) and b > 0, with ul <= 0 <= uh, the
 *    step takes the VIRTUAL region (a, b_max, c): every completion's input u (region r) maps to
 *    s = u b_r / b_max, which meets v' = a v + b_max s + c and the input box, with Qu s^2 <= Qu u^2;
 *    otherwise the velocity dynamics, input rows and input cost of the step are dropped.
 * Both keep the QP of the prefix a lower bound of every completion. */
typedef struct {
    double vlo[OR_MAX_N + 1], vhi[OR_MAX_N + 1]; /* interval of v_k, k = K..N */
    int virt[OR_MAX_N];                          /* region index carrying (a, c), or -1 */
    double bmax[OR_MAX_N];
    double blo, bhi; /* state box of v */
} or_relax;

static int g_cent_relax = 1;
void oracle_set_cent_relax(int on) { g_cent_relax = on; }

static void relax_tail(const or_vmodel* vm, int nreg, const or_cfg* cf, int K, double lo, double hi, or_relax* X) {
    const int N = cf->N;
    for (int k = 0; k < N; ++k) X->virt[k] = -1;
    X->blo = vm->blo; X->bhi = vm->bhi;
    for (int k = 0; k <= N; ++k) { X->vlo[k] = vm->blo; X->vhi[k] = vm->bhi; }
    if (!g_cent_relax) return;
    X->vlo[K] = lo; X->vhi[K] = hi;
    for (int k = K; k < N; ++k) {
        const double dec = cf->a_dec * cf->ts + k * cf->tight, acc = cf->a_acc * cf->ts - k * cf->tight;
        double nlo = OR_BIG, nhi = -OR_BIG, bmax = 0.0;
        int first = -1, shared = vm->ul <= 0.0 && vm->uh >= 0.0 && vm->uh > vm->ul;
        for (int r = 0; r < nreg; ++r) {
            if (!vm->rok[r]) continue;
            double ilo = fmax(X->vlo[k], vm->rlo[r]), ihi = fmin(X->vhi[k], vm->rhi[r]);
            if (ilo > ihi + 1e-9 * (1.0 + fabs(ihi))) continue;
            if (ilo > ihi) ilo = ihi = 0.5 * (ilo + ihi);
            double a, b;
            if (!next_interval(ilo, ihi, vm->a[r], vm->b[r], vm->c[r], vm->ul, vm->uh, dec, acc, vm->blo, vm->bhi, &a,
                               &b))
                continue;
            nlo = fmin(nlo, a); nhi = fmax(nhi, b);
            if (first < 0) first = r;
            else if (vm->a[r] != vm->a[first] || vm->c[r] != vm->c[first]) shared = 0;
            if (!(vm->b[r] > 0.0)) shared = 0;
            bmax = fmax(bmax, vm->b[r]);
        }
        if (first < 0) { /* no completion: keep the plain relaxation from here on */
            for (int j = k + 1; j <= N; ++j) { X->vlo[j] = vm->blo; X->vhi[j] = vm->bhi; }
            return;
        }
        if (shared) { X->virt[k] = first; X->bmax[k] = bmax; }
        X->vlo[k + 1] = nlo; X->vhi[k + 1] = nhi;
    }
}

typedef void (*or_visit)(const int* sigma, void* ctx);

static void dfs(const or_vmodel* vm, int nreg, const or_cfg* cf, int k, double lo, double hi, int* sigma,
                or_visit visit, void* ctx, int* count) {
    const int N = cf->N;
    if (k == N) { (*count)++; if (visit) visit(sigma, ctx); return; }
    double dec = cf->a_dec * cf->ts + k * cf->tight, acc = cf->a_acc * cf->ts - k * cf->tight;
    for (int r = 0; r < nreg; ++r) {
        if (!vm->rok[r]) continue;
        double ilo = fmax(lo, vm->rlo[r]), ihi = fmin(hi, vm->rhi[r]);
        if (ilo > ihi + 1e-9 * (1.0 + fabs(ihi))) continue;
        if (ilo > ihi) ilo = ihi = 0.5 * (ilo + ihi);
        double nlo, nhi;
        if (!next_interval(ilo, ihi, vm->a[r], vm->b[r], vm->c[r], vm->ul, vm->uh, dec, acc, vm->blo, vm->bhi,
                           &nlo, &nhi))
            continue;
        sigma[k] = r;
        dfs(vm, nreg, cf, k + 1, nlo, nhi, sigma, visit, ctx, count);
    }
}

/* ------------------------------------------------------------------ public API */
typedef struct {
    const or_model* md;
    const or_cfg* cf;
    const double *x0, *xf, *xb, *xl;
    or_qp* qp;
    or_work* w;
    int maxit;
    int n_conv, n_cert, iters, n_qp;
    /* every candidate in DFS (= lexicographic) order */
    int ncand, cap;
    double* obj;
    int* sig;
    unsigned char* cert;
} or_ctx;

static void visit_qp(const int* sigma, void* vctx) {
    or_ctx* C = (or_ctx*)vctx;
    const int N = C->cf->N;
    if (C->ncand == C->cap) {
        int nc = C->cap ? 2 * C->cap : 64;
        C->obj = (double*)realloc(C->obj, sizeof(double) * nc);
        C->sig = (int*)realloc(C->sig, sizeof(int) * (size_t)nc * N);
        C->cert = (unsigned char*)realloc(C->cert, (size_t)nc);
        C->cap = nc;
    }
    double obj = INFINITY;
    int cert = 0;
    if (build_qp(C->qp, C->md, C->cf, sigma, C->x0, C->xf, C->xb, C->xl) > 0 && !C->qp->infeasible_const) {
        or_result r = ipm_solve(C->qp, C->w, C->maxit);
        C->iters += r.iters;
        if (r.converged) {
            obj = direct_objective(C->cf, C->x0, C->xf, C->xb, C->xl, C->w->z);
            cert = r.certified; C->n_conv++; C->n_cert += cert;
        }
    }
    C->obj[C->ncand] = obj;
    C->cert[C->ncand] = (unsigned char)cert;
    memcpy(C->sig + (size_t)C->ncand * N, sigma, sizeof(int) * N);
    C->ncand++;
}

/* ------------------------------------------------------------------ branch and bound
 * Depth-first branch and bound over the region sequences (the search Gurobi performs over the
 * MLD binaries, restated): children of a prefix are the regions reachable at the next step;
 * each child gets the optimum of its relaxation (build_qp_k) as lower bound, children are
 * visited in increasing bound order, and a child whose bound exceeds the best leaf so far by
 * more than 1e-7 relative is pruned (100x the 1e-9 tie window, so every sequence tied with the
 * optimum is still evaluated and the tie rule below sees it).  Leaves are exact fixed-sequence
 * QPs and go through visit-style bookkeeping. */
static int g_method = 0; /* 0 exhaustive enumeration, 1 branch and bound */

static void bnb_record(or_ctx* C, const int* sigma, double obj, int cert) {
    const int N = C->cf->N;
    if (C->ncand == C->cap) {
        int nc = C->cap ? 2 * C->cap : 64;
        C->obj = (double*)realloc(C->obj, sizeof(double) * nc);
        C->sig = (int*)realloc(C->sig, sizeof(int) * (size_t)nc * N);
        C->cert = (unsigned char*)realloc(C->cert, (size_t)nc);
        C->cap = nc;
    }
    C->obj[C->ncand] = obj;
    C->cert[C->ncand] = (unsigned char)cert;
    memcpy(C->sig + (size_t)C->ncand * N, sigma, sizeof(int) * N);
    C->ncand++;
}

/* relaxed (K < N) or exact (K = N) QP of prefix sigma[0..K-1]: objective or +inf */
static double bnb_qp(or_ctx* C, const int* sigma, int K, int* cert) {
    *cert = 0;
    C->n_qp++;
    if (build_qp_k(C->qp, C->md, C->cf, sigma, K, C->x0, C->xf, C->xb, C->xl) <= 0 || C->qp->infeasible_const)
        return INFINITY;
    or_result r = ipm_solve(C->qp, C->w, C->maxit);
    C->iters += r.iters;
    if (!r.converged) return K < C->cf->N ? -INFINITY : INFINITY; /* an unsolved bound prunes nothing */
    *cert = r.certified;
    if (C->cf->admm && !C->cf->quadratic && !C->cf->gadmm) admm_l1_exact_copies(C->cf, C->x0, C->w->z);
    return direct_objective_k(C->cf, C->x0, C->xf, C->xb, C->xl, C->w->z, K);
}

static void bnb_dfs(or_ctx* C, const or_vmodel* vm, int nreg, int k, double lo, double hi, int* sigma, double* inc,
                    int* count) {
    const int N = C->cf->N;
    const or_cfg* cf = C->cf;
    double dec = cf->a_dec * cf->ts + k * cf->tight, acc = cf->a_acc * cf->ts - k * cf->tight;
    int child[OR_MAX_REG], nch = 0;
    double clo[OR_MAX_REG], chi[OR_MAX_REG], lb[OR_MAX_REG];
    for (int r = 0; r < nreg; ++r) {
        if (!vm->rok[r]) continue;
        double ilo = fmax(lo, vm->rlo[r]), ihi = fmin(hi, vm->rhi[r]);
        if (ilo > ihi + 1e-9 * (1.0 + fabs(ihi))) continue;
        if (ilo > ihi) ilo = ihi = 0.5 * (ilo + ihi);
        double nlo, nhi;
        if (!next_interval(ilo, ihi, vm->a[r], vm->b[r], vm->c[r], vm->ul, vm->uh, dec, acc, vm->blo, vm->bhi,
                           &nlo, &nhi))
            continue;
        sigma[k] = r;
        int cert;
        double b = bnb_qp(C, sigma, k + 1, &cert);
        if (k + 1 == N) {
            (*count)++;
            if (isfinite(b)) { C->n_conv++; C->n_cert += cert; }
            bnb_record(C, sigma, b, cert);
            if (b < *inc) *inc = b;
            continue;
        }
        child[nch] = r; clo[nch] = nlo; chi[nch] = nhi; lb[nch] = b; nch++;
    }
    /* visit in increasing bound order (insertion sort, stable) */
    for (int i = 1; i < nch; ++i)
        for (int j = i; j > 0 && lb[j] < lb[j - 1]; --j) {
            double t = lb[j]; lb[j] = lb[j - 1]; lb[j - 1] = t;
            t = clo[j]; clo[j] = clo[j - 1]; clo[j - 1] = t;
            t = chi[j]; chi[j] = chi[j - 1]; chi[j - 1] = t;
            int ti = child[j]; child[j] = child[j - 1]; child[j - 1] = ti;
        }
    for (int i = 0; i < nch; ++i) {
        if (lb[i] > *inc + 1e-7 * (1.0 + fabs(*inc))) continue;
        sigma[k] = child[i];
        bnb_dfs(C, vm, nreg, k + 1, clo[i], chi[i], sigma, inc, count);
    }
}

void oracle_set_method(int m) { g_method = m; }

/* The relaxation drops only velocity rows: the position row of the dynamics must be the same
 * in every region (true for the reference's PWA models, models.py:370-387). */
static int oracle_bnb_ok(const or_model* md) {
    for (int r = 1; r < md->nreg; ++r)
        if (md->A[r][0][0] != md->A[0][0][0] || md->A[r][0][1] != md->A[0][0][1] || md->B[r][0] != md->B[0][0] ||
            md->c[r][0] != md->c[0][0])
            return 0;
    return 1;
}

/* Winner: the minimum objective; among candidates within 1e-9 relative of it the first in
 * lexicographic sequence order.  Returns -1 when no candidate converged. */
static int select_winner(const double* obj, int n) {
    double best = INFINITY;
    for (int i = 0; i < n; ++i) best = fmin(best, obj[i]);
    if (!isfinite(best)) return -1;
    double tol = 1e-9 * fmax(1.0, fabs(best));
    for (int i = 0; i < n; ++i)
        if (obj[i] <= best + tol) return i;
    return -1;
}

typedef struct { int* out; int cap, n, N; } or_collect;
static void collect_visit(const int* s, void* p) {
    or_collect* c = (or_collect*)p;
    if (c->out && c->n < c->cap) memcpy(c->out + (size_t)c->n * c->N, s, sizeof(int) * c->N);
    c->n++;
}

static int unpack_model(or_model* md, int nreg, int nsr, const double* S, const double* R, const double* T,
                        const double* A, const double* B, const double* c, int nd, const double* D,
                        const double* E, int nf, const double* F, const double* G) {
    if (nreg > OR_MAX_REG || nsr > 4 || nd > 8 || nf > 4) return -1;
    md->nreg = nreg; md->nsr = nsr; md->nd = nd; md->nf = nf;
    for (int r = 0; r < nreg; ++r) {
        for (int i = 0; i < nsr; ++i) {
            md->S[r][i][0] = S[(r * nsr + i) * 2]; md->S[r][i][1] = S[(r * nsr + i) * 2 + 1];
            md->R[r][i] = R[r * nsr + i]; md->T[r][i] = T[r * nsr + i];
        }
        for (int i = 0; i < 2; ++i) {
            md->A[r][i][0] = A[r * 4 + i * 2]; md->A[r][i][1] = A[r * 4 + i * 2 + 1];
            md->B[r][i] = B[r * 2 + i]; md->c[r][i] = c[r * 2 + i];
        }
    }
    for (int i = 0; i < nd; ++i) { md->D[i][0] = D[2 * i]; md->D[i][1] = D[2 * i + 1]; md->E[i] = E[i]; }
    for (int i = 0; i < nf; ++i) { md->F[i] = F[i]; md->G[i] = G[i]; }
    return 0;
}

static void unpack_cfg(or_cfg* cf, int N, int quadratic, int role, const double* p) {
    /* p = [Qx00 Qx01 Qx10 Qx11 Qu Qdu w a_acc a_dec ts d_safe tight d0 t0] */
    cf->N = N; cf->quadratic = quadratic; cf->role = role;
    cf->admm = 0; cf->rho = 0.0; cf->yf = cf->zf = cf->yb = cf->zb = NULL;
    cf->gadmm = 0; cf->back_copy = 0; cf->yo = cf->zo = NULL;
    cf->Qx[0][0] = p[0]; cf->Qx[0][1] = p[1]; cf->Qx[1][0] = p[2]; cf->Qx[1][1] = p[3];
    cf->Qu = p[4]; cf->Qdu = p[5]; cf->w = p[6]; cf->a_acc = p[7]; cf->a_dec = p[8]; cf->ts = p[9];
    cf->d_safe = p[10]; cf->tight = p[11]; cf->d0 = p[12]; cf->t0 = p[13];
}

/* Number of candidate region sequences (DFS order) for one instance; -1 on bad model. */
int oracle_count_candidates(int N, int nreg, int nsr, const double* S, const double* R, const double* T,
                            const double* A, const double* B, const double* c, int nd, const double* D,
                            const double* E, int nf, const double* F, const double* G, const double* cfgp,
                            const double* x0, int* sigmas_out, int cap) {
    or_model md;
    or_cfg cf;
    or_vmodel vm;
    if (N > OR_MAX_N || unpack_model(&md, nreg, nsr, S, R, T, A, B, c, nd, D, E, nf, F, G)) return -1;
    unpack_cfg(&cf, N, 1, 0, cfgp);
    if (make_vmodel(&md, &vm)) return -1;
    int sigma[OR_MAX_N], count = 0;
    or_collect sc = {sigmas_out, cap, 0, N};
    dfs(&vm, md.nreg, &cf, 0, x0[1], x0[1], sigma, collect_visit, &sc, &count);
    return count;
}

/* Solves one local MIQP.  x_out (2, N+1) row-major, u_out (N), sigma_out (N),
 * info_out = [cost, n_candidates, n_converged, n_certified, best_certified, status, iters].
 * cand_obj / cand_sigma (optional) receive every candidate's objective (inf = not converged). */
int oracle_solve_miqp(int N, int nreg, int nsr, const double* S, const double* R, const double* T, const double* A,
                      const double* B, const double* c, int nd, const double* D, const double* E, int nf,
                      const double* F, const double* G, const double* cfgp, int quadratic, int role,
                      const double* x0, const double* xf, const double* xb, const double* xl, int maxit,
                      double* x_out, double* u_out, int* sigma_out, double* info_out, double* cand_obj,
                      int* cand_sigma, int cand_cap) {
    or_model md;
    or_cfg cf;
    or_vmodel vm;
    if (N > OR_MAX_N || unpack_model(&md, nreg, nsr, S, R, T, A, B, c, nd, D, E, nf, F, G)) return -1;
    unpack_cfg(&cf, N, quadratic, role, cfgp);
    if (make_vmodel(&md, &vm)) return -2;
    or_qp* qp = (or_qp*)malloc(sizeof(or_qp));
    or_work* w = (or_work*)malloc(sizeof(or_work));
    if (!qp || !w) { free(qp); free(w); return -3; }
    or_ctx C;
    memset(&C, 0, sizeof(C));
    C.md = &md; C.cf = &cf; C.x0 = x0; C.xf = xf; C.xb = xb; C.xl = xl; C.qp = qp; C.w = w;
    C.maxit = maxit > 0 ? maxit : 200;
    int sigma[OR_MAX_N], count = 0;
    int win;
    if (g_method == 1) {
        if (!oracle_bnb_ok(&md)) { free(qp); free(w); return -4; }
        double inc = INFINITY;
        bnb_dfs(&C, &vm, md.nreg, 0, x0[1], x0[1], sigma, &inc, &count);
        /* exploration order is by bound: the tie rule compares sequences lexicographically */
        win = -1;
        if (isfinite(inc)) {
            double tol = 1e-9 * fmax(1.0, fabs(inc));
            for (int i = 0; i < C.ncand; ++i) {
                if (!(C.obj[i] <= inc + tol)) continue;
                int less = win < 0;
                for (int k = 0; k < N && !less; ++k) {
                    int a = C.sig[(size_t)i * N + k], b = C.sig[(size_t)win * N + k];
                    if (a != b) { less = a < b; break; }
                }
                if (less) win = i;
            }
        }
        /* nodes = QPs of the search (the reference's Gurobi NodeCount analogue); no leaf at all
         * means no feasible sequence */
        count = count ? C.n_qp : 0;
    } else {
        dfs(&vm, md.nreg, &cf, 0, x0[1], x0[1], sigma, visit_qp, &C, &count);
        win = select_winner(C.obj, C.ncand);
    }
    int status = win >= 0 ? 0 : (count == 0 ? 1 : 2);
    int best_cert = 0;
    double best_obj = INFINITY;
    if (win >= 0) {
        /* re-solve the winner to recover its trajectory */
        const int* ws = C.sig + (size_t)win * N;
        build_qp(qp, &md, &cf, ws, x0, xf, xb, xl);
        or_result r = ipm_solve(qp, w, C.maxit);
        best_obj = direct_objective(&cf, x0, xf, xb, xl, w->z);
        best_cert = r.certified;
        for (int i = 0; i < 2; ++i) x_out[i * (N + 1)] = x0[i];
        for (int k = 1; k <= N; ++k)
            for (int i = 0; i < 2; ++i) x_out[i * (N + 1) + k] = w->z[2 * (k - 1) + i];
        for (int k = 0; k < N; ++k) u_out[k] = w->z[2 * N + k];
        for (int k = 0; k < N; ++k) sigma_out[k] = ws[k];
    }
    for (int i = 0; i < C.ncand && i < cand_cap; ++i) {
        if (cand_obj) cand_obj[i] = C.obj[i];
        if (cand_sigma) memcpy(cand_sigma + (size_t)i * N, C.sig + (size_t)i * N, sizeof(int) * N);
    }
    free(C.obj); free(C.sig); free(C.cert);
    info_out[0] = best_obj;
    info_out[1] = count;
    info_out[2] = C.n_conv;
    info_out[3] = C.n_cert;
    info_out[4] = best_cert;
    info_out[5] = status;
    info_out[6] = C.iters;
    free(qp);
    free(w);
    return 0;
}

/* Naive-ADMM local MIQP (LocalMpcADMM, fleet_naive_admm.py:24-253), by branch and bound.
 * p = [x0 (2) | y_front | z_front | y_back | z_back | leader_x] (each (2, N+1)), as
 * hvp_params_stride_admm.  Outputs as oracle_solve_miqp plus the copies xf_out / xb_out.
 * role bit 17: min_1_norm (LocalMpcADMM(quadratic_cost=False), fleet_naive_admm.py:74-77): every
 * tracking / input term priced sum_i Q_ii |e_i| through add_norm's epigraph variables, the ADMM
 * terms y'(c - z) + rho/2 |c - z|^2 of the copies (:172-198) unchanged -- a QP with L1 terms. */
int oracle_solve_admm_miqp(int N, int nreg, int nsr, const double* S, const double* R, const double* T,
                           const double* A, const double* B, const double* c, int nd, const double* D, const double* E,
                           int nf, const double* F, const double* G, const double* cfgp, int role, double rho,
                           const double* p, int maxit, double* x_out, double* u_out, int* sigma_out, double* info_out,
                           double* xf_out, double* xb_out) {
    or_model md;
    or_cfg cf;
    or_vmodel vm;
    if (N > OR_MAX_N || unpack_model(&md, nreg, nsr, S, R, T, A, B, c, nd, D, E, nf, F, G)) return -1;
    const int quadratic = !((role >> 17) & 1);
    role &= 0xffff;
    unpack_cfg(&cf, N, quadratic, role, cfgp);
    const int K1 = 2 * (N + 1);
    cf.admm = 1;
    cf.rho = rho;
    cf.yf = p + 2; cf.zf = p + 2 + K1; cf.yb = p + 2 + 2 * K1; cf.zb = p + 2 + 3 * K1;
    const double* xl = p + 2 + 4 * K1;
    if (make_vmodel(&md, &vm) || !oracle_bnb_ok(&md)) return -2;
    or_qp* qp = (or_qp*)malloc(sizeof(or_qp));
    or_work* w = (or_work*)malloc(sizeof(or_work));
    if (!qp || !w) { free(qp); free(w); return -3; }
    static const double zero[2 * (OR_MAX_N + 1)] = {0};
    or_ctx C;
    memset(&C, 0, sizeof(C));
    C.md = &md; C.cf = &cf; C.x0 = p; C.xf = zero; C.xb = zero; C.xl = xl; C.qp = qp; C.w = w;
    C.maxit = maxit > 0 ? maxit : 200;
    int sigma[OR_MAX_N], count = 0;
    double inc = INFINITY;
    bnb_dfs(&C, &vm, md.nreg, 0, p[1], p[1], sigma, &inc, &count);
    int win = -1;
    if (isfinite(inc)) {
        double tol = 1e-9 * fmax(1.0, fabs(inc));
        for (int i = 0; i < C.ncand; ++i) {
            if (!(C.obj[i] <= inc + tol)) continue;
            int less = win < 0;
            for (int k = 0; k < N && !less; ++k) {
                int a = C.sig[(size_t)i * N + k], b = C.sig[(size_t)win * N + k];
                if (a != b) { less = a < b; break; }
            }
            if (less) win = i;
        }
    }
    int status = win >= 0 ? 0 : (count == 0 ? 1 : 2);
    double best_obj = INFINITY;
    int best_cert = 0;
    memset(xf_out, 0, sizeof(double) * K1);
    memset(xb_out, 0, sizeof(double) * K1);
    if (win >= 0) {
        const int* ws = C.sig + (size_t)win * N;
        build_qp(qp, &md, &cf, ws, p, zero, zero, xl);
        or_result r = ipm_solve(qp, w, C.maxit);
        if (!quadratic) admm_l1_exact_copies(&cf, p, w->z);
        best_obj = direct_objective(&cf, p, zero, zero, xl, w->z);
        best_cert = r.certified;
        for (int i = 0; i < 2; ++i) x_out[i * (N + 1)] = p[i];
        for (int k = 1; k <= N; ++k)
            for (int i = 0; i < 2; ++i) x_out[i * (N + 1) + k] = w->z[2 * (k - 1) + i];
        for (int k = 0; k < N; ++k) u_out[k] = w->z[2 * N + k];
        for (int k = 0; k < N; ++k) sigma_out[k] = ws[k];
        int idx = 3 * N + ((role & R_SF) ? N + 1 : 0) + ((role & R_SB) ? N + 1 : 0);
        if (role & R_SF) { memcpy(xf_out, w->z + idx, sizeof(double) * K1); idx += K1; }
        if (role & R_SB) memcpy(xb_out, w->z + idx, sizeof(double) * K1);
    }
    free(C.obj); free(C.sig); free(C.cert);
    info_out[0] = best_obj;
    info_out[1] = count ? C.n_qp : 0;
    info_out[2] = C.n_conv;
    info_out[3] = C.n_cert;
    info_out[4] = best_cert;
    info_out[5] = status;
    info_out[6] = C.iters;
    free(qp);
    free(w);
    return 0;
}

/* Batch of independent instances sharing one model table set (models indexed per instance).
 * Model arrays are stacked per system: S[nsys][nreg][nsr][2] etc.  OpenMP over instances. */
int oracle_solve_batch(int B, int N, int nsys, int nreg, int nsr, const double* S, const double* R,
                       const double* T, const double* A, const double* B_, const double* c, int nd,
                       const double* D, const double* E, int nf, const double* F, const double* G,
                       const double* cfgp, int quadratic, const int* sys, const int* role, const double* params,
                       int maxit, double* x_out, double* u_out, int* sigma_out, double* info_out, int nthreads) {
    const int P = 2 + 6 * (N + 1);
    int err = 0;
    (void)nsys;
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1) reduction(| : err)
    for (int i = 0; i < B; ++i) {
        const int s = sys[i];
        const double* p = params + (size_t)i * P;
        int rc = oracle_solve_miqp(
            N, nreg, nsr, S + (size_t)s * nreg * nsr * 2, R + (size_t)s * nreg * nsr, T + (size_t)s * nreg * nsr,
            A + (size_t)s * nreg * 4, B_ + (size_t)s * nreg * 2, c + (size_t)s * nreg * 2, nd, D + (size_t)s * nd * 2,
            E + (size_t)s * nd, nf, F + (size_t)s * nf, G + (size_t)s * nf, cfgp, quadratic, role[i], p, p + 2,
            p + 2 + 2 * (N + 1), p + 2 + 4 * (N + 1), maxit, x_out + (size_t)i * 2 * (N + 1), u_out + (size_t)i * N,
            sigma_out + (size_t)i * N, info_out + (size_t)i * 7, NULL, NULL, 0);
        if (rc) err |= 1;
    }
    return err ? -1 : 0;
}

/* Solve ONE fixed-sigma QP (exposed for the tests that cross-check against scipy). */
int oracle_solve_qp(int N, int nreg, int nsr, const double* S, const double* R, const double* T, const double* A,
                    const double* B, const double* c, int nd, const double* D, const double* E, int nf,
                    const double* F, const double* G, const double* cfgp, int quadratic, int role, const int* sigma,
                    const double* x0, const double* xf, const double* xb, const double* xl, double* z_out,
                    double* info_out) {
    or_model md;
    or_cfg cf;
    if (N > OR_MAX_N || unpack_model(&md, nreg, nsr, S, R, T, A, B, c, nd, D, E, nf, F, G)) return -1;
    unpack_cfg(&cf, N, quadratic, role, cfgp);
    or_qp* qp = (or_qp*)malloc(sizeof(or_qp));
    or_work* w = (or_work*)malloc(sizeof(or_work));
    if (!qp || !w) { free(qp); free(w); return -3; }
    int nz = build_qp(qp, &md, &cf, sigma, x0, xf, xb, xl);
    or_result r = {0, 0, 0, INFINITY};
    if (nz > 0 && !qp->infeasible_const) r = ipm_solve(qp, w, 200);
    if (nz > 0) memcpy(z_out, w->z, sizeof(double) * nz);
    info_out[0] = r.converged ? r.obj : INFINITY;
    info_out[1] = r.converged;
    info_out[2] = r.certified;
    info_out[3] = r.iters;
    info_out[4] = nz;
    info_out[5] = qp->m;
    info_out[6] = qp->neq;
    free(qp);
    free(w);
    return 0;
}

/* Certificate of a batch of answers (tests only): for every instance the fixed-sigma QP of the
 * sequence sigma_in[i] (the product's chosen regions) solved and KKT-certified by the IPM above;
 * out[i*(2+N)] = objective (INFINITY if not converged), out[..+1] = certified, then u (N).
 * A product answer is certified when its cost equals this objective and its u this u (the QP is
 * strictly convex in u, so the certified u is THE optimum of that sequence). */
int oracle_certify_batch(int B, int N, int nsys, int nreg, int nsr, const double* S, const double* R,
                         const double* T, const double* A, const double* B_, const double* c, int nd,
                         const double* D, const double* E, int nf, const double* F, const double* G,
                         const double* cfgp, int quadratic, const int* sys, const int* role, const double* params,
                         const int* sigma_in, double* out, int nthreads) {
    const int P = 2 + 6 * (N + 1);
    int err = 0;
    (void)nsys;
    if (N > OR_MAX_N) return -1;
#pragma omp parallel num_threads(nthreads > 0 ? nthreads : 1) reduction(| : err)
    {
        or_qp* qp = (or_qp*)malloc(sizeof(or_qp));
        or_work* w = (or_work*)malloc(sizeof(or_work));
        if (!qp || !w) err |= 1;
#pragma omp for schedule(dynamic, 64)
        for (int i = 0; i < B; ++i) {
            if (!qp || !w) continue;
            const int s = sys[i];
            const double* p = params + (size_t)i * P;
            or_model md;
            or_cfg cf;
            double* o = out + (size_t)i * (2 + N);
            if (unpack_model(&md, nreg, nsr, S + (size_t)s * nreg * nsr * 2, R + (size_t)s * nreg * nsr,
                             T + (size_t)s * nreg * nsr, A + (size_t)s * nreg * 4, B_ + (size_t)s * nreg * 2,
                             c + (size_t)s * nreg * 2, nd, D + (size_t)s * nd * 2, E + (size_t)s * nd, nf,
                             F + (size_t)s * nf, G + (size_t)s * nf)) {
                err |= 1;
                continue;
            }
            unpack_cfg(&cf, N, quadratic, role[i], cfgp);
            const int nz = build_qp(qp, &md, &cf, sigma_in + (size_t)i * N, p, p + 2, p + 2 + 2 * (N + 1),
                                    p + 2 + 4 * (N + 1));
            or_result r = {0, 0, 0, INFINITY};
            if (nz > 0 && !qp->infeasible_const) r = ipm_solve(qp, w, 200);
            o[0] = r.converged ? r.obj : INFINITY;
            o[1] = r.certified;
            for (int k = 0; k < N; ++k) o[2 + k] = (nz > 0 && r.converged) ? w->z[2 * N + k] : NAN;
        }
        free(qp);
        free(w);
    }
    return err ? -1 : 0;
}

/* Dense export of one fixed-sigma QP (tests only): P[nz*nz], q[nz], Aeq[neq*nz], beq, G[m*nz], h,
 * dims_out = [nz, neq, m, r0, infeasible_const]. Capacity of each buffer given by cap_* . */
int oracle_export_qp(int N, int nreg, int nsr, const double* S, const double* R, const double* T, const double* A,
                     const double* B, const double* c, int nd, const double* D, const double* E, int nf,
                     const double* F, const double* G, const double* cfgp, int quadratic, int role, const int* sigma,
                     const double* x0, const double* xf, const double* xb, const double* xl, double* P_out,
                     double* q_out, double* A_out, double* b_out, double* G_out, double* h_out, double* dims_out) {
    or_model md;
    or_cfg cf;
    if (N > OR_MAX_N || unpack_model(&md, nreg, nsr, S, R, T, A, B, c, nd, D, E, nf, F, G)) return -1;
    unpack_cfg(&cf, N, quadratic, role, cfgp);
    or_qp* qp = (or_qp*)malloc(sizeof(or_qp));
    if (!qp) return -3;
    int nz = build_qp(qp, &md, &cf, sigma, x0, xf, xb, xl);
    for (int i = 0; i < nz; ++i) {
        q_out[i] = qp->q[i];
        for (int j = 0; j < nz; ++j) P_out[i * nz + j] = qp->P[i][j];
    }
    for (int e = 0; e < qp->neq; ++e) {
        b_out[e] = qp->beq[e];
        for (int j = 0; j < nz; ++j) A_out[e * nz + j] = qp->Aeq[e][j];
    }
    for (int r = 0; r < qp->m; ++r) {
        h_out[r] = qp->h[r];
        for (int j = 0; j < nz; ++j) G_out[r * nz + j] = qp->G[r][j];
    }
    dims_out[0] = nz; dims_out[1] = qp->neq; dims_out[2] = qp->m; dims_out[3] = qp->r0;
    dims_out[4] = qp->infeasible_const;
    free(qp);
    return 0;
}

/* Local QP of the switching ADMM (fleet_g_admm.LocalMpc, :22-205) for a GIVEN region sequence
 * (MpcSwitching [EXT]: dynamics and region rows of sigma_k at every step, no binaries).
 * p = [x0 (2) | y_front | z_front | y_back | z_back | leader_x | y_own | z_own], each (2, N+1).
 * back_copy: the vehicle holds a copy of the one behind (ADMM term only).
 * Outputs: x (2, N+1), u (N), xf / xb (2, N+1) (zero when absent), info = [objective (the
 * local cost incl. every ADMM term, sol.f), status (0 ok, 1 infeasible / not converged),
 * certified, switch bits].  Switch bits (the switching rule, see oracle.py GAdmmCoordinator):
 * bit 2 (k - 1) + 0 / + 1 for k = 1..N-1 when the lower / upper velocity edge of region
 * sigma_k is an active region row with multiplier > 1e-6 and lies strictly inside the state
 * box (crossing it leads into the neighbouring region). */
int oracle_solve_gadmm_qp(int N, int nreg, int nsr, const double* S, const double* R, const double* T,
                          const double* A, const double* B, const double* c, int nd, const double* D,
                          const double* E, int nf, const double* F, const double* G, const double* cfgp, int role,
                          int back_copy, double rho, const double* p, const int* sigma, double* x_out,
                          double* u_out, double* xf_out, double* xb_out, double* info_out) {
    or_model md;
    or_cfg cf;
    or_vmodel vm;
    if (N > OR_MAX_N || unpack_model(&md, nreg, nsr, S, R, T, A, B, c, nd, D, E, nf, F, G)) return -1;
    if (make_vmodel(&md, &vm)) return -2;
    unpack_cfg(&cf, N, 1, role, cfgp);
    const int K1 = 2 * (N + 1);
    cf.admm = 1; cf.gadmm = 1; cf.back_copy = back_copy; cf.rho = rho;
    cf.yf = p + 2; cf.zf = p + 2 + K1; cf.yb = p + 2 + 2 * K1; cf.zb = p + 2 + 3 * K1;
    const double* xl = p + 2 + 4 * K1;
    cf.yo = p + 2 + 5 * K1; cf.zo = p + 2 + 6 * K1;
    static const double zero[2 * (OR_MAX_N + 1)] = {0};
    or_qp* qp = (or_qp*)malloc(sizeof(or_qp));
    or_work* w = (or_work*)malloc(sizeof(or_work));
    if (!qp || !w) { free(qp); free(w); return -3; }
    int nz = build_qp(qp, &md, &cf, sigma, p, zero, zero, xl);
    or_result r = {0, 0, 0, INFINITY};
    if (nz > 0 && !qp->infeasible_const) r = ipm_solve(qp, w, 200);
    memset(xf_out, 0, sizeof(double) * K1);
    memset(xb_out, 0, sizeof(double) * K1);
    double bits = 0.0;
    if (r.converged) {
        for (int i = 0; i < 2; ++i) x_out[i * (N + 1)] = p[i];
        for (int k = 1; k <= N; ++k)
            for (int i = 0; i < 2; ++i) x_out[i * (N + 1) + k] = w->z[2 * (k - 1) + i];
        for (int k = 0; k < N; ++k) u_out[k] = w->z[2 * N + k];
        int idx = 3 * N + ((role & R_SF) ? N + 1 : 0);
        if (role & R_SF) { memcpy(xf_out, w->z + idx, sizeof(double) * K1); idx += K1; }
        if (back_copy) memcpy(xb_out, w->z + idx, sizeof(double) * K1);
        unsigned mask = 0;
        for (int k = 1; k < N; ++k) {
            const int rg = sigma[k];
            for (int row = 0; row < md.nsr; ++row) {
                const int m = qp->reg_row[k][row];
                if (m < 0 || !(w->lam[m] > 1e-6)) continue;
                const double s = md.S[rg][row][1];
                if (md.S[rg][row][0] != 0.0 || s == 0.0) continue;
                const double edge = md.T[rg][row] / s;
                if (s > 0 && edge < vm.bhi - 1e-9 * (1.0 + fabs(edge))) mask |= 1u << (2 * (k - 1) + 1);
                if (s < 0 && edge > vm.blo + 1e-9 * (1.0 + fabs(edge))) mask |= 1u << (2 * (k - 1));
            }
        }
        bits = (double)mask;
    }
    info_out[0] = r.converged ? direct_objective(&cf, p, zero, zero, xl, w->z) : INFINITY;
    info_out[1] = r.converged ? 0 : 1;
    info_out[2] = r.certified;
    info_out[3] = bits;
    free(qp);
    free(w);
    return 0;
}

/* ================================================================== centralised MLD (a20)
 * MpcMldCent (mpcs/cent_mld.py:21-182): ONE MIQP over the platoon.  Per vehicle i the MLD model
 * of MpcMldCentDecup [EXT] (region rows / dynamics of sigma_{i,k}, D x <= E for k >= 1, F u <= G),
 * the acceleration rows (:145-163); cost: leader tracking of x_ref by vehicle L (:85-105, with
 * spacing when real_vehicle_as_reference), the chain terms |x_i - x_{i-1} - spacing(x_i)|^2_Q for
 * i >= 1 (:106-117), Q_u u^2, Q_du (du)^2 (:119-135) and w s (:137-140) with the soft safe rows
 * p_i <= p_{i-1} - d_safe + s_i (:170-177) and, with real_vehicle_as_reference, the leader's row
 * p_0 <= x_ref - d_safe + s_0 (:164-169).  Vehicle i's steps k >= K[i] are relaxed as in
 * build_qp_k (branch and bound).  Layout per vehicle: x (2N) | u (N) | s (N+1, if it has a safe
 * row).  x0 = [p0 v0] per vehicle, xl = leader_x (2, N+1). */
#define OR_MAX_VEH 16
typedef struct {
    int n, lsp, L;
    int xo[OR_MAX_VEH], uo[OR_MAX_VEH], so[OR_MAX_VEH];
} or_cent_layout;

static lin CX(const or_cent_layout* CL, const double* x0, int N, int i, int k, int c) {
    if (k == 0) return lin_const(x0[2 * i + c]);
    lin e = lin_const(0.0);
    lin_add(&e, CL->xo[i] + 2 * (k - 1) + c, 1.0);
    return e;
    (void)N;
}

static int build_cent_qp(or_qp* qp, const or_model* md, const or_cfg* cf, or_cent_layout* CL, const int* sigma,
                         const int* K, const or_relax* RX, const double* x0, const double* xl) {
    const int N = cf->N, n = CL->n;
    int nz = 0;
    for (int i = 0; i < n; ++i) {
        CL->xo[i] = nz; nz += 2 * N;
        CL->uo[i] = nz; nz += N;
        const int has_s = i >= 1 || (CL->lsp && CL->L == 0);
        CL->so[i] = has_s ? nz : -1;
        if (has_s) nz += N + 1;
    }
    if (nz > OR_MAX_NZ) return 0;
    memset(qp->P, 0, sizeof(qp->P));
    memset(qp->q, 0, sizeof(qp->q));
    qp->r0 = 0.0; qp->neq = 0; qp->m = 0; qp->infeasible_const = 0;
    for (int i = 0; i < n; ++i) {
        const or_model* m = &md[i];
        const int* sg = sigma + i * N;
        for (int k = 0; k < N; ++k) {
            const int virt = k < K[i] ? -1 : RX[i].virt[k]; /* relaxed step in its virtual region */
            int r = k < K[i] ? sg[k] : (virt >= 0 ? virt : 0);
            for (int c = 0; c < (k < K[i] || virt >= 0 ? 2 : 1); ++c) {
                lin e = CX(CL, x0, N, i, k + 1, c);
                for (int j = 0; j < 2; ++j) { lin xj = CX(CL, x0, N, i, k, j); e = lin_axpy(-m->A[r][c][j], &xj, &e); }
                lin uk = lin_const(0.0);
                lin_add(&uk, CL->uo[i] + k, 1.0);
                e = lin_axpy(-(virt >= 0 && c == 1 ? RX[i].bmax[k] : m->B[r][c]), &uk, &e);
                if (qp->neq >= OR_MAX_EQ) return 0;
                qp_add_eq(qp, &e, m->c[r][c]);
            }
        }
        for (int k = 0; k < K[i]; ++k) {
            int r = sg[k];
            for (int row = 0; row < m->nsr; ++row) {
                lin e = lin_const(0.0);
                for (int j = 0; j < 2; ++j) { lin xj = CX(CL, x0, N, i, k, j); e = lin_axpy(m->S[r][row][j], &xj, &e); }
                lin uk = lin_const(0.0);
                lin_add(&uk, CL->uo[i] + k, 1.0);
                e = lin_axpy(m->R[r][row], &uk, &e);
                qp_add_le(qp, &e, m->T[r][row]);
            }
        }
        for (int k = K[i] + 1; k <= N; ++k) { /* reachable interval of relaxed v_k (v_K's is implied) */
            lin v = CX(CL, x0, N, i, k, 1);
            if (RX[i].vhi[k] < RX[i].bhi) qp_add_le(qp, &v, RX[i].vhi[k]);
            lin nv = lin_axpy(-1.0, &v, &(lin){.n = 0, .cst = 0.0});
            if (RX[i].vlo[k] > RX[i].blo) qp_add_le(qp, &nv, -RX[i].vlo[k]);
        }
        for (int k = 1; k <= N; ++k)
            for (int row = 0; row < m->nd; ++row) {
                lin e = lin_const(0.0);
                for (int j = 0; j < 2; ++j) { lin xj = CX(CL, x0, N, i, k, j); e = lin_axpy(m->D[row][j], &xj, &e); }
                qp_add_le(qp, &e, m->E[row]);
            }
        for (int k = 0; k < N; ++k)
            for (int row = 0; row < m->nf; ++row) {
                lin e = lin_const(0.0);
                lin_add(&e, CL->uo[i] + k, m->F[row]);
                qp_add_le(qp, &e, m->G[row]);
            }
        for (int k = 0; k < N; ++k) {
            lin v1 = CX(CL, x0, N, i, k + 1, 1), v0 = CX(CL, x0, N, i, k, 1);
            lin dv = lin_axpy(-1.0, &v0, &v1);
            lin ndv = lin_axpy(-1.0, &dv, &(lin){.n = 0, .cst = 0.0});
            qp_add_le(qp, &ndv, -(cf->a_dec * cf->ts) - k * cf->tight);
            qp_add_le(qp, &dv, cf->a_acc * cf->ts - k * cf->tight);
        }
        if (CL->so[i] >= 0)
            for (int k = 0; k <= N; ++k) {
                lin s = lin_const(0.0);
                lin_add(&s, CL->so[i] + k, 1.0);
                lin ns = lin_axpy(-1.0, &s, &(lin){.n = 0, .cst = 0.0});
                qp_add_le(qp, &ns, 0.0);
                lin pk = CX(CL, x0, N, i, k, 0);
                lin e = lin_axpy(-1.0, &s, &pk); /* p_i - s <= p_{i-1} - d_safe  (or x_ref) */
                if (i >= 1) {
                    lin pm = CX(CL, x0, N, i - 1, k, 0);
                    e = lin_axpy(-1.0, &pm, &e);
                    qp_add_le(qp, &e, -cf->d_safe);
                } else {
                    qp_add_le(qp, &e, par(xl, N, 0, k) - cf->d_safe);
                }
                lin ws = lin_axpy(cf->w, &s, &(lin){.n = 0, .cst = 0.0});
                qp_add_lin(qp, &ws);
            }
    }
    /* tracking: leader and chain terms, k = 0..N.  min_1_norm: every |Q_ii e_i| term gets its
     * epigraph variable appended after the platoon's variables (add_norm through AL) */
    or_layout AL;
    memset(&AL, 0, sizeof(AL));
    AL.nsb_idx = nz;
    if (!cf->quadratic && nz + 2 * (N + 1) * n + 2 * n * N > OR_MAX_NZ) return 0;
    for (int k = 0; k <= N; ++k) {
        for (int i = 0; i < n; ++i) {
            lin p = CX(CL, x0, N, i, k, 0), v = CX(CL, x0, N, i, k, 1);
            lin e[2];
            if (i == CL->L) {
                if (CL->lsp) { e[0] = lin_axpy(cf->t0, &v, &p); e[0].cst += cf->d0; }
                else e[0] = p;
                e[0].cst -= par(xl, N, 0, k);
                e[1] = v; e[1].cst -= par(xl, N, 1, k);
                add_norm(qp, &AL, cf, e, cf->Qx, 2);
            }
            if (i >= 1) {
                lin pm = CX(CL, x0, N, i - 1, k, 0), vm = CX(CL, x0, N, i - 1, k, 1);
                e[0] = lin_axpy(cf->t0, &v, &p);
                e[0].cst += cf->d0;
                e[0] = lin_axpy(-1.0, &pm, &e[0]);
                e[1] = lin_axpy(-1.0, &vm, &v);
                add_norm(qp, &AL, cf, e, cf->Qx, 2);
            }
        }
    }
    double Qu[2][2] = {{cf->Qu, 0}, {0, 0}}, Qdu[2][2] = {{cf->Qdu, 0}, {0, 0}};
    for (int i = 0; i < n; ++i) {
        for (int k = 0; k < N; ++k) {
            if (k >= K[i] && RX[i].virt[k] < 0) continue;
            lin e[2]; e[0] = lin_const(0.0); lin_add(&e[0], CL->uo[i] + k, 1.0); e[1] = lin_const(0.0);
            add_norm(qp, &AL, cf, e, Qu, 1);
        }
        for (int k = 0; k + 1 < K[i]; ++k) {
            if (cf->Qdu == 0.0) continue;
            lin e[2]; e[0] = lin_const(0.0);
            lin_add(&e[0], CL->uo[i] + k + 1, 1.0);
            lin_add(&e[0], CL->uo[i] + k, -1.0);
            e[1] = lin_const(0.0);
            add_norm(qp, &AL, cf, e, Qdu, 1);
        }
    }
    qp->nz = nz + AL.naux;
    return qp->nz;
}

/* direct objective of a centralised solution z (relaxed steps without input cost) */
static double cent_objective(const or_cfg* cf, const or_cent_layout* CL, const int* K, const or_relax* RX,
                             const double* x0, const double* xl, const double* z) {
    const int N = cf->N, n = CL->n;
    double J = 0.0;
    for (int k = 0; k <= N; ++k)
        for (int i = 0; i < n; ++i) {
            double p = k ? z[CL->xo[i] + 2 * (k - 1)] : x0[2 * i], v = k ? z[CL->xo[i] + 2 * (k - 1) + 1] : x0[2 * i + 1];
            double e0, e1;
            /* min_2_norm e'Qe, min_1_norm sum_i |Q_ii e_i| (cent_mld.py:58-61) */
#define CENT_NORM(e0, e1) (cf->quadratic ? cf->Qx[0][0] * (e0) * (e0) + (cf->Qx[0][1] + cf->Qx[1][0]) * (e0) * (e1) + \
                                               cf->Qx[1][1] * (e1) * (e1)                                          \
                                         : fabs(cf->Qx[0][0] * (e0)) + fabs(cf->Qx[1][1] * (e1)))
            if (i == CL->L) {
                e0 = p - par(xl, N, 0, k) + (CL->lsp ? cf->t0 * v + cf->d0 : 0.0);
                e1 = v - par(xl, N, 1, k);
                J += CENT_NORM(e0, e1);
            }
            if (i >= 1) {
                double pm = k ? z[CL->xo[i - 1] + 2 * (k - 1)] : x0[2 * (i - 1)];
                double vm = k ? z[CL->xo[i - 1] + 2 * (k - 1) + 1] : x0[2 * (i - 1) + 1];
                e0 = p + cf->t0 * v + cf->d0 - pm;
                e1 = v - vm;
                J += CENT_NORM(e0, e1);
#undef CENT_NORM
                J += cf->w * fmax(0.0, p - pm + cf->d_safe);
            } else if (CL->lsp && CL->L == 0) {
                J += cf->w * fmax(0.0, p - par(xl, N, 0, k) + cf->d_safe);
            }
        }
    for (int i = 0; i < n; ++i)
        for (int k = 0; k < N; ++k) {
            if (k >= K[i] && RX[i].virt[k] < 0) continue;
            double u = z[CL->uo[i] + k];
            J += cf->quadratic ? cf->Qu * u * u : fabs(cf->Qu * u);
            if (k + 1 < K[i]) {
                double du = z[CL->uo[i] + k + 1] - u;
                J += cf->quadratic ? cf->Qdu * du * du : fabs(cf->Qdu * du);
            }
        }
    return J;
}

typedef struct {
    const or_model* md;
    const or_vmodel* vm;
    const or_cfg* cf;
    or_cent_layout CL;
    const double *x0, *xl;
    or_qp* qp;
    or_work* w;
    int n, N, maxit, n_qp, exhaustive;
    double inc;
    int best[OR_MAX_VEH * OR_MAX_N], have_best;
    long iters;
    int nleaf, capleaf; /* every leaf evaluated: the tie rule is applied at the end */
    double* leaf_obj;
    int* leaf_sig;
} or_cent;

/* lo, hi: per vehicle the exact interval of v_{K[i]} (the tail relaxation starts from it) */
static double cent_qp(or_cent* C, const int* sigma, const int* K, const double* lo, const double* hi, int leaf) {
    C->n_qp++;
    or_relax RX[OR_MAX_VEH];
    for (int i = 0; i < C->n; ++i) relax_tail(&C->vm[i], C->md[i].nreg, C->cf, K[i], lo[i], hi[i], &RX[i]);
    if (build_cent_qp(C->qp, C->md, C->cf, &C->CL, sigma, K, RX, C->x0, C->xl) <= 0 || C->qp->infeasible_const)
        return INFINITY;
    or_result r = ipm_solve(C->qp, C->w, C->maxit);
    C->iters += r.iters;
    if (!r.converged) return leaf ? INFINITY : -INFINITY;
    return cent_objective(C->cf, &C->CL, K, RX, C->x0, C->xl, C->w->z);
}

/* time-major decision order d -> (k = d / n, i = d % n); lexicographic key in that order */
static int cent_less(const int* a, const int* b, int n, int N) {
    for (int k = 0; k < N; ++k)
        for (int i = 0; i < n; ++i)
            if (a[i * N + k] != b[i * N + k]) return a[i * N + k] < b[i * N + k];
    return 0;
}

static void cent_leaf(or_cent* C, const int* sigma, const int* K, const double* lo, const double* hi) {
    double obj = cent_qp(C, sigma, K, lo, hi, 1);
    if (!isfinite(obj)) return;
    const int nN = C->n * C->N;
    if (C->nleaf == C->capleaf) {
        C->capleaf = C->capleaf ? 2 * C->capleaf : 64;
        C->leaf_obj = (double*)realloc(C->leaf_obj, sizeof(double) * C->capleaf);
        C->leaf_sig = (int*)realloc(C->leaf_sig, sizeof(int) * (size_t)C->capleaf * nN);
    }
    C->leaf_obj[C->nleaf] = obj;
    memcpy(C->leaf_sig + (size_t)C->nleaf * nN, sigma, sizeof(int) * nN);
    C->nleaf++;
    if (obj < C->inc) C->inc = obj;
    C->have_best = 1;
}

/* Pruning of the centralised search: gap = 0 is exact (bound above the incumbent by more than
 * 1e-7 (1 + |inc|), 100x the tie window); gap > 0 is Gurobi's relative MIPGap rule (the node
 * cannot improve the incumbent by more than gap |inc|; Gurobi's default is 1e-4). */
static double g_cent_gap = 0.0;
void oracle_set_cent_gap(double gap) { g_cent_gap = gap; }
static int cent_pruned(double lb, double inc) {
    if (g_cent_gap > 0.0) return lb >= inc - g_cent_gap * fabs(inc);
    return lb > inc + 1e-7 * (1.0 + fabs(inc));
}

/* QP budget of one oracle_solve_cent (0 = none): bench.py's bounded CPU sample of the search */
static long g_cent_cap = 0;
void oracle_set_cent_cap(long cap) { g_cent_cap = cap; }

static void cent_dfs(or_cent* C, int d, int* sigma, int* K, double* lo, double* hi) {
    const int n = C->n, N = C->N;
    if (g_cent_cap > 0 && C->n_qp >= g_cent_cap) return;
    if (d == n * N) { cent_leaf(C, sigma, K, lo, hi); return; }
    const int k = d / n, i = d % n;
    const or_vmodel* vm = &C->vm[i];
    const or_cfg* cf = C->cf;
    double dec = cf->a_dec * cf->ts + k * cf->tight, acc = cf->a_acc * cf->ts - k * cf->tight;
    int child[OR_MAX_REG], nch = 0;
    double clo[OR_MAX_REG], chi[OR_MAX_REG], lb[OR_MAX_REG];
    for (int r = 0; r < C->md[i].nreg; ++r) {
        if (!vm->rok[r]) continue;
        double ilo = fmax(lo[i], vm->rlo[r]), ihi = fmin(hi[i], vm->rhi[r]);
        if (ilo > ihi + 1e-9 * (1.0 + fabs(ihi))) continue;
        if (ilo > ihi) ilo = ihi = 0.5 * (ilo + ihi);
        double nlo, nhi;
        if (!next_interval(ilo, ihi, vm->a[r], vm->b[r], vm->c[r], vm->ul, vm->uh, dec, acc, vm->blo, vm->bhi, &nlo,
                           &nhi))
            continue;
        sigma[i * N + k] = r;
        K[i] = k + 1;
        const double slo = lo[i], shi = hi[i];
        lo[i] = nlo; hi[i] = nhi;
        lb[nch] = (d + 1 == n * N || C->exhaustive) ? 0.0 : cent_qp(C, sigma, K, lo, hi, 0);
        lo[i] = slo; hi[i] = shi;
        K[i] = k;
        child[nch] = r; clo[nch] = nlo; chi[nch] = nhi;
        nch++;
    }
    /* visit in increasing bound order (ties: lower region first) */
    for (int a = 0; a < nch; ++a) {
        int m = a;
        for (int b = a + 1; b < nch; ++b)
            if (lb[b] < lb[m] || (lb[b] == lb[m] && child[b] < child[m])) m = b;
        double tl = lb[a]; lb[a] = lb[m]; lb[m] = tl;
        int tc = child[a]; child[a] = child[m]; child[m] = tc;
        double t1 = clo[a]; clo[a] = clo[m]; clo[m] = t1;
        double t2 = chi[a]; chi[a] = chi[m]; chi[m] = t2;
    }
    for (int a = 0; a < nch; ++a) {
        if (C->have_best && cent_pruned(lb[a], C->inc)) continue;
        if (!(lb[a] < INFINITY)) continue;
        const double slo = lo[i], shi = hi[i];
        sigma[i * N + k] = child[a];
        K[i] = k + 1;
        lo[i] = clo[a]; hi[i] = chi[a];
        cent_dfs(C, d + 1, sigma, K, lo, hi);
        lo[i] = slo; hi[i] = shi;
        K[i] = k;
    }
}

/* Centralised MIQP of one platoon: sys models stacked per vehicle (as oracle_solve_batch), x0
 * (2n), xl (2, N+1), role = leader index | real_vehicle_as_reference << 8.  Outputs x (n, 2, N+1),
 * u (n, N), sigma (n, N), info = [objective, status (0 optimal, 1 infeasible), QPs solved].
 * role bit 16: exhaustive enumeration of the joint sequences instead of branch and bound; bit 17: the
 * min_1_norm cost (quadratic_cost=False, cent_mld.py:58-61). */
int oracle_solve_cent(int n, int N, int nreg, int nsr, const double* S, const double* R, const double* T,
                      const double* A, const double* B, const double* c, int nd, const double* D, const double* E, int nf,
                      const double* F, const double* G, const double* cfgp, int role, const double* x0,
                      const double* xl, double* x_out, double* u_out, int* sigma_out, double* info_out) {
    if (n < 1 || n > OR_MAX_VEH || N > OR_MAX_N) return -1;
    or_model md[OR_MAX_VEH];
    or_vmodel vm[OR_MAX_VEH];
    for (int i = 0; i < n; ++i) {
        const size_t so = (size_t)i * nreg * nsr, ao = (size_t)i * nreg;
        if (unpack_model(&md[i], nreg, nsr, S + 2 * so, R + so, T + so, A + 4 * ao, B + 2 * ao, c + 2 * ao, nd,
                         D + (size_t)i * 2 * nd, E + (size_t)i * nd, nf, F + (size_t)i * nf, G + (size_t)i * nf))
            return -1;
        if (make_vmodel(&md[i], &vm[i]) || !oracle_bnb_ok(&md[i])) return -2;
    }
    or_cfg cf;
    unpack_cfg(&cf, N, (role >> 17) & 1 ? 0 : 1, 0, cfgp); /* role bit 17: min_1_norm (the MILP) */
    or_cent* C = (or_cent*)calloc(1, sizeof(or_cent));
    or_qp* qp = (or_qp*)malloc(sizeof(or_qp));
    or_work* w = (or_work*)malloc(sizeof(or_work));
    if (!C || !qp || !w) { free(C); free(qp); free(w); return -3; }
    C->md = md; C->vm = vm; C->cf = &cf; C->x0 = x0; C->xl = xl; C->qp = qp; C->w = w;
    C->n = n; C->N = N; C->maxit = 200; C->inc = INFINITY;
    C->CL.n = n; C->CL.L = role & 0xff; C->CL.lsp = (role >> 8) & 1;
    C->exhaustive = (role >> 16) & 1; /* every velocity-feasible joint sequence (cross-check) */
    int sigma[OR_MAX_VEH * OR_MAX_N] = {0}, K[OR_MAX_VEH] = {0};
    double lo[OR_MAX_VEH], hi[OR_MAX_VEH];
    for (int i = 0; i < n; ++i) lo[i] = hi[i] = x0[2 * i + 1];
    cent_dfs(C, 0, sigma, K, lo, hi);
    if (C->have_best) { /* lexicographically first (time-major) leaf within 1e-9 relative of the minimum */
        const double tol = 1e-9 * fmax(1.0, fabs(C->inc));
        int win = -1;
        for (int l = 0; l < C->nleaf; ++l) {
            if (!(C->leaf_obj[l] <= C->inc + tol)) continue;
            if (win < 0 || cent_less(C->leaf_sig + (size_t)l * n * N, C->leaf_sig + (size_t)win * n * N, n, N)) win = l;
        }
        memcpy(C->best, C->leaf_sig + (size_t)win * n * N, sizeof(int) * n * N);
    }
    free(C->leaf_obj);
    free(C->leaf_sig);
    info_out[0] = C->have_best ? C->inc : INFINITY;
    info_out[1] = C->have_best ? 0 : 1;
    info_out[2] = C->n_qp;
    if (C->have_best) {
        for (int i = 0; i < n; ++i) {
            K[i] = N;
            for (int k = 0; k < N; ++k) sigma_out[i * N + k] = C->best[i * N + k];
        }
        /* re-evaluate the winner for its exact objective and trajectory */
        double obj = cent_qp(C, C->best, K, lo, hi, 1);
        info_out[0] = obj;
        for (int i = 0; i < n; ++i) {
            x_out[i * 2 * (N + 1)] = x0[2 * i];
            x_out[i * 2 * (N + 1) + N + 1] = x0[2 * i + 1];
            for (int k = 1; k <= N; ++k) {
                x_out[i * 2 * (N + 1) + k] = w->z[C->CL.xo[i] + 2 * (k - 1)];
                x_out[i * 2 * (N + 1) + N + 1 + k] = w->z[C->CL.xo[i] + 2 * (k - 1) + 1];
            }
            for (int k = 0; k < N; ++k) u_out[i * N + k] = w->z[C->CL.uo[i] + k];
        }
    }
    free(C); free(qp); free(w);
    return 0;
}
