// hvp_hostref.cpp -- TEST-ONLY host build of the lane algorithm in hvp_ipm.h.
//
// Compiled with g++ into lib/libhvp_hostref.so and loaded only by tests/ (to exercise the
// enumeration + per-lane IPM logic on a machine without a GPU) and by bench.py's extra
// "same algorithm on the host cores" baseline.  The product entry points live in
// libhvpsolve.so (hvp_kernels.hip) and never call into this library.
#include <stdio.h>
#include <string.h>

#include <map>
#include <vector>

#include "hvp_admm.h"
#include "hvp_bnb.h"
#include "hvp_gi.h"
#include "hvp_ipm.h"
#include "hvp_l1.h"
long long g_lp_why[5] = {0, 0, 0, 0, 0};
long long g_lp_pass = 0;
int g_admm_leaf_ipm = 0;  // hvp_hostref_set_admm_leaf_ipm: 1 every ADMM leaf by the interior point, 2 the
                          // device's HVP_LEAF_GI_CAP=2 (two active-set steps, then the interior point)  // ratio-test scans over the terms
#define HVP_LP_PASS() (__atomic_fetch_add(&g_lp_pass, 1, __ATOMIC_RELAXED))
#define HVP_LP_WHY(code) (__atomic_fetch_add(&g_lp_why[code], 1, __ATOMIC_RELAXED))
int g_lp_trace = 0;
// hvp_hostref_set_admm_warm (diagnostics, profiles/diag_admm_warm.py): starting hinge states of the
// naive-ADMM node QPs -- 0 constant-velocity (cold), 1 a child from its parent's final states,
// 2 as 1 and the root from the previous call's root states of the same batch index,
// 3 every node QP from the record of the same node (batch index, depth, region code) of the
// previous call: its final hinge states and active set (forced in as equalities, negative
// multipliers dropped), as a factor-carrying warm start would begin -- counted as one iteration
int g_admm_warm = 0;
struct WarmRec {
    uint64_t hs;
    int nact;
    int ids[16];
};
std::map<std::pair<uint64_t, int>, WarmRec> g_admm_recs[4096];
long long g_admm_rec_stats[4];  // lookups, hits, warm starts kept (dual feasible after the drops)
// 4: as 3 through a direct-mapped table per (batch index, depth) of g_admm_slots records, slot =
// hash(code); among a level's nodes that share a slot the smallest code owns it (reads and
// writes it), the others start cold -- the device's deterministic claim
int g_admm_slots = 64;
struct SlotRec {
    bool valid;
    uint64_t code;
    WarmRec rec;
};
std::vector<SlotRec> g_admm_tab[4096];
inline int admm_slot(uint64_t code, int sd) {
    return (int)((code * 0x9E3779B97F4A7C15ull) >> 40) & (sd - 1);
}
uint64_t g_admm_root_hs[4096];
long long g_admm_warm_stats[4];  // QPs, hinge rounds, QPs consistent in one round, failed
#define HVP_LP_TRACE(it, lv, sd, dv, en, t, bl, yy)                                                             \
    do {                                                                                                      \
        if (g_lp_trace)                                                                                       \
            fprintf(stderr, "[lp] it %d leave %d side %d D %.6e enter %d t %.6e bland %d y0 %.12f y1 %.12f\n", \
                    (int)(it), (int)(lv), (int)(sd), (double)(dv), (int)(en), (double)(t), (int)(bl), (yy)[0], (yy)[1]); \
    } while (0)
#include "hvp_lp.h"

namespace {

constexpr int kAutoEnumMaxN = 0;    // same crossovers as hvp_lane.h (HVP_METHOD_AUTO)
constexpr int kAutoEnumMaxNL1 = 0;

// 0: interior point only; 1: Goldfarb-Idnani active set, interior point on failure
int g_solver = 1;
// min_1_norm LPs: 0 the interior point (hvp_l1.h l1_solve), 1 as the product: the simplex
// (hvp_lp.h) up to N = 8, the interior point beyond (the device's wave kernels)
int g_l1_solver = 1;
long long g_lp_runs = 0, g_lp_iters = 0, g_lp_fail = 0;
long long g_lp_hist[64] = {};  // LPs by pivot count (the lane-utilisation model of the LP kernels)
long long g_lp_pc[32][32] = {};  // branch-and-bound node LPs by (parent's pivots, own pivots), capped at 31
long long g_bnb_nch[17][8] = {};  // unpruned branch-and-bound nodes by depth and number of children (7 = 7+)

// one min_1_norm LP (node: K < N with the reachable interval [lo, hi] of v_K) by the selected solver
template <int N>
int l1_lp(const hvp_system& S, const hvp::Consts& C, int role, const double* prm, uint64_t code, int K, double lo,
          double hi, double* y, int& it) {
    if (g_l1_solver == 1 && N <= HVP_MAX_N_ENUM) {
        hvp::LpData<N> D;
        const int st = hvp::lp_solve_l1<N>(D, S, C, role, prm, code, K, lo, hi, C.max_iter, y, it);
#pragma omp atomic
        g_lp_runs += 1;
#pragma omp atomic
        g_lp_iters += it;
#pragma omp atomic
        g_lp_hist[it < 63 ? it : 63] += 1;
        if (st == hvp::L1_FAIL) {
#pragma omp atomic
            g_lp_fail += 1;
        }
        return st;
    }
    hvp::L1Lp<N> lp;
    hvp::l1_setup<N>(lp, S, C, role, prm, code, K, lo, hi);
    for (int i = 0; i < N; ++i) lp.y[i] = prm[1];
    const int st = hvp::l1_infeasible<N>(S, C, prm, code, K, lo, hi)
                       ? hvp::L1_INFEASIBLE
                       : hvp::l1_solve<N>(lp, prm[1], C.max_iter, it, S.vmin, S.vmax);
    for (int i = 0; i < N; ++i) y[i] = lp.y[i];
    return st;
}
long long g_gi_fail = 0, g_gi_iters = 0, g_gi_runs = 0, g_gi_code[4] = {0, 0, 0, 0};

hvp::Consts make_consts(const hvp_problem& p) {
    hvp::Consts C;
    memset(&C, 0, sizeof(C));
    C.Qpp = p.Qx[0];
    C.Qpv = 0.5 * (p.Qx[1] + p.Qx[2]);
    C.Qvv = p.Qx[3];
    C.Qu = p.Qu;
    C.Qdu = p.Qdu;
    C.w = p.w;
    C.d_safe = p.d_safe;
    C.d0 = p.spacing_d0;
    C.t0 = p.spacing_t0;
    for (int k = 0; k < HVP_MAX_N; ++k) {
        C.dec[k] = p.a_dec * p.ts_acc + k * p.accel_tightening;
        C.acc[k] = p.a_acc * p.ts_acc - k * p.accel_tightening;
    }
    C.tol = p.tol > 0 ? p.tol : 1e-12;
    C.max_iter = p.max_iter > 0 ? p.max_iter : (p.quadratic_cost ? 60 : hvp::kL1MaxIter);
    C.N = p.N;
    C.form = p.formulation;
    C.stride = p.formulation == HVP_FORM_ADMM    ? hvp_params_stride_admm(p.N)
               : p.formulation == HVP_FORM_GADMM ? hvp_params_stride_gadmm(p.N)
                                                 : hvp_params_stride(p.N);
    C.rho = p.rho;
    C.l1 = p.quadratic_cost ? 0 : 1;
    return C;
}

template <int N>
void solve_one(const hvp_system& S, const hvp::Consts& C, int role, const double* prm, double* u, double* x,
               int8_t* region, double* cost, int32_t* status, int32_t* nodes, int32_t* iters, double* cand_cost,
               uint32_t* cand_code, int cand_cap) {
    struct Cand {
        uint32_t code;
        double cost;
        int status, iters;
        double y[N];
    };
    std::vector<Cand> cands;
    hvp::LaneQp<N> probe;
    const bool ok = hvp::setup_lane<N>(probe, S, C, role, prm, 0u);
    int n = 0;
    if (ok) {
        n = hvp::enumerate_sequences(S, C, prm[1], [&](uint32_t code, int) {
            hvp::LaneQp<N> q;
            if (C.l1) {  // min_1_norm: the fixed-sequence LP (hvp_l1.h / hvp_lp.h)
                Cand c;
                c.code = code;
                c.iters = 0;
                c.status = l1_lp<N>(S, C, role, prm, code, N, 0.0, -1.0, c.y, c.iters);
                c.cost = c.status == 0 ? hvp::l1_direct_cost<N>(c.y, S, C, role, prm, code) : 1e300;
                cands.push_back(c);
                return;
            }
            hvp::setup_lane<N>(q, S, C, role, prm, code);
            hvp::QpOut o;
            bool gi_done = false;
            if (g_solver == 1) {
                int it = 0;
                const int r = hvp::solve_gi<N>(q, C, 8 * hvp::GiConstraintSet<N>::NC, it);
#pragma omp atomic
                g_gi_runs += 1;
#pragma omp atomic
                g_gi_iters += it;
                if (r == hvp::GI_OK) {
                    o.status = 0;
                    o.iters = it;
                    o.cost = 0.0;
                    gi_done = true;
                } else {
#pragma omp atomic
                    g_gi_fail += 1;
#pragma omp atomic
                    g_gi_code[r - hvp::GI_FAIL_CHOL] += 1;
                    hvp::setup_lane<N>(q, S, C, role, prm, code);
                }
            }
            if (!gi_done) o = hvp::Solver<N, false>::solve(q, C);
            if (!gi_done && o.status == 0 && !hvp::pbox_ok<N>(q)) {
                // relaxed optimum leaves the position box: solve the full QP (exact fallback)
                hvp::setup_lane<N>(q, S, C, role, prm, code);
                const int it0 = o.iters;
                o = hvp::Solver<N, true>::solve(q, C);
                o.iters += it0;
            }
            Cand c;
            c.code = code;
            c.cost = o.status == 0 ? hvp::direct_cost<N>(q, S, C, role, prm, code) : o.cost;
            c.status = o.status;
            c.iters = o.iters;
            for (int i = 0; i < N; ++i) c.y[i] = q.y[i];
            cands.push_back(c);
        });
    }
    double best = 1e300;
    int tot = 0;
    bool unresolved = false;  // min_1_norm: an LP neither solved nor proven infeasible (k_select)
    for (const Cand& c : cands) {
        tot += c.iters;
        if (c.status == 0 && c.cost < best) best = c.cost;
        unresolved = unresolved || (C.l1 && c.status == hvp::L1_FAIL);
    }
    int win = -1;
    if (best < 1e300 && !unresolved) {
        const double tol = 1e-9 * fmax(1.0, fabs(best));
        for (size_t i = 0; i < cands.size(); ++i)
            if (cands[i].status == 0 && cands[i].cost <= best + tol) { win = (int)i; break; }
    }
    for (int i = 0; i < (int)cands.size() && i < cand_cap; ++i) {
        if (cand_cost) cand_cost[i] = cands[i].status == 0 ? cands[i].cost : 1e300;
        if (cand_code) cand_code[i] = cands[i].code;
    }
    *nodes = n;
    *iters = tot;
    if (win < 0) {
        // min_1_norm: every LP proven infeasible -> infeasible; an unresolved one -> MAXITER
        *status = (!ok || n == 0 || (C.l1 && !unresolved)) ? HVP_INFEASIBLE : HVP_MAXITER;
        *cost = 1e300;
        return;
    }
    const Cand& c = cands[win];
    *status = HVP_OPTIMAL;
    *cost = c.cost;
    const double p0 = prm[0], v0 = prm[1];
    x[0] = p0;
    x[N + 1] = v0;
    double p = p0, v = v0;
    for (int k = 0; k < N; ++k) {
        const int r = hvp::code_region(c.code, k);
        region[k] = (int8_t)r;
        const double vn = c.y[k];
        u[k] = (vn - S.a[r] * v - S.c[r]) / S.b[r];
        p = p + S.ts * v;
        v = vn;
        x[k + 1] = p;
        x[N + 1 + k + 1] = v;
    }
}

// diagnostics (g_admm_warm == 3): the hinge-state iteration of hvp_admm.h solve_admm_lane started
// from a record of the same node's previous solve
template <int N>
int admm_warm_solve(hvp::LaneQp<N>& q, const hvp_system& S, const hvp::Consts& C, int role, const double* prm,
                    uint64_t code, int K, int max_iter, int& iters, int& rounds, WarmRec& rec, bool have) {
    uint64_t hs;
    iters = 0;
    if (have) {
        hs = rec.hs;
    } else {
        double y[N];
        for (int k = 0; k < N; ++k) y[k] = prm[1];
        bool c;
        hs = hvp::admm_classify<N>(C, role, prm, prm[0] + S.ts * prm[1], S.ts, y, 0, &c);
    }
    for (int round = 0; round < hvp::kHubRounds; ++round) {
        rounds = round + 1;
        hvp::setup_lane_admm<N>(q, S, C, role, prm, code, K, hs);
        hvp::GiLane<N> g;
        if (g.init(q) != hvp::GI_OK) return hvp::GI_FAIL_CHOL;
        if (round == 0 && have && rec.hs == hs) {
            bool drop[16] = {};
            bool dual_ok = false;
            for (int attempt = 0; attempt < 4 && !dual_ok; ++attempt) {
                if (attempt) g.init(q);
                for (int j = 0; j < rec.nact; ++j)
                    if (!drop[j]) hvp::gi_force_add<N>(g, q, C, rec.ids[j]);
                dual_ok = true;
                for (int j = 0; j < g.nact; ++j)
                    if (g.u[j] < -1e-9 * C.w)
                        for (int i = 0; i < rec.nact; ++i)
                            if (rec.ids[i] == g.ids[j]) { drop[i] = true; dual_ok = false; }
                if (attempt == 0 && dual_ok) {
#pragma omp atomic
                    g_admm_rec_stats[3] += 1;
                }
            }
            iters += 1;  // the warm start itself
            if (!dual_ok) g.init(q);
#pragma omp atomic
            g_admm_rec_stats[2] += dual_ok ? 1 : 0;
        }
        int it = 0;
        const int st = hvp::gi_run<N>(g, q, C, max_iter, it, nullptr);
        iters += it;
        if (st != hvp::GI_OK) return st;
        bool consistent;
        const uint64_t hs2 = hvp::admm_classify<N>(C, role, prm, q.P1, q.ts, q.y, hs, &consistent);
        if (consistent) {
            rec.hs = hs;
            rec.nact = g.nact;
            for (int j = 0; j < g.nact && j < 16; ++j) rec.ids[j] = g.ids[j];
            return hvp::GI_OK;
        }
        hs = hs2;
    }
    return hvp::GI_FAIL_ITER;
}

// Branch and bound (hvp_bnb.h) with the same level-synchronous order as the gfx950 kernels:
// root bound + greedy dive, then per depth the children of the unpruned nodes, then the argmin
// and tie rule over the leaves.
template <int N>
void solve_one_bnb(const hvp_system& S, const hvp::Consts& C, int role, const double* prm, double* u, double* x,
                   int8_t* region, double* cost, int32_t* status, int32_t* nodes, int32_t* iters,
                   double* xf = nullptr, double* xb = nullptr, int idx = -1) {
    struct Node {
        uint64_t code;
        double lo, hi, lb;
        int stat;
        double y[N];
        uint64_t hs;
        int pit;  // min_1_norm: pivots of this node's LP (g_lp_pc, the parent / child correlation)
    };
    int nq = 0, nit = 0, last_it = 0;
    int l1_st = 0;  // status of the last min_1_norm LP (hvp_l1.h L1_*)
    const int SD = g_admm_slots;
    std::vector<uint64_t> claim;  // g_admm_warm == 4: owner code per (depth, slot) of this solve
    bool root_phase = true;
    if (g_admm_warm == 4 && idx >= 0 && idx < 4096) {
        claim.assign((size_t)(N + 1) * SD, ~0ull);
        if (g_admm_tab[idx].size() != (size_t)(N + 1) * SD) g_admm_tab[idx].assign((size_t)(N + 1) * SD, SlotRec{});
    }
    auto qp = [&](uint64_t code, int K, double lo, double hi, double& c, double* y, uint64_t* hs = nullptr) {
        hvp::LaneQp<N> q;
        int it = 0;
        if (C.l1) {  // min_1_norm: the node LP (relaxed after K steps), as k_l1_root / k_l1_bound
            double yl[N];
            l1_st = l1_lp<N>(S, C, role, prm, code, K, lo, hi, yl, it);
            ++nq;
            nit += it;
            last_it = it;
            if (l1_st != hvp::L1_OK) return false;
            c = hvp::l1_direct_cost<N>(yl, S, C, role, prm, code, K, lo, hi);
            if (y)
                for (int i = 0; i < N; ++i) y[i] = yl[i];
            return true;
        }
        if (C.form == HVP_FORM_ADMM) {
            // g_admm_leaf_ipm (tests): the leaves by the interior-point fallback (hvp_admm.h
            // solve_admm_ipm), as HVP_LEAF_GI_CAP forces on the device
            // (2: the leaves' active-set steps capped at 2, the interior point where that fails)
            int rounds = 0;
            if ((g_admm_warm == 3 || g_admm_warm == 4) && idx >= 0 && idx < 4096 && !g_admm_leaf_ipm) {
                auto& recs = g_admm_recs[idx];
                const auto key = std::make_pair(code, K);
                bool have;
                WarmRec rec{};
                SlotRec* sr = nullptr;
                if (g_admm_warm == 3) {
                    auto f = recs.find(key);
                    have = f != recs.end();
                    if (have) rec = f->second;
                } else {
                    const size_t si = (size_t)K * SD + admm_slot(code, SD);
                    const bool owner = K == 0 || (K == N && root_phase) || claim[si] == code;
                    sr = owner ? &g_admm_tab[idx][si] : nullptr;
                    have = sr && sr->valid && sr->code == code;
                    if (have) rec = sr->rec;
                }
#pragma omp atomic
                g_admm_rec_stats[0] += 1;
#pragma omp atomic
                g_admm_rec_stats[1] += have ? 1 : 0;
                const int r = admm_warm_solve<N>(q, S, C, role, prm, code, K, 8 * hvp::GiConstraintSet<N>::NC, it,
                                                 rounds, rec, have);
#pragma omp atomic
                g_admm_warm_stats[0] += 1;
#pragma omp atomic
                g_admm_warm_stats[1] += rounds;
                ++nq;
                nit += it;
                if (r != hvp::GI_OK) {
#pragma omp atomic
                    g_admm_warm_stats[3] += 1;
                    return false;
                }
                if (g_admm_warm == 3) recs[key] = rec;
                else if (sr) *sr = SlotRec{true, code, rec};
                c = hvp::admm_direct_cost<N>(q, S, C, role, prm, code, K);
                if (y)
                    for (int i = 0; i < N; ++i) y[i] = q.y[i];
                return true;
            }
            int r = g_admm_leaf_ipm == 1 && K == N
                        ? hvp::solve_admm_ipm<N>(q, S, C, role, prm, code, K, it)
                        : hvp::solve_admm_lane<N>(q, S, C, role, prm, code, K,
                                                   g_admm_leaf_ipm == 2 && K == N ? 2 : 8 * hvp::GiConstraintSet<N>::NC, it,
                                                   nullptr, g_admm_warm ? hs : nullptr, &rounds);
#pragma omp atomic
            g_admm_warm_stats[0] += 1;
#pragma omp atomic
            g_admm_warm_stats[1] += rounds;
            if (r == hvp::GI_OK && rounds == 1) {
#pragma omp atomic
                g_admm_warm_stats[2] += 1;
            }
            if (r != hvp::GI_OK) {
#pragma omp atomic
                g_admm_warm_stats[3] += 1;
            }
            if (r != hvp::GI_OK && g_admm_leaf_ipm == 2 && K == N) {
                int it2 = 0;
                r = hvp::solve_admm_ipm<N>(q, S, C, role, prm, code, K, it2);
                it += it2;
            }
            ++nq;
            nit += it;
            if (r != hvp::GI_OK) return false;
            c = hvp::admm_direct_cost<N>(q, S, C, role, prm, code, K);
            if (y)
                for (int i = 0; i < N; ++i) y[i] = q.y[i];
            return true;
        }
        hvp::setup_lane<N>(q, S, C, role, prm, code, K, lo, hi);
        const int r = hvp::solve_gi<N>(q, C, 8 * hvp::GiConstraintSet<N>::NC, it);
        ++nq;
        nit += it;
        if (r != hvp::GI_OK) {
            // leaves get the interior-point fallback (K_bnb_ipm on the device)
            if (K < N || N > HVP_MAX_N_ENUM) return false;
            hvp::setup_lane<N>(q, S, C, role, prm, code, K, lo, hi);
            const hvp::QpOut o = hvp::Solver<N, true>::solve(q, C);
            nit += o.iters;
            if (o.status != 0) return false;
        }
        c = hvp::direct_cost<N>(q, S, C, role, prm, code, K);
        if (y)
            for (int i = 0; i < N; ++i) y[i] = q.y[i];
        return true;
    };
    const double v0 = prm[1], P1 = prm[0] + S.ts * v0;
    const bool ok = P1 >= S.pmin - 1e-9 * (1.0 + fabs(S.pmin)) && P1 <= S.pmax + 1e-9 * (1.0 + fabs(S.pmax));
    std::vector<Node> lvl, nxt;
    double inc = HUGE_VAL;
    int nleaves = 0;
    if (ok) {
        Node root;
        root.code = 0;
        root.lo = root.hi = v0;
        root.lb = -1e300;
        root.hs = g_admm_warm == 2 && idx >= 0 && idx < 4096 ? g_admm_root_hs[idx] : hvp::kHubNone;
        double c0;
        const bool root_ok = qp(0, 0, v0, v0, c0, root.y, &root.hs);
        root.pit = last_it;
        if (root_ok) {
            root.lb = c0;
            if (g_admm_warm == 2 && idx >= 0 && idx < 4096) g_admm_root_hs[idx] = root.hs;
            uint64_t code;
            double c1;
            uint64_t dhs = root.hs;
            if (hvp::bnb_dive<N>(S, C, v0, root.y, &code) && qp(code, N, 0.0, -1.0, c1, nullptr, &dhs)) inc = c1;
            if (C.l1 && g_l1_solver == 1 && N <= HVP_MAX_N_ENUM) {
                // the simplex's root optimum is a vertex (an extreme point where the LP optimum is a
                // face): a second dive towards the constant-velocity trajectory (k_lp_root)
                double yt[N];
                for (int i = 0; i < N; ++i) yt[i] = v0;
                uint64_t code2;
                double c2;
                if (hvp::bnb_dive<N>(S, C, v0, yt, &code2) && code2 != code && qp(code2, N, 0.0, -1.0, c2, nullptr))
                    inc = fmin(inc, c2);
            }
        } else if (C.l1 && l1_st == hvp::L1_INFEASIBLE) {
            root.lb = 1e300;  // the root relaxation is infeasible: so is every sequence
        }
        lvl.push_back(root);
    }
    for (int k = 1; k <= N && !lvl.empty(); ++k) {
        nxt.clear();
        for (const Node& p : lvl) {
            if (hvp::bnb_pruned(p.lb, inc)) continue;
            int nch = 0;
            for (int r = 0; r < S.n_regions; ++r) {
                double a, b;
                nch += hvp::bnb_child(S, C, k - 1, p.lo, p.hi, r, &a, &b) ? 1 : 0;
            }
#pragma omp atomic
            g_bnb_nch[k - 1][nch < 7 ? nch : 7] += 1;
            for (int r = 0; r < S.n_regions; ++r) {
                Node c;
                if (!hvp::bnb_child(S, C, k - 1, p.lo, p.hi, r, &c.lo, &c.hi)) continue;
                c.code = hvp::code_with(p.code, k - 1, r);
                c.lb = p.lb;
                c.hs = p.hs;
                c.pit = p.pit;
                nxt.push_back(c);
            }
        }
        if (k == N) nleaves += (int)nxt.size();
        root_phase = false;
        if (!claim.empty())
            for (const Node& c : nxt) {
                uint64_t& w = claim[(size_t)k * SD + admm_slot(c.code, SD)];
                w = c.code < w ? c.code : w;
            }
        for (Node& c : nxt) {
            double lb;
            const double plb = c.lb;  // the parent's bound (min_1_norm: kept by an unresolved leaf)
            const bool good = qp(c.code, k, c.lo, c.hi, lb, c.y, &c.hs);
            if (C.l1) {
#pragma omp atomic
                g_lp_pc[c.pit < 31 ? c.pit : 31][last_it < 31 ? last_it : 31] += 1;
                c.pit = last_it;
            }
            c.stat = good ? 0 : HVP_MAXITER;
            c.lb = good ? lb : (k < N ? -1e300 : 1e300);
            if (!good && C.l1) {
                const bool infeasible = l1_st == hvp::L1_INFEASIBLE;
                c.stat = infeasible ? HVP_INFEASIBLE : HVP_MAXITER;
                c.lb = k < N ? (infeasible ? 1e300 : -1e300) : (infeasible ? 1e300 : plb);
            }
            if (k == N && good) inc = fmin(inc, lb);
        }
        lvl.swap(nxt);
    }
    *nodes = nq;
    *iters = nit;
    int win = -1;
    uint64_t wkey = ~0ull;
    bool contention = false;  // min_1_norm: an unresolved leaf that may hold the optimum (k_bnb_key)
    if (C.l1)
        for (const Node& c : lvl)
            contention = contention || (c.stat == HVP_MAXITER && !hvp::bnb_pruned(c.lb, inc));
    if (ok && inc < HUGE_VAL && !contention) {
        for (int i = 0; i < (int)lvl.size(); ++i) {
            const Node& c = lvl[i];
            if (c.stat != 0 || c.lb > inc + 1e-9 * fmax(1.0, fabs(inc))) continue;
            const uint64_t key = hvp::bnb_lexkey(c.code, N);
            if (key < wkey) { wkey = key; win = i; }
        }
    }
    if (win < 0) {
        bool unresolved = false;  // min_1_norm: only an unresolved leaf makes it MAXITER (k_bnb_finish)
        for (const Node& c : lvl) unresolved = unresolved || c.stat == HVP_MAXITER;
        *status = C.l1 ? (unresolved ? HVP_MAXITER : HVP_INFEASIBLE)
                       : ((ok && !lvl.empty() && lvl.size() > 0 && nleaves > 0) ? HVP_MAXITER : HVP_INFEASIBLE);
        *cost = 1e300;
        if (xf) memset(xf, 0, sizeof(double) * 2 * (N + 1));
        if (xb) memset(xb, 0, sizeof(double) * 2 * (N + 1));
        return;
    }
    const Node& c = lvl[win];
    *status = HVP_OPTIMAL;
    *cost = c.lb;
    x[0] = prm[0];
    x[N + 1] = v0;
    double p = prm[0], v = v0;
    for (int k = 0; k < N; ++k) {
        const int r = hvp::code_region(c.code, k);
        region[k] = (int8_t)r;
        const double vn = c.y[k];
        u[k] = (vn - S.a[r] * v - S.c[r]) / S.b[r];
        p = p + S.ts * v;
        v = vn;
        x[k + 1] = p;
        x[N + 1 + k + 1] = v;
    }
    if (C.form == HVP_FORM_ADMM) {
        const bool on[2] = {(role & HVP_ROLE_SAFE_FRONT) != 0, (role & HVP_ROLE_SAFE_BACK) != 0};
        const bool tr[2] = {(role & HVP_ROLE_TRACK_FRONT) != 0, (role & HVP_ROLE_TRACK_BACK) != 0};
        double* outs[2] = {xf, xb};
        for (int side = 0; side < 2; ++side) {
            if (!outs[side]) continue;
            for (int k = 0; k <= N; ++k) {
                double e = 0.0, g = 0.0;
                if (on[side])
                    hvp::admm_copy_value(C, tr[side], side, hvp::admm_y(prm, side, N)[k],
                                         hvp::admm_y(prm, side, N)[N + 1 + k], hvp::admm_z(prm, side, N)[k],
                                         hvp::admm_z(prm, side, N)[N + 1 + k], x[k], x[N + 1 + k], &e, &g);
                outs[side][k] = e;
                outs[side][N + 1 + k] = g;
            }
        }
    }
}

template <int N>
void solve_range(const hvp_problem& P, const hvp_system* systems, int B, const int32_t* sys, const int32_t* role,
                 const double* params, double* u, double* x, int8_t* region, double* cost, int32_t* status,
                 int32_t* nodes, int32_t* iters, int nthreads, double* xf = nullptr, double* xb = nullptr) {
    const hvp::Consts C = make_consts(P);
    const int stride = C.stride;
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1)
    for (int i = 0; i < B; ++i) {
        const bool bnb = P.method == HVP_METHOD_BNB ||
                         (P.method == HVP_METHOD_AUTO && N > (C.l1 ? kAutoEnumMaxNL1 : kAutoEnumMaxN));
        if (bnb || N > HVP_MAX_N_ENUM || C.form == HVP_FORM_ADMM) {
            solve_one_bnb<N>(systems[sys[i]], C, role[i], params + (size_t)i * stride, u + (size_t)i * N,
                             x + (size_t)i * 2 * (N + 1), region + (size_t)i * N, cost + i, status + i, nodes + i,
                             iters + i, xf ? xf + (size_t)i * 2 * (N + 1) : nullptr,
                             xb ? xb + (size_t)i * 2 * (N + 1) : nullptr, i);
            continue;
        }
        if constexpr (N <= HVP_MAX_N_ENUM)
            solve_one<N>(systems[sys[i]], C, role[i], params + (size_t)i * stride, u + (size_t)i * N,
                     x + (size_t)i * 2 * (N + 1), region + (size_t)i * N, cost + i, status + i, nodes + i, iters + i,
                     nullptr, nullptr, 0);
    }
}

// switching-ADMM local QP of one vehicle for its sequence (the lane path of k_gadmm_qp)
template <int N>
void gadmm_one(const hvp_system& S, const hvp::Consts& C, int role, const double* prm, const int8_t* seq, double* u,
               double* x, double* xf, double* xb, double* cost, int32_t* status, uint32_t* edge) {
    uint64_t code = 0;
    for (int k = 0; k < N; ++k) code = hvp::code_with(code, k, seq[k]);
    hvp::LaneQp<N> q;
    int it = 0;
    uint32_t raw = 0;
    // g_admm_leaf_ipm: 1 every local QP by the interior-point fallback, 2 the device's
    // HVP_LEAF_GI_CAP=2 (two active-set steps, then k_gadmm_ipm's solve)
    int st = g_admm_leaf_ipm == 1 ? hvp::GI_FAIL_ITER
                                  : hvp::solve_admm_lane<N>(q, S, C, role, prm, code, N,
                                                            g_admm_leaf_ipm == 2 ? 2 : 8 * hvp::GiConstraintSet<N>::NC,
                                                            it, &raw);
    if (st != hvp::GI_OK && g_admm_leaf_ipm) {
        int it2 = 0;
        st = hvp::solve_admm_ipm<N>(q, S, C, role, prm, code, N, it2, &raw);
    }
    if (st != hvp::GI_OK) {
        *status = st == hvp::GI_FAIL_DUAL ? HVP_INFEASIBLE : HVP_MAXITER;
        *cost = 1e300;
        *edge = 0;
        return;
    }
    *status = HVP_OPTIMAL;
    *cost = hvp::admm_direct_cost<N>(q, S, C, role, prm, code, N);
    uint32_t e = 0;  // region edges strictly inside the state box (k_gadmm_qp's gadmm_edges)
    for (int j = 0; j + 1 < N; ++j) {
        const int r = hvp::code_region(code, j + 1);
        if (((raw >> (2 * j)) & 1u) && S.vlo[r] > S.vmin + 1e-9 * (1.0 + fabs(S.vlo[r]))) e |= 1u << (2 * j);
        if (((raw >> (2 * j + 1)) & 1u) && S.vhi[r] < S.vmax - 1e-9 * (1.0 + fabs(S.vhi[r]))) e |= 1u << (2 * j + 1);
    }
    *edge = e;
    const int K1 = N + 1;
    double p = prm[0], v = prm[1];
    for (int k = 0; k <= N; ++k) {
        x[k] = p;
        x[K1 + k] = v;
        double fe = 0.0, fg = 0.0;
        if (role & HVP_ROLE_SAFE_FRONT)
            hvp::admm_copy_value(C, (role & HVP_ROLE_TRACK_FRONT) != 0, 0, hvp::admm_y(prm, 0, N)[k],
                                 hvp::admm_y(prm, 0, N)[K1 + k], hvp::admm_z(prm, 0, N)[k],
                                 hvp::admm_z(prm, 0, N)[K1 + k], p, v, &fe, &fg);
        xf[k] = fe;
        xf[K1 + k] = fg;
        const bool back = (role & HVP_ROLE_BACK_COPY) != 0;
        xb[k] = back ? hvp::admm_z(prm, 1, N)[k] - hvp::admm_y(prm, 1, N)[k] / C.rho : 0.0;
        xb[K1 + k] = back ? hvp::admm_z(prm, 1, N)[K1 + k] - hvp::admm_y(prm, 1, N)[K1 + k] / C.rho : 0.0;
        if (k < N) {
            const int r = hvp::code_region(code, k);
            u[k] = (q.y[k] - S.a[r] * v - S.c[r]) / S.b[r];
            p = p + S.ts * v;
            v = q.y[k];
        }
    }
}

}  // namespace

extern "C" {

// HVP_FORM_GADMM local QPs for given sequences (test use only): the lane algorithm on the host.
int hvp_hostref_gadmm_solve(const hvp_problem* P, const hvp_system* systems, int B, const int32_t* sys,
                            const int32_t* role, const double* params, const int8_t* seq, double* u, double* x,
                            double* xf, double* xb, double* cost, int32_t* status, uint32_t* edge) {
    if (P->formulation != HVP_FORM_GADMM) return HVP_E_ARG;
    const hvp::Consts C = make_consts(*P);
    const int N = P->N, E = 2 * (N + 1);
    for (int i = 0; i < B; ++i) {
        const double* prm = params + (size_t)i * C.stride;
        switch (N) {
#define HVP_CASE(n) \
    case n: gadmm_one<n>(systems[sys[i]], C, role[i], prm, seq + (size_t)i * N, u + (size_t)i * N, x + (size_t)i * E, xf + (size_t)i * E, xb + (size_t)i * E, cost + i, status + i, edge + i); break;
            HVP_CASE(2) HVP_CASE(3) HVP_CASE(4) HVP_CASE(5) HVP_CASE(6) HVP_CASE(7) HVP_CASE(8)
            HVP_CASE(9) HVP_CASE(10) HVP_CASE(11) HVP_CASE(12) HVP_CASE(13) HVP_CASE(14) HVP_CASE(15) HVP_CASE(16)
#undef HVP_CASE
            default: return HVP_E_UNSUPPORTED;
        }
    }
    return 0;
}

void hvp_hostref_set_solver(int s) { g_solver = s; }
void hvp_hostref_set_l1_solver(int s) { g_l1_solver = s; }
void hvp_hostref_set_lp_trace(int s) { g_lp_trace = s; }
void hvp_hostref_set_admm_leaf_ipm(int s) { g_admm_leaf_ipm = s; }
void hvp_hostref_set_admm_warm(int s) { g_admm_warm = s; }
void hvp_hostref_set_admm_slots(int s) { g_admm_slots = s; }
void hvp_hostref_reset_admm_warm() {
    for (uint64_t& h : g_admm_root_hs) h = hvp::kHubNone;
    for (auto& m : g_admm_recs) m.clear();
    for (auto& m : g_admm_tab) m.clear();
    for (long long& v : g_admm_rec_stats) v = 0;
    for (long long& v : g_admm_warm_stats) v = 0;
}
void hvp_hostref_admm_warm_stats(long long* out) {
    for (int i = 0; i < 4; ++i) out[i] = g_admm_warm_stats[i];
    for (int i = 0; i < 4; ++i) out[4 + i] = g_admm_rec_stats[i];
}
// unpruned branch-and-bound nodes by depth (0..16) and children (0..7+) since the last call (17 x 8)
void hvp_hostref_bnb_children(long long* out) {
    for (int i = 0; i < 17; ++i)
        for (int j = 0; j < 8; ++j) out[i * 8 + j] = g_bnb_nch[i][j], g_bnb_nch[i][j] = 0;
}
// the (parent pivots, child pivots) histogram of the min_1_norm node LPs since the last call (32 x 32)
void hvp_hostref_lp_parent_child(long long* out) {
    for (int i = 0; i < 32; ++i)
        for (int j = 0; j < 32; ++j) out[i * 32 + j] = g_lp_pc[i][j], g_lp_pc[i][j] = 0;
}
void hvp_hostref_lp_hist(long long* out) {
    for (int i = 0; i < 64; ++i) out[i] = g_lp_hist[i], g_lp_hist[i] = 0;
}
void hvp_hostref_lp_stats(long long* out) {
    out[0] = g_lp_runs;
    out[1] = g_lp_iters;
    out[2] = g_lp_fail;
    for (int i = 1; i < 5; ++i) out[2 + i] = g_lp_why[i], g_lp_why[i] = 0;
    out[7] = g_lp_pass;
    g_lp_pass = 0;
    g_lp_runs = g_lp_iters = g_lp_fail = 0;
}
void hvp_hostref_gi_stats(long long* out) {
    out[0] = g_gi_runs;
    out[1] = g_gi_fail;
    out[2] = g_gi_iters;
    for (int i = 0; i < 4; ++i) out[3 + i] = g_gi_code[i], g_gi_code[i] = 0;
    g_gi_runs = g_gi_fail = g_gi_iters = 0;
}

// Same outputs as hvp_solve_batch (host pointers); test / baseline use only.
int hvp_hostref_solve_batch(const hvp_problem* P, const hvp_system* systems, int B, const int32_t* sys,
                            const int32_t* role, const double* params, double* u, double* x, int8_t* region,
                            double* cost, int32_t* status, int32_t* nodes, int32_t* iters, int nthreads) {
    switch (P->N) {
#define HVP_CASE(n) \
    case n: solve_range<n>(*P, systems, B, sys, role, params, u, x, region, cost, status, nodes, iters, nthreads); return 0;
        HVP_CASE(2) HVP_CASE(3) HVP_CASE(4) HVP_CASE(5) HVP_CASE(6) HVP_CASE(7) HVP_CASE(8)
        HVP_CASE(9) HVP_CASE(10) HVP_CASE(11) HVP_CASE(12) HVP_CASE(13) HVP_CASE(14) HVP_CASE(15) HVP_CASE(16)
#undef HVP_CASE
        default: return HVP_E_UNSUPPORTED;
    }
}

// HVP_FORM_ADMM problems with the optimal neighbour copies (test / baseline use only).
int hvp_hostref_solve_admm_batch(const hvp_problem* P, const hvp_system* systems, int B, const int32_t* sys,
                                 const int32_t* role, const double* params, double* u, double* x, int8_t* region,
                                 double* cost, int32_t* status, int32_t* nodes, int32_t* iters, double* xf,
                                 double* xb, int nthreads) {
    if (P->formulation != HVP_FORM_ADMM) return HVP_E_ARG;
    switch (P->N) {
#define HVP_CASE(n) \
    case n: solve_range<n>(*P, systems, B, sys, role, params, u, x, region, cost, status, nodes, iters, nthreads, xf, xb); return 0;
        HVP_CASE(2) HVP_CASE(3) HVP_CASE(4) HVP_CASE(5) HVP_CASE(6) HVP_CASE(7) HVP_CASE(8)
        HVP_CASE(9) HVP_CASE(10) HVP_CASE(11) HVP_CASE(12) HVP_CASE(13) HVP_CASE(14) HVP_CASE(15) HVP_CASE(16)
#undef HVP_CASE
        default: return HVP_E_UNSUPPORTED;
    }
}

// Per-candidate costs of one instance in enumeration order (debugging / parity of every QP).
int hvp_hostref_candidates(const hvp_problem* P, const hvp_system* S, int role, const double* prm,
                           double* cand_cost, uint32_t* cand_code, int cap) {
    const hvp::Consts C = make_consts(*P);
    int n = 0;
    double u[HVP_MAX_N], x[2 * (HVP_MAX_N + 1)], cost;
    int8_t reg[HVP_MAX_N];
    int32_t st, nodes, it;
    switch (P->N) {
#define HVP_CASE(k) \
    case k: solve_one<k>(*S, C, role, prm, u, x, reg, &cost, &st, &nodes, &it, cand_cost, cand_code, cap); n = nodes; break;
        HVP_CASE(2) HVP_CASE(3) HVP_CASE(4) HVP_CASE(5) HVP_CASE(6) HVP_CASE(7) HVP_CASE(8)
#undef HVP_CASE
        default: return HVP_E_UNSUPPORTED;
    }
    return n;
}
}
