// hvp_cent_bnb.h -- depth-first branch and bound of the centralised platoon MIQP (MpcMldCent,
// mpcs/cent_mld.py:21-182), one 64-lane wavefront per platoon, on top of the wave QP of
// hvp_cent.h.
//
// Decision d = k n + i fixes sigma_{i,k} (time-major, the order of oracle/hvp_oracle.c
// cent_dfs).  A node's children are the regions reachable from the exact velocity interval of
// v_{i,k} (bnb_child); each child's bound is the platoon QP with the assigned prefix fixed and
// every later step relaxed (hvp_ipm.h relax_step): an undecided step keeps the
// interval of its next velocity reachable over every region it may still take and, where those
// regions share the velocity dynamics (a, c), a virtual region (a, b_max, c) whose input rows
// and input cost are kept on s = u b_r / b_max.  A valid lower bound of every completion: b_r <=
// b_max and umin <= 0 <= umax make s feasible with Q_u s^2 <= Q_u u^2, the reachable intervals
// contain every completion's velocities, and Q_du terms of undecided steps (>= 0) are dropped.
// Children are visited in increasing (bound, region) order and pruned when
// bound > incumbent + kPruneRel (1 + |incumbent|); leaves (all n N steps fixed) are exact QPs.
// The answer is the lexicographically first (time-major) joint sequence within 1e-9 relative of
// the minimum -- the oracle's rule -- and the exploration order, hence the QP count, is the
// oracle's too.
//
// Storage: the DFS frame headers live in lane d's registers (depth d < 64), the children of each
// frame in the platoon's global slice `frames` [D][nreg_max], the near-optimal leaves of the tie
// rule in `tie_codes` [kTie][n] (codes) and lane j's register (cost).
#pragma once

#include "hvp_bnb.h"
#include "hvp_cent.h"
#include "hvp_cent_l1.h"

namespace hvp {
namespace cent {

constexpr int kTie = 64;  // near-optimal leaves kept for the tie rule (per search / task; <= W: lane j holds cost j)
constexpr int kTieG = 64; // near-optimal leaves kept per platoon across the tasks of a split search

// ---- split searches (heavy platoons): a search that exceeds its QP budget exports the
// unexplored children of its open DFS frames as subtree TASKS; rounds of k_cent_tasks run the
// tasks of all split platoons on every wave of the chip (sharing each platoon's incumbent for
// pruning), and k_cent_final picks the winner from the platoon's merged near-optimal leaves.
constexpr int kSplit = 100;     // Result.status: exported as tasks (k_cent_final finishes it)
constexpr int kTaskDone = 101;  // Result.status of a finished subtree task

struct Task {
    int32_t p, d0;  // platoon; decisions fixed at the subtree root
    double lb;      // the root's bound
    uint64_t code[kMaxVeh];
    double lo[kMaxVeh], hi[kMaxVeh];  // exact interval of each vehicle's first undecided velocity
};

// per-platoon record of a split search (global memory, initialised per call)
struct PlatoonRec {
    unsigned long long inc_key;   // incumbent (order-preserving key of the cost; ~0: none)
    unsigned long long fail_key;  // smallest bound of a leaf whose QP failed (~0: none)
    unsigned long long nodes, iters;
    int tie_count;                // entries of the merged tie list
    int flags;                    // 1 split, 2 node limit, 4 tie list overflow, 8 task list overflow
};
// (bit 8, once REC_TASK_OVER, is free: a full task queue declines the split, export_tasks)
enum { REC_SPLIT = 1, REC_NODE_LIMIT = 2, REC_TIE_OVER = 4 };

__device__ inline unsigned long long ckey(double c) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(c);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ inline double kcost(unsigned long long k) {
    if (k == ~0ull) return __builtin_inf();
    return __longlong_as_double((long long)((k >> 63) ? (k & 0x7fffffffffffffffull) : ~k));
}

// device pointers of a call's split-search workspace (hvp_cent.hip)
struct SplitWs {
    PlatoonRec* rec;          // [P]
    uint64_t* tie_g;          // [P][kTieG][n]
    double* tie_gc;           // [P][kTieG]
    Task* out;                // next round's tasks
    unsigned long long* out_count;
    long long out_cap;
    const Task* in;           // this round's tasks (k_cent_tasks)
    unsigned long long* in_claim;
    unsigned long long in_count;
    int budget;               // QPs per search / task before it splits (0: no splitting)
};

struct SplitArgs {
    int mode;                  // 1 whole search that may split, 2 subtree task
    int budget;                // QPs of this search before it splits
    int p;                     // platoon
    const Task* task;          // mode 2: the subtree root
    PlatoonRec* rec;           // this platoon's record
    uint64_t* tie_g;           // [kTieG][n] merged near-optimal codes of this platoon
    double* tie_gc;            // [kTieG] their costs
    Task* out;                 // tasks for the next round
    unsigned long long* out_count;
    long long out_cap;
};

enum { QP_OK = 0, QP_INFEASIBLE = 1, QP_FAILED = 2, QP_CUT = 3 };  // QP_CUT: bound above the cut (solve's early stop)

// HVP_CENT_DEBUG=6 diagnostics: QPs per number of fixed decisions, [0] bound QPs of expansions,
// [1] visits (leaves / final), [2] bound QPs whose bound ended above the incumbent
__device__ unsigned long long g_cent_depth[3][64];

struct Child {
    double lb, lo, hi;
    int32_t r, pad;
};

struct Result {
    double cost;
    int status;  // HVP_*
    int nodes;   // QPs of the search: bounds and leaves (the oracle's count; the final re-solve of
                 // the winner is not counted)
    int iters;   // active-set iterations
};

// Register state of the search.  Lane i < n: vehicle i's region code and the reachable interval
// of its next undecided velocity.  Lane d < D: DFS frame d (children, cursor, the interval of
// vehicle d % n before the frame's decision, the bound of the child taken).  Lane j < ntie: cost
// of near-optimal leaf j.
struct Search {
    uint64_t vcode;
    double vlo, vhi;
    int f_n, f_cur;
    double f_slo, f_shi, f_lb;
    double tie_c;
};

// fixed steps of vehicle i once the first d decisions (time-major) are taken
__device__ inline int fixed_steps(int d, int n, int i) { return d / n + (i < d % n ? 1 : 0); }

// Platoon QP with the first `d` decisions fixed; lane j < n holds vehicle j's code and the exact
// interval [vlo, vhi] of its first undecided velocity.  QP_OK with the cost and the lanes' y.
// L1: the min_1_norm LP of the same rows (hvp_cent_l1.h): QP_INFEASIBLE when a vehicle's hard rows
// are proven infeasible (hvp_l1.h l1_infeasible, per vehicle: the hard rows do not couple
// vehicles), QP_FAILED when the interior point leaves it unresolved.
//
// cut < inf (quadratic cost): the QP may stop as soon as its dual bound exceeds cut (QP_CUT, cost =
// that bound): the caller passes a value above which the QP is pruned whatever its optimum.
template <bool L1>
__device__ inline int platoon_qp(Lane& L, const Lds& S, const Consts& C, const Inst& I, uint64_t vcode, double vlo,
                                 double vhi, int d, int max_iter, double& cost, int& iters, Prof& pf,
                                 double cut = __builtin_inf()) {
    const int t = lane();
    const int i = t < I.V ? t / I.N : 0;
    const uint64_t ci = bc(vcode, i);
    const double lo = bc(vlo, i), hi = bc(vhi, i);
    const int Ki = fixed_steps(d, I.n, i);
    int it = 0;
    iters = 0;
    wsync();
    pf.mark(10);
    pf.count(10);
    if (!setup(L, S, C, I, ci, Ki, lo, hi)) return QP_INFEASIBLE;
    if constexpr (L1) {
        const int N = I.N;
        int bad = 0;
        if (t < I.V && t % N == 0)
            bad = l1_infeasible_rt(I.systems[I.vsys[i]], C, I.x0[2 * i], I.x0[2 * i + 1], ci, Ki,
                                   Ki < N ? lo : 0.0, Ki < N ? hi : -1.0, N)
                      ? 1
                      : 0;
        if (wor(bad)) return QP_INFEASIBLE;
        LpCtx X;
        X.P1m = __shfl(L.P1, t >= N ? t - N : t, W);
        X.amm = shift_up1(L.am);
        X.ubm = shift_up1(L.ub);
        X.ucm = shift_up1(L.uc);
        X.Ki = Ki;
        const int r = lp_solve(L, S, C, I, X, C.max_iter, it);
        iters = it;
        if (r != L1_OK) return QP_FAILED;
        cost = lp_direct_cost(L, C, I, Ki);
        return QP_OK;
    }
    pf.mark(0);
    const int r = solve(L, S, C, I, max_iter, it, pf, Ki, cut, &cost);
    iters = it;
    if (r == GI_CUT) return QP_CUT;
    if (r == GI_FAIL_DUAL) return QP_INFEASIBLE;
    if (r != GI_OK) return QP_FAILED;
    cost = direct_cost(L, C, I, ci, Ki);
    pf.mark(9);
    return QP_OK;
}

// time-major lexicographic "a < b" of two joint sequences (lane i < n holds vehicle i's code)
__device__ inline bool joint_less(uint64_t a_code, uint64_t b_code, int n, int N) {
    const int t = lane();
    const int D = n * N;
    const int vi = t < D ? t % n : 0, vk = t < D ? t / n : 0;
    const uint64_t ca = bc(a_code, vi), cb = bc(b_code, vi);
    const int ra = t < D ? code_region(ca, vk) : 0, rb = t < D ? code_region(cb, vk) : 0;
    const unsigned long long diff = __ballot(t < D && ra != rb);
    if (!diff) return false;
    const int first = __ffsll((long long)diff) - 1;
    return bcu(ra, first) < bcu(rb, first);
}

// One child record, read with lane-dependent addresses (vector loads: the slice is rewritten
// during the search, so it must not go through the scalar cache) and broadcast.
__device__ inline Child load_child(const Child* c) {
    const int t = lane();
    const double* w = reinterpret_cast<const double*>(c);
    const double v = t < 4 ? w[t] : 0.0;
    Child ch;
    ch.lb = bcu(v, 0);
    ch.lo = bcu(v, 1);
    ch.hi = bcu(v, 2);
    ch.r = (int32_t)(__double_as_longlong(bcu(v, 3)) & 0xffffffffll);
    ch.pad = 0;
    return ch;
}

// Branch and bound of one platoon.  On return with status HVP_OPTIMAL the lanes' L.y and
// st.vcode hold the winner.  Written as a loop with ONE platoon-QP call site (bound QPs of a
// node's children, leaf QPs and the final re-solve all go through it), so the large QP body is
// inlined once and its state stays in registers.
//
// sp (split searches, see Task): mode 1 = the whole search of a platoon that exports its open
// frames as tasks once it has solved sp->budget QPs (then Result.status = kSplit); mode 2 = the
// subtree of sp->task, merged into the platoon's record when done (kTaskDone; it splits again
// past its budget).  Both prune against the platoon's shared incumbent.  Without sp the search
// runs to the end (the exhaustive mode and the searches that fit their budget behave alike:
// a platoon alone on its record sees only its own incumbent, so its QP count is the oracle's).
template <bool L1>
__device__ inline void bnb_platoon(Lane& L, const Lds& S, const Consts& C, const Inst& I, Search& st, Child* frames,
                                   int nreg_max, uint64_t* tie_codes, int max_nodes, bool exhaustive, int max_iter,
                                   Result& res, const SplitArgs* sp = nullptr) {
    const int t = lane();
    const int n = I.n, N = I.N, D = n * N;
    const double INF = __builtin_inf();
    const bool task = sp && sp->mode == 2;
    const int d0 = task ? sp->task->d0 : 0;  // the search ends when it backtracks above d0
    st.vcode = task && t < n ? sp->task->code[t] : 0;
    st.vlo = t < n ? (task ? sp->task->lo[t] : I.x0[2 * t + 1]) : 0.0;
    st.vhi = t < n ? (task ? sp->task->hi[t] : I.x0[2 * t + 1]) : 0.0;
    st.f_n = st.f_cur = 0;
    st.f_slo = st.f_shi = st.f_lb = 0.0;
    st.tie_c = INF;
    int ntie = 0;
    double inc = INF;
    bool have_best = false, node_limit = false, tie_over = false;
    double fail_lb = INF;  // smallest bound of a leaf whose QP failed (not infeasible)
    int nodes = 0, iters = 0, searched = 0;
    Prof pf;
    pf.start(I.debug >= 3);
    // the platoon's shared incumbent (split searches)
    auto shared_inc = [&]() -> double {
        if (!sp) return inc;
        unsigned long long k = 0;
        if (t == 0) k = __atomic_load_n(&sp->rec->inc_key, __ATOMIC_RELAXED);
        return fmin(inc, kcost(bcu((uint64_t)k, 0)));
    };

    // expansion of the node with d decisions taken: lane r holds child r's interval and bound
    enum { EXPAND = 0, VISIT = 1, FINAL = 2, LEAF = 3 };
    int phase = EXPAND, d = d0;
    unsigned long long ex_mask = 0, ex_todo = 0;
    uint64_t ex_save = 0;
    bool ex_ok = false;
    double ex_nlo = 0.0, ex_nhi = 0.0, ex_lb = 0.0;
    int ex_r = 0;

    auto begin_expand = [&](int dd) {
        const int k = dd / n, i = dd % n;
        const hvp_system& Si = I.systems[I.vsys[i]];
        const double lo = bcu(st.vlo, i), hi = bcu(st.vhi, i);
        ex_ok = false;
        ex_nlo = ex_nhi = 0.0;
        if (t < Si.n_regions) ex_ok = bnb_child(Si, C, k, lo, hi, t, &ex_nlo, &ex_nhi);
        ex_mask = __ballot(ex_ok);
        ex_todo = (dd + 1 < D && !exhaustive) ? ex_mask : 0ull;
        ex_lb = 0.0;
        ex_save = st.vcode;
        if (t == dd) {
            st.f_n = __popcll(ex_mask);
            st.f_cur = 0;
            st.f_slo = lo;
            st.f_shi = hi;
        }
    };
    // children sorted by (bound, region) into frame dd
    auto finish_expand = [&](int dd) {
        const hvp_system& Si = I.systems[I.vsys[dd % n]];
        int rank = 0;
        for (int c = 0; c < Si.n_regions; ++c) {
            const double lc = bcu(ex_lb, c);
            if (((ex_mask >> c) & 1ull) && (lc < ex_lb || (lc == ex_lb && c < t))) ++rank;
        }
        if (ex_ok) {
            Child ch;
            ch.lb = ex_lb;
            ch.lo = ex_nlo;
            ch.hi = ex_nhi;
            ch.r = t;
            ch.pad = 0;
            frames[(size_t)dd * nreg_max + rank] = ch;
        }
        __threadfence_block();
        wsync();
    };
    // a feasible leaf with the current codes: incumbent and tie set
    auto record = [&](double cost) {
        if (cost < inc) {
            inc = cost;
            const double tol = 1e-9 * fmax(1.0, fabs(inc));
            int w = 0;  // drop entries beyond the new window (rows only move down: serial copy)
            for (int j = 0; j < ntie; ++j) {
                const double cj = bcu(st.tie_c, j);
                if (!(cj <= inc + tol)) continue;
                if (w != j) {
                    if (t < n) tie_codes[(size_t)w * n + t] = tie_codes[(size_t)j * n + t];
                    if (t == w) st.tie_c = cj;
                }
                ++w;
            }
            ntie = w;
            if (t >= ntie) st.tie_c = INF;
        }
        if (cost <= inc + 1e-9 * fmax(1.0, fabs(inc))) {
            if (ntie < kTie) {
                if (t < n) tie_codes[(size_t)ntie * n + t] = st.vcode;
                if (t == ntie) st.tie_c = cost;
                ++ntie;
            } else {
                tie_over = true;
            }
        }
        have_best = true;
        if (I.debug == 6 && t == 0 && cost < inc + 1e-9 * fmax(1.0, fabs(inc)))
            printf("[cent-inc] platoon %d task %d QPs %d (platoon: %llu in finished tasks) leaf cost %.9e\n",
                   sp ? sp->p : (int)blockIdx.x, sp && sp->mode == 2 ? 1 : 0, nodes,
                   sp ? __atomic_load_n(&sp->rec->nodes, __ATOMIC_RELAXED) : 0ull, cost);
        if (sp && t == 0) atomicMin(&sp->rec->inc_key, ckey(cost));
    };
    // split searches: this search's leaves, counters and flags into the platoon's record
    auto merge = [&]() {
        // leaves outside the tie window of the platoon's incumbent (this task's local window
        // opened at +inf, and later improvements leave stale entries) take no slot
        const double incs = shared_inc();
        const double win = incs + 1e-9 * fmax(1.0, fabs(incs));
        for (int j = 0; j < ntie; ++j) {
            const double cj = bcu(st.tie_c, j);
            if (incs < INF && cj > win) continue;
            int slot = 0;
            if (t == 0) slot = atomicAdd(&sp->rec->tie_count, 1);
            slot = bcu(slot, 0);
            if (slot >= kTieG) {
                tie_over = true;
                continue;
            }
            if (t < n) sp->tie_g[(size_t)slot * n + t] = tie_codes[(size_t)j * n + t];
            if (t == 0) sp->tie_gc[slot] = cj;
        }
        if (t == 0) {
            atomicAdd(&sp->rec->nodes, (unsigned long long)nodes);
            atomicAdd(&sp->rec->iters, (unsigned long long)iters);
            if (fail_lb < INF) atomicMin(&sp->rec->fail_key, ckey(fail_lb));
            const int fl = (tie_over ? REC_TIE_OVER : 0) | (node_limit ? REC_NODE_LIMIT : 0);
            if (fl) atomicOr(&sp->rec->flags, fl);
        }
    };
    // split: the unexplored children of the open frames d .. d0 become tasks (deepest first;
    // each vehicle's interval goes back to its parent's as the DFS backtrack does).  The tasks'
    // slots are reserved at once (compare-and-swap on the list size, never past its capacity):
    // when the list cannot take them all, nothing is exported and the search goes on in this wave
    // (returns false) -- a full task list costs parallelism, never a platoon (no HVP_OVERFLOW).
    auto export_tasks = [&]() -> bool {
        const double incp = shared_inc();
        int want = 0;  // the tasks below, counted with the same incumbent
        for (int j = d; j >= d0; --j) {
            const int nch = bcu(st.f_n, j), cur = bcu(st.f_cur, j);
            for (int c = cur; c < nch; ++c) {
                const Child ch = load_child(frames + (size_t)j * nreg_max + c);
                if (!(ch.lb < INF)) continue;
                if (incp < INF && bnb_pruned(ch.lb, incp)) continue;
                ++want;
            }
        }
        unsigned long long base = 0;
        int ok = 1;
        if (t == 0) {
            unsigned long long cur = __atomic_load_n(sp->out_count, __ATOMIC_RELAXED);
            for (;;) {
                if ((long long)(cur + (unsigned long long)want) > sp->out_cap) {
                    ok = 0;
                    break;
                }
                const unsigned long long prev = atomicCAS(sp->out_count, cur, cur + (unsigned long long)want);
                if (prev == cur) break;
                cur = prev;
            }
            base = cur;
        }
        if (!bcu(ok, 0)) return false;
        base = bcu((uint64_t)base, 0);
        uint64_t vcode_w = st.vcode;
        double vlo_w = st.vlo, vhi_w = st.vhi;
        for (int j = d; j >= d0; --j) {
            const int nch = bcu(st.f_n, j), cur = bcu(st.f_cur, j);
            const int i = j % n, k = j / n;
            for (int c = cur; c < nch; ++c) {
                const Child ch = load_child(frames + (size_t)j * nreg_max + c);
                if (!(ch.lb < INF)) continue;
                if (incp < INF && bnb_pruned(ch.lb, incp)) continue;
                const uint64_t slot = base++;
                Task* tk = sp->out + slot;
                if (t < n) {
                    tk->code[t] = t == i ? code_with(vcode_w, k, ch.r) : vcode_w;
                    tk->lo[t] = t == i ? ch.lo : vlo_w;
                    tk->hi[t] = t == i ? ch.hi : vhi_w;
                }
                if (t == 0) {
                    tk->p = sp->p;
                    tk->d0 = j + 1;
                    tk->lb = ch.lb;
                }
            }
            const double slo = bcu(st.f_slo, j), shi = bcu(st.f_shi, j);
            if (t == i) {
                vlo_w = slo;
                vhi_w = shi;
            }
        }
        if (t == 0) atomicOr(&sp->rec->flags, REC_SPLIT);
        return true;
    };
    int split_at = sp ? sp->budget : 0;  // QPs after which the search tries to split

    if (task && d0 >= D) {
        phase = LEAF;  // the task is one leaf
    } else {
        begin_expand(d0);
    }
    for (;;) {
        // ---- decide the next QP (dfix decisions fixed), or move the search without one
        int dfix = -1;
        if (phase == EXPAND) {
            if (!ex_todo) {
                if (t == d % n) st.vcode = ex_save;
                finish_expand(d);
                phase = VISIT;
                continue;
            }
            ex_r = __ffsll((long long)ex_todo) - 1;
            if (t == d % n) st.vcode = code_with(ex_save, d / n, ex_r);
            dfix = d + 1;
        } else if (phase == LEAF) {
            dfix = D;
        } else if (phase == VISIT) {
            if (nodes >= max_nodes) {
                node_limit = true;
                break;
            }
            if (task && d < d0) {  // subtree done
                merge();
                res.status = kTaskDone;
                res.nodes = nodes;
                res.iters = iters;
                pf.flush();
                return;
            }
            if (sp && d >= d0 && nodes >= split_at) {  // past the budget: split
                if (export_tasks()) {
                    merge();
                    res.status = task ? kTaskDone : kSplit;
                    res.nodes = nodes;
                    res.iters = iters;
                    pf.flush();
                    return;
                }
                split_at = nodes + sp->budget;  // the task list is full: search on, try again later
            }
            if (d < 0) {  // search done
                searched = nodes;
                if (!have_best || tie_over) break;
                // the lexicographically first (time-major) leaf within the tie window
                const double tol = 1e-9 * fmax(1.0, fabs(inc));
                int win = -1;
                uint64_t wcode = 0;
                for (int j = 0; j < ntie; ++j) {
                    const double cj = bcu(st.tie_c, j);
                    if (!(cj <= inc + tol)) continue;
                    const uint64_t cj_code = t < n ? tie_codes[(size_t)j * n + t] : 0;
                    if (win < 0 || joint_less(cj_code, wcode, n, N)) {
                        win = j;
                        wcode = cj_code;
                    }
                }
                st.vcode = wcode;
                phase = FINAL;
                dfix = D;  // re-solve the winner for its trajectory (not counted)
            } else {
                const int nch = bcu(st.f_n, d), cur = bcu(st.f_cur, d);
                const int i = d % n, k = d / n;
                if (cur >= nch) {  // frame done: vehicle i's interval back to the parent's
                    const double slo = bcu(st.f_slo, d), shi = bcu(st.f_shi, d);
                    if (t == i) {
                        st.vlo = slo;
                        st.vhi = shi;
                    }
                    --d;
                    continue;
                }
                if (t == d) st.f_cur = cur + 1;
                const Child ch = load_child(frames + (size_t)d * nreg_max + cur);
                const double incp = shared_inc();
                if ((have_best || incp < INF) && bnb_pruned(ch.lb, incp)) continue;
                if (!(ch.lb < INF)) continue;
                if (t == i) {
                    st.vcode = code_with(st.vcode, k, ch.r);
                    st.vlo = ch.lo;
                    st.vhi = ch.hi;
                }
                if (t == d) st.f_lb = ch.lb;
                if (d + 1 < D) {
                    ++d;
                    begin_expand(d);
                    phase = EXPAND;
                    continue;
                }
                dfix = D;  // leaf: every step of every vehicle fixed
            }
        }
        // ---- the one QP call site
        double c = 0.0;
        int it = 0;
        ++nodes;
        // vehicle intervals of the QP: in EXPAND vehicle d % n takes the child's
        double qlo = st.vlo, qhi = st.vhi;
        if (phase == EXPAND) {
            const double clo = bcu(ex_nlo, ex_r), chi = bcu(ex_nhi, ex_r);
            if (t == d % n) {
                qlo = clo;
                qhi = chi;
            }
        }
        // early stop of QPs that end pruned: 10x the prune margin above the incumbent (the dual
        // bound's rounding is ~1e-9 relative); not for the final re-solve
        double cut = INF;
        if (phase != FINAL && C.cent_cut && !L1) {
            const double incc = shared_inc();
            if (incc < INF) cut = incc + 10.0 * kPruneRel * (1.0 + fabs(incc));
        }
        const int q = platoon_qp<L1>(L, S, C, I, st.vcode, qlo, qhi, dfix, max_iter, c, it, pf, cut);
        iters += it;
        if (I.debug == 6) {
            const double incd = shared_inc();
            const int dd = dfix < 63 ? dfix : 63;
            if (t == 0) {
                atomicAdd(&g_cent_depth[phase == EXPAND ? 0 : 1][dd], 1ull);
                if (phase == EXPAND && q == QP_OK && bnb_pruned(c, incd)) atomicAdd(&g_cent_depth[2][dd], 1ull);
            }
        }
        if (I.debug && I.debug < 3 && q != QP_OK) {
            const uint64_t c0 = bc(st.vcode, 0), c1 = bc(st.vcode, 1 < n ? 1 : 0), c2 = bc(st.vcode, 2 < n ? 2 : 0);
            if (t == 0)
                printf("[cent] platoon %d QP %d dfix %d phase %d -> %d (codes v0 %llx v1 %llx v2 %llx)\n",
                       (int)blockIdx.x, nodes, dfix, phase, q, (unsigned long long)c0, (unsigned long long)c1,
                       (unsigned long long)c2);
        }
        // ---- use its result
        if (phase == EXPAND) {
            const double lb = (q == QP_OK || q == QP_CUT) ? c : (q == QP_INFEASIBLE ? INF : -INF);
            if (t == ex_r) ex_lb = lb;
            ex_todo &= ex_todo - 1;
        } else if (phase == VISIT) {
            if (q == QP_OK) {
                record(c);
            } else if (q == QP_FAILED) {
                const double plb = D >= 2 ? bcu(st.f_lb, D - 2) : -INF;
                fail_lb = fmin(fail_lb, plb);
            }
        } else if (phase == LEAF) {  // a one-leaf task: its bound is the exported child's
            if (q == QP_OK) record(c);
            else if (q == QP_FAILED) fail_lb = fmin(fail_lb, sp->task->lb);
            phase = VISIT;
            d = d0 - 1;  // done
        } else {  // FINAL
            // a failed leaf whose bound is not above the incumbent could hide the optimum
            res.status = (fail_lb < INF && !bnb_pruned(fail_lb, inc)) ? HVP_MAXITER : HVP_OPTIMAL;
            if (q != QP_OK) res.status = HVP_MAXITER;
            res.cost = c;
            res.nodes = searched;
            res.iters = iters;
            pf.flush();
            return;
        }
    }
    if (task) {  // a subtree stopped by the QP cap
        merge();
        res.status = kTaskDone;
        res.nodes = nodes;
        res.iters = iters;
        pf.flush();
        return;
    }
    res.cost = INF;
    if (node_limit) res.status = HVP_MAXITER;
    else if (tie_over) res.status = HVP_OVERFLOW;
    else res.status = fail_lb < INF ? HVP_MAXITER : HVP_INFEASIBLE;
    res.nodes = node_limit ? nodes : searched;
    res.iters = iters;
    pf.flush();
}

}  // namespace cent
}  // namespace hvp
