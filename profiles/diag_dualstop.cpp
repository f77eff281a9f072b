// diag_dualstop.cpp -- host diagnostic (not product code): how many Goldfarb-Idnani trips of the
// decentralised branch-and-bound QPs could be skipped by stopping a QP as soon as its dual
// objective (every GI iterate is the optimum of a relaxation, so its objective is a lower bound of
// the QP's optimum) passes the incumbent.  Replays solve_one_bnb (hvp_hostref.cpp) on the host.
//
// build: g++ -O2 -fopenmp -shared -fPIC -I../hybrid-vehicle-platoon_amd/csrc -I../include
//        diag_dualstop.cpp -o /tmp/libdualstop.so
#include <math.h>
#include <string.h>

#include <vector>

#include "hvp_bnb.h"
#include "hvp_gi.h"
#include "hvp_ipm.h"

namespace {

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
    C.max_iter = p.max_iter > 0 ? p.max_iter : 60;
    C.N = p.N;
    C.form = p.formulation;
    C.stride = hvp_params_stride(p.N);
    return C;
}

// objective of the GI iterate: 1/2 y'Hy + f'y + C0 + w sum_sat (c.y - d)
template <int N>
double dual_obj(const hvp::LaneQp<N>& q, const hvp::GiLane<N>& g, const hvp::Consts& C) {
    double v = q.C0;
    for (int i = 0; i < N; ++i) {
        double hy = 0.0;
        for (int j = 0; j < N; ++j) hy += q.H[i >= j ? hvp::tri(i, j) : hvp::tri(j, i)] * q.y[j];
        v += q.y[i] * (0.5 * hy + q.f[i]);
    }
    for (int m = 0; m + 1 < N; ++m)
        for (int s = 0; s < 2; ++s)
            if ((g.sat >> (2 * m + s)) & 1u) {
                double c[N], d;
                hvp::gi_row<N>(q, C, 6 * N + 4 * m + 2 + s, c, d);
                double cy = 0.0;
                for (int i = 0; i < N; ++i) cy += c[i] * q.y[i];
                v += C.w * (cy - d);
            }
    return v;
}

struct Stat {
    long long qps = 0, steps = 0, steps_stop = 0, stopped = 0, bad = 0;
    double max_err = 0.0;  // |final dual obj - direct cost| / (1 + |cost|)
    std::vector<int> full, stop;  // per QP in order (for the wave model)
    std::vector<int> lvl_of, par_steps, par_nact, nact;
};

// GI with a dual-bound stop: returns the status; steps_all = steps to completion, steps_at = steps
// at which the iterate's objective first exceeded `cut` (-1: never)
template <int N>
int gi_trace(hvp::LaneQp<N>& q, const hvp::Consts& C, double cut, int& steps_all, int& steps_at, double& obj,
             int& nact) {
    hvp::GiLane<N> g;
    steps_at = -1;
    int st = g.init(q);
    if (st != hvp::GI_OK) return st;
    for (;;) {
        obj = dual_obj<N>(q, g, C);
        if (steps_at < 0 && obj > cut) steps_at = g.iter;
        if (!g.scan(q, C)) break;
        int r;
        do {
            r = g.step(q, C, 8 * hvp::GiConstraintSet<N>::NC);
        } while (r == hvp::GI_STEP_MORE);
        if (r != hvp::GI_STEP_NEXT) {
            steps_all = g.iter;
            return r;
        }
    }
    steps_all = g.iter;
    nact = g.nact;
    return g.verify(C, nullptr);
}

template <int N>
void one(const hvp_system& S, const hvp::Consts& C, int role, const double* prm, double marg, Stat& st) {
    struct Node {
        uint64_t code;
        double lo, hi, lb;
        int steps, nact;  // the node's own QP: GI steps, active rows at the optimum
        int psteps, pnact;
    };
    double inc = HUGE_VAL;
    int last_steps = 0, last_nact = 0;
    auto qp = [&](uint64_t code, int K, double lo, double hi, double& c, double* y, bool stat) {
        hvp::LaneQp<N> q;
        hvp::setup_lane<N>(q, S, C, role, prm, code, K, lo, hi);
        const double cut = inc < HUGE_VAL ? inc + marg * (1.0 + fabs(inc)) : HUGE_VAL;
        int sa = 0, sat = -1;
        double obj = 0.0;
        int na = 0;
        const int r = gi_trace<N>(q, C, cut, sa, sat, obj, na);
        last_steps = sa;
        last_nact = na;
        if (r != hvp::GI_OK) return false;
        c = hvp::direct_cost<N>(q, S, C, role, prm, code, K);
        if (y)
            for (int i = 0; i < N; ++i) y[i] = q.y[i];
        if (stat) {
            st.qps++;
            st.steps += sa;
            const int s2 = sat >= 0 ? sat : sa;
            st.steps_stop += s2;
            st.full.push_back(sa);
            st.stop.push_back(s2);
            if (sat >= 0) {
                st.stopped++;
                if (!hvp::bnb_pruned(c, inc)) st.bad++;  // would have stopped a QP that is not pruned
            }
            st.max_err = fmax(st.max_err, fabs(obj - c) / (1.0 + fabs(c)));
        }
        return true;
    };
    const double v0 = prm[1];
    std::vector<Node> lvl, nxt;
    Node root{0, v0, v0, -1e300, 0, 0, 0, 0};
    double ystar[N];
    double c0;
    if (!qp(0, 0, v0, v0, c0, ystar, false)) return;
    root.lb = c0;
    root.steps = last_steps;
    root.nact = last_nact;
    uint64_t code;
    double c1;
    if (hvp::bnb_dive<N>(S, C, v0, ystar, &code) && qp(code, N, 0.0, -1.0, c1, nullptr, false)) inc = c1;
    lvl.push_back(root);
    for (int k = 1; k <= N && !lvl.empty(); ++k) {
        nxt.clear();
        for (const Node& p : lvl) {
            if (hvp::bnb_pruned(p.lb, inc)) continue;
            for (int r = 0; r < S.n_regions; ++r) {
                Node c;
                if (!hvp::bnb_child(S, C, k - 1, p.lo, p.hi, r, &c.lo, &c.hi)) continue;
                c.code = hvp::code_with(p.code, k - 1, r);
                c.psteps = p.steps;
                c.pnact = p.nact;
                nxt.push_back(c);
            }
        }
        for (Node& c : nxt) {
            double lb;
            const bool good = qp(c.code, k, c.lo, c.hi, lb, nullptr, true);
            c.steps = last_steps;
            c.nact = last_nact;
            st.lvl_of.push_back(k);
            st.par_steps.push_back(c.psteps);
            st.par_nact.push_back(c.pnact);
            st.nact.push_back(c.nact);
            c.lb = good ? lb : (k < N ? -1e300 : 1e300);
            if (k == N && good) inc = fmin(inc, lb);
        }
        lvl.swap(nxt);
    }
}

}  // namespace

extern "C" int diag_dualstop(const hvp_problem* P, const hvp_system* systems, int B, const int32_t* sys,
                             const int32_t* role, const double* params, double marg, int gen, long long* out,
                             double* err, int* rec) {
    const hvp::Consts C = make_consts(*P);
    Stat tot;
    std::vector<Stat> per(B);
#pragma omp parallel for schedule(dynamic, 16)
    for (int i = 0; i < B; ++i) {
        if (P->N == 5) one<5>(systems[sys[i]], C, role[i], params + (size_t)i * C.stride, marg, per[i]);
    }
    // wave model: the QPs of consecutive instances in generations of `gen` lanes, each
    // generation as long as its slowest lane
    std::vector<int> full, stop;
    for (auto& s : per) {
        tot.qps += s.qps;
        tot.steps += s.steps;
        tot.steps_stop += s.steps_stop;
        tot.stopped += s.stopped;
        tot.bad += s.bad;
        tot.max_err = fmax(tot.max_err, s.max_err);
        full.insert(full.end(), s.full.begin(), s.full.end());
        stop.insert(stop.end(), s.stop.begin(), s.stop.end());
    }
    long long gf = 0, gs = 0;
    for (size_t a = 0; a < full.size(); a += gen) {
        int mf = 0, ms = 0;
        for (size_t b = a; b < a + gen && b < full.size(); ++b) {
            mf = full[b] > mf ? full[b] : mf;
            ms = stop[b] > ms ? stop[b] : ms;
        }
        gf += mf;
        gs += ms;
    }
    if (rec) {  // per QP: level, parent steps, parent nact, own steps, own nact, steps with the dual stop
        long long j = 0;
        for (auto& s : per)
            for (size_t a = 0; a < s.full.size(); ++a, ++j) {
                rec[6 * j + 0] = s.lvl_of[a];
                rec[6 * j + 5] = s.stop[a];
                rec[6 * j + 1] = s.par_steps[a];
                rec[6 * j + 2] = s.par_nact[a];
                rec[6 * j + 3] = s.full[a];
                rec[6 * j + 4] = s.nact[a];
            }
    }
    out[0] = tot.qps;
    out[1] = tot.steps;
    out[2] = tot.steps_stop;
    out[3] = tot.stopped;
    out[4] = tot.bad;
    out[5] = gf;
    out[6] = gs;
    *err = tot.max_err;
    return 0;
}
