// hvp_cent.hip -- the centralised MLD path of libhvpsolve.so (MpcMldCent, mpcs/cent_mld.py):
// the wave-per-platoon branch-and-bound kernel (hvp_cent_bnb.h) and hvp_cent_solve_batch
// (include/hvp.h).  A translation unit of its own: the search kernel is large and builds in
// seconds here instead of inside the decentralised kernels' unit.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#define HVP_HD __host__ __device__
#include "hvp.h"
#include "hvp_cent_bnb.h"
#include "hvp_internal.h"

using hvp_detail::fail;

// ================================================================== centralised MLD (MpcMldCent)
// One workgroup = one wavefront per platoon: the platoon's whole branch and bound
// (hvp_cent_bnb.h) runs inside the wave, J / R of its QPs in dynamic LDS (2 V (V+1) doubles,
// 41 KB at n = 10, N = 5: three platoons per CU).  Then the wave writes the winner: lane
// t = i N + a stores u_{i,a}, x_{i,a+1}, region and gear.
//
// Heavy platoons (a search past kSplitBudget QPs) split: their open DFS frames become subtree
// tasks that rounds of k_cent_tasks spread over every wave of the chip (the platoon's incumbent
// shared through its PlatoonRec), and k_cent_final picks and writes their winners.  A batch's
// time was set by its few heaviest platoons (one wave each, ~1 ms per QP, up to 1e5 QPs).
constexpr int kSplitBudget = 1000;  // QPs of a platoon's own search before it splits (p90: ~500)
constexpr int kTaskBudget = 256;    // QPs of a subtree task before it splits again
constexpr int kTaskRounds = 4096;   // bound on the rounds of k_cent_tasks (one host read each)

struct Epilogue {
    double* u_out;
    double* x_out;
    int8_t* region_out;
    int8_t* gear_out;
    double* cost_out;
    int32_t* status_out;
    int32_t* nodes_out;
    int32_t* iters_out;
    unsigned long long* counter;
};

__device__ inline hvp::cent::Inst cent_inst(int p, int n, int N, int leader, int lsp, const hvp_system* systems,
                                            const int32_t* sys, const double* x0, const double* xl, int debug) {
    hvp::cent::Inst I;
    I.n = n;
    I.N = N;
    I.V = n * N;
    I.L = leader;
    I.lsp = lsp != 0;
    I.systems = systems;
    I.vsys = sys + (size_t)p * n;
    I.x0 = x0 + (size_t)p * 2 * n;
    I.xl = xl + (size_t)p * 2 * (N + 1);
    I.debug = debug;
    return I;
}

// the winner's outputs (lanes' L.y and st.vcode hold it when res.status is HVP_OPTIMAL)
__device__ inline void cent_write(int p, hvp::cent::Lane& L, const hvp::Consts& C, const hvp::cent::Inst& I,
                                  const hvp::cent::Search& st, const hvp::cent::Result& res, const Epilogue& E) {
    using namespace hvp::cent;
    const int t = lane();
    const int n = I.n, N = I.N, V = I.V;
    const bool win = res.status == HVP_OPTIMAL;
    const int i = t < V ? t / N : 0, a = t < V ? t % N : 0;
    const uint64_t ci = bc(st.vcode, i);
    double u = 0.0;
    if (win) direct_cost(L, C, I, ci, N, &u);  // wave-uniform branch
    const double yv = win && t < V ? L.y : 0.0;
    const double cum = vehicle_prefix(yv, N);
    if (t < V) {
        const hvp_system& Sv = I.systems[I.vsys[i]];
        const size_t veh = (size_t)p * n + i;
        const double p0 = I.x0[2 * i], v0 = I.x0[2 * i + 1];
        if (E.x_out) {
            double* xo = E.x_out + veh * 2 * (N + 1);
            if (a == 0) {
                xo[0] = p0;
                xo[N + 1] = v0;
            }
            // no solution: the constant-velocity trajectory with u = 0 (as k_bnb_finish)
            xo[a + 1] = win ? p0 + Sv.ts * v0 + Sv.ts * cum : p0 + Sv.ts * v0 * (a + 1);
            xo[N + 1 + a + 1] = win ? yv : v0;
        }
        if (E.u_out) E.u_out[veh * N + a] = win ? u : 0.0;
        const int r = hvp::code_region(ci, a);
        if (E.region_out) E.region_out[veh * N + a] = (int8_t)(win ? r : -1);
        if (E.gear_out) E.gear_out[veh * N + a] = (int8_t)(win ? Sv.gear[r] : 0);
    }
    if (t == 0) {
        E.cost_out[p] = win ? res.cost : 1e300;
        E.status_out[p] = res.status;
        if (E.nodes_out) E.nodes_out[p] = res.nodes;
        if (E.iters_out) E.iters_out[p] = res.iters;
        atomicAdd(&E.counter[0], (unsigned long long)res.nodes);
        atomicAdd(&E.counter[1], (unsigned long long)res.iters);
    }
}

__global__ __launch_bounds__(64) void k_cent_init(int P, hvp::cent::PlatoonRec* rec, double inc0) {
    const int p = blockIdx.x * 64 + threadIdx.x;
    if (p >= P) return;
    rec[p].inc_key = inc0 < 1e300 ? hvp::cent::ckey(inc0) : ~0ull;
    rec[p].fail_key = ~0ull;
    rec[p].nodes = rec[p].iters = 0;
    rec[p].tie_count = 0;
    rec[p].flags = 0;
}

template <bool L1>
__global__ __launch_bounds__(64) void k_cent_bnb(int P, int n, int N, int leader, int lsp,
                                                 const hvp_system* __restrict__ systems,
                                                 const int32_t* __restrict__ sys, const double* __restrict__ x0,
                                                 const double* __restrict__ xl, const hvp::Consts* __restrict__ Cp, int nreg_max,
                                                 int max_nodes, int exhaustive, int max_iter, int debug,
                                                 hvp::cent::Child* frames, uint64_t* ties, hvp::cent::SplitWs ws,
                                                 Epilogue E) {
    using namespace hvp::cent;
    extern __shared__ double cent_lds[];
    const hvp::Consts& C = *Cp;  // in global memory: lane-indexed rows (C.dec[a]) stay loads
    const int p = blockIdx.x;
    if (p >= P) return;
    const int V = n * N;
    const Lds S = lds_carve(cent_lds, V);
    const Inst I = cent_inst(p, n, N, leader, lsp, systems, sys, x0, xl, debug);
    Lane L;
    Search st;
    Result res;
    SplitArgs sa;
    const bool split = ws.budget > 0 && !exhaustive;
    if (split) {
        sa.mode = 1;
        sa.budget = ws.budget;
        sa.p = p;
        sa.task = nullptr;
        sa.rec = ws.rec + p;
        sa.tie_g = ws.tie_g + (size_t)p * kTieG * n;
        sa.tie_gc = ws.tie_gc + (size_t)p * kTieG;
        sa.out = ws.out;
        sa.out_count = ws.out_count;
        sa.out_cap = ws.out_cap;
    }
    bnb_platoon<L1>(L, S, C, I, st, frames + (size_t)p * V * nreg_max, nreg_max, ties + (size_t)p * kTie * n,
                    max_nodes, exhaustive != 0, max_iter, res, split ? &sa : nullptr);
    if (res.status == kSplit) return;  // k_cent_final writes it
    cent_write(p, L, C, I, st, res, E);
}

// One round of subtree tasks: persistent waves claim tasks of any split platoon.  Each wave has
// its own DFS frames and tie slice (frames_w, ties_w at its wave index).
template <bool L1>
__global__ __launch_bounds__(64) void k_cent_tasks(int n, int N, int leader, int lsp,
                                                   const hvp_system* __restrict__ systems,
                                                   const int32_t* __restrict__ sys, const double* __restrict__ x0,
                                                   const double* __restrict__ xl, const hvp::Consts* __restrict__ Cp,
                                                   int nreg_max, int max_nodes, int max_iter, int debug,
                                                   hvp::cent::Child* frames_w, uint64_t* ties_w, hvp::cent::SplitWs ws) {
    using namespace hvp::cent;
    extern __shared__ double cent_lds[];
    const hvp::Consts& C = *Cp;
    const int t = lane();
    const int V = n * N;
    const Lds S = lds_carve(cent_lds, V);
    Child* frames = frames_w + (size_t)blockIdx.x * V * nreg_max;
    uint64_t* ties = ties_w + (size_t)blockIdx.x * kTie * n;
    for (;;) {
        uint64_t q = 0;
        if (t == 0) q = atomicAdd(ws.in_claim, 1ull);
        q = bcu(q, 0);
        if (q >= ws.in_count) break;
        const Task* tk = ws.in + q;
        const int p = tk->p;
        PlatoonRec* rec = ws.rec + p;
        uint64_t done_nodes = 0, ik = 0;
        if (t == 0) {
            done_nodes = __atomic_load_n(&rec->nodes, __ATOMIC_RELAXED);
            ik = __atomic_load_n(&rec->inc_key, __ATOMIC_RELAXED);
        }
        done_nodes = bcu(done_nodes, 0);
        const double incg = kcost(bcu(ik, 0));
        if (incg < __builtin_inf() && hvp::bnb_pruned(tk->lb, incg)) continue;  // pruned meanwhile
        if ((long long)done_nodes >= (long long)max_nodes) {  // the platoon's QP cap
            if (t == 0) atomicOr(&rec->flags, REC_NODE_LIMIT);
            continue;
        }
        const Inst I = cent_inst(p, n, N, leader, lsp, systems, sys, x0, xl, debug);
        SplitArgs sa;
        sa.mode = 2;
        sa.budget = ws.budget;
        sa.p = p;
        sa.task = tk;
        sa.rec = rec;
        sa.tie_g = ws.tie_g + (size_t)p * kTieG * n;
        sa.tie_gc = ws.tie_gc + (size_t)p * kTieG;
        sa.out = ws.out;
        sa.out_count = ws.out_count;
        sa.out_cap = ws.out_cap;
        Lane L;
        Search st;
        Result res;
        const long long c0 = debug ? (long long)wall_clock64() : 0;
        bnb_platoon<L1>(L, S, C, I, st, frames, nreg_max, ties, max_nodes - (int)done_nodes, false, max_iter, res, &sa);
        const long long dt = debug ? (long long)wall_clock64() - c0 : 0;
        if (t == 0 && debug != 6 && (debug >= 4 || (debug && (dt > 50000000ll || res.iters > 200 * (res.nodes + 1)))))
            printf("[cent-task] p %d d0 %d lb %.6g inc %.6g nodes %d iters %d ticks %lld\n", p, tk->d0, tk->lb, incg,
                   res.nodes, res.iters, dt);
    }
}

// tasks left when the round bound is reached: their platoons end as HVP_MAXITER (never a
// possibly wrong answer)
__global__ __launch_bounds__(64) void k_cent_abandon(const hvp::cent::Task* tasks, unsigned long long count,
                                                     hvp::cent::PlatoonRec* rec) {
    const unsigned long long q = (unsigned long long)blockIdx.x * 64 + threadIdx.x;
    if (q < count) atomicOr(&rec[tasks[q].p].flags, hvp::cent::REC_NODE_LIMIT);
}

// Winner of every split platoon: the lexicographically first (time-major) merged leaf within
// 1e-9 relative of the shared incumbent, re-solved for its trajectory (the oracle's rule).
template <bool L1>
__global__ __launch_bounds__(64) void k_cent_final(int P, int n, int N, int leader, int lsp,
                                                   const hvp_system* __restrict__ systems,
                                                   const int32_t* __restrict__ sys, const double* __restrict__ x0,
                                                   const double* __restrict__ xl, const hvp::Consts* __restrict__ Cp,
                                                   int max_iter, int debug, hvp::cent::SplitWs ws, Epilogue E) {
    using namespace hvp::cent;
    extern __shared__ double cent_lds[];
    const hvp::Consts& C = *Cp;
    const int p = blockIdx.x;
    if (p >= P) return;
    const PlatoonRec rec = ws.rec[p];
    if (!(rec.flags & REC_SPLIT)) return;
    const int t = lane();
    const int V = n * N;
    const Lds S = lds_carve(cent_lds, V);
    const Inst I = cent_inst(p, n, N, leader, lsp, systems, sys, x0, xl, debug);
    Lane L;
    Search st;
    Result res;
    res.nodes = (int)rec.nodes;
    res.iters = (int)rec.iters;
    res.cost = __builtin_inf();
    st.vcode = 0;
    const double inc = kcost(rec.inc_key);
    const int ntie = rec.tie_count < kTieG ? rec.tie_count : kTieG;
    const double fail_lb = kcost(rec.fail_key);
    if (rec.flags & REC_NODE_LIMIT) res.status = HVP_MAXITER;
    else if (rec.flags & REC_TIE_OVER) res.status = HVP_OVERFLOW;
    else if (!(inc < __builtin_inf())) res.status = fail_lb < __builtin_inf() ? HVP_MAXITER : HVP_INFEASIBLE;
    else res.status = HVP_OPTIMAL;
    if (res.status == HVP_OPTIMAL) {
        const double tol = 1e-9 * fmax(1.0, fabs(inc));
        int win = -1;
        uint64_t wcode = 0;
        for (int j = 0; j < ntie; ++j) {
            const double cj = ws.tie_gc[(size_t)p * kTieG + j];
            if (!(cj <= inc + tol)) continue;
            const uint64_t cj_code = t < n ? ws.tie_g[((size_t)p * kTieG + j) * n + t] : 0;
            if (win < 0 || joint_less(cj_code, wcode, n, N)) {
                win = j;
                wcode = cj_code;
            }
        }
        st.vcode = wcode;
        double c = 0.0;
        int it = 0;
        Prof pf;
        const int q = win < 0 ? QP_FAILED : platoon_qp<L1>(L, S, C, I, st.vcode, 0.0, 0.0, V, max_iter, c, it, pf);
        // a failed leaf whose bound is not above the incumbent could hide the optimum
        res.status = (fail_lb < __builtin_inf() && !hvp::bnb_pruned(fail_lb, inc)) ? HVP_MAXITER : HVP_OPTIMAL;
        if (q != QP_OK) res.status = HVP_MAXITER;
        res.cost = c;
    }
    cent_write(p, L, C, I, st, res, E);
}


extern "C" {

int hvp_cent_solve_batch(hvp_handle* h, int P, int n, int leader_index, int real_vehicle_as_reference,
                         const int32_t* sys, const double* x0, const double* leader_x, int max_nodes, double* u_out,
                         double* x_out, int8_t* region_out, int8_t* gear_out, double* cost_out, int32_t* status_out,
                         int32_t* nodes_out, int32_t* iters_out, void* stream) {
    if (!h) return fail(HVP_E_ARG, "hvp_cent_solve_batch: null handle");
    if (h->prob.formulation != HVP_FORM_CENT)
        return fail(HVP_E_ARG, "hvp_cent_solve_batch: the handle is not an HVP_FORM_CENT problem");
    const int N = h->prob.N;
    if (P < 0 || n < 1 || n > hvp::cent::kMaxVeh || n * N > hvp::cent::kMaxV)
        return fail(HVP_E_UNSUPPORTED, "hvp_cent_solve_batch: need 1 <= n <= " + std::to_string(hvp::cent::kMaxVeh) +
                                           " and n * N <= " + std::to_string(hvp::cent::kMaxV));
    if (leader_index < 0 || leader_index >= n) return fail(HVP_E_ARG, "hvp_cent_solve_batch: leader_index out of range");
    if (real_vehicle_as_reference && leader_index != 0)
        return fail(HVP_E_UNSUPPORTED, "hvp_cent_solve_batch: real_vehicle_as_reference needs leader_index 0 "
                                       "(mpcs/cent_mld.py:63-66)");
    if (P == 0) return 0;
    if (!sys || !x0 || !leader_x || !u_out || !cost_out || !status_out)
        return fail(HVP_E_ARG, "hvp_cent_solve_batch: bad argument");
    HIP_TRY(hipSetDevice(h->device));
    hipStream_t st = (hipStream_t)stream;
    const int V = n * N;
    const size_t fb = (size_t)P * V * h->nreg_max * sizeof(hvp::cent::Child);
    const size_t tb = (size_t)P * hvp::cent::kTie * n * sizeof(uint64_t);
    if (fb > h->cent_frames_bytes || tb > h->cent_ties_bytes) {
        HIP_TRY(hipDeviceSynchronize());
        if (fb > h->cent_frames_bytes) {
            (void)hipFree(h->cent_frames);
            h->cent_frames = nullptr;
            h->cent_frames_bytes = 0;
            if (hipMalloc(&h->cent_frames, fb) != hipSuccess)
                return fail(HVP_E_NOMEM, "hvp_cent_solve_batch: device allocation failed");
            h->cent_frames_bytes = fb;
        }
        if (tb > h->cent_ties_bytes) {
            (void)hipFree(h->cent_ties);
            h->cent_ties = nullptr;
            h->cent_ties_bytes = 0;
            if (hipMalloc(&h->cent_ties, tb) != hipSuccess)
                return fail(HVP_E_NOMEM, "hvp_cent_solve_batch: device allocation failed");
            h->cent_ties_bytes = tb;
        }
    }
    if (!h->d_consts) {
        if (hipMalloc(&h->d_consts, sizeof(hvp::Consts)) != hipSuccess)
            return fail(HVP_E_NOMEM, "hvp_cent_solve_batch: device allocation failed");
        HIP_TRY(hipMemcpy(h->d_consts, &h->C, sizeof(hvp::Consts), hipMemcpyHostToDevice));
    }
    // the min_1_norm cost (the MILP, hvp_cent_l1.h) runs its own instantiation of the search kernels
    const bool l1 = h->C.l1 != 0;
    const void* kb = l1 ? (const void*)k_cent_bnb<true> : (const void*)k_cent_bnb<false>;
    const void* kt = l1 ? (const void*)k_cent_tasks<true> : (const void*)k_cent_tasks<false>;
    const void* kf = l1 ? (const void*)k_cent_final<true> : (const void*)k_cent_final<false>;
    const size_t lds = hvp::cent::lds_doubles(V, l1) * sizeof(double);
    HIP_TRY(hipFuncSetAttribute(kb, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    HIP_TRY(hipFuncSetAttribute(kt, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    HIP_TRY(hipFuncSetAttribute(kf, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    HIP_TRY(hipMemsetAsync(h->g_counter, 0, 8 * sizeof(unsigned long long), st));
    const int exhaustive = h->prob.method == HVP_METHOD_ENUMERATE ? 1 : 0;
    const char* dbg = std::getenv("HVP_CENT_DEBUG");  // diagnostics: printf of failing QPs
    const int debug = dbg && dbg[0] ? std::atoi(dbg) : 0;  // 1: failures, 2: + every GI step, 6: QPs per depth
    const int cap = max_nodes > 0 ? max_nodes : 2000000;
    const int max_iter = 8 * hvp::cent::ROWS * V;  // active-set iterations per QP
    // split-search workspace: platoon records, merged tie lists, two task lists (ping-pong),
    // counters, and per-wave DFS frames / tie slices of the task kernel
    using hvp::cent::kTie;
    using hvp::cent::kTieG;
    const int waves = std::max(1, h->n_cu) * 3;  // LDS: three wave QPs per CU
    // task list capacity; a search whose open frames do not fit searches on in its wave (hvp_cent_bnb.h
    // export_tasks).  HVP_CENT_TASK_CAP (tests) shrinks it to exercise that path.
    long long task_cap = std::max<long long>(1 << 16, 64LL * P);
    if (const char* tc = std::getenv("HVP_CENT_TASK_CAP")) {
        task_cap = std::max<long long>(1, std::atoll(tc));
        static bool said = false;
        if (!said) std::fprintf(stderr, "[hvp] HVP_CENT_TASK_CAP=%lld: the split-task queue holds %lld tasks "
                                        "(test knob; answers unchanged, searches that do not fit stay in their wave)\n",
                                task_cap, task_cap);
        said = true;
    }
    auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
    const size_t b_rec = al(sizeof(hvp::cent::PlatoonRec) * P), b_tg = al(sizeof(uint64_t) * P * kTieG * n),
                 b_tgc = al(sizeof(double) * P * kTieG), b_task = al(sizeof(hvp::cent::Task) * task_cap),
                 b_cnt = al(8 * sizeof(unsigned long long)),
                 b_wf = al(sizeof(hvp::cent::Child) * (size_t)waves * V * h->nreg_max),
                 b_wt = al(sizeof(uint64_t) * (size_t)waves * kTie * n);
    const size_t sb = b_rec + b_tg + b_tgc + 2 * b_task + b_cnt + b_wf + b_wt;
    if (sb > h->cent_split_bytes) {
        HIP_TRY(hipDeviceSynchronize());
        (void)hipFree(h->cent_split);
        h->cent_split = nullptr;
        h->cent_split_bytes = 0;
        if (hipMalloc(&h->cent_split, sb) != hipSuccess)
            return fail(HVP_E_NOMEM, "hvp_cent_solve_batch: device allocation failed");
        h->cent_split_bytes = sb;
    }
    char* cp = h->cent_split;
    auto take = [&](size_t b) { char* r = cp; cp += b; return r; };
    hvp::cent::SplitWs ws{};
    ws.rec = (hvp::cent::PlatoonRec*)take(b_rec);
    ws.tie_g = (uint64_t*)take(b_tg);
    ws.tie_gc = (double*)take(b_tgc);
    hvp::cent::Task* lists[2] = {(hvp::cent::Task*)take(b_task), (hvp::cent::Task*)take(b_task)};
    unsigned long long* cnt = (unsigned long long*)take(b_cnt);  // [0], [1] list sizes, [2] claim
    hvp::cent::Child* frames_w = (hvp::cent::Child*)take(b_wf);
    uint64_t* ties_w = (uint64_t*)take(b_wt);
    ws.out_cap = task_cap;
    ws.budget = exhaustive ? 0 : kSplitBudget;
    if (const char* b = std::getenv("HVP_CENT_SPLIT")) ws.budget = std::atoi(b);  // 0: never split
    Epilogue E{u_out, x_out, region_out, gear_out, cost_out, status_out, nodes_out, iters_out, h->g_counter};
    HIP_TRY(hipMemsetAsync(cnt, 0, 8 * sizeof(unsigned long long), st));
    // diagnostics (HVP_CENT_INC, split searches only): every platoon starts from this incumbent
    const char* ie = std::getenv("HVP_CENT_INC");
    const double inc0 = ie && ie[0] && ws.budget > 0 ? std::atof(ie) : 1e300;
    if (inc0 < 1e300) {  // a diagnostic that changes answers: never silent
        static bool said = false;
        if (!said) std::fprintf(stderr, "[hvp] HVP_CENT_INC=%g: every split search starts from this incumbent "
                                        "(platoons whose optimum lies above it come back INFEASIBLE)\n", inc0);
        said = true;
    }
    hipLaunchKernelGGL(k_cent_init, dim3((P + 63) / 64), dim3(64), 0, st, P, ws.rec, inc0);
    HIP_TRY(hipEventRecord(h->ev0, st));
    HIP_TRY(hipEventRecord(h->evq0, st));
    ws.out = lists[0];
    ws.out_count = cnt + 0;
    if (l1)
        hipLaunchKernelGGL(k_cent_bnb<true>, dim3(P), dim3(64), lds, st, P, n, N, leader_index,
                           real_vehicle_as_reference ? 1 : 0, h->d_sys, sys, x0, leader_x, h->d_consts, h->nreg_max, cap,
                           exhaustive, max_iter, debug, h->cent_frames, h->cent_ties, ws, E);
    else
        hipLaunchKernelGGL(k_cent_bnb<false>, dim3(P), dim3(64), lds, st, P, n, N, leader_index,
                           real_vehicle_as_reference ? 1 : 0, h->d_sys, sys, x0, leader_x, h->d_consts, h->nreg_max, cap,
                           exhaustive, max_iter, debug, h->cent_frames, h->cent_ties, ws, E);
    HIP_TRY(hipGetLastError());
    if (ws.budget > 0) {
        // rounds of subtree tasks until none is left (one host read of the task count per round)
        int cur = 0;
        unsigned long long left = 0;
        ws.budget = kTaskBudget;
        if (const char* b = std::getenv("HVP_CENT_TASK_BUDGET")) ws.budget = std::max(1, std::atoi(b));
        for (int r = 0; r < kTaskRounds; ++r) {
            HIP_TRY(hipMemcpyAsync(&left, cnt + cur, sizeof(left), hipMemcpyDeviceToHost, st));
            HIP_TRY(hipStreamSynchronize(st));
            if (debug) {
                unsigned long long prog[2] = {0, 0};
                (void)hipMemcpy(prog, h->g_counter, sizeof(prog), hipMemcpyDeviceToHost);
                std::fprintf(stderr, "[cent] split round %d: %llu tasks (QPs of finished searches so far %llu)\n", r,
                             left, prog[0]);
            }
            if (!left) break;
            ws.in = lists[cur];
            ws.in_count = std::min<unsigned long long>(left, (unsigned long long)task_cap);
            ws.in_claim = cnt + 2;
            ws.out = lists[cur ^ 1];
            ws.out_count = cnt + (cur ^ 1);
            HIP_TRY(hipMemsetAsync(cnt + 2, 0, sizeof(unsigned long long), st));
            HIP_TRY(hipMemsetAsync(cnt + (cur ^ 1), 0, sizeof(unsigned long long), st));
            if (l1)
                hipLaunchKernelGGL(k_cent_tasks<true>, dim3(waves), dim3(64), lds, st, n, N, leader_index,
                                   real_vehicle_as_reference ? 1 : 0, h->d_sys, sys, x0, leader_x, h->d_consts,
                                   h->nreg_max, cap, max_iter, debug, frames_w, ties_w, ws);
            else
                hipLaunchKernelGGL(k_cent_tasks<false>, dim3(waves), dim3(64), lds, st, n, N, leader_index,
                                   real_vehicle_as_reference ? 1 : 0, h->d_sys, sys, x0, leader_x, h->d_consts,
                                   h->nreg_max, cap, max_iter, debug, frames_w, ties_w, ws);
            HIP_TRY(hipGetLastError());
            cur ^= 1;
            left = 0;
        }
        if (!left) {
            HIP_TRY(hipMemcpyAsync(&left, cnt + cur, sizeof(left), hipMemcpyDeviceToHost, st));
            HIP_TRY(hipStreamSynchronize(st));
        }
        if (left) {
            const unsigned long long c = std::min<unsigned long long>(left, (unsigned long long)task_cap);
            hipLaunchKernelGGL(k_cent_abandon, dim3((unsigned)((c + 63) / 64)), dim3(64), 0, st, lists[cur], c, ws.rec);
            HIP_TRY(hipGetLastError());
        }
        if (l1)
            hipLaunchKernelGGL(k_cent_final<true>, dim3(P), dim3(64), lds, st, P, n, N, leader_index,
                               real_vehicle_as_reference ? 1 : 0, h->d_sys, sys, x0, leader_x, h->d_consts, max_iter,
                               debug, ws, E);
        else
            hipLaunchKernelGGL(k_cent_final<false>, dim3(P), dim3(64), lds, st, P, n, N, leader_index,
                               real_vehicle_as_reference ? 1 : 0, h->d_sys, sys, x0, leader_x, h->d_consts, max_iter,
                               debug, ws, E);
        HIP_TRY(hipGetLastError());
    }
    if (debug == 6) {  // QPs per depth of the search (hvp_cent_bnb.h g_cent_depth), summed over all platoons
        unsigned long long hist[3][64];
        HIP_TRY(hipStreamSynchronize(st));
        HIP_TRY(hipMemcpyFromSymbol(hist, HIP_SYMBOL(hvp::cent::g_cent_depth), sizeof(hist)));
        for (int d = 0; d < 64; ++d)
            if (hist[0][d] || hist[1][d])
                std::fprintf(stderr, "[cent-depth] fixed %2d (vehicle %d step %d): bound QPs %llu (above incumbent %llu), visits %llu\n",
                             d, d > 0 ? (d - 1) % n : -1, d > 0 ? (d - 1) / n : -1, hist[0][d], hist[2][d], hist[1][d]);
        const unsigned long long zero[3][64] = {};
        HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(hvp::cent::g_cent_depth), zero, sizeof(zero)));
    }
#ifdef HVP_CENT_PROF
    if (debug >= 3) {  // phase profile of the wave QP (hvp_cent.h Prof), summed over all platoons
        unsigned long long prof[16];
        HIP_TRY(hipStreamSynchronize(st));
        HIP_TRY(hipMemcpyFromSymbol(prof, HIP_SYMBOL(hvp::cent::g_cent_prof), sizeof(prof)));
        const char* names[12] = {"setup", "cholesky", "minimiser+J", "most-violated", "dv+z", "r-backsolve",
                                 "steps", "add", "drop", "direct-cost", "QPs", "GI-steps"};
        unsigned long long tot = 0;
        for (int k = 0; k < 10; ++k) tot += prof[k];
        std::printf("[cent-prof] cycles %llu, QPs %llu, GI steps %llu\n", tot, prof[10], prof[11]);
        for (int k = 0; k < 10; ++k)
            std::printf("[cent-prof]   %-14s %6.2f%%  %8.0f cycles/QP\n", names[k], 100.0 * prof[k] / (tot ? tot : 1),
                        (double)prof[k] / (prof[10] ? prof[10] : 1));
        const unsigned long long zero[16] = {};
        HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(hvp::cent::g_cent_prof), zero, sizeof(zero)));
    }
#endif
    HIP_TRY(hipEventRecord(h->evq1, st));
    HIP_TRY(hipEventRecord(h->ev1, st));
    h->last_stream = st;
    h->last_B = P;
    h->last_bnb = false;
    return 0;
}

}  // extern "C"
