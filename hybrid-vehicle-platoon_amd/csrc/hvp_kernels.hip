// hvp_kernels.hip -- MI355X (gfx950) batched hybrid-MPC solver and its C ABI (include/hvp.h).
//
// One hvp_solve_batch call solves B independent local MIQPs (fleet_decent_mld.py:316: the n
// agents of a platoon step, times any number of platoons / seeds / sweep points) in three
// launches on the caller's stream:
//
//   K_enum   one thread per instance: depth-first enumeration of the velocity-feasible region
//            sequences (exact interval reachability), reservation of a contiguous slice of the
//            global candidate list with ONE atomicAdd per instance, and the candidate codes
//            (4 bits per step) written in lexicographic order.
//   K_qp     one LANE per candidate (instance, sigma): the condensed velocity-space QP is built
//            and solved by a Mehrotra IPM entirely in registers (hvp_ipm.h); writes cost, status,
//            iteration count and v_1..v_N.  Grid-stride over the candidate count read on the
//            device, so no host round trip sits between K_enum and K_qp.  Consecutive lanes carry
//            consecutive candidates of the same instance: the instance block (38 doubles) is read
//            once per wave from L1/L2 and the lanes of a wave share the iteration count closely.
//   K_select one thread per instance: min over its candidates, tie rule (first sequence within
//            1e-9 relative of the minimum), reconstruction of u and x, status / node counts.
//
// Memory: everything lives in caller-owned device buffers plus a handle-owned workspace sized
// once by hvp_reserve (no allocation inside hvp_solve_batch, so a call can be graph-captured).
#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "hvp_lane.h"

namespace hvp_detail {
thread_local std::string g_err;
int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}
}  // namespace hvp_detail

using namespace hvp_k;

namespace {

hvp::Consts make_consts(const hvp_problem& p) {
    hvp::Consts C;
    std::memset(&C, 0, sizeof(C));
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
    // max_iter: the quadratic path's fallback IPM cap (default 60); min_1_norm: the LP interior
    // point's cap (default hvp::kL1MaxIter)
    C.max_iter = p.max_iter > 0 ? p.max_iter : (p.quadratic_cost ? 60 : hvp::kL1MaxIter);
    C.N = p.N;
    C.form = p.formulation;
    C.stride = p.formulation == HVP_FORM_ADMM    ? hvp_params_stride_admm(p.N)
               : p.formulation == HVP_FORM_GADMM ? hvp_params_stride_gadmm(p.N)
                                                 : hvp_params_stride(p.N);
    C.rho = p.rho;
    C.l1 = p.quadratic_cost ? 0 : 1;
    const char* lc = std::getenv("HVP_LEAF_GI_CAP");
    C.leaf_cap = lc && lc[0] ? std::max(0, std::atoi(lc)) : 0;
    if (C.leaf_cap > 0) {  // a test knob in the production library: never silent
        static bool said = false;
        if (!said) std::fprintf(stderr, "[hvp] HVP_LEAF_GI_CAP=%d: leaf QPs capped at %d active-set steps "
                                        "(the rest go through the interior-point fallback)\n", C.leaf_cap, C.leaf_cap);
        said = true;
    }
    const char* cc = std::getenv("HVP_CENT_CUT");
    C.cent_cut = cc && cc[0] ? (std::atoi(cc) != 0 ? 1 : 0) : 1;
    return C;
}

// ================================================================== ADMM consensus update
// ADMMCoordinator.get_control z/y update (fleet_naive_admm.py:421-468), one thread per
// (platoon, vehicle, state entry).  Thread (p, i, e) recomputes z of i-1, i, i+1 (3 loads each),
// so the y-updates and the next parameter blocks of vehicle i need no second pass:
//   y_front_i += rho (xf_i - z_{i-1}),  y_back_i += rho (xb_i - z_{i+1}),
//   params_i: y_front_i, z_front = z_{i-1}, y_back_i, z_back = z_{i+1}.
__device__ inline double admm_z_of(int i, int n, const double* x, const double* xf, const double* xb, size_t base,
                                   int stride2, int e) {
    // base = platoon's first instance; entries of instance j at (base + j) * stride2 + e
    double s = x[(base + i) * stride2 + e];
    int cnt = 1;
    if (i + 1 < n) { s += xf[(base + i + 1) * stride2 + e]; ++cnt; }
    if (i >= 1) { s += xb[(base + i - 1) * stride2 + e]; ++cnt; }
    return cnt == 3 ? s * (1.0 / 3.0) : (cnt == 2 ? 0.5 * s : s);
}

__global__ __launch_bounds__(kBlock) void k_admm_update(int P, int n, int N, double rho, int pstride,
                                                        const double* __restrict__ x, const double* __restrict__ xf,
                                                        const double* __restrict__ xb, double* __restrict__ y_front,
                                                        double* __restrict__ y_back, double* __restrict__ params,
                                                        double* __restrict__ z_out) {
    const int E = 2 * (N + 1);
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (long long)P * n * E) return;
    const int e = (int)(t % E);
    const long long inst = t / E;
    const int i = (int)(inst % n);
    const size_t base = (size_t)(inst - i);
    const double zi = admm_z_of(i, n, x, xf, xb, base, E, e);
    if (z_out) z_out[inst * E + e] = zi;
    double* prm = params + inst * pstride;
    if (i >= 1) {
        const double zm = admm_z_of(i - 1, n, x, xf, xb, base, E, e);
        const double yf = y_front[inst * E + e] + rho * (xf[inst * E + e] - zm);
        y_front[inst * E + e] = yf;
        prm[2 + e] = yf;
        prm[2 + E + e] = zm;
    }
    if (i + 1 < n) {
        const double zp = admm_z_of(i + 1, n, x, xf, xb, base, E, e);
        const double yb = y_back[inst * E + e] + rho * (xb[inst * E + e] - zp);
        y_back[inst * E + e] = yb;
        prm[2 + 2 * E + e] = yb;
        prm[2 + 3 * E + e] = zp;
    }
}

// consensus step, one thread per (held vehicle, state entry); z of i-1, i, i+1 recomputed per
// thread so the y-updates need no second pass
__device__ inline double gadmm_z(int j, int n, size_t base, const double* x, const double* xf, const double* xb,
                                 int E, int e, bool init) {
    double s = x[(base + j) * E + e];
    if (init) return s;
    int cnt = 1;
    if (j >= 1) { s += xb[(base + j - 1) * E + e]; ++cnt; }
    if (j + 1 < n) { s += xf[(base + j + 1) * E + e]; ++cnt; }
    return cnt == 3 ? s * (1.0 / 3.0) : (cnt == 2 ? 0.5 * s : s);
}

__global__ __launch_bounds__(kBlock) void k_gadmm_update(int P, int n, int lo, int m, int N, double rho, int stride,
                                                         const double* __restrict__ x, const double* __restrict__ xf,
                                                         const double* __restrict__ xb, double* __restrict__ params,
                                                         const int32_t* __restrict__ state, int init) {
    const int E = 2 * (N + 1);
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (long long)P * m * E) return;
    const int e = (int)(t % E);
    const int b = (int)(t / E);
    const int p = b / m, i = lo + b % m;
    if (!(state[p] & 1)) return;
    const size_t base = (size_t)p * n;
    double* prm = params + (size_t)b * stride;
    const bool in = init != 0;
    const double zi = gadmm_z(i, n, base, x, xf, xb, E, e, in);
    prm[2 + 6 * E + e] = zi;
    prm[2 + 5 * E + e] = in ? 0.0 : prm[2 + 5 * E + e] + rho * (x[(base + i) * E + e] - zi);
    if (i >= 1) {
        const double zm = gadmm_z(i - 1, n, base, x, xf, xb, E, e, in);
        prm[2 + E + e] = zm;
        prm[2 + e] = in ? 0.0 : prm[2 + e] + rho * (xf[(base + i) * E + e] - zm);
    }
    if (i + 1 < n) {
        const double zp = gadmm_z(i + 1, n, base, x, xf, xb, E, e, in);
        prm[2 + 3 * E + e] = zp;
        prm[2 + 2 * E + e] = in ? 0.0 : prm[2 + 2 * E + e] + rho * (xb[(base + i) * E + e] - zp);
    }
}

__device__ inline int gadmm_neighbour(const hvp_system& S, int r, bool up) {
    const double edge = up ? S.vhi[r] : S.vlo[r];
    const double tol = 1e-9 * (1.0 + fabs(edge));
    for (int q = 0; q < S.n_regions; ++q) {
        if (q == r) continue;
        if (fabs((up ? S.vlo[q] : S.vhi[q]) - edge) <= tol) return q;
    }
    return -1;
}

__global__ __launch_bounds__(kBlock) void k_gadmm_switch(int P, int n, int lo, int m, int N,
                                                         const hvp_system* __restrict__ systems,
                                                         const int32_t* __restrict__ sys,
                                                         const uint32_t* __restrict__ edge, int8_t* __restrict__ seq,
                                                         int32_t* __restrict__ state) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= P * m) return;
    const int p = b / m;
    if (!(state[p] & 1)) return;
    const hvp_system& S = systems[sys[b]];
    const uint32_t bits = edge[b];
    bool changed = false;
    for (int k = 1; k < N; ++k) {
        const int r = seq[(size_t)b * N + k];
        int q = -1;
        if ((bits >> (2 * (k - 1))) & 1u) q = gadmm_neighbour(S, r, false);
        else if ((bits >> (2 * (k - 1) + 1)) & 1u) q = gadmm_neighbour(S, r, true);
        if (q >= 0) {
            seq[(size_t)b * N + k] = (int8_t)q;
            changed = true;
        }
    }
    if (changed) atomicOr(&state[p], 4);
}


void free_ws(Workspace& w) {
    (void)hipFree(w.inst_off);
    (void)hipFree(w.inst_cnt);
    (void)hipFree(w.inst_flag);
    (void)hipFree(w.counter);
    (void)hipFree(w.redo);
    (void)hipFree(w.task_inst);
    (void)hipFree(w.task_code);
    (void)hipFree(w.task_cost);
    (void)hipFree(w.task_stat);
    (void)hipFree(w.task_y);
    for (int b = 0; b < 2; ++b) {
        (void)hipFree(w.nd_inst[b]);
        (void)hipFree(w.nd_code[b]);
        (void)hipFree(w.nd_lo[b]);
        (void)hipFree(w.nd_hi[b]);
        (void)hipFree(w.nd_lb[b]);
    }
    (void)hipFree(w.leaf_stat);
    (void)hipFree(w.inc);
    (void)hipFree(w.key);
    (void)hipFree(w.nodes);
    (void)hipFree(w.iters);
    (void)hipFree(w.lvl);
    (void)hipFree(w.iq);
    (void)hipFree(w.dv_mem);
    (void)hipFree(w.win);
    w = Workspace{};
}

int64_t default_capacity(int N, int B, bool bnb, int form) {
    if (bnb) {
        // nodes of ONE tree level, pooled over the batch (C2..C5 means: 3 leaves at N = 5, 4 at
        // N = 10, 30 at N = 15; the widest level a few times that; the naive-ADMM local trees,
        // with their hinge states, ~8 per level at C3, a heavy tail far beyond -- 4x room)
        int64_t per = N <= 8 ? 64 : (N <= 12 ? 256 : 1024);
        if (form == HVP_FORM_ADMM) per *= 4;
        return per * (int64_t)std::max(B, 1);
    }
    // per-instance average budget: 7^N capped (N = 5: mean ~30, max ~85 region sequences)
    int64_t per = 1;
    for (int k = 0; k < N; ++k) per = std::min<int64_t>(per * 7, 1 << 20);
    per = std::min<int64_t>(per, N <= 5 ? 256 : (N <= 6 ? 1024 : 4096));
    return per * (int64_t)std::max(B, 1);
}

bool create_events(hipEvent_t* ev, int n) {
    for (int i = 0; i < n; ++i)
        if (hipEventCreate(&ev[i]) != hipSuccess) return false;
    return true;
}

bool valid_system(const hvp_system& s, std::string* why) {
    if (s.n_regions < 1 || s.n_regions > HVP_MAX_REGIONS) { *why = "n_regions out of range"; return false; }
    if (!(s.ts > 0)) { *why = "ts must be > 0"; return false; }
    for (int r = 0; r < s.n_regions; ++r) {
        if (!(s.b[r] > 0)) { *why = "input gain b must be > 0"; return false; }
        if (s.vlo[r] > s.vhi[r]) { *why = "empty region interval"; return false; }
    }
    if (!(s.umin <= s.umax) || !(s.vmin <= s.vmax) || !(s.pmin <= s.pmax)) { *why = "empty box"; return false; }
    return true;
}

}  // namespace

// ===================================================================== C ABI
extern "C" {

int hvp_abi_version(void) { return HVP_ABI_VERSION; }

int hvp_abi_sizes(int32_t* sizes) {
    if (!sizes) return HVP_E_ARG;
    sizes[0] = (int32_t)sizeof(hvp_system);
    sizes[1] = (int32_t)sizeof(hvp_problem);
    sizes[2] = (int32_t)sizeof(hvp_stats);
    return 0;
}

int hvp_last_error(char* buf, size_t len) {
    if (!buf || len == 0) return HVP_E_ARG;
    std::snprintf(buf, len, "%s", hvp_detail::g_err.c_str());
    return 0;
}

int hvp_create(hvp_handle** out, const hvp_problem* problem, const hvp_system* systems, int n_systems, int device) {
    if (!out || !problem || !systems || n_systems <= 0) return fail(HVP_E_ARG, "hvp_create: null argument");
    *out = nullptr;
    if (problem->N < 2 || problem->N > HVP_MAX_N)
        return fail(HVP_E_UNSUPPORTED, "hvp_create: horizon N must be in [2, " + std::to_string(HVP_MAX_N) + "]");
    if (problem->method < HVP_METHOD_AUTO || problem->method > HVP_METHOD_BNB)
        return fail(HVP_E_ARG, "hvp_create: unknown method");
    if (problem->method == HVP_METHOD_ENUMERATE && problem->N > HVP_MAX_N_ENUM)
        return fail(HVP_E_UNSUPPORTED, "hvp_create: enumeration supports N <= " + std::to_string(HVP_MAX_N_ENUM) +
                                           " (use HVP_METHOD_BNB)");
    if (problem->formulation != HVP_FORM_DECENT && problem->formulation != HVP_FORM_ADMM &&
        problem->formulation != HVP_FORM_GADMM && problem->formulation != HVP_FORM_CENT)
        return fail(HVP_E_ARG, "hvp_create: unknown formulation");
    if (problem->formulation == HVP_FORM_GADMM && !(problem->rho > 0))
        return fail(HVP_E_ARG, "hvp_create: the switching-ADMM formulation needs rho > 0");
    if (problem->formulation == HVP_FORM_ADMM && problem->method == HVP_METHOD_ENUMERATE)
        return fail(HVP_E_UNSUPPORTED, "hvp_create: the ADMM formulation is solved by branch and bound only");
    if (problem->formulation == HVP_FORM_ADMM && !(problem->rho > 0))
        return fail(HVP_E_ARG, "hvp_create: the ADMM formulation needs rho > 0");
    if (problem->quadratic_cost != 1 && problem->quadratic_cost != 0)
        return fail(HVP_E_ARG, "hvp_create: quadratic_cost must be 1 (min_2_norm) or 0 (min_1_norm)");
    if (problem->quadratic_cost == 0 && problem->formulation == HVP_FORM_GADMM)
        return fail(HVP_E_UNSUPPORTED, "hvp_create: the min_1_norm cost runs for the HVP_FORM_DECENT, HVP_FORM_ADMM and "
                                       "HVP_FORM_CENT problems (fleet_g_admm.LocalMpc is quadratic)");
    for (int i = 0; i < n_systems; ++i) {
        std::string why;
        if (!valid_system(systems[i], &why)) return fail(HVP_E_ARG, "hvp_create: system " + std::to_string(i) + ": " + why);
    }
    HIP_TRY(hipSetDevice(device));
    hvp_handle* h = new hvp_handle();
    h->device = device;
    h->prob = *problem;
    h->C = make_consts(*problem);
    h->bnb = problem->method == HVP_METHOD_BNB ||
             (problem->method == HVP_METHOD_AUTO && problem->N > (problem->quadratic_cost ? kAutoEnumMaxN : kAutoEnumMaxNL1));
    h->n_systems = n_systems;
    for (int i = 0; i < n_systems; ++i) h->nreg_max = std::max(h->nreg_max, (int)systems[i].n_regions);
    (void)hipDeviceGetAttribute(&h->n_cu, hipDeviceAttributeMultiprocessorCount, device);
    if (hipMalloc(&h->d_sys, sizeof(hvp_system) * n_systems) != hipSuccess ||
        hipMemcpy(h->d_sys, systems, sizeof(hvp_system) * n_systems, hipMemcpyHostToDevice) != hipSuccess ||
        hipEventCreate(&h->ev0) != hipSuccess || hipEventCreate(&h->ev1) != hipSuccess ||
        hipEventCreate(&h->evq0) != hipSuccess || hipEventCreate(&h->evq1) != hipSuccess ||
        hipMalloc(&h->g_counter, 8 * sizeof(unsigned long long)) != hipSuccess ||
        hipMalloc(&h->d_consts, sizeof(hvp::Consts)) != hipSuccess ||
        hipMemcpy(h->d_consts, &h->C, sizeof(hvp::Consts), hipMemcpyHostToDevice) != hipSuccess ||
        hipMalloc(&h->d_ws, 2 * sizeof(hvp_detail::Workspace)) != hipSuccess ||
        hipMemset(h->g_counter, 0, 8 * sizeof(unsigned long long)) != hipSuccess ||
        !create_events(h->evb, 2 * (HVP_MAX_N + 1))) {
        hvp_destroy(h);
        return fail(HVP_E_HIP, "hvp_create: device allocation failed");
    }
    *out = h;
    return 0;
}

int hvp_reserve(hvp_handle* h, int max_batch, int64_t cap) {
    if (!h || max_batch <= 0) return fail(HVP_E_ARG, "hvp_reserve: bad argument");
    if (cap <= 0) cap = default_capacity(h->prob.N, max_batch, h->bnb, h->prob.formulation);
    if (max_batch <= h->ws.max_batch && cap <= h->ws.cap) return 0;
    HIP_TRY(hipSetDevice(h->device));
    HIP_TRY(hipDeviceSynchronize());
    max_batch = std::max(max_batch, h->ws.max_batch);
    cap = std::max<int64_t>(cap, h->ws.cap);
    free_ws(h->ws);
    Workspace& w = h->ws;
    const int N = h->prob.N;
    bool ok = hipMalloc(&w.inst_off, sizeof(int32_t) * max_batch) == hipSuccess &&
              hipMalloc(&w.inst_cnt, sizeof(int32_t) * max_batch) == hipSuccess &&
              hipMalloc(&w.inst_flag, sizeof(int32_t) * max_batch) == hipSuccess &&
              hipMalloc(&w.counter, sizeof(unsigned long long) * 8) == hipSuccess &&
              hipMalloc(&w.redo, sizeof(int32_t) * cap) == hipSuccess &&
              hipMalloc(&w.task_inst, sizeof(int32_t) * cap) == hipSuccess &&
              hipMalloc(&w.task_code, sizeof(uint32_t) * cap) == hipSuccess &&
              hipMalloc(&w.task_cost, sizeof(double) * cap) == hipSuccess &&
              hipMalloc(&w.task_stat, sizeof(int32_t) * cap) == hipSuccess &&
              hipMalloc(&w.task_y, sizeof(double) * cap * N) == hipSuccess;
    if (ok && h->bnb) {
        for (int b = 0; b < 2 && ok; ++b)
            ok = hipMalloc(&w.nd_inst[b], sizeof(int32_t) * cap) == hipSuccess &&
                 hipMalloc(&w.nd_code[b], sizeof(uint64_t) * cap) == hipSuccess &&
                 hipMalloc(&w.nd_lo[b], sizeof(double) * cap) == hipSuccess &&
                 hipMalloc(&w.nd_hi[b], sizeof(double) * cap) == hipSuccess &&
                 hipMalloc(&w.nd_lb[b], sizeof(double) * cap) == hipSuccess;
        ok = ok && hipMalloc(&w.leaf_stat, sizeof(int32_t) * cap) == hipSuccess &&
             hipMalloc(&w.inc, sizeof(unsigned long long) * max_batch) == hipSuccess &&
             hipMalloc(&w.key, sizeof(unsigned long long) * max_batch) == hipSuccess &&
             hipMalloc(&w.nodes, sizeof(int32_t) * max_batch) == hipSuccess &&
             hipMalloc(&w.iters, sizeof(int32_t) * max_batch) == hipSuccess &&
             hipMalloc(&w.win, sizeof(int32_t) * max_batch) == hipSuccess &&
             hipMalloc(&w.lvl, sizeof(unsigned long long) * 6 * (HVP_MAX_N + 1)) == hipSuccess;  // hvp_lane.h LevelList
        // K_inst_prep's per-instance QP part: H (NT) + f (N) + hf, hb (N - 1 each), one row per instance
        // padded to 16 doubles (hvp_lane.h kIqStride)
        if (ok && N <= HVP_MAX_N_ENUM)
            ok = hipMalloc(&w.iq, sizeof(double) * (size_t)max_batch * ((N * (N + 1) / 2 + 3 * N - 2 + 15) / 16 * 16)) ==
                 hipSuccess;
        // the dive list of the lane path (hvp_lane.h launch_bnb): 8-byte fields first
        if (ok && N <= HVP_MAX_N_ENUM) {
            constexpr size_t M = HVP_MAX_N + 1;
            const size_t mb = 3 * (size_t)max_batch;  // up to 3 dive leaves per instance (min_1_norm)
            const size_t bytes = 8 * (6 * M + 8) + mb * (8 * (4 + N) + 3 * 4);
            ok = hipMalloc(&w.dv_mem, bytes) == hipSuccess;
            if (ok) {
                char* c = w.dv_mem;
                auto take = [&c](size_t n) { char* r = c; c += n; return r; };
                w.dv_lvl = (unsigned long long*)take(8 * 6 * M);
                w.dv_counter = (unsigned long long*)take(8 * 8);
                w.dv_code = (uint64_t*)take(8 * mb);
                w.dv_lo = (double*)take(8 * mb);
                w.dv_hi = (double*)take(8 * mb);
                w.dv_lb = (double*)take(8 * mb);
                w.dv_y = (double*)take(8 * mb * N);
                w.dv_inst = (int32_t*)take(4 * mb);
                w.dv_stat = (int32_t*)take(4 * mb);
                w.dv_redo = (int32_t*)take(4 * mb);
            }
        }
    }
    if (!ok) {
        free_ws(w);
        return fail(HVP_E_NOMEM, "hvp_reserve: device allocation failed");
    }
    w.max_batch = max_batch;
    w.cap = cap;
    return 0;
}

static int solve_impl(hvp_handle* h, int B, const int32_t* sys, const int32_t* role, const double* params,
                      double* u_out, double* x_out, int8_t* region_out, int8_t* gear_out, double* cost_out,
                      int32_t* status_out, int32_t* nodes_out, int32_t* iters_out, void* stream, double* xf_out,
                      double* xb_out);

int hvp_solve_batch(hvp_handle* h, int B, const int32_t* sys, const int32_t* role, const double* params,
                    double* u_out, double* x_out, int8_t* region_out, int8_t* gear_out, double* cost_out,
                    int32_t* status_out, int32_t* nodes_out, int32_t* iters_out, void* stream) {
    return solve_impl(h, B, sys, role, params, u_out, x_out, region_out, gear_out, cost_out, status_out, nodes_out,
                      iters_out, stream, nullptr, nullptr);
}

int hvp_solve_admm_batch(hvp_handle* h, int B, const int32_t* sys, const int32_t* role, const double* params,
                         double* u_out, double* x_out, int8_t* region_out, int8_t* gear_out, double* cost_out,
                         int32_t* status_out, int32_t* nodes_out, int32_t* iters_out, double* xf_out, double* xb_out,
                         void* stream) {
    if (h && h->prob.formulation != HVP_FORM_ADMM)
        return fail(HVP_E_ARG, "hvp_solve_admm_batch: the handle is not an HVP_FORM_ADMM problem");
    return solve_impl(h, B, sys, role, params, u_out, x_out, region_out, gear_out, cost_out, status_out, nodes_out,
                      iters_out, stream, xf_out, xb_out);
}

int hvp_set_region_hint(hvp_handle* h, const int8_t* region_hint) {
    if (!h) return fail(HVP_E_ARG, "hvp_set_region_hint: null handle");
    h->region_hint = region_hint;
    return 0;
}

int hvp_set_node_records(hvp_handle* h, int enable) {
    if (!h) return fail(HVP_E_ARG, "hvp_set_node_records: null handle");
    h->nrec_enable = enable != 0;
    return 0;
}

static int solve_impl(hvp_handle* h, int B, const int32_t* sys, const int32_t* role, const double* params,
                      double* u_out, double* x_out, int8_t* region_out, int8_t* gear_out, double* cost_out,
                      int32_t* status_out, int32_t* nodes_out, int32_t* iters_out, void* stream, double* xf_out,
                      double* xb_out) {
    if (!h || B < 0 || (B > 0 && (!sys || !role || !params || !cost_out || !status_out)))
        return fail(HVP_E_ARG, "hvp_solve_batch: bad argument");
    if (h->prob.formulation == HVP_FORM_GADMM)
        return fail(HVP_E_ARG, "hvp_solve_batch: HVP_FORM_GADMM handles are solved by hvp_gadmm_solve");
    if (h->prob.formulation == HVP_FORM_CENT)
        return fail(HVP_E_ARG, "hvp_solve_batch: HVP_FORM_CENT handles are solved by hvp_cent_solve_batch");
    if (B == 0) return 0;
    if (B > h->ws.max_batch) {
        int rc = hvp_reserve(h, B, default_capacity(h->prob.N, B, h->bnb, h->prob.formulation));
        if (rc) return rc;
    }
    HIP_TRY(hipSetDevice(h->device));
    hipStream_t st = (hipStream_t)stream;
    // the region hint: naive-ADMM solves, and decentralised solves on the 16-lane path (N > 8)
    h->ws.hint = h->prob.formulation == HVP_FORM_ADMM ||
                         (h->prob.formulation == HVP_FORM_DECENT && h->prob.N > HVP_MAX_N_ENUM)
                     ? h->region_hint
                     : nullptr;
    if (h->bnb) {
        switch (h->prob.N) {
#define HVP_CASE(n) \
    case n: return launch_bnb<n>(h, B, sys, role, params, u_out, x_out, region_out, gear_out, cost_out, status_out, nodes_out, iters_out, st, xf_out, xb_out);
            HVP_CASE(2) HVP_CASE(3) HVP_CASE(4) HVP_CASE(5) HVP_CASE(6) HVP_CASE(7) HVP_CASE(8)
            HVP_CASE(9) HVP_CASE(10) HVP_CASE(11) HVP_CASE(12) HVP_CASE(13) HVP_CASE(14) HVP_CASE(15) HVP_CASE(16)
#undef HVP_CASE
            default: return fail(HVP_E_UNSUPPORTED, "hvp_solve_batch: unsupported N");
        }
    }
    switch (h->prob.N) {
#define HVP_CASE(n) \
    case n: return launch_all<n>(h, B, sys, role, params, u_out, x_out, region_out, gear_out, cost_out, status_out, nodes_out, iters_out, st);
        HVP_CASE(2) HVP_CASE(3) HVP_CASE(4) HVP_CASE(5) HVP_CASE(6) HVP_CASE(7) HVP_CASE(8)
#undef HVP_CASE
        default: return fail(HVP_E_UNSUPPORTED, "hvp_solve_batch: unsupported N");
    }
}

int hvp_evaluate_batch(hvp_handle* h, int B, const int32_t* sys, const int32_t* role, const double* params,
                       const int8_t* gear_in, const double* u_in, double* cost_out, int32_t* status_out, double* x_out,
                       void* stream) {
    if (!h || B < 0 || (B > 0 && (!sys || !role || !params || !gear_in || !u_in || !cost_out || !status_out)))
        return fail(HVP_E_ARG, "hvp_evaluate_batch: bad argument");
    if (h->prob.formulation != HVP_FORM_DECENT)
        return fail(HVP_E_UNSUPPORTED, "hvp_evaluate_batch: HVP_FORM_DECENT problems only");
    if (B == 0) return 0;
    HIP_TRY(hipSetDevice(h->device));
    hipStream_t st = (hipStream_t)stream;
    switch (h->prob.N) {
#define HVP_CASE(n) \
    case n: return launch_evaluate<n>(h, B, sys, role, params, gear_in, u_in, cost_out, status_out, x_out, st);
        HVP_CASE(2) HVP_CASE(3) HVP_CASE(4) HVP_CASE(5) HVP_CASE(6) HVP_CASE(7) HVP_CASE(8)
        HVP_CASE(9) HVP_CASE(10) HVP_CASE(11) HVP_CASE(12) HVP_CASE(13) HVP_CASE(14) HVP_CASE(15) HVP_CASE(16)
#undef HVP_CASE
        default: return fail(HVP_E_UNSUPPORTED, "hvp_evaluate_batch: unsupported N");
    }
}

int hvp_admm_update(hvp_handle* h, int P, int n, const double* x, const double* xf, const double* xb,
                    double* y_front, double* y_back, double* params, double* z_out, void* stream) {
    if (!h || P < 0 || n < 1 || (P > 0 && (!x || !xf || !xb || !y_front || !y_back || !params)))
        return fail(HVP_E_ARG, "hvp_admm_update: bad argument");
    if (h->prob.formulation != HVP_FORM_ADMM)
        return fail(HVP_E_ARG, "hvp_admm_update: the handle is not an HVP_FORM_ADMM problem");
    if (P == 0) return 0;
    HIP_TRY(hipSetDevice(h->device));
    const int N = h->prob.N;
    const long long total = (long long)P * n * 2 * (N + 1);
    hipLaunchKernelGGL(k_admm_update, dim3(grid_for(total)), dim3(kBlock), 0, (hipStream_t)stream, P, n, N,
                       h->prob.rho, h->C.stride, x, xf, xb, y_front, y_back, params, z_out);
    HIP_TRY(hipGetLastError());
    return 0;
}

// ---------------------------------------------------------------- switching ADMM
static int gadmm_check(hvp_handle* h, int P, int n, int lo, int m, const char* who) {
    if (!h) return fail(HVP_E_ARG, std::string(who) + ": null handle");
    if (h->prob.formulation != HVP_FORM_GADMM)
        return fail(HVP_E_ARG, std::string(who) + ": the handle is not an HVP_FORM_GADMM problem");
    if (P < 0 || n < 1 || m < 1 || lo < 0 || lo + m > n)
        return fail(HVP_E_ARG, std::string(who) + ": bad platoon layout (P, n, lo, m)");
    return 0;
}

int hvp_gadmm_rollout(hvp_handle* h, int P, int n, int lo, int m, const int32_t* sys, const double* params, int mode,
                      const double* u_prev, double* x, int8_t* seq, double* u_ws, int32_t* state, void* stream) {
    if (int rc = gadmm_check(h, P, n, lo, m, "hvp_gadmm_rollout")) return rc;
    if (P == 0) return 0;
    if (!sys || !params || !x || !seq || !state || (mode != 0 && mode != 1) || (mode == 1 && !u_prev))
        return fail(HVP_E_ARG, "hvp_gadmm_rollout: bad argument");
    HIP_TRY(hipSetDevice(h->device));
    HIP_TRY(hipMemsetAsync(h->g_counter, 0, 8 * sizeof(unsigned long long), (hipStream_t)stream));
    h->gadmm_hs_valid = 0;  // a new warm start: the local QPs start from their own hinge guess
    switch (h->prob.N) {
#define HVP_CASE(nn) \
    case nn: return launch_gadmm_rollout<nn>(h, P, n, lo, m, sys, params, mode, u_prev, x, seq, u_ws, state, (hipStream_t)stream);
        HVP_CASE(2) HVP_CASE(3) HVP_CASE(4) HVP_CASE(5) HVP_CASE(6) HVP_CASE(7) HVP_CASE(8)
        HVP_CASE(9) HVP_CASE(10) HVP_CASE(11) HVP_CASE(12) HVP_CASE(13) HVP_CASE(14) HVP_CASE(15) HVP_CASE(16)
#undef HVP_CASE
        default: return fail(HVP_E_UNSUPPORTED, "hvp_gadmm_rollout: unsupported N");
    }
}

}  // extern "C"

extern "C" {

int hvp_gadmm_solve(hvp_handle* h, int P, int n, int lo, int m, const int32_t* sys, const int32_t* role,
                    const double* params, const int8_t* seq, int32_t* state, double* u_out, double* x, double* xf,
                    double* xb, double* cost_out, int32_t* status_out, uint32_t* edge_out, int32_t* iters_out,
                    void* stream) {
    if (int rc = gadmm_check(h, P, n, lo, m, "hvp_gadmm_solve")) return rc;
    if (P == 0) return 0;
    if (!sys || !role || !params || !seq || !state || !u_out || !x || !xf || !xb || !cost_out || !status_out ||
        !edge_out)
        return fail(HVP_E_ARG, "hvp_gadmm_solve: bad argument");
    HIP_TRY(hipSetDevice(h->device));
    hipStream_t st = (hipStream_t)stream;
    switch (h->prob.N) {
#define HVP_CASE(nn) \
    case nn: return launch_gadmm_qp<nn>(h, P, n, lo, m, sys, role, params, seq, state, u_out, x, xf, xb, cost_out, status_out, edge_out, iters_out, st);
        HVP_CASE(2) HVP_CASE(3) HVP_CASE(4) HVP_CASE(5) HVP_CASE(6) HVP_CASE(7) HVP_CASE(8)
        HVP_CASE(9) HVP_CASE(10) HVP_CASE(11) HVP_CASE(12) HVP_CASE(13) HVP_CASE(14) HVP_CASE(15) HVP_CASE(16)
#undef HVP_CASE
        default: return fail(HVP_E_UNSUPPORTED, "hvp_gadmm_solve: unsupported N");
    }
}

int hvp_gadmm_update(hvp_handle* h, int P, int n, int lo, int m, const double* x, const double* xf, const double* xb,
                     double* params, const int32_t* state, int init, void* stream) {
    if (int rc = gadmm_check(h, P, n, lo, m, "hvp_gadmm_update")) return rc;
    if (P == 0) return 0;
    if (!x || !xf || !xb || !params || !state) return fail(HVP_E_ARG, "hvp_gadmm_update: bad argument");
    HIP_TRY(hipSetDevice(h->device));
    const int N = h->prob.N;
    const long long total = (long long)P * m * 2 * (N + 1);
    hipLaunchKernelGGL(k_gadmm_update, dim3(grid_for(total)), dim3(kBlock), 0, (hipStream_t)stream, P, n, lo, m, N,
                       h->prob.rho, h->C.stride, x, xf, xb, params, state, init);
    HIP_TRY(hipGetLastError());
    return 0;
}

int hvp_gadmm_switch(hvp_handle* h, int P, int n, int lo, int m, const int32_t* sys, const uint32_t* edge,
                     int8_t* seq, int32_t* state, void* stream) {
    if (int rc = gadmm_check(h, P, n, lo, m, "hvp_gadmm_switch")) return rc;
    if (P == 0) return 0;
    if (!sys || !edge || !seq || !state) return fail(HVP_E_ARG, "hvp_gadmm_switch: bad argument");
    HIP_TRY(hipSetDevice(h->device));
    hipLaunchKernelGGL(k_gadmm_switch, dim3(grid_for((long long)P * m)), dim3(kBlock), 0, (hipStream_t)stream, P, n,
                       lo, m, h->prob.N, h->d_sys, sys, edge, seq, state);
    HIP_TRY(hipGetLastError());
    return 0;
}

int hvp_sync(hvp_handle* h, void* stream) {
    if (!h) return fail(HVP_E_ARG, "hvp_sync: null handle");
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    return 0;
}

int hvp_get_stats(hvp_handle* h, hvp_stats* out) {
    if (!h || !out) return fail(HVP_E_ARG, "hvp_get_stats: bad argument");
    HIP_TRY(hipStreamSynchronize(h->last_stream));
    unsigned long long c[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (h->prob.formulation == HVP_FORM_GADMM || h->prob.formulation == HVP_FORM_CENT) {
        // GADMM: cumulative since the last hvp_gadmm_rollout (one g_admm_control warm start);
        // CENT: QPs ([0]) and active-set iterations ([1]) of the last hvp_cent_solve_batch
        HIP_TRY(hipMemcpy(c, h->g_counter, sizeof(c), hipMemcpyDeviceToHost));
    } else if (h->ws.counter) {
        HIP_TRY(hipMemcpy(c, h->ws.counter, sizeof(c), hipMemcpyDeviceToHost));
    }
    float ms = 0.f, qms = 0.f;
    if (h->last_B > 0) {
        HIP_TRY(hipEventElapsedTime(&ms, h->ev0, h->ev1));
        HIP_TRY(hipEventElapsedTime(&qms, h->evq0, h->evq1));
    }
    out->qp_ms = qms;
    out->n_instances = h->last_B;
    out->n_candidates = (int64_t)c[0];
    out->n_failed_bounds = (int64_t)c[4];
    if (h->last_bnb) {
        // tree nodes solved: root + dive QPs (counter[3]) and every level's nodes
        // (the decentralised lane path keeps each level in `last_split` segments of the capacity;
        // bucket b > 0 counts at (1 + b)(HVP_MAX_N + 1), hvp_lane.h LevelList)
        constexpr int M = HVP_MAX_N + 1;
        unsigned long long lv[6 * M];
        HIP_TRY(hipMemcpy(lv, h->ws.lvl, sizeof(lv), hipMemcpyDeviceToHost));
        int64_t n = (int64_t)c[3];
        const unsigned long long cap = (unsigned long long)h->ws.cap;
        const int nb = std::max(1, h->last_split);
        const unsigned long long seg = cap >> (nb == 4 ? 2 : (nb == 2 ? 1 : 0));
        for (int k = 1; k <= h->prob.N; ++k)
            for (int b = 0; b < nb; ++b)
                n += (int64_t)std::min(b == 0 ? lv[k] : lv[(1 + b) * M + k], b + 1 < nb ? seg : cap - (nb - 1) * seg);
        // less the pass-through nodes (counter[6]): listed, but their parent's QP is theirs
        // (hvp_lane.h bnb_put_children kPassFlag)
        out->n_candidates = n - (int64_t)c[6];
        // QP time = K_bnb_root + every K_bnb_bound launch (the expand / select kernels excluded)
        float sum = 0.f;
        for (int k = 0; k <= h->prob.N; ++k) {
            float t = 0.f;
            HIP_TRY(hipEventElapsedTime(&t, h->evb[2 * k], h->evb[2 * k + 1]));
            sum += t;
        }
        out->qp_ms = sum;
    }
    out->qp_iterations = (int64_t)c[1];
    out->n_fallback = (int64_t)c[2];
    const bool own_counter = h->prob.formulation != HVP_FORM_GADMM && h->prob.formulation != HVP_FORM_CENT;
    out->n_spilled = own_counter ? (int64_t)c[5] : 0;  // ws.counter[5], hvp_lane.h bnb_put_children
#ifdef HVP_REFILL_PROF
    {
        unsigned long long lv2[2 * (HVP_MAX_N + 1)];
        HIP_TRY(hipMemcpy(lv2, h->ws.lvl, sizeof(lv2), hipMemcpyDeviceToHost));
        const unsigned long long* pf = lv2 + 2 * (HVP_MAX_N + 1) - 8;
        std::fprintf(stderr,
                     "[refill-prof] event cycles %llu of %llu (%.3f), wave trips %llu, busy lane-trips %llu (%.3f); "
                     "write-back %llu (until cost %llu, until children %llu), claim %llu\n",
                     pf[0], pf[1], pf[1] ? (double)pf[0] / (double)pf[1] : 0.0, pf[3], pf[2],
                     pf[3] ? (double)pf[2] / (64.0 * (double)pf[3]) : 0.0, pf[4], pf[6], pf[7], pf[5]);
    }
#endif
    out->capacity = h->ws.cap;
    out->last_ms = ms;
    return 0;
}

int hvp_solve_batch_host(hvp_handle* h, int B, const int32_t* sys, const int32_t* role, const double* params,
                         double* u_out, double* x_out, int8_t* region_out, int8_t* gear_out, double* cost_out,
                         int32_t* status_out, int32_t* nodes_out, int32_t* iters_out) {
    if (!h || B < 0) return fail(HVP_E_ARG, "hvp_solve_batch_host: bad argument");
    if (B == 0) return 0;
    const int N = h->prob.N;
    const size_t P = (size_t)h->C.stride;
    // staging layout (8-byte aligned pieces)
    const size_t s_sys = sizeof(int32_t) * B, s_role = s_sys, s_prm = sizeof(double) * P * B;
    const size_t s_u = sizeof(double) * N * B, s_x = sizeof(double) * 2 * (N + 1) * B;
    const size_t s_reg = (size_t)N * B, s_gear = s_reg, s_cost = sizeof(double) * B, s_i32 = sizeof(int32_t) * B;
    auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
    const size_t total = al(s_sys) + al(s_role) + al(s_prm) + al(s_u) + al(s_x) + al(s_reg) + al(s_gear) + al(s_cost) +
                         3 * al(s_i32);
    HIP_TRY(hipSetDevice(h->device));
    if (total > h->stage_bytes) {
        if (h->d_stage) (void)hipFree(h->d_stage);
        h->d_stage = nullptr;
        h->stage_bytes = 0;
        HIP_TRY(hipMalloc(&h->d_stage, total));
        h->stage_bytes = total;
    }
    char* p = h->d_stage;
    auto take = [&](size_t n) { char* r = p; p += al(n); return r; };
    int32_t* d_sys = (int32_t*)take(s_sys);
    int32_t* d_role = (int32_t*)take(s_role);
    double* d_prm = (double*)take(s_prm);
    double* d_u = (double*)take(s_u);
    double* d_x = (double*)take(s_x);
    int8_t* d_reg = (int8_t*)take(s_reg);
    int8_t* d_gear = (int8_t*)take(s_gear);
    double* d_cost = (double*)take(s_cost);
    int32_t* d_stat = (int32_t*)take(s_i32);
    int32_t* d_nodes = (int32_t*)take(s_i32);
    int32_t* d_iters = (int32_t*)take(s_i32);
    HIP_TRY(hipMemcpy(d_sys, sys, s_sys, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(d_role, role, s_role, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(d_prm, params, s_prm, hipMemcpyHostToDevice));
    int rc = hvp_solve_batch(h, B, d_sys, d_role, d_prm, d_u, d_x, d_reg, d_gear, d_cost, d_stat, d_nodes, d_iters,
                             nullptr);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(nullptr));
    if (u_out) HIP_TRY(hipMemcpy(u_out, d_u, s_u, hipMemcpyDeviceToHost));
    if (x_out) HIP_TRY(hipMemcpy(x_out, d_x, s_x, hipMemcpyDeviceToHost));
    if (region_out) HIP_TRY(hipMemcpy(region_out, d_reg, s_reg, hipMemcpyDeviceToHost));
    if (gear_out) HIP_TRY(hipMemcpy(gear_out, d_gear, s_gear, hipMemcpyDeviceToHost));
    if (cost_out) HIP_TRY(hipMemcpy(cost_out, d_cost, s_cost, hipMemcpyDeviceToHost));
    if (status_out) HIP_TRY(hipMemcpy(status_out, d_stat, s_i32, hipMemcpyDeviceToHost));
    if (nodes_out) HIP_TRY(hipMemcpy(nodes_out, d_nodes, s_i32, hipMemcpyDeviceToHost));
    if (iters_out) HIP_TRY(hipMemcpy(iters_out, d_iters, s_i32, hipMemcpyDeviceToHost));
    return 0;
}

void hvp_destroy(hvp_handle* h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    (void)hipDeviceSynchronize();
    free_ws(h->ws);
    if (h->d_sys) (void)hipFree(h->d_sys);
    if (h->d_stage) (void)hipFree(h->d_stage);
    if (h->g_counter) (void)hipFree(h->g_counter);
    if (h->cent_frames) (void)hipFree(h->cent_frames);
    if (h->cent_ties) (void)hipFree(h->cent_ties);
    if (h->cent_split) (void)hipFree(h->cent_split);
    if (h->gadmm_hs) (void)hipFree(h->gadmm_hs);
    if (h->nrec) (void)hipFree(h->nrec);
    if (h->nclaim) (void)hipFree(h->nclaim);
    if (h->d_consts) (void)hipFree(h->d_consts);
    if (h->d_ws) (void)hipFree(h->d_ws);
    if (h->gadmm_redo) (void)hipFree(h->gadmm_redo);
    if (h->ev0) (void)hipEventDestroy(h->ev0);
    if (h->ev1) (void)hipEventDestroy(h->ev1);
    if (h->evq0) (void)hipEventDestroy(h->evq0);
    if (h->evq1) (void)hipEventDestroy(h->evq1);
    for (hipEvent_t& e : h->evb)
        if (e) (void)hipEventDestroy(e);
    delete h;
}

}  // extern "C"
