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
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>

#define HVP_HD __host__ __device__
#include "hvp.h"
#include "hvp_internal.h"
#include "hvp_admm.h"
#include "hvp_bnb.h"
#include "hvp_coop.h"
#include "hvp_gi.h"
#include "hvp_ipm.h"

namespace hvp_detail {
thread_local std::string g_err;
int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}
}  // namespace hvp_detail

namespace {

using hvp_detail::fail;
using hvp_detail::Workspace;




constexpr int kBlock = 256;
// HVP_METHOD_AUTO: exhaustive enumeration up to this horizon, branch and bound beyond
constexpr int kAutoEnumMaxN = 0;  // measured: B&B beats enumeration already at N = 5 (profiles/)
// active-set iteration cap (then the interior-point fallback takes the candidate)
template <int N>
constexpr int kGiMaxIter = 8 * hvp::GiConstraintSet<N>::NC;

}  // namespace

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
    C.max_iter = p.max_iter > 0 ? p.max_iter : 60;
    C.N = p.N;
    C.form = p.formulation;
    C.stride = p.formulation == HVP_FORM_ADMM    ? hvp_params_stride_admm(p.N)
               : p.formulation == HVP_FORM_GADMM ? hvp_params_stride_gadmm(p.N)
                                                 : hvp_params_stride(p.N);
    C.rho = p.rho;
    return C;
}

// ------------------------------------------------------------------ K_enum
template <int N>
__global__ __launch_bounds__(kBlock) void k_enum(int B, const hvp_system* __restrict__ systems,
                                                 const int32_t* __restrict__ sys, const int32_t* __restrict__ role,
                                                 const double* __restrict__ params, hvp::Consts C, Workspace ws) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B) return;
    const hvp_system& S = systems[sys[i]];
    const double* prm = params + (size_t)i * (2 + 6 * (N + 1));
    const double p0 = prm[0], v0 = prm[1];
    const double P1 = p0 + S.ts * v0;
    // sigma-independent constant row: p_1 = p_0 + ts v_0 inside the position box
    const bool ok = P1 >= S.pmin - 1e-9 * (1.0 + fabs(S.pmin)) && P1 <= S.pmax + 1e-9 * (1.0 + fabs(S.pmax));
    int cnt = 0;
    if (ok) cnt = hvp::enumerate_sequences(S, C, v0, [](uint32_t, int) {});
    ws.inst_cnt[i] = cnt;
    ws.inst_flag[i] = ok ? 0 : 1;
    int off = -1;
    if (cnt > 0) {
        const unsigned long long o = atomicAdd(&ws.counter[0], (unsigned long long)cnt);
        if ((long long)o + cnt <= ws.cap) {
            off = (int)o;
        } else {
            // overflow: the part of the reserved range below the capacity is still swept by
            // K_qp / K_cost (they run over min(reserved, cap)): mark those slots dead
            for (long long t = (long long)o; t < ws.cap && t < (long long)o + cnt; ++t) ws.task_inst[t] = -1;
        }
    }
    ws.inst_off[i] = off;
    if (off < 0) return;
    hvp::enumerate_sequences(S, C, v0, [&](uint32_t code, int j) {
        ws.task_inst[off + j] = i;
        ws.task_code[off + j] = code;
    });
    (void)role;
}

// ------------------------------------------------------------------ K_qp
// Per-lane constant rows in LDS: field f, step j of lane l at s_rows[(f * N + j) * kBlock + l]
// (consecutive lanes -> consecutive 8-byte words: conflict-free ds_read_b64).  refresh() makes
// the lane offset opaque at the start of every IPM sweep so the compiler re-reads the rows from
// LDS instead of hoisting them into VGPRs for the whole solve.
extern __shared__ double s_rows[];

template <int N, int BS = kBlock>
struct LdsMem {
    unsigned lane;
    __device__ double get(int f, int j) const { return s_rows[(f * N + j) * BS + lane]; }
    __device__ void set(int f, int j, double x) { s_rows[(f * N + j) * BS + lane] = x; }
    __device__ void refresh() { asm volatile("" : "+v"(lane)); }
};

// K_qp: every candidate by the Goldfarb-Idnani active-set method (hvp_gi.h).  A lane whose
// result fails the KKT verification (or hits the iteration cap) is queued on the fallback list.
template <int N>
__global__ __launch_bounds__(kBlock) void k_qp_gi(const hvp_system* __restrict__ systems,
                                                  const int32_t* __restrict__ sys, const int32_t* __restrict__ role,
                                                  const double* __restrict__ params, hvp::Consts C, Workspace ws) {
    const unsigned long long reserved = ws.counter[0];
    const long long total = (long long)(reserved < (unsigned long long)ws.cap ? reserved : ws.cap);
    unsigned long long iter_sum = 0;
    for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (long long)gridDim.x * blockDim.x) {
        const int inst = ws.task_inst[t];
        if (inst < 0) continue;  // dead slot of an overflowed instance
        const uint32_t code = ws.task_code[t];
        const hvp_system& S = systems[sys[inst]];
        const int rl = role[inst];
        const double* prm = params + (size_t)inst * (2 + 6 * (N + 1));
        hvp::LaneQp<N, LdsMem<N>> q;
        q.mem.lane = threadIdx.x;
        hvp::setup_lane<N>(q, S, C, rl, prm, code);
        int iters = 0;
        int status = hvp::solve_gi<N>(q, C, kGiMaxIter<N>, iters);
        if (status != hvp::GI_OK) {
            const unsigned long long r = atomicAdd(&ws.counter[2], 1ull);
            ws.redo[r] = (int32_t)t;
            status = 4;  // pending: the fallback kernel overwrites it
        }
        ws.task_stat[t] = status | (iters << 8);
#pragma unroll
        for (int k = 0; k < N; ++k) ws.task_y[t * N + k] = q.y[k];
        iter_sum += (unsigned long long)iters;
    }
    // one atomic per wave for the iteration statistics
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) iter_sum += __shfl_down(iter_sum, off, 64);
    if ((threadIdx.x & 63) == 0 && iter_sum) atomicAdd(&ws.counter[1], iter_sum);
}

// K_qp_ipm: the fallback list only (normally empty: the launch reads a zero count and exits),
// full row set by the Mehrotra interior-point method (hvp_ipm.h).
template <int N>
__global__ __launch_bounds__(kBlock) void k_qp_ipm(const hvp_system* __restrict__ systems,
                                                   const int32_t* __restrict__ sys, const int32_t* __restrict__ role,
                                                   const double* __restrict__ params, hvp::Consts C, Workspace ws) {
    const unsigned long long reserved = ws.counter[2];
    const long long total = (long long)(reserved < (unsigned long long)ws.cap ? reserved : ws.cap);
    unsigned long long iter_sum = 0;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const long long t = (long long)ws.redo[i];
        const int inst = ws.task_inst[t];
        const uint32_t code = ws.task_code[t];
        const hvp_system& S = systems[sys[inst]];
        const int rl = role[inst];
        const double* prm = params + (size_t)inst * (2 + 6 * (N + 1));
        hvp::LaneQp<N, LdsMem<N>> q;
        q.mem.lane = threadIdx.x;
        hvp::setup_lane<N>(q, S, C, rl, prm, code);
        const hvp::QpOut o = hvp::Solver<N, true, LdsMem<N>>::solve(q, C);
        ws.task_stat[t] = o.status | ((o.iters + (ws.task_stat[t] >> 8)) << 8);
#pragma unroll
        for (int k = 0; k < N; ++k) ws.task_y[t * N + k] = q.y[k];
        iter_sum += (unsigned long long)o.iters;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) iter_sum += __shfl_down(iter_sum, off, 64);
    if ((threadIdx.x & 63) == 0 && iter_sum) atomicAdd(&ws.counter[1], iter_sum);
}

// ------------------------------------------------------------------ K_cost
// Objective of every converged candidate, evaluated term by term on its trajectory (separate
// launch: fused into K_qp its reference loads stay live across the IPM and spill).
template <int N>
__global__ __launch_bounds__(kBlock) void k_cost(const hvp_system* __restrict__ systems,
                                                 const int32_t* __restrict__ sys, const int32_t* __restrict__ role,
                                                 const double* __restrict__ params, hvp::Consts C, Workspace ws) {
    const unsigned long long reserved = ws.counter[0];
    const long long total = (long long)(reserved < (unsigned long long)ws.cap ? reserved : ws.cap);
    for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (long long)gridDim.x * blockDim.x) {
        const int inst = ws.task_inst[t];
        double cost = 1e300;
        if (inst >= 0 && (ws.task_stat[t] & 0xff) == 0) {
            const hvp_system& S = systems[sys[inst]];
            const double* prm = params + (size_t)inst * (2 + 6 * (N + 1));
            hvp::LaneQp<N> q;
            const int rl = role[inst];
            q.has_sf = (rl & HVP_ROLE_SAFE_FRONT) != 0;
            q.has_sb = (rl & HVP_ROLE_SAFE_BACK) != 0;
#pragma unroll
            for (int k = 0; k < N; ++k) q.y[k] = ws.task_y[t * N + k];
            cost = hvp::direct_cost<N>(q, S, C, rl, prm, ws.task_code[t]);
        }
        ws.task_cost[t] = cost;
    }
}

// ------------------------------------------------------------------ K_select
template <int N>
__global__ __launch_bounds__(kBlock) void k_select(int B, const hvp_system* __restrict__ systems,
                                                   const int32_t* __restrict__ sys, const double* __restrict__ params,
                                                   Workspace ws, double* __restrict__ u_out, double* __restrict__ x_out,
                                                   int8_t* __restrict__ region_out, int8_t* __restrict__ gear_out,
                                                   double* __restrict__ cost_out, int32_t* __restrict__ status_out,
                                                   int32_t* __restrict__ nodes_out, int32_t* __restrict__ iters_out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B) return;
    const int cnt = ws.inst_cnt[i], off = ws.inst_off[i];
    const hvp_system& S = systems[sys[i]];
    const double* prm = params + (size_t)i * (2 + 6 * (N + 1));
    int status;
    int win = -1;
    int iters = 0;
    if (ws.inst_flag[i] != 0 || cnt == 0) {
        status = HVP_INFEASIBLE;
    } else if (off < 0) {
        status = HVP_OVERFLOW;
    } else {
        double best = 1e300;
        for (int j = 0; j < cnt; ++j) {
            const int st = ws.task_stat[off + j];
            iters += st >> 8;
            if ((st & 0xff) == 0) best = fmin(best, ws.task_cost[off + j]);
        }
        if (best < 1e300) {
            const double tol = 1e-9 * fmax(1.0, fabs(best));
            for (int j = 0; j < cnt; ++j)
                if ((ws.task_stat[off + j] & 0xff) == 0 && ws.task_cost[off + j] <= best + tol) {
                    win = off + j;
                    break;
                }
        }
        status = win >= 0 ? HVP_OPTIMAL : HVP_MAXITER;
    }
    if (status_out) status_out[i] = status;
    if (nodes_out) nodes_out[i] = cnt;
    if (iters_out) iters_out[i] = iters;
    if (cost_out) cost_out[i] = win >= 0 ? ws.task_cost[win] : 1e300;
    const uint32_t code = win >= 0 ? ws.task_code[win] : 0u;
    double p = prm[0], v = prm[1];
    if (x_out) {
        x_out[(size_t)i * 2 * (N + 1)] = p;
        x_out[(size_t)i * 2 * (N + 1) + N + 1] = v;
    }
#pragma unroll
    for (int k = 0; k < N; ++k) {
        const int r = hvp::code_region(code, k);
        const double vn = win >= 0 ? ws.task_y[(size_t)win * N + k] : v;
        const double u = win >= 0 ? (vn - S.a[r] * v - S.c[r]) / S.b[r] : 0.0;
        p = p + S.ts * v;
        v = vn;
        if (u_out) u_out[(size_t)i * N + k] = u;
        if (x_out) {
            x_out[(size_t)i * 2 * (N + 1) + k + 1] = p;
            x_out[(size_t)i * 2 * (N + 1) + N + 1 + k + 1] = v;
        }
        if (region_out) region_out[(size_t)i * N + k] = (int8_t)(win >= 0 ? r : -1);
        if (gear_out) gear_out[(size_t)i * N + k] = (int8_t)(win >= 0 ? S.gear[r] : 0);
    }
}

// ================================================================== branch and bound
// Level-synchronous over the whole batch (hvp_bnb.h): K_root (relaxed root QP + greedy dive ->
// incumbent), then for every depth k = 1..N  K_expand (children of the unpruned parents, one
// atomicAdd per parent) and K_bound (one lane per child: QP with the tail relaxed after k steps;
// exact QP at k = N), then K_key / K_write / K_finish (argmin + tie rule over the leaves).
// Every kernel grid-strides over a count that lives on the device: no host round trip.
template <int N>
constexpr int kBnbBlock = N <= 8 ? 256 : 64;  // LDS rows: 7 N doubles per lane

// The incumbent is kept as an order-preserving 64-bit key of the double so that atomicMin on the
// key is a min on the cost -- for negative costs too (the ADMM objective carries y'(c - z)).
__device__ inline unsigned long long cost_key(double c) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(c);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ inline double key_cost(unsigned long long k) {
    return __longlong_as_double((long long)((k >> 63) ? (k & 0x7fffffffffffffffull) : ~k));
}
__device__ inline double inc_of(const Workspace& ws, int inst) { return key_cost(ws.inc[inst]); }

// Occupancy target of the lane B&B kernels (waves per SIMD).  Measured at C2: 2 waves/SIMD forces
// 800 B/lane of spills and runs 2.7x slower than 1 wave/SIMD with the register file to itself
#ifndef HVP_LANE_WAVES
#define HVP_LANE_WAVES 1
#endif
#define HVP_LANE_OCC __attribute__((amdgpu_waves_per_eu(HVP_LANE_WAVES)))

// ADMM: the formulation is a template parameter so that each kernel instantiation holds ONE
// QP path (both paths in one kernel pushed the lane kernels to 256 VGPRs + scratch spills)
template <int N, int BS, bool ADMM>
__device__ inline int bnb_qp(hvp::LaneQp<N, LdsMem<N, BS>>& q, const hvp_system& S, const hvp::Consts& C, int rl,
                             const double* prm, uint64_t code, int K, double lo, double hi, double& cost) {
    int it = 0, st;
    if constexpr (ADMM) {
        st = hvp::solve_admm_lane<N>(q, S, C, rl, prm, code, K, kGiMaxIter<N>, it);
        cost = st == hvp::GI_OK ? hvp::admm_direct_cost<N>(q, S, C, rl, prm, code, K) : 0.0;
    } else {
        hvp::setup_lane<N>(q, S, C, rl, prm, code, K, lo, hi);  // tail relaxed from v_K in [lo, hi]
        st = hvp::solve_gi<N>(q, C, kGiMaxIter<N>, it);
        cost = st == hvp::GI_OK ? hvp::direct_cost<N>(q, S, C, rl, prm, code, K) : 0.0;
    }
    return st == hvp::GI_OK ? it : -1 - it;
}

template <int N, bool ADMM>
__global__ __launch_bounds__(kBnbBlock<N>) HVP_LANE_OCC void k_bnb_root(int B, const hvp_system* __restrict__ systems,
                                                           const int32_t* __restrict__ sys,
                                                           const int32_t* __restrict__ role,
                                                           const double* __restrict__ params, hvp::Consts C,
                                                           Workspace ws) {
    constexpr int BS = kBnbBlock<N>;
    const int i = blockIdx.x * BS + threadIdx.x;
    if (i == 0) ws.lvl[0] = (unsigned long long)B;
    if (i >= B) return;
    const hvp_system& S = systems[sys[i]];
    const int rl = role[i];
    const double* prm = params + (size_t)i * C.stride;
    const double v0 = prm[1], P1 = prm[0] + S.ts * v0;
    const bool ok = P1 >= S.pmin - 1e-9 * (1.0 + fabs(S.pmin)) && P1 <= S.pmax + 1e-9 * (1.0 + fabs(S.pmax));
    ws.key[i] = ~0ull;
    ws.inst_flag[i] = ok ? 0 : 1;
    ws.nd_inst[0][i] = ok ? i : -1;
    ws.nd_code[0][i] = 0;
    ws.nd_lo[0][i] = v0;
    ws.nd_hi[0][i] = v0;
    double inc = __longlong_as_double(0x7ff0000000000000ll);  // +inf: no incumbent
    double lb = -1e300;
    int nodes = 0, iters = 0;
    if (ok) {
        hvp::LaneQp<N, LdsMem<N, BS>> q;
        q.mem.lane = threadIdx.x;
        double c0;
        int it = bnb_qp<N, BS, ADMM>(q, S, C, rl, prm, 0, 0, v0, v0, c0);
        ++nodes;
        iters += it >= 0 ? it : -1 - it;
        if (it >= 0) {
            lb = c0;
            double ystar[N];
#pragma unroll
            for (int k = 0; k < N; ++k) ystar[k] = q.y[k];
            uint64_t code;
            if (hvp::bnb_dive<N>(S, C, v0, ystar, &code)) {
                double c1;
                it = bnb_qp<N, BS, ADMM>(q, S, C, rl, prm, code, N, 0.0, -1.0, c1);
                ++nodes;
                iters += it >= 0 ? it : -1 - it;
                if (it >= 0) inc = c1;
            }
        }
    }
    ws.nd_lb[0][i] = lb;
    ws.inc[i] = cost_key(inc);
    ws.nodes[i] = nodes;
    ws.iters[i] = iters;
    atomicAdd(&ws.counter[3], (unsigned long long)nodes);
    atomicAdd(&ws.counter[1], (unsigned long long)iters);
}

// ---- long horizons: one QP per 16-lane group (hvp_coop.h), 4 groups per 64-lane block
template <int N>
constexpr bool kCoop = N > HVP_MAX_N_ENUM;
constexpr int kCoopBlock = 64;
constexpr int kCoopGroups = kCoopBlock / hvp::coop::G;

template <int N>
__global__ __launch_bounds__(kCoopBlock) void k_bnb_root_coop(int B, const hvp_system* __restrict__ systems,
                                                              const int32_t* __restrict__ sys,
                                                              const int32_t* __restrict__ role,
                                                              const double* __restrict__ params, hvp::Consts C,
                                                              Workspace ws) {
    __shared__ hvp::coop::GroupLds lds[kCoopGroups];
    const int g = threadIdx.x / hvp::coop::G, t = threadIdx.x % hvp::coop::G;
    const int i = blockIdx.x * kCoopGroups + g;
    if (blockIdx.x == 0 && threadIdx.x == 0) ws.lvl[0] = (unsigned long long)B;
    if (i >= B) return;  // group-uniform
    const hvp_system& S = systems[sys[i]];
    const int rl = role[i];
    const double* prm = params + (size_t)i * C.stride;
    const double v0 = prm[1], P1 = prm[0] + S.ts * v0;
    const bool ok = P1 >= S.pmin - 1e-9 * (1.0 + fabs(S.pmin)) && P1 <= S.pmax + 1e-9 * (1.0 + fabs(S.pmax));
    double inc = __longlong_as_double(0x7ff0000000000000ll);
    double lb = -1e300;
    int nodes = 0, iters = 0;
    if (ok) {
        hvp::coop::Lane<N> L;
        double c0 = 0.0;
        int it = 0;
        int st = hvp::coop::solve_qp<N>(L, lds[g], S, C, rl, prm, 0, 0, kGiMaxIter<N>, it, &c0, nullptr, prm[1], prm[1]);
        ++nodes;
        iters += it;
        if (st == hvp::GI_OK) {
            lb = c0;
            lds[g].v[t] = t < N ? L.y : 0.0;
            hvp::coop::gsync();
            unsigned long long code = 0;
            int dive_ok = 0;
            if (t == 0) {
                double ystar[N];
#pragma unroll
                for (int k = 0; k < N; ++k) ystar[k] = lds[g].v[k];
                uint64_t c64;
                dive_ok = hvp::bnb_dive<N>(S, C, v0, ystar, &c64) ? 1 : 0;
                code = c64;
            }
            dive_ok = hvp::coop::bcast(dive_ok, 0);
            code = hvp::coop::bcast(code, 0);
            if (dive_ok) {
                double c1 = 0.0;
                st = hvp::coop::solve_qp<N>(L, lds[g], S, C, rl, prm, code, N, kGiMaxIter<N>, it, &c1);
                ++nodes;
                iters += it;
                if (st == hvp::GI_OK) inc = c1;
            }
        }
    }
    if (t == 0) {
        ws.key[i] = ~0ull;
        ws.inst_flag[i] = ok ? 0 : 1;
        ws.nd_inst[0][i] = ok ? i : -1;
        ws.nd_code[0][i] = 0;
        ws.nd_lo[0][i] = v0;
        ws.nd_hi[0][i] = v0;
        ws.nd_lb[0][i] = lb;
        ws.inc[i] = cost_key(inc);
        ws.nodes[i] = nodes;
        ws.iters[i] = iters;
        atomicAdd(&ws.counter[3], (unsigned long long)nodes);
        atomicAdd(&ws.counter[1], (unsigned long long)iters);
    }
}

template <int N>
__global__ __launch_bounds__(kCoopBlock) void k_bnb_bound_coop(int k, const hvp_system* __restrict__ systems,
                                                               const int32_t* __restrict__ sys,
                                                               const int32_t* __restrict__ role,
                                                               const double* __restrict__ params, hvp::Consts C,
                                                               Workspace ws) {
    __shared__ hvp::coop::GroupLds lds[kCoopGroups];
    const int g = threadIdx.x / hvp::coop::G, t = threadIdx.x % hvp::coop::G;
    const int dst = k & 1;
    const unsigned long long nn = ws.lvl[k];
    const long long total = (long long)(nn < (unsigned long long)ws.cap ? nn : ws.cap);
    for (long long q = (long long)blockIdx.x * kCoopGroups + g; q < total; q += (long long)gridDim.x * kCoopGroups) {
        const int inst = ws.nd_inst[dst][q];
        if (inst < 0) {
            if (t == 0) {
                if (k == N) ws.leaf_stat[q] = HVP_OVERFLOW;
                else ws.nd_lb[dst][q] = 1e300;
            }
            continue;
        }
        const uint64_t code = ws.nd_code[dst][q];
        const hvp_system& S = systems[sys[inst]];
        const int rl = role[inst];
        const double* prm = params + (size_t)inst * C.stride;
        hvp::coop::Lane<N> L;
        double c = 0.0;
        int it = 0;
        const int st = hvp::coop::solve_qp<N>(L, lds[g], S, C, rl, prm, code, k, kGiMaxIter<N>, it, &c, nullptr,
                                              ws.nd_lo[dst][q], ws.nd_hi[dst][q]);
        const bool ok = st == hvp::GI_OK;
        if (k == N && t < N) ws.task_y[q * N + t] = L.y;
        if (t == 0) {
            atomicAdd(&ws.nodes[inst], 1);
            atomicAdd(&ws.iters[inst], it);
            atomicAdd(&ws.counter[1], (unsigned long long)it);
            if (k < N) {
                ws.nd_lb[dst][q] = ok ? c : -1e300;
                if (!ok) atomicAdd(&ws.counter[4], 1ull);
            } else {
                if (ok) ws.nd_lb[dst][q] = c;
                ws.leaf_stat[q] = ok ? 0 : HVP_MAXITER;
                if (ok) atomicMin(&ws.inc[inst], cost_key(c));
                else atomicOr(&ws.inst_flag[inst], 8);
            }
        }
    }
}

// children of the level-(k-1) nodes that survive the incumbent test
// Every instance may hold at most `quota` = capacity / B nodes per level: an instance whose
// tree outgrows its share (the heavy tail at long horizons, e.g. trajectories riding a region
// boundary) is cut off deterministically and reported HVP_OVERFLOW, so it can never crowd the
// other instances out of the pooled list.  The host path re-solves it alone (quota = capacity).
template <int N>
__global__ __launch_bounds__(kBlock) void k_bnb_expand(int k, int quota, const hvp_system* __restrict__ systems,
                                                       const int32_t* __restrict__ sys, hvp::Consts C, Workspace ws) {
    const int src = (k - 1) & 1, dst = k & 1;
    const unsigned long long np = ws.lvl[k - 1];
    const long long total = (long long)(np < (unsigned long long)ws.cap ? np : ws.cap);
    for (long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x; p < total;
         p += (long long)gridDim.x * blockDim.x) {
        const int inst = ws.nd_inst[src][p];
        if (inst < 0 || (ws.inst_flag[inst] & 2)) continue;
        const double plb = ws.nd_lb[src][p];
        if (hvp::bnb_pruned(plb, inc_of(ws, inst))) continue;
        const hvp_system& S = systems[sys[inst]];
        const double lo = ws.nd_lo[src][p], hi = ws.nd_hi[src][p];
        const uint64_t code = ws.nd_code[src][p];
        unsigned mask = 0;
        for (int r = 0; r < S.n_regions; ++r) {
            double a, b;
            if (hvp::bnb_child(S, C, k - 1, lo, hi, r, &a, &b)) mask |= 1u << r;
        }
        const int nc = __popc(mask);
        if (!nc) continue;
        if (atomicAdd(&ws.inst_lvl[inst], nc) + nc > quota) {
            atomicOr(&ws.inst_flag[inst], 2);
            continue;
        }
        const unsigned long long off = atomicAdd(&ws.lvl[k], (unsigned long long)nc);
        if (off + nc > (unsigned long long)ws.cap) {
            atomicOr(&ws.inst_flag[inst], 2);  // overflow: reported, never truncated silently
            // the slots of this reservation below the capacity are swept by the next kernels
            for (unsigned long long t = off; t < (unsigned long long)ws.cap && t < off + nc; ++t)
                ws.nd_inst[dst][t] = -1;
            continue;
        }
        int j = 0;
        for (int r = 0; r < S.n_regions; ++r) {
            if (!((mask >> r) & 1u)) continue;
            double a, b;
            hvp::bnb_child(S, C, k - 1, lo, hi, r, &a, &b);
            ws.nd_inst[dst][off + j] = inst;
            ws.nd_code[dst][off + j] = hvp::code_with(code, k - 1, r);
            ws.nd_lo[dst][off + j] = a;
            ws.nd_hi[dst][off + j] = b;
            ws.nd_lb[dst][off + j] = plb;  // inherited: kept by a leaf whose QP fails
            ++j;
        }
    }
}

// one lane per level-k node: bound (k < N) or exact leaf QP (k = N)
template <int N, bool ADMM>
__global__ __launch_bounds__(kBnbBlock<N>) HVP_LANE_OCC void k_bnb_bound(int k, const hvp_system* __restrict__ systems,
                                                            const int32_t* __restrict__ sys,
                                                            const int32_t* __restrict__ role,
                                                            const double* __restrict__ params, hvp::Consts C,
                                                            Workspace ws) {
    constexpr int BS = kBnbBlock<N>;
    const int dst = k & 1;
    const unsigned long long nn = ws.lvl[k];
    const long long total = (long long)(nn < (unsigned long long)ws.cap ? nn : ws.cap);
    unsigned long long iter_sum = 0, fails = 0;
    for (long long t = (long long)blockIdx.x * BS + threadIdx.x; t < total; t += (long long)gridDim.x * BS) {
        const int inst = ws.nd_inst[dst][t];
        if (inst < 0) {  // dead slot of an overflowed reservation
            if (k == N) ws.leaf_stat[t] = HVP_OVERFLOW;
            else ws.nd_lb[dst][t] = 1e300;
            continue;
        }
        const uint64_t code = ws.nd_code[dst][t];
        const hvp_system& S = systems[sys[inst]];
        const int rl = role[inst];
        const double* prm = params + (size_t)inst * C.stride;
        hvp::LaneQp<N, LdsMem<N, BS>> q;
        q.mem.lane = threadIdx.x;
        double c;
        const int it = bnb_qp<N, BS, ADMM>(q, S, C, rl, prm, code, k, ws.nd_lo[dst][t], ws.nd_hi[dst][t], c);
        const bool ok = it >= 0;
        const int its = ok ? it : -1 - it;
        iter_sum += (unsigned long long)its;
        atomicAdd(&ws.nodes[inst], 1);
        atomicAdd(&ws.iters[inst], its);
        if (k < N) {
            // a failed bound QP prunes nothing
            ws.nd_lb[dst][t] = ok ? c : -1e300;
            if (!ok) atomicAdd(&ws.counter[4], 1ull);
        } else {
            // a failed leaf keeps its parent's bound (K_key: MAXITER if it stays in contention
            // and no fallback exists)
            if (ok) ws.nd_lb[dst][t] = c;
            ws.leaf_stat[t] = ok ? 0 : HVP_MAXITER;
#pragma unroll
            for (int j = 0; j < N; ++j) ws.task_y[t * N + j] = q.y[j];
            if (ok) {
                atomicMin(&ws.inc[inst], cost_key(c));
            } else {
                ++fails;
                atomicOr(&ws.inst_flag[inst], 8);  // a velocity-feasible sequence exists
                if (N <= HVP_MAX_N_ENUM && C.form == HVP_FORM_DECENT) {  // K_bnb_ipm re-solves it
                    const unsigned long long r = atomicAdd(&ws.counter[2], 1ull);
                    if (r < (unsigned long long)ws.cap) ws.redo[r] = (int32_t)t;
                }
            }
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) iter_sum += __shfl_down(iter_sum, off, 64);
    if ((threadIdx.x & 63) == 0 && iter_sum) atomicAdd(&ws.counter[1], iter_sum);
    (void)fails;
}

// Leaves whose active-set solve failed its verification (degenerate vertices, e.g. the
// position box at p_max): re-solved by the interior-point method on the full row set
// (hvp_ipm.h), as K_qp_ipm does for the enumeration path.  Normally an empty list.
template <int N>
__global__ __launch_bounds__(kBnbBlock<N>) void k_bnb_ipm(const hvp_system* __restrict__ systems,
                                                          const int32_t* __restrict__ sys,
                                                          const int32_t* __restrict__ role,
                                                          const double* __restrict__ params, hvp::Consts C,
                                                          Workspace ws) {
    constexpr int BS = kBnbBlock<N>;
    const int src = N & 1;
    const unsigned long long nr = ws.counter[2];
    const long long total = (long long)(nr < (unsigned long long)ws.cap ? nr : ws.cap);
    for (long long i = (long long)blockIdx.x * BS + threadIdx.x; i < total; i += (long long)gridDim.x * BS) {
        const long long t = ws.redo[i];
        const int inst = ws.nd_inst[src][t];
        const uint64_t code = ws.nd_code[src][t];
        const hvp_system& S = systems[sys[inst]];
        const int rl = role[inst];
        const double* prm = params + (size_t)inst * C.stride;
        hvp::LaneQp<N, LdsMem<N, BS>> q;
        q.mem.lane = threadIdx.x;
        hvp::setup_lane<N>(q, S, C, rl, prm, code);
        const hvp::QpOut o = hvp::Solver<N, true, LdsMem<N, BS>>::solve(q, C);
        atomicAdd(&ws.iters[inst], o.iters);
        if (o.status != 0) continue;  // stays HVP_MAXITER with its parent's bound (K_key flags it)
        const double c = hvp::direct_cost<N>(q, S, C, rl, prm, code);
#pragma unroll
        for (int j = 0; j < N; ++j) ws.task_y[t * N + j] = q.y[j];
        ws.nd_lb[src][t] = c;
        ws.leaf_stat[t] = 0;
        atomicMin(&ws.inc[inst], cost_key(c));
    }
}

// tie rule: the lexicographically first leaf within 1e-9 relative of the minimum
template <int N>
__global__ __launch_bounds__(kBlock) void k_bnb_key(Workspace ws, int form) {
    const int src = N & 1;
    const unsigned long long nn = ws.lvl[N];
    const long long total = (long long)(nn < (unsigned long long)ws.cap ? nn : ws.cap);
    for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (long long)gridDim.x * blockDim.x) {
        const int inst = ws.nd_inst[src][t];
        if (inst < 0) continue;
        const double best = inc_of(ws, inst);
        if (ws.leaf_stat[t] != 0) {
            // Up to HVP_MAX_N_ENUM a leaf that fails the active-set method AND the interior-point
            // fallback is an infeasible QP (position box), excluded exactly as the enumeration
            // path and the oracle exclude it.  Beyond, there is no fallback: a failed leaf still
            // in contention makes the instance MAXITER rather than a possibly wrong answer.
            if ((N > HVP_MAX_N_ENUM || form != HVP_FORM_DECENT) && !hvp::bnb_pruned(ws.nd_lb[src][t], best))
                atomicOr(&ws.inst_flag[inst], 4);
            continue;
        }
        if (ws.nd_lb[src][t] <= best + 1e-9 * fmax(1.0, fabs(best)))
            atomicMin(&ws.key[inst], (unsigned long long)hvp::bnb_lexkey(ws.nd_code[src][t], N));
    }
}

template <int N>
__device__ inline void write_solution(int i, const hvp_system& S, const double* prm, bool win, uint64_t code,
                                      const double* y, double* u_out, double* x_out, int8_t* region_out,
                                      int8_t* gear_out) {
    double p = prm[0], v = prm[1];
    if (x_out) {
        x_out[(size_t)i * 2 * (N + 1)] = p;
        x_out[(size_t)i * 2 * (N + 1) + N + 1] = v;
    }
#pragma unroll
    for (int k = 0; k < N; ++k) {
        const int r = hvp::code_region(code, k);
        const double vn = win ? y[k] : v;
        const double u = win ? (vn - S.a[r] * v - S.c[r]) / S.b[r] : 0.0;
        p = p + S.ts * v;
        v = vn;
        if (u_out) u_out[(size_t)i * N + k] = u;
        if (x_out) {
            x_out[(size_t)i * 2 * (N + 1) + k + 1] = p;
            x_out[(size_t)i * 2 * (N + 1) + N + 1 + k + 1] = v;
        }
        if (region_out) region_out[(size_t)i * N + k] = (int8_t)(win ? r : -1);
        if (gear_out) gear_out[(size_t)i * N + k] = (int8_t)(win ? S.gear[r] : 0);
    }
}

// optimal neighbour copies of an ADMM solution (fleet_naive_admm.py: mpc.x_front.X / x_back.X)
template <int N>
__device__ inline void write_copies(int i, const hvp_system& S, const hvp::Consts& C, int rl, const double* prm,
                                    bool win, const double* y, double* xf_out, double* xb_out) {
    const bool side_on[2] = {(rl & HVP_ROLE_SAFE_FRONT) != 0, (rl & HVP_ROLE_SAFE_BACK) != 0};
    const bool track[2] = {(rl & HVP_ROLE_TRACK_FRONT) != 0, (rl & HVP_ROLE_TRACK_BACK) != 0};
    double* outs[2] = {xf_out, xb_out};
    const int K1 = N + 1;
    for (int side = 0; side < 2; ++side) {
        double* o = outs[side];
        if (!o) continue;
        o += (size_t)i * 2 * K1;
        double p = prm[0], v = prm[1];
        for (int k = 0; k <= N; ++k) {
            double e = 0.0, g = 0.0;
            if (win && side_on[side])
                hvp::admm_copy_value(C, track[side], side, hvp::admm_y(prm, side, N)[k],
                                     hvp::admm_y(prm, side, N)[K1 + k], hvp::admm_z(prm, side, N)[k],
                                     hvp::admm_z(prm, side, N)[K1 + k], p, v, &e, &g);
            o[k] = e;
            o[K1 + k] = g;
            if (k < N) {
                p = p + S.ts * v;
                v = win ? y[k] : v;
            }
        }
    }
}

template <int N>
__global__ __launch_bounds__(kBlock) void k_bnb_write(const hvp_system* __restrict__ systems,
                                                      const int32_t* __restrict__ sys,
                                                      const int32_t* __restrict__ role,
                                                      const double* __restrict__ params, hvp::Consts C, Workspace ws,
                                                      double* __restrict__ u_out, double* __restrict__ x_out,
                                                      int8_t* __restrict__ region_out, int8_t* __restrict__ gear_out,
                                                      double* __restrict__ cost_out, double* __restrict__ xf_out,
                                                      double* __restrict__ xb_out) {
    const int src = N & 1;
    const unsigned long long nn = ws.lvl[N];
    const long long total = (long long)(nn < (unsigned long long)ws.cap ? nn : ws.cap);
    for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (long long)gridDim.x * blockDim.x) {
        if (ws.leaf_stat[t] != 0) continue;
        const int inst = ws.nd_inst[src][t];
        if (inst < 0) continue;
        const uint64_t code = ws.nd_code[src][t];
        if (hvp::bnb_lexkey(code, N) != ws.key[inst]) continue;
        const hvp_system& S = systems[sys[inst]];
        double y[N];
#pragma unroll
        for (int j = 0; j < N; ++j) y[j] = ws.task_y[t * N + j];
        const double* prm = params + (size_t)inst * C.stride;
        write_solution<N>(inst, S, prm, true, code, y, u_out, x_out, region_out, gear_out);
        if (C.form == HVP_FORM_ADMM) write_copies<N>(inst, S, C, role[inst], prm, true, y, xf_out, xb_out);
        if (cost_out) cost_out[inst] = ws.nd_lb[src][t];
    }
}

template <int N>
__global__ __launch_bounds__(kBlock) void k_bnb_finish(int B, const hvp_system* __restrict__ systems,
                                                       const int32_t* __restrict__ sys,
                                                       const int32_t* __restrict__ role,
                                                       const double* __restrict__ params, hvp::Consts C, Workspace ws,
                                                       double* __restrict__ u_out, double* __restrict__ x_out,
                                                       int8_t* __restrict__ region_out, int8_t* __restrict__ gear_out,
                                                       double* __restrict__ cost_out, int32_t* __restrict__ status_out,
                                                       int32_t* __restrict__ nodes_out,
                                                       int32_t* __restrict__ iters_out,
                                                       double* __restrict__ xf_out, double* __restrict__ xb_out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B) return;
    const int flag = ws.inst_flag[i];
    const bool win = ws.key[i] != ~0ull;
    int status;
    if (flag & 1) status = HVP_INFEASIBLE;
    else if (flag & 2) status = HVP_OVERFLOW;
    else if (flag & 4) status = HVP_MAXITER;  // a leaf in contention whose QP did not converge
    else if (win) status = HVP_OPTIMAL;
    else status = (flag & 8) ? HVP_MAXITER : HVP_INFEASIBLE;  // sequences exist but no QP converged
    if (status_out) status_out[i] = status;
    if (nodes_out) nodes_out[i] = ws.nodes[i];
    if (iters_out) iters_out[i] = ws.iters[i];
    if (!win || status != HVP_OPTIMAL) {
        if (cost_out) cost_out[i] = 1e300;
        const double* prm = params + (size_t)i * C.stride;
        write_solution<N>(i, systems[sys[i]], prm, false, 0, nullptr, u_out, x_out, region_out, gear_out);
        if (C.form == HVP_FORM_ADMM) write_copies<N>(i, systems[sys[i]], C, role[i], prm, false, nullptr, xf_out, xb_out);
    }
}

// ================================================================== fixed-control evaluation
// MpcGear.evaluate_cost (mpcs/mpc_gear.py:137-170): with u (u_g for the gear model) and the
// gear of every step fixed, the MIQP has no free decision left but the slacks: the trajectory
// follows from the dynamics of the mode (gear label, region band containing v_k -- at a shared
// band edge the PWA dynamics coincide), the slacks take max(0, .), and the objective is the
// direct cost of that trajectory.  Status HVP_INFEASIBLE when a row of the MLD model fails.
template <int N>
__global__ __launch_bounds__(kBlock) void k_evaluate(int B, const hvp_system* __restrict__ systems,
                                                     const int32_t* __restrict__ sys, const int32_t* __restrict__ role,
                                                     const double* __restrict__ params, hvp::Consts C,
                                                     const int8_t* __restrict__ gear_in, const double* __restrict__ u_in,
                                                     double* __restrict__ cost_out, int32_t* __restrict__ status_out,
                                                     double* __restrict__ x_out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B) return;
    const hvp_system& S = systems[sys[i]];
    const int rl = role[i];
    const double* prm = params + (size_t)i * (2 + 6 * (N + 1));
    hvp::LaneQp<N> q;
    q.has_sf = (rl & HVP_ROLE_SAFE_FRONT) != 0;
    q.has_sb = (rl & HVP_ROLE_SAFE_BACK) != 0;
    double p = prm[0], v = prm[1];
    uint64_t code = 0;
    bool ok = true;
    if (x_out) {
        x_out[(size_t)i * 2 * (N + 1)] = p;
        x_out[(size_t)i * 2 * (N + 1) + N + 1] = v;
    }
    for (int k = 0; k < N; ++k) {
        const int g = gear_in[(size_t)i * N + k];
        const double u = u_in[(size_t)i * N + k];
        int r = -1;
        for (int m = 0; m < S.n_regions && r < 0; ++m) {
            const double tol = 1e-9 * (1.0 + fabs(v));
            if (S.gear[m] == g && v >= S.vlo[m] - tol && v <= S.vhi[m] + tol) r = m;
        }
        if (r < 0) { ok = false; r = 0; }
        const double vn = S.a[r] * v + S.b[r] * u + S.c[r];
        const double tolu = 1e-9 * (1.0 + fabs(u));
        if (u < S.umin - tolu || u > S.umax + tolu) ok = false;
        const double dv = vn - v, tola = 1e-9 * (1.0 + fabs(dv));
        if (dv < C.dec[k] - tola || dv > C.acc[k] + tola) ok = false;
        p = p + S.ts * v;
        v = vn;
        const double tolv = 1e-9 * (1.0 + fabs(v)), tolp = 1e-9 * (1.0 + fabs(p));
        if (v < S.vmin - tolv || v > S.vmax + tolv || p < S.pmin - tolp || p > S.pmax + tolp) ok = false;
        q.y[k] = v;
        code = hvp::code_with(code, k, r);
        if (x_out) {
            x_out[(size_t)i * 2 * (N + 1) + k + 1] = p;
            x_out[(size_t)i * 2 * (N + 1) + N + 1 + k + 1] = v;
        }
    }
    const double cost = hvp::direct_cost<N>(q, S, C, rl, prm, code);
    cost_out[i] = ok ? cost : 1e300;
    status_out[i] = ok ? HVP_OPTIMAL : HVP_INFEASIBLE;
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

// ================================================================== switching ADMM (HVP_FORM_GADMM)
// TrackingGAdmmCoordinator / GAdmmCoordinator (fleet_g_admm.py:208-301, dmpcpwa [EXT]) for P
// platoons: rollout of the warm start, per ADMM iteration one local-QP launch + one consensus
// launch, sequence switching per round (include/hvp.h "Switching ADMM").  Instance b holds
// vehicle i = lo + b % m of platoon p = b / m; trajectories live in full-platoon slots p n + i.
__device__ inline int gadmm_slot(int b, int n, int lo, int m) { return (b / m) * n + lo + b % m; }

__device__ inline void gadmm_fail(int32_t* state, int p) {
    atomicOr(&state[p], 2);
    atomicAnd(&state[p], ~1);
}

// first region whose closed velocity band holds v (buf widens the lower edge: the [0, 1e-4]
// buffer of PwaGearVehicle.find_region used by get_u_for_constant_vel, models.py:519-540)
__device__ inline int gadmm_region(const hvp_system& S, double v, double buf) {
    for (int r = 0; r < S.n_regions; ++r)
        if (v >= S.vlo[r] - buf && v <= S.vhi[r]) return r;
    return -1;
}

template <int N>
__global__ __launch_bounds__(kBlock) void k_gadmm_rollout(int P, int n, int lo, int m,
                                                          const hvp_system* __restrict__ systems,
                                                          const int32_t* __restrict__ sys,
                                                          const double* __restrict__ params, int stride, int mode,
                                                          const double* __restrict__ u_prev, double* __restrict__ x,
                                                          int8_t* __restrict__ seq, double* __restrict__ u_ws,
                                                          int32_t* __restrict__ state) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= P * m) return;
    const int p = b / m;
    const hvp_system& S = systems[sys[b]];
    const double* prm = params + (size_t)b * stride;
    double pk = prm[0], vk = prm[1];
    double* xs = x + (size_t)gadmm_slot(b, n, lo, m) * 2 * (N + 1);
    bool ok = true;
    double ucv = 0.0;
    if (mode == 0) {
        const int r = gadmm_region(S, vk, 1e-4);
        if (r < 0) ok = false;
        else ucv = ((1.0 - S.a[r]) * vk - S.c[r]) / S.b[r];
    }
    xs[0] = pk;
    xs[N + 1] = vk;
    for (int k = 0; k < N; ++k) {
        const double u = mode == 0 ? ucv : u_prev[(size_t)b * N + (k + 1 < N ? k + 1 : N - 1)];
        int r = gadmm_region(S, vk, 0.0);
        if (r < 0) { ok = false; r = 0; }
        seq[(size_t)b * N + k] = (int8_t)r;
        if (u_ws) u_ws[(size_t)b * N + k] = u;
        const double vn = S.a[r] * vk + S.b[r] * u + S.c[r];
        pk = pk + S.ts * vk;
        vk = vn;
        xs[k + 1] = pk;
        xs[N + 1 + k + 1] = vk;
    }
    if (!ok) gadmm_fail(state, p);
}

// edge bits of the switching rule: active V rows at a region edge strictly inside the state box
template <int N>
__device__ inline uint32_t gadmm_edges(const hvp_system& S, uint64_t code, uint32_t raw) {
    uint32_t out = 0;
#pragma unroll
    for (int j = 0; j + 1 < N; ++j) {
        const int r = hvp::code_region(code, j + 1);
        const double lo = S.vlo[r], hi = S.vhi[r];
        if (((raw >> (2 * j)) & 1u) && lo > S.vmin + 1e-9 * (1.0 + fabs(lo))) out |= 1u << (2 * j);
        if (((raw >> (2 * j + 1)) & 1u) && hi < S.vmax - 1e-9 * (1.0 + fabs(hi))) out |= 1u << (2 * j + 1);
    }
    return out;
}

// outputs of one solved local problem: u, trajectory slot, copies (front: closed-form optimum of
// its hinge problem, back: z_b - y_b / rho)
template <int N>
__device__ inline void gadmm_write(int b, int slot, const hvp_system& S, const hvp::Consts& C, int rl,
                                   const double* prm, uint64_t code, const double* y, double* u_out, double* x,
                                   double* xf, double* xb) {
    const int K1 = N + 1;
    double* xs = x + (size_t)slot * 2 * K1;
    double* fs = xf + (size_t)slot * 2 * K1;
    double* bs = xb + (size_t)slot * 2 * K1;
    const bool front = (rl & HVP_ROLE_SAFE_FRONT) != 0, back = (rl & HVP_ROLE_BACK_COPY) != 0;
    const bool tf = (rl & HVP_ROLE_TRACK_FRONT) != 0;
    const double* yb = hvp::admm_y(prm, 1, N);
    const double* zb = hvp::admm_z(prm, 1, N);
    double p = prm[0], v = prm[1];
    for (int k = 0; k <= N; ++k) {
        xs[k] = p;
        xs[K1 + k] = v;
        double e = 0.0, g = 0.0;
        if (front)
            hvp::admm_copy_value(C, tf, 0, hvp::admm_y(prm, 0, N)[k], hvp::admm_y(prm, 0, N)[K1 + k],
                                 hvp::admm_z(prm, 0, N)[k], hvp::admm_z(prm, 0, N)[K1 + k], p, v, &e, &g);
        fs[k] = e;
        fs[K1 + k] = g;
        bs[k] = back ? zb[k] - yb[k] / C.rho : 0.0;
        bs[K1 + k] = back ? zb[K1 + k] - yb[K1 + k] / C.rho : 0.0;
        if (k < N) {
            const int r = hvp::code_region(code, k);
            const double vn = y[k];
            u_out[(size_t)b * N + k] = (vn - S.a[r] * v - S.c[r]) / S.b[r];
            p = p + S.ts * v;
            v = vn;
        }
    }
}

template <int N>
__device__ inline uint64_t gadmm_code(const int8_t* seq, int b) {
    uint64_t code = 0;
#pragma unroll
    for (int k = 0; k < N; ++k) code = hvp::code_with(code, k, seq[(size_t)b * N + k]);
    return code;
}

// x-update, one lane per local QP (N <= 8)
template <int N>
__global__ __launch_bounds__(kBnbBlock<N>) void k_gadmm_qp(int P, int n, int lo, int m,
                                                           const hvp_system* __restrict__ systems,
                                                           const int32_t* __restrict__ sys,
                                                           const int32_t* __restrict__ role,
                                                           const double* __restrict__ params, hvp::Consts C,
                                                           const int8_t* __restrict__ seq,
                                                           int32_t* __restrict__ state, double* __restrict__ u_out,
                                                           double* __restrict__ x, double* __restrict__ xf,
                                                           double* __restrict__ xb, double* __restrict__ cost_out,
                                                           int32_t* __restrict__ status_out,
                                                           uint32_t* __restrict__ edge_out,
                                                           int32_t* __restrict__ iters_out,
                                                           unsigned long long* __restrict__ counter) {
    constexpr int BS = kBnbBlock<N>;
    const int b = blockIdx.x * BS + threadIdx.x;
    if (b >= P * m) return;
    const int p = b / m;
    if (!(state[p] & 1)) return;
    const hvp_system& S = systems[sys[b]];
    const int rl = role[b];
    const double* prm = params + (size_t)b * C.stride;
    const uint64_t code = gadmm_code<N>(seq, b);
    hvp::LaneQp<N, LdsMem<N, BS>> q;
    q.mem.lane = threadIdx.x;
    int it = 0;
    uint32_t raw = 0;
    const int st = hvp::solve_admm_lane<N>(q, S, C, rl, prm, code, N, kGiMaxIter<N>, it, &raw);
    if (iters_out) iters_out[b] = it;
    atomicAdd(&counter[1], (unsigned long long)it);
    if (st == hvp::GI_OK) {
        cost_out[b] = hvp::admm_direct_cost<N>(q, S, C, rl, prm, code, N);
        status_out[b] = HVP_OPTIMAL;
        edge_out[b] = gadmm_edges<N>(S, code, raw);
        gadmm_write<N>(b, gadmm_slot(b, n, lo, m), S, C, rl, prm, code, q.y, u_out, x, xf, xb);
    } else {
        cost_out[b] = 1e300;
        status_out[b] = st == hvp::GI_FAIL_DUAL ? HVP_INFEASIBLE : HVP_MAXITER;
        edge_out[b] = 0;
        gadmm_fail(state, p);
    }
}

// x-update, one 16-lane group per local QP (long horizons, hvp_coop.h)
template <int N>
__global__ __launch_bounds__(kCoopBlock) void k_gadmm_qp_coop(int P, int n, int lo, int m,
                                                              const hvp_system* __restrict__ systems,
                                                              const int32_t* __restrict__ sys,
                                                              const int32_t* __restrict__ role,
                                                              const double* __restrict__ params, hvp::Consts C,
                                                              const int8_t* __restrict__ seq,
                                                              int32_t* __restrict__ state, double* __restrict__ u_out,
                                                              double* __restrict__ x, double* __restrict__ xf,
                                                              double* __restrict__ xb, double* __restrict__ cost_out,
                                                              int32_t* __restrict__ status_out,
                                                              uint32_t* __restrict__ edge_out,
                                                              int32_t* __restrict__ iters_out,
                                                              unsigned long long* __restrict__ counter) {
    __shared__ hvp::coop::GroupLds lds[kCoopGroups];
    const int g = threadIdx.x / hvp::coop::G, t = threadIdx.x % hvp::coop::G;
    const int b = blockIdx.x * kCoopGroups + g;
    if (b >= P * m) return;  // group-uniform
    const int p = b / m;
    if (!(state[p] & 1)) return;
    const hvp_system& S = systems[sys[b]];
    const int rl = role[b];
    const double* prm = params + (size_t)b * C.stride;
    const uint64_t code = gadmm_code<N>(seq, b);
    hvp::coop::Lane<N> L;
    double cost = 0.0;
    int it = 0;
    unsigned raw = 0;
    const int st = hvp::coop::solve_qp<N>(L, lds[g], S, C, rl, prm, code, N, kGiMaxIter<N>, it, &cost, &raw);
    if (st == hvp::GI_OK) {
        lds[g].v[t] = t < N ? L.y : 0.0;
        hvp::coop::gsync();
    }
    if (t != 0) return;
    if (iters_out) iters_out[b] = it;
    atomicAdd(&counter[1], (unsigned long long)it);
    if (st == hvp::GI_OK) {
        double y[N];
#pragma unroll
        for (int k = 0; k < N; ++k) y[k] = lds[g].v[k];
        cost_out[b] = cost;
        status_out[b] = HVP_OPTIMAL;
        edge_out[b] = gadmm_edges<N>(S, code, raw);
        gadmm_write<N>(b, gadmm_slot(b, n, lo, m), S, C, rl, prm, code, y, u_out, x, xf, xb);
    } else {
        cost_out[b] = 1e300;
        status_out[b] = st == hvp::GI_FAIL_DUAL ? HVP_INFEASIBLE : HVP_MAXITER;
        edge_out[b] = 0;
        gadmm_fail(state, p);
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

int grid_for(long long n) { return (int)std::max<long long>(1, (n + kBlock - 1) / kBlock); }

template <int N>
int launch_bnb(hvp_handle* h, int B, const int32_t* sys, const int32_t* role, const double* params, double* u_out,
               double* x_out, int8_t* region_out, int8_t* gear_out, double* cost_out, int32_t* status_out,
               int32_t* nodes_out, int32_t* iters_out, hipStream_t st, double* xf_out = nullptr,
               double* xb_out = nullptr) {
    Workspace ws = h->ws;
    constexpr int BS = kBnbBlock<N>;
    HIP_TRY(hipMemsetAsync(ws.counter, 0, 8 * sizeof(unsigned long long), st));
    HIP_TRY(hipMemsetAsync(ws.lvl, 0, (HVP_MAX_N + 1) * sizeof(unsigned long long), st));
    HIP_TRY(hipEventRecord(h->ev0, st));
    HIP_TRY(hipEventRecord(h->evq0, st));
    const size_t lds = sizeof(double) * hvp::F_COUNT * N * BS;
    HIP_TRY(hipEventRecord(h->evb[0], st));
    if constexpr (kCoop<N>) {
        hipLaunchKernelGGL(k_bnb_root_coop<N>, dim3((B + kCoopGroups - 1) / kCoopGroups), dim3(kCoopBlock), 0, st, B,
                           h->d_sys, sys, role, params, h->C, ws);
    } else {
        if (h->C.form == HVP_FORM_ADMM)
            hipLaunchKernelGGL((k_bnb_root<N, true>), dim3((B + BS - 1) / BS), dim3(BS), lds, st, B, h->d_sys, sys,
                               role, params, h->C, ws);
        else
            hipLaunchKernelGGL((k_bnb_root<N, false>), dim3((B + BS - 1) / BS), dim3(BS), lds, st, B, h->d_sys, sys,
                               role, params, h->C, ws);
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(h->evb[1], st));
    const int g_small = (int)std::min<long long>(grid_for(h->ws.cap), (long long)h->n_cu * 8);
    const int g_qp = (int)std::min<long long>((h->ws.cap + BS - 1) / BS, (long long)h->n_cu * 8 * (kBlock / BS));
    const int quota = (int)std::min<int64_t>(h->ws.cap / B, 1 << 30);
    for (int k = 1; k <= N; ++k) {
        HIP_TRY(hipMemsetAsync(ws.inst_lvl, 0, sizeof(int32_t) * B, st));
        hipLaunchKernelGGL(k_bnb_expand<N>, dim3(g_small), dim3(kBlock), 0, st, k, quota, h->d_sys, sys, h->C, ws);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipEventRecord(h->evb[2 * k], st));
        if constexpr (kCoop<N>) {
            const int g_coop = (int)std::min<long long>((h->ws.cap + kCoopGroups - 1) / kCoopGroups,
                                                        (long long)h->n_cu * 32);
            hipLaunchKernelGGL(k_bnb_bound_coop<N>, dim3(g_coop), dim3(kCoopBlock), 0, st, k, h->d_sys, sys, role,
                               params, h->C, ws);
        } else {
            if (h->C.form == HVP_FORM_ADMM)
                hipLaunchKernelGGL((k_bnb_bound<N, true>), dim3(g_qp), dim3(BS), lds, st, k, h->d_sys, sys, role,
                                   params, h->C, ws);
            else
                hipLaunchKernelGGL((k_bnb_bound<N, false>), dim3(g_qp), dim3(BS), lds, st, k, h->d_sys, sys, role,
                                   params, h->C, ws);
        }
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipEventRecord(h->evb[2 * k + 1], st));
    }
    HIP_TRY(hipEventRecord(h->evq1, st));
    if constexpr (N <= HVP_MAX_N_ENUM) {
        if (h->C.form == HVP_FORM_DECENT)
        hipLaunchKernelGGL(k_bnb_ipm<N>, dim3(std::max(1, h->n_cu)), dim3(BS), lds, st, h->d_sys, sys, role, params,
                           h->C, ws);
        HIP_TRY(hipGetLastError());
    }
    hipLaunchKernelGGL(k_bnb_key<N>, dim3(g_small), dim3(kBlock), 0, st, ws, h->C.form);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(k_bnb_write<N>, dim3(g_small), dim3(kBlock), 0, st, h->d_sys, sys, role, params, h->C, ws,
                       u_out, x_out, region_out, gear_out, cost_out, xf_out, xb_out);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(k_bnb_finish<N>, dim3(grid_for(B)), dim3(kBlock), 0, st, B, h->d_sys, sys, role, params, h->C,
                       ws, u_out, x_out, region_out, gear_out, cost_out, status_out, nodes_out, iters_out, xf_out,
                       xb_out);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(h->ev1, st));
    h->last_stream = st;
    h->last_B = B;
    h->last_bnb = true;
    return 0;
}

template <int N>
int launch_all(hvp_handle* h, int B, const int32_t* sys, const int32_t* role, const double* params, double* u_out,
               double* x_out, int8_t* region_out, int8_t* gear_out, double* cost_out, int32_t* status_out,
               int32_t* nodes_out, int32_t* iters_out, hipStream_t st) {
    Workspace ws = h->ws;
    HIP_TRY(hipMemsetAsync(ws.counter, 0, 8 * sizeof(unsigned long long), st));
    HIP_TRY(hipEventRecord(h->ev0, st));
    hipLaunchKernelGGL(k_enum<N>, dim3(grid_for(B)), dim3(kBlock), 0, st, B, h->d_sys, sys, role, params, h->C, ws);
    HIP_TRY(hipGetLastError());
    // the candidate count is only known on the device: size the grid for the capacity bound
    // (≈ every CU x 8 blocks) and let the kernel grid-stride over the real count
    const long long want = std::min<long long>(grid_for(h->ws.cap), (long long)h->n_cu * 8);
    HIP_TRY(hipEventRecord(h->evq0, st));
    const size_t lds = sizeof(double) * hvp::F_COUNT * N * kBlock;
    hipLaunchKernelGGL(k_qp_gi<N>, dim3((int)want), dim3(kBlock), lds, st, h->d_sys, sys, role, params, h->C, ws);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(h->evq1, st));
    // fallback list (normally empty: the launch reads a zero count and exits)
    hipLaunchKernelGGL(k_qp_ipm<N>, dim3(std::max(1, h->n_cu)), dim3(kBlock), lds, st, h->d_sys, sys, role,
                       params, h->C, ws);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(k_cost<N>, dim3((int)want), dim3(kBlock), 0, st, h->d_sys, sys, role, params, h->C, ws);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(k_select<N>, dim3(grid_for(B)), dim3(kBlock), 0, st, B, h->d_sys, sys, params, ws, u_out,
                       x_out, region_out, gear_out, cost_out, status_out, nodes_out, iters_out);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(h->ev1, st));
    h->last_stream = st;
    h->last_B = B;
    h->last_bnb = false;
    return 0;
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
    (void)hipFree(w.inst_lvl);
    w = Workspace{};
}

int64_t default_capacity(int N, int B, bool bnb) {
    if (bnb) {
        // nodes of ONE tree level, pooled over the batch (C2..C5 means: 3 leaves at N = 5, 4 at
        // N = 10, 30 at N = 15; the widest level a few times that)
        const int64_t per = N <= 8 ? 64 : (N <= 12 ? 256 : 1024);
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
    if (problem->quadratic_cost != 1)
        return fail(HVP_E_UNSUPPORTED, "hvp_create: only the quadratic cost (min_2_norm) runs on the GPU");
    for (int i = 0; i < n_systems; ++i) {
        std::string why;
        if (!valid_system(systems[i], &why)) return fail(HVP_E_ARG, "hvp_create: system " + std::to_string(i) + ": " + why);
    }
    HIP_TRY(hipSetDevice(device));
    hvp_handle* h = new hvp_handle();
    h->device = device;
    h->prob = *problem;
    h->C = make_consts(*problem);
    h->bnb = problem->method == HVP_METHOD_BNB || (problem->method == HVP_METHOD_AUTO && problem->N > kAutoEnumMaxN);
    h->n_systems = n_systems;
    for (int i = 0; i < n_systems; ++i) h->nreg_max = std::max(h->nreg_max, (int)systems[i].n_regions);
    (void)hipDeviceGetAttribute(&h->n_cu, hipDeviceAttributeMultiprocessorCount, device);
    if (hipMalloc(&h->d_sys, sizeof(hvp_system) * n_systems) != hipSuccess ||
        hipMemcpy(h->d_sys, systems, sizeof(hvp_system) * n_systems, hipMemcpyHostToDevice) != hipSuccess ||
        hipEventCreate(&h->ev0) != hipSuccess || hipEventCreate(&h->ev1) != hipSuccess ||
        hipEventCreate(&h->evq0) != hipSuccess || hipEventCreate(&h->evq1) != hipSuccess ||
        hipMalloc(&h->g_counter, 8 * sizeof(unsigned long long)) != hipSuccess ||
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
    if (cap <= 0) cap = default_capacity(h->prob.N, max_batch, h->bnb);
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
             hipMalloc(&w.lvl, sizeof(unsigned long long) * (HVP_MAX_N + 1)) == hipSuccess &&
             hipMalloc(&w.inst_lvl, sizeof(int32_t) * max_batch) == hipSuccess;
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
        int rc = hvp_reserve(h, B, default_capacity(h->prob.N, B, h->bnb));
        if (rc) return rc;
    }
    HIP_TRY(hipSetDevice(h->device));
    hipStream_t st = (hipStream_t)stream;
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
#define HVP_CASE(n)                                                                                              \
    case n:                                                                                                      \
        hipLaunchKernelGGL(k_evaluate<n>, dim3(grid_for(B)), dim3(kBlock), 0, st, B, h->d_sys, sys, role, params, \
                           h->C, gear_in, u_in, cost_out, status_out, x_out);                                    \
        break;
        HVP_CASE(2) HVP_CASE(3) HVP_CASE(4) HVP_CASE(5) HVP_CASE(6) HVP_CASE(7) HVP_CASE(8)
        HVP_CASE(9) HVP_CASE(10) HVP_CASE(11) HVP_CASE(12) HVP_CASE(13) HVP_CASE(14) HVP_CASE(15) HVP_CASE(16)
#undef HVP_CASE
        default: return fail(HVP_E_UNSUPPORTED, "hvp_evaluate_batch: unsupported N");
    }
    HIP_TRY(hipGetLastError());
    return 0;
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
    const int B = P * m;
    HIP_TRY(hipMemsetAsync(h->g_counter, 0, 8 * sizeof(unsigned long long), (hipStream_t)stream));
    switch (h->prob.N) {
#define HVP_CASE(nn)                                                                                                \
    case nn:                                                                                                        \
        hipLaunchKernelGGL(k_gadmm_rollout<nn>, dim3(grid_for(B)), dim3(kBlock), 0, (hipStream_t)stream, P, n, lo, m, \
                           h->d_sys, sys, params, h->C.stride, mode, u_prev, x, seq, u_ws, state);                  \
        break;
        HVP_CASE(2) HVP_CASE(3) HVP_CASE(4) HVP_CASE(5) HVP_CASE(6) HVP_CASE(7) HVP_CASE(8)
        HVP_CASE(9) HVP_CASE(10) HVP_CASE(11) HVP_CASE(12) HVP_CASE(13) HVP_CASE(14) HVP_CASE(15) HVP_CASE(16)
#undef HVP_CASE
        default: return fail(HVP_E_UNSUPPORTED, "hvp_gadmm_rollout: unsupported N");
    }
    HIP_TRY(hipGetLastError());
    return 0;
}

}  // extern "C"

template <int N>
static int launch_gadmm_qp(hvp_handle* h, int P, int n, int lo, int m, const int32_t* sys, const int32_t* role,
                           const double* params, const int8_t* seq, int32_t* state, double* u_out, double* x,
                           double* xf, double* xb, double* cost_out, int32_t* status_out, uint32_t* edge_out,
                           int32_t* iters_out, hipStream_t st) {
    const int B = P * m;
    HIP_TRY(hipEventRecord(h->evq0, st));
    if constexpr (kCoop<N>) {
        hipLaunchKernelGGL(k_gadmm_qp_coop<N>, dim3((B + kCoopGroups - 1) / kCoopGroups), dim3(kCoopBlock), 0, st, P, n,
                           lo, m, h->d_sys, sys, role, params, h->C, seq, state, u_out, x, xf, xb, cost_out,
                           status_out, edge_out, iters_out, h->g_counter);
    } else {
        constexpr int BS = kBnbBlock<N>;
        const size_t lds = sizeof(double) * hvp::F_COUNT * N * BS;
        hipLaunchKernelGGL(k_gadmm_qp<N>, dim3((B + BS - 1) / BS), dim3(BS), lds, st, P, n, lo, m, h->d_sys, sys, role,
                           params, h->C, seq, state, u_out, x, xf, xb, cost_out, status_out, edge_out, iters_out,
                           h->g_counter);
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(h->evq1, st));
    h->last_stream = st;
    h->last_B = B;
    h->last_bnb = false;
    return 0;
}

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
        unsigned long long lv[HVP_MAX_N + 1];
        HIP_TRY(hipMemcpy(lv, h->ws.lvl, sizeof(lv), hipMemcpyDeviceToHost));
        int64_t n = (int64_t)c[3];
        for (int k = 1; k <= h->prob.N; ++k) n += (int64_t)std::min<unsigned long long>(lv[k], (unsigned long long)h->ws.cap);
        out->n_candidates = n;
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
    if (h->d_consts) (void)hipFree(h->d_consts);
    if (h->ev0) (void)hipEventDestroy(h->ev0);
    if (h->ev1) (void)hipEventDestroy(h->ev1);
    if (h->evq0) (void)hipEventDestroy(h->evq0);
    if (h->evq1) (void)hipEventDestroy(h->evq1);
    for (hipEvent_t& e : h->evb)
        if (e) (void)hipEventDestroy(e);
    delete h;
}

}  // extern "C"
