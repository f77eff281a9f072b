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
__global__ __launch_bounds__(64) void k_cent_bnb(int P, int n, int N, int leader, int lsp,
                                                 const hvp_system* __restrict__ systems,
                                                 const int32_t* __restrict__ sys, const double* __restrict__ x0,
                                                 const double* __restrict__ xl, const hvp::Consts* __restrict__ Cp, int nreg_max,
                                                 int max_nodes, int exhaustive, int max_iter, int debug,
                                                 hvp::cent::Child* frames, uint64_t* ties, double* __restrict__ u_out,
                                                 double* __restrict__ x_out, int8_t* __restrict__ region_out,
                                                 int8_t* __restrict__ gear_out, double* __restrict__ cost_out,
                                                 int32_t* __restrict__ status_out, int32_t* __restrict__ nodes_out,
                                                 int32_t* __restrict__ iters_out,
                                                 unsigned long long* __restrict__ counter) {
    using namespace hvp::cent;
    extern __shared__ double cent_lds[];
    const hvp::Consts& C = *Cp;  // in global memory: lane-indexed rows (C.dec[a]) stay loads
    const int p = blockIdx.x;
    if (p >= P) return;
    const int t = lane();
    const int V = n * N;
    const Lds S = lds_carve(cent_lds, V);
    Inst I;
    I.n = n;
    I.N = N;
    I.V = V;
    I.L = leader;
    I.lsp = lsp != 0;
    I.systems = systems;
    I.vsys = sys + (size_t)p * n;
    I.x0 = x0 + (size_t)p * 2 * n;
    I.xl = xl + (size_t)p * 2 * (N + 1);
    I.debug = debug;
    Lane L;
    Search st;
    Result res;
    bnb_platoon(L, S, C, I, st, frames + (size_t)p * V * nreg_max, nreg_max, ties + (size_t)p * kTie * n, max_nodes,
                exhaustive != 0, max_iter, res);
    const bool win = res.status == HVP_OPTIMAL;
    const int i = t < V ? t / N : 0, a = t < V ? t % N : 0;
    const uint64_t ci = bc(st.vcode, i);
    double u = 0.0;
    if (win) direct_cost(L, C, I, ci, N, &u);  // wave-uniform branch
    const double yv = win && t < V ? L.y : 0.0;
    const double cum = vehicle_prefix(yv, N);
    if (t < V) {
        const hvp_system& Sv = systems[I.vsys[i]];
        const size_t veh = (size_t)p * n + i;
        const double p0 = I.x0[2 * i], v0 = I.x0[2 * i + 1];
        if (x_out) {
            double* xo = x_out + veh * 2 * (N + 1);
            if (a == 0) {
                xo[0] = p0;
                xo[N + 1] = v0;
            }
            // no solution: the constant-velocity trajectory with u = 0 (as k_bnb_finish)
            xo[a + 1] = win ? p0 + Sv.ts * v0 + Sv.ts * cum : p0 + Sv.ts * v0 * (a + 1);
            xo[N + 1 + a + 1] = win ? yv : v0;
        }
        if (u_out) u_out[veh * N + a] = win ? u : 0.0;
        const int r = hvp::code_region(ci, a);
        if (region_out) region_out[veh * N + a] = (int8_t)(win ? r : -1);
        if (gear_out) gear_out[veh * N + a] = (int8_t)(win ? Sv.gear[r] : 0);
    }
    if (t == 0) {
        cost_out[p] = win ? res.cost : 1e300;
        status_out[p] = res.status;
        if (nodes_out) nodes_out[p] = res.nodes;
        if (iters_out) iters_out[p] = res.iters;
        atomicAdd(&counter[0], (unsigned long long)res.nodes);
        atomicAdd(&counter[1], (unsigned long long)res.iters);
    }
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
    const size_t lds = hvp::cent::lds_doubles(V) * sizeof(double);
    HIP_TRY(hipFuncSetAttribute((const void*)k_cent_bnb, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    HIP_TRY(hipMemsetAsync(h->g_counter, 0, 8 * sizeof(unsigned long long), st));
    const int exhaustive = h->prob.method == HVP_METHOD_ENUMERATE ? 1 : 0;
    const char* dbg = std::getenv("HVP_CENT_DEBUG");  // diagnostics: printf of failing QPs
    const int debug = dbg && dbg[0] ? std::atoi(dbg) : 0;  // 1: failures, 2: + every GI step
    const int cap = max_nodes > 0 ? max_nodes : 200000;
    const int max_iter = 8 * hvp::cent::ROWS * V;  // active-set iterations per QP
    HIP_TRY(hipEventRecord(h->ev0, st));
    HIP_TRY(hipEventRecord(h->evq0, st));
    hipLaunchKernelGGL(k_cent_bnb, dim3(P), dim3(64), lds, st, P, n, N, leader_index, real_vehicle_as_reference ? 1 : 0,
                       h->d_sys, sys, x0, leader_x, h->d_consts, h->nreg_max, cap, exhaustive, max_iter, debug, h->cent_frames,
                       h->cent_ties, u_out, x_out, region_out, gear_out, cost_out, status_out, nodes_out, iters_out,
                       h->g_counter);
    HIP_TRY(hipGetLastError());
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
