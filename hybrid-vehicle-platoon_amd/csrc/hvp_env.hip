// hvp_env.hip -- the caller side of the hot path on the device: the platoon plant step
// (env.py PlatoonEnv.step / get_stage_cost, models.py Platoon.step_platoon), batched over P
// platoons so a closed loop (solve -> step -> solve) never leaves HBM.
//
//   gear      from the action (MpcGear outputs) or, when the action carries none, the gear of
//             the PWA-gear model for the current velocity (env.py:198-204 ->
//             models.py:494-515: half-open bands between v_gear_lim = band midpoints of gears
//             2..6; below the first -> 1, from the last on -> 6), held over the sample;
//   stage     cost of (x, u) before the step (env.py:126-180; quad_cost, or lin_cost = ||Q e||_1
//             when the handle's problem has quadratic_cost = 0, env.py:118-124): leader tracking
//             (or real vehicle as reference with its spacing), the chain spacing terms,
//             Q_u u^2, Q_du (u - u_prev)^2, and the violation flag (100 when any gap
//             p_i - p_{i+1} < d_safe, or the leader gap with real_vehicle_as_reference);
//   step      10 explicit Euler sub-steps of the nonlinear vehicle (models.py:114-125,
//             236-257): p' = p + dt v, v' = v + dt (-(c_fric v^2)/m - mu g + F(v, gear) u / m)
//             with the traction curve F of models.py:10-51 (rise, plateau, fall per gear).
// One thread per vehicle (state update), one warp-reduction per platoon for the cost.
#include <hip/hip_runtime.h>

#include <string>

#define HVP_HD __host__ __device__
#include "hvp.h"
#include "hvp_internal.h"

using hvp_detail::fail;

namespace {

// models.py:13-40 traction table: per gear three force levels and four velocity knots
__constant__ double kTracT[6][3] = {{253.54, 4056.7, 3042.0},  {184.0, 2944.75, 2208.55}, {132.22, 2115.6, 1586.7},
                                    {100.0 / 415.0, 1605.0, 1205.0}, {72.88, 1166.0, 874.7},    {52.4, 838.0, 628.3}};
__constant__ double kTracV[6][4] = {{2.0706, 4.12158, 9.29, 12.38},    {2.85, 5.675, 12.7956, 17.06},
                                    {3.9705, 7.90316, 17.8105, 23.7474}, {5.228, 10.42, 23.454, 31.2704},
                                    {7.203, 14.335, 32.31, 43.0802},     {10.027, 19.956, 44.978, 59.9715}};
__constant__ double kVl[6] = {3.94, 5.43, 7.56, 9.96, 13.70, 19.10};
__constant__ double kVh[6] = {9.46, 13.04, 18.15, 23.90, 32.93, 45.84};
constexpr double kCFric = 0.5, kMu = 0.01, kGrav = 9.8;

// F(v, gear), false when v is outside the gear's curve (the reference raises)
__device__ inline bool traction(double v, int j, double* f) {
    const double v0 = kTracV[j - 1][0], v1 = kTracV[j - 1][1], v2 = kTracV[j - 1][2], v3 = kTracV[j - 1][3];
    const double flo = kTracT[j - 1][0], ftop = kTracT[j - 1][1], fend = kTracT[j - 1][2];
    if (v <= v0 || v >= v3) return false;
    // the reference's operation order (models.py:41-48)
    if (v < v1) *f = ((v - v0) / (v1 - v0)) * (ftop - flo) + flo;
    else if (v > v2) *f = ftop - ((v - v2) / (v3 - v2)) * (ftop - fend);
    else *f = ftop;
    return true;
}

// PwaGearVehicle.get_gear_from_velocity (models.py:494-515)
__device__ inline int gear_of_velocity(double v) {
    double g[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) g[i] = (kVh[i + 1] - kVl[i + 1]) / 2 + kVl[i + 1];
#pragma unroll
    for (int i = 0; i < 4; ++i)
        if (g[i] <= v && v < g[i + 1]) return i + 2;
    return v < g[0] ? 1 : 6;
}

__global__ __launch_bounds__(64) void k_env_step(int P, int n, const double* __restrict__ masses, double* __restrict__ x,
                                                 const double* __restrict__ u, const int8_t* __restrict__ gear,
                                                 const double* __restrict__ u_prev,
                                                 const double* __restrict__ leader_x, int leader, int rvar, double ts,
                                                 hvp::Consts C, double* __restrict__ cost_out,
                                                 int32_t* __restrict__ viol_out, int32_t* __restrict__ status_out) {
    // one 64-lane wave per platoon, lane i = vehicle i (n <= 64)
    const int p = blockIdx.x;
    const int i = threadIdx.x;
    if (p >= P) return;
    const bool on = i < n;
    double* xp = x + (size_t)p * 2 * n;
    const double pos = on ? xp[2 * i] : 0.0, vel = on ? xp[2 * i + 1] : 0.0;
    const double ui = on ? u[(size_t)p * n + i] : 0.0;
    const double upi = on ? u_prev[(size_t)p * n + i] : 0.0;
    // ---- stage cost of (x, u) (env.py:126-180)
    const double pm = __shfl(pos, i > 0 ? i - 1 : 0, 64), vm = __shfl(vel, i > 0 ? i - 1 : 0, 64);
    const double pn = __shfl(pos, i + 1 < n ? i + 1 : i, 64);
    // PlatoonEnv's own weights (env.py:16-18: Q_x = diag(1, 0.1), Q_u = 1, Q_du = 0), not the
    // controller's: the env prices every controller's actions alike
    constexpr double kQpp = 1.0, kQvv = 0.1, kQu = 1.0;
    const bool lin = C.l1 != 0;  // lin_cost (env.py:122-124): |Q_pp e_p| + |Q_vv e_v|, |Q_u u|
    auto quad = [&](double ep, double ev) {
        return lin ? fabs(kQpp * ep) + fabs(kQvv * ev) : kQpp * ep * ep + kQvv * ev * ev;
    };
    double c = 0.0;
    int close = 0;
    if (on) {
        const double rp = leader_x[(size_t)p * 2], rv = leader_x[(size_t)p * 2 + 1];
        if (rvar ? i == 0 : i == leader) c += quad(pos - rp + (rvar ? C.d0 + C.t0 * vel : 0.0), vel - rv);
        if (i >= 1) c += quad(pos - pm + C.d0 + C.t0 * vel, vel - vm);
        c += lin ? fabs(kQu * ui) : kQu * ui * ui;  // + the Q_du term, zero with Q_du = 0
        (void)upi;
        if (i + 1 < n && pos - pn < C.d_safe) close = 1;
        if (rvar && i == 0 && rp - pos < C.d_safe) close = 1;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    const bool any_close = __ballot(close != 0) != 0ull;
    // ---- 10 Euler sub-steps of the nonlinear model (models.py:236-257)
    int bad = 0;
    if (on) {
        const double m = masses[(size_t)p * n + i];
        int j = gear ? (int)gear[(size_t)p * n + i] : 0;
        if (j <= 0) j = gear_of_velocity(vel);
        if (j < 1 || j > 6) bad = 1;
        double pp = pos, vv = vel;
        const double dt = ts / 10.0;
        for (int s = 0; s < 10 && !bad; ++s) {
            double f = 0.0;
            if (vv < kTracV[0][0] || vv > kTracV[5][3] || !traction(vv, j, &f)) {
                bad = 1;
                break;
            }
            const double dp = vv;
            // x + dt (A(x) + B(x, j) u), models.py:99-125
            const double dv = (-(kCFric * (vv * vv)) / m - kMu * kGrav) + (f / m) * ui;
            pp = pp + dt * dp;
            vv = vv + dt * dv;
        }
        xp[2 * i] = pp;
        xp[2 * i + 1] = vv;
    }
    const bool any_bad = __ballot(bad != 0) != 0ull;
    if (i == 0) {
        cost_out[p] = c;
        viol_out[p] = any_close ? 100 : 0;
        status_out[p] = any_bad ? 1 : 0;
    }
}

// TrackingDecentMldCoordinator.observe_states (fleet_decent_mld.py:348-455) for P platoons: one
// thread per (platoon, vehicle) writes the vehicle's local-MPC parameter block (include/hvp.h
// layout: x0 | x_front | x_back | leader_x) and role bits.  est: 0 constant velocity (:421-428),
// 1 two-point (:430-440), 2 saturated two-point (:442-455); x_prev feeds the estimators.
__global__ __launch_bounds__(256) void k_decent_params(int P, int n, int N, const double* __restrict__ x,
                                                       const double* __restrict__ x_prev,
                                                       const double* __restrict__ leader_x, int leader, int rvar,
                                                       int est, double ts, double* __restrict__ params,
                                                       int32_t* __restrict__ roles) {
    const long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= (long long)P * n) return;
    const int p = (int)(g / n), i = (int)(g % n);
    const double* xp = x + (size_t)p * 2 * n;
    const double* xq = x_prev ? x_prev + (size_t)p * 2 * n : xp;
    const int K = N + 1;
    double* out = params + (size_t)g * (2 + 6 * K);
    out[0] = xp[2 * i];
    out[1] = xp[2 * i + 1];
    auto predict = [&](int j, double* dst) {  // extrapolate vehicle j's state into dst (2, N+1)
        double pp = xp[2 * j], vv = xp[2 * j + 1];
        const double dv = est ? vv - xq[2 * j + 1] : 0.0;
        dst[0] = pp;
        dst[K] = vv;
        for (int k = 0; k < N; ++k) {
            pp = pp + ts * vv;
            vv = vv + (est == 0 || (est == 2 && k >= N / 2) ? 0.0 : dv);
            dst[k + 1] = pp;
            dst[K + k + 1] = vv;
        }
    };
    double* xf = out + 2;
    double* xb = out + 2 + 2 * K;
    double* xl = out + 2 + 4 * K;
    if (i > 0) predict(i - 1, xf);
    else
        for (int k = 0; k < 2 * K; ++k) xf[k] = 0.0;
    if (i < n - 1) predict(i + 1, xb);
    else
        for (int k = 0; k < 2 * K; ++k) xb[k] = 0.0;
    const double* lw = leader_x + (size_t)p * 2 * K;
    for (int k = 0; k < 2 * K; ++k) xl[k] = i == leader ? lw[k] : 0.0;
    int r = 0;  // tables.role_bits (fleet_decent_mld.py:100-153, 191-208)
    if (i != 0) r |= HVP_ROLE_SAFE_FRONT;
    if (i != n - 1) r |= HVP_ROLE_SAFE_BACK;
    if (i != 0 && i != leader) r |= HVP_ROLE_TRACK_FRONT;
    if (i != n - 1 && i != leader) r |= HVP_ROLE_TRACK_BACK;
    if (i == leader) r |= HVP_ROLE_TRACK_LEADER | (rvar ? HVP_ROLE_LEADER_SPACING : 0);
    roles[g] = r;
}

}  // namespace

extern "C" {

int hvp_decent_params_batch(hvp_handle* h, int P, int n, const double* x, const double* x_prev,
                            const double* leader_x, int leader_index, int real_vehicle_as_reference, int estimator,
                            double* params, int32_t* roles, void* stream) {
    if (!h) return fail(HVP_E_ARG, "hvp_decent_params_batch: null handle");
    if (h->prob.formulation != HVP_FORM_DECENT)
        return fail(HVP_E_ARG, "hvp_decent_params_batch: the handle is not an HVP_FORM_DECENT problem");
    if (P < 0 || n < 1 || leader_index < 0 || leader_index >= n || estimator < 0 || estimator > 2)
        return fail(HVP_E_ARG, "hvp_decent_params_batch: bad layout / estimator");
    if (P == 0) return 0;
    if (!x || !leader_x || !params || !roles) return fail(HVP_E_ARG, "hvp_decent_params_batch: bad argument");
    HIP_TRY(hipSetDevice(h->device));
    const long long total = (long long)P * n;
    hipLaunchKernelGGL(k_decent_params, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream, P, n,
                       h->prob.N, x, x_prev, leader_x, leader_index, real_vehicle_as_reference ? 1 : 0, estimator,
                       h->prob.ts_acc, params, roles);
    HIP_TRY(hipGetLastError());
    return 0;
}

int hvp_env_step_batch(hvp_handle* h, int P, int n, const double* masses, double* x, const double* u,
                       const int8_t* gear, const double* u_prev, const double* leader_x, int leader_index,
                       int real_vehicle_as_reference, double ts, double* cost_out, int32_t* viol_out,
                       int32_t* status_out, void* stream) {
    if (!h) return fail(HVP_E_ARG, "hvp_env_step_batch: null handle");
    if (P < 0 || n < 1 || n > 64 || !(ts > 0))
        return fail(HVP_E_ARG, "hvp_env_step_batch: need P >= 0, 1 <= n <= 64, ts > 0");
    if (leader_index < 0 || leader_index >= n) return fail(HVP_E_ARG, "hvp_env_step_batch: leader_index out of range");
    if (P == 0) return 0;
    if (!masses || !x || !u || !u_prev || !leader_x || !cost_out || !viol_out || !status_out)
        return fail(HVP_E_ARG, "hvp_env_step_batch: bad argument");
    HIP_TRY(hipSetDevice(h->device));
    hipLaunchKernelGGL(k_env_step, dim3(P), dim3(64), 0, (hipStream_t)stream, P, n, masses, x, u, gear, u_prev,
                       leader_x, leader_index, real_vehicle_as_reference ? 1 : 0, ts, h->C, cost_out, viol_out,
                       status_out);
    HIP_TRY(hipGetLastError());
    return 0;
}

}  // extern "C"
