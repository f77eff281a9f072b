/*
 * hvp.h -- C ABI of libhvpsolve.so, the MI355X batched hybrid-MPC (MLD MIQP) solver.
 *
 * This is the drop-in boundary for the reference's per-timestep local MIQP solve:
 *
 *   reference call site                                   replaced by
 *   ----------------------------------------------------  ----------------------------------
 *   MpcMld.__init__(system, N, thread_limit,               hvp_create()   (model build, once)
 *     constrain_first_state=False)  [EXT dmpcpwa]
 *     called from fleet_decent_mld.py:46-48
 *   LocalMpcMld.setup_cost_and_constraints                 hvp_problem + HVP_ROLE_* flags
 *     fleet_decent_mld.py:61-208
 *   LocalMpcMld.set_leader_x / set_x_front / set_x_back    the params block of each instance
 *     fleet_decent_mld.py:210-223
 *   MpcMld.solve_mpc(state) -> gp.Model.optimize()         hvp_solve_batch() (B instances at once)
 *     [EXT], called via MldAgent.get_control at
 *     fleet_decent_mld.py:316
 *   gurobi Status / Runtime / NodeCount / NumBinVars       status_out / timing / nodes_out / 7N
 *     read at fleet_decent_mld.py:336-337, mpcs/mpc_gear.py:119
 *
 * Conventions
 *   - Plain C types only; every array is caller-owned.  hvp_solve_batch takes DEVICE pointers
 *     (e.g. torch tensors on the GPU) and is asynchronous on `stream` (a hipStream_t, NULL =
 *     the null stream); hvp_solve_batch_host takes host pointers and is synchronous.
 *   - Return value: 0 = ok, < 0 = error (HVP_E_*); the message is kept per thread and read
 *     with hvp_last_error().  No exception crosses the ABI.
 *   - One handle per host thread / stream; handles are independent.
 *   - All arithmetic is IEEE float64.  Region indices are 0-based; gears are the 1-based
 *     labels given in hvp_system.gear (PwaGearVehicle: 1,2,3,4,4,5,6).
 */
#ifndef HVP_H
#define HVP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HVP_ABI_VERSION 5
#define HVP_MAX_REGIONS 16
#define HVP_MAX_N 16     /* longest horizon (branch-and-bound path)            */
#define HVP_MAX_N_ENUM 8 /* longest horizon of the exhaustive-enumeration path */

/* Discrete-time PWA model of one vehicle, velocity-partitioned (the form every system dict of
 * models.py:370-492 has): region r holds for vlo[r] <= v <= vhi[r] (closed; overlapping
 * boundaries are feasible for both regions, as in the MLD big-M model) and then
 *     p+ = p + ts * v,        v+ = a[r] * v + b[r] * u + c[r].
 * hvp/tables.py builds it from the reference's {S,R,T,A,B,c,D,E,F,G} dict and rejects any dict
 * that is not of that form. */
typedef struct hvp_system {
    int32_t n_regions;
    int32_t gear[HVP_MAX_REGIONS]; /* gear label of each region                       */
    int32_t pad_;
    double ts;                     /* Ad[0][1]                                          */
    double a[HVP_MAX_REGIONS];     /* Ad[1][1]                                          */
    double b[HVP_MAX_REGIONS];     /* Bd[1][0]  (> 0)                                   */
    double c[HVP_MAX_REGIONS];     /* cd[1][0]                                          */
    double vlo[HVP_MAX_REGIONS];   /* region velocity interval (+-1e300 = unbounded)    */
    double vhi[HVP_MAX_REGIONS];
    double pmin, pmax, vmin, vmax; /* D x <= E, applied for k = 1..N                    */
    double umin, umax;             /* F u <= G, applied for k = 0..N-1                  */
} hvp_system;

/* Cost and constraint constants shared by every local MPC of one controller
 * (misc/common_controller_params.py:14-23, fleet_decent_mld.py:61-208). */
typedef struct hvp_problem {
    int32_t N;              /* prediction horizon (2..HVP_MAX_N)                      */
    int32_t quadratic_cost; /* 1 = min_2_norm (MIQP); 0 = min_1_norm (MILP,
                               fleet_decent_mld.py:73-76, mpcs/cent_mld.py:58-61):
                               HVP_FORM_DECENT, any N, by branch and bound over node LPs (AUTO /
                               BNB) or enumeration (ENUMERATE, N <= HVP_MAX_N_ENUM), LPs by
                               the per-lane simplex of csrc/hvp_lp.h (N <= 8) or the
                               interior point of csrc/hvp_l1.h; HVP_FORM_CENT, the platoon LP inside the joint
                               branch and bound (csrc/hvp_cent_l1.h; AUTO / BNB, or ENUMERATE =
                               the exhaustive joint search).  Every LP ends solved, proven
                               infeasible (excluded), or unresolved -- which makes its instance /
                               platoon HVP_MAXITER while it is still in contention.
                               HVP_FORM_ADMM (LocalMpcADMM(quadratic_cost=False),
                               fleet_naive_admm.py:74-77): L1 terms next to the quadratic ADMM
                               terms of the copies -- the node QPs by the wave interior point with
                               the copies as variables (csrc/hvp_lane.h L1AdmmWave), branch and
                               bound.  HVP_FORM_GADMM: HVP_E_UNSUPPORTED */
    double Qx[4];           /* 2x2 row-major state-tracking weight                     */
    double Qu;              /* control weight                                          */
    double Qdu;             /* control-variation weight                                */
    double w;               /* slack weight                                            */
    double a_acc, a_dec;    /* acceleration limits (per unit of ts_acc)                */
    double ts_acc;          /* Params.ts used in the accel rows                        */
    double d_safe;          /* safe distance                                           */
    double accel_tightening;
    double spacing_d0;      /* spacing(x) = [-d0 - t0 * v, 0]                          */
    double spacing_t0;
    int32_t max_iter;       /* fallback IPM iteration cap per candidate (<=0: 60);
                               min_1_norm: the LP solver's cap -- simplex pivots or
                               interior-point iterations (<=0: 120)                   */
    int32_t method;         /* HVP_METHOD_*: how the region sequences are searched     */
    double tol;             /* fallback IPM relative tolerance (<=0: 1e-12)            */
    int32_t formulation;    /* HVP_FORM_*: which local MPC (parameter layout, cost)    */
    int32_t pad_;
    double rho;             /* ADMM penalty (HVP_FORM_ADMM; fleet_naive_admm.py:600)   */
} hvp_problem;

/* Local MPC formulation (hvp_problem.formulation). */
enum {
    HVP_FORM_DECENT = 0, /* LocalMpcMld (fleet_decent_mld.py:21-223): fixed neighbour predictions   */
    HVP_FORM_ADMM = 1,   /* LocalMpcADMM (fleet_naive_admm.py:24-253): neighbour COPIES as decision
                            variables with ADMM terms y'(c - z) + rho/2 |c - z|^2; needs B&B      */
    HVP_FORM_GADMM = 2,  /* fleet_g_admm.LocalMpc (:22-205) under MpcSwitching [EXT]: convex QP for
                            a GIVEN region sequence; own state and copies in the augmented
                            Lagrangian; solved by hvp_gadmm_solve only                          */
    HVP_FORM_CENT = 3    /* MpcMldCent (mpcs/cent_mld.py:21-182): ONE MIQP over the whole platoon;
                            solved by hvp_cent_solve_batch only                                  */
};

/* Search over the region sequences (hvp_problem.method).  Both give the same sequence: the
 * exact argmin with ties to the lexicographically first sequence (DESIGN.md "Algorithm"). */
enum {
    HVP_METHOD_AUTO = 0,      /* branch and bound (measured faster from N = 5 on)          */
    HVP_METHOD_ENUMERATE = 1, /* every velocity-feasible sequence (N <= HVP_MAX_N_ENUM)     */
    HVP_METHOD_BNB = 2        /* branch and bound with horizon-relaxed QP bounds             */
};

/* Role of one local MPC (is_front / is_trailer / is_leader / real_vehicle_as_reference). */
enum {
    HVP_ROLE_SAFE_FRONT = 1,     /* not is_front : p_k - s_f,k <= pf_k - d_safe, s_f >= 0  */
    HVP_ROLE_SAFE_BACK = 2,      /* not is_trailer: p_k + s_b,k >= pb_k + d_safe, s_b >= 0 */
    HVP_ROLE_TRACK_FRONT = 4,    /* not is_front and not is_leader                         */
    HVP_ROLE_TRACK_BACK = 8,     /* not is_trailer and not is_leader                       */
    HVP_ROLE_TRACK_LEADER = 16,  /* is_leader                                              */
    HVP_ROLE_LEADER_SPACING = 32,/* is_leader and real_vehicle_as_reference                */
    HVP_ROLE_BACK_COPY = 64      /* HVP_FORM_GADMM: holds a copy of the vehicle behind (ADMM term
                                    only; G[i] contains i + 1, fleet_g_admm.py:341-353)     */
};

/* Per-instance status (Gurobi Status 2 <-> HVP_OPTIMAL). */
enum {
    HVP_OPTIMAL = 0,
    HVP_INFEASIBLE = 1,      /* no region sequence is feasible                          */
    HVP_MAXITER = 2,         /* no candidate converged within max_iter                  */
    HVP_OVERFLOW = 3         /* candidate workspace exhausted (raise hvp_reserve)        */
};

/* Error codes. */
enum {
    HVP_OK = 0,
    HVP_E_ARG = -1,
    HVP_E_HIP = -2,
    HVP_E_UNSUPPORTED = -3,
    HVP_E_NOMEM = -4
};

/* Instance parameter block, stride hvp_params_stride(N) doubles:
 *   [0..1]                x0 = (p0, v0)                      (solve_mpc(state))
 *   [2 .. 2+2(N+1))       x_front (2, N+1) row-major          (set_x_front)
 *   next 2(N+1)           x_back  (2, N+1) row-major          (set_x_back)
 *   next 2(N+1)           leader_x (2, N+1) row-major         (set_leader_x)
 * Blocks a role does not use are ignored. */
static inline int hvp_params_stride(int N) { return 2 + 6 * (N + 1); }

/* HVP_FORM_ADMM parameter block, stride hvp_params_stride_admm(N) doubles:
 *   [0..1] x0 | y_front | z_front | y_back | z_back | leader_x   (each (2, N+1) row-major)
 * (set_front_vars / set_back_vars / set_leader_x, fleet_naive_admm.py:239-258). */
static inline int hvp_params_stride_admm(int N) { return 2 + 10 * (N + 1); }

/* HVP_FORM_GADMM parameter block, stride hvp_params_stride_gadmm(N) doubles:
 *   [0..1] x0 | y_front | z_front | y_back | z_back | leader_x | y_own | z_own  (each (2, N+1))
 * i.e. the ADMM block plus the own-state multiplier / consensus value (MpcAdmm's augmented state
 * [EXT]: the y / z parameters of fleet_g_admm.LocalMpc cover own state and copies). */
static inline int hvp_params_stride_gadmm(int N) { return 2 + 14 * (N + 1); }

typedef struct hvp_handle hvp_handle;

typedef struct hvp_stats {
    int64_t n_instances;    /* instances in the last solve                            */
    int64_t n_candidates;   /* region sequences (QPs) solved in the last solve         */
    int64_t qp_iterations;  /* sum of QP iterations (active-set + fallback IPM)      */
    int64_t capacity;       /* candidate workspace                                     */
    double last_ms;         /* device time of the last solve (event-timed), ms         */
    double qp_ms;           /* device time of its QP kernel (K_qp), ms                 */
    int64_t n_fallback;     /* candidates re-solved by the interior-point fallback    */
    int64_t n_failed_bounds;/* B&B bound QPs that did not converge (they prune nothing) */
    int64_t n_spilled;      /* B&B child reservations placed in another level bucket   */
} hvp_stats;

int hvp_create(hvp_handle** out, const hvp_problem* problem, const hvp_system* systems,
               int n_systems, int device);
/* Workspace for batches up to max_batch.  candidate_capacity (<= 0: a default per method) is, for
 * branch and bound, the node capacity of ONE tree level pooled over the batch.  The decentralised
 * min_2_norm lane path (N <= 8) keeps every level in 2 buckets (HVP_SPLIT_LEVELS: 1, 2 or 4) of
 * capacity / buckets nodes each; children that do not fit their bucket spill into another
 * bucket's free segment (hvp_stats.n_spilled).  An instance whose children fit nowhere is reported
 * HVP_OVERFLOW (never truncated) and can be re-solved alone with a larger reserve. */
int hvp_reserve(hvp_handle* h, int max_batch, int64_t candidate_capacity);
/* Device-pointer entry point (async on stream).  Outputs may be NULL except cost/status. */
int hvp_solve_batch(hvp_handle* h, int B, const int32_t* sys, const int32_t* role,
                    const double* params, double* u_out, double* x_out, int8_t* region_out,
                    int8_t* gear_out, double* cost_out, int32_t* status_out,
                    int32_t* nodes_out, int32_t* iters_out, void* stream);
/* Host-pointer entry point (copies in, solves, copies out, synchronises). */
int hvp_solve_batch_host(hvp_handle* h, int B, const int32_t* sys, const int32_t* role,
                         const double* params, double* u_out, double* x_out,
                         int8_t* region_out, int8_t* gear_out, double* cost_out,
                         int32_t* status_out, int32_t* nodes_out, int32_t* iters_out);
/* HVP_FORM_ADMM solve: as hvp_solve_batch, plus the optimal neighbour copies the coordinator
 * reads as mpc.x_front.X / mpc.x_back.X (fleet_naive_admm.py:413-446): xf_out, xb_out
 * [B][2][N+1] (may be NULL; zero for a side the role does not have). */
int hvp_solve_admm_batch(hvp_handle* h, int B, const int32_t* sys, const int32_t* role,
                         const double* params, double* u_out, double* x_out, int8_t* region_out,
                         int8_t* gear_out, double* cost_out, int32_t* status_out, int32_t* nodes_out,
                         int32_t* iters_out, double* xf_out, double* xb_out, void* stream);

/* Region sequence hint for the HVP_FORM_ADMM solves of this handle and its HVP_FORM_DECENT
 * solves with N > 8: device pointer region_hint[B][N] (int8, e.g. the region_out of the previous
 * ADMM iteration, or the previous time step's sequences shifted by one step; NULL clears it),
 * read at the start of every later solve.  Instance i's hinted sequence, when it is
 * velocity-feasible, is solved as a second initial incumbent next to the greedy dive; it only
 * tightens pruning (prune margin 1e-7 > tie window 1e-9), the answer does not depend on it, and
 * nodes_out counts its QP.  The pointer must stay valid while solves may read it. */
int hvp_set_region_hint(hvp_handle* h, const int8_t* region_hint);

/* Naive-ADMM node records (HVP_FORM_ADMM, 8 < N <= 12): every branch-and-bound node
 * QP of instance i keeps its final active set and factors for the same node of instance i in the
 * next solve of this handle, which warm-starts from them (same answers to rounding; repeated runs
 * bit-identical).  On by default (HVP_ADMM_NODE_SLOTS records per instance and depth, 0: off).
 * The records are indexed by batch position like the region hint: a caller that re-solves a
 * subset of its batch (an overflow retry) turns them off for that solve (enable = 0), so the
 * subset neither reads nor overwrites the batch's records.  An instance whose search overflows
 * leaves no record behind. */
int hvp_set_node_records(hvp_handle* h, int enable);

/* ADMM z- and y-update of ADMMCoordinator.get_control (fleet_naive_admm.py:421-468) for P
 * platoons of n vehicles (instance p*n + i), device pointers, async on stream:
 *   z_i = mean of x_i, vehicle (i+1)'s front copy and vehicle (i-1)'s back copy;
 *   y_front_{i+1} += rho (xf_{i+1} - z_i);  y_back_{i-1} += rho (xb_{i-1} - z_i);
 * then writes every vehicle's next parameter blocks  (y_front_i, z_{i-1}) and (y_back_i, z_{i+1})
 * into params (HVP_FORM_ADMM layout) and z into z_out [P*n][2][N+1] (may be NULL).
 * y_front / y_back [P*n][2][N+1] are updated in place. */
int hvp_admm_update(hvp_handle* h, int P, int n, const double* x, const double* xf, const double* xb,
                    double* y_front, double* y_back, double* params, double* z_out, void* stream);

/* Cost of FIXED controls (device pointers, async on stream): replaces MpcGear.evaluate_cost
 * (mpcs/mpc_gear.py:137-170).  gear_in[B][N] = gear label per step (for the 7-region gear model
 * the label of the region the velocity lies in), u_in[B][N] = the control (u_g for the gear
 * model).  cost_out = objective of the resulting trajectory with optimal slacks, status_out =
 * HVP_OPTIMAL or HVP_INFEASIBLE (a constraint of the MLD model is violated; the reference returns
 * the string 'inf').  x_out[B][2][N+1] (may be NULL) receives the trajectory. */
int hvp_evaluate_batch(hvp_handle* h, int B, const int32_t* sys, const int32_t* role, const double* params,
                       const int8_t* gear_in, const double* u_in, double* cost_out, int32_t* status_out,
                       double* x_out, void* stream);
/* ---- Switching ADMM (fleet_g_admm.py: TrackingGAdmmCoordinator over GAdmmCoordinator /
 * MpcSwitching of dmpcpwa [EXT]; the restated rule is documented in DESIGN.md and
 * oracle/oracle.py GAdmmCoordinator).  Layout: P platoons of n vehicles; a process holds the
 * vehicles [lo, lo + m) of every platoon (m = n unsharded), instance b = p * m + (i - lo).
 * Trajectory arrays x / xf / xb are FULL-platoon [P][n][2][N+1] (vehicle slot p * n + i):
 * the solve writes the held vehicles' slots, a sharded caller fills the neighbouring slots
 * (halo) before hvp_gadmm_update.  state[P] (int32, device): bit 0 = still iterating (live),
 * bit 1 = failed (a rollout or local QP failed: the reference's error / infeasibility flag),
 * bit 2 = sequence changed in the last hvp_gadmm_switch. */

/* Warm start (fleet_g_admm.py:256-272): mode 0 = constant-velocity throttle of each vehicle's
 * v0 (Vehicle.get_u_for_constant_vel, models.py:537-556), mode 1 = u_prev [B][N] shifted by one
 * step (last column repeated).  Rolls the controls out through the PWA dynamics (region = first
 * closed velocity band holding v_k) from x0 = params[b][0..1]: x [P][n][2][N+1] slots, seq
 * [B][N] regions, u_ws [B][N] (may be NULL).  A velocity in no band sets state bit 1. */
int hvp_gadmm_rollout(hvp_handle* h, int P, int n, int lo, int m, const int32_t* sys, const double* params,
                      int mode, const double* u_prev, double* x, int8_t* seq, double* u_ws, int32_t* state,
                      void* stream);
/* One ADMM x-update: the local QP of every held vehicle of every live platoon for its sequence
 * seq [B][N].  Writes u_out [B][N], the vehicle's trajectory / optimal copies into the x / xf /
 * xb slots, cost_out [B] (the local objective incl. ADMM terms: sol.f), status_out [B],
 * edge_out [B] (bit 2(k-1) + 0/1: the lower / upper velocity edge of region seq_k, k = 1..N-1,
 * strictly inside the state box, is active with multiplier > 1e-6), iters_out [B] (may be
 * NULL).  A failed QP sets state bit 1 of its platoon and clears bit 0. */
int hvp_gadmm_solve(hvp_handle* h, int P, int n, int lo, int m, const int32_t* sys, const int32_t* role,
                    const double* params, const int8_t* seq, int32_t* state, double* u_out, double* x,
                    double* xf, double* xb, double* cost_out, int32_t* status_out, uint32_t* edge_out,
                    int32_t* iters_out, void* stream);
/* z- and y-update (consensus over G[i] = {i-1, i, i+1}):  z_j = mean(x_j, xb_{j-1}, xf_{j+1}),
 * y_own_i += rho (x_i - z_i), y_front_i += rho (xf_i - z_{i-1}), y_back_i += rho (xb_i - z_{i+1}),
 * and the z blocks of params <- z_i, z_{i-1}, z_{i+1}; for live platoons only.  init != 0
 * starts an ADMM run: z_j <- x_j (the rollout), every y <- 0. */
int hvp_gadmm_update(hvp_handle* h, int P, int n, int lo, int m, const double* x, const double* xf,
                     const double* xb, double* params, const int32_t* state, int init, void* stream);
/* Sequence switching after an ADMM run (live platoons): seq_k moves across every edge flagged
 * in edge [B] into the region on the other side; sets state bit 2 when a sequence changed. */
int hvp_gadmm_switch(hvp_handle* h, int P, int n, int lo, int m, const int32_t* sys, const uint32_t* edge,
                     int8_t* seq, int32_t* state, void* stream);
/* ---- Centralised MLD (mpcs/cent_mld.py MpcMldCent, fleet_cent_mld.py): replaces
 * MpcMldCent.__init__ + setup_cost_and_constraints (:21-177; the handle, formulation
 * HVP_FORM_CENT, and leader_index / real_vehicle_as_reference here), set_leader_traj (:179-182;
 * leader_x) and MldAgent.get_control -> solve_mpc -> Model.optimize() (fleet_cent_mld.py:183) for
 * P independent platoons of n vehicles in one call (device pointers, async on stream):
 *   sys [P*n] system index of vehicle i of platoon p at p*n + i; x0 [P][n][2] (p, v);
 *   leader_x [P][2][N+1] the leader window; n*N <= 64; real_vehicle_as_reference needs
 *   leader_index == 0 (the reference raises NotImplementedError otherwise, :63-66).
 * Exact branch and bound over the joint region sequence (time-major), ties to the
 * lexicographically first sequence in that order; hvp_problem.method == HVP_METHOD_ENUMERATE
 * visits every velocity-feasible joint sequence instead (cross-check, tiny instances only).
 * max_nodes (<= 0: 2000000) caps the QPs per platoon; a platoon that reaches it is HVP_MAXITER
 * (a split search, below, checks the cap per subtree task, so it may overshoot by the tasks in
 * flight).  A platoon whose search passes 1000 QPs is SPLIT: its open DFS frames become subtree
 * tasks that rounds of one kernel spread over every wave of the device (sharing the platoon's
 * incumbent); a final kernel applies the tie rule to the merged near-optimal leaves.  The answer
 * is the same; the QP count of a split platoon is not the sequential search's.  The call then
 * synchronises the stream once per round (it reads the number of tasks left).
 * Outputs: u [P][n][N], x [P][n][2][N+1] (may be NULL), region / gear [P][n][N] int8 (may be
 * NULL), cost [P], status [P], nodes [P] (QPs solved, Gurobi NodeCount analogue), iters [P] (may
 * be NULL).  Workspace grows on demand (one synchronisation when it does).  HVP_CENT_SPLIT=0 in
 * the environment disables the split (HVP_CENT_SPLIT=k: split past k QPs). */
int hvp_cent_solve_batch(hvp_handle* h, int P, int n, int leader_index, int real_vehicle_as_reference,
                         const int32_t* sys, const double* x0, const double* leader_x, int max_nodes,
                         double* u_out, double* x_out, int8_t* region_out, int8_t* gear_out,
                         double* cost_out, int32_t* status_out, int32_t* nodes_out, int32_t* iters_out,
                         void* stream);
/* ---- Plant step (the caller side of the hot path, env.py PlatoonEnv.step + get_stage_cost,
 * models.py Platoon.step_platoon) for P platoons of n vehicles (device pointers, async):
 *   x [P][2n] (p, v per vehicle) advanced IN PLACE by ts with 10 explicit Euler sub-steps of the
 *   nonlinear vehicle model (models.py:114-125, 236-257); masses [P][n]; u [P][n] the throttle;
 *   gear [P][n] int8 from the action, or NULL / entries <= 0: the PWA-gear model's gear of the
 *   current velocity (env.py:198-204, models.py:494-515); u_prev [P][n] the previous action
 *   (= u on the first step, env.py:127-128); leader_x [P][2] the leader state of this step.
 * Outputs: cost [P] the stage cost of (x, u) before the step (env.py:126-180: quad_cost, or
 * lin_cost = ||Q e||_1 when the handle's problem has quadratic_cost = 0, env.py:118-124; the
 * env's own weights, the handle's spacing / d_safe), viol [P] 100 when a gap is below d_safe (else 0),
 * status [P] 0 ok, 1 a velocity left the traction curve (the reference raises RuntimeError). */
int hvp_env_step_batch(hvp_handle* h, int P, int n, const double* masses, double* x, const double* u,
                       const int8_t* gear, const double* u_prev, const double* leader_x, int leader_index,
                       int real_vehicle_as_reference, double ts, double* cost_out, int32_t* viol_out,
                       int32_t* status_out, void* stream);
/* Neighbour predictions of TrackingDecentMldCoordinator.observe_states (fleet_decent_mld.py:348-455)
 * for P platoons (device pointers, async): x [P][2n] the measured states, x_prev [P][2n] the
 * previous ones (NULL: x; read by the two-point estimators), leader_x [P][2][N+1] the leader
 * window; estimator 0 constant velocity (:421-428), 1 two_point (:430-440), 2 sat (:442-455).
 * Writes params [P*n][hvp_params_stride(N)] and roles [P*n] (instance p*n + i), the input of
 * hvp_solve_batch.  HVP_FORM_DECENT handles (their N and ts). */
int hvp_decent_params_batch(hvp_handle* h, int P, int n, const double* x, const double* x_prev,
                            const double* leader_x, int leader_index, int real_vehicle_as_reference, int estimator,
                            double* params, int32_t* roles, void* stream);
int hvp_sync(hvp_handle* h, void* stream);
int hvp_get_stats(hvp_handle* h, hvp_stats* out); /* synchronises the handle's last stream */
void hvp_destroy(hvp_handle* h);
int hvp_last_error(char* buf, size_t len);
int hvp_abi_version(void);
/* sizes[0..2] = sizeof(hvp_system), sizeof(hvp_problem), sizeof(hvp_stats) (binding checks). */
int hvp_abi_sizes(int32_t* sizes);

#ifdef __cplusplus
}
#endif

#endif /* HVP_H */
