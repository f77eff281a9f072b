// hvp_internal.h -- definitions shared by the translation units of libhvpsolve.so
// (hvp_kernels.hip: decentralised / ADMM paths and the common C ABI; hvp_cent.hip: the
// centralised MLD path).  Not part of the public ABI (include/hvp.h).
#pragma once

#include <hip/hip_runtime.h>

#include <string>

#include "hvp.h"
#include "hvp_ipm.h"

namespace hvp {
namespace cent {
struct Child;  // hvp_cent_bnb.h (only the centralised unit needs its layout)
}  // namespace cent
}  // namespace hvp

namespace hvp_detail {

// sets the thread's last-error text (hvp_last_error) and returns code
int fail(int code, const std::string& msg);

#define HIP_TRY(expr)                                                                                     \
    do {                                                                                                  \
        hipError_t e_ = (expr);                                                                           \
        if (e_ != hipSuccess) return hvp_detail::fail(HVP_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

struct Workspace {
    int max_batch = 0;
    int64_t cap = 0;
    int32_t* inst_off = nullptr;   // [max_batch] first candidate slot (-1: overflow)
    int32_t* inst_cnt = nullptr;   // [max_batch] candidates of the instance
    int32_t* inst_flag = nullptr;  // [max_batch] 0 ok, 1 infeasible constant rows
    unsigned long long* counter = nullptr;  // [8] reserved slots, qp iterations, fallback count, root QPs, failed bounds
    int32_t* redo = nullptr;       // [cap] candidates the active-set method hands to the IPM
    int32_t* task_inst = nullptr;  // [cap]
    uint32_t* task_code = nullptr; // [cap]
    double* task_cost = nullptr;   // [cap]
    int32_t* task_stat = nullptr;  // [cap] status | iters << 8
    double* task_y = nullptr;      // [cap * N]
    // branch and bound (hvp_bnb.h): two node lists (parents / children of a level, ping-pong),
    // per-instance incumbent and winner key
    int32_t* nd_inst[2] = {nullptr, nullptr};    // [cap] owning instance (-1: dead)
    uint64_t* nd_code[2] = {nullptr, nullptr};   // [cap] region prefix, 4 bits per step
    double* nd_lo[2] = {nullptr, nullptr};       // [cap] reachable interval of v_depth
    double* nd_hi[2] = {nullptr, nullptr};
    double* nd_lb[2] = {nullptr, nullptr};       // [cap] bound (relaxed QP) or leaf cost
    int32_t* leaf_stat = nullptr;                // [cap] 0 ok, else the QP failed
    unsigned long long* inc = nullptr;           // [max_batch] incumbent cost (bits of a double >= 0)
    unsigned long long* key = nullptr;           // [max_batch] lexicographic key of the winner
    int32_t* nodes = nullptr;                    // [max_batch] QPs solved for the instance
    int32_t* iters = nullptr;                    // [max_batch] active-set iterations
    unsigned long long* lvl = nullptr;           // [6 (HVP_MAX_N + 1)], M = HVP_MAX_N + 1 rows per block:
                                                 // [0, M) nodes per level (bucket 0's count), [M, 2M)
                                                 // the refill kernels' per-level claim counters, [2M, 5M)
                                                 // buckets 1..3's counts (hvp_lane.h LevelList), [5M, 6M)
                                                 // free.  k_node_order (16-lane naive ADMM) keeps its
                                                 // per-level counters at rows 2M and 5M: bucket 1's
                                                 // count row, unused there because that path runs at
                                                 // split = 1 (launch_bnb: split > 1 only when fused)
    double* iq = nullptr;                        // [max_batch][fields, padded to 16] sigma-independent QP
                                                 // part per instance (decentralised branch and bound, N <= 8)
    const int8_t* hint = nullptr;                // [B][N] regions of a previous solve of the same
                                                 // instances (hvp_set_region_hint; ADMM form only)
    // the greedy dive's leaf of every instance (decentralised lane path, N <= 8): a node list of
    // its own, solved by the refill kernel after the root level (hvp_lane.h launch_bnb)
    int32_t* dv_inst = nullptr;                  // [3 max_batch] instance (-1: no dive); the
                                                 // min_1_norm search lists up to 3 per instance
    uint64_t* dv_code = nullptr;                 // [max_batch] the dive's sequence
    double* dv_lo = nullptr;                     // [max_batch] (unused at K = N: 0)
    double* dv_hi = nullptr;                     // [max_batch] (-1)
    double* dv_lb = nullptr;                     // [max_batch] leaf cost
    int32_t* dv_stat = nullptr;                  // [max_batch]
    double* dv_y = nullptr;                      // [max_batch * N]
    int32_t* dv_redo = nullptr;                  // [max_batch] (failed dives are not re-solved)
    unsigned long long* dv_lvl = nullptr;        // [(2 + 4)(HVP_MAX_N + 1)] counts / claims of the dive list
    unsigned long long* dv_counter = nullptr;    // [8]
    char* dv_mem = nullptr;                      // the allocation the dv_* arrays live in
    int split = 1;                               // buckets per level list (hvp_lane.h LevelList; > 1
                                                 // per launch for the decentralised lane path)
    int split_shift = 0;                         // log2(split): a bucket's segment is cap >> split_shift
    int pass = 0;                                // pass-through nodes (hvp_lane.h bnb_put_children;
                                                 // HVP_PASS_THROUGH=1 turns them on, launch_bnb)
    // naive-ADMM node records (16-lane path, 8 < N <= 12; hvp_lane.h node_index): the final hinge
    // states, active set and factors of every tree node's QP, for the same node in the next solve
    void* nrec = nullptr;                        // [max_batch][N + 1][nslots] hvp::coop::WarmRec<N>
    unsigned long long* nclaim = nullptr;        // [max_batch][N + 1][nslots] owner priority (node_prio)
    int nslots = 0;                              // records per (instance, depth), a power of two; 0: none
    int ndepth = 0;                              // N + 1
    unsigned long long nepoch = 0;               // this solve's epoch << 48
    int norder = 0;                              // k_bnb_bound_coop takes the level in k_node_order's order
    int32_t* win = nullptr;                      // [max_batch] the winning leaf's slot in level N's list
                                                 // (k_bnb_write), read by k_bnb_finish, which writes
                                                 // every per-instance output in instance order
};


}  // namespace hvp_detail

struct hvp_handle {
    int device = 0;
    hvp_problem prob{};
    hvp::Consts C{};
    int n_systems = 0;
    hvp_system* d_sys = nullptr;
    hvp_detail::Workspace ws;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;  // around the whole solve
    hipEvent_t evq0 = nullptr, evq1 = nullptr; // around K_qp (the dominant kernel)
    hipEvent_t evb[2 * (HVP_MAX_N + 1)] = {};    // B&B: around K_bnb_root and every K_bnb_bound
    hipStream_t last_stream = nullptr;
    int last_B = 0;
    bool bnb = false;       // search method resolved at hvp_create (HVP_METHOD_*)
    bool last_bnb = false;
    int last_split = 1;  // buckets of the last B&B solve's level lists (Workspace::split)
    int n_cu = 256;
    // host-pointer entry point staging (grown on demand)
    size_t stage_bytes = 0;
    char* d_stage = nullptr;
    unsigned long long* g_counter = nullptr;  // [8] switching-ADMM / centralised counters (QP iterations at [1])
    // centralised MLD (hvp_cent_solve_batch): per-platoon DFS child slices and tie-rule rows
    int nreg_max = 1;
    size_t cent_frames_bytes = 0, cent_ties_bytes = 0;
    hvp::cent::Child* cent_frames = nullptr;
    uint64_t* cent_ties = nullptr;
    hvp::Consts* d_consts = nullptr;  // device copy of C (the centralised kernel reads it by pointer)
    size_t cent_split_bytes = 0;      // split-search workspace of the centralised path (hvp_cent.hip)
    // switching ADMM: every local QP's final hinge states, active set and factors (hvp_coop.h
    // WarmQp), the next ADMM iteration's start; not used after hvp_gadmm_rollout (a new warm start)
    void* gadmm_hs = nullptr;
    long long gadmm_hs_cap = 0;
    int gadmm_hs_valid = 0;
    int32_t* gadmm_redo = nullptr;  // local QPs for the interior-point fallback (k_gadmm_ipm)
    long long gadmm_redo_cap = 0;
    char* cent_split = nullptr;
    const int8_t* region_hint = nullptr;  // hvp_set_region_hint (copied into ws.hint per solve)
    // naive-ADMM node records (Workspace::nrec), allocated at the first solve for the reserve
    void* nrec = nullptr;
    unsigned long long* nclaim = nullptr;
    long long nrec_batch = 0;   // batch the records were sized for (also set after a failed
                                // allocation, so the next solve does not try again)
    int nrec_want = 0;          // slots requested (HVP_ADMM_NODE_SLOTS, rounded to a power of two)
    int nrec_slots = 0;         // slots allocated (nrec_want, halved until it fits the free HBM)
    unsigned long long nrec_epoch = 0;
    bool nrec_enable = true;  // hvp_set_node_records
    // device copies of the workspace descriptors the refill kernel reads in its event code
    // (hvp_lane.h k_bnb_bound_refill): [0] the level lists, [1] the dive list; re-uploaded when
    // they change (a reserve, another bucket split)
    hvp_detail::Workspace* d_ws = nullptr;
    hvp_detail::Workspace ws_up[2];
    bool ws_up_valid = false;
};
