"""Diagnostic (round 5): per-phase clocks of the 16-lane QP (hvp_coop.h solve_qp / solve) in
k_bnb_bound_coop, for a variant build only.  Applies the instrumentation to the sources in place;
build with profiles/build_variant.sh coopprof "-DHVP_COOP_PROF", then restore the sources (git
checkout).  Each group's lane 0 adds s_memtime deltas per phase to its LDS pad; the kernel flushes
them into g_cp once per group; hvp_get_stats prints and clears them ([coop-prof] on stderr).

    python profiles/diag_coop_prof_patch.py
"""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
C = os.path.join(ROOT, "hybrid-vehicle-platoon_amd", "csrc")


def edit(path, pairs):
    s = open(path).read()
    for a, b in pairs:
        assert s.count(a) == 1, (path, a[:60], s.count(a))
        s = s.replace(a, b)
    open(path, "w").write(s)


coop = os.path.join(C, "hvp_coop.h")
edit(coop, [
    ("""__device__ inline int lane16() { return (int)(threadIdx.x & (G - 1)); }""",
     """__device__ inline int lane16() { return (int)(threadIdx.x & (G - 1)); }
#define CP_NOW() __builtin_amdgcn_s_memtime()
#define CP_ADD(Sg, slot, t0) do { if (lane16() == 0) (Sg).pad[slot] += (double)(CP_NOW() - (t0)); } while (0)"""),
    ("""    int warmed = WARM_COLD;
    if (wq && wtry && wq->valid && wq->code == wcode && wq->hs == whs && wq->key == wkey)  // group-uniform
        warmed = warm_start<N, W>(L, Sg, C, wq, u, id, act, nact);""",
     """    int warmed = WARM_COLD;
    unsigned long long cp0 = CP_NOW();
    if (wq && wtry && wq->valid && wq->code == wcode && wq->hs == whs && wq->key == wkey)  // group-uniform
        warmed = warm_start<N, W>(L, Sg, C, wq, u, id, act, nact);
    CP_ADD(Sg, 3, cp0);
    if (lane16() == 0 && warmed == WARM_OK) Sg.pad[10] += 1.0;
    cp0 = CP_NOW();"""),
    ("""    unsigned sat = 0;  // saturation bits (SF = 1, SB = 2) of lane t's prefix rows""",
     """    CP_ADD(Sg, 4, cp0);
    cp0 = CP_NOW();
    unsigned sat = 0;  // saturation bits (SF = 1, SB = 2) of lane t's prefix rows"""),
    ("""    // ---- verification: multipliers in [0, w] (soft) or >= 0""",
     """    CP_ADD(Sg, 5, cp0);
    cp0 = CP_NOW();
    // ---- verification: multipliers in [0, w] (soft) or >= 0"""),
    ("""        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        gsync();
    }
    return ok ? GI_OK : GI_FAIL_VERIFY;""",
     """        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        gsync();
    }
    CP_ADD(Sg, 6, cp0);
    return ok ? GI_OK : GI_FAIL_VERIFY;"""),
    ("""                const bool from_rec = w && wq->code == code && wq->hs == hs && wq->key == wkey;
                setup<N>(L, Sg, S, C, role, prm, code, K, hs, 0.0, -1.0, !from_rec);
                int it = 0;""",
     """                const bool from_rec = w && wq->code == code && wq->hs == hs && wq->key == wkey;
                unsigned long long cq = CP_NOW();
                setup<N>(L, Sg, S, C, role, prm, code, K, hs, 0.0, -1.0, !from_rec);
                CP_ADD(Sg, 1, cq);
                int it = 0;"""),
    ("""                bool consistent;
                hs = admm_classify_group<N>(L, C, role, prm, hs, &consistent);
                if (consistent) {
                    *cost = direct_cost_admm<N>(L, S, C, role, prm, code, K);
                    return GI_OK;
                }""",
     """                bool consistent;
                cq = CP_NOW();
                hs = admm_classify_group<N>(L, C, role, prm, hs, &consistent);
                CP_ADD(Sg, 7, cq);
                if (consistent) {
                    cq = CP_NOW();
                    *cost = direct_cost_admm<N>(L, S, C, role, prm, code, K);
                    CP_ADD(Sg, 8, cq);
                    return GI_OK;
                }"""),
])
lane = os.path.join(C, "hvp_lane.h")
edit(lane, [
    ("""    const unsigned long long nn = ws.lvl[k];
    const long long total = (long long)(nn < (unsigned long long)ws.cap ? nn : ws.cap);
    for (long long q0 = (long long)blockIdx.x * kCoopGroups + g; q0 < total; q0 += (long long)gridDim.x * kCoopGroups) {""",
     """    const unsigned long long nn = ws.lvl[k];
    const long long total = (long long)(nn < (unsigned long long)ws.cap ? nn : ws.cap);
    if (t < hvp::coop::G) lds[g].pad[t] = 0.0;
    hvp::coop::gsync();
    for (long long q0 = (long long)blockIdx.x * kCoopGroups + g; q0 < total; q0 += (long long)gridDim.x * kCoopGroups) {
        const unsigned long long cpn = CP_NOW();"""),
    ("""        const int st = hvp::coop::solve_qp<N, Rec>(L, lds[g], S, C, rl, prm, code, k, cap, it, &c, nullptr,
                                                   ws.nd_lo[dst][q], ws.nd_hi[dst][q], wq, wq != nullptr,
                                                   ((uint64_t)(uint32_t)sys[inst] << 32) | (uint32_t)rl);""",
     """        const unsigned long long cps = CP_NOW();
        if (t == 0) lds[g].pad[11] += (double)(cps - cpn);
        const int st = hvp::coop::solve_qp<N, Rec>(L, lds[g], S, C, rl, prm, code, k, cap, it, &c, nullptr,
                                                   ws.nd_lo[dst][q], ws.nd_hi[dst][q], wq, wq != nullptr,
                                                   ((uint64_t)(uint32_t)sys[inst] << 32) | (uint32_t)rl);
        if (t == 0) { lds[g].pad[0] += (double)(CP_NOW() - cps); lds[g].pad[9] += 1.0; }"""),
    ("""                    if (C.form == HVP_FORM_DECENT || C.form == HVP_FORM_ADMM) {  // K_bnb_ipm re-solves it
                        const unsigned long long r = atomicAdd(&ws.counter[2], 1ull);
                        if (r < (unsigned long long)ws.cap) ws.redo[r] = (int32_t)q;
                    }
                }
            }
        }
    }
}""",
     """                    if (C.form == HVP_FORM_DECENT || C.form == HVP_FORM_ADMM) {  // K_bnb_ipm re-solves it
                        const unsigned long long r = atomicAdd(&ws.counter[2], 1ull);
                        if (r < (unsigned long long)ws.cap) ws.redo[r] = (int32_t)q;
                    }
                }
            }
        }
        if (t == 0) lds[g].pad[12] += (double)(CP_NOW() - cpn);
    }
    hvp::coop::gsync();
    if (t < 13) atomicAdd(&g_cp[t], (unsigned long long)lds[g].pad[t]);
}"""),
    ("""template <int N>
__global__ __launch_bounds__(kCoopBlock) HVP_COOP_OCC void k_bnb_bound_coop(""",
     """__device__ unsigned long long g_cp[16];
template <int N>
__global__ __launch_bounds__(kCoopBlock) HVP_COOP_OCC void k_bnb_bound_coop("""),
    ("""    return 0;
}

template <int N>
int launch_all(""",
     """    if constexpr (kCoop<N>) {
        unsigned long long cp[16];
        HIP_TRY(hipStreamSynchronize(st));
        HIP_TRY(hipMemcpyFromSymbol(cp, HIP_SYMBOL(g_cp), sizeof(cp)));
        std::fprintf(stderr, "[coop-prof] qp %llu setup %llu solve-warm %llu solve-cold %llu gi %llu verify %llu classify %llu cost %llu nqp %llu nwarm %llu load %llu node %llu\\n",
                     cp[0], cp[1], cp[3], cp[4], cp[5], cp[6], cp[7], cp[8], cp[9], cp[10], cp[11], cp[12]);
        std::memset(cp, 0, sizeof(cp));
        HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_cp), cp, sizeof(cp)));
    }
    return 0;
}

template <int N>
int launch_all("""),
])
print("patched")
