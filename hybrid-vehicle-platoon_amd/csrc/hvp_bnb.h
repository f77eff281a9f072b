// hvp_bnb.h -- branch and bound over region sequences (horizons beyond exhaustive enumeration).
//
// The reference's MIQP is solved by Gurobi's branch and bound over the MLD binaries
// (MpcMld.solve_mpc -> gp.Model.optimize(), called at fleet_decent_mld.py:316 and, inside the
// ADMM loop, fleet_naive_admm.py:407-419).  Exhaustive enumeration of the velocity-feasible
// region sequences grows like ~7^N/..: about 34 sequences per vehicle at N = 5, 5.7e3 at N = 10
// and ~1e6 at N = 15 (C5 sweep).  This header holds the tree logic shared by the gfx950 kernels
// (hvp_kernels.hip) and the test-only host build (hvp_hostref.cpp):
//
//   node      a region prefix sigma_0..sigma_{k-1} (4 bits per step, step j at bits 4j) with the
//             exact interval [lo, hi] of v_k reachable under that prefix (reach_step).
//   bound     the QP of the prefix with the tail RELAXED (setup_lane(.., K = k)): steps >= k
//             keep the state box, acceleration rows, tracking and safe-distance terms, but
//             drop the region-dependent input rows and input cost.  Its optimum is <= the
//             optimum of every completion of the prefix (feasible set grows, cost terms >= 0
//             are dropped), so a node whose bound exceeds the incumbent cannot contain the
//             MIQP optimum -- nor any sequence tied with it (the tie window 1e-9 relative is
//             far inside the pruning margin kPruneRel).
//   incumbent a greedy dive: the fully relaxed QP (K = 0) gives velocities y*; the region
//             closest to y*_k that keeps the prefix reachable is taken at every step.
//   leaves    full sequences (K = N) solved exactly; the answer is the same argmin and tie rule
//             (lexicographically first sequence within 1e-9 relative of the minimum) as the
//             exhaustive path, so both paths return identical sequences.
#pragma once

#include <math.h>
#include <stdint.h>

#include "hvp_ipm.h"

namespace hvp {

// prune when bound > incumbent + kPruneRel * (1 + |incumbent|): 1e-7 relative is 100x the tie
// window and far above the bound's rounding (costs are evaluated term by term, ~1e-15 relative).
constexpr double kPruneRel = 1e-7;

// A bound of 1e300 or more marks a node proven to hold no feasible completion (min_1_norm's
// certified infeasible relaxations): pruned whatever the incumbent, even before there is one.
HVP_HD inline bool bnb_pruned(double lb, double inc) { return lb >= 1e300 || lb > inc + kPruneRel * (1.0 + fabs(inc)); }

// Lexicographic key of a full sequence (step 0 most significant): numeric order of the key is
// the enumeration order of enumerate_sequences.
HVP_HD inline uint64_t bnb_lexkey(uint64_t code, int N) {
    uint64_t key = 0;
    for (int k = 0; k < N; ++k) key = (key << kCodeBits) | (uint64_t)code_region(code, k);
    return key;
}

// Greedy dive from the root: at step k take the reachable region whose band is closest to the
// relaxed velocity target (v0 at k = 0, ystar[k-1] after), ties to the lower index.  Returns
// false when it runs into a dead end (no backtracking: the tree search stays exact without an
// incumbent, only slower).
template <int N>
HVP_HD inline bool bnb_dive(const hvp_system& S, const Consts& C, double v0, const double* ystar, uint64_t* code_out) {
    double lo = v0, hi = v0;
    uint64_t code = 0;
#pragma unroll
    for (int k = 0; k < N; ++k) {
        const double tgt = k == 0 ? v0 : ystar[k - 1];
        int best = -1;
        double bd = 1e300, blo = 0.0, bhi = 0.0;
        for (int r = 0; r < S.n_regions; ++r) {
            double nlo, nhi;
            if (!bnb_child(S, C, k, lo, hi, r, &nlo, &nhi)) continue;
            const double d = fmax(0.0, fmax(S.vlo[r] - tgt, tgt - S.vhi[r]));
            if (d < bd) { bd = d; best = r; blo = nlo; bhi = nhi; }
        }
        if (best < 0) return false;
        code = code_with(code, k, best);
        lo = blo;
        hi = bhi;
    }
    *code_out = code;
    return true;
}

}  // namespace hvp
