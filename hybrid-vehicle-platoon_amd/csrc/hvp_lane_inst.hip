// hvp_lane_inst.hip -- the lane-path launchers (hvp_lane.h) of one horizon N = HVP_N.  The
// Makefile compiles this file once per N in 2..16 (parallel objects; hvp_kernels.hip dispatches).
#define HVP_LANE_INST
#include "hvp_lane.h"

#ifndef HVP_N
#error "compile with -DHVP_N=<horizon>"
#endif

namespace hvp_k {
HVP_LANE_LAUNCHERS(, HVP_N)
#if HVP_N <= HVP_MAX_N_ENUM
HVP_ENUM_LAUNCHER(, HVP_N)
#endif
}  // namespace hvp_k
