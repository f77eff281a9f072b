"""hvp -- MI355X-native batched hybrid-MPC inner solver for the vehicle-platoon benchmark.

Product path: PWA vehicle tables (models, tables) -> libhvpsolve.so (HIP, gfx950) through the
C ABI of include/hvp.h (solver) -> the reference's call surface (mpc, agent, decent).
"""

__all__ = ["models", "params", "env", "tables", "solver", "batched", "mpc", "agent", "decent", "admm", "gadmm", "cent", "envdev"]
