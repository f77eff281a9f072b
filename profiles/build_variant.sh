#!/usr/bin/env bash
# A/B builds of the product library with extra compile definitions, next to the shipped one:
#   profiles/build_variant.sh NAME "-DFLAG=VALUE ..."  ->  hybrid-vehicle-platoon_amd/lib/libhvpsolve_NAME.so
# (selected at run time with HVP_LIB; the .so is git-ignored like the shipped library)
set -euo pipefail
NAME=$1
EXTRA=${2:-}
PKG=$(cd "$(dirname "$0")/../hybrid-vehicle-platoon_amd" && pwd)
B=$PKG/build_$NAME
mkdir -p "$B"
FLAGS="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=fast -munsafe-fp-atomics -Wall -Wno-unused-function $EXTRA"
INC="-I$PKG/../include -I$PKG/csrc"
cd "$PKG"
pids=()
/opt/rocm/bin/hipcc $FLAGS $INC -c -o "$B/hvp_kernels.o" csrc/hvp_kernels.hip & pids+=($!)
for n in 2 3 4 5 6 7 8 9 10 11 12 13 14 15 16; do
  /opt/rocm/bin/hipcc $FLAGS $INC -DHVP_N=$n -c -o "$B/hvp_lane_$n.o" csrc/hvp_lane_inst.hip & pids+=($!)
  if [ ${#pids[@]} -ge 8 ]; then wait "${pids[0]}"; pids=("${pids[@]:1}"); fi
done
/opt/rocm/bin/hipcc $FLAGS $INC -c -o "$B/hvp_cent.o" csrc/hvp_cent.hip & pids+=($!)
/opt/rocm/bin/hipcc $FLAGS $INC -c -o "$B/hvp_env.o" csrc/hvp_env.hip & pids+=($!)
for p in "${pids[@]}"; do wait "$p"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "lib/libhvpsolve_$NAME.so" "$B"/hvp_kernels.o "$B"/hvp_lane_*.o "$B"/hvp_cent.o "$B"/hvp_env.o
echo "lib/libhvpsolve_$NAME.so"
