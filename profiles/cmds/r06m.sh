#!/bin/bash
# round 6: N = 3 min_1_norm refill failure: (G) LevelList slot without the pivot record, (H) the pivot record without the slot map, (I) level_slot
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in _vG _vH _vI; do
  HVP_LIB=$PWD/hybrid-vehicle-platoon_amd/lib/libhvpsolve$v.so TAG="lib$v" timeout -k 10 120 python -u profiles/diag_l1_small.py >> gpurun_out/r06m.log 2>&1 || exit 1
  HVP_SPLIT_LEVELS=1 HVP_LIB=$PWD/hybrid-vehicle-platoon_amd/lib/libhvpsolve$v.so TAG="lib$v split1" timeout -k 10 120 python -u profiles/diag_l1_small.py >> gpurun_out/r06m.log 2>&1 || exit 1
done
