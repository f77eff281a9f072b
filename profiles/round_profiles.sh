#!/usr/bin/env bash
# Round-end refresh of the committed profiles: the four bench workloads (profile_all.sh) into
# gpurun_out/prof_<round>, then profiles/summarize.py condenses them (run here, on the CPU side).
#   profiles/round_profiles.sh r02r
set -euo pipefail
R=${1:?round tag}
bash profiles/profile_all.sh "gpurun_out/prof_$R"
