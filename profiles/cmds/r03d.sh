# r03d: kernel traces of the min_1_norm benches (branch and bound vs enumeration) at the C2 size
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03d
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/r03d/bnb -o run -- python3 bench.py --cost l1 --platoons 16384 --steps 2 --warmup 1 --no-cpu --method bnb --streams 1 > gpurun_out/r03d/bnb.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/r03d/enum -o run -- python3 bench.py --cost l1 --platoons 16384 --steps 2 --warmup 1 --no-cpu --method enum --streams 1 > gpurun_out/r03d/enum.log 2>&1 || exit 2
