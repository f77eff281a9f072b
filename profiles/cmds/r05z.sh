# r05z: same-box A/B of the C2 headline: the round's final library (this tree) against the round-5
# mid-round library dc99c3ae (commit 8217ace's tree with its own build, extracted under build_oldpkg/)
set -o pipefail
export TMPDIR=/tmp
R=r05z
for v in new old new old; do
  if [ $v = new ]; then D=.; else D=build_oldpkg; fi
  (cd $D && timeout -k 10 300 python bench.py --no-cpu --no-roofline-pass) >> gpurun_out/${R}_bench_default_ab.jsonl 2>> gpurun_out/${R}_bench_ab.err || exit 1
  echo "c2 $v done" >> gpurun_out/${R}_bench_default_ab.jsonl
done
