# Configs C and E of BASELINE.json: bench lines + kernel stats (rocprofv3).
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
TAG=${1:-r01}
mkdir -p gpurun_out/prof
for w in C E; do
  timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 2 > gpurun_out/bench_${TAG}_$w.log 2>&1 || { tail -20 gpurun_out/bench_${TAG}_$w.log; exit 1; }
  tail -1 gpurun_out/bench_${TAG}_$w.log
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/${TAG}_$w -o run --output-format csv -- python3 bench.py --workload $w --steps 5 --warmup 1 > gpurun_out/prof_${TAG}_$w.log 2>&1 || exit 1
done
echo done
