# Profile the bench: kernel trace + stats (rocprofv3), then a short bench line.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
TAG=${1:-r01}
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_${TAG}.log 2>&1 || exit $?
tail -2 gpurun_out/bench_${TAG}.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/${TAG} -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_${TAG}.log 2>&1
rc=$?
echo "rocprof rc=$rc"
find gpurun_out/prof/${TAG} -name "*stats*" | head
exit $rc
