# Round record, part 1: GPU parity tests, smoke(), the default bench line (as the driver runs it)
# and rocprofv3 kernel stats of the same command. Every GPU step has its own limit; stops at the
# first failure.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
TAG=${1:-r01}
mkdir -p gpurun_out/prof
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_${TAG}.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu_${TAG}.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 || { tail -20 gpurun_out/smoke_${TAG}.log; exit 1; }
tail -1 gpurun_out/smoke_${TAG}.log
timeout -k 10 600 python bench.py > gpurun_out/final_${TAG}.log 2>&1 || { tail -20 gpurun_out/final_${TAG}.log; exit 1; }
tail -1 gpurun_out/final_${TAG}.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/final_${TAG} -o run --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/final_prof_${TAG}.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
