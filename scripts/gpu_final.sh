# Round record for config B: the default bench line (as the driver runs it, with the CPU
# baseline) and the rocprofv3 kernel stats of the same command; copied to profiles/ by the caller.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
TAG=${1:-r01}
mkdir -p gpurun_out/prof
timeout -k 10 600 python bench.py > gpurun_out/final_${TAG}.log 2>&1 || { tail -20 gpurun_out/final_${TAG}.log; exit 1; }
tail -1 gpurun_out/final_${TAG}.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/final_${TAG} -o run --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/final_prof_${TAG}.log 2>&1
rc=$?
echo "rocprof rc=$rc"
exit $rc
