# Kernel trace + stats of the config C bench (nested build / probe / unnest).
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
TAG=${1:-c}
mkdir -p gpurun_out/prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/$TAG -o run --output-format csv -- python3 bench.py --workload C --steps 3 --warmup 1 > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "rocprof rc=$rc"
python3 scripts/kstats.py $(find gpurun_out/prof/$TAG -name "*kernel_stats.csv") | head -40
exit $rc
