cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -le 1 ]; then
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-reps 1 > gpurun_out/bench.log 2>&1
  brc=$?
  echo "bench rc=$brc"
  tail -5 gpurun_out/bench.log
fi
