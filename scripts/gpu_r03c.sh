# Round 3: the slice build (pk_build) on the GPU: its tests, the headline files, the config-D line.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r03c}
timeout -k 10 900 python -u -m pytest tests/test_gpu_pk_levels.py tests/test_gpu_headline.py -m gpu -x -v \
  --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --workload D --gpus 1 --steps 5 --warmup 2 --no-cpu-baseline --no-mintime \
  > gpurun_out/${T}_benchD.log 2>&1
rc=$?; echo "benchD rc=$rc"; tail -1 gpurun_out/${T}_benchD.log | cut -c1-600; exit $rc
