# Round 3: the GPU tier (pytest -m gpu, alphabetical like the driver's) then the reverse file
# order (state left by small tests before the headline sizes), the config-D bench line on one GPU
# and the 8-owner split emulation of config D.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r03a}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/${T}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_pk_levels.py tests/test_gpu_parity.py tests/test_gpu_headline.py \
  -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_pytest_rev.log 2>&1
rc=$?; echo "pytest (reverse order) rc=$rc"; tail -3 gpurun_out/${T}_pytest_rev.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --workload D --gpus 1 --steps 5 --warmup 2 --no-cpu-baseline --no-mintime \
  > gpurun_out/${T}_benchD.log 2>&1
rc=$?; echo "benchD rc=$rc"; tail -1 gpurun_out/${T}_benchD.log | cut -c1-1500; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u scripts/d_shards.py > gpurun_out/${T}_dshards.log 2>&1
rc=$?; echo "dshards rc=$rc"; tail -1 gpurun_out/${T}_dshards.log | cut -c1-1500; exit $rc
