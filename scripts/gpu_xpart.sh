# single-pass exchange partitioner: parity tests, timing against the stable one, the dist strand
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_xpart.py tests/test_gpu_dist.py "tests/test_gpu_parity.py::test_bucket_shards_sum_to_single_table" -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/xpart_tests.log 2>&1
rc=$?; tail -3 gpurun_out/xpart_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/time_exchange_partition.py 2 8 64 256 > gpurun_out/xpart_time.log 2>&1
rc=$?; cat gpurun_out/xpart_time.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --dist-path --steps 10 --warmup 3 --no-cpu-baseline --no-mintime --json-out gpurun_out/xpart_dist_single.json > gpurun_out/xpart_dist_single.log 2>&1
rc=$?; tail -c 600 gpurun_out/xpart_dist_single.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --dist-path --xpart stable --steps 10 --warmup 3 --no-cpu-baseline --no-mintime --json-out gpurun_out/xpart_dist_stable.json > gpurun_out/xpart_dist_stable.log 2>&1
rc=$?; tail -c 600 gpurun_out/xpart_dist_stable.log; exit $rc
