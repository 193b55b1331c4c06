cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -x -k num_distinct -p no:cacheprovider 2>&1 | tail -3
timeout -k 10 300 python bench.py --workload C --steps 5 --warmup 1 > gpurun_out/c_sort.log 2>&1; tail -1 gpurun_out/c_sort.log | cut -c1-900
timeout -k 10 300 python bench.py --workload C --steps 5 --warmup 1 --nested-radix > gpurun_out/c_radix.log 2>&1; tail -1 gpurun_out/c_radix.log | cut -c1-900
