TAG=r04c PART=c bash scripts/gpu_round.sh && \
HJ3D_COMM_PIECE_LOG2=28 timeout -k 10 180 python scripts/rccl_limits.py 268447801 28 > gpurun_out/r04c_rccl_default.jsonl 2>&1 && tail -1 gpurun_out/r04c_rccl_default.jsonl && \
for nb in agg slices; do timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/r04c_Bnrs_$nb -o run --output-format csv -- python3 bench.py --plan Nrs --steps 5 --warmup 1 --no-cpu-baseline --no-mintime --nested-build $nb > gpurun_out/r04c_Bnrs_$nb.log 2>&1 || exit 1; tail -c 300 gpurun_out/r04c_Bnrs_$nb.log; done && \
CMD=scripts/time_partition.py VARIANTS="xp512 xp512w3" bash scripts/gpu_ab.sh > gpurun_out/r04c_ab_xpart.log 2>&1 && cat gpurun_out/r04c_ab_xpart.log
