# Probe-kernel time vs table size at fixed |S| (is the probe bound by random table accesses?)
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
for nr in 262144 1000000 4000000 10000000 30000000; do
  timeout -k 10 120 python bench.py --nR $nr --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/sweep_$nr.log 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/sweep_$nr.log').read().strip().splitlines()[-1]); print($nr, 'probe_kernel_ms', round(d['roofline']['kernel_avg_ms'],3), 'build_ms', round(d['build_ms'],3), 'ok', d['verified_bit_exact'])"
done
for nr in 262144 10000000; do
  timeout -k 10 120 python bench.py --nR $nr --steps 5 --warmup 1 --no-cpu-baseline --no-emit > gpurun_out/sweepagg_$nr.log 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/sweepagg_$nr.log').read().strip().splitlines()[-1]); print($nr, 'AGG probe_kernel_ms', round(d['roofline']['kernel_avg_ms'],3))"
done
