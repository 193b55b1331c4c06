# Same-box A/B of bench.py workloads ($WLS, default "E C") for the working tree's library and the
# variants under 3d-hashjoin_amd/variants, two rounds interleaved; one summary line per run.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for round in 1 2; do
  for w in ${WLS:-E C}; do
    for v in default $(ls 3d-hashjoin_amd/variants 2>/dev/null); do
      if [ $v = default ]; then unset HJ3D_LIB; else export HJ3D_LIB=$GRAFT_REPO_ROOT/3d-hashjoin_amd/variants/$v/libhj3d.so; fi
      timeout -k 10 300 python bench.py --workload $w --steps ${STEPS:-8} --warmup 2 --no-cpu-baseline --no-mintime > gpurun_out/ab/$v.$w.log 2>&1 || { tail -5 gpurun_out/ab/$v.$w.log; exit 1; }
      python -c "import json; d=json.loads(open('gpurun_out/ab/$v.$w.log').read().strip().splitlines()[-1]); print('$w', '$v', 'build_ms', round(d['build_ms'],4), 'probe_ms', round(d['probe_ms'],4), 'exact', d['verified_bit_exact'])"
    done
  done
done
