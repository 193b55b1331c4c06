# A/B: k_nagg pass B in 1 / 2 / 4 parts of the sub range (HJ3D_NAGG_HALVES), config C build.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/ab
for h in 1 2 4; do
  HJ3D_NAGG_HALVES=$h timeout -k 10 200 python bench.py --workload C --steps 8 --warmup 2 > gpurun_out/ab/C_h$h.log 2>&1 || { tail -5 gpurun_out/ab/C_h$h.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/ab/C_h$h.log').read().strip().splitlines()[-1]); print('halves $h build_ms', round(d['build_ms'],3), 'probe_ms', round(d['probe_ms'],3), 'exact', d['verified_bit_exact'], d['counters'])"
done
HJ3D_NAGG_HALVES=2 timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -x -k "nested or Nrs or zipf" -p no:cacheprovider 2>&1 | tail -2
