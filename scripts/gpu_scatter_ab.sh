# A/B: build-side partition scatter with contiguous tile ranges per workgroup (default) vs strided
# tiles (HJ3D_SCATTER_STRIDED=1): config C build and config B build, plus rocprof stats of both.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for v in contig strided; do
  if [ $v = strided ]; then export HJ3D_SCATTER_STRIDED=1; else unset HJ3D_SCATTER_STRIDED; fi
  timeout -k 10 200 python bench.py --workload C --steps 8 --warmup 2 > gpurun_out/ab/C_$v.log 2>&1 || { tail -5 gpurun_out/ab/C_$v.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/ab/C_$v.log').read().strip().splitlines()[-1]); print('$v C build_ms', d['build_ms'], 'probe_ms', d['probe_ms'], 'exact', d['verified_bit_exact'])"
  timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab/B_$v.log 2>&1 || { tail -5 gpurun_out/ab/B_$v.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/ab/B_$v.log').read().strip().splitlines()[-1]); print('$v B build_ms', d['build_ms'], 'probe_ms', d['probe_ms'], 'exact', d['verified_bit_exact'])"
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ab/prof_$v -o run --output-format csv -- python3 bench.py --workload C --steps 4 --warmup 1 > gpurun_out/ab/prof_$v.log 2>&1 || exit 1
  grep -h "k_rp_scatter\|k_rp_hist\|\"k_nagg(" gpurun_out/ab/prof_$v/run_kernel_stats.csv | cut -d, -f1-4 | sed 's/(hj3d[^"]*//'
done
