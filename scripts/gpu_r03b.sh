# Round 3: where k_pk_part / k_pk_probe spend their time (diagnostic variants, config-B size), and the
# rocprofv3 kernel summaries of the config-D line and of its 8-owner split emulation.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
for v in default $(ls 3d-hashjoin_amd/variants); do
  if [ $v = default ]; then unset HJ3D_LIB; else export HJ3D_LIB=$GRAFT_REPO_ROOT/3d-hashjoin_amd/variants/$v/libhj3d.so; fi
  timeout -k 10 120 python scripts/time_pk.py --label $v || exit 1
  timeout -k 10 120 python scripts/time_pk.py --label $v-noemit --no-emit || exit 1
done
unset HJ3D_LIB
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/r03_D_shards -o run --output-format csv -- python3 scripts/d_shards.py --reps 2 > gpurun_out/r03b_dshards.log 2>&1
rc=$?; echo "dshards prof rc=$rc"; tail -1 gpurun_out/r03b_dshards.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/r03_D -o run --output-format csv -- python3 bench.py --workload D --steps 3 --warmup 1 --no-cpu-baseline --no-mintime > gpurun_out/r03b_benchD.log 2>&1
rc=$?; echo "benchD prof rc=$rc"; tail -1 gpurun_out/r03b_benchD.log | cut -c1-300; exit $rc
