# same-box A/B of exchange-partitioner variants (3d-hashjoin_amd/variants/<name>/libhj3d.so)
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in default "$@"; do
  if [ "$v" = default ]; then unset HJ3D_LIB; else export HJ3D_LIB=$PWD/3d-hashjoin_amd/variants/$v/libhj3d.so; fi
  echo "== $v"
  timeout -k 10 200 python -u scripts/time_exchange_partition.py 2 8 64 > gpurun_out/xpab_$v.log 2>&1 || { cat gpurun_out/xpab_$v.log; exit 1; }
  grep single gpurun_out/xpab_$v.log | cut -c1-90
done
