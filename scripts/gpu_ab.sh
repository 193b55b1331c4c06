# Same-box A/B of the working tree's library against the variants under 3d-hashjoin_amd/variants
# (scripts/time_pk.py, config-B size unless ARGS says otherwise), two rounds interleaved.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
for round in 1 2; do
  for v in default $(ls 3d-hashjoin_amd/variants 2>/dev/null); do
    if [ $v = default ]; then unset HJ3D_LIB; else export HJ3D_LIB=$GRAFT_REPO_ROOT/3d-hashjoin_amd/variants/$v/libhj3d.so; fi
    timeout -k 10 120 python scripts/time_pk.py --label $v $ARGS || exit 1
  done
done
