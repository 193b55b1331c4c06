# Same-box A/B of the working tree's library against variant builds under 3d-hashjoin_amd/variants
# (scripts/build_variants.sh), two rounds interleaved. CMD = the timing script (default
# scripts/time_pk.py; scripts/time_partition.py for the exchange partitioner), ARGS its arguments,
# VARIANTS the variant names (default: every variant but the commdiag diagnostic build).
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
CMD=${CMD:-scripts/time_pk.py}
VARIANTS=${VARIANTS:-$(ls 3d-hashjoin_amd/variants 2>/dev/null | grep -v '^commdiag$')}
for round in 1 2; do
  for v in default $VARIANTS; do
    if [ $v = default ]; then unset HJ3D_LIB; else export HJ3D_LIB=$GRAFT_REPO_ROOT/3d-hashjoin_amd/variants/$v/libhj3d.so; fi
    timeout -k 10 180 python $CMD --label $v $ARGS || exit 1
  done
done
