# RCCL message-size sweep of the exchange (scripts/rccl_limits.py), one process per setting, on a
# diagnostic build of the library (-DHJ3D_COMM_DIAG: the word / piece overrides exist only there;
# build it first on the CPU side: bash scripts/build_variants.sh commdiag -DHJ3D_COMM_DIAG).
# Single messages (piece 2^40 B) of 0.5 .. 1.9 GB as u64 words locate the size at which a message
# arrives corrupted; the product library (default 2^28-byte pieces) then carries 2.15e9 bytes.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
run() {  # pairs piece_log2 [lib]
  HJ3D_LIB=$3 HJ3D_COMM_PIECE_LOG2=$2 timeout -k 10 180 python scripts/rccl_limits.py $1 $2 2>&1 | grep -v amdgpu.ids
  rc=${PIPESTATUS[0]}
  [ $rc -eq 0 ] || { echo "rc=$rc pairs=$1 piece=$2"; exit $rc; }
}
DIAG=$PWD/3d-hashjoin_amd/variants/commdiag/libhj3d.so
for n in 62500000 93750000 118750000 125000000 131250000 134217728 137500000 156250000 187500000 237500000; do
  run $n 40 $DIAG
done
run 268447801 28 ""
