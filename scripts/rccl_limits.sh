# RCCL message-size limits of the exchange (scripts/rccl_limits.py), one process per setting:
# 8-byte words in 2^27-word pieces (the library's default), 8-byte words as one message, bytes as one
# message, bytes in 2^27-byte pieces; 2.5e8 pairs = 2e9 bytes (one config-D chunk) and 2^28 + 12345
# pairs (> 2^31 bytes).
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
for n in 250000000 268447801; do
  for setting in "auto 27" "auto 40" "1 40" "1 27"; do
    set -- $setting
    HJ3D_COMM_WORD=$([ $1 = auto ] || echo $1) HJ3D_COMM_PIECE_LOG2=$2 timeout -k 10 180 python scripts/rccl_limits.py $n 2>&1 | grep -v amdgpu.ids
    rc=${PIPESTATUS[0]}
    [ $rc -eq 0 ] || { echo "rc=$rc n=$n setting=$setting"; exit $rc; }
  done
done
