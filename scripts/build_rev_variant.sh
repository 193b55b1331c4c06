# Builds libhj3d.so of git revision $1 (default HEAD) into 3d-hashjoin_amd/variants/${2:-rev}/libhj3d.so,
# for same-box A/B timing against the working tree (scripts/time_pk.py under HJ3D_LIB).
set -e
REV=${1:-HEAD}
NAME=${2:-rev}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
git -C "$ROOT" archive "$REV" 3d-hashjoin_amd/Makefile 3d-hashjoin_amd/csrc include | tar -x -C "$TMP"
make -s -C "$TMP/3d-hashjoin_amd" -j8 lib/libhj3d.so
mkdir -p "$ROOT/3d-hashjoin_amd/variants/$NAME"
cp "$TMP/3d-hashjoin_amd/lib/libhj3d.so" "$ROOT/3d-hashjoin_amd/variants/$NAME/libhj3d.so"
rm -rf "$TMP"
echo "built $REV -> variants/$NAME"
