#!/bin/bash
# Build libxhe.so from a SNAPSHOT of the sources (xfl_amd/csrc + include), so
# that editing the tree while the ~12-minute device compile runs cannot mix
# two versions (hipcc reads the headers again for its host pass).
#   tools/snap_build.sh OUT.so [-DNAME ...]      (log: OUT.so.log; remarks: kernel resource usage)
set -e
OUT=$(realpath -m "$1")
shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SNAP=$(mktemp -d /tmp/xhe_snap.XXXXXX)
mkdir -p "$SNAP/xfl_amd/csrc" "$SNAP/include"
cp "$ROOT"/xfl_amd/csrc/* "$SNAP/xfl_amd/csrc/"
cp "$ROOT"/include/* "$SNAP/include/"
(cd "$SNAP" && git -C "$ROOT" rev-parse --short HEAD > "$SNAP/HEAD" 2>/dev/null || true)
{
  echo "snapshot $SNAP of $(cat "$SNAP/HEAD" 2>/dev/null)"
  time /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Werror=shift-count-overflow -Werror=shift-count-negative "$@" -Rpass-analysis=kernel-resource-usage \
    -c "$SNAP/xfl_amd/csrc/xhe.hip" -o "$SNAP/xhe.o"
  g++ -O3 -std=c++17 -fPIC -pthread -c "$SNAP/xfl_amd/csrc/wire_abi.cpp" -o "$SNAP/wire_abi.o"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -pthread "$SNAP/xhe.o" "$SNAP/wire_abi.o" -o "$OUT.tmp"
  mv "$OUT.tmp" "$OUT"
  echo "built $OUT"
} > "$OUT.log" 2>&1
rm -rf "$SNAP"
