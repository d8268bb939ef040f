#!/bin/bash
# Build the product library of another commit as radar-slam_amd/lib/librsl_ab.so (A/B timing in one GPU session:
# RSL_LIBRARY=radar-slam_amd/lib/librsl_ab.so python bench.py ...).   usage: tools/build_ab.sh <commit>
set -euo pipefail
REV=${1:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d /tmp/rsl_ab.XXXX)
git -C "$ROOT" archive "$REV" radar-slam_amd/csrc include | tar -x -C "$TMP"
make -C "$TMP/radar-slam_amd/csrc" -j8 > /dev/null
cp "$TMP/radar-slam_amd/lib/librsl.so" "$ROOT/radar-slam_amd/lib/librsl_ab.so"
rm -rf "$TMP"
echo "built $REV -> radar-slam_amd/lib/librsl_ab.so"
