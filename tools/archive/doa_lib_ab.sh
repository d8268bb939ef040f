#!/bin/bash
# K5 standalone times of two development libraries, alternating, in one call (tools/doa_skew_ablation.py VARIANTS=0,
# with and without the fused extras):  tools/doa_lib_ab.sh LIB_A LIB_B [ROUNDS]
set -euo pipefail
A=${1:-radar-slam_amd/lib/librsl_devprev.so}; B=${2:-radar-slam_amd/lib/librsl_dev.so}; R=${3:-3}
mkdir -p gpurun_out
for r in $(seq "$R"); do
  for L in "$A" "$B"; do
    echo "== $L round $r"
    VARIANTS=0 RSL_LIBRARY=$L timeout -k 10 120 python -u tools/doa_skew_ablation.py
  done
done
