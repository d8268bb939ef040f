#!/bin/bash
# K1 / K2 standalone times of two development libraries, alternating, in one call (box-to-box clock differences
# move single kernels by several %, so A/B only inside one call):  tools/lib_ab.sh LIB_A LIB_B [ROUNDS]
set -euo pipefail
A=${1:-radar-slam_amd/lib/librsl_devprev.so}; B=${2:-radar-slam_amd/lib/librsl_dev.so}; R=${3:-3}
mkdir -p gpurun_out
for r in $(seq "$R"); do
  for L in "$A" "$B"; do
    echo "== $L round $r"
    ONLY0=1 C64=0 RSL_LIBRARY=$L timeout -k 10 120 python -u tools/fft_ablation.py
  done
done
