#!/bin/bash
# GPU-box profiling recipe (run via gpurun from the repo root):
#   tools/profile.sh TAG
# 1) kernel trace + stats of bench.py, 2) FETCH_SIZE pass, 3) WRITE_SIZE pass, 4) MFMA/VALU busy pass,
# then tools/pmc_summary.py -> profiles/TAG_pmc.json and the stats CSV -> profiles/TAG_kernel_stats.csv.
set -euo pipefail
TAG=${1:-r2}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
B="bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-pcie --no-extra --no-timing --streams 1 --frames-per-step 2000"
# the kernel trace profiles the default bench command itself (its hipEvent averages are the ones reported)
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o trace -- python3 bench.py --no-cpu-baseline --no-pcie --no-extra > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o p -- python3 $B > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o p -- python3 $B > "$OUT/write.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES --output-format csv \
  -d "$OUT/busy" -o p -- python3 $B > "$OUT/busy.log" 2>&1
STATS=$(find "$OUT/trace" -name '*kernel_stats.csv' | head -1)
mkdir -p profiles
cp "$STATS" "profiles/${TAG}_kernel_stats.csv"
python3 tools/pmc_summary.py --stats "$STATS" --fetch "$OUT/fetch" --write "$OUT/write" --extra "$OUT/busy" \
  --out "profiles/${TAG}_pmc.json" --frames-per-launch 2000 \
  --note "bench.py --steps 3 --warmup 2 --no-extra (2000 cfg2 frames per launch); $(date -u)"
cp "profiles/${TAG}_pmc.json" "profiles/${TAG}_kernel_stats.csv" "$OUT/"
