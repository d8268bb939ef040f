#!/bin/bash
# rocprofv3 kernel trace + FETCH/WRITE passes of the configs[4] frame shape (bench.py --config cfg5):
#   tools/profile_cfg5.sh TAG  ->  profiles/TAG_cfg5_kernel_stats.csv, profiles/TAG_cfg5_pmc.json
set -euo pipefail
TAG=${1:-r2}
OUT=gpurun_out/profcfg5_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
B="bench.py --config cfg5 --steps 3 --warmup 1 --no-cpu-baseline --no-timing"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o trace -- python3 $B > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o p -- python3 $B > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o p -- python3 $B > "$OUT/write.log" 2>&1
STATS=$(find "$OUT/trace" -name '*kernel_stats.csv' | head -1)
mkdir -p profiles
cp "$STATS" "profiles/${TAG}_cfg5_kernel_stats.csv"
python3 tools/pmc_summary.py --stats "$STATS" --fetch "$OUT/fetch" --write "$OUT/write" \
  --out "profiles/${TAG}_cfg5_pmc.json" --frames-per-launch 400 \
  --note "bench.py --config cfg5 --steps 3 --warmup 1 (400 configs[4]-shape frames per launch); $(date -u)"
cp "profiles/${TAG}_cfg5_pmc.json" "profiles/${TAG}_cfg5_kernel_stats.csv" "$OUT/"
