#!/bin/bash
# rocprofv3 kernel trace + FETCH/WRITE passes of the configs[1] spectrum workload (bench.py --config spectrum):
#   tools/profile_spectrum.sh TAG  ->  profiles/TAG_spectrum_kernel_stats.csv, profiles/TAG_spectrum_pmc.json
set -euo pipefail
TAG=${1:-r2}
OUT=gpurun_out/profspec_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
B="bench.py --config spectrum --steps 3 --warmup 1 --no-cpu-baseline --no-timing"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o trace -- python3 $B > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o p -- python3 $B > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o p -- python3 $B > "$OUT/write.log" 2>&1
STATS=$(find "$OUT/trace" -name '*kernel_stats.csv' | head -1)
mkdir -p profiles
cp "$STATS" "profiles/${TAG}_spectrum_kernel_stats.csv"
python3 tools/pmc_summary.py --stats "$STATS" --fetch "$OUT/fetch" --write "$OUT/write" \
  --out "profiles/${TAG}_spectrum_pmc.json" --frames-per-launch 1000 \
  --note "bench.py --config spectrum --steps 3 --warmup 1 (1000 cfg2 frames per launch); $(date -u)"
cp "profiles/${TAG}_spectrum_pmc.json" "profiles/${TAG}_spectrum_kernel_stats.csv" "$OUT/"
