#!/bin/bash
# A/B of kernels between the in-tree librsl.so (B) and radar-slam_amd/lib/librsl_ab.so (A, tools/build_ab.sh),
# alternating, under a kernel trace each: PROG=tools/dd_only.py (K1 + K2, default) or tools/chain_only.py (the chain);
# KERN = a regex of the kernel names to report (default: the FFT kernels):
#   CFG=cfg5 F=400 tools/ab_front.sh TAG [ROUNDS]
set -euo pipefail
TAG=${1:-ab}
ROUNDS=${2:-2}
OUT=gpurun_out/abf_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
export REPS=${REPS:-8}
for r in $(seq 1 "$ROUNDS"); do
  for v in A B; do
    if [ "$v" = A ]; then export RSL_LIBRARY=$PWD/radar-slam_amd/lib/librsl_ab.so; else unset RSL_LIBRARY; fi
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${v}$r" -o tr -- python3 ${PROG:-tools/dd_only.py} > "$OUT/${v}$r.log" 2>&1
  done
done
python3 - "$OUT" "$ROUNDS" "${KERN:-rsl::k_(range|doppler)}" <<'PY'
import csv, sys, glob, re
out, rounds, kern = sys.argv[1], int(sys.argv[2]), re.compile(sys.argv[3])
for r in range(1, rounds + 1):
    for v in 'AB':
        f = glob.glob(f'{out}/{v}{r}/**/*kernel_stats.csv', recursive=True)[0]
        row = {x['Name'].split('(')[0][:40]: (float(x['AverageNs']) / 1e6, float(x['MinNs']) / 1e6)
               for x in csv.DictReader(open(f)) if kern.search(x['Name'])}
        print(v, r, {k: f'{a:.3f} (min {b:.3f})' for k, (a, b) in row.items()})
PY
