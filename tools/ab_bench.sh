#!/bin/bash
# A/B of the default bench line (cfg2 metric, no sub-measurements) between radar-slam_amd/lib/librsl_ab.so (A,
# tools/build_ab.sh) and the in-tree librsl.so (B), alternating:   tools/ab_bench.sh TAG [ROUNDS] [extra bench args]
set -euo pipefail
TAG=${1:-ab}
ROUNDS=${2:-3}
shift 2 || true
OUT=gpurun_out/abb_$TAG
mkdir -p "$OUT"
for r in $(seq 1 "$ROUNDS"); do
  for v in A B; do
    if [ "$v" = A ]; then export RSL_LIBRARY=$PWD/radar-slam_amd/lib/librsl_ab.so; else unset RSL_LIBRARY; fi
    timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-extra --no-pcie --no-cpu-baseline "$@" > "$OUT/${v}$r.json" 2> "$OUT/${v}$r.err"
  done
done
python3 - "$OUT" "$ROUNDS" <<'PY'
import json, sys
out, rounds = sys.argv[1], int(sys.argv[2])
for r in range(1, rounds + 1):
    for v in 'AB':
        d = json.load(open(f'{out}/{v}{r}.json'))
        ks = d.get('kernel_ms_standalone', {})
        print(v, r, round(d['value']), {k: round(x, 3) for k, x in ks.items()})
PY
