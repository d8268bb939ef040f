#!/bin/bash
# Runs bench.py once per environment setting given as arguments ("VAR=val VAR2=val" strings) and prints
# value + per-kernel times.  Usage (on the GPU box): tools/tune.sh "" "RSL_DD_KB=16" ...
set -uo pipefail
for cfg in "$@"; do
  out=$(env $cfg timeout -k 10 200 python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline 2>/dev/null | tail -1)
  rc=$?
  if [ $rc -ne 0 ]; then echo "[$cfg] FAILED rc=$rc"; exit $rc; fi
  echo "[$cfg] $(echo "$out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']), {k: round(v,3) for k,v in d['kernel_ms_per_step'].items()})")"
done
