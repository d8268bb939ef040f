#!/bin/bash
# Like tools/ab_front.sh, over any number of library builds: each named lib (radar-slam_amd/lib/librsl_<name>.so;
# "tree" = the in-tree librsl.so) is run in turn under a kernel trace, ROUNDS times, alternating:
#   CFG=cfg5 F=400 tools/ab_multi.sh TAG ROUNDS ab tree v1 v2
set -euo pipefail
TAG=${1:-abm}
ROUNDS=${2:-2}
shift 2
LIBS=("$@")
OUT=gpurun_out/abm_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
export REPS=${REPS:-8}
for r in $(seq 1 "$ROUNDS"); do
  for v in "${LIBS[@]}"; do
    if [ "$v" = tree ]; then unset RSL_LIBRARY; else export RSL_LIBRARY=$PWD/radar-slam_amd/lib/librsl_$v.so; fi
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${v}_$r" -o tr -- python3 ${PROG:-tools/dd_only.py} > "$OUT/${v}_$r.log" 2>&1
  done
done
python3 - "$OUT" "$ROUNDS" "${KERN:-rsl::k_(range|doppler)}" "${LIBS[@]}" <<'PY'
import csv, sys, glob, re
out, rounds, kern, libs = sys.argv[1], int(sys.argv[2]), re.compile(sys.argv[3]), sys.argv[4:]
for r in range(1, rounds + 1):
    for v in libs:
        f = glob.glob(f'{out}/{v}_{r}/**/*kernel_stats.csv', recursive=True)[0]
        row = {x['Name'].split('(')[0][:40]: (float(x['AverageNs']) / 1e6, float(x['MinNs']) / 1e6)
               for x in csv.DictReader(open(f)) if kern.search(x['Name'])}
        print(f'{v:6s}', r, {k: f'{a:.3f} (min {b:.3f})' for k, (a, b) in row.items()})
PY
